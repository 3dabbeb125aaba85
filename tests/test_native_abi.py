"""The C-ABI library loads (no GPU needed) and exports every symbol include/pbg.h declares."""
import ctypes
import os
import re

import pytest

import pybulletgym_amd  # noqa: F401
from pybulletgym_amd import _native

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "pbg.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pbg_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_abi():
    names = declared()
    for n in ("pbg_create", "pbg_step", "pbg_reset", "pbg_destroy", "pbg_last_error"):
        assert n in names


@pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="libpbg_amd.so not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native.LIB_PATH)
    for n in declared():
        assert hasattr(lib, n), n
    assert set(_native.EXPORTED) <= set(declared())


@pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="libpbg_amd.so not built")
def test_pack_record_sizes_without_gpu():
    lib = _native.lib()
    iw, ow = ctypes.c_int(), ctypes.c_int()
    assert lib.pbg_pack_record_sizes(b"AntPyBulletEnv-v0", ctypes.byref(iw), ctypes.byref(ow)) == 0
    assert ow.value == 28 + 4 + 4
    assert lib.pbg_pack_record_sizes(b"NoSuchEnv-v0", ctypes.byref(iw), ctypes.byref(ow)) != 0
    assert b"unknown env id" in lib.pbg_last_error()


def test_info_struct_matches_header():
    """_native.Info mirrors pbg_info_t field for field (all int)."""
    src = open(HEADER).read()
    body = src[src.index("typedef struct {", src.index("pbg_handle;")):src.index("} pbg_info_t;")]
    fields = re.findall(r"\bint\s+([a-z_]+);", body)
    assert fields == [f[0] for f in _native.Info._fields_]


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_native.PbgError):
        _native.lib()


def test_sim_params_struct_matches_header():
    """_native.SimParams mirrors pbg_sim_params_t field for field (types and order)."""
    src = open(HEADER).read()
    body = src[src.rindex("typedef struct {", 0, src.index("} pbg_sim_params_t;")):src.index("} pbg_sim_params_t;")]
    fields = re.findall(r"\b(double|int)\s+([a-z_]+);", body)
    ct = {"double": ctypes.c_double, "int": ctypes.c_int}
    assert [(n, ct[t]) for t, n in fields] == list(_native.SimParams._fields_)


@pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="libpbg_amd.so not built")
def test_default_sim_params_are_the_reference_scenes():
    """pbg_default_sim_params (host only) returns the scene each env builds: StadiumScene(gravity
    9.8, timestep 0.0165/4, frame_skip 4) for the walkers (roboschool and MuJoCo
    gym_locomotion_envs.py:18-19), SingleRobotEmptyScene(9.8, 0.0165, 1) for the pendulums
    (gym_pendulum_envs.py:14,48), StadiumScene(9.8, 0.0165/8, 8) for Atlas
    (gym_locomotion_envs.py:187), numSolverIterations 5
    (scene_bases.py:65)."""
    for env_id in _native.ROBOT_IDS:
        p = _native.default_sim_params(env_id)
        pend = "Pendulum" in env_id
        assert p.gravity == 9.8 and p.solver_iterations == 5, env_id
        fs = 1 if pend else (8 if "Atlas" in env_id else 4)
        assert p.frame_skip == fs, env_id
        assert p.timestep == 0.0165 / fs, env_id
        assert 0.0 <= p.contact_erp <= 1.0 and 0.0 <= p.joint_limit_erp <= 1.0
    over = _native.sim_params("AntPyBulletEnv-v0", {"gravity": 1.6, "frame_skip": 2})
    assert (over.gravity, over.frame_skip, over.solver_iterations) == (1.6, 2, 5)
    with pytest.raises(_native.PbgError):
        _native.sim_params("AntPyBulletEnv-v0", {"gravty": 1.0})
    with pytest.raises(_native.PbgError):
        _native.default_sim_params("NoSuchEnv-v0")


def test_create_opts_struct_matches_header():
    """_native.CreateOpts mirrors pbg_create_opts_t (struct_size first, then ints) and fills
    struct_size with its own size (the versioning rule of pbg_create_v2)."""
    src = open(HEADER).read()
    body = src[src.rindex("typedef struct {", 0, src.index("} pbg_create_opts_t;")):src.index("} pbg_create_opts_t;")]
    fields = re.findall(r"\b(uint32_t|int)\s+([a-z_0-9]+);", body)
    ct = {"uint32_t": ctypes.c_uint32, "int": ctypes.c_int}
    assert [(n, ct[t]) for t, n in fields] == list(_native.CreateOpts._fields_)
    o = _native.CreateOpts(precision=64)
    assert o.struct_size == ctypes.sizeof(_native.CreateOpts) and o.precision == 64 and o.kernel == -1
    assert _native.CreateOpts().precision == 64  # the reference's double is the default (round 6)


@pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="libpbg_amd.so not built")
def test_create_v2_refuses_bad_options_without_gpu():
    """pbg_create_v2 validates its versioned options before it touches a device: a struct_size that
    is no pbg_create_opts_t size and a precision other than 32 / 64 are PBG_E_ARG."""
    L = _native.lib()
    for size in (None, 4, 10, ctypes.sizeof(_native.CreateOpts) + 4):
        o = _native.CreateOpts(precision=16 if size is None else 64)
        if size is not None:
            o.struct_size = size  # shorter than struct_size + precision / not whole fields / too long
        h = ctypes.c_void_p(0x1234)  # a stale handle value: every failure must leave NULL
        rc = L.pbg_create_v2(b"AntPyBulletEnv-v0", 4, 0, 0, 0, None, ctypes.byref(o), ctypes.byref(h))
        assert rc == -1, (size, rc)
        assert not h.value, size
