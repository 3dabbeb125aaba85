"""ctypes binding of libpbg_amd.so (include/pbg.h).

The library is the product: there is no CPU fallback.  If it is missing or fails to
load, every entry point raises -- build it with ``python __graft_entry__.py`` (or
``make -C pybullet-gym_amd``)."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpbg_amd.so")

ROBOT_IDS = {"InvertedPendulumPyBulletEnv-v0": 0, "HopperPyBulletEnv-v0": 1, "HalfCheetahPyBulletEnv-v0": 2,
             "AntPyBulletEnv-v0": 3, "HumanoidPyBulletEnv-v0": 4, "Walker2DPyBulletEnv-v0": 5,
             "InvertedPendulumSwingupPyBulletEnv-v0": 6, "InvertedDoublePendulumPyBulletEnv-v0": 7,
             "HumanoidFlagrunPyBulletEnv-v0": 8, "HopperMuJoCoEnv-v0": 9, "Walker2DMuJoCoEnv-v0": 10,
             "HalfCheetahMuJoCoEnv-v0": 11, "AntMuJoCoEnv-v0": 12, "HumanoidMuJoCoEnv-v0": 13,
             "InvertedDoublePendulumMuJoCoEnv-v0": 14, "HumanoidFlagrunHarderPyBulletEnv-v0": 15,
             "AtlasPyBulletEnv-v0": 16}


class PbgError(RuntimeError):
    pass


class Info(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "robot_id", "n_envs", "action_dim", "obs_dim", "n_dof", "n_joints", "n_links", "n_feet", "state_words",
        "aux_words", "substeps", "max_episode_steps", "reset_dofs", "floating", "lanes_per_env", "block", "lds_bytes",
        "vgprs", "scratch_bytes", "lds_rows", "record_version")]


class StepIO(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("obs", ctypes.c_void_p), ("rew", ctypes.c_void_p),
                ("done", ctypes.c_void_p), ("rew64", ctypes.c_void_p), ("trunc", ctypes.c_void_p),
                ("term_obs", ctypes.c_void_p), ("ncontact", ctypes.c_void_p), ("autoreset", ctypes.c_int),
                ("rew_terms", ctypes.c_void_p), ("csig", ctypes.c_void_p)]


class DebugOpts(ctypes.Structure):
    """pbg_debug_opts_t: test / diagnostic launch options (-1 = default)."""
    _fields_ = [("kernel", ctypes.c_int), ("lds_rows", ctypes.c_int), ("gang_dist", ctypes.c_int),
                ("gang_lanes", ctypes.c_int)]


class CreateOpts(ctypes.Structure):
    """pbg_create_opts_t (pbg_create_v2): versioned by struct_size; precision 64 (default) or 32."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("precision", ctypes.c_int), ("kernel", ctypes.c_int),
                ("lds_rows", ctypes.c_int), ("gang_dist", ctypes.c_int), ("gang_lanes", ctypes.c_int)]

    def __init__(self, precision=64, kernel=-1, lds_rows=-1, gang_dist=-1, gang_lanes=-1):
        super().__init__(ctypes.sizeof(CreateOpts), precision, kernel, lds_rows, gang_dist, gang_lanes)


class SimParams(ctypes.Structure):
    """pbg_sim_params_t: the scene of a handle (scene_bases.py:8-18,58-73)."""
    _fields_ = [("gravity", ctypes.c_double), ("timestep", ctypes.c_double), ("frame_skip", ctypes.c_int),
                ("solver_iterations", ctypes.c_int), ("contact_erp", ctypes.c_double),
                ("joint_limit_erp", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {n: getattr(self, n) for n, _ in self._fields_}


_lib = None


def lib():
    """Load libpbg_amd.so, failing loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PbgError(f"{LIB_PATH} not found: the HIP extension is not built "
                       "(run `python __graft_entry__.py` or `make -C pybullet-gym_amd`)")
    L = ctypes.CDLL(LIB_PATH)
    P, I, H = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p
    L.pbg_create.argtypes = [ctypes.c_char_p, I, I, ctypes.c_uint64, I, ctypes.POINTER(H)]
    L.pbg_create.restype = I
    L.pbg_create_debug.argtypes = [ctypes.c_char_p, I, I, ctypes.c_uint64, I, ctypes.POINTER(DebugOpts),
                                   ctypes.POINTER(H)]
    L.pbg_create_ex.argtypes = [ctypes.c_char_p, I, I, ctypes.c_uint64, I, ctypes.POINTER(SimParams),
                                ctypes.POINTER(DebugOpts), ctypes.POINTER(H)]
    L.pbg_create_v2.argtypes = [ctypes.c_char_p, I, I, ctypes.c_uint64, I, ctypes.POINTER(SimParams),
                                ctypes.POINTER(CreateOpts), ctypes.POINTER(H)]
    L.pbg_precision.argtypes = [H]
    L.pbg_default_sim_params.argtypes = [ctypes.c_char_p, ctypes.POINTER(SimParams)]
    L.pbg_get_sim_params.argtypes = [H, ctypes.POINTER(SimParams)]
    L.pbg_sample_actions.argtypes = [I, I, I, ctypes.c_uint64, ctypes.c_uint32, I, P, P]
    L.pbg_destroy.argtypes = [H]
    L.pbg_destroy.restype = None
    L.pbg_info.argtypes = [H, ctypes.POINTER(Info)]
    L.pbg_reset.argtypes = [H, P, P, P, P]
    L.pbg_step.argtypes = [H, P, P, P, P, P]
    L.pbg_step_ex.argtypes = [H, ctypes.POINTER(StepIO), P]
    L.pbg_get_state.argtypes = [H, P, P, P]
    L.pbg_set_state.argtypes = [H, P, P, P]
    L.pbg_pack_record_sizes.argtypes = [ctypes.c_char_p, ctypes.POINTER(I), ctypes.POINTER(I)]
    L.pbg_pack.argtypes = [ctypes.c_char_p, I, P, P, P]
    if hasattr(L, "pbg_debug_poison"):  # diagnostic entry (tools/vgpr_poison_probe.py also loads older builds)
        L.pbg_debug_poison.argtypes = [H, ctypes.c_uint32, P]
        L.pbg_debug_poison.restype = I
    L.pbg_last_error.restype = ctypes.c_char_p
    for f in ("pbg_info", "pbg_reset", "pbg_step", "pbg_step_ex", "pbg_get_state", "pbg_set_state",
              "pbg_pack_record_sizes", "pbg_pack", "pbg_create_debug", "pbg_sample_actions", "pbg_create_ex",
              "pbg_default_sim_params", "pbg_get_sim_params", "pbg_create_v2", "pbg_precision"):
        getattr(L, f).restype = I
    _lib = L
    return L


EXPORTED = ("pbg_create", "pbg_create_debug", "pbg_create_ex", "pbg_create_v2", "pbg_precision",
            "pbg_default_sim_params", "pbg_get_sim_params",
            "pbg_destroy", "pbg_info", "pbg_reset", "pbg_step", "pbg_step_ex",
            "pbg_get_state", "pbg_set_state", "pbg_pack_record_sizes", "pbg_pack", "pbg_sample_actions",
            "pbg_debug_poison", "pbg_last_error")


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().pbg_last_error().decode(errors="replace")
        raise PbgError(f"{what} failed ({rc}): {msg}")


def default_sim_params(env_id: str) -> SimParams:
    """The scene parameters the reference builds env_id with (host-only call, no GPU needed)."""
    p = SimParams()
    check(lib().pbg_default_sim_params(env_id_bytes(env_id), ctypes.byref(p)), "pbg_default_sim_params")
    return p


def sim_params(env_id: str, overrides: dict = None) -> SimParams:
    """default_sim_params(env_id) with the fields in `overrides` replaced (unknown keys raise)."""
    p = default_sim_params(env_id)
    names = {n for n, _ in SimParams._fields_}
    for k, v in (overrides or {}).items():
        if k not in names:
            raise PbgError(f"unknown sim parameter {k!r}; known: {sorted(names)}")
        setattr(p, k, v)
    return p


def env_id_bytes(env_id: str) -> bytes:
    if env_id not in ROBOT_IDS:
        raise PbgError(f"unknown env id {env_id!r}; known: {sorted(ROBOT_IDS)}")
    return env_id.encode()
