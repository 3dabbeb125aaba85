"""The oracle's dynamics against independent finite-difference checks (kinetic energy,
gravity potential, bias accelerations), plus rollout sanity and reset semantics."""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle

KEYS = ["hopper", "halfcheetah", "ant", "humanoid", "walker2d"]
MODELS = os.path.join(os.path.dirname(__file__), "..", "pybullet-gym_amd", "models")


def tables(key):
    return json.load(open(os.path.join(MODELS, f"{key}.json")))


def _lib():
    L = oracle.lib()
    L.pbg_oracle_set_flags.argtypes = [ctypes.c_int]
    L.pbg_oracle_link_frames.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3
    L.pbg_oracle_link_vel.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5
    return L


def frames(key, s):
    info = oracle.Info(oracle.robot_id(key))
    R = np.zeros((info.NL + 1, 9))
    c = np.zeros((info.NL + 1, 3))
    _lib().pbg_oracle_link_frames(oracle.robot_id(key), oracle._p(np.ascontiguousarray(s)), oracle._p(R), oracle._p(c))
    return R.reshape(-1, 3, 3), c


def link_vel(key, s):
    info = oracle.Info(oracle.robot_id(key))
    out = [np.zeros((info.NL + 1, 3)) for _ in range(4)]
    _lib().pbg_oracle_link_vel(oracle.robot_id(key), oracle._p(np.ascontiguousarray(s)), *[oracle._p(o) for o in out])
    return out


def advance(info, s, nu, h):
    """Move a state by h along generalized velocity nu (base: world lin/ang velocity)."""
    s2 = s.copy()
    off = 0
    if info.floating:
        s2[0:3] += h * nu[0:3]
        w = nu[3:6]
        ang = np.linalg.norm(w) * h
        ax = w / np.linalg.norm(w)
        a, b, c, d = np.r_[ax * np.sin(ang / 2), np.cos(ang / 2)]
        x, y, z, ww = s[3:7]
        s2[3:7] = [d * x + a * ww + b * z - c * y, d * y - a * z + b * ww + c * x,
                   d * z + a * y - b * x + c * ww, d * ww - a * x - b * y - c * z]
        off = 6
    s2[13:13 + info.NJ] += h * nu[off:]
    return s2


def random_state(key, seed):
    t = tables(key)
    info = oracle.Info(oracle.robot_id(key))
    rng = np.random.default_rng(seed)
    s = np.zeros(info.SD)
    s[0:3] = t["base_pos"]
    s[3:7] = t["base_quat"]
    s[13:13 + info.NJ] = rng.uniform(-0.5, 0.5, info.NJ)
    return s, rng, info, t


@pytest.mark.parametrize("key", KEYS)
def test_mass_matrix_is_kinetic_energy(key):
    s, rng, info, t = random_state(key, 0)
    nu = rng.standard_normal(info.NDOF)
    M, _ = oracle.dynamics(key, s)
    eps = 1e-6
    R0, c0 = frames(key, advance(info, s, nu, -eps))
    R1, c1 = frames(key, advance(info, s, nu, eps))
    Rm, _ = frames(key, s)
    v = (c1 - c0) / (2 * eps)
    masses = [t["base_mass"]] + t["link_mass"]
    inert = [t["base_inertia"]] + t["link_inertia"]
    T = 0.0
    for b in range(info.NL + 1):
        if b == 0 and not info.floating:
            continue
        W = ((R1[b] - R0[b]) / (2 * eps)) @ Rm[b].T
        w = np.array([W[2, 1], W[0, 2], W[1, 0]])
        I6 = inert[b]
        I = np.array([[I6[0], I6[3], I6[4]], [I6[3], I6[1], I6[5]], [I6[4], I6[5], I6[2]]])
        T += 0.5 * masses[b] * v[b] @ v[b] + 0.5 * w @ (Rm[b] @ I @ Rm[b].T) @ w
    arm = np.zeros(info.NDOF)
    arm[(6 if info.floating else 0):] = t["dof_armature"]
    assert 0.5 * nu @ (M - np.diag(arm)) @ nu == pytest.approx(T, rel=1e-7)
    assert np.linalg.eigvalsh(M).min() > 0


@pytest.mark.parametrize("key", KEYS)
def test_gravity_is_potential_gradient(key):
    s, rng, info, t = random_state(key, 1)
    L = _lib()
    L.pbg_oracle_set_flags(4)  # no body damping; velocities are zero anyway
    try:
        _, C = oracle.dynamics(key, s)
        d = rng.standard_normal(info.NDOF)
        masses = [t["base_mass"]] + t["link_mass"]

        def V(st):
            _, c = frames(key, st)
            return sum(masses[b] * 9.8 * c[b][2] for b in range(info.NL + 1))

        eps = 1e-6
        dV = (V(advance(info, s, d, eps)) - V(advance(info, s, d, -eps))) / (2 * eps)
        assert C @ d == pytest.approx(dV, rel=1e-6, abs=1e-9)
    finally:
        L.pbg_oracle_set_flags(0)


@pytest.mark.parametrize("key", KEYS)
def test_bias_accelerations_are_jdot_nu(key):
    s, rng, info, t = random_state(key, 2)
    s[13 + info.NJ:] = rng.standard_normal(info.NJ)
    if info.floating:
        s[7:13] = rng.standard_normal(6)
    nu = np.r_[s[7:13], s[13 + info.NJ:]] if info.floating else s[13 + info.NJ:]
    eps = 1e-6
    v1, w1, _, _ = link_vel(key, advance(info, s, nu, eps))
    v0, w0, _, _ = link_vel(key, advance(info, s, nu, -eps))
    _, _, ac, al = link_vel(key, s)
    np.testing.assert_allclose((v1 - v0) / (2 * eps), ac, atol=1e-7 * max(1, np.abs(ac).max()))
    np.testing.assert_allclose((w1 - w0) / (2 * eps), al, atol=1e-7 * max(1, np.abs(al).max()))


@pytest.mark.parametrize("key", KEYS + ["pendulum", "pendulum_swingup", "double_pendulum"])
def test_random_rollout_stays_finite(key):
    n = 32
    e = oracle.OracleEnvs(key, n, nthreads=4)
    rng = np.random.default_rng(3)
    e.reset(rng.uniform(-0.1, 0.1, (n, e.info.NR)))
    for _ in range(100):
        obs, r, d, nc = e.step(rng.uniform(-1, 1, (n, e.info.NA)).astype(np.float32))
        assert np.isfinite(e.state).all()
        assert np.isfinite(obs).all() and np.isfinite(r).all()
        if "pendulum" not in key:
            assert np.abs(obs).max() <= 5.0  # robot_locomotors.py:64 (the pendulum does not clip)
    if "pendulum" not in key:
        assert (e.state[:, 13 + e.info.NJ:] ** 2).max() <= 100.0 ** 2 + 1e-6  # maxCoordinateVelocity


def test_ant_falls_onto_floor_and_rests():
    """Zero action: the Ant drops onto its four feet and stands (torso z between the sphere
    radius and the start, steady over the last 100 steps; the 96 kg ant on a 5-sweep PGS
    keeps a few cm/s of contact jitter, so 'at rest' is a loose bound)."""
    e = oracle.OracleEnvs("ant", 1)
    e.reset(np.zeros((1, 8)))
    zs = []
    for _ in range(300):
        obs, r, d, nc = e.step(np.zeros((1, 8), np.float32))
        zs.append(e.state[0, 2])
    z = e.state[0, 2]
    assert 0.25 < z < 0.75
    assert np.std(zs[-100:]) < 0.01
    assert nc[0] >= 4  # at least the four feet
    assert np.abs(e.state[0, 7:13]).max() < 0.3


def test_reset_semantics():
    """First reset excludes the floor from the parts mean, later resets include it
    (gym_locomotion_envs.py:27-31); potential = -dist/dt; feet_contact zero."""
    e = oracle.OracleEnvs("ant", 1)
    q = np.array([[0.09, -0.08, 0.07, 0.1, -0.02, 0.03, -0.1, 0.06]])
    o1 = e.reset(q)
    pot1 = e.aux[0, 0]
    assert e.aux[0, 3] == 1.0
    o2 = e.reset(q)
    pot2 = e.aux[0, 0]
    assert pot1 != pot2  # 13 vs 14 parts in the x mean
    np.testing.assert_array_equal(o1[0, -4:], 0)
    assert e.aux[0, 1] == pytest.approx(0.75)  # initial_z = torso z at reset
    h = oracle.OracleEnvs("humanoid", 1)
    h.reset(np.zeros((1, 17)))
    assert h.aux[0, 1] == 0.8  # Humanoid fixes initial_z (robot_locomotors.py:183)


@pytest.mark.parametrize("env_id", ["HopperPyBulletEnv-v0", "AntPyBulletEnv-v0"])
def test_mca_float32_runs_bracket_ieee_float32(env_id):
    """The float32 Monte Carlo arithmetic instantiation (oracle/mca.h, precision 33) that the
    GPU parity tests use to explain outliers: a stream is reproducible for a seed and differs
    across seeds; over a rollout its spread around float64 has the scale of the IEEE float32
    instantiation's error (median within 10x either way), far below the physics itself."""
    n, R = 64, 8
    e = oracle.OracleEnvs(env_id, n, nthreads=8)
    e.reset(np.random.default_rng(0).uniform(-0.1, 0.1, (n, e.info.NR)))
    acts = np.random.default_rng(1).uniform(-1, 1, (12, n, e.info.NA)).astype(np.float32)
    for t in range(10):
        e.step(acts[t])
    st, ax, a = e.state.copy(), e.aux.copy(), acts[10]

    def run(prec, seed=0, reps=1):
        o = oracle.OracleEnvs(env_id, n * reps, nthreads=8, precision=prec)
        oracle.set_mca_seed(seed)
        o.state[:] = np.repeat(st, reps, 0)
        o.aux[:] = np.repeat(ax, reps, 0)
        return o.step(np.repeat(a, reps, 0))[0]
    o64, o32 = run(64), run(32)
    m1, m2, m3 = run(33, 5), run(33, 5), run(33, 6)
    np.testing.assert_array_equal(m1, m2)
    assert (m1 != m3).any()
    rel = lambda x, y: (np.abs(x.astype(np.float64) - y) / np.maximum(1, np.abs(y))).max(axis=1)  # noqa: E731
    e32 = rel(o32, o64)
    emca = rel(run(33, 7, R), np.repeat(o64, R, 0)).reshape(n, R).max(axis=1)
    assert np.median(emca) <= 10 * max(np.median(e32), 1e-7) and np.median(e32) <= 10 * max(np.median(emca), 1e-7)
    assert np.median(emca) < 1e-3


def test_scene_parameters_enter_the_physics():
    """pbg_oracle_set_sim_params (the oracle side of pbg_create_ex's pbg_sim_params_t): the
    bias forces are the potential gradient under the new gravity; a changed sub-step count,
    iteration count or ERP changes the rollout; NULL restores the reference's scene bit for bit."""
    key = "hopper"
    s, rng, info, t = random_state(key, 1)
    L = _lib()
    sp = {"gravity": 3.7, "timestep": 0.0165 / 4, "frame_skip": 4, "solver_iterations": 5,
          "contact_erp": 0.2, "joint_limit_erp": 0.2}
    L.pbg_oracle_set_flags(4)
    oracle.set_sim_params(sp)
    try:
        _, C = oracle.dynamics(key, s)
        d = rng.standard_normal(info.NDOF)
        masses = [t["base_mass"]] + t["link_mass"]

        def V(st):
            _, c = frames(key, st)
            return sum(masses[b] * 3.7 * c[b][2] for b in range(info.NL + 1))

        eps = 1e-6
        dV = (V(advance(info, s, d, eps)) - V(advance(info, s, d, -eps))) / (2 * eps)
        assert C @ d == pytest.approx(dV, rel=1e-6, abs=1e-9)
    finally:
        L.pbg_oracle_set_flags(0)
        oracle.set_sim_params(None)

    def rollout(params):
        oracle.set_sim_params(params)
        try:
            e = oracle.OracleEnvs("ant", 4, nthreads=4)
            r = np.random.default_rng(5)
            e.reset(r.uniform(-0.1, 0.1, (4, 8)))
            for _ in range(20):
                obs, rew, _, _ = e.step(r.uniform(-1, 1, (4, 8)).astype(np.float32))
            return obs.copy(), rew.copy(), e.info.substeps
        finally:
            oracle.set_sim_params(None)

    base, rb, nsub = rollout(None)
    assert nsub == 4
    ref = dict(sp, gravity=9.8)
    same, rs, _ = rollout(ref)
    np.testing.assert_array_equal(base, same)
    np.testing.assert_array_equal(rb, rs)
    for over in ({"frame_skip": 5}, {"solver_iterations": 3}, {"contact_erp": 0.5}, {"gravity": 9.0}):
        other, _, ns = rollout(dict(ref, **over))
        assert np.isfinite(other).all() and np.abs(other - base).max() > 1e-3, over
        assert ns == ref["frame_skip"] if "frame_skip" not in over else ns == over["frame_skip"]
    again, ra, _ = rollout(None)
    np.testing.assert_array_equal(base, again)
