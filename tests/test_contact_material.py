"""Contact material of HalfCheetahMuJoCo: restitution and spinning / rolling friction.

The reference's mujoco HalfCheetah sets every part's material in robot_specific_reset
(/root/reference/pybulletgym/envs/mujoco/robot_locomotors.py:207-210: lateralFriction 0.8,
spinningFriction 0.1, rollingFriction 0.1, restitution 0.5) against the stadium floor's
lateralFriction 0.8 / restitution 0.5 (envs/mujoco/scene_stadium.py:33).  Bullet combines them
per contact ([EXT] btManifoldResult: restitution r_a r_b = 0.25, spinning / rolling s_a mu_b + mu_a s_b
= 0.08; pybullet_gym_amd/codegen.py); the solver adds e (-v_n) to a normal row's target when the
approach speed is at least 0.2 m/s and solves three angular rows per contact (spin about the
normal, roll about the tangents) bounded by +-0.08 lambda_n before the lateral friction
(oracle/pbg_physics.h, csrc/pbg_step.hip, csrc/pbg_gang.hip).  Bullet itself is absent, so the
rule is unpinned; these tests hold the oracle to the rule's visible effect and the kernels to
the oracle.

The probe: the same half cheetah dropped onto the floor under zero actions.  HalfCheetahPyBullet
(roboschool: no material) and HalfCheetahMuJoCo share the MJCF, the masses and the dof layout, so
with zero torques their physics differ only by the material: identical until the first
contact, then the mujoco variant bounces (restitution) -- its upward root velocity after impact
is about twice the roboschool variant's.
"""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import oracle  # noqa: E402

MJ, PB = "HalfCheetahMuJoCoEnv-v0", "HalfCheetahPyBulletEnv-v0"
# (lift of the root above the reset pose [m], root vertical velocity [m/s]); state words: base 13,
# q[9], qd[9]; dof 1 is rootz (prismatic)
DROPS = [(0.1, -1.0), (0.3, -2.0), (0.0, -0.5), (0.2, 0.0)]
Z, VZ = 13 + 1, 13 + 9 + 1
STEPS = 40


def _drop_states(state):
    s = state.copy()
    for k, (h, v) in enumerate(DROPS):
        s[k, Z] += h
        s[k, VZ] = v
    return s


def _oracle_drop(env_id):
    o = oracle.OracleEnvs(env_id, len(DROPS))
    o.reset(np.zeros((len(DROPS), o.info.NR)))
    o.state[:] = _drop_states(o.state)
    out = []
    for _ in range(STEPS):
        o.step(np.zeros((len(DROPS), o.info.NA), np.float32))
        out.append(o.state.copy())
    return np.stack(out)


def _rebound(tr):
    """per drop: the largest upward root velocity after the deepest downward one"""
    v = tr[:, :, VZ]
    return np.array([v[np.argmin(v[:, k]):, k].max() for k in range(v.shape[1])])


def test_models_carry_the_combined_material():
    import json
    base = os.path.join(HERE, "..", "pybullet-gym_amd", "models")
    mj = json.load(open(os.path.join(base, "halfcheetah_mujoco.json")))
    assert mj["restitution"] == pytest.approx(0.25) and mj["spin_mu"] == pytest.approx(0.08)
    assert mj["roll_mu"] == pytest.approx(0.08)
    for name in os.listdir(base):
        if name.endswith(".json") and name not in ("halfcheetah_mujoco.json", "importer_overrides.json"):
            t = json.load(open(os.path.join(base, name)))
            assert t["restitution"] == 0.0 and t["spin_mu"] == 0.0 and t["roll_mu"] == 0.0, name


def test_oracle_restitution_bounces_the_mujoco_cheetah():
    a, b = _oracle_drop(MJ), _oracle_drop(PB)
    # identical flight before any contact (same MJCF, zero torques): the first env step of the
    # drops that start above the contact threshold
    np.testing.assert_array_equal(a[0, [0, 1, 3]], b[0, [0, 1, 3]])
    ra, rb = _rebound(a), _rebound(b)
    print("rebound vz mujoco", ra, "roboschool", rb)
    assert (ra >= 1.5 * rb).all() and (ra > 0.25).all(), (ra, rb)
    assert np.isfinite(a).all()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [64, 32])
def test_gpu_drop_matches_oracle(precision):
    """The gang kernel (and, float64, the lane kernel) free-running from the drop states: within
    1e-9 (float64) / 1e-3 (float32) of the oracle's trajectory over 40 steps, the bounce included."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pybulletgym_amd  # noqa: F401
    from pybulletgym_amd.vec_env import VecEnv
    ref = _oracle_drop(MJ)
    tol = 1e-9 if precision == 64 else 1e-3
    for kw in ({}, {"kernel": 0}) if precision == 64 else ({},):
        env = VecEnv(MJ, len(DROPS), seed=0, autoreset=False, precision=precision, **kw)
        env.reset(init_q=torch.zeros((len(DROPS), env.info.reset_dofs)))
        phys, aux = env.get_state()
        env.set_state(torch.from_numpy(_drop_states(phys.cpu().numpy())).cuda(), aux)
        out = []
        for _ in range(STEPS):
            env.step(torch.zeros((len(DROPS), env.info.action_dim), device="cuda"))
            out.append(env.get_state()[0].cpu().numpy())
        env.close()
        g = np.stack(out)
        err = (np.abs(g - ref) / np.maximum(1.0, np.abs(ref))).max()
        print(f"precision {precision} {kw}: max rel err {err:.3e}, rebound {_rebound(g)}")
        assert err <= tol, (kw, err)
        assert (_rebound(g) >= 0.9 * _rebound(ref)).all()
