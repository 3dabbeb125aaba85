"""GPU parity: the HIP path (libpbg_amd.so through its C-ABI) against the golden vectors
and the CPU oracle.  Run on an MI355X:  python -m pytest tests -m gpu

Tolerances (stated per test):
  * pack on golden inputs: float32 obs bit-exact, done/feet exact, reward |d| <= 1e-9
    (float64 sum; the slack covers the BLAS dot order in np.linalg.norm).
  * reset (same init_q): obs |d| <= 1e-5 (float32 vs float64 forward kinematics).
  * one teacher-forced env step (GPU float32 physics vs oracle float64 from the same
    state): done flags identical; contact counts identical in >= 99.9% of env-steps;
    median per-env obs error <= 1e-4 and 99th percentile <= 1e-2.  The tails come from
    the contact/PGS sensitivity that the oracle shows against its OWN float32-rounded
    state (tools/gpu_check.py prints both); SURVEY.md section 7 "chaotic divergence".
"""
import os

import numpy as np
import pytest
import torch

import oracle
import pybulletgym_amd  # noqa: F401
from pybulletgym_amd import rng
from pybulletgym_amd.vec_env import VecEnv, pack, pack_record_sizes

pytestmark = pytest.mark.gpu

ENVS = ["InvertedPendulumPyBulletEnv-v0", "HopperPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0",
        "AntPyBulletEnv-v0", "HumanoidPyBulletEnv-v0", "Walker2DPyBulletEnv-v0",
        "InvertedPendulumSwingupPyBulletEnv-v0", "InvertedDoublePendulumPyBulletEnv-v0",
        "HumanoidFlagrunPyBulletEnv-v0", "HopperMuJoCoEnv-v0", "Walker2DMuJoCoEnv-v0",
        "HalfCheetahMuJoCoEnv-v0", "AntMuJoCoEnv-v0", "HumanoidMuJoCoEnv-v0", "InvertedDoublePendulumMuJoCoEnv-v0"]
KEY = {e: oracle.ENV_KEYS[e] for e in ENVS}
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# ------------------------------------------------------------------ pack vs reference golden vectors
@pytest.mark.parametrize("env_id", ENVS)
def test_device_pack_matches_reference_golden(env_id):
    key = KEY[env_id]
    g = np.load(os.path.join(GOLDEN, f"pack_{key}.npz"))
    info = oracle.Info(oracle.robot_id(key))
    iw, ow = pack_record_sizes(env_id)
    n = len(g["kind"])
    rec = np.zeros((n, iw))
    NP1 = info.NP + 1
    for i in range(n):
        o = 0
        if info.kind in (0, 3):
            px = np.zeros((NP1, 3))
            px[: g["n_parts"][i]] = g["part_xyz"][i][: g["n_parts"][i]]
            rec[i, : 3 * NP1] = px.ravel()
            rec[i, 3 * NP1] = g["n_parts"][i]
        o = 3 * NP1 + 1
        if info.kind in (0, 3):
            rec[i, o:o + 4] = g["body_quat"][i]
            rec[i, o + 4:o + 7] = g["body_pos"][i]
            rec[i, o + 7:o + 10] = g["body_vel"][i]
        elif "body_pos" in g.files and g["body_pos"].size:  # double pendulum: pole2; MuJoCo: robot_body
            rec[i, o + 4:o + 7] = g["body_pos"][i]
        o += 10
        rec[i, o:o + info.NO] = g["jq"][i]
        rec[i, o + info.NO:o + 2 * info.NO] = g["jqd"][i]
        o += 2 * info.NO
        if info.kind in (0, 3):
            rec[i, o:o + info.NF] = g["feet_prev"][i][: info.NF]
            rec[i, o + info.NF:o + 2 * info.NF] = g["feet_new"][i][: info.NF]
        o += 2 * info.NF
        rec[i, o:o + info.NA] = g["act"][i]
        o += info.NA
        rec[i, o] = g["potential_old"][i]
        rec[i, o + 1] = g["initial_z_in"][i] if info.kind in (0, 3) else 0.0
        rec[i, o + 2] = float(g["kind"][i] == 1)
        if "flag_in" in g.files:  # HumanoidFlagrun: target, flag_timeout, the recorded re-draw
            rec[i, o + 3:o + 8] = g["flag_in"][i]
        if "body_avel" in g.files:  # MuJoCo Ant / Humanoid: torso angular velocity
            rec[i, o + 3:o + 6] = g["body_avel"][i]
    out = pack(env_id, torch.from_numpy(rec).cuda()).cpu().numpy()
    obs = out[:, : info.OBS].astype(np.float32)
    ref = g["obs"].astype(np.float32)
    np.testing.assert_array_equal(obs.view(np.uint32), ref.view(np.uint32))
    step = g["kind"] == 1
    np.testing.assert_array_equal(out[step, info.OBS + 1].astype(bool), g["done"][step])
    np.testing.assert_allclose(out[step, info.OBS], g["reward"][step], atol=1e-9, rtol=0)
    if info.kind == 2:  # MuJoCo planar: x_after
        np.testing.assert_array_equal(out[:, info.OBS + 2], g["potential"])
    if info.kind in (0, 3):
        np.testing.assert_allclose(out[:, info.OBS + 2], g["potential"], atol=1e-9, rtol=0)
        np.testing.assert_array_equal(out[:, info.OBS + 3], g["initial_z_out"])
        np.testing.assert_array_equal(out[:, info.OBS + 4:info.OBS + 4 + info.NF], g["feet_out"][:, : info.NF])
    if "flag_out" in g.files:
        np.testing.assert_array_equal(out[:, info.OBS + 4 + info.NF:], g["flag_out"])


# ------------------------------------------------------------------ reset
@pytest.mark.parametrize("env_id", ENVS)
def test_reset_matches_oracle(env_id):
    n = 128
    env = VecEnv(env_id, n, seed=5, autoreset=False)
    orc = oracle.OracleEnvs(env_id, n, seed=5)
    q0 = np.random.default_rng(0).uniform(-0.1, 0.1, (n, env.info.reset_dofs)).astype(np.float32)
    obs = env.reset(init_q=torch.from_numpy(q0)).cpu().numpy()
    obs_o = orc.reset(q0.astype(np.float64))
    np.testing.assert_allclose(obs, obs_o, atol=1e-5, rtol=0)
    phys, aux = env.get_state()
    np.testing.assert_allclose(phys.cpu().numpy(), orc.state, atol=1e-7, rtol=1e-7)  # float32 rounding of the float64 state
    np.testing.assert_allclose(aux.cpu().numpy(), orc.aux, atol=2e-6, rtol=0)


@pytest.mark.parametrize("env_id", ["AntPyBulletEnv-v0", "HumanoidPyBulletEnv-v0"])
def test_rng_reset_matches_host_philox(env_id):
    n, seed, off = 64, 1234, 1000
    env = VecEnv(env_id, n, seed=seed, env_offset=off, autoreset=False)
    env.reset()
    env.reset()  # second episode
    phys, _ = env.get_state()
    t = oracle.Info(oracle.robot_id(KEY[env_id]))
    import json
    tab = json.load(open(os.path.join(os.path.dirname(__file__), "..", "pybullet-gym_amd", "models",
                                      f"{KEY[env_id]}.json")))
    q = phys.cpu().numpy()[:, 13:13 + t.NJ]
    want = rng.reset_noise(seed, np.arange(off, off + n), 1, t.NR)
    np.testing.assert_array_equal(q[:, tab["reset_dof"]].astype(np.float32), want)


# ------------------------------------------------------------------ teacher-forced step parity
@pytest.mark.parametrize("env_id", ENVS)
def test_step_teacher_forced_parity(env_id):
    n, steps = 256, 40
    env = VecEnv(env_id, n, seed=3, autoreset=False)
    orc = oracle.OracleEnvs(env_id, n, nthreads=8, seed=3)
    r = np.random.default_rng(1)
    q0 = r.uniform(-0.1, 0.1, (n, env.info.reset_dofs)).astype(np.float32)
    env.reset(init_q=torch.from_numpy(q0))
    errs, cmis, total = [], 0, 0
    for _ in range(steps):
        phys, aux = env.get_state()
        orc.state[:] = phys.cpu().numpy()
        orc.aux[:] = aux.cpu().numpy()
        a = r.uniform(-1, 1, (n, env.info.action_dim)).astype(np.float32)
        res = env.step(torch.from_numpy(a).cuda(), want_reward64=True, want_contacts=True)
        og = res.obs.cpu().numpy()
        dg = res.done.cpu().numpy().astype(bool)
        cg = env.ncontact.cpu().numpy()
        oo, ro, do, co = orc.step(a)
        np.testing.assert_array_equal(dg, do)
        cmis += int((cg != co).sum())
        total += n
        errs.append(np.abs(og - oo).max(axis=1))
    e = np.concatenate(errs)
    assert np.median(e) <= 1e-4, np.median(e)
    assert np.percentile(e, 99) <= 1e-2, np.percentile(e, 99)
    assert cmis <= 0.001 * total, (cmis, total)


def test_free_running_short_horizon_ant():
    """No teacher forcing: 10 steps from identical resets stay within 1e-3 (obs)."""
    n = 128
    env = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False)
    orc = oracle.OracleEnvs("AntPyBulletEnv-v0", n)
    r = np.random.default_rng(2)
    q0 = r.uniform(-0.1, 0.1, (n, 8)).astype(np.float32)
    env.reset(init_q=torch.from_numpy(q0))
    orc.reset(q0.astype(np.float64))
    for _ in range(10):
        a = r.uniform(-1, 1, (n, 8)).astype(np.float32)
        og = env.step(torch.from_numpy(a).cuda()).obs.cpu().numpy()
        oo, _, _, _ = orc.step(a)
    assert np.median(np.abs(og - oo).max(axis=1)) < 1e-3


# ------------------------------------------------------------------ episode bookkeeping
def test_autoreset_and_time_limit():
    n = 64
    env = VecEnv("AntPyBulletEnv-v0", n, seed=9, autoreset=True)
    env.reset()
    phys, aux = env.get_state()
    aux[:, 2] = 999.0  # elapsed: next step hits max_episode_steps = 1000
    env.set_state(phys, aux)
    res = env.step(torch.zeros((n, 8), device="cuda"))
    assert res.done.all() and res.truncated.sum() >= 1
    _, aux2 = env.get_state()
    assert (aux2[:, 2] == 0).all()  # every env was reset in the same launch
    # the returned obs is the reset obs: zero feet_contact (robot_locomotors.py:22)
    assert (res.obs[:, -4:] == 0).all()
    assert torch.isfinite(res.terminal_obs).all()


def test_determinism_and_env_offset_invariance():
    """Same seed -> bitwise identical rollouts; env i of a shard with env_offset k equals
    env k+i of a bigger batch (sharding does not change trajectories)."""
    def run(n, off):
        env = VecEnv("HopperPyBulletEnv-v0", n, seed=21, env_offset=off, autoreset=True)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand((30, 64, 3), device="cuda", generator=g) * 2 - 1
        outs = []
        for t in range(30):
            outs.append(env.step(acts[t][off:off + n].contiguous()).obs.clone())
        return torch.stack(outs).cpu().numpy()
    a = run(64, 0)
    b = run(64, 0)
    np.testing.assert_array_equal(a, b)
    c = run(32, 32)
    np.testing.assert_array_equal(a[:, 32:], c)


def test_large_batch_stays_finite():
    """BASELINE config sizes: Ant 16,384 envs for 200 random steps with auto-reset."""
    n = 16384
    env = VecEnv("AntPyBulletEnv-v0", n, seed=4, autoreset=True)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    dones = 0
    for _ in range(200):
        res = env.step(torch.rand((n, 8), device="cuda", generator=g) * 2 - 1)
        dones += int(res.done.sum())
    assert torch.isfinite(res.obs).all() and torch.isfinite(res.reward).all()
    assert res.obs.abs().max() <= 5.0
    phys, _ = env.get_state()
    assert torch.isfinite(phys).all()
    assert dones < n * 200


# ------------------------------------------------------------------ gym-style facade
@pytest.mark.parametrize("env_id", ENVS)
def test_sanity_check_every_env(env_id):
    """gym_sanity_check.py:1-18: make, reset, one step of np.random.random(shape)."""
    from pybulletgym_amd import make
    env = make(env_id)
    obs = env.reset()
    assert obs.shape == env.observation_space.shape
    obs, r, done, info = env.step(np.random.random(env.action_space.shape))
    assert isinstance(r, float) and isinstance(done, bool) and isinstance(info, dict)
    f64 = "Pendulum" in env_id or env_id in ("AntMuJoCoEnv-v0", "HumanoidMuJoCoEnv-v0")  # float64 in the reference
    assert obs.dtype == (np.float64 if f64 else np.float32)
    env.close()


def test_facade_matches_vecenv_and_time_limit():
    from pybulletgym_amd import make
    env = make("HopperPyBulletEnv-v0")
    env.seed(3)
    o = env.reset()
    vec = VecEnv("HopperPyBulletEnv-v0", 1, seed=3, autoreset=False)
    ov = vec.reset()
    np.testing.assert_array_equal(o, ov[0].cpu().numpy())
    a = np.array([0.3, -0.2, 0.5], np.float32)
    o1, r1, d1, _ = env.step(a)
    res = vec.step(torch.from_numpy(a.reshape(1, 3)), want_reward64=True)
    np.testing.assert_array_equal(o1, res.obs[0].cpu().numpy())
    assert r1 == float(vec.reward64[0])
    env.env._vec.set_state(*env.env._vec.get_state())
    env._elapsed = 999
    _, _, done, info = env.step(a)
    assert done


# ------------------------------------------------------------------ kernel variants
def _ant_rollout(monkeypatch, n=256, steps=30, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = VecEnv("AntPyBulletEnv-v0", n, seed=11, autoreset=True)
    for k in env:
        monkeypatch.delenv(k)
    e.reset()
    g = torch.Generator(device="cuda").manual_seed(5)
    obs, nc = [], []
    for _ in range(steps):
        res = e.step(torch.rand((n, 8), device="cuda", generator=g) * 2 - 1, want_contacts=True)
        obs.append(res.obs.clone())
        nc.append(e.ncontact.clone())
    return torch.stack(obs).cpu().numpy(), torch.stack(nc).cpu().numpy()


@pytest.mark.parametrize("team", ["1", "0"])
def test_workspace_rows_bitwise_equal_lds_rows(monkeypatch, team):
    """Contact rows past the LDS capacity live in the device workspace: forcing every row
    there (PBG_LDS_ROWS=0) must not change a single bit (quad and lane kernels)."""
    a, ca = _ant_rollout(monkeypatch, PBG_TEAM=team)
    b, cb = _ant_rollout(monkeypatch, PBG_TEAM=team, PBG_LDS_ROWS="0")
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_quad_kernel_matches_lane_kernel_teacher_forced(monkeypatch):
    """Ant's quad-per-env kernel (pbg_team.hip) vs the one-lane-per-env kernel from the same
    states: same physics, different float32 summation order.  Tolerances as for the
    oracle comparison: done identical, contacts identical in >= 99.9 %, median obs error
    <= 1e-4, 99th percentile <= 1e-2."""
    n, steps = 512, 30
    quad = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False)
    monkeypatch.setenv("PBG_TEAM", "0")
    lane = VecEnv("AntPyBulletEnv-v0", n, seed=3, autoreset=False)
    monkeypatch.delenv("PBG_TEAM")
    r = np.random.default_rng(7)
    q0 = torch.from_numpy(r.uniform(-0.1, 0.1, (n, 8)).astype(np.float32))
    quad.reset(init_q=q0)
    errs, cmis = [], 0
    for _ in range(steps):
        lane.set_state(*quad.get_state())
        a = torch.from_numpy(r.uniform(-1, 1, (n, 8)).astype(np.float32)).cuda()
        rq = quad.step(a, want_contacts=True)
        rl = lane.step(a, want_contacts=True)
        np.testing.assert_array_equal(rq.done.cpu().numpy(), rl.done.cpu().numpy())
        cmis += int((quad.ncontact != lane.ncontact).sum())
        errs.append((rq.obs - rl.obs).abs().max(dim=1).values.cpu().numpy())
    e = np.concatenate(errs)
    assert np.median(e) <= 1e-4, np.median(e)
    assert np.percentile(e, 99) <= 1e-2, np.percentile(e, 99)
    assert cmis <= 0.001 * n * steps, cmis


def test_quad_kernel_determinism_and_offset_invariance():
    def run(n, off):
        env = VecEnv("AntPyBulletEnv-v0", n, seed=21, env_offset=off, autoreset=True)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand((30, 96, 8), device="cuda", generator=g) * 2 - 1
        return torch.stack([env.step(acts[t][off:off + n].contiguous()).obs.clone() for t in range(30)]).cpu().numpy()
    a = run(96, 0)
    np.testing.assert_array_equal(a, run(96, 0))
    np.testing.assert_array_equal(a[:, 40:], run(56, 40))


# ------------------------------------------------------------------ gang kernel (pbg_gang.hip)
def _variant_vs_lane(monkeypatch, env_id, n, steps, variant_env, seed=3):
    """Teacher-forced comparison of a kernel variant against the lane kernel from the same
    states each step; returns (per-env max obs errors, contact-count mismatches)."""
    for k, v in variant_env.items():
        monkeypatch.setenv(k, v)
    var = VecEnv(env_id, n, seed=seed, autoreset=False)
    for k in variant_env:
        monkeypatch.delenv(k)
    monkeypatch.setenv("PBG_TEAM", "0")
    lane = VecEnv(env_id, n, seed=seed, autoreset=False)
    monkeypatch.delenv("PBG_TEAM")
    assert lane.info.lanes_per_env == 1
    r = np.random.default_rng(7)
    na, nr = var.info.action_dim, var.info.reset_dofs
    var.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, nr)).astype(np.float32)))
    errs, cmis = [], 0
    for _ in range(steps):
        lane.set_state(*var.get_state())
        a = torch.from_numpy(r.uniform(-1, 1, (n, na)).astype(np.float32)).cuda()
        rv = var.step(a, want_contacts=True)
        rl = lane.step(a, want_contacts=True)
        np.testing.assert_array_equal(rv.done.cpu().numpy(), rl.done.cpu().numpy())
        cmis += int((var.ncontact != lane.ncontact).sum())
        errs.append((rv.obs - rl.obs).abs().max(dim=1).values.cpu().numpy())
    return var.info.lanes_per_env, np.concatenate(errs), cmis


@pytest.mark.parametrize("env_id,variant", [("HumanoidPyBulletEnv-v0", {}), ("HopperPyBulletEnv-v0", {}),
                                            ("HalfCheetahPyBulletEnv-v0", {}), ("Walker2DPyBulletEnv-v0", {}),
                                            ("AntPyBulletEnv-v0", {"PBG_TEAM": "2"}),
                                            ("HumanoidPyBulletEnv-v0", {"PBG_GANG_DIST": "0"}),
                                            ("Walker2DPyBulletEnv-v0", {"PBG_GANG_DIST": "1"})])
def test_gang_kernel_matches_lane_kernel_teacher_forced(monkeypatch, env_id, variant):
    """16-lanes-per-env gang kernel (distributed or replicated dynamics) vs the
    one-lane-per-env kernel from the same states: same physics and row order, different
    float32 summation order (DPP tree dots, level-order composites) and constant-table
    transforms.  Tolerances as for the oracle comparison: done identical,
    contacts identical in >= 99.9 %, median obs error <= 1e-4, 99th percentile <= 1e-2."""
    n, steps = 256, 30
    lanes, e, cmis = _variant_vs_lane(monkeypatch, env_id, n, steps, variant)
    assert lanes == 16
    assert np.median(e) <= 1e-4, np.median(e)
    assert np.percentile(e, 99) <= 1e-2, np.percentile(e, 99)
    assert cmis <= 0.001 * n * steps, cmis


def _rollout(monkeypatch, env_id, n=128, steps=40, seed=11, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = VecEnv(env_id, n, seed=seed, autoreset=True)
    for k in env:
        monkeypatch.delenv(k)
    e.reset()
    g = torch.Generator(device="cuda").manual_seed(5)
    obs, nc = [], []
    for _ in range(steps):
        res = e.step(torch.rand((n, e.info.action_dim), device="cuda", generator=g) * 2 - 1, want_contacts=True)
        obs.append(res.obs.clone())
        nc.append(e.ncontact.clone())
    return torch.stack(obs).cpu().numpy(), torch.stack(nc).cpu().numpy()


def test_gang_workspace_contacts_bitwise_equal_lds_contacts(monkeypatch):
    """Gang contacts past the LDS capacity live in the device workspace: forcing every
    contact there (PBG_LDS_ROWS=0) must not change a single bit (Humanoid: floor + self)."""
    a, ca = _rollout(monkeypatch, "HumanoidPyBulletEnv-v0")
    b, cb = _rollout(monkeypatch, "HumanoidPyBulletEnv-v0", PBG_LDS_ROWS="0")
    assert ca.max() > 0
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("env_id", ["HumanoidPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0"])
def test_gang_kernel_determinism_and_offset_invariance(env_id):
    """Bitwise reruns; env i of a batch starting at env_offset k == env k+i of a full batch
    (a partially filled last wave must not disturb the others)."""
    def run(n, off):
        env = VecEnv(env_id, n, seed=21, env_offset=off, autoreset=True)
        assert env.info.lanes_per_env == 16
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand((30, 97, env.info.action_dim), device="cuda", generator=g) * 2 - 1
        return torch.stack([env.step(acts[t][off:off + n].contiguous()).obs.clone() for t in range(30)]).cpu().numpy()
    a = run(97, 0)
    np.testing.assert_array_equal(a, run(97, 0))
    np.testing.assert_array_equal(a[:, 41:], run(56, 41))


# ------------------------------------------------------------------ HumanoidFlagrun
def test_flagrun_redraws_match_oracle():
    """HumanoidFlagrun's flag bookkeeping (robot_locomotors.py:219-226) over 155 teacher-forced
    steps, past the 150-calc_state timeout: walk target, flag_timeout and the draw counter
    identical to the oracle's (same Philox stream), obs within the step tolerances."""
    n, steps, seed = 64, 155, 17
    env = VecEnv("HumanoidFlagrunPyBulletEnv-v0", n, seed=seed, autoreset=False)
    orc = oracle.OracleEnvs("HumanoidFlagrunPyBulletEnv-v0", n, nthreads=8, seed=seed)
    r = np.random.default_rng(2)
    env.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, 17)).astype(np.float32)))
    NF = env.info.n_feet
    errs, redraws = [], 0
    for t in range(steps):
        phys, aux = env.get_state()
        orc.state[:] = phys.cpu().numpy()
        orc.aux[:] = aux.cpu().numpy()
        before = orc.aux[:, 4 + NF + 3].copy()
        a = r.uniform(-1, 1, (n, 17)).astype(np.float32)
        og = env.step(torch.from_numpy(a).cuda()).obs.cpu().numpy()
        oo, _, _, _ = orc.step(a)
        _, aux2 = env.get_state()
        np.testing.assert_array_equal(aux2.cpu().numpy()[:, 4 + NF:], orc.aux[:, 4 + NF:])
        redraws += int((orc.aux[:, 4 + NF + 3] != before).sum())
        errs.append(np.abs(og - oo).max(axis=1))
    assert redraws >= n  # every env's flag timed out at least once
    e = np.concatenate(errs)
    assert np.median(e) <= 1e-4 and np.percentile(e, 99) <= 1e-2
