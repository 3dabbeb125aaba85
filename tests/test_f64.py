"""Reference-precision (float64) physics path: parity against the float64 oracle.

pybullet steps in double (btScalar; stepSimulation, /root/reference/pybulletgym/envs/roboschool/
scene_bases.py:75-76).  ``VecEnv(..., precision=64)`` (pbg_create_v2) keeps the physical state in
float64 and runs the same algorithm as the float32 kernels -- and as the oracle -- in float64
arithmetic, with the IEEE sqrt, reciprocals within 1 ulp of IEEE division (v_rcp_f64 + two Newton
steps, finite non-zero arguments; pbg_math.h) and the device library's sin / cos.  Against the float64
oracle the remaining differences are float64 rounding (summation orders, the kernels' inertia-
about-O formulation of M), so the bounds here are nine orders tighter than the float32 tests':

  * teacher-forced env steps, split like tests/test_gpu.py by discrete state (same contact-set
    signature and discrete reward terms) and reported by conditioning (probes at PROBE_REL64 =
    1e-12 relative; class B: the oracle's own spread above 1e-10).  Unlike the float32 tests,
    conditioning exempts nothing: EVERY env-step with the oracle's discrete state (classes A and
    B) must have the float64 STATE after the step (pbg_get_state) within STATE_REL64 = 1e-9
    relative of the oracle's in >= 99.9 % of the env-steps, with a hard maximum of 1e-6; the
    float64 reward within 1e-9; the float32 observation equal to the oracle's float32 observation
    up to one float32 rounding (2^-23 relative: both round float64 values that agree to ~1e-15);
    done flags and contact counts identical.  Class C (another contact set) at most 1 %.
    (First GPU run, r05b: every env id's largest state error 4.3e-12, class C empty.)
  * free running at the north-star horizon: from the same float64 reset state and the same 1,000
    action batches the float64 GPU leaves the float64 oracle's trajectory (obs error above 1e-4)
    far later than float32 arithmetic of the same algorithm does (the oracle's IEEE-float32
    instantiation): median first step at least F64_FREE_FACTOR x float32's.
"""
import os
import sys
import time

import numpy as np
import pytest
import torch

import oracle
import pybulletgym_amd  # noqa: F401
from pybulletgym_amd._native import PbgError
from pybulletgym_amd.vec_env import VecEnv, sample_actions
from test_gpu import ENVS, _discrete_terms, _first_exceed, _rel, _report

pytestmark = pytest.mark.gpu

ENVS64 = list(ENVS)  # every env id (Atlas on one-wave gang workgroups of 4 envs, round 5)
STATE_REL64 = 1e-9
HARD_MAX64 = 1e-6
SHARE64 = 0.999
OBS_ULP = 2.0 ** -23
PROBE_REL64, PROBE_ABS64, COND_EPS64 = 1e-12, 1e-14, 1e-10
LOOSE_FRAC64 = 0.01
F64_FREE_FACTOR = 2.0


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _state_rel(a, b):
    return (np.abs(a - b) / np.maximum(1.0, np.abs(b))).max(axis=1)


def _teacher_forced64(env_id, n, steps, sample=None, seed=3, name=None, sim=None, on_step=None, **opts):
    """The GPU float64 handle steps all n envs (auto-reset, Philox actions); before each step the
    sampled envs' float64 state records go to the oracle (and to N probes perturbed by 1e-12
    relative), which steps them; compared as in the module docstring.  on_step(t, env) sees every
    step's whole-batch outputs (tests/test_full_configs.py digests them)."""
    if sim is not None:
        sp = VecEnv.default_sim_params(env_id)
        sp.update(sim)
        oracle.set_sim_params(sp)
    try:
        env = VecEnv(env_id, n, seed=seed, autoreset=True, precision=64, sim_params=sim, **opts)
        assert env.precision == 64
        env.reset()
        idx = np.arange(n) if sample is None else np.linspace(0, n - 1, sample).astype(np.int64)
        tidx = torch.from_numpy(idx).cuda()
        th = min(16, os.cpu_count() or 1)
        orc = oracle.OracleEnvs(env_id, len(idx), nthreads=th, seed=seed)
        prb = [oracle.OracleEnvs(env_id, len(idx), nthreads=th, seed=seed) for _ in range(3)]
        pert = np.random.default_rng(seed)
        kind = "harder" if "Harder" in env_id else orc.info.kind
        acts = sample_actions(env.info.action_dim, n, steps, seed=seed)
        errA, rewA, obsA, spreadB = [], [], [], []
        nA = nB = nC = dmis = cmis = 0
        t0 = time.time()
        for t in range(steps):
            if t % 20 == 0:
                print(f"  f64 {name or env_id}: step {t}/{steps} {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
            phys, aux = env.get_state()
            orc.state[:] = phys.index_select(0, tidx).cpu().numpy()
            orc.aux[:] = aux.index_select(0, tidx).cpu().numpy()
            for p in prb:
                p.state[:] = orc.state + pert.uniform(-1, 1, orc.state.shape) * (PROBE_REL64 * np.abs(orc.state) + PROBE_ABS64)
                p.aux[:] = orc.aux
            res = env.step(acts[t], want_reward64=True, want_contacts=True, want_terms=True)
            if on_step is not None:
                on_step(t, env)
            done_g = res.done.bool()
            og = torch.where(done_g[:, None], res.terminal_obs, res.obs).index_select(0, tidx).cpu().numpy()
            dg = (done_g & ~res.truncated.bool()).index_select(0, tidx).cpu().numpy()
            rg = env.reward64.index_select(0, tidx).cpu().numpy()
            cg = env.ncontact.index_select(0, tidx).cpu().numpy()
            sg = env.contact_sig.index_select(0, tidx).cpu().numpy().view(np.uint32)
            tg = env.reward_terms.index_select(0, tidx).cpu().numpy()
            ph2, _ = env.get_state()
            sgpu = ph2.index_select(0, tidx).cpu().numpy()
            a = acts[t].index_select(0, tidx).cpu().numpy()
            oo, ro, do, co = orc.step(a)
            spread = np.zeros(len(idx))
            cond = np.ones(len(idx), bool)
            for p in prb:
                p.step(a)
                spread = np.maximum(spread, _state_rel(p.state, orc.state))
                cond &= p.csig == orc.csig
            cond &= spread <= COND_EPS64
            same = (sg == orc.csig) & (_discrete_terms(tg, kind) == _discrete_terms(orc.terms, kind)).all(axis=1)
            live = ~done_g.index_select(0, tidx).cpu().numpy()  # the GPU auto-reset the others' state
            A = same  # every env-step of the oracle's discrete state is held to the bound
            B = same & ~cond  # (reported: ill conditioned at 1e-12)
            nA += int((same & cond).sum())
            nB += int(B.sum())
            nC += int((~same).sum())
            serr = _state_rel(sgpu, orc.state)
            errA.append(serr[A & live])
            rewA.append(np.abs(rg - ro)[A] / np.maximum(1.0, np.abs(ro[A])))
            obsA.append(_rel(og, oo)[A])
            dmis += int((dg[A] != do[A]).sum())
            cmis += int((cg[A] != co[A]).sum())
            if (B & live).any():
                spreadB.append(serr[B & live] / np.maximum(spread[B & live], COND_EPS64))
        env.close()
    finally:
        if sim is not None:
            oracle.set_sim_params(None)
    n_all = nA + nB + nC
    eA = np.concatenate(errA) if errA else np.zeros(1)
    rA = np.concatenate(rewA) if rewA else np.zeros(1)
    oA = np.concatenate(obsA) if obsA else np.zeros(1)
    rB = np.concatenate(spreadB) if spreadB else np.zeros(1)
    rec = dict(test=name or f"f64_teacher_forced[{env_id},{n}x{steps}]", env_steps=n_all, classA_frac=nA / n_all,
               classB_frac=nB / n_all, classC_frac=nC / n_all,
               same_state_share_within_1e_9=float((eA <= STATE_REL64).mean()), same_state_max_rel=float(eA.max()),
               same_state_p50_rel=float(np.median(eA)), same_reward_max_rel=float(rA.max()),
               same_obs_max_rel=float(oA.max()), same_done_mismatch=dmis, same_contact_count_mismatch=cmis,
               classB_ratio_to_spread_p99=float(np.percentile(rB, 99)))
    _report(rec)
    assert nA + nB > 0
    assert rec["same_state_share_within_1e_9"] >= SHARE64 and rec["same_state_max_rel"] <= HARD_MAX64, rec
    assert float((rA <= STATE_REL64).mean()) >= SHARE64, rec
    assert rec["same_obs_max_rel"] <= 1.01 * OBS_ULP, rec
    assert dmis == 0 and cmis == 0, rec
    assert rec["classC_frac"] <= LOOSE_FRAC64, rec
    return rec


@pytest.mark.parametrize("env_id", ENVS64)
def test_f64_reset_matches_oracle(env_id):
    """Reset from the same float32 init_q: float64 state records equal to the oracle's to 1e-13,
    observations equal up to one float32 rounding."""
    n = 128
    env = VecEnv(env_id, n, seed=5, autoreset=False, precision=64)
    orc = oracle.OracleEnvs(env_id, n, seed=5)
    q0 = np.random.default_rng(0).uniform(-0.1, 0.1, (n, env.info.reset_dofs)).astype(np.float32)
    obs = env.reset(init_q=torch.from_numpy(q0)).cpu().numpy()
    obs_o = orc.reset(q0.astype(np.float64))
    assert _rel(obs, obs_o).max() <= 1.01 * OBS_ULP
    phys, aux = env.get_state()
    np.testing.assert_allclose(phys.cpu().numpy(), orc.state, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(aux.cpu().numpy(), orc.aux, rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("env_id", ENVS64)
def test_f64_step_teacher_forced_parity(env_id):
    """Every float64 env id, 256 envs x 60 teacher-forced steps (Atlas, whose oracle is slow:
    128 x 30, as its float32 test)."""
    if env_id == "AtlasPyBulletEnv-v0":
        _teacher_forced64(env_id, 128, 30)
    else:
        _teacher_forced64(env_id, 256, 60)


CONFIGS64 = [("InvertedPendulumPyBulletEnv-v0", 1024, None), ("HopperPyBulletEnv-v0", 4096, 512),
             ("AntPyBulletEnv-v0", 16384, 512), ("HalfCheetahPyBulletEnv-v0", 8192, 384),
             ("HumanoidPyBulletEnv-v0", 4096, 192)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("env_id,n,sample", CONFIGS64)
def test_f64_config_parity(env_id, n, sample):
    """The BASELINE.json per-GPU config sizes, 200 teacher-forced steps, an evenly spread sample."""
    _teacher_forced64(env_id, n, 200, sample=sample, seed=7, name=f"f64_config[{env_id},{n}x200]")


def test_f64_sim_params_teacher_forced():
    """A changed scene reaches the float64 kernels at float64 precision (SimPT<double>)."""
    _teacher_forced64("AntPyBulletEnv-v0", 128, 30, sim={"gravity": 4.9, "solver_iterations": 8},
                      name="f64_sim_params[Ant,g=4.9,it=8]")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("env_id,n,sample", [("AntPyBulletEnv-v0", 16384, 512), ("HumanoidPyBulletEnv-v0", 4096, 192)])
def test_f64_free_running_divergence_far_later_than_float32(env_id, n, sample, steps=1000):
    env = VecEnv(env_id, n, seed=17, autoreset=False, precision=64)
    env.reset()
    idx = np.linspace(0, n - 1, sample).astype(np.int64)
    tidx = torch.from_numpy(idx).cuda()
    th = min(16, os.cpu_count() or 1)
    phys, aux = env.get_state()
    orcs = {}
    for name, prec in (("f64", 64), ("f32", 32)):
        o = oracle.OracleEnvs(env_id, sample, nthreads=th, seed=17, precision=prec)
        o.state[:] = phys.index_select(0, tidx).cpu().numpy()  # the same float64 reset state
        o.aux[:] = aux.index_select(0, tidx).cpu().numpy()
        orcs[name] = o
    acts = sample_actions(env.info.action_dim, n, steps, seed=0xF4EE)
    err = {k: np.zeros((steps, sample)) for k in ("gpu", "f32")}
    t0 = time.time()
    for t in range(steps):
        if t % 100 == 0:
            print(f"  f64 free_running[{env_id}]: step {t}/{steps} {time.time() - t0:.0f}s", file=sys.stderr, flush=True)
        res = env.step(acts[t])
        og = res.obs.index_select(0, tidx).cpu().numpy()
        a = acts[t].index_select(0, tidx).cpu().numpy()
        o64, _, _, _ = orcs["f64"].step(a)
        o32, _, _, _ = orcs["f32"].step(a)
        err["gpu"][t] = _rel(og, o64)
        err["f32"][t] = _rel(o32, o64)
    env.close()
    rec = dict(test=f"f64_free_running[{env_id},{n},{sample}x{steps}]")
    first = {}
    for thr in (1e-4, 1e-2):
        for k in ("gpu", "f32"):
            f = _first_exceed(err[k], thr)
            first[(k, thr)] = f
            rec[f"{k}_first_above_{thr:g}_p10_p50_p90"] = [float(np.percentile(f, q)) for q in (10, 50, 90)]
            rec[f"{k}_never_above_{thr:g}_frac"] = float((f == steps).mean())
    _report(rec)
    for thr in (1e-4, 1e-2):
        g, f = np.median(first[("gpu", thr)]), np.median(first[("f32", thr)])
        assert g >= F64_FREE_FACTOR * f, (thr, g, f, rec)


def test_f64_determinism_and_env_offset_invariance():
    """Bitwise reruns and shard invariance of the float64 handle (the multi-GPU split)."""
    def run(n, off):
        env = VecEnv("HopperPyBulletEnv-v0", n, seed=21, env_offset=off, autoreset=True, precision=64)
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand((30, 64, 3), device="cuda", generator=g) * 2 - 1
        out = [env.step(acts[t][off:off + n].contiguous()).obs.clone() for t in range(30)]
        st = env.get_state()[0].cpu().numpy()
        return torch.stack(out).cpu().numpy(), st
    a, sa = run(64, 0)
    b, sb = run(64, 0)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(sa, sb)
    c, sc = run(32, 32)
    np.testing.assert_array_equal(a[:, 32:], c)
    np.testing.assert_array_equal(sa[32:], sc)


@pytest.mark.parametrize("env_id", ENVS64)
def test_f64_facade_default_is_float64_and_matches_oracle(env_id):
    """the reference-compatible surface (``make`` and the per-env gym classes,
    envs/__init__.py:59-84) steps the reference's double-precision physics by default
    (scene_bases.py:75-76).  One env through ``make(env_id)`` -- the TimeLimit wrapper, the env class,
    its one-env handle -- teacher-forced against the float64 oracle for 40 steps (Atlas 20): the
    float64 state after every step within STATE_REL64 = 1e-9 relative, the returned reward within
    1e-9, the observation within one float32 rounding, done identical."""
    from pybulletgym_amd import make
    env = make(env_id)
    assert env.unwrapped.precision == 64 and env.unwrapped._vec.precision == 64
    env.seed(7)
    env.reset()
    vec = env.unwrapped._vec
    assert vec.precision == 64
    orc = oracle.OracleEnvs(env_id, 1, seed=7)
    rng = np.random.default_rng(7)
    errs = []
    for t in range(20 if env_id == "AtlasPyBulletEnv-v0" else 40):
        phys, aux = vec.get_state()
        orc.state[:] = phys.cpu().numpy()
        orc.aux[:] = aux.cpu().numpy()
        a = rng.uniform(-1, 1, env.action_space.shape).astype(np.float32)
        o, r, d, info = env.step(a)
        oo, ro, do, _ = orc.step(a[None])
        errs.append(float(_state_rel(vec.get_state()[0].cpu().numpy(), orc.state)[0]))
        assert abs(r - ro[0]) <= STATE_REL64 * max(1.0, abs(ro[0])), (t, r, ro[0])
        assert _rel(np.asarray(o, np.float32)[None], oo).max() <= 1.01 * OBS_ULP, t
        assert d == bool(do[0]), t
        if d:
            break
    _report(dict(test=f"f64_facade[{env_id}]", steps=len(errs), state_max_rel=max(errs)))
    assert max(errs) <= STATE_REL64, errs
    env.close()
    f32 = make(env_id, precision=32)
    assert f32.unwrapped._vec.precision == 32
    f32.close()


@pytest.mark.parametrize("precision", [64, 32])
def test_f64_atlas_lane_kernel_is_refused(precision):
    """Atlas has no lane kernel (886 contact slots) in either precision: kernel=0 is refused with
    PBG_E_ARG (-1), never a silent run of the gang kernel; gang_lanes = 32 on a robot
    without 32-lane gangs is PBG_E_ARG at float64 as at float32."""
    with pytest.raises(PbgError, match=r"failed \(-1\).*kernel = 0"):
        VecEnv("AtlasPyBulletEnv-v0", 4, precision=precision, kernel=0)
    with pytest.raises(PbgError, match=r"failed \(-1\).*gang_lanes = 32"):
        VecEnv("HopperPyBulletEnv-v0", 4, precision=precision, gang_lanes=32)


def test_f64_replicated_dynamics_only_under_8_dofs():
    """The float64 replicated-dynamics gang variant exists for robots under 8 dofs (Hopper); the
    float64 HalfCheetah has none (it would spill 1.3 KB): gang_dist = 0 is PBG_E_ARG there, and
    Hopper honours both variants."""
    with pytest.raises(PbgError, match=r"failed \(-1\).*replicated-dynamics"):
        VecEnv("HalfCheetahPyBulletEnv-v0", 64, precision=64, gang_dist=0)
    for d in (0, 1):
        VecEnv("HopperPyBulletEnv-v0", 64, precision=64, gang_dist=d).close()


# ------------------------------------------------------------------ float64 kernel variants
# The float64 walkers run the kernels of the float32 path instantiated on F64<R>: Ant the quad
# kernel (pbg_team.hip, 4 lanes per env; AntMuJoCo too), the Humanoid family 32-lane gangs, the
# other walkers the 16-lane gang kernel (pbg_gang.hip; kernel=2 puts Ant on it too, gang_lanes=16
# the Humanoids); kernel=0 selects the float64 lane-per-env kernel, which stays the
# pendulums' path and the quad / gang kernels' cross-check.
@pytest.mark.parametrize("env_id", ["AntPyBulletEnv-v0", "HumanoidPyBulletEnv-v0", "HopperPyBulletEnv-v0",
                                    "HumanoidFlagrunHarderPyBulletEnv-v0", "HalfCheetahMuJoCoEnv-v0"])
def test_f64_lane_kernel_teacher_forced(env_id):
    """The float64 lane kernel against the float64 oracle, same bounds."""
    _teacher_forced64(env_id, 128, 40, name=f"f64_lane[{env_id}]", kernel=0)


@pytest.mark.parametrize("env_id,kernel,lanes", [
    ("AntPyBulletEnv-v0", None, 4), ("AntMuJoCoEnv-v0", None, 4), ("AntPyBulletEnv-v0", 2, 16),
    ("HumanoidPyBulletEnv-v0", "g16", 16), ("HumanoidFlagrunHarderPyBulletEnv-v0", "g16", 16),
    ("HumanoidPyBulletEnv-v0", None, 32), ("HalfCheetahPyBulletEnv-v0", None, 16), ("Walker2DPyBulletEnv-v0", None, 16),
    ("HopperPyBulletEnv-v0", None, 16), ("HopperPyBulletEnv-v0", "dist", 16), ("HopperMuJoCoEnv-v0", None, 16),
    ("HumanoidFlagrunPyBulletEnv-v0", None, 32),
    ("HumanoidFlagrunHarderPyBulletEnv-v0", None, 32), ("HumanoidMuJoCoEnv-v0", None, 32),
    ("HalfCheetahMuJoCoEnv-v0", None, 16)])  # restitution + torsional rows (tests/test_contact_material.py)
def test_f64_quad_and_gang_match_f64_lane(env_id, kernel, lanes):
    """Float64 quad / gang vs float64 lane kernel from the same states every step: the same contact
    sets and the state within 1e-9 (different summation orders in float64).  The float64 Hopper runs
    the replicated-dynamics gang variant by default (round 6); "dist" forces its distributed one."""
    n = 256
    kw = {} if kernel is None else ({"gang_lanes": 16} if kernel == "g16" else
                                    ({"gang_dist": 1} if kernel == "dist" else {"kernel": kernel}))
    g = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, **kw)
    ln = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, kernel=0)
    assert g.info.lanes_per_env == lanes and ln.info.lanes_per_env == 1
    r = np.random.default_rng(7)
    g.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, g.info.reset_dofs)).astype(np.float32)))
    errs, same_n = [], 0
    for t in range(30):
        phys, aux = g.get_state()
        ln.set_state(phys, aux)
        a = torch.from_numpy(r.uniform(-1, 1, (n, g.info.action_dim)).astype(np.float32)).cuda()
        g.step(a, want_contacts=True)
        ln.step(a, want_contacts=True)
        same = (g.contact_sig == ln.contact_sig).cpu().numpy()
        sg, sl = g.get_state()[0].cpu().numpy(), ln.get_state()[0].cpu().numpy()
        errs.append(_state_rel(sg, sl)[same])
        same_n += int(same.sum())
        np.testing.assert_array_equal(g.ncontact.cpu().numpy()[same], ln.ncontact.cpu().numpy()[same])
    e = np.concatenate(errs)
    rec = dict(test=f"f64_{'quad' if lanes == 4 else ('gang32' if lanes == 32 else 'gang')}_vs_lane[{env_id}]", same_frac=same_n / (30 * n), max_rel=float(e.max()),
               share_within_1e_9=float((e <= STATE_REL64).mean()))
    _report(rec)
    assert rec["same_frac"] >= 1 - LOOSE_FRAC64 and rec["share_within_1e_9"] >= SHARE64 and rec["max_rel"] <= HARD_MAX64, rec


def test_f64_quad_workspace_rows_bitwise_equal_lds_rows():
    """Float64 quad (Ant): contact rows past the LDS capacity (lds_rows=0: every row in the device
    workspace) change no bit; the default plan keeps rows in LDS."""
    def run(**kw):
        e = VecEnv("AntPyBulletEnv-v0", 256, seed=13, autoreset=True, precision=64, **kw)
        assert e.info.lanes_per_env == 4
        e.reset()
        gen = torch.Generator(device="cuda").manual_seed(6)
        out, nc = [], []
        for _ in range(40):
            e.step(torch.rand((256, 8), device="cuda", generator=gen) * 2 - 1, want_contacts=True)
            out.append(e.get_state()[0].clone())
            nc.append(e.ncontact.clone())
        return torch.stack(out).cpu().numpy(), torch.stack(nc).cpu().numpy(), e.info.lds_rows
    a, ca, cap = run()
    b, cb, cap0 = run(lds_rows=0)
    assert ca.max() > 0 and cap > 0 and cap0 == 0
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))


@pytest.mark.parametrize("env_id", ["HumanoidPyBulletEnv-v0", "HalfCheetahMuJoCoEnv-v0"])
def test_f64_gang_workspace_contacts_bitwise_equal_lds_contacts(env_id):
    """Float64 gang contacts past the LDS capacity (lds_rows=0: all in the device workspace) change
    no bit (Humanoid: floor + self contacts; HalfCheetahMuJoCo: six rows per contact)."""
    def run(**kw):
        e = VecEnv(env_id, 128, seed=11, autoreset=True, precision=64, **kw)
        e.reset()
        gen = torch.Generator(device="cuda").manual_seed(5)
        out, nc = [], []
        for _ in range(40):
            e.step(torch.rand((128, e.info.action_dim), device="cuda", generator=gen) * 2 - 1, want_contacts=True)
            out.append(e.get_state()[0].clone())
            nc.append(e.ncontact.clone())
        return torch.stack(out).cpu().numpy(), torch.stack(nc).cpu().numpy()
    a, ca = run()
    b, cb = run(lds_rows=0)
    assert ca.max() > 0
    np.testing.assert_array_equal(ca, cb)
    np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64))


def test_f64_gang_determinism_and_offset_invariance():
    def run(n, off):
        env = VecEnv("HumanoidPyBulletEnv-v0", n, seed=21, env_offset=off, autoreset=True, precision=64)
        assert env.info.lanes_per_env == 32
        env.reset()
        g = torch.Generator(device="cuda").manual_seed(0)
        acts = torch.rand((30, 97, 17), device="cuda", generator=g) * 2 - 1
        out = [env.step(acts[t][off:off + n].contiguous()).obs.clone() for t in range(30)]
        return torch.stack(out).cpu().numpy(), env.get_state()[0].cpu().numpy()
    a, sa = run(97, 0)
    b, sb = run(97, 0)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(sa, sb)
    c, sc = run(56, 41)
    np.testing.assert_array_equal(a[:, 41:], c)
    np.testing.assert_array_equal(sa[41:], sc)


def test_f64_checkpoint_round_trip_bitwise_and_precision_guard():
    """A float64 handle's state_dict restores bit for bit across auto-resets (the float64 state
    record is the state itself), and a float64 checkpoint is refused by a float32 handle (its
    state would be rounded) and vice versa."""
    n = 64
    a = VecEnv("AntPyBulletEnv-v0", n, seed=9, autoreset=True, precision=64)
    a.reset()
    gen = torch.Generator(device="cuda").manual_seed(3)
    acts = torch.rand((60, n, 8), device="cuda", generator=gen) * 2 - 1
    for t in range(20):
        a.step(acts[t])
    sd = a.state_dict()
    assert sd["precision"] == 64
    b = VecEnv("AntPyBulletEnv-v0", n, seed=9, autoreset=True, precision=64)
    b.load_state_dict(sd)
    for t in range(20, 60):
        ra, rb = a.step(acts[t]), b.step(acts[t])
        np.testing.assert_array_equal(ra.obs.cpu().numpy().view(np.uint32), rb.obs.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(a.get_state()[0].cpu().numpy().view(np.uint64),
                                  b.get_state()[0].cpu().numpy().view(np.uint64))
    f32 = VecEnv("AntPyBulletEnv-v0", n, seed=9, autoreset=True, precision=32)
    with pytest.raises(PbgError):
        f32.load_state_dict(sd)
    with pytest.raises(PbgError):
        b.load_state_dict(f32.state_dict())
