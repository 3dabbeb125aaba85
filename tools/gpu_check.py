"""Quick GPU-vs-oracle check (dev tool): teacher-forced one-step parity for each robot."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np, torch
import pybulletgym_amd
from pybulletgym_amd.vec_env import VecEnv
import oracle

robots = sys.argv[1:] or ["InvertedPendulumPyBulletEnv-v0", "HopperPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0", "AntPyBulletEnv-v0", "HumanoidPyBulletEnv-v0"]
for env_id in robots:
    n = 256
    env = VecEnv(env_id, n, seed=1, autoreset=False, precision=32)
    orc = oracle.OracleEnvs(env_id, n, nthreads=16)
    rng = np.random.default_rng(0)
    q0 = rng.uniform(-0.1, 0.1, (n, env.info.reset_dofs)).astype(np.float32)
    obs_g = env.reset(init_q=torch.from_numpy(q0)).cpu().numpy()
    obs_o = orc.reset(q0.astype(np.float64))
    ph, ax = env.get_state()
    print(env_id, "reset obs maxdiff %.3g state maxdiff %.3g aux %.3g" % (np.abs(obs_g-obs_o).max(), np.abs(ph.cpu().numpy()-orc.state).max(), np.abs(ax.cpu().numpy()-orc.aux).max()))
    worst = 0; dmis = 0; cmis = 0; rmax = 0
    for k in range(60):
        a = rng.uniform(-1, 1, (n, env.info.action_dim)).astype(np.float32)
        # teacher forcing: copy GPU state into oracle
        ph, ax = env.get_state()
        orc.state[:] = ph.cpu().numpy(); orc.aux[:] = ax.cpu().numpy()
        r = env.step(torch.from_numpy(a).cuda(), want_reward64=True, want_contacts=True)
        og, rg, dg, cg = r.obs.cpu().numpy(), env.reward64.cpu().numpy(), r.done.cpu().numpy().astype(bool), env.ncontact.cpu().numpy()
        oo, ro, do, co = orc.step(a)
        ph2, _ = env.get_state()
        sd = np.abs(ph2.cpu().numpy() - orc.state)
        worst = max(worst, np.nanmax(np.abs(og - oo))); rmax = max(rmax, np.nanmax(np.abs(rg - ro)))
        dmis += (dg != do).sum(); cmis += (cg != co).sum()
    print("   60 teacher-forced steps: obs maxdiff %.3g reward maxdiff %.3g done mismatches %d contact-count mismatches %d  last state maxdiff %.3g" % (worst, rmax, dmis, cmis, np.nanmax(sd)))
    # throughput
    N = 16384 if "Humanoid" not in env_id else 4096
    env2 = VecEnv(env_id, N, seed=2, autoreset=True, precision=32)
    env2.reset()
    acts = torch.rand((50, N, env2.info.action_dim), device="cuda") * 2 - 1
    for i in range(5): env2.step(acts[i])
    torch.cuda.synchronize(); t = time.time()
    for i in range(50): env2.step(acts[i])
    torch.cuda.synchronize(); dt = time.time() - t
    print("   N=%d: %.3f ms/step, %.3g env-steps/s" % (N, dt/50*1e3, N*50/dt))
