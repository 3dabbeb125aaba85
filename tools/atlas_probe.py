"""Dev probe: one GPU env step vs the float64 oracle (and the float32 oracle) from the same
state, per kernel variant; prints the error medians / maxima and the worst columns."""
import sys, time, numpy as np, torch
sys.path.insert(0, '.')
from oracle import oracle
from pybulletgym_amd.vec_env import VecEnv, sample_actions
env_id = sys.argv[1] if len(sys.argv) > 1 else 'AtlasPyBulletEnv-v0'
n, steps = 64, 6
for opts in ({}, {"gang_dist": 0}, {"gang_dist": 1}, {"lds_rows": 0}):
    env = VecEnv(env_id, n, seed=3, autoreset=True, **opts, precision=32)
    env.reset(); torch.cuda.synchronize()
    acts = sample_actions(env.info.action_dim, n, steps, seed=3)
    orc = oracle.OracleEnvs(env_id, n, nthreads=8, seed=3)
    f32 = oracle.OracleEnvs(env_id, n, nthreads=8, seed=3, precision=32)
    for t in range(steps):
        phys, aux = env.get_state()
        orc.state[:] = phys.cpu().numpy(); orc.aux[:] = aux.cpu().numpy()
        f32.state[:] = orc.state; f32.aux[:] = orc.aux
        res = env.step(acts[t], want_reward64=True, want_contacts=True)
        oo, ro, do, co = orc.step(acts[t].cpu().numpy())
        of, _, _, _ = f32.step(acts[t].cpu().numpy())
        og = torch.where(res.done.bool()[:, None], res.terminal_obs, res.obs).cpu().numpy()
        err = np.abs(og - oo)
        e32 = np.abs(of - oo).max(1)
        nc = env.ncontact.cpu().numpy()
        nz = nc == 0
        print(opts, t, f"gpu med {np.median(err.max(1)):.2e} max {err.max():.2e} | no-contact envs med "
              f"{np.median(err.max(1)[nz]) if nz.any() else -1:.2e} | f32 med {np.median(e32):.2e} max {e32.max():.2e}"
              f" | nc match {(nc == co).mean():.2f} | worst cols {np.argsort(err.max(0))[-5:]}", flush=True)
    env.close()
