"""Float64 quad kernel vs float64 lane kernel, one step from the same states: max relative
difference per state word (dev diagnostic)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import pybulletgym_amd  # noqa
from pybulletgym_amd.vec_env import VecEnv

env_id = sys.argv[1] if len(sys.argv) > 1 else "AntPyBulletEnv-v0"
n = 64
for kw, tag in (({}, "quad"), ({"kernel": 2}, "gang"), ({"lds_rows": 0}, "quad_ws")):
    q = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, **kw)
    ln = VecEnv(env_id, n, seed=3, autoreset=False, precision=64, kernel=0)
    r = np.random.default_rng(7)
    q.reset(init_q=torch.from_numpy(r.uniform(-0.1, 0.1, (n, q.info.reset_dofs)).astype(np.float32)))
    for zero in (True, False):
        phys, aux = q.get_state()
        ln.set_state(phys, aux)
        a = torch.zeros((n, q.info.action_dim), device="cuda") if zero else \
            torch.from_numpy(r.uniform(-1, 1, (n, q.info.action_dim)).astype(np.float32)).cuda()
        q.step(a, want_contacts=True)
        ln.step(a, want_contacts=True)
        sq, sl = q.get_state()[0].cpu().numpy(), ln.get_state()[0].cpu().numpy()
        rel = (np.abs(sq - sl) / np.maximum(1.0, np.abs(sl))).max(axis=0)
        print(tag, "zero" if zero else "rand", "lanes", q.info.lanes_per_env, "lds_rows", q.info.lds_rows,
              "nc q/l", q.ncontact[:8].tolist(), ln.ncontact[:8].tolist())
        print("  per-word max rel:", np.array2string(rel, precision=1, max_line_width=200))
        print("  env0 q:", np.array2string(sq[0], precision=5, max_line_width=200))
        print("  env0 l:", np.array2string(sl[0], precision=5, max_line_width=200))
