"""Contact-count histogram per env-step under random actions (dev tool: LDS capacity sizing)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pybulletgym_amd  # noqa: F401
from pybulletgym_amd.vec_env import VecEnv
for env_id, n in [(a, int(b)) for a, b in (x.split(":") for x in (sys.argv[1:] or ["HumanoidPyBulletEnv-v0:4096"]))]:
    env = VecEnv(env_id, n, seed=3, autoreset=True, precision=32)
    env.reset()
    h = torch.zeros(64, dtype=torch.int64, device="cuda")
    hw = torch.zeros(64, dtype=torch.int64, device="cuda")  # max over each wave's 16 envs (quad kernel)
    for i in range(200):
        env.step(torch.rand((n, env.info.action_dim), device="cuda") * 2 - 1, want_contacts=True)
        if i >= 50:
            h += torch.bincount(env.ncontact.clamp(max=63).long(), minlength=64)
            if n % 16 == 0:
                hw += torch.bincount(env.ncontact.view(-1, 16).amax(dim=1).clamp(max=63).long(), minlength=64)
    h = h.cpu().tolist()
    tot = sum(h)
    print(env_id, "contacts per env-step:", {k: round(v / tot, 3) for k, v in enumerate(h) if v}, flush=True)
    hw = hw.cpu().tolist()
    if sum(hw):
        print(env_id, "max contacts over 16-env waves:", {k: round(v / sum(hw), 3) for k, v in enumerate(hw) if v}, flush=True)
