"""Extract the pretrained roboschool policies' weights into ``tests/golden/policy_<robot>.npz``.
Runs HERE only (reads /root/reference).

The reference ships small reactive MLP policies for its envs as literal numpy arrays in
``pybulletgym/examples/roboschool-weights/enjoy_TF_<Env>_2017may.py`` (e.g. the Ant one:
``weights_dense1_w`` at :78, ``SmallReactivePolicy.act`` at :25-31:
relu(x W1 + b1) -> relu(. W2 + b2) -> . W3 + b3, actions unclipped).  SURVEY.md section 8f
item 1 uses them as a behavioural regression: a policy trained on pybullet physics only
walks if the simulator is close to pybullet's.

The files are parsed with ``ast`` -- the array literals are evaluated with
``ast.literal_eval``; nothing from the reference is imported or executed.  Only the
weights (data) are written.

Usage:  python tests/golden/make_policies.py
"""
from __future__ import annotations

import ast
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/pybulletgym/examples/roboschool-weights"
POLICIES = {
    "InvertedPendulumPyBulletEnv-v0": "enjoy_TF_InvertedPendulumPyBulletEnv_v0_2017may.py",
    "InvertedPendulumSwingupPyBulletEnv-v0": "enjoy_TF_InvertedPendulumSwingupPyBulletEnv_v0_2017may.py",
    "InvertedDoublePendulumPyBulletEnv-v0": "enjoy_TF_InvertedDoublePendulumPyBulletEnv_v0_2017may.py",
    "HopperPyBulletEnv-v0": "enjoy_TF_HopperPyBulletEnv_v0_2017may.py",
    "Walker2DPyBulletEnv-v0": "enjoy_TF_Walker2DPyBulletEnv_v0_2017may.py",
    "HalfCheetahPyBulletEnv-v0": "enjoy_TF_HalfCheetahPyBulletEnv_v0_2017may.py",
    "AntPyBulletEnv-v0": "enjoy_TF_AntPyBulletEnv_v0_2017may.py",
    "HumanoidPyBulletEnv-v0": "enjoy_TF_HumanoidPyBulletEnv_v0_2017may.py",
    "HumanoidFlagrunPyBulletEnv-v0": "enjoy_TF_HumanoidFlagrunPyBulletEnv_v0_2017may.py",
    "HumanoidFlagrunHarderPyBulletEnv-v0": "enjoy_TF_HumanoidFlagrunHarderPyBulletEnv_v0_2017may.py",
    "AtlasPyBulletEnv-v0": "enjoy_TF_AtlasPyBulletEnv_v0_2017jul.py",
}
NAMES = ["weights_dense1_w", "weights_dense1_b", "weights_dense2_w", "weights_dense2_b",
         "weights_final_w", "weights_final_b"]


def fixture_name(env_id: str) -> str:
    return "policy_" + env_id.split("PyBulletEnv")[0].lower() + ".npz"


def extract(path: str) -> dict:
    """Module-level ``weights_* = np.array(<literal>)`` assignments -> float32 arrays."""
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    out = {}
    for node in tree.body:
        if not (isinstance(node, ast.Assign) and len(node.targets) == 1
                and isinstance(node.targets[0], ast.Name) and node.targets[0].id in NAMES):
            continue
        call = node.value
        assert isinstance(call, ast.Call) and getattr(call.func, "attr", None) == "array", ast.dump(call)[:80]
        out[node.targets[0].id] = np.asarray(ast.literal_eval(call.args[0]), dtype=np.float32)
    missing = [n for n in NAMES if n not in out]
    assert not missing, (path, missing)
    return out


def main():
    for env_id, fname in POLICIES.items():
        w = extract(os.path.join(SRC, fname))
        dst = os.path.join(HERE, fixture_name(env_id))
        np.savez_compressed(dst, env_id=np.array(env_id), source=np.array(fname), **w)
        shapes = ", ".join(f"{k.split('_', 1)[1]} {tuple(v.shape)}" for k, v in w.items() if k.endswith("_w"))
        print(f"{env_id:40s} {shapes} -> {os.path.basename(dst)}")


if __name__ == "__main__":
    main()
