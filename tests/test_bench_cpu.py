"""bench.py on CPU: the N > 1 control flow (gloo process group, barriers, max over ranks, the
padded flat gather, one JSON line from rank 0) with the --dry-run-cpu stand-in env, and the
CPU-baseline leg (oracle with auto-reset, Philox actions) on a short sample."""
import json
import os
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def test_bench_two_rank_dry_run_cpu():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29651", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--preroll", "2", "--envs-per-gpu", "5",
           "--dry-run-cpu", "--legs", "HopperPyBulletEnv-v0:3"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["config"]["global_envs"] == 10
    assert d["scaling"] == "weak" and "dry_run" in d and d["allgather_step_bytes"] == 10 * (28 + 2) * 4
    assert d["hopper_f32"]["global_envs"] == 6


def test_cpu_baseline_leg_with_autoreset():
    sys.path.insert(0, REPO)
    import bench
    d = bench.cpu_baseline(seconds=1.0)
    assert d["value"] > 0 and d["kind"] == "port" and d["cores"] >= 1
    assert "auto-reset" in d["sample"]
