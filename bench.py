"""Headline benchmark: random-action rollout env-steps/s on AntPyBulletEnv-v0.

BASELINE.json metric: "env steps/sec (whole node) at N parallel envs, Ant + Humanoid,
1/2/4/8 MI355X"; the single-GPU workload is config[2], AntPyBulletEnv-v0 at 16,384
envs per GPU (weak scaling: each rank owns 16,384 envs, no per-step collective).

One "step" = one batched env step of every env on every GPU: apply_action, 4 physics
sub-steps (Featherstone dynamics, contacts, 5-sweep PGS, integration), the
observation/reward/done pack, TimeLimit + auto-reset -- one kernel launch per GPU.
Actions are pre-generated U(-1, 1) float32 tensors already resident in HBM.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env steps/sec (whole node) at N parallel envs, Ant + Humanoid, 1/2/4/8 MI355X"  # BASELINE.json
ENV_ID = "AntPyBulletEnv-v0"
ENVS_PER_GPU = 16384
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SHORT = {"InvertedPendulumPyBulletEnv-v0": "pendulum", "HopperPyBulletEnv-v0": "hopper",
         "HalfCheetahPyBulletEnv-v0": "halfcheetah", "AntPyBulletEnv-v0": "ant",
         "HumanoidPyBulletEnv-v0": "humanoid", "Walker2DPyBulletEnv-v0": "walker2d"}


def alg_bytes_per_env_step(info):
    """Minimum HBM bytes per env-step (BASELINE.md section 4 / SURVEY.md 8d): 4 * (2S + n + D + 2),
    S = 13 (floating base) + 2 * joint dofs + 6 per-env scalars; Ant: S = 35 -> 432 B."""
    S = 13 * int(info.floating) + 2 * info.n_joints + 6
    return 4 * (2 * S + info.action_dim + info.obs_dim + 2)


def cpu_baseline(seconds=12.0):
    """The CPU oracle (float64 restatement of the same step) on the host's cores, on a
    bounded sample: 4,096 Ant envs stepped until ~`seconds` of wall time."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = 4096
    e = oracle.OracleEnvs(ENV_ID, n, nthreads=threads)
    rng = np.random.default_rng(0)
    e.reset(rng.uniform(-0.1, 0.1, (n, e.info.NR)))
    acts = rng.uniform(-1, 1, (8, n, e.info.NA)).astype(np.float32)
    e.step(acts[0])
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        e.step(acts[steps % 8])
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pbg_oracle.cpp (float64) on {n} Ant envs x {steps} steps, "
                      f"{threads} OpenMP threads, {dt:.1f} s; no auto-reset"}


def load_pmc(env_id, n):
    """PMC summary of the step kernel (profiles/pmc_step_<robot>.json, written by
    tools/pmc_summary.py from the committed rocprofv3 --pmc passes), if it was taken at
    this env count."""
    path = os.path.join(REPO, "profiles", f"pmc_step_{SHORT.get(env_id, env_id)}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    d["_path"] = path
    return d if d.get("envs") == n else None


def valu_roofline(pmc, kernel_ms, n):
    """VALU issue roofline (the binding one): wave64 VALU instructions per
    launch (PMC SQ_INSTS_VALU) / the kernel's HIP-event time, against the chip's issue
    peak: 256 CUs x 4 SIMDs x one wave64 VALU op per 2 cycles at 2.4 GHz."""
    peak = 256 * 4 * 2.4e9 / 2 / 1e12
    ach = pmc["valu_insts_per_launch"] / (kernel_ms * 1e-3) / 1e12
    return {"achieved": ach, "peak": peak, "unit": "T wave-instr/s", "frac": ach / peak,
            "valu_instr_per_env": pmc["valu_insts_per_launch"] * 64 / n,
            "source": "profiles/" + os.path.basename(pmc.get("_path", "pmc"))}


def occupancy(env):
    """Step-kernel occupancy (Humanoid row): lanes per env, workgroup, LDS per
    workgroup, registers per lane; waves per SIMD = min(register limit, LDS limit, waves the
    env count provides / (256 CUs x 4 SIMDs))."""
    i = env.info
    waves = -(-env.num_envs * i.lanes_per_env // 64)
    reg_limit = 512 // max(8 * -(-i.vgprs // 8), 1) if i.vgprs > 0 else 8
    wgs_per_cu = (160 * 1024) // i.lds_bytes if i.lds_bytes > 0 else 32
    lds_limit = max(1, wgs_per_cu * max(i.block // 64, 1) // 4)
    return {"lanes_per_env": i.lanes_per_env, "block": i.block, "lds_bytes_per_workgroup": i.lds_bytes,
            "vgprs": i.vgprs, "scratch_bytes": i.scratch_bytes, "lds_rows": i.lds_rows,
            "waves_per_simd": min(reg_limit, lds_limit, max(1, waves // 1024))}


def kernel_name(env):
    lpe = env.info.lanes_per_env
    k = {1: "pbg::step_kernel", 4: "pbg::team_step_kernel", 16: "pbg::gang_step_kernel"}.get(lpe, "pbg::step_kernel")
    return f"{k}<{env.env_id}>"


def timed_rollout(VecEnv, env_id, n, steps, warmup, dev, rank, world, no_graph):
    """Random-action rollout of n envs on this GPU: warmup steps, per-launch kernel time
    (HIP events on the launch stream), then exactly `steps` steps bracketed by a barrier +
    device sync on both sides; returns (env, elapsed_s max over ranks, kernel_ms, G)."""
    import torch
    import torch.distributed as dist
    env = VecEnv(env_id, n, device=dev, seed=0x5EED, env_offset=rank * n, autoreset=True)
    env.reset()
    na = env.info.action_dim
    total = warmup + steps
    pool = min(total, 256)  # distinct pre-generated action batches, cycled
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    acts = torch.rand((pool, n, na), device=dev, generator=g, dtype=torch.float32) * 2 - 1

    for i in range(warmup):
        env.step(acts[i % pool])
    stream = torch.cuda.current_stream(dev)
    # timed region: the K steps as HIP-graph replays of G captured steps (G divides K)
    G = 1
    if not no_graph:
        G = max(d for d in range(1, min(64, steps) + 1) if steps % d == 0)
        graph = env.capture([acts[j % pool] for j in range(G)])
    # per-launch kernel time (roofline.kernel_ms): HIP events on the launch stream around the
    # timed region itself (graph replays are back-to-back kernels), so it describes the same
    # launches as `value`; with --no-graph, events around each single launch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)] \
        if no_graph else None
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record(stream)
    if no_graph:
        for i in range(steps):
            ev[i][0].record(stream)
            env.step(acts[(warmup + i) % pool])
            ev[i][1].record(stream)
    else:
        for _ in range(steps // G):
            graph.replay()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = (sum(a.elapsed_time(b) for a, b in ev) if no_graph else e0.elapsed_time(e1)) / steps
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
    return env, elapsed, kernel_ms, G


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--envs-per-gpu", type=int, default=ENVS_PER_GPU)
    ap.add_argument("--env", default=ENV_ID)
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip timing the RCCL obs all-gather (timed separately, outside `value`)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch every step from the host (no HIP graph)")
    ap.add_argument("--second-env", default="HumanoidPyBulletEnv-v0", help="second workload of the metric ('none' = off)")
    ap.add_argument("--second-envs-per-gpu", type=int, default=4096)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import pybulletgym_amd  # noqa: F401
    from pybulletgym_amd.distributed import gather_flat
    from pybulletgym_amd.vec_env import VecEnv

    n = args.envs_per_gpu
    env, elapsed, kernel_ms, G = timed_rollout(VecEnv, args.env, n, args.steps, args.warmup, dev, rank, world,
                                               args.no_graph)
    second = None
    if args.second_env not in ("", "none") and args.second_env != args.env:
        # BASELINE metric names Ant + Humanoid: the Humanoid config (32,768 envs on 8 GPUs =
        # 4,096 per GPU, BASELINE.json configs[4]) timed the same way, reported beside `value`
        n2 = args.second_envs_per_gpu
        steps2 = max(1, min(args.steps, 200))
        env2, el2, km2, G2 = timed_rollout(VecEnv, args.second_env, n2, steps2, min(args.warmup, 20), dev, rank,
                                           world, args.no_graph)
        second = {"env": args.second_env, "envs_per_gpu": n2, "global_envs": world * n2, "steps": steps2,
                  "value": world * n2 * steps2 / el2, "unit": "env-steps/s", "ms_per_step": el2 / steps2 * 1e3,
                  "kernel": kernel_name(env2), "kernel_ms": km2, "lanes_per_env": env2.info.lanes_per_env,
                  "occupancy": occupancy(env2),
                  "obs_finite": bool(torch.isfinite(env2.obs).all())}
        alg2 = alg_bytes_per_env_step(env2.info)
        ach2 = alg2 * n2 / (km2 * 1e-3) / 1e9
        pmc2 = load_pmc(args.second_env, n2)
        second["roofline"] = {"bound": "hbm", "achieved": ach2, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": ach2 / HBM_PEAK_GBS, "traffic": pmc2.get("hbm_bytes_per_launch") if pmc2 else None,
                              "alg_bytes_per_env_step": alg2}
        if pmc2 and pmc2.get("valu_insts_per_launch"):
            second["valu_roofline"] = valu_roofline(pmc2, km2, n2)
        env2.close()

    gather_ms = None
    if not args.no_gather and world > 1:
        for _ in range(3):
            gather_flat(env.obs)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(20):
            gather_flat(env.obs)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - t1) / 20 * 1e3

    finite = bool(torch.isfinite(env.obs).all())
    if rank == 0:
        steps_total = world * n * args.steps
        value = steps_total / elapsed
        alg = alg_bytes_per_env_step(env.info)
        achieved = alg * n / (kernel_ms * 1e-3) / 1e9
        pmc = load_pmc(args.env, n)
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: U(-1,1) float32 actions pre-generated in HBM; robot compiled from the reference MJCF",
            "config": {"workload": f"{args.env} random-action rollout, auto-reset (TimeLimit 1000)",
                       "envs_per_gpu": n, "global_envs": world * n, "substeps": env.info.substeps,
                       "solver_iterations": 5, "parallelism": f"env-sharded x{world}, no per-step collective",
                       "launch": "host loop" if args.no_graph else f"hipGraph replay of {G} captured steps",
                       "lanes_per_env": env.info.lanes_per_env},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": kernel_name(env), "kernel_ms": kernel_ms,
                         "alg_bytes_per_env_step": alg},
            "obs_finite": finite,
            "occupancy": occupancy(env),
        }
        if pmc and pmc.get("valu_insts_per_launch"):
            out["valu_roofline"] = valu_roofline(pmc, kernel_ms, n)
        if second is not None:
            out["humanoid" if "Humanoid" in second["env"] else "second"] = second
        if gather_ms is not None:
            # the learner's optional flat batch: one all_gather_into_tensor of
            # [envs_per_gpu, obs_dim] float32 per rank over RCCL, timed after the rollout
            out["allgather_obs_ms"] = gather_ms
            out["allgather_obs_bytes"] = world * n * env.info.obs_dim * 4
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
