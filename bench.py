"""Headline benchmark: random-action rollout env-steps/s on AntPyBulletEnv-v0, float64 physics.

BASELINE.json metric: "env steps/sec (whole node) at N parallel envs, Ant + Humanoid,
1/2/4/8 MI355X"; the single-GPU workload is config[2], AntPyBulletEnv-v0 at 16,384
envs per GPU (weak scaling: each rank owns 16,384 envs, no per-step collective).

One "step" = one batched env step of every env on every GPU: apply_action, 4 physics
sub-steps (Featherstone dynamics, contacts, 5-sweep PGS, integration), the
observation/reward/done pack, TimeLimit + auto-reset -- one kernel launch per GPU.

Precision: the headline handle computes its physics in float64, as the reference does (pybullet's
btScalar is double; VERDICT r4 item 2: the reference-precision path is the credited headline).
The float32 handles -- the same kernels instantiated on float, about 1.7x faster for Ant -- are
timed beside it as labelled fast-mode legs (`*_f32`); --precision 32 makes float32 the headline.

Protocol: actions U(-1, 1) from Philox4x32-10 keyed by 0x5EED, counter
(step, global env) -- pbg_sample_actions, generated into HBM before the timed region, one
distinct batch per step; an untimed pre-roll (--preroll, 200 steps) ages the episodes past
their first steps so the timed window sees steady-state contact counts and auto-resets, then
W warm-up steps, then EXACTLY K timed steps (one HIP graph of the K launches) bracketed by a
barrier + device sync on both sides, max over ranks.  The timed windows (--windows, default 5;
value = the median window) replay the same captured graphs, i.e. the same K action batches;
the env state moves on between windows, so every window steps different states.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
  python -m torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2 --dry-run-cpu
      (CI: the N > 1 control flow -- gloo process group, barriers, max over ranks, the flat
       gather, the JSON line -- on CPU with a no-physics stand-in env; value meaningless)
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
ACTION_SEED = 0x5EED
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (non-matrix) peak
FP64_PEAK_TFLOPS = 78.6  # MI355X spec sheet: FP64 vector peak (the guide lists no FP64 figure)
SHORT = {"InvertedPendulumPyBulletEnv-v0": "pendulum", "HopperPyBulletEnv-v0": "hopper",
         "HalfCheetahPyBulletEnv-v0": "halfcheetah", "AntPyBulletEnv-v0": "ant",
         "HumanoidPyBulletEnv-v0": "humanoid", "Walker2DPyBulletEnv-v0": "walker2d"}
# BASELINE.json configs timed beside the headline (per-GPU env counts); a third field 64 = the
# reference-precision (float64 physics) handle of that config
EXTRA_LEGS = ("AntPyBulletEnv-v0:16384:32,HumanoidPyBulletEnv-v0:4096:64,HumanoidPyBulletEnv-v0:4096:32,"
              "HopperPyBulletEnv-v0:4096:64,HopperPyBulletEnv-v0:4096:32,"
              "HalfCheetahPyBulletEnv-v0:8192:64,HalfCheetahPyBulletEnv-v0:8192:32")


def alg_bytes_per_env_step(info, precision=32):
    """Minimum HBM bytes per env-step (BASELINE.md section 4 / SURVEY.md 8d): 4 * (2S + n + D + 2),
    S = 13 (floating base) + 2 * joint dofs + 6 per-env scalars; Ant: S = 35 -> 432 B.  The float64
    handle reads and writes its state in 8-byte words: 8 * 2S + 4 * (n + D + 2) (Ant 712 B)."""
    S = 13 * int(info.floating) + 2 * info.n_joints + 6
    if precision == 64:
        return 8 * 2 * S + 4 * (info.action_dim + info.obs_dim + 2)
    return 4 * (2 * S + info.action_dim + info.obs_dim + 2)


def host_threads():
    """Threads for the CPU leg: the CPUs this process may run on (sched_getaffinity), capped by
    OMP_NUM_THREADS when the launcher sets it (the GPU box sets it to its CPU share, 16)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(avail, omp) if omp > 0 else avail), avail


def _oracle_rollout(n, threads, seconds, chunk=64):
    """Step n Ant envs on the CPU oracle with `threads` OpenMP threads for ~`seconds` of timed
    work.  Every step gets its own Philox 0x5EED action batch (counter = step, env) and every
    auto-reset its own reset-noise draw (counter = env, episode), both generated in chunks
    outside the timed intervals; the oracle's step and masked reset are timed."""
    import numpy as np
    import oracle
    from pybulletgym_amd import rng
    e = oracle.OracleEnvs(ENV_ID, n, nthreads=threads, seed=ACTION_SEED)
    ids = np.arange(n)
    epi = np.zeros(n, np.int64)
    obs = e.reset(rng.reset_noise(ACTION_SEED, ids, 0, e.info.NR).astype(np.float64))
    steps = resets = 0
    timed = 0.0
    while timed < seconds:
        acts = rng.sample_actions(e.info.NA, ids, np.arange(steps, steps + chunk), seed=ACTION_SEED)
        for a in acts:
            t0 = time.perf_counter()
            obs, _, done, _ = e.step(a)
            timed += time.perf_counter() - t0
            steps += 1
            finished = done | (e.aux[:, 2] >= 1000)
            if finished.any():
                fin = np.flatnonzero(finished)
                epi[fin] += 1
                q = np.zeros((n, e.info.NR))
                q[fin] = rng.reset_noise(ACTION_SEED, fin, epi[fin], e.info.NR)
                t0 = time.perf_counter()
                e.reset(q, mask=finished, obs=obs)
                timed += time.perf_counter() - t0
                resets += len(fin)
            if timed >= seconds:
                break
    return steps, resets, timed


def cpu_baseline(seconds=12.0, single_core_seconds=3.0):
    """The CPU oracle (float64 restatement of the same step, OpenMP over envs) on the host's
    cores, on a bounded sample of the same workload: 4,096 Ant envs, distinct Philox 0x5EED
    actions per step, auto-reset on done or after 1,000 steps, ~`seconds` of timed stepping.
    Threads: the CPUs this job may use (OMP_NUM_THREADS caps sched_getaffinity; the GPU box
    grants one GPU job 16).  A short single-thread run gives the per-core rate, and the
    all-CPU figure is that rate times the CPUs in sched_getaffinity (an extrapolation that
    assumes linear scaling over envs, which the envs' independence allows; stated as such)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pybulletgym_amd  # noqa: F401
    threads, avail = host_threads()
    n = 4096
    steps, resets, dt = _oracle_rollout(n, threads, seconds)
    s1, _, dt1 = _oracle_rollout(512, 1, single_core_seconds)
    per_core = 512 * s1 / dt1
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "per_core_value": per_core, "affinity_cpus": avail,
            "extrapolated_all_affinity_cpus": per_core * avail,
            "sample": f"oracle/pbg_oracle.cpp (float64) on {n} Ant envs x {steps} steps with auto-reset "
                      f"({resets} resets), distinct Philox actions per step, {threads} OpenMP threads of {avail} "
                      f"CPUs in sched_getaffinity (OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}), "
                      f"{dt:.1f} s timed; per-core rate from 512 envs x {s1} steps on 1 thread ({dt1:.1f} s); "
                      f"extrapolated_all_affinity_cpus = per_core_value x {avail} (linear-scaling assumption, "
                      f"not measured)"}


# Roofline inputs shipped with the package (they travel to the GPU box with the code):
# the counted flops per env-step (tools/count_flops.py) and the PMC summaries of the step
# kernels (tools/pmc_summary.py, tagged with the round of the profile they come from; the raw
# rocprofv3 CSVs are under profiles/ with the same round prefix).
PERF = os.path.join(REPO, "pybullet-gym_amd", "perf")


def load_pmc(env_id, n, precision=32):
    """PMC summary of the step kernel (pybullet-gym_amd/perf/pmc_step_<robot>[_f64].json), if it
    was taken at this env count."""
    f64 = "_f64" if precision == 64 else ""
    path = os.path.join(PERF, f"pmc_step_{SHORT.get(env_id, env_id)}{f64}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    d["_path"] = path
    return d if d.get("envs") == n else None


def load_flops():
    """Counted FP32 flops per env-step per robot (pybullet-gym_amd/perf/flops_per_env_step.json,
    written by tools/count_flops.py from the op-counting build of the oracle; copy in profiles/)."""
    try:
        with open(os.path.join(PERF, "flops_per_env_step.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def valu_roofline(pmc, kernel_ms, n):
    """VALU issue roofline: wave64 VALU instructions per launch (PMC SQ_INSTS_VALU) / the
    kernel's HIP-event time, against the chip's issue peak: 256 CUs x 4 SIMDs x one wave64
    VALU op per 2 cycles at 2.4 GHz."""
    peak = 256 * 4 * 2.4e9 / 2 / 1e12
    ach = pmc["valu_insts_per_launch"] / (kernel_ms * 1e-3) / 1e12
    return {"achieved": ach, "peak": peak, "unit": "T wave-instr/s", "frac": ach / peak,
            "valu_instr_per_env": pmc["valu_insts_per_launch"] * 64 / n,
            "source": "pybullet-gym_amd/perf/" + os.path.basename(pmc.get("_path", "pmc")) + f" (round {pmc.get('round')})"}


def occupancy(env):
    """Step-kernel occupancy: lanes per env, workgroup, LDS per workgroup, registers per lane;
    waves per SIMD = min(register limit, LDS limit, waves the env count provides / 1024 SIMDs)."""
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
    k = {1: "pbg::step_kernel", 4: "pbg::team_step_kernel", 16: "pbg::gang_step_kernel",
         32: "pbg::gang_step_kernel"}.get(lpe, "pbg::step_kernel")
    f64 = getattr(env, "precision", 32) == 64
    return f"{k}<{'F64<' if f64 else ''}{env.env_id}{'>' if f64 else ''}>"


class DryRunEnv:
    """--dry-run-cpu stand-in: VecEnv's buffers and call shape, no physics (CI of the N > 1
    control flow only)."""

    def __init__(self, env_id, n, device, seed, env_offset, autoreset):
        import torch

        class _I:  # pbg_info_t fields bench reads
            floating, n_joints, action_dim, obs_dim, substeps = 1, 14, 8, 28, 4
            lanes_per_env, block, lds_bytes, vgprs, scratch_bytes, lds_rows = 1, 64, 0, 0, 0, 0
        self.info, self.env_id, self.num_envs = _I(), env_id, n
        self.obs = torch.zeros((n, 28))
        self.reward = torch.zeros(n)
        self.done = torch.zeros(n, dtype=torch.uint8)

    def reset(self):
        return self.obs

    def step(self, a):
        self.obs[:, :8] = a
        return self.obs

    def close(self):
        pass


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed_rollout(make_env, env_id, n, steps, warmup, preroll, dev, rank, world, no_graph, windows=1):
    """Rollout of n envs on this device: preroll + warmup untimed steps, then `windows` timed
    windows of exactly `steps` steps, each bracketed by a barrier + device sync on both sides
    (the same captured action batches replayed; the envs keep stepping).  Returns (env,
    elapsed_s, kernel_ms per launch, launches per graph, per-window ms per step): the median
    window, its time the max over ranks."""
    import torch
    import torch.distributed as dist
    env = make_env(env_id, n, dev, ACTION_SEED, rank * n, True)
    env.reset()
    na = env.info.action_dim
    total = preroll + warmup + steps
    if dev.type == "cuda":
        from pybulletgym_amd.vec_env import sample_actions
        # one distinct Philox batch per step, resident in HBM before the timed region
        acts = sample_actions(na, n, total, seed=ACTION_SEED, step0=0, env_offset=rank * n, device=dev)
    else:
        acts = torch.rand((total, n, na)) * 2 - 1
    for i in range(preroll + warmup):
        env.step(acts[i])
    t_first = preroll + warmup
    graph, G = None, 1
    if dev.type == "cuda" and not no_graph:
        # the timed steps as HIP-graph replays (G launches per graph, G divides K)
        G = max(d for d in range(1, min(1000, steps) + 1) if steps % d == 0)
        graphs = [env.capture([acts[t_first + r * G + j] for j in range(G)]) for r in range(steps // G)] \
            if G < steps else [env.capture([acts[t_first + j] for j in range(G)])]
    timing = dev.type == "cuda"
    if timing:
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)] \
            if no_graph else None
    runs = []
    for _ in range(windows):
        _sync(dev)
        if world > 1:
            dist.barrier()
        _sync(dev)
        t0 = time.perf_counter()
        if timing:
            e0.record(stream)
        if dev.type == "cuda" and not no_graph:
            for g in graphs:
                g.replay()
        else:
            for i in range(steps):
                if timing:
                    ev[i][0].record(stream)
                env.step(acts[t_first + i])
                if timing:
                    ev[i][1].record(stream)
        if timing:
            e1.record(stream)
        _sync(dev)
        if world > 1:
            dist.barrier()
        _sync(dev)
        elapsed = time.perf_counter() - t0
        if timing:
            kernel_ms = (sum(a.elapsed_time(b) for a, b in ev) if no_graph else e0.elapsed_time(e1)) / steps
        else:
            kernel_ms = elapsed / steps * 1e3
        if world > 1:
            t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, kernel_ms = float(t[0]), float(t[1])
        runs.append((elapsed, kernel_ms))
    elapsed, kernel_ms = sorted(runs)[len(runs) // 2]
    return env, elapsed, kernel_ms, G, [r[0] / steps * 1e3 for r in runs]


def leg_summary(env, world, n, steps, elapsed, kernel_ms, flops):
    """value / roofline block of one workload (HBM line from the algorithmic bytes; FP32 line
    from the counted flops when profiles/flops_per_env_step.json has the robot; float64 handles:
    the same counted flops against the FP64 vector peak)."""
    import torch
    prec = getattr(env, "precision", 32)
    alg = alg_bytes_per_env_step(env.info, prec)
    achieved = alg * n / (kernel_ms * 1e-3) / 1e9
    pmc = load_pmc(env.env_id, n, prec)
    d = {"env": env.env_id, "envs_per_gpu": n, "global_envs": world * n, "steps": steps,
         "dtype": "f64" if prec == 64 else "f32",
         "value": world * n * steps / elapsed, "unit": "env-steps/s", "ms_per_step": elapsed / steps * 1e3,
         "kernel": kernel_name(env), "kernel_ms": kernel_ms, "occupancy": occupancy(env),
         "obs_finite": bool(torch.isfinite(env.obs).all()),
         "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": achieved / HBM_PEAK_GBS, "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                      "traffic_source": (f"pybullet-gym_amd/perf/{os.path.basename(pmc['_path'])} (round "
                                         f"{pmc.get('round')}: FETCH_SIZE/WRITE_SIZE PMC passes, corrected)")
                      if pmc else None,
                      "kernel": kernel_name(env), "kernel_ms": kernel_ms, "alg_bytes_per_env_step": alg,
                      # the step is FP32-VALU (issue / latency) bound, not HBM bound (SURVEY.md 8d,
                      # BASELINE.md 4): the binding roofline is the `flop_roofline` block beside this one
                      "binding": "valu-fp64" if prec == 64 else "valu-fp32", "binding_line": "flop_roofline"}}
    f = flops.get(SHORT.get(env.env_id, env.env_id))
    if f:
        peak = FP64_PEAK_TFLOPS if prec == 64 else FP32_PEAK_TFLOPS
        tf = f["flops_per_env_step"] * n / (kernel_ms * 1e-3) / 1e12
        d["flop_roofline"] = {"bound": "valu-fp64" if prec == 64 else "valu-fp32", "achieved": tf, "peak": peak,
                              "unit": "TFLOP/s", "frac": tf / peak, "flops_per_env_step": f["flops_per_env_step"],
                              "source": "pybullet-gym_amd/perf/flops_per_env_step.json (counted, tools/count_flops.py)"}
    if pmc and pmc.get("valu_insts_per_launch"):
        d["valu_roofline"] = valu_roofline(pmc, kernel_ms, n)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--windows", type=int, default=5,
                    help="timed windows of --steps steps each; value and ms_per_step are the median window")
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--preroll", type=int, default=200, help="untimed steps before the warm-up (episode aging)")
    ap.add_argument("--envs-per-gpu", type=int, default=ENVS_PER_GPU)
    ap.add_argument("--env", default=ENV_ID)
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip timing the RCCL obs|reward|done all-gather (timed separately, outside `value`)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch every step from the host (no HIP graph)")
    ap.add_argument("--legs", default=EXTRA_LEGS,
                    help="extra workloads env:envs_per_gpu,... timed beside `value` ('none' = off)")
    ap.add_argument("--second-env", default=None, help="(compat) 'none' disables the extra legs")
    ap.add_argument("--leg-steps", type=int, default=200)
    ap.add_argument("--dry-run-cpu", action="store_true", help="CI: N > 1 control flow on CPU/gloo, no physics")
    ap.add_argument("--gang-lanes", type=int, default=-1,
                    help="A/B: gang width for the gang-kernel robots (16 or 32; -1 = the plan's choice)")
    ap.add_argument("--precision", type=int, default=64, choices=(32, 64),
                    help="the headline handle's physics precision (64, the default: float64, the reference's "
                         "btScalar; 32: the float32 fast mode)")
    args = ap.parse_args()
    if args.second_env == "none":
        args.legs = "none"

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run_cpu:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
        make_env = DryRunEnv
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)

    import pybulletgym_amd  # noqa: F401
    from pybulletgym_amd.distributed import gather_step
    if not args.dry_run_cpu:
        from pybulletgym_amd.vec_env import VecEnv

        def make_env(env_id, n, dev, seed, env_offset, autoreset, precision=None):
            precision = precision or args.precision
            lanes = args.gang_lanes if env_id.startswith("Humanoid") else -1
            return VecEnv(env_id, n, device=dev, seed=seed, env_offset=env_offset, autoreset=autoreset,
                          gang_lanes=lanes, precision=precision)

    flops = load_flops()
    n = args.envs_per_gpu
    env, elapsed, kernel_ms, G, windows_ms = timed_rollout(make_env, args.env, n, args.steps, args.warmup,
                                                           args.preroll, dev, rank, world, args.no_graph,
                                                           windows=args.windows)
    head = leg_summary(env, world, n, args.steps, elapsed, kernel_ms, flops)

    gather_ms = None
    if not args.no_gather and world > 1:
        for _ in range(3):
            gather_step(env.obs, env.reward, env.done)
        _sync(dev)
        t1 = time.perf_counter()
        for _ in range(20):
            gather_step(env.obs, env.reward, env.done)
        _sync(dev)
        gather_ms = (time.perf_counter() - t1) / 20 * 1e3

    legs = {}
    if args.legs not in ("", "none"):
        for spec in args.legs.split(","):
            eid, cnt, *pr = spec.split(":")
            prec = int(pr[0]) if pr else 32
            if (eid, int(cnt), prec) == (args.env, n, args.precision) or (args.dry_run_cpu and prec != 32):
                continue
            mk = (lambda *a, _p=prec: make_env(*a, precision=_p)) if not args.dry_run_cpu else make_env
            e2, el2, km2, _, _ = timed_rollout(mk, eid, int(cnt), args.leg_steps, min(args.warmup, 20),
                                               args.preroll, dev, rank, world, args.no_graph)
            legs[SHORT.get(eid, eid) + ("_f64" if prec == 64 else "_f32")] = \
                leg_summary(e2, world, int(cnt), args.leg_steps, el2, km2, flops)
            e2.close()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "timed_windows": len(windows_ms),
            "window_ms_per_step": windows_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == 64 else "f32",
            "data": "synthetic: Philox4x32-10 U(-1,1) float32 actions (key 0x5EED, counter (step, global env)) "
                    "generated in HBM before the timed region; robot compiled from the reference MJCF",
            "config": {"workload": f"{args.env} random-action rollout, auto-reset (TimeLimit 1000)",
                       "envs_per_gpu": n, "global_envs": world * n, "substeps": env.info.substeps,
                       "solver_iterations": 5, "parallelism": f"env-sharded x{world}, no per-step collective",
                       "preroll_steps": args.preroll,
                       "launch": "host loop" if args.no_graph or args.dry_run_cpu else
                       f"hipGraph replay, {G} captured launches per graph",
                       "lanes_per_env": env.info.lanes_per_env},
            "roofline": head["roofline"],
            "obs_finite": head["obs_finite"],
            "occupancy": head["occupancy"],
        }
        for k in ("flop_roofline", "valu_roofline"):
            if k in head:
                out[k] = head[k]
        out.update(legs)
        if gather_ms is not None:
            # the learner's optional flat batch: obs, reward and done packed into
            # one all_gather_into_tensor of [envs_per_gpu, obs_dim + 2] float32 per rank, timed
            # after the rollout (outside `value`)
            out["allgather_step_ms"] = gather_ms
            out["allgather_step_bytes"] = world * n * (env.info.obs_dim + 2) * 4
            out["allgather_payload"] = "obs | reward | done, float32 [global_envs, obs_dim + 2]"
        if args.dry_run_cpu:
            out["dry_run"] = "cpu/gloo stand-in env: control-flow check only, value is not a measurement"
        if world == 1 and not args.no_cpu_baseline and not args.dry_run_cpu:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
