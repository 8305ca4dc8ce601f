"""Env-steps/sec of the full VecTask.step hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--task Gogoro] [--num-envs 4096]

One process per GPU: under torchrun RANK/LOCAL_RANK/WORLD_SIZE come from the
env (WORLD_SIZE must equal --gpus); a plain ``python bench.py --gpus N`` with
N > 1 starts the N ranks itself (torch.distributed.run children).  Every
rank owns its own env batch (weak scaling, no collective on the hot path).  A "step" is one ``env.step(actions)`` call: pre-physics kernel,
``sim.substeps`` articulation substeps, post-physics kernel (observations,
reward, masked resets, timeouts) -- inputs resident in HBM, synthetic
actions U(-1,1) from torch.Generator(seed 1234 + rank).  Rank 0 prints one
JSON line; ``value`` = envs x steps x ranks / max-over-ranks wall time.

Roofline: the dominant kernel is the articulation step kernel
(tg::step_par_kernel, all substeps of one simulate() in one launch).  For the
one-launch steps (ThormangWalk*, Gogoro) the library brackets windows of
TIMING_WINDOW consecutive step-kernel launches with one HIP event pair on the
sim stream (tg_set_kernel_timing(-TIMING_WINDOW); a window any other launch of
the library falls into is dropped), so no event sits between the kernels it
times; otherwise it brackets every TIMING_PERIOD-th launch by itself (an event
pair stalls the queue ~5 us per side, which that figure then includes).  Its
algorithmic bytes per env-step
(state + inputs the kernel must read/write) give the achieved
HBM rate against the 8 TB/s MI355X peak.  ``traffic`` is the PMC-measured HBM
bytes per launch of the same kernel from a committed rocprofv3 summary
(scripts/gpu_profile.sh + scripts/pmc_summary.py) when one exists for this
workload, else null.  cpu_baseline: the CPU oracle env (oracle/: the same physics
+ task algorithm, OpenMP) on a bounded sample of the same workload, rank 0
only: its fp32 build (the GPU's arithmetic type) as the value, the fp64 parity
oracle beside it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0
TIMING_PERIOD = 16
TIMING_WINDOW = 16
MIN_KERNEL_SAMPLES = 32
ONE_LAUNCH_TASKS = ("ThormangWalk", "ThormangWalkDR", "Gogoro", "GogoroPaper")


def algorithmic_bytes_per_env_step(task_name: str, env) -> tuple[int, dict]:
    """Algorithmic HBM bytes of one env-step: the state and
    task buffers the step must read and write once -- inputs resident in HBM,
    model constants (shared by every env) excluded, and none of this
    library's own per-env caches counted.  Returns (bytes, breakdown)."""
    if task_name == "Gogoro":
        # §8(d) verbatim: read 444 B, write 457 B
        rd = dict(action=4, root=52, dof=312, cmd=4, a_hist=20, steer_off=4, speed=4, yaw_cmd=4, imu_off=4,
                  speed_off=4, progress=8, reset=8, steer_kd=4, seat_offsets=12)
        wr = dict(root=52, dof=312, cmd=4, a_hist=20, progress=8, reset=8, obs=24, buffer_obs=24, rew=4, time_out=1)
    elif task_name.startswith("ThormangWalk"):
        # §8(d) "Thormang walk" with the frozen observation layout
        # (13 + 3 D floats: height, body lin/ang vel, gravity, commands, dof pos/vel, actions)
        D, O = env.num_dof, env.num_obs
        rd = dict(action=4 * D, root=52, dof=8 * D, last_action=4 * D, commands=12, progress=8, reset=8)
        wr = dict(root=52, dof=8 * D, obs=4 * O, last_action=4 * D, rew=4, reset=8, progress=8, time_out=1)
        if task_name == "ThormangWalkDR":   # §8(d) cfg 5: body-mass scale, foot friction, push
            G = env.sim.model.num_groups
            rd.update(mass_scale=4 * G, friction=4 * len(env.sim.model.shapes), push=12)
    elif task_name == "GogoroPaper":
        # the paper variant's step: the Gogoro state plus its 20-step clean and
        # noisy observation histories (8 x 20 floats each, read + written), the
        # steering-delay ring and command history, the push wrench
        D, O = env.num_dof, env.num_obs
        rd = dict(action=4, root=52, dof=8 * D, buffer_obs=4 * O, buffer_obs_noisy=4 * O, cmd_hist=20,
                  steer_delay=4 * 20, scalars=40, progress=8, reset=8)
        wr = dict(root=52, dof=8 * D, buffer_obs=4 * O, buffer_obs_noisy=4 * O, obs=4 * O, cmd_hist=20,
                  steer_delay=4 * 20, rew=4, reset=8, progress=8, time_out=1, push=12)
    else:
        raise ValueError(f"no algorithmic byte count for task {task_name}")
    return sum(rd.values()) + sum(wr.values()), {"read": rd, "write": wr}


def kernel_bytes_per_env(task_name: str, env) -> int:
    """What the articulation step kernel itself moves per env (reported beside
    the algorithmic count, never as it): root / dof state, active-dof targets
    and property fields, lock windows, this library's per-env composite cache
    and shape friction, plus the fused walk post-physics I/O."""
    m = env.sim.model
    D, G, S = m.num_dof, m.num_groups, len(m.shapes)
    na = len(m.active_dofs)
    nl = len(m.locked_dofs)
    kc = 10 * G + 12 * (G - 1) + 12 * S
    read = 13 * 4 + na * 2 * 4 + na * 2 * 4 + na * 8 * 4 + nl * 2 * 4 + kc * 4 + S * 4 + 1
    write = 13 * 4 + D * 2 * 4
    if task_name.startswith("ThormangWalk"):
        read += 8 + 8 + D * 4 * 2 + 3 * 4
        write += env.num_obs * 4 + D * 4 + 4 + 8 + 1 + 8
        if getattr(env, "push_enabled", False):
            write += 6 * 4
    return read + write


def host_cpu_info() -> dict:
    """The GPU box's host CPU as this process sees it: model name, logical
    CPUs of the machine (nproc --all), CPUs this process may run on (affinity)
    and its cgroup CPU quota, if any."""
    info = {"model": None, "nproc_all": os.cpu_count(), "affinity": None, "cgroup_quota_cpus": None}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                info["cgroup_quota_cpus"] = float(q) / float(per)
    except (OSError, ValueError):
        pass
    return info


def baseline_threads(info: dict) -> int:
    """All the host cores this process may use: the affinity set, capped by the
    cgroup quota (a quota below the affinity count would only time-slice)."""
    n = info.get("affinity") or info.get("nproc_all") or 1
    q = info.get("cgroup_quota_cpus")
    if q:
        n = min(n, max(1, int(q)))
    return int(n)


def timed_region(step, steps: int, world: int, device, sync) -> float:
    """Time exactly ``steps`` calls of ``step`` between barriers + device syncs
    on both sides; with world > 1 return the max over ranks (all ranks get it)."""
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def committed_traffic(task_name: str, num_envs: int):
    """PMC HBM bytes per step-kernel launch from the newest committed summary for
    this workload (profiles/*/pmc_<task><envs>.json), or (None, None)."""
    import glob
    hits = sorted(glob.glob(os.path.join(REPO, "profiles", "*", f"pmc_{task_name.lower()}{num_envs}.json")))
    if not hits:
        return None, None
    with open(hits[-1]) as f:
        d = json.load(f)
    for k, v in d.items():
        if "step_par_kernel" in k and "hbm_bytes_per_dispatch" in v:
            return v["hbm_bytes_per_dispatch"], os.path.relpath(hits[-1], REPO) + " (FETCH_SIZE x2 + WRITE_SIZE)"
    return None, None


def committed_sq(task_name: str, num_envs: int):
    """VALU / wait fractions of the step kernel's wave cycles from the newest
    committed SQ-counter summary (profiles/*/sq_<task><envs>.json,
    scripts/gpu_pmc_sq.sh), or None.  SQ_WAVE_CYCLES, SQ_ACTIVE_INST_* and
    SQ_WAIT_* count the same (quad-)cycle unit, summed over the kernel's waves."""
    import glob
    hits = sorted(glob.glob(os.path.join(REPO, "profiles", "*", f"sq_{task_name.lower()}{num_envs}.json")))
    if not hits:
        return None
    with open(hits[-1]) as f:
        d = json.load(f)
    for k, v in d.items():
        a = v.get("avg", {})
        if "step_par_kernel" in k and a.get("SQ_WAVE_CYCLES"):
            wc = a["SQ_WAVE_CYCLES"]
            out = {"source": os.path.relpath(hits[-1], REPO)}
            for key, c in (("valu_active_frac", "SQ_ACTIVE_INST_VALU"), ("wait_any_frac", "SQ_WAIT_ANY"),
                           ("wait_inst_any_frac", "SQ_WAIT_INST_ANY"), ("active_inst_any_frac", "SQ_ACTIVE_INST_ANY"),
                           ("lds_active_frac", "SQ_ACTIVE_INST_LDS")):
                if c in a:
                    out[key] = a[c] / wc
            if a.get("SQ_WAVES"):
                out["valu_insts_per_wave"] = a.get("SQ_INSTS_VALU", 0.0) / a["SQ_WAVES"]
            if a.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in a:
                out["lds_bank_conflict_frac"] = a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"]
            return out
    return None


def cpu_baseline(task_name: str, num_envs: int, threads: int, terrain_env=None, precision: str = "f32",
                 seconds: float = 10.0):
    """The oracle env (oracle/: the same physics and task algorithm) on the
    host cores, bounded to ~``seconds``.  precision "f32" (real = float, the
    GPU's arithmetic type: the fair comparator, reported as the baseline) or
    "f64" (the parity oracle itself)."""
    from tests.gpu_harness import NumpyDraws, OracleGogoro, OracleWalk, parity_cfg, walk_cfg
    if terrain_env is not None:   # same heightfield and spawn heights as the GPU env
        from tests.oracle_lib import set_heightfield
        t = terrain_env.terrain
        o = -float(terrain_env._terrain_start_mid)
        set_heightfield(t.heightsamples.cpu().numpy(), t.V_scale, t.H_scale, o, o, friction=0.98)
    if task_name == "Gogoro":
        spawn = None if terrain_env is None else terrain_env.root_reset_tensor[:, 2].cpu().numpy()
        env = OracleGogoro(parity_cfg(num_envs), NumpyDraws(0), threads=threads, spawn_z=spawn, precision=precision)
        shape = (num_envs,)
    else:
        env = OracleWalk(walk_cfg(num_envs, task_name), NumpyDraws(0), threads=threads, precision=precision)
        shape = (num_envs, env.D)
    rs = np.random.default_rng(1234)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and steps < 400:
        env.step(rs.uniform(-1, 1, shape).astype(np.float32))
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{task_name} {num_envs} envs x {steps} steps (oracle/ {precision} physics + C task "
                      f"restatement, OpenMP {threads} threads) = {dt:.1f} s"}


def post_physics_only(num_envs: int) -> dict:
    """BASELINE.md's second context figure on this host: the reference's
    post-physics math alone (compute_gogoro_observations +
    compute_gogoro_reward, tasks/gogoro_new.py:645-723) -- here as the oracle's
    C restatement of it (oracle/gogoro_task.c), one thread, no physics."""
    from tests.oracle_lib import lib, ptr
    L = lib()
    rs = np.random.default_rng(7)
    root = rs.normal(0, 0.3, (num_envs, 13)).astype(np.float32)
    q = rs.normal(0, 1, (num_envs, 4)).astype(np.float32)
    root[:, 3:7] = q / np.linalg.norm(q, axis=1, keepdims=True)
    yaw = rs.uniform(-np.pi, np.pi, num_envs).astype(np.float32)
    cmd = rs.uniform(-0.5, 0.5, num_envs).astype(np.float32)
    ah = rs.uniform(-1, 1, (num_envs, 5)).astype(np.float32)
    prog = rs.integers(0, 1000, num_envs).astype(np.int64)
    obs = np.zeros((num_envs, 6), np.float32)
    rew = np.zeros(num_envs, np.float32)
    rst = np.zeros(num_envs, np.int64)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        L.oracle_gogoro_observations(num_envs, ptr(root), ptr(yaw), ptr(cmd), ptr(obs))
        L.oracle_gogoro_reward(num_envs, ptr(obs), ptr(prog), ptr(ah), 1000, ptr(rew), ptr(rst))
        n += 1
    dt = time.perf_counter() - t0
    return {"value": num_envs * n / dt, "unit": "env-steps/s", "cores": 1,
            "sample": f"observations + reward of {num_envs} envs x {n} calls, one thread = {dt:.2f} s"}


def solver_desc(env) -> str:
    """The contact solve the step ran (the cfg's sim.physx, as tg_sim_params holds it)."""
    sp = env.sim.get_sim_params()
    kind = "TGS" if sp.solver_type == 1 else "PGS"
    return (f"{kind}: {sp.contact_iterations} position iterations"
            f"{' (sub-steps)' if sp.solver_type == 1 else ''} + {sp.velocity_iterations} velocity iterations")


def launch_ranks(n: int, argv: list[str]) -> int:
    """``python bench.py --gpus N`` (N > 1, no WORLD_SIZE in the env): run the N
    ranks as fresh child processes under torch.distributed.run (one per GPU,
    LOCAL_RANK = i, rendezvous on 127.0.0.1), wait for them and return their
    exit status.  The caller has touched no GPU; rank 0 prints the JSON line.
    (reference: isaacgymenvs/train.py:74-82 -- one process per GPU, LOCAL_RANK
    -> device, seed + rank)"""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def stub_run(args, world: int, rank: int, local: int, rccl_world):
    """TG_BENCH_STUB=1: the launch / rank / timing path with a sleep in place of
    env.step and no GPU (CPU tests only; never a measured line)."""
    def step():
        time.sleep(0.001)
    for _ in range(args.warmup):
        step()
    elapsed = timed_region(step, args.steps, world, "cpu", lambda: None)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": args.num_envs * args.steps * world / elapsed,
                          "n_gpus": world, "steps": args.steps, "local_rank": local,
                          "dist": {"world_size": rccl_world or 1}}), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--task", default="ThormangWalk")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--solver-type", type=int, choices=(0, 1), default=None,
                    help="override the task cfg's sim.physx.solver_type (0 PGS, 1 TGS) for an A/B line")
    ap.add_argument("--contact-offset", type=float, default=None,
                    help="override sim.physx.contact_offset (0 = every point within contact_margin carries a row) "
                         "for an A/B line")
    ap.add_argument("--whole-body", action="store_true",
                    help="walk tasks: env.asset.wholeBodyCollision (feet, shins and hands collide; model thormang_wb)")
    ap.add_argument("--terrain", action="store_true",
                    help="Gogoro only: the reference's USE_TERAIN Perlin terrain (gogoro_new.py:26)")
    args = ap.parse_args()
    if args.terrain and args.task != "Gogoro":
        ap.error("--terrain applies to the Gogoro task (the reference has terrain only there)")

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched as `python bench.py --gpus N`: start the N ranks ourselves,
        # as child processes, before this process makes any GPU call
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher and the flag disagree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # developer rehearsal of the N > 1 path on a one-GPU box (not a scaling
    # number): TG_BENCH_DIST_BACKEND=gloo with TG_BENCH_SHARE_GPU=1 puts every
    # rank on cuda:0 (RCCL refuses two ranks on one device)
    backend = os.environ.get("TG_BENCH_DIST_BACKEND", "nccl")
    if os.environ.get("TG_BENCH_SHARE_GPU"):
        local = 0
    stub = os.environ.get("TG_BENCH_STUB") == "1"
    if stub:   # CPU test of the launch path (tests/test_bench_dist.py): no GPU, gloo
        backend = "gloo"
    rccl_world = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend=backend, init_method="env://")
        rccl_world = dist.get_world_size()   # what RCCL itself reports (the SCALE runs are checked on it)
        if rccl_world != world:
            raise RuntimeError(f"WORLD_SIZE {world} but the process group has {rccl_world} ranks")
    if stub:
        stub_run(args, world, rank, local, rccl_world)
        return
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"

    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg(args.task, num_envs=args.num_envs, sim_device=dev)
    if args.solver_type is not None:
        cfg["sim"]["physx"]["solver_type"] = args.solver_type
    if args.contact_offset is not None:
        cfg["sim"]["physx"]["contact_offset"] = args.contact_offset
    if args.whole_body:
        if not args.task.startswith("ThormangWalk"):
            ap.error("--whole-body applies to the ThormangWalk tasks")
        cfg["env"]["asset"] = dict(cfg["env"].get("asset", {}), wholeBodyCollision=True)
    if args.terrain:
        from thormang_isaacgym_amd.tasks import gogoro as gogoro_task
        gogoro_task.USE_TERAIN = True
        torch.manual_seed(42 + rank)        # the terrain draws from the CPU generator, as the reference
    env = tia.make(seed=42 + rank, task=args.task, num_envs=args.num_envs, sim_device=dev, rl_device=dev, cfg=cfg)
    gen = torch.Generator(device=dev).manual_seed(1234 + rank)
    N = args.num_envs
    acts = env.num_actions
    # synthetic actions resident in HBM before the timed region
    pool = torch.rand(min(args.steps + args.warmup, 512), N, acts, device=dev, generator=gen) * 2 - 1
    it = [0]

    def step():
        a = pool[it[0] % pool.shape[0]]
        it[0] += 1
        return env.step(a)

    for _ in range(args.warmup):
        step()
    env.sim.read_kernel_timing()
    windowed = args.task in ONE_LAUNCH_TASKS
    env.sim.set_kernel_timing(-TIMING_WINDOW if windowed else TIMING_PERIOD)
    elapsed = timed_region(step, args.steps, world, dev if backend == "nccl" else "cpu", torch.cuda.synchronize)
    # a short timed region (the driver's --steps 20) samples only a launch or
    # two: keep stepping, after the clock has stopped, until MIN_KERNEL_SAMPLES
    # launches are timed, so kernel_ms is never a one- or two-sample figure
    extra = 0
    while (args.steps + extra < MIN_KERNEL_SAMPLES + 2 * TIMING_WINDOW if windowed
           else (args.steps + extra) // TIMING_PERIOD < MIN_KERNEL_SAMPLES):
        step()
        extra += 1
    torch.cuda.synchronize()
    env.sim.set_kernel_timing(0)
    tot_ms, launches = env.sim.read_kernel_timing()
    if launches == 0 and windowed:   # every window had another launch in it: time launches one by one
        windowed = False
        env.sim.set_kernel_timing(TIMING_PERIOD)
        for _ in range(MIN_KERNEL_SAMPLES * TIMING_PERIOD):
            step()
        torch.cuda.synchronize()
        env.sim.set_kernel_timing(0)
        tot_ms, launches = env.sim.read_kernel_timing()
    kern_ms = tot_ms / max(launches, 1)
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    value = N * args.steps * world / elapsed
    bpe, breakdown = algorithmic_bytes_per_env_step(args.task, env)
    kbpe = kernel_bytes_per_env(args.task, env)
    # the committed PMC / SQ summaries profile the default workload of a task
    # (flat ground, the cfg's solver, the foot-only model): other variants
    # carry no traffic figure rather than another workload's
    profiled = not (args.terrain or args.whole_body or args.solver_type is not None
                    or args.contact_offset is not None)
    traffic, traffic_src = committed_traffic(args.task, N) if profiled else (None, None)
    achieved = bpe * N / (kern_ms * 1e-3) / 1e9
    sim_cfg = cfg["sim"]
    out = {
        "metric": "env-steps/sec (num_envs x step Hz)",
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
        "data": "synthetic (actions U(-1,1), seed 1234+rank; model compiled from the reference URDF)",
        "config": {"workload": f"{args.task} {N} envs/GPU, {'Perlin terrain' if args.terrain else 'flat ground'}, "
                               f"dt {sim_cfg['dt']} s x "
                               f"{sim_cfg.get('substeps', 2)} substeps ({1.0 / sim_cfg['dt']:.1f} Hz control)",
                   "num_envs_per_gpu": N, "parallelism": f"env-dp{world}",
                   "contact_solver": solver_desc(env),
                   "contact_shapes": f"{len(env.model.shapes)} ({', '.join(sorted(set(sh.kind for sh in env.model.shapes)))})"
                   if hasattr(env, "model") else None},
        "dist": {"backend": ("nccl (RCCL)" if backend == "nccl" else
                             f"{backend} (rehearsal{', ranks share cuda:0' if os.environ.get('TG_BENCH_SHARE_GPU') else ''})")
                 if rccl_world else None, "world_size": rccl_world or 1,
                 "collectives_in_timed_region": "barrier + max-over-ranks all_reduce of the elapsed time"
                 if rccl_world else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "tg::step_par_kernel (one launch per simulate)", "kernel_ms": kern_ms,
                     "kernel_launches": launches,
                     "kernel_timing": (f"HIP events around windows of {TIMING_WINDOW} consecutive step-kernel "
                                       "launches of the timed region" if windowed else
                                       f"HIP events around every {TIMING_PERIOD}th launch of the timed region")
                                      + (f" and of {extra} untimed steps after it" if extra else ""),
                     "bytes_per_env_step": bpe, "bytes_source": "SURVEY.md §8(d) algorithmic bytes per env-step",
                     "bytes_breakdown": breakdown, "algorithmic_bytes_per_launch": bpe * N,
                     "kernel_bytes_per_env_step": kbpe,
                     "traffic_over_algorithmic": traffic / (bpe * N) if traffic else None,
                     "traffic_source": traffic_src},
    }
    sq = committed_sq(args.task, N) if profiled else None
    if sq is not None:
        out["roofline"]["issue"] = sq
    if not args.no_cpu_baseline and world == 1:
        try:
            info = host_cpu_info()
            thr = baseline_threads(info)
            tenv = env if args.terrain else None
            out["cpu_baseline"] = cpu_baseline(args.task, N, threads=thr, terrain_env=tenv, precision="f32")
            out["cpu_baseline"]["fp64_oracle"] = cpu_baseline(args.task, N, threads=thr, terrain_env=tenv,
                                                              precision="f64", seconds=5.0)
            if args.task == "Gogoro":
                out["cpu_baseline"]["post_physics_only"] = post_physics_only(N)
            out["cpu_baseline"]["host"] = info
        except Exception as exc:  # baseline is reported, never the measured value
            out["cpu_baseline"] = {"value": None, "error": repr(exc)}
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
