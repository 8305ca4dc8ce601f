"""Env-steps/sec of the full VecTask.step hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--task Gogoro] [--num-envs 4096]

One process per GPU (torchrun for N>1, RANK/LOCAL_RANK/WORLD_SIZE from the
env); every rank owns its own env batch (weak scaling, no collective on the
hot path).  A "step" is one ``env.step(actions)`` call: pre-physics kernel,
``sim.substeps`` articulation substeps, post-physics kernel (observations,
reward, masked resets, timeouts) -- inputs resident in HBM, synthetic
actions U(-1,1) from torch.Generator(seed 1234 + rank).  Rank 0 prints one
JSON line; ``value`` = envs x steps x ranks / max-over-ranks wall time.

Roofline: the dominant kernel is the articulation step kernel
(tg::step_par_kernel, all substeps of one simulate() in one launch); the
library brackets every TIMING_PERIOD-th launch of the timed region with HIP
events on the sim stream (tg_set_kernel_timing; an event pair stalls the
queue ~5 us per side, so timing every launch would cost the measured
throughput ~13 %), and its algorithmic bytes per env-step
(state + inputs the kernel must read/write) give the achieved
HBM rate against the 8 TB/s MI355X peak.  ``traffic`` is the PMC-measured HBM
bytes per launch of the same kernel from a committed rocprofv3 summary
(scripts/gpu_profile.sh + scripts/pmc_summary.py) when one exists for this
workload, else null.  cpu_baseline: the CPU oracle env (oracle/, fp64 physics +
task restatement, OpenMP) on a bounded sample of the same workload, rank 0 only.
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


def kernel_bytes_per_env(task_name: str, env) -> int:
    """Algorithmic HBM bytes one articulation step reads + writes per env
    (DESIGN.md §Roofline): root state r/w, dof_state r/w, active-dof targets and
    properties, locked-dof lock windows, per-env composite cache, shape friction."""
    m = env.sim.model
    D, G, S = m.num_dof, m.num_groups, len(m.shapes)
    na = len(m.active_dofs)
    nl = len(m.locked_dofs)
    kc = 10 * G + 12 * (G - 1) + 12 * S
    read = 13 * 4 + na * 2 * 4 + na * 2 * 4 + na * 8 * 4 + nl * 2 * 4 + kc * 4 + S * 4 + 1
    write = 13 * 4 + D * 2 * 4
    if task_name.startswith("ThormangWalk"):
        # post-physics fused into the kernel (tg_walk_step): progress, reset flag,
        # actions, last actions, commands in; observations, last actions, reward,
        # reset, timeout, progress out (+ the push wrench row for the DR variant)
        read += 8 + 8 + D * 4 * 2 + 3 * 4
        write += env.num_obs * 4 + D * 4 + 4 + 8 + 1 + 8
        if getattr(env, "push_enabled", False):
            write += 6 * 4
    return read + write


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


def cpu_baseline(task_name: str, num_envs: int, threads: int, terrain_env=None):
    from tests.gpu_harness import NumpyDraws, OracleGogoro, OracleWalk, parity_cfg, walk_cfg
    if terrain_env is not None:   # same heightfield and spawn heights as the GPU env
        from tests.oracle_lib import set_heightfield
        t = terrain_env.terrain
        o = -float(terrain_env._terrain_start_mid)
        set_heightfield(t.heightsamples.cpu().numpy(), t.V_scale, t.H_scale, o, o, friction=0.98)
    if task_name == "Gogoro":
        spawn = None if terrain_env is None else terrain_env.root_reset_tensor[:, 2].cpu().numpy()
        env = OracleGogoro(parity_cfg(num_envs), NumpyDraws(0), threads=threads, spawn_z=spawn)
        shape = (num_envs,)
    else:
        env = OracleWalk(walk_cfg(num_envs, task_name), NumpyDraws(0), threads=threads)
        shape = (num_envs, env.D)
    rs = np.random.default_rng(1234)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 10.0 and steps < 400:
        env.step(rs.uniform(-1, 1, shape).astype(np.float32))
        steps += 1
    dt = time.perf_counter() - t0
    return {"value": num_envs * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{task_name} {num_envs} envs x {steps} steps (oracle/ fp64 physics + C task restatement, "
                      f"OpenMP {threads} threads) = {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--task", default="ThormangWalk")
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--terrain", action="store_true",
                    help="Gogoro only: the reference's USE_TERAIN Perlin terrain (gogoro_new.py:26)")
    args = ap.parse_args()
    if args.terrain and args.task != "Gogoro":
        ap.error("--terrain applies to the Gogoro task (the reference has terrain only there)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = f"cuda:{local}"

    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    cfg = load_task_cfg(args.task, num_envs=args.num_envs, sim_device=dev)
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
    env.sim.set_kernel_timing(TIMING_PERIOD)
    elapsed = timed_region(step, args.steps, world, dev, torch.cuda.synchronize)
    env.sim.set_kernel_timing(0)
    tot_ms, launches = env.sim.read_kernel_timing()
    kern_ms = tot_ms / max(launches, 1)
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    value = N * args.steps * world / elapsed
    bpe = kernel_bytes_per_env(args.task, env)
    traffic, traffic_src = committed_traffic(args.task, N)
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
                   "num_envs_per_gpu": N, "parallelism": f"env-dp{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "tg::step_par_kernel (one launch per simulate)", "kernel_ms": kern_ms,
                     "kernel_launches": launches, "kernel_timing": f"HIP events around every {TIMING_PERIOD}th launch of the timed region", "bytes_per_env_step": bpe,
                     "algorithmic_bytes_per_launch": bpe * N, "traffic_source": traffic_src},
    }
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.task, N, threads=min(16, os.cpu_count() or 1),
                                               terrain_env=env if args.terrain else None)
        except Exception as exc:  # baseline is reported, never the measured value
            out["cpu_baseline"] = {"value": None, "error": repr(exc)}
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
