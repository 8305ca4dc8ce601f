"""The N>1 bench path on CPU: two gloo ranks run bench.timed_region (barrier +
sync on both sides, max over ranks) with a rank-dependent synthetic step, and
rank 0 aggregates whole-job throughput the way bench.py does (weak scaling:
every rank owns its own env batch, no collective inside the timed region)."""
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    calls = [0]

    def step():   # rank 1 is the slow rank: the job time is its time
        calls[0] += 1
        time.sleep(0.002 * (1 + rank))

    el = bench.timed_region(step, 25, world, "cpu", lambda: None)
    t_local = torch.tensor([el])
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, t_local)
    out[rank] = (calls[0], el, [float(g) for g in gathered])
    dist.destroy_process_group()


def test_two_rank_timed_region_takes_max_over_ranks():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank, args=(world, port, out), nprocs=world, join=True)
    (c0, e0, g0), (c1, e1, _) = out[0], out[1]
    assert c0 == c1 == 25                      # exactly K timed steps on every rank
    assert e0 == e1                            # every rank reports the max
    assert e0 >= 25 * 0.004 * 0.95             # >= the slow rank's own time
    assert abs(g0[0] - g0[1]) < 1e-12
    N = 4096
    value = N * 25 * world / e0                # bench.py: whole-job env-steps/s
    assert value > 0


def _rank_rlgames(rank, world, port, out):
    """One torchrun-style rank: the env creator (make mocked) and the
    per-iteration episode-statistics gather over gloo."""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd import rlgames
    seen = {}

    def fake_make(seed, task, num_envs, sim_device, rl_device, **kw):
        seen.update(seed=seed, task=task, num_envs=num_envs, sim_device=sim_device, rl_device=rl_device)
        return "env"

    real = tia.make
    tia.make = fake_make
    try:
        # the seed as train.py:80 hands it over (cfg.seed += LOCAL_RANK)
        create = rlgames.get_rlgames_env_creator(seed=42 + rank, task_config={"env": {"numEnvs": 8}}, task_name="Gogoro",
                                                 sim_device="cuda:0", rl_device="cuda:0", multi_gpu=True)
        env = create()
    finally:
        tia.make = real
    # episode statistics: rank r runs 4 envs; env k finishes an episode of
    # length k + 1 with reward (r + 1) per step
    st = rlgames.EpisodeStats(4, "cpu")
    for t in range(4):
        rew = torch.full((4,), float(rank + 1))
        reset = (torch.arange(4) == t).long()
        st.update(rew, reset)
    g = st.gather()
    again = st.gather()
    out[rank] = (env, dict(seen), g, again)
    dist.destroy_process_group()


def test_two_rank_env_creator_and_episode_gather():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank_rlgames, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        env, seen, g, again = out[r]
        assert env == "env"
        # rank -> device (LOCAL_RANK); the seed passes through unchanged (train.py:80
        # offset it by LOCAL_RANK already), so each rank keys its own Philox streams
        assert seen["sim_device"] == seen["rl_device"] == f"cuda:{r}"
        assert seen["seed"] == 42 + r and seen["num_envs"] == 8
        # 4 episodes per rank, lengths 1..4; returns (r+1)*len; summed over both ranks
        assert g["episodes"] == 8
        assert abs(g["mean_length"] - 2.5) < 1e-12
        assert abs(g["mean_return"] - (1 * 10 + 2 * 10) / 8) < 1e-12
        assert again["episodes"] == 0          # sums reset after each gather


def _bench(args, extra_env=None, timeout=240):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TG_BENCH_STUB="1", **(extra_env or {}))
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env, cwd=REPO,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, [json.loads(ln) for ln in lines]


def test_bench_gpus_n_launches_n_ranks():
    """`python bench.py --gpus 2` (no WORLD_SIZE) starts two ranks itself; rank 0
    alone prints the line, with n_gpus and the process group's size both 2."""
    r, lines = _bench(["--gpus", "2", "--steps", "5", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["dist"]["world_size"] == 2
    assert lines[0]["steps"] == 5 and lines[0]["local_rank"] == 0


def test_bench_gpus_mismatch_with_world_size_raises():
    r, lines = _bench(["--gpus", "2", "--steps", "2", "--warmup", "0"],
                      extra_env=dict(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and not lines
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr


def test_bench_gpus_one_runs_in_process():
    r, lines = _bench(["--gpus", "1", "--steps", "3", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert lines[0]["n_gpus"] == 1 and lines[0]["dist"]["world_size"] == 1
