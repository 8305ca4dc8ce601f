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
