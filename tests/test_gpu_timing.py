"""The bench's kernel timing (tg_set_kernel_timing / tg_read_kernel_timing):
windows of W consecutive step-kernel launches bracketed by one HIP event pair
(no event between the kernels they time) against every launch bracketed by
its own pair, and a window another launch of the library falls into dropped."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def test_gpu_windowed_kernel_timing():
    _cuda()
    import thormang_isaacgym_amd as tia
    n = 1024
    env = tia.make(seed=2, task="ThormangWalk", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
    a = torch.zeros(n, env.num_actions, device="cuda:0")
    for _ in range(10):
        env.step(a)
    env.sim.read_kernel_timing()
    env.sim.set_kernel_timing(-8)          # windows of 8 launches
    for _ in range(44):
        env.step(a)
    torch.cuda.synchronize()
    env.sim.set_kernel_timing(0)           # the open window (4 launches) is dropped
    ms_w, n_w = env.sim.read_kernel_timing()
    assert n_w % 8 == 0 and 32 <= n_w <= 40, n_w
    env.sim.set_kernel_timing(1)           # every launch, one pair each
    for _ in range(32):
        env.step(a)
    torch.cuda.synchronize()
    env.sim.set_kernel_timing(0)
    ms_1, n_1 = env.sim.read_kernel_timing()
    assert n_1 == 32
    per_w, per_1 = ms_w / n_w, ms_1 / n_1
    # a window holds the kernels and the gaps between them, one pair its kernel
    # and the pair's own stall: the two agree to a few microseconds
    assert 0.0 < per_w and abs(per_w - per_1) < 0.01, (per_w, per_1)
    # another launch of the library inside a window drops that window
    env.sim.set_kernel_timing(-8)
    for i in range(16):
        env.step(a)
        if i == 3:
            env.sim.refresh_rigid_body_state_tensor()   # tg_rigid_body_states: a kernel launch
    torch.cuda.synchronize()
    env.sim.set_kernel_timing(0)
    _, n_d = env.sim.read_kernel_timing()
    assert n_d == 8, n_d                   # the first window was dropped, the second kept


def test_gpu_bench_gpus_two_launches_two_ranks_on_one_gpu():
    """`python bench.py --gpus 2` on the one-GPU box: the
    parent touches no GPU and starts two torch.distributed.run ranks, which
    share cuda:0 over gloo (TG_BENCH_SHARE_GPU: RCCL refuses two ranks on one
    device -- a rehearsal of the launch path, not a scaling number); rank 0
    prints one line with n_gpus 2 and the process group's size 2."""
    _cuda()
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(TG_BENCH_DIST_BACKEND="gloo", TG_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--num-envs", "1024", "--no-cpu-baseline"], env=env, cwd=repo, capture_output=True, text=True,
                       timeout=300)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    print({k: d[k] for k in ("value", "n_gpus", "ms_per_step")}, d["dist"])
    assert d["n_gpus"] == 2 and d["dist"]["world_size"] == 2
    assert d["value"] > 0 and d["config"]["parallelism"] == "env-dp2"
