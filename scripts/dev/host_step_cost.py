"""Developer probe: where the driver form's (--steps 20 --warmup 5) extra time
over the 2000-step steady state goes.

  1. host cost of one env.step call (Python + library launch), GPU queue not
     drained: the latency the first timed step adds before its kernel starts;
  2. the step kernel's duration (HIP events, one launch at a time) over the
     first launches after 5 warm-up steps, in windows of 8 launches: a clock /
     warm-cache ramp shows as longer early windows;
  3. the timed region as bench.py forms it, K = 20, after 5 and after 400
     warm-up steps.

    python scripts/dev/host_step_cost.py [task] [num_envs]
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import thormang_isaacgym_amd as tia  # noqa: E402
from bench import timed_region  # noqa: E402

task = sys.argv[1] if len(sys.argv) > 1 else "ThormangWalk"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
dev = "cuda:0"


def make():
    env = tia.make(seed=42, task=task, num_envs=n, sim_device=dev, rl_device=dev)
    gen = torch.Generator(device=dev).manual_seed(1234)
    pool = torch.rand(512, n, env.num_actions, device=dev, generator=gen) * 2 - 1
    it = [0]

    def step():
        a = pool[it[0] % pool.shape[0]]
        it[0] += 1
        return env.step(a)
    return env, step


env, step = make()
# 2. kernel ramp after 5 warm-up steps
for _ in range(5):
    step()
torch.cuda.synchronize()
env.sim.read_kernel_timing()
env.sim.set_kernel_timing(1)
win = []
for w in range(12):
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    ms, k = env.sim.read_kernel_timing()
    win.append(1e3 * ms / max(k, 1))
env.sim.set_kernel_timing(0)
print("kernel us per launch, windows of 8 launches after 5 warm-up steps:", " ".join(f"{x:.1f}" for x in win))

# 1. host cost per call with the queue not drained
for _ in range(200):
    step()
torch.cuda.synchronize()
for reps in (1, 50):
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host time per env.step over {reps} call(s), queue not drained: {1e6 * (t1 - t0) / reps:.1f} us")
a = torch.zeros(n, env.num_actions, device=dev)
t0 = time.perf_counter()
for _ in range(50):
    a.to(device=env.device, dtype=torch.float32).contiguous()
print(f"  actions.to().contiguous(): {1e6 * (time.perf_counter() - t0) / 50:.1f} us")
t0 = time.perf_counter()
for _ in range(50):
    env._rl_out()
print(f"  _rl_out(): {1e6 * (time.perf_counter() - t0) / 50:.1f} us")
torch.cuda.synchronize()

# 3. the timed region, K = 20, after 5 and after 400 warm-up steps
for wu in (5, 400):
    env2, step2 = make()
    for _ in range(wu):
        step2()
    el = timed_region(step2, 20, 1, dev, torch.cuda.synchronize)
    print(f"timed region K=20 after {wu} warm-up steps: {1e3 * el / 20:.2f} ms/step = {n * 20 / el:.3e} env-steps/s")
    del env2

# 4. clock or state: the same 5-warm-up form after 1 s of unrelated GPU work
#    (matmuls on other tensors; the env's state is that of step 5) and after
#    1 s idle
x = torch.randn(4096, 4096, device=dev)
for pre in ("busy", "idle"):
    env3, step3 = make()
    for _ in range(5):
        step3()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        if pre == "busy":
            y = x @ x
            torch.cuda.synchronize()
        else:
            time.sleep(0.01)
    el = timed_region(step3, 20, 1, dev, torch.cuda.synchronize)
    print(f"timed region K=20 after 5 warm-up steps and 1 s {pre}: {n * 20 / el:.3e} env-steps/s")
    del env3
