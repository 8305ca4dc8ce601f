"""Cost of the bias-free velocity iterations (developer tool): the task's step
time with sim.physx.num_velocity_iterations as configured and with 0, A/B
alternating, HIP events around 1000 steps.

    python scripts/dev/viters_cost.py [ThormangWalk|Gogoro] [num_envs]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import thormang_isaacgym_amd as tia  # noqa: E402


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "ThormangWalk"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    env = tia.make(seed=0, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
    sim = env.sim
    sp = sim.get_sim_params()
    vi0 = sp.velocity_iterations
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.rand(n, env.num_actions, device="cuda:0", generator=g) * 2 - 1 for _ in range(8)]

    def run(vi, steps=1000):
        sp.velocity_iterations = vi
        sim.set_sim_params(sp)
        for k in range(50):
            env.step(acts[k % 8])
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for k in range(steps):
            env.step(acts[k % 8])
        t1.record()
        torch.cuda.synchronize()
        return t0.elapsed_time(t1) / steps * 1000.0

    res = {vi0: [], 0: []}
    for _ in range(3):
        for vi in (vi0, 0):
            res[vi].append(run(vi))
    for vi, v in res.items():
        print(f"{task} {n} envs velocity_iterations={vi}: us/step " + " ".join(f"{x:.2f}" for x in v)
              + f"  (min {min(v):.2f})")
    print(f"{task}: velocity iterations cost {min(res[vi0]) - min(res[0]):.2f} us/step")


if __name__ == "__main__":
    main()
