"""Edge cases of the batch shape on the GPU: env counts that do not fill a
workgroup (the step kernel runs 16 envs per workgroup and the tail lanes redo
the last env without storing), a single env, the largest batch, empty index
lists -- each checked against the oracle or against an invariant."""
import numpy as np
import pytest
import torch
from tests.gpu_harness import within

pytestmark = pytest.mark.gpu


def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


@pytest.mark.parametrize("n", [1, 13, 37])
def test_gpu_ragged_batches_gogoro_env_matches_oracle(n):
    _cuda()
    from tests.gpu_harness import balance_policy, gogoro_env_vs_oracle
    err = gogoro_env_vs_oracle(num_envs=n, steps=80, seed=50 + n, policy=balance_policy)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


@pytest.mark.parametrize("n", [1, 19])
def test_gpu_ragged_batches_walk_env_matches_oracle(n):
    _cuda()
    from tests.gpu_harness import walk_env_vs_oracle
    err = walk_env_vs_oracle(num_envs=n, steps=40, seed=60 + n)
    assert within(err) and within(err, "rew"), err
    assert err["reset_equal"] and err["timeout_equal"], err


@pytest.mark.parametrize("name", ["thormang", "gogoro"])
def test_gpu_tail_envs_equal_full_batch(name):
    """The same 21 env states stepped as a batch of 21 (a partial workgroup)
    and as the first 21 of a batch of 48: identical results, bit for bit --
    the tail lanes of a partial workgroup never store."""
    _cuda()
    from tests.test_rigid_body_states import random_state
    from thormang_isaacgym_amd import abi
    from thormang_isaacgym_amd.sim import Sim, load_model
    m = load_model(name)
    root, dof = random_state(m, 48, np.random.default_rng(8))
    root[:, 2] = 2.0                       # clear of the ground: no contact ordering effects
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 2, "gravity": [0, 0, -9.81]}, {}, 48, warn=False)
    out = []
    for n in (21, 48):
        s = Sim(m, sp, n, "cuda:0")
        s.root_state.copy_(torch.from_numpy(root[:n]))
        s.dof_state.copy_(torch.from_numpy(dof.reshape(48, -1)[:n].reshape(-1, 2)))
        s.env_dirty.fill_(1)
        s.refresh()
        for _ in range(10):
            s.simulate()
        torch.cuda.synchronize()
        out.append((s.root_state[:21].cpu(), s.dof_state.view(n, -1, 2)[:21].cpu()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_gpu_reset_idx_empty_and_full():
    _cuda()
    import thormang_isaacgym_amd as tia
    env = tia.make(seed=3, task="Gogoro", num_envs=64, sim_device="cuda:0", rl_device="cuda:0")
    before = env.root_tensor.clone()
    env.reset_idx(torch.zeros(0, dtype=torch.long, device="cuda:0"))   # no-op
    torch.cuda.synchronize()
    assert torch.equal(before, env.root_tensor)
    env.reset_idx(torch.arange(64, device="cuda:0"))
    torch.cuda.synchronize()
    assert torch.isfinite(env.root_tensor).all()
    assert float(env.root_tensor[:, 7:13].abs().max()) == 0.0        # every env re-spawned at rest
    assert int(env.progress_buf.abs().max()) == 0


def test_gpu_walk_32768_envs_runs():
    """The largest batch in the tests (2x BASELINE config 5's 16384): finite
    state, resets and timeouts behave, no tail issues."""
    _cuda()
    import thormang_isaacgym_amd as tia
    env = tia.make(seed=5, task="ThormangWalk", num_envs=32768, sim_device="cuda:0", rl_device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(2)
    for _ in range(30):
        obs, rew, reset, extras = env.step(torch.rand(32768, env.num_actions, device="cuda:0", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert torch.isfinite(obs["obs"]).all() and torch.isfinite(rew).all()
    assert obs["obs"].shape == (32768, env.num_obs)


def test_gpu_rb_forces_survive_a_declined_fused_walk_step():
    """apply_rigid_body_force_tensors, then tg_walk_step on a
    heightfield.  There is no fused walk instantiation on terrain, so the
    launcher declines (rc 1) and the call falls back to compose + step +
    post.  The pending per-link forces must still be reduced and act on that
    step: the result equals the separate calls (tg_walk_pre_physics +
    tg_simulate + tg_walk_post_physics) with the same forces, and differs from
    a step without them."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.tasks.base.vec_task import VecTask
    n = 64
    envs = [tia.make(seed=5, task="ThormangWalk", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
            for _ in range(3)]
    for env in envs:   # a heightfield below the plane: flat-ground physics, the HF kernel
        env.sim.set_heightfield(np.zeros((8, 8), np.float32), 1.0, 1.0, -4.0, -4.0, friction=1.0)
    L = envs[0].sim.L
    f = torch.zeros(n, L, 3, device="cuda:0")
    f[:, 0, 0] = 400.0   # a push on the pelvis (link 0)
    g = torch.Generator(device="cuda:0").manual_seed(2)
    for _ in range(3):
        a = (torch.rand(n, envs[0].num_dof, device="cuda:0", generator=g) * 2 - 1) * 0.2
        envs[0].sim.apply_rigid_body_force_tensors(f.view(-1, 3).contiguous())
        envs[0].step(a)
        envs[1].sim.apply_rigid_body_force_tensors(f.view(-1, 3).contiguous())
        VecTask.step(envs[1], a)
        envs[2].step(a)
    torch.cuda.synchronize()
    r0, r1, r2 = (e.root_tensor.clone() for e in envs)
    assert torch.isfinite(r0).all()
    assert float((r0 - r1).abs().max()) < 1e-5, float((r0 - r1).abs().max())
    assert float((r0[:, 7] - r2[:, 7]).abs().min()) > 1e-2   # the push acted


def _probe_env(case, n):
    """The env of one stale-LDS probe case: a task, or a task on a model /
    kernel variant -- ``+wb`` the whole-body walk model (thormang_wb: 8-env
    workgroups, the looped table fill), ``+hf`` the heightfield instantiation
    of the step kernel (the walk on a heightfield below the plane; Gogoro
    with USE_TERAIN, its Perlin trimesh)."""
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.cfg import load_task_cfg
    task, _, var = case.partition("+")
    cfg = load_task_cfg(task, num_envs=n)
    if var == "wb":
        cfg["env"]["asset"] = dict(cfg["env"].get("asset", {}), wholeBodyCollision=True)
    if var == "hf" and task == "Gogoro":
        from thormang_isaacgym_amd.tasks import gogoro as gmod
        saved, gmod.USE_TERAIN = gmod.USE_TERAIN, True
        try:
            return tia.make(seed=11, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
        finally:
            gmod.USE_TERAIN = saved
    env = tia.make(seed=11, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0", cfg=cfg)
    if var == "hf":
        env.sim.set_heightfield(np.full((16, 16), 0.01, np.float32), 1.0, 1.0, -8.0, -8.0, friction=1.0)
    return env


@pytest.mark.parametrize("task", ["Gogoro", "GogoroPaper", "ThormangWalk", "ThormangWalkDR", "ThormangWalk+wb",
                                  "ThormangWalk+hf", "Gogoro+hf"])
def test_gpu_steps_read_no_stale_lds(task):
    """No kernel of a step reads LDS it has not written this launch (round 3:
    the Woodbury update once multiplied an unwritten slot by zero, and a NaN
    left there by an earlier kernel poisoned whole envs): an env steps 40
    random actions; a second env from the same seed (tia.make re-seeds torch,
    so the DR draws repeat) steps them again with every CU's LDS filled with
    a NaN or FLT_MAX pattern (tg_debug_fill_lds) before every step, and the
    results must be bit-identical.  48 envs: a partial last workgroup.
    Round 5: also the whole-body model (whose looped
    table fill once left the env state unloaded, caught only by its kneel
    test) and the heightfield instantiations."""
    _cuda()
    n, steps = 48, 40
    g = torch.Generator(device="cuda:0").manual_seed(4)
    acts = [torch.rand(n, 64, device="cuda:0", generator=g) * 2 - 1 for _ in range(steps)]
    runs = []
    for fill in (False, True):
        env = _probe_env(task, n)
        out = []
        for t in range(steps):
            if fill:
                env.sim.debug_fill_lds(0x7FC00000 if t % 2 == 0 else 0x7F7FFFFF)
            o, r, d, _ = env.step(acts[t][:, :env.num_actions].contiguous())
            out.append((o["obs"].clone(), r.clone(), d.clone(), env.root_tensor.clone()))
        runs.append(out)
        del env
    for t, (a, b) in enumerate(zip(*runs)):
        assert all(torch.equal(x, y) for x, y in zip(a, b)), (task, t)
    assert torch.isfinite(runs[1][-1][0]).all()


def test_gpu_shared_cache_is_invisible_to_property_writes(monkeypatch):
    """The shared composite cache (every env reads env 0's composite block
    while all blocks are equal) must not change what a DOF property write
    does.  A ThormangWalk env starts uniform, steps, then has one
    env's stiffness changed through set_dof_properties_indexed, another env's
    damping written through the zero-copy dof_props view with no refresh, and
    a third env's stiffness through the view plus refresh; the states over the
    following steps must be bit-identical to a run with the cache off
    (TG_NO_SHARED_CACHE=1, read at sim creation), and differ from a run
    without the writes in exactly those envs."""
    _cuda()
    import thormang_isaacgym_amd as tia
    from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_STIFFNESS
    n, steps = 64, 30
    g = torch.Generator(device="cuda:0").manual_seed(9)
    acts = [torch.rand(n, 33, device="cuda:0", generator=g) * 0.6 - 0.3 for _ in range(steps)]
    runs = []
    for off, writes in (("0", True), ("1", True), ("0", False)):
        monkeypatch.setenv("TG_NO_SHARED_CACHE", off)
        env = tia.make(seed=13, task="ThormangWalk", num_envs=n, sim_device="cuda:0", rl_device="cuda:0")
        sim, out = env.sim, []
        for t in range(steps):
            if writes and t == 5:
                vals = sim.dof_props[TG_PROP_STIFFNESS].clone()
                vals[3] *= 0.5
                sim.set_dof_properties_indexed(TG_PROP_STIFFNESS, vals, torch.tensor([3], device="cuda:0"))
                sim.dof_props[TG_PROP_DAMPING, 7] *= 3.0          # view write, no refresh
            if writes and t == 12:
                sim.dof_props[TG_PROP_STIFFNESS, 11] *= 0.3       # view write + refresh
                sim.refresh()
            env.step(acts[t])
            out.append(torch.cat([sim.root_state, sim.dof_state.view(n, -1)], 1).clone())
        runs.append(out)
        del env
    for t, (a, b) in enumerate(zip(runs[0], runs[1])):
        assert torch.equal(a, b), t
    moved = (runs[0][-1] != runs[2][-1]).any(1).nonzero().flatten().tolist()
    assert {3, 7, 11} <= set(moved), moved


@pytest.mark.parametrize("task", ["Gogoro", "ThormangWalk", "GogoroPaper"])
def test_gpu_step_is_deterministic(task):
    """Two envs from one seed, stepped with the same actions, stay bitwise
    equal (observations, rewards, resets, root states) -- the step kernels'
    results do not depend on timing (no race between an env's lanes, no
    order-dependent atomics).  Round 5 used this to tell a rounding-sensitive
    step from a nondeterministic one."""
    _cuda()
    import thormang_isaacgym_amd as tia
    n = 1024
    envs = [tia.make(seed=5, task=task, num_envs=n, sim_device="cuda:0", rl_device="cuda:0") for _ in range(2)]
    g = torch.Generator(device="cuda:0").manual_seed(7)
    resets = 0
    for _ in range(80):
        a = torch.rand(n, envs[0].num_actions, device="cuda:0", generator=g) * 2 - 1
        (o0, r0, d0, _), (o1, r1, d1, _) = (e.step(a) for e in envs)
        assert torch.equal(o0["obs"], o1["obs"]) and torch.equal(r0, r1) and torch.equal(d0, d1), task
        assert torch.equal(envs[0].root_tensor, envs[1].root_tensor), task
        resets += int(d0.sum())
    if task != "GogoroPaper":   # (its committed cfg is the fixed-base one: no falls in 80 steps)
        assert resets > 0, task
