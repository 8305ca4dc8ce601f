"""GPU-vs-oracle harness for the Gogoro task path (test infrastructure).

``OracleGogoro`` is the CPU restatement of the whole env step: the task
oracle (oracle/gogoro_task.c) around the fp64 physics oracle
(oracle/physics_ref.c), driven exactly like the product ``Gogoro`` class.
Both sides take their random draws from identically seeded ``NumpyDraws``
sources in the reference's call order, so any difference is numerics."""
from __future__ import annotations

import ctypes as C

import numpy as np

from tests.oracle_lib import lib, physics_step, ptr
from thormang_isaacgym_amd import abi
from thormang_isaacgym_amd.cfg import load_task_cfg
from thormang_isaacgym_amd.model.urdf import Model
from thormang_isaacgym_amd.tasks.gogoro_cfg import ASSET_OPTIONS, env_origins, gogoro_params, initial_dof_props, \
    thormang_pose
from thormang_isaacgym_amd.tasks.gogoro_draws import post_draws, reset_draws


def maxerr(a, b):
    """max |a - b| over two arrays; inf when either holds a non-finite value
    (a NaN would otherwise drop out of every max() and comparison here, and
    a run where both sides blow up would pass)"""
    a, b = np.asarray(a), np.asarray(b)
    if not (np.isfinite(a).all() and np.isfinite(b).all()):
        return float("inf")
    return float(np.abs(a - b).max()) if a.size else 0.0


def maxrel(a, b):
    """max |a - b| / max(1, |b|): the error measure for unbounded
    coordinates (a continuous wheel's angle grows by tens of radians over
    1000 steps and carries the fp32 ulp of its magnitude)"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if not (np.isfinite(a).all() and np.isfinite(b).all()):
        return float("inf")
    return float((np.abs(a - b) / np.maximum(1.0, np.abs(b))).max()) if a.size else 0.0


class NumpyDraws:
    """DrawSource over a seeded numpy generator (U[0,1) and N(0,1), float32)."""

    def __init__(self, seed):
        self.rs = np.random.default_rng(seed)

    def uniform(self, n):
        return self.rs.random(n, dtype=np.float32)

    def normal(self, n):
        return self.rs.standard_normal(n, dtype=np.float32)


def parity_cfg(num_envs, max_steps=1000, freq=300, dr=False):
    """The Gogoro cfg of the parity runs.  dr=False turns the reference's
    randomisation off (both sides share one model); dr=True keeps it
    (gravity x U[0.95,1.05] every 600 frames, link masses x U[0.95,1.05],
    cfg/task/Gogoro.yaml randomization_params) and the oracle is handed the
    GPU env's draws (sync_dr)."""
    cfg = load_task_cfg("Gogoro", num_envs=num_envs)
    cfg["env"]["max_steps"] = max_steps
    cfg["noises"]["speed_freq_update"] = freq
    cfg["noises"]["yaw_freq_update"] = freq
    if not dr:
        cfg["task"]["randomization_params"] = {"frequency": 10 ** 9}
    return cfg


def load_gogoro_model():
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "thormang_isaacgym_amd", "model", "compiled", "gogoro.json")) as f:
        return Model.from_json(f.read())


class OracleGogoro:
    def __init__(self, cfg, draws, env_spacing=1.0, threads=8, spawn_z=None, precision="f64", fix_base=False):
        self.L = L = lib(precision)
        self.dr = {}   # per-env mass scale / friction / gravity injected from a GPU env (sync_dr)
        self.cfg = cfg
        self.src = draws
        self.threads = threads
        self.model = m = load_gogoro_model()
        self.n = n = cfg["env"]["numEnvs"]
        self.D = D = m.num_dof
        self.dni = m.dof_name_to_id()
        self.desc = abi.ModelDesc(m)
        self.sp = abi.sim_params_from_cfg(cfg["sim"], dict(ASSET_OPTIONS, fix_base_link=fix_base), n, env_spacing)
        self.p = gogoro_params(cfg, self.dni, n)
        z = lambda *s, dt=np.float32: np.zeros(s, dt)
        self.a = dict(obs_buf=z(n, 6), rew_buf=z(n), reset_buf=np.ones(n, np.int64), progress_buf=z(n, dt=np.int64),
                      timeout_buf=z(n, dt=np.uint8), action_history=z(n, 5), curent_command=z(n), yaw_command=z(n),
                      curent_speed=z(n), steer_offsets=z(n), imu_offsets=z(n), speed_offset=z(n),
                      config_vector=z(n, 5), buffer_obs=z(n, 1, 6), thormang_pose=thormang_pose(cfg, self.dni),
                      root_reset=z(n, 13), root=z(n, 13), dof_state=z(n * D, 2), pos_target=z(n, D),
                      vel_target=z(n, D), dof_props=initial_dof_props(m, cfg, n), env_dirty=z(n, dt=np.uint8))
        org = env_origins(n, env_spacing)
        a = self.a
        a["root"][:, 0:2] = org[:, 0:2]
        a["root"][:, 2] = 1.0
        a["root"][:, 6] = 1.0
        a["root_reset"][:] = a["root"]
        a["root_reset"][:, 7:13] = 0
        if spawn_z is not None:   # USE_TERAIN: per-env spawn heights in the reset template
            a["root_reset"][:, 2] = spawn_z
            self.p.terrain_spawn = 1
        self.b = abi.tg_gogoro_buffers(**{k: v.ctypes.data for k, v in a.items()})
        lo, hi = cfg["noises"]["speed_range"]
        a["curent_speed"][:] = np.float32(lo) + draws.uniform(n) * np.float32(hi - lo)
        rd = reset_draws(draws, np.arange(n), n)
        for e in range(n):
            L.oracle_gogoro_reset_env(C.byref(self.p), C.byref(self.b), e, ptr(np.ascontiguousarray(rd[e])))
        a["obs_buf"][:] = 0
        a["buffer_obs"][:] = 0

    def step(self, actions):
        a, n = self.a, self.n
        pre = self.src.normal(n)
        self.L.oracle_gogoro_pre_physics(C.byref(self.p), C.byref(self.b),
                                         ptr(np.ascontiguousarray(actions, np.float32)), ptr(pre))
        physics_step(self.desc, self.sp, a["root"], a["dof_state"], a["dof_props"], a["pos_target"], a["vel_target"],
                     threads=self.threads, L=self.L, **self.dr)
        ids = np.nonzero(a["reset_buf"])[0]
        rd, od, sd, yd = post_draws(self.src, ids, a["progress_buf"].copy(), self.p.speed_freq_update,
                                    self.p.yaw_freq_update)
        self.L.oracle_gogoro_post_physics(C.byref(self.p), C.byref(self.b), ptr(rd), ptr(od), ptr(sd), ptr(yd))
        return a["obs_buf"], a["rew_buf"], a["reset_buf"], a["timeout_buf"]


def make_gpu_gogoro(cfg, draws, env_spacing=1.0):
    from thormang_isaacgym_amd.tasks.gogoro import Gogoro

    class ReplayGogoro(Gogoro):
        draw_source = draws

    ReplayGogoro.env_spacing = env_spacing
    return ReplayGogoro(cfg, "cuda:0", "cuda:0", -1, True, False, False)


def balance_policy(obs):
    """A hand-tuned steering controller that keeps the scooter up (turn into
    the lean), so long parity runs are not dominated by fall timing."""
    roll, droll = obs[:, 0], obs[:, 1]
    return np.clip(4.0 * roll + 0.8 * droll, -1.0, 1.0)[:, None].astype(np.float32)


def brief(err):
    """The error dict without its per-step traces (keys starting with _)."""
    return {k: v for k, v in err.items() if not k.startswith("_")}


def within(err, key="obs", tol=1e-3, min_horizon=None):
    """The parity bar, north_star's: the GPU-vs-fp64-oracle error under
    ``tol`` = 1e-3 at every compared step.

    The one qualification is a FREE-RUNNING run that carries the rounding
    control (the fp32 build of the same oracle, stepped beside the fp64 one
    on the same inputs) and whose control itself leaves the band: its first
    departure, ``err["ctl_first_bad"]`` (obs or reward over ``tol`` or a
    reset flag changed), is the step from which fp32 rounding alone no longer
    determines the trajectory to 1e-3 (a falling humanoid).  The GPU is then
    held to ``tol`` at every step BEFORE that step (the per-step trace
    ``err["_<key>_t"]``) and nothing is asserted after it -- the control
    never raises the bar (the round-4 form, 2x the control's
    whole-run maximum, let a diverged control loosen it to 10).  Without a
    departure, or without a control, the whole run is held to ``tol``;
    teacher-forced runs never set a departure step.

    The shortened window has a floor: a control that departs
    before ``min_horizon`` steps (default min(100, the run's length)) fails
    the check outright, so an early control can never empty the comparison;
    a test that means to accept a shorter window passes ``min_horizon``
    explicitly.  ``err["ctl_first_bad"]`` is in every test's assert message."""
    h = err.get("ctl_first_bad")
    trace = err.get("_" + key + "_t")
    if h is None or trace is None:
        return err[key] < tol
    if min_horizon is None:
        min_horizon = min(100, len(trace))
    if h < min_horizon:
        return False
    return max(trace[:h]) < tol


def note_control(err, t, c_obs, c_rew, c_reset, o_obs, o_rew, o_reset, tol=1e-3):
    """The fp32 rounding control's step-t errors against the fp64 oracle
    (maxima in ``obs_f32`` / ``rew_f32``) and its first departure from the
    band, ``ctl_first_bad`` (``within``)."""
    ce = maxerr(c_obs, o_obs)
    cr = maxerr(c_rew, o_rew)
    err["obs_f32"] = max(err.get("obs_f32", 0.0), ce)
    err["rew_f32"] = max(err.get("rew_f32", 0.0), cr)
    same = bool(np.array_equal(c_reset, o_reset))
    err["ctl_reset_equal"] = err.get("ctl_reset_equal", True) and same
    if (ce > tol or cr > tol or not same) and "ctl_first_bad" not in err:
        err["ctl_first_bad"] = t


def tgs_configured(cfg):
    return int(cfg["sim"].get("physx", {}).get("solver_type", 1)) == 1


def gogoro_env_vs_oracle(num_envs=64, steps=20, seed=0, policy=None, max_steps=1000, dr=False, fix_base=False,
                         control=None, f32_ensemble=0):
    """Free-running GPU Gogoro env vs the oracle env on the same draws; with
    ``control`` (default: when the cfg asks for TGS) the fp32 oracle build
    runs the same free-running episode beside the fp64 one (``within``); with
    ``f32_ensemble`` = K also K fp32 builds whose root and joint state is
    moved by relative 1e-7 (about an fp32 ulp) after the first step, whose departure
    steps from fp64 (obs or reward over 1e-3, or a reset flag changed) are
    ``f32_departures`` (as walk_env_vs_oracle's)."""
    import torch
    from thormang_isaacgym_amd.tasks import gogoro as gmod
    cfg = parity_cfg(num_envs, max_steps=max_steps, dr=dr)
    saved, gmod.DEBUGFIXBASE = gmod.DEBUGFIXBASE, fix_base
    try:
        env = make_gpu_gogoro(cfg, NumpyDraws(seed))
    finally:
        gmod.DEBUGFIXBASE = saved
    orc = OracleGogoro(parity_cfg(num_envs, max_steps=max_steps, dr=dr), NumpyDraws(seed), fix_base=fix_base)
    if control is None:
        control = tgs_configured(cfg)
    ctl = OracleGogoro(parity_cfg(num_envs, max_steps=max_steps, dr=dr), NumpyDraws(seed), fix_base=fix_base,
                       precision="f32") if control else None
    f32s = [OracleGogoro(parity_cfg(num_envs, max_steps=max_steps, dr=dr), NumpyDraws(seed), fix_base=fix_base,
                         precision="f32") for k in range(f32_ensemble)]

    def perturb(fk, k):
        # (after the first step: every env starts with a reset, whose spawn
        # would overwrite a perturbation of the initial state)
        prs = np.random.default_rng(100 + k)
        for name in ("root", "dof_state"):
            x = fk.a[name]
            x[...] = (x * (1 + 1e-7 * prs.standard_normal(x.shape))).astype(x.dtype)
    err = {"obs": 0.0, "rew": 0.0, "reset_equal": True, "timeout_equal": True, "root": 0.0, "steps": steps,
           "resets": 0, "_obs_t": [], "_rew_t": []}
    if ctl is not None:
        err["obs_f32"] = err["rew_f32"] = 0.0
    if f32s:
        err["f32_departures"] = [None] * len(f32s)
    obs_np = orc.a["obs_buf"].copy()
    for t in range(steps):
        if dr:
            sync_dr(orc, env)
            if ctl is not None:
                sync_dr(ctl, env)
        act = policy(obs_np) if policy is not None else np.zeros((num_envs, 1), np.float32)
        obs_d, rew, reset, extras = env.step(torch.from_numpy(act).to("cuda:0"))
        o_obs, o_rew, o_reset, o_to = orc.step(act[:, 0])
        if ctl is not None:
            c_obs, c_rew, c_reset = ctl.step(act[:, 0])[:3]
            note_control(err, t, c_obs, c_rew, c_reset, o_obs, o_rew, o_reset)
        for k, fk in enumerate(f32s):
            if t == 1:
                perturb(fk, k)
            f_obs, f_rew, f_reset = fk.step(act[:, 0])[:3]
            dep = err["f32_departures"]
            if dep[k] is None and (maxerr(f_obs, o_obs) > 1e-3 or
                                   maxerr(f_rew, o_rew) > 1e-3 or not np.array_equal(f_reset, o_reset)):
                dep[k] = t
        g_obs = obs_d["obs"].cpu().numpy()
        e_obs = maxerr(g_obs, o_obs)
        e_rew = maxerr(rew.cpu().numpy(), o_rew)
        err["_obs_t"].append(e_obs)
        err["_rew_t"].append(e_rew)
        err["obs"] = max(err["obs"], e_obs)
        err["rew"] = max(err["rew"], e_rew)
        err["root"] = max(err["root"], maxerr(env.root_tensor.cpu().numpy(), orc.a["root"]))
        q_g, q_o = env.sim.dof_state.cpu().numpy()[:, 0], orc.a["dof_state"][:, 0]
        err["dof"] = max(err.get("dof", 0.0), maxerr(q_g, q_o))
        err["dof_rel"] = max(err.get("dof_rel", 0.0), maxrel(q_g, q_o))
        err["dof_abs_max"] = max(err.get("dof_abs_max", 0.0), float(np.abs(q_o).max()))
        if err["reset_equal"] and not np.array_equal(reset.cpu().numpy(), o_reset):
            err["reset_diff_step"] = t
        err["reset_equal"] &= bool(np.array_equal(reset.cpu().numpy(), o_reset))
        err["timeout_equal"] &= bool(np.array_equal(extras["time_outs"].cpu().numpy().astype(np.uint8), o_to))
        err["resets"] += int(o_reset.sum())
        if (e_obs >= 1e-3 or e_rew >= 1e-3) and "first_bad_step" not in err:
            err["first_bad_step"] = t
        obs_np = o_obs.copy()
    err["resets_seen"] = int(orc.a["progress_buf"].min())
    if dr:
        err["mass_scale_range"] = [float(env.sim.body_mass_scale.min()), float(env.sim.body_mass_scale.max())]
        err["gravity"] = list(env.sim.gravity)
    return err


def sync_oracle_from_gpu(orc, env):
    """Teacher forcing: copy every task/state buffer the GPU env shares with its
    kernels into the oracle env, so the next step starts from identical state."""
    for k, t in env._buf_tensors.items():
        if t is None or k not in orc.a:
            continue
        dst = orc.a[k]
        src = t.detach().cpu().numpy()
        dst[...] = src.reshape(dst.shape).astype(dst.dtype, copy=False)


def sync_dr(orc, env):
    """Domain randomisation: hand the GPU env's current per-env link mass
    scales, shape frictions and gravity (the values its DR sampling drew, from
    the Sim mirrors) to the oracle env, which then simulates the same
    randomised models."""
    sim = env.sim
    orc.dr = {"mass_scale": np.ascontiguousarray(sim.body_mass_scale.cpu().numpy(), np.float32),
              "mu": np.ascontiguousarray(sim.shape_friction.cpu().numpy(), np.float32),
              "gravity": np.asarray(sim.gravity, np.float32)}


def certify_discontinuity(orc, e, gpu_root, tol=1e-3, draws=48, seed=5):
    """Is env ``e``'s one-step GPU-vs-oracle disagreement a discontinuity of
    the restated physics that rounding alone crosses?  The oracle env (one
    that keeps its physics inputs, ``OracleWalk.replay_env``) steps the env
    again from ``draws`` inputs each moved by about one fp32 ulp (relative
    1.2e-7, random signs): if any replay lands within ``tol`` of the GPU's
    root state, the GPU's result is one the fp64 oracle itself produces from
    inputs indistinguishable in fp32, i.e. the step is bimodal at rounding
    level (round 6: a foot corner at the contact gate, PhysX's pair rule,
    that takes ~1 N s when present and none when absent).
    An env whose unperturbed replay already matches the GPU's root is not
    certified (its disagreement is elsewhere).  Returns (certified, the
    nearest replay's distance)."""
    if not hasattr(orc, "replay_env"):
        return False, float("inf")
    rs = np.random.default_rng(seed)
    root0, dof0 = orc.phys_inputs(e)
    if float(np.abs(orc.replay_env(e, root0, dof0) - gpu_root).max()) < tol:
        return False, 0.0   # the root agrees: whatever differs is not a jump of the physics
    best = float("inf")
    for _ in range(draws):
        r = (root0 * (1 + rs.choice([-1.0, 1.0], root0.shape) * 1.2e-7)).astype(np.float32)
        d = (dof0 * (1 + rs.choice([-1.0, 1.0], dof0.shape) * 1.2e-7)).astype(np.float32)
        best = min(best, float(np.abs(orc.replay_env(e, r, d) - gpu_root).max()))
        if best < tol:
            return True, best
    return False, best


def forced_step_errors(env, orc, act_fn, steps, act_to_orc=lambda a: a, ctl=None, certify=False):
    """1-step GPU-vs-oracle errors along a GPU trajectory (oracle re-synced from
    the GPU state before every step).  Returns max errors and exact-match flags;
    with ``ctl`` (the fp32 oracle build, re-synced alike) also its one-step
    errors against the fp64 oracle (``within``).

    ``certify`` (oracles with ``replay_env``): an env-step whose GPU result
    leaves 1e-3 of the oracle's is checked with ``certify_discontinuity``; a
    certified one is left out of the maxima and the reset comparison of that
    step and listed in ``err["certified"]`` (step, env, its error, the
    nearest perturbed replay's distance) -- an uncertified one counts in full."""
    import torch
    err = {"obs": 0.0, "rew": 0.0, "root": 0.0, "reset_equal": True, "timeout_equal": True, "steps": steps,
           "resets": 0, "certified": []}
    if ctl is not None:
        err["obs_f32"] = err["rew_f32"] = 0.0
    obs = orc.a["obs_buf"].copy()
    for t in range(steps):
        sync_oracle_from_gpu(orc, env)
        sync_dr(orc, env)
        if ctl is not None:
            sync_oracle_from_gpu(ctl, env)
            sync_dr(ctl, env)
        act = act_fn(obs)
        obs_d, rew, reset, extras = env.step(torch.from_numpy(act).to("cuda:0"))
        o_obs, o_rew, o_reset, o_to = orc.step(act_to_orc(act))
        if ctl is not None:
            c_obs, c_rew = ctl.step(act_to_orc(act))[:2]
            err["obs_f32"] = max(err["obs_f32"], maxerr(c_obs, o_obs))
            err["rew_f32"] = max(err["rew_f32"], maxerr(c_rew, o_rew))
        g_obs = obs_d["obs"].cpu().numpy()
        g_rew, g_root, g_reset = rew.cpu().numpy(), env.root_tensor.cpu().numpy(), reset.cpu().numpy()
        keep = np.ones(len(g_rew), bool)
        if certify:
            pe = np.maximum(np.abs(g_obs - o_obs).reshape(len(g_rew), -1).max(1),
                            np.maximum(np.abs(g_rew - o_rew), np.abs(g_root - orc.a["root"]).max(1)))
            for i in np.nonzero(~(pe < 1e-3) | (g_reset != o_reset))[0]:
                ok, dist = certify_discontinuity(orc, int(i), g_root[i])
                if ok:
                    keep[i] = False
                    err["certified"].append((t, int(i), float(pe[i]), dist))
        err["obs"] = max(err["obs"], maxerr(g_obs[keep], o_obs[keep]))
        err["rew"] = max(err["rew"], maxerr(g_rew[keep], o_rew[keep]))
        err["root"] = max(err["root"], maxerr(g_root[keep], orc.a["root"][keep]))
        err["reset_equal"] &= bool(np.array_equal(g_reset[keep], o_reset[keep]))
        err["timeout_equal"] &= bool(np.array_equal(extras["time_outs"].cpu().numpy().astype(np.uint8), o_to))
        err["resets"] += int(o_reset.sum())
        obs = g_obs
    return err


def gogoro_forced(num_envs=64, steps=1000, seed=0, max_steps=300, dr=False, policy=None, threads=8):
    """Teacher-forced Gogoro (the oracle re-synced from the GPU env before
    every step) under ``policy`` (default: the balance controller)."""
    cfg = parity_cfg(num_envs, max_steps=max_steps, dr=dr)
    env = make_gpu_gogoro(cfg, NumpyDraws(seed))
    orc = OracleGogoro(parity_cfg(num_envs, max_steps=max_steps, dr=dr), NumpyDraws(seed), threads=threads)
    ctl = OracleGogoro(parity_cfg(num_envs, max_steps=max_steps, dr=dr), NumpyDraws(seed), threads=threads,
                       precision="f32") if tgs_configured(cfg) else None
    err = forced_step_errors(env, orc, policy or balance_policy, steps, act_to_orc=lambda a: a[:, 0], ctl=ctl)
    if dr:
        err["gravity"] = list(env.sim.gravity)
        err["mass_scale_range"] = [float(env.sim.body_mass_scale.min()), float(env.sim.body_mass_scale.max())]
    return err


def gogoro_terrain(num_envs=64, steps=300, seed=0, max_steps=300, terrain_seed=5, forced=True):
    """Gogoro with USE_TERAIN: the GPU env builds the Perlin terrain from the
    CPU torch generator (seeded here), the oracle gets the same height samples,
    origin and friction, and the envs' terrain spawn heights."""
    import torch
    from tests.oracle_lib import set_heightfield
    from thormang_isaacgym_amd.tasks import gogoro as gmod
    torch.manual_seed(terrain_seed)
    saved, gmod.USE_TERAIN = gmod.USE_TERAIN, True
    try:
        env = make_gpu_gogoro(parity_cfg(num_envs, max_steps=max_steps), NumpyDraws(seed))
    finally:
        gmod.USE_TERAIN = saved
    t = env.terrain
    o = -float(env._terrain_start_mid)
    set_heightfield(t.heightsamples.cpu().numpy(), t.V_scale, t.H_scale, o, o, friction=0.98)
    try:
        orc = OracleGogoro(parity_cfg(num_envs, max_steps=max_steps), NumpyDraws(seed),
                           spawn_z=env.root_reset_tensor[:, 2].cpu().numpy())
        if forced:
            err = forced_step_errors(env, orc, balance_policy, steps, act_to_orc=lambda a: a[:, 0])
        else:
            # Free running until the first step whose reset masks differ.  Such a
            # step is accepted only as a threshold tie: every env that disagrees
            # has its clean roll within `tie` of the 0.30 fall threshold
            # (gogoro_new.py:671-676), i.e. inside the fp32-vs-fp64 tolerance.
            # The reset draws are consumed in env order, so after a tie the two
            # random streams desynchronise and the comparison stops there.
            tie = 1e-3
            err = {"obs": 0.0, "rew": 0.0, "root": 0.0, "reset_equal": True, "compared_steps": steps,
                   "tie_envs": [], "ties_within_tol": True}
            obs = orc.a["obs_buf"].copy()
            for k in range(steps):
                act = balance_policy(obs)
                obs_d, rew, reset, _ = env.step(torch.from_numpy(act).to("cuda:0"))
                o_obs, o_rew, o_reset, _ = orc.step(act[:, 0])
                r_g = reset.cpu().numpy()
                if not np.array_equal(r_g, o_reset):
                    bad = np.nonzero(r_g != o_reset)[0]
                    roll = np.abs(orc.a["buffer_obs"][bad, -1, 0])
                    err["reset_equal"] = False
                    err["tie_envs"] = bad.tolist()
                    err["tie_roll"] = roll.tolist()
                    err["ties_within_tol"] = bool(np.all(np.abs(roll - 0.30) < tie))
                    err["compared_steps"] = k
                    break
                err["obs"] = max(err["obs"], maxerr(obs_d["obs"].cpu().numpy(), o_obs))
                err["rew"] = max(err["rew"], maxerr(rew.cpu().numpy(), o_rew))
                err["root"] = max(err["root"], maxerr(env.root_tensor.cpu().numpy(), orc.a["root"]))
                obs = o_obs.copy()
        err["spawn_z_max"] = float(env.root_reset_tensor[:, 2].max())
        return err
    finally:
        set_heightfield(None)


def walk_forced(num_envs=32, steps=1000, seed=0, task="ThormangWalk", dr=False, control=False, solver_type=None):
    """Teacher-forced walk (the oracle re-synced from the GPU env before every
    step); with ``control`` the fp32 oracle build is re-synced and stepped
    beside the fp64 one (``within``)."""
    mk = lambda: walk_cfg(num_envs, task, dr=dr, solver_type=solver_type)
    env = make_gpu_walk(mk(), NumpyDraws(seed))
    orc = OracleWalk(mk(), NumpyDraws(seed))
    ctl = OracleWalk(mk(), NumpyDraws(seed), precision="f32") if control else None
    rs = np.random.default_rng(seed + 100)
    err = forced_step_errors(env, orc, lambda o: rs.uniform(-0.5, 0.5, (num_envs, orc.D)).astype(np.float32), steps,
                             ctl=ctl, certify=True)
    if dr:
        note_dr_ranges(err, env)
    return err


def note_dr_ranges(err, env):
    """The spread of the per-env mass scales and shape frictions the GPU env
    drew (and the oracle was handed, sync_dr): a DR run whose draws never
    left 1.0 would compare nothing."""
    sim = env.sim
    err["mass_scale_range"] = [float(sim.body_mass_scale.min()), float(sim.body_mass_scale.max())]
    err["friction_range"] = [float(sim.shape_friction.min()), float(sim.shape_friction.max())]


# ----------------------------------------------------------------------------- ThormangWalk
class OracleWalk:
    """CPU restatement of the ThormangWalk env step (oracle/walk_task.c around
    oracle/physics_ref.c), driven like thormang_isaacgym_amd.tasks.thormang_walk."""

    def __init__(self, cfg, draws, threads=8, precision="f64"):
        import math
        self.L = L = lib(precision)
        self.dr = {}
        from thormang_isaacgym_amd.sim import load_model
        from thormang_isaacgym_amd.tasks.thormang_walk import walk_asset_options, walk_dof_props, walk_model_name, \
            walk_params
        self.cfg, self.src, self.threads = cfg, draws, threads
        self.model = m = load_model(walk_model_name(cfg))
        env = cfg["env"]
        self.n = n = env["numEnvs"]
        self.D = D = m.num_dof
        self.desc = abi.ModelDesc(m)
        spacing = float(env.get("envSpacing", 1.0))
        self.sp = abi.sim_params_from_cfg(cfg["sim"], walk_asset_options(cfg), n, spacing,
                                          default_contact_offset=0.016)
        props, kp, default = walk_dof_props(m, cfg, n)
        dt = float(cfg["sim"]["dt"])
        self.p = walk_params(cfg, m, n, m.num_groups, dt, int(math.ceil(env.get("episodeLength_s", 20) / dt)),
                             float(env.get("clipActions", math.inf)), float(env.get("clipObservations", math.inf)),
                             kp, default, 42)
        z = lambda *s, dt=np.float32: np.zeros(s, dt)
        self.a = dict(obs_buf=z(n, 13 + 3 * D), rew_buf=z(n), reset_buf=np.ones(n, np.int64),
                      progress_buf=z(n, dt=np.int64), timeout_buf=z(n, dt=np.uint8), actions=z(n, D),
                      last_actions=z(n, D), commands=z(n, 3), root_reset=z(n, 13), root=z(n, 13),
                      dof_state=z(n * D, 2), pos_target=z(n, D), body_force=z(n, m.num_groups, 6),
                      env_dirty=z(n, dt=np.uint8))
        self.props = props
        org = env_origins(n, spacing)
        a = self.a
        a["root"][:, 0:2] = org[:, 0:2]
        a["root"][:, 2] = float(env.get("spawnHeight", 0.79))
        a["root"][:, 6] = 1.0
        a["root_reset"][:] = a["root"]
        self.b = abi.tg_walk_buffers(**{k: v.ctypes.data for k, v in a.items()})
        self.push = self.p.push_force > 0
        if not self.push:
            self.b.body_force = None
        for e in range(n):
            r = np.ascontiguousarray(draws.uniform(4 + 2 * D))
            L.oracle_walk_reset_env(C.byref(self.p), C.byref(self.b), e, ptr(r))
        # the GPU reset_idx kernel also observes (prog 0): mirror it through a no-reset post pass
        self._observe_only()

    def _observe_only(self):
        a = self.a
        saved = a["progress_buf"].copy()
        a["progress_buf"][:] = -1
        a["reset_buf"][:] = 0
        zeros = np.zeros((self.n, 3), np.float32)
        self.L.oracle_walk_post_physics(C.byref(self.p), C.byref(self.b), None, ptr(zeros))
        a["progress_buf"][:] = saved

    def phys_inputs(self, e):
        """Env e's root and dof state as the last step's physics started from."""
        return self._pin["root"][e].copy(), self._pin["dof"][e * self.D:(e + 1) * self.D].copy()

    def replay_env(self, e, root, dof, precision="f64"):
        """The last step's physics of env e alone from the given root / dof
        state (every other input as that step had it); returns the root after
        it (certify_discontinuity)."""
        pin, D = self._pin, self.D
        r, d = np.array(root[None], np.float32), np.array(dof, np.float32)   # (copies: stepped in place)
        dr = {k: (np.ascontiguousarray(v[e:e + 1]) if k != "gravity" else v) for k, v in pin["dr"].items()}
        physics_step(self.desc, self.sp, r, d, np.ascontiguousarray(self.props[:, e:e + 1, :]),
                     pin["pos_target"][e:e + 1].copy(), np.zeros((1, D), np.float32),
                     force=None if pin["force"] is None else pin["force"][e:e + 1].copy(), threads=1,
                     L=lib(precision), **dr)
        return r[0]

    def step(self, actions):
        a, n, D = self.a, self.n, self.D
        self.L.oracle_walk_pre_physics(C.byref(self.p), C.byref(self.b),
                                       ptr(np.ascontiguousarray(actions, np.float32)))
        force = a["body_force"] if self.push else None
        self._pin = {"root": a["root"].copy(), "dof": a["dof_state"].copy(), "pos_target": a["pos_target"].copy(),
                     "force": None if force is None else force.copy(), "dr": dict(self.dr)}
        physics_step(self.desc, self.sp, a["root"], a["dof_state"], self.props, a["pos_target"],
                     np.zeros((n, D), np.float32), force=force, threads=self.threads, L=self.L, **self.dr)
        ids = np.nonzero(a["reset_buf"])[0]
        self.reset_count = getattr(self, "reset_count", 0) + len(ids)
        rd = np.zeros((n, 4 + 2 * D), np.float32)
        for i in ids:
            rd[i] = self.src.uniform(4 + 2 * D)
        pd = self.src.uniform(3 * n).reshape(n, 3)
        self.L.oracle_walk_post_physics(C.byref(self.p), C.byref(self.b), ptr(rd), ptr(np.ascontiguousarray(pd)))
        return a["obs_buf"], a["rew_buf"], a["reset_buf"], a["timeout_buf"]


def walk_cfg(num_envs, task="ThormangWalk", dr=False, fix_base=False, spawn_height=None, solver_type=None):
    """Walk cfg of the parity runs: the task's own DR (mass, friction) off
    unless dr=True (then the oracle is handed the GPU env's draws, sync_dr);
    pushes follow the task cfg; ``solver_type`` overrides the cfg's."""
    cfg = load_task_cfg(task, num_envs=num_envs)
    if solver_type is not None:
        cfg["sim"]["physx"]["solver_type"] = int(solver_type)
    cfg["task"]["randomize"] = bool(dr)
    if fix_base:
        cfg["env"]["asset"] = dict(cfg["env"].get("asset", {}), fix_base_link=True)
    if spawn_height is not None:
        cfg["env"]["spawnHeight"] = float(spawn_height)
    return cfg


def walk_kneel_cfg(num_envs, whole_body=True, spawn_height=0.6):
    """A kneel-and-fall scenario for whole-body contact: the PD targets fold
    the knees to 1.6 rad with the hips straight, the humanoid spawns 0.6 m
    up in that pose and drops onto its shins, then tips onto its hands; the
    terminations are off so it stays down.  With the foot boxes alone
    (whole_body=False) the pelvis sinks through the floor."""
    cfg = walk_cfg(num_envs, spawn_height=spawn_height)
    cfg["env"]["asset"] = dict(cfg["env"].get("asset", {}), wholeBodyCollision=bool(whole_body))
    cfg["env"]["defaultJointAngles"] = {"l_leg_hip_p": 0.0, "l_leg_kn_p": 1.6, "l_leg_an_p": 0.0,
                                        "r_leg_hip_p": 0.0, "r_leg_kn_p": -1.6, "r_leg_an_p": 0.0}
    cfg["env"]["learn"]["terminationHeight"] = -10.0
    cfg["env"]["learn"]["terminationUp"] = -2.0
    return cfg


def walk_kneel_forced(num_envs=32, steps=200, seed=0, amp=0.2):
    """Teacher-forced whole-body kneel (walk_kneel_cfg) GPU vs oracle; also
    the lowest pelvis height the GPU env reached."""
    import torch
    env = make_gpu_walk(walk_kneel_cfg(num_envs), NumpyDraws(seed))
    orc = OracleWalk(walk_kneel_cfg(num_envs), NumpyDraws(seed))
    rs = np.random.default_rng(seed + 100)
    zmin = [float("inf")]

    def act_fn(obs):
        zmin[0] = min(zmin[0], float(env.root_tensor[:, 2].min()))
        return rs.uniform(-amp, amp, (num_envs, orc.D)).astype(np.float32)
    err = forced_step_errors(env, orc, act_fn, steps, certify=True)
    torch.cuda.synchronize()
    err["pelvis_zmin"] = min(zmin[0], float(env.root_tensor[:, 2].min()))
    err["shapes"] = len(env.model.shapes)
    return err


def make_gpu_walk(cfg, draws, torch_seed=0):
    """The GPU walk env, its task draws replayed from ``draws``.  The
    randomization_params samples (vec_task.apply_randomizations) come from
    torch's global generator, as in the reference: seeded here so a DR run
    is the same whatever ran before it in the process."""
    import torch
    from thormang_isaacgym_amd.tasks.thormang_walk import ThormangWalk
    torch.manual_seed(torch_seed)

    class ReplayWalk(ThormangWalk):
        draw_source = draws

    return ReplayWalk(cfg, "cuda:0", "cuda:0", -1, True, False, False)


def n_resets(orc):
    return getattr(orc, "reset_count", 0)


def perturbed_walk_oracle(cfg, seed, k, eps=1e-7, precision="f64"):
    """The oracle env (fp64, or the fp32 build) with its initial pelvis height
    and every joint position moved by +-eps (random signs, stream k): a
    rounding-level perturbation of the reference itself
    (scripts/dev/standing_chaos_cpu.py, scripts/dev/standing_fp32_ensemble.py)."""
    p = OracleWalk(cfg, NumpyDraws(seed), precision=precision)
    rs = np.random.default_rng(1000 + k)
    p.a["root"][:, 2] += (eps * rs.choice([-1.0, 1.0], p.n)).astype(np.float32)
    p.a["dof_state"][:, 0] += (eps * rs.choice([-1.0, 1.0], p.a["dof_state"].shape[0])).astype(np.float32)
    return p


def walk_env_vs_oracle(num_envs=32, steps=30, seed=0, task="ThormangWalk", dr=False, fix_base=False,
                       spawn_height=None, amp=0.3, control=False, solver_type=None, perturbed=0, f32_ensemble=0):
    """Free-running GPU walk env vs the oracle env on the same draws and
    actions U(-amp, amp) (amp 0: the PD-held default pose); with ``control``
    the fp32 oracle build runs the same episode beside the fp64 one
    (``within``); with ``perturbed`` = K also K fp64 runs from initial states
    perturbed by 1e-7 (``perturbed_walk_oracle``): ``pert_first_bad`` is the
    first step any of them leaves 1e-3 of the unperturbed reference -- the
    reference's own predictability horizon at that precision; with
    ``f32_ensemble`` = K also K fp32 builds perturbed by 1e-7 (below an fp32
    ulp of the joint positions: the same fp32 computation rounded
    differently), whose departure steps (obs or reward over 1e-3, or a reset
    flag changed) are ``f32_departures``.  Per-step
    maxima of the GPU's errors are kept in ``_obs_t`` / ``_rew_t``
    (``brief`` drops them for printing)."""
    import torch
    mk = lambda: walk_cfg(num_envs, task, dr=dr, fix_base=fix_base, spawn_height=spawn_height,
                          solver_type=solver_type)
    env = make_gpu_walk(mk(), NumpyDraws(seed))
    orc = OracleWalk(mk(), NumpyDraws(seed))
    ctl = OracleWalk(mk(), NumpyDraws(seed), precision="f32") if control else None
    perts = [perturbed_walk_oracle(mk(), seed, k) for k in range(perturbed)]
    f32s = [perturbed_walk_oracle(mk(), seed, 100 + k, precision="f32") for k in range(f32_ensemble)]
    rs = np.random.default_rng(seed + 100)
    err = {"obs": 0.0, "rew": 0.0, "reset_equal": True, "timeout_equal": True, "root": 0.0, "steps": steps,
           "_obs_t": [], "_rew_t": []}
    if ctl is not None:
        # the control's own departure from fp64: its reset flags, the first
        # step it leaves 1e-3; and the GPU's distance to the control itself
        err.update(obs_f32=0.0, rew_f32=0.0, ctl_reset_equal=True, gpu_vs_f32=0.0)
    err["obs0"] = maxerr(env.obs_buf.cpu().numpy(), orc.a["obs_buf"])
    for t in range(steps):
        if dr:
            for o in [orc] + ([ctl] if ctl is not None else []) + f32s:
                sync_dr(o, env)
        act = rs.uniform(-amp, amp, (num_envs, orc.D)).astype(np.float32)
        obs_d, rew, reset, extras = env.step(torch.from_numpy(act).to("cuda:0"))
        o_obs, o_rew, o_reset, o_to = orc.step(act)
        g_obs = obs_d["obs"].cpu().numpy()
        if ctl is not None:
            c_obs, c_rew, c_reset = ctl.step(act)[:3]
            note_control(err, t, c_obs, c_rew, c_reset, o_obs, o_rew, o_reset)
            err["gpu_vs_f32"] = max(err["gpu_vs_f32"], maxerr(g_obs, c_obs))
        for k, fk in enumerate(f32s):
            f_obs, f_rew, f_reset = fk.step(act)[:3]
            dep = err.setdefault("f32_departures", [None] * len(f32s))
            if dep[k] is None and (maxerr(f_obs, o_obs) > 1e-3 or
                                   maxerr(f_rew, o_rew) > 1e-3 or not np.array_equal(f_reset, o_reset)):
                dep[k] = t
        for k, pk in enumerate(perts):
            p_obs, _, p_reset = pk.step(act)[:3]
            dep = err.setdefault("pert_departures", [None] * len(perts))
            if dep[k] is None and (maxerr(p_obs, o_obs) > 1e-3 or
                                   not np.array_equal(p_reset, o_reset)):
                dep[k] = t
                err.setdefault("pert_first_bad", t)
        e_obs = maxerr(g_obs, o_obs)
        if e_obs > 1e-3 and "first_over_tol" not in err:
            err["first_over_tol"] = t
        e_rew = maxerr(rew.cpu().numpy(), o_rew)
        err["_obs_t"].append(e_obs)
        err["_rew_t"].append(e_rew)
        err["obs"] = max(err["obs"], e_obs)
        err["rew"] = max(err["rew"], e_rew)
        err["root"] = max(err["root"], maxerr(env.root_tensor.cpu().numpy(), orc.a["root"]))
        q_g, q_o = env.sim.dof_state.cpu().numpy()[:, 0], orc.a["dof_state"][:, 0]
        err["dof"] = max(err.get("dof", 0.0), maxerr(q_g, q_o))
        err["dof_rel"] = max(err.get("dof_rel", 0.0), maxrel(q_g, q_o))
        err["dof_abs_max"] = max(err.get("dof_abs_max", 0.0), float(np.abs(q_o).max()))
        r_g = reset.cpu().numpy()
        if err["reset_equal"] and not np.array_equal(r_g, o_reset):
            # the first reset-mask disagreement: the envs' termination margins
            # in the oracle (pelvis height and uprightness against the cfg's
            # thresholds, oracle/walk_task.c observe) -- a threshold tie when
            # each disagreeing env sits within 1e-3 of a threshold, i.e. the
            # comparison's own tolerance
            bad = np.nonzero(r_g != o_reset)[0]
            margin = np.minimum(np.abs(o_obs[bad, 0] - orc.p.termination_height),
                                np.abs(-o_obs[bad, 9] - orc.p.termination_up))
            err.update(reset_diff_step=t, reset_diff_envs=bad.tolist(),
                       reset_diff_margin=[float(x) for x in margin],
                       reset_diff_obs_err=maxerr(g_obs[bad], o_obs[bad]),
                       reset_diff_tie=bool(np.all(margin < 1e-3)))
        err["reset_equal"] &= bool(np.array_equal(r_g, o_reset))
        err["timeout_equal"] &= bool(np.array_equal(extras["time_outs"].cpu().numpy().astype(np.uint8), o_to))
        if (e_obs >= 1e-3 or e_rew >= 1e-3) and "first_bad_step" not in err:
            err["first_bad_step"] = t
    err["resets"] = int(n_resets(orc))
    err["min_height"] = float(orc.a["root"][:, 2].min())
    if dr:
        note_dr_ranges(err, env)
    return err
