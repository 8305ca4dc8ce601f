"""Pin the paper-variant oracle (oracle/gogoro_paper_task.c) against fixtures
recorded from the reference's own gogoro_realistic_turning_sim_paper.py
(tests/golden/make_golden_paper.py): the oracle env replays the recorded
physics states and random draws and must reproduce every recorded buffer.  CPU only."""
import os

import numpy as np
import pytest

from tests.paper_harness import OraclePaper, fixture_cfg, switches_from
from thormang_isaacgym_amd.abi import TG_PROP_DAMPING, TG_PROP_EFFORT, TG_PROP_LOWER, TG_PROP_STIFFNESS, \
    TG_PROP_UPPER, TG_PROP_VELOCITY
from thormang_isaacgym_amd.tasks.gogoro_draws import RecordedDraws

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIXTURES = ("paper_steps.npz", "paper_falls.npz", "paper_steps_flags.npz")


def replay(f):
    src = RecordedDraws(f["draw_kind"], f["draw_size"], f["draw_vals"])
    sw = switches_from(f["flags"])
    cfg = fixture_cfg(f)
    orc = OraclePaper(cfg, src, sw)
    assert src.i == int(f["init_n_draws_init"])
    a = orc.a
    np.testing.assert_allclose(a["root"], f["init_root"], atol=1e-6)
    np.testing.assert_array_equal(a["dof_state"], f["init_dof"])
    for k in ("curent_speed", "steer_offsets", "steer_delay", "curent_speed_offset", "curent_imu_x_offset"):
        np.testing.assert_allclose(a[k], f["init_" + k], atol=2e-6, err_msg=k)
    dni = orc.model.dof_name_to_id()
    st, seat = dni["steering_joint"], [dni["base_x"], dni["base_y"], dni["base_z"]]
    err = {"obs": 0.0, "rew": 0.0}
    for t in range(f["actions"].shape[0]):
        orc.pre(f["actions"][t][:, 0])
        a["root"][:] = f["sim_root"][t]
        a["dof_state"][:] = f["sim_dof"][t]
        obs, rew, reset, to = orc.post()
        assert src.i == int(f["draw_end"][t]), t
        np.testing.assert_allclose(a["pos_target"], f["pos_target"][t], atol=1e-7, err_msg=f"pos_target {t}")
        np.testing.assert_array_equal(a["vel_target"], f["vel_target"][t])
        np.testing.assert_array_equal(reset, f["reset"][t], err_msg=f"reset step {t}")
        np.testing.assert_array_equal(to.astype(bool), f["time_outs"][t])
        np.testing.assert_array_equal(a["progress_buf"], f["progress"][t])
        err["obs"] = max(err["obs"], float(np.abs(obs - f["obs"][t]).max()))
        err["rew"] = max(err["rew"], float(np.abs(rew - f["rew"][t]).max()))
        for k in ("curent_command", "command_history", "yaw_command", "curent_speed", "steer_offsets",
                  "curent_speed_offset", "curent_imu_x_offset", "buffer_obs", "buffer_obs_noisy", "speed_no_noise"):
            np.testing.assert_allclose(a[k], f[k][t], atol=2e-5, err_msg=f"{k} step {t}")
        np.testing.assert_array_equal(a["steer_delay"], f["steer_delay"][t])
        np.testing.assert_allclose(a["perturbation"], f["perturbation"][t], atol=2e-5, err_msg=f"push {t}")
        np.testing.assert_allclose(a["root"], f["root_after"][t], atol=1e-6)
        np.testing.assert_array_equal(a["dof_state"], f["dof_after"][t])
        pr = a["dof_props"]
        for k, fld in (("steer_damping", TG_PROP_DAMPING), ("steer_stiffness", TG_PROP_STIFFNESS),
                       ("steer_effort", TG_PROP_EFFORT), ("steer_velocity", TG_PROP_VELOCITY)):
            np.testing.assert_allclose(pr[fld][:, st], f[k][t], rtol=1e-6, err_msg=f"{k} {t}")
        np.testing.assert_allclose(pr[TG_PROP_LOWER][:, seat], f["seat_lower"][t], atol=1e-7)
        np.testing.assert_allclose(pr[TG_PROP_UPPER][:, seat], f["seat_upper"][t], atol=1e-7)
    assert src.i == len(f["draw_kind"])
    return err


@pytest.mark.parametrize("name", FIXTURES)
def test_paper_oracle_replays_reference(name):
    f = np.load(os.path.join(GOLDEN, name))
    err = replay(f)
    print(name, err)
    assert err["obs"] < 2e-5 and err["rew"] < 2e-5, err
