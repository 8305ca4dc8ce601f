"""Domain-randomisation host logic (no GPU): the per-link mass scale the
library applies for IsaacGym's two DR operations (vec_task.py:538-768;
'scaling' m = m0 * s, 'additive' m = m0 + s), and the sampling semantics of
VecTask._sample (ranges, schedules) that every DR sample goes through."""
import torch

from thormang_isaacgym_amd.tasks.base.vec_task import VecTask, mass_scale


def test_mass_scale_scaling_is_the_sample():
    s = torch.tensor([[0.95, 1.05, 1.0]])
    assert torch.equal(mass_scale(s, "scaling", torch.tensor([2.0, 0.0, 5.0])), s)


def test_mass_scale_additive_adds_to_the_link_mass():
    m0 = torch.tensor([2.0, 0.5, 0.0])
    smp = torch.tensor([[0.1, -0.2, 0.3], [0.0, 0.25, 1.0]])
    sc = mass_scale(smp, "additive", m0)
    new_mass = sc * m0
    assert torch.allclose(new_mass[:, :2], m0[:2] + smp[:, :2])
    assert torch.equal(sc[:, 2], torch.ones(2))       # massless link keeps scale 1


class _Fake:
    device = "cpu"
    _sched = staticmethod(VecTask._sched)


def test_sample_uniform_scaling_range_and_schedule():
    f = _Fake()
    p = {"distribution": "uniform", "range": [0.95, 1.05], "operation": "scaling"}
    x = VecTask._sample(f, p, (20000,), 0)
    assert float(x.min()) >= 0.95 and float(x.max()) < 1.05
    assert abs(float(x.mean()) - 1.0) < 2e-3
    # linear schedule at step 0: scaling ranges collapse to 1
    p2 = dict(p, schedule="linear", schedule_steps=100)
    y = VecTask._sample(f, p2, (100,), 0)
    assert torch.allclose(y, torch.ones(100))
    z = VecTask._sample(f, p2, (20000,), 50)             # halfway: [0.975, 1.025]
    assert float(z.min()) >= 0.975 - 1e-6 and float(z.max()) <= 1.025 + 1e-6


def test_sample_gaussian_additive_moments():
    f = _Fake()
    p = {"distribution": "gaussian", "range": [0.5, 0.1], "operation": "additive"}
    x = VecTask._sample(f, p, (50000,), 0)
    assert abs(float(x.mean()) - 0.5) < 3e-3 and abs(float(x.std()) - 0.1) < 3e-3
