"""Device mapping of the reference's pipelines (vec_task.py:66-74), CPU only."""
import pytest
import torch

from thormang_isaacgym_amd.tasks.base.vec_task import pipeline_device


def test_gpu_pipeline_maps_to_the_sim_device():
    assert pipeline_device({"sim": {"use_gpu_pipeline": True}}, "cuda:3") == "cuda:3"


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU error")
def test_cpu_pipeline_without_gpu_raises_instead_of_falling_back():
    with pytest.raises(RuntimeError, match="no GPU"):
        pipeline_device({"sim": {"use_gpu_pipeline": False}}, "cpu")
