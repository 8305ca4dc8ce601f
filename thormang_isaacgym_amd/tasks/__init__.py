"""Task registry (mirror of isaacgymenvs/tasks/__init__.py:54-77, restricted to
the tasks this build provides)."""
from . import gogoro_paper
from .gogoro import Gogoro
from .thormang_walk import ThormangWalk

isaacgym_task_map = {
    "Gogoro": Gogoro,
    # tasks/gogoro_realistic_turning_sim_paper.py (not in the reference's map; cfg Gogoro_paper.yaml)
    "GogoroPaper": gogoro_paper.Gogoro,
    "ThormangWalk": ThormangWalk,
    "ThormangWalkDR": ThormangWalk,
}
