"""Task registry (mirror of isaacgymenvs/tasks/__init__.py:54-77, restricted to
the tasks this build provides)."""
from .gogoro import Gogoro
from .thormang_walk import ThormangWalk

isaacgym_task_map = {
    "Gogoro": Gogoro,
    "ThormangWalk": ThormangWalk,
}
