"""Empty ``terrain_utils`` stand-in; the reference does ``from isaacgym.terrain_utils import *``
(``tasks/gogoro_new.py:731``). TEST INFRASTRUCTURE ONLY."""
