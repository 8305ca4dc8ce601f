"""Recorder stubs for the few ``gymapi`` names the reference task touches at import
or inside the methods the fixture generator drives (TEST INFRASTRUCTURE ONLY)."""
DOF_MODE_NONE, DOF_MODE_POS, DOF_MODE_VEL, DOF_MODE_EFFORT = 0, 1, 2, 3
SIM_PHYSX, SIM_FLEX = 0, 1
UP_AXIS_Y, UP_AXIS_Z = 0, 1


class _Any:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, name):
        return _Any()

    def __call__(self, *a, **k):
        return _Any()


Vec3 = Transform = PlaneParams = TriangleMeshParams = AssetOptions = SimParams = CameraProperties = _Any


def acquire_gym():
    return _Any()
