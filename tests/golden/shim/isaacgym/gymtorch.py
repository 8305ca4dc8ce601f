"""``gymtorch`` stand-in: tensors pass straight through (TEST INFRASTRUCTURE ONLY)."""


def unwrap_tensor(t):
    return t


def wrap_tensor(t):
    return t
