"""Developer micro-benchmark: compose_kernel duration vs the number of dirty
envs (run under rocprofv3 --kernel-trace --stats, or read the printed HIP-event
times of whole simulate() calls)."""
import sys

import torch

sys.path.insert(0, ".")
from thormang_isaacgym_amd import abi  # noqa: E402
from thormang_isaacgym_amd.sim import Sim, load_model  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "gogoro"
    n = 4096
    m = load_model(name)
    sp = abi.sim_params_from_cfg({"dt": 0.01, "substeps": 1, "gravity": [0, 0, -9.81]}, {}, n)
    s = Sim(m, sp, n, "cuda:0")
    s.root_state[:, 2] = 1.0
    s.simulate()
    torch.cuda.synchronize()
    import ctypes as C
    from thormang_isaacgym_amd import _lib
    L = _lib.lib()
    prof = hasattr(L, "tg_cprof_read")
    if prof:
        L.tg_cprof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]

    def cprof():
        b = (C.c_ulonglong * 8)()
        if prof:
            L.tg_cprof_read(b, 8)
        return list(b)

    for k in (0, 1, 16, 256, 4096):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = 0.0
        c0 = cprof()
        for _ in range(20):
            s.env_dirty[:k] = 1
            ev0.record()
            s.simulate()
            ev1.record()
            torch.cuda.synchronize()
            t += ev0.elapsed_time(ev1)
        c1 = cprof()
        per = [(b - a) / max(20 * k, 1) for a, b in zip(c0, c1)][:4]
        print(f"{name} dirty={k:5d}: simulate {t / 20 * 1e3:8.1f} us" +
              (f"   compose cycles/env: loads {per[0]:.0f} fk {per[1]:.0f} sums {per[2]:.0f} shapes {per[3]:.0f}"
               if prof else ""))


if __name__ == "__main__":
    main()
