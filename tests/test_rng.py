"""The product's random-number generator on the host (no GPU needed).

Every in-kernel draw of the task kernels (reset speed / yaw / Kd / seat offsets,
sensor noise, walk joint noise, pushes) is a Philox4x32-10 block
(csrc/tg_kernels.h ``philox``) fed to ``u01`` / ``gauss``.  The library exports
the same block function on the host (``tg_philox4x32_10``); it is pinned here
to the known-answer vectors published with Random123 (Salmon, Moraes, Dror,
Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11; file
``examples/kat_vectors``, rows ``philox4x32 10``), and to an independent
numpy restatement on random inputs.  The device copy is compared with the host
one in tests/test_gpu_rng.py."""
import ctypes as C
import os

import numpy as np
import pytest

# Random123 kat_vectors, philox4x32 10: ctr[4] key[2] -> out[4]
KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox_np(ctr, key):
    """Philox4x32-10 restated with numpy uint64 arithmetic (vectorised over rows)."""
    c = [np.asarray(x, np.uint64) for x in ctr]
    k0, k1 = (np.asarray(x, np.uint64) for x in key)
    M0, M1, W0, W1, MASK = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint64(0x9E3779B9), \
        np.uint64(0xBB67AE85), np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & MASK, p1 & MASK, ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & MASK,
             p0 & MASK]
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return np.stack(c, -1).astype(np.uint32)


def host_block(ctr, key):
    from thormang_isaacgym_amd import _lib
    out = (C.c_uint32 * 4)()
    _lib.lib().tg_philox4x32_10((C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), out)
    return tuple(int(x) for x in out)


def _need_lib():
    from thormang_isaacgym_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libtgsim.so not built")


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_numpy_restatement_matches_random123_kat(ctr, key, want):
    assert tuple(int(x) for x in philox_np(ctr, key)) == want


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_library_philox_matches_random123_kat(ctr, key, want):
    _need_lib()
    assert host_block(ctr, key) == want


def test_library_philox_matches_restatement_on_random_blocks():
    _need_lib()
    rs = np.random.default_rng(7)
    ctr = rs.integers(0, 2**32, (64, 4), dtype=np.uint64)
    key = rs.integers(0, 2**32, (64, 2), dtype=np.uint64)
    ref = philox_np(ctr.T, key.T)
    for i in range(64):
        assert host_block(tuple(int(x) for x in ctr[i]), tuple(int(x) for x in key[i])) == \
            tuple(int(x) for x in ref[i])
