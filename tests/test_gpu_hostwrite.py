"""Device memory the host writes (bcp_dev_alloc_hostwrite, the P role's rows
under BCP_FOLD_DEVICE_ROWS): host stores through the BAR are what the fold
kernels read -- also after the same rows were read by an earlier kernel and
rewritten (no stale line of the earlier use), for pitched and unaligned rows."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,length", [(3, 512 * 1024), (8, 1_048_573), (1, 17)])
def test_host_stores_reach_the_fold(engine, queue, n, length):
    pitch = (length + 255) & ~255
    rows = engine.alloc_hostwrite(n * pitch)
    out = engine.alloc(pitch)
    rng = np.random.default_rng(n * 7 + length)
    try:
        for rnd in range(4):
            data = rng.integers(0, 256, size=(n, length), dtype=np.uint8)
            for j in range(n):
                ctypes.memmove(rows + j * pitch, data[j].ctypes.data, length)
            if rnd % 2:  # the descriptor kernel over unaligned lengths
                queue.xor_stripes([(out, length, 0, n, 0)], [(rows + j * pitch, length) for j in range(n)])
            else:
                queue.xor_strided(out, pitch, rows, 0, pitch, 1, n, length)
            got = np.empty(length, np.uint8)
            queue.d2h(got, out, length)
            queue.sync()
            assert np.array_equal(got, np.bitwise_xor.reduce(data, axis=0)), rnd
    finally:
        queue.sync()
        engine.free(rows)
        engine.free(out)
