"""GPU parity tests of the resident fold ring (bcp_ring_*, include/bcp.h):
stripes published from many threads into one launch that stays on the
device, every output byte against the oracle's xor_parity (the restatement
of task_processing.c:96-109, pinned to the reference's own function in
test_oracle_ref.py) on the zero-padded rows; the ring's lifecycle -- the
launch idling out and coming back, entries reused past the ring's size,
destroy with and without a live launch -- and its argument checks."""
import concurrent.futures as cf
import ctypes
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024


def host_view(addr, n):
    return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(addr))


def expect(oracle, chunks, out_len):
    """out_len bytes of the oracle's fold of the chunks, zero padded / cut."""
    n = len(chunks)
    data = np.zeros((n, max(out_len, 1)), dtype=np.uint8)
    for k, c in enumerate(chunks):
        m = min(len(c), out_len)
        data[k, :m] = c[:m]
    return oracle.xor_parity(data.reshape(-1), out_len, n)[:out_len]


class Arena:
    """Mapped pinned host memory carved into source and output blocks."""

    def __init__(self, eng, nbytes):
        self.eng, self.n = eng, nbytes
        self.base = eng.host_alloc(nbytes, mapped=True)
        self.view = host_view(self.base, nbytes)
        self.off = 0

    def take(self, n, align=16, skew=0):
        self.off = (self.off + align - 1) // align * align + skew
        assert self.off + n <= self.n
        a = self.base + self.off
        self.off += n
        return a

    def put(self, arr, align=16, skew=0):
        a = self.take(len(arr), align, skew)
        self.view[a - self.base:a - self.base + len(arr)] = arr
        return a

    def get(self, addr, n):
        return self.view[addr - self.base:addr - self.base + n].copy()

    def close(self):
        self.eng.host_free(self.base)


@pytest.fixture
def arena(engine):
    a = Arena(engine, 768 * MiB)
    yield a
    a.close()


def random_stripe(rng, arena, max_len, max_src=8):
    n = int(rng.integers(1, max_src + 1))
    lens = [int(rng.integers(0, max_len + 1)) for _ in range(n)]
    if rng.random() < 0.3:
        lens = [max_len] * n  # the uniform shape
    out_len = max(lens) if rng.random() < 0.7 else int(rng.integers(0, max_len + 1))
    chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
    aligned = rng.random() < 0.6
    srcs = [(arena.put(c, skew=0 if aligned else int(rng.integers(0, 16))), len(c)) for c in chunks]
    dst = arena.take(out_len, skew=0 if aligned else int(rng.integers(0, 16)))
    arena.view[dst - arena.base:dst - arena.base + out_len] = 0xA5
    return chunks, srcs, dst, out_len


def test_ring_folds_host_rows_from_many_threads(bcp, engine, arena, oracle):
    """The protocol's shape: rows in mapped host memory, one stripe per
    submission, 12 threads submitting and waiting at once."""
    rng = np.random.default_rng(7)
    cases = [random_stripe(rng, arena, int(rng.choice([4 * KiB, 64 * KiB, 512 * KiB, 1536 * KiB])))
             for _ in range(96)]
    ring = bcp.Ring(engine)
    try:
        def one(c):
            chunks, srcs, dst, out_len = c
            ring.wait(ring.submit(dst, out_len, srcs))
            return arena.get(dst, out_len)

        with cf.ThreadPoolExecutor(12) as ex:
            outs = list(ex.map(one, cases))
        for (chunks, _, _, out_len), got in zip(cases, outs):
            np.testing.assert_array_equal(got, expect(oracle, chunks, out_len))
        pieces, launches = ring.stats()
        assert pieces >= len(cases) and launches >= 1
    finally:
        ring.close()


def test_ring_wide_and_ragged_stripes(bcp, engine, arena, oracle):
    """Up to BCP_MAX_SOURCES sources, byte tails, empty sources, outputs
    shorter and longer than every source, several pieces per stripe."""
    rng = np.random.default_rng(11)
    ring = bcp.Ring(engine, workers=16)
    try:
        cases, handles = [], []
        for n, out_len, lens in [
            (56, 100 * KiB + 3, None),
            (13, 2 * MiB + 17, None),
            (3, 1 * MiB, [0, 0, 0]),
            (5, 700 * KiB, [1, 15, 16, 17, 700 * KiB + 9]),
            (2, 0, [10, 20]),
            (1, 1, [1]),
            (8, 3 * 512 * KiB, [512 * KiB] * 8),
        ]:
            lens = lens or [int(rng.integers(0, out_len + 2 * KiB)) for _ in range(n)]
            chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
            srcs = [(arena.put(c, skew=int(rng.integers(0, 16))), len(c)) for c in chunks]
            dst = arena.take(out_len, skew=int(rng.integers(0, 16)))
            cases.append((chunks, dst, out_len))
            handles.append(ring.submit(dst, out_len, srcs))
        for h in handles:
            ring.wait(h)
        for chunks, dst, out_len in cases:
            np.testing.assert_array_equal(arena.get(dst, out_len), expect(oracle, chunks, out_len))
    finally:
        ring.close()


def test_ring_device_memory_and_reuse_past_ring_size(bcp, engine, queue, oracle):
    """Sources and output in HBM; 1,300 tickets through 512 entries, each
    entry reused twice while later ones are in flight."""
    rng = np.random.default_rng(3)
    n, L, m = 3, 8 * KiB + 48, 1300
    src = rng.integers(0, 256, size=(m, n, L), dtype=np.uint8)
    d_src, d_out = engine.alloc(src.size), engine.alloc(m * L)
    ring = bcp.Ring(engine)
    try:
        queue.h2d(d_src, src)
        queue.sync()
        handles = [ring.submit(d_out + i * L, L, [(d_src + (i * n + k) * L, L) for k in range(n)])
                   for i in range(m)]
        assert all(ring.query(h) in (True, False) for h in handles[:4])
        for h in handles:
            ring.wait(h)
        out = np.empty(m * L, dtype=np.uint8)
        queue.d2h(out, d_out)
        queue.sync()
        want = np.bitwise_xor.reduce(src, axis=1).reshape(-1)
        np.testing.assert_array_equal(out, want)
        np.testing.assert_array_equal(out[:L], expect(oracle, list(src[0]), L))
        assert ring.stats()[0] == m
    finally:
        ring.close()
        engine.free(d_src)
        engine.free(d_out)


def test_ring_launch_idles_out_and_comes_back(bcp, engine, arena, oracle):
    """With a 2 ms idle limit the launch ends between bursts; the next
    submission (or a waiter) starts a new one from the first ticket the old
    one did not take, and nothing is folded twice or lost."""
    rng = np.random.default_rng(5)
    ring = bcp.Ring(engine, workers=8, idle_us=2000)
    try:
        for burst in range(4):
            cases = [random_stripe(rng, arena, 64 * KiB) for _ in range(10)]
            hs = [ring.submit(d, n, s) for _, s, d, n in cases]
            for h in hs:
                ring.wait(h)
            for chunks, _, d, n in cases:
                np.testing.assert_array_equal(arena.get(d, n), expect(oracle, chunks, n))
            time.sleep(0.03)
        pieces, launches = ring.stats()
        assert launches >= 4, (pieces, launches)
        # a waiter alone (no submit after the close) must also get its ticket
        chunks, srcs, d, n = random_stripe(rng, arena, 64 * KiB)
        h = ring.submit(d, n, srcs)
        while not ring.query(h):
            pass
        np.testing.assert_array_equal(arena.get(d, n), expect(oracle, chunks, n))
    finally:
        t0 = time.perf_counter()
        ring.close()
        assert time.perf_counter() - t0 < 2.0


def test_ring_destroy_paths_and_arguments(bcp, engine, arena):
    # never launched
    bcp.Ring(engine).close()
    # destroyed while its launch is live (default 5 ms idle): stops at once
    r = bcp.Ring(engine, idle_us=5_000_000)
    a = arena.put(np.arange(4096, dtype=np.uint8))
    d = arena.take(4096)
    r.wait(r.submit(d, 4096, [(a, 4096)]))
    t0 = time.perf_counter()
    r.close()
    assert time.perf_counter() - t0 < 1.0
    assert np.array_equal(arena.get(d, 4096), np.arange(4096, dtype=np.uint8))
    # argument checks
    r = bcp.Ring(engine)
    try:
        lib = bcp.lib()
        h = ctypes.c_uint64(0)
        so = (bcp.Source * 57)(*[bcp.Source(a, 16)] * 57)
        st = bcp.Stripe(d, 16, 0, 1, 1 << 20)  # window replay is not a ring stripe
        assert lib.bcp_ring_submit(r.h, ctypes.byref(st), so, ctypes.byref(h)) == -22
        st = bcp.Stripe(d, 16, 0, 57, 0)
        assert lib.bcp_ring_submit(r.h, ctypes.byref(st), so, ctypes.byref(h)) == -22
        st = bcp.Stripe(d, 256 * 512 * KiB, 0, 1, 0)
        assert lib.bcp_ring_submit(r.h, ctypes.byref(st), so, ctypes.byref(h)) == -22
        st = bcp.Stripe(d, 16, 0, 1, 0)
        bad = (bcp.Source * 1)(bcp.Source(0, 16))
        assert lib.bcp_ring_submit(r.h, ctypes.byref(st), bad, ctypes.byref(h)) == -22
        st = bcp.Stripe(0, 0, 0, 1, 0)  # empty output: nothing to wait for
        assert lib.bcp_ring_submit(r.h, ctypes.byref(st), so, ctypes.byref(h)) == 0
        r.wait(h.value)
        assert lib.bcp_ring_create(None, 0, 0, ctypes.byref(ctypes.c_void_p())) == -22
        assert lib.bcp_ring_create(engine.h, -1, 0, ctypes.byref(ctypes.c_void_p())) == -22
        assert r.stats() == (0, 0)
    finally:
        r.close()
