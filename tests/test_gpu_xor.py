"""GPU parity tests: every XOR entry point of libbcp.so (through the C ABI)
against the oracle restatement, the committed golden vectors and, at the
BASELINE sizes, size-independent properties (XOR-fold conservation, sampled
oracle stripes, rebuild round trip)."""
import concurrent.futures as cf
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))
KiB, MiB = 1024, 1024 * 1024


class Dev:
    """Scratch device allocations freed at test end."""

    def __init__(self, eng, q):
        self.eng, self.q, self.ptrs = eng, q, []

    def alloc(self, n):
        p = self.eng.alloc(max(n, 16))
        self.ptrs.append(p)
        return p

    def put(self, arr, pad=0):
        """Upload arr at byte offset `pad` inside a fresh allocation; returns device address."""
        arr = np.ascontiguousarray(arr, dtype=np.uint8)
        base = self.alloc(arr.size + pad + 16)
        if arr.size:
            self.q.h2d(base + pad, arr)
        return base + pad

    def get(self, ptr, n):
        out = np.empty(max(n, 1), dtype=np.uint8)
        if n:
            self.q.d2h(out, ptr, n)
        self.q.sync()
        return out[:n]

    def free(self):
        self.q.sync()
        for p in self.ptrs:
            self.eng.free(p)
        self.ptrs = []


@pytest.fixture
def dev(engine, queue):
    d = Dev(engine, queue)
    yield d
    d.free()


def gpu_stripes(dev, queue, stripes):
    """stripes: list of dict(chunks=[np arrays or None], out_len, window, pads) -> list of outputs."""
    descs, sources, outs = [], [], []
    for st in stripes:
        pads = st.get("pads") or [0] * len(st["chunks"])
        first = len(sources)
        for c, pad in zip(st["chunks"], pads):
            if c is None or len(c) == 0:
                sources.append((0, 0))
            else:
                sources.append((dev.put(c, pad), len(c)))
        dptr = dev.alloc(st["out_len"] + 32) + st.get("dst_pad", 0)
        outs.append((dptr, st["out_len"]))
        descs.append((dptr, st["out_len"], first, len(st["chunks"]), st.get("window", 0)))
    queue.xor_stripes(descs, sources)
    queue.sync()
    return [dev.get(p, n) for p, n in outs]


# --------------------------------------------------------------------------
# drop-in xor_parity (task_processing.c:96-109)
# --------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 13, 56])
@pytest.mark.parametrize("nbytes", [1, 7, 8, 9, 15, 16, 17, 4095, 65536, 524288, 524289])
def test_dropin_xor_parity(bcp, oracle, engine, n, nbytes):
    rng = np.random.default_rng(n * 1000003 + nbytes)
    data = rng.integers(0, 256, size=n * nbytes, dtype=np.uint8)
    dst = np.full(nbytes, 0xA5, dtype=np.uint8)
    bcp.xor_parity(dst, nbytes, data, n)
    assert np.array_equal(dst, oracle.xor_parity(data, nbytes, n))


@pytest.mark.parametrize("doff,soff", [(1, 3), (7, 0), (0, 15), (13, 9)])
def test_dropin_misaligned_host_buffers(bcp, oracle, engine, doff, soff):
    """The reference's callers pass data_a + src*buffer_size and a malloc'd
    P_block: any alignment.  The drop-in stages rows to 256-byte device
    pitch, so host buffers at odd addresses and bytes around the
    destination stay as they were."""
    rng = np.random.default_rng(doff * 31 + soff)
    for n, nb in ((3, 100003), (8, 4097), (1, 17)):
        sbuf = rng.integers(0, 256, size=n * nb + soff, dtype=np.uint8)
        dbuf = np.full(nb + doff + 16, 0x5A, dtype=np.uint8)
        data, dst = sbuf[soff:soff + n * nb], dbuf[doff:doff + nb]
        bcp.xor_parity(dst, nb, data, n)
        assert np.array_equal(dst, oracle.xor_parity(np.ascontiguousarray(data), nb, n))
        assert (dbuf[:doff] == 0x5A).all() and (dbuf[doff + nb:] == 0x5A).all()


def test_dropin_golden_edge_vectors(bcp, oracle, engine):
    for fx in GOLD["edge"]:
        if fx["kind"] != "xor_parity":
            continue
        data = oracle.kat1_data(fx["n"], fx["s"])
        dst = np.empty(fx["s"], dtype=np.uint8)
        bcp.xor_parity(dst, fx["s"], data, fx["n"])
        assert hashlib.sha256(dst.tobytes()).hexdigest() == fx["sha256"], fx


def test_dropin_kat1(bcp, oracle, engine):
    k = GOLD["survey_kats"]["KAT-1"]
    data = oracle.kat1_data(k["n"], k["s"])
    dst = np.full(k["s"], 7, dtype=np.uint8)
    bcp.xor_parity(dst, k["s"], data, k["n"])
    assert hashlib.sha256(dst.tobytes()).hexdigest() == k["sha256"]


def test_dropin_concurrent_lanes(bcp, oracle, engine):
    """Twelve lane threads (gen/main.c:821) calling the drop-in at once."""
    def lane(i):
        rng = np.random.default_rng(i)
        for it in range(5):
            n, nb = int(rng.integers(2, 10)), int(rng.integers(1, 300000))
            data = rng.integers(0, 256, size=n * nb, dtype=np.uint8)
            dst = np.empty(nb, dtype=np.uint8)
            bcp.xor_parity(dst, nb, data, n)
            if not np.array_equal(dst, oracle.xor_parity(data, nb, n)):
                return False
        return True
    with cf.ThreadPoolExecutor(12) as ex:
        assert all(ex.map(lane, range(12)))


# --------------------------------------------------------------------------
# uniform / strided fast path
# --------------------------------------------------------------------------
@pytest.mark.parametrize("nsrc", [1, 2, 3, 7, 8, 9, 13, 16, 17, 56])
@pytest.mark.parametrize("chunk", [16, 4096, 8192 + 16, 524288, 524289, 1000])
def test_uniform_vs_oracle(oracle, dev, queue, nsrc, chunk):
    nstripes = 3
    rng = np.random.default_rng(nsrc * 7 + chunk)
    data = rng.integers(0, 256, size=nstripes * nsrc * chunk, dtype=np.uint8)
    src = dev.put(data)
    dst = dev.alloc(nstripes * chunk)
    queue.xor_uniform(dst, src, nstripes, nsrc, chunk)
    out = dev.get(dst, nstripes * chunk)
    for s in range(nstripes):
        ref = oracle.xor_parity(data[s * nsrc * chunk:(s + 1) * nsrc * chunk], chunk, nsrc)
        assert np.array_equal(out[s * chunk:(s + 1) * chunk], ref), (s, nsrc, chunk)


def test_strided_layout(oracle, dev, queue):
    """Sources interleaved [k][s] instead of [s][k]; outputs at a padded pitch."""
    nstripes, nsrc, chunk = 5, 8, 65536
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, size=nsrc * nstripes * chunk, dtype=np.uint8)  # [k][s][chunk]
    src = dev.put(data)
    pitch = chunk + 4096
    dst = dev.alloc(nstripes * pitch)
    queue.xor_strided(dst, pitch, src, chunk, nstripes * chunk, nstripes, nsrc, chunk)
    out = dev.get(dst, nstripes * pitch)
    d = data.reshape(nsrc, nstripes, chunk)
    for s in range(nstripes):
        ref = np.bitwise_xor.reduce(d[:, s, :], axis=0)
        assert np.array_equal(out[s * pitch:s * pitch + chunk], ref)


@pytest.mark.parametrize("bpc,vecs", [(1, 1), (2, 4), (4, 2), (8, 1), (16, 4), (1, 8), (3, 8)])
def test_tuning_variants_agree(oracle, engine, dev, queue, bpc, vecs):
    nstripes, nsrc, chunk = 7, 8, 524288 + 4096
    rng = np.random.default_rng(bpc * 10 + vecs)
    data = rng.integers(0, 256, size=nstripes * nsrc * chunk, dtype=np.uint8)
    src = dev.put(data)
    dst = dev.alloc(nstripes * chunk)
    engine.tune(bpc, vecs)
    engine.option("desc_blocks_per_cu", bpc)
    engine.option("desc_vecs_per_thread", vecs)
    try:
        queue.xor_uniform(dst, src, nstripes, nsrc, chunk)
        out = dev.get(dst, nstripes * chunk)
        # variable-length path with the same tuning
        res = gpu_stripes(dev, queue, [dict(chunks=[data[:1000], data[5:70000], None], out_len=70000 - 5)])
    finally:
        engine.tune(0, 0)
        engine.option("desc_blocks_per_cu", 0)
        engine.option("desc_vecs_per_thread", 0)
    ref = np.bitwise_xor.reduce(data.reshape(nstripes, nsrc, chunk), axis=1).reshape(-1)
    assert np.array_equal(out, ref)
    assert np.array_equal(res[0], oracle.xor_padded_np([data[:1000], data[5:70000]]))


@pytest.mark.parametrize("vecs", [8, 4, 1])
@pytest.mark.parametrize("chunk", [1, 15, 17, 1000, 4095, 524289, 3145745])
@pytest.mark.parametrize("nsrc", [1, 3, 8, 13])
def test_strided_byte_tail(oracle, engine, dev, queue, vecs, chunk, nsrc):
    """Rows at a 256-byte pitch (the P role's window rows and the drop-in's
    device layout) with a chunk length that is not a multiple of 16: the
    streaming kernel's byte tail.  Bytes past each row's end stay untouched."""
    nstripes = 3
    pitch = (chunk + 255) // 256 * 256
    rng = np.random.default_rng(chunk * 31 + nsrc * 7 + vecs)
    rows = rng.integers(0, 256, size=(nstripes, nsrc, pitch), dtype=np.uint8)
    src = dev.put(rows.reshape(-1))
    out_pitch = pitch + 256
    dst = dev.put(np.full(nstripes * out_pitch, 0xA5, dtype=np.uint8))
    engine.tune(0, vecs)
    try:
        queue.xor_strided(dst, out_pitch, src, nsrc * pitch, pitch, nstripes, nsrc, chunk)
        out = dev.get(dst, nstripes * out_pitch).reshape(nstripes, out_pitch)
    finally:
        engine.tune(0, 0)
    for s in range(nstripes):
        ref = np.bitwise_xor.reduce(rows[s, :, :chunk], axis=0)
        assert np.array_equal(out[s, :chunk], ref), s
        assert (out[s, chunk:] == 0xA5).all(), s


@pytest.mark.parametrize("nstripes,want_u,nsrc", [(1, 2, 8), (2, 2, 8), (16, 4, 8), (128, 4, 8), (256, 8, 8),
                                                  (256, 4, 16), (300, 4, 12)])
def test_auto_tile_size_by_batch(engine, dev, queue, nstripes, want_u, nsrc):
    """Default tuning (vecs_per_thread 0): the streaming kernel's tile size is
    chosen per launch from the batch's tile count (U = 2 / 4 / 8 for 8 x
    512 KiB stripes at 15/16 of 256 CUs), strided and pointer-table forms
    alike, and every choice is bit-exact (checked on the device against a
    per-stripe reference fold by U = 1 launches).  Stripes wider than 8
    sources take U = 4."""
    chunk = 512 * KiB
    assert engine.option("vecs_per_thread") == 0
    cus, _ = engine.info()
    if cus != 256:
        pytest.skip("thresholds checked for 256 CUs")
    src = dev.alloc(nstripes * nsrc * chunk)
    queue.fill_synthetic(src, nstripes * nsrc * chunk, seed=nstripes)
    out = dev.alloc(nstripes * chunk)
    out_t = dev.alloc(nstripes * chunk)
    ref = dev.alloc(nstripes * chunk)
    queue.xor_uniform(out, src, nstripes, nsrc, chunk)
    queue.sync()
    assert engine.option("last_stream_vecs") == want_u
    queue.xor_stripes([(out_t + s * chunk, chunk, s * nsrc, nsrc, 0) for s in range(nstripes)],
                      [(src + (s * nsrc + k) * chunk, chunk) for s in range(nstripes) for k in range(nsrc)])
    queue.sync()
    assert engine.option("last_stream_vecs") == want_u
    engine.tune(0, 1)
    try:
        queue.xor_uniform(ref, src, nstripes, nsrc, chunk)
        queue.sync()
        assert engine.option("last_stream_vecs") == 1
    finally:
        engine.tune(0, 0)
    flag = dev.alloc(16)
    for got in (out, out_t):
        queue.compare(got, ref, nstripes * chunk, flag)
        assert int(dev.get(flag, 8).view("<u8")[0]) == 0
    # sampled stripe against numpy
    s = nstripes // 2
    data = dev.get(src + s * nsrc * chunk, nsrc * chunk).reshape(nsrc, chunk)
    assert np.array_equal(dev.get(out + s * chunk, chunk), np.bitwise_xor.reduce(data, axis=0))


@pytest.mark.parametrize("out_len", [1000, 524288 + 9, 65536 - 3])
def test_uniform_batch_with_byte_tail(oracle, dev, queue, out_len):
    """Rebuild shape with a length that is not a multiple of 16 (aligned
    sources, some longer than out_len): pointer-table streaming kernel."""
    rng = np.random.default_rng(out_len)
    n = 8
    stripes, refs = [], []
    for _ in range(5):
        lens = [out_len + int(rng.integers(0, 40)) for _ in range(n)]
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        stripes.append(dict(chunks=chunks, out_len=out_len))
        refs.append(np.bitwise_xor.reduce(np.stack([c[:out_len] for c in chunks]), axis=0))
    outs = gpu_stripes(dev, queue, stripes)
    for o, r in zip(outs, refs):
        assert np.array_equal(o, r)


def test_work_queue_back_to_back_and_two_queues(oracle, engine, dev, queue):
    """The work-queue counter is monotone per queue: many launches in a row on
    one queue, a second queue interleaved, and a change of tile size and grid
    (different tile and failing-grab counts per launch) and back must all cover
    every tile exactly once."""
    rng = np.random.default_rng(77)
    q2 = engine.queue()
    try:
        jobs = []
        for i in range(24):
            n, chunk, ns = int(rng.integers(1, 10)), 16 * int(rng.integers(1, 40000)), int(rng.integers(1, 6))
            data = rng.integers(0, 256, size=ns * n * chunk, dtype=np.uint8)
            src, dst = dev.put(data), dev.alloc(ns * chunk)
            queue.sync()  # the upload ran on `queue`; q2's kernel must see it
            q = queue if i % 3 else q2
            if i == 10:
                engine.tune(3, 2)
            if i == 14:
                engine.tune(0, 0)
            q.xor_uniform(dst, src, ns, n, chunk)
            jobs.append((data, dst, ns, n, chunk))
        q2.sync()
        for data, dst, ns, n, chunk in jobs:
            out = dev.get(dst, ns * chunk)
            ref = np.bitwise_xor.reduce(data.reshape(ns, n, chunk), axis=1).reshape(-1)
            assert np.array_equal(out, ref)
    finally:
        engine.tune(0, 0)
        q2.close()


@pytest.mark.parametrize("seed", range(4))
def test_uniform_descriptor_batch_takes_pointer_table_path(oracle, dev, queue, seed):
    """Rebuild shape: every stripe has the same nsrc and out_len and every
    source is at least out_len long (longer sources are truncated) -> the
    streaming kernel's pointer-table form; results identical to the oracle."""
    rng = np.random.default_rng(300 + seed)
    n = int(rng.integers(1, 10))
    out_len = 16 * int(rng.integers(1, 50000))
    stripes, refs = [], []
    for _ in range(int(rng.integers(1, 9))):
        lens = [out_len + 16 * int(rng.integers(0, 3)) for _ in range(n)]
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        stripes.append(dict(chunks=chunks, out_len=out_len))
        refs.append(oracle.xor_padded_np([c[:out_len] for c in chunks]))
    for o, r in zip(gpu_stripes(dev, queue, stripes), refs):
        assert np.array_equal(o, r)


# --------------------------------------------------------------------------
# descriptor path: variable lengths, padding, alignment, windows, rebuild
# --------------------------------------------------------------------------
@pytest.fixture(params=["args", "general"])
def desc_path(request, engine):
    """Small descriptor batches through the kernel-argument form
    (xor_desc_args, desc_args_max 4) and through desc_tiles + xor_desc (0)."""
    prev = engine.option("desc_args_max")
    engine.option("desc_args_max", 16 if request.param == "args" else 0)
    yield request.param
    engine.option("desc_args_max", prev)


@pytest.mark.parametrize("seed", range(8))
def test_descriptor_mixed_lengths_and_alignment(oracle, dev, queue, seed, desc_path):
    rng = np.random.default_rng(100 + seed)
    stripes, refs = [], []
    for _ in range(int(rng.integers(1, 12))):
        n = int(rng.integers(1, 10))
        lens = [int(x) for x in rng.integers(0, 300000, size=n)]
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        pads = [int(x) for x in rng.integers(0, 16, size=n)]
        m = max(lens)
        stripes.append(dict(chunks=chunks, out_len=m, pads=pads, dst_pad=int(rng.integers(0, 16))))
        refs.append(np.frombuffer(oracle.gen_parity_file(chunks)[8 * n:], np.uint8))
    outs = gpu_stripes(dev, queue, stripes)
    for o, r in zip(outs, refs):
        assert np.array_equal(o, r)


@pytest.mark.parametrize("vecs", [16, 8, 4, 2, 1])
def test_descriptor_grouped_tiles(oracle, engine, dev, queue, vecs, desc_path):
    """Staircase lengths whose covering sets hold for many consecutive
    subtiles: every grouped-tile shape (1 source x 2..8 subtiles, 2 x 2..4,
    3 x 2, 4 x 2), their boundaries with plain and partial tiles, the last
    partial output tile, misaligned sources and outputs."""
    T = 256 * vecs * 16
    rng = np.random.default_rng(900 + vecs)
    stripes, refs = [], []
    shapes = [[9 * T], [9 * T, 1 * T], [5 * T, 4 * T + 3], [6 * T, 6 * T, 2 * T + 17],
              [3 * T, 3 * T, 3 * T, 1 * T], [4 * T, 4 * T, 4 * T, 4 * T, 1 * T + 5],
              [17 * T + 9, 12 * T, 7 * T, 3 * T, T // 2, 0], [2 * T, 2 * T, 2 * T, 2 * T, 2 * T]]
    for lens in shapes:
        for jitter in (0, 1):
            ls = [L + (int(rng.integers(0, 40)) if jitter and L else 0) for L in lens]
            chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in ls]
            pads = [int(x) for x in rng.integers(0, 16, size=len(ls))] if jitter else None
            stripes.append(dict(chunks=chunks, out_len=max(ls), pads=pads, dst_pad=3 * jitter))
            refs.append(oracle.xor_padded_np(chunks))
    engine.option("desc_vecs_per_thread", vecs)
    try:
        outs = gpu_stripes(dev, queue, stripes)
        # the same stripes a few at a time: small batches (the args form when on)
        outs4 = []
        for i in range(0, len(stripes), 3):
            outs4 += gpu_stripes(dev, queue, stripes[i:i + 3])
    finally:
        engine.option("desc_vecs_per_thread", 0)
    for i, (o, o4, r) in enumerate(zip(outs, outs4, refs)):
        assert np.array_equal(o, r), i
        assert np.array_equal(o4, r), i


@pytest.mark.parametrize("nstripes,nsrc", [(1, 1), (1, 8), (2, 5), (4, 8), (16, 8), (17, 8), (3, 9), (12, 7)])
def test_small_batches_in_kernel_arguments(oracle, engine, dev, queue, nstripes, nsrc, desc_path):
    """Batches of at most 16 stripes and 128 sources (<= 8 per stripe) travel
    in the kernel arguments; 17 stripes or 9 sources take the general path.
    Mixed lengths (zero padding, byte tails, a zero-length source), unsorted
    input order, misaligned sources and outputs, every auto tile size."""
    rng = np.random.default_rng(31 * nstripes + nsrc)
    for scale in (40_000, 600_000, 3_000_000):
        stripes, refs = [], []
        for _ in range(nstripes):
            lens = [int(x) for x in rng.integers(0, scale, size=nsrc)]
            if nsrc > 2:
                lens[1] = 0
            chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
            pads = [int(x) for x in rng.integers(0, 16, size=nsrc)]
            stripes.append(dict(chunks=chunks, out_len=max(lens) + int(rng.integers(0, 3)), pads=pads,
                                dst_pad=int(rng.integers(0, 16))))
            ref = np.zeros(stripes[-1]["out_len"], np.uint8)
            for c in chunks:
                ref[:len(c)] ^= c
            refs.append(ref)
        outs = gpu_stripes(dev, queue, stripes)
        for i, (o, r) in enumerate(zip(outs, refs)):
            assert np.array_equal(o, r), (scale, i)


@pytest.mark.parametrize("side", [1, 0])
def test_large_mixed_batch_side_stream_tiles(oracle, engine, dev, queue, side):
    """A batch large enough for desc_tiles to run on the side stream (>= 2 x
    grid tiles; side 1), or one past the argument form but below that (side 0:
    desc_tiles in line), submitted twice back to back (the second desc_tiles
    overlaps the first fold, on another ring slot's records): both outputs
    exact."""
    rng = np.random.default_rng(77 + side)
    nstripes, top = (60, 4 * MiB) if side else (20, 256 * KiB)
    stripes, refs = [], []
    for _ in range(nstripes):
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(top), size=8))]
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        stripes.append(dict(chunks=chunks, out_len=max(lens)))
        refs.append(oracle.xor_padded_np(chunks))
    a = gpu_stripes(dev, queue, stripes)
    assert engine.option("last_desc_form") == 1
    b = gpu_stripes(dev, queue, stripes)
    for i, (x, y, r) in enumerate(zip(a, b, refs)):
        assert np.array_equal(x, r) and np.array_equal(y, r), i


def test_reused_tile_records_follow_data_and_table_changes(oracle, engine, dev, queue):
    """desc_reuse_records (the desc_tiles A/B option): a batch resubmitted with
    identical tables on a ring slot folds from that slot's records -- the
    records hold addresses, so new input bytes are still folded -- and any
    change of the tables (here an output length) makes records afresh."""
    rng = np.random.default_rng(313)
    stripes, chunks_all = [], []
    for _ in range(60):
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
        chunks_all.append([rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens])
    descs, sources, outs = [], [], []
    for chunks in chunks_all:
        first = len(sources)
        for c in chunks:
            sources.append((dev.put(c), len(c)))
        m = max(len(c) for c in chunks)
        dptr = dev.alloc(m + 32)
        outs.append((dptr, m))
        descs.append((dptr, m, first, len(chunks), 0))
    prev = engine.option("desc_reuse_records")
    engine.option("desc_reuse_records", 1)
    try:
        for rnd in range(10):  # 4 ring slots: from the 5th launch on, records are reused
            if rnd == 7:  # new bytes in one source: the reused records must fold them
                chunks_all[3][2] = rng.integers(0, 256, size=len(chunks_all[3][2]), dtype=np.uint8)
                queue.h2d(sources[3 * 8 + 2][0], chunks_all[3][2])
            d = list(descs)
            if rnd == 9:  # a changed table: out_len of stripe 5 shortened
                dptr, m, first, n, w = d[5]
                d[5] = (dptr, m - 4097, first, n, w)
            for o, n in outs:
                queue.memset(o, 0xA5, n)
            queue.xor_stripes(d, sources)
            queue.sync()
            for i, (o, n) in enumerate(outs):
                n_i = d[i][1]
                ref = oracle.xor_padded_np(chunks_all[i])[:n_i]
                assert np.array_equal(dev.get(o, n_i), ref), (rnd, i)
    finally:
        engine.option("desc_reuse_records", prev)


def test_reused_tile_records_never_follow_a_uniform_batch_on_the_slot(oracle, engine, dev, queue):
    """desc_reuse_records with device-resident tables: a uniform batch that
    took the same ring slot in between (it uploads its own tables over the
    slot's) must make the descriptor batch stage and cut its tables afresh,
    even though the descriptor tables are byte-identical to that slot's last
    descriptor batch (stale tables reused)."""
    rng = np.random.default_rng(515)
    chunks_all = [[rng.integers(0, 256, size=int(x), dtype=np.uint8)
                   for x in rng.integers(70_000, 300_000, size=6)] for _ in range(24)]
    descs, sources, outs = [], [], []
    for chunks in chunks_all:
        first = len(sources)
        for c in chunks:
            sources.append((dev.put(c), len(c)))
        m = max(len(c) for c in chunks)
        dptr = dev.alloc(m + 32)
        outs.append((dptr, m))
        descs.append((dptr, m, first, len(chunks), 0))
    # a uniform batch of 64 stripes x 8 x 64 KiB (pointer tables > table_host_max: uploaded)
    C, NS, NU = 64 * KiB, 8, 64
    ubuf = rng.integers(0, 256, size=NU * NS * C, dtype=np.uint8)
    usrc = dev.put(ubuf)
    uout = dev.alloc(NU * C)
    ustripes = [(uout + s * C, C, s * NS, NS, 0) for s in range(NU)]
    usources = [(usrc + (s * NS + k) * C, C) for s in range(NU) for k in range(NS)]
    keys = ("desc_reuse_records", "desc_table_host_max")
    prev = [engine.option(k) for k in keys]
    engine.option("desc_reuse_records", 1)
    engine.option("desc_table_host_max", 0)  # descriptor tables read from the slot's device copy
    try:
        for rnd in range(3):
            for o, n in outs:
                queue.memset(o, 0xA5, n)
            queue.xor_stripes(descs, sources)  # slot s (rnd > 0: the same tables as last time on s)
            queue.sync()
            for i, (o, n) in enumerate(outs):
                assert np.array_equal(dev.get(o, n), oracle.xor_padded_np(chunks_all[i])), (rnd, i)
            for _ in range(7):  # slots s+1 .. s+3, s (overwritten), s+1 .. s+3
                queue.xor_stripes(ustripes, usources)
            queue.sync()
            got = dev.get(uout, NU * C)
            for s_ in (0, NU - 1):
                ref = np.bitwise_xor.reduce(ubuf[s_ * NS * C:(s_ + 1) * NS * C].reshape(NS, C), axis=0)
                assert np.array_equal(got[s_ * C:(s_ + 1) * C], ref), (rnd, s_)
    finally:
        for k, v in zip(keys, prev):
            engine.option(k, v)


@pytest.mark.parametrize("n", [9, 12, 20, 56])
def test_descriptor_wide_stripes(oracle, dev, queue, n):
    """Stripes wider than a tile record holds (> 8 sources reaching into a
    tile, up to MAX_STORAGE_TARGETS - 1 + parity): mixed lengths,
    misaligned sources and output, zero-length and equal-length sources."""
    rng = np.random.default_rng(700 + n)
    stripes, refs = [], []
    for _ in range(3):
        lens = [int(x) for x in rng.integers(0, 200_000, size=n)]
        lens[0] = lens[1] = max(lens)  # ties
        lens[2] = 0
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        pads = [int(x) for x in rng.integers(0, 16, size=n)]
        stripes.append(dict(chunks=chunks, out_len=max(lens), pads=pads, dst_pad=int(rng.integers(0, 16))))
        refs.append(oracle.xor_padded_np(chunks))
    # uniform lengths too (a 16-multiple out_len with one short source keeps
    # the batch off the pointer-table fast path)
    lens = [65536] * n
    lens[-1] = 65536 - 48
    chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
    stripes.append(dict(chunks=chunks, out_len=65536))
    refs.append(oracle.xor_padded_np(chunks))
    outs = gpu_stripes(dev, queue, stripes)
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o, r), i


def test_golden_gen_files_on_gpu(oracle, dev, queue):
    for fx in GOLD["edge"]:
        if fx["kind"] != "gen_file":
            continue
        lens, W = fx["lens"], fx.get("window", 0)
        chunks = [oracle.synthetic(L, 1000 + k) for k, L in enumerate(lens)]
        m = max(lens)
        window = W if (W and m > W) else 0
        out = gpu_stripes(dev, queue, [dict(chunks=chunks, out_len=m, window=window)])[0]
        hdr = np.array(lens, dtype="<u8").tobytes()
        assert hashlib.sha256(hdr + out.tobytes()).hexdigest() == fx["sha256"], fx


def test_survey_kats_on_gpu(oracle, dev, queue):
    for name in ("KAT-2", "KAT-3", "KAT-4"):
        k = GOLD["survey_kats"][name]
        chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(k["lens"])]
        m = max(k["lens"])
        window = oracle.WINDOW if m > oracle.WINDOW else 0
        out = gpu_stripes(dev, queue, [dict(chunks=chunks, out_len=m, window=window)])[0]
        hdr = np.array(k["lens"], dtype="<u8").tobytes()
        assert hashlib.sha256(hdr + out.tobytes()).hexdigest() == k["sha256"], name


@pytest.mark.parametrize("args_max", [16, 0])
@pytest.mark.parametrize("knob,value", [("vecs_per_thread", v) for v in (1, 2, 4, 8)] +
                         [("desc_vecs_per_thread", v) for v in (1, 2, 4, 8, 16)])
def test_kernel_forms_agree(oracle, engine, dev, queue, knob, value, args_max):
    """Every instantiated tile size of both kernels -- xor_stream<8,U> and its
    register-budget form at U = 8 (strided and pointer table, full and partial
    tiles), xor_desc<U> and the rolling-window xor_desc_p<8|16, 5>, through
    desc_tiles (args_max 0) or the argument form -- gives the oracle's bytes on
    descriptor tiles with 1..8 covering sources."""
    rng = np.random.default_rng(value * 7 + len(knob) + args_max)
    nstripes, nsrc = 5, 8
    default = engine.option(knob)
    engine.option(knob, value)
    engine.option("desc_args_max", args_max)
    try:
        res = {}
        for chunk in (512 * KiB, 512 * KiB + 4096 + 16):
            data = rng.integers(0, 256, size=nstripes * nsrc * chunk, dtype=np.uint8)
            src = dev.put(data)
            dst = dev.alloc(nstripes * chunk)
            queue.xor_uniform(dst, src, nstripes, nsrc, chunk)
            ref = np.bitwise_xor.reduce(data.reshape(nstripes, nsrc, chunk), axis=1).reshape(-1)
            assert np.array_equal(dev.get(dst, nstripes * chunk), ref), chunk
            # pointer-table form (uniform descriptor batch)
            dst2 = dev.alloc(nstripes * chunk)
            queue.xor_stripes([(dst2 + s * chunk, chunk, s * nsrc, nsrc, 0) for s in range(nstripes)],
                              [(src + (s * nsrc + k) * chunk, chunk) for s in range(nstripes) for k in range(nsrc)])
            assert np.array_equal(dev.get(dst2, nstripes * chunk), ref), chunk
        shapes = [[300000] * 8, [300000] * 7 + [5], [200000, 150000, 140000, 70000, 66000, 65536, 1, 0],
                  [int(x) for x in rng.integers(1, 300000, size=8)], [131072, 131072, 40000]]
        stripes = [dict(chunks=[rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens], out_len=max(lens))
                   for lens in shapes]
        outs = gpu_stripes(dev, queue, stripes)
        if knob == "desc_vecs_per_thread":
            form = engine.option("last_desc_form")
            assert form == (1 if args_max == 0 else 2)  # (the argument form runs U = 16 as 8)
            assert engine.option("last_desc_vecs") == (value if form == 1 else min(value, 8))
    finally:
        engine.option(knob, default)
        engine.option("desc_args_max", 16)
    for o, st in zip(outs, stripes):
        assert np.array_equal(o, oracle.xor_padded_np(st["chunks"]))


@pytest.mark.parametrize("host_max", [0, 1 << 24])
def test_table_residency(oracle, engine, dev, queue, host_max):
    """Descriptor tables read by the kernels from pinned host memory
    (table_host_max / desc_table_host_max at 16 MiB) or copied to the device
    first (0): same bytes for every tile kind -- plain, grouped, partial,
    wide (12 sources), window replay through the general path (window not a
    tile multiple) -- and for a uniform batch (pointer-table xor_stream)."""
    rng = np.random.default_rng(host_max + 5)
    W = 64 * KiB + 16
    shapes = [[300000, 70000, 1, 0, 150001, 299999, 65536, 17],
              [int(x) for x in rng.integers(1, 200000, size=12)],
              [3 * W + 5, W, W - 1, 17],
              [524288] * 8]
    stripes, refs = [], []
    for i, lens in enumerate(shapes):
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        if i == 2:
            stripes.append(dict(chunks=chunks, out_len=max(lens), window=W))
            refs.append(np.frombuffer(oracle.gen_parity_file(chunks, window=W)[8 * len(lens):], dtype=np.uint8))
        else:
            stripes.append(dict(chunks=chunks, out_len=max(lens)))
            refs.append(oracle.xor_padded_np(chunks))
    uniform = [dict(chunks=[rng.integers(0, 256, size=4096, dtype=np.uint8) for _ in range(8)], out_len=4096)
               for _ in range(3)]
    engine.option("table_host_max", host_max)
    engine.option("desc_table_host_max", host_max)
    try:
        outs = gpu_stripes(dev, queue, stripes)
        outs_u = gpu_stripes(dev, queue, uniform)
    finally:
        engine.option("table_host_max", 4096)
        engine.option("desc_table_host_max", 128 * 1024)
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o, r), i
    for o, st in zip(outs_u, uniform):
        assert np.array_equal(o, oracle.xor_padded_np(st["chunks"]))


@pytest.mark.parametrize("lens", [[10485760, 26214405], [26214405, 1, 15 * MiB + 3], [21 * MiB, 0, 10 * MiB + 17]])
def test_window_replay_random_data(oracle, dev, queue, lens):
    rng = np.random.default_rng(sum(lens))
    chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
    ref = oracle.gen_parity_file(chunks)[8 * len(lens):]
    out = gpu_stripes(dev, queue, [dict(chunks=chunks, out_len=max(lens), window=oracle.WINDOW)])[0]
    assert out.tobytes() == ref


@pytest.mark.parametrize("vecs", [16, 8, 4, 1])
@pytest.mark.parametrize("window", [64 * 1024, 64 * 1024 + 16, 4 * 1024 * 1024])
def test_window_replay_tiles(oracle, engine, dev, queue, vecs, window):
    """Replay stripes (max_cs > window) folded as plain tiles with remapped
    source addresses when the window is a multiple of the tile size, through
    the general path when it is not (64 KiB + 16): eight sources around window
    boundaries, misaligned sources and output, a wide (10-source) stripe,
    rebuild-style truncation (out_len shorter than the longest source)."""
    rng = np.random.default_rng(window + vecs)
    W = window
    stripes, refs = [], []
    shapes = [[3 * W + 5, W, W - 1, 2 * W + 16, 17, 0, W + W // 2, 3 * W],
              [4 * W - 3, 4 * W - 3, W // 3, 2 * W, 2 * W + 1, 3 * W + 100, 5, 4 * W - 16, 7, 2 * W - 9],
              [2 * W + 1, 1]]
    for ls in shapes:
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in ls]
        pads = [int(x) for x in rng.integers(0, 16, size=len(ls))]
        ref = np.frombuffer(oracle.gen_parity_file(chunks, window=W)[8 * len(ls):], np.uint8)
        out_len = max(ls)
        stripes.append(dict(chunks=chunks, out_len=out_len, window=W, pads=pads, dst_pad=5))
        refs.append(ref)
        cut = out_len - W // 2 - 3  # truncated output (rebuild of a shorter victim)
        stripes.append(dict(chunks=chunks, out_len=cut, window=W, pads=pads))
        refs.append(ref[:cut])
    engine.option("desc_vecs_per_thread", vecs)
    try:
        outs = gpu_stripes(dev, queue, stripes)
    finally:
        engine.option("desc_vecs_per_thread", 0)
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o, r), i


@pytest.mark.parametrize("seed", range(6))
def test_rebuild_truncates_to_victim(oracle, dev, queue, seed):
    """Rebuild (task_processing.c:146-174,228-230): survivors + parity body,
    output truncated to header[victim]; max_cs from the header."""
    rng = np.random.default_rng(200 + seed)
    n = int(rng.integers(2, 9))
    lens = [int(x) for x in rng.integers(1, 600000, size=n)]
    chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
    pf = oracle.gen_parity_file(chunks)
    v = int(rng.integers(0, n))
    survivors = [c for i, c in enumerate(chunks) if i != v]
    body = np.frombuffer(pf[8 * n:], np.uint8)
    out = gpu_stripes(dev, queue, [dict(chunks=survivors + [body], out_len=lens[v])])[0]
    assert out.tobytes() == chunks[v].tobytes()
    assert out.tobytes() == oracle.rebuild_chunk(pf, survivors, v)


def test_empty_and_degenerate_stripes(oracle, dev, queue):
    a = np.arange(100, dtype=np.uint8)
    outs = gpu_stripes(dev, queue, [
        dict(chunks=[a], out_len=0),                 # nothing to write
        dict(chunks=[None, None], out_len=64),       # unreadable sources -> zeros
        dict(chunks=[a, a], out_len=100),            # cancels
        dict(chunks=[a], out_len=37),                # truncated copy
        dict(chunks=[], out_len=20),                 # no sources -> zeros
    ])
    assert outs[0].size == 0
    assert not outs[1].any() and outs[1].size == 64
    assert not outs[2].any()
    assert np.array_equal(outs[3], a[:37])
    assert not outs[4].any()


def test_invalid_descriptors_rejected(bcp, dev, queue):
    with pytest.raises(bcp.BcpError):
        queue.xor_stripes([(dev.alloc(64), 64, 0, 3, 0)], [(dev.alloc(64), 64)])   # sources out of range
    with pytest.raises(bcp.BcpError):
        queue.xor_stripes([(dev.alloc(64), 64, 0, 1, 7)], [(dev.alloc(64), 64)])   # window % 16
    with pytest.raises(bcp.BcpError):
        queue.xor_stripes([(dev.alloc(64), 64, 0, 1, 0)], [(0, 64)])               # null source
    queue.sync()


# --------------------------------------------------------------------------
# synthetic data / fold / compare utilities
# --------------------------------------------------------------------------
@pytest.mark.parametrize("n,off", [(1, 0), (17, 0), (4096, 8), (100003, 3), (1 << 20, 16)])
def test_fill_synthetic_matches_oracle(oracle, dev, queue, n, off):
    p = dev.alloc(n + 16)
    queue.fill_synthetic(p, n, 77, off)
    assert np.array_equal(dev.get(p, n), oracle.synthetic(n, 77, off))


def test_fold_and_compare(dev, queue):
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, size=1000003, dtype=np.uint8)
    b = a.copy()
    b[[0, 17, 999999, 1000002]] ^= 0x5A
    pa, pb = dev.put(a), dev.put(b)
    res = dev.alloc(32)
    queue.xor_fold(pa, a.size, res)
    fold = dev.get(res, 16)
    ref = np.zeros(16, np.uint8)
    for i in range(16):
        ref[i] = np.bitwise_xor.reduce(a[i::16])
    assert np.array_equal(fold, ref)
    queue.compare(pa, pb, a.size, res)
    assert int(dev.get(res, 8).view("<u8")[0]) == 4


# --------------------------------------------------------------------------
# BASELINE sizes: config 2 (gen) and config 3 (rebuild), 12,500 stripes of
# 8 x 512 KiB device-resident, and config 4's per-GPU shard (1,000,000 chunks
# over 8 GPUs = 15,625 stripes, 61 GiB of chunks + parity + rebuild buffers
# ~84 GiB on one GPU) -- size-independent properties
# --------------------------------------------------------------------------
@pytest.mark.parametrize("nstripes", [12500, 15625], ids=["config2-3", "config4-shard"])
def test_config2_and_config3_full_size(oracle, dev, queue, nstripes):
    nsrc, chunk = 8, 512 * KiB
    total = nstripes * nsrc * chunk
    src = dev.alloc(total)
    par = dev.alloc(nstripes * chunk)
    reb = dev.alloc(nstripes * chunk)
    res = dev.alloc(64)
    queue.fill_synthetic(src, total, 1)
    queue.memset(par, 0xA5, nstripes * chunk)  # no stale parity from an earlier test can pass
    queue.xor_uniform(par, src, nstripes, nsrc, chunk)
    # (1) XOR-fold conservation: fold(parity) == fold(all sources)
    queue.xor_fold(par, nstripes * chunk, res)
    queue.xor_fold(src, total, res + 16)
    f = dev.get(res, 32)
    assert np.array_equal(f[:16], f[16:]) and f[:16].any()
    # (2) sampled stripes against the oracle
    rng = np.random.default_rng(2)
    for s in [0, nstripes - 1] + [int(x) for x in rng.integers(0, nstripes, size=6)]:
        data = dev.get(src + s * nsrc * chunk, nsrc * chunk)
        assert np.array_equal(data, oracle.synthetic(nsrc * chunk, 1, s * nsrc * chunk))
        assert np.array_equal(dev.get(par + s * chunk, chunk), oracle.xor_parity(data, chunk, nsrc))
    # (3) config 3: rebuild target 3 of every stripe from 7 survivors + parity
    victim = 3
    stripes, sources = [], []
    for s in range(nstripes):
        first = len(sources)
        for k in range(nsrc):
            if k != victim:
                sources.append((src + (s * nsrc + k) * chunk, chunk))
        sources.append((par + s * chunk, chunk))
        stripes.append((reb + s * chunk, chunk, first, nsrc, 0))
    queue.xor_stripes(stripes, sources)
    # gather the original victims with a 1-source strided XOR (a copy), then
    # compare all 6.1 GiB on the device
    gathered = dev.alloc(nstripes * chunk)
    queue.xor_strided(gathered, chunk, src + victim * chunk, nsrc * chunk, chunk, nstripes, 1, chunk)
    queue.compare(reb, gathered, nstripes * chunk, res)
    bad = int(dev.get(res, 8).view("<u8")[0])
    assert bad == 0


# Documented engine knobs (include/bcp.h): defaults, valid values round-trip,
# invalid values are refused with -EINVAL and leave the knob unchanged.
KNOBS = {
    "blocks_per_cu": (1, [1, 2, 32], [0, 33]),
    "vecs_per_thread": (0, [0, 1, 2, 4, 8], [3, 16]),
    "desc_blocks_per_cu": (0, [0, 1, 32], [-1, 33]),
    "desc_vecs_per_thread": (0, [0, 1, 2, 4, 8, 16], [3, 32]),
    "desc_args_max": (16, [0, 1, 16], [-1, 17]),
    "stream_grid": (0, [0, 1, 65536], [-1, 65537]),
    "desc_grid": (0, [0, 7], [-1]),
    "contiguous_alloc": (0, [0, 1], [2]),
    "table_host_max": (4096, [0, 1 << 24], [-1, (1 << 24) + 1]),
    "desc_table_host_max": (128 * 1024, [0, 1 << 24], [-1]),
    "host_registered": (1, [0, 1], [2]),
    "desc_reuse_records": (0, [0, 1], [2, -1]),
}


@pytest.mark.parametrize("key", sorted(KNOBS))
def test_engine_knobs(bcp, engine, key):
    default, good, bad = KNOBS[key]
    assert engine.option(key) == default, key
    try:
        for v in good:
            assert engine.option(key, v) == v
        for v in bad:
            with pytest.raises(bcp.BcpError):
                engine.option(key, v)
            assert engine.option(key) == good[-1]
    finally:
        engine.option(key, default)
    assert engine.option(key) == default


def test_unknown_knob_refused(bcp, engine):
    with pytest.raises(bcp.BcpError):
        engine.option("no_such_knob", 1)
    with pytest.raises(bcp.BcpError):
        engine.option("no_such_knob")


@pytest.mark.parametrize("vecs", [0, 1, 8])
@pytest.mark.parametrize("nsrc", [1, 2, 3, 4])
def test_narrow_stripes_multi_tile_grabs(engine, dev, queue, nsrc, vecs):
    """Stripes of 1-4 sources take two tiles per work-queue grab: every tile
    folded exactly once (odd and even tile counts, full and partial last
    tiles), strided and pointer-table forms."""
    rng = np.random.default_rng(nsrc * 10 + vecs)
    engine.tune(0, vecs)
    try:
        for nstripes, chunk in ((37, 512 * KiB), (5, 3 * 32 * KiB + 48), (1, 16)):
            data = rng.integers(0, 256, size=nstripes * nsrc * chunk, dtype=np.uint8)
            src = dev.put(data)
            dst = dev.alloc(nstripes * chunk)
            queue.xor_uniform(dst, src, nstripes, nsrc, chunk)
            ref = np.bitwise_xor.reduce(data.reshape(nstripes, nsrc, chunk), axis=1).reshape(-1)
            assert np.array_equal(dev.get(dst, nstripes * chunk), ref), (nstripes, chunk)
            dst2 = dev.alloc(nstripes * chunk)
            queue.xor_stripes([(dst2 + s * chunk, chunk, s * nsrc, nsrc, 0) for s in range(nstripes)],
                              [(src + (s * nsrc + k) * chunk, chunk) for s in range(nstripes) for k in range(nsrc)])
            assert np.array_equal(dev.get(dst2, nstripes * chunk), ref), (nstripes, chunk)
    finally:
        engine.tune(0, 0)


@pytest.mark.parametrize("nsrc", [5, 6, 7, 9, 10, 11, 12, 16])
def test_budget_widths_default_tuning(engine, dev, queue, nsrc):
    """Widths that take the waves_per_eu(6) instantiations by default
    (5-7 at U = 8, 12 and 16 at U = 4): full and partial tiles, bit-exact."""
    rng = np.random.default_rng(nsrc)
    for nstripes, chunk in ((300, 512 * KiB), (7, 5 * 16 * KiB + 32)):
        data = rng.integers(0, 256, size=nstripes * nsrc * chunk, dtype=np.uint8)
        src = dev.put(data)
        dst = dev.alloc(nstripes * chunk)
        queue.xor_uniform(dst, src, nstripes, nsrc, chunk)
        queue.sync()
        if nstripes == 300:
            assert engine.option("last_stream_vecs") == (8 if nsrc <= 8 else 4)
        ref = np.bitwise_xor.reduce(data.reshape(nstripes, nsrc, chunk), axis=1).reshape(-1)
        assert np.array_equal(dev.get(dst, nstripes * chunk), ref), (nstripes, chunk)


def test_launch_after_pending_query_keeps_the_work_queue(bcp, engine, dev, queue):
    """A query that reports pending work (-EAGAIN, hipErrorNotReady left on the
    thread) must not be read as a failed launch by the next submission: the
    work-queue base stays in step and every later launch folds all its tiles
    (qbase advancement after a launch error)."""
    nstripes, nsrc, chunk = 2000, 8, 512 * KiB
    src = dev.alloc(nstripes * nsrc * chunk)
    out = dev.alloc(nstripes * chunk)
    res = dev.alloc(64)
    queue.fill_synthetic(src, nstripes * nsrc * chunk, 5)
    L = bcp.lib()
    pending = 0
    for rep in range(4):
        queue.memset(out, 0xA5, nstripes * chunk)
        queue.xor_uniform(out, src, nstripes, nsrc, chunk)
        pending += L.bcp_queue_query(queue.h) == -11  # -EAGAIN while the big launch runs
        queue.xor_uniform(out, src, nstripes, nsrc, chunk)  # submitted right after the query
        queue.xor_fold(out, nstripes * chunk, res)
        queue.xor_fold(src, nstripes * nsrc * chunk, res + 16)
        f = dev.get(res, 32)
        assert np.array_equal(f[:16], f[16:]), rep
    assert pending >= 1  # the scenario actually happened
    # a small descriptor batch after another pending query
    queue.xor_uniform(out, src, nstripes, nsrc, chunk)
    L.bcp_queue_query(queue.h)
    queue.xor_stripes([(out, 1000, 0, 2, 0)], [(src, 1000), (src + chunk, 999)])
    got = dev.get(out, 1000)
    a, b = dev.get(src, 1000), dev.get(src + chunk, 999)
    ref = a.copy()
    ref[:999] ^= b
    assert np.array_equal(got, ref)


def test_descriptor_u16_mixed_batch(oracle, engine, dev, queue):
    """64 KiB descriptor subtiles (desc_vecs_per_thread 16, the rolling
    window) on a config-5-like batch -- log-uniform 1 KiB..1.5 MiB lengths,
    widths 1..12 (wide tiles), misaligned sources and outputs, zero-length
    chunks -- through desc_tiles + xor_desc_p, against the oracle."""
    rng = np.random.default_rng(1605)
    stripes, refs = [], []
    for _ in range(40):
        n = int(rng.integers(1, 13))
        lens = [int(x) for x in np.exp(rng.uniform(np.log(1024), np.log(1536 * 1024), size=n))]
        if n > 2 and rng.random() < 0.2:
            lens[-1] = 0
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        pads = [int(x) for x in rng.integers(0, 16, size=n)]
        stripes.append(dict(chunks=chunks, out_len=max(lens), pads=pads, dst_pad=int(rng.integers(0, 16))))
        refs.append(oracle.xor_padded_np(chunks))
    prev = {k: engine.option(k) for k in ("desc_vecs_per_thread", "desc_args_max")}
    engine.option("desc_vecs_per_thread", 16)
    engine.option("desc_args_max", 0)
    try:
        outs = gpu_stripes(dev, queue, stripes)
        assert engine.option("last_desc_vecs") == 16
    finally:
        for k, v in prev.items():
            engine.option(k, v)
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o, r), i


def test_registered_caller_memory_folds_in_place(oracle, engine, queue):
    """bcp_host_register: a shared anonymous mapping (the kind of memory the
    rank pool's row arena and a connected client's memfd are) registered by
    the caller; a descriptor batch reads its rows and writes its output in
    place over PCIe, then the memory is unregistered.  Same bytes as the
    oracle."""
    import mmap
    n, L = 5, 300_000
    m = mmap.mmap(-1, 4 << 20, flags=mmap.MAP_SHARED)
    buf = np.frombuffer(m, dtype=np.uint8)
    base = buf.ctypes.data
    rng = np.random.default_rng(77)
    rows = [rng.integers(0, 256, size=L - 1000 * k, dtype=np.uint8) for k in range(n)]
    pitch = 320 * 1024
    for k, r in enumerate(rows):
        buf[k * pitch:k * pitch + r.size] = r
    out_off = n * pitch
    engine.host_register(base, 4 << 20)
    try:
        queue.xor_stripes([(base + out_off, L, 0, n, 0)], [(base + k * pitch, rows[k].size) for k in range(n)])
        queue.sync()
        got = buf[out_off:out_off + L].copy()
    finally:
        engine.host_unregister(base)
    assert np.array_equal(got, oracle.xor_padded_np(rows))
    del buf
    m.close()
