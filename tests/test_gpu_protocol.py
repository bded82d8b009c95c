"""The host protocol with the real GPU fold: process_task over loopback ranks
(bcp_gen_run / bcp_rebuild_run), parity files compared with the oracle and
the survey KATs, rebuilds compared with the lost chunks."""
import hashlib
import json
import os

import numpy as np
import pytest

import bcp_store as S

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "kats.json")))
KiB = 1024
MiB = 1024 * KiB


@pytest.fixture(autouse=True)
def gpu_fold(bcp, engine):
    bcp.set_xor_hook(None)  # the product path: fold on the device
    yield
    bcp.task_shutdown()


@pytest.fixture(params=["copy", "direct"])
def read_path(request, monkeypatch):
    """Both read paths of the batched pipeline (bcp_pipeline_opts.read_mode
    AUTO resolves through BCP_PIPELINE_READ): chunks read into pinned slabs,
    or chunks read with O_DIRECT into the slabs."""
    monkeypatch.setenv("BCP_PIPELINE_READ", request.param)
    return request.param


@pytest.fixture(params=["pipelined", "pipelined_queues", "batched"])
def fold_mode(request, bcp):
    """Every form of the P role's GPU fold (bcp_task_set_fold_mode): PIPELINED
    through the device's resident fold ring (the default), PIPELINED with
    range launches on the lanes' queues and the fold service for whole
    windows (bcp_task_set_fold_ring(0)), BATCHED."""
    mode = {"batched": bcp.FOLD_BATCHED, "pipelined": bcp.FOLD_PIPELINED,
            "pipelined_queues": bcp.FOLD_PIPELINED}[request.param]
    prev = bcp.set_fold_mode(mode)
    prev_ring = bcp.set_fold_ring(request.param != "pipelined_queues")
    p0 = bcp.ring_stats()[0]
    yield request.param
    used = bcp.ring_stats()[0] - p0
    bcp.set_fold_ring(prev_ring)
    bcp.set_fold_mode(prev)
    assert (used > 0) == (request.param == "pipelined"), (request.param, used)


@pytest.mark.parametrize("name", ["KAT-2", "KAT-3", "KAT-4"])
def test_survey_kats_end_to_end(bcp, oracle, tmp_path, name, fold_mode):
    k = GOLD["survey_kats"][name]
    n = len(k["lens"])
    p = 8 if n == 8 else 4
    nt = max(9, p + 1)
    root = str(tmp_path)
    S.make_store(root, nt)
    chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(k["lens"])]
    for i, c in enumerate(chunks):
        S.write_chunk(root, i, "a/b/chunk1", c)
    items = [("a/b/chunk1", 2**40, S.with_p((1 << n) - 1, p))]
    st = bcp.gen_run(root, nt, items)
    assert st.errors == 0
    pf = S.read_file(S.parity_path(root, p, "a/b/chunk1"))
    assert len(pf) == k["file_len"] and hashlib.sha256(pf).hexdigest() == k["sha256"]
    v = k["rebuild_victim"]
    os.remove(S.chunk_path(root, v, "a/b/chunk1"))
    st = bcp.rebuild_run(root, nt, v, items)
    assert st.errors == 0
    assert S.read_file(S.chunk_path(root, v, "a/b/chunk1")) == chunks[v].tobytes()


@pytest.mark.parametrize("seed", range(3))
def test_random_worklists_end_to_end(bcp, oracle, tmp_path, seed, fold_mode):
    rng = np.random.default_rng(50 + seed)
    ntargets = int(rng.integers(5, 14))
    files = []
    for i in range(60):
        width = int(rng.integers(1, min(8, ntargets - 1) + 1))
        holders, p = S.random_layout(rng, ntargets, width)
        lens = [int(x) for x in rng.integers(0, 700_000, size=width)]
        files.append((f"u{i % 7}/{i:04x}/chunk{i}", holders, p, lens))
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=seed)
    st = bcp.gen_run(root, ntargets, items, nlanes=12)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    victim = int(rng.integers(0, ntargets))
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    st = bcp.rebuild_run(root, ntargets, victim, items)
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


def test_config1_shape_small(bcp, oracle, tmp_path):
    """Config 1's layout at reduced size: 4 targets, 3-wide stripes, P
    rotating over the target left out, 512 KiB chunks."""
    root = str(tmp_path)
    files = []
    for i in range(48):
        p = i % 4
        holders = [t for t in range(4) if t != p]
        files.append((f"c1/f{i}", holders, p, [512 * KiB] * 3))
    items, contents = S.populate(root, 4, files, seed=9)
    st = bcp.gen_run(root, 4, items)
    assert st.errors == 0 and st.tasks == 48 * 4
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])


@pytest.mark.parametrize("completion,depth", [(4, 1), (0, 1), (2, 3)])
def test_fold_ring_and_lane_queues_write_the_same_files(bcp, oracle, tmp_path, completion, depth):
    """Config 1's shape through the resident fold ring and through the lane
    queues: identical parity files and rebuilt chunks, every window of the
    ring run published to the ring (one piece per range at least).  The
    ring's deferred completions on the completion threads (default 4, and 2
    with depth 3) and on the lanes themselves (0)."""
    old_c = bcp.set_fold_tuning("completion_threads", completion)
    old_d = bcp.set_fold_tuning("defer_depth", depth)
    try:
        _ring_vs_queues(bcp, oracle, tmp_path)
    finally:
        bcp.set_fold_tuning("completion_threads", old_c)
        bcp.set_fold_tuning("defer_depth", old_d)


def _ring_vs_queues(bcp, oracle, tmp_path):
    root = str(tmp_path)
    files = []
    for i in range(36):
        p = i % 4
        holders = [t for t in range(4) if t != p]
        lens = [512 * KiB, 512 * KiB - 17 * (i % 3), 300 * KiB + i]
        files.append((f"c1/f{i}", holders, p, lens))
    items, contents = S.populate(root, 4, files, seed=21)
    prev = bcp.set_fold_ring(True)
    try:
        results = {}
        for ring in (True, False, True):
            bcp.set_fold_ring(ring)
            p0, _ = bcp.ring_stats()
            st = bcp.gen_run(root, 4, items)
            pieces = bcp.ring_stats()[0] - p0
            assert st.errors == 0
            assert (pieces >= len(files)) if ring else pieces == 0, (ring, pieces)
            got = {path: S.read_file(S.parity_path(root, p, path)) for path, _, p, _ in files}
            for path, _, p, _ in files:
                assert got[path] == oracle.gen_parity_file(contents[path]), (ring, path)
            results.setdefault(ring, got)
            victim = 1
            for path, holders, p, lens in files:
                if victim in holders:
                    os.remove(S.chunk_path(root, victim, path))
            st = bcp.rebuild_run(root, 4, victim, items)
            assert st.errors == 0
            for path, holders, p, lens in files:
                if victim in holders:
                    k = holders.index(victim)
                    assert S.read_file(S.chunk_path(root, victim, path)) == bytes(contents[path][k]), (ring, path)
        assert results[True] == results[False]
    finally:
        bcp.set_fold_ring(prev)


def test_ring_worker_count_change_remakes_the_rings(bcp, oracle, tmp_path):
    """bcp_task_set_fold_tuning("ring_workers") between runs ends the current
    rings; the next fold makes new ones with that many workers (1, 8, 40,
    then the default): every run's parity files exact."""
    root = str(tmp_path)
    files = [(f"w/f{i}", [t for t in range(4) if t != i % 4], i % 4, [400 * KiB + 7 * i, 512 * KiB, 64 * KiB])
             for i in range(16)]
    items, contents = S.populate(root, 4, files, seed=12)
    old = bcp.set_fold_tuning("ring_workers", 16)
    try:
        for w in (1, 8, 40, old):
            bcp.set_fold_tuning("ring_workers", w)
            p0, l0 = bcp.ring_stats()
            assert bcp.gen_run(root, 4, items).errors == 0, w
            p1, l1 = bcp.ring_stats()
            assert p1 > p0 and l1 > l0, (w, p0, p1, l0, l1)
            for (path, _, p, _) in files:
                assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), (w, path)
    finally:
        bcp.set_fold_tuning("ring_workers", old)


@pytest.mark.parametrize("completion", [4, 0])
def test_deferred_parity_write_failure_is_sticky(bcp, oracle, tmp_path, completion):
    """Through the fold ring with lane deferral, a parity write fails (ENOSPC,
    injected) in a deferred completion -- on a completion thread (4) or on
    the lane (0): exactly that rank's error is sticky, every other rank's
    parity files are exact, rebuilds of a clean rerun are exact."""
    root = str(tmp_path)
    files = [(f"d/f{i}", [t for t in range(4) if t != i % 4], i % 4, [512 * KiB - 3 * i, 512 * KiB, 200 * KiB])
             for i in range(24)]
    items, contents = S.populate(root, 4, files, seed=31)
    old_c = bcp.set_fold_tuning("completion_threads", completion)
    bcp.inject_failure(bcp.INJECT_PARITY_WRITE, 5, 1)
    try:
        st = bcp.gen_run(root, 4, items)
    finally:
        bcp.inject_failure(bcp.INJECT_PARITY_WRITE, 0, 0)
    try:
        assert st.errors == 1
        good = sum(1 for (path, _, p, _) in files if os.path.exists(S.parity_path(root, p, path))
                   and S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]))
        assert 18 <= good < len(files)  # one rank of four failed: at most its 6 files
        assert bcp.gen_run(root, 4, items).errors == 0
        for (path, _, p, _) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    finally:
        bcp.set_fold_tuning("completion_threads", old_c)


def test_fold_ring_idles_out_between_runs_and_shuts_down_live(bcp, oracle, tmp_path):
    """The ring's launch ends 5 ms after the last fold and the next run
    relaunches it; bcp_task_shutdown right after a run (launch still live)
    stops it at once; the next run makes a new ring."""
    import time
    root = str(tmp_path)
    files = [(f"r/f{i}", [t for t in range(5) if t != i % 5][:3], i % 5, [200 * KiB] * 3) for i in range(20)]
    items, contents = S.populate(root, 5, files, seed=4)
    _, l0 = bcp.ring_stats()
    for _ in range(3):
        assert bcp.gen_run(root, 5, items).errors == 0
        time.sleep(0.05)
    _, l1 = bcp.ring_stats()
    assert l1 - l0 >= 3
    assert bcp.gen_run(root, 5, items).errors == 0
    t0 = time.perf_counter()
    bcp.task_shutdown()  # the launch is live (idle limit 5 ms)
    assert time.perf_counter() - t0 < 1.0
    assert bcp.gen_run(root, 5, items).errors == 0
    for path, holders, p, lens in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])


# --------------------------------------------------------------------------
# batched pipeline (bcp_pipeline_gen): same files as the per-task protocol
# --------------------------------------------------------------------------
@pytest.mark.parametrize("slab", [1 << 20, 64 << 20])
@pytest.mark.usefixtures("read_path")
def test_pipeline_matches_oracle_mixed_sizes(bcp, oracle, tmp_path, slab):
    rng = np.random.default_rng(77)
    ntargets = 10
    files = []
    for i in range(80):
        width = int(rng.integers(1, 9))
        holders, p = S.random_layout(rng, ntargets, width)
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=width))]
        lens[0] = lens[0] + int(rng.integers(0, 15))     # not 16-byte rounded
        files.append((f"m/{i % 9}/c{i}", holders, p, lens))
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=5)
    os.remove(S.chunk_path(root, files[3][1][0], files[3][0]))   # a missing chunk: size 0 / zeros
    contents[files[3][0]][0] = None
    st = bcp.pipeline_gen(root, ntargets, items, slab_bytes=slab, io_threads=4, nslots=3)
    assert st.errors == 0 and st.tasks == len(files)
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.usefixtures("read_path")
def test_pipeline_wide_and_windowed_stripes(bcp, oracle, tmp_path):
    """The batched pipeline on stripes wider than a tile record (up to 15
    sources), chunks past the 10 MiB transfer window (replay) and grouped
    sparse tiles; then a rebuild of one target through the pipeline."""
    rng = np.random.default_rng(91)
    ntargets = 16
    files = []
    for i in range(14):
        width = int(rng.integers(9, 16)) if i % 2 else int(rng.integers(2, 9))
        holders, p = S.random_layout(rng, ntargets, width)
        hi = 24 * 1024 * KiB if i % 3 == 0 else 3 * 1024 * KiB
        lens = [int(x) for x in np.exp(rng.uniform(np.log(16 * KiB), np.log(hi), size=width))]
        lens[-1] += 7
        files.append((f"w/{i % 4}/c{i}", holders, p, lens))
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=12)
    st = bcp.pipeline_gen(root, ntargets, items, slab_bytes=64 << 20, io_threads=4, nslots=3)
    assert st.errors == 0 and st.tasks == len(files)
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    victim = 5
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    assert lost
    pl = bcp.Pipeline(io_threads=4)
    try:
        st = pl.rebuild(root, ntargets, victim, sorted(items, key=lambda x: x[0].encode()))
    finally:
        pl.close()
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


@pytest.mark.usefixtures("read_path")
def test_pipeline_multiwindow_and_delete(bcp, oracle, tmp_path):
    root = str(tmp_path)
    files = [("big/a", [0, 1], 4, [10485760, 26214405]),
             ("big/b", [1, 2, 3], 0, [21 * 1024 * KiB, 0, 10 * 1024 * KiB + 17]),
             ("small", [0, 2], 3, [100, 5])]
    items, contents = S.populate(root, 5, files, seed=6)
    bcp.pipeline_gen(root, 5, items, slab_bytes=8 << 20)
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    bcp.pipeline_gen(root, 5, [("small", 0, S.with_p(0, 3))])
    assert not os.path.exists(S.parity_path(root, 3, "small"))


@pytest.mark.usefixtures("read_path")
def test_pipeline_refuses_paths_outside_the_store(bcp, oracle, tmp_path):
    """As process_task: an item whose path would leave the targets'
    directories is skipped (gen and rebuild); the others run."""
    root = str(tmp_path)
    items, contents = S.populate(root, 4, [("ok", [0, 1], 2, [5000, 7000])])
    for h in (0, 1):
        os.makedirs(os.path.join(root, f"st{h}", "outside"), exist_ok=True)
        with open(os.path.join(root, f"st{h}", "outside", "x"), "wb") as f:
            f.write(b"z" * 100)
    items = [("../outside/x", 2**40, S.with_p(0b11, 2))] + items
    st = bcp.pipeline_gen(root, 4, items)
    assert st.errors == 0 and st.tasks == 1 and st.refused == 1
    assert S.read_file(S.parity_path(root, 2, "ok")) == oracle.gen_parity_file(contents["ok"])
    assert not os.path.exists(os.path.join(root, "st2", "outside"))
    os.remove(S.chunk_path(root, 1, "ok"))
    pl = bcp.Pipeline()
    try:
        st = pl.rebuild(root, 4, 1, items)
    finally:
        pl.close()
    assert st.errors == 0 and st.tasks == 1 and st.refused == 1
    assert S.read_file(S.chunk_path(root, 1, "ok")) == contents["ok"][1].tobytes()
    assert S.read_file(os.path.join(root, "st1", "outside", "x")) == b"z" * 100


@pytest.mark.usefixtures("read_path")
def test_pipeline_object_reuse_and_growth(bcp, oracle, tmp_path):
    """One long-lived pipeline, several runs; the second needs bigger slabs."""
    root = str(tmp_path)
    small = [("s/a", [0, 1], 2, [5000, 7000]), ("s/b", [1, 2], 0, [64 * KiB, 3])]
    big = [("b/a", [0, 1, 2], 3, [3 * 1024 * KiB, 2 * 1024 * KiB + 5, 1])]
    it1, c1 = S.populate(root, 4, small, seed=1)
    it2, c2 = S.populate(root, 4, big, seed=2)
    pl = bcp.Pipeline(slab_bytes=1 << 20, io_threads=2, nslots=2)
    try:
        for items, files, contents in ((it1, small, c1), (it2, big, c2), (it1, small, c1)):
            st = pl.run(root, 4, items)
            assert st.errors == 0
            for (path, holders, p, lens) in files:
                assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
            # one io read job per 1 MiB piece of every chunk read into a slab
            # (bcp_pipeline_last_timing); DIRECT reads the page-rounded file,
            # the same pieces for a gen
            tm = pl.last_timing()
            pieces = sum((n + MiB - 1) // MiB for f in files for n in f[3])
            assert tm["read_jobs"] == pieces, tm
            assert 1 <= tm["batches"] <= len(files) and min(tm[k] for k in ("stat", "read_wait", "submit")) >= 0
    finally:
        pl.close()


def test_protocol_repeated_runs_reuse_pool(bcp, oracle, tmp_path):
    root = str(tmp_path)
    files = [(f"r/{i}", [0, 1, 2], 3, [100000 + i, 90000, 5]) for i in range(20)]
    items, contents = S.populate(root, 4, files, seed=3)
    for _ in range(3):
        st = bcp.gen_run(root, 4, items, nlanes=4)
        assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])


def test_pool_reuse_with_changing_data_and_teardown(bcp, oracle, tmp_path):
    """The pooled window rows and outputs (registered host memory) are
    rewritten between runs, the modes alternate, and every other round tears
    the engines, fold services and pool down and builds them again (freed
    memory's addresses are re-issued to new allocations), with a batched
    pipeline run between: no fold may see a previous task's bytes."""
    root = str(tmp_path)
    rng = np.random.default_rng(77)
    modes = [bcp.FOLD_PIPELINED, bcp.FOLD_BATCHED] * 4
    for rnd, mode in enumerate(modes):
        files = [(f"z/{i}", [0, 1, 2], 3, [int(x) for x in rng.integers(1, 600_000, size=3)]) for i in range(24)]
        items, contents = S.populate(root, 4, files, seed=100 + rnd)
        prev = bcp.set_fold_mode(mode)
        try:
            st = bcp.gen_run(root, 4, items, nlanes=6)
        finally:
            bcp.set_fold_mode(prev)
        assert st.errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), (rnd, path)
        if rnd % 2:
            bcp.task_shutdown()
            assert bcp.pipeline_gen(root, 4, items).errors == 0
            for (path, holders, p, lens) in files:
                assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), (rnd, path)


def test_pipelined_read_error_refold_on_device(bcp, oracle, tmp_path):
    """The pipelined fold on the device when a source's read fails after
    ranges of its row were already folded (in flight on the lane's queue):
    the P role refolds the whole window, the failed row counts as zeros (the
    reference's zero-filled window), the source's rank is in error."""
    KiBl, MiBl = 1024, 1024 * 1024
    root = str(tmp_path)
    lens = [7, 100 * KiBl, 4 * MiBl + 3]
    items, contents = S.populate(root, 4, [("e/x", [0, 1, 2], 3, lens)], seed=6)
    prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
    bcp.inject_failure(bcp.INJECT_READ, 10, 1)
    try:
        st = bcp.gen_run(root, 4, items, nlanes=1)
    finally:
        bcp.inject_failure(bcp.INJECT_READ, 0, 0)
        bcp.set_fold_mode(prev)
    assert st.errors == 1
    pf = S.read_file(S.parity_path(root, 3, "e/x"))
    assert np.frombuffer(pf[:24], "<u8").tolist() == lens
    expect = np.zeros(max(lens), np.uint8)
    for c in contents["e/x"][:2]:
        expect[:c.size] ^= c
    assert np.array_equal(np.frombuffer(pf[24:], np.uint8), expect)
    # and the lanes fold correctly afterwards
    items, contents = S.populate(root, 4, [("e/y", [0, 1, 2], 3, [3 * MiBl, 5, 700 * KiBl])], seed=7)
    assert bcp.gen_run(root, 4, items, nlanes=2).errors == 0
    assert S.read_file(S.parity_path(root, 3, "e/y")) == oracle.gen_parity_file(contents["e/y"])


def test_fold_mode_rejects_unknown(bcp):
    with pytest.raises(bcp.BcpError):
        bcp.set_fold_mode(7)


@pytest.mark.parametrize("engine_kind", ["protocol", "pipeline"])
def test_db_round_then_partial_round_then_rebuild(bcp, oracle, tmp_path, engine_kind):
    """A full gen round from chunk events (plan + DB replicas), a changelog
    round that recomputes only the modified stripe, then a rebuild walking
    the DB -- on the device, with both engines.  The layout (holders, weights)
    is tests/golden/ref_round.json's, and every file's parity must land on the
    P target the REFERENCE'S OWN select_P picks for it (gen/main.c:388-401,
    compiled unchanged; tests/golden/make_ref_plan_golden.py)."""
    import json
    import planner as PL
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_round.json")))
    rng = np.random.default_rng(11)
    root, nt = str(tmp_path), fx["ntargets"]
    S.make_store(root, nt)
    cw = fx["cum_weight"]
    streams, contents, files, ref_p = {k: [] for k in range(nt)}, {}, {}, {}
    for i, (path, holders, loc) in enumerate(fx["files"]):
        lens = [int(x) for x in np.exp(rng.uniform(np.log(1024), np.log(3 << 20), size=len(holders)))]
        arrs = []
        for h, L in zip(holders, lens):
            d = S.synthetic_chunk(i * 97 + h, L)
            S.write_chunk(root, h, path, d)
            streams[h].append((1000 + i, L, "m", path))
            arrs.append(d)
        files[path], contents[path], ref_p[path] = holders, arrs, PL.get_p(loc)
    pl = bcp.Pipeline() if engine_kind == "pipeline" else None

    def round_(streams):
        es = bcp.EventSet()
        for k, recs in streams.items():
            es.feed(k, bcp.pack_records(recs))
        r = pl.round(root, nt, es, cum_weight=cw) if pl else bcp.gen_round(root, nt, es, cum_weight=cw, nlanes=4)
        es.close()
        return r

    try:
        st, n = round_(streams)
        assert st.errors == 0 and n == 24
        db = bcp.PDB(os.path.join(root, "st3", "db"))
        placed = {k.decode(): loc for k, _, loc in db.items()}
        db.close()
        for path, holders in files.items():
            p = ref_p[path]
            assert PL.get_p(placed[path]) == p, path  # the reference's placement
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        # partial round: one chunk modified
        path = "d1/c5"
        h = files[path][2]
        assert len(files[path]) > 2
        new = S.synthetic_chunk(4242, 777_777)
        S.write_chunk(root, h, path, new)
        contents[path][2] = new
        st, n = round_({h: [(5000, 777_777, "m", path)]})
        assert n == 1 and st.errors == 0
        assert S.read_file(S.parity_path(root, PL.get_p(placed[path]), path)) == oracle.gen_parity_file(contents[path])
    finally:
        if pl:
            pl.close()
    victim = 5
    lost = {}
    for path, holders in files.items():
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    st = bcp.rebuild_run_db(root, nt, victim)
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


POOL_SCRIPT = r"""
import os, sys
root = sys.argv[1]
here = sys.argv[2]
sys.path[:0] = [os.path.join(here, "..", "beegfs-chunk-parity_amd"), os.path.join(here, "..", "oracle")]
import numpy as np
import bcp_ctypes as bcp, bcp_store as S, oracle
rng = np.random.default_rng(7)
nt = 6
files = []
for i in range(24):
    holders, p = S.random_layout(rng, nt, int(rng.integers(2, 6)))
    files.append((f"q{i % 3}/c{i}", holders, p, [int(x) for x in rng.integers(1, 900_000, size=len(holders))]))
def check(files, contents):
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
with bcp.RankPool(nt) as pool:   # this process never touches the GPU; the ranks do
    items, contents = S.populate(root, nt, files, seed=1)
    assert pool.gen(root, items, nlanes=4).errors == 0
    check(files, contents)
    small = [(path, h, p, [L // 5 + 1 for L in lens]) for (path, h, p, lens) in files]
    items, contents = S.populate(root, nt, small, seed=2)
    assert pool.gen(root, items, nlanes=4).errors == 0
    check(small, contents)
    victim, lost = 1, {}
    for (path, holders, p, lens) in small:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    assert lost and pool.rebuild(root, victim, items).errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path
print("pool ok")
"""


@pytest.mark.parametrize("mode", ["ranks", "fold-server", "no-arena"])
def test_rank_pool_on_device(tmp_path, mode):
    """Rank processes kept alive across runs: two gen runs over different
    data and a rebuild through ONE pool, the P roles folding on the device,
    parity and rebuilt chunks checked against the oracle.  "ranks": every
    rank holds its own HIP context and folds through its batched service,
    its sources filling P roles' rows in the shared arena; "fold-server":
    one server process holds the GPU and folds every rank's windows
    (BCP_FOLD_SERVER=1; the ranks never start HIP); "no-arena": rows in each
    rank's own registered memory, windows through the sockets.  In a fresh
    process: a pool cannot be forked from one that has used the GPU."""
    import subprocess
    import sys
    env = dict(os.environ)
    env["BCP_FOLD_SERVER"] = "1" if mode == "fold-server" else "0"
    if mode == "no-arena":
        env["BCP_SOCK_ARENA_MB"] = "0"
    r = subprocess.run([sys.executable, "-c", POOL_SCRIPT, str(tmp_path), HERE], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0 and "pool ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("engine_kind", ["default", "protocol", "pipeline", "pipeline_direct", "procs",
                                         "procs_batched", "protocol_ranked", "default_ranked", "procs_ranked"])
def test_cli_complete_partial_rebuild(bcp, oracle, tmp_path, engine_kind):
    """bin/bcp end to end on the device: --complete (scan of every target),
    --partial from changelog record files, then parity-rebuild from the DB --
    ranks as threads, the batched pipeline, or ranks as processes (--procs:
    one forked process per target on the socketpair transport, each with its
    the node fold server holding the GPU for all of them, in the default fold
    mode or batched).  *_ranked: the store states a permuted MPI rank order
    (<root>/rank_order), so the coordinators' rounds run in that order -- the
    same files and DB state."""
    import subprocess
    import planner as PL
    rng = np.random.default_rng(21)
    root, nt = str(tmp_path / "store"), 6
    S.make_store(root, nt)
    if engine_kind.endswith("_ranked"):  # ids default to k + 1 (no targetNumID files)
        with open(os.path.join(root, "rank_order"), "w") as f:
            f.write("4 1 6 2 5 3\n")
        assert bcp.store_round_order(root, nt) == [3, 0, 5, 1, 4, 2]
        engine_kind = engine_kind[:-len("_ranked")]
    files, contents = {}, {}
    for i in range(20):
        path = f"u{i % 2}/{i:02X}/c{i}"
        holders = sorted(int(x) for x in rng.choice(nt, size=int(rng.integers(1, nt)), replace=False))
        arrs = []
        for h in holders:
            d = S.synthetic_chunk(i * 13 + h, int(rng.integers(1, 300_000)))
            S.write_chunk(root, h, path, d)
            arrs.append(d)
        files[path], contents[path] = holders, arrs
    flags = {"default": [], "protocol": ["--protocol"], "pipeline": ["--pipeline"],
             "pipeline_direct": ["--read", "direct"],
             "procs": ["--procs"], "procs_batched": ["--procs", "--fold", "batched"]}[engine_kind]
    r = subprocess.run([bcp.BIN_PATH, "parity-gen", "--complete", *flags, root, str(nt)], capture_output=True)
    assert r.returncode == 0, r.stderr
    engine_named = {"protocol": b"(protocol)"}.get(
        engine_kind, b"(rank processes)" if engine_kind.startswith("procs") else b"(pipeline)")
    assert engine_named in r.stdout, r.stdout  # the batched pipeline is the default engine
    db = bcp.PDB(os.path.join(root, "st0", "db"))
    placed = {k.decode(): loc for k, _, loc in db.items()}
    db.close()
    for path, holders in files.items():
        assert placed[path] & PL.L_MASK == sum(1 << h for h in holders)
        assert S.read_file(S.parity_path(root, PL.get_p(placed[path]), path)) == \
            oracle.gen_parity_file(contents[path]), path
    # a second --complete needs --force
    r = subprocess.run([bcp.BIN_PATH, "parity-gen", "--complete", *flags, root, str(nt)], capture_output=True)
    assert r.returncode == 1
    # --partial: one chunk rewritten, its record in the changelog of its target
    path = "u1/03/c3"
    h = files[path][0]
    new = S.synthetic_chunk(999, 123_457)
    S.write_chunk(root, h, path, new)
    contents[path][0] = new
    os.makedirs(os.path.join(root, "changelog"))
    with open(os.path.join(root, "changelog", f"st{h}"), "wb") as f:
        f.write(bcp.pack_records([(2_000_000_000, len(new), "m", path)]))
    r = subprocess.run([bcp.BIN_PATH, "parity-gen", "--partial", *flags, root, str(nt)], capture_output=True)
    assert r.returncode == 0, r.stderr
    assert S.read_file(S.parity_path(root, PL.get_p(placed[path]), path)) == oracle.gen_parity_file(contents[path])
    # lose a target, rebuild it from the DB
    victim = 2
    lost = {}
    for p_, holders in files.items():
        if victim in holders:
            lost[p_] = S.read_file(S.chunk_path(root, victim, p_))
            os.remove(S.chunk_path(root, victim, p_))
    rflags = flags + (["--lanes", "4"] if engine_kind in ("protocol", "procs") else [])  # rebuild lanes
    r = subprocess.run([bcp.BIN_PATH, "parity-rebuild", *rflags, root, str(nt), str(victim)], capture_output=True)
    assert r.returncode == 0, r.stderr
    for p_, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, p_)) == data, p_


@pytest.mark.parametrize("ndevices,nslots", [(2, 2), (3, 2), (8, 3)])
@pytest.mark.usefixtures("read_path")
def test_pipeline_multi_device_lanes(bcp, oracle, tmp_path, ndevices, nslots):
    """Batches round-robin over several device lanes (on a one-GPU box the
    lanes wrap onto the same GPU, each with its own engine, queues and
    slots); small slabs force many batches so every lane and slot recycles."""
    rng = np.random.default_rng(ndevices)
    files = []
    for i in range(60):
        holders, p = S.random_layout(rng, 9, int(rng.integers(1, 9)))
        files.append((f"m/{i}", holders, p, [int(x) for x in rng.integers(0, 400_000, size=len(holders))]))
    root = str(tmp_path)
    items, contents = S.populate(root, 9, files, seed=ndevices)
    pl = bcp.Pipeline(slab_bytes=1 << 20, io_threads=4, nslots=nslots, ndevices=ndevices)
    try:
        for _ in range(2):
            st = pl.run(root, 9, items)
            assert st.errors == 0 and st.tasks == len(files)
            for (path, holders, p, lens) in files:
                assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    finally:
        pl.close()


@pytest.mark.usefixtures("read_path")
def test_pipeline_rebuild_matches_protocol_rebuild(bcp, oracle, tmp_path):
    """bcp_pipeline_rebuild == bcp_rebuild_run byte for byte: mixed sizes,
    multi-window stripes (replay), a missing survivor, a survivor rewritten
    after generation (corrupt list), a missing parity file and skip rules."""
    rng = np.random.default_rng(31)
    nt = 7
    MiB = 1024 * 1024
    files = []
    for i in range(30):
        holders, p = S.random_layout(rng, nt, int(rng.integers(1, 6)))
        lens = [int(x) for x in rng.integers(0, 600_000, size=len(holders))]
        files.append((f"r/{i}", holders, p, lens))
    files.append(("big/0", [0, 1, 2], 3, [10 * MiB + 17, 26 * MiB + 5, 3]))   # windows + replay
    files.append(("big/1", [1, 4], 0, [21 * MiB, 1]))
    outs = {}
    for mode in ("protocol", "pipeline"):
        root = str(tmp_path / mode)
        items, contents = S.populate(root, nt, files, seed=5, timestamp=2_000_000_000)
        bcp.gen_run(root, nt, items)
        victim = 1
        # a survivor rewritten after generation -> corrupt list; a survivor lost
        for path, holders, p, lens in files:
            if victim in holders and len(holders) > 2:
                other = next(h for h in holders if h != victim)
                os.utime(S.chunk_path(root, other, path), (2_100_000_000, 2_100_000_000))
                break
        for path, holders, p, lens in files:
            if victim in holders and len(holders) > 2 and path != "big/0":
                os.remove(S.chunk_path(root, [h for h in holders if h != victim][-1], path))
                break
        os.remove(S.parity_path(root, files[-1][2], "big/1"))             # parity lost too
        for path, holders, p, lens in files:
            if victim in holders:
                os.remove(S.chunk_path(root, victim, path))
        ordered = sorted(items, key=lambda x: x[0].encode())
        corrupt = str(tmp_path / f"corrupt_{mode}")
        if mode == "protocol":
            st = bcp.rebuild_run(root, nt, victim, ordered, corrupt_list=corrupt)
        else:
            pl = bcp.Pipeline(slab_bytes=4 * MiB, nslots=2)
            try:
                st = pl.rebuild(root, nt, victim, ordered, corrupt_list=corrupt)
            finally:
                pl.close()
        assert st.errors == 0
        got = {}
        for path, holders, p, lens in files:
            if victim in holders:
                got[path] = S.read_file(S.chunk_path(root, victim, path))
        outs[mode] = (got, sorted(open(corrupt).read().split()))
    assert outs["protocol"] == outs["pipeline"]
    # and the survivors that were intact reproduce the lost chunks exactly
    got = outs["pipeline"][0]
    assert got["big/0"] == S.synthetic_chunk(5 * 1_000_003 + 30 * 61 + 1, 26 * MiB + 5).tobytes()
    assert got["big/1"] == b""   # parity gone: header reads as zeros -> empty chunk, as the reference


@pytest.mark.parametrize("fold", ["pipelined", "batched"])
def test_node_fold_server_for_connected_clients(tmp_path, fold):
    """The node fold server as an MPI job would use it: a server process on a
    Unix socket holds the GPU (bcp_fold_server_serve); two client processes
    connect (bcp_fold_server_connect, memfd arenas the server maps at its own
    addresses) and run gen + rebuild with loopback ranks inside; every fold
    runs on the device in the server.  Parity and rebuilds vs the oracle."""
    import json
    import subprocess
    import sys
    import time
    import test_fold_server_cpu as F
    sock = str(tmp_path / "fs.sock")
    srv = subprocess.Popen([sys.executable, "-c", F.SERVER, sock, F.ROOT, "6", "gpu", ""], stdout=subprocess.PIPE,
                           text=True)
    assert srv.stdout.readline().strip() == "serving"
    for _ in range(500):
        if os.path.exists(sock):
            break
        time.sleep(0.01)
    clients = [subprocess.Popen([sys.executable, "-c", F.CLIENT, sock, F.ROOT, str(tmp_path / f"store{k}"), "gpu", "",
                                 "3", fold, str(20 + k)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
               for k in range(2)]
    for c in clients:
        out, err = c.communicate(timeout=200)
        assert c.returncode == 0, err[-3000:]
        d = json.loads(out.strip().splitlines()[-1])
        assert d["errors"] == 0 and d["rb_errors"] == 0 and d["bad"] == [], d
        assert d["server_folds"] > 0, d
    srv_out, _ = srv.communicate(timeout=60)
    assert srv.returncode == 0 and "served" in srv_out


POOL5_SCRIPT = r"""
import os, sys
root, here = sys.argv[1], sys.argv[2]
sys.path[:0] = [os.path.join(here, "..", "beegfs-chunk-parity_amd"), os.path.join(here, "..", "oracle")]
import numpy as np
import bcp_ctypes as bcp, bcp_store as S, oracle
rng = np.random.default_rng(55)
nt, KiB, MiB = 9, 1024, 1024 * 1024
files = []
for i in range(150):
    holders, p = S.random_layout(rng, nt, 8)
    lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
    files.append((f"c5/{i % 7}/x{i}", holders, p, lens))
items, contents = S.populate(root, nt, files, seed=6)
with bcp.RankPool(nt) as pool:
    assert pool.gen(root, items, nlanes=12).errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    victim, lost = 4, {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    bcp.set_rebuild_lanes(6)
    assert lost and pool.rebuild(root, victim, items).errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path
print("pool5 ok")
"""


def test_rank_pool_config5_shapes_every_file(tmp_path):
    """Config-5 shapes (9 targets, 8-wide stripes of 64 KiB-4 MiB chunks,
    150 stripes) through nine rank processes and the node fold server (the
    default), every parity file against the oracle, then a 6-lane rebuild
    of one target, every rebuilt chunk compared."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", POOL5_SCRIPT, str(tmp_path), HERE], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "pool5 ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_caller_transport_table_on_device(bcp, oracle, tmp_path, foreign_ops_addr, fold_mode):
    """process_task over a caller's transport table (an MPI binding's shape:
    no send_fill) with the GPU fold: the reference's padded wire, every window
    through the device's fold service (the pipelined fold cannot follow such a
    transport), multi-window replay; parity and rebuild exact."""
    rng = np.random.default_rng(707)
    nt = 8
    files = []
    for i in range(40):
        holders, p = S.random_layout(rng, nt, int(rng.integers(1, 7)))
        lens = [int(x) for x in np.exp(rng.uniform(np.log(1024), np.log(4 << 20), size=len(holders)))]
        files.append((f"g/{i % 5}/c{i}", holders, p, lens))
    files[0] = ("g/big", [0, 1, 3], 2, [10 << 20, (21 << 20) + 9, 5])
    root = str(tmp_path)
    items, contents = S.populate(root, nt, files, seed=71)
    bcp.set_transport(foreign_ops_addr)
    try:
        assert bcp.gen_run(root, nt, items, nlanes=6).errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        victim = 3
        lost = {}
        for (path, holders, p, lens) in files:
            if victim in holders:
                lost[path] = S.read_file(S.chunk_path(root, victim, path))
                os.remove(S.chunk_path(root, victim, path))
        assert lost
        assert bcp.rebuild_run(root, nt, victim, items).errors == 0
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, path
    finally:
        bcp.set_transport(None)


@pytest.mark.parametrize("mode", ["copy", "direct"])
def test_pipeline_read_modes_byte_identical_and_fallback(bcp, oracle, tmp_path, mode):
    """Both read paths write the same parity files; a chunk that cannot be
    opened (mode 000: stat works, open does not) counts as unreadable (zeros)
    in either.  DIRECT: every chunk is read with O_DIRECT
    (timing.direct_bytes), or through the page cache where the filesystem
    refuses it, with the same output."""
    rng = np.random.default_rng(4242)
    nt = 9
    files = []
    for i in range(120):
        holders, p = S.random_layout(rng, nt, 8)
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=8))]
        files.append((f"r/{i % 7}/c{i}", holders, p, lens))
    root = str(tmp_path / "store")
    items, contents = S.populate(root, nt, files, seed=17)
    bad = S.chunk_path(root, files[40][1][2], files[40][0])
    want_mode = {"copy": bcp.READ_COPY, "direct": bcp.READ_DIRECT}[mode]
    outs = {}
    for locked in (False, True):
        if locked:
            if os.geteuid() == 0:
                pytest.skip("root opens mode-000 files")
            os.chmod(bad, 0)
        pl = bcp.Pipeline(slab_bytes=16 << 20, io_threads=4, nslots=3, read_mode=want_mode)
        try:
            st = pl.run(root, nt, items)
            tm = pl.last_timing()
        finally:
            pl.close()
            os.chmod(bad, 0o600)
        assert st.errors == 0 and st.tasks == len(files)
        assert tm["read_mode"] == want_mode and tm["batches"] > 4
        if mode == "direct":
            total = sum(sum(f[3]) for f in files)
            # all of it with O_DIRECT, or pieces through the page cache (a
            # filesystem without O_DIRECT; locked: the unopenable chunk)
            assert tm["direct_bytes"] == st.bytes_read or tm["direct_fallbacks"] > 0, tm
            if not locked:
                assert st.bytes_read == total
        else:
            assert tm["direct_bytes"] == 0 and tm["direct_fallbacks"] == 0
        outs[locked] = {path: S.read_file(S.parity_path(root, p, path)) for path, _, p, _ in files}
    for path, holders, p, lens in files:
        assert outs[False][path] == oracle.gen_parity_file(contents[path]), path
    # the unreadable chunk: every other file unchanged, its own as COPY mode gives it
    diff = [path for path in outs[False] if outs[False][path] != outs[True][path]]
    assert diff == [files[40][0]]
    body = np.frombuffer(outs[True][files[40][0]][64:], dtype=np.uint8)
    chunks = [c for k, c in enumerate(contents[files[40][0]]) if k != 2]
    ref = np.zeros(len(body), dtype=np.uint8)
    for c in chunks:
        ref[:len(c)] ^= c
    assert np.array_equal(body, ref)


@pytest.mark.parametrize("slab", ["registered", "hipHostMalloc"])
def test_pipeline_direct_reads_fall_back_piece_by_piece(bcp, oracle, tmp_path, monkeypatch, slab):
    """DIRECT read mode: an O_DIRECT read that ends short before the end of
    its file (injected: the bytes it did deliver past the cut are spoilt) is
    finished through the page cache from the cut -- the same parity files and
    rebuilt chunks, one fallback per injected piece.  Over either kind of
    pinned slab (BCP_HOST_REGISTERED: registered THP memory, the default, or
    hipHostMalloc'd memory, which O_DIRECT may refuse: then every piece falls
    back, with the same output)."""
    monkeypatch.setenv("BCP_HOST_REGISTERED", "1" if slab == "registered" else "0")
    rng = np.random.default_rng(99)
    nt = 9
    files = []
    for i in range(40):
        holders, p = S.random_layout(rng, nt, 8)
        lens = [int(x) for x in rng.integers(1, 3 * MiB, size=8)]
        files.append((f"d/{i % 5}/c{i}", holders, p, lens))
    root = str(tmp_path / "store")
    items, contents = S.populate(root, nt, files, seed=23)
    pl = bcp.Pipeline(slab_bytes=16 << 20, io_threads=4, nslots=3, read_mode=bcp.READ_DIRECT)
    try:
        bcp.inject_failure(bcp.INJECT_DIRECT_READ, 5, 3)
        st = pl.run(root, nt, items)
        tm = pl.last_timing()
        bcp.inject_failure(bcp.INJECT_DIRECT_READ, 0, 0)
        assert st.errors == 0 and st.tasks == len(files)
        assert st.bytes_read == sum(sum(f[3]) for f in files)
        if tm["direct_bytes"]:  # O_DIRECT worked: exactly the injected pieces fell back
            assert tm["direct_fallbacks"] == 3, tm
        else:
            assert tm["direct_fallbacks"] > 3, tm
        for path, holders, p, lens in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        # rebuild through the same fallback (parity bodies start 8n into their files)
        victim = 4
        lost = {path: S.read_file(S.chunk_path(root, victim, path)) for path, holders, _, _ in files
                if victim in holders}
        for path in lost:
            os.remove(S.chunk_path(root, victim, path))
        bcp.inject_failure(bcp.INJECT_DIRECT_READ, 2, 2)
        st = pl.rebuild(root, nt, victim, sorted(items, key=lambda x: x[0].encode()))
        tm = pl.last_timing()
        bcp.inject_failure(bcp.INJECT_DIRECT_READ, 0, 0)
        assert st.errors == 0 and st.tasks == len(lost)
        if tm["direct_bytes"]:
            assert tm["direct_fallbacks"] == 2, tm
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, path
    finally:
        bcp.inject_failure(bcp.INJECT_DIRECT_READ, 0, 0)
        pl.close()


@pytest.mark.parametrize("mode", ["copy", "direct"])
def test_pipeline_small_pool_and_odd_holder_counts(bcp, oracle, tmp_path, mode):
    """The io pool (reads ahead of writes) with few threads and small slabs,
    so jobs of both kinds queue up: the same parity files and rebuilt chunks.
    Holder counts 2..8 give rebuild stripes of every source count n, so for
    odd n the parity body starts 8n bytes into its file -- an 8-byte-aligned
    source in the slab's page layout under DIRECT, 256-byte
    aligned under COPY -- and the rebuilt chunks must still match byte for
    byte."""
    rng = np.random.default_rng(17)
    nt = 9
    files = []
    for i in range(60):
        holders, p = S.random_layout(rng, nt, int(rng.integers(2, 9)))
        files.append((f"p/{i % 4}/c{i}", holders, p, [int(x) for x in rng.integers(1, 1 * MiB, size=len(holders))]))
    root = str(tmp_path)
    items, contents = S.populate(root, nt, files, seed=19)
    want_mode = {"copy": bcp.READ_COPY, "direct": bcp.READ_DIRECT}[mode]
    victim = 3
    ns = {len(h) for _, h, _, _ in files if victim in h}   # rebuild sources: survivors + parity body
    assert {3, 5, 7} <= ns, ns
    pl = bcp.Pipeline(slab_bytes=4 << 20, io_threads=2, nslots=2, read_mode=want_mode)
    try:
        st = pl.run(root, nt, items)
        assert st.errors == 0 and st.tasks == len(files)
        for path, holders, p, lens in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        lost = {path: S.read_file(S.chunk_path(root, victim, path)) for path, holders, _, _ in files
                if victim in holders}
        for path in lost:
            os.remove(S.chunk_path(root, victim, path))
        st = pl.rebuild(root, nt, victim, sorted(items, key=lambda x: x[0].encode()))
        assert st.errors == 0 and st.tasks == len(lost)
        assert pl.last_timing()["read_mode"] == want_mode
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, path
    finally:
        pl.close()


def _resident_fraction(paths):
    """Page-cache residency of files: mincore over a read-only mapping of each
    (mapping does not fault the pages in)."""
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.mincore.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p]
    PROT_READ, MAP_SHARED = 1, 1
    pages = resident = 0
    for p in paths:
        n = os.path.getsize(p)
        if not n:
            continue
        fd = os.open(p, os.O_RDONLY)
        addr = libc.mmap(None, n, PROT_READ, MAP_SHARED, fd, 0)
        os.close(fd)
        if addr in (None, ctypes.c_void_p(-1).value):
            continue
        np_ = (n + 4095) // 4096
        vec = ctypes.create_string_buffer(np_)
        if libc.mincore(addr, n, vec) == 0:
            pages += np_
            resident += sum(b & 1 for b in vec.raw[:np_])
        libc.munmap(addr, n)
    return resident / pages if pages else 1.0


def test_pipeline_auto_read_path_follows_the_page_cache(bcp, oracle, tmp_path, monkeypatch):
    """read_mode AUTO picks per run: COPY while the chunks are in the page
    cache (just written) or on tmpfs, DIRECT once they are not (written back
    and dropped: a cold store on a disk) -- the same parity files either way
    (bcp_pipeline_timing.read_mode says which path ran)."""
    monkeypatch.delenv("BCP_PIPELINE_READ", raising=False)
    rng = np.random.default_rng(5)
    nt = 9
    files = []
    for i in range(24):
        holders, p = S.random_layout(rng, nt, 8)
        files.append((f"a/{i % 3}/c{i}", holders, p, [int(x) for x in rng.integers(1, 2 * MiB, size=8)]))
    stores = {"disk": str(tmp_path / "store")}
    if os.path.isdir("/dev/shm"):
        stores["shm"] = f"/dev/shm/bcp_auto_{os.getpid()}"
    pl = bcp.Pipeline(slab_bytes=16 << 20, io_threads=4, nslots=3)
    try:
        for kind, root in stores.items():
            items, contents = S.populate(root, nt, files, seed=8)
            chunks = [S.chunk_path(root, h, path) for path, holders, _, _ in files for h in holders]
            for cold in (False, True):
                if cold:
                    for c in chunks:
                        fd = os.open(c, os.O_RDONLY)
                        os.fsync(fd)
                        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                        os.close(fd)
                frac = _resident_fraction(chunks)
                st = pl.run(root, nt, items)
                tm = pl.last_timing()
                print(f"auto read path: {kind} cold={cold} resident={frac:.2f} -> mode {tm['read_mode']}")
                assert st.errors == 0 and st.tasks == len(files)
                for path, holders, p, lens in files:
                    assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])
                if kind == "shm":
                    assert tm["read_mode"] == bcp.READ_COPY, (kind, cold, frac, tm)
                elif frac > 0.9:  # (a filesystem that keeps the pages, e.g. tmpfs: COPY;
                    # the decision samples a subset: clear cases only)
                    assert tm["read_mode"] == bcp.READ_COPY, (kind, cold, frac, tm)
                elif frac < 0.1:
                    assert tm["read_mode"] == bcp.READ_DIRECT, (kind, cold, frac, tm)
                    assert tm["direct_bytes"] > 0 or tm["direct_fallbacks"] > 0, tm
                assert tm["read_mode"] in (bcp.READ_COPY, bcp.READ_DIRECT)
            if kind == "shm":
                import shutil
                shutil.rmtree(root, ignore_errors=True)
    finally:
        pl.close()
        if "shm" in stores:
            import shutil
            shutil.rmtree(stores["shm"], ignore_errors=True)


@pytest.mark.usefixtures("read_path")
def test_pipeline_overwrites_shorter_parity_files_exactly(bcp, oracle, tmp_path):
    """Parity files are overwritten in place and cut to their new length: a
    second run after the chunks shrank (a partial round's changed chunks)
    leaves exactly the new file, no stale tail; a rebuilt chunk likewise."""
    root = str(tmp_path)
    files = [("o/a", [0, 1, 2], 3, [300_000, 200_000, 5]), ("o/b", [1, 2, 3], 0, [4 * MiB, 1, 70_000])]
    items, contents = S.populate(root, 4, files, seed=3)
    pl = bcp.Pipeline(io_threads=3)
    try:
        assert pl.run(root, 4, items).errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])
        # every chunk shorter now
        for (path, holders, p, lens) in files:
            for k, h in enumerate(holders):
                short = contents[path][k][: len(contents[path][k]) // 3]
                S.write_chunk(root, h, path, short)
                contents[path][k] = short
        assert pl.run(root, 4, items).errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        # a rebuilt chunk written over a longer stale file of the same name
        victim_path, holders, p, _ = files[1]
        stale = S.chunk_path(root, 2, victim_path)
        want = S.read_file(stale)
        with open(stale, "wb") as f:
            f.write(b"x" * (len(want) * 5 + 123))
        assert pl.rebuild(root, 4, 2, sorted(items, key=lambda x: x[0].encode())).errors == 0
        assert S.read_file(stale) == want
    finally:
        pl.close()
