"""BCP_FOLD_PIPELINED on the CPU (the P role's range folds go to the test
double of tests/native/cpu_xor_hook.c): sources filling a watched row read
their chunk in pieces and publish each final prefix; the P role folds every
range all rows have delivered while the rest is still being read.  Parity
and rebuilds against the oracle, the counters showing the ranges really
overlapped, the transports and windows it cannot follow (socket ranks,
multi-window stripes), the reference's padded wire, and a read error in
the middle of a chunk (the published prefix is refolded as zeros, the
reference's semantics for a failed read, task_processing.c:296-299)."""
import os

import numpy as np
import pytest

import bcp_store as S

KiB, MiB = 1024, 1024 * 1024


@pytest.fixture(autouse=True)
def pipelined(bcp, cpu_hook):
    prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
    yield
    bcp.set_fold_mode(prev)
    bcp.inject_failure(bcp.INJECT_READ, 0, 0)
    bcp.set_transport(None)
    # every row watch ended with its window (successful, failed or drained):
    # none may outlive it into memory a later task reuses
    assert bcp.lib().bcp_task_watch_live() == 0


@pytest.mark.timeout(120)
def test_row_watches_end_with_their_windows_on_failures(bcp, oracle, tmp_path):
    """Watches are removed on every path out of a pipelined window: fold
    resources missing (the P role drains), a read error mid-row, and normal
    completion -- then a run over the same (pooled) rows folds correctly."""
    root = str(tmp_path)
    files = [(f"q/{i}", [0, 1, 2], 3, [64 * KiB * (i + 1), 7, 300 * KiB]) for i in range(6)]
    items, contents = S.populate(root, 4, files, seed=9)
    bcp.inject_failure(bcp.INJECT_FOLD_RES, 2, 1)
    assert bcp.gen_run(root, 4, items, nlanes=2).errors >= 1
    bcp.inject_failure(bcp.INJECT_FOLD_RES, 0, 0)
    assert bcp.lib().bcp_task_watch_live() == 0
    bcp.inject_failure(bcp.INJECT_READ, 1, 1)
    assert bcp.gen_run(root, 4, items, nlanes=2).errors >= 1
    bcp.inject_failure(bcp.INJECT_READ, 0, 0)
    assert bcp.lib().bcp_task_watch_live() == 0
    assert bcp.gen_run(root, 4, items, nlanes=2).errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


def _files(rng, nt, nfiles, hi):
    files = []
    for i in range(nfiles):
        holders, p = S.random_layout(rng, nt, int(rng.integers(1, min(8, nt - 1) + 1)))
        lens = [int(x) for x in rng.integers(0, hi, size=len(holders))]
        files.append((f"pp/{i % 4}/c{i}", holders, p, lens))
    return files


@pytest.mark.timeout(300)
@pytest.mark.parametrize("explicit", [False, True], ids=["implicit-pad", "reference-wire"])
def test_pipelined_gen_and_rebuild(bcp, oracle, tmp_path, explicit):
    rng = np.random.default_rng(401)
    nt = 7
    files = _files(rng, nt, 40, 3 * MiB)
    files[0] = ("pp/big", [0, 1, 2], 3, [3 * MiB + 5, 2 * MiB, 1])
    files[1] = ("pp/tiny", [1, 4], 0, [0, 17])
    root = str(tmp_path)
    items, contents = S.populate(root, nt, files, seed=4)
    prev = bcp.set_explicit_padding(explicit)
    try:
        w0, r0 = bcp.pipe_stats()
        assert bcp.gen_run(root, nt, items, nlanes=6).errors == 0
        w1, r1 = bcp.pipe_stats()
    finally:
        bcp.set_explicit_padding(prev)
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    assert w1 - w0 == len(files) and r1 - r0 >= w1 - w0  # every window was followed
    victim = 2
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    assert bcp.rebuild_run(root, nt, victim, items).errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


@pytest.mark.timeout(300)
def test_pipelined_falls_back_where_it_cannot_follow(bcp, oracle, tmp_path):
    """Multi-window stripes (replay) fold whole windows like BATCHED; rank
    processes (socket transport, node fold server) fold whole windows
    through the server; the parity is the same."""
    root = str(tmp_path)
    files = [("w/a", [0, 1], 2, [10 * MiB, 25 * MiB + 5]), ("w/b", [0, 2], 1, [300 * KiB, 7])]
    items, contents = S.populate(root, 3, files, seed=5)
    assert bcp.gen_run(root, 3, items, nlanes=2).errors == 0
    assert bcp.gen_run_procs(root, 3, items, nlanes=2).errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(120)
def test_pipelined_folds_ranges_while_a_row_is_read(bcp, oracle, tmp_path):
    """One 4 MiB source read in 16 pieces beside two small rows: once the
    small rows are in, each piece's range is folded by the source that
    completed it while it reads the next (up to 17 range folds for the
    window); the parity is exact however the threads were scheduled (the
    overlap itself is measured on the device: tools/proto_compare.py
    reports range folds per window)."""
    root = str(tmp_path)
    items, contents = S.populate(root, 4, [("o/x", [0, 1, 2], 3, [7, 100 * KiB, 4 * MiB + 3])], seed=8)
    w0, r0 = bcp.pipe_stats()
    assert bcp.gen_run(root, 4, items, nlanes=1).errors == 0
    w1, r1 = bcp.pipe_stats()
    assert w1 - w0 == 1 and 1 <= r1 - r0 <= 17
    assert S.read_file(S.parity_path(root, 3, "o/x")) == oracle.gen_parity_file(contents["o/x"])


@pytest.mark.timeout(120)
@pytest.mark.parametrize("procs", [False, True], ids=["threads", "rank-processes"])
def test_pipelined_read_error_refolds_the_window(bcp, oracle, tmp_path, procs):
    """A 4 MiB source (read in 16 pieces) fails its twelfth piece after the
    ranges it published were folded, beside two small rows complete before
    it.  Its row becomes zeros (the reference zero-fills a
    window whose read failed) although its prefix was already folded: the P
    role refolds the whole window, the parity holds the XOR of the other
    rows, the source's rank is in error.  Rank processes (whole windows
    through the node fold server, one read per window): every rank's first
    read fails (each rank process inherits the injection), so every row
    arrives as zeros and so does the parity body."""
    root = str(tmp_path)
    lens = [7, 100 * KiB, 4 * MiB + 3]
    items, contents = S.populate(root, 4, [("e/x", [0, 1, 2], 3, lens)], seed=6)
    # threads: pieces 2..11 of the big row pass, the 12th fails
    bcp.inject_failure(bcp.INJECT_READ, 0 if procs else 10, 1)
    w0, r0 = bcp.pipe_stats()
    st = (bcp.gen_run_procs if procs else bcp.gen_run)(root, 4, items, nlanes=1)
    w1, r1 = bcp.pipe_stats()
    if procs:
        assert st.errors >= 1
    else:
        assert st.errors == 1
        assert w1 - w0 == 1 and r1 - r0 >= 1
    pf = S.read_file(S.parity_path(root, 3, "e/x"))
    assert np.frombuffer(pf[:24], "<u8").tolist() == lens  # the sizes were sent before the read
    body = np.frombuffer(pf[24:], np.uint8)
    expect = np.zeros(max(lens), np.uint8)
    for c in ([] if procs else contents["e/x"][:2]):  # a failed row folds as zeros
        expect[:c.size] ^= c
    assert np.array_equal(body, expect)
