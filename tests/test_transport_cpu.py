"""The transport seam under process_task, ranks as processes, and the
failure paths that used to abort -- host logic on the CPU (the P role's fold
is the test double of tests/native/cpu_xor_hook.c; no GPU).

* bcp_gen_run_procs / bcp_rebuild_run_procs: one forked process per storage
  target, socketpair transport (bcp_sock_world), parity files and rebuilds
  compared with the oracle -- including multi-window stripes (replay quirk
  A3-q1) and the corrupt list;
* the transport table: loopback installed explicitly, incomplete tables
  refused;
* failure injection: the P role without fold resources still drains its
  senders (one bounded row, or a 16 KiB truncating one) and raises the
  sticky error; a source without a window buffer sends zeros and raises it;
  a lane thread that cannot be created cancels the run before any task
  (-EAGAIN) -- in both runners, no abort, no hang.
"""
import os
import subprocess

import numpy as np
import pytest

import bcp_store as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KiB, MiB = 1024, 1024 * 1024


@pytest.fixture(autouse=True)
def _clean(bcp):
    yield
    for site in (bcp.INJECT_FOLD_RES, bcp.INJECT_DRAIN_ROW, bcp.INJECT_SEND_BUF, bcp.INJECT_THREAD,
                 bcp.INJECT_FOLD_SERVER, bcp.INJECT_PARITY_WRITE):
        bcp.inject_failure(site, 0, 0)
    bcp.set_transport(None)


def _random_files(rng, ntargets, nfiles, maxlen):
    files = []
    for i in range(nfiles):
        width = int(rng.integers(1, min(8, ntargets - 1) + 1))
        holders, p = S.random_layout(rng, ntargets, width)
        lens = [int(x) for x in rng.integers(0, maxlen, size=width)]
        files.append((f"p{i % 5}/{i:04x}/chunk{i}", holders, p, lens))
    return files


@pytest.mark.timeout(300)
@pytest.mark.parametrize("seed", range(2))
def test_rank_processes_gen_and_rebuild(bcp, oracle, cpu_hook, tmp_path, seed):
    rng = np.random.default_rng(700 + seed)
    ntargets = int(rng.integers(5, 10))
    files = _random_files(rng, ntargets, 40, 600_000)
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=seed)
    st = bcp.gen_run_procs(root, ntargets, items, nlanes=12)
    assert st.errors == 0
    assert st.tasks == sum(len(h) + 1 for (_, h, _, _) in files)
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    victim = int(rng.integers(0, ntargets))
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    corrupt = str(tmp_path / "corrupt.txt")
    st = bcp.rebuild_run_procs(root, ntargets, victim, items, corrupt_list=corrupt)
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path
    assert open(corrupt).read() == ""  # every survivor is older than its FileInfo timestamp


@pytest.mark.timeout(300)
def test_rank_processes_multiwindow_replay(bcp, oracle, cpu_hook, tmp_path):
    """Stripes above the 10 MiB window across processes: the socket transport
    carries the replayed windows (A3-q1) exactly as the loopback does."""
    root = str(tmp_path)
    files = [("big/a", [0, 1], 2, [10 * MiB, 25 * MiB + 5]), ("big/b", [1, 2, 3], 0, [3, 21 * MiB, 0])]
    items, contents = S.populate(root, 4, files, seed=3)
    st = bcp.gen_run_procs(root, 4, items, nlanes=2)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(300)
@pytest.mark.parametrize("explicit", [False, True], ids=["implicit-pad", "reference-wire"])
@pytest.mark.parametrize("procs", [False, True], ids=["threads", "rank-processes"])
def test_implicit_padding_never_folds_stale_row_bytes(bcp, oracle, cpu_hook, tmp_path, procs, explicit):
    """Gen with one window: sources send their chunk's bytes only (a shorter
    message on the socket transport, a shorter fill on the loopback) and the
    P role supplies the zeros past each chunk.  Large chunks first, then the
    same stripes with small / empty chunks next to large ones, so the reused
    window rows hold stale bytes exactly where the padding belongs.  Also
    with the reference's wire restored (bcp_task_set_explicit_padding)."""
    prev = bcp.set_explicit_padding(explicit)
    try:
        _padding_rounds(bcp, oracle, tmp_path, procs)
    finally:
        bcp.set_explicit_padding(prev)


def _padding_rounds(bcp, oracle, tmp_path, procs):
    rng = np.random.default_rng(31)
    root = str(tmp_path)
    ntargets = 6
    run = bcp.gen_run_procs if procs else bcp.gen_run
    big = []
    for i in range(30):
        holders, p = S.random_layout(rng, ntargets, 4)
        big.append((f"s/{i}", holders, p, [int(x) for x in rng.integers(700_000, 900_000, size=4)]))
    items, contents = S.populate(root, ntargets, big, seed=1)
    assert run(root, ntargets, items, nlanes=4).errors == 0
    small = [(path, holders, p, [int(rng.choice([0, 1, 17, 4096, 333_333])), 850_000,
                                 int(rng.integers(0, 5000)), 3])
             for (path, holders, p, _) in big]
    items, contents = S.populate(root, ntargets, small, seed=2)
    assert run(root, ntargets, items, nlanes=4).errors == 0
    for (path, holders, p, lens) in small:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(300)
def test_rank_pool_serves_many_runs(bcp, oracle, cpu_hook, tmp_path):
    """One pool of rank processes, several runs: gen, gen again over rewritten
    (smaller) chunks with the reference's padded wire switched on in between,
    a rebuild with its corrupt list, a gen on another store -- every result
    checked; the ranks' window rows and pools live across the runs."""
    rng = np.random.default_rng(88)
    nt = 6
    files = _random_files(rng, nt, 30, 500_000)
    root = str(tmp_path / "a")
    with bcp.RankPool(nt) as pool:
        items, contents = S.populate(root, nt, files, seed=1)
        st = pool.gen(root, items, nlanes=5)
        assert st.errors == 0 and st.tasks == sum(len(h) + 1 for (_, h, _, _) in files)
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        small = [(path, h, p, [max(0, L // 7 - 3) for L in lens]) for (path, h, p, lens) in files]
        items, contents = S.populate(root, nt, small, seed=2)
        prev = bcp.set_explicit_padding(True)  # taken by the ranks with the next run
        try:
            assert pool.gen(root, items, nlanes=3).errors == 0
        finally:
            bcp.set_explicit_padding(prev)
        for (path, holders, p, lens) in small:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        victim = 2
        lost = {}
        for (path, holders, p, lens) in small:
            if victim in holders:
                lost[path] = S.read_file(S.chunk_path(root, victim, path))
                os.remove(S.chunk_path(root, victim, path))
        corrupt = str(tmp_path / "corrupt.txt")
        assert pool.rebuild(root, victim, items, corrupt_list=corrupt).errors == 0
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, path
        assert open(corrupt).read() == ""
        root_b = str(tmp_path / "b")
        items_b, contents_b = S.populate(root_b, nt, files[:10], seed=3)
        assert pool.gen(root_b, items_b, nlanes=12).errors == 0
        for (path, holders, p, lens) in files[:10]:
            assert S.read_file(S.parity_path(root_b, p, path)) == oracle.gen_parity_file(contents_b[path]), path


@pytest.mark.timeout(120)
def test_rank_pool_broken_by_a_rank_that_cannot_start(bcp, cpu_hook, tmp_path):
    """Every rank fails to open a store that does not exist: the run fails
    (no hang), the pool refuses later runs (-EPIPE) and closes cleanly."""
    root, files, items, contents = _config(tmp_path, nfiles=6)
    pool = bcp.RankPool(6)
    try:
        with pytest.raises(bcp.BcpError) as ei:
            pool.gen(str(tmp_path / "missing"), items, nlanes=2)
        assert ei.value.rc in (-2, -10)  # -ENOENT from a rank, or -ECHILD
        with pytest.raises(bcp.BcpError) as ei:
            pool.gen(root, items, nlanes=2)
        assert ei.value.rc == -32  # -EPIPE
    finally:
        pool.close()


@pytest.mark.timeout(120)
def test_rank_pool_refuses_a_hook_loaded_after_the_fork(bcp, cpu_hook, tmp_path):
    """The hook is code of the caller's process: a library loaded after the
    ranks were forked is not mapped in them (-EFAULT, not a crash)."""
    import ctypes
    root, files, items, contents = _config(tmp_path, nfiles=4)
    with bcp.RankPool(6) as pool:
        src = tmp_path / "late.c"
        src.write_text("#include <stddef.h>\n#include <stdint.h>\nint late_fold(uint8_t *d, size_t n, const uint8_t"
                       " *s, size_t p, int k, void *c) { (void)d; (void)n; (void)s; (void)p; (void)k; (void)c;"
                       " return 0; }\n")
        so = tmp_path / "liblate.so"
        subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
        late = ctypes.CDLL(str(so))
        bcp.set_xor_hook(ctypes.cast(late.late_fold, ctypes.c_void_p).value)
        with pytest.raises(bcp.BcpError) as ei:
            pool.gen(root, items, nlanes=2)
        assert ei.value.rc in (-14, -10)  # -EFAULT from a rank, or -ECHILD


def test_explicit_loopback_transport_and_validation(bcp, oracle, cpu_hook, tmp_path):
    import ctypes
    L = bcp.lib()
    bcp.set_transport(L.bcp_lb_transport())
    root = str(tmp_path)
    files = [(f"x/{i}", [0, 1, 2], 3, [100_000 + i, 64 * KiB, 7]) for i in range(6)]
    items, contents = S.populate(root, 4, files, seed=1)
    st = bcp.gen_run(root, 4, items)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path])
    # a table without its mandatory entries is refused
    empty = (ctypes.c_void_p * 8)()
    assert L.bcp_task_set_transport(ctypes.addressof(empty)) == -22


def _config(tmp_path, seed=5, nfiles=24):
    rng = np.random.default_rng(seed)
    files = _random_files(rng, 6, nfiles, 300_000)
    root = str(tmp_path)
    items, contents = S.populate(root, 6, files, seed=seed)
    return root, files, items, contents


@pytest.mark.timeout(200)
@pytest.mark.parametrize("spin_us", [0, 3, 200])
def test_loopback_spin_waits_give_the_same_files(bcp, oracle, cpu_hook, tmp_path, spin_us):
    """The loopback transport's receives and fill sends poll for spin_us
    before they sleep (lb_spin_us): gen (12 lanes, mixed sizes, multi-window
    stripes) and a rebuild give the oracle's files whatever the budget."""
    rng = np.random.default_rng(41)
    files = _random_files(rng, 6, 30, 300_000)
    files.append(("w/big", [0, 2], 4, [10 * MiB + 7, 3 * MiB]))  # two windows, the second replays
    root = str(tmp_path)
    items, contents = S.populate(root, 6, files, seed=41)
    old = bcp.set_fold_tuning("lb_spin_us", spin_us)
    try:
        assert bcp.gen_run(root, 6, items, nlanes=12).errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        victim = 2
        for (path, holders, p, lens) in files:
            if victim in holders:
                os.remove(S.chunk_path(root, victim, path))
        assert bcp.rebuild_run(root, 6, victim, items).errors == 0
        for (path, holders, p, lens) in files:
            if victim in holders:
                assert S.read_file(S.chunk_path(root, victim, path)) == bytes(contents[path][holders.index(victim)])
    finally:
        bcp.set_fold_tuning("lb_spin_us", old)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("drain_row", [True, False], ids=["one-row-drain", "16KiB-truncating-drain"])
def test_p_role_without_resources_drains_and_raises(bcp, oracle, cpu_hook, tmp_path, drain_row):
    root, files, items, contents = _config(tmp_path)
    bcp.inject_failure(bcp.INJECT_FOLD_RES, 0, 1)
    if not drain_row:
        bcp.inject_failure(bcp.INJECT_DRAIN_ROW, 0, 1)
    st = bcp.gen_run(root, 6, items, nlanes=4)  # returns: no hang, no abort
    assert st.errors == 1  # exactly the rank whose P role had no resources
    bad = 0
    for (path, holders, p, lens) in files:
        f = S.parity_path(root, p, path)
        if os.path.exists(f) and S.read_file(f) == oracle.gen_parity_file(contents[path]):
            continue
        bad += 1
    # the failing rank's parity files (that task and its later ones) are missing;
    # every other rank's are exact
    assert 1 <= bad < len(files)


@pytest.mark.timeout(120)
def test_parity_write_failure_is_sticky_on_its_rank(bcp, oracle, cpu_hook, tmp_path):
    """The P role's parity write fails (ENOSPC, injected) on one task: its
    rank's error is sticky (that rank's later parity files go to the null
    device), every other rank's files are exact, and the next run is clean."""
    root, files, items, contents = _config(tmp_path)
    bcp.inject_failure(bcp.INJECT_PARITY_WRITE, 3, 1)
    st = bcp.gen_run(root, 6, items, nlanes=4)
    assert st.errors == 1
    good = sum(1 for (path, holders, p, lens) in files
               if os.path.exists(S.parity_path(root, p, path))
               and S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]))
    assert 1 <= len(files) - good < len(files)
    bcp.inject_failure(bcp.INJECT_PARITY_WRITE, 0, 0)
    assert bcp.gen_run(root, 6, items, nlanes=4).errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(120)
def test_source_without_buffer_sends_zeros_and_raises(bcp, oracle, cpu_hook, tmp_path):
    """The buffered source path (a window that could be replayed) with its
    buffer allocation failing: zeros go out, the rank's error is sticky."""
    root = str(tmp_path)
    files = [("w/a", [0, 1], 2, [10 * MiB + 1, 21 * MiB])]
    items, contents = S.populate(root, 3, files, seed=2)
    bcp.inject_failure(bcp.INJECT_SEND_BUF, 0, 1)
    st = bcp.gen_run(root, 3, items, nlanes=1)
    assert st.errors == 1
    # the P role still wrote a parity file: chunk 0's stream was zeros
    pf = S.read_file(S.parity_path(root, 2, "w/a"))
    hdr = np.frombuffer(pf[:16], "<u8").tolist()
    assert hdr == [10 * MiB + 1, 21 * MiB]
    body = np.frombuffer(pf[16:], np.uint8)
    assert body.tobytes() == oracle.gen_parity_file([contents["w/a"][1]])[8:]


@pytest.mark.timeout(120)
@pytest.mark.parametrize("after", [0, 5, 17])
def test_lane_thread_failure_cancels_before_any_task(bcp, cpu_hook, tmp_path, after):
    root, files, items, contents = _config(tmp_path, nfiles=10)
    bcp.inject_failure(bcp.INJECT_THREAD, after, 1)
    with pytest.raises(bcp.BcpError) as ei:
        bcp.gen_run(root, 6, items, nlanes=4)
    assert ei.value.rc == -11  # -EAGAIN
    assert not any(os.path.exists(S.parity_path(root, p, path)) for (path, _, p, _) in files)
    bcp.inject_failure(bcp.INJECT_THREAD, min(after, 3), 1)  # the rebuild starts one thread per rank
    with pytest.raises(bcp.BcpError) as ei:
        bcp.rebuild_run(root, 6, 0, items)
    assert ei.value.rc == -11
    # and the library is usable afterwards
    bcp.inject_failure(bcp.INJECT_THREAD, 0, 0)
    assert bcp.gen_run(root, 6, items, nlanes=4).errors == 0


@pytest.mark.timeout(120)
def test_rank_process_failure_is_reported_not_hung(bcp, cpu_hook, tmp_path):
    """One rank process cannot start its lanes (injected before the fork, so
    the first child to create lane 3 fails): it exits, its partners see its
    sockets close and fail their shared tasks, the run returns an error."""
    root, files, items, contents = _config(tmp_path, nfiles=10)
    bcp.inject_failure(bcp.INJECT_THREAD, 2, 1)  # inherited by every child: each fails its 3rd lane
    with pytest.raises(bcp.BcpError) as ei:
        bcp.gen_run_procs(root, 6, items, nlanes=4)
    assert ei.value.rc in (-11, -10)  # -EAGAIN from a rank, or -ECHILD


@pytest.mark.timeout(200)
def test_caller_defined_st2rank_and_hoststate(bcp, tmp_path):
    """A C caller shaped like gen/main.c: its own int st2rank[56] and
    HostState, sizeof/offsetof of FileInfo / TaskInfo / HostState checked
    against the reference's layout, ranks as forked processes on the
    socketpair transport calling process_task directly, parity checked."""
    exe = tmp_path / "caller"
    lib = bcp.LIB_PATH  # the product library (or its sanitizer build under tools/asan_host.sh)
    san = ["-fsanitize=address,undefined"] if "asan" in os.path.basename(lib) else []
    subprocess.run(["gcc", "-std=gnu99", "-O1", "-Wall", "-Werror", "-pthread", *san, "-I",
                    os.path.join(ROOT, "include"), "-o", str(exe), os.path.join(ROOT, "tests", "native", "caller_test.c"),
                    lib, f"-Wl,-rpath,{os.path.dirname(lib)}"], check=True)
    r = subprocess.run([str(exe), str(tmp_path / "store")], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "caller_test ok" in r.stdout


def _fill_counts(path):
    arena = msg = srv = 0
    for line in open(path):
        if "fill sends" in line:
            # "rank k: fill sends A into arena rows, M as messages; S windows folded by the server"
            w = line.split()
            arena += int(w[4])
            msg += int(w[8])
            srv += int(w[11])
    return arena, msg, srv


@pytest.mark.timeout(300)
@pytest.mark.parametrize("arena_mb,server", [("2048", "0"), ("0", "0"), ("2048", "1"), ("0", "1")],
                         ids=["arena", "no-arena", "arena-fold-server", "no-arena-no-server"])
def test_rank_processes_fill_into_shared_rows(bcp, oracle, cpu_hook, tmp_path, monkeypatch, arena_mb, server):
    """Rank processes with the shared row arena (bcp_sock.c): every
    single-window source reads its chunk straight into the P role's row in
    the arena (RTS / CTS / DONE over the sockets, no payload through them);
    multi-window stripes with replay (A3-q1) still go as messages.  Without
    the arena (BCP_SOCK_ARENA_MB=0) no fill sends at all.  With the node
    fold server (BCP_FOLD_SERVER=1, arena only) every P role's window goes to
    the server process over its connections (here it folds with the test
    double it inherited).  Parity and a rebuild equal the oracle each way."""
    import ctypes
    monkeypatch.setenv("BCP_SOCK_STATS", "1")
    monkeypatch.setenv("BCP_SOCK_ARENA_MB", arena_mb)
    monkeypatch.setenv("BCP_FOLD_SERVER", server)
    rng = np.random.default_rng(77)
    root = str(tmp_path / "store")
    ntargets = 5
    files = _random_files(rng, ntargets, 40, 700_000)
    files.append(("big/r", [0, 3], 1, [10 * MiB + 3, 21 * MiB]))
    items, contents = S.populate(root, ntargets, files, seed=5)
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    logp = str(tmp_path / "ranks.log")
    f = libc.fopen(logp.encode(), b"w")
    try:
        st = bcp.gen_run_procs(root, ntargets, items, nlanes=3, log=f)
    finally:
        libc.fclose(f)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    arena, msg, srv = _fill_counts(logp)
    if arena_mb == "0":
        assert arena == 0 and msg == 0 and srv == 0
    else:
        assert arena >= sum(len(h) for (_, h, _, _) in files[:-1]) and msg == 0
        # with the server every window goes to it: one per window of every
        # stripe with a source (the 21 MiB one has 3)
        assert srv == (len([f for f in files if f[1]]) + 2 if server == "1" else 0)
    victim = 2
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    st = bcp.rebuild_run_procs(root, ntargets, victim, items)
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


@pytest.mark.timeout(300)
def test_fold_server_losing_a_connection_fails_tasks_not_the_run(bcp, oracle, cpu_hook, tmp_path, monkeypatch):
    """The node fold server drops a rank's connection instead of answering
    (failure injection, taken by the server when the pool forks it): the
    lanes folding through it get EPIPE -- no SIGPIPE, no hang --, their P
    roles raise the sticky error and the run ends with errors.  A new pool
    (a new server) then writes every parity file correctly."""
    monkeypatch.setenv("BCP_FOLD_SERVER", "1")
    rng = np.random.default_rng(91)
    root = str(tmp_path)
    ntargets = 5
    files = _random_files(rng, ntargets, 30, 300_000)
    items, contents = S.populate(root, ntargets, files, seed=4)
    bcp.inject_failure(bcp.INJECT_FOLD_SERVER, 3, 1)
    prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)  # every window through the server
    try:
        st = bcp.gen_run_procs(root, ntargets, items, nlanes=3)
    finally:
        bcp.set_fold_mode(prev)
    assert st.errors > 0
    bcp.inject_failure(bcp.INJECT_FOLD_SERVER, 0, 0)
    st = bcp.gen_run_procs(root, ntargets, items, nlanes=3)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(300)
def test_rank_processes_wide_world(bcp, oracle, cpu_hook, tmp_path):
    """A pool of 32 storage targets (33 rank processes, ~4,200 socket ends
    before fork with the fold server's connections -- beyond a default soft
    descriptor limit, which the world raises to the hard one): 16-wide
    stripes through every rank, parity against the oracle."""
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if hard != resource.RLIM_INFINITY and hard < 6000:
        pytest.skip(f"hard descriptor limit {hard}")
    rng = np.random.default_rng(5150)
    root = str(tmp_path)
    nt = 32
    files = []
    for i in range(24):
        holders, p = S.random_layout(rng, nt, 16)
        files.append((f"w/{i}", holders, p, [int(x) for x in rng.integers(0, 40_000, size=16)]))
    items, contents = S.populate(root, nt, files, seed=9)
    st = bcp.gen_run_procs(root, nt, items, nlanes=2)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path


@pytest.mark.timeout(300)
@pytest.mark.parametrize("procs", [False, True], ids=["threads", "rank-processes"])
def test_rebuild_lanes(bcp, oracle, cpu_hook, tmp_path, procs):
    """bcp_task_set_rebuild_lanes(4): item i on lane i % 4 with tag i % 4 on
    every rank; the rebuilt chunks and the corrupt list (as a set of lines)
    equal the single-lane rebuild's."""
    rng = np.random.default_rng(4242)
    ntargets = 6
    files = _random_files(rng, ntargets, 40, 400_000)
    files.append(("big/r", [0, 2, 4], 5, [10 * MiB + 7, 3, 12 * MiB]))
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=12, timestamp=0)  # every chunk newer: all corrupt
    assert (bcp.gen_run_procs if procs else bcp.gen_run)(root, ntargets, items, nlanes=3).errors == 0
    victim = 2
    lost = {path: S.read_file(S.chunk_path(root, victim, path)) for (path, h, p, lens) in files if victim in h}
    results = {}
    for lanes in (1, 4):
        for path in lost:
            os.remove(S.chunk_path(root, victim, path))
        prev = bcp.set_rebuild_lanes(lanes)
        try:
            corrupt = str(tmp_path / f"corrupt{lanes}.txt")
            st = (bcp.rebuild_run_procs if procs else bcp.rebuild_run)(root, ntargets, victim, items,
                                                                         corrupt_list=corrupt)
        finally:
            bcp.set_rebuild_lanes(prev)
        assert st.errors == 0 and st.tasks > 0
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, (lanes, path)
        results[lanes] = sorted(open(corrupt).read().splitlines())
    assert results[1] and results[1] == results[4]
    with pytest.raises(bcp.BcpError):
        bcp.set_rebuild_lanes(0)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("pad,expect", [("auto", "foreign_wire ok"), ("implicit", "foreign_wire mismatch")])
def test_foreign_transport_gets_the_reference_wire(bcp, tmp_path, pad, expect):
    """libbcp senders through a caller's transport table (an MPI binding's
    shape) to a P role shaped like the reference's parity_generator, which
    folds whole buffer_size rows it never clears (task_processing.c:176-211):
    by default (BCP_PAD_AUTO) the senders use the reference's zero-padded
    windows (:302-303) through such a table and every parity is exact; with
    implicit padding forced the stale row bytes are folded (the hazard)."""
    exe = tmp_path / "fw"
    lib = bcp.LIB_PATH
    san = ["-fsanitize=address,undefined"] if "asan" in os.path.basename(lib) else []
    subprocess.run(["gcc", "-std=gnu99", "-O1", "-Wall", "-Werror", "-pthread", *san, "-I",
                    os.path.join(ROOT, "include"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "foreign_wire_test.c"), lib,
                    f"-Wl,-rpath,{os.path.dirname(lib)}"], check=True)
    r = subprocess.run([str(exe), str(tmp_path / "store"), pad], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == expect, r.stdout + r.stderr


def test_sock_world_raises_nofile_only_as_needed_and_restores_it(bcp):
    """bcp_sock_world_create raises the soft RLIMIT_NOFILE only as far as the
    live worlds' socket ends need (not to the hard limit), and the last
    bcp_sock_world_destroy restores the caller's limit."""
    import ctypes
    import resource
    L = bcp.lib()
    L.bcp_sock_world_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    L.bcp_sock_world_destroy.argtypes = [ctypes.c_void_p]
    soft0, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    low = min(soft0, 1024)
    resource.setrlimit(resource.RLIMIT_NOFILE, (low, hard))
    try:
        worlds = []
        for n in (30, 20):  # 2*30*29 + 2*20*19 ends: beyond 1,024
            w = ctypes.c_void_p()
            assert L.bcp_sock_world_create(n, ctypes.byref(w)) == 0
            worlds.append(w)
        soft1, _ = resource.getrlimit(resource.RLIMIT_NOFILE)
        need = 2 * 30 * 29 + 2 * 20 * 19
        assert soft1 >= min(hard, low + need)
        assert soft1 <= low + need + 256 or hard <= low + need + 256
        for w in worlds:
            assert L.bcp_sock_world_destroy(w) == 0
        assert resource.getrlimit(resource.RLIMIT_NOFILE)[0] == low
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft0, hard))


@pytest.mark.timeout(200)
def test_caller_transport_table_gen_and_rebuild(bcp, oracle, cpu_hook, foreign_ops_addr, tmp_path):
    """process_task over a caller's transport table (an MPI binding's shape:
    no send_fill): the sources send the reference's padded windows (the
    default for a foreign table), the P role folds whole windows through the
    fold service, multi-window stripes replay -- parity and rebuild exact."""
    rng = np.random.default_rng(606)
    nt = 7
    files = []
    for i in range(30):
        holders, p = S.random_layout(rng, nt, int(rng.integers(1, 6)))
        lens = [int(x) for x in rng.integers(0, 900_000, size=len(holders))]
        files.append((f"f/{i % 3}/c{i}", holders, p, lens))
    files[0] = ("f/big", [0, 1], 2, [10 * 1024 * 1024, 25 * 1024 * 1024 + 5])
    root = str(tmp_path)
    items, contents = S.populate(root, nt, files, seed=61)
    bcp.set_transport(foreign_ops_addr)
    try:
        assert bcp.gen_run(root, nt, items, nlanes=4).errors == 0
        for (path, holders, p, lens) in files:
            assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
        victim = 1
        lost = {}
        for (path, holders, p, lens) in files:
            if victim in holders:
                lost[path] = S.read_file(S.chunk_path(root, victim, path))
                os.remove(S.chunk_path(root, victim, path))
        assert bcp.rebuild_run(root, nt, victim, items).errors == 0
        for path, data in lost.items():
            assert S.read_file(S.chunk_path(root, victim, path)) == data, path
    finally:
        bcp.set_transport(None)
