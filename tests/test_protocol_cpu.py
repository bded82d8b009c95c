"""Host-layer tests without a GPU: process_task over loopback ranks
(bcp_gen_run / bcp_rebuild_run) with the P role's fold routed through a test
double (tests/native/cpu_xor_hook.c).  Output files are compared with the
oracle's restatement of the reference protocol and with the survey KATs.
The GPU-folded runs of the same drivers are in tests/test_gpu_protocol.py."""
import ctypes
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

import bcp_store as S

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "kats.json")))
MiB = 1024 * 1024


def parity_of(root, p_st, path):
    return S.read_file(S.parity_path(root, p_st, path))


def test_kat2_through_protocol(bcp, oracle, cpu_hook, tmp_path):
    """KAT-2: 9 targets, chunk k on target k, P = 8, path a/b/chunk1."""
    k = GOLD["survey_kats"]["KAT-2"]
    root = str(tmp_path)
    S.make_store(root, 9)
    chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(k["lens"])]
    for i, c in enumerate(chunks):
        S.write_chunk(root, i, "a/b/chunk1", c)
    items = [("a/b/chunk1", 2**40, S.with_p(0xFF, 8))]
    st = bcp.gen_run(root, 9, items)
    pf = parity_of(root, 8, "a/b/chunk1")
    assert len(pf) == k["file_len"] and hashlib.sha256(pf).hexdigest() == k["sha256"]
    assert st.errors == 0 and st.tasks == 9
    # lose target 3, rebuild it
    os.remove(S.chunk_path(root, 3, "a/b/chunk1"))
    st = bcp.rebuild_run(root, 9, 3, items, corrupt_list=str(tmp_path / "corrupt"))
    assert S.read_file(S.chunk_path(root, 3, "a/b/chunk1")) == chunks[3].tobytes()
    assert st.errors == 0
    assert open(tmp_path / "corrupt").read() == ""


@pytest.mark.parametrize("name", ["KAT-3", "KAT-4"])
def test_mixed_and_multiwindow_kats_through_protocol(bcp, oracle, cpu_hook, tmp_path, name):
    k = GOLD["survey_kats"][name]
    root = str(tmp_path)
    n = len(k["lens"])
    p = 8 if n == 8 else 4
    S.make_store(root, max(9, p + 1))
    chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(k["lens"])]
    for i, c in enumerate(chunks):
        S.write_chunk(root, i, "x/y", c)
    items = [("x/y", 2**40, S.with_p((1 << n) - 1, p))]
    bcp.gen_run(root, max(9, p + 1), items, nlanes=3)
    pf = parity_of(root, p, "x/y")
    assert len(pf) == k["file_len"] and hashlib.sha256(pf).hexdigest() == k["sha256"]
    v = k["rebuild_victim"]
    os.remove(S.chunk_path(root, v, "x/y"))
    bcp.rebuild_run(root, max(9, p + 1), v, items)
    assert S.read_file(S.chunk_path(root, v, "x/y")) == chunks[v].tobytes()


@pytest.mark.parametrize("seed", range(3))
def test_random_worklist_gen_and_rebuild(bcp, oracle, cpu_hook, tmp_path, seed):
    rng = np.random.default_rng(seed)
    ntargets = int(rng.integers(4, 12))
    files = []
    for i in range(40):
        width = int(rng.integers(1, min(8, ntargets - 1) + 1))
        holders, p = S.random_layout(rng, ntargets, width)
        lens = [int(x) for x in rng.integers(0, 300_000, size=width)]
        files.append((f"d{i % 5}/sub{i % 3}/file{i}", holders, p, lens))
    root = str(tmp_path)
    items, contents = S.populate(root, ntargets, files, seed=seed)
    st = bcp.gen_run(root, ntargets, items, nlanes=12)
    assert st.errors == 0
    for (path, holders, p, lens) in files:
        assert parity_of(root, p, path) == oracle.gen_parity_file(contents[path]), path
    victim = int(rng.integers(0, ntargets))
    lost = {}
    for (path, holders, p, lens) in files:
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    bcp.rebuild_run(root, ntargets, victim, items)
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


def test_assign_lanes_matches_reference_semantics(bcp):
    """Greedy lane assignment (gen/assign_lanes.c:12-46): restated here in
    Python independently and compared, including NO_P items."""
    rng = np.random.default_rng(3)
    locs = []
    for _ in range(300):
        loc = int(rng.integers(1, 1 << 20))
        p = 0xFF if rng.random() < 0.1 else int(rng.integers(20, 40))
        locs.append(S.with_p(loc, p))
    got = bcp.assign_lanes(12, locs)

    def ref(nlanes, locs):
        prev = [0] * (nlanes * 16)
        offs = [0] * nlanes
        out = []
        for i, x in enumerate(locs):
            p = x >> 56
            bit = (1 << (p & 31))
            if bit & 0x80000000:  # int sign-extension into the u64 mask
                bit |= 0xFFFFFFFF00000000
            tgt = (x & ((1 << 56) - 1)) | bit
            lo = i % nlanes
            best, best_d = lo, 0
            for j0 in range(nlanes):
                j = (lo + j0) % nlanes
                d = 16
                for k in range(16):
                    if tgt & prev[j * 16 + ((offs[j] + k) & 15)]:
                        d = 16 - k
                if d > best_d:
                    best_d, best = d, j
            out.append(best)
            prev[best * 16 + offs[best]] = tgt
            offs[best] = (offs[best] + 1) & 15
        return out
    assert got == ref(12, locs)


def test_delete_task_unlinks_parity(bcp, cpu_hook, tmp_path):
    root = str(tmp_path)
    items, contents = S.populate(root, 4, [("f", [0, 1], 3, [1000, 2000])])
    bcp.gen_run(root, 4, items)
    assert os.path.exists(S.parity_path(root, 3, "f"))
    # every chunk gone: locations 0 with P kept -> parity chunk unlinked (:141-144)
    st = bcp.gen_run(root, 4, [("f", 0, S.with_p(0, 3))])
    assert not os.path.exists(S.parity_path(root, 3, "f"))
    assert st.tasks == 0


def test_missing_chunk_sends_zeros_and_size_zero(bcp, oracle, cpu_hook, tmp_path):
    root = str(tmp_path)
    items, contents = S.populate(root, 5, [("g/h", [0, 1, 2], 4, [5000, 7000, 3000])])
    os.remove(S.chunk_path(root, 1, "g/h"))  # ENOENT: tolerated, zeros sent
    st = bcp.gen_run(root, 5, items)
    pf = parity_of(root, 4, "g/h")
    assert pf == oracle.gen_parity_file([contents["g/h"][0], None, contents["g/h"][2]])
    assert st.errors == 0  # ENOENT is not escalated


def test_no_p_items_are_skipped(bcp, cpu_hook, tmp_path):
    root = str(tmp_path)
    items, _ = S.populate(root, 4, [("k", [0, 1], 2, [100, 100])])
    items = [(p, ts, S.with_p(loc, 0xFF)) for (p, ts, loc) in items]
    st = bcp.gen_run(root, 4, items)
    assert st.tasks == 0
    assert not os.path.exists(S.parity_path(root, 2, "k"))


def test_rebuild_skip_rules_and_corrupt_list(bcp, oracle, cpu_hook, tmp_path):
    root = str(tmp_path)
    files = [("a", [0, 1, 2], 3, [4000, 4000, 10]),   # victim 1 holds a chunk -> rebuilt
             ("b", [0, 2], 1, [300, 300]),            # victim is P -> skipped (parity stays lost)
             ("c", [0, 2], 3, [300, 300])]            # victim not involved -> skipped
    items, contents = S.populate(root, 4, files, timestamp=1000)
    bcp.gen_run(root, 4, items)
    # survivors newer than the timestamp land in the corrupt list (:268-271);
    # populate() wrote them "now", far after timestamp 1000
    a_orig = S.read_file(S.chunk_path(root, 1, "a"))
    os.remove(S.chunk_path(root, 1, "a"))
    st = bcp.rebuild_run(root, 4, 1, items, corrupt_list=str(tmp_path / "corrupt.txt"))
    assert S.read_file(S.chunk_path(root, 1, "a")) == a_orig
    assert st.tasks == 4  # item "a" only: the victim (P role), survivors 0 and 2, parity holder 3
    corrupt = sorted(open(tmp_path / "corrupt.txt").read().split())
    assert corrupt == ["a", "a"]  # targets 0 and 2 (chunks), not the parity holder


@pytest.mark.parametrize("bad", ["../outside/x", "/abs/x", "a/../../outside/x"])
def test_paths_outside_the_store_are_refused_by_every_rank(bcp, oracle, cpu_hook, tmp_path, bad):
    """process_task refuses a path that would leave the targets' chunks /
    parity directories -- on every rank, so the task is skipped everywhere
    (nothing unanswered) and the next task runs; the reference trusts its
    worklist here."""
    root = str(tmp_path)
    items, contents = S.populate(root, 4, [("ok", [0, 1], 2, [5000, 7000])])
    for h in (0, 1):  # the chunks the escaping path would read, if it were taken
        os.makedirs(os.path.join(root, f"st{h}", "outside"), exist_ok=True)
        with open(os.path.join(root, f"st{h}", "outside", "x"), "wb") as f:
            f.write(b"z" * 100)
    items = [(bad, 2**40, S.with_p(0b11, 2))] + items
    st = bcp.gen_run(root, 4, items, nlanes=1)
    assert st.errors == 0 and st.tasks == 3  # "ok" only: P 2 and sources 0, 1
    assert st.refused == 1  # reported to the caller, not only logged
    assert parity_of(root, 2, "ok") == oracle.gen_parity_file(contents["ok"])
    assert not os.path.exists(os.path.join(root, "st2", "outside"))
    os.remove(S.chunk_path(root, 1, "ok"))
    st = bcp.rebuild_run(root, 4, 1, items)
    assert st.errors == 0 and S.read_file(S.chunk_path(root, 1, "ok")) == contents["ok"][1].tobytes()
    assert st.refused == 1
    assert S.read_file(os.path.join(root, "st1", "outside", "x")) == b"z" * 100


def test_refused_paths_get_no_db_entry(bcp, oracle, cpu_hook, tmp_path):
    """With the persistent state (process_list's pdb_set, gen/main.c:146-149):
    a refused item got no parity, so no replica may record it as protected
    (a later rebuild would refuse it too and the chunk would be lost
    silently); the caller sees it in stats.refused."""
    root = str(tmp_path)
    items, contents = S.populate(root, 4, [("ok", [0, 1], 2, [5000, 7000])])
    items = [("../outside/x", 2**40, S.with_p(0b11, 2)), ("/abs/y", 2**40, S.with_p(0b101, 1))] + items
    st = bcp.gen_run_db(root, 4, items, nlanes=2)
    assert st.errors == 0 and st.refused == 2
    for k in range(4):
        db = bcp.PDB(os.path.join(root, f"st{k}", "db"))
        try:
            assert len(db) == 1 and db.get("ok") is not None
            assert db.get("../outside/x") is None and db.get("/abs/y") is None
        finally:
            db.close()


def test_unreadable_parity_root_is_an_error(bcp, tmp_path):
    with pytest.raises(bcp.BcpError):
        bcp.gen_run(str(tmp_path / "missing"), 3, [("x", 0, S.with_p(1, 2))])


def test_invalid_items_rejected(bcp, tmp_path):
    S.make_store(str(tmp_path), 3)
    with pytest.raises(bcp.BcpError):   # P also a holder
        bcp.gen_run(str(tmp_path), 3, [("x", 0, S.with_p(0b101, 2))])
    with pytest.raises(bcp.BcpError):   # holder outside the world
        bcp.gen_run(str(tmp_path), 3, [("x", 0, S.with_p(0b1000, 2))])


def test_without_gpu_or_hook_the_p_role_fails_loudly(bcp, oracle, tmp_path):
    if bcp.device_count() > 0:
        pytest.skip("GPU present")
    root = str(tmp_path)
    items, _ = S.populate(root, 3, [("z", [0, 1], 2, [1000, 1000])])
    st = bcp.gen_run(root, 3, items)
    assert st.errors == 1                      # sticky ENODEV on the P rank
    assert not os.path.exists(S.parity_path(root, 2, "z"))
