"""Parity-generation rounds with the persistent state, on CPU (the P role's
fold routed through the test double tests/native/cpu_xor_hook.c):

  bcp_gen_run_db      process_list + pdb_set / pdb_del per task (gen/main.c:146-149)
  bcp_rebuild_run_db  pdb_iterate -> do_file (rebuild/main.c:223-225)
  bcp_gen_round       load DB, plan from chunk events, run (gen/main.c:716-797)

Worklists and P placement are checked against oracle/planner.py, parity files
against the oracle's restatement of the protocol."""
import os

import numpy as np
import pytest

import bcp_store as S
import planner as PL


def replica_items(bcp, root, k):
    db = bcp.PDB(os.path.join(root, f"st{k}", "db"))
    try:
        return db.items()
    finally:
        db.close()


def test_gen_run_db_updates_every_replica(bcp, cpu_hook, tmp_path):
    root = str(tmp_path)
    files = [("a/1", [0, 1], 3, [5000, 100]), ("a/2", [1, 2], 0, [10, 20]), ("b", [2], 1, [77])]
    items, _ = S.populate(root, 4, files, timestamp=500)
    items.append(("gone", 600, S.with_p(0, 2)))          # no holders left -> deleted from the DB
    items.append(("same", 700, S.with_p(0b11, PL.NO_P)))  # NO_P -> not processed, DB untouched
    bcp.gen_run_db(root, 4, items, nlanes=3)
    want = sorted((p.encode(), ts, loc) for p, ts, loc in items[:3])
    for k in range(4):
        assert replica_items(bcp, root, k) == want


@pytest.mark.parametrize("ranked", [False, True])
@pytest.mark.parametrize("seed", range(2))
def test_round_plan_run_update_and_rebuild(bcp, oracle, cpu_hook, tmp_path, seed, ranked):
    """ranked: the store names a permuted MPI rank order (<root>/rank_order),
    so the round plans its coordinators' rounds in that order -- the same
    items, files and DB state, another schedule."""
    rng = np.random.default_rng(seed)
    root = str(tmp_path)
    ntargets = int(rng.integers(4, 10))
    S.make_store(root, ntargets)
    if ranked:  # no targetNumID files: target k's id is k + 1
        order = [int(x) for x in rng.permutation(ntargets)]
        (tmp_path / "rank_order").write_text(" ".join(str(k + 1) for k in order))
        assert bcp.store_round_order(root, ntargets) == order
    cw = list(np.cumsum([int(x) for x in rng.integers(500, 7000, size=ntargets)]))
    files, contents, ts0 = {}, {}, 1_700_000_000
    streams = {k: [] for k in range(ntargets)}
    for i in range(30):
        path = f"u{i % 3}/{i:04X}/c{i}"
        width = int(rng.integers(1, min(6, ntargets - 1) + 1))
        holders = sorted(int(x) for x in rng.choice(ntargets, size=width, replace=False))
        lens = [int(x) for x in rng.integers(1, 200_000, size=width)]
        arrs = []
        for h, L in zip(holders, lens):
            d = S.synthetic_chunk(seed * 7919 + i * 31 + h, L)
            S.write_chunk(root, h, path, d)
            streams[h].append((ts0 + i, L, "m", path))
            arrs.append(d)
        files[path] = holders
        contents[path] = arrs

    def round_(streams):
        es = bcp.EventSet()
        for k, recs in streams.items():
            es.feed(k, bcp.pack_records(recs))
        st, n = bcp.gen_round(root, ntargets, es, cum_weight=cw, nlanes=4)
        es.close()
        return st, n

    def expected_plan(streams, prev):
        agg = PL.aggregate([(k, bcp.pack_records(r)) for k, r in streams.items()])
        return PL.plan(agg, ntargets, cw, prev)

    # round 1: every file new
    want = expected_plan(streams, {})
    st, n = round_(streams)
    assert st.errors == 0 and n == len(files)
    placed = {p.decode(): loc for p, _, loc in want}
    for path, holders in files.items():
        loc = placed[path]
        assert loc & PL.L_MASK == sum(1 << h for h in holders)
        p = PL.get_p(loc)
        assert p not in holders
        assert S.read_file(S.parity_path(root, p, path)) == oracle.gen_parity_file(contents[path]), path
    db_want = sorted((p, ts, loc) for p, ts, loc in want)
    for k in range(ntargets):
        assert replica_items(bcp, root, k) == db_want

    # round 2, same events: everything unchanged -> NO_P, nothing processed
    st, n = round_(streams)
    assert n == len(files) and st.tasks == 0

    # round 3: one chunk rewritten (newer event), one file deleted on every holder
    mod_path = "u1/0001/c1"
    h = files[mod_path][0]
    newdata = S.synthetic_chunk(99, 150_000)
    S.write_chunk(root, h, mod_path, newdata)
    contents[mod_path][0] = newdata
    del_path = "u2/0002/c2"
    streams3 = {k: [] for k in range(ntargets)}
    streams3[h].append((ts0 + 1000, 150_000, "m", mod_path))
    for hh in files[del_path]:
        streams3[hh].append((ts0 + 1001, 0, "d", del_path))
    prev = {p: (ts, loc) for p, ts, loc in replica_items(bcp, root, 0)}
    want3 = expected_plan(streams3, prev)
    del_p = PL.get_p(placed[del_path])
    st, n = round_(streams3)
    assert n == 2 and st.errors == 0
    p_mod = PL.get_p(dict((p.decode(), loc) for p, _, loc in want3)[mod_path])
    assert p_mod == PL.get_p(placed[mod_path])  # the DB keeps P where it was
    assert S.read_file(S.parity_path(root, p_mod, mod_path)) == oracle.gen_parity_file(contents[mod_path])
    assert not os.path.exists(S.parity_path(root, del_p, del_path))  # unlinked (task_processing.c:141-144)
    keys = [k for k, _, _ in replica_items(bcp, root, 0)]
    assert del_path.encode() not in keys and mod_path.encode() in keys
    for hh in files[del_path]:
        os.remove(S.chunk_path(root, hh, del_path))
    del files[del_path]

    # rebuild one target from the DB (key order), then compare the lost chunks
    victim = int(rng.integers(0, ntargets))
    lost = {}
    for path, holders in files.items():
        if victim in holders:
            lost[path] = S.read_file(S.chunk_path(root, victim, path))
            os.remove(S.chunk_path(root, victim, path))
    st = bcp.rebuild_run_db(root, ntargets, victim)
    assert st.errors == 0
    for path, data in lost.items():
        assert S.read_file(S.chunk_path(root, victim, path)) == data, path


def test_rebuild_without_db_is_an_error(bcp, tmp_path):
    S.make_store(str(tmp_path), 3)
    with pytest.raises(bcp.BcpError):
        bcp.rebuild_run_db(str(tmp_path), 3, 1)


def test_store_cum_weights(bcp, tmp_path):
    root = str(tmp_path)
    S.make_store(root, 3)
    (tmp_path / "st1" / "free_space.override").write_text("0")
    cw = bcp.store_cum_weights(root, 3)
    fd = os.open(str(tmp_path / "st0"), os.O_DIRECTORY | os.O_RDONLY)
    w0 = bcp.lib().bcp_store_weight(fd)
    os.close(fd)
    assert cw[0] == w0 and cw[1] == w0 + int(1000 * np.log2(0 + 1.1)) and cw[2] == cw[1] + w0
