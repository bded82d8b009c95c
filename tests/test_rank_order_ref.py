"""The coordinators' rounds in MPI rank order, pinned to
the reference's own code.

tests/golden/ref_rank.json (tests/golden/make_ref_rank_golden.py) holds the
outputs of the reference's target mapping -- gen/main.c:498-499, 506-541
compiled unchanged into oracle/_ref/ref_map_targets -- for permuted and grown
target lists, including its fatal checks, and 24 whole worklists whose rounds
follow such a list (ref_round_order_ranked around the reference's planner
functions).  libbcp's bcp_map_targets, bcp_plan_rounds_ordered and
bcp_assign_lanes_rounds must reproduce every one; where oracle/_ref exists,
fresh random target lists are compared with the reference program itself.
The store-level reading (<root>/rank_order) and bcp_check_targets' rule for
targets added since the last run are checked on temporary stores."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_store as S  # noqa: E402

FIX_PATH = os.path.join(ROOT, "tests", "golden", "ref_rank.json")  # CPU fixtures (not shipped to GPU boxes)
MAP_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_map_targets")
ERR = {"Fewer targets": -19, "Duplicate targetNumID": -17, "Storage target missing": -19}  # -ENODEV, -EEXIST


@pytest.fixture(scope="module")
def FIX():
    if not os.path.exists(FIX_PATH):
        pytest.skip("tests/golden/ref_rank.json not in this tree")
    with open(FIX_PATH) as f:
        return json.load(f)


def _map(bcp, prev, rank):
    try:
        return bcp.map_targets(prev, rank)
    except bcp.BcpError as e:
        return e.rc


def test_map_targets_fixtures(bcp, FIX):
    errors = 0
    for case in FIX["map"]:
        got = _map(bcp, case["prev"], case["rank"])
        if "error" in case:
            errors += 1
            want = next(rc for msg, rc in ERR.items() if case["error"].startswith(msg))
            assert got == want, case
        else:
            assert got == (case["st_ids"], case["round_st"]), case
            # st2rank: target i's eater is world rank 2r+1 for its rank position r
            assert [2 * got[1].index(k) + 1 for k in range(len(case["rank"]))] == case["st2rank"], case
    assert errors >= 4


def test_whole_worklists_in_rank_order(bcp, FIX):
    """Every fixture worklist: the same mapping, then the reference's order
    (rounds in rank order, each eater's shuffle + qsort), items, round
    bounds and the 12 lanes of every round."""
    kinds = set()
    for case in FIX["plan"]:
        nt, paths = case["ntargets"], case["paths"]
        kinds.add(case["kind"])
        st_ids, round_st = bcp.map_targets(case["prev_ids"], case["rank_ids"])
        assert (st_ids, round_st) == (case["st_ids"], case["round_st"])
        assert round_st != list(range(nt))  # the case is one the identity order would get wrong
        es = bcp.EventSet()
        try:
            for st, recs in case["streams"]:
                es.feed(st, bcp.pack_records([(ts, size, ev, paths[pi]) for ts, size, ev, pi in recs]))
            prev = [(paths[pi], ts, loc) for pi, ts, loc in case["prev"]]
            got, starts = es.plan_rounds(nt, case["cum_weight"], prev, round_st=round_st)
            ident, _ = es.plan_rounds(nt, case["cum_weight"], prev)
        finally:
            es.close()
        want = [(paths[pi], ts, loc) for pi, ts, loc in case["worklist"]]
        assert got == want
        assert starts == case["round_start"]
        assert bcp.assign_lanes_rounds(12, starts, [loc for _, _, loc in got]) == case["lanes12"]
        assert sorted(ident) == sorted(got) and ident != got  # same items, the reference's order only ranked
    assert kinds == {"permuted", "grown", "grown+permuted"}


def test_plan_rounds_ordered_refuses_a_non_permutation(bcp):
    import ctypes
    es = bcp.EventSet()
    try:
        es.feed(0, bcp.pack_records([(5, 100, "m", "a/b")]))
        for bad in ([0, 0, 1], [0, 1, 3], [-1, 0, 1]):
            with pytest.raises(bcp.BcpError) as e:
                es.plan_rounds(3, [1, 2, 3], (), round_st=bad)
            assert e.value.rc == -22
    finally:
        es.close()
    del ctypes


@pytest.mark.skipif(not os.path.exists(MAP_BIN), reason="oracle/_ref not built here (needs /root/reference)")
@pytest.mark.parametrize("seed", range(4))
def test_random_target_lists_against_the_reference_program(bcp, seed):
    rng = np.random.default_rng(500 + seed)
    for _ in range(60):
        nt = int(rng.integers(1, 57))
        ids = [int(x) for x in rng.choice(np.arange(1, 300), size=nt + 6, replace=False)]
        nprev = int(rng.integers(0, nt + 2))
        prev = ids[:nprev] if nprev <= nt + 6 else ids
        rank = [prev[int(i)] for i in rng.permutation(min(nprev, nt))] + ids[nprev:nprev + max(0, nt - nprev)]
        rank = [rank[int(i)] for i in rng.permutation(len(rank))][:nt]
        if rng.random() < 0.15 and nt > 1:  # a repeated id
            rank[int(rng.integers(0, nt))] = rank[int(rng.integers(0, nt))]
        if rng.random() < 0.1 and nt > 1:  # an unknown id instead of a known one
            rank[int(rng.integers(0, nt))] = 999
        r = subprocess.run([MAP_BIN, str(len(prev)), *map(str, prev), str(len(rank)), *map(str, rank)],
                           capture_output=True, text=True)
        got = _map(bcp, prev, rank)
        if r.returncode:
            msg = r.stderr.strip().split(": ", 1)[-1]
            assert got == next(rc for m, rc in ERR.items() if msg.startswith(m)), (prev, rank, msg)
        else:
            out = {ln.split()[0]: [int(x) for x in ln.split()[1:]] for ln in r.stdout.splitlines()}
            assert got == (out["st_ids"], out["round_st"]), (prev, rank)


def _store(tmp_path, ids):
    root = str(tmp_path)
    S.make_store(root, len(ids))
    for k, tid in enumerate(ids):
        (tmp_path / f"st{k}" / "targetNumID").write_text(f"{tid}\n")
    return root


def test_store_round_order_from_rank_order_file(bcp, tmp_path):
    root = _store(tmp_path, [101, 102, 103, 104])
    assert bcp.store_round_order(root, 4) == [0, 1, 2, 3]            # no file: target order
    (tmp_path / "rank_order").write_text("103 101\n104 102\n")      # hosts listed in another order
    assert bcp.store_round_order(root, 4) == [2, 0, 3, 1]
    for bad, rc in (("103 101 104", -71), ("103 101 104 102 105", -71), ("103 x 104 102", -71),
                    ("103 103 104 102", -17), ("103 101 104 999", -19)):
        (tmp_path / "rank_order").write_text(bad)
        with pytest.raises(bcp.BcpError) as e:
            bcp.store_round_order(root, 4)
        assert e.value.rc == rc, bad


def test_check_targets_with_a_grown_and_permuted_rank_order(bcp, tmp_path):
    """A first run indexes the directories in their own order; a later run
    keeps every known target's index (bcp_map_targets over the run_data), and
    targets added since must be numbered in the order the reference appends
    them -- rank order -- or the check refuses (-EPROTO)."""
    root = _store(tmp_path, [11, 12, 13])
    rd = str(tmp_path / "run_data")
    (tmp_path / "rank_order").write_text("13 11 12")
    bcp.check_targets(root, 3, rd)                                   # first run: any permutation
    assert bcp.store_round_order(root, 3) == [2, 0, 1]
    S.make_store(root, 5)                                            # two targets added
    (tmp_path / "st3" / "targetNumID").write_text("21")
    (tmp_path / "st4" / "targetNumID").write_text("22")
    (tmp_path / "rank_order").write_text("21 13 11 22 12")           # new ones appended in rank order: 21, 22
    bcp.check_targets(root, 5, rd)
    assert bcp.store_round_order(root, 5) == [3, 2, 0, 4, 1]
    assert bcp.map_targets([11, 12, 13], [21, 13, 11, 22, 12]) == ([11, 12, 13, 21, 22], [3, 2, 0, 4, 1])
    rd2 = str(tmp_path / "run_data2")
    (tmp_path / "rank_order").write_text("11 12 13")
    S.make_store(root, 3)
    bcp.check_targets(root, 3, rd2)
    (tmp_path / "rank_order").write_text("22 13 11 21 12")           # 22 before 21: the reference puts 22 at st3
    with pytest.raises(bcp.BcpError) as e:
        bcp.check_targets(root, 5, rd2)
    assert e.value.rc == -71
