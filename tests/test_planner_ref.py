"""Worklist planner pinned to the REFERENCE'S OWN functions (SURVEY.md §8(f)
row 2: the same P target, the same order, the same lanes as the reference).

tests/golden/ref_plan.json holds outputs of gen/main.c simple_hash, PCG32,
shuffle + qsort(cmp_entries), select_P, fill_in_missing_fields,
gen/file_info_hash.c fih_add_info and gen/assign_lanes.c, compiled unchanged
from /root/reference into oracle/_ref/libref_plan.so
(tests/golden/make_ref_plan_golden.py).  libbcp's bcp_plan_worklist,
bcp_assign_lanes and bcp_path_hash must reproduce every case, and so must the
Python restatement oracle/planner.py.  Where oracle/_ref is built (this
container) the product is also compared with the reference functions directly
on fresh random inputs and on a real store's free-space weight."""
import json
import os

import numpy as np
import pytest

import planner as PL

HERE = os.path.dirname(os.path.abspath(__file__))
U64 = (1 << 64) - 1


class _Doc:
    """tests/golden/ref_plan.json, read on first use (CPU tests only: the
    file stays off the GPU box, so collection must not need it)."""
    _d = None

    def __getitem__(self, k):
        if _Doc._d is None:
            _Doc._d = json.load(open(os.path.join(HERE, "golden", "ref_plan.json")))
        return _Doc._d[k]


DOC = _Doc()


def _plan_product(bcp, case):
    paths = case["paths"]
    es = bcp.EventSet()
    try:
        for st, recs in case["streams"]:
            if recs:
                es.feed(st, bcp.pack_records([(ts, size, ev, paths[pi]) for ts, size, ev, pi in recs]))
        prev = [(paths[pi], ts, loc) for pi, ts, loc in case["prev"]]
        return es.plan_rounds(case["ntargets"], case["cum_weight"], prev)
    finally:
        es.close()


def test_simple_hash_fixtures(bcp):
    for path, h in DOC["hash"]:
        b = path.encode()
        assert bcp.lib().bcp_path_hash(b, len(b)) == h, path
        assert PL.simple_hash(b) == h, path


def test_pcg32_fixtures():
    for state, seq, bound, outs in DOC["pcg32"]:
        r = PL.PCG32.seeded(state, seq)
        assert [r.bounded(bound) if bound else r.next() for _ in outs] == outs


def test_select_P_fixtures(bcp):
    """P placement: one event set per weight vector, one path per case whose
    holders are its 'm' records (a 'd' record where it has none); no previous
    state, so bcp_plan_worklist calls select_P on every path."""
    by_w = {}
    for path, loc, wi, out in DOC["select_P"]:
        by_w.setdefault(wi, []).append((path, loc, out))
    n = 0
    for wi, cases in by_w.items():
        cum = DOC["weights"][wi]
        es = bcp.EventSet()
        try:
            recs = {}
            for path, loc, _ in cases:
                holders = [t for t in range(len(cum)) if loc >> t & 1]
                for t in holders or [0]:
                    recs.setdefault(t, []).append((1, 4096, "m" if holders else "d", path))
            for t, r in sorted(recs.items()):
                es.feed(t, bcp.pack_records(r))
            got = {p: l for p, _, l in es.plan(len(cum), cum)}
        finally:
            es.close()
        for path, loc, out in cases:
            assert got[path] == out, (path, hex(loc), hex(got[path]), hex(out))
            assert PL.select_p(path.encode(), loc, len(cum), cum) == out
            n += 1
    assert n == len(DOC["select_P"]) >= 3000


def test_fill_in_missing_fixtures():
    for dst, src, out in DOC["fill"]:
        assert PL.fill_in_missing(dst, src) == out


def test_worklist_order_fixtures(bcp):
    """shuffle (fixed seed) then qsort by total size, many equal sizes: the
    order of ties is exactly the reference's (one target: one eater, one
    round holding every path)."""
    for sizes, order in DOC["order"]:
        es = bcp.EventSet()
        try:
            recs = [(1, s, "m", f"p{i}") for i, s in enumerate(sizes)]
            if recs:
                es.feed(0, bcp.pack_records(recs))
            got = [int(p[1:]) for p, _, _ in es.plan(1, [1])]
        finally:
            es.close()
        assert got == order, len(sizes)
        agg = {f"p{i}".encode(): [1, 1, 0, s] for i, s in enumerate(sizes)}
        assert [int(p[1:]) for p, _, _ in PL.plan(agg, 1, [1], {})] == order


def test_assign_lanes_fixtures(bcp):
    for nlanes, locs, lanes in DOC["lanes"]:
        assert bcp.assign_lanes(nlanes, locs) == lanes, (nlanes, len(locs))


def test_whole_worklist_fixtures(bcp):
    """Record streams -> aggregation -> eaters (simple_hash % ntargets) ->
    order per eater -> the coordinators' rounds -> merge with the previous DB
    state -> P or NO_P: the whole phase-2 worklist item for item, the rounds'
    bounds and the 12 lanes of every round."""
    nitems = nnop = nrounds = 0
    for case in DOC["plan"]:
        paths = case["paths"]
        want = [(paths[pi], ts, loc) for pi, ts, loc in case["worklist"]]
        got, starts = _plan_product(bcp, case)
        assert got == want and starts == case["round_start"]
        assert bcp.assign_lanes_rounds(12, starts, [loc for _, _, loc in got]) == case["lanes12"]
        nrounds += sum(1 for a, b in zip(starts, starts[1:]) if b > a)
        packed = [(st, bcp.pack_records([(ts, size, ev, paths[pi]) for ts, size, ev, pi in recs]))
                  for st, recs in case["streams"]]
        agg = PL.aggregate(packed)
        prev = {paths[pi].encode(): (ts, loc) for pi, ts, loc in case["prev"]}
        assert PL.plan(agg, case["ntargets"], case["cum_weight"], prev, rounds=True) == \
            ([(p.encode(), ts, loc) for p, ts, loc in want], case["round_start"])
        nitems += len(want)
        nnop += sum(1 for _, _, loc in want if loc >> 56 == 0xFF)
    assert nitems > 3000 and nnop > 300  # unchanged items (NO_P) are covered
    assert nrounds > 150  # non-empty rounds, 2..19 targets


# ---- against the reference functions directly (container: oracle/_ref) ------------
def _ref():
    import oracle as O
    L = O.ref_plan_lib()
    if L is None:
        pytest.skip("oracle/_ref/libref_plan.so not built here (needs /root/reference)")
    return L


@pytest.mark.parametrize("seed", range(4))
def test_random_worklists_against_reference_functions(bcp, seed):
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_ref_plan_golden as G
    L = _ref()
    rng = np.random.default_rng(1000 + seed)
    nt = int(rng.integers(2, 57))
    paths = [G.rand_path(rng, i) for i in range(300)]
    streams = []
    for st in range(nt):
        recs = [(int(rng.integers(0, 1 << 40)), int(rng.choice([0, 4096, 524288])),
                 "d" if rng.random() < 0.1 else "m", paths[int(rng.integers(0, len(paths)))])
                for _ in range(int(rng.integers(0, 40)))]
        streams.append((st, recs))
    cum = G.weight_vector(rng, nt)
    agg = G.r_aggregate(L, streams)
    prev = {p: [ts - int(rng.integers(0, 2)), G.with_p(m & ~d, G.NO_P if rng.random() < 0.3 else
                                                    next((t for t in range(nt) if not (m & ~d) >> t & 1), G.NO_P))]
            for p, (ts, m, d, _) in list(agg.items())[::3]}
    want, starts = G.r_plan(L, streams, nt, cum, prev, rounds=True)
    if any(loc == U64 for _, _, loc in want):
        pytest.skip("select_P would not terminate for this draw")
    es = bcp.EventSet()
    try:
        for st, recs in streams:
            if recs:
                es.feed(st, bcp.pack_records(recs))
        got, got_starts = es.plan_rounds(nt, cum, [(p, ts, loc) for p, (ts, loc) in prev.items()])
    finally:
        es.close()
    assert got == want and got_starts == starts
    locs = [loc for _, _, loc in want]
    for nlanes in (1, 3, 12):
        assert bcp.assign_lanes(nlanes, locs) == G.r_lanes(L, nlanes, locs)
        per_round = []
        for k in range(nt):
            per_round += G.r_lanes(L, nlanes, locs[starts[k]:starts[k + 1]])
        assert bcp.assign_lanes_rounds(nlanes, starts, locs) == per_round


def test_store_weight_against_reference_function(bcp, tmp_path):
    L = _ref()
    fd = os.open(str(tmp_path), os.O_DIRECTORY | os.O_RDONLY)
    try:
        assert bcp.lib().bcp_store_weight(fd) == L.ref_store_weight(fd)
        st = os.statvfs(str(tmp_path))
        for avail in (0, 1, st.f_bsize * 3, st.f_blocks * st.f_bsize // 3, st.f_blocks * st.f_bsize):
            (tmp_path / "free_space.override").write_text(str(avail))
            assert bcp.lib().bcp_store_weight(fd) == L.ref_store_weight(fd), avail
    finally:
        os.close(fd)
