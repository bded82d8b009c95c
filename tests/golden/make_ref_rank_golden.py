"""Regenerates tests/golden/ref_rank.json: the reference's storage-target
mapping and the eaters' round order in MPI rank order.

Container only: needs oracle/_ref/ref_map_targets and libref_plan.so, which
`make -C oracle ref` compiles from the reference's text streamed unchanged
(SHA-checked) out of /root/reference/src/beegfs-raid5:

  ref_map_targets   gen/main.c:498-499, 506-541 (the coordinator after the
                    Gathers: the previous run's list kept, new targets appended
                    in rank order, st2rank / rank2st; "Fewer targets",
                    "Duplicate targetNumID", "Storage target missing!" with the
                    C library's errx) -- oracle/ref_map_head.c, ref_map_tail.c
  libref_plan.so    simple_hash, PCG32 shuffle, cmp_entries, select_P,
                    fill_in_missing_fields, fih_add_info, assign_lanes; glue
                    ref_round_order_ranked (round r = the eater of target
                    rank2st[2r+1], gen/main.c:758) -- oracle/ref_plan_glue.c

The fixtures are data: inputs and the reference's outputs.

  "map"    (prev ids in index order, ids in rank order) -> st_ids, st2rank,
           round_st, or the reference's error message
  "plan"   whole worklists whose rounds follow a target list the hosts
           permuted or grew: the mapping above, then record streams ->
           aggregation -> eaters -> order per eater -> rounds in rank order ->
           items planned against a previous DB state, with the round bounds
           and the 12 lanes of every round

    make -C oracle ref && python tests/golden/make_ref_rank_golden.py
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402
from make_ref_plan_golden import r_aggregate, r_lanes, r_set_weights, rand_path, weight_vector, with_p  # noqa: E402

MAP_BIN = os.path.join(HERE, "..", "..", "oracle", "_ref", "ref_map_targets")
NO_P = 0xFF


def r_map(prev, rank_ids):
    """The reference's mapping: dict of st_ids / st2rank / round_st, or error."""
    r = subprocess.run([MAP_BIN, str(len(prev)), *map(str, prev), str(len(rank_ids)), *map(str, rank_ids)],
                       capture_output=True, text=True)
    if r.returncode:
        return {"error": r.stderr.strip().split(": ", 1)[-1], "rc": r.returncode}
    out = {}
    for line in r.stdout.splitlines():
        k, *v = line.split()
        out[k] = [int(x) for x in v]
    return out


def r_rounds_ranked(L, paths, sizes, ntargets, round_st):
    n = len(paths)
    arr = (ctypes.c_char_p * max(n, 1))(*[p.encode() for p in paths])
    idx = (ctypes.c_uint64 * max(n, 1))()
    rs = (ctypes.c_size_t * (ntargets + 1))()
    L.ref_round_order_ranked(arr, (ctypes.c_uint64 * max(n, 1))(*sizes), n, ntargets,
                             (ctypes.c_int * ntargets)(*round_st), idx, rs)
    return list(idx)[:n], list(rs)


def r_plan_ranked(L, streams, ntargets, cum, prev, round_st):
    agg = r_aggregate(L, streams)
    paths = list(agg)
    order, starts = r_rounds_ranked(L, paths, [agg[p][3] for p in paths], ntargets, round_st)
    r_set_weights(L, cum)
    out = []
    for i in order:
        p = paths[i]
        ts, mod, dele, _ = agg[p]
        old = prev.get(p)
        loc = L.ref_plan_item(p.encode(), ts, mod, dele, 1 if old else 0,
                              old[0] if old else 0, old[1] if old else 0, ntargets)
        out.append((p, ts, loc))
    return out, starts


def target_lists(rng, nt):
    """(prev ids in index order, ids in rank order): a permuted host list, a
    grown one (new targets at random rank positions), or both."""
    ids = [int(x) for x in rng.choice(np.arange(1, 500), size=nt + 8, replace=False)]
    kind = int(rng.integers(0, 3))
    if kind == 0:  # the same targets, hosts listed in another order
        prev = ids[:nt]
        rank = [prev[int(i)] for i in rng.permutation(nt)]
    else:  # targets added since the last run (1-3), the old ones maybe permuted
        add = min(int(rng.integers(1, 4)), nt - 1)
        prev = ids[:nt - add]
        old = prev if kind == 1 else [prev[int(i)] for i in rng.permutation(len(prev))]
        rank = list(old)
        for t in ids[nt:nt + add]:
            rank.insert(int(rng.integers(0, len(rank) + 1)), t)
    return prev, rank, kind


def main():
    L = O.ref_plan_lib()
    if L is None or not os.path.exists(MAP_BIN):
        sys.exit("oracle/_ref not built (make -C oracle ref)")
    L.ref_round_order_ranked.restype = None
    rng = np.random.default_rng(20261018)
    doc = {"source": "reference code compiled unchanged (oracle/_ref/ref_map_targets, libref_plan.so); see docstring",
           "generator": "tests/golden/make_ref_rank_golden.py"}

    maps = []
    for _ in range(150):
        nt = int(rng.choice([1, 2, 3, 4, 5, 8, 9, 13, 28, 56]))
        prev, rank, _ = target_lists(rng, nt) if nt > 1 else ([7], [7], 0)
        maps.append({"prev": prev, "rank": rank, **r_map(prev, rank)})
    # the reference's fatal checks
    bad = [([11, 12, 13], [11, 12]),                # fewer targets than last run
           ([11, 12], [11, 11]),                    # a rank repeats a placed id
           ([11, 12, 13], [11, 14, 13]),            # 12 gone, 14 new: missing
           ([11, 12], [12, 11, 12]),                # duplicate after a permutation
           ([], [5, 5]),                            # two new ranks with one id: the reference accepts it
           ([11], [11, 20, 20])]                    # the same, after a known target
    for prev, rank in bad:
        maps.append({"prev": prev, "rank": rank, **r_map(prev, rank)})
    doc["map"] = maps

    plans = []
    case = 0
    while len(plans) < 24:
        case += 1
        nt = int(rng.integers(2, 20))
        prev_ids, rank_ids, kind = target_lists(rng, nt)
        m = r_map(prev_ids, rank_ids)
        if "error" in m or m["round_st"] == list(range(nt)):  # only orders the identity would get wrong
            continue
        npaths = int(rng.integers(1, 400))
        paths = [rand_path(rng, i) for i in range(npaths)]
        streams = []
        for st in range(nt):
            recs = []
            for _ in range(int(rng.integers(0, npaths // 2 + 2))):
                ts = int(rng.integers(1, 1 << 40))
                size = int(rng.choice([0, 4096, 65536, 524288, int(rng.integers(0, 1 << 23))]))
                recs.append([ts, size, "d" if rng.random() < 0.15 else "m", int(rng.integers(0, npaths))])
            streams.append([st, recs])
        expand = [(st, [(ts, size, ev, paths[pi]) for ts, size, ev, pi in recs]) for st, recs in streams]
        cum = weight_vector(rng, nt)
        agg = r_aggregate(L, expand)
        prev = {}
        for p, (ts, mm, d, sz) in list(agg.items())[::2]:
            p_old = int(rng.integers(0, nt))
            held = int(rng.integers(0, 1 << nt)) & ~(1 << p_old)
            prev[p] = [ts if rng.random() < 0.6 else ts - 1, with_p(held, p_old)]
        plan, starts = r_plan_ranked(L, expand, nt, cum, prev, m["round_st"])
        if any(loc == (1 << 64) - 1 for _, _, loc in plan):
            continue
        lanes12 = []
        for r in range(nt):
            lanes12 += r_lanes(L, 12, [loc for _, _, loc in plan[starts[r]:starts[r + 1]]])
        pidx = {p: i for i, p in enumerate(paths)}
        plans.append({"ntargets": nt, "kind": ["permuted", "grown", "grown+permuted"][kind],
                      "prev_ids": prev_ids, "rank_ids": rank_ids, "st_ids": m["st_ids"], "round_st": m["round_st"],
                      "cum_weight": cum, "paths": paths, "streams": streams,
                      "prev": [[pidx[p], ts, loc] for p, (ts, loc) in sorted(prev.items())],
                      "worklist": [[pidx[p], ts, loc] for p, ts, loc in plan],
                      "round_start": starts, "lanes12": lanes12})
    doc["plan"] = plans
    out = os.path.join(HERE, "ref_rank.json")
    with open(out, "w") as f:
        json.dump(doc, f, separators=(",", ":"))
    print(out, os.path.getsize(out), "bytes;", len(maps), "mappings,", len(plans), "plans")


if __name__ == "__main__":
    main()
