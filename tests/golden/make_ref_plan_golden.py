"""Regenerates tests/golden/ref_plan.json from the REFERENCE'S OWN planner
functions (P placement, worklist order, lanes).

Container only: needs oracle/_ref/libref_plan.so, which `make -C oracle ref`
compiles from the reference's text streamed unchanged (SHA-checked) out of
/root/reference/src/beegfs-raid5: gen/main.c simple_hash :67-74, PCG32
:338-371, shuffle :373-386, select_P :388-401, SizeIndex/cmp_entries
:174-189, fill_in_missing_fields :92-100; gen/file_info_hash.c fih_add_info
:24-31; gen/assign_lanes.c :7-46 (see oracle/ref_plan_glue.c).  The fixtures
are data: inputs and the reference's outputs -- no reference text.

  "hash"        path bytes -> simple_hash
  "pcg32"       (initstate, initseq, bound) -> first outputs
  "select_P"    (path, locations, ntargets, weight vector) -> locations with P
  "fill"        (dst, src) -> fill_in_missing_fields
  "order"       total sizes (many ties) -> worklist order (shuffle + qsort)
  "lanes"       (nlanes, locations incl. P and NO_P) -> assign_lanes
  "plan"        record streams per target (records name paths by index into
                "paths") + previous DB state + weights ->
                the whole worklist: order, timestamps, locations with P / NO_P
                (gen/main.c:688 aggregation, :310 eater = simple_hash %
                ntargets, :710-711 order per eater, :758-797 the eaters'
                rounds in target order, :772-788 items), the rounds' bounds
                and the 12 lanes of every round (:823)

    make -C oracle ref && python tests/golden/make_ref_plan_golden.py
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

NO_P = 0xFF
L_MASK = (1 << 56) - 1


def with_p(loc, p):
    return (loc & L_MASK) | ((p & 0xFF) << 56)


# ---- the reference's functions, through oracle/_ref --------------------------
def r_hash(L, b: bytes) -> int:
    return L.ref_simple_hash(b, len(b))


def r_pcg32(L, state, seq, bound, n):
    out = (ctypes.c_uint32 * n)()
    L.ref_pcg32(state, seq, bound, out, n)
    return list(out)


def r_set_weights(L, cum):
    L.ref_set_st_weight((ctypes.c_int * len(cum))(*cum), len(cum))


def r_select_p(L, path: bytes, loc, ntargets, cum):
    r_set_weights(L, cum)
    return L.ref_select_P(path, loc, ntargets)


def r_order(L, sizes):
    n = len(sizes)
    idx = (ctypes.c_uint64 * max(n, 1))()
    L.ref_sort_order((ctypes.c_uint64 * max(n, 1))(*sizes), n, idx)
    return list(idx)[:n]


def r_lanes(L, nlanes, locs):
    n = len(locs)
    fis = (ctypes.c_uint64 * (2 * max(n, 1)))()
    for i, loc in enumerate(locs):
        fis[2 * i + 1] = loc  # FileInfo {i64 timestamp; u64 locations}
    out = (ctypes.c_int * max(n, 1))()
    L.assign_lanes(nlanes, n, fis, out)
    return list(out)[:n]


def r_aggregate(L, streams):
    """gen/main.c:650-688 per record, in feed order: a new path gets a zeroed
    FatFileInfo (:674) and its index in first-seen order (fih_get_or_create),
    size += chunk_size (:683), fih_add_info (:684-688)."""
    agg = {}
    for st, recs in streams:
        for ts, size, ev, path in recs:
            e = agg.setdefault(path, [0, 0, 0, 0])
            t, m, d = ctypes.c_int64(e[0]), ctypes.c_uint64(e[1]), ctypes.c_uint64(e[2])
            L.ref_fih_add_info(ctypes.byref(t), ctypes.byref(m), ctypes.byref(d), st, ts, 1 if ev == "d" else 0)
            e[0], e[1], e[2] = t.value, m.value, d.value
            e[3] = (e[3] + size) & ((1 << 64) - 1)
    return agg


def r_rounds(L, paths, sizes, ntargets):
    """ref_round_order: (indices in worklist order, round_start)."""
    n = len(paths)
    enc = [p.encode() for p in paths]
    arr = (ctypes.c_char_p * max(n, 1))(*enc)
    idx = (ctypes.c_uint64 * max(n, 1))()
    rs = (ctypes.c_size_t * (ntargets + 1))()
    L.ref_round_order(arr, (ctypes.c_uint64 * max(n, 1))(*sizes), n, ntargets, idx, rs)
    return list(idx)[:n], list(rs)


def r_plan(L, streams, ntargets, cum, prev, rounds=False):
    """The worklist of one gen run: list of (path, timestamp, locations), the
    coordinators' rounds back to back (rounds=True: and the round starts)."""
    agg = r_aggregate(L, streams)
    paths = list(agg)
    order, starts = r_rounds(L, paths, [agg[p][3] for p in paths], ntargets)
    r_set_weights(L, cum)
    out = []
    for i in order:
        p = paths[i]
        ts, mod, dele, _ = agg[p]
        old = prev.get(p)
        loc = L.ref_plan_item(p.encode(), ts, mod, dele, 1 if old else 0,
                              old[0] if old else 0, old[1] if old else 0, ntargets)
        out.append((p, ts, loc))
    return (out, starts) if rounds else out


# ---- inputs --------------------------------------------------------------------
def rand_path(rng, i):
    """chunk-path-like names; some with UTF-8 bytes >= 0x80 (simple_hash adds
    signed chars).  Paths are UTF-8 everywhere (fixtures, libbcp calls)."""
    base = f"u{int(rng.integers(0, 6))}/{int(rng.integers(0, 1 << 24)):06X}/{int(rng.integers(0, 1 << 30)):08X}-{i}"
    if rng.random() < 0.1:
        base += "éÿ"
    return base


def weight_vector(rng, ntargets):
    w = [int(x) for x in rng.integers(0, 7000, size=ntargets)]
    if rng.random() < 0.3:  # some empty stores
        for t in rng.integers(0, ntargets, size=max(1, ntargets // 4)):
            w[int(t)] = 0
    if rng.random() < 0.2:  # equal weights
        w = [6000] * ntargets
    if sum(w) == 0:
        w[int(rng.integers(0, ntargets))] = 1
    return [int(x) for x in np.cumsum(w)]


def main():
    L = O.ref_plan_lib()
    if L is None:
        sys.exit("oracle/_ref/libref_plan.so not built (make -C oracle ref)")
    rng = np.random.default_rng(20260316)
    doc = {"source": "reference functions compiled unchanged (oracle/_ref/libref_plan.so); see docstring",
           "generator": "tests/golden/make_ref_plan_golden.py"}

    hp = ["", "a", "u0/5F/12-5F8A2B3C-1/1A-5F8A2B3C-1", "x" * 300] + [rand_path(rng, i) for i in range(200)]
    hp.append("éÿ\u0080/bytes")
    doc["hash"] = [[p, r_hash(L, p.encode())] for p in hp]

    doc["pcg32"] = []
    for state, seq, bound in [(42, 54, 0), (0, 0, 0), (0x853C49E6748FEA9B, 0xDA3E39CB94B95BDB, 0),
                              (5381, 0, 7000), (123456789, 0, 3), (2 ** 64 - 1, 2 ** 63, 1 << 31),
                              (77, 0, 56 * 6643)]:
        doc["pcg32"].append([state, seq, bound, r_pcg32(L, state, seq, bound, 16)])

    # select_P: weight vectors shared by index; locations with no P (NO_P) or a holder's P
    wvs = []
    for _ in range(80):
        nt = int(rng.choice([1, 2, 3, 4, 5, 8, 9, 12, 16, 31, 32, 33, 40, 55, 56]))
        wvs.append(weight_vector(rng, nt))
    doc["weights"] = wvs
    sel = []
    while len(sel) < 3000:
        wi = int(rng.integers(0, len(wvs)))
        cum = wvs[wi]
        nt = len(cum)
        holders = int(rng.integers(0, 1 << nt)) if nt < 63 else 0
        if rng.random() < 0.1:
            holders = (1 << nt) - 1  # every target holds a chunk: no P
        loc = with_p(holders, NO_P)
        path = rand_path(rng, len(sel)).encode()
        out = r_select_p(L, path, loc, nt, cum)
        if out == (1 << 64) - 1:  # the reference would retry forever
            continue
        sel.append([path.decode(), loc, wi, out])
    doc["select_P"] = sel

    fill = []
    for _ in range(500):
        nt = int(rng.integers(1, 57))
        dst = with_p(int(rng.integers(0, 1 << min(nt, 62))), NO_P)
        src = with_p(int(rng.integers(0, 1 << min(nt, 62))), int(rng.choice([NO_P, int(rng.integers(0, nt))])))
        fill.append([dst, src, L.ref_fill_in_missing_fields(dst, src)])
    doc["fill"] = fill

    orders = []
    for n in (0, 1, 2, 3, 5, 17, 100, 1000, 3000):
        for kinds in (2, 5, 1000000):
            sizes = [int(x) for x in rng.integers(0, kinds, size=n)]
            sizes = [s * 4096 for s in sizes]
            orders.append([sizes, r_order(L, sizes)])
    doc["order"] = orders

    lanes = []
    for nlanes in (1, 2, 5, 12, 16):
        for njobs in (0, 1, 40, 700):
            nt = int(rng.integers(3, 57))
            locs = []
            for _ in range(njobs):
                h = int(rng.integers(0, 1 << min(nt, 62))) & ~(1 << int(rng.integers(0, nt)))
                p = int(rng.integers(0, nt))
                if h & (1 << p):
                    h &= ~(1 << p)
                locs.append(with_p(h, NO_P if rng.random() < 0.15 else p))
            lanes.append([nlanes, locs, r_lanes(L, nlanes, locs)])
    doc["lanes"] = lanes

    plans = []
    for case in range(24):
        nt = int(rng.integers(2, 20)) if case else 4
        npaths = int(rng.integers(1, 400))
        paths = [rand_path(rng, i) for i in range(npaths)]
        streams = []
        for st in range(nt):
            recs = []
            for _ in range(int(rng.integers(0, npaths // 2 + 2))):
                ts = int(rng.integers(-5, 1 << 40)) if rng.random() < 0.05 else int(rng.integers(1, 1 << 40))
                size = int(rng.choice([0, 4096, 65536, 524288, int(rng.integers(0, 1 << 23))]))
                recs.append([ts, size, "d" if rng.random() < 0.15 else "m", int(rng.integers(0, npaths))])
            streams.append([st, recs])
        expand = [(st, [(ts, size, ev, paths[pi]) for ts, size, ev, pi in recs]) for st, recs in streams]
        cum = weight_vector(rng, nt)
        agg = r_aggregate(L, expand)
        prev = {}
        for p, (ts, m, d, sz) in list(agg.items())[::2]:
            p_old = int(rng.integers(0, nt))
            held = int(rng.integers(0, 1 << nt)) & ~(1 << p_old)
            if rng.random() < 0.4:  # previous state equal to this round's -> NO_P
                held = m & ~d
                free = [t for t in range(nt) if not held >> t & 1]
                p_old = free[int(rng.integers(0, len(free)))] if free else None
            prev[p] = [ts if rng.random() < 0.6 else ts - 1, with_p(held, NO_P if p_old is None else p_old)]
        plan, starts = r_plan(L, expand, nt, cum, prev, rounds=True)
        if any(loc == (1 << 64) - 1 for _, _, loc in plan):
            continue
        lanes12 = []
        for k in range(nt):
            lanes12 += r_lanes(L, 12, [loc for _, _, loc in plan[starts[k]:starts[k + 1]]])
        pidx = {p: i for i, p in enumerate(paths)}
        plans.append({"ntargets": nt, "cum_weight": cum, "paths": paths, "streams": streams,
                      "prev": [[pidx[p], ts, loc] for p, (ts, loc) in sorted(prev.items())],
                      "worklist": [[pidx[p], ts, loc] for p, ts, loc in plan],
                      "round_start": starts, "lanes12": lanes12})
    doc["plan"] = plans

    out = os.path.join(HERE, "ref_plan.json")
    with open(out, "w") as f:
        json.dump(doc, f, separators=(",", ":"))

    # ref_round.json: the layout of tests/test_gpu_protocol.py's DB round test
    # (9 targets, 3-7 holders per file) and the reference's P for every file.
    nt, cw = 9, [1000 * (k + 1) for k in range(9)]
    files = []
    for i in range(24):
        holders = sorted(int(x) for x in rng.choice(nt, size=int(rng.integers(3, 8)), replace=False))
        mask = sum(1 << h for h in holders)
        path = f"d{i % 4}/c{i}"
        loc = r_select_p(L, path.encode(), with_p(mask, NO_P), nt, cw)
        files.append([path, holders, loc])
    with open(os.path.join(HERE, "ref_round.json"), "w") as f:
        json.dump({"source": doc["source"], "ntargets": nt, "cum_weight": cw, "files": files}, f, indent=0)
    print(out, os.path.getsize(out), "bytes;", len(sel), "select_P,", len(orders), "orders,", len(lanes),
          "lane sets,", len(plans), "plans")


if __name__ == "__main__":
    main()
