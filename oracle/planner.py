"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of the worklist side
of parity generation, the checker for libbcp's
bcp_eventset_* / bcp_plan_worklist.

  record stream     bp-find-all-chunks/main.c:25-33, gen/main.c:286-336
  aggregation       gen/file_info_hash.c:24-31 (fih_add_info), gen/main.c:688
  simple_hash       gen/main.c:67-74
  PCG32             gen/main.c:338-372 (pcg-random.org minimal C)
  shuffle + sort    gen/main.c:373-386, 703-715, per eater
  rounds            gen/main.c:310 (eater = simple_hash % ntargets), 758-797
  worklist item     gen/main.c:768-791 (fill_in_missing_fields :92-100,
                    select_P :388-401)

Pinning: every function above against tests/golden/ref_plan.json -- outputs
of the reference's OWN simple_hash, PCG32, shuffle + qsort, select_P,
fill_in_missing_fields, fih_add_info and assign_lanes, compiled unchanged from
/root/reference into oracle/_ref/libref_plan.so (oracle/Makefile `ref`,
tests/golden/make_ref_plan_golden.py; checked by tests/test_planner_ref.py);
PCG32 also against the pcg32 demo's published first outputs (seed 42, seq 54).
The sort is Python's stable sort: equal to glibc <= 2.36's qsort (a merge
sort), which this image's reference build links.  The one deviation: where no
non-holder target carries weight select_P returns the locations unchanged
(the reference retries forever; fixtures never contain that case).
"""
from __future__ import annotations

import struct

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
L_MASK = (1 << 56) - 1
NO_P = 0xFF


def simple_hash(path: bytes) -> int:
    h = 5381
    for c in path:
        sc = c - 256 if c >= 128 else c          # char is signed on x86
        h = (h + (h << 5) + sc) & M32
    return h


class PCG32:
    def __init__(self, state: int = 0, inc: int = 1):
        self.state, self.inc = state, inc

    @classmethod
    def seeded(cls, initstate: int, initseq: int) -> "PCG32":
        r = cls(0, ((initseq << 1) | 1) & M64)
        r.next()
        r.state = (r.state + initstate) & M64
        r.next()
        return r

    def next(self) -> int:
        old = self.state
        self.state = (old * 6364136223846793005 + (self.inc | 1)) & M64
        xs = (((old >> 18) ^ old) >> 27) & M32
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & M32

    def bounded(self, bound: int) -> int:
        threshold = ((-bound) & M32) % bound
        while True:
            r = self.next()
            if r >= threshold:
                return r % bound


def with_p(loc: int, p: int) -> int:
    return (loc & L_MASK) | ((p & 0xFF) << 56)


def get_p(loc: int) -> int:
    return loc >> 56


def test_bit(x: int, i: int) -> bool:
    return bool(x & (1 << (i & 63)))        # x86 masks the shift count


def p_is_invalid(loc: int) -> bool:
    return get_p(loc) == NO_P or test_bit(loc, get_p(loc))


def parse_records(data: bytes):
    """-> list of (timestamp, size, event, path bytes); trailing partial dropped."""
    out, off = [], 0
    while len(data) - off >= 32:
        ts, size, ev, n = struct.unpack_from("<qQQQ", data, off)
        if len(data) - off - 32 < n:
            break
        out.append((ts, size, ev, data[off + 32: off + 32 + n]))
        off += 32 + n
    return out


def aggregate(streams):
    """streams: list of (storage_target, bytes) in feed order ->
    ordered dict path -> [timestamp, modified, deleted, size]."""
    agg = {}
    for st, data in streams:
        for ts, size, ev, path in parse_records(data):
            e = agg.setdefault(path, [0, 0, 0, 0])
            e[0] = max(e[0], ts)
            if ev == ord("d"):
                e[2] |= 1 << st
            else:
                e[1] |= 1 << st
            e[3] += size
    return agg


def select_p(path: bytes, loc: int, ntargets: int, cum_weight) -> int:
    if bin(loc & L_MASK).count("1") == ntargets:
        return loc
    if not any(not test_bit(loc, t) and cum_weight[t] - (cum_weight[t - 1] if t else 0) > 0 for t in range(ntargets)):
        return loc
    rng = PCG32.seeded(simple_hash(path), 0)
    while True:
        r = rng.bounded(cum_weight[ntargets - 1])
        p = 0
        while r >= cum_weight[p]:
            p += 1
        if not test_bit(loc, p):
            return with_p(loc, p)


def fill_in_missing(dst: int, src: int) -> int:
    old_p = get_p(src)
    loc = (dst | src) & L_MASK
    return with_p(loc, old_p) if not test_bit(loc, old_p) else with_p(loc, NO_P)


def round_order(entries, ntargets: int):
    """-> (entry indices in worklist order, round_start): eater k gets the
    paths with simple_hash % ntargets == k in arrival order (gen/main.c:310),
    shuffles them with a fresh fixed-seed PCG32 and sorts them by total size
    (:710-711); the eaters' lists follow each other in target order (:758)."""
    order, starts = [], []
    for k in range(ntargets):
        starts.append(len(order))
        mine = [i for i, (path, _) in enumerate(entries) if simple_hash(path) % ntargets == k]
        if len(mine) > 1:
            rng = PCG32(0x853C49E6748FEA9B, 0xDA3E39CB94B95BDB)
            for i in range(len(mine) - 1, 0, -1):
                j = rng.next() % (i + 1)
                mine[i], mine[j] = mine[j], mine[i]
        mine.sort(key=lambda i: entries[i][1][3])      # stable
        order += mine
    starts.append(len(order))
    return order, starts


def plan(agg, ntargets: int, cum_weight, prev: dict, rounds: bool = False):
    """-> list of (path bytes, timestamp, locations) in worklist order
    (rounds=True: and the round starts)."""
    entries = list(agg.items())
    order, starts = round_order(entries, ntargets)
    out = []
    for i in order:
        path, (ts, mod, dele, size) = entries[i]
        loc = with_p(mod, NO_P)
        old = prev.get(path)
        if old is not None:
            loc = fill_in_missing(loc, old[1])
        loc &= ~dele & ((1 << 64) - 1)
        if p_is_invalid(loc):
            loc = select_p(path, loc, ntargets, cum_weight)
        if old is not None and old[0] == ts and old[1] == loc:
            loc = with_p(loc, NO_P)
        out.append((path, ts, loc))
    return (out, starts) if rounds else out
