"""Chunk-event records and worklist planning (libbcp bcp_eventset_* /
bcp_plan_worklist) against the Python restatement oracle/planner.py."""
import os
import struct

import numpy as np
import pytest

import planner as PL


def test_pcg32_reference_vector():
    """pcg32-demo (pcg-random.org): srandom(42, 54) -> 0xa15c02b7 0x7b47f409 ..."""
    r = PL.PCG32.seeded(42, 54)
    got = [r.next() for _ in range(6)]
    assert got == [0xA15C02B7, 0x7B47F409, 0xBA1D3330, 0x83D2F293, 0xBFA4784B, 0xCBED606E]


def test_simple_hash_matches(bcp):
    for p in ["", "a", "u0/5F/12-5F8A2B3C-1/1A-5F8A2B3C-1", "caf\xe9/\xff\x80", "x" * 300]:
        b = p.encode("latin-1")
        assert bcp.lib().bcp_path_hash(b, len(b)) == PL.simple_hash(b), p


def random_streams(rng, ntargets, npaths, nrec):
    paths = [f"u{int(rng.integers(0, 4))}/{int(rng.integers(0, 1 << 24)):06X}/c{i}" for i in range(npaths)]
    streams = []
    for st in range(ntargets):
        recs = []
        for _ in range(int(rng.integers(0, nrec))):
            recs.append((int(rng.integers(1, 1 << 40)), int(rng.integers(0, 1 << 23)),
                         "d" if rng.random() < 0.15 else "m", paths[int(rng.integers(0, npaths))]))
        streams.append((st, recs))
    return streams


@pytest.mark.parametrize("seed", range(5))
def test_eventset_and_plan_match_restatement(bcp, seed):
    rng = np.random.default_rng(seed)
    ntargets = int(rng.integers(3, 20))
    streams = random_streams(rng, ntargets, 200, 150)
    es = bcp.EventSet()
    packed = []
    for st, recs in streams:
        data = bcp.pack_records(recs)
        packed.append((st, data))
        # feed in uneven pieces: partial records must carry over
        cuts = sorted(int(x) for x in rng.integers(0, len(data) + 1, size=3))
        for a, b in zip([0] + cuts, cuts + [len(data)]):
            es.feed(st, data[a:b])
    agg = PL.aggregate(packed)
    got = es.entries()
    assert [(p.encode(), ts, m, d, sz) for p, ts, m, d, sz in got] == \
        [(p, *v) for p, v in agg.items()]
    weights = [int(x) for x in rng.integers(0, 7000, size=ntargets)]
    weights[int(rng.integers(0, ntargets))] += 1
    cum = list(np.cumsum(weights))
    # previous state: some paths known, some with identical state (-> NO_P)
    prev = {}
    for p, (ts, m, d, sz) in list(agg.items())[::3]:
        p_old = int(rng.integers(0, ntargets))
        prev[p] = (ts if rng.random() < 0.5 else ts - 1, PL.with_p(int(rng.integers(0, 1 << ntargets)) & ~(1 << p_old),
                                                                     p_old))
    want = PL.plan(agg, ntargets, cum, prev)
    got = es.plan(ntargets, cum, [(p.decode(), ts, loc) for p, (ts, loc) in prev.items()])
    assert [(p.encode(), ts, loc) for p, ts, loc in got] == want
    es.close()


def test_plan_properties(bcp):
    es = bcp.EventSet()
    recs = [(100, 4096, "m", "a"), (101, 4096, "m", "b"), (99, 10, "d", "c")]
    es.feed(0, bcp.pack_records(recs))
    es.feed(2, bcp.pack_records([(105, 4096, "m", "a")]))
    items = {p: (ts, loc) for p, ts, loc in es.plan(4, [1000, 2000, 3000, 4000])}
    ts, loc = items["a"]
    assert ts == 105 and loc & PL.L_MASK == 0b101
    assert PL.get_p(loc) in (1, 3)                    # never a holder
    # all holders deleted: locations empty, P still chosen -> parity unlinked downstream
    assert items["c"][1] & PL.L_MASK == 0
    # unchanged against the previous state -> NO_P
    items2 = es.plan(4, [1000, 2000, 3000, 4000], prev=[("a", ts, loc)])
    assert dict((p, l) for p, _, l in items2)["a"] >> 56 == PL.NO_P
    es.close()


def test_truncated_stream_rejected(bcp, tmp_path):
    data = bcp.pack_records([(1, 2, "m", "abc"), (1, 2, "m", "defg")])
    f = tmp_path / "log"
    f.write_bytes(data[:-2])
    es = bcp.EventSet()
    with pytest.raises(bcp.BcpError):
        es.feed_file(0, str(f))
    es.close()
    es = bcp.EventSet()
    f.write_bytes(data)
    es.feed_file(3, str(f))
    assert [e[0] for e in es.entries()] == ["abc", "defg"]
    assert es.entries()[0][2] == 1 << 3
    es.close()


def test_absolute_paths_rejected(bcp):
    es = bcp.EventSet()
    with pytest.raises(bcp.BcpError):
        es.feed(0, bcp.pack_records([(1, 2, "m", "/abs")]))
    es.close()


@pytest.mark.parametrize("bad", ["../x", "a/../../x", "a/..", "..", "a\0b"])
def test_paths_leaving_the_store_rejected(bcp, bad):
    """A record path names <store>/st<k>/chunks/<path> and the parity file on
    P: no ".." component and no embedded NUL."""
    es = bcp.EventSet()
    with pytest.raises(bcp.BcpError):
        es.feed(0, bcp.pack_records([(1, 2, "m", bad)]))
    es.close()
    es = bcp.EventSet()
    es.feed(0, bcp.pack_records([(1, 2, "m", "a/..b/c..d/...")]))  # dots inside names are fine
    assert [e[0] for e in es.entries()] == ["a/..b/c..d/..."]
    es.close()


def test_store_weight(bcp, tmp_path):
    fd = os.open(str(tmp_path), os.O_DIRECTORY | os.O_RDONLY)
    try:
        w = bcp.lib().bcp_store_weight(fd)
        st = os.statvfs(str(tmp_path))
        pct = float(100 * st.f_bfree // st.f_blocks)
        import math
        assert w == int(1000 * math.log2(pct + 1.1))
        (tmp_path / "free_space.override").write_text(str(st.f_blocks * st.f_bsize // 2))
        w2 = bcp.lib().bcp_store_weight(fd)
        pct2 = float(100 * (st.f_blocks * st.f_bsize // 2 // st.f_bsize) // st.f_blocks)
        assert w2 == int(1000 * math.log2(pct2 + 1.1))
    finally:
        os.close(fd)
