"""Oracle pinning: the C restatement (oracle/bcp_oracle.c) must reproduce the
known answers SURVEY.md §8(c) recorded from the unchanged reference, and the
committed regression vectors (tests/golden/kats.json)."""
import hashlib
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kats.json")))


def fnv1a64(b: bytes) -> str:
    a = np.frombuffer(b, dtype=np.uint8)
    h = 0xCBF29CE484222325
    # chunked pure-python loop is too slow for 512 KiB; do it in numpy-free C-ish steps
    for x in a.tolist():
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def test_kat1_xor_parity(oracle):
    k = GOLD["survey_kats"]["KAT-1"]
    data = oracle.kat1_data(k["n"], k["s"])
    par = oracle.xor_parity(data, k["s"], k["n"]).tobytes()
    assert hashlib.sha256(par).hexdigest() == k["sha256"]
    # KAT-1 is degenerate: rows 2^19 apart cancel, so its parity is all zero
    # (its SHA-256 is that of 512 KiB of zeros).  The FNV value SURVEY.md lists
    # (0feb61957bfd0383) matches neither FNV-1a nor FNV-1 of these bytes
    # (fc31bff590c22325); SHA-256 is the pin.  KAT-2..4 carry the real signal.
    assert not par.strip(b"\0")
    assert fnv1a64(par) == "fc31bff590c22325"


@pytest.mark.parametrize("name", ["KAT-2", "KAT-3", "KAT-4"])
def test_kat_protocol_gen_and_rebuild(oracle, name):
    k = GOLD["survey_kats"][name]
    chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(k["lens"])]
    pf = oracle.gen_parity_file(chunks)
    assert len(pf) == k["file_len"]
    assert hashlib.sha256(pf).hexdigest() == k["sha256"]
    # The KAT generator's byte j does not depend on k (k only moves bits >= 32
    # before the >> 13), so KAT-2 (8 equal chunks) and KAT-4 (window 0 cancels,
    # windows 1-2 replay identical bytes) have all-zero bodies; KAT-3's mixed
    # lengths make it the non-degenerate one.  Random-data cases below and in
    # the GPU suite carry the rest of the signal.
    nz = np.count_nonzero(np.frombuffer(pf[8 * len(chunks):], np.uint8))
    assert (nz > 0) == (name == "KAT-3")
    hdr = np.frombuffer(pf[: 8 * len(chunks)], dtype="<u8")
    assert hdr.tolist() == k["lens"]
    v = k["rebuild_victim"]
    rb = oracle.rebuild_chunk(pf, [c for i, c in enumerate(chunks) if i != v], v)
    assert rb == chunks[v].tobytes()


def test_kat4_differs_from_zero_padding(oracle):
    """Quirk A3-q1: past one window a short source replays its last window."""
    lens = GOLD["survey_kats"]["KAT-4"]["lens"]
    chunks = [oracle.kat_chunk(i, L) for i, L in enumerate(lens)]
    body = np.frombuffer(oracle.gen_parity_file(chunks)[16:], dtype=np.uint8)
    padded = oracle.xor_padded_np(chunks)
    W = oracle.WINDOW
    assert np.array_equal(body[:W], padded[:W])
    assert not np.array_equal(body[W:], padded[W:])
    # window 1 and 2 of source 0 replay its window 0
    replay = padded.copy()
    for w in (1, 2):
        lo, hi = w * W, min((w + 1) * W, len(replay))
        replay[lo:hi] ^= chunks[0][: hi - lo]
    assert np.array_equal(body, replay)


def test_generators_agree(oracle):
    for k in (0, 1, 7, 55):
        assert np.array_equal(oracle.kat_chunk(k, 5000), oracle.kat_chunk_np(k, 5000))


@pytest.mark.parametrize("fx", GOLD["edge"], ids=lambda fx: f"{fx['kind']}-{fx.get('n', len(fx.get('lens', [])))}-"
                         f"{fx.get('s', fx.get('lens'))}-{fx.get('window', 0)}")
def test_edge_vectors(oracle, fx):
    if fx["kind"] == "xor_parity":
        data = oracle.kat1_data(fx["n"], fx["s"])
        out = oracle.xor_parity(data, fx["s"], fx["n"]).tobytes()
    else:
        chunks = [oracle.synthetic(L, 1000 + i) for i, L in enumerate(fx["lens"])]
        out = oracle.gen_parity_file(chunks, window=fx.get("window", oracle.WINDOW))
        assert len(out) == fx["file_len"]
    assert hashlib.sha256(out).hexdigest() == fx["sha256"]


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_numpy_padding_below_window(oracle, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 12))
    lens = [int(x) for x in rng.integers(0, 70000, size=n)]
    chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
    pf = oracle.gen_parity_file(chunks)
    assert np.array_equal(np.frombuffer(pf[8 * n:], np.uint8), oracle.xor_padded_np(chunks))
    v = int(rng.integers(0, n))
    rb = oracle.rebuild_chunk(pf, [c for i, c in enumerate(chunks) if i != v], v)
    assert rb == chunks[v].tobytes()


def test_unreadable_source_sends_zeros(oracle):
    a = oracle.kat_chunk(0, 1000)
    pf = oracle.gen_parity_file([a, None])
    hdr = np.frombuffer(pf[:16], dtype="<u8")
    assert hdr.tolist() == [1000, 0]
    assert pf[16:] == a.tobytes()


def test_all_empty_sources(oracle):
    pf = oracle.gen_parity_file([np.zeros(0, np.uint8)] * 3)
    assert pf == b"\0" * 24


def test_rebuild_index(oracle):
    # chunks on targets {0,2,5,7}, parity on 3; rebuilding 5 -> re-roled
    # locations = {0,2,3,7} (P bit on, victim off); index of 5 among {0,2,5,7} = 2
    loc = (1 << 0) | (1 << 2) | (1 << 3) | (1 << 7)
    assert oracle.rebuild_index(loc, 3, 5) == 2
    assert oracle.rebuild_index(loc, 3, 1) == 1


def test_synthetic_stream_offsets(oracle):
    full = oracle.synthetic(1000, 42)
    assert np.array_equal(oracle.synthetic(100, 42, 333), full[333:433])
