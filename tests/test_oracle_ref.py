"""Oracle pinning against the REFERENCE'S OWN xor_parity.

tests/golden/ref_xor.json holds outputs of task_processing.c:96-109 compiled
unchanged (oracle/_ref, tests/golden/make_ref_golden.py) on distinct random
rows.  The C restatement (oracle/bcp_oracle.c) must reproduce every one; so
must the GPU path (tests/test_gpu_ref.py).  Where oracle/_ref was built (this
container) the restatement is also cross-checked against the reference
function directly on random shapes and pointer alignments."""
import hashlib
import json
import os

import numpy as np
import pytest

DOC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_xor.json")))
XOR = [c for c in DOC["cases"] if c["kind"] == "xor_parity"]
GEN = [c for c in DOC["cases"] if c["kind"] == "gen_file"]


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def rows(oracle, n, length, seed):
    return np.concatenate([oracle.synthetic(length, seed + k) for k in range(n)])


def test_fixture_coverage():
    assert {c["n"] for c in XOR} == {1, 2, 3, 5, 8, 13, 56}
    assert {c["len"] for c in XOR} == {1, 7, 8, 9, 15, 16, 17, 4095, 65536, 524288, 524289}
    assert len(XOR) == 77 and len(GEN) == 4
    # distinct rows: the parity of >= 2 random rows is not all zero
    assert all(c["sha256"] != sha(bytes(c["len"])) for c in XOR if c["n"] >= 2)


@pytest.mark.parametrize("fx", XOR, ids=lambda c: f"n{c['n']}-len{c['len']}")
def test_oracle_reproduces_reference_xor_parity(oracle, fx):
    data = rows(oracle, fx["n"], fx["len"], fx["seed"])
    assert sha(data) == fx["input_sha256"]
    out = oracle.xor_parity(data, fx["len"], fx["n"])
    assert sha(out) == fx["sha256"]
    if "out_hex" in fx:
        assert out.tobytes().hex() == fx["out_hex"]


@pytest.mark.parametrize("fx", GEN, ids=lambda c: c["name"])
def test_oracle_protocol_assembly_on_reference_folds(oracle, fx):
    chunks = [oracle.synthetic(L, fx["seed"] + k) for k, L in enumerate(fx["lens"])]
    assert [sha(c) for c in chunks] == fx["inputs_sha256"]
    pf = oracle.gen_parity_file(chunks)
    assert len(pf) == fx["file_len"] and sha(pf) == fx["sha256"]
    v = fx["rebuild_victim"]
    rb = oracle.rebuild_chunk(pf, [c for k, c in enumerate(chunks) if k != v], v)
    assert sha(rb) == fx["rebuilt_sha256"] == fx["inputs_sha256"][v]


def _ref_or_skip(oracle):
    if oracle.ref_lib() is None and oracle.build_ref() is None:
        pytest.skip("oracle/_ref not built here (no /root/reference)")
    return oracle.ref_lib()


@pytest.mark.parametrize("fx", [c for c in XOR if c["n"] * c["len"] <= 1 << 20], ids=lambda c: f"n{c['n']}-len{c['len']}")
def test_fixtures_still_match_reference(oracle, fx):
    _ref_or_skip(oracle)
    data = rows(oracle, fx["n"], fx["len"], fx["seed"])
    assert sha(oracle.ref_xor_parity(data, fx["len"], fx["n"])) == fx["sha256"]


@pytest.mark.parametrize("seed", range(40))
def test_oracle_vs_reference_random_shapes(oracle, seed):
    """Random n, length and a misaligned data/dst start (the reference does
    unaligned u64 accesses, task_processing.c:104-105)."""
    _ref_or_skip(oracle)
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 57))
    L = int(rng.choice([int(rng.integers(0, 64)), int(rng.integers(64, 70000))]))
    shift = int(rng.integers(0, 8))
    buf = rng.integers(0, 256, size=n * L + shift, dtype=np.uint8)
    data = buf[shift:]
    a = oracle.ref_xor_parity(data, L, n)
    b = oracle.xor_parity(data, L, n)
    assert np.array_equal(a, b)
    if n * L:
        assert np.array_equal(b, np.bitwise_xor.reduce(data[: n * L].reshape(n, L), axis=0))
