"""The GPU path against the REFERENCE'S OWN xor_parity outputs
(tests/golden/ref_xor.json, made by compiling task_processing.c:96-109
unchanged; tests/golden/make_ref_golden.py).  Every fixture goes through the
C ABI: the xor_parity drop-in (bcp_xor_parity), the batched device entry
points, and -- for the parity-file fixtures -- the per-rank protocol
(process_task over loopback ranks, both fold modes) and the batched pipeline,
gen and rebuild."""
import hashlib
import json
import os

import numpy as np
import pytest

import bcp_store as S

pytestmark = pytest.mark.gpu
DOC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ref_xor.json")))
XOR = [c for c in DOC["cases"] if c["kind"] == "xor_parity"]
GEN = [c for c in DOC["cases"] if c["kind"] == "gen_file"]


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def rows(oracle, fx):
    return np.concatenate([oracle.synthetic(fx["len"], fx["seed"] + k) for k in range(fx["n"])])


@pytest.mark.parametrize("fx", XOR, ids=lambda c: f"n{c['n']}-len{c['len']}")
def test_dropin_matches_reference(bcp, engine, oracle, fx):
    data = rows(oracle, fx)
    assert sha(data) == fx["input_sha256"]
    dst = np.full(max(fx["len"], 1), 0xA5, np.uint8)
    bcp.xor_parity(dst, fx["len"], data, fx["n"])
    assert sha(dst[:fx["len"]]) == fx["sha256"]


@pytest.mark.parametrize("fx", XOR, ids=lambda c: f"n{c['n']}-len{c['len']}")
def test_device_batch_matches_reference(engine, queue, oracle, fx):
    """The same rows as one device-resident stripe ([n][len] contiguous, so
    rows are unaligned for odd lengths: the descriptor kernel) and as a
    256-byte-pitched stripe (the streaming kernel), plus an 8-stripe batch of
    the same stripe for the batched shapes."""
    n, L = fx["n"], fx["len"]
    data = rows(oracle, fx)
    pitch = (L + 255) & ~255
    src = engine.alloc(n * pitch + 16)
    dst = engine.alloc(8 * pitch + 16)
    try:
        queue.h2d(src, data)
        queue.memset(dst, 0x5A, pitch)
        queue.xor_uniform(dst, src, 1, n, L)
        out = np.empty(L, np.uint8)
        queue.d2h(out, dst, L)
        queue.sync()
        assert sha(out) == fx["sha256"], "contiguous rows"
        for k in range(n):  # re-lay at a 256-byte pitch
            queue.h2d(src + k * pitch, data[k * L:(k + 1) * L])
        queue.memset(dst, 0x5A, 8 * pitch)
        queue.xor_strided(dst, pitch, src, 0, pitch, 8, n, L)  # stripe_stride 0: the same stripe 8 times
        outs = np.empty(8 * pitch, np.uint8)
        queue.d2h(outs, dst, 8 * pitch)
        queue.sync()
        for s in range(8):
            assert sha(outs[s * pitch:s * pitch + L]) == fx["sha256"], f"pitched stripe {s}"
    finally:
        queue.sync()
        engine.free(src)
        engine.free(dst)


@pytest.fixture
def gpu_protocol(bcp, engine):
    bcp.set_xor_hook(None)
    yield
    bcp.task_shutdown()


@pytest.mark.parametrize("mode", ["pipelined", "batched", "pipeline"])
@pytest.mark.parametrize("fx", GEN, ids=lambda c: c["name"])
def test_parity_files_match_reference_folds(bcp, oracle, tmp_path, gpu_protocol, fx, mode):
    lens = fx["lens"]
    n = len(lens)
    p = n  # parity on the target after the holders
    nt = n + 1
    root = str(tmp_path)
    S.make_store(root, nt)
    chunks = [oracle.synthetic(L, fx["seed"] + k) for k, L in enumerate(lens)]
    for k, c in enumerate(chunks):
        S.write_chunk(root, k, "r/e/f", c)
    items = [("r/e/f", 2**40, S.with_p((1 << n) - 1, p))]
    prev = None if mode == "pipeline" else bcp.set_fold_mode(
        {"batched": bcp.FOLD_BATCHED, "pipelined": bcp.FOLD_PIPELINED}[mode])
    try:
        _gen_and_rebuild(bcp, root, nt, p, items, fx, mode)
    finally:
        if prev is not None:
            bcp.set_fold_mode(prev)


def _gen_and_rebuild(bcp, root, nt, p, items, fx, mode):
    st = bcp.pipeline_gen(root, nt, items) if mode == "pipeline" else bcp.gen_run(root, nt, items)
    assert st.errors == 0
    pf = S.read_file(S.parity_path(root, p, "r/e/f"))
    assert len(pf) == fx["file_len"] and sha(pf) == fx["sha256"]
    v = fx["rebuild_victim"]
    os.remove(S.chunk_path(root, v, "r/e/f"))
    if mode == "pipeline":
        pl = bcp.Pipeline()
        try:
            st = pl.rebuild(root, nt, v, items)
        finally:
            pl.close()
    else:
        st = bcp.rebuild_run(root, nt, v, items)
    assert st.errors == 0
    assert sha(S.read_file(S.chunk_path(root, v, "r/e/f"))) == fx["rebuilt_sha256"]
