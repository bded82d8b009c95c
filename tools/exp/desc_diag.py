#!/usr/bin/env python3
"""Diagnostic (tools only): tests/test_gpu_xor.py::test_descriptor_mixed_lengths_and_alignment
inputs, per-stripe mismatch report against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import oracle  # noqa: E402

eng = bcp.Engine(0)
q = eng.queue()
T = 32768
for seed in range(3):
    rng = np.random.default_rng(100 + seed)
    stripes, sources, outs, refs, meta = [], [], [], [], []
    ptrs = []
    for _ in range(int(rng.integers(1, 12))):
        n = int(rng.integers(1, 10))
        lens = [int(x) for x in rng.integers(0, 300000, size=n)]
        chunks = [rng.integers(0, 256, size=L, dtype=np.uint8) for L in lens]
        pads = [int(x) for x in rng.integers(0, 16, size=n)]
        m = max(lens)
        dst_pad = int(rng.integers(0, 16))
        first = len(sources)
        for c, pad in zip(chunks, pads):
            if len(c) == 0:
                sources.append((0, 0))
                continue
            base = eng.alloc(len(c) + pad + 16)
            ptrs.append(base)
            q.h2d(base + pad, c)
            sources.append((base + pad, len(c)))
        d = eng.alloc(m + 32)
        ptrs.append(d)
        stripes.append((d + dst_pad, m, first, n, 0))
        outs.append((d + dst_pad, m))
        refs.append(np.frombuffer(oracle.gen_parity_file(chunks)[8 * n:], np.uint8))
        meta.append((lens, pads, dst_pad))
    q.xor_stripes(stripes, sources)
    q.sync()
    for i, ((p, m), r) in enumerate(zip(outs, refs)):
        got = np.empty(max(m, 1), np.uint8)
        if m:
            q.d2h(got, p, m)
        q.sync()
        got = got[:m]
        bad = np.nonzero(got != r)[0]
        lens, pads, dpad = meta[i]
        if len(bad):
            tiles = sorted(set(int(x) // T for x in bad))
            print(f"seed {seed} stripe {i}: lens {lens} pads {pads} dst_pad {dpad}: {len(bad)} bad bytes, "
                  f"first {bad[:4].tolist()} last {bad[-1]}, tiles {tiles[:10]}", flush=True)
        else:
            print(f"seed {seed} stripe {i}: ok (n={len(lens)}, m={m})", flush=True)
    for p in ptrs:
        eng.free(p)
