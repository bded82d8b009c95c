#!/usr/bin/env python3
"""Latency of one protocol window fold (the P role's per-task GPU work) and
where it goes: pinned rows -> H2D -> xor kernel -> D2H -> sync, each step
alone, and the zero-copy form (kernel reads the pinned rows and writes the
pinned output over PCIe directly).  One JSON line per measurement.

    python tools/proto_latency.py [--n 3] [--chunk 524288] [--iters 300]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import ctypes  # noqa: E402

import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=3)
ap.add_argument("--chunk", type=int, default=512 * 1024)
ap.add_argument("--iters", type=int, default=300)
ap.add_argument("--vecs", default="", help="comma list: also time the zero-copy mapped fold at these tile sizes")
a = ap.parse_args()

eng = bcp.Engine(0)
q = eng.queue()
n, C = a.n, a.chunk
h_rows = eng.host_alloc(n * C)
h_out = eng.host_alloc(C)
d_src = eng.alloc(n * C)
d_out = eng.alloc(C)
rows = np.ctypeslib.as_array((ctypes.c_uint8 * (n * C)).from_address(h_rows))
out = np.ctypeslib.as_array((ctypes.c_uint8 * C).from_address(h_out))
rows[:] = np.random.default_rng(1).integers(0, 256, size=n * C, dtype=np.uint8)
ref = np.bitwise_xor.reduce(rows.reshape(n, C), axis=0)


def timed(label, fn, check=None):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    ok = None
    if check is not None:
        out[:] = 0
        fn()
        ok = bool(np.array_equal(out, ref))
    med = statistics.median(ts)
    print(json.dumps({"step": label, "n": n, "chunk": C, "median_us": round(med, 1),
                      "p10_us": round(sorted(ts)[len(ts) // 10], 1), "GBps_moved": round((n + 1) * C / med / 1e3, 2),
                      "correct": ok}), flush=True)


def full():
    q.h2d(d_src, h_rows, n * C)
    q.xor_strided(d_out, C, d_src, n * C, C, 1, n, C)
    q.d2h(h_out, d_out, C)
    q.sync()


def zero_copy():
    q.xor_strided(h_out, C, h_rows, n * C, C, 1, n, C)
    q.sync()


def h2d_only():
    q.h2d(d_src, h_rows, n * C)
    q.sync()


def kern_only():
    q.xor_strided(d_out, C, d_src, n * C, C, 1, n, C)
    q.sync()


def d2h_only():
    q.d2h(h_out, d_out, C)
    q.sync()


timed("empty_sync", q.sync)
timed("h2d+sync", h2d_only)
timed("kernel+sync", kern_only)
timed("d2h+sync", d2h_only)
timed("fold_window(h2d,kernel,d2h,sync)", full, check=True)
timed("zero_copy(kernel on pinned host rows)", zero_copy, check=True)
# the same on coherent mapped memory (what the P role's fold resources use)
m_rows = eng.host_alloc(n * C, mapped=True)
m_out = eng.host_alloc(C, mapped=True)
mrows = np.ctypeslib.as_array((ctypes.c_uint8 * (n * C)).from_address(m_rows))
mout = np.ctypeslib.as_array((ctypes.c_uint8 * C).from_address(m_out))
mrows[:] = rows


def zero_copy_mapped():
    q.xor_strided(m_out, C, m_rows, n * C, C, 1, n, C)
    q.sync()


timed("zero_copy_mapped(kernel on coherent mapped rows)", zero_copy_mapped)
mout[:] = 0
zero_copy_mapped()
print(json.dumps({"step": "zero_copy_mapped_check", "correct": bool(np.array_equal(mout, ref))}))
# changing data in the same buffers between folds (no stale lines)
rng = np.random.default_rng(7)
bad = 0
for i in range(50):
    mrows[:] = rng.integers(0, 256, size=n * C, dtype=np.uint8)
    zero_copy_mapped()
    bad += not np.array_equal(mout, np.bitwise_xor.reduce(mrows.reshape(n, C), axis=0))
print(json.dumps({"step": "zero_copy_mapped_reuse_50", "mismatching_folds": bad}))
for v in filter(None, a.vecs.split(",")):
    eng.tune(0, int(v))
    timed(f"zero_copy_mapped vecs={v}", zero_copy_mapped)
eng.tune(0, 0)
pg_rows = rows.copy()
pg_out = np.empty(C, dtype=np.uint8)
timed("bcp_xor_parity(drop-in, pageable)", lambda: bcp.xor_parity(pg_out, C, pg_rows, n))
