#!/usr/bin/env python3
"""Interleaved A/B sweep of the 8-wide fast-path knobs in ONE process
(cdna_hip_programming.md §5.4 rule 24): blocks_per_cu x vecs_per_thread,
each launch timed alone with HIP events on the kernel's stream.  (r01 also
swept a static tile schedule, since removed: profiles/r01/sweep_fast*.jsonl.)
Also compares back-to-back launches with isolated ones.

    python tools/sweep_fast.py [--stripes 12500] [--reps 5] > sweep.jsonl
"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--stripes", type=int, default=12500)
ap.add_argument("--nsrc", type=int, default=8)
ap.add_argument("--chunk", type=int, default=512 * 1024)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--bpc", default="1,2,4")
ap.add_argument("--vecs", default="2,4,8")
a = ap.parse_args()

eng = bcp.Engine(0)
q = eng.queue()
S, N, C = a.stripes, a.nsrc, a.chunk
src = eng.alloc(S * N * C)
out = eng.alloc(S * C)
q.fill_synthetic(src, S * N * C, 1)
q.sync()
bytes_per = S * (N + 1) * C
variants = list(itertools.product([int(x) for x in a.bpc.split(",")], [int(x) for x in a.vecs.split(",")]))
res = {v: [] for v in variants}
t_start = time.time()
for rep in range(a.reps):
    for v in variants:
        eng.tune(v[0], v[1])
        q.xor_uniform(out, src, S, N, C)  # warm this variant
        q.mark(0)
        q.xor_uniform(out, src, S, N, C)
        q.mark(1)
        res[v].append(q.elapsed_ms(0, 1))
    print(json.dumps({"progress": rep + 1, "of": a.reps, "elapsed_s": round(time.time() - t_start, 1)}),
          file=sys.stderr, flush=True)
rows = []
for v, ts in res.items():
    med = statistics.median(ts)
    rows.append({"blocks_per_cu": v[0], "vecs": v[1], "median_ms": round(med, 4),
                 "min_ms": round(min(ts), 4), "GBps_median": round(bytes_per / med / 1e6, 1),
                 "frac_8TBs": round(bytes_per / med / 1e6 / 8000, 4)})
rows.sort(key=lambda r: r["median_ms"])
for r in rows:
    print(json.dumps(r))

# back-to-back vs isolated for the best and the default variant
for v in (tuple(rows[0][k] for k in ("blocks_per_cu", "vecs")), (0, 0)):
    eng.tune(v[0], v[1])
    q.mark(2)
    for i in range(10):
        q.xor_uniform(out, src, S, N, C)
    q.mark(3)
    b2b = q.elapsed_ms(2, 3) / 10
    iso = []
    for i in range(10):
        q.sync()
        time.sleep(0.02)
        q.mark(4)
        q.xor_uniform(out, src, S, N, C)
        q.mark(5)
        iso.append(q.elapsed_ms(4, 5))
    print(json.dumps({"variant": v, "b2b_ms": round(b2b, 4), "isolated_median_ms": round(statistics.median(iso), 4),
                      "b2b_GBps": round(bytes_per / b2b / 1e6, 1),
                      "isolated_GBps": round(bytes_per / statistics.median(iso) / 1e6, 1)}))
q.close()
eng.close()
