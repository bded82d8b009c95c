#!/usr/bin/env python3
"""Throughput and latency against batch size (stripes per launch), 8 x 512 KiB
stripes, device-resident.  For each batch size and each entry point:

  stream  bcp_xor_uniform_async (xor_stream<8,U>, the config-2 kernel)
  table   bcp_xor_stripes_async with a descriptor table of the same stripes
          (uniform: host staging + the pointer-table xor_stream, the rebuild form)
  desc    the same stripes with the first stripe's last source 16 bytes short
          (zero padding: not uniform, so the descriptor kernel takes the batch;
          batches of <= 16 stripes in the kernel arguments, xor_desc_args;
          larger ones host staging + desc_tiles + xor_desc, the config-5 kernel)
  desc_tiles  as desc with desc_args_max = 0: always desc_tiles + xor_desc

two figures:
  pipelined_us  launches back to back, HIP-event time per launch on the queue
                (what a caller that keeps the queue fed sees)
  latency_us    submit + bcp_queue_sync, host wall clock per call (one batch
                in flight at a time: what a per-task caller sees)

GB/s uses algorithmic bytes ((N+1) x 512 KiB per stripe).  One JSON line per
(batch, entry point).

    python tools/batch_curve.py [--reps 50] [--batches 1,2,4,...]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

KiB = 1024
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--batches", default="1,2,4,8,16,32,64,128,256,512,1024,2048,4096,12500")
ap.add_argument("--entries", default="stream,table,desc,desc_tiles")
ap.add_argument("--table-host-max", default="", help="comma list: time table/desc at each engine table_host_max")
ap.add_argument("--tunings", default="",
                help="U:bpc list: time the stream entry with each explicit tuning (A/B for small batches)")
a = ap.parse_args()

N, C = 8, 512 * KiB
batches = [int(x) for x in a.batches.split(",")]
smax = max(batches)
eng = bcp.Engine(0)
q = eng.queue()
src = eng.alloc(smax * N * C)
dst = eng.alloc(smax * C)
q.fill_synthetic(src, smax * N * C, seed=1)
q.sync()


def tables(s, short=0):
    stripes = (bcp.Stripe * s)(*[bcp.Stripe(dst + i * C, C, i * N, N, 0) for i in range(s)])
    sources = (bcp.Source * (s * N))(*[bcp.Source(src + (i * N + k) * C, C - (short if i * N + k == N - 1 else 0))
                                        for i in range(s) for k in range(N)])
    return stripes, sources


for s in batches:
    nbytes = s * (N + 1) * C
    st, so = tables(s)
    dst_, dso = tables(s, short=16)
    L = bcp.lib()
    table = lambda: bcp.check("xor_stripes", L.bcp_xor_stripes_async(q.h, st, s, so, s * N))  # noqa: E731
    desc = lambda: bcp.check("xor_stripes", L.bcp_xor_stripes_async(q.h, dst_, s, dso, s * N))  # noqa: E731
    entry = {
        "stream": lambda: q.xor_uniform(dst, src, s, N, C),
        "table": table,
        "desc": desc,
        "desc_tiles": desc,
    }
    runs = [(n, entry[n], None) for n in a.entries.split(",") if n]
    for thm in filter(None, a.table_host_max.split(",")):
        runs += [("table", table, ("thm", int(thm))), ("desc", desc, ("thm", int(thm)))]
    for tun in filter(None, a.tunings.split(",")):
        u, bpc = (int(x) for x in tun.split(":"))
        runs.append(("stream", entry["stream"], (u, bpc)))
    for name, fn, tun in runs:
        eng.option("desc_args_max", 0 if name == "desc_tiles" else 16)
        if tun and tun[0] == "thm":
            eng.option("table_host_max", tun[1])
        elif tun:
            eng.tune(tun[1], tun[0])
        reps = max(3, min(a.reps, int(2e9 // nbytes)))
        for _ in range(3):
            fn()
        q.sync()
        fn()  # one launch queued ahead of the first mark
        q.mark(0)
        for _ in range(reps):
            fn()
        q.mark(1)
        q.sync()
        pip_us = q.elapsed_ms(0, 1) / reps * 1e3
        lat = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            q.sync()
            lat.append((time.perf_counter() - t0) * 1e6)
        lat_us = statistics.median(lat)
        print(json.dumps({"stripes": s, "entry": name, "tuning": tun, "bytes": nbytes, "reps": reps,
                          "pipelined_us": round(pip_us, 2), "pipelined_GBps": round(nbytes / pip_us / 1e3, 1),
                          "pipelined_frac_8TBs": round(nbytes / pip_us / 8e6, 4),
                          "latency_us": round(lat_us, 2), "latency_GBps": round(nbytes / lat_us / 1e3, 1)}),
              flush=True)
