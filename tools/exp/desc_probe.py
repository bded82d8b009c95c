#!/usr/bin/env python3
"""Where does the descriptor kernel (xor_desc) lose against xor_stream?
(tools only).  Times xor_desc on shapes that separate the effects:

  uniform_forced config 2 (8 x 512 KiB) through xor_desc (engine option desc_force)
  uniform_desc   12,500 stripes x 8 x (512 KiB - 8 B): config-2 bytes, but a
                 non-16-multiple length forces the descriptor path
  mixed          config-5 shapes (bench.py --mode mixed): log-uniform lengths
  mixed_equal    the same stripe maxima, every source of a stripe as long as
                 the maximum (no zero padding, fewer bytes per tile varies
                 only across stripes)
  mixed_big      like mixed, lengths log-uniform in [1 MiB, 4 MiB]
  wide16         16-wide stripes with config-5 lengths (> 8 sources per tile)
  window         8 sources of 4-24 MiB: stripes past the 10 MiB transfer window
                 (window replay, quirk A3-q1)

Each line: workload, tuning, kernel ms (HIP events on the queue), algorithmic
GB/s and fraction of 8 TB/s.

    python tools/exp/desc_probe.py [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

KiB, MiB = 1024, 1024 ** 2
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--tunings", default="8:2,8:1,8:3,4:2")
ap.add_argument("--workloads", default="uniform_forced,uniform_desc,mixed,mixed_equal,mixed_big")
ap.add_argument("--pipes", default="0", help="engine desc_pipe values to time (rolling load window)")
ap.add_argument("--rounds", type=int, default=1, help="repeat the whole sweep (interleaved A/B)")
a = ap.parse_args()

eng = bcp.Engine(0)
q = eng.queue()
BUDGET = 12_500 * 8 * 512 * KiB
src = eng.alloc(BUDGET + 64 * MiB)
q.fill_synthetic(src, BUDGET + 64 * MiB, seed=1)
q.sync()
align = lambda x: (x + 255) & ~255  # noqa: E731


def shapes(kind, rng):
    lens_all, tot = [], 0
    while True:
        if kind == "uniform_desc":
            ls = np.full(8, 512 * KiB - 8, dtype=np.int64)
        elif kind == "uniform_forced":
            ls = np.full(8, 512 * KiB, dtype=np.int64)
        elif kind == "window":
            ls = np.exp(rng.uniform(np.log(4 * MiB), np.log(24 * MiB), size=8)).astype(np.int64)
        elif kind == "wide16":
            ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=16)).astype(np.int64)
        elif kind == "mixed_big":
            ls = np.exp(rng.uniform(np.log(1 * MiB), np.log(4 * MiB), size=8)).astype(np.int64)
        else:
            ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8)).astype(np.int64)
            if kind == "mixed_equal":
                ls = np.full(8, int(ls.max()), dtype=np.int64)
        if tot + sum(align(int(x)) for x in ls) > BUDGET:
            return lens_all
        lens_all.append(ls)
        tot += sum(align(int(x)) for x in ls)


def build(lens_all, out):
    stripes, sources, so_off, do_off = [], [], 0, 0
    for ls in lens_all:
        first = len(sources)
        for x in ls:
            sources.append((src + so_off, int(x)))
            so_off += align(int(x))
        m = int(ls.max())
        W = 10 * MiB
        stripes.append((out + do_off, m, first, len(ls), W if m > W else 0))
        do_off += align(m)
    st = (bcp.Stripe * len(stripes))(*[bcp.Stripe(*x) for x in stripes])
    so = (bcp.Source * len(sources))(*[bcp.Source(*x) for x in sources])
    nbytes = sum(int(ls.sum()) + int(ls.max()) for ls in lens_all)
    assert so_off <= BUDGET + 64 * MiB and do_off <= out_bytes(lens_all)
    return st, so, nbytes


def out_bytes(lens_all):
    return sum(align(int(ls.max())) for ls in lens_all)


L = bcp.lib()
for rnd, kind in [(r, k) for r in range(a.rounds) for k in a.workloads.split(",")]:
    eng.option("desc_force", 1 if kind == "uniform_forced" else 0)
    lens_all = shapes(kind, np.random.default_rng(3))
    out = eng.alloc(out_bytes(lens_all))
    st, so, nbytes = build(lens_all, out)
    for tun, pipe in [(t, int(p)) for t in a.tunings.split(",") for p in a.pipes.split(",")]:
        eng.option("desc_pipe", pipe)
        parts = [int(x) for x in tun.split(":")]
        u, bpc = parts[0], parts[1]
        grid = parts[2] if len(parts) > 2 else 0
        eng.option("desc_vecs_per_thread", u)
        eng.option("desc_blocks_per_cu", bpc)
        eng.option("desc_grid", grid)
        for _ in range(2):
            bcp.check("x", L.bcp_xor_stripes_async(q.h, st, len(st), so, len(so)))
        q.sync()
        # steady state as bench.py runs it: launches back to back, the host
        # stages launch k+1 while the device runs launch k (one launch is
        # queued ahead of the first mark so the device is busy from the start)
        bcp.check("x", L.bcp_xor_stripes_async(q.h, st, len(st), so, len(so)))
        q.mark(0)
        for _ in range(a.reps):
            bcp.check("x", L.bcp_xor_stripes_async(q.h, st, len(st), so, len(so)))
        q.mark(1)
        q.sync()
        ms = q.elapsed_ms(0, 1) / a.reps
        tiles = sum((int(ls.max()) + 4096 * u - 1) // (4096 * u) for ls in lens_all)
        print(json.dumps({"workload": kind, "round": rnd, "pipe": pipe, "vecs": u, "blocks_per_cu": bpc, "grid": grid, "stripes": len(st),
                          "subtiles": tiles, "bytes_per_subtile": round(nbytes / tiles), "kernel_ms": round(ms, 4),
                          "GBps": round(nbytes / ms / 1e6, 1), "frac_8TBs": round(nbytes / ms / 8e9, 4)}),
              flush=True)
    eng.free(out)
