#!/usr/bin/env python3
"""Does desc_tiles' HBM traffic, running beside the fold on the copy stream,
cost the descriptor kernel anything on config-5 shapes?  (tools only; VERDICT
r02 item 8.)  bench.py --mode mixed's batch (seeded log-uniform 64 KiB-4 MiB
lengths, 6,601 stripes x 8), timed interleaved in one process:

  records_each_launch   the shipped path: every launch uploads its tables and
                        runs desc_tiles on the copy stream (overlapping the
                        previous launch's fold), then xor_desc
  records_precomputed   engine option desc_reuse_records: the tables and tile
                        records made by the warm-up launches stand (each of
                        the 4 ring slots made its own), so the timed launches
                        are xor_desc alone

Each line: variant, round, kernel ms per launch (HIP events on the queue's
stream, so the records' side work counts where it delays the fold), fraction
of 8 TB/s on the algorithmic bytes (sum of lengths + stripe maxima).  The
output of both variants is checked equal (device checksum).

    python tools/exp/desc_records_ab.py [--rounds 6 --steps 20]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

KiB = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    eng = bcp.Engine(0)
    q = eng.queue()
    S, N, C = 12_500, 8, 512 * KiB
    rng = np.random.default_rng(3)
    budget = S * N * C
    lens_all, tot = [], 0
    while tot < budget:
        ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=N)).astype(np.int64)
        lens_all.append(ls)
        tot += int(ls.sum())
    align = lambda x: (x + 255) & ~255  # noqa: E731
    src_bytes = sum(int(sum(align(int(x)) for x in ls)) for ls in lens_all)
    out_bytes = sum(align(int(ls.max())) for ls in lens_all)
    src = eng.alloc(src_bytes)
    out = eng.alloc(out_bytes)
    chk = eng.alloc(64)
    q.fill_synthetic(src, src_bytes, seed=1)
    stripes, sources, so_off, do_off = [], [], 0, 0
    for ls in lens_all:
        first = len(sources)
        for x in ls:
            sources.append((src + so_off, int(x)))
            so_off += align(int(x))
        m = int(ls.max())
        stripes.append((out + do_off, m, first, N, 0))
        do_off += align(m)
    st = (bcp.Stripe * len(stripes))(*[bcp.Stripe(*x) for x in stripes])
    so = (bcp.Source * len(sources))(*[bcp.Source(*x) for x in sources])
    L = bcp.lib()
    nbytes = sum(int(ls.sum()) + int(ls.max()) for ls in lens_all)

    def step():
        bcp.check("bcp_xor_stripes_async", L.bcp_xor_stripes_async(q.h, st, len(stripes), so, len(sources)))

    def checksum():
        q.memset(out, 0xA5, out_bytes)
        step()
        q.xor_fold(out, out_bytes, chk)
        buf = np.empty(16, np.uint8)
        q.d2h(buf, chk, 16)
        q.sync()
        return buf.tobytes().hex()

    variants = [("records_each_launch", 0), ("records_precomputed", 1)]
    sums = {}
    for r in range(a.rounds):
        for name, opt in (variants if r % 2 == 0 else variants[::-1]):
            eng.option("desc_reuse_records", opt)
            for _ in range(6):  # every ring slot makes (and, with the option, keeps) its records
                step()
            q.sync()
            q.mark(0)
            for _ in range(a.steps):
                step()
            q.mark(1)
            q.sync()
            ms = q.elapsed_ms(0, 1) / a.steps
            sums.setdefault(name, checksum())
            print(json.dumps({"variant": name, "round": r, "kernel_ms": round(ms, 4),
                              "frac_hbm": round(nbytes / (ms * 1e-3) / 8e12, 4), "stripes": len(stripes),
                              "algorithmic_bytes": nbytes}), flush=True)
    eng.option("desc_reuse_records", 0)
    same = len(set(sums.values())) == 1
    print(json.dumps({"summary": True, "outputs_equal": same, "checksums": sums}), flush=True)
    q.close()
    eng.close()
    sys.exit(0 if same else 3)


if __name__ == "__main__":
    main()
