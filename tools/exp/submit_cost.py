#!/usr/bin/env python3
"""Host-side cost of one descriptor-batch submission (bcp_xor_stripes_async)
at bench.py --mode mixed's shapes (config 5: 8-wide stripes, log-uniform
64 KiB-4 MiB, ~6,600 stripes): the call's wall time with the queue idle
(what the first timed launch of a block pays before its kernel can start)
and with a kernel in flight, plus the kernel's own event time.  One JSON
line per case.  VERDICT r05 next #4: the first timed launch's extra 1.7 ms.

  python tools/exp/submit_cost.py [--stripes 12500] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

KiB = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=12500, help="config-2 volume budget as bench.py computes it")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--uniform", action="store_true",
                    help="bench.py --mode rebuild's batch instead: --stripes x 8 x 512 KiB, one pointer table")
    a = ap.parse_args()
    N, C = 8, 512 * KiB
    rng = np.random.default_rng(3)
    budget = a.stripes * N * C
    lens_all, tot = [], 0
    if a.uniform:
        lens_all = [np.full(N, C, dtype=np.int64) for _ in range(a.stripes)]
    while tot < budget and not a.uniform:
        ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=N)).astype(np.int64)
        lens_all.append(ls)
        tot += int(ls.sum())
    align = lambda x: (x + 255) & ~255  # noqa: E731
    eng = bcp.Engine(0)
    q = eng.queue()
    src_bytes = sum(int(sum(align(int(x)) for x in ls)) for ls in lens_all)
    out_bytes = sum(align(int(ls.max())) for ls in lens_all)
    src, out = eng.alloc(src_bytes), eng.alloc(out_bytes)
    stripes, sources, so_off, do_off = [], [], 0, 0
    for ls in lens_all:
        first = len(sources)
        for x in ls:
            sources.append((src + so_off, int(x)))
            so_off += align(int(x))
        stripes.append((out + do_off, int(ls.max()), first, N, 0))
        do_off += align(int(ls.max()))
    st = (bcp.Stripe * len(stripes))(*[bcp.Stripe(*x) for x in stripes])
    so = (bcp.Source * len(sources))(*[bcp.Source(*x) for x in sources])
    L = bcp.lib()

    def submit():
        t0 = time.perf_counter()
        bcp.check("bcp_xor_stripes_async", L.bcp_xor_stripes_async(q.h, st, len(stripes), so, len(sources)))
        return time.perf_counter() - t0
    for _ in range(3):
        submit()
    q.sync()
    idle, busy, first_ev, next_ev = [], [], [], []
    for _ in range(a.reps):
        q.sync()
        q.mark(0)
        idle.append(submit())
        q.mark(1)
        busy.append(submit())
        q.mark(2)
        q.sync()
        first_ev.append(q.elapsed_ms(0, 1))
        next_ev.append(q.elapsed_ms(1, 2))
    print(json.dumps({"uniform": a.uniform, "stripes": len(stripes), "sources": len(sources),
                      "submit_ms_queue_idle": [round(x * 1e3, 3) for x in idle],
                      "submit_ms_kernel_in_flight": [round(x * 1e3, 3) for x in busy],
                      "event_ms_first_after_idle": [round(x, 3) for x in first_ev],
                      "event_ms_next": [round(x, 3) for x in next_ev],
                      "median_submit_idle_ms": round(statistics.median(idle) * 1e3, 3),
                      "median_first_minus_next_ms": round(statistics.median(first_ev) - statistics.median(next_ev), 3)}),
          flush=True)
    q.close()
    eng.free(src)
    eng.free(out)
    eng.close()


if __name__ == "__main__":
    main()
