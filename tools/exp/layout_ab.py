#!/usr/bin/env python3
"""Where the parity lands in HBM (tools only): one mechanism the r01-r03
sweeps did not try.  The streaming kernel's gap to its read-only ceiling is
the write stream's turnaround; with the parity of stripe s written right
after its sources ([stripes][N+1][S], `interleaved`), the writes fall inside
the address window the reads are working through, instead of a second window
48 GiB away (`separate`: [stripes][N][S] + [stripes][S], bench.py's layout).
Same kernel (bcp_xor_strided_async, strided addressing), same inputs, both
layouts in one allocation each, interleaved rounds, HIP-event time per launch.

    python tools/exp/layout_ab.py --rounds 4
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--stripes", type=int, default=12500)
a = ap.parse_args()

N, C, S = 8, 512 * 1024, a.stripes
eng = bcp.Engine(0)
q = eng.queue()
sep_src = eng.alloc(S * N * C)
sep_dst = eng.alloc(S * C)
inter = eng.alloc(S * (N + 1) * C)
q.fill_synthetic(sep_src, S * N * C, seed=1)
# the same source bytes, stripe by stripe, into the interleaved layout
q.xor_strided(inter, (N + 1) * C, sep_src, N * C, C, S, 1, N * C)  # 1 "source" of N*C bytes = a copy
q.sync()
chk = eng.alloc(64)
bytes_per = S * (N + 1) * C


def launch(layout):
    if layout == "separate":
        q.xor_strided(sep_dst, C, sep_src, N * C, C, S, N, C)
    else:
        q.xor_strided(inter + N * C, (N + 1) * C, inter, (N + 1) * C, C, S, N, C)


def timed(layout):
    launch(layout)
    q.sync()
    q.mark(0)
    for _ in range(a.reps):
        launch(layout)
    q.mark(1)
    q.sync()
    return q.elapsed_ms(0, 1) / a.reps


res = {"separate": [], "interleaved": []}
for r in range(a.rounds):
    for layout in (("separate", "interleaved") if r % 2 == 0 else ("interleaved", "separate")):
        ms = timed(layout)
        res[layout].append(ms)
        print(json.dumps({"round": r, "layout": layout, "ms": round(ms, 4),
                          "pct_hbm": round(100 * bytes_per / (ms * 1e-3) / 8e12, 2)}), flush=True)
# the two outputs agree (fold of each layout's parity region)
q.xor_fold(sep_dst, S * C, chk)
q.sync()
import numpy as np  # noqa: E402
a16 = np.empty(16, np.uint8)
q.d2h(a16, chk, 16)
gathered = eng.alloc(S * C)
q.xor_strided(gathered, C, inter + N * C, (N + 1) * C, C, S, 1, C)
q.xor_fold(gathered, S * C, chk + 16)
b16 = np.empty(16, np.uint8)
q.d2h(b16, chk + 16, 16)
q.sync()
med = {k: float(np.median(v)) for k, v in res.items()}
print(json.dumps({"summary": True, "median_ms": med,
                  "pct_hbm": {k: round(100 * bytes_per / (v * 1e-3) / 8e12, 2) for k, v in med.items()},
                  "outputs_equal": bool(np.array_equal(a16, b16))}), flush=True)
