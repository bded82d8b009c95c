#!/usr/bin/env python3
"""HBM rate by read:write mix, ours beside the vendor's kernels (tools only).

VERDICT r01 #5 asks the descriptor kernel for >= 85 % of 8 TB/s on config-5
shapes, which read ~3.3 bytes per byte written.  This probe measures, in ONE
process on ONE set of allocations, what the device gives at each mix:

  memset      hipMemsetAsync (the runtime's fill kernel)        0 : 1
  d2d         hipMemcpyAsync device->device (the runtime's blit) 1 : 1
  torch_xor2  torch.bitwise_xor(a, b, out=c), uint8             2 : 1
  torch_xor3  torch: c = a ^ b; c ^= d (two passes, 3 reads 2 writes)
  stream N    xor_stream over N uniform 512 KiB sources          N : 1
  fold        xor_fold (reads, 16-byte result)                   1 : 0

Input volume is held near --gib GiB for every row.  Rate = algorithmic bytes
(read + written) / HIP-event time of one launch, median over --reps; rounds
are interleaved so box drift hits every row alike.

    python tools/exp/mix_ceiling.py --rounds 3 > mix.jsonl
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=24.0, help="input bytes per launch")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--widths", default="1,2,3,4,6,8")
ap.add_argument("--no-torch", action="store_true")
a = ap.parse_args()

C = 512 * 1024
PEAK = 8.0e12
IN = int(a.gib * (1 << 30)) // C * C
torch = None
if not a.no_torch:
    import torch as _t  # initialised before the engine: torch's HIP init fails after ours
    torch = _t
    torch.cuda.init()
eng = bcp.Engine(0)
q = eng.queue()
src = eng.alloc(IN + (1 << 20))
out = eng.alloc(IN + (1 << 20))  # as large as the input: d2d / memset write it whole
red = eng.alloc(64)
q.fill_synthetic(src, IN, seed=7)
q.sync()

def timed(fn, nbytes):
    ms = []
    for _ in range(a.reps):
        q.mark(0)
        fn()
        q.mark(1)
        q.sync()
        ms.append(q.elapsed_ms(0, 1))
    m = statistics.median(ms)
    return m, nbytes / (m * 1e-3)


def torch_timed(fn, nbytes):
    ms = []
    for _ in range(a.reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    m = statistics.median(ms)
    return m, nbytes / (m * 1e-3)


rows = {}


def row(name, mix, fn, nbytes, use_torch=False):
    ms, bps = (torch_timed if use_torch else timed)(fn, nbytes)
    rows.setdefault(name, []).append(bps)
    print(json.dumps({"row": name, "read_per_write": mix, "ms": round(ms, 4), "bytes": nbytes,
                      "GBps": round(bps / 1e9, 1), "pct_hbm_peak": round(100 * bps / PEAK, 2)}), flush=True)


if torch is not None:
    h = IN // 3 // 4096 * 4096
    ta = torch.empty(h, dtype=torch.uint8, device="cuda")
    tb = torch.empty(h, dtype=torch.uint8, device="cuda")
    td = torch.empty(h, dtype=torch.uint8, device="cuda")
    tc = torch.empty(h, dtype=torch.uint8, device="cuda")
    for t in (ta, tb, td):
        t.random_(0, 256)
    torch.cuda.synchronize()

widths = [int(x) for x in a.widths.split(",") if x]
for r in range(a.rounds):
    row("memset", 0.0, lambda: q.memset(out, 0x5A, IN), IN)
    row("d2d", 1.0, lambda: q.d2d(out, src, IN), 2 * IN)
    for n in widths:
        stripes = IN // (n * C)
        row(f"stream_n{n}", float(n), lambda n=n, s=stripes: q.xor_uniform(out, src, s, n, C),
            stripes * (n + 1) * C)
    row("fold", None, lambda: q.xor_fold(src, IN, red), IN)
    if torch is not None:
        row("torch_xor2", 2.0, lambda: torch.bitwise_xor(ta, tb, out=tc), 3 * h, use_torch=True)

        def x3():
            torch.bitwise_xor(ta, tb, out=tc)
            tc.bitwise_xor_(td)
        row("torch_xor3", 1.5, x3, 5 * h, use_torch=True)

summary = {k: round(100 * statistics.median(v) / PEAK, 2) for k, v in rows.items()}
print(json.dumps({"summary_pct_hbm_peak_median": summary, "input_bytes": IN, "rounds": a.rounds,
                  "reps": a.reps}), flush=True)
