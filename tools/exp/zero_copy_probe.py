#!/usr/bin/env python3
"""How fast can the GPU fold stripes that live in pinned HOST memory? (r05:
the per-task protocol's GPU fold reaches 62-80 % of config 1's link ceiling.)

The protocol's P role hands its window rows (pinned host memory, filled by
the senders' reads) to bcp_xor_stripes_async, whose kernel reads them across
PCIe in place and writes the parity into a pinned host block.  Here, over
the same shape (3 sources x 512 KiB per stripe, config 1):
  zero_copy   kernel reads host rows, writes host output (the protocol's fold)
  dma         hipMemcpyAsync rows H2D, kernel in HBM, output D2H, one queue
  ring        (r06) the resident fold ring (bcp_ring_*): each lane publishes
              its K stripes and waits for them, no launch and no stream sync
for K stripes per launch and Q queues launching concurrently (the lanes),
as GB/s of chunk bytes read (the link's H2D direction).  One JSON line per
(mode, K, Q).

  python tools/exp/zero_copy_probe.py
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

KiB = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,4,16")
    ap.add_argument("--qs", default="1,4,12")
    ap.add_argument("--total-stripes", type=int, default=768)
    ap.add_argument("--nsrc", type=int, default=3)
    ap.add_argument("--chunk-kib", type=int, default=512, help="bytes per row (the protocol's range folds: 128)")
    ap.add_argument("--modes", default="zero_copy,dma,ring")
    ap.add_argument("--ring-workers", default="64")
    ap.add_argument("--dirty", default="none",
                    help="comma list of row states before each fold: none (rows untouched since the first fill), "
                         "copy (each lane memcpy's its stripe's rows first, as the sources' read() does), "
                         "copy_elsewhere (the same copies into a scratch buffer: the rows stay clean), "
                         "copy_only (the copies alone, no fold: their own cost)")
    a = ap.parse_args()
    C, N = a.chunk_kib * KiB, a.nsrc
    T = a.total_stripes
    eng = bcp.Engine(0)
    rows = eng.host_alloc(T * N * C)
    outs = eng.host_alloc(T * C)
    qmax = max(int(x) for x in a.qs.split(","))
    kmax = max(int(x) for x in a.ks.split(","))
    dev_rows = [eng.alloc(kmax * N * C) for _ in range(qmax)]
    dev_out = [eng.alloc(kmax * C) for _ in range(qmax)]
    queues = [eng.queue() for _ in range(qmax)]
    import ctypes
    L = bcp.lib()
    # ring submissions prebuilt (ctypes argument building is not what is measured)
    ring_args = []
    for s in range(T):
        st = bcp.Stripe(outs + s * C, C, 0, N, 0)
        so = (bcp.Source * N)(*[bcp.Source(rows + (s * N + j) * C, C) for j in range(N)])
        ring_args.append((st, so))
    ring = None

    import numpy as np
    pool = np.random.default_rng(1).integers(0, 256, size=64 << 20, dtype=np.uint8)
    pool_addr = pool.ctypes.data
    dirty_state = {"mode": "none"}

    scratch = np.empty(qmax * N * C, dtype=np.uint8)

    def dirty(s0, k):
        if dirty_state["mode"] == "none":
            return
        for i in range(k):
            s_ = s0 + i
            src_ = pool_addr + (s_ * 7919 * 4096) % ((64 << 20) - N * C)
            if dirty_state["mode"] == "copy_elsewhere":  # the same copies, into a lane's scratch: rows stay clean
                lane = threading.get_ident() % qmax
                ctypes.memmove(scratch.ctypes.data + lane * N * C, src_, N * C)
            else:
                ctypes.memmove(rows + s_ * N * C, src_, N * C)

    def launch(q, qi, s0, k, mode):
        dirty(s0, k)
        if dirty_state["mode"] == "copy_only":
            return
        if mode == "ring":
            hs = []
            for i in range(k):
                st, so = ring_args[s0 + i]
                h = ctypes.c_uint64(0)
                bcp.check("bcp_ring_submit", L.bcp_ring_submit(ring.h, ctypes.byref(st), so, ctypes.byref(h)))
                hs.append(h.value)
            for h in hs:
                bcp.check("bcp_ring_wait", L.bcp_ring_wait(ring.h, h))
            return
        if mode == "zero_copy":
            q.xor_stripes([(outs + (s0 + i) * C, C, i * N, N, 0) for i in range(k)],
                          [(rows + ((s0 + i) * N + j) * C, C) for i in range(k) for j in range(N)])
        else:
            q.h2d(dev_rows[qi], rows + s0 * N * C, k * N * C)
            q.xor_stripes([(dev_out[qi] + i * C, C, i * N, N, 0) for i in range(k)],
                          [(dev_rows[qi] + (i * N + j) * C, C) for i in range(k) for j in range(N)])
            q.d2h(outs + s0 * C, dev_out[qi], k * C)

    def run(mode, k, nq):
        # each queue owns a contiguous range of stripes, k per launch, then one sync
        per_q = T // nq // k * k

        def worker(qi):
            q = queues[qi]
            base = qi * per_q
            for s0 in range(base, base + per_q, k):
                launch(q, qi, s0, k, mode)
                if mode != "ring" and dirty_state["mode"] != "copy_only":
                    q.sync()  # the protocol's P lane waits for every window

        ths = [threading.Thread(target=worker, args=(i,)) for i in range(nq)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
        return per_q * nq, dt

    for dm in a.dirty.split(","):
      dirty_state["mode"] = dm
      for mode in a.modes.split(","):
        for w in ([int(x) for x in a.ring_workers.split(",")] if mode == "ring" else [0]):
          if mode == "ring":
            if ring is not None:
                ring.close()
            ring = bcp.Ring(eng, workers=w)
          for k in (int(x) for x in a.ks.split(",")):
            for nq in (int(x) for x in a.qs.split(",")):
                run(mode, k, nq)  # warm
                res = [run(mode, k, nq) for _ in range(3)]
                st, dt = min(res, key=lambda x: x[1])
                print(json.dumps({"chunk_kib": a.chunk_kib, "dirty": dm, "mode": mode, "ring_workers": w, "stripes_per_launch": k, "queues": nq, "stripes": st,
                                  "best_s": round(dt, 4), "read_GBps": round(st * N * C / dt / 1e9, 2),
                                  "read_plus_write_GiBps": round(st * (N + 1) * C / dt / 2 ** 30, 2)}), flush=True)
    if ring is not None:
        ring.close()
    for q in queues:
        q.close()
    for p in dev_rows + dev_out:
        eng.free(p)
    eng.host_free(rows)
    eng.host_free(outs)
    eng.close()


if __name__ == "__main__":
    main()
