#!/usr/bin/env python3
"""What bounds the batched pipeline's copies (tools only): host<->device
rates over pinned memory on GPU 0, alone, together (both directions at once,
on two queues, as the pipeline runs them), and beside host threads that copy
memory (the pipeline's io threads read chunk files into the pinned slabs
while the DMA engine reads the previous slab).  One JSON line per case; rates
in GB/s of each direction's bytes over the case's wall time."""
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

GB = 1e9
MiB = 1 << 20
libc = ctypes.CDLL("libc.so.6")
libc.memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]


def main():
    n_up = 1024 * MiB
    eng = bcp.Engine(0)
    qh, qd = eng.queue(), eng.queue()
    h_up, h_dn = eng.host_alloc(n_up), eng.host_alloc(n_up)
    d_up, d_dn = eng.alloc(n_up), eng.alloc(n_up)

    def timed(fn, reps=5):
        ts = []
        for _ in range(reps):
            qh.sync()
            qd.sync()
            t0 = time.perf_counter()
            fn()
            qh.sync()
            qd.sync()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    def emit(**kw):
        print(json.dumps(kw), flush=True)

    t = timed(lambda: qh.h2d(d_up, h_up, n_up))
    emit(case="h2d alone", h2d_GBps=round(n_up / t / GB, 1))
    t = timed(lambda: qd.d2h(h_dn, d_dn, n_up))
    emit(case="d2h alone", d2h_GBps=round(n_up / t / GB, 1))
    for frac in (0.36, 1.0):  # config 5's parity : input bytes, and equal volumes
        n_dn = int(n_up * frac) // 4096 * 4096
        t = timed(lambda: (qh.h2d(d_up, h_up, n_up), qd.d2h(h_dn, d_dn, n_dn)))
        emit(case=f"h2d {n_up >> 20} MiB + d2h {n_dn >> 20} MiB at once", seconds=round(t, 5),
             h2d_only_would_take=round(n_up / 57.3e9, 5), total_GBps=round((n_up + n_dn) / t / GB, 1))
    for piece in (16, 64, 256):
        p = piece * MiB

        def pieces():
            for off in range(0, n_up, p):
                qh.h2d(d_up + off, h_up + off, p)
        t = timed(pieces)
        emit(case=f"h2d in {piece} MiB copies back to back", h2d_GBps=round(n_up / t / GB, 1))
    # host memory traffic beside the DMA: k threads memcpy 256 MiB blocks
    # between two private buffers (what the io threads do: page cache -> slab)
    src = [np.empty(256 * MiB, dtype=np.uint8) for _ in range(16)]
    dst = [np.empty(256 * MiB, dtype=np.uint8) for _ in range(16)]
    for a in src + dst:
        a.fill(1)
    for k in (4, 8, 16):
        stop = threading.Event()
        moved = [0] * k

        def worker(i):
            while not stop.is_set():
                libc.memcpy(dst[i].ctypes.data, src[i].ctypes.data, 256 * MiB)
                moved[i] += 256 * MiB

        ths = [threading.Thread(target=worker, args=(i,)) for i in range(k)]
        for th in ths:
            th.start()
        time.sleep(0.2)
        m0 = sum(moved)
        t0 = time.perf_counter()
        t = timed(lambda: qh.h2d(d_up, h_up, n_up), reps=7)
        dt = time.perf_counter() - t0
        cpu = (sum(moved) - m0) / dt
        stop.set()
        for th in ths:
            th.join()
        emit(case=f"h2d beside {k} memcpy threads", h2d_GBps=round(n_up / t / GB, 1),
             memcpy_GBps=round(cpu / GB, 1))
    qh.sync()
    qd.sync()
    for p in (d_up, d_dn):
        eng.free(p)
    for p in (h_up, h_dn):
        eng.host_free(p)
    qh.close()
    qd.close()
    eng.close()


if __name__ == "__main__":
    main()
