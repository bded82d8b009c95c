#!/usr/bin/env python3
"""Probe (tools/exp), second half of host_to_vram.py: would P-role window rows
in device memory pay?  (1) the fold kernel's rate reading fine-grained /
uncached device memory vs ordinary (coarse-grained) HBM and vs mapped host
rows; (2) aggregate CPU write rate into each memory kind from 1..12 threads
(memcpy and read() from a page-cached file, the two ways chunk bytes reach a
row).  One JSON line per measurement."""
import ctypes
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.read.restype = ctypes.c_ssize_t
libc.read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
libc.pread.restype = ctypes.c_ssize_t
libc.pread.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_long]
eng = bcp.Engine(0)
q = eng.queue()
MiB = 1 << 20
NSRC, SLICE = 8, 64 * MiB
REGION = 12 * SLICE


def emit(**kw):
    print(json.dumps(kw), flush=True)


def ext_alloc(n, flag):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(n), ctypes.c_uint(flag))
    if rc:
        raise RuntimeError(f"hipExtMallocWithFlags({flag}) rc {rc}")
    return p.value


kinds = {
    "coarse": (eng.alloc(REGION), eng.free),
    "finegrained": (ext_alloc(REGION, 0x1), lambda p: hip.hipFree(ctypes.c_void_p(p))),
    "uncached": (ext_alloc(REGION, 0x3), lambda p: hip.hipFree(ctypes.c_void_p(p))),
    "host_mapped": (eng.host_alloc(REGION, mapped=True), eng.host_free),
}
out_dev = eng.alloc(SLICE)
out_host = eng.host_alloc(SLICE, mapped=True)

# (1) fold kernel: 8 sources of 64 MiB -> 1 output, stream kernel (pitched rows)
for name, (base, _) in kinds.items():
    q.memset(base, 0x11, NSRC * SLICE) if name != "host_mapped" else ctypes.memset(base, 0x11, NSRC * SLICE)
    for oname, out in (("out_hbm", out_dev), ("out_host", out_host)):
        ts = []
        for rep in range(6):
            q.mark(0)
            q.xor_uniform(out, base, 1, NSRC, SLICE)
            q.mark(1)
            ts.append(q.elapsed_ms(0, 1))
        t = float(np.median(ts[1:])) * 1e-3
        emit(kernel="xor_uniform", rows=name, out=oname, sources=NSRC, slice_MiB=SLICE // MiB,
             GBps=round((NSRC + 1) * SLICE / t / 1e9, 1), ms=round(t * 1e3, 3))

# (2) CPU writes, T threads, each its own 64 MiB slice
src = np.random.default_rng(1).integers(0, 256, size=SLICE, dtype=np.uint8)
tmpd = tempfile.mkdtemp(dir="/dev/shm")
fpath = os.path.join(tmpd, "chunk")
src.tofile(fpath)


def run_threads(T, fn):
    bar = threading.Barrier(T + 1)
    done = []

    def body(i):
        bar.wait()
        fn(i)
        done.append(time.perf_counter())
    th = [threading.Thread(target=body, args=(i,)) for i in range(T)]
    for t in th:
        t.start()
    bar.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    return max(done) - t0


for name, (base, _) in kinds.items():
    if name == "coarse":
        continue  # not CPU-addressable
    for T in (1, 4, 12):
        for op in ("memcpy", "read"):
            def fn(i, base=base, op=op):
                dst = base + i * SLICE
                if op == "memcpy":
                    ctypes.memmove(dst, src.ctypes.data, SLICE)
                else:
                    fd = os.open(fpath, os.O_RDONLY)
                    got = 0
                    while got < SLICE:
                        r = libc.pread(fd, ctypes.c_void_p(dst + got), SLICE - got, got)
                        if r <= 0:
                            break
                        got += r
                    os.close(fd)
            ts = [run_threads(T, fn) for _ in range(3)]
            t = min(ts)
            emit(cpu_write=op, rows=name, threads=T, GBps=round(T * SLICE / t / 1e9, 2))
    # the device sees the last writes (every slice = src)
    chk = eng.alloc(64)
    q.xor_fold(base, 2 * SLICE, chk)
    got = np.empty(16, np.uint8)
    q.d2h(got, chk, 16)
    q.sync()
    eng.free(chk)
    emit(check=name, device_sees_cpu_writes=bool(np.array_equal(got, np.zeros(16, np.uint8))))
os.remove(fpath)
os.rmdir(tmpd)
for name, (base, free) in kinds.items():
    free(base)
