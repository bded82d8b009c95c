#!/usr/bin/env python3
"""Probe (tools/exp): can host threads write chunk bytes straight into device
memory through the PCIe BAR, fast enough for the P role's window rows to live
in HBM?  Fine-grained device memory (hipExtMallocWithFlags(Finegrained)):
CPU memcpy into it, read() from a page-cached file into it, then the device
checks the bytes (XOR-fold on the GPU vs numpy).  Prints one JSON line per
measurement."""
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.read.restype = ctypes.c_ssize_t
libc.read.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
eng = bcp.Engine(0)
q = eng.queue()
N = 64 << 20
src = np.random.default_rng(1).integers(0, 256, size=N, dtype=np.uint8)
fd_path = os.path.join(tempfile.mkdtemp(dir="/dev/shm"), "chunk")
src.tofile(fd_path)


def emit(**kw):
    print(json.dumps(kw), flush=True)


def check(p, label):
    """the device's XOR-fold of the region vs numpy's"""
    out = eng.alloc(64)
    q.xor_fold(p, N, out)
    got = np.empty(16, np.uint8)
    q.d2h(got, out, 16)
    q.sync()
    ref = np.bitwise_xor.reduce(src.reshape(-1, 16), axis=0)
    eng.free(out)
    emit(check=label, device_sees_cpu_writes=bool(np.array_equal(got, ref)))


for flag_name, flag in (("finegrained", 0x1), ("uncached", 0x3)):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(N), ctypes.c_uint(flag))
    emit(alloc=flag_name, rc=rc)
    if rc != 0:
        continue
    dst = (ctypes.c_uint8 * N).from_address(p.value)
    for rep in range(3):
        t0 = time.perf_counter()
        ctypes.memmove(p.value, src.ctypes.data, N)
        dt = time.perf_counter() - t0
        emit(memory=flag_name, op="cpu_memcpy_into_vram", GBps=round(N / dt / 1e9, 2))
    check(p.value, f"{flag_name}_memcpy")
    for rep in range(3):
        fd = os.open(fd_path, os.O_RDONLY)
        t0 = time.perf_counter()
        got = 0
        while got < N:
            r = libc.read(fd, ctypes.c_void_p(p.value + got), N - got)
            if r <= 0:
                break
            got += r
        dt = time.perf_counter() - t0
        os.close(fd)
        emit(memory=flag_name, op="read_file_into_vram", bytes=got, GBps=round(got / dt / 1e9, 2))
    check(p.value, f"{flag_name}_read")
    t0 = time.perf_counter()
    back = np.empty(1 << 20, np.uint8)
    ctypes.memmove(back.ctypes.data, p.value, 1 << 20)
    dt = time.perf_counter() - t0
    emit(memory=flag_name, op="cpu_read_from_vram_1MiB", GBps=round((1 << 20) / dt / 1e9, 3))
    hip.hipFree(p)
# reference: the same copies into registered host memory
h = eng.host_alloc(N)
for rep in range(3):
    t0 = time.perf_counter()
    ctypes.memmove(h, src.ctypes.data, N)
    emit(memory="host_registered", op="cpu_memcpy", GBps=round(N / (time.perf_counter() - t0) / 1e9, 2))
os.remove(fd_path)
