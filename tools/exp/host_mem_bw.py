#!/usr/bin/env python3
"""Host copy bandwidth into the memory kinds the protocol uses (tools only):
malloc'd (numpy), pinned (hipHostMalloc default) and mapped coherent pinned
(the P role's fold rows).  A file read into P's rows is this copy."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

N = 32 << 20
eng = bcp.Engine(0)
src = np.random.default_rng(1).integers(0, 256, size=N, dtype=np.uint8)
bufs = {"malloc": np.empty(N, dtype=np.uint8)}
for name, mapped in (("pinned", False), ("mapped_coherent", True)):
    p = eng.host_alloc(N, mapped=mapped)
    bufs[name] = np.ctypeslib.as_array((ctypes.c_uint8 * N).from_address(p))
# malloc'd, 2 MiB-aligned, madvise(MADV_HUGEPAGE), then hipHostRegister(Mapped)
libc = ctypes.CDLL("libc.so.6", use_errno=True)
hip = ctypes.CDLL("libamdhip64.so")
libc.posix_memalign.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_size_t]
for name, huge in (("registered_thp", True), ("registered_4k", False)):
    pp = ctypes.c_void_p()
    assert libc.posix_memalign(ctypes.byref(pp), 2 << 20, N) == 0
    if huge:
        libc.madvise(ctypes.c_void_p(pp.value), ctypes.c_size_t(N), 14)  # MADV_HUGEPAGE
    arr = np.ctypeslib.as_array((ctypes.c_uint8 * N).from_address(pp.value))
    arr[:] = 0  # fault the pages in
    rc = hip.hipHostRegister(ctypes.c_void_p(pp.value), ctypes.c_size_t(N), ctypes.c_uint(2))
    print(json.dumps({"memory": name, "hipHostRegister_rc": rc}), flush=True)
    bufs[name] = arr
for name, b in bufs.items():
    for direction in ("write_into", "read_from"):
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            if direction == "write_into":
                np.copyto(b, src)
            else:
                np.copyto(src, b)
            ts.append(time.perf_counter() - t0)
        ts.sort()
        print(json.dumps({"memory": name, "op": direction, "GBps": round(N / ts[len(ts) // 2] / 1e9, 2)}), flush=True)
