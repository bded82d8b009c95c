#!/usr/bin/env python3
"""How fast does the device read P-role rows in place over PCIe, by host
memory kind (tools only)?  Registered with bcp_host_register: (a) a shared
anonymous mapping -- the rank pool's row arena, 4 KiB shmem pages on hosts
whose shmem_enabled is "never"; (b) private anonymous memory with
MADV_HUGEPAGE -- the threads' rows (bcp_host_alloc_mapped's registered
form).  One descriptor batch of S stripes x 8 rows x 1 MiB folded from host
rows into a device buffer, HIP-event time, median of reps, interleaved.

    python tools/exp/host_read_kinds.py > kinds.jsonl
"""
import ctypes
import json
import mmap
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

MiB = 1 << 20
N, L, S = 8, MiB, 32  # 256 MiB of rows
SIZE = N * L * S
libc = ctypes.CDLL(None)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE = 14

eng = bcp.Engine(0)
q = eng.queue()
out = eng.alloc(S * L)
kinds = {}
shared = mmap.mmap(-1, SIZE, flags=mmap.MAP_SHARED)
kinds["shared_anon"] = np.frombuffer(shared, dtype=np.uint8)
priv = mmap.mmap(-1, SIZE + 2 * MiB, flags=mmap.MAP_PRIVATE)
pa = np.frombuffer(priv, dtype=np.uint8)
off = (-pa.ctypes.data) % (2 * MiB)
libc.madvise(pa.ctypes.data + off, SIZE, MADV_HUGEPAGE)
kinds["private_thp"] = pa[off:off + SIZE]
for k, a in kinds.items():
    a[:] = 7  # touch every page before the registration pins it
    eng.host_register(a.ctypes.data, SIZE)
res = {k: [] for k in kinds}
for r in range(6):
    for k, a in kinds.items():
        base = a.ctypes.data
        stripes = [(out + s * L, L, s * N, N, 0) for s in range(S)]
        sources = [(base + (s * N + j) * L, L) for s in range(S) for j in range(N)]
        q.mark(0)
        q.xor_stripes(stripes, sources)
        q.mark(1)
        q.sync()
        ms = q.elapsed_ms(0, 1)
        if r:
            res[k].append(ms)
for k, a in kinds.items():
    eng.host_unregister(a.ctypes.data)
    m = statistics.median(res[k])
    print(json.dumps({"kind": k, "rows_bytes": SIZE, "median_ms": round(m, 3),
                      "GBps_read_over_pcie": round(SIZE / (m * 1e-3) / 1e9, 1)}), flush=True)
