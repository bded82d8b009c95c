#!/usr/bin/env python3
"""Probe (tools/exp): after bcp_dev_alloc_hostwrite memory is freed, do new
registered host buffers / device buffers behave?  Mimics the fold pool
switching row kinds: hostwrite rows used and freed, then host rows + a staged
H2D -> D2H round trip.  Prints addresses and whether each copy is exact."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402

eng = bcp.Engine(0)
q = eng.queue()
rng = np.random.default_rng(3)
MiB = 1 << 20


def emit(**kw):
    print(json.dumps(kw), flush=True)


def staged_roundtrip(h, n, label):
    d = eng.alloc(n)
    data = rng.integers(0, 256, size=n, dtype=np.uint8)
    ctypes.memmove(h, data.ctypes.data, n)
    q.h2d(d, h, n)
    back = np.empty(n, np.uint8)
    q.d2h(back, d, n)
    q.sync()
    bad = np.flatnonzero(back != data)
    emit(step=label, host=hex(h), dev=hex(d), exact=bool(bad.size == 0),
         first_bad=int(bad[0]) if bad.size else None, nbad=int(bad.size))
    eng.free(d)


for size in (1 * MiB, 2 * MiB, 4 * MiB, 16 * MiB):
    hw = eng.alloc_hostwrite(size)
    data = rng.integers(0, 256, size=size, dtype=np.uint8)
    ctypes.memmove(hw, data.ctypes.data, size)
    out = eng.alloc(64)
    q.xor_fold(hw, size, out)
    got = np.empty(16, np.uint8)
    q.d2h(got, out, 16)
    q.sync()
    eng.free(out)
    emit(step="hostwrite", size=size, addr=hex(hw),
         ok=bool(np.array_equal(got, np.bitwise_xor.reduce(data.reshape(-1, 16), axis=0))))
    eng.free(hw)
    h = eng.host_alloc(size, mapped=True)
    staged_roundtrip(h, size, f"after_free_{size}")
    # and a mapped zero-copy read of the new host rows by a kernel
    data = rng.integers(0, 256, size=size, dtype=np.uint8)
    ctypes.memmove(h, data.ctypes.data, size)
    out = eng.alloc(64)
    q.xor_fold(h, size, out)
    q.d2h(got, out, 16)
    q.sync()
    eng.free(out)
    emit(step="mapped_read", size=size, host=hex(h),
         ok=bool(np.array_equal(got, np.bitwise_xor.reduce(data.reshape(-1, 16), axis=0))))
    eng.host_free(h)
