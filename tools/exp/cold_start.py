#!/usr/bin/env python3
"""Probe (tools/exp): what a fresh process pays before its first fold --
engine creation (HIP init), queue creation, registered host rows -- the
cold start of every bin/bcp run.  One JSON line per step."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


t = time.perf_counter()
eng = bcp.Engine(0)
emit(step="engine_create", ms=round((time.perf_counter() - t) * 1e3, 2))
for n in (1, 8, 48):
    t = time.perf_counter()
    qs = [eng.queue() for _ in range(n)]
    dt = time.perf_counter() - t
    emit(step="queue_create", n=n, ms_each=round(dt / n * 1e3, 3))
    t = time.perf_counter()
    for q in qs:
        q.sync()
    emit(step="queue_first_sync", n=n, ms_each=round((time.perf_counter() - t) / n * 1e3, 3))
    for q in qs:
        q.close()
for mib in (1, 2, 4, 8):
    t = time.perf_counter()
    hs = [eng.host_alloc(mib << 20, mapped=True) for _ in range(8)]
    emit(step="host_alloc_registered", MiB=mib, ms_each=round((time.perf_counter() - t) / 8 * 1e3, 3))
    for h in hs:
        eng.host_free(h)
eng.close()
