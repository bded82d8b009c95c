#!/usr/bin/env python3
"""Protocol cost breakdown (tools only): config-1 gen over the per-rank protocol
with (a) the GPU fold, (b) the reference CPU fold, (c) a fold that does
nothing (upper bound of the protocol itself), (d) lane counts.  Not verified
(the no-op fold writes no parity)."""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile
import argparse
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402
from e2e_bench import write_store, total_bytes  # noqa: E402

KiB, GiB = 1024, 1024 ** 3
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--lanes", default="12,24")
ap.add_argument("--folds", default="gpu_zero_copy,cpu_reference,noop")
a = ap.parse_args()
tmp = tempfile.mkdtemp(dir="/tmp")  # /dev/shm is noexec
src = os.path.join(tmp, "noop.c")
open(src, "w").write("#include <stddef.h>\n#include <stdint.h>\nint noop_fold(uint8_t *d, size_t n, const uint8_t *s,"
                     " size_t p, int k, void *c) { (void)d; (void)n; (void)s; (void)p; (void)k; (void)c; return 0; }\n")
so = os.path.join(tmp, "libnoop.so")
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src], check=True)
noop = ctypes.CDLL(so)
root = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bcp_noop")
shutil.rmtree(root, ignore_errors=True)
files = []
for i in range(1333):
    p = i % 4
    holders = [t for t in range(4) if t != p]
    files.append((f"u0/{i % 64:02X}/chunk{i}", holders, p, [512 * KiB] * 3))
write_store(root, files, 1)
items = [(path, 2 ** 40, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
rd, wr = total_bytes(root, files)


def timed(label, lanes, hook=None):
    if hook:
        bcp.set_xor_hook(hook)
    try:
        ts = []
        for r in range(a.reps):
            for p in range(4):
                shutil.rmtree(os.path.join(root, f"st{p}", "parity"), ignore_errors=True)
                os.makedirs(os.path.join(root, f"st{p}", "parity"))
            t0 = time.perf_counter()
            bcp.gen_run(root, 4, items, nlanes=lanes)
            ts.append(time.perf_counter() - t0)
    finally:
        bcp.set_xor_hook(None)
    w = float(np.median(ts[1:]))
    print(f'{{"fold": "{label}", "lanes": {lanes}, "warm_s": {w:.4f}, "GiBps": {(rd + wr) / w / GiB:.2f}}}', flush=True)


ol = oracle.lib()
hooks = {"gpu_zero_copy": None, "cpu_reference": ctypes.cast(ol.oracle_xor_rows, ctypes.c_void_p).value,
         "noop": ctypes.cast(noop.noop_fold, ctypes.c_void_p).value}
for lanes in (int(x) for x in a.lanes.split(",")):
    for f in a.folds.split(","):
        timed(f, lanes, hooks[f])
bcp.task_shutdown()
shutil.rmtree(root, ignore_errors=True)
