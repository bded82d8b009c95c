#!/usr/bin/env python3
"""Probe (tools/exp): batched-pipeline rate against job size on config-5
shapes -- warm runs over the first 100 / 300 / 1000 stripes of one store
(is a changelog round's small subset slow per byte, and why)."""
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "beegfs-chunk-parity_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
from e2e_bench import total_bytes, write_store  # noqa: E402

KiB, MiB, GiB = 1024, 1 << 20, 1 << 30
root = "/dev/shm/bcp_psizes"
shutil.rmtree(root, ignore_errors=True)
r5 = np.random.default_rng(5)
files = []
for i in range(1000):
    holders, p = S.random_layout(r5, 9, 8)
    lens = [int(x) for x in np.exp(r5.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
    files.append((f"u{i % 8}/{(i * 2654435761) % 65536:04X}/chunk{i}", holders, p, lens))
write_store(root, files, 2)
if len(sys.argv) > 1 and sys.argv[1] == "preread":  # read every chunk file once before the runs
    for dirpath, _, names in os.walk(root):
        for nm in names:
            with open(os.path.join(dirpath, nm), "rb") as f:
                while f.read(1 << 22):
                    pass
    print(json.dumps({"preread": True}), flush=True)
items = [(path, 1_700_000_000, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
pl = bcp.Pipeline(io_threads=16)
for n in (100, 300, 1000, 100):
    rd, wr = total_bytes(root, files[:n])
    ts = []
    for rep in range(4):
        t0 = time.perf_counter()
        st = pl.run(root, 9, items[:n])
        ts.append(time.perf_counter() - t0)
    w = float(np.median(ts[1:]))
    print(json.dumps(dict(stripes=n, GiB=round((rd + wr) / GiB, 3), warm_ms=round(w * 1e3, 2),
                          GiBps=round((rd + wr) / w / GiB, 2), runs_ms=[round(t * 1e3, 2) for t in ts],
                          errors=int(st.errors))), flush=True)
# the changelog round's situation: the same 100 stripes' chunks rewritten,
# then one run -- with and without reading the rewritten files first
for preread in (False, True, False, True):
    rng = np.random.default_rng(11)
    for path, holders, p, lens in files[:100]:
        for h, L in zip(holders, lens):
            S.write_chunk(root, h, path, rng.integers(0, 256, size=L, dtype=np.uint8))
    if preread:
        for path, holders, p, lens in files[:100]:
            for h in holders:
                with open(S.chunk_path(root, h, path), "rb") as f:
                    while f.read(1 << 22):
                        pass
    t0 = time.perf_counter()
    st = pl.run(root, 9, items[:100])
    t1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    pl.run(root, 9, items[:100])
    t2 = time.perf_counter() - t0
    print(json.dumps(dict(after_rewrite=True, preread=preread, first_ms=round(t1 * 1e3, 2),
                          second_ms=round(t2 * 1e3, 2), errors=int(st.errors))), flush=True)
pl.close()
shutil.rmtree(root, ignore_errors=True)
