#!/usr/bin/env python3
"""Batched pipeline tuning sweep on config-5 stores (tools only): slab size,
io threads, slots; warm median per setting, same store, same process."""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
from e2e_bench import write_store, total_bytes  # noqa: E402

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3
ap = argparse.ArgumentParser()
ap.add_argument("--stripes", type=int, default=1000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--settings", default="256:8:3,256:16:3,256:16:4,128:16:4,512:16:3,64:16:6,256:32:4")
a = ap.parse_args()
root = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bcp_psweep")
shutil.rmtree(root, ignore_errors=True)
rng = np.random.default_rng(5)
files = []
for i in range(a.stripes):
    holders, p = S.random_layout(rng, 9, 8)
    lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
    files.append((f"u{i % 8}/{(i * 2654435761) % 65536:04X}/chunk{i}", holders, p, lens))
write_store(root, files, 2)
items = [(path, 1_700_000_000, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
rd, wr = total_bytes(root, files)
for st in a.settings.split(","):
    slab, io, slots = (int(x) for x in st.split(":"))
    pl = bcp.Pipeline(slab_bytes=slab * MiB, io_threads=io, nslots=slots)
    ts = []
    for r in range(1 + a.reps):
        t0 = time.perf_counter()
        pl.run(root, 9, items)
        ts.append(time.perf_counter() - t0)
    pl.close()
    w = float(np.median(ts[1:]))
    print(json.dumps({"slab_MiB": slab, "io_threads": io, "nslots": slots, "warm_s": round(w, 4),
                      "GiBps": round((rd + wr) / w / GiB, 2), "runs": [round(x, 4) for x in ts]}), flush=True)
shutil.rmtree(root, ignore_errors=True)
