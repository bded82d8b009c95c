#!/usr/bin/env python3
"""Rank pools with the node fold server, created and destroyed again and
again (tools only): every round a new pool (new server, new arena) runs a gen
over fresh random stripes and a rebuild, parity checked against the oracle
on a sample; prints one JSON line per round.  Run in a process that never
touches the GPU (the pools' servers do).

    python tools/exp/fold_server_stress.py --rounds 12 > stress.jsonl
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "beegfs-chunk-parity_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--root", default="/dev/shm/bcp_fs_stress")
ap.add_argument("--targets", type=int, default=7)
a = ap.parse_args()
nt = a.targets
for r in range(a.rounds):
    root = os.path.join(a.root, f"r{r}")
    shutil.rmtree(root, ignore_errors=True)
    rng = np.random.default_rng(900 + r)
    files = []
    for i in range(60):
        holders, p = S.random_layout(rng, nt, int(rng.integers(1, nt)))
        files.append((f"s{i % 4}/c{i}", holders, p, [int(x) for x in rng.integers(0, 2_000_000, size=len(holders))]))
    if r % 3 == 0:
        files.append(("big/w", [0, 1], 2, [10 * 1024 * 1024 + 5, 14 * 1024 * 1024]))
    items, contents = S.populate(root, nt, files, seed=r)
    t0 = time.perf_counter()
    with bcp.RankPool(nt) as pool:
        g = pool.gen(root, items, nlanes=6)
        bad = [path for (path, h, p, lens) in files[::5]
               if S.read_file(S.parity_path(root, p, path)) != oracle.gen_parity_file(contents[path])]
        victim = r % nt
        lost = {}
        for (path, holders, p, lens) in files:
            if victim in holders:
                lost[path] = S.read_file(S.chunk_path(root, victim, path))
                os.remove(S.chunk_path(root, victim, path))
        b = pool.rebuild(root, victim, items)
        bad += [path for path, data in lost.items() if S.read_file(S.chunk_path(root, victim, path)) != data]
    dt = time.perf_counter() - t0
    shutil.rmtree(root, ignore_errors=True)
    print(json.dumps({"round": r, "gen_errors": g.errors, "rebuild_errors": b.errors, "bad": bad[:5],
                      "seconds": round(dt, 3)}), flush=True)
    if g.errors or b.errors or bad:
        sys.exit(1)
shutil.rmtree(a.root, ignore_errors=True)
print(json.dumps({"ok": True, "rounds": a.rounds}))
