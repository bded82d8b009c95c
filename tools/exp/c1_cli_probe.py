#!/usr/bin/env python3
"""Config 1 through the CLI (`bin/bcp parity-gen --complete --force`), the
whole beegfs-parity-gen flow in one process per run: where the wall time
goes besides the engine run (the CLI's own `timings:` line -- init, phase 1
scan, engine setup, round, total), for the pipeline and the protocol
engines, interleaved.  One JSON line per engine with the per-run timings.

  python tools/exp/c1_cli_probe.py --runs 4
"""
import argparse
import concurrent.futures as cf
import json
import os
import re
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_store as BS  # noqa: E402

KiB = 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1333)
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--dir", default="/dev/shm")
    ap.add_argument("--engines", default="pipeline,protocol")
    ap.add_argument("--tools", default="", help="CLI builds to alternate (comma separated paths to bin/bcp; "
                                                   "default: the in-tree one)")
    a = ap.parse_args()
    NT, C = 4, 512 * KiB
    root = os.path.join(a.dir, f"c1cli_{os.getpid()}")
    rng = np.random.default_rng(1)
    block = rng.integers(0, 256, size=8 << 20, dtype=np.uint8)
    BS.make_store(root, NT)

    def write_file(i):
        for k, h in enumerate(t for t in range(NT) if t != i % NT):
            fn = BS.chunk_path(root, h, f"u0/{i % 64:02X}/chunk{i}")
            os.makedirs(os.path.dirname(fn), exist_ok=True)
            off = ((i * 3 + k) * 40961) % ((8 << 20) - C)
            with open(fn, "wb") as f:
                f.write(memoryview(block[off:off + C]))
    with cf.ThreadPoolExecutor(8) as ex:
        list(ex.map(write_file, range(a.files)))
    tools = [os.path.abspath(t) for t in a.tools.split(",") if t] or \
        [os.path.join(ROOT, "beegfs-chunk-parity_amd", "bin", "bcp")]
    keys = [(t, e) for t in tools for e in a.engines.split(",")]
    res = {k: [] for k in keys}
    for r in range(a.runs):
        for tool, e in keys[r % len(keys):] + keys[:r % len(keys)]:
            t0 = time.perf_counter()
            p = subprocess.run([tool, "parity-gen", "--complete", "--force", f"--{e}", root, str(NT)],
                               capture_output=True, text=True)
            wall = time.perf_counter() - t0
            line = next((ln for ln in p.stdout.splitlines() if ln.startswith("timings:")), "")
            stages = {k: float(v) for k, v in re.findall(r"([a-z0-9 ()]+?) ([0-9.]+) s", line.replace("timings: ", ""))}
            res[(tool, e)].append({"rc": p.returncode, "wall_s": round(wall, 4),
                           "stages": {k.strip(" ,()"): v for k, v in stages.items()},
                           "err": p.stderr[-300:] if p.returncode else None})
    import statistics
    for (tool, e), runs in res.items():
        warm = runs[1:] or runs
        print(json.dumps({"tool": os.path.relpath(tool, ROOT), "engine": e,
                          "wall_median_s": round(statistics.median(x["wall_s"] for x in warm), 4),
                          "setup_median_s": round(statistics.median(x["stages"].get("engine setup", 0) for x in warm), 4),
                          "total_median_s": round(statistics.median(x["stages"].get("total", 0) for x in warm), 4),
                          "runs": runs}), flush=True)
    shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
