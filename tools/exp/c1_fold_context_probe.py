#!/usr/bin/env python3
"""Config 1 gen through the per-task protocol (GPU fold), in contexts the
bench's configs.config1 leg creates: whether a live bcp_pipeline (its three
queues, pinned slabs, io threads) or a prior 55 GB device allocation in the
same process slows the protocol's GPU fold (r05: the bench leg measured the
GPU fold at 34-48 GiB/s, tools/proto_compare.py at 52 on another box).

Settings, interleaved in rotating order (one cold round, then --rounds):
  gpu_alone     bcp_gen_run, default (pipelined) GPU fold
  gpu_with_pl   the same while a bcp.Pipeline() is alive (created once)
  ref_fold      the reference's xor_parity as the P-role fold (oracle/_ref)
--big: allocate and free 55 GB of device memory first (as the bench's
device-resident timing does).  One JSON line per setting.
"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as BS  # noqa: E402
import oracle  # noqa: E402  (the reference fold, tools only)

KiB, GiB = 1024, 1024 ** 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--dir", default="/dev/shm")
    a = ap.parse_args()
    if a.big:
        eng = bcp.Engine(0)
        ptrs = [eng.alloc(S) for S in (48_828 << 20, 6_103 << 20)]
        for p in ptrs:
            eng.free(p)
        eng.close()
    NT, C, nfiles = 4, 512 * KiB, 1333
    root = os.path.join(a.dir, f"c1ctx_{os.getpid()}")
    rng = np.random.default_rng(1)
    block = rng.integers(0, 256, size=8 << 20, dtype=np.uint8)
    files = [(f"u0/{i % 64:02X}/chunk{i}", [t for t in range(NT) if t != i % NT], i % NT) for i in range(nfiles)]
    items = [(p, 2 ** 40, BS.with_p(sum(1 << h for h in hs), pp)) for p, hs, pp in files]
    BS.make_store(root, NT)

    def write_file(i):
        path, holders, _ = files[i]
        for k, h in enumerate(holders):
            fn = BS.chunk_path(root, h, path)
            os.makedirs(os.path.dirname(fn), exist_ok=True)
            off = ((i * 3 + k) * 40961) % ((8 << 20) - C)
            with open(fn, "wb") as f:
                f.write(memoryview(block[off:off + C]))
    with cf.ThreadPoolExecutor(8) as ex:
        list(ex.map(write_file, range(nfiles)))
    rd, wr = nfiles * 3 * C, nfiles * (24 + C)
    ref_fold, ref_name = oracle.cpu_fold_hook()

    def reset():
        for k in range(NT):
            shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{k}", "parity"))
    pl = None
    settings = ["gpu_alone", "gpu_with_pl", "ref_fold"]
    times = {s: [] for s in settings}
    for r in range(1 + a.rounds):
        for s in settings[r % 3:] + settings[:r % 3]:
            if s == "gpu_with_pl" and pl is None:
                pl = bcp.Pipeline()
            if s != "gpu_with_pl" and pl is not None:
                pl.close()
                pl = None
            reset()
            if s == "ref_fold":
                prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)
                bcp.set_xor_hook(ref_fold)
                prev_pad = bcp.set_explicit_padding(True)
            t0 = time.perf_counter()
            st = bcp.gen_run(root, NT, items, nlanes=12)
            times[s].append(time.perf_counter() - t0)
            if s == "ref_fold":
                bcp.set_explicit_padding(prev_pad)
                bcp.set_xor_hook(None)
                bcp.set_fold_mode(prev)
            assert st.errors == 0
    if pl is not None:
        pl.close()
    for s in settings:
        med = statistics.median(times[s][1:])
        print(json.dumps({"setting": s, "big_alloc_first": a.big, "warm_median_s": round(med, 4),
                          "GiBps": round((rd + wr) / med / GiB, 2), "runs_s": [round(x, 4) for x in times[s]]}),
              flush=True)
    bcp.task_shutdown()
    shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
