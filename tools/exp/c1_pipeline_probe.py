#!/usr/bin/env python3
"""Config 1 (4 targets, 1,333 x 3 x 512 KiB, P rotating) through the batched
pipeline under several settings, interleaved, one process: where its time
goes against the per-task protocol's (r05: the driver's configs.config1 had
the pipeline at 0.75x the protocol with the reference's fold).

Each setting: --rounds interleaved warm runs after one cold run; per run the
wall time and bcp_pipeline_last_timing (stat, read_wait, slot_wait, submit,
drain, batches).  Settings: io threads per pool half (io_threads), slots,
slab size, the protocol (GPU fold), and `copies` (the same file reads and
parity writes from 16 C threads, nothing else) beside them; CPU seconds per
run.  One JSON line each.

  python tools/exp/c1_pipeline_probe.py --rounds 5
"""
import argparse
import concurrent.futures as cf
import json
import os
import resource
import shutil
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as BS  # noqa: E402

KiB, GiB = 1024, 1024 ** 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1333)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dir", default="/dev/shm")
    ap.add_argument("--settings", default="io8,io4,io6,io12,slots6,slab64,slab512,protocol")
    a = ap.parse_args()
    NT, C = 4, 512 * KiB
    root = os.path.join(a.dir, f"c1probe_{os.getpid()}")
    rng = np.random.default_rng(1)
    block = rng.integers(0, 256, size=8 << 20, dtype=np.uint8)
    files = [(f"u0/{i % 64:02X}/chunk{i}", [t for t in range(NT) if t != i % NT], i % NT) for i in range(a.files)]
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
        list(ex.map(write_file, range(a.files)))
    rd, wr = a.files * 3 * C, a.files * (24 + C)

    def reset():
        for k in range(NT):
            shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{k}", "parity"))

    settings = a.settings.split(",")
    floor = None
    if "copies" in settings:  # the kernel-copy floor of the same files (tools/exp/c1_cpu_cost.py)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import c1_cpu_cost
        floor = c1_cpu_cost.copy_floor_lib()
    pls = {}
    for s in settings:
        kw = {}
        if s.startswith("io"):
            kw["io_threads"] = int(s[2:])
        elif s.startswith("slots"):
            kw["nslots"] = int(s[5:])
        elif s.startswith("slab"):
            kw["slab_bytes"] = int(s[4:]) << 20
        if s not in ("protocol", "copies"):
            pls[s] = bcp.Pipeline(**kw)
    times = {s: [] for s in settings}
    timing = {s: [] for s in settings}
    cpu = {s: [] for s in settings}  # (CPU seconds, voluntary context switches) per run
    for r in range(1 + a.rounds):
        for s in settings[r % len(settings):] + settings[:r % len(settings)]:
            reset()
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            t0 = time.perf_counter()
            if s == "protocol":
                st = bcp.gen_run(root, NT, items, nlanes=12)
            elif s == "copies":
                assert floor.c1_copies(root.encode(), a.files, NT, C, 16) == 0
                st = None
            else:
                st = pls[s].run(root, NT, items)
            times[s].append(time.perf_counter() - t0)
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            cpu[s].append((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, ru1.ru_nvcsw - ru0.ru_nvcsw))
            assert st is None or st.errors == 0
            if s not in ("protocol", "copies"):
                timing[s].append(pls[s].last_timing())
    for s in settings:
        warm = times[s][1:]
        med = statistics.median(warm)
        out = {"setting": s, "warm_median_s": round(med, 4), "GiBps": round((rd + wr) / med / GiB, 2),
               "cpu_s": round(statistics.median(c[0] for c in cpu[s][1:]), 4),
               "vol_ctxsw": int(statistics.median(c[1] for c in cpu[s][1:])),
               "runs_s": [round(x, 4) for x in times[s]]}
        if timing[s]:
            keys = ("stat", "read_wait", "slot_wait", "submit", "drain")
            out["timing_median"] = {k: round(statistics.median(t[k] for t in timing[s][1:]), 4) for k in keys}
            out["batches"] = timing[s][-1]["batches"]
        print(json.dumps(out), flush=True)
    for p in pls.values():
        p.close()
    bcp.task_shutdown()
    shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
