#!/usr/bin/env python3
"""End to end at the BASELINE sizes of config 2 and config 3 (tools only).

A store of 12,500 stripes x 8 x 512 KiB chunk files (100,000 data chunks,
48.8 GiB; 9 storage targets, P rotating over the target left out) in memory
(/dev/shm); the batched pipeline generates every parity file (one cold run,
then --reps warm runs), then target --victim is lost (its chunk files
deleted) and rebuilt through the pipeline (the deletion outside the timing).
Sampled stripes are checked against the oracle, sampled rebuilt chunks
against the originals.  Rates: (chunk bytes read + bytes written) / wall
time; the host-to-device link's bound beside them (tools/box_probe.py).
One JSON line per measurement.
"""
import argparse
import concurrent.futures as cf
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402  (checker only)

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3
NT = 9


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/dev/shm/bcp_e2e_full")
    ap.add_argument("--stripes", type=int, default=12_500)
    ap.add_argument("--chunk", type=int, default=512 * KiB)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--victim", type=int, default=4)
    ap.add_argument("--sample", type=int, default=16)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import box_probe
    box = box_probe.cpu_info()
    box.update(box_probe.pcie_rates(bcp))
    emit(box=box)
    C = a.chunk
    shutil.rmtree(a.root, ignore_errors=True)
    S.make_store(a.root, NT)
    files = []
    for i in range(a.stripes):
        p = i % NT
        files.append((f"c2/{i % 128:02X}/chunk{i}", [t for t in range(NT) if t != p], p))
    block = np.random.default_rng(1).integers(0, 256, size=8 * MiB + 64 * KiB, dtype=np.uint8)

    def chunk_of(i, k):  # distinct bytes per chunk, from one random block
        off = ((i * 8 + k) * 4099) % (8 * MiB + 64 * KiB - C)
        return block[off:off + C]

    def write_stripe(i):
        path, holders, _ = files[i]
        for k, h in enumerate(holders):
            fn = S.chunk_path(a.root, h, path)
            os.makedirs(os.path.dirname(fn), exist_ok=True)
            with open(fn, "wb") as f:
                f.write(memoryview(chunk_of(i, k)))

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(a.threads) as ex:
        for n, _ in enumerate(ex.map(write_stripe, range(a.stripes))):
            if n % 2500 == 2499:
                emit(stage="writing store", stripes=n + 1, seconds=round(time.perf_counter() - t0, 1))
    ts = int(time.time()) + 3600
    items = [(path, ts, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p in files]
    emit(stage="store written", stripes=a.stripes, chunk_bytes=C, GiB=round(a.stripes * 8 * C / GiB, 2),
         seconds=round(time.perf_counter() - t0, 1))
    rng = np.random.default_rng(7)
    sample = sorted({0, a.stripes - 1} | {int(x) for x in rng.choice(a.stripes, size=a.sample, replace=False)})
    h2d = box["h2d_GBps"] * 1e9

    pl = bcp.Pipeline()
    try:
        # ---- config 2: parity gen over the whole store
        rd = a.stripes * 8 * C
        wr = a.stripes * (8 * 8 + C)
        times, timing = [], []
        for r in range(1 + a.reps):
            t0 = time.perf_counter()
            st = pl.run(a.root, NT, items)
            times.append(time.perf_counter() - t0)
            timing.append(pl.last_timing())
            if st.errors or st.tasks != a.stripes:
                sys.exit(f"gen run: errors {st.errors}, tasks {st.tasks}")
        bad = [files[i][0] for i in sample
               if S.read_file(S.parity_path(a.root, files[i][2], files[i][0]))
               != oracle.gen_parity_file([chunk_of(i, k) for k in range(8)])]
        w = float(np.median(times[1:])) if a.reps else times[0]
        emit(config=2, path="pipeline_gen(1 GPU, full size)", stripes=a.stripes, bytes_read=rd, bytes_written=wr,
             cold_seconds=round(times[0], 4), warm_seconds=round(w, 4), runs_s=[round(x, 4) for x in times],
             GiBps=round((rd + wr) / w / GiB, 2), h2d_bound_seconds=round(rd / h2d, 4),
             input_over_link=round(rd / w / h2d, 3), timing=timing[-1], verified=not bad, bad=bad[:3])
        # ---- config 3: lose target victim, rebuild it from 7 survivors + parity
        v = a.victim
        lost = [i for i in range(a.stripes) if v in files[i][1]]
        keep = {i: chunk_of(i, files[i][1].index(v)) for i in sample if v in files[i][1]}
        ordered = sorted(items, key=lambda x: x[0].encode())  # DB key order (rebuild/main.c:223-225)
        rd3 = len(lost) * (8 * C + 8 * 8)     # 7 survivors + parity body, + the header
        wr3 = len(lost) * C
        times, timing = [], []
        for r in range(1 + a.reps):
            with cf.ThreadPoolExecutor(a.threads) as ex:
                list(ex.map(lambda i: os.remove(S.chunk_path(a.root, v, files[i][0])), lost))
            t0 = time.perf_counter()
            st = pl.rebuild(a.root, NT, v, ordered)
            times.append(time.perf_counter() - t0)
            timing.append(pl.last_timing())
            if st.errors or st.tasks != len(lost):
                sys.exit(f"rebuild run: errors {st.errors}, tasks {st.tasks}")
        bad = [files[i][0] for i, want in keep.items()
               if S.read_file(S.chunk_path(a.root, v, files[i][0])) != want.tobytes()]
        w = float(np.median(times[1:])) if a.reps else times[0]
        emit(config=3, path=f"pipeline_rebuild(1 GPU, full size, target {v})", stripes=len(lost), bytes_read=rd3,
             bytes_written=wr3, cold_seconds=round(times[0], 4), warm_seconds=round(w, 4),
             runs_s=[round(x, 4) for x in times], GiBps=round((rd3 + wr3) / w / GiB, 2),
             h2d_bound_seconds=round(rd3 / h2d, 4), input_over_link=round(rd3 / w / h2d, 3), timing=timing[-1],
             verified=not bad and len(keep) > 0, bad=bad[:3], sampled=len(keep))
    finally:
        pl.close()
        shutil.rmtree(a.root, ignore_errors=True)


if __name__ == "__main__":
    main()
