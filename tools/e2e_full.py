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

--modes copy,direct: the pipeline's read paths (bcp_pipeline_opts.read_mode),
interleaved run by run; --contend 0,16: with N host threads memcpy'ing
64 MiB buffers meanwhile (host memory bandwidth taken, as by the other GPUs'
pipelines of one node), also interleaved.

--modes copy,direct --evict --root <a disk-backed directory>: every file of
the store is written back and dropped from the page cache (fsync +
POSIX_FADV_DONTNEED, untimed) before each timed run, so COPY reads from the
disk through the page cache and DIRECT with O_DIRECT into the slabs -- the
cold store a storage server sees, instead of the warm tmpfs of the default.
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
    ap.add_argument("--modes", default="copy")
    ap.add_argument("--contend", default="0")
    ap.add_argument("--evict", action="store_true")
    a = ap.parse_args()
    modes = {"copy": bcp.READ_COPY, "direct": bcp.READ_DIRECT}
    mode_list = a.modes.split(",")
    contend_list = [int(x) for x in a.contend.split(",")]
    import box_probe
    box = box_probe.cpu_info()
    box.update(box_probe.pcie_rates(bcp))
    os.makedirs(a.root, exist_ok=True)
    sf = os.statvfs(a.root)
    box["store_root"] = a.root
    box["store_free_GiB"] = round(sf.f_bavail * sf.f_frsize / GiB, 1)
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

    import ctypes
    import threading

    class Contention:
        """n threads copying 64 MiB buffers (ctypes.memmove drops the GIL)."""

        def __init__(self, n):
            self.n, self.stop, self.th = n, False, []
            self.bufs = [(np.ones(64 * MiB, np.uint8), np.zeros(64 * MiB, np.uint8)) for _ in range(n)]

        def run(self, i):
            a, b = self.bufs[i]
            while not self.stop:
                ctypes.memmove(b.ctypes.data, a.ctypes.data, a.nbytes)

        def __enter__(self):
            self.th = [threading.Thread(target=self.run, args=(i,)) for i in range(self.n)]
            for t in self.th:
                t.start()
            return self

        def __exit__(self, *exc):
            self.stop = True
            for t in self.th:
                t.join()

    def evict():
        """Every file under the store: written back and dropped from the page cache."""
        t0 = time.perf_counter()
        names = [os.path.join(d, f) for d, _, fs in os.walk(a.root) for f in fs]

        def drop(fn):
            fd = os.open(fn, os.O_RDONLY)
            try:
                os.fsync(fd)
                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            finally:
                os.close(fd)
        with cf.ThreadPoolExecutor(a.threads) as ex:
            list(ex.map(drop, names))
        return round(time.perf_counter() - t0, 2)

    pls = {m: bcp.Pipeline(read_mode=modes[m]) for m in mode_list}
    try:
        rd = a.stripes * 8 * C
        wr = a.stripes * (8 * 8 + C)
        v = a.victim
        lost = [i for i in range(a.stripes) if v in files[i][1]]
        keep = {i: chunk_of(i, files[i][1].index(v)) for i in sample if v in files[i][1]}
        ordered = sorted(items, key=lambda x: x[0].encode())  # DB key order (rebuild/main.c:223-225)
        rd3 = len(lost) * (8 * C + 8 * 8)     # 7 survivors + parity body, + the header
        wr3 = len(lost) * C
        res = {}
        for r in range(1 + a.reps):
            for nc in contend_list:
                for m in mode_list:
                    pl = pls[m]
                    ev = evict() if a.evict else None
                    with Contention(nc):
                        # ---- config 2: parity gen over the whole store
                        t0 = time.perf_counter()
                        st = pl.run(a.root, NT, items)
                        tg = time.perf_counter() - t0
                        tmg = pl.last_timing()
                        if st.errors or st.tasks != a.stripes:
                            sys.exit(f"gen run: errors {st.errors}, tasks {st.tasks}")
                    bad = [files[i][0] for i in sample
                           if S.read_file(S.parity_path(a.root, files[i][2], files[i][0]))
                           != oracle.gen_parity_file([chunk_of(i, k) for k in range(8)])]
                    # ---- config 3: lose target v, rebuild it (the deletion untimed)
                    with cf.ThreadPoolExecutor(a.threads) as ex:
                        list(ex.map(lambda i: os.remove(S.chunk_path(a.root, v, files[i][0])), lost))
                    ev3 = evict() if a.evict else None
                    with Contention(nc):
                        t0 = time.perf_counter()
                        st = pl.rebuild(a.root, NT, v, ordered)
                        tr = time.perf_counter() - t0
                        tmr = pl.last_timing()
                        if st.errors or st.tasks != len(lost):
                            sys.exit(f"rebuild run: errors {st.errors}, tasks {st.tasks}")
                    bad3 = [files[i][0] for i, want in keep.items()
                            if S.read_file(S.chunk_path(a.root, v, files[i][0])) != want.tobytes()]
                    key = (m, nc)
                    res.setdefault(key, {"gen": [], "rebuild": []})
                    res[key]["gen"].append(tg)
                    res[key]["rebuild"].append(tr)
                    emit(rep=r, mode=m, contend=nc, evict_s=[ev, ev3], gen_s=round(tg, 4), rebuild_s=round(tr, 4),
                         gen_GiBps=round((rd + wr) / tg / GiB, 2), rebuild_GiBps=round((rd3 + wr3) / tr / GiB, 2),
                         gen_input_over_link=round(rd / tg / h2d, 3), rebuild_input_over_link=round(rd3 / tr / h2d, 3),
                         gen_timing=tmg, rebuild_timing=tmr, verified=not bad and not bad3 and len(keep) > 0)
        for (m, nc), d in res.items():
            g = float(np.median(d["gen"][1:])) if a.reps else d["gen"][0]
            rb = float(np.median(d["rebuild"][1:])) if a.reps else d["rebuild"][0]
            emit(summary=True, mode=m, contend=nc, stripes=a.stripes, warm_gen_s=round(g, 4),
                 gen_GiBps=round((rd + wr) / g / GiB, 2), gen_input_over_link=round(rd / g / h2d, 3),
                 warm_rebuild_s=round(rb, 4), rebuild_GiBps=round((rd3 + wr3) / rb / GiB, 2),
                 rebuild_input_over_link=round(rd3 / rb / h2d, 3), cold_gen_s=round(d["gen"][0], 4))
    finally:
        for pl in pls.values():
            pl.close()
        shutil.rmtree(a.root, ignore_errors=True)


if __name__ == "__main__":
    main()
