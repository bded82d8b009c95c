#!/usr/bin/env python3
"""End-to-end measurements (chunk files in host storage -> parity files).

config 1 (BASELINE.json configs[0] shape): 4 storage targets as loopback
  ranks, 3-wide stripes with P rotating over the target left out, 1333 files
  -> ~1000 x 512 KiB chunk files per target.  Timed three ways over the same
  files: the per-rank protocol with the GPU fold (bcp_gen_run), the same
  protocol with the reference's own CPU fold as the P role's fold hook (the
  reference's xor_parity compiled unchanged, oracle/_ref ref_xor_rows, where
  built; else the oracle's restatement, oracle_xor_rows -- the line names
  which) in two forms -- folded like the reference's P role (the whole
  window once every row has arrived, senders on the reference's zero-padded
  wire: "reference fold in libbcp's protocol", protocol_cpu_fold_reference)
  and the restated fold inside this protocol's pipelined P role (source
  threads fold ranges as rows fill: protocol_cpu_fold_pipelined) -- and the
  batched pipeline (bcp_pipeline_gen).  Neither CPU line is the reference
  PROGRAM (its roles need MPI): the protocol around the fold is libbcp's.
  Then target 2 is lost and rebuilt through bcp_rebuild_run.
config 5: 9 targets, 8-wide stripes, chunk sizes log-uniform in
  [64 KiB, 4 MiB] (not 16-byte rounded); full parity gen (pipeline), then a
  seeded 10 % of stripes is rewritten, their chunk events are emitted as the
  binary record streams of bp-find-all-chunks (one per target), and one
  changelog round (bcp_gen_round_pipeline) parses them, plans them against
  the persistent state (per-target DB replicas), recomputes only that subset
  through the pipeline (pinned H2D/D2H on side queues) and updates the DB.

Rates are (sum of chunk bytes read + parity bytes written) / wall time.  The
stores are freshly written, so reads come from the page cache: these are
host-memory + PCIe rates, not disk rates.  Prints one JSON line per
measurement.
"""
import argparse
import ctypes
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402  (checker + CPU fold for the reference path)

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3
CPU_REF, CPU_PIPE = "protocol_cpu_fold_reference", "protocol_cpu_fold_pipelined"


def fold_ctx(mode, hook, ref_wire):
    """Set a P-role fold (mode None: the default; ref_wire: the senders pad
    every window as the reference's do, task_processing.c:302-303); returns
    the restore callable."""
    prev = bcp.set_fold_mode(mode) if mode is not None else None
    bcp.set_xor_hook(hook)
    prev_pad = bcp.set_explicit_padding(True) if ref_wire else None

    def restore():
        if prev_pad is not None:
            bcp.set_explicit_padding(prev_pad)
        bcp.set_xor_hook(None)
        if prev is not None:
            bcp.set_fold_mode(prev)
    return restore


def emit(**kw):
    print(json.dumps(kw), flush=True)


def total_bytes(root, files):
    rd = sum(sum(lens) for _, _, _, lens in files)
    wr = sum(8 * len(lens) + max(lens) for _, _, _, lens in files)
    return rd, wr


def verify(root, files, contents, sample, rng):
    idx = rng.choice(len(files), size=min(sample, len(files)), replace=False)
    for i in idx:
        path, holders, p, lens = files[i]
        got = S.read_file(S.parity_path(root, p, path))
        if got != oracle.gen_parity_file(contents[path]):
            return False, path
    return True, None


def write_store(root, files, seed):
    """Chunk contents from a fast generator (one random block, rotated per chunk)."""
    S.make_store(root, max(max(h) for _, h, _, _ in files) + 1 if files else 1)
    rng = np.random.default_rng(seed)
    block = rng.integers(0, 256, size=8 * MiB + 4096, dtype=np.uint8)
    contents = {}
    for i, (path, holders, p, lens) in enumerate(files):
        arrs = []
        for h, L in zip(holders, lens):
            off = int(rng.integers(0, 4096))
            data = block[off:off + L] if L <= 8 * MiB else rng.integers(0, 256, size=L, dtype=np.uint8)
            S.write_chunk(root, h, path, data)
            arrs.append(data)
        contents[path] = arrs
    return contents


def config1(a):
    root = os.path.join(a.root, "c1")
    shutil.rmtree(root, ignore_errors=True)
    files = []
    for i in range(a.c1_files):
        p = i % 4
        holders = [t for t in range(4) if t != p]
        files.append((f"u0/{i % 64:02X}/chunk{i}", holders, p, [512 * KiB] * 3))
    t = time.time()
    contents = write_store(root, files, 1)
    emit(stage="config1_store_written", files=len(files), seconds=round(time.time() - t, 2))
    items = [(path, 2 ** 40, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
    rd, wr = total_bytes(root, files)
    rng = np.random.default_rng(0)

    def reset_parity():
        for p in range(4):
            shutil.rmtree(os.path.join(root, f"st{p}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{p}", "parity"))

    def run(label, fn, extra=None):
        """first (cold: pinning, queues) run, then a.reps warm runs; median reported;
        extra() adds fields (the pipeline's stage timing of its last run)."""
        times = []
        for r in range(1 + a.reps):
            reset_parity()
            t0 = time.perf_counter()
            st = fn()
            times.append(time.perf_counter() - t0)
        ok, bad = verify(root, files, contents, a.verify, rng)
        warm = float(np.median(times[1:])) if a.reps else times[0]
        emit(config=1, path=label, cold_seconds=round(times[0], 3), warm_seconds=round(warm, 3),
             GiBps=round((rd + wr) / warm / GiB, 3), cold_GiBps=round((rd + wr) / times[0] / GiB, 3),
             bytes_read=rd, bytes_written=wr, tasks=int(st.tasks), errors=int(st.errors), verified=ok, bad=bad,
             **(extra() if extra else {}))
        return ok

    # the per-task protocol with three folds, interleaved in rotating order
    # (one cold round, then a.reps warm ones) so host drift lands on all
    ref_fold, ref_name = oracle.cpu_fold_hook()
    pipe_fold = ctypes.cast(oracle.lib().oracle_xor_rows, ctypes.c_void_p).value  # takes ranges (any pitch)
    variants = [("protocol_gpu_fold(bcp_gen_run,12 lanes)", None, None, False),
                ("protocol_gpu_fold_batched(12 lanes)", bcp.FOLD_BATCHED, None, False),
                (CPU_REF + f"({ref_name},reference wire,12 lanes)", bcp.FOLD_BATCHED, ref_fold, True),
                (CPU_PIPE + "(oracle_xor_rows,12 lanes)", None, pipe_fold, False)]
    times = {v[0]: [] for v in variants}
    ok = True
    preps = max(a.reps, 7)  # ~0.1 s runs: more rounds than the other measurements
    nv = len(variants)
    for r in range(1 + preps):
        for label, mode, hook, ref_wire in variants[r % nv:] + variants[:r % nv]:
            reset_parity()
            restore = fold_ctx(mode, hook, ref_wire)
            try:
                t0 = time.perf_counter()
                st = bcp.gen_run(root, 4, items, nlanes=12)
                times[label].append(time.perf_counter() - t0)
            finally:
                restore()
            if r == preps:
                okv, badv = verify(root, files, contents, a.verify, rng)
                ok &= okv
                warm = float(np.median(times[label][1:]))
                emit(config=1, path=label, cold_seconds=round(times[label][0], 3), warm_seconds=round(warm, 3),
                     GiBps=round((rd + wr) / warm / GiB, 3), runs_s=[round(x, 4) for x in times[label]],
                     bytes_read=rd, bytes_written=wr, tasks=int(st.tasks), errors=int(st.errors), verified=okv,
                     bad=badv, order="interleaved")
    pl = bcp.Pipeline(io_threads=a.io_threads, ndevices=a.ndevices)
    ok &= run(f"pipeline(bcp_pipeline_run,{a.ndevices} GPU)", lambda: pl.run(root, 4, items),
              lambda: {"last_run_timing": pl.last_timing()})
    pl.close()
    # the whole beegfs-parity-gen --complete flow through the CLI: scan every
    # target, plan (P per select_P), run, fill the DB replicas (warm median)
    tool = os.path.join(ROOT, "beegfs-chunk-parity_amd", "bin", "bcp")
    no_server = dict(os.environ, BCP_FOLD_SERVER="0")
    for label, extra, env in (("cli_parity_gen_complete(protocol)", ["--protocol"], None),
                              ("cli_parity_gen_complete(protocol, --fold batched)", ["--protocol", "--fold", "batched"],
                               None),
                              ("cli_parity_gen_complete(pipeline, the default engine)", [], None),
                              ("cli_parity_gen_complete(procs, node fold server)", ["--procs"], None),
                              ("cli_parity_gen_complete(procs, HIP context per rank)", ["--procs"], no_server)):
        times = []
        for r in range(1 + a.reps):
            t0 = time.perf_counter()
            res = subprocess.run([tool, "parity-gen", "--complete", "--force"] + extra + [root, "4"],
                                 capture_output=True, text=True, env=env)
            times.append(time.perf_counter() - t0)
            if res.returncode != 0:
                emit(config=1, path=label, error=res.stderr[-500:])
                break
        else:
            w = float(np.median(times[1:])) if a.reps else times[0]
            stages = next((ln for ln in res.stdout.splitlines() if ln.startswith("timings:")), "")
            emit(config=1, path=label, cold_seconds=round(times[0], 3), warm_seconds=round(w, 3),
                 GiBps=round((rd + wr) / w / GiB, 3), note="process wall time: start-up, scan, planning, DB updates",
                 last_run_stages=stages)
    # rebuild target 2 through the protocol
    lost = {}
    for path, holders, p, _ in files:
        if 2 in holders:
            lost[path] = S.chunk_path(root, 2, path)
            os.remove(lost[path])
    rb_bytes = len(lost) * 3 * (512 * KiB) + len(lost) * 512 * KiB

    def drop_lost():
        for fn in lost.values():
            if os.path.exists(fn):
                os.remove(fn)

    def rebuilt_ok():
        good = 0
        for k, (path, fn) in enumerate(lost.items()):
            if k % max(1, len(lost) // a.verify) == 0:
                holders = next(h for pth, h, _, _ in files if pth == path)
                good += S.read_file(fn) == contents[path][holders.index(2)].tobytes()
        return good, good == len(range(0, len(lost), max(1, len(lost) // a.verify)))

    # single lane, as rebuild/main.c, and 12 rebuild lanes (bcp_task_set_rebuild_lanes); the folds
    # interleaved in rotating order
    rvariants = [("rebuild_protocol_gpu_fold(bcp_rebuild_run)", None, None, False, 1),
                 ("rebuild_" + CPU_REF + f"({ref_name})", bcp.FOLD_BATCHED, ref_fold, True, 1),
                 ("rebuild_" + CPU_PIPE + "(oracle_xor_rows)", None, pipe_fold, False, 1),
                 ("rebuild_protocol_gpu_fold(bcp_rebuild_run,12 lanes)", None, None, False, 12),
                 ("rebuild_" + CPU_REF + f"({ref_name},12 lanes)", bcp.FOLD_BATCHED, ref_fold, True, 12)]
    rtimes = {v[0]: [] for v in rvariants}
    nv = len(rvariants)
    for r in range(1 + preps):
        for label, mode, hook, ref_wire, lanes in rvariants[r % nv:] + rvariants[:r % nv]:
            drop_lost()
            restore = fold_ctx(mode, hook, ref_wire)
            prev_lanes = bcp.set_rebuild_lanes(lanes)
            try:
                t0 = time.perf_counter()
                st = bcp.rebuild_run(root, 4, 2, items)
                rtimes[label].append(time.perf_counter() - t0)
            finally:
                bcp.set_rebuild_lanes(prev_lanes)
                restore()
            if r == preps:
                good, okv = rebuilt_ok()
                ok &= okv
                dt = float(np.median(rtimes[label][1:]))
                emit(config=1, path=label, cold_seconds=round(rtimes[label][0], 3), warm_seconds=round(dt, 3),
                     GiBps=round(rb_bytes / dt / GiB, 3), runs_s=[round(x, 4) for x in rtimes[label]],
                     rebuilt=len(lost), errors=int(st.errors), sampled_ok=good, order="interleaved")
    # the same rebuild through the batched pipeline (warm median of a.reps)
    pl = bcp.Pipeline(io_threads=a.io_threads, ndevices=a.ndevices)
    ordered = sorted(items, key=lambda x: x[0].encode())
    times = []
    for r in range(1 + a.reps):
        for fn in lost.values():
            if os.path.exists(fn):
                os.remove(fn)
        t0 = time.perf_counter()
        st = pl.rebuild(root, 4, 2, ordered)
        times.append(time.perf_counter() - t0)
    pl.close()
    dt = float(np.median(times[1:])) if a.reps else times[0]
    good = 0
    for k, (path, fn) in enumerate(lost.items()):
        if k % max(1, len(lost) // a.verify) == 0:
            holders = next(h for pth, h, _, _ in files if pth == path)
            good += S.read_file(fn) == contents[path][holders.index(2)].tobytes()
    emit(config=1, path=f"rebuild_pipeline({a.ndevices} GPU)", cold_seconds=round(times[0], 3), warm_seconds=round(dt, 3),
         GiBps=round(rb_bytes / dt / GiB, 3), rebuilt=len(lost), errors=int(st.errors), sampled_ok=good)
    ok &= good == len(range(0, len(lost), max(1, len(lost) // a.verify)))
    bcp.task_shutdown()
    if not a.keep:
        shutil.rmtree(root, ignore_errors=True)
    return ok


def config5(a):
    root = os.path.join(a.root, "c5")
    shutil.rmtree(root, ignore_errors=True)
    rng = np.random.default_rng(5)
    ntargets = 9
    files = []
    for i in range(a.c5_stripes):
        holders, p = S.random_layout(rng, ntargets, 8)
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
        files.append((f"u{i % 8}/{(i * 2654435761) % 65536:04X}/chunk{i}", holders, p, lens))
    t = time.time()
    contents = write_store(root, files, 2)
    emit(stage="config5_store_written", stripes=len(files), GiB=round(sum(sum(f[3]) for f in files) / GiB, 2),
         seconds=round(time.time() - t, 2))
    ts0 = 1_700_000_000
    items = [(path, ts0, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
    rd, wr = total_bytes(root, files)
    ok_proto = True
    # full generation through the per-task protocol first (12 lanes), the
    # default GPU fold against the reference CPU fold, interleaved: 8 rows of
    # up to 4 MiB per window
    ref_fold, ref_name = oracle.cpu_fold_hook()
    pipe_fold = ctypes.cast(oracle.lib().oracle_xor_rows, ctypes.c_void_p).value
    pvariants = [("protocol_gpu_fold(bcp_gen_run,12 lanes)", None, None, False),
                 (CPU_REF + f"({ref_name},reference wire,12 lanes)", bcp.FOLD_BATCHED, ref_fold, True),
                 (CPU_PIPE + "(oracle_xor_rows,12 lanes)", None, pipe_fold, False)]
    ptimes = {v[0]: [] for v in pvariants}
    preps = max(a.reps, 5)
    nv = len(pvariants)
    for r in range(1 + preps):
        for label, mode, hook, ref_wire in pvariants[r % nv:] + pvariants[:r % nv]:
            for k in range(ntargets):
                shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
                os.makedirs(os.path.join(root, f"st{k}", "parity"))
            restore = fold_ctx(mode, hook, ref_wire)
            try:
                t0 = time.perf_counter()
                st = bcp.gen_run(root, ntargets, items, nlanes=12)
                ptimes[label].append(time.perf_counter() - t0)
            finally:
                restore()
            if r == preps:
                okp, badp = verify(root, files, contents, a.verify, rng)
                ok_proto &= okp
                dtp = float(np.median(ptimes[label][1:]))
                emit(config=5, path=label, cold_seconds=round(ptimes[label][0], 3), warm_seconds=round(dtp, 3),
                     GiBps=round((rd + wr) / dtp / GiB, 3), runs_s=[round(x, 4) for x in ptimes[label]],
                     bytes_read=rd, bytes_written=wr, tasks=int(st.tasks), errors=int(st.errors), verified=okp,
                     bad=badp, order="interleaved")
    bcp.task_shutdown()  # the protocol's engine goes before the pipeline's comes
    pl = bcp.Pipeline(io_threads=a.io_threads, ndevices=a.ndevices)
    times = []
    for r in range(1 + a.reps):
        t0 = time.perf_counter()
        st = pl.run(root, ntargets, items)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times[1:])) if a.reps else times[0]
    ok, bad = verify(root, files, contents, a.verify, rng)
    emit(config=5, path=f"pipeline_full_gen({a.ndevices} GPU)", cold_seconds=round(times[0], 3), warm_seconds=round(dt, 3),
         GiBps=round((rd + wr) / dt / GiB, 3), bytes_read=rd, bytes_written=wr, tasks=int(st.tasks), verified=ok,
         bad=bad, runs_s=[round(x, 4) for x in times], last_run_timing=pl.last_timing())
    ok &= ok_proto
    # changelog: a seeded 10 % of stripes rewritten -> record streams per target
    sub = sorted(int(x) for x in rng.choice(len(files), size=max(1, len(files) // 10), replace=False))
    streams = {t: [] for t in range(ntargets)}
    ts1 = ts0 + 3600
    for i in sub:
        path, holders, p, lens = files[i]
        new = []
        for h, L in zip(holders, lens):
            data = rng.integers(0, 256, size=L, dtype=np.uint8)
            S.write_chunk(root, h, path, data)
            new.append(data)
            streams[h].append((ts1, L, "m", path))
        contents[path] = new
    # persistent state: seed every target's DB replica with the state of the
    # full generation above (what that round's process_list updates leave)
    def seed_dbs():
        for k in range(ntargets):
            db = bcp.PDB(os.path.join(root, f"st{k}", "db"))
            for path, ts, loc in items:
                db.set(path, ts, loc)
            db.close()
    t0 = time.perf_counter()
    seed_dbs()
    emit(config=5, stage="db_seeded", replicas=ntargets, entries=len(items), seconds=round(time.perf_counter() - t0, 3))
    # changelog round: events -> plan against the DB -> pipeline -> DB update;
    # a first round, then a.reps more, each after re-seeding the replicas
    # (outside the timing) so that every round plans the same subset
    cum = list(np.cumsum([1000] * ntargets))
    rtimes, rpipe, rtiming = [], [], []
    for r in range(1 + a.reps):
        if r:
            seed_dbs()
        t0 = time.perf_counter()
        es = bcp.EventSet()
        for t, recs in streams.items():
            es.feed(t, bcp.pack_records(recs))
        st, nplanned = pl.round(root, ntargets, es, cum_weight=cum)
        rtimes.append(time.perf_counter() - t0)
        es.close()
        rpipe.append(st.seconds)
        rtiming.append(pl.last_timing())
    # the planner keeps each stripe's P (fill_in_missing_fields) -> same targets
    db = bcp.PDB(os.path.join(root, "st0", "db"))
    state = {k.decode(): (ts, loc) for k, ts, loc in db.items()}
    db.close()
    want = {files[i][0]: items[i][2] for i in sub}
    plan_ok = nplanned == len(sub) and all(state[p] == (ts1, loc) for p, loc in want.items())
    sub_files = [files[i] for i in sub]
    srd, swr = total_bytes(root, sub_files)
    pl.close()
    ok2, bad2 = verify(root, sub_files, contents, a.verify, rng)
    dt = float(np.median(rtimes[1:])) if a.reps else rtimes[0]
    dtp = float(np.median(rpipe[1:])) if a.reps else rpipe[0]
    emit(config=5, path="changelog_round_pipeline(events->plan vs DB->pipeline->DB)", stripes=len(sub),
         plan_matches=plan_ok, seconds=round(dt, 4), cold_seconds=round(rtimes[0], 4), pipeline_seconds=round(dtp, 4),
         outside_pipeline_seconds=round(dt - dtp, 4), GiBps=round((srd + swr) / dt / GiB, 3),
         cold_GiBps=round((srd + swr) / rtimes[0] / GiB, 3), runs_s=[round(x, 4) for x in rtimes],
         bytes_read=srd, bytes_written=swr, tasks=int(st.tasks), verified=ok2, bad=bad2,
         pipeline_timing=rtiming[-1])
    if not a.keep:
        shutil.rmtree(root, ignore_errors=True)
    return ok and ok2 and plan_ok


def main():
    ap = argparse.ArgumentParser()
    # stores in memory (page cache without a disk behind it): /dev/shm where it exists
    ap.add_argument("--root", default=("/dev/shm" if os.path.isdir("/dev/shm") else os.environ.get("TMPDIR", "/tmp"))
                    + "/bcp_e2e")
    ap.add_argument("--configs", default="1,5")
    ap.add_argument("--c1-files", type=int, default=1333)
    ap.add_argument("--c5-stripes", type=int, default=1000)
    ap.add_argument("--io-threads", type=int, default=0, help="pipeline io threads (0: the library's 8 per GPU)")
    ap.add_argument("--ndevices", type=int, default=0, help="GPUs for the pipeline (0 = all visible)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--verify", type=int, default=20)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import box_probe
    box = box_probe.cpu_info()
    box.update(box_probe.pcie_rates(bcp))
    emit(box=box)
    if a.ndevices <= 0:
        a.ndevices = max(1, bcp.device_count())
    ok = True
    cfgs = a.configs.split(",")
    if "1" in cfgs:
        ok &= config1(a)
    if "5" in cfgs:
        ok &= config5(a)
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
