"""bench_legs.py -- the legs of bench.py's line beside the device timing.

bench.py times the device-resident kernel and assembles the line; every
other figure in it comes from a leg here, each called behind bench.run_leg
(a failure becomes {"error": ...} in its block and never costs the device
figures):
  cpu_baseline      the reference CPU path (its own xor_parity,
                    task_processing.c:96-109, oracle/_ref) on this box's cores
  config1_leg       BASELINE config 1 through the per-task protocol with the
                    reference's fold, the GPU fold and the pipeline
  e2e_leg           every rank's batched pipeline over its own chunk-file
                    store (config-5 shapes), config 5's changelog-driven
                    partial round, and (rank 0) config 5 through the per-task
                    protocol (config5_protocol)
  trace_profile /   the rocprofv3 figures: the kernel trace of the line's own
  pmc_passes        timed launches, the PMC passes of the same workload
"""
from __future__ import annotations

import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))

import bcp_ctypes as bcp  # noqa: E402

KiB = 1024
GiB = 1024 ** 3
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md chip table


def maybe_fail(leg: str):
    """Test hook: BCP_BENCH_FAIL_LEG=name[,name] makes these legs raise (the
    line must stand without them, tests/test_gpu_bench.py)."""
    if leg in os.environ.get("BCP_BENCH_FAIL_LEG", "").split(","):
        raise RuntimeError(f"injected failure of the {leg} leg")

def cpu_quota(cgroup_root: str = "/sys/fs/cgroup"):
    """CPUs the cgroup quota allows (cgroup v2 cpu.max, else v1 cfs), or None."""
    try:
        q, per = open(os.path.join(cgroup_root, "cpu.max")).read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open(os.path.join(cgroup_root, "cpu", "cpu.cfs_quota_us")).read())
        per = int(open(os.path.join(cgroup_root, "cpu", "cpu.cfs_period_us")).read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None

def usable_cpus() -> tuple[int, int, float | None]:
    """(threads worth running, affinity count, quota) -- affinity capped by the
    quota: threads beyond the quota only measure oversubscription."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = cpu_quota()
    use = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    return min(use, 256), affinity, quota

def pmc_traffic(workload_key: str, kernel_tag: str):
    """Committed profile summary (tools/pmc_summary.py) of this workload and
    kernel: per-launch HBM bytes (PMC), rocprofv3 kernel-trace average, the
    files and the code commit they came from: from the set profiles/CURRENT_SET
    names when it has one, else the last matching one in path order."""
    best = None
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc*.json"), recursive=True))
    try:
        cur = open(os.path.join(ROOT, "profiles", "CURRENT_SET")).read().strip()
    except OSError:
        cur = ""
    if cur:  # the current set last, so its match wins
        key = os.path.join(ROOT, cur) + os.sep
        paths = [x for x in paths if not x.startswith(key)] + [x for x in paths if x.startswith(key)]
    for path in paths:
        try:
            doc = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (doc.get("workload_key") == workload_key and doc.get("hbm_bytes_per_launch")
                and kernel_tag in doc.get("kernel", "")):
            doc.setdefault("files", {})["pmc_summary"] = os.path.relpath(path, ROOT)
            best = doc
    return best

def cpu_baseline(a, N: int, C: int, lens_all) -> dict:
    """The reference CPU path on this box's host cores (rank 0, after the
    device timing): its own xor_parity over a bounded sample of the timed
    workload's stripe shapes, at 1 thread and at usable_cpus() threads."""
    maybe_fail("cpu_baseline")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only
    use_ref = oracle.ref_lib() is not None
    use, affinity, quota = usable_cpus()
    legs_t = sorted({1, use})
    leg_s = a.cpu_seconds / len(legs_t)
    legs = []
    if lens_all is not None:
        import numpy as np
        shapes = np.asarray(lens_all[:min(len(lens_all), 64)], dtype=np.uint64)
        for t in legs_t:
            bps = oracle.bench_xor_shapes(t, shapes, leg_s, use_ref=use_ref)
            legs.append({"threads": t, "value": round(bps / GiB, 3), "stripe_shapes": int(len(shapes))})
        what = (f"each thread folds its share of the first {len(shapes)} timed stripe shapes ({N} chunks, "
                f"log-uniform 64 KiB-4 MiB) as the reference's P role does: one window of max_cs per source, "
                f"zero-padded rows; sum of lengths + max_cs bytes per stripe")
    else:
        for t in legs_t:
            # private pool per thread: ~2 GiB in all at 16 threads (out of
            # cache), at least 4 stripes each when many threads run
            per_thread = a.cpu_stripes if t == 1 else max(4, a.cpu_stripes * 2 // t)
            bps = oracle.bench_xor(t, per_thread, N, C, leg_s, use_ref=use_ref)
            legs.append({"threads": t, "value": round(bps / GiB, 3), "pool_stripes_per_thread": per_thread})
        what = (f"each thread folds a private pool of {N} x {C // KiB} KiB synthetic stripes; "
                f"(N+1)*S bytes per stripe")
    best = max(legs, key=lambda x: x["value"])
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    fn = ("the reference's own xor_parity (task_processing.c:96-109 compiled unchanged, -std=gnu99 -Os, "
          "oracle/_ref)") if use_ref else "oracle_xor_parity (the reference's xor_parity restated, -std=gnu99 -Os)"
    return {"value": best["value"], "unit": "GiB/s", "cores": best["threads"],
            "kind": "reference" if use_ref else "port",
            "sample": f"{fn}: {what}, in a loop for >= {leg_s:g} s per leg; legs at 1 thread and at the "
                      f"usable CPUs (affinity capped by the cgroup quota), value = the faster leg; "
                      f"rank 0, after the device timing",
            "legs": legs, "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "quota_cpus": None if quota is None else round(quota, 2), "cpu_model": model}

def cpu_baseline_fold():
    """The cpu_baseline leg's library as a P-role fold hook (bcp_xor_hook_fn):
    the reference's own xor_parity, task_processing.c:96-109 compiled
    unchanged into oracle/_ref (oracle.cpu_fold_hook; the restatement where
    _ref was not built).  Only config1_leg's reference_fold leg uses it --
    the reference CPU path timed beside the product, never the product."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only
    return oracle.cpu_fold_hook()

def link_rates(device: int) -> dict:
    """This process's H2D / D2H over pinned memory on `device` (256 MiB, median of 5)."""
    import numpy as np
    eng = bcp.Engine(device)
    q = eng.queue()
    nb = 256 << 20
    h = eng.host_alloc(nb)
    dv = eng.alloc(nb)
    out = {}
    try:
        for name, fn in (("h2d_GBps", lambda: q.h2d(dv, h, nb)), ("d2h_GBps", lambda: q.d2h(h, dv, nb))):
            tt = []
            for _ in range(5):
                q.sync()
                t0 = time.perf_counter()
                fn()
                q.sync()
                tt.append(time.perf_counter() - t0)
            out[name] = round(nb / float(np.median(tt)) / 1e9, 2)
    finally:
        q.sync()
        eng.free(dv)
        eng.host_free(h)
        q.close()
        eng.close()
    return out

def zero_copy_fold_rate(device: int, lanes: int = 12, stripes: int = 768, nsrc: int = 3,
                        chunk: int = 512 * KiB) -> dict:
    """The config-1 protocol's GPU fold shape with nothing else: `lanes`
    threads, each folding one stripe of `nsrc` x `chunk` bytes that lives in
    pinned HOST memory and waiting for it, as the P role does -- through the
    device's resident fold ring (the product's fold since r06: one
    publication per stripe, the kernel reads the rows in place across PCIe
    and writes the parity into pinned host memory), and, beside it, with one
    launch + sync per stripe (bcp_xor_stripes_async, r05's shape).  Returns
    the ring's chunk bytes read per second and (read + written) GiB/s, the
    launch shape under `per_launch` (tools/exp/zero_copy_probe.py has the
    sweep)."""
    import ctypes
    import threading
    eng = bcp.Engine(device)
    rows = eng.host_alloc(stripes * nsrc * chunk)
    outs = eng.host_alloc(stripes * chunk)
    qs = [eng.queue() for _ in range(lanes)]
    ring = bcp.Ring(eng)
    L = bcp.lib()
    per = stripes // lanes
    args = []
    for s in range(stripes):
        st = bcp.Stripe(outs + s * chunk, chunk, 0, nsrc, 0)
        so = (bcp.Source * nsrc)(*[bcp.Source(rows + (s * nsrc + j) * chunk, chunk) for j in range(nsrc)])
        args.append((st, so))

    def lane_launch(i):
        q = qs[i]
        for s in range(i * per, (i + 1) * per):
            st, so = args[s]
            bcp.check("bcp_xor_stripes_async", L.bcp_xor_stripes_async(q.h, ctypes.byref(st), 1, so, nsrc))
            q.sync()

    def lane_ring(i):
        h = ctypes.c_uint64(0)
        for s in range(i * per, (i + 1) * per):
            st, so = args[s]
            bcp.check("bcp_ring_submit", L.bcp_ring_submit(ring.h, ctypes.byref(st), so, ctypes.byref(h)))
            bcp.check("bcp_ring_wait", L.bcp_ring_wait(ring.h, h.value))

    def best_of(fn):
        best = None
        for _ in range(3):
            ths = [threading.Thread(target=fn, args=(i,)) for i in range(lanes)]
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best
    try:
        t_ring = best_of(lane_ring)
        t_launch = best_of(lane_launch)
    finally:
        ring.close()
        for q in qs:
            q.close()
        eng.host_free(rows)
        eng.host_free(outs)
        eng.close()
    n = per * lanes

    def rates(t):
        return {"read_GBps": round(n * nsrc * chunk / t / 1e9, 2), "GiBps": round(n * (nsrc + 1) * chunk / t / GiB, 2)}
    return dict(rates(t_ring), lanes=lanes, stripes=n, shape="resident fold ring, one stripe per publication",
                per_launch=dict(rates(t_launch), shape="one launch + sync per stripe"))


def proc_cpu_s() -> float:
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime

def config1_leg(a, device: int = 0) -> dict:
    """BASELINE config 1 (configs[0]): beegfs-parity-gen --complete over 4
    loopback storage-target ranks, ~1000 x 512 KiB chunk files per rank --
    files -> per-task protocol -> XOR -> parity files, timed end to end in this
    process on rank 0 (after cpu_baseline; the other ranks wait).  SURVEY
    section 8(d): 4 targets, 3-wide stripes with P rotating over the target
    left out, --c1-files files round-robin over the 4 rotations.  Over the same
    store, interleaved in rotating order (one cold round, then --c1-reps warm):
      reference_fold  bcp_gen_run (process_task, 12 lanes per rank, the MPI
                      subset on loopback threads) with the P role folding every
                      window with the reference's OWN xor_parity
                      (task_processing.c:96-109 compiled unchanged, oracle/_ref,
                      the cpu_baseline leg's library; the restatement where
                      _ref is absent -- `kind` says which) on the reference's
                      zero-padded wire (task_processing.c:302-303), as
                      parity_generator folds (:203-226): kind "reference";
      gpu_fold        the same protocol, the P role folding on the GPU (the
                      product's default fold);
      pipeline        bcp_pipeline_run, the batched engine.
    Then target 2 is lost and rebuilt by each (protocol: one lane, tag 0, as
    rebuild/main.c:63).  Sampled parity files and rebuilt chunks are checked
    with numpy.  Rate = (chunk bytes read + parity bytes written) / warm run.
    The protocol around the reference fold is libbcp's: the reference program
    itself needs MPI.  Every leg runs on this rank's GPU
    (`device`): the P roles of all four targets are mapped to it
    (bcp_task_set_device_map; by default target st would fold on GPU st %
    count, other ranks' GPUs on a multi-GPU node)."""
    import concurrent.futures as cf
    import shutil

    import numpy as np
    import bcp_store as BS
    maybe_fail("config1")
    t_start = time.perf_counter()
    NT, C, VICTIM = 4, 512 * KiB, 2
    nfiles = a.c1_files
    need = nfiles * 3 * C
    want = int(need * 1.4)  # chunks + parity (1/3 of them) + slack
    base, room, reason = e2e_store_dir([a.e2e_dir], 1, want)
    if reason or room < want:
        return {"skipped": reason or f"{base}: room for {room / GiB:.2f} GiB, config 1 needs {want / GiB:.2f}"}
    root = os.path.join(base, f"bcp_bench_c1_{os.getpid()}")
    rng = np.random.default_rng(1)
    block = rng.integers(0, 256, size=8 << 20, dtype=np.uint8)
    files = []
    for i in range(nfiles):
        p = i % NT
        files.append((f"u0/{i % 64:02X}/chunk{i}", [t for t in range(NT) if t != p], p))

    def chunk_of(i, k):
        off = ((i * 3 + k) * 40961) % ((8 << 20) - C)
        return block[off:off + C]
    items = [(path, 2 ** 40, BS.with_p(sum(1 << h for h in hs), p)) for path, hs, p in files]
    rd, wr = nfiles * 3 * C, nfiles * (3 * 8 + C)
    lost = [i for i in range(nfiles) if VICTIM in files[i][1]]
    rb_rd = len(lost) * 3 * C + len(lost) * 3 * 8  # 2 survivors + the parity file (header + body)
    rb_wr = len(lost) * C
    vr = np.random.default_rng(13)
    sample = sorted({0, nfiles - 1} | {int(x) for x in vr.integers(0, nfiles, 10)})
    rsample = sorted({lost[0], lost[-1]} | {lost[int(x)] for x in vr.integers(0, len(lost), 8)})
    ref_fold, ref_name = cpu_baseline_fold()
    kind = "reference" if ref_name == "ref_xor_parity" else "port"
    errors = []

    def parity_ok(i):
        body = np.zeros(C, dtype=np.uint8)
        for k in range(3):
            body ^= chunk_of(i, k)
        want = np.full(3, C, dtype="<u8").tobytes() + body.tobytes()
        return BS.read_file(BS.parity_path(root, files[i][2], files[i][0])) == want

    def rebuilt_ok(i):
        return BS.read_file(BS.chunk_path(root, VICTIM, files[i][0])) == \
            chunk_of(i, files[i][1].index(VICTIM)).tobytes()

    def reset_parity():
        for k in range(NT):
            shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{k}", "parity"))

    def drop_victim():
        for i in lost:
            try:
                os.remove(BS.chunk_path(root, VICTIM, files[i][0]))
            except FileNotFoundError:
                pass

    def with_fold(leg, fn):
        """fn under the leg's P-role fold (reference: the batched fold service
        handing whole windows to the hook, senders padding as the reference's)."""
        if leg != "reference_fold":
            return fn()
        prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)
        bcp.set_xor_hook(ref_fold)
        prev_pad = bcp.set_explicit_padding(True)
        try:
            return fn()
        finally:
            bcp.set_explicit_padding(prev_pad)
            bcp.set_xor_hook(None)
            bcp.set_fold_mode(prev)

    # the two folds always; the pipeline unless --c1-legs leaves it out (A/B)
    legs = ["reference_fold", "gpu_fold"] + (["pipeline"] if "pipeline" in a.c1_legs.split(",") else [])
    pl_timing = {}
    link, zc = {}, {}
    gen_t = {x: [] for x in legs}
    reb_t = {x: [] for x in legs}
    gen_c = {x: [] for x in legs}  # this process's CPU seconds (all threads, user + system) per run
    reb_c = {x: [] for x in legs}
    ok = {x: True for x in legs}
    rok = {x: True for x in legs}
    pl = None
    import ctypes
    bcp.lib().bcp_task_set_device_map((ctypes.c_int * NT)(*([device] * NT)), NT)
    try:
        BS.make_store(root, NT)

        def write_file(i):
            path, holders, _ = files[i]
            for k, h in enumerate(holders):
                fn = BS.chunk_path(root, h, path)
                os.makedirs(os.path.dirname(fn), exist_ok=True)
                with open(fn, "wb") as f:
                    f.write(memoryview(chunk_of(i, k)))
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(write_file, range(nfiles)))
        t_store = time.perf_counter() - t0
        # diagnostics beside the legs: a failure here is reported, never costs the legs
        try:
            link = link_rates(device)
            zc = zero_copy_fold_rate(device)
        except Exception as e:
            link, zc = {"error": f"{type(e).__name__}: {e}"}, {}
        pl = bcp.Pipeline(device=device) if "pipeline" in legs else None
        runs = 1 + max(1, a.c1_reps)
        for r in range(runs):
            for leg in legs[r % len(legs):] + legs[:r % len(legs)]:
                reset_parity()
                c0 = proc_cpu_s()
                t0 = time.perf_counter()
                if leg == "pipeline":
                    st = pl.run(root, NT, items)
                    pl_timing["gen"] = pl.last_timing()
                else:
                    st = with_fold(leg, lambda: bcp.gen_run(root, NT, items, nlanes=12))
                gen_t[leg].append(time.perf_counter() - t0)
                gen_c[leg].append(proc_cpu_s() - c0)
                good = st.errors == 0 and st.tasks == (nfiles if leg == "pipeline" else 4 * nfiles)
                if r == runs - 1:
                    good = good and all(parity_ok(i) for i in sample)
                ok[leg] = ok[leg] and good
        # rebuild of target VICTIM (protocol: one lane, tag 0, as rebuild/main.c)
        ordered = sorted(items, key=lambda x: x[0].encode())
        prev_lanes = bcp.set_rebuild_lanes(1)
        try:
            for r in range(runs):
                for leg in legs[r % len(legs):] + legs[:r % len(legs)]:
                    drop_victim()
                    c0 = proc_cpu_s()
                    t0 = time.perf_counter()
                    if leg == "pipeline":
                        st = pl.rebuild(root, NT, VICTIM, ordered)
                        pl_timing["rebuild"] = pl.last_timing()
                    else:
                        st = with_fold(leg, lambda: bcp.rebuild_run(root, NT, VICTIM, ordered))
                    reb_t[leg].append(time.perf_counter() - t0)
                    reb_c[leg].append(proc_cpu_s() - c0)
                    good = st.errors == 0
                    if r == runs - 1:
                        good = good and all(rebuilt_ok(i) for i in rsample)
                    rok[leg] = rok[leg] and good
        finally:
            bcp.set_rebuild_lanes(prev_lanes)
    except Exception as e:  # reported in the block, never raised: the device line stands
        errors.append(f"{type(e).__name__}: {e}")
    finally:
        if pl is not None:
            pl.close()
        bcp.task_shutdown()
        bcp.lib().bcp_task_set_device_map(None, 0)
        shutil.rmtree(root, ignore_errors=True)
    if errors:
        return {"error": errors[0], "wall_s": round(time.perf_counter() - t_start, 1)}
    import statistics

    def summary(t, c, b, good):
        warm = statistics.median(t[1:])
        return {"cold_s": round(t[0], 4), "warm_s": round(warm, 4), "runs_s": [round(x, 4) for x in t],
                "GiBps": round(b / warm / GiB, 2), "verified": good,
                "cpu_s": round(statistics.median(c[1:]), 3),
                "cores_busy": round(statistics.median(x / y for x, y in zip(c[1:], t[1:])), 1)}
    gen = {leg: summary(gen_t[leg], gen_c[leg], rd + wr, ok[leg]) for leg in legs}
    reb = {leg: summary(reb_t[leg], reb_c[leg], rb_rd + rb_wr, rok[leg]) for leg in legs}
    gen["reference_fold"]["kind"] = reb["reference_fold"]["kind"] = kind
    if "pipeline" in legs:
        gen["pipeline"]["last_run_timing"] = pl_timing.get("gen")
        reb["pipeline"]["last_run_timing"] = pl_timing.get("rebuild")
    return {
        "workload": f"config1: beegfs-parity-gen --complete, {NT} loopback storage-target ranks, {nfiles} files x 3 "
                    f"x {C // KiB} KiB chunks ({nfiles * 3 // NT} per rank), P rotating over the target left out",
        "store": {"dir": base, "chunk_GiB": round(rd / GiB, 3), "write_s": round(t_store, 2)},
        "device": device,
        "gen": gen,
        "rebuild": {"target": VICTIM, "files": len(lost), **reb},
        "gpu_fold_over_reference_fold": round(gen["gpu_fold"]["GiBps"] / gen["reference_fold"]["GiBps"], 3),
        "pipeline_over_reference_fold": (round(gen["pipeline"]["GiBps"] / gen["reference_fold"]["GiBps"], 3)
                                         if "pipeline" in gen else None),
        "rebuild_gpu_fold_over_reference_fold": round(reb["gpu_fold"]["GiBps"] / reb["reference_fold"]["GiBps"], 3),
        # every chunk byte a GPU fold folds crosses the host-to-device link once (parity comes back
        # on the other direction): the gen rate it cannot pass on this link
        "link": link,
        "gpu_fold_link_ceiling_GiBps": (round((rd + wr) / (rd / (link["h2d_GBps"] * 1e9)) / GiB, 2)
                                        if link.get("h2d_GBps") else None),
        # ... and what the device folds of rows in pinned host memory reach in the protocol's shape
        # (12 lanes, one stripe per launch, read in place), the fold alone: the GPU fold's own bound
        "gpu_fold_in_place_bound": zc,
        "gpu_fold_over_link_ceiling": (round(gen["gpu_fold"]["GiBps"] / ((rd + wr) / (rd / (link["h2d_GBps"] * 1e9))
                                                                         / GiB), 3) if link.get("h2d_GBps") else None),
        "gpu_fold_over_in_place_bound": (round(gen["gpu_fold"]["GiBps"] / zc["GiBps"], 3)
                                         if isinstance(zc, dict) and zc.get("GiBps") else None),
        "bytes": {"gen_read": rd, "gen_written": wr, "rebuild_read": rb_rd, "rebuild_written": rb_wr},
        "cpu_quota": cpu_quota(),
        "cpu_note": "cpu_s: this process's CPU seconds (all threads, user + system, getrusage) per warm run, median; "
                    "cores_busy: cpu_s / wall per run, median -- against cpu_quota, the host CPU time bounds the "
                    "protocol legs (tmpfs reads and parity writes are kernel copies)",
        "legs_note": "reference_fold: bcp_gen_run / bcp_rebuild_run (process_task over loopback threads, 12 lanes "
                     "per rank for gen, 1 for rebuild) with the P role's fold = the reference's own xor_parity "
                     f"({ref_name}) over whole windows on the reference's zero-padded wire; gpu_fold: the same "
                     "protocol, GPU fold; pipeline: bcp_pipeline_run / _rebuild. Interleaved in rotating order, "
                     "one cold round then warm ones (median); GiBps = (bytes read + written) / warm run",
        "wall_s": round(time.perf_counter() - t_start, 1),
    }

def _with_fold(leg: str, fn, ref_fold):
    """fn under a protocol leg's P-role fold: reference_fold -- the batched
    fold service handing whole windows to the reference's own xor_parity,
    senders on the reference's zero-padded wire; gpu_fold -- the product's
    default (PIPELINED through the device's resident fold ring)."""
    if leg != "reference_fold":
        return fn()
    prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)
    bcp.set_xor_hook(ref_fold)
    prev_pad = bcp.set_explicit_padding(True)
    try:
        return fn()
    finally:
        bcp.set_explicit_padding(prev_pad)
        bcp.set_xor_hook(None)
        bcp.set_fold_mode(prev)


def config5_protocol(a, root, NT, victim, files, items, ordered, lens, lost, chunk_of, device) -> dict:
    """BASELINE config 5's shapes (8-wide stripes, chunks log-uniform 64 KiB-
    4 MiB) through the per-task protocol, on the e2e leg's store, in this
    process (rank 0; the other ranks wait): the P role folding with the
    reference's own xor_parity (task_processing.c:96-109 compiled unchanged,
    oracle/_ref, kind "reference"; whole windows on the reference's zero-padded
    wire, as parity_generator folds them, :203-226) against the GPU fold (the
    product's default: PIPELINED through the resident fold ring, lane
    deferral).  Gen over loopback ranks with 12 lanes each (gen/main.c:116-164,
    821-889), then the rebuild of target `victim` with one lane
    (rebuild/main.c:40-89); legs interleaved in rotating order, one cold round
    then --c5-reps warm ones (gen; the rebuild one warm), the parity
    directories emptied before every gen run; sampled parity files and rebuilt
    chunks checked with numpy.  Rate = (bytes read + written) / warm run."""
    import ctypes
    import shutil
    import statistics

    import numpy as np
    import bcp_store as BS
    maybe_fail("config5_protocol")
    t_start = time.perf_counter()
    W = 8
    ref_fold, ref_name = cpu_baseline_fold()
    kind = "reference" if ref_name == "ref_xor_parity" else "port"
    legs = ["reference_fold", "gpu_fold"]
    nst = len(files)
    rd = int(sum(int(x.sum()) for x in lens))
    wr = int(sum(8 * W + int(x.max()) for x in lens))
    rb_rd = sum(int(lens[i].sum()) - int(lens[i][files[i][1].index(victim)]) + int(lens[i].max()) + 8 * W
                for i in lost)
    rb_wr = sum(int(lens[i][files[i][1].index(victim)]) for i in lost)
    vr = np.random.default_rng(23)
    sample = sorted({0, nst - 1} | {int(x) for x in vr.integers(0, nst, 8)})
    lost_set = set(lost)
    rsample = sorted({lost[0], lost[-1]} | {lost[int(x)] for x in vr.integers(0, len(lost), 6)})

    def parity_ok(i):
        ch = [chunk_of(i, k) for k in range(W)]
        m = max(len(c) for c in ch)
        body = np.zeros(m, dtype=np.uint8)
        for c in ch:
            body[:len(c)] ^= c
        return BS.read_file(BS.parity_path(root, files[i][2], files[i][0])) == \
            np.asarray([len(c) for c in ch], dtype="<u8").tobytes() + body.tobytes()

    def rebuilt_ok(i):
        return BS.read_file(BS.chunk_path(root, victim, files[i][0])) == \
            chunk_of(i, files[i][1].index(victim)).tobytes()

    def reset_parity():
        for k in range(NT):
            shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{k}", "parity"))

    def drop_victim():
        for i in lost:
            try:
                os.remove(BS.chunk_path(root, victim, files[i][0]))
            except FileNotFoundError:
                pass
    gen_t = {x: [] for x in legs}
    reb_t = {x: [] for x in legs}
    gen_c = {x: [] for x in legs}
    ok = {x: True for x in legs}
    rok = {x: True for x in legs}
    bcp.lib().bcp_task_set_device_map((ctypes.c_int * NT)(*([device] * NT)), NT)
    p0, l0 = bcp.ring_stats()
    try:
        runs = 1 + max(1, a.c5_reps)
        for r in range(runs):
            for leg in legs[r % 2:] + legs[:r % 2]:
                reset_parity()
                c0 = proc_cpu_s()
                t0 = time.perf_counter()
                st = _with_fold(leg, lambda: bcp.gen_run(root, NT, items, nlanes=12), ref_fold)
                gen_t[leg].append(time.perf_counter() - t0)
                gen_c[leg].append(proc_cpu_s() - c0)
                good = st.errors == 0
                if r == runs - 1:
                    good = good and all(parity_ok(i) for i in sample)
                ok[leg] = ok[leg] and good
        prev_lanes = bcp.set_rebuild_lanes(1)
        try:
            for r in range(2):
                for leg in legs[r % 2:] + legs[:r % 2]:
                    drop_victim()
                    t0 = time.perf_counter()
                    st = _with_fold(leg, lambda: bcp.rebuild_run(root, NT, victim, ordered), ref_fold)
                    reb_t[leg].append(time.perf_counter() - t0)
                    good = st.errors == 0
                    if r == 1:
                        good = good and all(rebuilt_ok(i) for i in rsample if i in lost_set)
                    rok[leg] = rok[leg] and good
        finally:
            bcp.set_rebuild_lanes(prev_lanes)
        p1, l1 = bcp.ring_stats()
    finally:
        bcp.task_shutdown()
        bcp.lib().bcp_task_set_device_map(None, 0)

    def summary(t, b, good, c=None):
        warm = statistics.median(t[1:])
        out = {"cold_s": round(t[0], 4), "warm_s": round(warm, 4), "runs_s": [round(x, 4) for x in t],
               "GiBps": round(b / warm / GiB, 2), "verified": good}
        if c:
            out["cpu_s"] = round(statistics.median(c[1:]), 3)
        return out
    gen = {leg: summary(gen_t[leg], rd + wr, ok[leg], gen_c[leg]) for leg in legs}
    reb = {leg: summary(reb_t[leg], rb_rd + rb_wr, rok[leg]) for leg in legs}
    gen["reference_fold"]["kind"] = reb["reference_fold"]["kind"] = kind
    return {"workload": f"config5 shapes through process_task: {NT} loopback storage-target ranks, {nst} stripes x "
                        f"{W} chunks log-uniform 64 KiB-4 MiB ({rd / GiB:.2f} GiB), P rotating over the target "
                        f"left out; the e2e leg's store",
            "gen": gen, "rebuild": dict(reb, target=victim, stripes=len(lost)),
            "gpu_fold_over_reference_fold": round(gen["gpu_fold"]["GiBps"] / gen["reference_fold"]["GiBps"], 3),
            "rebuild_gpu_fold_over_reference_fold": round(reb["gpu_fold"]["GiBps"] /
                                                          reb["reference_fold"]["GiBps"], 3),
            "ring": {"pieces": p1 - p0, "launches": l1 - l0},
            "bytes": {"gen_read": rd, "gen_written": wr, "rebuild_read": rb_rd, "rebuild_written": rb_wr},
            "legs_note": "reference_fold: bcp_gen_run / bcp_rebuild_run (process_task over loopback threads, 12 lanes "
                         "per rank for gen, 1 for rebuild) with the P role's fold = the reference's own xor_parity "
                         f"({ref_name}) over whole windows on the reference's zero-padded wire; gpu_fold: the same "
                         "protocol, the product's GPU fold (PIPELINED, resident fold ring, lane deferral)",
            "wall_s": round(time.perf_counter() - t_start, 1)}


def e2e_store_dir(dirs, world: int, want: int):
    """(directory, bytes per rank, reason or None) for the ranks' end-to-end
    stores: the first of dirs, then the temp dir, with room for every rank's
    store (chunks + parity, ~35 % of the chunk bytes at config-5 shapes, + one
    rebuilt target: 1.7x the chunk bytes), else the roomiest, the stores shrunk
    to fit; a reason when not even 64 MiB per rank fit."""
    import tempfile
    base, room, reason = None, 0, None
    for cand in dict.fromkeys(list(dirs) + [tempfile.gettempdir()]):
        try:
            stv = os.statvfs(cand)
        except OSError as e:
            reason = f"{cand}: {e}"
            continue
        r = int(stv.f_bavail * stv.f_frsize / (1.7 * world))
        if r > room:
            base, room = cand, r
        if r >= want:
            break
    if base is None:
        return dirs[0], 0, reason or "no directory for the stores"
    want = min(want, room)
    if want < (64 << 20):
        return base, want, f"{base}: {room * 1.7 * world / GiB:.1f} GiB free for {world} stores"
    return base, want, None

def e2e_leg(a, d, device: int, bus_id: str):
    """End to end from chunk files, every rank on its own GPU at once: a store
    of config-5 shapes (8-wide stripes, chunk lengths log-uniform in
    [64 KiB, 4 MiB], 9 storage targets, P rotating over the one left out) of
    about --e2e-gib per rank in --e2e-dir; the batched pipeline generates every
    parity file (one cold run, --e2e-reps warm), then target 4 is lost (its
    chunk files deleted, outside the timing) and rebuilt -- each through the
    pipeline's read paths of --e2e-modes, interleaved (the first is the
    headline `gen` / `rebuild`, the others in `by_read_mode`).  The reference's
    I/O path: task_processing.c:62-79,186,199-226 (read, fold, write).
    Returns the rank-0 summary (None elsewhere); never part of `value`.
    A failure on any rank is reported in the block (`errors`), never raised:
    every rank keeps making the same collective calls, so the bench line of
    the device-resident measurement is printed whatever happens here."""
    import concurrent.futures as cf
    import shutil

    import numpy as np
    import bcp_store as BS
    t_start = time.perf_counter()
    NT, W, VICTIM = 9, 8, 4
    modes = [m for m in a.e2e_modes.split(",") if m in ("copy", "direct")] or ["copy"]
    base, want, reason = e2e_store_dir([a.e2e_dir], d.world, int(a.e2e_gib * GiB))
    rank_root = os.path.join(base, f"bcp_bench_e2e_{os.getppid()}_{d.rank}")
    # every rank agrees to run (or not): a rank that skipped would leave the
    # others waiting at the barriers below
    if d.sum(0.0 if reason else 1.0) != d.world:
        if d.rank == 0:
            return {"skipped": reason or "another rank could not create its store"}
        return None
    errors = []

    def guard(what, fn, default=None):
        try:
            return fn()
        except Exception as e:  # reported in the block, never raised (see above)
            errors.append(f"{what}: {type(e).__name__}: {e}")
            return default

    rng = np.random.default_rng(5 + d.rank)
    lens, tot = [], 0
    while tot < want:
        ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=W)).astype(np.int64)
        lens.append(ls)
        tot += int(ls.sum())
    nst = len(lens)
    block = rng.integers(0, 256, size=12 << 20, dtype=np.uint8)
    files = []
    for i in range(nst):
        p = i % NT
        files.append((f"e2e/{i % 64:02x}/chunk{i}", [t for t in range(NT) if t != p], p))
    ts = int(time.time()) + 3600
    items = [(path, ts, BS.with_p(sum(1 << h for h in hs), p)) for path, hs, p in files]
    rd = int(sum(int(x.sum()) for x in lens))
    wr = int(sum(8 * W + int(x.max()) for x in lens))
    lost = [i for i in range(nst) if VICTIM in files[i][1]]
    ordered = sorted(items, key=lambda x: x[0].encode())  # DB key order (rebuild/main.c:223-225)
    rd3 = sum(int(lens[i].sum()) - int(lens[i][files[i][1].index(VICTIM)]) + int(lens[i].max()) + 8 * W
              for i in lost)
    wr3 = sum(int(lens[i][files[i][1].index(VICTIM)]) for i in lost)
    vr = np.random.default_rng(11 + d.rank)
    sample = sorted({0, nst - 1} | {int(x) for x in vr.integers(0, nst, 6)})
    rsample = [i for i in sample if i in set(lost)] or lost[:2]

    cur_off = {}  # (stripe, chunk) -> block offset once the partial round rewrote it

    def chunk_of(i, k):
        off = cur_off.get((i, k), ((i * W + k) * 40961) % (8 << 20))
        return block[off:off + int(lens[i][k])]

    def write_store():
        if os.environ.get("BCP_BENCH_E2E_FAIL_RANK") == str(d.rank):  # test hook: a rank whose store fails
            raise OSError(f"injected store failure on rank {d.rank}")
        shutil.rmtree(rank_root, ignore_errors=True)
        BS.make_store(rank_root, NT)

        def write_stripe(i):
            path, holders, _ = files[i]
            for k, h in enumerate(holders):
                fn = BS.chunk_path(rank_root, h, path)
                os.makedirs(os.path.dirname(fn), exist_ok=True)
                with open(fn, "wb") as f:
                    f.write(memoryview(chunk_of(i, k)))
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(write_stripe, range(nst)))
        return time.perf_counter() - t0

    def parity_ok(i):
        ch = [chunk_of(i, k) for k in range(W)]
        m = max(len(c) for c in ch)
        body = np.zeros(m, dtype=np.uint8)
        for c in ch:
            body[:len(c)] ^= c
        want_file = np.asarray([len(c) for c in ch], dtype="<u8").tobytes() + body.tobytes()
        return BS.read_file(BS.parity_path(rank_root, files[i][2], files[i][0])) == want_file

    def rebuilt_ok(i):
        return BS.read_file(BS.chunk_path(rank_root, VICTIM, files[i][0])) == \
            chunk_of(i, files[i][1].index(VICTIM)).tobytes()

    def drop_victim():
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda i: os.remove(BS.chunk_path(rank_root, VICTIM, files[i][0])), lost))

    def partial_round(pl):
        """A seeded 10 % of the stripes is rewritten (new chunk contents, same
        lengths, outside the timing); their chunk events go out as one binary
        record stream per target ({i64 ts, u64 size, u64 'm', u64 len, path},
        bp-find-all-chunks/main.c:25-33); every target's DB replica holds the
        full generation's state (seeded outside the timing, as the full run's
        process_list updates leave it, gen/main.c:146-149).  Timed, every rank
        at once: bcp_gen_round_pipeline -- records parsed into the event set
        (gen/main.c:286-336), the worklist planned against the DB (merge, P
        kept, NO_P when unchanged: :772-788; bcp_plan_rounds), only the subset
        recomputed through the pipeline, the replicas updated.  One cold and
        two warm rounds (the replicas re-seeded between them, so each plans the
        same subset); checked: the plan is exactly the subset with each
        stripe's P kept, and sampled parity files against numpy.  Every rank
        makes the same barrier calls whatever fails (failures are reported)."""
        prng = np.random.default_rng(17 + d.rank)
        sub = sorted(int(x) for x in prng.choice(nst, size=max(1, nst // 10), replace=False))
        ts1 = ts + 3600
        new_off = {}

        def prepare():
            streams = {t: [] for t in range(NT)}
            for i in sub:
                path, holders, _ = files[i]
                for k, h in enumerate(holders):
                    off = ((i * W + k) * 65537 + 12345) % (8 << 20)
                    new_off[(i, k)] = off
                    cur_off[(i, k)] = off
                    with open(BS.chunk_path(rank_root, h, path), "wb") as f:
                        f.write(memoryview(block[off:off + int(lens[i][k])]))
                    streams[h].append((ts1, int(lens[i][k]), "m", path))
            return {t: bcp.pack_records(recs) for t, recs in streams.items()}

        def seed_dbs():
            for k in range(NT):
                dbdir = os.path.join(rank_root, f"st{k}", "db")
                shutil.rmtree(dbdir, ignore_errors=True)
                db = bcp.PDB(dbdir)
                for path, t_, loc in items:
                    db.set(path, t_, loc)
                db.close()

        def one_round():
            t0 = time.perf_counter()
            es = bcp.EventSet()
            try:
                for t, data in packed.items():
                    es.feed(t, data)
                t_parse = time.perf_counter() - t0
                st, nplanned = pl.round(rank_root, NT, es, cum_weight=[1000 * (k + 1) for k in range(NT)])
            finally:
                es.close()
            return (time.perf_counter() - t0, st.seconds, nplanned == len(sub) and st.errors == 0 and st.tasks == len(sub),
                    pl.last_timing(), dict(bcp.round_timing(), parse_s=round(t_parse, 5)))

        packed = guard("partial: rewriting the subset", prepare) if pl is not None else None
        runs_p = []
        for r in range(3):
            if packed is not None:
                guard("partial: seeding the DB replicas", seed_dbs)
            d.barrier()
            if packed is not None:
                res = guard("partial round", one_round)
                if res is not None:
                    runs_p.append(res)

        def check():
            db = bcp.PDB(os.path.join(rank_root, "st0", "db"))
            state = {k.decode(): (t_, loc) for k, t_, loc in db.items()}
            db.close()
            plan_ok = all(x[2] for x in runs_p) and all(state[files[i][0]] == (ts1, items[i][2]) for i in sub)

            def sub_parity_ok(i):
                ch = [block[new_off[(i, k)]:new_off[(i, k)] + int(lens[i][k])] for k in range(W)]
                m = max(len(c) for c in ch)
                body = np.zeros(m, dtype=np.uint8)
                for c in ch:
                    body[:len(c)] ^= c
                return BS.read_file(BS.parity_path(rank_root, files[i][2], files[i][0])) == \
                    np.asarray([len(c) for c in ch], dtype="<u8").tobytes() + body.tobytes()
            ssample = sorted({sub[0], sub[-1]} | {sub[int(x)] for x in prng.integers(0, len(sub), 6)})
            return plan_ok, plan_ok and all(sub_parity_ok(i) for i in ssample)
        if len(runs_p) != 3:
            return None
        plan_ok, verified = guard("partial: checking", check, (False, False))
        times = [x[0] for x in runs_p]
        warm = runs_p[1:]
        stages = {k: round(float(np.median([x[4][k] for x in warm])), 5) for k in warm[0][4]}
        return {"stripes": len(sub), "bytes_read": sum(int(lens[i].sum()) for i in sub),
                "bytes_written": sum(8 * W + int(lens[i].max()) for i in sub),
                "own_runs_s": [round(x, 4) for x in times], "own_warm_s": round(float(np.median(times[1:])), 4),
                "own_pipeline_warm_s": round(float(np.median([x[1] for x in runs_p][1:])), 4),
                "stages_warm_s": stages,
                "pipeline_timing_last": runs_p[-1][3],
                "plan_ok": bool(plan_ok), "verified": bool(verified)}

    pls = {}
    c5p = None
    runs = {m: [] for m in modes}
    rruns = {m: [] for m in modes}
    ok = {m: True for m in modes}
    rok = {m: True for m in modes}

    def timed(m, what, before=None):
        """One run of mode m on every rank at once: (own s, slowest rank's s, timing)."""
        pl = pls.get(m)
        if before and pl is not None:
            guard("delete the lost target", before)
        d.barrier()
        t0 = time.perf_counter()
        st = guard(f"{what} ({m})", (lambda: pl.run(rank_root, NT, items)) if what == "gen" else
                   (lambda: pl.rebuild(rank_root, NT, VICTIM, ordered))) if pl is not None else None
        dt = time.perf_counter() - t0
        dmax = d.max(dt)
        tim = guard("timing", pl.last_timing, {}) if pl is not None else {}
        good = st is not None and st.errors == 0 and st.tasks == (nst if what == "gen" else len(lost))
        if what == "gen":
            good = good and st.bytes_read == rd
        return (dt, dmax, tim), good

    # every rank's pipeline in the host's CPU share: readers and writers each
    # half of the rank's part of it, 2..8 (the library's own rule for one
    # process, which cannot see its sibling ranks)
    io_threads = max(2, min(8, usable_cpus()[0] // (2 * d.world)))
    partial = None
    try:
        t_store = guard("writing the store", write_store, 0.0)
        d.barrier()
        link = guard("link probe", lambda: link_rates(device), {}) or {}
        for m in modes:
            pl = guard(f"pipeline ({m})", lambda: bcp.Pipeline(
                device=device, io_threads=io_threads,
                read_mode={"copy": bcp.READ_COPY, "direct": bcp.READ_DIRECT}[m]))
            if pl is not None:
                pls[m] = pl
        # ---- gen: one cold run, then warm runs, the read paths interleaved
        nrep = 1 + max(1, a.e2e_reps)
        for r in range(nrep):
            last_rep = r == nrep - 1 or (r > 1 and d.max(time.perf_counter() - t_start) > a.e2e_max_s)
            for m in modes:
                res, good = timed(m, "gen")
                runs[m].append(res)
                ok[m] = ok[m] and good
                if last_rep:  # this mode's files, checked before the next mode rewrites them
                    ok[m] = ok[m] and bool(guard("checking parity", lambda: all(parity_ok(i) for i in sample)))
            if last_rep:
                break
        # ---- rebuild target VICTIM from 7 survivors + parity, each read path
        for r in range(2):
            for m in modes:
                res, good = timed(m, "rebuild", before=drop_victim)
                rruns[m].append(res)
                rok[m] = rok[m] and good
                if r == 1:
                    rok[m] = rok[m] and bool(guard("checking rebuilt chunks",
                                                   lambda: all(rebuilt_ok(i) for i in rsample)))
        # ---- config 5's changelog-driven partial update (BASELINE configs[4])
        partial = partial_round(pls.get(modes[0]))
        # ---- config 5 through the per-task protocol (rank 0, same store)
        if d.rank == 0 and not a.no_configs:
            try:  # its own block: a failure here is not the pipeline's
                c5p = config5_protocol(a, rank_root, NT, VICTIM, files, items, ordered, lens, lost, chunk_of, device)
            except Exception as e:
                c5p = {"error": f"{type(e).__name__}: {e}"}
        d.barrier()
    finally:
        for p_ in pls.values():
            guard("closing a pipeline", p_.close)
        shutil.rmtree(rank_root, ignore_errors=True)

    def summary(m):
        g, rb = runs[m], rruns[m]
        warm = [x[1] for x in g[1:]] or [g[0][1]]
        warm_own = [x[0] for x in g[1:]] or [g[0][0]]
        return ({"read_mode": m, "cold_s": round(g[0][1], 4), "warm_s": round(float(np.median(warm)), 4),
                 "runs_s": [round(x[1], 4) for x in g], "own_warm_s": round(float(np.median(warm_own)), 4),
                 "timing": g[-1][2], "verified": ok[m]},
                {"read_mode": m, "cold_s": round(rb[0][1], 4), "warm_s": round(rb[-1][1], 4),
                 "own_warm_s": round(rb[-1][0], 4), "timing": rb[-1][2], "verified": rok[m]})
    per_mode = {m: summary(m) for m in modes}
    gen, reb = per_mode[modes[0]]
    mine = {"rank": d.rank, "pci_bus_id": bus_id, **link, "stripes": nst, "bytes_read": rd, "bytes_written": wr,
            "gen_own_warm_s": gen["own_warm_s"], "gen_GiBps": round((rd + wr) / gen["own_warm_s"] / GiB, 2),
            "gen_input_over_link": (round(rd / gen["own_warm_s"] / (link["h2d_GBps"] * 1e9), 3)
                                    if link.get("h2d_GBps") else None),
            "rebuild_bytes_read": rd3, "rebuild_bytes_written": wr3, "rebuild_own_warm_s": reb["own_warm_s"],
            "gen_verified": all(ok.values()), "rebuild_verified": all(rok.values()),
            "store_write_s": round(t_store, 2),
            "partial": partial or None,
            "config5_protocol": c5p,
            "own_warm_s_by_mode": {m: [per_mode[m][0]["own_warm_s"], per_mode[m][1]["own_warm_s"]] for m in modes},
            "errors": errors or None}
    ranks = d.gather(mine)
    if d.rank != 0:
        return None
    rd_all = sum(r["bytes_read"] for r in ranks)
    wr_all = sum(r["bytes_written"] for r in ranks)
    rd3_all = sum(r["rebuild_bytes_read"] for r in ranks)
    wr3_all = sum(r["rebuild_bytes_written"] for r in ranks)
    h2d_all = sum(r.get("h2d_GBps") or 0.0 for r in ranks) * 1e9
    all_errors = {r["rank"]: r["errors"] for r in ranks if r.get("errors")}

    def over_link(b, t):
        return round(b / t / h2d_all, 3) if h2d_all > 0 and not all_errors else None

    def rates(m):
        gen, reb = per_mode[m]
        return ({**gen, "bytes_read": rd_all, "bytes_written": wr_all,
                 "GiBps": round((rd_all + wr_all) / gen["warm_s"] / GiB, 2),
                 "input_GiBps": round(rd_all / gen["warm_s"] / GiB, 2),
                 "input_over_link": over_link(rd_all, gen["warm_s"]),
                 "verified": all(r["gen_verified"] for r in ranks) and not all_errors},
                {**reb, "target": VICTIM, "bytes_read": rd3_all, "bytes_written": wr3_all,
                 "GiBps": round((rd3_all + wr3_all) / reb["warm_s"] / GiB, 2),
                 "input_over_link": over_link(rd3_all, reb["warm_s"]),
                 "verified": all(r["rebuild_verified"] for r in ranks) and not all_errors})
    by_mode = {m: rates(m) for m in modes}
    gen, reb = by_mode[modes[0]]

    def partial_summary(rs):
        ps = [r.get("partial") for r in rs]
        if not all(ps):
            return {"error": "a rank did not finish its partial round", "ranks": ps}
        slow_warm = max(p["own_warm_s"] for p in ps)  # every rank at once behind a barrier: the slowest bounds
        b = sum(p["bytes_read"] + p["bytes_written"] for p in ps)
        return {"what": "config 5 changelog-driven partial update: record streams of a seeded 10 % of the "
                        "stripes (rewritten) -> bcp_gen_round_pipeline (parse, plan vs the DB replicas with "
                        "bcp_plan_rounds, pipeline over the subset, replicas updated), every rank at once",
                "stripes": sum(p["stripes"] for p in ps), "bytes_read": sum(p["bytes_read"] for p in ps),
                "bytes_written": sum(p["bytes_written"] for p in ps), "warm_s": slow_warm,
                "GiBps": round(b / slow_warm / GiB, 2),
                "bytes_read_per_rank_min": min(p["bytes_read"] for p in ps),
                "pipeline_warm_s_rank0": ps[0]["own_pipeline_warm_s"],
                "stages_warm_s_rank0": ps[0].get("stages_warm_s"),
                "pipeline_timing_rank0": ps[0].get("pipeline_timing_last"),
                "runs_s_rank0": ps[0]["own_runs_s"],
                "plan_ok": all(p["plan_ok"] for p in ps), "verified": all(p["verified"] for p in ps)}
    return {
        "path": ("bcp_pipeline_run / bcp_pipeline_rebuild on every rank's own GPU: chunk files (tmpfs) -> "
                 "pinned slabs (io threads; read_mode direct: O_DIRECT reads) -> "
                 "H2D on a side queue -> xor_desc -> D2H on a side queue -> parity files / rebuilt chunks"),
        "store": {"dir": os.path.dirname(rank_root), "shapes": "config 5: 8-wide stripes, chunks log-uniform "
                                                               "64 KiB-4 MiB, 9 targets, P rotating",
                  "stripes_per_rank": ranks[0]["stripes"], "chunk_GiB_per_rank": round(ranks[0]["bytes_read"] / GiB, 3)},
        "ranks": d.world,
        "io_threads_per_rank": io_threads,
        "read_mode": modes[0],
        "gen": gen,
        "rebuild": reb,
        "by_read_mode": {m: {"gen_GiBps": by_mode[m][0]["GiBps"], "gen_input_over_link": by_mode[m][0]["input_over_link"],
                             "gen_warm_s": by_mode[m][0]["warm_s"], "rebuild_GiBps": by_mode[m][1]["GiBps"],
                             "rebuild_warm_s": by_mode[m][1]["warm_s"],
                             "gen_timing": by_mode[m][0]["timing"]}
                         for m in modes},
        "partial": partial_summary(ranks),
        "config5_protocol": ranks[0].get("config5_protocol"),
        "link_h2d_GBps_sum": round(h2d_all / 1e9, 2),
        "errors": all_errors or None,
        "rate_note": "GiBps = (chunk bytes read + parity bytes written) of all ranks / the slowest rank's warm "
                     "run (median); input_over_link = input bytes / that time / the summed H2D rates the ranks "
                     "measured together over pinned memory; timing = rank 0's host-thread stages (seconds)",
        "wall_s": round(time.perf_counter() - t_start, 1),
        "per_rank": ranks,
    }


# ---------------------------------------------------------------------------
# rocprofv3 figures of the line's own launches
# ---------------------------------------------------------------------------
def rocprof_exe():
    import shutil
    return shutil.which("rocprofv3")


def _one(d_, pattern):
    hits = sorted(glob.glob(os.path.join(d_, "**", pattern), recursive=True))
    if not hits:
        raise RuntimeError(f"no {pattern} under {d_}")
    return hits[-1]


def trace_figures(out_dir: str, kernel_tag: str, warmup: int, steps: int, bytes_per_step: int,
                  event_ms_steps=None, event_ms_avg=None) -> dict:
    """The kernel trace of a profiled bench run (rocprofv3 --kernel-trace,
    csv): the dispatches of the timed kernel in dispatch order are the
    warm-up ones, the timed ones, the verification one, then whatever the
    later legs launch; the timed ones [warmup, warmup + steps) are averaged.
    event_ms_*: the same process's HIP-event times of those launches (the
    line's kernel_ms / kernel_ms_steps), for the two clocks' ratio."""
    import csv
    import statistics
    rows = sorted(csv.DictReader(open(_one(out_dir, "*kernel_trace.csv"))), key=lambda r: int(r["Dispatch_Id"]))
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if kernel_tag in r["Kernel_Name"]]
    if len(durs) < warmup + steps + 1:
        raise RuntimeError(f"{len(durs)} dispatches of {kernel_tag}, expected at least {warmup} + {steps} + 1")
    timed = durs[warmup:warmup + steps]
    avg = statistics.fmean(timed)
    out = {"in_process": True,
           "rocprof_avg_ns": round(avg, 1), "rocprof_median_ns": float(statistics.median(timed)),
           "rocprof_min_ns": float(min(timed)), "rocprof_max_ns": float(max(timed)),
           "rocprof_timed_launches": len(timed), "tagged_dispatches": len(durs),
           "rocprof_timed_ms_steps": [round(x / 1e6, 4) for x in timed],
           "frac_rocprof": round(bytes_per_step / (avg * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)}
    if event_ms_avg:
        out["event_over_rocprof"] = round(event_ms_avg * 1e6 / avg, 4)
    if event_ms_steps and len(event_ms_steps) == len(timed):
        out["event_over_rocprof_median"] = round(statistics.median(event_ms_steps) * 1e6 / statistics.median(timed), 4)
    return out


def pmc_passes(child_cmd: list, env: dict, kernel_tag: str, bytes_per_step: int, timeout_s: float = 150,
               keep_dir=None) -> dict:
    """HBM bytes per launch of the same workload on this box: `--pmc
    FETCH_SIZE` and `--pmc WRITE_SIZE` in child runs of their own (counters
    in separate passes, MI355X_MICROARCH.md's HBM recipe), FETCH_SIZE x2 (the
    gfx950 wide-read correction), KiB -> B; the median over the workload's
    dispatches of the kernel."""
    import csv
    import shutil
    import signal
    import statistics
    import subprocess
    import tempfile
    exe = rocprof_exe()
    if not exe:
        return {"skipped": "rocprofv3 not on PATH"}
    t0 = time.perf_counter()
    out = keep_dir or tempfile.mkdtemp(prefix="bcp_bench_pmc_")
    try:
        vals = {}
        for name in ("FETCH_SIZE", "WRITE_SIZE"):
            d_ = os.path.join(out, {"FETCH_SIZE": "pmc_fetch", "WRITE_SIZE": "pmc_write"}[name])
            cmd = [exe, "--pmc", name, "-d", d_, "-o", "run", "--output-format", "csv", "--"] + child_cmd
            p = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                                 start_new_session=True)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                raise RuntimeError(f"rocprofv3 --pmc {name}: time limit")
            if p.returncode:
                raise RuntimeError(f"rocprofv3 --pmc {name}: exit {p.returncode}: {err[-300:]}")
            v = [float(r["Counter_Value"]) for r in csv.DictReader(open(_one(d_, "*counter_collection.csv")))
                 if r["Counter_Name"] == name and kernel_tag in r["Kernel_Name"]]
            if not v:
                raise RuntimeError(f"no {name} rows for {kernel_tag}")
            vals[name] = (statistics.median(v), len(v))
        traffic = vals["FETCH_SIZE"][0] * 1024 * 2 + vals["WRITE_SIZE"][0] * 1024
        return {"traffic": round(traffic), "traffic_over_algorithmic": round(traffic / bytes_per_step, 5),
                "dispatches": {"fetch": vals["FETCH_SIZE"][1], "write": vals["WRITE_SIZE"][1]},
                "source": "live: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate child runs of this workload "
                          "on this box; FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE x1; KiB->B x1024",
                "wall_s": round(time.perf_counter() - t0, 1)}
    except Exception as e:  # reported, never fatal: the committed set stands in
        return {"error": f"{type(e).__name__}: {e}", "wall_s": round(time.perf_counter() - t0, 1)}
    finally:
        if not keep_dir:
            shutil.rmtree(out, ignore_errors=True)
