#!/usr/bin/env python3
"""bench.py -- device-resident chunk-XOR parity throughput on MI355X.

Workload (BASELINE.json configs[1], "config 2"): 12,500 stripes x 8 sources
x 512 KiB (100,000 data chunks = 48.8 GiB) resident in HBM per GPU (at 8
GPUs config 4: 1,000,000 chunks = 15,625 stripes per GPU); one step
= one pass of the parity kernel over all stripes (xor_stream<8,U>,
the reference's xor_parity, task_processing.c:96-109, batched).
`--mode rebuild` times config 3 instead (7 survivors + parity body ->
rebuilt chunk; a uniform descriptor batch, so the same streaming kernel in
its pointer-table form).  `--mode mixed` times the config-5 chunk shapes
device-resident: 8-wide stripes with seeded log-uniform chunk lengths in
[64 KiB, 4 MiB] (not 16-byte multiples) at 256-byte-aligned offsets, zero
padding to the stripe maximum (descriptor kernel xor_desc); algorithmic bytes
per stripe = sum of lengths + max length (padding is not read).

value = algorithmic bytes of all ranks / max-over-ranks wall time, with
algorithmic bytes = sum of source lengths + output length per stripe
((N+1) x 512 KiB = 4,718,592 B for config 2).  N>1 (torchrun): each rank owns
its own stripe shard on its own GPU (no data-path collective; gloo only for
the start barrier and the max-time reduction), scaling "weak".  `--gpus N`
without a launcher starts the N ranks itself (a torchrun child process, before
any HIP call) and relays rank 0's line and the exit code; it refuses when the
ranks would share GPUs unless --allow-shared.

roofline.achieved / frac (= frac_event) use the kernel's HIP-event time on the
stream it runs on (an event pair at every step boundary: kernel_ms is the
average, kernel_ms_median / min / max / steps the per-launch spread);
frac_rocprof and traffic come from a live profile on this box (rank 0, after
the timing: the same workload under rocprofv3 in child processes -- kernel
trace + stats over the parent's warm-up and steps, of which the timed
dispatches alone are averaged, then --pmc FETCH_SIZE and --pmc WRITE_SIZE in
runs of their own; roofline.live_profile, same_box true), or, with
--no-prof or when a child run fails, from the committed profile set of the
same workload (profiles/CURRENT_SET, profiles/**/*pmc*.json,
tools/pmc_summary.py), reported beside it as roofline.committed_set.
n_gpus counts DISTINCT devices (PCI bus ids gathered over gloo): ranks that
share a GPU are flagged shared_gpu instead of being reported as more GPUs.
cpu_baseline (every N and every mode): after the device timing and its
verification, rank 0 times the reference's OWN xor_parity
(task_processing.c:96-109 compiled unchanged -std=gnu99 -Os into oracle/_ref,
kind "reference"; the oracle's restatement, kind "port", where _ref was not
built) on a bounded sample of the same stripe shapes -- mixed mode: each stripe
one window of max_cs per source, zero-padded rows, as the reference's P role
folds them -- while the other ranks wait at a gloo barrier.  Legs at 1 thread
and at the CPUs this process may really use (affinity capped by the cgroup CPU
quota, /sys/fs/cgroup/cpu.max; the quota is stated); value = the faster leg.
e2e (every N, out of `value`): each rank then runs the batched pipeline on its
own GPU over its own store of chunk files in /dev/shm (config-5 shapes, about
--e2e-gib GiB per rank, created and removed by the rank): gen (cold + warm
runs) and the rebuild of one lost target, all ranks at once, sampled parity
files and rebuilt chunks checked with numpy; rates against the H2D link each
rank measures over pinned memory at the same time; then config 5's
changelog-driven partial update on the same store (e2e.partial).
configs (BASELINE configs[0] and [4] as BASELINE states them): config1 -- rank
0 runs config 1 end to end (4 loopback storage-target ranks, 3-wide stripes,
1,333 x 512 KiB files) through the per-task protocol with the reference's own
xor_parity as the P-role fold (the cpu_baseline leg's library, kind
"reference"), with the GPU fold, and through the pipeline, gen and rebuild, on
one store in one process; config5_partial -- the e2e block's partial round.
The output is verified after timing: cleared, one more step, then fold
conservation plus sampled stripes compared byte for byte with numpy.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))

import bcp_ctypes as bcp  # noqa: E402
from bcp_dist import Dist, shard_range  # noqa: E402

KiB = 1024
GiB = 1024 ** 3
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md chip table
METRIC = "GiB/s device-resident XOR parity, 512 KiB chunks, 8-wide stripe; % HBM peak"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["gen", "rebuild", "mixed"], default="gen")
    ap.add_argument("--stripes", type=int, default=0,
                    help="stripes per GPU (default: 12,500 = config 2; at 8 GPUs 15,625 = config 4's 1M chunks)")
    ap.add_argument("--nsrc", type=int, default=8)
    ap.add_argument("--rebuild-layout", choices=["packed", "split"], default="packed",
                    help="rebuild inputs per stripe: packed as the pipeline stages them, or split over two arrays")
    ap.add_argument("--chunk", type=int, default=512 * KiB)
    ap.add_argument("--blocks-per-cu", type=int, default=0)
    ap.add_argument("--vecs", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0, help="explicit workgroup count of the streaming kernel (A/B)")
    ap.add_argument("--contig", action="store_true", help="physically contiguous device allocations (A/B knob)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="engine option (bcp_set_option) for A/B runs; repeatable")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget over its legs")
    ap.add_argument("--cpu-stripes", type=int, default=256, help="stripes in the 1-thread CPU sample pool")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e-gib", type=float, default=2.0, help="chunk bytes per rank in the end-to-end store")
    ap.add_argument("--e2e-reps", type=int, default=3, help="warm end-to-end gen runs (after one cold run)")
    ap.add_argument("--e2e-dir", default="/dev/shm", help="where the end-to-end stores are created")
    ap.add_argument("--e2e-max-s", type=float, default=150.0, help="wall-time cap of the end-to-end leg")
    ap.add_argument("--e2e-modes", default="copy,direct",
                    help="pipeline read paths timed end to end, interleaved; the first is the headline")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the config-1 protocol leg (rank 0)")
    ap.add_argument("--c1-files", type=int, default=1333, help="config 1: files (3 chunks of 512 KiB each)")
    ap.add_argument("--c1-reps", type=int, default=7, help="config 1: warm rounds per leg (after one cold round)")
    ap.add_argument("--no-prof", action="store_true",
                    help="skip the live rocprofv3 kernel-trace and PMC passes of this workload on this box")
    ap.add_argument("--allow-shared", action="store_true",
                    help="run N ranks even when fewer than N distinct GPUs exist (rehearsal; "
                         "the line then says shared_gpu true and counts distinct GPUs)")
    return ap.parse_args()


def box_of(pci_bus_id: str) -> dict:
    """The machine this process runs on -- so figures measured on different
    boxes read as such: the kernel's boot id (one per host boot; container host
    names are not unique on this pool), the GPU's unique id and PCI bus id, the
    CPU model and the host name."""
    import socket

    def read(path):
        try:
            return open(path).read().strip() or None
        except OSError:
            return None
    model = ""
    try:
        model = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    bus = (pci_bus_id or "").lower()
    return {"boot_id": read("/proc/sys/kernel/random/boot_id"),
            "gpu_unique_id": read(f"/sys/bus/pci/devices/{bus}/unique_id") if bus else None,
            "pci_bus_id": pci_bus_id, "cpu_model": model, "host": socket.gethostname()}


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpus(nodes_dir: str = KFD_NODES, dri_dir: str = "/dev/dri", env=None) -> int:
    """GPUs this process could use, counted WITHOUT touching HIP: KFD topology
    nodes with a non-zero gfx_target_version whose render node exists here and
    is read-write (a container sees every node of the host in sysfs but only
    its own render nodes), capped by ROCR_/HIP_/CUDA_VISIBLE_DEVICES when set."""
    env = os.environ if env is None else env
    n = 0
    for p in sorted(glob.glob(os.path.join(nodes_dir, "*", "properties"))):
        kv = {}
        try:
            for line in open(p):
                k, _, v = line.strip().partition(" ")
                kv[k] = v
        except OSError:
            continue
        try:
            gfx, minor = int(kv.get("gfx_target_version", "0")), int(kv.get("drm_render_minor", "0"))
        except ValueError:
            continue
        dri = os.path.join(dri_dir, f"renderD{minor}")
        if gfx > 0 and minor > 0 and os.access(dri, os.R_OK | os.W_OK):
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


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


def launch_ranks(a) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): run N ranks,
    one process per GPU, as a torchrun CHILD process and return its exit code.
    This parent never touches HIP or torch: the GPUs are counted from KFD
    sysfs (kfd_gpus).  Refuses (rc 4) when fewer than N GPUs are visible,
    unless --allow-shared; the ranks check the distinct PCI bus ids themselves too."""
    import socket
    import subprocess
    if not a.allow_shared:
        ndev = kfd_gpus()
        if ndev < a.gpus:
            print(f"bench.py: --gpus {a.gpus} but {ndev} GPU(s) visible; refusing to report "
                  f"{a.gpus} GPUs (pass --allow-shared to rehearse with shared devices)", file=sys.stderr)
            return 4
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


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


def live_profile(a, stripes_arg: int, kernel_tag: str, bytes_per_step: int) -> dict:
    """The same workload on THIS box, now, under rocprofv3 (rank 0, after the
    device timing): one kernel-trace + stats run and the two PMC passes
    (FETCH_SIZE, WRITE_SIZE: counters in runs of their own, as
    MI355X_MICROARCH.md's HBM recipe prescribes), each a child process
    `rocprofv3 ... -- python3 bench.py <same workload> --no-e2e --no-cpu
    --no-prof --no-configs` under its own time limit; HBM bytes per launch with
    the gfx950 corrections of tools/pmc_summary.py (FETCH_SIZE x2, KiB).  So
    the line's frac_rocprof and traffic come from the machine its frac_event
    does.  The kernel-trace child runs the parent's --warmup and --steps; its
    timed launches -- the dispatches after the warm-up ones, before the
    verification one -- are the rocprof figure, and the child's own per-step
    HIP events time those SAME launches (child_event_ms), so the two clocks
    are compared on one launch set in one process."""
    import csv
    import shutil
    import signal
    import statistics
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"skipped": "rocprofv3 not on PATH"}
    t0 = time.perf_counter()
    out = tempfile.mkdtemp(prefix="bcp_bench_prof_")
    child = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--mode", a.mode, "--stripes", str(stripes_arg),
             "--nsrc", str(a.nsrc), "--chunk", str(a.chunk), "--rebuild-layout", a.rebuild_layout,
             "--no-cpu", "--no-e2e", "--no-prof", "--no-configs"]
    for flag, val in (("--blocks-per-cu", a.blocks_per_cu), ("--vecs", a.vecs), ("--grid", a.grid)):
        if val:
            child += [flag, str(val)]
    if a.contig:
        child.append("--contig")
    for kv in a.opt:
        child += ["--opt", kv]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT") and not k.startswith("TORCHELASTIC")}

    child_line = {}

    def run(tag, args, steps, warmup):
        d_ = os.path.join(out, tag)
        cmd = ([exe] + args + ["-d", d_, "-o", "run", "--output-format", "csv", "--"] if args is not None else []) + \
            child + ["--steps", str(steps), "--warmup", str(warmup)]
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                             start_new_session=True)
        try:
            so, err = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            raise RuntimeError(f"rocprofv3 {tag}: time limit")
        if p.returncode:
            raise RuntimeError(f"rocprofv3 {tag}: exit {p.returncode}: {err[-300:]}")
        lines = [x for x in so.splitlines() if x.startswith("{")]
        if lines:
            child_line[tag] = json.loads(lines[-1])
        return d_

    def one(d_, pattern):
        hits = sorted(glob.glob(os.path.join(d_, "**", pattern), recursive=True))
        if not hits:
            raise RuntimeError(f"no {pattern} under {d_}")
        return hits[-1]

    def counter(path, name):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if r["Counter_Name"] == name and kernel_tag in r["Kernel_Name"]]
        if not vals:
            raise RuntimeError(f"no {name} rows for {kernel_tag}")
        return statistics.median(vals), len(vals)

    try:
        steps = max(1, min(a.steps, 63))
        d_trace = run("trace", ["--kernel-trace", "--stats"], steps, a.warmup)
        stats = one(d_trace, "*kernel_stats.csv")
        row = next((r for r in csv.DictReader(open(stats)) if kernel_tag in r["Name"]), None)
        if row is None:
            raise RuntimeError(f"{kernel_tag} not in the kernel statistics")
        # the timed dispatches: after the warm-up ones, before the verification one
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                for r in sorted(csv.DictReader(open(one(d_trace, "*kernel_trace.csv"))), key=lambda r: int(r["Dispatch_Id"]))
                if kernel_tag in r["Kernel_Name"]]
        timed = durs[a.warmup:a.warmup + steps]
        if len(timed) != steps or len(durs) != a.warmup + steps + 1:
            raise RuntimeError(f"{len(durs)} dispatches of {kernel_tag}, expected {a.warmup} + {steps} + 1")
        cl = child_line.get("trace", {}).get("roofline", {})
        ev = cl.get("kernel_ms_steps")
        # the same child without the profiler: whether a process-to-process
        # difference or the profiler sets the gap to the parent's events
        run("plain", None, steps, a.warmup)
        plain = child_line.get("plain", {}).get("roofline", {}).get("kernel_ms_median")
        fetch, nf = counter(one(run("pmc_fetch", ["--pmc", "FETCH_SIZE"], 3, 1), "*counter_collection.csv"), "FETCH_SIZE")
        write, nw = counter(one(run("pmc_write", ["--pmc", "WRITE_SIZE"], 3, 1), "*counter_collection.csv"), "WRITE_SIZE")
        traffic = fetch * 1024 * 2 + write * 1024
        avg_t = statistics.fmean(timed)
        return {"rocprof_avg_ns": round(avg_t, 1), "rocprof_median_ns": float(statistics.median(timed)),
                "rocprof_min_ns": float(min(timed)), "rocprof_max_ns": float(max(timed)),
                "rocprof_timed_launches": len(timed),
                "rocprof_all_dispatches": {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"])},
                "child_event_ms_median": (round(statistics.median(ev), 4) if ev else None),
                "child_event_over_rocprof": (round(statistics.median(ev) * 1e6 / statistics.median(timed), 4)
                                             if ev else None),
                "child_event_ms_steps": ev,
                "plain_child_event_ms_median": plain,
                "rocprof_timed_ms_steps": [round(x / 1e6, 4) for x in timed],
                "traffic": round(traffic),
                "traffic_over_algorithmic": round(traffic / bytes_per_step, 5),
                "dispatches": {"fetch": nf, "write": nw},
                "source": "live: rocprofv3 --kernel-trace --stats, then --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate "
                          "child runs of this workload on this box); FETCH_SIZE x2 (gfx950 wide-read correction), "
                          "WRITE_SIZE x1; KiB->B x1024",
                "wall_s": round(time.perf_counter() - t0, 1)}
    except Exception as e:  # reported, never fatal: the committed set stands in
        return {"error": f"{type(e).__name__}: {e}", "wall_s": round(time.perf_counter() - t0, 1)}
    finally:
        shutil.rmtree(out, ignore_errors=True)


def cpu_baseline(a, N: int, C: int, lens_all) -> dict:
    """The reference CPU path on this box's host cores (rank 0, after the
    device timing): its own xor_parity over a bounded sample of the timed
    workload's stripe shapes, at 1 thread and at usable_cpus() threads."""
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


def default_stripes(world: int, rank: int) -> int:
    """Stripes per GPU without --stripes: config 2's 12,500 (100k chunks per
    GPU) up to 4 GPUs; at 8 GPUs config 4 -- 1,000,000 chunks = 125,000
    stripes sharded contiguously, 15,625 per GPU (bcp_dist.shard_range)."""
    if world == 8:
        lo, hi = shard_range(125_000, world, rank)
        return hi - lo
    return 12_500


def gen_config_label(world: int, stripes: int) -> str:
    """The BASELINE config a gen line measures: config 4 exactly when 8 ranks
    each run config 4's 15,625-stripe shard, else config 2."""
    return "config4" if world == 8 and stripes == 15_625 else "config2"


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
    """The config-1 protocol's GPU fold shape with nothing else: `lanes` queues
    (threads), each launching one stripe of `nsrc` x `chunk` bytes that lives
    in pinned HOST memory and waiting for it (bcp_xor_stripes_async reads the
    rows in place across PCIe and writes the parity into pinned host memory,
    as the P role's fold does).  Returns the chunk bytes read per second and
    (read + written) GiB/s (tools/exp/zero_copy_probe.py has the sweep)."""
    import threading
    eng = bcp.Engine(device)
    rows = eng.host_alloc(stripes * nsrc * chunk)
    outs = eng.host_alloc(stripes * chunk)
    qs = [eng.queue() for _ in range(lanes)]
    per = stripes // lanes

    def lane(i):
        q = qs[i]
        for s in range(i * per, (i + 1) * per):
            q.xor_stripes([(outs + s * chunk, chunk, 0, nsrc, 0)],
                          [(rows + (s * nsrc + j) * chunk, chunk) for j in range(nsrc)])
            q.sync()

    try:
        best = None
        for _ in range(3):
            ths = [threading.Thread(target=lane, args=(i,)) for i in range(lanes)]
            t0 = time.perf_counter()
            for t in ths:
                t.start()
            for t in ths:
                t.join()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
    finally:
        for q in qs:
            q.close()
        eng.host_free(rows)
        eng.host_free(outs)
        eng.close()
    n = per * lanes
    return {"read_GBps": round(n * nsrc * chunk / best / 1e9, 2),
            "GiBps": round(n * (nsrc + 1) * chunk / best / GiB, 2), "lanes": lanes, "stripes": n}


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

    legs = ["reference_fold", "gpu_fold", "pipeline"]
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
        pl = bcp.Pipeline(device=device)
        runs = 1 + max(1, a.c1_reps)
        for r in range(runs):
            for leg in legs[r % 3:] + legs[:r % 3]:
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
                for leg in legs[r % 3:] + legs[:r % 3]:
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
        "pipeline_over_reference_fold": round(gen["pipeline"]["GiBps"] / gen["reference_fold"]["GiBps"], 3),
        "rebuild_gpu_fold_over_reference_fold": round(reb["gpu_fold"]["GiBps"] / reb["reference_fold"]["GiBps"], 3),
        # every chunk byte a GPU fold folds crosses the host-to-device link once (parity comes back
        # on the other direction): the gen rate it cannot pass on this link
        "link": link,
        "gpu_fold_link_ceiling_GiBps": (round((rd + wr) / (rd / (link["h2d_GBps"] * 1e9)) / GiB, 2)
                                        if link.get("h2d_GBps") else None),
        # ... and what the device folds of rows in pinned host memory reach in the protocol's shape
        # (12 lanes, one stripe per launch, read in place), the fold alone: the GPU fold's own bound
        "gpu_fold_in_place_bound": zc,
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

    def chunk_of(i, k):
        off = ((i * W + k) * 40961) % (8 << 20)
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
                st, nplanned = pl.round(rank_root, NT, es, cum_weight=[1000 * (k + 1) for k in range(NT)])
            finally:
                es.close()
            return (time.perf_counter() - t0, st.seconds, nplanned == len(sub) and st.errors == 0 and st.tasks == len(sub),
                    pl.last_timing())

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
        return {"stripes": len(sub), "bytes_read": sum(int(lens[i].sum()) for i in sub),
                "bytes_written": sum(8 * W + int(lens[i].max()) for i in sub),
                "own_runs_s": [round(x, 4) for x in times], "own_warm_s": round(float(np.median(times[1:])), 4),
                "own_pipeline_warm_s": round(float(np.median([x[1] for x in runs_p][1:])), 4),
                "pipeline_timing_last": runs_p[-1][3],
                "plan_ok": bool(plan_ok), "verified": bool(verified)}

    pls = {}
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
                "pipeline_warm_s_rank0": ps[0]["own_pipeline_warm_s"],
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
        "link_h2d_GBps_sum": round(h2d_all / 1e9, 2),
        "errors": all_errors or None,
        "rate_note": "GiBps = (chunk bytes read + parity bytes written) of all ranks / the slowest rank's warm "
                     "run (median); input_over_link = input bytes / that time / the summed H2D rates the ranks "
                     "measured together over pinned memory; timing = rank 0's host-thread stages (seconds)",
        "wall_s": round(time.perf_counter() - t_start, 1),
        "per_rank": ranks,
    }

def main():
    a = parse()
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    d = Dist()
    if d.world != a.gpus and d.rank == 0:
        print(f"bench.py: note: launched with {d.world} ranks for --gpus {a.gpus}; "
              f"the line reports the ranks and distinct GPUs actually used", file=sys.stderr)
    ndev = bcp.device_count()
    assert ndev > 0, "bench.py needs a HIP device (there is no CPU path)"
    eng = bcp.Engine(d.local_rank % ndev)
    # physical GPUs in the job: ranks that map to the same device share it
    bus_ids = d.gather(eng.pci_bus_id())
    n_devices = len(set(bus_ids))
    shared_gpu = n_devices < d.world
    if shared_gpu and not a.allow_shared:
        if d.rank == 0:
            print(f"bench.py: {d.world} ranks but only {n_devices} distinct GPU(s) (PCI bus ids "
                  f"{sorted(set(bus_ids))}); refusing (pass --allow-shared to rehearse)", file=sys.stderr)
        eng.close()
        d.close()
        sys.exit(4)
    if a.mode == "mixed":  # the timed kernel is the descriptor kernel
        if a.blocks_per_cu:
            eng.option("desc_blocks_per_cu", a.blocks_per_cu)
        if a.vecs:
            eng.option("desc_vecs_per_thread", a.vecs)
    elif a.blocks_per_cu or a.vecs:
        eng.tune(a.blocks_per_cu, a.vecs)
    if a.grid:
        eng.option("stream_grid", a.grid)
    if a.contig:
        eng.option("contiguous_alloc", 1)
    for kv in a.opt:
        k, v = kv.split("=")
        eng.option(k, int(v))
    cus, devname = eng.info()
    q = eng.queue()
    # config 2 (100k chunks per GPU) up to 4 GPUs; at 8 GPUs config 4: 1,000,000
    # chunks = 125,000 stripes sharded 15,625 per GPU (bcp_dist.shard_range)
    if not a.stripes:
        a.stripes = default_stripes(d.world, d.rank)
    stripes_arg = a.stripes
    S, N, C = a.stripes, a.nsrc, a.chunk
    chk = eng.alloc(64)
    lens_all = None
    if a.mode == "mixed":
        import numpy as np
        rng = np.random.default_rng(3 + d.rank)
        # log-uniform lengths; as many stripes as fit the config-2 input volume
        budget = S * N * C
        lens_all, tot = [], 0
        while tot < budget:
            ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=N)).astype(np.int64)
            lens_all.append(ls)
            tot += int(ls.sum())
        align = lambda x: (x + 255) & ~255
        src_bytes = sum(int(sum(align(int(x)) for x in ls)) for ls in lens_all)
        out_bytes = sum(align(int(ls.max())) for ls in lens_all)
        src = eng.alloc(src_bytes)
        out = eng.alloc(out_bytes)
    else:
        src = eng.alloc(S * N * C)
        out = eng.alloc(S * C)
        src_bytes = S * N * C
    q.fill_synthetic(src, src_bytes, seed=1 + d.rank)

    if a.mode == "mixed":
        stripes, sources, so_off, do_off = [], [], 0, 0
        for ls in lens_all:
            first = len(sources)
            for x in ls:
                sources.append((src + so_off, int(x)))
                so_off += align(int(x))
            m = int(ls.max())
            stripes.append((out + do_off, m, first, N, 0))
            do_off += align(m)
        st = (bcp.Stripe * len(stripes))(*[bcp.Stripe(*x) for x in stripes])
        so = (bcp.Source * len(sources))(*[bcp.Source(*x) for x in sources])
        L = bcp.lib()

        def step():
            bcp.check("bcp_xor_stripes_async", L.bcp_xor_stripes_async(q.h, st, len(stripes), so, len(sources)))
        bytes_per_step = sum(int(ls.sum()) + int(ls.max()) for ls in lens_all)
        S = len(stripes)
        U = 0  # read back after the timed launches (auto tile size)
        pipe = 0
        kernel = f"xor_desc_p<{U},{pipe}>" if pipe else f"xor_desc<{U}>"
        kernel_tag = f"xor_desc_p<{U}, {pipe}>" if pipe else f"xor_desc<{U}>"
        workload = (f"config5 shapes: {S} stripes x {N} chunks, log-uniform 64 KiB-4 MiB, "
                    f"zero-padded to the stripe max, device-resident")
    elif a.mode == "gen":
        def step():
            q.xor_uniform(out, src, S, N, C)
        bytes_per_step = S * (N + 1) * C
        kernel = "xor_stream<{N},{U},strided>"
        kernel_tag = "xor_stream<{N}, {U}, 0, "
        cfg = gen_config_label(d.world, S)
        workload = f"{cfg}: parity gen, {S} stripes x {N} x {C // KiB} KiB device-resident per GPU"
    else:
        # config 3: parity first, then rebuild source index 3 from the other
        # N-1 chunks + parity body.  Layout "packed" (default): each stripe's
        # inputs staged contiguously as bcp_pipeline_rebuild stages them in its
        # slab (survivors and the parity body in ascending target order, here
        # the parity body in the lost chunk's slot); "split": survivors read in
        # place from the gen source array + parity bodies from a second array.
        par = eng.alloc(S * C)
        q.xor_uniform(par, src, S, N, C)
        victim = min(3, N - 1)
        stripes, sources = [], []
        if a.rebuild_layout == "packed":
            rin = eng.alloc(S * N * C)
            q.d2d(rin, src, S * N * C)
            q.xor_strided(rin + victim * C, N * C, par, C, C, S, 1, C)  # parity body -> the lost slot
            for s in range(S):
                first = len(sources)
                for k in range(N):
                    sources.append((rin + (s * N + k) * C, C))
                stripes.append((out + s * C, C, first, N, 0))
        else:
            for s in range(S):
                first = len(sources)
                for k in range(N):
                    if k != victim:
                        sources.append((src + (s * N + k) * C, C))
                sources.append((par + s * C, C))
                stripes.append((out + s * C, C, first, N, 0))
        import ctypes
        st = (bcp.Stripe * len(stripes))(*[bcp.Stripe(*x) for x in stripes])
        so = (bcp.Source * len(sources))(*[bcp.Source(*x) for x in sources])
        L = bcp.lib()

        def step():
            bcp.check("bcp_xor_stripes_async", L.bcp_xor_stripes_async(q.h, st, len(stripes), so, len(sources)))
        bytes_per_step = S * (N + 1) * C
        kernel = "xor_stream<{N},{U},gather>"
        kernel_tag = "xor_stream<{N}, {U}, 1, "
        workload = (f"config3: rebuild, {S} stripes x ({N - 1} survivors + parity) x {C // KiB} KiB device-resident, "
                    f"{a.rebuild_layout} layout")

    for _ in range(a.warmup):
        step()
    q.sync()

    # one HIP event per step boundary on the kernel's stream (BCP_TIMER_SLOTS
    # = 64 slots: beyond 63 steps, boundaries every g steps), so the line
    # carries the per-launch spread, not only the block's average
    g = -(-a.steps // 63)
    bounds = list(range(0, a.steps, g)) + [a.steps]
    d.barrier()
    q.sync()
    t0 = time.perf_counter()
    q.mark(0)
    for i in range(a.steps):
        step()
        if (i + 1) in bounds:
            q.mark(bounds.index(i + 1))
    q.sync()
    t1 = time.perf_counter()
    d.barrier()
    wall = t1 - t0
    seg_ms = [q.elapsed_ms(j, j + 1) / (bounds[j + 1] - bounds[j]) for j in range(len(bounds) - 1)]
    kern_ms = q.elapsed_ms(0, len(bounds) - 1) / a.steps  # avg launch duration on the kernel's stream
    if a.mode == "mixed":  # the descriptor kernel's form and tile size of the timed launches
        U = eng.option("last_desc_vecs")
        pipe = 5 if U >= 8 else 0  # the rolling-window form at U = 8 and 16 (launch_xor_desc)
        if eng.option("last_desc_form") == 2:
            kernel, kernel_tag = f"xor_desc_args<{U}>", f"xor_desc_args<{U}>"
        else:
            kernel = f"xor_desc_p<{U},{pipe}>" if pipe else f"xor_desc<{U}>"
            kernel_tag = f"xor_desc_p<{U}, {pipe}>" if pipe else f"xor_desc<{U}>"
    if a.mode != "mixed":  # tile size the engine chose for the timed launches
        U = eng.option("last_stream_vecs")
        # register-budget (W = 6) instantiations (launch_xor_stream in bcp_kernels.hip)
        budget = (N == 8 and U == 8) or (a.mode == "gen" and ((5 <= N <= 7 and U == 8) or
                                                              (N in (9, 10, 11, 12, 16) and U == 4)))
        if budget:
            form, gather = ("gather", 1) if a.mode == "rebuild" else ("strided", 0)
            kernel = "xor_stream_w<{N},{U},%s,wpe6>" % form
            kernel_tag = "xor_stream_w<{N}, {U}, %d, 0, 6>" % gather
        NS = N if (1 <= N <= 12 or N == 16) else 0  # widths without a specialisation run xor_stream<0, ...>
        kernel, kernel_tag = kernel.format(N=NS, U=U), kernel_tag.format(N=NS, U=U)

    # Verification after the timed region: clear the output, run ONE more
    # step, then check it on the device (fold conservation / rebuild compare)
    # and sampled stripes byte for byte against numpy (not the oracle).
    import numpy as np
    q.memset(out, 0xA5, out_bytes if a.mode == "mixed" else S * C)
    step()
    q.sync()
    rng = np.random.default_rng(7 + d.rank)

    def sampled(idx, fetch_inputs, out_ptr, out_len):
        ok = True
        for i in idx:
            ins = fetch_inputs(i)
            ref = np.zeros(out_len, dtype=np.uint8)
            for buf in ins:
                ref[:len(buf)] ^= buf[:out_len]
            got = np.empty(out_len, dtype=np.uint8)
            q.d2h(got, out_ptr(i), out_len)
            q.sync()
            ok = ok and bool(np.array_equal(got, ref))
        return ok

    def dget(ptr, n):
        buf = np.empty(n, dtype=np.uint8)
        q.d2h(buf, ptr, n)
        q.sync()
        return buf

    verified = None
    if a.mode == "mixed":
        ok = True
        for i in sorted({0, len(stripes) - 1, len(stripes) // 2} | {int(x) for x in rng.integers(0, len(stripes), 3)}):
            dptr, m, first, n, _ = stripes[i]
            ok = ok and sampled([i], lambda i: [dget(*sources[first + k]) for k in range(n)], lambda i: dptr, m)
        verified = ok
    elif a.mode == "gen":
        q.xor_fold(out, S * C, chk)
        q.xor_fold(src, S * N * C, chk + 16)
        f = dget(chk, 32)
        idx = sorted({0, S - 1} | {int(x) for x in rng.integers(0, S, 4)})
        verified = bool(np.array_equal(f[:16], f[16:])) and sampled(
            idx, lambda i: [dget(src + (i * N + k) * C, C) for k in range(N)], lambda i: out + i * C, C)
    else:
        victim = min(3, N - 1)
        gathered = eng.alloc(S * C)
        q.xor_strided(gathered, C, src + victim * C, N * C, C, S, 1, C)
        q.compare(out, gathered, S * C, chk)
        f = dget(chk, 8)
        idx = sorted({0, S - 1} | {int(x) for x in rng.integers(0, S, 4)})
        verified = int(f.view("<u8")[0]) == 0 and sampled(
            idx, lambda i: [dget(src + (i * N + victim) * C, C)], lambda i: out + i * C, C)

    wall_max = d.max(wall)
    total_bytes = d.sum(float(bytes_per_step * a.steps))
    ok_all = d.sum(1.0 if verified else 0.0) == d.world
    kern_ms_max = d.max(kern_ms)
    # every rank's own figures (per-GPU rates of the N-GPU line): bus id, HIP-event
    # kernel time, its share of the wall clock
    import statistics
    seg_med = statistics.median(seg_ms)
    per_rank = d.gather({"rank": d.rank, "pci_bus_id": bus_ids[d.rank], "kernel_ms": round(kern_ms, 4),
                         "kernel_ms_median": round(seg_med, 4), "kernel_ms_min": round(min(seg_ms), 4),
                         "kernel_ms_max": round(max(seg_ms), 4),
                         "GiBps": round(bytes_per_step * a.steps / wall / GiB, 2),
                         "pct_hbm_peak": round(100.0 * bytes_per_step / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 2),
                         "verified": bool(verified)})

    # end to end from chunk files (every rank on its own GPU, all at once)
    e2e = None
    if not a.no_e2e:
        q.sync()
        e2e = e2e_leg(a, d, eng.device, bus_ids[d.rank])
    # the reference CPU path, rank 0 only, after every device figure; the
    # other ranks wait at the barrier
    cpu = None
    if d.rank == 0 and not a.no_cpu:
        try:
            cpu = cpu_baseline(a, N, C, lens_all if a.mode == "mixed" else None)
        except Exception as e:  # a reported baseline: never worth the device line
            cpu = {"error": f"{type(e).__name__}: {e}"}
    # BASELINE config 1 end to end (rank 0; the reference's xor_parity as the
    # P-role fold beside the GPU fold and the pipeline, same store)
    c1 = None
    if d.rank == 0 and not a.no_configs:
        try:
            c1 = config1_leg(a, eng.device)
        except Exception as e:  # reported, never worth the device line
            c1 = {"error": f"{type(e).__name__}: {e}"}
    # rocprofv3 on this box: rank 0's device, child processes (the device
    # buffers of this run are released first)
    live = None
    if d.rank == 0 and not a.no_prof:
        for ptr in (src, out):
            eng.free(ptr)
        src = out = None
        live = live_profile(a, stripes_arg, kernel_tag, bytes_per_step)
    d.barrier()

    if d.rank == 0:
        value = total_bytes / wall_max / GiB
        achieved = bytes_per_step / (kern_ms_max * 1e-3) / 1e9
        mode_key = "rebuild_packed" if (a.mode == "rebuild" and a.rebuild_layout == "packed") else a.mode
        wkey = f"{mode_key}:{S}x{N}x{C}"
        pmc = pmc_traffic(wkey, kernel_tag)
        run_box = box_of(bus_ids[0])
        live_ok = bool(live and live.get("traffic"))
        frac_rocprof = None
        if live_ok:
            frac_rocprof = round(bytes_per_step / (live["rocprof_avg_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
        elif pmc and (pmc.get("rocprof_timed_avg_ns") or pmc.get("rocprof_avg_ns")):
            frac_rocprof = round(bytes_per_step / ((pmc.get("rocprof_timed_avg_ns") or pmc["rocprof_avg_ns"]) * 1e-9)
                                 / 1e9 / HBM_PEAK_GBS, 4)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": n_devices,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(wall_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 stream, seed 1+rank), generated on device",
            "config": {
                "workload": workload,
                "mode": a.mode,
                "stripes_per_gpu": S,
                "nsrc": N,
                "chunk_bytes": C,
                "bytes_per_step_per_gpu": bytes_per_step,
                "data_rate_GiBps": round(value * N / (N + 1), 2) if a.mode != "mixed" else None,
                "pct_hbm_peak": round(100.0 * achieved / HBM_PEAK_GBS, 2),
                # whole job (wall clock, all ranks) against (distinct GPUs) x 8 TB/s
                "pct_aggregate_hbm_peak": round(100.0 * total_bytes / wall_max / 1e9 / (HBM_PEAK_GBS * n_devices), 2),
                "parallelism": f"shard{d.world} (stripes per rank, no collective)",
                "ranks": d.world,
                "shared_gpu": shared_gpu,
                "device": devname,
                "pci_bus_ids": sorted(set(bus_ids)),
                "cus": cus,
                "verified_on_device": ok_all,
                "per_rank": per_rank,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel,
                "kernel_tag": kernel_tag,  # as rocprofv3 names it
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "frac_event": round(achieved / HBM_PEAK_GBS, 4),
                "frac_rocprof": frac_rocprof,
                "kernel_ms": round(kern_ms_max, 4),
                # rank 0's per-launch spread (HIP event pairs at every step boundary)
                "kernel_ms_median": round(seg_med, 4),
                "kernel_ms_min": round(min(seg_ms), 4),
                "kernel_ms_max": round(max(seg_ms), 4),
                "kernel_ms_steps": [round(x, 4) for x in seg_ms],
                "steps_per_event_pair": g,
                "frac_event_median": round(bytes_per_step / (seg_med * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": (live["traffic"] if live_ok else pmc["hbm_bytes_per_launch"] if pmc else None),
                "traffic_source": (live["source"] if live_ok else pmc["source"] if pmc else None),
                "live_profile": live,
                "profile_files": pmc.get("files") if pmc else None,
                "profile_commit": pmc.get("code_commit") if pmc else None,
                "run_box": run_box,
                "profile_box": run_box if live_ok else (pmc.get("box") if pmc else None),
                "same_box": live_ok or bool(pmc and pmc.get("box") and run_box["boot_id"]
                                            and pmc["box"].get("boot_id") == run_box["boot_id"]),
                "committed_set": ({"frac_rocprof": round(bytes_per_step / ((pmc.get("rocprof_timed_avg_ns") or
                                                                            pmc["rocprof_avg_ns"]) * 1e-9) / 1e9 /
                                                         HBM_PEAK_GBS, 4) if pmc.get("rocprof_avg_ns") else None,
                                   "timed_launches_only": bool(pmc.get("rocprof_timed_avg_ns")),
                                   "traffic": pmc.get("hbm_bytes_per_launch"), "box": pmc.get("box")}
                                  if pmc else None),
                "frac_note": "frac = frac_event: algorithmic bytes / the average HIP-event time of the timed "
                             "launches in this run (run_box; the slowest rank's); frac_event_median and "
                             "kernel_ms_median/min/max/steps: rank 0's event pair per step; frac_rocprof: the same "
                             "bytes / the rocprofv3 kernel-trace average over the timed launches only (warm-up and "
                             "verification dispatches excluded) of a live child run of this workload with this "
                             "run's --warmup/--steps on this box, whose own per-step events over those same "
                             "launches are live_profile.child_event_ms_*; traffic: the PMC passes of that child "
                             "workload -- or, where those failed or --no-prof, the committed profile set "
                             "(profile_files, measured on profile_box)",
            },
            "cpu_baseline": (dict(cpu, config1_protocol_reference_fold=(
                {"gen_GiBps": c1["gen"]["reference_fold"]["GiBps"],
                 "rebuild_GiBps": c1["rebuild"]["reference_fold"]["GiBps"], "kind": c1["gen"]["reference_fold"]["kind"],
                 "see": "configs.config1"} if isinstance(c1, dict) and "gen" in c1 else None))
                             if isinstance(cpu, dict) else cpu),
            "per_rank": per_rank,
            "e2e": e2e,
            # BASELINE configs[0] and configs[4] as BASELINE states them (rank 0's config-1 protocol
            # leg; the config-5 changelog subset of every rank's e2e store)
            "configs": {"config1": c1,
                        "config5_partial": (e2e or {}).get("partial") if isinstance(e2e, dict) else None},
        }
        print(json.dumps(line), flush=True)
    q.close()
    eng.close()
    d.close()
    if not ok_all:
        sys.exit(3)


if __name__ == "__main__":
    main()
