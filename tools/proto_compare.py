#!/usr/bin/env python3
"""Per-task protocol (process_task over loopback ranks) with every P-role fold,
interleaved in ONE run on ONE box:

  gpu_pipelined  BCP_FOLD_PIPELINED (default): the fold follows the senders'
                 reads -- each range all rows have delivered is folded (by
                 the source that completed it) while the rest is read; the P
                 role folds the tail and waits.  Since r06 through the
                 device's resident fold ring (= gpu_ring); gpu_queues: the
                 same with range launches on the lanes' queues (ring off)
  gpu_batched[K] BCP_FOLD_BATCHED: the device's fold service batches the
                 pending windows of every lane into one launch (K batches in
                 flight, default 4)
  cpu_reference  the reference fold in libbcp's protocol: the reference's own
                 xor_parity (task_processing.c:96-109 compiled unchanged,
                 oracle/_ref ref_xor_rows; the restatement oracle_xor_rows
                 where _ref was not built -- the line says which) over the
                 whole window once every row has arrived, with the senders on
                 the reference's zero-padded wire.  Not the reference PROGRAM:
                 its roles need MPI; the protocol around the fold is libbcp's
  cpu_pipelined  the restated CPU fold (oracle_xor_rows) inside this
                 protocol's pipelined P role: the source threads fold ranges
                 as the rows fill
  noop           a fold that does nothing: the bound of the protocol itself
                 (no parity is correct; not verified)

Workloads: config 1 (4 targets, 1333 x 3-wide 512 KiB stripes, 12 lanes; gen,
and rebuild of target 2 with the single rebuild lane) and config 5 (9
targets, 8-wide stripes of log-uniform 64 KiB-4 MiB chunks, 12 lanes).
Rate = (chunk bytes read + parity bytes written) / wall; each round runs
every fold once in a rotating order, medians over rounds after a cold one.
Parity of the GPU and CPU runs is checked against the oracle on a sample.
--procs: every storage target's rank is its own PROCESS (socketpair
transport), kept alive across runs in a rank pool (bcp_rank_pool_*: HIP init
and row registration paid once per rank, as by a long-lived job's ranks);
--procs-cold forks fresh ranks for every run (bcp_gen_run_procs /
bcp_rebuild_run_procs).  This process never touches the GPU then (the ranks
create their own HIP contexts), and the per-phase and fold-service counters
live in the ranks (not reported).
One JSON line per (workload, fold); tools only.
"""
import argparse
import ctypes
import json
import os
import resource
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402  (checker + the reference CPU fold)
from e2e_bench import total_bytes, verify, write_store  # noqa: E402

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3


def emit(**kw):
    print(json.dumps(kw), flush=True)


def noop_hook():
    tmp = tempfile.mkdtemp(dir="/tmp")  # /dev/shm may be noexec
    src = os.path.join(tmp, "noop.c")
    open(src, "w").write("#include <stddef.h>\n#include <stdint.h>\nint noop_fold(uint8_t *d, size_t n, const uint8_t"
                         " *s, size_t p, int k, void *c) { (void)d; (void)n; (void)s; (void)p; (void)k; (void)c;"
                         " return 0; }\n")
    so = os.path.join(tmp, "libnoop.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src], check=True)
    return ctypes.CDLL(so)


def cpu_now():
    """(process CPU seconds over all threads, cgroup throttled periods, throttled us,
    cgroup CPU seconds: every process of the container, rank processes included)."""
    ru = resource.getrusage(resource.RUSAGE_SELF)
    nr = us = 0
    cg = None
    try:
        for ln in open("/sys/fs/cgroup/cpu.stat"):
            k, v = ln.split()
            nr = int(v) if k == "nr_throttled" else nr
            us = int(v) if k == "throttled_usec" else us
            cg = int(v) / 1e6 if k == "usage_usec" else cg
    except OSError:
        pass
    return ru.ru_utime + ru.ru_stime, nr, us, cg


TUNING_KEYS = {"piece": "pipe_piece_kib", "step": "pipe_step_kib", "depth": "defer_depth",
               "completion": "completion_threads", "spin": "lb_spin_us", "workers": "ring_workers"}
# keys whose new value ends the current rings (the next fold makes new ones)
RING_REMAKE = {"ring_workers"}


def fold_setup(fold, hooks):
    """Returns a context restore callable.  <fold>%k=v+k=v: any fold with
    protocol tuning (bcp_task_set_fold_tuning, TUNING_KEYS) around it, e.g.
    cpu_reference%spin=20."""
    if "%" in fold:
        base, tun = fold.split("%", 1)
        olds = [(TUNING_KEYS[k], bcp.set_fold_tuning(TUNING_KEYS[k], int(v)))
                for k, v in (kv.split("=") for kv in tun.split("+"))]
        inner = fold_setup(base, hooks)

        def restore_pct():
            inner()
            for k, v in reversed(olds):
                bcp.set_fold_tuning(k, v)
        return restore_pct
    if fold.startswith("gpu_batched"):
        # gpu_batched[K]: K concurrent batches (bcp_task_set_fold_inflight)
        k = int(fold[len("gpu_batched"):] or 4)
        prev_k = bcp.set_fold_inflight(k)
        prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)

        def restore():
            bcp.set_fold_mode(prev)
            bcp.set_fold_inflight(prev_k)
        return restore
    if fold.startswith("gpu_ring@"):
        # gpu_ring@piece=K+step=K+depth=D+completion=T: the ring with another pipelined shape
        # (bcp_task_set_fold_tuning: KiB per publish, smallest range, lane deferral depth,
        # completion threads)
        keys = TUNING_KEYS
        prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
        prev_ring = bcp.set_fold_ring(True)
        olds = []
        for kv in fold.split("@", 1)[1].split("+"):
            k, v = kv.split("=")
            olds.append((keys[k], bcp.set_fold_tuning(keys[k], int(v))))

        def restore_t():
            for k, v in reversed(olds):
                bcp.set_fold_tuning(k, v)
            bcp.set_fold_ring(prev_ring)
            bcp.set_fold_mode(prev)
        return restore_t
    if fold.startswith("gpu_ring_w"):
        # gpu_ring_w<spin>_<sleep>: the ring with waiters spinning <spin> us,
        # then sleeping <sleep> us between looks (0: sched_yield)
        spin, sleep = (int(x) for x in fold[len("gpu_ring_w"):].split("_"))
        prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
        prev_ring = bcp.set_fold_ring(True)
        bcp.call("bcp_task_set_ring_wait", spin, sleep)

        def restore_w():
            bcp.call("bcp_task_set_ring_wait", 4, 10)
            bcp.set_fold_ring(prev_ring)
            bcp.set_fold_mode(prev)
        return restore_w
    if fold in ("gpu_pipelined", "gpu_ring", "gpu_queues"):
        # gpu_ring / gpu_pipelined: PIPELINED through the resident fold ring
        # (the default since r06); gpu_queues: range launches on the lanes'
        # queues, whole windows by the fold service (bcp_task_set_fold_ring(0))
        prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
        prev_ring = bcp.set_fold_ring(fold != "gpu_queues")

        def restore_pipe():
            bcp.set_fold_ring(prev_ring)
            bcp.set_fold_mode(prev)
        return restore_pipe
    if fold == "cpu_reference":
        prev = bcp.set_fold_mode(bcp.FOLD_BATCHED)  # the hook folds whole windows after every row arrived
        prev_pad = bcp.set_explicit_padding(True)  # the reference's wire
        bcp.set_xor_hook(hooks[fold])

        def restore_ref():
            bcp.set_xor_hook(None)
            bcp.set_explicit_padding(prev_pad)
            bcp.set_fold_mode(prev)
        return restore_ref
    prev = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
    bcp.set_xor_hook(hooks[fold])

    def restore_hook():
        bcp.set_xor_hook(None)
        bcp.set_fold_mode(prev)
    return restore_hook


def measure(name, folds, rounds, run_once, verify_fn, nbytes, hooks, extra=None, prepare=None):
    times = {f: [] for f in folds}
    cpu = {f: [] for f in folds}  # (CPU seconds, throttled periods, throttled ms) per run
    batching = {}
    phases = {}
    for r in range(rounds + 1):
        order = folds[r % len(folds):] + folds[:r % len(folds)]
        for f in order:
            if prepare:
                prepare()  # outside the timed region (removing old parity files)
            restore = fold_setup(f, hooks)
            remake = any(TUNING_KEYS.get(kv.split("=")[0]) in RING_REMAKE
                         for kv in (f.split("@", 1)[1].split("+") if "@" in f else []))
            if remake:  # a new ring: made and launched by one untimed run
                run_once()
                if prepare:
                    prepare()
            try:
                w0, l0 = bcp.fold_stats()
                pw0, pr0 = bcp.pipe_stats()
                bcp.phase_stats(reset=True)
                c0 = cpu_now()
                t0 = time.perf_counter()
                st = run_once()
                dt = time.perf_counter() - t0
                c1 = cpu_now()
                cpu[f].append((c1[0] - c0[0], c1[1] - c0[1], (c1[2] - c0[2]) / 1e3,
                               c1[3] - c0[3] if c0[3] is not None else None))
                w1, l1 = bcp.fold_stats()
                pw1, pr1 = bcp.pipe_stats()
                ph = bcp.phase_stats()
                if r > 0:
                    acc = phases.setdefault(f, {})
                    for k, v in ph.items():
                        acc[k] = acc.get(k, 0) + v
            finally:
                restore()
            if remake:  # the default ring again, made outside the next fold's timing
                if prepare:
                    prepare()
                bcp.set_fold_ring(True)
                prev_mode = bcp.set_fold_mode(bcp.FOLD_PIPELINED)
                run_once()
                bcp.set_fold_mode(prev_mode)
            if st.errors:
                raise RuntimeError(f"{name}/{f}: {st.errors} rank errors")
            times[f].append(dt)
            if f.startswith("gpu_batched") and r > 0:
                b = batching.setdefault(f, {"windows": 0, "launches": 0})
                b["windows"] += w1 - w0
                b["launches"] += l1 - l0
            if (f.split("%")[0] in ("gpu_pipelined", "gpu_ring", "gpu_queues") or f.startswith(("gpu_ring_w", "gpu_ring@"))) \
                    and r > 0:
                b = batching.setdefault(f, {"windows": 0, "launches": 0})
                b["windows"] += pw1 - pw0
                b["launches"] += pr1 - pr0
            if r == rounds and not f.startswith("noop"):
                ok, bad = verify_fn()
                if not ok:
                    raise RuntimeError(f"{name}/{f}: parity mismatch on {bad}")
    res = {}
    for f in folds:
        warm = float(np.median(times[f][1:]))
        res[f] = nbytes / warm / GiB
        line = dict(workload=name, fold=f, GiBps=round(res[f], 3), warm_median_s=round(warm, 4),
                    runs_s=[round(x, 4) for x in times[f]], cold_s=round(times[f][0], 4),
                    cpu_s_median=round(float(np.median([c[0] for c in cpu[f][1:]])), 4),
                    cores_busy_median=round(float(np.median([c[0] / t for c, t in zip(cpu[f][1:], times[f][1:])])), 2),
                    cgroup_cpu_s_median=(round(float(np.median([c[3] for c in cpu[f][1:]])), 4)
                                         if cpu[f][-1][3] is not None else None),
                    throttled_periods=sum(c[1] for c in cpu[f][1:]),
                    throttled_ms_runs=[round(c[2], 1) for c in cpu[f]])
        if (f.split("%")[0] in ("gpu_pipelined", "gpu_ring", "gpu_queues") or f.startswith(("gpu_ring_w", "gpu_ring@"))) \
                and batching.get(f, {}).get("windows"):
            line["range_folds_per_window"] = round(batching[f]["launches"] / batching[f]["windows"], 2)
        elif batching.get(f, {}).get("launches"):
            line["windows_per_launch"] = round(batching[f]["windows"] / batching[f]["launches"], 2)
        acc = phases.get(f)
        if acc and acc.get("p_tasks"):
            # mean wall microseconds per P task / per source task in each phase
            line["p_phase_us"] = {k[2:]: round(acc[k] / acc["p_tasks"] * 1e6, 1) for k in acc
                                  if k.startswith("p_") and k != "p_tasks"}
            line["s_phase_us"] = {k[2:]: round(acc[k] / max(acc["s_tasks"], 1) * 1e6, 1) for k in acc
                                  if k.startswith("s_") and k != "s_tasks"}
        if extra:
            line.update(extra)
        emit(**line)
    if "noop" in res:
        emit(workload=name, summary={f: round(v, 3) for f, v in res.items()},
             frac_of_noop_bound={f: round(v / res["noop"], 3) for f, v in res.items() if not f.startswith("noop")},
             gpu_vs_cpu={f: round(v / res["cpu_reference"], 3) for f, v in res.items() if f.startswith("gpu_")}
             if "cpu_reference" in res else None,
             gpu_vs_cpu_pipelined={f: round(v / res["cpu_pipelined"], 3) for f, v in res.items()
                                   if f.startswith("gpu_")} if "cpu_pipelined" in res else None)
    return res


def reset_parity(root, ntargets):
    for k in range(ntargets):
        shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
        os.makedirs(os.path.join(root, f"st{k}", "parity"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/dev/shm/bcp_proto")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--folds", default="gpu_pipelined,gpu_batched,cpu_reference,cpu_pipelined,noop")
    ap.add_argument("--workloads", default="c1_gen,c1_rebuild,c5_gen")
    ap.add_argument("--c1-files", type=int, default=1333)
    ap.add_argument("--c5-stripes", type=int, default=1000)
    ap.add_argument("--c5-targets", type=int, default=9, help="config 5: storage targets (stripe width min(8, t-1))")
    ap.add_argument("--lanes", type=int, default=12)
    ap.add_argument("--procs", action="store_true", help="ranks as processes kept alive across runs")
    ap.add_argument("--procs-cold", action="store_true", help="ranks as processes forked for every run")
    ap.add_argument("--rebuild-lanes", type=int, default=1,
                    help="lanes per rank of the rebuild (bcp_task_set_rebuild_lanes; 1 = the reference's)")
    ap.add_argument("--fold-server", action="store_true",
                    help="ranks as threads, every GPU fold through a node fold server process on a socket "
                         "(bcp_fold_server_connect: an MPI job's shape)")
    ap.add_argument("--no-gpu", action="store_true", help="CPU folds only (cpu_*, noop): no link probe, runs without a GPU")
    a = ap.parse_args()
    server = None
    if a.fold_server:  # before this process touches the GPU: the server is the only HIP context
        sock = os.path.join("/tmp", f"bcp_fs_{os.getpid()}.sock")
        code = ("import sys; sys.path.insert(0, %r); import bcp_ctypes as b; print('serving', flush=True); "
                "b.fold_server_serve(%r, 0)" % (os.path.join(ROOT, "beegfs-chunk-parity_amd"), sock))
        server = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
        assert server.stdout.readline().strip() == "serving"
        for _ in range(500):
            if os.path.exists(sock):
                break
            time.sleep(0.01)
        bcp.fold_server_connect(sock, 2 << 30, 12)
    pools = {}

    def pool_for(nt):
        if nt not in pools:
            close_pools()  # one pool at a time: idle ranks keep their GPU contexts
            pools[nt] = bcp.RankPool(nt)
        return pools[nt]

    def close_pools():
        for p in pools.values():
            p.close()
        pools.clear()
    if a.procs:
        def gen(root, nt, items, nlanes=12):
            return pool_for(nt).gen(root, items, nlanes=nlanes)

        def rebuild(root, nt, victim, items):
            return pool_for(nt).rebuild(root, victim, items)
    elif a.procs_cold:
        gen, rebuild = bcp.gen_run_procs, bcp.rebuild_run_procs
    else:
        gen, rebuild = bcp.gen_run, bcp.rebuild_run
    folds = a.folds.split(",")
    bcp.set_rebuild_lanes(a.rebuild_lanes)
    noop = noop_hook()
    ref_fold, ref_name = oracle.cpu_fold_hook()
    hooks = {"cpu_reference": ref_fold,
             "cpu_pipelined": ctypes.cast(oracle.lib().oracle_xor_rows, ctypes.c_void_p).value,
             "noop": ctypes.cast(noop.noop_fold, ctypes.c_void_p).value}
    rng = np.random.default_rng(0)
    wl = a.workloads.split(",")
    import box_probe
    box = box_probe.cpu_info()
    if not (a.procs or a.procs_cold or a.fold_server or a.no_gpu):  # those keep the GPU out of this process
        box.update(box_probe.pcie_rates(bcp))
    emit(box=box, cpu_reference_fold=ref_name)
    tr = {"transport": "socketpair rank processes, pooled" if a.procs else
          "socketpair rank processes, forked per run" if a.procs_cold else "loopback threads"}
    if a.fold_server:
        tr["fold_server"] = "connected (bcp_fold_server_connect)"
    if "c1_gen" in wl or "c1_rebuild" in wl:
        root = os.path.join(a.root, "c1")
        shutil.rmtree(root, ignore_errors=True)
        files = []
        for i in range(a.c1_files):
            p = i % 4
            files.append((f"u0/{i % 64:02X}/chunk{i}", [t for t in range(4) if t != p], p, [512 * KiB] * 3))
        contents = write_store(root, files, 1)
        items = [(path, 2 ** 40, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
        rd, wr = total_bytes(root, files)
        if "c1_gen" in wl:
            def run_gen():
                return gen(root, 4, items, nlanes=a.lanes)
            measure("config1_gen", folds, a.rounds, run_gen, lambda: verify(root, files, contents, 20, rng), rd + wr,
                    hooks, {"lanes": a.lanes, **tr}, prepare=lambda: reset_parity(root, 4))
        if "c1_rebuild" in wl:
            # parity from a correct run, then rebuild target 2 again and again
            bcp.set_xor_hook(hooks["cpu_pipelined"])  # (takes ranges of any pitch)
            try:
                reset_parity(root, 4)
                gen(root, 4, items, nlanes=a.lanes)
            finally:
                bcp.set_xor_hook(None)
            lost = {path: S.chunk_path(root, 2, path) for path, holders, _, _ in files if 2 in holders}
            rb_bytes = len(lost) * 4 * 512 * KiB

            def drop_lost():
                for fn in lost.values():
                    if os.path.exists(fn):
                        os.remove(fn)

            def run_rb():
                return rebuild(root, 4, 2, items)

            def check_rb():
                for k, (path, fn) in enumerate(lost.items()):
                    if k % 50 == 0:
                        holders = next(h for pth, h, _, _ in files if pth == path)
                        if S.read_file(fn) != contents[path][holders.index(2)].tobytes():
                            return False, path
                return True, None
            measure("config1_rebuild", folds, a.rounds, run_rb, check_rb, rb_bytes, hooks, {"lanes": a.rebuild_lanes, **tr},
                    prepare=drop_lost)
        shutil.rmtree(root, ignore_errors=True)
    if "c5_gen" in wl:
        root = os.path.join(a.root, "c5")
        shutil.rmtree(root, ignore_errors=True)
        r5 = np.random.default_rng(5)
        files = []
        nt5, w5 = a.c5_targets, min(8, a.c5_targets - 1)
        for i in range(a.c5_stripes):
            holders, p = S.random_layout(r5, nt5, w5)
            lens = [int(x) for x in np.exp(r5.uniform(np.log(64 * KiB), np.log(4 * MiB), size=w5))]
            files.append((f"u{i % 8}/{(i * 2654435761) % 65536:04X}/chunk{i}", holders, p, lens))
        contents = write_store(root, files, 2)
        items = [(path, 1_700_000_000, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
        rd, wr = total_bytes(root, files)

        def run5():
            return gen(root, nt5, items, nlanes=a.lanes)
        measure("config5_gen", folds, a.rounds, run5, lambda: verify(root, files, contents, 20, rng), rd + wr, hooks,
                {"lanes": a.lanes, "stripes": len(files), "targets": nt5, **tr},
                prepare=lambda: reset_parity(root, nt5))
        shutil.rmtree(root, ignore_errors=True)
    close_pools()
    if not (a.procs or a.procs_cold):
        bcp.task_shutdown()
    if server:
        server.kill()  # serves forever; its socket file goes with /tmp


if __name__ == "__main__":
    main()
