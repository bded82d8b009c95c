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
average, kernel_ms_median / min / max / steps the per-launch spread).  Rank
0's device timing runs in a child of the rank process under `rocprofv3
--kernel-trace --stats` (profiled_rank: the device helper, started before
anything touches HIP, never an exec; its barriers go through the rank
process, which stays the job's member), so frac_rocprof is the rocprof
average of the SAME timed launches (roofline.live_profile:
event_over_rocprof), and nothing else runs under the profiler: the rank
process then runs the legs itself and the PMC passes (FETCH_SIZE,
WRITE_SIZE, runs of their own) of the same workload for traffic.  With
--no-prof, or when a pass fails, the committed profile set of the workload
(profiles/CURRENT_SET, profiles/**/*pmc*.json, tools/pmc_summary.py) stands
in, reported as roofline.committed_set.
The legs beside the device timing are bench_legs.py's, each behind run_leg.
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
from bench_legs import (HBM_PEAK_GBS, config1_leg, cpu_baseline, cpu_quota, e2e_leg,  # noqa: E402,F401
                        e2e_store_dir, pmc_passes, pmc_traffic, rocprof_exe, trace_figures, usable_cpus)

KiB = 1024
GiB = 1024 ** 3
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
    ap.add_argument("--e2e-gib", type=float, default=10.0,
                    help="chunk bytes per rank in the end-to-end store (its 10 %% changelog subset: >= 1 GiB)")
    ap.add_argument("--e2e-reps", type=int, default=3, help="warm end-to-end gen runs (after one cold run)")
    ap.add_argument("--e2e-dir", default="/dev/shm", help="where the end-to-end stores are created")
    ap.add_argument("--e2e-max-s", type=float, default=150.0, help="wall-time cap of the end-to-end leg")
    ap.add_argument("--e2e-modes", default="copy,direct",
                    help="pipeline read paths timed end to end, interleaved; the first is the headline")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the config-1 protocol leg (rank 0)")
    ap.add_argument("--c1-first", action=argparse.BooleanOptionalAction, default=False,
                    help="run the config-1 protocol leg before the e2e and CPU-baseline legs")
    ap.add_argument("--c1-legs", default="reference_fold,gpu_fold,pipeline",
                    help="config-1 legs (the two folds always run; the pipeline can be left out for A/B runs)")
    ap.add_argument("--c1-files", type=int, default=1333, help="config 1: files (3 chunks of 512 KiB each)")
    ap.add_argument("--c1-reps", type=int, default=7, help="config 1: warm rounds per leg (after one cold round)")
    ap.add_argument("--c5-reps", type=int, default=3,
                    help="config 5 through the protocol (rank 0, the e2e store): warm gen rounds per leg")
    ap.add_argument("--no-prof", action="store_true",
                    help="skip the live rocprofv3 kernel-trace and PMC passes of this workload on this box")
    ap.add_argument("--profile-dir", default=None,
                    help="keep rank 0's kernel trace (<dir>/trace) and the PMC passes (<dir>/pmc_fetch, pmc_write) "
                         "there (tools/gpu_profiles.sh, the committed profile sets)")
    ap.add_argument("--device-helper", default=None, metavar="RANK,WORLD,LOCAL_RANK",
                    help=argparse.SUPPRESS)  # internal: profiled_rank's device helper under rocprofv3
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


def leg_blocks(cpu, c1, e2e) -> dict:
    """The line's blocks from the legs' results (each a dict, an {"error": ...}
    dict, or None when not run): cpu_baseline (with config 1's reference-fold
    rates beside it), e2e, and configs -- config1, config5_partial (the e2e
    block's partial round), config5_protocol (rank 0's protocol run on the
    e2e store).  A failed leg shows in its own block only."""
    def ok(x, key):
        return isinstance(x, dict) and key in x
    cpu_block = cpu
    if isinstance(cpu, dict) and "error" not in cpu:
        cpu_block = dict(cpu, config1_protocol_reference_fold=(
            {"gen_GiBps": c1["gen"]["reference_fold"]["GiBps"],
             "rebuild_GiBps": c1["rebuild"]["reference_fold"]["GiBps"], "kind": c1["gen"]["reference_fold"]["kind"],
             "see": "configs.config1"} if ok(c1, "gen") else None))
    e2e_d = e2e if isinstance(e2e, dict) else {}
    return {"cpu_baseline": cpu_block,
            "e2e": e2e,
            # BASELINE configs[0] and configs[4] as BASELINE states them: rank 0's config-1 protocol leg; the
            # config-5 changelog subset of every rank's e2e store; config 5 through the protocol (rank 0)
            "configs": {"config1": c1, "config5_partial": e2e_d.get("partial"),
                        "config5_protocol": e2e_d.get("config5_protocol")}}


def run_leg(name: str, fn, *args):
    """One leg of the line (bench_legs): its block, or {"error": ...} -- a leg
    never costs the device figures the line is for."""
    try:
        return fn(*args)
    except Exception as e:  # reported in the block, never raised
        return {"error": f"{name}: {type(e).__name__}: {e}"}


PROFILED_ENV = "BCP_BENCH_PROFILED"  # set in the device helper that runs under rocprofv3
HELPER_TAG = "BCPDEV "  # the device helper's messages on its stdout


def _last_json(text: str):
    lines = [x for x in (text or "").splitlines() if x.startswith("{")]
    return json.loads(lines[-1]) if lines else None


class DistCoord:
    """device_phase's two collectives, in the rank process itself."""

    def __init__(self, d):
        self.d = d

    def gather_bus(self, bus: str) -> list:
        return self.d.gather(bus)

    def barrier(self):
        self.d.barrier()


class PipeCoord:
    """device_phase's collectives from the profiled device helper: each is a
    message to the rank process (the helper's parent, the job's member), which
    runs it in the job and answers on the helper's stdin."""

    def _send(self, obj):
        sys.stdout.write(HELPER_TAG + json.dumps(obj) + "\n")
        sys.stdout.flush()

    def _recv(self) -> dict:
        line = sys.stdin.readline()
        if not line:
            raise SystemExit(5)  # the rank process is gone
        return json.loads(line)

    def gather_bus(self, bus: str) -> list:
        self._send({"op": "gather_bus", "bus": bus})
        return self._recv()["bus_ids"]

    def barrier(self):
        self._send({"op": "barrier"})
        self._recv()

    def done(self, dev: dict):
        self._send({"op": "device", "dev": dev})


def serve_helper(p, d) -> tuple:
    """The rank process's side of PipeCoord: answer the helper's collectives in
    the job until it exits; (its device figures or None, whether it got as far
    as a collective, its exit status)."""
    dev, started = None, False
    for line in p.stdout:
        if not line.startswith(HELPER_TAG):
            sys.stderr.write(line)  # the helper's own output, kept off the line's stdout
            continue
        m = json.loads(line[len(HELPER_TAG):])
        started = True
        if m["op"] == "gather_bus":
            reply = {"bus_ids": d.gather(m["bus"])}
        elif m["op"] == "barrier":
            d.barrier()
            reply = {}
        else:
            dev = m["dev"]
            continue
        p.stdin.write(json.dumps(reply) + "\n")
        p.stdin.flush()
    p.stdin.close()
    return dev, started, p.wait()


def profiled_rank(a, d) -> int:
    """Rank 0 (or the one rank): the device timing runs in a CHILD process
    under `rocprofv3 --kernel-trace --stats` (this process has not touched HIP;
    never an exec) -- the device helper, which sets up the stripes, times the
    steps and verifies them, and sends its figures back; the helper's two
    collectives (the bus-id gather, the barriers around the timed region) go
    through this process, the job's member (PipeCoord / serve_helper).  So the
    trace holds exactly the launches the line's HIP events time, and only the
    device timing runs under the profiler: this process then runs the legs
    (e2e, cpu_baseline, configs) itself, reads the trace (the rocprof average
    of the timed launches), runs the two PMC passes of the same workload, puts
    both in the line's roofline and prints it.  A helper that fails before its
    first collective (or at one rank, any time) is replaced by the same device
    phase in this process, without the profiler; one that fails later in an
    N-rank job fails the rank."""
    import shutil
    import subprocess
    import tempfile
    exe = rocprof_exe()
    keep = a.profile_dir is not None
    if keep:
        out = os.path.join(os.path.abspath(a.profile_dir), "trace")
        os.makedirs(out, exist_ok=True)
    else:
        out = tempfile.mkdtemp(prefix="bcp_bench_trace_")
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV and not k.startswith("TORCHELASTIC")}
    env[PROFILED_ENV] = "1"
    me = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:] + [
        "--device-helper", f"{d.rank},{d.world},{d.local_rank}"]
    t0 = time.perf_counter()
    p = subprocess.Popen([exe, "--kernel-trace", "--stats", "-d", out, "-o", "run", "--output-format", "csv", "--"]
                         + me, env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    dev, started, rc = serve_helper(p, d)
    note = None
    if dev is None:
        if started and d.world > 1:  # the other ranks are inside a collective with it
            print(f"bench.py: the profiled device helper exited {rc} in the middle of the run", file=sys.stderr)
            if not keep:
                shutil.rmtree(out, ignore_errors=True)
            return rc or 1
        note = f"the profiled device helper exited {rc} without its figures; timed without the profiler"
        print(f"bench.py: {note}", file=sys.stderr)
        dev = device_phase(a, d.rank, d.world, d.local_rank, DistCoord(d))
    if dev.get("refused"):
        return dev["refused"]
    dev["profiled"] = note is None
    line, rc2 = finish(a, d, dev)
    if line is None:
        if not keep:
            shutil.rmtree(out, ignore_errors=True)
        return rc2 or 1
    rf = line["roofline"]
    cfg = line["config"]
    bps = cfg["bytes_per_step_per_gpu"]
    r0 = (cfg.get("per_rank") or [{}])[0]
    try:
        tr = (trace_figures(out, rf["kernel_tag"], line["warmup"], line["steps"], bps,
                            event_ms_steps=rf.get("kernel_ms_steps") if rf.get("steps_per_event_pair") == 1 else None,
                            event_ms_avg=r0.get("kernel_ms"))
              if note is None else {"error": note})
    except Exception as e:
        tr = {"error": f"trace: {type(e).__name__}: {e}"}
    finally:
        if not keep:
            shutil.rmtree(out, ignore_errors=True)
    penv = {k: v for k, v in os.environ.items()
            if k not in DIST_ENV and k != PROFILED_ENV and not k.startswith("TORCHELASTIC")}
    pm = pmc_passes(workload_cmd(a), penv, rf["kernel_tag"], bps,
                    keep_dir=os.path.abspath(a.profile_dir) if keep else None)
    live = dict(tr)
    for k, v in pm.items():
        live[{"error": "pmc_error", "wall_s": "pmc_wall_s", "skipped": "pmc_skipped"}.get(k, k)] = v
    live["wall_s"] = round(time.perf_counter() - t0, 1)
    rf["live_profile"] = live
    if tr.get("frac_rocprof"):
        rf["frac_rocprof"] = tr["frac_rocprof"]
        rf["frac_event_over_rocprof"] = round(rf["frac_event"] / tr["frac_rocprof"], 4)
    if pm.get("traffic"):
        rf["traffic"] = pm["traffic"]
        rf["traffic_source"] = pm["source"]
    if tr.get("frac_rocprof") and pm.get("traffic"):
        rf["profile_box"] = rf["run_box"]
        rf["same_box"] = True
    print(json.dumps(line), flush=True)
    return rc2


DIST_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
            "MASTER_PORT")


def workload_cmd(a) -> list:
    """This run's device workload alone (the PMC passes' child): a fresh
    process, one rank, no legs, a few steps."""
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--mode", a.mode, "--stripes", str(a.stripes),
           "--nsrc", str(a.nsrc), "--chunk", str(a.chunk), "--rebuild-layout", a.rebuild_layout,
           "--no-cpu", "--no-e2e", "--no-prof", "--no-configs", "--steps", "3", "--warmup", "1"]
    for flag, val in (("--blocks-per-cu", a.blocks_per_cu), ("--vecs", a.vecs), ("--grid", a.grid)):
        if val:
            cmd += [flag, str(val)]
    if a.contig:
        cmd.append("--contig")
    for kv in a.opt:
        cmd += ["--opt", kv]
    return cmd


def mixed_lengths(stripes: int, N: int, C: int, rank: int) -> list:
    """--mode mixed's stripe shapes (seeded per rank): log-uniform chunk
    lengths in [64 KiB, 4 MiB], as many 8-wide stripes as fit config 2's input
    volume (stripes x N x C)."""
    import numpy as np
    rng = np.random.default_rng(3 + rank)
    budget = stripes * N * C
    lens_all, tot = [], 0
    while tot < budget:
        ls = np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * 1024 * KiB), size=N)).astype(np.int64)
        lens_all.append(ls)
        tot += int(ls.sum())
    return lens_all


def device_phase(a, rank: int, world: int, local_rank: int, coord) -> dict:
    """The device timing of one rank: stripes set up in HBM, warm-up, the
    timed steps between two barriers (coord: DistCoord in the rank process,
    PipeCoord in the profiled device helper), one more step verified on the
    device and against numpy.  Returns the figures finish() needs (JSON), or
    {"refused": 4} when ranks share a GPU without --allow-shared."""
    ndev = bcp.device_count()
    assert ndev > 0, "bench.py needs a HIP device (there is no CPU path)"
    eng = bcp.Engine(local_rank % ndev)
    # physical GPUs in the job: ranks that map to the same device share it
    bus_ids = coord.gather_bus(eng.pci_bus_id())
    n_devices = len(set(bus_ids))
    shared_gpu = n_devices < world
    if shared_gpu and not a.allow_shared:
        if rank == 0:
            print(f"bench.py: {world} ranks but only {n_devices} distinct GPU(s) (PCI bus ids "
                  f"{sorted(set(bus_ids))}); refusing (pass --allow-shared to rehearse)", file=sys.stderr)
        eng.close()
        return {"refused": 4}
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
        a.stripes = default_stripes(world, rank)
    S, N, C = a.stripes, a.nsrc, a.chunk
    chk = eng.alloc(64)
    lens_all = None
    if a.mode == "mixed":
        lens_all = mixed_lengths(S, N, C, rank)
        align = lambda x: (x + 255) & ~255
        src_bytes = sum(int(sum(align(int(x)) for x in ls)) for ls in lens_all)
        out_bytes = sum(align(int(ls.max())) for ls in lens_all)
        src = eng.alloc(src_bytes)
        out = eng.alloc(out_bytes)
    else:
        src = eng.alloc(S * N * C)
        out = eng.alloc(S * C)
        src_bytes = S * N * C
    q.fill_synthetic(src, src_bytes, seed=1 + rank)

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
        cfg = gen_config_label(world, S)
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
    coord.barrier()
    q.sync()
    t0 = time.perf_counter()
    q.mark(0)
    for i in range(a.steps):
        step()
        if (i + 1) in bounds:
            q.mark(bounds.index(i + 1))
    q.sync()
    t1 = time.perf_counter()
    coord.barrier()
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
    rng = np.random.default_rng(7 + rank)

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

    device = eng.device
    q.close()
    eng.close()
    return {"rank": rank, "world": world, "device": device, "bus_ids": bus_ids, "n_devices": n_devices,
            "shared_gpu": shared_gpu, "cus": cus, "devname": devname, "S": S, "N": N, "C": C, "U": U,
            "kernel": kernel, "kernel_tag": kernel_tag, "workload": workload, "bytes_per_step": bytes_per_step,
            "wall": wall, "kern_ms": kern_ms, "seg_ms": seg_ms, "g": g, "verified": bool(verified)}


def finish(a, d, dev: dict) -> tuple:
    """After the device phase (dev: device_phase's figures, this rank's): the
    max-over-ranks reductions, the legs (bench_legs, each behind run_leg; they
    run in the rank process, never under the profiler) and, on rank 0, the
    line.  Returns (the line or None, exit status)."""
    S, N, C, U = dev["S"], dev["N"], dev["C"], dev["U"]
    kernel, kernel_tag, workload = dev["kernel"], dev["kernel_tag"], dev["workload"]
    bytes_per_step, wall, kern_ms, seg_ms, g = (dev["bytes_per_step"], dev["wall"], dev["kern_ms"], dev["seg_ms"],
                                                dev["g"])
    verified, bus_ids, n_devices, shared_gpu = dev["verified"], dev["bus_ids"], dev["n_devices"], dev["shared_gpu"]
    cus, devname = dev["cus"], dev["devname"]
    lens_all = mixed_lengths(a.stripes, N, C, d.rank) if a.mode == "mixed" and not a.no_cpu and d.rank == 0 else None
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

    # BASELINE config 1 end to end (rank 0; the reference's xor_parity as the
    # P-role fold beside the GPU fold and the pipeline, same store); first
    # with --c1-first, before the e2e store's churn and the CPU baseline's
    # all-core run (the other ranks wait at the barrier)
    c1 = None
    if a.c1_first:
        c1 = run_leg("config1", config1_leg, a, dev["device"]) if d.rank == 0 and not a.no_configs else None
        d.barrier()
    # end to end from chunk files (every rank on its own GPU, all at once;
    # e2e_leg keeps every rank's collective calls in step whatever fails)
    e2e = None
    if not a.no_e2e:
        e2e = e2e_leg(a, d, dev["device"], bus_ids[d.rank])
    # the reference CPU path, rank 0 only, after every device figure; the
    # other ranks wait at the barrier
    cpu = run_leg("cpu_baseline", cpu_baseline, a, N, C, lens_all if a.mode == "mixed" else None) \
        if d.rank == 0 and not a.no_cpu else None
    if not a.c1_first:
        c1 = run_leg("config1", config1_leg, a, dev["device"]) if d.rank == 0 and not a.no_configs else None
    d.barrier()

    if d.rank == 0:
        value = total_bytes / wall_max / GiB
        achieved = bytes_per_step / (kern_ms_max * 1e-3) / 1e9
        mode_key = "rebuild_packed" if (a.mode == "rebuild" and a.rebuild_layout == "packed") else a.mode
        wkey = f"{mode_key}:{S}x{N}x{C}"
        pmc = pmc_traffic(wkey, kernel_tag)
        run_box = box_of(bus_ids[0])
        # frac_rocprof and traffic of this run: filled in by the profiling
        # parent (profiled_rank) from this process's own trace and the PMC
        # passes; the committed set until then (and with --no-prof)
        frac_rocprof = None
        if pmc and (pmc.get("rocprof_timed_avg_ns") or pmc.get("rocprof_avg_ns")):
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
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "traffic_source": pmc["source"] if pmc else None,
                "live_profile": None,
                # the timed launches ran in the device helper under rocprofv3 (profiled_rank); the legs not
                "profiled_in_process": bool(dev.get("profiled")),
                "profile_files": pmc.get("files") if pmc else None,
                "profile_commit": pmc.get("code_commit") if pmc else None,
                "run_box": run_box,
                "profile_box": pmc.get("box") if pmc else None,
                "same_box": bool(pmc and pmc.get("box") and run_box["boot_id"]
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
                             "bytes / the rocprofv3 kernel-trace average of THE SAME launches -- rank 0 runs under "
                             "rocprofv3 --kernel-trace (profiled_in_process) and the trace's timed dispatches "
                             "(warm-up and verification excluded) are averaged; live_profile.event_over_rocprof = "
                             "rank 0's event average / that; traffic: the PMC passes (FETCH_SIZE, WRITE_SIZE) of "
                             "this workload in child runs on this box -- or, where those failed or --no-prof, the "
                             "committed profile set (profile_files, measured on profile_box)",
            },
            **leg_blocks(cpu, c1, e2e),
            "per_rank": per_rank,
        }
    else:
        line = None
    d.close()
    return line, (0 if ok_all else 3)


def main():
    a = parse()
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if a.device_helper:  # the profiled device helper (profiled_rank's child)
        rank, world, local_rank = (int(x) for x in a.device_helper.split(","))
        pc = PipeCoord()
        dev = device_phase(a, rank, world, local_rank, pc)
        pc.done(dev)
        sys.exit(0)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    d = Dist()
    if d.world != a.gpus and d.rank == 0:
        print(f"bench.py: note: launched with {d.world} ranks for --gpus {a.gpus}; "
              f"the line reports the ranks and distinct GPUs actually used", file=sys.stderr)
    if not a.stripes:
        a.stripes = default_stripes(d.world, d.rank)
    # rank 0's device timing runs in a child under the profiler (this process has not touched HIP)
    if not a.no_prof and d.rank == 0 and rocprof_exe():
        sys.exit(profiled_rank(a, d))
    dev = device_phase(a, d.rank, d.world, d.local_rank, DistCoord(d))
    if dev.get("refused"):
        d.close()
        sys.exit(dev["refused"])
    line, rc = finish(a, d, dev)
    if line is not None:
        print(json.dumps(line), flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
