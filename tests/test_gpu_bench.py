"""bench.py as the driver runs it, at a small size: one rank, and two ranks
under torchrun (a child process, never an exec).  Checks the on-device
verification and the GPU-count labels: ranks that share a device are
reported as that many distinct GPUs with shared_gpu set, never as more."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _run(cmd, timeout):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return _last_json(r.stdout)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("mode", ["gen", "rebuild", "mixed"])
def test_bench_one_rank_small(bcp, mode):
    line = _run([sys.executable, "bench.py", "--stripes", "64", "--steps", "5", "--warmup", "1", "--no-cpu",
                 "--no-e2e", "--no-prof", "--no-configs", "--mode", mode], 300)
    assert line["config"]["verified_on_device"] is True
    assert line["n_gpus"] == 1 and line["config"]["ranks"] == 1 and line["config"]["shared_gpu"] is False
    rf = line["roofline"]
    assert rf["frac"] == rf["frac_event"] > 0
    # the per-launch spread: one event pair per step, the average in between
    assert len(rf["kernel_ms_steps"]) == 5 and rf["steps_per_event_pair"] == 1
    assert rf["kernel_ms_min"] <= rf["kernel_ms_median"] <= rf["kernel_ms_max"]
    assert rf["kernel_ms_min"] <= rf["kernel_ms"] * 1.0001 and rf["kernel_ms"] <= rf["kernel_ms_max"] * 1.0001
    assert line["configs"]["config1"] is None


@pytest.mark.timeout(500)
def test_bench_torchrun_two_ranks_labels(bcp):
    ndev = bcp.device_count()
    line = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                 "bench.py", "--gpus", "2", "--stripes", "64", "--steps", "2", "--warmup", "1", "--no-cpu",
                 "--no-e2e", "--no-prof", "--no-configs", "--allow-shared"], 420)
    assert line["config"]["verified_on_device"] is True
    assert line["config"]["ranks"] == 2
    distinct = min(ndev, 2)  # bench maps local rank r to device r % ndev
    assert line["n_gpus"] == distinct
    assert line["config"]["shared_gpu"] is (distinct < 2)
    assert line["roofline"]["run_box"]["pci_bus_id"] in line["config"]["pci_bus_ids"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_gpus_n_launches_its_own_ranks(bcp, n):
    """The driver's form, `python3 bench.py --gpus N` with no launcher: bench.py
    starts N ranks itself.  With fewer GPUs than N it refuses (non-zero exit,
    no line) unless --allow-shared, which reports the ranks and the distinct GPUs.
    N = 8 rehearses every branch of the driver's 8-GPU run on one device (an
    explicit --stripes: the config-4 default shard is 68.6 GiB per rank; the
    default itself is pinned on CPU, tests/test_dist_cpu.py)."""
    ndev = bcp.device_count()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    args = [sys.executable, "bench.py", "--gpus", str(n), "--stripes", "64", "--steps", "2", "--warmup", "1",
            "--cpu-seconds", "1", "--cpu-stripes", "16", "--e2e-gib", "0.1" if n == 8 else "0.25", "--e2e-reps", "1",
            "--c1-files", "48", "--c1-reps", "1", "--c5-reps", "1"]
    args += [] if n == 2 else ["--no-prof"]  # the live profile from rank 0 of an N-rank job
    if ndev < n:
        r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 4, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        assert "refusing" in r.stderr
        assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    r = subprocess.run(args + ["--allow-shared"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = _last_json(r.stdout)
    assert line["config"]["ranks"] == n
    assert line["n_gpus"] == min(ndev, n)
    assert line["config"]["shared_gpu"] is (ndev < n)
    assert line["config"]["verified_on_device"] is True
    per = line["config"]["per_rank"]  # each GPU's own rate in the N-GPU line
    assert [r["rank"] for r in per] == list(range(n)) and all(r["verified"] and r["GiBps"] > 0 for r in per)
    # the N-GPU line is complete: per-rank rates, the reference CPU path timed
    # in the same run, and the end-to-end figure at every N
    assert line["per_rank"] == per
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "reference" and cpu["value"] > 0 and cpu["cores"] >= 1
    assert cpu["legs"][0]["threads"] == 1 and "quota_cpus" in cpu
    e2e = line["e2e"]
    assert e2e["ranks"] == n and len(e2e["per_rank"]) == n
    assert 2 <= e2e["io_threads_per_rank"] <= 8  # the ranks share the host's CPU quota
    assert e2e["gen"]["verified"] is True and e2e["rebuild"]["verified"] is True
    assert e2e["gen"]["GiBps"] > 0 and e2e["rebuild"]["GiBps"] > 0
    assert e2e["gen"]["bytes_read"] == sum(r["bytes_read"] for r in e2e["per_rank"])
    assert set(e2e["by_read_mode"]) == {"copy", "direct"} and e2e["read_mode"] == "copy"
    dt = e2e["by_read_mode"]["direct"]["gen_timing"]
    assert dt["read_mode"] == 3 and (dt["direct_bytes"] > 0 or dt["direct_fallbacks"] > 0), dt
    # the config-5 changelog subset on every rank, the config-1 protocol leg on rank 0
    part = line["configs"]["config5_partial"]
    assert part == e2e["partial"] and part["verified"] is True and part["plan_ok"] is True, part
    assert part["stripes"] == sum(r["partial"]["stripes"] for r in e2e["per_rank"]) > 0
    c1 = line["configs"]["config1"]
    assert "gen" in c1 and all(c1["gen"][k]["verified"] for k in ("reference_fold", "gpu_fold", "pipeline")), c1
    assert c1["gen"]["reference_fold"]["kind"] == "reference"
    assert "error" not in line["configs"]["config5_protocol"], line["configs"]["config5_protocol"]
    if n == 2:
        live = line["roofline"]["live_profile"]
        assert live and "error" not in live and line["roofline"]["same_box"] is True, live
        assert line["roofline"]["profiled_in_process"] is True
    if n == 8:
        assert "config2" in line["config"]["workload"]  # an explicit --stripes is never labelled config 4
    assert line["config"]["bytes_per_step_per_gpu"] * n * line["steps"] / 2**30 / (line["ms_per_step"] *
                                                                                   line["steps"] * 1e-3) == \
        pytest.approx(line["value"], rel=5e-3)  # value = the whole job's bytes / the slowest rank's time


@pytest.mark.timeout(400)
def test_bench_mixed_line_carries_cpu_baseline_and_e2e(bcp):
    """Mixed mode (config-5 shapes): the reference's fold timed over the same
    zero-padded stripe shapes, and the end-to-end leg, in the one-rank line."""
    line = _run([sys.executable, "bench.py", "--mode", "mixed", "--stripes", "64", "--steps", "2", "--warmup", "1",
                 "--cpu-seconds", "1", "--e2e-gib", "0.25", "--e2e-reps", "1", "--no-prof", "--no-configs"], 300)
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "reference" and cpu["value"] > 0 and "stripe_shapes" in cpu["legs"][0]
    assert line["e2e"]["gen"]["verified"] is True and line["e2e"]["rebuild"]["verified"] is True
    assert line["per_rank"][0]["verified"] is True


@pytest.mark.timeout(400)
def test_bench_configs_block_one_rank(bcp):
    """BASELINE configs 1 and 5 in the driver's line: config 1 (4 loopback
    ranks, 3-wide stripes, P rotating) through the per-task protocol with the
    reference's own xor_parity as the P-role fold, with the GPU fold and
    through the pipeline, gen and rebuild, all verified; config 5's changelog
    subset planned against the DB and recomputed, verified."""
    line = _run([sys.executable, "bench.py", "--stripes", "64", "--steps", "2", "--warmup", "1", "--no-prof",
                 "--cpu-seconds", "1", "--e2e-gib", "0.25", "--e2e-reps", "1", "--c1-files", "96",
                 "--c1-reps", "1", "--c5-reps", "1"], 360)
    c1 = line["configs"]["config1"]
    assert "error" not in c1 and "skipped" not in c1, c1
    for what in ("gen", "rebuild"):
        for leg in ("reference_fold", "gpu_fold", "pipeline"):
            x = c1[what][leg]
            assert x["verified"] is True and x["GiBps"] > 0 and len(x["runs_s"]) == 2, (what, leg, x)
            assert x["cpu_s"] > 0 and x["cores_busy"] > 0, (what, leg, x)
    assert c1["gen"]["reference_fold"]["kind"] == "reference" and c1["rebuild"]["files"] == 72
    assert c1["bytes"]["gen_read"] == 96 * 3 * 512 * 1024
    assert c1["link"]["h2d_GBps"] > 0 and c1["gpu_fold_link_ceiling_GiBps"] > 0, c1
    assert c1["gpu_fold_in_place_bound"]["GiBps"] > 0 and c1["gpu_fold_in_place_bound"]["lanes"] == 12, c1
    assert c1["gpu_fold_over_link_ceiling"] == round(
        c1["gen"]["gpu_fold"]["GiBps"] / ((c1["bytes"]["gen_read"] + c1["bytes"]["gen_written"]) /
                                          (c1["bytes"]["gen_read"] / (c1["link"]["h2d_GBps"] * 1e9)) / 1024 ** 3), 3)
    assert c1["gpu_fold_over_in_place_bound"] > 0, c1
    part = line["configs"]["config5_partial"]
    assert part["verified"] is True and part["plan_ok"] is True and part["GiBps"] > 0, part
    assert part["stripes"] == max(1, line["e2e"]["per_rank"][0]["stripes"] // 10)
    st = part["stages_warm_s_rank0"]
    assert set(st) == {"parse_s", "db_read_s", "plan_s", "run_s", "replicas_s"} and st["run_s"] > 0, st
    c5 = line["configs"]["config5_protocol"]
    assert "error" not in c5, c5
    for what in ("gen", "rebuild"):
        for leg in ("reference_fold", "gpu_fold"):
            x = c5[what][leg]
            assert x["verified"] is True and x["GiBps"] > 0 and len(x["runs_s"]) == 2, (what, leg, x)
    assert c5["gen"]["reference_fold"]["kind"] == "reference" and c5["ring"]["pieces"] > 0, c5
    ib = c1["gpu_fold_in_place_bound"]
    assert ib["per_launch"]["GiBps"] > 0 and "ring" in ib["shape"], ib


@pytest.mark.timeout(400)
def test_bench_line_survives_an_e2e_failure_on_one_rank(bcp):
    """The end-to-end leg never costs the N-GPU line: a rank whose store
    cannot be written (injected) keeps making the collective calls, and rank 0
    prints the device line with the failure reported inside `e2e`."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BCP_BENCH_E2E_FAIL_RANK="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--allow-shared", "--stripes", "64", "--steps", "2",
                        "--warmup", "1", "--no-cpu", "--e2e-gib", "0.25", "--e2e-reps", "1", "--no-prof", "--no-configs"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=360)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = _last_json(r.stdout)
    assert line["config"]["verified_on_device"] is True and line["value"] > 0
    e2e = line["e2e"]
    assert list(e2e["errors"]) in (["1"], [1]) and "injected" in str(e2e["errors"])
    assert e2e["gen"]["verified"] is False and e2e["per_rank"][0]["errors"] is None
    assert "error" in e2e["partial"]  # the failed rank's partial round is reported, rank 0's line stands


@pytest.mark.timeout(500)
@pytest.mark.parametrize("mode", ["gen", "mixed"])
def test_bench_live_profile_on_its_own_box(bcp, mode):
    """The roofline's rocprof figures come from the line's own launches: the
    rank runs under rocprofv3 --kernel-trace as a child of bench.py, the
    trace's timed dispatches (warm-up and verification excluded) are averaged
    and compared with the same process's HIP events over the same launches;
    then the two PMC passes of the workload (traffic within 1 % of the
    algorithmic bytes), same_box set."""
    line = _run([sys.executable, "bench.py", "--mode", mode, "--stripes", "256", "--steps", "4", "--warmup", "2",
                 "--no-cpu", "--no-e2e", "--no-configs"], 450)
    rf = line["roofline"]
    live = rf["live_profile"]
    assert live and "error" not in live and "pmc_error" not in live, live
    assert rf["profiled_in_process"] is True and live["in_process"] is True
    assert live["rocprof_timed_launches"] == 4 and len(live["rocprof_timed_ms_steps"]) == 4
    assert live["tagged_dispatches"] == 2 + 4 + 1
    # the events of a step bracket the fold alone in gen; in mixed mode also the
    # step's desc_tiles and, on an idle queue, its host staging (tiny steps here)
    hi = 1.1 if mode == "gen" else 1.3
    assert 0.9 < live["event_over_rocprof"] < hi and 0.9 < live["event_over_rocprof_median"] < hi, live
    assert live["rocprof_min_ns"] <= live["rocprof_median_ns"] <= live["rocprof_max_ns"]
    assert 0.99 < live["traffic_over_algorithmic"] < 1.02, live
    assert rf["same_box"] is True and rf["traffic"] == live["traffic"]
    assert rf["frac_rocprof"] > 0 and rf["profile_box"] == rf["run_box"]
    # frac_event / frac_rocprof = rocprof time / event time of the same launches
    assert abs(rf["frac_event_over_rocprof"] * live["event_over_rocprof"] - 1.0) < 2e-3


@pytest.mark.timeout(500)
def test_bench_line_survives_failed_legs(bcp):
    """Every leg beside the device timing fails (injected): the CPU baseline,
    config 1, config 5 through the protocol -- the line is printed, verified,
    with each failure in its own block and the e2e block intact."""
    env = dict(os.environ, BCP_BENCH_FAIL_LEG="cpu_baseline,config1,config5_protocol")
    r = subprocess.run([sys.executable, "bench.py", "--stripes", "64", "--steps", "2", "--warmup", "1", "--no-prof",
                        "--cpu-seconds", "1", "--e2e-gib", "0.25", "--e2e-reps", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    line = _last_json(r.stdout)
    assert line["config"]["verified_on_device"] is True and line["value"] > 0
    assert "injected" in line["cpu_baseline"]["error"]
    assert "injected" in line["configs"]["config1"]["error"]
    assert "injected" in line["configs"]["config5_protocol"]["error"]
    assert line["e2e"]["gen"]["verified"] is True and line["e2e"]["errors"] is None
    assert line["configs"]["config5_partial"]["verified"] is True
