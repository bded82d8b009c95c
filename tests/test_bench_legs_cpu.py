"""bench.py's structure on CPU: every leg behind run_leg, each leg's failure
confined to its own block of the line (leg_blocks), the failure hook, and the
profiled-rank orchestration -- rank 0 under rocprofv3 as a child, the trace
of the line's own timed launches and the PMC passes patched into the line --
driven by a stand-in rocprofv3 that writes the files the real one writes."""
import json
import os
import stat
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_run_leg_reports_instead_of_raising():
    import bench

    def boom():
        raise OSError("disk on fire")
    assert bench.run_leg("x", lambda v: v + 1, 1) == 2
    assert bench.run_leg("cpu_baseline", boom) == {"error": "cpu_baseline: OSError: disk on fire"}


def test_each_failed_leg_stays_in_its_own_block():
    import bench
    cpu = {"value": 40.0, "kind": "reference", "cores": 16}
    c1 = {"gen": {"reference_fold": {"GiBps": 70.0, "kind": "reference"}},
          "rebuild": {"reference_fold": {"GiBps": 10.0}}}
    e2e = {"gen": {"GiBps": 50}, "partial": {"GiBps": 30}, "config5_protocol": {"gen": {}}}
    full = bench.leg_blocks(cpu, c1, e2e)
    assert full["cpu_baseline"]["config1_protocol_reference_fold"]["gen_GiBps"] == 70.0
    assert full["configs"] == {"config1": c1, "config5_partial": {"GiBps": 30}, "config5_protocol": {"gen": {}}}
    err = {"error": "x: RuntimeError: injected"}
    # the CPU baseline failed: config 1 and the e2e blocks stand
    b = bench.leg_blocks(err, c1, e2e)
    assert b["cpu_baseline"] == err and b["configs"]["config1"] == c1 and b["e2e"] == e2e
    # config 1 failed: the CPU baseline stands, without config 1's rates beside it
    b = bench.leg_blocks(cpu, err, e2e)
    assert b["cpu_baseline"]["value"] == 40.0 and b["cpu_baseline"]["config1_protocol_reference_fold"] is None
    assert b["configs"]["config1"] == err
    # the e2e leg failed or was not run
    b = bench.leg_blocks(cpu, c1, None)
    assert b["e2e"] is None and b["configs"]["config5_partial"] is None and b["configs"]["config5_protocol"] is None
    b = bench.leg_blocks(None, None, {"skipped": "no room"})
    assert b["cpu_baseline"] is None and b["configs"]["config5_partial"] is None


def test_failure_hook(monkeypatch):
    import bench_legs
    monkeypatch.setenv("BCP_BENCH_FAIL_LEG", "config1,cpu_baseline")
    with pytest.raises(RuntimeError, match="config1"):
        bench_legs.maybe_fail("config1")
    bench_legs.maybe_fail("config5_protocol")  # not named: passes


def _write_trace(d, tag, durs, other=0):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w") as f:
        f.write("Dispatch_Id,Kernel_Name,Start_Timestamp,End_Timestamp\n")
        i, t = 1, 1000
        for dur in durs:
            for _ in range(other):  # another kernel's dispatches in between
                f.write(f"{i},\"desc_tiles(bcp::DescBatch)\",{t},{t + 5}\n")
                i += 1
                t += 10
            f.write(f"{i},\"void bcp::{tag}(bcp::StreamArgs)\",{t},{t + dur}\n")
            i += 1
            t += dur + 10


def test_trace_figures_average_the_timed_launches_only(tmp_path):
    import bench_legs
    tag = "xor_stream_w<8, 8, 0, 0, 6>"
    # 2 warm-up, 4 timed, 1 verification, then 3 from later legs
    _write_trace(str(tmp_path), tag, [9_000_000, 9_000_000, 8_000_000, 8_200_000, 8_100_000, 8_300_000, 7_000_000,
                                      1, 1, 1], other=1)
    bps = 58_982_400_000 // 12_500 * 12_500
    fig = bench_legs.trace_figures(str(tmp_path), tag, 2, 4, bps, event_ms_steps=[8.0, 8.2, 8.1, 8.3],
                                   event_ms_avg=8.15)
    assert fig["rocprof_timed_launches"] == 4 and fig["tagged_dispatches"] == 10
    assert fig["rocprof_avg_ns"] == 8_150_000 and fig["rocprof_min_ns"] == 8_000_000
    assert fig["event_over_rocprof"] == 1.0 and fig["event_over_rocprof_median"] == 1.0
    assert fig["frac_rocprof"] == round(bps / 8.15e-3 / 1e9 / 8000.0, 4)
    with pytest.raises(RuntimeError, match="expected at least"):
        bench_legs.trace_figures(str(tmp_path), tag, 5, 6, bps)


FAKE_ROCPROF = textwrap.dedent('''\
    #!{py}
    """Stand-in rocprofv3: writes the csv files the real one writes and, for a
    kernel trace, plays the device helper (bench.PipeCoord's messages)."""
    import json, os, sys
    args = sys.argv[1:]
    d = args[args.index("-d") + 1]
    os.makedirs(d, exist_ok=True)
    tag = "xor_stream_w<8, 8, 0, 0, 6>"
    mode = os.environ.get("FAKE_ROCPROF_MODE", "ok")
    if "--kernel-trace" in args:
        if mode == "fail":
            sys.exit(3)
        assert os.environ.get("BCP_BENCH_PROFILED") == "1" and "RANK" not in os.environ
        assert "--device-helper" in args

        def send(obj):
            print("BCPDEV " + json.dumps(obj), flush=True)

        def recv():
            return json.loads(sys.stdin.readline())
        print("noise before the messages", flush=True)
        send({{"op": "gather_bus", "bus": "0000:00:00.0"}})
        assert recv()["bus_ids"][0] == "0000:00:00.0"
        if mode == "midway":
            sys.exit(3)
        send({{"op": "barrier"}})
        recv()
        send({{"op": "barrier"}})
        recv()
        with open(os.path.join(d, "run_kernel_trace.csv"), "w") as f:
            f.write("Dispatch_Id,Kernel_Name,Start_Timestamp,End_Timestamp\\n")
            for i, dur in enumerate([9000000, 8400000, 8400000, 8400000, 7000000]):
                f.write(f"{{i + 1}},\\"{{tag}}\\",{{i * 20000000}},{{i * 20000000 + dur}}\\n")
        send({{"op": "device", "dev": {{
            "rank": 0, "world": 1, "device": 0, "bus_ids": ["0000:00:00.0"], "n_devices": 1, "shared_gpu": False,
            "cus": 256, "devname": "fake", "S": 12500, "N": 8, "C": 524288, "U": 8,
            "kernel": "xor_stream_w<8,8,strided,wpe6>", "kernel_tag": tag, "workload": "config2: fake",
            "bytes_per_step": 58982400000, "wall": 0.0252, "kern_ms": 8.4, "seg_ms": [8.4, 8.4, 8.4], "g": 1,
            "verified": True}}}})
        sys.exit(0)
    name = args[args.index("--pmc") + 1]
    assert "BCP_BENCH_PROFILED" not in os.environ and "RANK" not in os.environ
    with open(os.path.join(d, "run_counter_collection.csv"), "w") as f:
        f.write("Kernel_Name,Counter_Name,Counter_Value\\n")
        v = 25600000 if name == "FETCH_SIZE" else 6400000
        f.write(f"\\"{{tag}}\\",{{name}},{{v}}\\n")
''')


@pytest.fixture
def fake_rocprof(tmp_path, monkeypatch):
    b = tmp_path / "bin"
    b.mkdir()
    exe = b / "rocprofv3"
    exe.write_text(FAKE_ROCPROF.format(py=sys.executable))
    exe.chmod(exe.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setenv("PATH", f"{b}{os.pathsep}{os.environ['PATH']}")
    monkeypatch.delenv("BCP_BENCH_PROFILED", raising=False)
    monkeypatch.delenv("RANK", raising=False)
    return exe


def test_profiled_rank_patches_the_line(fake_rocprof, monkeypatch, capsys):
    """The device timing runs in the helper under the profiler, its collectives
    answered by the rank process; the rank process makes the line (legs off
    here) with the rocprof figures of the helper's own timed launches and the
    PMC traffic of the same workload, and says the timed launches were
    profiled."""
    import bench
    from bcp_dist import Dist
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "3", "--warmup", "1", "--no-e2e", "--no-cpu",
                                      "--no-configs"])
    a = bench.parse()
    a.stripes = 12_500
    assert bench.profiled_rank(a, Dist()) == 0
    out, err = capsys.readouterr()
    assert "noise before the messages" in err and "BCPDEV" not in out
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    rf = line["roofline"]
    live = rf["live_profile"]
    assert rf["profiled_in_process"] is True and line["config"]["verified_on_device"] is True
    assert live["in_process"] is True and live["rocprof_timed_launches"] == 3 and live["tagged_dispatches"] == 5
    assert live["rocprof_avg_ns"] == 8_400_000 and live["event_over_rocprof"] == 1.0
    assert rf["frac_rocprof"] == round(58982400000 / 8.4e-3 / 1e9 / 8000.0, 4)
    assert abs(rf["frac_event_over_rocprof"] - 1.0) < 0.005
    assert rf["traffic"] == 25600000 * 1024 * 2 + 6400000 * 1024 and rf["same_box"] is True
    assert rf["profile_box"] == rf["run_box"]
    assert 0.99 < live["traffic_over_algorithmic"] < 1.01
    assert line["value"] == round(58982400000 * 3 / 0.0252 / 1024 ** 3, 2)


@pytest.mark.parametrize("mode", ["fail", "midway"])
def test_profiled_rank_without_figures_times_in_process(fake_rocprof, monkeypatch, capsys, mode):
    """rocprofv3 exits with a status and no figures (before any message, or
    after its first collective -- at one rank both can be retried): the
    device phase runs in the rank process without the profiler (here it
    cannot: no GPU, so it fails loudly), and no line is made up."""
    import bench
    from bcp_dist import Dist
    monkeypatch.setenv("FAKE_ROCPROF_MODE", mode)  # no message at all / gone after its first collective
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "3", "--warmup", "1", "--no-e2e", "--no-cpu",
                                      "--no-configs"])
    a = bench.parse()
    a.stripes = 64
    with pytest.raises(AssertionError, match="needs a HIP device"):
        bench.profiled_rank(a, Dist())
    out, err = capsys.readouterr()
    assert not [x for x in out.splitlines() if x.startswith("{")]
    assert "without the profiler" in err


def test_profiled_rank_helper_lost_midway_fails_an_n_rank_job(fake_rocprof, monkeypatch, capsys):
    """In an N-rank job a helper gone after its first collective cannot be
    replaced (the other ranks are inside the job's collectives with it): the
    rank returns the helper's status, no line, no in-process retry."""
    import bench

    class TwoRanks:
        world, rank, local_rank = 2, 0, 0

        def gather(self, x):
            return [x, "0000:01:00.0"]

        def barrier(self):
            pass

        def close(self):
            pass
    monkeypatch.setenv("FAKE_ROCPROF_MODE", "midway")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "3", "--warmup", "1", "--no-e2e", "--no-cpu",
                                      "--no-configs"])
    a = bench.parse()
    a.stripes = 64
    assert bench.profiled_rank(a, TwoRanks()) == 3
    out, err = capsys.readouterr()
    assert not [x for x in out.splitlines() if x.startswith("{")]
    assert "in the middle of the run" in err
