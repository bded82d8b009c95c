"""N>1 plumbing on CPU: world_size-2 gloo processes exercise the barrier and
the max/sum reductions bench.py uses, and the stripe sharding."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

import bcp_dist


def test_shard_range_covers_everything_once():
    for total in (0, 1, 7, 12500, 125000):
        for world in (1, 2, 3, 8):
            spans = [bcp_dist.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    # config 4: 125,000 stripes over 8 GPUs = 15,625 each
    assert all(b - a == 15625 for a, b in (bcp_dist.shard_range(125000, 8, r) for r in range(8)))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    d = bcp_dist.Dist()
    d.barrier()
    mx = d.max(float(rank + 1) * 1.5)
    sm = d.sum(float(rank + 1))
    ids = d.gather(f"0000:{rank % 1:02x}:00.0")  # two ranks on one device, as bench.py sees them
    d.barrier()
    d.close()
    q.put((rank, mx, sm, tuple(ids)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_gloo_world2_reductions():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[:3] for r in res] == [(0, 3.0, 3.0), (1, 3.0, 3.0)]
    assert all(r[3] == ("0000:00:00.0", "0000:00:00.0") for r in res)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(120)
def test_bench_gpus_n_refuses_without_enough_gpus():
    """`python3 bench.py --gpus 2` (the driver's form) with no GPU visible: a
    clear refusal with a non-zero exit, no bench line -- never a silent 1-GPU run."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--stripes", "8", "--no-cpu"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 4, (r.returncode, r.stderr[-2000:])
    assert "refusing" in r.stderr and "--allow-shared" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_gpus_n_launches_a_torchrun_child(monkeypatch):
    """--gpus N without WORLD_SIZE runs N ranks as a torchrun CHILD (never an
    exec), passes every argument through and returns the child's exit code."""
    import subprocess
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5", "--allow-shared"])
    a = bench.parse()
    assert bench.launch_ranks(a) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[-5:] == ["--gpus", "8", "--steps", "5", "--allow-shared"]
    assert cmd[-6].endswith("bench.py")
    assert seen["env"]["MASTER_ADDR"] == "127.0.0.1"


def _props(root, node, gfx, minor):
    d = os.path.join(root, "nodes", str(node))
    os.makedirs(d)
    with open(os.path.join(d, "properties"), "w") as f:
        f.write(f"cpu_cores_count 0\ngfx_target_version {gfx}\ndrm_render_minor {minor}\n")


def test_kfd_gpus_counts_usable_gpu_nodes_without_hip(tmp_path):
    """The launcher counts GPUs from KFD sysfs: GPU nodes (gfx_target_version
    > 0) whose render node is usable here; CPU nodes and GPUs of other
    containers (no render node) do not count; *_VISIBLE_DEVICES caps it."""
    sys.path.insert(0, ROOT)
    import bench
    root, dri = str(tmp_path / "kfd"), tmp_path / "dri"
    dri.mkdir()
    _props(root, 0, 0, 0)          # CPU node
    _props(root, 1, 90500, 128)    # this container's GPU
    _props(root, 2, 90500, 136)    # this container's GPU
    _props(root, 3, 90500, 144)    # another container's GPU: no render node here
    for m in (128, 136):
        (dri / f"renderD{m}").write_text("")
    nodes = os.path.join(root, "nodes")
    assert bench.kfd_gpus(nodes, str(dri), env={}) == 2
    assert bench.kfd_gpus(nodes, str(dri), env={"HIP_VISIBLE_DEVICES": "0"}) == 1
    assert bench.kfd_gpus(nodes, str(dri), env={"ROCR_VISIBLE_DEVICES": "0,1,2,3"}) == 2
    assert bench.kfd_gpus(str(tmp_path / "absent"), str(dri), env={}) == 0


def test_cpu_quota_caps_the_cpu_baseline_threads(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    import bench_legs
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert bench.cpu_quota(str(tmp_path)) == 16.0
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert bench.cpu_quota(str(tmp_path)) is None
    assert bench.cpu_quota(str(tmp_path / "none")) is None
    monkeypatch.setattr(bench_legs, "cpu_quota", lambda: 16.0)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    assert bench.usable_cpus() == (16, 256, 16.0)
    monkeypatch.setattr(bench_legs, "cpu_quota", lambda: None)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    assert bench.usable_cpus() == (8, 8, None)


def test_launcher_parent_never_imports_torch():
    """The launcher parent (bench.py --gpus N, no WORLD_SIZE) refuses or
    starts its ranks without importing torch or loading libbcp: nothing in it
    can initialise HIP."""
    import subprocess
    code = ("import sys, runpy; sys.argv = ['bench.py', '--gpus', '2', '--stripes', '8', '--no-cpu'];\n"
            "try:\n    runpy.run_path('bench.py', run_name='__main__')\n"
            "except SystemExit as e:\n    rc = e.code\n"
            "import bcp_ctypes\n"
            "print('RC', rc, 'TORCH', 'torch' in sys.modules, 'LIB', bcp_ctypes._lib is not None)\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert "RC 4 TORCH False LIB False" in r.stdout, (r.stdout, r.stderr[-2000:])


def test_e2e_store_dir_fits_every_rank(tmp_path, monkeypatch):
    """The end-to-end stores go where every rank's store fits: the asked
    directory, else the temp dir, else the roomiest, shrunk; a reason when
    nothing fits."""
    import collections
    sys.path.insert(0, ROOT)
    import bench
    GiB = 1 << 30
    free = {"/shm": 3 * GiB, "/tmpdir": 100 * GiB}
    St = collections.namedtuple("St", "f_bavail f_frsize")
    monkeypatch.setattr(os, "statvfs", lambda p: St(free[p] // 4096, 4096) if p in free else (_ for _ in ()).throw(
        FileNotFoundError(p)))
    import tempfile
    monkeypatch.setattr(tempfile, "gettempdir", lambda: "/tmpdir")
    assert bench.e2e_store_dir(["/shm"], 1, 1 * GiB) == ("/shm", 1 * GiB, None)
    base, want, why = bench.e2e_store_dir(["/shm"], 8, 2 * GiB)   # 8 x 2 GiB x 1.7 > 3 GiB
    assert base == "/tmpdir" and want == 2 * GiB and why is None
    free["/tmpdir"] = 1 * GiB
    base, want, why = bench.e2e_store_dir(["/shm"], 8, 2 * GiB)   # neither fits: the roomiest, shrunk
    assert base == "/shm" and want == int(3 * GiB / (1.7 * 8)) and why is None
    free["/shm"] = free["/tmpdir"] = 16 << 20
    assert bench.e2e_store_dir(["/shm"], 8, 2 * GiB)[2] is not None
    assert bench.e2e_store_dir(["/absent"], 1, GiB)[0] == "/tmpdir"


def test_bench_default_shard_and_label_per_world():
    """The driver's N = 8 run takes the config-4 branch: 125,000 stripes over 8
    ranks = 15,625 each, labelled config4; every other N runs config 2's
    12,500 per GPU; an explicit stripe count is never labelled config 4."""
    import bench
    for world in (1, 2, 4):
        assert all(bench.default_stripes(world, r) == 12_500 for r in range(world))
        assert bench.gen_config_label(world, 12_500) == "config2"
    shards = [bench.default_stripes(8, r) for r in range(8)]
    assert shards == [15_625] * 8 and sum(shards) * 8 == 1_000_000  # config 4: 1M chunks
    assert bench.gen_config_label(8, 15_625) == "config4"
    assert bench.gen_config_label(8, 64) == "config2" and bench.gen_config_label(4, 15_625) == "config2"
