"""The producers around a round and the command-line front end:
bcp_scan_chunks (bp-find-all-chunks, src/bp-find-all-chunks/main.c:17-45),
bcp_check_targets (gen/main.c:472-551) and bin/bcp.  GPU runs of the CLI
are in test_gpu_protocol.py."""
import os
import struct
import subprocess

import numpy as np
import pytest

import bcp_store as S
import planner as PL


def walk_records(chunks_dir):
    out = {}
    for dp, _, fns in os.walk(chunks_dir):
        for fn in fns:
            full = os.path.join(dp, fn)
            st = os.lstat(full)
            out[os.path.relpath(full, chunks_dir).encode()] = (int(st.st_mtime), st.st_size)
    return out


def make_chunks(root, rng, ntargets, nfiles):
    S.make_store(root, ntargets)
    for i in range(nfiles):
        for h in rng.choice(ntargets, size=int(rng.integers(1, ntargets)), replace=False):
            S.write_chunk(root, int(h), f"u{i % 3}/{i:03X}/c{i}", S.synthetic_chunk(i, int(rng.integers(0, 5000))))


def test_find_all_chunks_stream(bcp, tmp_path):
    rng = np.random.default_rng(0)
    make_chunks(str(tmp_path), rng, 3, 40)
    cdir = os.path.join(str(tmp_path), "st1", "chunks")
    out = subprocess.run([bcp.BIN_PATH, "find-all-chunks", cdir], check=True, capture_output=True).stdout
    recs = PL.parse_records(out)
    got = {p: (ts, sz) for ts, sz, ev, p in recs}
    assert all(ev == ord("m") for _, _, ev, _ in recs)
    assert got == walk_records(cdir) and len(recs) == len(got)
    # trailing slash and the library entry give the same stream
    out2 = subprocess.run([bcp.BIN_PATH, "find-all-chunks", cdir + "/"], check=True, capture_output=True).stdout
    assert sorted(PL.parse_records(out2)) == sorted(recs)


def test_eventset_scan_matches_fed_stream(bcp, tmp_path):
    rng = np.random.default_rng(1)
    root = str(tmp_path)
    make_chunks(root, rng, 4, 60)
    a, b = bcp.EventSet(), bcp.EventSet()
    for k in range(4):
        cdir = os.path.join(root, f"st{k}", "chunks")
        a.scan(k, cdir)
        b.feed(k, subprocess.run([bcp.BIN_PATH, "find-all-chunks", cdir], check=True, capture_output=True).stdout)
    assert sorted(a.entries()) == sorted(b.entries())
    ent = {p: m for p, _, m, _, _ in a.entries()}
    for k in range(4):
        for p in walk_records(os.path.join(root, f"st{k}", "chunks")):
            assert ent[p.decode()] & (1 << k)
    a.close()
    b.close()


def test_check_targets_bookkeeping(bcp, tmp_path):
    root, rd = str(tmp_path), str(tmp_path / "run_data")
    S.make_store(root, 3)
    for k, tid in enumerate((101, 102, 103)):
        (tmp_path / f"st{k}" / "targetNumID").write_text(f"{tid}\n")
    bcp.check_targets(root, 3, rd)
    bcp.check_targets(root, 3, rd)                   # same targets: fine
    S.make_store(root, 4)
    (tmp_path / "st3" / "targetNumID").write_text("104")
    bcp.check_targets(root, 4, rd)                   # a target added: fine
    with pytest.raises(bcp.BcpError):                # "Fewer targets than last run"
        bcp.check_targets(root, 3, rd)
    (tmp_path / "st1" / "targetNumID").write_text("999")
    with pytest.raises(bcp.BcpError):                # "Storage target missing!"
        bcp.check_targets(root, 4, rd)
    (tmp_path / "st1" / "targetNumID").write_text("101")
    with pytest.raises(bcp.BcpError):                # "Duplicate targetNumID"
        bcp.check_targets(root, 4, str(tmp_path / "other"))


def test_run_data_stamp_is_the_file_format_not_the_abi(bcp, tmp_path):
    """run_data carries its own format stamp (1), independent of
    the struct ABI; a store the r04 build stamped 2 still passes (the format
    is the same) and is rewritten as 1; any other stamp is refused."""
    import struct
    root, rd = str(tmp_path), tmp_path / "run_data"
    S.make_store(root, 3)
    bcp.check_targets(root, 3, str(rd))
    raw = bytearray(rd.read_bytes())
    assert raw[:8] == b"BCPRUN01" and struct.unpack_from("<I", raw, 8)[0] == 1
    struct.pack_into("<I", raw, 8, 2)                # as the r04 build wrote it
    rd.write_bytes(bytes(raw))
    bcp.check_targets(root, 3, str(rd))
    assert struct.unpack_from("<I", rd.read_bytes(), 8)[0] == 1
    struct.pack_into("<I", raw, 8, 7)
    rd.write_bytes(bytes(raw))
    with pytest.raises(bcp.BcpError):                # "Version mismatch"
        bcp.check_targets(root, 3, str(rd))


def test_read_and_fold_flags_only_with_their_engine(bcp, tmp_path):
    """--read names a pipeline read path, --fold a protocol P-role
    fold; given to the other engine they would be ignored, so they are refused."""
    S.make_store(str(tmp_path), 3)
    for cmd in (["parity-gen", "--complete", "--protocol", "--read", "copy", str(tmp_path), "3"],
                ["parity-gen", "--complete", "--procs", "--read", "direct", str(tmp_path), "3"],
                ["parity-gen", "--complete", "--fold", "batched", str(tmp_path), "3"],
                ["parity-rebuild", "--protocol", "--read", "copy", str(tmp_path), "3", "1"],
                ["parity-rebuild", "--pipeline", "--fold", "batched", str(tmp_path), "3", "1"],
                ["parity-gen", "--complete", "--read", "map", str(tmp_path), "3"]):   # MAP: removed in ABI 3
        r = subprocess.run([bcp.BIN_PATH, *cmd], capture_output=True)
        assert r.returncode == 1 and b"usage" in r.stderr, cmd
    assert not os.path.exists(tmp_path / "run_data")  # refused before touching the store


def test_pipeline_refuses_the_removed_map_read_mode(bcp):
    """read_mode 2 (MAP, ABI 2) is rejected before any device is touched."""
    import ctypes
    opts = bcp.PipelineOpts(0, 1 << 20, 1, 2, 1, 2)
    pl = ctypes.c_void_p()
    assert bcp.lib().bcp_pipeline_create(ctypes.byref(opts), ctypes.byref(pl)) == -22
    assert not pl.value


def test_cli_usage_and_loud_failure_without_gpu(bcp, tmp_path):
    r = subprocess.run([bcp.BIN_PATH], capture_output=True)
    assert r.returncode == 1 and b"usage" in r.stderr
    r = subprocess.run([bcp.BIN_PATH, "parity-gen", str(tmp_path), "3"], capture_output=True)
    assert r.returncode == 1                         # neither --complete nor --partial
    for bad in (["--read", "mmap"], ["--read"]):     # an unknown read path, a missing one
        r = subprocess.run([bcp.BIN_PATH, "parity-gen", "--complete", *bad, str(tmp_path), "3"], capture_output=True)
        assert r.returncode == 1 and b"usage" in r.stderr
    if bcp.device_count() > 0:
        pytest.skip("GPU present: the GPU run is in test_gpu_protocol.py")
    rng = np.random.default_rng(2)
    make_chunks(str(tmp_path), rng, 3, 5)
    r = subprocess.run([bcp.BIN_PATH, "parity-gen", "--complete", str(tmp_path), "3"], capture_output=True)
    assert r.returncode == 1                         # no device: P ranks fail, no silent CPU path
    assert not os.path.exists(tmp_path / "last-gen-timestamp")
