"""Randomised worklists through the whole per-task protocol and the batched
pipeline on the device, for a time budget (BCP_FUZZ_SECONDS, default 8 s; the
same test with a larger budget is a soak).  Each round draws a store (3..16
targets), a worklist (widths 1..15, chunk lengths from 0 B to 4 MiB, now and
then past the 10 MiB transfer window so sources replay their last window,
quirk A3-q1; a chunk file missing after planning), the P-role fold
(pipelined through the fold ring -- with a random deferral depth, number of
completion threads, transport spin and range shape -- pipelined on the
lanes' queues, or batched) or the pipeline, the lanes, the padding rule on the
wire (implicit / the reference's) and the fold service width; every parity
file must equal the oracle's (oracle.gen_parity_file, the reference's
parity_generator restated).  Then a random target is lost and rebuilt by
the protocol (1..4 rebuild lanes) or the pipeline (either read path, COPY or
DIRECT); every lost chunk of a
stripe without a missing chunk must come back byte for byte."""
import os
import shutil
import time

import numpy as np
import pytest

import bcp_store as S

pytestmark = pytest.mark.gpu
KiB, MiB = 1024, 1024 * 1024


@pytest.fixture(autouse=True)
def gpu_fold(bcp, engine):
    bcp.set_xor_hook(None)  # the product path: fold on the device
    yield
    bcp.task_shutdown()


def _length(rng, allow_big):
    r = rng.random()
    if r < 0.05:
        return 0
    if r < 0.15:
        return int(rng.integers(1, 65))
    if r < 0.75:
        return int(rng.integers(1, 700 * KiB))
    if r < 0.97 or not allow_big:
        return int(rng.integers(1 * MiB, 4 * MiB + 1))
    return int(rng.integers(10 * MiB + 1, 24 * MiB))        # past the window: replay


def _worklist(rng, ntargets):
    files, big = [], 0
    for i in range(int(rng.integers(4, 31))):
        wmax = min(15, ntargets - 1) if rng.random() < 0.2 else min(8, ntargets - 1)
        width = int(rng.integers(1, wmax + 1))
        holders, p = S.random_layout(rng, ntargets, width)
        lens = [_length(rng, big < 2) for _ in range(width)]
        big += sum(L > 10 * MiB for L in lens)
        files.append((f"d{i % 5}/{int(rng.integers(0, 1 << 16)):04x}/c{i}", holders, p, lens))
    return files


def test_random_rounds_match_the_oracle(bcp, oracle, tmp_path):
    fuzz_rounds(bcp, oracle, tmp_path, float(os.environ.get("BCP_FUZZ_SECONDS", "8")),
                int(os.environ.get("BCP_FUZZ_SEED", "3")), ("pipelined", "pipelined_queues", "batched", "pipeline"))


def fuzz_rounds(bcp, oracle, tmp_path, budget, seed, engines):
    rng = np.random.default_rng(seed)
    prev = (bcp.set_fold_mode(bcp.FOLD_PIPELINED), bcp.set_rebuild_lanes(1), bcp.set_explicit_padding(bcp.PAD_AUTO),
            bcp.set_fold_inflight(1), bcp.set_fold_ring(True))
    prev_tuning = {}
    for k, probe in (("defer_depth", 1), ("completion_threads", 4), ("lb_spin_us", 0), ("pipe_piece_kib", 256),
                     ("pipe_step_kib", 128)):
        prev_tuning[k] = bcp.set_fold_tuning(k, probe)  # (read by setting; restored below)
        bcp.set_fold_tuning(k, prev_tuning[k])
    t_end = time.monotonic() + budget
    rounds = files_done = 0
    seen = set()
    try:
        while time.monotonic() < t_end or rounds < 2:
            root = str(tmp_path / f"r{rounds}")
            ntargets = int(rng.integers(3, 17))
            files = _worklist(rng, ntargets)
            items, contents = S.populate(root, ntargets, files, seed=seed * 1000 + rounds)
            missing = set()
            if rng.random() < 0.3:  # a chunk file gone after planning: its source sends zeros, size 0
                path, holders, p, lens = files[int(rng.integers(0, len(files)))]
                k = int(rng.integers(0, len(holders)))
                os.remove(S.chunk_path(root, holders[k], path))
                contents[path][k] = None
                missing.add(path)
            how = str(rng.choice(list(engines)))
            pad = int(rng.choice([bcp.PAD_AUTO, 1]))
            bcp.set_explicit_padding(pad)
            bcp.set_fold_inflight(int(rng.choice([1, 1, 2, 4])))
            what = f"seed {seed} round {rounds} {how} pad {pad}"
            if how in ("pipelined", "procs"):  # the ring's deferral, completion threads, transport waits, range shape
                tn = {"defer_depth": int(rng.integers(1, 5)), "completion_threads": int(rng.choice([0, 1, 4])),
                      "lb_spin_us": int(rng.choice([0, 0, 20])), "pipe_piece_kib": int(rng.choice([64, 256, 1024])),
                      "pipe_step_kib": int(rng.choice([32, 128]))}
                for k, v in tn.items():
                    bcp.set_fold_tuning(k, v)
                what += f" {tn}"
            read_mode = int(rng.choice([bcp.READ_AUTO, bcp.READ_COPY, bcp.READ_DIRECT]))  # the pipeline's read path
            if how == "pipeline":
                what += f" read_mode {read_mode}"
                if rng.random() < 0.3:  # a cold store: written back and dropped (AUTO then reads with O_DIRECT)
                    what += " cold"
                    for path, holders, _, _ in files:
                        for h in holders:
                            c = S.chunk_path(root, h, path)
                            if os.path.exists(c):
                                fd = os.open(c, os.O_RDONLY)
                                os.fsync(fd)
                                os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
                                os.close(fd)
                st = bcp.pipeline_gen(root, ntargets, items, slab_bytes=int(rng.choice([1, 8, 64])) << 20,
                                      io_threads=int(rng.integers(1, 9)), nslots=int(rng.integers(2, 5)),
                                      read_mode=read_mode)
            elif how == "procs":  # every rank its own process (socketpair transport), P roles fold pipelined
                bcp.set_fold_mode(bcp.FOLD_PIPELINED)
                st = bcp.gen_run_procs(root, ntargets, items, nlanes=int(rng.integers(1, 13)))
            else:
                # pipelined: through the device's fold ring (lane deferral in the runner's lanes);
                # pipelined_queues: range launches on the lanes' queues
                bcp.set_fold_mode(bcp.FOLD_BATCHED if how == "batched" else bcp.FOLD_PIPELINED)
                bcp.set_fold_ring(how != "pipelined_queues")
                st = bcp.gen_run(root, ntargets, items, nlanes=int(rng.integers(1, 13)))
            assert st.errors == 0, what
            for (path, holders, p, lens) in files:
                want = oracle.gen_parity_file(contents[path])
                assert S.read_file(S.parity_path(root, p, path)) == want, (what, path, lens)
            victim = int(rng.integers(0, ntargets))
            lost = {}
            for (path, holders, p, lens) in files:
                if victim in holders and path not in missing:
                    lost[path] = S.read_file(S.chunk_path(root, victim, path))
                    os.remove(S.chunk_path(root, victim, path))
            ordered = sorted(items, key=lambda x: x[0].encode())  # a DB walk: key order
            if how == "pipeline" and rng.random() < 0.7:
                pl = bcp.Pipeline(io_threads=int(rng.integers(1, 9)), read_mode=read_mode)
                try:
                    st = pl.rebuild(root, ntargets, victim, ordered)
                finally:
                    pl.close()
                rb = "pipeline"
            else:
                bcp.set_rebuild_lanes(int(rng.integers(1, 5)))
                st = (bcp.rebuild_run_procs if how == "procs" else bcp.rebuild_run)(root, ntargets, victim, ordered)
                bcp.set_rebuild_lanes(1)
                rb = "procs" if how == "procs" else "protocol"
            assert st.errors == 0, (what, rb)
            for path, data in lost.items():
                assert S.read_file(S.chunk_path(root, victim, path)) == data, (what, rb, path)
            seen.add((how, rb))
            rounds += 1
            files_done += len(files)
            if rounds % 100 == 0:
                print(f"protocol fuzz: {rounds} rounds ...", flush=True)  # progress for long soaks
            shutil.rmtree(root, ignore_errors=True)
    finally:
        for k, v in prev_tuning.items():
            bcp.set_fold_tuning(k, v)
        bcp.set_fold_mode(prev[0])
        bcp.set_rebuild_lanes(prev[1])
        bcp.set_explicit_padding(prev[2])
        bcp.set_fold_inflight(prev[3])
        bcp.set_fold_ring(prev[4])
    print(f"protocol fuzz: {rounds} rounds, {files_done} stripes, engines {sorted(seen)}")
    assert rounds >= 2
