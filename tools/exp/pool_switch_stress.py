#!/usr/bin/env python3
"""Stress (tools/exp): the per-task protocol switching fold modes round after
round, optionally tearing the engines, fold services and row pool down after
every round (--shutdown: freed memory's addresses are re-issued) and running
the batched pipeline over the same files (--pipeline) -- the r02 fault
hunt's run (tests/test_gpu_protocol.py
::test_pool_reuse_with_changing_data_and_teardown, longer).  On a mismatch it
describes the wrong bytes: ranges, zeros or not, and whether the got bytes
equal the XOR of a subset of the sources (a source missing from the fold)."""
import argparse
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402  (the checker)


def emit(**kw):
    print(json.dumps(kw), flush=True)


def ranges(mask):
    idx = np.flatnonzero(mask)
    if idx.size == 0:
        return []
    cuts = np.flatnonzero(np.diff(idx) > 1)
    starts = np.concatenate([[idx[0]], idx[cuts + 1]])
    ends = np.concatenate([idx[cuts], [idx[-1]]])
    return [[int(a), int(b) + 1] for a, b in zip(starts[:8], ends[:8])]


def describe(got, want, chunks):
    n = len(chunks)
    g = np.frombuffer(got, np.uint8)[8 * n:]
    w = np.frombuffer(want, np.uint8)[8 * n:]
    m = min(g.size, w.size)
    bad = g[:m] != w[:m]
    info = dict(len_got=len(got), len_want=len(want), nbad=int(bad.sum()), ranges=ranges(bad),
                header_ok=got[:8 * n] == want[:8 * n], chunk_lens=[int(c.size) for c in chunks])
    if bad.any():
        gb = g[:m][bad]
        info["bad_zero_frac"] = round(float((gb == 0).mean()), 3)
        idx = np.flatnonzero(bad)
        subsets = []
        for mask in range(1 << n):
            acc = np.zeros(idx.size, np.uint8)
            for j, c in enumerate(chunks):
                if mask >> j & 1:
                    sel = idx < c.size
                    acc[sel] ^= c[idx[sel]]
            if np.array_equal(acc, gb):
                subsets.append(mask)
        info["got_equals_xor_of_subsets"] = subsets
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/dev/shm/bcp_switch")
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--shutdown", action="store_true", help="bcp_task_shutdown after every round")
    ap.add_argument("--pipeline", action="store_true", help="a pipeline gen of the same files every round")
    a = ap.parse_args()
    bcp.set_xor_hook(None)
    rng = np.random.default_rng(77)
    cycle = [bcp.FOLD_PIPELINED, bcp.FOLD_BATCHED]
    names = {bcp.FOLD_BATCHED: "batched", bcp.FOLD_PIPELINED: "pipelined"}
    fails = 0
    for rnd in range(a.rounds):
        mode = cycle[rnd % len(cycle)]
        shutil.rmtree(a.root, ignore_errors=True)
        files = [(f"z/{i}", [0, 1, 2], 3, [int(x) for x in rng.integers(1, 600_000, size=3)]) for i in range(24)]
        items, contents = S.populate(a.root, 4, files, seed=100 + rnd)
        prev = bcp.set_fold_mode(mode)
        try:
            st = bcp.gen_run(a.root, 4, items, nlanes=6)
        finally:
            bcp.set_fold_mode(prev)
        bad = []
        for (path, holders, p, lens) in files:
            got = S.read_file(S.parity_path(a.root, p, path))
            want = oracle.gen_parity_file(contents[path])
            if got != want:
                bad.append(dict(path=path, **describe(got, want, contents[path])))
        if a.pipeline:
            pst = bcp.pipeline_gen(a.root, 4, items)
            for (path, holders, p, lens) in files:
                got = S.read_file(S.parity_path(a.root, p, path))
                want = oracle.gen_parity_file(contents[path])
                if got != want:
                    bad.append(dict(path=path, engine="pipeline", **describe(got, want, contents[path])))
            if pst.errors:
                bad.append(dict(engine="pipeline", errors=pst.errors))
        if a.shutdown:
            bcp.task_shutdown()
        fails += bool(bad)
        emit(round=rnd, mode=names[mode], errors=st.errors, bad_files=len(bad), detail=bad[:3])
        if bad:
            break  # stop at the first wrong round: never run on into a fault
    shutil.rmtree(a.root, ignore_errors=True)
    bcp.task_shutdown()
    emit(summary=True, rounds=rnd + 1, failing_rounds=fails)


if __name__ == "__main__":
    main()
