#!/usr/bin/env python3
"""Readers and writers in one pool? (tools only).  The bench's 2 GiB e2e
block is bound by host CPU time (8 readers need ~41 ms
of the 50 ms run, 8 writers ~35 ms), so idle threads of one kind could carry
the other's jobs.  Two pipelines in one process, interleaved run by run over
the same in-memory stores: separate pools (8 readers + 8 writers, the
default before r4al) and one pool of 16 threads taking writes before reads
(BCP_PIPELINE_SHARED_IO=1 at creation; =2 the same pool in push order, =3
reads first, =0 the separate pools).  Config-5 shapes (2 GiB, as the
bench's e2e block) and config-1 shapes (4 targets, 3-wide, 512 KiB).

    python tools/exp/shared_io_ab.py --rounds 8
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3


def stores():
    rng = np.random.default_rng(5)
    c5, tot = [], 0
    while tot < 2 * GiB:
        i = len(c5)
        ls = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
        c5.append((f"e/{i % 64:02x}/c{i}", [t for t in range(9) if t != i % 9], i % 9, ls))
        tot += sum(ls)
    c1 = [(f"c1/{i % 16:02x}/f{i}", [t for t in range(4) if t != i % 4], i % 4, [512 * KiB] * 3) for i in range(1333)]
    return {"config5_2GiB": (9, c5), "config1": (4, c1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--dir", default="/dev/shm")
    a = ap.parse_args()
    work = {}
    for name, (nt, files) in stores().items():
        root = os.path.join(a.dir, f"bcp_shared_io_{name}")
        shutil.rmtree(root, ignore_errors=True)
        items, _ = S.populate(root, nt, files, seed=3)
        rd = sum(sum(f[3]) for f in files)
        wr = sum(8 * len(f[3]) + max(f[3]) for f in files)
        work[name] = (root, nt, items, rd + wr)
    pls = {}
    kinds = {"separate": "0", "shared_writes_first": "1", "shared_fifo": "2", "shared_reads_first": "3"}
    for kind, v in kinds.items():
        os.environ["BCP_PIPELINE_SHARED_IO"] = v
        pls[kind] = bcp.Pipeline(read_mode=bcp.READ_COPY)
    os.environ.pop("BCP_PIPELINE_SHARED_IO", None)
    res = {}
    try:
        for name, (root, nt, items, nbytes) in work.items():
            for kind in pls:  # warm both once
                pls[kind].run(root, nt, items)
            for r in range(a.rounds):
                order = list(kinds) if r % 2 == 0 else list(kinds)[::-1]
                for kind in order:
                    t0 = time.perf_counter()
                    st = pls[kind].run(root, nt, items)
                    dt = time.perf_counter() - t0
                    tm = pls[kind].last_timing()
                    assert st.errors == 0
                    res.setdefault((name, kind), []).append(dt)
                    print(json.dumps({"store": name, "round": r, "io": kind, "s": round(dt, 4),
                                      "GiBps": round(nbytes / dt / GiB, 2),
                                      "read_wait": tm["read_wait"], "slot_wait": tm["slot_wait"]}), flush=True)
        for (name, kind), ts in sorted(res.items()):
            med = float(np.median(ts))
            print(json.dumps({"summary": True, "store": name, "io": kind, "median_s": round(med, 4),
                              "GiBps": round(work[name][3] / med / GiB, 2), "runs": len(ts)}), flush=True)
    finally:
        for p in pls.values():
            p.close()
        for root, *_ in work.values():
            shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
