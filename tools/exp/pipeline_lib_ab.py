#!/usr/bin/env python3
"""A/B of two libbcp builds on the batched pipeline (tools only).

  --make ROOT            write the stores once: config 1 (4 targets, 1333 x 3 x
                         512 KiB) and config 5 (9 targets, 1000 x 8 log-uniform
                         64 KiB-4 MiB chunks) plus the seeded 10 % subset of
                         config 5 that a changelog round recomputes
  --run ROOT --label L   in THIS process (the library bcp_ctypes loads: $BCP_LIB
                         or the in-tree build) time each workload -- one cold
                         run, then --reps warm runs, median -- check sampled
                         parity files against the oracle, print one JSON line
                         per workload with the pipeline's stage timing

tools/exp/pipeline_lib_ab.sh alternates processes of the two builds on one box.
Rates: (chunk bytes read + parity bytes written) / wall time, page-cache stores.
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402

import bcp_store as S  # noqa: E402

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3


def layouts():
    c1 = []
    for i in range(1333):
        p = i % 4
        c1.append((f"u0/{i % 64:02X}/chunk{i}", [t for t in range(4) if t != p], p, [512 * KiB] * 3))
    rng = np.random.default_rng(5)
    c5 = []
    for i in range(1000):
        holders, p = S.random_layout(rng, 9, 8)
        lens = [int(x) for x in np.exp(rng.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
        c5.append((f"u{i % 8}/{(i * 2654435761) % 65536:04X}/chunk{i}", holders, p, lens))
    sub = sorted(int(x) for x in np.random.default_rng(6).choice(len(c5), size=len(c5) // 10, replace=False))
    return {"config1": (4, c1), "config5_full": (9, c5), "config5_subset10": (9, [c5[i] for i in sub])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--make")
    ap.add_argument("--run")
    ap.add_argument("--label", default="")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    L = layouts()
    if a.make:
        from e2e_bench import write_store
        for name in ("config1", "config5_full"):
            root = os.path.join(a.make, name)
            shutil.rmtree(root, ignore_errors=True)
            write_store(root, L[name][1], 1 if name == "config1" else 2)
        print(json.dumps({"stores": a.make}), flush=True)
        return
    import ctypes
    import bcp_ctypes as bcp
    import oracle
    # an older build lacks the newer entry points (bcp_pipeline_last_timing):
    # bind only what it exports (an A/B tool; the product binds everything)
    probe = ctypes.CDLL(bcp.LIB_PATH)
    for name in [n for n in bcp._SIGS if not hasattr(probe, n)]:
        del bcp._SIGS[name]
    nslots = int(os.environ.get("PLAB_NSLOTS", "4"))  # the .sh's "lib@nslots" entries
    pl = bcp.Pipeline(nslots=nslots)
    try:
        for name, (nt, files) in L.items():
            root = os.path.join(a.run, "config1" if name == "config1" else "config5_full")
            items = [(p, 2 ** 40, S.with_p(sum(1 << h for h in hs), P)) for p, hs, P, _ in files]
            rd = sum(sum(ls) for *_, ls in files)
            wr = sum(8 * len(ls) + max(ls) for *_, ls in files)
            ts = []
            for _ in range(1 + a.reps):
                t0 = time.perf_counter()
                st = pl.run(root, nt, items)
                ts.append(time.perf_counter() - t0)
                if st.errors:
                    sys.exit(f"{name}: {st.errors} errors")
            tm = pl.last_timing() if "bcp_pipeline_last_timing" in bcp._SIGS else None
            bad = 0
            for i in np.random.default_rng(1).choice(len(files), size=min(12, len(files)), replace=False):
                path, hs, P, _ = files[i]
                chunks = [np.fromfile(S.chunk_path(root, h, path), dtype=np.uint8) for h in hs]
                bad += S.read_file(S.parity_path(root, P, path)) != oracle.gen_parity_file(chunks)
            w = float(np.median(ts[1:]))
            print(json.dumps({"label": a.label, "lib": os.environ.get("BCP_LIB", "in-tree"), "nslots": nslots,"workload": name,
                              "stripes": len(files), "warm_s": round(w, 5), "GiBps": round((rd + wr) / w / GiB, 2),
                              "cold_s": round(ts[0], 5), "runs": [round(x, 5) for x in ts], "timing": tm,
                              "verified": bad == 0}), flush=True)
            if bad:
                sys.exit(3)
    finally:
        pl.close()


if __name__ == "__main__":
    main()
