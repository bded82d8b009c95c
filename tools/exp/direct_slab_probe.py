#!/usr/bin/env python3
"""Does O_DIRECT read into each kind of pinned slab, on each filesystem of the
box? (tools only).  A small config-5-shaped store on tmpfs and on the working
directory's filesystem; the batched pipeline in DIRECT read mode over slabs
of registered THP memory (BCP_HOST_REGISTERED=1, the default) and of
hipHostMalloc'd memory (=0): bytes read with O_DIRECT, pieces that fell back
to the page cache, and the warm rate.  One JSON line per case."""
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


def main():
    rng = np.random.default_rng(3)
    files, tot = [], 0
    while tot < (1 << 30):
        i = len(files)
        ls = [int(x) for x in np.exp(rng.uniform(np.log(64 << 10), np.log(4 << 20), size=8))]
        files.append((f"p/{i % 32:02x}/c{i}", [t for t in range(9) if t != i % 9], i % 9, ls))
        tot += sum(ls)
    for where in ("/dev/shm/bcp_direct_probe", os.path.join(os.getcwd(), "bcp_direct_probe")):
        items, _ = S.populate(where, 9, files, seed=1)
        try:
            fs = os.statvfs(where)
            for reg in ("1", "0"):
                os.environ["BCP_HOST_REGISTERED"] = reg
                pl = bcp.Pipeline(read_mode=bcp.READ_DIRECT)
                try:
                    ts = []
                    for _ in range(4):
                        t0 = time.perf_counter()
                        st = pl.run(where, 9, items)
                        ts.append(time.perf_counter() - t0)
                        assert st.errors == 0
                    tm = pl.last_timing()
                finally:
                    pl.close()
                print(json.dumps({"store": where, "f_bsize": fs.f_bsize, "slab": "registered" if reg == "1" else
                                  "hipHostMalloc", "bytes_read": st.bytes_read, "direct_bytes": tm["direct_bytes"],
                                  "direct_fallbacks": tm["direct_fallbacks"], "read_jobs": tm["read_jobs"],
                                  "warm_s": round(float(np.median(ts[1:])), 4),
                                  "input_GiBps": round(st.bytes_read / float(np.median(ts[1:])) / 2**30, 2)}),
                      flush=True)
        finally:
            shutil.rmtree(where, ignore_errors=True)
    os.environ.pop("BCP_HOST_REGISTERED", None)


if __name__ == "__main__":
    main()
