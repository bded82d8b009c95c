#!/usr/bin/env python3
"""Host memory kind of the P role's rows (tools/exp): config-5 gen over the
per-task protocol with the batched GPU fold and the reference CPU fold, the
CPU fold once over malloc'd rows and once over the same pinned mapped rows
the GPU uses (BCP_HOOK_PINNED_ROWS), for each BCP_MAPPED_FLAGS variant
(0 coherent, 1 non-coherent, 2 coherent + NUMA by policy, 3 both, 4 THP
malloc + hipHostRegister).  A warm-up run per variant (pinning) is dropped.
Interleaved rounds; one JSON line per (variant, fold)."""
import ctypes
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("beegfs-chunk-parity_amd", "oracle", "tools"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402
import oracle  # noqa: E402
from e2e_bench import total_bytes, write_store  # noqa: E402

KiB, MiB, GiB = 1024, 1024 ** 2, 1024 ** 3
root = "/dev/shm/bcp_kind"
shutil.rmtree(root, ignore_errors=True)
r5 = np.random.default_rng(5)
files = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 400):
    holders, p = S.random_layout(r5, 9, 8)
    lens = [int(x) for x in np.exp(r5.uniform(np.log(64 * KiB), np.log(4 * MiB), size=8))]
    files.append((f"u{i % 8}/{i:05d}", holders, p, lens))
write_store(root, files, 2)
items = [(path, 1_700_000_000, S.with_p(sum(1 << h for h in holders), p)) for path, holders, p, _ in files]
rd, wr = total_bytes(root, files)
cpu = ctypes.cast(oracle.lib().oracle_xor_rows, ctypes.c_void_p).value


def run():
    for k in range(9):
        shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
        os.makedirs(os.path.join(root, f"st{k}", "parity"))
    t0 = time.perf_counter()
    st = bcp.gen_run(root, 9, items, nlanes=12)
    assert st.errors == 0
    return time.perf_counter() - t0


res = {}
VARS = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "4"]
for rnd in range(4):
    for var in VARS:
        os.environ["BCP_MAPPED_FLAGS"] = var
        bcp.task_shutdown()  # drop pooled rows: the next allocations take the variant
        bcp.set_fold_mode(bcp.FOLD_BATCHED)
        run()  # warm-up: the variant's rows get allocated and pinned
        for fold in ("gpu_batched", "cpu_pinned_rows", "cpu_malloc_rows"):
            if fold == "gpu_batched":
                bcp.set_fold_mode(bcp.FOLD_BATCHED)
            else:
                bcp.set_xor_hook(cpu)
                if fold == "cpu_pinned_rows":
                    os.environ["BCP_HOOK_PINNED_ROWS"] = "1"
            try:
                dt = run()
            finally:
                bcp.set_xor_hook(None)
                os.environ.pop("BCP_HOOK_PINNED_ROWS", None)
            if rnd >= 0:
                res.setdefault((var, fold), []).append(dt)
for (var, fold), ts in sorted(res.items()):
    print(json.dumps({"mapped_flags": int(var), "fold": fold, "GiBps": round((rd + wr) / float(np.median(ts)) / GiB, 3),
                      "runs_s": [round(x, 4) for x in ts]}), flush=True)
bcp.task_shutdown()
shutil.rmtree(root, ignore_errors=True)
