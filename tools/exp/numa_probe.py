#!/usr/bin/env python3
"""Does it matter which NUMA node the host side of a GPU's pipeline lives on?
(tools only).  For each NUMA node of the box: bind this process to the node's
CPUs, allocate pinned staging (bcp_host_alloc: first touch by the calling
thread, so the pages land on that node), and time H2D / D2H of 256 MiB; then
a batched-pipeline gen over a 2 GiB config-5-shaped store in /dev/shm whose
files were written by threads on the same node.  One JSON line per node, plus
the GPU's own node from sysfs.  On an 8-GPU host one process per GPU would
bind to its GPU's node; this says what is at stake."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as S  # noqa: E402


def cpulist(text):
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def main():
    nodes = {}
    base = "/sys/devices/system/node"
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            nodes[int(d[4:])] = cpulist(open(os.path.join(base, d, "cpulist")).read())
    allowed = os.sched_getaffinity(0)
    eng = bcp.Engine(0)
    bus = eng.pci_bus_id().lower()
    try:
        gpu_node = int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
    except (OSError, ValueError):
        gpu_node = None
    eng.close()
    print(json.dumps({"nodes": {k: len(v) for k, v in nodes.items()}, "allowed": len(allowed), "gpu_bus": bus,
                      "gpu_numa_node": gpu_node}), flush=True)
    rng = np.random.default_rng(5)
    files, lens = [], []
    tot = 0
    while tot < (2 << 30):
        ls = [int(x) for x in np.exp(rng.uniform(np.log(64 << 10), np.log(4 << 20), size=8))]
        i = len(files)
        files.append((f"n/{i % 64:02x}/c{i}", [t for t in range(9) if t != i % 9], i % 9, ls))
        tot += sum(ls)
    for node, cpus in sorted(nodes.items()):
        use = cpus & allowed
        if not use:
            continue
        os.sched_setaffinity(0, use)
        eng = bcp.Engine(0)
        q = eng.queue()
        nb = 256 << 20
        h = eng.host_alloc(nb)
        dv = eng.alloc(nb)
        rates = {}
        for name, fn in (("h2d_GBps", lambda: q.h2d(dv, h, nb)), ("d2h_GBps", lambda: q.d2h(h, dv, nb))):
            tt = []
            for _ in range(7):
                q.sync()
                t0 = time.perf_counter()
                fn()
                q.sync()
                tt.append(time.perf_counter() - t0)
            rates[name] = round(nb / float(np.median(tt)) / 1e9, 2)
        eng.free(dv)
        eng.host_free(h)
        q.close()
        eng.close()
        root = f"/dev/shm/bcp_numa_{node}"
        items, _ = S.populate(root, 9, files, seed=node)
        rd = sum(sum(f[3]) for f in files)
        wr = sum(8 * 8 + max(f[3]) for f in files)
        pl = bcp.Pipeline()
        ts = []
        try:
            for _ in range(5):
                t0 = time.perf_counter()
                st = pl.run(root, 9, items)
                ts.append(time.perf_counter() - t0)
                assert st.errors == 0
        finally:
            pl.close()
            import shutil
            shutil.rmtree(root, ignore_errors=True)
        w = float(np.median(ts[1:]))
        print(json.dumps({"node": node, "cpus": len(use), "is_gpu_node": node == gpu_node, **rates,
                          "pipeline_gen_warm_s": round(w, 4), "pipeline_gen_GiBps": round((rd + wr) / w / 2**30, 2),
                          "runs": [round(x, 4) for x in ts]}), flush=True)
    os.sched_setaffinity(0, allowed)


if __name__ == "__main__":
    main()
