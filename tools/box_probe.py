"""The box a measurement ran on (tools only): CPU model and counts, and the
host<->device copy rates of GPU 0 over pinned memory (hipMemcpyAsync through
the engine), so that runs from different boxes of the pool can be read side
by side.  Touches the GPU: not for processes that fork rank processes."""
import os
import time

import numpy as np


def cpu_info() -> dict:
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "cpu_quota": quota}


def pcie_rates(bcp, nbytes: int = 256 << 20, reps: int = 5) -> dict:
    eng = bcp.Engine(0)
    q = eng.queue()
    h = eng.host_alloc(nbytes)
    d = eng.alloc(nbytes)
    try:
        out = {}
        for name, fn in (("h2d_GBps", lambda: q.h2d(d, h, nbytes)), ("d2h_GBps", lambda: q.d2h(h, d, nbytes))):
            ts = []
            for _ in range(reps):
                q.sync()
                t0 = time.perf_counter()
                fn()
                q.sync()
                ts.append(time.perf_counter() - t0)
            out[name] = round(nbytes / float(np.median(ts)) / 1e9, 1)
        out["pci_bus_id"] = eng.pci_bus_id()
        return out
    finally:
        q.sync()
        eng.free(d)
        eng.host_free(h)
        q.close()
        eng.close()
