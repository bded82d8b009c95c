#!/usr/bin/env python3
"""Config 1 gen through the per-task protocol with a fold that does nothing
(no GPU needed): CPU seconds per run (getrusage over all threads, user and
system apart) and wall time, against lanes per rank, so the protocol's own
host cost can be measured and cut where it is paid (r05: on the GPU boxes
the protocol burns 1.4-1.5 CPU-seconds per config-1 gen run, ~22 cores busy
under a 16-CPU quota, whatever the fold; tools/proto_compare.py r5u).  The
`copies` leg reads every chunk file and writes every parity file of the same
run from --copy-threads C threads with nothing else: the kernel-copy floor.

  python tools/exp/c1_cpu_cost.py --rounds 5 --lanes 12,4
"""
import argparse
import concurrent.futures as cf
import ctypes
import json
import os
import resource
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import numpy as np  # noqa: E402

import bcp_ctypes as bcp  # noqa: E402
import bcp_store as BS  # noqa: E402

KiB, GiB = 1024, 1024 ** 3


def noop_hook():
    tmp = tempfile.mkdtemp(dir="/tmp")
    src = os.path.join(tmp, "noop.c")
    open(src, "w").write("#include <stddef.h>\n#include <stdint.h>\nint noop_fold(uint8_t *d, size_t n, const uint8_t"
                         " *s, size_t p, int k, void *c) { (void)d; (void)n; (void)s; (void)p; (void)k; (void)c;"
                         " return 0; }\n")
    so = os.path.join(tmp, "libnoop.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    return lib, ctypes.cast(lib.noop_fold, ctypes.c_void_p).value


COPY_FLOOR_C = r"""
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
typedef struct { const char *root; int files, nt, k, nth; size_t c; int rc; } job;
static void *run(void *p)
{
    job *j = p;
    char fn[512];
    char *b = malloc(24 + j->c);
    memset(b, 0, 24 + j->c);
    for (int i = j->k; i < j->files; i += j->nth) {
        const int P = i % j->nt;
        for (int h = 0; h < j->nt; h++) {
            if (h == P)
                continue;
            snprintf(fn, sizeof fn, "%s/st%d/chunks/u0/%02X/chunk%d", j->root, h, i % 64, i);
            int fd = open(fn, O_RDONLY);
            if (fd < 0 || read(fd, b + 24, j->c) != (ssize_t)j->c) { j->rc = 1; return NULL; }
            close(fd);
        }
        snprintf(fn, sizeof fn, "%s/st%d/parity/u0", j->root, P);
        mkdir(fn, 0755);
        snprintf(fn, sizeof fn, "%s/st%d/parity/u0/%02X", j->root, P, i % 64);
        mkdir(fn, 0755);
        snprintf(fn, sizeof fn, "%s/st%d/parity/u0/%02X/chunk%d", j->root, P, i % 64, i);
        int fd = open(fn, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0 || write(fd, b, 24 + j->c) != (ssize_t)(24 + j->c)) { j->rc = 2; return NULL; }
        close(fd);
    }
    free(b);
    return NULL;
}
int c1_copies(const char *root, int files, int nt, size_t c, int nth)
{
    pthread_t t[256];
    job j[256];
    for (int k = 0; k < nth; k++) {
        j[k] = (job){root, files, nt, k, nth, c, 0};
        pthread_create(&t[k], NULL, run, &j[k]);
    }
    int rc = 0;
    for (int k = 0; k < nth; k++) {
        pthread_join(t[k], NULL);
        rc |= j[k].rc;
    }
    return rc;
}
"""


def copy_floor_lib():
    tmp = tempfile.mkdtemp(dir="/tmp")
    src = os.path.join(tmp, "floor.c")
    open(src, "w").write(COPY_FLOOR_C)
    so = os.path.join(tmp, "libfloor.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-pthread", "-o", so, src], check=True)
    lib = ctypes.CDLL(so)
    lib.c1_copies.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1333)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--lanes", default="12")
    ap.add_argument("--dir", default="/dev/shm")
    ap.add_argument("--copy-threads", type=int, default=16)
    a = ap.parse_args()
    NT, C = 4, 512 * KiB
    root = os.path.join(a.dir, f"c1cpu_{os.getpid()}")
    rng = np.random.default_rng(1)
    block = rng.integers(0, 256, size=8 << 20, dtype=np.uint8)
    files = [(f"u0/{i % 64:02X}/chunk{i}", [t for t in range(NT) if t != i % NT], i % NT) for i in range(a.files)]
    items = [(p, 2 ** 40, BS.with_p(sum(1 << h for h in hs), pp)) for p, hs, pp in files]
    BS.make_store(root, NT)

    def write_file(i):
        path, holders, _ = files[i]
        for k, h in enumerate(holders):
            fn = BS.chunk_path(root, h, path)
            os.makedirs(os.path.dirname(fn), exist_ok=True)
            off = ((i * 3 + k) * 40961) % ((8 << 20) - C)
            with open(fn, "wb") as f:
                f.write(memoryview(block[off:off + C]))
    with cf.ThreadPoolExecutor(8) as ex:
        list(ex.map(write_file, range(a.files)))
    nbytes = a.files * 3 * C + a.files * (24 + C)
    _keep, hook = noop_hook()
    bcp.set_xor_hook(hook)

    def reset():
        for k in range(NT):
            shutil.rmtree(os.path.join(root, f"st{k}", "parity"), ignore_errors=True)
            os.makedirs(os.path.join(root, f"st{k}", "parity"))
    floor = copy_floor_lib()
    lanes = [int(x) for x in a.lanes.split(",")] + ["copies"]
    res = {n: [] for n in lanes}
    for r in range(1 + a.rounds):
        for n in lanes[r % len(lanes):] + lanes[:r % len(lanes)]:
            reset()
            ru0 = resource.getrusage(resource.RUSAGE_SELF)
            t0 = time.perf_counter()
            if n == "copies":
                rc = floor.c1_copies(root.encode(), a.files, NT, C, a.copy_threads)
                assert rc == 0, rc
                st = None
            else:
                st = bcp.gen_run(root, NT, items, nlanes=n)
            dt = time.perf_counter() - t0
            ru1 = resource.getrusage(resource.RUSAGE_SELF)
            assert st is None or st.errors == 0
            res[n].append((dt, ru1.ru_utime - ru0.ru_utime, ru1.ru_stime - ru0.ru_stime,
                           ru1.ru_nvcsw - ru0.ru_nvcsw, ru1.ru_nivcsw - ru0.ru_nivcsw,
                           ru1.ru_minflt - ru0.ru_minflt))
    for n in lanes:
        warm = res[n][1:]
        med = lambda i: statistics.median(x[i] for x in warm)  # noqa: E731
        print(json.dumps({"lib": os.environ.get("BCP_LIB", "in-tree"), "lanes": n, "wall_s": round(med(0), 4), "GiBps": round(nbytes / med(0) / GiB, 2),
                          "user_s": round(med(1), 4), "sys_s": round(med(2), 4),
                          "cpu_s": round(med(1) + med(2), 4), "vol_ctxsw": int(med(3)),
                          "invol_ctxsw": int(med(4)), "minflt": int(med(5)),
                          "runs": [[round(v, 4) for v in x] for x in res[n]]}), flush=True)
    bcp.set_xor_hook(None)
    shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
