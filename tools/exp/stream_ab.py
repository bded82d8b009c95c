#!/usr/bin/env python3
"""Same-allocation A/B on the streaming kernel (tools only).  Allocates the
config-2 gen layout and the config-3 rebuild layout once, then for R rounds
times each variant -- a list of KEY=VALUE engine options, every other option
of the list reset to its default first -- on

  gen               xor_uniform over [stripes][8][512 KiB] -> [stripes][512 KiB]
  rebuild           7 survivors (of the same source array) + parity body from
                    a second array -> a third array (pointer table)
  table_gen_layout  the gen layout through the pointer table

so placement differences between processes (which move rebuild by +-3
points run to run) cancel out.  --offsets "P:O,..." also times the rebuild
with the parity and output arrays shifted by P and O bytes.

    python tools/exp/stream_ab.py --variants "stream_wpe=0;stream_wpe=6" --rounds 4
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "beegfs-chunk-parity_amd"))
import bcp_ctypes as bcp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="", help="';'-separated variants, each ','-separated KEY=VALUE")
ap.add_argument("--offsets", default="", help="','-separated P:O byte shifts of the parity / output arrays")
ap.add_argument("--modes", default="gen,rebuild,table_gen_layout")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--stripes", type=int, default=12500)
ap.add_argument("--contig", action="store_true", help="engine contiguous_alloc = 1 before allocating")
a = ap.parse_args()

N, C, S = 8, 512 * 1024, a.stripes
SLACK = 16 << 20
eng = bcp.Engine(0)
if a.contig:
    eng.option("contiguous_alloc", 1)
q = eng.queue()
src = eng.alloc(S * N * C + S * C)  # + room for a parity array inside the same allocation
out0 = eng.alloc(S * C + SLACK)
par0 = eng.alloc(S * C + SLACK)
q.fill_synthetic(src, S * N * C, seed=1)
q.sync()
L = bcp.lib()
victim = 3


def rebuild_tables(par, out, victim=3, par_first=False):
    stripes, sources = [], []
    for s in range(S):
        first = len(sources)
        run = [bcp.Source(src + (s * N + k) * C, C) for k in range(N) if k != victim]
        p = bcp.Source(par + s * C, C)
        sources += [p] + run if par_first else run + [p]
        stripes.append(bcp.Stripe(out + s * C, C, first, N, 0))
    return (bcp.Stripe * S)(*stripes), (bcp.Source * len(sources))(*sources)


def submit(st, so):
    bcp.check("x", L.bcp_xor_stripes_async(q.h, st, len(st), so, len(so)))


nbytes = S * (N + 1) * C
work = {}
offsets = [(0, 0)] + [tuple(int(x) for x in o.split(":")) for o in filter(None, a.offsets.split(","))]
for po, oo in offsets:
    par, out = par0 + po, out0 + oo
    q.xor_uniform(par, src, S, N, C)
    q.sync()
    st, so = rebuild_tables(par, out)
    tag = "" if (po, oo) == (0, 0) else f"@{po}:{oo}"
    if "rebuild" in a.modes:
        work["rebuild" + tag] = (lambda st=st, so=so: submit(st, so))
    if (po, oo) != (0, 0):
        continue
    if "gen" in a.modes:
        work["gen"] = lambda: q.xor_uniform(out0, src, S, N, C)
    if "rebuild_orders" in a.modes:
        for v, pf in ((7, False), (0, False), (3, True), (7, True)):
            st_o, so_o = rebuild_tables(par, out0, victim=v, par_first=pf)
            work[f"rebuild_victim{v}{'_par_first' if pf else ''}"] = (lambda st_o=st_o, so_o=so_o: submit(st_o, so_o))
    if "rebuild_one_alloc" in a.modes:  # parity array in the tail of the source allocation
        par_in = src + S * N * C
        q.xor_uniform(par_in, src, S, N, C)
        q.sync()
        st_i, so_i = rebuild_tables(par_in, out0)
        work["rebuild_one_alloc"] = lambda st_i=st_i, so_i=so_i: submit(st_i, so_i)
    if "table_gen_layout" in a.modes:
        so_g = (bcp.Source * (S * N))(*[bcp.Source(src + (s * N + k) * C, C) for s in range(S) for k in range(N)])
        st_g = (bcp.Stripe * S)(*[bcp.Stripe(out0 + s * C, C, s * N, N, 0) for s in range(S)])
        work["table_gen_layout"] = lambda st_g=st_g, so_g=so_g: submit(st_g, so_g)
variants = [dict(kv.split("=") for kv in v.split(",")) for v in filter(None, a.variants.split(";"))] or [{}]
keys = sorted({k for v in variants for k in v})
defaults = {k: eng.option(k) for k in keys}
for r in range(a.rounds):
    for mode, fn in work.items():
        for v in variants:
            for k in keys:
                eng.option(k, int(v.get(k, defaults[k])))
            fn()
            q.sync()
            fn()
            q.mark(0)
            for _ in range(a.reps):
                fn()
            q.mark(1)
            q.sync()
            ms = q.elapsed_ms(0, 1) / a.reps
            print(json.dumps({"round": r, "mode": mode, "variant": v, "kernel_ms": round(ms, 4),
                              "frac_8TBs": round(nbytes / ms / 8e9, 4)}), flush=True)
