#!/usr/bin/env python3
"""Turn a tools/gpu_profiles.sh run (gpurun_out/prof_<tag>/) into the
committed profile set profiles/<round>/final/: per mode the bench line, the
rocprofv3 kernel-trace stats CSV and the PMC summary (tools/pmc_summary.py)
carrying the code commit the box ran and the committed file names -- what
bench.py reports as roofline.traffic / frac_rocprof and their provenance.

    python tools/collect_profiles.py --src gpurun_out/prof_r02 --dst profiles/r02/final --commit <sha>
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        sys.exit(f"missing {pattern}")
    return hits[-1]


def derive_tag(kern: str) -> str:
    """rocprofv3 name fragment of a bench.py display name (lines written
    before bench.py reported kernel_tag)."""
    import re
    m = re.match(r"xor_stream_w<(\d+),(\d+),(strided|gather),wpe(\d+)>", kern)
    if m:
        return f"xor_stream_w<{m[1]}, {m[2]}, {1 if m[3] == 'gather' else 0}, 0, {m[4]}>"
    m = re.match(r"xor_desc_p<(\d+),(\d+)>", kern)
    if m:
        return f"xor_desc_p<{m[1]}, {m[2]}, 0>"
    return kern


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", required=True)
    ap.add_argument("--dst", required=True)
    ap.add_argument("--commit", required=True)
    a = ap.parse_args()
    os.makedirs(a.dst, exist_ok=True)
    shutil.copy(os.path.join(a.src, "bench_gen.json"), os.path.join(a.dst, "bench_gen.json"))
    for m in ("gen", "rebuild", "mixed", "config4"):
        d = os.path.join(a.src, m)
        bench = os.path.join(a.src, "bench_gen.json") if m == "gen" else os.path.join(d, "bench.json")
        line = json.loads([l for l in open(bench) if l.startswith("{")][-1])
        if m != "gen":
            shutil.copy(bench, os.path.join(a.dst, f"bench_{m}.json"))
        stats = os.path.join(a.dst, f"{m}_kernel_stats.csv")
        shutil.copy(one(os.path.join(d, "trace", "**", "*kernel_stats.csv")), stats)
        trace = os.path.join(a.dst, f"{m}_kernel_trace.csv")
        shutil.copy(one(os.path.join(d, "trace", "**", "*kernel_trace.csv")), trace)
        fetch = os.path.join(a.dst, f"{m}_pmc_fetch.csv")
        write = os.path.join(a.dst, f"{m}_pmc_write.csv")
        shutil.copy(one(os.path.join(d, "pmc_fetch", "**", "*counter_collection.csv")), fetch)
        shutil.copy(one(os.path.join(d, "pmc_write", "**", "*counter_collection.csv")), write)
        tag = line["roofline"].get("kernel_tag") or derive_tag(line["roofline"]["kernel"])
        cfg = line["config"]
        mode_key = "rebuild_packed" if m == "rebuild" else ("gen" if m == "config4" else m)
        wkey = f"{mode_key}:{cfg['stripes_per_gpu']}x{cfg['nsrc']}x{cfg['chunk_bytes']}"
        rel = lambda p: os.path.relpath(p, ROOT)  # noqa: E731
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), "--fetch", fetch, "--write", write,
                        "--kernel", tag, "--workload-key", wkey, "--algorithmic", str(cfg["bytes_per_step_per_gpu"]),
                        "--stats", rel(stats), "--trace", rel(trace), "--warmup", str(line["warmup"]),
                        "--steps", str(line["steps"]), "--commit", a.commit, "--files", rel(fetch), rel(write),
                        rel(os.path.join(a.dst, f"bench_{m}.json")),  # the committed copy of the bench line
                        "--out", os.path.join(a.dst, f"pmc_{m}.json")], check=True)
        # the box the set was measured on (bench.py's run_box), for bench.py's profile_box
        box = line["roofline"].get("run_box")
        if box:
            out = os.path.join(a.dst, f"pmc_{m}.json")
            doc = json.load(open(out))
            doc["box"] = box
            with open(out, "w") as f:
                json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
