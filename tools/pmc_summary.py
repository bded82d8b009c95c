#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in
separate runs) into HBM bytes per launch of one kernel.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half
the bytes of a wide coalesced 16-B-per-lane stream, so it is doubled;
WRITE_SIZE is exact for 16-B streaming stores.  Both are in KiB.

    python tools/pmc_summary.py --fetch DIR/run_counter_collection.csv \
        --write DIR2/run_counter_collection.csv --kernel xor_strided_fast \
        --workload-key gen:12500x8x524288 --algorithmic 58982400000 --out profiles/r01_pmc_gen.json
"""
import argparse
import csv
import json
import statistics


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter or kernel not in row["Kernel_Name"]:
                continue
            vals[row["Dispatch_Id"]] = (float(row["Counter_Value"]), row["Kernel_Name"],
                                        int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--workload-key", required=True)
    ap.add_argument("--algorithmic", type=float, required=True, help="algorithmic bytes per launch")
    ap.add_argument("--out", required=True)
    ap.add_argument("--stats", help="rocprofv3 --kernel-trace --stats kernel_stats.csv of the same command")
    ap.add_argument("--trace", help="rocprofv3 kernel_trace.csv of the same command: the timed launches alone")
    ap.add_argument("--warmup", type=int, default=3, help="warm-up launches of the traced bench command")
    ap.add_argument("--steps", type=int, default=20, help="timed launches of the traced bench command")
    ap.add_argument("--commit", help="code commit the profiled tree was built from")
    ap.add_argument("--files", nargs="*", default=[], help="committed copies of the raw inputs (provenance)")
    a = ap.parse_args()
    fe = per_dispatch(a.fetch, "FETCH_SIZE", a.kernel)
    wr = per_dispatch(a.write, "WRITE_SIZE", a.kernel)
    assert fe and wr, "no matching dispatches"
    fetch_b = statistics.median(v[0] for v in fe.values()) * 1024 * 2
    write_b = statistics.median(v[0] for v in wr.values()) * 1024
    avg_ns = None
    if a.stats:
        with open(a.stats) as f:
            for row in csv.DictReader(f):
                if a.kernel in row["Name"]:
                    avg_ns = float(row["AverageNs"])
                    break
    timed = None
    if a.trace:  # dispatches in order; drop the warm-up ones and the verification one after the timed steps
        with open(a.trace) as f:
            rows = sorted((r for r in csv.DictReader(f) if a.kernel in r["Kernel_Name"]),
                          key=lambda r: int(r["Dispatch_Id"]))
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        if len(durs) == a.warmup + a.steps + 1:
            timed = durs[a.warmup:a.warmup + a.steps]
    doc = {
        "workload_key": a.workload_key,
        "code_commit": a.commit,
        "rocprof_avg_ns": avg_ns,
        "rocprof_timed_avg_ns": round(statistics.fmean(timed), 1) if timed else None,
        "rocprof_timed_median_ns": statistics.median(timed) if timed else None,
        "rocprof_timed_launches": len(timed) if timed else None,
        "files": {"stats": a.stats, "trace": a.trace, "raw": a.files},
        "kernel": next(iter(fe.values()))[1],
        "dispatches": {"fetch_pass": len(fe), "write_pass": len(wr)},
        "fetch_bytes_per_launch": round(fetch_b),
        "write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(fetch_b + write_b),
        "algorithmic_bytes_per_launch": round(a.algorithmic),
        "traffic_over_algorithmic": round((fetch_b + write_b) / a.algorithmic, 5),
        "profiled_kernel_ns_median": statistics.median(v[2] for v in fe.values()),
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); FETCH_SIZE x2 (gfx950 "
                  "wide-read correction), WRITE_SIZE x1; KiB->B x1024",
    }
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
