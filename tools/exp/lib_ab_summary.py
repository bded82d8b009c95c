#!/usr/bin/env python3
"""Median warm run per (library, workload) of a tools/exp/pipeline_lib_ab.sh
output (tools only).    python tools/exp/lib_ab_summary.py out.jsonl"""
import collections
import json
import statistics
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("{") and "workload" in line:
        j = json.loads(line)
        d[(j["lib"].split("/")[-1], j["workload"])].append(j["warm_s"])
for k, v in sorted(d.items()):
    print(k, [round(x * 1e3, 1) for x in v], "median", round(statistics.median(v) * 1e3, 1))
