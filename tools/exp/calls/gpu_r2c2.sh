# r02 call C2: descriptor kernel with 64 KiB subtiles (U = 16) -- parity tests, then
# interleaved A/B against U = 8 on config-5 shapes and friends.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_xor.py -x -q --timeout 120 --timeout-method thread -k "grouped or window_replay or u16 or knob or schedule_variants or mixed" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u tools/exp/desc_probe.py --workloads mixed,mixed_big,mixed_equal,wide16 --tunings 8:1,16:1 --pipes 5,6 --rounds 3 > $O/desc.jsonl 2> $O/desc.err || { echo DESC_FAIL; tail -20 $O/desc.err; exit 1; }
python3 - <<'PY'
import json,collections,statistics
agg=collections.defaultdict(list)
for l in open("gpurun_out/r2c2/desc.jsonl"):
    d=json.loads(l)
    if "frac_8TBs" in d: agg[(d["workload"],d["vecs"],d["pipe"])].append(d["frac_8TBs"])
for k,v in sorted(agg.items()): print(k, [round(x*100,2) for x in v], round(100*statistics.median(v),2))
PY
echo ALL_OK
