# bench.py run-to-run spread on one box: alternating processes, default
# allocations vs physically contiguous ones (--contig), per mode; one JSON
# line per process.   MODES="gen rebuild mixed" ROUNDS=4 bash tools/exp/bench_variance.sh
set -o pipefail
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-4}); do
  for m in ${MODES:-gen}; do
    for c in "" "--contig"; do
      out=gpurun_out/var_${m}_$r$c.json
      timeout -k 10 120 python -u bench.py --mode $m --no-cpu --steps 20 --warmup 5 $c > $out 2>/dev/null || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'round': $r, 'mode': '$m', 'contig': '$c'!='', 'ms': d['ms_per_step'], 'frac_event': d['roofline']['frac_event'], 'verified': d['config']['verified_on_device']}))" $out || exit 1
    done
  done
done
