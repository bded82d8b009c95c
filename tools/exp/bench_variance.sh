# bench.py run-to-run spread on one box: alternating processes, default allocations vs
# physically contiguous ones (--contig); one JSON line per process.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for c in "" "--contig"; do
    timeout -k 10 120 python -u bench.py --no-cpu --steps 20 --warmup 5 $c > gpurun_out/var_$r$c.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'round': $r, 'contig': '$c'!='', 'ms': d['ms_per_step'], 'frac_event': d['roofline']['frac_event']}))" gpurun_out/var_$r$c.json
  done
done
