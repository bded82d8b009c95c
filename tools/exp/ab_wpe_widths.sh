#!/bin/bash
# GPU call: waves_per_eu(6) budget for widths other than 8 (stream_wpe=16 is
# the A/B switch for those instantiations).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_wpe_widths.jsonl; : > $out
for r in 1 2; do
for n in 3 4 5 6 7 12 16; do
  s=$(( 100000 / n ))
  for w in 0 16; do
    timeout -k 10 120 python3 bench.py --no-cpu --steps 8 --warmup 2 --nsrc $n --stripes $s --opt stream_wpe=$w \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'nsrc': $n, 'wpe': $w, 'frac': d['roofline']['frac']}))" >> $out || exit $?
  done
done
done
