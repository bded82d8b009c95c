#!/bin/bash
# GPU call: streaming kernel at other stripe widths (default tuning).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/widths_sweep.jsonl; : > $out
for n in ${WIDTHS:-9 10 11 13 14 15 20 24 32 48}; do
  s=$(( 100000 / n ))
  timeout -k 10 120 python3 bench.py --no-cpu --steps 8 --warmup 2 --nsrc $n --stripes $s \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'nsrc': $n, 'kernel': d['roofline']['kernel'], 'frac': d['roofline']['frac']}))" >> $out || exit $?
done
