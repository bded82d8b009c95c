#!/bin/bash
# GPU call: uniform N-source streaming kernel, tile size U = 4 vs 8 for
# N = 6, 12, 16 (bench.py --nsrc N --vecs U), interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_wide_stream.jsonl; : > $out
for r in 1 2; do
  for n in 6 12 16; do
    for u in 8 4 2; do
      s=$(( 100000 / n ))
      timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 --nsrc $n --stripes $s --vecs $u \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'nsrc': $n, 'vecs': $u, 'frac': d['roofline']['frac'], 'kernel': d['roofline']['kernel']}))" >> $out || exit $?
    done
  done
done
