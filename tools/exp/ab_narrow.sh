#!/bin/bash
# GPU call: narrow uniform stripes (N = 1..4 sources, 512 KiB) -- tile size
# and workgroups per CU of the streaming kernel (bench.py --vecs --blocks-per-cu;
# register budget off for the non-8 widths anyway).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_narrow.jsonl; : > $out
for n in 1 2 3 4; do
  s=$(( 100000 / n ))
  for t in 8:1 8:2 8:3 8:4 4:2 4:4 4:8 2:8; do
    u=${t%:*}; b=${t#*:}
    timeout -k 10 120 python3 bench.py --no-cpu --steps 8 --warmup 2 --nsrc $n --stripes $s --vecs $u --blocks-per-cu $b \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'nsrc': $n, 'vecs': $u, 'bpc': $b, 'frac': d['roofline']['frac']}))" >> $out || exit $?
  done
done
