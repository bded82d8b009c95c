#!/bin/bash
# GPU call: (1) HBM efficiency of xor_stream against the read:write mix
# (N sources : 1 output, 512 KiB chunks, same input volume per launch), the
# ceiling the descriptor kernel's config-5 shapes are compared with;
# (2) throughput / latency against batch size (tools/batch_curve.py).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/rw_mix.jsonl; : > $out
for n in 1 2 3 4 6 8 12 16; do
  s=$(( 100000 / n ))
  timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 --nsrc $n --stripes $s >> $out || exit $?
done
[ -n "$SKIP_BATCH" ] || timeout -k 10 300 python3 tools/batch_curve.py > gpurun_out/batch_curve.jsonl
