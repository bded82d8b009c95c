#!/bin/bash
# GPU call: per-task protocol with 12 lanes against the number of hardware
# queues the HIP runtime spreads the lanes' streams over (GPU_MAX_HW_QUEUES:
# the box default 4, then 8 and 16), config 1 end to end, two rounds.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_hwq.jsonl; : > $out
for r in 1 2; do
  for hq in 4 8 16; do
    GPU_MAX_HW_QUEUES=$hq timeout -k 10 300 python3 -u tools/e2e_bench.py --configs 1 --root /dev/shm/bcp_hwq \
      > gpurun_out/hwq_$hq.jsonl 2> gpurun_out/hwq_$hq.err; rc=$?
    rm -rf /dev/shm/bcp_hwq
    [ $rc -eq 0 ] || exit $rc
    python3 -c "
import json
for l in open('gpurun_out/hwq_$hq.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d: print(json.dumps({'round': $r, 'hw_queues': $hq, 'path': d['path'], 'GiBps': d['GiBps']}))" >> $out
  done
done
