#!/bin/bash
# GPU call: per-task protocol with the fold wait as hipStreamSynchronize (0)
# or a blocking-sync event (1), configs 1 and 5 end to end, separate processes.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_sync_mode.jsonl; : > $out
for r in 1 2; do
  for m in 0 1; do
    BCP_SYNC_MODE=$m timeout -k 10 600 python3 -u tools/e2e_bench.py --configs 1,5 --root /dev/shm/bcp_sm \
      > gpurun_out/sm_$m.jsonl 2> gpurun_out/sm_$m.err; rc=$?
    rm -rf /dev/shm/bcp_sm
    [ $rc -eq 0 ] || exit $rc
    python3 -c "
import json
for l in open('gpurun_out/sm_$m.jsonl'):
    d=json.loads(l)
    if 'GiBps' in d and 'protocol' in d.get('path', ''): print(json.dumps({'round': $r, 'sync_mode': $m, 'config': d['config'], 'path': d['path'], 'GiBps': d['GiBps']}))" >> $out
  done
done
