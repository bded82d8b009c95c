#!/bin/bash
# GPU call: explicit rolling load window (stream_pipe 1..6) against the
# compiler's schedule (0) and the waves_per_eu(6) budget, gen and rebuild,
# interleaved rounds; descriptor kernel desc_pipe 0,4,5,6.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xor.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "schedule_variants" > gpurun_out/ab_depth2_pytest.log 2>&1 || exit $?
out=gpurun_out/ab_depth2_bench.jsonl; : > $out
for r in 1 2 3; do
  for mode in gen rebuild; do
    for v in "stream_pipe=0" "stream_pipe=1" "stream_pipe=2" "stream_pipe=3" "stream_pipe=4" "stream_pipe=5" "stream_pipe=6" "stream_wpe=6"; do
      timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 --mode $mode --opt $v \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'mode': '$mode', 'variant': '$v', 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> $out || exit $?
    done
  done
done
timeout -k 10 400 python3 tools/exp/desc_probe.py --workloads uniform_forced,mixed,mixed_big --tunings 8:0 \
  --pipes 0,4,5,6,2 --rounds 2 > gpurun_out/ab_depth2_desc.jsonl
