#!/bin/bash
# GPU call: loads-in-flight A/B.  (1) correctness of the variants; (2) bench
# gen / rebuild with xor_stream's register budget (engine stream_wpe; 0 = the
# compiler's choice), interleaved rounds; (3) xor_desc's rolling load window
# (desc_pipe) through tools/exp/desc_probe.py.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xor.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "schedule_variants or tuning_variants or table_residency" > gpurun_out/ab_depth_pytest.log 2>&1 || exit $?
out=gpurun_out/ab_depth_bench.jsonl; : > $out
for r in 1 2 3; do
  for mode in gen rebuild; do
    for w in 0 6 7 5; do
      timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 --mode $mode --opt stream_wpe=$w \
        | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'mode': '$mode', 'wpe': $w, 'frac': d['roofline']['frac'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> $out || exit $?
    done
  done
done
timeout -k 10 400 python3 tools/exp/desc_probe.py --workloads uniform_forced,mixed,mixed_big,wide16 --tunings 8:0 \
  --pipes 0,1,2,3,4 --rounds 2 > gpurun_out/ab_depth_desc.jsonl
