#!/bin/bash
# GPU call: tiles per queue grab for narrow stripes (N = 1..4), then the
# correctness tests of the grab path.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xor.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "narrow_stripes or knobs" > gpurun_out/ab_grab_pytest.log 2>&1 || exit $?
out=gpurun_out/ab_grab.jsonl; : > $out
for r in 1 2; do
for n in 1 2 3 4; do
  s=$(( 100000 / n ))
  for g in 1 2 3 4 8; do
    timeout -k 10 120 python3 bench.py --no-cpu --steps 8 --warmup 2 --nsrc $n --stripes $s --opt stream_grab=$g \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'nsrc': $n, 'grab': $g, 'frac': d['roofline']['frac']}))" >> $out || exit $?
  done
done
done
