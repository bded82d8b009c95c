# r02 call L: descriptor-kernel changes -- GPU tests, mixed bench with and
# without side-stream desc_tiles, batch curve for small batches.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_xor.py tests/test_gpu_ref.py tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL $rc; grep -B5 -A30 "Error\|FAILED" $O/pytest_gpu.log | head -80; exit 1; }
for i in 1 2; do
for side in 1 0 A; do
  timeout -k 10 300 python -u bench.py --mode mixed --no-cpu $( [ $side = A ] && echo "--opt desc_ahead=1" || echo "--opt desc_side_tiles=$side" ) > $O/bench_mixed_side$side.$i.json 2> $O/bench_mixed_side$side.$i.err || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_mixed_side$side.$i.json')); print('side', $side, d['roofline']['kernel'], d['roofline']['frac'], d['value'], d['config']['verified_on_device'])"
done
done
timeout -k 10 300 python -u tools/batch_curve.py --batches 1,2,4,8,16,64,512 > $O/batch_curve.jsonl 2> $O/batch_curve.err || { echo CURVE_FAIL; exit 1; }
python -c "
import json
for l in open('$O/batch_curve.jsonl'):
    d=json.loads(l); print(d['stripes'], d['entry'], d['pipelined_us'], d['latency_us'], d['pipelined_frac_8TBs'])"
echo ALL_OK
