# r02 call AX: shared range queues -- full GPU suite + smoke + bench, then
# the interleaved comparison.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ax; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -B5 -A30 "FAILED\|Error" $O/pytest_gpu.log | head -60; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
timeout -k 10 700 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep -h '"box"' $O/proto.jsonl; grep summary $O/proto.jsonl
echo ALL_OK
