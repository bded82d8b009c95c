# r02 call AK: fold service with targeted wakeups
# vs per-lane zero-copy: GPU protocol/ref tests, then interleaved comparison.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ak; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_protocol.py tests/test_gpu_ref.py > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 python -u tools/proto_compare.py --rounds 6 --folds gpu_zero_copy,gpu_batched1,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep summary $O/proto.jsonl
echo ALL_OK
