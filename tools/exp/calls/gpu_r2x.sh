# r02 call X: implicit padding + device rows: GPU protocol/ref tests, then
# the protocol comparison (threads).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hostwrite.py tests/test_gpu_protocol.py tests/test_gpu_ref.py > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u tools/proto_compare.py --rounds 6 > $O/proto_threads.jsonl 2> $O/proto_threads.err || { echo THREADS_FAIL; tail -30 $O/proto_threads.err; exit 1; }
grep summary $O/proto_threads.jsonl
echo ALL_OK
