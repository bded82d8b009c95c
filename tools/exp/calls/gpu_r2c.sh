# r02 call B: GPU tests of the protocol paths (batched fold mode added, and
# the reference fixtures), then the interleaved per-task protocol comparison.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_ref.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL $rc; exit 1; }
timeout -k 10 600 python -u tools/proto_compare.py --rounds 4 > $O/proto_compare.jsonl 2> $O/proto_compare.err || { echo PROTO_FAIL; tail -20 $O/proto_compare.err; exit 1; }
grep summary $O/proto_compare.jsonl
echo ALL_OK
