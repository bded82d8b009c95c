# r02 call H: GPU tests (protocol + knobs), the protocol fold comparison with
# registered rows (default now), and the end-to-end pipeline with registered
# vs hipHostMalloc slabs.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_xor.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL $rc; exit 1; }
timeout -k 10 600 python -u tools/proto_compare.py --rounds 6 --folds gpu_batched,gpu_zero_copy,cpu_reference,noop,gpu_streamed > $O/proto_compare.jsonl 2> $O/proto_compare.err || { echo PROTO_FAIL; tail -20 $O/proto_compare.err; exit 1; }
grep summary $O/proto_compare.jsonl
for hr in 1 0; do
  BCP_HOST_REGISTERED=$hr timeout -k 10 400 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e --reps 3 > $O/e2e_hostreg$hr.jsonl 2> $O/e2e_hostreg$hr.err || { echo E2E_FAIL $hr; tail -20 $O/e2e_hostreg$hr.err; exit 1; }
  grep -h '"path"' $O/e2e_hostreg$hr.jsonl | python -c "import sys,json; [print($hr, d.get('config'), d['path'][:40], d.get('GiBps')) for d in map(json.loads, sys.stdin)]"
done
echo ALL_OK
