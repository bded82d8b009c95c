# r02 call D0: pipelined fold across rank processes (PROG frames + fold server ranges):
# device tests, then rank processes with pipelined / batched GPU folds and the CPU fold
# interleaved in one pool, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d0; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_ref.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 500 python -u tools/proto_compare.py --procs --rounds 5 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/procs_$i.jsonl 2> $O/procs_$i.err || { echo PC_FAIL $i; tail -20 $O/procs_$i.err; exit 1; }
  grep summary $O/procs_$i.jsonl | cut -c1-300
done
echo ALL_OK
