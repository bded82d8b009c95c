# r02 call C4: rank processes with the shared row arena (fill sends into the P role's
# rows) -- device protocol tests, then the per-task protocol over rank processes with
# and without the arena, alternating processes on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c4; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_protocol.py tests/test_gpu_ref.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for mb in 2048 0; do
    BCP_SOCK_ARENA_MB=$mb timeout -k 10 400 python -u tools/proto_compare.py --procs --rounds 4 --workloads c1_gen,c5_gen --folds gpu_batched,cpu_reference,noop > $O/pc_${mb}_$i.jsonl 2> $O/pc_${mb}_$i.err || { echo PC_FAIL $mb $i; tail -20 $O/pc_${mb}_$i.err; exit 1; }
    echo "arena_mb=$mb run $i"; grep summary $O/pc_${mb}_$i.jsonl
  done
done
echo ALL_OK
