# r02 call C5: node fold server for rank processes -- device tests, then the per-task
# protocol over rank processes: fold server / per-rank contexts (arena) / no arena.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 240 --timeout-method thread -k "rank_pool or cli" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for m in server ranks noarena; do
    case $m in server) E="BCP_FOLD_SERVER=1";; ranks) E="BCP_FOLD_SERVER=0";; noarena) E="BCP_SOCK_ARENA_MB=0";; esac
    env $E timeout -k 10 400 python -u tools/proto_compare.py --procs --rounds 4 --workloads c1_gen,c5_gen --folds gpu_batched,cpu_reference,noop > $O/pc_${m}_$i.jsonl 2> $O/pc_${m}_$i.err || { echo PC_FAIL $m $i; tail -20 $O/pc_${m}_$i.err; exit 1; }
    echo "$m run $i"; grep summary $O/pc_${m}_$i.jsonl | cut -c1-200
  done
done
echo ALL_OK
