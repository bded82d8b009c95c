# r02 call C6: node fold server width (batches in flight) on rank processes; the
# reference CPU fold measured without a server in the same call.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 240 --timeout-method thread -k "rank_pool" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for k in 1 2 4; do
    BCP_FOLD_SERVER=1 BCP_FOLD_SERVER_INFLIGHT=$k timeout -k 10 400 python -u tools/proto_compare.py --procs --rounds 4 --workloads c1_gen,c5_gen --folds gpu_batched,noop > $O/pc_server_k${k}_$i.jsonl 2> $O/pc_server_k${k}_$i.err || { echo PC_FAIL $k $i; tail -20 $O/pc_server_k${k}_$i.err; exit 1; }
    echo "server K=$k run $i"; grep summary $O/pc_server_k${k}_$i.jsonl | cut -c1-160
  done
  BCP_FOLD_SERVER=0 timeout -k 10 400 python -u tools/proto_compare.py --procs --rounds 4 --workloads c1_gen,c5_gen --folds cpu_reference,noop > $O/pc_cpu_$i.jsonl 2> $O/pc_cpu_$i.err || { echo PC_FAIL cpu $i; tail -20 $O/pc_cpu_$i.err; exit 1; }
  echo "no server, CPU fold, run $i"; grep summary $O/pc_cpu_$i.jsonl | cut -c1-160
done
echo ALL_OK
