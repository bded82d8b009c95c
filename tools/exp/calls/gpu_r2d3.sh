# r02 call D3: loopback ranks folding through a connected node fold server (an MPI
# job's shape) vs in-process folds, alternating processes, twice.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d3; mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/proto_compare.py --fold-server --rounds 5 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/server_$i.jsonl 2> $O/server_$i.err || { echo PC_SERVER_FAIL $i; tail -20 $O/server_$i.err; exit 1; }
  echo "connected server run $i"; grep summary $O/server_$i.jsonl | cut -c1-260
  timeout -k 10 500 python -u tools/proto_compare.py --rounds 5 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/inproc_$i.jsonl 2> $O/inproc_$i.err || { echo PC_INPROC_FAIL $i; tail -20 $O/inproc_$i.err; exit 1; }
  echo "in-process run $i"; grep summary $O/inproc_$i.jsonl | cut -c1-260
done
echo ALL_OK
