# r02 call AU: HW queues per process (4 default / 8 / 16) for the in-process
# per-task protocol (48 lanes launching on their own queues): pipelined and
# batched against the CPU fold, interleaved within each setting.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2au; mkdir -p $O
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u tools/proto_compare.py --rounds 6 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/hwq$q.jsonl 2> $O/hwq$q.err || { echo PROTO_FAIL $q; tail -20 $O/hwq$q.err; exit 1; }
  echo "q=$q"; grep -h summary $O/hwq$q.jsonl | python -c "import sys,json; [print(' ', d['workload'], d['summary']) for d in map(json.loads, sys.stdin)]"
done
echo ALL_OK
