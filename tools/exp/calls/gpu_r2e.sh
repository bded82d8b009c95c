# r02 call D: GPU protocol tests (incl. CLI --procs), then the per-task
# protocol fold comparison with per-phase timings.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2e; mkdir -p $O
nproc > $O/host.txt; cat /sys/fs/cgroup/cpu.max >> $O/host.txt 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/host.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL $rc; exit 1; }
timeout -k 10 600 python -u tools/proto_compare.py --rounds 4 --folds gpu_batched,gpu_zero_copy,cpu_reference,noop,gpu_streamed > $O/proto_compare.jsonl 2> $O/proto_compare.err || { echo PROTO_FAIL; tail -20 $O/proto_compare.err; exit 1; }
cat $O/host.txt
echo ALL_OK
