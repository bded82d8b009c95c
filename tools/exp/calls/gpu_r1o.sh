set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1o; mkdir -p $O
timeout -k 10 300 python -u tools/sweep_fast.py --reps 7 --bpc 1,2 --vecs 4,8 --sched 0 > $O/sweep_fast.jsonl 2> $O/sweep.err || { echo SWEEP_FAIL; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for v in 4 8; do for b in 1 2; do
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu --steps 10 --vecs $v --blocks-per-cu $b >> $O/bench_rebuild.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
done; done
echo ALL_OK
