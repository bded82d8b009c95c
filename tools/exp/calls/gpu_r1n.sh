set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1n; mkdir -p $O
timeout -k 10 600 ./tools/exp/xor_exp2 12500 5 > $O/exp7.jsonl 2> $O/exp7.err || { echo EXP_FAIL; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u tools/sweep_fast.py --reps 5 --bpc 1,2,4,8 --vecs 4,8 --sched 0 > $O/sweep_fast.jsonl 2> $O/sweep.err || { echo SWEEP_FAIL; exit 1; }
for b in 1 2 4 8; do
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --blocks-per-cu $b >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
done
timeout -k 10 300 python -u bench.py --no-cpu > $O/bench_gen.json 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > $O/bench_rebuild.json 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
