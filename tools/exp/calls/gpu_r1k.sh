set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --schedule 1 >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
for g in 1 2 3 4 8; do
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --schedule 0 --grab $g >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
done
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --schedule 1 >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
