set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for v in 4; do for sc in 0 1; do
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --vecs $v --schedule $sc >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
done; done
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu --steps 10 >> $O/bench_rebuild.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 >> $O/bench_gen.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
