set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1f_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r1f_smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r1f_bench.json 2> gpurun_out/r1f_bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > gpurun_out/r1f_bench_reb.json 2>> gpurun_out/r1f_bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
