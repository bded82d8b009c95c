set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1b_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
for i in 1 2 3; do timeout -k 10 300 python -u bench.py --no-cpu >> gpurun_out/r1b_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }; done
timeout -k 10 300 python -u bench.py --steps 50 --no-cpu >> gpurun_out/r1b_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > gpurun_out/r1b_bench_rebuild.log 2>&1 || { echo BENCHRB_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1b_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/gpurun_out/r1b_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r1b_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/r1b_pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r1b_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/r1b_pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo ALL_OK
