# rocprofv3 kernel-trace summary + PMC HBM traffic of the descriptor kernel on
# the config-5 shapes (bench.py --mode mixed).  Run through gpurun from the repo root.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu > gpurun_out/mx_bench.json 2> gpurun_out/mx_bench.err || { echo BENCH_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/mx_prof -o run --output-format csv -- python3 $R/bench.py --mode mixed --no-cpu > $R/gpurun_out/mx_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/mx_pmc_fetch -o run -- python3 $R/bench.py --mode mixed --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/mx_pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/mx_pmc_write -o run -- python3 $R/bench.py --mode mixed --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/mx_pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo ALL_OK
