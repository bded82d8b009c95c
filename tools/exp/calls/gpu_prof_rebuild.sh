# rocprofv3 kernel-trace summary of the config-3 rebuild bench (bench.py --mode rebuild).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > gpurun_out/rb_bench.json 2> gpurun_out/rb_bench.err || { echo BENCH_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rb_prof -o run --output-format csv -- python3 $R/bench.py --mode rebuild --no-cpu > $R/gpurun_out/rb_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
