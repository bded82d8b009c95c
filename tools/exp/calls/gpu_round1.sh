set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
rocm-smi --showproductname > gpurun_out/r1_smi.txt 2>&1 || true
lscpu > gpurun_out/r1_lscpu.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r1_smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r1_bench.log 2>&1 || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > gpurun_out/r1_bench_rebuild.log 2>&1 || { echo BENCHRB_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r1_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/r1_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
