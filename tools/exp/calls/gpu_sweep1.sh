set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python -u tools/sweep_fast.py --reps 5 > gpurun_out/s1_sweep.jsonl 2> gpurun_out/s1_sweep.err || { echo SWEEP_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/s1_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/s1_pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/s1_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/s1_pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo ALL_OK
