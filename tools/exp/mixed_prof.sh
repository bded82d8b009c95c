#!/bin/bash
# GPU call: bench + rocprofv3 kernel-trace stats + PMC passes for one bench
# mode (MODE env, default mixed).  Output under gpurun_out/prof_$MODE/.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
M=${MODE:-mixed}
O=$R/gpurun_out/prof_$M
mkdir -p $O
timeout -k 10 300 python -u bench.py --mode $M --no-cpu > $O/bench_$M.json 2> $O/bench.err || { echo BENCH_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --mode $M --no-cpu > $O/trace.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --mode $M --steps 3 --warmup 1 --no-cpu > $O/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --mode $M --steps 3 --warmup 1 --no-cpu > $O/pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo ALL_OK
