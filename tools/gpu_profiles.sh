# Round profile set, one box, one call (run through gpurun from the repo
# root): bench.py default line (config 2 gen, with the CPU baseline), the
# rebuild and mixed bench lines, and for each of gen / rebuild / mixed the
# rocprofv3 kernel-trace stats of the same command and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs) for HBM traffic.  Output under
# gpurun_out/prof_<tag>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${PROF_TAG:-r01}
O=$R/gpurun_out/prof_$T
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_gen.json 2> $O/bench_gen.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > $O/bench_rebuild.json 2> $O/bench_rebuild.err || { echo BENCH_RB_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu > $O/bench_mixed.json 2> $O/bench_mixed.err || { echo BENCH_MX_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gen_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu > $O/gen_trace.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
for m in rebuild mixed; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${m}_trace -o run --output-format csv -- python3 $R/bench.py --mode $m --no-cpu > $O/${m}_trace.log 2>&1 || { echo PROF_${m}_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${m}_pmc_fetch -o run -- python3 $R/bench.py --mode $m --steps 3 --warmup 1 --no-cpu > $O/${m}_pmc_fetch.log 2>&1 || { echo PMC1_${m}_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${m}_pmc_write -o run -- python3 $R/bench.py --mode $m --steps 3 --warmup 1 --no-cpu > $O/${m}_pmc_write.log 2>&1 || { echo PMC2_${m}_FAIL; exit 1; }
done
echo ALL_OK
