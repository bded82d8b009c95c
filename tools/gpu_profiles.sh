# Round profile set, one box, one call (run through gpurun from the repo
# root): bench.py lines (config 2 gen with the CPU baseline, config 3
# rebuild, config-5 mixed shapes, config 4's per-GPU shard), and for each the
# rocprofv3 kernel-trace stats of the same command and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs) for HBM traffic.  Profiled runs
# pass --no-e2e --no-configs: the end-to-end and config legs launch the descriptor kernel too and
# would mix its launches into the kernel statistics.  Output under
# gpurun_out/prof_<tag>/<mode>/.  tools/collect_profiles.py turns it into
# profiles/<round>/final/ with provenance (commit, files).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${PROF_TAG:-r05}
O=$R/gpurun_out/prof_$T
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_gen.json 2> $O/bench_gen.err || { echo BENCH_FAIL; exit 1; }
cat $O/bench_gen.json
cd /tmp && export TMPDIR=/tmp
for m in gen rebuild mixed config4; do
  args="--mode $m"
  [ $m = config4 ] && args="--mode gen --stripes 15625"
  mkdir -p $O/$m
  if [ $m != gen ]; then
    timeout -k 10 300 python3 $R/bench.py $args --no-cpu --no-e2e --no-prof --no-configs > $O/$m/bench.json 2> $O/$m/bench.err || { echo BENCH_${m}_FAIL; exit 1; }
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$m/trace -o run --output-format csv -- python3 $R/bench.py $args --no-cpu --no-e2e --no-prof --no-configs > $O/$m/trace.log 2>&1 || { echo PROF_${m}_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$m/pmc_fetch -o run -- python3 $R/bench.py $args --steps 3 --warmup 1 --no-cpu --no-e2e --no-prof --no-configs > $O/$m/pmc_fetch.log 2>&1 || { echo PMC1_${m}_FAIL; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$m/pmc_write -o run -- python3 $R/bench.py $args --steps 3 --warmup 1 --no-cpu --no-e2e --no-prof --no-configs > $O/$m/pmc_write.log 2>&1 || { echo PMC2_${m}_FAIL; exit 1; }
  echo PROF_${m}_OK
done
echo ALL_OK
