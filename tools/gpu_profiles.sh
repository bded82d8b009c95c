# Round profile set, one box, one call (run through gpurun from the repo
# root): per mode -- config 2 gen (the default line, every leg), config 3
# rebuild, config-5 mixed shapes, config 4's per-GPU shard -- one bench.py
# run whose rank 0 runs under rocprofv3 --kernel-trace (bench.py's profiled
# rank: the trace holds the line's own timed launches) and whose parent then
# runs the two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs);
# --profile-dir keeps the trace and the counter files.  The modes other than
# gen pass --no-e2e --no-configs --no-cpu (their legs are the gen line's).
# Output under gpurun_out/prof_<tag>/<mode>/.  tools/collect_profiles.py
# turns it into profiles/<round>/final_<commit>/ with provenance.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
T=${PROF_TAG:-r06}
O=$R/gpurun_out/prof_$T
mkdir -p $O
export TMPDIR=/tmp
for m in gen rebuild mixed config4; do
  args="--mode $m"
  [ $m = config4 ] && args="--mode gen --stripes 15625"
  [ $m != gen ] && args="$args --no-cpu --no-e2e --no-configs"
  mkdir -p $O/$m
  timeout -k 10 600 python3 $R/bench.py $args --profile-dir $O/$m > $O/$m/bench.json 2> $O/$m/bench.err || { echo BENCH_${m}_FAIL; exit 1; }
  [ $m = gen ] && cp $O/gen/bench.json $O/bench_gen.json
  echo PROF_${m}_OK
done
echo ALL_OK
