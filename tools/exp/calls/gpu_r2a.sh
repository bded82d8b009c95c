# r02 call A: full GPU suite (incl. reference fixtures, config-4 shard, bench
# under torchrun), then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -eq 0 ] || { echo PYTEST_FAIL $rc; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_gen.json 2> $O/bench_gen.err || { echo BENCH_FAIL; exit 1; }
cat $O/bench_gen.json
echo ALL_OK
