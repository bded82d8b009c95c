# One gpurun call, from the repo root: the device test suite, smoke(), the
# pooled-rows stress with teardowns (tools/exp/pool_switch_stress.py) and one
# bench.py line.  Every GPU step has its own time limit; the first failure
# ends the call.  Output under gpurun_out/check_<tag>/.
#   gpurun --timeout 1200 -- 'TAG=r3b bash tools/gpu_check.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/check_${TAG:-x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
cat $O/smoke.log
if [ -z "$NO_STRESS" ]; then
  timeout -k 10 300 python -u tools/exp/pool_switch_stress.py --rounds ${STRESS_ROUNDS:-30} --shutdown --pipeline \
    > $O/pool_switch.jsonl 2> $O/pool_switch.err || { echo STRESS_FAIL; tail -5 $O/pool_switch.jsonl; exit 1; }
  tail -1 $O/pool_switch.jsonl
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; exit 1; }
cat $O/bench.json
echo ALL_OK
