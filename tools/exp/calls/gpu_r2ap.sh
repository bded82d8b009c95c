# kind-switch stress incl. the pipelined fold, with engine
# teardown + pipeline runs (stops at the first wrong round), then the protocol tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ap; mkdir -p $O
timeout -k 10 300 python -u tools/exp/pool_switch_stress.py --rounds 40 --shutdown --pipeline > $O/stress.jsonl 2> $O/stress.err; rc=$?
grep -v '"bad_files": 0' $O/stress.jsonl | cut -c1-1500; tail -3 $O/stress.err; echo STRESS_RC $rc
[ $rc = 0 ] || exit 1
grep -q '"failing_rounds": 0' $O/stress.jsonl || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hostwrite.py > $O/pytest.log 2>&1; echo TEST_RC $?
grep -E "AssertionError|diff|passed|failed" $O/pytest.log
