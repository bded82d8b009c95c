set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2s; mkdir -p $O
timeout -k 10 120 python -u tools/exp/hostwrite_free.py > $O/probe.jsonl 2> $O/probe.err; echo PROBE_RC $?
cat $O/probe.jsonl; tail -5 $O/probe.err
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_protocol.py -k pool_reuse > $O/pytest.log 2>&1; echo TEST_RC $?
grep -E "AssertionError|diff|passed|failed" $O/pytest.log
