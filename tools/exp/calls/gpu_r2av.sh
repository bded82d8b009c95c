# r02 call AV: pipeline batch planning for small jobs -- pipeline GPU tests,
# then config 5 end to end (full gen + changelog round).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2av; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_protocol.py -k "pipeline or round or cli" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u tools/e2e_bench.py --configs 5 --root /dev/shm/bcp_e2e --reps 3 > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; tail -20 $O/e2e.err; exit 1; }
grep -h '"path"' $O/e2e.jsonl | python -c "import sys,json; [print(d.get('config'), d['path'][:60], d.get('GiBps'), d.get('pipeline_seconds'), d.get('verified')) for d in map(json.loads, sys.stdin)]"
echo ALL_OK
