# r02 call AO: refined pipelined fold (quarter-window step, batched fallback)
# against the batched service, CPU fold and no-op, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2ao; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_protocol.py tests/test_gpu_ref.py -k "pipelined or pool" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 python -u tools/proto_compare.py --rounds 8 --folds gpu_pipelined,gpu_batched,cpu_reference,noop > $O/proto.jsonl 2> $O/proto.err || { echo PROTO_FAIL; tail -20 $O/proto.err; exit 1; }
grep summary $O/proto.jsonl
grep -h range_folds $O/proto.jsonl | python -c "import sys,json; [print(d['workload'], d['range_folds_per_window'], d.get('p_phase_us')) for d in map(json.loads, sys.stdin)]"
echo ALL_OK
