# r02 call BJ: the open-after-receives change alone (early prefix write
# removed): protocol GPU tests, then the interleaved A/B against the
# reference's order and both CPU baselines.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2bj; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_protocol.py tests/test_gpu_ref.py -p no:cacheprovider > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u tools/proto_compare.py --rounds 7 --folds gpu_pipelined,gpu_pipelined_serial,cpu_reference,cpu_pipelined,noop > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; exit 1; }
grep -h '"box"' $O/ab.jsonl; grep summary $O/ab.jsonl
echo ALL_OK
