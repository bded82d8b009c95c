set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2u; mkdir -p $O
for f in /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag /sys/kernel/mm/transparent_hugepage/khugepaged/defrag /proc/sys/vm/compact_unevictable_allowed; do echo "$f: $(cat $f 2>&1)"; done > $O/sys.txt
cat $O/sys.txt
timeout -k 10 300 python -u tools/exp/pool_switch_stress.py --rounds 30 --shutdown --pipeline > $O/stress.jsonl 2> $O/stress.err; echo RC $?
grep -v '"bad_files": 0' $O/stress.jsonl | cut -c1-1500; tail -3 $O/stress.err
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_protocol.py > $O/pytest.log 2>&1; echo TEST_RC $?
grep -E "AssertionError|diff|passed|failed" $O/pytest.log
