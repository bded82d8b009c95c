set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_gen.json 2> $O/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > $O/bench_rebuild.json 2>> $O/bench.err || { echo BENCHRB_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu > $O/bench_mixed.json 2>> $O/bench.err || { echo BENCHMX_FAIL; exit 1; }
timeout -k 10 900 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e > $O/e2e.jsonl 2> $O/e2e.err || { echo E2E_FAIL; exit 1; }
rm -rf /dev/shm/bcp_e2e
echo ALL_OK
