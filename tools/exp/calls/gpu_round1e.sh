set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1e_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 900 python -u tools/e2e_bench.py --root /dev/shm/bcp_e2e > gpurun_out/r1e_e2e.jsonl 2> gpurun_out/r1e_e2e.err || { echo E2E_FAIL; exit 1; }
echo ALL_OK
