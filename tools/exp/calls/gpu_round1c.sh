set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1c_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
echo ALL_OK
