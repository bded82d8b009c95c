# r02 call D2: the node fold server for connected client processes on the device,
# the rank-pool tests, and a per-task comparison: loopback ranks in one client
# process folding through a server process vs folding in-process.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 240 --timeout-method thread -k "node_fold_server or rank_pool" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo ALL_OK
