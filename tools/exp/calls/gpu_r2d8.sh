# r02 call D8: rank pools with the node fold server created and destroyed 12 times
# (new server, arena and HIP context each round), gen + rebuild checked.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2d8; mkdir -p $O
timeout -k 10 600 python -u tools/exp/fold_server_stress.py --rounds 12 > $O/stress.jsonl 2> $O/stress.err || { echo STRESS_FAIL; tail -5 $O/stress.jsonl; tail -20 $O/stress.err; rm -rf /dev/shm/bcp_fs_stress; exit 1; }
tail -3 $O/stress.jsonl
echo ALL_OK
