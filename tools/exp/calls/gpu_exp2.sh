set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 ./tools/exp/xor_exp2 12500 5 > gpurun_out/exp7.jsonl 2> gpurun_out/exp7.err || { echo EXP_FAIL; exit 1; }
echo ALL_OK
