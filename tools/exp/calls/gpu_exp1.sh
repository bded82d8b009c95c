set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 ./tools/exp/xor_exp 12500 5 7,8,16 > gpurun_out/exp3.jsonl 2> gpurun_out/exp3.err || { echo EXP_FAIL; exit 1; }
echo ALL_OK
