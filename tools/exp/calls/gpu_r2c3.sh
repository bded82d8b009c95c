# r02 call C3: narrow-stripe schedule variants (tools/exp/xor_exp6.hip), N = 3 and 4.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c3; mkdir -p $O
timeout -k 10 300 ./tools/exp/xor_exp6 24 5 > $O/exp6.jsonl 2> $O/exp6.err || { echo EXP_FAIL; tail -20 $O/exp6.err; exit 1; }
cat $O/exp6.jsonl
timeout -k 10 300 ./tools/exp/xor_exp6 24 5 > $O/exp6b.jsonl 2> $O/exp6b.err || { echo EXP_FAIL; tail -20 $O/exp6b.err; exit 1; }
cat $O/exp6b.jsonl
echo ALL_OK
