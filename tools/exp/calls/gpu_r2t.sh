set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2t; mkdir -p $O
timeout -k 10 300 python -u tools/exp/pool_switch_stress.py --rounds 36 > $O/stress.jsonl 2> $O/stress.err; echo RC $?
cat $O/stress.jsonl | cut -c1-600; tail -5 $O/stress.err
