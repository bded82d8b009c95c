set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1q; mkdir -p $O
for v in 4 8; do for b in 1 2; do for g in 1 2; do
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu --steps 10 --vecs $v --blocks-per-cu $b --grab $g >> $O/bench_mixed.jsonl 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
done; done; done
echo ALL_OK
