# r02 call C1: HBM rate by read:write mix (ours vs the runtime's blit/fill and torch),
# descriptor kernel on config-5 shapes in the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c1; mkdir -p $O
timeout -k 10 400 python -u tools/exp/mix_ceiling.py --rounds 3 > $O/mix.jsonl 2> $O/mix.err || { echo MIX_FAIL; tail -20 $O/mix.err; exit 1; }
tail -1 $O/mix.jsonl
timeout -k 10 300 python -u tools/exp/desc_probe.py --workloads mixed,mixed_equal --tunings 8:1 --pipes 5 --rounds 2 > $O/desc.jsonl 2> $O/desc.err || { echo DESC_FAIL; tail -20 $O/desc.err; exit 1; }
cat $O/desc.jsonl
echo ALL_OK
