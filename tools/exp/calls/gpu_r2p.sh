# r02 call P: CPU writes into fine-grained device memory (BAR) probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2p; mkdir -p $O
timeout -k 10 120 python -u tools/exp/host_to_vram.py > $O/host_to_vram.jsonl 2> $O/host_to_vram.err; rc=$?
cat $O/host_to_vram.jsonl; tail -5 $O/host_to_vram.err
echo RC $rc
