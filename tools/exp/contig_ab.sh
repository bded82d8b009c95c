# physically contiguous vs default device allocations (tools only)
set -e
for round in 1 2 3; do
for c in 0 1; do
  XE3_CONTIG=$c timeout -k 10 150 ./tools/exp/xor_exp3 12500 5 2>>gpurun_out/contig.err | sed "s/^{/{\"contig\": $c, \"round\": $round, /" >> gpurun_out/contig.jsonl
done; done
