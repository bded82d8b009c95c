# same-box A/B of library builds on the descriptor probe (tools only)
set -e
for rep in 1 2; do
for lib in $AB_LIBS; do
BCP_LIB=$PWD/beegfs-chunk-parity_amd/lib/$lib timeout -k 10 200 python tools/exp/desc_probe.py --tunings ${AB_TUNINGS:-8:0} 2>>gpurun_out/ab_desc.err | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/ab_desc.jsonl
done; done
