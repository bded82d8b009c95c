set -e
for rep in 1 2; do
for lib in libbcp_old.so libbcp.so; do
for cfg in "2 8" "2 4" "4 4"; do
set -- $cfg
BCP_LIB=$PWD/beegfs-chunk-parity_amd/lib/$lib timeout -k 10 120 python bench.py --mode mixed --no-cpu --steps 10 --blocks-per-cu $1 --vecs $2 > gpurun_out/tmp.json 2>>gpurun_out/ab.err
python3 -c "import json,sys; d=json.load(open('gpurun_out/tmp.json')); r=d['roofline']; print(json.dumps({'lib':'$lib','bpc':$1,'vecs':$2,'kernel_ms':r['kernel_ms'],'frac':r['frac'],'verified':d['config'].get('verified_on_device')}))" >> gpurun_out/ab_mixed.jsonl
done; done; done
