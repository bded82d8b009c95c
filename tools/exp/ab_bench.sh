# bench.py A/B of two library builds (tools only): AB_MODE, AB_ROUNDS
set -e
for round in $(seq ${AB_ROUNDS:-3}); do
for lib in libbcp_old.so libbcp.so; do
BCP_LIB=$PWD/beegfs-chunk-parity_amd/lib/$lib timeout -k 10 200 python bench.py --no-cpu --steps 20 --mode ${AB_MODE:-gen} 2>>gpurun_out/ab_bench.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','mode':'${AB_MODE:-gen}','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_bench.jsonl
done; done
