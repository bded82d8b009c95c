set -e
for rep in 1 2; do
for lib in libbcp_old.so libbcp.so; do
export BCP_LIB=$PWD/beegfs-chunk-parity_amd/lib/$lib
timeout -k 10 200 python tools/exp/desc_probe.py --workloads uniform_desc --tunings 8:0 2>>gpurun_out/ab_tail.err | sed "s/^{/{\"lib\": \"$lib\", /" >> gpurun_out/ab_tail.jsonl
timeout -k 10 200 python bench.py --no-cpu --chunk 528384 --stripes 12000 --steps 10 2>>gpurun_out/ab_tail.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','workload':'gen_512K+4K','frac_8TBs':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_tail.jsonl
timeout -k 10 200 python bench.py --no-cpu --steps 10 2>>gpurun_out/ab_tail.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','workload':'gen_512K','frac_8TBs':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_tail.jsonl
done; done
