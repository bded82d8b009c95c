# bench.py A/B: contiguous (default) vs default device allocations (tools only)
set -e
for round in 1 2 3; do
for flag in "" "--no-contig"; do
for mode in gen rebuild mixed; do
timeout -k 10 200 python bench.py --no-cpu --steps 20 --mode $mode $flag 2>>gpurun_out/ab_contig.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'contig': '$flag' == '', 'mode':'$mode','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_contig.jsonl
done; done; done
