# bench.py A/B of the streaming kernel's grid (tools only)
set -e
for round in 1 2 3 4 5; do
for g in 256 240; do
for mode in gen rebuild; do
timeout -k 10 200 python bench.py --no-cpu --steps 20 --mode $mode --grid $g 2>>gpurun_out/ab_grid.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'grid':$g,'mode':'$mode','frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms']}))" >> gpurun_out/ab_grid.jsonl
done; done; done
