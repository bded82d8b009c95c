# Round-end check on one GPU box: the O_DIRECT slab probe, the whole GPU
# suite, smoke() and a default bench line; every step under its own limit,
# the first failure ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r4z}
mkdir -p $OUT
timeout -k 10 120 python -u tools/exp/direct_slab_probe.py > $OUT/direct_slab.jsonl 2> $OUT/direct_slab.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
