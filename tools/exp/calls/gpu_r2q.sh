set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
mkdir -p gpurun_out/r2q
timeout -k 10 240 python -u tools/exp/vram_rows.py > gpurun_out/r2q/vram_rows.jsonl 2> gpurun_out/r2q/vram_rows.err
rc=$?; cat gpurun_out/r2q/vram_rows.jsonl; tail -5 gpurun_out/r2q/vram_rows.err; echo RC $rc
