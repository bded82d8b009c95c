set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
df -h /tmp $R /dev/shm > gpurun_out/r1d_df.txt 2>&1 || true
free -g >> gpurun_out/r1d_df.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > gpurun_out/r1d_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 900 python -u tools/e2e_bench.py --root /tmp/bcp_e2e > gpurun_out/r1d_e2e.jsonl 2> gpurun_out/r1d_e2e.err || { echo E2E_FAIL; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 6000 > gpurun_out/r1d_bench_n2.log 2>&1 || { echo BENCH2_FAIL; exit 1; }
echo ALL_OK
