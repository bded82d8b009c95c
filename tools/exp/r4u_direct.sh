set -o pipefail
mkdir -p gpurun_out/r4u
( df -T . /tmp /dev/shm ${TMPDIR:-/tmp}; echo TMPDIR=$TMPDIR; stat -f -c '%T %n' . /tmp /dev/shm; nproc; free -g ) > gpurun_out/r4u/fs.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pipeline or read_modes or cli" > gpurun_out/r4u/tests.log 2>&1 &&
timeout -k 10 500 python -u tools/e2e_full.py --root ./e2e_disk_store --stripes 2500 --reps 2 --modes copy,direct --evict > gpurun_out/r4u/e2e_disk.jsonl 2> gpurun_out/r4u/e2e_disk.err &&
timeout -k 10 300 python -u tools/e2e_full.py --root /dev/shm/bcp_e2e_r4u --stripes 2500 --reps 2 --modes copy,direct > gpurun_out/r4u/e2e_shm.jsonl 2> gpurun_out/r4u/e2e_shm.err
rc=$?; rm -rf ./e2e_disk_store /dev/shm/bcp_e2e_r4u; exit $rc
