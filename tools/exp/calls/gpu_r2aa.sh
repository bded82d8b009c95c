# r02 call AA: rank processes sharing ONE GPU -- 9 vs 8 vs 5 processes
# (config-5 shapes), to see whether GPU folds collapse past the number of
# processes the GPU schedules concurrently.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2aa; mkdir -p $O
for f in /sys/module/amdgpu/parameters/hws_max_conc_proc /sys/module/amdgpu/parameters/sched_policy /sys/module/amdgpu/parameters/vm_size; do echo "$f: $(cat $f 2>&1)"; done > $O/sys.txt; cat $O/sys.txt
for t in 9 8 5; do
  timeout -k 10 300 python -u tools/proto_compare.py --procs --rounds 4 --workloads c5_gen --c5-targets $t --c5-stripes 600 --folds gpu_batched,cpu_reference > $O/pool_t$t.jsonl 2> $O/pool_t$t.err || { echo POOL_FAIL $t; tail -20 $O/pool_t$t.err; exit 1; }
  grep summary $O/pool_t$t.jsonl
done
echo ALL_OK
