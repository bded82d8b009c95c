set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r1p; mkdir -p $O
timeout -k 10 300 python -u tools/sweep_fast.py --reps 7 --bpc 1,2 --vecs 4,8 --sched 0 > $O/sweep_fast.jsonl 2> $O/sweep.err || { echo SWEEP_FAIL; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python -u __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench_gen.json 2> $O/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode rebuild --no-cpu > $O/bench_rebuild.json 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --mode mixed --no-cpu > $O/bench_mixed.json 2>> $O/bench.err || { echo BENCH_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_gen -o run --output-format csv -- python3 $R/bench.py --no-cpu > $R/$O/prof_gen.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_reb -o run --output-format csv -- python3 $R/bench.py --mode rebuild --no-cpu > $R/$O/prof_reb.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_mix -o run --output-format csv -- python3 $R/bench.py --mode mixed --no-cpu > $R/$O/prof_mix.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/$O/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $R/$O/pmc_write.log 2>&1 || { echo PMC2_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmcr_fetch -o run -- python3 $R/bench.py --mode rebuild --steps 3 --warmup 1 --no-cpu > $R/$O/pmcr_fetch.log 2>&1 || { echo PMC3_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmcr_write -o run -- python3 $R/bench.py --mode rebuild --steps 3 --warmup 1 --no-cpu > $R/$O/pmcr_write.log 2>&1 || { echo PMC4_FAIL; exit 1; }
cd $R
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 6000 > $O/bench_n2.log 2>&1 || { echo BENCH2_FAIL; exit 1; }
echo ALL_OK
