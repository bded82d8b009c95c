# r02 re-entry call C0: GPU suite, smoke and bench at head (container re-created),
# rocprofv3 kernel-trace summary of the default bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2c0; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 $R/bench.py --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -20 $O/bench_prof.err; exit 1; }
echo ALL_OK
