# rocprofv3 kernel-trace of the descriptor probe (tools only)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/probe_prof -o run --output-format csv -- python3 $R/tools/exp/desc_probe.py --tunings 8:1 --workloads mixed,uniform_forced > $R/gpurun_out/probe_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo OK
