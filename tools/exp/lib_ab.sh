# A/B of two libbcp builds through bench.py in alternating processes on one
# box (bcp_ctypes loads $BCP_LIB when set).  Used in r03 to check that pruning
# the losing kernel variants left the shipped kernels' rates unchanged.
#   LIB_A=ab_lib/libbcp_old.so ROUNDS=3 MODES="gen mixed" bash tools/exp/lib_ab.sh > out.jsonl
set -o pipefail
A=${LIB_A:?}; B=${LIB_B:-beegfs-chunk-parity_amd/lib/libbcp.so}
for r in $(seq 1 ${ROUNDS:-3}); do
  for m in ${MODES:-gen mixed}; do
    for lib in "$A" "$B"; do
      line=$(BCP_LIB=$lib timeout -k 10 120 python -u bench.py --mode $m --steps 20 --warmup 3 --no-cpu | tail -1) || exit 1
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $r, 'mode': '$m', 'lib': sys.argv[2], 'ms': d['ms_per_step'], 'frac_event': d['roofline']['frac_event'], 'kernel': d['roofline'].get('kernel'), 'verified': d['config']['verified_on_device']}))" "$line" "$lib" || exit 1
    done
  done
done
