# A/B of two libbcp builds on the batched pipeline, alternating processes on
# one box over the same page-cache stores (tools/exp/pipeline_lib_ab.py).
#   LIB_A=ab_lib/libbcp_old.so ROUNDS=3 bash tools/exp/pipeline_lib_ab.sh > out.jsonl
# The old build has no bcp_pipeline_last_timing: its lines carry timing null.
set -o pipefail
A=${LIB_A:?}; B=${LIB_B:-beegfs-chunk-parity_amd/lib/libbcp.so}
D=${STORE:-${TMPDIR:-/tmp}/bcp_plab}
timeout -k 10 300 python -u tools/exp/pipeline_lib_ab.py --make $D || exit 1
for r in $(seq 1 ${ROUNDS:-3}); do
  for lib in "$A" "$B"; do
    BCP_LIB=$lib timeout -k 10 240 python -u tools/exp/pipeline_lib_ab.py --run $D --label "r$r" || exit 1
  done
done
rm -rf $D
