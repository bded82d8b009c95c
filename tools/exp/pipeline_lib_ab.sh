# A/B of libbcp builds on the batched pipeline, alternating processes on one
# box over the same page-cache stores (tools/exp/pipeline_lib_ab.py).
#   LIBS="ab_lib/libbcp_old.so beegfs-chunk-parity_amd/lib/libbcp.so" ROUNDS=3 \
#     bash tools/exp/pipeline_lib_ab.sh > out.jsonl
# (LIB_A=x alone: x against the in-tree build.)  Builds without
# bcp_pipeline_last_timing print timing null.  The order rotates per round.
set -o pipefail
LIBS=${LIBS:-"${LIB_A:?} beegfs-chunk-parity_amd/lib/libbcp.so"}
D=${STORE:-/dev/shm/bcp_plab}  # in memory: no disk writeback behind the page cache
timeout -k 10 300 python -u tools/exp/pipeline_lib_ab.py --make $D || exit 1
set -- $LIBS
for r in $(seq 1 ${ROUNDS:-3}); do
  for ent in "$@"; do  # "lib" or "lib@nslots"
    lib=${ent%@*}; ns=4; [ "$ent" != "$lib" ] && ns=${ent#*@}
    PLAB_NSLOTS=$ns BCP_LIB=$lib timeout -k 10 240 python -u tools/exp/pipeline_lib_ab.py --run $D --label "r$r" || exit 1
  done
  set -- "${@:2}" "$1"
done
rm -rf $D
