# r02 call BF: when does HIP load a TU's code object (deferred loading)?
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=$R/gpurun_out/r2bf; mkdir -p $O
for i in 1 2 3; do timeout -k 10 60 tools/exp/coload/coload > $O/deferred_$i.jsonl || { echo FAIL; exit 1; }; done
for i in 1 2; do HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 60 tools/exp/coload/coload > $O/eager_$i.jsonl || { echo FAIL; exit 1; }; done
for f in $O/*.jsonl; do echo "== $f"; cat $f; done
echo ALL_OK
