#!/bin/bash
# Alternating-process A/B of two libbcp builds on tools/proto_compare.py
# (the per-task protocol with the GPU fold, the reference's fold and a no-op
# fold; config 1 gen and rebuild by default).  Each line gains "lib".  Usage:
#   bash tools/exp/proto_lib_ab.sh <old libbcp.so> <rounds> [proto_compare args] > out.jsonl
set -e
OLD=$(readlink -f "$1"); ROUNDS=${2:-3}; shift 2
ARGS=${*:-"--workloads c1_gen,c1_rebuild --rounds 5 --folds gpu_pipelined,cpu_reference,noop"}
NEW=$(readlink -f "$(dirname "$0")/../../beegfs-chunk-parity_amd/lib/libbcp.so")
for r in $(seq 1 "$ROUNDS"); do
  if [ $((r % 2)) -eq 1 ]; then order="$OLD $NEW"; else order="$NEW $OLD"; fi
  for lib in $order; do
    # shellcheck disable=SC2086
    BCP_LIB=$lib timeout -k 10 300 python3 -u "$(dirname "$0")/../proto_compare.py" $ARGS --root /dev/shm/bcp_proto_ab \
      | python3 -c "import json,sys
for l in sys.stdin:
    d = json.loads(l); d['lib'] = sys.argv[1]; print(json.dumps(d), flush=True)" "$lib"
  done
done
