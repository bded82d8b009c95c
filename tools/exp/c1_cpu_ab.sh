#!/bin/bash
# Alternating-process A/B of two libbcp builds on tools/exp/c1_cpu_cost.py
# (config 1 gen through the protocol with a no-op fold: CPU seconds and wall
# per run, beside the kernel-copy floor).  Usage:
#   bash tools/exp/c1_cpu_ab.sh <old libbcp.so> <rounds> [lanes] > out.jsonl
set -e
OLD=$1; ROUNDS=${2:-3}; LANES=${3:-12}
NEW=$(dirname "$0")/../../beegfs-chunk-parity_amd/lib/libbcp.so
for r in $(seq 1 "$ROUNDS"); do
  if [ $((r % 2)) -eq 1 ]; then order="$OLD $NEW"; else order="$NEW $OLD"; fi
  for lib in $order; do
    BCP_LIB=$(readlink -f "$lib") timeout -k 10 200 python3 -u "$(dirname "$0")/c1_cpu_cost.py" --rounds 3 --lanes "$LANES"
  done
done
