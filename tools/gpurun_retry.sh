# Local helper (this container): run one gpurun call, and only when gpurun
# reports that NO box ran the command (all slots busy / box lost while being
# prepared: status=transient, nothing charged) wait and submit it again.  A
# call that ran -- whatever its exit code -- is never repeated.
#   bash tools/gpurun_retry.sh <out file> <timeout s> '<command>'
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  if grep -q "status=transient rc=None" "$out"; then
    sleep 120
    continue
  fi
  break
done
tail -30 "$out"
