#!/bin/bash
# Diagnostic libbcp with lock-contention counters (tools/exp/lockstat/lockstat.h)
# into ab_lib/lockstat/lib/libbcp.so; the HIP objects are the in-tree ones.
set -e
R=$(cd "$(dirname "$0")/../../.." && pwd)
P=$R/beegfs-chunk-parity_amd
O=$R/ab_lib/lockstat
make -C "$P" -j16 >/dev/null
mkdir -p "$O/build" "$O/lib"
for c in "$P"/csrc/*.c; do
  [ "$(basename "$c")" = bcp_tool.c ] && continue
  gcc -std=gnu11 -D_GNU_SOURCE -O2 -fPIC -pthread -I"$R/include" -I"$P/csrc" -include "$R/tools/exp/lockstat/lockstat.h" \
      -c "$c" -o "$O/build/$(basename "${c%.c}").o"
done
gcc -O2 -fPIC -pthread -c "$R/tools/exp/lockstat/lockstat.c" -o "$O/build/lockstat.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$O/lib/libbcp.so" "$O"/build/*.o \
    "$P/build/bcp_kernels.o" "$P/build/bcp_engine.o" -lpthread
echo "$O/lib/libbcp.so"
