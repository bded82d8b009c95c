#!/bin/bash
# AddressSanitizer + UBSan run of the host C layer (CPU only): the C sources
# are rebuilt instrumented with gcc, linked with the (uninstrumented) HIP
# objects into build-asan/libbcp_asan.so, and the CPU test suite runs against
# it (BCP_LIB) with libasan preloaded into python.  No GPU is touched (the P
# role's fold goes through the tests' CPU test double).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/beegfs-chunk-parity_amd
B=$P/build-asan
mkdir -p $B
make -s -C $P build/bcp_kernels.o build/bcp_engine.o
CF="-std=gnu11 -O1 -g -fPIC -Wall -pthread -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -I$R/include -I$P/csrc"
objs=""
for c in $P/csrc/*.c; do
  n=$(basename $c .c)
  [ "$n" = bcp_tool ] && continue
  gcc $CF -c $c -o $B/$n.o
  objs="$objs $B/$n.o"
done
gcc -shared -fsanitize=address,undefined -o $B/libbcp_asan.so $objs $P/build/bcp_kernels.o $P/build/bcp_engine.o \
  -Wl,--version-script=$P/csrc/libbcp.map -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lstdc++ -pthread
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
cd $R
BCP_LIB=$B/libbcp_asan.so LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
  UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider --deselect tests/test_sanitize_cpu.py::test_protocol_under_threadsanitizer "$@"
