#!/bin/bash
# ThreadSanitizer run of the host C layer (CPU only): the C sources and a C
# protocol driver (tests/native/protocol_driver.c: parity gen over 12 lanes x
# 6 loopback ranks with the CPU test-double fold, then a rebuild; again with
# the pipelined fold) are built
# with -fsanitize=thread and linked with the uninstrumented HIP objects.  No
# GPU call is made.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/beegfs-chunk-parity_amd
B=$P/build-tsan
mkdir -p $B
make -s -C $P build/bcp_kernels.o build/bcp_engine.o
CF="-std=gnu11 -O1 -g -fPIC -Wall -pthread -fsanitize=thread -fno-omit-frame-pointer -I$R/include -I$P/csrc"
objs=""
for c in $P/csrc/*.c; do
  n=$(basename $c .c)
  [ "$n" = bcp_tool ] && continue
  gcc $CF -c $c -o $B/$n.o
  objs="$objs $B/$n.o"
done
gcc $CF -c $R/tests/native/protocol_driver.c -o $B/driver.o
gcc $CF -c $R/tests/native/cpu_xor_hook.c -o $B/hook.o
gcc -fsanitize=thread -o $B/protocol_driver $B/driver.o $B/hook.o $objs $P/build/bcp_kernels.o $P/build/bcp_engine.o \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lstdc++ -lm -pthread
rm -rf /tmp/bcp_tsan_store
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $B/protocol_driver /tmp/bcp_tsan_store
rm -rf /tmp/bcp_tsan_store
# the pipelined fold: row watches, sources folding the ranges they complete
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $B/protocol_driver /tmp/bcp_tsan_store pipelined
rm -rf /tmp/bcp_tsan_store
# ranks as processes: the C caller (its own st2rank / HostState) forks one
# process per target on the socketpair transport; 3 lanes per rank share
# that rank's sockets (progress by the waiting threads, unexpected messages)
gcc $CF -c $R/tests/native/caller_test.c -o $B/caller.o
gcc -fsanitize=thread -o $B/caller_test $B/caller.o $objs $P/build/bcp_kernels.o $P/build/bcp_engine.o \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lstdc++ -lm -pthread
rm -rf /tmp/bcp_tsan_caller
TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $B/caller_test /tmp/bcp_tsan_caller
rm -rf /tmp/bcp_tsan_caller
# 12 lanes per rank: the socket readers hand over and wake per request
BCP_CALLER_LANES=12 TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" $B/caller_test /tmp/bcp_tsan_caller
rm -rf /tmp/bcp_tsan_caller
