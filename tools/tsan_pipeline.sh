#!/bin/bash
# ThreadSanitizer (SAN=thread, the default) or AddressSanitizer + UBSan
# (SAN=address) run of the batched pipeline's host code ON A GPU BOX
# (tests/test_gpu_sanitize.py): the C sources are built with -fsanitize=...
# (gcc, host code only) and linked with the uninstrumented HIP objects;
# tests/native/pipeline_driver.c runs parity gen through both read paths and
# two device lanes, checks every parity file against its own CPU XOR, then
# rebuilds a lost target.  Fails on any sanitizer report.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/beegfs-chunk-parity_amd
SAN=${SAN:-thread}
B=${TSAN_BUILD:-$P/build-tsan}
mkdir -p $B
FS=$([ "$SAN" = address ] && echo "-fsanitize=address,undefined -fno-sanitize-recover=undefined" || echo "-fsanitize=thread")
CF="-std=gnu11 -O1 -g -fPIC -Wall -pthread $FS -fno-omit-frame-pointer -I$R/include -I$P/csrc"
objs=""
for c in $P/csrc/*.c; do
  n=$(basename $c .c)
  [ "$n" = bcp_tool ] && continue
  gcc $CF -c $c -o $B/$n.o
  objs="$objs $B/$n.o"
done
gcc $CF -c $R/tests/native/pipeline_driver.c -o $B/pipeline_driver.o
gcc $FS -o $B/pipeline_driver $B/pipeline_driver.o $objs $P/build/bcp_kernels.o $P/build/bcp_engine.o \
  -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lstdc++ -lm -pthread
if [ -n "${BUILD_ONLY:-}" ]; then exit 0; fi
S=${TMPDIR:-/tmp}/bcp_tsan_pipeline_$$
rm -rf $S
# setarch -R: no address-space randomisation (TSan's fixed shadow layout
# refuses the high-entropy mmap bases of newer kernels: "unexpected memory
# mapping"); the driver is exec'ed before anything touches the GPU
if [ "$SAN" = address ]; then
  # protect_shadow_gap=0: the GPU driver maps memory inside ASan's shadow gap
  ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:protect_shadow_gap=0" UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" \
    $B/pipeline_driver $S
else
  # TSAN_SUPP / TSAN_HALT: another suppression file (e.g. /dev/null) and
  # halt_on_error=0 -- to list the ROCm-runtime reports the file suppresses
  TSAN_OPTIONS="halt_on_error=${TSAN_HALT:-1} second_deadlock_stack=1 suppressions=${TSAN_SUPP:-$R/tools/tsan_rocm.supp}" \
    setarch "$(uname -m)" -R $B/pipeline_driver $S
fi
rm -rf $S
