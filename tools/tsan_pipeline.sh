#!/bin/bash
# ThreadSanitizer (SAN=thread, the default) or AddressSanitizer + UBSan
# (SAN=address) run of libbcp's host code ON A GPU BOX
# (tests/test_gpu_sanitize.py): tests/native/pipeline_driver.c runs parity gen
# and a rebuild through the batched pipeline (both read paths, two device
# lanes) and through the per-task protocol over loopback ranks (fold ring with
# lane deferral, then the lane queues), checking every parity file and rebuilt
# chunk.  Fails on any sanitizer report.
#  thread:  the C host layer with ROCm's clang and the engine's host code
#           (bcp_engine.hip: fold ring submission / waits, queues, pools) with
#           hipcc -Xarch_host -fsanitize=thread; device code uninstrumented.
#  address: the C host layer with gcc; the HIP objects uninstrumented.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/beegfs-chunk-parity_amd
SAN=${SAN:-thread}
B=${TSAN_BUILD:-$P/build-tsan}
ROCM=${ROCM:-/opt/rocm}
mkdir -p $B
if [ "$SAN" = address ]; then
  CC=gcc
  FS="-fsanitize=address,undefined -fno-sanitize-recover=undefined"
  LD="gcc $FS"
  HIPOBJS="$P/build/bcp_kernels.o $P/build/bcp_engine.o"
else
  CC=$ROCM/lib/llvm/bin/clang
  FS="-fsanitize=thread"
  LD="$ROCM/lib/llvm/bin/clang++ $FS"
  HF="--offload-arch=gfx950 -O1 -g -fPIC -std=c++17 -Wall -I$R/include -I$P/csrc"
  $ROCM/bin/hipcc $HF -Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer -c $P/csrc/bcp_engine.hip -o $B/bcp_engine.o
  HIPOBJS="$P/build/bcp_kernels.o $B/bcp_engine.o"
fi
CF="-std=gnu11 -O1 -g -fPIC -Wall -pthread $FS -fno-omit-frame-pointer -I$R/include -I$P/csrc"
objs=""
for c in $P/csrc/*.c; do
  n=$(basename $c .c)
  [ "$n" = bcp_tool ] && continue
  $CC $CF -c $c -o $B/$n.o
  objs="$objs $B/$n.o"
done
$CC $CF -c $R/tests/native/pipeline_driver.c -o $B/pipeline_driver.o
$LD -o $B/pipeline_driver $B/pipeline_driver.o $objs $HIPOBJS \
  -L$ROCM/lib -lamdhip64 -Wl,-rpath,$ROCM/lib -lstdc++ -lm -pthread
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
