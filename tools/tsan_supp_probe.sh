#!/bin/bash
# Which ROCm-runtime reports does tools/tsan_rocm.supp hide?  On a GPU box:
# the sanitizer test (default suppressions, must pass), then the TSan driver
# with only the called_from_lib lines (race:<lib> lines dropped) and with no
# suppressions at all, halt_on_error=0; logs under gpurun_out/$TAG/.
export TMPDIR=/tmp; mkdir -p gpurun_out/${TAG:-tsan_probe}
printf 'called_from_lib:libhsa-runtime64.so\ncalled_from_lib:libamdhip64.so\n' > /tmp/narrow.supp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sanitize.py -x -v --timeout 280 --timeout-method thread > gpurun_out/${TAG:-tsan_probe}/pytest_sanitize.log 2>&1 || { echo SAN_TEST_FAIL; exit 1; }
timeout -k 10 300 env TSAN_BUILD=/tmp/tsb2 TSAN_SUPP=/tmp/narrow.supp TSAN_HALT=0 bash tools/tsan_pipeline.sh > gpurun_out/${TAG:-tsan_probe}/tsan_narrow.log 2>&1; rc=$?
echo narrow_rc=$rc
[ $rc = 0 ] || [ $rc = 66 ] || exit 1
timeout -k 10 300 env TSAN_BUILD=/tmp/tsb2 TSAN_SUPP=/dev/null TSAN_HALT=0 bash tools/tsan_pipeline.sh > gpurun_out/${TAG:-tsan_probe}/tsan_none.log 2>&1; rc=$?
echo none_rc=$rc
