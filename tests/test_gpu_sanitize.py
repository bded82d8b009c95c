"""Sanitizer runs of libbcp's host code on the device (tools/tsan_pipeline.sh):
tests/native/pipeline_driver.c runs parity gen and a rebuild through the
batched pipeline (both read paths, two device lanes, small slabs and few io
threads -- batches, slot reuse, reads and parity writes interleaving in the one
io pool) and through the per-task protocol over loopback ranks (the resident
fold ring with lane deferral, then the lane queues), every parity file checked
against the driver's own CPU XOR and every rebuilt chunk against the lost one.
ThreadSanitizer (the C host layer and the engine's host code instrumented,
device code not), then AddressSanitizer + UBSan (the C host layer); fails on
any report."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("san", ["thread", "address"])
def test_pipeline_under_sanitizers(bcp, tmp_path, san):
    env = dict(os.environ, TSAN_BUILD=str(tmp_path / "build"), TMPDIR=str(tmp_path), SAN=san)
    r = subprocess.run([os.path.join(ROOT, "tools", "tsan_pipeline.sh")], capture_output=True, text=True,
                       timeout=540, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert "OK: 0 problems" in out
