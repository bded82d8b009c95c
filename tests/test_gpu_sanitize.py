"""Sanitizer runs of the batched pipeline's host code on the device
(tools/tsan_pipeline.sh): the C host layer built with -fsanitize=thread
(host code only; the HIP objects uninstrumented), tests/native/
pipeline_driver.c running parity gen through both read paths and two device
lanes with small slabs and few io threads -- batches, slot reuse, reads and
parity writes interleaving in the one io pool -- every parity file checked
against the driver's own CPU XOR, then a lost target rebuilt and compared.
ThreadSanitizer, then AddressSanitizer + UBSan; fails on any report."""
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
