"""Loopback transport (the MPI stand-in) on the CPU: zero-copy fill sends
(bcp_lb_send_fill) against late and early receives, ordering with plain
sends, truncation and fill errors (tests/native/lb_test.c, linked against
libbcp.so; no GPU call is made)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "beegfs-chunk-parity_amd", "lib")


def test_fill_send_semantics(bcp, tmp_path):
    exe = tmp_path / "lb_test"
    subprocess.run(["gcc", "-O2", "-pthread", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "lb_test.c"), "-o", str(exe),
                    "-L" + LIB, "-lbcp", "-Wl,-rpath," + LIB], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
