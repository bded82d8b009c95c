"""ThreadSanitizer run of the host C layer on the CPU (tools/tsan_host.sh):
parity gen over 6 loopback ranks x 12 lanes and a rebuild (CPU test-double
fold), a run where one rank's parity writes fail from many lanes at
once (the sticky error is raised once, race-free; the reference writes it
unlocked), and the C caller test with one forked process per
rank on the socketpair transport (3, then 12 lanes per rank share its sockets).  Fails
on any TSan report."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_protocol_under_threadsanitizer(bcp):
    r = subprocess.run([os.path.join(ROOT, "tools", "tsan_host.sh")], capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ThreadSanitizer" not in out, out[-4000:]
    assert "OK: 0 problems" in out
    assert "caller_test ok" in out
