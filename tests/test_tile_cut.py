"""The descriptor kernel's tile cut, on the CPU: the engine's O(nsrc) tile
count (count_tiles) against the per-subtile rule desc_tiles applies on the
device (tests/native/tile_cut_test.cpp, built with hipcc, host code only)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tile_count_matches_device_rule(tmp_path):
    exe = tmp_path / "tile_cut_test"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17",
                    "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "beegfs-chunk-parity_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "tile_cut_test.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
