"""C-ABI checks that need no GPU: libbcp.so loads, exports every function
include/*.h declares, and fails loudly (-ENODEV) instead of falling back to
the CPU when no device is present."""
import ctypes
import errno
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*\**\s*([a-z_][a-z0-9_]*)\s*\(", re.M)


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", text)
        text = re.sub(r"typedef\s+struct[^{;]*\{.*?\}[^;]*;", "", text, flags=re.S)  # struct bodies
        text = re.sub(r"typedef[^;]*;", "", text)
        for m in DECL.finditer(text):
            name = m.group(1)
            if name not in ("if", "while", "for", "return", "sizeof"):
                names.add(name)
    return sorted(names)


def test_headers_declare_functions():
    names = declared_functions()
    assert "bcp_xor_parity" in names and "bcp_xor_stripes_async" in names
    assert "process_task" in names and "bcp_gen_run" in names and "bcp_lb_send" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol(bcp):
    out = subprocess.run(["nm", "-D", "--defined-only", bcp.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_abi_version(bcp):
    assert bcp.lib().bcp_abi_version() == 4


def test_headers_compile_as_c_and_cxx(tmp_path):
    src = tmp_path / "t.c"
    src.write_text("".join(f'#include "{os.path.basename(h)}"\n' for h in glob.glob(os.path.join(ROOT, "include", "*.h")))
                   + "int main(void){return 0;}\n")
    for cc, extra in (("gcc", ["-std=c99"]), ("g++", ["-x", "c++", "-std=c++17"])):
        subprocess.run([cc, *extra, "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o",
                        str(tmp_path / "t.o")], check=True)


def test_no_device_is_an_error_not_a_fallback(bcp):
    if bcp.device_count() > 0:
        pytest.skip("a GPU is present")
    L = bcp.lib()
    h = ctypes.c_void_p()
    assert L.bcp_engine_create(0, ctypes.byref(h)) == -errno.ENODEV
    dst = (ctypes.c_uint8 * 64)()
    src = (ctypes.c_uint8 * 128)()
    assert L.bcp_xor_parity(dst, 64, src, 2) == -errno.ENODEV


def test_argument_validation_without_device(bcp):
    L = bcp.lib()
    assert L.bcp_xor_parity(None, 0, None, 1) == 0           # nothing to do
    assert L.bcp_xor_parity(None, 16, None, 0) == -errno.EINVAL
    assert L.bcp_xor_parity(None, 16, None, 57) == -errno.EINVAL
    assert L.bcp_engine_create(0, None) == -errno.EINVAL
    assert L.bcp_queue_sync(None) == -errno.EINVAL
    assert L.bcp_strerror(-errno.ENODEV) == b"no usable HIP device"
    t = bcp.PipelineTiming()
    assert L.bcp_pipeline_last_timing(None, ctypes.byref(t)) == -errno.EINVAL
    assert L.bcp_pipeline_destroy(None) == -errno.EINVAL
    r = ctypes.c_void_p()
    assert L.bcp_ring_create(None, 0, 0, ctypes.byref(r)) == -errno.EINVAL
    assert L.bcp_ring_wait(None, 0) == -errno.EINVAL
    assert L.bcp_ring_query(None, 0) == -errno.EINVAL
    assert L.bcp_ring_destroy(None) == -errno.EINVAL
    assert L.bcp_ring_submit(None, None, None, None) == -errno.EINVAL


def test_host_buffer_bounds_checked(bcp):
    """The binding refuses an nbytes beyond the host buffer and a read-only
    buffer as a copy destination, before any HIP call."""
    import numpy as np
    a = np.zeros(64, np.uint8)
    assert bcp._host_addr(a, 64) == (a.ctypes.data, 64)
    with pytest.raises(ValueError):
        bcp._host_addr(a, 65)
    with pytest.raises(ValueError):
        bcp._host_addr(b"\0" * 16, 16, writable=True)
    ro = np.zeros(16, np.uint8)
    ro.flags.writeable = False
    with pytest.raises(ValueError):
        bcp._host_addr(ro, None, writable=True)
    with pytest.raises(ValueError):
        bcp._host_addr(a[::2], None)
    with pytest.raises(ValueError):
        bcp._host_addr(12345, None)
    with pytest.raises(ValueError):
        bcp.xor_parity(np.zeros(8, np.uint8), 8, np.zeros(15, np.uint8), 2)  # data shorter than 2 rows
