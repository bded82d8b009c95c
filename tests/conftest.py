import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "beegfs-chunk-parity_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbcp.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def bcp():
    """libbcp ctypes module; GPU tests fail (not skip) when the device or library is missing."""
    import bcp_ctypes
    if not os.path.exists(bcp_ctypes.LIB_PATH):
        bcp_ctypes.build()
    bcp_ctypes.lib()
    return bcp_ctypes


@pytest.fixture(scope="session")
def engine(bcp):
    n = bcp.device_count()
    assert n > 0, "gpu test needs a HIP device (no CPU fallback exists)"
    eng = bcp.Engine(0)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def queue(engine):
    q = engine.queue()
    yield q
    q.close()


@pytest.fixture(scope="session")
def cpu_hook_lib(bcp, tmp_path_factory):
    """Test double for the P role's fold (tests/native/cpu_xor_hook.c)."""
    out = tmp_path_factory.mktemp("hook") / "libcpuxor.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", str(out),
                    os.path.join(os.path.dirname(__file__), "native", "cpu_xor_hook.c")], check=True)
    return ctypes.CDLL(str(out))


@pytest.fixture(scope="session")
def foreign_ops_addr(bcp, tmp_path_factory):
    """Address of a caller's transport table (tests/native/foreign_ops.c: the
    loopback ranks behind wrappers, no send_fill -- an MPI binding's shape)."""
    out = tmp_path_factory.mktemp("fops") / "libforeignops.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", os.path.join(ROOT, "include"), "-o", str(out),
                    os.path.join(os.path.dirname(__file__), "native", "foreign_ops.c"), bcp.LIB_PATH,
                    f"-Wl,-rpath,{os.path.dirname(bcp.LIB_PATH)}"], check=True)
    L = ctypes.CDLL(str(out))
    L.foreign_ops.restype = ctypes.c_void_p
    return L.foreign_ops()


@pytest.fixture
def cpu_hook(bcp, cpu_hook_lib):
    """Route the P role's fold to the CPU test double for one test (host-logic
    tests on machines without a GPU; the product never sets the hook)."""
    bcp.set_xor_hook(ctypes.cast(cpu_hook_lib.test_cpu_xor, ctypes.c_void_p).value)
    yield cpu_hook_lib
    bcp.set_xor_hook(None)
