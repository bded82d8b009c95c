"""The node fold server for rank processes that no rank pool forked (an MPI
job's shape): a server process on a Unix socket (bcp_fold_server_serve),
clients that connect (bcp_fold_server_connect) and then run the per-task
protocol -- their window rows in a memfd arena the server maps at another
address, their folds done by the server.  On the CPU both sides use the
test double of tests/native/cpu_xor_hook.c (the server folds with its own
copy); parity against the oracle, the server's fold count, and a client
whose server went away failing its tasks instead of hanging."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bcp_store as S

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

SERVER = r"""
import ctypes, os, sys
sys.path[:0] = [os.path.join(sys.argv[2], "beegfs-chunk-parity_amd"), os.path.join(sys.argv[2], "tests")]
import bcp_ctypes as bcp
if sys.argv[4] == "hook":
    h = ctypes.CDLL(sys.argv[5])
    bcp.set_xor_hook(ctypes.cast(h.test_cpu_xor, ctypes.c_void_p).value)
print("serving", flush=True)
bcp.fold_server_serve(sys.argv[1], int(sys.argv[3]))
print("served", flush=True)
"""

CLIENT = r"""
import ctypes, os, sys, json
sys.path[:0] = [os.path.join(sys.argv[2], "beegfs-chunk-parity_amd"), os.path.join(sys.argv[2], "oracle"),
                os.path.join(sys.argv[2], "tests")]
import numpy as np
import bcp_ctypes as bcp, bcp_store as S, oracle
root, mode, nconn = sys.argv[3], sys.argv[4], int(sys.argv[6])
if mode == "hook":
    h = ctypes.CDLL(sys.argv[5])
    bcp.set_xor_hook(ctypes.cast(h.test_cpu_xor, ctypes.c_void_p).value)
bcp.set_fold_mode({"pipelined": bcp.FOLD_PIPELINED, "batched": bcp.FOLD_BATCHED}[sys.argv[7]])
bcp.fold_server_connect(sys.argv[1], 256 << 20, nconn)
rng = np.random.default_rng(int(sys.argv[8]))
nt = 6
files = []
for i in range(30):
    holders, p = S.random_layout(rng, nt, int(rng.integers(1, 6)))
    files.append((f"f{i % 3}/c{i}", holders, p, [int(x) for x in rng.integers(0, 700_000, size=len(holders))]))
files.append(("big/m", [0, 2], 4, [10 * 1024 * 1024 + 9, 12 * 1024 * 1024]))
items, contents = S.populate(root, nt, files, seed=3)
st = bcp.gen_run(root, nt, items, nlanes=4)
def same(fn, want):
    try:
        return S.read_file(fn) == want
    except OSError:
        return False
bad = [path for (path, h, p, lens) in files if not same(S.parity_path(root, p, path), oracle.gen_parity_file(contents[path]))]
victim, lost = 1, {}
for (path, holders, p, lens) in files:
    if victim in holders:
        lost[path] = S.read_file(S.chunk_path(root, victim, path))
        os.remove(S.chunk_path(root, victim, path))
rb = bcp.rebuild_run(root, nt, victim, items)
bad += [path for path, data in lost.items() if not same(S.chunk_path(root, victim, path), data)]
print(json.dumps({"errors": st.errors, "rb_errors": rb.errors, "bad": bad, "server_folds": bcp.fold_server_stats(),
                  "pipe": bcp.pipe_stats()}))
"""


def _hook_so(tmp_path):
    so = str(tmp_path / "libcpuhook.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(HERE, "native", "cpu_xor_hook.c")],
                   check=True)
    return so


@pytest.mark.timeout(240)
@pytest.mark.parametrize("fold", ["pipelined", "batched"])
def test_connected_clients_fold_through_the_server(tmp_path, fold):
    """Two client processes (loopback ranks inside each) on one server, 3
    connections each: every window the clients' P roles fold goes to the
    server, which maps each client's memfd arena at its own address."""
    so = _hook_so(tmp_path)
    sock = str(tmp_path / "fs.sock")
    srv = subprocess.Popen([sys.executable, "-c", SERVER, sock, ROOT, "6", "hook", so], stdout=subprocess.PIPE,
                           text=True)
    assert srv.stdout.readline().strip() == "serving"
    import time
    for _ in range(200):
        if os.path.exists(sock):
            break
        time.sleep(0.01)
    clients = [subprocess.Popen([sys.executable, "-c", CLIENT, sock, ROOT, str(tmp_path / f"store{k}"), "hook", so,
                                 "3", fold, str(10 + k)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
               for k in range(2)]
    import json
    for c in clients:
        out, err = c.communicate(timeout=200)
        assert c.returncode == 0, err[-3000:]
        d = json.loads(out.strip().splitlines()[-1])
        assert d["errors"] == 0 and d["rb_errors"] == 0 and d["bad"] == [], d
        # every window (a P role folding through a server takes whole windows
        # in PIPELINED mode too)
        assert d["server_folds"] > 40, d
    srv_out, _ = srv.communicate(timeout=60)
    assert srv.returncode == 0 and "served" in srv_out


@pytest.mark.timeout(120)
def test_client_without_a_server_fails_tasks_not_the_run(tmp_path):
    """The server accepts the client's connections and exits at once (it was
    told to serve 0 requests by closing them): the client's folds fail, its
    ranks raise the sticky error, and the run returns."""
    so = _hook_so(tmp_path)
    sock = str(tmp_path / "fs.sock")
    # a "server" that accepts and closes every connection
    import socket
    import threading
    ls = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    ls.bind(sock)
    ls.listen(16)

    def closer():
        for _ in range(3):
            c, _ = ls.accept()
            c.recv(64)
            c.close()
    t = threading.Thread(target=closer, daemon=True)
    t.start()
    c = subprocess.run([sys.executable, "-c", CLIENT, sock, ROOT, str(tmp_path / "store"), "hook", so, "3",
                        "batched", "5"], capture_output=True, text=True, timeout=100)
    ls.close()
    assert c.returncode == 0, c.stderr[-3000:]
    import json
    d = json.loads(c.stdout.strip().splitlines()[-1])
    assert d["errors"] > 0 and d["server_folds"] == 0
