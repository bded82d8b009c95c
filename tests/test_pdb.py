"""Persistent chunk state (bcp_pdb_*), the replacement of persistent_db.{c,h}
(src/beegfs-raid5/common/persistent_db.c:23-145, LevelDB): checked against a
Python dict with LevelDB's bytewise key order, across reopen, torn-tail
recovery, compaction, version mismatch and concurrent writers."""
import os
import threading

import numpy as np
import pytest


def ref_order(d):
    return [(k, v[0], v[1]) for k, v in sorted(d.items())]  # bytes sort = memcmp, shorter first


def test_set_get_del_iterate_order(bcp, tmp_path):
    db = bcp.PDB(str(tmp_path / "db"))
    ref = {}
    rng = np.random.default_rng(1)
    keys = [b"a", b"ab", b"b", b"a/b/c", b"\xffz", b"\x01", b"u0/5F/12-5F8A2B3C-1"] + \
           [bytes(rng.integers(1, 256, size=int(rng.integers(1, 60)), dtype=np.uint8)) for _ in range(300)]
    for i, k in enumerate(keys):
        db.set(k, i, (i * 7919) & ((1 << 64) - 1))
        ref[k] = (i, (i * 7919) & ((1 << 64) - 1))
    for k in keys[::5]:
        db.delete(k)
        ref.pop(k, None)
    db.delete(b"never-set")          # deleting an absent key is a no-op
    db.set(keys[1], -5, 1 << 63)     # overwrite, negative timestamp
    ref[keys[1]] = (-5, 1 << 63)
    assert len(db) == len(ref)
    assert db.items() == ref_order(ref)
    for k in keys:
        assert db.get(k) == ref.get(k)
    db.close()


def test_reopen_persists_and_version_checked(bcp, tmp_path):
    d = str(tmp_path / "db")
    db = bcp.PDB(d)
    ref = {f"p{i:05d}".encode(): (i, i + 1) for i in range(2000)}
    for k, (ts, loc) in ref.items():
        db.set(k, ts, loc)
    for i in range(0, 2000, 3):
        db.delete(f"p{i:05d}".encode())
        ref.pop(f"p{i:05d}".encode())
    db.close()
    db = bcp.PDB(d)
    assert db.items() == ref_order(ref)
    db.close()
    # incompatible version (persistent_db.c:72-75) -> error, not silent reuse
    with pytest.raises(bcp.BcpError) as e:
        bcp.PDB(d, version=2)
    assert e.value.rc == -71  # -EPROTO


def test_torn_tail_is_dropped(bcp, tmp_path):
    d = str(tmp_path / "db")
    db = bcp.PDB(d)
    for i in range(10):
        db.set(f"k{i}", i, i)
    db.close()
    log = os.path.join(d, "bcp_pdb.log")
    good = os.path.getsize(log)
    with open(log, "ab") as f:
        f.write(b"\x01\x00\x05\x00abc")  # a record cut mid-write
    db = bcp.PDB(d)
    assert [k for k, _, _ in db.items()] == [f"k{i}".encode() for i in range(10)]
    db.set("k10", 10, 10)             # appends after the cut point
    db.close()
    assert os.path.getsize(log) > good
    db = bcp.PDB(d)
    assert len(db) == 11 and db.get("k10") == (10, 10)
    db.close()
    # a flipped byte in the last record: that record and everything after are dropped
    raw = bytearray(open(log, "rb").read())
    raw[-6] ^= 0xFF
    open(log, "wb").write(raw)
    db = bcp.PDB(d)
    assert len(db) == 10 and db.get("k10") is None
    db.close()


def test_compaction_keeps_live_entries(bcp, tmp_path):
    d = str(tmp_path / "db")
    db = bcp.PDB(d)
    for r in range(6):
        for i in range(2000):
            db.set(f"f{i}", r, i)
    for i in range(1500):
        db.delete(f"f{i}")
    size_before = os.path.getsize(os.path.join(d, "bcp_pdb.log"))
    db.close()  # 13,500 records for 500 live keys -> rewritten
    assert os.path.getsize(os.path.join(d, "bcp_pdb.log")) < size_before // 10
    db = bcp.PDB(d)
    assert db.items() == [(f"f{i}".encode(), 5, i) for i in sorted(range(1500, 2000), key=lambda i: f"f{i}")]
    db.close()


def test_reserved_and_invalid_keys(bcp, tmp_path):
    db = bcp.PDB(str(tmp_path / "db"))
    for bad in (b"?db_version", b"", b"x" * 256, b"a\x00b"):
        with pytest.raises(bcp.BcpError):
            db.set(bad, 1, 1)
    db.set(b"x" * 255, 1, 2)
    assert db.get(b"x" * 255) == (1, 2)
    db.close()


def test_concurrent_lanes(bcp, tmp_path):
    """Twelve gen lanes updating one replica at once (gen/main.c:146-149)."""
    d = str(tmp_path / "db")
    db = bcp.PDB(d)

    def lane(l):
        for i in range(400):
            db.set(f"l{l}/c{i}", l, i)
            if i % 4 == 0:
                db.delete(f"l{l}/c{i}")
    th = [threading.Thread(target=lane, args=(l,)) for l in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    want = sorted((f"l{l}/c{i}".encode(), l, i) for l in range(12) for i in range(400) if i % 4)
    assert db.items() == want
    db.close()
    db = bcp.PDB(d)
    assert db.items() == want
    db.close()
