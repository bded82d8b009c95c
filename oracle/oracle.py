"""TEST INFRASTRUCTURE ONLY -- the parity oracle.

ctypes wrapper over ``oracle/build/liboracle.so`` (the C restatement of the
reference XOR path in ``bcp_oracle.c``) plus numpy helpers for small cases.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg import this module, and only as the checker or the timed CPU baseline.
The product library never loads it.

Reference behaviour restated (paths relative to the reference repo):
  * ``xor_parity``               src/beegfs-raid5/common/task_processing.c:96-109
  * windowed P role / senders    task_processing.c:117-245 / :247-322
  * parity chunk file format     task_processing.c:168,186,199-201,213-214
  * rebuild index / truncation   task_processing.c:169-174,228-230
Pinning: ``oracle_xor_parity`` reproduces the reference's OWN xor_parity
(task_processing.c:96-109 compiled unchanged into oracle/_ref/libref_xor.so,
container only) on every fixture of tests/golden/ref_xor.json; the MPI-role
assembly (windows, padding, replay, file format) is pinned by SURVEY.md §8(c)
KAT-1..4 (tests/golden/kats.json).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libref_xor.so")  # reference's own xor_parity (container-built)
WINDOW = 10 * 1024 * 1024  # FILE_TRANSFER_BUFFER_SIZE, task_processing.c:20
KAT_MUL = 2654435761

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def build_ref() -> str | None:
    """Build oracle/_ref (only where /root/reference exists); path or None."""
    subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)
    return REF_LIB_PATH if os.path.exists(REF_LIB_PATH) else None


_ref = None


def ref_lib():
    """The reference's own xor_parity as ref_xor_parity(), or None when
    oracle/_ref was not built (no /root/reference where it was built)."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB_PATH):
        L = ctypes.CDLL(REF_LIB_PATH)
        L.ref_xor_parity.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        L.ref_xor_parity.restype = None
        _ref = L
    return _ref


def cpu_fold_hook():
    """(address, label) of the CPU fold the tools time inside libbcp's
    protocol (a bcp_xor_hook_fn): the reference's OWN xor_parity
    (task_processing.c:96-109 compiled unchanged, oracle/_ref ref_xor_rows)
    where it was built, else this restatement's oracle_xor_rows."""
    L = ref_lib()
    if L is not None and hasattr(L, "ref_xor_rows"):
        return ctypes.cast(L.ref_xor_rows, ctypes.c_void_p).value, "ref_xor_parity"
    return ctypes.cast(lib().oracle_xor_rows, ctypes.c_void_p).value, "oracle_xor_rows"


REF_PLAN_PATH = os.path.join(HERE, "_ref", "libref_plan.so")  # reference's own planner functions
_ref_plan = None


def ref_plan_lib():
    """The reference's own planner functions (gen/main.c simple_hash, PCG32,
    shuffle + qsort order, select_P, fill_in_missing_fields, get_store_weight;
    file_info_hash.c fih_add_info; assign_lanes.c) compiled unchanged into
    oracle/_ref/libref_plan.so by `make -C oracle ref`, or None where absent."""
    global _ref_plan
    if _ref_plan is None and os.path.exists(REF_PLAN_PATH):
        L = ctypes.CDLL(REF_PLAN_PATH)
        u64, i64, P = ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER
        sig = {
            "ref_simple_hash": ([ctypes.c_char_p, ctypes.c_int], ctypes.c_uint),
            "ref_sts_in_use": ([u64], ctypes.c_int),
            "ref_pcg32": ([u64, u64, ctypes.c_uint32, P(ctypes.c_uint32), ctypes.c_int], None),
            "ref_set_st_weight": ([P(ctypes.c_int), ctypes.c_int], None),
            "ref_select_P": ([ctypes.c_char_p, u64, ctypes.c_uint], u64),
            "ref_fill_in_missing_fields": ([u64, u64], u64),
            "ref_fih_add_info": ([P(i64), P(u64), P(u64), ctypes.c_int, i64, ctypes.c_int], None),
            "ref_sort_order": ([P(u64), ctypes.c_size_t, P(u64)], None),
            "ref_plan_item": ([ctypes.c_char_p, i64, u64, u64, ctypes.c_int, i64, u64, ctypes.c_uint], u64),
            "ref_store_weight": ([ctypes.c_int], ctypes.c_int),
            "assign_lanes": ([ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p, P(ctypes.c_int)], None),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes, fn.restype = args, res
        _ref_plan = L
    return _ref_plan


def ref_xor_parity(data: np.ndarray, nbytes: int, nsources: int) -> np.ndarray:
    """task_processing.c:96-109 itself (oracle/_ref); raises if not built."""
    L = ref_lib()
    if L is None:
        raise FileNotFoundError(REF_LIB_PATH)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert data.size >= nbytes * nsources
    dst = np.empty(max(nbytes, 1), dtype=np.uint8)
    L.ref_xor_parity(_ptr(dst), nbytes, _ptr(data), nsources)
    return dst[:nbytes]


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_xor_parity.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        L.oracle_xor_parity.restype = None
        L.oracle_gen_parity_file.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_uint64]
        L.oracle_gen_parity_file.restype = ctypes.c_int64
        L.oracle_rebuild_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                           ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.c_int, ctypes.c_int, ctypes.c_uint64]
        L.oracle_rebuild_chunk.restype = ctypes.c_int64
        L.oracle_rebuild_index.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.oracle_rebuild_index.restype = ctypes.c_int
        L.oracle_fill_kat1.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_fill_kat_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_fill_synthetic.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_bench_xor.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_double]
        L.oracle_bench_xor.restype = ctypes.c_double
        L.oracle_bench_xor_fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_uint64, ctypes.c_double]
        L.oracle_bench_xor_fn.restype = ctypes.c_double
        L.oracle_bench_xor_shapes_fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_int, ctypes.c_double]
        L.oracle_bench_xor_shapes_fn.restype = ctypes.c_double
        del u8p
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---- generators --------------------------------------------------------

def kat1_data(n: int, s: int) -> np.ndarray:
    """KAT-1 input: contiguous [n][s] with data[i] = (u8)((i*2654435761) >> 13)."""
    buf = np.empty(n * s, dtype=np.uint8)
    lib().oracle_fill_kat1(_ptr(buf), buf.size)
    return buf


def kat_chunk(k: int, length: int) -> np.ndarray:
    """KAT-2..4 chunk k: byte j = (u8)((((k<<32)+j)*2654435761 mod 2^64) >> 13)."""
    buf = np.empty(length, dtype=np.uint8)
    if length:
        lib().oracle_fill_kat_chunk(_ptr(buf), length, k)
    return buf


def kat_chunk_np(k: int, length: int) -> np.ndarray:
    """Pure-numpy form of kat_chunk (cross-checks the C generator)."""
    j = np.arange(length, dtype=np.uint64)
    with np.errstate(over="ignore"):
        v = ((np.uint64(k) << np.uint64(32)) + j) * np.uint64(KAT_MUL)
    return (v >> np.uint64(13)).astype(np.uint8)


def synthetic(length: int, seed: int, byte_offset: int = 0) -> np.ndarray:
    """splitmix64 byte stream, identical to libbcp's bcp_dev_fill_synthetic."""
    buf = np.empty(length, dtype=np.uint8)
    if length:
        lib().oracle_fill_synthetic(_ptr(buf), length, seed, byte_offset)
    return buf


# ---- the restated path -------------------------------------------------

def xor_parity(data: np.ndarray, nbytes: int, nsources: int) -> np.ndarray:
    """task_processing.c:96-109 on contiguous [nsources][nbytes] data."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert data.size >= nbytes * nsources
    dst = np.empty(max(nbytes, 1), dtype=np.uint8)
    lib().oracle_xor_parity(_ptr(dst), nbytes, _ptr(data), nsources)
    return dst[:nbytes]


def xor_padded_np(chunks) -> np.ndarray:
    """Plain zero-padded XOR (numpy); equals the reference when max len <= W."""
    m = max((len(c) for c in chunks), default=0)
    out = np.zeros(m, dtype=np.uint8)
    for c in chunks:
        out[: len(c)] ^= c
    return out


def _arrays(chunks):
    keep = [None if c is None else np.ascontiguousarray(c, dtype=np.uint8) for c in chunks]
    ptrs = (ctypes.c_void_p * len(keep))(*[None if c is None else (c.ctypes.data if c.size else _ptr(np.zeros(1, np.uint8))) for c in keep])
    lens = (ctypes.c_uint64 * len(keep))(*[0 if c is None else c.size for c in keep])
    return keep, ptrs, lens


def gen_parity_file(chunks, window: int = WINDOW) -> bytes:
    """Parity chunk file (header + windowed XOR) for chunks in ascending target order.
    A chunk given as None models an unreadable source (sends zeros, size 0)."""
    keep, ptrs, lens = _arrays(chunks)
    n = len(keep)
    cap = 8 * n + max([0] + [int(l) for l in lens])
    out = np.empty(max(cap, 1), dtype=np.uint8)
    r = lib().oracle_gen_parity_file(_ptr(out), cap, ptrs, lens, n, window)
    if r < 0:
        raise ValueError("oracle_gen_parity_file failed")
    return out[:r].tobytes()


def rebuild_chunk(parity_file: bytes, survivors, victim_index: int, window: int = WINDOW) -> bytes:
    """Rebuilt chunk of the victim from its surviving chunks + the parity file."""
    keep, ptrs, lens = _arrays(survivors)
    pf = np.frombuffer(parity_file, dtype=np.uint8).copy()
    n = len(keep) + 1
    sizes = np.frombuffer(parity_file[: 8 * n], dtype="<u8")
    cap = int(sizes[victim_index])
    out = np.empty(max(cap, 1), dtype=np.uint8)
    r = lib().oracle_rebuild_chunk(_ptr(out), cap, _ptr(pf), pf.size, ptrs, lens, len(keep), victim_index, window)
    if r < 0:
        raise ValueError("oracle_rebuild_chunk failed")
    return out[:r].tobytes()


def rebuild_index(locations: int, actual_p: int, victim: int) -> int:
    return lib().oracle_rebuild_index(locations, actual_p, victim)


def bench_xor(nthreads: int, nstripes: int, nsrc: int, chunk: int, seconds: float, use_ref: bool = False) -> float:
    """Algorithmic bytes/s ((nsrc+1)*chunk per stripe) of oracle_xor_parity, or
    of the reference's own xor_parity (oracle/_ref) when use_ref."""
    fn = None
    if use_ref:
        L = ref_lib()
        if L is None:
            raise FileNotFoundError(REF_LIB_PATH)
        fn = ctypes.cast(L.ref_xor_parity, ctypes.c_void_p).value
    r = lib().oracle_bench_xor_fn(fn, nthreads, nstripes, nsrc, chunk, seconds)
    if r < 0:
        raise MemoryError(f"oracle_bench_xor_fn: {r}")
    return r


def bench_xor_shapes(nthreads: int, lens, seconds: float, use_ref: bool = False) -> float:
    """Algorithmic bytes/s (sum of lengths + max per stripe) of the reference's
    fold over mixed chunk sizes as its P role runs it: each stripe one window
    of max_cs bytes per source, zero-padded rows (task_processing.c:209,
    302-303).  lens: [nstripes][nsrc] chunk lengths (each <= one window)."""
    arr = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    assert arr.ndim == 2 and arr.size
    fn = None
    if use_ref:
        L = ref_lib()
        if L is None:
            raise FileNotFoundError(REF_LIB_PATH)
        fn = ctypes.cast(L.ref_xor_parity, ctypes.c_void_p).value
    r = lib().oracle_bench_xor_shapes_fn(fn, nthreads, arr.ctypes.data, arr.shape[0], arr.shape[1], seconds)
    if r < 0:
        raise MemoryError(f"oracle_bench_xor_shapes_fn: {r}")
    return r
