"""ctypes binding of libbcp.so (include/bcp.h) for tests, the bench and
Python callers.  Thin: every call goes straight to the C ABI; there is no
Python or CPU compute path here.  A missing library or GPU raises.
"""
from __future__ import annotations

import ctypes
import errno
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BCP_LIB") or os.path.join(PKG_DIR, "lib", "libbcp.so")  # BCP_LIB: A/B of another build
HEADER_DIR = os.path.join(os.path.dirname(PKG_DIR), "include")

MAX_SOURCES = 56
WINDOW_BYTES = 10 * 1024 * 1024


class BcpError(RuntimeError):
    def __init__(self, fn: str, rc: int):
        super().__init__(f"{fn} failed: rc={rc} ({os.strerror(-rc) if rc < 0 else rc})")
        self.rc = rc


class Source(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_uint64), ("len", ctypes.c_uint64)]


class Stripe(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_uint64), ("out_len", ctypes.c_uint64), ("first_src", ctypes.c_uint32),
                ("nsrc", ctypes.c_uint32), ("window", ctypes.c_uint64)]


class FileInfo(ctypes.Structure):
    _fields_ = [("timestamp", ctypes.c_int64), ("locations", ctypes.c_uint64)]


class WorkItem(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("fi", FileInfo)]


class RunStats(ctypes.Structure):
    _fields_ = [("seconds", ctypes.c_double), ("tasks", ctypes.c_uint64), ("bytes_read", ctypes.c_uint64),
                ("bytes_written", ctypes.c_uint64), ("errors", ctypes.c_int), ("refused", ctypes.c_uint64)]


class PipelineTiming(ctypes.Structure):
    _fields_ = [("stat", ctypes.c_double), ("read_wait", ctypes.c_double), ("slot_wait", ctypes.c_double),
                ("submit", ctypes.c_double), ("drain", ctypes.c_double), ("batches", ctypes.c_uint32),
                ("read_jobs", ctypes.c_uint32), ("read_mode", ctypes.c_int),
                ("direct_bytes", ctypes.c_uint64), ("direct_fallbacks", ctypes.c_uint32)]


class PipelineOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("slab_bytes", ctypes.c_size_t), ("io_threads", ctypes.c_int),
                ("nslots", ctypes.c_int), ("ndevices", ctypes.c_int), ("read_mode", ctypes.c_int)]


READ_AUTO, READ_COPY, READ_DIRECT = 0, 1, 3  # 2 was MAP (removed in ABI 3)


XOR_HOOK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                            ctypes.c_int, ctypes.c_void_p)

L_MASK = (1 << 56) - 1
NO_P = 0xFF


def with_p(locations: int, p: int) -> int:
    """WITH_P (common.h:22)."""
    return (locations & L_MASK) | ((p & 0xFF) << 56)


def get_p(locations: int) -> int:
    return locations >> 56


_lib = None

_V = ctypes.c_void_p
_SIGS = {
    "bcp_abi_version": ([], ctypes.c_int),
    "bcp_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "bcp_strerror": ([ctypes.c_int], ctypes.c_char_p),
    "bcp_engine_create": ([ctypes.c_int, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_engine_destroy": ([_V], ctypes.c_int),
    "bcp_engine_info": ([_V, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "bcp_engine_pci_bus_id": ([_V, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "bcp_queue_create": ([_V, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_queue_destroy": ([_V], ctypes.c_int),
    "bcp_queue_sync": ([_V], ctypes.c_int),
    "bcp_queue_query": ([_V], ctypes.c_int),
    "bcp_event_create": ([_V, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_event_destroy": ([_V], ctypes.c_int),
    "bcp_event_record": ([_V, _V], ctypes.c_int),
    "bcp_queue_wait_event": ([_V, _V], ctypes.c_int),
    "bcp_event_sync": ([_V], ctypes.c_int),
    "bcp_event_query": ([_V], ctypes.c_int),
    "bcp_dev_alloc": ([_V, ctypes.c_size_t, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_dev_free": ([_V, _V], ctypes.c_int),
    "bcp_host_alloc": ([_V, ctypes.c_size_t, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_host_alloc_mapped": ([_V, ctypes.c_size_t, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_host_free": ([_V, _V], ctypes.c_int),
    "bcp_host_register": ([_V, _V, ctypes.c_size_t], ctypes.c_int),
    "bcp_host_unregister": ([_V, _V], ctypes.c_int),
    "bcp_h2d_async": ([_V, _V, _V, ctypes.c_size_t], ctypes.c_int),
    "bcp_d2h_async": ([_V, _V, _V, ctypes.c_size_t], ctypes.c_int),
    "bcp_d2d_async": ([_V, _V, _V, ctypes.c_size_t], ctypes.c_int),
    "bcp_h2d_2d_async": ([_V, _V, ctypes.c_size_t, _V, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t],
                         ctypes.c_int),
    "bcp_memset_async": ([_V, _V, ctypes.c_int, ctypes.c_size_t], ctypes.c_int),
    "bcp_xor_uniform_async": ([_V, _V, _V, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64], ctypes.c_int),
    "bcp_xor_strided_async": ([_V, _V, ctypes.c_uint64, _V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                               ctypes.c_uint32, ctypes.c_uint64], ctypes.c_int),
    "bcp_xor_stripes_async": ([_V, ctypes.POINTER(Stripe), ctypes.c_uint32, ctypes.POINTER(Source), ctypes.c_uint32],
                              ctypes.c_int),
    "bcp_xor_parity": ([_V, ctypes.c_size_t, _V, ctypes.c_int], ctypes.c_int),
    "bcp_ring_create": ([_V, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_ring_submit": ([_V, ctypes.POINTER(Stripe), ctypes.POINTER(Source), ctypes.POINTER(ctypes.c_uint64)],
                        ctypes.c_int),
    "bcp_ring_wait": ([_V, ctypes.c_uint64], ctypes.c_int),
    "bcp_ring_query": ([_V, ctypes.c_uint64], ctypes.c_int),
    "bcp_ring_destroy": ([_V], ctypes.c_int),
    "bcp_ring_set_wait": ([_V, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "bcp_task_set_ring_wait": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "bcp_task_set_fold_tuning": ([ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "bcp_ring_stats": ([_V, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_dev_fill_synthetic_async": ([_V, _V, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64], ctypes.c_int),
    "bcp_dev_xor_fold_async": ([_V, _V, ctypes.c_uint64, _V], ctypes.c_int),
    "bcp_dev_compare_async": ([_V, _V, _V, ctypes.c_uint64, _V], ctypes.c_int),
    "bcp_queue_mark": ([_V, ctypes.c_int], ctypes.c_int),
    "bcp_queue_elapsed_ms": ([_V, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
    "bcp_set_tuning": ([_V, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "bcp_set_option": ([_V, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "bcp_get_option": ([_V, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "bcp_task_set_device_map": ([ctypes.POINTER(ctypes.c_int), ctypes.c_int], ctypes.c_int),
    "bcp_task_shutdown": ([], ctypes.c_int),
    "bcp_task_set_xor_hook": ([_V, _V], None),
    "bcp_task_set_fold_mode": ([ctypes.c_int], ctypes.c_int),
    "bcp_task_set_explicit_padding": ([ctypes.c_int], ctypes.c_int),
    "bcp_task_watch_live": ([], ctypes.c_size_t),
    "bcp_task_pipe_stats": ([ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_task_set_fold_inflight": ([ctypes.c_int], ctypes.c_int),
    "bcp_task_fold_stats": ([ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_task_set_fold_ring": ([ctypes.c_int], ctypes.c_int),
    "bcp_gen_round_timing": ([ctypes.POINTER(ctypes.c_double), ctypes.c_int], ctypes.c_int),
    "bcp_task_ring_stats": ([ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_task_inject_failure": ([ctypes.c_int, ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "bcp_task_phase_stats": ([ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "bcp_task_set_transport": ([_V], ctypes.c_int),
    "bcp_task_set_rebuild_lanes": ([ctypes.c_int], ctypes.c_int),
    "bcp_fold_server_serve": ([ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
    "bcp_fold_server_connect": ([ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int], ctypes.c_int),
    "bcp_fold_server_stats": ([ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_lb_transport": ([], _V),
    "bcp_gen_run_procs": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int), _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rebuild_run_procs": ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t,
                               ctypes.c_char_p, _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rank_pool_create": ([ctypes.c_int, _V, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_rank_pool_gen": ([_V, ctypes.c_char_p, ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_int), ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rank_pool_rebuild": ([_V, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t,
                               ctypes.c_char_p, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rank_pool_destroy": ([_V], ctypes.c_int),
    "bcp_assign_lanes": ([ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(FileInfo), ctypes.POINTER(ctypes.c_int)], None),
    "bcp_gen_run": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.c_int,
                     ctypes.POINTER(ctypes.c_int), _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rebuild_run": ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t,
                         ctypes.c_char_p, _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_pipeline_gen": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t,
                          ctypes.POINTER(PipelineOpts), _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_pipeline_create": ([ctypes.POINTER(PipelineOpts), ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_pipeline_run": ([_V, ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t, _V,
                          ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_pipeline_destroy": ([_V], ctypes.c_int),
    "bcp_pipeline_last_timing": ([_V, ctypes.POINTER(PipelineTiming)], ctypes.c_int),
    "bcp_pipeline_rebuild": ([_V, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(WorkItem),
                              ctypes.c_size_t, ctypes.c_char_p, _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_lb_init": ([ctypes.c_int], ctypes.c_int),
    "bcp_eventset_create": ([ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_eventset_destroy": ([_V], None),
    "bcp_eventset_feed": ([_V, ctypes.c_int, _V, ctypes.c_size_t], ctypes.c_int),
    "bcp_eventset_feed_file": ([_V, ctypes.c_int, ctypes.c_char_p], ctypes.c_int),
    "bcp_eventset_count": ([_V], ctypes.c_size_t),
    "bcp_eventset_get": ([_V, ctypes.c_size_t, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int64),
                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                          ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_path_hash": ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_uint32),
    "bcp_store_weight": ([ctypes.c_int], ctypes.c_int),
    "bcp_plan_worklist": ([_V, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(WorkItem), ctypes.c_size_t,
                           ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "bcp_plan_rounds": ([_V, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(WorkItem), ctypes.c_size_t,
                         ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
                         ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "bcp_plan_rounds_ordered": ([_V, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.POINTER(WorkItem), ctypes.c_size_t,
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "bcp_map_targets": ([ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "bcp_store_round_order": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "bcp_assign_lanes_rounds": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(FileInfo),
                                 ctypes.POINTER(ctypes.c_int)], None),
    "bcp_lb_finalize": ([], ctypes.c_int),
    "bcp_pdb_open": ([ctypes.c_char_p, ctypes.c_uint64, ctypes.POINTER(_V)], ctypes.c_int),
    "bcp_pdb_close": ([_V], ctypes.c_int),
    "bcp_pdb_set": ([_V, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(FileInfo)], ctypes.c_int),
    "bcp_pdb_del": ([_V, ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "bcp_pdb_get": ([_V, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(FileInfo)], ctypes.c_int),
    "bcp_pdb_count": ([_V], ctypes.c_size_t),
    "bcp_pdb_sync": ([_V], ctypes.c_int),
    "bcp_pdb_items": ([_V, ctypes.POINTER(ctypes.POINTER(WorkItem)), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "bcp_pdb_items_free": ([ctypes.POINTER(WorkItem)], None),
    "bcp_gen_run_db": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(WorkItem), ctypes.c_size_t, ctypes.c_int,
                        ctypes.POINTER(ctypes.c_int), _V, ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_rebuild_run_db": ([ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, _V,
                            ctypes.POINTER(RunStats)], ctypes.c_int),
    "bcp_store_cum_weights": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    "bcp_scan_chunks": ([ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_eventset_scan": ([_V, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
    "bcp_check_targets": ([ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, _V], ctypes.c_int),
    "bcp_gen_round_pipeline": ([_V, ctypes.c_char_p, ctypes.c_int, _V, ctypes.POINTER(ctypes.c_int), _V,
                                ctypes.POINTER(RunStats), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
    "bcp_gen_round": ([ctypes.c_char_p, ctypes.c_int, _V, ctypes.POINTER(ctypes.c_int), ctypes.c_int, _V,
                       ctypes.POINTER(RunStats), ctypes.POINTER(ctypes.c_size_t)], ctypes.c_int),
}


def build() -> str:
    subprocess.run(["make", "-s", "-j8", "-C", PKG_DIR], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    """Load libbcp.so (raises if it is missing: there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"libbcp.so not built: {LIB_PATH} (run make -C {PKG_DIR})")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(fn: str, rc: int) -> int:
    if rc != 0:
        raise BcpError(fn, rc)
    return rc


def call(fn: str, *args) -> int:
    return check(fn, getattr(lib(), fn)(*args))


def device_count() -> int:
    n = ctypes.c_int(0)
    call("bcp_device_count", ctypes.byref(n))
    return n.value


class Engine:
    """One engine per device (bcp_engine_create)."""

    def __init__(self, device: int = 0):
        h = _V()
        call("bcp_engine_create", device, ctypes.byref(h))
        self.h = h
        self.device = device
        self._allocs: list[int] = []

    def info(self):
        cus = ctypes.c_int(0)
        name = ctypes.create_string_buffer(256)
        call("bcp_engine_info", self.h, ctypes.byref(cus), name, 256)
        return cus.value, name.value.decode()

    def pci_bus_id(self) -> str:
        """PCI bus id of the device (distinct per physical GPU)."""
        buf = ctypes.create_string_buffer(64)
        call("bcp_engine_pci_bus_id", self.h, buf, 64)
        return buf.value.decode()

    def tune(self, blocks_per_cu: int = 0, vecs_per_thread: int = 0):
        call("bcp_set_tuning", self.h, blocks_per_cu, vecs_per_thread)

    def option(self, key: str, value: int | None = None) -> int:
        """Set a named knob (value given) or read it back."""
        if value is not None:
            call("bcp_set_option", self.h, key.encode(), value)
        v = ctypes.c_int(0)
        call("bcp_get_option", self.h, key.encode(), ctypes.byref(v))
        return v.value

    def queue(self) -> "Queue":
        return Queue(self)

    def event(self) -> "Event":
        return Event(self)

    def alloc(self, nbytes: int) -> int:
        p = _V()
        call("bcp_dev_alloc", self.h, nbytes, ctypes.byref(p))
        return p.value

    def free(self, ptr: int):
        call("bcp_dev_free", self.h, _V(ptr))

    def host_alloc(self, nbytes: int, mapped: bool = False) -> int:
        """Pinned host memory; mapped=True: coherent, read/written by kernels in place."""
        p = _V()
        call("bcp_host_alloc_mapped" if mapped else "bcp_host_alloc", self.h, nbytes, ctypes.byref(p))
        return p.value

    def host_free(self, ptr: int):
        call("bcp_host_free", self.h, _V(ptr))

    def host_register(self, ptr: int, nbytes: int):
        """Caller-owned host memory the kernels then read and write in place."""
        call("bcp_host_register", self.h, _V(ptr), nbytes)

    def host_unregister(self, ptr: int):
        call("bcp_host_unregister", self.h, _V(ptr))

    def close(self):
        if self.h:
            call("bcp_engine_destroy", self.h)
            self.h = None


class Event:
    def __init__(self, eng: Engine):
        h = _V()
        call("bcp_event_create", eng.h, ctypes.byref(h))
        self.h = h

    def record(self, q: "Queue"):
        call("bcp_event_record", self.h, q.h)

    def sync(self):
        call("bcp_event_sync", self.h)

    def close(self):
        if self.h:
            call("bcp_event_destroy", self.h)
            self.h = None


class Queue:
    """One in-order HIP stream (bcp_queue_create)."""

    def __init__(self, eng: Engine):
        h = _V()
        call("bcp_queue_create", eng.h, ctypes.byref(h))
        self.h = h
        self.eng = eng

    def sync(self):
        call("bcp_queue_sync", self.h)

    def wait(self, ev: Event):
        call("bcp_queue_wait_event", self.h, ev.h)

    def h2d(self, dptr: int, host, nbytes: int | None = None):
        """host: numpy array / bytes / int address."""
        addr, n = _host_addr(host, nbytes)
        call("bcp_h2d_async", self.h, _V(dptr), _V(addr), n)

    def d2h(self, host, dptr: int, nbytes: int | None = None):
        addr, n = _host_addr(host, nbytes, writable=True)
        call("bcp_d2h_async", self.h, _V(addr), _V(dptr), n)

    def d2d(self, dst: int, src: int, nbytes: int):
        call("bcp_d2d_async", self.h, _V(dst), _V(src), nbytes)

    def memset(self, dptr: int, value: int, nbytes: int):
        call("bcp_memset_async", self.h, _V(dptr), value, nbytes)

    def xor_uniform(self, dst: int, src: int, nstripes: int, nsrc: int, chunk: int):
        call("bcp_xor_uniform_async", self.h, _V(dst), _V(src), nstripes, nsrc, chunk)

    def xor_strided(self, dst: int, dst_stride: int, src: int, stripe_stride: int, src_stride: int,
                    nstripes: int, nsrc: int, chunk: int):
        call("bcp_xor_strided_async", self.h, _V(dst), dst_stride, _V(src), stripe_stride, src_stride,
             nstripes, nsrc, chunk)

    def xor_stripes(self, stripes, sources):
        """stripes: list of (dst, out_len, first_src, nsrc, window); sources: list of (ptr, len)."""
        st = (Stripe * max(len(stripes), 1))(*[Stripe(*s) for s in stripes])
        so = (Source * max(len(sources), 1))(*[Source(*s) for s in sources])
        call("bcp_xor_stripes_async", self.h, st, len(stripes), so, len(sources))

    def fill_synthetic(self, dptr: int, nbytes: int, seed: int, byte_offset: int = 0):
        call("bcp_dev_fill_synthetic_async", self.h, _V(dptr), nbytes, seed, byte_offset)

    def xor_fold(self, src: int, nbytes: int, out16: int):
        call("bcp_dev_xor_fold_async", self.h, _V(src), nbytes, _V(out16))

    def compare(self, a: int, b: int, nbytes: int, out8: int):
        call("bcp_dev_compare_async", self.h, _V(a), _V(b), nbytes, _V(out8))

    def mark(self, slot: int):
        call("bcp_queue_mark", self.h, slot)

    def elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float(0)
        call("bcp_queue_elapsed_ms", self.h, a, b, ctypes.byref(ms))
        return ms.value

    def close(self):
        if self.h:
            call("bcp_queue_destroy", self.h)
            self.h = None


class Ring:
    """Resident fold ring (bcp_ring_create): one launch that folds stripes
    published from any thread, no launch or sync per stripe."""

    def __init__(self, eng: Engine, workers: int = 0, idle_us: int = 0):
        h = _V()
        call("bcp_ring_create", eng.h, workers, idle_us, ctypes.byref(h))
        self.h = h
        self.eng = eng

    def submit(self, dst: int, out_len: int, sources) -> int:
        """sources: list of (ptr, len); returns the handle."""
        st = Stripe(dst, out_len, 0, len(sources), 0)
        so = (Source * max(len(sources), 1))(*[Source(*s) for s in sources])
        hnd = ctypes.c_uint64(0)
        call("bcp_ring_submit", self.h, ctypes.byref(st), so, ctypes.byref(hnd))
        return hnd.value

    def wait(self, handle: int):
        call("bcp_ring_wait", self.h, handle)

    def query(self, handle: int) -> bool:
        rc = lib().bcp_ring_query(self.h, handle)
        if rc == -11:  # -EAGAIN
            return False
        check("bcp_ring_query", rc)
        return True

    def stats(self) -> tuple[int, int]:
        p, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        call("bcp_ring_stats", self.h, ctypes.byref(p), ctypes.byref(n))
        return p.value, n.value

    def close(self):
        if self.h:
            call("bcp_ring_destroy", self.h)
            self.h = None


def _host_addr(host, nbytes, writable: bool = False):
    """(address, nbytes) of a host buffer: numpy array, bytes / bytearray, or an
    int address (then nbytes is required and trusted).  nbytes may not exceed
    the buffer; a copy destination (writable) must be a writable buffer."""
    import numpy as np
    if isinstance(host, int):
        if nbytes is None:
            raise ValueError("an int host address needs an explicit nbytes")
        return host, nbytes
    if isinstance(host, (bytes, bytearray, memoryview)):
        if writable and (isinstance(host, bytes) or (isinstance(host, memoryview) and host.readonly)):
            raise ValueError("read-only host buffer as a copy destination")
        arr = np.frombuffer(host, dtype=np.uint8)
    elif isinstance(host, np.ndarray):
        if writable and not host.flags.writeable:
            raise ValueError("read-only numpy array as a copy destination")
        if not host.flags.c_contiguous:
            raise ValueError("host buffer must be C-contiguous")
        arr = host
    else:
        raise TypeError(f"unsupported host buffer {type(host).__name__}")
    size = arr.nbytes
    if nbytes is None:
        nbytes = size
    if nbytes < 0 or nbytes > size:
        raise ValueError(f"nbytes {nbytes} outside the {size}-byte host buffer")
    return arr.ctypes.data, nbytes


def xor_parity(dst, nbytes: int, data, nsources: int):
    """Drop-in for task_processing.c:96-109 on numpy buffers (GPU)."""
    d, _ = _host_addr(dst, nbytes, writable=True)
    s, _ = _host_addr(data, nbytes * max(nsources, 0))
    call("bcp_xor_parity", _V(d), nbytes, _V(s), nsources)


# ---------------------------------------------------------------------------
# host layer: loopback gen / rebuild drivers (include/bcp_task.h)
# ---------------------------------------------------------------------------
def _items(items):
    """items: list of (path, timestamp, locations)."""
    arr = (WorkItem * max(len(items), 1))()
    keep = []
    for i, (path, ts, loc) in enumerate(items):
        b = path.encode() if isinstance(path, str) else path
        keep.append(b)
        arr[i].path = b
        arr[i].fi.timestamp = ts
        arr[i].fi.locations = loc
    return arr, keep


def assign_lanes_rounds(nlanes: int, round_start, locations) -> list:
    """bcp_assign_lanes_rounds: assign_lanes over each round separately."""
    n = len(locations)
    fis = (FileInfo * max(n, 1))(*[FileInfo(0, x) for x in locations])
    out = (ctypes.c_int * max(n, 1))()
    rs = (ctypes.c_size_t * len(round_start))(*round_start)
    lib().bcp_assign_lanes_rounds(nlanes, len(round_start) - 1, rs, fis, out)
    return list(out)[:n]


def assign_lanes(nlanes: int, locations) -> list:
    n = len(locations)
    fis = (FileInfo * max(n, 1))(*[FileInfo(0, loc) for loc in locations])
    out = (ctypes.c_int * max(n, 1))()
    lib().bcp_assign_lanes(nlanes, n, fis, out)
    return list(out)[:n]


def gen_run(store_root: str, ntargets: int, items, nlanes: int = 12, lanes=None, log=None) -> RunStats:
    """Parity generation over loopback ranks (bcp_gen_run).  log: a C FILE* or None."""
    arr, keep = _items(items)
    st = RunStats()
    ln = None
    if lanes is not None:
        ln = (ctypes.c_int * max(len(lanes), 1))(*lanes)
    rc = lib().bcp_gen_run(store_root.encode(), ntargets, arr, len(items), nlanes, ln, log, ctypes.byref(st))
    check("bcp_gen_run", rc)
    del keep
    return st


def rebuild_run(store_root: str, ntargets: int, rebuild_target: int, items, corrupt_list: str | None = None,
                log=None) -> RunStats:
    arr, keep = _items(items)
    st = RunStats()
    rc = lib().bcp_rebuild_run(store_root.encode(), ntargets, rebuild_target, arr, len(items),
                               corrupt_list.encode() if corrupt_list else None, log, ctypes.byref(st))
    check("bcp_rebuild_run", rc)
    del keep
    return st


def gen_run_procs(store_root: str, ntargets: int, items, nlanes: int = 12, lanes=None, log=None) -> RunStats:
    """bcp_gen_run with every target's rank as its own forked process
    (socketpair transport).  Only from a process that has not used the GPU."""
    arr, keep = _items(items)
    st = RunStats()
    ln = None
    if lanes is not None:
        ln = (ctypes.c_int * max(len(lanes), 1))(*lanes)
    rc = lib().bcp_gen_run_procs(store_root.encode(), ntargets, arr, len(items), nlanes, ln, log, ctypes.byref(st))
    check("bcp_gen_run_procs", rc)
    del keep
    return st


def rebuild_run_procs(store_root: str, ntargets: int, rebuild_target: int, items, corrupt_list: str | None = None,
                      log=None) -> RunStats:
    arr, keep = _items(items)
    st = RunStats()
    rc = lib().bcp_rebuild_run_procs(store_root.encode(), ntargets, rebuild_target, arr, len(items),
                                     corrupt_list.encode() if corrupt_list else None, log, ctypes.byref(st))
    check("bcp_rebuild_run_procs", rc)
    del keep
    return st


class RankPool:
    """Rank processes kept alive across runs (bcp_rank_pool_*): one forked
    process per storage target; each run takes this process's P-role settings
    at call time.  Create it before this process touches the GPU."""

    def __init__(self, ntargets: int, log=None):
        h = _V()
        check("bcp_rank_pool_create", lib().bcp_rank_pool_create(ntargets, log, ctypes.byref(h)))
        self.h = h
        self.ntargets = ntargets

    def gen(self, store_root: str, items, nlanes: int = 12, lanes=None) -> RunStats:
        arr, keep = _items(items)
        st = RunStats()
        ln = (ctypes.c_int * max(len(lanes), 1))(*lanes) if lanes is not None else None
        rc = lib().bcp_rank_pool_gen(self.h, store_root.encode(), arr, len(items), nlanes, ln, ctypes.byref(st))
        check("bcp_rank_pool_gen", rc)
        del keep
        return st

    def rebuild(self, store_root: str, rebuild_target: int, items, corrupt_list: str | None = None) -> RunStats:
        arr, keep = _items(items)
        st = RunStats()
        rc = lib().bcp_rank_pool_rebuild(self.h, store_root.encode(), rebuild_target, arr, len(items),
                                         corrupt_list.encode() if corrupt_list else None, ctypes.byref(st))
        check("bcp_rank_pool_rebuild", rc)
        del keep
        return st

    def close(self):
        if self.h:
            h, self.h = self.h, None
            check("bcp_rank_pool_destroy", lib().bcp_rank_pool_destroy(h))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def gen_run_db(store_root: str, ntargets: int, items, nlanes: int = 12, lanes=None, log=None) -> RunStats:
    """bcp_gen_run + per-target DB replicas <root>/st<k>/db (gen/main.c:146-149)."""
    arr, keep = _items(items)
    st = RunStats()
    ln = (ctypes.c_int * max(len(lanes), 1))(*lanes) if lanes is not None else None
    call("bcp_gen_run_db", store_root.encode(), ntargets, arr, len(items), nlanes, ln, log, ctypes.byref(st))
    del keep
    return st


def rebuild_run_db(store_root: str, ntargets: int, rebuild_target: int, db_folder: str | None = None,
                   corrupt_list: str | None = None, log=None) -> RunStats:
    """Rebuild walking a DB in key order (rebuild/main.c:223-225)."""
    st = RunStats()
    call("bcp_rebuild_run_db", store_root.encode(), ntargets, rebuild_target,
         db_folder.encode() if db_folder else None, corrupt_list.encode() if corrupt_list else None, log,
         ctypes.byref(st))
    return st


def store_cum_weights(store_root: str, ntargets: int) -> list:
    out = (ctypes.c_int * ntargets)()
    call("bcp_store_cum_weights", store_root.encode(), ntargets, out)
    return list(out)


def gen_round(store_root: str, ntargets: int, events: "EventSet", cum_weight=None, nlanes: int = 12, log=None):
    """One phase-2 round: plan from events + DB, run, update the DB.  Returns (RunStats, nplanned)."""
    st = RunStats()
    n = ctypes.c_size_t(0)
    cw = (ctypes.c_int * ntargets)(*cum_weight) if cum_weight is not None else None
    call("bcp_gen_round", store_root.encode(), ntargets, events.h, cw, nlanes, log, ctypes.byref(st), ctypes.byref(n))
    return st, n.value


DB_VERSION = 1  # common.h:31


class PDB:
    """Persistent chunk state (bcp_pdb_*, persistent_db.{c,h})."""

    def __init__(self, folder: str, version: int = DB_VERSION):
        h = _V()
        call("bcp_pdb_open", folder.encode(), version, ctypes.byref(h))
        self.h = h

    @staticmethod
    def _k(key):
        return key.encode() if isinstance(key, str) else bytes(key)

    def set(self, key, timestamp: int, locations: int):
        k = self._k(key)
        fi = FileInfo(timestamp, locations)
        call("bcp_pdb_set", self.h, k, len(k), ctypes.byref(fi))

    def delete(self, key):
        k = self._k(key)
        call("bcp_pdb_del", self.h, k, len(k))

    def get(self, key):
        k = self._k(key)
        fi = FileInfo()
        rc = lib().bcp_pdb_get(self.h, k, len(k), ctypes.byref(fi))
        if rc < 0:
            raise BcpError("bcp_pdb_get", rc)
        return (fi.timestamp, fi.locations) if rc == 1 else None

    def __len__(self):
        return lib().bcp_pdb_count(self.h)

    def items(self):
        """[(key bytes, timestamp, locations)] in key order."""
        p = ctypes.POINTER(WorkItem)()
        n = ctypes.c_size_t(0)
        call("bcp_pdb_items", self.h, ctypes.byref(p), ctypes.byref(n))
        out = [(p[i].path, p[i].fi.timestamp, p[i].fi.locations) for i in range(n.value)]
        lib().bcp_pdb_items_free(p)
        return out

    def sync(self):
        call("bcp_pdb_sync", self.h)

    def close(self):
        if self.h:
            call("bcp_pdb_close", self.h)
            self.h = None


def pipeline_gen(store_root: str, ntargets: int, items, device: int = 0, slab_bytes: int = 256 << 20,
                 io_threads: int = 0, nslots: int = 4, log=None, ndevices: int = 1, read_mode: int = 0) -> RunStats:
    """Batched end-to-end parity generation (bcp_pipeline_gen)."""
    arr, keep = _items(items)
    st = RunStats()
    opts = PipelineOpts(device, slab_bytes, io_threads, nslots, ndevices, read_mode)
    rc = lib().bcp_pipeline_gen(store_root.encode(), ntargets, arr, len(items), ctypes.byref(opts), log,
                                ctypes.byref(st))
    check("bcp_pipeline_gen", rc)
    del keep
    return st


class Pipeline:
    """Long-lived batched pipeline (bcp_pipeline_create / run / destroy)."""

    def __init__(self, device: int = 0, slab_bytes: int = 256 << 20, io_threads: int = 0, nslots: int = 4,
                 ndevices: int = 1, read_mode: int = 0):
        h = _V()
        opts = PipelineOpts(device, slab_bytes, io_threads, nslots, ndevices, read_mode)
        call("bcp_pipeline_create", ctypes.byref(opts), ctypes.byref(h))
        self.h = h

    def run(self, store_root: str, ntargets: int, items, log=None) -> RunStats:
        arr, keep = _items(items)
        st = RunStats()
        call("bcp_pipeline_run", self.h, store_root.encode(), ntargets, arr, len(items), log, ctypes.byref(st))
        del keep
        return st

    def rebuild(self, store_root: str, ntargets: int, rebuild_target: int, items, corrupt_list: str | None = None,
                log=None) -> RunStats:
        """bcp_pipeline_rebuild: items in DB key order, as bcp_rebuild_run takes them."""
        arr, keep = _items(items)
        st = RunStats()
        call("bcp_pipeline_rebuild", self.h, store_root.encode(), ntargets, rebuild_target, arr, len(items),
             corrupt_list.encode() if corrupt_list else None, log, ctypes.byref(st))
        del keep
        return st

    def round(self, store_root: str, ntargets: int, events: "EventSet", cum_weight=None, log=None):
        """bcp_gen_round_pipeline: plan from events + DB, run batched, update the DB."""
        st = RunStats()
        n = ctypes.c_size_t(0)
        cw = (ctypes.c_int * ntargets)(*cum_weight) if cum_weight is not None else None
        call("bcp_gen_round_pipeline", self.h, store_root.encode(), ntargets, events.h, cw, log, ctypes.byref(st),
             ctypes.byref(n))
        return st, n.value

    def last_timing(self) -> dict:
        """bcp_pipeline_last_timing: the host thread's wall time of the last run by stage."""
        t = PipelineTiming()
        call("bcp_pipeline_last_timing", self.h, ctypes.byref(t))
        return {f: round(getattr(t, f), 5) if isinstance(getattr(t, f), float) else getattr(t, f)
                for f, _ in PipelineTiming._fields_}

    def close(self):
        if self.h:
            call("bcp_pipeline_destroy", self.h)
            self.h = None


def set_xor_hook(fn_addr: int | None, ctx: int | None = None):
    """Test injection point: route the P role's fold to a C function (address)."""
    lib().bcp_task_set_xor_hook(_V(fn_addr) if fn_addr else None, _V(ctx) if ctx else None)


FOLD_BATCHED, FOLD_PIPELINED = 2, 5
PAD_AUTO = -1
INJECT_FOLD_RES, INJECT_DRAIN_ROW, INJECT_SEND_BUF, INJECT_THREAD, INJECT_READ = 1, 2, 4, 8, 16
INJECT_FOLD_SERVER, INJECT_DIRECT_READ, INJECT_PARITY_WRITE = 32, 64, 128


def set_fold_mode(mode: int) -> int:
    """P-role fold: FOLD_PIPELINED (default) or FOLD_BATCHED; returns the previous mode."""
    rc = lib().bcp_task_set_fold_mode(mode)
    if rc < 0:
        raise BcpError("bcp_task_set_fold_mode", rc)
    return rc


def set_rebuild_lanes(n: int) -> int:
    """Lanes per rank of the rebuild runners (1 = the reference's); returns the previous value."""
    rc = lib().bcp_task_set_rebuild_lanes(n)
    if rc < 0:
        raise BcpError("bcp_task_set_rebuild_lanes", rc)
    return rc


def fold_server_serve(socket_path: str, max_conns: int = 0) -> None:
    """Run a node fold server on a Unix socket (blocks; 0 = forever)."""
    call("bcp_fold_server_serve", socket_path.encode(), max_conns)


def fold_server_connect(socket_path: str, arena_bytes: int = 1 << 30, nconn: int = 12) -> None:
    """This process's P roles fold through the node fold server at socket_path."""
    call("bcp_fold_server_connect", socket_path.encode(), arena_bytes, nconn)


def fold_server_stats() -> int:
    """Windows the node fold server folded for this process."""
    w = ctypes.c_uint64(0)
    call("bcp_fold_server_stats", ctypes.byref(w))
    return w.value


def pipe_stats() -> tuple:
    """(windows folded by following their rows, range folds launched) -- FOLD_PIPELINED."""
    w, r = ctypes.c_uint64(0), ctypes.c_uint64(0)
    lib().bcp_task_pipe_stats(ctypes.byref(w), ctypes.byref(r))
    return w.value, r.value


def set_explicit_padding(on) -> int:
    """The wire of a one-window gen task: True / 1 the reference's (every
    window zero-padded), False / 0 implicit padding (a chunk's bytes only),
    PAD_AUTO (default) implicit through libbcp's own transports and the
    reference's through a caller's table; returns the previous setting
    (PAD_AUTO, 0 or 1)."""
    v = PAD_AUTO if on == PAD_AUTO else int(bool(on))
    rc = lib().bcp_task_set_explicit_padding(v)
    if rc < PAD_AUTO:
        raise BcpError("bcp_task_set_explicit_padding", rc)
    return rc


def task_shutdown():
    call("bcp_task_shutdown")


def set_fold_inflight(k: int) -> int:
    """Concurrent batches of the batched fold service; returns the previous value."""
    rc = lib().bcp_task_set_fold_inflight(k)
    if rc < 0:
        raise BcpError("bcp_task_set_fold_inflight", rc)
    return rc


def set_fold_tuning(key: str, value: int) -> int:
    """The P role's fold shape for tools / A/B runs (bcp_task_set_fold_tuning); returns the previous value."""
    prev = lib().bcp_task_set_fold_tuning(key.encode(), value)
    check("bcp_task_set_fold_tuning", min(prev, 0))
    return prev


def round_timing() -> dict:
    """Stage times of this process's latest changelog round (bcp_gen_round_timing)."""
    t = (ctypes.c_double * 4)()
    n = lib().bcp_gen_round_timing(t, 4)
    check("bcp_gen_round_timing", min(n, 0))
    return {"db_read_s": round(t[0], 5), "plan_s": round(t[1], 5), "run_s": round(t[2], 5), "replicas_s": round(t[3], 5)}


def set_fold_ring(on: bool) -> bool:
    """PIPELINED folds through the device's resident fold ring (default on);
    returns the previous setting."""
    prev = lib().bcp_task_set_fold_ring(1 if on else 0)
    check("bcp_task_set_fold_ring", min(prev, 0))
    return bool(prev)


def ring_stats() -> tuple[int, int]:
    """(pieces published to the fold rings, launches of them) since start."""
    p, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
    call("bcp_task_ring_stats", ctypes.byref(p), ctypes.byref(n))
    return p.value, n.value


def fold_stats() -> tuple[int, int]:
    """(windows folded, launches) of the batched fold service."""
    w, l = ctypes.c_uint64(0), ctypes.c_uint64(0)
    call("bcp_task_fold_stats", ctypes.byref(w), ctypes.byref(l))
    return w.value, l.value


PHASES = ("p_sizes", "p_open", "p_rows", "p_fold", "p_write", "p_close", "s_sizes", "s_send", "p_tasks", "s_tasks")


def phase_stats(reset: bool = False) -> dict:
    """Per-phase protocol wall time summed over tasks (bcp_task_phase_stats);
    p_tasks / s_tasks are counts."""
    buf = (ctypes.c_double * len(PHASES))()
    rc = lib().bcp_task_phase_stats(buf, len(PHASES), 1 if reset else 0)
    if rc < 0:
        raise BcpError("bcp_task_phase_stats", rc)
    out = {k: buf[i] for i, k in enumerate(PHASES)}
    out["p_tasks"] = int(out["p_tasks"])
    out["s_tasks"] = int(out["s_tasks"])
    return out


def inject_failure(site: int, after: int = 0, count: int = 1):
    """Test hook: the next `count` passes through `site` fail after `after` succeed (0 clears)."""
    call("bcp_task_inject_failure", site, after, count)


def set_transport(ops_addr: int | None):
    """Install a bcp_transport_ops table by address (None: the loopback default)."""
    call("bcp_task_set_transport", ops_addr)


# ---------------------------------------------------------------------------
# chunk-event records and worklist planning
# ---------------------------------------------------------------------------
def pack_records(records) -> bytes:
    """records: (timestamp, size, event 'm'|'d', path) -> the binary stream
    of bp-find-all-chunks/main.c:25-33."""
    import struct
    out = bytearray()
    for ts, size, ev, path in records:
        b = path.encode() if isinstance(path, str) else path
        out += struct.pack("<qQQQ", ts, size, ord(ev), len(b)) + b
    return bytes(out)


class EventSet:
    def __init__(self):
        h = _V()
        call("bcp_eventset_create", ctypes.byref(h))
        self.h = h

    def feed(self, st: int, data: bytes):
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        call("bcp_eventset_feed", self.h, st, buf, len(data))

    def feed_file(self, st: int, path: str):
        call("bcp_eventset_feed_file", self.h, st, path.encode())

    def scan(self, st: int, chunks_dir: str) -> int:
        """Feed a bp-find-all-chunks walk of chunks_dir as target st's stream."""
        n = ctypes.c_uint64(0)
        call("bcp_eventset_scan", self.h, st, chunks_dir.encode(), ctypes.byref(n))
        return n.value

    def __len__(self):
        return lib().bcp_eventset_count(self.h)

    def entries(self):
        out = []
        for i in range(len(self)):
            p, ts, m, d, sz = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
            call("bcp_eventset_get", self.h, i, ctypes.byref(p), ctypes.byref(ts), ctypes.byref(m), ctypes.byref(d),
                 ctypes.byref(sz))
            out.append((p.value.decode(), ts.value, m.value, d.value, sz.value))
        return out

    def plan(self, ntargets: int, cum_weight, prev=()):
        """prev: iterable of (path, timestamp, locations); returns [(path, timestamp, locations)]."""
        return self.plan_rounds(ntargets, cum_weight, prev)[0]

    def plan_rounds(self, ntargets: int, cum_weight, prev=(), round_st=None):
        """bcp_plan_rounds: (worklist, round_start) -- the coordinators' rounds
        back to back, round k = worklist[round_start[k]:round_start[k+1]];
        round_st (bcp_plan_rounds_ordered): the target whose eater broadcasts
        round r, in MPI rank order (None = target order)."""
        prev = sorted(prev, key=lambda x: x[0].encode())
        parr, keep = _items(prev)
        cw = (ctypes.c_int * ntargets)(*cum_weight)
        n = ctypes.c_size_t(0)
        call("bcp_plan_worklist", self.h, ntargets, cw, parr, len(prev), None, 0, ctypes.byref(n))
        out = (WorkItem * max(n.value, 1))()
        rs = (ctypes.c_size_t * (ntargets + 1))()
        if round_st is None:
            call("bcp_plan_rounds", self.h, ntargets, cw, parr, len(prev), out, n.value, ctypes.byref(n), rs)
        else:
            call("bcp_plan_rounds_ordered", self.h, ntargets, cw, (ctypes.c_int * ntargets)(*round_st), parr,
                 len(prev), out, n.value, ctypes.byref(n), rs)
        del keep
        return ([(out[i].path.decode(), out[i].fi.timestamp, out[i].fi.locations) for i in range(n.value)],
                list(rs))

    def close(self):
        if self.h:
            lib().bcp_eventset_destroy(self.h)
            self.h = None


BIN_PATH = os.path.join(PKG_DIR, "bin", "bcp")


def check_targets(store_root: str, ntargets: int, run_data: str):
    call("bcp_check_targets", store_root.encode(), ntargets, run_data.encode(), None)


def map_targets(prev_ids, rank_ids):
    """bcp_map_targets (gen/main.c:498-499, 506-541): (st_ids, round_st), or
    BcpError (-EEXIST duplicate, -ENODEV fewer / missing)."""
    n = len(rank_ids)
    st = (ctypes.c_int32 * max(n, 1))()
    rs = (ctypes.c_int * max(n, 1))()
    call("bcp_map_targets", (ctypes.c_int32 * max(len(prev_ids), 1))(*prev_ids), len(prev_ids),
         (ctypes.c_int32 * max(n, 1))(*rank_ids), n, st, rs)
    return list(st)[:n], list(rs)[:n]


def store_round_order(store_root: str, ntargets: int) -> list:
    """bcp_store_round_order: the target of every round from <root>/rank_order."""
    rs = (ctypes.c_int * ntargets)()
    call("bcp_store_round_order", store_root.encode(), ntargets, rs)
    return list(rs)


def path_hash(path: str) -> int:
    b = path.encode()
    return lib().bcp_path_hash(b, len(b))
