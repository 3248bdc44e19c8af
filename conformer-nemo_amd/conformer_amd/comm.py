"""ctypes binding of include/cfm_comm.h: RCCL data parallelism through the C-ABI, without
torch.distributed (a non-Python host makes the same calls).

* `NativeComm` — cfm_comm_init over a unique id shared by the caller (rank 0 creates it with
  `NativeComm.unique_id()`); `allreduce(t, scale)`; `allreduce_cb` is the SyncBatchNorm callback.
* `NativeGradBuckets` — conformer_amd.dist.GradBuckets with the reductions done by the library:
  the native backward calls cfm_grad_buckets_ready_cb itself (no Python in the loop), which
  all-reduces each layer's gradients on the bucket's own stream while the backward continues;
  finish() runs cfm_grad_buckets_finish (remainder, wait, 1/world) on torch's current stream.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import torch

from . import _lib
from .dist import GradBuckets


def _bind(lib) -> None:
    if getattr(lib, "_cfm_comm_bound", False):
        return
    vp, ci, i64, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    for name, res, args in (
            ("cfm_comm_get_unique_id", ci, [ctypes.c_char_p]),
            ("cfm_comm_init", ci, [ci, ci, ctypes.c_char_p, ci, ctypes.POINTER(vp)]),
            ("cfm_comm_destroy", ci, [vp]),
            ("cfm_comm_world", ci, [vp]),
            ("cfm_allreduce_grads", ci, [vp, vp, i64, cf, vp]),
            ("cfm_grad_buckets_create", ci, [vp, vp, i64, ci, ctypes.POINTER(i64), ctypes.POINTER(i64), ci,
                                             ctypes.POINTER(vp)]),
            ("cfm_grad_buckets_finish", ci, [vp, vp]),
            ("cfm_grad_buckets_issued", ci, [vp]),
            ("cfm_grad_buckets_destroy", ci, [vp])):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._cfm_comm_bound = True


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class NativeComm:
    def __init__(self, rank: int, world: int, unique_id: bytes, device: int = 0):
        self.lib = _lib.load()
        _bind(self.lib)
        if len(unique_id) != 128:
            raise ValueError("unique_id must be the 128 bytes cfm_comm_get_unique_id returned")
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_comm_init(rank, world, unique_id, device, ctypes.byref(h)), "cfm_comm_init")
        self.handle, self.rank, self.world, self.device = h, rank, world, device

    @staticmethod
    def unique_id() -> bytes:
        lib = _lib.load()
        _bind(lib)
        buf = ctypes.create_string_buffer(128)
        _lib.check(lib.cfm_comm_get_unique_id(buf), "cfm_comm_get_unique_id")
        return buf.raw

    def allreduce(self, t: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError("allreduce takes a contiguous fp32 CUDA tensor")
        _lib.check(self.lib.cfm_allreduce_grads(self.handle, t.data_ptr(), t.numel(), float(scale), _stream()),
                   "cfm_allreduce_grads")
        return t

    @property
    def allreduce_cb(self):
        """(function pointer, user) for cfm_train_opts.allreduce / allreduce_user (SyncBatchNorm)."""
        return ctypes.cast(self.lib.cfm_comm_allreduce_cb, ctypes.c_void_p), self.handle

    def close(self) -> None:
        if self.handle:
            _lib.check(self.lib.cfm_comm_destroy(self.handle), "cfm_comm_destroy")
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:   # noqa: BLE001
            pass


class NativeGradBuckets(GradBuckets):
    """GradBuckets whose per-layer all-reduces the library issues from inside cfm_train_backward."""

    def __init__(self, comm: NativeComm, table_params: Sequence[Optional[torch.Tensor]],
                 other_params: Iterable[torch.nn.Parameter] = (), average: bool = True):
        super().__init__(table_params, other_params, group=None, average=average)
        self.comm = comm
        self.world = comm.world
        lib = comm.lib
        n = len(self.rows)
        offs = (ctypes.c_int64 * max(n, 1))(*[r[0] if r else 0 for r in self.rows])
        cnts = (ctypes.c_int64 * max(n, 1))(*[r[1] if r else 0 for r in self.rows])
        h = ctypes.c_void_p()
        _lib.check(lib.cfm_grad_buckets_create(comm.handle, self.flat.data_ptr(), self.numel, n, offs, cnts,
                                               1 if average else 0, ctypes.byref(h)), "cfm_grad_buckets_create")
        self.handle = h
        # read by EncoderTrainer.backward: the C callback and its user pointer go into cfm_train_opts
        self.native_ready = (ctypes.cast(lib.cfm_grad_buckets_ready_cb, ctypes.c_void_p), h)

    def on_ready(self, first: int, n: int, stream=None) -> None:   # only used when called from Python
        fn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)(
            self.native_ready[0].value)
        if fn(self.handle, first, n, stream) != 0:
            raise RuntimeError("cfm_grad_buckets_ready_cb failed: " + _lib.load().cfm_last_error().decode(errors="replace"))

    def issued_count(self) -> int:
        return int(self.comm.lib.cfm_grad_buckets_issued(self.handle))

    def _finish_impl(self) -> None:
        _lib.check(self.comm.lib.cfm_grad_buckets_finish(self.handle, _stream()), "cfm_grad_buckets_finish")

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                self.comm.lib.cfm_grad_buckets_destroy(self.handle)
                self.handle = None
        except Exception:   # noqa: BLE001
            pass
