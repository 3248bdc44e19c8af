"""Host runtime of the native training step (include/cfm_train.h, csrc/train.hip).

`EncoderTrainer` drives `cfm_train_forward` / `cfm_train_backward` on one GPU: the train-mode
encoder forward records an activation tape (a torch-owned device buffer), the backward replays it
and writes every parameter gradient in the reference state_dict layout.  `encoder_train_forward`
wraps the pair as one torch.autograd.Function, so the drop-in `ConformerEncoder` in `.train()` mode
behaves like the reference module under autograd (EncDecCTCModel.training_step -> loss.backward(),
ctc_models.py:485-514): gradients land in each nn.Parameter's `.grad`.

Multi-GPU: SyncBatchNorm statistics are summed across ranks by a host callback that runs a
torch.distributed (RCCL) all-reduce on a view of the library's workspace, ordered after the
library's stream.  The gradient exchange is `conformer_amd.dist.GradBuckets` (gradients as views
of one flat buffer, each layer's bucket all-reduced asynchronously as soon as the native backward
has enqueued it: `grad_ready` in cfm_train.h) or, without buckets, the one flat all-reduce of
`conformer_amd.dist.allreduce_gradients` after the backward.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
GRAD_READY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p)


class CfmTrainOpts(ctypes.Structure):
    _fields_ = [("dropout", ctypes.c_float), ("dropout_emb", ctypes.c_float), ("dropout_att", ctypes.c_float),
                ("bn_momentum", ctypes.c_float), ("update_running_stats", ctypes.c_int), ("world", ctypes.c_int),
                ("seed", ctypes.c_uint64), ("allreduce", ALLREDUCE_FN), ("allreduce_user", ctypes.c_void_p),
                ("grad_ready", GRAD_READY_FN), ("grad_ready_user", ctypes.c_void_p)]


def _bind(lib) -> None:
    if getattr(lib, "_cfm_train_bound", False):
        return
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    pp = ctypes.POINTER(ctypes.c_void_p)
    for name, res, args in (
            ("cfm_train_tape_size", sz, [vp, ci, ci]),
            ("cfm_train_workspace_size", sz, [vp, ci, ci]),
            ("cfm_train_forward", ci, [vp, pp, ci, vp, vp, ci, ci, ctypes.POINTER(CfmTrainOpts), vp, vp, vp, sz, vp,
                                       sz, vp]),
            ("cfm_train_backward", ci, [vp, pp, ci, vp, ci, ci, ctypes.POINTER(CfmTrainOpts), pp, vp, sz, vp, sz,
                                        vp])):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._cfm_train_bound = True


class EncoderTrainer:
    """Training step of one encoder handle (a `NativeEncoder`) on one GPU."""

    def __init__(self, native):
        self.native = native
        self.lib = native.lib
        _bind(self.lib)
        self.device = torch.device("cuda", native.device)
        self.names: List[str] = list(native.param_names().keys())
        self._ws: Optional[torch.Tensor] = None
        self._cb = None          # keep the ctypes callbacks alive
        self._ready_cb = None
        self._group = None
        self.world = 1
        self.use_pad_mask = True   # ConformerEncoder.enable_pad_mask: the conv module's pad mask
        self.grad_buckets = None   # conformer_amd.dist.GradBuckets (data parallelism), or None

    # ---- SyncBatchNorm plumbing ---------------------------------------------------------------
    def set_sync_group(self, group=None, world: Optional[int] = None) -> None:
        """Share BatchNorm statistics over `group` (torch.distributed, RCCL on ROCm)."""
        import torch.distributed as dist
        self._group = group
        self.world = int(world if world is not None else dist.get_world_size(group))

    def _make_callback(self):
        if self.world <= 1:
            return None

        def cb(user, buf, n, stream):
            try:
                import torch.distributed as dist
                ws = self._ws
                off = int(buf) - ws.data_ptr()
                if off < 0 or off % 4 or off + 4 * n > ws.numel():
                    return 1
                view = ws[off:off + 4 * n].view(torch.float32)
                with on_library_stream(stream, ws.device):   # ordered after the library's kernels
                    dist.all_reduce(view, group=self._group)
                return 0
            except Exception:   # noqa: BLE001  (no exception may cross the C boundary)
                return 1
        return ALLREDUCE_FN(cb)

    # ---- step ------------------------------------------------------------------------------------
    def _opts(self, dropout: float, seed: int, update_running_stats: bool, bn_momentum: float,
              dropout_emb: float = 0.0, dropout_att: float = 0.0) -> CfmTrainOpts:
        o = CfmTrainOpts()
        o.dropout = float(dropout)
        o.dropout_emb = float(dropout_emb)
        o.dropout_att = float(dropout_att)
        o.bn_momentum = float(bn_momentum)
        o.update_running_stats = 1 if update_running_stats else 0
        o.world = self.world
        o.seed = int(seed) & ((1 << 64) - 1)
        self._cb = self._make_callback()
        if self._cb is not None:
            o.allreduce = self._cb
        o.allreduce_user = None
        return o

    def _make_ready_callback(self):
        gb = self.grad_buckets

        def cb(user, first, n, stream):
            try:
                gb.on_ready(first, n, stream)
                return 0
            except Exception:   # noqa: BLE001
                return 1
        return GRAD_READY_FN(cb)

    def _workspace(self, B: int, T: int) -> torch.Tensor:
        n = int(self.lib.cfm_train_workspace_size(self.native.handle, B, T))
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self._ws

    def _ptrs(self, tensors: Sequence[Optional[torch.Tensor]]):
        arr = (ctypes.c_void_p * len(tensors))()
        for i, t in enumerate(tensors):
            arr[i] = None if t is None else t.data_ptr()
        return arr

    def _grad_views(self, params: Sequence[torch.Tensor], want: Sequence[bool]) -> List[Optional[torch.Tensor]]:
        """Fresh gradient tensors for one backward: views of ONE new flat allocation (one caching-
        allocator call instead of one per parameter; ~480 separate allocations kept the host busy for
        ~1.8 ms between the CTC head's backward and the encoder's, with the GPU idle)."""
        key = tuple(want)
        meta = getattr(self, "_gv_meta", None)
        if meta is None or meta[0] != key:
            sizes = [p.numel() if w else 0 for p, w in zip(params, want)]
            offs, o = [], 0
            for n in sizes:
                offs.append(o)
                o += n
            meta = (key, sizes, offs, o, [tuple(p.shape) for p in params])
            self._gv_meta = meta
        _, sizes, offs, total, shapes = meta
        flat = torch.empty(max(total, 1), dtype=torch.float32, device=self.device)
        parts = flat[:total].split(sizes)
        self._gv_flat = (flat, offs)
        return [parts[i].view(shapes[i]) if w else None for i, w in enumerate(want)]

    def _out_ptrs(self, out: Sequence[Optional[torch.Tensor]]):
        gv = getattr(self, "_gv_flat", None)
        if gv is not None and out and any(t is not None for t in out):
            flat, offs = gv
            first = next(t for t in out if t is not None)
            if first.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr():
                base = flat.data_ptr()
                self._gv_flat = None
                return (ctypes.c_void_p * len(out))(*[None if t is None else base + 4 * o for t, o in zip(out, offs)])
        return self._ptrs(out)

    def check_params(self, params: Sequence[torch.Tensor]) -> None:
        if len(params) != len(self.names):
            raise ValueError(f"expected {len(self.names)} parameter tensors, got {len(params)}")
        for n, p in zip(self.names, params):
            if p.device != self.device or p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError(f"{n}: parameters must be contiguous fp32 tensors on {self.device}")

    def forward(self, x_bft: torch.Tensor, lengths: Optional[torch.Tensor], params: Sequence[torch.Tensor],
                dropout: float = 0.0, seed: int = 0, update_running_stats: bool = True, bn_momentum: float = 0.1,
                dropout_emb: float = 0.0, dropout_att: float = 0.0):
        from .runtime import encoded_length
        self.check_params(params)
        x = x_bft.detach().to(self.device, torch.float32).contiguous()
        B, F, T = x.shape
        Tp = encoded_length(T)
        d = self.native.cfg.d_model
        y = torch.empty((B, d, Tp), dtype=torch.float32, device=self.device)
        ylen = torch.empty((B,), dtype=torch.int32, device=self.device)
        ln = None
        if lengths is not None:
            ln = lengths.to(device=self.device, dtype=torch.int32).contiguous()
        tape = torch.empty(int(self.lib.cfm_train_tape_size(self.native.handle, B, T)), dtype=torch.uint8,
                           device=self.device)
        ws = self._workspace(B, T)
        self.native.set_pad_mask(self.use_pad_mask)
        o = self._opts(dropout, seed, update_running_stats, bn_momentum, dropout_emb, dropout_att)
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        pptr = self._ptrs(params)
        _lib.check(self.lib.cfm_train_forward(self.native.handle, pptr, len(params), x.data_ptr(),
                                              None if ln is None else ln.data_ptr(), B, T, ctypes.byref(o),
                                              y.data_ptr(), ylen.data_ptr(), tape.data_ptr(), tape.numel(),
                                              ws.data_ptr(), ws.numel(), st), "cfm_train_forward", lib=self.lib)
        state = dict(tape=tape, B=B, T=T, dropout=dropout, seed=seed, bn_momentum=bn_momentum, x=x, ln=ln, pptr=pptr,
                     dropout_emb=dropout_emb, dropout_att=dropout_att, use_pad_mask=self.use_pad_mask)
        return y, ylen, state

    def backward(self, dy_bdt: torch.Tensor, state: Dict, params: Sequence[torch.Tensor],
                 want: Sequence[bool]) -> List[Optional[torch.Tensor]]:
        dy = dy_bdt.detach().to(self.device, torch.float32).contiguous()
        gb = self.grad_buckets
        if gb is not None:
            # gradients written straight into the bucket views (p.grad); autograd gets None for them
            out = gb.native_outputs(params, want)
            grads = [None] * len(params)
        else:
            out = grads = self._grad_views(params, want)
        ws = self._workspace(state["B"], state["T"])
        o = self._opts(state["dropout"], state["seed"], False, state["bn_momentum"], state["dropout_emb"],
                       state["dropout_att"])
        if gb is not None:
            if gb.overlap and getattr(gb, "native_ready", None) is not None:
                # conformer_amd.comm.NativeGradBuckets: the library's own callback issues the RCCL
                # all-reduces (cfm_grad_buckets_ready_cb), no Python in the backward
                fn, user = gb.native_ready
                self._ready_cb = GRAD_READY_FN(fn.value)
                o.grad_ready = self._ready_cb
                o.grad_ready_user = user
            elif gb.overlap:
                self._ready_cb = self._make_ready_callback()
                o.grad_ready = self._ready_cb
            # the remaining (non-encoder, or accumulated) gradients are final only when the whole
            # backward is done
            gb.queue_finish()
        tape = state["tape"]
        self.native.set_pad_mask(state.get("use_pad_mask", True))   # the forward's setting
        st = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        pptr = state.get("pptr") or self._ptrs(params)   # the forward's table (same tensors)
        _lib.check(self.lib.cfm_train_backward(self.native.handle, pptr, len(params), dy.data_ptr(),
                                               state["B"], state["T"], ctypes.byref(o), self._out_ptrs(out),
                                               tape.data_ptr(), tape.numel(), ws.data_ptr(), ws.numel(), st),
                   "cfm_train_backward", lib=self.lib)
        if gb is not None:
            gb.after_backward()
        return grads


class on_library_stream:
    """Context: make `stream` (a hipStream_t the library passed to a callback) torch's current stream,
    so a torch.distributed collective issued inside is ordered after the library's enqueued work."""

    def __init__(self, stream, device):
        self.stream, self.device = stream, device
        self._ctx = None

    def __enter__(self):
        if self.stream and getattr(self.device, "type", "cpu") == "cuda":
            s = torch.cuda.ExternalStream(int(self.stream), device=self.device)
            self._ctx = torch.cuda.stream(s)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
        return False


class _EncoderTrainFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, trainer: EncoderTrainer, x, lengths, cfg: Tuple, *params):
        dropout, seed, update_stats, momentum, dropout_emb, dropout_att = cfg
        y, ylen, state = trainer.forward(x, lengths, params, dropout, seed, update_stats, momentum, dropout_emb,
                                         dropout_att)
        ctx.trainer = trainer
        ctx.state = state
        ctx.params = params
        ctx.mark_non_differentiable(ylen)
        return y, ylen

    @staticmethod
    def backward(ctx, dy, _dylen):
        want = [bool(ctx.needs_input_grad[4 + i]) for i in range(len(ctx.params))]
        if dy is None:
            dy = torch.zeros((ctx.state["B"], ctx.trainer.native.cfg.d_model, 1), device=ctx.trainer.device)
        grads = ctx.trainer.backward(dy, ctx.state, ctx.params, want)
        ctx.state = None
        return (None, None, None, None, *grads)


def encoder_train_forward(trainer: EncoderTrainer, x: torch.Tensor, lengths: Optional[torch.Tensor],
                          params: Sequence[torch.Tensor], dropout: float, seed: int,
                          update_running_stats: bool = True, bn_momentum: float = 0.1,
                          dropout_emb: float = 0.0, dropout_att: float = 0.0):
    """Differentiable native train-mode encoder forward: returns (y (B, d, T'), lengths (B,) int32).
    dropout: embedding / FFN / residual-branch dropout; dropout_emb: positional-embedding dropout
    (multi_head_attention.py:316); dropout_att: attention-probability dropout (:111)."""
    return _EncoderTrainFn.apply(trainer, x, lengths, (float(dropout), int(seed), bool(update_running_stats),
                                                       float(bn_momentum), float(dropout_emb), float(dropout_att)),
                                 *params)
