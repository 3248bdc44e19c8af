"""Host runtime of the RNN-T prediction network and greedy decoding (include/cfm_rnnt_decode.h).

`NativePredictionNet` owns one `cfm_rnnt_decoder*` (embedding + packed LSTM layers on one GPU):
`predict` is RNNTDecoder.predict (rnnt.py:190-283) and `greedy` runs the whole greedy batch decode
(rnnt_greedy_decoding.py:453-616) on the device, returning per-utterance tokens, timesteps, scores
and final LSTM states.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib

ACTIVATIONS = {"relu": 0, "sigmoid": 1, "tanh": 2}


def _bind(lib) -> None:
    if getattr(lib, "_cfm_rnnt_decode_bound", False):
        return
    vp, ci, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    pp = ctypes.POINTER(ctypes.c_void_p)
    for name, res, args in (
            ("cfm_rnnt_decoder_create", ci, [ci, ci, ci, ci, ctypes.POINTER(vp)]),
            ("cfm_rnnt_decoder_destroy", None, [vp]),
            ("cfm_rnnt_decoder_set_weights", ci, [vp, vp, pp, pp, pp, pp, vp]),
            ("cfm_rnnt_decoder_predict_workspace_size", sz, [vp, ci, ci]),
            ("cfm_rnnt_decoder_predict", ci, [vp, vp, ci, ci, ci, vp, vp, vp, vp, vp, vp, sz, vp]),
            ("cfm_rnnt_greedy_workspace_size", sz, [vp, ci, ci, ci]),
            ("cfm_rnnt_decoder_train_tape_size", sz, [vp, ci, ci, ci]),
            ("cfm_rnnt_decoder_train_forward", ci, [vp, vp, ci, ci, ci, ctypes.c_float, ctypes.c_uint64, vp, vp, sz, vp]),
            ("cfm_rnnt_decoder_backward_workspace_size", sz, [vp, ci, ci, ci]),
            ("cfm_rnnt_decoder_backward", ci, [vp, vp, ci, ci, ci, ctypes.c_float, ctypes.c_uint64, vp, vp, pp, pp, vp, pp,
                                               pp, pp, pp, vp, sz, vp]),
            ("cfm_rnnt_greedy_decode", ci, [vp, vp, vp, ci, ci, ci, ci, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, vp, vp,
                                            vp, vp, vp, vp, vp, sz, vp])):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib._cfm_rnnt_decode_bound = True


def _ptrs(ts: Sequence[torch.Tensor]):
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), arr


class NativePredictionNet:
    """Embedding + LSTM stack of RNNTDecoder on one GPU (fp32)."""

    def __init__(self, vocab_size: int, pred_hidden: int, layers: int, device=None):
        self.lib = _lib.load()
        _bind(self.lib)
        if not torch.cuda.is_available():
            raise _lib.CfmError("the native RNN-T prediction network needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.V, self.H, self.L = int(vocab_size), int(pred_hidden), int(layers)
        h = ctypes.c_void_p()
        _lib.check(self.lib.cfm_rnnt_decoder_create(self.V, self.H, self.L, self.device.index, ctypes.byref(h)),
                   "cfm_rnnt_decoder_create")
        self.handle = h
        self._ws: Optional[torch.Tensor] = None

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            self.lib.cfm_rnnt_decoder_destroy(h)
            self.handle = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _workspace(self, n: int) -> torch.Tensor:
        if self._ws is None or self._ws.numel() < n:
            self._ws = None
            self._ws = torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    def set_weights(self, embed: torch.Tensor, w_ih: List[torch.Tensor], w_hh: List[torch.Tensor],
                    b_ih: List[torch.Tensor], b_hh: List[torch.Tensor]) -> None:
        f = lambda t: t.detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        emb = f(embed)
        lists = [[f(t) for t in ts] for ts in (w_ih, w_hh, b_ih, b_hh)]
        keep = [_ptrs(ts) for ts in lists]
        _lib.check(self.lib.cfm_rnnt_decoder_set_weights(self.handle, emb.data_ptr(), *[k[0] for k in keep],
                                                         self._stream()), "cfm_rnnt_decoder_set_weights")
        # stream-ordered: the copies freed here are only reused by work queued after the pack (torch's
        # caching allocator), so no host synchronisation (it would drain the queue every training step)

    def predict(self, y: Optional[torch.Tensor], h0: Optional[torch.Tensor], c0: Optional[torch.Tensor],
                add_sos: bool, batch_size: int) -> Tuple[torch.Tensor, Tuple[torch.Tensor, torch.Tensor]]:
        dev = self.device
        if y is not None:
            y = y.to(dev, torch.int64).contiguous()
            B, U = y.shape
        else:
            B, U = int(batch_size), 1
        S = (U if y is not None else 1) + (1 if add_sos else 0)
        g = torch.empty((B, S, self.H), dtype=torch.float32, device=dev)
        h = torch.empty((self.L, B, self.H), dtype=torch.float32, device=dev)
        c = torch.empty_like(h)
        hs = None if h0 is None else h0.detach().to(dev, torch.float32).contiguous()
        cs = None if c0 is None else c0.detach().to(dev, torch.float32).contiguous()
        n = int(self.lib.cfm_rnnt_decoder_predict_workspace_size(self.handle, B, U))
        ws = self._workspace(n)
        _lib.check(self.lib.cfm_rnnt_decoder_predict(
            self.handle, None if y is None else y.data_ptr(), B, U if y is not None else 0, 1 if add_sos else 0,
            None if hs is None else hs.data_ptr(), None if cs is None else cs.data_ptr(), g.data_ptr(), h.data_ptr(),
            c.data_ptr(), ws.data_ptr(), ws.numel(), self._stream()), "cfm_rnnt_decoder_predict")
        return g, (h, c)

    # ---- training (cfm_rnnt_decoder_train_forward / _backward) ---------------------------------
    def train_forward(self, y: torch.Tensor, add_sos: bool, dropout: float, seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Teacher-forced g (B, S, H) from the zero state, plus the tape the backward needs."""
        y = y.to(self.device, torch.int64).contiguous()
        B, U = y.shape
        S = U + (1 if add_sos else 0)
        g = torch.empty((B, S, self.H), dtype=torch.float32, device=self.device)
        n = int(self.lib.cfm_rnnt_decoder_train_tape_size(self.handle, B, U, 1 if add_sos else 0))
        tape = torch.empty(n, dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.cfm_rnnt_decoder_train_forward(self.handle, y.data_ptr(), B, U, 1 if add_sos else 0,
                                                           ctypes.c_float(dropout), ctypes.c_uint64(seed), g.data_ptr(),
                                                           tape.data_ptr(), n, self._stream()),
                   "cfm_rnnt_decoder_train_forward")
        return g, tape

    def backward(self, y: torch.Tensor, add_sos: bool, dropout: float, seed: int, tape: torch.Tensor, dg: torch.Tensor,
                 w_ih: List[torch.Tensor], w_hh: List[torch.Tensor], want: Sequence[bool]):
        """(d_embed, [dw_ih], [dw_hh], [db_ih], [db_hh]); `want` = (embed, w_ih, w_hh, b_ih, b_hh)."""
        y = y.to(self.device, torch.int64).contiguous()
        B, U = y.shape
        dg = dg.detach().to(self.device, torch.float32).contiguous()
        f = lambda t: t.detach().to(self.device, torch.float32).contiguous()  # noqa: E731
        wi, wh = [f(t) for t in w_ih], [f(t) for t in w_hh]
        z = lambda shape, on: [torch.empty(shape, device=self.device) for _ in range(self.L)] if on else None  # noqa: E731
        demb = torch.empty((self.V + 1, self.H), device=self.device) if want[0] else None
        dwi = z((4 * self.H, self.H), want[1])
        dwh = z((4 * self.H, self.H), want[2])
        dbi = z((4 * self.H,), want[3] or want[4])
        dbh = z((4 * self.H,), want[4])
        n = int(self.lib.cfm_rnnt_decoder_backward_workspace_size(self.handle, B, U, 1 if add_sos else 0))
        ws = self._workspace(n)
        keep = []

        def arr(ts):
            if ts is None:
                return None
            p, a = _ptrs(ts)
            keep.append(a)
            return p
        pwi, pwh = arr(wi), arr(wh)
        _lib.check(self.lib.cfm_rnnt_decoder_backward(
            self.handle, y.data_ptr(), B, U, 1 if add_sos else 0, ctypes.c_float(dropout), ctypes.c_uint64(seed),
            tape.data_ptr(), dg.data_ptr(), pwi, pwh, None if demb is None else demb.data_ptr(), arr(dwi), arr(dwh),
            arr(dbi), arr(dbh), ws.data_ptr(), n, self._stream()), "cfm_rnnt_decoder_backward")
        return demb, dwi, dwh, (dbi if want[3] else None), dbh

    def greedy(self, enc_bdt: torch.Tensor, enc_len: torch.Tensor, joint_params: Sequence[torch.Tensor],
               activation: str, max_symbols: int, log_normalize: bool, sos_until_label: bool = False):
        """-> tokens (B, T*max_symbols) int32, timesteps, ntok (B) int32, scores (B) float64,
        h, c (L, B, H) — all on the device; the call returns when decoding has finished."""
        dev = self.device
        e = enc_bdt.detach().to(dev, torch.float32).contiguous()
        B, D1, T = e.shape
        ln = enc_len.detach().to(dev, torch.int64).contiguous()
        w_enc, b_enc, w_pred, b_pred, w_out, b_out = [t.detach().to(dev, torch.float32).contiguous()
                                                      for t in joint_params]
        J = w_enc.shape[0]
        if w_out.shape[0] != self.V + 1 or w_pred.shape[1] != self.H or w_enc.shape[1] != D1:
            raise ValueError("joint parameters do not match the prediction network / encoder output")
        cap = max(1, T * int(max_symbols))
        tokens = torch.empty((B, cap), dtype=torch.int32, device=dev)
        tsteps = torch.empty_like(tokens)
        ntok = torch.empty((B,), dtype=torch.int32, device=dev)
        scores = torch.empty((B,), dtype=torch.float64, device=dev)
        h = torch.empty((self.L, B, self.H), dtype=torch.float32, device=dev)
        c = torch.empty_like(h)
        n = int(self.lib.cfm_rnnt_greedy_workspace_size(self.handle, B, T, J))
        ws = self._workspace(n)
        _lib.check(self.lib.cfm_rnnt_greedy_decode(
            self.handle, e.data_ptr(), ln.data_ptr(), B, T, D1, J, w_enc.data_ptr(), b_enc.data_ptr(),
            w_pred.data_ptr(), b_pred.data_ptr(), w_out.data_ptr(), b_out.data_ptr(), ACTIVATIONS[activation.lower()],
            int(max_symbols), 1 if log_normalize else 0, 1 if sos_until_label else 0, tokens.data_ptr(), tsteps.data_ptr(), ntok.data_ptr(),
            scores.data_ptr(), h.data_ptr(), c.data_ptr(), ws.data_ptr(), ws.numel(), self._stream()),
            "cfm_rnnt_greedy_decode")
        return tokens, tsteps, ntok, scores, h, c
