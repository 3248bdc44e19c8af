"""Data-parallel plumbing of the training step: one process per GPU, torch.distributed
with the "nccl" backend (RCCL over xGMI on ROCm; "gloo" in the CPU tests).

* `GradBuckets` / `enable_gradient_buckets` — the step's gradient exchange (DDP's averaging, which
  with CTC `mean_batch` and equal per-rank batches gives the global-batch gradient), overlapped
  with the backward: every trainable parameter's `.grad` is a VIEW of one flat fp32 buffer (no
  copy-in / copy-out), laid out in the native parameter-table order so that each Conformer layer's
  gradients are one contiguous bucket (~6.8 MB for Large); the native backward reports each layer
  as soon as its last gradient kernel is enqueued (`grad_ready`, cfm_train.h) and the bucket's
  RCCL all-reduce is issued right then, ordered after the library's stream, so it runs while the
  earlier layers' backward computes.  Buckets are per layer (17 of them, not DDP's 25 MB cap):
  xGMI rings are per-link bound (7 x ~153 GB/s), a 6.8 MB bucket already runs at bandwidth, and
  per-layer granularity lets the exchange start one layer's backward after the loss.  At the end
  of the backward (autograd's queue_callback) the non-encoder gradients (CTC head) go as one last
  bucket, every bucket is waited for (stream-level, no host sync) and the buffer scaled by 1/world.
* `allreduce_gradients` — the same exchange without overlap: one flat all-reduce after the
  backward (the bitwise reference of the bucketed path in the tests).
* `convert_sync_batchnorm` — the counterpart of torch.nn.SyncBatchNorm.convert_sync_batchnorm,
  which Lightning applies for `sync_batchnorm: true` (conformer_ctc_bpe.yaml:175): the native
  encoder then sums its BatchNorm statistics over the group (see cfm_train.h).
* `shard_batch` — the utterance partition: rank r of N takes rows [r*B/N, (r+1)*B/N).
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple

import torch


def _world(group=None) -> int:
    import torch.distributed as dist
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def flatten_grads(params: Iterable[torch.nn.Parameter]) -> List[torch.nn.Parameter]:
    """Parameters that hold a gradient, in a fixed order (deduplicated shared parameters)."""
    seen, out = set(), []
    for p in params:
        if p.grad is None or id(p) in seen:
            continue
        seen.add(id(p))
        out.append(p)
    return out


def allreduce_gradients(params: Iterable[torch.nn.Parameter], group=None, average: bool = True,
                        bucket: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Sum (and average) every `.grad` across the group with ONE all-reduce on a flat bucket.
    Returns the bucket (pass it back in to reuse the allocation)."""
    import torch.distributed as dist
    world = _world(group)
    ps = flatten_grads(params)
    if world <= 1 or not ps:
        return bucket
    n = sum(p.grad.numel() for p in ps)
    dev = ps[0].grad.device
    if bucket is None or bucket.numel() < n or bucket.device != dev:
        bucket = torch.empty(n, dtype=torch.float32, device=dev)
    off = 0
    for p in ps:
        k = p.grad.numel()
        bucket[off:off + k].copy_(p.grad.reshape(-1))
        off += k
    flat = bucket[:n]
    dist.all_reduce(flat, group=group)
    if average:
        flat.mul_(1.0 / world)
    off = 0
    for p in ps:
        k = p.grad.numel()
        p.grad.copy_(flat[off:off + k].view_as(p.grad))
        off += k
    return bucket


def convert_sync_batchnorm(module: torch.nn.Module, group=None) -> torch.nn.Module:
    """Make every native ConformerEncoder inside `module` share BatchNorm statistics over `group`."""
    from nemo.collections.asr.modules import ConformerEncoder
    for m in module.modules():
        if isinstance(m, ConformerEncoder):
            m.set_sync_batchnorm(group)
    return module


def shard_batch(x: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Rows of the global batch owned by `rank` (equal shares; B must divide by world)."""
    B = x.shape[0]
    if B % world:
        raise ValueError(f"global batch {B} does not split evenly over {world} ranks")
    per = B // world
    return x[rank * per:(rank + 1) * per]


class GradBuckets:
    """Per-layer gradient buckets over one flat buffer (see the module docstring).

    table_params: the native parameter-table rows in order (None / buffers / frozen parameters are
      skipped); a `grad_ready(first, n)` range of rows is one contiguous slice of the buffer.
    other_params: every other trainable parameter (reduced as the last bucket)."""

    def __init__(self, table_params: Sequence[Optional[torch.Tensor]], other_params: Iterable[torch.nn.Parameter] = (),
                 group=None, average: bool = True):
        seen = set()
        self.rows: List[Optional[Tuple[int, int]]] = []      # table row -> (offset, numel) or None
        self.members: List[torch.nn.Parameter] = []
        self.offsets: List[int] = []
        off = 0
        for p in table_params:
            if isinstance(p, torch.nn.Parameter) and p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                self.rows.append((off, p.numel()))
                self.members.append(p)
                self.offsets.append(off)
                off += p.numel()
            else:
                self.rows.append(None)
        self.table_end = off
        self.n_table_members = len(self.members)
        for p in other_params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                self.members.append(p)
                self.offsets.append(off)
                off += p.numel()
        self.numel = off
        dev = self.members[0].device if self.members else torch.device("cpu")
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.views = [self.flat[o:o + p.numel()].view_as(p) for o, p in zip(self.offsets, self.members)]
        self.group = group
        self.average = average
        self.world = _world(group)
        self._works = []
        self._reduced = []           # (start, end) slices already issued this step
        self._fresh, self._pending, self._finish_queued, self._scratch, self._direct = True, 0, False, None, True
        self._rescale_owed = False   # the buffer holds sums reduced without averaging (see the step notes)
        for p, v in zip(self.members, self.views):
            p.grad = v
        # the owed rescale runs before autograd adds a later backward's gradient into a non-table view
        for p in self.members[self.n_table_members:]:
            p.register_hook(self._pay_rescale_hook)

    # ---- per step -------------------------------------------------------------------------------
    # Gradient accumulation (several backward() calls per optimizer step, or an encoder run twice in
    # one graph): a fresh step (some member's .grad is None, e.g. after zero_grad(set_to_none=True))
    # zeroes the buffer and the first native backward writes straight into it, with the per-layer
    # all-reduces overlapped.  Any later native backward of the same step writes into a scratch buffer
    # that is then added into the views, and its exchange is one all-reduce of the whole buffer at the
    # end of the backward.  All-reducing the accumulated sum is exact: the part already reduced is equal
    # on every rank, so sum_r(avg(g1) + g2_r) / W = avg(g1) + avg(g2).  Without averaging the reduced
    # part R = sum(g1) would come back W times, so the buffer is scaled by 1/W before the next backward
    # of the step writes into it: sum_r(R / W + g2_r) = sum(g1) + sum(g2).  That rescale is owed from
    # the moment a finish() leaves reduced sums in the buffer and is paid by the first write of the next
    # backward that actually runs - a gradient hook on every non-table member (it fires before autograd
    # accumulates into the view) or `native_outputs` for the encoder rows - never by a forward: a
    # train-mode forward with no backward after it must leave the reduced gradients alone, and with
    # pipelined accumulation (fwd1, fwd2, bwd1, bwd2) the second forward runs before the first finish.
    # A new step is recognised by a member's .grad being None or not its view: use
    # zero_grad(set_to_none=True) (the default) or call begin_step(); after zero_grad(set_to_none=False)
    # the next backward is taken for an accumulation (still exact, but without the per-layer overlap).
    def _pay_rescale(self) -> None:
        if self._rescale_owed:
            self._rescale_owed = False
            self.flat.mul_(1.0 / self.world)

    def _pay_rescale_hook(self, grad):
        self._pay_rescale()
        return grad

    def begin_step(self) -> None:
        """Start a new optimizer step explicitly: zero the buffer, the next backward overlaps per layer."""
        self.flat.zero_()
        self._fresh, self._pending, self._finished, self._rescale_owed = True, 0, False, False
        for p, v in zip(self.members, self.views):
            p.grad = v

    def attach(self) -> None:
        """Point every member's .grad at its view; zero the buffer when a new step starts (a member's
        .grad is None or not the view).  Called by every train-mode encoder forward."""
        fresh = any(p.grad is None or p.grad.data_ptr() != v.data_ptr() for p, v in zip(self.members, self.views))
        if fresh:
            self.flat.zero_()
            self._fresh = True
            self._pending = 0
            self._finished = False
            self._rescale_owed = False
        for p, v in zip(self.members, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v
        self._pending = getattr(self, "_pending", 0) + 1

    @property
    def overlap(self) -> bool:
        """The next native backward may write into the views directly and all-reduce layer by layer:
        it is the first of a fresh step and the step runs the encoder once."""
        return getattr(self, "_fresh", True) and getattr(self, "_pending", 1) <= 1

    def native_outputs(self, params: Sequence[torch.Tensor], want: Sequence[bool]) -> List[Optional[torch.Tensor]]:
        """Output pointers for cfm_train_backward: table row i writes straight into its view (first
        backward of a fresh step) or into the accumulation scratch (see `accumulate_scratch`)."""
        self._pay_rescale()
        direct = getattr(self, "_fresh", True)
        if direct:
            base = self.flat
        else:
            if getattr(self, "_scratch", None) is None or self._scratch.numel() < self.table_end:
                self._scratch = torch.empty(max(self.table_end, 1), dtype=torch.float32, device=self.flat.device)
            self._scratch.zero_()
            base = self._scratch
        out = []
        for i, (p, w) in enumerate(zip(params, want)):
            if not w:
                out.append(None)
                continue
            r = self.rows[i] if i < len(self.rows) else None
            if r is None:
                raise RuntimeError(f"table row {i} wants a gradient but is not in the gradient buckets")
            out.append(base[r[0]:r[0] + r[1]])
        self._direct = direct
        return out

    def after_backward(self) -> None:
        """After cfm_train_backward was enqueued: fold a scratch-written gradient into the views."""
        if not getattr(self, "_direct", True):
            self.flat[:self.table_end].add_(self._scratch[:self.table_end])
        self._fresh = False

    def queue_finish(self) -> None:
        """Run `finish` once at the end of the current autograd backward pass."""
        if getattr(self, "_finish_queued", False):
            return
        self._finish_queued = True
        torch.autograd.Variable._execution_engine.queue_callback(self.finish)

    def _issue(self, start: int, end: int, stream=None) -> None:
        if end <= start:
            return
        self._reduced.append((start, end))
        if self.world <= 1:
            return
        import torch.distributed as dist
        from .train import on_library_stream
        with on_library_stream(stream, self.flat.device):
            self._works.append(dist.all_reduce(self.flat[start:end], group=self.group, async_op=True))

    def on_ready(self, first: int, n: int, stream=None) -> None:
        """grad_ready(first, n): all-reduce the slice of table rows [first, first + n)."""
        spans = [self.rows[i] for i in range(first, min(first + n, len(self.rows))) if self.rows[i] is not None]
        if spans:
            self._issue(min(o for o, _ in spans), max(o + k for o, k in spans), stream)

    def finish(self) -> None:
        """End of the backward: reduce whatever no grad_ready covered, wait, average."""
        try:
            self._finish_impl()
            self._finished = True
            self._rescale_owed = not self.average and self.world > 1
        finally:
            self._finish_queued = False
            self._pending = 0
            self._issued_last, self._reduced = self._reduced, []

    def _finish_impl(self) -> None:
        covered = sorted(self._reduced)
        pos, gaps = 0, []
        for a, b in covered:
            if a > pos:
                gaps.append((pos, a))
            pos = max(pos, b)
        if pos < self.numel:
            gaps.append((pos, self.numel))
        for a, b in gaps:
            self._issue(a, b)
        for w in self._works:
            w.wait()
        if self.average and self.world > 1:
            self.flat.mul_(1.0 / self.world)
        self._works = []

    @property
    def issued(self) -> List[Tuple[int, int]]:
        """Slices issued so far in this backward, or after `finish` those of the last one."""
        return list(self._reduced or getattr(self, "_issued_last", []))


def enable_gradient_buckets(model: torch.nn.Module, group=None, average: bool = True) -> GradBuckets:
    """Bucketed, overlapped gradient all-reduce for a model holding one native ConformerEncoder:
    the encoder's parameters in native table order, then every other trainable parameter."""
    from nemo.collections.asr.modules import ConformerEncoder
    encs = [m for m in model.modules() if isinstance(m, ConformerEncoder)]
    if len(encs) != 1:
        raise ValueError("enable_gradient_buckets expects exactly one ConformerEncoder in the model")
    enc = encs[0]
    names = enc.native_param_names()
    sd = enc.state_dict(keep_vars=True)
    table = [sd.get(n) for n in names]
    ids = {id(t) for t in table if t is not None}
    others = [p for p in model.parameters() if id(p) not in ids]
    gb = GradBuckets(table, others, group=group, average=average)
    enc.set_grad_buckets(gb)
    return gb
