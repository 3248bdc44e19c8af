"""Data-parallel plumbing of the training step: one process per GPU, torch.distributed
with the "nccl" backend (RCCL over xGMI on ROCm; "gloo" in the CPU tests).

* `allreduce_gradients` — the step's single gradient exchange: every parameter gradient is packed
  into ONE flat fp32 bucket, summed with one all-reduce and scaled by 1/world (DDP's averaging,
  which with CTC `mean_batch` and equal per-rank batches gives the global-batch gradient).
  One large collective instead of DDP's 25 MB buckets: on xGMI the ring is per-link bandwidth
  bound, and 461 MB in one call amortises the launch/latency terms best.
* `convert_sync_batchnorm` — the counterpart of torch.nn.SyncBatchNorm.convert_sync_batchnorm,
  which Lightning applies for `sync_batchnorm: true` (conformer_ctc_bpe.yaml:175): the native
  encoder then sums its BatchNorm statistics over the group (see cfm_train.h).
* `shard_batch` — the utterance partition: rank r of N takes rows [r*B/N, (r+1)*B/N).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

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
