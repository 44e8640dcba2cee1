"""View-sharded multi-GPU rendering: one process per GPU, torch.distributed
over RCCL (backend "nccl" on ROCm) on the GPU path, gloo in the CPU tests.

Views are independent given the replicated mesh, so a batch of G·n views is split contiguously:
rank r renders views [r·n, (r+1)·n) (weak scaling: n fixed per GPU). The only exchanges a
training step needs are

* ``allreduce_grads``: one all_reduce(sum) of the shared-parameter gradients (vertex positions /
  colours; V x 3 f32 = 35 KB for the cow), flattened into a single bucket;
* ``gather_to_root`` (optional, e.g. C4's image gather): each rank's slice goes to the root over
  its own point-to-point link (batched isend/irecv). On a fully connected xGMI node every slice
  crosses a different direct link in parallel, instead of a ring all-gather pushing (G-1)/G of
  the whole tensor through every link.

Per-view pose gradients stay on their rank. Packed face ids stay global (view n of the whole
batch keeps id n·F + f) via ``global_view_offset``.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    """(rank, world_size); (0, 1) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n_total: int, rank: int, world_size: int):
    """Contiguous [start, stop) of views for `rank`; the first n_total % world_size ranks get one extra."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} / world size {world_size}")
    base, extra = divmod(n_total, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_views(*tensors, n_total=None, rank=None, world_size=None):
    """Slice per-view tensors (leading dim = view) to this rank's shard."""
    r, w = world()
    rank = r if rank is None else rank
    world_size = w if world_size is None else world_size
    n_total = tensors[0].shape[0] if n_total is None else n_total
    s, e = shard_range(n_total, rank, world_size)
    out = tuple(t[s:e] for t in tensors)
    return out[0] if len(out) == 1 else out


def global_view_offset(n_total, rank=None, world_size=None):
    r, w = world()
    return shard_range(n_total, r if rank is None else rank, w if world_size is None else world_size)[0]


def allreduce_grads(params, group=None):
    """Sum the .grad of replicated parameters over ranks in ONE flattened all_reduce.

    Every rank must call the same collective with a buffer of the same size, whatever it rendered: a
    rank with an empty view shard (``shard_range`` hands them out when there are fewer views than
    ranks) or a parameter its views did not reach has ``.grad`` None. Such a gradient travels as zeros,
    so the flattened buffer always holds every gradient-requiring parameter of ``params`` in list order
    (the list is the same replicated parameters on every rank), followed by one presence flag per
    parameter (1 where the rank had a gradient). After the reduction a parameter that NO rank reached
    gets ``.grad = None`` back, as on one rank and as DDP leaves globally unused parameters, so that an
    optimiser skips it (Adam's moments and weight decay would otherwise move it). Only a rank that had
    no gradient of its own reads the flags back to the host (one synchronisation); a rank whose
    parameters all had gradients keeps the step asynchronous."""
    _, w = world()
    if w == 1:
        return
    live = [p for p in params if p is not None and p.requires_grad]
    if not live:
        return
    had = [p.grad is not None for p in live]
    ref = next((p.grad for p in live if p.grad is not None), live[0])
    dev, dt = ref.device, ref.dtype
    parts = [(p.grad if h else torch.zeros_like(p, dtype=dt)).reshape(-1) for p, h in zip(live, had)]
    parts.append(torch.tensor([1.0 if h else 0.0 for h in had], dtype=dt, device=dev))
    flat = torch.cat(parts)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for p, h in zip(live, had):
        n = p.numel()
        if h:
            p.grad.copy_(flat[off:off + n].view_as(p.grad))
        else:
            p.grad = flat[off:off + n].view_as(p).clone()
        off += n
    if not all(had):
        flags = flat[off:].tolist()  # (this rank lacked a gradient: is the parameter used anywhere?)
        for p, h, f in zip(live, had, flags):
            if not h and f == 0.0:
                p.grad = None


def gather_to_root(local: torch.Tensor, n_total: int, root: int = 0, group=None):
    """Assemble the per-rank view slices into the full (n_total, ...) tensor on `root`
    (returns None elsewhere) with one batched set of point-to-point transfers. Over gloo (the CPU
    tests, and the 1-GPU rehearsal of the N-rank path) device tensors travel through host copies."""
    rank, w = world()
    if w == 1:
        return local
    host = local.is_cuda and dist.get_backend(group) == "gloo"
    if rank != root:
        s, e = shard_range(n_total, rank, w)
        if e > s:
            src = local.contiguous().cpu() if host else local.contiguous()
            dist.batch_isend_irecv([dist.P2POp(dist.isend, src, root, group)])[0].wait()
        return None
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device="cpu" if host else local.device)
    ops = []
    for r in range(w):
        s, e = shard_range(n_total, r, w)
        if r == root:
            out[s:e].copy_(local)
        elif e > s:
            ops.append(dist.P2POp(dist.irecv, out[s:e], r, group))
    for req in dist.batch_isend_irecv(ops) if ops else []:
        req.wait()
    return out.to(local.device) if host else out
