"""Scale-out for the EEGNet step on one 8 x MI355X node.

Two shapes of parallelism, one process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm):

* data parallel (cfg4): every rank runs the fused HIP step on its own slice of the global batch,
  the flat fp32 gradient (1,716 floats = 6.9 KB for EEGNet-8,2) is summed with ONE all-reduce per
  step, averaged, then clamped (model.py:44/84 hooks AFTER the reduction, so the clamp sees the
  global-batch gradient) and Adam runs replicated.  BatchNorm uses per-rank batch
  statistics (the DDP default).  The message is latency-bound (~7 KB), so there is exactly one
  collective per step and nothing to bucket.
* fold sharding (cfg3): independent cross-/within-subject folds are dealt to ranks by
  longest-processing-time order with no communication on the data path; results are merged on the
  host (``gather_results``).
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import ops
from .model import EEGNet, FusedAdamState


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init_process_group(backend: str | None = None):
    """Initialise torch.distributed from the torchrun environment (MASTER_ADDR/PORT, RANK ...)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


class DataParallelTrainer:
    """Fused HIP train step + one RCCL gradient all-reduce per step (cfg4)."""

    def __init__(self, model: EEGNet, lr=1e-3, betas=(0.9, 0.999), eps=1e-7, group=None):
        self.model = model
        self.lr, self.betas, self.eps = lr, betas, eps
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.adam = FusedAdamState(model)
        flat = model.flat_parameters()
        if self.world > 1:   # identical start on every rank
            dist.broadcast(flat, 0, group=group)
        self.loss = torch.zeros(1, dtype=torch.float32, device=flat.device)
        self._ws = {}
        self._step = 0

    def workspace(self, B):
        ws = self._ws.get(B)
        if ws is None:
            ws = ops.new_workspace(self.model.shape, B, self.model.flat_parameters().device)
            self._ws[B] = ws
        return ws

    def step(self, x, y):
        m = self.model
        shape = m.shape
        self._step += 1
        seed = 0x5EED_0000 + self._step
        offset = self._step * self.world + self.rank        # distinct masks on every rank
        flat = m.flat_parameters()
        grads = self.adam.grads
        ops.train_step(shape, flat, m.flat_bn_buffers(), x, y, seed, offset, grads, None, None,
                       self.workspace(x.shape[0]), self.loss, clamp=False)
        if self.world > 1:
            dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=self.group)
            grads.mul_(1.0 / self.world)
        ops.clamp_grads(shape, grads)
        n = flat.numel()
        ops.adam_step(flat, grads, self.adam.state[:n], self.adam.state[n:], self.adam.step,
                      lr=self.lr, betas=self.betas, eps=self.eps)
        for bn in m._bns():
            bn.num_batches_tracked.add_(1)
        return self.loss


def lpt_assign(costs, n_ranks):
    """Longest-processing-time-first assignment of independent units to ranks.
    Returns a list (per rank) of unit indices; deterministic (ties by index)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    loads = [0.0] * n_ranks
    out = [[] for _ in range(n_ranks)]
    for i in order:
        r = min(range(n_ranks), key=lambda k: (loads[k], k))
        out[r].append(i)
        loads[r] += costs[i]
    for lst in out:
        lst.sort()
    return out


def gather_results(local: dict, group=None) -> dict:
    """Merge per-rank {unit_id: result} dicts onto every rank (host-side, after the work)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return dict(local)
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, local, group=group)
    merged = {}
    for p in parts:
        merged.update(p)
    return merged
