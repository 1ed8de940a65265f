"""Scale-out for the EEGNet step on one 8 x MI355X node.

Two shapes of parallelism, one process per GPU (torch.distributed; backend "nccl" = RCCL on ROCm):

* data parallel (cfg4): every rank runs the fused HIP step on its own slice of the global batch,
  the flat fp32 gradient (1,716 floats = 6.9 KB for EEGNet-8,2) is summed with ONE all-reduce per
  step, averaged, then clamped (model.py:44/84 hooks AFTER the reduction, so the clamp sees the
  global-batch gradient) and Adam runs replicated.  BatchNorm normalises with per-rank
  batch statistics; rank 0's running statistics and the global mean loss ride in the same message
  (DDP's broadcast_buffers).  The message is latency-bound (~7 KB), so there is exactly one
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


def allreduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean over ranks: ONE all-reduce of the whole flat buffer (latency-bound message)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / dist.get_world_size(group))
    return t


class DataParallelTrainer:
    """Fused HIP train step + ONE collective per step (cfg4).

    Per step (``step``): local gradients (HIP, clamps deferred) -> one all-reduce (SUM) of the flat
    communication buffer ``[grads | loss | BN running statistics]`` -> x 1/world on the gradient and
    the loss -> model.py:44/84 clamps -> Adam, replicated on every rank.

    BatchNorm normalises with per-rank batch statistics.  Running statistics follow DDP's default
    ``broadcast_buffers=True`` -- every rank ends each step holding rank 0's -- but they travel in the
    same all-reduce as the gradient: rank 0 contributes its freshly updated buffers, every other rank
    contributes zeros, so the sum IS rank 0's buffers (x + 0 == x exactly).  In train mode the
    forward reads batch statistics, never the running ones, so moving the broadcast from before the
    forward (DDP) to after it changes no result; it leaves every rank with rank 0's buffers after
    every step, including the last (what eval and checkpoints read).  ``num_batches_tracked`` is
    broadcast once at construction with the parameters: every rank then adds exactly one per step.
    The loss returned is the global-batch mean (the all-reduced per-rank means / world).

    ``sync_bn=True`` (SURVEY 8(e)2's SyncBN option): BatchNorm normalises with GLOBAL-batch statistics.
    The step is the single-device step of model.py:141-148 over the concatenated batch, split at its
    five batch-global reductions (eegnet_train_stage): per pass, the HIP kernel leaves its fp64 sums in
    the workspace, ONE all-reduce (SUM) of those sums runs (352 / 32 / 549 / 544 / 896 doubles for
    EEGNet-8,2 at 22 x 256), and the pass's finalize runs on the global sums -- so BN statistics,
    running statistics, the CE mean, the gradients, the clamps (on the global gradient) and the fused
    Adam come out the same on every rank, with no separate gradient all-reduce and no buffer
    broadcast.  Five latency-bound collectives per step instead of one; every rank's shard must have
    the same size.

    The stages are methods so the orchestration can be exercised on CPU (gloo) with stand-ins for
    the device kernels.
    """

    def __init__(self, model: EEGNet, lr=1e-3, betas=(0.9, 0.999), eps=1e-7, group=None,
                 broadcast_buffers=True, sync_bn=False):
        self.model = model
        self.sync_bn = bool(sync_bn)
        if self.sync_bn and model.shape.F2 > 16:
            raise ValueError("sync_bn: F1*D > 16 is not supported (eegnet_train_stage)")
        self.lr, self.betas, self.eps = lr, betas, eps
        self.group = group
        self.broadcast_buffers = broadcast_buffers
        # collectives run whenever a process group exists -- at world 1 too, where each is an
        # identity (x 1/1, rank 0's own buffers) and the step stays bit-identical to FusedTrainer:
        # that is how a one-GPU box exercises the RCCL path (tests/test_gpu_distributed.py)
        self.dist = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        flat = model.flat_parameters()
        if self.dist:        # identical start on every rank: parameters, BN buffers and counters
            self.broadcast_state()
        self._init_state(flat)
        self._ws = {}
        self._step = 0

    def _src(self, r):
        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _init_state(self, flat):
        n, nb = flat.numel(), self.model.flat_bn_buffers().numel()
        self.adam = FusedAdamState(self.model)
        # the step's single message: [grads n | loss 1 | BN running statistics nb], fp32
        self.comm = torch.zeros(n + 1 + nb, dtype=torch.float32, device=flat.device)
        self.adam.grads = self.comm[:n]
        self.loss = self.comm[n:n + 1]

    def broadcast_state(self):
        """Rank 0's parameters, BN running statistics and num_batches_tracked to every rank, as ONE
        float64 broadcast (fp32 and the int64 counters below 2^53 round-trip exactly)."""
        m = self.model
        flat, bn, nbt = m.flat_views()
        buf = torch.cat([flat.detach().double(), bn.double(), nbt.double()])
        dist.broadcast(buf, self._src(0), group=self.group)
        n, nb = flat.numel(), bn.numel()
        with torch.no_grad():
            flat.copy_(buf[:n])
            bn.copy_(buf[n:n + nb])
            nbt.copy_(buf[n + nb:].round().to(torch.int64))

    def workspace(self, B):
        ws = self._ws.get(B)
        if ws is None:
            ws = ops.new_workspace(self.model.shape, B, self.model.flat_parameters().device)
            self._ws[B] = ws
        return ws

    # -- stages ------------------------------------------------------------------------------
    def local_grads(self, x, y, seed, offset):
        m = self.model
        flat, bn, nbt = m.flat_views()
        ops.train_step(m.shape, flat, bn, x, y, seed, offset,
                       self.adam.grads, None, None, self.workspace(x.shape[0]), self.loss,
                       clamp=False, nbt=nbt)
        return self.adam.grads

    def reduce(self, grads):
        """ONE all-reduce (SUM) of [grads | loss | rank 0's BN buffers], then x 1/world on the
        gradient and the loss (CE is a batch mean) and rank 0's buffers into every rank's BN."""
        if not self.dist:
            return grads
        n = grads.numel()
        bn = self.model.flat_bn_buffers()
        tail = self.comm[n + 1:]
        if not self.broadcast_buffers:
            tail.zero_()
        elif self.rank == 0:
            tail.copy_(bn)
        else:
            tail.zero_()
        dist.all_reduce(self.comm, op=dist.ReduceOp.SUM, group=self.group)
        self.comm[:n + 1].mul_(1.0 / self.world)
        if self.broadcast_buffers:
            with torch.no_grad():
                bn.copy_(tail)
        return grads

    def clamp(self, grads):
        ops.clamp_grads(self.model.shape, grads)

    def update(self, grads):
        flat = self.model.flat_parameters()
        n = flat.numel()
        ops.adam_step(flat, grads, self.adam.state[:n], self.adam.state[n:], self.adam.step,
                      lr=self.lr, betas=self.betas, eps=self.eps)

    # -- synchronised BatchNorm stages ----------------------------------------------------------
    def global_batch(self, B):
        """The batch the synchronised statistics and the CE mean are normalised by: the sum of the
        ranks' local batches, all-reduced every step (a short last batch on one rank -- a sampler with
        drop_last=False -- must not mis-normalise every rank's statistics and gradients).  One small
        collective and a host read per step, in the sync_bn path only."""
        if not self.dist:
            return B
        t = torch.tensor([B], dtype=torch.float64, device=self.model.flat_parameters().device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return int(t.item())

    def stage(self, k, x, y, seed, offset, norm_batch=None):
        """eegnet_train_stage k (2j: pass j with its sums left in the workspace; 2j + 1: its finalize)."""
        m = self.model
        B = x.shape[0]
        nb = B * self.world if norm_batch is None else norm_batch
        ops.train_stage(m.shape, k, nb, m.flat_parameters(), m.flat_bn_buffers(), x, y, seed,
                        offset, self.adam.grads, self.adam.state, self.adam.step, self.workspace(B),
                        self.loss, lr=self.lr, betas=self.betas, eps=self.eps, nbt=m.flat_num_batches_tracked())

    def stage_sums(self, B):
        key = ("sums", B)
        v = self._ws.get(key)
        if v is None:
            v = ops.stage_sums(self.model.shape, B, self.workspace(B))
            self._ws[key] = v
        return v

    def reduce_sums(self, sums):
        """ONE all-reduce (SUM) of a pass's fp64 sums."""
        if self.dist:
            dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=self.group)
        return sums

    def step_sync_bn(self, x, y):
        self._step += 1
        seed = 0x5EED_0000 + self._step
        offset = self._step * self.world + self.rank
        sums = self.stage_sums(x.shape[0])
        nb = self.global_batch(x.shape[0])
        for j in range(5):
            self.stage(2 * j, x, y, seed, offset, nb)
            self.reduce_sums(sums[j])
            self.stage(2 * j + 1, x, y, seed, offset, nb)
        return self.loss

    def step(self, x, y):
        if self.sync_bn:
            return self.step_sync_bn(x, y)
        self._step += 1
        seed = 0x5EED_0000 + self._step
        offset = self._step * self.world + self.rank        # distinct masks on every rank
        grads = self.local_grads(x, y, seed, offset)
        self.reduce(grads)
        self.clamp(grads)
        self.update(grads)
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
