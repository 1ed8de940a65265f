"""Torch-facing wrappers of the HIP C-ABI: train/eval forward, backward, Adam, fused train step.

Every function here runs the HIP kernels of ``csrc/eegnet_kernels.hip`` through
``libeegnet_hip.so``; tensors must live on a HIP device.  There is no CPU or eager-PyTorch path.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib

NCLS = 4


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_device(t: torch.Tensor, what: str):
    if t.device.type != "cuda":
        raise RuntimeError(
            f"{what} is on '{t.device}': the MI355X EEGNet path runs on a HIP device only "
            f"(move the model and the inputs to 'cuda').")


@dataclass(frozen=True)
class Shape:
    """Static dims of one EEGNet instance (model.py:13)."""
    C: int
    T: int
    F1: int = 8
    D: int = 2
    K1: int = 32
    p: float = 0.5
    eps: float = 1e-5
    momentum: float = 0.1

    @property
    def F2(self):
        return self.F1 * self.D

    @property
    def T1(self):
        return self.T // 4

    @property
    def T2(self):
        return self.T1 // 8

    def dims(self, B: int, p: float | None = None, x_pitch: int = 0) -> _lib.Dims:
        if p is None:                 # per-(B, pitch) cache (the struct is only read by the library)
            cache = self.__dict__.setdefault("_dims_cache", {})
            d = cache.get((B, x_pitch))
            if d is None:
                d = cache[(B, x_pitch)] = _lib.dims(B, self.C, self.T, self.F1, self.D, self.K1, self.p,
                                                    self.eps, self.momentum, x_pitch)
            return d
        return _lib.dims(B, self.C, self.T, self.F1, self.D, self.K1, p, self.eps, self.momentum, x_pitch)

    def x_pitch(self) -> int:
        """The x row pitch the training kernels load fastest (eegnet_x_pitch): T rounded up to 4
        floats for 22 x 257, else T."""
        return int(_lib.load().eegnet_x_pitch(ctypes.byref(self.dims(1))))

    def param_shapes(self):
        """(name, shape) in nn.Module.named_parameters() order (model.py:22-84)."""
        F1, F2, C, K1 = self.F1, self.F2, self.C, self.K1
        nf = F2 * (self.T // 32)
        return [
            ("temporal.0.weight", (F1, 1, 1, K1)), ("temporal.1.weight", (F1,)),
            ("temporal.1.bias", (F1,)), ("spatial.weight", (F2, 1, C, 1)),
            ("aggregation.0.weight", (F2,)), ("aggregation.0.bias", (F2,)),
            ("block_2.0.weight", (F2, 1, 1, 16)), ("block_2.1.weight", (F2, F2, 1, 1)),
            ("block_2.2.weight", (F2,)), ("block_2.2.bias", (F2,)),
            ("classifier.weight", (NCLS, nf)), ("classifier.bias", (NCLS,)),
        ]

    def n_params(self):
        n = 0
        for _, s in self.param_shapes():
            k = 1
            for d in s:
                k *= d
            n += k
        return n

    def bn_layout(self):
        """Flat bn_buffers order of the ABI: rm1, rv1, rm2, rv2, rm3, rv3."""
        F1, F2 = self.F1, self.F2
        return [("temporal.1.running_mean", F1), ("temporal.1.running_var", F1),
                ("aggregation.0.running_mean", F2), ("aggregation.0.running_var", F2),
                ("block_2.2.running_mean", F2), ("block_2.2.running_var", F2)]


def new_workspace(shape: Shape, B: int, device) -> torch.Tensor:
    nbytes = _lib.workspace_bytes(shape.dims(B))
    return torch.zeros(nbytes, dtype=torch.uint8, device=device)   # zero-filled once (tickets)


def forward_train(shape: Shape, flat_params, bn_flat, x, ws, seed: int, offset: int,
                  masks=None, p: float | None = None, nbt=None) -> torch.Tensor:
    """Train-mode forward: BN batch stats (+ running-stat update in bn_flat), dropout."""
    B = x.shape[0]
    logits = torch.empty((B, NCLS), dtype=torch.float32, device=x.device)
    m2, m3 = masks if masks is not None else (None, None)
    d = shape.dims(B, p, x_pitch_of(x))
    _lib.check(_lib.load().eegnet_forward_train(
        ctypes.byref(d), _ptr(flat_params), _ptr(bn_flat), _ptr(x), _ptr(m2), _ptr(m3),
        ctypes.c_uint64(seed), ctypes.c_uint64(offset), _ptr(logits), _ptr(ws), _stream(),
        _ptr(nbt)), "eegnet_forward_train")
    return logits


NO_CLAMP = 1
KEY_FROM_STEP = 2      # include/eegnet_abi.h: dropout key follows the device Adam step (graphs)


def backward(shape: Shape, flat_params, x, ws, seed: int, offset: int, dlogits=None, labels=None,
             masks=None, p: float | None = None, grads=None, loss=None, clamp=True) -> torch.Tensor:
    B = x.shape[0]
    if grads is None:
        grads = torch.empty_like(flat_params)
    m2, m3 = masks if masks is not None else (None, None)
    d = shape.dims(B, p, x_pitch_of(x))
    _lib.check(_lib.load().eegnet_backward(
        ctypes.byref(d), _ptr(flat_params), _ptr(x), _ptr(dlogits), _ptr(labels), _ptr(m2),
        _ptr(m3), ctypes.c_uint64(seed), ctypes.c_uint64(offset), _ptr(grads), _ptr(loss), _ptr(ws),
        _stream(), 0 if clamp else NO_CLAMP), "eegnet_backward")
    return grads


def clamp_grads(shape: Shape, grads):
    """model.py:44/84 gradient clamps on a flat grad buffer (after a data-parallel all-reduce)."""
    _lib.check(_lib.load().eegnet_clamp_grads(ctypes.byref(shape.dims(1)), _ptr(grads), _stream()),
               "eegnet_clamp_grads")


def forward_eval(shape: Shape, flat_params, bn_flat, x) -> torch.Tensor:
    x = x.contiguous()                # the eval kernels read [B][C][T] rows (no pitch)
    B = x.shape[0]
    logits = torch.empty((B, NCLS), dtype=torch.float32, device=x.device)
    d = shape.dims(B)
    _lib.check(_lib.load().eegnet_forward_eval(
        ctypes.byref(d), _ptr(flat_params), _ptr(bn_flat), _ptr(x), _ptr(logits), _stream()),
        "eegnet_forward_eval")
    return logits


def forward_eval_bf16(shape: Shape, flat_params, bn_flat, x) -> torch.Tensor:
    """Eval-mode forward on bf16 input (bf16 MFMA operands, fp32 accumulation, fp32 logits)."""
    if x.dtype != torch.bfloat16:
        raise RuntimeError(f"forward_eval_bf16 expects bfloat16 input (got {x.dtype})")
    x = x.contiguous()
    B = x.shape[0]
    logits = torch.empty((B, NCLS), dtype=torch.float32, device=x.device)
    d = shape.dims(B)
    _lib.check(_lib.load().eegnet_forward_eval_bf16(
        ctypes.byref(d), _ptr(flat_params), _ptr(bn_flat), _ptr(x), _ptr(logits), _stream()),
        "eegnet_forward_eval_bf16")
    return logits


def adam_step(params, grads, exp_avg, exp_avg_sq, step_i32, lr=1e-3, betas=(0.9, 0.999), eps=1e-7):
    _lib.check(_lib.load().eegnet_adam_step(
        ctypes.c_int64(params.numel()), _ptr(params), _ptr(grads), _ptr(exp_avg), _ptr(exp_avg_sq),
        _ptr(step_i32), ctypes.c_float(lr), ctypes.c_float(betas[0]), ctypes.c_float(betas[1]),
        ctypes.c_float(eps), _stream()), "eegnet_adam_step")


def x_pitch_of(x: torch.Tensor) -> int:
    """eegnet_dims.x_pitch for x: 0 for a contiguous [B, C, T] tensor, the channel-row pitch for a
    [B, C, T] view of [B, C, pitch] rows (``pad_x_rows``)."""
    if x.is_contiguous():
        return 0
    B, C, T = x.shape
    if x.stride(2) != 1 or x.stride(0) != C * x.stride(1) or x.stride(1) < T:
        raise ValueError("x must be a contiguous [B, C, T] tensor or a [B, C, T] view of [B, C, pitch] rows")
    if x.data_ptr() % 16:
        # pitched rows go to LDS in 16-byte DMA units: every row must start 16-byte aligned
        raise ValueError("a pitched x view must start 16-byte aligned")
    return int(x.stride(1))


def pad_x_rows(x: torch.Tensor, pitch: int) -> torch.Tensor:
    """A copy of x [N, C, T] with its rows at ``pitch`` floats (zeros after T), returned as the
    [N, C, T] view the training entry points take (x_pitch_of): 22 x 257 trials then load in 16-byte
    units."""
    N, C, T = x.shape
    if pitch == T:
        return x.contiguous()
    xp = torch.zeros((N, C, pitch), dtype=x.dtype, device=x.device)
    xp[:, :, :T] = x
    return xp[:, :, :T]


def train_step(shape: Shape, flat_params, bn_flat, x, labels, seed: int, offset: int, grads,
               adam_state, step_i32, ws, loss, logits=None, lr=1e-3, betas=(0.9, 0.999), eps=1e-7,
               p: float | None = None, clamp=True, nbt=None, key_from_step=False):
    """One fused hot-loop iteration (model.py:141-148) on the device, no host sync.
    ``adam_state=None`` stops after the gradients (data-parallel)."""
    d = shape.dims(x.shape[0], p, x_pitch_of(x))
    _lib.check(_lib.load().eegnet_train_step(
        ctypes.byref(d), _ptr(flat_params), _ptr(bn_flat), _ptr(x), _ptr(labels),
        ctypes.c_uint64(seed), ctypes.c_uint64(offset), _ptr(grads), _ptr(adam_state),
        _ptr(step_i32), ctypes.c_float(lr), ctypes.c_float(betas[0]), ctypes.c_float(betas[1]),
        ctypes.c_float(eps), _ptr(loss), _ptr(logits), _ptr(ws), _stream(),
        (0 if clamp else NO_CLAMP) | (KEY_FROM_STEP if key_from_step else 0),
        _ptr(nbt)), "eegnet_train_step")


def train_stage(shape: Shape, stage: int, norm_batch: int, flat_params, bn_flat, x, labels, seed: int,
                offset: int, grads, adam_state, step_i32, ws, loss, lr=1e-3, betas=(0.9, 0.999), eps=1e-7,
                p: float | None = None, nbt=None):
    """eegnet_train_stage: stage 2k = pass k with its finalize deferred (sums left in ``ws``),
    stage 2k + 1 = pass k's finalize on the (all-reduced) sums; statistics normalised by
    ``norm_batch`` (the global batch of a synchronised-BatchNorm data-parallel step)."""
    d = shape.dims(x.shape[0], p, x_pitch_of(x))
    _lib.check(_lib.load().eegnet_train_stage(
        ctypes.byref(d), ctypes.c_int(stage), ctypes.c_int64(norm_batch), _ptr(flat_params), _ptr(bn_flat),
        _ptr(x), _ptr(labels), ctypes.c_uint64(seed), ctypes.c_uint64(offset), _ptr(grads), _ptr(adam_state),
        _ptr(step_i32), ctypes.c_float(lr), ctypes.c_float(betas[0]), ctypes.c_float(betas[1]),
        ctypes.c_float(eps), _ptr(loss), _ptr(ws), _stream(), 0, _ptr(nbt)), "eegnet_train_stage")


def stage_sums(shape: Shape, B: int, ws: torch.Tensor, p: float | None = None) -> list[torch.Tensor]:
    """The five float64 views of ``ws`` (a uint8 workspace tensor) that stages 0, 2, 4, 6, 8 leave
    their sums in (one buffer, reused by every pass: view k holds pass k's sums after stage 2k)."""
    d = shape.dims(B, p)
    lib = _lib.load()
    out = []
    for k in range(5):
        off, n = ctypes.c_size_t(0), ctypes.c_int(0)
        _lib.check(lib.eegnet_stage_sums(ctypes.byref(d), ctypes.c_int(k), ctypes.byref(off), ctypes.byref(n)),
                   "eegnet_stage_sums")
        out.append(ws[off.value:off.value + 8 * n.value].view(torch.float64))
    return out


def x_stats(shape: Shape, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """eegnet_x_stats: the per-trial, parameter-free BN1 statistics of x [N, C, T] (contiguous or a
    pad_x_rows view) as a [N, width] float32 device tensor -- the lag sums of each trial's zero-padded
    rows over the channels, its window-0 sample sum and the 'same' padding's edge products / sums.
    A fold whose training set is fixed reads a batch's rows of it instead of recomputing them."""
    require_device(x, "x")
    lib = _lib.load()
    N = x.shape[0]
    d = shape.dims(1, None, x_pitch_of(x))
    width = int(lib.eegnet_x_stats_width(ctypes.byref(d)))
    if width <= 0:
        _lib.check(width, "eegnet_x_stats_width")
    if out is None:
        out = torch.empty((N, width), dtype=torch.float32, device=x.device)
    elif tuple(out.shape) != (N, width) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError(f"out must be a contiguous float32 [{N}, {width}] tensor")
    if N:
        _lib.check(lib.eegnet_x_stats(ctypes.byref(d), ctypes.c_int64(N), _ptr(x), _ptr(out), _stream()),
                   "eegnet_x_stats")
    return out


def fold_table(entries, device) -> torch.Tensor:
    """Device array of ``eegnet_fold`` entries (a uint8 tensor holding the packed structs).
    ``entries``: dicts with the eegnet_fold fields as tensors (or None) and ``seed`` as an int."""
    n = len(entries)
    arr = (_lib.Fold * n)()
    for i, e in enumerate(entries):
        for name, _ in _lib.Fold._fields_:
            if name == "seed":
                continue
            t = e.get(name)
            setattr(arr[i], name, 0 if t is None else t.data_ptr())
        arr[i].seed = int(e["seed"]) & ((1 << 64) - 1)
    raw = bytes(arr)
    return torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)


def train_step_folds(shape: Shape, B: int, table: torch.Tensor, nfolds: int, row0: int, slot: int,
                     offset: int = 0, lr=1e-3, betas=(0.9, 0.999), eps=1e-7, p: float | None = None,
                     x_pitch: int = 0):
    """eegnet_train_step_folds: one fused step of ``nfolds`` independent models in one launch per
    pass (fold index = grid y).  ``table`` from fold_table(); every fold trains on rows
    [row0, row0 + B) of its own x / labels and writes its loss to losses[slot].  ``x_pitch``: the
    row pitch of every fold's x (0: contiguous [N, C, T]; pad_x_rows)."""
    d = shape.dims(B, p, x_pitch)
    _lib.check(_lib.load().eegnet_train_step_folds(
        ctypes.byref(d), ctypes.c_int(nfolds), _ptr(table), ctypes.c_int64(row0), ctypes.c_int64(slot),
        ctypes.c_uint64(offset), ctypes.c_float(lr), ctypes.c_float(betas[0]), ctypes.c_float(betas[1]),
        ctypes.c_float(eps), _stream()), "eegnet_train_step_folds")
