"""Drop-in for ``eegnet_repl.model`` (PraKesEy/EEGNetReplication src/eegnet_repl/model.py).

``EEGNet`` keeps the reference's submodule tree, parameter/buffer names and shapes
(model.py:22-84) so ``state_dict`` round-trips with reference checkpoints and any ``torch.optim``
optimizer can step it; the grad-clamp hooks of model.py:44 and model.py:84 are registered the same
way.  ``forward`` never runs those submodules: it runs the MI355X HIP kernels through
``libeegnet_hip.so`` (train mode: 5-pass fused step; eval mode: one fused inference kernel).

``train`` / ``evaluate_model`` mirror model.py:101-189 / 191-227 (same arguments, returns, logging
cadence and the F4 "best model aliases the live weights" behaviour), with the epoch loss and
accuracy accumulated on the device (one host sync per epoch instead of one per batch).  When the
optimizer is ``torch.optim.Adam`` and the loss is a default ``nn.CrossEntropyLoss`` the whole step
(forward, CE, backward, clamps, Adam) runs as one fused device sequence.
"""

from __future__ import annotations

import logging

import torch
import torch.nn as nn

from . import ops
from .ops import Shape, require_device

logger = logging.getLogger("eegnet_repl")


class EEGNet(nn.Module):
    """EEGNet-F1,D (Lawhern et al. 2018) with the reference's module layout (model.py:12-99).

    C, T: channels and samples per trial; F1 temporal filters; D depth multiplier; p dropout.
    ``K1`` (temporal kernel length) defaults to the reference's 32 (model.py:26).
    """

    def __init__(self, C, T, F1=8, D=2, p=0.5, K1=32):
        super().__init__()
        F2 = F1 * D
        self.temporal = nn.Sequential(
            nn.Conv2d(1, F1, kernel_size=(1, K1), padding="same", bias=False),
            nn.BatchNorm2d(F1))
        self.spatial = nn.Conv2d(F1, D * F1, kernel_size=(C, 1), padding="valid", groups=F1,
                                 bias=False)
        self.spatial.weight.register_hook(lambda g: torch.clamp(g, min=-1.0, max=1.0))
        self.aggregation = nn.Sequential(nn.BatchNorm2d(D * F1), nn.ELU(),
                                         nn.AvgPool2d(kernel_size=(1, 4)), nn.Dropout(p=p))
        self.block_2 = nn.Sequential(
            nn.Conv2d(D * F1, D * F1, kernel_size=(1, 16), padding="same", groups=D * F1,
                      bias=False),
            nn.Conv2d(D * F1, F2, kernel_size=(1, 1), padding="same", bias=False),
            nn.BatchNorm2d(F2), nn.ELU(), nn.AvgPool2d(kernel_size=(1, 8)), nn.Dropout(p=p),
            nn.Flatten())
        self.classifier = nn.Linear(F2 * (T // 32), 4, bias=True)
        self.classifier.weight.register_hook(lambda g: torch.clamp(g, min=-0.25, max=0.25))
        self.C, self.T, self.F1, self.D, self.K1 = C, T, F1, D, K1
        self._masks = None
        self._rng_offset = 0
        self._flatten()

    # -- flat device layout -----------------------------------------------------------------
    def _bns(self):
        return (self.temporal[1], self.aggregation[0], self.block_2[2])

    def _flatten(self):
        """Re-home every parameter (and BN running stat) as a view of one flat fp32 buffer, in
        named_parameters() order -- the layout of include/eegnet_abi.h.  Parameter identity is
        kept (``.data`` is rebound), so optimizers built before ``.to()`` keep working."""
        # (module, attribute) of every parameter, in named_parameters() order: _flat_ok checks that
        # each slot still holds the Parameter re-homed here (a caller may assign a new one)
        self._pslots = [(mod, name) for mod in self.modules() for name, q in mod._parameters.items()
                        if q is not None]
        params = [mod._parameters[name] for mod, name in self._pslots]
        assert len(params) == len(list(self.parameters()))
        dev = params[0].device
        n = sum(p.numel() for p in params)
        flat = torch.empty(n, dtype=torch.float32, device=dev)
        o = 0
        for p in params:
            k = p.numel()
            flat[o:o + k].copy_(p.data.reshape(-1))
            p.data = flat[o:o + k].view(p.shape)
            o += k
        self._flat = flat
        bufs = []
        for bn in self._bns():
            bufs += [bn.running_mean, bn.running_var]
        nb = sum(b.numel() for b in bufs)
        bflat = torch.empty(nb, dtype=torch.float32, device=dev)
        o = 0
        views = []
        for b in bufs:
            k = b.numel()
            bflat[o:o + k].copy_(b.reshape(-1))
            views.append(bflat[o:o + k])
            o += k
        for bn, (rm, rv) in zip(self._bns(), zip(views[0::2], views[1::2])):
            bn.running_mean = rm
            bn.running_var = rv
        self._bn_flat = bflat
        # the three num_batches_tracked counters as views of one int64[3] buffer: the HIP forward
        # increments them in-kernel (no per-step host-side add_ launches)
        nflat = torch.zeros(3, dtype=torch.int64, device=dev)
        for i, bn in enumerate(self._bns()):
            if bn.num_batches_tracked is not None:
                nflat[i:i + 1].copy_(bn.num_batches_tracked.reshape(1))
                bn.num_batches_tracked = nflat[i:i + 1].view(())
        self._nbt_flat = nflat
        # the tensors _flat_ok checks, gathered once (a module-tree walk per call costs ~25 us of
        # host time, the whole budget of a batch-64 step)
        self._plist = params
        self._blist = [t for bn in self._bns() for t in (bn.running_mean, bn.running_var)]
        self._nlist = [bn.num_batches_tracked for bn in self._bns()]
        # every view's expected address, computed once: _flat_ok compares data_ptr() only
        base, o, ptrs = flat.data_ptr(), 0, []
        for q in params:
            ptrs.append(base + 4 * o)
            o += q.numel()
        b = bflat.data_ptr()
        bptrs, o = [], 0
        for t in self._blist:
            bptrs.append(b + 4 * o)
            o += t.numel()
        self._pexpect = list(zip(params, ptrs))
        self._bexpect = list(zip(self._blist, bptrs))
        self._nexpect = [(t, nflat.data_ptr() + 8 * i) for i, t in enumerate(self._nlist) if t is not None]
        self._shape_cache = None

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        if all(p.dtype == torch.float32 for p in self.parameters()):
            self._flatten()
        return self

    def _flat_ok(self) -> bool:
        """Every parameter / BN buffer still a view of the flat buffers (a caller may rebind
        ``p.data``, assign a new Parameter or replace a buffer)."""
        for (mod, name), p in zip(self._pslots, self._plist):
            if mod._parameters.get(name) is not p:
                return False
        bns = self._bns()
        for i, bn in enumerate(bns):
            if bn.running_mean is not self._blist[2 * i] or bn.running_var is not self._blist[2 * i + 1] \
                    or bn.num_batches_tracked is not self._nlist[i]:
                return False
        for p, ptr in self._pexpect:
            if p.data_ptr() != ptr or not p.is_contiguous():
                return False
        for t, ptr in self._bexpect:
            if t.data_ptr() != ptr:
                return False
        for t, ptr in self._nexpect:
            if t.data_ptr() != ptr:
                return False
        return True

    def flat_views(self):
        """(flat parameters, flat BN buffers, num_batches_tracked buffer) after ONE layout check (a
        fused step needs all three; the check is the larger part of its host time)."""
        if not self._flat_ok():
            self._flatten()
        return self._flat, self._bn_flat, self._nbt_flat

    def flat_parameters(self) -> torch.Tensor:
        if not self._flat_ok():
            self._flatten()
        return self._flat

    def flat_bn_buffers(self) -> torch.Tensor:
        if not self._flat_ok():
            self._flatten()
        return self._bn_flat

    def flat_num_batches_tracked(self) -> torch.Tensor:
        """int64[3] device buffer behind the three BatchNorm2d.num_batches_tracked counters."""
        if not self._flat_ok():
            self._flatten()
        return self._nbt_flat

    @property
    def shape(self) -> Shape:
        bn = self.temporal[1]
        if bn.momentum is None:
            raise NotImplementedError("BatchNorm momentum=None (cumulative average) is not supported")
        key = (float(self.aggregation[3].p), float(bn.eps), float(bn.momentum))
        if self._shape_cache is None or self._shape_cache[0] != key:
            self._shape_cache = (key, Shape(C=self.C, T=self.T, F1=self.F1, D=self.D, K1=self.K1,
                                            p=key[0], eps=key[1], momentum=key[2]))
        return self._shape_cache[1]

    # -- dropout control (test hook) ------------------------------------------------------------
    def set_dropout_masks(self, m2, m3):
        """Inject keep-masks ([B,F2,T//4], [B,F2,T//128] uint8, 1 = keep) for the train-mode
        forward/backward, or ``None`` to return to the on-device generator."""
        self._masks = None if m2 is None else (m2.to(torch.uint8).contiguous(),
                                               m3.to(torch.uint8).contiguous())

    def next_dropout_key(self):
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._rng_offset += 1
        return seed, self._rng_offset

    # -- forward -------------------------------------------------------------------------------
    def forward(self, x):
        require_device(x, "EEGNet input")
        if x.dtype == torch.bfloat16 and not self.training:
            # bf16 batched inference: bf16 MFMA operands, fp32 accumulation
            if x.dim() != 3 or x.shape[1] != self.C or x.shape[2] != self.T:
                raise RuntimeError(f"expected input [B,{self.C},{self.T}], got {list(x.shape)}")
            with torch.no_grad():
                return ops.forward_eval_bf16(self.shape, self.flat_parameters(), self._bn_flat, x)
        if x.dtype != torch.float32:
            raise RuntimeError(f"EEGNet expects float32 input (got {x.dtype}; bfloat16 is accepted in "
                               f"eval mode); the reference casts with signals.float() (model.py:137)")
        if x.dim() != 3 or x.shape[1] != self.C or x.shape[2] != self.T:
            raise RuntimeError(f"expected input [B,{self.C},{self.T}], got {list(x.shape)}")
        if x.requires_grad:
            raise NotImplementedError("gradients with respect to the EEG input are not provided")
        x = x.contiguous()
        flat = self.flat_parameters()
        require_device(flat, "EEGNet parameters")
        shape = self.shape
        params = list(self.parameters())
        if self.training:
            seed, offset = self.next_dropout_key()
            masks = self._masks
            if masks is not None and masks[0].shape[0] != x.shape[0]:
                raise RuntimeError("injected dropout masks do not match the batch size")
            return _TrainFn.apply(x, self, shape, seed, offset, masks, *params)
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _EvalFn.apply(x, self, shape, *params)
        return ops.forward_eval(shape, flat, self._bn_flat, x)


class _TrainFn(torch.autograd.Function):
    """Train-mode EEGNet step as one autograd node: forward = passes A,B,C of the HIP pipeline,
    backward(dlogits) = passes C,D,E + finalizes (grads already clamped as model.py:44,84)."""

    @staticmethod
    def forward(ctx, x, mod, shape, seed, offset, masks, *params):
        ws = ops.new_workspace(shape, x.shape[0], x.device)
        flat = mod.flat_parameters().clone()
        logits = ops.forward_train(shape, flat, mod.flat_bn_buffers(), x, ws, seed, offset,
                                   masks=masks, nbt=mod.flat_num_batches_tracked())
        ctx.shape, ctx.seed, ctx.offset, ctx.masks = shape, seed, offset, masks
        ctx.param_shapes = [p.shape for p in params]
        ctx.save_for_backward(x, ws, flat)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        x, ws, flat = ctx.saved_tensors
        g = ops.backward(ctx.shape, flat, x, ws, ctx.seed, ctx.offset,
                         dlogits=dlogits.contiguous().float(), masks=ctx.masks)
        out, o = [], 0
        for s in ctx.param_shapes:
            k = 1
            for d in s:
                k *= d
            out.append(g[o:o + k].view(s))
            o += k
        return (None, None, None, None, None, None, *out)


class _EvalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mod, shape, *params):
        return ops.forward_eval(shape, mod.flat_parameters(), mod.flat_bn_buffers(), x)

    @staticmethod
    def backward(ctx, dlogits):
        raise NotImplementedError(
            "backward through an eval-mode EEGNet forward is not provided; call model.train() "
            "for a differentiable forward")


# ----------------------------------------------------------------------------------------------
# train / evaluate_model  (model.py:101-227)
# ----------------------------------------------------------------------------------------------
def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device: the MI355X EEGNet build runs on an AMD GPU only")
    return "cuda"


def _fusable(model, optimizer, loss_fn) -> bool:
    if not isinstance(model, EEGNet) or type(optimizer) is not torch.optim.Adam:
        return False
    if type(loss_fn) is not nn.CrossEntropyLoss:
        return False
    if loss_fn.weight is not None or loss_fn.reduction != "mean" or loss_fn.label_smoothing != 0.0:
        return False
    if len(optimizer.param_groups) != 1:
        return False
    grp = optimizer.param_groups[0]
    if [id(p) for p in grp["params"]] != [id(p) for p in model.parameters()]:
        return False
    if grp["weight_decay"] != 0 or grp["amsgrad"] or grp.get("maximize", False):
        return False
    if isinstance(grp["lr"], torch.Tensor) or grp.get("differentiable", False):
        return False
    return True


class FusedAdamState:
    """Device-side Adam state for the fused step, synchronised with a torch.optim.Adam."""

    def __init__(self, model: EEGNet, optimizer=None):
        flat = model.flat_parameters()
        n = flat.numel()
        self.state = torch.zeros(2 * n, dtype=torch.float32, device=flat.device)
        self.step = torch.zeros(1, dtype=torch.int32, device=flat.device)
        self.grads = torch.zeros(n, dtype=torch.float32, device=flat.device)
        if optimizer is not None:
            self.load_from(model, optimizer)

    def load_from(self, model, optimizer):
        n = model.flat_parameters().numel()
        o = 0
        steps = set()
        for p in model.parameters():
            st = optimizer.state.get(p, {})
            k = p.numel()
            if "exp_avg" in st:
                self.state[o:o + k].copy_(st["exp_avg"].reshape(-1))
                self.state[n + o:n + o + k].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(st["step"]))
            o += k
        if len(steps) > 1:
            raise RuntimeError("inconsistent Adam step counts across parameters")
        self.step.fill_(steps.pop() if steps else 0)

    def store_to(self, model, optimizer):
        n = model.flat_parameters().numel()
        step = int(self.step.item())
        o = 0
        for p in model.parameters():
            k = p.numel()
            st = optimizer.state[p]
            st["step"] = torch.tensor(float(step))
            st["exp_avg"] = self.state[o:o + k].view(p.shape).clone()
            st["exp_avg_sq"] = self.state[n + o:n + o + k].view(p.shape).clone()
            p.grad = self.grads[o:o + k].view(p.shape).clone()
            o += k


class FusedTrainer:
    """Whole hot-loop iteration (model.py:141-148) as one device sequence per batch."""

    def __init__(self, model: EEGNet, lr=1e-3, betas=(0.9, 0.999), eps=1e-7, optimizer=None):
        self.model = model
        self.lr, self.betas, self.eps = lr, betas, eps
        self.adam = FusedAdamState(model, optimizer)
        dev = model.flat_parameters().device
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self._ws = {}

    def workspace(self, B):
        ws = self._ws.get(B)
        if ws is None:
            ws = ops.new_workspace(self.model.shape, B, self.model.flat_parameters().device)
            self._ws[B] = ws
        return ws

    def step(self, x, y, logits=None):
        m = self.model
        seed, offset = m.next_dropout_key()
        flat, bn_flat, nbt = m.flat_views()
        ops.train_step(m.shape, flat, bn_flat, x, y, seed, offset,
                       self.adam.grads, self.adam.state, self.adam.step, self.workspace(x.shape[0]),
                       self.loss, logits=logits, lr=self.lr, betas=self.betas, eps=self.eps,
                       nbt=nbt)
        return self.loss


def train(model, optimizer, loss_fn, train_loader, val_loader, nepochs=500, *, true_best=False,
          fused=None):
    """Train and validate every epoch (model.py:101-189).

    Returns (best_state_dict, train_losses, val_losses, val_accuracies).  As in the reference the
    "best" state dict is a shallow copy of the live state, i.e. the final weights;
    ``true_best=True`` snapshots the best-validation weights instead.
    """
    device = _device()
    logger.info(f"Training on {device} device")
    model = model.to(device)
    use_fused = _fusable(model, optimizer, loss_fn) if fused is None else fused
    trainer = None
    if use_fused:
        grp = optimizer.param_groups[0]
        trainer = FusedTrainer(model, lr=grp["lr"], betas=grp["betas"], eps=grp["eps"],
                               optimizer=optimizer)

    train_losses, val_losses, val_accuracies = [], [], []
    best_model = model.state_dict()
    best_val_acc = 0
    for e in range(1, nepochs + 1):
        model.train()
        run_loss = torch.zeros((), dtype=torch.float64, device=device)
        n_train = 0
        for signals, labels in train_loader:
            signals = signals.float().to(device, non_blocking=True)
            labels = labels.to(device, non_blocking=True)
            if trainer is not None:
                run_loss += trainer.step(signals, labels)[0]
            else:
                preds = model(signals)
                loss = loss_fn(preds, labels)
                run_loss += loss.detach()
                optimizer.zero_grad()
                loss.backward()
                optimizer.step()
            n_train += 1

        model.eval()
        run_val = torch.zeros((), dtype=torch.float64, device=device)
        correct = torch.zeros((), dtype=torch.int64, device=device)
        total = 0
        n_val = 0
        with torch.no_grad():
            for signals, labels in val_loader:
                signals = signals.float().to(device, non_blocking=True)
                labels = labels.to(device, non_blocking=True)
                preds = model(signals)
                run_val += loss_fn(preds, labels)
                correct += (torch.argmax(preds, dim=1) == labels).sum()
                total += labels.size(0)
                n_val += 1

        epoch_train_loss = float(run_loss.item()) / max(n_train, 1)
        epoch_val_loss = float(run_val.item()) / max(n_val, 1)
        epoch_val_acc = 100 * int(correct.item()) / total
        train_losses.append(epoch_train_loss)
        val_losses.append(epoch_val_loss)
        val_accuracies.append(epoch_val_acc)
        if epoch_val_acc > best_val_acc:
            best_val_acc = epoch_val_acc
            if true_best:
                best_model = {k: v.detach().clone() for k, v in model.state_dict().items()}
            else:
                best_model = model.state_dict().copy()
        if e == 1 or e % 50 == 0 or e == nepochs:
            logger.info(f"Epoch: {e}/{nepochs}.. Train Loss: {epoch_train_loss:.3f}.. "
                        f"Val Loss: {epoch_val_loss:.3f}.. Val Acc: {epoch_val_acc:.2f}%..")
    if trainer is not None:
        trainer.adam.store_to(model, optimizer)
    return best_model, train_losses, val_losses, val_accuracies


def evaluate_model(model, test_loader) -> float:
    """Test accuracy in percent (model.py:191-227).  Like the reference it does not call
    ``model.eval()``: the caller's mode is used."""
    device = _device()
    logger.info(f"Testing on {device} device")
    model = model.to(device)
    correct = torch.zeros((), dtype=torch.int64, device=device)
    total = 0
    with torch.no_grad():
        for signals, labels in test_loader:
            signals = signals.float().to(device, non_blocking=True)
            labels = labels.to(device, non_blocking=True)
            preds = model(signals)
            correct += (torch.argmax(preds, dim=1) == labels).sum()
            total += labels.size(0)
    return 100 * int(correct.item()) / total
