"""Fold-batched training: k independent EEGNet fold runs advanced in lock-step on one GPU
(SURVEY.md 8(f) row 1).

The real protocol trains at batch 64 (train.py:87,229): one fused step is a few microseconds of
work spread over a handful of small launches, so a single fold leaves most of the 256 CUs idle
and the host waits on every launch.  The within-subject protocol has 36 independent runs and the
cross-subject one 90 (train.py:50,73,182,194).  ``FoldBatch`` keeps k of them resident (own
parameters, BN buffers, Adam state and workspace each) and enqueues step j of every fold before
step j+1 of any, each fold on its own HIP stream, so the kernels of different folds overlap on
the device and no host synchronisation happens inside an epoch.

Per fold the arithmetic is ``FusedTrainer.step``'s (model.py:141-148 semantics: forward, CE,
backward with the two clamps, Adam); only the interleaving changes.  Dropout keys are
counter-based per fold -- (fold seed, step counter) -- and a fold-indexed launch splits each fold's
batch over workgroups by the batch size alone, so a fold's trajectory does not depend on how many
other folds run beside it or on which rank it was dealt to (tests/test_gpu_folds.py checks
bit-equality with the same fold run alone).
"""

from __future__ import annotations

import torch

from . import ops
from .dataset import epoch_permutation
from .model import EEGNet, FusedAdamState


class _FoldGraph:
    """One fold's captured epoch: the key it was captured under (every raw device pointer the graph
    holds), static permutation and per-step loss slots, and the graph."""

    def __init__(self, key, perm, losses, graph):
        self.key = key
        self.perm, self.losses, self.graph = perm, losses, graph


class FoldBatch:
    """k independent fold runs on one GPU, one HIP stream each.

    ``graphs=True`` captures each fold's epoch (batch gathers + fused steps) as a hipGraph after
    its first, eager epoch and replays it afterwards: one host call per fold per epoch instead of
    ~10 launches per step.  Dropout keys follow the device Adam step (EEGNET_KEY_FROM_STEP) in both
    modes, so replays draw fresh masks each step and graph and eager runs are bit-identical."""

    def __init__(self, models: list[EEGNet], seeds: list[int], lr=1e-3, betas=(0.9, 0.999),
                 eps=1e-7, graphs=False, fused=None, xstats=True):
        """``fused``: advance all folds with ONE launch per pass (eegnet_train_step_folds, the fold
        index in the grid) instead of one stream per fold.  ``None`` picks it whenever it applies:
        same model shape for every fold, F1*D <= 16, and (per epoch) the same number of trials.
        ``xstats``: fused launches read each batch's parameter-free BN1 statistics from a per-trial
        table of every fold's X (ops.x_stats, computed once per X and refreshed when X changes in
        place) instead of recomputing the lag-Gram from x every step.

        Change detection is PyTorch's version counter (``X._version``), which tracked in-place ops
        bump.  Writes that bypass it -- through ``X.data``, DLPack or another library's view of the
        storage, a ctypes / HIP kernel -- must be followed by ``invalidate_x()``: without it the
        table (and, at 22 x 257, the padded copy the kernels read) keeps the old trials."""
        if len(models) != len(seeds) or not models:
            raise ValueError("need one seed per model and at least one model")
        dev = models[0].flat_parameters().device
        if dev.type != "cuda":
            raise RuntimeError("FoldBatch runs on a HIP device only")
        self.models = models
        self.seeds = [int(s) for s in seeds]
        self.lr, self.betas, self.eps = lr, betas, eps
        self.graphs = graphs
        self.adam = [FusedAdamState(m) for m in models]
        self.streams = [torch.cuda.Stream(device=dev) for _ in models]
        self._ws: list[dict] = [{} for _ in models]
        self._graph: list[_FoldGraph | None] = [None] * len(models)
        same = all(m.shape == models[0].shape for m in models) and models[0].shape.F2 <= 16
        if fused and not same:
            raise ValueError("fused fold launches need the same EEGNet shape (F1*D <= 16) for every fold")
        self.fused = same if fused is None else bool(fused)
        self.xstats = bool(xstats)
        self._fz = None                     # fused-launch state: buffers, fold tables, graph

    def __len__(self):
        return len(self.models)

    def invalidate_x(self):
        """Recompute every fold's padded x copy and per-trial BN1 table from its X at the next epoch
        (for writes to X that PyTorch's version counter does not see: ``X.data``, DLPack, foreign
        kernels).  Same storage: the fold tables and the captured graph stay valid."""
        if self._fz is not None:
            for ent in self._fz["xsrc"].values():
                ent["ver"] = None

    def _workspace(self, k, B):
        ws = self._ws[k].get(B)
        if ws is None:
            ws = ops.new_workspace(self.models[k].shape, B, self.models[k].flat_parameters().device)
            self._ws[k][B] = ws
        return ws

    def _steps(self, k, X, y, perm, losses, batch_size):
        """Enqueue one epoch of fold k on the current stream: the epoch's shuffled copy of X is
        gathered once (one launch, not two per step), batch j is its rows [jB, (j+1)B), and its
        loss lands in losses[j] (no accumulation kernel)."""
        m = self.models[k]
        a = self.adam[k]
        Xp, yp = X.index_select(0, perm), y.index_select(0, perm)
        flat, bn, nbt = m.flat_views()
        for j, i in enumerate(range(0, perm.shape[0], batch_size)):
            xb, yb = Xp[i:i + batch_size], yp[i:i + batch_size]
            ops.train_step(m.shape, flat, bn, xb, yb, self.seeds[k],
                           0, a.grads, a.state, a.step, self._workspace(k, xb.shape[0]),
                           losses[j:j + 1], lr=self.lr, betas=self.betas, eps=self.eps,
                           nbt=nbt, key_from_step=True)

    def _fold_key(self, k, X, y, batch_size):
        """What fold k's captured epoch baked in: its model / Adam buffers (re-created by ``.to()``,
        ``.float()`` or a re-flatten), its X and y, the batch size and workspace."""
        m, a = self.models[k], self.adam[k]
        return (X.shape[0], batch_size, id(X), X.data_ptr(), id(y), y.data_ptr(),
                m.flat_parameters().data_ptr(), m.flat_bn_buffers().data_ptr(),
                m.flat_num_batches_tracked().data_ptr(), a.state.data_ptr(), a.grads.data_ptr(),
                a.step.data_ptr())

    # -- fused launches: all folds in one grid --------------------------------------------------
    def _fused_key(self, data, batch_size):
        """Everything a fold table or the captured graph holds a raw device pointer to: each
        model's flat parameters, BN buffers, counters, Adam state and gradients, and the identity
        of every fold's X and y.  ``.to()`` / ``.cuda()`` / ``.float()`` or a re-flatten re-creates
        the model buffers; a caller may pass new y tensors with the same X."""
        ptrs = []
        for m, a in zip(self.models, self.adam):
            ptrs += [m.flat_parameters().data_ptr(), m.flat_bn_buffers().data_ptr(),
                     m.flat_num_batches_tracked().data_ptr(), a.state.data_ptr(), a.grads.data_ptr(),
                     a.step.data_ptr()]
        return (data[0][0].shape[0], batch_size, tuple(ptrs),
                tuple((id(X), X.data_ptr(), id(y), y.data_ptr()) for X, y in data))

    def _fused_state(self, data, batch_size):
        X0, _ = data[0]
        n = X0.shape[0]
        key = self._fused_key(data, batch_size)
        st = self._fz
        if st is not None and st["key"] == key:
            return st
        dev = X0.device
        K = len(self.models)
        nsteps = (n + batch_size - 1) // batch_size
        # any change: new tables, and the graph (which baked the old pointers in) is dropped.
        # The folds' permutations and loss slots are rows of one [K, n] / [K, nsteps] buffer each:
        # an epoch refreshes every permutation with ONE asynchronous copy from a pinned host buffer
        # (two, alternating: the host fills the next epoch's while the device runs this one) and
        # sums every fold's losses with one kernel.
        perm2 = torch.zeros((K, n), dtype=torch.int64, device=dev)
        loss2 = torch.zeros((K, nsteps), dtype=torch.float32, device=dev)
        st = {"key": key, "src": [d for d in data], "graph": None,
              "perm2": perm2, "perm": list(perm2.unbind(0)),
              "loss2": loss2, "losses": list(loss2.unbind(0)),
              "host": [torch.zeros((K, n), dtype=torch.int64).pin_memory() for _ in range(2)],
              "copied": [None, None], "epoch": 0,
              "tables": {}, "steps": []}
        # x rows at the pitch the kernels load fastest (22 x 257: 260 floats, 16-byte DMA units):
        # one padded copy per distinct X, kept for the life of this state and refreshed in place
        # (same storage: the tables and the graph stay valid) whenever X changes in place
        # (X._version: a caller refilling a preallocated augmentation buffer)
        shape = self.models[0].shape
        xp = shape.x_pitch()
        st["x_pitch"] = 0 if xp == shape.T else xp
        st["xsrc"] = {}

        def xrows(X):
            """(the rows the kernels read, the per-trial BN1 table or None) of X, made once per X"""
            ent = st["xsrc"].get(id(X))
            if ent is None:
                rows = X if ops.x_pitch_of(X) == st["x_pitch"] else ops.pad_x_rows(X, xp)
                stat = ops.x_stats(shape, rows) if self.xstats else None
                ent = st["xsrc"][id(X)] = {"X": X, "rows": rows, "stat": stat, "ver": X._version}
            return ent["rows"], ent["stat"]
        for j, i in enumerate(range(0, n, batch_size)):
            B = min(batch_size, n - i)
            st["steps"].append((i, j, B))
            if B not in st["tables"]:
                ents = []
                for k, m in enumerate(self.models):
                    a = self.adam[k]
                    # x / labels stay unshuffled: the kernels read batch row r as row perm[r]
                    X, y = data[k]
                    rows, stat = xrows(X)
                    ents.append(dict(params=m.flat_parameters(), bn_buffers=m.flat_bn_buffers(),
                                     num_batches_tracked=m.flat_num_batches_tracked(), x=rows, xstat=stat,
                                     labels=y,
                                     perm=st["perm"][k], grads=a.grads, adam_state=a.state, step=a.step,
                                     losses=st["losses"][k], ws=self._workspace(k, B), seed=self.seeds[k]))
                st["tables"][B] = ops.fold_table(ents, dev)
        self._fz = st
        return st

    def _fused_steps(self, st, data):
        shape = self.models[0].shape
        K = len(self.models)
        for i, j, B in st["steps"]:
            ops.train_step_folds(shape, B, st["tables"][B], K, row0=i, slot=j, offset=0, lr=self.lr,
                                 betas=self.betas, eps=self.eps, x_pitch=st["x_pitch"])

    def _refresh_padded(self, st):
        """Every X that changed in place since its padded copy / BN1 table were made: re-copy and
        recompute them in their own storage (the fold tables and the captured graph keep pointing
        there)."""
        shape = self.models[0].shape
        for ent in st["xsrc"].values():
            X = ent["X"]
            if X._version != ent["ver"]:
                with torch.no_grad():
                    if ent["rows"] is not X:
                        ent["rows"].copy_(X)
                    if ent["stat"] is not None:
                        ops.x_stats(shape, ent["rows"], out=ent["stat"])
                ent["ver"] = X._version

    def _epoch_fused(self, data, batch_size, generators):
        n = data[0][0].shape[0]
        st = self._fused_state(data, batch_size)
        self._refresh_padded(st)
        i = st["epoch"] & 1
        st["epoch"] += 1
        if st["copied"][i] is not None:     # this pinned buffer's copy (two epochs ago) has run
            st["copied"][i].synchronize()
        host = st["host"][i]
        for k in range(len(self.models)):
            g = generators[k] if generators is not None else None
            host[k].copy_(epoch_permutation(n, g) if g is not None else torch.arange(n))
        st["perm2"].copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        st["copied"][i] = ev
        if st["graph"] is not None:
            st["graph"].replay()
        else:
            self._fused_steps(st, data)
            if self.graphs:                 # capture for the next epochs (tables / workspaces exist)
                torch.cuda.synchronize()
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr):
                    self._fused_steps(st, data)
                st["graph"] = gr
                # the capture recorded without executing: run this epoch's work once more is NOT
                # wanted -- the eager pass above already trained the epoch
        return list(st["loss2"].sum(dim=1, dtype=torch.float64).unbind(0))

    def epoch(self, data: list[tuple[torch.Tensor, torch.Tensor]], batch_size: int = 64,
              generators: list[torch.Generator] | None = None) -> list[torch.Tensor]:
        """One training epoch of every fold.  ``data[k] = (X_k [N_k,C,T] fp32, y_k [N_k] int64)``,
        device-resident.  Each fold is shuffled by its own generator exactly as
        DataLoader(shuffle=True, generator=g) would (train.py:87; dataset.epoch_permutation) and cut into batches of ``batch_size`` with a short last batch
        (drop_last=False).  Returns per-fold float64 device scalars: the sum of the batch losses
        (the reference's running loss, model.py:150).  Nothing is synchronised."""
        if len(data) != len(self.models):
            raise ValueError("one (X, y) per fold")
        if self.fused and all(X.shape[0] == data[0][0].shape[0] for X, _ in data):
            return self._epoch_fused(data, batch_size, generators)
        cur = torch.cuda.current_stream()
        sums = []
        for k, (X, y) in enumerate(data):
            n = X.shape[0]
            nsteps = (n + batch_size - 1) // batch_size
            g = generators[k] if generators is not None else None
            perm = epoch_permutation(n, g) if g is not None else torch.arange(n)
            s = self.streams[k]
            s.wait_stream(cur)
            st = self._graph[k]
            with torch.cuda.stream(s):
                key = self._fold_key(k, X, y, batch_size)
                if st is not None and st.key == key:
                    st.perm.copy_(perm, non_blocking=True)
                    st.graph.replay()
                    sums.append(st.losses.sum(dtype=torch.float64))
                    continue
                perm_d = perm.to(X.device)
                losses = torch.zeros(nsteps, dtype=torch.float32, device=X.device)
                self._steps(k, X, y, perm_d, losses, batch_size)
                sums.append(losses.sum(dtype=torch.float64))
                if self.graphs:                 # capture for the next epochs (workspaces exist now)
                    gr = torch.cuda.CUDAGraph()
                    sperm = perm_d.clone()
                    slosses = torch.zeros_like(losses)
                    with torch.cuda.graph(gr, stream=s):
                        self._steps(k, X, y, sperm, slosses, batch_size)
                    self._graph[k] = _FoldGraph(key, sperm, slosses, gr)
        for s in self.streams:
            cur.wait_stream(s)
        for t in sums:
            t.record_stream(cur)
        return sums
