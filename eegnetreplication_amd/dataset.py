"""Data feed for the EEGNet step.

* ``BCICI2ADataset`` -- the reference's Dataset type (dataset.py:30-43): ``X[n,C,T]`` float64,
  ``y[n]`` int, ``__getitem__ -> (X[i], int(y[i]))``.
* ``build_dataset_from_preprocessed(src, subject, mode)`` -- same call and error behaviour as the
  reference (dataset.py:239-281).  The reference epochs MNE/braindecode-preprocessed GDF
  recordings; those libraries and the BCI IV-2a files are not available offline, so
  this build loads ``data/processed/A0{subject}{T|E}.npz`` (arrays ``X``, ``y``) and raises
  ``ValueError`` when a file is missing.  Only with ``EEGNET_SYNTHETIC=1`` (CLI ``--synthetic``)
  does it generate a seeded synthetic motor-imagery-like session instead, with the real shape:
  288 trials x 22 channels x 257 samples (128 Hz, 0.5-2.5 s), 4 balanced classes.
* ``DeviceLoader`` -- a device-resident replacement for ``DataLoader(batch_size, shuffle)``: the
  whole split is cast to fp32 and moved to HBM once; batches are index_select views, so the hot
  loop has no per-batch host->device copy (the reference copies every batch, model.py:138).
"""

from __future__ import annotations

import logging
import os
from dataclasses import dataclass

import numpy as np
import torch

logger = logging.getLogger("eegnet_repl")

N_CHANNELS = 22
N_SAMPLES = 257
SFREQ = 128.0
TRIALS_PER_SESSION = 288
# 10-20 positions of the BCI IV-2a montage used for the class-dependent rhythms
C3, CZ, C4 = 7, 9, 11


@dataclass(frozen=True)
class BCICI2ADataset(torch.utils.data.Dataset):
    """dataset.py:30-43: X [n, C, T] float64, y [n] int."""
    X: np.ndarray
    y: np.ndarray

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        return self.X[i], int(self.y[i])


def _pink_noise(rng, shape, T):
    """1/f noise along the last axis (spectral shaping of white noise)."""
    white = rng.standard_normal(shape[:-1] + (T,))
    f = np.fft.rfftfreq(T, d=1.0 / SFREQ)
    scale = 1.0 / np.sqrt(np.maximum(f, 1.0))
    return np.fft.irfft(np.fft.rfft(white, axis=-1) * scale, n=T, axis=-1)


# population / subject parameters of the synthetic sessions: each subject draws its mu and beta
# frequencies, its class-effect strength and its spatial-mixing jitter from these ranges.  Round 4
# (tools/synth_cs_sweep.py preset "v9"; profiles/r4d_sweep.log): a shared class signature -- the same
# C3 / C4 / Cz topography with narrow mu / beta bands and a small per-subject mixing jitter -- so the
# cross-subject protocol learns (68.6 % at 500 epochs, per test subject 38-97 %) and the within-subject
# one is not saturated (86.1 %).  Round 3's ranges (mu 9-11.5 Hz, beta 19-24 Hz, strength 0.25-0.6,
# mix 0.15) left cross-subject at 31 %, near the 25 % chance level.
SYNTH_PARAMS = dict(mu=(9.5, 10.5), beta=(20.0, 22.0), strength=(0.35, 0.65), mix=0.06)


def synthetic_session(subject: int, mode: str = "Train", n=TRIALS_PER_SESSION, C=N_CHANNELS,
                      T=N_SAMPLES) -> BCICI2ADataset:
    """Seeded SMR-like session: classes 0..3 = left hand / right hand / feet /
    tongue.  Hand imagery desynchronises the mu (8-12 Hz) and beta (18-26 Hz) rhythm over the
    contralateral sensorimotor cortex (C4 for left, C3 for right), feet over Cz, tongue weakly
    everywhere; each subject gets its own strength and spatial mixing, on top of 1/f noise.  The
    effect sizes (SYNTH_PARAMS) put per-subject test accuracy in the 40-100 % range (cross-subject
    mean 69 %, within-subject 86 %), so both protocols learn and neither comparison is saturated.
    Trials are standardised per channel like the reference's exponential moving standardisation."""
    sess = 0 if mode == "Train" else 1
    rng = np.random.default_rng(1000 * subject + 17 * sess + 3)
    srng = np.random.default_rng(1000 * subject)          # subject-specific, session-independent
    y = np.repeat(np.arange(4), n // 4)
    y = rng.permutation(np.concatenate([y, rng.integers(0, 4, n - y.size)]))
    t = np.arange(T) / SFREQ
    X = _pink_noise(rng, (n, C, T), T) * 2.0
    sp = SYNTH_PARAMS
    mu_f = srng.uniform(*sp["mu"])
    beta_f = srng.uniform(*sp["beta"])
    strength = srng.uniform(*sp["strength"])
    mix = np.eye(C) + sp["mix"] * srng.standard_normal((C, C))
    for i in range(n):
        ph = rng.uniform(0, 2 * np.pi, 2)
        rhythm = np.sin(2 * np.pi * mu_f * t + ph[0]) + 0.5 * np.sin(2 * np.pi * beta_f * t + ph[1])
        amp = np.full(C, 1.0)
        if y[i] == 0:
            amp[C4] -= 0.8 * strength
            amp[C3] += 0.3 * strength
        elif y[i] == 1:
            amp[C3] -= 0.8 * strength
            amp[C4] += 0.3 * strength
        elif y[i] == 2:
            amp[CZ] -= 0.9 * strength
        else:
            amp *= 1.0 - 0.25 * strength
        X[i] += mix @ (amp[:, None] * rhythm[None, :])
    X = (X - X.mean(axis=2, keepdims=True)) / (X.std(axis=2, keepdims=True) + 1e-6)
    return BCICI2ADataset(X.astype(np.float64), y.astype(np.int64))


def data_dir() -> str:
    return os.environ.get("EEGNET_DATA_DIR", os.path.join(os.getcwd(), "data", "processed"))


SYNTHETIC_ENV = "EEGNET_SYNTHETIC"


def synthetic_enabled() -> bool:
    """Synthetic sessions are opt-in: ``EEGNET_SYNTHETIC=1`` (or the train CLI's ``--synthetic``)."""
    return os.environ.get(SYNTHETIC_ENV, "0").lower() not in ("", "0", "false", "no")


def _load_session(subject: int, mode: str, synthetic: bool) -> BCICI2ADataset:
    tag = mode[0]                                  # 'T' (Train) / 'E' (Eval), dataset.py:262
    path = os.path.join(data_dir(), f"A0{int(subject)}{tag}.npz")
    if os.path.exists(path):
        z = np.load(path, allow_pickle=False)
        return BCICI2ADataset(np.asarray(z["X"], dtype=np.float64), np.asarray(z["y"], dtype=np.int64))
    if synthetic:
        logger.warning(f"{path} not found: using the seeded SYNTHETIC session for subject {subject} "
                       f"({mode}) -- results are not BCI IV-2a results")
        return synthetic_session(int(subject), mode)
    raise ValueError(f"No preprocessed files found in {data_dir()} for subject {subject} ({path}); "
                     f"set {SYNTHETIC_ENV}=1 (CLI: --synthetic) to train on seeded synthetic sessions")


def build_dataset_from_preprocessed(src="kaggle", subject="all", mode="Train",
                                    synthetic: bool | None = None) -> BCICI2ADataset:
    """dataset.py:239-281 call signature and error behaviour.

    Loads the epoched session ``data/processed/A0{subject}{T|E}.npz`` (arrays ``X [288,22,257]``,
    ``y [288]``; the reference's MNE/braindecode epoching is out of scope).
    ``subject='all'`` concatenates subjects 1-9 as the reference globs every file.  A missing file
    raises ``ValueError`` as the reference does (dataset.py:266-267) unless synthetic sessions are
    enabled (``synthetic=True`` or ``EEGNET_SYNTHETIC=1``), which logs a warning per session.
    ``src`` must be 'kaggle' or 'moabb' (dataset.py:252-257); both read the same directory here."""
    if src not in ("kaggle", "moabb"):
        raise ValueError(f"Unknown source: {src}")
    if mode not in ("Train", "Eval"):
        raise ValueError(f"mode must be 'Train' or 'Eval' (got {mode!r})")
    syn = synthetic_enabled() if synthetic is None else bool(synthetic)
    subjects = range(1, 10) if subject == "all" else [int(subject)]
    parts = [_load_session(s, mode, syn) for s in subjects]
    if len(parts) == 1:
        return parts[0]
    return BCICI2ADataset(np.concatenate([p.X for p in parts]), np.concatenate([p.y for p in parts]))


def epoch_permutation(n: int, generator=None) -> torch.Tensor:
    """The trial order ``DataLoader(ds, batch_size, shuffle=True, generator=g)`` produces for one
    epoch (train.py:87), consuming ``g`` exactly as torch does: the iterator draws a base seed
    (``_BaseDataLoaderIter``: ``random_(generator=g)``), then ``RandomSampler`` draws
    ``randperm(n, g)`` and, at exhaustion, one more ``randperm(n, g)`` for the empty remainder."""
    if generator is None:
        return torch.randperm(n)
    torch.empty((), dtype=torch.int64).random_(generator=generator)
    perm = torch.randperm(n, generator=generator)
    torch.randperm(n, generator=generator)
    return perm


class DeviceLoader:
    """``DataLoader(ds, batch_size, shuffle)`` with the split resident in HBM as fp32."""

    def __init__(self, X, y, batch_size=64, shuffle=False, device="cuda", generator=None):
        self.X = torch.as_tensor(np.asarray(X), dtype=torch.float32).to(device).contiguous()
        self.y = torch.as_tensor(np.asarray(y), dtype=torch.int64).to(device)
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.generator = generator

    def __len__(self):
        return (len(self.y) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.y)
        if self.shuffle:
            idx = epoch_permutation(n, self.generator).to(self.X.device)
            for s in range(0, n, self.batch_size):
                j = idx[s:s + self.batch_size]
                yield self.X.index_select(0, j), self.y.index_select(0, j)
        else:
            for s in range(0, n, self.batch_size):
                yield self.X[s:s + self.batch_size], self.y[s:s + self.batch_size]
