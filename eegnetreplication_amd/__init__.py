"""MI355X-native EEGNet train/infer step (drop-in for PraKesEy/EEGNetReplication's hot path).

Public surface mirrors ``eegnet_repl.model``: ``EEGNet``, ``train``, ``evaluate_model``.
The compute runs in ``libeegnet_hip.so`` (hand-written gfx950 HIP kernels, C-ABI in
``include/eegnet_abi.h``).
"""

from .model import EEGNet, FusedTrainer, evaluate_model, train  # noqa: F401
from .folds import FoldBatch  # noqa: F401
from .ops import Shape  # noqa: F401

__all__ = ["EEGNet", "FoldBatch", "FusedTrainer", "Shape", "evaluate_model", "train"]
