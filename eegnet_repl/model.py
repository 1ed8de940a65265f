"""``eegnet_repl.model`` -> the MI355X EEGNet (see eegnetreplication_amd/model.py)."""
from eegnetreplication_amd.model import EEGNet, evaluate_model, train  # noqa: F401
