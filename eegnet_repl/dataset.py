"""``eegnet_repl.dataset`` -> the MI355X data feed (see eegnetreplication_amd/dataset.py)."""
from eegnetreplication_amd.dataset import *  # noqa: F401,F403
