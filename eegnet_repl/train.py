"""``eegnet_repl.train`` -> the MI355X CLI (see eegnetreplication_amd/train.py)."""
from eegnetreplication_amd.train import *  # noqa: F401,F403
from eegnetreplication_amd.train import main

if __name__ == "__main__":
    main()
