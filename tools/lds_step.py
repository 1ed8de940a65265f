"""A few cfg2 train steps (EEGNet-8,2, 22x256, B = 4096) through the library EEGNET_LIB names: the
workload of tools/lds_probe.sh's counter passes (the knockout builds compute garbage; nothing is
checked)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eegnetreplication_amd import EEGNet, FusedTrainer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = EEGNet(22, 256, p=0.5).to(dev).train()
rng = np.random.default_rng(5)
x = torch.from_numpy(rng.standard_normal((4096, 22, 256), dtype=np.float32)).to(dev)
y = torch.from_numpy(rng.integers(0, 4, 4096)).to(dev)
tr = FusedTrainer(model)
for _ in range(int(os.environ.get("STEPS", 4))):
    tr.step(x, y)
torch.cuda.synchronize()
print("ok", os.environ.get("EEGNET_LIB", "libeegnet_hip.so"))
