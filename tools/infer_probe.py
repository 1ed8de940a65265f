"""k_infer_bf16_cfg5 time per 16,384-trial launch for the library EEGNET_LIB names (the EEGNET_KX timing
builds of tools/infer_probe.sh): bench.py's cfg5 bf16 inference leg, kernel time only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

r = bench.bench_infer_bf16(torch.device("cuda", 0), 16384, 64, 512, 16, 4, steps=20, warmup=3)
print(os.environ.get("EEGNET_LIB", "libeegnet_hip.so"), "avg_us", r["roofline"]["avg_us"], "frac", r["roofline"]["frac"])
