"""Per-kernel VGPR / AGPR / SGPR / spill / occupancy of libeegnet_hip (hipcc resource remarks).

    python tools/resource_usage.py [substring-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
       "-fno-slp-vectorize", "-Wno-unused-result", "-Wno-unused-value", "-I", os.path.join(ROOT, "include"),
       "-o", "/tmp/_ru.so", os.path.join(ROOT, "eegnetreplication_amd", "csrc", "eegnet_kernels.hip"),
       "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("EXTRA", "").split() + (["-DEEGNET_TRACE"] if os.environ.get("TRACE") else [])
out = subprocess.run(cmd, capture_output=True, text=True).stderr
filt = sys.argv[1] if len(sys.argv) > 1 else "ILi32ELi22ELi256E"
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([\w \[\]/]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if filt not in k:
        continue
    name = re.sub(r"_ZN3eeg\d+", "", k)[:34]
    g = lambda key: v.get(key, "?")
    print(f"{name:34s} VGPR {g('VGPRs'):>4} AGPR {g('AGPRs'):>4} SGPR {g('TotalSGPRs'):>4} "
          f"vspill {g('VGPRs Spill'):>4} sspill {g('SGPRs Spill'):>3} scratch {g('ScratchSize [bytes/lane]'):>4} "
          f"occ {g('Occupancy [waves/SIMD]')}")
