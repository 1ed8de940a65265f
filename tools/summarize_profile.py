"""Turn a tools_profile.sh run (gpurun_out/prof) into the committed profile summaries:

    profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary, as written
    profiles/<tag>_pmc_summary.json   per-kernel mean of every PMC counter over the dispatches
    profiles/pmc_traffic.json         HBM bytes per launch for the pass kernels (read by bench.py)
    profiles/pmc_util.json            occupancy and VALU utilisation per kernel (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md 'HBM': FETCH_SIZE (KB) is doubled on gfx950 (wide coalesced
reads are tallied at half their bytes); WRITE_SIZE (KB) is taken as-is.
"""
import csv
import json
import os
import re
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.search(r"eeg::(k_\w+)", name)
    return m.group(1) if m else name.split("(")[0][:60]


NCU, NSIMD = 256, 4            # MI355X: CUs, SIMDs per CU


def derive_util(summ, tag):
    """Occupancy and VALU utilisation per launch from the SQ / GRBM counters (MI355X_MICROARCH.md: the
    SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* counters count quad-cycles, summed over the chip; GRBM_GUI_ACTIVE
    is summed over the 8 XCDs, so GRBM_GUI_ACTIVE / 8 is the launch's duration in shader cycles):
      waves_per_simd    = 4 SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs)
                          (mean resident waves per SIMD over the launch, ramp and tail included)
      valu_of_wave      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's life spent issuing VALU)
      valu_busy_simd    = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
                          (share of SIMD cycles with a VALU instruction issuing, MFMA excluded)
      wait_over_active  = SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
      lds_bank_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"""
    util = {}
    for k, cs in summ.items():
        if not k.startswith("k_") or "SQ_WAVE_CYCLES" not in cs or not cs.get("GRBM_GUI_ACTIVE"):
            continue
        cyc = cs["GRBM_GUI_ACTIVE"] / 8.0
        e = {"clock_cycles": round(cyc), "waves": cs.get("SQ_WAVES"),
             "waves_per_simd": round(4.0 * cs["SQ_WAVE_CYCLES"] / (cyc * NCU * NSIMD), 3),
             "source": f"profiles/{tag}_pmc_summary.json"}
        if "SQ_ACTIVE_INST_VALU" in cs:
            e["valu_of_wave"] = round(cs["SQ_ACTIVE_INST_VALU"] / cs["SQ_WAVE_CYCLES"], 4)
            e["valu_busy_simd"] = round(4.0 * cs["SQ_ACTIVE_INST_VALU"] / (cyc * NCU * NSIMD), 4)
        if cs.get("SQ_ACTIVE_INST_ANY") and "SQ_WAIT_INST_ANY" in cs:
            e["wait_over_active"] = round(cs["SQ_WAIT_INST_ANY"] / cs["SQ_ACTIVE_INST_ANY"], 3)
        if cs.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in cs:
            e["lds_bank_conflict"] = round(cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"], 4)
        util[k] = e
    with open(os.path.join(ROOT, "profiles", "pmc_util.json"), "w") as fh:
        json.dump(util, fh, indent=1, sort_keys=True)
    return util


def main(tag, src=os.path.join(ROOT, "gpurun_out", "prof")):
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"),
                os.path.join(out, f"{tag}_kernel_stats.csv"))
    acc = defaultdict(lambda: defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc") or not os.path.exists(f):
            continue
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summ = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    with open(os.path.join(out, f"{tag}_pmc_summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1, sort_keys=True)
    traffic = {}
    for k, cs in summ.items():
        if not k.startswith("k_") or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2.0 * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        traffic[k] = {"hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd),
                      "write_bytes": round(wr), "source": f"profiles/{tag}_pmc_summary.json"}
    with open(os.path.join(out, "pmc_traffic.json"), "w") as fh:
        json.dump(traffic, fh, indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))
    print(json.dumps(derive_util(summ, tag), indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--util-only":     # from a committed summary
        with open(os.path.join(ROOT, "profiles", f"{sys.argv[2]}_pmc_summary.json")) as fh:
            print(json.dumps(derive_util(json.load(fh), sys.argv[2]), indent=1))
    else:
        main(*sys.argv[1:])
