#!/bin/bash
# fold leg under rocprofv3 kernel trace: per fold-step kernel durations and the gaps between them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fgap
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fgap/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-infer --no-cfg5 --no-cfg4 > gpurun_out/fgap/kt.log 2>&1 || { echo KT_FAIL; tail -20 gpurun_out/fgap/kt.log; exit 1; }
python3 - <<'PY' > gpurun_out/fgap/summary.txt
import csv, glob, re, collections
f = glob.glob("gpurun_out/fgap/kt/**/run_kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = []
for r in rows:
    n = r["Kernel_Name"]
    if re.search(r"eeg::k_pass_\w<32, 22, 257, 16, true", n):
        m = re.search(r"eeg::(k_\w+)", n)
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1)))
ks.sort()
print("fold kernels", len(ks))
# the last 2 * 23 * 5 launches: the timed epochs' steps (23 steps per epoch of 1440 trials at 64)
tail = ks[-(2 * 23 * 5):]
dur = collections.defaultdict(list)
gaps = collections.defaultdict(list)
for i, (s, e, n) in enumerate(tail):
    dur[n].append((e - s) / 1e3)
    if i:
        gaps[n].append((s - tail[i - 1][1]) / 1e3)
span = (tail[-1][1] - tail[0][0]) / 1e3
busy = sum(sum(v) for v in dur.values())
print(f"timed span {span:.1f} us, kernel busy {busy:.1f} us, gaps {span - busy:.1f} us over {len(tail)} launches")
for n in sorted(dur):
    print(f"{n:12s} n {len(dur[n]):4d} avg {sum(dur[n])/len(dur[n]):7.2f} us  gap-before avg {sum(gaps[n])/max(1,len(gaps[n])):6.2f} max {max(gaps[n] or [0]):7.2f}")
trans = collections.defaultdict(list)
for i in range(1, len(tail)):
    trans[tail[i - 1][2] + "->" + tail[i][2]].append((tail[i][0] - tail[i - 1][1]) / 1e3)
for t, v in sorted(trans.items()):
    v.sort()
    print(f"gap {t:22s} n {len(v):4d} median {v[len(v)//2]:8.2f} us  max {v[-1]:9.2f}")
others = [r for r in rows if int(r["Start_Timestamp"]) >= tail[0][0] and int(r["End_Timestamp"]) <= tail[-1][1] and not re.search(r"eeg::k_pass_\w<32, 22, 257, 16, true", r["Kernel_Name"])]
c = collections.Counter(re.sub(r"\(.*", "", r["Kernel_Name"])[:70] for r in others)
print("other kernels inside the timed span:", dict(c))
PY
cat gpurun_out/fgap/summary.txt
rm -f gpurun_out/fgap/kt/*/run_kernel_trace.csv gpurun_out/fgap/kt/run_kernel_trace.csv
