"""Benchmark: EEGNet-8,2 train step (forward + CE + backward + clamps + Adam) on synthetic
22ch x 256 trials, batch 4096 per GPU, fp32, HIP kernels (BASELINE.json configs[1] / cfg4).

    python bench.py [--gpus N --steps K --warmup W]            (N=1)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line on rank 0.  `value` = trials/s over all ranks (weak scaling: 4096 trials per
GPU per step; N>1 = data parallel with one RCCL all-reduce per step).  `cfg4_dp` is BASELINE
configs[3] at its own size: global batch 65,536 split over the ranks (strong scaling).  `roofline`
is for the kernel with the largest device time, from HIP events recorded inside the timed region,
priced on SURVEY 8(d)'s algorithmic bytes (x reads) and the implemented FLOPs (max of the two
bounds); `step_roofline` does the same for the whole step.  `cpu_baseline` times the stock-PyTorch
CPU restatement of the reference step (oracle/torch_ref.py) on this host's cores over bounded
samples: the cfg2 step and the reference's real loop (batch 64, 22 x 257).
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_TFLOPS = 157.3      # MI355X FP32 dense (vector == matrix on gfx950), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E spec
REF_FLOP_PER_TRIAL = 6_507_520   # reference formulation, fwd+bwd conv/linear MACx2
ALG_BYTES_PER_TRIAL = 45_056     # x read twice
CFG4_GLOBAL_BATCH = 65536        # BASELINE configs[3]
# untimed steps before the headline's timed region, in all (warm-up W + the event survey + settle steps):
# at the driver's W = 5 (20 timed steps) the timed window otherwise starts ~3 ms into the run, and the
# number swings 16.0-17.2 M trials/s with the GPU's state (profiles/r6zc_warmup.txt); W >= MIN_UNTIMED
# adds none
MIN_UNTIMED = 60


def settle_steps(warmup, survey, prof):
    """Untimed settle steps after the W warm-up and the survey (5 event-bracketed steps + the one that
    fills the event pool), so that at least MIN_UNTIMED untimed steps precede the timed region."""
    return max(0, MIN_UNTIMED - warmup - (survey + 1 if prof else 0))


def kernel_alg_bytes(C=22, T=256, wide=False):
    """SURVEY 8(d)'s algorithmic HBM bytes per trial, attributed to the kernels that need them: x
    is read once for the forward (pass A) and once for the weight gradients (pass E); the labels
    (8 B) by the CE pass C; every intermediate stays on chip or is recomputed (8(d)'s B_alg
    45,056 B at 22 x 256).  The planes a kernel chooses to materialise are NOT algorithmic: they
    show up in its ``impl_bytes`` and in its PMC ``traffic``."""
    xb = C * T * 4
    if wide:
        return {"k_wpass_a": xb, "k_wpass_b": 0, "k_wpass_b2": 0, "k_wpass_c": 8, "k_wpass_d": 0,
                "k_wpass_e": xb}
    return {"k_pass_a": xb, "k_pass_b": 0, "k_pass_c": 8, "k_pass_d": 0, "k_pass_e": xb}


def kernel_algorithmic(C=22, T=256, F1=8, D=2, K1=32):
    """Per-trial algorithmic FLOPs (MAC x 2) and HBM bytes of each pass kernel as implemented
    (DESIGN.md section 4).  Returns {kernel: (flop, bytes)}.  Pass A writes the s and v planes
    ([F2, T] fp32 each) that pass B (v) and pass E (s, v) read instead of recomputing the spatial
    GEMM and the FIR; pass B writes the block-2 q and r planes that passes C (r) and D (q, r) read
    instead of recomputing the depthwise and pointwise convolutions."""
    F2 = F1 * D
    T1, T2 = T // 4, T // 32          # pooled lengths: T/4 (block 1), T/32 (block 2)
    npairs = K1 * (K1 - 1) // 2
    sp = F2 * C * T                  # spatial GEMM
    fir = F2 * T * K1                # one 32-tap FIR over the F2 rows
    b2 = F2 * T1 * 16 + F2 * F2 * T1  # block_2 forward (dw16 + pw)
    xb = C * T * 4
    row = F2 * T1 * 4
    sv = F2 * ((T + 7) // 8 * 8) * 4  # one s / v plane row block of a trial
    return {
        "k_pass_a": (2 * (sp + fir + C * T * K1 + 2 * C * npairs), xb + 2 * sv),
        "k_pass_b": (2 * b2, sv + 5 * row),                        # + q, r planes out
        "k_pass_c": (2 * (2 * 4 * F2 * T2), row + 16),               # r plane in: BN3 + head only
        "k_pass_d": (2 * (2 * F2 * F2 * T1 + 2 * F2 * T1 * 16), 6 * row + 16),   # d2, q, r, E1, E2 in
        "k_pass_e": (2 * (2 * fir + sp), xb + 2 * sv + row),
    }


def kernel_algorithmic_wide(C=64, T=512, F1=16, D=4, K1=32):
    """The same for the F2 > 16 passes (csrc/eegnet_wide.hip, cfg5).  Bytes: x is read from HBM
    once per streaming pass that reads it (the o-chunk workgroups of a trial share it through L2);
    pass A writes the s / v planes, pass B reads v, pass E reads s and v; pass B2 writes the q / r
    planes, pass C reads r, pass D reads q and r."""
    F2 = F1 * D
    T1, T2 = T // 4, T // 32          # pooled lengths: T/4 (block 1), T/32 (block 2)
    npairs = K1 * (K1 - 1) // 2
    sp = F2 * C * T
    fir = F2 * T * K1
    b2 = F2 * T1 * 16 + F2 * F2 * T1
    xb = C * T * 4
    row = F2 * T1 * 4
    sv = F2 * ((T + 7) // 8 * 8) * 4
    return {
        "k_wpass_a": (2 * (sp + fir + C * T * K1 + 2 * C * npairs), xb + 2 * sv),
        "k_wpass_b": (0, sv + 3 * row),
        "k_wpass_b2": (2 * b2, 3 * row),
        "k_wpass_c": (2 * (2 * 4 * F2 * T2), row + 16),
        "k_wpass_d": (2 * (2 * F2 * F2 * T1 + 2 * F2 * T1 * 16), 6 * row + 16),
        "k_wpass_e": (2 * (2 * fir + sp), xb + 2 * sv + row),
    }


# waves per SIMD each kernel's launch configuration admits (workgroup size x workgroups per CU / 4 SIMDs)
LAUNCH_WAVES_PER_SIMD = {"k_pass_a": 4, "k_pass_b": 4, "k_pass_c": 4, "k_pass_d": 4, "k_pass_dr": 4, "k_pass_e": 4,
                         "k_infer": 4, "k_wpass_a": 4, "k_wpass_b": 4, "k_wpass_b2": 2, "k_wpass_c": 2,
                         "k_wpass_d": 2, "k_wpass_e": 4, "k_infer_bf16_cfg5": 4}


def load_util():
    """profiles/pmc_util.json (tools/summarize_profile.py): occupancy and VALU utilisation per kernel
    from the committed rocprofv3 SQ / GRBM counters."""
    path = os.path.join(ROOT, "profiles", "pmc_util.json")
    if os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return {}


def util_fields(name):
    """The roofline line's occupancy / VALU fields for kernel ``name`` (north_star: "achieved HBM GB/s
    and occupancy"), from the committed PMC passes; None where that kernel was not profiled."""
    u = load_util().get(name)
    if not u:
        return {"occupancy": None, "valu_util": None}
    lim = LAUNCH_WAVES_PER_SIMD.get(name)
    occ = {"waves_per_simd": u["waves_per_simd"], "launch_bound_waves_per_simd": lim,
           "frac": round(u["waves_per_simd"] / lim, 4) if lim else None,
           "def": "4 SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs): mean resident waves per SIMD over the launch",
           "source": u["source"]}
    valu = {"busy_simd": u.get("valu_busy_simd"), "of_wave_cycles": u.get("valu_of_wave"),
            "wait_over_active": u.get("wait_over_active"), "lds_bank_conflict": u.get("lds_bank_conflict"),
            "def": "busy_simd = 4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); of_wave_cycles = "
                   "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES", "source": u["source"]}
    return {"occupancy": occ, "valu_util": valu}


def roofline_entry(name, fl, by_alg, by_impl, avg_s, traffic=None):
    """Roofline of one kernel, SURVEY 8(d): t_F = implemented FLOPs / FP32 peak (vector == f32
    MFMA on gfx950), t_B = algorithmic bytes (x reads) / HBM peak; the larger is the bound and
    ``frac`` = that time / the measured average launch.  ``traffic`` = rocprofv3 PMC bytes per launch
    (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md); its ratio to the algorithmic bytes is the
    wasted (materialised-plane) traffic."""
    t_f = fl / (PEAK_FP32_TFLOPS * 1e12)
    t_b = by_alg / (PEAK_HBM_GBS * 1e9)
    e = {"kernel": name, "avg_us": round(avg_s * 1e6, 2), "impl_flop_per_launch": fl,
         "alg_bytes_per_launch": by_alg, "impl_bytes_per_launch": by_impl, "traffic": traffic,
         "traffic_over_alg": round(traffic / by_alg, 3) if traffic and by_alg else None,
         "t_fp32_us": round(t_f * 1e6, 2), "t_hbm_us": round(t_b * 1e6, 2)}
    if t_f >= t_b:
        ach = fl / avg_s / 1e12
        e.update({"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                  "frac": round(ach / PEAK_FP32_TFLOPS, 4),
                  "note": "FP32 roof: fp32 VALU + f32 MFMA share the 157.3 TFLOP/s FP32 peak on gfx950"})
    else:
        ach = by_alg / avg_s / 1e9
        e.update({"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                  "frac": round(ach / PEAK_HBM_GBS, 4)})
    # the same launch against the other roof, for reference
    e["fp32_frac"] = round(t_f / avg_s, 4)
    e["hbm_frac_alg"] = round(t_b / avg_s, 4)
    e.update(util_fields(name))
    return {k: e[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")} | e


def step_roofline(flop_trial, alg_bytes_trial, impl_bytes_trial, trials_per_s, pmc_step_bytes=None,
                  B=None):
    """The whole step against SURVEY 8(d): max(B_alg / HBM, F_impl / FP32) per trial over the
    measured time per trial; plus the step's PMC traffic against B_alg."""
    t_f = flop_trial / (PEAK_FP32_TFLOPS * 1e12)
    t_b = alg_bytes_trial / (PEAK_HBM_GBS * 1e9)
    t = 1.0 / trials_per_s
    out = {"bound": "mfma" if t_f >= t_b else "hbm", "frac": round(max(t_f, t_b) / t, 4),
           "fp32_frac": round(t_f / t, 4), "hbm_frac_alg": round(t_b / t, 4),
           "impl_flop_per_trial": flop_trial, "alg_bytes_per_trial": alg_bytes_trial,
           "impl_bytes_per_trial": impl_bytes_trial}
    if pmc_step_bytes and B:
        out["traffic_per_step"] = pmc_step_bytes
        out["traffic_over_alg"] = round(pmc_step_bytes / (alg_bytes_trial * B), 3)
        out["traffic_gbs"] = round(pmc_step_bytes * trials_per_s / B / 1e9, 1)
    return out


def pmc_step_bytes(pmc, names):
    """Sum of the committed rocprofv3 PMC bytes per launch over one step's pass kernels (measured at
    cfg2 B = 4096 / cfg5 B = 1024), or None if any is missing."""
    tot = 0
    for k in names:
        v = pmc.get(k, {}).get("hbm_bytes_per_launch")
        if v is None:
            return None
        tot += v
    return tot


def timed_steps(trainer, xs, ys, steps, alg, B, barrier, prof=True, survey=5, settle=0):
    """Warm-up done by the caller.  An untimed 5-step survey brackets every kernel with HIP events
    (per-kernel table, dominant kernel); the timed region brackets only the dominant one.  Steps
    rotate over the distinct input buffers ``xs`` (so x comes from HBM, not the 256 MB MALL).
    Returns (seconds, per-kernel survey table, dominant kernel, its (launches, ms) in the timed
    region)."""
    from eegnetreplication_amd import _lib
    table, dom, kern = {}, None, {}
    nx = len(xs)
    if prof:
        _lib.profile_enable(True)
        for i in range(survey):
            trainer.step(xs[i % nx], ys[i % nx])
        torch.cuda.synchronize()
        table = _lib.profile_collect()
        cand = {k: v for k, v in table.items() if k in alg}
        dom = max(cand, key=lambda k: cand[k][1]) if cand else None
        _lib.profile_enable(dom is not None, kernels=[dom] if dom else None)
        trainer.step(xs[0], ys[0])          # fill the event pool outside the timed region
        torch.cuda.synchronize()
        _lib.profile_collect()
    # untimed settle steps (no events) right before the timed region: a short run's number otherwise
    # depends on where the GPU's clocks are after a few ms of work
    if prof and dom is not None:
        _lib.profile_enable(False)
    for i in range(settle):
        trainer.step(xs[i % nx], ys[i % nx])
    if prof and dom is not None:
        _lib.profile_enable(True, kernels=[dom])
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        trainer.step(xs[i % nx], ys[i % nx])
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if prof:
        kern = _lib.profile_collect()
        _lib.profile_enable(False)
    return dt, table, dom, kern.get(dom) if dom else None


def kernel_table(table, alg, B, alg_bytes=None):
    """Per-kernel survey: implemented FLOP rate, implemented bytes rate (x + the planes the kernel
    reads / writes) and the 8(d) algorithmic bytes rate (x reads only)."""
    out = {}
    tot_all = max(sum(v[1] for v in table.values()), 1e-12)
    for name, (cnt, tot) in table.items():
        avg_ms = tot / max(cnt, 1)
        e = {"launches": cnt, "avg_us": round(1e3 * avg_ms, 2), "share": round(tot / tot_all, 4)}
        if name in alg:
            fl, by = alg[name]
            e["impl_tflops"] = round(fl * B / (avg_ms * 1e-3) / 1e12, 2)
            e["impl_gbs"] = round(by * B / (avg_ms * 1e-3) / 1e9, 1)
            if alg_bytes is not None:
                e["alg_gbs"] = round(alg_bytes.get(name, 0) * B / (avg_ms * 1e-3) / 1e9, 1)
        out[name] = e
    return out


def bench_train_cfg5(dev, B, steps, warmup, p=0.5):
    """BASELINE cfg5 training leg: EEGNet-16,4 on synthetic 64ch x 512 trials, fp32, batch B, p=0.5
    with on-device masks, one step = forward + CE + backward + clamps + Adam (eegnet_train_step over
    the o-chunked wide passes).  3 distinct x buffers in rotation."""
    from eegnetreplication_amd import EEGNet, FusedTrainer
    C, T, F1, D = 64, 512, 16, 4
    torch.manual_seed(5)
    model = EEGNet(C, T, F1=F1, D=D, p=p).to(dev).train()
    g = torch.Generator(device=dev).manual_seed(6)
    xs = [torch.randn(B, C, T, device=dev, generator=g) for _ in range(3)]
    ys = [torch.randint(0, 4, (B,), device=dev, generator=g) for _ in range(3)]
    tr = FusedTrainer(model)
    for i in range(warmup):
        tr.step(xs[i % 3], ys[i % 3])
    alg = kernel_algorithmic_wide(C, T, F1, D)
    dt, table, dom, dk = timed_steps(tr, xs, ys, steps, alg, B, lambda: None)
    ab = kernel_alg_bytes(C, T, wide=True)
    pmc = load_pmc() if B == 1024 else {}
    roof = None
    if dom and dk:
        fl, by = alg[dom]
        roof = roofline_entry(dom, fl * B, ab[dom] * B, by * B, dk[1] / dk[0] * 1e-3,
                              pmc.get(dom, {}).get("hbm_bytes_per_launch"))
    fl_step = sum(v[0] for v in alg.values())
    tps = B * steps / dt
    return {"metric": "train trials/sec (fwd+CE+bwd+Adam) EEGNet-16,4 64ch x 512, fp32",
            "value": round(tps, 1), "unit": "trials/s", "batch": B, "steps": steps,
            "ms_per_step": round(1e3 * dt / steps, 4), "loss": round(float(tr.loss.item()), 5),
            "implemented_flop_per_trial": fl_step,
            "step_fp32_frac": round(fl_step * tps / (PEAK_FP32_TFLOPS * 1e12), 4),
            "hbm_fraction": round(2 * C * T * 4 * tps / (PEAK_HBM_GBS * 1e9), 4),
            "roofline": roof,
            "step_roofline": step_roofline(fl_step, 2 * C * T * 4, sum(v[1] for v in alg.values()), tps,
                                           pmc_step_bytes(pmc, list(alg) + ["k_coltail"] * 3), B),
            "kernels": kernel_table(table, alg, B, ab)}


def load_pmc():
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            return json.load(f)
    return {}


def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(B, C, T, steps, threads, real_loop=False):
    """Reference CPU path (stock ATen via oracle/torch_ref.py) on this host; trials/s over the median
    of ``steps`` individually timed steps after one warm-up.  ``real_loop``: the reference's own loop
    body (model.py:136-148) -- float64 batch from the loader, ``signals.float()``, forward, CE,
    ``loss.item()`` (a sync per step), zero_grad, backward, Adam step.  Returns (trials/s at the
    median step, total timed seconds, per-step seconds)."""
    from oracle import torch_ref as tr
    from eegnetreplication_amd import EEGNet
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        state = {k: v.numpy() for k, v in EEGNet(C, T, p=0.5).state_dict().items()}
        ref = tr.TorchRefEEGNet(state, p=0.5)
        opt = tr.make_optimizer(ref)
        rng = np.random.default_rng(1234)
        x = rng.standard_normal((B, C, T))
        x = torch.from_numpy(x) if real_loop else torch.from_numpy(x.astype(np.float32))
        y = torch.from_numpy(np.random.default_rng(1235).integers(0, 4, B))

        def one():
            loss, _ = tr.train_step(ref, opt, x.float() if real_loop else x, y)
            if real_loop:
                loss.item()

        one()                                    # warm-up
        times = []
        for _ in range(steps):
            t0 = time.perf_counter()
            one()
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    return B / float(np.median(times)), float(sum(times)), times


def host_cpu_info():
    """lscpu's model / topology lines (record the host's CPU), or /proc/cpuinfo's
    model name when lscpu is missing."""
    import subprocess
    keep = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)", "NUMA node(s)")
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        info = {}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keep:
                info[k.strip()] = v.strip()
        if info:
            return info
    except (OSError, subprocess.SubprocessError):
        pass
    return {"Model name": cpu_model_name()}


def cpu_baselines(C, T, B, steps):
    """BASELINE.md section 3's CPU leg: the cfg2 step at B on 1 thread, on the box's per-GPU share (16)
    and on every CPU of the affinity mask (torch.set_num_threads(len(os.sched_getaffinity(0)))), each
    ``steps`` individually timed steps after one warm-up, trials/s at the median step; the headline is
    the best leg.  Plus the reference's real loop at batch 64, 22 x 257 (train.py:25,87;
    model.py:136-148) on 1 and 16 threads.  Returns (cpu_baseline dict, real-loop dict)."""
    affinity = len(os.sched_getaffinity(0))
    many = min(16, affinity)
    legs = {}
    for th in dict.fromkeys((1, many, affinity)):          # distinct thread counts, in this order
        v, secs, times = cpu_baseline(B, C, T, steps, th)
        legs[th] = {"value": round(v, 1), "cores": th, "seconds": round(secs, 2), "steps": steps,
                    "median_step_s": round(float(np.median(times)), 3),
                    "step_s": [round(t, 3) for t in times]}
    best = max(legs.values(), key=lambda e: e["value"])
    cpu = {"value": best["value"], "unit": "trials/s", "cores": best["cores"], "kind": "port",
           "sample": f"train steps (fwd+CE+bwd+Adam) of B={B} x {C}x{T}: {steps} individually timed steps "
                     f"per leg after 1 warm-up, trials/s at the median step, legs of "
                     f"{', '.join(str(k) for k in legs)} threads ({affinity} CPUs in the affinity mask, "
                     f"{many} = the box's share per GPU); the best leg is the value; torch "
                     f"{torch.__version__} CPU (stock ATen, oracle/torch_ref.py)",
           "legs": list(legs.values()), "host": host_cpu_info()}
    real = {}
    for th in dict.fromkeys((many, 1)):
        v, secs, _ = cpu_baseline(64, 22, 257, 40, th, real_loop=True)
        real[th] = {"value": round(v, 1), "cores": th, "seconds": round(secs, 2)}
    rb = max(real.values(), key=lambda e: e["value"])
    real_out = {"value": rb["value"], "unit": "trials/s", "cores": rb["cores"], "kind": "port",
                "sample": "40 steps of the reference loop body (float64 batch -> .float(), forward, CE, "
                          ".item(), zero_grad, backward, Adam) at batch 64 x 22x257 after 1 warm-up, "
                          f"trials/s at the median step, best of {many} threads and 1 thread",
                "legs": list(real.values())}
    cpu["real_protocol_b64_t257"] = real_out
    return cpu, real_out


def cpu_eval(B, C, T, F1, D, steps, threads):
    """Reference eval forward on CPU (model.py:156-168 / evaluate_model model.py:191-227 after
    model.eval(): running statistics, no dropout), stock ATen via oracle/torch_ref.py, fp32 (the CPU
    bf16 eval of cfg5 asks for 68.7 GB: SURVEY 6).  Trials/s at the median of ``steps`` timed batches
    after one warm-up; returns (trials/s, seconds)."""
    from oracle import torch_ref as tr
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in tr.init_state(C, T, F1, D).items()}, p=0.5)
        ref.training = False
        x = torch.from_numpy(np.random.default_rng(1234).standard_normal((B, C, T), dtype=np.float32))
        times = []
        with torch.no_grad():
            ref(x)
            for _ in range(steps):
                t0 = time.perf_counter()
                ref(x)
                times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    return B / float(np.median(times)), float(sum(times))


def cpu_train_wide(B, C, T, F1, D, steps, threads):
    """Reference train step (fwd + CE + bwd + clamps + Adam, model.py:141-148) of EEGNet-F1,D on CPU,
    stock ATen via oracle/torch_ref.py; trials/s at the median of ``steps`` timed steps after one
    warm-up; returns (trials/s, seconds)."""
    from oracle import torch_ref as tr
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        torch.manual_seed(0)
        ref = tr.TorchRefEEGNet({k: v.numpy() for k, v in tr.init_state(C, T, F1, D).items()}, p=0.5)
        opt = tr.make_optimizer(ref)
        x = torch.from_numpy(np.random.default_rng(1234).standard_normal((B, C, T), dtype=np.float32))
        y = torch.from_numpy(np.random.default_rng(1235).integers(0, 4, B))
        tr.train_step(ref, opt, x, y)
        times = []
        for _ in range(steps):
            t0 = time.perf_counter()
            tr.train_step(ref, opt, x, y)
            times.append(time.perf_counter() - t0)
    finally:
        torch.set_num_threads(prev)
    return B / float(np.median(times)), float(sum(times))


def cpu_legs(fn, sample, threads_list):
    """Run a CPU baseline at each thread count; the best leg is the value."""
    legs = []
    for th in dict.fromkeys(threads_list):
        v, secs = fn(th)
        legs.append({"value": round(v, 1), "cores": th, "seconds": round(secs, 2)})
    best = max(legs, key=lambda e: e["value"])
    return {"value": best["value"], "unit": "trials/s", "cores": best["cores"], "kind": "port",
            "sample": sample, "legs": legs}


def bench_infer_fp32(dev, B, C, T, steps, warmup, nx=4):
    """fp32 eval forward of EEGNet-8,2 at cfg2's shape (k_infer: the validation loop model.py:156-168
    and evaluate_model model.py:191-227 after train() left the model in eval mode, model.py:151),
    x rotating over ``nx`` distinct batches already in HBM.  Roofline on SURVEY 8(d)'s BN-folded
    inference FLOPs and bytes (x once, logits out)."""
    from eegnetreplication_amd import EEGNet, _lib
    torch.manual_seed(1)
    m = EEGNet(C, T, F1=8, D=2, p=0.5).to(dev).eval()
    with torch.no_grad():
        for name, b in m.named_buffers():
            if name.endswith("running_var"):
                b.uniform_(0.5, 1.5)
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randn(B, C, T, device=dev, generator=g) for _ in range(nx)]
    with torch.no_grad():
        for i in range(warmup):
            m(xs[i % nx])
        _lib.profile_enable(True)
        m(xs[0])
        torch.cuda.synchronize()
        _lib.profile_collect()
        t0 = time.perf_counter()
        for i in range(steps):
            out = m(xs[i % nx])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kern = _lib.profile_collect()
        _lib.profile_enable(False)
    cnt, tot = kern.get("k_infer", (0, 0.0))
    avg_s = tot / max(cnt, 1) * 1e-3
    fl, by = INFER_FLOP(C, T, 16), 4 * C * T + 16
    roof = roofline_entry("k_infer", fl * B, 4 * C * T * B, by * B, avg_s, None) if cnt else None
    return {"metric": "fp32 eval trials/sec EEGNet-8,2 22ch x 256 (k_infer)", "value": round(B * steps / dt, 1),
            "unit": "trials/s", "batch": B, "steps": steps, "x_buffers": nx,
            "finite": bool(torch.isfinite(out).all()), "roofline": roof}


INFER_BF16_BYTES = lambda C, T: 2 * C * T + 16          # bf16 x in, fp32 logits out, per trial
# BN-folded inference FLOPs per trial: spatial GEMM + FIR + dw16 + pw + classifier
INFER_FLOP = lambda C, T, F2, K1=32: 2 * (F2 * C * T + F2 * T * K1 + F2 * (T // 4) * 16
                                          + F2 * F2 * (T // 4) + 4 * F2 * (T // 32))


def bench_infer_bf16(dev, B, C, T, F1, D, steps, warmup):
    """BASELINE cfg5 inference leg: bf16 batched eval forward of EEGNet-F1,D (random init, running
    statistics perturbed so BN is not the identity) on synthetic x ~ N(0,1) already in HBM."""
    from eegnetreplication_amd import EEGNet, _lib
    torch.manual_seed(1)
    m = EEGNet(C, T, F1=F1, D=D, p=0.5).to(dev).eval()
    with torch.no_grad():
        for name, b in m.named_buffers():
            if name.endswith("running_var"):
                b.uniform_(0.5, 1.5)
    x = torch.randn(B, C, T, device=dev, generator=torch.Generator(device=dev).manual_seed(2)).to(torch.bfloat16)
    with torch.no_grad():
        for _ in range(warmup):
            m(x)
        _lib.profile_enable(True)
        m(x)
        torch.cuda.synchronize()
        _lib.profile_collect()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = m(x)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        kern = _lib.profile_collect()
        _lib.profile_enable(False)
    cnt, tot = kern.get("k_infer_bf16", (0, 0.0))
    # the cfg5 shape runs the time-chunked kernel (csrc/eegnet_infer_bf16c.hip), any other the generic one
    kname = "k_infer_bf16_cfg5" if (C, T, F1, D) == (64, 512, 16, 4) else "k_infer_bf16"
    traffic = None                    # HBM bytes per launch from the committed rocprofv3 PMC passes
    if B == 16384:
        traffic = load_pmc().get(kname, {}).get("hbm_bytes_per_launch")
    avg_s = tot / max(cnt, 1) * 1e-3
    by, fl = INFER_BF16_BYTES(C, T), INFER_FLOP(C, T, F1 * D)
    ach = by * B / avg_s / 1e9
    return {
        "metric": f"bf16 batched inference trials/sec EEGNet-{F1},{D} {C}ch x {T}",
        "value": round(B * steps / dt, 1), "unit": "trials/s", "batch": B, "steps": steps,
        "dtype": "bf16 operands, fp32 accumulation", "finite": bool(torch.isfinite(out).all()),
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic, "kernel": kname,
                     "avg_us": round(avg_s * 1e6, 2), "alg_bytes_per_launch": by * B,
                     "alg_tflops": round(fl * B / avg_s / 1e12, 2)},
    }


def bench_folds(dev, n_folds, n_train, epochs, rank=0, world=1, barrier=lambda: None, fused_epochs=8):
    """SURVEY 8(f) row 1 / BASELINE configs[2] leg: the real training protocol (batch 64, 22 x 257
    trials, EEGNet-8,2, p=0.5; train.py:87,229) with n_folds independent cross-subject-sized folds
    (1,440 training trials each, train.py:182-231), dealt to the ranks by lpt_assign (cfg3: fold
    sharding, no communication) and trained on each rank as ONE fold batch (FoldBatch: fold-indexed
    launches, the epoch captured as one hipGraph).  `value` = all folds' trials / the slowest rank's
    time.  At world 1 the same folds per-fold-streamed and one after another (the reference's order)
    are timed beside it.  Synthetic data in HBM.  Runs on every rank; returns rank 0's record."""
    from eegnetreplication_amd import EEGNet, FoldBatch
    from eegnetreplication_amd.distributed import lpt_assign
    C, T = 22, 257
    rng = np.random.default_rng(77)
    X = torch.from_numpy(rng.standard_normal((n_train, C, T), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.integers(0, 4, n_train)).to(dev)
    mine = lpt_assign([1.0] * n_folds, world)[rank] if world > 1 else list(range(n_folds))
    torch.manual_seed(3)
    models = {k: EEGNet(C, T, p=0.5).to(dev).train() for k in mine}

    def run(batches, ep, sync=False):
        gens = {k: torch.Generator().manual_seed(100 + k) for k in mine}
        for fb, ks in batches:                                  # warm-up epoch (workspaces, graphs)
            fb.epoch([(X, y)] * len(ks), 64, [gens[k] for k in ks])
        torch.cuda.synchronize()
        if sync:
            barrier()
        t0 = time.perf_counter()
        for _ in range(ep):
            for fb, ks in batches:
                fb.epoch([(X, y)] * len(ks), 64, [gens[k] for k in ks])
        torch.cuda.synchronize()
        if sync:
            barrier()
        return time.perf_counter() - t0

    # the fold-indexed leg over 8 epochs: an epoch's host work (90 permutations drawn from the folds'
    # generators, ~3 ms) overlaps the previous epoch on the device, except for the first timed one
    dt = run([(FoldBatch([models[k] for k in mine], mine, graphs=True, fused=True), mine)], fused_epochs, sync=True)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    fused = n_folds * n_train * fused_epochs / float(t.item())
    out = {"metric": "real-protocol train trials/sec, batch 64, EEGNet-8,2 22ch x 257",
           "value": round(fused, 1), "unit": "trials/s", "folds": n_folds, "n_gpus": world,
           "folds_per_gpu": len(mine), "train_trials_per_fold": n_train, "epochs": fused_epochs,
           "comparison_epochs": epochs,
           "scaling": "strong (the folds are dealt to the ranks, no communication)",
           "mode": "fold-indexed launches (eegnet_train_step_folds: fold = grid y), epoch captured "
                   "as one hipGraph"}
    if world == 1:
        streams = n_folds * n_train * epochs / run(
            [(FoldBatch([models[k] for k in mine], mine, graphs=True, fused=False), mine)], epochs)
        alone = n_folds * n_train * epochs / run(
            [(FoldBatch([models[k]], [k], fused=False), [k]) for k in mine], epochs)
        out.update({"per_fold_streams_graphed_value": round(streams, 1),
                    "sequential_folds_value": round(alone, 1), "speedup": round(fused / alone, 2)})
        if n_folds == 90:
            out.update(fold_shares(dev, X, y, fused, fused_epochs))
    return out if rank == 0 else None


def fold_shares(dev, X, y, rate90, epochs):
    """cfg3's per-rank operating points on this one GPU: lpt_assign deals the 90 cross-subject folds
    as 45 | 23, 22 | 12, 11 folds per rank at 2 / 4 / 8 GPUs, and each rank trains its share as one
    fold batch (one launch per pass serves every resident fold), so the 8-GPU curve is set by the
    fold launch's rate at 11-12 folds.  Times the fold-indexed, graphed epoch at each share (same data,
    models seeded per fold) and predicts the n-GPU aggregate as 90 folds over the slowest rank's time
    (the largest share; no communication).  Returns {"per_share": ..., "predicted_scaling": ...}."""
    from eegnetreplication_amd import EEGNet, FoldBatch
    from eegnetreplication_amd.distributed import lpt_assign
    n_train = X.shape[0]
    rates = {}
    for k in (11, 12, 22, 23, 45):
        torch.manual_seed(3)
        fb = FoldBatch([EEGNet(22, 257, p=0.5).to(dev).train() for _ in range(k)], list(range(k)),
                       graphs=True, fused=True)
        gens = [torch.Generator().manual_seed(100 + j) for j in range(k)]
        fb.epoch([(X, y)] * k, 64, gens)                      # warm-up (workspaces, graph capture)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(epochs):
            fb.epoch([(X, y)] * k, 64, gens)
        torch.cuda.synchronize()
        rates[k] = k * n_train * epochs / (time.perf_counter() - t0)
        del fb
    rates[90] = rate90
    pred = {}
    for n in (1, 2, 4, 8):
        share = max(len(r) for r in lpt_assign([1.0] * 90, n))
        pred[str(n)] = round(90 * n_train / (share * n_train / rates[share]), 1)
    return {"per_share": {str(k): round(v, 1) for k, v in sorted(rates.items())},
            "predicted_scaling": pred,
            "predicted_note": "n-GPU trials/s = 90 folds x 1,440 trials / the largest rank share's time at the "
                              "per-share rate measured here (lpt_assign: 90 | 45 | 23 | 12 folds on the "
                              "busiest rank at 1 / 2 / 4 / 8 GPUs); no data-path communication"}


def bench_cfg4(dev, rank, world, G, steps, warmup, barrier, nx=2):
    """BASELINE configs[3]: EEGNet-8,2 data parallel at global batch G = 65,536 split over the
    ranks (strong scaling: G / world trials per rank per step), one all-reduce per step
    (DataParallelTrainer; the fused single-device step at world 1).  Runs on every rank; returns
    the rank-0 record (None elsewhere)."""
    from eegnetreplication_amd import EEGNet, FusedTrainer, _lib
    from eegnetreplication_amd.distributed import DataParallelTrainer
    C, T = 22, 256
    B = G // world
    torch.manual_seed(0)
    model = EEGNet(C, T, F1=8, D=2, p=0.5).to(dev).train()
    g = torch.Generator(device=dev).manual_seed(4242 + rank)
    xs = [torch.randn(B, C, T, device=dev, generator=g) for _ in range(nx)]
    ys = [torch.randint(0, 4, (B,), device=dev, generator=g) for _ in range(nx)]
    tr = DataParallelTrainer(model) if world > 1 else FusedTrainer(model)
    for i in range(warmup):
        tr.step(xs[i % nx], ys[i % nx])
    alg = kernel_algorithmic(C, T)
    alg_k, ab_k = alg, kernel_alg_bytes(C, T)
    dt, table, dom, dk = timed_steps(tr, xs, ys, steps, alg_k, B, barrier)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    del xs, ys
    if rank != 0:
        return None
    tps = G * steps / dt
    roof = None
    if dom and dk:
        fl, by = alg_k[dom]
        roof = roofline_entry(dom, fl * B, ab_k[dom] * B, by * B, dk[1] / dk[0] * 1e-3, None)
    flop = sum(v[0] for v in alg.values())
    return {"metric": "train trials/sec (fwd+CE+bwd+Adam) EEGNet-8,2 22ch x 256, data parallel",
            "value": round(tps, 1), "unit": "trials/s", "global_batch": G, "batch_per_gpu": B,
            "n_gpus": world, "steps": steps, "warmup": warmup, "scaling": "strong",
            "ms_per_step": round(1e3 * dt / steps, 4), "loss": round(float(tr.loss.item()), 5),
            "collectives_per_step": 1 if world > 1 else 0,
            "roofline": roof,
            "step_roofline": step_roofline(flop, ALG_BYTES_PER_TRIAL, sum(v[1] for v in alg.values()),
                                           tps / world),
            "hbm_fraction": round(ALG_BYTES_PER_TRIAL * tps / (PEAK_HBM_GBS * 1e9 * world), 4),
            "kernels": kernel_table(table, alg_k, B, ab_k)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--survey", type=int, default=5, help="untimed per-kernel survey steps (HIP events on every launch) before the timed region")
    ap.add_argument("--batch", type=int, default=4096, help="trials per GPU per step")
    ap.add_argument("--C", type=int, default=22)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-infer", action="store_true", help="skip the inference legs (cfg5 bf16, cfg2 fp32)")
    ap.add_argument("--infer-batch", type=int, default=16384)
    ap.add_argument("--no-folds", action="store_true", help="skip the fold-batched real-protocol leg")
    ap.add_argument("--folds", type=int, default=90,
                    help="folds of the real-protocol leg (90: the cross-subject protocol's folds, one fold batch "
                         "at the CLI's --fold-batch 90)")
    ap.add_argument("--nx", type=int, default=4, help="distinct x buffers rotated in the timed region")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the cfg5 EEGNet-16,4 training leg")
    ap.add_argument("--cfg5-batch", type=int, default=1024)
    ap.add_argument("--no-cfg4", action="store_true", help="skip the cfg4 global-batch-65536 leg")
    ap.add_argument("--global-batch", type=int, default=CFG4_GLOBAL_BATCH,
                    help="cfg4 leg: global batch split over the ranks (strong scaling)")
    args = ap.parse_args()

    from eegnetreplication_amd import EEGNet, FusedTrainer, _lib
    from eegnetreplication_amd.distributed import DataParallelTrainer, init_process_group

    rank, world, local = init_process_group()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B, C, T = args.batch, args.C, args.T

    torch.manual_seed(0)
    model = EEGNet(C, T, F1=8, D=2, p=0.5).to(dev).train()
    # NX distinct synthetic batches in rotation (4 x 92 MB at cfg2 > the 256 MB MALL): a training
    # loop reads a new batch every step, so x must come from HBM in the timed region too
    xs, ys = [], []
    for i in range(args.nx):
        rng = np.random.default_rng(1234 + 100 * rank + i)
        xs.append(torch.from_numpy(rng.standard_normal((B, C, T), dtype=np.float32)).to(dev))
        ys.append(torch.from_numpy(np.random.default_rng(1235 + 100 * rank + i).integers(0, 4, B)).to(dev))
    trainer = DataParallelTrainer(model) if world > 1 else FusedTrainer(model)

    def barrier():
        if world > 1:
            dist.barrier()

    prof = not args.no_profile
    for i in range(args.warmup):
        trainer.step(xs[i % args.nx], ys[i % args.nx])
    alg = kernel_algorithmic(C, T)
    alg_k, ab_k = alg, kernel_alg_bytes(C, T)
    # at least MIN_UNTIMED untimed steps in all (warm-up + survey + settle) before the K timed ones
    settle = settle_steps(args.warmup, args.survey, prof)
    dt, table, dom, dk = timed_steps(trainer, xs, ys, args.steps, alg_k, B, barrier, prof, args.survey, settle)
    loss = float(trainer.loss.item())

    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms_per_step = 1e3 * dt / args.steps
    trials_per_s = world * B * args.steps / dt

    del xs, ys
    cfg4 = None
    if not args.no_cfg4:
        cfg4 = bench_cfg4(dev, rank, world, args.global_batch, steps=10, warmup=3, barrier=barrier)
    folds = None
    if not args.no_folds:
        folds = bench_folds(dev, args.folds, 1440, 2, rank, world, barrier)
    if rank == 0:
        ab = kernel_alg_bytes(C, T)
        per_kernel = kernel_table(table, alg_k, B, ab_k)
        pmc = load_pmc() if (B, C, T) == (4096, 22, 256) else {}
        roof = None
        if dom is not None and dk:
            fl, by = alg_k[dom]
            roof = roofline_entry(dom, fl * B, ab_k[dom] * B, by * B, dk[1] / dk[0] * 1e-3,
                                  pmc.get(dom, {}).get("hbm_bytes_per_launch"))
        impl_flop = sum(v[0] for v in alg.values())
        impl_bytes = sum(v[1] for v in alg.values())
        infer = None
        if not args.no_infer:
            infer = bench_infer_bf16(dev, args.infer_batch, 64, 512, 16, 4, steps=20, warmup=3)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu, real_cpu = cpu_baselines(C, T, B, args.cpu_steps)
            if folds is not None:
                folds["cpu_baseline"] = real_cpu
        cfg5 = None
        if not args.no_cfg5:
            cfg5 = bench_train_cfg5(dev, args.cfg5_batch, steps=30, warmup=3)
        eval2 = None
        if not args.no_infer:
            eval2 = bench_infer_fp32(dev, B, C, T, steps=20, warmup=3)
        if not args.no_cpu_baseline and world == 1:
            many = min(16, len(os.sched_getaffinity(0)))
            if eval2 is not None:
                eval2["cpu_baseline"] = cpu_legs(
                    lambda th: cpu_eval(B, C, T, 8, 2, 3, th),
                    f"eval forward (running statistics, no dropout) of B={B} x {C}x{T}, EEGNet-8,2, fp32: 3 timed "
                    f"batches per leg after 1 warm-up, trials/s at the median batch; oracle/torch_ref.py on "
                    f"stock ATen", (1, many))
            if cfg5 is not None:
                cfg5["cpu_baseline"] = cpu_legs(
                    lambda th: cpu_train_wide(256, 64, 512, 16, 4, 2, th),
                    "train steps (fwd+CE+bwd+clamps+Adam) of EEGNet-16,4 at B=256 x 64x512, fp32: 2 timed steps "
                    "per leg after 1 warm-up (a bounded sample of the B=1024 workload: the reference's "
                    "[B,16,64,512] conv1 activations are 0.5 GB per 256 trials), trials/s at the median step; "
                    "oracle/torch_ref.py on stock ATen", (1, many))
            if infer is not None:
                infer["cpu_baseline"] = cpu_legs(
                    lambda th: cpu_eval(512, 64, 512, 16, 4, 2, th),
                    "fp32 eval forward of EEGNet-16,4 at B=512 x 64x512 (BASELINE.md section 3's cfg5 CPU "
                    "workload; the CPU bf16 eval asks for 68.7 GB, SURVEY 6): 2 timed batches per leg after "
                    "1 warm-up, trials/s at the median batch; oracle/torch_ref.py on stock ATen", (1, many))
        out = {
            "metric": "train trials/sec (fwd+bwd) EEGNet-8,2 22ch x 256",
            "value": round(trials_per_s, 1),
            "unit": "trials/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "untimed_steps": args.warmup + (args.survey + 1 if prof else 0) + settle,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (N(0,1) x, uniform labels; random-init EEGNet-8,2)",
            "config": {"workload": f"EEGNet-8,2 train step (fwd+CE+bwd+clamps+Adam), {C}ch x {T}, "
                                   f"batch {B}/GPU, p=0.5, fp32 HIP kernels",
                       "model": "EEGNet-8,2", "global_batch": B * world, "seq_len": T,
                       "channels": C, "parallelism": f"dp{world}"},
            "roofline": roof,
            "step_roofline": step_roofline(impl_flop, ALG_BYTES_PER_TRIAL, impl_bytes, trials_per_s / world,
                                           pmc_step_bytes(pmc, alg), B),
            "cpu_baseline": cpu,
            "hbm_fraction": round(ALG_BYTES_PER_TRIAL * trials_per_s / world / (PEAK_HBM_GBS * 1e9), 4),
            "step_fp32_frac": round(impl_flop * trials_per_s / world / (PEAK_FP32_TFLOPS * 1e12), 4),
            "implemented_flop_per_trial": impl_flop,
            # the step's own HBM traffic (x twice, the s / v planes, the block-2 planes) against peak
            "implemented_bytes_per_trial": impl_bytes,
            "step_hbm_frac": round(impl_bytes * trials_per_s / world / (PEAK_HBM_GBS * 1e9), 4),
            "x_buffers": args.nx,
            "ref_formulation_tflops": round(REF_FLOP_PER_TRIAL * trials_per_s / 1e12, 2),
            "kernels": per_kernel,
            "final_loss": round(loss, 5),
            "cfg4_dp": cfg4,
            "cfg5_train": cfg5,
            "cfg5_infer_bf16": infer,
            "cfg2_eval_fp32": eval2,
            "real_protocol_folds": folds,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
