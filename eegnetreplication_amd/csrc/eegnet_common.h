// eegnet_common.h -- geometry, constants and device helpers shared by the EEGNet HIP kernels.
// Part of the single translation unit built from eegnet_kernels.hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

namespace eeg {

// One 1024-thread workgroup (16 waves of 64) per CU for the streaming passes.  A wave owns one
// output row o of the per-trial [F2, T] planes, so row-wise work (FIR taps, reductions) is
// wave-uniform: taps live in SGPRs and per-row partial sums stay in registers across trials.
constexpr int NTH = 1024;
constexpr int NWAVE = NTH / 64;
constexpr int K2 = 16;        // block_2 depthwise taps (model.py:57)
constexpr int NCLS = 4;       // classes (model.py:80)
constexpr int LP2 = 8;        // left pad of d2 / dq rows in LDS (>= 7, multiple of 4)
constexpr int MAXPF = 16;     // prefetch registers per thread: C*T <= NTH*MAXPF floats
constexpr int F2MAX = 16;     // rows per trial plane this build keeps one-per-wave
constexpr int MAXT1Q = 4;     // pooled samples per lane: T1 = T/4 <= 256 (T <= 1024)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// 16-byte LDS accesses as one <4 x float> with alignment 16 (ds_read_b128 / ds_write_b128); a HIP
// float4 struct access gets scalarised into lane-strided ds_read_b32, a 4-way bank conflict
__device__ __forceinline__ floatx4 lds_ld4(const float* p) {
    return *reinterpret_cast<const floatx4*>(__builtin_assume_aligned(p, 16));
}
__device__ __forceinline__ void lds_st4(float* p, floatx4 v) {
    *reinterpret_cast<floatx4*>(__builtin_assume_aligned(p, 16)) = v;
}
typedef float floatx2 __attribute__((ext_vector_type(2)));
// 8-byte LDS read (ds_read_b64; p 8-byte aligned)
__device__ __forceinline__ floatx2 lds_ld2(const float* p) {
    return *reinterpret_cast<const floatx2*>(__builtin_assume_aligned(p, 8));
}
// An octet of a row (8 floats at p, 16-byte aligned; `oc` its index along the row) as two 16-byte
// stores, the halves swapped for octets 4-7 of every 8: ds_write_b128 serves 8 consecutive lanes per
// LDS cycle with banks (a/4) mod 32, so 8 lanes on consecutive octets storing the same half hit every
// bank quad twice (octets oc and oc + 4 are 32 dwords apart) -- a 2-way conflict on every store
__device__ __forceinline__ void lds_st_oct(float* p, int oc, floatx4 lo, floatx4 hi) {
    const bool sw = (oc >> 2) & 1;
    lds_st4(p + (sw ? 4 : 0), sw ? hi : lo);
    lds_st4(p + (sw ? 0 : 4), sw ? lo : hi);
}

// ------------------------------------------------------------------------------------------------
// Geometry shared by host and device (passed by value).  All LDS carve sizes come from the host.
// ------------------------------------------------------------------------------------------------
struct Geo {
    int B, C, T, F1, D, F2, K1, P, R;
    int T1, T2, NF;
    int LP, RS;          // x / s / dy / e rows in LDS: left pad, row stride (floats, RS/4 odd)
    int TQ, NT16;        // ceil(T/4) quads, ceil(T/16) MFMA column tiles
    int RS2;             // block_2 rows (d2 / q / dq) stride
    int RSW;             // per-wave block-2 rows of passes C / D (row_stride_b2)
    int nwC, nwD;        // trial streams (waves) per workgroup of passes C / D
    int CK, NCT, NKG;    // C padded to 4, ceil(C/16), ceil(T/16) k-groups of the dws GEMM
    int nH, nTl, nedge;  // lag-Gram edge terms: head pairs R(R+1)/2, tail pairs P(P+1)/2, + R + P sums
    float p, scale, eps, mom;
    int drop;
    int noclamp;         // skip the model.py:44/84 clamps (data-parallel: clamp after all-reduce)
    unsigned long long key;
    unsigned key0, key1;  // per-layer 32-bit dropout keys (derived from key)
    unsigned pthr;        // dropout threshold p * 2^24
    // graph-replayable keys (EEGNET_KEY_FROM_STEP): key = mix(kseed, koff + *keystep), read on device
    const int32_t* keystep;
    unsigned long long kseed, koff;
    // flat parameter offsets (named_parameters order)
    int o_w1, o_g1, o_b1, o_ws, o_g2, o_b2, o_w2, o_W3, o_g3, o_b3, o_Wfc, o_bfc, nparam;
    // partial-row lengths of the five passes and the (common) workgroup count
    int nA, nB, nC, nD, nE;
    int QR;              // rows of pass E's lag correlation Q in its partial row: F1 when every wave's
                         // rows share one temporal group (narrow path, D = 2: summed before publishing), else F2
    int grid;            // workgroups of passes C, D and the eval forward
    int gridS;           // workgroups of the streaming passes A, B, D (k_pass_dr), E (two per CU)
    int gridA, gridE;    // passes A and E: gridS, or their own trials-per-workgroup in fold launches
    // LDS (floats)
    int ldsA, ldsB, ldsC, ldsD, ldsE, ldsI;
    // optional timeline instrumentation (eegnet_trace_enable): [pass][workgroup][TR_SLOTS] stamps
    unsigned long long* trace;
    // F2 > 16 (eegnet_wide.hip): o-chunks of 16 rows, Gram electrode slice per chunk, block-2 rows
    // padded to F2P (32 / 64), block-2 row stride; LDS (floats) of the wide kernels
    int wide, NOC, CPC, F2P, RB, gridB2;
    int gridW2;          // wide passes B2 and C (whole-job launches): two workgroups per CU at cfg5
    int splitC, splitD, splitE;   // wide passes whose reduction + finalize run in k_coltail (wide rows)
    int ldsWA, ldsWB, ldsWB2, ldsWC, ldsWD, ldsWE, ldsWI;
    // batch the statistics and the CE mean are normalised by: B, or the global batch of a data-parallel
    // step with synchronised BatchNorm (eegnet_train_stage), whose per-pass sums are all-reduced
    int Bn;
    int defer;           // the reduction's winner leaves the pass's sums in part2 row 0; no finalize
    int XP;              // x row pitch (floats between channel rows; T unless eegnet_dims.x_pitch)
};

// Compile-time cfg5 geometry (EEGNet-16,4 at 64ch x 512, K1 = 32): the shape fields make_geo computes
// for those dims (everything but B, the grids and the run-time keys / pointers).  The host launches
// the SPEC instantiations of the wide kernels only when the run-time geometry matches these field for
// field (eegnet_host.hip same_shape_w5), so a specialisation cannot disagree with the generic path;
// with the bounds, strides and offsets constant the kernels fold their index arithmetic and unroll
// (the bf16 eval kernel's kGeoCfg5 does the same, eegnet_infer_bf16.hip).
#define EEG_SHAPE_W5(X)                                                                             \
    X(C, 64) X(T, 512) X(F1, 16) X(D, 4) X(F2, 64) X(K1, 32) X(P, 15) X(R, 16) X(T1, 128) X(T2, 16)  \
    X(NF, 1024) X(LP, 16) X(RS, 548) X(TQ, 128) X(NT16, 32) X(RS2, 144) X(RSW, 156) X(CK, 64)       \
    X(NCT, 4) X(NKG, 32) X(nH, 136) X(nTl, 120) X(nedge, 287) X(o_w1, 0) X(o_g1, 512) X(o_b1, 528)   \
    X(o_ws, 544) X(o_g2, 4640) X(o_b2, 4704) X(o_w2, 4768) X(o_W3, 5792) X(o_g3, 9888) X(o_b3, 9952) \
    X(o_Wfc, 10016) X(o_bfc, 14112) X(nparam, 14116) X(nA, 448) X(nB, 128) X(nC, 4229) X(nD, 5248)    \
    X(nE, 6272) X(QR, 64) X(wide, 1) X(NOC, 4) X(CPC, 16) X(F2P, 64) X(RB, 144) X(splitC, 1)         \
    X(splitD, 1) X(splitE, 1) X(ldsWA, 36656) X(ldsWB, 0) X(ldsWB2, 19712) X(ldsWC, 10528)           \
    X(ldsWD, 37952) X(ldsWE, 29504) X(ldsWI, 37760)
__host__ __device__ __forceinline__ void shape_w5(Geo& g) {
#define EEG_SET_(f, v) g.f = v;
    EEG_SHAPE_W5(EEG_SET_)
#undef EEG_SET_
}
template <bool SPEC>
__device__ __forceinline__ Geo geo_w(const Geo& gin) {
    Geo g = gin;
    if constexpr (SPEC) shape_w5(g);
    return g;
}

// timeline stamps: wall clock (100 MHz) at kernel phase boundaries, shader-clock phase sums (loop)
constexpr int TR_SLOTS = 16, TR_MAXWG = 2048;
enum TraceEv { TR_ENTRY = 0, TR_PRO, TR_LOOP, TR_PUB, TR_GRP, TR_TOP, TR_FIN, TR_PH0 = 8 };
// compiled in only with -DEEGNET_TRACE (libeegnet_hip_trace.so, tools/trace_step.py)
#ifdef EEGNET_TRACE
#define TRACE_ON(g_) ((g_).trace != nullptr)
#else
#define TRACE_ON(g_) false
#endif
#define TRACE(g_, pass_, ev_)                                                                    \
    do {                                                                                         \
        if (TRACE_ON(g_) && threadIdx.x == 0)                                                      \
            (g_).trace[((size_t)(pass_) * TR_MAXWG + blockIdx.x) * TR_SLOTS + (ev_)] = wall_clock64(); \
    } while (0)
// contiguous trial range [b0, b1) of this workgroup in a streaming pass: a static, call-invariant
// assignment, so each partial row sums a fixed trial set in a fixed order.  (An uneven split between
// a CU's first and second resident workgroup was measured and does not move the pass's end: the CU
// pair's joint throughput does.)
__device__ __forceinline__ void trial_range(const Geo& g, int& b0, int& b1) {
    const long long w = blockIdx.x, G = gridDim.x;
    b0 = (int)(w * g.B / G);
    b1 = (int)((w + 1) * g.B / G);
}

// fine stamps of the reduction / finalize critical path (row TR_FINE + pass, slot k), thread 0 only
constexpr int TR_FINE = 6;
#define TRACE_FS(g_, pass_, k_)                                                                  \
    do {                                                                                         \
        if (TRACE_ON(g_) && threadIdx.x == 0)                                                      \
            (g_).trace[((size_t)TR_FINE * TR_MAXWG + (pass_)) * TR_SLOTS + (k_)] = wall_clock64(); \
    } while (0)
// per-workgroup prologue stamps of one pass (row TR_FINE + 1, slot k)
#define TRACE_PS(g_, k_)                                                                         \
    do {                                                                                         \
        if (TRACE_ON(g_) && threadIdx.x == 0)                                                      \
            (g_).trace[((size_t)(TR_FINE + 1) * TR_MAXWG + blockIdx.x) * TR_SLOTS + (k_)] = wall_clock64(); \
    } while (0)
#define TRACE_PH(g_, pass_, ph_, t0_)                                                            \
    do {                                                                                         \
        if (TRACE_ON(g_) && threadIdx.x == 0) {                                                  \
            const unsigned long long t1_ = clock64();                                            \
            tr_lds_[ph_] += t1_ - (t0_);                                                         \
            (t0_) = t1_;                                                                         \
        }                                                                                        \
    } while (0)
// loop-end stamp plus the phase sums (kept in a static LDS slot, not registers: tracing must not
// change the register allocation of the kernel it measures)
#define TRACE_LOOP(g_, pass_)                                                                    \
    do {                                                                                         \
        TRACE(g_, pass_, TR_LOOP);                                                               \
        if (TRACE_ON(g_) && threadIdx.x == 0)                                                    \
            for (int ph_ = 0; ph_ < 8; ++ph_)                                                    \
                (g_).trace[((size_t)(pass_) * TR_MAXWG + blockIdx.x) * TR_SLOTS + TR_PH0 + ph_] = tr_lds_[ph_]; \
    } while (0)
#ifdef EEGNET_TRACE
#define TRACE_DECL()                                                                             \
    __shared__ unsigned long long tr_lds_[8];                                                    \
    if (threadIdx.x == 0)                                                                        \
        for (int ph_ = 0; ph_ < 8; ++ph_) tr_lds_[ph_] = 0;                                      \
    unsigned long long tph_ = clock64();                                                         \
    (void)tph_
#else
#define TRACE_DECL() unsigned long long tph_ = 0; unsigned long long* tr_lds_ = nullptr; (void)tph_; (void)tr_lds_
#endif

// coefficient block layout (float, CSTR per field; F1, F2 <= 64)
enum CoefField {
    CF_A1 = 0, CF_C1, CF_INV1, CF_MU1, CF_AL2, CF_BE2, CF_INV2, CF_MU3, CF_INV3,
    CF_A3, CF_B3, CF_C3, CF_AO, CF_BO, CF_CO, CF_W, CF_LOSS, CF_ADAM, CF_COUNT
};
constexpr int CSTR = 64;

enum PassCMode { PC_LOGITS = 1, PC_BWD = 2, PC_CE = 4 };

// In-kernel reduction + finalize (eegnet_finalize.hip): every pass kernel ends with a ticketed
// two-level fp64 reduction of its per-workgroup partial rows; the last workgroup to arrive runs that
// pass's finalize.  Ticket words: NCNT per pass, zeroed by a memset node at the start of every call.
constexpr int KSMAX = 16;       // ws MFMA k-steps: ceil(C / 4), C <= 64
#ifndef EEGNET_NGRPMAX
#define EEGNET_NGRPMAX 16
#endif
constexpr int NGRPMAX = EEGNET_NGRPMAX;   // groups <= NCNT - 1 (ticket words)
constexpr int NCNT = 40;
constexpr int SPLIT_COLS = 2048;  // wide passes with more partial-row columns reduce in k_coltail          // [0, ngrp) group tickets, [NCNT-1] the top-level ticket
constexpr int TK_PASSES = 5;      // ticket blocks: passes A..E, contiguous from pass A's
struct FinArgs {
    double* part2;                // [ngrp][ncols] fp64 group partials
    unsigned* cnt;                // this pass's NCNT ticket words
    double* stats;                // G w1 per filter + window sums S1 (fin1 writes, fin5 reads)
    float* coef;
    float* bn;                    // running statistics (fin1/fin2, when update_running)
    float* grads;
    float* loss;
    int64_t* nbt;                 // BatchNorm num_batches_tracked x3 (fin2 increments; nullable)
    int update_running, ce;
    int tpass;                    // pass index for the timeline stamps
    // Adam (torch.optim.Adam) fused into pass E's finalize when adam_m != nullptr
    float* params;
    float* adam_m;
    float* adam_v;
    int32_t* step;
    float lr, b1, b2, eps;
};

// ticket blocks of the five passes in a workspace
enum { TK_A = 0, TK_B, TK_C, TK_D, TK_E, TK_COUNT };

// Fold-indexed launches (eegnet_train_step_folds): blockIdx.y is the fold; a fold's pointers come
// from its eegnet_fold entry and its workspace regions sit at the same offsets in every workspace.
struct WsOff {
    unsigned long long cnt, partA, partB, partC, partD, partE, sums, stats, coef, d2, E1, E2, dp2, dl, s, v, q3, r3;
};
struct FoldCall {
    const eegnet_fold* folds;     // nullptr: single-model launch (pointers from the kernel arguments)
    long long row0, slot;         // first trial of the batch in every fold's epoch data; loss slot
    unsigned long long koff;      // dropout key offset (key = mix(seed, koff + *step))
    float lr, b1, b2, eps;        // Adam (pass E's finalize)
    WsOff off;
};

// Issue priority paced by progress through the workgroup's trial range.  Two workgroups share a CU in
// passes A, B and E, and the wave arbiter favours the older one: the first-dispatched half of the
// grid finished its trials in 32 µs and the second half in 53 µs (pass E, B = 4096, r3 stamps), so
// each CU ran its last ~20 µs at one workgroup's occupancy.  A workgroup drops a priority level per
// quarter of its range, so the one ahead yields to the one behind.
// cache policy of the step's plane stores (A/B build options): 1 = nontemporal (the default), 0 = plain
// stores.  NT_MID: d2/E1/E2 (pass B, read by D) and dp2 (pass D, read by E); NT_SV: s and v (pass A)
#ifndef EEGNET_NT_MID
#define EEGNET_NT_MID 1
#endif
#ifndef EEGNET_NT_SV
#define EEGNET_NT_SV 1
#endif
template <int NT, typename V>
__device__ __forceinline__ void st_pol(V v, V* p) {
    if constexpr (NT != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}

#ifndef EEGNET_PRIO
#define EEGNET_PRIO 1
#endif
__device__ __forceinline__ void pace_prio(int done, int total) {
    if constexpr (EEGNET_PRIO != 0) {
        switch ((done * 4) / total) {
        case 0: __builtin_amdgcn_s_setprio(3); break;
        case 1: __builtin_amdgcn_s_setprio(2); break;
        case 2: __builtin_amdgcn_s_setprio(1); break;
        default: __builtin_amdgcn_s_setprio(0); break;
        }
    }
}
__device__ __forceinline__ void tail_prio() {       // publish / reduction / finalize: ahead of loops
    if constexpr (EEGNET_PRIO != 0) __builtin_amdgcn_s_setprio(3);
}

// this workgroup's record of a fold-indexed launch, read through the constant address space: the
// pointers loaded from it are then known to be global (as kernel-argument pointers are), so the
// accesses through them compile to global loads / stores instead of flat ones (a flat load also
// counts against lgkmcnt, so every LDS wait would wait for the loads in flight too)
__device__ __forceinline__ eegnet_fold fold_rec(const FoldCall& fc) {
#if defined(__HIP_DEVICE_COMPILE__)
    return ((const __attribute__((address_space(4))) eegnet_fold*)fc.folds)[blockIdx.y];
#else
    return fc.folds[blockIdx.y];                   // (the host pass of a device function)
#endif
}

// batch row bb of a fold-indexed launch in the fold's epoch data: through the fold's epoch permutation
// when it has one (FoldBatch keeps X / y unshuffled, so an epoch needs no gather of the trials), else
// row row0 + bb.  Single-model launches pass perm = nullptr, row0 = 0: row bb.
__device__ __forceinline__ long long fold_row(const int64_t* __restrict__ perm, long long row0, int bb) {
    return perm ? perm[row0 + bb] : row0 + bb;
}

__device__ __forceinline__ FinArgs fold_fin(const FoldCall& fc, const eegnet_fold& f, int tk, int update_running,
                                            int ce, bool nbt, bool adam, int nparam) {
    char* ws = (char*)f.ws;
    FinArgs a;
    a.part2 = (double*)(ws + fc.off.sums);
    a.cnt = (unsigned*)(ws + fc.off.cnt) + tk * NCNT;
    a.stats = (double*)(ws + fc.off.stats);
    a.coef = (float*)(ws + fc.off.coef);
    a.bn = f.bn_buffers;
    a.grads = f.grads;
    a.loss = f.losses ? f.losses + fc.slot : nullptr;
    a.nbt = nbt ? f.num_batches_tracked : nullptr;
    a.update_running = update_running;
    a.ce = ce;
    a.tpass = tk;
    a.params = adam ? f.params : nullptr;
    a.adam_m = adam ? f.adam_state : nullptr;
    a.adam_v = adam ? f.adam_state + nparam : nullptr;
    a.step = adam ? f.step : nullptr;
    a.lr = fc.lr; a.b1 = fc.b1; a.b2 = fc.b2; a.eps = fc.eps;
    return a;
}

// padded-row strides, shared by host (make_geo) and the compile-time-shape kernels
__host__ __device__ constexpr int rup4(int a) { return (a + 3) & ~3; }
__host__ __device__ constexpr int imax(int a, int b) { return a > b ? a : b; }
// row pitch of the s plane [B][F2][s_pitch(T)] (floats): T rounded up to 4, so rows are 16-byte units
__host__ __device__ constexpr int s_pitch(int T) { return (T + 3) & ~3; }

__host__ __device__ constexpr int row_stride(int K1, int T) {
    // rows of x / s / dy / e: [LP zeros | T samples | >= R zeros]; long enough for the last 4-output
    // FIR window, the last 16-column MFMA tile and the last lag-correlation B tile of pass E; RS/4 odd so that column reads of 16 rows (MFMA
    // operands) land in 16 different bank groups
    const int P = (K1 - 1) / 2, R = K1 - 1 - P, LP = (R + 3) & ~3, OFF = LP - P, OFFD = LP - R;
    const int NW = (OFF + K1 + 6) / 4, TQ = (T + 3) / 4, NT16 = (T + 15) / 16;
    const int NW8 = (imax(OFF, OFFD) + K1 + 10) / 4, NO = (T + 7) / 8;     // 8-output windows
    const int NWT = (15 + K1 - 1) / 16 + 1;                               // pass E lag-correlation tiles
    const int rs = rup4(imax(imax(imax(imax(4 * (TQ - 1) + 4 * NW, 8 * (NO - 1) + 4 * NW8), LP + 16 * NT16), LP + T + R),
                             OFF + 16 * (NT16 + NWT - 1)));
    return ((rs / 4) & 1) ? rs : rs + 4;
}
__host__ __device__ constexpr int row_stride2(int T) { return rup4(LP2 + T / 4 + 8); }
// per-wave block-2 rows of passes C / D (T1 = T/4 pooled samples): pads of 7 / 8 on the left and
// room for the last 16-column MFMA group; RSW/4 odd so 16 rows read as float4 columns hit distinct banks
__host__ __device__ constexpr int row_stride_b2(int T1) {
    const int r = rup4(T1 + 24);
    return ((r / 4) & 1) ? r : r + 4;
}

// compile-time row geometry for a temporal kernel length
template <int K1>
struct KG {
    static constexpr int P = (K1 - 1) / 2;          // left 'same' pad (model.py:27)
    static constexpr int R = K1 - 1 - P;            // right pad
    static constexpr int LP = (R + 3) & ~3;         // LDS left pad (>= P, >= R, multiple of 4)
    static constexpr int OFF = LP - P;              // window offset of the forward FIR / Gram
    static constexpr int OFFD = LP - R;             // window offset of the transposed FIR
    static constexpr int NW = (OFF + K1 + 3 + 3) / 4;   // float4s per 4-output window
    static constexpr int NW8 = ((OFF > OFFD ? OFF : OFFD) + K1 + 7 + 3) / 4;   // float4s per 8-output window
    // lag-Gram edge items per thread of an NT-thread workgroup
    template <int NT>
    static constexpr int nei() { return ((R * (R + 1) / 2 + P * (P + 1) / 2 + R + P) + NT - 1) / NT; }
};

// ------------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------------
// ELU (alpha = 1) and its derivative on the hardware exp2 (v_exp_f32): exp(z) = 2^(z log2 e), a
// few ulp for the |z| BatchNorm produces -- against ~12 instructions for libm's expf / expm1f.
// Below 0 the absolute error of exp(z) - 1 is that of exp(z) (~1e-7), far inside the parity bar.
__device__ __forceinline__ float fast_exp(float z) { return __builtin_amdgcn_exp2f(z * 1.4426950408889634f); }
__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : fast_exp(z) - 1.f; }
__device__ __forceinline__ float elu_d(float z) { return z > 0.f ? 1.f : fast_exp(z); }

// Dropout keep factor (model.py:50,74 nn.Dropout: x * mask / (1-p)).  Injected masks win; otherwise a
// counter-based draw: murmur3's 32-bit finalizer of (flat index * golden ratio + per-layer key), top
// 24 bits against p * 2^24.  Identical in forward and backward, a few VALU ops per element.
// splitmix64 finalizer of (seed, offset): the host's mix_key (eegnet_host.hip), restated for keys
// read on the device
__device__ __forceinline__ unsigned long long mix_key_dev(unsigned long long seed, unsigned long long off) {
    unsigned long long z = seed * 0xD1B54A32D192ED03ull + off * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// per-layer 32-bit dropout key of this call, hoisted to kernel entry by the passes that draw masks.
// With keystep set (graph replays) the offset advances with the device Adam step, which only pass
// E's finalize increments -- after every reader of this step has run.
__device__ __forceinline__ unsigned drop_key(const Geo& g, int layer) {
    if (!g.keystep) return layer ? g.key1 : g.key0;
    const unsigned long long k = mix_key_dev(g.kseed, g.koff + (unsigned long long)(*g.keystep));
    return layer ? (unsigned)(k >> 32) ^ 0x5BD1E995u : (unsigned)k;
}
__device__ __forceinline__ unsigned fold_drop_key(const FoldCall& fc, const eegnet_fold& f, int layer) {
    const unsigned long long k = mix_key_dev(f.seed, fc.koff + (unsigned long long)(*f.step));
    return layer ? (unsigned)(k >> 32) ^ 0x5BD1E995u : (unsigned)k;
}
__device__ __forceinline__ float keep_mul(const Geo& g, const uint8_t* __restrict__ mask, unsigned key,
                                          unsigned idx) {
    if (!g.drop) return 1.f;
    if (mask) return mask[idx] ? g.scale : 0.f;
    unsigned h = idx * 0x9E3779B1u + key;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return (h >> 8) >= g.pthr ? g.scale : 0.f;
}

// Drain every outstanding memory operation before a trial loop.  The waitcnt pass merges the
// pre-loop state of register-resident operands (MFMA A fragments, taps) into the loop header and
// then guards their first in-loop use with vmcnt waits -- which, vmcnt being in order, also wait for
// the NEXT trial's x prefetch issued at the top of the iteration.  One explicit drain here resolves
// those operands for good.
__device__ __forceinline__ void drain_prologue_loads() { __builtin_amdgcn_s_waitcnt(0); }

// Batched staging of a small global array into LDS: U unconditional loads per thread (indices
// clamped, so no per-load branch and wait), then the guarded stores.  Callers issue every batch they
// need before the first store, so a finalize pays one global round trip instead of one per element
// group.  Elements beyond U * blockDim.x (large non-default geometries) are copied by store() itself.
template <int U, typename T>
struct Stage {
    T v[U];
    const T* src;
    __device__ __forceinline__ void load(const T* s, int n) {
        src = s;
        const int nth = blockDim.x, last = n > 0 ? n - 1 : 0;
#pragma unroll
        for (int j = 0; j < U; ++j) v[j] = s[min((int)threadIdx.x + j * nth, last)];
    }
    template <typename D>
    __device__ __forceinline__ void store(D* dst, int n) const {
        const int nth = blockDim.x;
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int i = threadIdx.x + j * nth;
            if (i < n) dst[i] = (D)v[j];
        }
        for (int i = threadIdx.x + U * nth; i < n; i += nth) dst[i] = (D)src[i];
    }
};

// A wave-uniform load through the constant address space: the scalar unit (s_load, counted by
// lgkmcnt), so a prologue's weight / coefficient loads are not queued behind -- vmcnt being in order --
// the first trial's LDS-DMA and plane loads issued before them.  Only for data no workgroup of the
// running kernel writes before every workgroup has passed its prologue (parameters, the previous
// launches' coefficients: the scalar cache is invalidated at every kernel start).
template <typename T>
__device__ __forceinline__ T ldc(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) T*)p;
#else
    return *p;
#endif
}

// a wave-uniform zero the compiler cannot see through: added to a weight-row offset it pins that
// row's scalar loads next to their use (otherwise every row of every table is hoisted into SGPRs and
// spilled)
__device__ __forceinline__ int opaque0() {
    int z = 0;
    asm volatile("" : "+s"(z));
    return z;
}
// the same, ordered after `dep` is computed: chains row r's weight loads behind row r-1's result so
// the compiler cannot hoist every row's loads to the top (asm volatile alone may all move up)
__device__ __forceinline__ int opaque0_after(float dep) {
    int z = 0;
    asm volatile("" : "+s"(z) : "v"(dep));
    return z;
}

// ---- cross-lane reductions: v_permlane32/16_swap halving + DPP within 16-lane rows ----
// (the builtins' second result is mis-compiled by this toolchain -- it returns the first result
// twice -- so the swaps are inline asm; tools/lane_ops_check.hip pins the operand semantics:
// swap32 a.hi <-> b.lo, swap16 a.rows{1,3} <-> b.rows{0,2})
__device__ __forceinline__ void swap32(float& a, float& b) {
    asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    asm("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// every lane gets the sum over its 16-lane row: quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, 8
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x124>(v);
    v += dpp<0x128>(v);
    return v;
}

// N independent sums over each half-wave (lanes 0-31, 32-63) at once (N % 2 == 0): one halving
// swap then 4 DPP steps on N/2 registers.  On return v[j] holds, in lane 0 / 16 / 32 / 48, the sum of
// value j / j + N/2 over half-wave 0 / 0 / 1 / 1 (every lane of a 16-lane row holds the same).
template <int N>
__device__ __forceinline__ void half_reduce(float (&v)[N]) {
    static_assert(N % 2 == 0, "half_reduce: N must be even");
#pragma unroll
    for (int j = 0; j < N / 2; ++j) {
        swap16(v[j], v[j + N / 2]);
        v[j] += v[j + N / 2];
    }
#pragma unroll
    for (int j = 0; j < N / 2; ++j) v[j] = row_sum16(v[j]);
}

// sum over the 64 lanes, result in every lane
__device__ __forceinline__ float wave_sum(float v) {
    float a = v, b = v;
    swap32(a, b);
    v = a + b;
    a = v; b = v;
    swap16(a, b);
    return row_sum16(a + b);
}

// N independent 64-lane sums at once (N % 4 == 0): two halving swaps then 4 DPP steps on N/4
// registers (~2.5 instructions per value instead of 6 dependent shuffles).  On return, lane
// 16*r (r < 4) holds sum[j + r*N/4] in v[j] for j < N/4 (every lane of row r holds the same).
template <int N>
__device__ __forceinline__ void wave_reduce(float (&v)[N]) {
    static_assert(N % 4 == 0, "wave_reduce: N must be a multiple of 4");
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
        swap32(v[i], v[i + N / 2]);
        v[i] += v[i + N / 2];
    }
#pragma unroll
    for (int j = 0; j < N / 4; ++j) {
        swap16(v[j], v[j + N / 4]);
        v[j] += v[j + N / 4];
    }
#pragma unroll
    for (int j = 0; j < N / 4; ++j) v[j] = row_sum16(v[j]);
}

// column c of a workgroup's per-wave partial rows red[w][stride], w < nw <= NWMAX, summed in wave
// order: every row's LDS read issues before the first add (one LDS round trip, not nw)
template <int NWMAX>
__device__ __forceinline__ float wave_rows_sum(const float* red, int nw, int stride, int c) {
    float v[NWMAX];
#pragma unroll
    for (int w = 0; w < NWMAX; ++w) v[w] = red[min(w, nw - 1) * stride + c];
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NWMAX; ++w) a += w < nw ? v[w] : 0.f;
    return a;
}

// order this wave's LDS writes before its later LDS reads (rows a wave owns need no block barrier)
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// NW aligned float4 loads from LDS (p must be 16-byte aligned: row base + multiple of 4 floats)
template <int NW>
__device__ __forceinline__ void lds_window(const float* __restrict__ p, float (&w)[4 * NW]) {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const floatx4 f = lds_ld4(p + 4 * i);
        w[4 * i + 0] = f[0]; w[4 * i + 1] = f[1]; w[4 * i + 2] = f[2]; w[4 * i + 3] = f[3];
    }
}

// 4 outputs of a K-tap correlation from a window: out[i] = sum_k tap[k] * w[OFF + i + k]
template <int K, int OFF, int NWF>
__device__ __forceinline__ void fir4(const float (&w)[NWF], const float (&tap)[K], float (&out)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) a = fmaf(tap[k], w[OFF + i + k], a);
        out[i] = a;
    }
}

// 8 outputs of a K-tap correlation from a window: out[i] = sum_k tap[k] * w[OFF + i + k]; two
// independent 4-output chains per lane -- twice the FMAs per LDS window of fir4
template <int K, int OFF, int NWF>
__device__ __forceinline__ void fir8(const float (&w)[NWF], const float (&tap)[K], float (&out)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = fmaf(tap[k], w[OFF + i + k], out[i]);
}

// ---- x staging: global -> registers (issued a whole trial ahead) -> LDS rows ----
// PF floats per thread cover one trial: C*T <= NTH*PF.
template <int PF, int NT = NTH>
__device__ __forceinline__ void x_prefetch(const float* __restrict__ xb, int C, int T, float (&pf)[PF], int tid) {
    const int n = C * T;
    if ((T & 3) == 0) {
        const float4* src = reinterpret_cast<const float4*>(xb);
#pragma unroll
        for (int j = 0; j < PF / 4; ++j) {
            const int i = tid + NT * j;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (4 * i < n) v = src[i];
            pf[4 * j] = v.x; pf[4 * j + 1] = v.y; pf[4 * j + 2] = v.z; pf[4 * j + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int i = tid + NT * j;
            pf[j] = i < n ? xb[i] : 0.f;
        }
    }
}

template <int PF, int NT = NTH>
__device__ __forceinline__ void x_store(const float (&pf)[PF], int C, int T, int RS, int LP, float* Xs, int tid) {
    const int n = C * T;
    if ((T & 3) == 0) {
        const int TQ = T >> 2;
#pragma unroll
        for (int j = 0; j < PF / 4; ++j) {
            const int i = tid + NT * j;
            if (4 * i < n) {
                const int c = i / TQ, q = i - c * TQ;
                lds_st4(Xs + c * RS + LP + 4 * q, (floatx4){pf[4 * j], pf[4 * j + 1], pf[4 * j + 2], pf[4 * j + 3]});
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            const int i = tid + NT * j;
            if (i < n) {
                const int c = i / T, t = i - c * T;
                Xs[c * RS + LP + t] = pf[j];
            }
        }
    }
}

// spatial A operand (ws, 16 o x 4 c per k-step) kept in registers for the whole workgroup:
// lane l holds ws[o = l&15][c = 4s + (l>>4)] for k-step s (zero outside F2 x C); KS = ceil(C/4)
// EEGNET_LDSX_A = n (counter builds only, wrong results): drop one class of pass A's LDS accesses
// (tools/lds_probe.sh): 1 spatial GEMM operands, 3 lag-Gram windows, 5 s-plane store reads, 6 FIR
// windows, 7 the in-loop x DMA
#ifndef EEGNET_LDSX_A
#define EEGNET_LDSX_A 0
#endif
// the channel of MFMA k-row lk (0-3) in k-step s of the spatial GEMM.  ds_read_b32 serves each
// 32-lane half (lk = 0, 1 | lk = 2, 3) in one cycle over 32 banks: rows c and c + 1 (RS = 4 mod 8
// floats apart) put 16 lanes on overlapping banks, a 2-way conflict on every operand read.  Steps
// 2j, 2j + 1 instead take channels 8j .. 8j + 7 with each half on rows c, c + 4 (4 RS = 16 mod 32:
// disjoint banks).  Odd KS keeps the plain order.
#ifndef EEGNET_SPATIAL_PLAIN
#define EEGNET_SPATIAL_PLAIN 0      // (A/B builds: 1 = the plain channel order)
#endif
template <int KS>
__device__ __forceinline__ int spatial_ch(int s, int lk) {
    if constexpr (KS % 2 == 0 && !EEGNET_SPATIAL_PLAIN) {
        // step part (compile-time: an immediate LDS offset) + lane part (in the base address)
        return (8 * (s >> 1) + 2 * (s & 1)) + ((lk >> 1) + 4 * (lk & 1));
    } else {
        return 4 * s + lk;
    }
}

template <int KS>
__device__ __forceinline__ void load_ws_frag(const float* __restrict__ ws, int C, int F2, float (&aw)[KS],
                                             int lane) {
    const int o = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        const int c = spatial_ch<KS>(s, lk);
        aw[s] = (o < F2 && c < C) ? ws[o * C + c] : 0.f;
    }
}

// s[o,t] = sum_c ws[o,c] x[c,t] on the matrix cores: v_mfma_f32_16x16x4_f32, A = ws (registers),
// B = x tile (4 c x 16 t).  Lane l: A[l&15][spatial_ch(s, l>>4)], B[spatial_ch(s, l>>4)][l&15];
// D[4(l>>4)+r][l&15] (CDNA4 maps).  Exact f32 up to the order of the channel sum.  Wave w computes
// column tiles w, w+16, ...
template <int KS, int NW = NWAVE>
__device__ __forceinline__ void spatial_mfma(const float* Xs, const float (&aw)[KS], float* Ss, int C, int F2,
                                             int NT16, int RS, int LP, int wave, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    int ks = (C + 3) >> 2;
    if constexpr (KS % 2 == 0 && !EEGNET_SPATIAL_PLAIN) ks = (ks + 1) & ~1;   // spatial_ch: steps 2j, 2j + 1 hold 8 channels
    const int cl = spatial_ch<KS>(0, lk);
    const float* xcol = Xs + LP + li + cl * RS;
    for (int n = wave; n < NT16; n += NW) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s < ks) {
                const int c = spatial_ch<KS>(s, lk), cs = c - cl;     // cs: the step's part
#if EEGNET_LDSX_A == 1
                const float b = 0.01f * (c + n);
#else
                const float b = (c < C) ? xcol[cs * RS + 16 * n] : 0.f;
#endif
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(aw[s], b, acc, 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = 4 * lk + r;
            if (o < F2) Ss[o * RS + LP + 16 * n + li] = acc[r];
        }
    }
}

// Static shape of a kernel instantiation: CC/TT/FF = 0 means "runtime value from Geo".  The
// specialised shapes are EEGNet-8,2 (F2 = 16, D = 2); PF = x prefetch floats per thread of an
// NT_-thread workgroup.
#define EEG_DIMS(g) EEG_DIMS_NT(g, NTH)
#define EEG_DIMS_NT(g, NT_)                                                                 \
    const int C = CC ? CC : (g).C;                                                          \
    const int T = TT ? TT : (g).T;                                                          \
    const int F2 = FF ? FF : (g).F2;                                                        \
    const int TQ = (T + 3) >> 2, T1 = T >> 2, T2 = T1 >> 3, NF = F2 * T2;                   \
    const int RS = TT ? row_stride(K1, TT) : (g).RS;                                        \
    const int RS2 = TT ? row_stride2(TT) : (g).RS2;                                         \
    const int NT16 = (T + 15) >> 4, NCT = (C + 15) >> 4;                                    \
    constexpr int LP = KG<K1>::LP;                                                          \
    constexpr int PF = (CC && TT) ? ((CC * TT + (NT_) - 1) / (NT_) + 3) / 4 * 4 : MAXPF * NTH / (NT_); \
    constexpr int KS = CC ? (CC + 3) / 4 : 16;                                              \
    (void)TQ; (void)T1; (void)T2; (void)NF; (void)RS2; (void)NT16; (void)NCT; (void)LP

}  // namespace eeg
