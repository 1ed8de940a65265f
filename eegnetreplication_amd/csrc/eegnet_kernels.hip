// eegnet_kernels.hip -- MI355X (gfx950, CDNA4) EEGNet train / infer step behind include/eegnet_abi.h.
//
// Reference being replaced (PraKesEy/EEGNetReplication, /root/reference):
//   EEGNet layers         src/eegnet_repl/model.py:22-84, forward model.py:91-99
//   grad clamps           model.py:43-44 (spatial +-1), 83-84 (classifier +-0.25)
//   CE loss / Adam        train.py:94-103, hot loop model.py:136-148
//
// Algorithm.  The reference materialises the [B,F1,C,T] temporal-conv tensor
// (738 MB at B=4096) and spends 58 % of its step in that conv's weight gradient.  This build never
// forms it.  Everything before the first nonlinearity is linear, so per trial:
//     s[o,t]  = sum_c ws[o,c] x[c,t]                       (spatial first; MFMA f32 16x16x4)
//     v[o,t]  = sum_k w1[o/D,k] s[o,t+k-P]                 (32-tap FIR on 16 rows, not 176)
//     y2[o,t] = a1[g] v[o,t] + c1[g] sum_c ws[o,c]         (BN1 affine folded: a1 = g1/sd1)
// BN1's batch statistics come from the lag-Gram of x (G[k,k'] = sum xpad[t+k] xpad[t+k']) and window
// sums; BN2's from sum v, sum v^2.  Every backward weight-gradient reduction is linear in dy2 and is
// written as per-trial partial sums that finalize kernels combine with the BN constants at the end.
// Five streaming passes over the batch (A..E), each followed by a deterministic fp64 column
// reduction and a one-workgroup finalize:
//   A  x -> Gram/window sums of x, sum v, sum v^2                       (BN1, BN2 statistics)
//   B  x -> v -> BN2 -> ELU -> pool4 -> dropout -> d2, dw16, pw -> sum r, r^2 (BN3 statistics)
//   C  d2 -> block2 -> BN3 -> ELU -> pool8 -> dropout -> FC -> logits [-> CE, dFC, BN3-bwd sums]
//   D  d2 -> block2 bwd (dW3, dw2), dp2, BN2-bwd sums (via pooled ELU' sums E1/E2 stored by B)
//   E  x -> v, dy2 -> dW1 correlation sums, FIR^T(dy2) -> dws GEMM (MFMA)
// All fp32 arithmetic; BN/gradient totals in fp64.  No hipify, no dual paths: gfx950 only.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <string>
#include <algorithm>
#include <vector>
#include <stdarg.h>

#include "../../include/eegnet_abi.h"

namespace eeg {

constexpr int NT = 256;       // threads per workgroup (4 waves of 64)
constexpr int K2 = 16;        // block_2 depthwise taps (model.py:57)
constexpr int NCLS = 4;       // classes (model.py:80)
constexpr int LP2 = 8;        // left pad of d2 / dq rows in LDS (>= 7, multiple of 4)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// Geometry shared by host and device.  All LDS carve offsets are computed once on the host.
// ------------------------------------------------------------------------------------------------
struct Geo {
    int B, C, T, F1, D, F2, K1, P, R;
    int T1, T2, NF;
    int LP, RS;          // x / s / dy / e rows in LDS: left pad, row stride (floats)
    int TQ, NT16;        // ceil(T/4) quads, ceil(T/16) MFMA column tiles
    int nseg, nsegC;     // threads per o-row (FIR ownership), per c-row (Gram ownership)
    int TQ1, RS2;        // block_2 rows: ceil(T1/4), row stride
    int FO, CK, NCT;     // F2 padded to 16, C padded to 4, ceil(C/16)
    int npairs;          // lag-Gram edge pairs K1*(K1-1)/2
    float p, scale, eps, mom;
    int drop;
    int noclamp;          // skip the model.py:44/84 clamps (data-parallel: clamp after all-reduce)
    unsigned long long key;
    // flat parameter offsets (named_parameters order)
    int o_w1, o_g1, o_b1, o_ws, o_g2, o_b2, o_w2, o_W3, o_g3, o_b3, o_Wfc, o_bfc, nparam;
    // partial-row lengths and workgroup counts of the five passes
    int nA, nB, nC, nD, nE;
    int gA, gB, gC, gD, gE;
    // LDS (floats) of the passes
    int ldsA, ldsB, ldsC, ldsD, ldsE, ldsI;
};

// coefficient block layout (float, 64 per field; F1, F2 <= 64)
enum CoefField {
    CF_A1 = 0, CF_C1, CF_INV1, CF_MU1, CF_AL2, CF_BE2, CF_INV2, CF_MU3, CF_INV3,
    CF_A3, CF_B3, CF_C3, CF_AO, CF_BO, CF_CO, CF_W, CF_LOSS, CF_COUNT
};
constexpr int CSTR = 64;

enum PassCMode { PC_LOGITS = 1, PC_BWD = 2, PC_CE = 4 };

// ------------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : expm1f(z); }
__device__ __forceinline__ float elu_d(float z) { return z > 0.f ? 1.f : expf(z); }

// Dropout keep factor (model.py:50,74 nn.Dropout: x * mask / (1-p)).  Injected masks win; otherwise a
// counter-based splitmix64 draw keyed by (key, layer, flat index) -- identical in forward and backward.
__device__ __forceinline__ float keep_mul(const Geo& g, const uint8_t* __restrict__ mask, int layer,
                                          unsigned long long idx) {
    if (!g.drop) return 1.f;
    if (mask) return mask[idx] ? g.scale : 0.f;
    unsigned long long z = g.key + ((unsigned long long)(layer + 1) << 56) + idx * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const float u = (float)(unsigned)(z >> 40) * (1.0f / 16777216.0f);
    return u >= g.p ? g.scale : 0.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int NW>
__device__ __forceinline__ void lds_window(const float* __restrict__ p, float (&w)[4 * NW]) {
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const float4 f = *reinterpret_cast<const float4*>(p + 4 * i);
        w[4 * i + 0] = f.x; w[4 * i + 1] = f.y; w[4 * i + 2] = f.z; w[4 * i + 3] = f.w;
    }
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
    static constexpr int NPI = (K1 * (K1 - 1) / 2 + NT - 1) / NT;   // edge pairs per thread
};

// Stage one trial of x [C,T] into LDS rows (left pad LP, stride RS).  Pads are never written.
__device__ __forceinline__ void load_x(const Geo& g, const float* __restrict__ xb, float* Xs, int tid) {
    if ((g.T & 3) == 0) {
        const int TQ = g.T >> 2;
        const float4* src = reinterpret_cast<const float4*>(xb);
        for (int i = tid; i < g.C * TQ; i += NT) {
            const int c = i / TQ, q = i - c * TQ;
            *reinterpret_cast<float4*>(Xs + c * g.RS + g.LP + 4 * q) = src[i];
        }
    } else {
        for (int i = tid; i < g.C * g.T; i += NT) {
            const int c = i / g.T, t = i - c * g.T;
            Xs[c * g.RS + g.LP + t] = xb[i];
        }
    }
}

// s[o,t] = sum_c ws[o,c] x[c,t] on the matrix cores: v_mfma_f32_16x16x4_f32, A = ws tile (16 o x 4 c),
// B = x tile (4 c x 16 t).  Lane l: A[l&15][l>>4], B[l>>4][l&15]; D[4(l>>4)+r][l&15] (CDNA4 maps).
// Exact f32 (a k-ordered fmaf chain), so no precision is traded for the pipe.
__device__ __forceinline__ void spatial_mfma(const Geo& g, const float* Xs, const float* Wsh, float* Ss,
                                             int wave, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    const int NOT = g.FO >> 4, KS = g.CK >> 2, WST = g.CK + 1;
    for (int item = wave; item < NOT * g.NT16; item += 4) {
        const int ot = item / g.NT16, n = item - ot * g.NT16;
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
        const float* wrow = Wsh + (ot * 16 + li) * WST + lk;
        const float* xcol = Xs + lk * g.RS + g.LP + 16 * n + li;
        for (int s = 0; s < KS; ++s) {
            const int c = 4 * s + lk;
            const float a = wrow[4 * s];
            const float b = (c < g.C) ? xcol[4 * s * g.RS] : 0.f;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int o = ot * 16 + 4 * lk + r;
            if (o < g.F2) Ss[o * g.RS + g.LP + 16 * n + li] = acc[r];
        }
    }
}

// ws copy [FO][CK+1] (zero padded) used as the MFMA A operand
__device__ __forceinline__ void load_ws(const Geo& g, const float* __restrict__ prm, float* Wsh, int tid) {
    const int WST = g.CK + 1;
    for (int i = tid; i < g.FO * WST; i += NT) {
        const int o = i / WST, c = i - o * WST;
        Wsh[i] = (o < g.F2 && c < g.C) ? prm[g.o_ws + o * g.C + c] : 0.f;
    }
}

// block_2 forward on one trial (model.py:54-69): q = dw16(d2) ('same', pad 7|8), r = W3 q.
// D2s rows: d2 at [LP2, LP2+T1), zeros elsewhere; Qs/Rs rows at [0, 4*TQ1).
__device__ void block2_fwd(const Geo& g, const float* D2s, const float* W2sh, const float* W3sh,
                           float* Qs, float* Rs, int tid) {
    for (int it = tid; it < g.F2 * g.TQ1; it += NT) {
        const int o = it / g.TQ1, tq = it - o * g.TQ1;
        float w[20];
        lds_window<5>(D2s + o * g.RS2 + 4 * tq, w);
        float tp[16];
        lds_window<4>(W2sh + o * 16, tp);
        float q[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) a = fmaf(tp[k], w[1 + i + k], a);
            q[i] = (4 * tq + i < g.T1) ? a : 0.f;
        }
        *reinterpret_cast<float4*>(Qs + o * g.RS2 + 4 * tq) = make_float4(q[0], q[1], q[2], q[3]);
    }
    __syncthreads();
    for (int it = tid; it < g.F2 * g.TQ1; it += NT) {
        const int j = it / g.TQ1, tq = it - j * g.TQ1;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = 0; i < g.F2; ++i) {
            const float w = W3sh[j * g.F2 + i];
            const float4 q = *reinterpret_cast<const float4*>(Qs + i * g.RS2 + 4 * tq);
            acc.x = fmaf(w, q.x, acc.x); acc.y = fmaf(w, q.y, acc.y);
            acc.z = fmaf(w, q.z, acc.z); acc.w = fmaf(w, q.w, acc.w);
        }
        *reinterpret_cast<float4*>(Rs + j * g.RS2 + 4 * tq) = acc;
    }
    __syncthreads();
}

__device__ __forceinline__ void load_block2_weights(const Geo& g, const float* __restrict__ prm,
                                                    float* W2sh, float* W3sh, int tid) {
    for (int i = tid; i < g.F2 * 16; i += NT) W2sh[i] = prm[g.o_w2 + i];
    for (int i = tid; i < g.F2 * g.F2; i += NT) W3sh[i] = prm[g.o_W3 + i];
}

// ================================================================================================
// Pass A: BN1 / BN2 batch statistics.
// part row: [G0 K1][S0][Ed npairs][e1 K1-1][Sv F2][Sv2 F2]
// ================================================================================================
template <int K1>
__global__ __launch_bounds__(NT, 2) void k_pass_a(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ x, float* __restrict__ part) {
    using G_ = KG<K1>;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Xs = sm;
    float* Ss = Xs + g.C * g.RS;
    float* Wsh = Ss + g.F2 * g.RS;
    float* red = Wsh + ((g.FO * (g.CK + 1) + 3) & ~3);      // NT*2 scratch
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < (g.C + g.F2) * g.RS; i += NT) sm[i] = 0.f;
    load_ws(g, prm, Wsh, tid);

    // FIR ownership: thread -> (o, seg), quads seg, seg+nseg, ...
    const int fo = tid / g.nseg, fseg = tid - fo * g.nseg;
    const bool fir_on = fo < g.F2;
    float tap[K1];
    {
        const int gg = fir_on ? fo / g.D : 0;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    }
    float sv = 0.f, sv2 = 0.f;
    // Gram ownership: thread -> (c, seg)
    const int gc = tid / g.nsegC, gseg = tid - gc * g.nsegC;
    const bool gram_on = gc < g.C;
    float G0[K1];
#pragma unroll
    for (int d = 0; d < K1; ++d) G0[d] = 0.f;
    float s0 = 0.f;
    // edge pairs p = tid + NT*i, enumerated d-major: (d, j), j < K1-1-d
    float eacc[G_::NPI];
    int ed[G_::NPI], ej[G_::NPI];
#pragma unroll
    for (int i = 0; i < G_::NPI; ++i) {
        eacc[i] = 0.f;
        int p = tid + NT * i, d = 0;
        while (d < K1 && p >= K1 - 1 - d) { p -= K1 - 1 - d; ++d; }
        ed[i] = d; ej[i] = p;            // d == K1 -> unused slot
    }
    float e1acc = 0.f;
    __syncthreads();

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        load_x(g, x + (size_t)b * g.C * g.T, Xs, tid);
        __syncthreads();
        spatial_mfma(g, Xs, Wsh, Ss, wave, lane);
        // lag-Gram of the padded rows: G0[d] += sum_{t<T} X[t] X[t+d]
        if (gram_on) {
            const float* row = Xs + gc * g.RS;
            for (int q = gseg; q < g.TQ; q += g.nsegC) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float a[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = (4 * q + i < g.T) ? w[G_::OFF + i] : 0.f;
                s0 += (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
                for (int d = 0; d < K1; ++d) {
                    float acc = G0[d];
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc = fmaf(a[i], w[G_::OFF + i + d], acc);
                    G0[d] = acc;
                }
            }
        }
        // edge corrections: Ed[d][j] += sum_c X[T+j]X[T+j+d] - X[j]X[j+d]
        {
            const float* X0 = Xs + G_::OFF;
#pragma unroll
            for (int i = 0; i < G_::NPI; ++i) {
                if (ed[i] < K1) {
                    const int d = ed[i], j = ej[i];
                    float acc = eacc[i];
                    for (int c = 0; c < g.C; ++c) {
                        const float* r = X0 + c * g.RS;
                        acc = fmaf(r[g.T + j], r[g.T + j + d], acc);
                        acc = fmaf(-r[j], r[j + d], acc);
                    }
                    eacc[i] = acc;
                }
            }
            if (tid < K1 - 1) {
                float acc = e1acc;
                for (int c = 0; c < g.C; ++c) {
                    const float* r = X0 + c * g.RS;
                    acc += r[g.T + tid] - r[tid];
                }
                e1acc = acc;
            }
        }
        __syncthreads();
        // v = w1[g] (*) s; accumulate sum v, sum v^2
        if (fir_on) {
            const float* row = Ss + fo * g.RS;
            for (int q = fseg; q < g.TQ; q += g.nseg) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < K1; ++k) v = fmaf(tap[k], w[G_::OFF + i + k], v);
                    if (4 * q + i < g.T) { sv += v; sv2 = fmaf(v, v, sv2); }
                }
            }
        }
        __syncthreads();
    }

    // ---- workgroup reduction -> one partial row ----
    float* row = part + (size_t)blockIdx.x * g.nA;
    float* wred = red;   // [4][K1+1]
#pragma unroll
    for (int d = 0; d < K1; ++d) {
        const float t = wave_sum(G0[d]);
        if (lane == 0) wred[wave * (K1 + 1) + d] = t;
    }
    {
        const float t = wave_sum(s0);
        if (lane == 0) wred[wave * (K1 + 1) + K1] = t;
    }
    __syncthreads();
    if (tid <= K1) {
        float t = 0.f;
        for (int w = 0; w < 4; ++w) t += wred[w * (K1 + 1) + tid];
        row[tid] = t;          // G0[0..K1), S0 at K1
    }
#pragma unroll
    for (int i = 0; i < G_::NPI; ++i)
        if (ed[i] < K1) row[K1 + 1 + tid + NT * i] = eacc[i];
    if (tid < K1 - 1) row[K1 + 1 + g.npairs + tid] = e1acc;
    __syncthreads();
    red[tid] = fir_on ? sv : 0.f;
    red[NT + tid] = fir_on ? sv2 : 0.f;
    __syncthreads();
    if (tid < g.F2) {
        float a = 0.f, b2 = 0.f;
        for (int s = 0; s < g.nseg; ++s) { a += red[tid * g.nseg + s]; b2 += red[NT + tid * g.nseg + s]; }
        const int base = K1 + 1 + g.npairs + K1 - 1;
        row[base + tid] = a;
        row[base + g.F2 + tid] = b2;
    }
}

// ================================================================================================
// Pass B: forward to d2, E1/E2 (pooled ELU' sums for BN2 backward), BN3 statistics.
// part row: [Sr F2][Sr2 F2]
// ================================================================================================
template <int K1>
__global__ __launch_bounds__(NT, 2) void k_pass_b(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ coef,
                                               const float* __restrict__ x,
                                               const uint8_t* __restrict__ mask2,
                                               float* __restrict__ d2g, float* __restrict__ E1g,
                                               float* __restrict__ E2g, float* __restrict__ part) {
    using G_ = KG<K1>;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Xs = sm;
    float* Ss = Xs + g.C * g.RS;
    float* D2s = Ss + g.F2 * g.RS;
    float* Qs = D2s + g.F2 * g.RS2;
    float* Rs = Qs + g.F2 * g.RS2;
    float* W2sh = Rs + g.F2 * g.RS2;
    float* W3sh = W2sh + g.F2 * 16;
    float* Wsh = W3sh + ((g.F2 * g.F2 + 3) & ~3);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < (g.C + g.F2) * g.RS + 3 * g.F2 * g.RS2; i += NT) sm[i] = 0.f;
    load_ws(g, prm, Wsh, tid);
    load_block2_weights(g, prm, W2sh, W3sh, tid);

    const int fo = tid / g.nseg, fseg = tid - fo * g.nseg;
    const bool fir_on = fo < g.F2;
    float tap[K1];
    float al = 0.f, be = 0.f, ga = 0.f, bt = 0.f;
    {
        const int o = fir_on ? fo : 0, gg = o / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
        al = coef[CF_AL2 * CSTR + o]; be = coef[CF_BE2 * CSTR + o];
        ga = prm[g.o_g2 + o]; bt = prm[g.o_b2 + o];
    }
    double sr = 0.0, sr2 = 0.0;     // owner j = tid < F2
    __syncthreads();

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        load_x(g, x + (size_t)b * g.C * g.T, Xs, tid);
        __syncthreads();
        spatial_mfma(g, Xs, Wsh, Ss, wave, lane);
        __syncthreads();
        if (fir_on) {
            const float* row = Ss + fo * g.RS;
            for (int q = fseg; q < g.T1; q += g.nseg) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float pe = 0.f, e1 = 0.f, e2 = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < K1; ++k) v = fmaf(tap[k], w[G_::OFF + i + k], v);
                    const float xh = fmaf(al, v, be);
                    const float z = fmaf(ga, xh, bt);
                    const float dz = elu_d(z);
                    pe += z > 0.f ? z : dz - 1.f;      // ELU(z) = exp(z)-1 on the negative side
                    e1 += dz;
                    e2 = fmaf(dz, xh, e2);
                }
                const size_t gi = ((size_t)b * g.F2 + fo) * g.T1 + q;
                const float d2 = pe * 0.25f * keep_mul(g, mask2, 0, gi);
                d2g[gi] = d2; E1g[gi] = e1; E2g[gi] = e2;
                D2s[fo * g.RS2 + LP2 + q] = d2;
            }
        }
        __syncthreads();
        block2_fwd(g, D2s, W2sh, W3sh, Qs, Rs, tid);
        if (tid < g.F2) {
            float a = 0.f, a2 = 0.f;
            const float* rr = Rs + tid * g.RS2;
            for (int t = 0; t < g.T1; ++t) { const float r = rr[t]; a += r; a2 = fmaf(r, r, a2); }
            sr += a; sr2 += a2;
        }
        __syncthreads();
    }
    if (tid < g.F2) {
        float* row = part + (size_t)blockIdx.x * g.nB;
        row[tid] = (float)sr;
        row[g.F2 + tid] = (float)sr2;
    }
}

// ================================================================================================
// Pass C: head.  logits, and (PC_BWD) classifier grads + BN3 backward sums.
// part row: [dWfc 4*NF][dbfc 4][Sdz3 F2][Sdz3x F2][loss]
// ================================================================================================
__global__ __launch_bounds__(NT) void k_pass_c(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ coef,
                                               const float* __restrict__ d2g,
                                               const uint8_t* __restrict__ mask3,
                                               const float* __restrict__ dlin,
                                               const int64_t* __restrict__ labels,
                                               float* __restrict__ logits, float* __restrict__ dlout,
                                               float* __restrict__ part, int mode) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2s = sm;
    float* Qs = D2s + g.F2 * g.RS2;       // q, then z3
    float* Rs = Qs + g.F2 * g.RS2;        // r, then xh3
    float* W2sh = Rs + g.F2 * g.RS2;
    float* W3sh = W2sh + g.F2 * 16;
    float* Hs = W3sh + ((g.F2 * g.F2 + 3) & ~3);
    float* DP3s = Hs + ((g.NF + 3) & ~3);
    float* acc = DP3s + ((g.NF + 3) & ~3);       // 4*NF + 4
    float* Ls = acc + ((4 * g.NF + 4 + 3) & ~3);  // 8
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < 3 * g.F2 * g.RS2; i += NT) sm[i] = 0.f;
    for (int i = tid; i < 4 * g.NF + 4; i += NT) acc[i] = 0.f;
    load_block2_weights(g, prm, W2sh, W3sh, tid);
    double sdz = 0.0, sdzx = 0.0, lossacc = 0.0;
    __syncthreads();

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        for (int i = tid; i < g.F2 * g.T1; i += NT) {
            const int o = i / g.T1, t = i - o * g.T1;
            D2s[o * g.RS2 + LP2 + t] = d2g[(size_t)b * g.F2 * g.T1 + i];
        }
        __syncthreads();
        block2_fwd(g, D2s, W2sh, W3sh, Qs, Rs, tid);
        for (int i = tid; i < g.F2 * g.T1; i += NT) {
            const int j = i / g.T1, t = i - j * g.T1;
            const float xh = (Rs[j * g.RS2 + t] - coef[CF_MU3 * CSTR + j]) * coef[CF_INV3 * CSTR + j];
            Rs[j * g.RS2 + t] = xh;
            Qs[j * g.RS2 + t] = fmaf(prm[g.o_g3 + j], xh, prm[g.o_b3 + j]);
        }
        __syncthreads();
        for (int i = tid; i < g.NF; i += NT) {
            const int j = i / g.T2, t2 = i - j * g.T2;
            const float* z = Qs + j * g.RS2 + 8 * t2;
            float s = 0.f;
#pragma unroll
            for (int m = 0; m < 8; ++m) s += elu_f(z[m]);
            Hs[i] = s * 0.125f * keep_mul(g, mask3, 1, (size_t)b * g.NF + i);
        }
        __syncthreads();
        {   // logits: wave n computes class n (4 waves, 4 classes)
            const int n = wave;
            float a = 0.f;
            for (int i = lane; i < g.NF; i += 64) a = fmaf(prm[g.o_Wfc + n * g.NF + i], Hs[i], a);
            a = wave_sum(a);
            if (lane == 0) Ls[n] = a + prm[g.o_bfc + n];
        }
        __syncthreads();
        if ((mode & PC_LOGITS) && tid < NCLS) logits[(size_t)b * NCLS + tid] = Ls[tid];
        if (mode & PC_BWD) {
            if (tid == 0) {
                float dl[NCLS];
                if (mode & PC_CE) {
                    float m = Ls[0];
                    for (int n = 1; n < NCLS; ++n) m = fmaxf(m, Ls[n]);
                    float se = 0.f;
                    for (int n = 0; n < NCLS; ++n) se += expf(Ls[n] - m);
                    const float lse = m + logf(se);
                    const int y = (int)labels[b];
                    lossacc += (double)(lse - Ls[y]);
                    const float invB = 1.0f / (float)g.B;
                    for (int n = 0; n < NCLS; ++n)
                        dl[n] = (expf(Ls[n] - lse) - (n == y ? 1.f : 0.f)) * invB;
                    for (int n = 0; n < NCLS; ++n) dlout[(size_t)b * NCLS + n] = dl[n];
                } else {
                    for (int n = 0; n < NCLS; ++n) dl[n] = dlin[(size_t)b * NCLS + n];
                }
                for (int n = 0; n < NCLS; ++n) Ls[4 + n] = dl[n];
            }
            __syncthreads();
            const float* DL = Ls + 4;
            for (int p = tid; p < NCLS * g.NF; p += NT) acc[p] = fmaf(DL[p / g.NF], Hs[p % g.NF], acc[p]);
            if (tid < NCLS) acc[NCLS * g.NF + tid] += DL[tid];
            for (int i = tid; i < g.NF; i += NT) {
                float dh = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dh = fmaf(DL[n], prm[g.o_Wfc + n * g.NF + i], dh);
                DP3s[i] = dh * keep_mul(g, mask3, 1, (size_t)b * g.NF + i);
            }
            __syncthreads();
            if (tid < g.F2) {
                const int j = tid;
                float a = 0.f, ax = 0.f;
                for (int t = 0; t < 8 * g.T2; ++t) {
                    const float dz = DP3s[j * g.T2 + (t >> 3)] * 0.125f * elu_d(Qs[j * g.RS2 + t]);
                    a += dz;
                    ax = fmaf(dz, Rs[j * g.RS2 + t], ax);
                }
                sdz += a; sdzx += ax;
            }
        }
        __syncthreads();
    }
    if (mode & PC_BWD) {
        float* row = part + (size_t)blockIdx.x * g.nC;
        for (int p = tid; p < NCLS * g.NF + NCLS; p += NT) row[p] = acc[p];
        if (tid < g.F2) {
            row[NCLS * g.NF + NCLS + tid] = (float)sdz;
            row[NCLS * g.NF + NCLS + g.F2 + tid] = (float)sdzx;
        }
        if (tid == 0) row[NCLS * g.NF + NCLS + 2 * g.F2] = (float)lossacc;
    }
}

// ================================================================================================
// Pass D: block_2 backward (dW3, dw2), dp2 = d(pooled ELU output), BN2-backward sums.
// part row: [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2]
// ================================================================================================
__global__ __launch_bounds__(NT) void k_pass_d(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ coef,
                                               const float* __restrict__ d2g,
                                               const float* __restrict__ E1g,
                                               const float* __restrict__ E2g,
                                               const uint8_t* __restrict__ mask2,
                                               const uint8_t* __restrict__ mask3,
                                               const float* __restrict__ dl,
                                               float* __restrict__ dp2g, float* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2s = sm;
    float* Qs = D2s + g.F2 * g.RS2;        // q
    float* Rs = Qs + g.F2 * g.RS2;         // r -> xh3 -> dr
    float* Zs = Rs + g.F2 * g.RS2;         // z3, then products for the BN2 sums
    float* DQs = Zs + g.F2 * g.RS2;        // dq, padded LP2 | 8
    float* W2sh = DQs + g.F2 * g.RS2;
    float* W3sh = W2sh + g.F2 * 16;
    float* DP3s = W3sh + ((g.F2 * g.F2 + 3) & ~3);
    float* acc = DP3s + ((g.NF + 3) & ~3);     // F2*F2 + 16*F2 + 2*F2
    const int tid = threadIdx.x;
    const int nacc = g.F2 * g.F2 + 16 * g.F2 + 2 * g.F2;

    for (int i = tid; i < 5 * g.F2 * g.RS2; i += NT) sm[i] = 0.f;
    for (int i = tid; i < nacc; i += NT) acc[i] = 0.f;
    load_block2_weights(g, prm, W2sh, W3sh, tid);
    __syncthreads();

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        for (int i = tid; i < g.F2 * g.T1; i += NT) {
            const int o = i / g.T1, t = i - o * g.T1;
            D2s[o * g.RS2 + LP2 + t] = d2g[(size_t)b * g.F2 * g.T1 + i];
        }
        __syncthreads();
        block2_fwd(g, D2s, W2sh, W3sh, Qs, Rs, tid);
        for (int i = tid; i < g.F2 * g.T1; i += NT) {
            const int j = i / g.T1, t = i - j * g.T1;
            const float xh = (Rs[j * g.RS2 + t] - coef[CF_MU3 * CSTR + j]) * coef[CF_INV3 * CSTR + j];
            Rs[j * g.RS2 + t] = xh;
            Zs[j * g.RS2 + t] = fmaf(prm[g.o_g3 + j], xh, prm[g.o_b3 + j]);
        }
        for (int i = tid; i < g.NF; i += NT) {
            float dh = 0.f;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) dh = fmaf(dl[(size_t)b * NCLS + n], prm[g.o_Wfc + n * g.NF + i], dh);
            DP3s[i] = dh * keep_mul(g, mask3, 1, (size_t)b * g.NF + i);
        }
        __syncthreads();
        // dr = A3 dz3 + B3 + C3 xh3   (BN3 backward with the batch constants of finalize 3)
        for (int i = tid; i < g.F2 * g.T1; i += NT) {
            const int j = i / g.T1, t = i - j * g.T1;
            const float dz = (t < 8 * g.T2)
                ? DP3s[j * g.T2 + (t >> 3)] * 0.125f * elu_d(Zs[j * g.RS2 + t]) : 0.f;
            const float xh = Rs[j * g.RS2 + t];
            Rs[j * g.RS2 + t] = fmaf(coef[CF_A3 * CSTR + j], dz,
                                     fmaf(coef[CF_C3 * CSTR + j], xh, coef[CF_B3 * CSTR + j]));
        }
        __syncthreads();
        // dW3[j][i] += sum_t dr[j][t] q[i][t]
        for (int p = tid; p < g.F2 * g.F2; p += NT) {
            const int j = p / g.F2, i = p - j * g.F2;
            const float* a = Rs + j * g.RS2;
            const float* q = Qs + i * g.RS2;
            float s = 0.f;
            for (int t = 0; t < g.T1; ++t) s = fmaf(a[t], q[t], s);
            acc[p] += s;
        }
        // dq[i][t] = sum_j W3[j][i] dr[j][t]
        for (int it = tid; it < g.F2 * g.T1; it += NT) {
            const int i = it / g.T1, t = it - i * g.T1;
            float s = 0.f;
            for (int j = 0; j < g.F2; ++j) s = fmaf(W3sh[j * g.F2 + i], Rs[j * g.RS2 + t], s);
            DQs[i * g.RS2 + LP2 + t] = s;
        }
        __syncthreads();
        // dw2[o][k] += sum_t dq[o][t] d2pad[o][t+k]
        for (int p = tid; p < g.F2 * 16; p += NT) {
            const int o = p >> 4, k = p & 15;
            const float* a = DQs + o * g.RS2 + LP2;
            const float* d = D2s + o * g.RS2 + 1 + k;
            float s = 0.f;
            for (int t = 0; t < g.T1; ++t) s = fmaf(a[t], d[t], s);
            acc[g.F2 * g.F2 + p] += s;
        }
        // dd2[o][t] = sum_k w2[o][k] dq[o][t+7-k]  -> dp2 = dd2 * keep / (1-p)
        for (int it = tid; it < g.F2 * g.T1; it += NT) {
            const int o = it / g.T1, t = it - o * g.T1;
            const float* a = DQs + o * g.RS2 + LP2 + t + 7;
            float s = 0.f;
#pragma unroll
            for (int k = 0; k < 16; ++k) s = fmaf(W2sh[o * 16 + k], a[-k], s);
            const size_t gi = (size_t)b * g.F2 * g.T1 + it;
            const float dp = s * keep_mul(g, mask2, 0, gi);
            dp2g[gi] = dp;
            Zs[o * g.RS2 + t] = dp * 0.25f * E1g[gi];
            Qs[o * g.RS2 + t] = dp * 0.25f * E2g[gi];
        }
        __syncthreads();
        if (tid < g.F2) {
            float a = 0.f, a2 = 0.f;
            for (int t = 0; t < g.T1; ++t) { a += Zs[tid * g.RS2 + t]; a2 += Qs[tid * g.RS2 + t]; }
            acc[g.F2 * g.F2 + 16 * g.F2 + tid] += a;
            acc[g.F2 * g.F2 + 17 * g.F2 + tid] += a2;
        }
        __syncthreads();
    }
    float* row = part + (size_t)blockIdx.x * g.nD;
    for (int p = tid; p < nacc; p += NT) row[p] = acc[p];
}

// ================================================================================================
// Pass E: dy2 and the three weight-gradient reductions that need full-rate data.
// part row: [Q F2*K1][Xm F2*C][Sdy F2][Sdyv F2]
// ================================================================================================
template <int K1>
__global__ __launch_bounds__(NT, 2) void k_pass_e(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ coef,
                                               const float* __restrict__ x,
                                               const float* __restrict__ dp2g,
                                               float* __restrict__ part) {
    using G_ = KG<K1>;
    constexpr int MAXU = 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Xs = sm;
    float* Ss = Xs + g.C * g.RS;            // s, then e
    float* Dys = Ss + g.F2 * g.RS;          // dy2 (same padded layout)
    float* DP = Dys + g.F2 * g.RS;          // dp2 [F2][T1]
    float* Wsh = DP + ((g.F2 * g.T1 + 3) & ~3);
    float* red = Wsh + ((g.FO * (g.CK + 1) + 3) & ~3);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;

    for (int i = tid; i < (g.C + 2 * g.F2) * g.RS; i += NT) sm[i] = 0.f;
    load_ws(g, prm, Wsh, tid);

    const int fo = tid / g.nseg, fseg = tid - fo * g.nseg;
    const bool fir_on = fo < g.F2;
    float tap[K1];
    float al = 0.f, be = 0.f, ga = 0.f, bt = 0.f, Ao = 0.f, Bo = 0.f, Co = 0.f;
    {
        const int o = fir_on ? fo : 0, gg = o / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
        al = coef[CF_AL2 * CSTR + o]; be = coef[CF_BE2 * CSTR + o];
        ga = prm[g.o_g2 + o]; bt = prm[g.o_b2 + o];
        Ao = coef[CF_AO * CSTR + o]; Bo = coef[CF_BO * CSTR + o]; Co = coef[CF_CO * CSTR + o];
    }
    float Q[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k) Q[k] = 0.f;
    float sdy = 0.f, sdyv = 0.f;
    // Xm MFMA units: tile (ot, ct) x k-split
    const int NOT = g.FO >> 4, ntile = NOT * g.NCT;
    const int ksplit = ntile >= 4 ? 1 : 4 / ntile;
    const int nunit = ntile * ksplit;
    floatx4 xacc[MAXU];
#pragma unroll
    for (int u = 0; u < MAXU; ++u) xacc[u] = (floatx4){0.f, 0.f, 0.f, 0.f};
    __syncthreads();

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        load_x(g, x + (size_t)b * g.C * g.T, Xs, tid);
        for (int i = tid; i < g.F2 * g.T1; i += NT) DP[i] = dp2g[(size_t)b * g.F2 * g.T1 + i];
        __syncthreads();
        spatial_mfma(g, Xs, Wsh, Ss, wave, lane);
        __syncthreads();
        // v, BN2 backward -> dy2; sums; dW1 correlation Q[k] += sum_i dy[i] spad[t0+i+k]
        if (fir_on) {
            const float* row = Ss + fo * g.RS;
            float* drow = Dys + fo * g.RS + g.LP;
            for (int q = fseg; q < g.TQ; q += g.nseg) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                const float dpq = (q < g.T1) ? DP[fo * g.T1 + q] * 0.25f : 0.f;
                float dy[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < K1; ++k) v = fmaf(tap[k], w[G_::OFF + i + k], v);
                    const float xh = fmaf(al, v, be);
                    const float z = fmaf(ga, xh, bt);
                    const float dz = dpq * elu_d(z);
                    float d = fmaf(Ao, dz, fmaf(Co, xh, Bo));
                    d = (4 * q + i < g.T) ? d : 0.f;
                    dy[i] = d;
                    sdy += d;
                    sdyv = fmaf(d, v, sdyv);
                }
#pragma unroll
                for (int k = 0; k < K1; ++k) {
                    float a = Q[k];
#pragma unroll
                    for (int i = 0; i < 4; ++i) a = fmaf(dy[i], w[G_::OFF + i + k], a);
                    Q[k] = a;
                }
                *reinterpret_cast<float4*>(drow + 4 * q) = make_float4(dy[0], dy[1], dy[2], dy[3]);
            }
        }
        __syncthreads();
        // e[P+s] = sum_m w1[K1-1-m] dypad[s+m]  (transposed FIR) -> overwrites s rows
        if (fir_on) {
            const float* row = Dys + fo * g.RS;
            float* erow = Ss + fo * g.RS + g.LP;
            for (int q = fseg; q < g.TQ; q += g.nseg) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float e[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int m = 0; m < K1; ++m) a = fmaf(tap[K1 - 1 - m], w[G_::OFFD + i + m], a);
                    e[i] = (4 * q + i < g.T) ? a : 0.f;
                }
                *reinterpret_cast<float4*>(erow + 4 * q) = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
        __syncthreads();
        // Xm[o][c] += sum_t e[o][t] x[c][t]  on the matrix cores (A = e 16o x 4t, B = x 4t x 16c)
#pragma unroll
        for (int ui = 0; ui < MAXU; ++ui) {
            const int u = wave + 4 * ui;
            if (u < nunit) {
                const int tile = u % ntile, ks = u / ntile;
                const int ot = tile / g.NCT, ct = tile - ot * g.NCT;
                const int o = ot * 16 + li, c = ct * 16 + li;
                const int k0 = (g.TQ * ks) / ksplit, k1 = (g.TQ * (ks + 1)) / ksplit;
                const float* arow = Ss + (o < g.F2 ? o : 0) * g.RS + g.LP + lk;
                const float* brow = Xs + (c < g.C ? c : 0) * g.RS + g.LP + lk;
                floatx4 a4 = xacc[ui];
                for (int kq = k0; kq < k1; ++kq) {
                    const float a = (o < g.F2) ? arow[4 * kq] : 0.f;
                    const float bb = (c < g.C) ? brow[4 * kq] : 0.f;
                    a4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, a4, 0, 0, 0);
                }
                xacc[ui] = a4;
            }
        }
        __syncthreads();
    }

    // ---- reductions ----
    float* row = part + (size_t)blockIdx.x * g.nE;
    for (int k = 0; k < K1; ++k) {
        red[tid] = fir_on ? Q[k] : 0.f;
        __syncthreads();
        if (tid < g.F2) {
            float a = 0.f;
            for (int s = 0; s < g.nseg; ++s) a += red[tid * g.nseg + s];
            row[tid * K1 + k] = a;
        }
        __syncthreads();
    }
    red[tid] = fir_on ? sdy : 0.f;
    red[NT + tid] = fir_on ? sdyv : 0.f;
    __syncthreads();
    if (tid < g.F2) {
        float a = 0.f, a2 = 0.f;
        for (int s = 0; s < g.nseg; ++s) { a += red[tid * g.nseg + s]; a2 += red[NT + tid * g.nseg + s]; }
        row[g.F2 * K1 + g.F2 * g.C + tid] = a;
        row[g.F2 * K1 + g.F2 * g.C + g.F2 + tid] = a2;
    }
    __syncthreads();
    // Xm: waves hold (tile, ksplit) accumulators -> LDS [ksplit][FO][16*NCT] -> sum over ksplit
    float* XR = Xs;      // reuse the x / s / dy rows (contiguous, (C + 2 F2) * RS floats)
    const int XW = 16 * g.NCT;
#pragma unroll
    for (int ui = 0; ui < MAXU; ++ui) {
        const int u = wave + 4 * ui;
        if (u < nunit) {
            const int tile = u % ntile, ks = u / ntile;
            const int ot = tile / g.NCT, ct = tile - ot * g.NCT;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                XR[(ks * g.FO + ot * 16 + 4 * lk + r) * XW + ct * 16 + li] = xacc[ui][r];
        }
    }
    __syncthreads();
    for (int p = tid; p < g.F2 * g.C; p += NT) {
        const int o = p / g.C, c = p - o * g.C;
        float a = 0.f;
        for (int ks = 0; ks < ksplit; ++ks) a += XR[(ks * g.FO + o) * XW + c];
        row[g.F2 * K1 + p] = a;
    }
}

// ================================================================================================
// Eval-mode forward: one fused kernel per trial (BN running statistics folded; no dropout).
// ================================================================================================
template <int K1>
__global__ __launch_bounds__(NT, 2) void k_infer(Geo g, const float* __restrict__ prm,
                                              const float* __restrict__ bn,
                                              const float* __restrict__ x, float* __restrict__ logits) {
    using G_ = KG<K1>;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Xs = sm;
    float* Ss = Xs + g.C * g.RS;
    float* D2s = Ss + g.F2 * g.RS;
    float* Qs = D2s + g.F2 * g.RS2;
    float* Rs = Qs + g.F2 * g.RS2;
    float* W2sh = Rs + g.F2 * g.RS2;
    float* W3sh = W2sh + g.F2 * 16;
    float* Wsh = W3sh + ((g.F2 * g.F2 + 3) & ~3);
    float* Hs = Wsh + ((g.FO * (g.CK + 1) + 3) & ~3);
    float* cf = Hs + ((g.NF + 3) & ~3);          // [al F2][be F2][a3 F2][b3 F2]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* rm1 = bn;                 const float* rv1 = bn + g.F1;
    const float* rm2 = bn + 2 * g.F1;      const float* rv2 = rm2 + g.F2;
    const float* rm3 = rm2 + 2 * g.F2;     const float* rv3 = rm3 + g.F2;

    for (int i = tid; i < (g.C + g.F2) * g.RS + 3 * g.F2 * g.RS2; i += NT) sm[i] = 0.f;
    load_ws(g, prm, Wsh, tid);
    load_block2_weights(g, prm, W2sh, W3sh, tid);
    if (tid < g.F2) {
        const int o = tid, gg = o / g.D;
        // eval BN1 (model.py:32) and BN2 (model.py:47) folded into z2 = al*v + be
        const float a1 = prm[g.o_g1 + gg] / sqrtf(rv1[gg] + g.eps);
        const float c1 = prm[g.o_b1 + gg] - a1 * rm1[gg];
        float W = 0.f;
        for (int c = 0; c < g.C; ++c) W += prm[g.o_ws + o * g.C + c];
        const float s2 = prm[g.o_g2 + o] / sqrtf(rv2[o] + g.eps);
        cf[o] = a1 * s2;
        cf[g.F2 + o] = (c1 * W - rm2[o]) * s2 + prm[g.o_b2 + o];
        const float s3 = prm[g.o_g3 + o] / sqrtf(rv3[o] + g.eps);
        cf[2 * g.F2 + o] = s3;
        cf[3 * g.F2 + o] = prm[g.o_b3 + o] - rm3[o] * s3;
    }
    const int fo = tid / g.nseg, fseg = tid - fo * g.nseg;
    const bool fir_on = fo < g.F2;
    float tap[K1];
    {
        const int gg = (fir_on ? fo : 0) / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    }
    __syncthreads();
    const float al = fir_on ? cf[fo] : 0.f, be = fir_on ? cf[g.F2 + fo] : 0.f;

    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        load_x(g, x + (size_t)b * g.C * g.T, Xs, tid);
        __syncthreads();
        spatial_mfma(g, Xs, Wsh, Ss, wave, lane);
        __syncthreads();
        if (fir_on) {
            const float* row = Ss + fo * g.RS;
            for (int q = fseg; q < g.T1; q += g.nseg) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float pe = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float v = 0.f;
#pragma unroll
                    for (int k = 0; k < K1; ++k) v = fmaf(tap[k], w[G_::OFF + i + k], v);
                    pe += elu_f(fmaf(al, v, be));
                }
                D2s[fo * g.RS2 + LP2 + q] = pe * 0.25f;
            }
        }
        __syncthreads();
        block2_fwd(g, D2s, W2sh, W3sh, Qs, Rs, tid);
        for (int i = tid; i < g.NF; i += NT) {
            const int j = i / g.T2, t2 = i - j * g.T2;
            const float* r = Rs + j * g.RS2 + 8 * t2;
            const float s3 = cf[2 * g.F2 + j], b3 = cf[3 * g.F2 + j];
            float s = 0.f;
#pragma unroll
            for (int m = 0; m < 8; ++m) s += elu_f(fmaf(s3, r[m], b3));
            Hs[i] = s * 0.125f;
        }
        __syncthreads();
        {
            const int n = wave;
            float a = 0.f;
            for (int i = lane; i < g.NF; i += 64) a = fmaf(prm[g.o_Wfc + n * g.NF + i], Hs[i], a);
            a = wave_sum(a);
            if (lane == 0) logits[(size_t)b * NCLS + n] = a + prm[g.o_bfc + n];
        }
        __syncthreads();
    }
}

// ================================================================================================
// Deterministic fp64 column reduction of per-workgroup partial rows, stage 1: the rows are cut into
// RCH chunks; workgroup (column block, chunk) writes one fp64 partial per column.  Stage 2 (the
// RCH-way sum per column) is the prologue of the finalize kernel that consumes the sums.
// ================================================================================================
constexpr int RCH = 32;

__global__ __launch_bounds__(NT) void k_colsum(const float* __restrict__ part, int nrows, int ncols,
                                               double* __restrict__ part2) {
    __shared__ double red[4][64];
    const int tid = threadIdx.x, col = blockIdx.x * 64 + (tid & 63), rg = tid >> 6;
    const int r0 = (nrows * (int)blockIdx.y) / RCH, r1 = (nrows * ((int)blockIdx.y + 1)) / RCH;
    double a = 0.0;
    if (col < ncols)
        for (int r = r0 + rg; r < r1; r += 4) a += (double)part[(size_t)r * ncols + col];
    red[rg][tid & 63] = a;
    __syncthreads();
    if (tid < 64 && col < ncols)
        part2[(size_t)blockIdx.y * ncols + col] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

// stage 2, run by the one finalize workgroup: S[c] = sum over the RCH chunk partials
__device__ __forceinline__ void reduce_chunks(const double* __restrict__ part2, int ncols, double* S) {
    for (int c = threadIdx.x; c < ncols; c += NT) {
        double a = 0.0;
#pragma unroll 8
        for (int r = 0; r < RCH; ++r) a += part2[(size_t)r * ncols + c];
        S[c] = a;
    }
    __syncthreads();
}

// ================================================================================================
// Finalize kernels (one workgroup each): BN constants, running statistics, parameter gradients.
// ================================================================================================
__device__ __forceinline__ void bn_running(float* rm, float* rv, double mu, double var, double n,
                                           float mom) {
    *rm = (float)((1.0 - mom) * (double)*rm + mom * mu);
    *rv = (float)((1.0 - mom) * (double)*rv + mom * var * n / (n - 1.0));
}

// after pass A: BN1 (model.py:32) and BN2 (model.py:47) batch statistics
__global__ __launch_bounds__(NT) void k_fin1(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             double* __restrict__ stats, float* __restrict__ coef,
                                             float* __restrict__ bn, int update_running) {
    extern __shared__ __attribute__((aligned(16))) double dsm[];
    const int K1 = g.K1;
    double* Gm = dsm;                 // K1*K1
    double* S1 = Gm + K1 * K1;        // K1
    double* a1s = S1 + K1;            // F1
    double* c1s = a1s + 64;
    double* sums = c1s + 64;          // nA
    const int tid = threadIdx.x;
    reduce_chunks(part2, g.nA, sums);
    const double* G0 = sums;
    const double S0 = sums[K1];
    const double* Ed = sums + K1 + 1;
    const double* e1 = Ed + g.npairs;
    const double* Sv = e1 + K1 - 1;
    const double* Sv2 = Sv + g.F2;
    if (tid < K1) {
        const int d = tid;
        int base = 0;
        for (int dd = 0; dd < d; ++dd) base += K1 - 1 - dd;
        double acc = G0[d];
        for (int k = 0; k + d < K1; ++k) {
            Gm[k * K1 + k + d] = acc;
            Gm[(k + d) * K1 + k] = acc;
            if (k < K1 - 1 - d) acc += Ed[base + k];
        }
    }
    if (tid == 0) {
        double acc = S0;
        for (int k = 0; k < K1; ++k) { S1[k] = acc; if (k < K1 - 1) acc += e1[k]; }
    }
    __syncthreads();
    for (int i = tid; i < K1 * K1 + K1; i += NT) stats[i] = Gm[i];
    const double n1 = (double)g.B * g.C * g.T;
    if (tid < g.F1) {
        const float* w = prm + g.o_w1 + tid * K1;
        double mu = 0.0, e2 = 0.0;
        for (int k = 0; k < K1; ++k) {
            mu += (double)w[k] * S1[k];
            double r = 0.0;
            for (int l = 0; l < K1; ++l) r += Gm[k * K1 + l] * (double)w[l];
            e2 += (double)w[k] * r;
        }
        mu /= n1;
        const double var = e2 / n1 - mu * mu;
        const double inv = 1.0 / sqrt(var + (double)g.eps);
        const double a1 = (double)prm[g.o_g1 + tid] * inv;
        const double c1 = (double)prm[g.o_b1 + tid] - a1 * mu;
        a1s[tid] = a1; c1s[tid] = c1;
        coef[CF_A1 * CSTR + tid] = (float)a1;
        coef[CF_C1 * CSTR + tid] = (float)c1;
        coef[CF_INV1 * CSTR + tid] = (float)inv;
        coef[CF_MU1 * CSTR + tid] = (float)mu;
        if (update_running) bn_running(bn + tid, bn + g.F1 + tid, mu, var, n1, g.mom);
    }
    __syncthreads();
    const double n2 = (double)g.B * g.T;
    if (tid < g.F2) {
        const int o = tid, gg = o / g.D;
        double W = 0.0;
        for (int c = 0; c < g.C; ++c) W += (double)prm[g.o_ws + o * g.C + c];
        const double mv = Sv[o] / n2;
        const double varv = Sv2[o] / n2 - mv * mv;
        const double mu2 = a1s[gg] * mv + c1s[gg] * W;
        const double var2 = a1s[gg] * a1s[gg] * varv;
        const double inv2 = 1.0 / sqrt(var2 + (double)g.eps);
        const double alpha = a1s[gg] * inv2;
        coef[CF_AL2 * CSTR + o] = (float)alpha;
        coef[CF_BE2 * CSTR + o] = (float)(-alpha * mv);
        coef[CF_INV2 * CSTR + o] = (float)inv2;
        coef[CF_W * CSTR + o] = (float)W;
        float* rm2 = bn + 2 * g.F1;
        if (update_running) bn_running(rm2 + o, rm2 + g.F2 + o, mu2, var2, n2, g.mom);
    }
}

// after pass B: BN3 (model.py:71) batch statistics
__global__ __launch_bounds__(NT) void k_fin2(Geo g, const double* __restrict__ part2,
                                             float* __restrict__ coef, float* __restrict__ bn,
                                             int update_running) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nB, sums);
    const int j = threadIdx.x;
    if (j >= g.F2) return;
    const double n3 = (double)g.B * g.T1;
    const double mu = sums[j] / n3;
    const double var = sums[g.F2 + j] / n3 - mu * mu;
    coef[CF_MU3 * CSTR + j] = (float)mu;
    coef[CF_INV3 * CSTR + j] = (float)(1.0 / sqrt(var + (double)g.eps));
    float* rm3 = bn + 2 * g.F1 + 2 * g.F2;
    if (update_running) bn_running(rm3 + j, rm3 + g.F2 + j, mu, var, n3, g.mom);
}

// after pass C: classifier grads (+ clamp, model.py:84), BN3 grads and backward constants
__global__ __launch_bounds__(NT) void k_fin3(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             float* __restrict__ coef, float* __restrict__ grads,
                                             float* __restrict__ loss, int ce) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nC, sums);
    const int tid = threadIdx.x;
    const int n4 = NCLS * g.NF;
    for (int p = tid; p < n4; p += NT) {
        const float v = (float)sums[p];
        grads[g.o_Wfc + p] = g.noclamp ? v : fminf(fmaxf(v, -0.25f), 0.25f);
    }
    if (tid < NCLS) grads[g.o_bfc + tid] = (float)sums[n4 + tid];
    if (tid < g.F2) {
        const int j = tid;
        const double sdz = sums[n4 + NCLS + j], sdzx = sums[n4 + NCLS + g.F2 + j];
        grads[g.o_b3 + j] = (float)sdz;
        grads[g.o_g3 + j] = (float)sdzx;
        const double n3 = (double)g.B * g.T1;
        const double A = (double)prm[g.o_g3 + j] * (double)coef[CF_INV3 * CSTR + j];
        coef[CF_A3 * CSTR + j] = (float)A;
        coef[CF_B3 * CSTR + j] = (float)(-A * sdz / n3);
        coef[CF_C3 * CSTR + j] = (float)(-A * sdzx / n3);
    }
    if (tid == 0 && ce) {
        const float l = (float)(sums[n4 + NCLS + 2 * g.F2] / (double)g.B);
        coef[CF_LOSS * CSTR] = l;
        if (loss) *loss = l;
    }
}

// after pass D: block_2 grads, BN2 grads and the dy2 constants
__global__ __launch_bounds__(NT) void k_fin4(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             float* __restrict__ coef, float* __restrict__ grads) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nD, sums);
    const int tid = threadIdx.x;
    for (int p = tid; p < g.F2 * g.F2; p += NT) grads[g.o_W3 + p] = (float)sums[p];
    for (int p = tid; p < g.F2 * 16; p += NT) grads[g.o_w2 + p] = (float)sums[g.F2 * g.F2 + p];
    if (tid < g.F2) {
        const int o = tid;
        const double sdz = sums[g.F2 * g.F2 + 16 * g.F2 + o];
        const double sdzx = sums[g.F2 * g.F2 + 17 * g.F2 + o];
        grads[g.o_b2 + o] = (float)sdz;
        grads[g.o_g2 + o] = (float)sdzx;
        const double n2 = (double)g.B * g.T;
        const double A = (double)prm[g.o_g2 + o] * (double)coef[CF_INV2 * CSTR + o];
        coef[CF_AO * CSTR + o] = (float)A;
        coef[CF_BO * CSTR + o] = (float)(-A * sdz / n2);
        coef[CF_CO * CSTR + o] = (float)(-A * sdzx / n2);
    }
}

// after pass E: spatial grad (+ clamp, model.py:44), BN1 grads, temporal-conv grad
__global__ __launch_bounds__(NT) void k_fin5(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             const double* __restrict__ stats,
                                             const float* __restrict__ coef,
                                             float* __restrict__ grads) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nE, sums);
    __shared__ double db1s[64], dg1s[64];
    const int tid = threadIdx.x, K1 = g.K1;
    const double* Q = sums;
    const double* Xm = sums + g.F2 * K1;
    const double* Sdy = Xm + g.F2 * g.C;
    const double* Sdyv = Sdy + g.F2;
    const double* Gm = stats;
    const double* S1 = stats + K1 * K1;
    for (int p = tid; p < g.F2 * g.C; p += NT) {
        const int o = p / g.C, gg = o / g.D;
        const double v = (double)coef[CF_A1 * CSTR + gg] * Xm[p] + (double)coef[CF_C1 * CSTR + gg] * Sdy[o];
        grads[g.o_ws + p] = g.noclamp ? (float)v : fminf(fmaxf((float)v, -1.0f), 1.0f);
    }
    const double n1 = (double)g.B * g.C * g.T;
    if (tid < g.F1) {
        const int gg = tid;
        double db1 = 0.0, dyu = 0.0;
        for (int o = gg * g.D; o < (gg + 1) * g.D; ++o) {
            db1 += (double)coef[CF_W * CSTR + o] * Sdy[o];
            dyu += Sdyv[o];
        }
        const double inv1 = coef[CF_INV1 * CSTR + gg], mu1 = coef[CF_MU1 * CSTR + gg];
        const double dg1 = inv1 * (dyu - mu1 * db1);
        db1s[gg] = db1; dg1s[gg] = dg1;
        grads[g.o_b1 + gg] = (float)db1;
        grads[g.o_g1 + gg] = (float)dg1;
    }
    __syncthreads();
    for (int p = tid; p < g.F1 * K1; p += NT) {
        const int gg = p / K1, k = p - gg * K1;
        const float* w = prm + g.o_w1 + gg * K1;
        double qg = 0.0;
        for (int o = gg * g.D; o < (gg + 1) * g.D; ++o) qg += Q[o * K1 + k];
        double ux = 0.0;
        for (int l = 0; l < K1; ++l) ux += (double)w[l] * Gm[l * K1 + k];
        const double inv1 = coef[CF_INV1 * CSTR + gg], mu1 = coef[CF_MU1 * CSTR + gg];
        const double xhx = inv1 * (ux - mu1 * S1[k]);
        const double a1 = coef[CF_A1 * CSTR + gg];
        const double v = a1 * (qg - db1s[gg] / n1 * S1[k] - dg1s[gg] / n1 * xhx);
        grads[g.o_w1 + p] = (float)v;
    }
}

// torch.optim.Adam (weight_decay=0, amsgrad=False): torch/optim/adam.py:457,476,531-547
__global__ __launch_bounds__(NT) void k_adam(int64_t n, float* __restrict__ p, const float* __restrict__ gr,
                                             float* __restrict__ m, float* __restrict__ v,
                                             int32_t* __restrict__ step, float lr, float b1, float b2,
                                             float eps) {
    const int s = *step + 1;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) {
        const float g = gr[i];
        const float mi = m[i] + (1.f - b1) * (g - m[i]);
        const float vi = b2 * v[i] + (1.f - b2) * g * g;
        m[i] = mi; v[i] = vi;
        const double bc1 = 1.0 - pow((double)b1, (double)s);
        const double bc2 = 1.0 - pow((double)b2, (double)s);
        const float step_size = (float)(lr / bc1);
        const float bc2s = (float)sqrt(bc2);
        const float denom = sqrtf(vi) / bc2s + eps;
        p[i] = p[i] - step_size * (mi / denom);
    }
}

__global__ void k_step_inc(int32_t* step) { if (threadIdx.x == 0) *step += 1; }

// the two gradient hooks of model.py:44 and model.py:84, applied to a flat grad buffer
__global__ __launch_bounds__(NT) void k_clamp(Geo g, float* __restrict__ grads) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < g.F2 * g.C) grads[g.o_ws + i] = fminf(fmaxf(grads[g.o_ws + i], -1.0f), 1.0f);
    if (i < NCLS * g.NF) grads[g.o_Wfc + i] = fminf(fmaxf(grads[g.o_Wfc + i], -0.25f), 0.25f);
}

}  // namespace eeg

// ================================================================================================
// Host side: geometry, validation, launch sequences, C-ABI.
// ================================================================================================
using namespace eeg;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

static inline int rup(int a, int m) { return (a + m - 1) / m * m; }
static inline size_t rupz(size_t a, size_t m) { return (a + m - 1) / m * m; }

struct WsLayout {
    size_t partA, partB, partC, partD, partE, sums, stats, coef, d2, E1, E2, dp2, dl, total;
};

static int make_geo(const eegnet_dims* d, Geo* g, bool launch = true) {
    if (!d) return fail(EEGNET_EINVAL, "dims is NULL");
    memset(g, 0, sizeof(*g));
    g->B = d->B; g->C = d->C; g->T = d->T; g->F1 = d->F1; g->D = d->D; g->K1 = d->K1;
    g->F2 = d->F1 * d->D;
    if (g->B < 1) return fail(EEGNET_EINVAL, "B must be >= 1 (got %d)", g->B);
    if (g->K1 != 32 && g->K1 != 64) return fail(EEGNET_EINVAL, "K1 must be 32 or 64 (got %d)", g->K1);
    if (g->C < 1 || g->C > 64) return fail(EEGNET_EINVAL, "C must be in [1,64] (got %d)", g->C);
    if (g->F1 < 1 || g->D < 1 || g->F2 > 64 || (g->F2 & 3))
        return fail(EEGNET_EINVAL, "F1*D must be a multiple of 4 in [4,64] (got F1=%d D=%d)", g->F1, g->D);
    if (g->T < 32 || g->T < g->K1 || g->T > 2048)
        return fail(EEGNET_EINVAL, "T must be in [max(32,K1), 2048] (got %d)", g->T);
    g->P = (g->K1 - 1) / 2; g->R = g->K1 - 1 - g->P;
    g->T1 = g->T / 4; g->T2 = g->T1 / 8; g->NF = g->F2 * g->T2;
    g->LP = (g->R + 3) & ~3;
    g->TQ = (g->T + 3) / 4; g->NT16 = (g->T + 15) / 16;
    {
        const int OFF = g->LP - g->P;
        const int NW = (OFF + g->K1 + 6) / 4;
        int rs = std::max(4 * (g->TQ - 1) + 4 * NW, g->LP + 16 * g->NT16);
        rs = std::max(rs, g->LP + g->T + g->R);
        rs = rup(rs, 4);
        if (((rs / 4) & 1) == 0) rs += 4;
        g->RS = rs;
    }
    g->nseg = NT / g->F2;
    g->nsegC = NT / g->C;
    g->TQ1 = (g->T1 + 3) / 4;
    g->RS2 = rup(std::max(4 * g->TQ1 + 20, LP2 + g->T1 + 8 + 4), 4);
    g->FO = rup(g->F2, 16); g->CK = rup(g->C, 4); g->NCT = (g->C + 15) / 16;
    g->npairs = g->K1 * (g->K1 - 1) / 2;
    g->p = d->p_drop; g->eps = d->bn_eps; g->mom = d->bn_momentum;
    if (!(g->p >= 0.f && g->p <= 1.f)) return fail(EEGNET_EINVAL, "p_drop must be in [0,1]");
    g->scale = g->p < 1.f ? 1.f / (1.f - g->p) : 0.f;
    // parameter offsets (named_parameters order)
    int o = 0;
    g->o_w1 = o; o += g->F1 * g->K1;
    g->o_g1 = o; o += g->F1;
    g->o_b1 = o; o += g->F1;
    g->o_ws = o; o += g->F2 * g->C;
    g->o_g2 = o; o += g->F2;
    g->o_b2 = o; o += g->F2;
    g->o_w2 = o; o += g->F2 * 16;
    g->o_W3 = o; o += g->F2 * g->F2;
    g->o_g3 = o; o += g->F2;
    g->o_b3 = o; o += g->F2;
    g->o_Wfc = o; o += NCLS * g->NF;
    g->o_bfc = o; o += NCLS;
    g->nparam = o;
    if (g->NF < 1) return fail(EEGNET_EINVAL, "T//32 must be >= 1");
    // partial rows
    g->nA = 2 * g->K1 + g->npairs + 2 * g->F2;
    g->nB = 2 * g->F2;
    g->nC = NCLS * g->NF + NCLS + 2 * g->F2 + 1;
    g->nD = g->F2 * g->F2 + 18 * g->F2;
    g->nE = g->F2 * g->K1 + g->F2 * g->C + 2 * g->F2;
    const int cap = 256 * 3;
    g->gA = std::min(g->B, cap); g->gB = std::min(g->B, cap); g->gE = std::min(g->B, cap);
    g->gC = std::min(g->B, 1024); g->gD = std::min(g->B, 1024);
    // LDS sizes (floats)
    const int wsh = rup(g->FO * (g->CK + 1), 4);
    const int rows = (g->C + g->F2) * g->RS;
    const int b2 = 3 * g->F2 * g->RS2 + g->F2 * 16 + rup(g->F2 * g->F2, 4);
    g->ldsA = rows + wsh + 2 * NT;
    g->ldsB = rows + b2 + wsh;
    g->ldsC = b2 + 2 * rup(g->NF, 4) + rup(4 * g->NF + 4, 4) + 8;
    g->ldsD = 5 * g->F2 * g->RS2 + g->F2 * 16 + rup(g->F2 * g->F2, 4) + rup(g->NF, 4) +
              g->F2 * g->F2 + 18 * g->F2;
    {
        const int xr = 4 * g->FO * 16 * g->NCT;    // Xm reduction scratch (reuses Xs)
        if (launch && xr > (g->C + 2 * g->F2) * g->RS)
            return fail(EEGNET_EINVAL, "internal: Xm scratch does not fit");
    }
    g->ldsE = rows + g->F2 * g->RS + rup(g->F2 * g->T1, 4) + wsh + 2 * NT;
    g->ldsI = rows + b2 + wsh + rup(g->NF, 4) + 4 * g->F2;
    const int lmax = std::max(std::max(std::max(g->ldsA, g->ldsB), std::max(g->ldsC, g->ldsD)),
                              std::max(g->ldsE, g->ldsI));
    if (launch && lmax * 4 > 160 * 1024) return fail(EEGNET_EINVAL, "dims need %d B of LDS (> 160 KiB)", lmax * 4);
    return 0;
}

static WsLayout make_layout(const Geo& g) {
    WsLayout L;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = rupz(o + bytes, 256); return r; };
    L.partA = take((size_t)g.gA * g.nA * 4);
    L.partB = take((size_t)g.gB * g.nB * 4);
    L.partC = take((size_t)g.gC * g.nC * 4);
    L.partD = take((size_t)g.gD * g.nD * 4);
    L.partE = take((size_t)g.gE * g.nE * 4);
    const int nmax = std::max(std::max(std::max(g.nA, g.nB), std::max(g.nC, g.nD)), g.nE);
    L.sums = take((size_t)nmax * 8 * RCH);
    L.stats = take((size_t)(g.K1 * g.K1 + g.K1) * 8);
    L.coef = take((size_t)CF_COUNT * CSTR * 4);
    const size_t per = (size_t)g.B * g.F2 * g.T1 * 4;
    L.d2 = take(per); L.E1 = take(per); L.E2 = take(per); L.dp2 = take(per);
    L.dl = take((size_t)g.B * NCLS * 4);
    L.total = o;
    return L;
}

static uint64_t mix_key(uint64_t seed, uint64_t offset) {
    uint64_t z = seed * 0xD1B54A32D192ED03ull + offset * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---- optional per-kernel device timing (bench / roofline), off by default ----
enum KernelId { KID_A = 0, KID_B, KID_C, KID_D, KID_E, KID_COLSUM, KID_FIN, KID_ADAM, KID_INFER, KID_COUNT };
static const char* kKernelNames[KID_COUNT] = {"k_pass_a", "k_pass_b", "k_pass_c", "k_pass_d", "k_pass_e",
                                              "k_colsum", "k_fin", "k_adam", "k_infer"};
struct ProfRec { int kid; hipEvent_t a, b; };
struct ProfState { bool on = false; std::vector<ProfRec> recs; std::vector<hipEvent_t> pool; };
static thread_local ProfState g_prof;

static hipEvent_t prof_event() {
    if (!g_prof.pool.empty()) { hipEvent_t e = g_prof.pool.back(); g_prof.pool.pop_back(); return e; }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}
struct ProfScope {
    int kid; hipStream_t s; hipEvent_t a = nullptr;
    ProfScope(int k, hipStream_t st) : kid(k), s(st) {
        if (g_prof.on) { a = prof_event(); hipEventRecord(a, s); }
    }
    ~ProfScope() {
        if (a) { hipEvent_t b = prof_event(); hipEventRecord(b, s); g_prof.recs.push_back({kid, a, b}); }
    }
};
#define PROF(kid) ProfScope prof_scope_##kid(kid, s)

#define LAUNCH_CHECK(what)                                                            \
    do {                                                                              \
        hipError_t e_ = hipGetLastError();                                            \
        if (e_ != hipSuccess) return fail(EEGNET_ELAUNCH, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

static bool g_attr_done = false;

template <int K1>
static void set_attrs() {
    hipFuncSetAttribute((const void*)k_pass_a<K1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_pass_b<K1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_pass_e<K1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_infer<K1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

static void ensure_attrs() {
    if (g_attr_done) return;
    set_attrs<32>();
    set_attrs<64>();
    hipFuncSetAttribute((const void*)k_pass_c, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_pass_d, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_fin1, hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024);
    g_attr_done = true;
}

static int colsum(const float* part, int nrows, int ncols, double* out, hipStream_t s) {
    PROF(KID_COLSUM);
    hipLaunchKernelGGL(k_colsum, dim3((ncols + 63) / 64, RCH), dim3(NT), 0, s, part, nrows, ncols, out);
    LAUNCH_CHECK("k_colsum");
    return 0;
}

template <int K1>
static int run_forward(const Geo& g, const WsLayout& L, char* ws, const float* params, float* bn,
                       const float* x, const uint8_t* m2, float* logits, int update_running,
                       int c_mode, const int64_t* labels, float* loss, float* grads, hipStream_t s) {
    double* sums = (double*)(ws + L.sums);
    float* coef = (float*)(ws + L.coef);
    { PROF(KID_A); hipLaunchKernelGGL(k_pass_a<K1>, dim3(g.gA), dim3(NT), g.ldsA * 4, s, g, params, x, (float*)(ws + L.partA));
    } LAUNCH_CHECK("k_pass_a");
    if (int r = colsum((float*)(ws + L.partA), g.gA, g.nA, sums, s)) return r;
    { PROF(KID_FIN); hipLaunchKernelGGL(k_fin1, dim3(1), dim3(NT), (g.K1 * g.K1 + g.K1 + 128 + g.nA) * 8, s, g, params, sums,
                       (double*)(ws + L.stats), coef, bn, update_running);
    } LAUNCH_CHECK("k_fin1");
    { PROF(KID_B); hipLaunchKernelGGL(k_pass_b<K1>, dim3(g.gB), dim3(NT), g.ldsB * 4, s, g, params, coef, x, m2,
                       (float*)(ws + L.d2), (float*)(ws + L.E1), (float*)(ws + L.E2), (float*)(ws + L.partB));
    } LAUNCH_CHECK("k_pass_b");
    if (int r = colsum((float*)(ws + L.partB), g.gB, g.nB, sums, s)) return r;
    { PROF(KID_FIN); hipLaunchKernelGGL(k_fin2, dim3(1), dim3(NT), g.nB * 8, s, g, sums, coef, bn, update_running);
    } LAUNCH_CHECK("k_fin2");
    (void)labels; (void)loss; (void)grads; (void)c_mode; (void)logits;
    return 0;
}

template <int K1>
static int run_backward(const Geo& g, const WsLayout& L, char* ws, const float* params,
                        const float* x, const uint8_t* m2, const uint8_t* m3, const float* dlogits,
                        const int64_t* labels, float* logits, float* grads, float* loss, int c_mode,
                        hipStream_t s) {
    double* sums = (double*)(ws + L.sums);
    float* coef = (float*)(ws + L.coef);
    float* dl = dlogits ? (float*)dlogits : (float*)(ws + L.dl);
    { PROF(KID_C); hipLaunchKernelGGL(k_pass_c, dim3(g.gC), dim3(NT), g.ldsC * 4, s, g, params, coef,
                       (const float*)(ws + L.d2), m3, dlogits, labels, logits, (float*)(ws + L.dl),
                       (float*)(ws + L.partC), c_mode);
    } LAUNCH_CHECK("k_pass_c(bwd)");
    if (int r = colsum((float*)(ws + L.partC), g.gC, g.nC, sums, s)) return r;
    { PROF(KID_FIN); hipLaunchKernelGGL(k_fin3, dim3(1), dim3(NT), g.nC * 8, s, g, params, sums, coef, grads, loss,
                       (c_mode & PC_CE) ? 1 : 0);
    } LAUNCH_CHECK("k_fin3");
    { PROF(KID_D); hipLaunchKernelGGL(k_pass_d, dim3(g.gD), dim3(NT), g.ldsD * 4, s, g, params, coef,
                       (const float*)(ws + L.d2), (const float*)(ws + L.E1), (const float*)(ws + L.E2),
                       m2, m3, (const float*)dl, (float*)(ws + L.dp2), (float*)(ws + L.partD));
    } LAUNCH_CHECK("k_pass_d");
    if (int r = colsum((float*)(ws + L.partD), g.gD, g.nD, sums, s)) return r;
    { PROF(KID_FIN); hipLaunchKernelGGL(k_fin4, dim3(1), dim3(NT), g.nD * 8, s, g, params, sums, coef, grads);
    } LAUNCH_CHECK("k_fin4");
    { PROF(KID_E); hipLaunchKernelGGL(k_pass_e<K1>, dim3(g.gE), dim3(NT), g.ldsE * 4, s, g, params, coef, x,
                       (const float*)(ws + L.dp2), (float*)(ws + L.partE));
    } LAUNCH_CHECK("k_pass_e");
    if (int r = colsum((float*)(ws + L.partE), g.gE, g.nE, sums, s)) return r;
    { PROF(KID_FIN); hipLaunchKernelGGL(k_fin5, dim3(1), dim3(NT), g.nE * 8, s, g, params, sums, (const double*)(ws + L.stats),
                       (const float*)coef, grads);
    } LAUNCH_CHECK("k_fin5");
    return 0;
}

static int check_ptrs(const void* a, const char* na, const void* b = (const void*)1, const char* nb = "") {
    if (!a) return fail(EEGNET_EINVAL, "%s is NULL", na);
    if (!b) return fail(EEGNET_EINVAL, "%s is NULL", nb);
    return 0;
}

extern "C" {

int eegnet_param_count(const eegnet_dims* dims, int64_t* out) {
    Geo g;
    if (int r = make_geo(dims, &g, false)) return r;
    if (!out) return fail(EEGNET_EINVAL, "out is NULL");
    *out = g.nparam;
    return 0;
}

int eegnet_workspace_bytes(const eegnet_dims* dims, size_t* out) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (!out) return fail(EEGNET_EINVAL, "out is NULL");
    *out = make_layout(g).total;
    return 0;
}

int eegnet_forward_train(const eegnet_dims* dims, const float* params, float* bn_buffers,
                         const float* x, const uint8_t* mask2, const uint8_t* mask3,
                         uint64_t seed, uint64_t offset, float* logits, void* ws, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", logits, "logits")) return r;
    if (int r = check_ptrs(ws, "ws")) return r;
    g.drop = g.p > 0.f ? 1 : 0;
    g.key = mix_key(seed, offset);
    ensure_attrs();
    const WsLayout L = make_layout(g);
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    int r = g.K1 == 32 ? run_forward<32>(g, L, w, params, bn_buffers, x, mask2, logits, 1, 0, nullptr, nullptr, nullptr, s)
                       : run_forward<64>(g, L, w, params, bn_buffers, x, mask2, logits, 1, 0, nullptr, nullptr, nullptr, s);
    if (r) return r;
    { PROF(KID_C); hipLaunchKernelGGL(k_pass_c, dim3(g.gC), dim3(NT), g.ldsC * 4, s, g, params, (const float*)(w + L.coef),
                       (const float*)(w + L.d2), mask3, (const float*)nullptr, (const int64_t*)nullptr,
                       logits, (float*)nullptr, (float*)nullptr, (int)PC_LOGITS);
    } LAUNCH_CHECK("k_pass_c(fwd)");
    return 0;
}

int eegnet_backward(const eegnet_dims* dims, const float* params, const float* x,
                    const float* dlogits, const int64_t* labels, const uint8_t* mask2,
                    const uint8_t* mask3, uint64_t seed, uint64_t offset, float* grads, float* loss,
                    void* ws, void* stream, int flags) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    g.noclamp = (flags & EEGNET_NO_CLAMP) ? 1 : 0;
    if (int r = check_ptrs(params, "params", x, "x")) return r;
    if (int r = check_ptrs(grads, "grads", ws, "ws")) return r;
    if (!dlogits && !labels) return fail(EEGNET_EINVAL, "need dlogits or labels");
    g.drop = g.p > 0.f ? 1 : 0;
    g.key = mix_key(seed, offset);
    ensure_attrs();
    const WsLayout L = make_layout(g);
    const int mode = PC_BWD | (dlogits ? 0 : PC_CE);
    hipStream_t s = (hipStream_t)stream;
    return g.K1 == 32
        ? run_backward<32>(g, L, (char*)ws, params, x, mask2, mask3, dlogits, labels, nullptr, grads, loss, mode, s)
        : run_backward<64>(g, L, (char*)ws, params, x, mask2, mask3, dlogits, labels, nullptr, grads, loss, mode, s);
}

int eegnet_forward_eval(const eegnet_dims* dims, const float* params, const float* bn_buffers,
                        const float* x, float* logits, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", logits, "logits")) return r;
    ensure_attrs();
    hipStream_t s = (hipStream_t)stream;
    const int grid = std::min(g.B, 1024);
    PROF(KID_INFER);
    if (g.K1 == 32)
        hipLaunchKernelGGL(k_infer<32>, dim3(grid), dim3(NT), g.ldsI * 4, s, g, params, bn_buffers, x, logits);
    else
        hipLaunchKernelGGL(k_infer<64>, dim3(grid), dim3(NT), g.ldsI * 4, s, g, params, bn_buffers, x, logits);
    LAUNCH_CHECK("k_infer");
    return 0;
}

int eegnet_adam_step(int64_t n, float* params, const float* grads, float* exp_avg,
                     float* exp_avg_sq, int32_t* step, float lr, float beta1, float beta2,
                     float eps, void* stream) {
    if (n <= 0) return fail(EEGNET_EINVAL, "n must be > 0");
    if (!params || !grads || !exp_avg || !exp_avg_sq || !step) return fail(EEGNET_EINVAL, "null pointer");
    hipStream_t s = (hipStream_t)stream;
    { PROF(KID_ADAM); hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, s, n, params, grads,
                       exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps);
    } LAUNCH_CHECK("k_adam");
    hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(64), 0, s, step);
    LAUNCH_CHECK("k_step_inc");
    return 0;
}

int eegnet_train_step(const eegnet_dims* dims, float* params, float* bn_buffers, const float* x,
                      const int64_t* labels, uint64_t seed, uint64_t offset, float* grads,
                      float* adam_state, int32_t* step, float lr, float beta1, float beta2,
                      float eps, float* loss, float* logits, void* ws, void* stream, int flags) {
    Geo g;
    if (int r = make_geo(dims, &g)) return r;
    if (int r = check_ptrs(params, "params", bn_buffers, "bn_buffers")) return r;
    if (int r = check_ptrs(x, "x", labels, "labels")) return r;
    if (int r = check_ptrs(grads, "grads", ws, "ws")) return r;
    if (adam_state && !step) return fail(EEGNET_EINVAL, "step is NULL");
    g.noclamp = (flags & EEGNET_NO_CLAMP) ? 1 : 0;
    g.drop = g.p > 0.f ? 1 : 0;
    g.key = mix_key(seed, offset);
    ensure_attrs();
    const WsLayout L = make_layout(g);
    hipStream_t s = (hipStream_t)stream;
    char* w = (char*)ws;
    int r = g.K1 == 32 ? run_forward<32>(g, L, w, params, bn_buffers, x, nullptr, nullptr, 1, 0, nullptr, nullptr, nullptr, s)
                       : run_forward<64>(g, L, w, params, bn_buffers, x, nullptr, nullptr, 1, 0, nullptr, nullptr, nullptr, s);
    if (r) return r;
    const int mode = PC_BWD | PC_CE | (logits ? PC_LOGITS : 0);
    r = g.K1 == 32
        ? run_backward<32>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, logits, grads, loss, mode, s)
        : run_backward<64>(g, L, w, params, x, nullptr, nullptr, nullptr, labels, logits, grads, loss, mode, s);
    if (r) return r;
    if (!adam_state) return 0;       // gradients only (data-parallel: all-reduce, clamp, then Adam)
    return eegnet_adam_step(g.nparam, params, grads, adam_state, adam_state + g.nparam, step, lr,
                            beta1, beta2, eps, stream);
}

int eegnet_clamp_grads(const eegnet_dims* dims, float* grads, void* stream) {
    Geo g;
    if (int r = make_geo(dims, &g, false)) return r;
    if (!grads) return fail(EEGNET_EINVAL, "grads is NULL");
    hipStream_t s = (hipStream_t)stream;
    const int n = std::max(g.F2 * g.C, NCLS * g.NF);
    hipLaunchKernelGGL(k_clamp, dim3((n + NT - 1) / NT), dim3(NT), 0, s, g, grads);
    LAUNCH_CHECK("k_clamp");
    return 0;
}

const char* eegnet_last_error(void) { return g_err.c_str(); }

int eegnet_profile_enable(int on) {
    g_prof.on = on != 0;
    return 0;
}

int eegnet_profile_collect(char* names, int* counts, double* total_ms, int cap, int* n_out) {
    double tot[KID_COUNT] = {0};
    int cnt[KID_COUNT] = {0};
    for (auto& r : g_prof.recs) {
        hipEventSynchronize(r.b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, r.a, r.b);
        tot[r.kid] += ms;
        cnt[r.kid] += 1;
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.recs.clear();
    int n = 0;
    for (int k = 0; k < KID_COUNT && n < cap; ++k) {
        if (!cnt[k]) continue;
        if (names) { strncpy(names + 32 * n, kKernelNames[k], 31); names[32 * n + 31] = 0; }
        if (counts) counts[n] = cnt[k];
        if (total_ms) total_ms[n] = tot[k];
        ++n;
    }
    if (n_out) *n_out = n;
    return 0;
}

const char* eegnet_build_info(void) {
    return "libeegnet_hip: gfx950 (CDNA4), fp32 VALU FIR/Gram + f32 MFMA 16x16x4 GEMMs, "
           "5-pass restructured EEGNet train step";
}

}  // extern "C"
