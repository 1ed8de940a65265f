// eegnet_infer_bf16.hip -- bf16 batched eval-mode forward (BASELINE cfg5:
// EEGNet-16,4 on 64ch x 512 high-density EEG).  Included by eegnet_kernels.hip (one translation unit).
//
// Reference: EEGNet.forward in eval mode, src/eegnet_repl/model.py:91-99 (called at model.py:161,220
// and ui.py:35).  Eval BatchNorm is affine, so conv1 -> BN1 -> spatial collapses to
//     s[o,t]  = sum_c ws[o,c] x[c,t]                   spatial GEMM  (bf16 MFMA 16x16x32, K = c)
//     v[o,t]  = sum_k w1[o/D,k] s[o,t+k-P]             temporal FIR  (bf16 MFMA: banded Toeplitz)
//     a[o,q]  = 1/4 sum_{t in 4q..4q+3} ELU(al[o] v[o,t] + be[o])      BN1+BN2 folded, ELU, pool4
//     z[o,q]  = sum_k w2[o,k] a[o,q+k-7]               depthwise 1x16 (fp32 VALU)
//     r[j,q]  = sum_i W3[j,i] z[i,q]                   pointwise      (bf16 MFMA 16x16x32, K = i)
//     h[j,u]  = 1/8 sum ELU(s3[j] r[j,q] + b3[j])      BN3 folded, ELU, pool8;  logits = Wfc h + bfc
// Operands are bf16 (x arrives as bf16: 64 KB per cfg5 trial, the HBM floor of the path), every
// accumulation is fp32.  One 512-thread workgroup per CU streams whole trials through LDS; the next
// trial's x is in flight in registers during the current trial's compute.
//
// MFMA operand images.  Both GEMMs contract over a ROW index of a row-major [row][time] plane (x over
// electrodes c, z over rows i), so their time-major operand is read with ds_read_b64_tr_b16 (the
// gfx950 transposing LDS read) from an image whose 8-byte chunks are XOR-swizzled per row:
// chunk' = chunk ^ 4*h(row), h(row) = (row & 3) | ((row >> 1) & 4), rows a multiple of 128 elements.
// A 32-lane half of one transposed read then touches 8 distinct h x 4 chunks = all 64 banks.
// The FIR contracts over time, so its window operand is a plain 16-byte ds_read_b128 of an s row.
#pragma once

namespace eeg {

constexpr int NTI = 512;               // threads of the bf16 eval workgroup (8 waves, 2 per SIMD)
constexpr int NWI = NTI / 64;
constexpr int LAI = 8;                 // left pad of the pooled rows a[o,.] (>= 7, multiple of 4)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
typedef unsigned uintx2 __attribute__((ext_vector_type(2)));

struct GeoI {
    int B, C, T, F1, D, F2, K1, P;
    int CP, KC;            // C padded to 32; K-steps of the spatial GEMM
    int F2P, NOT;          // rows padded to 16 / 32 / 64; 16-row tiles
    int F2K, KCW;          // pointwise contraction rows (F2P padded to 32); its K-steps
    int TX;                // x image row (elements, multiple of 128)
    int NT, NBLK;          // 16-sample output tiles of s / v; 16-tile FIR column blocks
    int LPs, KSF, SXs;     // s rows: left pad (P+1), FIR K-steps, row stride (elements)
    int T1, T2, NF;        // pooled lengths, classifier inputs F2*T2
    int RA, TZ, NT1;       // a row stride (floats), z image row (elements), pointwise 16-col tiles
    int PFU;               // 16-byte x units per thread (0: T % 8 != 0, element staging)
    float eps;
    int o_w1, o_g1, o_b1, o_ws, o_g2, o_b2, o_w2, o_W3, o_g3, o_b3, o_Wfc, o_bfc;
    int offZ, offS, offW1, offW2, offCo, offL, lds;     // LDS carve (bytes)
    int offF;              // classifier weights [NCLS][NF] fp32 in LDS (0: read from global)
    float* dbg;            // eegnet_debug_bf16: workgroup 0's first trial's s, a, z planes (fp32)
};

// swizzled byte offset of 8-byte chunk `ch` of row `r` in a transposed-read image with rows of
// `rowb` bytes
__device__ __forceinline__ int trimg_off(int r, int ch, int rowb) {
    const int h = (r & 3) | ((r >> 1) & 4);
    return r * rowb + 8 * (ch ^ (4 * h));
}

__device__ __forceinline__ shortx4 lds_tr16(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) shortx4*)(p));
}

// MFMA operand fragment of a [k][n] image read transposed: lane l gets B[k = k0 + 8(l>>4) + j][n0 + l&15]
// (equally A[m = n0 + l&15][k] of the transposed plane) for j = 0..7: two 4-row transposed reads.
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int rowb, int k0, int n0, int lane) {
    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r = k0 + 8 * G + q;
    const int ch = (n0 >> 2) + p;
    const shortx4 lo = lds_tr16(img + trimg_off(r, ch, rowb));
    const shortx4 hi = lds_tr16(img + trimg_off(r + 4, ch, rowb));
    const shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ floatx4 mfma_bf16(bf16x8 a, bf16x8 b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
    const unsigned short lo = __builtin_bit_cast(unsigned short, (__bf16)a);
    const unsigned short hi = __builtin_bit_cast(unsigned short, (__bf16)b);
    return (unsigned)lo | ((unsigned)hi << 16);
}

// x staging, 16-byte path (T % 8 == 0): image unit u = tid + NTI*j covers row c = u / (TX/8),
// samples 8*(u % (TX/8)) .. +7; units outside [0,C) x [0,T) are the image's zero padding
template <int PFU>
__device__ __forceinline__ void xi_load(const GeoI& g, const uint16_t* __restrict__ xb, uintx4 (&pf)[PFU], int tid) {
    const int upr = g.TX >> 3;
#pragma unroll
    for (int j = 0; j < PFU; ++j) {
        const int u = tid + NTI * j;
        const int c = u / upr, tt = 8 * (u - c * upr);
        if (c < g.C && tt < g.T)
            pf[j] = __builtin_nontemporal_load(reinterpret_cast<const uintx4*>(xb + (size_t)c * g.T + tt));
        else
            pf[j] = (uintx4){0u, 0u, 0u, 0u};
    }
}
template <int PFU>
__device__ __forceinline__ void xi_store(const GeoI& g, const uintx4 (&pf)[PFU], char* Xi, int tid) {
    const int upr = g.TX >> 3, rowb = 2 * g.TX;
#pragma unroll
    for (int j = 0; j < PFU; ++j) {
        const int u = tid + NTI * j;
        const int c = u / upr, ch = 2 * (u - c * upr);
        if (c < g.CP) *reinterpret_cast<uintx4*>(Xi + trimg_off(c, ch, rowb)) = pf[j];
    }
}
// element path for T % 8 != 0 (e.g. T = 257): no prefetch, 2-byte loads
__device__ __forceinline__ void xi_stage_elems(const GeoI& g, const uint16_t* __restrict__ xb, char* Xi, int tid) {
    const int rowb = 2 * g.TX;
    for (int i = tid; i < g.CP * g.TX; i += NTI) {
        const int c = i / g.TX, t = i - c * g.TX;
        const uint16_t v = (c < g.C && t < g.T) ? xb[(size_t)c * g.T + t] : (uint16_t)0;
        *reinterpret_cast<uint16_t*>(Xi + trimg_off(c, t >> 2, rowb) + 2 * (t & 3)) = v;
    }
}

// Compile-time geometry of BASELINE cfg5 (EEGNet-16,4 on 64ch x 512): the values make_geo_bf16
// computes for those dims.  The host launches the CFG5 instantiation only when its runtime geometry
// equals this one field for field (B, eps and dbg excepted), so every loop bound, stride and LDS
// offset below folds to a constant there.
constexpr GeoI kGeoCfg5 = {
    0, 64, 512, 16, 4, 64, 32, 15,          // B, C, T, F1, D, F2, K1, P
    64, 2, 64, 4, 64, 2, 512,               // CP, KC, F2P, NOT, F2K, KCW, TX
    32, 2, 16, 2, 568,                      // NT, NBLK, LPs, KSF, SXs
    128, 16, 1024, 144, 128, 8, 8,          // T1, T2, NF, RA, TZ, NT1, PFU
    1e-5f,                                  // eps (runtime)
    0, 512, 528, 544, 4640, 4704, 4768, 5792, 9888, 9952, 10016, 14112,   // o_w1 .. o_bfc
    36864, 65536, 138240, 140288, 144384, 145408, 161920,                 // offZ .. offL, lds
    145536,                                 // offF
    nullptr};

template <int PFU, bool CFG5 = false>
__global__ __launch_bounds__(NTI) void k_infer_bf16(GeoI gin, const float* __restrict__ prm,
                                                    const float* __restrict__ bn,
                                                    const uint16_t* __restrict__ x, float* __restrict__ logits) {
    GeoI g = gin;
    if constexpr (CFG5) {
        g = kGeoCfg5;
        g.B = gin.B; g.eps = gin.eps; g.dbg = gin.dbg;
    }
    extern __shared__ __attribute__((aligned(16))) char smi[];
    char* const Xi = smi;                                   // x image (bf16, swizzled)
    float* const Aa = reinterpret_cast<float*>(smi);        // pooled rows a (fp32), aliases Xi
    char* const Zi = smi + g.offZ;                          // z image (bf16, swizzled), aliases Xi
    char* const Si = smi + g.offS;                          // s rows (bf16)
    float* const W1t = reinterpret_cast<float*>(smi + g.offW1);
    float* const W2t = reinterpret_cast<float*>(smi + g.offW2);
    float* const Co = reinterpret_cast<float*>(smi + g.offCo);   // [4][F2P]: al, be, s3, b3
    float* const Lg = reinterpret_cast<float*>(smi + g.offL);    // [NWI][4] logit partials
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = lane >> 4, l15 = lane & 15;
    const int F2 = g.F2, F2P = g.F2P, C = g.C;
    const int xrow = 2 * g.TX, srow = 2 * g.SXs, zrow = 2 * g.TZ;

    // ---- prologue: folded BN constants, tap tables, zero s rows (their pads stay zero) ----
    if (tid < F2P) {
        const int o = tid;
        float al = 0.f, be = 0.f, s3 = 0.f, b3 = 0.f;
        if (o < F2) {
            const int gg = o / g.D;
            const float* rm1 = bn;             const float* rv1 = bn + g.F1;
            const float* rm2 = bn + 2 * g.F1;  const float* rv2 = rm2 + F2;
            const float* rm3 = rm2 + 2 * F2;   const float* rv3 = rm3 + F2;
            const float a1 = prm[g.o_g1 + gg] / sqrtf(rv1[gg] + g.eps);
            const float c1 = prm[g.o_b1 + gg] - a1 * rm1[gg];
            float W = 0.f;
            for (int c = 0; c < C; ++c) W += prm[g.o_ws + o * C + c];
            const float s2 = prm[g.o_g2 + o] / sqrtf(rv2[o] + g.eps);
            al = a1 * s2;
            be = (c1 * W - rm2[o]) * s2 + prm[g.o_b2 + o];
            s3 = prm[g.o_g3 + o] / sqrtf(rv3[o] + g.eps);
            b3 = prm[g.o_b3 + o] - rm3[o] * s3;
        }
        Co[o] = al; Co[F2P + o] = be; Co[2 * F2P + o] = s3; Co[3 * F2P + o] = b3;
    }
    for (int i = tid; i < g.F1 * g.K1; i += NTI) W1t[i] = prm[g.o_w1 + i];
    for (int i = tid; i < F2P * K2; i += NTI) W2t[i] = (i / K2) < F2 ? prm[g.o_w2 + i] : 0.f;
    for (int i = tid; i < F2P * g.SXs / 2; i += NTI) reinterpret_cast<unsigned*>(Si)[i] = 0u;
    float* const Wf = reinterpret_cast<float*>(smi + g.offF);
    if (g.offF)
        for (int i = tid; i < NCLS * g.NF; i += NTI) Wf[i] = prm[g.o_Wfc + i];

    // spatial GEMM B operand (ws^T, K = c): this wave's 16-row o-tile, all K-steps, in registers
    const int ot = wave % g.NOT, wpo = NWI / g.NOT;
    bf16x8 wsf[2];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
        const int o = ot * 16 + l15;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = kc * 32 + 8 * G + j;
            wsf[kc][j] = (__bf16)((kc < g.KC && o < F2 && c < C) ? prm[g.o_ws + o * C + c] : 0.f);
        }
    }
    // pointwise A operand (W3, K = i): this wave's 16-row j-tile
    bf16x8 w3f[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int j0 = ot * 16 + l15;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = ks * 32 + 8 * G + j;
            w3f[ks][j] = (__bf16)((ks < g.KCW && j0 < F2 && i < F2) ? prm[g.o_W3 + j0 * F2 + i] : 0.f);
        }
    }

    uintx4 pf[PFU > 0 ? PFU : 1];
    int b = blockIdx.x;
    if constexpr (PFU > 0) {
        if (b < g.B) {
            xi_load<PFU>(g, x + (size_t)b * C * g.T, pf, tid);
            xi_store<PFU>(g, pf, Xi, tid);
        }
        if (b + (int)gridDim.x < g.B) xi_load<PFU>(g, x + (size_t)(b + gridDim.x) * C * g.T, pf, tid);
    } else {
        if (b < g.B) xi_stage_elems(g, x + (size_t)b * C * g.T, Xi, tid);
    }
    __syncthreads();

    const int rpw = F2P / NWI;                 // FIR rows per wave (>= 1)
    for (; b < g.B; b += gridDim.x) {
        // ---- 1. spatial GEMM: s^T[t, o] tiles (16 t x 16 o), A = x^T by transposed reads ----
        // two t-tiles per iteration: all transposed reads issue before the first MFMA (the s
        // stores of the previous iteration may alias Xi as far as the compiler knows)
        auto s_store = [&](const floatx4& acc, int n) {
            // lane: s[o = ot*16 + l15][t = 16n + 4G + r], r = 0..3 -> one 8-byte store
            const int o = ot * 16 + l15;
            uintx2 pk;
            pk[0] = pack_bf16x2(acc[0], acc[1]);
            pk[1] = pack_bf16x2(acc[2], acc[3]);
            *reinterpret_cast<uintx2*>(Si + o * srow + 2 * (g.LPs + 16 * n + 4 * G)) = pk;
        };
        int n = wave / g.NOT;
        for (; n + wpo < g.NT; n += 2 * wpo) {
            const int n1 = n + wpo;
            const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
            if (g.KC > 1) {
                const bf16x8 a00 = tr_frag(Xi, xrow, 0, 16 * n, lane), a10 = tr_frag(Xi, xrow, 0, 16 * n1, lane);
                const bf16x8 a01 = tr_frag(Xi, xrow, 32, 16 * n, lane), a11 = tr_frag(Xi, xrow, 32, 16 * n1, lane);
                floatx4 c0 = mfma_bf16(a00, wsf[0], z4), c1 = mfma_bf16(a10, wsf[0], z4);
                c0 = mfma_bf16(a01, wsf[1], c0);
                c1 = mfma_bf16(a11, wsf[1], c1);
                s_store(c0, n);
                s_store(c1, n1);
            } else {
                const bf16x8 a00 = tr_frag(Xi, xrow, 0, 16 * n, lane), a10 = tr_frag(Xi, xrow, 0, 16 * n1, lane);
                s_store(mfma_bf16(a00, wsf[0], z4), n);
                s_store(mfma_bf16(a10, wsf[0], z4), n1);
            }
        }
        if (n < g.NT) {
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = mfma_bf16(tr_frag(Xi, xrow, 0, 16 * n, lane), wsf[0], acc);
            if (g.KC > 1) acc = mfma_bf16(tr_frag(Xi, xrow, 32, 16 * n, lane), wsf[1], acc);
            s_store(acc, n);
        }
        __syncthreads();
        const bool dump = g.dbg != nullptr && b == 0;
        if (dump)
            for (int i = tid; i < g.CP * g.T; i += NTI) {      // the x image as the spatial read it
                const int c = i / g.T, t = i - c * g.T;
                g.dbg[F2P * (g.T + 2 * g.T1) + i] =
                    (float)*reinterpret_cast<const __bf16*>(Xi + trimg_off(c, t >> 2, xrow) + 2 * (t & 3));
            }
        if (dump)
            for (int i = tid; i < F2P * g.T; i += NTI) {
                const int o = i / g.T, t = i - o * g.T;
                g.dbg[i] = (float)*reinterpret_cast<const __bf16*>(Si + o * srow + 2 * (g.LPs + t));
            }

        // ---- 2. FIR as banded-Toeplitz MFMA: V[i][n] = sum_j A_g[i][j] Win_n[j], A_g[i][j] = w1[g][j-i-1]
        //         (window j of tile n starts at s position 16n = sample 16n - P - 1), then BN, ELU, pool4
        int gcur = -1;
        bf16x8 af[3];
        for (int rr = 0; rr < rpw; ++rr) {
            const int o = wave * rpw + rr;
            const int gg = min(o, F2 - 1) / g.D;
            if (gg != gcur) {
                gcur = gg;
#pragma unroll
                for (int s = 0; s < 3; ++s)
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = 32 * s + 8 * G + j - l15 - 1;
                        af[s][j] = (__bf16)((s < g.KSF && k >= 0 && k < g.K1) ? W1t[gg * g.K1 + k] : 0.f);
                    }
            }
            // in log2 units: y = log2(e) * (al v + be); ELU summed over the pool window as
            // ln2 * sum max(y, 0) + sum exp2(min(y, 0)) - 4 (no per-element compare/select)
            const float al = Co[o] * 1.4426950408889634f, be = Co[F2P + o] * 1.4426950408889634f;
            const char* srw = Si + o * srow;
            float* arow = Aa + o * g.RA;
            for (int nb = 0; nb < g.NBLK; ++nb) {
                const int n = 16 * nb + l15;
                floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    if (s < g.KSF) {
                        const bf16x8 win = *reinterpret_cast<const bf16x8*>(srw + 2 * (16 * n + 8 * G + 32 * s));
                        acc = mfma_bf16(af[s], win, acc);
                    }
                }
                // lane: v[o][t = 16n + 4G + r]; pooled sample q = 4n + G
                float pp = 0.f, pn = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float y = fmaf(al, acc[r], be);
                    pp += fmaxf(y, 0.f);
                    pn += __builtin_amdgcn_exp2f(fminf(y, 0.f));
                }
                const int q = 4 * n + G;
                if (q < g.T1) arow[LAI + q] = fmaf(0.25f * 0.6931471805599453f, pp, 0.25f * pn - 1.f);
            }
            if (lane < LAI) arow[lane] = 0.f;                              // 'same' pad of block_2[0]
            else if (lane < 2 * LAI) arow[LAI + g.T1 + lane - LAI] = 0.f;
        }
        __syncthreads();
        if (dump)
            for (int i = tid; i < F2P * g.T1; i += NTI) {
                const int o = i / g.T1, q = i - o * g.T1;
                g.dbg[F2P * g.T + i] = Aa[o * g.RA + LAI + q];
            }

        // ---- 3. depthwise 1x16 (pad 7 | 8): 4 outputs per item from 20-float windows -> z image ----
        const int nq = (g.T1 + 3) >> 2;
        for (int it = tid; it < g.F2K * nq; it += NTI) {
            const int o = it / nq, m = it - o * nq;
            uintx2 pk = {0u, 0u};
            if (o < F2P) {
                const float* arow = Aa + o * g.RA + 4 * m;
                float w[20], tp[K2];
#pragma unroll
                for (int u = 0; u < 5; ++u) {
                    const floatx4 v = lds_ld4(arow + 4 * u);
                    w[4 * u] = v[0]; w[4 * u + 1] = v[1]; w[4 * u + 2] = v[2]; w[4 * u + 3] = v[3];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const floatx4 v = lds_ld4(W2t + o * K2 + 4 * u);
                    tp[4 * u] = v[0]; tp[4 * u + 1] = v[1]; tp[4 * u + 2] = v[2]; tp[4 * u + 3] = v[3];
                }
                float z[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < K2; ++k) a = fmaf(tp[k], w[i + k + 1], a);
                    z[i] = a;
                }
                pk[0] = pack_bf16x2(z[0], z[1]);
                pk[1] = pack_bf16x2(z[2], z[3]);
            }
            *reinterpret_cast<uintx2*>(Zi + trimg_off(o, m, zrow)) = pk;
        }
        __syncthreads();
        if (dump)
            for (int i = tid; i < F2P * g.T1; i += NTI) {
                const int o = i / g.T1, t = i - o * g.T1;
                g.dbg[F2P * (g.T + g.T1) + i] =
                    (float)*reinterpret_cast<const __bf16*>(Zi + trimg_off(o, t >> 2, zrow) + 2 * (t & 3));
            }

        // ---- 4. pointwise MFMA (A = W3, B = z by transposed reads), BN3, ELU, pool8, classifier ----
        float lp[NCLS] = {0.f, 0.f, 0.f, 0.f};
        for (int n = wave / g.NOT; n < g.NT1; n += wpo) {
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = mfma_bf16(w3f[0], tr_frag(Zi, zrow, 0, 16 * n, lane), acc);
            if (g.KCW > 1) acc = mfma_bf16(w3f[1], tr_frag(Zi, zrow, 32, 16 * n, lane), acc);
            // lane: r[j = ot*16 + 4G + r][t = 16n + l15]
            const int t2 = 2 * n + (l15 >> 3);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = ot * 16 + 4 * G + r;
                float e = elu_f(fmaf(Co[2 * F2P + j], acc[r], Co[3 * F2P + j]));
                e += dpp<0xB1>(e);            // 8-lane sums by DPP (xor 1, xor 2, half-row mirror)
                e += dpp<0x4E>(e);
                e += dpp<0x141>(e);
                if ((lane & 7) == 0 && j < F2 && t2 < g.T2) {
                    const float hv = 0.125f * e;
                    const int f = j * g.T2 + t2;
#pragma unroll
                    for (int c = 0; c < NCLS; ++c)
                        lp[c] = fmaf(g.offF ? Wf[c * g.NF + f] : prm[g.o_Wfc + c * g.NF + f], hv, lp[c]);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < NCLS; ++c) lp[c] = wave_sum(lp[c]);
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NCLS; ++c) Lg[wave * NCLS + c] = lp[c];
        }
        __syncthreads();

        // ---- 5. logits; next trial's x into the (now dead) image; re-arm the prefetch ----
        if (tid < NCLS) {
            float a = prm[g.o_bfc + tid];
            for (int w = 0; w < NWI; ++w) a += Lg[w * NCLS + tid];
            logits[(size_t)b * NCLS + tid] = a;
        }
        const int bn1 = b + gridDim.x;
        if constexpr (PFU > 0) {
            if (bn1 < g.B) {
                xi_store<PFU>(g, pf, Xi, tid);
                if (bn1 + (int)gridDim.x < g.B) xi_load<PFU>(g, x + (size_t)(bn1 + gridDim.x) * C * g.T, pf, tid);
            }
        } else {
            if (bn1 < g.B) xi_stage_elems(g, x + (size_t)bn1 * C * g.T, Xi, tid);
        }
        __syncthreads();
    }
}

}  // namespace eeg
