// eegnet_passes.hip -- the block-2-rate passes C and D of the restructured EEGNet train step and
// the fused eval-mode forward.  Included by eegnet_kernels.hip (one translation unit); the passes
// that stream x (A, B, E) are in eegnet_stream.hip.
//
// k_infer: workgroup = 1024 threads = 16 waves, one workgroup per CU, trials strided over the
// grid.  Wave w owns output row o = w of every per-trial [F2, T] plane (F2 <= 16), so its FIR taps
// are wave-uniform (SGPRs) and the FIR windows it reads are lane-contiguous float4s.

namespace eeg {

// block_2 forward of one trial in the row-per-wave layout: D2s (padded d2 rows) -> q (Qs) -> r.
// Returns r[m] for t = lane + 64 m (m < MAXT1Q) of row o.  Contains one workgroup barrier.

__device__ __forceinline__ void block2_rows(int F2, int T1, int RS2, const float* D2s, float* Qs,
                                            const float (&w2)[K2], const float (&w3)[F2MAX], bool row_on,
                                            int o, int lane, float (&r)[MAXT1Q]) {
    if (row_on) {
        const float* dr = D2s + o * RS2 + 1;
#pragma unroll
        for (int m = 0; m < MAXT1Q; ++m) {
            const int t = lane + 64 * m;
            if (t < T1) {
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < K2; ++k) a = fmaf(w2[k], dr[t + k], a);
                Qs[o * RS2 + t] = a;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MAXT1Q; ++m) {
        const int t = lane + 64 * m;
        float a = 0.f;
        if (row_on && t < T1) {
#pragma unroll
            for (int i = 0; i < F2MAX; ++i)
                if (i < F2) a = fmaf(w3[i], Qs[i * RS2 + t], a);
        }
        r[m] = a;
    }
}

// ================================================================================================
// Block-2-rate passes C and D: one trial per wave.  Lane t holds pooled sample t (+64 m) of all F2
// rows, so block_2's pointwise mix, BN3, ELU and the backward elementwise chain are lane-local
// register work with wave-uniform (scalar) weights, and the two depthwise 1x16 convolutions take
// their neighbours from DPP lane shifts (wave_shr / wave_shl).  No workgroup barrier inside the
// trial loop: the waves of a workgroup are independent trial streams until the final reduction.
// ================================================================================================
constexpr int NTHS = 512;       // workgroup bound of pass D and of the runtime-shape pass C
constexpr int LPQ = 8;          // left pad of pass D's LDS rows (16-byte aligned MFMA / window reads)
constexpr int LPD = 7;          // left pad of pass D's d2 rows: d2p[t + k - 7] sits at [t + k]
constexpr int MAXNFQ = 8;       // flattened head features per lane: F2*(T/32) <= 512

// 8-lane sums of consecutive lanes: after the three DPP steps lanes 8i+4..8i+7 hold the sum of
// lanes 8i..8i+7 (quad sums, then row_shr:4 adds the neighbouring quad; bound_ctrl zero-fills)
__device__ __forceinline__ float sum8_hi(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xF, 0xF, true));
    return v;
}

// a wave-uniform value (e.g. from a uniform-address LDS read) moved to an SGPR
__device__ __forceinline__ float sgpr_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// x[t] <- x[t-1] / x[t+1] over the row t = lane + 64 m, zero shifted in at the ends
template <int MQ>
__device__ __forceinline__ void shr1(float (&x)[MQ], int lane) {
#pragma unroll
    for (int m = MQ - 1; m >= 0; --m) {
        const float carry = m > 0 ? readlane_f(x[m > 0 ? m - 1 : 0], 63) : 0.f;
        const float v = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x[m]), 0x138, 0xF, 0xF, true));
        x[m] = (m > 0 && lane == 0) ? carry : v;
    }
}
template <int MQ>
__device__ __forceinline__ void shl1(float (&x)[MQ], int lane) {
#pragma unroll
    for (int m = 0; m < MQ; ++m) {
        const float carry = m < MQ - 1 ? readlane_f(x[m < MQ - 1 ? m + 1 : m], 0) : 0.f;
        const float v = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x[m]), 0x130, 0xF, 0xF, true));
        x[m] = (m < MQ - 1 && lane == 63) ? carry : v;
    }
}

// transposed depthwise 1x16: y[t] = sum_k w[k] x[t + 7 - k] (the input gradient of the 'same' conv, model.py:54-61)
template <int MQ>
__device__ __forceinline__ void conv16_same_t(const float (&x)[MQ], const float* __restrict__ w, float (&y)[MQ],
                                              int lane) {
    float s[MQ];
#pragma unroll
    for (int m = 0; m < MQ; ++m) { y[m] = w[7] * x[m]; s[m] = x[m]; }
#pragma unroll
    for (int k = 6; k >= 0; --k) {                 // s = x[t + 7 - k]
        shl1<MQ>(s, lane);
#pragma unroll
        for (int m = 0; m < MQ; ++m) y[m] = fmaf(w[k], s[m], y[m]);
    }
#pragma unroll
    for (int m = 0; m < MQ; ++m) s[m] = x[m];
#pragma unroll
    for (int k = 8; k < K2; ++k) {                 // s = x[t - (k - 7)]
        shr1<MQ>(s, lane);
#pragma unroll
        for (int m = 0; m < MQ; ++m) y[m] = fmaf(w[k], s[m], y[m]);
    }
}

// the same as two independent chains (taps 0-7 over left shifts, 8-15 over right shifts) added at
// the end: half the dependent-latency chain per row
template <int MQ>
__device__ __forceinline__ void conv16_same_t2(const float (&x)[MQ], const float* __restrict__ w, float (&y)[MQ],
                                               int lane) {
    float s[MQ], u[MQ], y1[MQ];
#pragma unroll
    for (int m = 0; m < MQ; ++m) { y[m] = w[7] * x[m]; s[m] = x[m]; u[m] = x[m]; y1[m] = 0.f; }
#pragma unroll
    for (int k = 6; k >= 0; --k) {
        shl1<MQ>(s, lane);                         // s = x[t + 7 - k]
        shr1<MQ>(u, lane);                         // u = x[t - (14 - k - 7)] for tap 14 - k
#pragma unroll
        for (int m = 0; m < MQ; ++m) { y[m] = fmaf(w[k], s[m], y[m]); y1[m] = fmaf(w[14 - k], u[m], y1[m]); }
    }
    shr1<MQ>(u, lane);                             // tap 15: x[t - 8]
#pragma unroll
    for (int m = 0; m < MQ; ++m) y[m] += fmaf(w[15], u[m], y1[m]);
}

// d2 rows of trial b into registers (lane t, chunk m); zero beyond T1.  Wave-uniform row base:
// saddr + 32-bit lane offset loads.
template <int MQ>
__device__ __forceinline__ void load_rows(const float* __restrict__ src, int b, int F2, int T1, int lane,
                                          float (&d)[F2MAX][MQ]) {
    const float* base = src + (size_t)b * F2 * T1;
#pragma unroll
    for (int o = 0; o < F2MAX; ++o)
#pragma unroll
        for (int m = 0; m < MQ; ++m) {
            const int t = lane + 64 * m;
            d[o][m] = (o < F2 && t < T1) ? base[o * T1 + t] : 0.f;
        }
}

// xh[j] = BN3-normalised r[j] (batch statistics of finalize 2), r from pass B's r plane
template <int MQ>
__device__ __forceinline__ void bn3_rows(const float* coef, int F2, const float (&r)[F2MAX][MQ],
                                         float (&xh)[F2MAX][MQ]) {
#pragma unroll
    for (int j = 0; j < F2MAX; ++j) {
        const float mu3 = j < F2 ? coef[CF_MU3 * CSTR + j] : 0.f, inv3 = j < F2 ? coef[CF_INV3 * CSTR + j] : 0.f;
#pragma unroll
        for (int m = 0; m < MQ; ++m) xh[j][m] = (r[j][m] - mu3) * inv3;
    }
}

// ================================================================================================
// Pass C: head (model.py:71-84).  logits, and (PC_BWD) CE, classifier grads, BN3-backward sums.
// part row: [dWfc 4*NF][dbfc 4][Sdz3 F2][Sdz3x F2][loss]
// Per-wave LDS: Hs [NF] -- the flattened head features (model.py:75 Flatten order), then their
// gradients.
// ================================================================================================
template <int K1, int CC, int TT, int FF, bool FOLD>
__device__ __forceinline__ void pass_c_body(const Geo& g, const float* __restrict__ prm,
                                            const float* coef,    // the finalize writes it: no __restrict__
                                            const float* __restrict__ r3g,
                                            const uint8_t* __restrict__ mask3,
                                            const float* __restrict__ dlin,
                                            const int64_t* __restrict__ labels,
                                            float* __restrict__ logits, float* __restrict__ dlout,
                                            float* __restrict__ part, int mode, FinArgs fa, const FoldCall& fc,
                                            float* sm) {
    EEG_DIMS(g);
    TRACE(g, 2, TR_ENTRY);
    unsigned dk1;
    const int64_t* perm = nullptr;                     // fold launches: labels through the permutation
    long long row0 = 0;
    if (FOLD) {
        const eegnet_fold f = fold_rec(fc);
        char* ws = (char*)f.ws;
        prm = f.params;
        coef = (const float*)(ws + fc.off.coef);
        r3g = (const float*)(ws + fc.off.r3);
        mask3 = nullptr; dlin = nullptr; logits = nullptr;
        labels = f.labels;
        perm = f.perm; row0 = fc.row0;
        dlout = (float*)(ws + fc.off.dl);
        part = (float*)(ws + fc.off.partC);
        fa = fold_fin(fc, f, TK_C, 0, 1, false, false, g.nparam);
        dk1 = fold_drop_key(fc, f, 1);
    } else {
        dk1 = drop_key(g, 1);
    }
    constexpr int MQ = TT ? (TT / 4 + 63) / 64 : MAXT1Q;
    constexpr int NFQ = (TT && FF) ? (FF * (TT / 32) + 63) / 64 : MAXNFQ;
    const int NFP = rup4(NF);
    const int nw = blockDim.x >> 6;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float* Hs = sm + wave * NFP;
    // the rows' BN3 constants [mu3 inv3 g3 b3] x F2MAX after the waves' Hs rows, read with wave-uniform
    // 16-byte LDS reads (row-chained scalar loads serialised one L2 round trip per row: the ELU / pool
    // phase of a trial took ~5 K cycles for ~1 K of work)
    float* const Ct = sm + nw * NFP;
    if (tid < F2MAX) {
        const int j = tid < F2 ? tid : 0;
        const bool on = tid < F2;
        Ct[4 * tid + 0] = on ? coef[CF_MU3 * CSTR + j] : 0.f;
        Ct[4 * tid + 1] = on ? coef[CF_INV3 * CSTR + j] : 0.f;
        Ct[4 * tid + 2] = on ? prm[g.o_g3 + j] : 0.f;
        Ct[4 * tid + 3] = on ? prm[g.o_b3 + j] : 0.f;
    }

    float wf[NCLS][NFQ], wacc[NCLS][NFQ];
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            wf[n][u] = i < NF ? prm[g.o_Wfc + n * NF + i] : 0.f;
            wacc[n][u] = 0.f;
        }
    float sdz[2 * F2MAX];                 // [Sdz3 F2MAX][Sdz3x F2MAX], per-lane partials
#pragma unroll
    for (int j = 0; j < 2 * F2MAX; ++j) sdz[j] = 0.f;
    float bacc[NCLS] = {0.f, 0.f, 0.f, 0.f}, lossacc = 0.f;
    const float invB = 1.0f / (float)g.Bn;
    const int bfirst = blockIdx.x * nw + wave, bstop = g.B, bstep = gridDim.x * nw;

    __syncthreads();                          // the constant table
    TRACE(g, 2, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = bfirst; b < bstop; b += bstep) {
        float xh[F2MAX][MQ];
        {
            // block 2 up to the pointwise mix is pass B's (its r plane): BN3 normalisation only
            float r[F2MAX][MQ];
            load_rows<MQ>(r3g, b, F2, T1, lane, r);
            TRACE_PH(g, 2, 0, tph_);
#pragma unroll
            for (int j = 0; j < F2MAX; ++j) {
                const floatx4 c = lds_ld4(Ct + 4 * j);
                const float mu = sgpr_f(c[0]), inv = sgpr_f(c[1]);
#pragma unroll
                for (int m = 0; m < MQ; ++m) xh[j][m] = (r[j][m] - mu) * inv;
            }
            TRACE_PH(g, 2, 1, tph_);
        }
        // ELU -> AvgPool(1,8) -> Hs (flattened index j*T2 + t/8)
#pragma unroll
        for (int j = 0; j < F2MAX; ++j) {
            if (j >= F2) continue;
            const floatx4 c = lds_ld4(Ct + 4 * j);
            const float g3 = sgpr_f(c[2]), b3 = sgpr_f(c[3]);
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int t = lane + 64 * m;
                float e = t < 8 * T2 ? elu_f(fmaf(g3, xh[j][m], b3)) : 0.f;
                e = sum8_hi(e);
                if ((lane & 7) == 7 && t < 8 * T2) Hs[j * T2 + (t >> 3)] = e * 0.125f;
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 2, 2, tph_);
        float hv[NFQ], kp[NFQ];
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            kp[u] = i < NF ? keep_mul(g, mask3, dk1, (unsigned)(b * NF + i)) : 0.f;
            hv[u] = i < NF ? Hs[i] * kp[u] : 0.f;          // dropout (model.py:74)
        }
        // logits (model.py:78-82)
        float lg[NCLS];
#pragma unroll
        for (int n = 0; n < NCLS; ++n) {
            float a = 0.f;
#pragma unroll
            for (int u = 0; u < NFQ; ++u) a = fmaf(wf[n][u], hv[u], a);
            lg[n] = a;
        }
        wave_reduce<NCLS>(lg);                              // lane 16n: class n
        float L[NCLS];
#pragma unroll
        for (int n = 0; n < NCLS; ++n) L[n] = readlane_f(lg[0], 16 * n) + prm[g.o_bfc + n];
        if ((mode & PC_LOGITS) && lane < NCLS)
            logits[(size_t)b * NCLS + lane] = lane == 0 ? L[0] : lane == 1 ? L[1] : lane == 2 ? L[2] : L[3];
        if (mode & PC_BWD) {
            float dl[NCLS];
            if (mode & PC_CE) {                              // nn.CrossEntropyLoss, mean (train.py:103)
                const float mx = fmaxf(fmaxf(L[0], L[1]), fmaxf(L[2], L[3]));
                float se = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) se += expf(L[n] - mx);
                const float lse = mx + logf(se);
                const int y = (int)labels[fold_row(perm, row0, b)];
                const float Ly = y == 0 ? L[0] : y == 1 ? L[1] : y == 2 ? L[2] : L[3];
                lossacc += lse - Ly;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dl[n] = (expf(L[n] - lse) - (n == y ? 1.f : 0.f)) * invB;
                if (lane < NCLS)
                    dlout[(size_t)b * NCLS + lane] = lane == 0 ? dl[0] : lane == 1 ? dl[1] : lane == 2 ? dl[2] : dl[3];
            } else {
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dl[n] = dlin[(size_t)b * NCLS + n];
            }
#pragma unroll
            for (int n = 0; n < NCLS; ++n) {
                bacc[n] += dl[n];
#pragma unroll
                for (int u = 0; u < NFQ; ++u) wacc[n][u] = fmaf(dl[n], hv[u], wacc[n][u]);
            }
            // dh -> dropout -> dp3 (flattened), overwriting h in Hs (each lane its own slots)
#pragma unroll
            for (int u = 0; u < NFQ; ++u) {
                const int i = lane + 64 * u;
                float d = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) d = fmaf(dl[n], wf[n][u], d);
                if (i < NF) Hs[i] = d * kp[u];
            }
            wave_lds_fence();
            TRACE_PH(g, 2, 3, tph_);
            // BN3-backward sums: dz3 = dp3/8 * ELU'(z3)
#pragma unroll
            for (int j = 0; j < F2MAX; ++j) {
                if (j >= F2) continue;
                const floatx4 c = lds_ld4(Ct + 4 * j);
                const float g3 = sgpr_f(c[2]), b3 = sgpr_f(c[3]);
#pragma unroll
                for (int m = 0; m < MQ; ++m) {
                    const int t = lane + 64 * m;
                    if (t < 8 * T2) {
                        const float dz = Hs[j * T2 + (t >> 3)] * 0.125f * elu_d(fmaf(g3, xh[j][m], b3));
                        sdz[j] += dz;
                        sdz[F2MAX + j] = fmaf(dz, xh[j][m], sdz[F2MAX + j]);
                    }
                }
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 2, 4, tph_);
    }
    TRACE_LOOP(g, 2);
    if (!(mode & PC_BWD)) return;
    // ---- workgroup reduction: every wave writes a full partial row, then the waves are summed ----
    __syncthreads();
    TRACE_PS(g, 8);
    float* red = sm;                         // [nw][nC]
    float* rw = red + wave * g.nC;
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            if (i < NF) rw[n * NF + i] = wacc[n][u];
        }
    wave_reduce<2 * F2MAX>(sdz);
    TRACE_PS(g, 9);
    if ((lane & 15) == 0) {
        const int r0 = (lane >> 4) * (F2MAX / 2);
#pragma unroll
        for (int j = 0; j < F2MAX / 2; ++j) {
            const int idx = j + r0;
            if (idx < F2MAX) { if (idx < F2) rw[NCLS * NF + NCLS + idx] = sdz[j]; }
            else if (idx - F2MAX < F2) rw[NCLS * NF + NCLS + F2 + idx - F2MAX] = sdz[j];
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int n = 0; n < NCLS; ++n) rw[NCLS * NF + n] = bacc[n];
        rw[NCLS * NF + NCLS + 2 * F2] = lossacc;
    }
    __syncthreads();
    TRACE_PS(g, 10);
    float* row = part + (size_t)blockIdx.x * g.nC;
    for (int c = tid; c < g.nC; c += blockDim.x) pub(row + c, wave_rows_sum<NTH / 64>(red, nw, g.nC, c));
    TRACE_PS(g, 11);
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nC, fa, dsm)) { fin3(g, prm, dsm + 2, fa); TRACE(g, 2, TR_FIN); }
}

template <int K1, int CC, int TT, int FF, bool FOLD = false>
__global__ __launch_bounds__(TT ? NTH : NTHS) void k_pass_c(Geo g, const float* __restrict__ prm,
                                                const float* coef,    // the finalize writes it: no __restrict__
                                                const float* __restrict__ r3g,
                                                const uint8_t* __restrict__ mask3,
                                                const float* __restrict__ dlin,
                                                const int64_t* __restrict__ labels,
                                                float* __restrict__ logits, float* __restrict__ dlout,
                                                float* __restrict__ part, int mode, FinArgs fa, FoldCall fc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    pass_c_body<K1, CC, TT, FF, FOLD>(g, prm, coef, r3g, mask3, dlin, labels, logits, dlout, part, mode, fa, fc, sm);
}

#if EEGNET_D1
// ================================================================================================
// Pass D: block_2 backward (dW3, dw2), dp2 = d(pooled ELU output), BN2-backward sums.
// (rounds 1-5; built only by -DEEGNET_D1=1 A/B builds since k_pass_dr replaced it)
// part row: [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2]
// Per-wave LDS rows (stride RSW): P0 d2 (pad LPD) | P1 q, then dq (pad LPQ) | P2 dr (pad LPQ) | Hs [NF].
// ================================================================================================
// MASK = false: dropout from the device generator only (mask2 / mask3 are null).  The host-mask
// path costs registers in this kernel (256 VGPRs + spills against 156), so it is its own instantiation.
template <int K1, int CC, int TT, int FF, bool FOLD = false, bool MASK = true>
__global__ __launch_bounds__(NTHS) void k_pass_d(Geo g, const float* __restrict__ prm,
                                                 const float* coef,    // the finalize writes it: no __restrict__
                                                 const float* __restrict__ d2g,
                                                 const float* __restrict__ E1g,
                                                 const float* __restrict__ E2g,
                                                 const float* __restrict__ q3g,
                                                 const float* __restrict__ r3g,
                                                 const uint8_t* __restrict__ mask2,
                                                 const uint8_t* __restrict__ mask3,
                                                 const float* __restrict__ dl,
                                                 float* __restrict__ dp2g, float* __restrict__ part,
                                                 FinArgs fa, FoldCall fc) {
    EEG_DIMS(g);
    TRACE(g, 3, TR_ENTRY);
    unsigned dk0, dk1;
    if (FOLD) {
        const eegnet_fold f = fold_rec(fc);
        char* ws = (char*)f.ws;
        prm = f.params;
        coef = (const float*)(ws + fc.off.coef);
        d2g = (const float*)(ws + fc.off.d2);
        E1g = (const float*)(ws + fc.off.E1); E2g = (const float*)(ws + fc.off.E2);
        q3g = (const float*)(ws + fc.off.q3); r3g = (const float*)(ws + fc.off.r3);
        mask2 = nullptr; mask3 = nullptr;
        dl = (const float*)(ws + fc.off.dl);
        dp2g = (float*)(ws + fc.off.dp2);
        part = (float*)(ws + fc.off.partD);
        fa = fold_fin(fc, f, TK_D, 0, 0, false, false, g.nparam);
        dk0 = fold_drop_key(fc, f, 0);
        dk1 = fold_drop_key(fc, f, 1);
    } else {
        dk0 = drop_key(g, 0);
        dk1 = drop_key(g, 1);
    }
    if constexpr (!MASK) { mask2 = nullptr; mask3 = nullptr; }
    constexpr int MQ = TT ? (TT / 4 + 63) / 64 : MAXT1Q;
    constexpr int NFQ = (TT && FF) ? (FF * (TT / 32) + 63) / 64 : MAXNFQ;
    const int RSW = TT ? row_stride_b2(TT / 4) : g.RSW;
    const int NFP = rup4(NF);
    const int nw = blockDim.x >> 6;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int li = lane & 15, lk = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float* P0 = sm + wave * (3 * F2 * RSW + NFP);
    float* P1 = P0 + F2 * RSW;
    float* P2 = P1 + F2 * RSW;
    float* Hs = P2 + F2 * RSW;

    for (int i = lane; i < 3 * F2 * RSW; i += 64) P0[i] = 0.f;   // pads stay zero
    float wf[NCLS][NFQ];
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            wf[n][u] = i < NF ? prm[g.o_Wfc + n * NF + i] : 0.f;
        }
    floatx4 acc3 = {0.f, 0.f, 0.f, 0.f};        // dW3 tile: D[j = 4 lk + r][i = li]
    const int o2 = lane >> 2, kq = lane & 3;   // dw2 item of this lane: row o2, taps 4 kq .. 4 kq + 3
    float acc2[4] = {0.f, 0.f, 0.f, 0.f};
    float sz[2 * F2MAX];                       // [Sdz2 F2MAX][Sdz2x F2MAX], per-lane partials
#pragma unroll
    for (int j = 0; j < 2 * F2MAX; ++j) sz[j] = 0.f;
    const int nkg = (T1 + 15) >> 4, ntq = (T1 + 3) >> 2;
    wave_lds_fence();

    TRACE(g, 3, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    // a trial's pass-B rows (d2, q, r) and dlogits go out together -- one global round trip, not three
    // -- and the next trial's are loaded into the same registers as soon as this trial has consumed
    // them (after the BN3 backward), so they land during the dW3 / dq / dw2 / dd2 phases
    float dlv[NCLS];
    float d[F2MAX][MQ], q[F2MAX][MQ], r[F2MAX][MQ];
    auto load_trial = [&](int bb) {
#pragma unroll
        for (int n = 0; n < NCLS; ++n) dlv[n] = dl[(size_t)bb * NCLS + n];
        load_rows<MQ>(d2g, bb, F2, T1, lane, d);
        load_rows<MQ>(q3g, bb, F2, T1, lane, q);
        load_rows<MQ>(r3g, bb, F2, T1, lane, r);
    };
    const int bstep = gridDim.x * nw;
    if (blockIdx.x * nw + wave < g.B) load_trial(blockIdx.x * nw + wave);
    for (int b = blockIdx.x * nw + wave; b < g.B; b += bstep) {
        // d2 rows -> P0 (read back by the dw2 correlation)
#pragma unroll
        for (int o = 0; o < F2MAX; ++o)
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int t = lane + 64 * m;
                if (o < F2 && t < T1) P0[o * RSW + LPD + t] = d[o][m];
            }
        // dh -> dropout -> dp3 (flattened) into Hs
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            float dd = 0.f;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) dd = fmaf(dlv[n], wf[n][u], dd);
            if (i < NF) Hs[i] = dd * keep_mul(g, mask3, dk1, (unsigned)(b * NF + i));
        }
        TRACE_PH(g, 3, 0, tph_);
        // block-2 depthwise output (pass B's q plane) -> P1
#pragma unroll
        for (int o = 0; o < F2MAX; ++o)
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int t = lane + 64 * m;
                if (o < F2 && t < T1) P1[o * RSW + LPQ + t] = q[o][m];
            }
        wave_lds_fence();
        TRACE_PH(g, 3, 1, tph_);
        // BN3 backward with the batch constants of finalize 3: dr = A3 dz3 + B3 + C3 xh3,
        // dz3 = dp3/8 * ELU'(z3); zero beyond T1 (the dq / dd2 shifts read it)
        float dr[F2MAX][MQ];
        {
            float xh[F2MAX][MQ];
            bn3_rows<MQ>(coef, F2, r, xh);          // r: pass B's pointwise output
#pragma unroll
            for (int j = 0; j < F2MAX; ++j) {
                if (j < F2) {
                    const int oz = opaque0();
                    const float g3 = prm[g.o_g3 + j + oz], b3 = prm[g.o_b3 + j + oz];
                    const float A3 = coef[CF_A3 * CSTR + j + oz], B3 = coef[CF_B3 * CSTR + j + oz];
                    const float C3 = coef[CF_C3 * CSTR + j + oz];
#pragma unroll
                    for (int m = 0; m < MQ; ++m) {
                        const int t = lane + 64 * m;
                        const float dz = t < 8 * T2 ? Hs[j * T2 + (t >> 3)] * 0.125f * elu_d(fmaf(g3, xh[j][m], b3)) : 0.f;
                        dr[j][m] = t < T1 ? fmaf(A3, dz, fmaf(C3, xh[j][m], B3)) : 0.f;
                        if (t < T1) P2[j * RSW + LPQ + t] = dr[j][m];
                    }
                } else {
#pragma unroll
                    for (int m = 0; m < MQ; ++m) dr[j][m] = 0.f;
                }
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 3, 2, tph_);
        // E1 / E2 of pass B for the BN2-backward sums at the end (issued here, consumed last), then
        // the next trial's rows (younger: the E1 / E2 wait does not wait for them)
        float e1v[F2MAX][MQ], e2v[F2MAX][MQ];
        load_rows<MQ>(E1g, b, F2, T1, lane, e1v);
        load_rows<MQ>(E2g, b, F2, T1, lane, e2v);
        if (b + bstep < g.B) load_trial(b + bstep);
        // dW3[j][i] += sum_t dr[j][t] q[i][t] on the matrix cores (float4 k-permuted operands)
        {
            // (ds_read_b64 operands, t = 16 kg + 2 lk + {0, 1}, + 8: conflict-free, as pass E's dws GEMM)
            const bool on = li < F2;
            const float* ar = P2 + (on ? li : 0) * RSW + LPQ + 2 * lk;
            const float* br = P1 + (on ? li : 0) * RSW + LPQ + 2 * lk;
            for (int kg = 0; kg < nkg; ++kg) {
                floatx2 a0 = lds_ld2(ar + 16 * kg), a1 = lds_ld2(ar + 16 * kg + 8);
                floatx2 b0 = lds_ld2(br + 16 * kg), b1 = lds_ld2(br + 16 * kg + 8);
                if (!on) { a0 = (floatx2){0.f, 0.f}; a1 = a0; b0 = a0; b1 = a0; }
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0], b0[0], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1], b0[1], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0], b1[0], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1], b1[1], acc3, 0, 0, 0);
            }
        }
        wave_lds_fence();                          // q rows consumed before dq overwrites them
        TRACE_PH(g, 3, 3, tph_);
        // dq[i][t] = sum_j W3[j][i] dr[j][t] (registers, and P1 for the dw2 correlation)
        float dq[F2MAX][MQ];
#pragma unroll
        for (int i = 0; i < F2MAX; ++i) {
            if (i < F2) {
                const int oz = i >= 2 ? opaque0_after(dq[i >= 2 ? i - 2 : 0][0]) : opaque0();
                const float* w3c = prm + (g.o_W3 + i + oz);      // column i of W3 (stride F2)
#pragma unroll
                for (int m = 0; m < MQ; ++m) {
                    const int t = lane + 64 * m;
                    float a = 0.f;
#pragma unroll
                    for (int j = 0; j < F2MAX; ++j)
                        if (j < F2) a = fmaf(w3c[j * F2], dr[j][m], a);
                    dq[i][m] = a;
                    if (t < T1) P1[i * RSW + LPQ + t] = a;
                }
            } else {
#pragma unroll
                for (int m = 0; m < MQ; ++m) dq[i][m] = 0.f;
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 3, 4, tph_);
        // dw2[o][k] += sum_t dq[o][t] d2p[o][t+k-7]: lane -> (row o2, taps 4 kq + kk), loop over t
        if (o2 < F2) {
            const float* dqr = P1 + o2 * RSW + LPQ;
            const float* d2r = P0 + o2 * RSW + 4 * kq;      // d2p[t + k - 7] = P0[row + t + k]
            for (int tq = 0; tq < ntq; ++tq) {
                const floatx4 a4 = lds_ld4(dqr + 4 * tq);
                const floatx4 w0 = lds_ld4(d2r + 4 * tq), w1 = lds_ld4(d2r + 4 * tq + 4);
                const float w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc2[kk] = fmaf(a4[i], w[i + kk], acc2[kk]);
            }
        }
        TRACE_PH(g, 3, 5, tph_);
        // dd2 = conv16_same_t(dq) -> dropout -> dp2; BN2-backward sums (E1/E2 of pass B)
        const size_t rb = (size_t)b * F2 * T1;
#pragma unroll
        for (int o = 0; o < F2MAX; ++o) {
            if (o >= F2) continue;
            float a[MQ];
            const int oz = o >= 2 ? opaque0_after(sz[o >= 2 ? o - 2 : 0]) : opaque0();
            conv16_same_t<MQ>(dq[o], prm + (g.o_w2 + o * K2 + oz), a, lane);
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int t = lane + 64 * m;
                if (t < T1) {
                    const int gi = o * T1 + t;
                    const float dp = a[m] * keep_mul(g, mask2, dk0, (unsigned)(rb + gi));
                    st_pol<EEGNET_NT_MID>(dp, dp2g + rb + gi);
                    sz[o] = fmaf(dp * 0.25f, e1v[o][m], sz[o]);
                    sz[F2MAX + o] = fmaf(dp * 0.25f, e2v[o][m], sz[F2MAX + o]);
                }
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 3, 6, tph_);
    }
    TRACE_LOOP(g, 3);
    // ---- workgroup reduction ----
    __syncthreads();
    float* red = sm;                         // [nw][nD]
    float* rw = red + wave * g.nD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int j = 4 * lk + r;
        if (j < F2 && li < F2) rw[j * F2 + li] = acc3[r];
    }
    if (o2 < F2) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) rw[F2 * F2 + o2 * K2 + 4 * kq + kk] = acc2[kk];
    }
    wave_reduce<2 * F2MAX>(sz);
    if ((lane & 15) == 0) {
        const int r0 = (lane >> 4) * (F2MAX / 2);
#pragma unroll
        for (int j = 0; j < F2MAX / 2; ++j) {
            const int idx = j + r0;
            if (idx < F2MAX) { if (idx < F2) rw[F2 * F2 + 16 * F2 + idx] = sz[j]; }
            else if (idx - F2MAX < F2) rw[F2 * F2 + 17 * F2 + idx - F2MAX] = sz[j];
        }
    }
    __syncthreads();
    float* row = part + (size_t)blockIdx.x * g.nD;
    for (int c = tid; c < g.nD; c += blockDim.x) pub(row + c, wave_rows_sum<NTHS / 64>(red, nw, g.nD, c));
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nD, fa, dsm)) { fin4(g, prm, dsm + 2, fa); TRACE(g, 3, TR_FIN); }
}
#endif  // EEGNET_D1

// ================================================================================================
// Pass D in the streaming passes' row layout (k_pass_dr, the default; k_pass_d above is the
// -DEEGNET_D1=1 build).  k_pass_d gives each wave a whole trial, so one trial is a ~12 us serial chain
// of one wave at two waves per SIMD (225 VGPRs): scalar weight loads chained row after row, the
// pointwise mix over 16 rows in one lane, and 16 conv rows back to back.  Here the workgroup works on
// one trial at a time like passes B and E: wave w owns rows o = 2w, 2w + 1 of the trial's [F2, T1]
// planes, lane t owns pooled sample t (+ 64 m), two 512-thread workgroups per CU.
//   step 1 (row-local): BN3 backward of the own rows -> dr rows and the q rows into LDS (alternate
//     buffers per trial, so one barrier per trial)
//   barrier
//   step 2: dW3 += dr q^T (MFMA, the T1 k-steps dealt over the waves), dq = W3^T dr for the own rows
//     (all dr rows from LDS), dw2 (own rows, lane-shifted d2), dd2 = the transposed 1x16 conv (lane
//     shifts), dropout -> dp2, BN2-backward sums
// The trial's five plane rows per lane and its dlogits come a trial ahead (registers / SGPRs); the
// block-2 weights sit in LDS and reach the SGPRs by readfirstlane.
// part row: [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2] (k_pass_d's, finalize 4 unchanged)
// LDS: dr rows x 2 | q rows x 2 (F2MAX rows of RSD floats) | W3^T [F2MAX][F2MAX] | w2 [F2MAX][16]
// ================================================================================================
// row stride 64 MQ + 2: a 32-lane group of the MFMA operand reads (16 rows x 2 consecutive k) covers
// banks 2 li + lk -- 32 distinct banks (ds_read_b32 banks mod 32 per 32-lane group)
__host__ __device__ constexpr int dr_stride(int MQ) { return 64 * MQ + 2; }
__host__ __device__ constexpr int dr_lds_floats(int MQ) { return 4 * F2MAX * dr_stride(MQ) + F2MAX * (F2MAX + K2); }
// after the loop: dW3 tiles [NWB][256], the owned row [18 F2MAX], and (T1 = 64) the Hankel tiles
__host__ __device__ constexpr int dr_tail_floats(bool hankel) { return NWB * 256 + 18 * F2MAX + (hankel ? NWB * RPW * 2 * 256 : 0); }

template <int K1, int CC, int TT, int FF, bool FOLD = false, bool MASK = true>
__global__ __launch_bounds__(NTB, TT ? WPEB : 2) void k_pass_dr(Geo g, const float* __restrict__ prm,
                                                  const float* coef,    // the finalize writes it: no __restrict__
                                                  const float* __restrict__ d2g,
                                                  const float* __restrict__ E1g,
                                                  const float* __restrict__ E2g,
                                                  const float* __restrict__ q3g,
                                                  const float* __restrict__ r3g,
                                                  const uint8_t* __restrict__ mask2,
                                                  const uint8_t* __restrict__ mask3,
                                                  const float* __restrict__ dl,
                                                  float* __restrict__ dp2g, float* __restrict__ part,
                                                  FinArgs fa, FoldCall fc) {
    EEG_DIMS_NT(g, NTB);
    TRACE(g, 3, TR_ENTRY);
    unsigned dk0, dk1;
    if (FOLD) {
        const eegnet_fold f = fold_rec(fc);
        char* ws = (char*)f.ws;
        prm = f.params;
        coef = (const float*)(ws + fc.off.coef);
        d2g = (const float*)(ws + fc.off.d2);
        E1g = (const float*)(ws + fc.off.E1); E2g = (const float*)(ws + fc.off.E2);
        q3g = (const float*)(ws + fc.off.q3); r3g = (const float*)(ws + fc.off.r3);
        mask2 = nullptr; mask3 = nullptr;
        dl = (const float*)(ws + fc.off.dl);
        dp2g = (float*)(ws + fc.off.dp2);
        part = (float*)(ws + fc.off.partD);
        fa = fold_fin(fc, f, TK_D, 0, 0, false, false, g.nparam);
        dk0 = fold_drop_key(fc, f, 0);
        dk1 = fold_drop_key(fc, f, 1);
    } else {
        dk0 = drop_key(g, 0);
        dk1 = drop_key(g, 1);
    }
    if constexpr (!MASK) { mask2 = nullptr; mask3 = nullptr; }
    constexpr int MQ = TT ? (TT / 4 + 63) / 64 : MAXT1Q;
    constexpr int RSD = dr_stride(MQ);
    constexpr int NKS = TT ? (TT / 4 + 3) / 4 : 16 * MAXT1Q;    // MFMA k-steps bound (rows are zero past T1)
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const DR0 = sm;                              // [2][F2MAX][RSD]
    float* const Q0 = DR0 + 2 * F2MAX * RSD;            // [2][F2MAX][RSD]
    float* const W3t = Q0 + 2 * F2MAX * RSD;            // W3t[i][j] = W3[j][i]
    float* const W2t = W3t + F2MAX * F2MAX;             // w2[o][k]
    const int tid = threadIdx.x, lane = tid & 63;
    const int li = lane & 15, lk = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b0, b1;
    trial_range(g, b0, b1);
    const int nks = TT ? NKS : (T1 + 3) >> 2;
    // the compile-time shapes fill every row and lane (F2 = 16 rows, T1 = 64 samples): no guards, so no
    // branches around loads -- a branch makes the waitcnt pass wait for every load in flight (vmcnt(0))
    // at the loop top, which turned the prefetch into a stall
    constexpr bool FULL = TT && FF == F2MAX && TT / 4 == 64 * MQ;

    // plane rows of a trial in two register slots (rows RPW w + r, lanes t = lane + 64 m; zero past
    // T1 / F2).  The loop runs the trials in pairs, slot 0 then slot 1, and a slot is reloaded with
    // the trial two ahead as soon as its rows have been read (r, q and dlogits after step 1; d2, E1, E2
    // after step 2): no register copies, so a load is never waited for before its own trial (copies
    // of freshly loaded registers had made the waitcnt pass wait for the newest loads every trial).
    // An odd trial range ends with a ghost trial: the last trial again, its sums gated off (its dp2
    // stores repeat the same values).
    float sr[2][RPW][MQ], sq[2][RPW][MQ], sd[2][RPW][MQ], se1[2][RPW][MQ], se2[2][RPW][MQ];
    floatx4 sdl[2];
    // a row's wave-uniform base (scalar) and the lane's 32-bit offset: saddr-form loads, no 64-bit
    // address VGPRs
    auto row_base = [&](int bb, int r) {
        const int o = RPW * wave + r;
        return (size_t)bb * F2 * T1 + (size_t)((FULL || o < F2) ? o * T1 : 0);
    };
    auto lane_off = [&](int r, int m, bool& ok) {
        const int o = RPW * wave + r, t = lane + 64 * m;
        ok = FULL || (o < F2 && t < T1);
        return ok ? t : 0;
    };
    auto load_rq = [&](int bb, float (&xr)[RPW][MQ], float (&xq)[RPW][MQ], floatx4& xdl) {
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                bool ok;
                const int i = lane_off(r, m, ok);
                const size_t rb_ = row_base(bb, r);
                const float vr = (r3g + rb_)[i], vq = (q3g + rb_)[i];
                xr[r][m] = ok ? vr : 0.f;
                xq[r][m] = ok ? vq : 0.f;
            }
        xdl = ldc(reinterpret_cast<const floatx4*>(dl) + bb);
    };
    auto load_de = [&](int bb, float (&xd)[RPW][MQ], float (&x1)[RPW][MQ], float (&x2)[RPW][MQ]) {
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                bool ok;
                const int i = lane_off(r, m, ok);
                const size_t rb_ = row_base(bb, r);
                const float vd = (d2g + rb_)[i], v1 = (E1g + rb_)[i], v2 = (E2g + rb_)[i];
                xd[r][m] = ok ? vd : 0.f;
                x1[r][m] = ok ? v1 : 0.f;
                x2[r][m] = ok ? v2 : 0.f;
            }
    };

    // weight tables; rows F2 .. F2MAX - 1 of the four row buffers stay zero (MFMA operand reads)
    for (int i = tid; i < F2MAX * (F2MAX + K2); i += NTB) {
        float v = 0.f;
        if (i < F2MAX * F2MAX) {
            const int ii = i / F2MAX, j = i - ii * F2MAX;
            if (ii < F2 && j < F2) v = prm[g.o_W3 + j * F2 + ii];
        } else {
            const int k = i - F2MAX * F2MAX, o = k / K2;
            if (o < F2) v = prm[g.o_w2 + k];
        }
        W3t[i] = v;
    }
    if (F2 < F2MAX)
        for (int i = tid; i < 4 * (F2MAX - F2) * RSD; i += NTB) {
            const int buf = i / ((F2MAX - F2) * RSD), k = i - buf * ((F2MAX - F2) * RSD);
            DR0[buf * F2MAX * RSD + F2 * RSD + k] = 0.f;
        }
    // per-row BN3 constants (scalar loads: parameters and finalize 2 / 3's coefficients) and the
    // classifier weights of the lane's pooled feature
    float g3[RPW], b3[RPW], mu3[RPW], inv3[RPW], A3[RPW], B3[RPW], C3[RPW];
    float wfl[RPW][MQ][NCLS];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int o = RPW * wave + r, oo = (FULL || o < F2) ? o : 0;
        const bool on = FULL || o < F2;
        g3[r] = on ? ldc(prm + g.o_g3 + oo) : 0.f;
        b3[r] = on ? ldc(prm + g.o_b3 + oo) : 0.f;
        mu3[r] = on ? ldc(coef + CF_MU3 * CSTR + oo) : 0.f;
        inv3[r] = on ? ldc(coef + CF_INV3 * CSTR + oo) : 0.f;
        A3[r] = on ? ldc(coef + CF_A3 * CSTR + oo) : 0.f;
        B3[r] = on ? ldc(coef + CF_B3 * CSTR + oo) : 0.f;
        C3[r] = on ? ldc(coef + CF_C3 * CSTR + oo) : 0.f;
#pragma unroll
        for (int m = 0; m < MQ; ++m) {
            const int t = lane + 64 * m;
            const bool ft = on && t < 8 * T2;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) wfl[r][m][n] = ft ? prm[g.o_Wfc + n * NF + oo * T2 + (t >> 3)] : 0.f;
        }
    }
    floatx4 acc3 = {0.f, 0.f, 0.f, 0.f};        // dW3 tile: D[j = 4 lk + r][i = li]
    // dw2 of the own rows.  FULL (T1 = 64): as pass E's lag correlation, a Hankel block product on the
    // matrix cores -- t = 16 a + u, Cq[u][w] = sum_a dq[16 a + u] d2p[16 a + w - 7] (two 16 x 16 tiles,
    // w < 32, K = the 4 blocks a), accumulated over the trials; dw2[k] = sum_u Cq[u][u + k] once, after
    // the loop.  The A operand is the lane's own dq, the B operand its d2 row shifted by 7 / -9 lanes
    // (ds_bpermute).  Other shapes: per-lane partials over lane-shifted d2 rows.
    floatx4 hq[RPW][2];
    float acc2[RPW][K2];
    float sz1[RPW], sz2[RPW];                   // BN2-backward sums of the own rows
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        sz1[r] = 0.f; sz2[r] = 0.f;
        hq[r][0] = acc3; hq[r][1] = acc3;
#pragma unroll
        for (int k = 0; k < K2; ++k) acc2[r][k] = 0.f;
    }
    // the first two trials' rows: issued after the table / weight loads, so the LDS stores above wait
    // for those alone (trials past the range load the last trial's rows: unconditional loads)
    const int blast = b1 > b0 ? b1 - 1 : b0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        load_rq(min(b0 + k, blast), sr[k], sq[k], sdl[k]);
        load_de(min(b0 + k, blast), sd[k], se1[k], se2[k]);
    }
    barrier_lds();                           // tables and zero rows written (the row loads stay in flight)

    TRACE(g, 3, TR_PRO);
    TRACE_DECL();
    auto trial = [&](const int bt, const bool live, const int buf, float (&xr)[RPW][MQ], float (&xq)[RPW][MQ],
                     float (&xd)[RPW][MQ], float (&x1)[RPW][MQ], float (&x2)[RPW][MQ], floatx4& xdl) {
        const int b = min(bt, blast), bn = min(bt + 2, blast);
        float* DR = DR0 + buf * F2MAX * RSD;
        float* Qb = Q0 + buf * F2MAX * RSD;
        TRACE_PH(g, 3, 0, tph_);
        // step 1: dh -> dropout -> dp3 -> dz3 = dp3/8 ELU'(z3) -> dr = A3 dz3 + B3 + C3 xh3 (finalize 3's
        // batch constants), own rows; q rows alongside (the dW3 B operand)
        const floatx4 dlv = xdl;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int o = RPW * wave + r;
            if (FULL || o < F2) {
#pragma unroll
                for (int m = 0; m < MQ; ++m) {
                    const int t = lane + 64 * m;
                    const float xh = (xr[r][m] - mu3[r]) * inv3[r];
                    float dd = 0.f;
#pragma unroll
                    for (int n = 0; n < NCLS; ++n) dd = fmaf(dlv[n], wfl[r][m][n], dd);
                    const bool ft = t < 8 * T2;
                    const float kp = keep_mul(g, mask3, dk1, (unsigned)(b * NF + (ft ? o * T2 + (t >> 3) : 0)));
                    const float dz = ft ? dd * kp * 0.125f * elu_d(fmaf(g3[r], xh, b3[r])) : 0.f;
                    DR[o * RSD + t] = (FULL || t < T1) ? fmaf(A3[r], dz, fmaf(C3[r], xh, B3[r])) : 0.f;
                    Qb[o * RSD + t] = xq[r][m];
                }
            }
        }
        load_rq(bn, xr, xq, xdl);
        TRACE_PH(g, 3, 1, tph_);
        // the trial's dr / q rows complete; the other buffers are rewritten only after every wave has
        // passed the next trial's barrier (LDS only: the row loads stay in flight)
        barrier_lds();
        TRACE_PH(g, 3, 2, tph_);
        // dW3[j][i] += sum_t dr[j][t] q[i][t] on the matrix cores: k-steps dealt over the waves
        for (int ks = wave; ks < nks; ks += NWB) {
            const float a = DR[li * RSD + 4 * ks + lk], bq = Qb[li * RSD + 4 * ks + lk];
            acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(live ? a : 0.f, bq, acc3, 0, 0, 0);
        }
        // dq[i][t] = sum_j W3[j][i] dr[j][t] for the own rows i
        float dq[RPW][MQ];
        {
            float dv[F2MAX][MQ];
#pragma unroll
            for (int j = 0; j < F2MAX; ++j)
#pragma unroll
                for (int m = 0; m < MQ; ++m) dv[j][m] = j < F2 ? DR[j * RSD + lane + 64 * m] : 0.f;
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int o = RPW * wave + r, oo = (FULL || o < F2) ? o : 0;
                float w3r[F2MAX];
#pragma unroll
                for (int q4 = 0; q4 < F2MAX / 4; ++q4) {
                    const floatx4 w = lds_ld4(W3t + oo * F2MAX + 4 * q4);
                    w3r[4 * q4] = sgpr_f(w[0]); w3r[4 * q4 + 1] = sgpr_f(w[1]);
                    w3r[4 * q4 + 2] = sgpr_f(w[2]); w3r[4 * q4 + 3] = sgpr_f(w[3]);
                }
#pragma unroll
                for (int m = 0; m < MQ; ++m) {
                    float a = 0.f;
#pragma unroll
                    for (int j = 0; j < F2MAX; ++j)
                        if (j < F2) a = fmaf(w3r[j], dv[j][m], a);
                    dq[r][m] = a;
                }
            }
        }
        TRACE_PH(g, 3, 3, tph_);
        const size_t rb = (size_t)b * F2 * T1;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int o = RPW * wave + r;
            if (!FULL && o >= F2) continue;
            // dw2[o][k] += sum_t dq[o][t] d2p[o][t + k - 7]
            if constexpr (FULL) {
                const float dqg = live ? dq[r][0] : 0.f;
                const int i0 = lane - 7, i1 = lane + 9;
                const float d0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(max(i0, 0) * 4, __builtin_bit_cast(int, xd[r][0])));
                const float d1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(min(i1, 63) * 4, __builtin_bit_cast(int, xd[r][0])));
                hq[r][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(dqg, i0 >= 0 ? d0 : 0.f, hq[r][0], 0, 0, 0);
                hq[r][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(dqg, i1 < 64 ? d1 : 0.f, hq[r][1], 0, 0, 0);
            } else {
                float s[MQ], dqg[MQ];
#pragma unroll
                for (int m = 0; m < MQ; ++m) {
                    dqg[m] = live ? dq[r][m] : 0.f;
                    s[m] = xd[r][m];
                    acc2[r][7] = fmaf(dqg[m], s[m], acc2[r][7]);
                }
#pragma unroll
                for (int k = 8; k < K2; ++k) {
                    shl1<MQ>(s, lane);
#pragma unroll
                    for (int m = 0; m < MQ; ++m) acc2[r][k] = fmaf(dqg[m], s[m], acc2[r][k]);
                }
#pragma unroll
                for (int m = 0; m < MQ; ++m) s[m] = xd[r][m];
#pragma unroll
                for (int k = 6; k >= 0; --k) {
                    shr1<MQ>(s, lane);
#pragma unroll
                    for (int m = 0; m < MQ; ++m) acc2[r][k] = fmaf(dqg[m], s[m], acc2[r][k]);
                }
            }
            // dd2 = conv16_same_t(dq) -> dropout -> dp2; BN2-backward sums (E1 / E2 of pass B)
            float w2r[K2];
#pragma unroll
            for (int q4 = 0; q4 < K2 / 4; ++q4) {
                const floatx4 w = lds_ld4(W2t + o * K2 + 4 * q4);
                w2r[4 * q4] = sgpr_f(w[0]); w2r[4 * q4 + 1] = sgpr_f(w[1]);
                w2r[4 * q4 + 2] = sgpr_f(w[2]); w2r[4 * q4 + 3] = sgpr_f(w[3]);
            }
            float y[MQ];
            conv16_same_t2<MQ>(dq[r], w2r, y, lane);
#pragma unroll
            for (int m = 0; m < MQ; ++m) {
                const int t = lane + 64 * m;
                if (FULL || t < T1) {
                    const int gi = o * T1 + t;
                    const float dp = y[m] * keep_mul(g, mask2, dk0, (unsigned)(rb + gi));
                    st_pol<EEGNET_NT_MID>(dp, dp2g + rb + gi);
                    const float dpg = live ? dp * 0.25f : 0.f;
                    sz1[r] = fmaf(dpg, x1[r][m], sz1[r]);
                    sz2[r] = fmaf(dpg, x2[r][m], sz2[r]);
                }
            }
        }
        load_de(bn, xd, x1, x2);
        TRACE_PH(g, 3, 4, tph_);
    };
    for (int b = b0; b < b1; b += 2) {
        pace_prio(b - b0, b1 - b0);
        trial(b, true, 0, sr[0], sq[0], sd[0], se1[0], se2[0], sdl[0]);
        trial(b + 1, b + 1 < b1, 1, sr[1], sq[1], sd[1], se1[1], se2[1], sdl[1]);
    }
    TRACE_LOOP(g, 3);
    tail_prio();
    // ---- workgroup reduction: dW3 tiles summed over the waves in wave order; dw2 / sums per owner ----
    __syncthreads();                         // every wave is done with the row buffers
    float* red = sm;                         // [NWB][256]
    float* own = red + NWB * 256;            // [dw2 F2*16][Sdz2 F2][Sdz2x F2]
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave * 256 + (4 * lk + r) * 16 + li] = acc3[r];
    if constexpr (FULL) {
        // dw2[k] = sum_u Cq[u][u + k] from the wave's Hankel tiles (its own LDS scratch)
        float* hs = own + 18 * F2MAX + wave * (RPW * 2 * 256);
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int i = 0; i < 4; ++i) hs[((r * 2 + h) * 16 + 4 * lk + i) * 16 + li] = hq[r][h][i];
        wave_lds_fence();
        if (lane < RPW * K2) {
            const int r = lane / K2, k = lane % K2;
            float a = 0.f;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int w = u + k;
                a += hs[((r * 2 + (w >> 4)) * 16 + u) * 16 + (w & 15)];
            }
            own[(RPW * wave + r) * K2 + k] = a;
        }
        float v[4] = {sz1[0], sz1[1], sz2[0], sz2[1]};
        wave_reduce<4>(v);                   // lane 16 q: item q = (sz1, sz2)[q / 2] of row q % 2
        if ((lane & 15) == 0) {
            const int q = lane >> 4;
            own[F2 * K2 + (q >> 1) * F2 + RPW * wave + (q & 1)] = v[0];
        }
    } else {
        constexpr int NV = RPW * K2 + 2 * RPW;          // 36 items; lane 16 q holds item j + 9 q in v[j]
        float v[NV];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
#pragma unroll
            for (int k = 0; k < K2; ++k) v[r * K2 + k] = acc2[r][k];
            v[RPW * K2 + r] = sz1[r];
            v[RPW * K2 + RPW + r] = sz2[r];
        }
        wave_reduce<NV>(v);
        if ((lane & 15) == 0) {
            const int q = lane >> 4;
#pragma unroll
            for (int j = 0; j < NV / 4; ++j) {
                const int item = j + (NV / 4) * q;
                if (item < RPW * K2) {
                    const int o = RPW * wave + item / K2;
                    if (o < F2) own[o * K2 + item % K2] = v[j];
                } else {
                    const int e = item - RPW * K2, o = RPW * wave + (e % RPW);
                    if (o < F2) own[F2 * K2 + (e / RPW) * F2 + o] = v[j];
                }
            }
        }
    }
    __syncthreads();
    float* row = part + (size_t)blockIdx.x * g.nD;
    for (int c = tid; c < g.nD; c += NTB) {
        float val;
        if (c < F2 * F2) {
            const int j = c / F2, i = c - j * F2;
            val = wave_rows_sum<NWB>(red, NWB, 256, j * 16 + i);
        } else {
            val = own[c - F2 * F2];
        }
        pub(row + c, val);
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nD, fa, dsm)) { fin4(g, prm, dsm + 2, fa); TRACE(g, 3, TR_FIN); }
}

// ================================================================================================
// Eval-mode forward (model.py:91-99 with .eval()): one fused kernel, BN running statistics folded
// into per-row affine maps, no dropout.
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_infer(Geo g, const float* __restrict__ prm,
                                               const float* __restrict__ bn,
                                               const float* __restrict__ x, float* __restrict__ logits) {
    using G_ = KG<K1>;
    EEG_DIMS(g);
    TRACE(g, 5, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Xb0 = sm;             // one x buffer: the next trial lands after its last reader
    float* Ss = sm + C * RS;
    float* D2s = Ss + F2 * RS;
    float* Qs = D2s + F2 * RS2;
    float* Hs = Qs + F2 * RS2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* rm1 = bn;                 const float* rv1 = bn + g.F1;
    const float* rm2 = bn + 2 * g.F1;      const float* rv2 = rm2 + F2;
    const float* rm3 = rm2 + 2 * F2;     const float* rv3 = rm3 + F2;

    for (int i = tid; i < (C + F2) * RS + 2 * F2 * RS2; i += NTH) sm[i] = 0.f;
    float aw[KS];
    load_ws_frag<KS>(prm + g.o_ws, C, F2, aw, lane);
    const int o = wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0, gg = oo / g.D;
    float tap[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    float w2[K2], w3[F2MAX];
#pragma unroll
    for (int k = 0; k < K2; ++k) w2[k] = prm[g.o_w2 + oo * K2 + k];
#pragma unroll
    for (int i = 0; i < F2MAX; ++i) w3[i] = i < F2 ? prm[g.o_W3 + oo * F2 + i] : 0.f;
    // eval BN1 (model.py:32) and BN2 (model.py:47) folded: z2 = al * v + be; BN3: z3 = s3 r + b3
    float al, be, s3, b3;
    {
        const float a1 = prm[g.o_g1 + gg] / sqrtf(rv1[gg] + g.eps);
        const float c1 = prm[g.o_b1 + gg] - a1 * rm1[gg];
        float W = 0.f;
        for (int c = 0; c < C; ++c) W += prm[g.o_ws + oo * C + c];
        const float s2 = prm[g.o_g2 + oo] / sqrtf(rv2[oo] + g.eps);
        al = a1 * s2;
        be = (c1 * W - rm2[oo]) * s2 + prm[g.o_b2 + oo];
        s3 = prm[g.o_g3 + oo] / sqrtf(rv3[oo] + g.eps);
        b3 = prm[g.o_b3 + oo] - rm3[oo] * s3;
    }
    float pf[PF];
    if ((int)blockIdx.x < g.B) x_prefetch<PF>(x + (size_t)blockIdx.x * C * T, C, T, pf, tid);
    __syncthreads();
    x_store<PF>(pf, C, T, RS, LP, Xb0, tid);
    __syncthreads();

    int it = 0;
    TRACE(g, 5, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = blockIdx.x; b < g.B; b += gridDim.x, ++it) {
        const float* Xc = Xb0;
        float* Xn = Xb0;
        const int bnx = b + gridDim.x;
        if (bnx < g.B) x_prefetch<PF>(x + (size_t)bnx * C * T, C, T, pf, tid);
        spatial_mfma<KS>(Xc, aw, Ss, C, F2, NT16, RS, LP, wave, lane);
        __syncthreads();
        if (row_on) {
            const float* row = Ss + o * RS;
            float* drow = D2s + o * RS2 + LP2;
            for (int q = lane; q < T1; q += 64) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float v[4];
                fir4<K1, G_::OFF>(w, tap, v);
                float pe = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) pe += elu_f(fmaf(al, v[i], be));
                drow[q] = pe * 0.25f;
            }
        }
        if (bnx < g.B) x_store<PF>(pf, C, T, RS, LP, Xn, tid);
        __syncthreads();
        float r[MAXT1Q];
        block2_rows(F2, T1, RS2, D2s, Qs, w2, w3, row_on, o, lane, r);
#pragma unroll
        for (int m = 0; m < MAXT1Q; ++m) {
            const int t = lane + 64 * m;
            float e = (row_on && t < 8 * T2) ? elu_f(fmaf(s3, r[m], b3)) : 0.f;
            e += dpp<0xB1>(e);                 // 8-lane sums by DPP (xor 1, xor 2, half-row mirror)
            e += dpp<0x4E>(e);
            e += dpp<0x141>(e);
            if (row_on && (t & 7) == 0 && t < 8 * T2) Hs[o * T2 + (t >> 3)] = e * 0.125f;
        }
        __syncthreads();
        if (wave < NCLS) {
            const int n = wave;
            float a = 0.f;
            for (int i = lane; i < NF; i += 64) a = fmaf(prm[g.o_Wfc + n * NF + i], Hs[i], a);
            a = wave_sum(a);
            if (lane == 0) logits[(size_t)b * NCLS + n] = a + prm[g.o_bfc + n];
        }
        __syncthreads();
    }
}

}  // namespace eeg
