// eegnet_passes.hip -- the five streaming passes of the restructured EEGNet train step and the
// fused eval-mode forward.  Included by eegnet_kernels.hip (one translation unit).
//
// Workgroup = 1024 threads = 16 waves, one workgroup per CU, trials strided over the grid.  Wave w
// owns output row o = w of every per-trial [F2, T] plane (F2 <= 16), so its FIR taps are
// wave-uniform (SGPRs), the FIR windows it reads are lane-contiguous float4s (no LDS bank
// conflicts), and its per-row partial sums live in registers until the workgroup ends.  The next
// trial's x is fetched into registers a whole trial ahead and lands in the second LDS buffer.

namespace eeg {

// ================================================================================================
// Pass A: BN1 / BN2 batch statistics (model.py:32, 47).
// part row: [G0 K1][S0][H nH][Tl nTl][hs R][ts P][Sv F2][Sv2 F2]
//   G0[d] = sum_{c,t<T} X[t] X[t+d]       (lag-Gram of the padded rows, window start 0)
//   H[a,b] = sum_c x[a] x[b], 0<=a<=b<R    (head outer products -> Gram edge corrections)
//   Tl[u,v] = sum_c x[T-P+u] x[T-P+v]     (tail outer products)
//   hs / ts = head / tail sample sums       (window-sum corrections)
//   Sv, Sv2 = sum v, sum v^2 per row o      (BN2: y2 = a1 v + c1 W)
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_pass_a(Geo g, const float* __restrict__ prm,
                                                const float* __restrict__ x, float* __restrict__ part,
                                                FinArgs fa) {
    using G_ = KG<K1>;
    EEG_DIMS(g);
    TRACE(g, 0, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Xb0 = sm;             // one x buffer: the next trial lands after its last reader
    float* Ss = sm + C * RS;
    float* red = Ss + F2 * RS;                        // NWAVE * (K1 + 1)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < (C + F2) * RS; i += NTH) sm[i] = 0.f;
    float aw[KS];
    load_ws_frag<KS>(prm + g.o_ws, C, F2, aw, lane);

    // FIR row (wave-uniform) and its taps
    const int o = wave;
    const bool fir_on = o < F2;
    float tap[K1];
    {
        const int gg = (fir_on ? o : 0) / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    }
    float sv = 0.f, sv2 = 0.f;
    float G0[K1];
#pragma unroll
    for (int d = 0; d < K1; ++d) G0[d] = 0.f;
    float s0 = 0.f;
    // edge items: decode (row-index a, row-index b) once; b < 0 -> a plain sample sum
    float eacc[G_::NEI];
    int ea[G_::NEI], eb[G_::NEI];
#pragma unroll
    for (int i = 0; i < G_::NEI; ++i) {
        eacc[i] = 0.f;
        int e = tid + NTH * i;
        ea[i] = -1; eb[i] = -1;
        if (e < g.nH) {                                  // head pair (a <= b < R), a-major
            int a = 0;
            while (e >= g.R - a) { e -= g.R - a; ++a; }
            ea[i] = a; eb[i] = a + e;
        } else if ((e -= g.nH) < g.nTl) {                // tail pair (u <= v < P)
            int u = 0;
            while (e >= g.P - u) { e -= g.P - u; ++u; }
            ea[i] = T - g.P + u; eb[i] = T - g.P + u + e;
        } else if ((e -= g.nTl) < g.R) {
            ea[i] = e;
        } else if ((e -= g.R) < g.P) {
            ea[i] = T - g.P + e;
        } else {
            ea[i] = -2;                                  // unused slot
        }
    }
    float pf[PF];
    if ((int)blockIdx.x < g.B) x_prefetch<PF>(x + (size_t)blockIdx.x * C * T, C, T, pf, tid);
    __syncthreads();
    x_store<PF>(pf, C, T, RS, LP, Xb0, tid);
    __syncthreads();

    int it = 0;
    TRACE(g, 0, TR_PRO);
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
    for (int b = blockIdx.x; b < g.B; b += gridDim.x, ++it) {
        const float* Xc = Xb0;
        float* Xn = Xb0;
        const int bn = b + gridDim.x;
        if (bn < g.B) x_prefetch<PF>(x + (size_t)bn * C * T, C, T, pf, tid);
        spatial_mfma<KS>(Xc, aw, Ss, C, F2, NT16, RS, LP, wave, lane);
        // lag-Gram: items (c, quad), lanes of a wave on consecutive quads of one row
        for (int j = tid; j < C * TQ; j += NTH) {
            const int c = j / TQ, q = j - c * TQ;
            float w[4 * G_::NW];
            lds_window<G_::NW>(Xc + c * RS + 4 * q, w);
            float a[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = (4 * q + i < T) ? w[G_::OFF + i] : 0.f;
            s0 += (a[0] + a[1]) + (a[2] + a[3]);
#pragma unroll
            for (int d = 0; d < K1; ++d) {
                float acc = G0[d];
#pragma unroll
                for (int i = 0; i < 4; ++i) acc = fmaf(a[i], w[G_::OFF + i + d], acc);
                G0[d] = acc;
            }
        }
        // edge outer products / sums over channels
#pragma unroll
        for (int i = 0; i < G_::NEI; ++i) {
            if (ea[i] >= 0) {
                const float* xa = Xc + LP + ea[i];
                float acc0 = 0.f, acc1 = 0.f;
                if (eb[i] >= 0) {
                    const float* xb2 = Xc + LP + eb[i];
                    int c = 0;
                    for (; c + 1 < C; c += 2) {
                        acc0 = fmaf(xa[c * RS], xb2[c * RS], acc0);
                        acc1 = fmaf(xa[(c + 1) * RS], xb2[(c + 1) * RS], acc1);
                    }
                    if (c < C) acc0 = fmaf(xa[c * RS], xb2[c * RS], acc0);
                } else {
                    int c = 0;
                    for (; c + 1 < C; c += 2) { acc0 += xa[c * RS]; acc1 += xa[(c + 1) * RS]; }
                    if (c < C) acc0 += xa[c * RS];
                }
                eacc[i] += acc0 + acc1;
            }
        }
        TRACE_PH(g, 0, 0, tph_);
        __syncthreads();                                   // Ss complete
        TRACE_PH(g, 0, 1, tph_);
        if (fir_on) {
            const float* row = Ss + o * RS;
            for (int q = lane; q < TQ; q += 64) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float v[4];
                fir4<K1, G_::OFF>(w, tap, v);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (4 * q + i < T) { sv += v[i]; sv2 = fmaf(v[i], v[i], sv2); }
            }
        }
        TRACE_PH(g, 0, 2, tph_);
        if (bn < g.B) x_store<PF>(pf, C, T, RS, LP, Xn, tid);
        TRACE_PH(g, 0, 3, tph_);
        __syncthreads();                                   // Xn staged, Ss free
        TRACE_PH(g, 0, 4, tph_);
    }
    TRACE_LOOP(g, 0);

    // ---- workgroup reduction -> one partial row ----
    float* row = part + (size_t)blockIdx.x * g.nA;
    {
        constexpr int NR = K1 + 4, NQ = NR / 4;       // [G0 K1][s0][sv][sv2][pad]
        float rv[NR];
#pragma unroll
        for (int d = 0; d < K1; ++d) rv[d] = G0[d];
        rv[K1] = s0; rv[K1 + 1] = sv; rv[K1 + 2] = sv2; rv[K1 + 3] = 0.f;
        wave_reduce<NR>(rv);
        if ((lane & 15) == 0) {
            const int r0 = (lane >> 4) * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int idx = j + r0;
                if (idx <= K1) red[wave * (K1 + 1) + idx] = rv[j];
                else if (fir_on && idx == K1 + 1) pub(row + (K1 + 1 + g.nedge + o), rv[j]);
                else if (fir_on && idx == K1 + 2) pub(row + (K1 + 1 + g.nedge + F2 + o), rv[j]);
            }
        }
    }
    __syncthreads();
    if (tid <= K1) {
        float t = 0.f;
        for (int w = 0; w < NWAVE; ++w) t += red[w * (K1 + 1) + tid];
        pub(row + (tid), t);
    }
#pragma unroll
    for (int i = 0; i < G_::NEI; ++i)
        if (ea[i] != -2 && tid + NTH * i < g.nedge) pub(row + (K1 + 1 + tid + NTH * i), eacc[i]);
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nA, fa, dsm)) { fin1(g, prm, dsm + 2, dsm + tail_s_doubles(g.nA), fa); TRACE(g, 0, TR_FIN); }
}

// ================================================================================================
// Pass B: forward to d2, E1/E2 (pooled ELU' sums for the BN2 backward), BN3 statistics.
// part row: [Sr F2][Sr2 F2]
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_pass_b(Geo g, const float* __restrict__ prm,
                                                const float* coef,    // the finalize writes it: no __restrict__
                                                const float* __restrict__ x,
                                                const uint8_t* __restrict__ mask2,
                                                float* __restrict__ d2g, float* __restrict__ E1g,
                                                float* __restrict__ E2g, float* __restrict__ part,
                                                FinArgs fa) {
    using G_ = KG<K1>;
    EEG_DIMS(g);
    TRACE(g, 1, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Xb0 = sm;             // one x buffer: the next trial lands after its last reader
    float* Ss = sm + C * RS;
    float* D2s = Ss + F2 * RS;
    float* Qs = D2s + F2 * RS2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < (C + F2) * RS + 2 * F2 * RS2; i += NTH) sm[i] = 0.f;
    float aw[KS];
    load_ws_frag<KS>(prm + g.o_ws, C, F2, aw, lane);
    const int o = wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0;
    float tap[K1];
    {
        const int gg = oo / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    }
    float w2[K2], w3[F2MAX];
#pragma unroll
    for (int k = 0; k < K2; ++k) w2[k] = prm[g.o_w2 + oo * K2 + k];
#pragma unroll
    for (int i = 0; i < F2MAX; ++i) w3[i] = i < F2 ? prm[g.o_W3 + oo * F2 + i] : 0.f;
    const float al = coef[CF_AL2 * CSTR + oo], be = coef[CF_BE2 * CSTR + oo];
    const float ga = prm[g.o_g2 + oo], bt = prm[g.o_b2 + oo];
    float sr = 0.f, sr2 = 0.f;
    float pf[PF];
    if ((int)blockIdx.x < g.B) x_prefetch<PF>(x + (size_t)blockIdx.x * C * T, C, T, pf, tid);
    __syncthreads();
    x_store<PF>(pf, C, T, RS, LP, Xb0, tid);
    __syncthreads();

    int it = 0;
    TRACE(g, 1, TR_PRO);
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
    for (int b = blockIdx.x; b < g.B; b += gridDim.x, ++it) {
        const float* Xc = Xb0;
        float* Xn = Xb0;
        const int bn = b + gridDim.x;
        if (bn < g.B) x_prefetch<PF>(x + (size_t)bn * C * T, C, T, pf, tid);
        spatial_mfma<KS>(Xc, aw, Ss, C, F2, NT16, RS, LP, wave, lane);
        __syncthreads();                                   // Ss complete; Qs free
        // d2 / E1 / E2 of this row stay in registers until the next trial's x is staged: a global
        // store issued before that x_store would hold its vmcnt wait (loads and stores drain in order)
        float d2v[MAXT1Q], e1v[MAXT1Q], e2v[MAXT1Q];
        if (row_on) {
            const float* row = Ss + o * RS;
            float* drow = D2s + o * RS2 + LP2;
#pragma unroll
            for (int m = 0; m < MAXT1Q; ++m) {             // pool-4 windows = quads
                const int q = lane + 64 * m;
                if (q >= T1) break;
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float v[4];
                fir4<K1, G_::OFF>(w, tap, v);
                float pe = 0.f, e1 = 0.f, e2 = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float xh = fmaf(al, v[i], be);
                    const float z = fmaf(ga, xh, bt);
                    const float dz = elu_d(z);
                    pe += z > 0.f ? z : dz - 1.f;          // ELU(z) = exp(z) - 1 below 0
                    e1 += dz;
                    e2 = fmaf(dz, xh, e2);
                }
                const size_t gi = ((size_t)b * F2 + o) * T1 + q;
                const float d2 = pe * 0.25f * keep_mul(g, mask2, 0, gi);
                d2v[m] = d2; e1v[m] = e1; e2v[m] = e2;
                drow[q] = d2;
            }
            wave_lds_fence();
            // depthwise 1x16 'same' conv of this row (model.py:54-61): pad 7 | 8
            const float* dr = D2s + o * RS2 + 1;
            for (int t = lane; t < T1; t += 64) {
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < K2; ++k) a = fmaf(w2[k], dr[t + k], a);
                Qs[o * RS2 + t] = a;
            }
        }
        if (bn < g.B) x_store<PF>(pf, C, T, RS, LP, Xn, tid);
        if (row_on) {
#pragma unroll
            for (int m = 0; m < MAXT1Q; ++m) {
                const int q = lane + 64 * m;
                if (q >= T1) break;
                const size_t gi = ((size_t)b * F2 + o) * T1 + q;
                d2g[gi] = d2v[m]; E1g[gi] = e1v[m]; E2g[gi] = e2v[m];
            }
        }
        __syncthreads();                                   // Qs complete, Xn staged
        if (row_on) {                                      // pointwise F2 x F2 (model.py:62-69)
            for (int t = lane; t < T1; t += 64) {
                float r = 0.f;
#pragma unroll
                for (int i = 0; i < F2MAX; ++i)
                    if (i < F2) r = fmaf(w3[i], Qs[i * RS2 + t], r);
                sr += r;
                sr2 = fmaf(r, r, sr2);
            }
        }
    }
    TRACE_LOOP(g, 1);
    {
        float rv[4] = {sr, sr2, 0.f, 0.f};
        wave_reduce<4>(rv);                        // lane 0: sum sr, lane 16: sum sr2
        if (row_on && (lane == 0 || lane == 16)) {
            float* row = part + (size_t)blockIdx.x * g.nB;
            pub(row + (lane ? F2 + o : o), rv[0]);
        }
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nB, fa, dsm)) { fin2(g, dsm + 2, fa); TRACE(g, 1, TR_FIN); }
}

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
// Pass C: head (model.py:71-84).  logits, and (PC_BWD) classifier grads + BN3 backward sums.
// part row: [dWfc 4*NF][dbfc 4][Sdz3 F2][Sdz3x F2][loss]
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_pass_c(Geo g, const float* __restrict__ prm,
                                                const float* coef,    // the finalize writes it: no __restrict__
                                                const float* __restrict__ d2g,
                                                const uint8_t* __restrict__ mask3,
                                                const float* __restrict__ dlin,
                                                const int64_t* __restrict__ labels,
                                                float* __restrict__ logits, float* __restrict__ dlout,
                                                float* __restrict__ part, int mode, FinArgs fa) {
    EEG_DIMS(g);
    TRACE(g, 2, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2s = sm;
    float* Qs = D2s + F2 * RS2;
    float* Hs = Qs + F2 * RS2;
    float* DP3s = Hs + ((NF + 3) & ~3);
    float* Ls = DP3s + ((NF + 3) & ~3);        // 8
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int o = wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0;

    for (int i = tid; i < 2 * F2 * RS2; i += NTH) sm[i] = 0.f;
    float w2[K2], w3[F2MAX];
#pragma unroll
    for (int k = 0; k < K2; ++k) w2[k] = prm[g.o_w2 + oo * K2 + k];
#pragma unroll
    for (int i = 0; i < F2MAX; ++i) w3[i] = i < F2 ? prm[g.o_W3 + oo * F2 + i] : 0.f;
    const float mu3 = coef[CF_MU3 * CSTR + oo], inv3 = coef[CF_INV3 * CSTR + oo];
    const float g3 = prm[g.o_g3 + oo], b3 = prm[g.o_b3 + oo];
    // classifier-weight gradient items owned by this thread: p = tid + NTH * i < 4 * NF
    constexpr int MAXW = 4;                      // NF <= 1024
    float wacc[MAXW];
#pragma unroll
    for (int i = 0; i < MAXW; ++i) wacc[i] = 0.f;
    float bacc = 0.f, sdz = 0.f, sdzx = 0.f, lossacc = 0.f;
    const int nd2 = F2 * T1;
    float pfd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + NTH * j;
        pfd[j] = ((int)blockIdx.x < g.B && i < nd2) ? d2g[(size_t)blockIdx.x * nd2 + i] : 0.f;
    }
    __syncthreads();

    TRACE(g, 2, TR_PRO);
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + NTH * j;
            if (i < nd2) {
                const int oo2 = i / T1, t = i - oo2 * T1;
                D2s[oo2 * RS2 + LP2 + t] = pfd[j];
            }
        }
        const int bn = b + gridDim.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + NTH * j;
            if (bn < g.B && i < nd2) pfd[j] = d2g[(size_t)bn * nd2 + i];
        }
        TRACE_PH(g, 2, 0, tph_);
        __syncthreads();
        float r[MAXT1Q];
        block2_rows(F2, T1, RS2, D2s, Qs, w2, w3, row_on, o, lane, r);
        TRACE_PH(g, 2, 1, tph_);
        // BN3 (batch stats) -> ELU -> AvgPool(1,8) via 8-lane sums -> dropout -> h
        float xh[MAXT1Q], z[MAXT1Q];
#pragma unroll
        for (int m = 0; m < MAXT1Q; ++m) {
            const int t = lane + 64 * m;
            xh[m] = (r[m] - mu3) * inv3;
            z[m] = fmaf(g3, xh[m], b3);
            float e = (row_on && t < 8 * T2) ? elu_f(z[m]) : 0.f;
            e += __shfl_xor(e, 1, 64);
            e += __shfl_xor(e, 2, 64);
            e += __shfl_xor(e, 4, 64);
            if (row_on && (t & 7) == 0 && t < 8 * T2) {
                const int i = o * T2 + (t >> 3);
                Hs[i] = e * 0.125f * keep_mul(g, mask3, 1, (size_t)b * NF + i);
            }
        }
        __syncthreads();
        TRACE_PH(g, 2, 2, tph_);
        if (wave < NCLS) {                        // logits (model.py:78-82): wave n -> class n
            const int n = wave;
            float a = 0.f;
            for (int i = lane; i < NF; i += 64) a = fmaf(prm[g.o_Wfc + n * NF + i], Hs[i], a);
            a = wave_sum(a);
            if (lane == 0) Ls[n] = a + prm[g.o_bfc + n];
        }
        __syncthreads();
        TRACE_PH(g, 2, 3, tph_);
        if ((mode & PC_LOGITS) && tid < NCLS) logits[(size_t)b * NCLS + tid] = Ls[tid];
        if (mode & PC_BWD) {
            if (tid == 0) {
                float dl[NCLS];
                if (mode & PC_CE) {                  // nn.CrossEntropyLoss, mean (train.py:103)
                    float mx = Ls[0];
                    for (int n = 1; n < NCLS; ++n) mx = fmaxf(mx, Ls[n]);
                    float se = 0.f;
                    for (int n = 0; n < NCLS; ++n) se += expf(Ls[n] - mx);
                    const float lse = mx + logf(se);
                    const int y = (int)labels[b];
                    lossacc += lse - Ls[y];
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
            TRACE_PH(g, 2, 4, tph_);
            const float* DL = Ls + 4;
#pragma unroll
            for (int i = 0; i < MAXW; ++i) {
                const int p = tid + NTH * i;
                if (p < NCLS * NF) wacc[i] = fmaf(DL[p / NF], Hs[p % NF], wacc[i]);
            }
            if (tid < NCLS) bacc += DL[tid];
            for (int i = tid; i < NF; i += NTH) {
                float dh = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dh = fmaf(DL[n], prm[g.o_Wfc + n * NF + i], dh);
                DP3s[i] = dh * keep_mul(g, mask3, 1, (size_t)b * NF + i);
            }
            __syncthreads();
            TRACE_PH(g, 2, 5, tph_);
            if (row_on) {
#pragma unroll
                for (int m = 0; m < MAXT1Q; ++m) {
                    const int t = lane + 64 * m;
                    if (t < 8 * T2) {
                        const float dz = DP3s[o * T2 + (t >> 3)] * 0.125f * elu_d(z[m]);
                        sdz += dz;
                        sdzx = fmaf(dz, xh[m], sdzx);
                    }
                }
            }
        }
        __syncthreads();
        TRACE_PH(g, 2, 6, tph_);
    }
    TRACE_LOOP(g, 2);
    if (mode & PC_BWD) {
        float* row = part + (size_t)blockIdx.x * g.nC;
#pragma unroll
        for (int i = 0; i < MAXW; ++i) {
            const int p = tid + NTH * i;
            if (p < NCLS * NF) pub(row + (p), wacc[i]);
        }
        if (tid < NCLS) pub(row + (NCLS * NF + tid), bacc);
        const float a = wave_sum(sdz), ax = wave_sum(sdzx);
        if (row_on && lane == 0) {
            pub(row + (NCLS * NF + NCLS + o), a);
            pub(row + (NCLS * NF + NCLS + F2 + o), ax);
        }
        if (tid == 0) pub(row + (NCLS * NF + NCLS + 2 * F2), lossacc);
        double* dsm = (double*)sm;
        if (grid_reduce(g, part, g.nC, fa, dsm)) { fin3(g, prm, dsm + 2, fa); TRACE(g, 2, TR_FIN); }
    }
}

// ================================================================================================
// Pass D: block_2 backward (dW3, dw2), dp2 = d(pooled ELU output), BN2-backward sums.
// part row: [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2]
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_pass_d(Geo g, const float* __restrict__ prm,
                                                const float* coef,    // the finalize writes it: no __restrict__
                                                const float* __restrict__ d2g,
                                                const float* __restrict__ E1g,
                                                const float* __restrict__ E2g,
                                                const uint8_t* __restrict__ mask2,
                                                const uint8_t* __restrict__ mask3,
                                                const float* __restrict__ dl,
                                                float* __restrict__ dp2g, float* __restrict__ part,
                                                FinArgs fa) {
    EEG_DIMS(g);
    TRACE(g, 3, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2s = sm;
    float* Qs = D2s + F2 * RS2;        // q
    float* DRs = Qs + F2 * RS2;        // dr
    float* DQs = DRs + F2 * RS2;       // dq, padded LP2 | 8
    float* DP3s = DQs + F2 * RS2;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int o = wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0;

    for (int i = tid; i < 4 * F2 * RS2; i += NTH) sm[i] = 0.f;
    float w2[K2], w3[F2MAX], w3c[F2MAX];
#pragma unroll
    for (int k = 0; k < K2; ++k) w2[k] = prm[g.o_w2 + oo * K2 + k];
#pragma unroll
    for (int i = 0; i < F2MAX; ++i) {
        w3[i] = i < F2 ? prm[g.o_W3 + oo * F2 + i] : 0.f;     // row o of W3 (pw forward)
        w3c[i] = i < F2 ? prm[g.o_W3 + i * F2 + oo] : 0.f;    // column o of W3 (dq)
    }
    const float mu3 = coef[CF_MU3 * CSTR + oo], inv3 = coef[CF_INV3 * CSTR + oo];
    const float g3 = prm[g.o_g3 + oo], b3 = prm[g.o_b3 + oo];
    const float A3 = coef[CF_A3 * CSTR + oo], B3 = coef[CF_B3 * CSTR + oo], C3 = coef[CF_C3 * CSTR + oo];
    float dW3p[F2MAX], dw2p[K2];
#pragma unroll
    for (int i = 0; i < F2MAX; ++i) dW3p[i] = 0.f;
#pragma unroll
    for (int k = 0; k < K2; ++k) dw2p[k] = 0.f;
    float sz = 0.f, szx = 0.f;
    const int nd2 = F2 * T1;
    float pfd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int i = tid + NTH * j;
        pfd[j] = ((int)blockIdx.x < g.B && i < nd2) ? d2g[(size_t)blockIdx.x * nd2 + i] : 0.f;
    }
    __syncthreads();

    TRACE(g, 3, TR_PRO);
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + NTH * j;
            if (i < nd2) {
                const int oo2 = i / T1, t = i - oo2 * T1;
                D2s[oo2 * RS2 + LP2 + t] = pfd[j];
            }
        }
        const int bn = b + gridDim.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = tid + NTH * j;
            if (bn < g.B && i < nd2) pfd[j] = d2g[(size_t)bn * nd2 + i];
        }
        // dh -> dp3 (independent of block_2): DP3s[i] = (dl . Wfc[:,i]) * keep
        for (int i = tid; i < NF; i += NTH) {
            float dh = 0.f;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) dh = fmaf(dl[(size_t)b * NCLS + n], prm[g.o_Wfc + n * NF + i], dh);
            DP3s[i] = dh * keep_mul(g, mask3, 1, (size_t)b * NF + i);
        }
        __syncthreads();
        float r[MAXT1Q];
        block2_rows(F2, T1, RS2, D2s, Qs, w2, w3, row_on, o, lane, r);
        // BN3 backward with the batch constants of finalize 3: dr = A3 dz3 + B3 + C3 xh3
        if (row_on) {
#pragma unroll
            for (int m = 0; m < MAXT1Q; ++m) {
                const int t = lane + 64 * m;
                if (t < T1) {
                    const float xh = (r[m] - mu3) * inv3;
                    const float z = fmaf(g3, xh, b3);
                    const float dz = (t < 8 * T2) ? DP3s[o * T2 + (t >> 3)] * 0.125f * elu_d(z) : 0.f;
                    const float d = fmaf(A3, dz, fmaf(C3, xh, B3));
                    DRs[o * RS2 + t] = d;
                    // dW3[o][i] += dr[o][t] q[i][t]
#pragma unroll
                    for (int i = 0; i < F2MAX; ++i)
                        if (i < F2) dW3p[i] = fmaf(d, Qs[i * RS2 + t], dW3p[i]);
                }
            }
        }
        __syncthreads();
        if (row_on) {
            // dq[o][t] = sum_j W3[j][o] dr[j][t]
#pragma unroll
            for (int m = 0; m < MAXT1Q; ++m) {
                const int t = lane + 64 * m;
                if (t < T1) {
                    float a = 0.f;
#pragma unroll
                    for (int j = 0; j < F2MAX; ++j)
                        if (j < F2) a = fmaf(w3c[j], DRs[j * RS2 + t], a);
                    DQs[o * RS2 + LP2 + t] = a;
                }
            }
            wave_lds_fence();
            const float* dqr = DQs + o * RS2 + LP2;
            const float* d2r = D2s + o * RS2 + 1;
#pragma unroll
            for (int m = 0; m < MAXT1Q; ++m) {
                const int t = lane + 64 * m;
                if (t < T1) {
                    const float dq = dqr[t];
                    // dw2[o][k] += dq[o][t] d2pad[o][t+k]
#pragma unroll
                    for (int k = 0; k < K2; ++k) dw2p[k] = fmaf(dq, d2r[t + k], dw2p[k]);
                    // dd2[o][t] = sum_k w2[o][k] dq[o][t+7-k]
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < K2; ++k) a = fmaf(w2[k], dqr[t + 7 - k], a);
                    const size_t gi = ((size_t)b * F2 + o) * T1 + t;
                    const float dp = a * keep_mul(g, mask2, 0, gi);
                    dp2g[gi] = dp;
                    sz = fmaf(dp * 0.25f, E1g[gi], sz);
                    szx = fmaf(dp * 0.25f, E2g[gi], szx);
                }
            }
        }
        __syncthreads();
    }
    TRACE_LOOP(g, 3);
    float* row = part + (size_t)blockIdx.x * g.nD;
    {
        constexpr int NR = F2MAX + K2 + 4, NQ = NR / 4;   // [dW3 F2MAX][dw2 K2][sz][szx][pad 2]
        float rv[NR];
#pragma unroll
        for (int i = 0; i < F2MAX; ++i) rv[i] = dW3p[i];
#pragma unroll
        for (int k = 0; k < K2; ++k) rv[F2MAX + k] = dw2p[k];
        rv[F2MAX + K2] = sz; rv[F2MAX + K2 + 1] = szx; rv[F2MAX + K2 + 2] = 0.f; rv[F2MAX + K2 + 3] = 0.f;
        wave_reduce<NR>(rv);
        if (row_on && (lane & 15) == 0) {
            const int r0 = (lane >> 4) * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int idx = j + r0;
                if (idx < F2MAX) { if (idx < F2) pub(row + (o * F2 + idx), rv[j]); }
                else if (idx < F2MAX + K2) pub(row + (F2 * F2 + o * K2 + idx - F2MAX), rv[j]);
                else if (idx == F2MAX + K2) pub(row + (F2 * F2 + 16 * F2 + o), rv[j]);
                else if (idx == F2MAX + K2 + 1) pub(row + (F2 * F2 + 17 * F2 + o), rv[j]);
            }
        }
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nD, fa, dsm)) { fin4(g, prm, dsm + 2, fa); TRACE(g, 3, TR_FIN); }
}

// ================================================================================================
// Pass E: dy2 and the weight-gradient reductions that need full-rate data.
// part row: [Q F2*K1][Xm F2*C][Sdy F2][Sdyv F2]
// ================================================================================================
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTH) void k_pass_e(Geo g, const float* prm,   // Adam (finalize) writes it
                                                const float* coef,    // the finalize writes it: no __restrict__
                                                const float* __restrict__ x,
                                                const float* __restrict__ dp2g,
                                                float* __restrict__ part, FinArgs fa) {
    using G_ = KG<K1>;
    EEG_DIMS(g);
    TRACE(g, 4, TR_ENTRY);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    // x rows double-buffered when LDS allows (g.xdb): the next trial lands during phase B; otherwise
    // one buffer refilled after the dws GEMM, behind one extra barrier
    const bool xdb = g.xdb != 0;
    float* const Xb0 = sm;
    float* const Xb1 = sm + (xdb ? C * RS : 0);
    float* Ss = sm + (xdb ? 2 : 1) * C * RS;     // s, then e
    float* Dys = Ss + F2 * RS;                   // dy2 (same padded layout)
    float* DP = Dys + F2 * RS;                   // dp2 [F2][T1]
    float* red = sm;                             // NWAVE * 256, reused after the trial loop
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;

    for (int i = tid; i < ((xdb ? 2 : 1) * C + 2 * F2) * RS; i += NTH) sm[i] = 0.f;
    float aw[KS];
    load_ws_frag<KS>(prm + g.o_ws, C, F2, aw, lane);
    const int o = wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0;
    float tap[K1];
    {
        const int gg = oo / g.D;
#pragma unroll
        for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + gg * K1 + k];
    }
    const float al = coef[CF_AL2 * CSTR + oo], be = coef[CF_BE2 * CSTR + oo];
    const float ga = prm[g.o_g2 + oo], bt = prm[g.o_b2 + oo];
    const float Ao = coef[CF_AO * CSTR + oo], Bo = coef[CF_BO * CSTR + oo], Co = coef[CF_CO * CSTR + oo];
    float Q[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k) Q[k] = 0.f;
    float sdy = 0.f, sdyv = 0.f;
    // dws GEMM split: wave -> (c-tile ct, k-group range)
    const int wpc = NWAVE / NCT;
    const bool gemm_on = wave < wpc * NCT;
    const int ct = gemm_on ? wave / wpc : 0, part_ = gemm_on ? wave - ct * wpc : 0;
    const int kg0 = (NT16 * part_) / wpc, kg1 = gemm_on ? (NT16 * (part_ + 1)) / wpc : 0;
    floatx4 xacc = {0.f, 0.f, 0.f, 0.f};
    float pf[PF];
    // dp2 rows of the next trial ride along with its x (one trial ahead, registers): a synchronous
    // load here would wait (vmcnt is in order) for the whole x prefetch issued before it
    constexpr int NDP = (CC && TT) ? (FF * (TT / 4) + NTH - 1) / NTH : 4;   // F2 * T1 <= NDP * NTH
    const int ndp = F2 * T1;
    float pdp[NDP];
    if ((int)blockIdx.x < g.B) {
        x_prefetch<PF>(x + (size_t)blockIdx.x * C * T, C, T, pf, tid);
        for (int i = tid; i < ndp; i += NTH) DP[i] = dp2g[(size_t)blockIdx.x * ndp + i];
    }
    __syncthreads();
    x_store<PF>(pf, C, T, RS, LP, Xb0, tid);
    __syncthreads();

    int it = 0;
    TRACE(g, 4, TR_PRO);
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
    for (int b = blockIdx.x; b < g.B; b += gridDim.x, ++it) {
        const float* Xc = (it & 1) ? Xb1 : Xb0;
        float* Xn = (it & 1) ? Xb0 : Xb1;
        const int bn = b + gridDim.x;
        if (bn < g.B) {
            x_prefetch<PF>(x + (size_t)bn * C * T, C, T, pf, tid);
#pragma unroll
            for (int j = 0; j < NDP; ++j) {
                const int i = tid + NTH * j;
                if (i < ndp) pdp[j] = dp2g[(size_t)bn * ndp + i];
            }
        }
        spatial_mfma<KS>(Xc, aw, Ss, C, F2, NT16, RS, LP, wave, lane);
        TRACE_PH(g, 4, 0, tph_);
        __syncthreads();                                   // Ss, DP complete
        TRACE_PH(g, 4, 1, tph_);
        if (row_on) {
            const float* row = Ss + o * RS;
            float* drow = Dys + o * RS + LP;
            for (int q = lane; q < TQ; q += 64) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(row + 4 * q, w);
                float v[4];
                fir4<K1, G_::OFF>(w, tap, v);
                const float dpq = (q < T1) ? DP[o * T1 + q] * 0.25f : 0.f;
                float dy[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float xh = fmaf(al, v[i], be);
                    const float z = fmaf(ga, xh, bt);
                    const float dz = dpq * elu_d(z);
                    float d = fmaf(Ao, dz, fmaf(Co, xh, Bo));
                    d = (4 * q + i < T) ? d : 0.f;
                    dy[i] = d;
                    sdy += d;
                    sdyv = fmaf(d, v[i], sdyv);
                }
                // dW1 correlation: Q[k] += sum_i dy[i] * spad[t0+i+k]
#pragma unroll
                for (int k = 0; k < K1; ++k) {
                    float a = Q[k];
#pragma unroll
                    for (int i = 0; i < 4; ++i) a = fmaf(dy[i], w[G_::OFF + i + k], a);
                    Q[k] = a;
                }
                lds_st4(drow + 4 * q, (floatx4){dy[0], dy[1], dy[2], dy[3]});
            }
            TRACE_PH(g, 4, 2, tph_);
            wave_lds_fence();
            // e[P+s] = sum_m w1[K1-1-m] dypad[s+m]  (transposed FIR) -> overwrites this row of s
            const float* dyr = Dys + o * RS;
            float* erow = Ss + o * RS + LP;
            for (int q = lane; q < TQ; q += 64) {
                float w[4 * G_::NW];
                lds_window<G_::NW>(dyr + 4 * q, w);
                float e[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int m = 0; m < K1; ++m) a = fmaf(tap[K1 - 1 - m], w[G_::OFFD + i + m], a);
                    e[i] = (4 * q + i < T) ? a : 0.f;
                }
                lds_st4(erow + 4 * q, (floatx4){e[0], e[1], e[2], e[3]});
            }
        }
        TRACE_PH(g, 4, 3, tph_);
        if (xdb && bn < g.B) x_store<PF>(pf, C, T, RS, LP, Xn, tid);
        TRACE_PH(g, 4, 4, tph_);
        __syncthreads();                                   // e rows complete, Xn staged
        TRACE_PH(g, 4, 5, tph_);
        // Xm[o][c] += sum_t e[o][t] x[c][t] on the matrix cores; lane lk holds 4 consecutive t of
        // each 16-t group as a float4 (the k order inside a group is permuted identically in A and B)
        if (gemm_on) {
            const int c = ct * 16 + li;
            const float* arow = Ss + (li < F2 ? li : 0) * RS + LP + 4 * lk;
            const float* brow = Xc + (c < C ? c : 0) * RS + LP + 4 * lk;
            const bool aon = li < F2, bon = c < C;
            for (int kg = kg0; kg < kg1; ++kg) {
                floatx4 a4 = lds_ld4(arow + 16 * kg);
                floatx4 b4 = lds_ld4(brow + 16 * kg);
                if (!aon) a4 = (floatx4){0.f, 0.f, 0.f, 0.f};
                if (!bon) b4 = (floatx4){0.f, 0.f, 0.f, 0.f};
                xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[0], b4[0], xacc, 0, 0, 0);
                xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[1], b4[1], xacc, 0, 0, 0);
                xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[2], b4[2], xacc, 0, 0, 0);
                xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[3], b4[3], xacc, 0, 0, 0);
            }
        }
        if (bn < g.B) {                            // next trial's dp2 rows: every FIR reader is past
#pragma unroll
            for (int j = 0; j < NDP; ++j) {
                const int i = tid + NTH * j;
                if (i < ndp) DP[i] = pdp[j];
            }
        }
        TRACE_PH(g, 4, 6, tph_);
        __syncthreads();                                   // e rows consumed before the next s
        TRACE_PH(g, 4, 7, tph_);
        if (!xdb && bn < g.B) {
            x_store<PF>(pf, C, T, RS, LP, Xn, tid);
            __syncthreads();
        }
    }
    TRACE_LOOP(g, 4);
    __syncthreads();

    // ---- reductions ----
    float* row = part + (size_t)blockIdx.x * g.nE;
    {
        constexpr int NR = K1 + 4, NQ = NR / 4;         // [Q K1][sdy][sdyv][pad 2]
        float rv[NR];
#pragma unroll
        for (int k = 0; k < K1; ++k) rv[k] = Q[k];
        rv[K1] = sdy; rv[K1 + 1] = sdyv; rv[K1 + 2] = 0.f; rv[K1 + 3] = 0.f;
        wave_reduce<NR>(rv);
        if (row_on && (lane & 15) == 0) {
            const int r0 = (lane >> 4) * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int idx = j + r0;
                if (idx < K1) pub(row + (o * K1 + idx), rv[j]);
                else if (idx == K1) pub(row + (F2 * K1 + F2 * C + o), rv[j]);
                else if (idx == K1 + 1) pub(row + (F2 * K1 + F2 * C + F2 + o), rv[j]);
            }
        }
    }
    // Xm: wave -> 16x16 tile partial (rows 4lk+r, col li) -> LDS [wave][256] -> sum over the
    // waves of each c-tile
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave * 256 + (4 * lk + r) * 16 + li] = gemm_on ? xacc[r] : 0.f;
    __syncthreads();
    for (int p = tid; p < F2 * C; p += NTH) {
        const int oo2 = p / C, c = p - oo2 * C;
        const int ct2 = c >> 4, cc = c & 15;
        float a = 0.f;
        for (int w = ct2 * wpc; w < (ct2 + 1) * wpc; ++w) a += red[w * 256 + oo2 * 16 + cc];
        pub(row + (F2 * K1 + p), a);
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nE, fa, dsm)) { fin5(g, prm, dsm + 2, dsm + tail_s_doubles(g.nE), fa); TRACE(g, 4, TR_FIN); }
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
    unsigned long long tph_ = clock64(), tacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; (void)tph_; (void)tacc_;
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
            e += __shfl_xor(e, 1, 64);
            e += __shfl_xor(e, 2, 64);
            e += __shfl_xor(e, 4, 64);
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
