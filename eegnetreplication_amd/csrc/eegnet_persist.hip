// eegnet_persist.hip -- the persistent train step: ONE launch per step for the compile-time EEGNet-8,2
// shapes (22 x 256, 22 x 257), the five passes as phases of one co-resident grid.
// Included by eegnet_kernels.hip (one translation unit).
//
// Why.  The five-launch step (passes A..E, each ending in a ticketed two-level reduction and a
// one-workgroup finalize) pays, at every pass boundary, the reduction's serial tail, the finalize on
// one CU with the rest of the chip idle, the kernel drain and launch gap, and the next pass's prologue
// (~45 us of tails + ~14 us of prologues in a ~240 us B = 4096 step).
//
// How.  Every phase maps trials to workgroups the same way (trial_range over the grid of two 512-thread
// workgroups per CU), so every plane a phase reads (s, v, d2, E1, E2, q, r, dlogits, dp2) was written by
// the SAME workgroup in an earlier phase: the only cross-workgroup data of a step are the BatchNorm /
// gradient sums.  A phase boundary is then
//   publish the partial row -> grid barrier -> each workgroup sums its share of the columns (fp64, in a
//   fixed row order) -> grid barrier -> every workgroup reads the column totals and runs the pass's
//   finalize ITSELF (its own coefficient block, its own gradient copy; workgroup 0's are the real
//   gradients / running statistics / loss)
// with the next phase's first-trial loads issued before the wait (the body's `hook`).  Adam runs
// distributed: each workgroup updates its slice of the parameters from its own gradient copy.
//
// Residency.  The grid barriers need every workgroup resident: grid <= 2 x CUs, <= 128 VGPRs and
// <= 80 KB of LDS per workgroup (checked on the host with the occupancy query; the multi-launch step
// runs otherwise).  Every spin is bounded (a timeout sets the sticky error word, the step's loss
// becomes NaN, and the kernel finishes).
// Two persistent steps must never run concurrently on one device (they would split the CUs and wait
// for each other's workgroups): the step is opt-in per call (EEGNET_PERSIST), set by FusedTrainer,
// whose steps are stream-ordered.

namespace eeg {

// ---------------------------------------------------------------------------------------------
// Synchronisation words (one per 64-byte line): the departure counter (the last workgroup out of the
// kernel re-arms the release word and itself), the sticky error word (a bounded wait timed out: the
// grid was not co-resident; the last workgroup out then writes NaN into the loss, and the word stays
// set), and the release word (the grid reduction k of this launch is done: preduce).  Partial rows and
// column totals are written with agent-scope (sc1) stores and read with sc1 loads, drained before the
// hand-off (MI355X_MICROARCH.md, inter-workgroup visibility).
// ---------------------------------------------------------------------------------------------
constexpr int PS_STRIDE = 16;        // unsigned words between synchronisation words (64 B)
constexpr int PS_DEP = 0;            // departure word (index in PS_STRIDE units)
constexpr int PS_ERR = 1;            // error word
constexpr int PS_REL = 2;            // release word
constexpr int PS_WORDS = 3 * PS_STRIDE;
constexpr unsigned long long PS_TIMEOUT_TICKS = 100000000ull;   // 1 s of the 100 MHz wall clock

// fp64 sum over the 64 lanes, fixed butterfly order (every lane gets the total)
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// The grid reduction of one phase, every workgroup ending with the column totals in LDS S[ncols]
// (fp64).  The partial rows reduce exactly as in the stand-alone passes (grid_reduce: groups of 32
// rows reduced by the group's last arriving workgroup, the group partials by the last group reducer,
// tickets counted in `fa.cnt`, in a fixed row order -- the same totals bit for bit); that last
// reducer publishes the totals (sc1 stores) and raises the release word to k, which every other
// workgroup polls (one lane, bounded) before reading the totals (sc1 loads).  One poller per
// workgroup on one word: a barrier of 16 words polled by 16 lanes of every workgroup took 3-5 us.
// LDS: grid_reduce's [flag | S | scratch] from dsm.  (stamps, -DEEGNET_TRACE builds: row tp, TR_GRP
// when this workgroup is released, TR_TOP with the totals in LDS)
__device__ __forceinline__ double* preduce(const Geo& g, int tp, const float* part, int ncols, double* tot,
                                           unsigned* sync, unsigned k, double* dsm, FinArgs fa) {
    fa.tpass = tp;
    double* S = dsm + 2;
    if (grid_reduce(g, part, ncols, fa, dsm)) {
        for (int c = threadIdx.x; c < ncols; c += blockDim.x) pub(tot + c, S[c]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(sync + PS_STRIDE * PS_REL, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        TRACE(g, tp, TR_GRP);
    } else {
        if (threadIdx.x == 0) {
            const unsigned long long t0 = wall_clock64();
            while (__hip_atomic_load(sync + PS_STRIDE * PS_REL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t0 > PS_TIMEOUT_TICKS) {      // not co-resident: give up, flag it
                    __hip_atomic_store(sync + PS_STRIDE * PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
        TRACE(g, tp, TR_GRP);
        for (int c = threadIdx.x; c < ncols; c += blockDim.x) S[c] = ld_pub(tot + c);
    }
    __syncthreads();
    TRACE(g, tp, TR_TOP);
    return S;
}
// LDS doubles preduce uses from dsm: grid_reduce's flag, S and its flat-mode scratch
__host__ __device__ constexpr int preduce_doubles(int ncols) { return tail_s_doubles(ncols) + tail_scratch_doubles(ncols); }

// ---------------------------------------------------------------------------------------------
// Pass D for the persistent step (22 x 256 / 257, EEGNet-8,2): the block-2 backward of pass D
// (eegnet_passes.hip k_pass_d) re-laid for two workgroups per CU -- <= 80 KB of LDS and <= 128 VGPRs
// per workgroup (k_pass_d runs one 8-wave workgroup per CU with 145 KB and 225 VGPRs).  One trial per
// wave, lane t = pooled sample t (T/4 = 64).  Per-wave LDS, two row blocks:
//   P1 [16][68]: the q rows (pass B's depthwise output), then dq
//   P2 [16][84]: Hs (the head's input gradient, 128 floats), then the dr rows at +8, then the d2 rows
//                with their zero pads (7 | 64 | 13) for the dw2 correlation
// so d2 is re-read from the plane after the dW3 GEMM instead of held in registers across it, and the
// BN2-backward sums are folded per trial into 32 per-wave LDS accumulators instead of 32 registers.
// Partial row [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2], the layout of k_pass_d / fin4.
// ---------------------------------------------------------------------------------------------
constexpr int PD_RSQ = 68;                       // /4 odd: 16 rows read as float4 columns hit 16 bank quads
constexpr int PD_RSD = 84;
constexpr int PD_PW = 16 * PD_RSQ + 16 * PD_RSD; // floats per wave
constexpr int PD_NSZ = 2 * F2MAX;                // per-wave BN2-backward accumulators
__host__ __device__ constexpr int pd_lds_floats() { return (NTB / 64) * (PD_PW + PD_NSZ); }

template <int K1, int CC, int TT, int FF, class Hook>
__device__ __forceinline__ void pass_d_persist(const Geo& g, const float* __restrict__ prm, const float* coef,
                                               const float* __restrict__ d2g, const float* __restrict__ E1g,
                                               const float* __restrict__ E2g, const float* __restrict__ q3g,
                                               const float* __restrict__ r3g, const float* __restrict__ dl,
                                               float* __restrict__ dp2g, float* __restrict__ part, float* sm,
                                               const Hook& hook) {
    EEG_DIMS(g);
    static_assert(FF == F2MAX && TT / 4 == 64, "pass_d_persist: the 22 x 256 / 257 EEGNet-8,2 shapes");
    TRACE(g, 3, TR_ENTRY);
    constexpr int NFQ = (FF * (TT / 32) + 63) / 64;
    constexpr int NW = NTB / 64;
    const int tid = threadIdx.x, lane = tid & 63, li = lane & 15, lk = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    float* const P1 = sm + wave * PD_PW;
    float* const P2 = P1 + 16 * PD_RSQ;
    float* const Hs = P2;
    float* const SZ = sm + NW * PD_PW + wave * PD_NSZ;
    const unsigned dk0 = drop_key(g, 0), dk1 = drop_key(g, 1);
    int b0, b1;
    trial_range(g, b0, b1);
    const int bfirst = b0 + wave;
    float wf[NCLS][NFQ];
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            wf[n][u] = i < NF ? prm[g.o_Wfc + n * NF + i] : 0.f;
        }
    float q[F2MAX], r[F2MAX], dlv[NCLS];
    auto load_trial = [&](int bb) {
#pragma unroll
        for (int n = 0; n < NCLS; ++n) dlv[n] = dl[(size_t)bb * NCLS + n];
        const float* qb = q3g + (size_t)bb * F2 * T1;
        const float* rb = r3g + (size_t)bb * F2 * T1;
#pragma unroll
        for (int o = 0; o < F2MAX; ++o) { q[o] = qb[o * T1 + lane]; r[o] = rb[o * T1 + lane]; }
    };
#ifdef EEGNET_PD_PRELOAD
    if (bfirst < b1) load_trial(bfirst);
#endif
    hook();                                        // (k_step: pass C's sums -> fin3: BN3-backward constants)
    if (lane < PD_NSZ) SZ[lane] = 0.f;
    floatx4 acc3 = {0.f, 0.f, 0.f, 0.f};           // dW3 tile: D[j = 4 lk + r][i = li]
    const int o2 = lane >> 2, kq = lane & 3;       // dw2 item: row o2, taps 4 kq .. 4 kq + 3
    float acc2[4] = {0.f, 0.f, 0.f, 0.f};
    TRACE(g, 3, TR_PRO);
    for (int b = bfirst; b < b1; b += NW) {
#ifndef EEGNET_PD_PRELOAD
        load_trial(b);
#endif
        // dh -> dropout -> dp3 (flattened, model.py:74-75) into Hs
#pragma unroll
        for (int u = 0; u < NFQ; ++u) {
            const int i = lane + 64 * u;
            float dd = 0.f;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) dd = fmaf(dlv[n], wf[n][u], dd);
            if (i < NF) Hs[i] = dd * keep_mul(g, nullptr, dk1, (unsigned)(b * NF + i));
        }
#pragma unroll
        for (int o = 0; o < F2MAX; ++o) P1[o * PD_RSQ + lane] = q[o];
        wave_lds_fence();
        // BN3 backward (model.py:71, finalize 3's constants): dr = A3 dz3 + B3 + C3 xh3
        float dr[F2MAX];
#pragma unroll
        for (int j = 0; j < F2MAX; ++j) {
            const int oz = opaque0();
            const float mu3 = coef[CF_MU3 * CSTR + j + oz], inv3 = coef[CF_INV3 * CSTR + j + oz];
            const float g3 = prm[g.o_g3 + j + oz], b3 = prm[g.o_b3 + j + oz];
            const float A3 = coef[CF_A3 * CSTR + j + oz], B3 = coef[CF_B3 * CSTR + j + oz];
            const float C3 = coef[CF_C3 * CSTR + j + oz];
            const float xh = (r[j] - mu3) * inv3;
            const float dz = Hs[j * T2 + (lane >> 3)] * 0.125f * elu_d(fmaf(g3, xh, b3));
            dr[j] = fmaf(A3, dz, fmaf(C3, xh, B3));
        }
        wave_lds_fence();                          // every Hs read done: dr rows over it
#pragma unroll
        for (int j = 0; j < F2MAX; ++j) P2[j * PD_RSD + 8 + lane] = dr[j];
        wave_lds_fence();
        // dW3[j][i] += sum_t dr[j][t] q[i][t] on the matrix cores (float4 k-permuted operands)
        {
            const float* ar = P2 + li * PD_RSD + 8 + 2 * lk;
            const float* br = P1 + li * PD_RSQ + 2 * lk;
#pragma unroll
            for (int kg = 0; kg < 4; ++kg) {
                const floatx2 a0 = lds_ld2(ar + 16 * kg), a1 = lds_ld2(ar + 16 * kg + 8);
                const floatx2 b0 = lds_ld2(br + 16 * kg), b1 = lds_ld2(br + 16 * kg + 8);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0], b0[0], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1], b0[1], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0], b1[0], acc3, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1], b1[1], acc3, 0, 0, 0);
            }
        }
        // this trial's d2 rows and pass B's E1 / E2 (land during the dq phase).  The compiler barriers
        // keep loads where they are written: hoisted (the planes are __restrict__) they would hold 48
        // more registers through the BN3 backward
        float d[F2MAX], e1v[F2MAX], e2v[F2MAX];
        asm volatile("" ::: "memory");
        {
            const size_t rb = (size_t)b * F2 * T1;
#pragma unroll
            for (int o = 0; o < F2MAX; ++o) {
                d[o] = d2g[rb + o * T1 + lane];
                e1v[o] = E1g[rb + o * T1 + lane];
                e2v[o] = E2g[rb + o * T1 + lane];
            }
        }
        wave_lds_fence();                          // the GEMM's q / dr reads done
        // dq[i][t] = sum_j W3[j][i] dr[j][t] (registers, and over the q rows for the dw2 correlation)
        float dq[F2MAX];
#pragma unroll
        for (int i = 0; i < F2MAX; ++i) {
            const int oz = i >= 2 ? opaque0_after(dq[i >= 2 ? i - 2 : 0]) : opaque0();
            const float* w3c = prm + (g.o_W3 + i + oz);         // column i of W3 (stride F2)
            float a = 0.f;
#pragma unroll
            for (int j = 0; j < F2MAX; ++j) a = fmaf(w3c[j * F2], dr[j], a);
            dq[i] = a;
            P1[i * PD_RSQ + lane] = a;
        }
        // d2 rows over the dr rows: [0, 7) zero | d2 | [71, 84) zero (d2p[t + k - 7] at [t + k])
#pragma unroll
        for (int o = 0; o < F2MAX; ++o) {
            float* row = P2 + o * PD_RSD;
            row[7 + lane] = d[o];
            if (lane < 7) row[lane] = 0.f;
            if (lane < PD_RSD - 71) row[71 + lane] = 0.f;
        }
        wave_lds_fence();
        // dw2[o][k] += sum_t dq[o][t] d2p[o][t + k - 7]
        {
            const float* dqr = P1 + o2 * PD_RSQ;
            const float* d2r = P2 + o2 * PD_RSD + 4 * kq;
#pragma unroll 4
            for (int tq = 0; tq < 16; ++tq) {
                const floatx4 a4 = lds_ld4(dqr + 4 * tq);
                const floatx4 w0 = lds_ld4(d2r + 4 * tq), w1 = lds_ld4(d2r + 4 * tq + 4);
                const float w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc2[kk] = fmaf(a4[i], w[i + kk], acc2[kk]);
            }
        }
        // dd2 = conv16_same_t(dq) -> dropout -> dp2 (pass E's input); BN2-backward sums with E1 / E2
        float sz[2 * F2MAX];
        {
            const size_t rb = (size_t)b * F2 * T1;
#pragma unroll
            for (int o = 0; o < F2MAX; ++o) {
                const int oz = o >= 2 ? opaque0_after(sz[o >= 2 ? o - 2 : 0]) : opaque0();
                const float xo[1] = {dq[o]};
                float a[1];
                conv16_same_t<1>(xo, prm + (g.o_w2 + o * K2 + oz), a, lane);
                const int gi = o * T1 + lane;
                const float dp = a[0] * keep_mul(g, nullptr, dk0, (unsigned)(rb + gi));
                __builtin_nontemporal_store(dp, dp2g + rb + gi);
                sz[o] = dp * 0.25f * e1v[o];
                sz[F2MAX + o] = dp * 0.25f * e2v[o];
            }
        }
        wave_reduce<2 * F2MAX>(sz);                // lane 16 r: item j + 8 r in sz[j]
        if ((lane & 15) == 0) {
#pragma unroll
            for (int j = 0; j < 2 * F2MAX / 4; ++j) SZ[j + (lane >> 4) * (2 * F2MAX / 4)] += sz[j];
        }
        wave_lds_fence();
#ifdef EEGNET_PD_PRELOAD
        asm volatile("" ::: "memory");
        if (b + NW < b1) load_trial(b + NW);
#endif
    }
    TRACE(g, 3, TR_LOOP);
    // ---- workgroup reduction -> one partial row ----
    __syncthreads();
    float* red = sm;                               // [NW][nD] (the row blocks are done; SZ lies beyond)
    float* rw = red + wave * g.nD;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) rw[(4 * lk + rr) * F2 + li] = acc3[rr];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) rw[F2 * F2 + o2 * K2 + 4 * kq + kk] = acc2[kk];
    if (lane < PD_NSZ) rw[F2 * F2 + 16 * F2 + lane] = SZ[lane];      // [Sdz2 F2][Sdz2x F2]
    __syncthreads();
    float* row = part + (size_t)blockIdx.x * g.nD;
    for (int c = tid; c < g.nD; c += NTB) pub(row + c, wave_rows_sum<NW>(red, NW, g.nD, c));
}

// ---------------------------------------------------------------------------------------------
// The persistent step kernel
// ---------------------------------------------------------------------------------------------
struct StepArgs {
    const float* x;
    const int64_t* labels;
    float* params;           // flat parameters (Adam updates them at the end of the step)
    float* bn;               // running statistics
    int64_t* nbt;            // num_batches_tracked x 3 (nullable)
    float* grads;            // the step's (clamped) gradients
    float* adam_m;           // nullable: gradients only
    float* adam_v;
    int32_t* step;
    float lr, b1, b2, eps;
    float* loss;
    float* logits;           // nullable
    int cmode;               // pass C mode (PC_*)
    // workspace
    float *s, *v, *d2, *E1, *E2, *q3, *r3, *dl, *dp2;
    float *partA, *partB, *partC, *partD, *partE;
    double* tot;             // column totals of the current reduction
    unsigned* sync;          // PS_WORDS barrier words
    unsigned* cnt;           // the passes' ticket words (TK_COUNT x NCNT)
    double* part2;           // group partials of the ticketed reductions
    float* wcoef;            // [grid][CF_COUNT * CSTR]: each workgroup's coefficient block
    double* wstats;          // [grid][F1 K1 + K1]: each workgroup's fin1 -> fin5 statistics
    float* wgrads;           // [grid][nparam]: each workgroup's gradient copy (workgroup 0: `grads`)
};

#ifndef EEGNET_PHASES
#define EEGNET_PHASES 63      // (bisecting builds only: the phases compiled into k_step)
#endif
template <int K1, int CC, int TT, int FF>
__global__ __launch_bounds__(NTB, WPEB) void k_step(Geo gin, StepArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    Geo g = gin;
    shape_n22<TT>(g);                              // the shape fields as constants (EEG_SHAPE_N22)
    const int G = gridDim.x, wg = blockIdx.x, tid = threadIdx.x;
    TRACE(g, 0, TR_ENTRY);
    // this workgroup's finalize outputs: its own coefficient block, statistics and gradient copy;
    // workgroup 0's gradients are the real ones, and only it updates the running statistics, the
    // batch counters and the loss
    FinArgs fw;
    memset(&fw, 0, sizeof(fw));
    fw.coef = a.wcoef + (size_t)wg * (CF_COUNT * CSTR);
    fw.stats = a.wstats + (size_t)wg * (g.F1 * g.K1 + g.K1);
    fw.grads = wg == 0 ? a.grads : a.wgrads + (size_t)wg * g.nparam;
    fw.bn = wg == 0 ? a.bn : nullptr;
    fw.update_running = wg == 0 ? 1 : 0;
    fw.nbt = wg == 0 ? a.nbt : nullptr;
    fw.loss = wg == 0 ? a.loss : nullptr;
    fw.ce = (a.cmode & PC_CE) ? 1 : 0;
    // the Adam step counter as of this step (workgroup 0 advances it after the last barrier, when every
    // workgroup has read it and every dropout key derived from it has been drawn)
    const int step0 = a.adam_m ? *a.step : 0;
    const FoldCall fc0{};
    // the ticket words and group partials of pass tp's reduction (the stand-alone passes' own)
    auto tick = [&](int tp) {
        FinArgs f;
        memset(&f, 0, sizeof(f));
        f.cnt = a.cnt + tp * NCNT;
        f.part2 = a.part2;
        return f;
    };

    // ---- phase A: BN1 / BN2 statistics, the s and v planes ----
    if constexpr (EEGNET_PHASES & 1) pass_a_body<K1, CC, TT, FF, false, true>(g, a.params, a.x, a.s, a.v, a.partA, fw, fc0, sm);
    TRACE(g, 0, TR_PUB);
    // ---- phase B: after fin1 (every workgroup: BN1 / BN2 constants, the statistics for fin5) ----
    auto hookB = [&]() {
        double* dsm = (double*)sm;
        double* S = preduce(g, 0, a.partA, g.nA, a.tot, a.sync, 1, dsm, tick(0));
        fin1<K1>(g, a.params, S, dsm + preduce_doubles(g.nA), fw);
        __syncthreads();
        TRACE(g, 0, TR_FIN);
    };
    if constexpr (EEGNET_PHASES & 2) pass_b_body<K1, CC, TT, FF, false, true>(g, a.params, fw.coef, a.v, nullptr, a.d2, a.E1, a.E2, a.q3, a.r3,
                                             a.partB, fw, fc0, sm, hookB);
    TRACE(g, 1, TR_PUB);
    // ---- phase C: after fin2 (BN3 statistics) ----
    auto hookC = [&]() {
        double* S = preduce(g, 1, a.partB, g.nB, a.tot, a.sync, 2, (double*)sm, tick(1));
        fin2(g, S, fw);
        __syncthreads();
        TRACE(g, 1, TR_FIN);
    };
    if constexpr (EEGNET_PHASES & 4) pass_c_body<K1, CC, TT, FF, false, true>(g, a.params, fw.coef, a.r3, nullptr, nullptr, a.labels, a.logits, a.dl,
                                             a.partC, a.cmode, fw, fc0, sm, hookC);
    TRACE(g, 2, TR_PUB);
    // ---- phase D: after fin3 (classifier / BN3 gradients, BN3-backward constants, loss) ----
    auto hookD = [&]() {
        double* S = preduce(g, 2, a.partC, g.nC, a.tot, a.sync, 3, (double*)sm, tick(2));
        fin3(g, a.params, S, fw);
        __syncthreads();
        TRACE(g, 2, TR_FIN);
    };
    if constexpr (EEGNET_PHASES & 8) pass_d_persist<K1, CC, TT, FF>(g, a.params, fw.coef, a.d2, a.E1, a.E2, a.q3, a.r3, a.dl, a.dp2, a.partD, sm,
                                   hookD);
    TRACE(g, 3, TR_PUB);
    // ---- phase E: after fin4 (block-2 / BN2 gradients, BN2-backward constants); the hook's LDS is pass
    // E's dy / x rows, which its prologue does not touch before the first trial ----
    auto hookE = [&]() {
        double* dsm = (double*)(sm + 16 * row_stride(K1, TT));
        double* S = preduce(g, 3, a.partD, g.nD, a.tot, a.sync, 4, dsm, tick(3));
        fin4(g, a.params, S, fw);
        __syncthreads();
        TRACE(g, 3, TR_FIN);
    };
    if constexpr (EEGNET_PHASES & 16) pass_e_body<K1, CC, TT, FF, false, true>(g, a.params, fw.coef, a.x, a.s, a.v, a.dp2, a.partE, fw, fc0, sm, hookE);
    TRACE(g, 4, TR_PUB);
    // ---- after E: fin5 (spatial / BN1 / temporal-conv gradients) in every workgroup, then its Adam slice
    if constexpr (EEGNET_PHASES & 32) {
        __syncthreads();                           // pass E's LDS (its reduction scratch) is free
        double* S = preduce(g, 4, a.partE, g.nE, a.tot, a.sync, 5, (double*)sm, tick(4));
        fin5(g, a.params, S, (double*)sm + preduce_doubles(g.nE), fw);   // fw.adam_m == nullptr: gradients only
        __syncthreads();
        TRACE(g, 4, TR_FIN);
    }
    if (a.adam_m) {
        // torch.optim.Adam over this workgroup's slice of the flat parameters, from its own gradient
        // copy (identical in every workgroup); the same element update as fin5 / k_adam
        const int per = (g.nparam + G - 1) / G;
        const int i0 = min(g.nparam, wg * per), i1 = min(g.nparam, i0 + per);
        for (int i = i0 + tid; i < i1; i += NTB) {
            float step_size, bc2s;
            FinArgs fa;
            fa.lr = a.lr; fa.b1 = a.b1; fa.b2 = a.b2;
            adam_scalars(fa, step0 + 1, step_size, bc2s);
            float p = a.params[i], m = a.adam_m[i], v = a.adam_v[i];
            adam_elem(&p, fw.grads[i], &m, &v, a.b1, a.b2, step_size, bc2s, a.eps);
            a.params[i] = p; a.adam_m[i] = m; a.adam_v[i] = v;
        }
    }
    // ---- departure: the last workgroup out re-arms the barrier words; workgroup 0 advances the step
    __syncthreads();
    if (tid == 0) {
        if (wg == 0 && a.adam_m) *a.step = step0 + 1;
        const unsigned prev = __hip_atomic_fetch_add(a.sync + PS_STRIDE * PS_DEP, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)G - 1u) {
            // a timed-out wait anywhere in this step (or an earlier one: the word is sticky) makes the
            // step's loss NaN, so the failure cannot pass unnoticed
            if (a.loss && __hip_atomic_load(a.sync + PS_STRIDE * PS_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                *a.loss = __builtin_nanf("");
            __hip_atomic_store(a.sync + PS_STRIDE * PS_REL, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.sync + PS_STRIDE * PS_DEP, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace eeg
