// eegnet_infer_bf16r.hip -- bf16 batched eval forward of BASELINE cfg5 (EEGNet-16,4 on 64ch x 512),
// time-chunked with no x halo.  Included by eegnet_kernels.hip.
//
// Same arithmetic as k_infer_bf16 / k_infer_bf16_cfg5 (BN-folded spatial GEMM, 32-tap FIR, folded BN1 /
// BN2 + ELU + pool4, depthwise 1x16, pointwise, BN3 + ELU + pool8, classifier; bf16 operands, fp32
// accumulation; reference: EEGNet.forward in eval mode, src/eegnet_repl/model.py:91-99).  What changes
// against k_infer_bf16_cfg5 (eegnet_infer_bf16c.hip) is how x reaches the spatial GEMM:
//
// * A chunk is the 64 NEW samples of every channel row -- no 'same' halo.  The FIR runs one step
//   behind the spatial GEMM: step j produces v at t = 64j - 16 .. 64j + 47 from s at 64j - 31 .. 64j + 63,
//   i.e. from this chunk's s and the last 32 s samples of the previous one, which the spatial GEMM of
//   the previous step also wrote into a small tail buffer (two, alternating by step).  A ninth step per
//   trial drains the lag with s = 0 past the trial's end.  The spatial GEMM therefore runs on 64 samples
//   per chunk instead of 96 (2/3 of the MFMAs) and each x byte crosses L2 -> LDS once instead of 1.5x.
// * A 64-sample chunk is half an x image row (128 bf16: the transposed-read swizzle's row), so two
//   16 KB images hold FOUR chunk slots: three chunks are in flight (LDS-DMA, no registers) while the
//   fourth is read, against one in k_infer_bf16_cfg5.
// * Logits are staged in LDS and stored after the loop (or when the staging fills): a global store in
//   the loop would sit in the vector-memory queue between the chunk DMAs.
namespace eeg {
namespace c5r {

constexpr int C = 64, T = 512, F1 = 16, D = 4, F2 = 64, K1 = 32, T1 = 128, T2 = 16, NF = F2 * T2;
constexpr int TC = 64;                       // new samples per chunk
constexpr int NCH = T / TC;                  // chunks per trial
constexpr int NST = NCH + 1;                 // FIR steps per trial (the last drains the lag)
constexpr int XROWB = 256;                   // x image row (bytes): 128 bf16 = two chunk slots
constexpr int XIMG = C * XROWB;              // 16 KB per image, two chunk slots
constexpr int NROW = 88;                     // new-s row (bf16): 0..63 written, 64..79 read at zero
                                             // weight (kept 0); 44 dwords = 4 mod 8
constexpr int TROW = 40;                     // tail row (bf16): 32 samples; 20 dwords = 4 mod 8
constexpr int AROW = 144;                    // a row (bf16): [8 zeros | 128 pooled | 8 zeros]
constexpr int W2R = 48;                      // depthwise taps, bf16, [16 zeros | 16 taps | 16 zeros]
constexpr int NT = 512;                      // threads: 8 waves
constexpr int NW = NT / 64;
constexpr int LGCAP = 64;                    // logits staged per workgroup between flushes
// LDS carve (bytes)
constexpr int OFF_X = 0;                     // two images = four chunk slots
constexpr int OFF_N = 2 * XIMG;              // new-s rows
constexpr int TBUF = F2 * TROW * 2;
constexpr int OFF_T = OFF_N + F2 * NROW * 2; // two tail buffers
constexpr int OFF_A = OFF_T + 2 * TBUF;      // a rows
constexpr int OFF_Z = OFF_N;                 // z image (after the trial's last FIR step): over the new-s
                                             // rows and tail buffer 0
constexpr int OFF_W2 = OFF_A + F2 * AROW * 2;
constexpr int OFF_CO = OFF_W2 + F2 * W2R * 2;
constexpr int OFF_LG = OFF_CO + 4 * F2 * 4;  // [NW][NCLS] logit partials
constexpr int OFF_LS = OFF_LG + NW * NCLS * 4;   // [LGCAP][NCLS] staged logits
constexpr int LDS = OFF_LS + LGCAP * NCLS * 4;
static_assert(LDS <= 80 * 1024, "two workgroups per CU");
static_assert(OFF_Z + F2 * XROWB <= OFF_T + TBUF, "the z image covers the new-s rows and tail buffer 0 only");
static_assert(F1 * K1 * 4 <= TBUF, "the prologue's tap table fits in tail buffer 1");
static_assert(F2 % 16 == 0 && 16 % D == 0 && TC == 16 * (16 / D), "FIR columns = rows of a group x tiles");

}  // namespace c5r

// chunk q of trial xb (bf16 [C][T]) into chunk slot `slot` (image slot >> 1, row half slot & 1):
// samples 64q .. 64q + 63 of every channel row.  Physical 16-byte unit up of row r holds logical unit
// up ^ 2h(r) (trimg_off's 8-byte chunk swizzle ch ^ 4h, on unit pairs); the logical units of this slot
// are the row's half `slot & 1`.  A wave-instruction writes 1 KiB contiguous (4 rows): the lanes whose
// physical unit belongs to the other slot are masked off.  Each wave issues 2 wave-instructions.
__device__ __forceinline__ void x_chunk_dma_r(const uint16_t* __restrict__ xb, int q, char* smc, int slot,
                                              int wave, int lane) {
    using namespace c5r;
    char* const img = smc + OFF_X + (slot >> 1) * XIMG;
    const int half = slot & 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * (wave + NW * i);
        const int r = r0 + (lane >> 4), up = lane & 15;
        const int h = (r & 3) | ((r >> 1) & 4);
        const int u = up ^ (2 * h);
        if ((u >> 3) == half) dma16c(xb + (size_t)r * T + TC * q + 8 * (u & 7), img + r0 * XROWB);
    }
}

// wait for the chunk DMAs issued before the `newer` most recent chunks (2 wave-instructions each)
__device__ __forceinline__ void wait_chunk_r(int newer) {
    switch (newer) {
        case 3: asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
}

// __launch_bounds__ second argument: minimum waves per SIMD (4: two 8-wave workgroups per CU, <= 128 VGPRs)
__global__ __launch_bounds__(c5r::NT, 4) void k_infer_bf16_cfg5r(GeoI g, const float* __restrict__ prm,
                                                                 const float* __restrict__ bn,
                                                                 const uint16_t* __restrict__ x,
                                                                 float* __restrict__ logits) {
    using namespace c5r;
    extern __shared__ __attribute__((aligned(16))) char smr[];
    char* const Ni = smr + OFF_N;                       // new s rows of the current step
    char* const Ai = smr + OFF_A;                       // pooled rows a (bf16), whole trial
    char* const Zi = smr + OFF_Z;                       // z image (bf16, swizzled) over new-s / tail 0
    float* const W1t = reinterpret_cast<float*>(smr + OFF_T + TBUF);   // prologue only (tail buffer 1)
    uint16_t* const W2p = reinterpret_cast<uint16_t*>(smr + OFF_W2);
    float* const Co = reinterpret_cast<float*>(smr + OFF_CO);   // [4][F2]: al, be, s3, b3
    float* const Lg = reinterpret_cast<float*>(smr + OFF_LG);   // [NW][4] logit partials
    float* const Ls = reinterpret_cast<float*>(smr + OFF_LS);   // [LGCAP][4] staged logits
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = lane >> 4, l15 = lane & 15;
    const int B = g.B, gs = gridDim.x, b0 = blockIdx.x;
    const int ntr = (B - b0 + gs - 1) / gs;             // this workgroup's trials (>= 1: grid <= B)
    const int ntot = NCH * ntr;                         // and chunks
    auto chunk_dma = [&](int qx) {                      // chunk qx of the workgroup's sequence -> slot qx & 3
        const int b = b0 + gs * (qx / NCH);
        x_chunk_dma_r(x + (size_t)b * C * T, qx % NCH, smr, qx & 3, wave, lane);
    };

    // ---- prologue: the first four chunks in flight, then tables and zero fills ----
    for (int qx = 0; qx < 4 && qx < ntot; ++qx) chunk_dma(qx);
    if (tid < F2) {
        const int o = tid, gg = o / D;
        const float* rm1 = bn;             const float* rv1 = bn + F1;
        const float* rm2 = bn + 2 * F1;    const float* rv2 = rm2 + F2;
        const float* rm3 = rm2 + 2 * F2;   const float* rv3 = rm3 + F2;
        const float a1 = prm[g.o_g1 + gg] / sqrtf(rv1[gg] + g.eps);
        const float c1 = prm[g.o_b1 + gg] - a1 * rm1[gg];
        float W = 0.f;
        for (int c = 0; c < C; ++c) W += prm[g.o_ws + o * C + c];
        const float s2 = prm[g.o_g2 + o] / sqrtf(rv2[o] + g.eps);
        const float s3 = prm[g.o_g3 + o] / sqrtf(rv3[o] + g.eps);
        Co[o] = a1 * s2;
        Co[F2 + o] = (c1 * W - rm2[o]) * s2 + prm[g.o_b2 + o];
        Co[2 * F2 + o] = s3;
        Co[3 * F2 + o] = prm[g.o_b3 + o] - rm3[o] * s3;
    }
    for (int i = tid; i < F1 * K1; i += NT) W1t[i] = prm[g.o_w1 + i];
    for (int i = tid; i < F2 * W2R; i += NT) {
        const int o = i / W2R, k = i - o * W2R - 16;
        W2p[i] = __builtin_bit_cast(uint16_t, (__bf16)((k >= 0 && k < K2) ? prm[g.o_w2 + o * K2 + k] : 0.f));
    }
    // new-s rows (positions 64..79 stay 0), tail buffer 0 (s before t = 0 is 0), a rows (pads)
    for (int i = tid; i < F2 * NROW / 2; i += NT) reinterpret_cast<uint32_t*>(Ni)[i] = 0u;
    for (int i = tid; i < TBUF / 4; i += NT) reinterpret_cast<uint32_t*>(smr + OFF_T)[i] = 0u;
    for (int i = tid; i < F2 * AROW / 2; i += NT) reinterpret_cast<uint32_t*>(Ai)[i] = 0u;

    // spatial GEMM: this wave's o-tile (ws^T B operand, K = c, both K-steps in registers) and t-tiles
    const int ot = wave & 3, tt0 = wave >> 2;
    bf16x8 wsf[2];
#pragma unroll
    for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
            wsf[kc][jj] = (__bf16)prm[g.o_ws + (ot * 16 + l15) * C + kc * 32 + 8 * G + jj];
    // pointwise A operand (W3, K = i): the same o-tile of output rows j
    bf16x8 w3f[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
            w3f[ks][jj] = (__bf16)prm[g.o_W3 + (ot * 16 + l15) * F2 + ks * 32 + 8 * G + jj];
    // classifier weights this lane multiplies (k_infer_bf16_cfg5's layout: after pool8 the lanes of an
    // 8-lane group hold the group's 4 pooled values; lane p = l15 & 7 takes row p >> 1, classes 2 (p & 1) + {0, 1})
    const int prr = (l15 & 7) >> 1, pc0 = 2 * (l15 & 1);
    float wfl[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int f = (ot * 16 + 4 * G + prr) * T2 + 2 * (tt0 + 2 * m) + (l15 >> 3);
        wfl[m][0] = prm[g.o_Wfc + pc0 * NF + f];
        wfl[m][1] = prm[g.o_Wfc + (pc0 + 1) * NF + f];
    }
    __syncthreads();                                   // tables (not the DMA: asm, waited per chunk)

    // FIR: this wave's two temporal groups gi = 2 wave + {0, 1}; banded Toeplitz A operand of each
    // group's taps, A[i][j] = w1[g][j - i - 1] over K = 64 (two K-steps), held for the whole kernel
    bf16x8 af[2][2];
    float al2[2], be2[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int gg = 2 * wave + q;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const int k = 32 * s + 8 * G + jj - l15 - 1;
                af[q][s][jj] = (__bf16)((k >= 0 && k < K1) ? W1t[gg * K1 + k] : 0.f);
            }
        const int o = D * gg + (l15 >> 2);
        al2[q] = Co[o] * 1.4426950408889634f;              // ELU in log2 units (k_infer_bf16)
        be2[q] = Co[F2 + o] * 1.4426950408889634f;
    }
    // the classifier bias: held in a register (a global load in the loop would wait, in order, for the
    // chunk DMAs issued before it)
    const float bfc = tid < NCLS ? prm[g.o_bfc + tid] : 0.f;
    float s3r[4], b3r[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        s3r[rr] = Co[2 * F2 + ot * 16 + 4 * G + rr];
        b3r[rr] = Co[3 * F2 + ot * 16 + 4 * G + rr];
    }
#ifdef EEGNET_TRACE
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_ = clock64();
#define PH_(k) do { if (g.dbg && tid == 0) { const unsigned long long t1_ = clock64(); ph[k] += t1_ - t_; t_ = t1_; } } while (0)
#else
#define PH_(k) do {} while (0)
#endif

    int qc = 0, J = 0, ls = 0;                          // chunk / step counters, staged logits
    for (int it = 0; it < ntr; ++it) {
#pragma unroll 1
        for (int j = 0; j < NST; ++j) {
            char* const Tcur = smr + OFF_T + (J & 1) * TBUF;        // s 64j - 32 .. 64j - 1
            char* const Tnxt = smr + OFF_T + ((J + 1) & 1) * TBUF;  // the next step's
            // ---- 1. spatial GEMM s^T[t][o] of chunk j (16 t x 16 o tiles, A = x^T by transposed
            //         reads) -> new-s rows, and the chunk's last 32 samples -> the next tail buffer;
            //         the draining step writes zeros (s past the trial's end) ----
            if (j < NCH) {
                wait_chunk_r(min(3, ntot - 1 - qc));   // chunk qc landed; every FIR read of Ni / Tnxt done
                PH_(0);
                const char* Xi = smr + OFF_X + ((qc & 3) >> 1) * XIMG;
                const int nb = 4 * (qc & 1);
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const int nl = tt0 + 2 * m, n = nb + nl;
                    const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
                    const bf16x8 a0 = tr_frag(Xi, XROWB, 0, 16 * n, lane), a1 = tr_frag(Xi, XROWB, 32, 16 * n, lane);
                    floatx4 acc = mfma_bf16(a0, wsf[0], z4);
                    acc = mfma_bf16(a1, wsf[1], acc);
                    uintx2 pk;
                    pk[0] = pack_bf16x2(acc[0], acc[1]);
                    pk[1] = pack_bf16x2(acc[2], acc[3]);
                    const int o = ot * 16 + l15;
                    *reinterpret_cast<uintx2*>(Ni + o * (2 * NROW) + 2 * (16 * nl + 4 * G)) = pk;
                    if (nl >= 2) *reinterpret_cast<uintx2*>(Tnxt + o * (2 * TROW) + 2 * (16 * (nl - 2) + 4 * G)) = pk;
                }
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // FIR reads done
                PH_(0);
                const uintx2 zz = {0u, 0u};
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const int nl = tt0 + 2 * m, o = ot * 16 + l15;
                    *reinterpret_cast<uintx2*>(Ni + o * (2 * NROW) + 2 * (16 * nl + 4 * G)) = zz;
                    if (nl >= 2) *reinterpret_cast<uintx2*>(Tnxt + o * (2 * TROW) + 2 * (16 * (nl - 2) + 4 * G)) = zz;
                }
            }
            PH_(1);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");       // s rows complete
            PH_(2);
            if (j < NCH) {                                 // chunk qc's slot is free: chunk qc + 4 into it
                if (qc + 4 < ntot) chunk_dma(qc + 4);
                ++qc;
            }
            // ---- 2. FIR (banded Toeplitz MFMA), folded BN, ELU, pool4 -> a rows ----
            // window position p (0..111) of the step's s row: p < 32 in the tail buffer, else new-s p - 32
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int gg = 2 * wave + q;
                const int o = D * gg + (l15 >> 2), tile = l15 & 3;
                const int p0 = 16 * tile + 8 * G;
                const char* w0 = p0 < 32 ? Tcur + o * (2 * TROW) + 2 * p0 : Ni + o * (2 * NROW) + 2 * (p0 - 32);
                const char* w1 = Ni + o * (2 * NROW) + 2 * p0;
                floatx4 acc = {0.f, 0.f, 0.f, 0.f};
                acc = mfma_bf16(af[q][0], *reinterpret_cast<const bf16x8*>(w0), acc);
                acc = mfma_bf16(af[q][1], *reinterpret_cast<const bf16x8*>(w1), acc);
                // lane: v[o][t = 64j - 16 + 16 tile + 4G + r]; pooled sample 16j - 4 + 4 tile + G
                float pp = 0.f, pn = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float y = fmaf(al2[q], acc[r], be2[q]);
                    pp += fmaxf(y, 0.f);
                    pn += __builtin_amdgcn_exp2f(fminf(y, 0.f));
                }
                const float a = fmaf(0.25f * 0.6931471805599453f, pp, 0.25f * pn - 1.f);
                const int pq = 16 * j - 4 + 4 * tile + G;
                if (pq >= 0 && pq < T1) reinterpret_cast<__bf16*>(Ai)[o * AROW + 8 + pq] = (__bf16)a;
            }
            PH_(3);
            ++J;
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");           // a rows complete
        PH_(4);

        // ---- 3. depthwise 1x16 (pad 7 | 8) on the matrix cores -> z image ----
        // z[o][16n + i] = sum_j A[i][j] W_n[j], A[i][j] = w2[o][j - i - 1], W_n[j] = a[o][16n + j - 8]
#pragma unroll 4
        for (int rr = 0; rr < F2 / NW; ++rr) {
            const int o = wave * (F2 / NW) + rr;
            const uint16_t* wp = W2p + o * W2R + 15 + 8 * G - l15;
            bf16x8 aw;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) aw[jj] = __builtin_bit_cast(__bf16, wp[jj]);
            const int tile = l15 & 7;
            const bf16x8 win = *reinterpret_cast<const bf16x8*>(Ai + o * (2 * AROW) + 2 * (16 * tile + 8 * G));
            const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
            const floatx4 acc = mfma_bf16(aw, win, z4);
            if (l15 < 8) {                                 // lane: z[o][16 l15 + 4G + r]
                uintx2 pk;
                pk[0] = pack_bf16x2(acc[0], acc[1]);
                pk[1] = pack_bf16x2(acc[2], acc[3]);
                *reinterpret_cast<uintx2*>(Zi + trimg_off(o, 4 * l15 + G, XROWB)) = pk;
            }
        }
        PH_(5);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");           // z image complete
        PH_(4);

        // ---- 4. pointwise MFMA (A = W3, B = z by transposed reads), BN3, ELU, pool8, classifier ----
        float lp0 = 0.f, lp1 = 0.f;                       // classes pc0, pc0 + 1 of this lane's row prr
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int n = tt0 + 2 * m;
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = mfma_bf16(w3f[0], tr_frag(Zi, XROWB, 0, 16 * n, lane), acc);
            acc = mfma_bf16(w3f[1], tr_frag(Zi, XROWB, 32, 16 * n, lane), acc);
            float e[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] = elu_f(fmaf(s3r[rr], acc[rr], b3r[rr]));
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += __shfl_xor(e[rr], 1, 64);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += __shfl_xor(e[rr], 2, 64);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += __shfl_xor(e[rr], 4, 64);
            const float hv = 0.125f * (prr == 0 ? e[0] : prr == 1 ? e[1] : prr == 2 ? e[2] : e[3]);
            lp0 = fmaf(wfl[m][0], hv, lp0);
            lp1 = fmaf(wfl[m][1], hv, lp1);
        }
        {
            float lp[NCLS];
            lp[0] = pc0 == 0 ? lp0 : 0.f;
            lp[1] = pc0 == 0 ? lp1 : 0.f;
            lp[2] = pc0 == 2 ? lp0 : 0.f;
            lp[3] = pc0 == 2 ? lp1 : 0.f;
            wave_reduce<NCLS>(lp);                        // lane 16 r holds class r in lp[0]
            if ((lane & 15) == 0) Lg[wave * NCLS + (lane >> 4)] = lp[0];
        }
        PH_(6);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");           // partials; z image read
        PH_(4);
        if (tid < NCLS) {
            float a = bfc;
            for (int w = 0; w < NW; ++w) a += Lg[w * NCLS + tid];
            Ls[ls * NCLS + tid] = a;
        }
        // the z image overwrote tail buffer 0, which the next trial's first step may read as s before
        // t = 0: zero it again (the new-s rows' zero-weight positions only need to be finite)
        for (int i = tid; i < TBUF / 16; i += NT)
            *reinterpret_cast<uintx4*>(smr + OFF_T + 16 * i) = (uintx4){0u, 0u, 0u, 0u};
        ++ls;
        if (ls == LGCAP || it == ntr - 1) {               // flush the staged logits (rarely mid-loop: the
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");       // stores join the DMA queue)
            const int i0 = it + 1 - ls;
            for (int i = tid; i < ls * NCLS; i += NT)
                logits[(size_t)(b0 + gs * (i0 + i / NCLS)) * NCLS + (i % NCLS)] = Ls[i];
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");       // Ls read before reuse
            ls = 0;
        }
        PH_(7);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef EEGNET_TRACE
    if (g.dbg && tid == 0)
        for (int k = 0; k < 8; ++k) reinterpret_cast<unsigned long long*>(g.dbg)[blockIdx.x * 8 + k] = ph[k];
#endif
#undef PH_
}

}  // namespace eeg
