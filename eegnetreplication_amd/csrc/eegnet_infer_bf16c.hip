// eegnet_infer_bf16c.hip -- bf16 batched eval forward of BASELINE cfg5 (EEGNet-16,4 on 64ch x 512),
// time-chunked so that two trials are resident per CU.  Included by eegnet_kernels.hip.
//
// Same arithmetic as k_infer_bf16 (eegnet_infer_bf16.hip: BN-folded spatial GEMM, 32-tap FIR, folded
// BN1/BN2 + ELU + pool4, depthwise 1x16, pointwise, BN3 + ELU + pool8, classifier; bf16 operands, fp32
// accumulation; reference: EEGNet.forward in eval mode, src/eegnet_repl/model.py:91-99).  What changes
// is the data flow, for occupancy:
//
// * k_infer_bf16 keeps a whole trial's x image (64 KB) and s rows (72 KB) in LDS, so one 8-wave
//   workgroup fits a CU and every SIMD runs the same phase at the same time.  Here a trial is cut into
//   NCH = 8 time chunks of TC = 64 output samples: a chunk's x image (96 samples incl. the 'same'
//   halo, 16 KB, two buffers) and s rows (12 KB) are all the full-rate data in LDS, and the pooled
//   rows a (bf16, 18 KB) accumulate over the chunks.  74 KB per workgroup: two workgroups (16 waves)
//   per CU, on different trials and out of phase.
// * x arrives by LDS-DMA (global_load_lds_dwordx4) straight into the swizzled transposed-read image
//   -- the swizzle is applied to the per-lane SOURCE address, the 16-byte units of a wave land
//   contiguously -- one chunk ahead, with no prefetch registers (<= 128 VGPRs for 4 waves / SIMD).
// * Round 5: ONE workgroup barrier per chunk.  The s rows are double-buffered, so chunk j's spatial
//   GEMM and chunk j - 1's FIR run in the same barrier interval (19 -> 12 barriers per trial); the
//   LDS for the second s buffer comes from the x images' unused quarter (rows of 192 bytes, the 96
//   samples of a chunk, instead of 256) and from the w1 table (the FIR taps are read from global
//   memory once, into registers).
// * FIR on the matrix cores with a full MFMA per chunk: the 16 columns are (row r of a temporal
//   group, 16-sample tile) -- the D = 4 rows of a group share the banded Toeplitz A operand of the
//   group's taps -- so a 64-sample chunk still fills all 16 columns.
// * depthwise 1x16 on the matrix cores too (banded Toeplitz of the row's 16 taps, K = 32 window;
//   8 of 16 columns used), instead of 131 K VALU FMAs per trial.
// EEGNET_KX = n (timing builds only, wrong results; tools/infer_probe.sh): 1 no spatial GEMM, 2 no FIR
// phase, 3 no block-2 tail, 4 no compute (DMA and barriers only), 5 no x DMA
#ifndef EEGNET_KX
#define EEGNET_KX 0
#endif
namespace eeg {
namespace c5 {

constexpr int C = 64, T = 512, F1 = 16, D = 4, F2 = 64, K1 = 32, T1 = 128, T2 = 16, NF = F2 * T2;
constexpr int TC = 64;                       // output samples per chunk: D rows x TC/16 tiles = 16 columns
constexpr int NCH = T / TC;                  // chunks per trial
constexpr int NTS = 6;                       // spatial 16-sample tiles per chunk (64j - 16 .. 64j + 80)
constexpr int XROWB = 192;                   // x image row (bytes): the chunk's 96 samples
constexpr int XIMG = C * XROWB;              // 12 KB per chunk buffer
constexpr int ZROWB = 256;                   // z image row (bytes): 128 pooled samples (block-2 tail)
constexpr int SROW = 120;                    // s row stride (bf16): 112 read, 60 dwords = 4 mod 8
constexpr int AROW = 144;                    // a row (bf16): [8 zeros | 128 pooled | 8 zeros]
constexpr int W2R = 48;                      // depthwise taps, bf16, [16 zeros | 16 taps | 16 zeros]
constexpr int NT = 512;                      // threads: 8 waves
constexpr int NW = NT / 64;
// LDS carve (bytes): x images 0 / 1, s rows 0 / 1 (the z image of the tail over both), a rows, tables
constexpr int SIMG = F2 * SROW * 2;
constexpr int OFF_X0 = 0, OFF_X1 = XIMG, OFF_S = 2 * XIMG;
constexpr int OFF_A = OFF_S + 2 * SIMG;
constexpr int OFF_W2 = OFF_A + F2 * AROW * 2;
constexpr int OFF_CO = OFF_W2 + F2 * W2R * 2;
constexpr int OFF_LG = OFF_CO + 4 * F2 * 4;
constexpr int LDS = OFF_LG + NW * NCLS * 4;
static_assert(LDS <= 80 * 1024, "two workgroups per CU");
static_assert(F2 * ZROWB <= 2 * SIMG, "the z image fits over the two s buffers");
static_assert(F2 % 16 == 0 && 16 % D == 0 && TC == 16 * (16 / D), "FIR columns = rows of a group x tiles");

}  // namespace c5

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4] = {0u, 0u, 0u, 0u};   // DMA source of the pads

// LDS-DMA of one 16-byte unit per lane (wave-instruction: 64 units, 1 KiB contiguous at ldst), from
// inline asm so the compiler's waitcnt pass does not treat it as an LDS write (eegnet_stream.hip dma16)
__device__ __forceinline__ void dma16c(const void* gsrc, const void* ldst) {
    const unsigned la = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)ldst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(gsrc), "s"(la) : "memory", "m0");
}

// chunk j of trial xb (bf16 [C][T]) into an x image: samples 64j - 16 .. 64j + 79 of every channel row,
// 16-byte units u = 0..11 of the row.  Row r of the image is 192 bytes at 192 r; its 32-byte groups are
// swizzled g -> g ^ sig(r), sig(r) = bit 3 of r (x_img_off), so physical unit u' holds unit u' ^ 2 sig(r).
// One wave-instruction writes 4 rows (48 lanes x 16 bytes, contiguous); units outside the trial read
// zeros ('same' padding).  Each wave issues 2 wave-instructions.
__device__ __forceinline__ void x_chunk_dma(const uint16_t* __restrict__ xb, int j, char* img, int wave, int lane) {
    using namespace c5;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int r0 = 4 * (wave + NW * i);
        const int rr = lane / 12, up = lane - 12 * rr;
        const int r = r0 + rr;
        const int u = up ^ (2 * ((r >> 3) & 1));
        if (lane < 48) {
            const int s0 = TC * j - 16 + 8 * u;
            const void* src = (s0 >= 0 && s0 < T) ? (const void*)(xb + (size_t)r * T + s0) : (const void*)g_zero16;
            dma16c(src, img + r0 * XROWB);
        }
    }
}

// byte offset of 8-byte chunk `ch` of row r in the x image.  A ds_read_b64_tr_b16 half-wave reads
// rows k0 + q and k0 + 8 + q (q = 0..3), 32 bytes each: 192-byte rows put row q's bytes at bank
// offset 48 q mod 64 dwords (0, 48, 32, 16), and the group swizzle moves rows 8..11 by one 32-byte
// group (8 dwords): the 8 rows cover the 64 banks once
__device__ __forceinline__ int x_img_off(int r, int ch) {
    return r * c5::XROWB + 8 * (ch ^ (4 * ((r >> 3) & 1)));
}
__device__ __forceinline__ bf16x8 tr_frag_x(const char* img, int k0, int n0, int lane) {
    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r = k0 + 8 * G + q;
    const int ch = (n0 >> 2) + p;
    const shortx4 lo = lds_tr16(img + x_img_off(r, ch));
    const shortx4 hi = lds_tr16(img + x_img_off(r + 4, ch));
    const shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

template <int N>
__device__ __forceinline__ void barrier_vm_c() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(N) : "memory");
}
__device__ __forceinline__ void barrier_lds_c() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// __launch_bounds__ second argument: minimum waves per SIMD (4: two 8-wave workgroups per CU, <= 128 VGPRs)
__global__ __launch_bounds__(c5::NT, 4) void k_infer_bf16_cfg5(GeoI g, const float* __restrict__ prm,
                                                               const float* __restrict__ bn,
                                                               const uint16_t* __restrict__ x,
                                                               float* __restrict__ logits) {
    using namespace c5;
    extern __shared__ __attribute__((aligned(16))) char smc[];
    char* const Ai = smc + OFF_A;                       // pooled rows a (bf16), whole trial
    char* const Zi = smc + OFF_S;                       // z image (bf16, swizzled, 256-byte rows): over the
                                                        // two s buffers, between trials
    uint16_t* const W2p = reinterpret_cast<uint16_t*>(smc + OFF_W2);
    float* const Co = reinterpret_cast<float*>(smc + OFF_CO);   // [4][F2]: al, be, s3, b3
    float* const Lg = reinterpret_cast<float*>(smc + OFF_LG);   // [NW][4] logit partials
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = lane >> 4, l15 = lane & 15;
    const int B = g.B;

    // ---- prologue: the first trial's chunk 0 DMA first (the tables below overlap it), then tables
    // and zero pads ----
    int b = blockIdx.x;
    if (b < B) x_chunk_dma(x + (size_t)b * C * T, 0, smc + OFF_X0, wave, lane);
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
    {
        constexpr int NW2 = (F2 * W2R + NT - 1) / NT;
        float w2v[NW2];
#pragma unroll
        for (int u = 0; u < NW2; ++u) {
            const int i = min(tid + NT * u, F2 * W2R - 1), o = i / W2R, k = i - o * W2R - 16;
            w2v[u] = prm[g.o_w2 + o * K2 + min(max(k, 0), K2 - 1)];
        }
#pragma unroll
        for (int u = 0; u < NW2; ++u) {
            const int i = tid + NT * u, o = i / W2R, k = i - o * W2R - 16;
            if (i < F2 * W2R) W2p[i] = __builtin_bit_cast(uint16_t, (__bf16)((k >= 0 && k < K2) ? w2v[u] : 0.f));
        }
    }
    // s rows: positions 96..111 meet only zero taps but must be finite (re-zeroed after every trial's
    // tail, whose z image lies over them); a rows: 'same' pads of the dw16
    for (int i = tid; i < 2 * F2 * SROW / 2; i += NT) reinterpret_cast<uint32_t*>(smc + OFF_S)[i] = 0u;
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
    // FIR: this wave's two temporal groups gi = 2 wave + {0, 1}; banded Toeplitz A operand of each
    // group's taps, A[i][j] = w1[g][j - i - 1] over K = 64 (two K-steps), held for the whole kernel;
    // this lane's FIR column is (row r = l15 >> 2 of the group, tile l15 & 3)
    // (unconditional loads at clamped taps, masked after: a guarded load is a branch and a full wait
    // each -- 32 serialised L2 round trips per workgroup)
    bf16x8 af[2][2];
    {
        float wv[2][2][8];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const int k = 32 * s + 8 * G + jj - l15 - 1;
                    wv[q][s][jj] = prm[g.o_w1 + (2 * wave + q) * K1 + min(max(k, 0), K1 - 1)];
                }
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const int k = 32 * s + 8 * G + jj - l15 - 1;
                    af[q][s][jj] = (__bf16)((k >= 0 && k < K1) ? wv[q][s][jj] : 0.f);
                }
    }
    __syncthreads();                                   // tables (not the DMA: asm, waited per chunk)
    float al2[2], be2[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int o = D * (2 * wave + q) + (l15 >> 2);
        al2[q] = Co[o] * 1.4426950408889634f;              // ELU in log2 units (k_infer_bf16)
        be2[q] = Co[F2 + o] * 1.4426950408889634f;
    }
    // classifier weights this lane multiplies: after pool8 every lane of an 8-lane group holds the
    // group's 4 pooled values (rows rr); lane p = l15 & 7 takes row rr = p >> 1 and classes 2 (p & 1),
    // 2 (p & 1) + 1, for each of its wave's 4 pointwise tiles (8 weights).  Loaded per trial at the
    // tail, like the BN3 constants: registers held across the chunk loop serialised its phases
    const int prr = (l15 & 7) >> 1, pc0 = 2 * (l15 & 1);
#ifdef EEGNET_TRACE
    // traced build (tools/trace_bf16.py): thread 0's shader cycles per phase, summed over the trials
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_ = clock64();
#define PH_(k) do { if (g.dbg && tid == 0) { const unsigned long long t1_ = clock64(); ph[k] += t1_ - t_; t_ = t1_; } } while (0)
#else
#define PH_(k) do {} while (0)
#endif

    // FIR (banded Toeplitz MFMA), folded BN, ELU, pool4 of chunk jf from s buffer Sf -> a rows
    // (reads, then MFMAs: issuing the reads before the spatial GEMM's stores instead spilled 10 VGPRs)
    constexpr int NQ = (EEGNET_KX == 2 || EEGNET_KX == 4) ? 0 : 2;
    bf16x8 fw[2][2];
    auto fir_load = [&](const char* Sf) {                  // both groups' s windows
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int o = D * (2 * wave + q) + (l15 >> 2), tile = l15 & 3;
            const char* srw = Sf + o * (2 * SROW) + 2 * (16 * tile + 8 * G);
            fw[q][0] = *reinterpret_cast<const bf16x8*>(srw);
            fw[q][1] = *reinterpret_cast<const bf16x8*>(srw + 64);
        }
    };
    auto fir_chunk = [&](int jf) {
        floatx4 facc[2];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
            facc[q] = mfma_bf16(af[q][0], fw[q][0], z4);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) facc[q] = mfma_bf16(af[q][1], fw[q][1], facc[q]);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int gg = 2 * wave + q;
            const int o = D * gg + (l15 >> 2), tile = l15 & 3;
            const floatx4 acc = facc[q];
            // lane: v[o][t = 64 jf + 16 tile + 4G + r]; pooled sample 16 jf + 4 tile + G
            float pp = 0.f, pn = 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float y = fmaf(al2[q], acc[r], be2[q]);
                pp += fmaxf(y, 0.f);
                pn += __builtin_amdgcn_exp2f(fminf(y, 0.f));
            }
            const float a = fmaf(0.25f * 0.6931471805599453f, pp, 0.25f * pn - 1.f);
            reinterpret_cast<__bf16*>(Ai)[o * AROW + 8 + 16 * jf + 4 * tile + G] = (__bf16)a;
        }
    };

    for (; b < B; b += gridDim.x) {
        const bool more = b + (int)gridDim.x < B;
        const uint16_t* xn = x + (size_t)(b + gridDim.x) * C * T;
        // Per chunk j, ONE barrier: x chunk j landed (its DMA, issued at the top of chunk j - 1, is
        // the only one in flight), s buffer j & 1 free (chunk j - 2's FIR finished before the previous
        // barrier), s buffer (j - 1) & 1 complete (chunk j - 1's spatial GEMM, idem), x buffer
        // (j + 1) & 1 free (read by chunk j - 1's spatial GEMM).  Then: the next chunk's DMA, this
        // chunk's spatial GEMM and the previous chunk's FIR.
#pragma unroll 1
        for (int j = 0; j < NCH; ++j) {
            char* const Xi = smc + ((j & 1) ? OFF_X1 : OFF_X0);
            char* const Si = smc + OFF_S + (j & 1) * SIMG;
            barrier_vm_c<0>();
            PH_(0);
            if (EEGNET_KX == 5) {
            } else if (j + 1 < NCH) x_chunk_dma(x + (size_t)b * C * T, j + 1, smc + (((j + 1) & 1) ? OFF_X1 : OFF_X0), wave, lane);
            else if (more) x_chunk_dma(xn, 0, smc + OFF_X0, wave, lane);      // next trial's chunk 0
            // ---- spatial GEMM s^T[t][o] (16 t x 16 o tiles, A = x^T by transposed reads): every
            // tile's transposed reads first, then the MFMAs, then the stores (one tile at a time, the
            // compiler reused the fragment registers and serialised read -> MFMA -> store per tile) ----
            constexpr int NSP = (EEGNET_KX == 1 || EEGNET_KX == 4) ? 0 : 3;
            bf16x8 sa[3][2];
#pragma unroll
            for (int m = 0; m < NSP; ++m) {
                sa[m][0] = tr_frag_x(Xi, 0, 16 * (tt0 + 2 * m), lane);
                sa[m][1] = tr_frag_x(Xi, 32, 16 * (tt0 + 2 * m), lane);
            }
            floatx4 sacc[3];
#pragma unroll
            for (int m = 0; m < NSP; ++m) {
                const floatx4 z4 = {0.f, 0.f, 0.f, 0.f};
                sacc[m] = mfma_bf16(sa[m][0], wsf[0], z4);
            }
#pragma unroll
            for (int m = 0; m < NSP; ++m) sacc[m] = mfma_bf16(sa[m][1], wsf[1], sacc[m]);
#pragma unroll
            for (int m = 0; m < NSP; ++m) {
                uintx2 pk;
                pk[0] = pack_bf16x2(sacc[m][0], sacc[m][1]);
                pk[1] = pack_bf16x2(sacc[m][2], sacc[m][3]);
                *reinterpret_cast<uintx2*>(Si + (ot * 16 + l15) * (2 * SROW) + 2 * (16 * (tt0 + 2 * m) + 4 * G)) = pk;
            }
            PH_(1);
            if (j > 0) {                                   // the previous chunk's FIR
                fir_load(smc + OFF_S + ((j - 1) & 1) * SIMG);
                fir_chunk(j - 1);
            }
            PH_(3);
        }
        barrier_lds_c();                                   // chunk 7's s rows complete
        PH_(2);
        fir_load(smc + OFF_S + ((NCH - 1) & 1) * SIMG);
        fir_chunk(NCH - 1);
        PH_(3);
        barrier_lds_c();                                   // a rows complete; the s buffers are free
        PH_(4);

        // the tail's per-lane constants (L2-resident classifier weights, BN3 constants from LDS): issued
        // here, used after the depthwise
        float wfl[4][2];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int f = (ot * 16 + 4 * G + prr) * T2 + 2 * (tt0 + 2 * m) + (l15 >> 3);
            wfl[m][0] = prm[g.o_Wfc + pc0 * NF + f];
            wfl[m][1] = prm[g.o_Wfc + (pc0 + 1) * NF + f];
        }
        // ---- depthwise 1x16 (pad 7 | 8) on the matrix cores -> z image (over the s buffers) ----
        // z[o][16n + i] = sum_j A[i][j] W_n[j], A[i][j] = w2[o][j - i - 1], W_n[j] = a[o][16n + j - 8]
#pragma unroll 4
        for (int rr = 0; rr < ((EEGNET_KX == 3 || EEGNET_KX == 4) ? 0 : F2 / NW); ++rr) {
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
                *reinterpret_cast<uintx2*>(Zi + trimg_off(o, 4 * l15 + G, ZROWB)) = pk;
            }
        }
        PH_(5);
        barrier_lds_c();
        PH_(4);

        // ---- pointwise MFMA (A = W3, B = z by transposed reads), BN3, ELU, pool8, classifier ----
        float s3r[4], b3r[4];                              // this lane's 4 output rows j = ot*16 + 4G + rr
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            s3r[rr] = Co[2 * F2 + ot * 16 + 4 * G + rr];
            b3r[rr] = Co[3 * F2 + ot * 16 + 4 * G + rr];
        }
        float lp0 = 0.f, lp1 = 0.f;                       // classes pc0, pc0 + 1 of this lane's row prr
#pragma unroll
        for (int m = 0; m < ((EEGNET_KX == 3 || EEGNET_KX == 4) ? 0 : 4); ++m) {
            const int n = tt0 + 2 * m;
            floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = mfma_bf16(w3f[0], tr_frag(Zi, ZROWB, 0, 16 * n, lane), acc);
            acc = mfma_bf16(w3f[1], tr_frag(Zi, ZROWB, 32, 16 * n, lane), acc);
            // lane: r[j = ot*16 + 4G + rr][q = 16n + l15]; pool8 over the 8 lanes of q (every lane of
            // the group ends with the sums).  DPP within each 8-lane group: quad_perm [1,0,3,2],
            // [2,3,0,1], then row_half_mirror adds the other quad (__shfl_xor compiled to three
            // dependent ds_bpermute round trips per row)
            float e[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] = elu_f(fmaf(s3r[rr], acc[rr], b3r[rr]));
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += dpp<0xB1>(e[rr]);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += dpp<0x4E>(e[rr]);
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) e[rr] += dpp<0x141>(e[rr]);
            const float hv = 0.125f * (prr == 0 ? e[0] : prr == 1 ? e[1] : prr == 2 ? e[2] : e[3]);
            lp0 = fmaf(wfl[m][0], hv, lp0);
            lp1 = fmaf(wfl[m][1], hv, lp1);
        }
        {   // per class: the lanes holding it (p & 1 selects the class pair) summed over the wave
            float lp[NCLS];
            lp[0] = pc0 == 0 ? lp0 : 0.f;
            lp[1] = pc0 == 0 ? lp1 : 0.f;
            lp[2] = pc0 == 2 ? lp0 : 0.f;
            lp[3] = pc0 == 2 ? lp1 : 0.f;
            wave_reduce<NCLS>(lp);                        // lane 16 r holds class r in lp[0]
            if ((lane & 15) == 0) Lg[wave * NCLS + (lane >> 4)] = lp[0];
        }
        PH_(6);
        barrier_lds_c();                                   // logit partials complete; z image consumed
        PH_(4);
        // the z image lay over both s buffers: re-zero each s row's positions 96..111 (bytes 192..223,
        // read by the FIR with zero taps only), so a non-finite z of this trial cannot reach the next
        // trial's FIR as 0 * Inf (trials are independent in the reference).  One 8-byte store per
        // thread: 2 buffers x 64 rows x 4; ordered before the next trial's FIR by its chunk barriers.
        static_assert(2 * F2 * 4 == NT, "one 8-byte pad store per thread");
        {
            const int row = tid >> 2, part = tid & 3;     // row 0..127 over both buffers
            *reinterpret_cast<uintx2*>(smc + OFF_S + row * (2 * SROW) + 192 + 8 * part) = uintx2{0u, 0u};
        }
        if (tid < NCLS) {
            float a = prm[g.o_bfc + tid];
            for (int w = 0; w < NW; ++w) a += Lg[w * NCLS + tid];
            logits[(size_t)b * NCLS + tid] = a;
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
