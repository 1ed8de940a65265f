// eegnet_wide.hip -- the EEGNet train step and fp32 eval forward for F2 = F1*D > 16 (BASELINE cfg5:
// EEGNet-16,4 on 64ch x 512 high-density EEG; reference model.py:13,21-84 with F1=16, D=4).
// Included by eegnet_kernels.hip (one translation unit).
//
// Same restructured algorithm as the F2 <= 16 passes (eegnet_stream.hip), re-laid out
// for planes that no longer fit one workgroup's LDS next to the trial's x (64 x 512 fp32 = 128 KB):
//
//  * streaming passes (A, B, E: full-rate data) work on o-CHUNKS of 16 rows.  A workgroup owns one
//    chunk j for a contiguous trial range, one row per wave (16 waves); the spatial GEMM's x operand
//    is read from global memory (the NOC workgroups of one trial range share an XCD, so x comes
//    from that XCD's L2 after the first of them), so LDS holds only the chunk's s / dy rows.
//    Pass A also forms the lag-Gram of a 1/NOC slice of the electrodes, so every trial's Gram is
//    built once in total.  Per-row partial sums stay in registers, as in the narrow passes.
//  * block-2-rate passes (B2, C, D: [F2, T/4] planes) work on whole trials, 8 waves per workgroup;
//    the F2 x F2 pointwise mix, its weight gradient and its input gradient run on
//    v_mfma_f32_16x16x4_f32 (exact fp32 fmaf chains, as the spatial GEMM).
//  * every reducing pass ends in the same ticketed fp64 grid reduction and finalize (fin1..fin5).
//
//   A   x -> Gram slice, s chunk -> v -> sum v, v^2                      fin1 (BN1, BN2 constants)
//   B   x -> s chunk -> v -> BN2 -> ELU -> pool4 -> dropout -> d2, E1, E2   (no reduction)
//   B2  d2 -> dw16 -> pw (MFMA) -> sum r, r^2                            fin2 (BN3 constants)
//   C   d2 -> block2 -> BN3 -> ELU -> pool8 -> dropout -> FC [-> CE, dFC, BN3-bwd sums]   fin3
//   D   d2 -> block2 bwd: dW3, dq (MFMA), dw2, dd2 -> dp2, BN2-bwd sums  fin4
//   E   x -> s chunk, v, dy2 -> Q correlation, FIR^T -> dws GEMM (MFMA)  fin5 (+ Adam)
//   eval: one fused kernel per trial (chunks of s / v, then block 2 and the head)

namespace eeg {

constexpr int NTW = 1024;              // threads of the wide streaming passes and the wide eval
constexpr int NWW = NTW / 64;          // = 16 rows of an o-chunk, one per wave
constexpr int NTB2 = 512;              // threads of the wide block-2 passes (8 waves)
constexpr int NWB2 = NTB2 / 64;
constexpr int LQW = 8;                 // left pad of block-2 rows (dw16 reads t-7, its transpose t+7)
constexpr int KSW = 16;                // spatial GEMM k-steps: C <= 64
constexpr int MAXNOC = 4;              // o-chunks: F2 <= 64
constexpr int MAXKS3 = 16;             // pointwise k-steps: F2P <= 64
constexpr int MAXNFW = 4;              // head features per thread of a block-2 pass: NF <= 4 * 512

// block-2 row stride (floats): [LQW zeros | T1P | >= 8 zeros], = 16 mod 64 so the 4 rows of one
// MFMA B-fragment read (lk = 0..3, 16 consecutive t each) fall on 4 disjoint 16-bank groups
__host__ __device__ constexpr int rb_stride(int T1) {
    const int t1p = (T1 + 15) & ~15;
    int r = LQW + t1p + 8;
    while (r % 64 != 16) r += 4;
    return r;
}

// workgroup -> (o-chunk j, trial range [b0, b1)).  When the grid allows, the NOC chunk workgroups
// of one trial range get blockIdx values equal mod 8 -- the same XCD -- so they share its L2 for x.
__device__ __forceinline__ void wide_unit(const Geo& g, int& j, int& b0, int& b1, int& r) {
    const int G = gridDim.x, bi = blockIdx.x, NOC = g.NOC;
    const int nr = G / NOC;
    if (G % (8 * NOC) == 0) {
        const int xcd = bi & 7, slot = bi >> 3;
        j = slot % NOC;
        r = (slot / NOC) * 8 + xcd;
    } else {
        j = bi % NOC;
        r = bi / NOC;
    }
    b0 = (int)((long long)r * g.B / nr);
    b1 = (int)((long long)(r + 1) * g.B / nr);
}
__device__ __forceinline__ void wide_unit(const Geo& g, int& j, int& b0, int& b1) {
    int r;
    wide_unit(g, j, b0, b1, r);
}

// s[i][t] = sum_c ws[o0 + i][c] x[c][t] for the 16 rows of one chunk (v_mfma_f32_16x16x4_f32).
// A = ws fragments from an LDS table awl[KSW][64] (lane l of k-step s: ws[o0 + (l & 15)][4s + (l >> 4)],
// zero outside), B = x from global memory (unconditional loads at clamped addresses, masked to
// zero).  Tiles n = wave, wave + NWW, ...; rows land in S at [i * RS + LP + t] (t < 16 NT16 <= RS - LP).
__device__ __forceinline__ void spatial_chunk(const float* __restrict__ xb, const float* awl, float* Ss,
                                              int C, int T, int NT16, int RS, int LP, int wave, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    const int ks = (C + 3) >> 2;
    for (int n = wave; n < NT16; n += NWW) {
        const int t = 16 * n + li;
        const bool ton = t < T;
        const int tc = ton ? t : T - 1;
        // all KSW loads unconditional (clamped rows, lane-dependent masks only): a k-step guard
        // (s < ks, wave-uniform) turns every load into a branch plus a full vmcnt wait
        float bv[KSW];
#pragma unroll
        for (int s = 0; s < KSW; ++s) {
            const int c = 4 * s + lk;
            const float v = xb[(size_t)(c < C ? c : C - 1) * T + tc];
            bv[s] = (c < C && ton) ? v : 0.f;
        }
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KSW; ++s)
            if (s < ks) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(awl[64 * s + lane], bv[s], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) Ss[(4 * lk + r) * RS + LP + t] = acc[r];
    }
}

// The cfg5 geometry (C = 64, T = 512: NT16 = 32 tiles, two per wave, all 16 k-steps in range): the
// B operands of tile m of this wave for trial xb (k_wpass_a loads the first tile's a trial ahead), and
// the tile's GEMM into the s rows
constexpr int SPT = 2;                 // spatial tiles per wave at cfg5
__device__ __forceinline__ void spatial_load5(const float* __restrict__ xb, float (&bv)[KSW], int m, int wave, int lane) {
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < KSW; ++s) bv[s] = xb[(size_t)(4 * s + lk) * 512 + 16 * (wave + NWW * m) + li];
}
// k-steps [s0, s1) of tile m's B operands only
__device__ __forceinline__ void spatial_load5r(const float* __restrict__ xb, float (&bv)[KSW], int m, int wave, int lane,
                                               int s0, int s1) {
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < KSW; ++s)
        if (s >= s0 && s < s1) bv[s] = xb[(size_t)(4 * s + lk) * 512 + 16 * (wave + NWW * m) + li];
}
__device__ __forceinline__ void spatial_mfma5(const float (&bv)[KSW], const float* awl, float* Ss, int RS, int LP, int m,
                                              int wave, int lane) {
    const int li = lane & 15, lk = lane >> 4;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSW; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(awl[64 * s + lane], bv[s], acc, 0, 0, 0);
    const int t = 16 * (wave + NWW * m) + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) Ss[(4 * lk + r) * RS + LP + t] = acc[r];
}

// the ws fragment table of chunk rows [o0, o0 + 16) into LDS (KSW * 64 floats)
__device__ __forceinline__ void stage_aw_chunk(const Geo& g, const float* __restrict__ prm, int o0, float* awl,
                                               int tid, int nth) {
    for (int i = tid; i < KSW * 64; i += nth) {
        const int s = i >> 6, l = i & 63, o = o0 + (l & 15), c = 4 * s + (l >> 4);
        awl[i] = (o < g.F2 && c < g.C) ? prm[g.o_ws + o * g.C + c] : 0.f;
    }
}

// x rows [c0, c0 + nc) of one trial into padded LDS rows (data window [LP, LP + T)): LDS-DMA of
// 256-sample pieces when T is a multiple of 256 (no registers; from inline asm, as eegnet_stream.hip's
// dma16, so the compiler does not make the next LDS read of ANY address wait for it: the caller's
// barrier drains it), else a plain copy
__device__ __forceinline__ void stage_slice(const float* __restrict__ xs, int nc, int T, int RS, int LP, float* Xg,
                                            int tid, int wave, int lane) {
    if ((T & 255) == 0) {
        const int np = T >> 8;
        for (int i = wave; i < nc * np; i += NWW) {
            const int c = i / np, p = i - c * np;
            dma16(xs + (size_t)c * T + 256 * p + 4 * lane, Xg + c * RS + LP + 256 * p);
        }
    } else {
        for (int i = tid; i < nc * T; i += NTW) {
            const int c = i / T, t = i - c * T;
            Xg[c * RS + LP + t] = xs[i];
        }
    }
}

// ================================================================================================
// Wide pass A: BN1 / BN2 batch statistics.  Same partial row as k_pass_a:
//   [G0 K1][S0][H nH][Tl nTl][hs R][ts P][Sv F2][Sv2 F2]
// LDS: Gram slice rows [CPC][RS] | s rows [16][RS] | wave partials [NWW][K1 + 3]
// ================================================================================================
template <int K1, bool SPEC = false>
__global__ __launch_bounds__(NTW) void k_wpass_a(Geo gin, const float* __restrict__ prm,
                                                 const float* __restrict__ x, float* __restrict__ sg,
                                                 float* __restrict__ vg, float* __restrict__ part,
                                                 FinArgs fa) {
    TRACE(gin, 0, TR_ENTRY);
    const Geo g = geo_w<SPEC>(gin);
    using G_ = KG<K1>;
    constexpr int LP = G_::LP;
    constexpr int NEI = G_::template nei<NTW>();
    const int C = g.C, T = g.T, F2 = g.F2, RS = g.RS, TQ = (T + 3) >> 2, NT16 = (T + 15) >> 4;
    if (blockIdx.x == 0 && threadIdx.x < (TK_PASSES - 1) * NCNT)
        __hip_atomic_store(fa.cnt + NCNT + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    int j, b0, b1;
    wide_unit(g, j, b0, b1);
    const int o0 = 16 * j;
    const int c0 = j * g.CPC, nc = max(0, min(g.CPC, C - c0));      // this workgroup's Gram slice
    // cfg5: slice and s rows double-buffered over alternate trials (one workgroup barrier per trial,
    // below); 147 KB of LDS
    constexpr int NBUF = SPEC ? 2 : 1;
    float* Xg = sm;
    float* Ss = Xg + NBUF * g.CPC * RS;
    float* red = Ss + NBUF * 16 * RS;
    float* awl = red + NWW * (K1 + 1) + 2 * NWW;        // ws fragments [KSW][64]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < NBUF * (g.CPC + 16) * RS; i += NTW) sm[i] = 0.f;
    stage_aw_chunk(g, prm, o0, awl, tid, NTW);
    const int o = o0 + wave;
    const bool row_on = o < F2;
    float tap[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k)       // wave-uniform: SGPRs (readfirstlane), not K1 VGPRs
        tap[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(prm[g.o_w1 + ((row_on ? o : 0) / g.D) * K1 + k])));
    const int NO = (T + 7) >> 3;
    float svl = 0.f, sv2l = 0.f, s0 = 0.f;
    // lag-Gram of this wave's slice channel on the matrix cores (the Hankel block product of pass E's
    // lag correlation): with t' = 16a + u - P over the window [-P, T - P) of the zero-padded row,
    // Cg[u][w] = sum_a xp[16a+u-P] xp[16a+w-P] accumulated over trials and G0[d] = sum_u Cg[u][u+d]
    constexpr int NWT = (15 + K1 - 1) / 16 + 1;
    floatx4 cg[NWT];
#pragma unroll
    for (int jt = 0; jt < NWT; ++jt) cg[jt] = (floatx4){0.f, 0.f, 0.f, 0.f};
    const int KQ = (NT16 + 3) >> 2;
    const int li = lane & 15, lk = lane >> 4;
    float eacc[NEI];
    int ea[NEI], eb[NEI];
#pragma unroll
    for (int i = 0; i < NEI; ++i) {
        eacc[i] = 0.f;
        int e = tid + NTW * i;
        ea[i] = -1; eb[i] = -1;
        if (e < g.nH) {
            int a = 0;
            while (e >= g.R - a) { e -= g.R - a; ++a; }
            ea[i] = a; eb[i] = a + e;
        } else if ((e -= g.nH) < g.nTl) {
            int u = 0;
            while (e >= g.P - u) { e -= g.P - u; ++u; }
            ea[i] = T - g.P + u; eb[i] = T - g.P + u + e;
        } else if ((e -= g.nTl) < g.R) {
            ea[i] = e;
        } else if ((e -= g.R) < g.P) {
            ea[i] = T - g.P + e;
        } else {
            ea[i] = -2;
        }
    }
    // cfg5: the B operands of this wave's two spatial tiles, loaded at the top of the trial
    float bv5[SPEC ? KSW : 1], bw5[SPEC ? KSW : 1];
    __syncthreads();                                   // zero fill done before the first slice lands
    if (b0 < b1 && nc > 0) stage_slice(x + ((size_t)b0 * C + c0) * T, nc, T, RS, LP, Xg, tid, wave, lane);
    barrier_vm<0>();                                   // the first slice landed (asm DMA: explicit vmcnt)
    constexpr int KPF = KSW / 2;                       // cfg5: tile 0's first KPF k-steps come a trial ahead
    if constexpr (SPEC)
        if (b0 < b1) spatial_load5r(x + (size_t)b0 * C * T, bv5, 0, wave, lane, 0, KPF);
    TRACE(g, 0, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    // the cfg5 geometry: every wave owns a row, whose s and v stores are SV_ST wave-instructions (2 v
    // octet halves + T / 256 s pieces); the closing barrier lets exactly those stay in flight
    constexpr int SV_ST = 2 + 512 / 256;
    // cfg5: the s / v plane stores of trial bd (v octet in vd, s row still in its LDS buffer), issued
    // at the top of the next trial (below)
    float vd[8];
    int bd = -1;
    auto plane_stores = [&](int bb) {
        const float* rowp = sm + 2 * g.CPC * RS + ((bb - b0) & 1) * 16 * RS + wave * RS;
        float* vrow = vg + ((size_t)bb * F2 + o) * (8 * NO);
        st_pol<EEGNET_NT_SV>((floatx4){vd[0], vd[1], vd[2], vd[3]}, reinterpret_cast<floatx4*>(vrow + 8 * lane));
        st_pol<EEGNET_NT_SV>((floatx4){vd[4], vd[5], vd[6], vd[7]}, reinterpret_cast<floatx4*>(vrow + 8 * lane + 4));
        float* srow = sg + ((size_t)bb * F2 + o) * s_pitch(T);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            st_pol<EEGNET_NT_SV>(lds_ld4(rowp + LP + 4 * lane + 256 * q), reinterpret_cast<floatx4*>(srow + 4 * lane + 256 * q));
    };
    for (int b = b0; b < b1; ++b) {
        const int bn = b + 1;
        // cfg5: this trial's buffers.  Per trial: spatial GEMM -> s rows | barrier (s rows complete,
        // this trial's slice landed) | lag-Gram + edges on the slice | next slice's DMA into the other
        // buffer | FIR of the own row -> v, s planes.  The next trial's spatial GEMM writes the other s
        // buffer (last read by this trial's predecessor's FIR, before this trial's barrier) and its
        // slice DMA the other slice buffer (last read by the predecessor's lag-Gram, idem): no closing
        // barrier.
        if constexpr (SPEC) {
            Xg = sm + ((b - b0) & 1) * g.CPC * RS;
            Ss = sm + 2 * g.CPC * RS + ((b - b0) & 1) * 16 * RS;
            spatial_load5r(x + (size_t)b * C * T, bv5, 0, wave, lane, KPF, KSW);
            spatial_load5(x + (size_t)b * C * T, bw5, 1, wave, lane);
            // the previous trial's s / v plane stores go out after this trial's operand loads, so
            // waiting for those loads (vmcnt is in order) does not wait for the stores to drain: at
            // cfg5 the planes are 256 KB per trial and their drain was what the trial's first phase
            // waited for (profiles/r4k_timeline_cfg5.txt; the registers of a trial-ahead operand
            // prefetch now hold the deferred v octet)
            if (bd >= 0) plane_stores(bd);
            spatial_mfma5(bv5, awl, Ss, RS, LP, 0, wave, lane);
            if (bn < b1) spatial_load5r(x + (size_t)bn * C * T, bv5, 0, wave, lane, 0, KPF);
            spatial_mfma5(bw5, awl, Ss, RS, LP, 1, wave, lane);
            TRACE_PH(g, 0, 0, tph_);
            barrier_vm<SV_ST + KPF>();
        } else {
            spatial_chunk(x + (size_t)b * C * T, awl, Ss, C, T, NT16, RS, LP, wave, lane);
        }
        TRACE_PH(g, 0, 1, tph_);
        for (int c = wave; c < nc; c += NWW) {
            const float* xr = Xg + c * RS + G_::OFF + li;        // xp[i - P] = row[OFF + i]
            for (int ks = 0; ks < KQ; ++ks) {
                const int a = 4 * ks + lk;
                const bool on = a < NT16;
                const int ac = on ? a : 0;
                float av = xr[16 * ac];
                av = (on && 16 * ac + li < T) ? av : 0.f;        // window [-P, T - P)
                s0 += av;
#pragma unroll
                for (int jt = 0; jt < NWT; ++jt) {
                    float bv = xr[16 * (ac + jt)];
                    bv = on ? bv : 0.f;
                    cg[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, cg[jt], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < NEI; ++i) {
            if (ea[i] >= 0) {
                const float* xa = Xg + LP + ea[i];
                float acc = 0.f;
                if (eb[i] >= 0) {
                    const float* xb2 = Xg + LP + eb[i];
                    for (int c = 0; c < nc; ++c) acc = fmaf(xa[c * RS], xb2[c * RS], acc);
                } else {
                    for (int c = 0; c < nc; ++c) acc += xa[c * RS];
                }
                eacc[i] += acc;
            }
        }
        TRACE_PH(g, 0, 2, tph_);
        if constexpr (SPEC) {
            if (bn < b1 && nc > 0)
                stage_slice(x + ((size_t)bn * C + c0) * T, nc, T, RS, LP, sm + ((bn - b0) & 1) * g.CPC * RS, tid, wave, lane);
        } else {
            barrier_lds();                                 // s rows complete, slice read for good (LDS
                                                           // only: no stores of this trial are out yet)
            if (bn < b1 && nc > 0) stage_slice(x + ((size_t)bn * C + c0) * T, nc, T, RS, LP, Xg, tid, wave, lane);
        }
        if (row_on) {
            const float* row = Ss + wave * RS;
            // this wave's s row -> the s plane [B][F2][T], its v octets -> the v plane [B][F2][8 NO]
            // (passes B and E read them instead of recomputing the spatial GEMM and the FIR)
            float* vrow = vg + ((size_t)b * F2 + o) * (8 * NO);
            if constexpr (SPEC) {                          // one octet per lane; stored next trial
                float w[4 * G_::NW8];
                lds_window<G_::NW8>(row + 8 * lane, w);
                fir8<K1, G_::OFF>(w, tap, vd);
#pragma unroll
                for (int i = 0; i < 8; ++i) { svl += vd[i]; sv2l = fmaf(vd[i], vd[i], sv2l); }
                bd = b;
            } else
            for (int oc = lane; oc < NO; oc += 64) {
                float w[4 * G_::NW8];
                lds_window<G_::NW8>(row + 8 * oc, w);
                float v[8];
                fir8<K1, G_::OFF>(w, tap, v);
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (8 * oc + i < T) { svl += v[i]; sv2l = fmaf(v[i], v[i], sv2l); }
                st_pol<EEGNET_NT_SV>((floatx4){v[0], v[1], v[2], v[3]}, reinterpret_cast<floatx4*>(vrow + 8 * oc));
                st_pol<EEGNET_NT_SV>((floatx4){v[4], v[5], v[6], v[7]}, reinterpret_cast<floatx4*>(vrow + 8 * oc + 4));
            }
            float* srow = sg + ((size_t)b * F2 + o) * s_pitch(T);
            if constexpr (SPEC) { (void)srow; } else
            if ((T & 3) == 0) {
                for (int t = 4 * lane; t < T; t += 256)
                    st_pol<EEGNET_NT_SV>(lds_ld4(row + LP + t), reinterpret_cast<floatx4*>(srow + t));
            } else {
                for (int t = lane; t < T; t += 64) srow[t] = row[LP + t];
            }
        }
        TRACE_PH(g, 0, 3, tph_);
        // next slice staged, s rows free (the generic geometry: one slice and one s buffer)
        if constexpr (!SPEC) barrier_vm<0>();
    }
    if constexpr (SPEC)
        if (bd >= 0) plane_stores(bd);                    // the last trial's planes
    TRACE_LOOP(g, 0);

    // ---- workgroup reduction -> one partial row (other chunks' Sv / Sv2 entries are zero) ----
    float* row = part + (size_t)blockIdx.x * g.nA;
    float* svw = red + NWW * (K1 + 1);               // [NWW][2]
    // Gram tiles [NWW][16][16 NWT]: over the dead slice / s rows when they fit, else past the tables
    // (eegnet_host.hip sizes ldsWA the same way)
    float* CG = ((g.CPC + 16) * RS >= NWW * 256 * NWT) ? sm : awl + KSW * 64;
    __syncthreads();
#pragma unroll
    for (int jt = 0; jt < NWT; ++jt)
#pragma unroll
        for (int q = 0; q < 4; ++q) CG[wave * 256 * NWT + (4 * lk + q) * (16 * NWT) + 16 * jt + li] = cg[jt][q];
    {
        float rv[4] = {s0, svl, sv2l, 0.f};                   // [s0][sv][sv2][pad]
        wave_reduce<4>(rv);
        if (lane == 0) red[wave * (K1 + 1) + K1] = rv[0];
        if (lane == 16) svw[2 * wave] = rv[0];
        if (lane == 32) svw[2 * wave + 1] = rv[0];
    }
    __syncthreads();
    if (tid < K1) {
        float t = 0.f;
        for (int w = 0; w < NWW; ++w) {
            const float* cw = CG + w * 256 * NWT + tid;
#pragma unroll
            for (int u = 0; u < 16; ++u) t += cw[u * (16 * NWT + 1)];
        }
        pub(row + tid, t);
    } else if (tid == K1) {
        float t = 0.f;
        for (int w = 0; w < NWW; ++w) t += red[w * (K1 + 1) + K1];
        pub(row + K1, t);
    }
#pragma unroll
    for (int i = 0; i < NEI; ++i)
        if (ea[i] != -2 && tid + NTW * i < g.nedge) pub(row + (K1 + 1 + tid + NTW * i), eacc[i]);
    for (int q = tid; q < 2 * F2; q += NTW) {
        const int oo = q < F2 ? q : q - F2, w = oo - o0;
        const float v = (w >= 0 && w < NWW) ? svw[2 * w + (q < F2 ? 0 : 1)] : 0.f;
        pub(row + (K1 + 1 + g.nedge + q), v);
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nA, fa, dsm)) fin1<K1>(g, prm, dsm + 2, dsm + tail_s_doubles(g.nA), fa);
}

// ================================================================================================
// Wide pass B: forward to the pooled block-2 input d2 = dropout(pool4(ELU(BN2(y2)))) and the pooled
// ELU' sums E1 / E2 of the BN2 backward, per o-chunk.  v comes from pass A's v plane (one octet of
// this wave's row per lane, the next trial's loaded a trial ahead): no LDS, no barrier.  No
// reduction (BN3's statistics are pass B2's).
// ================================================================================================
template <int K1, bool SPEC = false>
__global__ __launch_bounds__(NTW) void k_wpass_b(Geo gin, const float* __restrict__ prm, const float* coef,
                                                 const float* __restrict__ vg, const uint8_t* __restrict__ mask2,
                                                 float* __restrict__ d2g, float* __restrict__ E1g,
                                                 float* __restrict__ E2g) {
    const Geo g = geo_w<SPEC>(gin);
    const int T = g.T, F2 = g.F2, T1 = T >> 2;
    const unsigned dk0 = drop_key(g, 0);
    int j, b0, b1;
    wide_unit(g, j, b0, b1);
    const int o0 = 16 * j;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    (void)tid;
    const int o = o0 + wave;
    const bool row_on = o < F2;
    const int oo = row_on ? o : 0;
    const float alh = coef[CF_AL2 * CSTR + oo], beh = coef[CF_BE2 * CSTR + oo];
    const float gah = prm[g.o_g2 + oo], bth = prm[g.o_b2 + oo];
    const int NO = (T + 7) >> 3;
    constexpr int MOW = 4;                                 // octets per lane: T <= 2048
    const int nmo = (NO + 63) >> 6;
    auto vload = [&](int bb, float (&v)[MOW][8]) {
        const float* vrow = vg + ((size_t)bb * F2 + oo) * (8 * NO);
#pragma unroll
        for (int m = 0; m < MOW; ++m) {
            if (m < nmo) {
                const int oc = min(lane + 64 * m, NO - 1);
                const floatx4 a = *reinterpret_cast<const floatx4*>(vrow + 8 * oc);
                const floatx4 c = *reinterpret_cast<const floatx4*>(vrow + 8 * oc + 4);
                v[m][0] = a[0]; v[m][1] = a[1]; v[m][2] = a[2]; v[m][3] = a[3];
                v[m][4] = c[0]; v[m][5] = c[1]; v[m][6] = c[2]; v[m][7] = c[3];
            }
        }
    };
    float vpf[MOW][8];
    if (b0 < b1) vload(b0, vpf);
    for (int b = b0; b < b1; ++b) {
        float v[MOW][8];
#pragma unroll
        for (int m = 0; m < MOW; ++m)
#pragma unroll
            for (int i = 0; i < 8; ++i) v[m][i] = vpf[m][i];
        if (b + 1 < b1) vload(b + 1, vpf);
        if (row_on) {
            const size_t rb = ((size_t)b * F2 + o) * T1;
#pragma unroll
            for (int m = 0; m < MOW; ++m) {
                const int oc = lane + 64 * m;
                if (m < nmo && oc < NO) {
                    float d2o[2], e1o[2], e2o[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int q = 2 * oc + h;
                        float pe = 0.f, e1 = 0.f, e2 = 0.f;
#pragma unroll
                        for (int i = 4 * h; i < 4 * h + 4; ++i) {
                            const float xh = fmaf(alh, v[m][i], beh);
                            const float z = fmaf(gah, xh, bth);
                            const float dz = elu_d(z);
                            pe += z > 0.f ? z : dz - 1.f;
                            e1 += dz;
                            e2 = fmaf(dz, xh, e2);
                        }
                        d2o[h] = pe * 0.25f * keep_mul(g, mask2, dk0, (unsigned)(rb + q));
                        e1o[h] = e1;
                        e2o[h] = e2;
                    }
                    // the octet's two pooled samples as one 8-byte store per plane (T1 even: both in
                    // range or neither), else one store per sample
                    const int q0 = 2 * oc;
                    if ((T1 & 1) == 0) {
                        if (q0 < T1) {
                            *reinterpret_cast<floatx2*>(d2g + rb + q0) = (floatx2){d2o[0], d2o[1]};
                            *reinterpret_cast<floatx2*>(E1g + rb + q0) = (floatx2){e1o[0], e1o[1]};
                            *reinterpret_cast<floatx2*>(E2g + rb + q0) = (floatx2){e2o[0], e2o[1]};
                        }
                    } else {
#pragma unroll
                        for (int h = 0; h < 2; ++h)
                            if (q0 + h < T1) { d2g[rb + q0 + h] = d2o[h]; E1g[rb + q0 + h] = e1o[h]; E2g[rb + q0 + h] = e2o[h]; }
                    }
                }
            }
        }
    }
}

// ================================================================================================
// Block-2-rate helpers (whole trial per 512-thread workgroup, F2P = 16 * NJT rows, NJT in {2, 4})
// ================================================================================================
// pointwise tile ownership: wave w -> row tile jt = w % NJT, time tiles n = w / NJT + (8 / NJT) i
struct B2Map {
    int jt, n0, dn;
};
__device__ __forceinline__ B2Map b2_map(int NJT, int wave, int nw) {
    B2Map m;
    m.jt = wave % NJT;
    m.n0 = wave / NJT;
    m.dn = nw / NJT;
    return m;
}

// stage trial b's [F2][T1] rows of a global plane into padded LDS rows [F2P][RB] (pads untouched)
__device__ __forceinline__ void b2_stage(const float* __restrict__ src, int F2, int T1, int RB, float* dst,
                                         int tid, int nth) {
    const int n = F2 * T1;
    if ((T1 & 3) == 0) {
        const int TQ1 = T1 >> 2;
        for (int i = tid; i < n / 4; i += nth) {
            const int o = i / TQ1, q = i - o * TQ1;
            const float4 v = reinterpret_cast<const float4*>(src)[i];
            lds_st4(dst + o * RB + LQW + 4 * q, (floatx4){v.x, v.y, v.z, v.w});
        }
    } else {
        for (int i = tid; i < n; i += nth) {
            const int o = i / T1, t = i - o * T1;
            dst[o * RB + LQW + t] = src[i];
        }
    }
}

// cfg5 (F2 = 64, T1 = 128, 512 threads): one trial's [F2][T1] block-2 plane is 4 float4 per thread --
// loaded into registers a trial ahead (b2_pf_load) and stored into the padded LDS rows at the top of
// the trial (b2_pf_store), instead of a synchronous b2_stage whose load latency every trial waited
constexpr int B2PF = 4;
__device__ __forceinline__ void b2_pf_load(const float* __restrict__ src, floatx4 (&v)[B2PF], int tid) {
#pragma unroll
    for (int j = 0; j < B2PF; ++j) v[j] = reinterpret_cast<const floatx4*>(src)[tid + 512 * j];
}
__device__ __forceinline__ void b2_pf_store(const floatx4 (&v)[B2PF], int RB, float* dst, int tid) {
#pragma unroll
    for (int j = 0; j < B2PF; ++j) {
        const int i = tid + 512 * j, o = i >> 5, q = i & 31;     // TQ1 = 32 float4 per row
        lds_st4(dst + o * RB + LQW + 4 * q, v[j]);
    }
}

// the inverse: padded LDS rows [F2P][RB] -> trial b's [F2][T1] rows of a global plane
__device__ __forceinline__ void b2_put(const float* src, int F2, int T1, int RB, float* __restrict__ dst, int tid,
                                       int nth) {
    const int n = F2 * T1;
    if ((T1 & 3) == 0) {
        const int TQ1 = T1 >> 2;
        for (int i = tid; i < n / 4; i += nth) {
            const int o = i / TQ1, q = i - o * TQ1;
            const floatx4 v = lds_ld4(src + o * RB + LQW + 4 * q);
            reinterpret_cast<float4*>(dst)[i] = make_float4(v[0], v[1], v[2], v[3]);
        }
    } else {
        for (int i = tid; i < n; i += nth) {
            const int o = i / T1, t = i - o * T1;
            dst[i] = src[o * RB + LQW + t];
        }
    }
}

// one 16 x 16 MFMA-layout tile (rows 16 jt + 4 (lane >> 4) + r, column 16 n + (lane & 15)) into
// padded LDS rows [F2P][RB]
__device__ __forceinline__ void tile_lds(float* dst, const floatx4& a, int RB, int jt, int n, int lane) {
    float* p = dst + (16 * jt + 4 * (lane >> 4)) * RB + LQW + 16 * n + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[r * RB] = a[r];
}

// q[o][t] = sum_k w2[o][k] d2[o][t + k - 7] (model.py:54-61, 'same', pad 7 | 8) for every row and
// 4-sample quad: windows of 24 floats from the padded rows (start t - 8), taps from an LDS table
__device__ __forceinline__ void b2_dw16(const float* D2, const float* W2s, float* Q, int F2, int T1, int RB,
                                        int tid, int nth) {
    const int TQ1 = (T1 + 3) >> 2;
    for (int it = tid; it < F2 * TQ1; it += nth) {
        const int o = it / TQ1, qd = it - o * TQ1;
        float w[24];
        lds_window<6>(D2 + o * RB + LQW + 4 * qd - 8, w);
        float wt[K2];
        lds_window<4>(W2s + o * K2, wt);
        float out[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < K2; ++k) a = fmaf(wt[k], w[1 + i + k], a);
            out[i] = (4 * qd + i < T1) ? a : 0.f;
        }
        lds_st4(Q + o * RB + LQW + 4 * qd, (floatx4){out[0], out[1], out[2], out[3]});
    }
}

// r[j][t] = sum_i W3[j][i] q[i][t] (model.py:62-69) for one time tile n of row tile jt:
// A = W3 fragments from the LDS table W3s [F2P][F2P + 1] (lane l of k-step s: W3[16 jt + (l & 15)]
// [4 s + (l >> 4)]; the odd row stride keeps the 16 rows of a fragment on distinct banks), B = q
// rows from LDS.
__device__ __forceinline__ floatx4 b2_pw_tile(const float* Q, const float* W3s, int F2P, int jt, int n, int RB,
                                              int lane) {
    const int li = lane & 15, lk = lane >> 4, W3S = F2P + 1;
    const float* qc = Q + lk * RB + LQW + 16 * n + li;
    const float* ar = W3s + (16 * jt + li) * W3S + lk;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < MAXKS3; ++s)
        if (4 * s < F2P) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[4 * s], qc[4 * s * RB], acc, 0, 0, 0);
    return acc;
}

template <int NTT>
__device__ __forceinline__ void b2_pw(const float* Q, const float* W3s, int F2P, int NT1, int RB, const B2Map& mp,
                                      floatx4 (&acc)[NTT], int lane) {
#pragma unroll
    for (int i = 0; i < NTT; ++i) {
        const int n = mp.n0 + mp.dn * i;
        acc[i] = n < NT1 ? b2_pw_tile(Q, W3s, F2P, mp.jt, n, RB, lane) : (floatx4){0.f, 0.f, 0.f, 0.f};
    }
}

// W3 [F2][F2] into the LDS table W3s [F2P][F2P + 1] (zero padding)
__device__ __forceinline__ void stage_w3(const Geo& g, const float* __restrict__ prm, float* W3s, int F2P, int tid,
                                         int nth) {
    const int W3S = F2P + 1;
    for (int i = tid; i < F2P * W3S; i += nth) {
        const int jj = i / W3S, ii = i - jj * W3S;
        W3s[i] = (jj < g.F2 && ii < g.F2) ? prm[g.o_W3 + jj * g.F2 + ii] : 0.f;
    }
}

// w2 taps [F2P][16] (zero rows beyond F2)
__device__ __forceinline__ void load_w2s(const Geo& g, const float* __restrict__ prm, float* W2s, int F2P, int tid,
                                         int nth) {
    for (int i = tid; i < F2P * K2; i += nth) W2s[i] = i < g.F2 * K2 ? prm[g.o_w2 + i] : 0.f;
}

// time tiles per wave of the block-2 MFMA loops: NT1 = ceil(T1 / 16) <= 16 (T <= 1024) over
// 8 / NJT waves per row tile
constexpr int NTTW = 8;

// ================================================================================================
// Wide pass B2: block 2's depthwise and pointwise convolutions -> the q and r planes (read by passes
// C and D) and BN3 (model.py:71) batch statistics.  Partial row [Sr F2][Sr2 F2].
// LDS: D2 [F2P][RB] | Q [F2P][RB] | W2s [F2P][16] | wave sums [NWB2][2][16]
// ================================================================================================
template <int NT, bool SPEC = false>
__global__ __launch_bounds__(NT) void k_wpass_b2(Geo gin, const float* __restrict__ prm,
                                                   const float* __restrict__ d2g, float* __restrict__ q3g,
                                                   float* __restrict__ r3g, float* __restrict__ part, FinArgs fa) {
    const Geo g = geo_w<SPEC>(gin);
    const int F2 = g.F2, F2P = g.F2P, T1 = g.T1, RB = g.RB, NJT = F2P >> 4;
    const int NT1 = (T1 + 15) >> 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2 = sm;
    float* Q = D2 + F2P * RB;
    float* W2s = Q + F2P * RB;
    float* W3s = W2s + F2P * K2;
    // cfg5: each wave's W3 fragments (row tile mp.jt, all 16 k-steps) live in 16 registers instead of
    // an LDS table, so two workgroups fit per CU (make_geo_wide: ldsWB2 without the table, gridW2)
    constexpr bool W3R = SPEC && NT == 512;
    float* ws_ = W3R ? W3s : W3s + F2P * (F2P + 1);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 2 * F2P * RB; i += NT) sm[i] = 0.f;
    load_w2s(g, prm, W2s, F2P, tid, NT);
    const B2Map mp = b2_map(NJT, wave, NT / 64);
    float w3r[W3R ? MAXKS3 : 1];
    if constexpr (W3R) {
        static_assert(!W3R || MAXKS3 * 4 == 64, "cfg5: F2 = F2P = 64");
#pragma unroll
        for (int k = 0; k < MAXKS3; ++k) w3r[k] = prm[g.o_W3 + (16 * mp.jt + li) * F2 + 4 * k + lk];
    } else {
        stage_w3(g, prm, W3s, F2P, tid, NT);
    }
    float sr[4] = {0.f, 0.f, 0.f, 0.f}, sr2[4] = {0.f, 0.f, 0.f, 0.f};
    constexpr bool PF = SPEC && NT == 512;             // cfg5: d2 rows a trial ahead in registers
    floatx4 pd2[PF ? B2PF : 1];
    if constexpr (PF)
        if ((int)blockIdx.x < g.B) b2_pf_load(d2g + (size_t)blockIdx.x * F2 * T1, pd2, tid);
    __syncthreads();
    drain_prologue_loads();
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        if constexpr (PF) {
            b2_pf_store(pd2, RB, D2, tid);
            if (b + (int)gridDim.x < g.B) b2_pf_load(d2g + (size_t)(b + gridDim.x) * F2 * T1, pd2, tid);
        } else {
            b2_stage(d2g + (size_t)b * F2 * T1, F2, T1, RB, D2, tid, NT);
        }
        __syncthreads();
        b2_dw16(D2, W2s, Q, F2, T1, RB, tid, NT);
        __syncthreads();
        const size_t rb = (size_t)b * F2 * T1;
        floatx4 acc[NTTW];
        if constexpr (W3R) {
#pragma unroll
            for (int i = 0; i < NTTW; ++i) {
                const int n = mp.n0 + mp.dn * i;
                floatx4 a = {0.f, 0.f, 0.f, 0.f};
                if (n < NT1) {
                    const float* qc = Q + lk * RB + LQW + 16 * n + li;
#pragma unroll
                    for (int k = 0; k < MAXKS3; ++k) a = __builtin_amdgcn_mfma_f32_16x16x4f32(w3r[k], qc[4 * k * RB], a, 0, 0, 0);
                }
                acc[i] = a;
            }
        } else {
            b2_pw<NTTW>(Q, W3s, F2P, NT1, RB, mp, acc, lane);
        }
#pragma unroll
        for (int i = 0; i < NTTW; ++i) {
            const int n = mp.n0 + mp.dn * i, t = 16 * n + li;
            if (n < NT1) tile_lds(D2, acc[i], RB, mp.jt, n, lane);          // d2 rows are dead
            if (t < T1) {
#pragma unroll
                for (int r = 0; r < 4; ++r) { sr[r] += acc[i][r]; sr2[r] = fmaf(acc[i][r], acc[i][r], sr2[r]); }
            }
        }
        __syncthreads();                                   // r rows complete
        b2_put(Q, F2, T1, RB, q3g + rb, tid, NT);
        b2_put(D2, F2, T1, RB, r3g + rb, tid, NT);
        __syncthreads();                                   // D2 / Q free for the next trial
    }
    // rows 16 jt + 4 lk + r: sums over the 16 lanes li, then over the waves sharing jt
    float v[8] = {sr[0], sr[1], sr[2], sr[3], sr2[0], sr2[1], sr2[2], sr2[3]};
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = row_sum16(v[q]);
    if (li == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ws_[(wave * 2 + 0) * 16 + 4 * lk + r] = v[r];
            ws_[(wave * 2 + 1) * 16 + 4 * lk + r] = v[4 + r];
        }
    }
    __syncthreads();
    float* row = part + (size_t)blockIdx.x * g.nB;
    for (int q = tid; q < 2 * F2; q += NT) {
        const int o = q < F2 ? q : q - F2, h = q < F2 ? 0 : 1, jt = o >> 4;
        float a = 0.f;
        for (int w = jt; w < (NT / 64); w += NJT) a += ws_[(w * 2 + h) * 16 + (o & 15)];
        pub(row + q, a);
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nB, fa, dsm)) fin2(g, dsm + 2, fa);
}

// xh3 = BN3-normalised r (batch statistics of finalize 2) for this wave's rows, in place
__device__ __forceinline__ void b2_bn3(const float* coef, const B2Map& mp, floatx4 (&acc)[NTTW], int lane,
                                       float (&mu)[4], float (&inv)[4]) {
    const int lk = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int jj = 16 * mp.jt + 4 * lk + r;
        mu[r] = coef[CF_MU3 * CSTR + jj];
        inv[r] = coef[CF_INV3 * CSTR + jj];
    }
#pragma unroll
    for (int i = 0; i < NTTW; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][r] = (acc[i][r] - mu[r]) * inv[r];
}

// ================================================================================================
// Wide pass C: head (model.py:71-84) from the r plane of pass B2 (or narrow pass B).  logits, and
// (PC_BWD) CE, classifier grads, BN3-bwd sums.  Partial row [dWfc 4*NF][dbfc 4][Sdz3 F2][Sdz3x F2][loss].
// LDS: H [NF] (features, then their gradients) | class partials [(NT / 64)][4] | sums | XH [F2P][RB]
// ================================================================================================
template <int NT, bool FOLD = false, bool SPEC = false>
__global__ __launch_bounds__(NT, (SPEC && NT == 512) ? 4 : 1) void k_wpass_c(Geo gin, const float* __restrict__ prm, const float* coef,
                                                  const float* __restrict__ r3g, const uint8_t* __restrict__ mask3,
                                                  const float* __restrict__ dlin, const int64_t* __restrict__ labels,
                                                  float* __restrict__ logits, float* __restrict__ dlout,
                                                  float* __restrict__ part, int mode, FinArgs fa, FoldCall fc) {
    const Geo g = geo_w<SPEC>(gin);
    const int F2 = g.F2, F2P = g.F2P, T1 = g.T1, T2 = g.T2, NF = g.NF, RB = g.RB;
    const int NJT = F2P >> 4, NT1 = (T1 + 15) >> 4;
    unsigned dk1;
    const int64_t* perm = nullptr;                     // fold launches: labels through the permutation
    long long row0 = 0;
    if (FOLD) {                                        // fold-indexed launch: this fold's pointers
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
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* H = sm;
    float* lgs = H + ((NF + 3) & ~3);
    float* ws_ = lgs + (NT / 64) * 4;
    float* XH = ws_ + (NT / 64) * 2 * 16;                   // BN3-normalised r [F2P][RB] (t at LQW + t)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const B2Map mp = b2_map(NJT, wave, NT / 64);
    for (int i = tid; i < F2P * RB; i += NT) XH[i] = 0.f;
    float g3[4], b3[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int jj = 16 * mp.jt + 4 * lk + r, jc = jj < F2 ? jj : 0;
        g3[r] = prm[g.o_g3 + jc]; b3[r] = prm[g.o_b3 + jc];
    }
    float wf[NCLS][MAXNFW], wacc[NCLS][MAXNFW];
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < MAXNFW; ++u) {
            const int f = tid + NT * u;
            wf[n][u] = f < NF ? prm[g.o_Wfc + n * NF + f] : 0.f;
            wacc[n][u] = 0.f;
        }
    float bfc[NCLS];
#pragma unroll
    for (int n = 0; n < NCLS; ++n) bfc[n] = prm[g.o_bfc + n];
    float sdz[4] = {0.f, 0.f, 0.f, 0.f}, sdzx[4] = {0.f, 0.f, 0.f, 0.f};
    float bacc[NCLS] = {0.f, 0.f, 0.f, 0.f}, lossacc = 0.f;
    const float invB = 1.0f / (float)g.Bn;
    constexpr bool PF = SPEC && NT == 512;             // cfg5: r rows a trial ahead in registers
    floatx4 pr[PF ? B2PF : 1];
    if constexpr (PF)
        if ((int)blockIdx.x < g.B) b2_pf_load(r3g + (size_t)blockIdx.x * F2 * T1, pr, tid);
    __syncthreads();
    drain_prologue_loads();
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        if constexpr (PF) {                                                  // r rows (pass B2)
            b2_pf_store(pr, RB, XH, tid);
            if (b + (int)gridDim.x < g.B) b2_pf_load(r3g + (size_t)(b + gridDim.x) * F2 * T1, pr, tid);
        } else {
            b2_stage(r3g + (size_t)b * F2 * T1, F2, T1, RB, XH, tid, NT);   // r rows (pass B / B2)
        }
        __syncthreads();
        {
            float mu[4], inv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = 16 * mp.jt + 4 * lk + r;
                mu[r] = coef[CF_MU3 * CSTR + jj];
                inv[r] = coef[CF_INV3 * CSTR + jj];
            }
            // per time tile: BN3 -> XH (in place over r); ELU -> AvgPool(1,8) -> H (flattened index
            // j*T2 + t/8, model.py:75)
            for (int i = 0; i < NTTW; ++i) {
                const int n = mp.n0 + mp.dn * i;
                if (n >= NT1) break;
                const int t = 16 * n + li;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int jj = 16 * mp.jt + 4 * lk + r;
                    const float xh = (XH[jj * RB + LQW + t] - mu[r]) * inv[r];
                    XH[jj * RB + LQW + t] = xh;
                    float e = t < 8 * T2 ? elu_f(fmaf(g3[r], xh, b3[r])) : 0.f;
                    e = sum8_hi(e);
                    if ((lane & 7) == 7 && t < 8 * T2 && jj < F2) H[jj * T2 + (t >> 3)] = e * 0.125f;
                }
            }
        }
        __syncthreads();                                   // H complete
        float hv[MAXNFW], kp[MAXNFW];
        float lg[NCLS] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < MAXNFW; ++u) {
            const int f = tid + NT * u;
            kp[u] = f < NF ? keep_mul(g, mask3, dk1, (unsigned)(b * NF + f)) : 0.f;
            hv[u] = f < NF ? H[f] * kp[u] : 0.f;                       // dropout (model.py:74)
#pragma unroll
            for (int n = 0; n < NCLS; ++n) lg[n] = fmaf(wf[n][u], hv[u], lg[n]);
        }
        wave_reduce<NCLS>(lg);                                         // lane 16n: class n
        if ((lane & 15) == 0) lgs[wave * 4 + (lane >> 4)] = lg[0];
        __syncthreads();
        float L[NCLS];
#pragma unroll
        for (int n = 0; n < NCLS; ++n) {
            float a = 0.f;
            for (int w = 0; w < (NT / 64); ++w) a += lgs[w * 4 + n];
            L[n] = a + bfc[n];
        }
        if ((mode & PC_LOGITS) && tid < NCLS)
            logits[(size_t)b * NCLS + tid] = tid == 0 ? L[0] : tid == 1 ? L[1] : tid == 2 ? L[2] : L[3];
        if (mode & PC_BWD) {
            float dl[NCLS];
            if (mode & PC_CE) {                                        // nn.CrossEntropyLoss, mean
                const float mx = fmaxf(fmaxf(L[0], L[1]), fmaxf(L[2], L[3]));
                float se = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) se += expf(L[n] - mx);
                const float lse = mx + logf(se);
                const int y = (int)labels[fold_row(perm, row0, b)];
                const float Ly = y == 0 ? L[0] : y == 1 ? L[1] : y == 2 ? L[2] : L[3];
                if (tid == 0) lossacc += lse - Ly;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dl[n] = (expf(L[n] - lse) - (n == y ? 1.f : 0.f)) * invB;
                if (tid < NCLS)
                    dlout[(size_t)b * NCLS + tid] = tid == 0 ? dl[0] : tid == 1 ? dl[1] : tid == 2 ? dl[2] : dl[3];
            } else {
#pragma unroll
                for (int n = 0; n < NCLS; ++n) dl[n] = dlin[(size_t)b * NCLS + n];
            }
            if (tid == 0)
#pragma unroll
                for (int n = 0; n < NCLS; ++n) bacc[n] += dl[n];
#pragma unroll
            for (int u = 0; u < MAXNFW; ++u) {
                const int f = tid + NT * u;
                float d = 0.f;
#pragma unroll
                for (int n = 0; n < NCLS; ++n) {
                    wacc[n][u] = fmaf(dl[n], hv[u], wacc[n][u]);
                    d = fmaf(dl[n], wf[n][u], d);
                }
                if (f < NF) H[f] = d * kp[u];                           // dp3 (own slots)
            }
            __syncthreads();
            // BN3-backward sums: dz3 = dp3 / 8 * ELU'(z3) (this wave's own XH entries)
            for (int i = 0; i < NTTW; ++i) {
                const int n = mp.n0 + mp.dn * i;
                if (n >= NT1) break;
                const int t = 16 * n + li;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int jj = 16 * mp.jt + 4 * lk + r;
                    if (t < 8 * T2 && jj < F2) {
                        const float xh = XH[jj * RB + LQW + t];
                        const float dz = H[jj * T2 + (t >> 3)] * 0.125f * elu_d(fmaf(g3[r], xh, b3[r]));
                        sdz[r] += dz;
                        sdzx[r] = fmaf(dz, xh, sdzx[r]);
                    }
                }
            }
        }
        __syncthreads();                                   // H, XH free for the next trial
    }
    if (!(mode & PC_BWD)) return;
    float* row = part + (size_t)blockIdx.x * g.nC;
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < MAXNFW; ++u) {
            const int f = tid + NT * u;
            if (f < NF) pub(row + n * NF + f, wacc[n][u]);
        }
    float v[8] = {sdz[0], sdz[1], sdz[2], sdz[3], sdzx[0], sdzx[1], sdzx[2], sdzx[3]};
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = row_sum16(v[q]);
    if (li == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ws_[(wave * 2 + 0) * 16 + 4 * lk + r] = v[r];
            ws_[(wave * 2 + 1) * 16 + 4 * lk + r] = v[4 + r];
        }
    }
    __syncthreads();
    for (int q = tid; q < 2 * F2; q += NT) {
        const int o = q < F2 ? q : q - F2, h = q < F2 ? 0 : 1, jt = o >> 4;
        float a = 0.f;
        for (int w = jt; w < (NT / 64); w += NJT) a += ws_[(w * 2 + h) * 16 + (o & 15)];
        pub(row + NCLS * NF + NCLS + q, a);
    }
    if (tid == 0) {
#pragma unroll
        for (int n = 0; n < NCLS; ++n) pub(row + NCLS * NF + n, bacc[n]);
        pub(row + NCLS * NF + NCLS + 2 * F2, lossacc);
    }
    double* dsm = (double*)sm;
    if (g.splitC) return;                            // k_coltail reduces and finalizes
    if (grid_reduce(g, part, g.nC, fa, dsm)) fin3(g, prm, dsm + 2, fa);
}

// ================================================================================================
// Wide pass D: block_2 backward from the d2, q and r planes -- dW3 and dq on the matrix cores, dw2,
// dd2 -> dropout -> dp2, and the BN2-backward sums from pass B's pooled ELU' sums.  Partial row
// [dW3 F2*F2][dw2 F2*16][Sdz2 F2][Sdz2x F2].
// LDS: D2 [F2P][RB] | Q [F2P][RB] (q, then dq) | DR [F2P][RB] | W2s | Hd [NF] | item sums
// ================================================================================================
template <int NT, bool FOLD = false, bool SPEC = false>
__global__ __launch_bounds__(NT, 2) void k_wpass_d(Geo gin, const float* __restrict__ prm, const float* coef,
                                                  const float* __restrict__ d2g, const float* __restrict__ E1g,
                                                  const float* __restrict__ E2g, const float* __restrict__ q3g,
                                                  const float* __restrict__ r3g, const uint8_t* __restrict__ mask2,
                                                  const uint8_t* __restrict__ mask3, const float* __restrict__ dl,
                                                  float* __restrict__ dp2g, float* __restrict__ part, FinArgs fa,
                                                  FoldCall fc) {
    const Geo g = geo_w<SPEC>(gin);
    const int F2 = g.F2, F2P = g.F2P, T1 = g.T1, T2 = g.T2, NF = g.NF, RB = g.RB;
    const int NJT = F2P >> 4, KS3 = F2P >> 2, NT1 = (T1 + 15) >> 4, TQ1 = (T1 + 3) >> 2;
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
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* D2 = sm;
    float* Q = D2 + F2P * RB;
    float* DR = Q + F2P * RB;
    float* W2s = DR + F2P * RB;
    float* W3s = W2s + F2P * K2;
    float* Hd = W3s + F2P * (F2P + 1);
    float* IS = Hd + ((NF + 3) & ~3);                  // [2][F2 * TQ1] BN2-bwd item sums (per thread)
    const int nit = F2 * TQ1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 3 * F2P * RB; i += NT) sm[i] = 0.f;
    for (int i = tid; i < 2 * nit; i += NT) IS[i] = 0.f;
    load_w2s(g, prm, W2s, F2P, tid, NT);
    stage_w3(g, prm, W3s, F2P, tid, NT);
    const B2Map mp = b2_map(NJT, wave, NT / 64);
    float g3[4], b3[4], A3[4], B3[4], C3[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int jj = 16 * mp.jt + 4 * lk + r, jc = jj < F2 ? jj : 0;
        g3[r] = prm[g.o_g3 + jc]; b3[r] = prm[g.o_b3 + jc];
        A3[r] = coef[CF_A3 * CSTR + jc]; B3[r] = coef[CF_B3 * CSTR + jc]; C3[r] = coef[CF_C3 * CSTR + jc];
    }
    float wf[NCLS][MAXNFW];
#pragma unroll
    for (int n = 0; n < NCLS; ++n)
#pragma unroll
        for (int u = 0; u < MAXNFW; ++u) {
            const int f = tid + NT * u;
            wf[n][u] = f < NF ? prm[g.o_Wfc + n * NF + f] : 0.f;
        }
    // dW3 tiles of this wave: (jt, it) = q / NJT, q % NJT for q = wave + (NT / 64) m
    constexpr int MW3 = 16 / (NT / 64);                 // dW3 tiles per wave: NJT^2 <= 16
    floatx4 accW[MW3];
#pragma unroll
    for (int m = 0; m < MW3; ++m) accW[m] = (floatx4){0.f, 0.f, 0.f, 0.f};
    // dw2 item of this thread: row o2, taps 4 kq .. 4 kq + 3
    const int o2 = tid >> 2, kq = tid & 3;
    float acc2[4] = {0.f, 0.f, 0.f, 0.f};
    // cfg5 (compile-time F2 = 64, T1 = 128, 512 threads): a trial's d2 / q / r rows are four float4
    // per thread and plane, loaded into registers a whole trial ahead and stored to LDS at the top of
    // the trial; the dd2 phase loads its items' E1 / E2 two items at a time (each of the four items
    // waited one global round trip for them; all four at once, or from the top of the trial, spill)
    constexpr bool PFD = SPEC && NT == 512;
    constexpr int NPD = 4;                             // float4 per thread and plane at cfg5
    floatx4 pd[PFD ? 3 : 1][PFD ? NPD : 1], pe1[PFD ? NPD : 1], pe2[PFD ? NPD : 1];
    auto planes_load = [&](int bb) {
        if constexpr (PFD) {               // (the only caller; keeps the 1 x 1 arrays of !PFD unindexed)
            const floatx4* s0 = reinterpret_cast<const floatx4*>(d2g + (size_t)bb * F2 * T1);
            const floatx4* s1 = reinterpret_cast<const floatx4*>(q3g + (size_t)bb * F2 * T1);
            const floatx4* s2 = reinterpret_cast<const floatx4*>(r3g + (size_t)bb * F2 * T1);
#pragma unroll
            for (int j = 0; j < NPD; ++j) {
                pd[0][j] = s0[tid + NT * j]; pd[1][j] = s1[tid + NT * j]; pd[2][j] = s2[tid + NT * j];
            }
        }
    };
    if constexpr (PFD)
        if ((int)blockIdx.x < g.B) planes_load(blockIdx.x);
    __syncthreads();
    drain_prologue_loads();
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        float dlv[NCLS];
#pragma unroll
        for (int n = 0; n < NCLS; ++n) dlv[n] = dl[(size_t)b * NCLS + n];
        const size_t rb = (size_t)b * F2 * T1;
        if constexpr (PFD) {
            constexpr int TQ1C = 128 / 4;
#pragma unroll
            for (int j = 0; j < NPD; ++j) {
                const int i = tid + NT * j, o = i / TQ1C, qq = i - o * TQ1C;
                lds_st4(D2 + o * RB + LQW + 4 * qq, pd[0][j]);
                lds_st4(Q + o * RB + LQW + 4 * qq, pd[1][j]);
                lds_st4(DR + o * RB + LQW + 4 * qq, pd[2][j]);
            }
            if (b + (int)gridDim.x < g.B) planes_load(b + gridDim.x);   // registers free again
        } else {
            b2_stage(d2g + rb, F2, T1, RB, D2, tid, NT);
            b2_stage(q3g + rb, F2, T1, RB, Q, tid, NT);
            b2_stage(r3g + rb, F2, T1, RB, DR, tid, NT);  // r rows, then dr in place
        }
        // dh -> dropout -> dp3 (flattened) into Hd
#pragma unroll
        for (int u = 0; u < MAXNFW; ++u) {
            const int f = tid + NT * u;
            float d = 0.f;
#pragma unroll
            for (int n = 0; n < NCLS; ++n) d = fmaf(dlv[n], wf[n][u], d);
            if (f < NF) Hd[f] = d * keep_mul(g, mask3, dk1, (unsigned)(b * NF + f));
        }
        __syncthreads();
        {   // BN3 backward (finalize 3's batch constants): dr = A3 dz3 + B3 + C3 xh3 -> DR rows
            float mu[4], inv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = 16 * mp.jt + 4 * lk + r;
                mu[r] = coef[CF_MU3 * CSTR + jj];
                inv[r] = coef[CF_INV3 * CSTR + jj];
            }
            for (int i = 0; i < NTTW; ++i) {
                const int n = mp.n0 + mp.dn * i;
                if (n >= NT1) break;
                const int t = 16 * n + li;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int jj = 16 * mp.jt + 4 * lk + r;
                    const float xh = (DR[jj * RB + LQW + t] - mu[r]) * inv[r];
                    const float dz = (t < 8 * T2 && jj < F2)
                                         ? Hd[jj * T2 + (t >> 3)] * 0.125f * elu_d(fmaf(g3[r], xh, b3[r])) : 0.f;
                    const float d = (t < T1 && jj < F2) ? fmaf(A3[r], dz, fmaf(C3[r], xh, B3[r])) : 0.f;
                    DR[jj * RB + LQW + t] = d;
                }
            }
        }
        __syncthreads();                                   // DR complete
        // dW3[j][i] += sum_t dr[j][t] q[i][t] (float4 k-permuted operands; model.py:62-69 weight grad)
#pragma unroll
        for (int m = 0; m < MW3; ++m) {
            const int q = wave + (NT / 64) * m;
            if (q < NJT * NJT) {
                const int jt = q / NJT, it = q - jt * NJT;
                const float* ar = DR + (16 * jt + li) * RB + LQW + 4 * lk;
                const float* br = Q + (16 * it + li) * RB + LQW + 4 * lk;
                for (int kg = 0; kg < NT1; ++kg) {
                    const floatx4 a4 = lds_ld4(ar + 16 * kg), b4 = lds_ld4(br + 16 * kg);
                    accW[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[0], b4[0], accW[m], 0, 0, 0);
                    accW[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[1], b4[1], accW[m], 0, 0, 0);
                    accW[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[2], b4[2], accW[m], 0, 0, 0);
                    accW[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[3], b4[3], accW[m], 0, 0, 0);
                }
            }
        }
        __syncthreads();                                   // every reader of q is past: dq -> Q
        // dq[i][t] = sum_j W3[j][i] dr[j][t]: A = W3^T fragments (W3s[4 s + lk][16 it + li]), B = DR
        for (int i = 0; i < NTTW; ++i) {
            const int n = mp.n0 + mp.dn * i;
            if (n >= NT1) break;
            const float* dc = DR + lk * RB + LQW + 16 * n + li;
            const float* at = W3s + lk * (F2P + 1) + 16 * mp.jt + li;
            floatx4 dq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < MAXKS3; ++s)
                if (s < KS3)
                    dq = __builtin_amdgcn_mfma_f32_16x16x4f32(at[4 * s * (F2P + 1)], dc[4 * s * RB], dq, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) Q[(16 * mp.jt + 4 * lk + r) * RB + LQW + 16 * n + li] = dq[r];
        }
        __syncthreads();
        // dw2[o][k] += sum_t dq[o][t] d2p[o][t + k - 7]
        if (o2 < F2) {
            const float* dqr = Q + o2 * RB + LQW;
            const float* d2r = D2 + o2 * RB + LQW - 8 + 4 * kq;     // d2p[t + k - 7] = d2r[t + 1 + k - 4 kq]
            for (int tq = 0; tq < TQ1; ++tq) {
                const floatx4 a4 = lds_ld4(dqr + 4 * tq);
                const floatx4 w0 = lds_ld4(d2r + 4 * tq), w1 = lds_ld4(d2r + 4 * tq + 4);
                const float w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int i = 0; i < 4; ++i) acc2[kk] = fmaf(a4[i], w[1 + i + kk], acc2[kk]);
            }
        }
        // dd2[t] = sum_k w2[k] dq[t + 7 - k] -> dropout -> dp2; BN2-backward sums (E1 / E2 of pass B)
        auto dd2_item = [&](int it, const float* e1, const float* e2) {
            const int o = it / TQ1, qd = it - o * TQ1;
            float s1 = 0.f, s2 = 0.f;
            float w[24];
            lds_window<6>(Q + o * RB + LQW + 4 * qd - 8, w);              // dq[t - 8 .. t + 15]
            float wt[K2];
            lds_window<4>(W2s + o * K2, wt);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int t = 4 * qd + i;
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < K2; ++k) a = fmaf(wt[k], w[15 + i - k], a);
                if (t < T1) {
                    const size_t gi = rb + (size_t)o * T1 + t;
                    const float dp = a * keep_mul(g, mask2, dk0, (unsigned)gi);
                    dp2g[gi] = dp;
                    s1 = fmaf(dp * 0.25f, e1 ? e1[i] : E1g[gi], s1);
                    s2 = fmaf(dp * 0.25f, e2 ? e2[i] : E2g[gi], s2);
                }
            }
            IS[it] += s1;                                  // this thread's own slots
            IS[nit + it] += s2;
        };
        if constexpr (PFD) {
#pragma unroll
            for (int h = 0; h < NPD; h += 2) {         // two items' E1 / E2 per round trip
#pragma unroll
                for (int j = h; j < h + 2; ++j) {
                    const int it = tid + NT * j, o = it / (128 / 4), qd = it - o * (128 / 4);
                    pe1[j] = *reinterpret_cast<const floatx4*>(E1g + rb + o * 128 + 4 * qd);
                    pe2[j] = *reinterpret_cast<const floatx4*>(E2g + rb + o * 128 + 4 * qd);
                }
#pragma unroll
                for (int j = h; j < h + 2; ++j) {
                    const float e1[4] = {pe1[j][0], pe1[j][1], pe1[j][2], pe1[j][3]};
                    const float e2[4] = {pe2[j][0], pe2[j][1], pe2[j][2], pe2[j][3]};
                    dd2_item(tid + NT * j, e1, e2);
                }
            }
        } else {
            for (int it = tid; it < nit; it += NT) dd2_item(it, nullptr, nullptr);
        }
        __syncthreads();                                   // D2, Q, DR, Hd free for the next trial
    }
    // ---- workgroup reduction ----
    float* row = part + (size_t)blockIdx.x * g.nD;
#pragma unroll
    for (int m = 0; m < MW3; ++m) {
        const int q = wave + (NT / 64) * m;
        if (q < NJT * NJT) {
            const int jt = q / NJT, it = q - jt * NJT;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = 16 * jt + 4 * lk + r, ii = 16 * it + li;
                if (jj < F2 && ii < F2) pub(row + jj * F2 + ii, accW[m][r]);
            }
        }
    }
    if (o2 < F2) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) pub(row + F2 * F2 + o2 * K2 + 4 * kq + kk, acc2[kk]);
    }
    // item partials -> per-row sums in a fixed order (items of row o are it = o TQ1 + qd)
    for (int q = tid; q < 2 * F2; q += NT) {
        const int o = q < F2 ? q : q - F2, h = q < F2 ? 0 : 1;
        float a = 0.f;
        for (int qd = 0; qd < TQ1; ++qd) a += IS[h * nit + o * TQ1 + qd];
        pub(row + F2 * F2 + 16 * F2 + q, a);
    }
    double* dsm = (double*)sm;
    if (g.splitD) return;                            // k_coltail reduces and finalizes
    if (grid_reduce(g, part, g.nD, fa, dsm)) fin4(g, prm, dsm + 2, fa);
}

// ================================================================================================
// Wide pass E: dy2 and the weight-gradient reductions that need full-rate data, per o-chunk.  s and v
// come from pass A's planes; every wave stages and reads only its own s / dy / dp2 rows until the
// dws GEMM, which reads all e rows of the chunk and x (global memory, L2).
// Partial row [Q F2*K1][Xm F2*C][Sdy F2][Sdyv F2] (other chunks' entries zero).
// LDS: s rows [16][RS] | dy rows, then (in place) e [16][RS], two buffers (alternate trials) | dp2 rows [16][T1] | coefficient table
// [16][8]; after the loop: dws tiles [NWW][256], row sums, lag-correlation tiles [NWW][16][16 NWT]
// Per trial and wave: v (loaded a trial ahead) -> dy2 | next dp2 row (DMA) | lag correlation |
// FIR^T -> e over the dy row | next s row (DMA) | barrier | dws GEMM | own DMAs landed (no barrier)
// ================================================================================================
template <int K1, bool SPEC = false>
__global__ __launch_bounds__(NTW) void k_wpass_e(Geo gin, const float* prm, const float* coef,
                                                 const float* __restrict__ x, const float* __restrict__ sg,
                                                 const float* __restrict__ vg, const float* __restrict__ dp2g,
                                                 float* __restrict__ part, FinArgs fa) {
    TRACE(gin, 4, TR_ENTRY);
    const Geo g = geo_w<SPEC>(gin);
    using G_ = KG<K1>;
    constexpr int LP = G_::LP;
    const int C = g.C, T = g.T, F2 = g.F2, RS = g.RS, T1 = T >> 2, NT16 = (T + 15) >> 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    int j, b0, b1, rr;
    wide_unit(g, j, b0, b1, rr);
    const int o0 = 16 * j, nrows = min(16, F2 - o0);
    float* Ss = sm;
    // dy / e rows, two buffers (alternate trials): the next trial's dy2 phase writes the other one
    // while slower waves still read this trial's e rows in the dws GEMM, so one barrier per trial
    float* const Dys0 = Ss + 16 * RS;
    float* DP = Dys0 + 2 * 16 * RS;
    float* CT = DP + ((16 * T1 + 3) & ~3);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 3 * 16 * RS; i += NTW) sm[i] = 0.f;
    const int o = o0 + wave;
    const bool row_on = wave < nrows;
    const int oo = row_on ? o : 0;
    float tap[K1];
#pragma unroll
    for (int k = 0; k < K1; ++k)       // wave-uniform: SGPRs (readfirstlane), not K1 VGPRs
        tap[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(prm[g.o_w1 + (oo / g.D) * K1 + k])));
    if (tid < 8 * 16) {
        const int r = tid >> 3, f = tid & 7, orr = min(o0 + r, F2 - 1);
        const float* src = f == 0 ? coef + CF_AL2 * CSTR : f == 1 ? coef + CF_BE2 * CSTR
                         : f == 2 ? prm + g.o_g2 : f == 3 ? prm + g.o_b2 : f == 4 ? coef + CF_AO * CSTR
                         : f == 5 ? coef + CF_BO * CSTR : coef + CF_CO * CSTR;
        CT[tid] = src[orr];
    }
    const int NO = (T + 7) >> 3;
    constexpr int MOW = SPEC ? 1 : 2;                      // octets per lane: T <= 1024 (cfg5: 512, one)
    float sdyl = 0.f, sdyvl = 0.f;
    // this wave's row of the dW1 lag correlation on the matrix cores, as in k_pass_e:
    // Cq[u][w] = sum_a dy[16a+u] s'[16a+w] accumulated over the trials, Q[k] = sum_u Cq[u][u+k]
    constexpr int NWT = (15 + K1 - 1) / 16 + 1;
    floatx4 cq[NWT];
#pragma unroll
    for (int jt = 0; jt < NWT; ++jt) cq[jt] = (floatx4){0.f, 0.f, 0.f, 0.f};
    const int KQ = (NT16 + 3) >> 2;
    // dws GEMM split: wave -> (c-tile ct, k-group range)
    const int NCT = (C + 15) >> 4, wpc = NWW / NCT;
    const bool gemm_on = wave < wpc * NCT;
    const int ct = gemm_on ? wave / wpc : 0, pt = gemm_on ? wave - ct * wpc : 0;
    const int kg0 = (NT16 * pt) / wpc, kg1 = gemm_on ? (NT16 * (pt + 1)) / wpc : 0;
    floatx4 xacc = {0.f, 0.f, 0.f, 0.f};
    // this wave's s and dp2 rows of trial bb into LDS: LDS-DMA (inline asm: the caller's barrier_vm
    // drains it) when the rows are whole 1 KiB / 256 B pieces, else synchronous copies
    const bool rdma = (T & 255) == 0;
    auto stage_rows = [&](int bb) {
        if (!row_on) return;
        const float* srow = sg + ((size_t)bb * F2 + o) * s_pitch(T);
        const float* drow = dp2g + ((size_t)bb * F2 + o) * T1;
        if (rdma) {
            for (int p = 0; p < (T >> 8); ++p) dma16(srow + 256 * p + 4 * lane, Ss + wave * RS + LP + 256 * p);
            for (int p = 0; p < (T1 >> 6); ++p) dma4(drow + 64 * p + lane, DP + wave * T1 + 64 * p);
        } else {
            for (int t = lane; t < T; t += 64) Ss[wave * RS + LP + t] = srow[t];
            for (int t = lane; t < T1; t += 64) DP[wave * T1 + t] = drow[t];
        }
    };
    auto vload = [&](int bb, float (&v)[MOW][8]) {
        const float* vrow = vg + ((size_t)bb * F2 + oo) * (8 * NO);
#pragma unroll
        for (int m = 0; m < MOW; ++m) {
            const int oc = min(lane + 64 * m, NO - 1);
            const floatx4 a = *reinterpret_cast<const floatx4*>(vrow + 8 * oc);
            const floatx4 c = *reinterpret_cast<const floatx4*>(vrow + 8 * oc + 4);
            v[m][0] = a[0]; v[m][1] = a[1]; v[m][2] = a[2]; v[m][3] = a[3];
            v[m][4] = c[0]; v[m][5] = c[1]; v[m][6] = c[2]; v[m][7] = c[3];
        }
    };
    float vpf[MOW][8];
    adam_slice(g, fa, blockIdx.x, gridDim.x, adam_step0(g, fa));
    adam_scalars_publish(g, fa);
    __syncthreads();                                       // zero fill before the first rows land
    if (b0 < b1) { stage_rows(b0); vload(b0, vpf); }
    barrier_vm<0>();
    TRACE(g, 4, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = b0; b < b1; ++b) {
        const int bn = b + 1;
        float* const Dys = Dys0 + ((b - b0) & 1) * 16 * RS;
        float vc[MOW][8];
#pragma unroll
        for (int m = 0; m < MOW; ++m)
#pragma unroll
            for (int i = 0; i < 8; ++i) vc[m][i] = vpf[m][i];
        if (bn < b1) vload(bn, vpf);
        if (row_on) {
            float* drow = Dys + wave * RS + LP;
            const floatx4 c0v = lds_ld4(CT + 8 * wave), c1v = lds_ld4(CT + 8 * wave + 4);
            const float alh = c0v[0], beh = c0v[1], gah = c0v[2], bth = c0v[3];
            const float Aoh = c1v[0], Boh = c1v[1], Coh = c1v[2];
#pragma unroll
            for (int m = 0; m < MOW; ++m) {
                const int oc = lane + 64 * m;
                if (oc < NO) {
                    float dpq[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) dpq[h] = (2 * oc + h < T1) ? DP[wave * T1 + 2 * oc + h] * 0.25f : 0.f;
                    float dy[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const bool in = 8 * oc + i < T;
                        const float v = in ? vc[m][i] : 0.f;
                        const float xh = fmaf(alh, v, beh);
                        const float z = fmaf(gah, xh, bth);
                        const float dz = dpq[i >> 2] * elu_d(z);
                        float d = fmaf(Aoh, dz, fmaf(Coh, xh, Boh));
                        d = in ? d : 0.f;
                        dy[i] = d;
                        sdyl += d;
                        sdyvl = fmaf(d, v, sdyvl);
                    }
                    lds_st_oct(drow + 8 * oc, oc, (floatx4){dy[0], dy[1], dy[2], dy[3]}, (floatx4){dy[4], dy[5], dy[6], dy[7]});
                }
            }
        }
        TRACE_PH(g, 4, 0, tph_);
        wave_lds_fence();                                  // dy row complete, dp2 row read
        // cfg5: the next trial's dp2 row of this wave now (its only reader, the dy2 phase, is done) and
        // its s row after the lag correlation -- not both after the FIR^T: the dws GEMM's x-operand
        // wait (vmcnt is in order, and the compiler, not seeing the asm DMAs, waits for zero) then
        // waited for DMAs issued just before it (profiles/r4k_timeline_cfg5.txt: 6.8 K cycles)
        if constexpr (SPEC)
            if (bn < b1 && row_on)
                for (int p = 0; p < (T1 >> 6); ++p)
                    dma4(dp2g + ((size_t)bn * F2 + o) * T1 + 64 * p + lane, DP + wave * T1 + 64 * p);
        if (row_on) {                                      // lag correlation of this wave's row
            const float* dyr = Dys + wave * RS + LP + li;
            const float* sr = Ss + wave * RS + G_::OFF + li;
            for (int ks = 0; ks < KQ; ++ks) {
                const int a = 4 * ks + lk;
                const bool on = a < NT16;
                const int ac = on ? a : 0;
                float av = dyr[16 * ac];
                av = on ? av : 0.f;
#pragma unroll
                for (int jt = 0; jt < NWT; ++jt) {
                    float bv = sr[16 * (ac + jt)];
                    bv = on ? bv : 0.f;
                    cq[jt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, cq[jt], 0, 0, 0);
                }
            }
        }
        if constexpr (SPEC)
            if (bn < b1 && row_on) {
                wave_lds_fence();                          // the lag correlation's s-row reads are done
                for (int p = 0; p < (T >> 8); ++p)
                    dma16(sg + ((size_t)bn * F2 + o) * s_pitch(T) + 256 * p + 4 * lane, Ss + wave * RS + LP + 256 * p);
            }
        TRACE_PH(g, 4, 1, tph_);
        if (row_on) {                                      // e = FIR^T(dy) -> over this wave's dy row
            const float* dyr = Dys + wave * RS;
            float e[MOW][8];
#pragma unroll
            for (int m = 0; m < MOW; ++m) {
                const int oc = lane + 64 * m;
                if (oc < NO) {
                    float w[4 * G_::NW8];
                    lds_window<G_::NW8>(dyr + 8 * oc, w);
#pragma unroll
                    for (int i = 0; i < 8; ++i) e[m][i] = 0.f;
#pragma unroll
                    for (int k = 0; k < K1; ++k)
#pragma unroll
                        for (int i = 0; i < 8; ++i) e[m][i] = fmaf(tap[K1 - 1 - k], w[G_::OFFD + i + k], e[m][i]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) e[m][i] = (8 * oc + i < T) ? e[m][i] : 0.f;
                }
            }
            wave_lds_fence();                              // every dy / s read of this wave is done
            float* erow = Dys + wave * RS + LP;
#pragma unroll
            for (int m = 0; m < MOW; ++m) {
                const int oc = lane + 64 * m;
                if (oc < NO) {
                    lds_st_oct(erow + 8 * oc, oc, (floatx4){e[m][0], e[m][1], e[m][2], e[m][3]},
                               (floatx4){e[m][4], e[m][5], e[m][6], e[m][7]});
                }
            }
        }
        // Xm[o][c] += sum_t e[o][t] x[c][t]: A = e rows (LDS), B = x (global / L2), float4 k-permuted.
        // This wave's x operand goes out XPF k-groups at a time, the first batch BEFORE the next rows'
        // DMA and the barrier: its latency overlaps the other waves' FIR^T (loaded one k-group per
        // iteration inside the GEMM, every load waited for its own round trip).
        constexpr int XPF = 4;
        const int cx = ct * 16 + li;
        const bool bon = cx < C;
        // k permutation of the operands (the same in A and B).  cfg5 (SPEC, T = 512): k-group kg of a
        // 128-sample block gives lane lk the float4 at t = 128 (kg >> 3) + 8 (kg & 7) + 64 (lk & 1) +
        // 4 (lk >> 1): x is one 16-byte global load, the e rows one ds_read_b128 whose 16-lane groups
        // (lk = 0 with 1, 2 with 3) read 16 distinct rows at offsets equal mod 64 floats -- conflict-free
        // (pass E's narrow GEMM, eegnet_stream.hip).  Other shapes: x as a 16-byte load of t = 16 kg +
        // 4 lk + {0..3}, two v_permlane16_swap exchange the middle pairs of rows lk = 0 / 1 and 2 / 3,
        // and the e rows are read in that order as two ds_read_b64 (a 32-lane group covers 16 rows x
        // one 4-dword slot per read)
        const int lo = SPEC ? 64 * (lk & 1) + 4 * (lk >> 1) : 4 * lk;
        auto tof = [&](int kg) { return SPEC ? 128 * (kg >> 3) + 8 * (kg & 7) : 16 * kg; };
        const float* xr = x + ((size_t)b * C + (bon ? cx : 0)) * T + lo;
        floatx4 xpf[XPF];
        auto xload = [&](int kgs) {
#pragma unroll
            for (int i = 0; i < XPF; ++i) {
                const int kg = min(kgs + i, kg1 - 1), t0 = tof(kg) + lo;
                if ((T & 3) == 0 && t0 + 3 < T) {
                    xpf[i] = *reinterpret_cast<const floatx4*>(xr + tof(kg));
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) xpf[i][e] = (t0 + e < T) ? xr[tof(kg) + e] : 0.f;
                }
            }
        };
        TRACE_PH(g, 4, 2, tph_);
        if (gemm_on && kg0 < kg1) xload(kg0);
        if (!SPEC && bn < b1) stage_rows(bn);              // the next trial's s / dp2 rows of this wave
        barrier_lds();                                     // e rows complete
        TRACE_PH(g, 4, 3, tph_);
        if (gemm_on) {
            const float* arow = Dys + li * RS + LP + (SPEC ? lo : 8 * (lk >> 1) + 2 * (lk & 1));
            const float* arow4 = arow + (4 + opaque0());     // (generic: not merged into a ds_read2_b64)
            for (int kgs = kg0; kgs < kg1; kgs += XPF) {   // (one batch at cfg5: 8 k-groups per wave)
#pragma unroll
                for (int i = 0; i < XPF; ++i) {
                    const int kg = kgs + i;
                    if (kg < kg1) {
                        if constexpr (SPEC) {
                            const floatx4 a4 = lds_ld4(arow + tof(kg));
                            const floatx4 b4 = bon ? xpf[i] : (floatx4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                            for (int e = 0; e < 4; ++e) xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], xacc, 0, 0, 0);
                        } else {
                            const floatx2 a0 = lds_ld2(arow + 16 * kg), a1 = lds_ld2(arow4 + 16 * kg);
                            floatx4 b4 = xpf[i];
                            float b0 = b4[0], b1 = b4[1], b2 = b4[2], b3 = b4[3];
                            swap16(b0, b2);                // rows 1 / 3: t 4, 5 <-> rows 0 / 2: t 2, 3
                            swap16(b1, b3);
                            b4 = bon ? (floatx4){b0, b1, b2, b3} : (floatx4){0.f, 0.f, 0.f, 0.f};
                            xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0], b4[0], xacc, 0, 0, 0);
                            xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1], b4[1], xacc, 0, 0, 0);
                            xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0], b4[2], xacc, 0, 0, 0);
                            xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1], b4[3], xacc, 0, 0, 0);
                        }
                    }
                }
                if (kgs + XPF < kg1) xload(kgs + XPF);
            }
        }
        TRACE_PH(g, 4, 4, tph_);
        // no second barrier: the next trial writes the other dy / e buffer (this one is rewritten two
        // trials on, after the next trial's barrier, which every wave passes only once its GEMM here
        // is done); its s / dp2 rows are this wave's own, so the wave waits for its own DMAs only
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        TRACE_PH(g, 4, 5, tph_);
    }
    TRACE_LOOP(g, 4);
    __syncthreads();

    // ---- reductions ----
    float* red = sm;                                       // [NWW][256] dws tiles | row sums | Cq tiles
    float* rsum = red + NWW * 256;                         // [16][2]: sdy, sdyv
    float* CQ = rsum + 32;                                 // [NWW][16 u][16 NWT w]
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave * 256 + (4 * lk + q) * 16 + li] = gemm_on ? xacc[q] : 0.f;
#pragma unroll
    for (int jt = 0; jt < NWT; ++jt)
#pragma unroll
        for (int q = 0; q < 4; ++q) CQ[wave * 256 * NWT + (4 * lk + q) * (16 * NWT) + 16 * jt + li] = cq[jt][q];
    {
        float rv[4] = {sdyl, sdyvl, 0.f, 0.f};
        wave_reduce<4>(rv);
        if (lane == 0) rsum[2 * wave] = rv[0];
        if (lane == 16) rsum[2 * wave + 1] = rv[0];
    }
    __syncthreads();
    const int nQ = F2 * K1, nX = F2 * C;
    if (g.splitE) {
        // k_coltail reduces: the NOC chunk workgroups of trial range rr write the disjoint column
        // segments of their rows o0 .. o0 + nrows into ONE partial row rr (the rest of a full-width row
        // per workgroup was zeros: 4x the publish and column-reduction bytes at cfg5)
        float* rowr = part + (size_t)rr * g.nE;
        for (int p = tid; p < nrows * K1; p += NTW) {       // Q[o][k]
            const int w = p / K1, k = p - w * K1;
            const float* cw = CQ + w * 256 * NWT + k;
            float v = 0.f;
#pragma unroll
            for (int u = 0; u < 16; ++u) v += cw[u * (16 * NWT + 1)];
            pub(rowr + (o0 * K1 + p), v);
        }
        for (int p = tid; p < nrows * C; p += NTW) {        // Xm[o][c]
            const int w = p / C, c = p - w * C;
            const int ct2 = c >> 4, cc = c & 15;
            float v = 0.f;
            for (int ww = ct2 * wpc; ww < (ct2 + 1) * wpc; ++ww) v += red[ww * 256 + w * 16 + cc];
            pub(rowr + (nQ + o0 * C + p), v);
        }
        if (tid < nrows) {                                  // Sdy, Sdyv
            pub(rowr + (nQ + nX + o0 + tid), rsum[2 * tid]);
            pub(rowr + (nQ + nX + F2 + o0 + tid), rsum[2 * tid + 1]);
        }
        return;
    }
    float* row = part + (size_t)blockIdx.x * g.nE;
    for (int p = tid; p < g.nE; p += NTW) {
        float v = 0.f;
        if (p < nQ) {                                       // Q[o][k]
            const int oq = p / K1, k = p - oq * K1, w = oq - o0;
            if (w >= 0 && w < nrows) {
                const float* cw = CQ + w * 256 * NWT + k;
#pragma unroll
                for (int u = 0; u < 16; ++u) v += cw[u * (16 * NWT + 1)];
            }
        } else if (p < nQ + nX) {                           // Xm[o][c]
            const int pp = p - nQ, ox = pp / C, c = pp - ox * C, w = ox - o0;
            if (w >= 0 && w < nrows) {
                const int ct2 = c >> 4, cc = c & 15;
                for (int ww = ct2 * wpc; ww < (ct2 + 1) * wpc; ++ww) v += red[ww * 256 + w * 16 + cc];
            }
        } else {                                            // Sdy, Sdyv
            const int pp = p - nQ - nX, os = pp < F2 ? pp : pp - F2, w = os - o0;
            if (w >= 0 && w < nrows) v = rsum[2 * w + (pp < F2 ? 0 : 1)];
        }
        pub(row + p, v);
    }
    double* dsm = (double*)sm;
    if (grid_reduce(g, part, g.nE, fa, dsm)) fin5(g, prm, dsm + 2, dsm + tail_s_doubles(g.nE), fa);
}

// ================================================================================================
// Wide eval forward (model.py:91-99 with .eval(), F2 > 16): one trial per 1024-thread workgroup.
// Per o-chunk: spatial GEMM -> FIR -> folded BN1/BN2 -> ELU -> pool4 into the d2 rows; then dw16,
// pointwise (MFMA), BN3 (running statistics), ELU, pool8 and the classifier.
// LDS: s rows [16][RS] | D2 [F2P][RB] | Q [F2P][RB] | W2s [F2P][16] | H [NF] | affine [F2P][4]
// ================================================================================================
template <int K1, bool SPEC = false>
__global__ __launch_bounds__(NTW) void k_winfer(Geo gin, const float* __restrict__ prm, const float* __restrict__ bn,
                                                const float* __restrict__ x, float* __restrict__ logits) {
    const Geo g = geo_w<SPEC>(gin);
    using G_ = KG<K1>;
    constexpr int LP = G_::LP;
    const int C = g.C, T = g.T, F2 = g.F2, F2P = g.F2P, RS = g.RS, T1 = T >> 2, T2 = g.T2, NF = g.NF;
    const int RB = g.RB, NT16 = (T + 15) >> 4, NT1 = (T1 + 15) >> 4, KS3 = F2P >> 2, NJT = F2P >> 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* Ss = sm;
    float* D2 = Ss + 16 * RS;
    float* Q = D2 + F2P * RB;
    float* W2s = Q + F2P * RB;
    float* W3s = W2s + F2P * K2;
    float* H = W3s + F2P * (F2P + 1);
    float* AF = H + ((NF + 3) & ~3);                   // [F2P][4]: al, be (BN1+BN2), s3, b3 (BN3)
    float* awl = AF + 4 * F2P;                         // ws fragments [NOC][KSW][64]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 16 * RS + 2 * F2P * RB; i += NTW) sm[i] = 0.f;
    for (int i = tid; i < F2P * K2; i += NTW) W2s[i] = i < F2 * K2 ? prm[g.o_w2 + i] : 0.f;
    const float* rm1 = bn;              const float* rv1 = bn + g.F1;
    const float* rm2 = bn + 2 * g.F1;   const float* rv2 = rm2 + F2;
    const float* rm3 = rm2 + 2 * F2;    const float* rv3 = rm3 + F2;
    if (tid < F2P) {
        const int oo = tid < F2 ? tid : 0, gg = oo / g.D;
        const float a1 = prm[g.o_g1 + gg] / sqrtf(rv1[gg] + g.eps);
        const float c1 = prm[g.o_b1 + gg] - a1 * rm1[gg];
        float W = 0.f;
        for (int c = 0; c < C; ++c) W += prm[g.o_ws + oo * C + c];
        const float s2 = prm[g.o_g2 + oo] / sqrtf(rv2[oo] + g.eps);
        const float s3 = prm[g.o_g3 + oo] / sqrtf(rv3[oo] + g.eps);
        AF[4 * tid + 0] = a1 * s2;
        AF[4 * tid + 1] = (c1 * W - rm2[oo]) * s2 + prm[g.o_b2 + oo];
        AF[4 * tid + 2] = s3;
        AF[4 * tid + 3] = prm[g.o_b3 + oo] - rm3[oo] * s3;
    }
    stage_w3(g, prm, W3s, F2P, tid, NTW);
    for (int j = 0; j < g.NOC; ++j) stage_aw_chunk(g, prm, 16 * j, awl + j * KSW * 64, tid, NTW);
    // pointwise tiles: wave w -> (row tile jt = w % NJT, time tiles n = w / NJT + (NWW / NJT) i)
    const int jt = wave % NJT, n0 = wave / NJT, dn = NWW / NJT;
    const int NO = (T + 7) >> 3;
    __syncthreads();
    for (int b = blockIdx.x; b < g.B; b += gridDim.x) {
        const float* xb = x + (size_t)b * C * T;
        for (int j = 0; j < g.NOC; ++j) {
            spatial_chunk(xb, awl + j * KSW * 64, Ss, C, T, NT16, RS, LP, wave, lane);
            __syncthreads();
            const int o = 16 * j + wave;
            if (o < F2) {
                float tap[K1];
#pragma unroll
                for (int k = 0; k < K1; ++k) tap[k] = prm[g.o_w1 + (o / g.D) * K1 + k];
                const float al = AF[4 * o], be = AF[4 * o + 1];
                const float* row = Ss + wave * RS;
                for (int oc = lane; oc < NO; oc += 64) {
                    float w[4 * G_::NW8];
                    lds_window<G_::NW8>(row + 8 * oc, w);
                    float v[8];
                    fir8<K1, G_::OFF>(w, tap, v);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int q = 2 * oc + h;
                        float pe = 0.f;
#pragma unroll
                        for (int i = 4 * h; i < 4 * h + 4; ++i) pe += elu_f(fmaf(al, v[i], be));
                        if (q < T1) D2[o * RB + LQW + q] = pe * 0.25f;
                    }
                }
            }
            __syncthreads();                               // s rows free, d2 rows of chunk j done
        }
        // depthwise 1x16 (model.py:54-61)
        const int TQ1 = (T1 + 3) >> 2;
        for (int it = tid; it < F2 * TQ1; it += NTW) {
            const int o = it / TQ1, qd = it - o * TQ1;
            float w[24];
            lds_window<6>(D2 + o * RB + LQW + 4 * qd - 8, w);
            float wt[K2];
            lds_window<4>(W2s + o * K2, wt);
            float out[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float a = 0.f;
#pragma unroll
                for (int k = 0; k < K2; ++k) a = fmaf(wt[k], w[1 + i + k], a);
                out[i] = (4 * qd + i < T1) ? a : 0.f;
            }
            lds_st4(Q + o * RB + LQW + 4 * qd, (floatx4){out[0], out[1], out[2], out[3]});
        }
        __syncthreads();
        // pointwise (MFMA), BN3 (eval), ELU, pool8 -> H
        for (int n = n0; n < NT1; n += dn) {
            const floatx4 acc = b2_pw_tile(Q, W3s, F2P, jt, n, RB, lane);
            const int t = 16 * n + li;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int jj = 16 * jt + 4 * lk + r;
                float e = (t < 8 * T2) ? elu_f(fmaf(AF[4 * jj + 2], acc[r], AF[4 * jj + 3])) : 0.f;
                e = sum8_hi(e);
                if ((lane & 7) == 7 && t < 8 * T2 && jj < F2) H[jj * T2 + (t >> 3)] = e * 0.125f;
            }
        }
        __syncthreads();
        if (wave < NCLS) {                                 // classifier (model.py:78-82)
            float a = 0.f;
            for (int i = lane; i < NF; i += 64) a = fmaf(prm[g.o_Wfc + wave * NF + i], H[i], a);
            a = wave_sum(a);
            if (lane == 0) logits[(size_t)b * NCLS + wave] = a + prm[g.o_bfc + wave];
        }
        __syncthreads();
    }
}

}  // namespace eeg
