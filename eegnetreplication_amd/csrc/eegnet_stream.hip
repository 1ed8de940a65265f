// eegnet_stream.hip -- the three passes that stream x (full-rate [C, T] trials): A (BN1 / BN2
// batch statistics), B (forward to the pooled block-2 input, BN3 statistics) and E (dy2 and the
// weight gradients that need full-rate data).  Included by eegnet_kernels.hip (one translation unit).
//
// Workgroup = 512 threads = 8 waves, two workgroups per CU (each <= 80 KB of LDS), trials strided
// over the grid.  Wave w owns rows o = 2w, 2w+1 of every per-trial [F2, T] plane (F2 <= 16; with
// EEGNet's D = 2 both rows share one temporal filter), so FIR taps are wave-uniform, the FIR windows
// it reads are lane-contiguous float4s and its per-row partial sums stay in registers until the
// workgroup ends.  The two workgroups of a CU run different trials and drift out of phase, so one's
// MFMA / LDS / barrier phases overlap the other's VALU FIR work -- with one 16-wave workgroup per
// CU every SIMD ran the same phase at the same time and the matrix and vector pipes took turns.

namespace eeg {

constexpr int NTB = 512;               // threads per workgroup of the streaming passes
constexpr int NWB = NTB / 64;          // waves per workgroup
constexpr int RPW = F2MAX / NWB;       // rows per wave (2)
constexpr int WGPC = 2;                // workgroups per CU
constexpr int WPEB = NWB * WGPC / 4;   // waves per SIMD: HIP's __launch_bounds__ second argument is
                                       // the minimum waves per execution unit (caps VGPRs at 128)

// FIR work layout: lane l takes row 2w + fir_row(l) and the 8 consecutive samples of octet
// fir_oct(l) + 32 m: both rows of a wave advance together, with two independent 4-output chains per
// lane per window load.  Each 16-lane group of a ds_read_b128 covers 8 octets of EACH row: octet
// starts 8 floats apart repeat a bank group every 8 octets, and the other row's base is RS = 4 mod
// 8 floats away, so the 16 windows of a group land on 16 disjoint bank quads (a half-wave per row
// put octets oc and oc + 8 of one row in the same group: a 2-way conflict on every window read).
__device__ __forceinline__ int fir_row(int lane) { return (lane >> 3) & 1; }
__device__ __forceinline__ int fir_oct(int lane) { return (lane & 7) | ((lane >> 4) << 3); }
// x row pitch: the compile-time shapes with T a multiple of 4 take contiguous rows only (make_geo), so
// their pitch is the constant T -- no run-time stride or (XP & 3) branch in the DMA loops
#define EEG_XP(TT, g) (((TT) && ((TT) & 3) == 0) ? (TT) : (g).XP)
#define EEG_NO(TT) ((TT) ? ((TT) + 7) / 8 : ((T + 7) >> 3))
#define EEG_MO(TT) ((TT) ? (((TT) + 7) / 8 + 31) / 32 : 4)

// x staging by LDS-DMA (global_load_lds_dwordx4: no VGPR destination, the wave's 64 lanes write
// 1 KiB contiguously): one wave-instruction per 256-sample piece of a channel row, rows dealt
// round-robin over the waves.  Used by the compile-time shapes (22 x 256 and 22 x 257); the
// runtime-shape kernels stage through registers (x_prefetch / x_store).  The DMA is issued right after the
// last reader of the x buffer and drains at the next __syncthreads() (the compiler's vmcnt(0)).
typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;
// Rows of other lengths (22 x 257, the real recordings) go by 4-byte pieces: 64 samples per wave
// instruction, the row's last piece on its first T mod 64 lanes only (the pads stay zero).
__device__ __forceinline__ void x_dma(const float* __restrict__ xb, int C, int T, int RS, int LP, float* Xs,
                                      int wave, int lane) {
    if ((T & 255) == 0) {
        const int np = T >> 8;                         // 256-sample pieces per row
        for (int i = wave; i < C * np; i += NWB) {
            const int c = i / np, p = i - c * np;
            __builtin_amdgcn_global_load_lds((gvoid_t*)(xb + (size_t)c * T + 256 * p + 4 * lane),
                                             (lvoid_t*)(Xs + c * RS + LP + 256 * p), 16, 0, 0);
        }
    } else {
        const int np = (T + 63) >> 6;                  // 64-sample pieces per row
        for (int i = wave; i < C * np; i += NWB) {
            const int c = i / np, p = i - c * np;
            if (lane < T - 64 * p)
                __builtin_amdgcn_global_load_lds((gvoid_t*)(xb + (size_t)c * T + 64 * p + lane),
                                                 (lvoid_t*)(Xs + c * RS + LP + 64 * p), 4, 0, 0);
        }
    }
}

// The same DMA issued from inline asm, so the compiler does not see an LDS write: its waitcnt pass
// otherwise makes the next LDS read of ANY address wait (vmcnt) for the DMA to land, which turns a
// prefetch issued ahead of a phase's LDS work into a stall at its first read.  The caller owns the
// hand-off: the data is read only after a barrier preceded by a vmcnt wait that covers the DMA
// (__syncthreads(), or barrier_vm<N> with N vector-memory operations issued after it).
__device__ __forceinline__ void dma16(const float* gsrc, const float* ldst) {
    const unsigned la = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)ldst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(gsrc), "s"(la) : "memory", "m0");
}
__device__ __forceinline__ void dma4(const float* gsrc, const float* ldst) {    // 4 bytes per lane
    const unsigned la = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)ldst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                 :: "v"(gsrc), "s"(la) : "memory", "m0");
}
// C rows of T samples at row pitch XP (floats) into LDS rows (stride RS, left pad LP).  Rows at a pitch
// that is a multiple of 4 go in 16-byte units -- 4 [T/4] of them, then T mod 4 dwords -- else in dwords
// (a 257-sample row at pitch 257 is not 16-byte aligned: five dword DMAs per row instead of two).
__device__ __forceinline__ void x_dma_asm(const float* __restrict__ xb, int C, int T, int XP, int RS, int LP,
                                          float* Xs, int wave, int lane) {
    if ((T & 255) == 0 && (XP & 3) == 0) {
        const int np = T >> 8;
        for (int i = wave; i < C * np; i += NWB) {
            const int c = i / np, p = i - c * np;
            dma16(xb + (size_t)c * XP + 256 * p + 4 * lane, Xs + c * RS + LP + 256 * p);
        }
    } else if ((XP & 3) == 0) {
        const int nu = T >> 2, np = (nu + 63) >> 6, nt = T & 3, per = np + (nt ? 1 : 0);
        for (int i = wave; i < C * per; i += NWB) {
            const int c = i / per, p = i - c * per;
            if (p < np) {
                if (lane < nu - 64 * p) dma16(xb + (size_t)c * XP + 256 * p + 4 * lane, Xs + c * RS + LP + 256 * p);
            } else if (lane < nt) {
                dma4(xb + (size_t)c * XP + 4 * nu + lane, Xs + c * RS + LP + 4 * nu);
            }
        }
    } else {
        const int np = (T + 63) >> 6;
        for (int i = wave; i < C * np; i += NWB) {
            const int c = i / np, p = i - c * np;
            if (lane < T - 64 * p) dma4(xb + (size_t)c * XP + 64 * p + lane, Xs + c * RS + LP + 64 * p);
        }
    }
}
__device__ __forceinline__ void flat_dma_asm(const float* __restrict__ src, int n, float* dst, int wave, int lane) {
    for (int i = wave; i < (n >> 8); i += NWB) dma16(src + 256 * i + 4 * lane, dst + 256 * i);
}

// Zero the workgroup's LDS rows [0, n) before the first trial.  With LDS-DMA staging (SKIPX) the x
// data windows [LP, LP + T) of the first C rows are left to the DMA, so fill and DMA touch disjoint
// words and need no barrier between them (the barrier would also wait for every weight load).
template <bool SKIPX>
__device__ __forceinline__ void zero_fill(float* sm, int n, int C, int RS, int LP, int T, int tid) {
    if constexpr (SKIPX) {
        const int wave = tid >> 6, lane = tid & 63;
        for (int r = wave; r < C; r += NWB) {
            float* row = sm + r * RS;
            for (int k = lane; k < LP; k += 64) row[k] = 0.f;
            for (int k = LP + T + lane; k < RS; k += 64) row[k] = 0.f;
        }
        for (int i = C * RS + tid; i < n; i += NTB) sm[i] = 0.f;
    } else {
        for (int i = tid; i < n; i += NTB) sm[i] = 0.f;
    }
}

// Zero only the pads [0, LP) and [LP + T, RS) of nrows LDS rows: the compile-time-shape passes DMA or
// fully write every row's data window before its first read, so the prologue need not clear it (a
// full clear of the x / s / dy rows was ~1.5 us of pass E's prologue, and it ran before the first
// trial's loads were issued)
__device__ __forceinline__ void zero_pads(float* sm, int nrows, int RS, int LP, int T, int tid) {
    const int npad = RS - T;
    for (int i = tid; i < nrows * npad; i += NTB) {
        const int r = i / npad, k = i - r * npad;
        sm[r * RS + (k < LP ? k : T + k)] = 0.f;
    }
}

// LDS-DMA of n floats (n % 256 == 0, 16-byte aligned source) into a contiguous LDS array
__device__ __forceinline__ void flat_dma(const float* __restrict__ src, int n, float* dst, int wave, int lane) {
    for (int i = wave; i < (n >> 8); i += NWB)
        __builtin_amdgcn_global_load_lds((gvoid_t*)(src + 256 * i + 4 * lane), (lvoid_t*)(dst + 256 * i), 16, 0, 0);
}

// workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not drain the wave's
// global loads and stores (vmcnt); their register results are still waited for at first use
__device__ __forceinline__ void barrier_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// the same after the wave's vector-memory operations except its N most recent have completed (vmcnt
// counts loads, stores and LDS-DMA in issue order): LDS-DMA issued before those N has landed
template <int N>
__device__ __forceinline__ void barrier_vm() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(N) : "memory");
}

// one trial's s rows (LDS, [LP | T samples] per row) -> a contiguous [F2][s_pitch(T)] block in global
// memory.  The s plane's rows are padded to s_pitch(T) floats (eegnet_common.h), zeros after T (the LDS rows'
// right pads), so every shape stores and DMAs them in 16-byte units (22 x 257: 65 float4 per row
// instead of 257 dwords).
template <int NT>
__device__ __forceinline__ void s_rows_store(const float* Ss, float* __restrict__ sb, int F2, int T, int RS, int LP,
                                             int tid) {
    const int TQ4 = s_pitch(T) >> 2;
    for (int i = tid; i < F2 * TQ4; i += NT) {
        const int o = i / TQ4, q = i - o * TQ4;
        st_pol<EEGNET_NT_SV>(lds_ld4(Ss + o * RS + LP + 4 * q), reinterpret_cast<floatx4*>(sb + 4 * i));
    }
}
// rows [0, rows) of one trial's s plane into LDS rows (stride RS, left pad LP), 16-byte LDS-DMA units
__device__ __forceinline__ void s_dma_asm(const float* __restrict__ sb, int rows, int T, int RS, int LP, float* Ss,
                                          int wave, int lane) {
    const int TS = s_pitch(T), np = (TS + 255) >> 8;
    for (int i = wave; i < rows * np; i += NWB) {
        const int c = i / np, p = i - c * np;
        if (4 * lane < TS - 256 * p) dma16(sb + (size_t)c * TS + 256 * p + 4 * lane, Ss + c * RS + LP + 256 * p);
    }
}

// this wave's v octets (fir_row / fir_oct layout) of trial b from the v plane: MO octets of 8
// samples per lane; unconditional loads at clamped addresses (a guarded load compiles to a branch
// and a wait), so rows o >= F2 and octets >= NO hold copies that the callers never use
template <int MO>
__device__ __forceinline__ void v_load(const float* __restrict__ vg, int b, int F2, int NO, int oh, int lane,
                                       float (&v)[MO][8]) {
    const float* vrow = vg + ((size_t)b * F2 + min(oh, F2 - 1)) * (8 * NO);
#pragma unroll
    for (int m = 0; m < MO; ++m) {
        const int oc = min(fir_oct(lane) + 32 * m, NO - 1);
        const floatx4 a = *reinterpret_cast<const floatx4*>(vrow + 8 * oc);
        const floatx4 c = *reinterpret_cast<const floatx4*>(vrow + 8 * oc + 4);
        v[m][0] = a[0]; v[m][1] = a[1]; v[m][2] = a[2]; v[m][3] = a[3];
        v[m][4] = c[0]; v[m][5] = c[1]; v[m][6] = c[2]; v[m][7] = c[3];
    }
}

// this half-wave's taps (a per-lane select only when the two rows of a wave use different filters)
template <int K1, int NTS>
__device__ __forceinline__ void half_taps(const float (&tap)[NTS][K1], int hr, float (&tl)[K1]) {
#pragma unroll
    for (int k = 0; k < K1; ++k) tl[k] = hr ? tap[NTS - 1][k] : tap[0][k];
}

// Temporal taps of this wave's rows: one shared set for the specialised EEGNet-8,2 shapes (the
// rows 2w, 2w+1 of a wave are group w when D = 2), one set per row otherwise.  Wave-uniform scalar
// loads (ldc): the taps land in SGPRs even when prm comes from a fold record, and the prologue does
// not wait on them behind the first trial's DMA (no pass writes w1 before every prologue is done: fin5's
// Adam runs after the last workgroup has published).
template <int K1, int NTS>
__device__ __forceinline__ void load_taps(const Geo& g, const float* __restrict__ prm, int D, int F2, int wave,
                                          float (&tap)[NTS][K1]) {
#pragma unroll
    for (int r = 0; r < NTS; ++r) {
        const int o = RPW * wave + r;
        const int gg = (o < F2 ? o : 0) / D;
#pragma unroll
        for (int k = 0; k < K1; ++k)
            tap[r][k] = ldc(prm + (g.o_w1 + gg * K1 + k));
    }
}

// ================================================================================================
// Pass A: BN1 / BN2 batch statistics (model.py:32, 47).
// part row: [G0 K1][S0][H nH][Tl nTl][hs R][ts P][Sv F2][Sv2 F2]
//   G0[d] = sum_{c,t<T} X[t] X[t+d]       (lag-Gram of the padded rows, window start 0)
//   H[a,b] = sum_c x[a] x[b], 0<=a<=b<R    (head outer products -> Gram edge corrections)
//   Tl[u,v] = sum_c x[T-P+u] x[T-P+v]     (tail outer products)
//   hs / ts = head / tail sample sums       (window-sum corrections)
//   Sv, Sv2 = sum v, sum v^2 per row o      (BN2: y2 = a1 v + c1 W)
// ================================================================================================
template <int K1, int CC, int TT, int FF, bool FOLD>
__device__ __forceinline__ void pass_a_body(const Geo& g, const float* __restrict__ prm,
                                            const float* __restrict__ x, float* __restrict__ sg,
                                            float* __restrict__ vg, float* __restrict__ part,
                                            FinArgs fa, const FoldCall& fc, float* sm) {
    using G_ = KG<K1>;
    EEG_DIMS_NT(g, NTB);
    const int XP = EEG_XP(TT, g);
    TRACE(g, 0, TR_ENTRY);
    const int64_t* perm = nullptr;                 // fold launches: trial rows through the permutation
    long long row0 = 0;
    // fold launches with eegnet_fold.xstat: the batch's BN1 lag sums are summed from the per-trial
    // table (eegnet_x_stats) instead of computed from x; x is still staged for the spatial GEMM
    const float* xst = nullptr;
    if (FOLD) {                                    // fold-indexed launch: this fold's pointers
        const eegnet_fold f = fold_rec(fc);
        prm = f.params;
        x = f.x;
        xst = f.xstat;
        perm = f.perm; row0 = fc.row0;
        sg = (float*)((char*)f.ws + fc.off.s);
        vg = (float*)((char*)f.ws + fc.off.v);
        part = (float*)((char*)f.ws + fc.off.partA);
        fa = fold_fin(fc, f, TK_A, 1, 0, false, false, g.nparam);
    }
    // every pass re-arms its own tickets when it finishes; pass A also clears those of the later
    // passes of this call (stream order), so a call never depends on how the previous one ended
    if (blockIdx.x == 0 && threadIdx.x < (TK_PASSES - 1) * NCNT)
        __hip_atomic_store(fa.cnt + NCNT + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr int NTS = FF ? 1 : RPW;
    constexpr int NEI = G_::template nei<NTB>();
    const int D = FF ? 2 : g.D;
    constexpr bool XDMA = TT != 0;                    // compile-time shapes: x / s rows by LDS-DMA
    // x buffers: compile-time shapes double-buffer x (trial b + 1 goes out by DMA at the top of trial
    // b, a whole trial ahead of its use); the others stage through registers into one buffer
    constexpr int NXB = XDMA ? 2 : 1;
    float* Xb = sm;
    float* Ss = sm + NXB * C * RS;
    float* red = Ss + F2 * RS;                        // NWB * (K1 + 1)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b0, b1;
    trial_range(g, b0, b1);

    // compile-time shapes: the first trial's x goes out by LDS-DMA before anything else; the pad fill,
    // the weight loads and the edge decode below overlap it, and one barrier waits for all of it
    if constexpr (XDMA) {
        if (b0 < b1) x_dma_asm(x + fold_row(perm, row0, b0) * (C * XP), C, T, XP, RS, LP, Xb, wave, lane);
        zero_pads(sm, NXB * C + F2, RS, LP, T, tid);
    } else {
        zero_fill<false>(sm, (C + F2) * RS, C, RS, LP, T, tid);
    }
    float aw[KS];
    load_ws_frag<KS>(prm + g.o_ws, C, F2, aw, lane);
    float tap[NTS][K1];
    load_taps<K1, NTS>(g, prm, D, F2, wave, tap);
    const int NO = EEG_NO(TT);
    float svl = 0.f, sv2l = 0.f;                     // this lane's row (half-wave) sums of v, v^2
    float G0[K1];
#pragma unroll
    for (int d = 0; d < K1; ++d) G0[d] = 0.f;
    float s0 = 0.f;
    // The 22 x 256 shape (LAGM): the lag-Gram in 8-sample items (a 40-float window per 256 FMAs:
    // 124 KB of LDS reads per 22 x 256 trial instead of 203 KB in 4-sample items), and the edge
    // products H[a][b] = sum_c x[c][a] x[c][b] (head a, b < R) and Tl (tail) as two 16 x 16 Grams on
    // the matrix cores -- A[m][k] = x[k][m] and B[k][n] = x[k][n] are the same lane value, so one LDS
    // read feeds both operands (6 k-steps for C = 22: 12 MFMAs and 12 reads per trial, against 287
    // items x 22 channels x 2 scalar LDS reads on the VALU).  Waves EW_H / EW_T run the two Grams and
    // EW_S the head / tail sample sums, each in the second lag iteration, which only waves 0-3 fill.
    constexpr bool LAGM = XDMA && K1 == 32 && TT == 256;    // (22 x 257: 5 VGPRs spill)
    constexpr int EW_S = 5, EW_H = 6, EW_T = 7;
    // xstat table row width and per-thread columns (the partial row's [G0][S0][edges] head)
    const int NV = K1 + 1 + g.nedge;
    constexpr int NXI = FOLD ? (K1 + 1 + KG<K1>::R * (KG<K1>::R + 1) / 2 + KG<K1>::P * (KG<K1>::P + 1) / 2 +
                                KG<K1>::R + KG<K1>::P + NTB - 1) / NTB : 1;
    float xacc[NXI];
#pragma unroll
    for (int k = 0; k < NXI; ++k) xacc[k] = 0.f;
    // DMA shapes: a trial's xstat row travels by LDS-DMA with its x rows, a trial ahead, into the
    // other of two slots; the trial sums it from LDS at its top (landed by the previous closing
    // barrier).  A global load of it would be waited for behind the next trial's asm x DMA (the
    // compiler cannot see that DMA: a vmcnt wait for the load is vmcnt(0)).  Wave w DMAs and reads
    // exactly the columns 64 w + NTB k + lane, so a slot is refilled only after its own readers.
    constexpr bool XSDMA = FOLD && XDMA;
    constexpr int NVP = (K1 + 1 + KG<K1>::R * (KG<K1>::R + 1) / 2 + KG<K1>::P * (KG<K1>::P + 1) / 2 +
                         KG<K1>::R + KG<K1>::P + 3) & ~3;
    float* const XSt = red + NWB * (K1 + 1);          // [2][NVP] (fold launches with xstat)
    auto xstat_dma = [&](int bb, int slot) {
        if (XSDMA && xst) {
            const float* xr = xst + (size_t)fold_row(perm, row0, bb) * NV;
#pragma unroll
            for (int k = 0; k < NXI; ++k) {
                const int c0 = 64 * wave + NTB * k;
                if (c0 < NV && lane < NV - c0) dma4(xr + c0 + lane, XSt + slot * NVP + c0);
            }
        }
    };
    static_assert(!LAGM || (KG<K1>::R <= 16 && KG<K1>::P <= 16), "edge Grams are one 16 x 16 tile");
    floatx4 egram = {0.f, 0.f, 0.f, 0.f};            // wave EW_H: head Gram tile, EW_T: tail
    float esum = 0.f;                                // wave EW_S: lane a < R head sum, R + u tail sum
    // edge items: decode (row-index a, row-index b) once; b < 0 -> a plain sample sum
    constexpr int NEIX = LAGM ? 1 : NEI;
    float eacc[NEIX];
    int ea[NEIX], eb[NEIX];
#pragma unroll
    for (int i = 0; i < NEIX; ++i) {
        eacc[i] = 0.f;
        int e = tid + NTB * i;
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
    float pf[XDMA ? 1 : PF];
    if (b0 < b1) xstat_dma(b0, 0);
    if constexpr (XDMA) {
        barrier_vm<0>();                              // the first x landed, pads and tables written
    } else {
        if (b0 < b1) x_prefetch<PF, NTB>(x + fold_row(perm, row0, b0) * (C * XP), C, T, pf, tid);
        __syncthreads();
        x_store<PF, NTB>(pf, C, T, RS, LP, Xb, tid);
        __syncthreads();
    }

    TRACE(g, 0, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = b0; b < b1; ++b) {
        const int bn = b + 1;
        pace_prio(b - b0, b1 - b0);
        if constexpr (XDMA) {
            // this trial's buffer; the next trial's x into the other one, whose last reader (the
            // previous trial) finished before the previous closing barrier.  It lands by this trial's
            // closing barrier, a whole trial later (one buffer gave it only the FIR: ~1,500 shader
            // cycles per trial waited for it, profiles/r4d_timeline.txt phase 4).
            Xb = sm + ((b - b0) & 1) * C * RS;
            if (XSDMA && xst) {                       // this trial's xstat row (landed), then the next's
#pragma unroll
                for (int k = 0; k < NXI; ++k)
                    if (tid + NTB * k < NV) xacc[k] += XSt[((b - b0) & 1) * NVP + tid + NTB * k];
            }
            if (bn < b1) {
                if (EEGNET_LDSX_A != 7)
                    x_dma_asm(x + fold_row(perm, row0, bn) * (C * XP), C, T, XP, RS, LP,
                              sm + ((bn - b0) & 1) * C * RS, wave, lane);
                xstat_dma(bn, (bn - b0) & 1);
            }
        }
        spatial_mfma<KS, NWB>(Xb, aw, Ss, C, F2, NT16, RS, LP, wave, lane);
        if (FOLD && xst) {
            if constexpr (!XDMA) {                    // register-staged shapes: no asm DMA to wait behind
                const float* xr = xst + (size_t)fold_row(perm, row0, b) * NV;
#pragma unroll
                for (int k = 0; k < NXI; ++k) {
                    const int c = tid + NTB * k;
                    if (c < NV) xacc[k] += xr[c];
                }
            }
        } else if constexpr (LAGM) {
            // lag-Gram: items (c, octet); a wave's 64 items are rows 2p, 2p + 1 in the FIR layout
            // (fir_row / fir_oct): every 16-lane group of a ds_read_b128 then covers 8 octets of EACH
            // row, 16 disjoint bank quads (rows RS = 4 mod 8 floats apart).  One row per wave, lanes on
            // consecutive octets, put octets o and o + 8 in one group: a 2-way conflict on every
            // window read (34 % of pass A's LDS cycles in round 4, profiles/r4m_pmc_summary.json).
            constexpr int TO = (TT + 7) / 8;
            static_assert(TO == 32 && CC % 2 == 0, "LAGM: two rows of 32 octets per wave");
            for (int j = tid; j < CC * TO; j += NTB) {
                const int c = 2 * (j >> 6) + fir_row(j & 63), o = fir_oct(j & 63);
                float w[4 * G_::NW8];
                if (EEGNET_LDSX_A == 3) {
#pragma unroll
                    for (int i = 0; i < 4 * G_::NW8; ++i) w[i] = 0.001f * (j + i);
                } else
                    lds_window<G_::NW8>(Xb + c * RS + 8 * o, w);
                float a[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) a[i] = (8 * o + i < T) ? w[G_::OFF + i] : 0.f;
                s0 += ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
                for (int d = 0; d < K1; ++d) {
                    float acc = G0[d];
#pragma unroll
                    for (int i = 0; i < 8; ++i) acc = fmaf(a[i], w[G_::OFF + i + d], acc);
                    G0[d] = acc;
                }
            }
            if (wave == EW_H || wave == EW_T) {
                // head (x[c][a], a < R) or tail (x[c][T - P + u], u < P; u = P is the zero pad) Gram
                const int t0 = wave == EW_H ? 0 : T - G_::P, m = lane & 15, kq = lane >> 4;
                const float* xc = Xb + LP + t0 + m;
#pragma unroll
                for (int st = 0; st < KS; ++st) {
                    const int c = 4 * st + kq;
                    const float v = c < C ? xc[c * RS] : 0.f;
                    egram = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v, egram, 0, 0, 0);
                }
            } else if (wave == EW_S && lane < G_::R + G_::P) {
                const float* xc = Xb + LP + (lane < G_::R ? lane : T - G_::P + lane - G_::R);
                float e0 = 0.f, e1 = 0.f;
#pragma unroll
                for (int c = 0; c + 1 < CC; c += 2) { e0 += xc[c * RS]; e1 += xc[(c + 1) * RS]; }
                if (CC & 1) e0 += xc[(CC - 1) * RS];
                esum += e0 + e1;
            }
        } else {
        // lag-Gram: items (c, quad), lanes of a wave on consecutive quads of one row
        for (int j = tid; j < C * TQ; j += NTB) {
            const int c = j / TQ, q = j - c * TQ;
            float w[4 * G_::NW];
            lds_window<G_::NW>(Xb + c * RS + 4 * q, w);
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
        for (int i = 0; i < NEIX; ++i) {
            if (ea[i] >= 0) {
                const float* xa = Xb + LP + ea[i];
                float acc0 = 0.f, acc1 = 0.f;
                if (eb[i] >= 0) {
                    const float* xb2 = Xb + LP + eb[i];
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
        }
        TRACE_PH(g, 0, 0, tph_);
        barrier_lds();                                     // Ss complete, x read for good (LDS only:
                                                           // the previous trial's v stores stay in flight)
        if constexpr (!XDMA)
            if (bn < b1) x_prefetch<PF, NTB>(x + fold_row(perm, row0, bn) * (C * XP), C, T, pf, tid);   // live over the FIR only
        TRACE_PH(g, 0, 1, tph_);
        // s rows -> the s plane [B][F2][T] (pass E's lag-correlation operand)
        if (EEGNET_LDSX_A != 5) s_rows_store<NTB>(Ss, sg + (size_t)b * F2 * s_pitch(T), F2, T, RS, LP, tid);
        // v = 32-tap FIR of this wave's s rows; BN2 sums of v; v -> the v plane [B][F2][8 NO] (passes
        // B and E read it back instead of recomputing the spatial GEMM and the FIR).  Compile-time
        // shapes hold v in registers across the trial's closing barrier and store it after, so the
        // barrier's vmcnt(0) -- there for the next x DMA -- does not wait for these stores.
        const int hr = fir_row(lane), o = RPW * wave + hr;
        float* const vrow = vg + ((size_t)b * F2 + (o < F2 ? o : 0)) * (8 * NO);
        constexpr bool DEFER = XDMA;                       // (without DMA the barrier waits for no store)
        constexpr int MOA = DEFER ? EEG_MO(TT) : 1;
        float vs[MOA][8];
        {
            float tl[K1];
            half_taps<K1, NTS>(tap, hr, tl);
            if (o < F2) {
                const float* row = Ss + o * RS;
                if constexpr (DEFER) {
                    // 22 x 257: the last octet holds one sample (T - 1 = 256), one 32-tap dot product
                    constexpr bool TAIL1 = TT && (TT % 8 == 1) && (EEG_NO(TT) % 32 == 1);
#pragma unroll
                    for (int m = 0; m < MOA; ++m) {
                        const int oc = fir_oct(lane) + 32 * m;
                        if (oc < NO) {
                            float w[4 * G_::NW8];
                            if (EEGNET_LDSX_A == 6) {
#pragma unroll
                                for (int i = 0; i < 4 * G_::NW8; ++i) w[i] = 0.001f * (oc + i);
                            } else
                                lds_window<G_::NW8>(row + 8 * oc, w);
                            if (TAIL1 && m == MOA - 1) {
                                float a = 0.f;
#pragma unroll
                                for (int k = 0; k < K1; ++k) a = fmaf(tl[k], w[G_::OFF + k], a);
                                vs[m][0] = a;
#pragma unroll
                                for (int i = 1; i < 8; ++i) vs[m][i] = 0.f;
                                svl += a;
                                sv2l = fmaf(a, a, sv2l);
                            } else {
                                fir8<K1, G_::OFF>(w, tl, vs[m]);
#pragma unroll
                                for (int i = 0; i < 8; ++i)
                                    if (8 * oc + i < T) { svl += vs[m][i]; sv2l = fmaf(vs[m][i], vs[m][i], sv2l); }
                            }
                        }
                    }
                } else {
                    for (int oc = fir_oct(lane); oc < NO; oc += 32) {
                        float w[4 * G_::NW8];
                        lds_window<G_::NW8>(row + 8 * oc, w);
                        float v[8];
                        fir8<K1, G_::OFF>(w, tl, v);
#pragma unroll
                        for (int i = 0; i < 8; ++i)
                            if (8 * oc + i < T) { svl += v[i]; sv2l = fmaf(v[i], v[i], sv2l); }
                        st_pol<EEGNET_NT_SV>((floatx4){v[0], v[1], v[2], v[3]}, reinterpret_cast<floatx4*>(vrow + 8 * oc));
                        st_pol<EEGNET_NT_SV>((floatx4){v[4], v[5], v[6], v[7]}, reinterpret_cast<floatx4*>(vrow + 8 * oc + 4));
                    }
                }
            }
        }
        TRACE_PH(g, 0, 2, tph_);
        if constexpr (!XDMA)
            if (bn < b1) x_store<PF, NTB>(pf, C, T, RS, LP, Xb, tid);
        TRACE_PH(g, 0, 3, tph_);
        // next x landed (asm DMA, issued at the top of the trial: explicit vmcnt), Ss free.  The
        // trial's s-plane stores are younger than that DMA, so the barrier lets them stay in flight:
        // s_rows_store issues at least NSST = floor(F2 s_pitch(T) / 4 / NTB) float4 stores per thread
        // (2 at 22 x 256, 2 or 3 at 22 x 257), so vmcnt(NSST) waits for the DMA whatever the shape
        constexpr int NSST = (TT && FF) ? imax(0, (FF * (s_pitch(TT) / 4)) / NTB) : 0;
        static_assert(NSST <= 16, "vmcnt window");
        if constexpr (XDMA) barrier_vm<NSST>();
        else __syncthreads();                              // Xb staged, Ss free
        if constexpr (DEFER) {
            if (o < F2) {
#pragma unroll
                for (int m = 0; m < MOA; ++m) {
                    const int oc = fir_oct(lane) + 32 * m;
                    if (oc < NO) {
                        st_pol<EEGNET_NT_SV>((floatx4){vs[m][0], vs[m][1], vs[m][2], vs[m][3]}, reinterpret_cast<floatx4*>(vrow + 8 * oc));
                        st_pol<EEGNET_NT_SV>((floatx4){vs[m][4], vs[m][5], vs[m][6], vs[m][7]}, reinterpret_cast<floatx4*>(vrow + 8 * oc + 4));
                    }
                }
            }
        }
        TRACE_PH(g, 0, 4, tph_);
    }
    TRACE_LOOP(g, 0);
    tail_prio();

    // ---- workgroup reduction -> one partial row ----
    float* row = part + (size_t)blockIdx.x * g.nA;
    {
        constexpr int NR = K1 + 8, NQ = NR / 4;       // [G0 K1][s0][sv RPW][sv2 RPW][pad]
        float rv[NR];
#pragma unroll
        for (int d = 0; d < K1; ++d) rv[d] = G0[d];
        rv[K1] = s0;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            rv[K1 + 1 + r] = fir_row(lane) == r ? svl : 0.f;
            rv[K1 + 1 + RPW + r] = fir_row(lane) == r ? sv2l : 0.f;
        }
#pragma unroll
        for (int i = K1 + 1 + 2 * RPW; i < NR; ++i) rv[i] = 0.f;
        wave_reduce<NR>(rv);
        if ((lane & 15) == 0) {
            const int r0 = (lane >> 4) * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j) {
                const int idx = j + r0;
                if (idx <= K1) {
                    red[wave * (K1 + 1) + idx] = rv[j];
                } else if (idx < K1 + 1 + 2 * RPW) {
                    const int k = idx - K1 - 1, r = k % RPW, o = RPW * wave + r;
                    if (o < F2) pub(row + (K1 + 1 + g.nedge + (k < RPW ? 0 : F2) + o), rv[j]);
                }
            }
        }
    }
    __syncthreads();
    if (FOLD && xst) {
#pragma unroll
        for (int k = 0; k < NXI; ++k) {
            const int c = tid + NTB * k;
            if (c < NV) pub(row + c, xacc[k]);
        }
    } else {
    if (tid <= K1) {
        float t = 0.f;
        for (int w = 0; w < NWB; ++w) t += red[w * (K1 + 1) + tid];
        pub(row + (tid), t);
    }
    if constexpr (LAGM) {
        constexpr int R_ = G_::R, P_ = G_::P, nH_ = R_ * (R_ + 1) / 2, nTl_ = P_ * (P_ + 1) / 2;
        if (wave == EW_H || wave == EW_T) {
            // D[m][n] of the Gram tile: lane l holds rows m = 4 (l >> 4) + r, column n = l & 15;
            // pairs m <= n published a-major (H: a < R; Tl: u < P, after H)
            const int n = lane & 15, E = wave == EW_H ? R_ : P_;
            const int base = K1 + 1 + (wave == EW_H ? 0 : nH_);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = 4 * (lane >> 4) + r;
                if (m <= n && n < E) pub(row + (base + m * E - m * (m - 1) / 2 + (n - m)), egram[r]);
            }
        } else if (wave == EW_S && lane < R_ + P_) {
            pub(row + (K1 + 1 + nH_ + nTl_ + lane), esum);      // hs [R] then ts [P]
        }
    } else {
#pragma unroll
    for (int i = 0; i < NEIX; ++i)
        if (ea[i] != -2 && tid + NTB * i < g.nedge) pub(row + (K1 + 1 + tid + NTB * i), eacc[i]);
    }
    }
    {
        double* dsm = (double*)sm;
        Fin1Stage f1;                              // fin1's inputs, before the ticket (Fin1Stage)
        if (!g.defer) fin1_load(g, prm, fa, f1);
        if (grid_reduce(g, part, g.nA, fa, dsm)) {
            fin1_body<K1, true>(g, prm, dsm + 2, dsm + tail_s_doubles(g.nA), fa, f1);
            TRACE(g, 0, TR_FIN);
        }
    }
}

template <int K1, int CC, int TT, int FF, bool FOLD = false>
__global__ __launch_bounds__(NTB, WPEB) void k_pass_a(Geo g, const float* __restrict__ prm,
                                                      const float* __restrict__ x, float* __restrict__ sg,
                                                      float* __restrict__ vg, float* __restrict__ part,
                                                      FinArgs fa, FoldCall fc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    pass_a_body<K1, CC, TT, FF, FOLD>(g, prm, x, sg, vg, part, fa, fc, sm);
}

// ================================================================================================
// eegnet_x_stats: the parameter-free part of pass A's BN1 statistics, per trial.  Row n of `out`:
// [G0 K1][S0][H nH][Tl nTl][hs R][ts P] of trial n alone -- the layout of pass A's partial-row head, so
// a fold-indexed pass A (eegnet_fold.xstat) sums a batch's rows of it in place of the lag-Gram.  One
// trial at a time per workgroup (run once per fold set, not per step): x rows staged into LDS, the
// 4-sample lag items and the edge items of pass A's generic path, G0 / S0 reduced over the workgroup.
// ================================================================================================
template <int K1>
__global__ __launch_bounds__(NTB) void k_xstats(Geo g, long long n, const float* __restrict__ x,
                                                float* __restrict__ out) {
    using G_ = KG<K1>;
    constexpr int NEI = G_::template nei<NTB>();
    const int C = g.C, T = g.T, RS = g.RS, XP = g.XP, TQ = (T + 3) >> 2;
    constexpr int LP = G_::LP;
    const int NV = K1 + 1 + g.nedge;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float* const Xb = sm;
    float* const red = sm + C * RS;                   // [NWB][K1 + 1]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < C * RS; i += NTB) Xb[i] = 0.f;     // pads stay zero
    int ea[NEI], eb[NEI];
#pragma unroll
    for (int i = 0; i < NEI; ++i) {                   // edge items, decoded as in pass A
        int e = tid + NTB * i;
        ea[i] = -2; eb[i] = -1;
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
        }
    }
    for (long long b = blockIdx.x; b < n; b += gridDim.x) {
        __syncthreads();                              // the previous trial's reads of Xb are done
        const float* xb = x + (size_t)b * C * XP;
        for (int i = tid; i < C * T; i += NTB) {
            const int c = i / T, t = i - c * T;
            Xb[c * RS + LP + t] = xb[(size_t)c * XP + t];
        }
        __syncthreads();
        float G0[K1];
#pragma unroll
        for (int d = 0; d < K1; ++d) G0[d] = 0.f;
        float s0 = 0.f;
        for (int j = tid; j < C * TQ; j += NTB) {
            const int c = j / TQ, q = j - c * TQ;
            float w[4 * G_::NW];
            lds_window<G_::NW>(Xb + c * RS + 4 * q, w);
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
        float* orow = out + (size_t)b * NV;
#pragma unroll
        for (int i = 0; i < NEI; ++i) {
            if (ea[i] >= 0) {
                const float* xa = Xb + LP + ea[i];
                float acc = 0.f;
                if (eb[i] >= 0) {
                    const float* xb2 = Xb + LP + eb[i];
                    for (int c = 0; c < C; ++c) acc = fmaf(xa[c * RS], xb2[c * RS], acc);
                } else {
                    for (int c = 0; c < C; ++c) acc += xa[c * RS];
                }
                orow[K1 + 1 + tid + NTB * i] = acc;
            }
        }
        constexpr int NR = (K1 + 1 + 3) & ~3, NQ = NR / 4;
        float rv[NR];
#pragma unroll
        for (int d = 0; d < K1; ++d) rv[d] = G0[d];
        rv[K1] = s0;
#pragma unroll
        for (int i = K1 + 1; i < NR; ++i) rv[i] = 0.f;
        wave_reduce<NR>(rv);
        if ((lane & 15) == 0) {
            const int r0 = (lane >> 4) * NQ;
#pragma unroll
            for (int j = 0; j < NQ; ++j)
                if (j + r0 <= K1) red[wave * (K1 + 1) + j + r0] = rv[j];
        }
        __syncthreads();
        if (tid <= K1) {
            float t = 0.f;
            for (int w = 0; w < NWB; ++w) t += red[w * (K1 + 1) + tid];
            orow[tid] = t;
        }
    }
}

// ================================================================================================
// Pass B: forward to d2, E1/E2 (pooled ELU' sums for the BN2 backward), BN3 statistics; the block-2
// depthwise and pointwise outputs q, r go to their planes for passes C and D.  v comes
// from pass A's v plane (no spatial GEMM, no FIR here): the pass streams 16 KB of v per trial in and
// 12 KB of d2 / E1 / E2 out, with one workgroup barrier per trial.
// part row: [Sr F2][Sr2 F2]
// LDS: d2 rows (pad LP2) | q rows x 2 (alternate trials) | weight table [w2 F2MAX x 16][W3 F2MAX x F2MAX]
// ================================================================================================
template <int K1, int CC, int TT, int FF, bool FOLD>
__device__ __forceinline__ void pass_b_body(const Geo& g, const float* __restrict__ prm,
                                            const float* coef,    // the finalize writes it: no __restrict__
                                            const float* __restrict__ vg,
                                            const uint8_t* __restrict__ mask2,
                                            float* __restrict__ d2g, float* __restrict__ E1g,
                                            float* __restrict__ E2g, float* __restrict__ q3g,
                                            float* __restrict__ r3g, float* __restrict__ part,
                                            FinArgs fa, const FoldCall& fc, float* sm) {
    EEG_DIMS_NT(g, NTB);
    TRACE(g, 1, TR_ENTRY);
    unsigned dk0;
    if (FOLD) {
        const eegnet_fold f = fold_rec(fc);
        char* ws = (char*)f.ws;
        prm = f.params;
        coef = (const float*)(ws + fc.off.coef);
        vg = (const float*)(ws + fc.off.v);
        mask2 = nullptr;
        d2g = (float*)(ws + fc.off.d2); E1g = (float*)(ws + fc.off.E1); E2g = (float*)(ws + fc.off.E2);
        q3g = (float*)(ws + fc.off.q3); r3g = (float*)(ws + fc.off.r3);
        part = (float*)(ws + fc.off.partB);
        fa = fold_fin(fc, f, TK_B, 1, 0, true, false, g.nparam);
        dk0 = fold_drop_key(fc, f, 0);
    } else {
        dk0 = drop_key(g, 0);
    }
    float* D2s = sm;
    float* Qs0 = D2s + F2 * RS2;
    float* Wt = Qs0 + 2 * F2 * RS2;    // block-2 weights, read with wave-uniform addresses
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b0, b1;
    trial_range(g, b0, b1);
    const int NO = EEG_NO(TT);
    constexpr int MO = EEG_MO(TT);
    const int hr = fir_row(lane), oh = RPW * wave + hr;
    // v of the next trial rides one trial ahead in registers (compile-time shapes); the first trial's
    // is requested before anything else, so the table and coefficient loads below overlap it
    constexpr bool VPF = TT != 0;
    float vpf[MO][8];
    if (VPF && b0 < b1) v_load<MO>(vg, b0, F2, NO, oh, lane, vpf);

    for (int i = tid; i < 3 * F2 * RS2; i += NTB) sm[i] = 0.f;     // pads stay zero
    for (int i = tid; i < F2MAX * (K2 + F2MAX); i += NTB) {
        float v = 0.f;
        if (i < F2MAX * K2) { if (i < F2 * K2) v = prm[g.o_w2 + i]; }
        else {
            const int j = (i - F2MAX * K2) / F2MAX, c = (i - F2MAX * K2) % F2MAX;
            if (j < F2 && c < F2) v = prm[g.o_W3 + j * F2 + c];
        }
        Wt[i] = v;
    }
    float sr[RPW], sr2[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) { sr[r] = 0.f; sr2[r] = 0.f; }
    // BN2 constants of this lane's FIR row (fir_row)
    float alh, beh, gah, bth;
    {
        const int oo = oh < F2 ? oh : 0;
        alh = coef[CF_AL2 * CSTR + oo]; beh = coef[CF_BE2 * CSTR + oo];
        gah = prm[g.o_g2 + oo]; bth = prm[g.o_b2 + oo];
    }
    __syncthreads();

    TRACE(g, 1, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = b0; b < b1; ++b) {
        const int bn = b + 1;
        pace_prio(b - b0, b1 - b0);
        float* Qs = Qs0 + ((b - b0) & 1) * F2 * RS2;
        float vc[MO][8];
        if constexpr (VPF) {
#pragma unroll
            for (int m = 0; m < MO; ++m)
#pragma unroll
                for (int i = 0; i < 8; ++i) vc[m][i] = vpf[m][i];
            if (bn < b1) v_load<MO>(vg, bn, F2, NO, oh, lane, vpf);
        } else {
            v_load<MO>(vg, b, F2, NO, oh, lane, vc);
        }
        TRACE_PH(g, 1, 0, tph_);
        // BN2, ELU, pool4, dropout (model.py:47-50) of this lane's octets
        float d2v[MO][2], e1v[MO][2], e2v[MO][2];
        if (oh < F2) {
            float* drow = D2s + oh * RS2 + LP2;
#pragma unroll
            for (int m = 0; m < MO; ++m) {
                const int oc = fir_oct(lane) + 32 * m;
                if (oc >= NO) break;
#pragma unroll
                for (int h = 0; h < 2; ++h) {                // the octet's two pool-4 windows
                    const int q = 2 * oc + h;
                    float pe = 0.f, e1 = 0.f, e2 = 0.f;
#pragma unroll
                    for (int i = 4 * h; i < 4 * h + 4; ++i) {
                        const float xh = fmaf(alh, vc[m][i], beh);
                        const float z = fmaf(gah, xh, bth);
                        const float dz = elu_d(z);
                        pe += z > 0.f ? z : dz - 1.f;          // ELU(z) = exp(z) - 1 below 0
                        e1 += dz;
                        e2 = fmaf(dz, xh, e2);
                    }
                    const float d2 = q < T1 ? pe * 0.25f * keep_mul(g, mask2, dk0, (unsigned)((b * F2 + oh) * T1 + q)) : 0.f;
                    d2v[m][h] = d2; e1v[m][h] = e1; e2v[m][h] = e2;
                    if (q < T1) drow[q] = d2;
                }
            }
        }
        wave_lds_fence();
        TRACE_PH(g, 1, 1, tph_);
        // depthwise 1x16 'same' conv of this wave's rows (model.py:54-61): pad 7 | 8
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int o = RPW * wave + r;
            if (o < F2) {
                const float* dr = D2s + o * RS2 + LP2 - 7;
                const float* w2 = Wt + o * K2;
                for (int t = lane; t < T1; t += 64) {
                    float a = 0.f;
#pragma unroll
                    for (int k = 0; k < K2; ++k) a = fmaf(w2[k], dr[t + k], a);
                    Qs[o * RS2 + t] = a;
                    q3g[((size_t)b * F2 + o) * T1 + t] = a;       // q plane (pass D)
                }
            }
        }
        TRACE_PH(g, 1, 2, tph_);
        if (oh < F2) {
#pragma unroll
            for (int m = 0; m < MO; ++m) {
                const int oc = fir_oct(lane) + 32 * m;
                if (oc >= NO) break;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int q = 2 * oc + h;
                    if (q < T1) {
                        const size_t gi = ((size_t)b * F2 + oh) * T1 + q;
                        st_pol<EEGNET_NT_MID>(d2v[m][h], d2g + gi); st_pol<EEGNET_NT_MID>(e1v[m][h], E1g + gi);
                        st_pol<EEGNET_NT_MID>(e2v[m][h], E2g + gi);
                    }
                }
            }
        }
        TRACE_PH(g, 1, 3, tph_);
        // Qs complete.  The other q buffer is written by the next trial only after every wave has
        // passed the next trial's barrier, i.e. finished this trial's pointwise reads below.  An
        // LDS-only barrier: the d2 / E1 / E2 stores and the next trial's v loads stay in flight.
        barrier_lds();
        TRACE_PH(g, 1, 4, tph_);
        // pointwise F2 x F2 (model.py:62-69) for this wave's rows; BN3 sums
        for (int t = lane; t < T1; t += 64) {
            float qv[F2MAX];
#pragma unroll
            for (int i = 0; i < F2MAX; ++i) qv[i] = i < F2 ? Qs[i * RS2 + t] : 0.f;
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int o = RPW * wave + r;
                if (o < F2) {
                    const float* w3 = Wt + F2MAX * K2 + o * F2MAX;
                    float rr = 0.f;
#pragma unroll
                    for (int i = 0; i < F2MAX; ++i) rr = fmaf(w3[i], qv[i], rr);
                    r3g[((size_t)b * F2 + o) * T1 + t] = rr;      // r plane (passes C, D)
                    sr[r] += rr;
                    sr2[r] = fmaf(rr, rr, sr2[r]);
                }
            }
        }
        TRACE_PH(g, 1, 5, tph_);
    }
    TRACE_LOOP(g, 1);
    tail_prio();
    {
        float rv[4] = {sr[0], sr[1], sr2[0], sr2[1]};
        wave_reduce<4>(rv);                        // lane 16k: item k = (k < 2 ? sr : sr2)[k % 2]
        const int k = lane >> 4, o = RPW * wave + (k & 1);
        if ((lane & 15) == 0 && o < F2) {
            float* row = part + (size_t)blockIdx.x * g.nB;
            pub(row + ((k < 2 ? 0 : F2) + o), rv[0]);
        }
    }
    {
        double* dsm = (double*)sm;
        if (grid_reduce(g, part, g.nB, fa, dsm)) { fin2(g, dsm + 2, fa); TRACE(g, 1, TR_FIN); }
    }
}

template <int K1, int CC, int TT, int FF, bool FOLD = false>
__global__ __launch_bounds__(NTB, WPEB) void k_pass_b(Geo g, const float* __restrict__ prm,
                                                      const float* coef,    // the finalize writes it: no __restrict__
                                                      const float* __restrict__ vg,
                                                      const uint8_t* __restrict__ mask2,
                                                      float* __restrict__ d2g, float* __restrict__ E1g,
                                                      float* __restrict__ E2g, float* __restrict__ q3g,
                                                      float* __restrict__ r3g, float* __restrict__ part,
                                                      FinArgs fa, FoldCall fc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    pass_b_body<K1, CC, TT, FF, FOLD>(g, prm, coef, vg, mask2, d2g, E1g, E2g, q3g, r3g, part, fa, fc, sm);
}

// ================================================================================================
// Pass E: dy2 and the weight-gradient reductions that need full-rate data.  s and v come from pass
// A's planes (no spatial GEMM, no forward FIR here); x is read once, as the dws GEMM's operand.
// part row: [Q F2*K1][Xm F2*C][Sdy F2][Sdyv F2]
// LDS: s rows | dy rows, then e rows | x rows | dp2 [F2][T1] | BN2 constants; after the loop: dws
// tiles | lag tiles
// Per trial: x DMA (for this trial's dws GEMM) | dy2 from v -> dy rows | lag correlation (dy, s) and
// FIR^T (dy -> e, in place) | barrier | next trial's s / dp2 DMA and v loads | dws GEMM (e, x) | barrier
// ================================================================================================
// EEGNET_LDSX_E = n (counter builds only, wrong results): drop one class of pass E's LDS accesses to
// read its share of SQ_LDS_BANK_CONFLICT (tools/lds_probe.sh): 1 dp2 reads, 2 FIR^T windows, 3 lag
// correlation operands, 4 dws GEMM operands, 5 dy stores, 6 e stores, 7 the in-loop LDS-DMAs
#ifndef EEGNET_LDSX_E
#define EEGNET_LDSX_E 0
#endif
template <int K1, int CC, int TT, int FF, bool FOLD>
__device__ __forceinline__ void pass_e_body(const Geo& g, const float* prm,   // Adam (finalize) writes it
                                            const float* coef,    // the finalize writes it: no __restrict__
                                            const float* __restrict__ x,
                                            const float* __restrict__ sg, const float* __restrict__ vg,
                                            const float* __restrict__ dp2g,
                                            float* __restrict__ part, FinArgs fa, const FoldCall& fc, float* sm) {
    using G_ = KG<K1>;
    EEG_DIMS_NT(g, NTB);
    const int XP = EEG_XP(TT, g);
    TRACE(g, 4, TR_ENTRY);
    const int64_t* perm = nullptr;                 // fold launches: trial rows through the permutation
    long long row0 = 0;
    if (FOLD) {
        const eegnet_fold f = fold_rec(fc);
        char* ws = (char*)f.ws;
        prm = f.params;
        coef = (const float*)(ws + fc.off.coef);
        x = f.x;
        perm = f.perm; row0 = fc.row0;
        sg = (const float*)(ws + fc.off.s);
        vg = (const float*)(ws + fc.off.v);
        dp2g = (const float*)(ws + fc.off.dp2);
        part = (float*)(ws + fc.off.partE);
        fa = fold_fin(fc, f, TK_E, 0, 0, false, true, g.nparam);
    }
    constexpr int NTS = FF ? 1 : RPW;
    const int D = FF ? 2 : g.D;
    const int QR = FF ? FF / 2 : g.QR;           // Q rows in the partial row (EEGNet-8,2 shapes: F1)
    float* const Ss = sm;                        // s rows
    float* const Dys = Ss + F2 * RS;             // dy2 rows, then (in place) e = FIR^T(dy2)
    float* const Xb = Dys + F2 * RS;             // x rows (the dws GEMM's operand)
    float* const DP = Xb + C * RS;               // dp2 [F2][T1]
    float* red = sm;                             // NWB * 256 dws tiles, reused after the trial loop
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b0, b1;
    trial_range(g, b0, b1);
    const int li = lane & 15, lk = lane >> 4;
    constexpr bool XDMA = TT != 0;                    // compile-time shapes: x / s rows by LDS-DMA
    static_assert(!XDMA || (CC && FF), "LDS-DMA staging is specialised to compile-time C and F2");

    TRACE_PS(g, 0);
    if constexpr (!XDMA) zero_fill<false>(sm, (2 * F2 + C) * RS, F2, RS, LP, T, tid);
    TRACE_PS(g, 1);
    float tap[NTS][K1];
    float* CT = DP + ((F2 * T1 + 3) & ~3);       // BN2 forward / backward constants per row, [F2][8]
    const int NO = EEG_NO(TT);
    constexpr int MO = EEG_MO(TT);
    const int hr = fir_row(lane), oh = RPW * wave + hr;
    // specialised shapes with one octet per lane and every row live: e overwrites the dy rows in place;
    // otherwise e goes to the s rows
    constexpr bool ONEOC = FF && TT && (EEG_NO(TT) <= 32) && (FF == RPW * NWB);
    // with the s rows staged by DMA (the next trial's land during the dws GEMM) e must not go to them:
    // it overwrites the dy rows in place, from registers once every read of the row is done
    constexpr bool EINPL = ONEOC || XDMA;
    float* const Eb = EINPL ? Dys : Ss;
    constexpr bool XDMA_ = TT != 0;
    constexpr bool DPDMA_ = XDMA_ && FF && ((FF * (TT / 4)) % 256 == 0);
    // the specialised pipeline (EEGNet-8,2 at T = 256): every wave DMAs its own rows of the next
    // trial's dp2 (right after its dy2 phase) and s (right after its lag correlation), the next v is
    // loaded a whole trial ahead, and the first barrier waits only for this trial's x
    constexpr bool PIPEE = ONEOC && XDMA_ && DPDMA_ && (TT / 4 == 64) && (TT == 256);
    float sdyl = 0.f, sdyvl = 0.f;                   // this lane's row (half-wave) sums of dy, dy v
    // dW1 lag correlation Q[o][k] = sum_t dy[o][t] s[o][t+k-P] on the matrix cores.  With t = 16a + u
    // and s'[i] = s[i-P]:
    //     Cq[u][w] = sum_a dy[16a+u] s'[16a+w]        (16 x 16 NWT, K = the 16-sample blocks a)
    //     Q[k]     = sum_u Cq[u][u+k]                  (diagonal sums, once, after the trial loop)
    // Cq is linear in the trial, so it accumulates over the workgroup's trials in the MFMA
    // accumulators (1.5x the MACs of the direct sum, none of its VALU issue slots or registers).
    constexpr int NWT = (15 + K1 - 1) / 16 + 1;
    floatx4 cq[RPW][NWT];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
#pragma unroll
        for (int j = 0; j < NWT; ++j) cq[r][j] = (floatx4){0.f, 0.f, 0.f, 0.f};
    // dws GEMM split: wave -> (c-tile ct, k-group range)
    const int wpc = NWB / NCT;
    const bool gemm_on = wave < wpc * NCT;
    const int ct = gemm_on ? wave / wpc : 0, part_ = gemm_on ? wave - ct * wpc : 0;
    const int kg0 = (NT16 * part_) / wpc, kg1 = gemm_on ? (NT16 * (part_ + 1)) / wpc : 0;
    floatx4 xacc = {0.f, 0.f, 0.f, 0.f};
    // without DMA (T % 256 != 0) x rows are staged through registers (pfx, during the dws GEMM) and
    // each wave stages its own s rows (RPW rows, MS samples per lane per row), so only
    // the wave itself reads them before its next barrier (the lag correlation reads own rows)
    constexpr int MS = TT ? (TT + 63) / 64 : 16;
    float pws[XDMA ? 1 : RPW][XDMA ? 1 : MS];
    auto s_rows_load = [&](int bb) {
        if constexpr (!XDMA) {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const float* src = sg + ((size_t)bb * F2 + min(RPW * wave + r, F2 - 1)) * s_pitch(T);
#pragma unroll
                for (int k = 0; k < MS; ++k) pws[r][k] = src[min(lane + 64 * k, T - 1)];
            }
        }
    };
    auto s_rows_put = [&]() {
        if constexpr (!XDMA) {
#pragma unroll
            for (int r = 0; r < RPW; ++r) {
                const int o = RPW * wave + r;
#pragma unroll
                for (int k = 0; k < MS; ++k)
                    if (o < F2 && lane + 64 * k < T) Ss[o * RS + LP + lane + 64 * k] = pws[r][k];
            }
        }
    };
    float pfx[XDMA ? 1 : PF];
    // v of the next trial: registers, loaded after the FIR^T (DMA shapes; the others load it at the
    // top of the trial, keeping registers for the register-staged x and s rows)
    constexpr bool VPF = XDMA;
    float vpf[MO][8];
    // dp2 rows of the next trial ride along (registers, one trial ahead): a synchronous load would
    // wait (vmcnt is in order) for every memory operation issued before it
    constexpr int NDP = (CC && TT) ? (FF * (TT / 4) + NTB - 1) / NTB : 8;   // F2 * T1 <= NDP * NTB
    const int ndp = F2 * T1;
    float pdp[NDP];
    // specialised shapes: dp2 rows go straight to LDS by DMA (no registers, no exposed load)
    constexpr bool DPDMA = TT && FF && ((FF * (TT / 4)) % 256 == 0);
    // compile-time shapes: the first trial's s / dp2 rows go out by LDS-DMA and its v into registers
    // before anything else; the pad fill, the tap / coefficient loads overlap them and one barrier
    // waits for all of it (in sequence these were four dependent round trips, ~6 us of prologue)
    if (b0 < b1) {
        if constexpr (XDMA) s_dma_asm(sg + (size_t)b0 * F2 * s_pitch(T), F2, T, RS, LP, Ss, wave, lane);
        else s_rows_load(b0);
        TRACE_PS(g, 3);
        if constexpr (DPDMA) flat_dma_asm(dp2g + (size_t)b0 * ndp, ndp, DP, wave, lane);
        else {
#pragma unroll
            for (int j = 0; j < NDP; ++j) pdp[j] = dp2g[(size_t)b0 * ndp + min(tid + NTB * j, ndp - 1)];
#pragma unroll
            for (int j = 0; j < NDP; ++j)
                if (tid + NTB * j < ndp) DP[tid + NTB * j] = pdp[j];
            for (int i = tid + NTB * NDP; i < ndp; i += NTB) DP[i] = dp2g[(size_t)b0 * ndp + i];
        }
        if constexpr (VPF) v_load<MO>(vg, b0, F2, NO, oh, lane, vpf);
        TRACE_PS(g, 4);
    }
    if constexpr (XDMA) zero_pads(sm, 2 * F2 + C, RS, LP, T, tid);   // the data windows are DMA'd / written
    load_taps<K1, NTS>(g, prm, D, F2, wave, tap);
    TRACE_PS(g, 2);
    {   // the BN2 forward / backward constants of this wave's rows [o][8], by scalar loads (ldc: not
        // queued behind the DMAs above; coef is the earlier finalizes', g2 / b2 change only in fin5)
        float cv = 0.f;
#pragma unroll
        for (int k = 0; k < 8 * RPW; ++k) {
            const int o = RPW * wave + (k >> 3), f = k & 7;
            if (o < F2 && f < 7) {
                const float* src = f == 0 ? coef + CF_AL2 * CSTR : f == 1 ? coef + CF_BE2 * CSTR
                                 : f == 2 ? prm + g.o_g2 : f == 3 ? prm + g.o_b2 : f == 4 ? coef + CF_AO * CSTR
                                 : f == 5 ? coef + CF_BO * CSTR : coef + CF_CO * CSTR;
                const float v = ldc(src + o);
                cv = lane == k ? v : cv;
            }
        }
        if (lane < 8 * RPW && RPW * wave + (lane >> 3) < F2) CT[8 * RPW * wave + lane] = cv;
    }
    adam_scalars_publish(g, fa);
    const int step0 = adam_step0(g, fa);   // before the reduction ticket (adam_slice)
    if constexpr (XDMA) barrier_vm<0>();          // first s / dp2 landed (asm DMA), pads and tables written
    else __syncthreads();
    if constexpr (!XDMA) {
        if (b0 < b1) {
            s_rows_put();
            x_prefetch<PF, NTB>(x + fold_row(perm, row0, b0) * (C * XP), C, T, pfx, tid);
            x_store<PF, NTB>(pfx, C, T, RS, LP, Xb, tid);
        }
        __syncthreads();
    }

    TRACE(g, 4, TR_PRO);
    TRACE_DECL();
    drain_prologue_loads();
    for (int b = b0; b < b1; ++b) {
        const int bn = b + 1;
        pace_prio(b - b0, b1 - b0);
        float vc[MO][8];
        if constexpr (VPF) {
#pragma unroll
            for (int m = 0; m < MO; ++m)
#pragma unroll
                for (int i = 0; i < 8; ++i) vc[m][i] = vpf[m][i];
            if constexpr (PIPEE)
                if (bn < b1) v_load<MO>(vg, bn, F2, NO, oh, lane, vpf);
        } else {
            v_load<MO>(vg, b, F2, NO, oh, lane, vc);
        }
        TRACE_PH(g, 4, 0, tph_);
        // dy2 = A dz2 + B + C xh2 (BN2 backward) of this lane's octets; sums of dy and dy v
        if (oh < F2) {
            float* drow = Dys + oh * RS + LP;
            const floatx4 c0 = lds_ld4(CT + 8 * oh), c1 = lds_ld4(CT + 8 * oh + 4);
            const float alh = c0[0], beh = c0[1], gah = c0[2], bth = c0[3];
            const float Aoh = c1[0], Boh = c1[1], Coh = c1[2];
#pragma unroll
            for (int m = 0; m < MO; ++m) {
                const int oc = fir_oct(lane) + 32 * m;
                if (oc >= NO) break;
                float dpq[2];
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    dpq[h] = EEGNET_LDSX_E == 1 ? 0.01f * (oc + h) : (2 * oc + h < T1) ? DP[oh * T1 + 2 * oc + h] * 0.25f : 0.f;
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
                if (EEGNET_LDSX_E != 5)
                    lds_st_oct(drow + 8 * oc, oc, (floatx4){dy[0], dy[1], dy[2], dy[3]}, (floatx4){dy[4], dy[5], dy[6], dy[7]});
            }
        }
        TRACE_PH(g, 4, 1, tph_);
        wave_lds_fence();                                  // dy rows complete, this wave's dp2 rows read
        if constexpr (PIPEE) {                             // next trial's dp2 rows of this wave
            if (bn < b1) {
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    const int o = RPW * wave + r;
                    if (EEGNET_LDSX_E != 7) dma4(dp2g + (size_t)bn * ndp + o * T1 + lane, DP + o * T1);
                }
            }
        }
        // this trial's x rows for the dws GEMM (the buffer was last read by the previous trial's
        // GEMM); they land during the lag correlation / FIR^T, by the next barrier
        if constexpr (XDMA)
            if (EEGNET_LDSX_E != 7) x_dma_asm(x + fold_row(perm, row0, b) * (C * XP), C, T, XP, RS, LP, Xb, wave, lane);
        TRACE_PH(g, 4, 2, tph_);
        {
            float tl[K1];
            half_taps<K1, NTS>(tap, hr, tl);
            // this wave's rows of the lag correlation (its own dy and s rows), then the transposed FIR
            // e[P+s] = sum_m w1[K1-1-m] dypad[s+m], written over this wave's dy rows once every read
            // of them is done.  Specialised shapes (one octet per lane, every row live) run both as one
            // straight-line block, the lag-correlation MFMAs spread through the FIR^T's FMAs.
            if constexpr (ONEOC) {
                constexpr int NT16C = (TT + 15) / 16, KQC = (NT16C + 3) / 4, NQ = RPW * KQC * NWT;
                const int oc = fir_oct(lane);
                float w[4 * G_::NW8];
                if (EEGNET_LDSX_E == 2) {
#pragma unroll
                    for (int i = 0; i < 4 * G_::NW8; ++i) w[i] = 0.001f * (lane + i);
                } else
                    lds_window<G_::NW8>(Dys + oh * RS + 8 * oc, w);
                float e[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) e[i] = 0.f;
#pragma unroll
                for (int m = 0; m < K1; ++m) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) e[i] = fmaf(tl[K1 - 1 - m], w[G_::OFFD + i + m], e[i]);
                    // lag-correlation MFMAs n in [m NQ / K1, (m+1) NQ / K1)
#pragma unroll
                    for (int n = (m * NQ) / K1; n < ((m + 1) * NQ) / K1; ++n) {
                        const int r = n / (KQC * NWT), ks = (n / NWT) % KQC, j = n % NWT;
                        const int o = RPW * wave + r, a = 4 * ks + lk;
                        const bool on = a < NT16C;
                        const int ac = on ? a : 0;
                        float av = EEGNET_LDSX_E == 3 ? 0.01f * (li + n) : Dys[o * RS + LP + li + 16 * ac];
                        float bv = EEGNET_LDSX_E == 3 ? 0.02f * (lk + n) : Ss[o * RS + G_::OFF + li + 16 * (ac + j)];
                        av = on ? av : 0.f;
                        bv = on ? bv : 0.f;
                        cq[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, cq[r][j], 0, 0, 0);
                    }
                }
                float* erow = Dys + oh * RS + LP;
#pragma unroll
                for (int i = 0; i < 8; ++i) e[i] = (8 * oc + i < T) ? e[i] : 0.f;
                wave_lds_fence();                          // every dy / s read of this wave is done
                if (EEGNET_LDSX_E != 6)
                    lds_st_oct(erow + 8 * oc, oc, (floatx4){e[0], e[1], e[2], e[3]}, (floatx4){e[4], e[5], e[6], e[7]});
                if constexpr (PIPEE) {                     // next trial's s rows of this wave
                    if (bn < b1 && EEGNET_LDSX_E != 7) {
#pragma unroll
                        for (int r = 0; r < RPW; ++r) {
                            const int o = RPW * wave + r;
                            dma16(sg + ((size_t)bn * F2 + o) * s_pitch(T) + 4 * lane, Ss + o * RS + LP);
                        }
                    }
                }
            } else {
                const int KQ = (NT16 + 3) >> 2;
#pragma unroll
                for (int r = 0; r < RPW; ++r) {
                    const int o = RPW * wave + r;
                    if (o < F2) {
                        const float* dyr = Dys + o * RS + LP + li;
                        const float* sr = Ss + o * RS + G_::OFF + li;
                        for (int ks = 0; ks < KQ; ++ks) {
                            const int a = 4 * ks + lk;
                            const bool on = a < NT16;
                            const int ac = on ? a : 0;
                            float av = dyr[16 * ac];
                            av = on ? av : 0.f;
#pragma unroll
                            for (int j = 0; j < NWT; ++j) {
                                float bv = sr[16 * (ac + j)];
                                bv = on ? bv : 0.f;
                                cq[r][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, cq[r][j], 0, 0, 0);
                            }
                        }
                    }
                }
                if constexpr (EINPL) {                     // e over this wave's dy rows (MO octets per lane)
                    float e[MO][8];
                    if (oh < F2) {
                        const float* dyr = Dys + oh * RS;
                        constexpr bool TAIL1 = TT && (TT % 8 == 1) && (EEG_NO(TT) % 32 == 1);
#pragma unroll
                        for (int m = 0; m < MO; ++m) {
                            const int oc = min(fir_oct(lane) + 32 * m, NO - 1);
                            float w[4 * G_::NW8];
                            lds_window<G_::NW8>(dyr + 8 * oc, w);
#pragma unroll
                            for (int i = 0; i < 8; ++i) e[m][i] = 0.f;
                            if (TAIL1 && m == MO - 1) {            // the last octet: sample T - 1 only
#pragma unroll
                                for (int k = 0; k < K1; ++k) e[m][0] = fmaf(tl[K1 - 1 - k], w[G_::OFFD + k], e[m][0]);
                            } else {
#pragma unroll
                                for (int k = 0; k < K1; ++k)
#pragma unroll
                                    for (int i = 0; i < 8; ++i)
                                        e[m][i] = fmaf(tl[K1 - 1 - k], w[G_::OFFD + i + k], e[m][i]);
                            }
                        }
                    }
                    wave_lds_fence();                      // every dy / s read of this wave is done
                    if (oh < F2) {
                        float* erow = Dys + oh * RS + LP;
#pragma unroll
                        for (int m = 0; m < MO; ++m) {
                            const int oc = fir_oct(lane) + 32 * m;
                            if (oc < NO) {
#pragma unroll
                                for (int i = 0; i < 8; ++i) e[m][i] = (8 * oc + i < T) ? e[m][i] : 0.f;
                                lds_st_oct(erow + 8 * oc, oc, (floatx4){e[m][0], e[m][1], e[m][2], e[m][3]},
                                           (floatx4){e[m][4], e[m][5], e[m][6], e[m][7]});
                            }
                        }
                    }
                } else
                // e -> this wave's s rows (the lag correlation above was their last reader; a wave's
                // LDS reads and writes stay in order)
                if (oh < F2) {
                    const float* dyr = Dys + oh * RS;
                    float* erow = Ss + oh * RS + LP;
                    for (int oc = fir_oct(lane); oc < NO; oc += 32) {
                        float w[4 * G_::NW8];
                        lds_window<G_::NW8>(dyr + 8 * oc, w);
                        float e[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) e[i] = 0.f;
#pragma unroll
                        for (int k = 0; k < K1; ++k)
#pragma unroll
                            for (int i = 0; i < 8; ++i) e[i] = fmaf(tl[K1 - 1 - k], w[G_::OFFD + i + k], e[i]);
#pragma unroll
                        for (int i = 0; i < 8; ++i) e[i] = (8 * oc + i < T) ? e[i] : 0.f;
                        lds_st_oct(erow + 8 * oc, oc, (floatx4){e[0], e[1], e[2], e[3]}, (floatx4){e[4], e[5], e[6], e[7]});
                    }
                }
            }
        }
        TRACE_PH(g, 4, 3, tph_);
        // the next trial's dp2 (register staging only; unconditional loads at clamped addresses)
        if (!DPDMA && bn < b1) {
#pragma unroll
            for (int j = 0; j < NDP; ++j) pdp[j] = dp2g[(size_t)bn * ndp + min(tid + NTB * j, ndp - 1)];
        }
        // e rows, x rows complete; s rows, dp2 consumed (the x DMA is asm: explicit vmcnt)
        if constexpr (PIPEE) {                             // the RPW s DMAs of this wave may stay in flight
            if (bn < b1) barrier_vm<RPW>();
            else barrier_vm<0>();
        } else if constexpr (XDMA) barrier_vm<0>();
        else __syncthreads();
        TRACE_PH(g, 4, 4, tph_);
        if (!PIPEE && bn < b1) {
            if constexpr (XDMA) s_dma_asm(sg + (size_t)bn * F2 * s_pitch(T), F2, T, RS, LP, Ss, wave, lane);
            else {                                         // registers over the dws GEMM only
                s_rows_load(bn);
                x_prefetch<PF, NTB>(x + fold_row(perm, row0, bn) * (C * XP), C, T, pfx, tid);
            }
            if constexpr (DPDMA) flat_dma_asm(dp2g + (size_t)bn * ndp, ndp, DP, wave, lane);
            asm volatile("" ::: "memory");                 // the v loads issue after the DMA (barrier_vm)
            if constexpr (VPF) v_load<MO>(vg, bn, F2, NO, oh, lane, vpf);
        }
        TRACE_PH(g, 4, 5, tph_);
        // Xm[o][c] += sum_t e[o][t] x[c][t] on the matrix cores (16 e rows x 16 x rows of this wave's
        // c-tile; the k order inside the wave's t range is permuted identically in A and B)
        if (gemm_on) {
            const int c = ct * 16 + li;
            const bool aon = li < F2, bon = c < C;
            if constexpr (TT != 0 && TT / 128 >= 2) {
                // k-group kg of a 128-sample block: lane lk takes the float4 at t = 128 (kg >> 3) +
                // 8 (kg & 7) + 64 (lk & 1) + 4 (lk >> 1), one ds_read_b128 per operand.  The 16-lane
                // groups of ds_read_b128 ({0-3, 12-15, 20-27}, ...) pair lk = 0 with 1 and 2 with 3, whose
                // offsets now agree mod 64 floats (one bank row): a group is 16 distinct rows li, each on
                // its own 4-bank slot (RS / 4 odd) -- conflict-free at one instruction per operand (the
                // plain t = 16 kg + 4 lk order was 2-way; two ds_read_b64 per operand are conflict-free
                // but cost more issue than the conflicts did)
                // (a lane past the last channel reads -- and zeroes -- row li, not row 0: row 0 shares
                // its 4-bank slot with row 16, which lane li = 0 of the second c-tile reads)
                // 22×257: the k-groups past the last whole 128-sample block (kg 16: t = 256 and the
                // zero pad) keep the plain order t = 16 kg + 4 lk, the only 2-way group of the trial
                constexpr int KGP = 8 * (TT / 128);
                const int lo = 64 * (lk & 1) + 4 * (lk >> 1);
                const float* arow = Eb + (aon ? li : 0) * RS + LP + lo;
                const float* brow = Xb + (bon ? c : li) * RS + LP + lo;
                for (int kg = kg0; kg < kg1; ++kg) {
                    const int to = kg < KGP ? 128 * (kg >> 3) + 8 * (kg & 7) : 16 * kg + 4 * lk - lo;
                    floatx4 a4, b4;
                    if (EEGNET_LDSX_E == 4) {
                        a4 = (floatx4){0.01f * kg, 0.02f * li, 0.f, 1.f};
                        b4 = (floatx4){0.03f * kg, 0.01f * lk, 1.f, 0.f};
                    } else {
                        a4 = lds_ld4(arow + to);
                        b4 = lds_ld4(brow + to);
                    }
                    if (!aon) a4 = (floatx4){0.f, 0.f, 0.f, 0.f};
                    if (!bon) b4 = (floatx4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int e = 0; e < 4; ++e) xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[e], b4[e], xacc, 0, 0, 0);
                }
            } else {
                // operands by ds_read_b64: lane lk takes t = 16 kg + 2 lk + {0, 1} and 16 kg + 8 + 2 lk +
                // {0, 1}.  A 32-lane group then reads 16 rows x 4 dwords = all 64 banks once (RS / 4 odd).
                // The +8 halves go through an offset the compiler cannot see: two plain ds_read_b64 8
                // floats apart merge into one ds_read2_b64, which banks mod 32 in 16-lane groups (2-way)
                const float* arow = Eb + (aon ? li : 0) * RS + LP + 2 * lk;
                const float* brow = Xb + (bon ? c : (li < C ? li : 0)) * RS + LP + 2 * lk;
                const int o8 = 8 + opaque0();
                const float* arow8 = arow + o8;
                const float* brow8 = brow + o8;
                for (int kg = kg0; kg < kg1; ++kg) {
                    floatx2 a0 = lds_ld2(arow + 16 * kg), a1 = lds_ld2(arow8 + 16 * kg);
                    floatx2 b0 = lds_ld2(brow + 16 * kg), b1 = lds_ld2(brow8 + 16 * kg);
                    if (!aon) { a0 = (floatx2){0.f, 0.f}; a1 = a0; }
                    if (!bon) { b0 = (floatx2){0.f, 0.f}; b1 = b0; }
                    xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[0], b0[0], xacc, 0, 0, 0);
                    xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[1], b0[1], xacc, 0, 0, 0);
                    xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[0], b1[0], xacc, 0, 0, 0);
                    xacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[1], b1[1], xacc, 0, 0, 0);
                }
            }
        }
        if (bn < b1) {
            if constexpr (!DPDMA) {                        // next trial's dp2 rows: every reader is past
#pragma unroll
                for (int j = 0; j < NDP; ++j) {
                    const int i = tid + NTB * j;
                    if (i < ndp) DP[i] = pdp[j];
                }
            }
        }
        TRACE_PH(g, 4, 6, tph_);
        // (without DMA the next trial's x rows are stored right after the barrier: the next reader of
        // the x buffer is that trial's dws GEMM, behind its first barrier)
        // e, x rows consumed; next s rows and dp2 staged.  With both by DMA the barrier waits for the
        // DMA only: the 2 MO v loads issued after it stay in flight into the next trial.
        if constexpr (PIPEE) barrier_vm<0>();
        else if constexpr (XDMA && DPDMA && VPF) barrier_vm<2 * MO>();
        else if constexpr (XDMA || DPDMA) barrier_vm<0>();
        else __syncthreads();
        if constexpr (!XDMA)
            if (bn < b1) {
                x_store<PF, NTB>(pfx, C, T, RS, LP, Xb, tid);
                s_rows_put();
            }
        TRACE_PH(g, 4, 7, tph_);
    }
    TRACE_LOOP(g, 4);
    tail_prio();
    __syncthreads();

    // ---- reductions ----
    float* row = part + (size_t)blockIdx.x * g.nE;
    {
        // per-row sums: [sdy][sdyv][pad 2]; a row's lanes (fir_row) are first gathered into
        // one half-wave (lane L of half h takes the lane that held octet L & 31 of row h)
        constexpr int NR = 4, NH = NR / 2;
        float rv[NR];
        rv[0] = sdyl; rv[1] = sdyvl; rv[2] = 0.f; rv[3] = 0.f;
        {
            const int ocl = lane & 31;
            const int src = (ocl & 7) | ((ocl >> 3) << 4) | ((lane >> 5) << 3);
#pragma unroll
            for (int k = 0; k < NR; ++k) rv[k] = __shfl(rv[k], src, 64);
        }
        half_reduce<NR>(rv);
        if ((lane & 15) == 0) {
            const int o = RPW * wave + (lane >> 5), off = ((lane >> 4) & 1) * NH;
            if (o < F2) {
#pragma unroll
                for (int j = 0; j < NH; ++j) {
                    const int idx = j + off;
                    if (idx == 0) pub(row + (QR * K1 + F2 * C + o), rv[j]);
                    else if (idx == 1) pub(row + (QR * K1 + F2 * C + F2 + o), rv[j]);
                }
            }
        }
    }
    // Q: this wave's Cq tiles -> its own LDS slice [16 u][16 NWT w] (past the dws tiles) -> diagonal
    // sums; with D = 2 (QR = F1) the wave's two rows are one temporal group and publish their sum
    {
        float* CQ = red + NWB * 256 + wave * (256 * NWT);
        const bool grp = QR != F2;
        float qg = 0.f;                                // K1 <= 64: lane = lag k
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int o = RPW * wave + r;
            if (o < F2) {
#pragma unroll
                for (int j = 0; j < NWT; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) CQ[(4 * lk + q) * (16 * NWT) + 16 * j + li] = cq[r][j][q];
                wave_lds_fence();
                if (lane < K1) {
                    float a = 0.f;
#pragma unroll
                    for (int u = 0; u < 16; ++u) a += CQ[u * (16 * NWT) + u + lane];
                    if (grp) qg += a;
                    else pub(row + (o * K1 + lane), a);
                }
                wave_lds_fence();
            }
        }
        if (grp && RPW * wave < F2 && lane < K1) pub(row + (wave * K1 + lane), qg);
    }
    // Xm: wave -> 16x16 tile partial (rows 4lk+q, col li) -> LDS [wave][256] -> sum over the
    // waves of each c-tile
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave * 256 + (4 * lk + q) * 16 + li] = gemm_on ? xacc[q] : 0.f;
    __syncthreads();
    for (int p = tid; p < F2 * C; p += NTB) {
        const int oo2 = p / C, c = p - oo2 * C;
        const int ct2 = c >> 4, cc = c & 15;
        float a = 0.f;
        for (int w = ct2 * wpc; w < (ct2 + 1) * wpc; ++w) a += red[w * 256 + oo2 * 16 + cc];
        pub(row + (QR * K1 + p), a);
    }
    {
        double* dsm = (double*)sm;
        // fin5's inputs, loaded before the ticket by every workgroup (the winner's are in hand when it
        // starts fin5; eegnet_finalize.hip Fin5Stage).  Not for a deferred (synchronised-BN) pass: its
        // k_fin runs fin5.
        Fin5Stage f5;
        if (!g.defer) fin5_load(g, fa, blockIdx.x, f5);
        if (grid_reduce(g, part, g.nE, fa, dsm)) {
            fin5_body<true>(g, prm, dsm + 2, dsm + tail_s_doubles(g.nE), fa, blockIdx.x, f5);
            TRACE(g, 4, TR_FIN);
        } else {
            adam_slice(g, fa, blockIdx.x, gridDim.x, step0);  // off the critical path: the winner is still reducing
        }
    }
}

template <int K1, int CC, int TT, int FF, bool FOLD = false>
__global__ __launch_bounds__(NTB, WPEB) void k_pass_e(Geo g, const float* prm,   // Adam (finalize) writes it
                                                      const float* coef,    // the finalize writes it: no __restrict__
                                                      const float* __restrict__ x,
                                                      const float* __restrict__ sg, const float* __restrict__ vg,
                                                      const float* __restrict__ dp2g,
                                                      float* __restrict__ part, FinArgs fa, FoldCall fc) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    pass_e_body<K1, CC, TT, FF, FOLD>(g, prm, coef, x, sg, vg, dp2g, part, fa, fc, sm);
}

}  // namespace eeg
