// eegnet_finalize.hip -- the in-kernel deterministic fp64 reduction that ends every pass, the finalize
// bodies its last workgroup runs (BN constants, running statistics, parameter gradients, clamps, Adam)
// and the standalone Adam / clamp kernels of the data-parallel path.
// Included by eegnet_kernels.hip (one translation unit).

namespace eeg {

// ================================================================================================
// In-kernel deterministic fp64 reduction of the per-workgroup partial rows (cdna_hip_programming.md
// §6 Guideline 16, counter form).  Every workgroup of a pass publishes its row (write-through stores,
// every wave drains, barrier, one lane: relaxed agent ticket add).  The last arriver of
// each group of rgs rows sums the group's rows in fp64 (agent acquire first) into part2; the last
// of those group reducers sums the ngrp group partials into S (LDS) and runs the pass's finalize.
// The summation order is fixed by (row, column) alone, so results do not depend on arrival order.
// ================================================================================================

// Partial rows and group partials are published write-through (sc1 stores, Guideline 16 R1), so no
// agent release fence is needed: each storing wave drains its stores before the workgroup barrier,
// then one lane adds the ticket.  The ticket winner's agent acquire drops this CU's stale L1 lines
// before its plain loads.
__device__ __forceinline__ void pub(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pub(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Agent-coherent loads of published rows (sc1 loads, AMDGPUUsage GFX942 "load atomic monotonic
// agent"): the reader needs no L2 invalidate (buffer_inv sc1) after its ticket, which measured at
// microseconds of stall for the loads that follow it.
__device__ __forceinline__ float ld_pub(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_pub(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads call; returns (workgroup-uniformly) whether this workgroup took the last of `target`
// tickets on *w.  `flag` is one LDS word nobody else touches between the two barriers.
__device__ __forceinline__ bool take_ticket(unsigned* w, unsigned target, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // every storing wave drains
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == target - 1u;
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}

// LDS carve-up of the tail (doubles, from the start of the pass kernel's dynamic LDS, which is no
// longer in use once the partial row is written): [flag 2][S rup2(ncols)][scratch]
__host__ __device__ constexpr int tail_scratch_doubles(int ncols) { return ncols > NTH ? ncols : NTH; }
#ifndef EEGNET_RGB
#define EEGNET_RGB 32
#endif
constexpr int RGB = EEGNET_RGB;   // partial rows per group reducer batch (one round trip)
// 32-row groups, at most 16 of them (EEGNET_NGRPMAX): both levels read about the same bytes in one
// batch each.  Against 16-row groups / 32 groups at B = 4096 the top level took 2.5-3.3 µs instead of
// 4.2-5.2 µs per pass, the group level the same (r3 step timelines), +3 % cfg2 train trials/s.
constexpr int FLAT_PH = 16;       // row phases per column of a one-level reduction
constexpr long long FLAT_ELEMS = 16384;   // partial-row elements (grid x ncols) reduced in one level
// (and grids of at most 128 rows: 512 workgroups on one ticket word serialise their atomics -- pass B
// at B = 4096 took 11.6 µs from the last publish to its end, 7.3 through two levels)
#ifndef EEGNET_FLAT_MAXGRID
#define EEGNET_FLAT_MAXGRID 128
#endif
__host__ __device__ constexpr int tail_s_doubles(int ncols) { return 2 + ((ncols + 1) & ~1); }

// copy n published doubles into LDS, NLB loads in flight per thread (a one-load-per-iteration loop
// waits a global round trip per iteration: k_coltail's 4-6 K totals at cfg5)
template <int NLB>
__device__ __forceinline__ void stage_pub(double* dst, const double* src, int n) {
    const int nth = blockDim.x;
    for (int i0 = threadIdx.x; i0 < n; i0 += NLB * nth) {
        double v[NLB];
#pragma unroll
        for (int j = 0; j < NLB; ++j) v[j] = ld_pub(src + min(i0 + j * nth, n - 1));
#pragma unroll
        for (int j = 0; j < NLB; ++j)
            if (i0 + j * nth < n) dst[i0 + j * nth] = v[j];
    }
}

__device__ bool grid_reduce(const Geo& g, const float* part, int ncols, const FinArgs& fa, double* dsm) {
    const int tid = threadIdx.x, nth = blockDim.x;
    int* flag = (int*)dsm;
    double* S = dsm + 2;
    // partial rows per group / groups from this launch's own grid (passes use different grids):
    // groups of <= RGB rows, so a group reducer fetches each column's rows in one batch
    const int grid = gridDim.x;
    // narrow partial rows (pass B's 32 columns): every row in ONE group, read by all threads at once
    // (column x row phase), so the pass ends in one ticket and one batch of loads
    const bool flat = (long long)grid * ncols <= FLAT_ELEMS && ncols * FLAT_PH <= nth && grid <= EEGNET_FLAT_MAXGRID;
    const int rgs = flat ? grid : max(RGB, (grid + NGRPMAX - 1) / NGRPMAX), ngrp = (grid + rgs - 1) / rgs;
    const int grp = blockIdx.x / rgs;
    const int r0 = grp * rgs, r1 = min(grid, r0 + rgs);
    const int tp = fa.tpass;
    TRACE(g, tp, TR_PUB);
    if (!take_ticket(fa.cnt + grp, (unsigned)(r1 - r0), flag)) return false;
    TRACE_FS(g, tp, 0);            // last writer wins: about the last group
    if (flat) {
        // thread (column c, phase ph) sums rows ph, ph + FLAT_PH, ... in order; the phases are then
        // combined in phase order (fixed by (row, column) alone: deterministic)
        double* ph = S + ((ncols + 1) & ~1);           // [ncols][FLAT_PH] scratch after S
        const int c = tid / FLAT_PH, q = tid - c * FLAT_PH;
        if (c < ncols) {
            const float* col = part + c;
            double a = 0.0;
            for (int rb = q; rb < grid; rb += RGB * FLAT_PH) {
                float v[RGB];
#pragma unroll
                for (int j = 0; j < RGB; ++j) v[j] = ld_pub(col + (size_t)min(rb + j * FLAT_PH, grid - 1) * ncols);
#pragma unroll
                for (int j = 0; j < RGB; ++j) a += rb + j * FLAT_PH < grid ? (double)v[j] : 0.0;
            }
            ph[c * FLAT_PH + q] = a;
        }
        if (tid == 0) __hip_atomic_store(fa.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        for (int cc = tid; cc < ncols; cc += nth) {
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < FLAT_PH; ++k) a += ph[cc * FLAT_PH + k];
            S[cc] = a;
        }
        __syncthreads();
        TRACE(g, tp, TR_TOP);
        if (g.defer) {
            for (int cc = tid; cc < ncols; cc += nth) fa.part2[cc] = S[cc];
            return false;
        }
        return true;
    }
    if (ngrp == 1) {
        // one group (small grids: fold-indexed launches, small batches): its reducer IS the top level --
        // the same sums in the same order as through part2 (0.0 + v == v), one round trip fewer
        for (int c = tid; c < ncols; c += nth) {
            const float* col = part + c;
            double a = 0.0;
            for (int rb = r0; rb < r1; rb += RGB) {
                float v[RGB];
#pragma unroll
                for (int j = 0; j < RGB; ++j) v[j] = ld_pub(col + (size_t)min(rb + j, r1 - 1) * ncols);
#pragma unroll
                for (int j = 0; j < RGB; ++j) a += rb + j < r1 ? (double)v[j] : 0.0;
            }
            S[c] = a;
        }
        if (tid == 0) __hip_atomic_store(fa.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        TRACE(g, tp, TR_TOP);
        if (g.defer) {
            for (int c = tid; c < ncols; c += nth) fa.part2[c] = S[c];
            return false;
        }
        return true;
    }
    // group reducer: each thread sums whole columns, RGB row loads in flight, in row order
    for (int c = tid; c < ncols; c += nth) {
        const float* col = part + c;
        double a = 0.0;
        for (int rb = r0; rb < r1; rb += RGB) {
            // unconditional loads (clamped rows): a guarded load compiles to a branch and a wait each
            float v[RGB];
#pragma unroll
            for (int j = 0; j < RGB; ++j) v[j] = ld_pub(col + (size_t)min(rb + j, r1 - 1) * ncols);
#pragma unroll
            for (int j = 0; j < RGB; ++j) a += rb + j < r1 ? (double)v[j] : 0.0;
        }
        pub(fa.part2 + (size_t)grp * ncols + c, a);
    }
    TRACE(g, tp, TR_GRP);
    TRACE_FS(g, tp, 1);            // last writer wins: about the last group
    if (!take_ticket(fa.cnt + (NCNT - 1), (unsigned)ngrp, flag)) return false;
    TRACE_FS(g, tp, 2);
    for (int c = tid; c < ncols; c += nth) {
        double v[NGRPMAX];
#pragma unroll
        for (int q = 0; q < NGRPMAX; ++q) v[q] = ld_pub(fa.part2 + (size_t)min(q, ngrp - 1) * ncols + c);
        double a = 0.0;
#pragma unroll
        for (int q = 0; q < NGRPMAX; ++q) a += q < ngrp ? v[q] : 0.0;
        S[c] = a;
    }
    TRACE_FS(g, tp, 9);
    // every ticket of this pass has been taken: re-arm them for the next call
    if (tid < ngrp) __hip_atomic_store(fa.cnt + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) __hip_atomic_store(fa.cnt + (NCNT - 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    TRACE_FS(g, tp, 10);
    __syncthreads();
    TRACE(g, tp, TR_TOP);
    TRACE_FS(g, tp, 3);
    if (g.defer) {                 // synchronised BatchNorm: the host all-reduces the sums, then k_fin
        for (int c = tid; c < ncols; c += nth) fa.part2[c] = S[c];
        return false;
    }
    return true;
}

// ================================================================================================
// Finalize bodies (run by the last workgroup of each pass, blockDim.x threads): BN constants, running
// statistics, parameter gradients, clamps; Adam after pass E.
// ================================================================================================
__device__ __forceinline__ void bn_running(float* rm, float* rv, double mu, double var, double n,
                                           float mom) {
    *rm = (float)((1.0 - mom) * (double)*rm + mom * mu);
    *rv = (float)((1.0 - mom) * (double)*rv + mom * var * n / (n - 1.0));
}

// Finalize scratch (doubles) of fin1 / fin5; both begin with ONE batch of global loads into LDS
// (a finalize runs on the critical path between two launches: every dependent global round trip
// there is a few hundred ns with the rest of the GPU idle)
__host__ __device__ constexpr int fin1_scratch_doubles(int K1, int F1, int F2, int C) {
    // G [K1][K1+1] | S1 | a1, c1 [64 each] | staged floats | G w1 products [2][F1 K1]
    return K1 * (K1 + 1) + K1 + 128 + (F1 * K1 + 2 * F1 + F2 * C + 2 * F1 + 2 * F2 + 3) / 2 + 2 * F1 * K1 + 2;
}
// (ng = the number of leading parameters fin5 itself differentiates: o_g2)
__host__ __device__ constexpr int fin5_scratch_doubles(int K1, int F1, int ng) {
    // G w1 [F1 K1] | S1 [K1] | db1, dg1 [64 each] | coefficient block | gradients [0, ng) (floats)
    return F1 * K1 + K1 + 128 + (CF_COUNT * CSTR + ng + 1) / 2 + 2;
}

// after pass A: BN1 (model.py:32) and BN2 (model.py:47) batch statistics.  Latency is what matters
// here (one workgroup on the critical path between two launches), so every dependent step is short:
// the lag-Gram's edge differences Ed[d][j] in parallel, one serial prefix per lag d (a lane each), the
// matrix-vector products G w1 as (filter, tap) lanes with four partial chains, and the filters' sums
// over taps from LDS -- no shuffle scans.  G w1 and S1 go to fa.stats for fin5 (dW1 needs exactly those,
// the same parameters being in force through pass E).
// fin1's one batch of global loads (w1 | g1 | b1 | ws and the BN running statistics) as registers:
// k_pass_a issues it in every workgroup before the reduction ticket (as k_pass_e does fin5's).  The
// parameters change only in the previous step's fin5, the running statistics only in fin1 itself.
struct Fin1Stage {
    Stage<2, float> sp;
    Stage<1, float> sb;
};
__device__ __forceinline__ void fin1_load(const Geo& g, const float* prm, const FinArgs& fa, Fin1Stage& st) {
    st.sp.load(prm + g.o_w1, g.F1 * g.K1 + 2 * g.F1 + g.F2 * g.C);
    if (fa.update_running) st.sb.load(fa.bn, 2 * g.F1 + 2 * g.F2);
}
template <int K1, bool PRE>
__device__ __forceinline__ void fin1_body(const Geo& g, const float* prm, const double* sums, double* scr,
                                          const FinArgs& fa, Fin1Stage& st) {
    const int F1 = g.F1, F2 = g.F2, C = g.C, nth = blockDim.x;
    constexpr int P = (K1 - 1) / 2, R = K1 - 1 - P, NH = R * (R + 1) / 2, NTL = P * (P + 1) / 2;
    const int GS = K1 + 1;            // padded row stride of G and Ed (conflict-free column walks)
    double* Gm = scr;                 // K1 * GS
    double* S1 = Gm + K1 * GS;        // K1
    double* a1s = S1 + K1;            // F1 (<= 64)
    double* c1s = a1s + 64;
    // staged global inputs (floats): w1 | g1 | b1 | ws | rm1 rv1 | rm2 rv2
    float* pl = (float*)(c1s + 64);
    float* pw1 = pl;
    float* pg1 = pw1 + F1 * K1;
    float* pb1 = pg1 + F1;
    float* pws = pb1 + F1;
    float* pbn = pws + F2 * C;
    // after the staged floats: the per-(filter, tap) products [2][F1 K1]
    double* pq = (double*)(pl + ((F1 * K1 + 2 * F1 + F2 * C + 2 * F1 + 2 * F2 + 3) & ~1));
    double* pm = pq + F1 * K1;
    const int tid = threadIdx.x;
    {   // w1 | g1 | b1 | ws are contiguous in the parameter vector (eegnet_host.hip param layout)
        const int nl = F1 * K1 + 2 * F1 + F2 * C, nb = 2 * F1 + 2 * F2;
        if constexpr (!PRE) fin1_load(g, prm, fa, st);
        st.sp.store(pl, nl);
        if (fa.update_running) st.sb.store(pbn, nb);
    }
    TRACE_FS(g, fa.tpass, 11);
    const double* G0 = sums;
    const double S0 = sums[K1];
    const double* H = sums + K1 + 1;                 // head pairs (a <= b < R), a-major
    const double* Tl = H + NH;                       // tail pairs (u <= v < P), u-major
    const double* hs = Tl + NTL;                     // head sample sums [R]
    const double* ts = hs + R;                       // tail sample sums [P]
    const double* Sv = ts + P;
    const double* Sv2 = Sv + F2;
    // lag-Gram of the padded rows: G[k][k+d] = G0[d] + sum_{j<k} Ed[d][j], with
    // Ed[d][j] = sum_c X[T+j]X[T+j+d] - X[j]X[j+d] = Tl[j][j+d] (j+d < P) - H[j-P][j-P+d] (j >= P).
    // Lag d is a group of 8 lanes, lane q owning positions k = 4q .. 4q + 3 (K1 <= 32) or 8q .. 8q + 7
    // (K1 = 64): each lane sums its own Ed terms, the group's exclusive prefix over q takes three
    // shuffles, then each lane writes its positions.  (A serial 32-step prefix per lag, one lane each,
    // took 5.5 µs of the 9.4 µs finalize: every step waited an LDS round trip.)  Every load is
    // unconditional at a clamped index (a guarded load is a branch and a wait each) and selected after.
    constexpr int KPL = K1 / 8;                       // positions per lane
    if (tid < 8 * K1) {
        const int d = tid >> 3, q = tid & 7, k0 = KPL * q;
        double tv[KPL], hv[KPL];
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int k = k0 + i, a = k - P;
            tv[i] = Tl[min(max(k * P - k * (k - 1) / 2 + d, 0), NTL - 1)];
            hv[i] = H[min(max(a * R - a * (a - 1) / 2 + d, 0), NH - 1)];
        }
        double ed[KPL], seg = 0.0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int k = k0 + i;
            const bool on = k < K1 - 1 - d;
            const double v = (on && k + d < P ? tv[i] : 0.0) - (on && k >= P ? hv[i] : 0.0);
            ed[i] = v;
            seg += v;
        }
        // exclusive prefix of the segment sums over the 8 lanes of lag d
        double inc = seg;
#pragma unroll
        for (int sh = 1; sh < 8; sh <<= 1) {
            const double u = __shfl_up(inc, sh, 8);
            if (q >= sh) inc += u;
        }
        double v = G0[d] + (inc - seg);
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int k = k0 + i;
            if (k + d < K1) {
                Gm[k * GS + k + d] = v;
                Gm[(k + d) * GS + k] = v;
            }
            v += ed[i];
        }
    }
    // window sums S1[k] = S0 + sum_{j<k} (X[T+j] - X[j]): the same 8-lane segmented prefix, by the 8
    // lanes after the lag groups (K1 = 64 at 512 threads: lanes 0-7, after a barrier)
    auto window_sums = [&](int q) {
        const int k0 = KPL * q;
        double es[KPL], seg = 0.0;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            const int k = k0 + i;
            const double tsv = ts[min(k, P - 1)], hsv = hs[min(max(k - P, 0), R - 1)];
            const double v = (k < P ? tsv : 0.0) - (k >= P ? hsv : 0.0);
            es[i] = v;
            seg += v;
        }
        double inc = seg;
#pragma unroll
        for (int sh = 1; sh < 8; sh <<= 1) {
            const double u = __shfl_up(inc, sh, 8);
            if (q >= sh) inc += u;
        }
        double v = S0 + (inc - seg);
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
            S1[k0 + i] = v;
            v += es[i];
        }
    };
    const bool s1_now = 8 * K1 + 8 <= nth;
    if (s1_now && tid >= 8 * K1 && tid < 8 * K1 + 8) window_sums(tid - 8 * K1);
    __syncthreads();
    if (!s1_now) {
        if (tid < 8) window_sums(tid);
        __syncthreads();
    }
    TRACE_FS(g, fa.tpass, 4);
    // G w1 per (filter, tap): row k of the symmetric G, four partial chains
    for (int p = tid; p < F1 * K1; p += nth) {
        const int gg = p / K1, k = p - gg * K1;
        const float* w = pw1 + gg * K1;
        const double* gr = Gm + k * GS;
        double r0 = 0.0, r1 = 0.0, r2 = 0.0, r3 = 0.0;
        for (int l = 0; l < K1; l += 4) {
            r0 += gr[l] * (double)w[l];
            r1 += gr[l + 1] * (double)w[l + 1];
            r2 += gr[l + 2] * (double)w[l + 2];
            r3 += gr[l + 3] * (double)w[l + 3];
        }
        const double r = (r0 + r1) + (r2 + r3);
        const double wk = (double)w[k];
        pq[p] = wk * r;
        pm[p] = wk * S1[k];
        fa.stats[p] = r;                                   // fin5: (G w1)[k]
        if (gg == 0) fa.stats[F1 * K1 + k] = S1[k];        // fin5: S1[k]
    }
    __syncthreads();
    // BN1 moments from the quadratic forms w^T G w and w^T S1 (a filter per thread)
    const double n1 = (double)g.Bn * C * g.T;
    if (tid < F1) {
        const int gg = tid;
        double q0 = 0.0, q1 = 0.0, m0 = 0.0, m1 = 0.0;
        for (int k = 0; k < K1; k += 2) {
            q0 += pq[gg * K1 + k]; q1 += pq[gg * K1 + k + 1];
            m0 += pm[gg * K1 + k]; m1 += pm[gg * K1 + k + 1];
        }
        const double q = q0 + q1, m = m0 + m1;
        const double mu = m / n1;
        const double var = fmax(q / n1 - mu * mu, 0.0);   // E[u^2] - mu^2: never below 0
        const double inv = 1.0 / sqrt(var + (double)g.eps);
        const double a1 = (double)pg1[gg] * inv;
        const double c1 = (double)pb1[gg] - a1 * mu;
        a1s[gg] = a1; c1s[gg] = c1;
        fa.coef[CF_A1 * CSTR + gg] = (float)a1;
        fa.coef[CF_C1 * CSTR + gg] = (float)c1;
        fa.coef[CF_INV1 * CSTR + gg] = (float)inv;
        fa.coef[CF_MU1 * CSTR + gg] = (float)mu;
        if (fa.update_running) {
            const double mom = g.mom;
            fa.bn[gg] = (float)((1.0 - mom) * (double)pbn[gg] + mom * mu);
            fa.bn[F1 + gg] = (float)((1.0 - mom) * (double)pbn[F1 + gg] + mom * var * n1 / (n1 - 1.0));
        }
    }
    __syncthreads();
    TRACE_FS(g, fa.tpass, 5);
    const double n2 = (double)g.Bn * g.T;
    if (tid < F2) {
        const int o = tid, gg = o / g.D;
        double W = 0.0;
        for (int c = 0; c < C; ++c) W += (double)pws[o * C + c];
        const double mv = Sv[o] / n2;
        const double varv = fmax(Sv2[o] / n2 - mv * mv, 0.0);
        const double mu2 = a1s[gg] * mv + c1s[gg] * W;
        const double var2 = a1s[gg] * a1s[gg] * varv;
        const double inv2 = 1.0 / sqrt(var2 + (double)g.eps);
        const double alpha = a1s[gg] * inv2;
        fa.coef[CF_AL2 * CSTR + o] = (float)alpha;
        fa.coef[CF_BE2 * CSTR + o] = (float)(-alpha * mv);
        fa.coef[CF_INV2 * CSTR + o] = (float)inv2;
        fa.coef[CF_W * CSTR + o] = (float)W;
        if (fa.update_running) {
            const double mom = g.mom;
            float* rm2 = fa.bn + 2 * F1;
            rm2[o] = (float)((1.0 - mom) * (double)pbn[2 * F1 + o] + mom * mu2);
            rm2[F2 + o] = (float)((1.0 - mom) * (double)pbn[2 * F1 + F2 + o] + mom * var2 * n2 / (n2 - 1.0));
        }
    }
}

template <int K1>
__device__ __forceinline__ void fin1(const Geo& g, const float* prm, const double* sums, double* scr, const FinArgs& fa) {
    Fin1Stage st;
    fin1_body<K1, false>(g, prm, sums, scr, fa, st);
}

// after pass B: BN3 (model.py:71) batch statistics
__device__ void fin2(const Geo& g, const double* sums, const FinArgs& fa) {
    const int j = threadIdx.x;
    if (j >= g.F2) return;
    const double n3 = (double)g.Bn * g.T1;
    const double mu = sums[j] / n3;
    const double var = fmax(sums[g.F2 + j] / n3 - mu * mu, 0.0);
    fa.coef[CF_MU3 * CSTR + j] = (float)mu;
    fa.coef[CF_INV3 * CSTR + j] = (float)(1.0 / sqrt(var + (double)g.eps));
    float* rm3 = fa.bn + 2 * g.F1 + 2 * g.F2;
    if (fa.update_running) bn_running(rm3 + j, rm3 + g.F2 + j, mu, var, n3, g.mom);
    // BatchNorm2d.num_batches_tracked += 1 for the three BN layers (train-mode forward)
    if (fa.update_running && fa.nbt && j < 3) fa.nbt[j] += 1;
}

// after pass C: classifier grads (+ clamp, model.py:84), BN3 grads and backward constants
__device__ void fin3(const Geo& g, const float* prm, const double* sums, const FinArgs& fa) {
    const int tid = threadIdx.x;
    const int n4 = NCLS * g.NF;
    for (int p = tid; p < n4; p += (int)blockDim.x) {
        const float v = (float)sums[p];
        fa.grads[g.o_Wfc + p] = g.noclamp ? v : fminf(fmaxf(v, -0.25f), 0.25f);
    }
    if (tid < NCLS) fa.grads[g.o_bfc + tid] = (float)sums[n4 + tid];
    if (tid < g.F2) {
        const int j = tid;
        const double sdz = sums[n4 + NCLS + j], sdzx = sums[n4 + NCLS + g.F2 + j];
        fa.grads[g.o_b3 + j] = (float)sdz;
        fa.grads[g.o_g3 + j] = (float)sdzx;
        const double n3 = (double)g.Bn * g.T1;
        const double A = (double)prm[g.o_g3 + j] * (double)fa.coef[CF_INV3 * CSTR + j];
        fa.coef[CF_A3 * CSTR + j] = (float)A;
        fa.coef[CF_B3 * CSTR + j] = (float)(-A * sdz / n3);
        fa.coef[CF_C3 * CSTR + j] = (float)(-A * sdzx / n3);
    }
    if (tid == 0 && fa.ce) {
        const float l = (float)(sums[n4 + NCLS + 2 * g.F2] / (double)g.Bn);
        fa.coef[CF_LOSS * CSTR] = l;
        if (fa.loss) *fa.loss = l;
    }
}

// after pass D: block_2 grads, BN2 grads and the dy2 constants
__device__ void fin4(const Geo& g, const float* prm, const double* sums, const FinArgs& fa) {
    const int tid = threadIdx.x;
    for (int p = tid; p < g.F2 * g.F2; p += (int)blockDim.x) fa.grads[g.o_W3 + p] = (float)sums[p];
    for (int p = tid; p < g.F2 * 16; p += (int)blockDim.x) fa.grads[g.o_w2 + p] = (float)sums[g.F2 * g.F2 + p];
    if (tid < g.F2) {
        const int o = tid;
        const double sdz = sums[g.F2 * g.F2 + 16 * g.F2 + o];
        const double sdzx = sums[g.F2 * g.F2 + 17 * g.F2 + o];
        fa.grads[g.o_b2 + o] = (float)sdz;
        fa.grads[g.o_g2 + o] = (float)sdzx;
        const double n2 = (double)g.Bn * g.T;
        const double A = (double)prm[g.o_g2 + o] * (double)fa.coef[CF_INV2 * CSTR + o];
        fa.coef[CF_AO * CSTR + o] = (float)A;
        fa.coef[CF_BO * CSTR + o] = (float)(-A * sdz / n2);
        fa.coef[CF_CO * CSTR + o] = (float)(-A * sdzx / n2);
    }
}

// one torch.optim.Adam element update (weight_decay=0, amsgrad=False): torch/optim/adam.py
// :457,476,531-547 (single-tensor path)
// Contraction off: the fused (fin5) and standalone (k_adam) instances must round identically, so
// the data-parallel path is bit-identical to the fused single-device step.
__device__ __forceinline__ void adam_elem(float* p, float g, float* m, float* v, float b1, float b2,
                                          float step_size, float bc2s, float eps) {
#pragma clang fp contract(off)
    const float mi = *m + (1.f - b1) * (g - *m);
    const float vi = b2 * *v + (1.f - b2) * g * g;
    *m = mi; *v = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    *p = *p - step_size * (mi / denom);
}

// Adam step size and sqrt(bias correction 2) of step s (torch/optim/adam.py single-tensor path)
__device__ __forceinline__ void adam_scalars(const FinArgs& fa, int s, float& step_size, float& bc2s) {
    step_size = (float)((double)fa.lr / (1.0 - pow((double)fa.b1, (double)s)));
    bc2s = (float)sqrt(1.0 - pow((double)fa.b2, (double)s));
}

// The parameters pass E never reads -- [o_w2, nparam): block-2 depthwise and pointwise weights, BN3,
// the classifier -- have their final gradients after pass D (fin3, fin4).  Pass E's workgroups take
// their Adam update, a slice each: the narrow pass E's workgroups once they have lost the reduction
// ticket (while the winner reduces; the winner's own slice rides in fin5's staged batch), the wide
// pass E's in its prologue.  fin5 then updates [0, o_w2).  The same element update with the same
// step: bit-identical.  Not for a deferred (synchronised-BN) pass, whose k_fin runs the whole update.
__device__ __forceinline__ bool adam_early(const Geo& g, const FinArgs& fa) {
    return fa.adam_m != nullptr && !g.defer;
}
__device__ __forceinline__ void adam_slice_range(const Geo& g, int part, int nparts, int& i0, int& i1) {
    const int lo = g.o_w2, per = (g.nparam - lo + nparts - 1) / nparts;
    i0 = min(g.nparam, lo + part * per);
    i1 = min(g.nparam, i0 + per);
}
// pass E's workgroup 0 computes this step's Adam scalars in its prologue and publishes them in the
// coefficient block (CF_ADAM), so the double-precision pow()s are off the finalize's critical path
__device__ __forceinline__ void adam_scalars_publish(const Geo& g, const FinArgs& fa) {
    if (blockIdx.x != 0 || threadIdx.x != 0 || !adam_early(g, fa)) return;
    float step_size, bc2s;
    adam_scalars(fa, ldc(fa.step) + 1, step_size, bc2s);
    pub(fa.coef + CF_ADAM * CSTR, step_size);
    pub(fa.coef + CF_ADAM * CSTR + 1, bc2s);
}
// step0: the device step counter as this workgroup read it BEFORE taking its reduction ticket.  fin5
// (run by the ticket winner) advances *fa.step, and nothing orders a loser's later read against that
// write: a loser descheduled past fin5 would apply the bias correction of the step after.  The wide
// pass E calls this in its prologue (its finalize is a later launch), the narrow one passes the value
// it read in its prologue.
__device__ __forceinline__ int adam_step0(const Geo& g, const FinArgs& fa) {
    return adam_early(g, fa) ? ldc(fa.step) : 0;        // scalar load: not behind the prologue's DMAs
}
__device__ void adam_slice(const Geo& g, const FinArgs& fa, int part, int nparts, int step0) {
    if (!adam_early(g, fa)) return;
    int i0, i1;
    adam_slice_range(g, part, nparts, i0, i1);
    const int i = i0 + (int)threadIdx.x;
    if (i0 + (int)(threadIdx.x & ~63u) >= i1) return;    // waves without an element (wave-uniform)
    float step_size, bc2s;
    adam_scalars(fa, step0 + 1, step_size, bc2s);
    for (int k = i; k < i1; k += (int)blockDim.x) {
        float pp = fa.params[k], mm = fa.adam_m[k], vv = fa.adam_v[k];
        adam_elem(&pp, fa.grads[k], &mm, &vv, fa.b1, fa.b2, step_size, bc2s, fa.eps);
        fa.params[k] = pp; fa.adam_m[k] = mm; fa.adam_v[k] = vv;
    }
}

// after pass E: spatial grad (+ clamp, model.py:44), BN1 grads, temporal-conv grad; then Adam
constexpr int APT = 8;            // Adam elements per finalize thread: nparam <= APT * blockDim
// fin5's one batch of global loads -- statistics, coefficients, the Adam state of its elements --
// as registers (Fin5Stage).  k_pass_e issues it in every workgroup BEFORE the reduction ticket, so the
// winner starts fin5 with its inputs in hand instead of one more global round trip on the critical path
// (2.3 µs in the r4f timeline); the losers drop it.  Nothing read here changes during the pass: the
// statistics and coefficients are the earlier finalizes', [0, o_w2) and the own slice are written only
// by this finalize, the gradients >= o_g2 by fin3 / fin4, the step counter by fin5 at its very end.
// own_slice >= 0: this workgroup's adam_slice (of gridDim.x) joins the staged Adam elements
struct Fin5Stage {
    Stage<3, double> s0;
    Stage<3, float> s2;
    float ap[APT], am[APT], av[APT], ag[APT];
    int step0;
};
__device__ __forceinline__ void fin5_load(const Geo& g, const FinArgs& fa, int own_slice, Fin5Stage& st) {
    const int nth = blockDim.x, tid = threadIdx.x;
    const bool adam = fa.adam_m != nullptr;
    const bool early = adam_early(g, fa);
    const int na = early ? g.o_w2 : g.nparam;
    int si0 = 0, si1 = 0;
    if (early && own_slice >= 0) adam_slice_range(g, own_slice, gridDim.x, si0, si1);
    const int ne = na + (si1 - si0);
    auto pidx = [&](int e) { return e < na ? e : si0 + (e - na); };
    st.s0.load(fa.stats, g.F1 * g.K1 + g.K1);
    st.s2.load(fa.coef, CF_COUNT * CSTR);
    if (adam) {   // parameters, moments and the earlier finalizes' gradients (indices >= o_g2)
        const int last = ne - 1;
#pragma unroll
        for (int j = 0; j < APT; ++j) {
            if (nth * j >= ne) break;     // block-uniform: only the batches that hold elements
            const int i = pidx(min(tid + nth * j, last));
            st.ap[j] = fa.params[i]; st.am[j] = fa.adam_m[i]; st.av[j] = fa.adam_v[i]; st.ag[j] = fa.grads[i];
        }
    }
    st.step0 = adam ? *fa.step : 0;
}
// PRE: st already holds fin5_load's batch (k_pass_e); otherwise fin5 loads it here
template <bool PRE>
__device__ __forceinline__ void fin5_body(const Geo& g, const float* prm, const double* sums, double* scr,
                                          const FinArgs& fa, int own_slice, Fin5Stage& st) {
    const int tid = threadIdx.x, nth = blockDim.x, K1 = g.K1, F1 = g.F1;
    double* Gw = scr;                 // (G w1)[filter][tap] (F1*K1) + S1 (K1), fin1's, from fa.stats
    double* S1 = Gw + F1 * K1;
    double* db1s = S1 + K1;           // 64
    double* dg1s = db1s + 64;         // 64
    float* cf = (float*)(dg1s + 64);             // coefficient block [CF_COUNT][CSTR]
    float* gL = cf + CF_COUNT * CSTR;            // [0, o_g2): the gradients this finalize computes
    const double* Q = sums;
    const double* Xm = sums + g.QR * K1;
    const double* Sdy = Xm + g.F2 * g.C;
    const double* Sdyv = Sdy + g.F2;
    const bool adam = fa.adam_m != nullptr;
    const bool early = adam_early(g, fa);
    const int na = early ? g.o_w2 : g.nparam;     // [o_w2, nparam): pass E's workgroups (adam_slice)
    int si0 = 0, si1 = 0;                         // + this workgroup's own slice, as elements na ...
    if (early && own_slice >= 0) adam_slice_range(g, own_slice, gridDim.x, si0, si1);
    const int ne = na + (si1 - si0);
    auto pidx = [&](int e) { return e < na ? e : si0 + (e - na); };
    if constexpr (!PRE) fin5_load(g, fa, own_slice, st);
    float* const ap = st.ap;
    float* const am = st.am;
    float* const av = st.av;
    const float* const ag = st.ag;
    const int step0 = st.step0;
    float es0 = 0.f, es1 = 0.f;
    if (early) {                      // adam_scalars_publish (pass E, workgroup 0), after the ticket
        es0 = ld_pub(fa.coef + CF_ADAM * CSTR);
        es1 = ld_pub(fa.coef + CF_ADAM * CSTR + 1);
    }
    st.s0.store(Gw, F1 * K1 + K1);
    st.s2.store(cf, CF_COUNT * CSTR);
    __syncthreads();
    TRACE_FS(g, fa.tpass, 4);
    for (int p = tid; p < g.F2 * g.C; p += nth) {
        const int o = p / g.C, gg = o / g.D;
        const double v = (double)cf[CF_A1 * CSTR + gg] * Xm[p] + (double)cf[CF_C1 * CSTR + gg] * Sdy[o];
        const float vf = g.noclamp ? (float)v : fminf(fmaxf((float)v, -1.0f), 1.0f);
        fa.grads[g.o_ws + p] = vf;
        gL[g.o_ws + p] = vf;
    }
    if (tid < F1) {
        const int gg = tid;
        double db1 = 0.0, dyu = 0.0;
        for (int o = gg * g.D; o < (gg + 1) * g.D; ++o) {
            db1 += (double)cf[CF_W * CSTR + o] * Sdy[o];
            dyu += Sdyv[o];
        }
        const double inv1 = cf[CF_INV1 * CSTR + gg], mu1 = cf[CF_MU1 * CSTR + gg];
        const double dg1 = inv1 * (dyu - mu1 * db1);
        db1s[gg] = db1; dg1s[gg] = dg1;
        fa.grads[g.o_b1 + gg] = (float)db1;
        fa.grads[g.o_g1 + gg] = (float)dg1;
        gL[g.o_b1 + gg] = (float)db1;
        gL[g.o_g1 + gg] = (float)dg1;
    }
    __syncthreads();
    TRACE_FS(g, fa.tpass, 5);
    const double n1 = (double)g.Bn * g.C * g.T;
    for (int p = tid; p < F1 * K1; p += nth) {
        const int gg = p / K1, k = p - gg * K1;
        double qg = 0.0;
        if (g.QR == F1) qg = Q[gg * K1 + k];           // rows of a group summed in pass E
        else for (int o = gg * g.D; o < (gg + 1) * g.D; ++o) qg += Q[o * K1 + k];
        const double ux = Gw[p];                       // (G w1)[k], fin1's (same w1: Adam runs after)
        const double inv1 = cf[CF_INV1 * CSTR + gg], mu1 = cf[CF_MU1 * CSTR + gg];
        const double xhx = inv1 * (ux - mu1 * S1[k]);
        const double a1 = cf[CF_A1 * CSTR + gg];
        const double v = a1 * (qg - db1s[gg] / n1 * S1[k] - dg1s[gg] / n1 * xhx);
        fa.grads[g.o_w1 + p] = (float)v;
        gL[g.o_w1 + p] = (float)v;
    }
    if (!adam) return;
    __syncthreads();                  // gL complete
    TRACE_FS(g, fa.tpass, 6);
    const int s = step0 + 1;
    float step_size, bc2s;
    if (early) {                      // adam_scalars_publish (pass E, workgroup 0): published in this launch
        step_size = es0;
        bc2s = es1;
    } else {
        adam_scalars(fa, s, step_size, bc2s);
    }
#pragma unroll
    for (int j = 0; j < APT; ++j) {
        const int e = tid + nth * j;
        if (e < ne) {
            const int i = pidx(e);
            const float gr = i < g.o_g2 ? gL[i] : ag[j];
            adam_elem(&ap[j], gr, &am[j], &av[j], fa.b1, fa.b2, step_size, bc2s, fa.eps);
            fa.params[i] = ap[j]; fa.adam_m[i] = am[j]; fa.adam_v[i] = av[j];
        }
    }
    // parameters beyond the staged block (large models, e.g. EEGNet-16,4 at 64 x 512: 14,116)
    for (int e = tid + nth * APT; e < ne; e += nth) {
        const int i = pidx(e);
        float pp = fa.params[i], mm = fa.adam_m[i], vv = fa.adam_v[i];
        const float gr = i < g.o_g2 ? gL[i] : fa.grads[i];
        adam_elem(&pp, gr, &mm, &vv, fa.b1, fa.b2, step_size, bc2s, fa.eps);
        fa.params[i] = pp; fa.adam_m[i] = mm; fa.adam_v[i] = vv;
    }
    if (tid == 0) *fa.step = s;
}
__device__ __forceinline__ void fin5(const Geo& g, const float* prm, const double* sums, double* scr,
                                     const FinArgs& fa, int own_slice = -1) {
    Fin5Stage st;
    fin5_body<false>(g, prm, sums, scr, fa, own_slice, st);
}

// One pass's finalize as its own one-workgroup launch (eegnet_train_stage: synchronised-BatchNorm data
// parallel).  The pass kernel ran with g.defer and left its sums in part2 row 0; the host all-reduced them.
__global__ __launch_bounds__(512) void k_fin(Geo g, const float* prm, FinArgs fa, int pass, int ncols) {
    extern __shared__ __attribute__((aligned(16))) double dfin[];
    double* S = dfin + 2;
    stage_pub<8>(S, fa.part2, ncols);
    __syncthreads();
    double* scr = dfin + tail_s_doubles(ncols);
    switch (pass) {
        case 0: if (g.K1 == 32) fin1<32>(g, prm, S, scr, fa); else fin1<64>(g, prm, S, scr, fa); break;
        case 1: fin2(g, S, fa); break;
        case 2: fin3(g, prm, S, fa); break;
        case 3: fin4(g, prm, S, fa); break;
        default: fin5(g, prm, S, scr, fa); break;
    }
}

// ================================================================================================
// Column-parallel tail for passes with wide partial rows (cfg5 EEGNet-16,4: passes C, D, E carry
// 4-6 K columns per workgroup row).  The in-kernel two-level reduction funnels every column through
// one workgroup at the top (ngrp x ncols doubles, ~1 MB at cfg5: tens of microseconds); here the pass
// kernel only publishes its rows and NB = ceil(ncols / 64) workgroups each sum all rows of 64
// columns in fp64 in a fixed row order (four row phases, combined in phase order), publish the
// totals, and the last of them (ticket) stages the totals into LDS and runs the pass's finalize.
// ================================================================================================
constexpr int NTCT = 1024;        // threads of k_coltail: 64 columns x 16 row phases
template <int FIN, bool SPEC = false>
__global__ __launch_bounds__(NTCT) void k_coltail(Geo gin, const float* prm, const float* part, int nrows, int ncols,
                                                  FinArgs fa) {
    const Geo g = geo_w<SPEC>(gin);
    extern __shared__ __attribute__((aligned(16))) double dsmt[];
    constexpr int NPH = NTCT / 64, NB8 = 16;               // row phases; loads in flight per thread
    const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
    const int c = blockIdx.x * 64 + lane;
    double* ph = dsmt + 2;                                 // [NPH][64] row-phase partials
    double a = 0.0;
    if (c < ncols) {
        for (int r0 = q; r0 < nrows; r0 += NPH * NB8) {
            float v[NB8];
#pragma unroll
            for (int j = 0; j < NB8; ++j) v[j] = ld_pub(part + (size_t)min(r0 + NPH * j, nrows - 1) * ncols + c);
#pragma unroll
            for (int j = 0; j < NB8; ++j) a += r0 + NPH * j < nrows ? (double)v[j] : 0.0;
        }
    }
    ph[q * 64 + lane] = a;
    __syncthreads();
    if (q == 0 && c < ncols) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < NPH; ++k) t += ph[k * 64 + lane];
        pub(fa.part2 + c, t);
    }
    if (!take_ticket(fa.cnt + (NCNT - 1), gridDim.x, (int*)dsmt)) return;
    double* S = dsmt + 2;
    stage_pub<8>(S, fa.part2, ncols);
    if (tid == 0) __hip_atomic_store(fa.cnt + (NCNT - 1), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if constexpr (FIN == 3) fin3(g, prm, S, fa);
    else if constexpr (FIN == 4) fin4(g, prm, S, fa);
    else fin5(g, prm, S, dsmt + tail_s_doubles(ncols), fa);
}

// torch.optim.Adam (weight_decay=0, amsgrad=False): torch/optim/adam.py:457,476,531-547
__global__ __launch_bounds__(256) void k_adam(int64_t n, float* __restrict__ p, const float* __restrict__ gr,
                                             float* __restrict__ m, float* __restrict__ v,
                                             int32_t* __restrict__ step, float lr, float b1, float b2,
                                             float eps) {
    const int s = *step + 1;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const float step_size = (float)((double)lr / (1.0 - pow((double)b1, (double)s)));
        const float bc2s = (float)sqrt(1.0 - pow((double)b2, (double)s));
        adam_elem(p + i, gr[i], m + i, v + i, b1, b2, step_size, bc2s, eps);
    }
}

__global__ void k_step_inc(int32_t* step) { if (threadIdx.x == 0) *step += 1; }

// the two gradient hooks of model.py:44 and model.py:84, applied to a flat grad buffer
__global__ __launch_bounds__(256) void k_clamp(Geo g, float* __restrict__ grads) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < g.F2 * g.C) grads[g.o_ws + i] = fminf(fmaxf(grads[g.o_ws + i], -1.0f), 1.0f);
    if (i < NCLS * g.NF) grads[g.o_Wfc + i] = fminf(fmaxf(grads[g.o_Wfc + i], -0.25f), 0.25f);
}

}  // namespace eeg
