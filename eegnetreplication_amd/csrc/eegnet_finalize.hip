// eegnet_finalize.hip -- deterministic fp64 reductions, the one-workgroup finalize kernels (BN
// constants, running statistics, parameter gradients, clamps) and the Adam update.
// Included by eegnet_kernels.hip (one translation unit).

namespace eeg {

// ================================================================================================
// Deterministic fp64 column reduction of per-workgroup partial rows, stage 1: the rows are cut into
// RCH chunks; workgroup (column block, chunk) writes one fp64 partial per column.  Stage 2 (the
// RCH-way sum per column) is the prologue of the finalize kernel that consumes the sums.
// ================================================================================================
constexpr int RCH = 32;

__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ part, int nrows, int ncols,
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
    for (int c = threadIdx.x; c < ncols; c += 256) {
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
__global__ __launch_bounds__(256) void k_fin1(Geo g, const float* __restrict__ prm,
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
    const double* H = sums + K1 + 1;                 // head pairs (a <= b < R), a-major
    const double* Tl = H + g.nH;                     // tail pairs (u <= v < P), u-major
    const double* hs = Tl + g.nTl;                   // head sample sums [R]
    const double* ts = hs + g.R;                     // tail sample sums [P]
    const double* Sv = ts + g.P;
    const double* Sv2 = Sv + g.F2;
    // lag-Gram of the padded rows: G[k][k+d] = G0[d] + sum_{j<k} Ed[d][j], with
    // Ed[d][j] = sum_c X[T+j]X[T+j+d] - X[j]X[j+d] = Tl[j][j+d] (j+d < P) - H[j-P][j-P+d] (j >= P)
    if (tid < K1) {
        const int d = tid;
        double acc = G0[d];
        for (int k = 0; k + d < K1; ++k) {
            Gm[k * K1 + k + d] = acc;
            Gm[(k + d) * K1 + k] = acc;
            if (k < K1 - 1 - d) {
                const int j = k;
                double ed = 0.0;
                if (j + d < g.P) ed += Tl[j * g.P - j * (j - 1) / 2 + d];
                if (j >= g.P) {
                    const int a = j - g.P;
                    ed -= H[a * g.R - a * (a - 1) / 2 + d];
                }
                acc += ed;
            }
        }
    }
    if (tid == 0) {      // window sums S1[k] = S0 + sum_{j<k} (X[T+j] - X[j])
        double acc = S0;
        for (int k = 0; k < K1; ++k) {
            S1[k] = acc;
            if (k < K1 - 1) acc += (k < g.P ? ts[k] : 0.0) - (k >= g.P ? hs[k - g.P] : 0.0);
        }
    }
    __syncthreads();
    for (int i = tid; i < K1 * K1 + K1; i += 256) stats[i] = Gm[i];
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
__global__ __launch_bounds__(256) void k_fin2(Geo g, const double* __restrict__ part2,
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
__global__ __launch_bounds__(256) void k_fin3(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             float* __restrict__ coef, float* __restrict__ grads,
                                             float* __restrict__ loss, int ce) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nC, sums);
    const int tid = threadIdx.x;
    const int n4 = NCLS * g.NF;
    for (int p = tid; p < n4; p += 256) {
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
__global__ __launch_bounds__(256) void k_fin4(Geo g, const float* __restrict__ prm,
                                             const double* __restrict__ part2,
                                             float* __restrict__ coef, float* __restrict__ grads) {
    extern __shared__ __attribute__((aligned(16))) double sums[];
    reduce_chunks(part2, g.nD, sums);
    const int tid = threadIdx.x;
    for (int p = tid; p < g.F2 * g.F2; p += 256) grads[g.o_W3 + p] = (float)sums[p];
    for (int p = tid; p < g.F2 * 16; p += 256) grads[g.o_w2 + p] = (float)sums[g.F2 * g.F2 + p];
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
__global__ __launch_bounds__(256) void k_fin5(Geo g, const float* __restrict__ prm,
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
    for (int p = tid; p < g.F2 * g.C; p += 256) {
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
    for (int p = tid; p < g.F1 * K1; p += 256) {
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
__global__ __launch_bounds__(256) void k_adam(int64_t n, float* __restrict__ p, const float* __restrict__ gr,
                                             float* __restrict__ m, float* __restrict__ v,
                                             int32_t* __restrict__ step, float lr, float b1, float b2,
                                             float eps) {
    const int s = *step + 1;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
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
__global__ __launch_bounds__(256) void k_clamp(Geo g, float* __restrict__ grads) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < g.F2 * g.C) grads[g.o_ws + i] = fminf(fmaxf(grads[g.o_ws + i], -1.0f), 1.0f);
    if (i < NCLS * g.NF) grads[g.o_Wfc + i] = fminf(fmaxf(grads[g.o_Wfc + i], -0.25f), 0.25f);
}

}  // namespace eeg
