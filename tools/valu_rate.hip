// Micro-benchmark: wave64 VALU issue rate on gfx950 for the FIR inner-loop shapes of the streaming
// passes (SGPR taps x VGPR window, independent accumulator chains), at a chosen occupancy.
// hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o tools/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int NACC>
__global__ __launch_bounds__(512) void k_fma(const float* __restrict__ taps, float* out, int iters) {
    float acc[NACC], w[NACC + 32];
#pragma unroll
    for (int i = 0; i < NACC + 32; ++i) w[i] = threadIdx.x * 0.001f + i;
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const float t = taps[k];
#pragma unroll
            for (int i = 0; i < NACC; ++i) acc[i] = fmaf(t, w[i + k], acc[i]);
        }
        w[0] += acc[0];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
// packed: NACC accumulators as NACC/2 float2, v_pk_fma_f32 with a broadcast tap
template <int NACC>
__global__ __launch_bounds__(512) void k_pkfma(const float* __restrict__ taps, float* out, int iters) {
    f2 acc[NACC / 2], w[(NACC + 32) / 2 + 1];
#pragma unroll
    for (int i = 0; i < (NACC + 32) / 2 + 1; ++i) w[i] = (f2){threadIdx.x * 0.001f + i, i + 0.5f};
#pragma unroll
    for (int i = 0; i < NACC / 2; ++i) acc[i] = (f2){0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 32; k += 2) {
            const float t = taps[k];
            const f2 tt = (f2){t, t};
#pragma unroll
            for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_elementwise_fma(tt, w[i + k / 2], acc[i]);
            const float t1 = taps[k + 1];
            const f2 tt1 = (f2){t1, t1};
#pragma unroll
            for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_elementwise_fma(tt1, w[i + k / 2 + 1], acc[i]);
        }
        w[0] += acc[0];
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC / 2; ++i) s += acc[i].x + acc[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
void run_pk(int wg_per_cu, int nthreads) {
    float *taps, *out;
    hipMalloc(&taps, 32 * 4);
    hipMemset(taps, 0, 128);
    const int grid = 256 * wg_per_cu;
    hipMalloc(&out, (size_t)grid * nthreads * 4);
    const int iters = 2000;
    k_pkfma<NACC><<<grid, nthreads>>>(taps, out, 10);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k_pkfma<NACC><<<grid, nthreads>>>(taps, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double fmas = (double)grid * nthreads * iters * 32 * NACC;
    printf("PK NACC=%2d waves/SIMD=%.2f: %.3f ms  %.1f TFLOP/s\n", NACC, (double)wg_per_cu * nthreads / 256, ms,
           2 * fmas / ms / 1e9);
    hipFree(taps); hipFree(out);
}

template <int NACC>
void run(int wg_per_cu, int nthreads) {
    float *taps, *out;
    hipMalloc(&taps, 32 * 4);
    hipMemset(taps, 0, 128);
    const int grid = 256 * wg_per_cu;
    hipMalloc(&out, (size_t)grid * nthreads * 4);
    const int iters = 2000;
    k_fma<NACC><<<grid, nthreads>>>(taps, out, 10);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k_fma<NACC><<<grid, nthreads>>>(taps, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double fmas = (double)grid * nthreads * iters * 32 * NACC;
    const double waves_per_simd = (double)wg_per_cu * nthreads / 64 / 4;
    const double instr_per_simd = (double)iters * 32 * NACC * waves_per_simd;
    printf("NACC=%2d waves/SIMD=%.0f: %.3f ms  %.1f TFLOP/s  %.2f ns per wave-instr per SIMD (%.2f cyc @2.4GHz)\n",
           NACC, waves_per_simd, ms, 2 * fmas / ms / 1e9, ms * 1e6 / instr_per_simd, ms * 1e6 / instr_per_simd * 2.4);
    hipFree(taps); hipFree(out);
}

int main() {
    run<4>(1, 64); run<4>(1, 256); run<4>(2, 512);
    run<8>(1, 64); run<8>(1, 256); run<8>(2, 512);
    run<16>(1, 256); run<16>(2, 512);
    run_pk<8>(1, 256); run_pk<8>(2, 512); run_pk<16>(1, 256); run_pk<16>(2, 512);
    return 0;
}
