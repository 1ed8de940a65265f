// Micro-benchmark: do f32 MFMA (v_mfma_f32_16x16x4_f32) and f32 VALU FMA share the FP32 pipe on gfx950?
// Waves 0..NM-1 of each 512-thread workgroup run MFMA chains, the rest VALU FMA chains.
// hipcc --offload-arch=gfx950 -O3 tools/pipe_share.hip -o tools/pipe_share
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void k_mix(const float* __restrict__ taps, float* out, int iters, int nm_waves,
                                             int valu_on, int mfma_on) {
    const int wave = threadIdx.x >> 6;
    float s = 0.f;
    if (wave < nm_waves) {
        if (mfma_on) {
            floatx4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
            float a = threadIdx.x * 1e-3f, b = 0.5f;
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
                    c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
                    c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
                }
                a += 1e-7f;
            }
            s = c0[0] + c1[1] + c2[2] + c3[3];
        }
    } else if (valu_on) {
        float acc[8], w[40];
#pragma unroll
        for (int i = 0; i < 40; ++i) w[i] = threadIdx.x * 0.001f + i;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const float t = taps[k];
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = fmaf(t, w[i + k], acc[i]);
            }
            w[0] += acc[0];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) s += acc[i];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static float run(int nm, int valu_on, int mfma_on, int iters) {
    float *taps, *out;
    hipMalloc(&taps, 64 * 4);
    hipMemset(taps, 0, 256);
    const int grid = 512;  // 2 workgroups per CU
    hipMalloc(&out, (size_t)grid * 512 * 4);
    k_mix<<<grid, 512>>>(taps, out, 10, nm, valu_on, mfma_on);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k_mix<<<grid, 512>>>(taps, out, iters, nm, valu_on, mfma_on);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    hipFree(taps); hipFree(out);
    return ms;
}

int main() {
    const int it = 4000;
    // per iteration: MFMA wave 32 MFMAs = 32768 MAC-lanes... report TFLOP/s of each part
    for (int nm : {4}) {
        const float tm = run(nm, 0, 1, it), tv = run(nm, 1, 0, it), tb = run(nm, 1, 1, it);
        const double mflop = 512.0 * nm * it * 32 * 16 * 16 * 4 * 2;     // grid * waves * MFMAs * MACs * 2
        const double vflop = 512.0 * (8 - nm) * 64 * it * 16 * 8 * 2;
        printf("MFMA waves %d/8: MFMA only %.3f ms (%.1f TF) | VALU only %.3f ms (%.1f TF) | both %.3f ms (%.1f TF total)\n",
               nm, tm, mflop / tm / 1e9, tv, vflop / tv / 1e9, tb, (mflop + vflop) / tb / 1e9);
    }
    return 0;
}
