// tools/mfma_bf16_check.hip -- pins v_mfma_f32_16x16x32_bf16 operand maps with exact integer data:
// A[m][k] = (k == m) + 2 (k == m + 16), B[k][n] = k + 32 n, so D[m][n] = B[m][n] + 2 B[m+16][n].
// Lane l supplies A[l&15][8(l>>4) + j] and B[8(l>>4) + j][l&15] (the assumed map).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, float* conv) {
    const int l = threadIdx.x, G = l >> 4, r = l & 15;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        const int kk = 8 * G + j;
        a[j] = (__bf16)(float)((kk == r) + 2 * (kk == r + 16));
        b[j] = (__bf16)(float)(kk + 32 * r);
    }
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = acc[i];
    conv[l] = (float)(__bf16)(0.0347f * (l + 1));
}
int main() {
    float *d, *c; float h[256], hc[64];
    (void)hipMalloc(&d, 1024); (void)hipMalloc(&c, 256);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, c);
    (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hc, c, 256, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
            const int m = 4 * (l >> 4) + i, n = l & 15;
            const float want = (m + 32 * n) + 2 * (m + 16 + 32 * n);
            if (h[l * 4 + i] != want && bad++ < 12) printf("D[%d][%d] = %g want %g\n", m, n, h[l * 4 + i], want);
        }
    printf("mismatches %d\n", bad);
    for (int l = 0; l < 4; ++l) printf("cvt %g -> %g\n", 0.0347f * (l + 1), hc[l]);
    return 0;
}
