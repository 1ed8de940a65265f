// tools/tr_check.hip -- pins the lane semantics of ds_read_b64_tr_b16 (gfx950): LDS holds
// img[r][c] = 256 r + c; lane 4q+p of each 16-lane group G supplies &img[4G + q][4p]; prints what each
// lane receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short shortx4 __attribute__((ext_vector_type(4)));
__global__ void k(unsigned short* out) {
    __shared__ __attribute__((aligned(16))) unsigned short img[16 * 64];
    for (int i = threadIdx.x; i < 16 * 64; i += 64) img[i] = (unsigned short)((i / 64) * 256 + (i % 64));
    __syncthreads();
    const int l = threadIdx.x, G = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const char* a = (const char*)&img[(4 * G + q) * 64 + 4 * p];
    shortx4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) shortx4*)(a));
    for (int j = 0; j < 4; ++j) out[l * 4 + j] = (unsigned short)v[j];
}
int main() {
    unsigned short* d; unsigned short h[256];
    hipMalloc(&d, 512);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int j = 0; j < 4; ++j) printf(" (r%d,c%d)", h[l * 4 + j] / 256, h[l * 4 + j] % 256);
        printf("\n");
    }
    return 0;
}
