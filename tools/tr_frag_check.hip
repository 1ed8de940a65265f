// tools/tr_frag_check.hip -- checks tr_frag (eegnet_infer_bf16.hip) as the kernel uses it: a swizzled
// [64][TXc] bf16 image with img[r][t] = r + 64 * (t % 4) (exact in bf16), the fragment fed to the MFMA
// as A (m = t, k = r) against B = e_k (one k per pass), so D[m][0] recovers A[m][k].
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../eegnetreplication_amd/csrc/eegnet_common.h"
#include "../eegnetreplication_amd/csrc/eegnet_infer_bf16.hip"
using namespace eeg;
constexpr int R = 64, TXc = 512;
__global__ void k(float* out, int k0, int n0, int kk) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    for (int i = threadIdx.x; i < R * TXc; i += 64) {
        const int r = i / TXc, t = i % TXc;
        *reinterpret_cast<__bf16*>(sm + trimg_off(r, t >> 2, 2 * TXc) + 2 * (t & 3)) = (__bf16)(float)(r + 64 * (t % 4));
    }
    __syncthreads();
    const int l = threadIdx.x;
    bf16x8 a = tr_frag(sm, 2 * TXc, k0, n0, l);
    bf16x8 b;
    for (int j = 0; j < 8; ++j) b[j] = (__bf16)((8 * (l >> 4) + j == kk && (l & 15) == 0) ? 1.f : 0.f);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma_bf16(a, b, acc);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = acc[i];
}
int main() {
    float* d; float h[256];
    (void)hipMalloc(&d, 1024);
    int bad = 0, tot = 0;
    for (int k0 : {0, 32})
        for (int n0 : {0, 16, 496})
            for (int kk = 0; kk < 32; ++kk) {
                hipLaunchKernelGGL(k, dim3(1), dim3(64), R * TXc * 2, 0, d, k0, n0, kk);
                (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
                for (int l = 0; l < 64; ++l)
                    for (int i = 0; i < 4; ++i) {
                        if ((l & 15) != 0) continue;          // column n = 0 holds A[:, kk]
                        const int m = 4 * (l >> 4) + i, t = n0 + m, r = k0 + kk;
                        const float want = (float)(r + 64 * (t % 4));
                        ++tot;
                        if (h[l * 4 + i] != want && bad++ < 12)
                            printf("k0=%d n0=%d k=%d m=%d: got %g want %g\n", k0, n0, kk, m, h[l * 4 + i], want);
                    }
            }
    printf("tr_frag->mfma mismatches: %d of %d\n", bad, tot);
    return 0;
}
