// Standalone check of the gfx950 cross-lane primitives the reductions rely on
// (v_permlane32_swap / v_permlane16_swap operand order, DPP row_ror).  hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(float* out) {
    const int l = threadIdx.x;
    const float a = 1000.f + l, b = 2000.f + l;
    auto p = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), false, false);
    auto q = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b), false, false);
    out[l] = __builtin_bit_cast(float, p[0]);
    out[64 + l] = __builtin_bit_cast(float, p[1]);
    out[128 + l] = __builtin_bit_cast(float, q[0]);
    out[192 + l] = __builtin_bit_cast(float, q[1]);
    out[256 + l] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x124, 0xF, 0xF, false));
    out[320 + l] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x138, 0xF, 0xF, true));  // wave_shr:1
    out[384 + l] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x130, 0xF, 0xF, true));  // wave_shl:1
    out[448 + l] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a), 0x114, 0xF, 0xF, true));  // row_shr:4
}
int main() {
    float* d; hipMalloc(&d, 512 * 4);
    k<<<1, 64>>>(d);
    float h[512]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[8] = {"p32.x", "p32.y", "p16.x", "p16.y", "ror4", "wshr1", "wshl1", "rshr4"};
    for (int r = 0; r < 8; ++r) {
        printf("%s:", nm[r]);
        for (int l = 0; l < 64; l += (r >= 5 ? 1 : 4)) printf(" %g", h[r * 64 + l]);
        printf("\n");
    }
    return 0;
}
