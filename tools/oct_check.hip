// Checks the octet cross-lane helpers of kad_engine.hip (DPP / ds_swizzle) against __shfl forms on one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false); }
template <int O> __device__ __forceinline__ uint32_t oct_xor(uint32_t v) {
    if constexpr (O == 1) return qdpp<0xB1>(v);
    else if constexpr (O == 2) return qdpp<0x4E>(v);
    else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
}
template <int O> __device__ __forceinline__ uint32_t oct_up(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 | O, 0xF, 0xF, true);
}
template <int O> __device__ __forceinline__ uint32_t oct_down(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 | O, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t oct_last(uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (0x07 << 5)); }
__global__ void k(uint32_t* out) {
    const uint32_t lane = threadIdx.x, g = lane & 7u, v = lane * 2654435761u + 7u;
    uint32_t r[10];
    r[0] = oct_xor<1>(v) == (uint32_t)__shfl_xor((int)v, 1, 8);
    r[1] = oct_xor<2>(v) == (uint32_t)__shfl_xor((int)v, 2, 8);
    r[2] = oct_xor<4>(v) == (uint32_t)__shfl_xor((int)v, 4, 8);
    const uint32_t u1 = oct_up<1>(v), u2 = oct_up<2>(v), u4 = oct_up<4>(v);
    const uint32_t d1 = oct_down<1>(v), d2 = oct_down<2>(v), d4 = oct_down<4>(v);
    const uint32_t s1 = __shfl_up((int)v, 1, 8), s2 = __shfl_up((int)v, 2, 8), s4 = __shfl_up((int)v, 4, 8);
    const uint32_t e1 = __shfl_down((int)v, 1, 8), e2 = __shfl_down((int)v, 2, 8), e4 = __shfl_down((int)v, 4, 8);
    r[3] = g < 1 || u1 == s1;
    r[4] = g < 2 || u2 == s2;
    r[5] = g < 4 || u4 == s4;
    r[6] = g + 1 > 7 || d1 == e1;
    r[7] = g + 2 > 7 || d2 == e2;
    r[8] = g + 4 > 7 || d4 == e4;
    r[9] = oct_last(v) == (uint32_t)__shfl((int)v, (int)((lane & ~7u) | 7u), 64);
    for (int i = 0; i < 10; i++) out[i * 64 + lane] = r[i];
}
int main() {
    uint32_t* d; hipMalloc(&d, 640 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    uint32_t h[640]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[10] = {"xor1", "xor2", "xor4", "up1", "up2", "up4", "down1", "down2", "down4", "last"};
    for (int i = 0; i < 10; i++) {
        int bad = 0; for (int l = 0; l < 64; l++) bad += h[i * 64 + l] == 0;
        printf("%s bad=%d\n", nm[i], bad);
    }
    return 0;
}
