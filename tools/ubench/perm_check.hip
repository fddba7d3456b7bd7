// checks register-only lane exchanges against __shfl_xor (partner = lane ^ m) on gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __forceinline__ int xchg(int v, int m, int lane)
{
    switch (m) {
    case 1: return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);
    case 2: return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);
    case 4: return __builtin_amdgcn_ds_swizzle(v, 0x101F);
    case 8: return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);
    case 16: { auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false); return (lane & 16) ? r[0] : r[1]; }
    default: { auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false); return (lane & 32) ? r[0] : r[1]; }
    }
}
__global__ void k(int *bad)
{
    const int lane = threadIdx.x & 63;
    const int v = lane * 7 + 3 + blockIdx.x;
    int b = 0;
    for (int s = 0; s < 6; s++) {
        const int m = 1 << s;
        int got;
        switch (s) {
        case 0: got = xchg(v, 1, lane); break;
        case 1: got = xchg(v, 2, lane); break;
        case 2: got = xchg(v, 4, lane); break;
        case 3: got = xchg(v, 8, lane); break;
        case 4: got = xchg(v, 16, lane); break;
        default: got = xchg(v, 32, lane); break;
        }
        if (got != __shfl_xor(v, m, 64)) b |= 1 << s;
    }
    atomicOr(bad, b);
}
int main()
{
    int *d, h = 0;
    hipMalloc(&d, 4);
    hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k, dim3(4), dim3(256), 0, 0, d);
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("mismatch mask (bit s = stride 1<<s): 0x%x\n", h);
    return 0;
}
