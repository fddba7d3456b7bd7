// Checks the register-only lane exchanges the kernels use -- dsp_device.h's shfl_xor_k (32- and
// 64-bit; DPP, row_half_mirror + quad_perm for m = 4, permlane16/32 swaps) and lane_xor_f (the
// KNN screen's threshold exchange) -- against __shfl_xor (partner = lane ^ m) on gfx950.
//   hipcc -O3 --offload-arch=gfx950 -I../../include -I../../dsp-audioreclabs_amd/csrc perm_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "dsp_device.h"

__global__ void k(int *bad)
{
    const int lane = threadIdx.x & 63;
    const int v = lane * 7 + 3 + blockIdx.x * 977;
    const unsigned long long v64 = ((unsigned long long)(unsigned)(v * 31 + 5) << 32) | (unsigned)v;
    int b = 0;
#pragma unroll
    for (int s = 0; s < 6; s++) {
        const int m = 1 << s;
        if ((int)dsp::shfl_xor_k((unsigned)v, m, lane) != __shfl_xor(v, m, 64)) b |= 1 << s;
        const unsigned long long g = dsp::shfl_xor_k(v64, m, lane);
        const unsigned long long want = ((unsigned long long)(unsigned)__shfl_xor((int)(v64 >> 32), m, 64) << 32) |
                                        (unsigned)__shfl_xor((int)v64, m, 64);
        if (g != want) b |= 1 << (8 + s);
        if (m >= 16 && dsp::lane_xor_f((float)v, m, lane) != (float)__shfl_xor(v, m, 64)) b |= 1 << (16 + s);
    }
    atomicOr(bad, b);
}
int main()
{
    int *d, h = 0;
    (void)hipMalloc(&d, 4);
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k, dim3(8), dim3(256), 0, 0, d);
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("perm_check mismatch mask (bits 0-5: shfl_xor_k 32-bit, 8-13: 64-bit, 20-21: lane_xor_f; "
           "bit s = stride 1<<s): 0x%x %s\n", h, h ? "FAIL" : "OK");
    return h != 0;
}
