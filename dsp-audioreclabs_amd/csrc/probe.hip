// probe.hip -- measurement kernels for bench.py (diagnostic library libdsp_probe.so, not part of
// the C ABI in include/dsp_audiorec.h): the HBM read and copy rates this box reaches, so the
// extraction's roofline can be stated against a measured peak beside the 8 TB/s spec
// ("Baselines per §8d").
//
// probe_read: every byte of a buffer read once with 16-B loads (the extraction's own access
// width), four loads in flight per thread, grid-stride over a persistent grid of 8 workgroups per
// CU; the XOR of what was read goes to one word so the loads cannot be dropped.
// probe_copy: the same walk storing what it read to a second buffer (read + write bytes).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int PT = 256;  // threads per workgroup
constexpr int UNR = 4;   // 16-B loads in flight per thread

__global__ __launch_bounds__(PT) void probe_read(const uint4 *__restrict__ src, int64_t n16, unsigned *out)
{
    const int64_t stride = (int64_t)gridDim.x * PT;
    uint4 acc = {0, 0, 0, 0};
    int64_t i = (int64_t)blockIdx.x * PT + threadIdx.x;
    for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNR; u++) {
            acc.x ^= v[u].x;
            acc.y ^= v[u].y;
            acc.z ^= v[u].z;
            acc.w ^= v[u].w;
        }
    }
    for (; i < n16; i += stride) {
        const uint4 v = src[i];
        acc.x ^= v.x;
        acc.y ^= v.y;
        acc.z ^= v.z;
        acc.w ^= v.w;
    }
    const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) out[0] = x;  // practically never true; keeps the loads
}

__global__ __launch_bounds__(PT) void probe_copy(const uint4 *__restrict__ src, uint4 *__restrict__ dst, int64_t n16)
{
    const int64_t stride = (int64_t)gridDim.x * PT;
    int64_t i = (int64_t)blockIdx.x * PT + threadIdx.x;
    for (; i + (UNR - 1) * stride < n16; i += UNR * stride) {
        uint4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < UNR; u++) dst[i + u * stride] = v[u];
    }
    for (; i < n16; i += stride) dst[i] = src[i];
}

int grid()
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return 8 * cus;
}

}  // namespace

// bytes: multiple of 16; src / dst 16-B aligned device pointers; out: one device word (scratch)
extern "C" int dsp_probe_read(const void *src, int64_t bytes, unsigned *out, void *stream)
{
    if (!src || !out || bytes < 16 || (bytes & 15) || ((uintptr_t)src & 15)) return 1;
    hipLaunchKernelGGL(probe_read, dim3(grid()), dim3(PT), 0, (hipStream_t)stream, (const uint4 *)src, bytes / 16, out);
    return hipGetLastError() == hipSuccess ? 0 : 1000;
}

extern "C" int dsp_probe_copy(const void *src, void *dst, int64_t bytes, void *stream)
{
    if (!src || !dst || bytes < 16 || (bytes & 15) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return 1;
    hipLaunchKernelGGL(probe_copy, dim3(grid()), dim3(PT), 0, (hipStream_t)stream, (const uint4 *)src, (uint4 *)dst,
                       bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : 1000;
}
