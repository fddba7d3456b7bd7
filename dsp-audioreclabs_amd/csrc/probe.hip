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

// probe_reread: the read walk in blocks of `blk` 16-B vectors (one workgroup per block, blocks
// b, b + G, ...), and after each block the vectors [off, off + len) of the workgroup's PREVIOUS
// block read again -- the extraction's access shape (a clip read whole, its crop re-read some
// microseconds later while other clips stream in).  Timed against probe_read over the same bytes,
// it shows whether such re-reads cost HBM time or are served on-die (L2 / Infinity Cache), which
// FETCH_SIZE cannot tell apart (MI355X_MICROARCH.md, HBM section).
__global__ __launch_bounds__(PT) void probe_reread(const uint4 *__restrict__ src, int64_t n16, int64_t blk, int64_t off,
                                                    int64_t len, unsigned *out)
{
    uint4 acc = {0, 0, 0, 0};
    const int64_t nblk = n16 / blk;
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint4 *p = src + b * blk;
#pragma unroll 8
        for (int64_t i = threadIdx.x; i < blk; i += PT) {
            const uint4 v = p[i];
            acc.x ^= v.x;
            acc.y ^= v.y;
            acc.z ^= v.z;
            acc.w ^= v.w;
        }
        if (b >= (int64_t)gridDim.x) {
            const uint4 *q = src + (b - gridDim.x) * blk + off;
#pragma unroll 8
            for (int64_t i = threadIdx.x; i < len; i += PT) {
                const uint4 v = q[i];
                acc.x ^= v.x;
                acc.y ^= v.y;
                acc.z ^= v.z;
                acc.w ^= v.w;
            }
        }
    }
    const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) out[0] = x;
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

// blk_bytes / off_bytes / len_bytes: multiples of 16 (off + len <= blk); grid: workgroups (0: 3 per CU, the extraction's)
extern "C" int dsp_probe_reread(const void *src, int64_t bytes, int64_t blk_bytes, int64_t off_bytes, int64_t len_bytes,
                                int grid_wgs, unsigned *out, void *stream)
{
    if (!src || !out || blk_bytes < 16 || ((blk_bytes | off_bytes | len_bytes) & 15) || off_bytes + len_bytes > blk_bytes ||
        bytes < blk_bytes || ((uintptr_t)src & 15))
        return 1;
    const int g = grid_wgs > 0 ? grid_wgs : 3 * (grid() / 8);
    hipLaunchKernelGGL(probe_reread, dim3(g), dim3(PT), 0, (hipStream_t)stream, (const uint4 *)src, bytes / 16,
                       blk_bytes / 16, off_bytes / 16, len_bytes / 16, out);
    return hipGetLastError() == hipSuccess ? 0 : 1000;
}
