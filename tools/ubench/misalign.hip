// Streaming rate of 16-B buffer loads whose base is 2-byte aligned (clip-relative words of a
// packed int16 buffer) against 16-B aligned ones, on gfx950.  Each wave streams consecutive
// 1 KiB chunks (lane l: bytes 16 l .. 16 l + 15 of the chunk) of its own region, 12 loads in
// flight per lane as the extraction kernel holds them; the byte offset of every region is `mis`.
// usage: misalign   (prints GB/s for mis = 0, 2, 6, 14 and a checksum test)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef short short8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(512) void stream_k(const int16_t *x, long region_bytes, int nreg, int mis,
                                                unsigned long long *out)
{
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int nw = (gridDim.x * blockDim.x) >> 6;
    long long s = 0;
    for (int r = wave; r < nreg; r += nw) {
        const char *base = (const char *)x + (long)r * region_bytes + mis;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)region_bytes, 0x00020000);
        for (int c0 = 0; c0 < region_bytes; c0 += 12 * 1024) {
            short8 v[12];
#pragma unroll
            for (int k = 0; k < 12; k++)
                v[k] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, c0 + 1024 * k + 16 * lane, 0, 0));
#pragma unroll
            for (int k = 0; k < 12; k++)
#pragma unroll
                for (int e = 0; e < 8; e++) s += v[k][e];
        }
    }
    atomicAdd(out, (unsigned long long)s);
}

int main()
{
    const long region = 12 * 1024 * 8;  // 96 KiB per wave region (~ one clip)
    const int nreg = 40000;             // 3.9 GB
    const long n = region * nreg / 2 + 64;
    std::vector<int16_t> h(n);
    for (long i = 0; i < n; i++) h[i] = (int16_t)((i * 2654435761u) >> 17);
    int16_t *d;
    unsigned long long *o;
    hipMalloc(&d, n * 2);
    hipMalloc(&o, 8);
    hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int mis_list[4] = {0, 2, 6, 14};
    for (int rep = 0; rep < 2; rep++)
        for (int mi = 0; mi < 4; mi++) {
            const int mis = mis_list[mi];
            float best = 1e9;
            unsigned long long got = 0;
            for (int it = 0; it < 5; it++) {
                hipMemset(o, 0, 8);
                hipEventRecord(a);
                stream_k<<<512, 512>>>(d, region, nreg, mis, o);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
                hipMemcpy(&got, o, 8, hipMemcpyDeviceToHost);
            }
            unsigned long long want = 0;
            if (rep == 0) {
                for (long r = 0; r < nreg; r++)
                    for (long i = 0; i < region / 2; i++) want += (unsigned long long)(long long)h[r * region / 2 + mis / 2 + i];
            }
            printf("mis %2d B: %.3f ms  %.1f GB/s %s\n", mis, best, (double)region * nreg / best / 1e6,
                   rep == 0 ? (got == want ? "checksum OK" : "MISMATCH") : "");
        }
    return 0;
}
