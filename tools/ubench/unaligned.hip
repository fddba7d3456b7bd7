// Unaligned 16-B buffer loads on gfx950: correctness and streaming rate.
//   (a) aligned: lane-contiguous 16-B loads
//   (b) hop layout: hop h, lane l loads 8 int16 at sample h*S + 7*l (2-byte aligned), uses 7
// Both reduce a checksum of the samples they own; the host checks it.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

typedef short short8 __attribute__((ext_vector_type(8)));

__global__ void aligned_k(const int16_t *x, long n8, unsigned long long *out)
{
    long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    long stride = (long)gridDim.x * blockDim.x;
    long long s = 0;
    for (; i < n8; i += stride) {
        short8 v = reinterpret_cast<const short8 *>(x)[i];
        for (int e = 0; e < 8; e++) s += v[e];
    }
    atomicAdd(out, (unsigned long long)s);
}

// one wave per hop group; S = 441, lanes 0..62 own 7 samples each
__global__ void hop_k(const int16_t *x, long nhop, unsigned long long *out, int S)
{
    const int lane = threadIdx.x & 63;
    long w = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
    long nw = ((long)gridDim.x * blockDim.x) >> 6;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t *>(x), 0, 0x7fffffff, 0x00020000);
    long long s = 0;
    for (long h = w; h < nhop; h += nw) {
        const int off = (int)((h * S + 7 * lane) * 2);
        short8 v = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        if (lane < 63)
            for (int e = 0; e < 7; e++) s += v[e];
    }
    atomicAdd(out, (unsigned long long)s);
}

int main()
{
    const int S = 441;
    const long nhop = 400000;  // 353 MB
    const long n = nhop * S;
    std::vector<int16_t> h(n + 64);
    unsigned long long ref = 0;
    for (long i = 0; i < n + 64; i++) h[i] = (int16_t)((i * 2654435761u) >> 17);
    for (long i = 0; i < n; i++) ref += (unsigned long long)(long long)h[i];
    int16_t *d;
    unsigned long long *o;
    hipMalloc(&d, (n + 64) * 2);
    hipMalloc(&o, 8);
    hipMemcpy(d, h.data(), (n + 64) * 2, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int which = 0; which < 2; which++) {
        float best = 1e9;
        unsigned long long got = 0;
        for (int rep = 0; rep < 10; rep++) {
            hipMemset(o, 0, 8);
            hipEventRecord(a);
            if (which == 0)
                aligned_k<<<4096, 256>>>(d, n / 8, o);
            else
                hop_k<<<4096, 256>>>(d, nhop, o, S);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (ms < best) best = ms;
            hipMemcpy(&got, o, 8, hipMemcpyDeviceToHost);
        }
        unsigned long long want = ref;
        if (which == 0) {  // aligned covers n/8*8 samples
            want = 0;
            for (long i = 0; i < (n / 8) * 8; i++) want += (unsigned long long)(long long)h[i];
        }
        printf("%s: %.3f ms  %.1f GB/s  checksum %s\n", which ? "hop-unaligned" : "aligned", best,
               n * 2 / best / 1e6, got == want ? "OK" : "MISMATCH");
    }
    return 0;
}
