// Load-only probes of the clip streaming pattern at 100k x 1 s clips (8.8 GB): what HBM rate a
// persistent grid reaches when a workgroup reads a whole 88 KB clip into registers per step.
//   probe <mode> : 0 = 512-thread WGs, 2/CU, 3 words (12 x 16 B) per thread per clip
//                  1 = 256-thread WGs, 4/CU, 6 words per thread per clip
//                  2 = 1024-thread WGs, 1/CU, 1.5 words
//                  3 = flat grid-stride 16-B reads over the whole buffer (copy-kernel peak)
//                  4 = mode 0 with an LDS reduction + barrier per clip (the kernel's skeleton)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
typedef short short8 __attribute__((ext_vector_type(8)));

template <int NT, int RW, bool BAR>
__global__ __launch_bounds__(NT) void clips(const int16_t *pcm, int B, int clip_bytes, int *out)
{
    __shared__ int red[NT / 64];
    int acc = 0;
    for (int i = blockIdx.x; i < B; i += gridDim.x) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)pcm + (size_t)i * clip_bytes), 0, clip_bytes, 0x00020000);
        short8 r[4 * RW];
#pragma unroll
        for (int w = 0; w < RW; w++)
#pragma unroll
            for (int k = 0; k < 4; k++)
                r[4 * w + k] = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, 64 * (w * NT + threadIdx.x) + 16 * k, 0, 0));
        int s = 0;
#pragma unroll
        for (int k = 0; k < 4 * RW; k++) s += r[k][0] ^ r[k][7];
        acc += s;
        if (BAR) {
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
            __syncthreads();
            acc += red[(threadIdx.x >> 6) ^ 1];
            __syncthreads();
        }
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

__global__ void flat(const int4 *p, size_t n, int *out)
{
    int acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int4 v = p[i];
        acc += v.x ^ v.w;
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int main(int argc, char **argv)
{
    const int B = 100000, N = 44100, cb = 2 * N + 8;  // 16-B aligned clip slots
    int dev = 0;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, dev);
    const int cus = prop.multiProcessorCount;
    int16_t *pcm;
    int *out;
    const size_t bytes = (size_t)B * cb;
    hipMalloc(&pcm, bytes);
    hipMalloc(&out, 4);
    hipMemset(pcm, 1, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 5; mode++) {
        float best = 1e9;
        for (int rep = 0; rep < 6; rep++) {
            hipEventRecord(a);
            switch (mode) {
            case 0: clips<512, 3, false><<<2 * cus, 512>>>(pcm, B, cb, out); break;
            case 1: clips<256, 6, false><<<4 * cus, 256>>>(pcm, B, cb, out); break;
            case 2: clips<1024, 2, false><<<cus, 1024>>>(pcm, B, cb, out); break;
            case 3: flat<<<8 * cus, 512>>>((const int4 *)pcm, bytes / 16, out); break;
            case 4: clips<512, 3, true><<<2 * cus, 512>>>(pcm, B, cb, out); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep > 0 && ms < best) best = ms;
        }
        printf("mode %d: %.3f ms  %.2f TB/s\n", mode, best, bytes / (best * 1e-3) / 1e12);
    }
    return 0;
}
