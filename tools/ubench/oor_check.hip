// Range-checked raw buffer loads (16 B) that straddle num_records, at 4-B and 2-B aligned
// offsets: which bytes come back (whole load zeroed, or only the out-of-range dwords)?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(const uint16_t *x, uint16_t *out)
{
    const int t = threadIdx.x;  // offset in bytes = 2 * t
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(x), 0, 40, 0x00020000);
    typedef uint16_t u8v __attribute__((ext_vector_type(8)));
    u8v v = __builtin_bit_cast(u8v, __builtin_amdgcn_raw_buffer_load_b128(rs, 2 * t, 0, 0));
    for (int e = 0; e < 8; e++) out[t * 8 + e] = v[e];
}

int main()
{
    uint16_t h[64];
    for (int i = 0; i < 64; i++) h[i] = (uint16_t)(100 + i);
    uint16_t *d, *o;
    hipMalloc(&d, 128);
    hipMalloc(&o, 32 * 16);
    hipMemcpy(d, h, 128, hipMemcpyHostToDevice);
    k<<<1, 24>>>(d, o);
    uint16_t r[24 * 8];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    printf("num_records = 40 bytes (samples 0..19 in range)\n");
    for (int t = 0; t < 24; t++) {
        printf("byte offset %2d:", 2 * t);
        for (int e = 0; e < 8; e++) printf(" %3d", r[t * 8 + e]);
        printf("\n");
    }
    return 0;
}
