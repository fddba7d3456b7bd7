// Range checking of a raw-buffer 16-B load that straddles num_records, with a 2-byte aligned
// base (clip-relative descriptors of a packed int16 buffer).  For num_records = 2n and a load at
// byte 16 v, prints which int16 of the vector come back (sample index or 0).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef short short8 __attribute__((ext_vector_type(8)));

__global__ void probe(const int16_t *x, int base_elems, int n, int v, short *out)
{
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(x + base_elems), 0, 2 * n, 0x00020000);
    short8 q = __builtin_bit_cast(short8, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * v, 0, 0));
    for (int e = 0; e < 8; e++) out[e] = q[e];
}

int main()
{
    int16_t h[256];
    for (int i = 0; i < 256; i++) h[i] = (int16_t)(1000 + i);
    int16_t *d;
    short *o;
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, 16);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    const int bases[3] = {0, 1, 3};
    for (int b = 0; b < 3; b++)
        for (int n = 9; n <= 16; n++) {
            probe<<<1, 1>>>(d, bases[b], n, 1, o);  // vector 1 = samples 8..15, the clip ends at n
            short r[8];
            hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
            printf("base %d n %2d :", bases[b], n);
            for (int e = 0; e < 8; e++) printf(" %5d", r[e] ? r[e] - 1000 - bases[b] : -1);
            printf("\n");
        }
    return 0;
}
