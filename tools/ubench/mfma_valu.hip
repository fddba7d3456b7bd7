// Do v_mfma_f32_4x4x1f32 and plain VALU work overlap on one SIMD?  One 512-thread workgroup per CU
// (two waves per SIMD: waves w and w + 4 share SIMD w % 4); waves 0-3 run MFMA chains, waves 4-7 VALU
// chains (v_pk_fma_f32 or v_fma_f32), alone and together.  Overlap: "both" close to the max of the
// two alone; shared hardware: close to their sum.
//   hipcc -O3 --offload-arch=gfx950 mfma_valu.hip -o mfma_valu && ./mfma_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>  // bit 0: MFMA waves run, bit 1: VALU waves run, bit 2: VALU is packed
__global__ __launch_bounds__(512) void k(float *out, long long *cyc, int n)
{
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const long long t0 = __builtin_amdgcn_s_memtime();
    float r = 0.f;
    if (w < 4) {
        if (MODE & 1) {
            float a = 1.0f + l * 1e-7f, b = 0.999f;
            f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
            for (int i = 0; i < n; i++) {
                c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
                c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
                c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
                asm volatile("" : "+v"(a));
            }
            const f4 s = c0 + c1 + c2 + c3;
            r = s[0] + s[1] + s[2] + s[3];
        }
    } else if (MODE & 2) {
        if (MODE & 4) {
            f2 x[8];
            for (int j = 0; j < 8; j++) x[j] = (f2){1.0f + j, 2.0f + l};
            const f2 m = {0.9999f, 0.9998f}, ad = {1e-3f, 2e-3f};
            for (int i = 0; i < n; i++) {
#pragma unroll
                for (int j = 0; j < 8; j++) x[j] = __builtin_elementwise_fma(x[j], m, ad);
                asm volatile("" : "+v"(x[0]));
            }
            for (int j = 0; j < 8; j++) r += x[j].x + x[j].y;
        } else {
            float x[8];
            for (int j = 0; j < 8; j++) x[j] = 1.0f + j + l;
            for (int i = 0; i < n; i++) {
#pragma unroll
                for (int j = 0; j < 8; j++) x[j] = __builtin_fmaf(x[j], 0.9999f, 1e-3f);
                asm volatile("" : "+v"(x[0]));
            }
            for (int j = 0; j < 8; j++) r += x[j];
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 512 + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
double run(float *d, long long *dc, int n, int grid)
{
    long long h[1024];
    hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(512), 0, 0, d, dc, n);
    hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(512), 0, 0, d, dc, n);
    (void)hipMemcpy(h, dc, 8 * grid, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < grid; i++) s += h[i];
    return s / grid;
}

int main()
{
    float *d;
    long long *dc;
    const int grid = 256, n = 2048;
    (void)hipMalloc(&d, 512 * 4 * grid);
    (void)hipMalloc(&dc, 8 * 1024);
    const double m = run<1>(d, dc, n, grid);
    const double vp = run<2 | 4>(d, dc, n, grid), bp = run<1 | 2 | 4>(d, dc, n, grid);
    const double vs = run<2>(d, dc, n, grid), bs = run<1 | 2>(d, dc, n, grid);
    printf("cycles per iteration (4 MFMA 4x4x1f32 | 8 VALU fma):\n");
    printf("  MFMA waves alone      %.1f\n", m / n);
    printf("  v_pk_fma_f32 alone    %.1f   both %.1f   (sum %.1f, max %.1f)\n", vp / n, bp / n, (m + vp) / n,
           (m > vp ? m : vp) / n);
    printf("  v_fma_f32 alone       %.1f   both %.1f   (sum %.1f, max %.1f)\n", vs / n, bs / n, (m + vs) / n,
           (m > vs ? m : vs) / n);
    return 0;
}
