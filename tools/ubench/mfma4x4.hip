// v_mfma_f32_4x4x1f32 (16 blocks of 4x4, K = 1) on gfx950: operand / result lane layout, whether a
// step is one fused multiply-add, and the issue interval of dependent chains -- the facts the
// MFMA crop-frame sums (extract.hip R4, dsp_device.h) rely on.
//   hipcc -O3 --offload-arch=gfx950 mfma4x4.hip -o mfma4x4 && ./mfma4x4
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void layout(float *out)
{
    const int l = threadIdx.x;
    const float a = (float)(l + 1), b = (float)(1000 * (l + 1));
    f4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int v = 0; v < 4; v++) out[l * 4 + v] = c[v];
}

__global__ void fused(float *out, float a, float b, float c0)
{
    f4 c = {c0, c0, c0, c0};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    if (threadIdx.x == 0) out[0] = c[0];
}

template <int CH>
__global__ void chain(float *out, long long *cyc, int n)
{
    const int l = threadIdx.x & 63;
    float a = 1.0f + l * 1e-7f, b = 0.999f;
    f4 c[CH];
    for (int k = 0; k < CH; k++) c[k] = (f4){0.f, 0.f, 0.f, 0.f};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < CH; k++) c[k] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[k], 0, 0, 0);
        asm volatile("" : "+v"(a));
    }
    f4 s = c[0];
    for (int k = 1; k < CH; k++) s += c[k];
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    float *d, h[256];
    long long *dc, hc[1024];
    (void)hipMalloc(&d, 1 << 20);
    (void)hipMalloc(&dc, 8192);
    hipLaunchKernelGGL(layout, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
    // hypothesis: lane l supplies A[block l/4][row l%4] and B[block l/4][col l%4];
    // result VGPR v of lane l = D[block l/4][row v][col l%4] = A(4*(l/4)+v) * B(l)
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int v = 0; v < 4; v++) {
            const float want = (float)(4 * (l / 4) + v + 1) * (float)(1000 * (l + 1));
            if (h[l * 4 + v] != want) bad++;
        }
    printf("layout: %d of 256 results differ from the hypothesis %s\n", bad, bad ? "FAIL" : "OK");
    if (bad)
        for (int l = 0; l < 8; l++) printf("  lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
    const float a = 1.0f + ldexpf(1.f, -12), b = a;
    hipLaunchKernelGGL(fused, dim3(1), dim3(64), 0, 0, d, a, b, -1.0f);
    (void)hipMemcpy(h, d, 4, hipMemcpyDeviceToHost);
    printf("fused: mfma %.10e, fmaf %.10e, mul+add %.10e -> %s\n", h[0], fmaf(a, b, -1.f), (a * b) - 1.f,
           h[0] == fmaf(a, b, -1.f) ? "one rounding (fma)" : h[0] == (a * b) - 1.f ? "two roundings" : "other");
    const int n = 4096;
    for (int waves = 1; waves <= 2; waves++) {
        hipLaunchKernelGGL(chain<1>, dim3(256), dim3(64 * 4 * waves), 0, 0, d, dc, n);
        (void)hipMemcpy(hc, dc, 8 * 256, hipMemcpyDeviceToHost);
        printf("1 chain, %d wave/SIMD: %.2f cycles per MFMA per wave\n", waves, (double)hc[0] / n * 1.0);
        hipLaunchKernelGGL(chain<2>, dim3(256), dim3(64 * 4 * waves), 0, 0, d, dc, n);
        (void)hipMemcpy(hc, dc, 8 * 256, hipMemcpyDeviceToHost);
        printf("2 chains, %d wave/SIMD: %.2f cycles per MFMA per wave\n", waves, (double)hc[0] / (2.0 * n));
        hipLaunchKernelGGL(chain<4>, dim3(256), dim3(64 * 4 * waves), 0, 0, d, dc, n);
        (void)hipMemcpy(hc, dc, 8 * 256, hipMemcpyDeviceToHost);
        printf("4 chains, %d wave/SIMD: %.2f cycles per MFMA per wave\n", waves, (double)hc[0] / (4.0 * n));
    }
    printf("(s_memtime ticks; compare with the shader clock)\n");
    return bad != 0;
}
