// dependent-chain latency and independent-stream throughput of single instructions on gfx950
#include <hip/hip_runtime.h>
#include <stdio.h>
#define N 64
__global__ void kern(unsigned long long *out, float fin, double din, int iin) {
  __shared__ int lds[1024];
  __shared__ double ldd[1024];
  const int tid = threadIdx.x;
  for (int i = tid; i < 1024; i += blockDim.x) { lds[i] = (i * 5 + 3) & 1023; ldd[i] = i; }
  __syncthreads();
  unsigned long long t0, t1; int slot = 0;
  auto rec = [&](unsigned long long d) { if (tid == 0) out[blockIdx.x * 32 + slot] = d; slot++; };
  // 1 fp32 fma dependent
  float f = fin + tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++) f = __builtin_fmaf(f, 1.0001f, 0.5f);
  asm volatile("" :: "v"(f)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 2 fp32 fma 8 independent chains
  float g[8]; for (int k = 0; k < 8; k++) g[k] = fin + k + tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) g[k] = __builtin_fmaf(g[k], 1.0001f, 0.5f);
  for (int k = 0; k < 8; k++) asm volatile("" :: "v"(g[k]));
  t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);  // per 8 ops
  // 3 fp64 fma dependent
  double d = din + tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++) d = __builtin_fma(d, 1.0000001, 0.5);
  asm volatile("" :: "v"(d)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 4 fp64 fma 8 independent
  double h[8]; for (int k = 0; k < 8; k++) h[k] = din + k + tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) h[k] = __builtin_fma(h[k], 1.0000001, 0.5);
  for (int k = 0; k < 8; k++) asm volatile("" :: "v"(h[k]));
  t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 5 int add dependent
  int a = iin + tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++) { a = a + (a >> 3); }
  asm volatile("" :: "v"(a)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);  // 2 ops each
  // 6 LDS dependent read
  int p = tid & 1023;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < N; i++) p = lds[p];
  asm volatile("" :: "v"(p)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 7 LDS broadcast (uniform address) read + fp compare accumulate (rank inner loop)
  double e = ldd[tid & 1023]; int r = 0;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int j = 0; j < N; j++) { double o = ldd[j]; r += (o < e) || (o == e && j < tid); }
  asm volatile("" :: "v"(r)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 8 ballot+popc chain (uniform)
  int cnt = 0;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int j = 0; j < N; j++) cnt += __popcll(__ballot(e > (double)j));
  asm volatile("" :: "s"(cnt)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 9 readlane chain
  int q = tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int j = 0; j < N; j++) q = __builtin_amdgcn_readlane(q + 1, j & 63);
  asm volatile("" :: "s"(q)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 10 DPP row_shr reduce chain
  int v = tid;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int j = 0; j < N; j++) v = v + __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
  asm volatile("" :: "v"(v)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 11 ds_read_b128 independent throughput (16 per iteration)
  int4 acc = make_int4(0,0,0,0);
  const int4* l4 = reinterpret_cast<const int4*>(lds);
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int j = 0; j < N; j++) { int4 x = l4[(tid + j * 64) & 255]; acc.x += x.x; acc.y ^= x.y; acc.z += x.z; acc.w ^= x.w; }
  asm volatile("" :: "v"(acc.x), "v"(acc.y), "v"(acc.z), "v"(acc.w)); t1 = __builtin_amdgcn_s_memtime(); rec(t1 - t0);
  // 12 barrier
  t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 16; j++) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime(); rec((t1 - t0) * 4);
}
int main() {
  unsigned long long *d; hipMalloc(&d, 256 * 32 * 8);
  unsigned long long h[32];
  const char* names[12] = {"f32 fma dep", "f32 fma x8 indep (per op)", "f64 fma dep", "f64 fma x8 indep (per op)",
     "int add+shr dep (per op)", "lds dep read", "rank iter (bcast ld+cmp)", "ballot+popc", "readlane chain",
     "dpp add chain", "ds_read_b128 stream (per read)", "barrier"};
  double div[12] = {N, 8.0*N, N, 8.0*N, 2.0*N, N, N, N, N, N, N, 64};
  for (int bs : {64, 256, 512, 1024}) {
    hipLaunchKernelGGL(kern, dim3(256), dim3(bs), 0, 0, d, 1.0f, 1.0, 1);
    hipLaunchKernelGGL(kern, dim3(256), dim3(bs), 0, 0, d, 1.0f, 1.0, 1);
    hipDeviceSynchronize();
    hipMemcpy(h, d, 32 * 8, hipMemcpyDeviceToHost);
    printf("waves/SIMD %.2f:", bs / 256.0);
    for (int i = 0; i < 12; i++) printf(" | %s %.1f", names[i], h[i] / div[i]);
    printf("\n");
  }
}
