// micro-benchmarks of basic latencies on gfx950 (cycles via s_memtime), one workgroup per CU
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned long long* out, int n, int nthreads_active) {
  __shared__ int lds[4096];
  __shared__ double ldd[512];
  int tid = threadIdx.x;
  for (int i = tid; i < 4096; i += blockDim.x) lds[i] = (i * 7 + 1) & 4095;
  for (int i = tid; i < 512; i += blockDim.x) ldd[i] = 1.0 + i;
  __syncthreads();
  unsigned long long t0, t1;
  // 1: dependent LDS read chain
  int p = tid & 4095;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) p = lds[p];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 0] = (t1 - t0);
  // 2: fp64 dependent add chain
  double x = ldd[tid & 511];
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = x * 1.0000001 + 0.5;
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 1] = (t1 - t0);
  // 3: fp64 division chain
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) x = 3.0 / (x + 1.0);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 2] = (t1 - t0);
  // 4: barriers
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) __syncthreads();
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 3] = (t1 - t0);
  // 5: independent LDS reads, 8 in flight then wait
  int acc = 0;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 8) {
    int a0 = lds[(tid + i) & 4095], a1 = lds[(tid + i + 64) & 4095], a2 = lds[(tid + i + 128) & 4095], a3 = lds[(tid + i + 192) & 4095];
    int a4 = lds[(tid + i + 256) & 4095], a5 = lds[(tid + i + 320) & 4095], a6 = lds[(tid + i + 384) & 4095], a7 = lds[(tid + i + 448) & 4095];
    acc += a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 4] = (t1 - t0);
  // 6: shfl_xor chain (ds_bpermute)
  int v = tid;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) v += __shfl_xor(v, 1 + (i & 31), 64);
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 5] = (t1 - t0);
  // 7: VALU int chain
  int w = tid;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i++) w = w * 3 + 1;
  t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x * 8 + 6] = (t1 - t0);
  if (tid == 0) out[blockIdx.x * 8 + 7] = (unsigned long long)(p + acc + v + w + (int)x);
}
int main() {
  unsigned long long* d; hipMalloc(&d, 256 * 8 * 8);
  unsigned long long h[8];
  const char* names[7] = {"lds dep read", "fp64 fma chain", "fp64 div chain", "syncthreads", "lds 8-indep (per read)", "shfl_xor chain", "int mad chain"};
  for (int bs : {64, 512, 1024}) {
    for (int grid : {1, 256}) {
      int n = 256;
      hipLaunchKernelGGL(k, dim3(grid), dim3(bs), 0, 0, d, n, bs);
      hipLaunchKernelGGL(k, dim3(grid), dim3(bs), 0, 0, d, n, bs);
      hipDeviceSynchronize();
      hipMemcpy(h, d, 64, hipMemcpyDeviceToHost);
      printf("block %4d grid %3d: ", bs, grid);
      for (int i = 0; i < 7; i++) printf("%s=%.1f  ", names[i], (double)h[i] / n);
      printf("\n");
    }
  }
  return 0;
}
