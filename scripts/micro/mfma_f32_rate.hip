// Microbenchmark: v_mfma_f32_16x16x4_f32 / 32x32x2_f32 issue rate on MI355X
// for 1..4 independent accumulators per wave and 1..2 waves per SIMD.
// Prints cycles per MFMA per SIMD (s_memtime) and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void k16(float* out, int iters, long long* cyc) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int NACC>
__global__ void k32(float* out, int iters, long long* cyc) {
  f32x16 acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][5];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int nacc, int threads, int flop_per_mfma) {
  const int blocks = 256, iters = 2000;
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipMalloc(&cyc, sizeof(long long));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 10, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  const double n_mfma_wave = (double)iters * 8 * nacc;
  const int waves_per_simd = threads / 256;
  const double flops = (double)blocks * (threads / 64) * n_mfma_wave * flop_per_mfma;
  printf("%-10s nacc=%d waves/SIMD=%d  cycles/MFMA/wave=%.1f  per-SIMD=%.1f  %.1f TFLOP/s (%.3f ms)\n", name, nacc,
         waves_per_simd, c / n_mfma_wave, c / n_mfma_wave / waves_per_simd, flops / ms / 1e9, ms);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int threads : {256, 512}) {
    run("16x16x4", k16<1>, 1, threads, 2048);
    run("16x16x4", k16<2>, 2, threads, 2048);
    run("16x16x4", k16<4>, 4, threads, 2048);
    run("32x32x2", k32<1>, 1, threads, 4096);
    run("32x32x2", k32<2>, 2, threads, 4096);
  }
  return 0;
}
