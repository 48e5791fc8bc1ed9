// Microbenchmark: v_mfma_f32_16x16x4_f32 / 32x32x2_f32 issue rate on MI355X
// for 1..4 independent accumulators per wave and 1..2 waves per SIMD.
// Prints cycles per MFMA per SIMD (s_memtime) and TFLOP/s.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// random operands (a fixed operand understates the power draw: DVFS) and the
// in-kernel clock (s_memtime / s_memrealtime at 100 MHz) of block 0, wave 0
__device__ unsigned rng_u(unsigned& x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}
__device__ long long g_rt[2];
template <int NACC>
__global__ void k16(float* out, int iters, long long* cyc) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  unsigned x = 2463534242u + blockIdx.x * 977u + threadIdx.x * 131u;
  float a[8], b[8];
  for (int r = 0; r < 8; ++r) {
    a[r] = (float)(rng_u(x) & 0xffff) * 3.0e-5f - 1.f;
    b[r] = (float)(rng_u(x) & 0xffff) * 3.0e-5f - 1.f;
  }
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[r], b[(r + i) & 7], acc[i], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *cyc = t1 - t0;
    g_rt[0] = r1 - r0;
  }
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
  const int blocks = 256, iters = 20000;
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
  long long rt[2] = {0, 0};
  hipMemcpyFromSymbol(rt, HIP_SYMBOL(g_rt), sizeof(rt));
  const double ghz = rt[0] > 0 ? (double)c / (double)rt[0] * 0.1 : 0.0;
  printf("%-10s nacc=%d waves/SIMD=%d  cycles/MFMA/wave=%.1f  per-SIMD=%.1f  %.1f TFLOP/s (%.3f ms) clock %.2f GHz\n",
         name, nacc, waves_per_simd, c / n_mfma_wave, c / n_mfma_wave / waves_per_simd, flops / ms / 1e9, ms, ghz);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int threads : {256, 512}) {
    run("16x16x4", k16<1>, 1, threads, 2048);
    run("16x16x4", k16<2>, 2, threads, 2048);
    run("16x16x4", k16<4>, 4, threads, 2048);
    run("16x16x4", k16<8>, 8, threads, 2048);
  }
  return 0;
}
