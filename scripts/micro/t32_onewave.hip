// Timing experiment for the fp32 tower forward (csrc/hip/tower32.hip
// k_t32_fwd): ONE wave per SIMD (256-thread workgroup, one 32-row tile per
// CU) instead of two.  Each wave owns a pair of 16-column blocks for both
// 16-row halves: four independent v_mfma_f32_16x16x4_f32 accumulators, every
// weight fragment feeds 2 MFMAs and every LDS A fragment 2 MFMAs.  The wave's
// weight stream (2 KB per 16-deep k-group: the pair's two fragments) runs
// through a register ring of R k-groups with no partner wave to share the
// matrix pipe with, so nothing is left running alone at the end of a layer.
//
// Layers 304 -> 400 -> 400 -> 400 at M = 8192 (the DeepFM headline tower).
// Column blocks: 25 per 400-wide layer = 12 pairs (3 per wave) + block 24,
// which LEFT = 0 drops (ceiling), 1 gives to wave 0, 2 splits over the four
// waves by K range (partial sums through LDS, added in wave order).
// Checks a few output rows against a CPU fp32 reference.
// build: hipcc --offload-arch=gfx950 -O3 -o t32_onewave t32_onewave.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int BM = 32;
constexpr int NW = 4;

struct Layer {
  const f32x4* ws;  // per-wave streams, concatenated: [w][units][ngp][2][64] f32x4
  const f32x4* wl;  // leftover block stream [ngp][64] (LEFT 1 / 2)
  const float* bias;
  int K, N, ng, ngp, np;  // np: pairs per wave
  long long wave_stride;  // f32x4 per wave stream
};
struct Args {
  const float* x0;
  float* out;  // [M][N_last]
  Layer ly[3];
  int L, M, ldl;
};

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int R>
struct Ring {
  f32x4 b[R][2];
};

// one k-group: 16 MFMAs (4 k-steps x {2 blocks} x {2 halves})
__device__ __forceinline__ void kgroup(const f32x4& a0, const f32x4& a1, const f32x4& b0, const f32x4& b1,
                                       f32x4 (&acc)[2][2]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[0][0] = mfma(a0[t], b0[t], acc[0][0]);
    acc[0][1] = mfma(a1[t], b0[t], acc[0][1]);
    acc[1][0] = mfma(a0[t], b1[t], acc[1][0]);
    acc[1][1] = mfma(a1[t], b1[t], acc[1][1]);
  }
}

template <int R, int LEFT>
__global__ __launch_bounds__(256) void k_fwd(Args a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int ldl = a.ldl;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * BM;
  float* src = lds;
  float* dst = lds + BM * ldl;
  float* part = lds + 2 * BM * ldl + 64;  // [4 waves][2 halves][64][4]
  {
    const int K0 = a.ly[0].K;
    const int c4n = K0 / 4;
    for (int i = tid; i < BM * c4n; i += 256) {
      const int r = i / c4n, cc = i - r * c4n;
      *reinterpret_cast<float4*>(src + r * ldl + cc * 4) =
          *reinterpret_cast<const float4*>(a.x0 + (long long)(m0 + r) * K0 + cc * 4);
    }
  }
  __syncthreads();
  for (int l = 0; l < a.L; ++l) {
    const Layer& ly = a.ly[l];
    const int ng = ly.ng, ngp = ly.ngp;
    const f32x4* bp = ly.ws + w * ly.wave_stride + lane;
    Ring<R> rg;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      rg.b[r][0] = bp[(r * 2) * 64];
      rg.b[r][1] = bp[(r * 2 + 1) * 64];
    }
    const float* A0 = src + c * ldl + 4 * g;
    const float* A1 = A0 + 16 * ldl;
    for (int u = 0; u < ly.np; ++u) {
      f32x4 acc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int g0 = 0; g0 < ngp; g0 += R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int gg = g0 + r;
          if (gg < ng) {
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(A0 + 16 * gg);
            const f32x4 a1 = *reinterpret_cast<const f32x4*>(A1 + 16 * gg);
            kgroup(a0, a1, rg.b[r][0], rg.b[r][1], acc);
          }
          __builtin_amdgcn_sched_barrier(0);
          // refill: the k-group R ahead in this wave's stream (across units)
          rg.b[r][0] = bp[((g0 + r + R) * 2) * 64];
          rg.b[r][1] = bp[((g0 + r + R) * 2 + 1) * 64];
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      bp += ngp * 2 * 64;
      // epilogue: pair p = u * 4 + w -> blocks 2p, 2p + 1
      const int p = u * NW + w;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = (2 * p + j) * 16 + c;
        const float bias = ly.bias[n];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float v = acc[j][h][t] + bias;
            dst[(16 * h + 4 * g + t) * ldl + n] = v > 0.f ? v : 0.f;
          }
      }
    }
    if (LEFT == 1 && w == 0) {  // block 24 whole on wave 0
      const f32x4* lp = ly.wl + lane;
      f32x4 s0 = (f32x4){0.f, 0.f, 0.f, 0.f}, s1 = s0;
      for (int gg = 0; gg < ng; ++gg) {
        const f32x4 b = lp[gg * 64];
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(A0 + 16 * gg);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(A1 + 16 * gg);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s0 = mfma(a0[t], b[t], s0);
          s1 = mfma(a1[t], b[t], s1);
        }
      }
      const int n = 24 * 16 + c;
      const float bias = ly.bias[n];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float v0 = s0[t] + bias, v1 = s1[t] + bias;
        dst[(4 * g + t) * ldl + n] = v0 > 0.f ? v0 : 0.f;
        dst[(16 + 4 * g + t) * ldl + n] = v1 > 0.f ? v1 : 0.f;
      }
    }
    if (LEFT == 2) {  // block 24 split over the waves by K range
      const int lo = w * ng / NW, hi = (w + 1) * ng / NW;
      const f32x4* lp = ly.wl + lane;
      f32x4 s0 = (f32x4){0.f, 0.f, 0.f, 0.f}, s1 = s0;
      for (int gg = lo; gg < hi; ++gg) {
        const f32x4 b = lp[gg * 64];
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(A0 + 16 * gg);
        const f32x4 a1 = *reinterpret_cast<const f32x4*>(A1 + 16 * gg);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s0 = mfma(a0[t], b[t], s0);
          s1 = mfma(a1[t], b[t], s1);
        }
      }
      *reinterpret_cast<f32x4*>(part + (w * 2 + 0) * 256 + lane * 4) = s0;
      *reinterpret_cast<f32x4*>(part + (w * 2 + 1) * 256 + lane * 4) = s1;
    }
    __syncthreads();
    if (LEFT == 2 && w < 2) {  // wave h sums half h in wave order
      f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f};
      for (int ww = 0; ww < NW; ++ww) s += *reinterpret_cast<const f32x4*>(part + (ww * 2 + w) * 256 + lane * 4);
      const int n = 24 * 16 + c;
      const float bias = ly.bias[n];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float v = s[t] + bias;
        dst[(16 * w + 4 * g + t) * ldl + n] = v > 0.f ? v : 0.f;
      }
    }
    if (LEFT == 2) __syncthreads();
    float* tt = src;
    src = dst;
    dst = tt;
  }
  const int NL = a.ly[a.L - 1].N;
  for (int i = tid; i < BM * NL; i += 256) {
    const int r = i / NL, cc = i - r * NL;
    a.out[(long long)(m0 + r) * NL + cc] = src[r * ldl + cc];
  }
}

// host packing: W [N][K] row-major -> per-wave pair streams / leftover stream
static void pack_layer(const std::vector<float>& W, int N, int K, int R, std::vector<float>& ws,
                       std::vector<float>& wl, int& ng, int& ngp, int& np, long long& wave_stride) {
  ng = K / 16;
  ngp = (ng + R - 1) / R * R;
  const int nblk = N / 16;
  const int pairs = nblk / 2;  // 12
  np = pairs / NW;             // 3
  // per unit: ngp k-groups x 2 blocks x 64 lanes x 4; + R k-groups of slack
  wave_stride = ((long long)np * ngp + R) * 2 * 64;
  ws.assign((size_t)NW * wave_stride * 4, 0.f);
  auto frag = [&](float* dstp, int blk, int kg) {
    for (int ln = 0; ln < 64; ++ln)
      for (int t = 0; t < 4; ++t) {
        const int n = blk * 16 + (ln & 15), k = kg * 16 + 4 * (ln >> 4) + t;
        dstp[ln * 4 + t] = W[(size_t)n * K + k];
      }
  };
  for (int w = 0; w < NW; ++w)
    for (int u = 0; u < np; ++u) {
      const int p = u * NW + w;
      for (int kg = 0; kg < ng; ++kg)
        for (int j = 0; j < 2; ++j) {
          float* d = &ws[(((size_t)w * wave_stride) + ((size_t)(u * ngp + kg) * 2 + j) * 64) * 4];
          frag(d, 2 * p + j, kg);
        }
    }
  wl.assign((size_t)ng * 64 * 4, 0.f);
  if (nblk % 2)
    for (int kg = 0; kg < ng; ++kg) frag(&wl[(size_t)kg * 64 * 4], nblk - 1, kg);
}

template <int R, int LEFT>
static float run(Args a, int iters, size_t lds) {
  CK(hipFuncSetAttribute((const void*)k_fwd<R, LEFT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k_fwd<R, LEFT>), dim3(a.M / BM), dim3(256), lds, 0, a);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_fwd<R, LEFT>), dim3(a.M / BM), dim3(256), lds, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int M = 8192, L = 3;
  const int dims[4] = {304, 400, 400, 400};
  const int iters = argc > 1 ? atoi(argv[1]) : 50;
  srand(1);
  auto rnd = [] { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; };
  std::vector<float> x0((size_t)M * dims[0]);
  for (auto& v : x0) v = rnd();
  std::vector<std::vector<float>> W(L), B(L);
  for (int l = 0; l < L; ++l) {
    W[l].resize((size_t)dims[l + 1] * dims[l]);
    for (auto& v : W[l]) v = rnd() * 0.08f;
    B[l].resize(dims[l + 1]);
    for (auto& v : B[l]) v = rnd() * 0.1f;
  }
  // CPU reference of rows 0..63
  const int RR = 64;
  std::vector<float> ref((size_t)RR * dims[L]);
  {
    std::vector<float> h(x0.begin(), x0.begin() + (size_t)RR * dims[0]);
    for (int l = 0; l < L; ++l) {
      std::vector<float> o((size_t)RR * dims[l + 1]);
      for (int r = 0; r < RR; ++r)
        for (int n = 0; n < dims[l + 1]; ++n) {
          double s = B[l][n];
          for (int k = 0; k < dims[l]; ++k) s += (double)h[(size_t)r * dims[l] + k] * W[l][(size_t)n * dims[l] + k];
          o[(size_t)r * dims[l + 1] + n] = s > 0 ? (float)s : 0.f;
        }
      h.swap(o);
    }
    ref = h;
  }
  float *dx0, *dout;
  CK(hipMalloc(&dx0, x0.size() * 4));
  CK(hipMemcpy(dx0, x0.data(), x0.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&dout, (size_t)M * dims[L] * 4));
  const int ldl = 420;  // >= 400 + R*16 read-ahead slack is not needed (pads skipped)
  const size_t lds = ((size_t)2 * BM * ldl + 64 + NW * 2 * 256) * 4;
  auto build = [&](int R, Args& a, std::vector<void*>& bufs) {
    a.x0 = dx0;
    a.out = dout;
    a.L = L;
    a.M = M;
    a.ldl = ldl;
    for (int l = 0; l < L; ++l) {
      std::vector<float> ws, wl;
      Layer& ly = a.ly[l];
      long long st;
      pack_layer(W[l], dims[l + 1], dims[l], R, ws, wl, ly.ng, ly.ngp, ly.np, st);
      ly.wave_stride = st;
      ly.K = dims[l];
      ly.N = dims[l + 1];
      void *p1, *p2, *p3;
      CK(hipMalloc(&p1, ws.size() * 4));
      CK(hipMemcpy(p1, ws.data(), ws.size() * 4, hipMemcpyHostToDevice));
      CK(hipMalloc(&p2, wl.size() * 4));
      CK(hipMemcpy(p2, wl.data(), wl.size() * 4, hipMemcpyHostToDevice));
      CK(hipMalloc(&p3, B[l].size() * 4));
      CK(hipMemcpy(p3, B[l].data(), B[l].size() * 4, hipMemcpyHostToDevice));
      ly.ws = (const f32x4*)p1;
      ly.wl = (const f32x4*)p2;
      ly.bias = (const float*)p3;
      bufs.push_back(p1);
      bufs.push_back(p2);
      bufs.push_back(p3);
    }
  };
  auto check = [&](const char* tag, float us) {
    std::vector<float> o((size_t)RR * dims[L]);
    CK(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
    double md = 0;
    int bad24 = 0;
    for (size_t i = 0; i < o.size(); ++i) {
      const int n = (int)(i % dims[L]);
      const double d = fabs(o[i] - ref[i]);
      if (n >= 384) {
        bad24 += d > 1e-3;
        continue;
      }
      md = d > md ? d : md;
    }
    const double fl = 2.0 * M * (304.0 * 400 + 400.0 * 400 * 2);
    printf("%-16s %7.1f us  %5.1f TFLOP/s  max|err| (blocks 0-23) %.2e  block-24 mismatches %d\n", tag, us,
           fl / us / 1e6, md, bad24);
  };
  {
    Args a;
    std::vector<void*> b;
    build(4, a, b);
    check("R4 LEFT0", run<4, 0>(a, iters, lds));
    check("R4 LEFT1", run<4, 1>(a, iters, lds));
    check("R4 LEFT2", run<4, 2>(a, iters, lds));
  }
  {
    Args a;
    std::vector<void*> b;
    build(2, a, b);
    check("R2 LEFT2", run<2, 2>(a, iters, lds));
  }
  {
    Args a;
    std::vector<void*> b;
    build(6, a, b);
    check("R6 LEFT2", run<6, 2>(a, iters, lds));
  }
  {
    Args a;
    std::vector<void*> b;
    build(8, a, b);
    check("R8 LEFT0", run<8, 0>(a, iters, lds));
    check("R8 LEFT2", run<8, 2>(a, iters, lds));
  }
  return 0;
}
