// Pieces shared by the bf16 tower (tower.hip) and the fp32 tower (tower32.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {

// Column reductions that ride along with the dW launch, one 256-thread
// workgroup per 32 columns (rb = workgroup index past the dW tiles):
//  * rb < nbias: sum the per-row-tile bias partials [nwg][bias_ld] into the
//    layer biases' grads, dw_out and db_out (accumulated, +=);
//  * otherwise: data_norm batch statistics from the head's per-block
//    partials [dn_rows][2C] -> stats [3][C] = (1, sum/M, sq/M + eps).
// tbm = rows per fwd/bwd workgroup (nwg = Mp / tbm bias-partial rows).
__device__ inline void tower_col_reduce(const TowerArgs& a, int rb, int tbm) {
  __shared__ float red[2][8][32];
  const int tid = threadIdx.x;
  const int cl = tid & 31, rg = tid >> 5;
  const int nbias = (a.bias_ld + 31) / 32;
  if (rb < nbias) {
    const int col = rb * 32 + cl;
    const int nwg = a.Mp / tbm;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (col < a.bias_ld) {
      int r = rg;
      for (; r + 24 < nwg; r += 32) {
        s0 += a.bias_part[(int64_t)r * a.bias_ld + col];
        s1 += a.bias_part[(int64_t)(r + 8) * a.bias_ld + col];
        s2 += a.bias_part[(int64_t)(r + 16) * a.bias_ld + col];
        s3 += a.bias_part[(int64_t)(r + 24) * a.bias_ld + col];
      }
      for (; r < nwg; r += 8) s0 += a.bias_part[(int64_t)r * a.bias_ld + col];
    }
    red[0][rg][cl] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (rg == 0 && col < a.bias_ld) {
      float s = 0.f;
      for (int g = 0; g < 8; ++g) s += red[0][g][cl];
      if (col == a.dbout_off) {
        if (a.db_out) a.db_out[0] += s;
      } else if (col >= a.dwout_off) {
        if (a.dw_out && col - a.dwout_off < a.ly[a.L - 1].N) a.dw_out[col - a.dwout_off] += s;
      } else {
        for (int l = 0; l < a.L; ++l) {
          const TowerLayerDev& ly = a.ly[l];
          if (col >= ly.bias_off && col < ly.bias_off + ly.N) {
            if (ly.db) ly.db[col - ly.bias_off] += s;
            break;
          }
        }
      }
    }
    return;
  }
  const int c = (rb - nbias) * 32 + cl;
  const int C = a.dn_C;
  float sx = 0.f, sq = 0.f, sx1 = 0.f, sq1 = 0.f;
  if (a.dn_part && c < C) {
    int r = rg;
    for (; r + 8 < a.dn_rows; r += 16) {
      sx += a.dn_part[(int64_t)r * 2 * C + c];
      sq += a.dn_part[(int64_t)r * 2 * C + C + c];
      sx1 += a.dn_part[(int64_t)(r + 8) * 2 * C + c];
      sq1 += a.dn_part[(int64_t)(r + 8) * 2 * C + C + c];
    }
    for (; r < a.dn_rows; r += 8) {
      sx += a.dn_part[(int64_t)r * 2 * C + c];
      sq += a.dn_part[(int64_t)r * 2 * C + C + c];
    }
  }
  red[0][rg][cl] = sx + sx1;
  red[1][rg][cl] = sq + sq1;
  __syncthreads();
  if (rg == 0 && a.dn_part && c < C) {
    float tx = 0.f, tq = 0.f;
    for (int g = 0; g < 8; ++g) {
      tx += red[0][g][cl];
      tq += red[1][g][cl];
    }
    a.dn_stats[c] = 1.f;
    a.dn_stats[C + c] = tx / (float)a.M;
    a.dn_stats[2 * C + c] = tq / (float)a.M + a.dn_eps;
  }
}

// Workgroup index -> work id such that consecutive work ids land on one XCD
// (blocks are dealt to the 8 XCDs round-robin; speed only, never correctness).
__device__ inline int xcd_work_id(int block, int n) {
  const int q = n / 8, rr = n % 8, xcd = block % 8;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + block / 8;
}

// 16-B-per-lane LDS-DMA (lane l lands at lds_byte + 16 l), issued from inline
// asm so hipcc does not drain the ring with vmcnt(0) at every later ds_read.
__device__ __forceinline__ void tower_glds16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ unsigned tower_lds_addr(const void* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// fp32 tower packed-weight index maps (kernels.h layout comment): element
// W[n][k] in packed W (forward B operand) and packed W^T (backward B operand)
__device__ __forceinline__ int64_t tower_wp32_index(int n, int k, int Kp) {
  return ((int64_t)((n >> 4) * (Kp >> 4) + (k >> 4)) * 64 + (n & 15) + 16 * ((k & 15) >> 2)) * 4 + (k & 3);
}
__device__ __forceinline__ int64_t tower_wtp32_index(int n, int k, int Np) {
  return ((int64_t)((k >> 4) * (Np >> 4) + (n >> 4)) * 64 + (k & 15) + 16 * ((n & 15) >> 2)) * 4 + (n & 3);
}

}  // namespace pbx
