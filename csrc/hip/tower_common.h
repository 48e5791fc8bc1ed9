// Pieces shared by the bf16 tower (tower.hip) and the fp32 tower (tower32.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "tower32_sched.h"

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
    const float mx = tx / (float)a.M, sq = tq / (float)a.M + a.dn_eps;
    a.dn_stats[c] = 1.f;
    a.dn_stats[C + c] = mx;
    a.dn_stats[2 * C + c] = sq;
    if (a.dn_bsize) {  // same arithmetic as k_dn_update (dense_ops.hip)
      a.dn_bsize[c] = a.dn_bsize[c] * a.dn_decay + 1.f;
      a.dn_bsum[c] = a.dn_bsum[c] * a.dn_decay + mx;
      a.dn_bsq[c] = a.dn_bsq[c] * a.dn_decay + sq;
    }
  }
}

// Per-row inputs of the loss tail, loaded by waves 0 and 1 (lane r = row r)
// at kernel start so that their latency hides under the layer loop.
struct TowerRowIn {
  float lin, y, mask, bout;
};
__device__ inline TowerRowIn tower_row_in(const TowerArgs& a, int m0, int lane, int rows) {
  TowerRowIn r{0.f, 0.f, 0.f, 0.f};
  const int m = m0 + lane;
  r.bout = a.b_out ? a.b_out[0] : 0.f;
  if (lane < rows && m < a.M) {
    r.lin = a.lin ? a.lin[m] : 0.f;
    r.y = a.label[(int64_t)m * a.label_stride];
    r.mask = (a.auc_table && (!a.auc_mask || a.auc_mask[m] != 0.f)) ? 1.f : 0.f;
  }
  return r;
}

// Loss tail of the forward launches, once zrow[r] (the output-layer GEMV of
// row r) is in LDS and the workgroup has synchronised.  One lane per row:
// wave 0 computes the loss / AUC partial sums and runs the cross-workgroup
// ticket; wave 1 stores pred / dz and adds the AUC histogram, so the drain
// before wave 0's ticket waits only for its own six partial stores.  The
// last workgroup reduces the partials in a fixed lane order and tree
// (deterministic).  Semantics: sigmoid + log_loss (phi/kernels/gpu/log_loss_kernel.cu),
// auc histogram (phi/kernels/gpu/auc_kernel.cu:25-80).
__device__ inline void tower_loss_tail(const TowerArgs& a, const float* zrow, const TowerRowIn& in, int m0, int w,
                                       int lane, int rows) {
  if (w > 1) return;
  const int m = m0 + lane;
  const bool valid = lane < rows && m < a.M;
  const float inv = 1.f / (float)a.M;
  float z = 0.f, p = 0.f;
  if (valid) {
    z = zrow[lane] + in.bout + in.lin;
    p = 1.f / (1.f + __expf(-z));
  }
  if (w == 1) {
    int key = -1;
    if (valid) {
      a.pred[m] = p;
      a.dz[m] = (p - in.y) * inv;
      if (in.mask != 0.f) {
        const int lab = in.y > 0.5f ? 1 : 0;
        const int T = a.auc_buckets;
        int pos = (int)(p * T);
        pos = pos < 0 ? 0 : (pos > T - 1 ? T - 1 : pos);
        key = lab * T + pos;
      }
    }
    // Histogram adds merged per wave: once the model has converged most rows'
    // predictions share a handful of buckets, and 8192 float64 atomics on one
    // address serialise in L2 (step time drifted 0.35 -> 0.40 ms over 2000
    // steps, profiles/r6_auc_contention.txt).  Up to 8 rounds: the lanes on
    // the lowest active lane's bucket add their count with one atomic; lanes
    // left over after that add 1 each.
    unsigned long long act = __ballot(key >= 0);
    for (int it = 0; act != 0ull && it < 8; ++it) {
      const int leader = __builtin_ctzll(act);
      const int k = __shfl(key, leader);
      const unsigned long long same = __ballot(key == k);
      if (lane == leader) atomicAdd(&a.auc_table[k], (double)__popcll(same));
      act &= ~same;
      if (key == k) key = -1;
    }
    if (key >= 0) atomicAdd(&a.auc_table[key], 1.0);
    return;
  }
  float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (valid) {
    v[0] = fmaxf(z, 0.f) - z * in.y + log1pf(__expf(-fabsf(z)));
    if (in.mask != 0.f) {
      const float d = p - (in.y > 0.5f ? 1.f : 0.f);
      v[1] = fabsf(d);
      v[2] = d * d;
      v[3] = p;
      v[4] = in.y > 0.5f ? 1.f : 0.f;
      v[5] = 1.f;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v[i] += __shfl_xor(v[i], off);
  if (a.debug & 1) return;
  int last = 0;
  if (lane == 0) {
    // hand-off without fences (MI355X_MICROARCH.md, valid-forms table row 1):
    // write-through (sc1) partial stores, drained, then the ticket; the last
    // adder reads them back with sc1 loads
    float* pp = a.part + (int64_t)blockIdx.x * 8;
#pragma unroll
    for (int i = 0; i < 6; ++i) __hip_atomic_store(&pp[i], v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
  }
  last = __shfl(last, 0);
  if (!last) return;
  float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (unsigned int k = lane; k < gridDim.x; k += 64) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
      acc[i] += __hip_atomic_load(&a.part[(int64_t)k * 8 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
    for (int off = 32; off > 0; off >>= 1) acc[i] += __shfl_xor(acc[i], off);
  if (lane == 0) {
    a.loss[0] = acc[0] * inv;
    if (a.auc_stats && acc[5] > 0.f) {
      for (int i = 0; i < 5; ++i) a.auc_stats[i] += (double)acc[1 + i];
    }
    *a.ticket = 0u;
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

// fp32 tower wave-stream schedule: tower32_sched.h
// element W[n][k] in packed W (forward B operand: column block n / 16,
// k-group k / 16; lane (n % 16) + 16 ((k % 16) / 4), component k % 4) and in
// packed W^T (backward B operand: column block k / 16, k-group n / 16)
__device__ __forceinline__ int64_t tower_wp32_index(int n, int k, int Np, int Kp) {
  return (t32_group_pos(Np >> 4, Kp >> 4, n >> 4, k >> 4) * 64 + (n & 15) + 16 * ((k & 15) >> 2)) * 4 + (k & 3);
}
__device__ __forceinline__ int64_t tower_wtp32_index(int n, int k, int Np, int Kp) {
  return (t32_group_pos(Kp >> 4, Np >> 4, k >> 4, n >> 4) * 64 + (k & 15) + 16 * ((n & 15) >> 2)) * 4 + (n & 3);
}
// the same through precomputed group positions (pos [Np/16][Kp/16], posT [Kp/16][Np/16])
__device__ __forceinline__ int64_t tower_wp32_index_pos(const int* pos, int n, int k, int Kp) {
  return ((int64_t)pos[(n >> 4) * (Kp >> 4) + (k >> 4)] * 64 + (n & 15) + 16 * ((k & 15) >> 2)) * 4 + (k & 3);
}
__device__ __forceinline__ int64_t tower_wtp32_index_pos(const int* posT, int n, int k, int Np) {
  return ((int64_t)posT[(k >> 4) * (Np >> 4) + (n >> 4)] * 64 + (k & 15) + 16 * ((n & 15) >> 2)) * 4 + (n & 3);
}

}  // namespace pbx
