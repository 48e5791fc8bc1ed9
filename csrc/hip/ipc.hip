// In-house IPC mesh collective for one node (xGMI peer-to-peer writes).
//
// Every rank owns an inbox (2 parities x W slots x slot_bytes) and a flag
// word per source rank, both exported with hipIpcGetMemHandle and mapped by
// every peer.  One kernel per collective, graph-capturable and host-sync
// free:
//   1. put:    the grid writes its payload (slot p of the send buffer, or the
//              whole buffer for a broadcast) straight into peer p's inbox
//              slot [parity][rank] -- one pass over xGMI, no staging;
//   2. signal: every block fences at system scope and arrives on a local
//              counter; the last block publishes the epoch into each peer's
//              flag word [rank] (system-scope release store);
//   3. wait:   every block waits (bounded spin, acquire loads) until all W
//              flags of its own inbox carry the epoch;
//   4. reduce: (all-reduce) out = scale * sum over the W slots.
// The epoch lives in device memory and is advanced by the last block to
// leave, so replays of a captured graph keep counting.  Parity
// double-buffering makes inbox reuse safe: a peer can only write parity
// (e+2)%2 after it saw this rank's epoch e+1 flag, which is published after
// this rank finished reading epoch e.  A spin that exceeds its bound sets
// err[0] = 1 and the kernel exits (a lost peer cannot hang the GPU).
// Reference: the in-process c_mixallgather / heter_comm peer copies
// (c_mixallgather_op.cc:221-327, heter_comm_inl.h:273-490).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

__device__ __forceinline__ uint64_t ld_acquire_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_release_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_ipc_collective(IpcPeers pt, const unsigned char* __restrict__ send,
                                                        int64_t nbytes, int broadcast, float* out, int64_t nfloat,
                                                        float scale, int reduce) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_last;
  const int W = pt.world, me = pt.rank;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(pt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int par = (int)(epoch & 1);
  const int64_t slot = pt.slot_bytes;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  // 1. put (16-byte vectors + a byte tail; slot_bytes is a multiple of 16)
  const int64_t nv = nbytes >> 4;
  for (int p = 0; p < W; ++p) {
    const unsigned char* sb = send + (broadcast ? 0 : p * slot);
    unsigned char* db = pt.inbox[p] + ((int64_t)par * W + me) * slot;
    const uint4* src = reinterpret_cast<const uint4*>(sb);
    uint4* dst = reinterpret_cast<uint4*>(db);
    for (int64_t i = tid; i < nv; i += nth) dst[i] = src[i];
    if (tid < (nbytes & 15)) db[(nv << 4) + tid] = sb[(nv << 4) + tid];
  }
  // 2. signal
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int a = atomicAdd(pt.arrive, 1u) + 1u;
    s_last = (a % gridDim.x) == 0;
  }
  __syncthreads();
  if (s_last && threadIdx.x < W) st_release_sys(pt.flags[threadIdx.x] + me, epoch);
  // 3. wait for every source's flag in this rank's inbox
  if (threadIdx.x < W) {
    const uint64_t* f = pt.flags[me] + threadIdx.x;
    int64_t spins = 0;
    while (ld_acquire_sys(f) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (int64_t)1 << 24) {
        pt.err[0] = 1;
        break;
      }
    }
  }
  __syncthreads();
  // 4. reduce the W slots of this parity
  if (reduce) {
    const float* base = reinterpret_cast<const float*>(pt.inbox[me] + (int64_t)par * W * slot);
    const int64_t fs = slot / 4;
    for (int64_t i = tid; i < nfloat; i += nth) {
      float s = 0.f;
      for (int p = 0; p < W; ++p) s += __builtin_nontemporal_load(base + p * fs + i);
      out[i] = s * scale;
    }
  }
  // the last block to leave advances the epoch for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned int d = atomicAdd(pt.depart, 1u) + 1u;
    if ((d % gridDim.x) == 0) __hip_atomic_store(pt.epoch, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

void launch_ipc_collective(const IpcPeers& pt, const void* send, int64_t nbytes, bool broadcast, float* out,
                           int64_t nfloat, float scale, bool reduce, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_collective, dim3(blocks), dim3(256), 0, s, pt,
                     reinterpret_cast<const unsigned char*>(send), nbytes, broadcast ? 1 : 0, out, nfloat, scale,
                     reduce ? 1 : 0);
}

}  // namespace pbx
