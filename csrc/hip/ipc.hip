// In-house IPC mesh collectives for the GPUs of one node (xGMI peer writes).
//
// Every rank owns an inbox [depth][2][W][slot_bytes] and 2W flag words, both
// exported with hipIpcGetMemHandle and mapped by every peer.  One kernel per
// collective, graph-capturable and free of host synchronisation:
//   put     the grid writes its payload straight into peer p's inbox slot
//           [e % depth][phase][me] (one pass over xGMI);
//   signal  every block drains its puts, one lane releases at system scope and
//           arrives on a local counter; the last block publishes
//           (epoch << 28 | count) into each peer's flag word [phase][me];
//   wait    every block polls (bounded, relaxed system-scope loads) until all
//           W flags of its own inbox carry the epoch, then acquires once; the
//           counts ride along.
// Collectives:
//   exchange   all-to-all of per-peer records: only counts[p] records of slot
//              p travel (the sparse step's keys / values / gradients, sized by
//              the unique keys per owner, not by the padded capacity); the
//              receiver learns the counts from the flags, copies the valid
//              records to its destination buffer, writes the counts to
//              rcounts and may fill the rest with 0xFF bytes (= -1 keys);
//   allreduce  one-shot (W copies summed by every rank, latency-bound sizes)
//              or two-phase (reduce-scatter + all-gather: each rank moves
//              2(W-1)/W of the buffer instead of W-1 times it).
// The epoch lives in device memory and is advanced by the last block to
// leave, so replays of a captured graph keep counting.  A call uses inbox
// slot epoch % depth and consumes it inside the launch (the reduce, or the
// exchange's copy-out into the caller's buffer).  A peer writes the same slot
// again only at epoch e + depth, after it saw this rank's flag of epoch
// e + depth - 1, which this rank publishes in a later launch -- so no slot is
// overwritten while it is read, whatever the caller does between calls.
// Failure: a wait that exceeds its bound sets the sticky err word, poisons the
// result (NaN sums / zero counts and -1 keys) and later launches skip their
// waits, so a lost peer fails every rank fast instead of hanging the GPU or
// training silently on stale slots; IpcMesh.check() raises on the host.
// Reference: the in-process c_mixallgather / heter_comm peer copies
// (c_mixallgather_op.cc:221-327, heter_comm_inl.h:273-490).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace pbx {
namespace {

// flag word = epoch << kCountBits | count: 2^28 records per peer slot (the
// host refuses bigger slots), 36 epoch bits (~6.9e10 collectives)
constexpr int kCountBits = kIpcCountBits;
constexpr uint64_t kCountMask = (1ull << kCountBits) - 1;

__device__ __forceinline__ unsigned char* slot_ptr(const IpcPeers& pt, int owner, int slot, int phase, int src) {
  const int64_t s = pt.slot_bytes;
  const int W = pt.world;
  return pt.inbox[owner] + ((((int64_t)slot * 2 + phase) * W + src) * s);
}

// grid-strided copy of n bytes (16-B vectors + byte tail; both ends 16-B
// aligned).  Four independent 16-B loads are in flight per lane before their
// stores: a copy loop with one load per iteration waits a full (remote)
// memory latency per 16 B and runs at a fraction of the link / HBM rate.
__device__ __forceinline__ void put_bytes(unsigned char* dst, const unsigned char* src, int64_t n, int64_t tid,
                                          int64_t nth) {
  const int64_t nv = n >> 4;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  int64_t i = tid;
  for (; i + 3 * nth < nv; i += 4 * nth) {
    const uint4 a = s4[i], b = s4[i + nth], c = s4[i + 2 * nth], d = s4[i + 3 * nth];
    d4[i] = a;
    d4[i + nth] = b;
    d4[i + 2 * nth] = c;
    d4[i + 3 * nth] = d;
  }
  for (; i < nv; i += nth) d4[i] = s4[i];
  if (tid < (n & 15)) dst[(nv << 4) + tid] = src[(nv << 4) + tid];
}

// Publish: every wave drains its own puts (vmcnt 0), the workgroup meets at
// a barrier, ONE lane issues the system-scope release (write-back of the
// XCD's L2, for puts that went through it) and arrives on the local counter;
// the last-arriving block then stores (epoch, count[p]) into each peer's
// flag word with a relaxed system-scope store.  One release per block, not
// one per thread (MI355X_MICROARCH.md, valid forms: producer).
__device__ __forceinline__ void signal(const IpcPeers& pt, uint64_t epoch, int phase, const int32_t* counts,
                                       int* s_last, int64_t max_count = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int a = atomicAdd(pt.arrive, 1u) + 1u;
    *s_last = (a % gridDim.x) == 0;
  }
  __syncthreads();
  if (*s_last && (int)threadIdx.x < pt.world) {
    const int p = threadIdx.x;
    int64_t cn = counts ? (int64_t)counts[p] : 0;
    cn = cn < 0 ? 0 : (cn > max_count ? max_count : cn);  // an overflowing sender sends (and announces) a full slot
    const uint64_t c = (uint64_t)cn & kCountMask;
    __hip_atomic_store(pt.flags[p] + phase * pt.world + pt.rank, (epoch << kCountBits) | c, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait for all W flags of phase: relaxed system-scope polls (no cache
// invalidation per poll), then ONE system-scope acquire per block before
// anything reads the inbox (the consumer form of the same table).  Returns
// false (and sets the sticky err) on timeout; the counts land in s_cnt[src].
__device__ __forceinline__ bool wait_all(const IpcPeers& pt, uint64_t epoch, int phase, int* s_cnt, int* s_ok) {
  if (threadIdx.x == 0) *s_ok = 1;
  __syncthreads();
  if ((int)threadIdx.x < pt.world) {
    const uint64_t* f = pt.flags[pt.rank] + phase * pt.world + threadIdx.x;
    const bool dead = __hip_atomic_load(pt.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    uint64_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    int64_t spins = 0;
    while (!dead && (v >> kCountBits) < epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > pt.spin_limit) {
        atomicExch(pt.err, 1);
        break;
      }
      v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if ((v >> kCountBits) < epoch) {
      *s_ok = 0;
      s_cnt[threadIdx.x] = 0;
    } else {
      s_cnt[threadIdx.x] = (int)(v & kCountMask);
    }
  }
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return *s_ok != 0;
}

// the last block to leave advances the epoch for the next launch
__device__ __forceinline__ void depart(const IpcPeers& pt, uint64_t epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int d = atomicAdd(pt.depart, 1u) + 1u;
    if ((d % gridDim.x) == 0) __hip_atomic_store(pt.epoch, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// out[i0 .. i1) = scale * sum over the W source slots (float4 body + tail);
// NaN when a wait failed
__device__ __forceinline__ void reduce_slots(const IpcPeers& pt, int sl, int phase, int W, int64_t i0, int64_t i1,
                                             float* out, float scale, bool ok, int64_t tid, int64_t nth) {
  const float qnan = __int_as_float(0x7fc00000);
  const int64_t n = i1 - i0;
  const bool vec = ((reinterpret_cast<uintptr_t>(out + i0) & 15) == 0);
  const int64_t n4 = vec ? n / 4 : 0;
  for (int64_t i4 = tid; i4 < n4; i4 += nth) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < W; ++p) {
      const float4 v = reinterpret_cast<const float4*>(slot_ptr(pt, pt.rank, sl, phase, p))[i4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(out + i0)[i4] =
        ok ? make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale) : make_float4(qnan, qnan, qnan, qnan);
  }
  for (int64_t i = n4 * 4 + tid; i < n; i += nth) {
    float s = 0.f;
    for (int p = 0; p < W; ++p) s += reinterpret_cast<const float*>(slot_ptr(pt, pt.rank, sl, phase, p))[i];
    out[i0 + i] = ok ? s * scale : qnan;
  }
}


__global__ __launch_bounds__(256) void k_ipc_exchange(IpcPeers pt, const unsigned char* __restrict__ send,
                                                      unsigned char* __restrict__ dst, const int32_t* counts,
                                                      int64_t rec_bytes, int fill_tail, int32_t* rcounts) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_last, s_ok;
  __shared__ int s_cnt[kIpcMaxRanks];
  const int W = pt.world, me = pt.rank;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(pt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int sl = (int)(epoch % (uint64_t)pt.depth);
  const int64_t slot = pt.slot_bytes;  // bytes per source
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int p = 0; p < W; ++p) {
    int64_t n = counts ? (int64_t)counts[p] * rec_bytes : slot;
    n = n < 0 ? 0 : (n > slot ? slot : n);
    put_bytes(slot_ptr(pt, p, sl, 0, me), send + p * slot, n, tid, nth);
  }
  signal(pt, epoch, 0, counts, &s_last, slot / rec_bytes);
  const bool ok = wait_all(pt, epoch, 0, s_cnt, &s_ok);
  // receiver side: the valid records of every source slot are copied out of
  // the inbox into dst (so the slot is free when this launch ends), counts
  // out, unused tails filled (keys -> -1)
  for (int src = 0; src < W; ++src) {
    int64_t have = counts ? (ok ? (int64_t)s_cnt[src] * rec_bytes : 0) : (ok ? slot : 0);
    have = have < slot ? have : slot;
    if (rcounts && tid == 0) rcounts[src] = ok ? (counts ? s_cnt[src] : (int)(slot / rec_bytes)) : 0;
    unsigned char* d = dst + src * slot;
    put_bytes(d, slot_ptr(pt, me, sl, 0, src), have, tid, nth);
    if (fill_tail || !ok) {
      if ((have & 7) == 0) {  // 8-B records (keys): word stores
        uint64_t* d8 = reinterpret_cast<uint64_t*>(d);
        for (int64_t i = (have >> 3) + tid; i < (slot >> 3); i += nth) d8[i] = ~0ull;
      } else {
        for (int64_t i = have + tid; i < slot; i += nth) d[i] = 0xFF;
      }
    }
  }
  depart(pt, epoch);
}

__global__ __launch_bounds__(256) void k_ipc_allreduce(IpcPeers pt, const float* __restrict__ src, float* out,
                                                       int64_t n, float scale, int two_phase) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_last, s_ok;
  __shared__ int s_cnt[kIpcMaxRanks];
  const int W = pt.world, me = pt.rank;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(pt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int sl = (int)(epoch % (uint64_t)pt.depth);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const float qnan = __int_as_float(0x7fc00000);
  if (!two_phase) {
    for (int p = 0; p < W; ++p)
      put_bytes(slot_ptr(pt, p, sl, 0, me), reinterpret_cast<const unsigned char*>(src), n * 4, tid, nth);
    signal(pt, epoch, 0, nullptr, &s_last);
    const bool ok = wait_all(pt, epoch, 0, s_cnt, &s_ok);
    reduce_slots(pt, sl, 0, W, 0, n, out, scale, ok, tid, nth);
    depart(pt, epoch);
    return;
  }
  // two-phase: chunk q (cs floats, 16-B multiple) is reduced by rank q
  const int64_t cs = ((n + W - 1) / W + 3) / 4 * 4;
  const int64_t mine0 = me * cs, mine1 = (me + 1) * cs < n ? (me + 1) * cs : n;
  for (int p = 0; p < W; ++p) {
    const int64_t a0 = p * cs, a1 = (p + 1) * cs < n ? (p + 1) * cs : n;
    if (a1 > a0)
      put_bytes(slot_ptr(pt, p, sl, 0, me), reinterpret_cast<const unsigned char*>(src + a0), (a1 - a0) * 4, tid,
                nth);
  }
  signal(pt, epoch, 0, nullptr, &s_last);
  bool ok = wait_all(pt, epoch, 0, s_cnt, &s_ok);
  // reduce my chunk and push each reduced float4 to every peer's gather area
  // (chunks are multiples of 4 floats; the last one may be short)
  const int64_t mc = mine1 - mine0;
  for (int64_t i4 = tid; i4 < (mc + 3) / 4; i4 += nth) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < W; ++p) {
      const float4 v = reinterpret_cast<const float4*>(slot_ptr(pt, me, sl, 0, p))[i4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s = ok ? make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale) : make_float4(qnan, qnan, qnan, qnan);
    for (int p = 0; p < W; ++p) reinterpret_cast<float4*>(slot_ptr(pt, p, sl, 1, me))[i4] = s;
  }
  signal(pt, epoch, 1, nullptr, &s_last);
  ok = wait_all(pt, epoch, 1, s_cnt, &s_ok) && ok;
  for (int q = 0; q < W; ++q) {  // gather: chunk q of every rank's result into out
    const int64_t a0 = q * cs, a1 = (q + 1) * cs < n ? (q + 1) * cs : n;
    if (a1 <= a0) continue;
    const float* g = reinterpret_cast<const float*>(slot_ptr(pt, me, sl, 1, q));
    if (ok) {
      put_bytes(reinterpret_cast<unsigned char*>(out + a0), reinterpret_cast<const unsigned char*>(g),
                (a1 - a0) * 4, tid, nth);
    } else {
      for (int64_t i = a0 + tid; i < a1; i += nth) out[i] = qnan;
    }
  }
  depart(pt, epoch);
}

}  // namespace

void launch_ipc_exchange(const IpcPeers& pt, const void* send, void* dst, const int32_t* counts, int64_t rec_bytes,
                         bool fill_tail, int32_t* rcounts, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_exchange, dim3(blocks), dim3(256), 0, s, pt, reinterpret_cast<const unsigned char*>(send),
                     reinterpret_cast<unsigned char*>(dst), counts, rec_bytes, fill_tail ? 1 : 0, rcounts);
}

void launch_ipc_allreduce(const IpcPeers& pt, const float* src, float* out, int64_t n, float scale, bool two_phase,
                          int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_allreduce, dim3(blocks), dim3(256), 0, s, pt, src, out, n, scale, two_phase ? 1 : 0);
}

}  // namespace pbx
