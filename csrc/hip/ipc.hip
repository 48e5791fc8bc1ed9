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
// Coherence: every access to an inbox or flag word is system-coherent at the
// instruction -- inbox stores and loads carry sc0 sc1 (write-through / miss in
// every cache level to the memory that owns the line, the per-access form of a
// system-scope release / acquire), the memory is uncached device memory
// (hipDeviceMallocUncached), and a producer's s_waitcnt vmcnt(0) orders its
// completed payload stores before its flag store -- and on top of that each
// block still issues the system-scope release before it arrives and the
// acquire after its wait (required: with the accesses alone the payload
// self-test failed on one mesh shape, profiles/r6_ipc_exchange_bench.txt).
// Failure: a wait that exceeds its bound sets the sticky err word, poisons the
// result (NaN sums / zero counts and -1 keys) and later launches skip their
// waits, so a lost peer fails every rank fast instead of hanging the GPU or
// training silently on stale slots; IpcMesh.check() raises on the host.
// Reference: the in-process c_mixallgather / heter_comm peer copies
// (c_mixallgather_op.cc:221-327, heter_comm_inl.h:273-490).
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "table_probe.h"

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
// DST_INBOX / SRC_INBOX: that side is an inbox slot (wave-uniform base),
// accessed through a buffer resource with sc0 sc1 (system coherence).
constexpr int kSys = 17;  // sc0 | sc1
typedef unsigned u32x4c __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t inbox_rsrc(const void* base, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(n < 0x7fffffff ? n : 0x7fffffff),
                                           0x00020000);
}
template <bool DST_INBOX, bool SRC_INBOX>
__device__ __forceinline__ void put_bytes(unsigned char* dst, const unsigned char* src, int64_t n, int64_t tid,
                                          int64_t nth) {
  const int64_t nv = n >> 4;
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const __amdgpu_buffer_rsrc_t rd = inbox_rsrc(dst, n), rs = inbox_rsrc(src, n);
  auto ld = [&](int64_t i) -> uint4 {
    if (SRC_INBOX) return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i << 4), 0, kSys));
    return s4[i];
  };
  auto st = [&](int64_t i, const uint4& v) {
    if (DST_INBOX)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4c, v), rd, (int)(i << 4), 0, kSys);
    else
      d4[i] = v;
  };
  int64_t i = tid;
  for (; i + 3 * nth < nv; i += 4 * nth) {
    const uint4 a = ld(i), b = ld(i + nth), c = ld(i + 2 * nth), d = ld(i + 3 * nth);
    st(i, a);
    st(i + nth, b);
    st(i + 2 * nth, c);
    st(i + 3 * nth, d);
  }
  for (; i < nv; i += nth) st(i, ld(i));
  if (tid < (n & 15)) {
    const int64_t o = (nv << 4) + tid;
    const unsigned char v = SRC_INBOX ? (unsigned char)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)o, 0, kSys) : src[o];
    if (DST_INBOX)
      __builtin_amdgcn_raw_buffer_store_b8(v, rd, (int)o, 0, kSys);
    else
      dst[o] = v;
  }
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
    if (pt.fence) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
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
  if (threadIdx.x == 0 && pt.fence) {
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
      const __amdgpu_buffer_rsrc_t r = inbox_rsrc(slot_ptr(pt, pt.rank, sl, phase, p), pt.slot_bytes);
      const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i4 << 4), 0, kSys));
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    reinterpret_cast<float4*>(out + i0)[i4] =
        ok ? make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale) : make_float4(qnan, qnan, qnan, qnan);
  }
  for (int64_t i = n4 * 4 + tid; i < n; i += nth) {
    float s = 0.f;
    for (int p = 0; p < W; ++p) {
      const __amdgpu_buffer_rsrc_t r = inbox_rsrc(slot_ptr(pt, pt.rank, sl, phase, p), pt.slot_bytes);
      s += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i << 2), 0, kSys));
    }
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
    put_bytes<true, false>(slot_ptr(pt, p, sl, 0, me), send + p * slot, n, tid, nth);
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
    put_bytes<false, true>(d, slot_ptr(pt, me, sl, 0, src), have, tid, nth);
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

// The sharded pull's key exchange with the owner pack fused into its put
// phase: the sender's unique keys (uniq_h[0 .. *u_count), the dedup output)
// are bucketed by owner -- per 256-key chunk, counts per owner in LDS and ONE
// global atomic per (chunk, owner) on ocnt reserve the positions -- and every
// key is written straight into its owner's inbox slot [sl][0][me] at that
// position, with send_index[u] = owner * cap + position (-1 + overflow flag
// past cap).  No send buffer is packed, read back and copied: the keys cross
// xGMI once, from the dedup output.  ocnt must be zero on entry (the dedup's
// first launch zeroes it) and holds the per-owner counts afterwards; the
// counts ride in the flag words, the receive side is k_ipc_exchange's
// (valid records copied out of the inbox, the tail filled with -1 keys).
// Reference: heter_comm_inl.h:273-490 (split_input_to_shard + the key walk).
__global__ __launch_bounds__(256) void k_ipc_pack_exchange(IpcPeers pt, const uint64_t* __restrict__ uniq_h,
                                                           const int32_t* __restrict__ u_count, int64_t cap,
                                                           int64_t* __restrict__ send_index, int32_t* ocnt,
                                                           int32_t* __restrict__ overflow, uint64_t* __restrict__ dst,
                                                           int32_t* rcounts) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_last, s_ok;
  __shared__ int s_cnt[kIpcMaxRanks];
  __shared__ int32_t lc[kIpcMaxRanks], lb[kIpcMaxRanks];
  const int W = pt.world, me = pt.rank;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(pt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int sl = (int)(epoch % (uint64_t)pt.depth);
  const int64_t slot = pt.slot_bytes;  // bytes per source
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  // each block packs one contiguous range of the unique keys, up to kPackJ
  // per thread held in registers: ONE round of key loads, LDS rank counts,
  // ONE global reservation per owner and the stores (a grid-stride loop of
  // 256-key chunks paid those round trips once per chunk)
  constexpr int kPackJ = 16;
  const int64_t U = *u_count;
  const int64_t per = (U + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < U ? lo + per : U;
  for (int64_t c0 = lo; c0 < hi; c0 += (int64_t)kPackJ * blockDim.x) {  // block-uniform
    if ((int)threadIdx.x < W) lc[threadIdx.x] = 0;
    __syncthreads();
    uint64_t h[kPackJ];
    uint32_t o[kPackJ];
    int lp[kPackJ];
#pragma unroll
    for (int j = 0; j < kPackJ; ++j) {
      const int64_t u = c0 + threadIdx.x + (int64_t)j * blockDim.x;
      h[j] = u < hi ? uniq_h[u] : 0;
    }
#pragma unroll
    for (int j = 0; j < kPackJ; ++j) {
      const int64_t u = c0 + threadIdx.x + (int64_t)j * blockDim.x;
      o[j] = owner_of(h[j], (uint32_t)W);
      lp[j] = u < hi ? atomicAdd(&lc[o[j]], 1) : -1;
    }
    __syncthreads();
    if ((int)threadIdx.x < W) lb[threadIdx.x] = lc[threadIdx.x] ? atomicAdd(&ocnt[threadIdx.x], lc[threadIdx.x]) : 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPackJ; ++j) {
      const int64_t u = c0 + threadIdx.x + (int64_t)j * blockDim.x;
      if (lp[j] < 0) continue;
      const int64_t p = (int64_t)lb[o[j]] + lp[j];
      if (p < cap) {
        // system-coherent 8-B store into the owner's inbox (per-lane owner:
        // a flat store carrying sc0 sc1, no uniform base for a buffer resource)
        __hip_atomic_store(reinterpret_cast<uint64_t*>(slot_ptr(pt, (int)o[j], sl, 0, me)) + p, h[j],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        send_index[u] = (int64_t)o[j] * cap + p;
      } else {
        send_index[u] = -1;
        atomicOr(overflow, 1);
      }
    }
    __syncthreads();  // lc / lb are reused by the next range
  }
  // every block's reservations precede its release + arrival, so the last
  // block announces the final per-owner counts
  signal(pt, epoch, 0, ocnt, &s_last, cap);
  const bool ok = wait_all(pt, epoch, 0, s_cnt, &s_ok);
  for (int src = 0; src < W; ++src) {
    int64_t have = ok ? (int64_t)s_cnt[src] * 8 : 0;
    have = have < cap * 8 ? have : cap * 8;
    if (rcounts && tid == 0) rcounts[src] = ok ? s_cnt[src] : 0;
    uint64_t* d = dst + src * cap;
    put_bytes<false, true>(reinterpret_cast<unsigned char*>(d), slot_ptr(pt, me, sl, 0, src), have, tid, nth);
    for (int64_t i = (have >> 3) + tid; i < cap; i += nth) d[i] = ~0ull;
  }
  (void)slot;
  depart(pt, epoch);
}

// The sharded pull's answer exchange with the owner's probe + gather fused
// into its put phase: entry i < rcnt[src] of the received keys recv[src][i]
// is probed in the table (one thread per key, table_probe.h) and its pull
// record (kPullHead + dim floats, zero padded to rec floats) is written
// straight into peer src's inbox slot at record i; rows[src * cap + i] gets
// the row (-1 for missing keys and for every padding entry: the owner-side
// push reads the whole array).  Each peer receives as many answers as it sent
// keys (the counts ride in the flags again); the receive side copies them out
// to dst [world][cap][rec] like k_ipc_exchange.  One launch instead of probe
// + gather into an answer buffer + exchange of that buffer.
// Reference: heter_comm_inl.h:1117-1171 (the owner-side pull + walk back).
__global__ __launch_bounds__(256) void k_ipc_answer_exchange(IpcPeers pt, TableDev t,
                                                             const uint64_t* __restrict__ recv,
                                                             const int32_t* __restrict__ rcnt, int64_t cap, int rec,
                                                             int64_t* __restrict__ rows, float* __restrict__ dst) {
  __shared__ uint64_t s_epoch;
  __shared__ int s_last, s_ok;
  __shared__ int s_cnt[kIpcMaxRanks];
  const int W = pt.world, me = pt.rank;
  if (threadIdx.x == 0) s_epoch = __hip_atomic_load(pt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint64_t epoch = s_epoch;
  const int sl = (int)(epoch % (uint64_t)pt.depth);
  const int64_t rec_bytes = (int64_t)rec * 4;
  const int64_t per_slot = pt.slot_bytes / rec_bytes;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  const int P = pull_width(t.dim);
  // kAnsJ keys per thread and round: their bucket lines, then their rows, are
  // loaded together (table_probe_thread_n), so a thread pays two or three
  // memory round trips per kAnsJ keys instead of per key
  constexpr int kAnsJ = 4;
  const int rq = rec >> 2;  // float4 per record
  for (int src = 0; src < W; ++src) {
    int64_t n = rcnt[src];
    n = n < 0 ? 0 : (n > cap ? cap : n);
    n = n > per_slot ? per_slot : n;
    const __amdgpu_buffer_rsrc_t ro = inbox_rsrc(slot_ptr(pt, src, sl, 0, me), pt.slot_bytes);
    for (int64_t i = n + tid; i < cap; i += nth) rows[src * cap + i] = -1;  // padding entries
    for (int64_t i0 = 0; i0 < n; i0 += nth * kAnsJ) {
      uint64_t key[kAnsJ];
      int64_t r[kAnsJ];
#pragma unroll
      for (int j = 0; j < kAnsJ; ++j) {
        const int64_t i = i0 + tid + nth * j;
        key[j] = i < n ? recv[src * cap + i] : kEmptyKey;
      }
      table_probe_thread_n<kAnsJ>(t, key, r);
#pragma unroll
      for (int j = 0; j < kAnsJ; ++j) {
        const int64_t i = i0 + tid + nth * j;
        if (i < n) rows[src * cap + i] = r[j];
      }
      // rec % 4 == 0 and the row stride % 4 == 0 (host checks): 16-B loads
      // of every record first, then system-coherent stores into the inbox
      for (int c = 0; c < rq; c += 4) {
        float4 x[kAnsJ][4];
#pragma unroll
        for (int j = 0; j < kAnsJ; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cc = (c + q) * 4;
            x[j][q] = (r[j] >= 0 && c + q < rq)
                          ? reinterpret_cast<const float4*>(t.values + r[j] * (int64_t)t.stride)[c + q]
                          : make_float4(0.f, 0.f, 0.f, 0.f);
            if (cc + 0 >= P) x[j][q].x = 0.f;
            if (cc + 1 >= P) x[j][q].y = 0.f;
            if (cc + 2 >= P) x[j][q].z = 0.f;
            if (cc + 3 >= P) x[j][q].w = 0.f;
          }
#pragma unroll
        for (int j = 0; j < kAnsJ; ++j) {
          const int64_t i = i0 + tid + nth * j;
          if (i >= n) continue;
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (c + q < rq)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4c, x[j][q]), ro,
                                                     (int)((i * rec + (c + q) * 4) * 4), 0, kSys);
        }
      }
    }
  }
  signal(pt, epoch, 0, rcnt, &s_last, per_slot < cap ? per_slot : cap);
  const bool ok = wait_all(pt, epoch, 0, s_cnt, &s_ok);
  for (int src = 0; src < W; ++src) {
    int64_t have = ok ? (int64_t)s_cnt[src] * rec_bytes : 0;
    have = have < pt.slot_bytes ? have : pt.slot_bytes;
    put_bytes<false, true>(reinterpret_cast<unsigned char*>(dst + src * cap * rec), slot_ptr(pt, me, sl, 0, src), have,
                           tid, nth);
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
      put_bytes<true, false>(slot_ptr(pt, p, sl, 0, me), reinterpret_cast<const unsigned char*>(src), n * 4, tid, nth);
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
      put_bytes<true, false>(slot_ptr(pt, p, sl, 0, me), reinterpret_cast<const unsigned char*>(src + a0), (a1 - a0) * 4, tid,
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
      const __amdgpu_buffer_rsrc_t r = inbox_rsrc(slot_ptr(pt, me, sl, 0, p), pt.slot_bytes);
      const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i4 << 4), 0, kSys));
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s = ok ? make_float4(s.x * scale, s.y * scale, s.z * scale, s.w * scale) : make_float4(qnan, qnan, qnan, qnan);
    for (int p = 0; p < W; ++p) {
      const __amdgpu_buffer_rsrc_t r = inbox_rsrc(slot_ptr(pt, p, sl, 1, me), pt.slot_bytes);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4c, s), r, (int)(i4 << 4), 0, kSys);
    }
  }
  signal(pt, epoch, 1, nullptr, &s_last);
  ok = wait_all(pt, epoch, 1, s_cnt, &s_ok) && ok;
  for (int q = 0; q < W; ++q) {  // gather: chunk q of every rank's result into out
    const int64_t a0 = q * cs, a1 = (q + 1) * cs < n ? (q + 1) * cs : n;
    if (a1 <= a0) continue;
    const float* g = reinterpret_cast<const float*>(slot_ptr(pt, me, sl, 1, q));
    if (ok) {
      put_bytes<false, true>(reinterpret_cast<unsigned char*>(out + a0), reinterpret_cast<const unsigned char*>(g),
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

void launch_ipc_pack_exchange(const IpcPeers& pt, const uint64_t* uniq_h, const int32_t* u_count, int64_t cap,
                              int64_t* send_index, int32_t* ocnt, int32_t* overflow, uint64_t* dst, int32_t* rcounts,
                              int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_pack_exchange, dim3(blocks), dim3(256), 0, s, pt, uniq_h, u_count, cap, send_index, ocnt,
                     overflow, dst, rcounts);
}

void launch_ipc_answer_exchange(const IpcPeers& pt, const TableDev& t, const uint64_t* recv, const int32_t* rcnt,
                                int64_t cap, int rec, int64_t* rows, float* dst, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_answer_exchange, dim3(blocks), dim3(256), 0, s, pt, t, recv, rcnt, cap, rec, rows, dst);
}

void launch_ipc_allreduce(const IpcPeers& pt, const float* src, float* out, int64_t n, float scale, bool two_phase,
                          int blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_ipc_allreduce, dim3(blocks), dim3(256), 0, s, pt, src, out, n, scale, two_phase ? 1 : 0);
}

}  // namespace pbx
