// Intra-node collectives by direct peer access over xGMI: every rank exports a
// staging buffer and a flag array through HIP IPC, every rank maps the others', and one kernel
// per collective moves the data with ordinary vector loads from the peers' HBM.  On an 8 x MI355X
// node each GPU has a link to each of its 7 peers, so a two-shot all-reduce -- every rank sums its
// 1/W shard straight out of the 7 peers' buffers (reduce-scatter), then copies the 7 other summed
// shards back out of their owners' buffers (all-gather) -- drives all 7 links at once, where a ring
// drives one; each rank reads 2 (W - 1) / W of the buffer, the ring's bus volume.  The same kernel
// does reduce-scatter (the first shot), all-gather (the second) and broadcast.
//
// Synchronisation is per workgroup: workgroup g of every rank handles the same sub-slices (of every
// shard) and meets only workgroup g of the other ranks, through monotonic flag values in the
// receivers' flag arrays (uncached memory: hipDeviceMallocUncached) -- no grid-wide barrier, no
// host round trip, and the whole collective is one kernel, so a HIP graph captures it.
//   * epoch: each workgroup keeps its own collective counter in device memory (ep[g]), read at its
//     start and advanced at its end, so a replayed graph runs a new collective every time.  The
//     staging buffer has two halves used alternately (epoch parity): a rank rewrites a half only
//     after the barrier of the NEXT collective, and a peer workgroup at that barrier means the
//     peer's previous collective kernel -- every workgroup of it, whatever sub-slices they read --
//     has finished (its kernels run in stream order).  (Point-to-point has no such ordering: a
//     sender waits for the ACKs of all of the receiver's workgroups before it reuses a half.)
//   * barrier value of phase k in epoch e: 2 e + k (k = 1, 2), so flags never need resetting.
//   * every wait is bounded (spin_limit polls): a peer that never arrives sets *error and the
//     kernel finishes -- the host raises on the error word (IpcComm.check) instead of hanging.
//   * sums are taken in rank order 0 .. W-1 in f32 by the shard's owner, and every rank copies the
//     owner's result: all ranks end with bitwise-identical buffers (DDP replicas stay identical).
// Peer data moves with system-scope (sc0 sc1) buffer loads and stores, so no stale line of a
// peer's buffer survives in this GPU's caches between the phases of one kernel; shards and
// sub-slices are whole multiples of 64 elements (>= 128 B), so no cache line straddles two regions
// written in different phases.
#include "common.h"

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dpc {

typedef unsigned v4u32_t __attribute__((ext_vector_type(4)));

constexpr int IPC_MAXW = 8;
// workgroups per collective (flag columns).  Few on purpose: a waiting workgroup holds a slot on
// its CU, and a persistent GEMM launched beside it (one 512-register wave per SIMD) cannot place
// its workgroup on that CU until the wait ends.  Across GPUs that only delays this GPU's own GEMM
// until the peer arrives; with two ranks sharing ONE GPU (the tests' rehearsal) the other rank's
// GEMM may be the one the waiting workgroups stall, and it must still find CUs free: 64 workgroups
// passed every rehearsal, 256 deadlocked the two-rank DDP step (round-6 job 14).  64 workgroups
// moved 180 GB/s on one GPU (profiles/r6_ipc/).
constexpr int IPC_G = 64;
constexpr int IPC_ALIGN = 64;  // elements: shard / sub-slice granularity

struct IpcCollArgs {
  void* slot[IPC_MAXW];        // every rank's staging buffer (two halves of half_bytes), this rank's at [rank]
  unsigned* flags[IPC_MAXW];   // every rank's flag arrays [3][IPC_MAXW][IPC_G] (uncached; [0]: barriers)
  unsigned* ep;                // this rank's per-workgroup collective counters [IPC_G]
  int* error;                  // set to 1 by a wait that timed out
  const void* in;
  void* out;
  long long n;                 // all-reduce / broadcast: elements; reduce-scatter: output elements;
                               // all-gather: input elements
  long long half_bytes;
  long long spin_limit;
  int op;                      // 0 all-reduce, 1 reduce-scatter, 2 all-gather, 3 broadcast
  int bf16;                    // element type: 1 bf16, 0 f32
  int rank, world, root;
};

enum { IPC_ALLREDUCE = 0, IPC_REDUCE_SCATTER = 1, IPC_ALLGATHER = 2, IPC_BROADCAST = 3 };

// system-scope (sc0 sc1) 16-B buffer accesses: aux = SC0 | SC1
constexpr int IPC_SYS = 1 | 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ipc_rsrc(const void* base, long long bytes) {
  const unsigned nrec = (unsigned)(bytes > 0xffffffffll ? 0xffffffffll : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nrec, 0x00020000);
}

// elements [lo, hi) of sub-slice g of a region of `len` elements (len a multiple of IPC_ALIGN)
__device__ __forceinline__ void ipc_sub(long long len, int g, long long& lo, long long& hi) {
  const long long blocks = len / IPC_ALIGN;
  const long long per = (blocks + IPC_G - 1) / IPC_G;
  lo = min(len, (long long)g * per * IPC_ALIGN);
  hi = min(len, lo + per * IPC_ALIGN);
}

__device__ __forceinline__ void ipc_unpack(const uint4& v, bool bf, float (&f)[8]) {
  if (bf) {
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    f[0] = __uint_as_float(v.x);
    f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z);
    f[3] = __uint_as_float(v.w);
  }
}

__device__ __forceinline__ uint4 ipc_pack(const float (&f)[8], bool bf) {
  uint4 v;
  if (bf) {
    v.x = pack2bf(f[0], f[1]);
    v.y = pack2bf(f[2], f[3]);
    v.z = pack2bf(f[4], f[5]);
    v.w = pack2bf(f[6], f[7]);
  } else {
    v.x = __float_as_uint(f[0]);
    v.y = __float_as_uint(f[1]);
    v.z = __float_as_uint(f[2]);
    v.w = __float_as_uint(f[3]);
  }
  return v;
}

// element-granular access for the unaligned edges of caller buffers (sys: system-scope, as the
// vector path's peer accesses)
__device__ __forceinline__ float ipc_ld1(const void* p, long long i, bool bf, bool sys) {
  if (bf) {
    const unsigned short* q = static_cast<const unsigned short*>(p) + i;
    const unsigned short v = sys ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : *q;
    return __uint_as_float((unsigned)v << 16);
  }
  const float* q = static_cast<const float*>(p) + i;
  return sys ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : *q;
}
__device__ __forceinline__ void ipc_st1(void* p, long long i, float v, bool bf, bool sys) {
  if (bf) {
    unsigned short* q = static_cast<unsigned short*>(p) + i;
    const unsigned short w = (unsigned short)(pack2bf(v, 0.f) & 0xffffu);
    if (sys) __hip_atomic_store(q, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *q = w;
  } else {
    float* q = static_cast<float*>(p) + i;
    if (sys) __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *q = v;
  }
}

// copy elements [lo, hi) from src (+ src_off) to dst (+ dst_off): 16-B vectors where both sides are
// aligned, elements otherwise.  sys_src / sys_dst: system-scope accesses (peer or peer-visible data)
__device__ void ipc_copy(const void* src, long long src_off, bool sys_src, void* dst, long long dst_off, bool sys_dst,
                         long long lo, long long hi, bool bf) {
  const int es = bf ? 2 : 4, E = 16 / es;
  const bool al = (((uintptr_t)src + src_off * es) % 16 == 0) && (((uintptr_t)dst + dst_off * es) % 16 == 0) &&
                  (lo % E == 0);
  long long i = lo;
  if (al) {
    const long long nv = (hi - lo) / E;
    const char* sb = static_cast<const char*>(src) + (src_off + lo) * es;
    char* db = static_cast<char*>(dst) + (dst_off + lo) * es;
    const __amdgpu_buffer_rsrc_t rs = ipc_rsrc(sb, nv * 16), rd = ipc_rsrc(db, nv * 16);
    for (long long v = threadIdx.x; v < nv; v += blockDim.x) {
      const int off = (int)(v * 16);
      uint4 x = sys_src ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, IPC_SYS))
                        : __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      if (sys_dst) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, x), rd, off, 0, IPC_SYS);
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, x), rd, off, 0, 0);
    }
    i = lo + nv * E;
  }
  for (long long k = i + threadIdx.x; k < hi; k += blockDim.x) {
    ipc_st1(dst, dst_off + k, ipc_ld1(src, src_off + k, bf, sys_src), bf, sys_dst);
  }
}

// dst[dst_off + k] = sum over ranks p of slot_p[src_off + k] (in rank order), k in [lo, hi); every
// slot is 16-B aligned at IPC_ALIGN granularity, dst may not be
__device__ void ipc_sum(const IpcCollArgs& a, long long half_off, long long src_off, void* dst, long long dst_off,
                        bool dst_sys, void* dst2, long long dst2_off, long long lo, long long hi, bool bf) {
  const int es = bf ? 2 : 4, E = 16 / es;
  const int W = a.world;
  const bool al = (((uintptr_t)dst + dst_off * es) % 16 == 0) && (dst2 == nullptr || ((uintptr_t)dst2 + dst2_off * es) % 16 == 0);
  long long i = lo;
  if (al) {
    const long long nv = (hi - lo) / E;
    __amdgpu_buffer_rsrc_t rs[IPC_MAXW];
#pragma unroll
    for (int p = 0; p < IPC_MAXW; ++p)
      if (p < W) rs[p] = ipc_rsrc(static_cast<const char*>(a.slot[p]) + half_off + (src_off + lo) * es, nv * 16);
    const __amdgpu_buffer_rsrc_t rd = ipc_rsrc(static_cast<char*>(dst) + (dst_off + lo) * es, nv * 16);
    for (long long v = threadIdx.x; v < nv; v += blockDim.x) {
      const int off = (int)(v * 16);
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      uint4 x[IPC_MAXW];
#pragma unroll
      for (int p = 0; p < IPC_MAXW; ++p)  // all W loads in flight before the adds
        if (p < W) x[p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs[p], off, 0, IPC_SYS));
#pragma unroll
      for (int p = 0; p < IPC_MAXW; ++p) {
        if (p < W) {
          float f[8];
          ipc_unpack(x[p], bf, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += f[e];
        }
      }
      const uint4 y = ipc_pack(acc, bf);
      if (dst_sys) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, y), rd, off, 0, IPC_SYS);
      else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, y), rd, off, 0, 0);
      if (dst2) *reinterpret_cast<uint4*>(static_cast<char*>(dst2) + (dst2_off + lo + v * E) * es) = y;
    }
    i = lo + nv * E;
  }
  for (long long k = i + threadIdx.x; k < hi; k += blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < W; ++p) s += ipc_ld1(static_cast<const char*>(a.slot[p]) + half_off, src_off + k, bf, true);
    ipc_st1(dst, dst_off + k, s, bf, dst_sys);
    if (dst2) ipc_st1(dst2, dst2_off + k, s, bf, false);
  }
}

// the workgroup's barrier with workgroup g of every other rank at flag value v: publish this
// workgroup's writes (system scope), raise the peers' flags, wait for theirs
__device__ void ipc_barrier(const IpcCollArgs& a, int g, unsigned v) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world && t != a.rank)
    __hip_atomic_store(a.flags[t] + a.rank * IPC_G + g, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t < a.world && t != a.rank) {
    const unsigned* f = a.flags[a.rank] + t * IPC_G + g;
    long long n = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - v) < 0) {
      if (++n > a.spin_limit) {
        __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void ipc_coll_kernel(IpcCollArgs a) {
  const int g = blockIdx.x;
  const bool bf = a.bf16 != 0;
  const int es = bf ? 2 : 4;
  const int W = a.world, r = a.rank;
  const unsigned e = a.ep[g];
  const long long half_off = (long long)(e & 1u) * a.half_bytes;
  char* mine = static_cast<char*>(a.slot[r]) + half_off;
  long long lo, hi;
  if (a.op == IPC_ALLREDUCE || a.op == IPC_REDUCE_SCATTER) {
    // shard c (a multiple of IPC_ALIGN): all-reduce pads n up to W c; reduce-scatter's input is W x n
    const long long n = a.n;
    const long long c = a.op == IPC_ALLREDUCE ? ((n + W - 1) / W + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN
                                              : (n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN;
    const long long total = a.op == IPC_ALLREDUCE ? n : (long long)W * n;  // valid input elements
    const long long in_c = a.op == IPC_ALLREDUCE ? c : n;                  // input stride between shards
    // phase 0: this rank's input into its slot, shard by shard (sub-slice g of each)
    ipc_sub(c, g, lo, hi);
    for (int s = 0; s < W; ++s) {
      const long long b = (long long)s * in_c;  // first input element of shard s
      const long long h = min(hi, max(lo, min(c, total - b)));
      if (h > lo) ipc_copy(a.in, b, false, mine, (long long)s * c, true, lo, h, bf);
    }
    ipc_barrier(a, g, 2 * e + 1);
    // phase 1: shard r summed over the ranks' slots (its valid part), kept in this rank's slot for
    // the second shot and written to the output
    const long long b = (long long)r * in_c;
    const long long h = min(hi, max(lo, min(c, total - b)));
    if (h > lo) {
      // (all-reduce: the sum overwrites this rank's own copy of shard r, which no peer reads in
      // this phase -- each reads only its own shard -- and which the peers copy in phase 2)
      if (a.op == IPC_ALLREDUCE) ipc_sum(a, half_off, (long long)r * c, mine, (long long)r * c, true, a.out, b, lo, h, bf);
      else ipc_sum(a, half_off, (long long)r * c, a.out, 0, false, nullptr, 0, lo, h, bf);
    }
    if (a.op == IPC_ALLREDUCE) {
      ipc_barrier(a, g, 2 * e + 2);
      // phase 2: the other ranks' summed shards, out of their slots
      for (int s = 0; s < W; ++s) {
        if (s == r) continue;
        const long long bs = (long long)s * c;
        const long long hs = min(hi, max(lo, min(c, n - bs)));
        if (hs > lo) ipc_copy(a.slot[s], half_off / es + bs, true, a.out, bs, false, lo, hs, bf);
      }
    }
  } else if (a.op == IPC_ALLGATHER) {
    const long long n = a.n;
    const long long c = (n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN;
    ipc_sub(c, g, lo, hi);
    const long long h = min(hi, n);
    if (h > lo) ipc_copy(a.in, 0, false, mine, 0, true, lo, h, bf);
    ipc_barrier(a, g, 2 * e + 1);
    for (int s = 0; s < W; ++s)
      if (h > lo) {
        if (s == r) ipc_copy(a.in, 0, false, a.out, (long long)s * n, false, lo, h, bf);
        else ipc_copy(a.slot[s], half_off / es, true, a.out, (long long)s * n, false, lo, h, bf);
      }
  } else {  // broadcast from a.root (in == out on every rank)
    const long long n = a.n;
    const long long c = (n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN;
    ipc_sub(c, g, lo, hi);
    const long long h = min(hi, n);
    if (r == a.root && h > lo) ipc_copy(a.in, 0, false, mine, 0, true, lo, h, bf);
    ipc_barrier(a, g, 2 * e + 1);
    if (r != a.root && h > lo) ipc_copy(a.slot[a.root], half_off / es, true, a.out, 0, false, lo, h, bf);
  }
  // the next collective of this workgroup (all its threads have read e)
  __syncthreads();
  if (threadIdx.x == 0) a.ep[g] = e + 1u;
}

// ---------------------------------------------------------------- point-to-point
// A grouped exchange (the pipeline's activations / gradients): per ordered pair (p -> q) a channel
// of two buffered messages in p's p2p staging buffer (half = message parity, region q of the half)
// and two monotonic counters per workgroup: READY (raised by p in q's flag array after a message's
// bytes are in place) and ACK (raised by q in p's array after it copied them out).  Workgroup g
// moves sub-slice g of every message and meets only workgroup g of the peer, as the collectives
// do.  A send waits only when its channel already holds two unconsumed messages, so a schedule
// that is deadlock-free under RCCL's blocking sends (parallel/pipeline.py:p2p_deadlock_free) is
// deadlock-free here; every wait is bounded like the barriers'.
constexpr int IPC_P2P_MAX = 8;

struct IpcP2PArgs {
  void* slot[IPC_MAXW];       // every rank's p2p staging buffer: 2 halves x world regions of region_bytes
  unsigned* flags[IPC_MAXW];  // every rank's flag arrays: [0] barriers, [1] READY, [2] ACK
  unsigned* cnt;              // this rank's counters [2][IPC_MAXW][IPC_G]: messages sent to / received from
  int* error;
  const void* send_ptr[IPC_P2P_MAX];
  void* recv_ptr[IPC_P2P_MAX];
  long long send_n[IPC_P2P_MAX];  // 2-byte units
  long long recv_n[IPC_P2P_MAX];
  int send_peer[IPC_P2P_MAX];
  int recv_peer[IPC_P2P_MAX];
  long long region_bytes, spin_limit;
  int nsend, nrecv, rank, world;
};

__device__ void ipc_wait(const unsigned* f, unsigned v, long long limit, int* error) {
  long long n = 0;
  while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - v) < 0) {
    if (++n > limit) {
      __hip_atomic_store(error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ __launch_bounds__(256) void ipc_p2p_kernel(IpcP2PArgs a) {
  const int g = blockIdx.x, r = a.rank;
  constexpr int FL = IPC_MAXW * IPC_G;  // one flag array
  unsigned* sent = a.cnt;
  unsigned* rcvd = a.cnt + FL;
  long long lo, hi;
  for (int i = 0; i < a.nsend; ++i) {
    const int q = a.send_peer[i];
    const unsigned c = sent[q * IPC_G + g];
    if (c >= 2) {
      // the message two back on this channel copied out of its half by EVERY workgroup of q: two
      // messages of different sizes split into different sub-slices, so this workgroup's part of
      // the new message may overlap another workgroup's part of the old one (one ACK per
      // workgroup of q, all in this rank's array)
      if (threadIdx.x < IPC_G) ipc_wait(a.flags[r] + 2 * FL + q * IPC_G + threadIdx.x, c - 1, a.spin_limit, a.error);
      __syncthreads();
    }
    const long long n = a.send_n[i];
    ipc_sub((n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN, g, lo, hi);
    hi = min(hi, n);
    char* dst = static_cast<char*>(a.slot[r]) + (long long)(c & 1u) * a.world * a.region_bytes + q * a.region_bytes;
    if (hi > lo) ipc_copy(a.send_ptr[i], 0, false, dst, 0, true, lo, hi, true);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.flags[q] + FL + r * IPC_G + g, c + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      sent[q * IPC_G + g] = c + 1u;
    }
    __syncthreads();  // (the next message to q reads the advanced counter)
  }
  for (int i = 0; i < a.nrecv; ++i) {
    const int p = a.recv_peer[i];
    const unsigned c = rcvd[p * IPC_G + g];
    if (threadIdx.x == 0) ipc_wait(a.flags[r] + FL + p * IPC_G + g, c + 1u, a.spin_limit, a.error);
    __syncthreads();
    const long long n = a.recv_n[i];
    ipc_sub((n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN, g, lo, hi);
    hi = min(hi, n);
    const char* src = static_cast<const char*>(a.slot[p]) + (long long)(c & 1u) * a.world * a.region_bytes + r * a.region_bytes;
    if (hi > lo) ipc_copy(src, 0, true, a.recv_ptr[i], 0, false, lo, hi, true);
    __threadfence_system();  // (this workgroup's reads of the message done before the ACK)
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_store(a.flags[p] + 2 * FL + r * IPC_G + g, c + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      rcvd[p * IPC_G + g] = c + 1u;
    }
    __syncthreads();
  }
}

}  // namespace dpc

using namespace dpc;

#define DPC_API extern "C" __attribute__((visibility("default")))

// staging / flag memory: `uncached` allocations (the flag arrays) are hipDeviceMallocUncached, so a
// peer's flag store and this GPU's polling load meet in memory, not in a cache
DPC_API int dpc_ipc_alloc(long long bytes, int uncached, void** out) {
  *out = nullptr;
  hipError_t e = uncached ? hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached)
                          : hipMalloc(out, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*out, 0, (size_t)bytes);
}

DPC_API int dpc_ipc_free(void* p) { return (int)hipFree(p); }

// the 64-byte IPC handle of an allocation
DPC_API int dpc_ipc_handle(void* p, void* handle_out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  __builtin_memcpy(handle_out, &h, sizeof(h));
  return 0;
}

DPC_API int dpc_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

DPC_API int dpc_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

DPC_API int dpc_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

DPC_API int dpc_ipc_coll(const IpcCollArgs* a, hipStream_t stream) {
  if (a->world < 1 || a->world > IPC_MAXW || a->rank < 0 || a->rank >= a->world) return (int)hipErrorInvalidValue;
  if (a->n <= 0) return 0;
  for (int p = 0; p < a->world; ++p)
    if (!a->slot[p] || !a->flags[p]) return (int)hipErrorInvalidValue;  // (a peer not mapped)
  if (!a->in || !a->out || !a->ep || !a->error || a->spin_limit <= 0) return (int)hipErrorInvalidValue;
  if (a->op == IPC_BROADCAST && (a->root < 0 || a->root >= a->world)) return (int)hipErrorInvalidValue;
  const int es = a->bf16 ? 2 : 4, W = a->world;
  // bytes of one half the collective stages (the host chunks larger buffers)
  long long need;
  if (a->op == IPC_ALLREDUCE) {
    const long long c = ((a->n + W - 1) / W + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN;
    need = (long long)W * c * es;
  } else if (a->op == IPC_REDUCE_SCATTER) {
    need = (long long)W * ((a->n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN) * es;
  } else {
    need = ((a->n + IPC_ALIGN - 1) / IPC_ALIGN * IPC_ALIGN) * es;
  }
  if (need > a->half_bytes || a->half_bytes % 256) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ipc_coll_kernel, dim3(IPC_G), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_ipc_p2p(const IpcP2PArgs* a, hipStream_t stream) {
  if (a->world < 1 || a->world > IPC_MAXW || a->rank < 0 || a->rank >= a->world) return (int)hipErrorInvalidValue;
  if (a->nsend < 0 || a->nsend > IPC_P2P_MAX || a->nrecv < 0 || a->nrecv > IPC_P2P_MAX) return (int)hipErrorInvalidValue;
  if (a->nsend + a->nrecv == 0) return 0;
  if (!a->cnt || !a->error || a->spin_limit <= 0 || a->region_bytes % 256) return (int)hipErrorInvalidValue;
  if (!a->slot[a->rank] || !a->flags[a->rank]) return (int)hipErrorInvalidValue;
  for (int i = 0; i < a->nsend; ++i) {
    const int q = a->send_peer[i];
    if (q < 0 || q >= a->world || q == a->rank || !a->flags[q] || (!a->send_ptr[i] && a->send_n[i] > 0))
      return (int)hipErrorInvalidValue;  // (an empty message may carry no pointer)
    if (a->send_n[i] < 0 || a->send_n[i] * 2 > a->region_bytes) return (int)hipErrorInvalidValue;
  }
  for (int i = 0; i < a->nrecv; ++i) {
    const int p = a->recv_peer[i];
    if (p < 0 || p >= a->world || p == a->rank || !a->slot[p] || !a->flags[p] || (!a->recv_ptr[i] && a->recv_n[i] > 0))
      return (int)hipErrorInvalidValue;
    if (a->recv_n[i] < 0 || a->recv_n[i] * 2 > a->region_bytes) return (int)hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(ipc_p2p_kernel, dim3(IPC_G), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_ipc_max_world() { return IPC_MAXW; }
DPC_API int dpc_ipc_p2p_max() { return IPC_P2P_MAX; }
DPC_API int dpc_ipc_groups() { return IPC_G; }
