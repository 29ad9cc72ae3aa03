// Deterministic embedding backward (no float atomics): dtok[ids[t]] += dout[t], dpos[pos[t]] +=
// dout[t] (reference: the embedding_dense_backward of the two nn.Embedding lookups,
// /root/reference/models/gpt.py:177-185; SURVEY.md §2.5 "deterministic scatter-add bwd").
//
// The atomic scatter (misc.hip: emb_bwd_kernel) adds 2 x T x D f32 values at the chip's
// memory-side atomic rate (~1.3 TB/s) and in an arbitrary order, so the gradient of a token that
// occurs more than once changes in its last bits from run to run.  Here each table is done as
//   1. (key, row) pairs: key = the token id (or position), row = 0 .. T-1;
//   2. a stable LSD radix sort of the pairs by key (hipcub / rocPRIM) -- rows of one key stay
//      in ascending order;
//   3. one wave per sorted position; the wave that starts a run of equal keys sums that run's
//      dout rows in sorted (= row) order in registers and adds the sum to the table row with
//      plain loads / stores: it is the only writer of that row (runs longer than a 64-row
//      chunk are summed chunk by chunk and the partial sums added in order by a second pass).
// The result is bitwise reproducible for any launch order; dout is read once per table with
// 16-B loads, the tables written once per distinct key.
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace dpc {

struct EmbBwdArgs {
  const long long* ids;  // [T]
  const long long* pos;  // [T]
  const float* dout;     // [T][D] f32
  float* dtok;           // [V][D] f32 (accumulated), or null
  float* dpos;           // [P][D] f32 (accumulated), or null
  void* ws;              // workspace (dpc_embedding_bwd_ws bytes)
  unsigned long long ws_bytes;
  int T, D, V, P;
};

// the workspace: keys in / out, rows in / out (T ints each), then hipcub's temporary storage
static size_t eb_sort_bytes(int T) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const int*)nullptr, (int*)nullptr, (const int*)nullptr,
                                     (int*)nullptr, T, 0, 32);
  return tmp;
}
static size_t eb_align(size_t x) { return (x + 255) & ~size_t(255); }

__global__ __launch_bounds__(256) void eb_keys_kernel(const long long* src, int T, int n_keys, int* keys,
                                                      int* rows) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= T) return;
  const long long k = src[t];
  keys[t] = (k >= 0 && k < n_keys) ? (int)k : n_keys;  // out-of-range ids sort last, skipped
  rows[t] = t;
}

// Runs are cut at every EB_CH-th sorted position so no wave sums more than EB_CH rows (a
// frequent token of real text has thousands; the position table's runs are one row per sequence:
// 64 at GPT-2 small B = 64, where EB_CH = 64 left 1,023 waves summing 64 rows each, latency-bound:
// 230 us per step against 125 at EB_CH = 8, bench/emb_bwd_time.py, profiles/r5_emb/).  One wave per sorted position i that starts a
// piece (a run start, or a chunk boundary inside a run).  A run that fits in its chunk is added
// to the table by its start wave; a run that crosses boundaries leaves per-chunk partial sums
// -- part[2 c] its first piece (the last run starting in chunk c), part[2 c + 1] the piece
// continuing at chunk c's first position -- and eb_runsum_kernel adds them in chunk order.
// Rows are read in groups of 8 / 4 / 2 / 1, all of a group's loads issued before its adds, in row order, so
// every sum has a fixed order: bitwise reproducible.
constexpr int EB_CH = 8;

// G rows (sorted positions j .. j+G-1, all of the run) summed into acc in row order: all G x NV
// loads issued before the first add, none under a branch (a load under a branch is waited for
// with vmcnt(0) at the join: G x NV serialized round trips); a lane past the row end re-reads
// the last chunk and never stores it
template <int NV, int G>
__device__ __forceinline__ void eb_add_group(float4 (&acc)[NV], const int* rows, const float* dout, int j, int D,
                                             int lane) {
  const int nv4 = D >> 2;
  float4 x[G][NV];
#pragma unroll
  for (int u = 0; u < G; ++u) {
    const float4* src = reinterpret_cast<const float4*>(dout + (long long)rows[j + u] * D);
#pragma unroll
    for (int v = 0; v < NV; ++v) x[u][v] = src[min(lane + 64 * v, nv4 - 1)];
  }
#pragma unroll
  for (int u = 0; u < G; ++u)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      acc[v].x += x[u][v].x; acc[v].y += x[u][v].y; acc[v].z += x[u][v].z; acc[v].w += x[u][v].w;
    }
}

// the rows of key k at sorted positions j0 .. jend-1 (a run's piece: <= EB_CH positions), in
// groups of 8 / 4 / 2 / 1 by the piece's length -- a random token's run is mostly ONE row, and
// a fixed group of 8 loaded 8 (the old form: conditionally, one round trip each)
template <int NV>
__device__ __forceinline__ void eb_add_rows(float4 (&acc)[NV], const int* keys, const int* rows, const float* dout,
                                            int j0, int jend, int k, int D, int lane) {
  int n = 0;
  while (j0 + n < jend && keys[j0 + n] == k) ++n;  // (wave-uniform: scalar loads)
  int j = j0;
  const int end = j0 + n;
  if constexpr (NV <= 4) {
    for (; j + 8 <= end; j += 8) eb_add_group<NV, 8>(acc, rows, dout, j, D, lane);
  }
  for (; j + 4 <= end; j += 4) eb_add_group<NV, 4>(acc, rows, dout, j, D, lane);
  if (j + 2 <= end) {
    eb_add_group<NV, 2>(acc, rows, dout, j, D, lane);
    j += 2;
  }
  if (j < end) eb_add_group<NV, 1>(acc, rows, dout, j, D, lane);
}

template <int NV>
__device__ __forceinline__ void eb_store_add(float* dst_row, const float4 (&acc)[NV], int D, int lane, bool add) {
  float4* dst = reinterpret_cast<float4*>(dst_row);
  const int nv4 = D >> 2;
  float4 t[NV];
  if (add) {  // (all of the row's reads issued before the first add: unconditional, clamped)
#pragma unroll
    for (int v = 0; v < NV; ++v) t[v] = dst[min(lane + 64 * v, nv4 - 1)];
  }
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int c = lane + 64 * v;
    float4 o = acc[v];
    if (add) {
      o.x += t[v].x; o.y += t[v].y; o.z += t[v].z; o.w += t[v].w;
    }
    if (c < nv4) dst[c] = o;
  }
}

template <int NV>
__global__ __launch_bounds__(256) void eb_segsum_kernel(const int* keys, const int* rows, const float* dout,
                                                        float* table, float* part, int T, int D, int n_keys) {
  const int lane = threadIdx.x & 63;
  const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (i >= T) return;
  const int k = keys[i];
  const bool run_start = i == 0 || keys[i - 1] != k;
  if (k >= n_keys || !(run_start || i % EB_CH == 0)) return;  // not the start of a piece
  const int cend = min(T, (i / EB_CH + 1) * EB_CH);            // the piece ends at the chunk end
  float4 acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = make_float4(0.f, 0.f, 0.f, 0.f);
  eb_add_rows<NV>(acc, keys, rows, dout, i, cend, k, D, lane);
  const bool crosses = cend < T && keys[cend] == k;
  if (run_start && !crosses) {
    eb_store_add<NV>(table + (long long)k * D, acc, D, lane, true);  // the run's only piece
  } else {
    const int c = i / EB_CH;
    eb_store_add<NV>(part + (long long)(2 * c + (run_start ? 0 : 1)) * D, acc, D, lane, false);
  }
}

// one wave per run start whose run crosses a chunk boundary: its first piece, then the
// continuation pieces of the following chunks, in order
template <int NV>
__global__ __launch_bounds__(256) void eb_runsum_kernel(const int* keys, const float* part, float* table, int T, int D,
                                                        int n_keys) {
  const int lane = threadIdx.x & 63;
  const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (i >= T) return;
  const int k = keys[i];
  if (k >= n_keys || (i > 0 && keys[i - 1] == k)) return;
  int c = i / EB_CH;
  int cend = min(T, (c + 1) * EB_CH);
  if (cend >= T || keys[cend] != k) return;  // fits in its chunk: done by eb_segsum_kernel
  const int nv4 = D >> 2;
  float4 acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v)  // (clamped, unconditional loads; lanes past the row end never store)
    acc[v] = reinterpret_cast<const float4*>(part + (long long)(2 * c) * D)[min(lane + 64 * v, nv4 - 1)];
  for (++c; c * EB_CH < T && keys[c * EB_CH] == k; ++c) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float4 t = reinterpret_cast<const float4*>(part + (long long)(2 * c + 1) * D)[min(lane + 64 * v, nv4 - 1)];
      acc[v].x += t.x; acc[v].y += t.y; acc[v].z += t.z; acc[v].w += t.w;
    }
  }
  eb_store_add<NV>(table + (long long)k * D, acc, D, lane, true);
}

}  // namespace dpc

using namespace dpc;

// bytes of workspace dpc_embedding_bwd_sorted needs for T rows of width D
static size_t eb_part_bytes(int T, int D) { return eb_align((size_t)2 * ((T + EB_CH - 1) / EB_CH) * D * 4); }
DPC_API unsigned long long dpc_embedding_bwd_ws(int T, int D) {
  if (T <= 0) return 0;
  return (unsigned long long)(4 * eb_align((size_t)T * 4) + eb_part_bytes(T, D) + eb_align(eb_sort_bytes(T)));
}

static int eb_table(const EmbBwdArgs* a, const long long* src, float* table, int n_keys, hipStream_t stream) {
  const int T = a->T;
  char* w = static_cast<char*>(a->ws);
  int* keys_in = reinterpret_cast<int*>(w);
  int* keys_out = reinterpret_cast<int*>(w + eb_align((size_t)T * 4));
  int* rows_in = reinterpret_cast<int*>(w + 2 * eb_align((size_t)T * 4));
  int* rows_out = reinterpret_cast<int*>(w + 3 * eb_align((size_t)T * 4));
  float* part = reinterpret_cast<float*>(w + 4 * eb_align((size_t)T * 4));
  void* tmp = w + 4 * eb_align((size_t)T * 4) + eb_part_bytes(T, a->D);
  size_t tmp_bytes = eb_sort_bytes(T);
  hipLaunchKernelGGL(eb_keys_kernel, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, stream, src, T, n_keys,
                     keys_in, rows_in);
  int bits = 1;
  while (bits < 31 && (1ll << bits) <= (long long)n_keys) ++bits;  // keys in [0, n_keys]
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, rows_in, rows_out, T, 0,
                                                    bits, stream);
  if (e != hipSuccess) return (int)e;
  const dim3 grid((unsigned)((T + 3) / 4));
#define EB_CASE(NV)                                                                                        \
  case NV:                                                                                                 \
    hipLaunchKernelGGL(eb_segsum_kernel<NV>, grid, dim3(256), 0, stream, keys_out, rows_out, a->dout, table, part, \
                       T, a->D, n_keys);                                                                   \
    hipLaunchKernelGGL(eb_runsum_kernel<NV>, grid, dim3(256), 0, stream, keys_out, part, table, T, a->D, n_keys); \
    break;
  switch ((a->D + 255) / 256) {
    EB_CASE(1) EB_CASE(2) EB_CASE(3) EB_CASE(4) EB_CASE(5) EB_CASE(6) EB_CASE(7) EB_CASE(8)
    default: return (int)hipErrorInvalidValue;
  }
#undef EB_CASE
  return (int)hipGetLastError();
}

// Requirements: D % 4 == 0, D <= 2048, 16-B aligned dout / tables, ws of dpc_embedding_bwd_ws(T)
// bytes (256-B aligned).  The two tables are done one after the other (the workspace is reused).
DPC_API int dpc_embedding_bwd_sorted(const EmbBwdArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->D % 4 || a->D > 2048 || !a->ws || a->ws_bytes < dpc_embedding_bwd_ws(a->T, a->D) || ((uintptr_t)a->ws % 256) ||
      ((uintptr_t)a->dout % 16))
    return (int)hipErrorInvalidValue;
  if (a->dtok) {
    const int rc = eb_table(a, a->ids, a->dtok, a->V, stream);
    if (rc) return rc;
  }
  if (a->dpos) {
    const int rc = eb_table(a, a->pos, a->dpos, a->P, stream);
    if (rc) return rc;
  }
  return 0;
}
