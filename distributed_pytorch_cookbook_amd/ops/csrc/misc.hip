// Memory-bound training kernels for gfx950: embedding gather / scatter-add, fused
// softmax-cross-entropy (forward + backward in one pass pair), flat AdamW, and the
// bias/activation-backward + column-sum kernel.  All move 16 B per lane.
//
// Reference parity:
//   embedding      models/gpt.py:177-185 (token + learned position embedding, summed, f32 out)
//   cross entropy  main-single.py:95-96  (F.cross_entropy, ignore_index=-100, mean over valid)
//                  + main-single.py:128-131 (eval argmax accuracy) fused into the same pass
//   adamw          main-single.py:42     (torch.optim.AdamW defaults: betas (0.9, 0.999),
//                  eps 1e-8, weight_decay 0.01, decoupled decay) over ONE flat buffer
//   bias/act bwd   gradient of nn.Linear bias + F.relu / gelu (models/gpt.py:34-38)
#include "common.h"
#include <cstdlib>

namespace dpc {

// ------------------------------------------------------------------ embedding
struct EmbArgs {
  const long long* ids;  // [T]
  const long long* pos;  // [T]
  const void* tok;       // [V][D] (f32 or bf16)
  const void* ptab;      // [P][D]
  float* out;            // [T][D] f32
  const float* dout;     // bwd [T][D]
  float* dtok;           // bwd [V][D] f32 (accumulate)
  float* dpos;           // bwd [P][D] f32 (accumulate)
  int T, D, V, P;
  int table_bf16;
};

__global__ __launch_bounds__(256) void emb_fwd_kernel(EmbArgs p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.T) return;
  long long id = p.ids[row], ps = p.pos[row];
  id = id < 0 ? 0 : (id >= p.V ? p.V - 1 : id);
  ps = ps < 0 ? 0 : (ps >= p.P ? p.P - 1 : ps);
  float4* o = reinterpret_cast<float4*>(p.out + row * p.D);
  const int nv4 = p.D >> 2;
  for (int c = lane; c < nv4; c += 64) {
    float4 a, b;
    if (p.table_bf16) {
      const uint2 ua = reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(p.tok) + id * p.D)[c];
      const uint2 ub = reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(p.ptab) + ps * p.D)[c];
      a = make_float4(__uint_as_float(ua.x << 16), __uint_as_float(ua.x & 0xffff0000u),
                      __uint_as_float(ua.y << 16), __uint_as_float(ua.y & 0xffff0000u));
      b = make_float4(__uint_as_float(ub.x << 16), __uint_as_float(ub.x & 0xffff0000u),
                      __uint_as_float(ub.y << 16), __uint_as_float(ub.y & 0xffff0000u));
    } else {
      a = reinterpret_cast<const float4*>(static_cast<const float*>(p.tok) + id * p.D)[c];
      b = reinterpret_cast<const float4*>(static_cast<const float*>(p.ptab) + ps * p.D)[c];
    }
    o[c] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
}

// scatter-add: one wave per token row, each wave-instruction adds 256 contiguous bytes
__global__ __launch_bounds__(256) void emb_bwd_kernel(EmbArgs p) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.T) return;
  long long id = p.ids[row], ps = p.pos[row];
  if (id < 0 || id >= p.V || ps < 0 || ps >= p.P) return;
  const float* g = p.dout + row * p.D;
  float* dt = p.dtok + id * p.D;
  float* dp = p.dpos + ps * p.D;
  for (int c = lane; c < p.D; c += 64) {
    const float v = g[c];
    if (p.dtok) atomicAdd(dt + c, v);
    if (p.dpos) atomicAdd(dp + c, v);
  }
}

// ------------------------------------------------------------------ cross entropy
struct CEArgs {
  const void* logits;          // [T][ld] bf16
  void* dlogits;               // [T][ld] bf16 (may alias logits)
  const long long* targets;    // [T]
  const float* inv_count;      // device scalar: 1 / #valid targets
  float* row_loss;             // [T] f32
  float* row_correct;          // [T] f32 (optional, argmax == target)
  long long ld;
  int T, V;
  int write_grad;
  int ignore_index;
};

__device__ __forceinline__ void ms_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// One workgroup per row.  The block reduction of (max, sum-exp, argmax) and the row's target
// logit; the target logit is captured in the first pass by the thread that owns its chunk
// (dlogits may alias logits, so it must not be re-read once the gradient pass has started).
template <int NW>
__device__ __forceinline__ void ce_block_reduce(float& m, float& s, float& bv, int& bi, float* red_m, float* red_s,
                                                float* red_v, int* red_i) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    ms_combine(m, s, m2, s2);
    const float v2 = __shfl_xor(bv, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (v2 > bv || (v2 == bv && i2 < bi)) { bv = v2; bi = i2; }
  }
  if (lane == 0) { red_m[w] = m; red_s[w] = s; red_v[w] = bv; red_i[w] = bi; }
  __syncthreads();
  m = red_m[0]; s = red_s[0]; bv = red_v[0]; bi = red_i[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) {
    ms_combine(m, s, red_m[i], red_s[i]);
    if (red_v[i] > bv || (red_v[i] == bv && red_i[i] < bi)) { bv = red_v[i]; bi = red_i[i]; }
  }
}

__device__ __forceinline__ void ce_chunk_stats(const uint4& raw, int c, int V, long long tgt, float& m, float& s,
                                               float& bv, int& bi, float* tval) {
  float f[8];
  unpack8(raw, f);
  float cm = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = c * 8 + j;
    if (idx >= V) f[j] = -INFINITY;
    if (idx == tgt) *tval = f[j];
    cm = fmaxf(cm, f[j]);
    if (f[j] > bv) { bv = f[j]; bi = idx; }
  }
  if (cm == -INFINITY) return;  // past the row end
  float cs = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) cs += __expf(f[j] - cm);
  ms_combine(m, s, cm, cs);
}

__device__ __forceinline__ uint4 ce_chunk_grad(const uint4& raw, int c, int V, long long tgt, float lse, float scale) {
  float f[8];
  unpack8(raw, f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int idx = c * 8 + j;
    f[j] = idx < V ? (__expf(f[j] - lse) - (idx == tgt ? 1.f : 0.f)) * scale : 0.f;
  }
  return pack8(f);
}

// Register-resident row (the GPT-2 head: V = 50257 -> 6283 16-B chunks, NC = 16 per thread
// of 512): every chunk is loaded once, all NC loads in flight per thread before any math,
// and the gradient pass runs from registers -- one HBM read of the logits and one write of
// dlogits (the earlier two-pass form re-read each 100 KB row and kept one load in flight per
// wave: 4.3 TB/s).
constexpr int CE_NT = 512;

template <int NC>
__global__ __launch_bounds__(CE_NT) void ce_kernel(CEArgs p) {
  __shared__ float red_m[CE_NT / 64], red_s[CE_NT / 64], red_v[CE_NT / 64], tv;
  __shared__ int red_i[CE_NT / 64];
  const long long row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* x = static_cast<const bf16_t*>(p.logits) + row * p.ld;
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  const long long tgt = p.targets[row];
  const bool valid = tgt != p.ignore_index && tgt >= 0 && tgt < p.V;
  const int nch = (p.V + 7) >> 3;
  uint4 raw[NC];
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    raw[u] = c < nch ? xv[c] : make_uint4(0u, 0u, 0u, 0u);
  }
  float m = -INFINITY, s = 0.f, bv = -INFINITY, tval = 0.f;
  int bi = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    if (c < nch) ce_chunk_stats(raw[u], c, p.V, tgt, m, s, bv, bi, &tval);
  }
  if (valid && tgt / 8 % CE_NT == tid) tv = tval;
  ce_block_reduce<CE_NT / 64>(m, s, bv, bi, red_m, red_s, red_v, red_i);  // (its barrier publishes tv)
  const float lse = m + __logf(s);
  if (tid == 0) {
    p.row_loss[row] = valid ? lse - tv : 0.f;
    if (p.row_correct) p.row_correct[row] = (valid && bi == tgt) ? 1.f : 0.f;
  }
  if (!p.write_grad) return;
  const float scale = valid ? *p.inv_count : 0.f;
  uint4* g = reinterpret_cast<uint4*>(static_cast<bf16_t*>(p.dlogits) + row * p.ld);
  const int nchl = (int)(p.ld >> 3);
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    if (c < nchl) g[c] = ce_chunk_grad(raw[u], c, p.V, tgt, lse, scale);
  }
}

// Register-resident row with the per-logit vector-ALU work cut to what the math needs (round 5;
// ce_kernel above measured ~24 VALU per logit -- per-element end-of-row, target and argmax
// compares -- and ran VALU-bound at 4.4 TB/s): per 16-B chunk one v_max3 tree, then
// 2^(x log2e - max log2e) by one FMA + v_exp_f32 per logit; the tail chunk (V % 8) masked in a
// branch only its thread takes; the target logit read by one lane from memory (before any
// gradient store: dlogits may alias logits); the argmax tracked per chunk (chunk max) and resolved
// inside the winning chunk by its owner after the block reduction; the gradient pass one FMA,
// v_exp_f32 and multiply per logit, the target's -1 applied by the chunk's owner only.
template <int NC>
__global__ __launch_bounds__(CE_NT) void ce_kernel2(CEArgs p) {
  __shared__ float red_m[CE_NT / 64], red_s[CE_NT / 64], red_v[CE_NT / 64], tv;
  __shared__ int red_i[CE_NT / 64];
  constexpr float L2E = 1.4426950408889634f;
  const long long row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* x = static_cast<const bf16_t*>(p.logits) + row * p.ld;
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  const long long tgt = p.targets[row];
  const bool valid = tgt != p.ignore_index && tgt >= 0 && tgt < p.V;
  const int nch = (p.V + 7) >> 3;
  const int tail = p.V & 7;  // valid logits of the last chunk (0: the chunk is full)
  uint4 raw[NC];
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    raw[u] = c < nch ? xv[c] : make_uint4(0u, 0u, 0u, 0u);
  }
  if (tid == 0) tv = valid ? bf2f(x[tgt]) : 0.f;  // (published by the reduction's barrier)
  float m = -INFINITY, s = 0.f, bv = -INFINITY;
  int bc = 0x7fffffff;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    if (c < nch) {
      float f[8];
      unpack8(raw[u], f);
      if (tail && c == nch - 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = j < tail ? f[j] : -INFINITY;
      }
      const float cm = fmaxf(fmaxf(fmaxf(f[0], f[1]), fmaxf(f[2], f[3])), fmaxf(fmaxf(f[4], f[5]), fmaxf(f[6], f[7])));
      // (a chunk of eight -inf logits: cm = -inf would make every exponent -inf + inf = NaN; with
      // 0 they are exp2(-inf) = 0 and the chunk adds nothing -- ms_combine skips an all -inf max)
      const float cml = cm == -INFINITY ? 0.f : cm * L2E;
      float cs = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) cs += __builtin_amdgcn_exp2f(fmaf(f[j], L2E, -cml));
      ms_combine(m, s, cm, cs);
      if (cm > bv) {  // (chunks visited in increasing order: the first maximal chunk)
        bv = cm;
        bc = c;
      }
    }
  }
  ce_block_reduce<CE_NT / 64>(m, s, bv, bc, red_m, red_s, red_v, red_i);
  const float lse = m + __logf(s);
  if (tid == 0) p.row_loss[row] = valid ? lse - tv : 0.f;
  if (p.row_correct && tid == (bc & (CE_NT - 1)) && bc < nch) {
    // the owner of the first maximal chunk finds the first maximal logit in it, re-reading the
    // chunk (only its owner writes it, later: safe under dlogits == logits; a select over raw[]
    // by a run-time index moved the whole row array to scratch)
    float f[8];
    unpack8(xv[bc], f);
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 7; j >= 0; --j) bi = f[j] == bv ? bc * 8 + j : bi;
    p.row_correct[row] = (valid && bi == tgt) ? 1.f : 0.f;
  }
  if (!p.write_grad) return;
  const float scale = valid ? *p.inv_count : 0.f;
  const float lsel = lse * L2E;
  uint4* g = reinterpret_cast<uint4*>(static_cast<bf16_t*>(p.dlogits) + row * p.ld);
  const int nchl = (int)(p.ld >> 3);
  const int tc = valid ? (int)(tgt >> 3) : -1;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const int c = tid + u * CE_NT;
    if (c < nchl) {
      float f[8];
      unpack8(raw[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = __builtin_amdgcn_exp2f(fmaf(f[j], L2E, -lsel)) * scale;
      if (c >= nch - 1 && (c >= nch || tail)) {  // past the vocabulary: zeros
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (c * 8 + j < p.V) ? f[j] : 0.f;
      }
      if (c == tc) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] -= (j == (int)(tgt & 7)) ? scale : 0.f;
      }
      g[c] = pack8(f);
    }
  }
}

// Streaming fallback for rows longer than CE_NT * 16 chunks (V > 65536): CE_UNROLL chunks in
// flight per thread per trip, the gradient pass re-reads the row.
template <int CE_UNROLL>
__global__ __launch_bounds__(256) void ce_stream_kernel(CEArgs p) {
  __shared__ float red_m[4], red_s[4], red_v[4], tv;
  __shared__ int red_i[4];
  const long long row = blockIdx.x;
  const int tid = threadIdx.x;
  const bf16_t* x = static_cast<const bf16_t*>(p.logits) + row * p.ld;
  const uint4* xv = reinterpret_cast<const uint4*>(x);
  const long long tgt = p.targets[row];
  const bool valid = tgt != p.ignore_index && tgt >= 0 && tgt < p.V;
  const int nch = (p.V + 7) >> 3;
  float m = -INFINITY, s = 0.f, bv = -INFINITY, tval = 0.f;
  int bi = 0x7fffffff;
  for (int c0 = tid; c0 < nch; c0 += 256 * CE_UNROLL) {
    uint4 raw[CE_UNROLL];
#pragma unroll
    for (int u = 0; u < CE_UNROLL; ++u) {
      const int c = c0 + u * 256;
      raw[u] = c < nch ? xv[c] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < CE_UNROLL; ++u) {
      const int c = c0 + u * 256;
      if (c < nch) ce_chunk_stats(raw[u], c, p.V, tgt, m, s, bv, bi, &tval);
    }
  }
  if (valid && tgt / 8 % 256 == tid) tv = tval;
  ce_block_reduce<4>(m, s, bv, bi, red_m, red_s, red_v, red_i);
  const float lse = m + __logf(s);
  if (tid == 0) {
    p.row_loss[row] = valid ? lse - tv : 0.f;
    if (p.row_correct) p.row_correct[row] = (valid && bi == tgt) ? 1.f : 0.f;
  }
  if (!p.write_grad) return;
  const float scale = valid ? *p.inv_count : 0.f;
  uint4* g = reinterpret_cast<uint4*>(static_cast<bf16_t*>(p.dlogits) + row * p.ld);
  const int nchl = (int)(p.ld >> 3);
  for (int c0 = tid; c0 < nchl; c0 += 256 * CE_UNROLL) {
    uint4 raw[CE_UNROLL];
#pragma unroll
    for (int u = 0; u < CE_UNROLL; ++u) {
      const int c = c0 + u * 256;
      raw[u] = c < nch ? xv[c] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < CE_UNROLL; ++u) {
      const int c = c0 + u * 256;
      if (c < nchl) g[c] = ce_chunk_grad(raw[u], c, p.V, tgt, lse, scale);
    }
  }
}

// ------------------------------------------------------------------ AdamW (flat)
struct AdamArgs {
  float* param;            // [n] f32 master
  const float* grad;       // [n] f32
  float* exp_avg;          // [n]
  float* exp_avg_sq;       // [n]
  void* shadow;            // [n] bf16 compute copy (optional)
  const float* grad_scale_ptr;  // optional device scalar multiplier on the gradient
  long long n;
  float lr, beta1, beta2, eps, weight_decay;
  float bias_correction1, bias_correction2_sqrt;
  float grad_scale;
  const float* step_ptr;  // optional device step counter (HIP-graph replay): bias corrections
                          // are then computed on the device from it
  const float* skip_ptr;  // optional device flag: != 0 -> leave everything untouched (the loss
                          // scaler found a non-finite gradient this step)
};

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  if (a.skip_ptr && *a.skip_ptr != 0.f) return;
  const long long n4 = a.n >> 2;
  float gs = a.grad_scale;
  if (a.grad_scale_ptr) gs *= *a.grad_scale_ptr;
  const float b1 = a.beta1, b2 = a.beta2;
  float bc1 = a.bias_correction1, bc2s = a.bias_correction2_sqrt;
  if (a.step_ptr) {
    const float t = *a.step_ptr;
    bc1 = 1.f - powf(b1, t);
    bc2s = sqrtf(1.f - powf(b2, t));
  }
  a.bias_correction2_sqrt = bc2s;
  const float step = a.lr / bc1;
  const float decay = 1.f - a.lr * a.weight_decay;
  const float inv_bc2s = 1.f / bc2s;
  // two float4 groups per thread per trip, all eight loads issued before any math (16 B per lane
  // per array in flight was 3.4 TB/s on the GPT-2 small step: 1.1 ms for 124M parameters), and
  // non-temporal accesses: the 1.9 GB of optimizer state streams once per step
  const long long stride = (long long)gridDim.x * 256;
  floatx4* P = reinterpret_cast<floatx4*>(a.param);
  const floatx4* G = reinterpret_cast<const floatx4*>(a.grad);
  floatx4* M = reinterpret_cast<floatx4*>(a.exp_avg);
  floatx4* V = reinterpret_cast<floatx4*>(a.exp_avg_sq);
  for (long long i0 = (long long)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += 2 * stride) {
    const long long idx[2] = {i0, i0 + stride};
    const bool has1 = idx[1] < n4;
    floatx4 p[2], g[2], m[2], v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !has1) break;
      p[u] = __builtin_nontemporal_load(P + idx[u]);
      g[u] = __builtin_nontemporal_load(G + idx[u]);
      m[u] = __builtin_nontemporal_load(M + idx[u]);
      v[u] = __builtin_nontemporal_load(V + idx[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !has1) break;
      floatx4 pp = p[u], mm = m[u], vv = v[u];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gj = g[u][j] * gs;
        mm[j] = b1 * mm[j] + (1.f - b1) * gj;
        vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
        const float denom = sqrtf(vv[j]) * inv_bc2s + a.eps;
        pp[j] = pp[j] * decay - step * mm[j] / denom;
      }
      __builtin_nontemporal_store(pp, P + idx[u]);
      __builtin_nontemporal_store(mm, M + idx[u]);
      __builtin_nontemporal_store(vv, V + idx[u]);
      if (a.shadow) {
        uint2 w;
        w.x = pack2bf(pp[0], pp[1]);
        w.y = pack2bf(pp[2], pp[3]);
        reinterpret_cast<uint2*>(a.shadow)[idx[u]] = w;
      }
    }
  }
}

// f32 -> bf16 copy of a flat buffer (shadow refresh after load / broadcast)
struct CastArgs {
  const float* src;
  void* dst;
  long long n;
};

__global__ __launch_bounds__(256) void cast_kernel(CastArgs a) {
  const long long n4 = a.n >> 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(a.src)[i];
    uint2 w;
    w.x = pack2bf(v.x, v.y);
    w.y = pack2bf(v.z, v.w);
    reinterpret_cast<uint2*>(a.dst)[i] = w;
  }
}

// ------------------------------------------------------------------ dynamic loss scaling
// Reference: torch.cuda.amp.GradScaler (main-single.py:78,99-101): _amp_foreach_non_finite_
// check_and_unscale_ + _amp_update_scale_.  Here the unscale is folded into AdamW (its
// grad_scale_ptr reads 1/scale), so the check only reads the flat gradient buffer once and
// raises a device flag that AdamW (skip_ptr) and the scale update consume -- no host sync,
// HIP-graph replayable.  Non-finite = exponent bits all ones (independent of fast-math flags).
struct AmpCheckArgs {
  const float* g;
  long long n;
  float* found_inf;
};

__device__ __forceinline__ bool nonfinite(float x) { return (__float_as_uint(x) & 0x7f800000u) == 0x7f800000u; }

__global__ __launch_bounds__(256) void amp_check_kernel(AmpCheckArgs a) {
  const long long n4 = a.n >> 2;
  bool bad = false;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(a.g)[i];
    bad |= nonfinite(v.x) | nonfinite(v.y) | nonfinite(v.z) | nonfinite(v.w);
  }
  if (blockIdx.x == 0 && threadIdx.x < (a.n & 3)) bad |= nonfinite(a.g[(n4 << 2) + threadIdx.x]);
  if (__any(bad) && (threadIdx.x & 63) == 0) *a.found_inf = 1.f;  // every writer stores 1
}

struct AmpUpdateArgs {
  float* scale;
  float* inv_scale;
  float* found_inf;  // consumed and cleared
  float* tracker;    // consecutive finite steps
  float growth, backoff;
  int interval;
};

__global__ void amp_update_kernel(AmpUpdateArgs a) {
  if (threadIdx.x != 0) return;
  float s = *a.scale;
  if (*a.found_inf != 0.f) {
    s *= a.backoff;
    *a.tracker = 0.f;
  } else {
    const float t = *a.tracker + 1.f;
    if (t >= (float)a.interval) {
      s *= a.growth;
      *a.tracker = 0.f;
    } else {
      *a.tracker = t;
    }
  }
  *a.scale = s;
  *a.inv_scale = 1.f / s;
  *a.found_inf = 0.f;
}

// ------------------------------------------------------------------ dropout
// Counter-based keep mask (common.h:drop_factor): element (t, c) of a [T, N] site has index
// t*N + c.  The map idx -> hash is a bijection for a fixed key, so nothing is stored between
// forward and backward: both regenerate it.  The torch twin is ops/dropout.py:keep_mask.

// out[t, c] = res[t, c] + y[t, c] * keep(t, c) / (1 - p)   (f32; out may alias y or res)
struct DropResArgs {
  const float* y;
  const float* res;
  float* out;
  long long ldy, ldr, ldo;
  int T, N;
  unsigned key, thresh;
  float scale;
  const unsigned* seed;  // device seed of the forward (common.h:drop_key_of); null: key
  unsigned site;
};

__global__ __launch_bounds__(256) void dropout_residual_kernel(DropResArgs p) {
  const uint32_t key = drop_key_of(p.seed, p.site, p.key);
  const int nq = p.N >> 2;
  const long long total = (long long)p.T * nq;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long t = i / nq;
    const int c = (int)(i - t * nq) * 4;
    const float4 y = *reinterpret_cast<const float4*>(p.y + t * p.ldy + c);
    const float4 r = *reinterpret_cast<const float4*>(p.res + t * p.ldr + c);
    const uint32_t idx = (uint32_t)(t * p.N + c);
    float4 o;
    o.x = r.x + y.x * drop_factor(idx + 0, key, p.thresh, p.scale);
    o.y = r.y + y.y * drop_factor(idx + 1, key, p.thresh, p.scale);
    o.z = r.z + y.z * drop_factor(idx + 2, key, p.thresh, p.scale);
    o.w = r.w + y.w * drop_factor(idx + 3, key, p.thresh, p.scale);
    *reinterpret_cast<float4*>(p.out + t * p.ldo + c) = o;
  }
}

// ------------------------------------------------------------------ bias / activation backward
// dz[t, c] = dy[t, c] * keep(t, c) * act'(z[t, c])  (bf16 out), db[c] += sum_t dz[t, c]
// (keep = 1 when drop_scale == 0).
// grid: (ceil(N / 256), ceil(T / BA_ROWS)); each lane owns 4 columns (one float4 of a row), the
// 4 waves of a block interleave its BA_ROWS rows, 4 rows in flight per wave.
struct BiasActArgs {
  const float* dy;     // [T][lddy] f32
  const void* z;       // [T][ldz] bf16 pre-activation (optional, needed when act != 0)
  void* dz;            // [T][lddz] bf16
  float* db;           // [N] f32 accumulate (optional)
  long long lddy, ldz, lddz;
  int T, N;
  int act;
  unsigned drop_key, drop_thresh;
  float drop_scale;    // 0: no dropout
  const unsigned* drop_seed;  // device seed of the forward (common.h:drop_key_of); null: drop_key
  unsigned drop_site;
};

constexpr int BA_ROWS = 128;

__global__ __launch_bounds__(256) void bias_act_bwd_kernel(BiasActArgs p) {
  const uint32_t dkey = p.drop_scale != 0.f ? drop_key_of(p.drop_seed, p.drop_site, p.drop_key) : 0u;
  __shared__ float red[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const bool colok = c < p.N;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const long long r0 = (long long)blockIdx.y * BA_ROWS;
  const int nrows = (int)min((long long)BA_ROWS, (long long)p.T - r0);
  const bf16_t* z = static_cast<const bf16_t*>(p.z);
  bf16_t* dz = static_cast<bf16_t*>(p.dz);
  if (colok) {
    // rows w, w + 4, ...; four of them loaded before any is used (memory-level parallelism)
    for (int i0 = w; i0 < nrows; i0 += 16) {
      float4 y[4];
      uint2 zz[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 4 * u;
        if (i < nrows) {
          const long long t = r0 + i;
          y[u] = *reinterpret_cast<const float4*>(p.dy + t * p.lddy + c);
          if (p.act) zz[u] = *reinterpret_cast<const uint2*>(z + t * p.ldz + c);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + 4 * u;
        if (i >= nrows) break;
        const long long t = r0 + i;
        float f[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
        if (p.act) {
          f[0] *= act_grad(__uint_as_float(zz[u].x << 16), p.act);
          f[1] *= act_grad(__uint_as_float(zz[u].x & 0xffff0000u), p.act);
          f[2] *= act_grad(__uint_as_float(zz[u].y << 16), p.act);
          f[3] *= act_grad(__uint_as_float(zz[u].y & 0xffff0000u), p.act);
        }
        if (p.drop_scale != 0.f) {
          const uint32_t idx = (uint32_t)(t * p.N + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) f[j] *= drop_factor(idx + j, dkey, p.drop_thresh, p.drop_scale);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += f[j];
        uint2 o;
        o.x = pack2bf(f[0], f[1]);
        o.y = pack2bf(f[2], f[3]);
        *reinterpret_cast<uint2*>(dz + t * p.lddz + c) = o;
      }
    }
  }
  if (!p.db) return;
#pragma unroll
  for (int j = 0; j < 4; ++j) red[w][lane * 4 + j] = acc[j];
  __syncthreads();
  // column sums of the block: lane-contiguous atomics (256 B per wave-instruction)
  const int col = threadIdx.x, n = blockIdx.x * 256 + col;
  if (n < p.N) atomicAdd(p.db + n, red[0][col] + red[1][col] + red[2][col] + red[3][col]);
}

}  // namespace dpc

using namespace dpc;

static inline unsigned grid_for(long long n4) {
  long long b = (n4 + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

DPC_API int dpc_embedding_fwd(const EmbArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->D % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)((a->T + 3) / 4)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_embedding_bwd(const EmbArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  hipLaunchKernelGGL(emb_bwd_kernel, dim3((unsigned)((a->T + 3) / 4)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

// 0: register-resident rows when they fit (default, ce_kernel2); 1 / 2: streaming with 1 / 4
// chunks in flight per thread; 3: the round-4 register-resident kernel (A/B sweeps:
// bench/ce_one.py).  GPT-2 small B = 64 (65472 x 50257 bf16 logits, in place), one MI355X:
// mode 0 2.52-2.54 ms (5.2 TB/s, the float4 copy roofline of profiles/r4_copylab/), mode 3
// 2.77 ms, torch's device copy of the same bytes 2.85 ms (profiles/r5_ce/); a round-4 variant with
// one exponential per logit (exp kept as f16 between the passes) measured 3.17 ms and was removed
// (profiles/r4_ce/).
static int g_ce_mode = -1;  // -1: DPC_CE_MODE (default 0)
DPC_API void dpc_ce_set_mode(int m) { g_ce_mode = m; }

DPC_API int dpc_cross_entropy(const CEArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->ld % 8) return (int)hipErrorInvalidValue;
  const long long nc = ((a->ld >> 3) + CE_NT - 1) / CE_NT;  // chunks per thread (ld >= V)
  const dim3 grid((unsigned)a->T);
  if (g_ce_mode < 0) g_ce_mode = getenv("DPC_CE_MODE") ? atoi(getenv("DPC_CE_MODE")) : 0;
  if (g_ce_mode == 1) hipLaunchKernelGGL(ce_stream_kernel<1>, grid, dim3(256), 0, stream, *a);
  else if (g_ce_mode == 2) hipLaunchKernelGGL(ce_stream_kernel<4>, grid, dim3(256), 0, stream, *a);
  else if (g_ce_mode == 3 && nc <= 13) hipLaunchKernelGGL(ce_kernel<13>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 1) hipLaunchKernelGGL(ce_kernel2<1>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 2) hipLaunchKernelGGL(ce_kernel2<2>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 4) hipLaunchKernelGGL(ce_kernel2<4>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 8) hipLaunchKernelGGL(ce_kernel2<8>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 13) hipLaunchKernelGGL(ce_kernel2<13>, grid, dim3(CE_NT), 0, stream, *a);
  else if (nc <= 16) hipLaunchKernelGGL(ce_kernel2<16>, grid, dim3(CE_NT), 0, stream, *a);
  else hipLaunchKernelGGL(ce_stream_kernel<4>, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_adamw(const AdamArgs* a, hipStream_t stream) {
  if (a->n <= 0) return 0;
  if (a->n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(a->n >> 2)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_amp_check(const AmpCheckArgs* a, hipStream_t stream) {
  if (a->n <= 0) return 0;
  hipLaunchKernelGGL(amp_check_kernel, dim3(grid_for((a->n + 3) >> 2)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_amp_update(const AmpUpdateArgs* a, hipStream_t stream) {
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_cast_f32_bf16(const CastArgs* a, hipStream_t stream) {
  if (a->n <= 0) return 0;
  if (a->n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(a->n >> 2)), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_bias_act_bwd(const BiasActArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->N % 4 || a->lddy % 4 || a->ldz % 4 || a->lddz % 4) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((a->N + 255) / 256), (unsigned)((a->T + BA_ROWS - 1) / BA_ROWS));
  hipLaunchKernelGGL(bias_act_bwd_kernel, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

DPC_API int dpc_dropout_residual(const DropResArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->N % 4 || a->ldy % 4 || a->ldr % 4 || a->ldo % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(dropout_residual_kernel, dim3(grid_for((long long)a->T * (a->N / 4))), dim3(256), 0,
                     stream, *a);
  return (int)hipGetLastError();
}

// ---- CU occupier (measurements of the GEMM resident-CU reserve, bench/cu_reserve.py): nwg
// small workgroups that spin for `ns` nanoseconds -- the footprint of an RCCL collective's
// channel workgroups resident beside the compute stream.  Every wave reaches the exit.
// 32 KiB of LDS per workgroup, like a collective kernel's shared staging: a CU hosting one
// cannot also host a 160 KiB GEMM workgroup
__global__ __launch_bounds__(256) void occupy_kernel(long long ticks, unsigned* sink) {
  __shared__ unsigned scratch[8192];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  unsigned spins = 0;
  scratch[threadIdx.x * 32] = threadIdx.x;
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) {
    __builtin_amdgcn_s_sleep(4);
    ++spins;
  }
  __syncthreads();
  if (threadIdx.x == 0 && spins == 0xffffffffu) sink[blockIdx.x] = scratch[(spins & 255) * 32];  // (never)
}

DPC_API int dpc_occupy(int nwg, long long ns, void* sink, hipStream_t stream) {
  if (nwg <= 0) return 0;
  hipLaunchKernelGGL(occupy_kernel, dim3((unsigned)nwg), dim3(256), 0, stream, ns / 10, static_cast<unsigned*>(sink));
  return (int)hipGetLastError();
}
