// f32 flash attention (forward + backward) on the f32 matrix cores (v_mfma_f32_32x32x2_f32):
// the --disable_amp path (/root/reference/main-single.py:88-90 runs the model in f32 with AMP
// off; /root/reference/models/gpt.py:75-100 is the attention), O(S) memory instead of the
// materialised [N, H, S, S] scores.  Same semantics and argument struct as attention.hip
// (causal + optional key padding, fused [T, 3*H*hd] QKV input, merged-head output, natural
// log-sum-exp saved for the backward); every operand f32, head_dim 32 or 64.
//
// MFMA 32x32x2 f32: A lane l = row (l & 31), k = l >> 5; B lane l = column (l & 31), k = l >> 5;
// C register r of lane l = (row (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31).  An
// accumulator feeds the next product as its B operand with the k order permuted: k-step s
// pairs the rows kappa(s, h) = (s & 3) + 8 (s >> 2) + 4 h held in register s of the two lane
// halves h, and the A operand is read from LDS at those same rows.
//   forward   S^T = K Q^T (query on the lane: row statistics lane-local), O^T += V^T P^T
//   dK / dV   S = Q K^T, dP = dO V^T (key on the lane), dV^T += dO^T P, dK^T += Q^T dS
//   dQ        S^T, dP^T (query on the lane), dQ^T += K^T dS^T
// Tiles of 64 rows are staged through LDS by registers (double buffered).  Row pads: images read
// by rows (32 rows x columns 2s, 2s+1 per instruction) use HD + 2 floats (64 distinct banks);
// the forward's V, read by columns at rows kappa and kappa + 4, uses HD + 8 (the halves 32
// banks apart).
#include "common.h"

namespace dpc {

struct AttnArgs {  // identical layout to attention.hip (f32 element pointers here)
  const void* q; const void* k; const void* v;
  void* o;
  float* lse;
  const unsigned char* pad;
  const void* dout;
  void* dq; void* dk; void* dv;
  float* delta;
  long long ld_qkv, ld_o, ld_dqkv;
  int N, S, H;
  float scale;
  int causal;
  int hd;
};

namespace f32a {

constexpr int T = 64;  // rows per staged tile
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ int crow(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
__device__ __forceinline__ floatx16 mma(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void zero(floatx16& x) {
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0.f;
}

// stage rows r0 .. r0+63 (zeros at or beyond S) of an [S][ld] f32 matrix, columns 0 .. HD-1,
// into registers (HD / 16 float4 per thread), then into LDS [64][LD]
template <int HD>
__device__ __forceinline__ void ld_tile(float4 (&v)[HD / 16], const float* X, long long ld, int r0, int S) {
#pragma unroll
  for (int i = 0; i < HD / 16; ++i) {
    const int e = (threadIdx.x + 256 * i) * 4;  // element of the 64 x HD tile
    const int r = e / HD, c = e % HD;
    v[i] = (r0 + r < S) ? *reinterpret_cast<const float4*>(X + (long long)(r0 + r) * ld + c)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int HD, int LD>
__device__ __forceinline__ void st_tile(const float4 (&v)[HD / 16], float* s) {
#pragma unroll
  for (int i = 0; i < HD / 16; ++i) {
    const int e = (threadIdx.x + 256 * i) * 4;
    const int r = e / HD, c = e % HD;
    float* d = s + r * LD + c;
    d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
  }
}

__device__ __forceinline__ unsigned long long pad_bits(const unsigned char* pad, int k0, int S, int lane) {
  if (!pad) return 0ull;
  const int k = k0 + lane;
  return __ballot(k < S && pad[k] != 0);
}

__device__ __forceinline__ void xcd_work(int nblk, int& bh, int& i) {
  const int b = blockIdx.x, nwg = gridDim.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  bh = t / nblk;
  i = t - bh * nblk;
}

// ------------------------------------------------------------------ forward
template <int HD>
__global__ __launch_bounds__(256, HD >= 128 ? 1 : 2) void fwd_kernel(AttnArgs p) {
  constexpr int LK = HD + 2, LV = HD + 8, NDT = HD / 32;
  __shared__ float sk[2][T * LK];
  __shared__ float sv[2][T * LV];
  const int S = p.S, H = p.H;
  const int nqb = (S + 127) / 128;
  int bh, bi;
  xcd_work(nqb, bh, bi);
  const int qb = nqb - 1 - bi;
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, hh = lane >> 5;
  const int q0 = qb * 128 + wid * 32, q = q0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const float* Q = static_cast<const float*>(p.q) + h * HD;
  const float* K = static_cast<const float*>(p.k) + tok0 * p.ld_qkv + h * HD;
  const float* V = static_cast<const float*>(p.v) + tok0 * p.ld_qkv + h * HD;
  const unsigned char* pad = p.pad ? p.pad + (long long)n * S : nullptr;

  float qf[HD / 2];  // Q[q][2 s + h]
#pragma unroll
  for (int s = 0; s < HD / 2; ++s) qf[s] = q < S ? Q[(tok0 + q) * p.ld_qkv + 2 * s + hh] : 0.f;
  const float c = p.scale * LOG2E;
  const int kend = p.causal ? min(S, qb * 128 + 128) : S;
  const int ntiles = (kend + T - 1) / T;
  float m = -INFINITY, l = 0.f;
  floatx16 o[NDT];
#pragma unroll
  for (int d = 0; d < NDT; ++d) zero(o[d]);

  float4 rk[HD / 16], rv[HD / 16];
  ld_tile<HD>(rk, K, p.ld_qkv, 0, S);
  ld_tile<HD>(rv, V, p.ld_qkv, 0, S);
  st_tile<HD, LK>(rk, sk[0]);
  st_tile<HD, LV>(rv, sv[0]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) {
      ld_tile<HD>(rk, K, p.ld_qkv, (t + 1) * T, S);
      ld_tile<HD>(rv, V, p.ld_qkv, (t + 1) * T, S);
    }
    const int kt0 = t * T;
    if (!(p.causal && kt0 > q0 + 31)) {
      const float* ks = sk[cur];
      const float* vs = sv[cur];
      floatx16 sc[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        zero(sc[kb]);
#pragma unroll
        for (int s = 0; s < HD / 2; ++s) sc[kb] = mma(ks[(kb * 32 + (lane & 31)) * LK + 2 * s + hh], qf[s], sc[kb]);
      }
      const bool need_mask = (p.causal && kt0 + T - 1 > q0) || (kt0 + T > S) || pad;
      if (need_mask) {
        const unsigned long long pm = pad_bits(pad, kt0, S, lane);
        const int lim = (p.causal ? min(q, S - 1) : S - 1) - kt0;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kl = kb * 32 + crow(r, lane);
            if (kl > lim || ((pm >> kl) & 1ull)) sc[kb][r] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sc[kb][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * c;
      const float mn = fmaxf(m, mx);
      if (mn > m) {  // exact online softmax (no lazy threshold on the f32 path)
        const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int d = 0; d < NDT; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
        m = mn;
      }
      const float nmu = (m == -INFINITY) ? 0.f : -m;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = exp2f(fmaf(sc[kb][r], c, nmu));
          sc[kb][r] = e;
          l += e;
        }
      // O^T[d][q] += sum_key V[key][d] P[key][q]; k-step (kb, s): keys kb*32 + kappa(s, h)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int key = kb * 32 + crow(s, lane);
#pragma unroll
          for (int d = 0; d < NDT; ++d) o[d] = mma(vs[key * LV + d * 32 + (lane & 31)], sc[kb][s], o[d]);
        }
    }
    if (t + 1 < ntiles) {
      __syncthreads();  // every wave is done with the other stage (tile t-1)
      st_tile<HD, LK>(rk, sk[cur ^ 1]);
      st_tile<HD, LV>(rv, sv[cur ^ 1]);
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  // O^T register r of lane l: d = dbase + crow(r, l), query l & 31
  if (q < S) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    float* O = static_cast<float*>(p.o) + (tok0 + q) * p.ld_o + h * HD;
#pragma unroll
    for (int d = 0; d < NDT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) O[d * 32 + crow(r, lane)] = o[d][r] * inv;
    if (hh == 0) p.lse[(long long)bh * S + q] = (l > 0.f) ? (m + log2f(l)) / LOG2E : INFINITY;
  }
}

// ------------------------------------------------------------------ backward
template <int HD>
__global__ __launch_bounds__(256) void pre_kernel(AttnArgs p) {
  // delta[n,h,s] = sum_d dO * O, one wave per (token, head) group of 64 / HD lanes each
  const long long rows = (long long)p.N * p.S * p.H;
  constexpr int LPR = HD / 4;  // lanes per row (float4 each)
  const long long row = ((long long)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  float acc = 0.f;
  long long t = 0;
  int h = 0;
  if (row < rows) {
    t = row / p.H;
    h = (int)(row % p.H);
    const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(p.o) + t * p.ld_o + h * HD + 4 * sub);
    const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(p.dout) + t * p.ld_o + h * HD + 4 * sub);
    acc = a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (row < rows && sub == 0) {
    const long long nn = t / p.S, s = t % p.S;
    p.delta[(nn * p.H + h) * p.S + s] = acc;
  }
}

template <int HD>
__global__ __launch_bounds__(256, HD >= 64 ? 1 : 2) void dkdv_kernel(AttnArgs p) {
  constexpr int LQ = HD + 2, NDT = HD / 32;
  __shared__ float sq[2][T * LQ];
  __shared__ float sd[2][T * LQ];
  __shared__ float srow[2][2][T];
  const int S = p.S, H = p.H;
  const int nkb = (S + 127) / 128;
  int bh, kb;
  xcd_work(nkb, bh, kb);
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, hh = lane >> 5;
  const int k0 = kb * 128 + wid * 32, key = k0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const float* Q = static_cast<const float*>(p.q) + tok0 * p.ld_qkv + h * HD;
  const float* Kp = static_cast<const float*>(p.k) + h * HD;
  const float* Vp = static_cast<const float*>(p.v) + h * HD;
  const float* dO = static_cast<const float*>(p.dout) + tok0 * p.ld_o + h * HD;
  const float* lse = p.lse + (long long)bh * S;
  const float* delta = p.delta + (long long)bh * S;
  const bool key_ok = key < S && !(p.pad && p.pad[(long long)n * S + min(key, S - 1)]);

  float kf[HD / 2], vf[HD / 2];  // K[key][2 s + h], V[key][2 s + h]
#pragma unroll
  for (int s = 0; s < HD / 2; ++s) {
    kf[s] = key < S ? Kp[(tok0 + key) * p.ld_qkv + 2 * s + hh] : 0.f;
    vf[s] = key < S ? Vp[(tok0 + key) * p.ld_qkv + 2 * s + hh] : 0.f;
  }
  const float c = p.scale * LOG2E;
  floatx16 dvt[NDT], dkt[NDT];
#pragma unroll
  for (int d = 0; d < NDT; ++d) {
    zero(dvt[d]);
    zero(dkt[d]);
  }
  const int qt_begin = p.causal ? (kb * 128) / T : 0;
  const int nqt = (S + T - 1) / T;
  float4 rq[HD / 16], rd[HD / 16];
  float rl = 0.f, rdl = 0.f;
  auto load = [&](int qt) {
    ld_tile<HD>(rq, Q, p.ld_qkv, qt * T, S);
    ld_tile<HD>(rd, dO, p.ld_o, qt * T, S);
    if (threadIdx.x < T) {
      const int qq = qt * T + threadIdx.x;
      rl = qq < S ? lse[qq] * LOG2E : INFINITY;
      rdl = qq < S ? delta[qq] : 0.f;
    }
  };
  auto store = [&](int stg) {
    st_tile<HD, LQ>(rq, sq[stg]);
    st_tile<HD, LQ>(rd, sd[stg]);
    if (threadIdx.x < T) {
      srow[stg][0][threadIdx.x] = rl;
      srow[stg][1][threadIdx.x] = rdl;
    }
  };
  load(qt_begin);
  store(0);
  __syncthreads();
  for (int qt = qt_begin; qt < nqt; ++qt) {
    const int cur = (qt - qt_begin) & 1;
    if (qt + 1 < nqt) load(qt + 1);
    const float* qs_ = sq[cur];
    const float* ds_ = sd[cur];
    const int qt0 = qt * T;
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qb0 = qt0 + 32 * qs;
      if (p.causal && qb0 + 31 < k0) continue;  // every query before every key
      floatx16 sa, dp;
      zero(sa);
      zero(dp);
#pragma unroll
      for (int s = 0; s < HD / 2; ++s) {
        const int rr = (32 * qs + (lane & 31)) * LQ + 2 * s + hh;
        sa = mma(qs_[rr], kf[s], sa);
        dp = mma(ds_[rr], vf[s], dp);
      }
      // sa[r]: query qt0 + 32 qs + crow(r), key = the lane's key
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = 32 * qs + crow(r, lane);
        float pv = exp2f(fmaf(sa[r], c, -srow[cur][0][qi]));
        if (p.causal && key > qt0 + qi) pv = 0.f;
        sa[r] = pv;
        dp[r] = pv * (dp[r] - srow[cur][1][qi]);
      }
      // dV^T[d][key] += sum_q dO[q][d] P[q][key]; dK^T[d][key] += sum_q Q[q][d] dS[q][key]
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int qi = 32 * qs + crow(s, lane);
#pragma unroll
        for (int d = 0; d < NDT; ++d) {
          dvt[d] = mma(ds_[qi * LQ + d * 32 + (lane & 31)], sa[s], dvt[d]);
          dkt[d] = mma(qs_[qi * LQ + d * 32 + (lane & 31)], dp[s], dkt[d]);
        }
      }
    }
    if (qt + 1 < nqt) {
      __syncthreads();
      store(cur ^ 1);
    }
    __syncthreads();
  }
  // dK^T / dV^T register r of lane l: d = dbase + crow(r, l), key l & 31
  if (key < S) {
    float* dK = static_cast<float*>(p.dk) + (tok0 + key) * p.ld_dqkv + h * HD;
    float* dV = static_cast<float*>(p.dv) + (tok0 + key) * p.ld_dqkv + h * HD;
#pragma unroll
    for (int d = 0; d < NDT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dK[d * 32 + crow(r, lane)] = key_ok ? dkt[d][r] * p.scale : 0.f;
        dV[d * 32 + crow(r, lane)] = key_ok ? dvt[d][r] : 0.f;
      }
  }
}

template <int HD>
__global__ __launch_bounds__(256, HD >= 128 ? 1 : 2) void dq_kernel(AttnArgs p) {
  constexpr int LK = HD + 2, NDT = HD / 32;
  __shared__ float sk[2][T * LK];
  __shared__ float sv[2][T * LK];
  const int S = p.S, H = p.H;
  const int nqb = (S + 127) / 128;
  int bh, bi;
  xcd_work(nqb, bh, bi);
  const int qb = nqb - 1 - bi;
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, hh = lane >> 5;
  const int q0 = qb * 128 + wid * 32, q = q0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const float* Q = static_cast<const float*>(p.q) + h * HD;
  const float* K = static_cast<const float*>(p.k) + tok0 * p.ld_qkv + h * HD;
  const float* V = static_cast<const float*>(p.v) + tok0 * p.ld_qkv + h * HD;
  const float* dO = static_cast<const float*>(p.dout) + h * HD;
  const unsigned char* pad = p.pad ? p.pad + (long long)n * S : nullptr;
  float qf[HD / 2], df[HD / 2];
#pragma unroll
  for (int s = 0; s < HD / 2; ++s) {
    qf[s] = q < S ? Q[(tok0 + q) * p.ld_qkv + 2 * s + hh] : 0.f;
    df[s] = q < S ? dO[(tok0 + q) * p.ld_o + 2 * s + hh] : 0.f;
  }
  const float c = p.scale * LOG2E;
  const float lse2 = q < S ? p.lse[(long long)bh * S + q] * LOG2E : INFINITY;
  const float dl = q < S ? p.delta[(long long)bh * S + q] : 0.f;
  floatx16 dqt[NDT];
#pragma unroll
  for (int d = 0; d < NDT; ++d) zero(dqt[d]);
  const int kend = p.causal ? min(S, qb * 128 + 128) : S;
  const int ntiles = (kend + T - 1) / T;
  float4 rk[HD / 16], rv[HD / 16];
  ld_tile<HD>(rk, K, p.ld_qkv, 0, S);
  ld_tile<HD>(rv, V, p.ld_qkv, 0, S);
  st_tile<HD, LK>(rk, sk[0]);
  st_tile<HD, LK>(rv, sv[0]);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) {
      ld_tile<HD>(rk, K, p.ld_qkv, (t + 1) * T, S);
      ld_tile<HD>(rv, V, p.ld_qkv, (t + 1) * T, S);
    }
    const int kt0 = t * T;
    const float* ks = sk[cur];
    const float* vs = sv[cur];
    const unsigned long long pm = pad_bits(pad, kt0, S, lane);
    const int lim = (p.causal ? min(q, S - 1) : S - 1) - kt0;
#pragma unroll
    for (int kbk = 0; kbk < 2; ++kbk) {
      if (p.causal && kt0 + 32 * kbk > q0 + 31) continue;
      floatx16 sa, dp;
      zero(sa);
      zero(dp);
#pragma unroll
      for (int s = 0; s < HD / 2; ++s) {
        const int rr = (32 * kbk + (lane & 31)) * LK + 2 * s + hh;
        sa = mma(ks[rr], qf[s], sa);
        dp = mma(vs[rr], df[s], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kl = 32 * kbk + crow(r, lane);
        float pv = exp2f(fmaf(sa[r], c, -lse2));
        if (kl > lim || ((pm >> kl) & 1ull)) pv = 0.f;
        dp[r] = pv * (dp[r] - dl);
      }
      // dQ^T[d][q] += sum_key K[key][d] dS^T[key][q]
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int kl = 32 * kbk + crow(s, lane);
#pragma unroll
        for (int d = 0; d < NDT; ++d) dqt[d] = mma(ks[kl * LK + d * 32 + (lane & 31)], dp[s], dqt[d]);
      }
    }
    if (t + 1 < ntiles) {
      __syncthreads();
      st_tile<HD, LK>(rk, sk[cur ^ 1]);
      st_tile<HD, LK>(rv, sv[cur ^ 1]);
    }
    __syncthreads();
  }
  if (q < S) {
    float* dQ = static_cast<float*>(p.dq) + (tok0 + q) * p.ld_dqkv + h * HD;
#pragma unroll
    for (int d = 0; d < NDT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) dQ[d * 32 + crow(r, lane)] = dqt[d][r] * p.scale;
  }
}

template <int HD>
int fwd(const AttnArgs* a, hipStream_t stream) {
  dim3 grid((unsigned)(((a->S + 127) / 128) * a->N * a->H));
  hipLaunchKernelGGL(fwd_kernel<HD>, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

template <int HD>
int bwd(const AttnArgs* a, hipStream_t stream) {
  const long long rows = (long long)a->N * a->S * a->H;
  dim3 gpre((unsigned)((rows * (HD / 4) + 255) / 256));
  hipLaunchKernelGGL(pre_kernel<HD>, gpre, dim3(256), 0, stream, *a);
  dim3 grid((unsigned)(((a->S + 127) / 128) * a->N * a->H));
  hipLaunchKernelGGL(dkdv_kernel<HD>, grid, dim3(256), 0, stream, *a);
  hipLaunchKernelGGL(dq_kernel<HD>, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

}  // namespace f32a
}  // namespace dpc

using namespace dpc;

static bool f32_attn_ok(const AttnArgs* a, bool bwd) {
  if (a->hd != 32 && a->hd != 64 && a->hd != 128) return false;
  if (a->N <= 0 || a->S <= 0 || a->H <= 0) return false;
  return !(a->ld_qkv % 4 || a->ld_o % 4 || (bwd && a->ld_dqkv % 4));
}

DPC_API int dpc_attn_fwd_f32(const AttnArgs* a, hipStream_t stream) {
  if (!f32_attn_ok(a, false)) return (int)hipErrorInvalidValue;
  if (a->hd == 128) return f32a::fwd<128>(a, stream);
  return a->hd == 32 ? f32a::fwd<32>(a, stream) : f32a::fwd<64>(a, stream);
}

DPC_API int dpc_attn_bwd_f32(const AttnArgs* a, hipStream_t stream) {
  if (!f32_attn_ok(a, true)) return (int)hipErrorInvalidValue;
  if (a->hd == 128) return f32a::bwd<128>(a, stream);
  return a->hd == 32 ? f32a::bwd<32>(a, stream) : f32a::bwd<64>(a, stream);
}
