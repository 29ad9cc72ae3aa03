// Single-query attention for KV-cache decoding (one new token per sequence).
//
// One workgroup per (sequence, head), 256 threads: append the new key / value row to the
// cache at the device-side length, scores of the query against every cached key (LDS),
// softmax, then P.V with each thread owning 8 head dims of a strided subset of the keys and
// an LDS reduction over the subsets.  The length is read on the device, so the launch has
// no length-dependent shape and the decode step can be captured in a HIP graph.  Decode is
// a memory-bound read of the K/V cache; there is no tile for MFMA to fill at one query row.
#include "common.h"

namespace dpc {

struct DecodeAttnArgs {
  const void* qkv;           // [N][ldqkv] bf16: q | k | v blocks of H*hd each
  void* kc;                  // [N][Smax][E] bf16 key cache
  void* vc;                  // [N][Smax][E] bf16 value cache
  void* o;                   // [N][ldo] bf16
  const long long* len;      // device: number of cached tokens before this one
  long long ldqkv, ldo;
  int N, H, hd, Smax;
  float scale;
};

constexpr int DA_NT = 256;
constexpr int DA_MAX_S = 16384;  // LDS score buffer: 64 KB

__global__ __launch_bounds__(DA_NT) void decode_attn_kernel(DecodeAttnArgs p) {
  __shared__ float sc[DA_MAX_S];
  __shared__ float qs[256];
  __shared__ float red[DA_NT];
  __shared__ float acc[DA_NT * 8];
  const int tid = threadIdx.x;
  const int n = blockIdx.x / p.H, h = blockIdx.x % p.H;
  const int hd = p.hd, E = p.H * hd;
  const long long pos = *p.len;
  const int L = (int)pos + 1;
  const bf16_t* qrow = static_cast<const bf16_t*>(p.qkv) + n * p.ldqkv + h * hd;
  const bf16_t* knew = qrow + E;
  const bf16_t* vnew = qrow + 2 * E;
  bf16_t* kc = static_cast<bf16_t*>(p.kc) + (long long)n * p.Smax * E + h * hd;
  bf16_t* vc = static_cast<bf16_t*>(p.vc) + (long long)n * p.Smax * E + h * hd;
  // append the new row (the score / PV loops read it from qkv, not back from the cache)
  for (int i = tid; i < 2 * hd; i += DA_NT) {  // (strided: hd may reach DA_NT)
    if (i < hd) kc[pos * E + i] = knew[i];
    else vc[pos * E + i - hd] = vnew[i - hd];
  }
  if (tid < hd) qs[tid] = bf2f(qrow[tid]) * p.scale;
  __syncthreads();

  const int nc = hd >> 3;  // 16-byte chunks per row
  float m = -INFINITY;
  for (int j = tid; j < L; j += DA_NT) {
    const uint4* kr = reinterpret_cast<const uint4*>(j == pos ? knew : kc + (long long)j * E);
    float s = 0.f;
    for (int c = 0; c < nc; ++c) {
      float f[8];
      unpack8(kr[c], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += f[e] * qs[c * 8 + e];
    }
    sc[j] = s;
    m = fmaxf(m, s);
  }
  red[tid] = m;
  __syncthreads();
  for (int st = DA_NT / 2; st > 0; st >>= 1) {
    if (tid < st) red[tid] = fmaxf(red[tid], red[tid + st]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float l = 0.f;
  for (int j = tid; j < L; j += DA_NT) {
    const float e = __expf(sc[j] - m);
    sc[j] = e;
    l += e;
  }
  red[tid] = l;
  __syncthreads();
  for (int st = DA_NT / 2; st > 0; st >>= 1) {
    if (tid < st) red[tid] += red[tid + st];
    __syncthreads();
  }
  const float inv_l = 1.f / red[0];

  // P.V: thread = (key group g, 8-dim chunk c), tid = g * nc + c; with nc not dividing
  // DA_NT (e.g. hd 24, 40, 48, 56) the last DA_NT - G nc threads sit out
  const int G = DA_NT / nc;
  const int c = tid % nc, g = tid / nc;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j = g; g < G && j < L; j += G) {
    const uint4* vr = reinterpret_cast<const uint4*>(j == pos ? vnew : vc + (long long)j * E);
    float f[8];
    unpack8(vr[c], f);
    const float pj = sc[j];
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += pj * f[e];
  }
  if (g < G) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[tid * 8 + e] = a[e];  // = acc[g][c * 8 + e]
  }
  __syncthreads();
  if (tid < hd) {
    float s = 0.f;
    for (int gg = 0; gg < G; ++gg) s += acc[gg * hd + tid];
    static_cast<bf16_t*>(p.o)[n * p.ldo + h * hd + tid] = f2bf(s * inv_l);
  }
}


// ---------------------------------------------------------------- few-row Linear (decode)
// y[m, n] = act(x[m, :] . w[n, :] + bias[n]) (+ residual[m, n]) for a handful of rows (M <= 16:
// one new token per sequence).  The product is a stream of the weight matrix (N x K bf16) with
// nothing for an MFMA tile to reuse, so it runs on the vector ALUs at the memory rate: a wave
// owns GV_NC consecutive output columns, lane l reads 16-B chunks k = 8 (l + 64 i) of those
// weight rows and of every x row (x is tiny and stays in L1 / L2), f32 accumulation, a
// butterfly reduction over the wave, and the bias / activation / f32 residual epilogue fused
// into the same launch (the decode step was bound by its launch count, not by the weights).
// Columns n >= Nw (a vocabulary padded past the weight's rows) are written as 0.
struct GemvArgs {
  const void* x;          // [M][ldx] bf16
  const void* w;          // [Nw][ldw] bf16, k contiguous (nn.Linear layout)
  const float* bias;      // [Nw] f32 or null
  const float* residual;  // [M][ldr] f32 or null
  void* y;                // [M][ldy] bf16 or f32
  long long ldx, ldw, ldr, ldy;
  int M, N, Nw, K;
  int act, y_f32;
};

constexpr int GV_NC = 4;  // output columns per wave

template <int MM>
__global__ __launch_bounds__(256) void gemv_kernel(GemvArgs p) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * GV_NC;
  if (n0 >= p.N) return;
  const bf16_t* X = static_cast<const bf16_t*>(p.x);
  const bf16_t* W = static_cast<const bf16_t*>(p.w);
  float acc[MM][GV_NC];
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int c = 0; c < GV_NC; ++c) acc[m][c] = 0.f;
  for (int k = 8 * lane; k < p.K; k += 512) {
    float wf[GV_NC][8];
#pragma unroll
    for (int c = 0; c < GV_NC; ++c) {
      const int n = n0 + c;
      uint4 wv = make_uint4(0u, 0u, 0u, 0u);
      if (n < p.Nw) wv = *reinterpret_cast<const uint4*>(W + (long long)n * p.ldw + k);
      unpack8(wv, wf[c]);
    }
#pragma unroll
    for (int m = 0; m < MM; ++m) {
      if (m < p.M) {
        float xf[8];
        unpack8(*reinterpret_cast<const uint4*>(X + (long long)m * p.ldx + k), xf);
#pragma unroll
        for (int c = 0; c < GV_NC; ++c)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[m][c] = fmaf(xf[e], wf[c][e], acc[m][c]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MM; ++m)
#pragma unroll
    for (int c = 0; c < GV_NC; ++c) acc[m][c] = wave_sum(acc[m][c]);
  // lane j writes (m, c) = (j / GV_NC, j % GV_NC)
  const int m = lane / GV_NC, c = lane % GV_NC, n = n0 + c;
  if (m >= p.M || n >= p.N) return;
  float v = 0.f;
#pragma unroll
  for (int mm = 0; mm < MM; ++mm)
#pragma unroll
    for (int cc = 0; cc < GV_NC; ++cc) v = (mm == m && cc == c) ? acc[mm][cc] : v;
  if (n < p.Nw) {
    if (p.bias) v += p.bias[n];
    v = act_fwd(v, p.act);
    if (p.residual) v += p.residual[(long long)m * p.ldr + n];
  } else {
    v = 0.f;
  }
  if (p.y_f32) static_cast<float*>(p.y)[(long long)m * p.ldy + n] = v;
  else static_cast<bf16_t*>(p.y)[(long long)m * p.ldy + n] = f2bf(v);
}

}  // namespace dpc

using namespace dpc;

DPC_API int dpc_decode_attn(const DecodeAttnArgs* a, hipStream_t stream) {
  if (a->N <= 0) return 0;
  if (a->hd <= 0 || a->hd % 8 || a->hd > 256 || a->Smax > DA_MAX_S || a->ldqkv % 8)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_attn_kernel, dim3((unsigned)(a->N * a->H)), dim3(DA_NT), 0, stream, *a);
  return (int)hipGetLastError();
}

// Requirements: M <= 16, K % 8 == 0, x / w rows 16-B aligned (ld % 8 == 0), N <= ldy.
DPC_API int dpc_gemv(const GemvArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  if (a->M > 16 || a->K <= 0 || a->K % 8 || a->ldx % 8 || a->ldw % 8 || a->Nw > a->N || a->N > a->ldy ||
      ((uintptr_t)a->x % 16) || ((uintptr_t)a->w % 16))
    return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((a->N + 4 * GV_NC - 1) / (4 * GV_NC)));
  if (a->M <= 1) hipLaunchKernelGGL(gemv_kernel<1>, grid, dim3(256), 0, stream, *a);
  else if (a->M <= 2) hipLaunchKernelGGL(gemv_kernel<2>, grid, dim3(256), 0, stream, *a);
  else if (a->M <= 4) hipLaunchKernelGGL(gemv_kernel<4>, grid, dim3(256), 0, stream, *a);
  else if (a->M <= 8) hipLaunchKernelGGL(gemv_kernel<8>, grid, dim3(256), 0, stream, *a);
  else hipLaunchKernelGGL(gemv_kernel<16>, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}
