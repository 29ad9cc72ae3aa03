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

}  // namespace dpc

using namespace dpc;

DPC_API int dpc_decode_attn(const DecodeAttnArgs* a, hipStream_t stream) {
  if (a->N <= 0) return 0;
  if (a->hd <= 0 || a->hd % 8 || a->hd > 256 || a->Smax > DA_MAX_S || a->ldqkv % 8)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_attn_kernel, dim3((unsigned)(a->N * a->H)), dim3(DA_NT), 0, stream, *a);
  return (int)hipGetLastError();
}
