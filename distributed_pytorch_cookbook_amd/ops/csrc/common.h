// Shared device helpers for the CDNA4 (gfx950 / MI355X) kernels of the cookbook.
//
// Conventions used by every kernel in this directory:
//   * wave64 everywhere: lane = threadIdx.x & 63, block sizes are multiples of 64.
//   * bf16 is carried as raw 16-bit payloads (unsigned short) in memory and widened
//     to f32 with a shift; narrowing uses the compiler's round-to-nearest-even cast
//     (hipcc emits v_cvt_pk_bf16_f32, which keeps NaNs NaN).
//   * memory-bound kernels move 16 B per lane (uint4 = 8 x bf16 or 4 x f32).
//   * every launcher is a C-ABI function taking an argument struct by pointer and a
//     hipStream_t, returning the hipError_t of the launch (0 == success).  Python
//     binds them with ctypes (ops/_lib.py); no torch headers are needed here, so the
//     whole library cross-compiles in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#define DPC_API extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;  // raw bf16 payload
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace dpc {

// sfor<N>(f): f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>) -- a loop whose index
// is a compile-time constant in the body (template arguments, register-array indices)
template <int... Is, class F>
__device__ __forceinline__ void sfor_seq(std::integer_sequence<int, Is...>, F&& f) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_seq(std::make_integer_sequence<int, N>{}, f);
}

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return *reinterpret_cast<bf16_t*>(&b);
}

// pack two floats into one dword of 2 x bf16 (lo = a, hi = b): ONE v_cvt_pk_bf16_f32.
// (Two scalar conversions OR-ed together cost ~5 instructions per pair.)
typedef __bf16 dpc_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float dpc_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack2bf(float a, float b) {
  const dpc_f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, dpc_bf16x2_t));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]);
  r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]);
  r.w = pack2bf(f[6], f[7]);
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blocks of NW waves; `red` must hold NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  return t;
}

template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  return t;
}

// GPT-2 "gelu_new": 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))).
// With 0.5 (1 + tanh(u)) = sigmoid(2u) this is x * sigmoid(2u): one v_exp_f32 and one
// v_rcp_f32 instead of libm tanhf (a branchy ~40-instruction routine that dominated the
// GEMM epilogues).  exp overflow (x << 0) gives rcp(inf) = 0, i.e. gelu -> -0.
__device__ __forceinline__ float sigmoid2u(float x, float x2) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u2 = -2.f * k0 * (x + k1 * x2 * x);
  return __builtin_amdgcn_rcpf(1.f + __expf(u2));
}

__device__ __forceinline__ float gelu_tanh(float x) { return x * sigmoid2u(x, x * x); }

// d/dx: s + x * s (1 - s) * 2 k0 (1 + 3 k1 x^2), s = sigmoid(2u)  (1 - tanh^2 = 4 s (1 - s))
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float s = sigmoid2u(x, x2);
  return s + x * s * (1.f - s) * (2.f * k0) * (1.f + 3.f * k1 * x2);
}

// gelu_tanh_grad of two values in packed-f32 math (v_pk_fma / v_pk_mul: half the vector-ALU
// issue of the scalar form; the exp / rcp stay per element).  Same formula, log2(e) folded
// into the exponent's coefficients.
typedef float dpc_f2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ dpc_f2_t gelu_tanh_grad2(dpc_f2_t x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, L2E = 1.4426950408889634f;
  const dpc_f2_t x2 = x * x;
  const dpc_f2_t u = x * (x2 * (-2.f * k0 * k1 * L2E) + (-2.f * k0 * L2E));  // -2 u log2(e)
  dpc_f2_t s;
  s.x = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.x));
  s.y = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.y));
  const dpc_f2_t t = x2 * (6.f * k0 * k1) + 2.f * k0;  // 2 k0 (1 + 3 k1 x^2)
  return (x * s) * (1.f - s) * t + s;
}

__device__ __forceinline__ dpc_f2_t gelu_tanh2(dpc_f2_t x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, L2E = 1.4426950408889634f;
  const dpc_f2_t u = x * ((x * x) * (-2.f * k0 * k1 * L2E) + (-2.f * k0 * L2E));
  dpc_f2_t s;
  s.x = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.x));
  s.y = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.y));
  return x * s;
}

// GELU and its derivative at once (packed f32): the forward epilogue of the FFN up-projection
// stores bf16 GELU'(z) as its second output, so the input-gradient epilogue of the backward is a
// plain multiply (ACT_MUL) instead of a second exp / rcp per element.  Same s = sigmoid(2u) for
// both: GELU = x s, GELU' = s + x s (1 - s) 2 k0 (1 + 3 k1 x^2).
__device__ __forceinline__ dpc_f2_t gelu_tanh_fg2(dpc_f2_t x, dpc_f2_t& d) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, L2E = 1.4426950408889634f;
  const dpc_f2_t x2 = x * x;
  const dpc_f2_t u = x * (x2 * (-2.f * k0 * k1 * L2E) + (-2.f * k0 * L2E));
  dpc_f2_t s;
  s.x = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.x));
  s.y = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u.y));
  const dpc_f2_t xs = x * s;
  const dpc_f2_t t = x2 * (6.f * k0 * k1) + 2.f * k0;
  d = (xs - xs * s) * t + s;
  return xs;
}

// ACT_MUL (input-gradient epilogues only): the act' operand already holds act'(z) -- written by
// a forward epilogue with GemmArgs::aux_deriv -- and is multiplied in as is
enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_MUL = 3 };

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_GELU) return gelu_tanh(v);
  return v;
}

// derivative of act evaluated from the saved pre-activation z
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_GELU) return gelu_tanh_grad(z);
  if (act == ACT_MUL) return z;
  return 1.f;
}

// ---- counter-based dropout keep mask (torch twin: ops/dropout.py:keep_mask).  Element idx
// of a site is kept iff fmix32(idx * 0x9E3779B1 ^ key) >= thresh; kept values are scaled.
__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float drop_factor(uint32_t idx, uint32_t key, uint32_t thresh, float scale) {
  return fmix32((idx * 0x9E3779B1u) ^ key) >= thresh ? scale : 0.f;
}

// The site key from a per-forward seed held in DEVICE memory (seed[0] = the model's forward
// counter, seed[1] = the per-rank base: ops/dropout.py:DropSpec.make's hash, bit for bit), so a
// replayed HIP graph draws fresh masks every step instead of the key frozen at capture.
// seed == nullptr: the host-computed key.
__device__ __forceinline__ uint32_t drop_key_of(const unsigned* seed, unsigned site, uint32_t host_key) {
  if (!seed) return host_key;
  return fmix32(fmix32(seed[0]) ^ fmix32(seed[1] + 0x632BE5ABu * (site + 1u)));
}

}  // namespace dpc
