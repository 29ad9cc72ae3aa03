// Shared pieces of the gfx950 GEMM kernels (gemm.hip: v1-v6 + dispatcher, gemm7.hip: the
// persistent 4-wave kernel): the argument struct, LDS operand images and their fragment reads,
// and the LDS-DMA (buffer_load ... lds) tile issue.
#pragma once
#include "common.h"

namespace dpc {

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const float* bias;      // [N] f32, optional
  const float* residual;  // [M][ldr] f32, optional (may alias C)
  const void* aux_in;     // [M][ld_aux_in] bf16, optional: multiply by act'(aux_in)
  void* aux_out;          // [M][ld_aux_out] bf16, optional: store pre-activation
  const float* alpha_ptr; // device scalar multiplier, optional
  float* colsum;          // [N] f32, optional: colsum[n] += sum_m v (v after act_bwd, before act)
  long long lda, ldb, ldc, ldr, ld_aux_in, ld_aux_out;
  int M, N, K;
  float alpha;
  int act;         // activation applied after bias (Act)
  int act_bwd;     // multiply by act'(aux_in) (Act)
  int out_f32;     // C is f32 (else bf16)
  int accumulate;  // C += result (f32 output only)
  int a_kmaj, b_kmaj;
  // stored extents of the operands ([rows][cols] as laid out in memory); reads beyond them
  // return zeros.  k-major: rows = M or N, cols = K;  mn-major: rows = K, cols = M or N.
  int a_r, a_c, b_r, b_c;
  // set by the dispatcher (callers pass 0): > 1 = XCD-aligned split-K into this many k-ranges
  int ksplit;
  // caller's implementation choice (0 = the dispatcher's shape policy), e.g. from the
  // measured per-shape table of ops/gemm.py (autotuned on MI355X); a forced global impl
  // (dpc_gemm_set_impl, sweeps / tests) takes precedence
  int impl;
  // gemm_f32.hip only: aux_in / aux_out are f32 (else bf16)
  int aux_f32;
  // split-K workspace (optional, f32, ws_bytes long): the v7 kernel stores each k-range's
  // partial tile there with plain stores and a reduction pass sums them into C, instead of
  // f32 atomics into C (gemm7.hip: dpc_gemm7)
  void* ws;
  long long ws_bytes;
  // set by the dispatcher (callers pass 0): epilogue stores with the non-temporal bit -- bit 0 the
  // bf16 C / aux_out stores, bit 1 the f32 C stores (DPC_GEMM_NT, default 3).  The short-K
  // forward products spent 20-35 % of their time in the tile-end store burst; with nt stores
  // v9 runs the GPT-2 QKV / up / LM-head forward 947 / 964 / 1031 -> 1151 / 1150 / 1163 TF/s
  // and 8192^3 1327 -> 1448 (bench/g7lab epi set, profiles/r4_gemm/lab_epi_nt.log)
  int nt_store;
  // forward epilogues with aux_out and act == ACT_GELU: aux_out = bf16(act'(v)) instead of the
  // pre-activation bf16(v), for an input gradient with act_bwd = ACT_MUL (models/fused.py: the
  // FFN up-projection)
  int aux_deriv;
};

// 16-B epilogue stores, plain or non-temporal (GemmArgs::nt_store; the flag is a kernel
// argument, so the branch is wave-uniform)
__device__ __forceinline__ void st16(void* ptr, uint4 v, bool nt) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  if (nt) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(ptr));
  else *reinterpret_cast<uint4*>(ptr) = v;
}
// the same with the epilogue's cache scope (GemmArgs::nt_store bits 2-3, default 3: gemm.hip
// gemm_nt_mode): 0 = st16's nt / plain, 1 = sc0 nt, 2 = sc1 nt, 3 = sc0 sc1 nt
// the f32 outputs' store scope: GemmArgs::nt_store bits 4-5 when bit 6 is set, else the bf16
// outputs' scope (bits 2-3).  (f32 outputs -- the residual stream, split-K slabs -- are re-read
// soon by the next kernel; A/B of a separate scope for them)
// With bit 6: 0 = plain stores (-1 here), 1 sc0 nt, 2 sc1 nt, 3 sc0 sc1 nt.
// the default bf16 store policy (DPC_GEMM_NT's default 77: bits 2-3 = 3, sc0 sc1 nt), which the
// fused epilogues specialised at compile time assume; the dispatcher sends a product to them only
// when its nt_store carries that policy (g_sp_default)
constexpr int G_SP_DEFAULT = 3;
__host__ __device__ __forceinline__ bool g_sp_default(int nt_store) { return ((nt_store >> 2) & 3) == G_SP_DEFAULT; }
__device__ __forceinline__ int g_f32_pol(int nt_store) {
  if (!(nt_store & 64)) return (nt_store >> 2) & 3;
  const int v = (nt_store >> 4) & 3;
  return v == 0 ? -1 : v;
}
__device__ __forceinline__ void st16p(void* ptr, uint4 v, bool nt, int pol) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 w{v.x, v.y, v.z, v.w};
  // (the trailing s_nop 1: gfx950's VMEM store-data hazard -- a VALU write to the data VGPRs of a
  // dwordx3 / x4 store within 2 cycles corrupts the stored data.  The compiler puts exactly this
  // s_nop 1 after its own stores (checked in a gfx950 listing) but cannot see inside asm: with a
  // compile-time policy there is no branch after the store to absorb it, and 87 of the 896 stores
  // of the v9 forward epilogue were followed at once by a VALU write of their data registers --
  // scattered NaNs in test_gemm_v7_v8_v9, round 6)
  if (pol == 1) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt\n\ts_nop 1" ::"v"(ptr), "v"(w) : "memory");
  else if (pol == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(ptr), "v"(w) : "memory");
  else if (pol == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt\n\ts_nop 1" ::"v"(ptr), "v"(w) : "memory");
  else if (nt) __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(ptr));
  else *reinterpret_cast<uint4*>(ptr) = v;
}
__device__ __forceinline__ void st16p(void* ptr, float4 v, bool nt, int pol) {
  st16p(ptr, make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)), nt,
        pol);
}
__device__ __forceinline__ void st8(void* ptr, uint2 v, bool nt) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  if (nt) __builtin_nontemporal_store(u32x2{v.x, v.y}, reinterpret_cast<u32x2*>(ptr));
  else *reinterpret_cast<uint2*>(ptr) = v;
}
__device__ __forceinline__ void st16(void* ptr, float4 v, bool nt) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  if (nt) __builtin_nontemporal_store(f32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4*>(ptr));
  else *reinterpret_cast<float4*>(ptr) = v;
}

constexpr int BM = 128, BN = 128, BKT = 64, NT = 256;
constexpr int TILE_ELEMS = BM * BKT;  // 8192 bf16 = 16 KiB per operand per stage
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) void* lds_void_t;

// ---- LDS addressing (element offsets inside one operand tile) ----
__device__ __forceinline__ int kmaj_off(int row, int chunk) {  // chunk = 8 k-elements
  return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3);
}
__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
__device__ __forceinline__ int mnmaj_off(int k, int col) {      // col multiple of 4
  const int blk = col >> 4, within = col & 15;
  return k * 128 + (((blk ^ mn_swz(k)) << 4) | within);
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X[r = l & 15][k = 8 (l >> 4) + j].
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const bf16_t* lds, int r0, int kstep, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int chunk = kstep * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off(row, chunk));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int k = kstep * 32 + 8 * g + q;
    const int col = r0 + 4 * pp;
    typedef short4_t __attribute__((address_space(3))) * lptr;
    short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds + mnmaj_off(k, col)));
    short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds + mnmaj_off(k + 4, col)));
    typedef short short8_t __attribute__((ext_vector_type(8)));
    short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, s);
  }
}

// ---- v2 geometry, templated on the k-depth KB of a stage (64 or 32)
template <int KB>
__device__ __forceinline__ int swz_k(int row) {  // 16-B chunk swizzle of a k-major [row][KB] tile
  if (KB == 64) return (row >> 1) & 7;
  const int q = (row >> 2) & 3;  // KB == 32: 4 chunks per 64-B row, 4 rows per bank row
  return (0x1320 >> (q * 4)) & 3;  // {0, 2, 3, 1}[q]
}
template <int KB>
__device__ __forceinline__ int kmaj_off_k(int row, int chunk) {
  return row * KB + ((chunk ^ swz_k<KB>(row)) << 3);
}

template <int KB, bool KMAJ>
__device__ __forceinline__ bf16x8 frag_k(const bf16_t* lds, int r0, int kstep, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int chunk = kstep * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off_k<KB>(row, chunk));
  }
  return frag<false>(lds, r0, kstep, lane);  // [KB][128] mn-major image, 256-B rows
}

// per-thread DMA source offsets of one operand tile (relative to the tile origin)
template <int KB, bool KMAJ>
__device__ __forceinline__ void dma_offsets(int (&v)[KB / 16], long long ld, int wid, int lane) {
  constexpr int NL = KB / 16;  // 1-KiB wave-instructions per wave per operand tile
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int j = wid * NL + i;
    if (KMAJ) {
      constexpr int LPR = KB / 8;       // lanes per row (16 B each)
      constexpr int RPI = 64 / LPR;     // rows per wave-instruction
      const int row = RPI * j + lane / LPR, pos = lane % LPR, c = pos ^ swz_k<KB>(row);
      v[i] = (int)(((long long)row * ld + c * 8) * 2);
    } else {
      const int kr = 4 * j + (lane >> 4), pos = lane & 15;
      const int c = (((pos >> 1) ^ mn_swz(kr)) << 1) | (pos & 1);
      v[i] = (int)(((long long)kr * ld + c * 8) * 2);
    }
  }
}

template <int KB, bool KMAJ, int NL>
__device__ __forceinline__ void dma_offsets3(int (&v)[NL], long long ld, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int j = wid * NL + i;
    if (KMAJ) {
      constexpr int LPR = KB / 8, RPI = 64 / LPR;
      const int row = RPI * j + lane / LPR, pos = lane % LPR, c = pos ^ swz_k<KB>(row);
      v[i] = (int)(((long long)row * ld + c * 8) * 2);
    } else {
      constexpr int IPH = KB / 4;  // wave-instructions per 128-column half
      const int h = j / IPH, kr = 4 * (j % IPH) + (lane >> 4), pos = lane & 15;
      const int c = (((pos >> 1) ^ mn_swz(kr)) << 1) | (pos & 1);
      v[i] = (int)(((long long)kr * ld + h * 128 + c * 8) * 2);
    }
  }
}

template <int KB, bool KMAJ>
__device__ __forceinline__ bf16x8 frag3(const bf16_t* lds, int r0, int kstep, int lane) {
  if (KMAJ) return frag_k<KB, true>(lds, r0, kstep, lane);
  return frag<false>(lds + (r0 >> 7) * KB * 128, r0 & 127, kstep, lane);
}

template <int NL>
__device__ __forceinline__ void issue_tile_v(const void* base, unsigned long long total, unsigned long long off,
                                             bool valid, const int* voff, bf16_t* lds_tile, int wave) {
  const unsigned long long left = (valid && off < total) ? total - off : 0ull;
  const unsigned nrec = left > 0xffffffffull ? 0xffffffffu : (unsigned)left;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (valid ? off : 0ull)), 0, nrec, 0x00020000);
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int j = wave * NL + i;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t)(lds_tile + j * 512), 16, voff[i], 0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace dpc
