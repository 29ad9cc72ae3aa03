// Device side of the persistent v7 / v8 / v7d GEMM kernels (host dispatch: gemm7.hip; the
// design notes are at the top of gemm7.hip).  A header so that bench/g7lab.hip can build
// single instantiations of the kernels for ablations and A/B runs in seconds.
#pragma once
#include "gemm.h"

#include <algorithm>
#include <cstdlib>
#include <utility>

namespace dpc {

constexpr int G7_KB = 32;              // k depth of a slice
constexpr int G7_TA = 256 * G7_KB;     // bf16 elements per operand per slice (16 KiB)
constexpr int G7_SLOT = 2 * G7_TA;     // A + B
constexpr int G7_NL = G7_TA / 512 / 4; // 1-KiB DMA pieces per wave per operand per slice (4)

struct G7Plan {
  int tiles_m, tiles_n;
  int tile_n;  // tile width: 256 (v7) or 128 (v8)
  int units;   // tiles x splits (split-major: unit = split * tiles + tile)
  int grid;    // workgroups launched
  int nk;      // k-slices per unit (even)
  int nk_all;  // k-slices of the whole product (slices of a unit past it read zeros)
  int splits;
  int store_cnt;  // vector-memory ops the epilogue issues per wave-lane (0: unknown -> no credit)
  int debug;      // experiments only (DPC_G7_DEBUG): 1 = no epilogue (main-loop ablations: ABL, bench/g7lab.hip)
};

// XCD-aware assignment: round i covers units [i*grid, (i+1)*grid); inside a round the blocks
// that share an XCD (b % 8) get a contiguous run of unit ids (bijective for any grid), and unit
// ids walk GROUP_M-row supertiles, so an XCD's concurrent tiles share A/B panels in its L2.
__device__ __forceinline__ int g7_local(int b, int grid) {
  const int xcd = b & 7, q = grid >> 3, r = grid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

__device__ __forceinline__ void g7_tile(const G7Plan& pl, int u, int& m0, int& n0) {
  const int group = GROUP_M * pl.tiles_n;
  const int gid = u / group, first_m = gid * GROUP_M;
  const int gsz = min(pl.tiles_m - first_m, GROUP_M);
  const int w = u - gid * group;
  m0 = (first_m + w % gsz) * 256;
  n0 = (w / gsz) * pl.tile_n;
}

// One 1-KiB LDS-DMA piece (buffer_load_dwordx4 ... lds: 64 lanes x 16 B, lane-linear at M0).
// Issued from inline asm ON PURPOSE: hipcc (ROCm 7.2) answers a compiler-visible LDS-DMA with an
// s_waitcnt vmcnt(0) in front of every later ds_read_b64_tr_b16 (the transposing read of the
// mn-major images), which drained the whole prefetch ring once per fragment and held the
// B-n-major / weight-gradient layouts at ~380 TF/s.  Hidden in asm the DMA is ordered only by
// this kernel's own counted vmcnt + barrier (see the synchronisation notes above); the compiler
// never counts these loads, so every vmcnt it emits for its own loads over-waits (safe).
// M0 (the LDS destination base) is saved and restored around the piece.
__device__ __forceinline__ void g7_piece(__amdgpu_buffer_rsrc_t rs, int voff, const bf16_t* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(la)
      : "memory");
}

// Two adjacent 1-KiB pieces under ONE M0 write (SCHED 3): the second lands 1 KiB later in
// LDS through the instruction offset, which MUBUF adds to the LDS address and to the memory
// offset alike -- so its voffset is pre-biased by -1024 (g7 host check: every biased voffset
// stays >= 0).  M0 is declared clobbered instead of saved / restored around each piece.
__device__ __forceinline__ void g7_piece2(__amdgpu_buffer_rsrc_t rs, int v0, int v1b, const bf16_t* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  asm volatile(
      "s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen offset:1024 lds"
      :
      : "v"(v0), "v"(v1b), "s"(rs), "s"(la)
      : "memory", "m0");
}

// Four adjacent pieces under one M0 write (SCHED 4): instruction offsets 0 / 1 / 2 / 3 KiB,
// voffsets pre-biased by the same amounts.
__device__ __forceinline__ void g7_piece4(__amdgpu_buffer_rsrc_t rs, int v0, int v1b, int v2b, int v3b,
                                          const bf16_t* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  asm volatile(
      "s_mov_b32 m0, %5\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %4, 0 offen lds\n\t"
      "buffer_load_dwordx4 %1, %4, 0 offen offset:1024 lds\n\t"
      "buffer_load_dwordx4 %2, %4, 0 offen offset:2048 lds\n\t"
      "buffer_load_dwordx4 %3, %4, 0 offen offset:3072 lds"
      :
      : "v"(v0), "v"(v1b), "v"(v2b), "v"(v3b), "s"(rs), "s"(la)
      : "memory", "m0");
}

// SCHED 6: a DMA pair split into its three instructions, so that each can sit in its own MFMA
// gap (one vector-memory / M0 instruction per 16-cycle MFMA instead of a 4-instruction burst at
// the head of a group).  M0 is written by the first and read by the two loads; nothing the
// compiler places between them (MFMAs, ds_read_b128 / ds_read_b64_tr_b16, SALU) uses M0 on
// gfx950.  The loads' voffsets are pre-biased as for g7_piece2.
__device__ __forceinline__ void g7_m0(const bf16_t* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  asm volatile("s_mov_b32 m0, %0" ::"s"(la) : "memory", "m0");
}
template <int OFF>
__device__ __forceinline__ void g7_ld(__amdgpu_buffer_rsrc_t rs, int voff) {
  asm volatile("buffer_load_dwordx4 %0, %1, 0 offen offset:%2 lds" ::"v"(voff), "s"(rs), "n"(OFF) : "memory");
}

template <int N>
__device__ __forceinline__ void g7_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- epilogue straight from the swapped accumulators.  Lane l, accumulator (i, j), register
// r holds C[mw + 16 i + (l & 15)][nw + 16 j + 4 (l >> 4) + r].  Same semantics and order as
// epi_tile (gemm.hip) / ops/gemm.py:_gemm_ref.
// MODE 0: plain products only (alpha, bf16 or f32 C, no accumulate) -- the hot path, with the
// register budget of the main loop untouched.  MODE 1: forward epilogues (bias, activation,
// the pre-activation aux_out, f32 residual or accumulated C).  MODE 3: input-gradient
// epilogues (act'(aux_in) and bias-gradient column sums).  Splitting the fused work in two
// keeps each epilogue's live set (operand prefetch + bias or column sums) small enough that
// nothing of the main loop spills: a spill reload in the loop is a vector-memory op, which
// breaks the counted DMA waits.
// (sfor<N>, the compile-time loop: common.h -- the fused row body is beyond clang's full-unroll
// threshold and a rolled loop indexes acc[i] dynamically, which moves all 256 accumulators to
// scratch)

#define G7_AI __attribute__((always_inline))
typedef unsigned g7_u32x4 __attribute__((ext_vector_type(4)));
// 16-B buffer store with the epilogue's cache policy (GemmArgs::nt_store bits 2-3, wave-uniform):
// 0 nt, 1 sc0 nt, 2 sc1 nt, 3 sc0 sc1 nt
__device__ __forceinline__ void g7_bst16(g7_u32x4 v, __amdgpu_buffer_rsrc_t rs, unsigned off, int pol) {
  if (pol == 2) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 18);
  else if (pol == 3) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 19);
  else if (pol == 1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 3);
  else if (pol < 0) __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 0);  // (g_f32_pol: plain)
  else __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 2);
}
typedef float g7_f32x4 __attribute__((ext_vector_type(4)));

// alpha x *alpha_ptr through the scalar cache.  As a vector load (what the compiler emits for
// the plain dereference) the value is waited for with vmcnt(0) at the top of every epilogue of
// the persistent kernels, which drains the next tile's already issued operand stages each tile.
__device__ __forceinline__ float g7_alpha(const GemmArgs& p) {
  float a = p.alpha;
  if (p.alpha_ptr) {
    float v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p.alpha_ptr) : "memory");
    a *= v;
  }
  return a;
}

#ifndef G7_EPI_PF
#define G7_EPI_PF 0  // 0 = the default depth per epilogue (A/B builds override)
#endif

// lane l <- lane l ^ 8 within each 16-lane row (DPP row_ror:8, a VALU op)
__device__ __forceinline__ unsigned g7_ror8(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);
}
__device__ __forceinline__ float g7_ror8(float v) { return __uint_as_float(g7_ror8(__float_as_uint(v))); }

// PK: GELU / GELU' in packed-f32 math (v8 with a K-major A, v7's forward epilogues)
// NOLD: MODE 1 known at compile time to read nothing per element (no residual / accumulate --
// v9's forward epilogue): no operand prefetch registers
// lbias (NOLD only): the wave's 128 bias values in LDS (v9 stages them by DMA with the tile's
// operands) -- no vector load in the epilogue, so nothing there waits on vmcnt, which would
// drain the next tile's operand stages already in flight
// FA / FULL (MODE 1 only): the activation known at compile time (-1: read p.act per element
// group) and a full 256 x 256 tile with a bf16 output -- no per-element bounds checks.  The
// round-5 asm of the v9 forward epilogue showed every element group wrapped in ~10 scalar
// branches (the runtime activation switch, the m / n guards of each store): the bias-only form
// ran 57 us over the plain product of the GPT-2 up-projection (bench/epi_decomp.py).
// AD (MODE 1, FA == ACT_GELU only): aux_out takes GELU'(v) (GemmArgs::aux_deriv known at compile
// time); the generic copy (FA < 0) reads p.aux_deriv instead
// SP (MODE 1): the bf16 stores' cache policy at compile time (st16p pol; -1 = GemmArgs::nt_store at
// run time).  The run-time policy is a 4-way switch in front of EVERY store of the unrolled
// epilogue -- ~2 scalar branches per 16-B store in the round-6 asm of the v9 forward epilogue.
template <int MODE, int NJ, bool PK = false, bool NOLD = false, int FA = -1, bool FULL = false, bool AD = false,
          int SP = -1>
__device__ __forceinline__ void g7_epilogue(const GemmArgs& p, floatx4 (&acc)[8][NJ], int mw, int nw, int lane,
                                            int dbg = 0, const float* lbias = nullptr) {
  static_assert(!FULL || MODE == 1, "full-tile fast path: forward epilogues");
  const float alpha = g7_alpha(p);
  const int g = lane >> 4, rl = lane & 15;
  // bf16 outputs leave in 16-B stores: after v_permlane16_swap of fragments (j, j+1) lane
  // group g holds columns 16 j + {0, 16, 8, 24}[g] .. +7 (host: N % 8 == 0, ldc % 8 == 0,
  // C 16-B aligned)
  const int coff = 16 * (g & 1) + 8 * (g >> 1);
  if constexpr (MODE == 0) {
    // Row-coalesced stores: a lane group of 16 lanes holds 16 rows, so one store instruction of
    // the register layout covers 16 rows x 64 B (half lines).  Lanes l and l ^ 8 (rows r and
    // r + 8) trade one 16-B chunk through a DPP row rotate, so each instruction covers 8 rows x
    // 128 B instead: rows 0-7 of two adjacent 64-B column chunks, then rows 8-15 -- the same
    // instruction count, full cache lines (measured +9-11 % on the K = 768 forward products with
    // a lane-linear layout of the same stores).
    const bool lo = rl < 8;
    const int rr = rl & 7, hi8 = rl >> 3;
    if (p.out_f32) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < NJ; j += 2) {
          // (the empty volatile asm pins each fragment's read here: hoisted, the reads of later
          // rows would all be live at once and spill)
          floatx4 a0 = acc[i][j], a1 = acc[i][j + 1];
          asm volatile("" : "+v"(a0), "+v"(a1));
          float4 c0 = make_float4(a0[0] * alpha, a0[1] * alpha, a0[2] * alpha, a0[3] * alpha);
          float4 c1 = make_float4(a1[0] * alpha, a1[1] * alpha, a1[2] * alpha, a1[3] * alpha);
          const float4 snd = make_float4(lo ? c1.x : c0.x, lo ? c1.y : c0.y, lo ? c1.z : c0.z, lo ? c1.w : c0.w);
          const float4 rcv = make_float4(g7_ror8(snd.x), g7_ror8(snd.y), g7_ror8(snd.z), g7_ror8(snd.w));
          const float4 dA = make_float4(lo ? c0.x : rcv.x, lo ? c0.y : rcv.y, lo ? c0.z : rcv.z, lo ? c0.w : rcv.w);
          const float4 dB = make_float4(lo ? rcv.x : c1.x, lo ? rcv.y : c1.y, lo ? rcv.z : c1.z, lo ? rcv.w : c1.w);
          const int m = mw + 16 * i + rr, n = nw + 16 * j + 4 * g + 16 * hi8;
          if (n < p.N) {
            float* C = static_cast<float*>(p.C) + (long long)m * p.ldc + n;
            if (m < p.M) st16p(C, dA, p.nt_store & 2, g_f32_pol(p.nt_store));
            if (m + 8 < p.M) st16p(C + 8 * p.ldc, dB, p.nt_store & 2, g_f32_pol(p.nt_store));
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; j += 4) {
        // c0: row rl, columns 16 j + coff .. +7 (blocks j, j+1); c1: the same 32 columns on
        // (blocks j+2, j+3).  Named values, never an array: a per-lane select between array
        // elements becomes a dynamically indexed private array (scratch).
        uint4 c0, c1;
        {
          floatx4 a0 = acc[i][j], a1 = acc[i][j + 1], a2 = acc[i][j + 2], a3 = acc[i][j + 3];
          asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));  // (pinned reads)
          const auto s0 = __builtin_amdgcn_permlane16_swap(pack2bf(a0[0] * alpha, a0[1] * alpha),
                                                           pack2bf(a1[0] * alpha, a1[1] * alpha), false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pack2bf(a0[2] * alpha, a0[3] * alpha),
                                                           pack2bf(a1[2] * alpha, a1[3] * alpha), false, false);
          const auto t0 = __builtin_amdgcn_permlane16_swap(pack2bf(a2[0] * alpha, a2[1] * alpha),
                                                           pack2bf(a3[0] * alpha, a3[1] * alpha), false, false);
          const auto t1 = __builtin_amdgcn_permlane16_swap(pack2bf(a2[2] * alpha, a2[3] * alpha),
                                                           pack2bf(a3[2] * alpha, a3[3] * alpha), false, false);
          c0 = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          c1 = make_uint4(t0[0], t1[0], t0[1], t1[1]);
        }
        const uint4 snd = make_uint4(lo ? c1.x : c0.x, lo ? c1.y : c0.y, lo ? c1.z : c0.z, lo ? c1.w : c0.w);
        const uint4 rcv = make_uint4(g7_ror8(snd.x), g7_ror8(snd.y), g7_ror8(snd.z), g7_ror8(snd.w));
        const uint4 dA = make_uint4(lo ? c0.x : rcv.x, lo ? c0.y : rcv.y, lo ? c0.z : rcv.z, lo ? c0.w : rcv.w);
        const uint4 dB = make_uint4(lo ? rcv.x : c1.x, lo ? rcv.y : c1.y, lo ? rcv.z : c1.z, lo ? rcv.w : c1.w);
        const int m = mw + 16 * i + rr, n = nw + 16 * j + coff + 32 * hi8;
        if ((dbg & 4) || ((dbg & 8) && (blockIdx.x & 1))) {  // (experiments: the epilogue's VALU
          // without its stores -- on every workgroup (4) or on every other one (8))
          asm volatile("" ::"v"(dA.x), "v"(dA.y), "v"(dA.z), "v"(dA.w), "v"(dB.x), "v"(dB.y), "v"(dB.z), "v"(dB.w));
        } else if (n < p.N) {
          bf16_t* C = static_cast<bf16_t*>(p.C) + (long long)m * p.ldc + n;
          const bool nt = (p.nt_store & 1) || (dbg & 16);  // (dbg 16: the lab's nt arm)
          if (m < p.M) st16p(C, dA, nt, (p.nt_store >> 2) & 3);
          if (m + 8 < p.M) st16p(C + 8 * p.ldc, dB, nt, (p.nt_store >> 2) & 3);
        }
      }
    }
    return;
  }
  constexpr bool FWD = MODE == 1;
  // per-element operand reads (FWD: the f32 residual / accumulated C; else act''s bf16
  // operand), prefetched PF row blocks ahead: as soon as fragment (i, j) is consumed, its slot
  // is refilled with (i + PF, j)
  const bf16_t* aux_in = static_cast<const bf16_t*>(p.aux_in);
  bf16_t* aux_out = static_cast<bf16_t*>(p.aux_out);
  const float* fsrc = (FWD && !NOLD)
                          ? (p.residual ? p.residual : (p.out_f32 && p.accumulate ? static_cast<const float*>(p.C) : nullptr))
                          : nullptr;
  const long long ldf = p.residual ? p.ldr : p.ldc;
  const bool has_ld = FWD ? fsrc != nullptr : p.act_bwd != 0;
  auto load_one = [&](int m, int n) G7_AI {
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
    if (!NOLD && has_ld && m < p.M && n < p.N) {
      if constexpr (FWD) {
        r = *reinterpret_cast<const uint4*>(fsrc + (long long)m * ldf + n);
      } else {
        const uint2 z = *reinterpret_cast<const uint2*>(aux_in + (long long)m * p.ld_aux_in + n);
        r.x = z.x;
        r.y = z.y;
      }
    }
    return r;
  };
  // PF row blocks of operand reads in flight: the input-gradient epilogue's act' operand is an
  // 8-B read per lane and fragment, latency-bound at one block ahead
  constexpr int PF = G7_EPI_PF > 0 ? G7_EPI_PF : (FWD || NJ > 4 ? 1 : 2);  // (v8; 3 - 4 spill there)
  uint4 ld[PF][NJ];
  float4 bias4[NJ];
  // (NOLD: the lane's bias column base as an LDS address)
  const float __attribute__((address_space(3)))* lb =
      (const float __attribute__((address_space(3)))*)(lds_void_t)(lbias) + 4 * g;
  float cs[NJ][4];
  sfor<NJ>([&](auto J) G7_AI {
    constexpr int j = decltype(J)::value;
    sfor<PF>([&](auto Q) G7_AI {
      constexpr int q = decltype(Q)::value;
      ld[q][j] = load_one(mw + 16 * q + rl, nw + 16 * j + 4 * g);
    });
    if constexpr (FWD && NOLD) {
      const floatx4 b = *reinterpret_cast<const floatx4 __attribute__((address_space(3)))*>(lb + 16 * j);
      bias4[j] = make_float4(b[0], b[1], b[2], b[3]);
    } else if constexpr (FWD) {
      const int n = nw + 16 * j + 4 * g;
      bias4[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else if constexpr (!FWD) {
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
    }
  });
  const int fact = FA >= 0 ? FA : p.act;  // (a constant when FA >= 0)
  sfor<8>([&](auto I) G7_AI {
    constexpr int i = decltype(I)::value;
    const int m = mw + 16 * i + rl;
    const bool mok = FULL || m < p.M;
    sfor<NJ / 2>([&](auto J) G7_AI {
      constexpr int j = 2 * decltype(J)::value;
      unsigned pa[2][2], pc[2][2];
      sfor<2>([&](auto H) G7_AI {
        constexpr int h = decltype(H)::value;
        constexpr int jj = j + h;
        const int n = nw + 16 * jj + 4 * g;
        const bool ok = FULL || (mok && n < p.N);
        const uint4 cur = ld[i % PF][jj];
        if (i + PF < 8) ld[i % PF][jj] = load_one(m + 16 * PF, n);
        float w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = acc[i][jj][r] * alpha;
        if constexpr (FWD) {
          w[0] += bias4[jj].x; w[1] += bias4[jj].y; w[2] += bias4[jj].z; w[3] += bias4[jj].w;
          if constexpr (AD) {  // GELU + GELU' (aux_out) from one sigmoid
            dpc_f2_t d01, d23;
            const dpc_f2_t g01 = gelu_tanh_fg2(dpc_f2_t{w[0], w[1]}, d01), g23 = gelu_tanh_fg2(dpc_f2_t{w[2], w[3]}, d23);
            pa[h][0] = pack2bf(d01.x, d01.y);
            pa[h][1] = pack2bf(d23.x, d23.y);
            w[0] = g01.x; w[1] = g01.y; w[2] = g23.x; w[3] = g23.y;
          } else {
            pa[h][0] = pack2bf(w[0], w[1]);  // the pre-activation (aux_out)
            pa[h][1] = pack2bf(w[2], w[3]);
            if (FA < 0 && p.aux_deriv) {  // (generic copy: act'(v) instead)
              pa[h][0] = pack2bf(act_grad(w[0], fact), act_grad(w[1], fact));
              pa[h][1] = pack2bf(act_grad(w[2], fact), act_grad(w[3], fact));
            }
            if (PK && fact == ACT_GELU) {
              const dpc_f2_t g01 = gelu_tanh2(dpc_f2_t{w[0], w[1]}), g23 = gelu_tanh2(dpc_f2_t{w[2], w[3]});
              w[0] = g01.x; w[1] = g01.y; w[2] = g23.x; w[3] = g23.y;
            } else if (FA != 0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) w[r] = act_fwd(w[r], fact);
            }
          }
          if (fsrc) {
            w[0] += __uint_as_float(cur.x); w[1] += __uint_as_float(cur.y);
            w[2] += __uint_as_float(cur.z); w[3] += __uint_as_float(cur.w);
          }
        } else {
          if (PK && p.act_bwd == ACT_GELU) {
            const dpc_f2_t g01 = gelu_tanh_grad2(dpc_f2_t{__uint_as_float(cur.x << 16), __uint_as_float(cur.x & 0xffff0000u)});
            const dpc_f2_t g23 = gelu_tanh_grad2(dpc_f2_t{__uint_as_float(cur.y << 16), __uint_as_float(cur.y & 0xffff0000u)});
            w[0] *= g01.x; w[1] *= g01.y; w[2] *= g23.x; w[3] *= g23.y;
          } else if (p.act_bwd) {
            w[0] *= act_grad(__uint_as_float(cur.x << 16), p.act_bwd);
            w[1] *= act_grad(__uint_as_float(cur.x & 0xffff0000u), p.act_bwd);
            w[2] *= act_grad(__uint_as_float(cur.y << 16), p.act_bwd);
            w[3] *= act_grad(__uint_as_float(cur.y & 0xffff0000u), p.act_bwd);
          }
          if (ok) {
#pragma unroll
            for (int r = 0; r < 4; ++r) cs[jj][r] += w[r];
          }
        }
        if (!FULL && p.out_f32) {
          if (ok) {
            float4* C = reinterpret_cast<float4*>(static_cast<float*>(p.C) + (long long)m * p.ldc + n);
            if (FWD && !NOLD && p.accumulate && p.residual) {  // (no caller does both; C read late)
              const float4 o = *C;
              w[0] += o.x; w[1] += o.y; w[2] += o.z; w[3] += o.w;
            }
            st16p(C, make_float4(w[0], w[1], w[2], w[3]), p.nt_store & 2, g_f32_pol(p.nt_store));
          }
        } else {
          pc[h][0] = pack2bf(w[0], w[1]);
          pc[h][1] = pack2bf(w[2], w[3]);
        }
      });
      const int n8 = nw + 16 * j + coff;
      const bool ok8 = FULL || (mok && n8 < p.N);
      if (FWD && aux_out) {
        const auto s0 = __builtin_amdgcn_permlane16_swap(pa[0][0], pa[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pa[0][1], pa[1][1], false, false);
        if (ok8)
          st16p(aux_out + (long long)m * p.ld_aux_out + n8, make_uint4(s0[0], s1[0], s0[1], s1[1]),
                SP >= 0 ? false : (p.nt_store & 1), SP >= 0 ? SP : (p.nt_store >> 2) & 3);
      }
      if (FULL || !p.out_f32) {
        const auto s0 = __builtin_amdgcn_permlane16_swap(pc[0][0], pc[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pc[0][1], pc[1][1], false, false);
        if (ok8)
          st16p(static_cast<bf16_t*>(p.C) + (long long)m * p.ldc + n8, make_uint4(s0[0], s1[0], s0[1], s1[1]),
                SP >= 0 ? false : (p.nt_store & 1), SP >= 0 ? SP : (p.nt_store >> 2) & 3);
      }
    });
  });
  if constexpr (!FWD) {
    if (p.colsum) {
      // sum over the 16 rows of a lane group, then lane t of group g adds columns 2t, 2t+1 of
      // the group's 32 (j = e >> 2, r = e & 3 -> column 16 j + 4 g + r)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = cs[j][r];
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          v += __shfl_xor(v, 4, 64);
          v += __shfl_xor(v, 8, 64);
          cs[j][r] = v;
        }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = 2 * rl + h;
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 4 * NJ; ++k) v = (e == k) ? cs[k >> 2][k & 3] : v;
        const int n = nw + 16 * (e >> 2) + 4 * g + (e & 3);
        if (e < 4 * NJ && n < p.N) atomicAdd(p.colsum + n, v);
      }
    }
  }
}

// MODE 3 with an act' operand on v7 (256 x 256 tiles), the operand staged through LDS: the
// per-lane 8-B reads of g7_epilogue (one 16-row block in flight ahead) leave the tile's act'
// operand as eight dependent HBM round trips -- measured ~35 us per tile on the GPT-2 up-proj
// input gradient (718 us against 299 us for the plain product).  Here the 128-KiB operand
// tile comes in four 64-row quarters (32 KiB each: the rows 32 q .. 32 q + 31 of both wave
// rows) by LDS-DMA into the two ring slots that are idle during an epilogue -- the last
// slice's (its next write is the next tile's body 0) and the next tile's slice 0 (read into
// registers by the last body) -- double-buffered, quarter q+2's DMA behind quarter q's
// processing.  A piece holds two 512-B rows; the 16-B chunk c of local row r sits at chunk
// position c ^ (r & 15), so the 16 rows a lane group reads at one column are 16 different
// bank groups.  Waits are counted: a quarter's DMA is older than the previous quarter's stores
// and the next DMA, which may stay in flight (full tiles; an edge tile, which may skip stores,
// waits for everything but the next DMA).
// (round 5: act' by a select, the next column pair's operand read ahead, bounded buffer stores --
// no branch inside the element loop; ONE copy per kernel, see the call site)
// MUL: the operand holds act'(z) already (act_bwd == ACT_MUL, written by the forward epilogue
// with aux_deriv): a plain multiply, no GELU' math (EPI 10, which also fixes the bf16 store policy
// at compile time -- SP, as in g7_epilogue -- instead of a run-time switch per store)
template <int NJ, bool MUL = false, int SP = -1>
__device__ __forceinline__ void g7_epilogue_act_lds(const GemmArgs& p, floatx4 (&acc)[8][NJ], int m0, int n0,
                                                    int wid, int lane_in, bf16_t* buf0, bf16_t* buf1) {
  static_assert(NJ == 8, "v7 tiles");
  const int fab = p.act_bwd;
  // the lane id through an opaque move: every per-lane address below is tile-invariant, and
  // hoisted out of the persistent tile loop they would stay live across the main loop (spills)
  int lane;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane_in));
  const float alpha = g7_alpha(p);
  const int g = lane >> 4, rl = lane & 15;
  const int wr = wid >> 1, wc = wid & 1;
  const int mw = m0 + wr * 128, nw = n0 + wc * 128;
  const int coff = 16 * (g & 1) + 8 * (g >> 1);
  const int ld = (int)p.ld_aux_in;
  const long long org = (long long)m0 * ld + n0;
  const long long rem = ((long long)(p.M - 1) * ld + p.N - org) * 2;  // bytes to the operand's end
  const unsigned nrec = rem <= 0 ? 0u : (rem >= 0xffffffffll ? 0xffffffffu : (unsigned)rem);
  const __amdgpu_buffer_rsrc_t rz =
      __builtin_amdgcn_make_buffer_rsrc((void*)(static_cast<const bf16_t*>(p.aux_in) + org), 0, nrec, 0x00020000);
  auto zdma = [&](int q, bf16_t* buf) G7_AI {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int lr = wid * 16 + 2 * k + (lane >> 5);  // local row 0..63
      const int tr = ((lr & 32) ? 128 : 0) + 32 * q + (lr & 31);
      const int c = (lane & 31) ^ (lr & 15);
      g7_piece(rz, (tr * ld + c * 8) * 2, buf + (wid * 8 + k) * 512);
    }
  };
  float cs[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
  // bf16 output through a buffer descriptor over the tile's span of C: a store whose row is past
  // M lies past num_records and is dropped by the hardware, one whose columns are past N gets an
  // out-of-range offset -- no per-store exec branch (the dispatcher sends f32 outputs to EPI 3)
  const long long corg = (long long)m0 * p.ldc + n0;
  const long long crem = ((long long)(p.M - 1) * p.ldc + p.N - corg) * 2;
  const unsigned cnrec = crem <= 0 ? 0u : (crem >= 0xffffffffll ? 0xffffffffu : (unsigned)crem);
  const __amdgpu_buffer_rsrc_t rc =
      __builtin_amdgcn_make_buffer_rsrc((void*)(static_cast<bf16_t*>(p.C) + corg), 0, cnrec, 0x00020000);
  const bool gelu = fab == ACT_GELU;  // (else ReLU: act_lds is taken only with an act')
  const int spol = SP >= 0 ? SP : (p.nt_store >> 2) & 3;
  auto proc = [&](auto Q, const bf16_t* buf) G7_AI {
    constexpr int q = decltype(Q)::value;
    sfor<2>([&](auto II) G7_AI {
      constexpr int i = 2 * q + decltype(II)::value;
      const int mt = wr * 128 + 16 * i + rl;  // row in the tile
      const bool rok = m0 + mt < p.M;
      const bf16_t* zrow = buf + (wr * 32 + 16 * decltype(II)::value + rl) * 256;
      auto zload = [&](int jj) G7_AI {
        const int c = wc * 16 + 2 * jj + (g >> 1);
        return *reinterpret_cast<const uint2*>(zrow + (c ^ rl) * 8 + 4 * (g & 1));
      };
      // the act' operand of the NEXT column pair is read before this pair's arithmetic: with
      // one pair per scheduling region (the barrier below) its LDS latency was exposed 128 times
      // per tile
      uint2 zc0 = zload(0), zc1 = zload(1);
      sfor<NJ / 2>([&](auto J) G7_AI {
        constexpr int j = 2 * decltype(J)::value;
        uint2 zn0 = zc0, zn1 = zc1;
        if constexpr (j + 2 < NJ) {
          zn0 = zload(j + 2);
          zn1 = zload(j + 3);
        }
        unsigned pc[2][2];
        sfor<2>([&](auto H) G7_AI {
          constexpr int h = decltype(H)::value;
          constexpr int jj = j + h;
          const uint2 z = h == 0 ? zc0 : zc1;
          float w[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) w[r] = acc[i][jj][r] * alpha;
          const float z0 = __uint_as_float(z.x << 16), z1 = __uint_as_float(z.x & 0xffff0000u);
          const float z2 = __uint_as_float(z.y << 16), z3 = __uint_as_float(z.y & 0xffff0000u);
          // GELU' in packed f32 (half the VALU issue of the scalar form), or ReLU' -- a select,
          // not a branch
          if constexpr (MUL) {
            w[0] *= z0; w[1] *= z1; w[2] *= z2; w[3] *= z3;
          } else {
            const dpc_f2_t g01 = gelu_tanh_grad2(dpc_f2_t{z0, z1}), g23 = gelu_tanh_grad2(dpc_f2_t{z2, z3});
            w[0] *= gelu ? g01.x : (z0 > 0.f ? 1.f : 0.f);
            w[1] *= gelu ? g01.y : (z1 > 0.f ? 1.f : 0.f);
            w[2] *= gelu ? g23.x : (z2 > 0.f ? 1.f : 0.f);
            w[3] *= gelu ? g23.y : (z3 > 0.f ? 1.f : 0.f);
          }
          // (rows past M: an M-major A reads the next k-row's data into acc there, and the act'
          // operand's LDS rows were never written by the DMA; columns past N may read the next
          // row's data: both are kept out of the column sums by a select)
          const bool cok = rok && n0 + wc * 128 + 16 * jj + 4 * g < p.N;
#pragma unroll
          for (int r = 0; r < 4; ++r) cs[jj][r] += cok ? w[r] : 0.f;
          pc[h][0] = pack2bf(w[0], w[1]);
          pc[h][1] = pack2bf(w[2], w[3]);
        });
        const int n8 = wc * 128 + 16 * j + coff;  // column in the tile
        const auto s0 = __builtin_amdgcn_permlane16_swap(pc[0][0], pc[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pc[0][1], pc[1][1], false, false);
        const unsigned off = (n0 + n8 < p.N) ? (unsigned)((mt * p.ldc + n8) * 2) : 0xfffffff0u;
        g7_bst16(__builtin_bit_cast(g7_u32x4, make_uint4(s0[0], s1[0], s0[1], s1[1])), rc, off, spol);
        zc0 = zn0;
        zc1 = zn1;
        __builtin_amdgcn_sched_barrier(0);  // one column pair at a time (else all are live: spills)
      });
    });
  };
  // wait until quarter q's pieces landed (every wave's): younger ops = the previous quarter's
  // 8 stores (st; every tile issues all of them now -- out-of-range ones are dropped by the
  // buffer descriptor, still counted) + the next quarter's DMA (8) when one was issued
  auto landed = [&](bool st, bool next) G7_AI {
    if (!next) {
      if (st) g7_wait<8>();
      else g7_wait<0>();
    } else if (st) {
      g7_wait<16>();
    } else {
      g7_wait<8>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto reads_done = [&]() G7_AI {  // every wave's reads of a buffer retired -> it may be refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  reads_done();  // (the last body's fragment reads of the next tile's slice 0 -- buf1)
  zdma(0, buf0);
  zdma(1, buf1);
  landed(false, true);
  proc(std::integral_constant<int, 0>{}, buf0);
  reads_done();
  zdma(2, buf0);
  landed(true, true);
  proc(std::integral_constant<int, 1>{}, buf1);
  reads_done();
  zdma(3, buf1);
  landed(true, true);
  proc(std::integral_constant<int, 2>{}, buf0);
  landed(true, false);
  proc(std::integral_constant<int, 3>{}, buf1);
  if (p.colsum) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cs[j][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        cs[j][r] = v;
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = 2 * rl + h;
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 4 * NJ; ++k) v = (e == k) ? cs[k >> 2][k & 3] : v;
      const int n = nw + 16 * (e >> 2) + 4 * g + (e & 3);
      if (n < p.N) {
        // the workspace form: this wave's partial column sums as row 2 (m0 / 256) + wr of a
        // [2 tiles_m][N] f32 matrix (g7_colsum_reduce adds its rows into colsum) -- the f32
        // atomics of every tile of a column block land on the same 256 addresses at nearly the
        // same time and serialise
        if (p.ws) static_cast<float*>(p.ws)[(long long)(2 * (m0 >> 8) + wr) * p.N + n] = v;
        else atomicAdd(p.colsum + n, v);
      }
    }
  }
  reads_done();  // both buffers are ring slots again: the next tile's bodies 0 / 1 refill them
}

// MODE 1 with an f32 residual and an f32 output on v7 (the FFN down-projection forward: bias +
// GELU + pre-activation aux_out + residual), the residual staged through LDS as in
// g7_epilogue_act_lds: eight 16-row "eighths" of the 256-KiB residual tile (row block i of both
// wave rows, 32 rows x 1 KiB = one ring slot) by LDS-DMA into the two idle ring slots,
// double-buffered; one piece = one 1-KiB row, 16-B chunk c of local row r at position
// c ^ (r & 15).  GELU in packed f32.
// (round 5: the activation by selects, the next column pair's residual read ahead, bounded buffer
// stores -- no branch inside the element loop)
template <int NJ>
__device__ __forceinline__ void g7_epilogue_res_lds(const GemmArgs& p, floatx4 (&acc)[8][NJ], int m0, int n0,
                                                    int wid, int lane_in, bf16_t* buf0, bf16_t* buf1) {
  static_assert(NJ == 8, "v7 tiles");
  const int fact = p.act;
  int lane;  // (opaque: tile-invariant per-lane addresses must not be hoisted out of the tile loop)
  asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"(lane_in));
  const float alpha = g7_alpha(p);
  const int g = lane >> 4, rl = lane & 15;
  const int wr = wid >> 1, wc = wid & 1;
  const int mw = m0 + wr * 128, nw = n0 + wc * 128;
  const int coff = 16 * (g & 1) + 8 * (g >> 1);
  const int ld = (int)p.ldr;
  const long long org = (long long)m0 * ld + n0;
  const long long rem = ((long long)(p.M - 1) * ld + p.N - org) * 4;
  const unsigned nrec = rem <= 0 ? 0u : (rem >= 0xffffffffll ? 0xffffffffu : (unsigned)rem);
  const __amdgpu_buffer_rsrc_t rr_ =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.residual + org), 0, nrec, 0x00020000);
  auto rdma = [&](int e, bf16_t* buf) G7_AI {  // eighth e: tile rows 16 e + (0..15) of both wave rows
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int lr = wid * 8 + k;  // local row 0..31 (one piece each)
      const int tr = ((lr & 16) ? 128 : 0) + 16 * e + (lr & 15);
      const int c = lane ^ (lr & 15);
      g7_piece(rr_, (tr * ld + c * 4) * 4, buf + lr * 512);
    }
  };
  // outputs through buffer descriptors over the tile's span (rows past M lie past num_records
  // and are dropped by the hardware; columns past N get an out-of-range offset; no aux_out:
  // num_records 0): every store is issued, none sits behind an exec branch
  auto span = [&](const void* base, long long ldo, int esz) G7_AI {
    const long long o = (long long)m0 * ldo + n0;
    const long long rem = base ? ((long long)(p.M - 1) * ldo + p.N - o) * esz : 0;
    const unsigned nr = rem <= 0 ? 0u : (rem >= 0xffffffffll ? 0xffffffffu : (unsigned)rem);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(static_cast<const char*>(base) + (base ? o * esz : 0)), 0, nr,
                                             0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rco = span(p.C, p.ldc, 4);
  const __amdgpu_buffer_rsrc_t rax = span(p.aux_out, p.ld_aux_out, 2);
  const bool gelu = fact == ACT_GELU, relu = fact == ACT_RELU;
  const int spol = (p.nt_store >> 2) & 3, fpol = g_f32_pol(p.nt_store);  // (bf16 aux / f32 C)
  float4 bias4[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = nw + 16 * j + 4 * g;
    bias4[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  auto proc = [&](auto E, const bf16_t* buf) G7_AI {
    constexpr int i = decltype(E)::value;
    const int mt = wr * 128 + 16 * i + rl;  // row in the tile
    const float* rrow = reinterpret_cast<const float*>(buf + (wr * 16 + rl) * 512);
    auto rload = [&](int jj) G7_AI {
      const int c = wc * 32 + 4 * jj + g;
      return *reinterpret_cast<const float4*>(rrow + (c ^ rl) * 4);
    };
    // the residual of the NEXT column pair is read before this pair's arithmetic (its LDS
    // latency was exposed once per pair behind the scheduling barrier below)
    float4 rc0 = rload(0), rc1 = rload(1);
    sfor<NJ / 2>([&](auto J) G7_AI {
      constexpr int j = 2 * decltype(J)::value;
      float4 rn0 = rc0, rn1 = rc1;
      if constexpr (j + 2 < NJ) {
        rn0 = rload(j + 2);
        rn1 = rload(j + 3);
      }
      unsigned pa[2][2];
      sfor<2>([&](auto H) G7_AI {
        constexpr int h = decltype(H)::value;
        constexpr int jj = j + h;
        const int ntc = wc * 128 + 16 * jj + 4 * g;  // column in the tile
        const float4 res = h == 0 ? rc0 : rc1;
        float w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = acc[i][jj][r] * alpha;
        w[0] += bias4[jj].x; w[1] += bias4[jj].y; w[2] += bias4[jj].z; w[3] += bias4[jj].w;
        pa[h][0] = pack2bf(w[0], w[1]);
        pa[h][1] = pack2bf(w[2], w[3]);
        // the activation by selects (GELU in packed f32, ReLU, or none), not branches
        const dpc_f2_t g01 = gelu_tanh2(dpc_f2_t{w[0], w[1]}), g23 = gelu_tanh2(dpc_f2_t{w[2], w[3]});
        const float ga[4] = {g01.x, g01.y, g23.x, g23.y};
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = gelu ? ga[r] : (relu ? fmaxf(w[r], 0.f) : w[r]);
        const unsigned off = (n0 + ntc < p.N) ? (unsigned)((mt * p.ldc + ntc) * 4) : 0xfffffff0u;
        g7_bst16(__builtin_bit_cast(g7_u32x4, make_float4(w[0] + res.x, w[1] + res.y, w[2] + res.z, w[3] + res.w)),
                 rco, off, fpol);
      });
      const int n8 = wc * 128 + 16 * j + coff;
      const auto s0 = __builtin_amdgcn_permlane16_swap(pa[0][0], pa[1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(pa[0][1], pa[1][1], false, false);
      const unsigned aoff = (n0 + n8 < p.N) ? (unsigned)((mt * p.ld_aux_out + n8) * 2) : 0xfffffff0u;
      g7_bst16(__builtin_bit_cast(g7_u32x4, make_uint4(s0[0], s1[0], s0[1], s1[1])), rax, aoff, spol);
      rc0 = rn0;
      rc1 = rn1;
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  // eighth e landed: younger = eighth e-1's stores (8 f32 + 4 aux per lane: every tile issues
  // all of them, out-of-range ones dropped by their descriptor) + the next DMA (8 pieces) when issued
  auto landed = [&](bool st, bool next) G7_AI {
    if (st) {
      if (next) g7_wait<20>();
      else g7_wait<12>();
    } else {
      if (next) g7_wait<8>();
      else g7_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto reads_done = [&]() G7_AI {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  reads_done();
  rdma(0, buf0);
  rdma(1, buf1);
  landed(false, true);
  proc(std::integral_constant<int, 0>{}, buf0);
  reads_done();
  rdma(2, buf0);
  landed(true, true);
  proc(std::integral_constant<int, 1>{}, buf1);
  reads_done();
  rdma(3, buf1);
  landed(true, true);
  proc(std::integral_constant<int, 2>{}, buf0);
  reads_done();
  rdma(4, buf0);
  landed(true, true);
  proc(std::integral_constant<int, 3>{}, buf1);
  reads_done();
  rdma(5, buf1);
  landed(true, true);
  proc(std::integral_constant<int, 4>{}, buf0);
  reads_done();
  rdma(6, buf0);
  landed(true, true);
  proc(std::integral_constant<int, 5>{}, buf1);
  reads_done();
  rdma(7, buf1);
  landed(true, true);
  proc(std::integral_constant<int, 6>{}, buf0);
  landed(true, false);
  proc(std::integral_constant<int, 7>{}, buf1);
  reads_done();
}

// split-K partial tile (non-swapped accumulators: lane l, register r of accumulator (i, j) holds
// C[mw + 16 i + 4 (l >> 4) + r][nw + 16 j + (l & 15)]): f32 atomic adds, each wave-instruction
// four rows x 64 contiguous bytes.  The host zeroes C first unless the product accumulates.
__device__ __forceinline__ void g7_epilogue_atomic(const GemmArgs& p, floatx4 (&acc)[8][8], int mw, int nw,
                                                   int lane) {
  const float alpha = g7_alpha(p);
  float* C = static_cast<float*>(p.C);
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nw + 16 * j + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mw + 16 * i + 4 * g + r;
        if (m < p.M && n < p.N) atomicAdd(C + (long long)m * p.ldc + n, acc[i][j][r] * alpha);
      }
    }
}

// EPI: 0 = plain products (bf16 / f32 C), 1 = forward fused epilogues, 2 = split-K f32 atomics,
// 3 = input-gradient fused epilogues (act', column sums), 4 = split-K partial tiles stored to
// the workspace slab of their k-range (plain 16-B stores; g7_splitk_reduce sums the slabs),
// 8 = EPI 3 with an act' operand staged through LDS (v7 only; g7_epilogue_act_lds; 10 = the same
// with act' precomputed, ACT_MUL), 9 = EPI 1
// with an f32 residual and output, the residual staged through LDS (v7 only; g7_epilogue_res_lds).
// WN: output columns per wave.  128 = v7 (a 256 x 256 tile, one workgroup per CU); 64 = v8 (a
// 256 x 128 tile, 128 accumulator registers, TWO workgroups per CU, each with a 3-slot ring:
// the two drift out of phase, so one's epilogue -- the bias / GELU / residual / act' VALU work
// and the store burst, which a lone wave per SIMD serialises against its MFMAs -- runs beside
// the other's main loop).
// ABL (bench/g7lab.hip only; every library instantiation has ABL = 0): main-loop ablations
// that keep the instruction stream otherwise unchanged -- 16 = no workgroup barrier per slice,
// 32 = no fragment reads (the prologue's fragments are reused), 64 = no counted vmcnt waits in
// the loop, 128 = per-workgroup clock stamps into g7_clk (the in-kernel clock, DVFS check).
static __device__ unsigned long long g7_clk[2 * 2048];  // (per translation unit: lab only)

template <int EPI, int SCHED, bool AK, bool BK, int WN = 128, int ABL = 0>
__global__ __launch_bounds__(256, WN == 128 ? 1 : 2) void gemm7_kernel(GemmArgs p, unsigned long long a_bytes,
                                                                       unsigned long long b_bytes, G7Plan pl) {
  constexpr int NJ = WN / 16;                 // 16-column accumulator blocks per wave
  constexpr int BW = 2 * WN;                  // tile width (B rows / columns per slice)
  constexpr int TB = BW * G7_KB;              // B elements per slice
  constexpr int SLOT = G7_TA + TB;
  constexpr int NLB = TB / 512 / 4;           // B pieces per wave per slice
  constexpr int NP = G7_NL + NLB;             // pieces per wave per slice
  constexpr int NS = WN == 128 ? 5 : 3, DIST = NS - 1;
  static_assert(NS * SLOT * 2 * (WN == 128 ? 1 : 2) <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * SLOT];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int ar = wr * 128, bc = wc * WN;

  const int local = g7_local(blockIdx.x, pl.grid);
  const int nmine = local < pl.units ? (pl.units - local + pl.grid - 1) / pl.grid : 0;
  if (nmine == 0) return;
  unsigned long long clk_t0 = 0, clk_r0 = 0;
  if constexpr ((ABL & 128) != 0) {
    clk_t0 = __builtin_amdgcn_s_memtime();
    clk_r0 = __builtin_amdgcn_s_memrealtime();
  }

  int va[G7_NL], vb[NLB];
  dma_offsets3<32, AK, G7_NL>(va, p.lda, wid, lane);
  dma_offsets3<32, BK, NLB>(vb, p.ldb, wid, lane);
  const unsigned long long a_step = AK ? 64ull : 32ull * p.lda * 2;
  const unsigned long long b_step = BK ? 64ull : 32ull * p.ldb * 2;

  // ---- DMA issue cursor (unit, slice, ring slot, byte offsets), all wave-uniform.  The
  // descriptor of a slice starts at its k-offset and ends with the operand (host: < 4 GiB), so
  // rows beyond the stored extent land in LDS as zeros.
  int is_u = 0, is_k = 0, is_slot = 0;
  unsigned long long is_aoff = 0, is_boff = 0;
  int is_kt0 = 0;  // first k-slice of the cursor's unit
  const int ntiles = pl.tiles_m * pl.tiles_n;
  auto set_org = [&](int ui) {
    const int uu = local + ui * pl.grid;
    const int sp = uu / ntiles;
    int m0, n0;
    g7_tile(pl, uu - sp * ntiles, m0, n0);
    is_kt0 = sp * pl.nk;
    is_aoff = (AK ? (unsigned long long)m0 * p.lda * 2 : (unsigned long long)m0 * 2) + a_step * is_kt0;
    is_boff = (BK ? (unsigned long long)n0 * p.ldb * 2 : (unsigned long long)n0 * 2) + b_step * is_kt0;
  };
  set_org(0);
  __amdgpu_buffer_rsrc_t rsa, rsb;
  const bf16_t* is_lds = smem;
  auto prep = [&]() {  // descriptors + LDS slot of the slice the cursor points at
    const bool valid = is_u < nmine && is_kt0 + is_k < pl.nk_all;
    const unsigned long long la = a_bytes - is_aoff, lb = b_bytes - is_boff;
    const unsigned na = valid ? ((la >> 32) ? 0xffffffffu : (unsigned)la) : 0u;
    const unsigned nb = valid ? ((lb >> 32) ? 0xffffffffu : (unsigned)lb) : 0u;
    rsa = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.A + is_aoff), 0, na, 0x00020000);
    rsb = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.B + is_boff), 0, nb, 0x00020000);
    is_lds = smem + is_slot * SLOT;
  };
  auto piece = [&](int i) {  // the pieces of one slice: A (G7_NL) then B (NLB)
    if (i < G7_NL) g7_piece(rsa, va[i], is_lds + (wid * G7_NL + i) * 512);
    else g7_piece(rsb, vb[i - G7_NL], is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
  };
  auto piece4 = [&](int i) {  // pieces i .. i+3 of one operand (NL == NLB == 4)
    if (i < G7_NL) g7_piece4(rsa, va[i], va[i + 1] - 1024, va[i + 2] - 2048, va[i + 3] - 3072, is_lds + (wid * G7_NL + i) * 512);
    else g7_piece4(rsb, vb[i - G7_NL], vb[i + 1 - G7_NL] - 1024, vb[i + 2 - G7_NL] - 2048, vb[i + 3 - G7_NL] - 3072,
                   is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
  };
  auto piece2 = [&](int i) {  // pieces i, i+1 (same operand: i even, NL and NLB even)
    if (i < G7_NL) g7_piece2(rsa, va[i], va[i + 1] - 1024, is_lds + (wid * G7_NL + i) * 512);
    else g7_piece2(rsb, vb[i - G7_NL], vb[i + 1 - G7_NL] - 1024, is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
  };
  auto advance = [&]() {
    is_slot = is_slot + 1 == NS ? 0 : is_slot + 1;
    is_aoff += a_step;
    is_boff += b_step;
    if (++is_k == pl.nk) {
      is_k = 0;
      ++is_u;
      if (is_u < nmine) set_org(is_u);
    }
  };

  // prologue: slices 0 .. DIST-1, then the descriptors of slice DIST for body 0
#pragma unroll
  for (int s = 0; s < DIST; ++s) {
    prep();
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if constexpr (SCHED == 4 && WN == 128) {
        if (!(i & 3)) piece4(i);
      } else if constexpr (SCHED >= 3) {
        if (!(i & 1)) piece2(i);
      } else {
        piece(i);
      }
    }
    advance();
  }
  prep();

  floatx4 acc[8][NJ];  // written first by each tile's FIRST body

  // slice 0 landed (DIST-1 slices younger) -> frags(0)
  g7_wait<(DIST - 1) * NP>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 a0[8], b0[NJ], a1[8], b1[NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = frag3<32, AK>(smem, ar + 16 * i, 0, lane);
#pragma unroll
  for (int j = 0; j < NJ; ++j) b0[j] = frag3<32, BK>(smem + G7_TA, bc + 16 * j, 0, lane);
  if constexpr ((ABL & 32) != 0) {  // (ablation: the loop re-uses these fragments)
#pragma unroll
    for (int i = 0; i < 8; ++i) a1[i] = a0[i];
#pragma unroll
    for (int j = 0; j < NJ; ++j) b1[j] = b0[j];
  }
  // slice 1 landed -> its slot may be read in body(0)
  g7_wait<(DIST - 2) * NP>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  int rd_slot = 1;          // slot of slice q+1
  int credit = 0;           // bodies left during which the last epilogue's stores may stay in flight

  // one slice: MFMAs on (ac, bcur), reads of slice q+1 into (an, bn), DMA of slice q+DIST,
  // then slice q+2 landed (younger: slices q+3 .. q+DIST, plus a recent epilogue's stores) +
  // barrier.  nk is even (padded with all-zero slices), so every unit starts on register set 0.
#define G7_MFMA_ROW(i_, ac, bcur, FIRST)                                                            \
  _Pragma("unroll") for (int j = 0; j < NJ; ++j) acc[i_][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(  \
      EPI == 2 ? ac[i_] : bcur[j], EPI == 2 ? bcur[j] : ac[i_],                                    \
      (FIRST) ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i_][j], 0, 0, 0)
  // DMA piece placement inside a body (SCHED): 0 = piece g at the head of group g, 1 = four
  // pieces at the head of groups 0 and 4, 2 = two pieces at the head of every even group
  // (measured on MI355X, bench/gemm_ab.py: 1 and 2 beat 0 by 2-6 %; all eight at the head
  // of the body or one at the tail of each group lost)
  auto piece_sched = [&](int g, bool tail) {
    if ((ABL & 256) && (pl.debug & 2)) return;  // (the old runtime switch, A/B only)
    if (ABL & 2) return;
    if (SCHED == 0 && !tail && g < NP) piece(g);

    if (SCHED == 2 && !tail && !(g & 1) && g < NP) { piece(g); piece(g + 1); }
    if (SCHED == 3 && !tail && !(g & 1) && g < NP) piece2(g);
    if (SCHED == 4 && !tail && !(g & 3) && g < NP) piece4(g);
    if (SCHED == 1 && !tail && !(g & 3) && g < NP) { piece(g); piece(g + 1); piece(g + 2); piece(g + 3); }

  };
  // one slice: MFMAs on (ac, bcur) -- FIRST: a tile's first slice, accumulating onto zero (an
  // inline-constant C operand: no accumulator clearing between tiles) --, reads of slice q+1
  // into (an, bn), DMA of slice q+DIST, then slice q+2 landed (younger: slices q+3 .. q+DIST,
  // plus a recent epilogue's stores) + barrier.  nk is even (padded with all-zero slices), so every unit
  // starts on register set 0.
  // SCHED 6 (v7 only): group i = the 8 MFMAs of row i with one other instruction in each gap:
  // the two fragment reads after MFMAs 0 and 1, and in the even groups the DMA pair's M0 write
  // and its two loads after MFMAs 2, 3 and 4; the next body's cursor (advance / prep) in group
  // 7 after MFMAs 1 and 4.  Every boundary pinned by sched_barrier.
  auto mf = [&](int i, int j, const bf16x8* ac, const bf16x8* bcur, bool first) G7_AI {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bcur[j], ac[i], first ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
                                                        0, 0, 0);
  };
  auto dma5 = [&](int g, int step) G7_AI {  // step 0: M0, 1 / 2: the pair's loads
    if constexpr ((ABL & 2) != 0) return;
    const int i = g;  // pieces i, i+1 (A: 0..3, B: 4..7)
    if (step == 0) {
      if (i < G7_NL) g7_m0(is_lds + (wid * G7_NL + i) * 512);
      else g7_m0(is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
    } else if (step == 1) {
      if (i < G7_NL) g7_ld<0>(rsa, va[i]);
      else g7_ld<0>(rsb, vb[i - G7_NL]);
    } else {
      if (i < G7_NL) g7_ld<1024>(rsa, va[i + 1] - 1024);
      else g7_ld<1024>(rsb, vb[i + 1 - G7_NL] - 1024);
    }
  };
#define G7_SB __builtin_amdgcn_sched_barrier(0)
#define G7_GROUP5(i, ac, bcur, an, bn, FIRST)                                                        \
  do {                                                                                              \
    mf(i, 0, ac, bcur, FIRST); G7_SB;                                                               \
    if (!(ABL & 32)) an[i] = frag3<32, AK>(la_, ar + 16 * i, 0, lane);                              \
    G7_SB; mf(i, 1, ac, bcur, FIRST); G7_SB;                                                        \
    if (!(ABL & 32)) bn[i] = frag3<32, BK>(la_ + G7_TA, bc + 16 * i, 0, lane);                      \
    G7_SB; mf(i, 2, ac, bcur, FIRST); G7_SB;                                                        \
    if (!((i) & 1) && (i) < NP) dma5(i, 0);                                                         \
    if ((i) == 7) advance();                                                                        \
    G7_SB; mf(i, 3, ac, bcur, FIRST); G7_SB;                                                        \
    if (!((i) & 1) && (i) < NP) dma5(i, 1);                                                         \
    G7_SB; mf(i, 4, ac, bcur, FIRST); G7_SB;                                                        \
    if (!((i) & 1) && (i) < NP) dma5(i, 2);                                                         \
    G7_SB; mf(i, 5, ac, bcur, FIRST); G7_SB;                                                        \
    if ((i) == 7) prep();                                                                           \
    G7_SB; mf(i, 6, ac, bcur, FIRST); G7_SB;                                                        \
    mf(i, 7, ac, bcur, FIRST); G7_SB;                                                               \
  } while (0)
#define G7_BODY(ac, bcur, an, bn, FIRST) G7_BODYC(ac, bcur, an, bn, FIRST, false)
#define G7_BODYC(ac, bcur, an, bn, FIRST, CREDIT)                                                   \
  do {                                                                                              \
    const bf16_t* la_ = smem + rd_slot * SLOT;                                                      \
    if constexpr (SCHED == 6 && !A1) {                                                              \
      G7_GROUP5(0, ac, bcur, an, bn, FIRST); G7_GROUP5(1, ac, bcur, an, bn, FIRST);                 \
      G7_GROUP5(2, ac, bcur, an, bn, FIRST); G7_GROUP5(3, ac, bcur, an, bn, FIRST);                 \
      G7_GROUP5(4, ac, bcur, an, bn, FIRST); G7_GROUP5(5, ac, bcur, an, bn, FIRST);                 \
      G7_GROUP5(6, ac, bcur, an, bn, FIRST); G7_GROUP5(7, ac, bcur, an, bn, FIRST);                 \
    } else                                                                                          \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                 \
      piece_sched(i, false);                                                                        \
      if (!A1 && !(ABL & 32)) an[i] = frag3<32, AK>(la_, ar + 16 * i, 0, lane);                     \
      if (i < NJ && !(ABL & 32)) bn[i] = frag3<32, BK>(la_ + G7_TA, bc + 16 * i, 0, lane);          \
      G7_MFMA_ROW(i, ac, bcur, FIRST);                                                              \
      if (A1) { /* after its MFMAs issued: the fragment's registers are reused */                   \
        __builtin_amdgcn_sched_barrier(0);                                                          \
        an[i] = frag3<32, AK>(la_, ar + 16 * i, 0, lane);                                           \
      }                                                                                             \
      piece_sched(i, true);                                                                         \
      if (i == 7) { /* next body's descriptors, in the shadow of this group's MFMAs */           \
        advance();                                                                                  \
        prep();                                                                                     \
      }                                                                                             \
      __builtin_amdgcn_sched_barrier(0);                                                            \
    }                                                                                               \
    rd_slot = rd_slot + 1 == NS ? 0 : rd_slot + 1;                                                  \
    if (ABL & 64) {                                                                                 \
    } else if ((CREDIT || (ABL & 256)) && credit > 0) {                                             \
      --credit;                                                                                     \
      if (pl.store_cnt >= 48) g7_wait<(DIST - 2) * NP + 47>();                                      \
      else g7_wait<(DIST - 2) * NP + 31>();                                                         \
    } else {                                                                                        \
      g7_wait<(DIST - 2) * NP>();                                                                   \
    }                                                                                               \
    if (!(ABL & 16)) __builtin_amdgcn_s_barrier();                                                  \
    asm volatile("" ::: "memory");                                                                  \
  } while (0)

  // A1 (v8): ONE A-fragment set, row i re-read for the next slice right after its MFMAs are
  // issued (the 128 accumulators + a double B set + one A set fit 256 registers: two waves per
  // SIMD); v7 double-buffers both
  constexpr bool A1 = WN == 64;
  for (int u = 0; u < nmine; ++u) {
    if constexpr (A1) {
      G7_BODYC(a0, b0, a0, b1, true, true);
      G7_BODYC(a0, b1, a0, b0, false, true);
      for (int k = 2; k < pl.nk; k += 2) {
        G7_BODY(a0, b0, a0, b1, false);
        G7_BODY(a0, b1, a0, b0, false);
      }
    } else {
      G7_BODYC(a0, b0, a1, b1, true, true);
      G7_BODYC(a1, b1, a0, b0, false, true);
      for (int k = 2; k < pl.nk; k += 2) {
        G7_BODY(a0, b0, a1, b1, false);
        G7_BODY(a1, b1, a0, b0, false);
      }
    }
    const int uu = local + u * pl.grid;
    int m0, n0;
    g7_tile(pl, uu % ntiles, m0, n0);
    if (pl.debug & 1) {
    } else if constexpr (EPI == 2) {
      if constexpr (NJ == 8) g7_epilogue_atomic(p, acc, m0 + ar, n0 + bc, lane);
    } else if constexpr (EPI == 4) {
      GemmArgs q = p;  // the k-range's slab: [M][N] f32 at ws + split * M * N
      q.C = static_cast<float*>(p.ws) + (long long)(uu / ntiles) * p.M * p.N;
      q.ldc = p.N;
      q.out_f32 = 1;
      g7_epilogue<0, NJ>(q, acc, m0 + ar, n0 + bc, lane);
    } else if constexpr (EPI == 0) {
      g7_epilogue<EPI, NJ, WN == 64 && AK>(p, acc, m0 + ar, n0 + bc, lane, pl.debug);
    } else if constexpr (EPI == 9) {
      static_assert(WN == 128, "v7 only");
      // (ONE epilogue copy per v7 kernel: with act-specialised full-tile copies beside the
      // generic one the allocator spilled 67 (EPI 9) / 304 (EPI 8) VGPRs into the main loop --
      // down-projection 369 -> 568 us, act' input gradient 535 -> 749 us, round 5)
      g7_epilogue_res_lds<NJ>(p, acc, m0, n0, wid, lane, smem + ((rd_slot + 3) % NS) * SLOT,
                              smem + ((rd_slot + 4) % NS) * SLOT);
    } else if constexpr (EPI == 8 || EPI == 10) {
      // (its own instantiation: beside g7_epilogue<3> in one kernel the register allocator
      // spilled ~120 registers, alone it spills 2; EPI 10 = the ACT_MUL form, another kernel)
      static_assert(WN == 128, "v7 only");
      g7_epilogue_act_lds<NJ, EPI == 10, EPI == 10 ? G_SP_DEFAULT : -1>(p, acc, m0, n0, wid, lane, smem + ((rd_slot + 3) % NS) * SLOT,
                              smem + ((rd_slot + 4) % NS) * SLOT);
    } else {
      // packed-f32 GELU: v8 with a k-major A, and the v7 forward epilogues (measured: the act'
      // epilogue's GELU' in packed math took the GPT-2 up-projection input gradient from 531 to
      // 725 TF/s -- the epilogue was VALU-bound)
      g7_epilogue<EPI, NJ, (WN == 64 && AK) || (WN == 128 && EPI == 1)>(p, acc, m0 + ar, n0 + bc, lane);
    }
    // the stores were issued after this tile's last wait: the next DIST-2 waits (slices whose
    // DMA is older than the stores) may leave them in flight -- full tiles only (an edge tile
    // skips stores, and the credit must not exceed what was issued)
    credit = (EPI != 2 && pl.store_cnt > 0 && m0 + 256 <= p.M && n0 + BW <= p.N) ? DIST - 2 : 0;
  }
#undef G7_MFMA_ROW
#undef G7_BODY
#undef G7_BODYC
#undef G7_GROUP5
#undef G7_SB
  g7_wait<0>();  // empty-descriptor DMA of the slices past the end: drained before exit
  if constexpr ((ABL & 128) != 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 2048) {
      g7_clk[2 * blockIdx.x] = t1 - clk_t0;
      g7_clk[2 * blockIdx.x + 1] = r1 - clk_r0;
    }
  }
}

// colsum[n] += sum over the R rows of ws [R][N] (g7_epilogue_act_lds's per-tile partial column
// sums): 4 columns per thread, 16 rows per workgroup row (grid.y), one atomic per column per 16
// rows
static __global__ __launch_bounds__(256) void g7_colsum_reduce(float* colsum, const float* ws, int R, int N) {
  const int c4 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c4 >= N) return;
  const int r0 = blockIdx.y * 16, r1 = min(R, r0 + 16);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 16
  for (int r = r0; r < r1; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(ws + (long long)r * N + c4);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  atomicAdd(colsum + c4, s.x);
  atomicAdd(colsum + c4 + 1, s.y);
  atomicAdd(colsum + c4 + 2, s.z);
  atomicAdd(colsum + c4 + 3, s.w);
}

// C (=, or += when accumulating) the sum of the s workspace slabs [s][M][N]; 4 columns per
// thread (N % 8 == 0, ldc % 8 == 0: 16-B rows)
static __global__ __launch_bounds__(256) void g7_splitk_reduce(float* C, long long ldc, const float* ws, int M, int N,
                                                       int s, int accumulate, int nt = 0) {
  const long long nq = (long long)M * (N >> 2);
  const long long slab = (long long)M * N;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nq; i += (long long)gridDim.x * 256) {
    const long long m = i / (N >> 2), n = (i - m * (N >> 2)) << 2;
    const float* w = ws + m * N + n;
    float4 v = *reinterpret_cast<const float4*>(w);
    // four slabs' loads in flight before their adds (the one-at-a-time loop waited for each:
    // 2.9 TB/s), the adds in the same order as before (bitwise the same sums)
    int k = 1;
    for (; k + 3 < s; k += 4) {
      const float4 u0 = *reinterpret_cast<const float4*>(w + k * slab);
      const float4 u1 = *reinterpret_cast<const float4*>(w + (k + 1) * slab);
      const float4 u2 = *reinterpret_cast<const float4*>(w + (k + 2) * slab);
      const float4 u3 = *reinterpret_cast<const float4*>(w + (k + 3) * slab);
      v.x += u0.x; v.y += u0.y; v.z += u0.z; v.w += u0.w;
      v.x += u1.x; v.y += u1.y; v.z += u1.z; v.w += u1.w;
      v.x += u2.x; v.y += u2.y; v.z += u2.z; v.w += u2.w;
      v.x += u3.x; v.y += u3.y; v.z += u3.z; v.w += u3.w;
    }
    for (; k < s; ++k) {
      const float4 u = *reinterpret_cast<const float4*>(w + k * slab);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    float4* c = reinterpret_cast<float4*>(C + m * ldc + n);
    if (accumulate) {
      const float4 o = *c;
      v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    st16(c, v, nt);
  }
}

// ------------------------------------------------------------------ v7d: deferred epilogues
// The fused GELU epilogues of the FFN products are VALU-heavy (~10 issue slots per element
// forward, ~18 for GELU' in the input gradient) and a one-wave-per-SIMD kernel runs them
// serially at the tile end: on the K = 768 GPT-2 products that is 50-60 % of the MFMA time
// (profiles/r3_gemm/st8_fused_0.log: up 0.50 ms, act' dgrad 0.53-0.56 against 0.28-0.32 for
// the plain products of the same shape).  Here the tile end does only the cheap part -- the
// accumulators (+ bias) rounded to bf16 and stored (the pre-activation into aux_out, EPI 5;
// the raw input gradient into C, EPI 6) -- and the element-wise rest is DEFERRED into the
// next tile's main loop: the 32 16-B chunks a lane stored come back by LDS-DMA (the lane reads
// exactly the addresses it wrote: same-wave program order), a few per k-slice, and their
// GELU / GELU' arithmetic sits in the MFMA groups, where a wave has ~8 free issue cycles per
// v_mfma_f32_16x16x32_bf16.  The results are stored a chunk or two per slice, so the output
// traffic is spread over the tile instead of leaving in one chip-wide burst.
// Rounding is the reference's (torch autocast): the GELU input is the bf16 pre-activation and
// the GELU' product starts from the bf16 input gradient, as aten computes them.
//   EPI 5: C = gelu(bf16(acc + bias)) bf16, aux_out = bf16(acc + bias).
//   EPI 6: C = bf16(dy * gelu'(aux_in)), dy = bf16(acc); colsum[n] += sum_m of the same.
//   EPI 7: C = residual + gelu(bf16(acc + bias)) f32, aux_out = bf16(acc + bias) (the FFN
//          down projection with the reference's second activation; K >= 1088, one chunk per
//          slice: a chunk carries 48 B of operands).
// Ring: 4 slots (DIST 3) to free LDS for the unit regions ([2 parities][4 waves][2 units] x 1
// or 2 KiB) and, EPI 5, the tile's 256 bias values (one DMA piece by wave 0 in body 1).
// Counting: a body issues [unit DMAs for body c+2 at group 2] [the 8 ring pieces, last at
// group 6] [its unit stores + column-sum atomic at the end]; at the end of body c the ring
// needs slice c+2 (body c-1's pieces), and everything a body issues before its last piece is
// older than it -- so the wait is vmcnt(ops issued after body c-1's last piece), computed per
// body (a runtime count -> one of the immediates, g7_wait_bs).  Tiles that are partial or last
// in a workgroup's list take the ordinary fused epilogue and drain (vmcnt(0)).
template <int LO, int HI>
__device__ __forceinline__ void g7_wait_bs(int n) {
  if constexpr (LO == HI) {
    g7_wait<LO>();
  } else {
    constexpr int MID = (LO + HI + 1) / 2;
    if (n >= MID) g7_wait_bs<MID, HI>(n);
    else g7_wait_bs<LO, MID - 1>(n);
  }
}

// x * sigmoid(2u) (gelu_tanh) with log2(e) folded into the exponent's coefficients
constexpr float G7_GK0 = 0.7978845608028654f, G7_GK1 = 0.044715f, G7_L2E = 1.4426950408889634f;
__device__ __forceinline__ float g7_gelu(float x) {
  const float e = __builtin_amdgcn_exp2f(x * fmaf(x * x, -2.f * G7_GK0 * G7_GK1 * G7_L2E, -2.f * G7_GK0 * G7_L2E));
  return x * __builtin_amdgcn_rcpf(1.f + e);
}
// d/dx = s + x s (1 - s) 2 k0 (1 + 3 k1 x^2), s = sigmoid(2u)
__device__ __forceinline__ float g7_gelu_grad(float x) {
  const float x2 = x * x;
  const float s = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * fmaf(x2, -2.f * G7_GK0 * G7_GK1 * G7_L2E, -2.f * G7_GK0 * G7_L2E)));
  const float t = x * fmaf(x2, 6.f * G7_GK0 * G7_GK1, 2.f * G7_GK0);
  return fmaf(t, fmaf(-s, s, s), s);
}

__device__ __forceinline__ unsigned g7_comp(const uint4& v, int c) {
  return c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w));
}
__device__ __forceinline__ void g7_setcomp(uint4& v, int c, unsigned w) {
  if (c == 0) v.x = w;
  else if (c == 1) v.y = w;
  else if (c == 2) v.z = w;
  else v.w = w;
}
__device__ __forceinline__ float g7_bf(unsigned w, int hi) {
  return hi ? __uint_as_float(w & 0xffff0000u) : __uint_as_float(w << 16);
}

// The tile end of a deferred tile: bf16(acc * alpha [+ bias]) in the row-coalesced layout of
// the MODE 0 epilogue (chunk (i, jb, half) of a lane: row mw + 16 i + rr + 8 half, columns
// nw + 64 jb + coff + 32 hi8 .. +7), 32 unconditional 16-B stores (full tiles only).
// CHECK (partial tiles): rows / columns past M / N skipped, the bias read from global memory
// (bl = the bias vector) instead of the tile's LDS copy.
template <bool BIAS, bool CHECK = false>
__device__ __forceinline__ void g7_split_store(bf16_t* dst, long long ld, floatx4 (&acc)[8][8], int mw, int nw,
                                               int lane, float alpha, const float* bl, bool nt, int M = 0, int N = 0) {
  const int g = lane >> 4, rl = lane & 15;
  const int coff = 16 * (g & 1) + 8 * (g >> 1);
  const bool lo = rl < 8;
  const int rr = rl & 7, hi8 = rl >> 3;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; j += 4) {
      uint4 c0, c1;
      {
        floatx4 a0 = acc[i][j], a1 = acc[i][j + 1], a2 = acc[i][j + 2], a3 = acc[i][j + 3];
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0, b2 = b0, b3 = b0;
        if constexpr (BIAS && !CHECK) {
          b0 = *reinterpret_cast<const float4*>(bl + 16 * j + 4 * g);
          b1 = *reinterpret_cast<const float4*>(bl + 16 * (j + 1) + 4 * g);
          b2 = *reinterpret_cast<const float4*>(bl + 16 * (j + 2) + 4 * g);
          b3 = *reinterpret_cast<const float4*>(bl + 16 * (j + 3) + 4 * g);
        } else if constexpr (BIAS) {
          const int n = nw + 16 * j + 4 * g;
          if (n < N) b0 = *reinterpret_cast<const float4*>(bl + n);
          if (n + 16 < N) b1 = *reinterpret_cast<const float4*>(bl + n + 16);
          if (n + 32 < N) b2 = *reinterpret_cast<const float4*>(bl + n + 32);
          if (n + 48 < N) b3 = *reinterpret_cast<const float4*>(bl + n + 48);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pack2bf(fmaf(a0[0], alpha, b0.x), fmaf(a0[1], alpha, b0.y)),
                                                         pack2bf(fmaf(a1[0], alpha, b1.x), fmaf(a1[1], alpha, b1.y)), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pack2bf(fmaf(a0[2], alpha, b0.z), fmaf(a0[3], alpha, b0.w)),
                                                         pack2bf(fmaf(a1[2], alpha, b1.z), fmaf(a1[3], alpha, b1.w)), false, false);
        const auto t0 = __builtin_amdgcn_permlane16_swap(pack2bf(fmaf(a2[0], alpha, b2.x), fmaf(a2[1], alpha, b2.y)),
                                                         pack2bf(fmaf(a3[0], alpha, b3.x), fmaf(a3[1], alpha, b3.y)), false, false);
        const auto t1 = __builtin_amdgcn_permlane16_swap(pack2bf(fmaf(a2[2], alpha, b2.z), fmaf(a2[3], alpha, b2.w)),
                                                         pack2bf(fmaf(a3[2], alpha, b3.z), fmaf(a3[3], alpha, b3.w)), false, false);
        c0 = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        c1 = make_uint4(t0[0], t1[0], t0[1], t1[1]);
      }
      const uint4 snd = make_uint4(lo ? c1.x : c0.x, lo ? c1.y : c0.y, lo ? c1.z : c0.z, lo ? c1.w : c0.w);
      const uint4 rcv = make_uint4(g7_ror8(snd.x), g7_ror8(snd.y), g7_ror8(snd.z), g7_ror8(snd.w));
      const uint4 dA = make_uint4(lo ? c0.x : rcv.x, lo ? c0.y : rcv.y, lo ? c0.z : rcv.z, lo ? c0.w : rcv.w);
      const uint4 dB = make_uint4(lo ? rcv.x : c1.x, lo ? rcv.y : c1.y, lo ? rcv.z : c1.z, lo ? rcv.w : c1.w);
      const int m = mw + 16 * i + rr, n = nw + 16 * j + coff + 32 * hi8;
      bf16_t* C = dst + (long long)m * ld + n;
      if (!CHECK || (n < N && m < M)) st16(C, dA, nt);
      if (!CHECK || (n < N && m + 8 < M)) st16(C + 8 * ld, dB, nt);
    }
  }
}

// The element-wise rest of a tile whose chunks were just stored by g7_split_store, done at
// once (partial tiles and each workgroup's last tile; the caller drained vmcnt): every lane
// reads back its own chunks, one at a time (a rolled loop: little register pressure beside
// the live accumulators of nothing -- the next tile has not started).
template <int EPI>
__device__ __forceinline__ void g7d_finish(const GemmArgs& p, int mw, int nw, int lane) {
  const int g = lane >> 4, rl = lane & 15, rr = rl & 7, hi8 = rl >> 3;
  const int coff = 16 * (g & 1) + 8 * (g >> 1);
#pragma unroll 1
  for (int jb = 0; jb < 2; ++jb) {
    const int n = nw + 64 * jb + coff + 32 * hi8;
    float cs[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) cs[v] = 0.f;
#pragma unroll 1
    for (int t = 0; t < 16; ++t) {
      const int m = mw + 16 * (t >> 1) + rr + 8 * (t & 1);
      if (m < p.M && n < p.N) {
        bf16_t* C = static_cast<bf16_t*>(p.C) + (long long)m * p.ldc + n;
        uint4 o;
        if constexpr (EPI == 7) {
          const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(p.aux_out) + (long long)m * p.ld_aux_out + n);
          const float* R = p.residual + (long long)m * p.ldr + n;
          const float4 r0 = *reinterpret_cast<const float4*>(R), r1 = *reinterpret_cast<const float4*>(R + 4);
          float* Cf = static_cast<float*>(p.C) + (long long)m * p.ldc + n;
          st16(Cf, make_float4(r0.x + g7_gelu(g7_bf(x.x, 0)), r0.y + g7_gelu(g7_bf(x.x, 1)),
                               r0.z + g7_gelu(g7_bf(x.y, 0)), r0.w + g7_gelu(g7_bf(x.y, 1))), p.nt_store & 2);
          st16(Cf + 4, make_float4(r1.x + g7_gelu(g7_bf(x.z, 0)), r1.y + g7_gelu(g7_bf(x.z, 1)),
                                   r1.z + g7_gelu(g7_bf(x.w, 0)), r1.w + g7_gelu(g7_bf(x.w, 1))), p.nt_store & 2);
          continue;
        } else if constexpr (EPI == 5) {
          const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(p.aux_out) + (long long)m * p.ld_aux_out + n);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const unsigned w = g7_comp(x, q);
            g7_setcomp(o, q, pack2bf(g7_gelu(g7_bf(w, 0)), g7_gelu(g7_bf(w, 1))));
          }
        } else {
          const uint4 dy = *reinterpret_cast<const uint4*>(C);
          const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const bf16_t*>(p.aux_in) + (long long)m * p.ld_aux_in + n);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y0 = g7_bf(g7_comp(dy, q), 0) * g7_gelu_grad(g7_bf(g7_comp(x, q), 0));
            const float y1 = g7_bf(g7_comp(dy, q), 1) * g7_gelu_grad(g7_bf(g7_comp(x, q), 1));
            cs[2 * q] += y0;
            cs[2 * q + 1] += y1;
            g7_setcomp(o, q, pack2bf(y0, y1));
          }
        }
        st16(C, o, p.nt_store & 1);
      }
    }
    if (EPI == 6 && p.colsum) {
      float pick = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        float s_ = cs[v];
        s_ += __shfl_xor(s_, 1, 64);
        s_ += __shfl_xor(s_, 2, 64);
        s_ += __shfl_xor(s_, 4, 64);
        pick = rr == v ? s_ : pick;
      }
      if (n + rr < p.N) atomicAdd(p.colsum + n + rr, pick);
    }
  }
}

template <int EPI, int SCHED, bool AK, bool BK>
__global__ __launch_bounds__(256, 1) void gemm7d_kernel(GemmArgs p, unsigned long long a_bytes,
                                                        unsigned long long b_bytes, G7Plan pl) {
  constexpr int NJ = 8, BW = 256, TB = BW * G7_KB, SLOT = G7_TA + TB;
  constexpr int NLB = TB / 512 / 4, NP = G7_NL + NLB;
  constexpr int NS = 4, DIST = NS - 1;
  constexpr int DPU = EPI == 5 ? 1 : (EPI == 6 ? 2 : 3);  // 1-KiB unit DMAs per unit
  constexpr int MAXU = EPI == 7 ? 1 : 2;                   // units per body at most
  constexpr bool FWD = EPI != 6;                           // bias + GELU of the pre-activation
  constexpr int UOFF = NS * SLOT;  // unit regions [parity][wave][unit][DPU] x 512 bf16
  constexpr int BOFF = UOFF + 2 * 4 * MAXU * DPU * 512;
  constexpr int LDS_E = BOFF + (FWD ? 512 : 0);
  static_assert(LDS_E * 2 <= 160 * 1024, "LDS");
  static_assert(EPI >= 5 && EPI <= 7, "v7d epilogues");
  __shared__ __attribute__((aligned(16))) bf16_t smem[LDS_E];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int ar = wr * 128, bc = wc * 128;
  const int rl = lane & 15, rr = rl & 7, hi8 = rl >> 3, lg = lane >> 4;
  const int coff = 16 * (lg & 1) + 8 * (lg >> 1);

  const int local = g7_local(blockIdx.x, pl.grid);
  const int nmine = local < pl.units ? (pl.units - local + pl.grid - 1) / pl.grid : 0;
  if (nmine == 0) return;

  int va[G7_NL], vb[NLB];
  dma_offsets3<32, AK, G7_NL>(va, p.lda, wid, lane);
  dma_offsets3<32, BK, NLB>(vb, p.ldb, wid, lane);
  const unsigned long long a_step = AK ? 64ull : 32ull * p.lda * 2;
  const unsigned long long b_step = BK ? 64ull : 32ull * p.ldb * 2;

  int is_u = 0, is_k = 0, is_slot = 0;
  unsigned long long is_aoff = 0, is_boff = 0;
  const int ntiles = pl.tiles_m * pl.tiles_n;
  auto set_org = [&](int ui) {
    const int uu = local + ui * pl.grid;
    int m0, n0;
    g7_tile(pl, uu % ntiles, m0, n0);
    is_aoff = AK ? (unsigned long long)m0 * p.lda * 2 : (unsigned long long)m0 * 2;
    is_boff = BK ? (unsigned long long)n0 * p.ldb * 2 : (unsigned long long)n0 * 2;
  };
  set_org(0);
  __amdgpu_buffer_rsrc_t rsa, rsb;
  const bf16_t* is_lds = smem;
  auto prep = [&]() {
    const bool valid = is_u < nmine && is_k < pl.nk_all;
    const unsigned long long la = a_bytes - is_aoff, lb = b_bytes - is_boff;
    const unsigned na = valid ? ((la >> 32) ? 0xffffffffu : (unsigned)la) : 0u;
    const unsigned nb = valid ? ((lb >> 32) ? 0xffffffffu : (unsigned)lb) : 0u;
    rsa = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.A + is_aoff), 0, na, 0x00020000);
    rsb = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.B + is_boff), 0, nb, 0x00020000);
    is_lds = smem + is_slot * SLOT;
  };
  auto piece = [&](int i) {
    if (i < G7_NL) g7_piece(rsa, va[i], is_lds + (wid * G7_NL + i) * 512);
    else g7_piece(rsb, vb[i - G7_NL], is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
  };
  auto piece2 = [&](int i) {
    if (i < G7_NL) g7_piece2(rsa, va[i], va[i + 1] - 1024, is_lds + (wid * G7_NL + i) * 512);
    else g7_piece2(rsb, vb[i - G7_NL], vb[i + 1 - G7_NL] - 1024, is_lds + G7_TA + (wid * NLB + i - G7_NL) * 512);
  };
  auto advance = [&]() {
    is_slot = is_slot + 1 == NS ? 0 : is_slot + 1;
    is_aoff += a_step;
    is_boff += b_step;
    if (++is_k == pl.nk) {
      is_k = 0;
      ++is_u;
      if (is_u < nmine) set_org(is_u);
    }
  };
  auto piece_sched = [&](int g) {  // two pieces at the head of every even group
    if (!(g & 1) && g < NP) {
      if constexpr (SCHED == 3) piece2(g);
      else { piece(g); piece(g + 1); }
    }
  };

#pragma unroll
  for (int s = 0; s < DIST; ++s) {
    prep();
#pragma unroll
    for (int i = 0; i < NP; i += 2) piece_sched(i);
    advance();
  }
  prep();

  floatx4 acc[8][NJ];
  g7_wait<(DIST - 1) * NP>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 a0[8], b0[NJ], a1[8], b1[NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = frag3<32, AK>(smem, ar + 16 * i, 0, lane);
#pragma unroll
  for (int j = 0; j < NJ; ++j) b0[j] = frag3<32, BK>(smem + G7_TA, bc + 16 * j, 0, lane);
  g7_wait<(DIST - 2) * NP>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int rd_slot = 1;

  // ---- deferred-unit state (scalars unless noted).  Schedule of a tile's consuming bodies
  // 2 .. nk-1 (B of them): nA bodies take two units, then nB one each (2 nA + nB = 32), the
  // rest none -- three sequential loops of one body form each (a per-body choice between
  // forms makes the register allocator spill the accumulators).
  const int Bc = pl.nk - 2;
  const int nA = Bc >= 32 ? 0 : 32 - Bc, nB = Bc >= 32 ? 32 : 2 * Bc - 32;
  int pend = 0, pm0 = 0, pn0 = 0;  // the previous tile left its units; its origin
  int post = 0;                    // vm ops issued after the previous body's last ring piece
  auto sched_at = [&](int cc, int& u0) G7_AI {  // units consumed in body cc (of a pending tile)
    const int q = cc - 2;
    if (q < 0) return 0;
    if (q < nA) { u0 = 2 * q; return 2; }
    if (q < nA + nB) { u0 = 2 * nA + (q - nA); return 1; }
    return 0;
  };
  const long long ld0 = FWD ? p.ld_aux_out : p.ldc;  // unit source 0: pre-activation / dy
  const long long ld1 = p.ld_aux_in;                      // EPI 6 unit source 1: act' operand
  const int lb0 = (int)(((long long)(ar + rr) * ld0 + bc + coff + 32 * hi8) * 2);
  const int lb1 = EPI == 6 ? (int)(((long long)(ar + rr) * ld1 + bc + coff + 32 * hi8) * 2) : 0;
  const int lbr = EPI == 7 ? (int)(((long long)(ar + rr) * p.ldr + bc + coff + 32 * hi8) * 4) : 0;
  __amdgpu_buffer_rsrc_t rsu0 = rsa, rsu1 = rsa;
  uint4 ud[2], ua[2], uo[2];
  float4 ur0[2], ur1[2], of0[2], of1[2];  // EPI 7: residual in, f32 out
  float yev[2], cs[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) cs[v] = 0.f;
  const float alpha = g7_alpha(p);
  const float* bl = reinterpret_cast<const float*>(smem + BOFF);
  auto ureg = [&](int r, int k, int q) G7_AI { return smem + UOFF + ((r * 4 + wid) * MAXU * DPU + k * DPU + q) * 512; };
  auto ugeo = [&](int u, long long ld) G7_AI {  // uniform byte offset of unit u in the tile
    const int i = (u >> 1) & 7, half = u & 1, jb = u >> 4;
    return (int)(((long long)(16 * i + 8 * half) * ld + 64 * jb) * 2);
  };
  auto udma = [&](int r, int n, int u0) G7_AI {  // units u0 .. u0+n-1 -> region r
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this region's last reads retired
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k < n) {
        g7_piece(rsu0, lb0 + ugeo(u0 + k, ld0), ureg(r, k, 0));
        if constexpr (EPI == 6) g7_piece(rsu1, lb1 + ugeo(u0 + k, ld1), ureg(r, k, 1));
        if constexpr (EPI == 7) {  // the f32 residual: two 16-B halves of the lane's 8 columns
          const int o = lbr + 2 * ugeo(u0 + k, p.ldr);
          g7_piece(rsu1, o, ureg(r, k, 1));
          g7_piece(rsu1, o + 16, ureg(r, k, 2));
        }
      }
    }
  };
  auto bias_dma = [&](int n0) G7_AI {
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bias + n0), 0, 1024u, 0x00020000);
    g7_piece(rb, lane * 16, smem + BOFF);
  };
  // value v of this body's unit k (in a compile-time group: v is a constant after unrolling)
  auto dvalue = [&](int k, int v) G7_AI {
    const unsigned w = g7_comp(ud[k], v >> 1);
    float y;
    if constexpr (EPI == 7) {
      y = g7_gelu(g7_bf(w, v & 1));
      const float4& rq = v < 4 ? ur0[k] : ur1[k];
      float4& oq = v < 4 ? of0[k] : of1[k];
      const int e = v & 3;
      const float r = e == 0 ? rq.x : (e == 1 ? rq.y : (e == 2 ? rq.z : rq.w));
      if (e == 0) oq.x = r + y;
      else if (e == 1) oq.y = r + y;
      else if (e == 2) oq.z = r + y;
      else oq.w = r + y;
      return;
    } else if constexpr (EPI == 5) {
      y = g7_gelu(g7_bf(w, v & 1));
    } else {
      y = g7_bf(w, v & 1) * g7_gelu_grad(g7_bf(g7_comp(ua[k], v >> 1), v & 1));
      cs[v] += y;
    }
    if (!(v & 1)) yev[k] = y;
    else g7_setcomp(uo[k], v >> 1, pack2bf(yev[k], y));
  };

#define G7_MFMA_ROW(i_, ac, bcur, FIRST)                                                            \
  _Pragma("unroll") for (int j = 0; j < NJ; ++j) acc[i_][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16( \
      bcur[j], ac[i_], (FIRST) ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i_][j], 0, 0, 0)
  // one slice (body c of the tile) with NU deferred units consumed
#define G7D_BODY(ac, bcur, an, bn, FIRST, NU)                                                       \
  do {                                                                                              \
    const int rg = c & 1;                                                                           \
    int ud0 = 0, uc0 = 0;                                                                           \
    const int nd = pend ? sched_at(c + 2, ud0) : 0; /* units DMA'd now for body c+2 */             \
    if constexpr (NU > 0) sched_at(c, uc0);                                                         \
    if constexpr (NU > 0) {                                                                         \
      _Pragma("unroll") for (int k = 0; k < NU; ++k) {                                              \
        ud[k] = *reinterpret_cast<const uint4*>(ureg(rg, k, 0) + lane * 8);                         \
        if constexpr (EPI == 6) ua[k] = *reinterpret_cast<const uint4*>(ureg(rg, k, 1) + lane * 8); \
        if constexpr (EPI == 7) {                                                                   \
          ur0[k] = *reinterpret_cast<const float4*>(ureg(rg, k, 1) + lane * 8);                     \
          ur1[k] = *reinterpret_cast<const float4*>(ureg(rg, k, 2) + lane * 8);                     \
        }                                                                                           \
      }                                                                                             \
    }                                                                                               \
    const bf16_t* la_ = smem + rd_slot * SLOT;                                                      \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) {                                                 \
      piece_sched(i);                                                                               \
      if (i == 2 && nd > 0) udma(rg, nd, ud0);                                                      \
      if (i == 4 && c == 1 && bdma) bias_dma(n0);                                                   \
      an[i] = frag3<32, AK>(la_, ar + 16 * i, 0, lane);                                             \
      bn[i] = frag3<32, BK>(la_ + G7_TA, bc + 16 * i, 0, lane);                                     \
      G7_MFMA_ROW(i, ac, bcur, FIRST);                                                              \
      _Pragma("unroll") for (int k = 0; k < NU; ++k) dvalue(k, i);                                  \
      if (i == 7) {                                                                                 \
        advance();                                                                                  \
        prep();                                                                                     \
      }                                                                                             \
      __builtin_amdgcn_sched_barrier(0);                                                            \
    }                                                                                               \
    rd_slot = rd_slot + 1 == NS ? 0 : rd_slot + 1;                                                  \
    int tail = 0;                                                                                   \
    if constexpr (NU > 0) {                                                                         \
      _Pragma("unroll") for (int k = 0; k < NU; ++k) {                                              \
        const int u_ = uc0 + k, i_ = (u_ >> 1) & 7, h_ = u_ & 1, jb_ = u_ >> 4;                     \
        const long long e_ = (long long)(pm0 + ar + 16 * i_ + rr + 8 * h_) * p.ldc + pn0 + bc + 64 * jb_ + \
                             coff + 32 * hi8;                                                       \
        if constexpr (EPI == 7) {                                                                   \
          st16(static_cast<float*>(p.C) + e_, of0[k], p.nt_store & 2);                               \
          st16(static_cast<float*>(p.C) + e_ + 4, of1[k], p.nt_store & 2);                           \
        } else {                                                                                    \
          st16(static_cast<bf16_t*>(p.C) + e_, uo[k], p.nt_store & 1);                               \
        }                                                                                           \
      }                                                                                             \
      tail = EPI == 7 ? 2 * NU : NU;                                                                \
      if constexpr (EPI == 6) {                                                                     \
        if (p.colsum && ((uc0 + NU) & 15) == 0) { /* a half (one column set) done */             \
          float pick = 0.f;                                                                         \
          _Pragma("unroll") for (int v = 0; v < 8; ++v) {                                           \
            float s_ = cs[v];                                                                       \
            s_ += __shfl_xor(s_, 1, 64);                                                            \
            s_ += __shfl_xor(s_, 2, 64);                                                            \
            s_ += __shfl_xor(s_, 4, 64);                                                            \
            pick = rr == v ? s_ : pick;                                                             \
            cs[v] = 0.f;                                                                            \
          }                                                                                         \
          atomicAdd(p.colsum + pn0 + bc + 64 * ((uc0 + NU - 1) >> 4) + coff + 32 * hi8 + rr, pick); \
          tail += 1;                                                                                \
        }                                                                                           \
      }                                                                                             \
    }                                                                                               \
    g7_wait_bs<0, 63>(min(63, post + NP + nd * DPU + ((c == 1 && bdma) ? 1 : 0) + tail));           \
    post = tail;                                                                                    \
    __builtin_amdgcn_s_barrier();                                                                   \
    asm volatile("" ::: "memory");                                                                  \
    ++c;                                                                                            \
  } while (0)

  for (int u = 0; u < nmine; ++u) {
    const int uu = local + u * pl.grid;
    int m0, n0;
    g7_tile(pl, uu % ntiles, m0, n0);
    const bool defer_me = m0 + 256 <= p.M && n0 + 256 <= p.N && u + 1 < nmine;
    const bool bdma = FWD && defer_me && p.bias && wid == 0;
    // this tile consumes the previous tile's units in its bodies 2 .. nk-1
    if (pend) {
      const long long ob0 = ((long long)pm0 * ld0 + pn0) * 2;
      const void* src0 = FWD ? p.aux_out : p.C;
      rsu0 = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)src0 + ob0), 0, 0xffffffffu, 0x00020000);
      if constexpr (EPI == 6) {
        const long long ob1 = ((long long)pm0 * ld1 + pn0) * 2;
        rsu1 = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.aux_in + ob1), 0, 0xffffffffu, 0x00020000);
      }
      if constexpr (EPI == 7) {
        const long long obr = ((long long)pm0 * p.ldr + pn0) * 4;
        rsu1 = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.residual + obr), 0, 0xffffffffu, 0x00020000);
      }
    }
    int c = 0;
    G7D_BODY(a0, b0, a1, b1, true, 0);
    G7D_BODY(a1, b1, a0, b0, false, 0);
    const int eA = pend ? 2 + nA : 2, eB = pend ? 2 + nA + nB : 2;
    if constexpr (MAXU == 2) {  // (EPI 7: nA == 0, host nk >= 34)
      for (; c < eA; ) {
        G7D_BODY(a0, b0, a1, b1, false, 2);
        G7D_BODY(a1, b1, a0, b0, false, 2);
      }
    }
    for (; c < eB; ) {
      G7D_BODY(a0, b0, a1, b1, false, 1);
      G7D_BODY(a1, b1, a0, b0, false, 1);
    }
    for (; c < pl.nk; ) {
      G7D_BODY(a0, b0, a1, b1, false, 0);
      G7D_BODY(a1, b1, a0, b0, false, 0);
    }
    if (defer_me) {
      if constexpr (FWD) {
        if (p.bias) g7_split_store<true>(static_cast<bf16_t*>(p.aux_out), p.ld_aux_out, acc, m0 + ar, n0 + bc, lane, alpha, bl + bc, p.nt_store & 1);
        else g7_split_store<false>(static_cast<bf16_t*>(p.aux_out), p.ld_aux_out, acc, m0 + ar, n0 + bc, lane, alpha, bl, p.nt_store & 1);
      } else {
        g7_split_store<false>(static_cast<bf16_t*>(p.C), p.ldc, acc, m0 + ar, n0 + bc, lane, alpha, bl, p.nt_store & 1);
      }
      post += 32;
      pend = 1;
      pm0 = m0;
      pn0 = n0;
    } else {
      // partial or last tile: the same two halves back to back
      if constexpr (FWD) {
        if (p.bias) g7_split_store<true, true>(static_cast<bf16_t*>(p.aux_out), p.ld_aux_out, acc, m0 + ar, n0 + bc, lane, alpha, p.bias, p.nt_store & 1, p.M, p.N);
        else g7_split_store<false, true>(static_cast<bf16_t*>(p.aux_out), p.ld_aux_out, acc, m0 + ar, n0 + bc, lane, alpha, p.bias, p.nt_store & 1, p.M, p.N);
      } else {
        g7_split_store<false, true>(static_cast<bf16_t*>(p.C), p.ldc, acc, m0 + ar, n0 + bc, lane, alpha, bl, p.nt_store & 1, p.M, p.N);
      }
      g7_wait<0>();
      g7d_finish<EPI>(p, m0 + ar, n0 + bc, lane);
      g7_wait<0>();
      post = 0;
      pend = 0;
    }
  }
#undef G7_MFMA_ROW
#undef G7D_BODY
  g7_wait<0>();
}

}  // namespace dpc
