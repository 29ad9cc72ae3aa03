// LayerNorm forward / backward (eps as nn.LayerNorm, default 1e-5) for gfx950.
//
// Reference: models/gpt.py:119,122,217 (nn.LayerNorm on the fp32 residual stream under
// autocast).  Forward reads the f32 residual row once (16 B per lane), keeps it in
// registers, and writes the bf16 normalised row that feeds the next MFMA GEMM plus the
// (mean, rstd) pair.  Backward recomputes x_hat from the f32 row, writes
// dx_total = dres + LN'(dy) IN PLACE into the residual-gradient buffer (the residual add
// of gpt.py:129/133 fused away), and reduces dgamma / dbeta per workgroup in registers
// before ONE f32 atomic per column per workgroup.
//
// One wave per row, NV float4 per lane (D <= 256 * NV), 4 rows (waves) per workgroup.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace dpc {

struct LNArgs {
  const float* x;      // [T][ldx] f32
  const float* gamma;  // [D]
  const float* beta;   // [D]
  void* y;             // fwd: [T][ldy] bf16 (or f32 if y_f32)
  float* mean;         // [T]
  float* rstd;         // [T]
  const float* dy;     // bwd: [T][lddy] f32
  float* dx;           // bwd: [T][lddx] f32, accumulated (dx += LN'(dy))
  float* dgamma;       // bwd: [D] f32 accumulated
  float* dbeta;        // bwd: [D] f32 accumulated
  long long ldx, ldy, lddy, lddx;
  int T, D;
  float eps;
  int y_f32;
  // bwd, optional fused consumer of the new dx (the bias / dropout backward of the
  // projection that produced the LayerNorm's input):  g = dx * keep  ->  gout (bf16),
  // gsum += column sums of g.  keep = dropout factor of element (row, col) of a [T, D]
  // site (misc.hip:drop_factor), 1 when drop_scale == 0.
  void* gout;
  float* gsum;
  long long ld_gout;
  unsigned drop_key, drop_thresh;
  float drop_scale;
  int dy_bf16;  // bwd: dy is bf16 (the input gradient of the next Linear, as autocast makes it)
  // fwd, optional fused producer (the residual add of the projection feeding this LayerNorm):
  // the normalised row is  xs = x + keep * (add_y + add_bias)  (add_y bf16, the plain GEMM's
  // output; keep as in the backward's drop_factor), and xs is written to x_out (f32).
  const void* add_y;
  const float* add_bias;
  float* x_out;
  long long ld_add, ld_xout;
  const unsigned* drop_seed;  // device seed of the forward (drop_key_of); null: drop_key
  unsigned drop_site;
  // bwd, the fused consumer with an activation in front of the dropout (the FFN down projection
  // of the PREVIOUS layer: x3 = x2 + drop(act(z2)), its bias / act / dropout backward fused into
  // the LayerNorm that consumes x3): g = dx * keep * act'(gz)  (gz bf16 [T][ld_gz], act per Act)
  const void* gz;
  long long ld_gz;
  int gact;
  int dx_set;  // bwd: dx = LN'(dy) (dx not read) instead of dx += LN'(dy)
  // fwd, the fused producer with an activation: xs = x + keep * act(add_y + add_bias) (Act; the
  // FFN down projection of the previous layer, whose GEMM then writes a plain bf16 z2)
  int add_act;
};

// Every load of the row (x, the fused add's y and bias, gamma, beta) is issued up front and
// unconditionally (a load under a branch is waited for with vmcnt(0) at the join): a lane past
// the row end re-reads the last chunk and is zeroed before the sums, and the add's operands read
// gamma (row stride 0, L1-resident) when the add has no bias.  ADD: the launch has the fused add
// (a template parameter: the plain form loads nothing of it).
// AACT (with ADD): the activation applied to the added term (Act; a template parameter so the
// element loop stays branch-free)
template <int NV, bool ADD, int AACT = 0>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LNArgs p) {
  const uint32_t dkey = p.drop_scale != 0.f ? drop_key_of(p.drop_seed, p.drop_site, p.drop_key) : 0u;
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.T) return;
  const int nv4 = p.D >> 2;
  constexpr bool has_add = ADD;
  const float4* xr = reinterpret_cast<const float4*>(p.x + row * p.ldx);
  const uint2* yr = reinterpret_cast<const uint2*>(has_add ? static_cast<const bf16_t*>(p.add_y) + row * p.ld_add
                                                           : nullptr);
  const bool has_bias = has_add && p.add_bias;
  const float4* ab4 = reinterpret_cast<const float4*>(has_bias ? p.add_bias : p.gamma);
  const float bsc = has_bias ? 1.f : 0.f;
  const float4* g4 = reinterpret_cast<const float4*>(p.gamma);
  const float4* b4 = reinterpret_cast<const float4*>(p.beta);
  float4 v[NV], ab[NV], gm[NV], bt[NV];
  uint2 yv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = min(lane + i * 64, nv4 - 1);
    v[i] = xr[c];
    if constexpr (ADD) {
      yv[i] = yr[c];
      ab[i] = ab4[c];
    }
    gm[i] = g4[c];
    bt[i] = b4[c];
  }
  __builtin_amdgcn_sched_barrier(0);
  float s = 0.f;
  float4* xo = reinterpret_cast<float4*>(p.x_out + row * p.ld_xout);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    const bool ok = c < nv4;
    if (!ok) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (ADD) {  // the fused residual add (no loads in here)
      float a[4] = {__uint_as_float(yv[i].x << 16) + ab[i].x * bsc, __uint_as_float(yv[i].x & 0xffff0000u) + ab[i].y * bsc,
                    __uint_as_float(yv[i].y << 16) + ab[i].z * bsc, __uint_as_float(yv[i].y & 0xffff0000u) + ab[i].w * bsc};
      if constexpr (AACT == ACT_GELU) {
        const dpc_f2_t g01 = gelu_tanh2(dpc_f2_t{a[0], a[1]}), g23 = gelu_tanh2(dpc_f2_t{a[2], a[3]});
        a[0] = g01.x; a[1] = g01.y; a[2] = g23.x; a[3] = g23.y;
      } else if constexpr (AACT == ACT_RELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = fmaxf(a[e], 0.f);
      }
      if (p.drop_scale != 0.f) {
        const uint32_t idx = (uint32_t)(row * p.D + 4 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] *= drop_factor(idx + e, dkey, p.drop_thresh, p.drop_scale);
      }
      if (ok) {
        v[i].x += a[0]; v[i].y += a[1]; v[i].z += a[2]; v[i].w += a[3];
        xo[c] = v[i];
      }
    }
    s += v[i].x + v[i].y + v[i].z + v[i].w;
  }
  const float mu = wave_sum(s) / p.D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nv4) {
      const float a = v[i].x - mu, b = v[i].y - mu, cc = v[i].z - mu, d = v[i].w - mu;
      ss += a * a + b * b + cc * cc + d * d;
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / p.D + p.eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nv4) {
      const float4 g = gm[i], b = bt[i];
      float4 o;
      o.x = (v[i].x - mu) * rs * g.x + b.x;
      o.y = (v[i].y - mu) * rs * g.y + b.y;
      o.z = (v[i].z - mu) * rs * g.z + b.z;
      o.w = (v[i].w - mu) * rs * g.w + b.w;
      if (p.y_f32) {
        reinterpret_cast<float4*>(static_cast<float*>(p.y) + row * p.ldy)[c] = o;
      } else {
        uint2 w;
        w.x = pack2bf(o.x, o.y);
        w.y = pack2bf(o.z, o.w);
        reinterpret_cast<uint2*>(static_cast<bf16_t*>(p.y) + row * p.ldy)[c] = w;
      }
    }
  }
  if (lane == 0) {
    p.mean[row] = mu;
    p.rstd[row] = rs;
  }
}

// One row's operands, loaded together (all of them before the row's reductions: the old
// dx += form read dx after the two wave sums, a second full memory latency per row, and the
// conditional read of the dx_set form was never hoisted above them by the compiler).
template <int NV, bool DYB>
struct LnBwdRow {
  float4 x[NV];
  typename std::conditional<DYB, uint2, float4>::type dy[NV];
  uint2 zz[NV];    // act' operand of the fused consumer (p.gz)
  float4 dold[NV]; // dx before this kernel (unless dx_set)
  float mu, rs;
};

// PF: the next row's operands are issued before this row's arithmetic (one row in flight
// behind the one being reduced), so a wave never waits a full memory latency per row.
template <int NV, bool DYB, bool PF>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LNArgs p) {
  const uint32_t dkey = p.drop_scale != 0.f ? drop_key_of(p.drop_seed, p.drop_site, p.drop_key) : 0u;
  __shared__ float red[4][2][NV * 256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nv4 = p.D >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(p.gamma);
  float4 gacc[NV], bacc[NV], gam[NV], cacc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    gacc[i] = bacc[i] = cacc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    gam[i] = c < nv4 ? g4[c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  bf16_t* gout = static_cast<bf16_t*>(p.gout);
  const bool use_z = gout && p.gz;
  using Row = LnBwdRow<NV, DYB>;
  // Branch-free loads (a load under a branch made the compiler wait for everything in flight at
  // the join, one memory latency per column chunk): a lane past the row end re-reads the row's
  // last chunk, and an operand the launch does not use is read from gamma with row stride 0
  // (L1-resident, D * 4 bytes >= what one row reads).  The results are ignored in those cases.
  const bf16_t* zbase = use_z ? static_cast<const bf16_t*>(p.gz) : reinterpret_cast<const bf16_t*>(p.gamma);
  const long long zld = use_z ? p.ld_gz : 0;
  const float* obase = p.dx_set ? p.gamma : p.dx;
  const long long old = p.dx_set ? 0 : p.lddx;
  const float keep_old = p.dx_set ? 0.f : 1.f;  // (gamma is finite: 0 * it is 0)
  auto load = [&](long long row, Row& r) {
    r.mu = p.mean[row];
    r.rs = p.rstd[row];
    const float4* xr = reinterpret_cast<const float4*>(p.x + row * p.ldx);
    const float4* dor = reinterpret_cast<const float4*>(obase + row * old);
    const uint2* zr = reinterpret_cast<const uint2*>(zbase + row * zld);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = min(lane + i * 64, nv4 - 1);
      r.x[i] = xr[c];
      if constexpr (DYB) r.dy[i] = reinterpret_cast<const uint2*>(static_cast<const bf16_t*>((const void*)p.dy) + row * p.lddy)[c];
      else r.dy[i] = reinterpret_cast<const float4*>(p.dy + row * p.lddy)[c];
      r.zz[i] = zr[c];
      r.dold[i] = dor[c];
    }
  };
  // compute: every operand is consumed outside any branch (a value used only under `c < nv4`
  // let the compiler sink its load into that branch, behind a vmcnt(0)); lanes past the row end
  // see dy = 0 (no contribution to the sums) and only their stores are skipped.
  auto compute = [&](long long row, const Row& r) {
    const float mu = r.mu, rs = r.rs;
    float4 xh[NV], dg[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const bool ok = lane + i * 64 < nv4;
      const float4 xv = r.x[i];
      float4 d;
      if constexpr (DYB) {
        const uint2 z = r.dy[i];
        d = make_float4(__uint_as_float(z.x << 16), __uint_as_float(z.x & 0xffff0000u),
                        __uint_as_float(z.y << 16), __uint_as_float(z.y & 0xffff0000u));
      } else {
        d = r.dy[i];
      }
      if (!ok) d = make_float4(0.f, 0.f, 0.f, 0.f);
      xh[i] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
      dg[i] = make_float4(d.x * gam[i].x, d.y * gam[i].y, d.z * gam[i].z, d.w * gam[i].w);
      s1 += dg[i].x + dg[i].y + dg[i].z + dg[i].w;
      s2 += dg[i].x * xh[i].x + dg[i].y * xh[i].y + dg[i].z * xh[i].z + dg[i].w * xh[i].w;
      gacc[i].x += d.x * xh[i].x; gacc[i].y += d.y * xh[i].y;
      gacc[i].z += d.z * xh[i].z; gacc[i].w += d.w * xh[i].w;
      bacc[i].x += d.x; bacc[i].y += d.y; bacc[i].z += d.z; bacc[i].w += d.w;
    }
    s1 = wave_sum(s1) / p.D;
    s2 = wave_sum(s2) / p.D;
    float4* dxr = reinterpret_cast<float4*>(p.dx + row * p.lddx);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + i * 64;
      const bool ok = c < nv4;
      // (a multiply, not a select: a select on the uniform flag became a branch with dx's load
      // sunk into it)
      float4 o = make_float4(r.dold[i].x * keep_old, r.dold[i].y * keep_old, r.dold[i].z * keep_old,
                             r.dold[i].w * keep_old);
      o.x += rs * (dg[i].x - s1 - xh[i].x * s2);
      o.y += rs * (dg[i].y - s1 - xh[i].y * s2);
      o.z += rs * (dg[i].z - s1 - xh[i].z * s2);
      o.w += rs * (dg[i].w - s1 - xh[i].w * s2);
      float4 og = o;
      if (use_z) {
        og.x *= act_grad(__uint_as_float(r.zz[i].x << 16), p.gact);
        og.y *= act_grad(__uint_as_float(r.zz[i].x & 0xffff0000u), p.gact);
        og.z *= act_grad(__uint_as_float(r.zz[i].y << 16), p.gact);
        og.w *= act_grad(__uint_as_float(r.zz[i].y & 0xffff0000u), p.gact);
      }
      if (gout && p.drop_scale != 0.f) {
        const uint32_t idx = (uint32_t)(row * p.D + 4 * c);
        og.x *= drop_factor(idx + 0, dkey, p.drop_thresh, p.drop_scale);
        og.y *= drop_factor(idx + 1, dkey, p.drop_thresh, p.drop_scale);
        og.z *= drop_factor(idx + 2, dkey, p.drop_thresh, p.drop_scale);
        og.w *= drop_factor(idx + 3, dkey, p.drop_thresh, p.drop_scale);
      }
      if (!ok) og = make_float4(0.f, 0.f, 0.f, 0.f);
      cacc[i].x += og.x; cacc[i].y += og.y; cacc[i].z += og.z; cacc[i].w += og.w;
      if (ok) {
        dxr[c] = o;
        if (gout) {
          uint2 wv;
          wv.x = pack2bf(og.x, og.y);
          wv.y = pack2bf(og.z, og.w);
          *reinterpret_cast<uint2*>(gout + row * p.ld_gout + 4 * c) = wv;
        }
      }
    }
  };
  const long long stride = (long long)gridDim.x * 4;
  long long row = (long long)blockIdx.x * 4 + w;
  if constexpr (PF) {
    // two rows per trip so the in-flight row alternates between ra and rb without copies; the
    // prefetch is unconditional (past the end it re-reads the last row): a load under a branch
    // would make the compiler wait for everything in flight before the current row's math
    Row ra, rb;
    const long long last = p.T - 1;
    if (row < p.T) {
      load(row, ra);
      // (scheduling barriers keep each row's loads issued as one group ahead of the other row's
      // math: interleaved, the waits for the row being reduced also covered the row in flight)
      while (true) {
        load(min(row + stride, last), rb);
        __builtin_amdgcn_sched_barrier(0);
        compute(row, ra);
        __builtin_amdgcn_sched_barrier(0);
        row += stride;
        if (row >= p.T) break;
        load(min(row + stride, last), ra);
        __builtin_amdgcn_sched_barrier(0);
        compute(row, rb);
        __builtin_amdgcn_sched_barrier(0);
        row += stride;
        if (row >= p.T) break;
      }
    }
  } else {
    for (; row < p.T; row += stride) {
      Row r;
      load(row, r);
      __builtin_amdgcn_sched_barrier(0);  // (all of the row's loads issued before any wait)
      compute(row, r);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // reduce dgamma / dbeta across the 4 waves, then one atomic per column per workgroup
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    reinterpret_cast<float4*>(&red[w][0][0])[c] = gacc[i];
    reinterpret_cast<float4*>(&red[w][1][0])[c] = bacc[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.D; c += 256) {
    float g = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
    float b = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    atomicAdd(p.dgamma + c, g);
    atomicAdd(p.dbeta + c, b);
  }
  if (!gout || !p.gsum) return;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + i * 64;
    if (c < nv4) reinterpret_cast<float4*>(&red[w][0][0])[c] = cacc[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.D; c += 256)
    atomicAdd(p.gsum + c, red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c]);
}

}  // namespace dpc

using namespace dpc;

template <int NV>
static void ln_fwd_nv(const LNArgs* a, dim3 grid, hipStream_t stream) {
  if (a->add_y && a->add_act == ACT_GELU) hipLaunchKernelGGL((ln_fwd_kernel<NV, true, ACT_GELU>), grid, dim3(256), 0, stream, *a);
  else if (a->add_y && a->add_act == ACT_RELU) hipLaunchKernelGGL((ln_fwd_kernel<NV, true, ACT_RELU>), grid, dim3(256), 0, stream, *a);
  else if (a->add_y) hipLaunchKernelGGL((ln_fwd_kernel<NV, true>), grid, dim3(256), 0, stream, *a);
  else hipLaunchKernelGGL((ln_fwd_kernel<NV, false>), grid, dim3(256), 0, stream, *a);
}

DPC_API int dpc_layernorm_fwd(const LNArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->D % 4 || a->add_act < 0 || a->add_act > ACT_GELU) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((a->T + 3) / 4));
  switch ((a->D + 255) / 256) {
    case 1: ln_fwd_nv<1>(a, grid, stream); break;
    case 2: ln_fwd_nv<2>(a, grid, stream); break;
    case 3: ln_fwd_nv<3>(a, grid, stream); break;
    case 4: ln_fwd_nv<4>(a, grid, stream); break;
    case 5: ln_fwd_nv<5>(a, grid, stream); break;
    case 6: ln_fwd_nv<6>(a, grid, stream); break;
    case 7: ln_fwd_nv<7>(a, grid, stream); break;
    case 8: ln_fwd_nv<8>(a, grid, stream); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// Workgroups of the persistent backward grid.  Each workgroup ends with 2 D column atomics
// (dgamma / dbeta), so the best grid shrinks as D grows: bench/ln_grid.py on MI355X, 1024 at
// D = 768 (5.2 TB/s; 512: 4.6, 2048: 4.3) and 512 at D = 1600 (4.4 TB/s; 1024: 4.1) -- i.e.
// ~786K column-atomics per launch, and at most one workgroup per 32 rows.  0 = that rule; > 0
// forces a size (sweeps).  The grid is also capped at what is resident at once (a second
// partial wave of workgroups would double the tail).
static int g_ln_bwd_blocks = getenv("DPC_LN_BWD_BLOCKS") ? atoi(getenv("DPC_LN_BWD_BLOCKS")) : 0;
DPC_API void dpc_layernorm_set_bwd_blocks(int n) { g_ln_bwd_blocks = n > 0 ? n : 0; }
// 1: the row-prefetch kernel (default), 0: one row at a time (DPC_LN_BWD_PF)
static int g_ln_bwd_pf = -1;
DPC_API void dpc_layernorm_set_bwd_prefetch(int v) { g_ln_bwd_pf = v; }

template <int NV, bool DYB, bool PF>
static int ln_bwd_launch(const LNArgs* a, long long cap, hipStream_t stream) {
  static int resident = 0;
  if (!resident) {
    int per_cu = 0, dev = 0, ncu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ln_bwd_kernel<NV, DYB, PF>, 256, 0) != hipSuccess)
      per_cu = 1;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
    resident = std::max(1, per_cu) * std::max(1, ncu);
  }
  const long long blocks = std::min<long long>((a->T + 3) / 4, std::min<long long>(cap, resident));
  hipLaunchKernelGGL((ln_bwd_kernel<NV, DYB, PF>), dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

template <int NV>
static int ln_bwd_nv(const LNArgs* a, long long cap, bool pf, hipStream_t stream) {
  if (a->dy_bf16) return pf ? ln_bwd_launch<NV, true, true>(a, cap, stream) : ln_bwd_launch<NV, true, false>(a, cap, stream);
  return pf ? ln_bwd_launch<NV, false, true>(a, cap, stream) : ln_bwd_launch<NV, false, false>(a, cap, stream);
}

DPC_API int dpc_layernorm_bwd(const LNArgs* a, hipStream_t stream) {
  if (a->T <= 0) return 0;
  if (a->D % 4) return (int)hipErrorInvalidValue;
  if (g_ln_bwd_pf < 0) g_ln_bwd_pf = getenv("DPC_LN_BWD_PF") ? atoi(getenv("DPC_LN_BWD_PF")) : 1;
  // (also at most one workgroup per 32 rows: the reference-default shape T = 16320, D = 256 ran
  // 36 us at 1024 workgroups, 25.6 us at 256-512 -- bench/ln_grid.py)
  long long cap = g_ln_bwd_blocks > 0 ? g_ln_bwd_blocks : std::min<long long>(786432 / a->D, (a->T + 31) / 32);
  cap = cap < 256 ? 256 : (cap > 1024 && g_ln_bwd_blocks <= 0 ? 1024 : cap);
  const bool pf = g_ln_bwd_pf != 0;
  switch ((a->D + 255) / 256) {
    case 1: return ln_bwd_nv<1>(a, cap, pf, stream);
    case 2: return ln_bwd_nv<2>(a, cap, pf, stream);
    case 3: return ln_bwd_nv<3>(a, cap, pf, stream);
    case 4: return ln_bwd_nv<4>(a, cap, pf, stream);
    case 5: return ln_bwd_nv<5>(a, cap, pf, stream);
    case 6: return ln_bwd_nv<6>(a, cap, pf, stream);
    case 7: return ln_bwd_nv<7>(a, cap, pf, stream);
    case 8: return ln_bwd_nv<8>(a, cap, pf, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
