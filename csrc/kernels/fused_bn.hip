// BatchNorm decomposed for conv fusion (training mode):
//   stats (sum, sumsq)  <- conv epilogue          (no separate statistics pass)
//   ss = finalize(stats, gamma, beta)             (per-channel, tiny; updates moving averages)
//   a  = relu(x*scale + shift)                    <- next conv's operand prologue (never stored)
//        or y = act(x*scale + shift + residual)   <- bn_apply (block outputs)
// Backward mirrors it:
//   bn_apply_bwd:  g = dy*[y>0];  dx = g*scale;  dres = g (or g*rscale);  sums (Σg·x, Σg) for dss
//   act_bwd:       same for the prologue-fused activation (mask recomputed from x)
//   finalize_bwd:  dss -> (dsum, dsumsq), dgamma, dbeta
//   stats_combine: dx_total = dx + dsum + 2*x*dsumsq   (the gradient through the statistics)
// Together these equal the textbook BN backward dx = scale*(g - mean(g) - xhat*mean(g*xhat)).
// Lane mapping: one fixed 8-channel column per lane (parameters in registers), 16-B accesses.
#include <cstring>

#include "common.h"

namespace dtm {

constexpr int FU2 = 4;

__device__ __forceinline__ void up8(uint4 u, float* f) {
  f[0] = lo_bf(u.x); f[1] = hi_bf(u.x); f[2] = lo_bf(u.y); f[3] = hi_bf(u.y);
  f[4] = lo_bf(u.z); f[5] = hi_bf(u.z); f[6] = lo_bf(u.w); f[7] = hi_bf(u.w);
}
__device__ __forceinline__ uint4 pk8(const float* f) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}


typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16(const bf16_t* p) {
  if (NT) {
    v4u_t v = __builtin_nontemporal_load((const v4u_t*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *(const uint4*)p;
}
template <bool NT>
__device__ __forceinline__ void st16(bf16_t* p, uint4 u) {
  if (NT) {
    v4u_t v = {u.x, u.y, u.z, u.w};
    __builtin_nontemporal_store(v, (v4u_t*)p);
  } else {
    *(uint4*)p = u;
  }
}

// y = act(x) path backward.  mode: 0 = plain BN (no relu), 1 = relu with mask from y, 2 = relu with
// mask recomputed from x*scale+shift.  res_mode 0/1/2 as in bn_apply.
// sx: [2][C] += (Σ g·x, Σ g)  (the dss of x's BN);  sr: same for a BN'd residual.
// mode 3: relu with the mask from the forward's bitmask (1 bit / element).  unscaled bit 0 (x) / bit 1
// (BN'd residual): that input's producer is a training conv+BN whose backward applies the BN scale
// itself (stats_combine_fin prescale), so the gradient handed to it is g, not g*scale; when dx and
// dres are both g, only dx is written and the caller aliases dres to it.
template <bool NT>
__global__ __launch_bounds__(256) void bn_apply_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                           const uint8_t* __restrict__ ymask,
                                                           const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                           const bf16_t* __restrict__ r, const float* __restrict__ rss,
                                                           bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                                           float* __restrict__ sx, float* __restrict__ sr, int M, int C,
                                                           int mode, int res_mode, int unscaled, int rpb, int lddy,
                                                           int direct) {
  __shared__ float red[2][256][8];
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  float sc[8], sh[8], rsc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = ss[c0 + e]; sh[e] = ss[C + c0 + e];
    rsc[e] = res_mode == 2 ? rss[c0 + e] : 1.f;
  }
  const bool ux = unscaled & 1, ur = (unscaled >> 1) & 1;
  float a1[8], a0[8], b1[8], b0[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a1[e] = a0[e] = b1[e] = b0[e] = 0.f;
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int row = lr0 < RP ? r0 + lr0 : r1; row < r1; row += RP * FU2) {
    uint4 vdy[FU2], vy[FU2], vx[FU2], vr[FU2];
    uint32_t mb[FU2];
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      int rr = row + u * RP;
      bool ok = rr < r1;
      size_t o = (size_t)rr * C + c0;
      uint4 z = make_uint4(0, 0, 0, 0);
      vdy[u] = ok ? ld16<NT>(dy + (size_t)rr * lddy + c0) : z;  // lddy > C: a concat slice
      vx[u] = ok ? ld16<NT>(x + o) : z;
      if (mode == 1) vy[u] = ok ? ld16<NT>(y + o) : z;
      if (mode == 3) mb[u] = ok ? (uint32_t)ymask[o >> 3] : 0u;
      if (res_mode == 2) vr[u] = ok ? ld16<NT>(r + o) : z;
    }
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      int rr = row + u * RP;
      if (rr >= r1) break;
      size_t o = (size_t)rr * C + c0;
      float g[8], xv[8];
      up8(vdy[u], g); up8(vx[u], xv);
      if (mode == 1) {
        float yv[8]; up8(vy[u], yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = yv[e] > 0.f ? g[e] : 0.f;
      } else if (mode == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = fmaf(xv[e], sc[e], sh[e]) > 0.f ? g[e] : 0.f;
      } else if (mode == 3) {
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = (mb[u] >> e) & 1u ? g[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) { a1[e] += g[e] * xv[e]; a0[e] += g[e]; }
      if (res_mode == 2) {
        float rv[8]; up8(vr[u], rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) { b1[e] += g[e] * rv[e]; b0[e] += g[e]; }
      }
      if (ux) {
        *(uint4*)(dx + o) = pk8(g);
      } else {
        float d[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = g[e] * sc[e];
        *(uint4*)(dx + o) = pk8(d);
      }
      // dres: skipped when it equals dx (the caller aliases the two)
      if (res_mode == 1 && !ux) {
        *(uint4*)(dres + o) = pk8(g);
      } else if (res_mode == 2 && !(ux && ur)) {
        if (ur) {
          *(uint4*)(dres + o) = pk8(g);
        } else {
          float dr[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) dr[e] = g[e] * rsc[e];
          *(uint4*)(dres + o) = pk8(dr);
        }
      }
    }
  }
  // partial row per block in the workspace: [Σg·x | Σg | (residual) Σg·r | Σg]
  if (direct) {  // small grid: atomics straight into the zeroed [Σg·x | Σg] outputs, no reduce launch
    col_reduce8(red, a1, a0, sx, sx + C, cols, c0, true);
    if (res_mode == 2) col_reduce8(red, b1, b0, sr, sr + C, cols, c0, true);
    return;
  }
  float* row = sx + (size_t)blockIdx.x * 4 * C;
  col_reduce8(red, a1, a0, row, row + C, cols, c0);
  if (res_mode == 2) col_reduce8(red, b1, b0, row + 2 * C, row + 3 * C, cols, c0);
}

// dx = dy + dsum[c] + 2*x*dsumsq[c]   (in place on dy allowed)
__global__ __launch_bounds__(256) void stats_combine_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                            const float* __restrict__ dstats, bf16_t* __restrict__ out,
                                                            int M, int C, int rpb) {
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  float a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { a[e] = dstats[c0 + e]; b[e] = 2.f * dstats[C + c0 + e]; }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int row = lr0 < RP ? r0 + lr0 : r1; row < r1; row += RP * FU2) {
    uint4 vd[FU2], vx[FU2];
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      int rr = row + u * RP;
      bool ok = rr < r1;
      size_t o = (size_t)rr * C + c0;
      vd[u] = ok ? *(const uint4*)(dy + o) : make_uint4(0, 0, 0, 0);
      vx[u] = ok ? *(const uint4*)(x + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      int rr = row + u * RP;
      if (rr >= r1) break;
      float d[8], xv[8];
      up8(vd[u], d); up8(vx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] += a[e] + b[e] * xv[e];
      *(uint4*)(out + (size_t)rr * C + c0) = pk8(d);
    }
  }
}

// stats_combine with the finalize backward folded in: the per-channel (dsum, dsumsq) come from
// fin_bwd_channel (common.h) in registers, and block 0 accumulates dgamma / dbeta.
// U rows in flight per lane; NT: non-temporal loads / stores (streamed once, keep L2/MALL for others)
template <int U, bool NT, bool NTS = NT>
__global__ __launch_bounds__(256) void stats_combine_fin_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                                const float* __restrict__ dss, const float* __restrict__ ss,
                                                                const float* __restrict__ gamma, float count,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                bf16_t* __restrict__ out, int M, int C, int prescale,
                                                                int rpb, int ldo) {
  __shared__ float s_ab[2][2048];
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  for (int c = t; c < C; c += 256) {  // one channel per thread, shared through LDS
    float ds, dq, dg, db;
    fin_bwd_channel(dss, ss, gamma, C, c, count, &ds, &dq, &dg, &db);
    s_ab[0][c] = ds;
    s_ab[1][c] = 2.f * dq;
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] += dg;
      if (dbeta) dbeta[c] += db;
    }
  }
  __syncthreads();
  float a[8], b[8], sc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = s_ab[0][c0 + e];
    b[e] = s_ab[1][c0 + e];
    sc[e] = prescale ? ss[c0 + e] : 1.f;  // dy is the unscaled g: the BN-apply gradient is g*scale
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  for (int row = lr0 < RP ? r0 + lr0 : r1; row < r1; row += RP * U) {
    uint4 vd[U], vx[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int rr = row + u * RP;
      bool ok = rr < r1;
      size_t o = (size_t)rr * C + c0;
      vd[u] = ok ? ld16<NT>(dy + o) : make_uint4(0, 0, 0, 0);
      vx[u] = ok ? ld16<NT>(x + o) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int rr = row + u * RP;
      if (rr >= r1) break;
      float d[8], xv[8];
      up8(vd[u], d); up8(vx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = fmaf(d[e], sc[e], a[e] + b[e] * xv[e]);
      st16<NTS>(out + (size_t)rr * ldo + c0, pk8(d));  // (ldo > C: a column slice of a wider buffer)
    }
  }
}

// finalize backward: dss [4][C] (dscale, dshift, dmean, drstd) -> dstats [2][C], dgamma, dbeta
// ss holds the forward's [scale, shift, mean, rstd].
__global__ void bn_finalize_bwd_kernel(const float* __restrict__ dss, const float* __restrict__ ss,
                                       const float* __restrict__ gamma, float* __restrict__ dstats,
                                       float* __restrict__ dgamma, float* __restrict__ dbeta, int C, float count) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float scale = ss[c], mean = ss[2 * C + c], rstd = ss[3 * C + c];
  const float g = gamma ? gamma[c] : 1.f;
  const float dsc = dss[c], dsh = dss[C + c];
  // shift = beta - mean*scale ; scale = g*rstd
  const float dscale_tot = dsc - dsh * mean;
  const float dmean = dss[2 * C + c] - dsh * scale;
  const float drstd = dss[3 * C + c] + dscale_tot * g;
  if (dgamma) dgamma[c] += dscale_tot * rstd;
  if (dbeta) dbeta[c] += dsh;
  // rstd = (var+eps)^-1/2, var = sumsq/M - mean^2, mean = sum/M
  const float dvar = drstd * (-0.5f) * rstd * rstd * rstd;
  dstats[c] = dmean / count - dvar * 2.f * mean / count;
  dstats[C + c] = dvar / count;
}

// stats-combine stream policy (A/B, tools/ab_step.py sc:): non-temporal loads of the two last-use
// streams, 4096-block cap: -0.9 % ResNet-50 step vs plain loads / 2048 blocks (nt stores: +0.4 %)
static int g_sc_var = 5, g_sc_cap = 4096;
// non-temporal input loads: bit 0 bn_apply_fast (forward), bit 1 bn_apply_bwd
static int g_ntld = 3;  // A/B (ResNet-50 b256): both on -1.5 % step time on top of the stats-combine policy

// ---- zero-copy concat, all parts in one launch (Inception mixed blocks: 3-4 BN'd branches per block) --------
// Part k owns channels [off, off + C) of the [M][Ct] concat; its BN-apply input raw / ss / mask are its own
// [M][C] tensors.  Each lane keeps one fixed 8-channel column of the CONCAT row (so it belongs to one part),
// so the whole block output is written / its gradient read in full coalesced rows, and the per-part
// launches (and, backward, their reduce launches) collapse into one.
constexpr int CAT_MAXP = 8;
struct CatPart {
  const bf16_t* raw;
  const float* ss;
  uint8_t* mask;
  bf16_t* dx;       // backward: the part's input gradient [M][C]
  int C, off, flags;  // flags bit 0: relu (forward) / unscaled (backward); bit 1: a plain tensor part (copied
                      // forward, no BN; its gradient is the caller's view of the concat gradient)
};
struct CatArgs {
  CatPart p[CAT_MAXP];
  int np, Ct, M, rpb;
};
__device__ __forceinline__ int cat_part(const CatArgs& a, int gc) {
  int k = 0;
#pragma unroll
  for (int i = 1; i < CAT_MAXP; ++i)
    if (i < a.np && gc >= a.p[i].off) k = i;
  return k;
}

__global__ __launch_bounds__(256) void cat_bn_apply_kernel(CatArgs a, bf16_t* __restrict__ out) {
  const int cols = a.Ct >> 3, t = threadIdx.x, RP = 256 / cols, gc = (t % cols) * 8, lr0 = t / cols;
  if (lr0 >= RP) return;
  const int k = cat_part(a, gc);
  const CatPart& P = a.p[k];
  const int cl = gc - P.off;
  const bool relu = P.flags & 1, plain = P.flags & 2;
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = plain ? 1.f : P.ss[cl + e];
    sh[e] = plain ? 0.f : P.ss[P.C + cl + e];
  }
  const int r0 = blockIdx.x * a.rpb, r1 = min(a.M, r0 + a.rpb);
  for (int row = r0 + lr0; row < r1; row += RP * FU2) {
    uint4 v[FU2];
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      const int rr = row + u * RP;
      v[u] = rr < r1 ? ld16<true>(P.raw + (size_t)rr * P.C + cl) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      const int rr = row + u * RP;
      if (rr >= r1) break;
      if (plain) {  // a plain part is copied bit for bit
        *(uint4*)(out + (size_t)rr * a.Ct + gc) = v[u];
        continue;
      }
      float f[8];
      up8(v[u], f);
      uint32_t bits = 0u;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f[e] = fmaf(f[e], sc[e], sh[e]);
        if (relu) f[e] = fmaxf(f[e], 0.f);
        bits |= (f[e] > 0.f ? 1u : 0u) << e;
      }
      *(uint4*)(out + (size_t)rr * a.Ct + gc) = pk8(f);
      if (P.mask) P.mask[((size_t)rr * P.C + cl) >> 3] = (uint8_t)bits;
    }
  }
}

// backward: g = d(concat slice) * mask bit; dx = g (unscaled producer) or g*scale; per block a partial row of
// width 4*Ct laid out as every part's [4][C] (Σg·x | Σg | 0 | 0), so ONE reduction yields the parts' dss
// buffers back to back
// NT lanes per block (cat_bwd_threads): 512 for the wide concats - every lane owns a column (a 768-channel concat
// at 256 lanes left a quarter of them idle, 1280 channels 38 %) and half the partial rows to reduce
// (profiles/ab/r5_ab_pool_k3s2.log, session s21: 17x17x768 69.7 -> 56.3 us, 8x8x2048 51.3 -> 40.2 us); 256 for
// the 35x35 ones (<= 64 columns), which measured 4 % slower on 512.
template <int NT>
__global__ __launch_bounds__(NT) void cat_bn_apply_bwd_kernel(CatArgs a, const bf16_t* __restrict__ dout,
                                                              float* __restrict__ ws) {
  __shared__ float red[2][NT][8];
  const int cols = a.Ct >> 3, t = threadIdx.x, RP = NT / cols, gc = (t % cols) * 8, lr0 = t / cols;
  const int k = cat_part(a, gc);
  const CatPart& P = a.p[k];
  const int cl = gc - P.off;
  const bool ux = P.flags & 1, plain = P.flags & 2;
  float sc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sc[e] = plain ? 1.f : P.ss[cl + e];
  float a1[8], a0[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a1[e] = a0[e] = 0.f;
  const int r0 = blockIdx.x * a.rpb, r1 = min(a.M, r0 + a.rpb);
  // (a plain part's lanes only join the block reduction below, with zeros)
  for (int row = (lr0 < RP && !plain) ? r0 + lr0 : r1; row < r1; row += RP * FU2) {
    uint4 vd[FU2], vx[FU2];
    uint32_t mb[FU2];
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      const int rr = row + u * RP;
      const bool ok = rr < r1;
      const size_t o = (size_t)rr * P.C + cl;
      vd[u] = ok ? ld16<true>(dout + (size_t)rr * a.Ct + gc) : make_uint4(0, 0, 0, 0);
      vx[u] = ok ? ld16<true>(P.raw + o) : make_uint4(0, 0, 0, 0);
      mb[u] = ok ? (uint32_t)P.mask[o >> 3] : 0u;
    }
#pragma unroll
    for (int u = 0; u < FU2; ++u) {
      const int rr = row + u * RP;
      if (rr >= r1) break;
      float g[8], xv[8];
      up8(vd[u], g);
      up8(vx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        g[e] = (mb[u] >> e) & 1u ? g[e] : 0.f;
        a1[e] += g[e] * xv[e];
        a0[e] += g[e];
        if (!ux) g[e] *= sc[e];
      }
      *(uint4*)(P.dx + (size_t)rr * P.C + cl) = pk8(g);
    }
  }
  float* row = ws + (size_t)blockIdx.x * 4 * a.Ct + 4 * P.off;  // this part's [4][C] image in the row
  col_reduce8<NT>(red, a1, a0, row - P.off, row + P.C - P.off, cols, gc);
  if (t < cols) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { row[2 * P.C + cl + e] = 0.f; row[3 * P.C + cl + e] = 0.f; }
  }
}

static int g_cpt = 8;  // A/B knob: 16-B chunks per thread the BN-stream grids aim for (dtm_set_grid_cpt)
DTM_API void dtm_set_grid_cpt(int n) { g_cpt = n > 0 ? n : 8; }
static void grid2(long M, int C, int* blocks, int* rpb, int cap = 2048, int nt = 256) {
  int cols = C / 8, RP = nt / cols;
  long chunks = M * cols;
  long b = chunks / ((long)nt * g_cpt);
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  long r = (M + b - 1) / b;
  r = (r + RP - 1) / RP * RP;
  *rpb = (int)r;
  *blocks = (int)((M + r - 1) / r);
}

}  // namespace dtm
using namespace dtm;

DTM_API void dtm_set_ntld_policy(int bits) { dtm::g_ntld = bits; }
int dtm_ntld_bits() { return dtm::g_ntld; }

static int shape_ok(long M, int C) {
  if (C % 8) return 0;
  int cols = C / 8;
  return cols <= 256 && M < (1l << 31);
}

DTM_API int dtm_bn_apply_bwd(const void* dy, const void* y, const void* ymask, const void* x, const float* ss,
                             const void* r, const float* rss, void* dx, void* dres, float* sx, float* sr, long M, int C,
                             int mode, int res_mode, int unscaled, void* stream) {
  if (!shape_ok(M, C)) return -1;
  if ((mode == 3 && !ymask) || (mode == 1 && !y)) return -2;
  int blocks, rpb;
  grid2(M, C, &blocks, &rpb);
  if (blocks <= dtm_reduce_direct_max()) {
    hipLaunchKernelGGL((g_ntld & 2) ? bn_apply_bwd_kernel<true> : bn_apply_bwd_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const bf16_t*)y, (const uint8_t*)ymask, (const bf16_t*)x, ss, (const bf16_t*)r, rss,
                       (bf16_t*)dx, (bf16_t*)dres, sx, sr, (int)M, C, mode, res_mode, unscaled, rpb, C, 1);
    return 0;
  }
  float* ws = dtm_ws_get_stream((size_t)blocks * 4 * C, (hipStream_t)stream);
  if (!ws) return -4;
  hipLaunchKernelGGL((g_ntld & 2) ? bn_apply_bwd_kernel<true> : bn_apply_bwd_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)y, (const uint8_t*)ymask, (const bf16_t*)x, ss, (const bf16_t*)r, rss, (bf16_t*)dx,
                     (bf16_t*)dres, ws, nullptr, (int)M, C, mode, res_mode, unscaled, rpb, C, 0);
  dtm_reduce_rows(ws, blocks, 2 * C, 4 * C, sx, (hipStream_t)stream);
  if (res_mode == 2) dtm_reduce_rows(ws + 2 * C, blocks, 2 * C, 4 * C, sr, (hipStream_t)stream);
  return 0;
}

// backward of dtm_bn_apply_ld: dy is the channel slice [0, C) of rows of lddy channels (the concat's
// gradient read in place), ReLU from the forward bitmask, no residual
DTM_API int dtm_bn_apply_bwd_ld(const void* dy, const void* ymask, const void* x, const float* ss, void* dx, float* sx,
                                long M, int C, int unscaled, int lddy, void* stream) {
  if (!shape_ok(M, C) || !ymask || lddy < C || lddy % 8 || ((uintptr_t)dy & 15)) return -1;
  int blocks, rpb;
  grid2(M, C, &blocks, &rpb);
  const int direct = blocks <= dtm_reduce_direct_max();
  float* ws = direct ? sx : dtm_ws_get_stream((size_t)blocks * 4 * C, (hipStream_t)stream);
  if (!ws) return -4;
  hipLaunchKernelGGL((g_ntld & 2) ? bn_apply_bwd_kernel<true> : bn_apply_bwd_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)nullptr, (const uint8_t*)ymask, (const bf16_t*)x, ss, (const bf16_t*)nullptr,
                     (const float*)nullptr, (bf16_t*)dx, (bf16_t*)nullptr, ws, nullptr, (int)M, C, 3, 0, unscaled & 1,
                     rpb, lddy, direct);
  if (!direct) dtm_reduce_rows(ws, blocks, 2 * C, 4 * C, sx, (hipStream_t)stream);
  return 0;
}

// Zero-copy concat of np BN'd parts in one launch: descs[np] = {raw, ss, mask, dx, C, off, flags}, from the
// host as a packed table (dtm_cat_desc_bytes per part).  Forward writes out [M][Ct] and the masks.
DTM_API int dtm_cat_desc_bytes() { return (int)sizeof(CatPart); }
static int cat_args(const void* descs, int np, long M, int Ct, CatArgs* a) {
  if (np < 1 || np > CAT_MAXP || Ct % 8 || Ct / 8 > 256 || M >= (1l << 31)) return -1;
  memcpy(a->p, descs, np * sizeof(CatPart));
  int off = 0;
  for (int i = 0; i < np; ++i) {
    if (a->p[i].off != off || a->p[i].C % 8 || !a->p[i].raw || (!a->p[i].ss && !(a->p[i].flags & 2))) return -1;
    off += a->p[i].C;
  }
  if (off != Ct) return -1;
  a->np = np; a->Ct = Ct; a->M = (int)M;
  return 0;
}
DTM_API int dtm_cat_bn_apply(const void* descs, int np, void* out, long M, int Ct, void* stream) {
  CatArgs a;
  if (cat_args(descs, np, M, Ct, &a) || ((uintptr_t)out & 15)) return -1;
  int blocks;
  grid2(M, Ct, &blocks, &a.rpb);
  hipLaunchKernelGGL(cat_bn_apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, (bf16_t*)out);
  return 0;
}
// Backward: dout [M][Ct]; every part's dx gets g (or g*scale), and sums [4*Ct] (zeroed by the caller) +=
// the parts' [4][C] ss gradients back to back (rows 0-1: Σg·x, Σg; rows 2-3 stay zero).
DTM_API int dtm_cat_bn_apply_bwd(const void* descs, int np, const void* dout, float* sums, long M, int Ct, void* stream) {
  CatArgs a;
  if (cat_args(descs, np, M, Ct, &a) || ((uintptr_t)dout & 15)) return -1;
  for (int i = 0; i < np; ++i)
    if (!(a.p[i].flags & 2) && (!a.p[i].mask || !a.p[i].dx)) return -1;
  int blocks;
  const int nt = Ct / 8 > 64 ? 512 : 256;
  grid2(M, Ct, &blocks, &a.rpb, 2048, nt);
  float* ws = dtm_ws_get_stream((size_t)blocks * 4 * Ct, (hipStream_t)stream);
  if (!ws) return -4;
  hipLaunchKernelGGL(nt == 512 ? cat_bn_apply_bwd_kernel<512> : cat_bn_apply_bwd_kernel<256>, dim3(blocks),
                     dim3((Ct / 8) * (nt / (Ct / 8))), 0, (hipStream_t)stream, a,
                     (const bf16_t*)dout, ws);
  dtm_reduce_rows(ws, blocks, 4 * Ct, 4 * Ct, sums, (hipStream_t)stream);
  return 0;
}

DTM_API int dtm_stats_combine(const void* dy, const void* x, const float* dstats, void* out, long M, int C,
                              void* stream) {
  if (!shape_ok(M, C)) return -1;
  int blocks, rpb;
  grid2(M, C, &blocks, &rpb);
  hipLaunchKernelGGL(stats_combine_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)x, dstats, (bf16_t*)out, (int)M, C, rpb);
  return 0;
}

DTM_API void dtm_bn_finalize_bwd(const float* dss, const float* ss, const float* gamma, float* dstats, float* dgamma,
                                 float* dbeta, int C, float count, void* stream) {
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, dss, ss, gamma,
                     dstats, dgamma, dbeta, C, count);
}

DTM_API int dtm_stats_combine_fin_ld(const void* dy, const void* x, const float* dss, const float* ss,
                                     const float* gamma, float count, float* dgamma, float* dbeta, void* out, long M, int C,
                                     int prescale, int ldo, void* stream);
DTM_API int dtm_stats_combine_fin(const void* dy, const void* x, const float* dss, const float* ss, const float* gamma,
                                  float count, float* dgamma, float* dbeta, void* out, long M, int C, int prescale,
                                  void* stream) {
  return dtm_stats_combine_fin_ld(dy, x, dss, ss, gamma, count, dgamma, dbeta, out, M, C, prescale, C, stream);
}

// out rows of ldo elements (ldo >= C, ldo % 8 == 0): the combined gradient of one conv written into its column
// slice of a buffer shared with sibling convs (one merged dgrad / wgrad over all of them, ops/fused.py)
DTM_API int dtm_stats_combine_fin_ld(const void* dy, const void* x, const float* dss, const float* ss,
                                     const float* gamma, float count, float* dgamma, float* dbeta, void* out, long M, int C,
                                     int prescale, int ldo, void* stream) {
  if (!shape_ok(M, C) || C > 2048 || ldo < C || ldo % 8) return -1;
  int blocks, rpb;
  grid2(M, C, &blocks, &rpb, g_sc_cap);
#define SCF_LAUNCH(U, NT, NTS)                                                                                    \
  hipLaunchKernelGGL((stats_combine_fin_kernel<U, NT, NTS>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,          \
                     (const bf16_t*)dy, (const bf16_t*)x, dss, ss, gamma, count, dgamma, dbeta, (bf16_t*)out, (int)M, \
                     C, prescale, rpb, ldo)
  switch (g_sc_var) {
    case 1: SCF_LAUNCH(8, false, false); break;
    case 2: SCF_LAUNCH(4, true, true); break;
    case 3: SCF_LAUNCH(8, true, true); break;
    case 4: SCF_LAUNCH(2, false, false); break;
    case 5: SCF_LAUNCH(4, true, false); break;
    case 6: SCF_LAUNCH(4, false, true); break;
    default: SCF_LAUNCH(4, false, false); break;
  }
#undef SCF_LAUNCH
  return 0;
}

// ---- grouped stats-combine of a merged sibling group (ops/fused.py _SiblingGroup): every member's combined
// gradient comb_i = g_i*scale_i + ds_i + 2*dq_i*y_i written into its column slice [off_i, off_i + C_i) of ONE
// [M][ldo] buffer, members as gridDim.y, in one launch instead of one per member; a member without BatchNorm
// (dss == nullptr: Inception's commuted pool-branch conv) is copied into its slice.
struct CombMember {
  const bf16_t* dy;
  const bf16_t* x;
  const float* dss;
  const float* ss;
  const float* gamma;
  float* dgamma;
  float* dbeta;
  int C, off;
};
struct CombGroup {
  CombMember m[8];
};

__global__ __launch_bounds__(256) void stats_combine_multi_kernel(CombGroup grp, float count, bf16_t* __restrict__ out,
                                                                  int M, int rpb, int ldo) {
  __shared__ float s_ab[2][2048];
  CombMember mb;
  // constant-index selection (a dynamically indexed argument array would go through scratch)
  switch (blockIdx.y) {
    case 0: mb = grp.m[0]; break;
    case 1: mb = grp.m[1]; break;
    case 2: mb = grp.m[2]; break;
    case 3: mb = grp.m[3]; break;
    case 4: mb = grp.m[4]; break;
    case 5: mb = grp.m[5]; break;
    case 6: mb = grp.m[6]; break;
    default: mb = grp.m[7]; break;
  }
  const int C = mb.C;
  const int cols = C >> 3, t = threadIdx.x, RP = 256 / cols, c0 = (t % cols) * 8, lr0 = t / cols;
  const bool bn = mb.dss != nullptr;
  for (int c = t; c < C; c += 256) {
    float ds = 0.f, dq = 0.f, dg, db;
    if (bn) {
      fin_bwd_channel(mb.dss, mb.ss, mb.gamma, C, c, count, &ds, &dq, &dg, &db);
      if (blockIdx.x == 0) {
        if (mb.dgamma) mb.dgamma[c] += dg;
        if (mb.dbeta) mb.dbeta[c] += db;
      }
    }
    s_ab[0][c] = ds;
    s_ab[1][c] = 2.f * dq;
  }
  __syncthreads();
  float a[8], b[8], sc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = s_ab[0][c0 + e];
    b[e] = s_ab[1][c0 + e];
    sc[e] = bn ? mb.ss[c0 + e] : 1.f;  // (dy is the unscaled g)
  }
  const int r0 = blockIdx.x * rpb, r1 = min(M, r0 + rpb);
  bf16_t* o = out + mb.off;
  for (int row = lr0 < RP ? r0 + lr0 : r1; row < r1; row += RP * 4) {
    uint4 vd[4], vx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rr = row + u * RP;
      const bool ok = rr < r1;
      const size_t q = (size_t)rr * C + c0;
      vd[u] = ok ? *(const uint4*)(mb.dy + q) : make_uint4(0, 0, 0, 0);
      vx[u] = (ok && bn) ? *(const uint4*)(mb.x + q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int rr = row + u * RP;
      if (rr >= r1) break;
      float d[8], xv[8];
      up8(vd[u], d); up8(vx[u], xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = fmaf(d[e], sc[e], a[e] + b[e] * xv[e]);
      *(uint4*)(o + (size_t)rr * ldo + c0) = pk8(d);
    }
  }
}

// descs: n x {dy, x, dss (or 0), ss, gamma, dgamma, dbeta} pointers as int64 + {C, off} ints, host memory
DTM_API int dtm_stats_combine_multi(const void* const* ptrs, const int* dims, int n, float count, void* out, long M,
                                    int ldo, void* stream) {
  if (n < 1 || n > 8 || ldo % 8 || M >= (1l << 31)) return -1;
  CombGroup g;
  int cmax = 0;
  for (int i = 0; i < 8; ++i) {
    CombMember& m = g.m[i];
    if (i >= n) {
      m = g.m[0];
      continue;
    }
    m.dy = (const bf16_t*)ptrs[7 * i];
    m.x = (const bf16_t*)ptrs[7 * i + 1];
    m.dss = (const float*)ptrs[7 * i + 2];
    m.ss = (const float*)ptrs[7 * i + 3];
    m.gamma = (const float*)ptrs[7 * i + 4];
    m.dgamma = (float*)ptrs[7 * i + 5];
    m.dbeta = (float*)ptrs[7 * i + 6];
    m.C = dims[2 * i];
    m.off = dims[2 * i + 1];
    if (!shape_ok(M, m.C) || m.C > 2048 || m.off % 8 || m.off + m.C > ldo) return -1;
    if (m.C > cmax) cmax = m.C;
  }
  int blocks, rpb;
  grid2(M, cmax, &blocks, &rpb, g_sc_cap);
  hipLaunchKernelGGL(stats_combine_multi_kernel, dim3(blocks, n), dim3(256), 0, (hipStream_t)stream, g, count,
                     (bf16_t*)out, (int)M, rpb, ldo);
  return 0;
}

// A/B policy of the stats-combine stream: variant (0 U4, 1 U8, 2 U4 nt, 3 U8 nt, 4 U2, 5 U4 nt loads,
// 6 U4 nt stores) and block cap
DTM_API void dtm_set_sc_policy(int variant, int cap) {
  g_sc_var = variant;
  g_sc_cap = cap > 0 ? cap : 2048;
}
