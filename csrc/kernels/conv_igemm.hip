// Implicit-GEMM convolution kernels for gfx950 (CDNA4), NHWC bf16, fp32 accumulate.
//
// Replaces the cuDNN Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter kernels that the
// reference gets from the TF runtime (call sites e.g.
// reference vgg/nets/resnet_v1.py:111-128 via slim.conv2d, inception/slim/ops.py:232).
//
// Design (MI355X-first, not a translation of any CUDA tiling):
//  * conv_nt:  C[chan][pix] = W[chan][k] . X[pix][k]  with k = (r, s, c).  Used for forward and
//    (with a flipped/transposed weight and input dilation UD = forward stride) for dgrad.
//    MFMA "A" operand = weight rows (output channels), "B" operand = gathered pixel rows, so
//    each lane of a 16x16 accumulator holds 4 consecutive output channels of one pixel -> one
//    8-byte NHWC store per lane, no LDS round trip in the epilogue.
//    Both operands are staged through LDS as [row][64 k] bf16 (128-B rows) with a
//    chunk ^= (row & 7) XOR swizzle: conflict-free ds_write_b128 and ds_read_b128 for the
//    v_mfma_f32_16x16x32_bf16 fragment pattern (checked by tools/lds_bank_check.py).
//    Zero padding comes for free from buffer loads with an out-of-range offset.
//    Optional fusions: per-input-channel affine+ReLU prologue (the previous layer's BatchNorm
//    apply, so the normalised activation is never written to HBM), bias/ReLU epilogue, and
//    per-output-channel sum / sum-of-squares for training BatchNorm (fp32 atomics, one per
//    channel per wave after a 16-lane shuffle reduction).
//  * conv_wgrad: dW[ko][(r,s,c)] = sum_pix dY[pix][ko] * X[pix @ tap][c].  Both operands are
//    k(=pixel)-major in memory, so they are staged as [k/4][row/16][4][16] blocks and read with
//    ds_read_b64_tr_b16 (the CDNA4 hardware transpose) straight into MFMA fragments.
//    Split-K over pixels; partial tiles are added into the fp32 gradient with float atomics.
#include "common.h"
#include <cstdio>

namespace dtm {

// (xcd_remap: common.h)

struct ConvNTArgs {
  const bf16_t* x;        // [N][Hin][Win][C]
  const bf16_t* w;        // [K][R][S][C]
  bf16_t* y;              // [N][P][Q][K]
  float* stats;           // nullptr or [2][K] : sum, sumsq of the (bf16-rounded) output
  const float* bias;      // nullptr or [K]
  const float* in_scale;  // nullptr or [C]: x <- relu(x*in_scale + in_shift) for in-bounds taps
  const float* in_shift;
  uint32_t x_bytes, w_bytes;
  int N, Hin, Win, C, K, R, S, P, Q;
  int stride, pad_h, pad_w;  // on the virtual (dilated) input
  int Hv, Wv;                // virtual input extent (Hin-1)*UD+1
  int M;                     // N*P*Q
  int Kg;                    // R*S*C
  int relu;
  FastDiv fd_PQ, fd_Q;
  // optional epilogue post-ops on the coalesced 16-B output chunks (used by dgrad):
  const bf16_t* add_src;  // out += add_src (the other consumer's gradient of a shared input)
  int add_stride;         //   > 1: add_src is [N][add_H][add_W][K], added at pixels (h, w) % add_stride == 0
  int add_H, add_W;       //   (the gradient of a strided subsample of this tensor)
  const bf16_t* act_x;    // fused activation backward of the input's BatchNorm+ReLU prologue:
  const float* act_ss;    //   g = out * [act_x*scale + shift > 0]; out <- g*scale;
  float* act_sums;        //   partial rows per pixel tile: [sum g*act_x (K) | sum g (K)]
  const bf16_t* zero;     // >= 16 B of zeros: the LDS-DMA source of padding / out-of-range chunks
  int act_unscaled;       // act path: out <- g (not g*scale); the producer's conv+BN backward scales it
  const uint8_t* act_mask;  // act path, block-output form: the ReLU mask is the forward's bitmask (1 bit per
                            //   element) of relu(bn(act_x) + residual) instead of act_x*scale+shift > 0
  const bf16_t* act_r;      //   + a BN'd residual: also sum g*act_r -> rows [g*x | g | g*r | g] (4K wide)
  int pix_bytes;          // byte pitch of one input pixel (C*2, or less for the packed-row stem view)
  bf16_t* dump;           // >= 16 B scratch: target of the out-of-range stores of the exact-count epilogue
  // output remap of a stride-decomposed dgrad (ostr > 1): output pixel (n, i, j) of this launch's P x Q
  // grid is pixel (n, i*ostr + oa, j*ostr + ob) of the OH x OW tensor that y and every epilogue side
  // input (add_src, act_x, act_r, act_mask) index.  ostr == 1: identity (OH = P, OW = Q, oa = ob = 0)
  int ostr, oa, ob, OH, OW;
  // spatial output tiles (conv3x3_direct_kernel): sp_tw > 0 -> pixel m of this launch is local pixel m % 128
  // (row-major 8 x 16) of spatial tile m / 128, tiles ordered [N][tiles_h][sp_tw]; pixels past P / Q are
  // out of range (M = tiles * 128)
  int sp_tw, sp_th;
  FastDiv fd_sp_img, fd_sp_tw;
  // grouped launch of a stride-decomposed dgrad (ngrp > 1, gridDim.z = ngrp): every output parity class is one
  // z-slice of ONE launch instead of a launch of its own; the classes share M / P / Q / K and differ in the
  // fields below (their taps of the decomposed weight, output parity, partial-sum rows)
  int ngrp;
  struct Grp {
    const bf16_t* w;
    float* act_sums;
    int R, S, pad_h, pad_w, oa, ob, Kg;
  } grp[4];
  // merged sibling convs (forward, nsplit > 0): output channel k belongs to member j (split[j].off <= k <
  // split[j+1].off) and is stored at split[j].y[pixel][k - off_j] (row of split[j].K) - one conv over the members'
  // concatenated weights writing each member's own contiguous output (ops/fused.py _SiblingGroup)
  int nsplit;
  struct Split {
    bf16_t* y;
    int off, K;
  } split[8];
};

// block -> (class, tile) of a grouped launch (XCD remap over the whole grid; class = z-slice of the logical
// order) and the class's fields copied into a; a plain launch (gridDim.z == 1) keeps the 2-D remap
__device__ __forceinline__ int grp_tile(ConvNTArgs& a) {
  const int gxy = gridDim.x * gridDim.y;
  const int t = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gxy * gridDim.z);
  if (gridDim.z > 1) {
    // constant indices only: a dynamically indexed member array would put the whole argument block in scratch
    const int g = t / gxy;
#define DTM_GRP_LOAD(k)                                                                   \
  a.w = a.grp[k].w; a.act_sums = a.grp[k].act_sums; a.R = a.grp[k].R; a.S = a.grp[k].S; \
  a.pad_h = a.grp[k].pad_h; a.pad_w = a.grp[k].pad_w; a.oa = a.grp[k].oa; a.ob = a.grp[k].ob; a.Kg = a.grp[k].Kg
    if (g == 0) { DTM_GRP_LOAD(0); }
    else if (g == 1) { DTM_GRP_LOAD(1); }
    else if (g == 2) { DTM_GRP_LOAD(2); }
    else { DTM_GRP_LOAD(3); }
#undef DTM_GRP_LOAD
  }
  return t % gxy;
}

// full-resolution coordinates / row of output pixel m (see ConvNTArgs::ostr)
__device__ __forceinline__ void out_nhw(const ConvNTArgs& a, int m, int& n, int& h, int& w) {
  if (a.sp_tw) {
    const uint32_t t = (uint32_t)m >> 7, l = (uint32_t)m & 127u;
    const uint32_t nn = fdiv(t, a.fd_sp_img), rem = t - nn * (a.sp_th * a.sp_tw);
    const uint32_t th = fdiv(rem, a.fd_sp_tw), tw = rem - th * a.sp_tw;
    n = (int)nn;
    h = (int)(th * 8u + (l >> 4));
    w = (int)(tw * 16u + (l & 15u));
    return;
  }
  const uint32_t nn = fdiv((uint32_t)m, a.fd_PQ), rem = m - nn * (a.P * a.Q);
  const uint32_t i = fdiv(rem, a.fd_Q), j = rem - i * a.Q;
  n = (int)nn;
  h = (int)i * a.ostr + a.oa;
  w = (int)j * a.ostr + a.ob;
}
__device__ __forceinline__ int out_row(const ConvNTArgs& a, int m) {
  if (a.ostr == 1 && !a.sp_tw) return m;
  int n, h, w;
  out_nhw(a, m, n, h, w);
  return (n * a.OH + h) * a.OW + w;
}

// spatial-tile launches: pixel m lies inside the P x Q output (always true otherwise)
__device__ __forceinline__ bool out_valid(const ConvNTArgs& a, int m) {
  if (!a.sp_tw) return true;
  int n, h, w;
  out_nhw(a, m, n, h, w);
  return h < a.P && w < a.Q;
}

// Shared epilogue of the conv_nt kernels (register-staged and LDS-DMA): acc[TC][TP] of wave (wp, wc)
// for the tile at pixel p0 / channel c0; smem must hold PT * (2*CT + 16) bytes and be free.
// RAWB: raw s_barrier (+ lgkmcnt) instead of __syncthreads(), so LDS-DMA prefetches of the next tile stay
// in flight across the epilogue; EXACT: every thread issues exactly PT*CT/8/256 staged 16-B stores
// (out-of-range ones go to a.dump), a lower bound the persistent kernel's counted vmcnt relies on.
template <bool RAWB>
__device__ __forceinline__ void epi_barrier() {
  if constexpr (RAWB) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
}

// STG: 1 = LDS-staged stores (K % 8 == 0), 2 = direct 8-B stores.  Kept compile-time: a runtime choice
// between an LDS and a global pointer makes hipcc emit flat stores, which wait on both counters.
// SACC (statistics accumulate, persistent kernels): the BatchNorm sums are not shuffle-reduced per tile;
// each thread adds the bf16 outputs of its fixed 8-channel chunk column in the staged-store loop to
// ssum / ssq (registers, across all the block's tiles) and the kernel reduces them once at its end.
// NT: threads of the block (256 = 4 waves, 512 = the 8-wave big-tile kernel).
// Staged-store tail of the conv_nt epilogues: the block's output tile is in LDS as bf16 rows of
// OROW bytes (pixel-major); each thread stores full 16-B chunks (coalesced NHWC rows) with the dgrad
// post-ops (add_src, activation backward, block-output BN-apply backward) and the BatchNorm statistics
// / post-op partial sums.  Shared by the 16x16x32 and the 32x32x16 MFMA register layouts.
// SIDE = false compiles the dgrad post-ops out: their loads are what the compiler's own vmcnt waits track,
// and a persistent kernel's loop-carried wait for them (vmcnt(n) with the LDS-DMA prefetch issued after
// them, which the compiler does not count) would drain the prefetch every tile.
// PRE: the side inputs were DMA'd to LDS by the kernel (pre: [NIT][NT] 16-B add_src chunks, then [NIT][NT]
// act_x chunks, slot = thread; pre_ss: the block's act scale / shift [2][CT]) - no global loads here, so no
// compiler-generated vmcnt waits (add_stride 1, no mask / act_r).
// aacc (persistent kernels, with SACC): the activation-backward sums [sum g*x | sum g | sum g*r] of this
// thread's chunk column are added into aacc[24] across all the block's tiles (one partial row per worker at the
// kernel's end, worker_row) instead of a per-tile LDS reduction + row.
// SPL: the merged-sibling split store (ConvNTArgs::split) - a separate instantiation, so the kernels without it
// carry no per-chunk branch or split-table kernel arguments in their store loop (measured +3.6 % ResNet-50 step
// when it was a runtime branch in every kernel: profiles/r4/README.md).
template <int PT, int CT, bool RAWB, bool EXACT, bool SACC, int NT, bool SIDE = true, bool PRE = false, bool SPL = false,
          int EG = 4>
__device__ __forceinline__ void conv_nt_epi_tail(const ConvNTArgs& a, char* smem, int p0, int c0, int by,
                                                 float* ssum, float* ssq, const char* pre = nullptr,
                                                 const float* pre_ss = nullptr, float* aacc = nullptr) {
  constexpr int OROW = CT * 2 + 16;
  const int tid = threadIdx.x;
  epi_barrier<RAWB>();
  constexpr int CPR = CT / 8;  // 16-B chunks per pixel row of the tile
  constexpr int NIT = PT * CPR / NT;
  static_assert(NT % CPR == 0 && (PT * CPR) % NT == 0, "staged-store mapping");
  const int chn = tid % CPR;   // fixed per thread (NT % CPR == 0)
  const int kc = c0 + chn * 8;
  const bool act = SIDE && a.act_x != nullptr;
  // BatchNorm statistics of a staged tile: each thread sums its fixed 8-channel chunk column over its
  // rows (bf16-rounded outputs) and the block reduces them once through LDS below -> ONE partial row
  // per pixel tile, no per-subtile shuffle trees (those cost up to +100 % on the wide-K 1x1 layers)
  const bool bstats = !SACC && a.stats != nullptr;
  float sc[8], sh[8], sgx[8], sg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = 1.f; sh[e] = 0.f; sgx[e] = 0.f; sg[e] = 0.f; }
  const bool amask = act && a.act_mask != nullptr;
  float sgr[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sgr[e] = 0.f;
  if (act && !amask && kc < a.K) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = PRE ? pre_ss[chn * 8 + e] : a.act_ss[kc + e];
      sh[e] = PRE ? pre_ss[CT + chn * 8 + e] : a.act_ss[a.K + kc + e];
    }
  }
  // side inputs of the dgrad post-ops (add_src, act_x, act_r, mask bytes) are loaded for a group of
  // GRP rows before any of them is used, so their latencies overlap instead of serialising per row
  constexpr int GRP = NIT < EG ? NIT : EG;  // (EG: rows whose side inputs are in flight together - registers)
  static_assert(NIT % GRP == 0, "epilogue row groups");
  const bool side = SIDE && (a.add_src != nullptr || act);
#pragma unroll
  for (int g0 = 0; g0 < NIT; g0 += GRP) {
    uint4 pa[GRP], px[GRP], pr[GRP];
    uint32_t pm[GRP];
    bool ph[GRP];
#pragma unroll
    for (int j = 0; j < GRP; ++j) {
      pa[j] = px[j] = pr[j] = make_uint4(0, 0, 0, 0);
      pm[j] = 0u;
      ph[j] = false;
    }
    if (PRE && side) {
#pragma unroll
      for (int j = 0; j < GRP; ++j) {
        if (a.add_src) {
          pa[j] = *(const uint4*)(pre + (size_t)(g0 + j) * NT * 16 + tid * 16);
          ph[j] = true;
        }
        if (act) px[j] = *(const uint4*)(pre + (size_t)(NIT + g0 + j) * NT * 16 + tid * 16);
      }
    } else if (side) {
#pragma unroll
      for (int j = 0; j < GRP; ++j) {
        const int row = ((g0 + j) * NT + tid) / CPR;
        const int m = p0 + row;
        if (m < a.M && kc < a.K && out_valid(a, m)) {
          const size_t o = (size_t)out_row(a, m) * a.K + kc;
          if (a.add_src) {
            const bf16_t* src = a.add_src + o;
            if (a.add_stride > 1) {
              int n, h, w;
              out_nhw(a, m, n, h, w);
              const int s = a.add_stride;
              src = (h % s == 0 && w % s == 0)
                        ? a.add_src + ((size_t)(n * a.add_H + h / s) * a.add_W + w / s) * a.K + kc
                        : nullptr;
            }
            if (src) {
              pa[j] = *(const uint4*)src;
              ph[j] = true;
            }
          }
          if (act) {
            px[j] = *(const uint4*)(a.act_x + o);
            if (amask) {
              pm[j] = a.act_mask[o >> 3];
              if (a.act_r) pr[j] = *(const uint4*)(a.act_r + o);
            }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < GRP; ++j) {
      const int idx = (g0 + j) * NT + tid;
      const int row = idx / CPR;
      const int m = p0 + row;
      const bool inb = m < a.M && kc < a.K && out_valid(a, m);
      if (EXACT || inb) {
        uint4 v = *(const uint4*)(smem + row * OROW + chn * 16);
        const size_t o = (size_t)(inb ? out_row(a, m) : m) * a.K + kc;
        if constexpr (SACC) {
          if (inb) {
            const float q[8] = {lo_bf(v.x), hi_bf(v.x), lo_bf(v.y), hi_bf(v.y),
                                lo_bf(v.z), hi_bf(v.z), lo_bf(v.w), hi_bf(v.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) { ssum[e] += q[e]; ssq[e] = fmaf(q[e], q[e], ssq[e]); }
          }
        } else {
          if (bstats && inb) {  // (sgx / sg double as the statistics accumulators: act is off here)
            const float q[8] = {lo_bf(v.x), hi_bf(v.x), lo_bf(v.y), hi_bf(v.y),
                                lo_bf(v.z), hi_bf(v.z), lo_bf(v.w), hi_bf(v.w)};
#pragma unroll
            for (int e = 0; e < 8; ++e) { sgx[e] += q[e]; sg[e] = fmaf(q[e], q[e], sg[e]); }
          }
        }
        if (inb && side) {
          float f[8];
          f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
          f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
          if (ph[j]) {
            const uint4 r = pa[j];
            f[0] += lo_bf(r.x); f[1] += hi_bf(r.x); f[2] += lo_bf(r.y); f[3] += hi_bf(r.y);
            f[4] += lo_bf(r.z); f[5] += hi_bf(r.z); f[6] += lo_bf(r.w); f[7] += hi_bf(r.w);
          }
          if (act) {
            const uint4 xu = px[j];
            float xv[8];
            xv[0] = lo_bf(xu.x); xv[1] = hi_bf(xu.x); xv[2] = lo_bf(xu.y); xv[3] = hi_bf(xu.y);
            xv[4] = lo_bf(xu.z); xv[5] = hi_bf(xu.z); xv[6] = lo_bf(xu.w); xv[7] = hi_bf(xu.w);
            if (amask) {
              // block-output form: g = d(out) * bit, sums against the raw conv output (and the raw
              // BN'd residual); out <- g (the producers' conv+BN backwards apply their scales)
              const uint32_t mb = pm[j];
              const uint4 ru = pr[j];
              const float rv[8] = {lo_bf(ru.x), hi_bf(ru.x), lo_bf(ru.y), hi_bf(ru.y),
                                   lo_bf(ru.z), hi_bf(ru.z), lo_bf(ru.w), hi_bf(ru.w)};
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float g = (mb >> e) & 1u ? f[e] : 0.f;
                sgx[e] += g * xv[e];
                sg[e] += g;
                sgr[e] += g * rv[e];  // (rv = 0 without a BN'd residual)
                f[e] = g;
              }
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float g = fmaf(xv[e], sc[e], sh[e]) > 0.f ? f[e] : 0.f;
                sgx[e] += g * xv[e];
                sg[e] += g;
                f[e] = a.act_unscaled ? g : g * sc[e];
              }
            }
          }
          v = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
        }
        if constexpr (SPL) {  // (merged siblings: each member's own output tensor; constant indices, no scratch)
          int off = a.split[0].off, kk = a.split[0].K;
          bf16_t* yb = a.split[0].y;
#pragma unroll
          for (int q = 1; q < 8; ++q)
            if (q < a.nsplit && kc >= a.split[q].off) { yb = a.split[q].y; off = a.split[q].off; kk = a.split[q].K; }
          *(uint4*)(inb ? yb + (size_t)out_row(a, m) * kk + (kc - off) : a.dump) = v;
        } else {
          *(uint4*)(inb ? a.y + o : a.dump) = v;
        }
      }
    }
  }
  if (act && aacc) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { aacc[e] += sgx[e]; aacc[8 + e] += sg[e]; aacc[16 + e] += sgr[e]; }
  } else if (act || bstats) {
    // reduce the per-thread partial sums over the threads sharing this chunk column, one partial
    // row per pixel tile (reduced over tiles by dtm_reduce_rows / stats_reduce_finalize)
    epi_barrier<RAWB>();
    float* red = (float*)smem;  // [NT][16]
#pragma unroll
    for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sgx[e]; red[tid * 16 + 8 + e] = sg[e]; }
    epi_barrier<RAWB>();
    // every thread finishes one (chunk column, value) output: NT/CPR partials each, instead of CPR
    // threads walking all NT rows of the table serially
    const int rw = (act && a.act_r) ? 4 : 2;  // row width in K units
    float* prow = (act ? a.act_sums : a.stats) + (size_t)by * (rw * a.K);
    for (int o = tid; o < CPR * 16; o += NT) {
      const int c = o >> 4, e = o & 15;
      float t = 0.f;
#pragma unroll 4
      for (int k = 0; k < NT / CPR; ++k) t += red[((c + k * CPR) << 4) + e];
      const int kk = c0 + c * 8 + (e & 7);
      if (kk < a.K) prow[(e < 8 ? 0 : a.K) + kk] = t;
    }
    if (act && a.act_r) {  // second round: [sum g*r | sum g] of the BN'd residual
      epi_barrier<RAWB>();
#pragma unroll
      for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sgr[e]; red[tid * 16 + 8 + e] = sg[e]; }
      epi_barrier<RAWB>();
      for (int o = tid; o < CPR * 16; o += NT) {
        const int c = o >> 4, e = o & 15;
        float t = 0.f;
#pragma unroll 4
        for (int k = 0; k < NT / CPR; ++k) t += red[((c + k * CPR) << 4) + e];
        const int kk = c0 + c * 8 + (e & 7);
        if (kk < a.K) prow[2 * a.K + (e < 8 ? 0 : a.K) + kk] = t;
      }
    }
  }
}

template <int PT, int CT, int WP, int WC, int STG, bool RAWB = false, bool EXACT = false, bool NOBIAS = false,
          bool SACC = false, int NT = 256, bool SIDE = true, bool PRE = false, bool SPL = false, int EG = 4>
__device__ __forceinline__ void conv_nt_epilogue(const ConvNTArgs& a, f32x4 (&acc)[WC / 16][WP / 16], char* smem,
                                                 int p0, int c0, int by, float* ssum = nullptr,
                                                 float* ssq = nullptr, const char* pre = nullptr,
                                                 const float* pre_ss = nullptr, float* aacc = nullptr) {
  constexpr int NWP = PT / WP;
  constexpr int TP = WP / 16, TC = WC / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave % NWP, wc = wave / NWP;
  const int fr = lane & 15, fk = lane >> 4;
  // epilogue: lane holds channels (fk*4 .. +3) of pixel fr for every subtile.  Bias/ReLU and the
  // BatchNorm statistics (from the bf16-rounded outputs) are done in registers; the tile is then
  // staged through LDS (padded rows: conflict-free 8-B lane writes) so that every global store is a
  // full 16-B chunk and consecutive lanes cover whole NHWC pixel rows (coalesced, 256-B rows for
  // CT = 128) instead of 16 scattered 32-B pieces per wave instruction.
  constexpr int OROW = CT * 2 + 16;
  constexpr bool staged = STG == 1;
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const int kloc = wc * WC + i * 16 + fk * 4;
    const int kch = c0 + kloc;
    float bsum[4] = {0.f, 0.f, 0.f, 0.f}, bsq[4] = {0.f, 0.f, 0.f, 0.f};
    float bia[4] = {0.f, 0.f, 0.f, 0.f};
    if (!NOBIAS && a.bias && kch < a.K) {  // (NOBIAS: no global load whose wait would drain a prefetch)
#pragma unroll
      for (int r = 0; r < 4; ++r) bia[r] = a.bias[kch + r];
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int mloc = wp * WP + j * 16 + fr;
      const int m = p0 + mloc;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bia[r];
        if (!NOBIAS && a.relu) v[r] = fmaxf(v[r], 0.f);
      }
      uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
      if constexpr (staged) {
        *(uint2*)(smem + mloc * OROW + kloc * 2) = make_uint2(lo, hi);
      } else if (m < a.M && kch < a.K && out_valid(a, m)) {
        *(uint2*)(a.y + (size_t)out_row(a, m) * a.K + kch) = make_uint2(lo, hi);
      }
      if (!SACC && !staged && a.stats && m < a.M && kch < a.K && out_valid(a, m)) {
        float q0 = lo_bf(lo), q1 = hi_bf(lo), q2 = lo_bf(hi), q3 = hi_bf(hi);
        bsum[0] += q0; bsq[0] += q0 * q0;
        bsum[1] += q1; bsq[1] += q1 * q1;
        bsum[2] += q2; bsq[2] += q2 * q2;
        bsum[3] += q3; bsq[3] += q3 * q3;
      }
    }
    if (!SACC && !staged && a.stats) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          bsum[r] += __shfl_xor(bsum[r], o, 64);
          bsq[r] += __shfl_xor(bsq[r], o, 64);
        }
      }
      // one partial row per (pixel tile, pixel wave): [sum(K) | sumsq(K)], reduced by reduce_rows
      if (fr == 0 && kch < a.K) {
        float* row = a.stats + (size_t)(by * NWP + wp) * (2 * a.K);
        *(float4*)(row + kch) = make_float4(bsum[0], bsum[1], bsum[2], bsum[3]);
        *(float4*)(row + a.K + kch) = make_float4(bsq[0], bsq[1], bsq[2], bsq[3]);
      }
    }
  }
  if constexpr (staged)
    conv_nt_epi_tail<PT, CT, RAWB, EXACT, SACC, NT, SIDE, PRE, SPL, EG>(a, smem, p0, c0, by, ssum, ssq, pre, pre_ss,
                                                                        aacc);
}

// LBW: minimum waves per SIMD the register allocation must allow (__launch_bounds__; 0 = none), EG: epilogue side-input
// row group - the occupancy variants of the register-staged dgrads with post-ops (A/B knob dtm_conv_set_act_occ)
template <int PT, int CT, int WP, int WC, int UD, int NBUF, bool SPL = false, int LBW = 0, int EG = 4>
__global__ __launch_bounds__(256, LBW > 0 ? LBW : 1) void conv_nt_kernel(ConvNTArgs a) {
  constexpr int BK = 64;
  constexpr int NWP = PT / WP;
  constexpr int NWC = CT / WC;
  static_assert(NWP * NWC == 4, "4 waves");
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int ACH = PT / 32;  // act chunks per thread (PT rows * 8 chunks / 256 threads)
  constexpr int WCH = CT / 32;
  constexpr int BUF = (PT + CT) * 128;
  constexpr int MAXC = 512;  // prologue scale/shift staged in LDS for C <= MAXC (bottleneck widths)
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + MAXC * 8];
  float* s_scale = (float*)(smem + NBUF * BUF);
  float* s_shift = s_scale + MAXC;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wp = wave % NWP, wc = wave / NWP;
  const int tile = grp_tile(a);
  const int bx = tile % gridDim.x, by = tile / gridDim.x;
  const int p0 = by * PT, c0 = bx * CT;
  const int ch = tid & 7, rb = tid >> 3;
  const bool lds_ss = a.in_scale && a.C <= MAXC;
  if (lds_ss) {
    for (int c = tid; c < a.C; c += 256) { s_scale[c] = a.in_scale[c]; s_shift[c] = a.in_shift[c]; }
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  // per-row pixel decode (rows rb + 32*i of the pixel tile)
  int ih0[ACH], iw0[ACH], pixbase[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    int m = p0 + rb + 32 * i;
    if (m < a.M) {
      uint32_t n = fdiv((uint32_t)m, a.fd_PQ);
      uint32_t rem = m - n * (a.P * a.Q);
      uint32_t p = fdiv(rem, a.fd_Q);
      uint32_t q = rem - p * a.Q;
      ih0[i] = (int)p * a.stride - a.pad_h;
      iw0[i] = (int)q * a.stride - a.pad_w;
      pixbase[i] = (int)n * a.Hin * a.Win;
    } else {
      ih0[i] = -(1 << 28);
      iw0[i] = -(1 << 28);
      pixbase[i] = 0;
    }
  }
  // decode of this thread's k chunk for tile 0; advanced incrementally by 64 per tile
  int kc = ch * 8;
  int cc = kc % a.C;
  int tap = kc / a.C;
  int rr = tap / a.S, ss = tap - (tap / a.S) * a.S;

  // one register stage of the operand pipeline (a 2-deep register prefetch was measured: it spills
  // at 128x128 and is 20-60 % slower at 128x64 from the lost occupancy)
  struct Stage {
    uint4 a[ACH], w[WCH];
    bool v[ACH];
    int c;  // channel of this stage's activation chunk (for the prologue affine)
  };

  auto gload = [&](int kt, Stage& st) {
    const int k = kt * BK + ch * 8;
    const bool kin = (k < a.Kg);
    st.c = cc;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int ihv = ih0[i] + rr, iwv = iw0[i] + ss;
      bool v = kin && ihv >= 0 && ihv < a.Hv && iwv >= 0 && iwv < a.Wv;
      if (UD > 1) v = v && ((ihv % UD) == 0) && ((iwv % UD) == 0);
      int ih = UD > 1 ? ihv / UD : ihv, iw = UD > 1 ? iwv / UD : iwv;
      uint32_t off = v ? (uint32_t)((pixbase[i] + ih * a.Win + iw) * a.pix_bytes + cc * 2) : OOB_OFFSET;
      st.v[i] = v;
      st.a[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      int row = c0 + rb + 32 * i;
      bool v = kin && row < a.K;
      uint32_t off = v ? (uint32_t)((row * a.Kg + k) * 2) : OOB_OFFSET;
      st.w[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
    }
    // advance (rr, ss, cc) by BK
    cc += BK;
    while (cc >= a.C) {
      cc -= a.C;
      if (++ss == a.S) { ss = 0; ++rr; }
    }
  };

  auto swrite = [&](int buf, Stage& st) {
    char* base = smem + buf * BUF;
    if (a.in_scale) {
      // fused BatchNorm-apply + ReLU of the previous layer on the gathered input
      float sc[8], sh[8];
      if (lds_ss) {
        const float4 s0 = *(const float4*)(s_scale + st.c), s1 = *(const float4*)(s_scale + st.c + 4);
        const float4 h0 = *(const float4*)(s_shift + st.c), h1 = *(const float4*)(s_shift + st.c + 4);
        sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
        sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
      } else {
        for (int e = 0; e < 8; ++e) { sc[e] = a.in_scale[st.c + e]; sh[e] = a.in_shift[st.c + e]; }
      }
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        if (st.v[i]) {
          uint32_t u[4] = {st.a[i].x, st.a[i].y, st.a[i].z, st.a[i].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float lo = fmaxf(fmaf(lo_bf(u[e]), sc[2 * e], sh[2 * e]), 0.f);
            float hi = fmaxf(fmaf(hi_bf(u[e]), sc[2 * e + 1], sh[2 * e + 1]), 0.f);
            u[e] = pack2bf(lo, hi);
          }
          st.a[i] = make_uint4(u[0], u[1], u[2], u[3]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int row = rb + 32 * i;
      *(uint4*)(base + row * 128 + ((ch ^ (row & 7)) << 4)) = st.a[i];
    }
#pragma unroll
    for (int i = 0; i < WCH; ++i) {
      int row = rb + 32 * i;
      *(uint4*)(base + PT * 128 + row * 128 + ((ch ^ (row & 7)) << 4)) = st.w[i];
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  auto compute = [&](int cur) {
    const char* base = smem + cur * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      short8 bf[TP], af[TC];
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        int row = wp * WP + j * 16 + fr;
        int chn = ks * 4 + fk;
        bf[j] = *(const short8*)(base + row * 128 + ((chn ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        int row = wc * WC + i * 16 + fr;
        int chn = ks * 4 + fk;
        af[i] = *(const short8*)(base + PT * 128 + row * 128 + ((chn ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = (a.Kg + BK - 1) / BK;
  Stage st;
  gload(0, st);
  swrite(0, st);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (NBUF == 2) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt + 1, st);
      compute(cur);
      if (kt + 1 < nk) swrite(cur ^ 1, st);
      __syncthreads();
    } else {
      // single LDS buffer (less LDS -> more resident blocks for short-K layers): the next tile's
      // global loads still overlap the MFMAs; the LDS write waits for every wave's reads
      if (kt + 1 < nk) gload(kt + 1, st);
      compute(0);
      __syncthreads();
      if (kt + 1 < nk) {
        swrite(0, st);
        __syncthreads();
      }
    }
  }

  static_assert(PT * (CT * 2 + 16) <= NBUF * BUF, "output staging fits in the operand buffers");
  if ((a.K & 7) == 0)
    conv_nt_epilogue<PT, CT, WP, WC, 1, false, false, false, false, 256, true, false, SPL, EG>(a, acc, smem, p0, c0,
                                                                                             by);
  else conv_nt_epilogue<PT, CT, WP, WC, 2>(a, acc, smem, p0, c0, by);
}


// Deep-K pipelined variant: both operand tiles go global -> LDS by LDS-DMA into an NS-slot ring with
// ONE raw s_barrier per k-tile and a counted vmcnt, so NS-2 k-tiles stay in flight across the
// barrier (an LDS-DMA is a pending write on the vector-memory counter: __syncthreads() would drain it).
// Waves 2x2, each (PT/2) x (CT/2).  With the prologue (BatchNorm-apply + ReLU of the previous layer)
// each lane transforms the chunks it DMA'd itself, in LDS, after its own vmcnt wait and before the
// barrier that publishes the stage; padding / out-of-range chunks (from the zero buffer) are left at
// zero, their validity recomputed from a lagging copy of the k iterator.  All LDS is ONE __shared__
// array (a second object makes hipcc drain vmcnt before the fragment reads).
// NWP: waves along the pixel dimension (4 / NWP along channels); NWP = 4 with PT = 512, CT = 64 gives every
// wave a 128 x 64 tile (the 64-channel 3x3 layers: 2x the MFMAs per LDS byte of the 2x2 layout's 64x32)
//
// (An ACTL form - the act dgrads' act_x tile LDS-DMA'd under the last k-tile, read by the epilogue from LDS - was
// neutral at step level, profiles/ab/r4_ab_sside_alds.log, and was removed.)
template <int PT, int CT, int NS, int UD, bool PRO, int NWP = 2, bool SPL = false>
__global__ __launch_bounds__(256) void conv_nt_pipe_kernel(ConvNTArgs a) {
  constexpr int BK = 64;
  constexpr int WP = PT / NWP, WC = CT / (4 / NWP);
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int AI = PT / 32, WI = CT / 32;  // 8-row DMA groups per wave per k-tile
  constexpr int G = AI + WI;                 // DMA instructions per wave per k-tile
  constexpr int BUF = (PT + CT) * 128;
  constexpr int OROW = CT * 2 + 16;
  constexpr int MAXC = 512;
  constexpr int RING = NS * BUF > PT * OROW ? NS * BUF : PT * OROW;
  __shared__ __attribute__((aligned(16))) char smem[RING + (PRO ? MAXC * 8 : 0)];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  static_assert(G <= 31 && NS >= 2 && NS <= 4, "vmcnt range");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = grp_tile(a);
  const int bx = tile % gridDim.x, by = tile / gridDim.x;
  const int p0 = by * PT, c0 = bx * CT;
  const int lr = lane >> 3;
  const int ch = (lane & 7) ^ lr;  // logical 16-B chunk this lane moves (source-side swizzle)
  float* s_scale = (float*)(smem + RING);
  float* s_shift = s_scale + MAXC;
  if constexpr (PRO) {
    for (int c = tid; c < a.C; c += 256) { s_scale[c] = a.in_scale[c]; s_shift[c] = a.in_shift[c]; }
    __syncthreads();
  }

  int ih0[AI], iw0[AI], pixbase[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = p0 + 8 * (wave + 4 * j) + lr;
    if (m < a.M) {
      uint32_t n = fdiv((uint32_t)m, a.fd_PQ);
      uint32_t rem = m - n * (a.P * a.Q);
      uint32_t p = fdiv(rem, a.fd_Q);
      uint32_t q = rem - p * a.Q;
      ih0[j] = (int)p * a.stride - a.pad_h;
      iw0[j] = (int)q * a.stride - a.pad_w;
      pixbase[j] = (int)n * a.Hin * a.Win;
    } else {
      ih0[j] = -(1 << 28);
      iw0[j] = -(1 << 28);
      pixbase[j] = 0;
    }
  }
  // issue-side k iterator of this lane's chunk, and (prologue) the lagging transform-side copy
  int cc = (ch * 8) % a.C, tap = (ch * 8) / a.C;
  int rr = tap / a.S, ss = tap - (tap / a.S) * a.S;
  int tcc = cc, trr = rr, tss = ss;
  const char* xg = (const char*)a.x;
  const char* wg = (const char*)a.w;
  const char* zg = (const char*)a.zero;

  // branch-free validity (bitwise &, unsigned range checks): hipcc turns && chains around the
  // DMA into exec-masked branches
  auto valid_at = [&](int j, int r, int s, int& ih, int& iw) -> bool {
    const int ihv = ih0[j] + r, iwv = iw0[j] + s;
    bool v = ((unsigned)ihv < (unsigned)a.Hv) & ((unsigned)iwv < (unsigned)a.Wv);
    if (UD > 1) v = v & (((ihv | iwv) & (UD - 1)) == 0);
    ih = UD > 1 ? ihv / UD : ihv;
    iw = UD > 1 ? iwv / UD : iwv;
    return v;
  };

  auto issue = [&](int kt, int slot) {
    char* base = smem + slot * BUF;
    const int k = kt * BK + ch * 8;
    const bool kin = k < a.Kg;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      int ih, iw;
      const bool v = kin & valid_at(j, rr, ss, ih, iw);
      const char* src = xg + (size_t)(uint32_t)((pixbase[j] + ih * a.Win + iw) * a.pix_bytes + cc * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + 4 * j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int row = c0 + 8 * (wave + 4 * j) + lr;
      const bool v = kin & (row < a.K);
      const char* src = wg + (size_t)(uint32_t)((row * a.Kg + k) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + PT * 128 + (wave + 4 * j) * 1024), 16,
                                       0, 0);
    }
    cc += BK;
    while (cc >= a.C) {
      cc -= a.C;
      if (++ss == a.S) { ss = 0; ++rr; }
    }
  };

  auto transform = [&](int kt, int slot) {
    char* base = smem + slot * BUF;
    const bool kin = kt * BK + ch * 8 < a.Kg;
    if (kin) {
      const float4 s0 = *(const float4*)(s_scale + tcc), s1 = *(const float4*)(s_scale + tcc + 4);
      const float4 h0 = *(const float4*)(s_shift + tcc), h1 = *(const float4*)(s_shift + tcc + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        int ih, iw;
        if (valid_at(j, trr, tss, ih, iw)) {
          uint4* p = (uint4*)(base + (wave + 4 * j) * 1024 + lane * 16);
          const uint4 q = *p;
          uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = fmaxf(fmaf(lo_bf(u[e]), sc[2 * e], sh[2 * e]), 0.f);
            const float hi = fmaxf(fmaf(hi_bf(u[e]), sc[2 * e + 1], sh[2 * e + 1]), 0.f);
            u[e] = pack2bf(lo, hi);
          }
          *p = make_uint4(u[0], u[1], u[2], u[3]);
        }
      }
    }
    tcc += BK;
    while (tcc >= a.C) {
      tcc -= a.C;
      if (++tss == a.S) { tss = 0; ++trr; }
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int wp = wave % NWP, wc = wave / NWP;
  const int fr = lane & 15, fk = lane >> 4;
  auto compute = [&](int slot) {
    const char* base = smem + slot * BUF;
    // all 2 x (TP + TC) fragment reads of the k-tile first: the ks = 1 reads are in flight under the
    // ks = 0 MFMAs (counted lgkmcnt) instead of a full LDS round trip between the two halves
    short8 bf[2][TP], af[2][TC];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chn = ks * 4 + fk;
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int row = wp * WP + j * 16 + fr;
        bf[ks][j] = *(const short8*)(base + row * 128 + ((chn ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int row = wc * WC + i * 16 + fr;
        af[ks][i] = *(const short8*)(base + PT * 128 + row * 128 + ((chn ^ (row & 7)) << 4));
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
  };

  const int nk = (a.Kg + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's DMA of k-tile kt has landed once at most the later stages are still counted
    const int ahead = min(nk - 1, kt + NS - 2) - kt;
    if (NS >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G) : "memory");
    else if (NS >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (PRO) transform(kt, slot);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt visible to all waves; stage kt-1 no longer read
    if (kt + NS - 1 < nk) issue(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
    compute(slot);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the ring
  if ((a.K & 7) == 0)
    conv_nt_epilogue<PT, CT, WP, WC, 1, false, false, false, false, 256, true, false, SPL>(a, acc, smem, p0, c0, by);
  else conv_nt_epilogue<PT, CT, WP, WC, 2>(a, acc, smem, p0, c0, by);
}

// 8-wave big-tile variant of the pipelined kernel: PT = 256 pixels x CT (128 | 256) channels per
// 512-thread block, waves NWP (pixels) x 8/NWP (channels), each wave a (PT/NWP) x (CT*NWP/8) tile of
// 16x16x32 MFMAs.  Why a bigger tile: the 4-wave 128x128 block (2 per CU) pulls one 32 KiB operand
// k-tile from L2 per 128 MFMAs, i.e. ~64 B/clk/CU at the MFMA rate - more than the L2 delivers
// (MI355X_MICROARCH: ~34.5 TB/s chip-wide); a 256x256 block halves the L2 bytes per MFMA (256x128: 0.75x).
// Same LDS image / source-side swizzle / counted-vmcnt ring as conv_nt_pipe_kernel (no input prologue);
// one 8-row x 128-B LDS-DMA group per wave-instruction, AI + WI of them per wave per k-tile.
// (32x32x16-MFMA forms of these tiles measured +0.6 % ResNet-50 step - LDS / DMA bound, not MFMA-issue bound -
// and were removed: profiles/ab/r3_ab_mfma32_step.log)
// (NTH = 256 builds the 4-wave form - waves 2x2 of 128x128, 64 accumulator tiles per wave, 1 wave per SIMD: half the
// LDS fragment reads per MFMA.  It measured 40 % slower per conv and 10-15 % per weight gradient (the 4-wave
// wgrad_pipe <256, 256, 2, 2, 256>), ResNet-50 step +11 %: one wave per SIMD cannot cover the LDS / DMA latency
// (profiles/r6/r6_s27_sweep_w4.log, r6_s27_ab_w4.log); not wired into the policy.)
template <int PT, int CT, int NWP, int NS, int UD, bool SPL = false, int NTH = 512>
__global__ __launch_bounds__(NTH) void conv_nt_w8_kernel(ConvNTArgs a) {
  constexpr int NT = NTH, NW = NTH / 64;
  constexpr int BK = 64;
  constexpr int NWC = NW / NWP;
  constexpr int WP = PT / NWP, WC = CT / NWC;
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int AI = PT / (8 * NW), WI = CT / (8 * NW);  // 8-row DMA groups per wave per k-tile
  constexpr int G = AI + WI;                 // DMA instructions per wave per k-tile
  constexpr int BUF = (PT + CT) * 128;
  constexpr int OROW = CT * 2 + 16;
  constexpr int RING = NS * BUF > PT * OROW ? NS * BUF : PT * OROW;
  static_assert(RING <= 160 * 1024, "LDS budget");
  static_assert(G <= 31 && NS >= 2 && NS <= 3, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[RING];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = grp_tile(a);
  const int bx = tile % gridDim.x, by = tile / gridDim.x;
  const int p0 = by * PT, c0 = bx * CT;
  const int lr = lane >> 3;
  const int ch = (lane & 7) ^ lr;  // logical 16-B chunk this lane moves (source-side swizzle)

  int ih0[AI], iw0[AI], pixbase[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = p0 + 8 * (wave + NW * j) + lr;
    if (m < a.M) {
      uint32_t n = fdiv((uint32_t)m, a.fd_PQ);
      uint32_t rem = m - n * (a.P * a.Q);
      uint32_t p = fdiv(rem, a.fd_Q);
      uint32_t q = rem - p * a.Q;
      ih0[j] = (int)p * a.stride - a.pad_h;
      iw0[j] = (int)q * a.stride - a.pad_w;
      pixbase[j] = (int)n * a.Hin * a.Win;
    } else {
      ih0[j] = -(1 << 28);
      iw0[j] = -(1 << 28);
      pixbase[j] = 0;
    }
  }
  int cc = (ch * 8) % a.C, tap = (ch * 8) / a.C;
  int rr = tap / a.S, ss = tap - (tap / a.S) * a.S;
  const char* xg = (const char*)a.x;
  const char* wg = (const char*)a.w;
  const char* zg = (const char*)a.zero;

  auto issue = [&](int kt, int slot) {
    char* base = smem + slot * BUF;
    const int k = kt * BK + ch * 8;
    const bool kin = k < a.Kg;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int ihv = ih0[j] + rr, iwv = iw0[j] + ss;
      bool v = kin & ((unsigned)ihv < (unsigned)a.Hv) & ((unsigned)iwv < (unsigned)a.Wv);
      if (UD > 1) v = v & (((ihv | iwv) & (UD - 1)) == 0);
      const int ih = UD > 1 ? ihv / UD : ihv, iw = UD > 1 ? iwv / UD : iwv;
      const char* src = xg + (size_t)(uint32_t)((pixbase[j] + ih * a.Win + iw) * a.pix_bytes + cc * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int row = c0 + 8 * (wave + NW * j) + lr;
      const bool v = kin & (row < a.K);
      const char* src = wg + (size_t)(uint32_t)((row * a.Kg + k) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + PT * 128 + (wave + NW * j) * 1024),
                                       16, 0, 0);
    }
    cc += BK;
    while (cc >= a.C) {
      cc -= a.C;
      if (++ss == a.S) { ss = 0; ++rr; }
    }
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int wp = wave % NWP, wc = wave / NWP;
  const int fr = lane & 15, fk = lane >> 4;
  auto compute = [&](int slot) {
    const char* base = smem + slot * BUF;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chn = ks * 4 + fk;
      short8 bf[TP], af[TC];
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int row = wp * WP + j * 16 + fr;
        bf[j] = *(const short8*)(base + row * 128 + ((chn ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int row = wc * WC + i * 16 + fr;
        af[i] = *(const short8*)(base + PT * 128 + row * 128 + ((chn ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = (a.Kg + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + NS - 2) - kt;
    if (NS >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt visible to all waves; stage kt-1 no longer read
    if (kt + NS - 1 < nk) issue(kt + NS - 1, slot == 0 ? NS - 1 : slot - 1);
    __builtin_amdgcn_s_setprio(1);
    compute(slot);
    __builtin_amdgcn_s_setprio(0);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the epilogue reuses the ring
  if ((a.K & 7) == 0)
    conv_nt_epilogue<PT, CT, WP, WC, 1, false, false, false, false, NT, true, false, SPL>(a, acc, smem, p0, c0, by);
  else conv_nt_epilogue<PT, CT, WP, WC, 2, false, false, false, false, NT>(a, acc, smem, p0, c0, by);
}

// 8-wave ping-pong ("8-phase") main loop of the 256 x 256 tiles (conv_nt_pp_kernel, conv_wgrad_pp_kernel): BK = 64,
// LDS-DMA operand staging, the k-loop split into 4 phases per k-tile, and the two wave groups (waves 0-3, 4-7: one
// wave of each on every SIMD) running one barrier apart, so on each SIMD one wave's 16 MFMAs overlap the other
// wave's LDS fragment reads and DMA issue (the w8 kernels: all 8 waves read, then all 8 multiply - the MFMA pipe
// idles during the read burst and the per-k-tile vmcnt(0) drain).
//   * k-tile slot = 4 half-tiles of 16 KiB: P0 / P1 (rows 0-127 / 128-255 of the operand whose rows are split over
//     the wave groups) and W0 / W1 (rows 0-127 / 128-255 of the other); 2 slots (128 KiB).  Wave (g = wave >> 2,
//     q = wave & 3) owns P rows {mi*128 + g*64 + 0..63} and W rows {ni*128 + q*32 + 0..31}, mi, ni in {0, 1}, so
//     the quadrant (ni, mi) of a phase reads ONE P half and ONE W half, and each half is consumed early in its
//     k-tile and restaged with k-tile t+2:
//       phase 0: read P(mi=0) + W(ni=0)      MFMA (0,0)   issue W1(t+1)
//       phase 1: read W(ni=1)                MFMA (1,0)   issue P1(t+1)
//       phase 2: read P(mi=1)                MFMA (1,1)   issue P0(t+2)
//       phase 3: (registers)                 MFMA (0,1)   issue W0(t+2)
//     (16 MFMAs of 16x16x32 per wave per phase.)
//   * every half is restaged >= 2 phases after its last read (the WAR distance two staggered groups need) and read
//     >= 1 phase after the vmcnt that retires it (RAW across the stagger); each phase waits with a counted vmcnt for
//     everything but the last 4 phases' DMAs (8 instructions in steady state, fewer in the tail, where the
//     past-the-end issues are skipped), so a half has ~8 barrier intervals to land.
//   * all LDS in ONE __shared__ array (the caller's), raw s_barrier, sched_barrier fences so the compiler keeps each
//     phase's reads / DMA / MFMAs on their side of the barriers.
// issue(kt, h): DMA of half h (0 W1, 1 P1, 2 P0, 3 W0) of k-tile kt into slot kt & 1 (2 LDS-DMA instructions per wave);
// rd_p(slot, mi) / rd_w(slot, ni): fragment reads; mma(ni, mi): the quadrant's 16 MFMAs.
template <class IssueF, class RdPF, class RdWF, class MmaF>
__device__ __forceinline__ void pp_mainloop(const char* smem, int slot_bytes, int nk, int grp, IssueF issue, RdPF rd_p,
                                            RdWF rd_w, MmaF mma) {
  // the DMA of global phase p (p = 4 t + q; the prologue is p = -6 .. -1): q 0 W1(t+1), 1 P1(t+1), 2 P0(t+2),
  // 3 W0(t+2); issued only for k-tiles < nk
  auto phase_kt = [&](int p) { return ((p + 8) >> 2) - 2 + ((p & 3) >= 2 ? 2 : 1); };
  auto issue_phase = [&](int p) {
    const int kt = phase_kt(p);
    if (kt < nk) issue(kt, p & 3);
  };
  // counted wait after phase p's issue: everything but the DMAs of phases p-3 .. p (2 per issuing phase)
  auto wait_phase = [&](int p) {
    int n = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) n += (p - d >= -6 && phase_kt(p - d) < nk) ? 2 : 0;
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // prologue: phases -6 .. -1 (k-tile 0 whole, P0 / W0 of k-tile 1), then wait for k-tile 0's P0 / W0
#pragma unroll
  for (int p = -6; p < 0; ++p) issue_phase(p);
  wait_phase(-1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  if (grp == 1) bar();  // the stagger: group 1 runs one barrier behind group 0
  for (int t = 0; t < nk; ++t) {
    const char* s = smem + (t & 1) * slot_bytes;
    const int pb = 4 * t;
    rd_w(s, 0);  // phase 0
    rd_p(s, 0);
    issue_phase(pb);
    wait_phase(pb);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    mma(0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    rd_w(s, 1);  // phase 1
    issue_phase(pb + 1);
    wait_phase(pb + 1);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    rd_p(s, 1);  // phase 2
    issue_phase(pb + 2);
    wait_phase(pb + 2);
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    mma(1, 1);
    __builtin_amdgcn_s_setprio(0);
    bar();
    issue_phase(pb + 3);  // phase 3
    wait_phase(pb + 3);
    bar();
    __builtin_amdgcn_s_setprio(1);
    mma(0, 1);
    __builtin_amdgcn_s_setprio(0);
    bar();
  }
  if (grp == 0) bar();  // match group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Ping-pong form of conv_nt_w8_kernel<256, 256>: the same GEMM (256 pixels x 256 channels per 512-thread block, the
// source-swizzled [row][128 B] LDS image), pixels as the P operand (A0 / A1), weight rows as W.  Epilogue: the shared
// staged-store tail (statistics, dgrad post-ops, split store) after a register -> LDS pass for this wave layout.
// No input prologue (like w8).
template <int UD, bool SPL = false>
__global__ __launch_bounds__(512) void conv_nt_pp_kernel(ConvNTArgs a) {
  constexpr int PT = 256, CT = 256, NW = 8, BK = 64;
  constexpr int HALF = 128 * 128;  // one half-tile: 128 rows x 64 k bf16
  constexpr int BUF = 4 * HALF;    // one k-tile slot [P0 | P1 | W0 | W1]
  constexpr int OROW = CT * 2 + 16;
  constexpr int RING = 2 * BUF > PT * OROW ? 2 * BUF : PT * OROW;
  static_assert(RING <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[RING];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave >> 2, wq = wave & 3;
  const int tile = grp_tile(a);
  const int bx = tile % gridDim.x, by = tile / gridDim.x;
  const int p0 = by * PT, c0 = bx * CT;
  const int lr = lane >> 3;
  const int ch = (lane & 7) ^ lr;  // logical 16-B chunk this lane moves (source-side swizzle)

  // pixel decode of this lane's 4 DMA rows 8 * (wave + 8 j) + lr (j = 0, 1: half P0; j = 2, 3: half P1)
  int ih0[4], iw0[4], pixbase[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = p0 + 8 * (wave + NW * j) + lr;
    if (m < a.M) {
      uint32_t n = fdiv((uint32_t)m, a.fd_PQ);
      uint32_t rem = m - n * (a.P * a.Q);
      uint32_t p = fdiv(rem, a.fd_Q);
      uint32_t q = rem - p * a.Q;
      ih0[j] = (int)p * a.stride - a.pad_h;
      iw0[j] = (int)q * a.stride - a.pad_w;
      pixbase[j] = (int)n * a.Hin * a.Win;
    } else {
      ih0[j] = -(1 << 28);
      iw0[j] = -(1 << 28);
      pixbase[j] = 0;
    }
  }
  // (r, s, c) iterators of this lane's chunk for the next P0 / P1 issue (the halves run a k-tile apart)
  int cc0 = (ch * 8) % a.C, rr0, ss0;
  {
    const int tap = (ch * 8) / a.C;
    rr0 = tap / a.S;
    ss0 = tap - rr0 * a.S;
  }
  int cc1 = cc0, rr1 = rr0, ss1 = ss0;
  const char* xg = (const char*)a.x;
  const char* wg = (const char*)a.w;
  const char* zg = (const char*)a.zero;
  const int nk = (a.Kg + BK - 1) / BK;

  auto issue_p = [&](int kt, int h, int& cc, int& rr, int& ss) {
    char* base = smem + (kt & 1) * BUF + h * HALF;
    const bool kin = kt * BK + ch * 8 < a.Kg;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = 2 * h + jj;
      const int ihv = ih0[j] + rr, iwv = iw0[j] + ss;
      bool v = kin & ((unsigned)ihv < (unsigned)a.Hv) & ((unsigned)iwv < (unsigned)a.Wv);
      if (UD > 1) v = v & (((ihv | iwv) & (UD - 1)) == 0);
      const int ih = UD > 1 ? ihv / UD : ihv, iw = UD > 1 ? iwv / UD : iwv;
      const char* src = xg + (size_t)(uint32_t)((pixbase[j] + ih * a.Win + iw) * a.pix_bytes + cc * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + NW * jj) * 1024), 16, 0, 0);
    }
    cc += BK;
    while (cc >= a.C) {
      cc -= a.C;
      if (++ss == a.S) { ss = 0; ++rr; }
    }
  };
  auto issue_w = [&](int kt, int h) {
    char* base = smem + (kt & 1) * BUF + (2 + h) * HALF;
    const int k = kt * BK + ch * 8;
    const bool kin = k < a.Kg;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = c0 + h * 128 + 8 * (wave + NW * jj) + lr;
      const bool v = kin & (row < a.K);
      const char* src = wg + (size_t)(uint32_t)((row * a.Kg + k) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + NW * jj) * 1024), 16, 0, 0);
    }
  };
  auto issue = [&](int kt, int h) {
    if (h == 0) issue_w(kt, 1);
    else if (h == 1) issue_p(kt, 1, cc1, rr1, ss1);
    else if (h == 2) issue_p(kt, 0, cc0, rr0, ss0);
    else issue_w(kt, 0);
  };

  f32x4 acc[2][2][2][4];  // [ni][ii][mi][jj]
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ni][ii][mi][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  short8 P[2][4], Wa[2][2], Wb[2][2];  // [ks][frag]
  auto rd_p = [&](const char* s, int mi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int row = mi * 128 + grp * 64 + jj * 16 + fr;
        P[ks][jj] = *(const short8*)(s + row * 128 + (((ks * 4 + fk) ^ (row & 7)) << 4));
      }
  };
  auto rd_w = [&](const char* s, int ni) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int row = ni * 128 + wq * 32 + ii * 16 + fr;
        const short8 v = *(const short8*)(s + 2 * HALF + row * 128 + (((ks * 4 + fk) ^ (row & 7)) << 4));
        if (ni == 0) Wa[ks][ii] = v;
        else Wb[ks][ii] = v;
      }
  };
  auto mma = [&](int ni, int mi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[ni][ii][mi][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ni == 0 ? Wa[ks][ii] : Wb[ks][ii], P[ks][jj],
                                                                        acc[ni][ii][mi][jj], 0, 0, 0);
  };
  pp_mainloop(smem, BUF, nk, grp, issue, rd_p, rd_w, mma);
  __syncthreads();  // the epilogue reuses the ring

  // register -> LDS staging of the bf16 tile (lane: channels fk*4 .. +3 of pixel fr per 16x16 subtile), then the
  // shared staged-store tail; bias / ReLU applied here like conv_nt_epilogue
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int kloc = ni * 128 + wq * 32 + ii * 16 + fk * 4;
      float bia[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.bias && c0 + kloc < a.K) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bia[r] = a.bias[c0 + kloc + r];
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int mloc = mi * 128 + grp * 64 + jj * 16 + fr;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[ni][ii][mi][jj][r] + bia[r];
            if (a.relu) v[r] = fmaxf(v[r], 0.f);
          }
          *(uint2*)(smem + mloc * OROW + kloc * 2) = make_uint2(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]));
        }
    }
  conv_nt_epi_tail<PT, CT, false, false, false, 512, true, false, SPL>(a, smem, p0, c0, by, nullptr, nullptr);
}

// Persistent streaming kernel for the short-reduction 1x1 stride-1 convs (K*R*S*C = 64 * NKT <= 256:
// the 56x56 / 28x28 expand and reduce layers and their dgrads).  They are pure HBM streams (read
// M x Kg, write M x K), so each block keeps its channel tile of the weights resident in LDS and walks
// pixel tiles p = y, y + gridDim.y, ...: the LDS-DMA of tile i+1 is issued before the MFMAs of tile i
// and stays in flight through tile i's epilogue (raw barriers; counted vmcnt with the epilogue's exact
// store count as the lower bound).  Optional BatchNorm-apply + ReLU prologue transformed in LDS.
// 16-B LDS-DMA issued through inline asm: hipcc does not see it as an LDS write, so it inserts none of
// its conservative vmcnt(0) waits before later LDS reads/writes (every use is ordered by this file's own
// counted vmcnt + barrier).  Its own waits for its own loads stay correct: the count is in issue order.
// One partial row per persistent worker: the 256 threads' per-chunk-column sums lo[8] / hi[8] (thread tid owns
// column tid % (CT/8)) are tree-reduced through red ([256][16] fp32 of free LDS) and written as
// row[c0 + c] = sum lo, row[K + c0 + c] = sum hi for this block's CT channels.
template <int CT>
__device__ __forceinline__ void worker_row(float* red, const float* lo, const float* hi, float* row, int c0, int K) {
  constexpr int CPR = CT / 8, RPT = 256 / CPR;
  const int tid = threadIdx.x;
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = lo[e]; red[tid * 16 + 8 + e] = hi[e]; }
  __syncthreads();
  for (int h = RPT / 2; h >= 1; h >>= 1) {
    if (tid < h * CPR) {
#pragma unroll
      for (int e = 0; e < 16; ++e) red[tid * 16 + e] += red[(tid + h * CPR) * 16 + e];
    }
    __syncthreads();
  }
  const int kc = c0 + tid * 8;
  if (tid < CPR && kc < K) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { row[kc + e] = red[tid * 16 + e]; row[K + kc + e] = red[tid * 16 + 8 + e]; }
  }
}

__device__ __forceinline__ void glds16(const void* gptr, const void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "s"(l) : "memory", "m0");
}

// STEM: the packed-row stem view (ConvDesc.pix_bytes = 8, C = 32 "channels" = 8 taps x 4 input channels,
// an R x 1 conv with stride): the A chunk of k for output pixel (n, p, q) is the 16 B at input row
// p*stride + k/32, column q*stride, byte (k % 32) * 2 of the zero-bordered [N][Hp][Wp][4] image -
// the 7x7/2 ResNet stem as a persistent stream with its 64 x 224 weights resident in LDS.  Its A tiles
// (28 KiB of L2-resident rows per 64 pixels) ride a 3-slot ring (NBUF = 3): two tiles in flight.
//
// (A form with the block-output dgrads' side inputs - add_src, x_raw, ReLU mask bytes, act_r - LDS-DMA'd one tile
// ahead was faster per kernel on the 28x28 stage but slower at step level: its 1-block/CU LDS footprint locks the
// side-stream weight gradients out of the CUs it holds; profiles/ab/r4_ab_sside_alds.log.  Removed.)
template <int PT, int CT, int NKT, bool PRO, bool STEM = false, int NBUF = 2, bool SIDE = true>
__global__ __launch_bounds__(256) void conv1x1_stream_kernel(ConvNTArgs a, int ntiles) {
  constexpr int WP = PT / 2, WC = CT / 2;
  constexpr int TP = WP / 16, TC = WC / 16;
  constexpr int AI = PT / 32, WI = CT / 32;      // 1-KiB DMA pieces per wave per 64-k sub-tile
  constexpr int ABUF = NKT * PT * 128;           // one pixel tile, all k
  constexpr int WBUF = NKT * CT * 128;
  constexpr int OROW = CT * 2 + 16;
  constexpr int STG = PT * OROW > 16384 ? PT * OROW : 16384;
  constexpr int NIT = PT * (CT / 8) / 256;      // exact staged stores per thread per tile
  constexpr int MAXC = 512;
  constexpr int OFF_A = WBUF, OFF_S = WBUF + NBUF * ABUF, OFF_P = OFF_S + STG;
  constexpr int NDMA = NKT * AI;                // DMA instructions per thread per tile
  static_assert(NBUF == 2 || NBUF == 3, "ring depth");
  static_assert(2 * NIT + NDMA <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[OFF_P + (PRO ? MAXC * 8 : 0)];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  static_assert(NIT >= 1 && NIT <= 15, "vmcnt lower bound");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = gridDim.x * gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nb);
  const int bx = bid % gridDim.x, by0 = bid / gridDim.x;
  const int c0 = bx * CT;
  const int lr = lane >> 3;
  const int ch = (lane & 7) ^ lr;
  const char* xg = (const char*)a.x;
  const char* wg = (const char*)a.w;
  const char* zg = (const char*)a.zero;
  float* s_scale = (float*)(smem + OFF_P);
  float* s_shift = s_scale + MAXC;
  if constexpr (PRO) {
    for (int c = tid; c < a.C; c += 256) { s_scale[c] = a.in_scale[c]; s_shift[c] = a.in_shift[c]; }
  }
  // resident weight tile: NKT sub-tiles [CT][64] (128-B rows, chunk ^= row & 7)
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
    for (int j = 0; j < WI; ++j) {
      const int row = c0 + 8 * (wave + 4 * j) + lr;
      const int k = kt * 64 + ch * 8;
      const bool v = (row < a.K) & (k < a.Kg);
      const char* src = wg + (size_t)(uint32_t)((row * a.Kg + k) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(smem + kt * CT * 128 + (wave + 4 * j) * 1024),
                                       16, 0, 0);
    }
  }
  // The DMA source addresses are kept live until the end of the iteration (asm use below): hipcc
  // waits vmcnt(0) before any instruction that overwrites an in-flight LDS-DMA's address VGPRs, which
  // would drain the prefetch at the first fragment read.
  const char* srcs[NKT * AI];
  auto issue = [&](int t, int buf) {
    char* base = smem + OFF_A + buf * ABUF;
    uint32_t pix[AI];  // STEM: byte offset of each of this lane's pixels' first tap
    if constexpr (STEM) {
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int m = t * PT + 8 * (wave + 4 * j) + lr;
        const uint32_t mm = m < a.M ? (uint32_t)m : 0u;
        const uint32_t n = fdiv(mm, a.fd_PQ), rem = mm - n * (a.P * a.Q);
        const uint32_t p = fdiv(rem, a.fd_Q), q = rem - p * a.Q;
        pix[j] = ((n * a.Hin + p * a.stride) * a.Win + q * a.stride) * 8u;
      }
    }
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int k = kt * 64 + ch * 8;
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const int m = t * PT + 8 * (wave + 4 * j) + lr;
        const bool v = (m < a.M) & (k < a.Kg);
        const char* src = STEM ? xg + (size_t)(pix[j] + (uint32_t)((k >> 5) * a.Win * 8 + (k & 31) * 2))
                               : xg + (size_t)(uint32_t)(m * a.pix_bytes + k * 2);
        srcs[kt * AI + j] = v ? src : zg;
        glds16(srcs[kt * AI + j], base + kt * PT * 128 + (wave + 4 * j) * 1024);
      }
    }
  };
  auto transform = [&](int t, int buf) {
    char* base = smem + OFF_A + buf * ABUF;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      const int k = kt * 64 + ch * 8;
      if (k < a.Kg) {
        const float4 s0 = *(const float4*)(s_scale + k), s1 = *(const float4*)(s_scale + k + 4);
        const float4 h0 = *(const float4*)(s_shift + k), h1 = *(const float4*)(s_shift + k + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int j = 0; j < AI; ++j) {
          const int m = t * PT + 8 * (wave + 4 * j) + lr;
          if (m < a.M) {
            uint4* pp = (uint4*)(base + kt * PT * 128 + (wave + 4 * j) * 1024 + lane * 16);
            const uint4 q = *pp;
            uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float lo = fmaxf(fmaf(lo_bf(u[e]), sc[2 * e], sh[2 * e]), 0.f);
              const float hi = fmaxf(fmaf(hi_bf(u[e]), sc[2 * e + 1], sh[2 * e + 1]), 0.f);
              u[e] = pack2bf(lo, hi);
            }
            *pp = make_uint4(u[0], u[1], u[2], u[3]);
          }
        }
      }
    }
  };

  const int wp = wave % 2, wc = wave / 2;
  const int fr = lane & 15, fk = lane >> 4;
  float ssum[8], ssq[8], aacc[24];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ssum[e] = 0.f; ssq[e] = 0.f; }
#pragma unroll
  for (int e = 0; e < 24; ++e) aacc[e] = 0.f;
  int t = by0;
  const int gy = gridDim.y;
  if (t < ntiles) issue(t, 0);
  if (NBUF == 3 && t + gy < ntiles) issue(t + gy, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // weights (+ prologue affine) resident, tile 0 (and 1) landed
  int buf = 0;
  for (int it = 0; t < ntiles; ++it, t += gy) {
    if constexpr (NBUF == 2) {
      // this wave's DMA of tile t has landed once at most the previous epilogue's NIT stores are pending
      if (it > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIT) : "memory");
    } else if (it >= 2) {
      // issued after this wave's DMA of tile t: stores(it-2), the DMA of tile t+gy (if any), stores(it-1)
      if (t + gy < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIT + NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIT) : "memory");
    }
    if constexpr (PRO) transform(t, buf);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t visible; the slot read last iteration and the stage area are free
    if constexpr (NBUF == 2) {
      if (t + gy < ntiles) issue(t + gy, buf ^ 1);
    } else {
      if (t + 2 * gy < ntiles) issue(t + 2 * gy, buf == 0 ? 2 : buf - 1);
    }
    f32x4 acc[TC][TP];
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const char* abase = smem + OFF_A + buf * ABUF;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        short8 bf[TP], af[TC];
        const int chn = ks * 4 + fk;
#pragma unroll
        for (int j = 0; j < TP; ++j) {
          const int row = wp * WP + j * 16 + fr;
          bf[j] = *(const short8*)(abase + kt * PT * 128 + row * 128 + ((chn ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int row = wc * WC + i * 16 + fr;
          af[i] = *(const short8*)(smem + kt * CT * 128 + row * 128 + ((chn ^ (row & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < TC; ++i)
#pragma unroll
          for (int j = 0; j < TP; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
    conv_nt_epilogue<PT, CT, WP, WC, 1, true, true, true, true, 256, SIDE>(a, acc, smem + OFF_S, t * PT, c0, t, ssum,
                                                                           ssq, nullptr, nullptr, aacc);
#pragma unroll
    for (int i = 0; i < NKT * AI; ++i) asm volatile("" ::"v"(srcs[i]));
    buf = buf + 1 == NBUF ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // one partial row per worker (pixel-tile walker): [sum(K) | sumsq(K)] statistics, or the dgrad's
  // activation-backward sums [sum g*x | sum g (| sum g*r | sum g)] (SIDE)
  if (a.stats) worker_row<CT>((float*)(smem + OFF_S), ssum, ssq, a.stats + (size_t)by0 * (2 * a.K), c0, a.K);
  if (SIDE && a.act_x && a.act_sums) {
    const int rw = a.act_r ? 4 : 2;
    float* row = a.act_sums + (size_t)by0 * (rw * a.K);
    worker_row<CT>((float*)(smem + OFF_S), aacc, aacc + 8, row, c0, a.K);
    if (a.act_r) worker_row<CT>((float*)(smem + OFF_S), aacc + 16, aacc + 8, row + 2 * a.K, c0, a.K);
  }
}

// ------------------------------------------------------------------------------------------
// Direct 3x3 stride-1 conv for narrow layers (C in {32, 64} input channels, CT = 32 / 64 output channels per
// block): the ResNet-50 stage-1 3x3 (64 -> 64) and the Inception-v3 stem 3x3s (32 -> 32 / 64) forward and
// dgrad.  As an implicit GEMM these re-read every input pixel from L2 once per tap (9x) with a 64-deep
// reduction per k-step; here a persistent block keeps the 9 x CT x C weights resident in LDS and streams
// spatial output tiles of 8 x 16 pixels: the tile's (8+2) x (16+2) input halo arrives by LDS-DMA (3-slot ring,
// two tiles in flight) and all nine taps read their MFMA fragments from it.  16-B chunk swizzle: chunk c of
// pixel / weight row p sits at slot c ^ ((p >> 1) & 7) (C = 64) or c ^ ((p >> 2) & 3) (C = 32), so the 16
// consecutive pixels / rows of a fragment read cover all 64 banks.  The finished tile is staged in its own
// (now free) halo slot for the shared epilogue (spatial output mapping: ConvNTArgs::sp_tw).
template <int CIN>
__device__ __forceinline__ int dsw(int p, int c) {
  return CIN == 64 ? (c ^ ((p >> 1) & 7)) : (c ^ ((p >> 2) & 3));
}

template <int CIN, int CT, bool SIDE>
__global__ __launch_bounds__(256) void conv3x3_direct_kernel(ConvNTArgs a, int ntiles) {
  constexpr int TH = 8, TW = 16, PT = TH * TW, HH = TH + 2, HW = TW + 2;
  constexpr int CPP = CIN / 8;                    // 16-B chunks per pixel
  constexpr int HCH = HH * HW * CPP;              // halo chunks
  constexpr int NDMA = (HCH + 255) / 256;         // halo DMA instructions per thread per tile
  constexpr int OROW = CT * 2 + 16;
  constexpr int HDMA = NDMA * 256 * 16;
  // a slot also holds the staged output tile (the post-op sums accumulate per worker: no per-tile table)
  constexpr int HBUF = HDMA > PT * OROW ? HDMA : PT * OROW;
  static_assert(3 * HBUF >= 256 * 16 * 4, "worker_row's reduction table fits in the ring");
  constexpr int WBUF = 9 * CT * CIN * 2;
  constexpr int NIT = PT * (CT / 8) / 256;        // exact staged stores per thread per tile
  constexpr int TC = CT / 16, TP = 2;
  // SIDE: the dgrad post-op inputs (add_src / act_x chunks of each staged store) arrive by LDS-DMA issued at the
  // top of the tile's iteration, and the act scale / shift sit in LDS: the epilogue makes no global loads
  constexpr int SD = SIDE ? 2 * NIT : 0;          // side DMA instructions per thread per tile
  constexpr int SBUF = SIDE ? 2 * NIT * 4096 + 2 * CT * 4 : 0;
  static_assert(2 * NIT + SD + NDMA <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[WBUF + 3 * HBUF + SBUF];
  char* sside = smem + WBUF + 3 * HBUF;
  float* s_ss = (float*)(sside + 2 * NIT * 4096);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = gridDim.x * gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nb);
  const int bx = bid % gridDim.x, by0 = bid / gridDim.x;
  const int c0 = bx * CT;
  const char* xg = (const char*)a.x;
  const char* zg = (const char*)a.zero;
  const int tiles_w = a.sp_tw, tiles_img = a.sp_th * a.sp_tw;

  if constexpr (SIDE) {
    for (int j = tid; j < 2 * CT; j += 256) {
      const int ch = j % CT, k = c0 + ch;
      s_ss[j] = (a.act_x && k < a.K) ? a.act_ss[(j / CT) * a.K + k] : (j < CT ? 1.f : 0.f);
    }
  }
  // resident weights: row (tap, channel) = tap * CT + ch, CIN-deep, swizzled 16-B chunks (plain loads)
  for (int q = tid; q < 9 * CT * CPP; q += 256) {
    const int row = q / CPP, c = q % CPP;
    const int tap = row / CT, ch = row % CT, k = c0 + ch;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k < a.K) v = *(const uint4*)(a.w + ((size_t)k * 9 + tap) * CIN + c * 8);
    *(uint4*)(smem + (row * CPP + dsw<CIN>(row, c)) * 16) = v;
  }
  // this thread's halo DMA slots (tile-independent part): slot q -> pixel hp, chunk c
  int hoff[NDMA], hrow[NDMA], hcol[NDMA];
#pragma unroll
  for (int j = 0; j < NDMA; ++j) {
    const int q = (j * 4 + wave) * 64 + lane;
    const int hp = q / CPP, sc = q % CPP;
    const int c = dsw<CIN>(hp, sc);
    const int hh = hp / HW, ww = hp % HW;
    hrow[j] = q < HCH ? hh : -100000;  // (slots past the halo load zeros)
    hcol[j] = ww;
    hoff[j] = (hh * a.Win + ww) * (CIN * 2) + c * 16;
  }
  const char* srcs[NDMA];
  auto issue = [&](int t, int buf) {
    const uint32_t n = (uint32_t)t / (uint32_t)tiles_img, rem = (uint32_t)t - n * tiles_img;
    const int th = (int)(rem / (uint32_t)tiles_w), tw = (int)(rem - th * tiles_w);
    const int h0 = th * TH - a.pad_h, w0 = tw * TW - a.pad_w;
    const int base = (((int)n * a.Hin + h0) * a.Win + w0) * (CIN * 2);
    char* dst = smem + WBUF + buf * HBUF;
#pragma unroll
    for (int j = 0; j < NDMA; ++j) {
      const int h = h0 + hrow[j], w = w0 + hcol[j];
      const bool v = ((unsigned)h < (unsigned)a.Hin) & ((unsigned)w < (unsigned)a.Win);
      srcs[j] = v ? xg + (size_t)(uint32_t)(base + hoff[j]) : zg;
      glds16(srcs[j], dst + (j * 4 + wave) * 1024);
    }
  };

  // side inputs of tile t: thread tid's staged store j is pixel row (j*256 + tid) / (CT/8), chunk tid % (CT/8)
  const char* ssrc[SIDE ? 2 * NIT : 1];
  auto side_issue = [&](int t) {
    if constexpr (SIDE) {
      constexpr int CPR = CT / 8;
      const int kc = c0 + (tid % CPR) * 8;
#pragma unroll
      for (int j = 0; j < NIT; ++j) {
        const int m = t * PT + (j * 256 + tid) / CPR;
        const bool v = (kc < a.K) && out_valid(a, m);
        const size_t o = v ? (size_t)out_row(a, m) * a.K + kc : 0;
        ssrc[j] = (v && a.add_src) ? (const char*)(a.add_src + o) : zg;
        ssrc[NIT + j] = (v && a.act_x) ? (const char*)(a.act_x + o) : zg;
        glds16(ssrc[j], sside + (j * 4 + wave) * 1024);
        glds16(ssrc[NIT + j], sside + ((NIT + j) * 4 + wave) * 1024);
      }
    }
  };

  const int fr = lane & 15, fk = lane >> 4;
  float ssum[8], ssq[8], aacc[24];
#pragma unroll
  for (int e = 0; e < 8; ++e) { ssum[e] = 0.f; ssq[e] = 0.f; }
#pragma unroll
  for (int e = 0; e < 24; ++e) aacc[e] = 0.f;
  const int gy = gridDim.y;
  int t = by0;
  if (t < ntiles) issue(t, 0);
  if (t + gy < ntiles) issue(t + gy, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // weights resident, tiles 0 and 1 landed
  int buf = 0;
  for (int it = 0; t < ntiles; ++it, t += gy) {
    if (it >= 2) {
      // issued after this wave's DMA of tile t: stores(it-2), side(it-1), the DMA of tile t+gy (if any),
      // stores(it-1)
      if (t + gy < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIT + SD + NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIT + SD) : "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t visible; the slot of tile t-1 (its staging area) is free
    side_issue(t);
    const bool pf = t + 2 * gy < ntiles;
    if (pf) issue(t + 2 * gy, buf == 0 ? 2 : buf - 1);
    f32x4 acc[TC][TP];
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const char* hb = smem + WBUF + buf * HBUF;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap % 3;
#pragma unroll
      for (int kc = 0; kc < CIN / 32; ++kc) {
        const int c = kc * 4 + fk;
        short8 bf[TP], af[TC];
#pragma unroll
        for (int j = 0; j < TP; ++j) {
          const int hp = (2 * wave + j + r) * HW + fr + s;
          bf[j] = *(const short8*)(hb + (hp * CPP + dsw<CIN>(hp, c)) * 16);
        }
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int row = tap * CT + i * 16 + fr;
          af[i] = *(const short8*)(smem + (row * CPP + dsw<CIN>(row, c)) * 16);
        }
#pragma unroll
        for (int i = 0; i < TC; ++i)
#pragma unroll
          for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      }
    }
    if constexpr (SIDE) {  // this thread's side chunks of tile t have landed (only the halo prefetch may pend)
      if (pf) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading the halo slot: it becomes the staging area
    conv_nt_epilogue<PT, CT, 32, CT, 1, true, true, true, true, 256, SIDE, SIDE>(a, acc, (char*)hb, t * PT, c0, t, ssum,
                                                                                  ssq, sside, s_ss, aacc);
#pragma unroll
    for (int i = 0; i < NDMA; ++i) asm volatile("" ::"v"(srcs[i]));
    if constexpr (SIDE) {
#pragma unroll
      for (int i = 0; i < 2 * NIT; ++i) asm volatile("" ::"v"(ssrc[i]));
    }
    buf = buf == 2 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // one partial row per worker: [sum(K) | sumsq(K)] statistics, or the dgrad's [sum g*x | sum g] (SIDE)
  float* red = (float*)(smem + WBUF);  // [256][16] (the halo ring is free)
  if (a.stats) worker_row<CT>(red, ssum, ssq, a.stats + (size_t)by0 * (2 * a.K), c0, a.K);
  if (SIDE && a.act_x && a.act_sums) worker_row<CT>(red, aacc, aacc + 8, a.act_sums + (size_t)by0 * (2 * a.K), c0, a.K);
}

// ------------------------------------------------------------------------------------------
// weight gradient
struct ConvWgradArgs {
  const bf16_t* x;   // [N][H][W][C] forward input
  const bf16_t* dy;  // [N][P][Q][K]
  float* dw;         // workspace slabs [splits][K][R*S*C] fp32 (summed into the gradient afterwards)
  const float* in_scale;  // optional prologue affine+relu on x (same as the forward's)
  const float* in_shift;
  uint32_t x_bytes, dy_bytes;
  int N, H, W, C, K, R, S, P, Q, stride, pad_h, pad_w;
  int Mpix;  // N*P*Q
  int Kg;    // R*S*C
  int pix_per_split;
  FastDiv fd_PQ, fd_Q;
  int pix_bytes;  // byte pitch of one x pixel (C*2, or less for the packed-row stem view)
  // optional BatchNorm backward of dy (register-staged kernels only): dy is the unscaled gradient g of
  // the BN output and the A operand is comb = g*scale + dsum + 2*dsumsq*ay (stats_combine_fin's algebra,
  // coefficients from dss / ss / gamma per block); the blocks of pixel split 0 / column tile 0 also
  // accumulate dgamma / dbeta.  Saves writing comb and reading it back when nothing else reads it.
  const bf16_t* ay;  // [N][P][Q][K] raw BN input, or nullptr
  const float* dss;
  const float* ss;
  const float* gamma;
  float count;
  float* dgamma;
  float* dbeta;
};

// byte offset of element (k, m) in a [64 k][ROWS] tile stored as [k/4][m/16][4][16] blocks,
// with bit 7 flipped for odd (k>>3) so that the two 16-lane groups of a transposed-read half
// wave hit opposite 128-B halves of the 256-B bank row.
template <int ROWS>
__device__ __forceinline__ int tr_off(int k, int m) {
  constexpr int MB = ROWS / 16;
  int b = (k >> 2) * MB + (m >> 4);
  return ((b << 7) + ((k & 3) << 5) + ((m & 15) << 1)) ^ (((k >> 3) & 1) << 7);
}

template <int MT, int NT, int WM, int WN, int NBUF>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvWgradArgs a) {
  constexpr int BK = 64;
  constexpr int NWM = MT / WM, NWN = NT / WN;
  static_assert(NWM * NWN == 4, "4 waves");
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int ACH = MT / 32;  // BK*MT/8 chunks / 256 threads
  constexpr int BCH = NT / 32;
  constexpr int BUF = BK * (MT + NT) * 2;
  __shared__ __attribute__((aligned(16))) char smem[NBUF * BUF + NT * 8 + MT * 12];
  float* s_scale = (float*)(smem + NBUF * BUF);  // prologue scale/shift of this block's NT columns
  float* s_shift = s_scale + NT;
  float* s_cs = s_shift + NT;  // BN-backward coefficients of this block's MT rows (a.ay)
  float* s_ca = s_cs + MT;
  float* s_cb = s_ca + MT;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int gxy = gridDim.x * gridDim.y;
  const int tile = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gxy * gridDim.z);
  const int bz = tile / gxy, by = (tile % gxy) / gridDim.x, bx = tile % gridDim.x;
  if (a.in_scale) {
    for (int j = tid; j < NT; j += 256) {
      int col = bx * NT + j;
      int c = col < a.Kg ? col % a.C : 0;
      s_scale[j] = a.in_scale[c];
      s_shift[j] = a.in_shift[c];
    }
    __syncthreads();
  }
  const int wm = wave % NWM, wn = wave / NWM;
  const int n0 = bx * NT, m0 = by * MT;
  const int pix_lo = bz * a.pix_per_split;
  const int pix_hi = min(a.Mpix, pix_lo + a.pix_per_split);
  // (an empty split still runs: it stores a zero slab, which the reduction relies on)
  if (a.ay) {
    for (int j = tid; j < MT; j += 256) {
      const int ko = m0 + j;
      float ds = 0.f, dq = 0.f, dg, db, sc = 0.f;
      if (ko < a.K) {
        fin_bwd_channel(a.dss, a.ss, a.gamma, a.K, ko, a.count, &ds, &dq, &dg, &db);
        sc = a.ss[ko];
        if (bx == 0 && bz == 0) {
          if (a.dgamma) a.dgamma[ko] += dg;
          if (a.dbeta) a.dbeta[ko] += db;
        }
      }
      s_cs[j] = sc;
      s_ca[j] = ds;
      s_cb[j] = 2.f * dq;
    }
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(a.ay ? a.ay : a.dy, a.dy_bytes);

  const int sub = tid & 7, kk = sub >> 1, half = sub & 1, grp = tid >> 3;
  // A (dy) chunk coordinates
  int a_k[ACH], a_m[ACH];
#pragma unroll
  for (int i = 0; i < ACH; ++i) {
    int G = grp + 32 * i;
    a_k[i] = (G / (MT / 16)) * 4 + kk;
    a_m[i] = (G % (MT / 16)) * 16 + half * 8;
  }
  // B (x) chunk coordinates; the column -> (r, s, c) decode is fixed for the block
  int b_k[BCH], b_n[BCH], b_r[BCH], b_s[BCH], b_c[BCH];
  bool b_colv[BCH];
#pragma unroll
  for (int i = 0; i < BCH; ++i) {
    int G = grp + 32 * i;
    b_k[i] = (G / (NT / 16)) * 4 + kk;
    b_n[i] = (G % (NT / 16)) * 16 + half * 8;
    int col = n0 + b_n[i];
    b_colv[i] = col < a.Kg;
    int tap = col / a.C;
    b_c[i] = col - tap * a.C;
    b_r[i] = tap / a.S;
    b_s[i] = tap - b_r[i] * a.S;
  }

  uint4 areg[ACH], breg[BCH], yreg[ACH];
  bool aval[ACH], bval[BCH];
  int bcc[BCH];
  auto gload = [&](int pbase) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      int pix = pbase + a_k[i];
      int ko = m0 + a_m[i];
      bool v = pix < pix_hi && ko < a.K;
      uint32_t off = v ? (uint32_t)(((size_t)pix * a.K + ko) * 2) : OOB_OFFSET;
      areg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(dr, off, 0, 0));
      aval[i] = v;
      if (a.ay) yreg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      int pix = pbase + b_k[i];
      bool v = b_colv[i] && pix < pix_hi;
      uint32_t n = fdiv((uint32_t)pix, a.fd_PQ);
      uint32_t rem = pix - n * (a.P * a.Q);
      uint32_t p = fdiv(rem, a.fd_Q);
      uint32_t q = rem - p * a.Q;
      int ih = (int)p * a.stride - a.pad_h + b_r[i];
      int iw = (int)q * a.stride - a.pad_w + b_s[i];
      v = v && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      uint32_t off = v ? (uint32_t)((((int)n * a.H + ih) * a.W + iw) * a.pix_bytes + b_c[i] * 2) : OOB_OFFSET;
      bval[i] = v;
      bcc[i] = b_c[i];
      breg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  auto swrite = [&](int buf) {
    char* base = smem + buf * BUF;
    if (a.ay) {
#pragma unroll
      for (int i = 0; i < ACH; ++i) {
        uint32_t u[4] = {areg[i].x, areg[i].y, areg[i].z, areg[i].w};
        const uint32_t yu[4] = {yreg[i].x, yreg[i].y, yreg[i].z, yreg[i].w};
        const int m = a_m[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c0 = m + 2 * e, c1 = c0 + 1;
          const float lo = aval[i] ? fmaf(lo_bf(u[e]), s_cs[c0], s_ca[c0] + s_cb[c0] * lo_bf(yu[e])) : 0.f;
          const float hi = aval[i] ? fmaf(hi_bf(u[e]), s_cs[c1], s_ca[c1] + s_cb[c1] * hi_bf(yu[e])) : 0.f;
          u[e] = pack2bf(lo, hi);
        }
        areg[i] = make_uint4(u[0], u[1], u[2], u[3]);
      }
    }
    if (a.in_scale) {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        if (bval[i]) {
          uint32_t u[4] = {breg[i].x, breg[i].y, breg[i].z, breg[i].w};
          const float4 s0 = *(const float4*)(s_scale + b_n[i]), s1 = *(const float4*)(s_scale + b_n[i] + 4);
          const float4 h0 = *(const float4*)(s_shift + b_n[i]), h1 = *(const float4*)(s_shift + b_n[i] + 4);
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float lo = fmaxf(fmaf(lo_bf(u[e]), sc[2 * e], sh[2 * e]), 0.f);
            float hi = fmaxf(fmaf(hi_bf(u[e]), sc[2 * e + 1], sh[2 * e + 1]), 0.f);
            u[e] = pack2bf(lo, hi);
          }
          breg[i] = make_uint4(u[0], u[1], u[2], u[3]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < ACH; ++i) *(uint4*)(base + tr_off<MT>(a_k[i], a_m[i])) = areg[i];
#pragma unroll
    for (int i = 0; i < BCH; ++i) *(uint4*)(base + BK * MT * 2 + tr_off<NT>(b_k[i], b_n[i])) = breg[i];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (pix_hi - pix_lo + BK - 1) / BK;
  gload(pix_lo);
  swrite(0);
  __syncthreads();
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  typedef __attribute__((address_space(3))) char lds_c;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NBUF == 2 ? (kt & 1) : 0;
    if (kt + 1 < nk) gload(pix_lo + (kt + 1) * BK);
    lds_c* lbase = (lds_c*)(smem + cur * BUF);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      short8 af[TM], bfr[TN];
      const int kb = ks * 32 + 8 * g;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int m = wm * WM + i * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(lbase + tr_off<MT>(kb + tq, m)));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(lbase + tr_off<MT>(kb + 4 + tq, m)));
        af[i] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int n = wn * WN + j * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(lbase + BK * MT * 2 + tr_off<NT>(kb + tq, n)));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_s4*)(lbase + BK * MT * 2 + tr_off<NT>(kb + 4 + tq, n)));
        bfr[j] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (NBUF == 2) {
      if (kt + 1 < nk) swrite(cur ^ 1);
      __syncthreads();
    } else {
      __syncthreads();
      if (kt + 1 < nk) {
        swrite(0);
        __syncthreads();
      }
    }
  }
  // epilogue: acc rows = ko (4 consecutive per lane), cols = flattened (r,s,c).  Each pixel split
  // writes its partial tile to its own workspace slab (plain stores); dtm_reduce_rows then sums the
  // slabs into dW.  (Split-K fp32 atomics onto the same tile serialise at the memory-side atomic
  // units: up to hundreds of splits hit one 64-KB tile for the K x 64 1x1 layers.)
  float* slab = a.dw + (size_t)bz * a.K * a.Kg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + li;
      const int ko = m0 + wm * WM + i * 16 + g * 4;
      if (col < a.Kg) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ko + r < a.K) {
            slab[(size_t)(ko + r) * a.Kg + col] = acc[i][j][r];
          }
      }
    }
  }
}

// Direct 3x3 stride-1 weight gradient for narrow layers (C in {32, 64} input channels, 32 dW rows per block; the
// Inception-v3 stem's 147x147 3x3s and ResNet-50's 56x56 3x3 64 -> 64): dW[k][r][s][c] = sum_p dy[p][k] x[p+(r,s)][c].
// As an implicit GEMM (conv_wgrad_kernel) every input pixel is fetched once per tap; here a persistent block walks
// 8 x 16 output-pixel tiles and stages each tile's operands ONCE, transposed to channel-major in LDS so that the
// reduction over pixels runs along contiguous memory: dy^T [32 k][128 px] and the (8+2)-row x halo as three
// column-shifted copies [s][c][10 rows][16 cols] (tap column s is then an aligned 8-pixel read).  The optional
// BN-apply prologue (relu(x*scale + shift), zero padding kept zero) is applied once per staged element.  Waves own
// 16 input channels each (C = 64: all 9 taps; C = 32: two waves per channel group, taps 0-4 / 5-8) and both 16-row
// halves of the block's 32 dW rows, so one dy^T fragment serves every tap and one x fragment both row halves.  The
// next tile's operands are loaded into registers while this one is multiplied.  One fp32 slab per block, summed by
// dtm_reduce_rows.
template <int CIN, int KT>
__global__ __launch_bounds__(256) void conv3x3_wgrad_direct_kernel(ConvWgradArgs a, int ntiles, int tiles_w,
                                                                   int tiles_img) {
  constexpr int TH = 8, TW = 16, HR = TH + 2, NKT = KT / 16;
  constexpr int NCG = CIN / 8;                       // 8-channel groups of x
  constexpr int NCT = CIN / 16;                      // 16-channel fragment columns
  constexpr int WPC = 4 / NCT;                       // waves per channel group (2 or 1)
  constexpr int TPW = (9 + WPC - 1) / WPC;           // taps per wave (5 or 9)
  constexpr int CS = 168;                            // x copy row pitch per channel (elements): 16-lane reads hit
                                                     // distinct banks
  constexpr int DS = 136;                            // dy^T pitch per k (elements)
  constexpr int XT = 3 * HR * 2 * NCG;               // x staging tasks (8 pixels x 8 channels) per tile
  constexpr int XPT = (XT + 255) / 256;              // per thread
  constexpr int DT = TH * 2 * (KT / 8);              // dy staging tasks per tile (64 / 128)
  static_assert(DT <= 256, "one dy task per thread");
  __shared__ __attribute__((aligned(16))) bf16_t xs[3 * CIN * CS];
  __shared__ __attribute__((aligned(16))) bf16_t dyt[KT * DS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = gridDim.x * gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nb);
  const int bx = bid % gridDim.x, by0 = bid / gridDim.x;
  const int k0 = bx * KT;
  const int ct = wave % NCT, th = wave / NCT;        // this wave's 16 input channels and tap range
  const int tap0 = th * TPW, tap1 = min(9, tap0 + TPW);
  const bf16_t* xg = a.x;
  const bf16_t* dg = a.dy;

  uint4 xr[XPT][8], dr[8];
  // loads of tile t's operands into registers (zeros out of range: padding, pixels past the map)
  auto load = [&](int t) {
    const int n = t / tiles_img, rem = t - n * tiles_img;
    const int oh0 = (rem / tiles_w) * TH, ow0 = (rem % tiles_w) * TW;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + 256 * i;
      const int cg = q % NCG, run = (q / NCG) % 2, hr = (q / (2 * NCG)) % HR, sc = q / (2 * NCG * HR);
      const int ih = oh0 + hr - a.pad_h;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int iw = ow0 + run * 8 + j + sc - a.pad_w;
        const bool v = q < XT && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        xr[i][j] = v ? *(const uint4*)(xg + (((size_t)n * a.H + ih) * a.W + iw) * CIN + cg * 8) : make_uint4(0, 0, 0, 0);
      }
    }
    if (tid < DT) {
      const int cg = tid % (KT / 8), run = (tid / (KT / 8)) % 2, row = tid / (KT / 4);
      const int oh = oh0 + row;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ow = ow0 + run * 8 + j;
        const bool v = oh < a.P && ow < a.Q && k0 + cg * 8 < a.K;
        dr[j] = v ? *(const uint4*)(dg + (((size_t)n * a.P + oh) * a.Q + ow) * a.K + k0 + cg * 8) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  // 8 pixels x 8 channels (rows = pixels) -> channel-major rows of 8 pixels: out[ch] = (q[0][ch] .. q[7][ch])
  auto transpose = [&](const uint4 (&q)[8], uint4 (&o)[8]) {
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
      const uint32_t sel = (ch & 1) ? 0x07060302u : 0x05040100u;
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint4& lo = q[2 * j];
        const uint4& hi = q[2 * j + 1];
        const uint32_t l = (ch >> 1) == 0 ? lo.x : (ch >> 1) == 1 ? lo.y : (ch >> 1) == 2 ? lo.z : lo.w;
        const uint32_t h = (ch >> 1) == 0 ? hi.x : (ch >> 1) == 1 ? hi.y : (ch >> 1) == 2 ? hi.z : hi.w;
        w[j] = __builtin_amdgcn_perm(h, l, sel);
      }
      o[ch] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  };
  auto store = [&](int t) {
    const int n = t / tiles_img, rem = t - n * tiles_img;
    const int oh0 = (rem / tiles_w) * TH, ow0 = (rem % tiles_w) * TW;
    (void)n;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + 256 * i;
      if (q < XT) {
        const int cg = q % NCG, run = (q / NCG) % 2, hr = (q / (2 * NCG)) % HR, sc = q / (2 * NCG * HR);
        uint4 px[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) px[j] = xr[i][j];
        if (a.in_scale) {  // BN-apply prologue on the valid (non-padding) pixels
          const int ih = oh0 + hr - a.pad_h;
          float sc8[8], sh8[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            sc8[e] = a.in_scale[cg * 8 + e];
            sh8[e] = a.in_shift[cg * 8 + e];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int iw = ow0 + run * 8 + j + sc - a.pad_w;
            if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) {
              const uint32_t u[4] = {px[j].x, px[j].y, px[j].z, px[j].w};
              uint32_t o[4];
#pragma unroll
              for (int e = 0; e < 4; ++e)
                o[e] = pack2bf(fmaxf(fmaf(lo_bf(u[e]), sc8[2 * e], sh8[2 * e]), 0.f),
                               fmaxf(fmaf(hi_bf(u[e]), sc8[2 * e + 1], sh8[2 * e + 1]), 0.f));
              px[j] = make_uint4(o[0], o[1], o[2], o[3]);
            }
          }
        }
        uint4 o[8];
        transpose(px, o);
#pragma unroll
        for (int ch = 0; ch < 8; ++ch)
          *(uint4*)&xs[(sc * CIN + cg * 8 + ch) * CS + hr * 16 + run * 8] = o[ch];
      }
    }
    if (tid < DT) {
      const int cg = tid % (KT / 8), run = (tid / (KT / 8)) % 2, row = tid / (KT / 4);
      uint4 o[8];
      transpose(dr, o);
#pragma unroll
      for (int ch = 0; ch < 8; ++ch) *(uint4*)&dyt[(cg * 8 + ch) * DS + row * 16 + run * 8] = o[ch];
    }
  };

  f32x4 acc[TPW][NKT];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) acc[i][kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, g = lane >> 4;
  const int gy = gridDim.y;
  int t = by0;
  if (t < ntiles) load(t);
  for (; t < ntiles; t += gy) {
    store(t);
    __syncthreads();
    if (t + gy < ntiles) load(t + gy);  // (in flight while this tile is multiplied)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {  // 32 pixels = output rows 2 ks, 2 ks + 1
      const int pix = ks * 32 + 8 * g;
      short8 af[NKT];
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) af[kt] = *(const short8*)&dyt[(kt * 16 + fr) * DS + pix];
      const int prow = 2 * ks + (g >> 1), pcol = 8 * (g & 1);
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int tap = tap0 + i;
        if (tap < tap1) {
          const int r = tap / 3, sc = tap - r * 3;
          const short8 b = *(const short8*)&xs[(sc * CIN + ct * 16 + fr) * CS + (prow + r) * 16 + pcol];
#pragma unroll
          for (int kt = 0; kt < NKT; ++kt)
            acc[i][kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kt], b, acc[i][kt], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // (the next store overwrites the staged operands)
  }
  // this block's partial dW: lane holds rows kt*16 + 4 g + e, column ct*16 + fr of each tap
  float* slab = a.dw + (size_t)by0 * a.K * a.Kg;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int tap = tap0 + i;
    if (tap < tap1) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = k0 + kt * 16 + 4 * g + e;
          if (k < a.K) slab[(size_t)k * a.Kg + tap * CIN + ct * 16 + fr] = acc[i][kt][e];
        }
    }
  }
}

// Pipelined LDS-DMA weight gradient (no input prologue): both pixel-major operand tiles go global ->
// LDS by LDS-DMA straight into the [k/4][row/16][4][16] transposed-read image.  An LDS-DMA writes
// lane-linear 16-B slots, so each lane loads the chunk whose tr_off position is its slot (the inverse
// of tr_off, fixed per lane for every k-tile).  NS-slot ring, one raw barrier per k-tile, counted
// vmcnt; waves 2x2 of (MT/2) x (NT/2).
template <int ROWS>
__device__ __forceinline__ void tr_inv(int q, int& k, int& m) {
  constexpr int MB = ROWS / 16;
  const int b1 = q >> 3, kq = b1 / MB;
  k = kq * 4 + ((q & 7) >> 1);
  const int b = b1 ^ ((kq >> 1) & 1);
  m = (b % MB) * 16 + (q & 1) * 8;
}

// NTH threads (256 = 4 waves 2x2; 512 = the 8-wave 256x256 variant, waves NWM x 8/NWM): the bigger tile
// halves the L2 operand bytes per MFMA (same reasoning as conv_nt_w8_kernel)
// BNA: the BatchNorm backward of dy fused into the A operand (ConvWgradArgs::ay, the stem's conv+BN with no input
// gradient): the raw BN input y is LDS-DMA'd beside g into a parallel image and, once this wave's DMAs of the k-tile
// have landed, each lane rewrites ITS OWN chunks to comb = g*scale + dsum + 2*dsumsq*y (stats_combine_fin's algebra)
// before the barrier that publishes the stage - the register-staged kernel's fusion on the pipelined tile.
template <int MT, int NT, int NS, int NWM = 2, int NTH = 256, bool BNA = false>
__global__ __launch_bounds__(NTH) void conv_wgrad_pipe_kernel(ConvWgradArgs a) {
  constexpr int BK = 64;
  constexpr int NW = NTH / 64;
  constexpr int NWN = NW / NWM;
  constexpr int WM = MT / NWM, WN = NT / NWN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AI = MT / (8 * NW), BI = NT / (8 * NW);  // 1-KiB DMA pieces per wave per k-tile
  constexpr int G = AI + BI + (BNA ? AI : 0);
  constexpr int BUF = BK * (MT + NT) * 2;
  constexpr int YBUF = BNA ? BK * MT * 2 : 0;  // the y image of one slot
  constexpr int OFF_Y = NS * BUF, OFF_C = OFF_Y + NS * YBUF;
  __shared__ __attribute__((aligned(16))) char smem[OFF_C + (BNA ? MT * 12 : 0)];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  static_assert(G <= 31 && NS >= 2 && NS <= 3, "vmcnt range");
  static_assert(AI * 8 * NW == MT && BI * 8 * NW == NT, "DMA piece mapping");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int gxy = gridDim.x * gridDim.y;
  const int tile = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gxy * gridDim.z);
  const int bz = tile / gxy, by = (tile % gxy) / gridDim.x, bx = tile % gridDim.x;
  const int wm = wave % NWM, wn = wave / NWM;
  const int n0 = bx * NT, m0 = by * MT;
  const int pix_lo = bz * a.pix_per_split;
  const int pix_hi = min(a.Mpix, pix_lo + a.pix_per_split);
  float* s_cs = (float*)(smem + OFF_C);  // BNA: comb = g*s_cs + s_ca + s_cb*y per row ko of this block
  float* s_ca = s_cs + MT;
  float* s_cb = s_ca + MT;
  if constexpr (BNA) {
    for (int j = tid; j < MT; j += NTH) {
      const int ko = m0 + j;
      float ds = 0.f, dq = 0.f, dg, db, sc = 0.f;
      if (ko < a.K) {
        fin_bwd_channel(a.dss, a.ss, a.gamma, a.K, ko, a.count, &ds, &dq, &dg, &db);
        sc = a.ss[ko];
        if (bx == 0 && bz == 0) {
          if (a.dgamma) a.dgamma[ko] += dg;
          if (a.dbeta) a.dbeta[ko] += db;
        }
      }
      s_cs[j] = sc;
      s_ca[j] = ds;
      s_cb[j] = 2.f * dq;
    }
    __syncthreads();
  }

  // per-lane chunk coordinates of its DMA slots
  int a_k[AI], a_off[AI];
  bool a_colv[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    int k, m;
    tr_inv<MT>((wave + NW * j) * 64 + lane, k, m);
    a_k[j] = k;
    a_colv[j] = m0 + m < a.K;
    a_off[j] = m0 + m;
  }
  int b_k[BI], b_r[BI], b_s[BI], b_c[BI];
  bool b_colv[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    int k, m;
    tr_inv<NT>((wave + NW * j) * 64 + lane, k, m);
    b_k[j] = k;
    const int col = n0 + m;
    b_colv[j] = col < a.Kg;
    const int tap = col / a.C;
    b_c[j] = col - tap * a.C;
    b_r[j] = tap / a.S;
    b_s[j] = tap - b_r[j] * a.S;
  }
  const char* xg = (const char*)a.x;
  const char* dg = (const char*)a.dy;
  const char* yg = (const char*)a.ay;
  const char* zg = (const char*)a.in_shift;  // the host passes a zero chunk here (no prologue in this kernel)

  auto issue = [&](int pbase, int slot) {
    char* base = smem + slot * BUF;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int pix = pbase + a_k[j];
      const bool v = (pix < pix_hi) & a_colv[j];
      const uint32_t off = (uint32_t)((pix * a.K + a_off[j]) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? dg + (size_t)off : zg), (lvoid*)(base + (wave + NW * j) * 1024),
                                       16, 0, 0);
      if constexpr (BNA)
        __builtin_amdgcn_global_load_lds((gvoid*)(v ? yg + (size_t)off : zg),
                                         (lvoid*)(smem + OFF_Y + slot * YBUF + (wave + NW * j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int pix = pbase + b_k[j];
      const uint32_t n = fdiv((uint32_t)pix, a.fd_PQ);
      const uint32_t rem = pix - n * (a.P * a.Q);
      const uint32_t p = fdiv(rem, a.fd_Q);
      const uint32_t q = rem - p * a.Q;
      const int ih = (int)p * a.stride - a.pad_h + b_r[j];
      const int iw = (int)q * a.stride - a.pad_w + b_s[j];
      const bool v = (pix < pix_hi) & b_colv[j] & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      const char* src = xg + (size_t)(uint32_t)((((int)n * a.H + ih) * a.W + iw) * a.pix_bytes + b_c[j] * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + BK * MT * 2 + (wave + NW * j) * 1024),
                                       16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  typedef __attribute__((address_space(3))) char lds_c;
  auto compute = [&](int slot) {
    lds_c* lbase = (lds_c*)(smem + slot * BUF);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      short8 af[TM], bfr[TN];
      const int kb = ks * 32 + 8 * g;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wm * WM + i * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lbase + tr_off<MT>(kb + tq, m)));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lbase + tr_off<MT>(kb + 4 + tq, m)));
        af[i] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * WN + j * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lbase + BK * MT * 2 + tr_off<NT>(kb + tq, n)));
        short4v hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lbase + BK * MT * 2 + tr_off<NT>(kb + 4 + tq, n)));
        bfr[j] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // BNA: this lane's landed A chunks of k-tile kt -> comb in place (padding / out-of-range pixels stay 0)
  auto transform = [&](int kt, int slot) {
    const int pbase = pix_lo + kt * BK;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int pix = pbase + a_k[j];
      if ((pix < pix_hi) & a_colv[j]) {
        uint4* pg = (uint4*)(smem + slot * BUF + (wave + NW * j) * 1024 + lane * 16);
        const uint4 gq = *pg;
        const uint4 yq = *(const uint4*)(smem + OFF_Y + slot * YBUF + (wave + NW * j) * 1024 + lane * 16);
        const uint32_t gu[4] = {gq.x, gq.y, gq.z, gq.w}, yu[4] = {yq.x, yq.y, yq.z, yq.w};
        uint32_t u[4];
        const int m = a_off[j] - m0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c0 = m + 2 * e, c1 = c0 + 1;
          const float lo = fmaf(lo_bf(gu[e]), s_cs[c0], s_ca[c0] + s_cb[c0] * lo_bf(yu[e]));
          const float hi = fmaf(hi_bf(gu[e]), s_cs[c1], s_ca[c1] + s_cb[c1] * hi_bf(yu[e]));
          u[e] = pack2bf(lo, hi);
        }
        *pg = make_uint4(u[0], u[1], u[2], u[3]);
      }
    }
  };

  const int nk = (pix_hi - pix_lo + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(pix_lo + s * BK, s);
  int slot = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1, kt + NS - 2) - kt;
    if (NS >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (BNA) transform(kt, slot);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) issue(pix_lo + (kt + NS - 1) * BK, slot == 0 ? NS - 1 : slot - 1);
    compute(slot);
    slot = slot == NS - 1 ? 0 : slot + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* slab = a.dw + (size_t)bz * a.K * a.Kg;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * WN + j * 16 + li;
      const int ko = m0 + wm * WM + i * 16 + g * 4;
      if (col < a.Kg) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (ko + r < a.K) {
            slab[(size_t)(ko + r) * a.Kg + col] = acc[i][j][r];
          }
      }
    }
  }
}

// Ping-pong form of conv_wgrad_pipe_kernel<256, 256> (pp_mainloop): dW rows ko as the P operand (dy), columns
// (r, s, c) as W (the gathered input), 64 pixels per k-tile.  Each half-tile is its own [k/4][m/16][4][16]
// transposed-read image of 128 rows (tr_off<128>), filled by LDS-DMA at the lane's inverse-image position (tr_inv<128>)
// and read with ds_read_b64_tr_b16.  Split-K slab epilogue as conv_wgrad_pipe_kernel.
__global__ __launch_bounds__(512) void conv_wgrad_pp_kernel(ConvWgradArgs a) {
  constexpr int NW = 8, BK = 64;
  constexpr int HALF = BK * 128 * 2;
  constexpr int BUF = 4 * HALF;  // [P0 | P1 | W0 | W1]
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  typedef __attribute__((address_space(1))) const void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave >> 2, wq = wave & 3;
  const int gxy = gridDim.x * gridDim.y;
  const int tile = xcd_remap((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x, gxy * gridDim.z);
  const int bz = tile / gxy, by = (tile % gxy) / gridDim.x, bx = tile % gridDim.x;
  const int n0 = bx * 256, m0 = by * 256;
  const int pix_lo = bz * a.pix_per_split;
  const int pix_hi = min(a.Mpix, pix_lo + a.pix_per_split);

  // per-lane chunk coordinates of its DMA slots: piece (wave + 8 jj) of a half, j = 2 h + jj for half h
  int a_k[4], a_off[4];
  bool a_colv[4];
  int b_k[4], b_r[4], b_s[4], b_c[4];
  bool b_colv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int k, m;
    tr_inv<128>((wave + NW * (j & 1)) * 64 + lane, k, m);
    const int h = j >> 1;
    a_k[j] = k;
    a_off[j] = m0 + h * 128 + m;
    a_colv[j] = a_off[j] < a.K;
    b_k[j] = k;
    const int col = n0 + h * 128 + m;
    b_colv[j] = col < a.Kg;
    const int tap = col / a.C;
    b_c[j] = col - tap * a.C;
    b_r[j] = tap / a.S;
    b_s[j] = tap - b_r[j] * a.S;
  }
  const char* xg = (const char*)a.x;
  const char* dg = (const char*)a.dy;
  const char* zg = (const char*)a.in_shift;  // the host passes a zero chunk here (no prologue in this kernel)
  const int nk = (pix_hi - pix_lo + BK - 1) / BK;

  auto issue_p = [&](int kt, int h) {
    char* base = smem + (kt & 1) * BUF + h * HALF;
    const int pbase = pix_lo + kt * BK;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = 2 * h + jj;
      const int pix = pbase + a_k[j];
      const bool v = (pix < pix_hi) & a_colv[j];
      const char* src = dg + (size_t)(uint32_t)((pix * a.K + a_off[j]) * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + NW * jj) * 1024), 16, 0, 0);
    }
  };
  auto issue_w = [&](int kt, int h) {
    char* base = smem + (kt & 1) * BUF + (2 + h) * HALF;
    const int pbase = pix_lo + kt * BK;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = 2 * h + jj;
      const int pix = pbase + b_k[j];
      const uint32_t n = fdiv((uint32_t)pix, a.fd_PQ);
      const uint32_t rem = pix - n * (a.P * a.Q);
      const uint32_t p = fdiv(rem, a.fd_Q);
      const uint32_t q = rem - p * a.Q;
      const int ih = (int)p * a.stride - a.pad_h + b_r[j];
      const int iw = (int)q * a.stride - a.pad_w + b_s[j];
      const bool v = (pix < pix_hi) & b_colv[j] & ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
      const char* src = xg + (size_t)(uint32_t)((((int)n * a.H + ih) * a.W + iw) * a.pix_bytes + b_c[j] * 2);
      __builtin_amdgcn_global_load_lds((gvoid*)(v ? src : zg), (lvoid*)(base + (wave + NW * jj) * 1024), 16, 0, 0);
    }
  };
  auto issue = [&](int kt, int h) {
    if (h == 0) issue_w(kt, 1);
    else if (h == 1) issue_p(kt, 1);
    else if (h == 2) issue_p(kt, 0);
    else issue_w(kt, 0);
  };

  f32x4 acc[2][2][2][4];  // [ni][ii][mi][jj]
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) acc[ni][ii][mi][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int lg = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  typedef __attribute__((address_space(3))) short4v lds_s4;
  typedef __attribute__((address_space(3))) char lds_c;
  short8 P[2][4], Wa[2][2], Wb[2][2];  // [ks][frag]
  auto frag = [&](const char* half, int ks, int m) -> short8 {
    lds_c* lb = (lds_c*)half;
    const int kb = ks * 32 + 8 * lg;
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lb + tr_off<128>(kb + tq, m)));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lb + tr_off<128>(kb + 4 + tq, m)));
    return (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto rd_p = [&](const char* s, int mi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) P[ks][jj] = frag(s + mi * HALF, ks, grp * 64 + jj * 16 + 4 * tp);
  };
  auto rd_w = [&](const char* s, int ni) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const short8 v = frag(s + (2 + ni) * HALF, ks, wq * 32 + ii * 16 + 4 * tp);
        if (ni == 0) Wa[ks][ii] = v;
        else Wb[ks][ii] = v;
      }
  };
  auto mma = [&](int ni, int mi) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          acc[ni][ii][mi][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(P[ks][jj], ni == 0 ? Wa[ks][ii] : Wb[ks][ii],
                                                                        acc[ni][ii][mi][jj], 0, 0, 0);
  };
  pp_mainloop(smem, BUF, nk, grp, issue, rd_p, rd_w, mma);

  // lane: rows ko .. +3 (lg * 4 + r) of column li per 16x16 subtile -> this split's slab
  float* slab = a.dw + (size_t)bz * a.K * a.Kg;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int col = n0 + ni * 128 + wq * 32 + ii * 16 + li;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int ko = m0 + mi * 128 + grp * 64 + jj * 16 + lg * 4;
          if (col < a.Kg) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (ko + r < a.K) slab[(size_t)(ko + r) * a.Kg + col] = acc[ni][ii][mi][jj][r];
          }
        }
    }
}

// ------------------------------------------------------------------------------------------
// weight re-layouts
// dgrad weight: Wt[c][R-1-r][S-1-s][k] = W[k][r][s][c]   (bf16 -> bf16)
// one launch refreshing the flipped/transposed dgrad copies of many conv weights (after the
// optimizer step) instead of one tiny launch per conv in every backward
struct FlipDesc {
  const bf16_t* w;
  bf16_t* wt;
  int K, R, S, C;
  int st, ph, pw, pad_;  // st > 1: the stride-decomposed layout for a stride-st conv with top/left pads ph/pw
};

// Stride decomposition of a stride-st dgrad along one dimension (kernel extent R, forward pad `pad`):
// the input pixels h = st*i + a (class a) receive exactly the taps r = r0 + st*t, t < T, from dy rows
// p = i + off - t.  So class a is a stride-1 correlation of dy with those T taps (flipped) and pad
// T-1-off, no zero-dilated input (the plain dgrad multiplies st^2 - 1 of every st^2 gathered rows by 0).
__host__ __device__ __forceinline__ void dec_dim(int R, int st, int pad, int a, int& r0, int& T, int& off) {
  r0 = ((a + pad) % st + st) % st;
  T = r0 < R ? (R - r0 + st - 1) / st : 0;
  off = (a + pad - r0) / st;
}
// element offset of class (a, b)'s block [C][Tr][Tu][K] in the decomposed layout (classes a-major)
__host__ __device__ __forceinline__ size_t dec_block(int R, int S, int C, int K, int st, int ph, int pw, int a, int b) {
  size_t off = 0;
  for (int a2 = 0; a2 < st; ++a2)
    for (int b2 = 0; b2 < st; ++b2) {
      if (a2 == a && b2 == b) return off;
      int r0, Tr, o1, s0, Tu, o2;
      dec_dim(R, st, ph, a2, r0, Tr, o1);
      dec_dim(S, st, pw, b2, s0, Tu, o2);
      off += (size_t)C * K * Tr * Tu;
    }
  return off;
}
// One 64(k) x 64(c) tile of one tap through LDS: the source rows are read along c and the flipped
// destination rows written along k, both coalesced (the old per-element gather read with a stride
// of R*S*C elements: 0.17 TB/s, 2.9 ms per VGG-16 step for its 103 M-element fc6 kernel).
constexpr int FLIP_T = 64;
__device__ __forceinline__ void flip_tile(const FlipDesc& f, int tile, uint16_t (*lds)[FLIP_T + 2]) {
  const int kt = (f.K + FLIP_T - 1) / FLIP_T, ct = (f.C + FLIP_T - 1) / FLIP_T;
  const int rs = tile / (kt * ct), rem = tile % (kt * ct);
  const int k0 = (rem / ct) * FLIP_T, c0 = (rem % ct) * FLIP_T;
  const int r = rs / f.S, s = rs % f.S;
  const int rs2 = (f.R - 1 - r) * f.S + (f.S - 1 - s);  // flipped tap in the destination
  const uint16_t* w = (const uint16_t*)f.w;
  uint16_t* wt = (uint16_t*)f.wt;
  const size_t RS = (size_t)f.R * f.S;
  // destination of element (c, k): wt[(c * dRS + drs) * K + k] (+ the class block offset)
  size_t dRS = RS, drs = rs2;
  if (f.st > 1) {
    const int a = ((r - f.ph) % f.st + f.st) % f.st, b = ((s - f.pw) % f.st + f.st) % f.st;
    int r0, Tr, o1, s0, Tu, o2;
    dec_dim(f.R, f.st, f.ph, a, r0, Tr, o1);
    dec_dim(f.S, f.st, f.pw, b, s0, Tu, o2);
    const int tq = Tr - 1 - (r - r0) / f.st, uq = Tu - 1 - (s - s0) / f.st;
    wt += dec_block(f.R, f.S, f.C, f.K, f.st, f.ph, f.pw, a, b);
    dRS = (size_t)Tr * Tu;
    drs = (size_t)tq * Tu + uq;
  }
#pragma unroll 4
  for (int i = threadIdx.x; i < FLIP_T * FLIP_T; i += 256) {
    const int kk = i / FLIP_T, cc = i % FLIP_T;
    const int k = k0 + kk, c = c0 + cc;
    if (k < f.K && c < f.C) lds[kk][cc] = w[((size_t)k * RS + rs) * f.C + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int i = threadIdx.x; i < FLIP_T * FLIP_T; i += 256) {
    const int cc = i / FLIP_T, kk = i % FLIP_T;
    const int k = k0 + kk, c = c0 + cc;
    if (k < f.K && c < f.C) wt[((size_t)c * dRS + drs) * f.K + k] = lds[kk][cc];
  }
  __syncthreads();
}

__device__ __forceinline__ int flip_tiles(const FlipDesc& f) {
  return ((f.K + FLIP_T - 1) / FLIP_T) * ((f.C + FLIP_T - 1) / FLIP_T) * f.R * f.S;
}

// grid (blocks per weight, weights): each block strides over its weight's tiles
__global__ __launch_bounds__(256) void weight_flip_batched_kernel(const FlipDesc* __restrict__ descs) {
  __shared__ uint16_t lds[FLIP_T][FLIP_T + 2];
  const FlipDesc f = descs[blockIdx.y];
  const int n = flip_tiles(f);
  for (int t = blockIdx.x; t < n; t += gridDim.x) flip_tile(f, t, lds);
}

__global__ __launch_bounds__(256) void weight_flip_tiled_kernel(FlipDesc f) {
  __shared__ uint16_t lds[FLIP_T][FLIP_T + 2];
  const int n = flip_tiles(f);
  for (int t = blockIdx.x; t < n; t += gridDim.x) flip_tile(f, t, lds);
}

}  // namespace dtm

using namespace dtm;

// ------------------------------------------------------------------------------------------
// host launchers (C ABI, called through ctypes; every launch is on the caller's stream so the
// whole training step can be captured in one hipGraph)
struct ConvDesc {
  int N, H, W, C, K, R, S, P, Q, stride, pad_h, pad_w;
  int pix_bytes;  // 0 = C*2 (dense NHWC); else the input pixel pitch in bytes (packed-row stem view)
  int dec;        // dgrad only: the weight is in the stride-decomposed flipped layout (see dec_dim)
};

static const bf16_t* zero_chunk() {
  static void* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 4096) != hipSuccess) return nullptr;
    hipMemset(z, 0, 4096);
    hipDeviceSynchronize();
  }
  return (const bf16_t*)z;
}
const void* dtm_zero_chunk() { return zero_chunk(); }  // (the stem-pool kernels' out-of-range tap source)

template <int PT, int CT, int NWP, int NS, int UD, bool SPL = false, int NTH = 512>
static void launch_w8(const ConvNTArgs& a, hipStream_t st) {
  dim3 grid((a.K + CT - 1) / CT, (a.M + PT - 1) / PT, a.ngrp > 1 ? a.ngrp : 1);
  hipLaunchKernelGGL((conv_nt_w8_kernel<PT, CT, NWP, NS, UD, SPL, NTH>), grid, dim3(NTH), 0, st, a);
}

template <int UD, bool SPL = false>
static void launch_pp(const ConvNTArgs& a, hipStream_t st) {
  dim3 grid((a.K + 255) / 256, (a.M + 255) / 256, a.ngrp > 1 ? a.ngrp : 1);
  hipLaunchKernelGGL((conv_nt_pp_kernel<UD, SPL>), grid, dim3(512), 0, st, a);
}

template <int PT, int CT, int NS, int UD, int NWP = 2, bool SPL = false>
static void launch_pipe(const ConvNTArgs& a, hipStream_t st) {
  dim3 grid((a.K + CT - 1) / CT, (a.M + PT - 1) / PT, a.ngrp > 1 ? a.ngrp : 1);
  if (SPL) hipLaunchKernelGGL((conv_nt_pipe_kernel<PT, CT, NS, UD, false, NWP, true>), grid, dim3(256), 0, st, a);
  else if (a.in_scale) hipLaunchKernelGGL((conv_nt_pipe_kernel<PT, CT, NS, UD, true, NWP>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((conv_nt_pipe_kernel<PT, CT, NS, UD, false, NWP>), grid, dim3(256), 0, st, a);
}

static int device_cus() { return dtm_compute_cus(); }  // (minus the CUs reserved for RCCL: workspace.hip)

static bf16_t* dump_chunk() {
  static void* z = nullptr;
  if (!z && hipMalloc(&z, 4096) != hipSuccess) return nullptr;
  return (bf16_t*)z;
}

// persistent streaming 1x1 kernel: blocks = resident capacity (occupancy x CUs), channel tiles x
// pixel-tile workers
template <int PT, int CT, int NKT, bool PRO, bool STEM = false, int NBUF = 2, bool SIDE = true>
static int stream_workers_k(const ConvNTArgs& a) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv1x1_stream_kernel<PT, CT, NKT, PRO, STEM, NBUF, SIDE>,
                                                     256, 0) !=
            hipSuccess || occ <= 0)
      occ = 1;
  }
  const int ctiles = (a.K + CT - 1) / CT;
  const int ntiles = (a.M + PT - 1) / PT;
  int workers = (occ * device_cus() + ctiles - 1) / ctiles;
  if (workers > ntiles) workers = ntiles;
  if (workers < 1) workers = 1;
  return workers;
}

template <int PT, int CT, int NKT, bool PRO, bool STEM = false, int NBUF = 2, bool SIDE = true>
static void launch_stream_k(const ConvNTArgs& a, hipStream_t st) {
  const int ctiles = (a.K + CT - 1) / CT;
  const int ntiles = (a.M + PT - 1) / PT;
  hipLaunchKernelGGL((conv1x1_stream_kernel<PT, CT, NKT, PRO, STEM, NBUF, SIDE>),
                     dim3(ctiles, stream_workers_k<PT, CT, NKT, PRO, STEM, NBUF, SIDE>(a)), dim3(256), 0, st, a, ntiles);
}

static bool stem_stream_ok(const ConvNTArgs& a) {
  // the packed-row stem view, no prologue / bias / relu, whole 64-channel tiles, R <= 8 kernel rows
  return a.pix_bytes == 8 && a.C == 32 && a.S == 1 && a.pad_h == 0 && a.pad_w == 0 && a.Kg == a.R * 32 &&
         a.Kg <= 256 && a.K % 64 == 0 && !a.in_scale && !a.bias && !a.relu && a.ostr == 1;
}

template <int CT, int NKT>
static void launch_stream(const ConvNTArgs& a, hipStream_t st) {
  const bool side = a.add_src || a.act_x;
  if (a.in_scale) {
    if (side) launch_stream_k<64, CT, NKT, true, false, 2, true>(a, st);
    else launch_stream_k<64, CT, NKT, true, false, 2, false>(a, st);
  } else if (side) launch_stream_k<64, CT, NKT, false, false, 2, true>(a, st);
  else launch_stream_k<64, CT, NKT, false, false, 2, false>(a, st);
}
template <int CT, int NKT>
static int stream_workers(const ConvNTArgs& a) {
  const bool side = a.add_src || a.act_x;
  if (a.in_scale) return side ? stream_workers_k<64, CT, NKT, true, false, 2, true>(a)
                              : stream_workers_k<64, CT, NKT, true, false, 2, false>(a);
  if (side) return stream_workers_k<64, CT, NKT, false, false, 2, true>(a);
  return stream_workers_k<64, CT, NKT, false, false, 2, false>(a);
}

// the stem forward as a persistent stream: -1: DTM_STEM_STREAM env (default 1), 0 off, 1 on (3-slot ring),
// 2 on with the 2-slot ring (A/B knob)
static int g_stem_stream = 1;  // A/B API dtm_conv_set_stem_stream (2 = the 2-slot ring)
DTM_API void dtm_conv_set_stem_stream(int on) { g_stem_stream = on; }
// statistics partial rows of the streaming kernel (tile id 30 / 31 / 33): one per worker
static int stream_rows(const ConvNTArgs& a, int id) {
  if (id == 33) return g_stem_stream == 2 ? stream_workers_k<64, 64, 4, false, true, 2, false>(a)
                                          : stream_workers_k<64, 64, 4, false, true, 3, false>(a);
  const bool k1 = a.Kg <= 64;
  if (id == 30) {
    return k1 ? stream_workers<128, 1>(a) : stream_workers<128, 2>(a);
  }
  return k1 ? stream_workers<64, 1>(a) : stream_workers<64, 2>(a);
}

static bool stream_ok(const ConvNTArgs& a) {
  return !a.bias && !a.relu && a.R == 1 && a.S == 1 && a.stride == 1 && a.pad_h == 0 && a.pad_w == 0 && a.Hv == a.Hin && a.Wv == a.Win &&
         a.P == a.Hin && a.Q == a.Win && a.Kg % 64 == 0 && a.Kg <= 128 && a.K % 8 == 0 &&
         (!a.in_scale || a.C <= 512) && a.dump != nullptr && a.ostr == 1;
}

template <int PT, int CT, int WP, int WC, int UD, int NBUF = 2, bool SPL = false, int LBW = 0, int EG = 4>
static void launch_nt(const ConvNTArgs& a, hipStream_t st) {
  dim3 grid((a.K + CT - 1) / CT, (a.M + PT - 1) / PT, a.ngrp > 1 ? a.ngrp : 1);
  hipLaunchKernelGGL((conv_nt_kernel<PT, CT, WP, WC, UD, NBUF, SPL, LBW, EG>), grid, dim3(256), 0, st, a);
}
// Occupancy variants of the register-staged 64x128 / 128x64 tiles (A/B knobs; DTM_ACT_OCC / DTM_NT_OCC set the initial
// values): 0 = as compiled (128 VGPR + 32 AGPR: 3 waves/SIMD), 1 = epilogue side rows 2 at a time, 2 = 4 waves/SIMD
// forced (__launch_bounds__(256, 4): 128 registers, no spill), 3 = both.  The memory-bound dgrads with post-ops (the
// block-output / act dgrads, side inputs) gain from the 4th resident block: 56x56 318.9 -> 268.9 us, 28x28 178.6 ->
// 158.9, 14x14 111.5 -> 102.0, 7x7 70.2 -> 65.6, ResNet-50 step -0.99 % (profiles/r6/r6_s17_act_occ.log,
// r6_s17_ab_aocc.log); so do the plain dgrads (28x28 87.4 -> 73.7 us), while forwards with BN statistics lose
// (56x56 256 -> 64: 111.3 -> 119.0 us, r6_s17_nt_occ.log): g_nt_occ applies to launches without statistics only.
static int g_act_occ = getenv("DTM_ACT_OCC") ? atoi(getenv("DTM_ACT_OCC")) : 2;
DTM_API void dtm_conv_set_act_occ(int v) { g_act_occ = v; }
static int g_nt_occ = getenv("DTM_NT_OCC") ? atoi(getenv("DTM_NT_OCC")) : 2;
DTM_API void dtm_conv_set_nt_occ(int v) { g_nt_occ = v; }
template <int PT, int CT, int UD>
static void launch_nt_act(const ConvNTArgs& a, hipStream_t st) {
  const bool side = (a.K & 7) == 0 && (a.add_src != nullptr || a.act_x != nullptr);
  const int v = side ? g_act_occ : (a.stats ? 0 : g_nt_occ);
  if (v == 1) launch_nt<PT, CT, 32, 64, UD, 1, false, 0, 2>(a, st);
  else if (v == 2) launch_nt<PT, CT, 32, 64, UD, 1, false, 4, 4>(a, st);
  else if (v == 3) launch_nt<PT, CT, 32, 64, UD, 1, false, 4, 2>(a, st);
  else launch_nt<PT, CT, 32, 64, UD, 1>(a, st);
}

// tile variants (the ones the shape policy uses; the rejected ones and their A/B logs are listed in
// profiles/ab/README.md): 0 = 128 pix x 128 ch register-staged (4 waves 2x2 of 64x64), 3 / 4 = 128 x 64 /
// 64 x 128 register-staged with a single LDS buffer (more resident blocks), 21 / 24 / 26 / 32 = LDS-DMA
// pipelined 128x128 / 256x64 / 128x64 / 256x32, 30 / 31 = the persistent streaming 1x1 kernel (128 / 64
// channels), 40 = the 8-wave 256x256 tile.  DTM_CONV_TILE forces one (sweeps: tools/conv_tile_sweep.py).
// the direct 3x3 kernel (tile id 60): -1: DTM_DIRECT3X3 env (default 1), 0 / 1: A/B knob
static int g_direct3 = 1;  // A/B API dtm_conv_set_direct3
DTM_API void dtm_conv_set_direct3(int on) { g_direct3 = on; }
// Measured (tools/conv_tile_sweep.py, profiles/r3/r3_sweep_direct3x3.log): 32 output channels win 1.8-2.2x
// (Inception stem 3x3 32->32 fwd 108 vs 185 us, dgrads 64->32 / 32->32 185 / 100 vs 274 / 182 us); 64 output
// channels lose ~10 % (ResNet-50 56x56 64->64: 114 vs 103 us): their 1-block/CU tile is LDS-bandwidth bound
// (6 fragment reads per 8 MFMAs).  The policy takes K == 32; tile id 60 forces it for any K % 32 == 0.
static bool direct_ok(const ConvNTArgs& a) {
  return a.R == 3 && a.S == 3 && a.stride == 1 && a.Hv == a.Hin && a.Wv == a.Win && (a.C == 32 || a.C == 64) &&
         a.K % 32 == 0 && !a.in_scale && !a.bias && !a.relu && a.pix_bytes == a.C * 2 && a.ostr == 1 &&
         a.pad_h <= 2 && a.pad_w <= 2 && !a.act_mask && !a.act_r && (!a.add_src || a.add_stride == 1);
}
// spatial 8 x 16 output tiles, M = tiles * 128 (ConvNTArgs::sp_tw)
static void direct_setup(ConvNTArgs& a) {
  a.sp_tw = (a.Q + 15) / 16;
  a.sp_th = (a.P + 7) / 8;
  a.fd_sp_img = make_fastdiv(a.sp_th * a.sp_tw);
  a.fd_sp_tw = make_fastdiv(a.sp_tw);
  a.M = a.N * a.sp_th * a.sp_tw * 128;
}
template <int CIN, int CT, bool SIDE>
static int direct_workers_k(const ConvNTArgs& a) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv3x3_direct_kernel<CIN, CT, SIDE>, 256, 0) != hipSuccess ||
        occ <= 0)
      occ = 1;
  }
  const int ctiles = a.K / CT, ntiles = a.M / 128;
  int w = occ * device_cus() / ctiles;
  if (w < 1) w = 1;
  return w < ntiles ? w : ntiles;
}
template <int CIN, int CT, bool SIDE>
static void launch_direct_k(const ConvNTArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((conv3x3_direct_kernel<CIN, CT, SIDE>), dim3(a.K / CT, direct_workers_k<CIN, CT, SIDE>(a)),
                     dim3(256), 0, st, a, a.M / 128);
}
// 32-channel output tiles also for K % 64 == 0 (half the resident weights and staging: 2 blocks per CU instead of 1;
// Inception-v3's 147x147 3x3 32 -> 64 forward 269 -> 227 us, profiles/r6/r6_s29_direct_ct32.log, step
// r6_s30_ab_ct32_inception.log).  A/B knob dtm_conv_set_direct_ct32 / DTM_DIRECT_CT32=0.
static int g_direct_ct32 = getenv("DTM_DIRECT_CT32") ? atoi(getenv("DTM_DIRECT_CT32")) : 1;
DTM_API void dtm_conv_set_direct_ct32(int on) { g_direct_ct32 = on; }
#define DTM_DIRECT_SEL(FN, ...)                                                                     \
  ((a.add_src || a.act_x)                                                                          \
       ? (a.C == 64 ? FN<64, 32, true>(__VA_ARGS__) : FN<32, 32, true>(__VA_ARGS__))                 \
       : (a.C == 64 ? ((a.K % 64 == 0 && !g_direct_ct32) ? FN<64, 64, false>(__VA_ARGS__)           \
                                                        : FN<64, 32, false>(__VA_ARGS__))           \
                    : ((a.K % 64 == 0 && !g_direct_ct32) ? FN<32, 64, false>(__VA_ARGS__)           \
                                                        : FN<32, 32, false>(__VA_ARGS__))))
static int direct_workers(const ConvNTArgs& a) { return DTM_DIRECT_SEL(direct_workers_k, a); }
static void launch_direct(const ConvNTArgs& a, hipStream_t st) { DTM_DIRECT_SEL(launch_direct_k, a, st); }

struct TileCfg {
  int id, PT, NWP;
};
static int g_tile_env = -2;
static int device_cus();
static int g_policy2 = 1;  // A/B knob: the v2 shape-policy rules (dtm_conv_set_policy2)
DTM_API void dtm_conv_set_policy2(int on) { g_policy2 = on; }
static int g_tile_w8 = 1;  // A/B knob: the 8-wave tile in the shape policy (dtm_conv_set_w8)
// A/B knob: the persistent streaming kernel also for act / block-output dgrads (off: -0.4 % ResNet-50 step once
// the act sums accumulate per worker, profiles/ab/r3_ab_stream_act.log)
static int g_stream_act = 0;
DTM_API void dtm_conv_set_stream_act(int on) { g_stream_act = on; }
static int g_kwide = 1;    // A/B knob: 64-channel tiles for K % 128 in (0, 64] (dtm_conv_set_kwide)
DTM_API void dtm_conv_set_kwide(int on) { g_kwide = on; }
DTM_API void dtm_conv_set_w8(int on) { g_tile_w8 = on; }
// A/B knob: the ping-pong 256x256 tile (conv_nt_pp_kernel) in place of the 8-wave w8 tile wherever the policy picks it
// (DTM_PP=0/1 sets the initial value: profiling runs of whole programs)
static int g_tile_pp = getenv("DTM_PP") ? atoi(getenv("DTM_PP")) : 0;
DTM_API void dtm_conv_set_pp(int on) { g_tile_pp = on; }
static int g_k64_tile = 3;  // tile of the 64-output-channel layers (A/B knob: dtm_conv_set_k64_tile)
DTM_API void dtm_conv_set_k64_tile(int id) { g_k64_tile = id; }
static int g_k32_tile = 1;  // A/B knob: the 256x32 tile for <= 32-channel spatial convs (dtm_conv_set_k32)
DTM_API void dtm_conv_set_k32(int on) { g_k32_tile = on; }
static int g_act_tile = -1;  // A/B knob: tile of the dgrads with a fused activation-backward epilogue (-1 = policy)
DTM_API void dtm_conv_set_act_tile(int id) { g_act_tile = id; }
static TileCfg pick_tile_impl(const ConvNTArgs& a, bool stats);
// DTM_TILE_LOG=1: one stderr line per conv_nt launch decision (shape, side inputs, tile) for profiling runs
static TileCfg pick_tile(const ConvNTArgs& a, bool stats = false) {
  static int log = -1;
  if (log < 0) {
    const char* e = getenv("DTM_TILE_LOG");
    log = e ? atoi(e) : 0;
  }
  const TileCfg t = pick_tile_impl(a, stats);
  if (log)
    fprintf(stderr, "dtm_tile M=%d K=%d C=%d RxS=%dx%d Kg=%d st=%d ostr=%d pro=%d stats=%d add=%d act=%d mask=%d r=%d -> %d\n",
            a.M, a.K, a.C, a.R, a.S, a.Kg, a.stride, a.ostr, a.in_scale != nullptr, (int)stats, a.add_src != nullptr,
            a.act_x != nullptr, a.act_mask != nullptr, a.act_r != nullptr, t.id);
  return t;
}
static TileCfg pick_tile_impl(const ConvNTArgs& a, bool stats) {
  if (g_tile_env == -2) {
    const char* e = getenv("DTM_CONV_TILE");
    g_tile_env = e ? atoi(e) : -1;
  }
  // measured per ResNet-50 shape (tools/conv_microbench.py, DTM_CONV_TILE sweep): the single-buffer
  // variants win almost everywhere (more resident blocks hide the short-K latency); the 2-buffer
  // 128x128 tile keeps the small-M / deep-K layers (7x7 maps, K-reduction >= 2048)
  int id = g_tile_env;
  // the packed-row stem as a persistent stream (weights resident, pixel tiles prefetched)
  if (id == -1 && g_stem_stream && stem_stream_ok(a)) return {33, 64, 2};
  // narrow 3x3 stride-1 layers: the direct kernel (resident weights, halo tiles; the caller sets the
  // spatial tiling with direct_setup)
  // (dgrad post-op inputs come by LDS-DMA: with per-tile global side loads in the epilogue the compiler's waits
  // drained the halo prefetch - Inception stem dgrads 551 / 252 us vs 355 / 195 on the GEMM tiles)
  if (((id == -1 && a.K == 32) || id == 60) && g_direct3 && direct_ok(a)) return {60, 128, 4};
  // ... and the 32 -> 64 3x3 of Inception-v3's stem (147x147 at batch 128: 282.6 -> 253.0 us forward with the BN
  // statistics, profiles/r5/r5_s31_inception_stem_sweep.log; ResNet-50's 64 -> 64 layers lose on it, see above)
  if (id == -1 && a.K == 64 && a.C == 32 && !a.in_scale && g_direct3 && direct_ok(a)) return {60, 128, 4};
  // the pipelined LDS-DMA 128x128 tile (2 slots, 2 blocks/CU) wins every deep-reduction layer without the
  // prologue (tools/conv_tile_sweep.py: 3x3 at 14x14 / 7x7 -13..-18 %, deep 1x1 -5..-16 %)
  if (id == -4) id = -1;  // (-4: the policy without the streaming kernel, for A/B runs)
  else if (id == -1 && a.Kg == 64 && stream_ok(a) && (g_stream_act || !a.act_x) &&
           (!g_policy2 || a.K % 128 == 0 || a.K <= 64))  // (v2: no partial channel tiles: 35x35 ->288 -33 %)
    id = a.K >= 128 ? 30 : 31;
  if (id == -1 && a.act_x && g_act_tile >= 0) id = g_act_tile;  // (A/B: the non-streaming act dgrads)
  // (the persistent streaming 1x1 kernel: the 64-deep 56x56 expand / reduce layers and their dgrads are
  // HBM streams: -20..-33 % (tools/conv_tile_sweep.py); at Kg 128 its 1 block/CU loses)
  // the 8-wave 256x256 tile (id 40) where it fills the chip: >= ~150 tiles (one round, 58-100 % of the
  // CUs), and not on the many-tile short-reduction layers without statistics (their 4-wave tiles stream
  // better).  Measured per ResNet-50 layer (tools/conv_tile_sweep.py STATS=1, profiles/r2_conv_tiles_w8.txt):
  // 14x14 3x3 fwd/dgrad -16 %, 7x7 1024->2048 -12 %, 28x28 256->512 fwd+stats -17 %; loses at <= 98 tiles.
  // (policy v2: the w8 tile only for whole 256-channel tiles - Inception's 384 = 256 + a half-empty tile ran
  //  147 us vs 91 on 128x128)
  if (id == -1 && !a.in_scale && a.K >= 256 && g_tile_w8 && (!g_policy2 || a.K % 256 == 0)) {
    const long tiles = (long)((a.M + 255) / 256) * ((a.K + 255) / 256);
    if (tiles >= 150 && !(tiles > 600 && a.Kg <= 256 && !stats)) id = 40;
  }
  // policy v2 (A/B knob dtm_conv_set_policy2), from the Inception-v3 shape sweep
  // (profiles/r2/r2_sweep_inception.log, batch 128):
  //  * <= 64 output channels with a spatial kernel: the 2-slot pipelined 128x64 tile whatever the reduction
  //    depth (5x5 48->64: 38.5 us vs 63.6 on the 128x128 tile the Kg >= 1024 rule picked; 3x3 -> 32: -10 %)
  //  * 64 < K <= 128 with a spatial kernel: the pipelined 128x128 tile (35x35 3x3 ->96: -11 %)
  if (id == -1 && g_policy2 && !a.in_scale && a.K % 8 == 0 && a.R * a.S > 1) {
    if (a.K <= 32 && g_k32_tile) id = 32;  // (Inception's 32-channel stem 3x3s: no half-empty 64-wide tile)
    else if (a.K <= 64) id = 26;
    else if (a.K <= 128) id = 21;
  }
  // output widths that leave the last 128-channel tile at most half full (Inception's 192 / 320 / 96 /
  // 160 ...): 64-channel tiles (A/B knob dtm_conv_set_kwide); v2: 256-pixel tiles on mid-size maps
  // (17x17 at batch 128: 1x7 / 7x1 / 1x1 -> 160 / 192 -19 %), not on small ones (8x8: +33 %)
  if (id == -1 && g_kwide && a.K > 64 && a.K % 128 != 0 && (a.K % 128) <= 64 && a.K % 8 == 0)
    id = a.in_scale ? 3 : ((g_policy2 && a.M >= 16384 && (a.M <= 65536 || a.M >= 262144)) ? 24 : 26);
  // (and on the stem-size maps: Inception-v3's 73x73 3x3 80 -> 192, 324.2 -> 306.2 us with statistics,
  //  profiles/r5/r5_s31_inception_stem_sweep.log)
  if (id == -1 && !a.in_scale && a.Kg >= 1024) {
    id = 21;  // (-3: the policy without it, for A/B runs)
    // v2: no more 128x128 tiles than CUs (8x8 maps at batch 128, VGG's 4x4 at 512): 128x64 tiles fill the
    // chip (-13 %; profiles/r2/r2_sweep_vgg.log)
    if (g_policy2 && (long)((a.M + 127) / 128) * ((a.K + 127) / 128) <= device_cus()) id = 26;
  }
  // 64-output-channel 3x3 layers (56x56 bottleneck conv2, fwd and dgrad): the 2-slot pipelined 128x64 tile
  // (profiles/r2_conv_tiles_k64.txt: -4 % vs the register-staged single-buffer tile)
  if (id == -1 && !a.in_scale && a.K <= 64 && a.R * a.S > 1 && a.K % 64 == 0) id = 26;
  if (id < 0) id = a.K <= 64 ? g_k64_tile : ((a.M <= 16384 && a.Kg >= 2048) ? 0 : 4);
  // pipelined LDS-DMA tiles stage the prologue affine in LDS: C <= 512
  if ((id == 21 || id == 24 || id == 26 || id == 32) && a.in_scale && a.C > 512) id = 0;
  if (id == 21 || id == 26) return {id, 128, 2};  // 128 x 128 / 128 x 64 pipelined, 2 slots
  if (id == 24) return {id, 256, 2};              // 256 x 64 pipelined (waves 2x2 of 128x32)
  if (id == 32) return {id, 256, 4};              // 256 x 32 pipelined, waves 4x1 of 64x32
  // 8-wave 256x256 tile (waves 2x4), no prologue
  // (3-slot 8-wave 256x128 / 128x256 forms of this tile - two k-tiles in flight, 144 KiB of LDS - measured slower
  // than the 2-slot 256x256 on every ResNet-50 shape, e.g. 14x14 3x3 82.5 / 79.7 vs 65.0 us, and were removed:
  // profiles/r5/r5_tile_sweep_w8ns3.log)
  if ((id == 40 || id == 41) && a.in_scale) id = 0;
  if (id == 40 && g_tile_pp && g_tile_env != 40) id = 41;
  if (id == 41 && a.K % 8) id = 40;  // (the ping-pong tile has only the LDS-staged epilogue)
  if (id == 40 || id == 41) return {id, 256, 2};
  if (id == 30 || id == 31) {
    if (stream_ok(a)) return {id, 64, 2};
    id = a.K <= 64 ? 3 : 4;
  }
  if (id == 3) return {id, 128, 4};
  if (id == 4) return {id, 64, 2};
  return {0, 128, 2};
}

// merged-sibling forwards (split store; no prologue, stride-1 1x1): the tiles conv_fwd_impl lets through
static void dispatch_split(const ConvNTArgs& a, const TileCfg& t, hipStream_t st) {
  if (t.id == 3) launch_nt<128, 64, 32, 64, 1, 1, true>(a, st);
  else if (t.id == 4) launch_nt<64, 128, 32, 64, 1, 1, true>(a, st);
  else if (t.id == 21) launch_pipe<128, 128, 2, 1, 2, true>(a, st);
  else if (t.id == 24) launch_pipe<256, 64, 2, 1, 2, true>(a, st);
  else if (t.id == 26) launch_pipe<128, 64, 2, 1, 2, true>(a, st);
  else if (t.id == 32) launch_pipe<256, 32, 2, 1, 4, true>(a, st);
  else if (t.id == 40) launch_w8<256, 256, 2, 2, 1, true>(a, st);
  else if (t.id == 41) launch_pp<1, true>(a, st);
  else launch_nt<128, 128, 64, 64, 1, 2, true>(a, st);
}

template <int UD>
static void dispatch_ud(const ConvNTArgs& a, const TileCfg& t, hipStream_t st) {
  if (UD == 1 && a.nsplit > 0) dispatch_split(a, t, st);
  else if (t.id == 3) launch_nt_act<128, 64, UD>(a, st);
  else if (t.id == 4) launch_nt_act<64, 128, UD>(a, st);
  else if (t.id == 30 && UD == 1) {
    if (a.Kg <= 64) launch_stream<128, 1>(a, st);
    else launch_stream<128, 2>(a, st);
  } else if (t.id == 60 && UD == 1) {
    launch_direct(a, st);
  } else if (t.id == 33 && UD == 1) {
    if (g_stem_stream == 2) launch_stream_k<64, 64, 4, false, true, 2, false>(a, st);  // (A/B: 2-slot ring)
    else launch_stream_k<64, 64, 4, false, true, 3, false>(a, st);
  } else if (t.id == 31 && UD == 1) {
    if (a.Kg <= 64) launch_stream<64, 1>(a, st);
    else launch_stream<64, 2>(a, st);
  } else if (t.id == 21) launch_pipe<128, 128, 2, UD>(a, st);
  else if (t.id == 24) launch_pipe<256, 64, 2, UD>(a, st);
  else if (t.id == 26) launch_pipe<128, 64, 2, UD>(a, st);
  else if (t.id == 32) launch_pipe<256, 32, 2, UD, 4>(a, st);   // waves 4x1 of 64x32 (32-channel outputs)
  else if (t.id == 40) launch_w8<256, 256, 2, 2, UD>(a, st);
  else if (t.id == 41) launch_pp<UD>(a, st);
  // (a stream-K form of this tile for the < 2-round grids - ResNet-50's 196-tile 14x14 layers - was correct but slower:
  //  a 256x256 fp32 partial is 256 KiB of slab traffic per hand-off; profiles/ab/r5_ab_stream_k_w8.log)
  else launch_nt<128, 128, 64, 64, UD>(a, st);
}

// tile override for A/B tests (-1 = the shape policy), same as DTM_CONV_TILE
DTM_API void dtm_conv_set_tile(int id) { g_tile_env = id; }

static void dispatch_nt(const ConvNTArgs& a, int ud, const TileCfg& t, hipStream_t st) {
  if (ud == 1) dispatch_ud<1>(a, t, st);
  else dispatch_ud<2>(a, t, st);
}

DTM_API int dtm_get_deterministic();

static int g_split_tile = 1;  // A/B knob: the merged-head tile rule in conv_fwd_impl (dtm_conv_set_split_tile)
DTM_API void dtm_conv_set_split_tile(int on) { g_split_tile = on; }

static int conv_fwd_impl(const void* x, const void* w, void* y, bool stats, const float* bias, const float* in_scale,
                         const float* in_shift, int relu, const ConvDesc* d, hipStream_t stream, float** rows_ws,
                         int* nrows, const ConvNTArgs::Split* split = nullptr, int nsplit = 0) {
  if (!dtm_device_ok()) return -9;
  if (d->C % 8 || d->K % 4) return -1;
  ConvNTArgs a;
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.y = (bf16_t*)y;
  a.ngrp = 0;
  a.nsplit = 0;
  a.stats = nullptr; a.bias = bias; a.in_scale = in_scale; a.in_shift = in_shift;
  a.add_src = nullptr; a.act_x = nullptr; a.act_ss = nullptr; a.act_sums = nullptr;
  a.act_mask = nullptr; a.act_r = nullptr;
  a.add_stride = 1; a.add_H = a.add_W = 0;
  a.act_unscaled = 0;
  a.zero = zero_chunk();
  a.dump = dump_chunk();
  a.pix_bytes = d->pix_bytes > 0 ? d->pix_bytes : d->C * 2;
  size_t xb = (size_t)d->N * d->H * d->W * a.pix_bytes, wb = (size_t)d->K * d->R * d->S * d->C * 2;
  if (xb >= (1ull << 31) || wb >= (1ull << 31)) return -2;
  a.x_bytes = (uint32_t)xb; a.w_bytes = (uint32_t)wb;
  a.N = d->N; a.Hin = d->H; a.Win = d->W; a.C = d->C; a.K = d->K; a.R = d->R; a.S = d->S;
  a.P = d->P; a.Q = d->Q; a.stride = d->stride; a.pad_h = d->pad_h; a.pad_w = d->pad_w;
  a.Hv = d->H; a.Wv = d->W;
  a.M = d->N * d->P * d->Q; a.Kg = d->R * d->S * d->C; a.relu = relu;
  a.fd_PQ = make_fastdiv(d->P * d->Q); a.fd_Q = make_fastdiv(d->Q);
  a.ostr = 1; a.oa = a.ob = 0; a.OH = a.P; a.OW = a.Q;
  a.sp_tw = a.sp_th = 0;
  if (nsplit > 0) {
    if (nsplit > 8 || d->K % 8) return -1;
    a.nsplit = nsplit;
    for (int i = 0; i < nsplit; ++i) {
      if (split[i].off % 8 || split[i].K % 8) return -1;
      a.split[i] = split[i];
    }
  }
  int rows = 0;
  TileCfg tc = pick_tile(a, stats);
  // (merged-sibling stores happen in the LDS-staged epilogue only: K % 8 == 0 above; the persistent / direct
  // kernels have their own store paths, so a split launch the policy sends there takes the 64x128 tile instead)
  if (nsplit > 0 && (tc.id == 30 || tc.id == 31 || tc.id == 33 || tc.id == 60)) tc = {4, 64, 2};
  // merged heads: the pipelined 128x128 tile unless the policy took the 8-wave one - measured on every Inception-v3
  // head shape (tools/split_tile_sweep.py, profiles/r4/r4_split_tile_sweep.log): 799 -> ~765 us per step, e.g.
  // 17x17 768 -> 640 85 -> 77 us, 35x35 288 -> 240 84 -> 80 us (the policy's 64x128 / 128x64 picks)
  if (nsplit > 0 && g_split_tile && g_tile_env < 0 && tc.id != 40 && tc.id != 21) tc = {21, 128, 2};
  if (tc.id == 60) direct_setup(a);
  if (stats) {
    // one per streaming / direct worker; one per pixel tile (staged epilogue, K % 8 == 0); else per (pixel
    // tile, pixel wave)
    rows = tc.id == 60 ? direct_workers(a)
           : (tc.id == 30 || tc.id == 31 || tc.id == 33) ? stream_rows(a, tc.id)
                                                          : ((a.M + tc.PT - 1) / tc.PT) * ((a.K & 7) == 0 ? 1 : tc.NWP);
    float* ws = dtm_ws_get_stream((size_t)rows * 2 * d->K, stream);
    if (!ws) return -4;
    a.stats = ws;
  }
  dispatch_nt(a, 1, tc, stream);
  *rows_ws = a.stats;
  *nrows = rows;
  return 0;
}

DTM_API int dtm_conv_fwd(const void* x, const void* w, void* y, float* stats, const float* bias,
                         const float* in_scale, const float* in_shift, int relu,
                         const ConvDesc* d, void* stream) {
  float* ws = nullptr;
  int rows = 0;
  int rc = conv_fwd_impl(x, w, y, stats != nullptr, bias, in_scale, in_shift, relu, d, (hipStream_t)stream, &ws, &rows);
  if (rc) return rc;
  if (stats) dtm_reduce_rows(ws, rows, 2 * d->K, 2 * d->K, stats, (hipStream_t)stream);
  return 0;
}

// Merged sibling 1x1 convs on one input (ops/fused.py _SiblingGroup, Inception mixed-block branch heads): ONE conv
// over the members' concatenated weights w [sum K][1][1][C] (d->K = sum K) storing each member's output in its own
// tensor (ys[j], K_j channels), the BatchNorm statistics of all columns from its epilogue, and ONE finalize writing
// every BN member's ss / moving statistics (bn_ptrs[j] = {gamma, beta, mov_mean, mov_var, ss} or ss = 0 for a
// member without BatchNorm).  Instead of one conv + one finalize launch per member.
DTM_API int dtm_conv_fwd_bn_multi(const void* x, const void* w, void* const* ys, const int* ks, int n,
                                  void* const* bn_ptrs, float count, float eps, float decay, int update, int bessel,
                                  const ConvDesc* d, void* stream) {
  if (n < 1 || n > 8) return -1;
  ConvNTArgs::Split sp[8];
  FinGroup fg;
  fg.n = n;
  int off = 0;
  for (int i = 0; i < n; ++i) {
    sp[i].y = (bf16_t*)ys[i];
    sp[i].off = off;
    sp[i].K = ks[i];
    FinMember& m = fg.m[i];
    m.gamma = (const float*)bn_ptrs[5 * i];
    m.beta = (const float*)bn_ptrs[5 * i + 1];
    m.mov_mean = (float*)bn_ptrs[5 * i + 2];
    m.mov_var = (float*)bn_ptrs[5 * i + 3];
    m.out = (float*)bn_ptrs[5 * i + 4];
    m.off = off;
    m.K = ks[i];
    off += ks[i];
  }
  for (int i = n; i < 8; ++i) fg.m[i] = fg.m[0];
  if (off != d->K || d->R != 1 || d->S != 1) return -1;
  float* ws = nullptr;
  int rows = 0;
  int rc = conv_fwd_impl(x, w, nullptr, true, nullptr, nullptr, nullptr, 0, d, (hipStream_t)stream, &ws, &rows, sp, n);
  if (rc) return rc;
  return dtm_bn_stats_finalize_g(ws, rows, d->K, nullptr, nullptr, nullptr, nullptr, nullptr, count, eps, decay, update,
                                 bessel, (hipStream_t)stream, &fg);
}

// Training conv -> BatchNorm statistics -> finalize in two launches: the conv (statistics partial
// rows from its epilogue) and stats_reduce_finalize, which writes ss = [scale; shift; mean; rstd] and
// updates the moving averages (see batchnorm.hip).
DTM_API int dtm_conv_fwd_bn(const void* x, const void* w, void* y, const float* in_scale, const float* in_shift,
                            const float* gamma, const float* beta, float* mov_mean, float* mov_var, float* ss,
                            float count, float eps, float decay, int update, int bessel, const ConvDesc* d,
                            void* stream) {
  float* ws = nullptr;
  int rows = 0;
  int rc = conv_fwd_impl(x, w, y, true, nullptr, in_scale, in_shift, 0, d, (hipStream_t)stream, &ws, &rows);
  if (rc) return rc;
  return dtm_bn_stats_finalize(ws, rows, d->K, gamma, beta, mov_mean, mov_var, ss, count, eps, decay, update, bessel,
                               (hipStream_t)stream);
}

// dgrad: dx[N][H][W][C] from dy[N][P][Q][K] and the flipped/transposed weight wt[C][R][S][K].
// Optional epilogue post-ops (nullptr = off):
//   add_src [N][H][W][C]: dx += add_src (gradient of the same input from its other consumer);
//   add_stride > 1: add_src is [N][(H-1)/s+1][(W-1)/s+1][C], the gradient of x[:, ::s, ::s] (a 1x1
//   stride-s subsample shortcut), added at the pixels that subsample read;
//   act_x [N][H][W][C] + act_ss [4][C] (scale, shift, ...): the input was relu(act_x*scale+shift)
//   (BatchNorm+ReLU fused into this conv's forward prologue); dx <- [act_x*scale+shift>0]*dx*scale and
//   act_sums[2][C] += (sum g*act_x, sum g) with g the masked gradient (the BN scale/shift grads).
// Block-output form (dtm_conv_dgrad_bnout): the input of this conv was y = relu(bn(act_x) [+ bn(act_r) |
// + identity]) with the ReLU mask kept as a bitmask; the epilogue applies that BN-apply's backward to
// the total input gradient (dgrad + add_src): dx <- g = (dgrad + add_src) * bit, act_sums[0..1][C] +=
// (sum g*act_x, sum g) and, with act_r, act_sums[4..5][C] += (sum g*act_r, sum g) - the separate
// bn_apply_bwd pass over the block output (read d(out), mask and act_x, write g) disappears.
static int conv_dgrad_impl(const void* dy, const void* wt, void* dx, const ConvDesc* d, const void* add_src,
                           int add_stride, const void* act_x, const float* act_ss, float* act_sums, int act_unscaled,
                           const void* act_mask, const void* act_r, void* stream);

DTM_API int dtm_conv_dgrad_bnout(const void* dy, const void* wt, void* dx, const ConvDesc* d, const void* add_src,
                                 int add_stride, const void* mask, const void* x_raw, const void* r_raw, float* sums,
                                 void* stream) {
  if (!mask || !x_raw || !sums) return -7;
  return conv_dgrad_impl(dy, wt, dx, d, add_src, add_stride, x_raw, nullptr, sums, 1, mask, r_raw, stream);
}

DTM_API int dtm_conv_dgrad_ex(const void* dy, const void* wt, void* dx, const ConvDesc* d, const void* add_src,
                              int add_stride, const void* act_x, const float* act_ss, float* act_sums,
                              int act_unscaled, void* stream) {
  return conv_dgrad_impl(dy, wt, dx, d, add_src, add_stride, act_x, act_ss, act_sums, act_unscaled, nullptr, nullptr,
                         stream);
}

// A/B knob (dtm_conv_set_dec_group): the parity classes of a stride-decomposed dgrad as one grouped launch
static int g_dec_group = 1;
DTM_API void dtm_conv_set_dec_group(int on) { g_dec_group = on; }
static int g_dec_lpt = 1;  // A/B knob: the grouped classes in descending tap count (dtm_conv_set_dec_lpt)
DTM_API void dtm_conv_set_dec_lpt(int on) { g_dec_lpt = on; }
// Tile of a grouped strided dgrad, chosen for the whole grouped grid rather than for its heaviest class alone (that
// class's own rule sees a quarter of the tiles).  Measured per tile on the ResNet-50 stride-2 3x3 dgrads
// (tools/conv_microbench.py STRIDED=1 DTM_CONV_TILE sweep, profiles/r4/r4_strided_dgrad_tiles.log): 256 output
// channels (dx 14x14) the 8-wave 256x256 tile 41 us vs 49 on the per-class pick (MIOpen 42), 128 channels (dx
// 28x28) the pipelined 128x64 tile 51 vs 57 (MIOpen 50-53), 64 channels (dx 56x56) already 128x64.
// A/B knob dtm_conv_set_dec_tile.
static int g_dec_tile = 1;
DTM_API void dtm_conv_set_dec_tile(int on) { g_dec_tile = on; }

static int conv_dgrad_impl(const void* dy, const void* wt, void* dx, const ConvDesc* d, const void* add_src,
                           int add_stride, const void* act_x, const float* act_ss, float* act_sums, int act_unscaled,
                           const void* act_mask, const void* act_r, void* stream) {
  if (!dtm_device_ok()) return -9;
  if (d->K % 8 || d->C % 4) return -1;
  if (add_stride < 1 || (add_stride > 1 && !add_src)) return -6;
  if ((add_src || act_x) && d->C % 8) return -5;
  ConvNTArgs a;
  a.x = (const bf16_t*)dy; a.w = (const bf16_t*)wt; a.y = (bf16_t*)dx;
  a.ngrp = 0;
  a.nsplit = 0;
  a.stats = nullptr; a.bias = nullptr; a.in_scale = nullptr; a.in_shift = nullptr;
  a.add_src = (const bf16_t*)add_src; a.act_x = (const bf16_t*)act_x; a.act_ss = act_ss; a.act_sums = nullptr;
  a.act_mask = (const uint8_t*)act_mask; a.act_r = (const bf16_t*)act_r;
  a.add_stride = add_stride;
  a.act_unscaled = act_unscaled;
  a.zero = zero_chunk();
  a.dump = dump_chunk();
  a.add_H = (d->H - 1) / add_stride + 1; a.add_W = (d->W - 1) / add_stride + 1;
  a.pix_bytes = d->K * 2;
  a.sp_tw = a.sp_th = 0;
  size_t xb = (size_t)d->N * d->P * d->Q * d->K * 2, wb = (size_t)d->K * d->R * d->S * d->C * 2;
  if (xb >= (1ull << 31) || wb >= (1ull << 31)) return -2;
  a.x_bytes = (uint32_t)xb; a.w_bytes = (uint32_t)wb;
  a.N = d->N; a.Hin = d->P; a.Win = d->Q; a.C = d->K; a.K = d->C; a.relu = 0;
  a.stride = 1;
  a.Hv = d->P; a.Wv = d->Q;
  a.OH = d->H; a.OW = d->W;
  const int rw = act_r ? 4 : 2;
  // launches: one plain dgrad over the zero-dilated dy (UD = stride), or (d->dec, stride > 1) one stride-1
  // conv per output parity class (a, b) with that class's taps of the decomposed weight (dec_dim)
  const int st = d->stride;
  const bool dec = d->dec && st > 1;
  if (!dec && st > 2) return -3;
  if (dec && (d->R < st || d->S < st)) return -8;  // a class without taps (1x1 strided): caller falls back
  ConvNTArgs la[16];
  TileCfg lt[16];
  int lrows[16], nl = 0, rows = 0;
  for (int ca = 0; ca < (dec ? st : 1); ++ca)
    for (int cb = 0; cb < (dec ? st : 1); ++cb) {
      ConvNTArgs b = a;
      if (dec) {
        int r0, Tr, offa, s0, Tu, offb;
        dec_dim(d->R, st, d->pad_h, ca, r0, Tr, offa);
        dec_dim(d->S, st, d->pad_w, cb, s0, Tu, offb);
        const int Hc = (d->H - ca + st - 1) / st, Wc = (d->W - cb + st - 1) / st;
        if (Hc <= 0 || Wc <= 0) continue;
        b.w = (const bf16_t*)wt + dec_block(d->R, d->S, d->C, d->K, st, d->pad_h, d->pad_w, ca, cb);
        b.R = Tr; b.S = Tu;
        b.P = Hc; b.Q = Wc;
        b.pad_h = Tr - 1 - offa; b.pad_w = Tu - 1 - offb;
        b.ostr = st; b.oa = ca; b.ob = cb;
      } else {
        b.R = d->R; b.S = d->S;
        b.P = d->H; b.Q = d->W;
        b.pad_h = d->R - 1 - d->pad_h; b.pad_w = d->S - 1 - d->pad_w;
        b.Hv = (d->P - 1) * st + 1; b.Wv = (d->Q - 1) * st + 1;
        b.ostr = 1; b.oa = b.ob = 0;
      }
      b.M = d->N * b.P * b.Q; b.Kg = b.R * b.S * d->K;
      b.fd_PQ = make_fastdiv(b.P * b.Q); b.fd_Q = make_fastdiv(b.Q);
      lt[nl] = pick_tile(b);
      if (lt[nl].id == 60) direct_setup(b);
      // act partial rows: one per pixel tile, or one per worker for the persistent kernels
      lrows[nl] = lt[nl].id == 60 ? direct_workers(b)
                  : (lt[nl].id == 30 || lt[nl].id == 31) ? stream_rows(b, lt[nl].id)
                                                         : (b.M + lt[nl].PT - 1) / lt[nl].PT;
      rows += lrows[nl];
      la[nl++] = b;
    }
  // the parity classes of a stride-decomposed dgrad as ONE grouped launch (z = class) on the tile of the class
  // with the most taps, when they share the output grid (even H, W) and that tile is a grouped-capable kernel
  int gi = -1;
  if (dec && nl > 1 && nl <= 4 && g_dec_group) {
    gi = 0;
    for (int i = 1; i < nl; ++i) {
      if (la[i].M != la[0].M || la[i].P != la[0].P || la[i].Q != la[0].Q) gi = -2;
      if (gi >= 0 && la[i].Kg > la[gi].Kg) gi = i;
    }
    int id = gi >= 0 ? lt[gi].id : -1;
    if (gi >= 0 && g_dec_tile && (id == 21 || id == 26) && g_tile_env < 0 && g_act_tile < 0) {
      if (la[gi].K % 256 == 0 && g_tile_w8) lt[gi] = {g_tile_pp ? 41 : 40, 256, 2};
      else if (la[gi].K <= 128) lt[gi] = {26, 128, 2};
      id = lt[gi].id;
    }
    if (!(id == 0 || id == 3 || id == 4 || id == 21 || id == 24 || id == 26 || id == 32 || id == 40 || id == 41)) gi = -1;
    if (gi >= 0) {  // every class on that tile: one partial-sum row per pixel tile of it
      rows = 0;
      for (int i = 0; i < nl; ++i) {
        lt[i] = lt[gi];
        lrows[i] = (la[i].M + lt[gi].PT - 1) / lt[gi].PT;
        rows += lrows[i];
      }
    }
  }
  float* ws = nullptr;
  if (act_x) {
    ws = dtm_ws_get_stream((size_t)rows * rw * d->C, (hipStream_t)stream);
    if (!ws) return -4;
  }
  for (int i = 0, r = 0; i < nl; r += lrows[i], ++i)
    // every launch's partial-sum rows go to its own slice of one table, reduced together below
    if (act_x) la[i].act_sums = ws + (size_t)r * rw * d->C;
  if (gi >= 0) {
    ConvNTArgs g = la[gi];
    g.ngrp = nl;
    // classes in descending tap count: blocks are dispatched roughly in grid order and z-slice g covers the g-th
    // block range, so the heaviest class (4 of a 3x3's 9 taps at stride 2) starts first and the 1-tap class fills
    // the tail (longest-processing-time order) instead of the reverse
    int ord[4] = {0, 1, 2, 3};
    for (int i = 1; i < nl; ++i)
      for (int j = i; j > 0 && la[ord[j]].Kg > la[ord[j - 1]].Kg; --j) {
        const int t = ord[j];
        ord[j] = ord[j - 1];
        ord[j - 1] = t;
      }
    for (int q = 0; q < nl; ++q) {
      const int i = g_dec_lpt ? ord[q] : q;
      g.grp[q] = {la[i].w, la[i].act_sums, la[i].R, la[i].S, la[i].pad_h, la[i].pad_w, la[i].oa, la[i].ob, la[i].Kg};
    }
    dispatch_nt(g, 1, lt[gi], (hipStream_t)stream);
  } else {
    for (int i = 0; i < nl; ++i) dispatch_nt(la[i], dec ? 1 : st, lt[i], (hipStream_t)stream);
  }
  if (act_x && act_r) {
    // [sum g*x | sum g] -> act_sums rows 0-1, [sum g*r | sum g] -> rows 4-5 of an [8][C] buffer: rows 0-3
    // and 4-7 are then directly the ss gradients of the two BatchNorms (no copies)
    dtm_reduce_rows(ws, rows, 2 * d->C, rw * d->C, act_sums, (hipStream_t)stream);
    dtm_reduce_rows(ws + 2 * d->C, rows, 2 * d->C, rw * d->C, act_sums + 4 * d->C, (hipStream_t)stream);
  } else if (act_x) {
    dtm_reduce_rows(ws, rows, rw * d->C, rw * d->C, act_sums, (hipStream_t)stream);
  }
  return 0;
}

DTM_API int dtm_conv_dgrad(const void* dy, const void* wt, void* dx, const ConvDesc* d, void* stream) {
  return dtm_conv_dgrad_ex(dy, wt, dx, d, nullptr, 1, nullptr, nullptr, nullptr, 0, stream);
}

template <int MT, int NT, int WM, int WN, int NBUF = 2>
static void launch_wgrad(const ConvWgradArgs& a, int splits, hipStream_t st) {
  dim3 grid((a.Kg + NT - 1) / NT, (a.K + MT - 1) / MT, splits);
  hipLaunchKernelGGL((conv_wgrad_kernel<MT, NT, WM, WN, NBUF>), grid, dim3(256), 0, st, a);
}

// wgrad tile override (-1 = policy) and the blocks-per-CU target of the split count for the pipelined
// kernels (A/B sweeps: tools/conv_tile_sweep.py)
static int g_wgrad_env = -2;
static int g_wgrad_occ = 4;
static int g_wgrad_k64 = 1;  // A/B knob (dtm_conv_set_wgrad_k64): the 64 x 256 pipelined tile for K % 128 != 0
DTM_API void dtm_conv_set_wgrad_k64(int on) { g_wgrad_k64 = on; }
static int g_stem_bna = 1;  // A/B knob: the stem's BN-fused weight gradient on the pipelined tile 15 (dtm_conv_set_stem_bna)
DTM_API void dtm_conv_set_stem_bna(int on) { g_stem_bna = on; }
DTM_API void dtm_conv_set_wgrad_tile(int id, int occ) {
  g_wgrad_env = id;
  if (occ > 0) g_wgrad_occ = occ;
}

struct WgradBN {
  const void* y;
  const float *dss, *ss, *gamma;
  float count;
  float *dgamma, *dbeta;
};

struct WgradDst {  // row-split destinations of one wgrad: rows [r0, r0 + rows) of dW go to dw (ops/fused.py siblings)
  float* const* dw;
  const int* rows;
  int n;
};
static int conv_wgrad_impl(const void* x, const void* dy, float* dw, const float* in_scale, const float* in_shift,
                           const ConvDesc* d, int num_cus, const WgradBN* bn, void* stream,
                           const WgradDst* dst = nullptr);

// direct 3x3 weight gradient (conv3x3_wgrad_direct_kernel) on maps of at least g_wgrad_direct_min pixels
static int g_wgrad_direct = getenv("DTM_WGRAD_DIRECT") ? atoi(getenv("DTM_WGRAD_DIRECT")) : 1;
static int g_wgrad_direct_min = 2500;
DTM_API void dtm_conv_set_wgrad_direct(int on, int min_pixels) {
  g_wgrad_direct = on;
  if (min_pixels > 0) g_wgrad_direct_min = min_pixels;
}
template <int CIN, int KT>
static int wgrad_direct_k(ConvWgradArgs& a, const ConvDesc* d, int num_cus, hipStream_t st, float* dw) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv3x3_wgrad_direct_kernel<CIN, KT>, 256, 0) !=
            hipSuccess ||
        occ <= 0)
      occ = 1;
  }
  const int tiles_w = (d->Q + 15) / 16, tiles_h = (d->P + 7) / 8, tiles_img = tiles_h * tiles_w;
  const long ntiles = (long)d->N * tiles_img;
  if (ntiles >= (1l << 31)) return -2;
  const int ktiles = d->K / KT;
  long workers = (long)occ * num_cus / ktiles;
  if (workers < 1) workers = 1;
  if (workers > ntiles) workers = ntiles;
  float* ws = dtm_ws_get_stream((size_t)workers * a.K * a.Kg, st);
  if (!ws) return -4;
  a.dw = ws;
  hipLaunchKernelGGL((conv3x3_wgrad_direct_kernel<CIN, KT>), dim3(ktiles, (unsigned)workers), dim3(256), 0, st, a,
                     (int)ntiles, tiles_w, tiles_img);
  dtm_reduce_rows(ws, (int)workers, a.K * a.Kg, a.K * a.Kg, dw, st);  // dW += sum over the workers' slabs
  return 0;
}
static int g_wgrad_direct_kt = 64;  // dW rows per block when K % 64 == 0 (A/B: dtm_conv_set_wgrad_direct_kt)
DTM_API void dtm_conv_set_wgrad_direct_kt(int kt) { g_wgrad_direct_kt = kt; }
static int wgrad_direct(ConvWgradArgs& a, const ConvDesc* d, int num_cus, hipStream_t st, float* dw) {
  const bool k64 = d->K % 64 == 0 && g_wgrad_direct_kt == 64;
  if (d->C == 32) return k64 ? wgrad_direct_k<32, 64>(a, d, num_cus, st, dw) : wgrad_direct_k<32, 32>(a, d, num_cus, st, dw);
  return k64 ? wgrad_direct_k<64, 64>(a, d, num_cus, st, dw) : wgrad_direct_k<64, 32>(a, d, num_cus, st, dw);
}

DTM_API int dtm_conv_wgrad(const void* x, const void* dy, float* dw, const float* in_scale,
                           const float* in_shift, const ConvDesc* d, int num_cus, void* stream) {
  return conv_wgrad_impl(x, dy, dw, in_scale, in_shift, d, num_cus, nullptr, stream);
}

// Weight gradient of a conv followed by a training BatchNorm whose stats-combine output (comb) has no
// other reader (the stem: no input gradient): comb is formed in the A-operand staging from g = the
// BN output's unscaled gradient and y = the raw conv output, and dgamma / dbeta are accumulated.
DTM_API int dtm_conv_wgrad_bnbwd(const void* x, const void* g, const void* y, const float* dss, const float* ss,
                                 const float* gamma, float count, float* dgamma, float* dbeta, float* dw,
                                 const ConvDesc* d, int num_cus, void* stream) {
  WgradBN bn{y, dss, ss, gamma, count, dgamma, dbeta};
  return conv_wgrad_impl(x, g, dw, nullptr, nullptr, d, num_cus, &bn, stream);
}

// dW of several convs that read the same input, from one wgrad over their output gradients laid side by side
// (dy [M][sum K_i]): the split-K slabs' row ranges are reduced into each conv's own dW (n <= 8)
DTM_API int dtm_conv_wgrad_multi(const void* x, const void* dy, float* const* dws, const int* rows, int n,
                                 const ConvDesc* d, int num_cus, void* stream) {
  if (n < 1 || n > 8) return -1;
  int tot = 0;
  for (int i = 0; i < n; ++i) tot += rows[i];
  if (tot != d->K) return -1;
  WgradDst dst{dws, rows, n};
  return conv_wgrad_impl(x, dy, dws[0], nullptr, nullptr, d, num_cus, nullptr, stream, &dst);
}

static int conv_wgrad_impl(const void* x, const void* dy, float* dw, const float* in_scale, const float* in_shift,
                           const ConvDesc* d, int num_cus, const WgradBN* bn, void* stream, const WgradDst* dst) {
  if (!dtm_device_ok()) return -9;
  if (d->C % 8 || d->K % 8) return -1;
  ConvWgradArgs a;
  a.x = (const bf16_t*)x; a.dy = (const bf16_t*)dy; a.dw = dw;
  a.in_scale = in_scale; a.in_shift = in_shift;
  a.ay = bn ? (const bf16_t*)bn->y : nullptr;
  a.dss = bn ? bn->dss : nullptr; a.ss = bn ? bn->ss : nullptr; a.gamma = bn ? bn->gamma : nullptr;
  a.count = bn ? bn->count : 0.f; a.dgamma = bn ? bn->dgamma : nullptr; a.dbeta = bn ? bn->dbeta : nullptr;
  a.pix_bytes = d->pix_bytes > 0 ? d->pix_bytes : d->C * 2;
  size_t xb = (size_t)d->N * d->H * d->W * a.pix_bytes, yb = (size_t)d->N * d->P * d->Q * d->K * 2;
  if (xb >= (1ull << 31) || yb >= (1ull << 31)) return -2;
  a.x_bytes = (uint32_t)xb; a.dy_bytes = (uint32_t)yb;
  a.N = d->N; a.H = d->H; a.W = d->W; a.C = d->C; a.K = d->K; a.R = d->R; a.S = d->S;
  a.P = d->P; a.Q = d->Q; a.stride = d->stride; a.pad_h = d->pad_h; a.pad_w = d->pad_w;
  a.Mpix = d->N * d->P * d->Q; a.Kg = d->R * d->S * d->C;
  a.fd_PQ = make_fastdiv(d->P * d->Q); a.fd_Q = make_fastdiv(d->Q);
  // wgrad tile variants: 0 = 128 (K) x 128 (RSC) register-staged, 1 = 64 x 128, 6 = 32 x 128, 11 = the pipelined
  // LDS-DMA 64 x 256, 10 = the
  // pipelined LDS-DMA 128 x 128, 12 = the 8-wave pipelined 256 x 256 (the rejected variants and their A/B
  // logs: profiles/ab/README.md).  dtm_conv_set_wgrad_tile forces one (A/B experiments).
  if (g_wgrad_env == -2) g_wgrad_env = -1;
  const int wenv = g_wgrad_env;
  // the direct 3x3 kernel (conv3x3_wgrad_direct_kernel; tile id 20 forces it where it applies)
  // (automatic for 32 input channels: Inception-v3's 147x147 3x3 32 -> 32 / 64, 238 -> 162 / 277 -> 216 us, with the
  //  BN-apply prologue 386 -> 199 / 407 -> 247 us; 64 channels lose on ResNet-50's 56x56 64 -> 64, 144 -> 187 us without
  //  the prologue, 218 vs 223 with it: profiles/r6/r6_s33_wdirect_sweep.log)
  if ((wenv == 20 || (wenv == -1 && g_wgrad_direct && d->C == 32)) && !bn && !dst && d->R == 3 && d->S == 3 &&
      d->stride == 1 && (d->C == 32 || d->C == 64) && d->K % 32 == 0 && a.pix_bytes == d->C * 2 && d->pad_h <= 2 &&
      d->pad_w <= 2 &&
      d->P == d->H + 2 * d->pad_h - 2 && d->Q == d->W + 2 * d->pad_w - 2 &&
      (d->H * d->W >= g_wgrad_direct_min || wenv == 20))
    return wgrad_direct(a, d, num_cus, (hipStream_t)stream, dw);
  int wt = wenv >= 0 ? wenv : (d->K <= 64 ? 1 : 0);
  // <= 32 output channels: 32-row tiles (no half-empty 64-row tile; A/B knob dtm_conv_set_k32)
  if (wenv == -1 && wt == 1 && d->K <= 32 && g_k32_tile) wt = 6;
  int occ = g_wgrad_occ;
  // policy (tools/conv_tile_sweep.py WTILES sweep, ResNet-50 shapes): the pipelined kernel at 2 blocks
  // per CU wins every layer with K > 64 (-10..-25 %); 4 blocks' worth of splits for the deep 3x3 7x7s
  if (wenv == -1 && !in_scale && d->K > 64) {  // (-3: the policy without it, for A/B runs)
    wt = 10;
    occ = (d->R * d->S > 1 && a.Mpix <= 16384) ? 4 : 2;
    // the 8-wave 256x256 tile on the wide deep-reduction layers (profiles/r2_wgrad_tiles_w8.txt:
    // 14x14 / 7x7 3x3 -8..-13 %, 7x7 1024->2048 -7 %; it loses on every K < 256 or short-RSC layer)
    if (g_tile_w8 && d->K >= 256 && a.Kg >= 1024 && (d->R * d->S > 1 || d->K >= 1024)) wt = 12;
    // (per-shape wins of the 256x256 tile on Inception's 17x17 1x7 / 7x1 layers and of 128x128 on its 8x8 1x3 / 3x1
    //  ones, profiles/r5/r5_s37_wgrad_occ_sweep.log, measured neutral on the step together: not adopted)
    // merged sibling heads (one wgrad over several 1x1 convs' output gradients, dst): the 256 x 256 tile also wins
    // at short reductions on <= 160k-pixel maps (profiles/r5/r5_s27_wgrad_heads_sweep.log, Inception-v3 batch 128:
    // 17x17 768 -> 704 87.9 -> 75.6 us, 35x35 192 -> 208 47.6 -> 42.0 us)
    if (g_tile_w8 && dst && d->K >= 208 && a.Mpix <= 163840) wt = 12;
  }
  // the pipelined 64 x 256 tile (tools/conv_tile_sweep.py WTILES, profiles/r5/r5_s25_wgrad_small_k_sweep.log, Inception-v3
  // at batch 128): the 5x5 48 -> 64 layers (Kg 1200: 79.1 us on the register-staged 64 x 128, 68.6 here) and the
  // stem's 3x3 80 -> 192 at 73x73 (645k pixels, K % 128 != 0: 389.7 us on 128 x 128, 365.6 here)
  if (wenv == -1 && g_wgrad_k64 && !in_scale && !bn &&
      ((wt == 1 && d->R * d->S >= 25 && a.Kg >= 1024) ||
       (wt == 10 && d->K % 128 != 0 && d->R * d->S > 1 && a.Mpix >= 262144)))
    wt = 11;
  if (wt >= 10 && wt <= 13 && (in_scale || bn)) wt = d->K <= 64 ? 1 : 0;  // (no x prologue in the pipelined kernels)
  // the pipelined 64 x 256 tile with the BN backward fused into its A staging (BNA): 14 = 4 waves 2 slots, 15 = 8
  // waves 2 slots, 16 = 8 waves 3 slots
  if (wt >= 14 && wt <= 16 && (in_scale || !bn || d->K > 64)) wt = d->K <= 64 ? 1 : 0;
  // the stem (BN backward fused, 64 x <= 256): tile 15 - the g / y operand read once and pipelined, 385.7 -> 357.1 us
  // at batch 256 (tools/stem_sweep.py, profiles/r6/r6_s10_stem_wgrad.log)
  // (not for 32 output channels: Inception-v3's packed 3x3/2 stem, K 32 x Kg 96, runs 119 us on the 32-row register-
  //  staged tile vs 294 us here - profiles/r6/r6_s41_stem_inception.log)
  if (wenv == -1 && g_stem_bna && bn && !in_scale && d->K > 32 && d->K <= 64 && a.Kg <= 256) wt = 15;
  if (wt == 12 && g_tile_pp && wenv == -1) wt = 13;  // (the ping-pong form of the 256x256 tile, A/B knob dtm_conv_set_pp)
  if (wt != 0 && wt != 1 && wt != 6 && wt != 7 && wt != 8 && !(wt >= 10 && wt <= 16)) wt = 0;
  {
    static int log = -1;  // DTM_TILE_LOG=1: one stderr line per weight-gradient decision too
    if (log < 0) {
      const char* e = getenv("DTM_TILE_LOG");
      log = e ? atoi(e) : 0;
    }
    if (log)
      fprintf(stderr, "dtm_wgrad M=%d K=%d C=%d RxS=%dx%d Kg=%d st=%d pro=%d bn=%d dst=%d -> %d\n", a.Mpix, d->K, d->C,
              d->R, d->S, a.Kg, d->stride, in_scale != nullptr, bn != nullptr, dst ? dst->n : 0, wt);
  }
  const bool big = wt == 12 || wt == 13;  // 8-wave 256x256 (one block per CU)
  const bool k64w = wt == 1 || wt == 7 || wt == 8 || wt == 11 || (wt >= 14 && wt <= 16);  // 64-row tiles
  const int MT = wt == 6 ? 32 : (k64w ? 64 : (big ? 256 : 128)), NT = (big || (k64w && wt != 1)) ? 256 : 128;
  if (big) occ = ((wenv == 12 || wenv == 13) && g_wgrad_occ != 4) ? g_wgrad_occ : 1;
  if (wt >= 14 && wt <= 16) occ = (wenv >= 14 && g_wgrad_occ != 4) ? g_wgrad_occ : 1;  // (the BNA tiles: 1 block per CU)  // (sweeps: WTILES=12:<occ>)
  long tiles = (long)((a.Kg + NT - 1) / NT) * ((a.K + MT - 1) / MT);
  // register-staged tiles: 3 blocks' worth of splits per CU (sweeps: WTILES=<1|6|0>:<occ>, occ != 4)
  const int rs_occ = (wenv >= 0 && g_wgrad_occ != 4) ? g_wgrad_occ : 3;
  long target = (long)num_cus * (wt >= 10 ? occ : rs_occ);
  long ksteps = (a.Mpix + 63) / 64;
  // the pipelined kernels run 2 blocks/CU: fill whole rounds of resident blocks (floor), a last
  // round with a few blocks doubles a layer's time
  long splits = wt >= 10 ? target / tiles : (target + tiles - 1) / tiles;
  if (splits > ksteps) splits = ksteps;
  if (splits < 1) splits = 1;
  long steps_per = (ksteps + splits - 1) / splits;
  a.pix_per_split = (int)(steps_per * 64);
  splits = (a.Mpix + a.pix_per_split - 1) / a.pix_per_split;
  // split-K partial slabs, summed into dW below (fp32 atomics straight into dW measured +2.4..+12 % step:
  // profiles/ab/r3_ab_wgrad_atomic_*.log)
  float* ws = dtm_ws_get_stream((size_t)splits * a.K * a.Kg, (hipStream_t)stream);
  if (!ws) return -4;
  a.dw = ws;
  if (wt >= 10) {
    a.in_shift = (const float*)zero_chunk();  // the zero DMA source
    dim3 grid((a.Kg + NT - 1) / NT, (a.K + MT - 1) / MT, splits);
    if (wt == 13) hipLaunchKernelGGL(conv_wgrad_pp_kernel, grid, dim3(512), 0, (hipStream_t)stream, a);
    else if (wt == 14)
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 256, 2, 2, 256, true>), grid, dim3(256), 0, (hipStream_t)stream, a);
    else if (wt == 15)
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 256, 2, 2, 512, true>), grid, dim3(512), 0, (hipStream_t)stream, a);
    else if (wt == 16)
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 256, 3, 2, 512, true>), grid, dim3(512), 0, (hipStream_t)stream, a);
    else if (wt == 12)
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<256, 256, 2, 2, 512>), grid, dim3(512), 0, (hipStream_t)stream, a);
    else if (wt == 11)
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 256, 2>), grid, dim3(256), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL((conv_wgrad_pipe_kernel<128, 128, 2>), grid, dim3(256), 0, (hipStream_t)stream, a);
  } else if (wt == 1) launch_wgrad<64, 128, 32, 64>(a, (int)splits, (hipStream_t)stream);
  else if (wt == 6) launch_wgrad<32, 128, 16, 64>(a, (int)splits, (hipStream_t)stream);
  // 64 x 256 register-staged (7: one LDS buffer, 8: two): every column of a <= 256-wide reduction in one tile, so the
  // dy operand (and the stem's fused BN backward inputs g, y) is read once instead of once per 128-column tile
  else if (wt == 7) launch_wgrad<64, 256, 32, 128, 1>(a, (int)splits, (hipStream_t)stream);
  else if (wt == 8) launch_wgrad<64, 256, 32, 128, 2>(a, (int)splits, (hipStream_t)stream);
  else launch_wgrad<128, 128, 64, 64>(a, (int)splits, (hipStream_t)stream);
  // dW += sum over the split slabs (every slab element is written: tiles cover [K][Kg] exactly).  (Running these
  // reductions on a second stream under the next conv - slabs in a 2-entry ring, event hand-offs, joined before the
  // optimizer - measured +5.8 % eager / +6.3 % captured Inception-v3 step and was removed in round 5:
  // profiles/ab/r5_ab_offload_inception.log, profiles/r5/r5_s6_bench_inc_*.log)
  if (dst) {
    // every member's row range of the slabs in one launch (a merged Inception head group: up to 4 members)
    const float* src[8];
    int widths[8];
    for (int i = 0, r0 = 0; i < dst->n; r0 += dst->rows[i], ++i) {
      src[i] = ws + (size_t)r0 * a.Kg;
      widths[i] = dst->rows[i] * a.Kg;
    }
    dtm_reduce_rows_multi(src, widths, dst->dw, dst->n, (int)splits, a.K * a.Kg, (hipStream_t)stream);
  } else {
    dtm_reduce_rows(ws, (int)splits, a.K * a.Kg, a.K * a.Kg, dw, (hipStream_t)stream);
  }
  return 0;
}

DTM_API int dtm_flip_desc_bytes() { return (int)sizeof(FlipDesc); }

DTM_API void dtm_weight_flip_transpose_batched(const void* descs, int n, void* stream) {
  if (n <= 0) return;
  // 512 blocks per weight: a small weight's extra blocks exit at once, a large one's stride over
  // its tiles with the chip covered
  hipLaunchKernelGGL(weight_flip_batched_kernel, dim3(512, n), dim3(256), 0, (hipStream_t)stream,
                     (const FlipDesc*)descs);
}

// the stride-decomposed flipped layout for a stride-st dgrad with forward pads ph / pw (ConvDesc::dec)
DTM_API void dtm_weight_flip_transpose_dec(const void* w, void* wt, int K, int R, int S, int C, int st, int ph, int pw,
                                           void* stream) {
  FlipDesc f{(const bf16_t*)w, (bf16_t*)wt, K, R, S, C, st, ph, pw, 0};
  int tiles = ((K + FLIP_T - 1) / FLIP_T) * ((C + FLIP_T - 1) / FLIP_T) * R * S;
  int blocks = tiles < 2048 ? tiles : 2048;
  hipLaunchKernelGGL(weight_flip_tiled_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, f);
}

DTM_API void dtm_weight_flip_transpose(const void* w, void* wt, int K, int R, int S, int C, void* stream) {
  FlipDesc f{(const bf16_t*)w, (bf16_t*)wt, K, R, S, C, 1, 0, 0, 0};
  int tiles = ((K + FLIP_T - 1) / FLIP_T) * ((C + FLIP_T - 1) / FLIP_T) * R * S;
  int blocks = tiles < 2048 ? tiles : 2048;
  hipLaunchKernelGGL(weight_flip_tiled_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, f);
}
