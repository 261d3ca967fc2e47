// One-pass backward of a training 1x1 conv + BatchNorm whose input is itself a BatchNorm+ReLU
// activation (the ResNet bottleneck expansion conv3: 64 -> 256 channels at 56x56).
//
// Unfused, that backward is three HBM passes over the 256-channel tensors:
//   stats_combine_fin   comb = g*scale + dsum + 2*dsumsq*y    (read g, y; write comb)
//   dgrad (act epilogue) g2 = relu'(x) * (comb . W^T)          (read comb, x; write g2)
//   wgrad               dW += comb^T . relu(bn(x))             (read comb, relu(bn(x)))
// = 5 reads/writes of a 256-channel tensor.  Here each 64-pixel tile of g and y is read ONCE: comb is
// formed in registers and written to an LDS image that feeds both GEMMs -- the dgrad (sums over the
// 256 channels: ds_read_b128 fragments) and the weight gradient (sums over the tile's pixels:
// ds_read_b64_tr_b16 fragments) -- with the conv input's activation relu(x*s+t) recomputed from the
// raw x that the dgrad epilogue needs anyway.  2 tensor reads instead of 5 (plus the 64-channel x).
//
// Persistent blocks of 8 waves; a block keeps its weight-gradient tile [256][64] fp32 in registers
// over all its pixel tiles and writes it once (a per-block slab, summed by dtm_reduce_rows), the same
// for the input-BN gradient sums.  The next tile's loads are issued before the current tile's
// MFMAs (register prefetch), so HBM streams while the matrix cores work.
// Reference op: the BatchNorm/conv gradient of a slim bottleneck (reference vgg/nets/resnet_v1.py:78-139,
// TF's FusedBatchNormGrad + Conv2DBackpropInput/Filter).
#include "common.h"

namespace dtm {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_stream(const bf16_t* p) {  // read-once operand: non-temporal
  const u32x4_t v = __builtin_nontemporal_load((const u32x4_t*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

struct Bwd1x1Args {
  const bf16_t* g;       // [M][KO] gradient of the BN output, unscaled (the BN-apply's g)
  const bf16_t* y;       // [M][KO] raw conv output (the BN input)
  const float* dss;      // [4][KO] gradient of ss
  const float* ss;       // [4][KO] scale, shift, mean, rstd
  const float* gamma;    // [KO] or nullptr
  float count;
  float* dgamma;         // [KO] += (block 0), or nullptr
  float* dbeta;
  const bf16_t* wt;      // [CI][KO]: the 1x1 weight transposed (W[k][c] at wt[c*KO + k])
  const bf16_t* x;       // [M][CI] raw input of the conv's input BatchNorm+ReLU
  const float* xss;      // [4][CI] its scale, shift
  int x_unscaled;        // the input gradient is g2 (1) or g2*scale (0)
  const bf16_t* add_src; // plain mode: [M][CI] gradient of x from its other consumer, added (or nullptr)
  bf16_t* dx;            // [M][CI] out
  float* sums;           // [blocks][2][CI] partial (sum g2*x, sum g2)
  float* slab;           // [blocks][KO][CI] weight-gradient partials
  int M, ntiles;
};

// LDS image of a [64 pixel][ROWS channel] bf16 tile, readable both ways: 128-B blocks of 4 pixels x
// 16 channels (the ds_read_b64_tr_b16 unit), block (p/4, c/16) at ((p/4)*(ROWS/16) + c/16)*128; inside
// a block the pixel row is permuted by the channel block ((p&3) ^ (c/16 & 3): the 8 consecutive 16-B
// chunks of one pixel written by 8 lanes land in 8 different bank slots), and bit 7 is flipped by
// (p/4)&1 (16 pixels' ds_read_b128 at one channel offset hit 8 slots, not 4).  Every 8-B piece (4
// channels) and 16-B piece (8 channels, 8-aligned) of one pixel stays contiguous.
template <int ROWS>
__device__ __forceinline__ int img_off(int p, int c) {
  constexpr int MB = ROWS / 16;
  const int b = c >> 4;
  return ((((p >> 2) * MB + b) << 7) + (((p & 3) ^ (b & 3)) << 5) + ((c & 15) << 1)) ^ (((p >> 2) & 1) << 7);
}

template <int KO, int CI>
struct Bwd1x1Smem {
  static constexpr int PT = 64;
  static constexpr int WROW = KO + 8;             // padded weight row (bf16): conflict-free b128 reads
  static constexpr int OROW = CI * 2 + 16;        // staged dgrad output row (bytes)
  static constexpr int WT = 0;                    // [CI][WROW] bf16
  static constexpr int DY = WT + CI * WROW * 2;   // image<KO> of comb
  static constexpr int XA = DY + PT * KO * 2;     // image<CI> of relu(x*s+t)
  static constexpr int OUT = XA + PT * CI * 2;    // [PT][OROW] staged dgrad tile
  static constexpr int CS = OUT + PT * OROW;      // [3][KO] comb coefficients (scale, add, x-factor)
  static constexpr int XS = CS + 3 * KO * 4;      // [2][CI] input BN scale / shift
  static constexpr int BYTES = XS + 2 * CI * 4;
};

// ACT: the conv input is relu(x*xs+xt) (recomputed; its backward in the dgrad epilogue); else the conv
// input is x itself (plain mode: the dgrad epilogue adds add_src)
template <int KO, int CI, bool ACT>
__global__ __launch_bounds__(512) void conv1x1_bnbwd_kernel(Bwd1x1Args a) {
  using L = Bwd1x1Smem<KO, CI>;
  constexpr int PT = L::PT;
  constexpr int KCH = KO / 8;                       // 16-B chunks per pixel of g / y
  constexpr int GI = PT * KCH / 512;                // g (and y) chunks per thread per tile
  static_assert(CI == 64 && PT * CI / 8 == 512, "one x chunk per thread");
  static_assert(KO == 256, "8 waves x 32 weight-gradient rows");
  static_assert(L::BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[L::BYTES];
  bf16_t* s_wt = (bf16_t*)(smem + L::WT);
  char* s_dy = smem + L::DY;
  char* s_xa = smem + L::XA;
  char* s_out = smem + L::OUT;
  float* s_cs = (float*)(smem + L::CS);
  float* s_ca = s_cs + KO;
  float* s_cb = s_ca + KO;
  float* s_xs = (float*)(smem + L::XS);
  float* s_xh = s_xs + CI;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;

  // per-channel coefficients of comb = g*scale + ds + 2*dq*y (stats_combine_fin's algebra)
  for (int c = tid; c < KO; c += 512) {
    float ds, dq, dg, db;
    fin_bwd_channel(a.dss, a.ss, a.gamma, KO, c, a.count, &ds, &dq, &dg, &db);
    s_cs[c] = a.ss[c];
    s_ca[c] = ds;
    s_cb[c] = 2.f * dq;
    if (blockIdx.x == 0) {
      if (a.dgamma) a.dgamma[c] += dg;
      if (a.dbeta) a.dbeta[c] += db;
    }
  }
  for (int c = tid; c < CI; c += 512) {
    s_xs[c] = ACT ? a.xss[c] : 1.f;
    s_xh[c] = ACT ? a.xss[CI + c] : 0.f;
  }
  for (int q = tid; q < CI * KCH; q += 512) {
    const int c = q / KCH, k = (q % KCH) * 8;
    *(uint4*)(s_wt + c * L::WROW + k) = *(const uint4*)(a.wt + (size_t)c * KO + k);
  }

  // load mapping: g / y chunk i of a tile = pixel (tid / KCH) + i * (512 / KCH), channels kc..kc+7;
  // x chunk = pixel tid / 8, channels xc..xc+7 (also this thread's dgrad-epilogue chunk)
  const int kc = (tid % KCH) * 8, gp0 = tid / KCH;
  constexpr int GPS = 512 / KCH;
  const int xc = (tid & 7) * 8, xp = tid >> 3;
  uint4 rg[GI], ry[GI], rx;
  auto gload = [&](int t) {
    const int pb = t * PT;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int p = pb + gp0 + i * GPS;
      const bool v = p < a.M;
      const size_t o = (size_t)(v ? p : 0) * KO + kc;
      rg[i] = v ? ld_stream(a.g + o) : make_uint4(0, 0, 0, 0);
      ry[i] = v ? ld_stream(a.y + o) : make_uint4(0, 0, 0, 0);
    }
    const int p = pb + xp;
    rx = p < a.M ? *(const uint4*)(a.x + (size_t)p * CI + xc) : make_uint4(0, 0, 0, 0);
  };

  f32x4 accw[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float sgx[8], sg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sgx[e] = 0.f; sg[e] = 0.f; }

  int t = blockIdx.x;
  if (t < a.ntiles) gload(t);
  __syncthreads();  // coefficients, weights
  float cs[8], ca[8], cb[8], xs[8], xh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    cs[e] = s_cs[kc + e]; ca[e] = s_ca[kc + e]; cb[e] = s_cb[kc + e];
    xs[e] = s_xs[xc + e]; xh[e] = s_xh[xc + e];
  }

  typedef __attribute__((address_space(3))) short4v lds_s4;
  typedef __attribute__((address_space(3))) char lds_c;
  lds_c* l_dy = (lds_c*)s_dy;
  lds_c* l_xa = (lds_c*)s_xa;

  for (; t < a.ntiles; t += gridDim.x) {
    const int pb = t * PT;
    // ---- comb and relu(bn(x)) tiles -> LDS images
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int pl = gp0 + i * GPS;
      float d[8], yv[8];
      d[0] = lo_bf(rg[i].x); d[1] = hi_bf(rg[i].x); d[2] = lo_bf(rg[i].y); d[3] = hi_bf(rg[i].y);
      d[4] = lo_bf(rg[i].z); d[5] = hi_bf(rg[i].z); d[6] = lo_bf(rg[i].w); d[7] = hi_bf(rg[i].w);
      yv[0] = lo_bf(ry[i].x); yv[1] = hi_bf(ry[i].x); yv[2] = lo_bf(ry[i].y); yv[3] = hi_bf(ry[i].y);
      yv[4] = lo_bf(ry[i].z); yv[5] = hi_bf(ry[i].z); yv[6] = lo_bf(ry[i].w); yv[7] = hi_bf(ry[i].w);
      const bool v = pb + pl < a.M;
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = v ? fmaf(d[e], cs[e], ca[e] + cb[e] * yv[e]) : 0.f;
      *(uint4*)(s_dy + img_off<KO>(pl, kc)) =
          make_uint4(pack2bf(d[0], d[1]), pack2bf(d[2], d[3]), pack2bf(d[4], d[5]), pack2bf(d[6], d[7]));
    }
    const uint4 cx = rx;  // this tile's raw x chunk (dgrad epilogue)
    float xv[8];
    xv[0] = lo_bf(cx.x); xv[1] = hi_bf(cx.x); xv[2] = lo_bf(cx.y); xv[3] = hi_bf(cx.y);
    xv[4] = lo_bf(cx.z); xv[5] = hi_bf(cx.z); xv[6] = lo_bf(cx.w); xv[7] = hi_bf(cx.w);
    {
      float av[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) av[e] = pb + xp < a.M ? (ACT ? fmaxf(fmaf(xv[e], xs[e], xh[e]), 0.f) : xv[e]) : 0.f;
      *(uint4*)(s_xa + img_off<CI>(xp, xc)) =
          make_uint4(pack2bf(av[0], av[1]), pack2bf(av[2], av[3]), pack2bf(av[4], av[5]), pack2bf(av[6], av[7]));
    }
    // ---- next tile's loads stream while this tile is multiplied
    if (t + (int)gridDim.x < a.ntiles) gload(t + gridDim.x);
    __syncthreads();

    // ---- dgrad: out[c][p] = sum_k Wt[c][k] comb[p][k]; wave: 16 channels x 32 pixels
    f32x4 accd[2];
    accd[0] = accd[1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int cbk = wave & 3, pbk = (wave >> 2) * 2;
#pragma unroll
    for (int ks = 0; ks < KO / 32; ++ks) {
      const int k0 = ks * 32 + 8 * g;
      const short8 af = *(const short8*)(s_wt + (cbk * 16 + li) * L::WROW + k0);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const short8 bfr = *(const short8*)(s_dy + img_off<KO>((pbk + j) * 16 + li, k0));
        accd[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, accd[j], 0, 0, 0);
      }
    }
    // ---- weight gradient: dW[ko][c] += sum_p comb[p][ko] relu(bn(x))[p][c]; wave: 32 rows x 64 cols
#pragma unroll
    for (int ks = 0; ks < PT / 32; ++ks) {
      const int kb = ks * 32 + 8 * g;
      short8 af[2], bfr[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = wave * 32 + i * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(l_dy + img_off<KO>(kb + tq, m)));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(l_dy + img_off<KO>(kb + 4 + tq, m)));
        af[i] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = j * 16 + 4 * tp;
        short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(l_xa + img_off<CI>(kb + tq, n)));
        short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(l_xa + img_off<CI>(kb + 4 + tq, n)));
        bfr[j] = (short8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) accw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], accw[i][j], 0, 0, 0);
    }
    // ---- dgrad epilogue: stage the bf16 tile, then per 16-B chunk the input BN+ReLU backward
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = (pbk + j) * 16 + li, c = cbk * 16 + 4 * g;
      *(uint2*)(s_out + p * L::OROW + c * 2) =
          make_uint2(pack2bf(accd[j][0], accd[j][1]), pack2bf(accd[j][2], accd[j][3]));
    }
    __syncthreads();
    {
      const uint4 v = *(const uint4*)(s_out + xp * L::OROW + xc * 2);
      float f[8];
      f[0] = lo_bf(v.x); f[1] = hi_bf(v.x); f[2] = lo_bf(v.y); f[3] = hi_bf(v.y);
      f[4] = lo_bf(v.z); f[5] = hi_bf(v.z); f[6] = lo_bf(v.w); f[7] = hi_bf(v.w);
      if (!ACT && pb + xp < a.M) {
        if (a.add_src) {
          const uint4 r = *(const uint4*)(a.add_src + (size_t)(pb + xp) * CI + xc);
          f[0] += lo_bf(r.x); f[1] += hi_bf(r.x); f[2] += lo_bf(r.y); f[3] += hi_bf(r.y);
          f[4] += lo_bf(r.z); f[5] += hi_bf(r.z); f[6] += lo_bf(r.w); f[7] += hi_bf(r.w);
        }
        *(uint4*)(a.dx + (size_t)(pb + xp) * CI + xc) =
            make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
      }
      if (ACT && pb + xp < a.M) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gg = fmaf(xv[e], xs[e], xh[e]) > 0.f ? f[e] : 0.f;
          sgx[e] += gg * xv[e];
          sg[e] += gg;
          f[e] = a.x_unscaled ? gg : gg * xs[e];
        }
        *(uint4*)(a.dx + (size_t)(pb + xp) * CI + xc) =
            make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
      }
    }
    // (the next iteration's image writes are ordered after every wave's MFMA reads by the barrier
    //  above; its staging writes come after its own post-transform barrier)
  }

  // ---- per-block outputs: weight-gradient slab, input-BN sums row
  float* slab = a.slab + (size_t)blockIdx.x * KO * CI;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(size_t)(wave * 32 + i * 16 + 4 * g + r) * CI + j * 16 + li] = accw[i][j][r];
  if constexpr (!ACT) return;
  __syncthreads();  // s_dy free
  float* red = (float*)s_dy;  // [512][16]
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[tid * 16 + e] = sgx[e]; red[tid * 16 + 8 + e] = sg[e]; }
  __syncthreads();
  float* row = a.sums + (size_t)blockIdx.x * 2 * CI;
  for (int o = tid; o < 8 * 16; o += 512) {
    const int c = o >> 4, e = o & 15;
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < 64; ++k) s += red[((c + 8 * k) << 4) + e];
    row[(e < 8 ? 0 : CI) + c * 8 + (e & 7)] = s;
  }
}

}  // namespace dtm
using namespace dtm;

static int bwd1x1_blocks(int ntiles) {
  static int occ = 0;
  if (!occ) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, conv1x1_bnbwd_kernel<256, 64, true>, 512, 0) != hipSuccess ||
        occ <= 0)
      occ = 1;
  }
  const int cap = occ * dtm_compute_cus();  // (minus the CUs reserved for RCCL)
  return ntiles < cap ? ntiles : cap;
}

// Fused backward of y = conv1x1(relu(x*xs+xt), W) -> BatchNorm (training): see the file comment.
// g: gradient of the BN output (unscaled), y: raw conv output, dss/ss/gamma: the BN's ss gradient and
// forward ss, wt: [C][K] transposed weight, x/xss: the input BN's raw input and ss.  Outputs: dx
// ([M][C] input gradient, masked), sums[2][C] += (sum dx*x, sum dx) (unscaled form), dw[K][C] +=,
// dgamma/dbeta +=.  xss == nullptr: plain mode, the conv input is x itself; dx = dgrad (+ add_src) and
// sums is untouched.  Returns -1 for a shape this kernel does not cover (the caller falls back).
DTM_API int dtm_conv1x1_bnbwd(const void* g, const void* y, const float* dss, const float* ss, const float* gamma,
                              float count, float* dgamma, float* dbeta, const void* wt, const void* x,
                              const float* xss, int x_unscaled, const void* add_src, void* dx, float* sums, float* dw,
                              long M, int K, int C, void* stream) {
  if (K != 256 || C != 64 || M <= 0 || M * (long)K >= (1l << 31)) return -1;
  if (((uintptr_t)g | (uintptr_t)y | (uintptr_t)wt | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)add_src) & 15) return -1;
  if (xss && !sums) return -1;
  Bwd1x1Args a;
  a.g = (const bf16_t*)g; a.y = (const bf16_t*)y; a.dss = dss; a.ss = ss; a.gamma = gamma; a.count = count;
  a.dgamma = dgamma; a.dbeta = dbeta; a.wt = (const bf16_t*)wt; a.x = (const bf16_t*)x; a.xss = xss;
  a.x_unscaled = x_unscaled; a.dx = (bf16_t*)dx; a.M = (int)M; a.add_src = (const bf16_t*)add_src;
  a.ntiles = (int)((M + 63) / 64);
  const int blocks = bwd1x1_blocks(a.ntiles);
  float* ws = dtm_ws_get_stream((size_t)blocks * (K * C + 2 * C), (hipStream_t)stream);
  if (!ws) return -4;
  a.slab = ws;
  a.sums = ws + (size_t)blocks * K * C;
  if (xss) hipLaunchKernelGGL((conv1x1_bnbwd_kernel<256, 64, true>), dim3(blocks), dim3(512), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL((conv1x1_bnbwd_kernel<256, 64, false>), dim3(blocks), dim3(512), 0, (hipStream_t)stream, a);
  dtm_reduce_rows(a.slab, blocks, K * C, K * C, dw, (hipStream_t)stream);
  if (xss) dtm_reduce_rows(a.sums, blocks, 2 * C, 2 * C, sums, (hipStream_t)stream);
  return 0;
}
