// Same-process A/B of the two gfx950 bf16 MFMA shapes on the conv kernels' inner loop pattern:
// v_mfma_f32_16x16x32_bf16 (what every conv / wgrad kernel of csrc/kernels uses) vs
// v_mfma_f32_32x32x16_bf16.  A block of 4 waves computes a 128x128 tile (waves 2x2 of 64x64) of
// A[128][64] . B[64][128] from LDS, re-reading its fragments with ds_read_b128 every pass (as the conv
// main loops do per k-tile), REPEAT passes, so the loop is bound by MFMA issue + LDS reads, not HBM.
// Both variants issue the same 16 ds_read_b128 and 512 MFMA cycles per wave per 64-deep pass; the
// result (REPEAT * A.B in fp32) is checked against a CPU reference.  Output: TFLOP/s of each, 5 runs.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_ab tools/mfma_ab.hip ; run: ./mfma_ab
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef short short8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TM = 128, TN = 128, KC = 64, PITCH = KC + 8;  // padded LDS rows (bf16 elements)

__device__ inline void load_tiles(const unsigned short* A, const unsigned short* Bt, unsigned short* sA,
                                  unsigned short* sB) {
  for (int i = threadIdx.x; i < TM * KC / 8; i += blockDim.x) {
    const int r = i / (KC / 8), c = (i % (KC / 8)) * 8;
    *(uint4*)(sA + r * PITCH + c) = *(const uint4*)(A + r * KC + c);
    *(uint4*)(sB + r * PITCH + c) = *(const uint4*)(Bt + r * KC + c);
  }
  __syncthreads();
}

// 16x16x32: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]; C col l&15, row 4(l>>4)+r
template <bool RELOAD>
__global__ __launch_bounds__(256) void mfma16_kernel(const unsigned short* A, const unsigned short* Bt, float* C,
                                                     int repeat) {
  __shared__ __attribute__((aligned(16))) unsigned short sA[TM * PITCH], sB[TN * PITCH];
  load_tiles(A, Bt, sA, sB);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int fr = lane & 15, fk = lane >> 4;
  f32x4 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < repeat; ++it) {
    // RELOAD: a compiler memory barrier per pass, so the fragments are re-read from LDS every pass (the
    // conv main loops' pattern); otherwise the loop-invariant reads are hoisted and only MFMAs remain
    if (RELOAD) asm volatile("" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < KC / 32; ++ks) {
      short8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const short8*)(sA + (wm + i * 16 + fr) * PITCH + ks * 32 + fk * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const short8*)(sB + (wn + j * 16 + fr) * PITCH + ks * 32 + fk * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  if (blockIdx.x != 0) return;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 4; ++r) C[(wm + i * 16 + fk * 4 + r) * TN + wn + j * 16 + fr] = acc[i][j][r];
}

// 32x32x16: lane l (r = l&31, h = l>>5) holds A[row r][k 8h+j], B[k 8h+j][col r];
// C col l&31, row (reg&3) + 8(reg>>2) + 4(l>>5)
template <bool RELOAD>
__global__ __launch_bounds__(256) void mfma32_kernel(const unsigned short* A, const unsigned short* Bt, float* C,
                                                     int repeat) {
  __shared__ __attribute__((aligned(16))) unsigned short sA[TM * PITCH], sB[TN * PITCH];
  load_tiles(A, Bt, sA, sB);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int fr = lane & 31, fh = lane >> 5;
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int it = 0; it < repeat; ++it) {
    if (RELOAD) asm volatile("" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < KC / 16; ++ks) {
      short8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const short8*)(sA + (wm + i * 32 + fr) * PITCH + ks * 16 + fh * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = *(const short8*)(sB + (wn + j * 32 + fr) * PITCH + ks * 16 + fh * 8);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  if (blockIdx.x != 0) return;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r)
        C[(wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh) * TN + wn + j * 32 + fr] = acc[i][j][r];
}

static unsigned short f2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
static float bf2f(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int repeat = argc > 1 ? atoi(argv[1]) : 2000;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  unsigned short *dA, *dB;
  float* dC;
  CK(hipMalloc(&dA, TM * KC * 2));
  CK(hipMalloc(&dB, TN * KC * 2));
  CK(hipMalloc(&dC, TM * TN * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, repeat %d; 128x128x64 block tile per pass, 4 waves (2x2 of 64x64)\n", cus, repeat);
  printf("%-9s %-7s %-8s %-24s %9s %9s %10s %s\n", "data", "reload", "waves/SIMD", "mfma", "min ms", "mean ms",
         "TFLOP/s", "check");
  for (int data = 0; data < 2; ++data) {  // 0: few-valued (k/8), 1: full-entropy random bf16 in [-1, 1)
    std::vector<unsigned short> hA(TM * KC), hB(TN * KC);
    srand(1 + data);
    for (auto& v : hA) v = data ? f2bf(2.f * rand() / RAND_MAX - 1.f) : f2bf((rand() % 17 - 8) / 8.f);
    for (auto& v : hB) v = data ? f2bf(2.f * rand() / RAND_MAX - 1.f) : f2bf((rand() % 17 - 8) / 8.f);
    std::vector<double> ref(TM * TN, 0.0), mag(TM * TN, 0.0);
    for (int m = 0; m < TM; ++m)
      for (int n = 0; n < TN; ++n) {
        double sm = 0, sa = 0;
        for (int k = 0; k < KC; ++k) {
          const double pr = (double)bf2f(hA[m * KC + k]) * bf2f(hB[n * KC + k]);
          sm += pr;
          sa += fabs(pr);
        }
        ref[m * TN + n] = sm * repeat;
        mag[m * TN + n] = sa * repeat;
      }
    CK(hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
    for (int reload = 0; reload < 2; ++reload)
      for (int occ = 1; occ <= 2; ++occ) {
        const int blocks = cus * occ;  // occ blocks of 4 waves per CU = occ waves per SIMD
        const double flop = 2.0 * TM * TN * KC * (double)repeat * blocks;
        std::vector<float> times[2];
        double err[2] = {0, 0};
        for (int run = 0; run < 12; ++run) {  // interleaved A/B; runs 0, 1 = warm-up
          const int variant = run & 1;
          CK(hipMemset(dC, 0, TM * TN * 4));
          CK(hipEventRecord(e0));
          if (variant == 0) {
            if (reload) hipLaunchKernelGGL(mfma16_kernel<true>, dim3(blocks), dim3(256), 0, 0, dA, dB, dC, repeat);
            else hipLaunchKernelGGL(mfma16_kernel<false>, dim3(blocks), dim3(256), 0, 0, dA, dB, dC, repeat);
          } else {
            if (reload) hipLaunchKernelGGL(mfma32_kernel<true>, dim3(blocks), dim3(256), 0, 0, dA, dB, dC, repeat);
            else hipLaunchKernelGGL(mfma32_kernel<false>, dim3(blocks), dim3(256), 0, 0, dA, dB, dC, repeat);
          }
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (run >= 2) times[variant].push_back(ms);
          if (run >= 10) {
            std::vector<float> hC(TM * TN);
            CK(hipMemcpy(hC.data(), dC, TM * TN * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < TM * TN; ++i) {
              const double d = fabs(hC[i] - ref[i]) / (mag[i] + 1e-30);
              if (d > err[variant]) err[variant] = d;
            }
          }
        }
        for (int variant = 0; variant < 2; ++variant) {
          float mn = 1e30f, sum = 0;
          for (float b : times[variant]) { mn = b < mn ? b : mn; sum += b; }
          printf("%-9s %-7s %-8d %-24s %9.3f %9.3f %10.1f %s (%.1e)\n", data ? "random" : "k/8", reload ? "LDS" : "regs",
                 occ, variant == 0 ? "mfma_f32_16x16x32_bf16" : "mfma_f32_32x32x16_bf16", mn,
                 sum / times[variant].size(), flop / (mn * 1e-3) / 1e12, err[variant] < 1e-4 ? "OK" : "MISMATCH",
                 err[variant]);
        }
      }
  }
  return 0;
}
