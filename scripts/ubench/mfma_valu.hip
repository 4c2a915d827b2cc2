// Micro-benchmark (gfx950): can the f32 matrix pipe (v_mfma_f32_16x16x4_f32)
// and the f32 vector pipe (v_pk_fma_f32) run at the same time on one SIMD,
// and is the f32 MFMA bitwise a k-ordered fmaf chain (incl. zero weights,
// as a banded / Toeplitz correlation would feed it)?
//
//   exact   : 64 random 16x16x4 problems chained 12 deep vs a host fmaf chain
//   mfma    : waves issuing only MFMAs (4 independent accumulators)
//   valu    : waves issuing only v_pk_fma_f32 (10 independent accumulators)
//   mixed   : 8-wave workgroups, waves 0-3 MFMA, waves 4-7 VALU (same work
//             per wave as above); time ~ max(mfma, valu) means the pipes overlap
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                             \
    }                                                                       \
  } while (0)

// ---- exactness: D = mfma(a_k, b_k, ...) chained DEPTH times
#define DEPTH 12
__global__ void k_exact(const float* A, const float* B, const float* C, float* D) {
  // A: [prob][DEPTH][16][4], B: [prob][DEPTH][4][16], C/D: [prob][16][16]
  const int p = blockIdx.x, l = threadIdx.x;
  f4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[(p * 16 + (l >> 4) * 4 + r) * 16 + (l & 15)];
  for (int d = 0; d < DEPTH; ++d) {
    const float a = A[((p * DEPTH + d) * 16 + (l & 15)) * 4 + (l >> 4)];
    const float b = B[((p * DEPTH + d) * 4 + (l >> 4)) * 16 + (l & 15)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[(p * 16 + (l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}

template <bool DO_MFMA, bool DO_VALU, int NW_MFMA>
__global__ __launch_bounds__(512) void k_pipe(const float* __restrict__ w, float* __restrict__ out, int iters) {
  const int wid = threadIdx.x >> 6;
  const bool mf = DO_MFMA && (!DO_VALU || wid < NW_MFMA);
  float s = 0.f;
  if (mf) {
    f4 acc[4];
    for (int c = 0; c < 4; ++c) acc[c] = (f4){(float)threadIdx.x, 1.f, 2.f, (float)c};
    float a = w[threadIdx.x & 63], b = w[(threadIdx.x + 7) & 63];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
      asm volatile("" : "+v"(a), "+v"(b));
    }
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  } else if (DO_VALU) {
    f2 acc[10];
    for (int c = 0; c < 10; ++c) acc[c] = (f2){(float)threadIdx.x + c, (float)c};
    f2 px[13];
    for (int q = 0; q < 13; ++q) px[q] = (f2){1.0001f * threadIdx.x + q, 0.999f * q};
    const float ws0 = w[0], ws1 = w[1], ws2 = w[2], ws3 = w[3];
    for (int it = 0; it < iters; ++it) {
      // 64 MFMAs of 16x16x4 = 64 * 2048 FLOP; match with 64 * 2048 / 256 (FLOP per pk_fma wave-instr) = 512 pk_fma
#pragma unroll
      for (int rep = 0; rep < 12; ++rep) {
        const float wv[4] = {ws0, ws1, ws2, ws3};
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int c = 0; c < 10; ++c) acc[c] = __builtin_elementwise_fma((f2){wv[j], wv[j]}, px[c + j], acc[c]);
      }
#pragma unroll
      for (int c = 0; c < 32; ++c) acc[c % 10] = __builtin_elementwise_fma((f2){ws0, ws0}, px[c % 13], acc[c % 10]);
      asm volatile("" : "+v"(px[0]), "+v"(px[1]));
    }
    for (int c = 0; c < 10; ++c) s += acc[c].x + acc[c].y;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static double time_kernel(K kern, int blocks, int threads, const float* w, float* out, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, w, out, iters);  // warm-up
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, w, out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

static uint64_t sm = 0x1234567;
static float rnd() {
  sm = sm * 6364136223846793005ull + 1442695040888963407ull;
  return ((int)(sm >> 40) % 20001 - 10000) / 977.0f;
}

int main() {
  // ---------------- exactness
  const int P = 64;
  std::vector<float> A((size_t)P * DEPTH * 64), B((size_t)P * DEPTH * 64), C((size_t)P * 256), D(C.size());
  for (auto& v : A) v = rnd() * 0.01f;
  for (size_t i = 0; i < A.size(); i += 3) A[i] = 0.0f;  // zero taps, as a banded A has
  for (auto& v : B) v = (float)((int)fabsf(rnd() * 25.f) % 256);  // u8 pixels
  for (auto& v : C) v = rnd();
  float *dA, *dB, *dC, *dD;
  CHK(hipMalloc(&dA, A.size() * 4));
  CHK(hipMalloc(&dB, B.size() * 4));
  CHK(hipMalloc(&dC, C.size() * 4));
  CHK(hipMalloc(&dD, D.size() * 4));
  CHK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  CHK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_exact, dim3(P), dim3(64), 0, 0, dA, dB, dC, dD);
  CHK(hipDeviceSynchronize());
  CHK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  long bad = 0, bad_unfused = 0;
  for (int p = 0; p < P; ++p)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        float acc = C[(p * 16 + i) * 16 + j], acc2 = acc;
        for (int d = 0; d < DEPTH; ++d)
          for (int k = 0; k < 4; ++k) {
            const float a = A[((p * DEPTH + d) * 16 + i) * 4 + k], b = B[((p * DEPTH + d) * 4 + k) * 16 + j];
            acc = std::fmaf(a, b, acc);
            volatile float pr = a * b;
            acc2 = acc2 + pr;
          }
        uint32_t x, y, z;
        const float g = D[(p * 16 + i) * 16 + j];
        memcpy(&x, &g, 4);
        memcpy(&y, &acc, 4);
        memcpy(&z, &acc2, 4);
        bad += x != y;
        bad_unfused += x != z;
      }
  printf("exact: %ld of %d outputs differ from the k-ordered fmaf chain (%ld from mul+add)\n", bad, P * 256,
         bad_unfused);

  // ---------------- pipes
  float *w, *out;
  CHK(hipMalloc(&w, 64 * 4));
  std::vector<float> hw(64);
  for (auto& v : hw) v = rnd() * 1e-3f;
  CHK(hipMemcpy(w, hw.data(), 64 * 4, hipMemcpyHostToDevice));
  const int blocks = 256 * 2, threads = 512, iters = 2000;
  CHK(hipMalloc(&out, (size_t)blocks * threads * 4));
  // per wave per iteration: MFMA 64 x 2048 FLOP; VALU (12*40 + 32) = 512 pk_fma x 256 FLOP
  const double flop_wave_it = 64.0 * 2048.0;
  const double waves = blocks * threads / 64.0;
  const double t_m = time_kernel(k_pipe<true, false, 8>, blocks, threads, w, out, iters);
  const double t_v = time_kernel(k_pipe<false, true, 0>, blocks, threads, w, out, iters);
  const double t_x = time_kernel(k_pipe<true, true, 4>, blocks, threads, w, out, iters);
  const double t_x2 = time_kernel(k_pipe<true, true, 2>, blocks, threads, w, out, iters);
  const double t_x6 = time_kernel(k_pipe<true, true, 6>, blocks, threads, w, out, iters);
  printf("mfma-only : %.3f ms  %.1f TFLOP/s\n", t_m, waves * iters * flop_wave_it / t_m / 1e9);
  printf("valu-only : %.3f ms  %.1f TFLOP/s\n", t_v, waves * iters * flop_wave_it / t_v / 1e9);
  printf("mixed 4+4 : %.3f ms  %.1f TFLOP/s (sum of both pipes' work)\n", t_x, waves * iters * flop_wave_it / t_x / 1e9);
  printf("mixed 2+6 : %.3f ms  %.1f TFLOP/s\n", t_x2, waves * iters * flop_wave_it / t_x2 / 1e9);
  printf("mixed 6+2 : %.3f ms  %.1f TFLOP/s\n", t_x6, waves * iters * flop_wave_it / t_x6 / 1e9);
  return 0;
}
