// Micro-benchmark: v_pk_fma_f32 issue rate on gfx950 with the weight operand
// in an SGPR pair (as in k_corr) vs a VGPR pair, and plain v_fma_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
#define NACC 10
template <int KW, int NA = NACC>
__global__ __launch_bounds__(192) void kern_px(const float* __restrict__ w, float* __restrict__ out, int iters) {
  f2 acc[NA];
  for (int c = 0; c < NA; ++c) acc[c] = (f2){(float)threadIdx.x + c, (float)c};
  f2 px[NA + KW - 1];
  for (int q = 0; q < NA + KW - 1; ++q) px[q] = (f2){1.0001f * threadIdx.x + q, 0.999f * q};
  float ws[KW];
  for (int k = 0; k < KW; ++k) ws[k] = w[k];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const f2 w2 = (f2){ws[j], ws[j]};
#pragma unroll
      for (int c = 0; c < NA; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + j], acc[c]);
    }
    asm volatile("" : "+v"(px[0]), "+v"(px[1]));  // keep px live / loop-variant
  }
  float s = 0;
  for (int c = 0; c < NA; ++c) s += acc[c].x + acc[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
__global__ __launch_bounds__(256) void kern(const float* __restrict__ w, float* __restrict__ out, int iters) {
  f2 acc[NACC];
  for (int c = 0; c < NACC; ++c) acc[c] = (f2){(float)threadIdx.x + c, (float)c};
  const f2 x = (f2){1.0001f * threadIdx.x, 0.999f};
  float ws[16];
  for (int k = 0; k < 16; ++k) ws[k] = w[k];  // uniform -> SGPRs
  float wv[16];
  for (int k = 0; k < 16; ++k) wv[k] = w[k + (threadIdx.x & 1)];  // divergent -> VGPRs
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (MODE == 0) {
        const f2 w2 = (f2){ws[k], ws[k]};
#pragma unroll
        for (int c = 0; c < NACC; ++c) acc[c] = __builtin_elementwise_fma(w2, x, acc[c]);
      } else if (MODE == 1) {
        const f2 w2 = (f2){wv[k], wv[k]};
#pragma unroll
        for (int c = 0; c < NACC; ++c) acc[c] = __builtin_elementwise_fma(w2, x, acc[c]);
      } else if (MODE == 2) {
#pragma unroll
        for (int c = 0; c < NACC; ++c) acc[c].x = __builtin_fmaf(ws[k], x.x, acc[c].x);
      }
    }
  }
  float s = 0;
  for (int c = 0; c < NACC; ++c) s += acc[c].x + acc[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  float *w, *o;
  hipMalloc(&w, 64 * 4);
  float hw[64];
  for (int i = 0; i < 64; ++i) hw[i] = 1e-7f * i;
  hipMemcpy(w, hw, 256, hipMemcpyHostToDevice);
  const int blocks = 256 * 16, threads = 256, iters = 2000;
  hipMalloc(&o, (size_t)blocks * threads * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[3] = {"pk_fma sgpr weight", "pk_fma vgpr weight", "v_fma_f32"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (mode == 0) kern<0><<<blocks, threads>>>(w, o, iters);
      if (mode == 1) kern<1><<<blocks, threads>>>(w, o, iters);
      if (mode == 2) kern<2><<<blocks, threads>>>(w, o, iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double fmas = (double)blocks * threads * iters * 16 * NACC * (mode == 2 ? 1 : 2);
      if (rep) printf("%-20s %.3f ms  %.1f TFLOP/s\n", names[mode], ms, 2 * fmas / ms / 1e9);
    }
  }
  for (int na : {3, 5, 10}) {
    for (int per_cu : {4, 5, 16}) {
      const int nb = 256 * per_cu;
      const int it2 = iters * 16 / 24 * 10 / na;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (na == 3) kern_px<24, 3><<<nb, 192>>>(w, o, it2);
        if (na == 5) kern_px<24, 5><<<nb, 192>>>(w, o, it2);
        if (na == 10) kern_px<24, 10><<<nb, 192>>>(w, o, it2);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double fmas = (double)nb * 192 * it2 * 24 * na * 2;
        if (rep) printf("px pattern, %2d accs, %2d WG(192)/CU = %4.1f waves/SIMD: %.3f ms  %.1f TFLOP/s\n", na, per_cu, per_cu * 3 / 4.0, ms, 2 * fmas / ms / 1e9);
      }
    }
  }
  return 0;
}
