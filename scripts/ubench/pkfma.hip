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


// px pattern + one ds_read2_b32 (or ds_read_b64) per 10-FMA block into a
// register that the FMAs do not read: cost of LDS returns alone.
template <int KW, int LDSK>
__global__ __launch_bounds__(192) void kern_lds(const float* __restrict__ w, float* __restrict__ out, int iters) {
  __shared__ float sh[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) sh[i] = (float)i;
  __syncthreads();
  f2 acc[10];
  for (int c = 0; c < 10; ++c) acc[c] = (f2){(float)threadIdx.x + c, (float)c};
  f2 px[10 + KW - 1];
  for (int q = 0; q < 10 + KW - 1; ++q) px[q] = (f2){1.0001f * threadIdx.x + q, 0.999f * q};
  float ws[KW];
  for (int k = 0; k < KW; ++k) ws[k] = w[k];
  const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(sh + (threadIdx.x & 63) * 5);
  f2 sink = (f2){0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const f2 w2 = (f2){ws[j], ws[j]};
#pragma unroll
      for (int c = 0; c < 10; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + j], acc[c]);
      f2 d;
      if (LDSK == 1) asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(d) : "v"(base), "i"(j), "i"(j + 116));
      else if (LDSK == 2) asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(j * 8));
      if (LDSK) {
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        sink = sink + d;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" : "+v"(px[0]), "+v"(px[1]));
  }
  float s = sink.x + sink.y;
  for (int c = 0; c < 10; ++c) s += acc[c].x + acc[c].y;
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
  for (int mode : {0, 1, 2}) {
    for (int per_cu : {4, 5, 8}) {
      const int nb = 256 * per_cu;
      const int it2 = iters * 16 / 24;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (mode == 0) kern_lds<24, 0><<<nb, 192>>>(w, o, it2);
        if (mode == 1) kern_lds<24, 1><<<nb, 192>>>(w, o, it2);
        if (mode == 2) kern_lds<24, 2><<<nb, 192>>>(w, o, it2);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double fmas = (double)nb * 192 * it2 * 24 * 10 * 2;
        if (rep) printf("px+lds mode %d (0 none, 1 ds_read2_b32, 2 ds_read_b64) per 10 pk_fma, %d WG/CU: %.3f ms %.1f TFLOP/s\n", mode, per_cu, ms, 2 * fmas / ms / 1e9);
      }
    }
  }
  return 0;
}
