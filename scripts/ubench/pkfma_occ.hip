// v_pk_fma_f32 issue rate against waves per SIMD (1..4) with the ring
// kernel's instruction shapes: blocks of 20 v_pk_fma_f32 (two weight pairs
// from SGPRs, ten accumulator pairs: the rw_pair_ab asm block), NB blocks per
// iteration, and per iteration, by MODE:
//   0: nothing else (FMAs only)
//   1: s_waitcnt lgkmcnt(0), then 2 ds_read2_b32 issued (used next iteration)
//   2: 2 ds_read2_b32 issued, no wait
//   3: s_waitcnt lgkmcnt(0) only
//   4: as 1 plus an s_load_dwordx4 of weights (SMEM in the same counter)
// k_corr_rw's kw-30 step is ~75 FMAs and ~9 ds_read2 per wait.
//   hipcc --offload-arch=gfx950 -O3 -o pkfma_occ pkfma_occ.hip && ./pkfma_occ
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
#define F(a, w, p, sel) "v_pk_fma_f32 %" #a ", %" #w ", %" #p ", %" #a " " sel "\n"
#define S0 "op_sel_hi:[0,1,1]"
#define S1 "op_sel:[1,0,0] op_sel_hi:[1,1,1]"
__device__ __forceinline__ void blk(f2 (&a)[5], f2 (&b)[5], f2 wa, f2 wb, const f2* px) {
  asm volatile(F(0, 10, 12, S0) F(1, 10, 13, S0) F(2, 10, 14, S0) F(3, 10, 15, S0) F(4, 10, 16, S0)
               F(5, 11, 12, S0) F(6, 11, 13, S0) F(7, 11, 14, S0) F(8, 11, 15, S0) F(9, 11, 16, S0)
               F(0, 10, 13, S1) F(1, 10, 14, S1) F(2, 10, 15, S1) F(3, 10, 16, S1) F(4, 10, 17, S1)
               F(5, 11, 13, S1) F(6, 11, 14, S1) F(7, 11, 15, S1) F(8, 11, 16, S1) F(9, 11, 17, S1)
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3]), "+v"(b[4])
               : "s"(wa), "s"(wb), "v"(px[0]), "v"(px[1]), "v"(px[2]), "v"(px[3]), "v"(px[4]), "v"(px[5]));
}

template <int MODE, int NB>
__global__ __launch_bounds__(256) void k(float* out, const float* w, int iters) {
  __shared__ float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = (float)(i & 7);
  __syncthreads();
  f2 a[5], b[5], px[6];
  for (int c = 0; c < 5; ++c) a[c] = b[c] = (f2){0.f, 0.f};
  for (int c = 0; c < 6; ++c) px[c] = (f2){(float)threadIdx.x, 1.f};
  const f2* W = reinterpret_cast<const f2*>(w);
  f2 wa = W[0], wb = W[1];
  unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)lds + (threadIdx.x & 63) * 4;
  f2 q0 = px[0], q1 = px[5];
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 1 || MODE == 3 || MODE == 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
      px[0] = q0;
      px[5] = q1;
      asm volatile("ds_read2_b32 %0, %2 offset0:0 offset1:72\n ds_read2_b32 %1, %2 offset0:1 offset1:73"
                   : "=v"(q0), "=v"(q1) : "v"(base) : "memory");
    }
    if constexpr (MODE == 4) {
      asm volatile("s_load_dwordx2 %0, %2, 0x0\n s_load_dwordx2 %1, %2, 0x8" : "=s"(wa), "=s"(wb) : "s"(W) : "memory");
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) blk(a, b, wa, wb, px);
  }
  float s = q0.x + q1.y;
  for (int c = 0; c < 5; ++c) s += a[c].x + a[c].y + b[c].x + b[c].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int NB>
void run(int cus, float* out, float* w) {
  const int iters = 80000 / NB;
  for (int wps = 1; wps <= 4; ++wps) {
    const int blocks = cus * wps;  // 4-wave workgroups, one wave per SIMD each
    k<MODE, NB><<<blocks, 256>>>(out, w, iters);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) k<MODE, NB><<<blocks, 256>>>(out, w, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flop = 3.0 * blocks * 4 * 64 * (double)iters * NB * 20 * 4;
    printf("mode %d fma/wait %3d waves/SIMD %d: %7.3f ms %6.1f TFLOP/s (%.3f of 157.3)\n", MODE, NB * 20, wps, ms / 3,
           flop / (ms / 1e3) / 1e12, flop / (ms / 1e3) / 1e12 / 157.3);
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  float *out, *w;
  (void)hipMalloc(&out, sizeof(float) * 256 * cus * 8);
  (void)hipMalloc(&w, 64);
  (void)hipMemset(w, 0, 64);
  run<0, 1>(cus, out, w);
  run<1, 1>(cus, out, w);
  run<2, 1>(cus, out, w);
  run<3, 1>(cus, out, w);
  run<1, 4>(cus, out, w);
  run<3, 4>(cus, out, w);
  run<4, 4>(cus, out, w);
  run<1, 8>(cus, out, w);
  run<4, 8>(cus, out, w);
  return 0;
}
