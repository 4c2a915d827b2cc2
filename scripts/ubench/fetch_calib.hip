// FETCH_SIZE / WRITE_SIZE calibration (gfx950) for the access widths the
// detection kernels use (MI355X_MICROARCH.md HBM section: only 16-B/lane
// streaming reads and stores are calibrated there).  Every kernel touches a
// known number of distinct bytes of a 1 GiB buffer (past the 256 MiB MALL, so
// each line comes from HBM once); run under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE  -- ./fetch_calib
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE  -- ./fetch_calib
// and divide the counter (KiB) by the byte count the program prints.
//   rd_b128   16 B per lane, consecutive (the guide's calibrated case)
//   rd_b32    4 B per lane, consecutive dwords (k_corr_rw's ring rows, k_tileflag)
//   rd_run5   five consecutive dwords per lane at a 16-B lane stride
//             (k_ingest's run gather: each dword read by one or two lanes)
//   rd_u8     1 B per lane, consecutive bytes
//   wr_b128   16 B per lane stores (k_ingest's ext-crop stores)
//   wr_b32    4 B per lane stores
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ void rd_b128(const uint4* __restrict__ a, size_t n, unsigned* __restrict__ sink) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) sink[0] = s;
}

__global__ void rd_b32(const unsigned* __restrict__ a, size_t n, unsigned* __restrict__ sink) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s ^= a[i];
  if (s == 0x12345678u) sink[0] = s;
}

__global__ void rd_run5(const unsigned* __restrict__ a, size_t nchunks, unsigned* __restrict__ sink) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nchunks; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned* p = a + 4 * i;
#pragma unroll
    for (int u = 0; u < 5; ++u) s ^= p[u];
  }
  if (s == 0x12345678u) sink[0] = s;
}

__global__ void rd_u8(const uint8_t* __restrict__ a, size_t n, unsigned* __restrict__ sink) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 0x12345678u) sink[0] = s;
}

__global__ void wr_b128(uint4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

__global__ void wr_b32(unsigned* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (unsigned)i;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  uint8_t* buf = nullptr;
  unsigned* sink = nullptr;
  CHK(hipMalloc(&buf, bytes + 64));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(buf, 1, bytes + 64));
  CHK(hipDeviceSynchronize());
  const dim3 grid(256 * 8), blk(256);
  // rd_run5 reads 16 B per lane plus 4 B of the next lane's chunk: distinct bytes = 16 * nchunks + 4
  const size_t nchunks = bytes / 16;
  for (int rep = 0; rep < 2; ++rep) {
    rd_b128<<<grid, blk>>>(reinterpret_cast<const uint4*>(buf), bytes / 16, sink);
    rd_b32<<<grid, blk>>>(reinterpret_cast<const unsigned*>(buf), bytes / 4, sink);
    rd_run5<<<grid, blk>>>(reinterpret_cast<const unsigned*>(buf), nchunks, sink);
    rd_u8<<<grid, blk>>>(buf, bytes, sink);
    wr_b128<<<grid, blk>>>(reinterpret_cast<uint4*>(buf), bytes / 16);
    wr_b32<<<grid, blk>>>(reinterpret_cast<unsigned*>(buf), bytes / 4);
  }
  CHK(hipDeviceSynchronize());
  printf("{\"bytes_per_dispatch\": %zu, \"kernels\": [\"rd_b128\", \"rd_b32\", \"rd_run5\", \"rd_u8\", \"wr_b128\", \"wr_b32\"]}\n",
         bytes);
  CHK(hipFree(buf));
  CHK(hipFree(sink));
  return 0;
}
