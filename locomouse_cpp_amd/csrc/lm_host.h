// lm_host.h — host-side utilities shared by the translation units of
// liblocomouse_hip.so (lm_runtime.hip, lm_bbox.hip): HIP error checking,
// device / pinned buffers (with the LM_GUARD diagnostics), and the C-ABI's
// status + last-error convention.
#ifndef LM_HOST_H
#define LM_HOST_H

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "locomouse_hip.h"

#define LM_API extern "C" __attribute__((visibility("default")))

// Error text of the last failing C-ABI call on this thread (lm_last_error).
inline thread_local std::string g_err = "";


struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPCHK(x) hip_check((x), #x)

// Copies and fills on a context's own (non-blocking) stream, waited for.
// Never the synchronous hipMemcpy / hipMemset: they run on the legacy stream,
// which HIP refuses while any other thread's stream is capturing a graph
// (several contexts, one per host thread).
#define COPY_SYNC(dst, src, bytes, kind, st) \
  do {                                              \
    HIPCHK(hipMemcpyAsync((dst), (src), (bytes), (kind), (st))); \
    HIPCHK(hipStreamSynchronize(st));                \
  } while (0)
#define SET_SYNC(dst, v, bytes, st)                   \
  do {                                              \
    HIPCHK(hipMemsetAsync((dst), (v), (bytes), (st))); \
    HIPCHK(hipStreamSynchronize(st));                \
  } while (0)

inline bool dbg_env(const char* name) {  // diagnostics switches (LM_* environment variables)
  const char* v = getenv(name);
  return v && atoi(v) != 0;
}

// Diagnostics (LM_GUARD=1): every device buffer gets 64 KiB guard zones on
// both sides filled with 0xA5; lm_detect_batch* checks them after each batch
// and fails with the buffer's address if a kernel wrote outside it.
constexpr size_t kGuard = 64 * 1024;
inline bool guard_mode() {
  static const bool on = [] {
    const char* v = getenv("LM_GUARD");
    return v && atoi(v) != 0;
  }();
  return on;
}
inline std::mutex g_guard_mu;
inline std::map<const void*, size_t> g_guarded;  // user pointer -> user bytes

inline void guard_check_all() {
  std::vector<std::pair<const void*, size_t>> bufs;
  {
    std::lock_guard<std::mutex> lk(g_guard_mu);
    bufs.assign(g_guarded.begin(), g_guarded.end());
  }
  std::vector<uint8_t> h(kGuard);
  for (const auto& b : bufs) {
    const uint8_t* u = static_cast<const uint8_t*>(b.first);
    for (int side = 0; side < 2; ++side) {
      const uint8_t* g = side ? u + b.second : u - kGuard;
      HIPCHK(hipMemcpy(h.data(), g, kGuard, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < kGuard; ++i)
        if (h[i] != 0xA5) {
          char m[256];
          snprintf(m, sizeof m, "guard: write %s buffer %p (%zu bytes) at offset %lld", side ? "past" : "before",
                   (const void*)u, b.second,
                   side ? (long long)(b.second + i) : -(long long)(kGuard - i));
          throw std::runtime_error(m);
        }
    }
  }
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    if (guard_mode()) {
      uint8_t* base = nullptr;
      const size_t bytes = count * sizeof(T);
      HIPCHK(hipMalloc(&base, bytes + 2 * kGuard));
      HIPCHK(hipMemset(base, 0xA5, kGuard));
      HIPCHK(hipMemset(base + kGuard + bytes, 0xA5, kGuard));
      p = reinterpret_cast<T*>(base + kGuard);
      std::lock_guard<std::mutex> lk(g_guard_mu);
      g_guarded[p] = bytes;
    } else {
      HIPCHK(hipMalloc(&p, count * sizeof(T)));
    }
    n = count;
  }
  void release() {
    if (p) {
      if (guard_mode()) {
        {
          std::lock_guard<std::mutex> lk(g_guard_mu);
          g_guarded.erase(p);
        }
        (void)hipFree(reinterpret_cast<uint8_t*>(p) - kGuard);
      } else {
        (void)hipFree(p);
      }
    }
    p = nullptr;
    n = 0;
  }
  ~DevBuf() { release(); }
};

template <class T>
struct HostBuf {  // pinned, mapped into the device address space (d: device-side pointer)
  T* p = nullptr;
  T* d = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    release();
    if (count == 0) count = 1;
    HIPCHK(hipHostMalloc(&p, count * sizeof(T), hipHostMallocMapped));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), p, 0));
    n = count;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    d = nullptr;
    n = 0;
  }
  ~HostBuf() { release(); }
};

inline lm_status fail(lm_status s, const std::string& m) {
  g_err = m;
  return s;
}

// Runs f, mapping the reference's exception types to lm_status codes.
template <class F>
lm_status guarded(F&& f) {
  try {
    f();
    return LM_OK;
  } catch (const std::invalid_argument& e) {
    return fail(LM_ERR_INVALID_ARGUMENT, e.what());
  } catch (const HipError& e) {
    return fail(LM_ERR_HIP, e.what());
  } catch (const std::exception& e) {
    return fail(LM_ERR_RUNTIME, e.what());
  }
}

// k_minmax + k_lut (lm_kernels.hip) for slots s0 .. n-1: the per-frame
// normalize LUT (+ TM imadjust when use_adj), shared with the BB pass.
hipError_t launch_minmax_lut(const uint8_t* const* frame_ptr, const uint8_t* bkg, int npix, int s0, int n,
                             unsigned* mm, const uint8_t* adj, int use_adj, uint8_t* luts, hipStream_t st);

#endif  // LM_HOST_H
