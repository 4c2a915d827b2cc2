// lm_dev_common.h — device-side helpers shared by the kernel translation
// units (lm_kernels.hip via lm_runtime.hip, lm_bbox.hip).
#ifndef LM_DEV_COMMON_H
#define LM_DEV_COMMON_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

// Frame pointers come from a device array (frame_ptr), so the compiler cannot
// tell that they point to global memory and would access the frames with FLAT
// instructions (longer latency, and they hold the LDS counter too); the casts
// below make those accesses global_load_*.
typedef __attribute__((address_space(1))) const uint8_t lm_gu8;
typedef __attribute__((address_space(1))) const uint32_t lm_gu32;
typedef unsigned lm_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const lm_u32x4 lm_gu4;
DEV const lm_gu8* as_global(const uint8_t* p) { return (const lm_gu8*)p; }

#endif  // LM_DEV_COMMON_H
