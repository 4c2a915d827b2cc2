/*
 * lm_synth.h — deterministic synthetic two-view mouse video (test & bench input).
 *
 * NOT part of the reference surface: the reference ships no video, model or
 * calibration fixtures, so parity tests and benchmarks run on
 * this generator.  Integer-only arithmetic (splitmix64 noise,
 * triangle-wave motion, integer ellipse/disc tests) so the C, HIP and numpy
 * implementations agree bit for bit on every pixel.
 *
 * Scene at scale s (s = 1 for 1024x256, s = 2 for the 1920x512 config):
 *   side view rows [0, 96 s), bottom view rows [96 s, H)
 *   body ellipse +80, 4 paw discs +100, snout disc +110, 3-px tail line +150,
 *   over background 16 + u16 and per-frame noise in [0, 6); saturating u8.
 */
#ifndef LM_SYNTH_H
#define LM_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define LM_SYNTH_FN __host__ __device__ static inline
#else
#define LM_SYNTH_FN static inline
#endif

typedef struct {
  int32_t rows, cols;   /* frame size */
  int32_t scale;        /* geometry scale s */
  int32_t cx0;          /* body centre x at phase 0 */
  int32_t side_cy, bottom_cy;
} lm_synth_scene;

LM_SYNTH_FN uint64_t lm_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Integer triangle wave: tri(0)=0, tri(P/4)=A, tri(P/2)=0, tri(3P/4)=-A. */
LM_SYNTH_FN int32_t lm_tri(int64_t t, int32_t period, int32_t amp) {
  int64_t p = t % period;
  if (p < 0) p += period;
  int64_t q = (4 * (int64_t)amp * p) / period; /* 0 .. 4A */
  if (q <= amp) return (int32_t)q;
  if (q <= 3 * (int64_t)amp) return (int32_t)(2 * amp - q);
  return (int32_t)(q - 4 * (int64_t)amp);
}

LM_SYNTH_FN lm_synth_scene lm_synth_default_scene(int32_t rows, int32_t cols) {
  lm_synth_scene s;
  s.rows = rows;
  s.cols = cols;
  s.scale = rows >= 512 ? 2 : 1;
  s.cx0 = (cols * 500) / 1024;
  s.side_cy = 48 * s.scale;
  s.bottom_cy = 176 * s.scale;
  return s;
}

LM_SYNTH_FN uint8_t lm_synth_background(int64_t idx) {
  return (uint8_t)(16 + lm_splitmix64(0xB4C0000000000000ull ^ (uint64_t)idx) % 16);
}

LM_SYNTH_FN int32_t lm_synth_in_ellipse(int32_t dx, int32_t dy, int32_t a, int32_t b) {
  /* (dx/a)^2 + (dy/b)^2 <= 1 in integers */
  int64_t lhs = (int64_t)dx * dx * b * b + (int64_t)dy * dy * a * a;
  return lhs <= (int64_t)a * a * b * b;
}

/* Pixel (r, c) of frame f. */
LM_SYNTH_FN uint8_t lm_synth_pixel(const lm_synth_scene* sc, int64_t f, int32_t r, int32_t c) {
  const int32_t s = sc->scale;
  const int64_t idx = (int64_t)r * sc->cols + c;
  int32_t v = lm_synth_background(idx);
  v += (int32_t)(lm_splitmix64(((uint64_t)(0x5EED0000u + (uint32_t)f) << 32) ^ (uint64_t)idx) % 6);
  const int32_t cx = sc->cx0 + s * lm_tri(f, 50, 40);
  const int32_t side = r < 96 * s;
  const int32_t cy = side ? sc->side_cy : sc->bottom_cy;
  /* body */
  if (lm_synth_in_ellipse(c - cx, r - cy, 150 * s, (side ? 30 : 50) * s)) v += 80;
  /* paws */
  for (int32_t k = 0; k < 4; ++k) {
    const int32_t dxk = (k == 0 ? -110 : k == 1 ? -40 : k == 2 ? 40 : 110) * s;
    const int32_t px = cx + dxk + s * lm_tri(f + 5 * k, 20, 30);
    const int32_t py = side ? 86 * s : sc->bottom_cy + ((k & 1) ? 58 : -58) * s;
    const int32_t dx = c - px, dy = r - py;
    if (dx * dx + dy * dy <= 36 * s * s) v += 100;
  }
  /* snout */
  {
    const int32_t dx = c - (cx + 158 * s), dy = r - cy;
    if (dx * dx + dy * dy <= 25 * s * s) v += 110;
  }
  /* tail: 3-px line from cx-150 leftwards for 180 px */
  if (c >= cx - 330 * s && c <= cx - 150 * s) {
    const int32_t dy = r - cy;
    if (dy >= -s && dy <= s) v += 150;
  }
  return (uint8_t)(v > 255 ? 255 : v);
}

#endif /* LM_SYNTH_H */
