/*
 * locomouse_track.h — C-ABI of the tracking stage that follows the per-frame
 * detection path, exported by liblocomouse_host.so.
 *
 * Host code (the tracker is sequential in frames and tiny next to detection);
 * it consumes the containers lm_detect_batch* returns (include/locomouse_hip.h)
 * and produces what the reference's exportResults writes.
 *
 *   lm_match2nd         replaces match2nd(...) + computeCostTrack(...)
 *                       (match2nd/match2nd.cpp:11-166, :168-190; the
 *                       MATLAB-side MEX of the same tracker binds the same
 *                       arrays)
 *   lm_compute_tracks   replaces LocoMouse::computeBottomTracks,
 *                       computeSideTracks and the track part of exportResults
 *                       (LocoMouse_class.cpp:2153-2214, :2216-2346, :2348-2482)
 *   lm_write_tracks_yaml  OUTPUT << "paw_tracks0" << M ... into
 *                       <outdir>/output_<stem>.yml (LocoMouse_class.cpp:360)
 *
 * Errors: LM_ERR_INVALID_ARGUMENT for malformed arrays, LM_ERR_RUNTIME for
 * the reference's runtime failures; text in lm_track_last_error() (per thread).
 * Output arrays are thread-local and valid until the next call on the thread.
 */
#ifndef LOCOMOUSE_TRACK_H
#define LOCOMOUSE_TRACK_H

#include "locomouse_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t n_frames;
  const int32_t* paw_tracks;         /* [4][n][3]: x, y (bottom), z (side); -1 = missing */
  const int32_t* snout_tracks;       /* [1][n][3] */
  const int32_t* tracks_tail;        /* [3][15 n] */
  const int32_t* track_index_bottom; /* [5][n]: TRACK_INDEX_PAW_BOTTOM rows 0-3, TRACK_INDEX_SNOUT_BOTTOM */
  const int32_t* track_index_side;   /* [5][n]: TRACK_INDEX_PAW_SIDE rows 0-3, TRACK_INDEX_SNOUT_SIDE */
} lm_tracks;

const char* lm_track_last_error(void);

/* match2nd over one video.  Frame f's unary MyMat is n_loc[f] x n_cols,
 * column-major, at unary[unary_offset[f] .. unary_offset[f+1]).  Transition
 * f -> f+1 (f < n_frames-1) is a MATSPARSE: pw_dims[3f..3f+2] = rows
 * (n_loc[f+1] + nong), cols (n_loc[f] + nong), nnz; Jc at
 * pw_jc + pw_jc_offset[f] (cols + 1 entries), Ir / Pr at pw_nz_offset[f].
 * labels: n_points x n_frames, row-major.  cost (may be NULL) receives
 * computeCostTrack(labels, ...), which needs n_points >= 4. */
lm_status lm_match2nd(int32_t n_frames, int32_t n_points, int32_t n_cols, int32_t nong, double occlusion_point_cost,
                      double bam_tie, const int32_t* n_loc, const int64_t* unary_offset, const double* unary,
                      const int32_t* pw_dims, const int64_t* pw_jc_offset, const int32_t* pw_jc,
                      const int64_t* pw_nz_offset, const int32_t* pw_ir, const double* pw_pr,
                      const int32_t* permutation, int32_t* labels, double* cost);

/* Bottom tracks (4 paw orders tried, snout), side tracks and their export
 * over a whole video's detection results (first_frame 0, n_frames = N_FRAMES).
 * geometry: lm_get_geometry of the detection context; bb: per-frame
 * bottom-right corners [n][3] = BB_X_POS, BB_Y_BOTTOM_POS, BB_Y_SIDE_POS. */
lm_status lm_compute_tracks(const lm_batch_result* video, const lm_geometry* geometry, const lm_params* params,
                            const uint32_t* bb, lm_tracks* out);

/* The exported tracks as OpenCV FileStorage YAML (!!opencv-matrix, dt: i). */
lm_status lm_write_tracks_yaml(const char* path, const lm_tracks* tracks);

#ifdef __cplusplus
}
#endif

#endif
