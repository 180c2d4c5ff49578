/*
 * bxstrongsort.h — C ABI of the StrongSort engine in libbxassoc.so (MI355X, gfx950).
 *
 * Boundary: everything the fork's "enhanced" StrongSort.update(dets, img, embs) computes per
 * frame — detection quality and ordering, crowd detection and its parameter adjustments, camera
 * warp, XYAH Kalman predict, the three-stage matching (appearance cascade on high- then
 * medium-confidence detections: NN-gallery cosine distance on the fp64 matrix cores, Mahalanobis
 * gating, motion/quality/confidence cost shaping, scipy's linear_sum_assignment; then IoU), the
 * Kalman/feature updates, misses, ID recovery from the lost-track buffer, births, deaths, the
 * gallery's partial_fit budget pruning and the output rows — runs on the GPU behind these entry
 * points: per frame a detection-feature kernel (wave per detection), the gallery distance
 * (fp64 MFMA, wave per confirmed track and detection block), the recovery similarities, the
 * pre-match kernel (one wave per sequence), the stage 1/2 costs (wave per confirmed track), the
 * matching kernel (one wave per sequence), the track updates (wave per match), the post-match
 * kernel (recovery, births, lost buffer, outputs; wave per sequence) and partial_fit (wave per
 * track).
 *
 * Reference interfaces replaced (file:line in muntherr/boxmot @ /root/reference):
 *   bx_ss_create/step/update_host  StrongSort.__init__ / StrongSort.update
 *                                  boxmot/trackers/strongsort/strongsort.py:45-181, 285-345
 *     Tracker                      trackers/strongsort/sort/tracker.py:63-344
 *     Track / Detection            sort/track.py:76-400, sort/detection.py:35-42
 *     matching_cascade, min_cost_matching, gate_cost_matrix + cost shaping,
 *     NearestNeighborDistanceMetric sort/linear_assignment.py:14-618
 *     iou_cost                     sort/iou_matching.py:10-87
 *     detect_crowd_situations      utils/occlusion_handler.py:45-87, 464-490
 * The fork needs the minimal patch P6; `born_confirmed` stands for its
 * GITHUB_ACTIONS=true switch (D8).  handle_occlusions=True (OcclusionAwareTracker,
 * utils/occlusion_handler.py:312-439) is a host post-process (boxmot_amd/occlusion.py) over the
 * track-attribute calls below; it raises where the reference crashes on mutual occlusion (D7).
 * Bit-identical to oracle/bxo_strongsort.c (pinned by tests/golden/trk_strongsort_*.npz).
 *
 * Conventions as in bxassoc.h: device pointers unless a name ends in _host, asynchronous on
 * `stream`, every function returns a bx_status (bx_last_error explains failures).
 */
#ifndef BXSTRONGSORT_H
#define BXSTRONGSORT_H

#include <stdint.h>

#include "bxassoc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* StrongSort constructor parameters (strongsort.py:45-66 names and defaults: min_conf .1,
 * max_cos_dist .15, max_iou_dist .7, max_age 50, n_init 2, nn_budget 150, mc_lambda .995,
 * ema_alpha .9, conf_thresh_high .7, conf_thresh_low .3, id_preservation_weight .1,
 * crowd_detection 1). */
typedef struct {
    int32_t n_seq;      /* independent sequences held by this engine */
    int32_t track_cap;  /* track slots per sequence, live + lost-buffer (<= 1024) */
    int32_t det_cap;    /* max detections per frame per sequence (<= 1024) */
    int32_t emb_dim;    /* embedding dimension F (float64 embeddings, required) */
    int32_t vec_cap;    /* feature vectors kept per track slot (its features + gallery
                           samples; <= 64, default 32).  max(nn_budget, crowd budget) + 10
                           <= 320 (gallery entries per track) */
    double min_conf, max_cos_dist, max_iou_dist;
    int32_t max_age, n_init, nn_budget;
    double mc_lambda, ema_alpha, conf_thresh_high, conf_thresh_low, id_preservation_weight;
    int32_t crowd_detection, born_confirmed;
} bx_ss_config;

typedef struct bx_ss bx_ss;

int bx_ss_create(const bx_ss_config *cfg, bx_ss **out);
int bx_ss_destroy(bx_ss *e);
/* Forget all tracks of sequences [seq0, seq0+nseq). */
int bx_ss_reset(bx_ss *e, int seq0, int nseq, void *stream);
/* One frame for sequences [seq0, seq0+nseq).
 *   dets    [sum N][6] float64 (x1,y1,x2,y2,conf,cls) — StrongSort has no setup_decorator,
 *           detections are not rounded to float32
 *   det_off [nseq+1] int32 prefix offsets
 *   embs    [sum N][emb_dim] float64
 *   warps   [nseq][6] float64 2x3 camera-motion affine per sequence, NULL = identity
 *   out     [sum N][10] float64 rows [x1,y1,x2,y2,id,conf,cls,det_ind,quality,occlusion(=0)]
 *           in track-list order, sequence k from row det_off[k]
 *   out_count [nseq] int32 */
int bx_ss_step(bx_ss *e, int seq0, int nseq, const double *dets, const int32_t *det_off,
               const double *embs, const double *warps, double *out, int32_t *out_count,
               void *stream);
/* Host-memory path for one sequence (the drop-in update). out must hold n rows of 10. */
int bx_ss_update_host(bx_ss *e, int seq, const double *dets, int n, const double *embs,
                      const double *warp, double *out, int *n_out, void *stream);
/* Latched device status (BX_OK, BX_ERR_TRACK_OVERFLOW — track slots or a slot's vector pool
 * exhausted — or BX_ERR_CAPACITY). */
/* Capacity growth (the reference's track list is unbounded: sort/tracker.py:118-181 (self.tracks), sort/track.py:98-105): copy every
 * sequence's tracker state of `src` into `dst`, a fresh engine with the same configuration and
 * sequences and track_cap / det_cap at least src's (slot ids stay valid).  Synchronous. */
int bx_ss_copy_state(bx_ss *dst, bx_ss *src);
int bx_ss_status(bx_ss *e, int *status);
/* Per-sequence counters (host): frame count, next id, live tracks, lost-buffer tracks. */
int bx_ss_counters_host(bx_ss *e, int seq, int *frame_count, int *next_id, int *n_tracks,
                        int *n_lost);
/* Track list in list order (host): ids, states (1 tentative, 2 confirmed), means [8], covs [64]. */
int bx_ss_tracks_host(bx_ss *e, int seq, int cap, int32_t *ids, int32_t *state, double *mean,
                      double *cov, int *n);
/* Write Track.mean [n][8] / Track.covariance [n][64] of live tracks by id (host, synchronous;
 * either may be NULL): the state edit OcclusionAwareTracker._update_track_with_predicted_position
 * makes (utils/occlusion_handler.py:380-398; sort/track.py:76-400 attributes).
 * BX_ERR_INVALID for an unknown id. */
int bx_ss_state_set_host(bx_ss *e, int seq, int n, const int32_t *ids, const double *mean,
                         const double *cov);
/* Track attributes the host-side OcclusionAwareTracker reads and edits
 * (utils/occlusion_handler.py:341-417; sort/track.py:76-131 attributes), host and synchronous,
 * list order / by id:
 *   bx_ss_track_attrs_host      ids, quality_score, conf, _max_age, len(features) (any NULL)
 *   bx_ss_track_attrs_set_host  quality_score / conf / _max_age by id (NULL arrays untouched)
 *   bx_ss_last_feature_host     features[-1] [n][emb_dim] by id
 *   bx_ss_last_feature_set_host `features[-1] = v` [n][emb_dim] by id (normalize: v / (wave-order
 *                               norm + 1e-8) first, the engine's np.linalg.norm order); the
 *                               gallery keeps the replaced vector's content
 * BX_ERR_INVALID for an unknown id (or a track without features for the feature calls). */
int bx_ss_track_attrs_host(bx_ss *e, int seq, int cap, int32_t *ids, double *quality,
                           double *conf, int32_t *max_age, int32_t *n_features, int *n);
int bx_ss_track_attrs_set_host(bx_ss *e, int seq, int n, const int32_t *ids, const double *quality,
                               const double *conf, const int32_t *max_age);
int bx_ss_last_feature_host(bx_ss *e, int seq, int n, const int32_t *ids, double *feats);
int bx_ss_last_feature_set_host(bx_ss *e, int seq, int n, const int32_t *ids, const double *feats,
                                int normalize);
/* Last-frame statistics over sequences [seq0, seq0+nseq) (host): sums[7] = {detections kept,
 * tracks entering the frame, confirmed tracks queried next frame, gallery sample rows compared,
 * output rows, max frame counter, matches} — bench.py's unit counts. */
int bx_ss_frame_stats_host(bx_ss *e, int seq0, int nseq, int64_t *sums);
/* How the cascade / IoU LSAPs (linear_assignment.py:14-93's linear_sum_assignment) are solved:
 * fast = 1 (default) solve + certify — rows' minima in parallel, Crouse's search for the
 * contested ones, then a reduced-cost certificate that the optimum is unique up to pairs
 * min_cost_matching rejects; scipy's own row order only for a tied level (and a whole cascade
 * stage in scipy's order when a tie follows a level whose unmatched order was not certified).
 * fast = 0: scipy's row order always.  Both give the reference's matches.  Synchronous. */
int bx_ss_set_lsap_mode(bx_ss *e, int fast);
/* LSAP counters of sequences [seq0, seq0+nseq) since creation: sums[5] = {solves, certified
 * unique, certified unique up to rejected pairs, ties re-solved in scipy's order, cascade stages
 * restarted in scipy's order}.  Synchronous. */
int bx_ss_lsap_stats_host(bx_ss *e, int seq0, int nseq, int64_t *sums);
/* Test entry point of the match kernel's LSAP on a dense row-major [R][CC] float64 cost (device),
 * 1 <= R <= CC <= 1024: fast = 0 scipy's linear_sum_assignment row order, 1 solve + certify
 * against max_d (min_cost_matching's rejection threshold).  rows / cols [R] (device) get the
 * pairs in row order; info[2] (device) = {pairs, or -1 when fast found a tie that could change a
 * real (<= max_d) pair; 0 unique, 1 unique up to rejected pairs, 2 tie}; status (device) is
 * latched BX_ERR_INVALID on an engine fault. */
int bx_ss_lsap_op(const double *cost, int R, int CC, double max_d, int fast, int32_t *rows,
                  int32_t *cols, int32_t *info, int32_t *status, void *stream);
/* Timing probe: stage 0 = detection features, 1 = gallery distance, 2 = recovery similarities,
 * 3 = pre-match (crowd, warp, quality, predict), 4 = stage 1/2 costs, 5 = matching, 6 = track
 * updates, 7 = post-match, 8 = partial_fit; -1 = off (see bx_boost_probe). */
int bx_ss_probe(bx_ss *e, int stage);
int bx_ss_probe_read(bx_ss *e, double *total_ms, int *count);

#ifdef __cplusplus
}
#endif

#endif /* BXSTRONGSORT_H */
