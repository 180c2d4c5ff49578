/*
 * bxboost.h — C ABI of the BoostTrack engine in libbxassoc.so (MI355X, gfx950).
 *
 * Boundary: everything BoostTrack.update(dets, img, embs) computes per frame — the camera-motion
 * warp of every track's box, the 8-state constant-noise Kalman predict, the detection-confidence
 * boosts (DLO: soft-BIoU / Mahalanobis-softmax / shape similarity; DUO: isolated low-confidence
 * detections), the association cost IoU + conf-weighted IoU + Mahalanobis softmax + shape + ReID
 * (dets_embs @ trk_embs.T on the fp64 matrix cores), the one-to-one fast path or lapx JV, the
 * IoU/appearance validation, Kalman updates, embedding EMA, births, deaths and the filtered
 * output rows — runs on the GPU behind these entry points: per frame a ReID contraction kernel
 * (workgroup per 32x64 output tile), the frame kernel (a 1-4 wave workgroup per sequence) and an
 * embedding-update kernel (wave per updated track).
 *
 * Reference interfaces replaced (file:line in muntherr/boxmot @ /root/reference):
 *   bx_boost_create/step/update_host  BoostTrack.__init__ / BoostTrack.update
 *                                     boxmot/trackers/boosttrack/boosttrack.py:123-341
 *     KalmanBoxTracker                boosttrack.py:45-121
 *     KalmanFilter + ConstantNoise    boxmot/trackers/boosttrack/kalmanfilter.py:8-157
 *     dlo/duo_confidence_boost,       boosttrack.py:356-456
 *     get_mh_dist_matrix
 *     associate / linear_assignment / boxmot/trackers/boosttrack/assoc.py:9-200
 *     match / iou_batch / soft_biou_batch / shape_similarity / MhDist_similarity
 * Bit-identical to oracle/bxo_boost.c (pinned by tests/golden/trk_boosttrack_*.npz).
 *
 * Conventions as in bxassoc.h: device pointers unless a name ends in _host, asynchronous on
 * `stream`, every function returns a bx_status (bx_last_error explains failures).
 */
#ifndef BXBOOST_H
#define BXBOOST_H

#include <stdint.h>

#include "bxassoc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* BoostTrack constructor parameters (boosttrack.py:154-181 names).  YAML defaults
 * (configs/trackers/boosttrack.yaml) = BoostTrack++: max_age 60, min_hits 3, det_thresh .6,
 * iou_threshold .3, use_ecc 1, min_box_area 10, aspect_ratio_thresh 1.6, lambda_iou .5,
 * lambda_mhd .25, lambda_shape .25, use_dlo_boost 1, use_duo_boost 1, dlo_boost_coef .65,
 * s_sim_corr 0, use_rich_s 1, use_sb 1, use_vt 1, with_reid 1. */
typedef struct {
    int32_t n_seq;      /* independent sequences held by this engine */
    int32_t track_cap;  /* track slots per sequence (<= 512) */
    int32_t det_cap;    /* max detections per frame per sequence (<= 512) */
    int32_t emb_dim;    /* with_reid: embedding dimension F (float64 embeddings), else 0 */
    int32_t max_age, min_hits;
    double det_thresh, iou_threshold, min_box_area, aspect_ratio_thresh;
    double lambda_iou, lambda_mhd, lambda_shape, dlo_boost_coef;
    int32_t use_ecc, use_dlo_boost, use_duo_boost, s_sim_corr, use_rich_s, use_sb, use_vt,
        with_reid;
} bx_boost_config;

typedef struct bx_boost bx_boost;

int bx_boost_create(const bx_boost_config *cfg, bx_boost **out);
int bx_boost_destroy(bx_boost *e);
/* Forget all tracks of sequences [seq0, seq0+nseq) (frame and id counters back to 0). */
int bx_boost_reset(bx_boost *e, int seq0, int nseq, void *stream);
/* One frame for sequences [seq0, seq0+nseq).
 *   dets    [sum N][6] float32 (x1,y1,x2,y2,conf,cls) — BaseTracker.setup_decorator's rounding
 *   det_off [nseq+1] int32 prefix offsets
 *   embs    [sum N][emb_dim] float64 (with_reid), else NULL
 *   warps   [nseq][6] float64 2x3 camera-motion affine per sequence (use_ecc), NULL = identity
 *   out     [sum N][8] float64 rows [x1,y1,x2,y2,id,conf,cls,det_ind], sequence k from row
 *           det_off[k], in the reference's track-list order (after filter_outputs)
 *   out_count [nseq] int32 */
int bx_boost_step(bx_boost *e, int seq0, int nseq, const float *dets, const int32_t *det_off,
                  const double *embs, const double *warps, double *out, int32_t *out_count,
                  void *stream);
/* Host-memory path for one sequence (the drop-in update): copies in, launches, copies out,
 * synchronises.  out must hold n rows. */
int bx_boost_update_host(bx_boost *e, int seq, const float *dets, int n, const double *embs,
                         const double *warp, double *out, int *n_out, void *stream);
/* Latched device status (BX_OK, BX_ERR_TRACK_OVERFLOW or BX_ERR_CAPACITY). */
/* per_class=True (boxmot/trackers/basetracker.py:155-201) for one sequence: one update per class
 * id 0..n_classes-1 on that class's detections with the frame counter held, rows stacked in class
 * order (det_ind indexes the class's subset).  BoostTrack keeps its tracks outside the swapped
 * active_tracks, so every class call sees every track.  Arguments as
 * bx_boost_update_host except warps: [n_classes][6] float64, the camera_update warp of each class
 * call (boosttrack.py:243-246 calls cmc.apply per class call), or NULL = no CMC. */
int bx_boost_update_classes_host(bx_boost *e, int seq, const float *dets, int n,
                                 const double *embs, const double *warps, int n_classes,
                                 double *out, int *n_out, void *stream);
/* Op-level BoostTrack filter (device arrays, async on `stream`), the frame kernel's octet code.
 * x [n][8], P [n][8][8] row-major, z [n][4] = convert_bbox_to_z (x, y, h, w/(h+1e-6)).
 *   bx_kf_boost_initiate  KalmanFilter.__init__   boxmot/trackers/boosttrack/kalmanfilter.py:47-73
 *   bx_kf_boost_predict   KalmanFilter.predict    kalmanfilter.py:75-107 (F(PF^T) + Q, constant Q)
 *   bx_kf_boost_update    KalmanFilter.update     kalmanfilter.py:127-157 (cho_factor / cho_solve,
 *                         R = diag(1, 1, 10, 0.01))
 *   bx_kf_boost_mh_dist   BoostTrack.get_mh_dist_matrix  boosttrack.py:356-369: detections
 *                         dets [nd][4] xyxy against the n filters -> out [nd][nt] */
int bx_kf_boost_initiate(int n, const double *z, double *x, double *P, void *stream);
int bx_kf_boost_predict(int n, double *x, double *P, void *stream);
int bx_kf_boost_update(int n, double *x, double *P, const double *z, void *stream);
int bx_kf_boost_mh_dist(int nd, const double *dets, int nt, const double *x, const double *P,
                        double *out, void *stream);
/* Capacity growth (the reference's track list is unbounded: boosttrack.py:221-341 (self.trackers)): copy every
 * sequence's tracker state of `src` into `dst`, a fresh engine with the same configuration and
 * sequences and track_cap / det_cap at least src's (slot ids stay valid).  Synchronous. */
int bx_boost_copy_state(bx_boost *dst, bx_boost *src);
int bx_boost_status(bx_boost *e, int *status);
int bx_boost_counters_host(bx_boost *e, int seq, int *frame_count, int *id_count, int *n_tracks);
/* KalmanBoxTracker.count is class-global in the reference (boosttrack.py:50,53-56, never reset
 * by the constructor); the Python drop-in mirrors it through this. */
int bx_boost_set_id_count(bx_boost *e, int seq, int id_count, void *stream);
/* Track list of a sequence in list order (host, synchronous): ids [cap], means x [cap][8],
 * covariances P [cap][64], embeddings emb [cap][emb_dim] (any may be NULL); *n = tracks. */
int bx_boost_tracks_host(bx_boost *e, int seq, int cap, int32_t *ids, double *x, double *p,
                         double *emb, int *n);
/* Write KalmanBoxTracker.kf.x [n][8] / .kf.covariance [n][64] of live tracks by id (host,
 * synchronous; either may be NULL) — trackers/boosttrack/boosttrack.py:45-121 /
 * kalmanfilter.py:8-157 state attributes.  BX_ERR_INVALID for an unknown id. */
int bx_boost_state_set_host(bx_boost *e, int seq, int n, const int32_t *ids, const double *x,
                            const double *p);
/* Last-frame statistics over sequences [seq0, seq0+nseq) (host, synchronous): sums[7] =
 * {detections, detections kept after the boosts, tracks entering the frame, output rows,
 * embedding-update records, max frame counter, sum of detections x tracks (the ReID
 * contraction's entries)} — bench.py's unit counts. */
int bx_boost_frame_stats_host(bx_boost *e, int seq0, int nseq, int64_t *sums);
/* Timing probe (benchmarks): stage 0 = ReID contraction, 1 = frame kernel, 2 = embedding
 * update; -1 = off.  While on, every step records a HIP event pair around that stage's launch;
 * probe_read synchronises, returns the summed milliseconds and launch count, then clears. */
int bx_boost_probe(bx_boost *e, int stage);
int bx_boost_probe_read(bx_boost *e, double *total_ms, int *count);

#ifdef __cplusplus
}
#endif

#endif /* BXBOOST_H */
