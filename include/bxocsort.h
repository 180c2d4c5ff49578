/*
 * bxocsort.h — C ABI of the OCSort engine in libbxassoc.so (MI355X, gfx950).
 *
 * Boundary: everything OcSort.update(dets, img) computes per frame — the XYSR Kalman predict
 * and update of every track with the observation-centric re-update (ORU) of a track that
 * reappears, the IoU + velocity-direction-consistency cost, the one-to-one fast path and the
 * legacy lapx JV assignment, the optional BYTE round on low-confidence detections, the
 * observation-centric recovery (OCR) round on last observations, track birth and death and the
 * output rows — runs on the GPU, one wave64 workgroup per sequence, behind these entry points.
 *
 * Reference interfaces replaced (file:line in muntherr/boxmot @ /root/reference):
 *   bx_ocsort_create/step/update_host  OcSort.__init__ / OcSort.update
 *                                      boxmot/trackers/ocsort/ocsort.py:195-439
 *     KalmanBoxTracker                 ocsort.py:56-192
 *     KalmanFilterXYSR (ORU)           boxmot/motion/kalman_filters/aabb/xysr_kf.py:48-291
 *     associate (enhanced)             boxmot/utils/association.py:377-536
 *     linear_assignment (legacy lapx)  boxmot/utils/association.py:105-114
 * The fork's OCSort does not run as shipped; the engine follows it with the minimal patches
 * P1-P5 listed in SURVEY.md Appendix A (bit-identical to oracle/bxo_ocsort.c, pinned by the
 * tests/golden/trk_ocsort_*.npz fixtures captured from the patched reference).
 *
 * Conventions as in bxassoc.h: device pointers unless a name ends in _host, asynchronous on
 * `stream`, every function returns a bx_status (bx_last_error explains failures).
 */
#ifndef BXOCSORT_H
#define BXOCSORT_H

#include <stdint.h>

#include "bxassoc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* OcSort constructor parameters (ocsort.py:197-235; YAML defaults in configs/trackers/ocsort.yaml:
 * min_conf .1, det_thresh .6, max_age 30, min_hits 3, asso_threshold .3, delta_t 3, inertia .1,
 * use_byte 0, Q_xy_scaling .01, Q_s_scaling 1e-4).  asso_kind is BaseTracker's asso_func
 * (basetracker.py:140-147; BX_ASSO_* of bxassoc.h, iou by default); centroid normalises by the
 * sequence's frame size, frame_w x frame_h until bx_ocsort_set_frame_size latches another. */
typedef struct {
    int32_t n_seq;      /* independent sequences held by this engine */
    int32_t track_cap;  /* track slots per sequence (<= 512) */
    int32_t det_cap;    /* max detections per frame per sequence (<= 512) */
    double min_conf, det_thresh, asso_threshold, inertia, q_xy_scaling, q_s_scaling;
    int32_t max_age, min_hits, delta_t, use_byte;
    int32_t asso_kind;
    double frame_w, frame_h;
} bx_ocsort_config;

typedef struct bx_ocsort bx_ocsort;

int bx_ocsort_create(const bx_ocsort_config *cfg, bx_ocsort **out);
int bx_ocsort_destroy(bx_ocsort *e);
/* Forget all tracks of sequences [seq0, seq0+nseq) (frame and id counters back to 0). */
int bx_ocsort_reset(bx_ocsort *e, int seq0, int nseq, void *stream);
/* One frame for sequences [seq0, seq0+nseq) — one kernel launch.
 *   dets    [sum N][6] float32 (x1,y1,x2,y2,conf,cls)
 *   det_off [nseq+1] int32 prefix offsets
 *   out     [sum N][8] float64 rows [x1,y1,x2,y2,id,conf,cls,det_ind], sequence k from row
 *           det_off[k], in the reference's (reversed track list) order
 *   out_count [nseq] int32 */
int bx_ocsort_step(bx_ocsort *e, int seq0, int nseq, const float *dets, const int32_t *det_off,
                   double *out, int32_t *out_count, void *stream);
/* Host-memory path for one sequence (the drop-in update): copies in, launches, copies out,
 * synchronises.  out must hold n rows. */
int bx_ocsort_update_host(bx_ocsort *e, int seq, const float *dets, int n, double *out,
                          int *n_out, void *stream);
/* per_class=True (boxmot/trackers/basetracker.py:155-201): class c (0..n_classes-1, the
 * reference's nr_classes = 80) is engine sequence seq0 + c — OCSort's whole state lives in the
 * active list the decorator swaps, so classes are isolated trackers — and the frame is one launch
 * over those sequences.  Output rows are stacked in class order (det_ind indexes the class's
 * subset) with ids renumbered in the reference's class-global birth order: *id_count is the
 * class-global KalmanBoxTracker.count, read and advanced.  out must hold n rows. */
int bx_ocsort_update_classes_host(bx_ocsort *e, int seq0, int n_classes, const float *dets,
                                  int n, int *id_count, double *out, int *n_out, void *stream);
/* Op-level XYSR filter of OCSort's KalmanBoxTracker (device arrays, async on `stream`), the
 * same octet code as the frame kernel.  x [n][7], P [n][7][7] row-major.
 *   bx_kf_xysr_initiate  KalmanBoxTracker.__init__ filter setup   ocsort.py:83-111
 *                        (x[:4] = xyxy2xysr(bbox [n][4]) (P1), P = 10*diag(1,1,1,1,1e3,1e3,1e3))
 *   bx_kf_xysr_predict   KalmanBoxTracker.predict's filter part  ocsort.py:177-180 +
 *                        KalmanFilterXYSR.predict  xysr_kf.py:137-175 (Q[4:6,4:6] *= q_xy,
 *                        Q[-1,-1] *= q_s; the s + ds <= 0 velocity clamp first)
 *   bx_kf_xysr_update    KalmanFilterXYSR.update's filter part xysr_kf.py:256-283 (R = diag(1,1,
 *                        10,10), explicit inv(S), Joseph form; z [n][4]; no history / ORU) */
int bx_kf_xysr_initiate(int n, const double *bbox, double *x, double *P, void *stream);
int bx_kf_xysr_predict(int n, double *x, double *P, double q_xy_scaling, double q_s_scaling,
                       void *stream);
int bx_kf_xysr_update(int n, double *x, double *P, const double *z, void *stream);
/* Latched device status (BX_OK, BX_ERR_TRACK_OVERFLOW or BX_ERR_CAPACITY). */
/* Capacity growth (the reference's track list is unbounded: ocsort.py:246-439 (self.active_tracks / KalmanBoxTracker list)): copy every
 * sequence's tracker state of `src` into `dst`, a fresh engine with the same configuration and
 * sequences and track_cap / det_cap at least src's (slot ids stay valid).  Synchronous. */
int bx_ocsort_copy_state(bx_ocsort *dst, bx_ocsort *src);
int bx_ocsort_status(bx_ocsort *e, int *status);
int bx_ocsort_counters_host(bx_ocsort *e, int seq, int *frame_count, int *id_count,
                            int *n_tracks);
/* KalmanBoxTracker.count is class-global in the reference (ocsort.py:61,115-116,244); the
 * Python drop-in mirrors it through this. */
int bx_ocsort_set_id_count(bx_ocsort *e, int seq, int id_count, void *stream);
/* Track list of a sequence in list order (host, synchronous): ids [cap], Kalman means x
 * [cap][7] and covariances p [cap][49] (any may be NULL); *n = number of tracks.  A sequence
 * driven by bx_ocsort_update_classes_host reports class-global ids (output id - 1). */
/* Frame size (w, h) of a sequence — BaseTracker latches img.shape on the first frame. */
int bx_ocsort_set_frame_size(bx_ocsort *e, int seq, double w, double h, void *stream);
int bx_ocsort_tracks_host(bx_ocsort *e, int seq, int cap, int32_t *ids, double *x, double *p,
                          int *n);
/* Write KalmanBoxTracker.kf.x [n][7] / .kf.P [n][49] of live tracks by id (host, synchronous;
 * either may be NULL) — host code editing `trk.kf.x` / `trk.kf.P` (ocsort.py:56-192,
 * motion/kalman_filters/aabb/xysr_kf.py state attributes).  BX_ERR_INVALID for an unknown id. */
int bx_ocsort_state_set_host(bx_ocsort *e, int seq, int n, const int32_t *ids, const double *x,
                             const double *p);
/* Last-frame statistics over sequences [seq0, seq0+nseq) (host, synchronous): sums[3] =
 * {tracks alive after the frame, output rows, max frame counter} — bench.py's unit counts. */
int bx_ocsort_frame_stats_host(bx_ocsort *e, int seq0, int nseq, int64_t *sums);
/* Timing probe (benchmarks): while on, every step records a HIP event pair around its kernel;
 * probe_read synchronises and returns the summed milliseconds and launch count, then clears. */
int bx_ocsort_probe(bx_ocsort *e, int on);
int bx_ocsort_probe_read(bx_ocsort *e, double *total_ms, int *count);

#ifdef __cplusplus
}
#endif

#endif /* BXOCSORT_H */
