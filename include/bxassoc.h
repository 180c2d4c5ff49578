/*
 * bxassoc.h — C ABI of libbxassoc.so, the MI355X-native per-frame association engine for
 * BoxMOT trackers (ByteTrack, BoT-SORT).
 *
 * Boundary: everything the reference computes inside `tracker.update(dets, img, embs)` for these
 * trackers — Kalman predict/update over all live tracks, the IoU / score-fusion / re-ID cosine
 * cost matrices, the Jonker–Volgenant-equivalent linear assignment with lapx `cost_limit`
 * semantics, and the track-list state machine — runs on the GPU behind these entry points.
 * Plain pointers and sizes only; no torch types.  Every function returns a bx_status (0 = ok).
 *
 * Reference interfaces replaced (file:line in muntherr/boxmot @ /root/reference):
 *   bx_engine_*            ByteTrack.update          boxmot/trackers/bytetrack/bytetrack.py:158-302
 *                          BotSort.update            boxmot/trackers/botsort/botsort.py:94-166
 *                          (+ per-frame glue         botsort.py:168-411, botsort_utils.py:1-81)
 *   bx_iou_batch           AssociationFunction.iou_batch   boxmot/utils/iou.py:50-67
 *   bx_aw_max_metric       compute_aw_max_metric            boxmot/utils/association.py:320-374
 *   bx_pairwise_cost       AssociationFunction.{iou,hmiou,giou,diou,ciou,centroid}_batch
 *                          boxmot/utils/iou.py:50-307, registry :320-346
 *   bx_fuse_score          matching.enhanced_fuse_score    boxmot/utils/matching.py:488-555
 *   bx_embedding_distance  matching.enhanced_embedding_distance  boxmot/utils/matching.py:230-316
 *   bx_kf_*                BaseKalmanFilter + XYAH/XYWH noise models
 *                          boxmot/motion/kalman_filters/aabb/base_kalman_filter.py:24-194,
 *                          xyah_kf.py:8-79, xywh_kf.py:8-66
 *   bx_nn_cosine_distance  StrongSort NearestNeighborDistanceMetric.distance (cosine)
 *                          boxmot/trackers/strongsort/sort/linear_assignment.py:468-618
 *   bx_linear_assignment   matching.enhanced_linear_assignment (lapx.lapjv extend_cost=True,
 *                          cost_limit=thresh)        boxmot/utils/matching.py:30-141
 *   bx_lapjv               lapx.lapjv itself (square / extend_cost / cost_limit), lapx's own
 *                          algorithm and tie order: association.linear_assignment
 *                          boxmot/utils/association.py:105-114, boosttrack/assoc.py:106-114,
 *                          matching.py:54
 *
 * Memory: unless a name ends in _host, pointer arguments are DEVICE pointers and the call is
 * asynchronous on `stream` (a hipStream_t; NULL = the default stream).  The engine owns its
 * device arena; no caller pointer is retained past a call.
 */
#ifndef BXASSOC_H
#define BXASSOC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    BX_OK = 0,
    BX_ERR_INVALID = 1,        /* bad argument (null handle, negative size, unknown kind) */
    BX_ERR_CAPACITY = 2,       /* detections per frame exceed det_cap */
    BX_ERR_TRACK_OVERFLOW = 3, /* a sequence ran out of track slots (raise track_cap) */
    BX_ERR_HIP = 4,            /* a HIP runtime call failed (see bx_last_error) */
    BX_ERR_NO_DEVICE = 5,      /* no HIP device visible */
    BX_ERR_SHAPE = 6           /* embedding count/dimension does not match the detections */
} bx_status;

typedef enum { BX_BYTETRACK = 0, BX_BOTSORT = 1 } bx_tracker_kind;

/* Tracker parameters (names and meaning as in the reference constructors / YAML defaults). */
typedef struct {
    int32_t kind;         /* bx_tracker_kind */
    int32_t n_seq;        /* independent sequences (video streams) held by this engine */
    int32_t track_cap;    /* track slots per sequence (active + lost tracks alive at once) */
    int32_t det_cap;      /* max detections per frame per sequence */
    int32_t emb_dim;      /* BoT-SORT with_reid: embedding dimension F (0 otherwise) */
    int32_t emb_f64;      /* 1: embeddings are float64 (numpy default), 0: float32 */
    /* ByteTrack (bytetrack.py:132-156) */
    double min_conf, track_thresh, match_thresh;
    int32_t track_buffer, frame_rate;
    /* BoT-SORT (botsort.py:49-92); match_thresh/track_buffer/frame_rate shared */
    double track_high_thresh, track_low_thresh, new_track_thresh;
    double proximity_thresh, appearance_thresh;
    int32_t fuse_first_associate, with_reid;
} bx_config;

typedef struct bx_engine bx_engine;

const char *bx_last_error(void);
int bx_device_count(int *n);

int bx_engine_create(const bx_config *cfg, bx_engine **out);
int bx_engine_destroy(bx_engine *e);
/* Forget all tracks of sequences [seq0, seq0+nseq) (frame and id counters back to 0). */
int bx_engine_reset(bx_engine *e, int seq0, int nseq, void *stream);

/* One frame for sequences [seq0, seq0+nseq): a short pipeline of kernels enqueued on `stream`
 * (per-detection features, Kalman predict, gating + re-ID distances, the per-sequence
 * association, Kalman/feature updates, duplicate removal + outputs).
 *   dets    [sum N][6] float32 (x1,y1,x2,y2,conf,cls) — the reference rounds dets to float32
 *           in BaseTracker.setup_decorator (basetracker.py:122-128)
 *   det_off [nseq+1] int32 prefix offsets: sequence k owns rows det_off[k]..det_off[k+1]
 *   embs    [sum N][emb_dim] float32|float64 (BoT-SORT with_reid), else NULL
 *   warps   [nseq][6] float64 2x3 camera-motion affine per sequence (BoT-SORT), NULL = identity
 *   out     [sum N][8] float64 rows [x1,y1,x2,y2,id,conf,cls,det_ind] (sequence k writes from
 *           row det_off[k]; a frame never outputs more tracks than it has detections)
 *   out_count [nseq] int32 rows written per sequence
 * Errors detected on the device (slot overflow) are latched: bx_engine_status reads them. */
int bx_engine_step(bx_engine *e, int seq0, int nseq, const float *dets, const int32_t *det_off,
                   const void *embs, const double *warps, double *out, int32_t *out_count,
                   void *stream);

/* Overlap mode (default off; bench.py turns it on): bx_engine_step
 * returns with the BoT-SORT feature EMA (K5) of that frame still running on the engine's side
 * stream instead of joining it onto `stream`.  The next bx_engine_step orders its own K1 after
 * it and its cosine pass (the first reader of smooth_feat) waits for it; every other bx_engine_*
 * call synchronises it first.  The caller must keep that step's dets / det_off / embs unmodified
 * until the next bx_engine_step is enqueued (or any other bx_engine_* call returns);
 * hipDeviceSynchronize covers it.  Saves the join and lets the next frame's K1 start as soon as
 * K5 ends instead of after the caller's stream drains. */
int bx_engine_set_overlap(bx_engine *e, int on);
/* Early-features mode (default off; BoT-SORT with ReID): the caller guarantees that the inputs
 * (dets, det_off, embs) of every bx_engine_step are complete in device memory when the step is
 * CALLED (not merely enqueued before it on `stream`) — e.g. produced before a host
 * synchronisation, as bench.py's resident frames are.  The detection-feature kernel (K1) of a
 * full launch (seq0 0, all sequences) then runs on a stream of its own that waits only for the
 * feature EMA (K5) two launches back (the last reader of the norms half it writes), so it starts
 * beside the previous frame's tail instead of after it.  Results are unchanged.  Chunked
 * launches keep the normal order.  Synchronises the engine's streams. */
int bx_engine_set_early_features(bx_engine *e, int on);
/* Overlap mode: make `stream` wait (stream-ordered, no host sync) until the last step's inputs
 * are no longer read — call it before refilling a reused dets / det_off / embs buffer on
 * `stream`.  A no-op when nothing is pending. */
int bx_engine_inputs_released(bx_engine *e, void *stream);

/* Host-memory convenience for one sequence (the drop-in `update` path): copies in, launches,
 * copies out and synchronises.  dets [n][6] float32; embs [n][emb_dim] or NULL; warp [6] or
 * NULL; out must hold n rows; *n_out receives the row count. */
int bx_engine_update_host(bx_engine *e, int seq, const float *dets, int n, const void *embs,
                          const double *warp, double *out, int *n_out, void *stream);

/* per_class=True (BaseTracker.per_class_decorator, boxmot/trackers/basetracker.py:155-201) for
 * one sequence: one update per class id 0..n_classes-1 (nr_classes = 80 in the reference) on the
 * detections whose float32 class equals it (det_ind then indexes that subset, as in the
 * reference), each with the class's own active list while the lost list and the id counter stay
 * shared, and the frame counter held across the frame's class calls; rows stacked in class
 * order.  Arguments as bx_engine_update_host except warps: [n_classes][6] float64, the warp of
 * each class call (the reference calls cmc.apply once per class call, botsort.py:218, so a
 * stateful CMC such as ECC returns the inter-frame warp to class 0 only), or NULL = identity;
 * n_classes must stay the same for an engine. */
int bx_engine_update_classes_host(bx_engine *e, int seq, const float *dets, int n,
                                  const void *embs, const double *warps, int n_classes,
                                  double *out, int *n_out, void *stream);

/* Stage timing probe (benchmarks): while enabled, bx_engine_step records a HIP event pair
 * around every launch of pipeline stage `stage` on its stream; bx_engine_probe_read
 * synchronises, returns the summed milliseconds and the number of timed launches, and clears
 * them.  stage < 0 disables the probe.  Costs two event records per step. */
typedef enum {
    BX_STAGE_DET_FEATURES = 0, BX_STAGE_PREDICT = 1, BX_STAGE_GATE = 2, BX_STAGE_COSINE = 3,
    BX_STAGE_ASSOC = 4, BX_STAGE_UPDATE = 5, BX_STAGE_COV_PREDICT = 6, BX_STAGE_FEATURES = 7,
    BX_STAGE_FINISH = 8, BX_STAGE_COUNT = 9
} bx_stage;
int bx_engine_probe(bx_engine *e, int stage);
/* Last-frame statistics summed over sequences [seq0, seq0+nseq) (host, synchronous):
 * sums[7] = {detections, high-confidence detections, active tracks, lost tracks, update records,
 * gated (track, det) pairs, frame counter} — the unit counts bench.py prices bytes with. */
int bx_engine_frame_stats_host(bx_engine *e, int seq0, int nseq, int64_t *sums);
int bx_engine_probe_read(bx_engine *e, double *total_ms, int *count);
/* Associations of sequences [seq0, seq0+nseq) whose optimum was tied and that were therefore
 * re-solved by lapx's own lapjv (see bx_linear_assignment), summed since creation / reset. */
int bx_engine_lap_ties_host(bx_engine *e, int seq0, int nseq, int64_t *total);
/* Connected components the sparse LAP solver (matching.py:30-108 restated) solved
 * with its per-lane SSP (small components past the register path, sums[0]), with its
 * wave-parallel SSP (components of more than 3 rows: sums[1]) and, of those, on the association
 * kernel's helper waves 1..3 (sums[2]), over sequences [seq0, seq0+nseq), summed since creation
 * / reset.  sums has 3 entries.  Diagnostic: the parity tests use it to show a workload
 * exercised every solver path. */
int bx_engine_lap_components_host(bx_engine *e, int seq0, int nseq, int64_t *sums);
/* Which build of the association kernel runs (BoT-SORT / ByteTrack engines): -1 (default) the
 * host picks per launch from the device's helper-wave cue; 0 always the wave-0-only build; 1
 * always the helper-wave build.  Both builds give identical results; tests force each to prove
 * it.  Settles overlap mode first. */
int bx_engine_force_assoc_build(bx_engine *e, int mode);
/* Turn the component counting of bx_engine_lap_components_host on (off by default: it costs the
 * association kernel reductions and atomics per LAP).  Diagnostic; settles overlap mode first. */
int bx_engine_set_lap_stats(bx_engine *e, int on);

/* Capacity growth (the reference's track lists are unbounded: bytetrack.py:272-346): copy every
 * sequence's tracker state of `src` into `dst`, a fresh engine with the same kind, sequences and
 * features and track_cap / det_cap at least src's (slot ids stay valid; per_class parked lists
 * included).  Synchronous.  The drop-ins grow this way before a frame could overflow. */
int bx_engine_copy_state(bx_engine *dst, bx_engine *src);
/* Track slots of sequence `seq` in use (live tracks), host, synchronous. */
int bx_engine_slots_used_host(bx_engine *e, int seq, int *used);
/* Latched device-side status of the whole engine (BX_OK or BX_ERR_TRACK_OVERFLOW). */
int bx_engine_status(bx_engine *e, int *status);
/* Per-sequence counters (host copies): frame_count, id_count, live tracks. */
int bx_engine_counters_host(bx_engine *e, int seq, int *frame_count, int *id_count,
                            int *n_active, int *n_lost);
/* Set the id counter of a sequence (ByteTrack's BaseTrack._count is process-global in the
 * reference, bytetrack/basetrack.py:16,37-40; the Python drop-in mirrors it through this). */
int bx_engine_set_id_count(bx_engine *e, int seq, int id_count, void *stream);
/* Snapshot the live tracks of a sequence (host): slot-ordered active then lost lists.
 * ids/state/is_activated/frame_id/start_frame [n] int32, mean [n][8], cov [n][64] float64.
 * cap = capacity of each array in tracks; *n receives n_active + n_lost. */
int bx_engine_tracks_host(bx_engine *e, int seq, int cap, int32_t *ids, int32_t *state,
                          int32_t *is_activated, int32_t *frame_id, int32_t *start_frame,
                          double *mean, double *cov, int *n_active, int *n_lost);
/* per_class mode: the active list of every class (basetracker.py:52-60,181-192
 * `per_class_active_tracks`), concatenated in class order; cls_off [n_classes+1] receives the
 * list offsets, the other arrays as in bx_engine_tracks_host (cap rows each).  All lists are empty
 * before the first bx_engine_update_classes_host of the sequence. */
int bx_engine_class_tracks_host(bx_engine *e, int seq, int n_classes, int cap, int32_t *cls_off,
                                int32_t *ids, int32_t *state, int32_t *is_activated,
                                int32_t *frame_id, int32_t *start_frame, double *mean,
                                double *cov);
/* Write the Kalman state of live tracks (host, synchronous), addressed by track id: mean [n][8],
 * cov [n][64] (either may be NULL).  What host code does to `STrack.mean` / `.covariance` in
 * the reference (the objects are plain attributes: bytetrack.py:40-53 / botsort_track.py:75-104
 * read them back on the next predict); the occlusion handler's edit is the model
 * (utils/occlusion_handler.py:380-398).  BX_ERR_INVALID if an id is not live. */
int bx_engine_state_set_host(bx_engine *e, int seq, int n, const int32_t *ids, const double *mean,
                             const double *cov);

/* ---------------------------- op-level kernels (device pointers) ---------------------------- */
int bx_iou_batch(const double *a, int na, const double *b, int nb, double *out, void *stream);
/* AssociationFunction registry (utils/iou.py:79-346, _get_asso_func :320-346): out[i][j] =
 * <kind>_batch(a, b)[i][j] for rows of stride lda / ldb (>= 4, xyxy first).  centroid
 * normalises by the frame diagonal sqrt(w^2 + h^2) (AssociationFunction(w, h), :36-49); the
 * other kinds ignore w, h.  giou's assert (enclosing box of positive size, :163) is the
 * caller's; the OBB modes (iou_obb, centroid_obb) are not provided. */
enum { BX_ASSO_IOU = 0, BX_ASSO_HMIOU = 1, BX_ASSO_GIOU = 2, BX_ASSO_DIOU = 3, BX_ASSO_CIOU = 4,
       BX_ASSO_CENTROID = 5 };
int bx_pairwise_cost(int kind, const double *a, int na, int lda, const double *b, int nb, int ldb,
                     double w, double h, double *out, void *stream);
int bx_fuse_score(double *cost, int nr, int nc, const double *confs, void *stream);
/* compute_aw_max_metric (utils/association.py:320-374, DeepOCSort's adaptive appearance weight):
 * out = ((w_assoc * row_weight) * col_weight) * emb, weights from the two largest positive entries
 * of each row / column; nr, nc <= 4096. */
int bx_aw_max_metric(const double *emb, int nr, int nc, double w_assoc, double bottom, double *out,
                     void *stream);
/* float32 features, numpy float32 norms, scipy cdist-cosine summation order, clipped at 0 */
int bx_embedding_distance(const float *trk, int nt, const float *det, int nd, int f, double *out,
                          void *stream);
/* kind: 0 = XYAH (ByteTrack), 1 = XYWH (BoT-SORT); arrays of n tracks, row-major [n][8], [n][64] */
int bx_kf_initiate(int kind, int n, const double *meas, double *mean, double *cov, void *stream);
int bx_kf_multi_predict(int kind, int n, double *mean, double *cov, void *stream);
int bx_kf_update(int kind, int n, double *mean, double *cov, const double *z, const double *conf,
                 void *stream);
int bx_kf_gating_distance(int kind, int n, const double *mean, const double *cov,
                          const double *z, int nz, double *out, void *stream);
/* StrongSort appearance metric (NearestNeighborDistanceMetric.distance with the cosine metric,
 * trackers/strongsort/sort/linear_assignment.py:468-497,595-618): samples [G][F] float64 is every
 * target's gallery packed by target (target t owns rows off[t]..off[t+1], off [T+1] int32 on the
 * device, off[T] == G); feats [D][F] float64.  out [T][D] = min over the target's samples of
 * 1 - clip(ŝ·d̂, -1, 1) with x̂ = x / (‖x‖ + 1e-8) (numpy's pairwise norm), 1e5 for a target
 * without samples.  fp64 matrix cores (k-ordered fma chain, bitwise = the oracle).
 * flags: BX_NN_SAMPLES_NORMALIZED = the samples are already x̂ (a gallery kept normalised). */
#define BX_NN_SAMPLES_NORMALIZED 1
int bx_nn_cosine_distance(const double *samples, int G, const int32_t *off, int T,
                          const double *feats, int D, int F, int flags, double *out, void *stream);
/* matching.enhanced_linear_assignment (matching.py:30-61: lap.lapjv(cost, extend_cost=True,
 * cost_limit=thresh), matches = rows with x >= 0 and cost <= thresh) on a dense [nr][nc] cost:
 * x [nr] = matched column, -1 = unmatched (in unmatched_a); y [nc] likewise.  Solved sparse (exact
 * shortest augmenting paths over the admissible pairs); when the optimal pair set is not unique
 * the problem is re-solved by lapx's own lapjv on the (nr+nc)^2 extension so ties resolve as
 * lapx's do.  -3 marks a row/column lapx assigned to a real partner above thresh (possible only
 * within rounding of a tie at thresh): the reference neither matches it nor lists it unmatched.
 * nr, nc <= 8192.  bx_linear_assignment_ex also writes tied[0] (device) = 1 when the lapx
 * re-solve ran, else 0. */
int bx_linear_assignment(const double *cost, int nr, int nc, double thresh, int32_t *x,
                         int32_t *y, void *stream);
int bx_linear_assignment_ex(const double *cost, int nr, int nc, double thresh, int32_t *x,
                            int32_t *y, int32_t *tied, void *stream);
/* lapx 0.5.11 lapjv(cost, extend_cost, cost_limit) on a dense [nr][nc] float64 cost, solved by
 * lapx's algorithm (_ccrrt_dense, two _carr_dense passes, _ca_dense) on one wave, so tied
 * problems return lapx's optimum.  cost_limit = +inf for none (then nr == nc unless
 * extend_cost).  x [nr] = column or -1, y [nc] = row or -1 (lapx's post-processing when
 * extended).  The (possibly extended) size must be <= 32768 (state in LDS up to ~4k, else in
 * global memory).  BX_ERR_INVALID carries lapx's
 * ValueError text for a non-square cost without extend_cost. */
int bx_lapjv(const double *cost, int nr, int nc, int extend_cost, double cost_limit, int32_t *x,
             int32_t *y, void *stream);
/* Test entry point of the legacy association.linear_assignment (association.py:109; OCSort /
 * BoostTrack) for a dense [nr][nc] float64 cost, nr, nc <= 64: lapx's lapjv order (the engines'
 * legacy_lap) into pairs_jv and the shortest-augmenting-path solve with its uniqueness
 * certificate (legacy_lap_ssp, which runs lapjv itself on a tie) into pairs_ssp, both
 * [min(nr,nc)][2] (row, col) in row order.  info[3] (device) = {pairs_jv count, pairs_ssp count,
 * 1 if legacy_lap_ssp fell back to lapjv}.  The two must always agree. */
int bx_legacy_lap_pair(const double *cost, int nr, int nc, int32_t *pairs_jv, int32_t *pairs_ssp,
                       int32_t *info, void *stream);

#ifdef __cplusplus
}
#endif
#endif
