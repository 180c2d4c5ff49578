/*
 * bxo — CPU restatement (fp64, plain C) of the BoxMOT per-frame association path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the oracle the HIP engine (libbxassoc.so) is checked
 * against, and the "port" CPU baseline bench.py times beside it.  Nothing in boxmot_amd/ links,
 * loads or calls it; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
 *
 * Parity pinning: every function here is checked against golden vectors captured from the Python
 * reference (tests/golden/make_golden.py, which imports /root/reference through an import shim)
 * by tests/test_oracle.py.  lapx (the reference's JV dependency, 0.5.11.post1) is absent from the
 * image; bxo_linear_assignment restates its wrapper semantics over a dense Jonker-Volgenant solve
 * of the same (n_r+n_c)^2 extended matrix.
 */
#ifndef BXO_H
#define BXO_H
#ifdef __cplusplus
extern "C" {
#endif

/* Worker threads of the few parallel oracle loops (StrongSort NN rows); 1 = single thread.
 * Results do not depend on it. */
void bxo_set_threads(int n);

enum { BXO_KF_XYAH = 0, BXO_KF_XYWH = 1 };

/* utils/iou.py:50-67  AssociationFunction.iou_batch  (a[na,4], b[nb,4] xyxy → out[na,nb]) */
void bxo_iou_batch(const double *a, int na, const double *b, int nb, double *out);
/* utils/iou.py:79-346  AssociationFunction registry: iou, hmiou, giou, diou, ciou, centroid
 * (centroid normalises by the frame diagonal sqrt(w^2 + h^2)). a[na,4], b[nb,4] -> out[na,nb] */
enum { BXO_ASSO_IOU = 0, BXO_ASSO_HMIOU = 1, BXO_ASSO_GIOU = 2, BXO_ASSO_DIOU = 3,
       BXO_ASSO_CIOU = 4, BXO_ASSO_CENTROID = 5 };
void bxo_asso_batch(int kind, const double *a, int na, const double *b, int nb, double w,
                    double h, double *out);
double bxo_atan(double x);
/* utils/association.py:320-374 compute_aw_max_metric: out[nr,nc] */
void bxo_aw_max_metric(const double *emb, int nr, int nc, double w_assoc, double bottom,
                       double *out);
/* utils/matching.py:488-555  enhanced_fuse_score, in place on cost[nr,nc] */
void bxo_fuse_score(double *cost, int nr, int nc, const double *confs);
/* utils/matching.py:230-316  enhanced_embedding_distance (float32 features, scipy cosine) */
void bxo_embedding_distance(const float *trk, int nt, const float *det, int nd, int f,
                            double *out);
/* numpy float32 np.linalg.norm(x, axis=1): pairwise summation of x*x, float32 sqrt */
float bxo_np_norm_f32(const float *x, int n);

/* motion/kalman_filters/aabb/base_kalman_filter.py:43-194 + xyah_kf.py / xywh_kf.py */
void bxo_kf_initiate(int kind, const double *meas, double *mean, double *cov);
void bxo_kf_multi_predict(int kind, int n, double *mean, double *cov);
void bxo_kf_update(int kind, double *mean, double *cov, const double *z, double conf);
void bxo_kf_gating_distance(int kind, const double *mean, const double *cov, const double *z,
                            int nz, double *out);

/* Dense square JV (Jonker & Volgenant 1987): x[row]→col, y[col]→row.  Returns 0 on success. */
int bxo_lapjv(int n, const double *cost, int *x, int *y);
/* utils/matching.py:30-141  linear_assignment(cost, thresh) with lapx extend_cost+cost_limit
 * semantics.  matches: 2*min(nr,nc) ints (row, col) in row order. */
int bxo_linear_assignment(const double *cost, int nr, int nc, double thresh, int *matches,
                          int *n_matches, int *ua, int *n_ua, int *ub, int *n_ub);

/* ----------------------------------------------------------------------------------------- */
/* Trackers: ByteTrack (trackers/bytetrack/bytetrack.py:119-302) and BoT-SORT                */
/* (trackers/botsort/botsort.py:27-411) per-frame update with the reference's list semantics. */
typedef struct bxo_tracker bxo_tracker;

bxo_tracker *bxo_bytetrack_new(double min_conf, double track_thresh, double match_thresh,
                               int track_buffer, int frame_rate);
bxo_tracker *bxo_botsort_new(double track_high_thresh, double track_low_thresh,
                             double new_track_thresh, int track_buffer, double match_thresh,
                             double proximity_thresh, double appearance_thresh, int frame_rate,
                             int fuse_first_associate, int with_reid);
/* dets[n,6] (x1,y1,x2,y2,conf,cls); embs[n,emb_dim] float32 (emb_is_f64=0) or float64;
 * warp[6] = 2x3 CMC affine (NULL = identity).  Writes out[M,8] and returns M (or <0 on error,
 * -2 when out_cap is too small). */
int bxo_update(bxo_tracker *t, const double *dets, int n, const void *embs, int emb_dim,
               int emb_is_f64, const double *warp, double *out, int out_cap);
int bxo_id_count(const bxo_tracker *t);
int bxo_frame_count(const bxo_tracker *t);
void bxo_free(bxo_tracker *t);
/* per_class mode (basetracker.py:155-201): swap in class `cls`'s active list (the lost list and
 * the id counter stay shared) and hold the frame counter across a frame's class calls */
void bxo_select_class(bxo_tracker *t, int cls);
void bxo_set_frame_count(bxo_tracker *t, int fc);

/* ----------------------------------------------------------------------------------------- */
/* StrongSort NearestNeighborDistanceMetric.distance, cosine (sort/linear_assignment.py:595-618):
 * samples [off[T]][F] (target t owns rows off[t]..off[t+1]), feats [D][F] -> out [T][D] */
int bxo_nn_cosine_distance(const double *samples, const int *off, int T, const double *feats,
                           int D, int F, double *out);
double bxo_np_norm_f64(const double *x, int n);

/* OCSort (trackers/ocsort/ocsort.py:195-439; XYSR KF xysr_kf.py; association.py) with the     */
/* minimal patches P1-P5 of SURVEY.md Appendix A (see bxo_ocsort.c).                          */
typedef struct bxo_ocsort bxo_ocsort;
bxo_ocsort *bxo_ocsort_new(double min_conf, double det_thresh, int max_age, int min_hits,
                           double asso_threshold, int delta_t, double inertia, int use_byte,
                           double q_xy_scaling, double q_s_scaling);
void bxo_ocsort_free(bxo_ocsort *o);
/* asso_func (BXO_ASSO_*) and the frame size its centroid mode normalises by */
void bxo_ocsort_set_asso(bxo_ocsort *o, int kind, double w, double h);
/* one pair of AssociationFunction.<kind>_batch */
double bxo_pair_cost(int kind, const double *a, const double *b, double w, double h);
int bxo_ocsort_id_count(bxo_ocsort *o);
void bxo_ocsort_set_id_count(bxo_ocsort *o, int c); /* KalmanBoxTracker.count is class-global */
/* track list in list order: ids [cap], XYSR means x [cap][7], covariances P [cap][49] */
int bxo_ocsort_tracks(bxo_ocsort *o, int cap, int *ids, double *x, double *P);
/* dets[n,6] float64 (float32-rounded); out[M,8]; returns M or -2 if out_cap is too small */
int bxo_ocsort_update(bxo_ocsort *o, const double *dets, int n, double *out, int out_cap);
double bxo_acos(double x);
/* op-level XYSR filter of KalmanBoxTracker (mirrors bx_kf_xysr_*): x [n][7], P [n][49] */
void bxo_kf_xysr_initiate(int n, const double *bbox, double *x, double *P);
void bxo_kf_xysr_predict(int n, double *x, double *P, double q_xy, double q_s);
void bxo_kf_xysr_update(int n, double *x, double *P, const double *z);

/* BoostTrack / BoostTrack++ (trackers/boosttrack/boosttrack.py:123-456, assoc.py,            */
/* kalmanfilter.py), as shipped (see bxo_boost.c for the fixed orders).                        */
typedef struct {
    int max_age, min_hits;
    double det_thresh, iou_threshold, min_box_area, aspect_ratio_thresh;
    double lambda_iou, lambda_mhd, lambda_shape, dlo_boost_coef;
    int use_ecc, use_dlo_boost, use_duo_boost, s_sim_corr, use_rich_s, use_sb, use_vt, with_reid;
} bxo_boost_params;
typedef struct bxo_boost bxo_boost;
bxo_boost *bxo_boost_new(const bxo_boost_params *p);
void bxo_boost_free(bxo_boost *b);
int bxo_boost_id_count(const bxo_boost *b);
void bxo_boost_set_id_count(bxo_boost *b, int c);
void bxo_boost_set_frame_count(bxo_boost *b, int fc); /* per_class: held across class calls */
/* track list in list order: ids [cap], means x [cap][8], covariances P [cap][64] */
int bxo_boost_tracks(const bxo_boost *b, int cap, int *ids, double *x, double *P);
/* dets[n,6] float64 (float32-rounded); embs [n][emb_dim] float64 or NULL; warp[6] 2x3 CMC
 * affine (NULL = identity).  out[M,8]; returns M, -2 if out_cap is too small. */
int bxo_boost_update(bxo_boost *b, const double *dets, int n, const double *embs, int emb_dim,
                     const double *warp, double *out, int out_cap);
double bxo_exp(double x);
/* op-level BoostTrack filter (mirrors bx_kf_boost_*): x [n][8], P [n][64], z [n][4] */
void bxo_kf_boost_initiate(int n, const double *z, double *x, double *P);
void bxo_kf_boost_predict(int n, double *x, double *P);
void bxo_kf_boost_update(int n, double *x, double *P, const double *z);
void bxo_kf_boost_mh_dist(int nd, const double *dets, int nt, const double *x, const double *P,
                          double *out);
double bxo_pow15(double x);

/* StrongSort, the fork's "enhanced" tracker (trackers/strongsort/strongsort.py:17-232, sort/...)
 * with P6, handle_occlusions=False and the born-Confirmed switch (see bxo_strongsort.c). */
typedef struct {
    double min_conf, max_cos_dist, max_iou_dist;
    int max_age, n_init, nn_budget;
    double mc_lambda, ema_alpha, conf_thresh_high, conf_thresh_low, id_preservation_weight;
    int crowd_detection, born_confirmed;
} bxo_ss_params;
typedef struct bxo_ss bxo_ss;
bxo_ss *bxo_ss_new(const bxo_ss_params *p);
void bxo_ss_free(bxo_ss *s);
int bxo_ss_next_id(const bxo_ss *s);
/* handle_occlusions=True: the OcclusionAwareTracker post-process after every update (then
 * bxo_ss_update returns -5 where the reference raises TypeError on mutual occlusion, D7) */
void bxo_ss_set_occlusion(bxo_ss *s, int on, double threshold);
/* CPython set iteration order of small positive ints added in order (returns the count) */
int bxo_pyset_order(const long *adds, int nadd, long *out);
/* host edits of the Kalman state by track id (mirrors of the engines' bx_*_state_set_host);
 * each returns the number of ids found */
int bxo_state_set(bxo_tracker *T, int n, const int *ids, const double *mean, const double *cov);
int bxo_ocsort_state_set(bxo_ocsort *o, int n, const int *ids, const double *x, const double *P);
int bxo_boost_state_set(bxo_boost *b, int n, const int *ids, const double *x, const double *P);
int bxo_ss_state_set(bxo_ss *s, int n, const int *ids, const double *mean, const double *cov);
/* ByteTrack / BoT-SORT: tracked then lost list — ids, states, mean [8], covariance [8x8] */
int bxo_tracks(const bxo_tracker *T, int cap, int *ids, int *state, double *mean, double *cov);
int bxo_ss_tracks(const bxo_ss *s, int cap, int *ids, int *state, double *mean, double *cov);
/* dets[n,6] float64; embs [n][F] float64 (required when a detection passes min_conf); warp[6]
 * 2x3 CMC affine (NULL = identity).  out [M][10] (x1,y1,x2,y2,id,conf,cls,det_ind,quality,
 * occlusion=0); returns M, -2 if out_cap is too small, -4 without embeddings. */
int bxo_ss_update(bxo_ss *s, const double *dets, int n, const double *embs, int F,
                  const double *warp, double *out, int out_cap);
/* scipy.optimize.linear_sum_assignment restated: pairs (rows[k], cols[k]) sorted by row;
 * returns the count (-1 if infeasible). */
int bxo_lsap(const double *cost, int nr, int nc, int *rows, int *cols);

#ifdef __cplusplus
}
#endif
#endif
