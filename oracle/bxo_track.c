/*
 * bxo_track.c — oracle per-frame drivers for ByteTrack and BoT-SORT with the reference's
 * Python list semantics restated over arrays of track pointers.  TEST INFRASTRUCTURE ONLY.
 *
 *   ByteTrack.update           trackers/bytetrack/bytetrack.py:158-302
 *   joint/sub/remove_duplicate trackers/bytetrack/bytetrack.py:308-346, botsort/botsort_utils.py
 *   STrack (ByteTrack)         trackers/bytetrack/bytetrack.py:14-116
 *   BotSort.update             trackers/botsort/botsort.py:94-411
 *   STrack (BoT-SORT)          trackers/botsort/botsort_track.py:10-159
 *
 * Track objects live until they have left both the active and the lost list: from then on the
 * reference can never reach them again (the only re-entry is through strack_pool = tracked ∪
 * lost), so freeing them is unobservable.  Membership of self.removed_stracks is kept as a flag
 * because sub_stracks only tests ids.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "bxo.h"
#include "bxo_internal.h"

enum { KIND_BYTE = 0, KIND_BOT = 1 };
enum { ST_NEW = 0, ST_TRACKED = 1, ST_LOST = 2, ST_REMOVED = 3 };
#define MAX_CLS_HIST 64

typedef struct Trk {
    double xywh[4], tlwh[4], xyah[4];
    double conf, cls, det_ind;
    double mean[8], cov[64];
    int has_mean;
    int id, state, is_activated, frame_id, start_frame, tracklet_len;
    int in_removed; /* appended to self.removed_stracks at some earlier frame */
    unsigned stamp; /* scratch membership mark */
    double *smooth;  /* smooth_feat (NULL = None) */
    double *curr;    /* det: curr_feat; aliases smooth right after construction */
    double cls_hist[MAX_CLS_HIST][2];
    int n_cls;
} Trk;

typedef struct {
    Trk **v;
    int n, cap;
} List;

static void lpush(List *l, Trk *t) {
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 16;
        l->v = (Trk **)realloc(l->v, sizeof(Trk *) * l->cap);
    }
    l->v[l->n++] = t;
}
static void lfree(List *l) {
    free(l->v);
    l->v = NULL;
    l->n = l->cap = 0;
}

struct bxo_tracker {
    int kind;
    double low, high, new_thresh, match_thresh, proximity, appearance;
    int fuse_first, with_reid, max_time_lost;
    int frame_count, id_count;
    unsigned stamp;
    List active, lost;
    int emb_dim, f64;
    /* per_class mode: the other classes' active lists, parked while `cur_cls` runs */
    List *parked;
    int nparked, cur_cls;
};

/* ---- feature helpers: values held in double, rounded to float32 after every op in f32 mode - */
static inline double rnd(const bxo_tracker *T, double x) { return T->f64 ? x : (double)(float)x; }

/* np.linalg.norm(1-D) = sqrt(x.dot(x)) — a BLAS dot whose summation order numpy does not pin.
 * The engine fixes it as the "wave order": 64 lane-strided sequential fp64 partial sums
 * (lane l: x[l], x[l+64], ...) combined by an xor butterfly (d = 32..1); restated here. */
static double vnorm(const bxo_tracker *T, const double *x) {
    double s[64], t[64];
    for (int l = 0; l < 64; l++) {
        s[l] = 0.0;
        for (int k = l; k < T->emb_dim; k += 64) s[l] += x[k] * x[k];
    }
    for (int d = 32; d >= 1; d >>= 1) {
        for (int l = 0; l < 64; l++) t[l] = s[l] + s[l ^ d];
        memcpy(s, t, sizeof s);
    }
    return T->f64 ? sqrt(s[0]) : (double)sqrtf((float)s[0]);
}

static void vdiv_inplace(const bxo_tracker *T, double *x, double n) {
    for (int k = 0; k < T->emb_dim; k++) x[k] = rnd(T, x[k] / n);
}

/* botsort_track.py:40-49 STrack.update_features (on the track `t`, source buffer `feat`). */
static void update_features(bxo_tracker *T, Trk *t, double *feat) {
    vdiv_inplace(T, feat, vnorm(T, feat)); /* feat /= norm(feat) (in place on the det buffer) */
    if (t->smooth == feat) {
        /* detection construction: smooth_feat = feat (same object as curr_feat) */
    } else if (t->smooth == NULL) {
        /* a track without features adopting a detection's: the reference aliases the det's
         * buffer; the det is never read again, so an owned copy is indistinguishable. */
        t->smooth = (double *)malloc(sizeof(double) * T->emb_dim);
        memcpy(t->smooth, feat, sizeof(double) * T->emb_dim);
    } else {
        const double a = rnd(T, 0.9), b = rnd(T, 1.0 - 0.9);
        for (int k = 0; k < T->emb_dim; k++)
            t->smooth[k] = rnd(T, rnd(T, a * t->smooth[k]) + rnd(T, b * feat[k]));
    }
    vdiv_inplace(T, t->smooth, vnorm(T, t->smooth));
}

/* botsort_track.py:51-64 update_cls */
static void update_cls(Trk *t, double cls, double conf) {
    double max_freq = 0.0;
    int found = 0;
    for (int k = 0; k < t->n_cls; k++) {
        if (cls == t->cls_hist[k][0]) {
            t->cls_hist[k][1] += conf;
            found = 1;
        }
        if (t->cls_hist[k][1] > max_freq) {
            max_freq = t->cls_hist[k][1];
            t->cls = t->cls_hist[k][0];
        }
    }
    if (!found && t->n_cls < MAX_CLS_HIST) {
        t->cls_hist[t->n_cls][0] = cls;
        t->cls_hist[t->n_cls][1] = conf;
        t->n_cls++;
        t->cls = cls;
    }
}

static Trk *new_det(bxo_tracker *T, const double *det7, const double *feat_src) {
    Trk *t = (Trk *)calloc(1, sizeof(Trk));
    bxo_xyxy2xywh(det7, t->xywh);
    if (T->kind == KIND_BYTE) {
        bxo_xywh2tlwh(t->xywh, t->tlwh);
        bxo_tlwh2xyah(t->tlwh, t->xyah);
    }
    t->conf = det7[4];
    t->cls = det7[5];
    t->det_ind = det7[6];
    if (T->kind == KIND_BOT) {
        update_cls(t, t->cls, t->conf);
        if (feat_src) {
            double *f = (double *)malloc(sizeof(double) * T->emb_dim);
            memcpy(f, feat_src, sizeof(double) * T->emb_dim);
            t->curr = f;
            update_features(T, t, f); /* curr_feat and smooth_feat alias the same buffer */
        }
    }
    return t;
}

static void free_trk(Trk *t) {
    if (t->curr && t->curr != t->smooth) free(t->curr);
    free(t->smooth);
    free(t);
}

/* STrack.xyxy (bytetrack.py:105-116, botsort_track.py:155-159) */
static void trk_xyxy(const bxo_tracker *T, const Trk *t, double *out) {
    double r[4];
    if (!t->has_mean) {
        memcpy(r, t->xywh, sizeof r);
    } else {
        memcpy(r, t->mean, sizeof r);
        if (T->kind == KIND_BYTE) r[2] *= r[3];
    }
    bxo_xywh2xyxy(r, out);
}

static double *iou_distance(const bxo_tracker *T, const List *a, const List *b) {
    double *c = (double *)malloc(sizeof(double) * (size_t)(a->n ? a->n : 1) * (b->n ? b->n : 1));
    double *bb = (double *)malloc(sizeof(double) * 4 * (b->n ? b->n : 1));
    for (int j = 0; j < b->n; j++) trk_xyxy(T, b->v[j], bb + 4 * j);
    for (int i = 0; i < a->n; i++) {
        double ab[4];
        trk_xyxy(T, a->v[i], ab);
        for (int j = 0; j < b->n; j++) c[(size_t)i * b->n + j] = 1 - bxo_iou_pair(ab, bb + 4 * j);
    }
    free(bb);
    return c;
}

static void fuse(double *c, const List *a, const List *b) {
    for (int i = 0; i < a->n; i++)
        for (int j = 0; j < b->n; j++)
            c[(size_t)i * b->n + j] = bxo_fuse_one(c[(size_t)i * b->n + j], b->v[j]->conf);
}

/* BoT-SORT appearance fusion (botsort.py:228-232, 318-324) applied to `c` (IoU distance, maybe
 * score-fused) with `iou` (raw IoU distance) providing the proximity mask. */
static void fuse_reid(const bxo_tracker *T, double *c, const double *iou, const List *a,
                      const List *b) {
    int F = T->emb_dim;
    if (a->n == 0 || b->n == 0) return;
    float *A = (float *)malloc(sizeof(float) * (size_t)a->n * F);
    float *B = (float *)malloc(sizeof(float) * (size_t)b->n * F);
    for (int i = 0; i < a->n; i++)
        for (int k = 0; k < F; k++)
            A[(size_t)i * F + k] = a->v[i]->smooth ? (float)a->v[i]->smooth[k] : 0.0f;
    for (int j = 0; j < b->n; j++)
        for (int k = 0; k < F; k++)
            B[(size_t)j * F + k] = b->v[j]->curr ? (float)b->v[j]->curr[k] : 0.0f;
    double *e = (double *)malloc(sizeof(double) * (size_t)a->n * b->n);
    bxo_embedding_distance(A, a->n, B, b->n, F, e);
    for (size_t k = 0; k < (size_t)a->n * b->n; k++) {
        double ed = e[k] / 2.0;
        if (ed > T->appearance) ed = 1.0;
        if (iou[k] > T->proximity) ed = 1.0;
        c[k] = c[k] < ed ? c[k] : ed; /* np.minimum */
    }
    free(A);
    free(B);
    free(e);
}

typedef struct {
    int *m, nm, *ua, nua, *ub, nub;
} Assign;

static void assign(const double *c, int nr, int nc, double thr, Assign *r) {
    int k = nr < nc ? nr : nc;
    r->m = (int *)malloc(sizeof(int) * 2 * (k ? k : 1));
    r->ua = (int *)malloc(sizeof(int) * (nr ? nr : 1));
    r->ub = (int *)malloc(sizeof(int) * (nc ? nc : 1));
    bxo_linear_assignment(c, nr, nc, thr, r->m, &r->nm, r->ua, &r->nua, r->ub, &r->nub);
}
static void afree(Assign *r) {
    free(r->m);
    free(r->ua);
    free(r->ub);
}

static void kf_update(const bxo_tracker *T, Trk *t, const Trk *det) {
    bxo_kf_update(T->kind == KIND_BYTE ? BXO_KF_XYAH : BXO_KF_XYWH, t->mean, t->cov,
                  T->kind == KIND_BYTE ? det->xyah : det->xywh, 0.0);
}

static void trk_update(bxo_tracker *T, Trk *t, Trk *det) { /* STrack.update */
    t->frame_id = T->frame_count;
    t->tracklet_len++;
    kf_update(T, t, det);
    if (T->kind == KIND_BOT && det->curr) update_features(T, t, det->curr);
    t->state = ST_TRACKED;
    t->is_activated = 1;
    t->conf = det->conf;
    t->cls = det->cls;
    t->det_ind = det->det_ind;
    if (T->kind == KIND_BOT) update_cls(t, det->cls, det->conf);
}

static void trk_reactivate(bxo_tracker *T, Trk *t, Trk *det) { /* STrack.re_activate */
    kf_update(T, t, det);
    if (T->kind == KIND_BOT && det->curr) update_features(T, t, det->curr);
    t->tracklet_len = 0;
    t->state = ST_TRACKED;
    t->is_activated = 1;
    t->frame_id = T->frame_count;
    t->conf = det->conf;
    t->cls = det->cls;
    t->det_ind = det->det_ind;
    if (T->kind == KIND_BOT) update_cls(t, det->cls, det->conf);
}

static void trk_activate(bxo_tracker *T, Trk *t) { /* STrack.activate */
    t->id = ++T->id_count;
    bxo_kf_initiate(T->kind == KIND_BYTE ? BXO_KF_XYAH : BXO_KF_XYWH,
                    T->kind == KIND_BYTE ? t->xyah : t->xywh, t->mean, t->cov);
    t->has_mean = 1;
    t->tracklet_len = 0;
    t->state = ST_TRACKED;
    if (T->frame_count == 1) t->is_activated = 1;
    t->frame_id = T->frame_count;
    t->start_frame = T->frame_count;
}

/* joint_stracks: a then b's members not already present (by id = object). */
static List joint(bxo_tracker *T, const List *a, const List *b) {
    List r = {0};
    unsigned s = ++T->stamp;
    for (int i = 0; i < a->n; i++) {
        a->v[i]->stamp = s;
        lpush(&r, a->v[i]);
    }
    for (int i = 0; i < b->n; i++)
        if (b->v[i]->stamp != s) {
            b->v[i]->stamp = s;
            lpush(&r, b->v[i]);
        }
    return r;
}

/* sub_stracks: a minus members of b (dict keeps first position of each id). */
static List sub(bxo_tracker *T, const List *a, const List *b) {
    List r = {0};
    unsigned s = ++T->stamp;
    for (int i = 0; i < b->n; i++) b->v[i]->stamp = s;
    unsigned s2 = ++T->stamp;
    for (int i = 0; i < a->n; i++)
        if (a->v[i]->stamp != s && a->v[i]->stamp != s2) {
            a->v[i]->stamp = s2;
            lpush(&r, a->v[i]);
        }
    return r;
}

bxo_tracker *bxo_bytetrack_new(double min_conf, double track_thresh, double match_thresh,
                               int track_buffer, int frame_rate) {
    bxo_tracker *T = (bxo_tracker *)calloc(1, sizeof(bxo_tracker));
    T->kind = KIND_BYTE;
    T->low = min_conf;
    T->high = track_thresh;
    T->new_thresh = track_thresh; /* det_thresh = track_thresh (bytetrack.py:153) */
    T->match_thresh = match_thresh;
    T->max_time_lost = (int)(frame_rate / 30.0 * track_buffer);
    return T;
}

bxo_tracker *bxo_botsort_new(double track_high_thresh, double track_low_thresh,
                             double new_track_thresh, int track_buffer, double match_thresh,
                             double proximity_thresh, double appearance_thresh, int frame_rate,
                             int fuse_first_associate, int with_reid) {
    bxo_tracker *T = (bxo_tracker *)calloc(1, sizeof(bxo_tracker));
    T->kind = KIND_BOT;
    T->low = track_low_thresh;
    T->high = track_high_thresh;
    T->new_thresh = new_track_thresh;
    T->match_thresh = match_thresh;
    T->proximity = proximity_thresh;
    T->appearance = appearance_thresh;
    T->max_time_lost = (int)(frame_rate / 30.0 * track_buffer);
    T->fuse_first = fuse_first_associate;
    T->with_reid = with_reid;
    return T;
}

/* tracked_stracks then lost_stracks (list order): ids, states, Kalman mean/covariance.  Returns
 * the count; fills at most cap entries (NULL arrays skipped). */
int bxo_tracks(const bxo_tracker *T, int cap, int *ids, int *state, double *mean, double *cov) {
    const int n = T->active.n + T->lost.n;
    for (int k = 0; k < n && k < cap; k++) {
        const Trk *t = k < T->active.n ? T->active.v[k] : T->lost.v[k - T->active.n];
        if (ids) ids[k] = t->id;
        if (state) state[k] = t->state;
        if (mean) memcpy(mean + 8 * k, t->mean, sizeof t->mean);
        if (cov) memcpy(cov + 64 * k, t->cov, sizeof t->cov);
    }
    return n;
}

/* host edit of STrack.mean / .covariance by id; returns the number of ids found */
int bxo_state_set(bxo_tracker *T, int n, const int *ids, const double *mean, const double *cov) {
    int found = 0;
    for (int j = 0; j < n; j++)
        for (int k = 0; k < T->active.n + T->lost.n; k++) {
            Trk *t = k < T->active.n ? T->active.v[k] : T->lost.v[k - T->active.n];
            if (t->id != ids[j]) continue;
            if (mean) memcpy(t->mean, mean + 8 * j, sizeof t->mean);
            if (cov) memcpy(t->cov, cov + 64 * j, sizeof t->cov);
            found++;
            break;
        }
    return found;
}

int bxo_id_count(const bxo_tracker *T) { return T->id_count; }
int bxo_frame_count(const bxo_tracker *T) { return T->frame_count; }
void bxo_set_frame_count(bxo_tracker *T, int fc) { T->frame_count = fc; }

/* BaseTracker.per_class_decorator (basetracker.py:181-192): `self.active_tracks =
 * self.per_class_active_tracks[cls_id]` before the class's update, saved back after it.  Only
 * the active list is swapped: lost_stracks, removed_stracks and the id counter stay shared. */
void bxo_select_class(bxo_tracker *T, int cls) {
    if (cls == T->cur_cls) return;
    const int need = (cls > T->cur_cls ? cls : T->cur_cls) + 1;
    if (need > T->nparked) {
        T->parked = (List *)realloc(T->parked, sizeof(List) * need);
        memset(T->parked + T->nparked, 0, sizeof(List) * (need - T->nparked));
        T->nparked = need;
    }
    T->parked[T->cur_cls] = T->active;
    T->active = T->parked[cls];
    memset(&T->parked[cls], 0, sizeof(List));
    T->cur_cls = cls;
}

void bxo_free(bxo_tracker *T) {
    for (int c = 0; c < T->nparked; c++) { /* parked lists hold tracks of no other list */
        for (int i = 0; i < T->parked[c].n; i++) free_trk(T->parked[c].v[i]);
        lfree(&T->parked[c]);
    }
    free(T->parked);
    unsigned s = ++T->stamp;
    for (int i = 0; i < T->active.n; i++) T->active.v[i]->stamp = s;
    for (int i = 0; i < T->lost.n; i++)
        if (T->lost.v[i]->stamp != s) free_trk(T->lost.v[i]);
    for (int i = 0; i < T->active.n; i++) free_trk(T->active.v[i]);
    lfree(&T->active);
    lfree(&T->lost);
    free(T);
}

static void gmc(const double *H, const List *l) { /* botsort_track.py:91-104 multi_gmc */
    if (!H) return;
    for (int n = 0; n < l->n; n++) {
        Trk *t = l->v[n];
        double m[8], RP[64];
        /* R8 = kron(I4, R): block-diagonal 2x2 blocks */
        for (int b = 0; b < 4; b++) {
            m[2 * b] = H[0] * t->mean[2 * b] + H[1] * t->mean[2 * b + 1];
            m[2 * b + 1] = H[3] * t->mean[2 * b] + H[4] * t->mean[2 * b + 1];
        }
        m[0] += H[2];
        m[1] += H[5];
        memcpy(t->mean, m, sizeof m);
        for (int b = 0; b < 4; b++)
            for (int c = 0; c < 8; c++) {
                RP[8 * (2 * b) + c] = H[0] * t->cov[8 * (2 * b) + c] + H[1] * t->cov[8 * (2 * b + 1) + c];
                RP[8 * (2 * b + 1) + c] =
                    H[3] * t->cov[8 * (2 * b) + c] + H[4] * t->cov[8 * (2 * b + 1) + c];
            }
        for (int r = 0; r < 8; r++)
            for (int b = 0; b < 4; b++) {
                t->cov[8 * r + 2 * b] = RP[8 * r + 2 * b] * H[0] + RP[8 * r + 2 * b + 1] * H[1];
                t->cov[8 * r + 2 * b + 1] = RP[8 * r + 2 * b] * H[3] + RP[8 * r + 2 * b + 1] * H[4];
            }
    }
}

int bxo_update(bxo_tracker *T, const double *dets, int n, const void *embs, int emb_dim,
               int emb_is_f64, const double *warp, double *out, int out_cap) {
    const int BOT = T->kind == KIND_BOT;
    if (BOT && T->with_reid) {
        if (!embs && n > 0) return -1; /* ReID inference is out of scope: embs required */
        T->emb_dim = emb_dim;
        T->f64 = emb_is_f64;
    }
    T->frame_count++;
    List high = {0}, second = {0}, unconfirmed = {0}, tracked = {0}, activated = {0},
         refind = {0}, lost_l = {0}, removed_l = {0}, dets_all = {0};
    double *fbuf = NULL;
    if (BOT && T->with_reid && n > 0) fbuf = (double *)malloc(sizeof(double) * emb_dim);
    for (int i = 0; i < n; i++) { /* np.hstack([dets, arange]) then conf splits */
        /* basetracker.py:122-128: a numpy array has `.data` (a memoryview), which the setup
         * decorator turns into np.array(..., dtype=np.float32): every det value is rounded to
         * float32 before np.hstack widens it back to float64. */
        const double *d = dets + 6 * i;
        double d7[7] = {(float)d[0], (float)d[1], (float)d[2], (float)d[3],
                        (float)d[4], (float)d[5], (double)i};
        double conf = d7[4];
        int is_high = conf > T->high;
        int is_second = conf > T->low && conf < T->high;
        if (!is_high && !is_second) continue;
        const double *fs = NULL;
        if (is_high && BOT && T->with_reid) {
            for (int k = 0; k < emb_dim; k++)
                fbuf[k] = emb_is_f64 ? ((const double *)embs)[(size_t)i * emb_dim + k]
                                     : (double)((const float *)embs)[(size_t)i * emb_dim + k];
            fs = fbuf;
        }
        Trk *t = new_det(T, d7, fs);
        lpush(is_high ? &high : &second, t);
        lpush(&dets_all, t);
    }
    free(fbuf);
    for (int i = 0; i < T->active.n; i++)
        lpush(T->active.v[i]->is_activated ? &tracked : &unconfirmed, T->active.v[i]);

    /* Step 2: first association */
    List pool = joint(T, &tracked, &T->lost);
    if (pool.n) {
        double *mean = (double *)malloc(sizeof(double) * 8 * pool.n);
        double *cov = (double *)malloc(sizeof(double) * 64 * pool.n);
        for (int i = 0; i < pool.n; i++) {
            memcpy(mean + 8 * i, pool.v[i]->mean, sizeof(double) * 8);
            memcpy(cov + 64 * i, pool.v[i]->cov, sizeof(double) * 64);
            if (pool.v[i]->state != ST_TRACKED) {
                if (BOT) mean[8 * i + 6] = 0;
                mean[8 * i + 7] = 0;
            }
        }
        bxo_kf_multi_predict(BOT ? BXO_KF_XYWH : BXO_KF_XYAH, pool.n, mean, cov);
        for (int i = 0; i < pool.n; i++) {
            memcpy(pool.v[i]->mean, mean + 8 * i, sizeof(double) * 8);
            memcpy(pool.v[i]->cov, cov + 64 * i, sizeof(double) * 64);
        }
        free(mean);
        free(cov);
    }
    if (BOT) {
        gmc(warp, &pool);
        gmc(warp, &unconfirmed);
    }
    double *c1 = iou_distance(T, &pool, &high);
    if (!BOT) {
        fuse(c1, &pool, &high);
    } else {
        size_t sz = (size_t)pool.n * high.n;
        double *raw = (double *)malloc(sizeof(double) * (sz ? sz : 1));
        memcpy(raw, c1, sizeof(double) * sz);
        if (T->fuse_first) fuse(c1, &pool, &high);
        if (T->with_reid) fuse_reid(T, c1, raw, &pool, &high);
        free(raw);
    }
    Assign a1;
    assign(c1, pool.n, high.n, T->match_thresh, &a1);
    free(c1);
    for (int k = 0; k < a1.nm; k++) {
        Trk *t = pool.v[a1.m[2 * k]], *d = high.v[a1.m[2 * k + 1]];
        if (t->state == ST_TRACKED) {
            trk_update(T, t, d);
            lpush(&activated, t);
        } else {
            trk_reactivate(T, t, d);
            lpush(&refind, t);
        }
    }

    /* Step 3: second association with low-confidence detections */
    List r_tracked = {0};
    for (int k = 0; k < a1.nua; k++)
        if (pool.v[a1.ua[k]]->state == ST_TRACKED) lpush(&r_tracked, pool.v[a1.ua[k]]);
    double *c2 = iou_distance(T, &r_tracked, &second);
    Assign a2;
    assign(c2, r_tracked.n, second.n, 0.5, &a2);
    free(c2);
    for (int k = 0; k < a2.nm; k++) {
        Trk *t = r_tracked.v[a2.m[2 * k]], *d = second.v[a2.m[2 * k + 1]];
        if (t->state == ST_TRACKED) {
            trk_update(T, t, d);
            lpush(&activated, t);
        } else {
            trk_reactivate(T, t, d);
            lpush(&refind, t);
        }
    }
    for (int k = 0; k < a2.nua; k++) {
        Trk *t = r_tracked.v[a2.ua[k]];
        if (t->state != ST_LOST) {
            t->state = ST_LOST;
            lpush(&lost_l, t);
        }
    }

    /* unconfirmed tracks vs remaining high detections */
    List rem = {0};
    for (int k = 0; k < a1.nub; k++) lpush(&rem, high.v[a1.ub[k]]);
    double *c3 = iou_distance(T, &unconfirmed, &rem);
    if (!BOT) {
        fuse(c3, &unconfirmed, &rem);
    } else {
        size_t sz = (size_t)unconfirmed.n * rem.n;
        double *raw = (double *)malloc(sizeof(double) * (sz ? sz : 1));
        memcpy(raw, c3, sizeof(double) * sz);
        fuse(c3, &unconfirmed, &rem);
        if (T->with_reid) fuse_reid(T, c3, raw, &unconfirmed, &rem);
        free(raw);
    }
    Assign a3;
    assign(c3, unconfirmed.n, rem.n, 0.7, &a3);
    free(c3);
    for (int k = 0; k < a3.nm; k++) {
        Trk *t = unconfirmed.v[a3.m[2 * k]];
        trk_update(T, t, rem.v[a3.m[2 * k + 1]]);
        lpush(&activated, t);
    }
    for (int k = 0; k < a3.nua; k++) {
        Trk *t = unconfirmed.v[a3.ua[k]];
        t->state = ST_REMOVED;
        lpush(&removed_l, t);
    }

    /* Step 4: new tracks */
    for (int k = 0; k < a3.nub; k++) {
        Trk *t = rem.v[a3.ub[k]];
        if (t->conf < T->new_thresh) continue;
        trk_activate(T, t);
        lpush(&activated, t);
    }

    /* Step 5: bookkeeping */
    for (int i = 0; i < T->lost.n; i++) {
        Trk *t = T->lost.v[i];
        if (T->frame_count - t->frame_id > T->max_time_lost) {
            t->state = ST_REMOVED;
            lpush(&removed_l, t);
        }
    }
    List old_active = T->active, old_lost = T->lost;
    List act0 = {0};
    for (int i = 0; i < old_active.n; i++)
        if (old_active.v[i]->state == ST_TRACKED) lpush(&act0, old_active.v[i]);
    List act1 = joint(T, &act0, &activated);
    List act2 = joint(T, &act1, &refind);
    List lost1 = sub(T, &old_lost, &act2);
    for (int i = 0; i < lost_l.n; i++) lpush(&lost1, lost_l.v[i]);
    List removed_prev = {0};
    for (int i = 0; i < lost1.n; i++)
        if (lost1.v[i]->in_removed) lpush(&removed_prev, lost1.v[i]);
    List lost2 = sub(T, &lost1, &removed_prev);
    for (int i = 0; i < removed_l.n; i++) removed_l.v[i]->in_removed = 1;

    /* remove_duplicate_stracks(active, lost) */
    double *pd = iou_distance(T, &act2, &lost2);
    char *dupa = (char *)calloc(act2.n + 1, 1), *dupb = (char *)calloc(lost2.n + 1, 1);
    for (int p = 0; p < act2.n; p++)
        for (int q = 0; q < lost2.n; q++)
            if (pd[(size_t)p * lost2.n + q] < 0.15) {
                int tp = act2.v[p]->frame_id - act2.v[p]->start_frame;
                int tq = lost2.v[q]->frame_id - lost2.v[q]->start_frame;
                if (tp > tq) dupb[q] = 1;
                else dupa[p] = 1;
            }
    free(pd);
    List new_active = {0}, new_lost = {0};
    for (int p = 0; p < act2.n; p++)
        if (!dupa[p]) lpush(&new_active, act2.v[p]);
    for (int q = 0; q < lost2.n; q++)
        if (!dupb[q]) lpush(&new_lost, lost2.v[q]);
    free(dupa);
    free(dupb);

    /* outputs: [*xyxy, id, conf, cls, det_ind] for activated active tracks */
    int m = 0, rc = 0;
    for (int p = 0; p < new_active.n; p++) {
        Trk *t = new_active.v[p];
        if (!t->is_activated) continue;
        if (m >= out_cap) {
            rc = -2;
            continue;
        }
        double *o = out + 8 * m++;
        trk_xyxy(T, t, o);
        o[4] = t->id;
        o[5] = t->conf;
        o[6] = t->cls;
        o[7] = t->det_ind;
    }

    /* free everything no longer reachable: old members and detections not in the new lists */
    unsigned s = ++T->stamp;
    for (int i = 0; i < new_active.n; i++) new_active.v[i]->stamp = s;
    for (int i = 0; i < new_lost.n; i++) new_lost.v[i]->stamp = s;
    unsigned s2 = ++T->stamp;
    List *pools[3] = {&old_active, &old_lost, &dets_all};
    for (int q = 0; q < 3; q++)
        for (int i = 0; i < pools[q]->n; i++) {
            Trk *t = pools[q]->v[i];
            if (t->stamp != s && t->stamp != s2) {
                t->stamp = s2;
                free_trk(t);
            }
        }
    T->active = new_active;
    T->lost = new_lost;

    afree(&a1);
    afree(&a2);
    afree(&a3);
    List *tmp[] = {&high, &second, &unconfirmed, &tracked, &activated, &refind, &lost_l,
                   &removed_l, &dets_all, &pool, &r_tracked, &rem, &act0, &act1, &act2,
                   &lost1, &removed_prev, &lost2, &old_active, &old_lost};
    for (size_t i = 0; i < sizeof tmp / sizeof tmp[0]; i++) lfree(tmp[i]);
    return rc ? rc : m;
}
