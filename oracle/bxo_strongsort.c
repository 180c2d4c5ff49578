/*
 * StrongSort ("enhanced" fork) per-frame update — trackers/strongsort/strongsort.py:17-232 and
 * sort/{tracker,track,detection,iou_matching,linear_assignment}.py — restated in plain C (fp64).
 *
 * TEST INFRASTRUCTURE ONLY (see bxo.h).  Runs the fork with the minimal patch P6
 * (`unmatched_tracks_3 = []`), handle_occlusions=False (D7: the occlusion
 * handler crashes on mutual occlusion; it is a host-side post-process) and a born-Confirmed flag
 * standing for the reference's GITHUB_ACTIONS=true switch (D8).  Pinned by
 * tests/golden/trk_strongsort_*.npz.
 *
 * Fixed orders where the reference's is not pinned (mirrored by the HIP engine):
 *   - np.linalg.norm of a 1-D feature and np.dot of two 1-D features (BLAS ddot) = the engine's
 *     "wave order" (64 lane-strided partial sums + xor butterfly; bxo_track.c vnorm);
 *   - the NN gallery's np.dot(samples, dets.T) = an ascending-k fma chain (the fp64 MFMA order,
 *     as bxo_nn_cosine_distance); row norms with axis=1 are numpy's pairwise sums (pinned);
 *   - Kalman update/gating: cho/triangular solves in bxo_ops.c's order (LAPACK order unpinned).
 * scipy.optimize.linear_sum_assignment is restated exactly (Crouse's rectangular shortest
 * augmenting path, its tie rules included) — checked against scipy by tests/test_oracle.py.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bxo.h"

#define SS_INFTY 1e5
#define SS_GATE 9.4877 /* chi2inv95[4] */
#define SS_MAXF 10
#define SS_MAXC 20
#define SS_MAXH 10
#define SS_LOST_CAP 30

/* ------------------------------------------------------------------------------------------ */
static double wave_dot(const double *a, const double *b, int n) {
    double s[64], t[64];
    for (int l = 0; l < 64; l++) {
        s[l] = 0.0;
        for (int k = l; k < n; k += 64) s[l] += a[k] * b[k];
    }
    for (int d = 32; d >= 1; d >>= 1) {
        for (int l = 0; l < 64; l++) t[l] = s[l] + s[l ^ d];
        memcpy(s, t, sizeof s);
    }
    return s[0];
}
static double wave_norm(const double *a, int n) { return sqrt(wave_dot(a, a, n)); }

/* numpy add.reduce on a contiguous float64 run (pairwise_sum, PW_BLOCKSIZE 128) */
static double pw_sum(const double *x, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; i++) r += x[i];
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; k++) r[k] = x[k];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; k++) r[k] += x[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += x[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_sum(x, n2) + pw_sum(x + n2, n - n2);
}
static double np_mean(const double *x, int n) { return pw_sum(x, n) / n; }
static double np_std(const double *x, int n) {
    const double m = np_mean(x, n);
    double d[SS_MAXC];
    for (int i = 0; i < n; i++) {
        d[i] = x[i] - m;
        d[i] = d[i] * d[i];
    }
    return sqrt(pw_sum(d, n) / n);
}
/* np.linalg.norm(x, axis=1) of one row: sqrt of the pairwise sum of squares */
static double np_row_norm(const double *x, int n) {
    double *sq = (double *)malloc(sizeof(double) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) sq[i] = x[i] * x[i];
    const double s = pw_sum(sq, n);
    free(sq);
    return sqrt(s);
}
static double clip(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static double pymax(double a, double b) { return b > a ? b : a; } /* Python max(a, b) */
static double pymin(double a, double b) { return b < a ? b : a; } /* Python min(a, b) */
static double norm2(double a, double b) { return sqrt(a * a + b * b); }

/* ------------------------------------------------------------------------------------------ */
/* XYAH Kalman filter, single-track predict (base_kalman_filter.py:61-78): mean = mean F^T;
 * cov = multi_dot((F, P, F^T)) + Q = F (P F^T) + Q (numpy picks A(BC) on the cost tie). */
static void kf_predict1(double *m, double *P) {
    const double sp = 1.0 / 20, sv = 1.0 / 160;
    double s[8] = {sp * m[3], sp * m[3], 1e-2, sp * m[3], sv * m[3], sv * m[3], 1e-5, sv * m[3]};
    double M[64];
    for (int k = 0; k < 4; k++) m[k] = m[k] + m[k + 4];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) M[8 * i + j] = j < 4 ? P[8 * i + j] + P[8 * i + j + 4] : P[8 * i + j];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            const double v = i < 4 ? M[8 * i + j] + M[8 * (i + 4) + j] : M[8 * i + j];
            P[8 * i + j] = i == j ? v + s[i] * s[i] : v;
        }
}

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    double tlwh[4], conf, cls, det_ind, quality;
    double *feat; /* F doubles (this frame's copy; normalised in place by a birth) */
} ss_det;

typedef struct ss_track {
    double mean[8], cov[64];
    int id, state, hits, age, tsu, max_age, n_init;
    double conf, cls, det_ind, base_alpha;
    double quality, stability, app_cons, motion_cons;
    double vel[SS_MAXH][2], pos[SS_MAXH][2];
    int nvel, npos;
    double confh[SS_MAXC];
    int nconf;
    double *feat[SS_MAXF];
    int nfeat;
    int missed, confirmed_det, low_streak, high_streak, lost_frame;
} ss_track;

typedef struct {
    int id, n, cap;
    double **vec; /* samples pre-normalised: x / (np_row_norm(x) + 1e-8), the divisions
                     _nn_cosine_distance performs (linear_assignment.py:468-497) — done once at
                     insertion, bit-identical to doing them per query */
    double *q;
    uint64_t *h;  /* content hash of the raw sample (duplicate samples give identical rows) */
} ss_gallery;

struct bxo_ss {
    bxo_ss_params p;
    int F, frame_count, next_id, crowd_mode, orig_stored, orig_max_age, orig_budget;
    int hist_len; /* len(Tracker.matching_history): updates so far, capped at 100 */
    double orig_thr;
    int max_age, budget; /* tracker.max_age, metric.budget (crowd-adjusted) */
    double thr;          /* metric.matching_threshold */
    ss_track **trk;
    int ntrk, captrk;
    ss_track **lost;
    int nlost;
    ss_gallery *gal;
    int ngal, capgal;
    /* OcclusionAwareTracker state (handle_occlusions=True): track_visibility by id, and the
     * occlusion_buffer (id -> deque(maxlen=10) of features[-1] copies) */
    int occ_on;
    double occ_thr;
    double *vis;
    int nvis;
    struct occ_buf *ob;
    int nob, capob;
};

typedef struct occ_buf {
    int id, n;
    double *f[10];
} occ_buf;

static double *vdup(const double *x, int F) {
    double *y = (double *)malloc(sizeof(double) * F);
    memcpy(y, x, sizeof(double) * F);
    return y;
}

static uint64_t fnv64(const double *x, int F) {
    const unsigned char *b = (const unsigned char *)x;
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(double) * (size_t)F; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static void track_free(ss_track *t) {
    if (!t) return;
    for (int k = 0; k < t->nfeat; k++) free(t->feat[k]);
    free(t);
}

bxo_ss *bxo_ss_new(const bxo_ss_params *p) {
    bxo_ss *s = (bxo_ss *)calloc(1, sizeof *s);
    s->p = *p;
    s->next_id = 1;
    s->max_age = p->max_age;
    s->budget = p->nn_budget;
    s->thr = p->max_cos_dist;
    s->captrk = 64;
    s->trk = (ss_track **)calloc(s->captrk, sizeof(ss_track *));
    s->lost = (ss_track **)calloc(SS_LOST_CAP + 1, sizeof(ss_track *));
    return s;
}

void bxo_ss_free(bxo_ss *s) {
    if (!s) return;
    for (int b = 0; b < s->nob; b++)
        for (int k = 0; k < s->ob[b].n; k++) free(s->ob[b].f[k]);
    free(s->ob);
    free(s->vis);
    for (int i = 0; i < s->ntrk; i++) track_free(s->trk[i]);
    for (int i = 0; i < s->nlost; i++) track_free(s->lost[i]);
    for (int g = 0; g < s->ngal; g++) {
        for (int k = 0; k < s->gal[g].n; k++) free(s->gal[g].vec[k]);
        free(s->gal[g].vec);
        free(s->gal[g].q);
        free(s->gal[g].h);
    }
    free(s->gal);
    free(s->trk);
    free(s->lost);
    free(s);
}

int bxo_ss_next_id(const bxo_ss *s) { return s->next_id; }

/* host edit of Track.mean / Track.covariance by id; returns the number of ids found */
int bxo_ss_state_set(bxo_ss *s, int n, const int *ids, const double *mean, const double *cov) {
    int found = 0;
    for (int j = 0; j < n; j++)
        for (int i = 0; i < s->ntrk; i++)
            if (s->trk[i]->id == ids[j]) {
                if (mean) memcpy(s->trk[i]->mean, mean + 8 * j, sizeof(double) * 8);
                if (cov) memcpy(s->trk[i]->cov, cov + 64 * j, sizeof(double) * 64);
                found++;
                break;
            }
    return found;
}

int bxo_ss_tracks(const bxo_ss *s, int cap, int *ids, int *state, double *mean, double *cov) {
    for (int i = 0; i < s->ntrk && i < cap; i++) {
        if (ids) ids[i] = s->trk[i]->id;
        if (state) state[i] = s->trk[i]->state;
        if (mean) memcpy(mean + 8 * i, s->trk[i]->mean, sizeof(double) * 8);
        if (cov) memcpy(cov + 64 * i, s->trk[i]->cov, sizeof(double) * 64);
    }
    return s->ntrk;
}

/* sort/track.py:137-166 */
static void to_tlwh(const ss_track *t, double *r) {
    r[0] = t->mean[0], r[1] = t->mean[1], r[2] = t->mean[2], r[3] = t->mean[3];
    r[2] *= r[3];
    r[0] -= r[2] / 2;
    r[1] -= r[3] / 2;
}
static void to_tlbr(const ss_track *t, double *r) {
    to_tlwh(t, r);
    r[2] = r[0] + r[2];
    r[3] = r[1] + r[3];
}
/* sort/detection.py:35-42 */
static void det_xyah(const ss_det *d, double *r) {
    r[0] = d->tlwh[0], r[1] = d->tlwh[1], r[2] = d->tlwh[2], r[3] = d->tlwh[3];
    r[0] += r[2] / 2;
    r[1] += r[3] / 2;
    r[2] /= r[3];
}

/* Track._update_motion_consistency (track.py:379-400) */
static void motion_cons(ss_track *t, const double *prev, const double *cur) {
    if (t->nvel < 2) return;
    const double *pv = t->vel[t->nvel - 1];
    const double pred[2] = {prev[0] + pv[0], prev[1] + pv[1]};
    const double act[2] = {cur[0] - prev[0], cur[1] - prev[1]};
    const double pm[2] = {pred[0] - prev[0], pred[1] - prev[1]};
    double c;
    if (norm2(pm[0], pm[1]) > 0) {
        const double err = norm2(act[0] - pm[0], act[1] - pm[1]);
        const double mx = pymax(norm2(pm[0], pm[1]) * 0.5, 10.0);
        c = pymax(0, 1.0 - (err / mx));
    } else {
        c = norm2(act[0], act[1]) < 5.0 ? 1.0 : 0.5;
    }
    t->motion_cons = 0.8 * t->motion_cons + 0.2 * c;
}

static void push2(double (*h)[2], int *n, const double *v) {
    if (*n == SS_MAXH) {
        memmove(h[0], h[1], sizeof(double) * 2 * (SS_MAXH - 1));
        (*n)--;
    }
    h[*n][0] = v[0];
    h[*n][1] = v[1];
    (*n)++;
}

/* Track.__init__ (track.py:76-131) */
static ss_track *track_new(const bxo_ss *s, ss_det *d, int id, int max_age) {
    const int F = s->F;
    ss_track *t = (ss_track *)calloc(1, sizeof *t);
    double bb[4];
    det_xyah(d, bb);
    t->id = id;
    t->conf = d->conf, t->cls = d->cls, t->det_ind = d->det_ind;
    t->hits = 1, t->age = 1, t->tsu = 0;
    t->base_alpha = s->p.ema_alpha;
    t->state = s->p.born_confirmed ? 2 : 1;
    t->confh[0] = d->conf;
    t->nconf = 1;
    if (d->feat) { /* detection.feat /= norm + 1e-8, in place; the track keeps that array */
        const double n = wave_norm(d->feat, F) + 1e-8;
        for (int k = 0; k < F; k++) d->feat[k] /= n;
        t->feat[0] = vdup(d->feat, F);
        t->nfeat = 1;
    }
    t->n_init = s->p.n_init;
    t->max_age = max_age;
    t->quality = d->quality;
    t->stability = 0.0;
    t->app_cons = 1.0;
    t->motion_cons = 1.0;
    t->confirmed_det = 1;
    t->high_streak = d->conf > 0.7 ? 1 : 0;
    bxo_kf_initiate(BXO_KF_XYAH, bb, t->mean, t->cov);
    push2(t->pos, &t->npos, bb);
    return t;
}

/* Track.predict (track.py:177-202) */
static void track_predict(ss_track *t) {
    kf_predict1(t->mean, t->cov);
    t->age++;
    t->tsu++;
    push2(t->vel, &t->nvel, t->mean + 4);
    push2(t->pos, &t->npos, t->mean);
    if (t->npos >= 2) motion_cons(t, t->pos[t->npos - 2], t->pos[t->npos - 1]);
}

/* Track.camera_update (track.py:163-175) */
static void track_camera(ss_track *t, const double *w) {
    double b[4];
    to_tlbr(t, b);
    const double x1 = (w[0] * b[0] + w[1] * b[1]) + w[2], y1 = (w[3] * b[0] + w[4] * b[1]) + w[5];
    const double x2 = (w[0] * b[2] + w[1] * b[3]) + w[2], y2 = (w[3] * b[2] + w[4] * b[3]) + w[5];
    const double ww = x2 - x1, hh = y2 - y1;
    const double cx = x1 + ww / 2, cy = y1 + hh / 2;
    const double prev[2] = {t->mean[0], t->mean[1]};
    t->mean[0] = cx, t->mean[1] = cy, t->mean[2] = ww / hh, t->mean[3] = hh;
    const double cur[2] = {cx, cy};
    motion_cons(t, prev, cur);
}

/* Track.update (track.py:204-277) and its helpers (:313-377) */
static void track_update(const bxo_ss *s, ss_track *t, const ss_det *d) {
    const int F = s->F;
    double bb[4];
    det_xyah(d, bb);
    t->conf = d->conf, t->cls = d->cls, t->det_ind = d->det_ind;
    bxo_kf_update(BXO_KF_XYAH, t->mean, t->cov, bb, t->conf);
    if (d->feat) {
        const double nd = wave_norm(d->feat, F) + 1e-8;
        double *nf = (double *)malloc(sizeof(double) * F);
        for (int k = 0; k < F; k++) nf[k] = d->feat[k] / nd;
        if (t->nfeat) {
            const double *last = t->feat[t->nfeat - 1];
            const double sim = wave_dot(nf, last, F) / (wave_norm(nf, F) * wave_norm(last, F) + 1e-8);
            t->app_cons = 0.9 * t->app_cons + 0.1 * sim;
            const double cf = d->conf > 0.7 ? 1.0 : (d->conf > 0.3 ? 0.5 : 0.2);
            const double af = sim > 0.7 ? 1.0 : (sim > 0.4 ? 0.7 : 0.4);
            const double a = clip(t->base_alpha * cf * af, 0.1, 0.95);
            double *sm = (double *)malloc(sizeof(double) * F);
            for (int k = 0; k < F; k++) sm[k] = a * last[k] + (1 - a) * nf[k];
            const double ns = wave_norm(sm, F) + 1e-8;
            for (int k = 0; k < F; k++) sm[k] /= ns;
            free(nf);
            nf = sm;
        }
        if (t->nfeat == SS_MAXF) { /* features[-max_features:] */
            free(t->feat[0]);
            memmove(t->feat, t->feat + 1, sizeof(double *) * (SS_MAXF - 1));
            t->nfeat--;
        }
        t->feat[t->nfeat++] = nf;
    }
    if (t->nconf == SS_MAXC) {
        memmove(t->confh, t->confh + 1, sizeof(double) * (SS_MAXC - 1));
        t->nconf--;
    }
    t->confh[t->nconf++] = d->conf;
    if (d->conf > 0.7) {
        t->high_streak++;
        t->low_streak = 0;
    } else if (d->conf < 0.3) {
        t->low_streak++;
        t->high_streak = 0;
    } else {
        t->low_streak = 0;
        t->high_streak = 0;
    }
    t->hits++;
    t->confirmed_det++;
    t->tsu = 0;
    /* _update_quality_score */
    double cq = d->conf;
    if (t->nconf > 1) {
        const double avg = np_mean(t->confh, t->nconf);
        const double stab = 1.0 - np_std(t->confh, t->nconf);
        cq = 0.7 * cq + 0.3 * avg * stab;
    }
    const double lb = pymin(t->hits / 20.0, 0.2);
    const double ab = pymax(0, (t->app_cons - 0.5) * 0.2);
    const double mb = pymax(0, (t->motion_cons - 0.5) * 0.1);
    t->quality = clip(((cq + lb) + ab) + mb, 0.0, 1.0);
    /* _update_stability_score */
    const double cs = t->nconf > 3 ? 1.0 - pymin(np_std(t->confh, t->nconf), 1.0) : 0.5;
    const double hr = (double)t->confirmed_det / (t->age > 1 ? t->age : 1);
    const double cons = (0.4 * t->app_cons + 0.3 * t->motion_cons) + 0.3 * cs;
    t->stability = clip(0.5 * hr + 0.5 * cons, 0.0, 1.0);
    if (t->state == 1 && (t->hits >= t->n_init || (t->hits >= 1 && t->quality > 0.8))) t->state = 2;
}

/* Track.mark_missed (track.py:279-293) */
static void track_missed(ss_track *t) {
    t->missed++;
    int thr = t->max_age;
    if (t->quality > 0.8)
        thr = (int)(t->max_age * 1.5);
    else if (t->quality < 0.3)
        thr = (int)(t->max_age * 0.5);
    if (t->state == 1)
        t->state = 3;
    else if (t->tsu > thr)
        t->state = 3;
}

/* ------------------------------------------------------------------------------------------ */
/* NearestNeighborDistanceMetric (sort/linear_assignment.py:499-618), cosine                   */
static ss_gallery *gal_find(bxo_ss *s, int id, int create) {
    for (int g = 0; g < s->ngal; g++)
        if (s->gal[g].id == id) return &s->gal[g];
    if (!create) return NULL;
    if (s->ngal == s->capgal) {
        s->capgal = s->capgal ? 2 * s->capgal : 32;
        s->gal = (ss_gallery *)realloc(s->gal, sizeof(ss_gallery) * s->capgal);
    }
    ss_gallery *g = &s->gal[s->ngal++];
    memset(g, 0, sizeof *g);
    g->id = id;
    return g;
}

/* samples_with_quality.sort(key=quality, reverse=True) (stable) + [:keep] */
static void gal_prune(ss_gallery *g, int keep) {
    for (int i = 1; i < g->n; i++) { /* stable insertion sort, descending */
        double *v = g->vec[i];
        const double q = g->q[i];
        const uint64_t h = g->h[i];
        int j = i - 1;
        while (j >= 0 && g->q[j] < q) {
            g->vec[j + 1] = g->vec[j];
            g->q[j + 1] = g->q[j];
            g->h[j + 1] = g->h[j];
            j--;
        }
        g->vec[j + 1] = v;
        g->q[j + 1] = q;
        g->h[j + 1] = h;
    }
    for (int k = keep; k < g->n; k++) free(g->vec[k]);
    if (g->n > keep) g->n = keep;
}

static void partial_fit(bxo_ss *s, double **feats, const int *tgt, int n, const int *active,
                        int nact) {
    const int F = s->F;
    for (int k = 0; k < n; k++) {
        ss_gallery *g = gal_find(s, tgt[k], 1);
        if (g->n == g->cap) {
            g->cap = g->cap ? 2 * g->cap : 16;
            g->vec = (double **)realloc(g->vec, sizeof(double *) * g->cap);
            g->q = (double *)realloc(g->q, sizeof(double) * g->cap);
            g->h = (uint64_t *)realloc(g->h, sizeof(uint64_t) * g->cap);
        }
        double *v = vdup(feats[k], F);
        const double den = np_row_norm(feats[k], F) + 1e-8;
        for (int q = 0; q < F; q++) v[q] = feats[k][q] / den;
        g->vec[g->n] = v;
        g->q[g->n] = wave_norm(feats[k], F);
        g->h[g->n] = fnv64(feats[k], F);
        g->n++;
        if (s->budget > 0 && g->n > s->budget) gal_prune(g, s->budget);
    }
    const int keep = s->budget > 0 ? (s->budget / 4 < 5 ? s->budget / 4 : 5) : 5;
    for (int gi = 0; gi < s->ngal; gi++) {
        ss_gallery *g = &s->gal[gi];
        int is_active = 0;
        for (int a = 0; a < nact && !is_active; a++) is_active = active[a] == g->id;
        if (is_active || g->n == 0) continue;
        if (g->n > keep) gal_prune(g, keep);
    }
}

/* distance(): min over the target's samples of 1 - clip(s^.d^, -1, 1); no samples -> 1e5.
 * One target against nd detections.  A sample equal to an earlier one (the tracker re-appends
 * the same smoothed features every frame, tracker.py:166-178) gives the same distances, so only
 * distinct samples are evaluated — the minimum is unchanged. */
static void nn_dist_row(bxo_ss *s, int id, double *const *dn, const int *di, int nd,
                        double *row) {
    ss_gallery *g = gal_find(s, id, 0);
    if (!g || g->n == 0) {
        for (int c = 0; c < nd; c++) row[c] = SS_INFTY;
        return;
    }
    const int F = s->F;
    int *uniq = (int *)malloc(sizeof(int) * g->n);
    int nu = 0;
    for (int k = 0; k < g->n; k++) {
        int dup = 0;
        for (int u = 0; u < nu && !dup; u++)
            dup = g->h[uniq[u]] == g->h[k] && !memcmp(g->vec[uniq[u]], g->vec[k], sizeof(double) * F);
        if (!dup) uniq[nu++] = k;
    }
    for (int c = 0; c < nd; c++) {
        const double *x = dn[di[c]];
        double best = 0.0;
        for (int u = 0; u < nu; u++) {
            const double *v = g->vec[uniq[u]];
            double acc = 0.0;
            for (int q = 0; q < F; q++) acc = fma(v[q], x[q], acc);
            const double d = 1.0 - clip(acc, -1.0, 1.0);
            if (u == 0 || d < best) best = d;
        }
        row[c] = best;
    }
    free(uniq);
}

/* ------------------------------------------------------------------------------------------ */
/* scipy.optimize.linear_sum_assignment (rectangular_lsap.cpp: Crouse's shortest augmenting   */
/* path), restated with its tie rules.  cost [nr][nc] row-major; pairs sorted by row.         */
int bxo_lsap(const double *cost_in, int nr, int nc, int *rows, int *cols) {
    if (nr == 0 || nc == 0) return 0;
    const int tr = nc < nr;
    int R = nr, C = nc;
    double *cost = (double *)malloc(sizeof(double) * nr * nc);
    if (tr) {
        for (int i = 0; i < nr; i++)
            for (int j = 0; j < nc; j++) cost[j * nr + i] = cost_in[i * nc + j];
        R = nc, C = nr;
    } else {
        memcpy(cost, cost_in, sizeof(double) * nr * nc);
    }
    double *u = (double *)calloc(R, sizeof(double)), *v = (double *)calloc(C, sizeof(double));
    double *spc = (double *)malloc(sizeof(double) * C);
    int *path = (int *)malloc(sizeof(int) * C), *col4row = (int *)malloc(sizeof(int) * R);
    int *row4col = (int *)malloc(sizeof(int) * C), *rem = (int *)malloc(sizeof(int) * C);
    unsigned char *SR = (unsigned char *)malloc(R), *SC = (unsigned char *)malloc(C);
    for (int j = 0; j < C; j++) path[j] = -1, row4col[j] = -1;
    for (int i = 0; i < R; i++) col4row[i] = -1;
    int rc = 0;
    for (int cur = 0; cur < R; cur++) {
        double minVal = 0.0;
        int nrem = C;
        for (int it = 0; it < C; it++) rem[it] = C - it - 1;
        memset(SR, 0, R);
        memset(SC, 0, C);
        for (int j = 0; j < C; j++) spc[j] = INFINITY;
        int sink = -1, i = cur;
        while (sink == -1) {
            int index = -1;
            double lowest = INFINITY;
            SR[i] = 1;
            for (int it = 0; it < nrem; it++) {
                const int j = rem[it];
                const double r = minVal + cost[i * C + j] - u[i] - v[j];
                if (r < spc[j]) {
                    path[j] = i;
                    spc[j] = r;
                }
                if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)) {
                    lowest = spc[j];
                    index = it;
                }
            }
            minVal = lowest;
            if (minVal == INFINITY) {
                rc = -1;
                goto done;
            }
            const int j = rem[index];
            if (row4col[j] == -1)
                sink = j;
            else
                i = row4col[j];
            SC[j] = 1;
            rem[index] = rem[--nrem];
        }
        u[cur] += minVal;
        for (int q = 0; q < R; q++)
            if (SR[q] && q != cur) u[q] += minVal - spc[col4row[q]];
        for (int j = 0; j < C; j++)
            if (SC[j]) v[j] -= minVal - spc[j];
        int j = sink;
        for (;;) {
            const int q = path[j];
            row4col[j] = q;
            const int t = col4row[q];
            col4row[q] = j;
            j = t;
            if (q == cur) break;
        }
    }
    if (tr) { /* argsort(col4row): pairs ordered by the original row */
        int k = 0;
        for (int orig_row = 0; orig_row < nr; orig_row++)
            for (int q = 0; q < R; q++)
                if (col4row[q] == orig_row) rows[k] = orig_row, cols[k] = q, k++;
        rc = k;
    } else {
        for (int q = 0; q < R; q++) rows[q] = q, cols[q] = col4row[q];
        rc = R;
    }
done:
    free(cost);
    free(u);
    free(v);
    free(spc);
    free(path);
    free(col4row);
    free(row4col);
    free(rem);
    free(SR);
    free(SC);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    ss_det *d;
    int nd;
    double **dn; /* detection features normalised with numpy's pairwise row norm (+1e-8) */
} ss_frame;

enum { METRIC_GATED = 0, METRIC_IOU = 1 };

/* gated_metric (tracker.py:186-206): NN distance, gate_cost_matrix (linear_assignment.py:174-248)
 * and _apply_id_preservation_weighting (tracker.py:283-298); or iou_cost (iou_matching.py). */
static void metric_cost(bxo_ss *s, ss_frame *fr, int kind, const int *ti, int nt, const int *di,
                        int nd, double *cost) {
    if (kind == METRIC_IOU) {
        for (int r = 0; r < nt; r++) {
            const ss_track *t = s->trk[ti[r]];
            if (t->tsu > 1) {
                for (int c = 0; c < nd; c++) cost[r * nd + c] = SS_INFTY;
                continue;
            }
            double b[4];
            to_tlwh(t, b);
            const double br0 = b[0] + b[2], br1 = b[1] + b[3];
            for (int c = 0; c < nd; c++) {
                const double *q = fr->d[di[c]].tlwh;
                const double tl0 = fmax(b[0], q[0]), tl1 = fmax(b[1], q[1]);
                const double e0 = fmin(br0, q[0] + q[2]), e1 = fmin(br1, q[1] + q[3]);
                const double w = fmax(0.0, e0 - tl0), h = fmax(0.0, e1 - tl1);
                const double ai = w * h;
                cost[r * nd + c] = 1.0 - ai / ((b[2] * b[3] + q[2] * q[3]) - ai);
            }
        }
        return;
    }
    double (*meas)[4] = (double(*)[4])malloc(sizeof(double) * 4 * (nd ? nd : 1));
    for (int c = 0; c < nd; c++) det_xyah(&fr->d[di[c]], meas[c]);
    double *gd = (double *)malloc(sizeof(double) * (nd ? nd : 1));
    /* the NN block is independent per target: rows in parallel (OpenMP; bxo_set_threads) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int r = 0; r < nt; r++) nn_dist_row(s, s->trk[ti[r]]->id, fr->dn, di, nd, cost + r * nd);
    for (int r = 0; r < nt; r++) {
        const ss_track *t = s->trk[ti[r]];
        double *row = cost + r * nd;
        bxo_kf_gating_distance(BXO_KF_XYAH, t->mean, t->cov, &meas[0][0], nd, gd);
        for (int c = 0; c < nd; c++)
            if (gd[c] > SS_GATE) row[c] = SS_INFTY;
        /* _compute_enhanced_motion_cost (:288-307) */
        const double mf = 2.0 - t->motion_cons;
        double pp[2] = {0, 0};
        if (t->nvel > 0) pp[0] = t->mean[0] + t->vel[t->nvel - 1][0], pp[1] = t->mean[1] + t->vel[t->nvel - 1][1];
        /* _compute_adaptive_lambda (:310-329) */
        const double af = pymin(t->age / 10.0, 1.0);
        double al = s->p.mc_lambda + (1 - s->p.mc_lambda) * af * 0.1;
        al = al * (0.8 + 0.4 * t->motion_cons);
        if (t->app_cons < 0.5) al = pymin(al * 1.2, 0.99);
        al = clip(al, 0.1, 0.99);
        for (int c = 0; c < nd; c++) {
            double m = gd[c] * mf;
            if (t->nvel > 0) {
                const double ve = norm2(meas[c][0] - pp[0], meas[c][1] - pp[1]);
                m *= 1.0 + pymin(ve / 50.0, 1.0);
            }
            double v = al * row[c] + (1 - al) * m;
            /* _apply_track_specific_adjustments (:332-352) */
            if (t->quality > 0.8) v *= 0.95;
            if (t->hits > 10 && t->tsu == 0) v *= 0.98;
            if (t->high_streak > 3) v *= 0.97;
            if (t->low_streak > 2) v *= 1.05;
            row[c] = v;
        }
        if (s->p.id_preservation_weight > 0) {
            const double pb = s->p.id_preservation_weight * pymin(t->hits / 10.0, 1.0);
            for (int c = 0; c < nd; c++) row[c] *= (1.0 - pb);
        }
    }
    free(meas);
    free(gd);
}

/* min_cost_matching (linear_assignment.py:14-93) with _enhance_cost_matrix (:251-273).
 * matches (track, det) appended at *nm; the unmatched detection list written to ud_out. */
static void min_cost_matching(bxo_ss *s, ss_frame *fr, int kind, double max_d, const int *ti,
                              int nt, const int *di, int nd, int *matches, int *nm, int *ut_out,
                              int *nut, int *ud_out, int *nud) {
    *nut = *nud = 0;
    if (nd == 0 || nt == 0) {
        for (int k = 0; k < nt; k++) ut_out[(*nut)++] = ti[k];
        for (int k = 0; k < nd; k++) ud_out[(*nud)++] = di[k];
        return;
    }
    double *cost = (double *)malloc(sizeof(double) * nt * nd);
    metric_cost(s, fr, kind, ti, nt, di, nd, cost);
    for (int r = 0; r < nt; r++) {
        const ss_track *t = s->trk[ti[r]];
        for (int c = 0; c < nd; c++) {
            const ss_det *d = &fr->d[di[c]];
            double *e = &cost[r * nd + c];
            const double cq = (t->quality + d->quality) / 2.0;
            *e *= clip(1.0 - (cq - 0.5) * 0.2, 0.8, 1.2);
            if (t->cls == d->cls) *e *= 0.9;
            double cf = 1.0;
            if (t->conf > 0.7 && d->conf > 0.7)
                cf = 0.9;
            else if (t->conf < 0.3 || d->conf < 0.3)
                cf = 1.1;
            *e *= cf;
        }
    }
    for (int q = 0; q < nt * nd; q++)
        if (cost[q] > max_d) cost[q] = max_d + 1e-5;
    const int k = nt < nd ? nt : nd;
    int *rr = (int *)malloc(sizeof(int) * k), *cc = (int *)malloc(sizeof(int) * k);
    const int np_ = bxo_lsap(cost, nt, nd, rr, cc);
    unsigned char *cu = (unsigned char *)calloc(nd, 1), *ru = (unsigned char *)calloc(nt, 1);
    for (int q = 0; q < np_; q++) cu[cc[q]] = 1, ru[rr[q]] = 1;
    for (int c = 0; c < nd; c++)
        if (!cu[c]) ud_out[(*nud)++] = di[c];
    for (int r = 0; r < nt; r++)
        if (!ru[r]) ut_out[(*nut)++] = ti[r];
    for (int q = 0; q < np_; q++) {
        if (cost[rr[q] * nd + cc[q]] > max_d) {
            ut_out[(*nut)++] = ti[rr[q]];
            ud_out[(*nud)++] = di[cc[q]];
        } else {
            matches[2 * *nm] = ti[rr[q]];
            matches[2 * *nm + 1] = di[cc[q]];
            (*nm)++;
        }
    }
    free(cost);
    free(rr);
    free(cc);
    free(cu);
    free(ru);
}

/* matching_cascade (linear_assignment.py:96-171) with _prioritize_tracks_by_quality */
static void matching_cascade(bxo_ss *s, ss_frame *fr, double max_d, const int *ti, int nt,
                             const int *di, int nd, int *matches, int *nm) {
    const int cap = nt + nd + 1;
    int *ud = (int *)malloc(sizeof(int) * cap), *ud2 = (int *)malloc(sizeof(int) * cap);
    int *lvl = (int *)malloc(sizeof(int) * cap), *ut = (int *)malloc(sizeof(int) * cap);
    int nud = nd;
    memcpy(ud, di, sizeof(int) * nd);
    int *ages = (int *)malloc(sizeof(int) * cap), na = 0;
    for (int k = 0; k < nt; k++) {
        const int a = s->trk[ti[k]]->tsu;
        int seen = 0;
        for (int q = 0; q < na && !seen; q++) seen = ages[q] == a;
        if (!seen) ages[na++] = a;
    }
    for (int x = 1; x < na; x++) /* sorted(keys) */
        for (int y = x; y > 0 && ages[y - 1] > ages[y]; y--) {
            const int tmp = ages[y];
            ages[y] = ages[y - 1];
            ages[y - 1] = tmp;
        }
    for (int q = 0; q < na; q++) {
        if (ages[q] > s->max_age) break;
        int nl = 0;
        for (int k = 0; k < nt; k++)
            if (s->trk[ti[k]]->tsu == ages[q]) lvl[nl++] = ti[k];
        for (int x = 1; x < nl; x++) { /* sorted by -(quality + stability), stable */
            const int v = lvl[x];
            const double key = -(s->trk[v]->quality + s->trk[v]->stability);
            int y = x - 1;
            while (y >= 0 && -(s->trk[lvl[y]]->quality + s->trk[lvl[y]]->stability) > key) {
                lvl[y + 1] = lvl[y];
                y--;
            }
            lvl[y + 1] = v;
        }
        int nut, nud2;
        min_cost_matching(s, fr, METRIC_GATED, max_d, lvl, nl, ud, nud, matches, nm, ut, &nut,
                          ud2, &nud2);
        memcpy(ud, ud2, sizeof(int) * nud2);
        nud = nud2;
    }
    free(ud);
    free(ud2);
    free(lvl);
    free(ut);
    free(ages);
}

static int in_list(const int *a, int n, int v) {
    for (int k = 0; k < n; k++)
        if (a[k] == v) return 1;
    return 0;
}

/* Tracker._enhanced_match (tracker.py:183-281) with P6 */
static void enhanced_match(bxo_ss *s, ss_frame *fr, int *matches, int *nm, int *fut, int *nfut,
                           int *aud, int *naud) {
    const int T = s->ntrk, D = fr->nd, cap = 2 * (T + D) + 2;
    int *conf_t = (int *)malloc(sizeof(int) * cap), nconf = 0;
    int *unconf_t = (int *)malloc(sizeof(int) * cap), nunconf = 0;
    int *hi = (int *)malloc(sizeof(int) * cap), nhi = 0, *med = (int *)malloc(sizeof(int) * cap), nmed = 0;
    int *lo = (int *)malloc(sizeof(int) * cap), nlo = 0;
    for (int i = 0; i < T; i++) {
        if (s->trk[i]->state == 2) conf_t[nconf++] = i;
        if (s->trk[i]->state != 1) unconf_t[nunconf++] = i;
    }
    for (int d = 0; d < D; d++) {
        const double c = fr->d[d].conf;
        if (c >= s->p.conf_thresh_high) hi[nhi++] = d;
        if (s->p.conf_thresh_low <= c && c < s->p.conf_thresh_high) med[nmed++] = d;
        if (c < s->p.conf_thresh_low) lo[nlo++] = d;
    }
    *nm = 0;
    int *aut = (int *)malloc(sizeof(int) * cap), naut = nconf;
    memcpy(aut, conf_t, sizeof(int) * nconf);
    *naud = D;
    for (int d = 0; d < D; d++) aud[d] = d;
    int *tmp = (int *)malloc(sizeof(int) * cap);
    for (int stage = 1; stage <= 2; stage++) {
        int m0 = *nm;
        if (stage == 1) {
            if (!(nhi && nconf)) continue;
            matching_cascade(s, fr, s->thr * 0.8, conf_t, nconf, hi, nhi, matches, nm);
        } else {
            int nrt = 0, nrm = 0;
            int *rt = tmp, *rm = (int *)malloc(sizeof(int) * cap);
            for (int k = 0; k < naut; k++)
                if (in_list(conf_t, nconf, aut[k])) rt[nrt++] = aut[k];
            for (int k = 0; k < nmed; k++)
                if (in_list(aud, *naud, med[k])) rm[nrm++] = med[k];
            if (nrm && nrt) {
                int *rtc = (int *)malloc(sizeof(int) * (nrt + 1));
                memcpy(rtc, rt, sizeof(int) * nrt);
                matching_cascade(s, fr, s->thr, rtc, nrt, rm, nrm, matches, nm);
                free(rtc);
            }
            free(rm);
        }
        int w = 0;
        for (int k = 0; k < naut; k++) {
            int hit = 0;
            for (int q = m0; q < *nm && !hit; q++) hit = matches[2 * q] == aut[k];
            if (!hit) aut[w++] = aut[k];
        }
        naut = w;
        w = 0;
        for (int k = 0; k < *naud; k++) {
            int hit = 0;
            for (int q = m0; q < *nm && !hit; q++) hit = matches[2 * q + 1] == aud[k];
            if (!hit) aud[w++] = aud[k];
        }
        *naud = w;
    }
    /* stage 3: IoU on unconfirmed + (unmatched with tsu == 1), excluding low-conf detections */
    int *cand = (int *)malloc(sizeof(int) * cap), ncand = 0;
    for (int k = 0; k < nunconf; k++) cand[ncand++] = unconf_t[k];
    for (int k = 0; k < naut; k++)
        if (s->trk[aut[k]]->tsu == 1) cand[ncand++] = aut[k];
    int *rd = (int *)malloc(sizeof(int) * cap), nrd = 0;
    for (int k = 0; k < *naud; k++)
        if (!in_list(lo, nlo, aud[k])) rd[nrd++] = aud[k];
    int *ut3 = (int *)malloc(sizeof(int) * cap), nut3 = 0;
    if (nrd && ncand) {
        const int m0 = *nm;
        int *ud3 = (int *)malloc(sizeof(int) * cap), nud3;
        min_cost_matching(s, fr, METRIC_IOU, s->p.max_iou_dist, cand, ncand, rd, nrd, matches, nm,
                          ut3, &nut3, ud3, &nud3);
        free(ud3);
        int w = 0;
        for (int k = 0; k < naut; k++) {
            int hit = 0;
            for (int q = m0; q < *nm && !hit; q++) hit = matches[2 * q] == aut[k];
            if (!hit) aut[w++] = aut[k];
        }
        naut = w;
        w = 0;
        for (int k = 0; k < *naud; k++) {
            int hit = 0;
            for (int q = m0; q < *nm && !hit; q++) hit = matches[2 * q + 1] == aud[k];
            if (!hit) aud[w++] = aud[k];
        }
        *naud = w;
    }
    *nfut = 0;
    for (int k = 0; k < naut; k++)
        if (!in_list(cand, ncand, aut[k])) fut[(*nfut)++] = aut[k];
    for (int k = 0; k < nut3; k++) fut[(*nfut)++] = ut3[k];
    free(conf_t);
    free(unconf_t);
    free(hi);
    free(med);
    free(lo);
    free(aut);
    free(tmp);
    free(cand);
    free(rd);
    free(ut3);
}

/* _attempt_id_recovery (tracker.py:300-344): returns the recovered detection or -1 */
static int id_recovery(bxo_ss *s, ss_frame *fr, int *ud, int *nud) {
    if (!s->nlost || !*nud) return -1;
    const int F = s->F;
    for (int li = 0; li < s->nlost; li++) {
        ss_track *lt = s->lost[li];
        if (!lt->nfeat) continue;
        const double *tf = lt->feat[lt->nfeat - 1];
        const double tn = wave_norm(tf, F);
        int best = 0;
        double bs = 0.0;
        for (int k = 0; k < *nud; k++) {
            const double *f = fr->d[ud[k]].feat;
            const double sim = wave_dot(f, tf, F) / (np_row_norm(f, F) * tn);
            if (k == 0 || sim > bs) bs = sim, best = k; /* np.argmax: first maximum */
        }
        if (bs > 0.7) {
            const int det = ud[best];
            lt->state = 1; /* "Confirmed state" in the reference's comment, TrackState.Tentative */
            lt->tsu = 0;
            track_update(s, lt, &fr->d[det]);
            if (s->ntrk == s->captrk) {
                s->captrk *= 2;
                s->trk = (ss_track **)realloc(s->trk, sizeof(ss_track *) * s->captrk);
            }
            s->trk[s->ntrk++] = lt;
            memmove(s->lost + li, s->lost + li + 1, sizeof(ss_track *) * (s->nlost - li - 1));
            s->nlost--;
            for (int k = best; k < *nud - 1; k++) ud[k] = ud[k + 1];
            (*nud)--;
            return det;
        }
    }
    return -1;
}

/* detect_crowd_situations (utils/occlusion_handler.py:464-490), OverlapAnalyzer
 * .compute_overlap_matrix (:45-87) — which reads the tlwh boxes it is given as xyxy. */
static int detect_crowd(const bxo_ss *s) {
    const int n = s->ntrk;
    if (n < 3) return 0;
    double (*b)[4] = (double(*)[4])malloc(sizeof(double) * 4 * n);
    for (int i = 0; i < n; i++) to_tlwh(s->trk[i], b[i]);
    long high = 0;
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) {
            const double xx1 = pymax(b[i][0], b[j][0]), yy1 = pymax(b[i][1], b[j][1]);
            const double xx2 = pymin(b[i][2], b[j][2]), yy2 = pymin(b[i][3], b[j][3]);
            const double w = pymax(0, xx2 - xx1), h = pymax(0, yy2 - yy1);
            const double inter = w * h;
            if (inter > 0) {
                const double ai = (b[i][2] - b[i][0]) * (b[i][3] - b[i][1]);
                const double aj = (b[j][2] - b[j][0]) * (b[j][3] - b[j][1]);
                const double m = pymax(inter / ai, inter / aj);
                if (m > 0.3) high += 2;
            }
        }
    free(b);
    const long total = (long)n * (n - 1) / 2;
    return (double)(high / 2) / (double)(total > 1 ? total : 1) > 0.3;
}

/* Tracker.update (tracker.py:125-180); frame_id 0 stands for the None the no-detection branch
 * passes (strongsort.py:156), where len(matching_history) replaces it. */
static void tracker_update(bxo_ss *s, ss_frame *fr, int frame_id) {
    if (!frame_id) frame_id = s->hist_len;
    const int T = s->ntrk, D = fr->nd, cap = 4 * (T + D) + 4;
    int *matches = (int *)malloc(sizeof(int) * 2 * cap), nm = 0;
    int *fut = (int *)malloc(sizeof(int) * cap), nfut = 0;
    int *ud = (int *)malloc(sizeof(int) * cap), nud = 0;
    if (D > 0 || T > 0) enhanced_match(s, fr, matches, &nm, fut, &nfut, ud, &nud);
    for (int q = 0; q < nm; q++) track_update(s, s->trk[matches[2 * q]], &fr->d[matches[2 * q + 1]]);
    for (int q = 0; q < nfut; q++) track_missed(s->trk[fut[q]]);
    id_recovery(s, fr, ud, &nud);
    for (int q = 0; q < nud; q++) { /* _initiate_track */
        if (s->ntrk == s->captrk) {
            s->captrk *= 2;
            s->trk = (ss_track **)realloc(s->trk, sizeof(ss_track *) * s->captrk);
        }
        s->trk[s->ntrk++] = track_new(s, &fr->d[ud[q]], s->next_id++, s->max_age);
    }
    /* deleted tracks -> lost buffer (tracker.py:152-164) */
    int w = 0;
    for (int i = 0; i < s->ntrk; i++) {
        ss_track *t = s->trk[i];
        if (t->state == 3) {
            int kept = 0;
            if (s->nlost < SS_LOST_CAP) {
                t->lost_frame = frame_id;
                s->lost[s->nlost++] = t;
                kept = 1;
            }
            int lw = 0;
            for (int k = 0; k < s->nlost; k++) {
                if (frame_id - s->lost[k]->lost_frame < s->max_age)
                    s->lost[lw++] = s->lost[k];
                else
                    track_free(s->lost[k]);
            }
            s->nlost = lw;
            if (!kept) track_free(t);
        } else {
            s->trk[w++] = t;
        }
    }
    s->ntrk = w;
    /* metric.partial_fit with the confirmed tracks' features (tracker.py:166-178) */
    int nf = 0, na = 0;
    for (int i = 0; i < s->ntrk; i++)
        if (s->trk[i]->state == 2) nf += s->trk[i]->nfeat, na++;
    if (nf) {
        double **fs = (double **)malloc(sizeof(double *) * nf);
        int *tg = (int *)malloc(sizeof(int) * nf), *act = (int *)malloc(sizeof(int) * (na + 1));
        int k = 0, a = 0;
        for (int i = 0; i < s->ntrk; i++) {
            const ss_track *t = s->trk[i];
            if (t->state != 2) continue;
            act[a++] = t->id;
            for (int q = 0; q < t->nfeat; q++) fs[k] = t->feat[q], tg[k++] = t->id;
        }
        partial_fit(s, fs, tg, nf, act, na);
        free(fs);
        free(tg);
        free(act);
    }
    s->hist_len = s->hist_len < 100 ? s->hist_len + 1 : 100;
    free(matches);
    free(fut);
    free(ud);
}

/* ------------------------------------------------------------------------------------------ */
/* OcclusionAwareTracker.update_with_occlusion_handling (utils/occlusion_handler.py:324-339),
 * run after the tracker update when handle_occlusions=True (strongsort.py:150-154, 195-201). */

void bxo_ss_set_occlusion(bxo_ss *s, int on, double threshold) {
    s->occ_on = on;
    s->occ_thr = threshold;
}

/* Iteration order of a CPython (3.10) set of small positive ints after adding `adds` in order:
 * Objects/setobject.c set_add_entry (linear probes of 9, then perturbation; hash(i) = i),
 * growth to 4x used when fill*5 >= mask*3 (set_table_resize + set_insert_clean), iteration in
 * table order.  Returns the number of distinct keys written to out. */
static int pyset_order(const long *adds, int nadd, long *out) {
    size_t mask = 7;
    long *tab = (long *)calloc(8, sizeof(long));
    int fill = 0;
    for (int a = 0; a < nadd; a++) {
        const long key = adds[a];
        size_t perturb = (size_t)key, i = (size_t)key & mask;
        long *e = NULL;
        int dup = 0;
        for (;;) {
            e = &tab[i];
            int probes = (i + 9 <= mask) ? 9 : 0;
            int hit = 0;
            do {
                if (*e == 0) { hit = 1; break; }
                if (*e == key) { hit = 1; dup = 1; break; }
                e++;
            } while (probes--);
            if (hit) break;
            perturb >>= 5;
            i = (i * 5 + 1 + perturb) & mask;
        }
        if (dup) continue;
        *e = key;
        fill++;
        if ((size_t)fill * 5 < mask * 3) continue;
        size_t nsz = 8;
        while (nsz <= (size_t)fill * 4) nsz <<= 1;
        long *nt = (long *)calloc(nsz, sizeof(long));
        const size_t nmask = nsz - 1;
        for (size_t q = 0; q <= mask; q++) {
            if (!tab[q]) continue;
            size_t pp = (size_t)tab[q], j = (size_t)tab[q] & nmask;
            for (;;) {
                long *f = &nt[j];
                if (*f == 0) { *f = tab[q]; break; }
                int done = 0;
                if (j + 9 <= nmask)
                    for (int l = 0; l < 9; l++) {
                        f++;
                        if (*f == 0) { *f = tab[q]; done = 1; break; }
                    }
                if (done) break;
                pp >>= 5;
                j = (j * 5 + 1 + pp) & nmask;
            }
        }
        free(tab);
        tab = nt;
        mask = nmask;
    }
    int m = 0;
    for (size_t q = 0; q <= mask; q++)
        if (tab[q]) out[m++] = tab[q];
    free(tab);
    return m;
}

/* exported for tests/test_oracle.py (checked against CPython's own sets) */
int bxo_pyset_order(const long *adds, int nadd, long *out) { return pyset_order(adds, nadd, out); }

static double occ_vis(const bxo_ss *s, int id) { return id < s->nvis ? s->vis[id] : 1.0; }

static occ_buf *occ_find(bxo_ss *s, int id) {
    for (int b = 0; b < s->nob; b++)
        if (s->ob[b].id == id) return &s->ob[b];
    return NULL;
}

/* Returns 0, or -5 where the reference raises TypeError (_resolve_mutual_occlusion, D7). */
static int occlusion_update(bxo_ss *s) {
    const int n = s->ntrk, F = s->F;
    if (n == 0) return 0;
    double(*b)[4] = (double(*)[4])malloc(sizeof(double) * 4 * n);
    double *area = (double *)malloc(sizeof(double) * n);
    double *ov = (double *)calloc((size_t)n * n, sizeof(double));
    double *sr = (double *)calloc((size_t)n * n, sizeof(double));
    long *adds = (long *)malloc(sizeof(long) * (size_t)n * n);
    int *nadd = (int *)calloc(n, sizeof(int));
    for (int i = 0; i < n; i++) {
        to_tlwh(s->trk[i], b[i]);
        /* the tlwh rows are read as xyxy (compute_overlap_matrix :49-56,
         * analyze_spatial_relationships :109-113) */
        area[i] = (b[i][2] - b[i][0]) * (b[i][3] - b[i][1]);
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) {
            const double xx1 = pymax(b[i][0], b[j][0]), yy1 = pymax(b[i][1], b[j][1]);
            const double xx2 = pymin(b[i][2], b[j][2]), yy2 = pymin(b[i][3], b[j][3]);
            const double inter = pymax(0, xx2 - xx1) * pymax(0, yy2 - yy1);
            if (inter > 0) {
                const double m = pymax(inter / area[i], inter / area[j]);
                ov[(size_t)i * n + j] = ov[(size_t)j * n + i] = m;
            }
            const double r = area[j] > 0 ? area[i] / area[j] : 1.0; /* size_ratio_matrix */
            sr[(size_t)i * n + j] = r;
            sr[(size_t)j * n + i] = 1.0 / r;
        }
    int rc = 0;
    double *vis = (double *)malloc(sizeof(double) * n);
    for (int i = 0; i < n && !rc; i++) { /* update_occlusion_state :163-207 */
        double v = 1.0;
        for (int j = 0; j < n; j++) {
            if (i == j) continue;
            const double o = ov[(size_t)i * n + j];
            if (!(o > s->occ_thr)) continue;
            const double r = sr[(size_t)i * n + j];
            int occluder, occluded;
            if (r > 1.2) occluder = i, occluded = j;
            else if (r < 0.8) occluder = j, occluded = i;
            else { rc = -5; break; } /* MUTUAL: `list(int)` raises TypeError (D7) */
            adds[(size_t)occluded * n + nadd[occluded]++] = s->trk[occluder]->id;
            if (occluded == i) v *= (1.0 - o);
        }
        vis[i] = v;
    }
    if (!rc) {
        for (int i = 0; i < n; i++) { /* track_visibility[track_i] = visibility_score */
            const int id = s->trk[i]->id;
            if (id >= s->nvis) {
                int nn = s->nvis ? s->nvis : 64;
                while (nn <= id) nn *= 2;
                s->vis = (double *)realloc(s->vis, sizeof(double) * nn);
                for (int q = s->nvis; q < nn; q++) s->vis[q] = 1.0;
                s->nvis = nn;
            }
            s->vis[id] = vis[i];
        }
        /* _apply_occlusion_modifications (:341-371), tracks in list order */
        for (int i = 0; i < n; i++) {
            ss_track *t = s->trk[i];
            const double level = 1.0 - occ_vis(s, t->id);
            if (level > 0.3) {
                /* int(track._max_age * 2.0): doubles every occluded frame; held at 2^30 (the
                 * deletion threshold int(max_age * 1.5) then still fits an int and is never
                 * reached) */
                t->max_age = t->max_age >= (1 << 29) ? (1 << 30) : (int)(t->max_age * 2.0);
                if (t->nfeat) {
                    occ_buf *q = occ_find(s, t->id);
                    if (!q) {
                        if (s->nob == s->capob) {
                            s->capob = s->capob ? 2 * s->capob : 16;
                            s->ob = (occ_buf *)realloc(s->ob, sizeof(occ_buf) * s->capob);
                        }
                        q = &s->ob[s->nob++];
                        q->id = t->id;
                        q->n = 0;
                    }
                    if (q->n == 10) { /* deque(maxlen=10) drops the oldest */
                        free(q->f[0]);
                        memmove(q->f, q->f + 1, sizeof(double *) * 9);
                        q->n--;
                    }
                    q->f[q->n++] = vdup(t->feat[t->nfeat - 1], F);
                }
                t->quality = pymax(t->quality, 0.6);
                if (level > 0.8) { /* predict_track_position (:268-305) + :373-392 */
                    long *order = (long *)malloc(sizeof(long) * (nadd[i] + 1));
                    const int k = pyset_order(adds + (size_t)i * n, nadd[i], order);
                    double c0 = 0.0, c1 = 0.0;
                    int kc = 0;
                    for (int q = 0; q < k; q++)
                        for (int j = 0; j < n; j++) {
                            if (j == i || s->trk[j]->id != order[q]) continue;
                            double bb[4];
                            to_tlwh(s->trk[j], bb); /* the current (possibly edited) mean */
                            const double cx = (bb[0] + bb[2]) / 2, cy = (bb[1] + bb[3]) / 2;
                            c0 = kc ? c0 + cx : cx;
                            c1 = kc ? c1 + cy : cy;
                            kc++;
                        }
                    free(order);
                    if (kc) {
                        const double px = c0 / kc - 50 / 2.0, py = c1 / kc - 100 / 2.0;
                        const double pw = 50.0, ph = 100.0;
                        t->mean[0] = px + pw / 2;
                        t->mean[1] = py + ph / 2;
                        t->mean[2] = pw / ph;
                        t->mean[3] = ph;
                        for (int r = 0; r < 4; r++)
                            for (int c = 0; c < 4; c++) t->cov[8 * r + c] *= 1.5;
                    }
                }
            } else {
                occ_buf *q = occ_find(s, t->id);
                if (q) { /* _handle_emerging_track (:394-417) */
                    t->conf = pymin(t->conf + 0.1, 1.0);
                    if (q->n && t->nfeat) {
                        int best = 0;
                        double bn = wave_norm(q->f[0], F);
                        for (int k = 1; k < q->n; k++) {
                            const double v = wave_norm(q->f[k], F);
                            if (v > bn) bn = v, best = k;
                        }
                        double *cur = t->feat[t->nfeat - 1];
                        double *bl = (double *)malloc(sizeof(double) * F);
                        for (int k = 0; k < F; k++) bl[k] = 0.7 * cur[k] + 0.3 * q->f[best][k];
                        const double nb = wave_norm(bl, F) + 1e-8;
                        for (int k = 0; k < F; k++) bl[k] /= nb;
                        free(cur);
                        t->feat[t->nfeat - 1] = bl;
                    }
                    for (int k = 0; k < q->n; k++) free(q->f[k]);
                    *q = s->ob[--s->nob]; /* del self.occlusion_buffer[track.id] */
                }
            }
        }
    }
    free(vis);
    free(b);
    free(area);
    free(ov);
    free(sr);
    free(adds);
    free(nadd);
    return rc;
}

static int format_outputs(const bxo_ss *s, double *out, int cap) {
    int m = 0;
    for (int i = 0; i < s->ntrk; i++) {
        const ss_track *t = s->trk[i];
        if (t->state != 2 || t->tsu >= 1) continue;
        if (m >= cap) return -2;
        double b[4];
        to_tlbr(t, b);
        double *o = out + 10 * m++;
        o[0] = b[0], o[1] = b[1], o[2] = b[2], o[3] = b[3];
        o[4] = t->id, o[5] = t->conf, o[6] = t->cls, o[7] = t->det_ind;
        /* occlusion level (strongsort.py:345-348): 0 unless handle_occlusions */
        o[8] = t->quality, o[9] = s->occ_on ? 1.0 - occ_vis(s, t->id) : 0.0;
    }
    return m;
}

/* StrongSort.update (strongsort.py:120-181) */
int bxo_ss_update(bxo_ss *s, const double *dets, int n, const double *embs, int F,
                  const double *warp, double *out, int out_cap) {
    static const double eye23[6] = {1, 0, 0, 0, 1, 0};
    if (embs && s->F && F != s->F) return -3;
    if (embs) s->F = F;
    s->frame_count++;
    ss_frame fr = {0};
    fr.d = (ss_det *)calloc(n > 0 ? n : 1, sizeof(ss_det));
    fr.dn = (double **)calloc(n > 0 ? n : 1, sizeof(double *));
    for (int i = 0; i < n; i++) {
        const double *r = dets + 6 * i;
        if (!(r[4] >= s->p.min_conf)) continue;
        if (!embs) { /* the reference extracts ReID features from the image here */
            free(fr.d);
            free(fr.dn);
            return -4;
        }
        ss_det *d = &fr.d[fr.nd++];
        d->tlwh[0] = r[0], d->tlwh[1] = r[1], d->tlwh[2] = r[2] - r[0], d->tlwh[3] = r[3] - r[1];
        d->conf = r[4], d->cls = r[5], d->det_ind = i;
        d->feat = vdup(embs + (size_t)i * F, F);
    }
    if (fr.nd == 0) {
        for (int i = 0; i < s->ntrk; i++) track_predict(s->trk[i]);
        tracker_update(s, &fr, 0);
    } else {
        if (s->p.crowd_detection) {
            s->crowd_mode = detect_crowd(s);
            if (s->crowd_mode) { /* _adjust_for_crowd_mode (strongsort.py:183-208) */
                if (!s->orig_stored) {
                    s->orig_max_age = s->max_age;
                    s->orig_thr = s->thr;
                    s->orig_budget = s->budget;
                    s->orig_stored = 1;
                }
                s->max_age = (int)(s->orig_max_age * 1.5);
                s->thr = s->orig_thr * 0.8;
                if (s->budget) s->budget = s->orig_budget * 2 < 300 ? s->orig_budget * 2 : 300;
            }
        }
        if (s->ntrk >= 1)
            for (int i = 0; i < s->ntrk; i++) track_camera(s->trk[i], warp ? warp : eye23);
        for (int k = 0; k < fr.nd; k++) { /* _compute_detection_quality (strongsort.py:285-311) */
            ss_det *d = &fr.d[k];
            double q = d->conf;
            const double fn = wave_norm(d->feat, F);
            q = 0.7 * q + 0.3 * pymin(fn / 10.0, 1.0);
            const double w = d->tlwh[2], h = d->tlwh[3];
            if (h > 0) {
                const double aq = pymax(0.1, 1.0 - fabs(w / h - 0.5) / 2.0);
                q = 0.9 * q + 0.1 * aq;
            }
            if (s->crowd_mode) q += pymin(w * h / 10000.0, 0.1);
            d->quality = q;
        }
        for (int x = 1; x < fr.nd; x++) { /* detections.sort(quality, reverse=True): stable */
            ss_det v = fr.d[x];
            int y = x - 1;
            while (y >= 0 && fr.d[y].quality < v.quality) {
                fr.d[y + 1] = fr.d[y];
                y--;
            }
            fr.d[y + 1] = v;
        }
        for (int k = 0; k < fr.nd; k++) {
            const double den = np_row_norm(fr.d[k].feat, F) + 1e-8;
            fr.dn[k] = (double *)malloc(sizeof(double) * F);
            for (int q = 0; q < F; q++) fr.dn[k][q] = fr.d[k].feat[q] / den;
        }
        for (int i = 0; i < s->ntrk; i++) track_predict(s->trk[i]);
        tracker_update(s, &fr, s->frame_count);
    }
    const int occ = s->occ_on ? occlusion_update(s) : 0;
    const int m = occ ? occ : format_outputs(s, out, out_cap);
    for (int k = 0; k < fr.nd; k++) {
        free(fr.d[k].feat);
        free(fr.dn[k]);
    }
    free(fr.d);
    free(fr.dn);
    return m;
}
