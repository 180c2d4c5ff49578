/*
 * OCSort per-frame update (trackers/ocsort/ocsort.py:195-439) with its XYSR Kalman filter
 * (motion/kalman_filters/aabb/xysr_kf.py:48-291) and association
 * (utils/association.py:10-20 speed_direction_batch, :377-536 enhanced_associate,
 * :105-114 legacy linear_assignment), restated in plain C (fp64).
 *
 * TEST INFRASTRUCTURE ONLY (see bxo.h).  The fork's OCSort path does not run as shipped
 * (SURVEY.md Appendix A, D1-D4); this follows it with the minimal patches P1-P5 that
 * tests/golden/make_golden.py applies when capturing the golden vectors:
 *   P1 xyxy2xysr = upstream semantics (centre, s = w*h, r = w/(h+1e-6)),
 *   P2 valid_mask repeated to (T, D), P3/P4 unmatched lists derived from the matches, the LAP
 *   branch = legacy linear_assignment(-total_cost) (lapx extend_cost, zero padding, no limit),
 *   P5 unmatched lists stay lists (rejected matches appended in match order).
 *
 * Fixed orders where the reference's is not pinned (documented, mirrored bit-for-bit by the
 * HIP engine): np.linalg.inv = LU with partial pivoting + triangular solves in reference
 * LAPACK/BLAS order (dgetf2/dgetrs/dtrsm); dot/matmul = sequential sums in index order, no
 * FMA; np.arccos = fdlibm's acos (<= 1 ulp from glibc's).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bxo.h"
#include "bxo_internal.h"

/* ------------------------------------------------------------------------------------------ */
/* fdlibm e_acos.c (public-domain algorithm): the engine restates the same operations.        */
static const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
                    pi_c = 3.14159265358979311600e+00, pS0 = 1.66666666666666657415e-01,
                    pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01,
                    pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04,
                    pS5 = 3.47933107596021167570e-05, qS1 = -2.40339491173441421878e+00,
                    qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01,
                    qS4 = 7.70381505559019352791e-02;

double bxo_acos(double x) {
    int64_t bits;
    memcpy(&bits, &x, 8);
    const int32_t hx = (int32_t)(bits >> 32);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (x == 1.0) return 0.0;
        if (x == -1.0) return pi_c + 2.0 * pio2_lo;
        return NAN;
    }
    if (ix < 0x3fe00000) {
        if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
        const double z = x * x;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    } else if (hx < 0) {
        const double z = (1.0 + x) * 0.5;
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double s = sqrt(z);
        const double r = p / q;
        const double w = r * s - pio2_lo;
        return pi_c - 2.0 * (s + w);
    } else {
        const double z = (1.0 - x) * 0.5;
        const double s = sqrt(z);
        int64_t sb;
        memcpy(&sb, &s, 8);
        sb &= (int64_t)0xffffffff00000000ULL;
        double df;
        memcpy(&df, &sb, 8);
        const double c = (z - df * df) / (s + df);
        const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const double r = p / q;
        const double w = r * s + c;
        return 2.0 * (df + w);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* XYSR Kalman filter, dim_x = 7, dim_z = 4 (xysr_kf.py; matrices set at ocsort.py:83-111).   */
#define HIST_CAP 64 /* >= max_obs (deque maxlen) */

typedef struct {
    double x[7], P[49];
} kf_state;

typedef struct {
    kf_state s;
    /* history_obs deque(maxlen = max_obs): entries are xysr boxes or None */
    double hbox[HIST_CAP][4];
    unsigned char hnone[HIST_CAP];
    int hlen;
    int observed;
    /* freeze() snapshot (attr_saved): the state, the history and `observed` at that time */
    int has_saved;
    kf_state saved;
    double sbox[HIST_CAP][4];
    unsigned char snone[HIST_CAP];
    int slen, sobserved;
} kf_xysr;

typedef struct {
    double q_xy, q_s;
    int max_obs;
} kf_params;

static void hist_push(double (*box)[4], unsigned char *none, int *len, int maxlen,
                      const double *z) {
    if (*len == maxlen) { /* deque(maxlen) drops from the left */
        memmove(box[0], box[1], sizeof(double) * 4 * (maxlen - 1));
        memmove(none, none + 1, maxlen - 1);
        (*len)--;
    }
    if (z) {
        memcpy(box[*len], z, sizeof(double) * 4);
        none[*len] = 0;
    } else {
        none[*len] = 1;
    }
    (*len)++;
}

static void kf_predict7(const kf_params *kp, kf_state *s) {
    /* x = F x ; P = 1.0 * (F P F') + Q  — F = I + (e_i, e_{i+4}) for i < 3 (two non-zero
     * terms per row/column, so every entry is order-independent) */
    for (int i = 0; i < 3; i++) s->x[i] = s->x[i] + s->x[i + 4];
    double FP[49];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++)
            FP[i * 7 + j] = i < 3 ? s->P[i * 7 + j] + s->P[(i + 4) * 7 + j] : s->P[i * 7 + j];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            double m = j < 3 ? FP[i * 7 + j] + FP[i * 7 + j + 4] : FP[i * 7 + j];
            double q = 0.0;
            if (i == j) q = (i == 4 || i == 5) ? kp->q_xy : (i == 6 ? kp->q_s : 1.0);
            s->P[i * 7 + j] = 1.0 * m + q;
        }
}

/* np.linalg.inv of a 4x4 (dgesv on the identity): dgetf2 LU with partial pivoting, then dgetrs
 * (dlaswp, unit-lower and upper dtrsm in reference BLAS order) */
static void inv4(const double *A_in, double *X) {
    double A[16];
    int piv[4];
    memcpy(A, A_in, sizeof(A));
    for (int k = 0; k < 4; k++) {
        int p = k;
        double mx = fabs(A[k * 4 + k]);
        for (int i = k + 1; i < 4; i++)
            if (fabs(A[i * 4 + k]) > mx) mx = fabs(A[i * 4 + k]), p = i;
        piv[k] = p;
        if (p != k)
            for (int j = 0; j < 4; j++) {
                double t = A[k * 4 + j];
                A[k * 4 + j] = A[p * 4 + j];
                A[p * 4 + j] = t;
            }
        if (A[k * 4 + k] != 0.0) {
            if (fabs(A[k * 4 + k]) >= DBL_MIN) {
                const double r = 1.0 / A[k * 4 + k];
                for (int i = k + 1; i < 4; i++) A[i * 4 + k] *= r;
            } else {
                for (int i = k + 1; i < 4; i++) A[i * 4 + k] /= A[k * 4 + k];
            }
        }
        for (int j = k + 1; j < 4; j++) {
            const double t = -A[k * 4 + j];
            for (int i = k + 1; i < 4; i++) A[i * 4 + j] = A[i * 4 + j] + A[i * 4 + k] * t;
        }
    }
    double B[16];
    for (int i = 0; i < 16; i++) B[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int k = 0; k < 4; k++)
        if (piv[k] != k)
            for (int j = 0; j < 4; j++) {
                double t = B[k * 4 + j];
                B[k * 4 + j] = B[piv[k] * 4 + j];
                B[piv[k] * 4 + j] = t;
            }
    for (int j = 0; j < 4; j++) {
        for (int k = 0; k < 4; k++)
            if (B[k * 4 + j] != 0.0)
                for (int i = k + 1; i < 4; i++) B[i * 4 + j] -= B[k * 4 + j] * A[i * 4 + k];
        for (int k = 3; k >= 0; k--)
            if (B[k * 4 + j] != 0.0) {
                B[k * 4 + j] /= A[k * 4 + k];
                for (int i = 0; i < k; i++) B[i * 4 + j] -= B[k * 4 + j] * A[i * 4 + k];
            }
    }
    memcpy(X, B, sizeof(B));
}

/* KF update with a measurement (xysr_kf.py:256-283, R = diag(1,1,10,10), H = [I4 0]) */
static void kf_update7_core(kf_state *s, const double *z) {
    static const double Rd[4] = {1.0, 1.0, 10.0, 10.0};
    double y[4], S[16], SI[16], K[28];
    for (int k = 0; k < 4; k++) y[k] = z[k] - s->x[k];
    for (int a = 0; a < 4; a++)
        for (int b = 0; b < 4; b++) S[a * 4 + b] = s->P[a * 7 + b] + (a == b ? Rd[a] : 0.0);
    inv4(S, SI);
    for (int i = 0; i < 7; i++)
        for (int b = 0; b < 4; b++) {
            double acc = 0.0;
            for (int a = 0; a < 4; a++) acc += s->P[i * 7 + a] * SI[a * 4 + b];
            K[i * 4 + b] = acc;
        }
    for (int i = 0; i < 7; i++) {
        double acc = 0.0;
        for (int b = 0; b < 4; b++) acc += K[i * 4 + b] * y[b];
        s->x[i] = s->x[i] + acc;
    }
    double IKH[49], A[49], Bm[49];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) IKH[i * 7 + j] = (i == j ? 1.0 : 0.0) - (j < 4 ? K[i * 4 + j] : 0.0);
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            double acc = 0.0;
            for (int k = 0; k < 7; k++) acc += IKH[i * 7 + k] * s->P[k * 7 + j];
            A[i * 7 + j] = acc;
        }
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            double acc = 0.0;
            for (int k = 0; k < 7; k++) acc += A[i * 7 + k] * IKH[j * 7 + k];
            Bm[i * 7 + j] = acc;
        }
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) {
            double acc = 0.0;
            for (int b = 0; b < 4; b++) acc += (K[i * 4 + b] * Rd[b]) * K[j * 4 + b];
            s->P[i * 7 + j] = Bm[i * 7 + j] + acc;
        }
}

static void kf_freeze(kf_xysr *k) {
    k->has_saved = 1;
    k->saved = k->s;
    memcpy(k->sbox, k->hbox, sizeof(k->hbox));
    memcpy(k->snone, k->hnone, sizeof(k->hnone));
    k->slen = k->hlen;
    k->sobserved = k->observed;
}

static void kf_update7(const kf_params *kp, kf_xysr *k, const double *z);

/* xysr_kf.py:183-209 — restore the frozen state and re-run the virtual trajectory between the
 * last two observations (linear interpolation in (x, y, w, h)). */
static void kf_unfreeze(const kf_params *kp, kf_xysr *k) {
    if (!k->has_saved) return;
    /* new_history = the current history (ends with the new observation) */
    int i2 = -1, i1 = -1;
    for (int i = k->hlen - 1; i >= 0; i--)
        if (!k->hnone[i]) {
            if (i2 < 0) i2 = i;
            else { i1 = i; break; }
        }
    double box1[4], box2[4];
    memcpy(box1, k->hbox[i1 < 0 ? 0 : i1], sizeof(box1));
    memcpy(box2, k->hbox[i2 < 0 ? 0 : i2], sizeof(box2));
    /* self.__dict__ = self.attr_saved */
    k->s = k->saved;
    memcpy(k->hbox, k->sbox, sizeof(k->hbox));
    memcpy(k->hnone, k->snone, sizeof(k->hnone));
    k->hlen = k->slen;
    k->observed = k->sobserved;
    k->has_saved = 0; /* the restored attr_saved is an older snapshot never used again */
    if (k->hlen > 0) k->hlen--; /* deque(list(history)[:-1]) */
    if (i1 < 0 || i2 < 0) return; /* (the reference would raise IndexError here) */
    const double x1 = box1[0], y1 = box1[1], s1 = box1[2], r1 = box1[3];
    const double w1 = sqrt(s1 * r1), h1 = sqrt(s1 / r1);
    const double x2 = box2[0], y2 = box2[1], s2 = box2[2], r2 = box2[3];
    const double w2 = sqrt(s2 * r2), h2 = sqrt(s2 / r2);
    const int time_gap = i2 - i1;
    const double dx = (x2 - x1) / time_gap, dy = (y2 - y1) / time_gap;
    const double dw = (w2 - w1) / time_gap, dh = (h2 - h1) / time_gap;
    for (int i = 0; i < time_gap; i++) {
        const double x = x1 + (i + 1) * dx, y = y1 + (i + 1) * dy;
        const double w = w1 + (i + 1) * dw, h = h1 + (i + 1) * dh;
        const double nb[4] = {x, y, w * h, w / (double)h};
        kf_update7(kp, k, nb);
        if (i != time_gap - 1) {
            kf_predict7(kp, &k->s);
            if (k->hlen > 0) k->hlen--; /* history_obs.pop() */
        }
    }
    if (k->hlen > 0) k->hlen--;
}

/* xysr_kf.py:211-291 (z = NULL: the None branch) */
static void kf_update7(const kf_params *kp, kf_xysr *k, const double *z) {
    hist_push(k->hbox, k->hnone, &k->hlen, kp->max_obs, z);
    if (!z) {
        if (k->observed) kf_freeze(k); /* last_measurement is unused on this path */
        k->observed = 0;
        return;
    }
    if (!k->observed) kf_unfreeze(kp, k);
    k->observed = 1;
    kf_update7_core(&k->s, z);
    hist_push(k->hbox, k->hnone, &k->hlen, kp->max_obs, z);
}

/* ------------------------------------------------------------------------------------------ */
/* KalmanBoxTracker (ocsort.py:56-192)                                                         */
#define OBS_KEEP 8

typedef struct {
    kf_xysr kf;
    int id, time_since_update, hits, hit_streak, age, det_ind;
    double conf, cls;
    double last_obs[5];            /* [-1]*5 placeholder until the first update */
    int obs_age[OBS_KEEP];         /* the most recent entries of the observations dict */
    double obs_box[OBS_KEEP][5];
    int n_obs;
    int has_vel;
    double vel[2];
} ocs_track;

struct bxo_ocsort {
    double min_conf, det_thresh, asso_threshold, inertia;
    int max_age, min_hits, delta_t, use_byte;
    kf_params kp;
    int frame_count, id_count;
    int asso_kind;       /* BXO_ASSO_* (BaseTracker asso_func, basetracker.py:140-147) */
    double fw, fh;       /* frame size latched from the first image (centroid) */
    ocs_track *tr;
    int ntr, cap;
};

/* ops.xyxy2xysr (P1, upstream semantics) */
static void xyxy2xysr(const double *b, double *z) {
    const double w = b[2] - b[0], h = b[3] - b[1];
    z[0] = b[0] + w / 2.0;
    z[1] = b[1] + h / 2.0;
    z[2] = w * h;
    z[3] = w / (h + 1e-6);
}

/* Op-level entries (mirrors of bx_kf_xysr_*): KalmanBoxTracker's filter without the tracker's
 * history/ORU bookkeeping.  initiate = ocsort.py:83-111 (P = eye; P[4:,4:] *= 1000; P *= 10;
 * x[:4] = xyxy2xysr(bbox)); predict = ocsort.py:177-180 (the s + ds <= 0 clamp, then
 * xysr_kf.py:137-175 with Q[4:6,4:6] *= q_xy, Q[-1,-1] *= q_s); update = xysr_kf.py:256-283. */
void bxo_kf_xysr_initiate(int n, const double *bbox, double *x, double *P) {
    for (int k = 0; k < n; k++) {
        double *xk = x + 7 * k, *Pk = P + 49 * k;
        memset(xk, 0, sizeof(double) * 7);
        memset(Pk, 0, sizeof(double) * 49);
        xyxy2xysr(bbox + 4 * k, xk);
        for (int i = 0; i < 7; i++) Pk[8 * i] = i < 4 ? 10.0 : 10000.0;
    }
}

void bxo_kf_xysr_predict(int n, double *x, double *P, double q_xy, double q_s) {
    const kf_params kp = {q_xy, q_s, 50};
    for (int k = 0; k < n; k++) {
        kf_state s;
        memcpy(s.x, x + 7 * k, sizeof s.x);
        memcpy(s.P, P + 49 * k, sizeof s.P);
        if (s.x[6] + s.x[2] <= 0) s.x[6] *= 0.0;
        kf_predict7(&kp, &s);
        memcpy(x + 7 * k, s.x, sizeof s.x);
        memcpy(P + 49 * k, s.P, sizeof s.P);
    }
}

void bxo_kf_xysr_update(int n, double *x, double *P, const double *z) {
    for (int k = 0; k < n; k++) {
        kf_state s;
        memcpy(s.x, x + 7 * k, sizeof s.x);
        memcpy(s.P, P + 49 * k, sizeof s.P);
        kf_update7_core(&s, z + 4 * k);
        memcpy(x + 7 * k, s.x, sizeof s.x);
        memcpy(P + 49 * k, s.P, sizeof s.P);
    }
}

/* ocsort.py:31-45 convert_x_to_bbox */
static void x_to_bbox(const double *x, double *b) {
    const double w = sqrt(x[2] * x[3]);
    const double h = x[2] / w;
    b[0] = x[0] - w / 2.0;
    b[1] = x[1] - h / 2.0;
    b[2] = x[0] + w / 2.0;
    b[3] = x[1] + h / 2.0;
}

/* ocsort.py:48-53 speed_direction */
static void speed_direction(const double *b1, const double *b2, double *v) {
    const double cx1 = (b1[0] + b1[2]) / 2.0, cy1 = (b1[1] + b1[3]) / 2.0;
    const double cx2 = (b2[0] + b2[2]) / 2.0, cy2 = (b2[1] + b2[3]) / 2.0;
    const double sy = cy2 - cy1, sx = cx2 - cx1;
    const double norm = sqrt((cy2 - cy1) * (cy2 - cy1) + (cx2 - cx1) * (cx2 - cx1)) + 1e-6;
    v[0] = sy / norm;
    v[1] = sx / norm;
}

static const double *obs_at(const ocs_track *t, int age) {
    for (int q = 0; q < t->n_obs; q++)
        if (t->obs_age[q] == age) return t->obs_box[q];
    return NULL;
}

/* ocsort.py:17-28 k_previous_obs */
static void k_previous_obs(const ocs_track *t, int k, double *out) {
    if (t->n_obs == 0) {
        for (int q = 0; q < 5; q++) out[q] = -1.0;
        return;
    }
    for (int i = 0; i < k; i++) {
        const double *o = obs_at(t, t->age - (k - i));
        if (o) { memcpy(out, o, sizeof(double) * 5); return; }
    }
    memcpy(out, t->obs_box[t->n_obs - 1], sizeof(double) * 5); /* max(observations.keys()) */
}

static void track_init(const struct bxo_ocsort *o, ocs_track *t, const double *bbox5, double cls,
                       int det_ind, int id) {
    memset(t, 0, sizeof(*t));
    t->det_ind = det_ind;
    for (int i = 0; i < 49; i++) t->kf.s.P[i] = 0.0;
    const double pd[7] = {10.0, 10.0, 10.0, 10.0, 10000.0, 10000.0, 10000.0};
    for (int i = 0; i < 7; i++) t->kf.s.P[i * 8] = pd[i];
    double z[4];
    xyxy2xysr(bbox5, z);
    for (int i = 0; i < 4; i++) t->kf.s.x[i] = z[i];
    t->kf.observed = 0;
    t->id = id;
    t->conf = bbox5[4];
    t->cls = cls;
    for (int q = 0; q < 5; q++) t->last_obs[q] = -1.0;
    (void)o;
}

static double sum5(const double *b) { return (((b[0] + b[1]) + b[2]) + b[3]) + b[4]; }

/* ocsort.py:136-171 */
static void track_update(const struct bxo_ocsort *o, ocs_track *t, const double *bbox5,
                         double cls, int det_ind) {
    t->det_ind = det_ind;
    if (bbox5) {
        t->conf = bbox5[4];
        t->cls = cls;
        if (sum5(t->last_obs) >= 0) {
            const double *prev = NULL;
            for (int i = 0; i < o->delta_t && !prev; i++) prev = obs_at(t, t->age - (o->delta_t - i));
            if (!prev) prev = t->last_obs;
            speed_direction(prev, bbox5, t->vel);
            t->has_vel = 1;
        }
        memcpy(t->last_obs, bbox5, sizeof(double) * 5);
        /* observations[age] = bbox (ages only grow, so the newest entry is appended/replaced) */
        if (t->n_obs > 0 && t->obs_age[t->n_obs - 1] == t->age) {
            memcpy(t->obs_box[t->n_obs - 1], bbox5, sizeof(double) * 5);
        } else {
            if (t->n_obs == OBS_KEEP) {
                memmove(t->obs_age, t->obs_age + 1, sizeof(int) * (OBS_KEEP - 1));
                memmove(t->obs_box, t->obs_box + 1, sizeof(double) * 5 * (OBS_KEEP - 1));
                t->n_obs--;
            }
            t->obs_age[t->n_obs] = t->age;
            memcpy(t->obs_box[t->n_obs], bbox5, sizeof(double) * 5);
            t->n_obs++;
        }
        t->time_since_update = 0;
        t->hits++;
        t->hit_streak++;
        double z[4];
        xyxy2xysr(bbox5, z);
        kf_update7(&o->kp, &t->kf, z);
    } else {
        kf_update7(&o->kp, &t->kf, NULL);
    }
}

/* ocsort.py:173-186 — returns the predicted box */
static void track_predict(const struct bxo_ocsort *o, ocs_track *t, double *box) {
    if ((t->kf.s.x[6] + t->kf.s.x[2]) <= 0) t->kf.s.x[6] *= 0.0;
    kf_predict7(&o->kp, &t->kf.s);
    t->age++;
    if (t->time_since_update > 0) t->hit_streak = 0;
    t->time_since_update++;
    x_to_bbox(t->kf.s.x, box);
}

/* ------------------------------------------------------------------------------------------ */
/* legacy linear_assignment (association.py:105-114): lapx lapjv(cost, extend_cost=True), zero
 * padding to a square max(nr, nc); returns (row, col) pairs in row order. */
static int legacy_lap(const double *cost, int nr, int nc, int *pairs) {
    const int n = nr > nc ? nr : nc;
    if (n == 0) return 0;
    double *E = (double *)calloc((size_t)n * n, sizeof(double));
    int *x = (int *)malloc(sizeof(int) * n), *y = (int *)malloc(sizeof(int) * n);
    for (int i = 0; i < nr; i++)
        for (int j = 0; j < nc; j++) E[(size_t)i * n + j] = cost[(size_t)i * nc + j];
    bxo_lapjv(n, E, x, y);
    int np_ = 0;
    for (int i = 0; i < nr; i++) {
        const int j = x[i];
        if (j >= 0 && j < nc) {
            pairs[2 * np_] = y[j]; /* [y[i], i] for i in x: y[j] == i */
            pairs[2 * np_ + 1] = j;
            np_++;
        }
    }
    free(E);
    free(x);
    free(y);
    return np_;
}

/* enhanced_associate (patched, association.py:377-536): dets[nd][5], trks[nt][5],
 * velocities[nt][2], prev_obs[nt][5].  Outputs matches (det, trk) and the two unmatched lists
 * in the reference's order. */
static void associate(int kind, double fw, double fh, const double *dets, int nd,
                      const double *trks, int nt, double thr,
                      const double *vel, const double *prev, double vdc_weight, int *matches,
                      int *nm, int *ud, int *nud, int *ut, int *nut) {
    *nm = *nud = *nut = 0;
    if (nt == 0) {
        for (int d = 0; d < nd; d++) ud[(*nud)++] = d;
        return;
    }
    double *iou = (double *)malloc(sizeof(double) * (size_t)(nd ? nd : 1) * nt);
    double *total = (double *)malloc(sizeof(double) * (size_t)(nd ? nd : 1) * nt);
    for (int d = 0; d < nd; d++)
        for (int t = 0; t < nt; t++) {
            const double *a = dets + 5 * d, *b = trks + 5 * t;
            /* self.asso_func (utils/iou.py:50-307; iou by default) */
            iou[(size_t)d * nt + t] = bxo_pair_cost(kind, a, b, fw, fh);
            /* speed_direction_batch (association.py:10-20) with the track's k-previous obs */
            const double *p = prev + 5 * t;
            const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
            const double cx2 = (p[0] + p[2]) / 2.0, cy2 = (p[1] + p[3]) / 2.0;
            double dx = cx1 - cx2, dy = cy1 - cy2;
            const double norm = sqrt(dx * dx + dy * dy) + 1e-6;
            dx = dx / norm;
            dy = dy / norm;
            double c = vel[2 * t + 1] * dx + vel[2 * t] * dy; /* inertia_X * X + inertia_Y * Y */
            c = c < -1 ? -1 : (c > 1 ? 1 : c);
            double ang = bxo_acos(c);
            ang = (M_PI / 2.0 - fabs(ang)) / M_PI;
            const double valid = p[4] < 0 ? 0.0 : 1.0;
            const double mc = (valid * ang) * vdc_weight;
            total[(size_t)d * nt + t] = iou[(size_t)d * nt + t] + mc;
        }
    int *mi = (int *)malloc(sizeof(int) * 2 * (size_t)(nd < nt ? (nd ? nd : 1) : nt));
    int nmi = 0;
    if (nd > 0) {
        int *rs = (int *)calloc(nd, sizeof(int)), *cs = (int *)calloc(nt, sizeof(int));
        int mr = 0, mc = 0;
        for (int d = 0; d < nd; d++)
            for (int t = 0; t < nt; t++)
                if (iou[(size_t)d * nt + t] > thr) { rs[d]++; cs[t]++; }
        for (int d = 0; d < nd; d++) mr = rs[d] > mr ? rs[d] : mr;
        for (int t = 0; t < nt; t++) mc = cs[t] > mc ? cs[t] : mc;
        if (mr == 1 && mc == 1) { /* one-to-one fast path: np.stack(np.where(a), 1) */
            for (int d = 0; d < nd; d++)
                for (int t = 0; t < nt; t++)
                    if (iou[(size_t)d * nt + t] > thr) {
                        mi[2 * nmi] = d;
                        mi[2 * nmi + 1] = t;
                        nmi++;
                    }
        } else { /* P4: legacy linear_assignment(-total_cost) */
            double *neg = (double *)malloc(sizeof(double) * (size_t)nd * nt);
            for (size_t q = 0; q < (size_t)nd * nt; q++) neg[q] = -total[q];
            nmi = legacy_lap(neg, nd, nt, mi);
            free(neg);
        }
        free(rs);
        free(cs);
    }
    /* P3/P4: unmatched = those absent from the matches, ascending */
    for (int d = 0; d < nd; d++) {
        int f = 0;
        for (int q = 0; q < nmi; q++) f |= mi[2 * q] == d;
        if (!f) ud[(*nud)++] = d;
    }
    for (int t = 0; t < nt; t++) {
        int f = 0;
        for (int q = 0; q < nmi; q++) f |= mi[2 * q + 1] == t;
        if (!f) ut[(*nut)++] = t;
    }
    /* IoU validation; P5: rejected pairs are appended to the unmatched lists in match order */
    for (int q = 0; q < nmi; q++) {
        const int d = mi[2 * q], t = mi[2 * q + 1];
        if (iou[(size_t)d * nt + t] >= thr) {
            matches[2 * *nm] = d;
            matches[2 * *nm + 1] = t;
            (*nm)++;
        } else {
            ud[(*nud)++] = d;
            ut[(*nut)++] = t;
        }
    }
    free(mi);
    free(iou);
    free(total);
}

static int cmp_int(const void *a, const void *b) {
    const int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

/* np.setdiff1d(a, b): sorted unique values of a not in b */
static int setdiff1d(int *a, int na, const int *b, int nb) {
    qsort(a, na, sizeof(int), cmp_int);
    int n = 0;
    for (int i = 0; i < na; i++) {
        if (i > 0 && a[i] == a[i - 1]) continue;
        int f = 0;
        for (int k = 0; k < nb; k++) f |= b[k] == a[i];
        if (!f) a[n++] = a[i];
    }
    return n;
}

/* self.asso_func of two small sets (rows a, cols b), [na][nb] */
static void iou_small(const bxo_ocsort *o, const double *a, int sa, int na, const double *b,
                      int sb, int nb, double *out) {
    for (int i = 0; i < na; i++)
        for (int j = 0; j < nb; j++)
            out[(size_t)i * nb + j] =
                bxo_pair_cost(o->asso_kind, a + (size_t)sa * i, b + (size_t)sb * j, o->fw, o->fh);
}

/* ------------------------------------------------------------------------------------------ */
bxo_ocsort *bxo_ocsort_new(double min_conf, double det_thresh, int max_age, int min_hits,
                           double asso_threshold, int delta_t, double inertia, int use_byte,
                           double q_xy_scaling, double q_s_scaling) {
    bxo_ocsort *o = (bxo_ocsort *)calloc(1, sizeof(bxo_ocsort));
    o->min_conf = min_conf;
    o->det_thresh = det_thresh;
    o->max_age = max_age;
    o->min_hits = min_hits;
    o->asso_threshold = asso_threshold;
    o->delta_t = delta_t;
    o->inertia = inertia;
    o->use_byte = use_byte;
    o->kp.q_xy = 1.0 * q_xy_scaling; /* Q = eye; Q[4:6,4:6] *= q_xy; Q[-1,-1] *= q_s */
    o->kp.q_s = 1.0 * q_s_scaling;
    /* basetracker.py:59-62: max_obs = 50, or max_age + 5 when max_age >= 50 */
    o->kp.max_obs = max_age >= 50 ? max_age + 5 : 50;
    if (o->kp.max_obs > HIST_CAP) o->kp.max_obs = HIST_CAP;
    o->cap = 64;
    o->tr = (ocs_track *)malloc(sizeof(ocs_track) * o->cap);
    return o;
}

/* BaseTracker: asso_func chosen by name, h/w latched from the first image (basetracker.py:140-147) */
void bxo_ocsort_set_asso(bxo_ocsort *o, int kind, double w, double h) {
    o->asso_kind = kind;
    o->fw = w;
    o->fh = h;
}

void bxo_ocsort_free(bxo_ocsort *o) {
    if (!o) return;
    free(o->tr);
    free(o);
}

int bxo_ocsort_id_count(bxo_ocsort *o) { return o->id_count; }
void bxo_ocsort_set_id_count(bxo_ocsort *o, int c) { o->id_count = c; }

/* host edit of trk.kf.x / trk.kf.P by id; returns the number of ids found */
int bxo_ocsort_state_set(bxo_ocsort *o, int n, const int *ids, const double *x, const double *P) {
    int found = 0;
    for (int j = 0; j < n; j++)
        for (int k = 0; k < o->ntr; k++)
            if (o->tr[k].id == ids[j]) {
                if (x) memcpy(o->tr[k].kf.s.x, x + 7 * j, sizeof(double) * 7);
                if (P) memcpy(o->tr[k].kf.s.P, P + 49 * j, sizeof(double) * 49);
                found++;
                break;
            }
    return found;
}

int bxo_ocsort_tracks(bxo_ocsort *o, int cap, int *ids, double *x, double *P) {
    for (int k = 0; k < o->ntr && k < cap; k++) {
        if (ids) ids[k] = o->tr[k].id;
        if (x) memcpy(x + 7 * k, o->tr[k].kf.s.x, sizeof(double) * 7);
        if (P) memcpy(P + 49 * k, o->tr[k].kf.s.P, sizeof(double) * 49);
    }
    return o->ntr;
}

/* dets[n][6] float64 (already float32-rounded, as setup_decorator leaves them) */
int bxo_ocsort_update(bxo_ocsort *o, const double *dets_in, int n, double *out, int out_cap) {
    o->frame_count++;
    /* dets = hstack([dets, arange]) ; splits (ocsort.py:265-275) */
    double *hi = (double *)malloc(sizeof(double) * 7 * (n ? n : 1));
    double *lo = (double *)malloc(sizeof(double) * 7 * (n ? n : 1));
    int nh = 0, nl = 0;
    for (int i = 0; i < n; i++) {
        const double *r = dets_in + 6 * i;
        const double c = r[4];
        double row[7] = {r[0], r[1], r[2], r[3], r[4], r[5], (double)i};
        if (c > o->min_conf && c < o->det_thresh) memcpy(lo + 7 * nl++, row, sizeof(row));
        if (c > o->det_thresh) memcpy(hi + 7 * nh++, row, sizeof(row));
    }
    /* predict every track; drop NaN predictions (ocsort.py:278-288) */
    const int nt0 = o->ntr;
    double *trks = (double *)malloc(sizeof(double) * 5 * (nt0 ? nt0 : 1));
    int nt = 0;
    {
        int w = 0;
        for (int t = 0; t < nt0; t++) {
            double b[4];
            track_predict(o, &o->tr[t], b);
            if (isnan(b[0]) || isnan(b[1]) || isnan(b[2]) || isnan(b[3])) continue;
            if (w != t) o->tr[w] = o->tr[t];
            trks[5 * w] = b[0];
            trks[5 * w + 1] = b[1];
            trks[5 * w + 2] = b[2];
            trks[5 * w + 3] = b[3];
            trks[5 * w + 4] = 0.0;
            w++;
        }
        nt = o->ntr = w;
    }
    double *vel = (double *)malloc(sizeof(double) * 2 * (nt ? nt : 1));
    double *lastb = (double *)malloc(sizeof(double) * 5 * (nt ? nt : 1));
    double *kobs = (double *)malloc(sizeof(double) * 5 * (nt ? nt : 1));
    for (int t = 0; t < nt; t++) {
        const ocs_track *tk = &o->tr[t];
        vel[2 * t] = tk->has_vel ? tk->vel[0] : 0.0;
        vel[2 * t + 1] = tk->has_vel ? tk->vel[1] : 0.0;
        memcpy(lastb + 5 * t, tk->last_obs, sizeof(double) * 5);
        k_previous_obs(tk, o->delta_t, kobs + 5 * t);
    }
    /* first association */
    double *hd5 = (double *)malloc(sizeof(double) * 5 * (nh ? nh : 1));
    for (int d = 0; d < nh; d++) memcpy(hd5 + 5 * d, hi + 7 * d, sizeof(double) * 5);
    const int big = (nh > nt ? nh : nt) + 1;
    int *matches = (int *)malloc(sizeof(int) * 2 * big), *ud = (int *)malloc(sizeof(int) * 2 * big);
    int *ut = (int *)malloc(sizeof(int) * 2 * big);
    int nm, nud, nut;
    associate(o->asso_kind, o->fw, o->fh, hd5, nh, trks, nt, o->asso_threshold, vel, kobs, o->inertia, matches, &nm, ud, &nud,
              ut, &nut);
    for (int q = 0; q < nm; q++) {
        const double *r = hi + 7 * matches[2 * q];
        track_update(o, &o->tr[matches[2 * q + 1]], r, r[5], (int)r[6]);
    }
    /* BYTE round (ocsort.py:330-356) */
    if (o->use_byte && nl > 0 && nut > 0) {
        double *ul = (double *)malloc(sizeof(double) * (size_t)nl * nut);
        double *utb = (double *)malloc(sizeof(double) * 5 * nut);
        for (int k = 0; k < nut; k++) memcpy(utb + 5 * k, trks + 5 * ut[k], sizeof(double) * 5);
        iou_small(o, lo, 7, nl, utb, 5, nut, ul);
        double mx = -INFINITY;
        for (int q = 0; q < nl * nut; q++) mx = ul[q] > mx ? ul[q] : mx;
        if (mx > o->asso_threshold) {
            double *neg = (double *)malloc(sizeof(double) * (size_t)nl * nut);
            for (int q = 0; q < nl * nut; q++) neg[q] = -ul[q];
            int *pr = (int *)malloc(sizeof(int) * 2 * (nl > nut ? nl : nut));
            const int np_ = legacy_lap(neg, nl, nut, pr);
            int *rm = (int *)malloc(sizeof(int) * (np_ + 1));
            int nrm = 0;
            for (int q = 0; q < np_; q++) {
                const int di = pr[2 * q], ti = ut[pr[2 * q + 1]];
                if (ul[(size_t)pr[2 * q] * nut + pr[2 * q + 1]] < o->asso_threshold) continue;
                const double *r = lo + 7 * di;
                track_update(o, &o->tr[ti], r, r[5], (int)r[6]);
                rm[nrm++] = ti;
            }
            nut = setdiff1d(ut, nut, rm, nrm);
            free(neg);
            free(pr);
            free(rm);
        }
        free(ul);
        free(utb);
    }
    /* OCR round on the last observations (ocsort.py:358-386) */
    if (nud > 0 && nut > 0) {
        double *ld = (double *)malloc(sizeof(double) * 5 * nud);
        double *lt = (double *)malloc(sizeof(double) * 5 * nut);
        for (int k = 0; k < nud; k++) memcpy(ld + 5 * k, hi + 7 * ud[k], sizeof(double) * 5);
        for (int k = 0; k < nut; k++) memcpy(lt + 5 * k, lastb + 5 * ut[k], sizeof(double) * 5);
        double *il = (double *)malloc(sizeof(double) * (size_t)nud * nut);
        iou_small(o, ld, 5, nud, lt, 5, nut, il);
        double mx = -INFINITY;
        for (int q = 0; q < nud * nut; q++) mx = il[q] > mx ? il[q] : mx;
        if (mx > o->asso_threshold) {
            double *neg = (double *)malloc(sizeof(double) * (size_t)nud * nut);
            for (int q = 0; q < nud * nut; q++) neg[q] = -il[q];
            int *pr = (int *)malloc(sizeof(int) * 2 * (nud > nut ? nud : nut));
            const int np_ = legacy_lap(neg, nud, nut, pr);
            int *rd = (int *)malloc(sizeof(int) * (np_ + 1)), *rt = (int *)malloc(sizeof(int) * (np_ + 1));
            int nr = 0;
            for (int q = 0; q < np_; q++) {
                const int di = ud[pr[2 * q]], ti = ut[pr[2 * q + 1]];
                if (il[(size_t)pr[2 * q] * nut + pr[2 * q + 1]] < o->asso_threshold) continue;
                const double *r = hi + 7 * di;
                track_update(o, &o->tr[ti], r, r[5], (int)r[6]);
                rd[nr] = di;
                rt[nr] = ti;
                nr++;
            }
            nud = setdiff1d(ud, nud, rd, nr);
            nut = setdiff1d(ut, nut, rt, nr);
            free(neg);
            free(pr);
            free(rd);
            free(rt);
        }
        free(ld);
        free(lt);
        free(il);
    }
    for (int k = 0; k < nut; k++) track_update(o, &o->tr[ut[k]], NULL, 0.0, -1);
    /* new tracks for the unmatched high detections, in list order */
    for (int k = 0; k < nud; k++) {
        if (o->ntr == o->cap) {
            o->cap *= 2;
            o->tr = (ocs_track *)realloc(o->tr, sizeof(ocs_track) * o->cap);
        }
        const double *r = hi + 7 * ud[k];
        track_init(o, &o->tr[o->ntr], r, r[5], (int)r[6], o->id_count++);
        o->ntr++;
    }
    /* outputs (reversed track order) and deletion of dead tracks (ocsort.py:414-436) */
    int m = 0;
    for (int i = o->ntr - 1; i >= 0; i--) {
        ocs_track *t = &o->tr[i];
        double d[4];
        if (sum5(t->last_obs) < 0) {
            x_to_bbox(t->kf.s.x, d);
        } else {
            memcpy(d, t->last_obs, sizeof(d));
        }
        if (t->time_since_update < 1 &&
            (t->hit_streak >= o->min_hits || o->frame_count <= o->min_hits)) {
            if (m < out_cap) {
                double *row = out + 8 * m;
                row[0] = d[0]; row[1] = d[1]; row[2] = d[2]; row[3] = d[3];
                row[4] = (double)(t->id + 1);
                row[5] = t->conf;
                row[6] = t->cls;
                row[7] = (double)t->det_ind;
            }
            m++;
        }
        if (t->time_since_update > o->max_age) {
            memmove(&o->tr[i], &o->tr[i + 1], sizeof(ocs_track) * (o->ntr - i - 1));
            o->ntr--;
        }
    }
    free(hi); free(lo); free(trks); free(vel); free(lastb); free(kobs); free(hd5);
    free(matches); free(ud); free(ut);
    return m <= out_cap ? m : -2;
}
