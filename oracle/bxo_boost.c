/*
 * BoostTrack / BoostTrack++ per-frame update (trackers/boosttrack/boosttrack.py:123-456) with its
 * 8-state Kalman filter (trackers/boosttrack/kalmanfilter.py:8-157) and association
 * (trackers/boosttrack/assoc.py:9-200), restated in plain C (fp64).
 *
 * TEST INFRASTRUCTURE ONLY (see bxo.h).  The reference runs as shipped (no patches).  Pinned by
 * tests/golden/trk_boosttrack_*.npz and boost_ops.npz (tests/test_oracle.py).
 *
 * Fixed orders where the reference's is not pinned (mirrored bit-for-bit by the HIP engine):
 *   - np.exp = fdlibm's exp (<= 1 ulp; numpy's own SIMD exp is not pinned either);
 *   - max_s ** 1.5 = x * sqrt(x) with a compensated (fma) correction: the correctly rounded
 *     value except in rare hard cases (glibc's pow is <= 0.52 ulp);
 *   - Kalman update = cho_factor/cho_solve restated as in bxo_ops.c (LAPACK order unpinned);
 *   - emb_cost = dets_embs @ trk_embs.T (BLAS dgemm) = an ascending-k fma chain per entry —
 *     what the engine's fp64 MFMA computes; np.linalg.norm (BLAS ddot) = the engine's "wave
 *     order" (64 lane-strided partial sums + xor butterfly, as bxo_track.c vnorm).
 * Everything the reference pins (elementwise numpy, axis reductions, the lapx JV's tie order via
 * bxo_lapjv, list order) is followed operation for operation.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bxo.h"

/* ------------------------------------------------------------------------------------------ */
/* fdlibm e_exp.c (public-domain algorithm).                                                    */
static const double ex_halF[2] = {0.5, -0.5}, ex_huge = 1.0e+300,
                    ex_twom1000 = 9.33263618503218878990e-302,
                    ex_o_threshold = 7.09782712893383973096e+02,
                    ex_u_threshold = -7.45133219101941108420e+02,
                    ex_ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
                    ex_ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
                    ex_invln2 = 1.44269504088896338700e+00, ex_P1 = 1.66666666666666019037e-01,
                    ex_P2 = -2.77777777770155933842e-03, ex_P3 = 6.61375632143793436117e-05,
                    ex_P4 = -1.65339022054652515390e-06, ex_P5 = 4.13813679705723846039e-08;

double bxo_exp(double x) {
    uint64_t bits;
    memcpy(&bits, &x, 8);
    uint32_t hx = (uint32_t)(bits >> 32);
    const uint32_t lx = (uint32_t)bits;
    const int xsb = (hx >> 31) & 1;
    hx &= 0x7fffffff;
    double hi = 0.0, lo = 0.0;
    int k = 0;
    if (hx >= 0x40862E42) { /* |x| >= 709.78 */
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | lx) != 0) return x + x; /* NaN */
            return xsb == 0 ? x : 0.0;                     /* exp(+-inf) */
        }
        if (x > ex_o_threshold) return ex_huge * ex_huge;
        if (x < ex_u_threshold) return ex_twom1000 * ex_twom1000;
    }
    if (hx > 0x3fd62e42) {     /* |x| > 0.5 ln2 */
        if (hx < 0x3FF0A2B2) { /* and |x| < 1.5 ln2 */
            hi = x - ex_ln2HI[xsb];
            lo = ex_ln2LO[xsb];
            k = 1 - xsb - xsb;
        } else {
            k = (int)(ex_invln2 * x + ex_halF[xsb]);
            const double t = k;
            hi = x - t * ex_ln2HI[0];
            lo = t * ex_ln2LO[0];
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) { /* |x| < 2^-28 */
        return 1.0 + x;
    } else {
        k = 0;
    }
    const double t = x * x;
    const double c = x - t * (ex_P1 + t * (ex_P2 + t * (ex_P3 + t * (ex_P4 + t * ex_P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    uint64_t yb;
    memcpy(&yb, &y, 8);
    if (k >= -1021) {
        yb += (uint64_t)((int64_t)k << 52);
        memcpy(&y, &yb, 8);
        return y;
    }
    yb += (uint64_t)((int64_t)(k + 1000) << 52);
    memcpy(&y, &yb, 8);
    return y * ex_twom1000;
}

/* x ** 1.5 (boosttrack.py:440 max_s**1.5): x*sqrt(x) plus the fma-exact residuals of both
 * roundings. */
double bxo_pow15(double x) {
    if (x != x) return x;
    if (x < 0.0) return NAN;
    if (x == 0.0) return 0.0;
    if (isinf(x)) return x;
    const double s = sqrt(x);
    const double r = fma(-s, s, x); /* x - s*s, exact */
    const double p = x * s;
    const double e = fma(x, s, -p); /* x*s - p, exact */
    return p + (e + x * (r / (2.0 * s)));
}

/* numpy NaN-propagating max/min (np.maximum, ndarray.max/min) */
static inline double nmax(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
static inline double nmin(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }

/* ------------------------------------------------------------------------------------------ */
/* Kalman filter (kalmanfilter.py:29-157), dt = 1, constant noise (ConstantNoise :8-26).       */
typedef struct {
    double x[8], P[64];
} bkf;

static void bkf_init(bkf *k, const double *z) { /* :47-73 */
    memset(k, 0, sizeof *k);
    for (int i = 0; i < 4; i++) k->x[i] = z[i];
    for (int i = 0; i < 8; i++) k->P[9 * i] = i < 4 ? 10.0 : 10000.0; /* eye; [4:,4:]*=1000; *=10 */
}

/* :75-107  x = F x; P = multi_dot((F, P, F.T)) + Q.  multi_dot of three equal squares takes
 * A(BC) (numpy _multi_dot_three, cost tie); F has two non-zero terms per row, so each entry is
 * one rounding whatever BLAS order: M = P F^T, P' = F M. */
static void bkf_predict(bkf *k) {
    double M[64];
    for (int i = 0; i < 4; i++) k->x[i] = k->x[i] + k->x[i + 4];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++)
            M[8 * i + j] = j < 4 ? k->P[8 * i + j] + k->P[8 * i + j + 4] : k->P[8 * i + j];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            const double v = i < 4 ? M[8 * i + j] + M[8 * (i + 4) + j] : M[8 * i + j];
            k->P[8 * i + j] = i == j ? v + (i < 4 ? 1.0 : 0.01) : v;
        }
}

static int chol4(const double *S, double *L) {
    memset(L, 0, sizeof(double) * 16);
    for (int j = 0; j < 4; j++) {
        double d = S[4 * j + j];
        for (int k = 0; k < j; k++) d -= L[4 * j + k] * L[4 * j + k];
        if (!(d > 0.0)) return -1;
        d = sqrt(d);
        L[4 * j + j] = d;
        for (int i = j + 1; i < 4; i++) {
            double s = S[4 * i + j];
            for (int k = 0; k < j; k++) s -= L[4 * i + k] * L[4 * j + k];
            L[4 * i + j] = s / d;
        }
    }
    return 0;
}

/* :127-157 with R = diag(1, 1, 10, 0.01) (get_r :20-22); loop order as bxo_kf_update. */
static void bkf_update(bkf *k, const double *z) {
    static const double R[4] = {1.0, 1.0, 10.0, 0.01};
    double S[16], L[16], K[32];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) S[4 * i + j] = k->P[8 * i + j] + (i == j ? R[i] : 0.0);
    if (chol4(S, L)) return;
    for (int c = 0; c < 8; c++) {
        double y[4], xx[4];
        for (int i = 0; i < 4; i++) {
            double s = k->P[8 * c + i];
            for (int q = 0; q < i; q++) s -= L[4 * i + q] * y[q];
            y[i] = s / L[4 * i + i];
        }
        for (int i = 3; i >= 0; i--) {
            double s = y[i];
            for (int q = i + 1; q < 4; q++) s -= L[4 * q + i] * xx[q];
            xx[i] = s / L[4 * i + i];
        }
        for (int i = 0; i < 4; i++) K[4 * c + i] = xx[i];
    }
    double innov[4];
    for (int q = 0; q < 4; q++) innov[q] = z[q] - k->x[q];
    for (int i = 0; i < 8; i++) {
        double s = 0.0;
        for (int q = 0; q < 4; q++) s += innov[q] * K[4 * i + q];
        k->x[i] = k->x[i] + s;
    }
    for (int i = 0; i < 8; i++) {
        double ks[4];
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int q = 0; q < 4; q++) s += K[4 * i + q] * S[4 * q + j];
            ks[j] = s;
        }
        for (int j = 0; j < 8; j++) {
            double s = 0.0;
            for (int q = 0; q < 4; q++) s += ks[q] * K[4 * j + q];
            k->P[8 * i + j] = k->P[8 * i + j] - s;
        }
    }
}

/* boosttrack.py:19-28 */
static void bbox_to_z(const double *b, double *z) {
    const double w = b[2] - b[0], h = b[3] - b[1];
    z[0] = b[0] + w / 2.0;
    z[1] = b[1] + h / 2.0;
    z[2] = h;
    z[3] = w / (h + 1e-6);
}

/* boosttrack.py:31-42 */
static void x_to_bbox(const double *x, double *b) {
    const double h = x[2], r = x[3];
    const double w = r <= 0 ? 0.0 : r * h;
    b[0] = x[0] - w / 2.0;
    b[1] = x[1] - h / 2.0;
    b[2] = x[0] + w / 2.0;
    b[3] = x[1] + h / 2.0;
}

/* ------------------------------------------------------------------------------------------ */
/* Pairwise terms (assoc.py).  a: detection row (xyxy...), b: tracker row.                      */
static double iou_b(const double *a, const double *b) { /* assoc.py:50-66 */
    const double xx1 = nmax(a[0], b[0]), yy1 = nmax(a[1], b[1]);
    const double xx2 = nmin(a[2], b[2]), yy2 = nmin(a[3], b[3]);
    const double w = nmax(0.0, xx2 - xx1), h = nmax(0.0, yy2 - yy1);
    const double wh = w * h;
    return wh / ((a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - wh);
}

static double soft_biou(const double *a, const double *b, double bconf) { /* assoc.py:69-103 */
    const double k1 = 0.25, k2 = 0.5, c = 1 - bconf;
    const double b1x1 = a[0] - (a[2] - a[0]) * c * k1, b2x1 = b[0] - (b[2] - b[0]) * c * k2;
    const double xx1 = nmax(b1x1, b2x1);
    const double b1y1 = a[1] - (a[3] - a[1]) * c * k1, b2y1 = b[1] - (b[3] - b[1]) * c * k2;
    const double yy1 = nmax(b1y1, b2y1);
    const double b1x2 = a[2] + (a[2] - a[0]) * c * k1, b2x2 = b[2] + (b[2] - b[0]) * c * k2;
    const double xx2 = nmin(b1x2, b2x2);
    const double b1y2 = a[3] + (a[3] - a[1]) * c * k1, b2y2 = b[3] + (b[3] - b[1]) * c * k2;
    const double yy2 = nmin(b1y2, b2y2);
    const double w = nmax(0.0, xx2 - xx1), h = nmax(0.0, yy2 - yy1);
    const double wh = w * h;
    return wh / ((b1x2 - b1x1) * (b1y2 - b1y1) + (b2x2 - b2x1) * (b2y2 - b2y1) - wh);
}

static double shape_sim(const double *a, const double *b, int v2) { /* assoc.py:9-34 */
    const double dw = a[2] - a[0], dh = a[3] - a[1];
    const double tw = b[2] - b[0], th = b[3] - b[1];
    const double mw = nmax(dw, tw), mh = v2 ? nmax(dh, th) : mw;
    return bxo_exp(-(fabs(dw - tw) / mw + fabs(dh - th) / mh));
}

/* get_mh_dist_matrix (boosttrack.py:356-369): sum over 4 dims, numpy's in-order n<8 sum */
static double mh_dist(const double *det, const double *x, const double *sinv) {
    double z[4];
    bbox_to_z(det, z);
    double s = 0.0;
    for (int q = 0; q < 4; q++) {
        const double d = z[q] - x[q];
        s += d * d * sinv[q];
    }
    return s;
}

/* Op-level entries (mirrors of bx_kf_boost_*): KalmanFilter.__init__ (kalmanfilter.py:47-73)
 * from a measurement z = convert_bbox_to_z, predict (:75-107), update (:127-157), and
 * get_mh_dist_matrix (boosttrack.py:356-369) of detections [nd][4] xyxy against tracks. */
void bxo_kf_boost_initiate(int n, const double *z, double *x, double *P) {
    for (int k = 0; k < n; k++) {
        bkf b;
        bkf_init(&b, z + 4 * k);
        memcpy(x + 8 * k, b.x, sizeof b.x);
        memcpy(P + 64 * k, b.P, sizeof b.P);
    }
}

void bxo_kf_boost_predict(int n, double *x, double *P) {
    for (int k = 0; k < n; k++) {
        bkf b;
        memcpy(b.x, x + 8 * k, sizeof b.x);
        memcpy(b.P, P + 64 * k, sizeof b.P);
        bkf_predict(&b);
        memcpy(x + 8 * k, b.x, sizeof b.x);
        memcpy(P + 64 * k, b.P, sizeof b.P);
    }
}

void bxo_kf_boost_update(int n, double *x, double *P, const double *z) {
    for (int k = 0; k < n; k++) {
        bkf b;
        memcpy(b.x, x + 8 * k, sizeof b.x);
        memcpy(b.P, P + 64 * k, sizeof b.P);
        bkf_update(&b, z + 4 * k);
        memcpy(x + 8 * k, b.x, sizeof b.x);
        memcpy(P + 64 * k, b.P, sizeof b.P);
    }
}

void bxo_kf_boost_mh_dist(int nd, const double *dets, int nt, const double *x, const double *P,
                          double *out) {
    for (int t = 0; t < nt; t++) {
        double sinv[4];
        for (int q = 0; q < 4; q++) sinv[q] = 1.0 / P[64 * t + 9 * q];
        for (int d = 0; d < nd; d++) out[(size_t)d * nt + t] = mh_dist(dets + 4 * d, x + 8 * t, sinv);
    }
}

#define MH_LIMIT 13.2767

/* MhDist_similarity (assoc.py:37-47): softmax over axis 0 (detections) per tracker column;
 * ndarray.sum(0) accumulates rows in order. mh [nd][nt] in place -> similarity. */
static void mh_similarity(double *mh, int nd, int nt, double temp) {
    double *colsum = (double *)calloc(nt ? nt : 1, sizeof(double));
    unsigned char *mask = (unsigned char *)malloc((size_t)(nd > 0 ? nd : 1) * (nt ? nt : 1));
    for (int d = 0; d < nd; d++)
        for (int t = 0; t < nt; t++) {
            double v = mh[(size_t)d * nt + t];
            const int m = v > MH_LIMIT;
            mask[(size_t)d * nt + t] = (unsigned char)m;
            if (m) v = MH_LIMIT;
            v = bxo_exp((MH_LIMIT - v) / temp);
            mh[(size_t)d * nt + t] = v;
            colsum[t] = d == 0 ? v : colsum[t] + v;
        }
    for (int d = 0; d < nd; d++)
        for (int t = 0; t < nt; t++) {
            double *p = mh + (size_t)d * nt + t;
            *p = mask[(size_t)d * nt + t] ? 0.0 : *p / colsum[t];
        }
    free(colsum);
    free(mask);
}

/* ------------------------------------------------------------------------------------------ */
typedef struct {
    bkf kf;
    double conf, cls, det_ind;
    int id, tsu, hit_streak, age;
    double *emb;
} btrk;

struct bxo_boost {
    bxo_boost_params p;
    int frame_count, id_count, n, cap, emb_dim;
    btrk *trk;
};

bxo_boost *bxo_boost_new(const bxo_boost_params *p) {
    bxo_boost *b = (bxo_boost *)calloc(1, sizeof *b);
    b->p = *p;
    b->cap = 64;
    b->trk = (btrk *)calloc(b->cap, sizeof(btrk));
    return b;
}

void bxo_boost_free(bxo_boost *b) {
    if (!b) return;
    for (int i = 0; i < b->n; i++) free(b->trk[i].emb);
    free(b->trk);
    free(b);
}

int bxo_boost_id_count(const bxo_boost *b) { return b->id_count; }

/* host edit of trk.kf.x / trk.kf.covariance by id; returns the number of ids found */
int bxo_boost_state_set(bxo_boost *b, int n, const int *ids, const double *x, const double *P) {
    int found = 0;
    for (int j = 0; j < n; j++)
        for (int i = 0; i < b->n; i++)
            if (b->trk[i].id == ids[j]) {
                if (x) memcpy(b->trk[i].kf.x, x + 8 * j, sizeof(double) * 8);
                if (P) memcpy(b->trk[i].kf.P, P + 64 * j, sizeof(double) * 64);
                found++;
                break;
            }
    return found;
}
void bxo_boost_set_id_count(bxo_boost *b, int c) { b->id_count = c; }
void bxo_boost_set_frame_count(bxo_boost *b, int fc) { b->frame_count = fc; }

int bxo_boost_tracks(const bxo_boost *b, int cap, int *ids, double *x, double *P) {
    for (int i = 0; i < b->n && i < cap; i++) {
        if (ids) ids[i] = b->trk[i].id;
        if (x) memcpy(x + 8 * i, b->trk[i].kf.x, sizeof(double) * 8);
        if (P) memcpy(P + 64 * i, b->trk[i].kf.P, sizeof(double) * 64);
    }
    return b->n;
}

/* get_confidence (boosttrack.py:66-70): coef ** k is Python's float pow = libm pow */
static double trk_confidence(const btrk *t) {
    const int n = 7;
    if (t->age < n) return pow(0.9, (double)(n - t->age));
    return pow(0.9, (double)(t->tsu - 1));
}

/* camera_update (boosttrack.py:81-103): warp the current box, rebuild x[:4] */
static void camera_update(btrk *t, const double *w) {
    double b[4];
    x_to_bbox(t->kf.x, b);
    const double x1 = (w[0] * b[0] + w[1] * b[1]) + w[2], y1 = (w[3] * b[0] + w[4] * b[1]) + w[5];
    const double x2 = (w[0] * b[2] + w[1] * b[3]) + w[2], y2 = (w[3] * b[2] + w[4] * b[3]) + w[5];
    const double ww = x2 - x1, hh = y2 - y1;
    t->kf.x[0] = x1 + ww / 2;
    t->kf.x[1] = y1 + hh / 2;
    t->kf.x[2] = hh;
    t->kf.x[3] = ww / hh;
}

/* the engine's fixed "wave order" for np.linalg.norm (see bxo_track.c vnorm) */
static double wave_norm64(const double *x, int n) {
    double s[64], t[64];
    for (int l = 0; l < 64; l++) {
        s[l] = 0.0;
        for (int k = l; k < n; k += 64) s[l] += x[k] * x[k];
    }
    for (int d = 32; d >= 1; d >>= 1) {
        for (int l = 0; l < 64; l++) t[l] = s[l] + s[l ^ d];
        memcpy(s, t, sizeof s);
    }
    return sqrt(s[0]);
}

/* dets_embs @ tracker_embs.T entry: ascending-k fma chain (the engine's fp64 MFMA order) */
static double emb_dot(const double *a, const double *b, int f) {
    double acc = 0.0;
    for (int k = 0; k < f; k++) acc = fma(a[k], b[k], acc);
    return acc;
}

/* assoc.match (assoc.py:106-114) + linear_assignment (:117-153) + associate (:156-200) */
static void boost_associate(const bxo_boost *B, const double *dk, int nd, const double *trk5,
                            int nt, const double *mh, const double *ec, int *matches, int *nm,
                            int *ud, int *nud, int *ut, int *nut) {
    const bxo_boost_params *p = &B->p;
    const double thr = p->iou_threshold;
    *nm = *nud = *nut = 0;
    if (nt == 0) {
        for (int d = 0; d < nd; d++) ud[(*nud)++] = d;
        return;
    }
    const size_t N = (size_t)(nd > 0 ? nd : 1) * nt;
    double *iou = (double *)malloc(sizeof(double) * N), *cost = (double *)malloc(sizeof(double) * N);
    double *mhs = (double *)malloc(sizeof(double) * N);
    if (nd) memcpy(mhs, mh, sizeof(double) * (size_t)nd * nt);
    mh_similarity(mhs, nd, nt, 1.0);
    const double lambda_emb = (((1 + p->lambda_iou) + p->lambda_shape) + p->lambda_mhd) * 1.5;
    for (int d = 0; d < nd; d++)
        for (int t = 0; t < nt; t++) {
            const size_t q = (size_t)d * nt + t;
            const double *a = dk + 7 * d, *b = trk5 + 5 * t;
            const double o = iou_b(a, b);
            iou[q] = o;
            double c = o;
            double cf = a[4] * b[4];
            if (o < thr) cf = 0.0;
            c += p->lambda_iou * cf * o;
            /* mahalanobis_distance.size > 0 here (nd > 0, nt > 0) */
            c += p->lambda_mhd * mhs[q];
            c += p->lambda_shape * cf * shape_sim(a, b, p->s_sim_corr);
            if (ec) c += lambda_emb * ec[q];
            cost[q] = c;
        }
    /* match(): one-to-one fast path, else lapx lapjv(-cost, extend_cost=True) */
    int *mi = (int *)malloc(sizeof(int) * 2 * (size_t)(nd < nt ? nt : nd) + 2);
    int nmi = 0;
    if (nd > 0) {
        int rmax = 0, cmax = 0;
        for (int d = 0; d < nd; d++) {
            int s = 0;
            for (int t = 0; t < nt; t++) s += cost[(size_t)d * nt + t] > thr;
            rmax = s > rmax ? s : rmax;
        }
        for (int t = 0; t < nt; t++) {
            int s = 0;
            for (int d = 0; d < nd; d++) s += cost[(size_t)d * nt + t] > thr;
            cmax = s > cmax ? s : cmax;
        }
        if (rmax == 1 && cmax == 1) {
            for (int d = 0; d < nd; d++)
                for (int t = 0; t < nt; t++)
                    if (cost[(size_t)d * nt + t] > thr) mi[2 * nmi] = d, mi[2 * nmi + 1] = t, nmi++;
        } else {
            const int n = nd > nt ? nd : nt;
            double *E = (double *)calloc((size_t)n * n, sizeof(double));
            int *x = (int *)malloc(sizeof(int) * n), *y = (int *)malloc(sizeof(int) * n);
            for (int d = 0; d < nd; d++)
                for (int t = 0; t < nt; t++) E[(size_t)d * n + t] = -cost[(size_t)d * nt + t];
            bxo_lapjv(n, E, x, y);
            for (int d = 0; d < nd; d++)
                if (x[d] >= 0 && x[d] < nt) mi[2 * nmi] = d, mi[2 * nmi + 1] = x[d], nmi++;
            free(E);
            free(x);
            free(y);
        }
    }
    unsigned char *dm = (unsigned char *)calloc(nd ? nd : 1, 1), *tm = (unsigned char *)calloc(nt, 1);
    for (int k = 0; k < nmi; k++) dm[mi[2 * k]] = 1, tm[mi[2 * k + 1]] = 1;
    for (int d = 0; d < nd; d++)
        if (!dm[d]) ud[(*nud)++] = d;
    for (int t = 0; t < nt; t++)
        if (!tm[t]) ut[(*nut)++] = t;
    for (int k = 0; k < nmi; k++) {
        const int d = mi[2 * k], t = mi[2 * k + 1];
        const size_t q = (size_t)d * nt + t;
        const int valid =
            iou[q] >= thr || (ec ? (iou[q] >= thr / 2 && ec[q] >= 0.75) : 0);
        if (valid) {
            matches[2 * *nm] = d;
            matches[2 * *nm + 1] = t;
            (*nm)++;
        } else {
            ud[(*nud)++] = d;
            ut[(*nut)++] = t;
        }
    }
    free(dm);
    free(tm);
    free(mi);
    free(iou);
    free(cost);
    free(mhs);
}

int bxo_boost_update(bxo_boost *B, const double *dets_in, int n, const double *embs, int emb_dim,
                     const double *warp, double *out, int out_cap) {
    const bxo_boost_params *p = &B->p;
    const int reid = p->with_reid && embs != NULL && emb_dim > 0;
    if (reid) {
        if (B->emb_dim && B->emb_dim != emb_dim) return -3;
        B->emb_dim = emb_dim;
    }
    B->frame_count++;
    const int T = B->n;
    double *dets = (double *)malloc(sizeof(double) * 7 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        memcpy(dets + 7 * i, dets_in + 6 * i, sizeof(double) * 6);
        dets[7 * i + 6] = (double)i;
    }
    /* CMC (boosttrack.py:241-244) then predict (:246-253) */
    static const double eye23[6] = {1, 0, 0, 0, 1, 0};
    if (p->use_ecc)
        for (int t = 0; t < T; t++) camera_update(&B->trk[t], warp ? warp : eye23);
    double *trk5 = (double *)malloc(sizeof(double) * 5 * (size_t)(T > 0 ? T : 1));
    double *sinv = (double *)malloc(sizeof(double) * 4 * (size_t)(T > 0 ? T : 1));
    for (int t = 0; t < T; t++) {
        btrk *k = &B->trk[t];
        bkf_predict(&k->kf);
        k->age++;
        if (k->tsu > 0) k->hit_streak = 0;
        k->tsu++;
        x_to_bbox(k->kf.x, trk5 + 5 * t);
        trk5[5 * t + 4] = trk_confidence(k);
        for (int q = 0; q < 4; q++) sinv[4 * t + q] = 1.0 / k->kf.P[9 * q];
    }
    const size_t NT = (size_t)(n > 0 ? n : 1) * (T ? T : 1);
    double *mh = (double *)malloc(sizeof(double) * NT);
    double *S = (double *)malloc(sizeof(double) * NT);

    /* DLO confidence boost (boosttrack.py:413-456) */
    if (p->use_dlo_boost && n > 0 && T > 0) {
        for (int d = 0; d < n; d++)
            for (int t = 0; t < T; t++)
                mh[(size_t)d * T + t] = mh_dist(dets + 7 * d, B->trk[t].kf.x, sinv + 4 * t);
        if (p->use_rich_s) {
            mh_similarity(mh, n, T, 1.0);
            for (int d = 0; d < n; d++)
                for (int t = 0; t < T; t++) {
                    const double *a = dets + 7 * d, *b = trk5 + 5 * t;
                    const double sh = shape_sim(a, b, p->s_sim_corr);
                    const double sb = soft_biou(a, b, b[4]);
                    S[(size_t)d * T + t] = ((mh[(size_t)d * T + t] + sh) + sb) / 3;
                }
        } else {
            for (int d = 0; d < n; d++)
                for (int t = 0; t < T; t++)
                    S[(size_t)d * T + t] = iou_b(dets + 7 * d, trk5 + 5 * t);
        }
        for (int d = 0; d < n; d++) {
            double *c = dets + 7 * d + 4;
            double max_s = S[(size_t)d * T];
            for (int t = 1; t < T; t++) max_s = nmax(max_s, S[(size_t)d * T + t]);
            if (!p->use_sb && !p->use_vt) {
                *c = nmax(*c, max_s * p->dlo_boost_coef);
                continue;
            }
            if (p->use_sb) {
                const double alpha = 0.65;
                *c = nmax(*c, alpha * *c + (1 - alpha) * bxo_pow15(max_s));
            }
            if (p->use_vt) {
                int hit = 0;
                for (int t = 0; t < T && !hit; t++) {
                    const double th = nmax(0.95 - (double)(B->trk[t].tsu - 1), 0.8);
                    hit = S[(size_t)d * T + t] > th;
                }
                if (hit) *c = nmax(*c, p->det_thresh + 1e-5);
            }
        }
    }
    /* DUO confidence boost (boosttrack.py:371-411) */
    if (p->use_duo_boost && n > 0 && T > 0) {
        int *bi = (int *)malloc(sizeof(int) * n), nb = 0;
        for (int d = 0; d < n; d++) {
            double m = 0.0;
            for (int t = 0; t < T; t++) {
                const double v = mh_dist(dets + 7 * d, B->trk[t].kf.x, sinv + 4 * t);
                m = t == 0 ? v : nmin(m, v);
            }
            if (m > MH_LIMIT && dets[7 * d + 4] < p->det_thresh) bi[nb++] = d;
        }
        if (nb) {
            double *bd = (double *)malloc(sizeof(double) * (size_t)nb * nb);
            double *mx = (double *)malloc(sizeof(double) * nb);
            unsigned char *rem = (unsigned char *)calloc(nb, 1), *inargs = (unsigned char *)calloc(nb, 1);
            for (int i = 0; i < nb; i++) {
                for (int j = 0; j < nb; j++)
                    bd[(size_t)i * nb + j] =
                        iou_b(dets + 7 * bi[i], dets + 7 * bi[j]) - (i == j ? 1.0 : 0.0);
                double m = bd[(size_t)i * nb];
                for (int j = 1; j < nb; j++) m = nmax(m, bd[(size_t)i * nb + j]);
                mx[i] = m;
                rem[i] = m <= 0.3;
                inargs[i] = m > 0.3;
            }
            for (int i = 0; i < nb; i++) {
                if (!inargs[i]) continue;
                double cm = dets[7 * bi[i] + 4];
                for (int j = 0; j < nb; j++)
                    if (bd[(size_t)i * nb + j] > 0.3 && inargs[j]) cm = nmax(cm, dets[7 * bi[j] + 4]);
                if (dets[7 * bi[i] + 4] == cm) rem[i] = 1;
            }
            for (int i = 0; i < nb; i++)
                if (rem[i]) dets[7 * bi[i] + 4] = p->det_thresh + 1e-4;
            free(bd);
            free(mx);
            free(rem);
            free(inargs);
        }
        free(bi);
    }
    /* keep dets[:, 4] >= det_thresh (boosttrack.py:262-266) */
    int *kd = (int *)malloc(sizeof(int) * (n ? n : 1)), nk = 0;
    for (int d = 0; d < n; d++)
        if (dets[7 * d + 4] >= p->det_thresh) kd[nk++] = d;
    double *dk = (double *)malloc(sizeof(double) * 7 * (size_t)(nk > 0 ? nk : 1));
    for (int i = 0; i < nk; i++) memcpy(dk + 7 * i, dets + 7 * kd[i], sizeof(double) * 7);
    /* emb_cost (boosttrack.py:274-281) */
    double *ec = NULL;
    if (reid && T > 0) {
        ec = (double *)malloc(sizeof(double) * (size_t)(nk > 0 ? nk : 1) * T);
        for (int i = 0; i < nk; i++)
            for (int t = 0; t < T; t++)
                ec[(size_t)i * T + t] =
                    emb_dot(embs + (size_t)kd[i] * emb_dim, B->trk[t].emb, emb_dim);
    }
    for (int i = 0; i < nk; i++)
        for (int t = 0; t < T; t++)
            mh[(size_t)i * T + t] = mh_dist(dk + 7 * i, B->trk[t].kf.x, sinv + 4 * t);
    int *mt = (int *)malloc(sizeof(int) * 2 * (size_t)(nk + T + 1));
    int *ud = (int *)malloc(sizeof(int) * (size_t)(nk + T + 1));
    int *ut = (int *)malloc(sizeof(int) * (size_t)(nk + T + 1));
    int nm, nud, nut;
    boost_associate(B, dk, nk, trk5, T, mh, ec, mt, &nm, ud, &nud, ut, &nut);
    /* updates (boosttrack.py:297-306) */
    for (int k = 0; k < nm; k++) {
        const double *d = dk + 7 * mt[2 * k];
        btrk *t = &B->trk[mt[2 * k + 1]];
        t->tsu = 0;
        t->hit_streak++;
        double z[4];
        bbox_to_z(d, z);
        bkf_update(&t->kf, z);
        t->conf = d[4];
        t->cls = d[5];
        t->det_ind = d[6];
        if (reid) {
            const double trust = (d[4] - p->det_thresh) / (1 - p->det_thresh);
            const double af = 0.95;
            const double alpha = af + (1 - af) * (1 - trust);
            const double *e = embs + (size_t)kd[mt[2 * k]] * emb_dim;
            for (int q = 0; q < emb_dim; q++) t->emb[q] = alpha * t->emb[q] + (1 - alpha) * e[q];
            const double nrm = wave_norm64(t->emb, emb_dim);
            for (int q = 0; q < emb_dim; q++) t->emb[q] = t->emb[q] / nrm;
        }
    }
    /* births (boosttrack.py:308-312) */
    for (int k = 0; k < nud; k++) {
        const double *d = dk + 7 * ud[k];
        if (!(d[4] >= p->det_thresh)) continue;
        if (B->n == B->cap) {
            B->cap *= 2;
            B->trk = (btrk *)realloc(B->trk, sizeof(btrk) * B->cap);
        }
        btrk *t = &B->trk[B->n++];
        memset(t, 0, sizeof *t);
        t->id = ++B->id_count;
        double z[4];
        bbox_to_z(d, z);
        bkf_init(&t->kf, z);
        t->conf = d[4];
        t->cls = d[5];
        t->det_ind = d[6];
        if (reid) {
            t->emb = (double *)malloc(sizeof(double) * emb_dim);
            memcpy(t->emb, embs + (size_t)kd[ud[k]] * emb_dim, sizeof(double) * emb_dim);
        }
    }
    /* outputs (boosttrack.py:314-323), deaths (:325), filter_outputs (:332-341) */
    int m = 0, rc = 0;
    for (int i = 0; i < B->n; i++) {
        btrk *t = &B->trk[i];
        if (t->tsu < 1 && (t->hit_streak >= p->min_hits || B->frame_count <= p->min_hits)) {
            double b[4];
            x_to_bbox(t->kf.x, b);
            const double w = b[2] - b[0], h = b[3] - b[1];
            if (!(w / h <= p->aspect_ratio_thresh && w * h > p->min_box_area)) continue;
            if (m >= out_cap) {
                rc = -2;
                continue;
            }
            double *o = out + 8 * m++;
            o[0] = b[0], o[1] = b[1], o[2] = b[2], o[3] = b[3];
            o[4] = t->id, o[5] = t->conf, o[6] = t->cls, o[7] = t->det_ind;
        }
    }
    int w = 0;
    for (int i = 0; i < B->n; i++) {
        if (B->trk[i].tsu <= p->max_age) {
            B->trk[w++] = B->trk[i];
        } else {
            free(B->trk[i].emb);
        }
    }
    B->n = w;
    free(dets);
    free(trk5);
    free(sinv);
    free(mh);
    free(S);
    free(kd);
    free(dk);
    free(ec);
    free(mt);
    free(ud);
    free(ut);
    return rc ? rc : m;
}
