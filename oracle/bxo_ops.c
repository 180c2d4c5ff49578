/*
 * bxo_ops.c — oracle kernels: box conversions, IoU, score fusion, cosine distance, Kalman
 * filters and the lapx-semantics linear assignment.  TEST INFRASTRUCTURE ONLY (see bxo.h).
 *
 * Elementwise arithmetic follows numpy's operation order one-for-one and is compiled with
 * -ffp-contract=off so products and sums round exactly as numpy's do.  Only the BLAS/LAPACK
 * contractions inside the Kalman update (cho_factor / cho_solve / multi_dot) have an order the
 * reference does not pin; those are restated straightforwardly and compared with a tolerance.
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <omp.h>

#include "bxo.h"
#include "bxo_internal.h"

#include <stdint.h>

/* ------------------------------------------------------------------------------------------ */
/* utils/ops.py:10-150 box conversions (numpy op order)                                        */

void bxo_xyxy2xywh(const double *x, double *y) { /* ops.py:10-24 */
    y[0] = (x[0] + x[2]) / 2;
    y[1] = (x[1] + x[3]) / 2;
    y[2] = x[2] - x[0];
    y[3] = x[3] - x[1];
}

void bxo_xywh2xyxy(const double *x, double *y) { /* ops.py:27-43 */
    double r[4];
    r[0] = x[0] - x[2] / 2;
    r[1] = x[1] - x[3] / 2;
    r[2] = x[0] + x[2] / 2;
    r[3] = x[1] + x[3] / 2;
    memcpy(y, r, sizeof r);
}

void bxo_xywh2tlwh(const double *x, double *y) { /* ops.py:46-58 */
    double r[4] = {x[0] - x[2] / 2, x[1] - x[3] / 2, x[2], x[3]};
    memcpy(y, r, sizeof r);
}

void bxo_tlwh2xyah(const double *x, double *y) { /* ops.py:89-103 */
    double r[4] = {x[0] + x[2] / 2, x[1] + x[3] / 2, x[2] / x[3], x[3]};
    memcpy(y, r, sizeof r);
}

/* ------------------------------------------------------------------------------------------ */
/* utils/iou.py:50-67 iou_batch                                                                */

double bxo_iou_pair(const double *b1, const double *b2) {
    double xx1 = fmax(b1[0], b2[0]);
    double yy1 = fmax(b1[1], b2[1]);
    double xx2 = fmin(b1[2], b2[2]);
    double yy2 = fmin(b1[3], b2[3]);
    double w = fmax(0.0, xx2 - xx1);
    double h = fmax(0.0, yy2 - yy1);
    double wh = w * h;
    return wh / ((b1[2] - b1[0]) * (b1[3] - b1[1]) + (b2[2] - b2[0]) * (b2[3] - b2[1]) - wh);
}

void bxo_iou_batch(const double *a, int na, const double *b, int nb, double *out) {
    for (int i = 0; i < na; i++)
        for (int j = 0; j < nb; j++) out[(size_t)i * nb + j] = bxo_iou_pair(a + 4 * i, b + 4 * j);
}

/* utils/matching.py:520-544: sim = 1-cost; w = conf>0.7 ? 1.2*conf : conf; mask conf>=0.5;
 * fuse = 1 - sim*w*mask; ×2 where conf < 0.5 */
double bxo_fuse_one(double cost, double conf) {
    double sim = 1 - cost;
    double w = conf > 0.7 ? conf * 1.2 : conf;
    double mask = conf >= 0.5 ? 1.0 : 0.0;
    double fuse = 1 - sim * w * mask;
    return conf < 0.5 ? fuse * 2.0 : fuse;
}

void bxo_fuse_score(double *cost, int nr, int nc, const double *confs) {
    for (int i = 0; i < nr; i++)
        for (int j = 0; j < nc; j++)
            cost[(size_t)i * nc + j] = bxo_fuse_one(cost[(size_t)i * nc + j], confs[j]);
}

/* ------------------------------------------------------------------------------------------ */
/* numpy float32 pairwise summation (numpy/core/src/umath/loops_utils.h pairwise_sum, PW_BLOCKSIZE
 * 128, 8 accumulators) as used by np.add.reduce inside np.linalg.norm(x, axis=1).            */
static float pairwise_sum_f32(const float *x, int n) {
    if (n < 8) {
        float res = 0.0f;
        for (int i = 0; i < n; i++) res += x[i];
        return res;
    }
    if (n <= 128) {
        float r[8];
        for (int k = 0; k < 8; k++) r[k] = x[k];
        int i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; k++) r[k] += x[i + k];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += x[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum_f32(x, n2) + pairwise_sum_f32(x + n2, n - n2);
}

float bxo_np_norm_f32(const float *x, int n) {
    float *sq = (float *)malloc(sizeof(float) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) sq[i] = x[i] * x[i];
    float s = pairwise_sum_f32(sq, n);
    free(sq);
    return sqrtf(s);
}

/* scipy cdist 'cosine' inner product: two interleaved accumulators, remainder added last. */
static double dot2(const double *u, const double *v, int n) {
    double a0 = 0.0, a1 = 0.0;
    int i = 0;
    for (; i + 2 <= n; i += 2) {
        a0 += u[i] * v[i];
        a1 += u[i + 1] * v[i + 1];
    }
    double s = a0 + a1;
    if (i < n) s += u[i] * v[i];
    return s;
}

/* matching.py:279-287: cast float32, x/(||x||+1e-8) in float32, max(0, cdist cosine). */
void bxo_embedding_distance(const float *trk, int nt, const float *det, int nd, int f,
                            double *out) {
    double *A = (double *)malloc(sizeof(double) * (size_t)(nt > 0 ? nt : 1) * f);
    double *B = (double *)malloc(sizeof(double) * (size_t)(nd > 0 ? nd : 1) * f);
    double *na = (double *)malloc(sizeof(double) * (nt > 0 ? nt : 1));
    double *nb = (double *)malloc(sizeof(double) * (nd > 0 ? nd : 1));
    for (int i = 0; i < nt; i++) {
        float dn = bxo_np_norm_f32(trk + (size_t)i * f, f) + 1e-8f;
        for (int k = 0; k < f; k++) A[(size_t)i * f + k] = (double)(trk[(size_t)i * f + k] / dn);
        na[i] = sqrt(dot2(A + (size_t)i * f, A + (size_t)i * f, f));
    }
    for (int j = 0; j < nd; j++) {
        float dn = bxo_np_norm_f32(det + (size_t)j * f, f) + 1e-8f;
        for (int k = 0; k < f; k++) B[(size_t)j * f + k] = (double)(det[(size_t)j * f + k] / dn);
        nb[j] = sqrt(dot2(B + (size_t)j * f, B + (size_t)j * f, f));
    }
    for (int i = 0; i < nt; i++)
        for (int j = 0; j < nd; j++) {
            double c = dot2(A + (size_t)i * f, B + (size_t)j * f, f) / (na[i] * nb[j]);
            if (fabs(c) > 1.0) c = copysign(1.0, c);
            double d = 1.0 - c;
            out[(size_t)i * nd + j] = d < 0.0 ? 0.0 : d;
        }
    free(A);
    free(B);
    free(na);
    free(nb);
}

/* ------------------------------------------------------------------------------------------ */
/* Kalman filters.  State [x,y,a|w,h,vx,vy,va|vw,vh], dt=1 (base_kalman_filter.py:29-41).      */

static const double STD_POS = 1.0 / 20, STD_VEL = 1.0 / 160;

void bxo_kf_initiate(int kind, const double *m, double *mean, double *cov) {
    double std[8];
    if (kind == BXO_KF_XYAH) { /* xyah_kf.py:16-28 */
        std[0] = 2 * STD_POS * m[3];
        std[1] = 2 * STD_POS * m[3];
        std[2] = 1e-2;
        std[3] = 2 * STD_POS * m[3];
        std[4] = 10 * STD_VEL * m[3];
        std[5] = 10 * STD_VEL * m[3];
        std[6] = 1e-5;
        std[7] = 10 * STD_VEL * m[3];
    } else { /* xywh_kf.py:16-26 */
        std[0] = 2 * STD_POS * m[2];
        std[1] = 2 * STD_POS * m[3];
        std[2] = 2 * STD_POS * m[2];
        std[3] = 2 * STD_POS * m[3];
        std[4] = 10 * STD_VEL * m[2];
        std[5] = 10 * STD_VEL * m[3];
        std[6] = 10 * STD_VEL * m[2];
        std[7] = 10 * STD_VEL * m[3];
    }
    for (int k = 0; k < 4; k++) mean[k] = m[k], mean[4 + k] = 0.0;
    memset(cov, 0, sizeof(double) * 64);
    for (int k = 0; k < 8; k++) cov[9 * k] = std[k] * std[k];
}

static void process_noise(int kind, const double *mean, double *q) {
    double s[8];
    if (kind == BXO_KF_XYAH) { /* xyah_kf.py:58-73 */
        s[0] = STD_POS * mean[3];
        s[1] = STD_POS * mean[3];
        s[2] = 1e-2;
        s[3] = STD_POS * mean[3];
        s[4] = STD_VEL * mean[3];
        s[5] = STD_VEL * mean[3];
        s[6] = 1e-5;
        s[7] = STD_VEL * mean[3];
    } else { /* xywh_kf.py:40-54 */
        s[0] = STD_POS * mean[2];
        s[1] = STD_POS * mean[3];
        s[2] = STD_POS * mean[2];
        s[3] = STD_POS * mean[3];
        s[4] = STD_VEL * mean[2];
        s[5] = STD_VEL * mean[3];
        s[6] = STD_VEL * mean[2];
        s[7] = STD_VEL * mean[3];
    }
    for (int k = 0; k < 8; k++) q[k] = s[k] * s[k];
}

/* base_kalman_filter.py:111-127.  F has two non-zero terms per row/column, so np.dot's sums
 * reduce to single roundings whatever BLAS order: cov' = (P_ij+P_i+4,j)+(P_i,j+4+P_i+4,j+4). */
void bxo_kf_multi_predict(int kind, int n, double *mean, double *cov) {
    for (int t = 0; t < n; t++) {
        double *m = mean + 8 * t, *P = cov + 64 * t, q[8], FP[64];
        process_noise(kind, m, q);
        for (int k = 0; k < 4; k++) m[k] = m[k] + m[k + 4];
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++)
                FP[8 * i + j] = i < 4 ? P[8 * i + j] + P[8 * (i + 4) + j] : P[8 * i + j];
        for (int i = 0; i < 8; i++)
            for (int j = 0; j < 8; j++) {
                double v = j < 4 ? FP[8 * i + j] + FP[8 * i + j + 4] : FP[8 * i + j];
                P[8 * i + j] = i == j ? v + q[i] : v;
            }
    }
}

static void meas_noise(int kind, const double *mean, double conf, double *r) {
    double s[4];
    if (kind == BXO_KF_XYAH) { /* xyah_kf.py:75-87 */
        s[0] = STD_POS * mean[3];
        s[1] = STD_POS * mean[3];
        s[2] = 1e-1;
        s[3] = STD_POS * mean[3];
    } else { /* xywh_kf.py:56-63 */
        s[0] = STD_POS * mean[2];
        s[1] = STD_POS * mean[3];
        s[2] = STD_POS * mean[2];
        s[3] = STD_POS * mean[3];
    }
    for (int k = 0; k < 4; k++) {
        double v = (1 - conf) * s[k]; /* base_kalman_filter.py:101 NSA scaling */
        r[k] = v * v;
    }
}

/* base_kalman_filter.py:86-109 project: S = P[:4,:4] + diag(R). */
static void project(int kind, const double *mean, const double *P, double conf, double *S) {
    double r[4];
    meas_noise(kind, mean, conf, r);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) S[4 * i + j] = P[8 * i + j] + (i == j ? r[i] : 0.0);
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

/* base_kalman_filter.py:129-155 */
void bxo_kf_update(int kind, double *mean, double *cov, const double *z, double conf) {
    double S[16], L[16], K[32], PHt[32];
    project(kind, mean, cov, conf, S);
    if (chol4(S, L)) return;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) PHt[4 * i + j] = cov[8 * i + j];
    /* K^T = S^{-1} (P H^T)^T : solve L L^T X = B column by column (B = PHt^T, 4 x 8) */
    for (int c = 0; c < 8; c++) {
        double y[4], x[4];
        for (int i = 0; i < 4; i++) {
            double s = PHt[4 * c + i];
            for (int k = 0; k < i; k++) s -= L[4 * i + k] * y[k];
            y[i] = s / L[4 * i + i];
        }
        for (int i = 3; i >= 0; i--) {
            double s = y[i];
            for (int k = i + 1; k < 4; k++) s -= L[4 * k + i] * x[k];
            x[i] = s / L[4 * i + i];
        }
        for (int i = 0; i < 4; i++) K[4 * c + i] = x[i]; /* K[c][i] (8 x 4) */
    }
    double innov[4];
    for (int k = 0; k < 4; k++) innov[k] = z[k] - mean[k];
    for (int i = 0; i < 8; i++) {
        double s = 0.0;
        for (int k = 0; k < 4; k++) s += innov[k] * K[4 * i + k];
        mean[i] = mean[i] + s;
    }
    double KS[32];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += K[4 * i + k] * S[4 * k + j];
            KS[4 * i + j] = s;
        }
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += KS[4 * i + k] * K[4 * j + k];
            cov[8 * i + j] = cov[8 * i + j] - s;
        }
}

/* base_kalman_filter.py:166-194 (metric 'maha', all 4 dims) */
void bxo_kf_gating_distance(int kind, const double *mean, const double *cov, const double *z,
                            int nz, double *out) {
    double S[16], L[16];
    project(kind, mean, cov, 0.0, S);
    if (chol4(S, L)) {
        for (int k = 0; k < nz; k++) out[k] = NAN;
        return;
    }
    for (int k = 0; k < nz; k++) {
        double d[4], y[4], s2 = 0.0;
        for (int i = 0; i < 4; i++) d[i] = z[4 * k + i] - mean[i];
        for (int i = 0; i < 4; i++) {
            double s = d[i];
            for (int j = 0; j < i; j++) s -= L[4 * i + j] * y[j];
            y[i] = s / L[4 * i + i];
            s2 += y[i] * y[i];
        }
        out[k] = s2;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* lapx 0.5.11.post1 `lapjv` (uv.lock:1789-1795; its lapjv.cpp is the gatagat/lap dense solver),  */
/* restated from the published algorithm: lapjv_internal = _ccrrt_dense (column reduction +      */
/* reduction transfer), at most two _carr_dense passes (augmenting row reduction), then          */
/* _ca_dense (one find_path_dense shortest augmenting path per remaining free row).  Every       */
/* comparison, its strictness and every scan order below decides which optimum a tied problem    */
/* returns, so they are kept exactly (callers: utils/association.py:105-114,                     */
/* trackers/boosttrack/assoc.py:106-114, utils/matching.py:54).  lapx's LARGE sentinel is 1e6.   */

#define LAPX_LARGE 1000000.0

/* _ccrrt_dense: v[j] = min_i c[i][j] (first row on ties, from a LARGE start), columns claimed
 * j = n-1..0 (a row keeps the first column it is found for, later ones are released and the row
 * marked non-unique), then for every uniquely-assigned row in row order v[x[i]] -= the row's
 * smallest other reduced cost.  Returns the free rows (no column) in row order. */
static int lapx_ccrrt(int n, const double *c, int *fr, int *x, int *y, double *v) {
    unsigned char *uniq = (unsigned char *)malloc((size_t)n);
    for (int i = 0; i < n; i++) {
        x[i] = -1;
        v[i] = LAPX_LARGE;
        y[i] = 0;
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const double h = c[(size_t)i * n + j];
            if (h < v[j]) {
                v[j] = h;
                y[j] = i;
            }
        }
    memset(uniq, 1, (size_t)n);
    for (int j = n - 1; j >= 0; j--) {
        const int i = y[j];
        if (x[i] < 0) {
            x[i] = j;
        } else {
            uniq[i] = 0;
            y[j] = -1;
        }
    }
    int nf = 0;
    for (int i = 0; i < n; i++) {
        if (x[i] < 0) {
            fr[nf++] = i;
        } else if (uniq[i]) {
            const int j = x[i];
            double mn = LAPX_LARGE;
            for (int j2 = 0; j2 < n; j2++) {
                if (j2 == j) continue;
                const double h = c[(size_t)i * n + j2] - v[j2];
                if (h < mn) mn = h;
            }
            v[j] -= mn;
        }
    }
    free(uniq);
    return nf;
}

/* _carr_dense: one augmenting-row-reduction pass over fr[0..nfree).  A free row takes its
 * cheapest column j1 (first index on ties; v2 = its second-cheapest reduced cost, first index
 * != j1, from a LARGE start) and lowers v[j1] by v2 - v1; the displaced owner is processed next
 * when v[j1] strictly dropped, else it (or, on a tie, the owner of j2 after switching to j2) is
 * queued for the next pass.  The rr_cnt < current*n guard bounds the pass.  Returns the number of
 * rows queued (they are written back into fr from the front). */
static int lapx_carr(int n, const double *c, int nfree, int *fr, int *x, int *y, double *v) {
    unsigned current = 0, rr_cnt = 0;
    int nnew = 0;
    while (current < (unsigned)nfree) {
        rr_cnt++;
        const int fi = fr[current++];
        int j1 = 0, j2 = -1;
        double v1 = c[(size_t)fi * n] - v[0], v2 = LAPX_LARGE;
        for (int j = 1; j < n; j++) {
            const double h = c[(size_t)fi * n + j] - v[j];
            if (h < v2) {
                if (h >= v1) {
                    v2 = h;
                    j2 = j;
                } else {
                    v2 = v1;
                    v1 = h;
                    j2 = j1;
                    j1 = j;
                }
            }
        }
        int i0 = y[j1];
        const double v1_new = v[j1] - (v2 - v1);
        const int lowers = v1_new < v[j1];
        if (rr_cnt < current * (unsigned)n) {
            if (lowers) {
                v[j1] = v1_new;
            } else if (i0 >= 0 && j2 >= 0) {
                j1 = j2;
                i0 = y[j2];
            }
            if (i0 >= 0) {
                if (lowers)
                    fr[--current] = i0;
                else
                    fr[nnew++] = i0;
            }
        } else if (i0 >= 0) {
            fr[nnew++] = i0;
        }
        x[fi] = j1;
        y[j1] = fi;
    }
    return nnew;
}

/* find_path_dense (with _find_dense / _scan_dense): Dijkstra from free row `start` over reduced
 * costs.  `cols` is a position permutation: [0, lo) scanned ("ready"), [lo, hi) the SCAN set at
 * the current minimum, [hi, n) TODO.  _find_dense moves every TODO column at the new minimum to
 * the SCAN set in position order and the path ends at the LAST unassigned one of them;
 * _scan_dense relaxes TODO columns from each SCAN column and ends at the FIRST column it lowers to
 * the minimum that is unassigned.  Ready columns' v are then raised by d - min. */
static int lapx_find_path(int n, const double *c, int start, const int *y, double *v, int *pred,
                          int *cols, double *d) {
    int lo = 0, hi = 0, final_j = -1, n_ready = 0;
    for (int j = 0; j < n; j++) {
        cols[j] = j;
        pred[j] = start;
        d[j] = c[(size_t)start * n + j] - v[j];
    }
    while (final_j == -1) {
        if (lo == hi) { /* _find_dense */
            n_ready = lo;
            hi = lo + 1;
            double mind = d[cols[lo]];
            for (int k = hi; k < n; k++) {
                const int j = cols[k];
                if (d[j] <= mind) {
                    if (d[j] < mind) {
                        hi = lo;
                        mind = d[j];
                    }
                    cols[k] = cols[hi];
                    cols[hi++] = j;
                }
            }
            for (int k = lo; k < hi; k++)
                if (y[cols[k]] < 0) final_j = cols[k];
        }
        if (final_j == -1) { /* _scan_dense: lo/hi are only written back when it exhausts SCAN */
            int l = lo, h = hi;
            while (l != h && final_j == -1) {
                int j = cols[l++];
                const int i = y[j];
                const double mind = d[j];
                const double hh = c[(size_t)i * n + j] - v[j] - mind;
                for (int k = h; k < n; k++) {
                    j = cols[k];
                    const double cred = c[(size_t)i * n + j] - v[j] - hh;
                    if (cred < d[j]) {
                        d[j] = cred;
                        pred[j] = i;
                        if (cred == mind) {
                            if (y[j] < 0) {
                                final_j = j;
                                break;
                            }
                            cols[k] = cols[h];
                            cols[h++] = j;
                        }
                    }
                }
            }
            if (final_j == -1) {
                lo = l;
                hi = h;
            }
        }
    }
    const double mind = d[cols[lo]];
    for (int k = 0; k < n_ready; k++) {
        const int j = cols[k];
        v[j] += d[j] - mind;
    }
    return final_j;
}

/* _ca_dense: augment along pred from each remaining free row, in list order. */
static void lapx_ca(int n, const double *c, int nfree, const int *fr, int *x, int *y, double *v) {
    int *pred = (int *)malloc(sizeof(int) * n), *cols = (int *)malloc(sizeof(int) * n);
    double *d = (double *)malloc(sizeof(double) * n);
    for (int f = 0; f < nfree; f++) {
        const int start = fr[f];
        int j = lapx_find_path(n, c, start, y, v, pred, cols, d), i = -1;
        while (i != start) {
            i = pred[j];
            y[j] = i;
            const int t = x[i];
            x[i] = j;
            j = t;
        }
    }
    free(pred);
    free(cols);
    free(d);
}

/* lapjv_internal on a dense n x n row-major matrix: x[row] = column, y[column] = row. */
int bxo_lapjv(int n, const double *c, int *x, int *y) {
    if (n <= 0) return 0;
    int *fr = (int *)malloc(sizeof(int) * n);
    double *v = (double *)malloc(sizeof(double) * n);
    int nf = lapx_ccrrt(n, c, fr, x, y, v);
    for (int pass = 0; nf > 0 && pass < 2; pass++) nf = lapx_carr(n, c, nf, fr, x, y, v);
    if (nf > 0) lapx_ca(n, c, nf, fr, x, y, v);
    free(fr);
    free(v);
    return 0;
}

/* matching.py:30-108 with lapx.lapjv(cost, extend_cost=True, cost_limit=thresh):
 * (nr+nc)^2 matrix, off-diagonal blocks cost_limit/2, bottom-right 0. */
int bxo_linear_assignment(const double *cost, int nr, int nc, double thresh, int *matches,
                          int *n_matches, int *ua, int *n_ua, int *ub, int *n_ub) {
    *n_matches = *n_ua = *n_ub = 0;
    if (nr == 0 || nc == 0) { /* matching.py:42-47 */
        for (int i = 0; i < nr; i++) ua[(*n_ua)++] = i;
        for (int j = 0; j < nc; j++) ub[(*n_ub)++] = j;
        return 0;
    }
    int n = nr + nc;
    double *E = (double *)malloc(sizeof(double) * (size_t)n * n);
    int *x = (int *)malloc(sizeof(int) * n), *y = (int *)malloc(sizeof(int) * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            double e;
            if (i < nr && j < nc) e = cost[(size_t)i * nc + j];
            else if (i >= nr && j >= nc) e = 0.0;
            else e = thresh / 2.0;
            E[(size_t)i * n + j] = e;
        }
    bxo_lapjv(n, E, x, y);
    for (int i = 0; i < nr; i++) {
        int j = x[i] >= nc ? -1 : x[i];
        if (j >= 0) {
            if (cost[(size_t)i * nc + j] <= thresh) {
                matches[2 * *n_matches] = i;
                matches[2 * *n_matches + 1] = j;
                (*n_matches)++;
            }
        } else {
            ua[(*n_ua)++] = i;
        }
    }
    for (int j = 0; j < nc; j++)
        if (y[j] >= nr) ub[(*n_ub)++] = j;
    free(E);
    free(x);
    free(y);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* StrongSort NearestNeighborDistanceMetric.distance, cosine metric
 * (trackers/strongsort/sort/linear_assignment.py:595-618 -> _nn_cosine_distance :468-497 ->
 * _cosine_distance :382-413).  Rows are normalised as x / (np.linalg.norm(x, axis=1) + 1e-8)
 * (numpy: sqrt of the pairwise sum of the squares, float64); the dot products are np.dot, a BLAS
 * dgemm of unpinned order — restated here as the k-ascending fma chain that the engine's fp64
 * MFMA (v_mfma_f64_16x16x4_f64, measured bitwise) computes; distance = 1 - clip(dot, -1, 1),
 * minimum over the target's samples; a target without samples costs INFTY_COST = 1e5. */
static double pairwise_sum_f64(const double *x, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; i++) res += x[i];
        return res;
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
    return pairwise_sum_f64(x, n2) + pairwise_sum_f64(x + n2, n - n2);
}

double bxo_np_norm_f64(const double *x, int n) {
    double *sq = (double *)malloc(sizeof(double) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) sq[i] = x[i] * x[i];
    double s = pairwise_sum_f64(sq, n);
    free(sq);
    return sqrt(s);
}

static void normalise_rows(const double *x, int n, int f, double *y) {
    for (int i = 0; i < n; i++) {
        const double d = bxo_np_norm_f64(x + (size_t)i * f, f) + 1e-8;
        for (int k = 0; k < f; k++) y[(size_t)i * f + k] = x[(size_t)i * f + k] / d;
    }
}

int bxo_nn_cosine_distance(const double *samples, const int *off, int T, const double *feats,
                           int D, int F, double *out) {
    const int G = T > 0 ? off[T] : 0;
    double *sh = (double *)malloc(sizeof(double) * ((size_t)G * F + 1));
    double *dh = (double *)malloc(sizeof(double) * ((size_t)D * F + 1));
    normalise_rows(samples, G, F, sh);
    normalise_rows(feats, D, F, dh);
    for (int t = 0; t < T; t++)
        for (int d = 0; d < D; d++) {
            if (off[t + 1] <= off[t]) {
                out[(size_t)t * D + d] = 1e5;
                continue;
            }
            double best = 0.0;
            for (int s = off[t]; s < off[t + 1]; s++) {
                const double *a = sh + (size_t)s * F, *b = dh + (size_t)d * F;
                double acc = 0.0;
                for (int k = 0; k < F; k++) acc = fma(a[k], b[k], acc);
                const double c = acc < -1.0 ? -1.0 : (acc > 1.0 ? 1.0 : acc);
                const double dist = 1.0 - c;
                if (s == off[t] || dist < best) best = dist; /* np.min over the samples */
            }
            out[(size_t)t * D + d] = best;
        }
    free(sh);
    free(dh);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* AssociationFunction variants (utils/iou.py:79-307), one pair per call; numpy op order.      */
/* fdlibm s_atan.c (public-domain algorithm) for np.arctan in ciou. */
static const double at_hi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                9.82793723247329054082e-01, 1.57079632679489655800e+00};
static const double at_lo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                1.39033110312309984516e-17, 6.12323399573676603587e-17};
static const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                              1.42857142725034663711e-01, -1.11111104054623557880e-01,
                              9.09088713343650656196e-02, -7.69187620504482999495e-02,
                              6.66107313738753120669e-02, -5.83357013379057348645e-02,
                              4.97687799461593236017e-02, -3.65315727442169155270e-02,
                              1.62858201153657823623e-02};

double bxo_atan(double x) {
    uint64_t bits;
    memcpy(&bits, &x, 8);
    const int32_t hx = (int32_t)(bits >> 32);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && (uint32_t)bits != 0)) return x + x;
        return hx > 0 ? at_hi[3] + at_lo[3] : -at_hi[3] - at_lo[3];
    }
    if (ix < 0x3fdc0000) {
        if (ix < 0x3e200000) return x;
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) {
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else {
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else {
            if (ix < 0x40038000) {
                id = 2;
                x = (x - 1.5) / (1.0 + 1.5 * x);
            } else {
                id = 3;
                x = -1.0 / x;
            }
        }
    }
    const double z = x * x, w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = at_hi[id] - ((x * (s1 + s2) - at_lo[id]) - x);
    return hx < 0 ? -r : r;
}

static double npmax(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
static double npmin(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }

double bxo_pair_cost(int kind, const double *a, const double *b, double w, double h) {
    const double xx1 = npmax(a[0], b[0]), yy1 = npmax(a[1], b[1]);
    const double xx2 = npmin(a[2], b[2]), yy2 = npmin(a[3], b[3]);
    const double iw = npmax(0.0, xx2 - xx1), ih = npmax(0.0, yy2 - yy1);
    const double wh = iw * ih;
    const double area1 = (a[2] - a[0]) * (a[3] - a[1]), area2 = (b[2] - b[0]) * (b[3] - b[1]);
    switch (kind) {
    case BXO_ASSO_IOU: /* :50-67 */
        return wh / (area1 + area2 - wh);
    case BXO_ASSO_HMIOU: { /* :79-127 */
        const double uh = npmax(1e-10, npmax(a[3], b[3]) - npmin(a[1], b[1]));
        const double o = ih / uh;
        const double iou = wh / ((area1 + area2 - wh) + 1e-10);
        return iou * o;
    }
    case BXO_ASSO_GIOU: { /* :129-169 */
        const double uni = area1 + area2 - wh;
        const double iou = wh / uni;
        const double wc = npmax(a[2], b[2]) - npmin(a[0], b[0]);
        const double hc = npmax(a[3], b[3]) - npmin(a[1], b[1]);
        const double enc = wc * hc;
        const double g = iou - (enc - uni) / enc;
        return (g + 1.0) / 2.0;
    }
    case BXO_ASSO_DIOU: { /* :266-307 */
        const double iou = wh / (area1 + area2 - wh);
        const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
        const double cx2 = (b[0] + b[2]) / 2.0, cy2 = (b[1] + b[3]) / 2.0;
        const double inner = (cx1 - cx2) * (cx1 - cx2) + (cy1 - cy2) * (cy1 - cy2);
        const double ow = npmax(a[2], b[2]) - npmin(a[0], b[0]);
        const double oh = npmax(a[3], b[3]) - npmin(a[1], b[1]);
        const double outer = ow * ow + oh * oh;
        return ((iou - inner / outer) + 1) / 2.0;
    }
    case BXO_ASSO_CIOU: { /* :199-264 */
        const double eps = 1e-7;
        const double iou = wh / (((area1 + area2) - wh) + eps);
        const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
        const double cx2 = (b[0] + b[2]) / 2.0, cy2 = (b[1] + b[3]) / 2.0;
        const double inner = (cx1 - cx2) * (cx1 - cx2) + (cy1 - cy2) * (cy1 - cy2);
        const double ow = npmax(a[2], b[2]) - npmin(a[0], b[0]);
        const double oh = npmax(a[3], b[3]) - npmin(a[1], b[1]);
        const double outer = (ow * ow + oh * oh) + eps;
        const double w1 = a[2] - a[0], h1 = (a[3] - a[1]) + eps;
        const double w2 = b[2] - b[0], h2 = (b[3] - b[1]) + eps;
        const double d = bxo_atan(w2 / h2) - bxo_atan(w1 / h1);
        const double pi = 3.141592653589793;
        const double v = (4 / (pi * pi)) * (d * d);
        const double S = 1 - iou;
        const double alpha = v / ((S + v) + eps);
        const double c = (iou - (inner / outer)) + (alpha * v);
        return (c + 1) / 2.0;
    }
    case BXO_ASSO_CENTROID: { /* :171-184 */
        const double cx1 = (a[0] + a[2]) / 2, cy1 = (a[1] + a[3]) / 2;
        const double cx2 = (b[0] + b[2]) / 2, cy2 = (b[1] + b[3]) / 2;
        const double dx = cx1 - cx2, dy = cy1 - cy2;
        const double dist = sqrt(dx * dx + dy * dy);
        const double nf = sqrt(w * w + h * h);
        return 1 - dist / nf;
    }
    }
    return NAN;
}

void bxo_asso_batch(int kind, const double *a, int na, const double *b, int nb, double w,
                    double h, double *out) {
    for (int i = 0; i < na; i++)
        for (int j = 0; j < nb; j++) out[(size_t)i * nb + j] = bxo_pair_cost(kind, a + 4 * i, b + 4 * j, w, h);
}

/* ------------------------------------------------------------------------------------------ */
/* utils/association.py:320-374 compute_aw_max_metric (DeepOCSort's adaptive embedding weight):
 * per row, then per column, over the strictly positive entries: weight = 1 - max(ratio - bottom,
 * 0) / (1 - bottom) with ratio = second largest / largest (1 when fewer than two), applied as
 * ((w * row_weight) * col_weight) * emb_cost. */
static double aw_weight(const double *v, int n, int stride, double bottom, int *apply) {
    double m1 = -INFINITY, m2 = -INFINITY;
    int cnt = 0;
    for (int k = 0; k < n; k++) {
        const double c = v[(size_t)k * stride];
        if (!(c > 0)) continue;
        cnt++;
        if (c > m1) {
            m2 = m1;
            m1 = c;
        } else if (c > m2) {
            m2 = c;
        }
    }
    *apply = cnt >= 2;
    if (cnt < 2) return 1.0;
    if (m1 == 0) return 0.0;
    const double ratio = m2 / m1;
    const double ex = ratio - bottom;
    return 1 - (ex > 0 ? ex : 0.0) / (1 - bottom);
}

void bxo_aw_max_metric(const double *emb, int nr, int nc, double w_assoc, double bottom,
                       double *out) {
    double *rw = (double *)malloc(sizeof(double) * (size_t)(nr ? nr : 1));
    double *cw = (double *)malloc(sizeof(double) * (size_t)(nc ? nc : 1));
    int *ra = (int *)malloc(sizeof(int) * (size_t)(nr ? nr : 1));
    int *ca = (int *)malloc(sizeof(int) * (size_t)(nc ? nc : 1));
    for (int i = 0; i < nr; i++) rw[i] = aw_weight(emb + (size_t)i * nc, nc, 1, bottom, ra + i);
    for (int j = 0; j < nc; j++) cw[j] = aw_weight(emb + j, nr, nc, bottom, ca + j);
    for (int i = 0; i < nr; i++)
        for (int j = 0; j < nc; j++) {
            double w = w_assoc;
            if (ra[i]) w *= rw[i];
            if (ca[j]) w *= cw[j];
            out[(size_t)i * nc + j] = w * emb[(size_t)i * nc + j];
        }
    free(rw);
    free(cw);
    free(ra);
    free(ca);
}

void bxo_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }
