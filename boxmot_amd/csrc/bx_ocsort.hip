// bx_ocsort.hip — the OCSort per-frame update on MI355X: one wave64 workgroup per sequence.
//
// Reference: boxmot/trackers/ocsort/ocsort.py:195-439 (OcSort.update), its KalmanBoxTracker
// (ocsort.py:56-192) over the XYSR Kalman filter with observation-centric re-update
// (motion/kalman_filters/aabb/xysr_kf.py:48-291), enhanced_associate
// (utils/association.py:377-536) and the legacy lapx linear_assignment (association.py:105-114),
// with the minimal patches P1-P5 documented in oracle/bxo_ocsort.c and SURVEY.md Appendix A.
//
// Every floating-point expression restates oracle/bxo_ocsort.c operation-for-operation (the
// library builds with -ffp-contract=off; f64 division and sqrt are correctly rounded), so track
// states, ids and outputs are bitwise those of the oracle.  The Jonker-Volgenant solve below is
// lapx's dense lapjv (oracle/bxo_ops.c bxo_lapjv) with the same tie order: its column minima,
// reduction-transfer minima and shortest-path relaxations run lane-parallel, and the steps
// whose order decides ties (the column-reduction sweep, the minimum scan over the `col`
// permutation, the swaps it makes, the augmentation) run in the oracle's order.
//
// Track state stays in HBM ([S][T] OcsTrk slots; the per-sequence list `order` keeps the
// reference's list order).  history_obs is kept compactly: the ORU replay only ever reads the
// last non-None box and how many Nones follow it, and the frozen history it restores is
// immediately overwritten by the new observation, so the snapshot needs only (x, P).
#include <float.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/bxocsort.h"
#include "bx_device.h"

using namespace bx;

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)

namespace {

constexpr int OW = 64;        // threads per workgroup: one wave per sequence
constexpr int OBS_KEEP = 8;   // newest observations kept (lookups reach back delta_t <= 7)
constexpr int SQO = 8;        // ints of per-sequence state
enum { SO_FRAME = 0, SO_IDS = 1, SO_NTR = 2, SO_NOUT = 3 };
constexpr int TB = 16;        // doubles per track of per-frame scratch (box4 kobs5 last5 vel2)

struct OcsTrk {
  double x[7], P[49];
  double sx[7], sP[49];         // freeze() snapshot (attr_saved)
  double hbox[4];               // last non-None entry of history_obs
  double last_obs[5];
  double obs_box[OBS_KEEP][5];  // observations dict, newest OBS_KEEP entries
  double vel[2];
  double conf, cls;
  int obs_age[OBS_KEEP];
  int n_obs, has_vel, id, tsu, hits, hit_streak, age, det_ind;
  int observed, has_saved, hvalid, htail;
};

struct OcsDev {
  int S, T, D, N;  // N = max(T, D): largest assignment problem
  double min_conf, det_thresh, asso_threshold, inertia, q_xy, q_s;
  int max_age, min_hits, delta_t, use_byte, max_obs;
  int cost_lds;     // doubles of LDS for a cost matrix (larger ones go to `cost_g`)
  OcsTrk* trk;      // [S][T]
  int* seqst;       // [S][SQO]
  int* order;       // [S][T] slot ids in the reference's list order
  double* tb;       // [S][T][TB]
  double* cost_g;   // [S][D*T] or null
  int* status;
};

// ------------------------------------------------------------------------------------------
// fdlibm acos (oracle/bxo_ocsort.c bxo_acos)
__device__ double ocs_acos(double x) {
  const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
               pi_c = 3.14159265358979311600e+00, pS0 = 1.66666666666666657415e-01,
               pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01,
               pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04,
               pS5 = 3.47933107596021167570e-05, qS1 = -2.40339491173441421878e+00,
               qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01,
               qS4 = 7.70381505559019352791e-02;
  const long long bits = __double_as_longlong(x);
  const int hx = (int)(bits >> 32);
  const int ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {
    if (x == 1.0) return 0.0;
    if (x == -1.0) return pi_c + 2.0 * pio2_lo;
    return __builtin_nan("");
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
    const double df = __longlong_as_double(__double_as_longlong(s) & (long long)0xffffffff00000000ULL);
    const double c = (z - df * df) / (s + df);
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const double r = p / q;
    const double w = r * s + c;
    return 2.0 * (df + w);
  }
}

// ------------------------------------------------------------------------------------------
// XYSR Kalman filter (xysr_kf.py), the oracle's kf_predict7 / inv4 / kf_update7_core.
__device__ void kf_predict7(const OcsDev& g, double* x, double* P) {
  for (int i = 0; i < 3; i++) x[i] = x[i] + x[i + 4];
  double FP[49];
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 7; j++) FP[i * 7 + j] = i < 3 ? P[i * 7 + j] + P[(i + 4) * 7 + j] : P[i * 7 + j];
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 7; j++) {
      const double m = j < 3 ? FP[i * 7 + j] + FP[i * 7 + j + 4] : FP[i * 7 + j];
      double q = 0.0;
      if (i == j) q = (i == 4 || i == 5) ? g.q_xy : (i == 6 ? g.q_s : 1.0);
      P[i * 7 + j] = 1.0 * m + q;
    }
}

__device__ void inv4(const double* Ain, double* B) {
  double A[16];
  int piv[4];
  for (int i = 0; i < 16; i++) A[i] = Ain[i];
  for (int k = 0; k < 4; k++) {
    int p = k;
    double mx = fabs(A[k * 4 + k]);
    for (int i = k + 1; i < 4; i++)
      if (fabs(A[i * 4 + k]) > mx) mx = fabs(A[i * 4 + k]), p = i;
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < 4; j++) {
        const double t = A[k * 4 + j];
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
  for (int i = 0; i < 16; i++) B[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int k = 0; k < 4; k++)
    if (piv[k] != k)
      for (int j = 0; j < 4; j++) {
        const double t = B[k * 4 + j];
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
}

__device__ void kf_update7_core(double* x, double* P, const double* z) {
  const double Rd[4] = {1.0, 1.0, 10.0, 10.0};
  double y[4], S[16], SI[16], K[28];
  for (int k = 0; k < 4; k++) y[k] = z[k] - x[k];
  for (int a = 0; a < 4; a++)
    for (int b = 0; b < 4; b++) S[a * 4 + b] = P[a * 7 + b] + (a == b ? Rd[a] : 0.0);
  inv4(S, SI);
  for (int i = 0; i < 7; i++)
    for (int b = 0; b < 4; b++) {
      double acc = 0.0;
      for (int a = 0; a < 4; a++) acc += P[i * 7 + a] * SI[a * 4 + b];
      K[i * 4 + b] = acc;
    }
  for (int i = 0; i < 7; i++) {
    double acc = 0.0;
    for (int b = 0; b < 4; b++) acc += K[i * 4 + b] * y[b];
    x[i] = x[i] + acc;
  }
  double IKH[49], A[49];
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 7; j++) IKH[i * 7 + j] = (i == j ? 1.0 : 0.0) - (j < 4 ? K[i * 4 + j] : 0.0);
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 7; j++) {
      double acc = 0.0;
      for (int k = 0; k < 7; k++) acc += IKH[i * 7 + k] * P[k * 7 + j];
      A[i * 7 + j] = acc;
    }
  // P = A IKH' + K R K' (the Joseph form), written back row by row
  for (int i = 0; i < 7; i++)
    for (int j = 0; j < 7; j++) {
      double acc = 0.0;
      for (int k = 0; k < 7; k++) acc += A[i * 7 + k] * IKH[j * 7 + k];
      double kr = 0.0;
      for (int b = 0; b < 4; b++) kr += (K[i * 4 + b] * Rd[b]) * K[j * 4 + b];
      P[i * 7 + j] = acc + kr;
    }
}

// xysr_kf.py:211-291 with a measurement (the None branch is ocs_update_none)
__device__ void kf_update7(const OcsDev& g, OcsTrk& t, const double* z) {
  if (!t.observed && t.has_saved) {  // unfreeze (xysr_kf.py:183-209)
    // new_history = history + [z]: the previous non-None entry is hbox, htail+1 steps back
    const double b1[4] = {t.hbox[0], t.hbox[1], t.hbox[2], t.hbox[3]};
    const int hv = t.hvalid, gap = t.htail + 1;
    for (int i = 0; i < 7; i++) t.x[i] = t.sx[i];
    for (int i = 0; i < 49; i++) t.P[i] = t.sP[i];
    t.has_saved = 0;
    if (hv) {
      const double x1 = b1[0], y1 = b1[1], s1 = b1[2], r1 = b1[3];
      const double w1 = sqrt(s1 * r1), h1 = sqrt(s1 / r1);
      const double x2 = z[0], y2 = z[1], s2 = z[2], r2 = z[3];
      const double w2 = sqrt(s2 * r2), h2 = sqrt(s2 / r2);
      const double dx = (x2 - x1) / gap, dy = (y2 - y1) / gap;
      const double dw = (w2 - w1) / gap, dh = (h2 - h1) / gap;
      for (int i = 0; i < gap; i++) {
        const double xx = x1 + (i + 1) * dx, yy = y1 + (i + 1) * dy;
        const double ww = w1 + (i + 1) * dw, hh = h1 + (i + 1) * dh;
        const double nb[4] = {xx, yy, ww * hh, ww / (double)hh};
        kf_update7_core(t.x, t.P, nb);
        if (i != gap - 1) kf_predict7(g, t.x, t.P);
      }
    }
  }
  t.observed = 1;
  kf_update7_core(t.x, t.P, z);
  for (int k = 0; k < 4; k++) t.hbox[k] = z[k];
  t.htail = 0;
  t.hvalid = 1;
}

// ocsort.py:31-45
__device__ void x_to_bbox(const double* x, double* b) {
  const double w = sqrt(x[2] * x[3]);
  const double h = x[2] / w;
  b[0] = x[0] - w / 2.0;
  b[1] = x[1] - h / 2.0;
  b[2] = x[0] + w / 2.0;
  b[3] = x[1] + h / 2.0;
}

__device__ double sum5(const double* b) { return (((b[0] + b[1]) + b[2]) + b[3]) + b[4]; }

__device__ int obs_find(const OcsTrk& t, int age) {
  for (int q = 0; q < t.n_obs; q++)
    if (t.obs_age[q] == age) return q;
  return -1;
}

// ocsort.py:136-171 (update with a detection row [x1,y1,x2,y2,conf] + cls)
__device__ void ocs_update_det(const OcsDev& g, OcsTrk& t, const double* b5, double cls,
                               int det_ind) {
  t.det_ind = det_ind;
  t.conf = b5[4];
  t.cls = cls;
  if (sum5(t.last_obs) >= 0) {
    int q = -1;
    for (int i = 0; i < g.delta_t && q < 0; i++) q = obs_find(t, t.age - (g.delta_t - i));
    const double* prev = q >= 0 ? t.obs_box[q] : t.last_obs;
    // ocsort.py:48-53 speed_direction
    const double cx1 = (prev[0] + prev[2]) / 2.0, cy1 = (prev[1] + prev[3]) / 2.0;
    const double cx2 = (b5[0] + b5[2]) / 2.0, cy2 = (b5[1] + b5[3]) / 2.0;
    const double sy = cy2 - cy1, sx = cx2 - cx1;
    const double norm = sqrt((cy2 - cy1) * (cy2 - cy1) + (cx2 - cx1) * (cx2 - cx1)) + 1e-6;
    t.vel[0] = sy / norm;
    t.vel[1] = sx / norm;
    t.has_vel = 1;
  }
  for (int k = 0; k < 5; k++) t.last_obs[k] = b5[k];
  if (t.n_obs > 0 && t.obs_age[t.n_obs - 1] == t.age) {
    for (int k = 0; k < 5; k++) t.obs_box[t.n_obs - 1][k] = b5[k];
  } else {
    if (t.n_obs == OBS_KEEP) {
      for (int q = 0; q + 1 < OBS_KEEP; q++) {
        t.obs_age[q] = t.obs_age[q + 1];
        for (int k = 0; k < 5; k++) t.obs_box[q][k] = t.obs_box[q + 1][k];
      }
      t.n_obs--;
    }
    t.obs_age[t.n_obs] = t.age;
    for (int k = 0; k < 5; k++) t.obs_box[t.n_obs][k] = b5[k];
    t.n_obs++;
  }
  t.tsu = 0;
  t.hits++;
  t.hit_streak++;
  // P1 xyxy2xysr
  const double w = b5[2] - b5[0], h = b5[3] - b5[1];
  const double z[4] = {b5[0] + w / 2.0, b5[1] + h / 2.0, w * h, w / (h + 1e-6)};
  kf_update7(g, t, z);
}

// update(None): history_obs gets a None; the first miss after an observation freezes
__device__ void ocs_update_none(const OcsDev& g, OcsTrk& t) {
  t.det_ind = -1;
  t.htail++;
  if (t.htail >= g.max_obs) t.hvalid = 0;  // the box left the deque(maxlen=max_obs)
  if (t.observed) {
    t.has_saved = 1;
    for (int i = 0; i < 7; i++) t.sx[i] = t.x[i];
    for (int i = 0; i < 49; i++) t.sP[i] = t.P[i];
  }
  t.observed = 0;
}

// ------------------------------------------------------------------------------------------
// Wave-cooperative lapx lapjv (oracle/bxo_ops.c bxo_lapjv) on the zero-padded square
// max(nr, nc) of a row-major nr x nc matrix (legacy linear_assignment, association.py:105-114).
struct JvLds {
  double *v, *d;
  int *x, *y, *matches, *freer, *pred, *col;
  int* sc;  // >= 8 ints of broadcast scratch
  double* sd;
};

__device__ __forceinline__ double cget(const double* C, int nr, int nc, int i, int j) {
  return (i < nr && j < nc) ? C[i * nc + j] : 0.0;
}

__device__ double wave_min_d(double a) {
  for (int o = 32; o >= 1; o >>= 1) a = fmin(a, __shfl_xor(a, o));
  return a;
}

__device__ void jv_wave(const double* C, int nr, int nc, JvLds& w) {
  const int n = nr > nc ? nr : nc;
  const int lane = threadIdx.x;
  // column reduction: minima (first row index on ties) lane-parallel ...
  for (int j = lane; j < n; j += OW) {
    double mn = cget(C, nr, nc, 0, j);
    int imin = 0;
    for (int i = 1; i < n; i++) {
      const double c = cget(C, nr, nc, i, j);
      if (c < mn) mn = c, imin = i;
    }
    w.d[j] = mn;
    w.pred[j] = imin;
    w.x[j] = -1;
    w.matches[j] = 0;
  }
  __syncthreads();
  // ... and the sweep j = n-1..0 that settles them in the oracle's order
  if (lane == 0) {
    for (int j = n - 1; j >= 0; j--) {
      const int imin = w.pred[j];
      w.v[j] = w.d[j];
      if (++w.matches[imin] == 1) {
        w.x[imin] = j;
        w.y[j] = imin;
      } else if (w.v[j] < w.v[w.x[imin]]) {
        const int j1 = w.x[imin];
        w.x[imin] = j;
        w.y[j] = imin;
        w.y[j1] = -1;
      } else {
        w.y[j] = -1;
      }
    }
  }
  __syncthreads();
  // reduction transfer (rows in order: each changes v[x[i]], read by the rows after it)
  int nfree = 0;
  for (int i = 0; i < n; i++) {
    const int m = w.matches[i];
    if (m == 0) {
      if (lane == 0) w.freer[nfree] = i;
      nfree++;
    } else if (m == 1) {
      const int j1 = w.x[i];
      double mn = DBL_MAX;
      for (int j = lane; j < n; j += OW) {
        const double h = cget(C, nr, nc, i, j) - w.v[j];
        if (j != j1 && h < mn) mn = h;
      }
      mn = wave_min_d(mn);
      __syncthreads();
      if (lane == 0 && mn < DBL_MAX) w.v[j1] = w.v[j1] - mn;
      __syncthreads();
    }
  }
  __syncthreads();
  // augmentation
  for (int f = 0; f < nfree; f++) {
    const int fr = w.freer[f];
    for (int j = lane; j < n; j += OW) {
      w.d[j] = cget(C, nr, nc, fr, j) - w.v[j];
      w.pred[j] = fr;
      w.col[j] = j;
    }
    __syncthreads();
    int low = 0, up = 0, last = 0, endofpath = -1, found = 0;
    double mn = 0.0;
    do {
      if (up == low) {
        // minimum scan over col[up..n): its swaps fix the later iteration order (lane 0)
        if (lane == 0) {
          last = low - 1;
          mn = w.d[w.col[up++]];
          for (int k = up; k < n; k++) {
            const int j = w.col[k];
            const double h = w.d[j];
            if (h <= mn) {
              if (h < mn) {
                up = low;
                mn = h;
              }
              w.col[k] = w.col[up];
              w.col[up++] = j;
            }
          }
          for (int k = low; k < up; k++)
            if (w.y[w.col[k]] < 0) {
              endofpath = w.col[k];
              found = 1;
              break;
            }
          w.sc[0] = last;
          w.sc[1] = up;
          w.sc[2] = endofpath;
          w.sc[3] = found;
          w.sd[0] = mn;
        }
        __syncthreads();
        last = w.sc[0];
        up = w.sc[1];
        endofpath = w.sc[2];
        found = w.sc[3];
        mn = w.sd[0];
        __syncthreads();
      }
      if (!found) {
        const int j1 = w.col[low++];
        const int i = w.y[j1];
        const double h = cget(C, nr, nc, i, j1) - w.v[j1] - mn;
        // relaxation from row i over col[up..n) in chunks of 64 positions; the first column
        // reached at distance mn that is unassigned ends the path (the oracle's break)
        const int up0 = up;
        for (int base = up0; base < n && !found; base += OW) {
          const int k = base + lane;
          int j = -1;
          double v2 = 0.0;
          bool A = false, B = false, E = false;
          if (k < n) {
            j = w.col[k];
            v2 = cget(C, nr, nc, i, j) - w.v[j] - h;
            A = v2 < w.d[j];
            B = A && v2 == mn;
            E = B && w.y[j] < 0;
          }
          const unsigned long long em = __ballot(E);
          int kE = OW;
          if (em) kE = __ffsll((long long)em) - 1;
          if (A && lane < kE) {
            w.pred[j] = i;
            w.d[j] = v2;
          }
          if (em && lane == kE) w.pred[j] = i;
          unsigned long long hm = __ballot(B && !E && lane < kE);
          __syncthreads();
          while (hm) {  // the swaps, in position order
            const int b = __ffsll((long long)hm) - 1;
            hm &= hm - 1;
            const int jb = __shfl(j, b);
            if (lane == 0) {
              w.col[base + b] = w.col[up];
              w.col[up] = jb;
            }
            up++;
            __syncthreads();
          }
          if (em) {
            endofpath = __shfl(j, kE);
            found = 1;
          }
        }
        __syncthreads();
      }
    } while (!found);
    for (int k = lane; k <= last; k += OW) {
      const int j1 = w.col[k];
      w.v[j1] = w.v[j1] + w.d[j1] - mn;
    }
    __syncthreads();
    if (lane == 0) {
      int i;
      do {
        i = w.pred[endofpath];
        w.y[endofpath] = i;
        const int j1 = endofpath;
        endofpath = w.x[i];
        w.x[i] = j1;
      } while (i != fr);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// Wave-order-preserving compaction: emit(k, pos) for k < n with pred(k); returns the count.
template <class P, class E>
__device__ int wave_compact(int n, P pred, E emit) {
  const int lane = threadIdx.x;
  int base = 0;
  for (int c = 0; c < n; c += OW) {
    const int k = c + lane;
    const bool f = k < n && pred(k);
    const unsigned long long m = __ballot(f);
    if (f) emit(k, base + __popcll(m & ((1ull << lane) - 1ull)));
    base += __popcll(m);
  }
  __syncthreads();
  return base;
}

struct OcsLds {
  double* dd;     // [D][6] detections of the frame (float32 values as f64)
  double* cost;   // [cost_lds]
  int *hi, *lo;   // [D] detection indices of the two confidence splits
  int *lst, *lst2;          // [T] slots in list order
  int *mi, *mm;             // [2N] candidate / validated (det, trk) pairs
  int *ud, *ut;             // [D+T] unmatched lists
  int *rowcnt, *colcnt, *rowcol;  // [N] each
  int *fl;                  // [N] flags
  int* sc;                  // [16] broadcast scalars
  double* sd;               // [4]
  JvLds jv;
};

__device__ void carve(const OcsDev& g, char* base, OcsLds& L) {
  size_t o = 0;
  auto takeD = [&](size_t n) { double* p = (double*)(base + o); o += n * 8; return p; };
  auto takeI = [&](size_t n) { int* p = (int*)(base + o); o += ((n * 4 + 7) / 8) * 8; return p; };
  const int N = g.N, D = g.D, T = g.T;
  L.dd = takeD((size_t)D * 6);
  L.cost = takeD(g.cost_lds);
  L.jv.v = takeD(N);
  L.jv.d = takeD(N);
  L.sd = takeD(4);
  L.jv.sd = takeD(2);
  L.hi = takeI(D);
  L.lo = takeI(D);
  L.lst = takeI(T);
  L.lst2 = takeI(T);
  L.mi = takeI(2 * N);
  L.mm = takeI(2 * N);
  L.ud = takeI(D + T);
  L.ut = takeI(D + T);
  L.rowcnt = takeI(N);
  L.colcnt = takeI(N);
  L.rowcol = takeI(N);
  L.fl = takeI(N);
  L.sc = takeI(16);
  L.jv.x = takeI(N);
  L.jv.y = takeI(N);
  L.jv.matches = takeI(N);
  L.jv.freer = takeI(N);
  L.jv.pred = takeI(N);
  L.jv.col = takeI(N);
  L.jv.sc = takeI(8);
}

size_t lds_bytes(int D, int T, int N, int cost_lds) {
  auto dI = [](size_t n) { return ((n * 4 + 7) / 8) * 8; };
  return (size_t)D * 6 * 8 + (size_t)cost_lds * 8 + 2 * (size_t)N * 8 + 6 * 8 + 2 * dI(D) +
         2 * dI(T) + 2 * dI(2 * N) + 2 * dI(D + T) + 4 * dI(N) + dI(16) + 6 * dI(N) + dI(8);
}

// legacy linear_assignment of the nr x nc matrix C: pairs (row, col) in row order into out
// (interleaved), returns the count (uniform)
__device__ int legacy_lap(const double* C, int nr, int nc, JvLds& jv, int* out) {
  jv_wave(C, nr, nc, jv);
  return wave_compact(
      nr, [&](int i) { return jv.x[i] < nc; },
      [&](int i, int p) {
        out[2 * p] = i;
        out[2 * p + 1] = jv.x[i];
      });
}

__global__ void __launch_bounds__(OW)
    ocsort_frame_kernel(OcsDev g, int seq0, const float* __restrict__ dets,
                        const int* __restrict__ det_off, double* __restrict__ out,
                        int* __restrict__ out_count) {
  extern __shared__ __align__(16) char lds_raw[];
  OcsLds L;
  carve(g, lds_raw, L);
  const int lane = threadIdx.x;
  const int b = blockIdx.x, seq = seq0 + b;
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) {  // the host checks det_cap; a device-side overflow is latched, never run past
    if (threadIdx.x == 0) atomicExch(g.status, (int)BX_ERR_CAPACITY);
    n = g.D;
  }
  int* sq = g.seqst + (size_t)seq * SQO;
  OcsTrk* trk = g.trk + (size_t)seq * g.T;
  int* order = g.order + (size_t)seq * g.T;
  double* tb = g.tb + (size_t)seq * g.T * TB;
  double* cost = g.cost_g ? g.cost_g + (size_t)seq * g.D * g.T : nullptr;
  const int frame = sq[SO_FRAME] + 1;
  const int id0 = sq[SO_IDS];
  const int nt0 = sq[SO_NTR];
  const double thr = g.asso_threshold;

  // detections (setup_decorator's float32 rounding is the input format) and the splits
  for (int q = lane; q < n * 6; q += OW) L.dd[q] = (double)dets[(size_t)r0 * 6 + q];
  for (int p = lane; p < nt0; p += OW) L.lst2[p] = order[p];
  __syncthreads();
  const int nl = wave_compact(
      n, [&](int i) { const double c = L.dd[6 * i + 4]; return c > g.min_conf && c < g.det_thresh; },
      [&](int i, int p) { L.lo[p] = i; });
  const int nh = wave_compact(
      n, [&](int i) { return L.dd[6 * i + 4] > g.det_thresh; }, [&](int i, int p) { L.hi[p] = i; });

  // predict every track; tracks whose prediction has a NaN leave the list (ocsort.py:278-288)
  int nt = 0;
  for (int c = 0; c < nt0; c += OW) {
    const int p = c + lane;
    double bx[4] = {0, 0, 0, 0};
    int slot = -1;
    bool keep = false;
    if (p < nt0) {
      slot = L.lst2[p];
      OcsTrk& t = trk[slot];
      if ((t.x[6] + t.x[2]) <= 0) t.x[6] *= 0.0;
      kf_predict7(g, t.x, t.P);
      t.age++;
      if (t.tsu > 0) t.hit_streak = 0;
      t.tsu++;
      x_to_bbox(t.x, bx);
      keep = !(isnan(bx[0]) || isnan(bx[1]) || isnan(bx[2]) || isnan(bx[3]));
    }
    const unsigned long long m = __ballot(keep);
    if (keep) {
      const int q = nt + __popcll(m & ((1ull << lane) - 1ull));
      L.lst[q] = slot;
      double* r = tb + (size_t)q * TB;
      const OcsTrk& t = trk[slot];
      for (int k = 0; k < 4; k++) r[k] = bx[k];
      // k_previous_obs (ocsort.py:17-28) -> r[4..8]; last_obs -> r[9..13]; velocity -> r[14..15]
      if (t.n_obs == 0) {
        for (int k = 0; k < 5; k++) r[4 + k] = -1.0;
      } else {
        int qq = -1;
        for (int i = 0; i < g.delta_t && qq < 0; i++) qq = obs_find(t, t.age - (g.delta_t - i));
        if (qq < 0) qq = t.n_obs - 1;
        for (int k = 0; k < 5; k++) r[4 + k] = t.obs_box[qq][k];
      }
      for (int k = 0; k < 5; k++) r[9 + k] = t.last_obs[k];
      r[14] = t.has_vel ? t.vel[0] : 0.0;
      r[15] = t.has_vel ? t.vel[1] : 0.0;
    }
    nt += __popcll(m);
  }
  __syncthreads();

  // ---- first association: enhanced_associate(high dets, predicted tracks) -----------------
  int nm = 0, nud = 0, nut = 0;
  if (nt == 0) {
    for (int k = lane; k < nh; k += OW) L.ud[k] = k;
    nud = nh;
  } else {
    int nmi = 0;
    if (nh > 0) {
      double* C = (nh * nt <= g.cost_lds) ? L.cost : cost;
      for (int k = lane; k < g.N; k += OW) L.rowcnt[k] = L.colcnt[k] = 0;
      __syncthreads();
      for (int q = lane; q < nh * nt; q += OW) {
        const int d = q / nt, ti = q - d * nt;
        const double* a = L.dd + 6 * L.hi[d];
        const double* r = tb + (size_t)ti * TB;
        const double o = iou_pair(a, r);
        // speed_direction_batch (association.py:10-20) against the k-previous observation
        const double* p = r + 4;
        const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
        const double cx2 = (p[0] + p[2]) / 2.0, cy2 = (p[1] + p[3]) / 2.0;
        double dx = cx1 - cx2, dy = cy1 - cy2;
        const double norm = sqrt(dx * dx + dy * dy) + 1e-6;
        dx = dx / norm;
        dy = dy / norm;
        double c = r[15] * dx + r[14] * dy;
        c = c < -1 ? -1 : (c > 1 ? 1 : c);
        double ang = ocs_acos(c);
        ang = (3.14159265358979323846 / 2.0 - fabs(ang)) / 3.14159265358979323846;
        const double valid = p[4] < 0 ? 0.0 : 1.0;
        const double mc = (valid * ang) * g.inertia;
        C[q] = -(o + mc);
        if (o > thr) {
          atomicAdd(&L.rowcnt[d], 1);
          atomicAdd(&L.colcnt[ti], 1);
          L.rowcol[d] = ti;
        }
      }
      __syncthreads();
      int mr = 0, mcx = 0;
      for (int k = lane; k < nh; k += OW) mr = max(mr, L.rowcnt[k]);
      for (int k = lane; k < nt; k += OW) mcx = max(mcx, L.colcnt[k]);
      for (int o = 32; o >= 1; o >>= 1) {
        mr = max(mr, __shfl_xor(mr, o));
        mcx = max(mcx, __shfl_xor(mcx, o));
      }
      if (mr == 1 && mcx == 1) {  // one-to-one: np.stack(np.where(iou > thr), 1), row-major
        nmi = wave_compact(
            nh, [&](int d) { return L.rowcnt[d] == 1; },
            [&](int d, int p) {
              L.mi[2 * p] = d;
              L.mi[2 * p + 1] = L.rowcol[d];
            });
      } else {  // P4: legacy linear_assignment(-total)
        nmi = legacy_lap(C, nh, nt, L.jv, L.mi);
      }
    }
    // P3: unmatched = absent from the candidate pairs, ascending; then the IoU validation with
    // rejected pairs appended in pair order (P5)
    for (int k = lane; k < g.N; k += OW) L.rowcnt[k] = L.colcnt[k] = 0;
    __syncthreads();
    for (int q = lane; q < nmi; q += OW) {
      L.rowcnt[L.mi[2 * q]] = 1;
      L.colcnt[L.mi[2 * q + 1]] = 1;
    }
    __syncthreads();
    nud = wave_compact(nh, [&](int d) { return L.rowcnt[d] == 0; }, [&](int d, int p) { L.ud[p] = d; });
    nut = wave_compact(nt, [&](int t) { return L.colcnt[t] == 0; }, [&](int t, int p) { L.ut[p] = t; });
    for (int c = 0; c < nmi; c += OW) {
      const int q = c + lane;
      bool ok = false, rej = false;
      int d = 0, ti = 0;
      if (q < nmi) {
        d = L.mi[2 * q];
        ti = L.mi[2 * q + 1];
        ok = iou_pair(L.dd + 6 * L.hi[d], tb + (size_t)ti * TB) >= thr;
        rej = !ok;
      }
      const unsigned long long mo = __ballot(ok), mr = __ballot(rej);
      const unsigned long long below = (1ull << lane) - 1ull;
      if (ok) {
        const int p = nm + __popcll(mo & below);
        L.mm[2 * p] = d;
        L.mm[2 * p + 1] = ti;
      }
      if (rej) {
        const int p = __popcll(mr & below);
        L.ud[nud + p] = d;
        L.ut[nut + p] = ti;
      }
      nm += __popcll(mo);
      nud += __popcll(mr);
      nut += __popcll(mr);
    }
    __syncthreads();
  }
  for (int q = lane; q < nm; q += OW) {
    const double* r = L.dd + 6 * L.hi[L.mm[2 * q]];
    ocs_update_det(g, trk[L.lst[L.mm[2 * q + 1]]], r, r[5], L.hi[L.mm[2 * q]]);
  }
  __syncthreads();

  // ---- BYTE round on the low-confidence detections (ocsort.py:330-356) ---------------------
  if (g.use_byte && nl > 0 && nut > 0) {
    double* C = (nl * nut <= g.cost_lds) ? L.cost : cost;
    double mx = -INF;
    for (int q = lane; q < nl * nut; q += OW) {
      const int d = q / nut, k = q - d * nut;
      const double o = iou_pair(L.dd + 6 * L.lo[d], tb + (size_t)L.ut[k] * TB);
      C[q] = -o;
      mx = fmax(mx, o);
    }
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    __syncthreads();
    if (mx > thr) {
      const int np_ = legacy_lap(C, nl, nut, L.jv, L.mi);
      for (int k = lane; k < g.N; k += OW) L.fl[k] = 0;
      __syncthreads();
      for (int q = lane; q < np_; q += OW) {
        const int dl = L.mi[2 * q], k = L.mi[2 * q + 1];
        if (-C[dl * nut + k] < thr) continue;
        const double* r = L.dd + 6 * L.lo[dl];
        ocs_update_det(g, trk[L.lst[L.ut[k]]], r, r[5], L.lo[dl]);
        L.fl[L.ut[k]] = 2;  // removed
      }
      __syncthreads();
      for (int k = lane; k < nut; k += OW)
        if (L.fl[L.ut[k]] == 0) L.fl[L.ut[k]] = 1;
      __syncthreads();
      // np.setdiff1d: ascending, unique
      nut = wave_compact(nt, [&](int t) { return L.fl[t] == 1; }, [&](int t, int p) { L.ut[p] = t; });
    }
  }

  // ---- OCR round on the last observations (ocsort.py:358-386) -------------------------------
  if (nud > 0 && nut > 0) {
    double* C = (nud * nut <= g.cost_lds) ? L.cost : cost;
    double mx = -INF;
    for (int q = lane; q < nud * nut; q += OW) {
      const int d = q / nut, k = q - d * nut;
      const double o = iou_pair(L.dd + 6 * L.hi[L.ud[d]], tb + (size_t)L.ut[k] * TB + 9);
      C[q] = -o;
      mx = fmax(mx, o);
    }
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    __syncthreads();
    if (mx > thr) {
      const int np_ = legacy_lap(C, nud, nut, L.jv, L.mi);
      for (int k = lane; k < g.N; k += OW) L.rowcnt[k] = L.fl[k] = 0;
      __syncthreads();
      for (int q = lane; q < np_; q += OW) {
        const int a = L.mi[2 * q], k = L.mi[2 * q + 1];
        if (-C[a * nut + k] < thr) continue;
        const int di = L.ud[a], ti = L.ut[k];
        const double* r = L.dd + 6 * L.hi[di];
        ocs_update_det(g, trk[L.lst[ti]], r, r[5], L.hi[di]);
        L.rowcnt[di] = 2;
        L.fl[ti] = 2;
      }
      __syncthreads();
      for (int k = lane; k < nud; k += OW)
        if (L.rowcnt[L.ud[k]] == 0) L.rowcnt[L.ud[k]] = 1;
      for (int k = lane; k < nut; k += OW)
        if (L.fl[L.ut[k]] == 0) L.fl[L.ut[k]] = 1;
      __syncthreads();
      nud = wave_compact(nh, [&](int d) { return L.rowcnt[d] == 1; }, [&](int d, int p) { L.ud[p] = d; });
      nut = wave_compact(nt, [&](int t) { return L.fl[t] == 1; }, [&](int t, int p) { L.ut[p] = t; });
    }
  }
  for (int k = lane; k < nut; k += OW) ocs_update_none(g, trk[L.lst[L.ut[k]]]);

  // ---- new tracks for the unmatched high detections (free slots ascending) ----------------
  for (int s = lane; s < g.T; s += OW) L.fl[s] = 0;
  __syncthreads();
  for (int p = lane; p < nt; p += OW) L.fl[L.lst[p]] = 1;
  __syncthreads();
  const int nfree = wave_compact(g.T, [&](int s) { return L.fl[s] == 0; }, [&](int s, int p) { L.lst2[p] = s; });
  int nnew = nud;
  if (nnew > nfree) {
    if (lane == 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
    nnew = nfree;
  }
  for (int k = lane; k < nnew; k += OW) {
    const int slot = L.lst2[k];
    const double* r = L.dd + 6 * L.hi[L.ud[k]];
    OcsTrk& t = trk[slot];
    for (int i = 0; i < 7; i++) t.x[i] = 0.0;
    for (int i = 0; i < 49; i++) t.P[i] = 0.0;
    const double pd[7] = {10.0, 10.0, 10.0, 10.0, 10000.0, 10000.0, 10000.0};
    for (int i = 0; i < 7; i++) t.P[i * 8] = pd[i];
    const double w = r[2] - r[0], h = r[3] - r[1];
    t.x[0] = r[0] + w / 2.0;
    t.x[1] = r[1] + h / 2.0;
    t.x[2] = w * h;
    t.x[3] = w / (h + 1e-6);
    t.observed = 0;
    t.has_saved = 0;
    t.hvalid = 0;
    t.htail = 0;
    t.id = id0 + k;
    t.conf = r[4];
    t.cls = r[5];
    t.det_ind = L.hi[L.ud[k]];
    for (int q = 0; q < 5; q++) t.last_obs[q] = -1.0;
    t.n_obs = 0;
    t.has_vel = 0;
    t.vel[0] = t.vel[1] = 0.0;
    t.tsu = t.hits = t.hit_streak = t.age = 0;
    L.lst[nt + k] = slot;
  }
  __syncthreads();
  const int ntr = nt + nnew;

  // ---- outputs in reversed list order, then deletion of the dead (ocsort.py:414-436) ---------
  double* orow = out + (size_t)r0 * 8;
  const int nout = wave_compact(
      ntr,
      [&](int k) {
        const OcsTrk& t = trk[L.lst[ntr - 1 - k]];
        return t.tsu < 1 && (t.hit_streak >= g.min_hits || frame <= g.min_hits);
      },
      [&](int k, int p) {
        const OcsTrk& t = trk[L.lst[ntr - 1 - k]];
        double d[4];
        if (sum5(t.last_obs) < 0) {
          x_to_bbox(t.x, d);
        } else {
          for (int q = 0; q < 4; q++) d[q] = t.last_obs[q];
        }
        if (p < n) {
          double* o = orow + (size_t)p * 8;
          o[0] = d[0]; o[1] = d[1]; o[2] = d[2]; o[3] = d[3];
          o[4] = (double)(t.id + 1);
          o[5] = t.conf;
          o[6] = t.cls;
          o[7] = (double)t.det_ind;
        }
      });
  const int nkeep = wave_compact(
      ntr, [&](int k) { return trk[L.lst[k]].tsu <= g.max_age; },
      [&](int k, int p) { order[p] = L.lst[k]; });
  if (lane == 0) {
    out_count[b] = nout < n ? nout : n;
    sq[SO_FRAME] = frame;
    sq[SO_IDS] = id0 + nnew;
    sq[SO_NTR] = nkeep;
    sq[SO_NOUT] = nout;
  }
}

__global__ void ocsort_reset_kernel(OcsDev g, int seq0, int nseq) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nseq * SQO) g.seqst[(size_t)seq0 * SQO + k] = 0;
}

thread_local std::string g_ocs_err;

}  // namespace

struct bx_ocsort {
  OcsDev dev;
  bx_ocsort_config cfg;
  void* arena = nullptr;
  size_t lds = 0;
  int device = 0;
  // host-path staging
  float* h_dets = nullptr;
  int* h_off = nullptr;
  double* h_out = nullptr;
  int* h_cnt = nullptr;
  // timing probe
  bool probe_on = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  int ev_used = 0;
};

#define OCHK(x)                                                                    \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess)                                                          \
      return bx_record_error(BX_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

static int launch(bx_ocsort* e, int seq0, int nseq, const float* dets, const int* off,
                  double* out, int* cnt, hipStream_t st) {
  if (e->probe_on) {
    if (e->ev_used == (int)e->ev.size()) {
      hipEvent_t a, b;
      OCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      OCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
      e->ev.push_back({a, b});
    }
    OCHK(hipEventRecord(e->ev[e->ev_used].first, st));
  }
  hipLaunchKernelGGL(ocsort_frame_kernel, dim3(nseq), dim3(OW), e->lds, st, e->dev, seq0, dets,
                     off, out, cnt);
  OCHK(hipGetLastError());
  if (e->probe_on) OCHK(hipEventRecord(e->ev[e->ev_used++].second, st));
  return BX_OK;
}

extern "C" {

int bx_ocsort_create(const bx_ocsort_config* c, bx_ocsort** out) {
  if (!c || !out) return bx_record_error(BX_ERR_INVALID, "null argument");
  if (c->n_seq <= 0 || c->track_cap <= 0 || c->det_cap <= 0 || c->track_cap > 4096 ||
      c->det_cap > 4096)
    return bx_record_error(BX_ERR_INVALID, "n_seq/track_cap/det_cap out of range");
  if (c->delta_t < 1 || c->delta_t > OBS_KEEP - 1)
    return bx_record_error(BX_ERR_INVALID, "delta_t must be in [1, 7]");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0)
    return bx_record_error(BX_ERR_NO_DEVICE, "no HIP device visible");
  bx_ocsort* e = new bx_ocsort();
  e->cfg = *c;
  OCHK(hipGetDevice(&e->device));
  OcsDev& d = e->dev;
  d.S = c->n_seq;
  d.T = c->track_cap;
  d.D = c->det_cap;
  d.N = d.T > d.D ? d.T : d.D;
  d.min_conf = c->min_conf;
  d.det_thresh = c->det_thresh;
  d.asso_threshold = c->asso_threshold;
  d.inertia = c->inertia;
  d.q_xy = 1.0 * c->q_xy_scaling;
  d.q_s = 1.0 * c->q_s_scaling;
  d.max_age = c->max_age;
  d.min_hits = c->min_hits;
  d.delta_t = c->delta_t;
  d.use_byte = c->use_byte;
  // basetracker.py:59-62: max_obs = 50, or max_age + 5 when max_age >= 50
  d.max_obs = c->max_age >= 50 ? c->max_age + 5 : 50;
  // LDS: the fixed part plus as much cost matrix as keeps ~4 workgroups per CU resident
  const size_t fixed = lds_bytes(d.D, d.T, d.N, 0);
  long budget = 40 * 1024 - (long)fixed;
  int cl = budget > 0 ? (int)(budget / 8) : 0;
  if (cl > d.D * d.T) cl = d.D * d.T;
  if (cl < 64) cl = 64;
  d.cost_lds = cl;
  e->lds = lds_bytes(d.D, d.T, d.N, cl);
  if (e->lds > 160 * 1024) {
    delete e;
    return bx_record_error(BX_ERR_INVALID, "track_cap/det_cap too large for one workgroup's LDS");
  }
  const bool need_g = (long)d.D * d.T > cl;
  const size_t S = d.S, T = d.T;
  size_t off = 0;
  auto carve_b = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_trk = carve_b(S * T * sizeof(OcsTrk));
  const size_t o_sq = carve_b(S * SQO * sizeof(int));
  const size_t o_ord = carve_b(S * T * sizeof(int));
  const size_t o_tb = carve_b(S * T * TB * sizeof(double));
  const size_t o_cg = need_g ? carve_b(S * (size_t)d.D * T * sizeof(double)) : 0;
  const size_t o_st = carve_b(sizeof(int) * 4);
  if (hipMalloc(&e->arena, off) != hipSuccess) {
    delete e;
    return bx_record_error(BX_ERR_HIP, "hipMalloc of the OCSort arena failed");
  }
  OCHK(hipMemset(e->arena, 0, off));
  char* base = (char*)e->arena;
  d.trk = (OcsTrk*)(base + o_trk);
  d.seqst = (int*)(base + o_sq);
  d.order = (int*)(base + o_ord);
  d.tb = (double*)(base + o_tb);
  d.cost_g = need_g ? (double*)(base + o_cg) : nullptr;
  d.status = (int*)(base + o_st);
  OCHK(hipFuncSetAttribute((const void*)ocsort_frame_kernel,
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->lds));
  OCHK(hipMalloc(&e->h_dets, sizeof(float) * 6 * d.D));
  OCHK(hipMalloc(&e->h_off, sizeof(int) * 2));
  OCHK(hipMalloc(&e->h_out, sizeof(double) * 8 * d.D));
  OCHK(hipMalloc(&e->h_cnt, sizeof(int)));
  *out = e;
  return BX_OK;
}

int bx_ocsort_destroy(bx_ocsort* e) {
  if (!e) return BX_OK;
  for (auto& p : e->ev) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  (void)hipFree(e->arena);
  (void)hipFree(e->h_dets);
  (void)hipFree(e->h_off);
  (void)hipFree(e->h_out);
  (void)hipFree(e->h_cnt);
  delete e;
  return BX_OK;
}

int bx_ocsort_reset(bx_ocsort* e, int seq0, int nseq, void* stream) {
  if (!e || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad sequence range");
  if (!nseq) return BX_OK;
  hipLaunchKernelGGL(ocsort_reset_kernel, dim3((nseq * SQO + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, e->dev, seq0, nseq);
  OCHK(hipGetLastError());
  return BX_OK;
}

int bx_ocsort_step(bx_ocsort* e, int seq0, int nseq, const float* dets, const int32_t* det_off,
                   double* out, int32_t* out_count, void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_step");
  return launch(e, seq0, nseq, dets, det_off, out, out_count, (hipStream_t)stream);
}

int bx_ocsort_update_host(bx_ocsort* e, int seq, const float* dets, int n, double* out,
                          int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!dets || !out)) || !n_out)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_update_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  hipStream_t st = (hipStream_t)stream;
  const int off[2] = {0, n};
  if (n) OCHK(hipMemcpyAsync(e->h_dets, dets, sizeof(float) * 6 * n, hipMemcpyHostToDevice, st));
  OCHK(hipMemcpyAsync(e->h_off, off, sizeof(off), hipMemcpyHostToDevice, st));
  int rc = launch(e, seq, 1, e->h_dets, e->h_off, e->h_out, e->h_cnt, st);
  if (rc) return rc;
  int cnt = 0;
  OCHK(hipMemcpyAsync(&cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  OCHK(hipStreamSynchronize(st));
  if (cnt) OCHK(hipMemcpy(out, e->h_out, sizeof(double) * 8 * cnt, hipMemcpyDeviceToHost));
  *n_out = cnt;
  int status = 0;
  OCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status)
    return bx_record_error(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

int bx_ocsort_status(bx_ocsort* e, int* status) {
  if (!e || !status) return bx_record_error(BX_ERR_INVALID, "null argument");
  OCHK(hipMemcpy(status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  return BX_OK;
}

int bx_ocsort_counters_host(bx_ocsort* e, int seq, int* frame_count, int* id_count,
                            int* n_tracks) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  int s[SQO];
  OCHK(hipDeviceSynchronize());
  OCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQO, sizeof(s), hipMemcpyDeviceToHost));
  if (frame_count) *frame_count = s[SO_FRAME];
  if (id_count) *id_count = s[SO_IDS];
  if (n_tracks) *n_tracks = s[SO_NTR];
  return BX_OK;
}

int bx_ocsort_set_id_count(bx_ocsort* e, int seq, int id_count, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  OCHK(hipMemcpyAsync(e->dev.seqst + (size_t)seq * SQO + SO_IDS, &id_count, sizeof(int),
                      hipMemcpyHostToDevice, (hipStream_t)stream));
  OCHK(hipStreamSynchronize((hipStream_t)stream));
  return BX_OK;
}

int bx_ocsort_tracks_host(bx_ocsort* e, int seq, int cap, int32_t* ids, double* x, double* p,
                          int* n) {
  if (!e || seq < 0 || seq >= e->dev.S || cap < 0 || !n)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_tracks_host");
  OCHK(hipDeviceSynchronize());
  int s[SQO];
  OCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQO, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[SO_NTR];
  std::vector<int> ord(nt);
  if (nt)
    OCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int k = 0; k < nt && k < cap; k++) {
    OcsTrk t;
    OCHK(hipMemcpy(&t, e->dev.trk + (size_t)seq * e->dev.T + ord[k], sizeof(OcsTrk),
                   hipMemcpyDeviceToHost));
    if (ids) ids[k] = t.id;
    if (x) memcpy(x + 7 * k, t.x, sizeof(t.x));
    if (p) memcpy(p + 49 * k, t.P, sizeof(t.P));
  }
  *n = nt;
  return BX_OK;
}

int bx_ocsort_probe(bx_ocsort* e, int on) {
  if (!e) return bx_record_error(BX_ERR_INVALID, "null engine");
  e->probe_on = on != 0;
  e->ev_used = 0;
  return BX_OK;
}

int bx_ocsort_probe_read(bx_ocsort* e, double* total_ms, int* count) {
  if (!e || !total_ms || !count) return bx_record_error(BX_ERR_INVALID, "null argument");
  double s = 0.0;
  for (int k = 0; k < e->ev_used; k++) {
    OCHK(hipEventSynchronize(e->ev[k].second));
    float ms = 0.f;
    OCHK(hipEventElapsedTime(&ms, e->ev[k].first, e->ev[k].second));
    s += ms;
  }
  *total_ms = s;
  *count = e->ev_used;
  e->ev_used = 0;
  return BX_OK;
}

}  // extern "C"
