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
hipError_t bx_lds_attr(const void* kern, size_t bytes);  // bx_engine.hip (never lowers a limit)

namespace {

constexpr int OBS_KEEP = 8;   // newest observations kept (lookups reach back delta_t <= 7)
constexpr int SQO = 8;        // ints of per-sequence state
enum { SO_FRAME = 0, SO_IDS = 1, SO_NTR = 2, SO_NOUT = 3 };
constexpr int TB = 16;        // doubles per track of per-frame scratch (box4 kobs5 last5 vel2)

struct OcsTrk {
  double x[7], P[49];
  double sx[7], sP[49];         // freeze() snapshot (attr_saved)
  double hbox[4];               // last non-None entry of history_obs
  double last_obs[5];
  double obs_box[OBS_KEEP][5];  // observations dict: the entry of age a sits in slot a % 8
  double vel[2];
  double conf, cls;
  int obs_age[OBS_KEEP];
  int last_age, has_vel, id, tsu, hits, hit_streak, age, det_ind;  // last_age < 0: no obs
  int observed, has_saved, hvalid, htail;
};

struct OcsDev {
  int S, T, D, N;  // N = max(T, D): largest assignment problem
  double min_conf, det_thresh, asso_threshold, inertia, q_xy, q_s;
  int max_age, min_hits, delta_t, use_byte, max_obs;
  int asso_kind;    // ASSO_* (BaseTracker asso_func): iou unless configured otherwise
  double* fsz;      // [S][2] frame (w, h) per sequence, for the centroid mode
  int cost_lds;     // doubles of LDS for a cost matrix (larger ones go to `cost_g`)
  OcsTrk* trk;      // [S][T]
  int* seqst;       // [S][SQO]
  int* order;       // [S][T] slot ids in the reference's list order
  double* tb;       // [S][T][TB]
  double* cost_g;   // [S][D*T] or null
  int* status;
  unsigned long long* dbg;  // [S][OCS_DBG] phase stamps (diagnostic builds only, else null)
};

// Diagnostic phase stamps and counters (build with -DBX_PHASE_TIMING; never shipped): per
// sequence, cycles accumulated per phase over all frames [0, 16), event counters [16, 24) and
// the JV's counters [24, 40).
constexpr int OCS_DBG = 40;
#ifdef BX_PHASE_TIMING
#define OSTAMP(k)                                                                    \
  do {                                                                               \
    __syncthreads();                                                                 \
    if (threadIdx.x == 0 && g.dbg) {                                                 \
      const unsigned long long _now = __builtin_amdgcn_s_memtime();                  \
      g.dbg[(size_t)seq * OCS_DBG + (k)] += _now - t_last;                           \
      t_last = _now;                                                                 \
    }                                                                                \
  } while (0)
#define OCOUNT(k, v)                                                                 \
  do {                                                                               \
    if (threadIdx.x == 0 && g.dbg) g.dbg[(size_t)seq * OCS_DBG + 16 + (k)] += (v);   \
  } while (0)
#else
#define OSTAMP(k) \
  do {            \
  } while (0)
#define OCOUNT(k, v) \
  do {               \
  } while (0)
#endif

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
// XYSR Kalman filter (xysr_kf.py) on 8 lanes per track (an "octet"): lane r of the octet owns
// row rr = min(r, 6) of the 7-state mean and covariance (lane 7 mirrors row 6 and never writes).
// Every element is computed by one lane with the oracle's operation order (kf_predict7,
// kf_update7_core in oracle/bxo_ocsort.c); shuffles only move operands between rows.
__device__ __forceinline__ double osh(double v, int src) { return __shfl(v, src, 8); }

struct KfRow {
  double x, P[7];
};

__device__ __forceinline__ void row_load(const double* x, const double* P, int rr, KfRow& k) {
  k.x = x[rr];
#pragma unroll
  for (int j = 0; j < 7; j++) k.P[j] = P[rr * 7 + j];
}

__device__ __forceinline__ void row_store(double* x, double* P, int r, const KfRow& k) {
  if (r < 7) {
    x[r] = k.x;
#pragma unroll
    for (int j = 0; j < 7; j++) P[r * 7 + j] = k.P[j];
  }
}

// x = F x ; P = 1.0 * (F P F') + Q  (F = I + e_i e_{i+4}' for i < 3)
__device__ void kfo_predict(const OcsDev& g, int rr, KfRow& k) {
  const int src = rr < 3 ? rr + 4 : rr;
  const double x4 = osh(k.x, src);
  k.x = rr < 3 ? k.x + x4 : k.x;
  double FP[7];
#pragma unroll
  for (int j = 0; j < 7; j++) {
    const double p4 = osh(k.P[j], src);
    FP[j] = rr < 3 ? k.P[j] + p4 : k.P[j];
  }
#pragma unroll
  for (int j = 0; j < 7; j++) {
    const double m = j < 3 ? FP[j] + FP[j + 4] : FP[j];
    double q = 0.0;
    if (rr == j) q = (rr == 4 || rr == 5) ? g.q_xy : (rr == 6 ? g.q_s : 1.0);
    k.P[j] = 1.0 * m + q;
  }
}

// np.linalg.inv of a 4x4 (oracle inv4: dgetf2 LU with partial pivoting, then dgetrs).  Row
// swaps are written as predicated swaps over constant indices so both matrices stay in VGPRs.
__device__ __forceinline__ void swap_rows4(double* M, int k, int p) {
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (i > k && i == p)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const double t = M[k * 4 + j];
        M[k * 4 + j] = M[i * 4 + j];
        M[i * 4 + j] = t;
      }
}

__device__ __forceinline__ void inv4(const double* Ain, double* B) {
  double A[16];
  int piv[4];
#pragma unroll
  for (int i = 0; i < 16; i++) A[i] = Ain[i];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int p = k;
    double mx = fabs(A[k * 4 + k]);
#pragma unroll
    for (int i = k + 1; i < 4; i++)
      if (fabs(A[i * 4 + k]) > mx) mx = fabs(A[i * 4 + k]), p = i;
    piv[k] = p;
    swap_rows4(A, k, p);
    if (A[k * 4 + k] != 0.0) {
      if (fabs(A[k * 4 + k]) >= DBL_MIN) {
        const double r = 1.0 / A[k * 4 + k];
#pragma unroll
        for (int i = k + 1; i < 4; i++) A[i * 4 + k] *= r;
      } else {
#pragma unroll
        for (int i = k + 1; i < 4; i++) A[i * 4 + k] /= A[k * 4 + k];
      }
    }
#pragma unroll
    for (int j = k + 1; j < 4; j++) {
      const double t = -A[k * 4 + j];
#pragma unroll
      for (int i = k + 1; i < 4; i++) A[i * 4 + j] = A[i * 4 + j] + A[i * 4 + k] * t;
    }
  }
#pragma unroll
  for (int i = 0; i < 16; i++) B[i] = (i % 5 == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) swap_rows4(B, k, piv[k]);
#pragma unroll
  for (int j = 0; j < 4; j++) {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (B[k * 4 + j] != 0.0)
#pragma unroll
        for (int i = k + 1; i < 4; i++) B[i * 4 + j] -= B[k * 4 + j] * A[i * 4 + k];
#pragma unroll
    for (int k = 3; k >= 0; k--)
      if (B[k * 4 + j] != 0.0) {
        B[k * 4 + j] /= A[k * 4 + k];
#pragma unroll
        for (int i = 0; i < k; i++) B[i * 4 + j] -= B[k * 4 + j] * A[i * 4 + k];
      }
  }
}

// update with a measurement (R = diag(1,1,10,10), H = [I4 0], Joseph form); z uniform per octet
__device__ void kfo_update(int rr, KfRow& k, const double* z) {
  const double Rd[4] = {1.0, 1.0, 10.0, 10.0};
  double y[4], S[16], SI[16];
#pragma unroll
  for (int a = 0; a < 4; a++) y[a] = z[a] - osh(k.x, a);
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 4; b++) S[a * 4 + b] = osh(k.P[b], a) + (a == b ? Rd[a] : 0.0);
  inv4(S, SI);  // every lane of the octet inverts the same S identically
  double K[4];
#pragma unroll
  for (int b = 0; b < 4; b++) {
    double acc = 0.0;
#pragma unroll
    for (int a = 0; a < 4; a++) acc += k.P[a] * SI[a * 4 + b];
    K[b] = acc;
  }
  {
    double acc = 0.0;
#pragma unroll
    for (int b = 0; b < 4; b++) acc += K[b] * y[b];
    k.x = k.x + acc;
  }
  double ikh[7], A[7];
#pragma unroll
  for (int c = 0; c < 7; c++) ikh[c] = (rr == c ? 1.0 : 0.0) - (c < 4 ? K[c] : 0.0);
#pragma unroll
  for (int j = 0; j < 7; j++) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 7; c++) acc += ikh[c] * osh(k.P[j], c);
    A[j] = acc;
  }
#pragma unroll
  for (int j = 0; j < 7; j++) {
    double Kj[4];
#pragma unroll
    for (int b = 0; b < 4; b++) Kj[b] = osh(K[b], j);
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 7; c++) acc += A[c] * ((j == c ? 1.0 : 0.0) - (c < 4 ? Kj[c] : 0.0));
    double kr = 0.0;
#pragma unroll
    for (int b = 0; b < 4; b++) kr += (K[b] * Rd[b]) * Kj[b];
    k.P[j] = acc + kr;
  }
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

// The observations dict (ocsort.py:73,158) is read only at ages within delta_t <= 7 of the
// current age, plus its newest key; keeping the entry of age a in slot a % 8 loses only entries
// at least 8 ages older than a newer one, which no lookup reaches.
// First hit of `want0 + i` for i < cnt (ascending), or -1; the probes are independent loads.
__device__ __forceinline__ int obs_first(const OcsTrk& t, int want0, int cnt) {
  int q = -1;
  for (int i = cnt - 1; i >= 0; i--) {
    const int want = want0 + i;
    if (want >= 0 && t.obs_age[want & (OBS_KEEP - 1)] == want) q = want & (OBS_KEEP - 1);
  }
  return q;
}

// ocsort.py:136-171 (update with a detection row [x1,y1,x2,y2,conf] + cls), octet-wide: lane 0
// keeps the track's bookkeeping, the octet runs the Kalman update (with the ORU replay of
// xysr_kf.py:183-209 when the track was frozen)
__device__ void ocs_update_det(const OcsDev& g, OcsTrk& t, int r, const double* b5, double cls,
                               int det_ind) {
  const int rr = r < 7 ? r : 6;
  const int observed = t.observed, has_saved = t.has_saved;
  const int hv = t.hvalid, gap = t.htail + 1;
  const double b1[4] = {t.hbox[0], t.hbox[1], t.hbox[2], t.hbox[3]};
  if (r == 0) {
    t.det_ind = det_ind;
    t.conf = b5[4];
    t.cls = cls;
    if (sum5(t.last_obs) >= 0) {
      const int q = obs_first(t, t.age - g.delta_t, g.delta_t);
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
    const int slot = t.age & (OBS_KEEP - 1);  // observations[age] = bbox
    t.obs_age[slot] = t.age;
    for (int k = 0; k < 5; k++) t.obs_box[slot][k] = b5[k];
    t.last_age = t.age;
    t.tsu = 0;
    t.hits++;
    t.hit_streak++;
  }
  // P1 xyxy2xysr
  const double w = b5[2] - b5[0], h = b5[3] - b5[1];
  const double z[4] = {b5[0] + w / 2.0, b5[1] + h / 2.0, w * h, w / (h + 1e-6)};
  KfRow k;
  const bool unfreeze = !observed && has_saved;
  if (unfreeze) {
    // new_history = history + [z]: the previous non-None entry is hbox, htail+1 steps back;
    // self.__dict__ = attr_saved restores (x, P); its history is overwritten by z below
    row_load(t.sx, t.sP, rr, k);
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
        kfo_update(rr, k, nb);
        if (i != gap - 1) kfo_predict(g, rr, k);
      }
    }
  } else {
    row_load(t.x, t.P, rr, k);
  }
  kfo_update(rr, k, z);
  row_store(t.x, t.P, r, k);
  if (r == 0) {
    if (unfreeze) t.has_saved = 0;
    t.observed = 1;
    for (int q = 0; q < 4; q++) t.hbox[q] = z[q];
    t.htail = 0;
    t.hvalid = 1;
  }
}

// update(None), octet-wide: history_obs gets a None; the first miss after an observation
// freezes (x, P)
__device__ void ocs_update_none(const OcsDev& g, OcsTrk& t, int r) {
  const int observed = t.observed;
  if (observed && r < 7) {
    t.sx[r] = t.x[r];
#pragma unroll
    for (int j = 0; j < 7; j++) t.sP[r * 7 + j] = t.P[r * 7 + j];
  }
  if (r == 0) {
    t.det_ind = -1;
    t.htail++;
    if (t.htail >= g.max_obs) t.hvalid = 0;  // the box left the deque(maxlen=max_obs)
    if (observed) t.has_saved = 1;
    t.observed = 0;
  }
}

#include "bx_jv.h"

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

// lapjv(-cost, extend_cost=True): the shortest-augmenting-path solve + uniqueness test first,
// lapjv itself for a tied optimum (legacy_lap_ssp; the IoU-only BYTE / OCR rounds tie more often:
// non-overlapping pairs cost exactly 0, like lapjv's padding).  BX_OCS_SSP=0: lapjv always.
#ifndef BX_OCS_SSP
#define BX_OCS_SSP 1
#endif
__device__ __forceinline__ int ocs_lap(const double* C, int nr, int nc, JvLds& jv, int* out) {
#if BX_OCS_SSP
  bool jv_ran;
  return legacy_lap_ssp(C, nr, nc, jv, out, SyncBlock{}, jv_ran);
#else
  return legacy_lap(C, nr, nc, jv, out);
#endif
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
  L.jv.dc = g.dbg ? g.dbg + (size_t)seq * OCS_DBG + 24 : nullptr;
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
#ifdef BX_PHASE_TIMING
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif
  const int frame = sq[SO_FRAME] + 1;
  const int id0 = sq[SO_IDS];
  const int nt0 = sq[SO_NTR];
  const double thr = g.asso_threshold;
  const int ak = g.asso_kind;
  const double fw = g.fsz[2 * seq], fh = g.fsz[2 * seq + 1];

  // detections (setup_decorator's float32 rounding is the input format) and the splits
  for (int q = lane; q < n * 6; q += OW) L.dd[q] = (double)dets[(size_t)r0 * 6 + q];
  for (int p = lane; p < nt0; p += OW) L.lst2[p] = order[p];
  __syncthreads();
  const int nl = wave_compact(
      n, [&](int i) { const double c = L.dd[6 * i + 4]; return c > g.min_conf && c < g.det_thresh; },
      [&](int i, int p) { L.lo[p] = i; });
  const int nh = wave_compact(
      n, [&](int i) { return L.dd[6 * i + 4] > g.det_thresh; }, [&](int i, int p) { L.hi[p] = i; });

  const int oct = lane >> 3, r8 = lane & 7, rr8 = r8 < 7 ? r8 : 6;

  // predict every track (an octet per track); tracks whose prediction has a NaN leave the list
  // (ocsort.py:278-288).  tb row per kept track: box[4], k-previous obs[5], last_obs[5], vel[2]
  int nt = 0;
  for (int c = 0; c < nt0; c += 8) {
    const int p = c + oct;
    bool keep = false;
    int slot = -1;
    double v0 = 0.0, v1 = 0.0;  // this lane's two tb entries: [r8] and [8 + r8]
    if (p < nt0) {
      slot = L.lst2[p];
      OcsTrk& t = trk[slot];
      KfRow k;
      row_load(t.x, t.P, rr8, k);
      if ((osh(k.x, 6) + osh(k.x, 2)) <= 0 && rr8 == 6) k.x *= 0.0;
      kfo_predict(g, rr8, k);
      row_store(t.x, t.P, r8, k);
      const int age = t.age + 1;
      if (r8 == 0) {
        t.age = age;
        if (t.tsu > 0) t.hit_streak = 0;
        t.tsu++;
      }
      double xs[4], bx[4];
#pragma unroll
      for (int q = 0; q < 4; q++) xs[q] = osh(k.x, q);
      x_to_bbox(xs, bx);
      keep = !(isnan(bx[0]) || isnan(bx[1]) || isnan(bx[2]) || isnan(bx[3]));
      // k_previous_obs (ocsort.py:17-28) with the post-predict age
      int qq = -1;
      const int last_age = t.last_age;
      if (last_age >= 0) {
        qq = obs_first(t, age - g.delta_t, g.delta_t);
        if (qq < 0) qq = last_age & (OBS_KEEP - 1);  // observations[max(keys)]
      }
      auto val = [&](int e) -> double {
        if (e < 4) return e == 0 ? bx[0] : e == 1 ? bx[1] : e == 2 ? bx[2] : bx[3];
        if (e < 9) return qq < 0 ? -1.0 : t.obs_box[qq][e - 4];
        if (e < 14) return t.last_obs[e - 9];
        return t.has_vel ? t.vel[e - 14] : 0.0;
      };
      v0 = val(r8);
      v1 = val(8 + r8);
    }
    const unsigned long long m = __ballot(keep && r8 == 0);
    if (keep) {
      const int q = nt + __popcll(m & ((1ull << (lane & ~7)) - 1ull));
      if (r8 == 0) L.lst[q] = slot;
      double* row = tb + (size_t)q * TB;
      row[r8] = v0;
      row[8 + r8] = v1;
    }
    nt += __popcll(m);
  }
  __syncthreads();
  OSTAMP(1);

  // ---- first association: enhanced_associate(high dets, predicted tracks) -----------------
  int nm = 0, nud = 0, nut = 0;
  if (nt == 0) {
    for (int k = lane; k < nh; k += OW) L.ud[k] = k;
    nud = nh;
  } else {
    int nmi = 0;
    if (nh > 0) {
      // pass 1 (lane per track, dets broadcast from LDS): IoU > threshold counts for the
      // one-to-one test.  A pair without overlap has IoU 0/U, never above a threshold >= 0, so
      // only overlapping pairs divide.
      for (int k = lane; k < g.N; k += OW) L.rowcnt[k] = 0;
      __syncthreads();
      for (int c = 0; c < nt; c += OW) {
        const int ti = c + lane;
        if (ti < nt) {
          const double* bq = tb + (size_t)ti * TB;
          const double b0 = bq[0], b1 = bq[1], b2 = bq[2], b3 = bq[3];
          const double at = (b2 - b0) * (b3 - b1);
          int cc = 0;
          for (int d = 0; d < nh; d++) {
            const double* a = L.dd + 6 * L.hi[d];
            const double xx1 = fmax(a[0], b0), yy1 = fmax(a[1], b1);
            const double xx2 = fmin(a[2], b2), yy2 = fmin(a[3], b3);
            const double w = fmax(0.0, xx2 - xx1), h = fmax(0.0, yy2 - yy1);
            const double wh = w * h;
            // the other registry modes score disjoint pairs too: no shortcut for them
            if (wh > 0.0 || thr < 0.0 || ak != ASSO_IOU) {
              const double o = ak == ASSO_IOU ? wh / ((a[2] - a[0]) * (a[3] - a[1]) + at - wh)
                                              : asso_pair(ak, a, bq, fw, fh);
              if (o > thr) {
                atomicAdd(&L.rowcnt[d], 1);
                L.rowcol[d] = ti;
                cc++;
              }
            }
          }
          L.colcnt[ti] = cc;
        }
      }
      __syncthreads();
      OSTAMP(2);
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
      } else {
        // pass 2: the full cost -(IoU + direction consistency) and P4's legacy
        // linear_assignment of it
        double* C = (nh * nt <= g.cost_lds) ? L.cost : cost;
        for (int c = 0; c < nt; c += OW) {
          const int ti = c + lane;
          if (ti < nt) {
            const double* r = tb + (size_t)ti * TB;
            const double* p = r + 4;
            const double cx2 = (p[0] + p[2]) / 2.0, cy2 = (p[1] + p[3]) / 2.0;
            const double vy = r[14], vx = r[15];
            const double valid = p[4] < 0 ? 0.0 : 1.0;
            for (int d = 0; d < nh; d++) {
              const double* a = L.dd + 6 * L.hi[d];
              const double o = asso_pair(ak, a, r, fw, fh);
              // speed_direction_batch (association.py:10-20) against the k-previous obs
              const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
              double dx = cx1 - cx2, dy = cy1 - cy2;
              const double norm = sqrt(dx * dx + dy * dy) + 1e-6;
              dx = dx / norm;
              dy = dy / norm;
              double cth = vx * dx + vy * dy;
              cth = cth < -1 ? -1 : (cth > 1 ? 1 : cth);
              double ang = ocs_acos(cth);
              ang = (3.14159265358979323846 / 2.0 - fabs(ang)) / 3.14159265358979323846;
              const double mc = (valid * ang) * g.inertia;
              C[d * nt + ti] = -(o + mc);
            }
          }
        }
        __syncthreads();
        nmi = ocs_lap(C, nh, nt, L.jv, L.mi);
        OCOUNT(0, 1);
        OCOUNT(1, nh > nt ? nh : nt);
      }
      OSTAMP(3);
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
        ok = asso_pair(ak, L.dd + 6 * L.hi[d], tb + (size_t)ti * TB, fw, fh) >= thr;
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
  for (int c = 0; c < nm; c += 8) {
    const int q = c + oct;
    if (q < nm) {
      const double* r = L.dd + 6 * L.hi[L.mm[2 * q]];
      ocs_update_det(g, trk[L.lst[L.mm[2 * q + 1]]], r8, r, r[5], L.hi[L.mm[2 * q]]);
    }
  }
  __syncthreads();
  OSTAMP(4);

  // IoU matrix of detections (LDS rows `dsel`) x track boxes (tb rows `tsel`, offset `boff`):
  // its maximum (overlapping pairs only divide: a threshold >= 0 never passes 0/U), and, when
  // asked, the full matrix -IoU into C [nr][nc]
  auto iou_max = [&](int nr, const int* dsel, const int* dmap, int nc, const int* tsel, int boff) {
    double mx = -INF;
    for (int c = 0; c < nc; c += OW) {
      const int k = c + lane;
      if (k < nc) {
        const double* bq = tb + (size_t)tsel[k] * TB + boff;
        const double b0 = bq[0], b1 = bq[1], b2 = bq[2], b3 = bq[3];
        const double at = (b2 - b0) * (b3 - b1);
        for (int d = 0; d < nr; d++) {
          const double* a = L.dd + 6 * dsel[dmap ? dmap[d] : d];
          const double xx1 = fmax(a[0], b0), yy1 = fmax(a[1], b1);
          const double xx2 = fmin(a[2], b2), yy2 = fmin(a[3], b3);
          const double w = fmax(0.0, xx2 - xx1), h = fmax(0.0, yy2 - yy1);
          const double wh = w * h;
          if (ak != ASSO_IOU)
            mx = fmax(mx, asso_pair(ak, a, bq, fw, fh));
          else if (wh > 0.0 || thr < 0.0)
            mx = fmax(mx, wh / ((a[2] - a[0]) * (a[3] - a[1]) + at - wh));
        }
      }
    }
    for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    return mx;
  };
  auto iou_fill = [&](double* C, int nr, const int* dsel, const int* dmap, int nc, const int* tsel,
                      int boff) {
    for (int c = 0; c < nc; c += OW) {
      const int k = c + lane;
      if (k < nc) {
        const double* bq = tb + (size_t)tsel[k] * TB + boff;
        for (int d = 0; d < nr; d++)
          C[d * nc + k] = -asso_pair(ak, L.dd + 6 * dsel[dmap ? dmap[d] : d], bq, fw, fh);
      }
    }
    __syncthreads();
  };

  // ---- BYTE round on the low-confidence detections (ocsort.py:330-356) ---------------------
  if (g.use_byte && nl > 0 && nut > 0) {
    const double mx = iou_max(nl, L.lo, nullptr, nut, L.ut, 0);
    if (mx > thr) {
      double* C = (nl * nut <= g.cost_lds) ? L.cost : cost;
      iou_fill(C, nl, L.lo, nullptr, nut, L.ut, 0);
      const int np_ = ocs_lap(C, nl, nut, L.jv, L.mi);
      for (int k = lane; k < g.N; k += OW) L.fl[k] = 0;
      __syncthreads();
      for (int c = 0; c < np_; c += 8) {
        const int q = c + oct;
        if (q < np_) {
          const int dl = L.mi[2 * q], k = L.mi[2 * q + 1];
          if (!(-C[dl * nut + k] < thr)) {
            const double* r = L.dd + 6 * L.lo[dl];
            ocs_update_det(g, trk[L.lst[L.ut[k]]], r8, r, r[5], L.lo[dl]);
            if (r8 == 0) L.fl[L.ut[k]] = 2;  // removed
          }
        }
      }
      __syncthreads();
      for (int k = lane; k < nut; k += OW)
        if (L.fl[L.ut[k]] == 0) L.fl[L.ut[k]] = 1;
      __syncthreads();
      // np.setdiff1d: ascending, unique
      nut = wave_compact(nt, [&](int t) { return L.fl[t] == 1; }, [&](int t, int p) { L.ut[p] = t; });
      OCOUNT(2, 1);
    }
  }
  OSTAMP(5);

  // ---- OCR round on the last observations (ocsort.py:358-386) -------------------------------
  if (nud > 0 && nut > 0) {
    const double mx = iou_max(nud, L.hi, L.ud, nut, L.ut, 9);
    OSTAMP(6);
    if (mx > thr) {
      double* C = (nud * nut <= g.cost_lds) ? L.cost : cost;
      iou_fill(C, nud, L.hi, L.ud, nut, L.ut, 9);
      const int np_ = ocs_lap(C, nud, nut, L.jv, L.mi);
      OCOUNT(3, 1);
      OCOUNT(4, nud > nut ? nud : nut);
      for (int k = lane; k < g.N; k += OW) L.rowcnt[k] = L.fl[k] = 0;
      __syncthreads();
      for (int c = 0; c < np_; c += 8) {
        const int q = c + oct;
        if (q < np_) {
          const int a = L.mi[2 * q], k = L.mi[2 * q + 1];
          if (!(-C[a * nut + k] < thr)) {
            const int di = L.ud[a], ti = L.ut[k];
            const double* r = L.dd + 6 * L.hi[di];
            ocs_update_det(g, trk[L.lst[ti]], r8, r, r[5], L.hi[di]);
            if (r8 == 0) {
              L.rowcnt[di] = 2;
              L.fl[ti] = 2;
            }
          }
        }
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
  OSTAMP(7);
  for (int c = 0; c < nut; c += 8) {
    const int k = c + oct;
    if (k < nut) ocs_update_none(g, trk[L.lst[L.ut[k]]], r8);
  }

  // ---- new tracks for the unmatched high detections (free slots ascending) ----------------
  for (int s2 = lane; s2 < g.T; s2 += OW) L.fl[s2] = 0;
  __syncthreads();
  for (int p = lane; p < nt; p += OW) L.fl[L.lst[p]] = 1;
  __syncthreads();
  const int nfree = wave_compact(g.T, [&](int s2) { return L.fl[s2] == 0; }, [&](int s2, int p) { L.lst2[p] = s2; });
  int nnew = nud;
  if (nnew > nfree) {
    if (lane == 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
    nnew = nfree;
  }
  for (int c = 0; c < nnew; c += 8) {
    const int k = c + oct;
    if (k < nnew) {
      const int slot = L.lst2[k];
      const double* r = L.dd + 6 * L.hi[L.ud[k]];
      OcsTrk& t = trk[slot];
      const double w = r[2] - r[0], h = r[3] - r[1];
      const double z[4] = {r[0] + w / 2.0, r[1] + h / 2.0, w * h, w / (h + 1e-6)};
      if (r8 < 7) {
        t.x[r8] = r8 == 0 ? z[0] : r8 == 1 ? z[1] : r8 == 2 ? z[2] : r8 == 3 ? z[3] : 0.0;
        const double pd = r8 < 4 ? 10.0 : 10000.0;
#pragma unroll
        for (int j = 0; j < 7; j++) t.P[r8 * 7 + j] = j == r8 ? pd : 0.0;
      }
      if (r8 == 0) {
        t.observed = 0;
        t.has_saved = 0;
        t.hvalid = 0;
        t.htail = 0;
        t.id = id0 + k;
        t.conf = r[4];
        t.cls = r[5];
        t.det_ind = L.hi[L.ud[k]];
        for (int q = 0; q < 5; q++) t.last_obs[q] = -1.0;
        t.last_age = -1;
        for (int q = 0; q < OBS_KEEP; q++) t.obs_age[q] = -1;
        t.has_vel = 0;
        t.vel[0] = t.vel[1] = 0.0;
        t.tsu = t.hits = t.hit_streak = t.age = 0;
        L.lst[nt + k] = slot;
      }
    }
  }
  __syncthreads();
  const int ntr = nt + nnew;
  OSTAMP(8);

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
  OSTAMP(9);
  OCOUNT(5, nt);
  OCOUNT(6, nh);
  OCOUNT(7, 1);
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

// Op-level XYSR filter (bx_kf_xysr_*): one octet per track running the frame kernel's octet code
// (kfo_predict / kfo_update), so the op and the tracker are bit-identical.  op 0 initiate
// (ocsort.py:83-111 from xyxy boxes), 1 predict (ocsort.py:177-180: the s + ds <= 0 clamp, then
// F/Q of the tracker), 2 update (xysr_kf.py:256-283 with R = diag(1, 1, 10, 10)).
__global__ __launch_bounds__(256) void kf_xysr_kernel(int op, int n, double* __restrict__ x,
                                                      double* __restrict__ P,
                                                      const double* __restrict__ arg, double q_xy,
                                                      double q_s) {
  const int gt = blockIdx.x * 256 + threadIdx.x;
  const int k = gt >> 3, r = gt & 7, rr = r < 7 ? r : 6;
  if (k >= n) return;  // whole octets leave together
  double* xk = x + 7 * (size_t)k;
  double* Pk = P + 49 * (size_t)k;
  if (op == 0) {
    const double* b = arg + 4 * (size_t)k;
    const double w = b[2] - b[0], h = b[3] - b[1];
    const double z[4] = {b[0] + w / 2.0, b[1] + h / 2.0, w * h, w / (h + 1e-6)};
    if (r < 7) {
      xk[r] = r < 4 ? z[r] : 0.0;
      for (int j = 0; j < 7; j++) Pk[7 * r + j] = j == r ? (r < 4 ? 10.0 : 10000.0) : 0.0;
    }
    return;
  }
  KfRow kr;
  row_load(xk, Pk, rr, kr);
  if (op == 1) {
    OcsDev g;
    g.q_xy = q_xy;
    g.q_s = q_s;
    if (rr == 6 && xk[6] + xk[2] <= 0) kr.x *= 0.0;
    kfo_predict(g, rr, kr);
  } else {
    const double* zk = arg + 4 * (size_t)k;
    const double z[4] = {zk[0], zk[1], zk[2], zk[3]};
    kfo_update(rr, kr, z);
  }
  row_store(xk, Pk, r, kr);
}

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
  // pinned mirrors for update_host (asynchronous copies, one sync per frame) and the counters
  // row of the last update_host sequence (bx_ocsort_counters_host answers from it)
  float* p_dets = nullptr;
  double* p_out = nullptr;
  int* p_cnt = nullptr;
  int* p_sq = nullptr;
  int cache_seq = -1;
  // per_class host path (bx_ocsort_update_classes_host): per sequence the local -> class-global
  // track id map and the local id counter the map covers; class offsets [C+1], counts [C]
  std::vector<std::vector<int>> gid;
  std::vector<int> lids;
  int* h_coff = nullptr;
  int* h_ccnt = nullptr;
  int ncls_alloc = 0;
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
  if (c->n_seq <= 0 || c->track_cap <= 0 || c->det_cap <= 0 || c->track_cap > 512 ||
      c->det_cap > 512)
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
  if (c->asso_kind < ASSO_IOU || c->asso_kind > ASSO_CENTROID) {
    delete e;
    return bx_record_error(BX_ERR_INVALID, "unknown asso_kind");
  }
  d.asso_kind = c->asso_kind;
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
  const size_t o_fsz = carve_b(S * 2 * sizeof(double));
#ifdef BX_PHASE_TIMING
  const size_t o_dbg = carve_b(S * OCS_DBG * sizeof(unsigned long long));
#endif
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
  d.fsz = (double*)(base + o_fsz);
  {
    std::vector<double> f(2 * S);
    for (size_t k = 0; k < S; k++) {
      f[2 * k] = c->frame_w;
      f[2 * k + 1] = c->frame_h;
    }
    OCHK(hipMemcpy(d.fsz, f.data(), sizeof(double) * 2 * S, hipMemcpyHostToDevice));
  }
#ifdef BX_PHASE_TIMING
  d.dbg = (unsigned long long*)(base + o_dbg);
#else
  d.dbg = nullptr;
#endif
  OCHK(bx_lds_attr((const void*)ocsort_frame_kernel, e->lds));
  OCHK(hipMalloc(&e->h_dets, sizeof(float) * 6 * d.D));
  OCHK(hipMalloc(&e->h_off, sizeof(int) * 2));
  OCHK(hipMalloc(&e->h_out, sizeof(double) * 8 * d.D));
  OCHK(hipMalloc(&e->h_cnt, sizeof(int)));
  OCHK(hipHostMalloc(&e->p_dets, sizeof(float) * 6 * d.D));
  OCHK(hipHostMalloc(&e->p_out, sizeof(double) * 8 * d.D));
  OCHK(hipHostMalloc(&e->p_cnt, sizeof(int) * 4));
  OCHK(hipHostMalloc(&e->p_sq, sizeof(int) * SQO));
  *out = e;
  return BX_OK;
}

int bx_ocsort_copy_state(bx_ocsort* dst, bx_ocsort* src) {
  if (!dst || !src) return bx_record_error(BX_ERR_INVALID, "null engine");
  const OcsDev &a = src->dev, &b = dst->dev;
  if (a.S != b.S || b.T < a.T || b.D < a.D)
    return bx_record_error(BX_ERR_INVALID, "bx_ocsort_copy_state: destination must have the "
                                           "source's sequences and at least its capacities");
  OCHK(hipDeviceSynchronize());
  const size_t S = a.S, Ta = a.T, Tb = b.T;
  // per-slot records [S][T] and the list order [S][T]; per-sequence scalars and frame sizes
  OCHK(hipMemcpy2D(b.trk, Tb * sizeof(OcsTrk), a.trk, Ta * sizeof(OcsTrk), Ta * sizeof(OcsTrk), S,
                   hipMemcpyDeviceToDevice));
  OCHK(hipMemcpy2D(b.order, Tb * sizeof(int), a.order, Ta * sizeof(int), Ta * sizeof(int), S,
                   hipMemcpyDeviceToDevice));
  OCHK(hipMemcpy(b.seqst, a.seqst, S * SQO * sizeof(int), hipMemcpyDeviceToDevice));
  OCHK(hipMemcpy(b.fsz, a.fsz, S * 2 * sizeof(double), hipMemcpyDeviceToDevice));
  OCHK(hipMemcpy(b.status, a.status, 4 * sizeof(int), hipMemcpyDeviceToDevice));
  dst->gid = src->gid;
  dst->lids = src->lids;
  dst->cache_seq = -1;
  OCHK(hipDeviceSynchronize());
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
  (void)hipHostFree(e->p_dets);
  (void)hipHostFree(e->p_out);
  (void)hipHostFree(e->p_cnt);
  (void)hipHostFree(e->p_sq);
  (void)hipFree(e->h_coff);
  (void)hipFree(e->h_ccnt);
  delete e;
  return BX_OK;
}

int bx_ocsort_reset(bx_ocsort* e, int seq0, int nseq, void* stream) {
  if (!e || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad sequence range");
  if (!nseq) return BX_OK;
  e->cache_seq = -1;
  hipLaunchKernelGGL(ocsort_reset_kernel, dim3((nseq * SQO + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, e->dev, seq0, nseq);
  OCHK(hipGetLastError());
  for (int s = seq0; s < seq0 + nseq && !e->lids.empty(); s++) {
    e->lids[s] = 0;
    e->gid[s].clear();
  }
  return BX_OK;
}

int bx_ocsort_step(bx_ocsort* e, int seq0, int nseq, const float* dets, const int32_t* det_off,
                   double* out, int32_t* out_count, void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_step");
  e->cache_seq = -1;
  return launch(e, seq0, nseq, dets, det_off, out, out_count, (hipStream_t)stream);
}

int bx_ocsort_update_host(bx_ocsort* e, int seq, const float* dets, int n, double* out,
                          int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!dets || !out)) || !n_out)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_update_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  hipStream_t st = (hipStream_t)stream;
  // pinned mirrors: asynchronous copies in, the frame, rows (at most n) + count + status +
  // counters back, one synchronisation
  if (n) {
    memcpy(e->p_dets, dets, sizeof(float) * 6 * n);
    OCHK(hipMemcpyAsync(e->h_dets, e->p_dets, sizeof(float) * 6 * n, hipMemcpyHostToDevice, st));
  }
  e->p_cnt[2] = 0;
  e->p_cnt[3] = n;
  OCHK(hipMemcpyAsync(e->h_off, e->p_cnt + 2, sizeof(int) * 2, hipMemcpyHostToDevice, st));
  e->cache_seq = -1;
  int rc = launch(e, seq, 1, e->h_dets, e->h_off, e->h_out, e->h_cnt, st);
  if (rc) return rc;
  OCHK(hipMemcpyAsync(e->p_cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  OCHK(hipMemcpyAsync(e->p_cnt + 1, e->dev.status, sizeof(int), hipMemcpyDeviceToHost, st));
  if (n) OCHK(hipMemcpyAsync(e->p_out, e->h_out, sizeof(double) * 8 * n, hipMemcpyDeviceToHost, st));
  OCHK(hipMemcpyAsync(e->p_sq, e->dev.seqst + (size_t)seq * SQO, sizeof(int) * SQO,
                      hipMemcpyDeviceToHost, st));
  OCHK(hipStreamSynchronize(st));
  const int cnt = e->p_cnt[0], status = e->p_cnt[1];
  e->cache_seq = seq;
  if (cnt) memcpy(out, e->p_out, sizeof(double) * 8 * cnt);
  *n_out = cnt;
  if (status)
    return bx_record_error(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

// per_class=True (basetracker.py:155-201): OCSort keeps all of its state in active_tracks, so
// the decorator's per-class swap gives every class an isolated tracker — only the frame counter
// (equal for all: each class is called once per frame) and KalmanBoxTracker.count (class-global,
// ocsort.py:61,115-116) are shared.  Here class c is engine sequence seq0 + c and the whole frame
// is ONE launch over the n_classes sequences; ids are then renumbered into the reference's
// class-global order (births of class 0 first, then class 1, ...), continuing *id_count.
int bx_ocsort_update_classes_host(bx_ocsort* e, int seq0, int n_classes, const float* dets,
                                  int n, int* id_count, double* out, int* n_out, void* stream) {
  if (!e || n_classes <= 0 || seq0 < 0 || seq0 + n_classes > e->dev.S || n < 0 ||
      (n && !dets) || !n_out || !id_count)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_update_classes_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  hipStream_t st = (hipStream_t)stream;
  const int C = n_classes;
  if (e->lids.empty()) {
    e->lids.assign(e->dev.S, 0);
    e->gid.assign(e->dev.S, {});
  }
  if (e->ncls_alloc < C) {
    (void)hipFree(e->h_coff);
    (void)hipFree(e->h_ccnt);
    OCHK(hipMalloc(&e->h_coff, sizeof(int) * (C + 1)));
    OCHK(hipMalloc(&e->h_ccnt, sizeof(int) * C));
    e->ncls_alloc = C;
  }
  auto cls_of = [&](int i) -> int {
    const float v = dets[6 * i + 5];
    return (v >= 0.f && v < (float)C && v == (float)(int)v) ? (int)v : -1;
  };
  std::vector<int> cnt(C + 1, 0);
  for (int i = 0; i < n; i++)
    if (cls_of(i) >= 0) cnt[cls_of(i) + 1]++;
  for (int c = 0; c < C; c++) cnt[c + 1] += cnt[c];
  const int m = cnt[C];
  std::vector<int> fill(cnt.begin(), cnt.end() - 1);
  std::vector<float> hd((size_t)6 * (m ? m : 1));
  for (int i = 0; i < n; i++) {
    const int c = cls_of(i);
    if (c >= 0) memcpy(&hd[6 * (size_t)fill[c]++], dets + 6 * (size_t)i, 6 * sizeof(float));
  }
  if (m) OCHK(hipMemcpyAsync(e->h_dets, hd.data(), sizeof(float) * 6 * m, hipMemcpyHostToDevice, st));
  OCHK(hipMemcpyAsync(e->h_coff, cnt.data(), sizeof(int) * (C + 1), hipMemcpyHostToDevice, st));
  e->cache_seq = -1;
  int rc = launch(e, seq0, C, e->h_dets, e->h_coff, e->h_out, e->h_ccnt, st);
  if (rc) return rc;
  std::vector<int> oc(C), sq((size_t)C * SQO);
  std::vector<double> ho((size_t)8 * (m ? m : 1));
  OCHK(hipMemcpyAsync(oc.data(), e->h_ccnt, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  if (m) OCHK(hipMemcpyAsync(ho.data(), e->h_out, sizeof(double) * 8 * m, hipMemcpyDeviceToHost, st));
  OCHK(hipMemcpyAsync(sq.data(), e->dev.seqst + (size_t)seq0 * SQO, sizeof(int) * C * SQO,
                      hipMemcpyDeviceToHost, st));
  OCHK(hipStreamSynchronize(st));
  int status = 0;
  OCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status)
    return bx_record_error(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  int g = *id_count;
  for (int c = 0; c < C; c++) {  // births in class order take the next class-global ids
    std::vector<int>& map = e->gid[seq0 + c];
    for (int l = e->lids[seq0 + c]; l < sq[(size_t)c * SQO + SO_IDS]; l++) {
      if ((int)map.size() <= l) map.resize(l + 1, -1);
      map[l] = g++;
    }
    e->lids[seq0 + c] = sq[(size_t)c * SQO + SO_IDS];
  }
  *id_count = g;
  int k = 0;
  for (int c = 0; c < C; c++)
    for (int j = 0; j < oc[c]; j++, k++) {
      double* o = out + 8 * (size_t)k;
      memcpy(o, &ho[8 * ((size_t)cnt[c] + j)], 8 * sizeof(double));
      o[4] = (double)(e->gid[seq0 + c][(int)o[4] - 1] + 1);
    }
  *n_out = k;
  return BX_OK;
}

static int kf_xysr_launch(int op, int n, double* x, double* P, const double* arg, double q_xy,
                          double q_s, void* stream) {
  if (n < 0 || !x || !P || (op != 1 && n && !arg))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_kf_xysr_*");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_xysr_kernel, dim3((8 * n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     op, n, x, P, arg, q_xy, q_s);
  OCHK(hipGetLastError());
  return BX_OK;
}

int bx_kf_xysr_initiate(int n, const double* bbox, double* x, double* P, void* stream) {
  return kf_xysr_launch(0, n, x, P, bbox, 0.0, 0.0, stream);
}
int bx_kf_xysr_predict(int n, double* x, double* P, double q_xy_scaling, double q_s_scaling,
                       void* stream) {
  return kf_xysr_launch(1, n, x, P, nullptr, q_xy_scaling, q_s_scaling, stream);
}
int bx_kf_xysr_update(int n, double* x, double* P, const double* z, void* stream) {
  return kf_xysr_launch(2, n, x, P, z, 0.0, 0.0, stream);
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
  if (seq == e->cache_seq) {
    memcpy(s, e->p_sq, sizeof(s));
  } else {
    OCHK(hipDeviceSynchronize());
    OCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQO, sizeof(s), hipMemcpyDeviceToHost));
  }
  if (frame_count) *frame_count = s[SO_FRAME];
  if (id_count) *id_count = s[SO_IDS];
  if (n_tracks) *n_tracks = s[SO_NTR];
  return BX_OK;
}

int bx_ocsort_set_id_count(bx_ocsort* e, int seq, int id_count, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  e->cache_seq = -1;
  OCHK(hipMemcpyAsync(e->dev.seqst + (size_t)seq * SQO + SO_IDS, &id_count, sizeof(int),
                      hipMemcpyHostToDevice, (hipStream_t)stream));
  OCHK(hipStreamSynchronize((hipStream_t)stream));
  return BX_OK;
}

int bx_ocsort_set_frame_size(bx_ocsort* e, int seq, double w, double h, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  const double f[2] = {w, h};
  OCHK(hipMemcpyAsync(e->dev.fsz + 2 * (size_t)seq, f, sizeof(f), hipMemcpyHostToDevice,
                      (hipStream_t)stream));
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
    // a per-class sequence reports the class-global id its rows carry (minus one)
    const bool g = seq < (int)e->gid.size() && t.id >= 0 && t.id < (int)e->gid[seq].size();
    if (ids) ids[k] = g ? e->gid[seq][t.id] : t.id;
    if (x) memcpy(x + 7 * k, t.x, sizeof(t.x));
    if (p) memcpy(p + 49 * k, t.P, sizeof(t.P));
  }
  *n = nt;
  return BX_OK;
}

int bx_ocsort_state_set_host(bx_ocsort* e, int seq, int n, const int32_t* ids, const double* x,
                             const double* p) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !ids))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_state_set_host");
  OCHK(hipDeviceSynchronize());
  int s[SQO];
  OCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQO, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[SO_NTR];
  std::vector<int> ord(nt);
  if (nt)
    OCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int j = 0; j < n; j++) {
    OcsTrk* dt = nullptr;
    OcsTrk t;
    for (int k = 0; k < nt && !dt; k++) {
      OcsTrk* cand = e->dev.trk + (size_t)seq * e->dev.T + ord[k];
      OCHK(hipMemcpy(&t, cand, sizeof(OcsTrk), hipMemcpyDeviceToHost));
      if (t.id == ids[j]) dt = cand;
    }
    if (!dt) return bx_record_error(BX_ERR_INVALID, "state_set: no live track with that id");
    if (x) memcpy(t.x, x + 7 * j, sizeof(t.x));
    if (p) memcpy(t.P, p + 49 * j, sizeof(t.P));
    OCHK(hipMemcpy(dt, &t, sizeof(OcsTrk), hipMemcpyHostToDevice));
  }
  return BX_OK;
}

int bx_ocsort_frame_stats_host(bx_ocsort* e, int seq0, int nseq, int64_t* sums) {
  if (!e || !sums || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ocsort_frame_stats_host");
  std::vector<int> s((size_t)nseq * SQO);
  OCHK(hipDeviceSynchronize());
  if (nseq)
    OCHK(hipMemcpy(s.data(), e->dev.seqst + (size_t)seq0 * SQO, sizeof(int) * s.size(),
                   hipMemcpyDeviceToHost));
  int64_t t = 0, o = 0, f = 0;
  for (int k = 0; k < nseq; k++) {
    t += s[(size_t)k * SQO + SO_NTR];
    o += s[(size_t)k * SQO + SO_NOUT];
    f = s[(size_t)k * SQO + SO_FRAME] > f ? s[(size_t)k * SQO + SO_FRAME] : f;
  }
  sums[0] = t;
  sums[1] = o;
  sums[2] = f;
  return BX_OK;
}

// diagnostic (not in the public header): the phase stamps of every sequence, [S][OCS_DBG]
int bx_ocsort_debug_host(bx_ocsort* e, unsigned long long* out) {
  if (!e || !out || !e->dev.dbg) return bx_record_error(BX_ERR_INVALID, "not a timing build");
  OCHK(hipDeviceSynchronize());
  OCHK(hipMemcpy(out, e->dev.dbg, sizeof(unsigned long long) * OCS_DBG * e->dev.S,
                 hipMemcpyDeviceToHost));
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
