// bx_strongsort.hip — the fork's "enhanced" StrongSort per-frame update on MI355X.
//
// Reference: boxmot/trackers/strongsort/strongsort.py:45-345 (StrongSort.update, detection
// quality, crowd mode), sort/tracker.py:63-344 (Tracker: three-stage matching, ID recovery,
// lost buffer, partial_fit), sort/track.py:76-400 (Track), sort/linear_assignment.py:14-618
// (matching_cascade, min_cost_matching, gate_cost_matrix + cost shaping,
// NearestNeighborDistanceMetric), sort/iou_matching.py:10-87, utils/occlusion_handler.py:45-87,
// 464-490 (detect_crowd_situations).  With P6 and handle_occlusions=False.
//
// Per frame, ten launches on the caller's stream:
//   ss_prep_kernel   wave per detection: the feature's wave-order norm (quality; BLAS order of
//                    the reference unpinned), its numpy pairwise norm, the NN-normalised row
//                    feat/(‖·‖₂+1e-8) and the track-feature row feat/(‖·‖_wave+1e-8) with its
//                    norms
//   ss_nn_kernel     wave per 1-4 confirmed tracks: min over its distinct gallery samples of
//                    1 − clip(ŝ·d̂) for every detection — the (samples × F)·(F × dets)
//                    contraction on the fp64 matrix cores (v_mfma_f64_16x16x4f64, ascending-k
//                    chain = the oracle's fma chain), max over rows by wave shuffles
//   ss_rec_kernel    wave per (lost track, detection): ID-recovery cosine similarity
//   ss_crowd_kernel  grid: detect_crowd_situations' pair test over all track pairs
//   ss_pre_kernel    one wave per sequence: crowd mode, CMC warp, detection quality + stable
//                    sort, Kalman predict
//   ss_cost_kernel   wave per confirmed track: gating + motion/quality cost shaping of the
//                    track against every detection (lanes over detections)
//   ss_match_kernel  one wave per sequence: the matching cascade (levels gathered from the
//                    cost kernel's matrix, scipy's linear_sum_assignment restated
//                    wave-parallel), the IoU stage
//   ss_update_kernel wave per match: Kalman update, feature EMA vector + norms, track scalars
//   ss_post_kernel   one wave per sequence: misses, ID recovery, births (lane per birth), lost
//                    buffer, output rows
//   ss_fit_kernel    wave per listed / lost track: partial_fit (append + budget truncation by
//                    rank in LDS), pool bookkeeping, the next frame's gallery queries
// Every floating-point expression restates oracle/bxo_strongsort.c operation for operation.
//
// Track state lives in HBM: SsTrk slots, each with a private pool of `vec_cap` feature vectors
// (its features list and its gallery samples reference pool entries: the gallery keeps (pool
// index, sample quality) pairs in the reference's list order, duplicates included, so
// partial_fit's stable sort-and-truncate is reproduced exactly while each vector is stored once).
#include <float.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bxstrongsort.h"
#include "bx_device.h"

using namespace bx;

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)
hipError_t bx_lds_attr(const void* kern, size_t bytes);  // bx_engine.hip (never lowers a limit)

namespace {

#include "bx_jv.h"

constexpr int MAXF = 10, MAXC = 20, MAXH = 10, LOSTN = 30;
constexpr double SS_INFTY = 1e5, SS_GATE = 9.4877;

struct SsTrk {
  double mean[8], cov[64];
  double conf, cls, det_ind, base_alpha, quality, stability, app_cons, motion_cons;
  double vel[MAXH][2], pos[MAXH][2];
  double confh[MAXC];
  int id, state, hits, age, tsu, max_age, n_init;
  int nvel, npos, nconf, nfeat, missed, confirmed_det, low_streak, high_streak, lost_frame;
  int gal_n;                 // gallery length (entries sorted by quality desc, time asc)
  int gal_clock;             // partial_fit append counter: the entries' insertion times
  int born_dk;               // input detection of this frame's birth (first vector copied by
                             // ss_fit_kernel), else -1
  int feat[MAXF];
  unsigned long long vmask;  // pool entries in use (features or gallery)
  unsigned long long gmask;  // pool entries referenced by the gallery
};

enum {
  Q_FRAME = 0, Q_NEXTID, Q_NTR, Q_NLOST, Q_CROWD, Q_ORIG, Q_OMAXAGE, Q_OBUDGET, Q_MAXAGE,
  Q_BUDGET, Q_HIST, Q_NNL, Q_NK, Q_NT0, Q_NOUT, Q_ROWS, Q_ROWSL,
  Q_NM, Q_NAUD, Q_FID, Q_ANYF, Q_NFUT, Q_NDUP,
  Q_CROWDN,  // high-overlap track pairs counted by ss_crowd_kernel for this frame  // handed from ss_match_kernel / ss_post_kernel to the next launch
  // LSAP statistics since creation (bx_ss_lsap_stats_host): solves; certified unique; certified
  // up to rejected (clamped) pairs; real ties re-solved in scipy's order; stages restarted in
  // scipy's order (a real tie after a level whose unmatched order was not certified)
  Q_LCALL, Q_LUNIQ, Q_LCLAMP, Q_LTIE, Q_LRESTART,
  Q_NNCTR,  // ss_nn_kernel's work counters, one per XCD (zeroed by ss_prep_kernel's pack block)
  SQS = Q_NNCTR + 8
};

struct SsDev {
  int S, T, D, F, VP, GB, N;
  double min_conf, max_iou, mc_lambda, ema_alpha, thi, tlo, idw;
  int n_init, crowd, born;
  SsTrk* trk;     // [S][T]
  int* gal_v;     // [S][T][GB] pool index
  double* gal_q;  // [S][T][GB] sample quality (wave norm)
  int* gal_t;     // [S][T][GB] insertion time (the reference list's order among equal qualities)
  double* vec;    // [S][T][VP][F]
  double* vecn;   // [S][T][VP][F] vec / vden: the sample as the NN metric normalises it
  double* vden;   // [S][T][VP] numpy pairwise norm + 1e-8 (NN sample normalisation)
  double* vwn;    // [S][T][VP] wave-order norm
  int* sq;        // [S][SQS]
  double* sqd;    // [S][2] metric.matching_threshold, its original
  int* order;     // [S][T] track list (slots)
  int* lost;      // [S][LOSTN] lost buffer (slots)
  int* nnl;       // [S][T] confirmed slots queried by the next frame's gallery distance
  int* pk;        // [S][T+3] packs of nnl for ss_nn_kernel: starts pk[0..P], P at pk[T+1];
                  // pk[T+2]: a detection passes min_conf this frame (ss_motion_kernel)
  double* nnd;    // [S][T][D] NN distance by (slot, input detection)
  double* dprep;  // [S][D][4] wave norm, pairwise norm of feat; wave norm, den of nf
  double* dn;     // [S][D][F] feat / (pairwise norm + 1e-8)
  double* nf;     // [S][D][F] feat / (wave norm + 1e-8)
  double* recsim; // [S][LOSTN][D]
  double* cost;   // [S][2T*D] scratch cost matrices
  double* cfull;  // [S][T][D] stage 1/2 cost by (cascade rank, sorted detection)
  double* cfullT; // [S][D][T] the same, detection-major
  int16_t* tlist; // [S][T][SS_TL] by cascade rank: the sorted detections of its real entries
  int* tcnt;      // [S][T] their count (-1: more than SS_TL, or a NaN cost in the row)
  int* crank;     // [S][T] cascade rank of a list position (confirmed tracks), else -1
  double* ckey;   // [S][T] quality + stability by list position
  int* ctsu;      // [S][T] time_since_update by list position (confirmed), else -1
  int* cpos;      // [S][T] list position of a cascade rank
  int* ncf;       // [S] confirmed tracks (ranks 0..ncf-1)
  double* fdt;    // [S][D][DTW] this frame's detection table (kept across the frame's launches)
  int* fdord;     // [S][D] detections in quality order
  int* faud;      // [S][D] unmatched detections after the three stages
  int* fmt;       // [S][4(D+2)] matches (track list position, sorted detection)
  int* ffut;      // [S][3T] unmatched track positions (duplicates kept: mark_missed per entry)
  int* wsi;       // [S][WSI] int scratch
  double* wsd;    // [S][WSD] double scratch
  int wsi_n, wsd_n;
  int ws_lds;     // 1: the whole frame-kernel workspace in LDS, 2: its LSAP state only
  int lsap_fast;  // 1: LSAPs solved then certified (scipy's order only on a tie); 0: scipy's order
  int* status;
  unsigned long long* dbg;  // [S][SS_DBG] phase stamps (diagnostic builds only, else null)
};

// Diagnostic phase stamps and counters (build with -DBX_PHASE_TIMING; never shipped): per
// sequence, cycles accumulated per phase [0, 16), sub-phase cycles / counters [16, 32).
constexpr int SS_DBG = 48;
constexpr int SS_TL = 16;  // real entries listed per track for the LSAP's sparse first step
#ifdef BX_PHASE_TIMING
#define SSTAMP(k)                                                                    \
  do {                                                                               \
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");                           \
    __builtin_amdgcn_wave_barrier();                                                 \
    if ((threadIdx.x & 63) == 0 && g.dbg) {                                          \
      const unsigned long long _now = __builtin_amdgcn_s_memtime();                  \
      g.dbg[(size_t)seq * SS_DBG + (k)] += _now - t_last;                            \
      t_last = _now;                                                                 \
    }                                                                                \
  } while (0)
#define SCOUNT(k, v)                                                                 \
  do {                                                                               \
    if ((threadIdx.x & 63) == 0 && g.dbg) g.dbg[(size_t)seq * SS_DBG + 16 + (k)] += (v);    \
  } while (0)
#define SS_NOW() __builtin_amdgcn_s_memtime()
#else
#define SSTAMP(k) \
  do {            \
  } while (0)
#define SCOUNT(k, v) \
  do {               \
  } while (0)
#define SS_NOW() 0ull
#endif

__device__ __forceinline__ double* vecp(const SsDev& g, int seq, int slot, int v) {
  return g.vec + ((((size_t)seq * g.T + slot) * g.VP + v) * (size_t)g.F);
}
// Where element q of a stored NN operand row (a gallery vector's vecn row, a detection's dn row)
// lives: within each whole 8-element block (F even; the rest in order) the order is
// [0 4 1 5 2 6 3 7], so lane group m's 16-byte load of positions (2m, 2m + 1) holds exactly the
// k-slots the fp64 MFMA takes from it in its two k-steps (k0 + m, k0 + 4 + m): ss_nn_kernel feeds
// its loads to the matrix cores as they arrive, and each output's chain stays ascending in k.
__device__ __forceinline__ int nn_pos(int q, int F) {
  const int FB = (F & 1) ? 0 : F - F % 8;
  return q < FB ? (q & ~7) | ((q & 3) << 1) | ((q >> 2) & 1) : q;
}
__device__ __forceinline__ double* vecnp(const SsDev& g, int seq, int slot, int v) {
  return g.vecn + ((((size_t)seq * g.T + slot) * g.VP + v) * (size_t)g.F);
}
__device__ __forceinline__ size_t vidx(const SsDev& g, int seq, int slot, int v) {
  return ((size_t)seq * g.T + slot) * g.VP + v;
}

// ---- wave-cooperative vector primitives (64 lanes) ----------------------------------------
// wave-order dot (oracle wave_dot): lane l sums a[l]b[l], a[l+64]b[l+64], ... then xor butterfly
__device__ __forceinline__ double wdot(const double* a, const double* b, int n) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int k = lane; k < n; k += 64) s += a[k] * b[k];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  return s;
}

// the calling wave's LDS / global writes visible to its other lanes (every user of it runs a whole
// wave on its own data: one wave per workgroup, or waves with disjoint scratch)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// numpy pairwise sum of x[k]^2 (PW_BLOCKSIZE 128): leaves found by numpy's halving, each leaf
// summed by 8 lanes (lane j keeps numpy's accumulator r[j]), the leaves folded in the tree's
// order by lane 0.  Called by all 64 lanes; result valid on every lane.
constexpr int PW_MAXLEAF = 160;
__device__ int pw_leaves(int n, int* lo, int* ln) {
  int cnt = 0, so[24], sn[24], top = 1;
  so[0] = 0;
  sn[0] = n;
  while (top > 0) {
    const int o = so[--top], m = sn[top];
    if (m <= 128) {
      lo[cnt] = o;
      ln[cnt] = m;
      cnt++;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    so[top] = o + n2;
    sn[top] = m - n2;
    top++;
    so[top] = o;
    sn[top] = n2;
    top++;
  }
  return cnt;
}
__device__ double pw_fold(int n, const double* leaf) {
  double acc[24];
  int ap = 0, li = 0, sn[24], st[24], top = 1;
  sn[0] = n;
  st[0] = 0;
  while (top > 0) {
    const int t = top - 1, m = sn[t];
    if (m <= 128) {
      acc[ap++] = leaf[li++];
      top--;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (st[t] == 0) {
      st[t] = 1;
      sn[top] = n2;
      st[top] = 0;
      top++;
    } else if (st[t] == 1) {
      st[t] = 2;
      sn[top] = m - n2;
      st[top] = 0;
      top++;
    } else {
      const double b = acc[--ap], a = acc[--ap];
      acc[ap++] = a + b;
      top--;
    }
  }
  return acc[0];
}
// sqrt of numpy's pairwise sum of squares of x[0..n); lo/ln/leaf: per-wave scratch
__device__ double wpw_norm(const double* x, int n, int* lo, int* ln, double* leaf) {
  const int lane = threadIdx.x & 63;
  const int nlf = n >> 7;
  if ((n & 127) == 0 && nlf > 0 && (nlf & (nlf - 1)) == 0 && nlf <= 32) {
    // n = 128·2^j: the split tree is balanced over 128-element leaves in order, so leaf sums
    // (8 lanes each, numpy's 8 accumulators) fold by xor shuffles across lane groups; up to 8
    // leaves per pass, the passes' sums folded as the tree's top levels
    const int grp = lane >> 3, k = lane & 7, np = nlf > 8 ? nlf / 8 : 1, gl = nlf < 8 ? nlf : 8;
    double part[4];
#pragma unroll
    for (int p = 0; p < 4; p++) {
      part[p] = 0.0;
      if (p < np) {
        double r = 0.0;
        if (grp < gl) {
          const double* o = x + 128 * (p * 8 + grp);
          r = o[k] * o[k];
          for (int i = 8 + k; i < 128; i += 8) r += o[i] * o[i];
        }
        r = r + __shfl_xor(r, 1);
        r = r + __shfl_xor(r, 2);
        r = r + __shfl_xor(r, 4);
        for (int d = 8; d < 8 * gl; d <<= 1) r = r + __shfl_xor(r, d);
        part[p] = r;
      }
    }
    const double s = np == 1 ? part[0]
                     : np == 2 ? part[0] + part[1]
                               : (part[0] + part[1]) + (part[2] + part[3]);
    return sqrt(__shfl(s, 0));
  }
  if (lane == 0) {
    const int c = pw_leaves(n, lo, ln);
    ln[PW_MAXLEAF - 1] = c;
  }
  wsync();
  const int nl = ln[PW_MAXLEAF - 1];
  for (int base = 0; base < nl; base += 8) {
    const int li = base + (lane >> 3), k = lane & 7;
    double r = 0.0;
    int m = 0, o = 0;
    if (li < nl) {
      m = ln[li];
      o = lo[li];
      if (m >= 8) {
        const int full = m - (m % 8);
        r = x[o + k] * x[o + k];
        for (int i = 8 + k; i < full; i += 8) r += x[o + i] * x[o + i];
      }
    }
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (li < nl && k == 0) {
      double res;
      if (m < 8) {
        res = 0.0;
        for (int i = 0; i < m; i++) res += x[o + i] * x[o + i];
      } else {
        res = r;
        for (int i = m - (m % 8); i < m; i++) res += x[o + i] * x[o + i];
      }
      leaf[li] = res;
    }
  }
  wsync();
  double s = 0.0;
  if (lane == 0) s = pw_fold(n, leaf);
  s = __shfl(s, 0);
  wsync();
  return sqrt(s);
}

// numpy pairwise sum of a short run (n <= 20: the confidence history), one lane
__device__ double pw_sum_short(const double* x, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; i++) r += x[i];
    return r;
  }
  double r[8];
  for (int k = 0; k < 8; k++) r[k] = x[k];
  int i;
  for (i = 8; i < n - (n % 8); i += 8)
    for (int k = 0; k < 8; k++) r[k] += x[i + k];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; i++) res += x[i];
  return res;
}
__device__ double np_mean(const double* x, int n) { return pw_sum_short(x, n) / n; }
__device__ double np_std(const double* x, int n) {
  const double m = np_mean(x, n);
  double d[MAXC];
  for (int i = 0; i < n; i++) {
    d[i] = x[i] - m;
    d[i] = d[i] * d[i];
  }
  return sqrt(pw_sum_short(d, n) / n);
}

__device__ __forceinline__ double clipd(double x, double lo, double hi) {
  return x < lo ? lo : (x > hi ? hi : x);
}
__device__ __forceinline__ double pymax(double a, double b) { return b > a ? b : a; }
__device__ __forceinline__ double pymin(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double norm2(double a, double b) { return sqrt(a * a + b * b); }

// ---- per-track scalar helpers (one lane) ----------------------------------------------------
__device__ void to_tlwh(const SsTrk& t, double* r) {
  r[0] = t.mean[0], r[1] = t.mean[1], r[2] = t.mean[2], r[3] = t.mean[3];
  r[2] *= r[3];
  r[0] -= r[2] / 2;
  r[1] -= r[3] / 2;
}
__device__ void to_tlbr(const SsTrk& t, double* r) {
  to_tlwh(t, r);
  r[2] = r[0] + r[2];
  r[3] = r[1] + r[3];
}
// dt row: tlwh[4], conf, cls, det_ind, quality
constexpr int DTW = 8;
__device__ void det_xyah(const double* d, double* r) {
  r[0] = d[0], r[1] = d[1], r[2] = d[2], r[3] = d[3];
  r[0] += r[2] / 2;
  r[1] += r[3] / 2;
  r[2] /= r[3];
}

__device__ void motion_cons(SsTrk& t, const double* prev, const double* cur) {
  if (t.nvel < 2) return;
  const double* pv = t.vel[t.nvel - 1];
  const double pred0 = prev[0] + pv[0], pred1 = prev[1] + pv[1];
  const double a0 = cur[0] - prev[0], a1 = cur[1] - prev[1];
  const double p0 = pred0 - prev[0], p1 = pred1 - prev[1];
  double c;
  if (norm2(p0, p1) > 0) {
    const double err = norm2(a0 - p0, a1 - p1);
    const double mx = pymax(norm2(p0, p1) * 0.5, 10.0);
    c = pymax(0, 1.0 - (err / mx));
  } else {
    c = norm2(a0, a1) < 5.0 ? 1.0 : 0.5;
  }
  t.motion_cons = 0.8 * t.motion_cons + 0.2 * c;
}

__device__ void push2(double (*h)[2], int& n, const double* v) {
  if (n == MAXH) {
    for (int k = 0; k < MAXH - 1; k++) h[k][0] = h[k + 1][0], h[k][1] = h[k + 1][1];
    n--;
  }
  h[n][0] = v[0];
  h[n][1] = v[1];
  n++;
}

// base_kalman_filter.py:61-78 single-track predict: F (P F^T) + Q
__device__ void track_predict(SsTrk& t) {
  double* m = t.mean;
  double* P = t.cov;
  double q[8];
  kf_process_noise(KIND_BYTE, m, q);
  for (int k = 0; k < 4; k++) m[k] = m[k] + m[k + 4];
  for (int i = 0; i < 8; i++) {
    double M[8], M4[8];
    for (int j = 0; j < 8; j++) {
      M[j] = j < 4 ? P[8 * i + j] + P[8 * i + j + 4] : P[8 * i + j];
      if (i < 4) M4[j] = j < 4 ? P[8 * (i + 4) + j] + P[8 * (i + 4) + j + 4] : P[8 * (i + 4) + j];
    }
    if (i < 4)
      for (int j = 0; j < 8; j++) {
        const double v = M[j] + M4[j];
        P[8 * i + j] = i == j ? v + q[i] : v;
      }
    else
      for (int j = 0; j < 8; j++) P[8 * i + j] = i == j ? M[j] + q[i] : M[j];
  }
  t.age++;
  t.tsu++;
  push2(t.vel, t.nvel, t.mean + 4);
  push2(t.pos, t.npos, t.mean);
  if (t.npos >= 2) motion_cons(t, t.pos[t.npos - 2], t.pos[t.npos - 1]);
}

__device__ void track_camera(SsTrk& t, const double* w) {
  double b[4];
  to_tlbr(t, b);
  const double x1 = (w[0] * b[0] + w[1] * b[1]) + w[2], y1 = (w[3] * b[0] + w[4] * b[1]) + w[5];
  const double x2 = (w[0] * b[2] + w[1] * b[3]) + w[2], y2 = (w[3] * b[2] + w[4] * b[3]) + w[5];
  const double ww = x2 - x1, hh = y2 - y1;
  const double cx = x1 + ww / 2, cy = y1 + hh / 2;
  const double prev[2] = {t.mean[0], t.mean[1]};
  t.mean[0] = cx, t.mean[1] = cy, t.mean[2] = ww / hh, t.mean[3] = hh;
  const double cur[2] = {cx, cy};
  motion_cons(t, prev, cur);
}

__device__ void track_missed(SsTrk& t) {
  t.missed++;
  int thr = t.max_age;
  if (t.quality > 0.8)
    thr = (int)(t.max_age * 1.5);
  else if (t.quality < 0.3)
    thr = (int)(t.max_age * 0.5);
  if (t.state == 1)
    t.state = 3;
  else if (t.tsu > thr)
    t.state = 3;
}

// Track.update's scalar part after the features (track.py:246-277)
__device__ void track_update_scalars(SsTrk& t, const double* d) {
  if (t.nconf == MAXC) {
    for (int k = 0; k < MAXC - 1; k++) t.confh[k] = t.confh[k + 1];
    t.nconf--;
  }
  t.confh[t.nconf++] = d[4];
  if (d[4] > 0.7) {
    t.high_streak++;
    t.low_streak = 0;
  } else if (d[4] < 0.3) {
    t.low_streak++;
    t.high_streak = 0;
  } else {
    t.low_streak = 0;
    t.high_streak = 0;
  }
  t.hits++;
  t.confirmed_det++;
  t.tsu = 0;
  double cq = d[4];
  if (t.nconf > 1) {
    const double avg = np_mean(t.confh, t.nconf);
    const double stab = 1.0 - np_std(t.confh, t.nconf);
    cq = 0.7 * cq + 0.3 * avg * stab;
  }
  const double lb = pymin(t.hits / 20.0, 0.2);
  const double ab = pymax(0, (t.app_cons - 0.5) * 0.2);
  const double mb = pymax(0, (t.motion_cons - 0.5) * 0.1);
  t.quality = clipd(((cq + lb) + ab) + mb, 0.0, 1.0);
  const double cs = t.nconf > 3 ? 1.0 - pymin(np_std(t.confh, t.nconf), 1.0) : 0.5;
  const double hr = (double)t.confirmed_det / (t.age > 1 ? t.age : 1);
  const double cons = (0.4 * t.app_cons + 0.3 * t.motion_cons) + 0.3 * cs;
  t.stability = clipd(0.5 * hr + 0.5 * cons, 0.0, 1.0);
  if (t.state == 1 && (t.hits >= t.n_init || (t.hits >= 1 && t.quality > 0.8))) t.state = 2;
}

// first free pool entry of a slot (-1 if the pool is exhausted)
__device__ int pool_alloc(SsTrk& t, int VP) {
  for (int v = 0; v < VP; v++)
    if (!((t.vmask >> v) & 1ull)) {
      t.vmask |= 1ull << v;
      return v;
    }
  return -1;
}

// ---- the match kernel's code generation ---------------------------------------------------
#ifndef SS_MATCH_ATTR  // everything inlined: a call left by the inliner keeps its frame in scratch
#define SS_MATCH_ATTR __attribute__((flatten))
#endif

// ---- the frame kernel's scratch -----------------------------------------------------------
struct SsWs {
  // ints
  int *lst, *conf_t, *unconf_t, *aut, *cand, *ut3, *fut, *hi, *med, *lo, *aud, *rd, *ud, *ud2;
  int *lvl, *ages, *mt, *tmp, *rows, *cols, *flag, *ti2, *dord;  // mt, dord, aud: HBM (fmt..)
  int *path, *col4row, *row4col, *rem, *pos, *SR, *SC, *pwlo, *pwln, *sc;
  // doubles
  double *dt, *u, *v, *spc, *meas, *key, *pwleaf, *sd;
  double* rowbuf = nullptr;  // optional LDS row (64·UQ) for track_update's pairwise norm
};

// The scratch of one sequence: the LSAP state (3N doubles u v spc, 7N ints path col4row row4col
// rem pos SR SC) and the rest.  The LSAP state always leads the dynamic LDS block (N <= 2048:
// 106 KB at most); ws_lds: 1 = the rest in LDS after it, 2 = the rest in HBM.
__host__ __device__ inline int ws_lsap_bytes(int N) { return 3 * N * 8 + 7 * N * 4; }
// (the LSAP state's 7N ints and 3N doubles are counted in the sizes below: the LDS block's total)
int ws_ints(int T, int D, int N) {
  return T /*lst*/ + T + T + T + 2 * T /*cand*/ + 2 * T /*ut3*/ + 3 * D +
         D /*rd*/ + 2 * (D + 2 * T) /*ud ud2*/ + T /*lvl*/ + T /*ages*/ +
         2 * (T + D) /*tmp*/ + 2 * N /*rows cols*/ + 2 * T /*flag*/ + 2 * T /*ti2*/ +
         7 * N + 2 * PW_MAXLEAF + 32;
}
int ws_doubles(int T, int D, int N) {
  return 3 * N + 4 * D + 2 * T + PW_MAXLEAF + 8;
}

// the per-frame tables that outlive one launch (match -> update -> post) live in HBM
__device__ void ws_frame(const SsDev& g, int seq, SsWs& w) {
  w.dt = g.fdt + (size_t)seq * g.D * DTW;
  w.dord = g.fdord + (size_t)seq * g.D;
  w.aud = g.faud + (size_t)seq * g.D;
  w.mt = g.fmt + (size_t)seq * 4 * (g.D + 2);
  w.fut = g.ffut + (size_t)seq * 3 * g.T;
}

__device__ void ws_carve(const SsDev& g, int seq, SsWs& w, char* lds) {
  const int T = g.T, D = g.D, N = g.N;
  // The LSAP state is carved from LDS unconditionally, so its accesses compile to ds_* LDS
  // instructions: a generic (flat) access counts against the vector-memory counter too, and every
  // wait on one would also wait for the solver's in-flight row loads.
  {
    double* ld = (double*)lds;
    int* li = (int*)(lds + (size_t)3 * N * 8);
    w.u = ld; w.v = ld + N; w.spc = ld + 2 * N;
    w.path = li; w.col4row = li + N; w.row4col = li + 2 * N; w.rem = li + 3 * N;
    w.pos = li + 4 * N; w.SR = li + 5 * N; w.SC = li + 6 * N;
  }
  int* pi = g.wsi + (size_t)seq * g.wsi_n;
  double* pd = g.wsd + (size_t)seq * g.wsd_n;
  if (g.ws_lds == 1) {  // the rest after the LSAP state: doubles first (8-byte alignment), ints
    pd = (double*)(lds + ws_lsap_bytes(N));
    pi = (int*)(lds + ws_lsap_bytes(N) + (size_t)(g.wsd_n - 3 * N) * 8);
  }
  auto I = [&](int n) { int* p = pi; pi += n; return p; };
  auto Dd = [&](int n) { double* p = pd; pd += n; return p; };
  w.lst = I(T); w.conf_t = I(T); w.unconf_t = I(T); w.aut = I(T); w.cand = I(2 * T);
  w.ut3 = I(2 * T); w.hi = I(D); w.med = I(D); w.lo = I(D);
  w.rd = I(D); w.ud = I(D + 2 * T); w.ud2 = I(D + 2 * T); w.lvl = I(T); w.ages = I(T);
  w.tmp = I(2 * (T + D)); w.rows = I(N); w.cols = I(N); w.flag = I(2 * T);
  w.ti2 = I(2 * T); w.pwlo = I(PW_MAXLEAF); w.pwln = I(PW_MAXLEAF); w.sc = I(32);
  ws_frame(g, seq, w);
  w.meas = Dd(4 * D); w.key = Dd(2 * T); w.pwleaf = Dd(PW_MAXLEAF); w.sd = Dd(8);
}

// broadcast an int from lane 0 (all lanes call)
__device__ __forceinline__ int bcast(int v) { return __shfl(v, 0); }
__device__ __forceinline__ double bcastd(double v) { return __shfl(v, 0); }

// The cross-lane hand-off of ONE wave (LDS / global stores complete and visible to its later
// loads): what __syncthreads() is in a one-wave workgroup, without waiting for other waves — the
// match kernel runs its cascade and its solver as two waves of one workgroup, each synchronising
// only itself.
template <class P, class E>
__device__ __forceinline__ int wcompact(int n, P pred, E emit) {
  return wave_compact_s(n, pred, emit, SyncWaveG{});
}

// stable sort of idx[0..n) by key descending (ties keep order): rank placement, lane-parallel,
// the keys staged in ks (LDS, n entries)
template <class K>
__device__ void stable_sort_desc(int* idx, int n, K key, int* tmp, double* ks) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < n; i += 64) {
    tmp[i] = idx[i];
    ks[i] = key(idx[i]);
  }
  __syncthreads();
  // rank of element i = #{j : key j before key i}; a lane ranks up to PB of its elements
  // (i = i0 + lane + 64 q) against each broadcast key j, so the key list is read once per pass
  // rather than once per element (C4: 514 keys, the sort was ~0.2 ms of one wave's loads)
  constexpr int PB = 16;
  for (int i0 = 0; i0 < n; i0 += 64 * PB) {
    const int nq = (n - i0 + 63) / 64;  // wave-uniform
    double ki[PB];
    int r[PB];
#pragma unroll
    for (int q = 0; q < PB; q++) {
      const int i = i0 + lane + 64 * q;
      ki[q] = q < nq && i < n ? ks[i] : 0.0;
      r[q] = 0;
    }
    for (int j = 0; j < n; j++) {
      const double kj = ks[j];
#pragma unroll
      for (int q = 0; q < PB; q++)
        if (q < nq) r[q] += (kj > ki[q]) || (kj == ki[q] && j < i0 + lane + 64 * q);
    }
#pragma unroll
    for (int q = 0; q < PB; q++) {
      const int i = i0 + lane + 64 * q;
      if (q < nq && i < n) idx[r[q]] = tmp[i];
    }
  }
  __syncthreads();
}

// keep a[k] unless it appears in column `col` of matches [m0, m1): in place via tmp
__device__ int filter_matched(int* a, int na, const int* mt, int m0, int m1, int col, int* tmp) {
  const int lane = threadIdx.x & 63;
  const int n = wcompact(
      na,
      [&](int k) {
        for (int q = m0; q < m1; q++)
          if (mt[2 * q + col] == a[k]) return false;
        return true;
      },
      [&](int k, int p) { tmp[p] = a[k]; });
  for (int k = lane; k < n; k += 64) a[k] = tmp[k];
  wsync();
  return n;
}

// filter_matched with a membership table fl[0..nu) (LDS): O(na + matches) instead of O(na x m)
__device__ int filter_matched_fl(int* a, int na, const int* mt, int m0, int m1, int col, int* tmp,
                                 int* fl, int nu) {
  const int lane = threadIdx.x & 63;
  for (int k = lane; k < nu; k += 64) fl[k] = 0;
  wsync();
  for (int q = m0 + lane; q < m1; q += 64) fl[mt[2 * q + col]] = 1;
  wsync();
  const int n = wcompact(na, [&](int k) { return fl[a[k]] == 0; }, [&](int k, int p) { tmp[p] = a[k]; });
  for (int k = lane; k < n; k += 64) a[k] = tmp[k];
  wsync();
  return n;
}

__device__ __forceinline__ bool in_list(const int* a, int n, int v) {
  for (int k = 0; k < n; k++)
    if (a[k] == v) return true;
  return false;
}

// ------------------------------------------------------------------------------------------
// Detection features (wave per input detection, 64-thread blocks): prep [wave norm of feat,
// pairwise norm of feat, wave norm of nf, pairwise norm of nf + 1e-8], dn, nf
__global__ void __launch_bounds__(64)
    ss_prep_kernel(SsDev g, int seq0, const int* __restrict__ det_off,
                   const double* __restrict__ embs, const double* __restrict__ dets) {
  __shared__ int lo[PW_MAXLEAF], ln[PW_MAXLEAF];
  __shared__ double leaf[PW_MAXLEAF];
  const int b = blockIdx.y, seq = seq0 + b, k = blockIdx.x;
  if (k == g.D) {  // the extra block: pack the gallery queries for ss_nn_kernel
    // greedy in list order, a pack holding <= 64 rows (4 MFMA row tiles): the pack starting at
    // track i ends before the first j with rows(i..j) > 64 — found for every i at once by a binary
    // search of the row prefix sums, then the chain of pack starts walked from track 0
    __shared__ int pre[1025], nxt[1024];
    const int nl = g.sq[(size_t)seq * SQS + Q_NNL], lane = threadIdx.x;
    const int* nnl = g.nnl + (size_t)seq * g.T;
    int carry = 0;
    if (lane == 0) pre[0] = 0;
    for (int i0 = 0; i0 < nl; i0 += 64) {
      const int i = i0 + lane;
      int v = i < nl ? __popcll(g.trk[(size_t)seq * g.T + nnl[i]].gmask) : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(v, o);
        if (lane >= o) v += t;
      }
      if (i < nl) pre[i + 1] = carry + v;  // rows of tracks [0, i]
      carry += __shfl(v, 63);
    }
    __syncthreads();
    for (int i = lane; i < nl; i += 64) {  // first j > i with pre[j + 1] - pre[i] > 64
      const int lim = pre[i] + 64;
      int lo2 = i + 1, hi2 = nl;  // answer in [i + 1, nl]
      while (lo2 < hi2) {
        const int mid = (lo2 + hi2) >> 1;
        if (pre[mid + 1] > lim) hi2 = mid; else lo2 = mid + 1;
      }
      nxt[i] = lo2;
    }
    __syncthreads();
    int keep = 0;  // ss_motion_kernel: does a detection pass min_conf (ss_pre_kernel's nk > 0)
    {
      const int r0 = det_off[b];
      int n = det_off[b + 1] - r0;
      if (n > g.D) n = g.D;
      for (int q = lane; q < n; q += 64) keep |= dets[(size_t)(r0 + q) * 6 + 4] >= g.min_conf;
      keep = __any(keep);
    }
    if (lane == 0) {
      int* pk = g.pk + (size_t)seq * (g.T + 3);
      int np = 0;
      for (int i = 0; i < nl; i = nxt[i]) pk[np++] = i;
      pk[np] = nl;
      pk[g.T + 1] = np;
      pk[g.T + 2] = keep;
      for (int x = 0; x < 8; x++) g.sq[(size_t)seq * SQS + Q_NNCTR + x] = 0;
    }
    return;
  }
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) n = g.D;
  if (k >= n) return;
  const int F = g.F, lane = threadIdx.x;
  const double* x = embs + (size_t)(r0 + k) * F;
  double* dn = g.dn + ((size_t)seq * g.D + k) * F;
  double* nf = g.nf + ((size_t)seq * g.D + k) * F;
  constexpr int PQ = 8;
  if (F <= 64 * PQ) {  // the row in registers (element lane + 64 r, wdot's order)
    double rx[PQ];
#pragma unroll
    for (int r = 0; r < PQ; r++) rx[r] = lane + 64 * r < F ? x[lane + 64 * r] : 0.0;
    auto rdot = [&]() {
      double sd = 0.0;
#pragma unroll
      for (int r = 0; r < PQ; r++)
        if (lane + 64 * r < F) sd += rx[r] * rx[r];
#pragma unroll
      for (int dd = 32; dd >= 1; dd >>= 1) sd += __shfl_xor(sd, dd);
      return sd;
    };
    const double fn = sqrt(rdot());
    const double pwn = wpw_norm(x, F, lo, ln, leaf);
    const double dd = pwn + 1e-8, dw = fn + 1e-8;
#pragma unroll
    for (int r = 0; r < PQ; r++) {
      const int q = lane + 64 * r;
      if (q < F) dn[nn_pos(q, F)] = rx[r] / dd;
      rx[r] = rx[r] / dw;
      if (q < F) nf[q] = rx[r];
    }
    const double wn = sqrt(rdot());
    __syncthreads();  // nf visible to the pairwise tree's lane mapping
    const double pn = wpw_norm(nf, F, lo, ln, leaf) + 1e-8;
    if (lane == 0) {
      double* p = g.dprep + ((size_t)seq * g.D + k) * 4;
      p[0] = fn;
      p[1] = pwn;
      p[2] = wn;
      p[3] = pn;
    }
    return;
  }
  const double fn = sqrt(wdot(x, x, F));
  const double pwn = wpw_norm(x, F, lo, ln, leaf);
  const double dd = pwn + 1e-8, dw = fn + 1e-8;
  for (int q = lane; q < F; q += 64) {
    dn[nn_pos(q, F)] = x[q] / dd;
    nf[q] = x[q] / dw;
  }
  __syncthreads();
  const double wn = sqrt(wdot(nf, nf, F));
  const double pn = wpw_norm(nf, F, lo, ln, leaf) + 1e-8;
  if (lane == 0) {
    double* p = g.dprep + ((size_t)seq * g.D + k) * 4;
    p[0] = fn;
    p[1] = pwn;
    p[2] = wn;
    p[3] = pn;
  }
}

typedef double d4 __attribute__((ext_vector_type(4)));

// The NN contraction's k loop for RT row tiles x NDT detection tiles (ap / bp: the lane's row
// bases): blocks of 8 k, one 16-byte load per tile and lane holding its two MFMA k-steps' operands
// (rows stored in MFMA order, nn_pos), the next block's loads in flight during this block's MFMAs; padded rows (past a
// track's samples) read valid rows and are discarded by the caller, so no branch splits the chains.
template <int RT, int NDT, int NA>
__device__ __forceinline__ void nn_kloop(const double* const (&ap)[RT],
                                         const double* const (&bp)[NA], int F, int kl,
                                         d4 (&acc)[RT][NA]) {
  const int FB = (F & 1) ? 0 : F - F % 8;  // 16-byte loads need even rows
  if (FB > 0) {
    // two operand buffers alternate (no register copies), the next block's loads issued before
    // this block's MFMAs and pinned there by scheduling barriers: left to itself the compiler
    // sank the loads to their MFMAs, so every block waited a full load round trip
    // (profiles/r06/nn_prefetch.txt)
    double2 a0[RT], b0[NDT], a1[RT], b1[NDT];
    auto ld = [&](double2* a, double2* bb, int k) {
      const int kk = k < FB ? k : FB - 8;  // past the end: re-read the last block
#pragma unroll
      for (int rt = 0; rt < RT; rt++) a[rt] = *(const double2*)(ap[rt] + kk + 2 * kl);
#pragma unroll
      for (int dt = 0; dt < NDT; dt++) bb[dt] = *(const double2*)(bp[dt] + kk + 2 * kl);
    };
    // (rows stored in MFMA order, nn_pos: .x is k-slot k + kl, .y is k + 4 + kl)
    auto mm = [&](const double2* a, const double2* bb) {
#pragma unroll
      for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int dt = 0; dt < NDT; dt++)
          acc[rt][dt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[rt].x, bb[dt].x, acc[rt][dt], 0, 0, 0);
#pragma unroll
      for (int rt = 0; rt < RT; rt++)
#pragma unroll
        for (int dt = 0; dt < NDT; dt++)
          acc[rt][dt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[rt].y, bb[dt].y, acc[rt][dt], 0, 0, 0);
    };
    ld(a0, b0, 0);
    for (int k = 0; k < FB; k += 16) {
      ld(a1, b1, k + 8);
      __builtin_amdgcn_sched_barrier(0);
      mm(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (k + 8 >= FB) break;
      ld(a0, b0, k + 16);
      __builtin_amdgcn_sched_barrier(0);
      mm(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (int k = FB; k < F; k += 4) {  // tail: lanes past F multiply zeros (a clamped read)
    const bool in = k + kl < F;
    const int kk = in ? k + kl : F - 1;
    double a[RT], bb[NDT];
#pragma unroll
    for (int rt = 0; rt < RT; rt++) { const double v = ap[rt][kk]; a[rt] = in ? v : 0.0; }
#pragma unroll
    for (int dt = 0; dt < NDT; dt++) { const double v = bp[dt][kk]; bb[dt] = in ? v : 0.0; }
#pragma unroll
    for (int rt = 0; rt < RT; rt++)
#pragma unroll
      for (int dt = 0; dt < NDT; dt++)
        acc[rt][dt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[rt], bb[dt], acc[rt][dt], 0, 0, 0);
  }
}

// NearestNeighborDistanceMetric.distance (linear_assignment.py:468-497, 595-618) for one pack of
// listed confirmed tracks per wave (ss_prep_kernel's greedy packing: <= 64 gallery rows, so up to
// four 16-row tiles with the tracks' rows back to back instead of a padded tile per track): rows =
// the tracks' distinct gallery vectors (pre-normalised x/den), columns = this frame's normalised
// detections in blocks of NDT 16-detection tiles; out = 1 - clip(max over the track's rows), the
// max taken per track over its row range by wave shuffles.  Each output's k-chain is the oracle's
// ascending fma chain whatever the tiling.
// Work items (pack, detection block) of the frame's actual sizes — packs x ceil(dets / DB) —
// are handed out by a per-sequence atomic counter to a fixed set of waves (blockIdx.x), each
// looping until the counter passes the last item (every wave reaches that exit): the launch is
// sized by capacities, the work by this frame's packs and detections, so no wave sits on an
// empty (pack, block) slot while another runs two.  With many waves per sequence (C4) the items
// are split by XCD: workgroups are dealt to the 8 XCDs round robin, so wave blockIdx.x runs on
// XCD blockIdx.x % 8 (gridDim.x a multiple of 8) and takes only packs p = xcd (mod 8) from that
// XCD's counter — every item of a pack reads its gallery rows through one XCD's L2 (HBM/MALL
// traffic per launch 881 -> see profiles/r06) instead of all eight.
template <int NDT>
__global__ void __launch_bounds__(64)
    ss_nn_kernel(SsDev g, int seq0, const int* __restrict__ det_off) {
  __shared__ int rowv[64], rowq[64], qoff[65], qslot[64];
  const int b = blockIdx.y, seq = seq0 + b, lane = threadIdx.x;
  const int* pk = g.pk + (size_t)seq * (g.T + 3);
  const int np = pk[g.T + 1];
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) n = g.D;
  if (n <= 0 || np <= 0) return;
  const int F = g.F;
  const double* dnb = g.dn + (size_t)seq * g.D * F;
  const int kl = lane >> 4, cl = lane & 15;
  constexpr int DB = 16 * NDT;  // detections per block
  const int nb = (n + DB - 1) / DB;
  const bool byx = gridDim.x >= 64;  // split by XCD
  const int xcd = byx ? (int)(blockIdx.x & 7) : 0;
  const int npx = byx ? (np > xcd ? (np - xcd + 7) / 8 : 0) : np;  // this XCD's packs
  const int total = npx * nb;
  int* ctr = g.sq + (size_t)seq * SQS + Q_NNCTR + xcd;
  for (;;) {
    int item = 0;
    if (lane == 0) item = atomicAdd(ctr, 1);
    item = __shfl(item, 0);
    if (item >= total) break;
    const int pi = item / nb, blk = item - pi * nb;
    const int p = byx ? xcd + 8 * pi : pi;
    const int t0 = pk[p], nq = pk[p + 1] - t0;  // this pack's tracks (<= 64)
    int slot = 0, c = 0;
    unsigned long long m = 0;
    if (lane < nq) {
      slot = g.nnl[(size_t)seq * g.T + t0 + lane];
      m = g.trk[(size_t)seq * g.T + slot].gmask;
      c = __popcll(m);
    }
    int inc = c;  // inclusive prefix of the row counts over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o);
      if (lane >= o) inc += t;
    }
    const int nrows = __shfl(inc, 63);
    __syncthreads();  // (the previous pack's tables are read no more)
    if (lane < nq) {
      int r = inc - c;
      qoff[lane] = r;
      qslot[lane] = slot;
      while (m) {
        rowv[r] = __ffsll((long long)m) - 1;
        rowq[r] = lane;
        r++;
        m &= m - 1;
      }
      if (blk == 0) atomicAdd(g.sq + (size_t)seq * SQS + Q_ROWS, c);  // a statistic
    }
    if (lane == 0) qoff[nq] = nrows;
    __syncthreads();
    const int ntile = (nrows + 15) / 16;
    if (ntile == 0) continue;
    const double* ap[4];
#pragma unroll
    for (int rt = 0; rt < 4; rt++) {  // padded rows read row 0 and are discarded below
      const int row = 16 * rt + cl, rr = row < nrows ? row : 0;
      ap[rt] = vecnp(g, seq, qslot[rowq[rr]], rowv[rr]);
    }
    {  // this item's detection block
      const int db = blk * DB;
      const int ndt = n - db >= DB ? NDT : (n - db + 15) / 16;
      const double* bp[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; dt++) {
        const int col = db + 16 * dt + cl;
        bp[dt] = dnb + (size_t)(col < n ? col : 0) * F;
      }
      d4 acc[4][NDT];
#pragma unroll
      for (int rt = 0; rt < 4; rt++)
#pragma unroll
        for (int dt = 0; dt < NDT; dt++) acc[rt][dt] = (d4){0.0, 0.0, 0.0, 0.0};
      // row / detection tile counts as compile-time parameters: no MFMA on absent tiles
      auto run = [&](auto rtc, auto ndc) {
        constexpr int RTN = decltype(rtc)::value, NDN = decltype(ndc)::value;
        const double* const(&apr)[RTN] = *reinterpret_cast<const double* const(*)[RTN]>(&ap);
        d4(&accr)[RTN][NDT] = *reinterpret_cast<d4(*)[RTN][NDT]>(&acc);
        nn_kloop<RTN, NDN, NDT>(apr, bp, F, kl, accr);
      };
      using I1 = std::integral_constant<int, 1>;
      using I2 = std::integral_constant<int, 2>;
      using I3 = std::integral_constant<int, 3>;
      using I4 = std::integral_constant<int, 4>;
      // a partial last block runs one tile when that covers it (NDT = 2), else all NDT tiles
      // (columns past n read row 0 and are not stored)
      if (ndt == NDT || (NDT > 2 && ndt > 1)) {
        if (ntile == 4) run(I4{}, std::integral_constant<int, NDT>{});
        else if (ntile == 3) run(I3{}, std::integral_constant<int, NDT>{});
        else if (ntile == 2) run(I2{}, std::integral_constant<int, NDT>{});
        else run(I1{}, std::integral_constant<int, NDT>{});
      } else {
        if (ntile == 4) run(I4{}, I1{});
        else if (ntile == 3) run(I3{}, I1{});
        else if (ntile == 2) run(I2{}, I1{});
        else run(I1{}, I1{});
      }
      // per track: max over its rows (lane holds rows 16 rt + kl + 4 j of column cl)
      for (int q = 0; q < nq; q++) {
        const int o = qoff[q], e = qoff[q + 1];
        if (o == e) continue;  // no gallery rows (never read by the cost kernel)
        double* out = g.nnd + ((size_t)seq * g.T + qslot[q]) * g.D;
#pragma unroll
        for (int dt = 0; dt < NDT; dt++) {
          double mx = -INF;
#pragma unroll
          for (int rt = 0; rt < 4; rt++) {
            if (16 * rt >= e || 16 * rt + 16 <= o) continue;
#pragma unroll
            for (int j = 0; j < 4; j++) {
              const int row = 16 * rt + kl + 4 * j;
              if (row >= o && row < e && acc[rt][dt][j] > mx) mx = acc[rt][dt][j];
            }
          }
          const double o1 = __shfl_xor(mx, 16);
          mx = o1 > mx ? o1 : mx;
          const double o2 = __shfl_xor(mx, 32);
          mx = o2 > mx ? o2 : mx;
          const int col = db + 16 * dt + cl;
          if (kl == 0 && dt < ndt && col < n) out[col] = 1.0 - clipd(mx, -1.0, 1.0);
        }
      }
    }
  }
}

// _attempt_id_recovery similarities: wave per (lost track, detection)
__global__ void __launch_bounds__(256)
    ss_rec_kernel(SsDev g, int seq0, const int* __restrict__ det_off,
                  const double* __restrict__ embs) {
  const int b = blockIdx.y, seq = seq0 + b, li = blockIdx.x;
  if (li >= g.sq[(size_t)seq * SQS + Q_NLOST]) return;
  const int slot = g.lost[(size_t)seq * LOSTN + li];
  const SsTrk& t = g.trk[(size_t)seq * g.T + slot];
  if (t.nfeat == 0) return;
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) n = g.D;
  const int v = t.feat[t.nfeat - 1], F = g.F;
  const double* tf = vecp(g, seq, slot, v);
  const double tn = g.vwn[vidx(g, seq, slot, v)];
  for (int d = threadIdx.x >> 6; d < n; d += 4) {
    const double* x = embs + (size_t)(r0 + d) * F;
    const double dot = wdot(x, tf, F);
    if ((threadIdx.x & 63) == 0)
      g.recsim[((size_t)seq * LOSTN + li) * g.D + d] =
          dot / (g.dprep[((size_t)seq * g.D + d) * 4 + 1] * tn);
  }
}

// ------------------------------------------------------------------------------------------
// The frame kernel: one wave64 per sequence.
// An LSAP handed by the match kernel's cascade wave to its solver wave (LDS): the matrix kind and
// orientation (lsap_mats), the clamp, the shape (the rows' offsets and the columns' indices are
// the kernel's LDS arrays, passed to every wave as such so their accesses compile to LDS
// instructions); np is the solver's answer.  flag: 0 idle (or done), 1 posted, -1 exit.
struct LsapJob {
  double max_d;
  int R, CC, tr, kind, np;
  int mode;  // 0 scipy's order; 1 solve + certify, a tie re-solved in scipy's order; 2 ... a tie
             // reported (stat 3) instead: the columns' order is not certified to be scipy's
  int stat;  // 0 unique, 1 unique up to rejected pairs, 2 tie re-solved, 3 tie not solved
  int flag;
  int abort;  // set by either wave on a timeout: both stop handing over, nobody writes np / flag
};
struct SsCtx {
  const SsDev& g;
  SsWs& w;
  int seq, lane;
  SsTrk* trk;
  int* sq;
  double* sqd;
  int* lost;
  int ntr, nlost, nk, nm;
  double* key;  // match kernel: quality + stability by list position (LDS)
  int* tsu;     // match kernel: time_since_update by list position (LDS)
  int* rank;    // match kernel: cascade rank by list position (LDS)
  int* gpos;    // match kernel: list position by cascade rank (LDS)
  int* inset;   // match kernel: membership table by list position (LDS)
  int ncf;      // confirmed tracks
  int* flt;     // match kernel: scratch table (LDS, 1024 ints)
  double* ks;   // match kernel: sort-key scratch (LDS)
  int* cidx;    // match kernel: the solver's column indices (LDS, 2048 ints)
  struct LsapJob* job;  // match kernel: the hand-off to its solver wave
  int lmode = 0, lstat = 0;  // match kernel: the next LSAP's LsapJob::mode, the last one's stat
  __device__ const double* det(int i) const { return w.dt + (size_t)w.dord[i] * DTW; }
  __device__ int det_in(int i) const { return (int)det(i)[6]; }
};

// The matrix of an LSAP (min_cost_matching) in the solver's orientation — derived from the kernel
// argument in the wave that reads it, so the loads compile to global (not flat) memory
// instructions, whose waits do not also wait for LDS.  kind 0: the gated cost by cascade rank
// (ss_cost_kernel's cfull / cfullT); 1: the IoU cost by list position (cost / its transpose).
__device__ __forceinline__ const double* lsap_mat(const SsDev& g, int seq, int kind, bool tr) {
  if (kind == 0)
    return tr ? g.cfullT + (size_t)seq * g.D * g.T : g.cfull + (size_t)seq * g.T * g.D;
  const double* io = g.cost + (size_t)seq * 4 * g.T * g.D;
  return tr ? io + (size_t)g.T * g.D : io;
}

// The match kernel's two waves hand LSAPs over through LDS flags.  A wait that outlasts any
// legitimate LSAP (SS_SPIN_TICKS of the 100 MHz real-time counter: 2 s) latches BX_ERR_INVALID
// in the engine status and gives up, so a fault in either wave ends the launch with an error
// instead of leaving the queue spinning.
#ifndef SS_SPIN_TICKS
#define SS_SPIN_TICKS 200000000ull
#endif
// wait until *flag != v (want_ne) or == v (!want_ne); returns the value seen, or v after a timeout
// or once the other wave has aborted (*abort set; a timeout here sets it): after that neither
// wave waits again, so one fault costs one SS_SPIN_TICKS, not one per remaining hand-off
__device__ __forceinline__ int lds_flag_wait(int* flag, int v, bool want_ne, int* status,
                                             int* abort, bool& timed_out) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const int f = (int)__builtin_amdgcn_readfirstlane(
        (unsigned)__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    if ((f != v) == want_ne) return f;
    const bool ab = __builtin_amdgcn_readfirstlane((unsigned)__hip_atomic_load(
                        abort, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
    if (ab || __builtin_amdgcn_s_memrealtime() - t0 > SS_SPIN_TICKS) {
      if ((threadIdx.x & 63) == 0) {
        atomicExch(status, (int)BX_ERR_INVALID);
        __hip_atomic_store(abort, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      timed_out = true;
      return v;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// scipy.optimize.linear_sum_assignment (Crouse's shortest augmenting path, rectangular),
// wave-parallel, in the solver's orientation: R x CC, R <= CC (`tr`: the caller's matrix was
// transposed to get there, so the output pairs are argsorted by the original row).  Entry (r, j)
// is P[roff[r] + cidx[j]], read straight from the stage's matrix — no per-level copy — which
// ss_cost_kernel stores with min_cost_matching's clamp already applied (above max_d -> max_d +
// 1e-5, max_d being the stage's: every detection takes part in one stage only).  Rows are read by
// buffer loads: the row's byte offset in a scalar register, the lane's column offsets in vector
// registers, no per-load address arithmetic.
//
// Lane l owns the columns j = l + 64 q (q < LQ, CC <= 64 LQ): their matrix index (cidx, or j
// itself when !IDX), v[j] and an assigned bit stay in registers.  Each row's first Dijkstra step —
// where most rows end — runs from registers: relax against v, wave minimum, scipy's tie rule (the
// last unassigned column at the minimum in `remaining` order, else the first; fresh positions are
// CC-1-j, so the smallest unassigned j, else the largest j), assignment.  Only a row whose minimum
// lands on an assigned column writes the search state out (rem / pos / SC / spc / path in LDS)
// and continues Crouse's search as scipy does; u[cur] is 0 before row cur (only rows already
// assigned are ever on a path).  Pairs sorted by row into w.rows / w.cols.
//
// Rows are taken in pairs (LQ <= 16): a row's first step depends on the rows before it only
// through v — which a row ending on its first step leaves unchanged — and through the assigned
// bits, which only its decision (ballots, tie rule) reads.  So both rows of a pair are relaxed
// and reduced against the same v (two independent chains for the scheduler to interleave), then
// decided in order; when the first row's search goes on (v changes), the second is reloaded and
// relaxed again first: every row is decided exactly as the sequential solver decides it.  The
// next pair's costs are in flight meanwhile.
//
// fast (solve, then certify; LQ <= 16): the same optimum without scipy's row order.  (A) every
// row's minimum and its lowest argmin column with v = 0, rows streamed two at a time with the
// next pair's loads in flight — no row waits for the one before; u[r] = the minimum, and a row
// whose argmin column is still free takes it (a feasible dual solution, tight on this partial
// matching).  (C) the rows that lost their column ("contested") run Crouse's search from there
// (finish_row, the same code as the exact path), in any order: the result is an optimum.  (D)
// certify it: the reduced costs c - u - v of every unmatched entry against LSAP_SS_TOL (far above
// both solvers' rounding).  Any optimum uses tight entries only, so an entry (r, j) that is not
// tight means no optimum assigns j to r.  If no unmatched entry is tight the optimum is unique
// and equals scipy's, pairs and all (fstat 0).  If the only tight unmatched entries are in rows
// whose matched entry and the tight one are both clamped (> max_d, min_cost_matching rejects
// them), every other optimum differs from this one in rejected pairs only: the same matches, the
// same unmatched sets, but possibly another ORDER of min_cost_matching's unmatched lists (fstat
// 1).  Otherwise a real pair could change: returns -1 (fstat 2) and the caller re-solves in
// scipy's order.  NaN costs (a failed Cholesky) also go back to the exact path.
constexpr double LSAP_SS_TOL = 1e-9;
template <int LQ, bool IDX>
__device__ __forceinline__ int lsap_wave(SsCtx& x, const double* __restrict__ P, const int* roff,
                                         const int* cidx, double max_d, int R, int CC, bool tr,
                                         bool fast, int& fstat, const int16_t* tl = nullptr,
                                         const int* tc = nullptr) {
  SsWs& w = x.w;
  const int lane = x.lane;
#ifdef BX_PHASE_TIMING
  const SsDev& g = x.g;
  const int seq = x.seq;
  SCOUNT(7, R);
  SCOUNT(8, CC);
  SCOUNT(16, (unsigned long long)R * CC);
  const bool big_call = (size_t)R * CC * 8 > 65536;
  SCOUNT(17, big_call ? 1 : 0);
  SCOUNT(18, big_call ? R : 0);
  unsigned long long t_slow = 0, t_all = SS_NOW();
#endif
  for (int i = lane; i < R; i += 64) w.u[i] = 0.0, w.col4row[i] = -1;
  for (int j = lane; j < CC; j += 64) w.path[j] = -1, w.row4col[j] = -1;
  unsigned cb[LQ];  // byte offset of the lane's column q in a row (column 0's past CC)
  double vr[LQ];    // v[j]; -INF past CC, so those columns relax to +INF
  unsigned asg = 0;
#pragma unroll
  for (int q = 0; q < LQ; q++) {
    const int j = lane + 64 * q;
    cb[q] = 8u * (unsigned)(j < CC ? (IDX ? cidx[j] : j) : 0);
    vr[q] = j < CC ? 0.0 : -INF;
  }
  wsync();
  // the matrix as a buffer (its base made provably wave-uniform: no waterfall loops)
  const unsigned long long pb = (unsigned long long)P;
  // (each half widened from unsigned: readfirstlane returns int, which would sign-extend)
  const unsigned long long pbu =
      (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(pb >> 32)) << 32 |
      (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)pb);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)pbu, (short)0, (int)__builtin_amdgcn_readfirstlane((unsigned)(8 * x.g.T * x.g.D)),
      0x00020000);
  auto ld_elem = [&](int roff_r, int q) {  // row element offset roff_r (wave-uniform), slot q
#ifdef BX_CHECK
    // debug builds: a raw buffer load past num_records reads 0 instead of faulting, so an
    // indexing slip would become a silent wrong cost; latch it as an engine error instead
    if ((unsigned long long)cb[q] + 8ull * (unsigned)roff_r >= 8ull * x.g.T * x.g.D)
      atomicExch(x.g.status, (int)BX_ERR_INVALID);
#endif
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                          rsrc, cb[q], __builtin_amdgcn_readfirstlane(8 * roff_r), 0));
  };
  // raw loads, unconditional: a load is waited for only when its value is needed
  auto load_row = [&](int off, double* dst) {
#pragma unroll
    for (int q = 0; q < LQ; q++) dst[q] = ld_elem(off, q);
  };
  // scipy's minVal + cost - u[cur] - v[j] with minVal = u[cur] = 0 (up to the sign of a zero,
  // which no comparison and no later sum can tell).  A NaN cost stays NaN here and loses every
  // comparison below, as the INF that scipy's `r < INF` test would make of it.  Returns the
  // lane's minimum.
  auto relax = [&](const double* raw, double* rv) {
#pragma unroll
    for (int q = 0; q < LQ; q++) rv[q] = raw[q] - vr[q];
    double lmin = rv[0];
#pragma unroll
    for (int q = 1; q < LQ; q++) lmin = fmin(lmin, rv[q]);
    return lmin;
  };
  bool bad = false;
  // fast mode's per-row flags (w.v, unused by the exact path): bit 0 = more than one entry
  // within LSAP_SS_TOL of the row's minimum at its claim, bit 1 = touched by a search (its u, or
  // its column, changed after the claim)
  int* rfl = (int*)w.v;
  // Row cur from its first step (rv, wave minimum m0): assigned when the step ends on an
  // unassigned column, else Crouse's search continued.  Returns true when v changed (the search
  // went on).
  auto finish_row = [&](int cur, double* rv, double m0) -> bool {
    if (fast && lane == 0) rfl[cur] |= 2;
    if (!(m0 < INF)) {  // infeasible (cannot happen with finite costs)
      bad = true;
      return false;
    }
    // the columns at the minimum: a wave mask per q (counted), their union, and per lane the
    // slot at the minimum (meaningful where the minimum is unique)
    int cnt = 0, qi = 0;
    unsigned long long un0 = 0;
#pragma unroll
    for (int q = 0; q < LQ; q++) {
      const bool eq = rv[q] == m0;
      const unsigned long long e = __ballot(eq);
      cnt += __popcll(e);
      un0 |= e;
      qi = eq ? q : qi;
    }
    int j0;
    bool sink;
    if (cnt == 1) {  // a unique minimum (the usual case)
      const int L = __ffsll((long long)un0) - 1;
      const int q0 = rl_i(qi, L);
      j0 = L + 64 * q0;
      sink = !((rl_i((int)asg, L) >> q0) & 1);
    } else {  // scipy's tie rule over the lanes
      unsigned eq = 0;
#pragma unroll
      for (int q = 0; q < LQ; q++) eq |= rv[q] == m0 ? 1u << q : 0u;
      const unsigned un = eq & ~asg;
      constexpr int BIG = 0x7fffffff;
      const int a = un ? lane + 64 * (__ffs(un) - 1) : BIG;
      const int b = eq ? lane + 64 * (31 - __clz(eq)) : -1;
      const int ja = wave_min_i(a), jb = -wave_min_i(-b);
      sink = ja != BIG;
      j0 = sink ? ja : jb;
    }
    if (sink) {  // an unassigned column: u[cur] += minVal, v[j0] -= 0, augment
      if (lane == (j0 & 63)) asg |= 1u << (j0 >> 6);
      if (lane == 0) {
        w.u[cur] = m0;
        w.row4col[j0] = cur;
        w.col4row[cur] = j0;
      }
      return false;
    }
#ifdef BX_PHASE_TIMING
    SCOUNT(9, 1);
    const unsigned long long t_s0 = SS_NOW();
#endif
    // The search continues as scipy's does, its per-column state in registers: spc (rv, NaN as
    // INF), the SC bits, v; `remaining` (rem / pos, for the tie rule), path and the visited rows
    // (with the minimum each was reached at: spc of its column) in LDS.
    const int index0 = CC - 1 - j0;
    double minVal = m0;
    int nrem = CC;
    unsigned sc = lane == (j0 & 63) ? 1u << (j0 >> 6) : 0u;
#pragma unroll
    for (int q = 0; q < LQ; q++) {  // the first step's relaxation
      const int j = lane + 64 * q;
      const bool ok = rv[q] < INF;
      rv[q] = ok ? rv[q] : INF;
      if (j < CC) {
        w.rem[CC - 1 - j] = j;
        w.pos[j] = CC - 1 - j;
        if (ok) w.path[j] = cur;
      }
    }
    wsync();
    if (lane == 0) {
      const int jl = w.rem[nrem - 1];
      w.rem[index0] = jl;
      w.pos[jl] = index0;
    }
    nrem--;
    int nvis = 0;  // visited rows other than cur: w.SR[k] (row), w.spc[k] (its minimum)
    int sk = -1, i = w.row4col[j0];
    if (lane == 0) w.SR[0] = i, w.spc[0] = m0;
    nvis = 1;
    while (sk == -1) {
      const double ui = w.u[i];
      const int roff_i = roff[i];
      double m = INF;
      constexpr int QB = LQ < 8 ? LQ : 8;  // loads in flight per lane
#pragma unroll
      for (int q0 = 0; q0 < LQ; q0 += QB) {
        double cv[QB];
#pragma unroll
        for (int u = 0; u < QB; u++) {
          cv[u] = ld_elem(roff_i, q0 + u);  // (stored clamped)
        }
#pragma unroll
        for (int u = 0; u < QB; u++) {
          const int q = q0 + u;
          if ((sc >> q) & 1u) continue;
          const double r = minVal + cv[u] - ui - vr[q];  // +INF past CC
          if (r < rv[q]) {
            rv[q] = r;
            w.path[lane + 64 * q] = i;
          }
          m = fmin(m, rv[q]);
        }
      }
      m = wave_min_bfly(m);
      if (!(m < INF)) {  // infeasible (cannot happen with finite costs)
        bad = true;
        return false;
      }
      int c1 = 0, qs = 0;
      unsigned long long es = 0;
#pragma unroll
      for (int q = 0; q < LQ; q++) {
        const unsigned long long e = __ballot(!((sc >> q) & 1u) && rv[q] == m);
        c1 += __popcll(e);
        if (e) qs = q, es = e;
      }
      int j;
      if (c1 == 1) {
        j = __ffsll((long long)es) - 1 + 64 * qs;
      } else {  // the last unassigned column at the minimum in `remaining` order, else the first
        int last_un = -1, first_eq = 0x7fffffff;
#pragma unroll
        for (int q = 0; q < LQ; q++) {
          const int jq = lane + 64 * q;
          if (!((sc >> q) & 1u) && rv[q] == m) {
            const int p = w.pos[jq];
            if (!((asg >> q) & 1u)) last_un = p > last_un ? p : last_un;
            first_eq = p < first_eq ? p : first_eq;
          }
        }
        last_un = -wave_min_i(-last_un);
        first_eq = wave_min_i(first_eq);
        j = w.rem[last_un >= 0 ? last_un : first_eq];
      }
      minVal = m;
      const bool un = !((rl_i((int)asg, j & 63) >> (j >> 6)) & 1);
      if (un) {
        sk = j;
      } else {
        i = w.row4col[j];
        if (lane == 0) w.SR[nvis] = i, w.spc[nvis] = m;
        nvis++;
      }
      if (lane == (j & 63)) sc |= 1u << (j >> 6);
      if (lane == 0) {
        const int index = w.pos[j];
        const int jl = w.rem[nrem - 1];
        w.rem[index] = jl;
        w.pos[jl] = index;
      }
      nrem--;
#ifdef BX_PHASE_TIMING
      if ((threadIdx.x & 63) == 0 && x.g.dbg) x.g.dbg[(size_t)x.seq * SS_DBG + 16 + 5] += 1;
#endif
    }
    wsync();
    // duals: u[cur] = minVal (it was 0), u[i] += minVal - spc[col4row[i]] for the visited rows,
    // v[j] -= minVal - spc[j] for the SC columns; then the augmentation along path
    for (int k = lane; k < nvis; k += 64) {
      const int r = w.SR[k];
      w.u[r] += minVal - w.spc[k];
      if (fast) rfl[r] |= 2;
    }
    if (lane == 0) w.u[cur] = 0.0 + minVal;
#pragma unroll
    for (int q = 0; q < LQ; q++)
      if ((sc >> q) & 1u) vr[q] -= minVal - rv[q];
    wsync();
    if (lane == 0) {
      int jj = sk;
      for (;;) {
        const int q = w.path[jj];
        w.row4col[jj] = q;
        const int t = w.col4row[q];
        w.col4row[q] = jj;
        jj = t;
        if (q == cur) break;
      }
    }
    if (lane == (sk & 63)) asg |= 1u << (sk >> 6);
    wsync();
#ifdef BX_PHASE_TIMING
    t_slow += SS_NOW() - t_s0;
#endif
    return true;
  };
  fstat = 0;
  if constexpr (LQ <= 16) {
   if (fast) {
    const int rlast = R - 1;
    auto roff_c = [&](int r) { return roff[r < rlast ? r : rlast]; };
    double A0[LQ], A1[LQ], B0[LQ], B1[LQ];
    bool nan_l = false;  // a NaN cost in a real column (lane-local)
    int ncont = 0;       // contested rows, listed in w.SC
    // (A) row r's minimum m over v = 0 (vr: 0, -INF past CC); it takes the lowest column at
    // the minimum that is still free (a row of rejected entries only — most of a cascade
    // level's detections — finds one), else it is contested
    auto claim = [&](int r, const double* a, double m) {
      if (!(m < INF)) {  // no finite entry: the exact path's business
        bad = true;
        return;
      }
      int j0 = -1, ntie = 0;
      const double mt = m + LSAP_SS_TOL;
#pragma unroll
      for (int q = 0; q < LQ; q++) {
        const double h = a[q] - vr[q];
        const unsigned long long e = __ballot(h == m && !((asg >> q) & 1u));
        if (j0 < 0 && e) j0 = 64 * q + __ffsll((long long)e) - 1;
        ntie += __popcll(__ballot(h <= mt));
      }
      if (j0 >= 0) {
        if (lane == (j0 & 63)) asg |= 1u << (j0 >> 6);
        if (lane == 0) {
          w.u[r] = m;
          w.col4row[r] = j0;
          w.row4col[j0] = r;
          rfl[r] = ntie > 1 ? 1 : 0;
        }
      } else {
        if (lane == 0) w.SC[ncont] = r, rfl[r] = 3;
        ncont++;
      }
    };
    auto minpair = [&](int r, const double* a0, const double* a1) {
      double m0 = INF, m1 = INF;
#pragma unroll
      for (int q = 0; q < LQ; q++) {
        m0 = fmin(m0, a0[q] - vr[q]);
        m1 = fmin(m1, a1[q] - vr[q]);
        nan_l |= (lane + 64 * q < CC) && (a0[q] != a0[q] || a1[q] != a1[q]);
      }
      wave_min_bfly2(m0, m1);
      claim(r, a0, m0);
      if (r + 1 < R && !bad) claim(r + 1, a1, m1);
    };
#ifdef BX_PHASE_TIMING
    unsigned long long tA = SS_NOW();
#endif
    // The sparse form of (A) for the cascade levels (tl: ss_cost_kernel's lists of each track's
    // real entries): every other entry of the matrix is the clamp K = max_d + 1e-5, so a row's
    // minimum is its least real entry in this LSAP's columns, or K.  Rows with a real minimum
    // bid for its column (the lowest row wins; the others are contested); the rows without
    // one take the columns left free, in order (there are enough: R <= CC).  Lane per row (per
    // column, scattering into the rows, when the rows are the detections).  Any track with an
    // overflowing or NaN list sends the LSAP through the dense form below.
    bool sparse = false;
    if (tl != nullptr) {
      const int T = x.g.T, D = x.g.D;
#ifdef BX_PHASE_TIMING
      unsigned long long tS = SS_NOW();
#endif
      bool ovf = false;
      if (!tr)
        for (int r = lane; r < R; r += 64) ovf |= tc[roff[r] / D] < 0;
      else
        for (int c = lane; c < CC; c += 64) ovf |= tc[cidx[c]] < 0;
      sparse = !__any(ovf);
#ifdef BX_PHASE_TIMING
      SCOUNT(27, SS_NOW() - tS);
      tS = SS_NOW();
#endif
      if (sparse) {
        const double K = max_d + 1e-5;
        auto ordb = [](double v) -> unsigned long long {  // order-preserving bits
          const unsigned long long bb = (unsigned long long)__double_as_longlong(v);
          return (bb >> 63) ? ~bb : (bb | 0x8000000000000000ull);
        };
        auto unord = [](unsigned long long bb) -> double {
          return __longlong_as_double(
              (long long)((bb >> 63) ? (bb & 0x7fffffffffffffffull) : ~bb));
        };
        int* pos = w.rem;  // sorted detection -> this LSAP's column (!tr) / row (tr), or -1
        // row minima (order-preserving bits) in w.v's upper half: rfl takes its first R ints and
        // R <= N/2 (R = min(tracks, detections) <= T, N >= 2T)
        unsigned long long* rmin = (unsigned long long*)w.v + x.g.N / 2;
        int* rcol = w.path;  // row -> lowest column at its real minimum
        int* rtie = w.pos;   // row -> real entries within LSAP_SS_TOL of it
        int* own = w.SR;     // column -> lowest bidding row
        for (int e = lane; e < D; e += 64) pos[e] = -1;
        for (int r = lane; r < R; r += 64)
          rmin[r] = ordb(INF), rcol[r] = 0x7fffffff, rtie[r] = 0;
        for (int c = lane; c < CC; c += 64) own[c] = 0x7fffffff;
        wsync();
        if (!tr)
          for (int c = lane; c < CC; c += 64) pos[cidx[c]] = c;
        else
          for (int r = lane; r < R; r += 64) pos[roff[r] / T] = r;
        wsync();
#ifdef BX_PHASE_TIMING
        SCOUNT(28, SS_NOW() - tS);
        tS = SS_NOW();
#endif
        if (!tr) {
          for (int r = lane; r < R; r += 64) {
            const int rank = roff[r] / D, n = tc[rank];
            const int16_t* L = tl + (size_t)rank * SS_TL;
            double m = INF;
            int jm = 0x7fffffff, nin = 0;
            for (int k = 0; k < n; k++) {
              const int e = L[k], c = pos[e];
              if (c < 0) continue;
              const double val = P[roff[r] + e];
              nin++;
              if (val < m || (val == m && c < jm)) m = val, jm = c;
            }
            int nt = nin;  // (one entry: itself)
            if (nin > 1) {
              nt = 0;
              for (int k = 0; k < n; k++) {
                const int e = L[k];
                nt += pos[e] >= 0 && P[roff[r] + e] <= m + LSAP_SS_TOL;
              }
            }
            rmin[r] = ordb(m);
            rcol[r] = jm;
            rtie[r] = nt;
          }
        } else {
          // lane per column (track): its real entries dealt into two LDS slots per row (w.spc
          // values, w.row4col columns — reset after: 2R <= N), counted in rtie; a row with more
          // than two in this LSAP (rare: a detection gated to three tracks of one cascade
          // level) sends the LSAP through the dense form
          double* sv = w.spc;
          int* sc2 = w.row4col;
          for (int c = lane; c < CC; c += 64) {
            const int rank = cidx[c], n = tc[rank];
            const int16_t* L = tl + (size_t)rank * SS_TL;
            for (int k = 0; k < n; k++) {
              const int r = pos[L[k]];
              if (r < 0) continue;
              const double val = P[roff[r] + rank];
              const int sl = atomicAdd(&rtie[r], 1);
              if (sl < 2) sv[2 * r + sl] = val, sc2[2 * r + sl] = c;
            }
          }
          wsync();
          bool many = false;
          for (int r = lane; r < R; r += 64) {
            const int n = rtie[r];
            many |= n > 2;
            double m = INF;
            int jm = 0x7fffffff, nt = 0;
            if (n >= 1 && n <= 2) {
              const double a0 = sv[2 * r], a1 = n == 2 ? sv[2 * r + 1] : INF;
              const int c0 = sc2[2 * r], c1 = n == 2 ? sc2[2 * r + 1] : 0x7fffffff;
              m = fmin(a0, a1);
              const int k0 = a0 == m ? c0 : 0x7fffffff, k1 = a1 == m ? c1 : 0x7fffffff;
              jm = k0 < k1 ? k0 : k1;
              nt = (a0 <= m + LSAP_SS_TOL) + (n == 2 && a1 <= m + LSAP_SS_TOL);
            }
            rmin[r] = ordb(m);
            rcol[r] = jm;
            rtie[r] = nt;
          }
          if (__any(many)) bad = true;  // (-> the exact path: rare)
          wsync();
          for (int j = lane; j < 2 * R || j < CC; j += 64) sc2[j] = -1;
        }
#ifdef BX_PHASE_TIMING
        wsync();
        SCOUNT(29, SS_NOW() - tS);
        tS = SS_NOW();
#endif
        wsync();
        for (int r = lane; r < R; r += 64)
          if (rcol[r] != 0x7fffffff) atomicMin(&own[rcol[r]], r);
        wsync();
        int* fcol = w.rem;  // the columns no row bid for, in order (pos is done)
        const int nfree = wcompact(CC, [&](int c) { return own[c] == 0x7fffffff; },
                                   [&](int c, int p) { fcol[p] = c; });
        int ncl = 0;
        for (int r0 = 0; r0 < R; r0 += 64) {
          const int r = r0 + lane;
          const bool in = r < R;
          const int jc = in ? rcol[r] : 0;
          const bool clampr = in && jc == 0x7fffffff;
          const bool wins = in && !clampr && own[jc] == r;
          const bool lost = in && !clampr && !wins;
          const unsigned long long mc = __ballot(clampr), ml = __ballot(lost);
          const unsigned long long below = (1ull << lane) - 1ull;
          if (clampr) {
            const int k = ncl + __popcll(mc & below);
            const int j = fcol[k < nfree ? k : nfree - 1];
            w.u[r] = K;
            w.col4row[r] = j;
            w.row4col[j] = r;
            rfl[r] = CC > 1 ? 1 : 0;
          } else if (wins) {
            w.u[r] = unord(rmin[r]);
            w.col4row[r] = jc;
            w.row4col[jc] = r;
            rfl[r] = rtie[r] > 1 ? 1 : 0;
          } else if (lost) {
            w.SC[ncont + __popcll(ml & below)] = r;
            rfl[r] = 3;
          }
          ncl += __popcll(mc);
          ncont += __popcll(ml);
        }
        if (ncl > nfree) bad = true;  // (cannot happen: R <= CC)
        wsync();
#ifdef BX_PHASE_TIMING
        SCOUNT(30, SS_NOW() - tS);
#endif
        asg = 0u;
#pragma unroll
        for (int q = 0; q < LQ; q++) {
          const int j = lane + 64 * q;
          if (j < CC) {
            w.path[j] = -1;
            if (w.row4col[j] >= 0) asg |= 1u << q;
          }
        }
        wsync();
      }
    }
    if (!sparse) {
      load_row(roff_c(0), A0);
      load_row(roff_c(1), A1);
      for (int r = 0; r < R && !bad;) {
        load_row(roff_c(r + 2), B0);
        load_row(roff_c(r + 3), B1);
        minpair(r, A0, A1);
        r += 2;
        if (r >= R || bad) break;
        load_row(roff_c(r + 2), A0);
        load_row(roff_c(r + 3), A1);
        minpair(r, B0, B1);
        r += 2;
      }
      if (__any(nan_l)) bad = true;
    }
#ifdef BX_PHASE_TIMING
    SCOUNT(20, ncont);
    wsync();
    SCOUNT(23, SS_NOW() - tA);
    tA = SS_NOW();
#endif
    wsync();
    // (C) the contested rows: Crouse's search from the partial matching (the next one's costs in
    // flight meanwhile; v changes between them, so each is relaxed when its turn comes)
    auto croff = [&](int k) {
      return roff[(int)__builtin_amdgcn_readfirstlane((unsigned)w.SC[k < ncont ? k : ncont - 1])];
    };
    auto contested = [&](int k, double* a) {
      const int cur = (int)__builtin_amdgcn_readfirstlane((unsigned)w.SC[k]);
      const double m0 = wave_min_bfly(relax(a, a));
      finish_row(cur, a, m0);
    };
    if (ncont > 0 && !bad) load_row(croff(0), A0);
    for (int k = 0; k < ncont && !bad;) {
      load_row(croff(k + 1), B0);
      contested(k, A0);
      if (++k >= ncont || bad) break;
      load_row(croff(k + 1), A0);
      contested(k, B0);
      ++k;
    }
    wsync();
#ifdef BX_PHASE_TIMING
    wsync();
    SCOUNT(24, SS_NOW() - tA);
    tA = SS_NOW();
#endif
    // (D) the certificate, rows streamed as in (A).  Per row r: its tight unmatched entries
    // (reduced cost <= LSAP_SS_TOL; a reduced cost below -LSAP_SS_TOL would mean broken duals:
    // back to the exact path), whether its column is free-priced (v >= -LSAP_SS_TOL: w.SR, the
    // "sources" below) and whether it is a candidate: a row with tight unmatched entries whose
    // matched entry or one of those tight entries is real (<= max_d) — only a candidate on a
    // cycle can change a real pair (w.SC, up to R of them; w.SR bit 1: matched entry real).
    constexpr int SS_CERT_ROUNDS = 4, SS_CERT_BUDGET = 256;
    bool infeas = false, tight_l = false;
    int ncand = 0;
    auto cert = [&](int r, const double* a) {
      const int cr = (int)__builtin_amdgcn_readfirstlane((unsigned)w.col4row[r]);
      if (cr < 0 || cr >= CC) {
        infeas = true;
        return;
      }
      const double ur = w.u[r];
      double mv = a[0], mvv = vr[0];
#pragma unroll
      for (int q = 1; q < LQ; q++) {
        mv = q == (cr >> 6) ? a[q] : mv;
        mvv = q == (cr >> 6) ? vr[q] : mvv;
      }
      const bool realm = rl_d(mv, cr & 63) <= max_d;
      const bool src = rl_d(mvv, cr & 63) >= -LSAP_SS_TOL;
      bool t_r = false, rt_r = false;
#pragma unroll
      for (int q = 0; q < LQ; q++) {
        const int j = lane + 64 * q;
        if (j < CC && j != cr) {
          const double rc = (a[q] - ur) - vr[q];
          infeas |= !(rc >= -LSAP_SS_TOL);
          if (rc <= LSAP_SS_TOL) {
            t_r = true;
            rt_r |= a[q] <= max_d;
          }
        }
      }
      const bool any_t = __any(t_r);
      tight_l |= any_t;
      const bool cand = any_t && (realm || __any(rt_r));
      if (lane == 0) {
        w.SR[r] = (src ? 1 : 0) | (realm ? 2 : 0);
        if (cand) w.SC[ncand] = r;
      }
      ncand += cand;
    };
    // A row no search touched kept its claim (column at its minimum m = u) and its u; v only
    // decreases, so its reduced costs only grew since the claim: its tight entries are among
    // those within LSAP_SS_TOL of m then.  With one such entry (its own) it has no tight
    // unmatched entry; with more but m > max_d they are all rejected entries (no candidate,
    // the order is not certified).  Neither needs its costs reloaded; the rest are rescanned.
    if (!bad) {
      for (int r0 = 0; r0 < R; r0 += 64) {
        const int r = r0 + lane;
        bool scan = false;
        if (r < R) {
          const int fl = rfl[r];
          const double ur = w.u[r];
          scan = (fl & 2) || ((fl & 1) && ur <= max_d);
          tight_l |= !scan && (fl & 1);
          w.SR[r] = ur <= max_d ? 2 : 0;  // (untouched: matched entry = m = u)
        }
        unsigned long long todo = __ballot(scan);
#ifdef BX_PHASE_TIMING
        SCOUNT(26, __popcll(todo));
#endif
        while (todo) {
          const int l = __ffsll((long long)todo) - 1;
          todo &= todo - 1ull;
          load_row(roff[r0 + l], A0);
          cert(r0 + l, A0);
        }
      }
      // sources: rows whose column is free-priced (v >= -LSAP_SS_TOL; v staged in w.spc)
#pragma unroll
      for (int q = 0; q < LQ; q++)
        if (lane + 64 * q < CC) w.spc[lane + 64 * q] = vr[q];
      wsync();
      for (int r = lane; r < R; r += 64) {
        const int cr = w.col4row[r];
        if (cr < 0 || cr >= CC) infeas = true;
        else if (w.spc[cr] >= -LSAP_SS_TOL) w.SR[r] |= 1;
      }
      wsync();
    }
    bool tie = bad || __any(infeas) || ncand > 64 * SS_CERT_ROUNDS;
    // Another optimum exists iff the tight digraph has a cycle: rows, plus a node Z for "a free
    // column"; row x -> the owner of each of x's tight unmatched columns (x could take it), or
    // -> Z for a free one; Z -> every source row (its column may be left free: v = 0).  An
    // optimum that changes a real pair needs a cycle through a real-matched candidate (it
    // leaves its real partner) or through a real tight edge of a candidate (a new real pair; a
    // cycle through a rejected-matched row over rejected entries only changes rejected pairs).
    // Up to 64 candidates at a time: candidate k's bit is seeded into its successors (all of
    // them when its matched entry is real, else those over real entries) and pushed along the tight
    // edges (each row expanded once per new bit set: its costs reloaded, its tight successors
    // OR-ed) until nothing changes; candidate k is on a cycle iff its own mask gets bit k.  Past
    // SS_CERT_BUDGET row expansions per LSAP: counted as a tie (scipy's order decides).
    if (!tie && ncand > 0) {
      unsigned long long* msk = (unsigned long long*)w.spc;  // reached-by bits per row
      unsigned long long* exm = (unsigned long long*)w.v;    // bits already pushed on per row
      int budget = SS_CERT_BUDGET;
      for (int c0 = 0; c0 < ncand && !tie; c0 += 64) {
        const int nc = ncand - c0 < 64 ? ncand - c0 : 64;
        wsync();
        for (int r = lane; r < R; r += 64) msk[r] = 0ull, exm[r] = 0ull;
        wsync();
        unsigned long long mz = 0ull, ez = 0ull;  // Z's
        // row x's tight successors (over real entries only: `ronly`) get `bits` (costs in `a`)
        auto push = [&](int x, const double* a, unsigned long long bits, bool ronly) {
          const int cx = (int)__builtin_amdgcn_readfirstlane((unsigned)w.col4row[x]);
          const double ux = w.u[x];
          bool zl = false;
#pragma unroll
          for (int q = 0; q < LQ; q++) {
            const int j = lane + 64 * q;
            if (j < CC && j != cx && (a[q] - ux) - vr[q] <= LSAP_SS_TOL &&
                (!ronly || a[q] <= max_d)) {
              const int y = w.row4col[j];
              if (y < 0) zl = true;
              else msk[y] |= bits;  // (distinct columns, distinct owners: no two lanes collide)
            }
          }
          if (__any(zl)) mz |= bits;
          wsync();
        };
        for (int k = 0; k < nc && !tie; k++) {
          const int cand = (int)__builtin_amdgcn_readfirstlane((unsigned)w.SC[c0 + k]);
          load_row(roff[cand], A0);
          push(cand, A0, 1ull << k, !(w.SR[cand] & 2));
          tie = --budget < 0;
        }
        bool changed = true;
        while (changed && !tie) {
          changed = false;
          for (int r0 = 0; r0 < R && !tie; r0 += 64) {
            const int r = r0 + lane;
            const unsigned long long nw = r < R ? msk[r] & ~exm[r] : 0ull;
            unsigned long long todo = __ballot(nw != 0ull);
            while (todo && !tie) {
              const int l = __ffsll((long long)todo) - 1;
              todo &= todo - 1ull;
              const int x = r0 + l;
              const unsigned long long bx =
                  (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(nw >> 32), l) << 32 |
                  (unsigned)__builtin_amdgcn_readlane((int)nw, l);
              if (lane == 0) exm[x] |= bx;
              load_row(roff[x], A0);
              push(x, A0, bx, false);
              changed = true;
              tie = --budget < 0;
            }
          }
          const unsigned long long nz = mz & ~ez;
          if (nz && !tie) {  // Z -> every source
            ez |= nz;
            for (int r = lane; r < R; r += 64)
              if (w.SR[r] & 1) msk[r] |= nz;
            wsync();
            changed = true;
          }
        }
        if (!tie) {
          bool hit = false;
          for (int k = lane; k < nc; k += 64)
            hit |= (msk[w.SC[c0 + k]] >> k) & 1ull;
          tie = __any(hit);
        }
      }
#ifdef BX_PHASE_TIMING
      SCOUNT(21, SS_CERT_BUDGET - budget);
#endif
    }
#ifdef BX_PHASE_TIMING
    SCOUNT(22, ncand);
    wsync();
    SCOUNT(25, SS_NOW() - tA);
#endif
    if (tie) {
      fstat = 2;
      wsync();
      return -1;  // (bad latched nothing: the exact path decides)
    }
    fstat = __any(tight_l) ? 1 : 0;
   } else {
    // Rows in pairs: the pair's two rows relaxed against the same v and their wave minima taken
    // together (two independent chains), then decided in order — the second one after the first
    // one's assignment, or relaxed again (its costs reloaded) when the first one's search changed
    // v.  The next pair's costs are in flight meanwhile: two register pairs alternate (an
    // unrolled pair of pair-steps), written only by unconditional loads (rows past the last one
    // re-read it), so no register row is ever merged or copied at a branch.
    double A0[LQ], A1[LQ], B0[LQ], B1[LQ];
    const int rlast = R - 1;
    auto roff_c = [&](int r) { return roff[r < rlast ? r : rlast]; };
    auto pair = [&](int cur, double* r0, double* r1) {
      double m0 = relax(r0, r0), m1 = relax(r1, r1);
      wave_min_bfly2(m0, m1);
      const bool chg = finish_row(cur, r0, m0);
      if (cur + 1 < R && !bad) {
        double m1b = m1;
        if (chg) {  // v changed: row cur+1 again
          load_row(roff_c(cur + 1), r1);
          m1b = wave_min_bfly(relax(r1, r1));
        }
        finish_row(cur + 1, r1, m1b);
      }
    };
    if (R > 0) {
      load_row(roff_c(0), A0);
      load_row(roff_c(1), A1);
    }
    for (int cur = 0; cur < R && !bad;) {
      load_row(roff_c(cur + 2), B0);
      load_row(roff_c(cur + 3), B1);
      pair(cur, A0, A1);
      cur += 2;
      if (cur >= R || bad) break;
      load_row(roff_c(cur + 2), A0);
      load_row(roff_c(cur + 3), A1);
      pair(cur, B0, B1);
      cur += 2;
    }
   }
  } else {  // LQ = 32 (IoU stage of more than 1024 candidates, rare): one row at a time
    double A[LQ], C[LQ];
    for (int cur = 0; cur < R && !bad; cur++) {
      load_row(roff[cur], C);
      const double m0 = wave_min_bfly(relax(C, A));
      finish_row(cur, A, m0);
    }
  }
  if (bad) {
    if (lane == 0) atomicExch(x.g.status, (int)BX_ERR_INVALID);
    return 0;
  }
  wsync();
#ifdef BX_PHASE_TIMING
  SCOUNT(10, t_slow);
  SCOUNT(11, SS_NOW() - t_all);
  SCOUNT(19, big_call ? SS_NOW() - t_all : 0);
#endif
  // every row is assigned a column in [0, CC) by now; a value outside it would be an engine
  // fault: latched as an error instead of indexing with it
  for (int q = lane; q < R; q += 64) {
    const int c = w.col4row[q];
    if (c < 0 || c >= CC) {
      atomicExch(x.g.status, (int)BX_ERR_INVALID);
      w.col4row[q] = 0;
    }
  }
  wsync();
  if (tr) {  // argsort(col4row): pairs ordered by the original row — col4row is injective
    // into [0, CC), so a table over the columns read in order sorts it (w.rem: free by now)
    int* t = w.rem;
    for (int j = lane; j < CC; j += 64) t[j] = -1;
    wsync();
    for (int q = lane; q < R; q += 64) t[w.col4row[q]] = q;
    wsync();
    wcompact(CC, [&](int j) { return t[j] >= 0; }, [&](int j, int p) {
      w.rows[p] = j;
      w.cols[p] = t[j];
    });
  } else {
    for (int q = lane; q < R; q += 64) {
      w.rows[q] = q;
      w.cols[q] = w.col4row[q];
    }
  }
  wsync();
  return R;
}

enum { M_GATED = 0, M_IOU = 1 };

// max_distance of the matching_cascade a detection takes part in (tracker.py:206-233): stage 1
// (confidence >= conf_thresh_high) matching_threshold * 0.8, stage 2 (medium confidence) the
// threshold itself.  The one definition both ss_cost_kernel's clamp and ss_match_kernel's stage
// loop use, so stage membership and the stored clamp can never disagree.
__device__ __forceinline__ double ss_stage_max_d(double thr, int stage) {
  return stage == 0 ? thr * 0.8 : thr;
}
__device__ __forceinline__ double ss_det_max_d(double conf, double thi, double thr) {
  return ss_stage_max_d(thr, conf >= thi ? 0 : 1);
}

// _enhance_cost_matrix (linear_assignment.py:251-273) of one entry, unclamped
__device__ __forceinline__ double enhance_v(double tq, double tcls, double tconf, const double* d,
                                            double e) {
  const double cq = (tq + d[7]) / 2.0;
  e *= clipd(1.0 - (cq - 0.5) * 0.2, 0.8, 1.2);
  if (tcls == d[5]) e *= 0.9;
  double cf = 1.0;
  if (tconf > 0.7 && d[4] > 0.7)
    cf = 0.9;
  else if (tconf < 0.3 || d[4] < 0.3)
    cf = 1.1;
  return e * cf;
}
__device__ __forceinline__ double enhance(const SsTrk& t, const double* d, double e) {
  return enhance_v(t.quality, t.cls, t.conf, d, e);
}
// ... and min_cost_matching's clamp at max_distance (linear_assignment.py:62-64)
__device__ __forceinline__ double enhance_clamp(const SsTrk& t, const double* d, double e,
                                                double max_d) {
  e = enhance(t, d, e);
  return e > max_d ? max_d + 1e-5 : e;
}

// Stage 1/2 cost of every confirmed track against every kept detection (wave per listed track,
// lanes over detections in quality order): gated_metric's NN distance, gate_cost_matrix with the
// motion / adaptive-lambda / track-specific shaping (linear_assignment.py:174-352), the
// id-preservation weight (tracker.py:283-298) and _enhance_cost_matrix — everything but the
// level's clamp.  And stage 3's cost of every listed track: iou_cost (iou_matching.py:55-87,
// INFTY past time_since_update 1) with _enhance_cost_matrix, unclamped.  Both only depend on the
// predicted tracks and the detections, so ss_match_kernel's solver reads them in place (by
// cascade rank / list position and sorted detection, in both orientations).
__global__ void __launch_bounds__(64) ss_cost_kernel(SsDev g, int seq0) {
  __shared__ double sh[32];
  const int b = blockIdx.y, seq = seq0 + b, k = blockIdx.x, lane = threadIdx.x;
  const int* sq = g.sq + (size_t)seq * SQS;
  if (k >= sq[Q_NTR]) return;
  const int nk = sq[Q_NK];
  const int slot = g.order[(size_t)seq * g.T + k];
  const SsTrk& t = g.trk[(size_t)seq * g.T + slot];
  if (nk == 0) return;
  {
    const double* dt = g.fdt + (size_t)seq * g.D * DTW;
    const int* dord = g.fdord + (size_t)seq * g.D;
    double* io = g.cost + (size_t)seq * 4 * g.T * g.D;  // [T][D] by list position
    double* ioT = io + (size_t)g.T * g.D;               // [D][T]
    const bool near = t.tsu <= 1;
    double bx[4];
    to_tlwh(t, bx);
    const double br0 = bx[0] + bx[2], br1 = bx[1] + bx[3], ab = bx[2] * bx[3];
    for (int c = lane; c < nk; c += 64) {
      const double* q = dt + (size_t)dord[c] * DTW;
      double e = SS_INFTY;
      if (near) {
        const double tl0 = fmax(bx[0], q[0]), tl1 = fmax(bx[1], q[1]);
        const double e0 = fmin(br0, q[0] + q[2]), e1 = fmin(br1, q[1] + q[3]);
        const double ww = fmax(0.0, e0 - tl0), hh = fmax(0.0, e1 - tl1);
        const double ai = ww * hh;
        e = 1.0 - ai / ((ab + q[2] * q[3]) - ai);
      }
      e = enhance(t, q, e);
      // stored with min_cost_matching's clamp (linear_assignment.py:67) at the IoU stage's
      // max_iou_distance, as the solver reads it
      if (e > g.max_iou) e = g.max_iou + 1e-5;
      io[(size_t)k * g.D + c] = e;
      ioT[(size_t)c * g.T + k] = e;
    }
  }
  if (t.state != 2) return;
  // this track's cascade rank: time_since_update ascending, -(quality + stability), list order
  int rk = 0;
  {
    const int ntr = sq[Q_NTR];
    const double* ck = g.ckey + (size_t)seq * g.T;
    const int* ca = g.ctsu + (size_t)seq * g.T;
    const int ai = ca[k];
    const double ki = ck[k];
    for (int q = lane; q < ntr; q += 64) {
      const int aq = ca[q];
      if (aq < 0) continue;
      const double kq = ck[q];
      rk += aq < ai || (aq == ai && (kq > ki || (kq == ki && q < k)));
    }
    for (int o = 32; o >= 1; o >>= 1) rk += __shfl_xor(rk, o);
    if (lane == 0) {
      g.crank[(size_t)seq * g.T + k] = rk;
      g.cpos[(size_t)seq * g.T + rk] = k;
    }
  }
  // per-track terms, computed once (lane 0) and shared through LDS
  if (lane == 0) {
    double S[16], L[16], rr[4];
    kf_meas_noise(KIND_BYTE, t.mean, 0.0, rr);
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) S[4 * i + j] = t.cov[8 * i + j] + (i == j ? rr[i] : 0.0);
    const bool ok = chol4(S, L);
    for (int i = 0; i < 16; i++) sh[i] = L[i];
    sh[16] = ok ? 1.0 : 0.0;
    sh[17] = 2.0 - t.motion_cons;
    double pp0 = 0.0, pp1 = 0.0;
    if (t.nvel > 0) pp0 = t.mean[0] + t.vel[t.nvel - 1][0], pp1 = t.mean[1] + t.vel[t.nvel - 1][1];
    sh[18] = pp0;
    sh[19] = pp1;
    const double af = pymin(t.age / 10.0, 1.0);
    double al = g.mc_lambda + (1 - g.mc_lambda) * af * 0.1;
    al = al * (0.8 + 0.4 * t.motion_cons);
    if (t.app_cons < 0.5) al = pymin(al * 1.2, 0.99);
    al = clipd(al, 0.1, 0.99);
    sh[20] = al;
    sh[21] = g.idw * pymin(t.hits / 10.0, 1.0);
    for (int i = 0; i < 4; i++) sh[22 + i] = t.mean[i];
  }
  __syncthreads();
  double L[16];
  for (int i = 0; i < 16; i++) L[i] = sh[i];
  const bool ok = sh[16] != 0.0;
  const double mf = sh[17], pp0 = sh[18], pp1 = sh[19], al = sh[20], pb = sh[21];
  const double m0 = sh[22], m1 = sh[23], m2 = sh[24], m3 = sh[25];
  const bool has_vel = t.nvel > 0, has_gal = t.gal_n > 0;
  const bool hq = t.quality > 0.8, hh = t.hits > 10 && t.tsu == 0, hs = t.high_streak > 3,
             ls = t.low_streak > 2;
  const double* dt = g.fdt + (size_t)seq * g.D * DTW;
  const int* dord = g.fdord + (size_t)seq * g.D;
  const double* nnd = g.nnd + ((size_t)seq * g.T + slot) * g.D;
  double* out = g.cfull + ((size_t)seq * g.T + rk) * g.D;
  double* outT = g.cfullT + (size_t)seq * g.D * g.T + rk;
  // min_cost_matching's clamp (linear_assignment.py:67) applied here, with the max_distance of the
  // one cascade a detection takes part in: stage 1 (high confidence) thr * 0.8, stage 2 (medium)
  // thr (tracker.py:206-233; thr after ss_pre_kernel's crowd-mode adjustment)
  const double thr = g.sqd[(size_t)seq * 2];
  // the track's real entries (<= its detections' max_distance: not clamped) as a list of sorted
  // detection indices for the solver's sparse first step; -1 when more than SS_TL, or when a
  // cost is NaN (only the dense path handles those)
  int16_t* tl = g.tlist + ((size_t)seq * g.T + rk) * SS_TL;
  int nreal = 0;
  bool nan_l = false;
  for (int c0 = 0; c0 < nk; c0 += 64) {
   const int c = c0 + lane;
   bool real = false;
   if (c < nk) {
    const double* d = dt + (size_t)dord[c] * DTW;
    double z[4];
    det_xyah(d, z);
    double gd;
    if (!ok) {
      gd = __builtin_nan("");
    } else {
      const double dd[4] = {z[0] - m0, z[1] - m1, z[2] - m2, z[3] - m3};
      double y[4], s2 = 0.0;
      for (int i = 0; i < 4; i++) {
        double sm = dd[i];
        for (int j = 0; j < i; j++) sm -= L[4 * i + j] * y[j];
        y[i] = sm / L[4 * i + i];
        s2 += y[i] * y[i];
      }
      gd = s2;
    }
    double v = has_gal ? nnd[(int)d[6]] : SS_INFTY;
    if (gd > SS_GATE) v = SS_INFTY;
    double m = gd * mf;
    if (has_vel) {
      const double ve = norm2(z[0] - pp0, z[1] - pp1);
      m *= 1.0 + pymin(ve / 50.0, 1.0);
    }
    v = al * v + (1 - al) * m;
    if (hq) v *= 0.95;
    if (hh) v *= 0.98;
    if (hs) v *= 0.97;
    if (ls) v *= 1.05;
    if (g.idw > 0) v *= (1.0 - pb);
    double e = enhance(t, d, v);
    const double md = ss_det_max_d(d[4], g.thi, thr);
    real = e <= md;
    nan_l |= e != e;
    if (e > md) e = md + 1e-5;
    out[c] = e;
    outT[(size_t)c * g.T] = e;
   }
   const unsigned long long m = __ballot(real);
   const int p = nreal + __popcll(m & ((1ull << lane) - 1ull));
   if (real && p < SS_TL) tl[p] = (int16_t)c;
   nreal += __popcll(m);
  }
  if (lane == 0) g.tcnt[(size_t)seq * g.T + rk] = (__any(nan_l) || nreal > SS_TL) ? -1 : nreal;
}

// The match kernel's solver wave: runs each posted LSAP (column slots per lane sized to CC: every
// slot past CC is a relaxation, a minimum and a ballot per row for nothing — measured at C4: 16 ->
// 8 slots for CC <= 512, match 1.63 -> 1.52 ms), answers with the pair count, until told to exit.
// Its own wave, so the solver's registers are not live across the cascade's bookkeeping.
__device__ __forceinline__ void lsap_server(SsCtx& x, LsapJob* jb, const int* roff,
                                            const int* cidx) {
  for (;;) {
    bool to = false;
    const int f = lds_flag_wait(&jb->flag, 0, true, x.g.status, &jb->abort, to);
    if (f < 0 || to) return;  // exit posted (the cascade always posts it last), or aborted
    const double mx = jb->max_d;
    const int R = jb->R, CC = jb->CC, kind = jb->kind, mode = jb->mode;
    const bool tr = jb->tr != 0;
    const double* P = lsap_mat(x.g, x.seq, kind, tr);
    // solve + certify first (mode 1, 2); on a tie scipy's order (mode 1) or a report (mode 2).
    // One call site per width: every inlined copy grows the kernel's register allocation.
    bool fast = mode != 0;
    int np = 0, st = 0;
    for (;;) {
      int fs = 0;
      // the cascade levels' matrices come with ss_cost_kernel's real-entry lists
      const int16_t* tl = kind == 0 ? x.g.tlist + (size_t)x.seq * x.g.T * SS_TL : nullptr;
      const int* tc = x.g.tcnt + (size_t)x.seq * x.g.T;
      np = CC <= 256    ? lsap_wave<4, true>(x, P, roff, cidx, mx, R, CC, tr, fast, fs, tl, tc)
           : CC <= 512  ? lsap_wave<8, true>(x, P, roff, cidx, mx, R, CC, tr, fast, fs, tl, tc)
           : CC <= 1024 ? lsap_wave<16, true>(x, P, roff, cidx, mx, R, CC, tr, fast, fs, tl, tc)
                        : lsap_wave<32, true>(x, P, roff, cidx, mx, R, CC, tr, fast, fs, tl, tc);
      if (np >= 0) {
        if (fast) st = fs;
        break;
      }
      if (mode == 2) {
        st = 3;
        np = 0;
        break;
      }
      fast = false;
      st = 2;
    }
    // the cascade gave up on this job (timeout): it may have posted another one since, which
    // this answer must not overwrite
    if (__builtin_amdgcn_readfirstlane((unsigned)__hip_atomic_load(
            &jb->abort, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0)
      return;
    if (x.lane == 0) jb->np = np, jb->stat = st;
    wsync();
    if (x.lane == 0) __hip_atomic_store(&jb->flag, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// min_cost_matching (linear_assignment.py:14-93) of track positions ti x sorted detections di:
// matches appended to w.mt at x.nm; unmatched tracks to ut_out (if non-null), detections to
// ud_out.  Cost rows lane per track (gated_metric + gate_cost_matrix + id preservation, or
// iou_cost), _enhance_cost_matrix and the max_distance clamp fused per entry.
__device__ __forceinline__ void min_cost_matching(SsCtx& x, int kind, double max_d, const int* ti, int nt,
                                  const int* di, int nd, int* ut_out, int& nut, int* ud_out,
                                  int& nud) {
  const SsDev& g = x.g;
  SsWs& w = x.w;
  const int lane = x.lane;
  x.lstat = 0;
  if (nd == 0 || nt == 0) {
    for (int k = lane; k < nt; k += 64)
      if (ut_out) ut_out[k] = ti[k];
    for (int k = lane; k < nd; k += 64) ud_out[k] = di[k];
    nut = nt;
    nud = nd;
    wsync();
    return;
  }
  // the solver's orientation: R x CC with R <= CC, transposed (tr) when detections are fewer
  const bool tr = nd < nt;
  const int R = tr ? nd : nt, CC = tr ? nt : nd;
  if (CC > 2048 || R > 1024) {  // track_cap, det_cap <= 1024
    if (lane == 0) atomicExch(g.status, (int)BX_ERR_INVALID);
    nut = nud = 0;
    return;
  }
  int* roff = x.flt;   // the solver rows' element offsets into P (LDS)
  int* cidx = x.cidx;  // the solver columns' element indices (LDS)
  const double* P = lsap_mat(g, x.seq, kind == M_GATED ? 0 : 1, tr);
  const int ld = tr ? g.T : g.D;
  double mx;
#ifdef BX_PHASE_TIMING
  const int seq = x.seq;
  wsync();
  unsigned long long t0 = SS_NOW();
#endif
  if (kind == M_GATED) {
    // ss_cost_kernel's gated + shaped + enhanced cost of (cascade rank, sorted detection), read
    // in place by the solver (its rows: tracks, or detections when tr, through cfullT); the
    // clamp at max_distance is this level's.
    const int* li = tr ? ti : di;  // columns
    const int* oi = tr ? di : ti;  // rows
    const int* rk = x.rank;        // track list position -> cascade rank
    for (int o = lane; o < R; o += 64) roff[o] = (tr ? oi[o] : rk[oi[o]]) * ld;
    for (int c = lane; c < CC; c += 64) cidx[c] = tr ? rk[li[c]] : li[c];
    mx = max_d;
  } else {
    // ss_cost_kernel's iou_cost + _enhance_cost_matrix of (list position, sorted detection),
    // read in place; the clamp at max_iou_distance here
    const int* li = tr ? ti : di;  // columns
    const int* oi = tr ? di : ti;  // rows
    for (int o = lane; o < R; o += 64) roff[o] = oi[o] * ld;
    for (int c = lane; c < CC; c += 64) cidx[c] = li[c];
    mx = max_d;
  }
  wsync();
#ifdef BX_PHASE_TIMING
  unsigned long long t1 = SS_NOW();
  SCOUNT(0, t1 - t0);
  SCOUNT(2, 1);
  SCOUNT(3, nt);
  SCOUNT(4, nd);
#endif
  // CC <= max(track_cap, det_cap) <= 1024, but for the IoU stage's candidates, which can list a
  // track twice (up to 2 track_cap columns)
  // (column slots per lane sized to CC: every slot past CC is a relaxation, a minimum and a
  // ballot per row for nothing — measured at C4: 16 -> 8 slots for CC <= 512, match 1.63 -> 1.52
  // ms; more instantiations (1, 2, 10, 12 slots) measured slower, 1.83 ms: the kernel's code and
  // register allocation grow with every inlined copy)
  // the LSAP runs on the solver wave (lsap_server): posted, then waited for
  int np_;
  {
    LsapJob* jb = x.job;
    if (lane == 0) {
      jb->max_d = mx;
      jb->R = R;
      jb->CC = CC;
      jb->tr = tr;
      jb->kind = kind;
      jb->mode = x.lmode;
    }
    wsync();
    bool to = __builtin_amdgcn_readfirstlane((unsigned)__hip_atomic_load(
                  &jb->abort, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
    if (!to) {  // (after an abort nothing is posted: the frame is void, BX_ERR_INVALID latched)
      if (lane == 0)
        __hip_atomic_store(&jb->flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      lds_flag_wait(&jb->flag, 0, false, g.status, &jb->abort, to);
    }
    np_ = to ? 0 : jb->np;
    x.lstat = to ? 0 : jb->stat;
    if (lane == 0 && !to) {
      x.sq[Q_LCALL]++;
      x.sq[x.lstat == 0 ? Q_LUNIQ : x.lstat == 1 ? Q_LCLAMP : Q_LTIE] += x.lstat <= 2;
    }
  }
#ifdef BX_PHASE_TIMING
  wsync();
  SCOUNT(1, SS_NOW() - t1);
#endif
  // assigned flags (w.SR rows, w.SC columns), unmatched in index order, then the rejected pairs
  for (int r = lane; r < nt; r += 64) w.SR[r] = 0;
  for (int c = lane; c < nd; c += 64) w.SC[c] = 0;
  wsync();
  for (int q = lane; q < np_; q += 64) w.SR[w.rows[q]] = 1, w.SC[w.cols[q]] = 1;
  wsync();
  nud = wcompact(nd, [&](int c) { return w.SC[c] == 0; }, [&](int c, int p) { ud_out[p] = di[c]; });
  nut = wcompact(nt, [&](int r) { return w.SR[r] == 0; },
                     [&](int r, int p) { if (ut_out) ut_out[p] = ti[r]; });
  for (int c0 = 0; c0 < np_; c0 += 64) {
    const int q = c0 + lane;
    bool ok = false, rej = false;
    int r = 0, c = 0;
    if (q < np_) {
      r = w.rows[q];
      c = w.cols[q];
      rej = (tr ? P[roff[c] + cidx[r]] : P[roff[r] + cidx[c]]) > max_d;
      ok = !rej;
    }
    const unsigned long long mo = __ballot(ok), mr = __ballot(rej);
    const unsigned long long below = (1ull << lane) - 1ull;
    if (ok) {
      const int p = x.nm + __popcll(mo & below);
      w.mt[2 * p] = ti[r];
      w.mt[2 * p + 1] = di[c];
    }
    if (rej) {
      const int p = __popcll(mr & below);
      if (ut_out) ut_out[nut + p] = ti[r];
      ud_out[nud + p] = di[c];
    }
    x.nm += __popcll(mo);
    nut += __popcll(mr);
    nud += __popcll(mr);
  }
  wsync();
}

// One matching stage of Tracker._enhanced_match with a single solver call site (the solver is
// inlined once per column-slot width, not once per stage: every inlined copy grows the kernel's
// register allocation).  M_GATED = matching_cascade (linear_assignment.py:96-171): levels by
// time_since_update ascending (up to tracker.max_age), each level's tracks ordered by
// -(quality + stability), stable; the unmatched detections end in w.ud.  M_IOU = one
// min_cost_matching of every track in ti (stage 3): unmatched tracks to ut_out, detections to w.ud.
__device__ void match_stage(SsCtx& x, int kind, double max_d, const int* ti, int nt, const int* di,
                            int nd, int* ut_out, int& nut) {
  SsWs& w = x.w;
  const int lane = x.lane;
  int nud = nd;
  for (int k = lane; k < nd; k += 64) w.ud[k] = di[k];
  int na = 1;
  const int max_age = x.sq[Q_MAXAGE];
  if (kind == M_GATED) {
    // the distinct time_since_update values, ascending (only levels <= max_age are matched)
    int* pres = x.flt;  // presence table over ages 0..max_age (LDS, 1024 entries)
    const int amax = max_age < 1023 ? max_age : 1023;
    for (int a = lane; a <= amax; a += 64) pres[a] = 0;
    wsync();
    int over = 0;
    for (int k = lane; k < nt; k += 64) {
      const int a = x.tsu[ti[k]];
      if (a <= amax)
        pres[a] = 1;
      else if (a <= max_age)
        over = 1;
    }
    over = __any(over);
    wsync();
    na = wcompact(amax + 1, [&](int a) { return pres[a] != 0; },
                      [&](int a, int p) { w.ages[p] = a; });
    if (over) {  // ages beyond the table (max_age >= 1024): the levels up to max_age, serially
      if (lane == 0) {
        for (int k = 0; k < nt; k++) {
          const int a = x.tsu[ti[k]];
          if (a <= amax || a > max_age) continue;
          bool seen = false;
          for (int q = 0; q < na && !seen; q++) seen = w.ages[q] == a;
          if (!seen) w.ages[na++] = a;
        }
        for (int p = 1; p < na; p++)
          for (int y = p; y > 0 && w.ages[y - 1] > w.ages[y]; y--) {
            const int tmp = w.ages[y];
            w.ages[y] = w.ages[y - 1];
            w.ages[y - 1] = tmp;
          }
      }
      na = bcast(na);
    }
    wsync();
    // members of ti by list position
    for (int p = lane; p < x.ntr; p += 64) x.inset[p] = 0;
    wsync();
    for (int k = lane; k < nt; k += 64) x.inset[ti[k]] = 1;
    wsync();
  }
  // LSAPs solved then certified; the columns' order (the previous level's unmatched detections)
  // is scipy's while every level so far was unique outright or tie-re-solved in scipy's order
  const int nm0 = x.nm;
  x.lmode = x.g.lsap_fast ? 1 : 0;
  for (int q = 0; q < na; q++) {
    const int* lt = ti;
    int nl = nt;
    if (kind == M_GATED) {
      const int age = w.ages[q];
      if (age > max_age) break;
      // the level's tracks in cascade order (its run of ranks, restricted to ti)
      nl = wcompact(
          x.ncf, [&](int r) { const int p = x.gpos[r]; return x.inset[p] && x.tsu[p] == age; },
          [&](int r, int p) { w.lvl[p] = x.gpos[r]; });
      lt = w.lvl;
    }
    int nud2 = 0, nut_l = 0;
    min_cost_matching(x, kind, max_d, lt, nl, w.ud, nud, kind == M_IOU ? ut_out : nullptr, nut_l,
                      w.ud2, nud2);
    if (x.lstat == 3) {
      // a real tie at a level whose columns' order may not be scipy's (an earlier level was only
      // unique up to rejected pairs): the whole stage again, every level in scipy's order
      x.nm = nm0;
      nud = nd;
      for (int k = lane; k < nd; k += 64) w.ud[k] = di[k];
      if (lane == 0) x.sq[Q_LRESTART]++;
      x.lmode = 0;
      q = -1;
      wsync();
      continue;
    }
    if (x.lstat == 1 && x.lmode == 1) x.lmode = 2;
    if (kind == M_IOU) nut = nut_l;
    for (int k = lane; k < nud2; k += 64) w.ud[k] = w.ud2[k];
    nud = nud2;
    wsync();
  }
}

// kf_update_soa(KIND_BYTE, mean, cov, 1, z, conf) on eight lanes (r = 0..7 of the same wave):
// lane r owns covariance row r and mean[r]; the innovation covariance and the gain rows travel
// by in-group shuffles, every entry being the expression kf_update_soa evaluates (same order).
__device__ void kf_update_octet(double* mean, double* cov, const double* z, double conf,
                                int r) {
  auto shfl = [](double v, int src) { return __shfl(v, src, 8); };
  double* crow = cov + 8 * r;
  double cr[8], mm[8];
  for (int j = 0; j < 8; j++) cr[j] = crow[j];
  for (int q = 0; q < 8; q++) mm[q] = mean[q];
  const double mr = mean[r];  // (not mm[r]: a run-time index sends the array to scratch)
  double rr[4], S[16], L[16];
  kf_meas_noise(KIND_BYTE, mm, conf, rr);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) S[4 * i + j] = shfl(cr[j], i) + (i == j ? rr[i] : 0.0);
  if (!chol4(S, L)) return;
  double Kr[4], y[4];  // gain row r
  for (int i = 0; i < 4; i++) {
    double sv = cr[i];
    for (int k = 0; k < i; k++) sv -= L[4 * i + k] * y[k];
    y[i] = sv / L[4 * i + i];
  }
  for (int i = 3; i >= 0; i--) {
    double sv = y[i];
    for (int k = i + 1; k < 4; k++) sv -= L[4 * k + i] * Kr[k];
    Kr[i] = sv / L[4 * i + i];
  }
  double sm = 0.0;
  for (int k = 0; k < 4; k++) sm += (z[k] - mm[k]) * Kr[k];
  const double mnew = mr + sm;
  double ks[4];
  for (int j = 0; j < 4; j++) {
    double sv = 0.0;
    for (int k = 0; k < 4; k++) sv += Kr[k] * S[4 * k + j];
    ks[j] = sv;
  }
  for (int j = 0; j < 8; j++) {
    double sv = 0.0;
    for (int k = 0; k < 4; k++) sv += ks[k] * shfl(Kr[k], j);
    crow[j] = cr[j] - sv;
  }
  mean[r] = mnew;  // the group read mean[] above (same wave, in order)
}

constexpr int UQ = 8;  // track_update keeps feature rows of up to 64·UQ elements in registers

// Track.update (track.py:204-277), wave-cooperative: Kalman update and scalars on lane 0, the
// feature vectors (similarity, adaptive-EMA smoothing, norms) on all lanes.
__device__ void track_update(SsCtx& x, int slot, int di) {
  const SsDev& g = x.g;
  const int lane = x.lane, F = g.F;
  SsTrk& t = x.trk[slot];
  const double* d = x.det(di);
  const int dk = x.det_in(di);
  const double* nf = g.nf + ((size_t)x.seq * g.D + dk) * F;
  const double* pr = g.dprep + ((size_t)x.seq * g.D + dk) * 4;
  // the register path's two feature rows are loaded before the Kalman update, their latency
  // under its arithmetic (pool_alloc below changes vmask only: nfeat / feat[] are final here)
  const int nfeat = t.nfeat;
  const bool in_regs = nfeat > 0 && F <= 64 * UQ;
  double rn[UQ], rl[UQ], wl = 0.0;
  if (in_regs) {
    const int lv = t.feat[nfeat - 1];
    const double* last = vecp(g, x.seq, slot, lv);
    wl = g.vwn[vidx(g, x.seq, slot, lv)];
#pragma unroll
    for (int r = 0; r < UQ; r++) {
      const int q = lane + 64 * r;
      rn[r] = q < F ? nf[q] : 0.0;
      rl[r] = q < F ? last[q] : 0.0;
    }
  }
  if (lane < 8) {
    double bb[4];
    det_xyah(d, bb);
    kf_update_octet(t.mean, t.cov, bb, d[4], lane);
  }
  if (lane == 0) t.conf = d[4], t.cls = d[5], t.det_ind = d[6];
  wsync();
  int v = -1;
  if (lane == 0) v = pool_alloc(t, g.VP);
  v = bcast(v);
  if (v < 0) {
    if (lane == 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
  } else {
    double* dst = vecp(g, x.seq, slot, v);
    const size_t vi = vidx(g, x.seq, slot, v);
    if (in_regs) {
      // the rows in registers (element lane + 64 r in slot r, wdot's order): the EMA vector is
      // written once and its norms come from registers; only numpy's pairwise tree reads it back
      auto rdot = [&](const double* u, const double* v2) {
        double sd = 0.0;
#pragma unroll
        for (int r = 0; r < UQ; r++)
          if (lane + 64 * r < F) sd += u[r] * v2[r];
#pragma unroll
        for (int dd = 32; dd >= 1; dd >>= 1) sd += __shfl_xor(sd, dd);
        return sd;
      };
      const double sim = rdot(rn, rl) / (pr[2] * wl + 1e-8);
      const double cf = d[4] > 0.7 ? 1.0 : (d[4] > 0.3 ? 0.5 : 0.2);
      const double af = sim > 0.7 ? 1.0 : (sim > 0.4 ? 0.7 : 0.4);
      const double a = clipd(t.base_alpha * cf * af, 0.1, 0.95);
#pragma unroll
      for (int r = 0; r < UQ; r++) rl[r] = a * rl[r] + (1 - a) * rn[r];
      const double ns = sqrt(rdot(rl, rl)) + 1e-8;
#pragma unroll
      for (int r = 0; r < UQ; r++) {
        rl[r] = rl[r] / ns;
        const int q = lane + 64 * r;
        if (q < F) dst[q] = rl[r];
      }
      const double wn = sqrt(rdot(rl, rl));
      // numpy's pairwise tree reads the row in its own lane mapping: from an LDS copy when the
      // caller gave one (no store -> load round trip through L2), else from dst
      const double* prow = dst;
      if (x.w.rowbuf) {
#pragma unroll
        for (int r = 0; r < UQ; r++) {
          const int q = lane + 64 * r;
          if (q < F) x.w.rowbuf[q] = rl[r];
        }
        prow = x.w.rowbuf;
      }
      wsync();  // the row visible to the pairwise tree's lane mapping
      const double pn = wpw_norm(prow, F, x.w.pwlo, x.w.pwln, x.w.pwleaf) + 1e-8;
      double* dstn = vecnp(g, x.seq, slot, v);
#pragma unroll
      for (int r = 0; r < UQ; r++) {
        const int q = lane + 64 * r;
        if (q < F) dstn[nn_pos(q, F)] = rl[r] / pn;
      }
      if (lane == 0) {
        t.app_cons = 0.9 * t.app_cons + 0.1 * sim;
        g.vwn[vi] = wn;
        g.vden[vi] = pn;
      }
    } else if (nfeat > 0) {
      const int lv = t.feat[nfeat - 1];
      const double* last = vecp(g, x.seq, slot, lv);
      const double wl = g.vwn[vidx(g, x.seq, slot, lv)];
      const double sim = wdot(nf, last, F) / (pr[2] * wl + 1e-8);
      const double cf = d[4] > 0.7 ? 1.0 : (d[4] > 0.3 ? 0.5 : 0.2);
      const double af = sim > 0.7 ? 1.0 : (sim > 0.4 ? 0.7 : 0.4);
      const double a = clipd(t.base_alpha * cf * af, 0.1, 0.95);
      for (int q = lane; q < F; q += 64) dst[q] = a * last[q] + (1 - a) * nf[q];
      wsync();
      const double ns = sqrt(wdot(dst, dst, F)) + 1e-8;
      for (int q = lane; q < F; q += 64) dst[q] = dst[q] / ns;
      wsync();
      const double wn = sqrt(wdot(dst, dst, F));
      const double pn = wpw_norm(dst, F, x.w.pwlo, x.w.pwln, x.w.pwleaf) + 1e-8;
      double* dstn = vecnp(g, x.seq, slot, v);
      for (int q = lane; q < F; q += 64) dstn[nn_pos(q, F)] = dst[q] / pn;
      if (lane == 0) {
        t.app_cons = 0.9 * t.app_cons + 0.1 * sim;
        g.vwn[vi] = wn;
        g.vden[vi] = pn;
      }
    } else {
      double* dstn = vecnp(g, x.seq, slot, v);
      const double pn = pr[3];
      for (int q = lane; q < F; q += 64) {
        dst[q] = nf[q];
        dstn[nn_pos(q, F)] = nf[q] / pn;
      }
      if (lane == 0) {
        g.vwn[vi] = pr[2];
        g.vden[vi] = pr[3];
      }
    }
    if (lane == 0) {
      if (t.nfeat == MAXF) {
        for (int k = 0; k < MAXF - 1; k++) t.feat[k] = t.feat[k + 1];
        t.nfeat--;
      }
      t.feat[t.nfeat++] = v;
    }
  }
  if (lane == 0) track_update_scalars(t, d);
  wsync();
}

// Track.__init__ (track.py:76-131) into a free slot, by one lane (births run lane-parallel).
// The detection's feature, normalised as the reference normalises it in place, becomes pool
// entry 0; ss_fit_kernel copies the vector (born_dk), nothing reads it earlier in the frame.
__device__ void track_birth(SsCtx& x, int slot, int di, int id) {
  const SsDev& g = x.g;
  SsTrk& t = x.trk[slot];
  const double* d = x.det(di);
  const int dk = x.det_in(di);
  double bb[4];
  det_xyah(d, bb);
  t.id = id;
  t.conf = d[4], t.cls = d[5], t.det_ind = d[6];
  t.hits = 1, t.age = 1, t.tsu = 0;
  t.base_alpha = g.ema_alpha;
  t.state = g.born ? 2 : 1;
  t.confh[0] = d[4];
  t.nconf = 1;
  t.n_init = g.n_init;
  t.max_age = x.sq[Q_MAXAGE];
  t.quality = d[7];
  t.stability = 0.0;
  t.app_cons = 1.0;
  t.motion_cons = 1.0;
  t.nvel = t.npos = 0;
  t.missed = 0;
  t.confirmed_det = 1;
  t.low_streak = 0;
  t.high_streak = d[4] > 0.7 ? 1 : 0;
  t.lost_frame = 0;
  t.gal_n = 0;
  t.gal_clock = 0;
  t.gmask = 0ull;
  t.vmask = 1ull;  // pool entry 0 holds the first feature
  t.born_dk = dk;
  kf_initiate(KIND_BYTE, bb, t.mean, t.cov);
  push2(t.pos, t.npos, bb);
  t.feat[0] = 0;
  t.nfeat = 1;
  const size_t vi = vidx(g, x.seq, slot, 0);
  const double* pr = g.dprep + ((size_t)x.seq * g.D + dk) * 4;
  g.vwn[vi] = pr[2];
  g.vden[vi] = pr[3];
}

// detect_crowd_situations' pair test (utils/occlusion_handler.py:45-87; the fork passes tlwh
// boxes that it reads as xyxy): the track pairs whose intersection exceeds 30 % of either box,
// counted over the whole grid (block per slice of rows, threads over partners) into Q_CROWDN.
// Blocks per sequence: 16 for a few sequences (C4's 1024 tracks), 2 for many (each block loads
// every box of its sequence: at 256 sequences 16 blocks each spent 154 us mostly on those loads);
// the boxes in dynamic LDS sized to the track capacity.
constexpr int CROWD_BLOCKS = 16;
#ifndef BX_CROWD_BLOCKS_MANY
#define BX_CROWD_BLOCKS_MANY 2
#endif
__host__ __device__ constexpr int crowd_blocks(int nseq) {
  return nseq >= 64 ? BX_CROWD_BLOCKS_MANY : CROWD_BLOCKS;
}
__global__ void __launch_bounds__(256) ss_crowd_kernel(SsDev g, int seq0) {
  extern __shared__ __align__(16) double box[];  // [4 * T]
  const int b = blockIdx.y, seq = seq0 + b;
  int* sq = g.sq + (size_t)seq * SQS;
  const int nn = sq[Q_NTR];
  if (!g.crowd || nn < 3) return;
  const int* order = g.order + (size_t)seq * g.T;
  const SsTrk* trk = g.trk + (size_t)seq * g.T;
  for (int k = threadIdx.x; k < nn; k += 256) to_tlwh(trk[order[k]], box + 4 * k);
  __syncthreads();
  int high = 0;
  for (int i = blockIdx.x; i < nn; i += gridDim.x) {
    const double* bi = box + 4 * i;
    for (int j = i + 1 + threadIdx.x; j < nn; j += 256) {
      const double* bj = box + 4 * j;
      const double xx1 = pymax(bi[0], bj[0]), yy1 = pymax(bi[1], bj[1]);
      const double xx2 = pymin(bi[2], bj[2]), yy2 = pymin(bi[3], bj[3]);
      const double ww = pymax(0, xx2 - xx1), hh = pymax(0, yy2 - yy1);
      const double inter = ww * hh;
      if (inter > 0) {
        const double ai = (bi[2] - bi[0]) * (bi[3] - bi[1]);
        const double aj = (bj[2] - bj[0]) * (bj[3] - bj[1]);
        if (pymax(inter / ai, inter / aj) > 0.3) high++;
      }
    }
  }
  for (int o = 32; o >= 1; o >>= 1) high += __shfl_xor(high, o);
  if ((threadIdx.x & 63) == 0 && high) atomicAdd(sq + Q_CROWDN, high);
}

// ss_pre_kernel (one wave per sequence): detections, crowd mode, CMC warp, quality + stable sort,
// Kalman predict.  The detection table (fdt, fdord) and the predicted tracks are the input of
// ss_cost_kernel and ss_match_kernel.
// Tracker.camera_update + Tracker.predict of every listed track (strongsort.py:144-149,
// tracker.py:63-70): wave per track, lane 8i + j owning covariance entry (i, j) — the row sums of
// F P F^T come by two shuffles, each entry the expression track_predict evaluates; the mean, the
// histories and the consistency scalars on lane 0.  With no detection kept the reference skips
// the camera update (tracker.update([]) path).  Runs before ss_pre_kernel on its stream.
__global__ void __launch_bounds__(64)
    ss_motion_kernel(SsDev g, int seq0, const double* __restrict__ warps) {
  const int b = blockIdx.y, seq = seq0 + b, p = blockIdx.x, lane = threadIdx.x;
  if (p >= g.sq[(size_t)seq * SQS + Q_NTR]) return;
  const bool keep = g.pk[(size_t)seq * (g.T + 3) + g.T + 2] != 0;
  SsTrk& t = g.trk[(size_t)seq * g.T + g.order[(size_t)seq * g.T + p]];
  if (keep && lane == 0) {
    double wm[6] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0};
    if (warps)
      for (int q = 0; q < 6; q++) wm[q] = warps[(size_t)b * 6 + q];
    track_camera(t, wm);
  }
  __syncthreads();
  // track_predict: q from the (camera-updated) mean, then P = F (P F^T) + Q entrywise
  double q[8];
  kf_process_noise(KIND_BYTE, t.mean, q);
  const int i = lane >> 3, j = lane & 7;
  const double pij = t.cov[lane];
  const double pj4 = __shfl(pij, (lane & ~7) | ((j + 4) & 7));
  const double mij = j < 4 ? pij + pj4 : pij;
  const double m4 = __shfl(mij, (lane + 32) & 63);
  double v;
  if (i < 4) {
    const double s2 = mij + m4;
    v = i == j ? s2 + q[i] : s2;
  } else {
    v = i == j ? mij + q[i] : mij;
  }
  __syncthreads();  // every lane read its operands (and q read the mean) before the writes
  t.cov[lane] = v;
  if (lane == 0) {
    double* m = t.mean;
    for (int k = 0; k < 4; k++) m[k] = m[k] + m[k + 4];
    t.age++;
    t.tsu++;
    push2(t.vel, t.nvel, t.mean + 4);
    push2(t.pos, t.npos, t.mean);
    if (t.npos >= 2) motion_cons(t, t.pos[t.npos - 2], t.pos[t.npos - 1]);
  }
}

__global__ void __launch_bounds__(64)
    ss_pre_kernel(SsDev g, int seq0, const double* __restrict__ dets,
                  const int* __restrict__ det_off, const double* __restrict__ warps) {
  extern __shared__ __align__(16) char ss_lds[];
  __shared__ double sbox[4 * 1024];  // crowd test: track boxes; then the detection sort keys
  const int lane = threadIdx.x, b = blockIdx.x, seq = seq0 + b;
  SsWs w;
  ws_carve(g, seq, w, ss_lds);
#ifdef BX_PHASE_TIMING
  unsigned long long t_last = SS_NOW();
#endif
  SsCtx x{g, w, seq, lane, g.trk + (size_t)seq * g.T, g.sq + (size_t)seq * SQS,
          g.sqd + (size_t)seq * 2, g.lost + (size_t)seq * LOSTN, 0, 0, 0, 0};
  int* sq = x.sq;
  int* order = g.order + (size_t)seq * g.T;
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) {
    if (lane == 0) atomicExch(g.status, (int)BX_ERR_CAPACITY);
    n = g.D;
  }
  const int frame = sq[Q_FRAME] + 1;
  x.ntr = sq[Q_NTR];
  x.nlost = sq[Q_NLOST];
  const int nt0 = x.ntr;
  for (int p = lane; p < x.ntr; p += 64) w.lst[p] = order[p];
  // detections with conf >= min_conf, input order (strongsort.py:141-143)
  x.nk = wave_compact(
      n, [&](int k) { return dets[(size_t)(r0 + k) * 6 + 4] >= g.min_conf; },
      [&](int k, int p) {
        const double* r = dets + (size_t)(r0 + k) * 6;
        double* d = w.dt + (size_t)p * DTW;
        d[0] = r[0], d[1] = r[1], d[2] = r[2] - r[0], d[3] = r[3] - r[1];
        d[4] = r[4], d[5] = r[5], d[6] = (double)k, d[7] = 0.0;
        w.dord[p] = p;
      });
  int fid = frame;
  SSTAMP(0);
  if (x.nk == 0) {  // (the tracks were predicted by ss_motion_kernel)
    fid = 0;  // tracker.update([]) passes frame_id=None
  } else {
    if (g.crowd) {  // detect_crowd_situations (reads the tlwh boxes as xyxy)
      int crowd = 0;
      const int nn = x.ntr;
      if (nn >= 3) {
        const long long high = sq[Q_CROWDN];  // ss_crowd_kernel's count
        const long long total = (long long)nn * (nn - 1) / 2;
        crowd = (double)high / (double)(total > 1 ? total : 1) > 0.3;
      }
      if (lane == 0) {
        sq[Q_CROWD] = crowd;
        if (crowd) {  // _adjust_for_crowd_mode (strongsort.py:183-208)
          if (!sq[Q_ORIG]) {
            sq[Q_OMAXAGE] = sq[Q_MAXAGE];
            x.sqd[1] = x.sqd[0];
            sq[Q_OBUDGET] = sq[Q_BUDGET];
            sq[Q_ORIG] = 1;
          }
          sq[Q_MAXAGE] = (int)(sq[Q_OMAXAGE] * 1.5);
          x.sqd[0] = x.sqd[1] * 0.8;
          if (sq[Q_BUDGET]) sq[Q_BUDGET] = sq[Q_OBUDGET] * 2 < 300 ? sq[Q_OBUDGET] * 2 : 300;
        }
      }
      __syncthreads();
    }
    SSTAMP(1);
#ifdef BX_PHASE_TIMING
    unsigned long long tq = SS_NOW();
#endif
    const int crowd_mode = sq[Q_CROWD];
    for (int i = lane; i < x.nk; i += 64) {  // _compute_detection_quality
      double* d = w.dt + (size_t)i * DTW;
      double q = d[4];
      const double fn = g.dprep[((size_t)seq * g.D + (int)d[6]) * 4 + 0];
      q = 0.7 * q + 0.3 * pymin(fn / 10.0, 1.0);
      const double ww = d[2], hh = d[3];
      if (hh > 0) {
        const double aq = pymax(0.1, 1.0 - fabs(ww / hh - 0.5) / 2.0);
        q = 0.9 * q + 0.1 * aq;
      }
      if (crowd_mode) q += pymin(ww * hh / 10000.0, 0.1);
      d[7] = q;
    }
    __syncthreads();
#ifdef BX_PHASE_TIMING
    SCOUNT(12, SS_NOW() - tq);
#endif
    // (the stable sort by quality is ss_sort_kernel's, next on this stream)
  }
  if (!fid) fid = sq[Q_HIST];
  // the cascade order of the confirmed tracks: time_since_update ascending, then -(quality +
  // stability) with list order on ties (linear_assignment.py:96-171, 276-285) — every cascade
  // level of stage 1 or 2 is a run of it (stage 2's a subsequence), so the cost kernel indexes
  // its matrix by this rank and the levels gather contiguous rows
  // (ranks: ss_cost_kernel, from these keys)
  {
    int nc = 0;
    for (int p = lane; p < x.ntr; p += 64) {
      const SsTrk& t = x.trk[w.lst[p]];
      g.ckey[(size_t)seq * g.T + p] = t.quality + t.stability;
      g.ctsu[(size_t)seq * g.T + p] = t.state == 2 ? t.tsu : -1;
      g.crank[(size_t)seq * g.T + p] = -1;
      nc += t.state == 2;
    }
    for (int o = 32; o >= 1; o >>= 1) nc += __shfl_xor(nc, o);
    if (lane == 0) g.ncf[seq] = nc;
  }
  if (lane == 0) {
    sq[Q_NK] = x.nk;
    sq[Q_FID] = fid;
    sq[Q_CROWDN] = 0;  // the next frame's ss_crowd_kernel counts from zero
  }
  SSTAMP(2);
}

// The detections' stable sort by quality, descending (tracker.py's sorted(..., reverse=True) of
// _compute_detection_quality): rank(i) = #{j : q_j > q_i} + #{j < i : q_j == q_i}, a thread per
// detection against all keys in LDS; dord[rank(i)] = i.  (In ss_pre_kernel's one wave this was
// 0.4 ms at C4 — ~514 keys, 16 per lane, beside the gallery distance's MFMA waves.)
__global__ void __launch_bounds__(256) ss_sort_kernel(SsDev g, int seq0) {
  __shared__ double ks[1024];
  const int seq = seq0 + blockIdx.y;
  const int nk = g.sq[(size_t)seq * SQS + Q_NK];
  if ((int)blockIdx.x * 256 >= nk) return;
  const double* dt = g.fdt + (size_t)seq * g.D * DTW;
  int* dord = g.fdord + (size_t)seq * g.D;
  for (int i = threadIdx.x; i < nk; i += 256) ks[i] = dt[(size_t)i * DTW + 7];
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nk) return;
  const double ki = ks[i];
  int r = 0;
  for (int j = 0; j < nk; j++) {
    const double kj = ks[j];
    r += (kj > ki) || (kj == ki && j < i);
  }
  dord[r] = i;
}

// ss_match_kernel (one two-wave workgroup per sequence): the three matching stages of
// Tracker._enhanced_match (stage 1/2 costs gathered from ss_cost_kernel's matrix).  Wave 0 runs
// the cascade and posts each LSAP (LsapJob) to wave 1, the solver, which keeps its own register
// context.  Hands the matches (fmt), the unmatched tracks (ffut) and detections (faud) to the next
// launches.
__global__ void __launch_bounds__(128) SS_MATCH_ATTR
    ss_match_kernel(SsDev g, int seq0) {
  extern __shared__ __align__(16) char ss_lds[];
  __shared__ int srank[1024], sgpos[1024], sinset[1024];
  __shared__ int flt[2048], fld[1024];  // solver column indices; sorted-detection membership
  __shared__ int stsu[1024], sage[1024];
  __shared__ LsapJob job;
  const int lane = threadIdx.x & 63, b = blockIdx.x, seq = seq0 + b;
  SsWs w;
  ws_carve(g, seq, w, ss_lds);
  if (threadIdx.x == 0) job.flag = 0, job.abort = 0;
  __syncthreads();  // the only barrier of both waves; from here each synchronises itself
  // the LSAP's rows' offsets and columns' indices (written by the cascade wave, read by the
  // solver wave): sage and flt
  // the wave's role, wave-uniform (readfirstlane: scalar branches, no divergent-region masks)
  const int wid = (int)__builtin_amdgcn_readfirstlane((unsigned)(threadIdx.x >> 6));
  if (wid == 1) {  // the solver wave
    SsCtx xs{g, w, seq, lane, g.trk + (size_t)seq * g.T, g.sq + (size_t)seq * SQS,
             g.sqd + (size_t)seq * 2, g.lost + (size_t)seq * LOSTN, 0, 0, 0, 0};
    lsap_server(xs, &job, sage, flt);
    return;
  }
#ifdef BX_PHASE_TIMING
  unsigned long long t_last = SS_NOW();
#endif
  SsCtx x{g, w, seq, lane, g.trk + (size_t)seq * g.T, g.sq + (size_t)seq * SQS,
          g.sqd + (size_t)seq * 2, g.lost + (size_t)seq * LOSTN, 0, 0, 0, 0};
  int* sq = x.sq;
  const int* order = g.order + (size_t)seq * g.T;
  x.ntr = sq[Q_NTR];
  x.nlost = sq[Q_NLOST];
  x.nk = sq[Q_NK];
  if (lane == 0) {  // gallery rows compared by this frame's ss_nn_kernel (a statistic)
    sq[Q_ROWSL] = sq[Q_ROWS];
    sq[Q_ROWS] = 0;
  }
  for (int p = lane; p < x.ntr; p += 64) {
    w.lst[p] = order[p];
    stsu[p] = x.trk[order[p]].tsu;
    const int r = g.crank[(size_t)seq * g.T + p];
    srank[p] = r;
    if (r >= 0) sgpos[r] = p;
  }
  x.ncf = g.ncf[seq];
  x.tsu = stsu;
  x.flt = sage;
  x.cidx = flt;
  x.rank = srank;
  x.gpos = sgpos;
  x.inset = sinset;
  x.job = &job;
  wsync();

  // ---- Tracker._enhanced_match (tracker.py:183-281, P6) --------------------------------------
  x.nm = 0;
  const int ncf = wcompact(x.ntr, [&](int p) { return x.trk[w.lst[p]].state == 2; },
                               [&](int p, int q) { w.conf_t[q] = p; });
  const int nun = wcompact(x.ntr, [&](int p) { return x.trk[w.lst[p]].state != 1; },
                               [&](int p, int q) { w.unconf_t[q] = p; });
  const int nhi = wcompact(x.nk, [&](int i) { return x.det(i)[4] >= g.thi; },
                               [&](int i, int q) { w.hi[q] = i; });
  const int nmed = wcompact(
      x.nk, [&](int i) { const double c = x.det(i)[4]; return g.tlo <= c && c < g.thi; },
      [&](int i, int q) { w.med[q] = i; });
  const int nlo = wcompact(x.nk, [&](int i) { return x.det(i)[4] < g.tlo; },
                               [&](int i, int q) { w.lo[q] = i; });
  int naut = ncf, naud = x.nk;
  for (int k = lane; k < ncf; k += 64) w.aut[k] = w.conf_t[k];
  for (int k = lane; k < x.nk; k += 64) w.aud[k] = k;
  wsync();
  const double thr = x.sqd[0];
  SSTAMP(3);
  const int NT = x.ntr, NK = x.nk;
  // stage 1: high-confidence detections x confirmed tracks (cascade); stage 2: medium-confidence
  // detections x the remaining confirmed tracks (cascade); stage 3: IoU on unconfirmed
  // (= non-tentative) + unmatched with time_since_update == 1 — one loop, one solver call site
  int ncand = 0, nut3 = 0;
  for (int st = 0; st < 3; st++) {
    if (st == 1) SSTAMP(4);
    if (st == 2) SSTAMP(5);
    const int* ti = w.conf_t;
    const int* di = w.hi;
    int nt = ncf, nd = nhi;
    double md = ss_stage_max_d(thr, 0);
    int kind = M_GATED;
    if (st == 1) {
      // the unmatched tracks are all confirmed (a subset of conf_t)
      for (int k = lane; k < naut; k += 64) w.ti2[k] = w.aut[k];
      for (int k = lane; k < NK; k += 64) fld[k] = 0;
      wsync();
      for (int k = lane; k < naud; k += 64) fld[w.aud[k]] = 1;
      wsync();
      nd = wcompact(nmed, [&](int k) { return fld[w.med[k]] != 0; },
                        [&](int k, int q) { w.rd[q] = w.med[k]; });
      ti = w.ti2;
      nt = naut;
      di = w.rd;
      md = ss_stage_max_d(thr, 1);
    } else if (st == 2) {
      ncand = nun;
      for (int k = lane; k < nun; k += 64) w.cand[k] = w.unconf_t[k];
      wsync();
      ncand += wcompact(naut, [&](int k) { return stsu[w.aut[k]] == 1; },
                            [&](int k, int q) { w.cand[nun + q] = w.aut[k]; });
      nd = wcompact(naud, [&](int k) { return !(x.det(w.aud[k])[4] < g.tlo); },
                        [&](int k, int q) { w.rd[q] = w.aud[k]; });
      ti = w.cand;
      nt = ncand;
      di = w.rd;
      md = g.max_iou;
      kind = M_IOU;
    }
    if (!(nd && nt)) continue;
    const int m0 = x.nm;
    match_stage(x, kind, md, ti, nt, di, nd, w.ut3, nut3);
    naut = filter_matched_fl(w.aut, naut, w.mt, m0, x.nm, 0, w.tmp, flt, NT);
    naud = filter_matched_fl(w.aud, naud, w.mt, m0, x.nm, 1, w.tmp, fld, NK);
  }
  (void)nlo;
  for (int k = lane; k < NT; k += 64) flt[k] = 0;
  wsync();
  for (int k = lane; k < ncand; k += 64) flt[w.cand[k]] = 1;
  wsync();
  int nfut = wcompact(naut, [&](int k) { return flt[w.aut[k]] == 0; },
                          [&](int k, int q) { w.fut[q] = w.aut[k]; });
  for (int k = lane; k < nut3; k += 64) w.fut[nfut + k] = w.ut3[k];
  nfut += nut3;
  wsync();
  SSTAMP(6);

  // the matched tracks' updates are ss_update_kernel's, the misses follow them (ss_post_kernel):
  // a track listed twice among stage 3's candidates can be both matched and missed, and
  // mark_missed must see the updated time_since_update (tracker.py:139-145)
  // a track listed twice among stage 3's candidates can also be matched twice: the reference
  // updates it twice, in match order.  Later occurrences are flagged (negative position) and
  // listed after the matches; ss_update_kernel does the first ones, ss_post_kernel these in order.
  // (a match is a repeat iff an earlier match has its track: the first match per list position
  // by an LDS atomicMin table — the membership table is free by now — not a scan of the earlier
  // matches per match, which at C4's ~470 matches was ~0.3 M cycles of the wave)
  int* dupl = w.mt + 2 * (g.D + 2);
  int* first = sinset;
  for (int p = lane; p < NT; p += 64) first[p] = 0x7fffffff;
  wsync();
  for (int q = lane; q < x.nm; q += 64) atomicMin(&first[w.mt[2 * q]], q);
  wsync();
  const int ndup = wcompact(
      x.nm, [&](int q) { return first[w.mt[2 * q]] < q; }, [&](int q, int p) { dupl[p] = q; });
  for (int k = lane; k < ndup; k += 64) w.mt[2 * dupl[k]] = -1 - w.mt[2 * dupl[k]];
  if (lane == 0) {
    sq[Q_NDUP] = ndup;
    sq[Q_NFUT] = nfut;
    sq[Q_NM] = x.nm;
    sq[Q_NAUD] = naud;
  }

  SCOUNT(6, x.nm);
  SSTAMP(7);
  wsync();
  // the solver wave's exit: the cascade must ALWAYS post it last (no early return above), or the
  // solver waits out SS_SPIN_TICKS and latches BX_ERR_INVALID
  if (lane == 0) __hip_atomic_store(&job.flag, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Track.update for every match of the three stages (tracker.py:139-141): wave per match.
// SS_UPD_W waves per workgroup, a match each with its own LDS scratch.  (Measured at 256 seq:
// one wave 0.100 ms, two or four 0.172-0.175 ms.)
#ifndef SS_UPD_W
#define SS_UPD_W 1
#endif
__global__ void __launch_bounds__(64 * SS_UPD_W) ss_update_kernel(SsDev g, int seq0) {
  __shared__ int lo[SS_UPD_W][PW_MAXLEAF], ln[SS_UPD_W][PW_MAXLEAF];
  __shared__ double leaf[SS_UPD_W][PW_MAXLEAF];
  __shared__ double row[SS_UPD_W][64 * UQ];
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int b = blockIdx.y, seq = seq0 + b, q = blockIdx.x * SS_UPD_W + wv;
  int* sq = g.sq + (size_t)seq * SQS;
  if (q >= sq[Q_NM]) return;  // (wave-uniform; no workgroup barrier below)
  SsWs w{};
  ws_frame(g, seq, w);
  if (w.mt[2 * q] < 0) return;  // a repeated track: ss_post_kernel
  w.pwlo = lo[wv];
  w.pwln = ln[wv];
  w.pwleaf = leaf[wv];
  w.rowbuf = row[wv];
  SsCtx x{g, w, seq, (int)threadIdx.x & 63, g.trk + (size_t)seq * g.T, sq,
          g.sqd + (size_t)seq * 2, g.lost + (size_t)seq * LOSTN, 0, 0, 0, 0};
  track_update(x, g.order[(size_t)seq * g.T + w.mt[2 * q]], w.mt[2 * q + 1]);
}

// ss_post_kernel (one wave per sequence): ID recovery, births, the lost buffer, the output rows.
__global__ void __launch_bounds__(64)
    ss_post_kernel(SsDev g, int seq0, const int* __restrict__ det_off, double* __restrict__ out,
                   int* __restrict__ out_count) {
  extern __shared__ __align__(16) char ss_lds[];
  const int lane = threadIdx.x, b = blockIdx.x, seq = seq0 + b;
  SsWs w;
  ws_carve(g, seq, w, ss_lds);
#ifdef BX_PHASE_TIMING
  unsigned long long t_last = SS_NOW();
#endif
  SsCtx x{g, w, seq, lane, g.trk + (size_t)seq * g.T, g.sq + (size_t)seq * SQS,
          g.sqd + (size_t)seq * 2, g.lost + (size_t)seq * LOSTN, 0, 0, 0, 0};
  int* sq = x.sq;
  int* order = g.order + (size_t)seq * g.T;
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) n = g.D;
  const int frame = sq[Q_FRAME] + 1;
  const int fid = sq[Q_FID];
  int naud = sq[Q_NAUD];
  x.ntr = sq[Q_NTR];
  x.nlost = sq[Q_NLOST];
  x.nk = sq[Q_NK];
  const int nt0 = x.ntr;
  for (int p = lane; p < x.ntr; p += 64) w.lst[p] = order[p];
  __syncthreads();
  // repeated matches of one track, in match order (see ss_match_kernel)
  {
    const int ndup = sq[Q_NDUP];
    const int* dupl = w.mt + 2 * (g.D + 2);
    for (int k = 0; k < ndup; k++) {
      const int q = dupl[k];
      track_update(x, w.lst[-1 - w.mt[2 * q]], w.mt[2 * q + 1]);
    }
  }
  // ---- misses (tracker.py:142-145), after the updates ------------------------------------------
  {
    const int nfut = sq[Q_NFUT];
    for (int k = 0; k < nfut; k += 64) {
      // a position may be listed twice: serialise duplicates by processing one wave-slice at a
      // time in list order, lanes of one slice never share a track (checked below)
      const int kk = k + lane;
      int pos = kk < nfut ? w.fut[kk] : -1;
      bool dup_before = false;
      for (int j = 0; j < 64; j++) {
        const int pj = __shfl(pos, j);
        if (j < lane && pj == pos) dup_before = true;
      }
      if (pos >= 0 && !dup_before) track_missed(x.trk[w.lst[pos]]);
      // duplicates inside this slice: apply them one by one
      for (int j = 0; j < 64; j++) {
        const int pj = __shfl(pos, j);
        const bool dj = __shfl((int)dup_before, j) != 0;
        if (dj && pj >= 0 && lane == 0) track_missed(x.trk[w.lst[pj]]);
        __syncthreads();
      }
      __syncthreads();
    }
  }
  SSTAMP(7);

  // ---- _attempt_id_recovery (tracker.py:300-344) ----------------------------------------------
  if (x.nlost && naud) {
    for (int li = 0; li < x.nlost; li++) {
      const int ls = x.lost[li];
      if (x.trk[ls].nfeat == 0) continue;
      const double* rs = g.recsim + ((size_t)seq * LOSTN + li) * g.D;
      double best = -INF;
      int bk = 0x7fffffff;
      for (int k = lane; k < naud; k += 64) {
        const double sv = rs[x.det_in(w.aud[k])];
        if (sv > best || (sv == best && k < bk)) best = sv, bk = k;
      }
      for (int o = 32; o >= 1; o >>= 1) {
        const double ob = __shfl_xor(best, o);
        const int ok = __shfl_xor(bk, o);
        if (ob > best || (ob == best && ok < bk)) best = ob, bk = ok;
      }
      if (best > 0.7) {
        const int di = w.aud[bk];
        if (lane == 0) {
          x.trk[ls].state = 1;  // the reference's "Confirmed state" comment sets Tentative (1)
          x.trk[ls].tsu = 0;
        }
        __syncthreads();
        track_update(x, ls, di);
        if (lane == 0) {
          w.lst[x.ntr] = ls;
          for (int k = li; k < x.nlost - 1; k++) x.lost[k] = x.lost[k + 1];
          for (int k = bk; k < naud - 1; k++) w.aud[k] = w.aud[k + 1];
        }
        x.ntr++;
        x.nlost--;
        naud--;
        __syncthreads();
        break;
      }
    }
  }

  SSTAMP(8);
  // ---- births (_initiate_track), free slots ascending ----------------------------------------
  if (naud) {
    for (int s2 = lane; s2 < g.T; s2 += 64) w.flag[s2] = 0;
    __syncthreads();
    for (int p = lane; p < x.ntr; p += 64) w.flag[w.lst[p]] = 1;
    for (int k = lane; k < x.nlost; k += 64) w.flag[x.lost[k]] = 1;
    __syncthreads();
    const int nfree = wave_compact(g.T, [&](int s2) { return w.flag[s2] == 0; },
                                   [&](int s2, int p) { w.tmp[p] = s2; });
    int nnew = naud;
    if (nnew > nfree) {
      if (lane == 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
      nnew = nfree;
    }
    const int id0 = sq[Q_NEXTID];
    for (int k = lane; k < nnew; k += 64) {
      track_birth(x, w.tmp[k], w.aud[k], id0 + k);
      w.lst[x.ntr + k] = w.tmp[k];
    }
    x.ntr += nnew;
    __syncthreads();
    if (lane == 0) sq[Q_NEXTID] = id0 + nnew;
  }

  SSTAMP(9);
  // ---- deleted tracks -> lost buffer (tracker.py:152-164) -------------------------------------
  // the surviving list by compaction; the deleted ones (few) through the lost buffer in order
  const int ndel = wave_compact(
      x.ntr, [&](int p) { return x.trk[w.lst[p]].state == 3; },
      [&](int p, int q) { w.flag[q] = w.lst[p]; });
  if (ndel) {
    const int nkeep = wave_compact(
        x.ntr, [&](int p) { return x.trk[w.lst[p]].state != 3; },
        [&](int p, int q) { w.tmp[q] = w.lst[p]; });
    for (int k = lane; k < nkeep; k += 64) w.lst[k] = w.tmp[k];
    if (lane == 0) {
      const int max_age = sq[Q_MAXAGE];
      for (int q = 0; q < ndel; q++) {
        const int s2 = w.flag[q];
        if (x.nlost < LOSTN) {
          x.trk[s2].lost_frame = fid;
          x.lost[x.nlost++] = s2;
        }
        int lw = 0;
        for (int k = 0; k < x.nlost; k++)
          if (fid - x.trk[x.lost[k]].lost_frame < max_age) x.lost[lw++] = x.lost[k];
        x.nlost = lw;
      }
      w.sc[1] = x.nlost;
    }
    __syncthreads();
    x.ntr = nkeep;
    x.nlost = w.sc[1];
  }
  __syncthreads();

  SSTAMP(10);
  // metric.partial_fit runs (ss_fit_kernel) iff a confirmed track has features (tracker.py:166-178)
  int anyf = 0;
  for (int p = lane; p < x.ntr; p += 64) {
    const SsTrk& t = x.trk[w.lst[p]];
    anyf |= t.state == 2 && t.nfeat > 0;
  }
  anyf = __any(anyf);

  // ---- outputs (strongsort.py:313-345) ---------------------------------------------------------
  double* orow = out + (size_t)r0 * 10;
  const int nout = wave_compact(
      x.ntr, [&](int p) { const SsTrk& t = x.trk[w.lst[p]]; return t.state == 2 && t.tsu < 1; },
      [&](int p, int q) {
        const SsTrk& t = x.trk[w.lst[p]];
        if (q < n) {
          double bx[4];
          to_tlbr(t, bx);
          double* o = orow + (size_t)q * 10;
          o[0] = bx[0], o[1] = bx[1], o[2] = bx[2], o[3] = bx[3];
          o[4] = (double)t.id, o[5] = t.conf, o[6] = t.cls, o[7] = t.det_ind;
          o[8] = t.quality, o[9] = 0.0;
        }
      });
  for (int p = lane; p < x.ntr; p += 64) order[p] = w.lst[p];
  if (lane == 0) {
    out_count[b] = nout < n ? nout : n;
    sq[Q_FRAME] = frame;
    sq[Q_NTR] = x.ntr;
    sq[Q_NLOST] = x.nlost;
    sq[Q_HIST] = sq[Q_HIST] < 100 ? sq[Q_HIST] + 1 : 100;
    sq[Q_NNL] = 0;  // ss_fit_kernel lists the next frame's gallery queries
    sq[Q_ANYF] = anyf;
    sq[Q_NT0] = nt0;
    sq[Q_NOUT] = nout;
  }
  SSTAMP(12);
}

// metric.partial_fit (linear_assignment.py:539-593) for one track of the list or the lost buffer
// (wave per track), then its pool bookkeeping and the next frame's query list.
//
// The gallery is kept as a multiset of (pool vector, quality, insertion time): the reference
// appends, and whenever a list grows past the budget stable-sorts it by quality descending and
// truncates.  Inductively its list is ordered by (quality desc, insertion time asc) from its first
// sort on, and a stable sort of appended entries keeps that order, so appending k features one by
// one with a truncation after each equals appending all k and keeping the `budget` best under
// (quality desc, time asc) — what this kernel does.  The stored gallery is kept in that order,
// so the new entries merge in by rank (O(n·k) comparisons in LDS, not a full re-rank).
constexpr int GB_MAX = 320;
__global__ void __launch_bounds__(64) ss_fit_kernel(SsDev g, int seq0) {
  __shared__ double q_s[GB_MAX];
  __shared__ int t_s[GB_MAX], v_s[GB_MAX];
  const int b = blockIdx.y, seq = seq0 + b, k = blockIdx.x, lane = threadIdx.x;
  int* sq = g.sq + (size_t)seq * SQS;
  const int ntr = sq[Q_NTR], nlost = sq[Q_NLOST];
  if (k >= ntr + nlost) return;
  const int slot = k < ntr ? g.order[(size_t)seq * g.T + k] : g.lost[(size_t)seq * LOSTN + k - ntr];
  SsTrk& t = g.trk[(size_t)seq * g.T + slot];
  const int F = g.F;
  const int bdk = t.born_dk;
  if (bdk >= 0) {  // a track born this frame: its first feature vector
    const double* nf = g.nf + ((size_t)seq * g.D + bdk) * F;
    double* dst = vecp(g, seq, slot, 0);
    double* dstn = vecnp(g, seq, slot, 0);
    const double pn = g.dprep[((size_t)seq * g.D + bdk) * 4 + 3];
    for (int q = lane; q < F; q += 64) {
      dst[q] = nf[q];
      dstn[nn_pos(q, F)] = nf[q] / pn;
    }
  }
  int* gv = g.gal_v + ((size_t)seq * g.T + slot) * g.GB;
  double* gq = g.gal_q + ((size_t)seq * g.T + slot) * g.GB;
  int* gt = g.gal_t + ((size_t)seq * g.T + slot) * g.GB;
  int n = t.gal_n;
  if (sq[Q_ANYF]) {
    const int budget = sq[Q_BUDGET];
    const int keep = budget / 4 < 5 ? budget / 4 : 5;
    if (k < ntr && t.state == 2) {  // active target: its features appended in list order
      // The stored gallery is sorted by (quality desc, time asc) — every update below keeps it
      // so — and the appended features are newer than all of it: an old entry's rank is its
      // index plus the new entries of higher quality, a new entry's the old entries of at least
      // its quality (binary search) plus the new ones ahead of it.  Entries ranked below the
      // budget land at their rank; old ones already there are not rewritten.
      const int nfe = t.nfeat, c0 = t.gal_clock, n0 = n, nt = n0 + nfe;
      for (int i = lane; i < n0; i += 64) {
        q_s[i] = gq[i];
        t_s[i] = gt[i];
        v_s[i] = gv[i];
      }
      for (int q = lane; q < nfe; q += 64) {
        const int v = t.feat[q];
        q_s[n0 + q] = g.vwn[vidx(g, seq, slot, v)];
        t_s[n0 + q] = c0 + q;
        v_s[n0 + q] = v;
      }
      __syncthreads();
      const int lim = (budget > 0 && nt > budget) ? budget : nt;
      for (int i = lane; i < nt; i += 64) {
        const double qi = q_s[i];
        int r;
        if (i < n0) {
          r = i;
          for (int j = n0; j < nt; j++) r += q_s[j] > qi;
        } else {
          int lo = 0, hi = n0;  // first old entry of lower quality
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (q_s[mid] >= qi) lo = mid + 1;
            else hi = mid;
          }
          r = lo;
          for (int j = n0; j < i; j++) r += q_s[j] >= qi;
          for (int j = i + 1; j < nt; j++) r += q_s[j] > qi;
        }
        if (r < lim && (i >= n0 || r != i)) {
          gv[r] = v_s[i];
          gq[r] = qi;
          gt[r] = t_s[i];
        }
      }
      n = lim;
      if (lane == 0) t.gal_clock = c0 + nfe;
    } else if (n > keep) {  // inactive target: trimmed to its min(budget // 4, 5) best
      n = keep;
    }
    __syncthreads();
    if (lane == 0) t.gal_n = n;
  }
  __syncthreads();
  // pool entries referenced by the gallery, then by the features list too
  unsigned long long m = 0ull;
  for (int i = lane; i < n; i += 64) m |= 1ull << gv[i];
  for (int o = 32; o >= 1; o >>= 1) m |= __shfl_xor(m, o);
  if (lane == 0) {
    t.gmask = m;
    for (int q = 0; q < t.nfeat; q++) m |= 1ull << t.feat[q];
    t.vmask = m;
    t.born_dk = -1;
    if (k < ntr && t.state == 2 && n > 0) g.nnl[(size_t)seq * g.T + atomicAdd(sq + Q_NNL, 1)] = slot;
  }
}

__global__ void ss_reset_kernel(SsDev g, int seq0, int nseq) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nseq) {
    int* q = g.sq + (size_t)(seq0 + k) * SQS;
    for (int i = 0; i < SQS; i++) q[i] = 0;
    q[Q_NEXTID] = 1;
    q[Q_MAXAGE] = g.sq[(size_t)g.S * SQS + 0];
    q[Q_BUDGET] = g.sq[(size_t)g.S * SQS + 1];
    g.sqd[(size_t)(seq0 + k) * 2] = g.sqd[(size_t)g.S * 2];
    g.sqd[(size_t)(seq0 + k) * 2 + 1] = g.sqd[(size_t)g.S * 2];
  }
}

// OcclusionAwareTracker._handle_emerging_track's `track.features[-1] = blended`
// (utils/occlusion_handler.py:405-413) for the host post-process: one wave per edited track.
// The vector replaces features[-1]; a pool entry the gallery also references keeps its old
// content (the reference's gallery holds copies) and the feature moves to a fresh entry.  The
// blend is normalised here when asked (`/= np.linalg.norm + 1e-8`, the engine's wave order) and
// the entry gets the norms every stored feature carries (wave norm, numpy pairwise + 1e-8, the
// NN-normalised copy).
__global__ void __launch_bounds__(64) ss_feat_set_kernel(SsDev g, int seq, const int* __restrict__ slots,
                                                         const double* __restrict__ src,
                                                         int normalize) {
  __shared__ int lo[PW_MAXLEAF], ln[PW_MAXLEAF];
  __shared__ double leaf[PW_MAXLEAF];
  __shared__ int sv;
  const int lane = threadIdx.x, F = g.F, slot = slots[blockIdx.x];
  SsTrk& t = g.trk[(size_t)seq * g.T + slot];
  const double* x = src + (size_t)blockIdx.x * F;
  if (lane == 0) {
    int v = -1;
    if (t.nfeat > 0) {
      const int lv = t.feat[t.nfeat - 1];
      v = ((t.gmask >> lv) & 1ull) ? pool_alloc(t, g.VP) : lv;
      if (v < 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
    }
    sv = v;
  }
  __syncthreads();
  const int v = sv;
  if (v < 0) return;
  double* dst = vecp(g, seq, slot, v);
  const double ns = normalize ? sqrt(wdot(x, x, F)) + 1e-8 : 1.0;
  for (int q = lane; q < F; q += 64) dst[q] = normalize ? x[q] / ns : x[q];
  __syncthreads();
  const double wn = sqrt(wdot(dst, dst, F));
  const double pn = wpw_norm(dst, F, lo, ln, leaf) + 1e-8;
  double* dstn = vecnp(g, seq, slot, v);
  for (int q = lane; q < F; q += 64) dstn[nn_pos(q, F)] = dst[q] / pn;
  if (lane == 0) {
    const size_t vi = vidx(g, seq, slot, v);
    g.vwn[vi] = wn;
    g.vden[vi] = pn;
    t.feat[t.nfeat - 1] = v;
  }
}

// Test entry point of the match kernel's LSAP (lsap_wave) on a dense row-major R x CC matrix,
// R <= CC <= 1024, one wave: mode 0 scipy's row order, 1 solve + certify (a tie answered -1).
__global__ void __launch_bounds__(64) ss_lsap_op_kernel(const double* C, int R, int CC,
                                                        double max_d, int fast, int32_t* rows,
                                                        int32_t* cols, int32_t* info,
                                                        int* status) {
  extern __shared__ __align__(16) char ss_lds[];
  const int N = CC;
  SsDev g{};
  g.T = R;
  g.D = CC;
  g.N = N;
  g.status = status;
  SsWs w{};
  double* ld = (double*)ss_lds;
  int* li = (int*)(ss_lds + (size_t)3 * N * 8);
  w.u = ld; w.v = ld + N; w.spc = ld + 2 * N;
  w.path = li; w.col4row = li + N; w.row4col = li + 2 * N; w.rem = li + 3 * N;
  w.pos = li + 4 * N; w.SR = li + 5 * N; w.SC = li + 6 * N;
  w.rows = li + 7 * N; w.cols = li + 8 * N;
  int* roff = li + 9 * N;
  int* cidx = li + 10 * N;
  const int lane = threadIdx.x;
  for (int r = lane; r < R; r += 64) roff[r] = r * CC;
  for (int j = lane; j < CC; j += 64) cidx[j] = j;
  __syncthreads();
  SsCtx x{g, w, 0, lane, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 0};
  int fs = 0;
  const bool f = fast != 0;
  const int np = CC <= 256   ? lsap_wave<4, true>(x, C, roff, cidx, max_d, R, CC, false, f, fs)
                 : CC <= 512 ? lsap_wave<8, true>(x, C, roff, cidx, max_d, R, CC, false, f, fs)
                             : lsap_wave<16, true>(x, C, roff, cidx, max_d, R, CC, false, f, fs);
  for (int q = lane; q < np; q += 64) rows[q] = w.rows[q], cols[q] = w.cols[q];
  if (lane == 0) info[0] = np, info[1] = fs;
}

}  // namespace

struct bx_ss {
  SsDev dev;
  bx_ss_config cfg;
  void* arena = nullptr;
  double* h_dets = nullptr;
  int* h_off = nullptr;
  double* h_embs = nullptr;
  double* h_warp = nullptr;
  double* h_out = nullptr;
  int* h_cnt = nullptr;
  // pinned mirrors for update_host (asynchronous copies, one sync per frame) and the counters
  // row of the last update_host sequence (bx_ss_counters_host answers from it)
  double* p_dets = nullptr;
  double* p_embs = nullptr;
  double* p_warp = nullptr;
  double* p_out = nullptr;
  int* p_cnt = nullptr;
  int* p_sq = nullptr;
  int cache_seq = -1;
  int probe_stage = -1;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  int ev_used = 0;
  // crowd test + ss_pre_kernel run on `side` beside ss_nn_kernel / ss_rec_kernel (neither reads
  // what the other writes); fork after ss_prep_kernel, join before ss_cost_kernel
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

#define SCHK(x)                                                                    \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess)                                                          \
      return bx_record_error(BX_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

static int ss_probe_begin(bx_ss* e, int stage, hipStream_t st) {
  if (e->probe_stage != stage) return BX_OK;
  if (e->ev_used == (int)e->ev.size()) {
    hipEvent_t a, b;
    SCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
    SCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    e->ev.push_back({a, b});
  }
  SCHK(hipEventRecord(e->ev[e->ev_used].first, st));
  return BX_OK;
}
static int ss_probe_end(bx_ss* e, int stage, hipStream_t st) {
  if (e->probe_stage != stage) return BX_OK;
  SCHK(hipEventRecord(e->ev[e->ev_used++].second, st));
  return BX_OK;
}

static size_t ss_lds_bytes(const SsDev& d) {
  return d.ws_lds == 1 ? (size_t)d.wsd_n * 8 + (size_t)d.wsi_n * 4 : (size_t)ws_lsap_bytes(d.N);
}

static int ss_launch(bx_ss* e, int seq0, int nseq, const double* dets, const int* off,
                     const double* embs, const double* warps, double* out, int* cnt,
                     hipStream_t st) {
  const SsDev& d = e->dev;
  int rc;
  if (!embs) return bx_record_error(BX_ERR_SHAPE, "StrongSort needs embeddings");
  if ((rc = ss_probe_begin(e, 0, st))) return rc;
  hipLaunchKernelGGL(ss_prep_kernel, dim3(d.D + 1, nseq), dim3(64), 0, st, d, seq0, off, embs,
                     dets);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 0, st))) return rc;
  // fork: ss_pre_kernel (crowd mode, quality + sort, cascade keys; one wave per sequence) on the
  // side stream beside the gallery distance
  const size_t lds = ss_lds_bytes(d);
  // The crowd test and the camera update + predict are short grids.  With few sequences they go
  // on the main stream before the gallery distance: queued beside its waves they wait for their
  // slots and become the critical path (C4: 1 sequence).  With many sequences they overlap it on
  // the side stream (measured: 256 sequences 0.654 -> 0.612 ms per step, C4 the reverse).
  const bool side_all = nseq >= 8;
  hipStream_t sm = side_all ? e->side : st;
  if (side_all) {
    SCHK(hipEventRecord(e->ev_fork, st));
    SCHK(hipStreamWaitEvent(e->side, e->ev_fork, 0));
  }
  if ((rc = ss_probe_begin(e, 3, sm))) return rc;
  if (d.crowd)
    hipLaunchKernelGGL(ss_crowd_kernel, dim3(crowd_blocks(nseq), nseq), dim3(256),
                       sizeof(double) * 4 * d.T, sm, d, seq0);
  hipLaunchKernelGGL(ss_motion_kernel, dim3(d.T, nseq), dim3(64), 0, sm, d, seq0, warps);
  SCHK(hipGetLastError());
  if (!side_all) {
    if ((rc = ss_probe_end(e, 3, st))) return rc;
    SCHK(hipEventRecord(e->ev_fork, st));
    SCHK(hipStreamWaitEvent(e->side, e->ev_fork, 0));
    if ((rc = ss_probe_begin(e, 3, e->side))) return rc;
  }
  hipLaunchKernelGGL(ss_pre_kernel, dim3(nseq), dim3(64), lds, e->side, d, seq0, dets, off,
                     warps);
  SCHK(hipGetLastError());
  hipLaunchKernelGGL(ss_sort_kernel, dim3((d.D + 255) / 256, nseq), dim3(256), 0, e->side, d,
                     seq0);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 3, e->side))) return rc;
  SCHK(hipEventRecord(e->ev_join, e->side));
  if ((rc = ss_probe_begin(e, 1, st))) return rc;
  // a fixed set of waves per sequence pulls (pack, 16 NDT-detection block) items off the
  // sequence's counter (ss_nn_kernel): ~BX_SS_NN_WAVES in all (two per SIMD), at least one per
  // sequence and no more than its largest item count (packs <= listed tracks)
  // detection tiles per item: 4 when the detection capacity is large (C4: 578 us per launch vs
  // 711 with 2 and 1024 waves 661 — profiles/r06/ab_ss_nn_work_counter.txt), 2 otherwise (the
  // 256-sequence config, ~24 detections: 417 k vs 412 k frames/s)
#ifndef BX_SS_NDT
#define BX_SS_NDT 4
#endif
#ifndef BX_SS_NN_WAVES
#define BX_SS_NN_WAVES 2048
#endif
  const int ndt = d.D >= 256 ? BX_SS_NDT : 2;
  const long items_max = (long)d.T * ((d.D + 16 * ndt - 1) / (16 * ndt));
  long gw = (BX_SS_NN_WAVES + nseq - 1) / nseq;
  gw = gw < 1 ? 1 : (gw > items_max ? items_max : gw);
  if (gw >= 64) gw = (gw + 7) / 8 * 8;  // (the kernel's XCD split needs a multiple of 8)
  const int gx = (int)gw;
  if (ndt == 4)
    hipLaunchKernelGGL((ss_nn_kernel<4>), dim3(gx, nseq, 1), dim3(64), 0, st, d, seq0, off);
  else if (ndt == 3)
    hipLaunchKernelGGL((ss_nn_kernel<3>), dim3(gx, nseq, 1), dim3(64), 0, st, d, seq0, off);
  else if (ndt == 2)
    hipLaunchKernelGGL((ss_nn_kernel<2>), dim3(gx, nseq, 1), dim3(64), 0, st, d, seq0, off);
  else
    hipLaunchKernelGGL((ss_nn_kernel<1>), dim3(gx, nseq, 1), dim3(64), 0, st, d, seq0, off);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 1, st))) return rc;
  if ((rc = ss_probe_begin(e, 2, st))) return rc;
  hipLaunchKernelGGL(ss_rec_kernel, dim3(LOSTN, nseq), dim3(256), 0, st, d, seq0, off, embs);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 2, st))) return rc;
  SCHK(hipStreamWaitEvent(st, e->ev_join, 0));  // join
  if ((rc = ss_probe_begin(e, 4, st))) return rc;
  hipLaunchKernelGGL(ss_cost_kernel, dim3(d.T, nseq), dim3(64), 0, st, d, seq0);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 4, st))) return rc;
  if ((rc = ss_probe_begin(e, 5, st))) return rc;
  hipLaunchKernelGGL(ss_match_kernel, dim3(nseq), dim3(128), lds, st, d, seq0);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 5, st))) return rc;
  if ((rc = ss_probe_begin(e, 6, st))) return rc;
  hipLaunchKernelGGL(ss_update_kernel,
                     dim3(((d.T < d.D ? d.T : d.D) + SS_UPD_W - 1) / SS_UPD_W, nseq),
                     dim3(64 * SS_UPD_W), 0, st, d, seq0);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 6, st))) return rc;
  if ((rc = ss_probe_begin(e, 7, st))) return rc;
  hipLaunchKernelGGL(ss_post_kernel, dim3(nseq), dim3(64), lds, st, d, seq0, off, out, cnt);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 7, st))) return rc;
  if ((rc = ss_probe_begin(e, 8, st))) return rc;
  hipLaunchKernelGGL(ss_fit_kernel, dim3(d.T + LOSTN, nseq), dim3(64), 0, st, d, seq0);
  SCHK(hipGetLastError());
  if ((rc = ss_probe_end(e, 8, st))) return rc;
  return BX_OK;
}

extern "C" {

int bx_ss_create(const bx_ss_config* c, bx_ss** out) {
  if (!c || !out) return bx_record_error(BX_ERR_INVALID, "null argument");
  const int vp = c->vec_cap > 0 ? c->vec_cap : 32;
  if (c->n_seq <= 0 || c->track_cap <= 0 || c->det_cap <= 0 || c->track_cap > 1024 ||
      c->det_cap > 1024 || c->emb_dim <= 0 || c->emb_dim > 8192 || vp > 64 || c->nn_budget <= 0 ||
      c->max_age < 0)
    return bx_record_error(BX_ERR_INVALID, "bx_ss_config out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return bx_record_error(BX_ERR_NO_DEVICE, "no HIP device visible");
  bx_ss* e = new bx_ss();
  e->cfg = *c;
  SsDev& d = e->dev;
  d.S = c->n_seq;
  d.T = c->track_cap;
  d.D = c->det_cap;
  d.F = c->emb_dim;
  d.VP = vp;
  const int crowd_budget = c->nn_budget * 2 < 300 ? c->nn_budget * 2 : 300;
  // partial_fit appends a track's <= MAXF features before truncating to the budget
  d.GB = (c->nn_budget > crowd_budget ? c->nn_budget : crowd_budget) + MAXF;
  if (d.GB > GB_MAX) {
    delete e;
    return bx_record_error(BX_ERR_INVALID, "nn_budget too large (gallery > 320 entries)");
  }
  d.N = 2 * d.T > d.D ? 2 * d.T : d.D;
  d.min_conf = c->min_conf;
  d.max_iou = c->max_iou_dist;
  d.mc_lambda = c->mc_lambda;
  d.ema_alpha = c->ema_alpha;
  d.thi = c->conf_thresh_high;
  d.tlo = c->conf_thresh_low;
  d.idw = c->id_preservation_weight;
  d.n_init = c->n_init;
  d.crowd = c->crowd_detection != 0;
  d.born = c->born_confirmed != 0;
  d.wsi_n = ws_ints(d.T, d.D, d.N);
  d.wsd_n = ws_doubles(d.T, d.D, d.N);
  // the frame kernel's workspace in LDS when it fits beside ~3 other workgroups per CU
  const size_t ws_bytes = (size_t)d.wsd_n * 8 + (size_t)d.wsi_n * 4;
  // all of it in LDS when it fits beside ~3 other workgroups per CU; else the LSAP state alone
  // (the solver's inner loops; track_cap, det_cap <= 1024 keep it within 106 KB)
  d.ws_lds = ws_bytes <= 48 * 1024 ? 1 : 2;
  d.lsap_fast = 1;
  const size_t S = d.S, T = d.T, D = d.D, F = d.F, VP = d.VP, GB = d.GB;
  size_t off = 0;
  auto cb = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_trk = cb(S * T * sizeof(SsTrk));
  const size_t o_gv = cb(S * T * GB * sizeof(int));
  const size_t o_gq = cb(S * T * GB * sizeof(double));
  const size_t o_gt = cb(S * T * GB * sizeof(int));
  const size_t o_vec = cb(S * T * VP * F * sizeof(double));
  const size_t o_vecn = cb(S * T * VP * F * sizeof(double));
  const size_t o_vden = cb(S * T * VP * sizeof(double));
  const size_t o_vwn = cb(S * T * VP * sizeof(double));
  const size_t o_sq = cb((S + 1) * SQS * sizeof(int));
  const size_t o_sqd = cb((S + 1) * 2 * sizeof(double));
  const size_t o_ord = cb(S * T * sizeof(int));
  const size_t o_lost = cb(S * LOSTN * sizeof(int));
  const size_t o_nnl = cb(S * T * sizeof(int));
  const size_t o_pk = cb(S * (T + 3) * sizeof(int));
  const size_t o_nnd = cb(S * T * D * sizeof(double));
  const size_t o_prep = cb(S * D * 4 * sizeof(double));
  const size_t o_dn = cb(S * D * F * sizeof(double));
  const size_t o_nf = cb(S * D * F * sizeof(double));
  const size_t o_rec = cb(S * LOSTN * D * sizeof(double));
  const size_t o_cost = cb(S * 4 * T * D * sizeof(double));
  const size_t o_cfull = cb(S * T * D * sizeof(double));
  const size_t o_cfullT = cb(S * T * D * sizeof(double));
  const size_t o_tlist = cb(S * T * SS_TL * sizeof(int16_t));
  const size_t o_tcnt = cb(S * T * sizeof(int));
  const size_t o_crank = cb(S * T * sizeof(int));
  const size_t o_ckey = cb(S * T * sizeof(double));
  const size_t o_ctsu = cb(S * T * sizeof(int));
  const size_t o_cpos = cb(S * T * sizeof(int));
  const size_t o_ncf = cb(S * sizeof(int));
  const size_t o_fdt = cb(S * D * DTW * sizeof(double));
  const size_t o_fdord = cb(S * D * sizeof(int));
  const size_t o_faud = cb(S * D * sizeof(int));
  const size_t o_fmt = cb(S * 4 * (D + 2) * sizeof(int));
  const size_t o_ffut = cb(S * 3 * T * sizeof(int));
  const size_t o_wsi = cb(S * (size_t)d.wsi_n * sizeof(int));
  const size_t o_wsd = cb(S * (size_t)d.wsd_n * sizeof(double));
  const size_t o_st = cb(sizeof(int) * 4);
#ifdef BX_PHASE_TIMING
  const size_t o_dbg = cb(S * SS_DBG * sizeof(unsigned long long));
#endif
  if (hipMalloc(&e->arena, off) != hipSuccess) {
    delete e;
    return bx_record_error(BX_ERR_HIP, "hipMalloc of the StrongSort arena failed");
  }
  SCHK(hipMemset(e->arena, 0, off));
  char* base = (char*)e->arena;
  d.trk = (SsTrk*)(base + o_trk);
  d.gal_v = (int*)(base + o_gv);
  d.gal_q = (double*)(base + o_gq);
  d.gal_t = (int*)(base + o_gt);
  d.vec = (double*)(base + o_vec);
  d.vecn = (double*)(base + o_vecn);
  d.vden = (double*)(base + o_vden);
  d.vwn = (double*)(base + o_vwn);
  d.sq = (int*)(base + o_sq);
  d.sqd = (double*)(base + o_sqd);
  d.order = (int*)(base + o_ord);
  d.lost = (int*)(base + o_lost);
  d.nnl = (int*)(base + o_nnl);
  d.pk = (int*)(base + o_pk);
  d.nnd = (double*)(base + o_nnd);
  d.dprep = (double*)(base + o_prep);
  d.dn = (double*)(base + o_dn);
  d.nf = (double*)(base + o_nf);
  d.recsim = (double*)(base + o_rec);
  d.cost = (double*)(base + o_cost);
  d.cfull = (double*)(base + o_cfull);
  d.cfullT = (double*)(base + o_cfullT);
  d.tlist = (int16_t*)(base + o_tlist);
  d.tcnt = (int*)(base + o_tcnt);
  d.crank = (int*)(base + o_crank);
  d.ckey = (double*)(base + o_ckey);
  d.ctsu = (int*)(base + o_ctsu);
  d.cpos = (int*)(base + o_cpos);
  d.ncf = (int*)(base + o_ncf);
  d.fdt = (double*)(base + o_fdt);
  d.fdord = (int*)(base + o_fdord);
  d.faud = (int*)(base + o_faud);
  d.fmt = (int*)(base + o_fmt);
  d.ffut = (int*)(base + o_ffut);
  d.wsi = (int*)(base + o_wsi);
  d.wsd = (double*)(base + o_wsd);
  d.status = (int*)(base + o_st);
#ifdef BX_PHASE_TIMING
  d.dbg = (unsigned long long*)(base + o_dbg);
#else
  d.dbg = nullptr;
#endif
  // per-sequence defaults (row S holds them for bx_ss_reset): max_age, budget, threshold
  std::vector<int> q((S + 1) * SQS, 0);
  std::vector<double> qd((S + 1) * 2, c->max_cos_dist);
  for (size_t k = 0; k < S; k++) {
    q[k * SQS + Q_NEXTID] = 1;
    q[k * SQS + Q_MAXAGE] = c->max_age;
    q[k * SQS + Q_BUDGET] = c->nn_budget;
  }
  q[S * SQS + 0] = c->max_age;
  q[S * SQS + 1] = c->nn_budget;
  SCHK(hipMemcpy(d.sq, q.data(), q.size() * sizeof(int), hipMemcpyHostToDevice));
  SCHK(hipMemcpy(d.sqd, qd.data(), qd.size() * sizeof(double), hipMemcpyHostToDevice));
  if (d.ws_lds) {
    const int lds = (int)ss_lds_bytes(d);
    SCHK(bx_lds_attr((const void*)ss_pre_kernel, lds));
    SCHK(bx_lds_attr((const void*)ss_match_kernel, lds));
    SCHK(bx_lds_attr((const void*)ss_post_kernel, lds));
  }
  SCHK(hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
  SCHK(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
  SCHK(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
  SCHK(hipMalloc(&e->h_dets, sizeof(double) * 6 * D));
  SCHK(hipMalloc(&e->h_off, sizeof(int) * 2));
  SCHK(hipMalloc(&e->h_embs, sizeof(double) * D * F));
  SCHK(hipMalloc(&e->h_warp, sizeof(double) * 6));
  SCHK(hipMalloc(&e->h_out, sizeof(double) * 10 * D));
  SCHK(hipMalloc(&e->h_cnt, sizeof(int)));
  SCHK(hipHostMalloc(&e->p_dets, sizeof(double) * 6 * d.D));
  SCHK(hipHostMalloc(&e->p_embs, sizeof(double) * (size_t)d.D * d.F));
  SCHK(hipHostMalloc(&e->p_warp, sizeof(double) * 8));
  SCHK(hipHostMalloc(&e->p_out, sizeof(double) * 10 * d.D));
  SCHK(hipHostMalloc(&e->p_cnt, sizeof(int) * 4));
  SCHK(hipHostMalloc(&e->p_sq, sizeof(int) * SQS));
  *out = e;
  return BX_OK;
}

int bx_ss_copy_state(bx_ss* dst, bx_ss* src) {
  if (!dst || !src) return bx_record_error(BX_ERR_INVALID, "null engine");
  const SsDev &a = src->dev, &b = dst->dev;
  if (a.S != b.S || a.F != b.F || a.VP != b.VP || a.GB != b.GB || b.T < a.T || b.D < a.D)
    return bx_record_error(BX_ERR_INVALID, "bx_ss_copy_state: destination must match the "
                                           "source's sequences, features, vector pool and budget "
                                           "and have at least its capacities");
  SCHK(hipDeviceSynchronize());
  const size_t S = a.S, Ta = a.T, Tb = b.T, F = a.F, VP = a.VP, GB = a.GB;
  auto rows = [&](void* d, const void* s_, size_t per_slot) -> hipError_t {
    return hipMemcpy2D(d, Tb * per_slot, s_, Ta * per_slot, Ta * per_slot, S,
                       hipMemcpyDeviceToDevice);
  };
  // per-slot state: track records, galleries (entries, qualities, times), the vector pools and
  // their norms, the list order and the next frame's query list
  SCHK(rows(b.trk, a.trk, sizeof(SsTrk)));
  SCHK(rows(b.gal_v, a.gal_v, GB * sizeof(int)));
  SCHK(rows(b.gal_q, a.gal_q, GB * sizeof(double)));
  SCHK(rows(b.gal_t, a.gal_t, GB * sizeof(int)));
  SCHK(rows(b.vec, a.vec, VP * F * sizeof(double)));
  SCHK(rows(b.vecn, a.vecn, VP * F * sizeof(double)));
  SCHK(rows(b.vden, a.vden, VP * sizeof(double)));
  SCHK(rows(b.vwn, a.vwn, VP * sizeof(double)));
  SCHK(rows(b.order, a.order, sizeof(int)));
  SCHK(rows(b.nnl, a.nnl, sizeof(int)));
  // per-sequence scalars (+ the defaults row S), the lost buffer (slot ids), status
  SCHK(hipMemcpy(b.sq, a.sq, (S + 1) * SQS * sizeof(int), hipMemcpyDeviceToDevice));
  SCHK(hipMemcpy(b.sqd, a.sqd, (S + 1) * 2 * sizeof(double), hipMemcpyDeviceToDevice));
  SCHK(hipMemcpy(b.lost, a.lost, S * LOSTN * sizeof(int), hipMemcpyDeviceToDevice));
  SCHK(hipMemcpy(b.status, a.status, 4 * sizeof(int), hipMemcpyDeviceToDevice));
  dst->cache_seq = -1;
  SCHK(hipDeviceSynchronize());
  return BX_OK;
}

int bx_ss_destroy(bx_ss* e) {
  if (!e) return BX_OK;
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  for (auto& p : e->ev) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  (void)hipFree(e->arena);
  (void)hipFree(e->h_dets);
  (void)hipFree(e->h_off);
  (void)hipFree(e->h_embs);
  (void)hipFree(e->h_warp);
  (void)hipFree(e->h_out);
  (void)hipFree(e->h_cnt);
  (void)hipHostFree(e->p_dets);
  (void)hipHostFree(e->p_embs);
  (void)hipHostFree(e->p_warp);
  (void)hipHostFree(e->p_out);
  (void)hipHostFree(e->p_cnt);
  (void)hipHostFree(e->p_sq);
  delete e;
  return BX_OK;
}

int bx_ss_reset(bx_ss* e, int seq0, int nseq, void* stream) {
  if (!e || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad sequence range");
  if (!nseq) return BX_OK;
  e->cache_seq = -1;
  hipLaunchKernelGGL(ss_reset_kernel, dim3((nseq + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     e->dev, seq0, nseq);
  SCHK(hipGetLastError());
  return BX_OK;
}

int bx_ss_step(bx_ss* e, int seq0, int nseq, const double* dets, const int32_t* det_off,
               const double* embs, const double* warps, double* out, int32_t* out_count,
               void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_step");
  e->cache_seq = -1;
  return ss_launch(e, seq0, nseq, dets, det_off, embs, warps, out, out_count, (hipStream_t)stream);
}

int bx_ss_update_host(bx_ss* e, int seq, const double* dets, int n, const double* embs,
                      const double* warp, double* out, int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!dets || !out || !embs)) || !n_out)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_update_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  hipStream_t st = (hipStream_t)stream;
  // pinned mirrors: asynchronous copies in, the frame, rows (at most n) + count + status +
  // counters back, one synchronisation
  if (n) {
    memcpy(e->p_dets, dets, sizeof(double) * 6 * n);
    memcpy(e->p_embs, embs, sizeof(double) * (size_t)n * e->dev.F);
    SCHK(hipMemcpyAsync(e->h_dets, e->p_dets, sizeof(double) * 6 * n, hipMemcpyHostToDevice, st));
    SCHK(hipMemcpyAsync(e->h_embs, e->p_embs, sizeof(double) * (size_t)n * e->dev.F,
                        hipMemcpyHostToDevice, st));
  }
  if (warp) {
    memcpy(e->p_warp, warp, sizeof(double) * 6);
    SCHK(hipMemcpyAsync(e->h_warp, e->p_warp, sizeof(double) * 6, hipMemcpyHostToDevice, st));
  }
  e->p_cnt[2] = 0;
  e->p_cnt[3] = n;
  SCHK(hipMemcpyAsync(e->h_off, e->p_cnt + 2, sizeof(int) * 2, hipMemcpyHostToDevice, st));
  e->cache_seq = -1;
  int rc = ss_launch(e, seq, 1, e->h_dets, e->h_off, e->h_embs, warp ? e->h_warp : nullptr,
                     e->h_out, e->h_cnt, st);
  if (rc) return rc;
  SCHK(hipMemcpyAsync(e->p_cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  SCHK(hipMemcpyAsync(e->p_cnt + 1, e->dev.status, sizeof(int), hipMemcpyDeviceToHost, st));
  if (n) SCHK(hipMemcpyAsync(e->p_out, e->h_out, sizeof(double) * 10 * n, hipMemcpyDeviceToHost, st));
  SCHK(hipMemcpyAsync(e->p_sq, e->dev.sq + (size_t)seq * SQS, sizeof(int) * SQS,
                      hipMemcpyDeviceToHost, st));
  SCHK(hipStreamSynchronize(st));
  const int cnt = e->p_cnt[0], status = e->p_cnt[1];
  e->cache_seq = seq;
  if (cnt) memcpy(out, e->p_out, sizeof(double) * 10 * cnt);
  *n_out = cnt;
  if (status) return bx_record_error(status, "StrongSort engine status latched (see bx_ss_status)");
  return BX_OK;
}

int bx_ss_status(bx_ss* e, int* status) {
  if (!e || !status) return bx_record_error(BX_ERR_INVALID, "null argument");
  SCHK(hipMemcpy(status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  return BX_OK;
}

int bx_ss_counters_host(bx_ss* e, int seq, int* frame_count, int* next_id, int* n_tracks,
                        int* n_lost) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  int s[SQS];
  if (seq == e->cache_seq) {
    memcpy(s, e->p_sq, sizeof(s));
  } else {
    SCHK(hipDeviceSynchronize());
    SCHK(hipMemcpy(s, e->dev.sq + (size_t)seq * SQS, sizeof(s), hipMemcpyDeviceToHost));
  }
  if (frame_count) *frame_count = s[Q_FRAME];
  if (next_id) *next_id = s[Q_NEXTID];
  if (n_tracks) *n_tracks = s[Q_NTR];
  if (n_lost) *n_lost = s[Q_NLOST];
  return BX_OK;
}

int bx_ss_tracks_host(bx_ss* e, int seq, int cap, int32_t* ids, int32_t* state, double* mean,
                      double* cov, int* n) {
  if (!e || seq < 0 || seq >= e->dev.S || cap < 0 || !n)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_tracks_host");
  SCHK(hipDeviceSynchronize());
  int s[SQS];
  SCHK(hipMemcpy(s, e->dev.sq + (size_t)seq * SQS, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[Q_NTR];
  std::vector<int> ord(nt);
  if (nt)
    SCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int k = 0; k < nt && k < cap; k++) {
    SsTrk t;
    SCHK(hipMemcpy(&t, e->dev.trk + (size_t)seq * e->dev.T + ord[k], sizeof(SsTrk),
                   hipMemcpyDeviceToHost));
    if (ids) ids[k] = t.id;
    if (state) state[k] = t.state;
    if (mean) memcpy(mean + 8 * k, t.mean, sizeof(t.mean));
    if (cov) memcpy(cov + 64 * k, t.cov, sizeof(t.cov));
  }
  *n = nt;
  return BX_OK;
}

// the sequence's track list (slots in list order) and its track records, one copy each
static int ss_read_list(bx_ss* e, int seq, std::vector<int>& ord, std::vector<SsTrk>& trk) {
  SCHK(hipDeviceSynchronize());
  int s[SQS];
  SCHK(hipMemcpy(s, e->dev.sq + (size_t)seq * SQS, sizeof(s), hipMemcpyDeviceToHost));
  ord.assign(s[Q_NTR], 0);
  if (!ord.empty())
    SCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * ord.size(),
                   hipMemcpyDeviceToHost));
  trk.resize(e->dev.T);
  SCHK(hipMemcpy(trk.data(), e->dev.trk + (size_t)seq * e->dev.T, sizeof(SsTrk) * e->dev.T,
                 hipMemcpyDeviceToHost));
  return BX_OK;
}

static int ss_find(const std::vector<int>& ord, const std::vector<SsTrk>& trk, int id) {
  for (int k : ord)
    if (trk[k].id == id) return k;
  return -1;
}

int bx_ss_track_attrs_host(bx_ss* e, int seq, int cap, int32_t* ids, double* quality,
                           double* conf, int32_t* max_age, int32_t* n_features, int* n) {
  if (!e || seq < 0 || seq >= e->dev.S || cap < 0 || !n)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_track_attrs_host");
  std::vector<int> ord;
  std::vector<SsTrk> trk;
  if (int rc = ss_read_list(e, seq, ord, trk)) return rc;
  for (int k = 0; k < (int)ord.size() && k < cap; k++) {
    const SsTrk& t = trk[ord[k]];
    if (ids) ids[k] = t.id;
    if (quality) quality[k] = t.quality;
    if (conf) conf[k] = t.conf;
    if (max_age) max_age[k] = t.max_age;
    if (n_features) n_features[k] = t.nfeat;
  }
  *n = (int)ord.size();
  return BX_OK;
}

int bx_ss_track_attrs_set_host(bx_ss* e, int seq, int n, const int32_t* ids, const double* quality,
                               const double* conf, const int32_t* max_age) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !ids))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_track_attrs_set_host");
  std::vector<int> ord;
  std::vector<SsTrk> trk;
  if (int rc = ss_read_list(e, seq, ord, trk)) return rc;
  for (int j = 0; j < n; j++) {
    const int k = ss_find(ord, trk, ids[j]);
    if (k < 0) return bx_record_error(BX_ERR_INVALID, "track_attrs_set: no live track with that id");
    SsTrk* dt = e->dev.trk + (size_t)seq * e->dev.T + k;
    if (quality) SCHK(hipMemcpy(&dt->quality, quality + j, sizeof(double), hipMemcpyHostToDevice));
    if (conf) SCHK(hipMemcpy(&dt->conf, conf + j, sizeof(double), hipMemcpyHostToDevice));
    if (max_age) SCHK(hipMemcpy(&dt->max_age, max_age + j, sizeof(int), hipMemcpyHostToDevice));
  }
  return BX_OK;
}

int bx_ss_last_feature_host(bx_ss* e, int seq, int n, const int32_t* ids, double* feats) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!ids || !feats)))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_last_feature_host");
  std::vector<int> ord;
  std::vector<SsTrk> trk;
  if (int rc = ss_read_list(e, seq, ord, trk)) return rc;
  const int F = e->dev.F;
  for (int j = 0; j < n; j++) {
    const int k = ss_find(ord, trk, ids[j]);
    if (k < 0 || trk[k].nfeat < 1)
      return bx_record_error(BX_ERR_INVALID, "last_feature: no live track with features and that id");
    const size_t vi = ((size_t)seq * e->dev.T + k) * e->dev.VP + trk[k].feat[trk[k].nfeat - 1];
    SCHK(hipMemcpy(feats + (size_t)j * F, e->dev.vec + vi * F, sizeof(double) * F,
                   hipMemcpyDeviceToHost));
  }
  return BX_OK;
}

int bx_ss_last_feature_set_host(bx_ss* e, int seq, int n, const int32_t* ids, const double* feats,
                                int normalize) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!ids || !feats)))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_last_feature_set_host");
  if (!n) return BX_OK;
  std::vector<int> ord;
  std::vector<SsTrk> trk;
  if (int rc = ss_read_list(e, seq, ord, trk)) return rc;
  std::vector<int> slots(n);
  for (int j = 0; j < n; j++) {
    slots[j] = ss_find(ord, trk, ids[j]);
    if (slots[j] < 0 || trk[slots[j]].nfeat < 1)
      return bx_record_error(BX_ERR_INVALID, "last_feature_set: no live track with features and that id");
    for (int q = 0; q < j; q++)
      if (slots[q] == slots[j]) return bx_record_error(BX_ERR_INVALID, "last_feature_set: repeated id");
  }
  const int F = e->dev.F;
  void* buf = nullptr;
  SCHK(hipMalloc(&buf, sizeof(int) * n + sizeof(double) * (size_t)n * F + 256));
  int* d_slots = (int*)buf;
  double* d_src = (double*)((char*)buf + ((sizeof(int) * n + 255) & ~(size_t)255));
  SCHK(hipMemcpy(d_slots, slots.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  SCHK(hipMemcpy(d_src, feats, sizeof(double) * (size_t)n * F, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ss_feat_set_kernel, dim3(n), dim3(64), 0, 0, e->dev, seq, d_slots, d_src,
                     normalize);
  SCHK(hipGetLastError());
  SCHK(hipDeviceSynchronize());
  SCHK(hipFree(buf));
  int status = 0;
  SCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status) return bx_record_error(status, "a track's feature pool is exhausted (raise vec_cap)");
  return BX_OK;
}

int bx_ss_state_set_host(bx_ss* e, int seq, int n, const int32_t* ids, const double* mean,
                         const double* cov) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !ids))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_state_set_host");
  SCHK(hipDeviceSynchronize());
  int s[SQS];
  SCHK(hipMemcpy(s, e->dev.sq + (size_t)seq * SQS, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[Q_NTR];
  std::vector<int> ord(nt);
  if (nt)
    SCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int j = 0; j < n; j++) {
    SsTrk* dt = nullptr;
    SsTrk t;
    for (int k = 0; k < nt && !dt; k++) {
      SsTrk* cand = e->dev.trk + (size_t)seq * e->dev.T + ord[k];
      SCHK(hipMemcpy(&t, cand, sizeof(SsTrk), hipMemcpyDeviceToHost));
      if (t.id == ids[j]) dt = cand;
    }
    if (!dt) return bx_record_error(BX_ERR_INVALID, "state_set: no live track with that id");
    if (mean) memcpy(t.mean, mean + 8 * j, sizeof(t.mean));
    if (cov) memcpy(t.cov, cov + 64 * j, sizeof(t.cov));
    SCHK(hipMemcpy(dt, &t, sizeof(SsTrk), hipMemcpyHostToDevice));
  }
  return BX_OK;
}

int bx_ss_lsap_op(const double* cost, int R, int CC, double max_d, int fast, int32_t* rows,
                  int32_t* cols, int32_t* info, int32_t* status, void* stream) {
  if (R < 1 || R > CC || CC > 1024 || !info || !status)
    return bx_record_error(BX_ERR_INVALID, "bx_ss_lsap_op: 1 <= R <= CC <= 1024");
  const size_t lds = (size_t)3 * CC * 8 + (size_t)11 * CC * 4;
  SCHK(bx_lds_attr((const void*)ss_lsap_op_kernel, lds));
  hipLaunchKernelGGL(ss_lsap_op_kernel, dim3(1), dim3(64), lds, (hipStream_t)stream, cost, R, CC,
                     max_d, fast, rows, cols, info, status);
  SCHK(hipGetLastError());
  return BX_OK;
}

int bx_ss_set_lsap_mode(bx_ss* e, int fast) {
  if (!e || fast < 0 || fast > 1) return bx_record_error(BX_ERR_INVALID, "bad lsap mode");
  SCHK(hipDeviceSynchronize());
  e->dev.lsap_fast = fast;
  return BX_OK;
}

int bx_ss_lsap_stats_host(bx_ss* e, int seq0, int nseq, int64_t* sums) {
  if (!e || !sums || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_lsap_stats_host");
  std::vector<int> s((size_t)nseq * SQS);
  SCHK(hipDeviceSynchronize());
  if (nseq)
    SCHK(hipMemcpy(s.data(), e->dev.sq + (size_t)seq0 * SQS, sizeof(int) * s.size(),
                   hipMemcpyDeviceToHost));
  for (int k = 0; k < 5; k++) sums[k] = 0;
  for (int k = 0; k < nseq; k++) {
    const int* q = s.data() + (size_t)k * SQS;
    sums[0] += q[Q_LCALL];
    sums[1] += q[Q_LUNIQ];
    sums[2] += q[Q_LCLAMP];
    sums[3] += q[Q_LTIE];
    sums[4] += q[Q_LRESTART];
  }
  return BX_OK;
}

int bx_ss_frame_stats_host(bx_ss* e, int seq0, int nseq, int64_t* sums) {
  if (!e || !sums || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_ss_frame_stats_host");
  std::vector<int> s((size_t)nseq * SQS);
  SCHK(hipDeviceSynchronize());
  if (nseq)
    SCHK(hipMemcpy(s.data(), e->dev.sq + (size_t)seq0 * SQS, sizeof(int) * s.size(),
                   hipMemcpyDeviceToHost));
  int64_t a[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < nseq; k++) {
    const int* q = s.data() + (size_t)k * SQS;
    a[0] += q[Q_NK];
    a[1] += q[Q_NT0];
    a[2] += q[Q_NNL];
    a[3] += q[Q_ROWSL];
    a[4] += q[Q_NOUT];
    a[5] = q[Q_FRAME] > a[5] ? q[Q_FRAME] : a[5];
    a[6] += q[Q_NM];
  }
  for (int k = 0; k < 7; k++) sums[k] = a[k];
  return BX_OK;
}

int bx_ss_probe(bx_ss* e, int stage) {
  if (!e) return bx_record_error(BX_ERR_INVALID, "null engine");
  e->probe_stage = stage;
  e->ev_used = 0;
  return BX_OK;
}

// Diagnostic (timing builds only; not in the public header): copies [S][32] phase counters.
int bx_ss_debug_host(bx_ss* e, unsigned long long* out) {
  if (!e || !out || !e->dev.dbg) return bx_record_error(BX_ERR_INVALID, "not a timing build");
  SCHK(hipDeviceSynchronize());
  SCHK(hipMemcpy(out, e->dev.dbg, sizeof(unsigned long long) * SS_DBG * e->dev.S,
                 hipMemcpyDeviceToHost));
  return BX_OK;
}

int bx_ss_probe_read(bx_ss* e, double* total_ms, int* count) {
  if (!e || !total_ms || !count) return bx_record_error(BX_ERR_INVALID, "null argument");
  double s = 0.0;
  for (int k = 0; k < e->ev_used; k++) {
    SCHK(hipEventSynchronize(e->ev[k].second));
    float ms = 0.f;
    SCHK(hipEventElapsedTime(&ms, e->ev[k].first, e->ev[k].second));
    s += ms;
  }
  *total_ms = s;
  *count = e->ev_used;
  e->ev_used = 0;
  return BX_OK;
}

}  // extern "C"
