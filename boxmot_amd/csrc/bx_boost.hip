// bx_boost.hip — the BoostTrack / BoostTrack++ per-frame update on MI355X.
//
// Reference: boxmot/trackers/boosttrack/boosttrack.py:123-456 (BoostTrack.update, its
// KalmanBoxTracker, the DLO/DUO confidence boosts, get_mh_dist_matrix), kalmanfilter.py:8-157
// (8-state constant-velocity filter with constant noise) and assoc.py:9-200 (iou_batch,
// soft_biou_batch, shape_similarity, MhDist_similarity, associate, match, linear_assignment).
//
// Per frame, three launches on the caller's stream:
//   boost_embcost_kernel  (with_reid) dets_embs @ trk_embs.T for every detection x live track of
//                         every sequence: fp64 MFMA (v_mfma_f64_16x16x4_f64), K staged through
//                         LDS, one 4-wave workgroup per sequence; the MFMA accumulates each entry
//                         as an ascending-k fma chain = oracle/bxo_boost.c emb_dot
//   boost_frame_kernel    one four-wave workgroup per sequence: CMC warp + Kalman predict (an
//                         octet of lanes per track, lane r owns row r), DLO/DUO boosts (thread
//                         per pair / lane groups per detection), the detection filter, the
//                         association cost (thread per entry), one-to-one fast path or lapx's JV
//                         (bx_jv.h, wave 0), validation, Kalman updates (octets), births,
//                         outputs, deaths; emits embedding-update records
//   boost_feature_kernel  (with_reid) wave per record: emb = a*emb + (1-a)*det, emb /= ||emb||
//                         (wave-order norm), or the newborn track's copy of its detection's
// Every floating-point expression restates oracle/bxo_boost.c operation for operation (built
// with -ffp-contract=off; f64 division and sqrt correctly rounded; exp = the same fdlibm exp),
// so ids, outputs and track states are bitwise those of the oracle.
#include <float.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/bxboost.h"
#include "bx_device.h"

using namespace bx;

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)
hipError_t bx_lds_attr(const void* kern, size_t bytes);  // bx_engine.hip (never lowers a limit)

namespace {

#include "bx_jv.h"

constexpr int SQB = 8;  // ints of per-sequence state
enum { SB_FRAME = 0, SB_IDS = 1, SB_NTR = 2, SB_NOUT = 3, SB_NREC = 4, SB_NDET = 5,
       SB_NKEEP = 6, SB_NT0 = 7 };
constexpr int TBB = 16;  // doubles per track of per-frame rows: box4 conf tsu x4 sinv4
constexpr double MH_LIMIT = 13.2767;

struct BstTrk {
  double x[8], P[64];
  double conf, cls, det_ind;
  int id, tsu, hit_streak, age;
};

struct BstDev {
  int S, T, D, N, F;
  double det_thresh, iou_thr, min_box_area, ar_thresh, l_iou, l_mhd, l_shape, dlo_coef;
  int max_age, min_hits, use_ecc, use_dlo, use_duo, s_sim_corr, rich_s, use_sb, use_vt, reid;
  int cost_lds, ntab;
  int tb_lds;             // the per-frame track rows staged in LDS (launches of <= 512 sequences)
  BstTrk* trk;            // [S][T]
  int* seqst;             // [S][SQB]
  int* order;             // [S][T] slot ids in the reference's list order
  double* tb;             // [S][T][TBB]
  double* cost_g;         // [S][D*T] or null
  double* e_g;            // [S][D*T] DLO MhDist numerators when they do not fit LDS, or null
  double* ec;             // [S][D][T] emb cost by (detection, list position)  (reid)
  double* emb;            // [S][T][F] track embeddings by slot                 (reid)
  int* rec;               // [S][D][2] (slot, global detection row)            (reid)
  double* rec_a;          // [S][D] EMA weight alpha, < 0: newborn copy          (reid)
  const double* conf_tab; // [ntab] 0.9 ** k (get_confidence)
  int* status;
  unsigned long long* dbg;  // [S][BST_DBG] phase stamps (diagnostic builds only, else null)
};

// Diagnostic phase stamps and counters (build with -DBX_PHASE_TIMING; never shipped): per
// sequence, cycles accumulated per phase over all frames [0, 16), event counters [16, 24) and
// the JV's counters [24, 40).
constexpr int BST_DBG = 40;
// lapjv(-cost, extend_cost=True) by the shortest-augmenting-path solve + uniqueness test, lapjv
// itself only for a tied optimum (legacy_lap_ssp); 0: lapjv always
#ifndef BX_BOOST_SSP
#define BX_BOOST_SSP 1
#endif
#ifdef BX_PHASE_TIMING
#define BSTAMP(k)                                                                    \
  do {                                                                               \
    __syncthreads();                                                                 \
    if (threadIdx.x == 0 && g.dbg) {                                                 \
      const unsigned long long _now = __builtin_amdgcn_s_memtime();                  \
      g.dbg[(size_t)seq * BST_DBG + (k)] += _now - t_last;                           \
      t_last = _now;                                                                 \
    }                                                                                \
  } while (0)
#define BCOUNT(k, v)                                                                 \
  do {                                                                               \
    if (threadIdx.x == 0 && g.dbg) g.dbg[(size_t)seq * BST_DBG + 16 + (k)] += (v);   \
  } while (0)
#else
#define BSTAMP(k) \
  do {            \
  } while (0)
#define BCOUNT(k, v) \
  do {               \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------
// fdlibm exp (oracle/bxo_boost.c bxo_exp)
__device__ double bst_exp(double x) {
  const double halF[2] = {0.5, -0.5}, huge = 1.0e+300, twom1000 = 9.33263618503218878990e-302,
               o_th = 7.09782712893383973096e+02, u_th = -7.45133219101941108420e+02,
               ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
               ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
               invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
               P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
               P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
  const unsigned long long bits = (unsigned long long)__double_as_longlong(x);
  unsigned hx = (unsigned)(bits >> 32);
  const unsigned lx = (unsigned)bits;
  const int xsb = (hx >> 31) & 1;
  hx &= 0x7fffffff;
  double hi = 0.0, lo = 0.0;
  int k = 0;
  if (hx >= 0x40862E42u) {
    if (hx >= 0x7ff00000u) {
      if (((hx & 0xfffffu) | lx) != 0) return x + x;
      return xsb == 0 ? x : 0.0;
    }
    if (x > o_th) return huge * huge;
    if (x < u_th) return twom1000 * twom1000;
  }
  if (hx > 0x3fd62e42u) {
    if (hx < 0x3FF0A2B2u) {
      hi = x - ln2HI[xsb];
      lo = ln2LO[xsb];
      k = 1 - xsb - xsb;
    } else {
      k = (int)(invln2 * x + halF[xsb]);
      const double t = k;
      hi = x - t * ln2HI[0];
      lo = t * ln2LO[0];
    }
    x = hi - lo;
  } else if (hx < 0x3e300000u) {
    return 1.0 + x;
  } else {
    k = 0;
  }
  const double t = x * x;
  const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  const double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  long long yb = __double_as_longlong(y);
  if (k >= -1021) return __longlong_as_double(yb + ((long long)k << 52));
  return __longlong_as_double(yb + ((long long)(k + 1000) << 52)) * twom1000;
}

// x ** 1.5 (oracle bxo_pow15)
__device__ double bst_pow15(double x) {
  if (x != x) return x;
  if (x < 0.0) return __builtin_nan("");
  if (x == 0.0) return 0.0;
  if (isinf(x)) return x;
  const double s = sqrt(x);
  const double r = fma(-s, s, x);
  const double p = x * s;
  const double e = fma(x, s, -p);
  return p + (e + x * (r / (2.0 * s)));
}

__device__ __forceinline__ double nmax(double a, double b) {
  return (a != a || b != b) ? __builtin_nan("") : (a > b ? a : b);
}
__device__ __forceinline__ double nmin(double a, double b) {
  return (a != a || b != b) ? __builtin_nan("") : (a < b ? a : b);
}

// boosttrack.py:19-28 convert_bbox_to_z
__device__ __forceinline__ void bbox_to_z(const double* b, double* z) {
  const double w = b[2] - b[0], h = b[3] - b[1];
  z[0] = b[0] + w / 2.0;
  z[1] = b[1] + h / 2.0;
  z[2] = h;
  z[3] = w / (h + 1e-6);
}

// boosttrack.py:31-42 convert_x_to_bbox
__device__ __forceinline__ void x_to_bbox(double x0, double x1, double x2, double x3, double* b) {
  const double h = x2, r = x3;
  const double w = r <= 0 ? 0.0 : r * h;
  b[0] = x0 - w / 2.0;
  b[1] = x1 - h / 2.0;
  b[2] = x0 + w / 2.0;
  b[3] = x1 + h / 2.0;
}

// assoc.py:50-66 iou_batch (a: detection row, b: tracker / detection row)
__device__ __forceinline__ double iou_b(const double* a, const double* b) {
  const double xx1 = nmax(a[0], b[0]), yy1 = nmax(a[1], b[1]);
  const double xx2 = nmin(a[2], b[2]), yy2 = nmin(a[3], b[3]);
  const double w = nmax(0.0, xx2 - xx1), h = nmax(0.0, yy2 - yy1);
  const double wh = w * h;
  return wh / ((a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - wh);
}

// assoc.py:69-103 soft_biou_batch
__device__ __forceinline__ double soft_biou(const double* a, const double* b, double bconf) {
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

// assoc.py:9-34 shape_similarity v1 / v2
__device__ __forceinline__ double shape_sim(const double* a, const double* b, int v2) {
  const double dw = a[2] - a[0], dh = a[3] - a[1];
  const double tw = b[2] - b[0], th = b[3] - b[1];
  const double mw = nmax(dw, tw), mh = v2 ? nmax(dh, th) : mw;
  return bst_exp(-(fabs(dw - tw) / mw + fabs(dh - th) / mh));
}

// get_mh_dist_matrix entry (boosttrack.py:356-369); det = LDS row (convert_bbox_to_z at +7),
// r = tb row (x at +6, 1/diag(P) at +10)
constexpr int DDW = 11;  // doubles per detection row: x1 y1 x2 y2 conf cls det_ind z[4]
__device__ __forceinline__ double mh_dist(const double* det, const double* r) {
  const double* z = det + 7;
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const double d = z[q] - r[6 + q];
    s += d * d * r[10 + q];
  }
  return s;
}

// exp(limit - min(mh, limit)): the softmax numerator of MhDist_similarity (assoc.py:37-47)
__device__ __forceinline__ double mh_num(double v, bool& mask) {
  mask = v > MH_LIMIT;
  if (mask) v = MH_LIMIT;
  return bst_exp(MH_LIMIT - v);
}

// ------------------------------------------------------------------------------------------
// Kalman filter on octets: lane r (0..7) of the octet owns x[r] and row r of P.
__device__ __forceinline__ double osh(double v, int src) { return __shfl(v, src, 8); }

// kalmanfilter.py:75-107: x = F x; P = F (P F^T) + Q (oracle bkf_predict)
__device__ __forceinline__ void okf_predict(int r, double& xr, double (&Pr)[8]) {
  const double x4 = osh(xr, (r + 4) & 7);
  if (r < 4) xr = xr + x4;
  double M[8];
#pragma unroll
  for (int j = 0; j < 8; j++) M[j] = j < 4 ? Pr[j] + Pr[j + 4] : Pr[j];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const double m4 = osh(M[j], (r + 4) & 7);
    const double v = r < 4 ? M[j] + m4 : M[j];
    Pr[j] = j == r ? v + (r < 4 ? 1.0 : 0.01) : v;
  }
}

// kalmanfilter.py:127-157, R = diag(1, 1, 10, 0.01) (oracle bkf_update)
__device__ __forceinline__ void okf_update(int r, double& xr, double (&Pr)[8], const double* z) {
  const double R[4] = {1.0, 1.0, 10.0, 0.01};
  double S[16], L[16];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) S[4 * i + j] = osh(Pr[j], i) + (i == j ? R[i] : 0.0);
  if (!chol4(S, L)) return;  // every lane of the octet sees the same S
  double y[4], K[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double s = Pr[i];
    for (int q = 0; q < i; q++) s -= L[4 * i + q] * y[q];
    y[i] = s / L[4 * i + i];
  }
#pragma unroll
  for (int i = 3; i >= 0; i--) {
    double s = y[i];
    for (int q = i + 1; q < 4; q++) s -= L[4 * q + i] * K[q];
    K[i] = s / L[4 * i + i];
  }
  double innov[4];
#pragma unroll
  for (int q = 0; q < 4; q++) innov[q] = z[q] - osh(xr, q);
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < 4; q++) s += innov[q] * K[q];
  xr = xr + s;
  double ks[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    double a = 0.0;
#pragma unroll
    for (int q = 0; q < 4; q++) a += K[q] * S[4 * q + j];
    ks[j] = a;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    double a = 0.0;
#pragma unroll
    for (int q = 0; q < 4; q++) a += ks[q] * osh(K[q], j);
    Pr[j] = Pr[j] - a;
  }
}

// ------------------------------------------------------------------------------------------
struct BstLds {
  double* dd;    // [D][DDW] detections of the frame (float32 values as f64, conf boosted,
                 // det_ind, convert_bbox_to_z)
  double* cost;  // [cost_lds]
  double* colsum;  // [T]
  double* tbl;     // [T][TBB] the frame's track rows (tb_lds) or null
  int *kd, *bi;    // [D] kept detections, DUO boost candidates
  int *lst, *lst2; // [T]
  int *mi, *mm;    // [2N] candidate / validated (kept det, list position) pairs
  int *ud, *ut;    // [D+T] unmatched lists
  int *rowcnt, *colcnt, *rowcol, *fl;  // [N] each
  int* u;          // [8] values one wave derives for all
  JvLds jv;
};

__device__ void carve(const BstDev& g, char* base, BstLds& L) {
  size_t o = 0;
  auto takeD = [&](size_t n) { double* p = (double*)(base + o); o += n * 8; return p; };
  auto takeI = [&](size_t n) { int* p = (int*)(base + o); o += ((n * 4 + 7) / 8) * 8; return p; };
  const int N = g.N, D = g.D, T = g.T;
  L.dd = takeD((size_t)D * DDW);
  L.cost = takeD(g.cost_lds);
  L.colsum = takeD(T);
  L.tbl = g.tb_lds ? takeD((size_t)T * TBB) : nullptr;
  L.jv.v = takeD(N);
  L.jv.d = takeD(N);
  L.jv.sd = takeD(2);
  L.kd = takeI(D);
  L.bi = takeI(D);
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
  L.jv.x = takeI(N);
  L.jv.y = takeI(N);
  L.jv.matches = takeI(N);
  L.jv.freer = takeI(N);
  L.jv.pred = takeI(N);
  L.jv.col = takeI(N);
  L.jv.sc = takeI(8);
  L.u = takeI(8);
  L.jv.dc = nullptr;
}

size_t lds_bytes(int D, int T, int N, int cost_lds, int tb_lds) {
  auto dI = [](size_t n) { return ((n * 4 + 7) / 8) * 8; };
  return (size_t)D * DDW * 8 + (size_t)cost_lds * 8 + (size_t)T * 8 + 2 * (size_t)N * 8 + 2 * 8 +
         (tb_lds ? (size_t)T * TBB * 8 : 0) +
         2 * dI(D) + 2 * dI(T) + 2 * dI(2 * N) + 2 * dI(D + T) + 4 * dI(N) + 6 * dI(N) + dI(8) +
         dI(8);
}

// One workgroup of 2-6 waves per sequence (frame_threads: six for up to 256 sequences in the
// launch, three up to 511, two from 512 on — at 1024 sequences two waves each measured 5% faster
// than one (C2 1.39 -> 1.46 M frames/s) and four 20% slower; at C5, since the LAP no longer runs
// lapjv, six waves 55.1 k frames/s against 52.5 k with four, 54.6 k with eight, 54.5 k with twelve).  Work over pairs, detections or tracks
// is spread over all the waves; the order-dependent steps (compactions, the validation's ballots)
// run in every wave at once on the same LDS data — each wave derives the same counts and writes the
// same values — except the JV, which wave 0 solves alone (SyncWaveL) while the others wait at the
// barrier after it.
#ifndef BX_BOOST_MAX_THREADS
#define BX_BOOST_MAX_THREADS 384
#endif
constexpr int BW = BX_BOOST_MAX_THREADS > 256 ? BX_BOOST_MAX_THREADS : 256;  // the most threads per sequence
#ifndef BX_BOOST_THREADS_1024
#define BX_BOOST_THREADS_1024 128
#endif
__host__ __device__ constexpr int frame_threads(int nseq) {
  return nseq >= 1024 ? BX_BOOST_THREADS_1024
                      : nseq >= 512 ? 128 : nseq > 256 ? 192 : BX_BOOST_MAX_THREADS;
}
constexpr int COST_KR = 4;  // cost entries per thread per chunk (registers held across a barrier)

__global__ void __launch_bounds__(BW)
    boost_frame_kernel(BstDev g, int seq0, const float* __restrict__ dets,
                       const int* __restrict__ det_off, const double* __restrict__ warps,
                       double* __restrict__ out, int* __restrict__ out_count) {
  extern __shared__ __align__(16) char lds_raw[];
  BstLds L;
  carve(g, lds_raw, L);
  const int tid = threadIdx.x, lane = tid & 63, nth = blockDim.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x, seq = seq0 + b;
  L.jv.dc = g.dbg ? g.dbg + (size_t)seq * BST_DBG + 24 : nullptr;
  const int r0 = det_off[b];
  int n = det_off[b + 1] - r0;
  if (n > g.D) {  // the host checks det_cap; a device-side overflow is latched, never run past
    if (tid == 0) atomicExch(g.status, (int)BX_ERR_CAPACITY);
    n = g.D;
  }
  int* sq = g.seqst + (size_t)seq * SQB;
  BstTrk* trk = g.trk + (size_t)seq * g.T;
  int* order = g.order + (size_t)seq * g.T;
  // the frame's track rows: written by the predict phase, read by every later phase (per pair in
  // DLO / DUO / the cost): in LDS when the launch leaves room, else this sequence's HBM rows
  double* tb = g.tb_lds ? L.tbl : g.tb + (size_t)seq * g.T * TBB;
  double* costg = g.cost_g ? g.cost_g + (size_t)seq * g.D * g.T : nullptr;
  double* eg = g.e_g ? g.e_g + (size_t)seq * g.D * g.T : nullptr;
  const double* ec = g.reid ? g.ec + (size_t)seq * g.D * g.T : nullptr;
  const int frame = sq[SB_FRAME] + 1;
  const int id0 = sq[SB_IDS];
  const int nt = sq[SB_NTR];
  const double thr = g.iou_thr;
  const double det_thresh = g.det_thresh;
#ifdef BX_PHASE_TIMING
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif

  // detections (x1,y1,x2,y2,conf,cls, det_ind = input row) and the track list
  for (int q = tid; q < n * 6; q += nth) L.dd[(q / 6) * DDW + q % 6] = (double)dets[(size_t)r0 * 6 + q];
  __syncthreads();
  for (int i = tid; i < n; i += nth) {
    L.dd[DDW * i + 6] = (double)i;
    bbox_to_z(L.dd + DDW * i, L.dd + DDW * i + 7);
  }
  for (int p = tid; p < nt; p += nth) L.lst[p] = order[p];
  __syncthreads();
  BSTAMP(0);

  // ---- CMC warp (camera_update, boosttrack.py:81-103) + predict (:105-111), octet per track;
  // tb row: box[4], get_confidence, time_since_update, x[0..3], 1/diag(P)[0..3]
  const int oct = tid >> 3, r = tid & 7;
  double w6[6] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0};
  if (warps)
    for (int q = 0; q < 6; q++) w6[q] = warps[(size_t)b * 6 + q];
  for (int c = 0; c < nt; c += nth / 8) {
    const int p = c + oct;
    if (p < nt) {
      BstTrk& t = trk[L.lst[p]];
      double xr = t.x[r], Pr[8];
#pragma unroll
      for (int j = 0; j < 8; j++) Pr[j] = t.P[8 * r + j];
      if (g.use_ecc) {
        double bx[4];
        x_to_bbox(osh(xr, 0), osh(xr, 1), osh(xr, 2), osh(xr, 3), bx);
        const double x1 = (w6[0] * bx[0] + w6[1] * bx[1]) + w6[2];
        const double y1 = (w6[3] * bx[0] + w6[4] * bx[1]) + w6[5];
        const double x2 = (w6[0] * bx[2] + w6[1] * bx[3]) + w6[2];
        const double y2 = (w6[3] * bx[2] + w6[4] * bx[3]) + w6[5];
        const double ww = x2 - x1, hh = y2 - y1;
        if (r == 0) xr = x1 + ww / 2;
        if (r == 1) xr = y1 + hh / 2;
        if (r == 2) xr = hh;
        if (r == 3) xr = ww / hh;
      }
      okf_predict(r, xr, Pr);
      t.x[r] = xr;
#pragma unroll
      for (int j = 0; j < 8; j++) t.P[8 * r + j] = Pr[j];
      const int age = t.age + 1, tsu0 = t.tsu, tsu = tsu0 + 1;
      double bx[4];
      x_to_bbox(osh(xr, 0), osh(xr, 1), osh(xr, 2), osh(xr, 3), bx);
      double* row = tb + (size_t)p * TBB;
      if (r < 4) {
        row[r] = bx[r];
        row[6 + r] = xr;
        row[10 + r] = 1.0 / Pr[r];
      } else if (r == 4) {
        // get_confidence (boosttrack.py:66-70): 0.9 ** k from the host's libm pow
        const int k = age < 7 ? 7 - age : tsu - 1;
        row[4] = g.conf_tab[k < g.ntab ? k : g.ntab - 1];
      } else if (r == 5) {
        row[5] = (double)tsu;
      } else if (r == 6) {
        t.age = age;
        if (tsu0 > 0) t.hit_streak = 0;
        t.tsu = tsu;
      }
    }
  }
  __syncthreads();
  BSTAMP(1);

  // ---- DLO confidence boost (boosttrack.py:413-456) ----------------------------------------
  // With rich_s: E[d][t] = the MhDist numerator of every (detection, track) pair, negated where
  // MhDist clipped (exp() > 0), thread per pair, staged in the cost matrix's LDS (not used yet)
  // or the sequence's global scratch; then the column sums in detection order (thread per track).
  // E stays intact for the association cost.
  const double* E = nullptr;
  if (g.use_dlo && n > 0 && nt > 0) {
    if (g.rich_s) {
      double* Ew = (n * nt <= g.cost_lds) ? L.cost : eg;
      for (int p = tid; p < n * nt; p += nth) {
        const int d = p / nt, t = p - d * nt;
        bool m;
        const double e = mh_num(mh_dist(L.dd + DDW * d, tb + (size_t)t * TBB), m);
        Ew[p] = m ? -e : e;
      }
      __syncthreads();
      for (int t = tid; t < nt; t += nth) {
        double cs = 0.0;
        for (int d = 0; d < n; d++) {
          const double e = fabs(Ew[d * nt + t]);
          cs = d == 0 ? e : cs + e;
        }
        L.colsum[t] = cs;
      }
      __syncthreads();
      E = Ew;
    }
    // S[d][t] = ((MhSim + shape) + soft-BIoU) / 3 (rich_s) or IoU: G threads per detection (G =
    // the largest power of two with n * G <= nth, at most 16), each over the tracks t = sub
    // (mod G); each detection's max over tracks (np.max: NaN-propagating, otherwise order-free)
    // and the VT test combined within the thread group by shuffles (the group stays in a wave)
    int G = 1;
    while (G < 16 && n * G * 2 <= nth) G *= 2;
    const int sub = tid & (G - 1);
    for (int d0 = 0; d0 < n * G; d0 += nth) {
      const int d = (d0 + tid) / G;
      const bool live = d < n;
      const double* a = L.dd + DDW * (live ? d : 0);
      double mx = -INF;
      bool nan = false, vt = false;
      if (live) {
        for (int t = sub; t < nt; t += G) {
          const double* rw = tb + (size_t)t * TBB;
          double S;
          if (E) {
            const double ev = E[d * nt + t];
            const double mhs = ev < 0 ? 0.0 : ev / L.colsum[t];
            S = ((mhs + shape_sim(a, rw, g.s_sim_corr)) + soft_biou(a, rw, rw[4])) / 3;
          } else {
            S = iou_b(a, rw);
          }
          if (S != S)
            nan = true;
          else
            mx = mx > S ? mx : S;
          if (g.use_vt && S > nmax(0.95 - (rw[5] - 1.0), 0.8)) vt = true;
        }
      }
      for (int o = 1; o < G; o <<= 1) {  // within the thread group (xor stays inside it)
        const double om = __shfl_xor(mx, o);
        mx = om > mx ? om : mx;
        nan = (__shfl_xor((int)nan, o) != 0) || nan;
        vt = (__shfl_xor((int)vt, o) != 0) || vt;
      }
      if (live && sub == 0) {
        const double max_s = nan ? __builtin_nan("") : mx;
        double c = a[4];
        if (!g.use_sb && !g.use_vt) {
          c = nmax(c, max_s * g.dlo_coef);
        } else {
          if (g.use_sb) {
            const double alpha = 0.65;
            c = nmax(c, alpha * c + (1 - alpha) * bst_pow15(max_s));
          }
          if (g.use_vt && vt) c = nmax(c, det_thresh + 1e-5);
        }
        L.dd[DDW * d + 4] = c;
      }
    }
    __syncthreads();
  }

  BSTAMP(2);
  // ---- DUO confidence boost (boosttrack.py:371-411) ----------------------------------------
  if (g.use_duo && n > 0 && nt > 0) {
    const int nb = wave_compact(
        n,
        [&](int d) {
          const double* a = L.dd + DDW * d;
          double m = 0.0;
          for (int t = 0; t < nt; t++) {
            const double v = mh_dist(a, tb + (size_t)t * TBB);
            m = t == 0 ? v : nmin(m, v);
          }
          return m > MH_LIMIT && a[4] < det_thresh;
        },
        [&](int d, int p) { L.bi[p] = d; });
    if (nb > 0) {
      // bdiou = iou(boost, boost) - eye: row maxima -> remaining (<= .3) / args (> .3)
      for (int i = tid; i < nb; i += nth) {
        const double* a = L.dd + DDW * L.bi[i];
        double m = 0.0;
        for (int j = 0; j < nb; j++) {
          const double v = iou_b(a, L.dd + DDW * L.bi[j]) - (i == j ? 1.0 : 0.0);
          m = j == 0 ? v : nmax(m, v);
        }
        L.fl[i] = (m <= 0.3 ? 1 : 0) | (m > 0.3 ? 2 : 0);
      }
      __syncthreads();
      // an overlapping candidate stays if it holds the maximum confidence of its overlaps
      for (int i = tid; i < nb; i += nth) {
        if (!(L.fl[i] & 2)) continue;
        const double* a = L.dd + DDW * L.bi[i];
        double cm = a[4];
        for (int j = 0; j < nb; j++) {
          if (!(L.fl[j] & 2)) continue;
          const double* bj = L.dd + DDW * L.bi[j];
          if (iou_b(a, bj) - (i == j ? 1.0 : 0.0) > 0.3) cm = nmax(cm, bj[4]);
        }
        if (a[4] == cm) L.fl[i] |= 4;
      }
      __syncthreads();
      for (int i = tid; i < nb; i += nth)
        if (L.fl[i] & 5) L.dd[DDW * L.bi[i] + 4] = det_thresh + 1e-4;
      __syncthreads();
    }
  }

  BSTAMP(3);
  // ---- detections kept for the association (boosttrack.py:262-266) ------------------------
  const int nk = wave_compact(n, [&](int d) { return L.dd[DDW * d + 4] >= det_thresh; },
                              [&](int d, int p) { L.kd[p] = d; });

  // ---- associate (assoc.py:156-200) ---------------------------------------------------------
  int nm = 0, nud = 0, nut = 0;
  if (nt == 0) {
    for (int k = tid; k < nk; k += nth) L.ud[k] = k;
    nud = nk;
    __syncthreads();
  } else {
    int nmi = 0;
    const double lambda_emb = (((1 + g.l_iou) + g.l_shape) + g.l_mhd) * 1.5;
    double* C = (nk * nt <= g.cost_lds) ? L.cost : costg;
    if (nk > 0) {
      // MhDist_similarity over the kept detections: column sums, thread per track (from the DLO
      // boost's E when it staged one: the boosts change confidences, never boxes)
      for (int t = tid; t < nt; t += nth) {
        const double* rw = tb + (size_t)t * TBB;
        double cs = 0.0;
        for (int i = 0; i < nk; i++) {
          double e;
          if (E) {
            e = fabs(E[L.kd[i] * nt + t]);
          } else {
            bool m;
            e = mh_num(mh_dist(L.dd + DDW * L.kd[i], rw), m);
          }
          cs = i == 0 ? e : cs + e;
        }
        L.colsum[t] = cs;
      }
      for (int k = tid; k < nk; k += nth) L.rowcnt[k] = 0;
      for (int k = tid; k < nt; k += nth) L.colcnt[k] = 0;
      __syncthreads();
      BSTAMP(4);
      // the cost matrix (stored negated for lapjv(-cost)), thread per entry p = i * nt + t; counts
      // of entries above the threshold per row/column for match()'s one-to-one test.  C may be E's
      // storage: entry p reads E at kd[i] * nt + t >= p, so a chunk's entries are all computed
      // before any is stored and no later chunk reads below its own first entry.
      const int np = nk * nt;
      for (int c0 = 0; c0 < np; c0 += nth * COST_KR) {
        double cv[COST_KR];
#pragma unroll
        for (int k = 0; k < COST_KR; k++) {
          const int p = c0 + k * nth + tid;
          cv[k] = 0.0;
          if (p < np) {
            const int i = p / nt, t = p - i * nt;
            const double* rw = tb + (size_t)t * TBB;
            const int d = L.kd[i];
            const double* a = L.dd + DDW * d;
            const double o = iou_b(a, rw);
            double cst = o;
            double cf = a[4] * rw[4];
            if (o < thr) cf = 0.0;
            cst += g.l_iou * cf * o;
            bool m;
            double e;
            if (E) {
              const double ev = E[d * nt + t];
              m = ev < 0;
              e = fabs(ev);
            } else {
              e = mh_num(mh_dist(a, rw), m);
            }
            cst += g.l_mhd * (m ? 0.0 : e / L.colsum[t]);
            cst += g.l_shape * cf * shape_sim(a, rw, g.s_sim_corr);
            if (ec) cst += lambda_emb * ec[(size_t)d * g.T + t];
            cv[k] = cst;
          }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < COST_KR; k++) {
          const int p = c0 + k * nth + tid;
          if (p < np) {
            const int i = p / nt, t = p - i * nt;
            C[p] = -cv[k];
            if (cv[k] > thr) {
              atomicAdd(&L.rowcnt[i], 1);
              L.rowcol[i] = t;  // read only where the row's count is 1
              atomicAdd(&L.colcnt[t], 1);
            }
          }
        }
      }
      __syncthreads();
      BSTAMP(5);
      int mr = 0, mc = 0;
      for (int k = lane; k < nk; k += OW) mr = max(mr, L.rowcnt[k]);
      for (int k = lane; k < nt; k += OW) mc = max(mc, L.colcnt[k]);
      for (int o = 32; o >= 1; o >>= 1) {
        mr = max(mr, __shfl_xor(mr, o));
        mc = max(mc, __shfl_xor(mc, o));
      }
      if (mr == 1 && mc == 1) {  // np.stack(np.where(cost > thr), 1): row-major
        nmi = wave_compact(
            nk, [&](int i) { return L.rowcnt[i] == 1; },
            [&](int i, int p) {
              L.mi[2 * p] = i;
              L.mi[2 * p + 1] = L.rowcol[i];
            });
      } else {  // lap.lapjv(-cost, extend_cost=True) -> [[y[i], i] for i in x if i >= 0]
        if (wid == 0) {
          // (generic cost loads: LDS-typed ones, legacy_lap's cas = 3, measured slower at C5,
          // frame kernel 0.413 vs 0.393 ms)
#if BX_BOOST_SSP
          bool jv_ran;
          nmi = legacy_lap_ssp(C, nk, nt, L.jv, L.mi, SyncWaveL{}, jv_ran);
          BCOUNT(6, jv_ran ? 1 : 0);
#else
          nmi = legacy_lap(C, nk, nt, L.jv, L.mi, SyncWaveL{});
#endif
          if (lane == 0) L.u[0] = nmi;
        }
        __syncthreads();
        nmi = L.u[0];
        BCOUNT(0, 1);
        BCOUNT(1, nk > nt ? nk : nt);
        BCOUNT(5, (nk > nt ? nk : nt) > OW ? 1 : 0);
      }
      BSTAMP(6);
    }
    // linear_assignment (assoc.py:117-153): unmatched = absent from the pairs, ascending; then
    // the validation, rejected pairs appended in pair order
    for (int k = tid; k < g.N; k += nth) L.rowcnt[k] = L.colcnt[k] = 0;
    __syncthreads();
    for (int q = tid; q < nmi; q += nth) {
      L.rowcnt[L.mi[2 * q]] = 1;
      L.colcnt[L.mi[2 * q + 1]] = 1;
    }
    __syncthreads();
    nud = wave_compact(nk, [&](int i) { return L.rowcnt[i] == 0; }, [&](int i, int p) { L.ud[p] = i; });
    nut = wave_compact(nt, [&](int t) { return L.colcnt[t] == 0; }, [&](int t, int p) { L.ut[p] = t; });
    for (int c = 0; c < nmi; c += OW) {
      const int q = c + lane;
      bool ok = false, rej = false;
      int i = 0, t = 0;
      if (q < nmi) {
        i = L.mi[2 * q];
        t = L.mi[2 * q + 1];
        const int d = L.kd[i];
        const double o = iou_b(L.dd + DDW * d, tb + (size_t)t * TBB);
        ok = o >= thr || (ec ? (o >= thr / 2 && ec[(size_t)d * g.T + t] >= 0.75) : false);
        rej = !ok;
      }
      const unsigned long long mo = __ballot(ok), mrj = __ballot(rej);
      const unsigned long long below = (1ull << lane) - 1ull;
      if (ok) {
        const int p = nm + __popcll(mo & below);
        L.mm[2 * p] = i;
        L.mm[2 * p + 1] = t;
      }
      if (rej) {
        const int p = __popcll(mrj & below);
        L.ud[nud + p] = i;
        L.ut[nut + p] = t;
      }
      nm += __popcll(mo);
      nud += __popcll(mrj);
      nut += __popcll(mrj);
    }
    __syncthreads();
  }

  BSTAMP(7);
  BCOUNT(2, nk);
  BCOUNT(3, nt);
  BCOUNT(4, 1);
  // ---- matched updates (boosttrack.py:297-306), octet per pair ------------------------------
  int* rec = g.reid ? g.rec + (size_t)seq * g.D * 2 : nullptr;
  double* rec_a = g.reid ? g.rec_a + (size_t)seq * g.D : nullptr;
  for (int c = 0; c < nm; c += nth / 8) {
    const int q = c + oct;
    if (q < nm) {
      const int d = L.kd[L.mm[2 * q]];
      const int slot = L.lst[L.mm[2 * q + 1]];
      const double* a = L.dd + DDW * d;
      BstTrk& t = trk[slot];
      double xr = t.x[r], Pr[8];
#pragma unroll
      for (int j = 0; j < 8; j++) Pr[j] = t.P[8 * r + j];
      double z[4];
      bbox_to_z(a, z);
      okf_update(r, xr, Pr, z);
      t.x[r] = xr;
#pragma unroll
      for (int j = 0; j < 8; j++) t.P[8 * r + j] = Pr[j];
      if (r == 0) {
        t.tsu = 0;
        t.hit_streak++;
        t.conf = a[4];
        t.cls = a[5];
        t.det_ind = a[6];
        if (rec) {  // update_emb weight (boosttrack.py:290-295)
          const double trust = (a[4] - det_thresh) / (1 - det_thresh);
          const double af = 0.95;
          rec[2 * q] = slot;
          rec[2 * q + 1] = r0 + d;
          rec_a[q] = af + (1 - af) * (1 - trust);
        }
      }
    }
  }
  __syncthreads();

  BSTAMP(8);
  // ---- births for the unmatched detections (boosttrack.py:308-312), free slots ascending ----
  for (int s2 = tid; s2 < g.T; s2 += nth) L.fl[s2] = 0;
  __syncthreads();
  for (int p = tid; p < nt; p += nth) L.fl[L.lst[p]] = 1;
  __syncthreads();
  const int nfree = wave_compact(g.T, [&](int s2) { return L.fl[s2] == 0; }, [&](int s2, int p) { L.lst2[p] = s2; });
  int nnew = nud;  // every kept detection satisfies dets[i, 4] >= det_thresh
  if (nnew > nfree) {
    if (tid == 0) atomicExch(g.status, (int)BX_ERR_TRACK_OVERFLOW);
    nnew = nfree;
  }
  for (int c = 0; c < nnew; c += nth / 8) {
    const int k = c + oct;
    if (k < nnew) {
      const int slot = L.lst2[k];
      const int d = L.kd[L.ud[k]];
      const double* a = L.dd + DDW * d;
      BstTrk& t = trk[slot];
      double z[4];
      bbox_to_z(a, z);
      t.x[r] = r < 4 ? z[r] : 0.0;
#pragma unroll
      for (int j = 0; j < 8; j++) t.P[8 * r + j] = j == r ? (r < 4 ? 10.0 : 10000.0) : 0.0;
      if (r == 0) {
        t.id = id0 + k + 1;
        t.conf = a[4];
        t.cls = a[5];
        t.det_ind = a[6];
        t.tsu = t.hit_streak = t.age = 0;
        L.lst[nt + k] = slot;
        if (rec) {
          rec[2 * (nm + k)] = slot;
          rec[2 * (nm + k) + 1] = r0 + d;
          rec_a[nm + k] = -1.0;
        }
      }
    }
  }
  __syncthreads();
  const int ntr = nt + nnew;
  BSTAMP(9);

  // ---- outputs in list order + filter_outputs (boosttrack.py:314-341), then deaths; every wave
  // counts, wave 0 writes ----------------------------------------------------------------------
  double* orow = out + (size_t)r0 * 8;
  auto out_box = [&](const BstTrk& t, double* bx) { x_to_bbox(t.x[0], t.x[1], t.x[2], t.x[3], bx); };
  const int nout = wave_compact(
      ntr,
      [&](int k) {
        const BstTrk& t = trk[L.lst[k]];
        if (!(t.tsu < 1 && (t.hit_streak >= g.min_hits || frame <= g.min_hits))) return false;
        double bx[4];
        out_box(t, bx);
        const double w = bx[2] - bx[0], h = bx[3] - bx[1];
        return (w / h <= g.ar_thresh) && (w * h > g.min_box_area);
      },
      [&](int k, int p) {
        if (wid != 0 || p >= n) return;
        const BstTrk& t = trk[L.lst[k]];
        double bx[4];
        out_box(t, bx);
        double* o = orow + (size_t)p * 8;
        o[0] = bx[0]; o[1] = bx[1]; o[2] = bx[2]; o[3] = bx[3];
        o[4] = (double)t.id;
        o[5] = t.conf;
        o[6] = t.cls;
        o[7] = t.det_ind;
      });
  const int nkeep = wave_compact(
      ntr, [&](int k) { return trk[L.lst[k]].tsu <= g.max_age; },
      [&](int k, int p) {
        if (wid == 0) order[p] = L.lst[k];
      });
  BSTAMP(10);
  if (tid == 0) {
    out_count[b] = nout < n ? nout : n;
    sq[SB_FRAME] = frame;
    sq[SB_IDS] = id0 + nnew;
    sq[SB_NTR] = nkeep;
    sq[SB_NOUT] = nout;
    sq[SB_NREC] = rec ? nm + nnew : 0;
    sq[SB_NDET] = n;
    sq[SB_NKEEP] = nk;
    sq[SB_NT0] = nt;
  }
}

// ------------------------------------------------------------------------------------------
// dets_embs @ trk_embs.T (boosttrack.py:274-281) for every detection x live track of a
// sequence, on the fp64 matrix cores.  One workgroup of 4 waves per output tile of 32 detections x
// 64 tracks (grid (sequences, tiles); wave (wr, wc): rows 16 wr, columns 32 wc + {0, 16}); K
// advances in chunks of 16 through LDS stored k-major, with EC_PF chunks' global loads in flight
// (a chunk's MFMAs take ~50 ns, a load round trip ~1 us: the loop is bound by how many round
// trips it waits for).  Entry (d, p) = ascending-k fma chain over F (oracle emb_dot).
constexpr int EC_BM = 32, EC_BN = 64, EC_KC = 16, EC_LDA = EC_BM + 16, EC_LDB = EC_BN + 16;
constexpr int EC_STAGE = EC_KC * (EC_LDA + EC_LDB);
#ifndef BX_EC_PF
#define BX_EC_PF 4
#endif
constexpr int EC_PF = BX_EC_PF;  // chunks in flight
typedef double d4 __attribute__((ext_vector_type(4)));
__host__ __device__ constexpr int ec_tiles_t(int T) { return (T + EC_BN - 1) / EC_BN; }
__host__ __device__ constexpr int ec_tiles(int D, int T) {
  return (D + EC_BM - 1) / EC_BM * ec_tiles_t(T);
}

__global__ void __launch_bounds__(256)
    boost_embcost_kernel(BstDev g, int seq0, const int* __restrict__ det_off,
                         const double* __restrict__ embs) {
  __shared__ double lds[2 * EC_STAGE];
  const int b = blockIdx.x, seq = seq0 + b;
  const int r0 = det_off[b];
  int nd = det_off[b + 1] - r0;
  if (nd > g.D) nd = g.D;
  const int nt = g.seqst[(size_t)seq * SQB + SB_NTR];
  const int d0 = (int)blockIdx.y / ec_tiles_t(g.T) * EC_BM;
  const int t0 = (int)blockIdx.y % ec_tiles_t(g.T) * EC_BN;
  if (d0 >= nd || t0 >= nt) return;  // workgroup-uniform
  const int F = g.F;
  const int* order = g.order + (size_t)seq * g.T;
  const double* temb = g.emb + (size_t)seq * g.T * F;
  double* ec = g.ec + (size_t)seq * g.D * g.T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w & 1, wc = w >> 1;
  // staging: A 32 rows x 16 k (8 threads x 2 per row), B 64 rows x 16 k (4 threads x 4)
  const int ar = tid >> 3, aq = (tid & 7) * 2, br = tid >> 2, bq = (tid & 3) * 4;
  const int nk = (F + EC_KC - 1) / EC_KC;
  const bool a_ok = d0 + ar < nd, b_ok = t0 + br < nt;
  const double* ap = embs + (size_t)(r0 + (a_ok ? d0 + ar : 0)) * F + aq;
  const double* bp = temb + (size_t)(b_ok ? order[t0 + br] : 0) * F + bq;
  double ra[EC_PF][2], rb[EC_PF][4];
  auto load = [&](int sl, int kc) {
    const int k0 = kc * EC_KC;
#pragma unroll
    for (int j = 0; j < 2; j++) ra[sl][j] = (a_ok && k0 + aq + j < F) ? ap[k0 + j] : 0.0;
#pragma unroll
    for (int j = 0; j < 4; j++) rb[sl][j] = (b_ok && k0 + bq + j < F) ? bp[k0 + j] : 0.0;
  };
  auto store = [&](int sl, double* buf) {
#pragma unroll
    for (int j = 0; j < 2; j++) buf[(aq + j) * EC_LDA + ar] = ra[sl][j];
#pragma unroll
    for (int j = 0; j < 4; j++) buf[EC_KC * EC_LDA + (bq + j) * EC_LDB + br] = rb[sl][j];
  };
  d4 acc[2];
  acc[0] = (d4){0.0, 0.0, 0.0, 0.0};
  acc[1] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < EC_PF; p++)
    if (p < nk) load(p, p);
  store(0, lds);
  __syncthreads();
  // chunk kc sits in LDS stage kc & 1 and register slot kc % EC_PF (free once stored); the loop
  // is unrolled by EC_PF so the slots are static
  for (int kb = 0; kb < nk; kb += EC_PF) {
#pragma unroll
    for (int u = 0; u < EC_PF; u++) {
      const int kc = kb + u;
      if (kc < nk) {
        if (kc + EC_PF < nk) load(u, kc + EC_PF);
        const double* cur = lds + (kc & 1) * EC_STAGE;
#pragma unroll
        for (int ks = 0; ks < EC_KC / 4; ks++) {
          const int kr = ks * 4 + (lane >> 4);
          const double a = cur[kr * EC_LDA + wr * 16 + (lane & 15)];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const double bb = cur[EC_KC * EC_LDA + kr * EC_LDB + wc * 32 + j * 16 + (lane & 15)];
            acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc[j], 0, 0, 0);
          }
        }
        if (kc + 1 < nk) store((u + 1) % EC_PF, lds + ((kc + 1) & 1) * EC_STAGE);
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const int col = t0 + wc * 32 + j * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int row = d0 + wr * 16 + (lane >> 4) + 4 * q;
      if (row < nd && col < nt) ec[(size_t)row * g.T + col] = acc[j][q];
    }
  }
}

// update_emb (boosttrack.py:117-119) / the newborn's emb = its detection's row; wave per record
__global__ void __launch_bounds__(256)
    boost_feature_kernel(BstDev g, int seq0, const double* __restrict__ embs) {
  const int b = blockIdx.y, seq = seq0 + b;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nrec = g.seqst[(size_t)seq * SQB + SB_NREC];
  if (k >= nrec) return;  // whole waves leave together
  const int F = g.F;
  const int slot = g.rec[((size_t)seq * g.D + k) * 2], row = g.rec[((size_t)seq * g.D + k) * 2 + 1];
  const double alpha = g.rec_a[(size_t)seq * g.D + k];
  double* e = g.emb + ((size_t)seq * g.T + slot) * F;
  const double* x = embs + (size_t)row * F;
  if (alpha < 0.0) {
    for (int q = lane; q < F; q += 64) e[q] = x[q];
    return;
  }
  const double om = 1 - alpha;
  constexpr int EQ = 8;
  if (F <= 64 * EQ) {  // the row in registers: one read of each input, one write of the result
    double v[EQ];
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < EQ; r++) {
      const int q = lane + 64 * r;
      v[r] = q < F ? alpha * e[q] + om * x[q] : 0.0;
      if (q < F) s += v[r] * v[r];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    const double nrm = sqrt(s);
#pragma unroll
    for (int r = 0; r < EQ; r++) {
      const int q = lane + 64 * r;
      if (q < F) e[q] = v[r] / nrm;
    }
    return;
  }
  double s = 0.0;
  for (int q = lane; q < F; q += 64) {
    const double v = alpha * e[q] + om * x[q];
    e[q] = v;
    s += v * v;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
  const double nrm = sqrt(s);
  for (int q = lane; q < F; q += 64) e[q] = e[q] / nrm;
}

__global__ void boost_reset_kernel(BstDev g, int seq0, int nseq) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nseq * SQB) g.seqst[(size_t)seq0 * SQB + k] = 0;
}

// Op-level BoostTrack filter (bx_kf_boost_*) with the frame kernel's octet code: op 0 initiate
// (kalmanfilter.py:47-73 from z = convert_bbox_to_z), 1 predict (:75-107), 2 update (:127-157).
__global__ __launch_bounds__(256) void kf_boost_kernel(int op, int n, double* __restrict__ x,
                                                       double* __restrict__ P,
                                                       const double* __restrict__ z) {
  const int gt = blockIdx.x * 256 + threadIdx.x;
  const int k = gt >> 3, r = gt & 7;
  if (k >= n) return;  // whole octets leave together
  double* xk = x + 8 * (size_t)k;
  double* Pk = P + 64 * (size_t)k;
  if (op == 0) {
    xk[r] = r < 4 ? z[4 * (size_t)k + r] : 0.0;
    for (int j = 0; j < 8; j++) Pk[8 * r + j] = j == r ? (r < 4 ? 10.0 : 10000.0) : 0.0;
    return;
  }
  double xr = xk[r], Pr[8];
  for (int j = 0; j < 8; j++) Pr[j] = Pk[8 * r + j];
  if (op == 1) {
    okf_predict(r, xr, Pr);
  } else {
    const double* zk = z + 4 * (size_t)k;
    const double zz[4] = {zk[0], zk[1], zk[2], zk[3]};
    okf_update(r, xr, Pr, zz);
  }
  xk[r] = xr;
  for (int j = 0; j < 8; j++) Pk[8 * r + j] = Pr[j];
}

// get_mh_dist_matrix (boosttrack.py:356-369): thread per (detection, track); the same sum order
// as the frame kernel's mh_dist (numpy's in-order 4-term sum)
__global__ __launch_bounds__(256) void kf_boost_mh_kernel(int nd, const double* __restrict__ dets,
                                                          int nt, const double* __restrict__ x,
                                                          const double* __restrict__ P,
                                                          double* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)nd * nt) return;
  const int d = (int)(i / nt), t = (int)(i % nt);
  double z[4];
  bbox_to_z(dets + 4 * (size_t)d, z);
  double s = 0.0;
  for (int q = 0; q < 4; q++) {
    const double v = z[q] - x[8 * (size_t)t + q];
    s += v * v * (1.0 / P[64 * (size_t)t + 9 * q]);
  }
  out[i] = s;
}

}  // namespace

// per_class: the frame counter is held across a frame's class calls (basetracker.py:177,186:
// `self.frame_count = frame_count` before every class's update) — saved by the first call
__global__ void boost_hold_frame_kernel(int* seqst, int s, int* hold, int first) {
  int* f = seqst + (size_t)s * SQB + SB_FRAME;
  if (first) hold[0] = *f;
  *f = hold[0];
}

struct bx_boost {
  BstDev dev;
  bx_boost_config cfg;
  void* arena = nullptr;
  size_t lds = 0;
  // host-path staging
  float* h_dets = nullptr;
  int* h_off = nullptr;
  double* h_embs = nullptr;
  double* h_warp = nullptr;
  double* h_out = nullptr;
  int* h_cnt = nullptr;
  // pinned mirrors for update_host (asynchronous copies, one sync per frame) and the counters
  // row of the last update_host sequence (bx_boost_counters_host answers from it)
  float* p_dets = nullptr;
  double* p_embs = nullptr;
  double* p_warp = nullptr;
  double* p_out = nullptr;
  int* p_cnt = nullptr;
  int* p_sq = nullptr;
  int cache_seq = -1;
  // per_class host path (bx_boost_update_classes_host): class offsets [C][2], counts [C], the
  // held frame counter
  int n_classes = 0;
  int* h_coff = nullptr;
  int* h_ccnt = nullptr;
  int* h_hold = nullptr;
  double* h_cwarp = nullptr;  // [C][6] the class calls' warps
  // timing probe
  int probe_stage = -1;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  int ev_used = 0;
};

#define BCHK(x)                                                                    \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess)                                                          \
      return bx_record_error(BX_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

static int probe_begin(bx_boost* e, int stage, hipStream_t st) {
  if (e->probe_stage != stage) return BX_OK;
  if (e->ev_used == (int)e->ev.size()) {
    hipEvent_t a, b;
    BCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
    BCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    e->ev.push_back({a, b});
  }
  BCHK(hipEventRecord(e->ev[e->ev_used].first, st));
  return BX_OK;
}

static int probe_end(bx_boost* e, int stage, hipStream_t st) {
  if (e->probe_stage != stage) return BX_OK;
  BCHK(hipEventRecord(e->ev[e->ev_used++].second, st));
  return BX_OK;
}

static int launch(bx_boost* e, int seq0, int nseq, const float* dets, const int* off,
                  const double* embs, const double* warps, double* out, int* cnt, hipStream_t st) {
  const BstDev& d = e->dev;
  int rc;
  if (d.reid) {
    if (!embs) return bx_record_error(BX_ERR_SHAPE, "with_reid BoostTrack needs embeddings");
    if ((rc = probe_begin(e, 0, st))) return rc;
    hipLaunchKernelGGL(boost_embcost_kernel, dim3(nseq, ec_tiles(d.D, d.T)), dim3(256), 0, st, d,
                       seq0, off, embs);
    BCHK(hipGetLastError());
    if ((rc = probe_end(e, 0, st))) return rc;
  }
  if ((rc = probe_begin(e, 1, st))) return rc;
  hipLaunchKernelGGL(boost_frame_kernel, dim3(nseq), dim3(frame_threads(nseq)), e->lds, st, d, seq0, dets, off,
                     d.use_ecc ? warps : nullptr, out, cnt);
  BCHK(hipGetLastError());
  if ((rc = probe_end(e, 1, st))) return rc;
  if (d.reid) {
    if ((rc = probe_begin(e, 2, st))) return rc;
    hipLaunchKernelGGL(boost_feature_kernel, dim3((d.D + 3) / 4, nseq), dim3(256), 0, st, d, seq0,
                       embs);
    BCHK(hipGetLastError());
    if ((rc = probe_end(e, 2, st))) return rc;
  }
  return BX_OK;
}

extern "C" {

int bx_boost_create(const bx_boost_config* c, bx_boost** out) {
  if (!c || !out) return bx_record_error(BX_ERR_INVALID, "null argument");
  if (c->n_seq <= 0 || c->track_cap <= 0 || c->det_cap <= 0 || c->track_cap > 512 ||
      c->det_cap > 512 || c->max_age < 0 || c->max_age > 100000)
    return bx_record_error(BX_ERR_INVALID, "n_seq/track_cap/det_cap/max_age out of range");
  if (c->with_reid && (c->emb_dim <= 0 || c->emb_dim > 16384))
    return bx_record_error(BX_ERR_INVALID, "with_reid needs 0 < emb_dim <= 16384");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0)
    return bx_record_error(BX_ERR_NO_DEVICE, "no HIP device visible");
  bx_boost* e = new bx_boost();
  e->cfg = *c;
  BstDev& d = e->dev;
  d.S = c->n_seq;
  d.T = c->track_cap;
  d.D = c->det_cap;
  d.N = d.T > d.D ? d.T : d.D;
  d.reid = c->with_reid ? 1 : 0;
  d.F = d.reid ? c->emb_dim : 0;
  d.det_thresh = c->det_thresh;
  d.iou_thr = c->iou_threshold;
  d.min_box_area = c->min_box_area;
  d.ar_thresh = c->aspect_ratio_thresh;
  d.l_iou = c->lambda_iou;
  d.l_mhd = c->lambda_mhd;
  d.l_shape = c->lambda_shape;
  d.dlo_coef = c->dlo_boost_coef;
  d.max_age = c->max_age;
  d.min_hits = c->min_hits;
  d.use_ecc = c->use_ecc != 0;
  d.use_dlo = c->use_dlo_boost != 0;
  d.use_duo = c->use_duo_boost != 0;
  d.s_sim_corr = c->s_sim_corr != 0;
  d.rich_s = c->use_rich_s != 0;
  d.use_sb = c->use_sb != 0;
  d.use_vt = c->use_vt != 0;
  // LDS: the fixed part plus as much cost matrix as keeps every sequence's workgroup resident
  // at once (256 CUs; at least 40 KB, i.e. 4 workgroups per CU, at most 152 KB)
  long cap = 160L * 1024 / ((d.S + 255) / 256);
  if (cap > 152L * 1024) cap = 152L * 1024;
  if (cap < 40L * 1024) cap = 40L * 1024;
  // the frame's track rows in LDS too when the cap leaves room for them beside the cost matrix
  // (up to 512 sequences: cap >= 80 KB)
  d.tb_lds = 0;
  size_t fixed = lds_bytes(d.D, d.T, d.N, 0, 0);
  if (d.S <= 512 && (long)(fixed + (size_t)d.T * TBB * 8) + 64 * 8 <= cap) {
    d.tb_lds = 1;
    fixed = lds_bytes(d.D, d.T, d.N, 0, 1);
  }
  long budget = cap - (long)fixed;
  int cl = budget > 0 ? (int)(budget / 8) : 0;
  if (cl > d.D * d.T) cl = d.D * d.T;
  if (cl < 64) cl = 64;
  d.cost_lds = cl;
  e->lds = lds_bytes(d.D, d.T, d.N, cl, d.tb_lds);
  if (e->lds > 160 * 1024) {
    delete e;
    return bx_record_error(BX_ERR_INVALID, "track_cap/det_cap too large for one workgroup's LDS");
  }
  const bool need_g = (long)d.D * d.T > cl;
  // get_confidence table: 0.9 ** k for k <= max_age + 1 (a track is dropped once its
  // time_since_update exceeds max_age), from the host's libm pow like Python's float pow
  d.ntab = c->max_age + 8;
  std::vector<double> tab(d.ntab);
  for (int k = 0; k < d.ntab; k++) tab[k] = std::pow(0.9, (double)k);
  const size_t S = d.S, T = d.T, D = d.D, F = d.F;
  size_t off = 0;
  auto carve_b = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_trk = carve_b(S * T * sizeof(BstTrk));
  const size_t o_sq = carve_b(S * SQB * sizeof(int));
  const size_t o_ord = carve_b(S * T * sizeof(int));
  const size_t o_tb = carve_b(S * T * TBB * sizeof(double));
  const size_t o_cg = need_g ? carve_b(S * D * T * sizeof(double)) : 0;
  // the DLO numerators spill only with use_dlo && rich_s (boost_frame_kernel's E staging)
  const bool need_eg = need_g && d.use_dlo && d.rich_s;
  const size_t o_eg = need_eg ? carve_b(S * D * T * sizeof(double)) : 0;
  const size_t o_ec = d.reid ? carve_b(S * D * T * sizeof(double)) : 0;
  const size_t o_emb = d.reid ? carve_b(S * T * F * sizeof(double)) : 0;
  const size_t o_rec = d.reid ? carve_b(S * D * 2 * sizeof(int)) : 0;
  const size_t o_reca = d.reid ? carve_b(S * D * sizeof(double)) : 0;
  const size_t o_tab = carve_b(tab.size() * sizeof(double));
  const size_t o_st = carve_b(sizeof(int) * 4);
#ifdef BX_PHASE_TIMING
  const size_t o_dbg = carve_b(S * BST_DBG * sizeof(unsigned long long));
#endif
  if (hipMalloc(&e->arena, off) != hipSuccess) {
    delete e;
    return bx_record_error(BX_ERR_HIP, "hipMalloc of the BoostTrack arena failed");
  }
  BCHK(hipMemset(e->arena, 0, off));
  char* base = (char*)e->arena;
  d.trk = (BstTrk*)(base + o_trk);
  d.seqst = (int*)(base + o_sq);
  d.order = (int*)(base + o_ord);
  d.tb = (double*)(base + o_tb);
  d.cost_g = need_g ? (double*)(base + o_cg) : nullptr;
  d.e_g = need_eg ? (double*)(base + o_eg) : nullptr;
  d.ec = d.reid ? (double*)(base + o_ec) : nullptr;
  d.emb = d.reid ? (double*)(base + o_emb) : nullptr;
  d.rec = d.reid ? (int*)(base + o_rec) : nullptr;
  d.rec_a = d.reid ? (double*)(base + o_reca) : nullptr;
  d.conf_tab = (const double*)(base + o_tab);
  d.status = (int*)(base + o_st);
#ifdef BX_PHASE_TIMING
  d.dbg = (unsigned long long*)(base + o_dbg);
#else
  d.dbg = nullptr;
#endif
  BCHK(hipMemcpy(base + o_tab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
  BCHK(bx_lds_attr((const void*)boost_frame_kernel, e->lds));
  BCHK(hipMalloc(&e->h_dets, sizeof(float) * 6 * D));
  BCHK(hipMalloc(&e->h_off, sizeof(int) * 2));
  if (d.reid) BCHK(hipMalloc(&e->h_embs, sizeof(double) * D * F));
  BCHK(hipMalloc(&e->h_warp, sizeof(double) * 6));
  BCHK(hipMalloc(&e->h_out, sizeof(double) * 8 * D));
  BCHK(hipMalloc(&e->h_cnt, sizeof(int)));
  BCHK(hipHostMalloc(&e->p_dets, sizeof(float) * 6 * d.D));
  BCHK(hipHostMalloc(&e->p_embs, sizeof(double) * (size_t)d.D * (d.F ? d.F : 1)));
  BCHK(hipHostMalloc(&e->p_warp, sizeof(double) * 8));
  BCHK(hipHostMalloc(&e->p_out, sizeof(double) * 8 * d.D));
  BCHK(hipHostMalloc(&e->p_cnt, sizeof(int) * 4));
  BCHK(hipHostMalloc(&e->p_sq, sizeof(int) * SQB));
  *out = e;
  return BX_OK;
}

int bx_boost_copy_state(bx_boost* dst, bx_boost* src) {
  if (!dst || !src) return bx_record_error(BX_ERR_INVALID, "null engine");
  const BstDev &a = src->dev, &b = dst->dev;
  if (a.S != b.S || a.reid != b.reid || a.F != b.F || b.T < a.T || b.D < a.D)
    return bx_record_error(BX_ERR_INVALID, "bx_boost_copy_state: destination must match the "
                                           "source's sequences and ReID and have at least its "
                                           "capacities");
  BCHK(hipDeviceSynchronize());
  const size_t S = a.S, Ta = a.T, Tb = b.T, F = a.F;
  BCHK(hipMemcpy2D(b.trk, Tb * sizeof(BstTrk), a.trk, Ta * sizeof(BstTrk), Ta * sizeof(BstTrk), S,
                   hipMemcpyDeviceToDevice));
  BCHK(hipMemcpy2D(b.order, Tb * sizeof(int), a.order, Ta * sizeof(int), Ta * sizeof(int), S,
                   hipMemcpyDeviceToDevice));
  if (a.reid && F)
    BCHK(hipMemcpy2D(b.emb, Tb * F * sizeof(double), a.emb, Ta * F * sizeof(double),
                     Ta * F * sizeof(double), S, hipMemcpyDeviceToDevice));
  BCHK(hipMemcpy(b.seqst, a.seqst, S * SQB * sizeof(int), hipMemcpyDeviceToDevice));
  BCHK(hipMemcpy(b.status, a.status, 4 * sizeof(int), hipMemcpyDeviceToDevice));
  dst->cache_seq = -1;
  BCHK(hipDeviceSynchronize());
  return BX_OK;
}

int bx_boost_destroy(bx_boost* e) {
  if (!e) return BX_OK;
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
  (void)hipFree(e->h_coff);
  (void)hipFree(e->h_ccnt);
  (void)hipFree(e->h_hold);
  (void)hipFree(e->h_cwarp);
  delete e;
  return BX_OK;
}

int bx_boost_reset(bx_boost* e, int seq0, int nseq, void* stream) {
  if (!e || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad sequence range");
  if (!nseq) return BX_OK;
  e->cache_seq = -1;
  hipLaunchKernelGGL(boost_reset_kernel, dim3((nseq * SQB + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, e->dev, seq0, nseq);
  BCHK(hipGetLastError());
  return BX_OK;
}

int bx_boost_step(bx_boost* e, int seq0, int nseq, const float* dets, const int32_t* det_off,
                  const double* embs, const double* warps, double* out, int32_t* out_count,
                  void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_step");
  e->cache_seq = -1;
  return launch(e, seq0, nseq, dets, det_off, embs, warps, out, out_count, (hipStream_t)stream);
}

int bx_boost_update_host(bx_boost* e, int seq, const float* dets, int n, const double* embs,
                         const double* warp, double* out, int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && (!dets || !out)) || !n_out)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_update_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  if (e->dev.reid && n && !embs)
    return bx_record_error(BX_ERR_SHAPE, "with_reid BoostTrack needs embeddings");
  hipStream_t st = (hipStream_t)stream;
  // pinned mirrors: asynchronous copies in, the frame, rows (at most n) + count + status +
  // counters back, one synchronisation
  if (n) {
    memcpy(e->p_dets, dets, sizeof(float) * 6 * n);
    BCHK(hipMemcpyAsync(e->h_dets, e->p_dets, sizeof(float) * 6 * n, hipMemcpyHostToDevice, st));
  }
  if (n && e->dev.reid) {
    memcpy(e->p_embs, embs, sizeof(double) * (size_t)n * e->dev.F);
    BCHK(hipMemcpyAsync(e->h_embs, e->p_embs, sizeof(double) * (size_t)n * e->dev.F,
                        hipMemcpyHostToDevice, st));
  }
  if (warp) {
    memcpy(e->p_warp, warp, sizeof(double) * 6);
    BCHK(hipMemcpyAsync(e->h_warp, e->p_warp, sizeof(double) * 6, hipMemcpyHostToDevice, st));
  }
  e->p_cnt[2] = 0;
  e->p_cnt[3] = n;
  BCHK(hipMemcpyAsync(e->h_off, e->p_cnt + 2, sizeof(int) * 2, hipMemcpyHostToDevice, st));
  e->cache_seq = -1;
  int rc = launch(e, seq, 1, e->h_dets, e->h_off, e->dev.reid ? e->h_embs : nullptr,
                  warp ? e->h_warp : nullptr, e->h_out, e->h_cnt, st);
  if (rc) return rc;
  BCHK(hipMemcpyAsync(e->p_cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  BCHK(hipMemcpyAsync(e->p_cnt + 1, e->dev.status, sizeof(int), hipMemcpyDeviceToHost, st));
  if (n) BCHK(hipMemcpyAsync(e->p_out, e->h_out, sizeof(double) * 8 * n, hipMemcpyDeviceToHost, st));
  BCHK(hipMemcpyAsync(e->p_sq, e->dev.seqst + (size_t)seq * SQB, sizeof(int) * SQB,
                      hipMemcpyDeviceToHost, st));
  BCHK(hipStreamSynchronize(st));
  const int cnt = e->p_cnt[0], status = e->p_cnt[1];
  e->cache_seq = seq;
  if (cnt) memcpy(out, e->p_out, sizeof(double) * 8 * cnt);
  *n_out = cnt;
  if (status)
    return bx_record_error(status, status == BX_ERR_CAPACITY ? "detections exceed det_cap"
                                                             : "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

// per_class=True (basetracker.py:155-201) for one sequence: BoostTrack keeps its `trackers`
// list outside active_tracks, so the decorator's swap does not isolate the classes:
// every class call predicts, associates and ages ALL tracks against that class's detections.
// Restated as one engine sequence stepped once per class id 0..C-1 with the frame counter held;
// rows stacked in class order, det_ind indexing the class's subset.  One sync at the end.
int bx_boost_update_classes_host(bx_boost* e, int seq, const float* dets, int n,
                                 const double* embs, const double* warps, int n_classes,
                                 double* out, int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !dets) || !n_out || n_classes <= 0 ||
      n_classes > 4096)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_update_classes_host");
  if (n > e->dev.D) return bx_record_error(BX_ERR_CAPACITY, "detections exceed det_cap");
  const bool reid = e->dev.reid;
  if (reid && n && !embs) return bx_record_error(BX_ERR_SHAPE, "with_reid BoostTrack needs embeddings");
  hipStream_t st = (hipStream_t)stream;
  const int C = n_classes, F = e->dev.F;
  if (e->n_classes && e->n_classes != C)
    return bx_record_error(BX_ERR_INVALID, "n_classes differs from the engine's first per-class call");
  e->cache_seq = -1;
  if (!e->n_classes) {
    e->n_classes = C;
    BCHK(hipMalloc(&e->h_coff, sizeof(int) * 2 * C));
    BCHK(hipMalloc(&e->h_ccnt, sizeof(int) * C));
    BCHK(hipMalloc(&e->h_hold, sizeof(int)));
    BCHK(hipMalloc(&e->h_cwarp, sizeof(double) * 6 * C));
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
  std::vector<double> he(reid ? (size_t)(m ? m : 1) * F : 1);
  for (int i = 0; i < n; i++) {
    const int c = cls_of(i);
    if (c < 0) continue;
    const int k = fill[c]++;
    memcpy(&hd[6 * (size_t)k], dets + 6 * (size_t)i, 6 * sizeof(float));
    if (reid) memcpy(&he[(size_t)F * k], embs + (size_t)F * i, sizeof(double) * F);
  }
  std::vector<int> hoff(2 * C);
  for (int c = 0; c < C; c++) { hoff[2 * c] = 0; hoff[2 * c + 1] = cnt[c + 1] - cnt[c]; }
  if (m) BCHK(hipMemcpyAsync(e->h_dets, hd.data(), sizeof(float) * 6 * m, hipMemcpyHostToDevice, st));
  if (m && reid)
    BCHK(hipMemcpyAsync(e->h_embs, he.data(), sizeof(double) * (size_t)m * F, hipMemcpyHostToDevice, st));
  BCHK(hipMemcpyAsync(e->h_coff, hoff.data(), sizeof(int) * 2 * C, hipMemcpyHostToDevice, st));
  if (warps) BCHK(hipMemcpyAsync(e->h_cwarp, warps, sizeof(double) * 6 * C, hipMemcpyHostToDevice, st));
  for (int c = 0; c < C; c++) {
    hipLaunchKernelGGL(boost_hold_frame_kernel, dim3(1), dim3(1), 0, st, e->dev.seqst, seq,
                       e->h_hold, c == 0 ? 1 : 0);
    BCHK(hipGetLastError());
    // class call c's camera_update warp (boosttrack.py:243-246 runs cmc.apply per class call)
    const double* wc = warps ? e->h_cwarp + 6 * (size_t)c : nullptr;
    int rc = launch(e, seq, 1, e->h_dets + 6 * (size_t)cnt[c], e->h_coff + 2 * c,
                    reid ? e->h_embs + (size_t)F * cnt[c] : nullptr, wc,
                    e->h_out + 8 * (size_t)cnt[c], e->h_ccnt + c, st);
    if (rc) return rc;
  }
  std::vector<int> oc(C);
  std::vector<double> ho((size_t)8 * (m ? m : 1));
  BCHK(hipMemcpyAsync(oc.data(), e->h_ccnt, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  if (m) BCHK(hipMemcpyAsync(ho.data(), e->h_out, sizeof(double) * 8 * m, hipMemcpyDeviceToHost, st));
  BCHK(hipStreamSynchronize(st));
  int k = 0;
  for (int c = 0; c < C; c++)
    for (int j = 0; j < oc[c]; j++, k++)
      if (out) memcpy(out + 8 * (size_t)k, &ho[8 * ((size_t)cnt[c] + j)], 8 * sizeof(double));
  *n_out = k;
  int status = 0;
  BCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status)
    return bx_record_error(status, status == BX_ERR_CAPACITY ? "detections exceed det_cap"
                                                             : "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

int bx_kf_boost_initiate(int n, const double* z, double* x, double* P, void* stream) {
  if (n < 0 || (n && (!z || !x || !P))) return bx_record_error(BX_ERR_INVALID, "bad arguments");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_boost_kernel, dim3((8 * n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     0, n, x, P, z);
  BCHK(hipGetLastError());
  return BX_OK;
}
int bx_kf_boost_predict(int n, double* x, double* P, void* stream) {
  if (n < 0 || (n && (!x || !P))) return bx_record_error(BX_ERR_INVALID, "bad arguments");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_boost_kernel, dim3((8 * n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     1, n, x, P, (const double*)nullptr);
  BCHK(hipGetLastError());
  return BX_OK;
}
int bx_kf_boost_update(int n, double* x, double* P, const double* z, void* stream) {
  if (n < 0 || (n && (!z || !x || !P))) return bx_record_error(BX_ERR_INVALID, "bad arguments");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_boost_kernel, dim3((8 * n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     2, n, x, P, z);
  BCHK(hipGetLastError());
  return BX_OK;
}
int bx_kf_boost_mh_dist(int nd, const double* dets, int nt, const double* x, const double* P,
                        double* out, void* stream) {
  if (nd < 0 || nt < 0 || ((size_t)nd * nt && (!dets || !x || !P || !out)))
    return bx_record_error(BX_ERR_INVALID, "bad arguments");
  const size_t m = (size_t)nd * nt;
  if (!m) return BX_OK;
  hipLaunchKernelGGL(kf_boost_mh_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, nd, dets, nt, x, P, out);
  BCHK(hipGetLastError());
  return BX_OK;
}

int bx_boost_status(bx_boost* e, int* status) {
  if (!e || !status) return bx_record_error(BX_ERR_INVALID, "null argument");
  BCHK(hipMemcpy(status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  return BX_OK;
}

int bx_boost_counters_host(bx_boost* e, int seq, int* frame_count, int* id_count, int* n_tracks) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  int s[SQB];
  if (seq == e->cache_seq) {
    memcpy(s, e->p_sq, sizeof(s));
  } else {
    BCHK(hipDeviceSynchronize());
    BCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQB, sizeof(s), hipMemcpyDeviceToHost));
  }
  if (frame_count) *frame_count = s[SB_FRAME];
  if (id_count) *id_count = s[SB_IDS];
  if (n_tracks) *n_tracks = s[SB_NTR];
  return BX_OK;
}

int bx_boost_set_id_count(bx_boost* e, int seq, int id_count, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S) return bx_record_error(BX_ERR_INVALID, "bad sequence");
  e->cache_seq = -1;
  BCHK(hipMemcpyAsync(e->dev.seqst + (size_t)seq * SQB + SB_IDS, &id_count, sizeof(int),
                      hipMemcpyHostToDevice, (hipStream_t)stream));
  BCHK(hipStreamSynchronize((hipStream_t)stream));
  return BX_OK;
}

int bx_boost_tracks_host(bx_boost* e, int seq, int cap, int32_t* ids, double* x, double* p,
                         double* emb, int* n) {
  if (!e || seq < 0 || seq >= e->dev.S || cap < 0 || !n)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_tracks_host");
  BCHK(hipDeviceSynchronize());
  int s[SQB];
  BCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQB, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[SB_NTR];
  std::vector<int> ord(nt);
  if (nt)
    BCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int k = 0; k < nt && k < cap; k++) {
    BstTrk t;
    BCHK(hipMemcpy(&t, e->dev.trk + (size_t)seq * e->dev.T + ord[k], sizeof(BstTrk),
                   hipMemcpyDeviceToHost));
    if (ids) ids[k] = t.id;
    if (x) memcpy(x + 8 * k, t.x, sizeof(t.x));
    if (p) memcpy(p + 64 * k, t.P, sizeof(t.P));
    if (emb && e->dev.reid)
      BCHK(hipMemcpy(emb + (size_t)k * e->dev.F,
                     e->dev.emb + ((size_t)seq * e->dev.T + ord[k]) * e->dev.F,
                     sizeof(double) * e->dev.F, hipMemcpyDeviceToHost));
  }
  *n = nt;
  return BX_OK;
}

int bx_boost_state_set_host(bx_boost* e, int seq, int n, const int32_t* ids, const double* x,
                            const double* p) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !ids))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_state_set_host");
  BCHK(hipDeviceSynchronize());
  int s[SQB];
  BCHK(hipMemcpy(s, e->dev.seqst + (size_t)seq * SQB, sizeof(s), hipMemcpyDeviceToHost));
  const int nt = s[SB_NTR];
  std::vector<int> ord(nt);
  if (nt)
    BCHK(hipMemcpy(ord.data(), e->dev.order + (size_t)seq * e->dev.T, sizeof(int) * nt,
                   hipMemcpyDeviceToHost));
  for (int j = 0; j < n; j++) {
    BstTrk* dt = nullptr;
    BstTrk t;
    for (int k = 0; k < nt && !dt; k++) {
      BstTrk* cand = e->dev.trk + (size_t)seq * e->dev.T + ord[k];
      BCHK(hipMemcpy(&t, cand, sizeof(BstTrk), hipMemcpyDeviceToHost));
      if (t.id == ids[j]) dt = cand;
    }
    if (!dt) return bx_record_error(BX_ERR_INVALID, "state_set: no live track with that id");
    if (x) memcpy(t.x, x + 8 * j, sizeof(t.x));
    if (p) memcpy(t.P, p + 64 * j, sizeof(t.P));
    BCHK(hipMemcpy(dt, &t, sizeof(BstTrk), hipMemcpyHostToDevice));
  }
  return BX_OK;
}

int bx_boost_frame_stats_host(bx_boost* e, int seq0, int nseq, int64_t* sums) {
  if (!e || !sums || seq0 < 0 || nseq < 0 || seq0 + nseq > e->dev.S)
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_boost_frame_stats_host");
  std::vector<int> s((size_t)nseq * SQB);
  BCHK(hipDeviceSynchronize());
  if (nseq)
    BCHK(hipMemcpy(s.data(), e->dev.seqst + (size_t)seq0 * SQB, sizeof(int) * s.size(),
                   hipMemcpyDeviceToHost));
  int64_t a[7] = {0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < nseq; k++) {
    const int* q = s.data() + (size_t)k * SQB;
    a[6] += (int64_t)q[SB_NDET] * q[SB_NT0];
    a[0] += q[SB_NDET];
    a[1] += q[SB_NKEEP];
    a[2] += q[SB_NT0];
    a[3] += q[SB_NOUT];
    a[4] += q[SB_NREC];
    a[5] = q[SB_FRAME] > a[5] ? q[SB_FRAME] : a[5];
  }
  for (int k = 0; k < 7; k++) sums[k] = a[k];
  return BX_OK;
}

// diagnostic (not in the public header): the phase stamps of every sequence, [S][BST_DBG]
int bx_boost_debug_host(bx_boost* e, unsigned long long* out) {
  if (!e || !out || !e->dev.dbg) return bx_record_error(BX_ERR_INVALID, "not a timing build");
  BCHK(hipDeviceSynchronize());
  BCHK(hipMemcpy(out, e->dev.dbg, sizeof(unsigned long long) * BST_DBG * e->dev.S,
                 hipMemcpyDeviceToHost));
  return BX_OK;
}

int bx_boost_probe(bx_boost* e, int stage) {
  if (!e) return bx_record_error(BX_ERR_INVALID, "null engine");
  e->probe_stage = stage;
  e->ev_used = 0;
  return BX_OK;
}

int bx_boost_probe_read(bx_boost* e, double* total_ms, int* count) {
  if (!e || !total_ms || !count) return bx_record_error(BX_ERR_INVALID, "null argument");
  double s = 0.0;
  for (int k = 0; k < e->ev_used; k++) {
    BCHK(hipEventSynchronize(e->ev[k].second));
    float ms = 0.f;
    BCHK(hipEventElapsedTime(&ms, e->ev[k].first, e->ev[k].second));
    s += ms;
  }
  *total_ms = s;
  *count = e->ev_used;
  e->ev_used = 0;
  return BX_OK;
}

}  // extern "C"
