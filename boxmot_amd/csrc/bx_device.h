// bx_device.h — device-side building blocks of the association engine (gfx950, wave64).
//
// All floating-point expressions restate the reference's numpy operation order one-for-one and
// the library is compiled with -ffp-contract=off, so every product/sum rounds exactly as numpy's
// (and as the C oracle's) do.  The Kalman update and the BLAS-ordered feature norms follow the
// oracle's fixed order (the reference's BLAS/LAPACK order is not pinned), making the GPU path
// bitwise identical to oracle/ and within ~1e-13 of the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace bx {

constexpr int WG = 256;  // threads per workgroup: 4 waves of 64
constexpr int WAVE = 64;
constexpr double INF = __builtin_huge_val();

// host: is a 2x3 row-major warp exactly the identity (what a static camera's CMC returns)?
inline bool is_identity_warp(const double* w) {
  return w[0] == 1.0 && w[1] == 0.0 && w[2] == 0.0 && w[3] == 0.0 && w[4] == 1.0 && w[5] == 0.0;
}

enum : int { KIND_BYTE = 0, KIND_BOT = 1 };
enum : uint32_t { ST_NEW = 0, ST_TRACKED = 1, ST_LOST = 2, ST_REMOVED = 3 };
// per-slot persistent flag word; F_INACT / F_INLOST: the slot is on the active / lost list
// (lets the slot-parallel kernels select joint(tracked, lost) without walking the lists)
// F_PRED / F_GMC / F_REC are frame-transient: mean predicted (covariance predict pending), CMC
// warp applied to the mean (covariance warp pending), slot has an update record this frame.
// F_PEND (bits 16-31, persistent): covariance predicts applied to the mean but not yet to the
// covariance — a track without an update keeps them pending until it is updated again (or its
// state is read), see bx_engine.hip K2/K4.
enum : uint32_t {
  F_STATE = 0x7u, F_ACT = 0x8u, F_INREM = 0x10u, F_INUSE = 0x20u, F_INACT = 0x40u,
  F_INLOST = 0x80u, F_PRED = 0x100u, F_GMC = 0x200u, F_REC = 0x400u, F_TRANSIENT = 0x700u,
  F_PARKED = 0x800u,  // per_class mode: on another class's (parked) active list — kept alive
  F_PEND1 = 0x10000u, F_PEND_MASK = 0xFFFF0000u
};

__device__ __forceinline__ uint32_t st_of(uint32_t f) { return f & F_STATE; }
__host__ __device__ __forceinline__ int pend_of(uint32_t f) { return (int)((f & F_PEND_MASK) >> 16); }

// ------------------------------------------------------------------------------------------
// utils/ops.py box conversions (numpy op order)
__device__ __forceinline__ void xyxy2xywh(const double* x, double* y) {
  double a = (x[0] + x[2]) / 2, b = (x[1] + x[3]) / 2, c = x[2] - x[0], d = x[3] - x[1];
  y[0] = a; y[1] = b; y[2] = c; y[3] = d;
}
__device__ __forceinline__ void xywh2xyxy(const double* x, double* y) {
  double a = x[0] - x[2] / 2, b = x[1] - x[3] / 2, c = x[0] + x[2] / 2, d = x[1] + x[3] / 2;
  y[0] = a; y[1] = b; y[2] = c; y[3] = d;
}
__device__ __forceinline__ void xywh2tlwh(const double* x, double* y) {
  double a = x[0] - x[2] / 2, b = x[1] - x[3] / 2, c = x[2], d = x[3];
  y[0] = a; y[1] = b; y[2] = c; y[3] = d;
}
__device__ __forceinline__ void tlwh2xyah(const double* x, double* y) {
  double a = x[0] + x[2] / 2, b = x[1] + x[3] / 2, c = x[2] / x[3], d = x[3];
  y[0] = a; y[1] = b; y[2] = c; y[3] = d;
}

// utils/iou.py:50-67 (no epsilon in the denominator)
__device__ __forceinline__ double iou_pair(const double* b1, const double* b2) {
  double xx1 = fmax(b1[0], b2[0]);
  double yy1 = fmax(b1[1], b2[1]);
  double xx2 = fmin(b1[2], b2[2]);
  double yy2 = fmin(b1[3], b2[3]);
  double w = fmax(0.0, xx2 - xx1);
  double h = fmax(0.0, yy2 - yy1);
  double wh = w * h;
  return wh / ((b1[2] - b1[0]) * (b1[3] - b1[1]) + (b2[2] - b2[0]) * (b2[3] - b2[1]) - wh);
}
// fdlibm s_atan.c (the algorithm oracle/bxo_ops.c restates as bxo_atan); within 1 ulp of
// np.arctan, bit-identical to the oracle.
__device__ inline double bx_atan(double x) {
  constexpr double hi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                            9.82793723247329054082e-01, 1.57079632679489655800e+00};
  constexpr double lo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                            1.39033110312309984516e-17, 6.12323399573676603587e-17};
  const int hx = __double2hiint(x);
  const int ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && __double2loint(x) != 0)) return x + x;
    return hx > 0 ? hi[3] + lo[3] : -hi[3] - lo[3];
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
    } else if (ix < 0x40038000) {
      id = 2;
      x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
      id = 3;
      x = -1.0 / x;
    }
  }
  const double z = x * x, w = z * z;
  const double s1 = z * (3.33333333333329318027e-01 +
                         w * (1.42857142725034663711e-01 +
                              w * (9.09088713343650656196e-02 +
                                   w * (6.66107313738753120669e-02 +
                                        w * (4.97687799461593236017e-02 + w * 1.62858201153657823623e-02)))));
  const double s2 = w * (-1.99999999998764832476e-01 +
                         w * (-1.11111104054623557880e-01 +
                              w * (-7.69187620504482999495e-02 +
                                   w * (-5.83357013379057348645e-02 + w * -3.65315727442169155270e-02))));
  if (id < 0) return x - x * (s1 + s2);
  const double r = hi[id] - ((x * (s1 + s2) - lo[id]) - x);
  return hx < 0 ? -r : r;
}

// AssociationFunction registry (utils/iou.py:79-346), numpy's operation order per mode.
// kind: 0 iou, 1 hmiou, 2 giou, 3 diou, 4 ciou, 5 centroid (frame size w, h).
enum { ASSO_IOU = 0, ASSO_HMIOU = 1, ASSO_GIOU = 2, ASSO_DIOU = 3, ASSO_CIOU = 4,
       ASSO_CENTROID = 5 };
__device__ inline double asso_pair(int kind, const double* a, const double* b, double fw,
                                   double fh) {
  if (kind == ASSO_IOU) return iou_pair(a, b);
  const double xx1 = fmax(a[0], b[0]), yy1 = fmax(a[1], b[1]);
  const double xx2 = fmin(a[2], b[2]), yy2 = fmin(a[3], b[3]);
  const double iw = fmax(0.0, xx2 - xx1), ih = fmax(0.0, yy2 - yy1);
  const double wh = iw * ih;
  const double area1 = (a[2] - a[0]) * (a[3] - a[1]), area2 = (b[2] - b[0]) * (b[3] - b[1]);
  const double ex = fmax(a[2], b[2]) - fmin(a[0], b[0]);  // enclosing box
  const double ey = fmax(a[3], b[3]) - fmin(a[1], b[1]);
  const double cx1 = (a[0] + a[2]) / 2.0, cy1 = (a[1] + a[3]) / 2.0;
  const double cx2 = (b[0] + b[2]) / 2.0, cy2 = (b[1] + b[3]) / 2.0;
  const double dx = cx1 - cx2, dy = cy1 - cy2;
  switch (kind) {
    case ASSO_HMIOU:  // :79-127
      return (wh / ((area1 + area2 - wh) + 1e-10)) * (ih / fmax(1e-10, ey));
    case ASSO_GIOU: {  // :129-169
      const double uni = area1 + area2 - wh;
      const double enc = ex * ey;
      return ((wh / uni - (enc - uni) / enc) + 1.0) / 2.0;
    }
    case ASSO_DIOU:  // :266-307
      return ((wh / (area1 + area2 - wh) - (dx * dx + dy * dy) / (ex * ex + ey * ey)) + 1) / 2.0;
    case ASSO_CIOU: {  // :199-264
      const double eps = 1e-7;
      const double iou = wh / (((area1 + area2) - wh) + eps);
      const double outer = (ex * ex + ey * ey) + eps;
      const double h1 = (a[3] - a[1]) + eps, h2 = (b[3] - b[1]) + eps;
      const double d = bx_atan((b[2] - b[0]) / h2) - bx_atan((a[2] - a[0]) / h1);
      const double pi = 3.141592653589793;
      const double v = (4 / (pi * pi)) * (d * d);
      const double alpha = v / (((1 - iou) + v) + eps);
      return (((iou - (dx * dx + dy * dy) / outer) + alpha * v) + 1) / 2.0;
    }
    default:  // ASSO_CENTROID :171-184
      return 1 - sqrt(dx * dx + dy * dy) / sqrt(fw * fw + fh * fh);
  }
}
// Positive-area intersection.  A pair that fails this has IoU exactly 0 (cost 1 or 2 after
// fuse_score), which is never admissible for a cost_limit <= 1.
__device__ __forceinline__ bool boxes_intersect(const double* b1, const double* b2) {
  return fmin(b1[2], b2[2]) > fmax(b1[0], b2[0]) && fmin(b1[3], b2[3]) > fmax(b1[1], b2[1]);
}

// utils/matching.py:520-544 enhanced_fuse_score (fork semantics)
__device__ __forceinline__ double fuse_one(double cost, double conf) {
  double sim = 1 - cost;
  double w = conf > 0.7 ? conf * 1.2 : conf;
  double mask = conf >= 0.5 ? 1.0 : 0.0;
  double fuse = 1 - sim * w * mask;
  return conf < 0.5 ? fuse * 2.0 : fuse;
}

// ------------------------------------------------------------------------------------------
// Kalman filters (base_kalman_filter.py; xyah_kf.py / xywh_kf.py).  dt = 1.
constexpr double STD_POS = 1.0 / 20, STD_VEL = 1.0 / 160;

__device__ inline void kf_initiate(int kind, const double* m, double* mean, double* cov) {
  double std[8];
  if (kind == KIND_BYTE) {
    std[0] = 2 * STD_POS * m[3]; std[1] = 2 * STD_POS * m[3]; std[2] = 1e-2;
    std[3] = 2 * STD_POS * m[3]; std[4] = 10 * STD_VEL * m[3]; std[5] = 10 * STD_VEL * m[3];
    std[6] = 1e-5; std[7] = 10 * STD_VEL * m[3];
  } else {
    std[0] = 2 * STD_POS * m[2]; std[1] = 2 * STD_POS * m[3]; std[2] = 2 * STD_POS * m[2];
    std[3] = 2 * STD_POS * m[3]; std[4] = 10 * STD_VEL * m[2]; std[5] = 10 * STD_VEL * m[3];
    std[6] = 10 * STD_VEL * m[2]; std[7] = 10 * STD_VEL * m[3];
  }
  for (int k = 0; k < 4; k++) { mean[k] = m[k]; mean[4 + k] = 0.0; }
  for (int k = 0; k < 64; k++) cov[k] = 0.0;
  for (int k = 0; k < 8; k++) cov[9 * k] = std[k] * std[k];
}

__device__ inline void kf_process_noise(int kind, const double* mean, double* q) {
  double s[8];
  if (kind == KIND_BYTE) {
    s[0] = STD_POS * mean[3]; s[1] = STD_POS * mean[3]; s[2] = 1e-2; s[3] = STD_POS * mean[3];
    s[4] = STD_VEL * mean[3]; s[5] = STD_VEL * mean[3]; s[6] = 1e-5; s[7] = STD_VEL * mean[3];
  } else {
    s[0] = STD_POS * mean[2]; s[1] = STD_POS * mean[3]; s[2] = STD_POS * mean[2];
    s[3] = STD_POS * mean[3]; s[4] = STD_VEL * mean[2]; s[5] = STD_VEL * mean[3];
    s[6] = STD_VEL * mean[2]; s[7] = STD_VEL * mean[3];
  }
  for (int k = 0; k < 8; k++) q[k] = s[k] * s[k];
}

// multi_predict on one track held in an SoA slab: element e of track t at base[e*stride].
// F has two non-zero terms per row/col: cov' = (P_ij + P_i+4,j) + (P_i,j+4 + P_i+4,j+4) + Q.
__device__ inline void kf_predict_soa(int kind, double* mean, double* cov, int stride) {
  double m[8], q[8];
  for (int k = 0; k < 8; k++) m[k] = mean[k * stride];
  kf_process_noise(kind, m, q);
  for (int k = 0; k < 4; k++) mean[k * stride] = m[k] + m[k + 4];
  // row-pair (i, i+4) at a time keeps the live set to two rows
  for (int i = 0; i < 4; i++) {
    double r0[8], r1[8], f0[8];
    for (int j = 0; j < 8; j++) { r0[j] = cov[(8 * i + j) * stride]; r1[j] = cov[(8 * (i + 4) + j) * stride]; }
    for (int j = 0; j < 8; j++) f0[j] = r0[j] + r1[j];  // (F P) row i
    for (int j = 0; j < 8; j++) {
      double v0 = j < 4 ? f0[j] + f0[j + 4] : f0[j];
      double v1 = j < 4 ? r1[j] + r1[j + 4] : r1[j];  // (F P) row i+4 = P row i+4
      cov[(8 * i + j) * stride] = (i == j) ? v0 + q[i] : v0;
      cov[(8 * (i + 4) + j) * stride] = (i + 4 == j) ? v1 + q[i + 4] : v1;
    }
  }
}

__device__ inline void kf_meas_noise(int kind, const double* mean, double conf, double* r) {
  double s[4];
  if (kind == KIND_BYTE) {
    s[0] = STD_POS * mean[3]; s[1] = STD_POS * mean[3]; s[2] = 1e-1; s[3] = STD_POS * mean[3];
  } else {
    s[0] = STD_POS * mean[2]; s[1] = STD_POS * mean[3]; s[2] = STD_POS * mean[2];
    s[3] = STD_POS * mean[3];
  }
  for (int k = 0; k < 4; k++) { double v = (1 - conf) * s[k]; r[k] = v * v; }
}

__device__ inline bool chol4(const double* S, double* L) {
  for (int k = 0; k < 16; k++) L[k] = 0.0;
  for (int j = 0; j < 4; j++) {
    double d = S[4 * j + j];
    for (int k = 0; k < j; k++) d -= L[4 * j + k] * L[4 * j + k];
    if (!(d > 0.0)) return false;
    d = sqrt(d);
    L[4 * j + j] = d;
    for (int i = j + 1; i < 4; i++) {
      double s = S[4 * i + j];
      for (int k = 0; k < j; k++) s -= L[4 * i + k] * L[4 * j + k];
      L[4 * i + j] = s / d;
    }
  }
  return true;
}

// base_kalman_filter.py:129-155 on one SoA track (same loop order as oracle/bxo_ops.c).
__device__ inline void kf_update_soa(int kind, double* mean, double* cov, int stride,
                                     const double* z, double conf) {
  double m[8], S[16], L[16], K[32];
  for (int k = 0; k < 8; k++) m[k] = mean[k * stride];
  double r[4];
  kf_meas_noise(kind, m, conf, r);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) S[4 * i + j] = cov[(8 * i + j) * stride] + (i == j ? r[i] : 0.0);
  if (!chol4(S, L)) return;
  for (int c = 0; c < 8; c++) {
    double y[4], x[4];
    for (int i = 0; i < 4; i++) {
      double s = cov[(8 * c + i) * stride];
      for (int k = 0; k < i; k++) s -= L[4 * i + k] * y[k];
      y[i] = s / L[4 * i + i];
    }
    for (int i = 3; i >= 0; i--) {
      double s = y[i];
      for (int k = i + 1; k < 4; k++) s -= L[4 * k + i] * x[k];
      x[i] = s / L[4 * i + i];
    }
    for (int i = 0; i < 4; i++) K[4 * c + i] = x[i];
  }
  double innov[4];
  for (int k = 0; k < 4; k++) innov[k] = z[k] - m[k];
  for (int i = 0; i < 8; i++) {
    double s = 0.0;
    for (int k = 0; k < 4; k++) s += innov[k] * K[4 * i + k];
    mean[i * stride] = m[i] + s;
  }
  for (int i = 0; i < 8; i++) {
    double ks[4];
    for (int j = 0; j < 4; j++) {
      double s = 0.0;
      for (int k = 0; k < 4; k++) s += K[4 * i + k] * S[4 * k + j];
      ks[j] = s;
    }
    for (int j = 0; j < 8; j++) {
      double s = 0.0;
      for (int k = 0; k < 4; k++) s += ks[k] * K[4 * j + k];
      cov[(8 * i + j) * stride] = cov[(8 * i + j) * stride] - s;
    }
  }
}

// base_kalman_filter.py:166-194 (maha, 4 dims) for one state vs nz measurements
__device__ inline void kf_gating_soa(int kind, const double* mean, const double* cov, int stride,
                                     const double* z, int nz, double* out) {
  double m[8], S[16], L[16], r[4];
  for (int k = 0; k < 8; k++) m[k] = mean[k * stride];
  kf_meas_noise(kind, m, 0.0, r);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) S[4 * i + j] = cov[(8 * i + j) * stride] + (i == j ? r[i] : 0.0);
  bool ok = chol4(S, L);
  for (int q = 0; q < nz; q++) {
    if (!ok) { out[q] = __builtin_nan(""); continue; }
    double d[4], y[4], s2 = 0.0;
    for (int i = 0; i < 4; i++) d[i] = z[4 * q + i] - m[i];
    for (int i = 0; i < 4; i++) {
      double s = d[i];
      for (int j = 0; j < i; j++) s -= L[4 * i + j] * y[j];
      y[i] = s / L[4 * i + i];
      s2 += y[i] * y[i];
    }
    out[q] = s2;
  }
}

// ------------------------------------------------------------------------------------------
// x / n correctly rounded to fp32 (what IEEE division gives), from r = RN64(1/n): RN64(x * r)
// is within 2^-52 (relative) of x/n, while a quotient of two floats lies >= 2^-47 (relative)
// from every fp32 rounding midpoint — it can never BE one (that would need 25 significant bits
// in the 24-bit numerator) — so rounding the product to fp32 lands on the same float.  Results
// outside the fp32 normal range, zeros and NaNs take the plain division.  Three instructions
// instead of the ~10 of a correctly rounded fp32 divide when one divisor serves a whole row.
struct Div32 {
  float n;
  double r;
  Div32() = default;
  __device__ explicit Div32(float n_) : n(n_), r(1.0 / (double)n_) {}
  __device__ __forceinline__ float operator()(float x) const {
    const double p = (double)x * r;
    return fabs(p) >= 0x1p-125 ? (float)p : x / n;
  }
};
// same interface for fp64 rows: plain division
struct Div64 {
  double n;
  Div64() = default;
  __device__ explicit Div64(double n_) : n(n_) {}
  __device__ __forceinline__ double operator()(double x) const { return x / n; }
};
template <typename FT>
using DivBy = typename std::conditional<sizeof(FT) == 4, Div32, Div64>::type;

// ------------------------------------------------------------------------------------------
// Feature numerics.
// numpy float32 pairwise sum (PW_BLOCKSIZE 128, 8 accumulators) of x[i]*x[i], sequential in
// one lane; the recursion (n2 = n/2 rounded down to a multiple of 8) unrolled with a stack.
template <typename XT>
__device__ inline float np_pairwise_sumsq_f32(const XT* xs, int n) {
  struct {
    const XT* p;
    __device__ float operator[](int i) const { return (float)p[i]; }
  } x{xs};
  float acc[24];
  int ap = 0;
  // iterative post-order walk over the split tree: leaves (<=128) summed, nodes combined
  int stk_off[24], stk_n[24], stk_state[24], top = 0;
  stk_off[0] = 0; stk_n[0] = n; stk_state[0] = 0; top = 1;
  while (top > 0) {
    int t = top - 1;
    int off = stk_off[t], m = stk_n[t];
    if (m <= 128) {
      float res;
      if (m < 8) {
        res = 0.0f;
        for (int i = 0; i < m; i++) { float v = x[off + i]; res += v * v; }
      } else {
        float r[8];
        for (int k = 0; k < 8; k++) { float v = x[off + k]; r[k] = v * v; }
        int i;
        for (i = 8; i < m - (m % 8); i += 8)
          for (int k = 0; k < 8; k++) { float v = x[off + i + k]; r[k] += v * v; }
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < m; i++) { float v = x[off + i]; res += v * v; }
      }
      acc[ap++] = res;
      top--;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (stk_state[t] == 0) {  // descend left
      stk_state[t] = 1;
      stk_off[top] = off; stk_n[top] = n2; stk_state[top] = 0; top++;
    } else if (stk_state[t] == 1) {  // descend right
      stk_state[t] = 2;
      stk_off[top] = off + n2; stk_n[top] = m - n2; stk_state[top] = 0; top++;
    } else {  // combine
      float b = acc[--ap], a = acc[--ap];
      acc[ap++] = a + b;
      top--;
    }
  }
  return acc[0];
}

// scipy cdist-cosine inner product: two interleaved fp64 accumulators, remainder added last.
template <typename A, typename B>
__device__ inline double dot2(const A& a, const B& b, int n) {
  double a0 = 0.0, a1 = 0.0;
  int i = 0;
  for (; i + 2 <= n; i += 2) { a0 += a(i) * b(i); a1 += a(i + 1) * b(i + 1); }
  double s = a0 + a1;
  if (i < n) s += a(i) * b(i);
  return s;
}

// ------------------------------------------------------------------------------------------
// Xor butterflies without LDS round trips.  `s += __shfl_xor(s, d)` is a ds_bpermute (an LDS
// pipe op, ~100+ cycles) per 32-bit word; these use DPP (a VALU operand modifier) within 16-lane
// rows and gfx950's v_permlane{16,32}_swap across rows.  Every step adds the same two values as
// the xor butterfly (IEEE addition is commutative, so a pair's two lanes get identical bits):
// a DPP rotate or mirror reads a lane whose value EQUALS lane l^d's once the earlier steps have
// made the values periodic (descending d = 32..1: rotate by d; ascending d = 1..: quad perms,
// then half-mirror / mirror).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// v[l] + v[l ^ 16] and v[l] + v[l ^ 32] (either operand order: same bits)
__device__ __forceinline__ float xsum16_f32(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32_f32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false,
                                                  false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ double xsum16_f64(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
__device__ __forceinline__ double xsum32_f64(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
}
constexpr int DPP_ROR = 0x120, DPP_QP_X1 = 0xB1, DPP_QP_X2 = 0x4E, DPP_HALF_MIRROR = 0x141,
              DPP_MIRROR = 0x140;
// the full descending butterfly d = 32, 16, ..., 1 of an fp64 value (all lanes end equal)
__device__ __forceinline__ double wave_bfly_desc_f64(double s) {
  s = xsum32_f64(s);
  s = xsum16_f64(s);
  s += dpp_f64<DPP_ROR + 8>(s);
  s += dpp_f64<DPP_ROR + 4>(s);
  s += dpp_f64<DPP_ROR + 2>(s);
  s += dpp_f64<DPP_ROR + 1>(s);
  return s;
}
// the ascending butterfly d = 1, 2, ..., < width (width a power of two <= 64) of a float
__device__ __forceinline__ float wave_bfly_asc_f32(float s, int width) {
  if (width > 1) s += dpp_f32<DPP_QP_X1>(s);
  if (width > 2) s += dpp_f32<DPP_QP_X2>(s);
  if (width > 4) s += dpp_f32<DPP_HALF_MIRROR>(s);
  if (width > 8) s += dpp_f32<DPP_MIRROR>(s);
  if (width > 16) s = xsum16_f32(s);
  if (width > 32) s = xsum32_f32(s);
  return s;
}

// np.linalg.norm of a 1-D feature is a BLAS dot with an unpinned order; the engine fixes the
// "wave order" (restated in oracle/bxo_track.c vnorm): lane l accumulates x[l], x[l+64], ...
// sequentially in fp64, then an xor butterfly d = 32..1 (commutative: every lane ends with the
// same bits).  Called by all 64 lanes of a wave.
template <typename FT>
__device__ inline double wave_sumsq(const FT* x, int n) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int k = lane; k < n; k += 64) { double v = (double)x[k]; s += v * v; }
  return wave_bfly_desc_f64(s);
}
template <typename FT>
__device__ inline FT wave_norm(const FT* x, int n) {
  double s = wave_sumsq(x, n);
  if constexpr (sizeof(FT) == 4) return sqrtf((float)s);
  else return sqrt(s);
}

// numpy float32 pairwise sum of squares, wave-parallel and bit-identical to the sequential
// recursion when n = 128 * 2^m (every split lands on a 128-element leaf): accumulator a (leaf
// a/8, slot a%8) sums x[128*(a/8) + 8i + a%8]^2 over i in order; slots and leaves then combine
// as balanced binary trees = xor butterflies.  Other n fall back to one lane's sequential walk.
__host__ __device__ inline bool np_wave_exact(int n) {
  const int nleaf = n >> 7;
  return (n & 127) == 0 && nleaf > 0 && (nleaf & (nleaf - 1)) == 0 && nleaf <= 32;
}
template <typename XT>
__device__ inline float np_sumsq_wave_fast(const XT* x, int n) {  // requires np_wave_exact(n)
  const int lane = threadIdx.x & 63;
  const int nacc = (n >> 7) * 8;  // 8 .. 256 accumulators
  const int regs = nacc > 64 ? nacc / 64 : 1;
  float part[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    part[r] = 0.0f;
    const int a = lane + 64 * r;
    if (r < regs && a < nacc) {
      const XT* p = x + 128 * (a >> 3) + (a & 7);
      float acc = (float)p[0] * (float)p[0];
      for (int i = 1; i < 16; i++) { float v = (float)p[8 * i]; acc += v * v; }
      part[r] = acc;
    }
    part[r] = wave_bfly_asc_f32(part[r], nacc < 64 ? nacc : 64);
  }
  // registers hold consecutive blocks of 8 leaves; combine them as a balanced tree
  float res = regs == 1 ? part[0]
              : regs == 2 ? part[0] + part[1]
                          : (part[0] + part[1]) + (part[2] + part[3]);
  return __shfl(res, 0);
}
// np_sumsq_wave_fast over a float row stored with 8 pad floats after every 128 elements (the
// accumulator reads of one instruction then fall in distinct LDS banks)
__device__ inline float np_sumsq_wave_fast_padded(const float* x, int n) {
  const int lane = threadIdx.x & 63;
  const int nacc = (n >> 7) * 8;
  const int regs = nacc > 64 ? nacc / 64 : 1;
  float part[4];
#pragma unroll
  for (int r = 0; r < 4; r++) {
    part[r] = 0.0f;
    const int a = lane + 64 * r;
    if (r < regs && a < nacc) {
      const float* p = x + 136 * (a >> 3) + (a & 7);
      float acc = p[0] * p[0];
      for (int i = 1; i < 16; i++) { float v = p[8 * i]; acc += v * v; }
      part[r] = acc;
    }
    part[r] = wave_bfly_asc_f32(part[r], nacc < 64 ? nacc : 64);
  }
  float res = regs == 1 ? part[0]
              : regs == 2 ? part[0] + part[1]
                          : (part[0] + part[1]) + (part[2] + part[3]);
  return __shfl(res, 0);
}
// NPF: the caller knows np_wave_exact(n) (compile-time split keeps the sequential fallback and
// its register footprint out of the fast kernels)
template <bool NPF, typename XT>
__device__ inline float np_sumsq_sel(const XT* x, int n) {
  if constexpr (NPF) return np_sumsq_wave_fast(x, n);
  else return __shfl(np_pairwise_sumsq_f32(x, n), 0);
}
template <typename XT>
__device__ inline float np_sumsq_wave(const XT* x, int n) {
  if (np_wave_exact(n)) return np_sumsq_wave_fast(x, n);
  float s = np_pairwise_sumsq_f32(x, n);
  return __shfl(s, 0);
}

// ------------------------------------------------------------------------------------------
// Block (256-thread) helpers.
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// exclusive prefix of a 0/1 flag over the block in thread order; `tmp` >= 4 ints of LDS.
__device__ inline int block_scan_flag(bool f, int* tmp, int& total) {
  const int lane = lane_id(), w = wave_id();
  unsigned long long m = __ballot(f);
  int pre = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) tmp[w] = __popcll(m);
  __syncthreads();
  int off = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) off += (k < w) ? tmp[k] : 0;
  total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return off + pre;
}

// Order-preserving compaction: emit(k, pos) for every k < n with pred(k).  Returns the count.
template <class P, class E>
__device__ inline int block_compact(int n, P pred, E emit, int* tmp) {
  int base = 0;
  for (int c = 0; c < n; c += WG) {
    int k = c + (int)threadIdx.x;
    bool f = k < n && pred(k);
    int tot;
    int pos = block_scan_flag(f, tmp, tot);
    if (f) emit(k, base + pos);
    base += tot;
  }
  __syncthreads();  // emitted entries are read by other threads right after
  return base;
}

// exclusive scan of cnt[0..n) in place by wave 0 (returns total via *total_out, also cnt[n]).
__device__ inline void wave0_exclusive_scan(int* cnt, int n) {
  if (wave_id() != 0) return;
  const int lane = lane_id();
  int carry = 0;
  for (int c = 0; c < n; c += WAVE) {
    int k = c + lane;
    int v = k < n ? cnt[k] : 0;
    int x = v;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      int y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    if (k < n) cnt[k] = carry + x - v;
    carry += __shfl(x, WAVE - 1);
  }
  if (lane == 0) cnt[n] = carry;
}

// ------------------------------------------------------------------------------------------
// Linear assignment with lapx `extend_cost=True, cost_limit=L` semantics on a sparse CSR of
// admissible edges (cost < L).  lapx's (n_r+n_c)^2 extension with L/2 fillers is exactly a
// max-gain partial matching with gains L - c, solved here by successive
// shortest augmenting paths (Dijkstra with potentials; rectangular LSAP) where every row owns a
// private zero-cost "dummy" column meaning "unmatched", rows processed in ascending order.
//
// A shortest-path search from a root only ever reaches rows and columns of the root's connected
// component of the candidate graph, so components are solved independently with the same
// per-component row order and the same result:
//   * single-edge components (a row whose only finite edge goes to a column no other row can
//     reach) are matched directly: exactly the path SSP would find (gain L-c>0, u = c-L, v = 0);
//   * small components run the sequential SSP on one lane each, all lanes in parallel;
//   * large components run it wave-parallel (relaxations over a row's edges and the argmin over
//     touched columns spread over the 64 lanes), one component after another.
// Every workspace array lives in LDS (the engine's association kernel and the op-level LAP
// kernel carve them from their dynamic LDS), so the pointers carry address space 3: their
// accesses compile to ds_* instructions, whose waits do not also wait for the vector-memory
// counter (a generic pointer is read by flat instructions, which wait on both).  Only the
// overflow edges (gcol / gcost) are global.
#define BX_LDS __attribute__((address_space(3)))
struct LapWS {
  const BX_LDS int* row_ptr;    // [R+1] edge offsets
  const BX_LDS uint16_t* ecol;  // edge columns (first elds in LDS, the rest in gcol)
  const BX_LDS double* ecost;   // edge costs  (first elds in LDS, the rest in gcost)
  const uint16_t* gcol;         // overflow edges in global memory
  const double* gcost;
  int elds;
  BX_LDS int16_t* col4row;      // [R] out: column or -1
  BX_LDS int16_t* row4col;      // [C] out: row or -1
  BX_LDS double* u;             // [R] row potentials
  BX_LDS double* v;             // [C] column potentials
  BX_LDS double* spc;           // [C] shortest-path costs (INF between solves)
  BX_LDS int16_t* path;         // [C]
  BX_LDS uint8_t* colflag;      // [C] bit0 = in SC, bit1 = touched
  BX_LDS uint16_t* touched;     // [C] touched column list (wave solver) / per-lane stretches
  BX_LDS uint16_t* srlist;      // [R] rows visited (SR) except the root / next-SR links (lane)
  BX_LDS int* coldeg;           // [C] finite-edge degree per column, then component labels
  BX_LDS uint16_t* roots;       // [R] rows left for the shortest-path phase, ascending
  BX_LDS int* rlab;             // [R] component label (smallest row index of the component)
  BX_LDS int* colaux;           // [C] multi-edge rows per column (star detection)
  BX_LDS int* colmin;           // [C] star components: winning row
  // Optional (null: wave 0 solves every component): scratch for the components handed to the
  // workgroup's other waves, one LDS block hs carved by the accessors below from the row bound
  // hT (R rounded up to 8) and the touched-list stride tws (C rounded up to 8) — per component
  // head row its row and column counts (cntr, cntc: [R]), the heads for the wave solver in
  // ascending order (big: [R], nbig: [1]), and for waves 1..3 their own touched-column and
  // visited-row lists (wave k: tw + (k-1) * tws, [C]; sw + (k-1) * hT, [R]).  Three fields, not
  // eight pointers: the association kernel runs at its SGPR limit, and every extra uniform live
  // across the LAP spilled.  lap_helper_bytes(hT, tws) is the block's size.
  BX_LDS int* hs = nullptr;
  int hT = 0, tws = 0;
  __device__ BX_LDS int* cntr() const { return hs; }
  __device__ BX_LDS int* cntc() const { return hs + hT; }
  __device__ BX_LDS int* nbig() const { return hs + 2 * hT; }
  __device__ BX_LDS uint16_t* big() const { return (BX_LDS uint16_t*)(hs + 2 * hT + 4); }
  __device__ BX_LDS uint16_t* tw() const { return big() + hT; }
  __device__ BX_LDS uint16_t* sw() const { return tw() + 3 * tws; }
  // if set: `stamp` stored (system scope: host-visible) whenever this LAP had a component for
  // the wave solver among more than BX_LAP_HELPER_ROOTS roots — the host's cue to launch the
  // helper-wave build of the association kernel (the two builds give identical results)
  int* bigmark = nullptr;
  int stamp = 0;
  int* comp_stats = nullptr;  // if set: [0] += components solved by the per-lane SSP (past the
                              // register path), [1] += components on the wave-parallel solver,
                              // [2] += those of [1] solved on the helper waves 1..3
  unsigned long long* dbg = nullptr;  // diagnostic counters (phase-timing builds only)
};
__host__ __device__ inline size_t lap_helper_bytes(int hT, int tws) {
  return 4 * (2 * (size_t)hT + 4) + 2 * (size_t)hT + 2 * 3 * (size_t)tws + 2 * 3 * (size_t)hT;
}
// a generic pointer into LDS (a __shared__ array or the dynamic LDS) as an address-space-3 one
template <typename T>
__device__ __forceinline__ BX_LDS T* lds_ptr(void* p) {
  return (BX_LDS T*)(p);
}
// LDS atomics on address-space-3 pointers
__device__ __forceinline__ void lds_add(BX_LDS int* p, int v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_min(BX_LDS int* p, int v) {
  __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_min(BX_LDS unsigned long long* p, unsigned long long v) {
  __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void lap_edge(const LapWS& w, int e, int& col, double& cost) {
  if (e < w.elds) { col = w.ecol[e]; cost = w.ecost[e]; }
  else { col = w.gcol[e - w.elds]; cost = w.gcost[e - w.elds]; }
}

// wave-wide argmin over (val, key); ties -> smaller key.  All lanes get the result.
__device__ __forceinline__ void wave_argmin(double& val, int& key) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    double ov = __shfl_xor(val, d);
    int ok = __shfl_xor(key, d);
    if (ov < val || (ov == val && ok < key)) { val = ov; key = ok; }
  }
}

// the same (value, key) argmin without LDS traffic: the value's minimum by DPP row rotations
// and gfx950's row / half swaps, then the smallest key among the lanes holding it (an int
// minimum the same way).  No NaNs.
__device__ __forceinline__ double lap_ror_d(double v, int ctrl_sel) {
  const long long b = __double_as_longlong(v);
  int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
  switch (ctrl_sel) {
    case 8: lo = __builtin_amdgcn_mov_dpp(lo, 0x128, 0xf, 0xf, false);
            hi = __builtin_amdgcn_mov_dpp(hi, 0x128, 0xf, 0xf, false); break;
    case 4: lo = __builtin_amdgcn_mov_dpp(lo, 0x124, 0xf, 0xf, false);
            hi = __builtin_amdgcn_mov_dpp(hi, 0x124, 0xf, 0xf, false); break;
    case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x122, 0xf, 0xf, false);
            hi = __builtin_amdgcn_mov_dpp(hi, 0x122, 0xf, 0xf, false); break;
    default: lo = __builtin_amdgcn_mov_dpp(lo, 0x121, 0xf, 0xf, false);
             hi = __builtin_amdgcn_mov_dpp(hi, 0x121, 0xf, 0xf, false); break;
  }
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double lap_swap_d(double v, bool half) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  unsigned a0, a1, h0, h1;
  if (half) {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a0 = l[0], a1 = l[1], h0 = h[0], h1 = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a0 = l[0], a1 = l[1], h0 = h[0], h1 = h[1];
  }
  return fmin(__longlong_as_double(((long long)h0 << 32) | a0),
              __longlong_as_double(((long long)h1 << 32) | a1));
}
__device__ __forceinline__ int lap_swap_i(int v, bool half) {
  const auto l = half ? __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false)
                      : __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return min((int)l[0], (int)l[1]);
}
__device__ __forceinline__ void wave_argmin_dpp(double& val, int& key) {
  double m = val;
  m = fmin(m, lap_ror_d(m, 8));
  m = fmin(m, lap_ror_d(m, 4));
  m = fmin(m, lap_ror_d(m, 2));
  m = fmin(m, lap_ror_d(m, 1));
  m = lap_swap_d(m, false);
  m = lap_swap_d(m, true);  // every lane: the wave minimum
  int k = val == m ? key : 0x7fffffff;
  k = min(k, __builtin_amdgcn_mov_dpp(k, 0x128, 0xf, 0xf, false));
  k = min(k, __builtin_amdgcn_mov_dpp(k, 0x124, 0xf, 0xf, false));
  k = min(k, __builtin_amdgcn_mov_dpp(k, 0x122, 0xf, 0xf, false));
  k = min(k, __builtin_amdgcn_mov_dpp(k, 0x121, 0xf, 0xf, false));
  k = lap_swap_i(k, false);
  k = lap_swap_i(k, true);
  val = m;
  key = k;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// augment along path[] ending at `sink` (>= 0 column, -2 dummy of dummy_row); one lane
__device__ __forceinline__ void lap_augment(const LapWS& w, int root, int sink, int dummy_row) {
  int j;
  if (sink == -2) {
    j = w.col4row[dummy_row];
    w.col4row[dummy_row] = -1;
    if (dummy_row == root) j = -1;
  } else {
    j = sink;
  }
  while (j >= 0) {
    int r = w.path[j];
    w.row4col[j] = (int16_t)r;
    int old = w.col4row[r];
    w.col4row[r] = (int16_t)j;
    if (r == root) break;
    j = old;
  }
}

// One SSP root on ONE lane (the lane's component only touches its own rows/columns).  Touched
// columns are appended to the lane's own stretch `tl` of touched[] (as long as its component has
// columns: the stretches of the wave's lanes are disjoint), so the argmin walks an array — the
// loads of consecutive entries are independent — instead of a linked list, whose every hop waited
// for the previous one's LDS load; touch order is kept, so ties resolve as before.  The
// relaxation loads the next edge's column state before storing the current one's (the columns of
// a row's edges are distinct; batches of four measured slower: K3's register budget).  Visited
// rows are kept as a linked list through srlist[].
__device__ __forceinline__ int lap_root_lane(int root, double L, const LapWS& w,
                                             BX_LDS uint16_t* tl) {
  double minVal = 0.0;
  int i = root, nt = 0, shead = -1, stail = -1, steps = 0;
  double dummy_best = INF;
  int dummy_row = -1, sink = -1;
  while (true) {
    const double ui = w.u[i];
    const int e1 = w.row_ptr[i + 1];
    int e = w.row_ptr[i];
    if (e < e1) {
      int j;
      double c;
      lap_edge(w, e, j, c);
      uint8_t f = w.colflag[j];
      double vj = w.v[j], sj = w.spc[j];
      for (; e < e1; e++) {
        int jn = j;
        double cn = 0.0, vn = 0.0, sn = 0.0;
        uint8_t fn = 0;
        if (e + 1 < e1) {
          lap_edge(w, e + 1, jn, cn);
          fn = w.colflag[jn];
          vn = w.v[jn];
          sn = w.spc[jn];
        }
        if (!(f & 1)) {
          const double r = minVal + (c - L) - ui - vj;
          if (r < sj) {
            w.spc[j] = r;
            w.path[j] = (int16_t)i;
            if (!(f & 2)) {
              w.colflag[j] = f | 2;
              tl[nt++] = (uint16_t)j;
            }
          }
        }
        j = jn;
        c = cn;
        f = fn;
        vj = vn;
        sj = sn;
      }
    }
    const double dv = minVal - ui;
    if (dv < dummy_best) { dummy_best = dv; dummy_row = i; }
    double bv = INF;
    int bj = -1;
    for (int k = 0; k < nt; k++) {
      const int j = tl[k];
      if (!(w.colflag[j] & 1) && w.spc[j] < bv) { bv = w.spc[j]; bj = j; }
    }
    if (dummy_best <= bv) { minVal = dummy_best; sink = -2; break; }
    minVal = bv;
    steps++;
    w.colflag[bj] |= 1;
    const int r4c = w.row4col[bj];
    if (r4c < 0) { sink = bj; break; }
    i = r4c;
    if (stail >= 0) w.srlist[stail] = (uint16_t)i; else shead = i;
    stail = i;
  }
  w.u[root] += minVal;
  for (int r = shead; r >= 0; r = (r == stail) ? -1 : (int)w.srlist[r])
    w.u[r] += minVal - w.spc[w.col4row[r]];
  for (int k = 0; k < nt; k++) {
    const int j = tl[k];
    if (w.colflag[j] & 1) w.v[j] -= minVal - w.spc[j];
  }
  lap_augment(w, root, sink, dummy_row);
  for (int k = 0; k < nt; k++) {
    const int j = tl[k];
    w.spc[j] = INF;
    w.colflag[j] = 0;
  }
  return steps;
}

// One SSP root, wave-parallel (called by all 64 lanes); tch / srl: this wave's touched-column and
// visited-row lists.
__device__ __forceinline__ int lap_root_wave(int root, double L, const LapWS& w,
                                             BX_LDS uint16_t* tch, BX_LDS uint16_t* srl) {
  const int lane = lane_id();
  double minVal = 0.0;
  int i = root, ntouched = 0, nsr = 0, steps = 0;
  double dummy_best = INF;
  int dummy_row = -1, sink = -1;  // sink >= 0 real column, -2 dummy of dummy_row
  while (true) {
    const double ui = w.u[i];
    const int b = w.row_ptr[i], e = w.row_ptr[i + 1];
    for (int base = b; base < e; base += WAVE) {
      int eidx = base + lane;
      bool newt = false;
      int j = 0;
      if (eidx < e) {
        double c;
        lap_edge(w, eidx, j, c);
        if (!(w.colflag[j] & 1)) {
          double r = minVal + (c - L) - ui - w.v[j];
          if (r < w.spc[j]) {
            w.spc[j] = r;
            w.path[j] = (int16_t)i;
            if (!(w.colflag[j] & 2)) { w.colflag[j] |= 2; newt = true; }
          }
        }
      }
      unsigned long long m = __ballot(newt);
      if (newt) tch[ntouched + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)j;
      ntouched += __popcll(m);
    }
    {  // dummy of row i: reduced cost 0 - u_i - 0 (its potential never moves)
      double dv = minVal - ui;
      if (dv < dummy_best) { dummy_best = dv; dummy_row = i; }
    }
    wave_sync_lds();
    // argmin over touched, not-yet-scanned columns; ties: a free column first (it ends the
    // search: on a tied problem the earliest-touched rule alone walks every matched column at
    // the same distance first — O(rows) steps per root, 467 ms at 512 x 512 all-equal), then the
    // earliest touched.  Any optimum will do here: a tied one is re-solved in lapx's order.
    double bv = INF;
    int bk = 0x7fffffff;
    for (int k = lane; k < ntouched; k += WAVE) {
      int j = tch[k];
      if (!(w.colflag[j] & 1)) {
        const double sv = w.spc[j];
        const int key = k | (w.row4col[j] >= 0 ? (1 << 30) : 0);
        if (sv < bv || (sv == bv && key < bk)) { bv = sv; bk = key; }
      }
    }
    wave_argmin_dpp(bv, bk);
    bk &= (1 << 30) - 1;
    if (dummy_best <= bv) {  // leave dummy_row unmatched (ties: stop early)
      minVal = dummy_best;
      sink = -2;
      break;
    }
    const int j = tch[bk];
    steps++;
    minVal = bv;
    if (lane == 0) w.colflag[j] |= 1;
    const int r4c = w.row4col[j];
    wave_sync_lds();
    if (r4c < 0) { sink = j; break; }
    i = r4c;
    if (lane == 0) srl[nsr] = (uint16_t)i;
    nsr++;
  }
  // dual updates
  if (lane == 0) w.u[root] += minVal;
  for (int k = lane; k < nsr; k += WAVE) {
    int r = srl[k];
    w.u[r] += minVal - w.spc[w.col4row[r]];
  }
  wave_sync_lds();
  for (int k = lane; k < ntouched; k += WAVE) {
    int j = tch[k];
    if (w.colflag[j] & 1) w.v[j] -= minVal - w.spc[j];
  }
  wave_sync_lds();
  if (lane == 0) lap_augment(w, root, sink, dummy_row);
  for (int k = lane; k < ntouched; k += WAVE) {
    int j = tch[k];
    w.spc[j] = INF;
    w.colflag[j] = 0;
  }
  wave_sync_lds();
  return steps;
}

// Register-resident SSP for a component of m <= LAP_RM rows (ascending) and at most LAP_CM
// columns, on one lane: the same successive-shortest-path steps as lap_root_lane, with the
// component's columns kept sorted by column index (= the CSR edge order of every row, so the
// relaxation and touch order are unchanged) and the argmin's ties broken by touch order.  No
// LDS round trips on the dependent chain.  Returns false (nothing written) when the component
// has more than LAP_CM columns.
constexpr int LAP_RM = 3, LAP_CM = 6;
// a[k] / a[k] = v on register arrays with a runtime k.  The per-element predicate goes through
// an empty asm so the compiler cannot fold the select chain back into a dynamically indexed
// (scratch-memory) array access.
__device__ __forceinline__ bool ropaque(bool b) {
  int x = b;
  asm volatile("" : "+v"(x));
  return x != 0;
}
template <int N, typename T>
__device__ __forceinline__ T rsel(const T (&a)[N], int k) {
  T r = a[0];
#pragma unroll
  for (int q = 1; q < N; q++) r = ropaque(q == k) ? a[q] : r;
  return r;
}
template <int N, typename T>
__device__ __forceinline__ void rput(T (&a)[N], int k, T v) {
#pragma unroll
  for (int q = 0; q < N; q++) a[q] = ropaque(q == k) ? v : a[q];
}
__device__ __forceinline__ bool lap_component_regs(const int (&rr)[LAP_RM], int m, double L,
                                                   const LapWS& w, int& steps) {
  constexpr int RM = LAP_RM, CM = LAP_CM;
  int cols[CM];
#pragma unroll
  for (int q = 0; q < CM; q++) cols[q] = 0x7fffffff;
  int nc = 0;
  bool over = false;
#pragma unroll
  for (int q = 0; q < RM; q++) {
    if (q >= m) break;
    for (int e = w.row_ptr[rr[q]]; e < w.row_ptr[rr[q] + 1]; e++) {
      int j;
      double c;
      lap_edge(w, e, j, c);
      if (!(c < INF)) continue;
      bool found = false;
#pragma unroll
      for (int t = 0; t < CM; t++) found |= cols[t] == j;
      if (found) continue;
      if (nc == CM) { over = true; continue; }
      rput(cols, nc, j);
      nc++;
    }
  }
  if (over) return false;
  // sort the column slots ascending (odd-even transposition network; empty slots = INT_MAX)
#pragma unroll
  for (int rd = 0; rd < CM; rd++)
#pragma unroll
    for (int t = rd & 1; t + 1 < CM; t += 2)
      if (cols[t] > cols[t + 1]) { const int x = cols[t]; cols[t] = cols[t + 1]; cols[t + 1] = x; }
  double cm[RM][CM];
#pragma unroll
  for (int q = 0; q < RM; q++)
#pragma unroll
    for (int t = 0; t < CM; t++) cm[q][t] = INF;
#pragma unroll
  for (int q = 0; q < RM; q++) {
    if (q >= m) break;
    for (int e = w.row_ptr[rr[q]]; e < w.row_ptr[rr[q] + 1]; e++) {
      int j;
      double c;
      lap_edge(w, e, j, c);
      if (!(c < INF)) continue;
#pragma unroll
      for (int t = 0; t < CM; t++)
        if (cols[t] == j) cm[q][t] = c;
    }
  }
  double u[RM], v[CM];
  int c4r[RM], r4c[CM];
#pragma unroll
  for (int q = 0; q < RM; q++) { u[q] = 0.0; c4r[q] = -1; }
#pragma unroll
  for (int t = 0; t < CM; t++) { v[t] = 0.0; r4c[t] = -1; }
#pragma unroll 1
  for (int q0 = 0; q0 < m; q0++) {
    double spc[CM];
    int path[CM], rank[CM];
    bool scanned[CM], touched[CM];
#pragma unroll
    for (int t = 0; t < CM; t++) {
      spc[t] = INF; path[t] = -1; rank[t] = 0; scanned[t] = false; touched[t] = false;
    }
    double minVal = 0.0, dummy_best = INF;
    int i = q0, dummy_row = -1, sink = -1, cnt = 0;
    unsigned srmask = 0;
    for (int it = 0; it <= RM; it++) {
      const double ui = rsel(u, i);
#pragma unroll
      for (int t = 0; t < CM; t++) {
        double c = cm[0][t];
#pragma unroll
        for (int q = 1; q < RM; q++) c = ropaque(q == i) ? cm[q][t] : c;
        if (!(c < INF) || scanned[t]) continue;
        const double r = minVal + (c - L) - ui - v[t];
        if (r < spc[t]) {
          spc[t] = r;
          path[t] = i;
          if (!touched[t]) { touched[t] = true; rank[t] = cnt++; }
        }
      }
      const double dv = minVal - ui;
      if (dv < dummy_best) { dummy_best = dv; dummy_row = i; }
      double bv = INF;
      int bs = -1, br = 0x7fffffff;
#pragma unroll
      for (int t = 0; t < CM; t++)
        if (touched[t] && !scanned[t] && (spc[t] < bv || (spc[t] == bv && rank[t] < br))) {
          bv = spc[t]; bs = t; br = rank[t];
        }
      if (dummy_best <= bv) { minVal = dummy_best; sink = -2; break; }
      minVal = bv;
      steps++;
      rput(scanned, bs, true);
      const int r4 = rsel(r4c, bs);
      if (r4 < 0) { sink = bs; break; }
      i = r4;
      srmask |= 1u << i;
    }
    // dual updates (u of the root and of the visited rows; v of the scanned columns)
#pragma unroll
    for (int q = 0; q < RM; q++) {
      if (ropaque(q == q0)) u[q] += minVal;
      else if ((srmask >> q) & 1u) u[q] += minVal - rsel(spc, c4r[q]);
    }
#pragma unroll
    for (int t = 0; t < CM; t++)
      if (scanned[t]) v[t] -= minVal - spc[t];
    // augment
    int j;
    if (sink == -2) {
      j = rsel(c4r, dummy_row);
      rput(c4r, dummy_row, -1);
      if (dummy_row == q0) j = -1;
    } else {
      j = sink;
    }
    for (int it = 0; it <= RM && j >= 0; it++) {
      const int r = rsel(path, j);
      rput(r4c, j, r);
      const int old = rsel(c4r, r);
      rput(c4r, r, j);
      if (r == q0) break;
      j = old;
    }
  }
#pragma unroll
  for (int q = 0; q < RM; q++)
    if (q < m) {
      w.col4row[rr[q]] = (int16_t)(c4r[q] >= 0 ? rsel(cols, c4r[q]) : -1);
      w.u[rr[q]] = u[q];  // the duals, for lap_tied_block
    }
#pragma unroll
  for (int t = 0; t < CM; t++)
    if (t < nc) {
      w.row4col[cols[t]] = (int16_t)(r4c[t] >= 0 ? rsel(rr, r4c[t]) : -1);
      w.v[cols[t]] = v[t];
    }
  return true;
}

#ifndef BX_HELP_MIN_BIG  // components for the wave solver in one LAP that cue the helper build
#define BX_HELP_MIN_BIG 1
#endif
#ifndef BX_LAP_HELPER_ROOTS
#define BX_LAP_HELPER_ROOTS 32
#endif
#ifndef BX_LAP_LANE_ROWS
#define BX_LAP_LANE_ROWS 3
#endif
constexpr int LAP_LANE_ROWS = BX_LAP_LANE_ROWS;  // components up to this many rows: one lane

// Preparation, called by ALL threads of the workgroup (block-wide syncs): initialise, settle
// single-edge and star components, and list the rows left for the searches (ascending) in
// w.roots.  Returns that count (uniform).  `scan_tmp`: >= 4 ints of LDS for block_compact.
__device__ __forceinline__ int lap_prepare_block(int R, int C, double L, const LapWS& w,
                                                 int* scan_tmp) {
  const int tid = threadIdx.x;
  for (int k = tid; k < R; k += WG) { w.col4row[k] = -1; w.u[k] = 0.0; }
  for (int k = tid; k < C; k += WG) {
    w.row4col[k] = -1; w.v[k] = 0.0; w.spc[k] = INF; w.colflag[k] = 0; w.coldeg[k] = 0;
    w.colaux[k] = 0;
  }
  __syncthreads();
  auto row_scan = [&](int r, int& nf, int& jj, double& cc) {
    nf = 0; jj = -1; cc = 0.0;
    for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
      int j;
      double c;
      lap_edge(w, e, j, c);
      if (c < INF) { nf++; jj = j; cc = c; }
    }
  };
  // finite-edge degree per column, and per column the rows with >= 2 finite edges
  for (int r = tid; r < R; r += WG) {
    int nf, jj;
    double cc;
    row_scan(r, nf, jj, cc);
    if (nf == 0) continue;
    for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
      int j;
      double c;
      lap_edge(w, e, j, c);
      if (!(c < INF)) continue;
      lds_add(&w.coldeg[j], 1);
      if (nf >= 2) lds_add(&w.colaux[j], 1);
    }
  }
  __syncthreads();
  // Single-edge components (a row whose only finite edge goes to a column no other row can
  // reach) are matched directly: that is exactly the path SSP would find for them (gain L-c>0,
  // potentials u = c-L, v = 0), and no other row can ever touch that row or column.
  // A "star" component — one column whose every finite-edge row has no other finite edge — is
  // also settled directly: rows taken in ascending order, a later row takes the column from
  // its holder iff strictly cheaper (its search scans the column, then the holder's dummy wins
  // exactly when c_new < c_holder), so the column ends with the cheapest row, ties to the
  // smallest row index, and every other row unmatched.
  auto okey = [](double c) {  // order-preserving double → u64
    const unsigned long long b = __builtin_bit_cast(unsigned long long, c);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  };
  BX_LDS unsigned long long* keyslot = (BX_LDS unsigned long long*)w.spc;  // INF outside searches
  int nstar = 0;
  for (int r = tid; r < R; r += WG) {
    int nf, jj;
    double cc;
    row_scan(r, nf, jj, cc);
    if (nf == 1 && w.coldeg[jj] == 1) {
      w.col4row[r] = (int16_t)jj;
      w.row4col[jj] = (int16_t)r;
      w.u[r] = cc - L;
    } else if (nf == 1 && w.colaux[jj] == 0) {
      keyslot[jj] = ~0ull;
      w.colmin[jj] = 0x7fffffff;
      nstar++;
    } else if (nf == 0) {
      w.col4row[r] = -2;  // only inadmissible candidates: its search would end at its dummy
    }
  }
  int tot;
  block_scan_flag(nstar > 0, scan_tmp, tot);  // (also a block barrier)
  if (tot) {
    auto star = [&](int r, int& jj, double& cc) {
      int nf;
      row_scan(r, nf, jj, cc);
      return nf == 1 && w.coldeg[jj] > 1 && w.colaux[jj] == 0;
    };
    for (int r = tid; r < R; r += WG) {
      int jj;
      double cc;
      if (star(r, jj, cc)) lds_min(&keyslot[jj], okey(cc));
    }
    __syncthreads();
    for (int r = tid; r < R; r += WG) {
      int jj;
      double cc;
      if (star(r, jj, cc) && okey(cc) == keyslot[jj]) lds_min(&w.colmin[jj], r);
    }
    __syncthreads();
    for (int r = tid; r < R; r += WG) {
      int jj;
      double cc;
      if (!star(r, jj, cc)) continue;
      if (w.colmin[jj] == r) {
        w.col4row[r] = (int16_t)jj;
        w.row4col[jj] = (int16_t)r;
        w.v[jj] = cc - L;  // optimal duals u = 0, v = c - L: every other row's edge has
                           // reduced cost c_r - c >= 0, zero exactly on a tie (lap_tied_block)
      } else {
        w.col4row[r] = -2;  // settled unmatched
      }
    }
    __syncthreads();
    for (int r = tid; r < R; r += WG) {  // give the star columns back their INF
      int jj;
      double cc;
      if (star(r, jj, cc)) w.spc[jj] = INF;
    }
    __syncthreads();
  }
  // rows that still need a shortest-path search (have a finite edge, not settled), ascending
  return block_compact(
      R, [&](int r) { return w.col4row[r] == -1 && w.row_ptr[r + 1] > w.row_ptr[r]; },
      [&](int r, int p) { w.roots[p] = (uint16_t)r; }, scan_tmp);
}

// The components for the wave-parallel solver (its one call site: a second inlined copy pushed
// the association kernel into scratch): on waves 1..3 from the big list, round-robin, each with
// its own lists — or, without helper scratch, on wave 0 after its lanes from the nbl heads they
// left in colaux (dead after lap_prepare_block; a component has a column of its own, so <= C
// heads).  Each component's roots in ascending order (a ballot over the ascending roots list, 64
// at a time).  Returns the components solved.
__device__ __forceinline__ int lap_wave_components(int nroots, double L, const LapWS& w,
                                                   bool helpers, int wid, int nbl, int& nsteps) {
  const int lane = lane_id();
  const int stride = helpers ? 3 : 1;
  const int nb = helpers ? *w.nbig() : nbl;
  BX_LDS uint16_t* tch = helpers ? w.tw() + (wid - 1) * w.tws : w.touched;
  BX_LDS uint16_t* srl = helpers ? w.sw() + (wid - 1) * w.hT : w.srlist;
  int ncomp = 0;
  for (int c = helpers ? wid - 1 : 0; c < nb; c += stride) {
    const int h = helpers ? (int)w.big()[c] : w.colaux[c];
    for (int k0 = 0; k0 < nroots; k0 += WAVE) {
      const int k = k0 + lane;
      unsigned long long m = __ballot(k < nroots && w.rlab[w.roots[k]] == h);
      while (m) {
        const int b = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        nsteps += lap_root_wave(w.roots[k0 + b], L, w, tch, srl);
      }
    }
    ncomp++;
  }
  return ncomp;
}

// The searches after lap_prepare_block, called by ALL threads of the workgroup.  Wave 0 labels
// the components; small ones (<= LAP_LANE_ROWS rows) are solved one lane each on wave 0, the rest
// by the wave-parallel solver on waves 1..3 (components dealt round-robin in head order, each
// wave with its own touched / visited lists) when the caller gave the scratch for that (w.cntr),
// else every component on wave 0's lanes.  Components are disjoint in rows and columns, so the
// waves share the per-row / per-column arrays without conflict, and every component's result is
// the same whichever solver takes it.  (One call site per solver: a second inlined copy of the
// wave solver pushed the association kernel into scratch.)
__device__ __forceinline__ void lap_solve_roots_block(int R, int C, int nroots, double L,
                                                      const LapWS& w) {
  const int lane = lane_id(), wid = wave_id();
  // (helper waves only past BX_LAP_HELPER_ROOTS roots: the scratch bookkeeping and the two
  // barriers cost the small LAPs of uncrowded scenes more than the occasional 4+-row component
  // solved on wave 0 after its lanes)
  const bool helpers = w.hT > 0 && nroots > BX_LAP_HELPER_ROOTS;
  const int lane_max = LAP_LANE_ROWS;  // rows of a lane-solved component
  int nsteps = 0, ncomp = 0, maxrows = 0, iters = 0, nlane = 0, nwave = 0, nbl = 0;
  if (w.dbg && wid == 0 && lane == 0) w.dbg[3] = __builtin_amdgcn_s_memtime();
  if (wid == 0 && nroots > 0) {
    // component labels by min-label propagation over the roots' finite edges (coldeg reused as
    // the per-column label; columns no root reaches keep "none")
    for (int j = lane; j < C; j += WAVE) w.coldeg[j] = 0x7fffffff;
    wave_sync_lds();
    for (int k = lane; k < nroots; k += WAVE) {
      const int r = w.roots[k];
      w.rlab[r] = r;
      for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
        int j;
        double c;
        lap_edge(w, e, j, c);
        if (c < INF) w.coldeg[j] = 0x7fffffff;
      }
    }
    wave_sync_lds();
    while (true) {
      for (int k = lane; k < nroots; k += WAVE) {
        const int r = w.roots[k], lr = w.rlab[r];
        for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
          int j;
          double c;
          lap_edge(w, e, j, c);
          if (c < INF) lds_min(&w.coldeg[j], lr);
        }
      }
      wave_sync_lds();
      bool changed = false;
      for (int k = lane; k < nroots; k += WAVE) {
        const int r = w.roots[k];
        int m = w.rlab[r];
        for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
          int j;
          double c;
          lap_edge(w, e, j, c);
          if (c < INF) m = min(m, w.coldeg[j]);
        }
        if (m < w.rlab[r]) { w.rlab[r] = m; changed = true; }
      }
      const bool any = __ballot(changed) != 0ull;
      wave_sync_lds();
      iters++;
      if (!any) break;
    }
    if (helpers) {
      // rows and columns per component (by head), then the heads for the wave solver
      BX_LDS int* cntr = w.cntr();
      BX_LDS int* cntc = w.cntc();
      for (int k = lane; k < nroots; k += WAVE) cntr[w.roots[k]] = 0, cntc[w.roots[k]] = 0;
      wave_sync_lds();
      for (int k = lane; k < nroots; k += WAVE) lds_add(&cntr[w.rlab[w.roots[k]]], 1);
      for (int j = lane; j < C; j += WAVE)
        if (w.coldeg[j] != 0x7fffffff) lds_add(&cntc[w.coldeg[j]], 1);
      wave_sync_lds();
      int nb = 0;
      for (int k0 = 0; k0 < nroots; k0 += WAVE) {
        const int k = k0 + lane;
        const int h = k < nroots ? w.roots[k] : 0;
        const bool bg = k < nroots && w.rlab[h] == h && cntr[h] > lane_max;
        const unsigned long long m = __ballot(bg);
        if (bg) w.big()[nb + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)h;
        nb += __popcll(m);
      }
      if (lane == 0) *w.nbig() = nb;
    }
    if (w.dbg && lane == 0) w.dbg[8] = __builtin_amdgcn_s_memtime();
  } else if (helpers && wid == 0 && lane == 0) {
    *w.nbig() = 0;
  }
  if (helpers) __syncthreads();
  if (wid == 0 && nroots > 0) {
    // small components: one lane each, in parallel.  The lanes take the component heads 64 at a
    // time; a lane solving its component gets a stretch of touched[] as long as the component's
    // column count (exclusive prefix over the wave: the components are disjoint, so the
    // stretches fit in C).
    for (int k0 = 0; k0 < nroots; k0 += WAVE) {
      const int k = k0 + lane;
      int h = -1, nrows = 0;
      bool mine = false, bigh = false;
      if (k < nroots) {
        h = w.roots[k];
        if (w.rlab[h] == h) {
          if (helpers) nrows = w.cntr()[h];
          else
            for (int q = k; q < nroots; q++) nrows += w.rlab[w.roots[q]] == h;
          ncomp++;
          maxrows = max(maxrows, nrows);
          mine = true;
          if (nrows > lane_max) {
            mine = false;  // the wave solver's
            bigh = !helpers;
          } else if (nrows <= LAP_RM) {  // register-resident solve when it fits
            int rr[LAP_RM];
            int n = 0;
#pragma unroll
            for (int t = 0; t < LAP_RM; t++) rr[t] = h;
            for (int q = k; q < nroots && n < nrows; q++) {
              const int r = w.roots[q];
              if (w.rlab[r] == h) { rput(rr, n, r); n++; }
            }
            if (lap_component_regs(rr, nrows, L, w, nsteps)) mine = false;
          }
          nlane += mine;  // (the per-lane SSP: past the register path)
        }
      }
      int ncols = 0;
      if (mine) {
        if (helpers) ncols = w.cntc()[h];
        else
          for (int j = 0; j < C; j++) ncols += w.coldeg[j] == h;
      }
      int off = ncols;  // inclusive prefix over the lanes, then exclusive
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) {
        const int o = __shfl_up(off, d);
        if (lane >= d) off += o;
      }
      off -= ncols;
      if (mine)
        for (int q = k; q < nroots; q++) {
          const int r = w.roots[q];
          if (w.rlab[r] == h) nsteps += lap_root_lane(r, L, w, w.touched + off);
        }
      const unsigned long long mb = __ballot(bigh);  // (ascending: the heads come in order)
      if (bigh) w.colaux[nbl + __popcll(mb & ((1ull << lane) - 1ull))] = h;
      nbl += __popcll(mb);
      wave_sync_lds();
    }
    if (w.dbg && lane == 0) w.dbg[9] = __builtin_amdgcn_s_memtime();
    if (w.bigmark && lane == 0 && nroots > BX_LAP_HELPER_ROOTS &&
        (helpers ? *w.nbig() : nbl) >= BX_HELP_MIN_BIG)
      __hip_atomic_store(w.bigmark, w.stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if ((helpers ? (wid >= 1 && wid <= 3) : wid == 0) && nroots > 0)
    nwave += lap_wave_components(nroots, L, w, helpers, wid, nbl, nsteps);
  if (helpers) __syncthreads();
  if (wid == 0)
    for (int r = lane; r < R; r += WAVE)
      if (w.col4row[r] == -2) w.col4row[r] = -1;
  if (w.comp_stats) {
    int sa = nlane;
    for (int d = 32; d >= 1; d >>= 1) sa += __shfl_xor(sa, d);
    if (lane == 0 && (sa | nwave)) {  // (nwave is wave-uniform)
      atomicAdd(&w.comp_stats[0], sa);
      atomicAdd(&w.comp_stats[1], nwave);
      if (helpers) atomicAdd(&w.comp_stats[2], nwave);
    }
  }
  if (w.dbg && wid == 0) {
    for (int d = 32; d >= 1; d >>= 1) {
      nsteps += __shfl_xor(nsteps, d);
      ncomp += __shfl_xor(ncomp, d);
      maxrows = max(maxrows, __shfl_xor(maxrows, d));
    }
    if (lane == 0) {
      w.dbg[0] = nroots;
      w.dbg[1] = nsteps;  // (wave 0's: the helper waves' steps are not counted)
      w.dbg[2] = R;
      w.dbg[4] = ncomp;
      w.dbg[5] = maxrows;
      w.dbg[6] = iters;
      w.dbg[7] = __builtin_amdgcn_s_memtime();  // after labels+solve
    }
  }
  if (!helpers) wave_sync_lds();
}

// ------------------------------------------------------------------------------------------
// Is the solved matching the UNIQUE optimum?  The sparse solver above equals lapx whenever the
// optimal pair set is unique; on a tie lapx's pick depends on its whole dense run, so the caller
// re-solves with lapx itself (bx_jv.h).  Max-gain view: gains g = L - c, duals U = -u >= 0,
// V = -v >= 0, reduced cost rc = U_i + V_j - g_ij = (c - L) - u_i - v_j >= 0, zero on every
// matched edge; unmatched rows/columns have zero duals.  Another optimum exists iff, in the
// directed graph of tight edges (unmatched edge row -> column, matched edge column -> row), there
// is a cycle or a path from a source (an unmatched row, or a matched column with V = 0) to a sink
// (an unmatched column, or a matched row with U = 0): swapping along it keeps the gain.  Tight
// and zero are taken within BX_TIE_EPS (float duals; a near-tie is re-solved too), and `pre`
// carries the caller's own flag (a pair whose cost is within BX_TIE_EPS of L: gain 0, which the
// CSR drops as inadmissible).  Called by ALL threads after lap_solve_block; returns a uniform
// answer.  Uses rlab / coldeg as scratch.
constexpr double BX_TIE_EPS = 1e-12;
__device__ inline bool lap_tied_block(int R, int C, double L, const LapWS& w, int* scan_tmp,
                                      bool pre) {
  const int tid = threadIdx.x;
  auto extra_tight = [&](int r, int e, int& j) {  // a tight unmatched edge of row r
    double c;
    lap_edge(w, e, j, c);
    if (!(c < INF) || j == w.col4row[r]) return false;
    return (c - L) - w.u[r] - w.v[j] <= BX_TIE_EPS;
  };
  // pass 0: a matched edge with both duals zero (gain 0) is a tie by itself; tight unmatched
  // edges decide whether the graph search runs at all (after a multi-step augmentation the
  // formerly matched edges stay tight, so they are common but rarely part of a swap)
  bool tie = pre, extra = false;
  for (int r = tid; r < R; r += WG) {
    const int jm = w.col4row[r];
    if (jm >= 0 && w.u[r] > -BX_TIE_EPS && w.v[jm] > -BX_TIE_EPS) tie = true;
    for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1] && !extra; e++) {
      int j;
      extra |= extra_tight(r, e, j);
    }
  }
  int ntie, nextra;
  block_scan_flag(tie, scan_tmp, ntie);
  block_scan_flag(extra, scan_tmp, nextra);
  if (ntie) return true;
  if (!nextra) return false;
  // reach-T: hc[j] = column j leads to a sink, hr[r] = row r does
  BX_LDS int* hr = w.rlab;
  BX_LDS int* hc = w.coldeg;
  for (int r = tid; r < R; r += WG) hr[r] = 0;
  for (int j = tid; j < C; j += WG) {
    const int r = w.row4col[j];
    hc[j] = r < 0 || w.u[r] > -BX_TIE_EPS;
  }
  __syncthreads();
  while (true) {
    bool ch = false;
    for (int r = tid; r < R; r += WG) {
      if (hr[r]) continue;
      for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1]; e++) {
        int j;
        if (extra_tight(r, e, j) && hc[j]) { hr[r] = 1; ch = true; break; }
      }
    }
    __syncthreads();
    for (int j = tid; j < C; j += WG) {
      const int r = w.row4col[j];
      if (!hc[j] && r >= 0 && hr[r]) { hc[j] = 1; ch = true; }
    }
    int nch;
    block_scan_flag(ch, scan_tmp, nch);
    if (!nch) break;
  }
  bool st = false;
  for (int r = tid; r < R; r += WG) st |= w.col4row[r] < 0 && hr[r];
  for (int j = tid; j < C; j += WG) st |= w.row4col[j] >= 0 && w.v[j] > -BX_TIE_EPS && hc[j];
  int nst;
  block_scan_flag(st, scan_tmp, nst);
  if (nst) return true;
  // cycles: peel rows without a live successor (row -> the row matched to a tight column);
  // whatever survives lies on or leads into a cycle
  BX_LDS int* al = w.rlab;
  for (int r = tid; r < R; r += WG) al[r] = 1;
  __syncthreads();
  while (true) {
    bool ch = false;
    for (int r = tid; r < R; r += WG) {
      if (!al[r]) continue;
      bool live = false;
      for (int e = w.row_ptr[r]; e < w.row_ptr[r + 1] && !live; e++) {
        int j;
        if (extra_tight(r, e, j)) {
          const int r2 = w.row4col[j];
          live = r2 >= 0 && al[r2];
        }
      }
      if (!live) { al[r] = 0; ch = true; }
    }
    int nch;
    block_scan_flag(ch, scan_tmp, nch);
    if (!nch) break;
  }
  bool cyc = false;
  for (int r = tid; r < R; r += WG) cyc |= al[r] != 0;
  int ncyc;
  block_scan_flag(cyc, scan_tmp, ncyc);
  return ncyc != 0;
}

// Whole solve, called by ALL threads of the workgroup.
__device__ __forceinline__ void lap_solve_block(int R, int C, double L, const LapWS& w,
                                                int* scan_tmp) {
  const int nroots = lap_prepare_block(R, C, L, w, scan_tmp);
  lap_solve_roots_block(R, C, nroots, L, w);
  __syncthreads();
}

}  // namespace bx
