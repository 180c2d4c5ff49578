// bx_engine.hip — the per-frame association engine.  One frame of many independent sequences is
// advanced by a short pipeline of kernels on one stream (bx_engine_step):
//
//   K1 det_feature_kernel   grid, wave per high-conf detection   (BoT-SORT + ReID only)
//   K2 predict_kernel       grid, thread per track slot           multi_predict (+ multi_gmc)
//   K3 assoc_kernel         workgroup per sequence                costs, 3 assignments, lists
//   K4 update_kernel        grid, thread per update record        KF update / initiate, scalars
//   K5 feature_kernel       grid, wave per record with a feature  feature EMA  (BoT-SORT + ReID)
//   K6 finish_kernel        workgroup per sequence                remove_duplicate, outputs
//
// Together they do what the reference's ByteTrack.update (trackers/bytetrack/bytetrack.py:
// 158-302) and BotSort.update (trackers/botsort/botsort.py:94-411) do for one frame.  The heavy,
// regular math (feature normalisation and EMA, Kalman predict/update) runs as full-width grid
// kernels; only the inherently sequential part of a frame (list bookkeeping, candidate CSR,
// shortest-augmenting-path assignment) runs one workgroup per sequence, on lean LDS.  Track
// state stays resident in HBM between frames (SoA per sequence).  Grids put the sequence index
// in blockIdx.x so that every kernel's workgroups for sequence s land on the same XCD (the
// dispatcher deals linear workgroup ids round-robin over the 8 XCDs): per-sequence state written
// by one kernel is re-read by the next from the same L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/bxassoc.h"
#include "bx_device.h"

using namespace bx;

namespace {

#include "bx_jv.h"

constexpr int CLS_HIST = 8;  // BoT-SORT per-track class-history entries (update_cls)
#ifndef BX_ELDS
#define BX_ELDS 1024
#endif
constexpr int ELDS_DEFAULT = BX_ELDS;  // LAP edges kept in LDS; the rest spill to global scratch
constexpr int REG_F = 512;   // feature rows up to this width live in registers: 8 per lane
constexpr int REG_EPL = REG_F / 64;
constexpr int REG_FP = REG_F + REG_F / 16;  // LDS row stride: 8 pad floats per 128 (np_dn)
constexpr int NWAVE = WG / WAVE;
// doubles per slot: mean[8], covariance[64], then the pre-predict mean[2], mean[3] of the first
// pending covariance predict and of the later ones (their process noise is computed from them;
// see K2)
constexpr int KF_STRIDE = 76;
constexpr int KF_QM = 72;
constexpr int KF_QM2 = 74;

// A feature row held by one wave, element q = lane + 64 r in v[r] (F <= REG_F).
template <typename FT>
struct RegRow {
  FT v[REG_EPL];
  __device__ void load(const FT* p, int F) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < REG_EPL; r++) {
      const int q = lane + 64 * r;
      v[r] = q < F ? p[q] : FT(0);
    }
  }
  template <typename OT>
  __device__ void store(OT* p, int F) const {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int r = 0; r < REG_EPL; r++) {
      const int q = lane + 64 * r;
      if (q < F) p[q] = (OT)v[r];
    }
  }
  // the engine's fixed BLAS-dot order (see wave_sumsq): lane-strided sequential, xor butterfly
  __device__ FT norm(int F) const {
    const int lane = threadIdx.x & 63;
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < REG_EPL; r++)
      if (lane + 64 * r < F) {
        const double d = (double)v[r];
        // a float's square is exact in fp64, so the fused form rounds identically to s + d*d
        if constexpr (sizeof(FT) == 4) s = __builtin_fma(d, d, s);
        else s += d * d;
      }
    s = wave_bfly_desc_f64(s);
    if constexpr (sizeof(FT) == 4) return sqrtf((float)s);
    else return sqrt(s);
  }
  // Div32's product form for the whole row under ONE wave-uniform test (zeros included: the
  // product keeps x/n's signed zero); a row with a tiny/NaN quotient anywhere takes Div32.
  __device__ void div(FT n) {
    if constexpr (sizeof(FT) == 4) {
      const double rn = 1.0 / (double)n;
      double p[REG_EPL];
      bool fast = true;
#pragma unroll
      for (int r = 0; r < REG_EPL; r++) {
        p[r] = (double)v[r] * rn;
        fast &= fabs(p[r]) >= 0x1p-125 || p[r] == 0.0;
      }
      if (__ballot(!fast) == 0ull) {
#pragma unroll
        for (int r = 0; r < REG_EPL; r++) v[r] = (float)p[r];
        return;
      }
    }
    const DivBy<FT> d(n);
#pragma unroll
    for (int r = 0; r < REG_EPL; r++) v[r] = d(v[r]);
  }
  // numpy float32 norm of the float32-cast row (+1e-8 as embedding_distance adds it), staged
  // through this wave's LDS row so lanes can read numpy's accumulator layout
  template <bool NPF>
  __device__ float np_dn(float* wbuf, int F) const {
    if constexpr (NPF) {  // padded layout (element e at e + 8·(e/128)): conflict-free LDS reads
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int r = 0; r < REG_EPL; r++) {
        const int q = lane + 64 * r;
        if (q < F) wbuf[q + 8 * (q >> 7)] = (float)v[r];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      float dn = sqrtf(np_sumsq_wave_fast_padded(wbuf, F)) + 1e-8f;
      __builtin_amdgcn_wave_barrier();
      return dn;
    }
    store(wbuf, F);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float dn = sqrtf(np_sumsq_sel<NPF>((const float*)wbuf, F)) + 1e-8f;
    __builtin_amdgcn_wave_barrier();
    return dn;
  }
};

// scipy cdist's two-accumulator inner product (see dot2) of two float32 rows, 16-byte loads
__device__ inline double dot2_f32(const float* a, const float* b, int n) {
  double a0 = 0.0, a1 = 0.0;
  int i = 0;
  if ((n & 3) == 0) {
    const float4* a4 = (const float4*)a;
    const float4* b4 = (const float4*)b;
    for (; i < n; i += 4) {
      const float4 x = a4[i >> 2], y = b4[i >> 2];
      a0 += (double)x.x * (double)y.x;
      a1 += (double)x.y * (double)y.y;
      a0 += (double)x.z * (double)y.z;
      a1 += (double)x.w * (double)y.w;
    }
    return a0 + a1;
  }
  for (; i + 2 <= n; i += 2) {
    a0 += (double)a[i] * (double)b[i];
    a1 += (double)a[i + 1] * (double)b[i + 1];
  }
  double s = a0 + a1;
  if (i < n) s += (double)a[i] * (double)b[i];
  return s;
}

// scipy cdist-cosine of two already-normalised float32 rows (matching.py:283-287), max(0, .)
__device__ inline double cosine_rows(const float* a, double na, const float* b, double nb,
                                     int F) {
  double c = dot2_f32(a, b, F) / (na * nb);
  if (fabs(c) > 1.0) c = copysign(1.0, c);
  double d = 1.0 - c;
  return d < 0.0 ? 0.0 : d;
}

thread_local std::string g_err;
int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess)                                                                  \
      return set_err(BX_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e));          \
  } while (0)

// Device-side view of an engine (passed by value to every kernel).
struct Dev {
  int S, T, D, F, kind, emb_f64, with_reid, fuse_first, max_time_lost, elds;
  int lap_stats;  // count LAP components per solver path (bx_engine_set_lap_stats; default off)
  int* lapmark;   // host-mapped: the launch stamp of the last LAP that wanted the helper waves
  int lapstamp;   // this launch's stamp
  double low, high, new_thresh, match_thresh, prox, app;
  int* seq;           // [S][SQ_STRIDE] per-sequence scalars (SQ_*)
  uint16_t* act;      // [S][T] active list (slots)
  uint16_t* lost;     // [S][T] lost list
  uint16_t* act2;     // [S][T] frame scratch: lists before remove_duplicate (K3 → K6)
  uint16_t* lost2;    // [S][T]
  uint32_t* flags;    // [S][T] F_* bits
  int* frame_id;      // [S][T]
  int* start;         // [S][T]
  int* id;            // [S][T]
  int* tlen;          // [S][T]
  int* detind;        // [S][T]
  double* conf;       // [S][T]
  double* cls;        // [S][T]
  double* kf;         // [S][T][KF_STRIDE] Kalman state per slot: mean[8], cov[64], qm[2], qm2[2]
  void* feat;         // [S][T][F] smooth_feat
  double* clsh;       // [S][T][CLS_HIST][2]
  int* ncls;          // [S][T]
  uint16_t* gcol;     // [S][T*D] LAP edge overflow
  double* gcost;      // [S][T*D]
  int2* rec;          // [S][D] frame scratch: update records (K3 → K4/K5)
  double* dnrm;       // [2][S][D][4] frame scratch: n1, n2 (update_features), dn
                      // (embedding_distance), by launch parity (early-features mode: K1 of the
                      // next frame writes the other half while this frame's K1c / K5 read)
  int dpar;           // this launch's half of dnrm
  float* tdn;         // [S][T] numpy float32 norm (+1e-8) of each track's smooth_feat (K5 keeps it)
  uint32_t* pairs;    // [S][T*D] frame scratch: gated (slot << 16 | det) pairs
  int* npair;         // [S] gated pair count (zeroed by K6 for the next frame)
  double* etab;       // [S][T][D] frame scratch: embedding distance of gated pairs
  unsigned char* jvs; // [S][jvs_stride] lapx lapjv state for tied associations (n = T + D)
  size_t jvs_stride;
  void* fscr;         // [S][D][F] frame scratch for F > REG_F only: twice-normalised det rows
  int* status;        // [1] latched engine status
  unsigned long long* dbg;  // [S][32] phase stamps (diagnostic builds only, else null)
};

// Diagnostic phase stamps (build with -DBX_PHASE_TIMING; never in the shipped library).
constexpr int BX_DBG_STRIDE = 64;  // stamps + counters per sequence
#ifdef BX_PHASE_TIMING
#define BX_STAMP(k)                                                                   \
  do {                                                                                \
    __syncthreads();                                                                  \
    if (threadIdx.x == 0 && P.dbg) P.dbg[(size_t)s * BX_DBG_STRIDE + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define BX_STAMP(k) \
  do {              \
  } while (0)
#endif

enum {
  SQ_NA = 0, SQ_NL, SQ_FC, SQ_IDC, SQ_STATUS, SQ_NA2, SQ_NL2, SQ_NREC, SQ_SKIP,
  SQ_NHIGH, SQ_NPAIR, SQ_NDET,  // last frame's high dets, gated pairs, dets (statistics)
  SQ_NTIE,                       // associations re-solved by lapx's lapjv (tied optimum), total
  SQ_NCOMP17, SQ_NCOMPW,         // LAP components on the per-lane SSP / the wave SSP
  SQ_NCOMPH,                     // ... of which on the helper waves 1..3 (helper build)
  SQ_STRIDE = 16
};
// update records: x = slot | kind << 16, y = detection index within the sequence's frame
enum : int { R_UPDATE = 0, R_REACT = 1, R_NEW = 2, R_FEAT = 4 };

constexpr int NBIN = 64;  // x-bins of the candidate sweep (one wave scans them)
// LDS carve-out of the association kernel (host and device agree on it).
struct LdsA {
  size_t o_dbox, o_dboxf, o_dconf, o_tboxf, o_cbox, o_bin, o_bcol, o_u, o_v, o_spc, o_ecost, o_flags, o_fid,
      o_rowptr, o_rlab, o_colaux, o_colmin, o_ints, o_act, o_lost, o_unconf, o_pool, o_rtr, o_lostl, o_refind, o_newt,
      o_c4r, o_srl, o_roots, o_r4c, o_path, o_touch, o_cdeg, o_hd, o_sd, o_rem, o_ecol, o_mark,
      o_colf, o_dkind, total;
  __host__ __device__ LdsA(int T, int D, int elds) {
    size_t o = 0;
    auto take = [&](size_t bytes) {
      size_t r = o;
      o += (bytes + 15) & ~size_t(15);
      return r;
    };
    o_dbox = take(sizeof(double) * 4 * D);
    o_dboxf = take(sizeof(float) * 4 * D);  // outward-rounded fp32 copy for candidate tests
    o_tboxf = take(sizeof(float) * 4 * T);  // same for the rows of the current association
    o_cbox = take(sizeof(float) * 4 * D);   // the current association's column boxes, in order
    o_bin = take(sizeof(int) * (2 * NBIN + 2));  // x-bin starts and cursors
    o_bcol = take(2 * D);                        // columns grouped by x-bin
    o_dconf = take(sizeof(double) * D);
    o_u = take(sizeof(double) * T);
    o_v = take(sizeof(double) * D);
    o_spc = take(sizeof(double) * D);
    o_ecost = take(sizeof(double) * elds);
    o_flags = take(sizeof(uint32_t) * T);
    o_fid = take(sizeof(int) * T);
    o_rowptr = take(sizeof(int) * (T + 1));
    o_cdeg = take(4 * D);
    o_rlab = take(4 * T);
    o_colaux = take(4 * D);
    o_colmin = take(4 * D);
    o_ints = take(sizeof(int) * 64);
    o_act = take(2 * T);
    o_lost = take(2 * T);
    o_unconf = take(2 * T);
    o_pool = take(2 * T);
    o_rtr = take(2 * T);
    o_lostl = take(2 * T);
    o_refind = take(2 * T);
    o_c4r = take(2 * T);
    o_srl = take(2 * T);
    o_roots = take(2 * T);
    o_newt = take(2 * D);
    o_r4c = take(2 * D);
    o_path = take(2 * D);
    o_touch = take(2 * D);
    o_hd = take(2 * D);
    o_sd = take(2 * D);
    o_rem = take(2 * D);
    o_ecol = take(2 * elds);
    o_mark = take(T);
    o_colf = take(D);
    o_dkind = take(D);
    total = o;
  }
};

// LDS carve-out of the finishing kernel.
struct LdsF {
  size_t o_lbox, o_lage, o_fa, o_fl, o_dupa, o_dupl, o_keep, o_ints, total;
  __host__ __device__ LdsF(int T) {
    size_t o = 0;
    auto take = [&](size_t bytes) {
      size_t r = o;
      o += (bytes + 15) & ~size_t(15);
      return r;
    };
    o_lbox = take(sizeof(double) * 4 * T);
    o_lage = take(sizeof(int) * T);
    o_fa = take(2 * T);
    o_fl = take(2 * T);
    o_dupa = take(T);
    o_dupl = take(T);
    o_keep = take(T);
    o_ints = take(sizeof(int) * 16);
    total = o;
  }
};

// mark bits (per slot, per frame)
enum : uint8_t { M_POOL = 1, M_ACT2 = 2, M_REMNOW = 4, M_TMP = 32 };
// ints[] scratch slots
enum { I_NA = 0, I_NL, I_FC, I_IDC, I_ERR, I_XMIN, I_XMAX, I_W, I_CLS0, I_SCAN = 32 };

// STrack.xyxy of a track (mean-based): KF mean (x, y, a|w, h) → xyxy
template <int KIND>
__device__ __forceinline__ void track_box(const double* g_kf, int slot, double* box) {
  const double2* m = (const double2*)(g_kf + (size_t)slot * KF_STRIDE);
  const double2 m01 = m[0], m23 = m[1];
  double r[4] = {m01.x, m01.y, m23.x, m23.y};
  if (KIND == KIND_BYTE) r[2] *= r[3];
  xywh2xyxy(r, box);
}

// measurement vector of a detection row (float32 as setup_decorator left it)
template <int KIND>
__device__ __forceinline__ void det_measurement(const float* r, double* meas) {
  double xyxy[4] = {(double)r[0], (double)r[1], (double)r[2], (double)r[3]};
  double xywh[4];
  xyxy2xywh(xyxy, xywh);
  if (KIND == KIND_BYTE) {
    double tlwh[4];
    xywh2tlwh(xywh, tlwh);
    tlwh2xyah(tlwh, meas);
  } else {
    for (int q = 0; q < 4; q++) meas[q] = xywh[q];
  }
}

// ------------------------------------------------------------------------------------------
// K1: BoT-SORT detection features.  STrack(det, feat) → update_features: f1 = f/|f|,
// f2 = f1/|f1| (botsort_track.py:40-49; curr == smooth for a fresh track), and the numpy
// float32 norm dn of (float)f2 that embedding_distance scales the det row by (matching.py:
// 266-287).  Only the three norms are stored: every later use (K1c's cosine rows, K5's EMA)
// recomputes f2 = (f / n1) / n2 elementwise from the input row, bit-identically.
// Grid (n_seq, ceil(D/K1_DETS)); each wave walks its block's detections with stride 4 (no
// prefetch of the next row: the lower VGPR count buys more resident waves, which hide more).
#ifndef BX_K1_DETS
#define BX_K1_DETS 16
#endif
// detections per K1 block (4 per wave; round 5, interleaved A/Bs at C3: 16 per block 0.5975 /
// 0.5997 ms per step against 0.6003 / 0.6011 with 8, 32 no better, 64 and 4 worse)
constexpr int K1_DETS = BX_K1_DETS;
// FC: the feature width when it is a compile-time constant (REG_F: bounds tests and per-element
// addressing fold away, measured ~1/3 of the row's VALU instructions), else 0 (P.F).
template <typename FT, bool NPF, int FC>
__global__ __launch_bounds__(WG) void det_feature_kernel(Dev P, int seq0,
                                                         const float* __restrict__ dets,
                                                         const int* __restrict__ det_off,
                                                         const FT* __restrict__ embs) {
  __shared__ __align__(16) float s_w[NWAVE * REG_FP];
  const int b = blockIdx.x, s = seq0 + b, w = wave_id(), lane = lane_id();
  const int F = FC ? FC : P.F, D = P.D;
  const int d0 = det_off[b], N = min(det_off[b + 1] - d0, D);
  const int k0 = blockIdx.y * K1_DETS, k1 = min(k0 + K1_DETS, N);
  if (k0 >= N) return;  // block-uniform
  __shared__ unsigned long long s_hi;  // bit k - k0: detection k is high
  if (w == 0) {
    const int k = k0 + lane;
    const unsigned long long m = __ballot(k < k1 && (double)dets[(size_t)(d0 + k) * 6 + 4] > P.high);
    if (lane == 0) s_hi = m;
  }
  __syncthreads();
  const unsigned long long hi = s_hi;
  auto next = [&](int k) {  // next high detection of this wave at or after k
    for (; k < k1; k += NWAVE)
      if ((hi >> (k - k0)) & 1ull) return k;
    return k1;
  };
  auto put_norms = [&](int k, FT n1, FT n2, float dn) {
    if (lane == 0) {
      double* o = P.dnrm + ((size_t)P.dpar * P.S * D + (size_t)s * D + k) * 4;
      o[0] = (double)n1;
      o[1] = (double)n2;
      o[2] = (double)dn;
    }
  };
  if (F <= REG_F) {
    float* wb = s_w + w * REG_FP;
    for (int k = next(k0 + w); k < k1; k = next(k + NWAVE)) {
      RegRow<FT> x;
      x.load(embs + (size_t)(d0 + k) * F, F);
      const FT n1 = x.norm(F);
      x.div(n1);
      const FT n2 = x.norm(F);
      x.div(n2);
      put_norms(k, n1, n2, x.template np_dn<NPF>(wb, F));
    }
    return;
  }
  for (int k = next(k0 + w); k < k1; k = next(k + NWAVE)) {
    const FT* f = embs + (size_t)(d0 + k) * F;
    FT* f2 = (FT*)P.fscr + ((size_t)s * D + k) * F;
    const FT n1 = wave_norm(f, F);
    for (int q = lane; q < F; q += WAVE) f2[q] = f[q] / n1;
    const FT n2 = wave_norm((const FT*)f2, F);  // same lane mapping: reads own writes
    for (int q = lane; q < F; q += WAVE) f2[q] = f2[q] / n2;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // other lanes read f2 next
    put_norms(k, n1, n2, sqrtf(np_sumsq_sel<NPF>((const FT*)f2, F)) + 1e-8f);
  }
}

// ------------------------------------------------------------------------------------------
// K1b: BoT-SORT gating (botsort.py:200-215): a (track, high det) pair enters the appearance
// term iff its IoU distance <= proximity_thresh.  Every listed track (active ++ lost = the rows
// of the first and third association) is tested against every high detection with the exact
// fp64 cost K3 uses, so K3 finds each gated edge's embedding distance precomputed.
// Grid (n_seq, GATE_BLOCKS); detection boxes staged in LDS (fp64 + outward-rounded fp32 for a
// conservative reject); one thread per track, detections walked in order from LDS (broadcast).
// (Fusing K2's predict into this kernel and overlapping it with K1 measured slower: the two
// VALU-bound kernels slowed each other down.)
#ifndef BX_GATE_BLOCKS
#define BX_GATE_BLOCKS 4
#endif
#ifndef BX_GATE_SPLIT
#define BX_GATE_SPLIT 4
#endif
constexpr int GATE_BLOCKS = BX_GATE_BLOCKS;
constexpr int GATE_SPLIT = BX_GATE_SPLIT;  // threads per track, each over every SPLIT-th detection
template <int KIND>
__global__ __launch_bounds__(WG) void gate_kernel(Dev P, int seq0, const float* __restrict__ dets,
                                                  const int* __restrict__ det_off) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int b = blockIdx.x, s = seq0 + b, T = P.T, D = P.D;
  double* s_db = (double*)smem;                             // [D][4]
  float4* s_fb = (float4*)(smem + sizeof(double) * 4 * D);  // [D], x1 = NaN if not high
  const int d0 = det_off[b], N = min(det_off[b + 1] - d0, D);
  for (int j = threadIdx.x; j < N; j += WG) {
    const float* r = dets + (size_t)(d0 + j) * 6;
    double xyxy[4] = {(double)r[0], (double)r[1], (double)r[2], (double)r[3]};
    double xywh[4], db[4];
    xyxy2xywh(xyxy, xywh);
    xywh2xyxy(xywh, db);
    for (int q = 0; q < 4; q++) s_db[4 * j + q] = db[q];
    s_fb[j] = (double)r[4] > P.high
                  ? make_float4(__double2float_rd(db[0]), __double2float_rd(db[1]),
                                __double2float_ru(db[2]), __double2float_ru(db[3]))
                  : make_float4(__builtin_nanf(""), 0.f, 0.f, 0.f);
  }
  __syncthreads();
  const int* seq = P.seq + (size_t)s * SQ_STRIDE;
  const int na = seq[SQ_NA], nl = seq[SQ_NL];
  const double* g_kf = P.kf + (size_t)s * T * KF_STRIDE;
  uint32_t* pairs = P.pairs + (size_t)s * T * D;
  const bool prefilter = P.prox < 1.0;  // gating needs IoU > 0, i.e. intersecting boxes
  const int part = threadIdx.x % GATE_SPLIT;
  for (int p = (blockIdx.y * WG + threadIdx.x) / GATE_SPLIT; p < na + nl;
       p += GATE_BLOCKS * WG / GATE_SPLIT) {
    const int slot = p < na ? P.act[(size_t)s * T + p] : P.lost[(size_t)s * T + p - na];
    double tb[4];
    track_box<KIND>(g_kf, slot, tb);
    const float4 tf = make_float4(__double2float_rd(tb[0]), __double2float_rd(tb[1]),
                                  __double2float_ru(tb[2]), __double2float_ru(tb[3]));
    for (int j = part; j < N; j += GATE_SPLIT) {
      const float4 db = s_fb[j];
      if (__builtin_isnan(db.x)) continue;  // not a high detection
      if (prefilter &&
          !((fminf(tf.z, db.z) > fmaxf(tf.x, db.x)) & (fminf(tf.w, db.w) > fmaxf(tf.y, db.y))))
        continue;
      if (!(1 - iou_pair(tb, s_db + 4 * j) > P.prox))
        pairs[atomicAdd(&P.npair[s], 1)] = (uint32_t)(slot << 16 | j);
    }
  }
}

// ------------------------------------------------------------------------------------------
// K1c: embedding distance of every gated pair (matching.py:266-287 + botsort.py:209-214):
// A = (float)smooth_feat / dn_t (dn_t kept per track by K5), B = (float)f2 / dn_d with f2 =
// (f / n1) / n2 rebuilt from the input row (K1's norms); scipy cdist cosine with its own
// two-accumulator dots for A.B, |A|, |B|; /2; > appearance_thresh → 1.  Stored in the dense
// per-sequence [T][D] table K3 reads.
// scipy's two accumulators are independent chains (even elements into one, odd into the other,
// summed at the end), so a pair's dots run on TWO lanes — lane 2p the even chain, lane 2p+1 the
// odd one — and a wave owns COS_P pairs: COS_P = 16 gives ~8 waves per SIMD at C3 (the kernel is
// load-latency bound; the old 64-pairs-per-wave layout left 2).  Rows stream through LDS in
// COS_CH = 32-element chunks (one whole 128-B line of each row per chunk: 8 lanes x 16 B), the
// elementwise divisions done by the loading lane, the next chunk's loads in flight meanwhile.
// Grid (n_seq, COS_BLOCKS).
#ifndef BX_COS_BLOCKS
#define BX_COS_BLOCKS 2
#endif
constexpr int COS_BLOCKS = BX_COS_BLOCKS;
constexpr int COS_CH = 32;
#ifndef BX_COS_P
#define BX_COS_P 16
#endif
constexpr int COS_P = BX_COS_P;  // 8 or 16 (a multiple of 8: 8 lanes load a row's chunk)
__device__ inline void cos_finish(Dev& P, int s, int slot, int dk, double ab, double aa,
                                  double bb) {
  double c = ab / (sqrt(aa) * sqrt(bb));
  if (fabs(c) > 1.0) c = copysign(1.0, c);
  double d = 1.0 - c;
  d = d < 0.0 ? 0.0 : d;
  double ed = d / 2.0;
  if (ed > P.app) ed = 1.0;
  P.etab[((size_t)s * P.T + slot) * P.D + dk] = ed;
}
template <typename FT>
__device__ __forceinline__ void load4(const FT* p, FT* v) {
  if constexpr (sizeof(FT) == 4) {
    const float4 t = *(const float4*)p;
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    const double2 t0 = *(const double2*)p, t1 = *(const double2*)(p + 2);
    v[0] = t0.x; v[1] = t0.y; v[2] = t1.x; v[3] = t1.y;
  }
}
template <typename FT, int FC>
__global__ __launch_bounds__(WG) void cosine_kernel(Dev P, int seq0, const int* __restrict__ det_off,
                                                    const FT* __restrict__ embs) {
  constexpr int KR = COS_P / 8;  // row pieces per lane on each side (A: tracks, B: detections)
  // row stride COS_CH + 2: the 32 chain lanes (pair p, parity) read banks 2p + parity
  __shared__ float s_a[NWAVE][COS_P][COS_CH + 2], s_b[NWAVE][COS_P][COS_CH + 2];
  const int b = blockIdx.x, s = seq0 + b, T = P.T, D = P.D, F = FC ? FC : P.F, w = wave_id(),
            lane = lane_id();
  const int np = P.npair[s], d0 = det_off[b];
  const uint32_t* pairs = P.pairs + (size_t)s * T * D;
  const int col = (lane & 7) * 4;  // this lane's 4 elements of every chunk
  const int cp = lane >> 1, par = lane & 1;  // chain lanes: pair cp, even/odd elements
  for (int p0 = (blockIdx.y * NWAVE + w) * COS_P; p0 < np; p0 += COS_BLOCKS * NWAVE * COS_P) {
    // row pieces: pairs (lane >> 3) + 8k, k < KR
    const FT* arow[KR];
    const FT* brow[KR];
    Div32 da[KR], db[KR];
    DivBy<FT> d1[KR], d2[KR];
#pragma unroll
    for (int k = 0; k < KR; k++) {
      const int pp = p0 + (lane >> 3) + 8 * k;
      const uint32_t pr = pp < np ? pairs[pp] : pairs[p0];
      const int slot = pr >> 16, dk = pr & 0xffff;
      arow[k] = (const FT*)P.feat + ((size_t)s * T + slot) * F + col;
      brow[k] = embs + (size_t)(d0 + dk) * F + col;
      da[k] = Div32(P.tdn[(size_t)s * T + slot]);
      const double* nr = P.dnrm + ((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4;
      d1[k] = DivBy<FT>((FT)nr[0]);
      d2[k] = DivBy<FT>((FT)nr[1]);
      db[k] = Div32((float)nr[2]);
    }
    double ab = 0.0, aa = 0.0, bb = 0.0;  // this lane's chain (even or odd elements)
    FT av[KR][4], bv[KR][4];  // raw elements of the current chunk; the next chunk's in flight
#pragma unroll
    for (int k = 0; k < KR; k++) { load4(arow[k], av[k]); load4(brow[k], bv[k]); }
    for (int c0 = 0; c0 < F; c0 += COS_CH) {
      FT nav[KR][4], nbv[KR][4];
      const int cn = c0 + COS_CH < F ? c0 + COS_CH : c0;
#pragma unroll
      for (int k = 0; k < KR; k++) { load4(arow[k] + cn, nav[k]); load4(brow[k] + cn, nbv[k]); }
#pragma unroll
      for (int k = 0; k < KR; k++) {
        const int row = (lane >> 3) + 8 * k;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          s_a[w][row][col + q] = da[k]((float)av[k][q]);
          s_b[w][row][col + q] = db[k]((float)d2[k](d1[k](bv[k][q])));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (lane < 2 * COS_P) {
#pragma unroll
        for (int q = par; q < COS_CH; q += 2) {
          // products of two floats are exact in fp64: fma rounds identically to acc + x*y
          const double x = (double)s_a[w][cp][q], y = (double)s_b[w][cp][q];
          ab = __builtin_fma(x, y, ab);
          aa = __builtin_fma(x, x, aa);
          bb = __builtin_fma(y, y, bb);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < KR; k++)
#pragma unroll
        for (int q = 0; q < 4; q++) { av[k][q] = nav[k][q]; bv[k][q] = nbv[k][q]; }
    }
    // even chain + odd chain, as scipy adds its two accumulators
    const double ab1 = __shfl_xor(ab, 1), aa1 = __shfl_xor(aa, 1), bb1 = __shfl_xor(bb, 1);
    if (lane < 2 * COS_P && par == 0 && p0 + cp < np) {
      const uint32_t pr = pairs[p0 + cp];
      cos_finish(P, s, pr >> 16, pr & 0xffff, ab + ab1, aa + aa1, bb + bb1);
    }
  }
}

// any F: thread per pair, element by element (same arithmetic as above)
template <typename FT>
__global__ __launch_bounds__(WG) void cosine_kernel_any(Dev P, int seq0,
                                                        const int* __restrict__ det_off,
                                                        const FT* __restrict__ embs) {
  const int b = blockIdx.x, s = seq0 + b, T = P.T, D = P.D, F = P.F;
  const int np = P.npair[s];
  const uint32_t* pairs = P.pairs + (size_t)s * T * D;
  for (int p = blockIdx.y * WG + threadIdx.x; p < np; p += COS_BLOCKS * WG) {
    const uint32_t pr = pairs[p];
    const int slot = pr >> 16, dk = pr & 0xffff;
    const FT* a = (const FT*)P.feat + ((size_t)s * T + slot) * F;
    const FT* f = embs + (size_t)(det_off[b] + dk) * F;
    const float dn = P.tdn[(size_t)s * T + slot];
    const double* nr = P.dnrm + ((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4;
    const FT n1 = (FT)nr[0], n2 = (FT)nr[1];
    const float bdn = (float)nr[2];
    auto A = [&](int q) { return (double)((float)a[q] / dn); };
    auto B = [&](int q) { return (double)((float)((f[q] / n1) / n2) / bdn); };
    double ab0 = 0.0, ab1 = 0.0, aa0 = 0.0, aa1 = 0.0, bb0 = 0.0, bb1 = 0.0;
    int q = 0;
    for (; q + 2 <= F; q += 2) {
      const double x0 = A(q), x1 = A(q + 1), y0 = B(q), y1 = B(q + 1);
      ab0 += x0 * y0; ab1 += x1 * y1;
      aa0 += x0 * x0; aa1 += x1 * x1;
      bb0 += y0 * y0; bb1 += y1 * y1;
    }
    double ab = ab0 + ab1, aa = aa0 + aa1, bb = bb0 + bb1;
    if (q < F) {
      const double x0 = A(q), y0 = B(q);
      ab += x0 * y0; aa += x0 * x0; bb += y0 * y0;
    }
    cos_finish(P, s, slot, dk, ab, aa, bb);
  }
}

// ------------------------------------------------------------------------------------------
// Kalman predict split in two (kf_predict_soa restated): the association only needs predicted
// MEANS (boxes), so K2 predicts the mean now and the covariance predict is deferred to the pass
// that updates the track anyway (K4) — one read/write of the 512-byte covariance per frame.
// F·P·Fᵀ with dt = 1 splits into 16 independent 2x2 "quads" {(i,j),(i,j+4),(i+4,j),(i+4,j+4)};
// quad (i, j) is exactly the expressions kf_predict_soa evaluates for those four entries.
__device__ __forceinline__ void kf_predict_quad(int kind, const double* qm, double* c, int i,
                                                int j) {
  double mv[4] = {0.0, 0.0, qm[0], qm[1]}, q[8];
  kf_process_noise(kind, mv, q);  // reads mean[2], mean[3] only (pre-predict values)
  const double p00 = c[8 * i + j], p10 = c[8 * (i + 4) + j], p01 = c[8 * i + j + 4],
               p11 = c[8 * (i + 4) + j + 4];
  double v = (p00 + p10) + (p01 + p11);
  double v11 = p11;
  if (i == j) { v = v + q[i]; v11 = v11 + q[i + 4]; }
  c[8 * i + j] = v;
  c[8 * i + j + 4] = p01 + p11;
  c[8 * (i + 4) + j] = p10 + p11;
  c[8 * (i + 4) + j + 4] = v11;
}
__device__ __forceinline__ void kf_predict_cov(int kind, const double* qm, double* c) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) kf_predict_quad(kind, qm, c, i, j);
}
// n pending covariance predicts of slot state m (K2): the first with qm, the rest with qm2
__device__ inline void kf_materialize(int kind, double* m, int n) {
  for (int k = 0; k < n; k++) kf_predict_cov(kind, m + (k ? KF_QM2 : KF_QM), m + 8);
}
// kf_materialize for K2's counter-overflow path, quad by quad through memory with no unrolling:
// the same expressions as kf_predict_quad, but it keeps the predict kernel's register budget
// (inlined, the 64-entry covariance in registers cost it 190 VGPRs and 2 waves/SIMD)
__device__ __noinline__ void kf_materialize_mem(int kind, double* m, int n) {
  double* c = m + 8;
#pragma nounroll
  for (int k = 0; k < n; k++) {
    const double* qm = m + (k ? KF_QM2 : KF_QM);
    double mv[4] = {0.0, 0.0, qm[0], qm[1]}, q[8];
    kf_process_noise(kind, mv, q);
#pragma nounroll
    for (int ij = 0; ij < 16; ij++) {
      const int i = ij >> 2, j = ij & 3;
      const double p00 = c[8 * i + j], p10 = c[8 * (i + 4) + j], p01 = c[8 * i + j + 4],
                   p11 = c[8 * (i + 4) + j + 4];
      double v = (p00 + p10) + (p01 + p11);
      double v11 = p11;
      if (i == j) { v = v + q[i]; v11 = v11 + q[i + 4]; }
      c[8 * i + j] = v;
      c[8 * i + j + 4] = p01 + p11;
      c[8 * (i + 4) + j] = p10 + p11;
      c[8 * (i + 4) + j + 4] = v11;
    }
  }
}
// multi_gmc covariance part: cov = R8·cov·R8ᵀ, R8 = kron(I4, R) (botsort.py:192-195)
__device__ inline void gmc_cov(const double* H, double* c) {
  double RP[64];
  for (int bq = 0; bq < 4; bq++)
    for (int cc = 0; cc < 8; cc++) {
      double x0 = c[8 * (2 * bq) + cc], x1 = c[8 * (2 * bq + 1) + cc];
      RP[8 * (2 * bq) + cc] = H[0] * x0 + H[1] * x1;
      RP[8 * (2 * bq + 1) + cc] = H[3] * x0 + H[4] * x1;
    }
  for (int r = 0; r < 8; r++)
    for (int bq = 0; bq < 4; bq++) {
      double y0 = RP[8 * r + 2 * bq], y1 = RP[8 * r + 2 * bq + 1];
      c[8 * r + 2 * bq] = y0 * H[0] + y1 * H[1];
      c[8 * r + 2 * bq + 1] = y0 * H[3] + y1 * H[4];
    }
}

// K2: STrack.multi_predict MEAN part over strack_pool = joint(tracked, lost) (bytetrack.py:
// 205-207, botsort.py:188-189) and, for BoT-SORT with a CMC warp, multi_gmc's mean part over the
// pool and the unconfirmed tracks (botsort.py:192-195).  Sets F_PRED / F_GMC for K4.
// Grid (n_seq, ceil(T/256)); thread per slot.
// The per-slot body is shared with the fused gating kernel (K1b predicts its listed tracks).
template <int KIND, bool GMC>
__device__ __forceinline__ void predict_slot(Dev& P, int s, int slot, uint32_t f,
                                             const double* __restrict__ H) {
  const bool pool = ((f & F_INACT) && (f & F_ACT)) || (f & F_INLOST);
  const bool unconf = (f & F_INACT) && !(f & F_ACT);
  if (!pool && !(GMC && unconf)) return;
  double* m = P.kf + ((size_t)s * P.T + slot) * KF_STRIDE;
  double2* m2 = (double2*)m;
  double mm[8];
  for (int q = 0; q < 4; q++) { const double2 t = m2[q]; mm[2 * q] = t.x; mm[2 * q + 1] = t.y; }
  uint32_t nf = f;
  if (pool) {
    if (st_of(f) != ST_TRACKED) {
      if (KIND == KIND_BOT) mm[6] = 0.0;
      mm[7] = 0.0;
    }
    // the covariance predict is deferred (pending count + the process-noise operands).  All
    // pending predicts after the first see the same (w, h) | h: a track without an update is
    // Lost from its next predict on, which zeroes the size velocities (v_w, v_h | v_h) first —
    // so two operand pairs describe any number of pending predicts exactly.
    int pend = pend_of(f);
    if (pend == 65535) {  // counter full (a lost track predicted 65535 times without an update)
      kf_materialize_mem(KIND, m, pend);
      pend = 0;
      nf &= ~F_PEND_MASK;
    }
    if (pend == 0) m2[KF_QM / 2] = make_double2(mm[2], mm[3]);
    else m2[KF_QM2 / 2] = make_double2(mm[2], mm[3]);
    for (int k = 0; k < 4; k++) mm[k] = mm[k] + mm[k + 4];
    nf = (nf | F_PRED) + F_PEND1;
  }
  if (GMC) {  // mean = R8·mean + t
    for (int q = 0; q < 4; q++) {
      double a0 = H[0] * mm[2 * q] + H[1] * mm[2 * q + 1];
      double a1 = H[3] * mm[2 * q] + H[4] * mm[2 * q + 1];
      mm[2 * q] = a0;
      mm[2 * q + 1] = a1;
    }
    mm[0] += H[2];
    mm[1] += H[5];
    nf |= F_GMC;
  }
  for (int q = 0; q < 4; q++) m2[q] = make_double2(mm[2 * q], mm[2 * q + 1]);
  P.flags[(size_t)s * P.T + slot] = nf;
}
template <int KIND, bool GMC>
__global__ __launch_bounds__(WG) void predict_kernel(Dev P, int seq0,
                                                     const double* __restrict__ warps) {
  const int b = blockIdx.x, s = seq0 + b, T = P.T;
  const int slot = blockIdx.y * WG + threadIdx.x;
  if (slot >= T) return;
  predict_slot<KIND, GMC>(P, s, slot, P.flags[(size_t)s * T + slot],
                          GMC ? warps + 6 * (size_t)b : nullptr);
}

// Without a CMC warp there is no K4b: a pool track without an update keeps its covariance
// predicts pending (a Lost track's covariance is only read again when it is re-found, K4, or
// when the host reads the state, materialize_kernel), so each frame touches the covariance of
// updated tracks only.  The pending predicts are applied in their original order with their
// original operands, so the result is bit-identical to predicting every frame.
// K4b (CMC warp frames): the pending predicts then the warp of pool tracks that got no update
// record, and the warp alone for unconfirmed tracks (multi_gmc, botsort.py:192-195): the warp
// does not commute with later predicts, so nothing stays pending across it.  Thread per slot.
template <int KIND>
__global__ __launch_bounds__(WG) void cov_predict_gmc_kernel(Dev P, int seq0,
                                                             const double* __restrict__ warps) {
  const int b = blockIdx.x, s = seq0 + b, T = P.T;
  const int slot = blockIdx.y * WG + threadIdx.x;
  if (slot >= T) return;
  uint32_t* fp = P.flags + (size_t)s * T + slot;
  const uint32_t f = *fp;
  if ((f & F_REC) || !(f & (F_PRED | F_GMC))) return;
  double* m = P.kf + ((size_t)s * T + slot) * KF_STRIDE;
  kf_materialize(KIND, m, pend_of(f));
  if (f & F_GMC) gmc_cov(warps + 6 * (size_t)b, m + 8);
  *fp = f & ~F_PEND_MASK;
}
// the host reads covariances (bx_engine_tracks_host): apply every pending predict first
template <int KIND>
__global__ __launch_bounds__(WG) void materialize_kernel(Dev P, int s) {
  const int T = P.T, slot = blockIdx.x * WG + threadIdx.x;
  if (slot >= T) return;
  uint32_t* fp = P.flags + (size_t)s * T + slot;
  const uint32_t f = *fp;
  if (!pend_of(f)) return;
  kf_materialize(KIND, P.kf + ((size_t)s * T + slot) * KF_STRIDE, pend_of(f));
  *fp = f & ~F_PEND_MASK;
}

// ------------------------------------------------------------------------------------------
// K3: the sequential heart of a frame, one workgroup per sequence: detection split, track lists,
// the three assignments (candidate CSR, exact fp64 costs, lapx-semantics LAP), state/list
// bookkeeping, id allocation.  Kalman/feature work is emitted as update records for K4/K5.
// HELP: the LAP's wave solver on the helper waves 1..3 (crowded scenes); without it the
// components for the wave solver run on wave 0 after its lanes (the host picks the build from the
// LAPs' marks, DESIGN §2.3: the helper machinery costs an uncrowded frame ~2.5 us of K3)
template <int KIND, bool HELP>
__global__ __launch_bounds__(WG) void assoc_kernel(Dev P, int seq0, const float* __restrict__ dets,
                                                   const int* __restrict__ det_off) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int T = P.T, D = P.D;
  const LdsA Lo(T, D, P.elds);
  uint16_t* s_act = (uint16_t*)(smem + Lo.o_act);
  uint16_t* s_lost = (uint16_t*)(smem + Lo.o_lost);
  uint16_t* s_unconf = (uint16_t*)(smem + Lo.o_unconf);
  uint16_t* s_pool = (uint16_t*)(smem + Lo.o_pool);
  uint16_t* s_rtr = (uint16_t*)(smem + Lo.o_rtr);
  uint16_t* s_lostl = (uint16_t*)(smem + Lo.o_lostl);
  uint16_t* s_refind = (uint16_t*)(smem + Lo.o_refind);
  uint16_t* s_newt = (uint16_t*)(smem + Lo.o_newt);
  uint32_t* s_flags = (uint32_t*)(smem + Lo.o_flags);
  int* s_fid = (int*)(smem + Lo.o_fid);
  uint8_t* s_mark = (uint8_t*)(smem + Lo.o_mark);
  int* s_rowptr = (int*)(smem + Lo.o_rowptr);
  int16_t* s_c4r = (int16_t*)(smem + Lo.o_c4r);
  uint16_t* s_srl = (uint16_t*)(smem + Lo.o_srl);
  int16_t* s_r4c = (int16_t*)(smem + Lo.o_r4c);
  double* s_dbox = (double*)(smem + Lo.o_dbox);
  float4* s_dboxf = (float4*)(smem + Lo.o_dboxf);
  float4* s_tboxf = (float4*)(smem + Lo.o_tboxf);
  double* s_dconf = (double*)(smem + Lo.o_dconf);
  uint8_t* s_dkind = (uint8_t*)(smem + Lo.o_dkind);
  uint16_t* s_hd = (uint16_t*)(smem + Lo.o_hd);
  uint16_t* s_sd = (uint16_t*)(smem + Lo.o_sd);
  uint16_t* s_rem = (uint16_t*)(smem + Lo.o_rem);
  uint16_t* s_ecol = (uint16_t*)(smem + Lo.o_ecol);
  double* s_ecost = (double*)(smem + Lo.o_ecost);
  int* I = (int*)(smem + Lo.o_ints);
  int* scan_tmp = I + I_SCAN;

  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const int s = seq0 + b;
  const size_t sT = (size_t)s * T;
  int* seq = P.seq + (size_t)s * SQ_STRIDE;
  uint32_t* g_flags = P.flags + sT;
  int* g_fid = P.frame_id + sT;
  const double* g_kf = P.kf + (size_t)s * T * KF_STRIDE;
  int2* g_rec = P.rec + (size_t)s * D;
  const bool REID = (KIND == KIND_BOT) && P.with_reid;

  const int d0 = det_off[b], N = det_off[b + 1] - det_off[b];
  const float* fdets = dets + (size_t)d0 * 6;

  BX_STAMP(0);
  // ---------------- P0: sequence state → LDS
  if (tid == 0) {
    I[I_NA] = seq[SQ_NA];
    I[I_NL] = seq[SQ_NL];
    I[I_FC] = seq[SQ_FC] + 1;
    I[I_IDC] = seq[SQ_IDC];
    I[I_ERR] = 0;
  }
  __syncthreads();
  const int na = I[I_NA], nl = I[I_NL], fc = I[I_FC];
  if (N > D || N < 0) {  // host checks det_cap; never trust it blindly
    if (tid == 0) {
      seq[SQ_SKIP] = 1;
      seq[SQ_NREC] = 0;
      atomicOr(P.status, 1 << BX_ERR_CAPACITY);
    }
    return;
  }
  for (int k = tid; k < na; k += WG) s_act[k] = P.act[sT + k];
  for (int k = tid; k < nl; k += WG) s_lost[k] = P.lost[sT + k];
  for (int k = tid; k < T; k += WG) {
    s_flags[k] = g_flags[k];
    s_fid[k] = g_fid[k];
    s_mark[k] = 0;
  }

  // ---------------- P1: detections (float32-rounded by setup_decorator) and conf splits
  for (int k = tid; k < N; k += WG) {
    const float* r = fdets + 6 * k;
    double xyxy[4] = {(double)r[0], (double)r[1], (double)r[2], (double)r[3]};
    double conf = (double)r[4];
    double xywh[4], box[4];
    xyxy2xywh(xyxy, xywh);
    xywh2xyxy(xywh, box);  // STrack.xyxy of a detection (mean is None)
    for (int q = 0; q < 4; q++) s_dbox[4 * k + q] = box[q];
    s_dboxf[k] = make_float4(__double2float_rd(box[0]), __double2float_rd(box[1]),
                             __double2float_ru(box[2]), __double2float_ru(box[3]));
    s_dconf[k] = conf;
    uint8_t kd = 0;
    if (conf > P.high) kd = 1;
    else if (conf > P.low && conf < P.high) kd = 2;
    s_dkind[k] = kd;
  }
  __syncthreads();
  const int Dh = block_compact(N, [&](int k) { return s_dkind[k] == 1; },
                               [&](int k, int p) { s_hd[p] = (uint16_t)k; }, scan_tmp);
  const int Ds = block_compact(N, [&](int k) { return s_dkind[k] == 2; },
                               [&](int k, int p) { s_sd[p] = (uint16_t)k; }, scan_tmp);

  BX_STAMP(1);
  // ---------------- P2: unconfirmed / strack_pool = joint(tracked, lost)
  const int ntr = block_compact(na, [&](int k) { return (s_flags[s_act[k]] & F_ACT) != 0; },
                                [&](int k, int p) {
                                  s_pool[p] = s_act[k];
                                  s_mark[s_act[k]] |= M_POOL;
                                },
                                scan_tmp);
  const int nun = block_compact(na, [&](int k) { return (s_flags[s_act[k]] & F_ACT) == 0; },
                                [&](int k, int p) { s_unconf[p] = s_act[k]; }, scan_tmp);
  const int npl = block_compact(nl, [&](int k) { return !(s_mark[s_lost[k]] & M_POOL); },
                                [&](int k, int p) { s_pool[ntr + p] = s_lost[k]; }, scan_tmp);
  const int npool = ntr + npl;
  for (int k = tid; k < npool; k += WG) s_mark[s_pool[k]] &= ~M_POOL;
  BX_STAMP(2);

  // LAP workspace (rows use s_c4r/s_u/s_srl, columns s_r4c/s_v/s_spc/...)
  LapWS W;
  W.row_ptr = lds_ptr<int>(s_rowptr); W.ecol = lds_ptr<uint16_t>(s_ecol);
  W.ecost = lds_ptr<double>(s_ecost);
  W.gcol = P.gcol + (size_t)s * T * D; W.gcost = P.gcost + (size_t)s * T * D;
  W.elds = P.elds; W.col4row = lds_ptr<int16_t>(s_c4r); W.row4col = lds_ptr<int16_t>(s_r4c);
  W.u = lds_ptr<double>(smem + Lo.o_u); W.v = lds_ptr<double>(smem + Lo.o_v);
  W.spc = lds_ptr<double>(smem + Lo.o_spc); W.path = lds_ptr<int16_t>(smem + Lo.o_path);
  W.colflag = lds_ptr<uint8_t>(smem + Lo.o_colf); W.touched = lds_ptr<uint16_t>(smem + Lo.o_touch);
  W.srlist = lds_ptr<uint16_t>(s_srl); W.coldeg = lds_ptr<int>(smem + Lo.o_cdeg);
  W.roots = lds_ptr<uint16_t>(smem + Lo.o_roots);
  W.rlab = lds_ptr<int>(smem + Lo.o_rlab);
  W.colaux = lds_ptr<int>(smem + Lo.o_colaux);
  W.colmin = lds_ptr<int>(smem + Lo.o_colmin);
  W.comp_stats = P.lap_stats ? seq + SQ_NCOMP17 : nullptr;  // (off: no reductions, no atomics)
  // the LAP's helper-wave scratch in the candidate sweep's LDS (tboxf .. dconf: dead while the
  // LAP runs; lap_helper_bytes(hT, tws) <= 16 T + 18 D, asserted by the host layout check)
  W.hs = lds_ptr<int>(smem + Lo.o_tboxf);
  W.hT = HELP ? (T + 7) & ~7 : 0;
  W.tws = (D + 7) & ~7;
  W.bigmark = P.lapmark;
  W.stamp = P.lapstamp;
  uint16_t* e_gcol = P.gcol + (size_t)s * T * D;
  double* e_gcost = P.gcost + (size_t)s * T * D;
  auto put_edge = [&](int e, int col, double cost) {
    if (e < P.elds) { s_ecol[e] = (uint16_t)col; s_ecost[e] = cost; }
    else { e_gcol[e - P.elds] = (uint16_t)col; e_gcost[e - P.elds] = cost; }
  };
  auto get_edge = [&](int e, int& col, double& cost) {
    if (e < P.elds) { col = s_ecol[e]; cost = s_ecost[e]; }
    else { col = e_gcol[e - P.elds]; cost = e_gcost[e - P.elds]; }
  };

  // Build the admissible-edge CSR for rows (slots rows[0..R)) x cols (det indices cols[0..C)),
  // then solve.  mode: 0 = IoU distance, 1 = fused (fuse_score), 2 = BoT-SORT first
  // association, 3 = BoT-SORT unconfirmed association.
  auto associate = [&](const uint16_t* rows, int R, const uint16_t* cols, int C, double L,
                       int mode, int stamp) {
    const bool reid = REID && (mode == 2 || mode == 3);
    // non-overlapping pairs have IoU 0: cost >= 1, never admissible nor tied with L (so L below
    // 1 by more than the tie tolerance), never gated (prox < 1)
    const bool prefilter = L < 1.0 - BX_TIE_EPS && (!reid || P.prox < 1.0);
    // the reference's cost of (track box tb, detection dk) — iou_distance, fuse_score, and for
    // BoT-SORT with ReID np.minimum with the gated embedding distance (1 where not gated)
    auto pair_cost = [&](const double* tb, int slot, int dk) -> double {
      double c = 1 - iou_pair(tb, s_dbox + 4 * dk);
      if (mode == 1) {
        c = fuse_one(c, s_dconf[dk]);
      } else if (mode >= 2) {
        const bool gated = reid && !(c > P.prox);
        if (mode == 3 || P.fuse_first) c = fuse_one(c, s_dconf[dk]);
        if (reid) {
          const double ed = gated ? P.etab[((size_t)s * T + slot) * D + dk] : 1.0;
          c = c < ed ? c : ed;  // np.minimum(ious_dists, emb_dists)
        }
      }
      return c;
    };
    // Candidates: a conservative fp32 intersection test on outward-rounded boxes (never misses
    // an fp64-intersecting pair); exact fp64 costs are then computed once per candidate with
    // every lane busy; candidates that turn out inadmissible stay in the CSR with cost INF,
    // which the solver treats as absent.  One thread per row walks the columns in order
    // (column boxes broadcast from LDS), so a row's candidates come out in column order.
    float4* s_cbox = (float4*)(smem + Lo.o_cbox);
    int* s_bin = (int*)(smem + Lo.o_bin);  // [NBIN + 1] starts, then [NBIN] cursors
    uint16_t* s_bcol = (uint16_t*)(smem + Lo.o_bcol);
    if (tid == 0) { I[I_XMIN] = INT_MAX; I[I_XMAX] = INT_MIN; I[I_W] = INT_MIN; }
    if (tid < NBIN) s_bin[tid] = 0;
    for (int j = tid; j < C; j += WG) s_cbox[j] = s_dboxf[cols[j]];
    for (int i = tid; i < R; i += WG) {
      double t[4];
      track_box<KIND>(g_kf, rows[i], t);
      s_tboxf[i] = make_float4(__double2float_rd(t[0]), __double2float_rd(t[1]),
                               __double2float_ru(t[2]), __double2float_ru(t[3]));
    }
    __syncthreads();
    if (stamp == 4) BX_STAMP(20);
    auto hit = [&](const float4& tb, const float4& db) -> bool {
      if (!prefilter) return true;
      return (fminf(tb.z, db.z) > fmaxf(tb.x, db.x)) & (fminf(tb.w, db.w) > fmaxf(tb.y, db.y));
    };
    // Column x-binning: a candidate needs db.x1 < tb.x2 and db.x2 > tb.x1, so with wmax >= every
    // column's width its x1 lies in (tb.x1 - wmax, tb.x2): a row scans only the bins covering that
    // range (the bin map is monotone in x; bounds rounded outward).  Non-finite boxes or no
    // prefilter: every row scans every column.
    auto okey = [](float f) {  // order-preserving float → int
      const int i = __builtin_bit_cast(int, f);
      return i >= 0 ? i : i ^ 0x7fffffff;
    };
    auto ofloat = [](int k) { return __builtin_bit_cast(float, k >= 0 ? k : k ^ 0x7fffffff); };
    if (prefilter) {
      int kmin = INT_MAX, kmax = INT_MIN, kw = INT_MIN;
      for (int j = tid; j < C; j += WG) {
        const float4 cb = s_cbox[j];
        kmin = min(kmin, okey(cb.x));
        kmax = max(kmax, okey(cb.x));
        kw = max(kw, okey(nextafterf(__double2float_ru((double)cb.z - (double)cb.x), INFINITY)));
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        kmin = min(kmin, __shfl_xor(kmin, d));
        kmax = max(kmax, __shfl_xor(kmax, d));
        kw = max(kw, __shfl_xor(kw, d));
      }
      if (lane_id() == 0) {
        atomicMin(&I[I_XMIN], kmin);
        atomicMax(&I[I_XMAX], kmax);
        atomicMax(&I[I_W], kw);
      }
      __syncthreads();
    }
    const float xmin = ofloat(I[I_XMIN]), xmax = ofloat(I[I_XMAX]), wmax = ofloat(I[I_W]);
    const bool binned = prefilter && C > 0 && isfinite(xmin) && isfinite(xmax) && isfinite(wmax) &&
                        wmax >= 0.f;
    const float inv = xmax > xmin ? (float)NBIN / (xmax - xmin) : 0.f;
    auto bin = [&](float x) {
      const float t = (x - xmin) * inv;
      return !(t > 0.f) ? 0 : (t >= (float)NBIN ? NBIN - 1 : (int)t);
    };
    int* s_bcur = s_bin + NBIN + 1;
    if (binned) {
      for (int j = tid; j < C; j += WG) atomicAdd(&s_bin[bin(s_cbox[j].x)], 1);
      __syncthreads();
      if (wave_id() == 0) {  // NBIN == WAVE: one exclusive scan step
        const int lane = lane_id(), v = s_bin[lane];
        int x = v;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
          const int y = __shfl_up(x, d);
          if (lane >= d) x += y;
        }
        s_bin[lane] = x - v;
        s_bcur[lane] = x - v;
        if (lane == WAVE - 1) s_bin[NBIN] = x;
      }
      __syncthreads();
      for (int j = tid; j < C; j += WG) s_bcol[atomicAdd(&s_bcur[bin(s_cbox[j].x)], 1)] = j;
      __syncthreads();
    }
    // visit the candidate columns of row box tb (binned: bin order, else column order)
    auto scan_row = [&](const float4& tb, auto&& on_hit) {
      if (binned) {
        const float lo =
            nextafterf(__double2float_rd((double)tb.x - (double)wmax), -INFINITY);
        const int b0 = bin(lo), b1 = bin(tb.z);
        for (int k = s_bin[b0]; k < s_bin[b1 + 1]; k++) {
          const int j = s_bcol[k];
          if (hit(tb, s_cbox[j])) on_hit(j);
        }
      } else {
        for (int j = 0; j < C; j++)
          if (hit(tb, s_cbox[j])) on_hit(j);
      }
    };
    // pass 1: count candidates per row (one thread per row)
    for (int i = tid; i < R; i += WG) {
      int cnt = 0;
      scan_row(s_tboxf[i], [&](int) { cnt++; });
      s_rowptr[i] = cnt;
    }
    __syncthreads();
    if (stamp == 4) BX_STAMP(21);
    wave0_exclusive_scan(s_rowptr, R);
    __syncthreads();
    if (stamp == 4) BX_STAMP(22);
    // pass 2: write each row's candidate columns, sorted ascending (the solver's tie-breaking
    // follows edge order); the row index is parked in the cost slot
    for (int i = tid; i < R; i += WG) {
      const int e0 = s_rowptr[i];
      int e = e0;
      scan_row(s_tboxf[i], [&](int j) { put_edge(e++, j, (double)i); });
      if (binned)
        for (int a = e0 + 1; a < e; a++) {  // insertion sort (a row has few candidates)
          int ca, cb;
          double d;
          get_edge(a, ca, d);
          int q = a - 1;
          for (; q >= e0; q--) {
            get_edge(q, cb, d);
            if (cb < ca) break;
            put_edge(q + 1, cb, d);
          }
          put_edge(q + 1, ca, d);
        }
    }
    __syncthreads();
    if (stamp == 4) BX_STAMP(23);
    // pass 3: exact fp64 cost per candidate; a gated pair (botsort.py:209-214) takes
    // min(iou cost, embedding distance) with the distance K1c precomputed for it.  A cost within
    // the tie tolerance of L (gain 0) makes the optimum non-unique by itself.
    const int E = s_rowptr[R];
    bool at_limit = false;
    for (int e = tid; e < E; e += WG) {
      int j;
      double ri;
      get_edge(e, j, ri);
      const int i = (int)ri;
      double tb[4];
      track_box<KIND>(g_kf, rows[i], tb);
      const double c = pair_cost(tb, rows[i], cols[j]);
      at_limit |= fabs(c - L) <= BX_TIE_EPS;
      put_edge(e, j, c < L ? c : INF);
    }
    __syncthreads();
    BX_STAMP(stamp);
#ifdef BX_PHASE_TIMING
    W.dbg = (stamp == 4 && P.dbg) ? P.dbg + (size_t)s * BX_DBG_STRIDE + 26 : nullptr;
#endif
    lap_solve_block(R, C, L, W, scan_tmp);
    if (lap_tied_block(R, C, L, W, scan_tmp, at_limit)) {
      // Tied optimum: lapx's own lapjv on the (R+C)^2 extension (matching.py:54-61), its state
      // in this sequence's global scratch, the exact R x C cost block in gcost (the CSR is done).
      double* M = e_gcost;
      for (int k = tid; k < R * C; k += WG) {
        const int i = k / C, j = k - i * C;
        double tb[4];
        track_box<KIND>(g_kf, rows[i], tb);
        M[k] = pair_cost(tb, rows[i], cols[j]);
      }
      __syncthreads();
      // row classes for the solver's scan skip (jv_wave_t): the dummy rows (0), and the real rows
      // whose every cost equals the first constant row's (1: a track with no candidate pair, all
      // 1.0 — most rows of a crowded scene); in the SSP's root list, dead until the next solve
      uint16_t* s_cls = (uint16_t*)(smem + Lo.o_roots);
      for (int i = tid; i < R; i += WG) {
        const double c0 = M[(size_t)i * C];
        bool cst = isfinite(c0);
        for (int j = 1; j < C && cst; j++) cst = M[(size_t)i * C + j] == c0;
        s_cls[i] = cst ? 1 : 0;
      }
      __syncthreads();
      if (tid == 0) {
        int i0 = 0;
        while (i0 < R && !s_cls[i0]) i0++;
        I[I_CLS0] = i0;
      }
      __syncthreads();
      {
        const int i0 = I[I_CLS0];
        const double K = i0 < R ? M[(size_t)i0 * C] : 0.0;
        for (int i = tid; i < R; i += WG) s_cls[i] = s_cls[i] && M[(size_t)i * C] == K ? 1 : 0;
      }
      __syncthreads();
      auto rk = [&](int i) { return i >= R ? 0 : (s_cls[i] ? 1 : -1); };
      // lapx's state in this association's LAP workspace and candidate-sweep LDS, which are dead
      // until the next association rebuilds them (three blocks: see LdsA's take order), when it
      // fits; else in the sequence's global scratch (one wave either way)
      const int n = R + C;
      const bool in_lds = jv_split_d_bytes(n) <= Lo.o_flags - Lo.o_u &&
                          jv_split_a_bytes(n) <= Lo.o_dconf - Lo.o_tboxf &&
                          jv_split_b_bytes(n) <= Lo.o_ints - Lo.o_rowptr;
      const double half = L / 2.;
      const JvExt ext{M, R, C, half};
#ifdef BX_PHASE_TIMING
      // (the diagnostic timing build solves in the same state layout through two call sites,
      // one per layout: with the stamps added, one call over a selected LDS-or-global state
      // pointer hits an instruction-selection error in this compiler — a generic-pointer
      // aperture compare given an SGPR operand)
      JvLds jw_l = jv_bind_split(smem + Lo.o_u, smem + Lo.o_tboxf, smem + Lo.o_rowptr, n);
      JvLds jw_g = jv_bind(P.jvs + (size_t)s * P.jvs_stride, n);
      if (wave_id() == 0) {
        if (in_lds) jv_wave_t(ext, n, jw_l, SyncWaveLG{false}, rk);
        else jv_wave_t(ext, n, jw_g, SyncWaveLG{true}, rk);
      }
      JvLds& jw = in_lds ? jw_l : jw_g;
#else
      JvLds jw = in_lds ? jv_bind_split(smem + Lo.o_u, smem + Lo.o_tboxf, smem + Lo.o_rowptr, n)
                        : jv_bind(P.jvs + (size_t)s * P.jvs_stride, n);
      if (wave_id() == 0) jv_wave_t(ext, n, jw, SyncWaveLG{!in_lds}, rk);
#endif
      __syncthreads();
      // x >= C: unmatched (-1); a real partner above L is neither matched nor listed (-3)
      for (int i = tid; i < R; i += WG) {
        const int j = jw.x[i];
        s_c4r[i] = (int16_t)(j >= C ? -1 : (M[(size_t)i * C + j] <= L ? j : -3));
      }
      for (int j = tid; j < C; j += WG) {
        const int i = jw.y[j];
        s_r4c[j] = (int16_t)(i >= R ? -1 : (M[(size_t)i * C + j] <= L ? i : -3));
      }
      if (tid == 0) seq[SQ_NTIE]++;
    }
    __syncthreads();
  };

  // matched rows of the last solve (rows[i] ↔ cols[c4r[i]]): STrack.update / re_activate state
  // changes here, the Kalman/feature/score work as records for K4/K5 (row order)
  int nrec = 0;
  auto record_matches = [&](const uint16_t* rows, int R, const uint16_t* cols, bool feat,
                            bool refind) {
    const int base = nrec;
    nrec += block_compact(
        R, [&](int i) { return s_c4r[i] >= 0; },
        [&](int i, int p) {
          const int slot = rows[i], dk = cols[s_c4r[i]];
          const uint32_t fl = s_flags[slot];
          const bool tracked = st_of(fl) == ST_TRACKED;
          s_flags[slot] = (fl & ~F_STATE) | ST_TRACKED | F_ACT | F_REC;
          s_fid[slot] = fc;
          if (refind && !tracked) s_mark[slot] |= M_TMP;
          const int kind = (tracked ? R_UPDATE : R_REACT) | (feat ? R_FEAT : 0);
          g_rec[base + p] = make_int2(slot | (kind << 16), dk);
        },
        scan_tmp);
  };

  // ---------------- P4..P8: the three associations (bytetrack.py:199-276, botsort.py:198-366)
  //   0: strack_pool x high dets (fused / BoT first association), match_thresh
  //   1: r_tracked x low-confidence dets, IoU, 0.5
  //   2: unconfirmed x remaining high dets (fused), 0.7
  // as ONE loop, so the candidate build and the solver exist once in the kernel's code
  int nref = 0, nrem = 0, nrtr = 0, nlostl = 0;
  for (int stage = 0; stage < 3; stage++) {
    const uint16_t* rows = stage == 0 ? s_pool : stage == 1 ? s_rtr : s_unconf;
    const int R = stage == 0 ? npool : stage == 1 ? nrtr : nun;
    const uint16_t* cols = stage == 0 ? s_hd : stage == 1 ? s_sd : s_rem;
    const int C = stage == 0 ? Dh : stage == 1 ? Ds : nrem;
    const double L = stage == 0 ? P.match_thresh : stage == 1 ? 0.5 : 0.7;
    const int mode = stage == 1 ? 0 : KIND == KIND_BYTE ? 1 : stage == 0 ? 2 : 3;
    if (stage == 0) BX_STAMP(3);
    if (stage == 1) BX_STAMP(6);
    if (stage == 2) BX_STAMP(8);
    associate(rows, R, cols, C, L, mode, stage == 0 ? 4 : stage == 1 ? 7 : 9);
    if (stage == 0) BX_STAMP(5);
    if (stage == 2) {
      BX_STAMP(10);
      for (int i = tid; i < nun; i += WG) {
        if (s_c4r[i] != -1) continue;  // u_unconfirmed = rows with x < 0 (-3: neither)
        const int slot = s_unconf[i];
        s_flags[slot] = (s_flags[slot] & ~F_STATE) | ST_REMOVED;  // mark_removed
        s_mark[slot] |= M_REMNOW;
      }
    }
    // second-stage dets carry no features
    record_matches(rows, R, cols, REID && stage != 1, stage == 0);
    if (stage == 0) {
      nref = block_compact(npool, [&](int k) { return (s_mark[s_pool[k]] & M_TMP) != 0; },
                           [&](int k, int p) { s_refind[p] = s_pool[k]; }, scan_tmp);
      // remaining high dets (u_detection, ascending) — saved before the next solve reuses r4c
      nrem = block_compact(Dh, [&](int j) { return s_r4c[j] == -1; },
                           [&](int j, int p) { s_rem[p] = s_hd[j]; }, scan_tmp);
      for (int k = tid; k < nref; k += WG) s_mark[s_refind[k]] &= ~M_TMP;
      // r_tracked = unmatched pool rows still Tracked
      nrtr = block_compact(
          npool, [&](int k) { return s_c4r[k] == -1 && st_of(s_flags[s_pool[k]]) == ST_TRACKED; },
          [&](int k, int p) { s_rtr[p] = s_pool[k]; }, scan_tmp);
    } else if (stage == 1) {
      nlostl = block_compact(
          nrtr, [&](int k) { return s_c4r[k] == -1; },
          [&](int k, int p) {
            const int slot = s_rtr[k];
            s_lostl[p] = (uint16_t)slot;
            s_flags[slot] = (s_flags[slot] & ~F_STATE) | ST_LOST;  // mark_lost
          },
          scan_tmp);
    }
  }

  // ---------------- P9: new tracks from the detections left over (conf >= det/new thresh)
  const int nnew = block_compact(
      nrem, [&](int k) { return s_r4c[k] == -1 && s_dconf[s_rem[k]] >= P.new_thresh; },
      [&](int k, int p) { s_newt[p] = s_rem[k]; /* det index for now */ }, scan_tmp);
  // allocate the first nnew free slots (ascending)
  {
    int base = 0;
    for (int c = 0; c < T && base < nnew; c += WG) {
      int k = c + tid;
      bool f = k < T && !(s_flags[k] & F_INUSE);
      int tot;
      int pos = block_scan_flag(f, scan_tmp, tot);
      if (f && base + pos < nnew) s_rtr[base + pos] = (uint16_t)k;  // s_rtr reused: slots
      base += tot;
    }
    if (tid == 0 && base < nnew) {
      I[I_ERR] = 1;
      atomicOr(P.status, 1 << BX_ERR_TRACK_OVERFLOW);
    }
  }
  __syncthreads();
  const int nnew_ok = I[I_ERR] ? 0 : nnew;
  const int idc0 = I[I_IDC];
  for (int p = tid; p < nnew_ok; p += WG) {  // STrack.activate (state, ids, frames)
    const int dk = s_newt[p], slot = s_rtr[p];
    P.id[sT + slot] = idc0 + 1 + p;
    P.start[sT + slot] = fc;
    s_flags[slot] = ST_TRACKED | F_INUSE | (fc == 1 ? F_ACT : 0u);
    s_fid[slot] = fc;
    g_rec[nrec + p] = make_int2(slot | ((R_NEW | (REID ? R_FEAT : 0)) << 16), dk);
    s_newt[p] = (uint16_t)slot;
  }
  nrec += nnew_ok;
  __syncthreads();

  BX_STAMP(11);
  // ---------------- P10: lost tracks past the buffer → removed
  for (int k = tid; k < nl; k += WG) {
    const int slot = s_lost[k];
    if (fc - s_fid[slot] > P.max_time_lost) {
      s_flags[slot] = (s_flags[slot] & ~F_STATE) | ST_REMOVED;
      s_mark[slot] |= M_REMNOW;
    }
  }
  __syncthreads();

  // ---------------- P11: list rebuild (bytetrack.py:278-289 / botsort.py:392-403), written to
  // act2/lost2 for K6's remove_duplicate_stracks
  // act2 = [t in active if Tracked] ++ new tracks ++ refind    (joint_stracks x2)
  uint16_t* g_act2 = P.act2 + sT;
  uint16_t* g_lost2 = P.lost2 + sT;
  int nact2 = block_compact(na, [&](int k) { return st_of(s_flags[s_act[k]]) == ST_TRACKED; },
                            [&](int k, int p) {
                              g_act2[p] = s_act[k];
                              s_mark[s_act[k]] |= M_ACT2;
                            },
                            scan_tmp);
  for (int k = tid; k < nnew_ok; k += WG) {
    g_act2[nact2 + k] = s_newt[k];
    s_mark[s_newt[k]] |= M_ACT2;
  }
  nact2 += nnew_ok;
  __syncthreads();
  nact2 += block_compact(nref, [&](int k) { return !(s_mark[s_refind[k]] & M_ACT2); },
                         [&](int k, int p) {
                           g_act2[nact2 + p] = s_refind[k];
                           s_mark[s_refind[k]] |= M_ACT2;
                         },
                         scan_tmp);
  // lost = sub(lost, active) ++ lost_local, then sub(., removed_stracks) with the removed list
  // of earlier frames only (F_INREM): the reference extends removed_stracks afterwards
  int nlost2 = block_compact(
      nl, [&](int k) { return !(s_mark[s_lost[k]] & M_ACT2) && !(s_flags[s_lost[k]] & F_INREM); },
      [&](int k, int p) { g_lost2[p] = s_lost[k]; }, scan_tmp);
  nlost2 += block_compact(nlostl, [&](int k) { return !(s_flags[s_lostl[k]] & F_INREM); },
                          [&](int k, int p) { g_lost2[nlost2 + p] = s_lostl[k]; }, scan_tmp);
  // removed_stracks.extend(removed_local); write back slot state
  for (int k = tid; k < T; k += WG) {
    uint32_t f = s_flags[k];
    if (s_mark[k] & M_REMNOW) f |= F_INREM;
    g_flags[k] = f;
    g_fid[k] = s_fid[k];
  }
  if (tid == 0) {
    seq[SQ_FC] = fc;
    seq[SQ_IDC] = idc0 + nnew_ok;
    seq[SQ_NA2] = nact2;
    seq[SQ_NL2] = nlost2;
    seq[SQ_NREC] = nrec;
    seq[SQ_NHIGH] = Dh;
    seq[SQ_NDET] = N;
    seq[SQ_SKIP] = 0;
    if (I[I_ERR]) seq[SQ_STATUS] |= 1 << BX_ERR_TRACK_OVERFLOW;
  }
  BX_STAMP(12);
}

// ------------------------------------------------------------------------------------------
// K4: per update record, STrack.update / re_activate / activate numerics: Kalman update
// (base_kalman_filter.py:129-155, after K2's deferred covariance predict + CMC warp) or
// initiate, tracklet_len, score, cls (+ BoT-SORT update_cls, botsort_track.py:51-64), det_ind.
// Eight lanes per record: lane r owns covariance row r (and mean[r]); the 4x4 innovation
// covariance and the Kalman gain rows are exchanged with in-group shuffles, every entry being
// the same expression kf_predict_soa / kf_update_soa evaluate.  Grid (n_seq, ceil(D/32)).
constexpr int UPD_PER_BLOCK = WG / 8;
template <int KIND>
__global__ __launch_bounds__(WG) void update_kernel(Dev P, int seq0, const float* __restrict__ dets,
                                                    const int* __restrict__ det_off,
                                                    const double* __restrict__ warps) {
  const int b = blockIdx.x, s = seq0 + b, T = P.T;
  const int ri = blockIdx.y * UPD_PER_BLOCK + (threadIdx.x >> 3), r = threadIdx.x & 7;
  const int* seq = P.seq + (size_t)s * SQ_STRIDE;
  if (ri >= seq[SQ_NREC]) return;  // whole 8-lane groups leave together
  const int2 rc = P.rec[(size_t)s * P.D + ri];
  const int slot = rc.x & 0xffff, kind = (rc.x >> 16) & 3, dk = rc.y;
  const size_t sT = (size_t)s * T;
  const float* row = dets + (size_t)(det_off[b] + dk) * 6;
  double meas[4];
  det_measurement<KIND>(row, meas);
  double* m = P.kf + ((size_t)s * T + slot) * KF_STRIDE;
  double2* crow = (double2*)(m + 8 + 8 * r);  // this lane's covariance row
  const double conf = (double)row[4], cls = (double)row[5];
  double* h = P.clsh + (sT + slot) * CLS_HIST * 2;
  auto shfl = [&](double v, int src) { return __shfl(v, src, 8); };
  if (kind == R_NEW) {  // kf_initiate (kf_initiate's expressions): mean = [z, 0], cov = diag(std^2)
    double dr;
    if (KIND == KIND_BYTE)
      dr = r == 2 ? 1e-2 : r == 6 ? 1e-5 : (r < 4 ? 2 * STD_POS : 10 * STD_VEL) * meas[3];
    else
      dr = (r < 4 ? 2 * STD_POS : 10 * STD_VEL) * ((r & 1) ? meas[3] : meas[2]);
    const double mz = r == 0 ? meas[0] : r == 1 ? meas[1] : r == 2 ? meas[2] : r == 3 ? meas[3]
                                                                                         : 0.0;
    m[r] = mz;
    for (int q = 0; q < 4; q++)
      crow[q] = make_double2(2 * q == r ? dr * dr : 0.0, 2 * q + 1 == r ? dr * dr : 0.0);
    if (r == 0) {
      P.conf[sT + slot] = conf;
      P.detind[sT + slot] = dk;
      P.tlen[sT + slot] = 0;
      P.cls[sT + slot] = cls;
      if (KIND == KIND_BOT) {
        h[0] = cls;
        h[1] = conf;
        P.ncls[sT + slot] = 1;
      }
    }
    return;
  }
  const uint32_t fl = P.flags[sT + slot];
  double cr[8];
  for (int q = 0; q < 4; q++) { const double2 t = crow[q]; cr[2 * q] = t.x; cr[2 * q + 1] = t.y; }
  const int npend = pend_of(fl);
  if (r == 0 && npend) P.flags[sT + slot] = fl & ~F_PEND_MASK;
  for (int k = 0; k < npend; k++) {  // K2's pending predicts: rows i < 4 need row i + 4
    double o[8];
    for (int j = 0; j < 8; j++) o[j] = shfl(cr[j], (r + 4) & 7);
    const int qi = k ? KF_QM2 : KF_QM;
    double mv[4] = {0.0, 0.0, m[qi], m[qi + 1]}, q[8];
    kf_process_noise(KIND, mv, q);
    double nr[8];
    if (r < 4) {
      for (int j = 0; j < 4; j++) {
        double v = (cr[j] + o[j]) + (cr[j + 4] + o[j + 4]);
        nr[j] = (j == r) ? v + q[j] : v;
        nr[j + 4] = cr[j + 4] + o[j + 4];
      }
    } else {
      for (int j = 0; j < 4; j++) {
        nr[j] = cr[j] + cr[j + 4];
        nr[j + 4] = (j + 4 == r) ? cr[j + 4] + q[j + 4] : cr[j + 4];
      }
    }
    for (int j = 0; j < 8; j++) cr[j] = nr[j];
  }
  if (fl & F_GMC) {  // cov = R8·cov·R8ᵀ: row pairs (2b, 2b+1) mix, then column pairs
    const double* H = warps + 6 * (size_t)b;
    double o[8], rp[8];
    for (int j = 0; j < 8; j++) o[j] = shfl(cr[j], r ^ 1);
    for (int j = 0; j < 8; j++)
      rp[j] = (r & 1) ? H[3] * o[j] + H[4] * cr[j] : H[0] * cr[j] + H[1] * o[j];
    for (int bq = 0; bq < 4; bq++) {
      const double y0 = rp[2 * bq], y1 = rp[2 * bq + 1];
      cr[2 * bq] = y0 * H[0] + y1 * H[1];
      cr[2 * bq + 1] = y0 * H[3] + y1 * H[4];
    }
  }
  // kf_update_soa, distributed
  double mm[8];
  for (int q = 0; q < 8; q++) mm[q] = m[q];
  double rr[4], S[16], L[16];
  kf_meas_noise(KIND, mm, 0.0, rr);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      const double v = shfl(cr[j], i);
      S[4 * i + j] = v + (i == j ? rr[i] : 0.0);
    }
  const bool ok = chol4(S, L);
  if (ok) {
    double Kr[4], y[4];  // gain row r: solves on covariance row r's first four entries
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
    double innov[4];
    for (int k = 0; k < 4; k++) innov[k] = meas[k] - mm[k];
    double sm = 0.0;
    for (int k = 0; k < 4; k++) sm += innov[k] * Kr[k];
    const double mnew = m[r] + sm;
    double ks[4];
    for (int j = 0; j < 4; j++) {
      double sv = 0.0;
      for (int k = 0; k < 4; k++) sv += Kr[k] * S[4 * k + j];
      ks[j] = sv;
    }
    for (int j = 0; j < 8; j++) {
      double Kj[4];
      for (int k = 0; k < 4; k++) Kj[k] = shfl(Kr[k], j);
      double sv = 0.0;
      for (int k = 0; k < 4; k++) sv += ks[k] * Kj[k];
      cr[j] = cr[j] - sv;
    }
    m[r] = mnew;  // every lane has read mean[] above (same wave, in order)
  }
  for (int q = 0; q < 4; q++) crow[q] = make_double2(cr[2 * q], cr[2 * q + 1]);
  if (r != 0) return;
  P.conf[sT + slot] = conf;
  P.detind[sT + slot] = dk;
  P.tlen[sT + slot] = kind == R_REACT ? 0 : P.tlen[sT + slot] + 1;
  double out_cls = cls;
  if (KIND == KIND_BOT) {  // update_cls
    const int nh = P.ncls[sT + slot];
    double max_freq = 0.0;
    bool found = false;
    for (int q = 0; q < nh; q++) {
      if (cls == h[2 * q]) { h[2 * q + 1] += conf; found = true; }
      if (h[2 * q + 1] > max_freq) { max_freq = h[2 * q + 1]; out_cls = h[2 * q]; }
    }
    if (!found) {
      if (nh < CLS_HIST) { h[2 * nh] = cls; h[2 * nh + 1] = conf; P.ncls[sT + slot] = nh + 1; }
      else atomicOr(P.status, 1 << BX_ERR_TRACK_OVERFLOW);
      out_cls = cls;
    }
  }
  P.cls[sT + slot] = out_cls;
}

// ------------------------------------------------------------------------------------------
// K5: BoT-SORT feature update per record carrying a detection feature (botsort_track.py:40-49):
// a new track's smooth_feat = f2; otherwise feat = f2/|f2|; smooth = 0.9 smooth + 0.1 feat;
// smooth /= |smooth|.  f2 is recomputed from the input row with K1's norms (bit-identical).  The
// new smooth_feat's numpy float32 norm (embedding_distance's track-side scale) is refreshed here,
// while the row is in registers, for the next frame's K1c.  Grid (n_seq, FEAT_BLOCKS); one wave
// per record.
#ifndef BX_FEAT_BLOCKS
#define BX_FEAT_BLOCKS 16
#endif
constexpr int FEAT_BLOCKS = BX_FEAT_BLOCKS;
template <typename FT, bool NPF, int FC>
__global__ __launch_bounds__(WG) void feature_kernel(Dev P, int seq0,
                                                     const int* __restrict__ det_off,
                                                     const FT* __restrict__ embs) {
  __shared__ __align__(16) float s_w[NWAVE * REG_FP];
  const int b = blockIdx.x, s = seq0 + b, F = FC ? FC : P.F, D = P.D, T = P.T, lane = lane_id();
  const int nrec = P.seq[(size_t)s * SQ_STRIDE + SQ_NREC];
  const FT a = (FT)0.9, bb = (FT)(1.0 - 0.9);
  float* wb = s_w + wave_id() * REG_FP;
  const FT* fembs = embs + (size_t)det_off[b] * F;
  FT* feat = (FT*)P.feat + (size_t)s * T * F;
  constexpr int STEP = FEAT_BLOCKS * NWAVE;
  // this block's records (r = blockIdx.y*NWAVE + w + k*STEP) staged in LDS up front
  constexpr int RMAX = 64;
  __shared__ int2 s_rec[RMAX];
  const int nmine = nrec > (int)blockIdx.y * NWAVE
                        ? (nrec - (int)blockIdx.y * NWAVE + STEP - 1) / STEP * NWAVE : 0;
  for (int t = threadIdx.x; t < min(nmine, RMAX); t += WG) {
    const int r = blockIdx.y * NWAVE + (t % NWAVE) + (t / NWAVE) * STEP;
    s_rec[t] = r < nrec ? P.rec[(size_t)s * D + r] : make_int2(0, 0);
  }
  __syncthreads();
  auto rec = [&](int r) {
    const int t = (r - (int)blockIdx.y * NWAVE) / STEP * NWAVE + (r - (int)blockIdx.y * NWAVE) % STEP;
    return t < RMAX ? s_rec[t] : P.rec[(size_t)s * D + r];
  };
  auto next = [&](int r) {  // next record with a feature at or after r
    for (; r < nrec; r += STEP)
      if ((rec(r).x >> 16) & R_FEAT) return r;
    return nrec;
  };
  if (F <= REG_F) {
    for (int r = next(blockIdx.y * NWAVE + wave_id()); r < nrec; r = next(r + STEP)) {
      const int2 rc = rec(r);
      const int slot = rc.x & 0xffff, kind = rc.x >> 16, dk = rc.y;
      RegRow<FT> g, m;  // no prefetch of the next record: fewer VGPRs, more waves in flight
      g.load(fembs + (size_t)dk * F, F);
      FT* sm = feat + (size_t)slot * F;
      if ((kind & 3) != R_NEW) m.load(sm, F);
      const FT n1 = (FT)P.dnrm[((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4];
      const FT n2 = (FT)P.dnrm[((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4 + 1];
      g.div(n1);
      g.div(n2);
      float dn;
      if ((kind & 3) == R_NEW) {
        g.store(sm, F);
        dn = g.template np_dn<NPF>(wb, F);
      } else {
        g.div(g.norm(F));
#pragma unroll
        for (int q = 0; q < REG_EPL; q++) m.v[q] = a * m.v[q] + bb * g.v[q];
        m.div(m.norm(F));
        m.store(sm, F);
        dn = m.template np_dn<NPF>(wb, F);
      }
      if (lane == 0) P.tdn[(size_t)s * T + slot] = dn;
    }
    return;
  }
  for (int r = next(blockIdx.y * NWAVE + wave_id()); r < nrec; r = next(r + STEP)) {
    const int2 rc = P.rec[(size_t)s * D + r];
    const int slot = rc.x & 0xffff, kind = rc.x >> 16, dk = rc.y;
    FT* sm = feat + (size_t)slot * F;
    const FT* f = fembs + (size_t)dk * F;
    const FT n1 = (FT)P.dnrm[((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4];
    const FT n2 = (FT)P.dnrm[((size_t)P.dpar * P.S * D + (size_t)s * D + dk) * 4 + 1];
    FT* f2 = (FT*)P.fscr + ((size_t)s * D + dk) * F;  // this wave's scratch row
    for (int q = lane; q < F; q += WAVE) f2[q] = (f[q] / n1) / n2;
    if ((kind & 3) == R_NEW) {
      for (int q = lane; q < F; q += WAVE) sm[q] = f2[q];
    } else {
      const FT n3 = wave_norm((const FT*)f2, F);  // same lane mapping: reads own writes
      for (int q = lane; q < F; q += WAVE) {
        FT g3 = f2[q] / n3;
        sm[q] = a * sm[q] + bb * g3;
      }
      const FT ns = wave_norm((const FT*)sm, F);
      for (int q = lane; q < F; q += WAVE) sm[q] = sm[q] / ns;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // other lanes read sm next
    const float dn = sqrtf(np_sumsq_sel<NPF>((const FT*)sm, F)) + 1e-8f;
    if (lane == 0) P.tdn[(size_t)s * T + slot] = dn;
  }
}

// ------------------------------------------------------------------------------------------
// K6: remove_duplicate_stracks(active, lost) (bytetrack.py:321-335) on the updated means,
// output rows [x1,y1,x2,y2,id,conf,cls,det_ind] for activated tracks, final lists, slot release.
// One workgroup per sequence.
template <int KIND>
__global__ __launch_bounds__(WG) void finish_kernel(Dev P, int seq0, const int* __restrict__ det_off,
                                                    double* __restrict__ out,
                                                    int* __restrict__ out_count) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int T = P.T;
  const LdsF Lo(T);
  double* s_lbox = (double*)(smem + Lo.o_lbox);
  int* s_lage = (int*)(smem + Lo.o_lage);
  uint16_t* s_fa = (uint16_t*)(smem + Lo.o_fa);
  uint16_t* s_fl = (uint16_t*)(smem + Lo.o_fl);
  uint8_t* s_dupa = (uint8_t*)(smem + Lo.o_dupa);
  uint8_t* s_dupl = (uint8_t*)(smem + Lo.o_dupl);
  uint8_t* s_keep = (uint8_t*)(smem + Lo.o_keep);
  int* scan_tmp = (int*)(smem + Lo.o_ints);
  const int tid = threadIdx.x, b = blockIdx.x, s = seq0 + b;
  const size_t sT = (size_t)s * T;
  int* seq = P.seq + (size_t)s * SQ_STRIDE;
  const double* g_kf = P.kf + (size_t)s * T * KF_STRIDE;
  const int* g_fid = P.frame_id + sT;
  const int* g_start = P.start + sT;
  uint32_t* g_flags = P.flags + sT;
  if (seq[SQ_SKIP]) {  // K3 refused the frame (capacity): state untouched, no output
    if (tid == 0) { out_count[b] = 0; P.npair[s] = 0; }
    return;
  }
  const int na2 = seq[SQ_NA2], nl2 = seq[SQ_NL2];
  for (int k = tid; k < na2; k += WG) { s_fa[k] = P.act2[sT + k]; s_dupa[k] = 0; }
  for (int q = tid; q < nl2; q += WG) {
    const int sl = P.lost2[sT + q];
    s_fl[q] = (uint16_t)sl;
    s_dupl[q] = 0;
    track_box<KIND>(g_kf, sl, s_lbox + 4 * q);
    s_lage[q] = g_fid[sl] - g_start[sl];
  }
  for (int k = tid; k < T; k += WG) s_keep[k] = 0;
  __syncthreads();
  // iou distance < 0.15 → drop the younger track (ties drop the active one)
  const int lane = lane_id();
  for (int p = wave_id(); p < na2; p += NWAVE) {  // wave per active track, lanes over lost
    const int sa = s_fa[p];
    double ba[4];
    track_box<KIND>(g_kf, sa, ba);
    const int ta = g_fid[sa] - g_start[sa];
    bool dupa = false;
    for (int q = lane; q < nl2; q += WAVE) {
      const double* bb = s_lbox + 4 * q;
      if (!boxes_intersect(ba, bb)) continue;
      if (1 - iou_pair(ba, bb) < 0.15) {
        if (ta > s_lage[q]) s_dupl[q] = 1;
        else dupa = true;
      }
    }
    if (__ballot(dupa) != 0ull && lane == 0) s_dupa[p] = 1;
  }
  __syncthreads();
  const int nfa = block_compact(na2, [&](int k) { return !s_dupa[k]; },
                                [&](int k, int p) {
                                  P.act[sT + p] = s_fa[k];
                                  s_keep[s_fa[k]] = 1;
                                },
                                scan_tmp);
  const int nfl = block_compact(nl2, [&](int k) { return !s_dupl[k]; },
                                [&](int k, int p) {
                                  P.lost[sT + p] = s_fl[k];
                                  s_keep[s_fl[k]] = 2;
                                },
                                scan_tmp);
  const int d0 = det_off[b];
  const int nout = block_compact(
      na2, [&](int k) { return !s_dupa[k] && (g_flags[s_fa[k]] & F_ACT) != 0; },
      [&](int k, int p) {
        const int slot = s_fa[k];
        double box[4];
        track_box<KIND>(g_kf, slot, box);
        double* o = out + (size_t)(d0 + p) * 8;
        o[0] = box[0]; o[1] = box[1]; o[2] = box[2]; o[3] = box[3];
        o[4] = (double)P.id[sT + slot];
        o[5] = P.conf[sT + slot];
        o[6] = P.cls[sT + slot];
        o[7] = (double)P.detind[sT + slot];
      },
      scan_tmp);
  // slots that left both lists are free from here on; list membership bits for K2/K3
  for (int k = tid; k < T; k += WG) {
    const uint32_t f = g_flags[k];
    const uint8_t kp = s_keep[k];
    const uint32_t nf =
        kp ? ((f & ~(F_INACT | F_INLOST | F_TRANSIENT)) | (kp == 1 ? F_INACT : F_INLOST))
           : (f & F_PARKED) ? f : 0u;
    if (nf != f) g_flags[k] = nf;
  }
  if (tid == 0) {
    seq[SQ_NA] = nfa;
    seq[SQ_NL] = nfl;
    out_count[b] = nout;
    seq[SQ_NPAIR] = P.npair[s];
    P.npair[s] = 0;
  }
}

// ------------------------------------------------------------------------------------------
__global__ void reset_kernel(int* seq, uint32_t* flags, int T, int seq0, int nseq) {
  const int s = seq0 + blockIdx.x;
  if (blockIdx.x >= nseq) return;
  for (int k = threadIdx.x; k < SQ_STRIDE; k += blockDim.x) seq[(size_t)s * SQ_STRIDE + k] = 0;
  for (int k = threadIdx.x; k < T; k += blockDim.x) flags[(size_t)s * T + k] = 0;
}

__global__ void set_id_kernel(int* seq, int s, int v) { seq[(size_t)s * SQ_STRIDE + SQ_IDC] = v; }

// per_class mode (BaseTracker.per_class_decorator, basetracker.py:181-192): before class
// `next`'s update the active list of the class that ran last (`cur`) is parked and `next`'s
// comes back — `self.active_tracks = self.per_class_active_tracks[cls_id]`.  Only the active list
// is swapped: the lost list, the removed flags and the id counter stay shared, as in the
// reference (ByteTrack / BoT-SORT keep lost_stracks / removed_stracks on the tracker).  Parked
// slots leave the pool (no F_INACT: K2 does not predict them) but stay allocated (F_PARKED).
// The frame counter is held across a frame's class calls (`self.frame_count = frame_count`):
// the first class call of a frame saves it, every class call starts from it.  One workgroup.
__global__ __launch_bounds__(WG) void class_swap_kernel(Dev P, int s, uint16_t* park, int* npark,
                                                        int C, int cur, int next, int first) {
  const int T = P.T, tid = threadIdx.x;
  const size_t sT = (size_t)s * T;
  int* seq = P.seq + (size_t)s * SQ_STRIDE;
  uint16_t* act = P.act + sT;
  uint32_t* fl = P.flags + sT;
  if (cur != next) {
    const int na = seq[SQ_NA];
    for (int k = tid; k < na; k += WG) {
      const int sl = act[k];
      park[(size_t)cur * T + k] = (uint16_t)sl;
      fl[sl] = (fl[sl] & ~F_INACT) | F_PARKED;
    }
    __syncthreads();
    const int nn = npark[next];
    for (int k = tid; k < nn; k += WG) {
      const int sl = park[(size_t)next * T + k];
      act[k] = (uint16_t)sl;
      fl[sl] = (fl[sl] & ~F_PARKED) | F_INACT;
    }
    __syncthreads();
    if (tid == 0) {
      npark[cur] = na;
      seq[SQ_NA] = nn;
    }
  }
  if (tid == 0) {
    if (first) npark[C] = seq[SQ_FC];
    seq[SQ_FC] = npark[C];
  }
}

}  // namespace

struct bx_engine {
  bx_config cfg;
  Dev dev;
  int device;
  size_t lds_assoc, lds_finish;
  // stage timing probe (bx_engine_probe)
  int probe_stage = -1;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> probe_ev;
  size_t probe_used = 0;
  void* arena;
  size_t arena_bytes;
  // host-path staging (device)
  float* h_dets;
  void* h_embs;
  int* h_off;
  double* h_out;
  int* h_cnt;
  double* h_warp;
  // pinned host mirrors of the staging buffers (update_host: true async copies, one sync):
  // dets, embs, offsets + counters, warp, output rows, out count + status
  float* p_dets = nullptr;
  char* p_embs = nullptr;
  int* p_off = nullptr;
  double* p_warp = nullptr;
  double* p_out = nullptr;
  int* p_cnt = nullptr;
  int* p_seq = nullptr;     // the sequence's counters row after the last update_host
  int cache_seq = -1;       // sequence whose counters p_seq holds (-1: none / stale)
  int* h_lapmark = nullptr;  // host-mapped helper-wave cue (Dev::lapmark)
  uint32_t nlaunch = 0;      // association launches so far (the cue's clock; wraps, compared mod 2^32)
  int force_help = -1;       // bx_engine_force_assoc_build: -1 cue-driven, 0 / 1 that build always
  // side stream of the frame's fork-join (launch_frame): the ReID feature kernels K1 and K5 run
  // there beside the Kalman/list kernels they share no data with
  hipStream_t side = nullptr;
  hipEvent_t ev_fork[2] = {nullptr, nullptr}, ev_join[2] = {nullptr, nullptr};
  // overlap mode (bx_engine_set_overlap): a step leaves K5 on the side stream unjoined; the next
  // step's K1 queues behind it there and its K1c join covers both, every other entry point
  // settles it first (side_pending)
  bool overlap = false, side_pending = false;
  // early-features mode (bx_engine_set_early_features): K1 on its own stream `k1s`, waiting only
  // for the K5 that last read its half of dnrm (ev_k5[parity]), not for the previous frame —
  // the caller guarantees each step's inputs are complete when the step is called
  bool early = false;
  hipStream_t k1s = nullptr;
  hipEvent_t ev_k1 = nullptr, ev_k5[2] = {nullptr, nullptr};
  bool k5_rec[2] = {false, false};
  int par = 0;  // the next full launch's dnrm half
  // serialises every entry point that touches side_pending / the host staging buffers
  // (recursive: the host paths call bx_engine_step while holding it)
  std::recursive_mutex mu;
  // per_class mode (bx_engine_update_classes_host), allocated on first use: per sequence the
  // parked active lists [C][T] + their lengths [C] + the held frame counter, the class that ran
  // last; host-path class offsets [C][2] and output counts [C]
  int n_classes = 0;
  std::vector<char*> park;
  std::vector<int> cur_cls;
  int* h_coff = nullptr;
  int* h_ccnt = nullptr;
  double* h_cwarp = nullptr;  // [C][6] the class calls' warps
};

hipError_t bx_lds_attr(const void* kern, size_t bytes);  // below (never lowers a limit)

namespace {

template <typename T>
T* carve(char*& p, size_t n) {
  size_t bytes = (sizeof(T) * n + 255) & ~size_t(255);
  T* r = (T*)p;
  p += bytes;
  return r;
}

// the dynamic-LDS limit for > 64 KiB, per device and never lowered (bx_lds_attr, below)
int lds_attr(const void* kern, size_t bytes) {
  if (bytes <= 65536) return BX_OK;
  HIPCHK(bx_lds_attr(kern, bytes));
  return BX_OK;
}

// per_class state of one sequence: parked lists [C][T] uint16, then npark [C] + held fc
size_t park_npark_off(const bx_engine* e) {
  return ((size_t)e->n_classes * e->dev.T * sizeof(uint16_t) + 255) & ~size_t(255);
}

// One frame of sequences [seq0, seq0+nseq): the K1..K6 pipeline on stream st.
template <int KIND, typename FT, bool NPF>
int launch_frame(bx_engine* e, int seq0, int nseq, const float* dets, const int* det_off,
                 const void* embs, const double* warps, double* out, int* out_count,
                 hipStream_t st) {
  const bool reid = KIND == KIND_BOT && e->dev.with_reid;
  // early features: full launches only (a chunked frame's launches would share the parity)
  const bool early = reid && e->early && seq0 == 0 && nseq == e->dev.S;
  const int par = early ? e->par : 0;
  if (early) e->par ^= 1;
  e->dev.dpar = par;
  const Dev& d = e->dev;
  // Fork-join: K1 (detection norms) only feeds K1c, and K5 (feature EMA) only reads K3's records
  // and K1's norms and writes smooth_feat / tdn, which nothing else in the frame touches — so K1
  // runs on the side stream beside K2/K1b, and K5 beside K4/K4b/K6.  Both joins land on `st`
  // before the frame returns (the next frame's K1 rewrites the norms K5 reads) — except in
  // overlap mode (bx_engine_set_overlap), where K5 stays unjoined: the next frame's K1 queues
  // behind it on the side stream and that frame's join before K1c covers both (measured: 0.615
  // -> 0.599 ms/step at C3; a greater or lesser side-stream priority measured slower).
  if (reid && !e->side) {
    HIPCHK(hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
    for (int k = 0; k < 2; k++) {
      HIPCHK(hipEventCreateWithFlags(&e->ev_fork[k], hipEventDisableTiming | hipEventDisableSystemFence));
      HIPCHK(hipEventCreateWithFlags(&e->ev_join[k], hipEventDisableTiming | hipEventDisableSystemFence));
    }
  }
  hipStream_t side = e->side;
  auto fork = [&](int k) -> int {
    HIPCHK(hipEventRecord(e->ev_fork[k], st));
    HIPCHK(hipStreamWaitEvent(side, e->ev_fork[k], 0));
    return BX_OK;
  };
  auto join = [&](int k) -> int {
    HIPCHK(hipEventRecord(e->ev_join[k], side));
    HIPCHK(hipStreamWaitEvent(st, e->ev_join[k], 0));
    return BX_OK;
  };
  auto probe_begin = [&](int stage, hipStream_t st) -> int {
    if (stage != e->probe_stage) return BX_OK;
    if (e->probe_used == e->probe_ev.size()) {
      hipEvent_t a, b;
      // timing-only events: no system-scope fence (cache writeback/invalidate) on record, so
      // the probe does not perturb the kernels around it
      HIPCHK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      HIPCHK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
      e->probe_ev.emplace_back(a, b);
    }
    HIPCHK(hipEventRecord(e->probe_ev[e->probe_used].first, st));
    return BX_OK;
  };
  auto probe_end = [&](int stage, hipStream_t st) -> int {
    if (stage != e->probe_stage) return BX_OK;
    HIPCHK(hipEventRecord(e->probe_ev[e->probe_used++].second, st));
    return BX_OK;
  };
  // a probed stage is timed by events on the stream it is launched on
#define BX_PROBED_ON(stage, sstream, ...)                     \
  do {                                                        \
    if (int rc_ = probe_begin(stage, sstream)) return rc_;    \
    __VA_ARGS__;                                              \
    HIPCHK(hipGetLastError());                                \
    if (int rc_ = probe_end(stage, sstream)) return rc_;      \
  } while (0)
#define BX_PROBED(stage, ...) BX_PROBED_ON(stage, st, __VA_ARGS__)
  const int gy_det64 = (d.D + K1_DETS - 1) / K1_DETS, gy_slot = (d.T + WG - 1) / WG;
  if (early && !e->k1s) {
    HIPCHK(hipStreamCreateWithFlags(&e->k1s, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&e->ev_k1, hipEventDisableTiming | hipEventDisableSystemFence));
    for (int k = 0; k < 2; k++)
      HIPCHK(hipEventCreateWithFlags(&e->ev_k5[k], hipEventDisableTiming | hipEventDisableSystemFence));
  }
  // early features: K1 on k1s after only the K5 two launches back (the last reader of this
  // dnrm half; K1c of that launch came before that K5); else on the side stream, forked here
  if (early && e->k5_rec[par]) HIPCHK(hipStreamWaitEvent(e->k1s, e->ev_k5[par], 0));
  hipStream_t k1st = early ? e->k1s : side;
  if (reid && !early)
    if (int rc = fork(0)) return rc;
  const bool gmc = KIND == KIND_BOT && warps;
  // K1 on the side stream, submitted first (measured: 0.644 ms/step; submitted after K2/K1b
  // 0.647; serial on the main stream 0.661)
  // the common width (512, the bench's and osnet's) as a compile-time constant
// Compile-time feature width (REG_F) per kernel, bit 0 K1, bit 1 K5, bit 2 K1c.  K1 only: at C3
// K1 0.124 -> 0.104 ms and the step 0.602 -> 0.593; a faster K5 (0.226 -> 0.18) took the GPU from
// K4 / K6 beside it and the step went to 0.633 (K5 submitted after K4, capped by LDS reservation,
// or on a lower-priority stream: no better); K1c unchanged (its loops were already fixed-stride).
#ifndef BX_FC_MASK
#define BX_FC_MASK 1
#endif
  const bool fc = NPF && d.F == REG_F && (BX_FC_MASK & 1);
  const bool fc5 = NPF && d.F == REG_F && (BX_FC_MASK & 2);
  if (reid && fc)
    BX_PROBED_ON(BX_STAGE_DET_FEATURES, k1st,
                 hipLaunchKernelGGL((det_feature_kernel<FT, NPF, (NPF ? REG_F : 0)>),
                                    dim3(nseq, gy_det64), dim3(WG), 0, k1st, d, seq0, dets,
                                    det_off, (const FT*)embs));
  else if (reid)
    BX_PROBED_ON(BX_STAGE_DET_FEATURES, k1st,
                 hipLaunchKernelGGL((det_feature_kernel<FT, NPF, 0>), dim3(nseq, gy_det64),
                                    dim3(WG), 0, k1st, d, seq0, dets, det_off, (const FT*)embs));
  if (early) HIPCHK(hipEventRecord(e->ev_k1, e->k1s));
  if (gmc)
    BX_PROBED(BX_STAGE_PREDICT,
              hipLaunchKernelGGL((predict_kernel<KIND, true>), dim3(nseq, gy_slot), dim3(WG), 0,
                                 st, d, seq0, warps));
  else
    BX_PROBED(BX_STAGE_PREDICT,
              hipLaunchKernelGGL((predict_kernel<KIND, false>), dim3(nseq, gy_slot), dim3(WG), 0,
                                 st, d, seq0, warps));
  if (reid) {
    const size_t glds = (sizeof(double) * 4 + sizeof(float4)) * d.D;  // det boxes in LDS
    BX_PROBED(BX_STAGE_GATE,
              hipLaunchKernelGGL(gate_kernel<KIND>, dim3(nseq, GATE_BLOCKS), dim3(WG), glds, st,
                                 d, seq0, dets, det_off));
    // K1c reads K1's norms and the smooth features the last K5 wrote (overlap mode: unjoined)
    if (early) HIPCHK(hipStreamWaitEvent(st, e->ev_k1, 0));
    if (!early || e->side_pending)
      if (int rc = join(0)) return rc;
    if (d.F == REG_F && (BX_FC_MASK & 4))
      BX_PROBED(BX_STAGE_COSINE,
                hipLaunchKernelGGL((cosine_kernel<FT, REG_F>), dim3(nseq, COS_BLOCKS), dim3(WG), 0,
                                   st, d, seq0, det_off, (const FT*)embs));
    else if (d.F % COS_CH == 0)
      BX_PROBED(BX_STAGE_COSINE,
                hipLaunchKernelGGL((cosine_kernel<FT, 0>), dim3(nseq, COS_BLOCKS), dim3(WG), 0, st,
                                   d, seq0, det_off, (const FT*)embs));
    else
      BX_PROBED(BX_STAGE_COSINE,
                hipLaunchKernelGGL(cosine_kernel_any<FT>, dim3(nseq, COS_BLOCKS), dim3(WG), 0, st,
                                   d, seq0, det_off, (const FT*)embs));
  }
  // the helper-wave build while LAPs that want it were seen in the last BX_HELP_WINDOW launches
#ifndef BX_HELP_WINDOW
#define BX_HELP_WINDOW 64
#endif
  e->dev.lapstamp = (int)++e->nlaunch;
  const bool help = e->force_help >= 0
                        ? e->force_help != 0
                        : e->h_lapmark && (uint32_t)(e->nlaunch - (uint32_t)*(volatile int*)
                                                         e->h_lapmark) <= BX_HELP_WINDOW;
  auto assoc = help ? assoc_kernel<KIND, true> : assoc_kernel<KIND, false>;
  if (int rc = lds_attr((const void*)assoc, e->lds_assoc)) return rc;
  BX_PROBED(BX_STAGE_ASSOC, hipLaunchKernelGGL(assoc, dim3(nseq), dim3(WG), e->lds_assoc, st, d,
                                               seq0, dets, det_off));
  auto launch_k5 = [&]() -> int {
    if (fc5)
      BX_PROBED_ON(BX_STAGE_FEATURES, side,
                   hipLaunchKernelGGL((feature_kernel<FT, NPF, (NPF ? REG_F : 0)>),
                                      dim3(nseq, FEAT_BLOCKS), dim3(WG), 0, side, d, seq0,
                                      det_off, (const FT*)embs));
    else
      BX_PROBED_ON(BX_STAGE_FEATURES, side,
                   hipLaunchKernelGGL((feature_kernel<FT, NPF, 0>), dim3(nseq, FEAT_BLOCKS),
                                      dim3(WG), 0, side, d, seq0, det_off, (const FT*)embs));
    e->side_pending = true;  // until joined below (or, in overlap mode, by the next frame)
    return BX_OK;
  };
  if (reid) {
    if (int rc = fork(1)) return rc;
    if (int rc = launch_k5()) return rc;
    if (early) {  // the last reader of this dnrm half: the launch after next's K1 waits for it
      HIPCHK(hipEventRecord(e->ev_k5[par], side));
      e->k5_rec[par] = true;
    }
  }
  BX_PROBED(BX_STAGE_UPDATE,
            hipLaunchKernelGGL(update_kernel<KIND>,
                               dim3(nseq, (d.D + UPD_PER_BLOCK - 1) / UPD_PER_BLOCK), dim3(WG), 0,
                               st, d, seq0, dets, det_off, warps));
  if (gmc)  // (without a warp the covariance predicts of tracks without an update stay pending)
    BX_PROBED(BX_STAGE_COV_PREDICT,
              hipLaunchKernelGGL(cov_predict_gmc_kernel<KIND>, dim3(nseq, gy_slot), dim3(WG), 0,
                                 st, d, seq0, warps));
  if (int rc = lds_attr((const void*)finish_kernel<KIND>, e->lds_finish)) return rc;
  BX_PROBED(BX_STAGE_FINISH,
            hipLaunchKernelGGL(finish_kernel<KIND>, dim3(nseq), dim3(WG), e->lds_finish, st, d,
                               seq0, det_off, out, out_count));
  if (reid && !e->overlap) {  // overlap mode: joined by the next step's K1c join, or settle()
    if (int rc = join(1)) return rc;
    e->side_pending = false;
  }
#undef BX_PROBED
#undef BX_PROBED_ON
  return BX_OK;
}

}  // namespace

// shared by the other translation units of the library (bx_ocsort.hip) so that bx_last_error
// reports their failures too
// overlap mode: wait for a step's unjoined K5 (side stream) before any other use of the engine
static int settle(bx_engine* e) {
  if (!e) return BX_OK;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (e->side_pending) {
    e->side_pending = false;
    HIPCHK(hipStreamSynchronize(e->side));
  }
  return BX_OK;
}

int bx_record_error(int code, const char* msg) { return set_err(code, msg); }

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) that never lowers a kernel's limit: engines of
// different capacities share the kernels, and a later, smaller engine must not shrink the limit
// an earlier one launches with (shared by every translation unit of the library).  The attribute
// belongs to the current device, so the cache is keyed by (device, kernel).
hipError_t bx_lds_attr(const void* kern, size_t bytes) {
  struct Entry {
    int dev;
    const void* kern;
    size_t bytes;
  };
  static std::mutex mu;
  static std::vector<Entry> done;
  int dev = 0;
  if (const hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& d : done)
    if (d.dev == dev && d.kern == kern) {
      if (d.bytes >= bytes) return hipSuccess;
      const hipError_t e =
          hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
      if (e == hipSuccess) d.bytes = bytes;
      return e;
    }
  const hipError_t e =
      hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) done.push_back({dev, kern, bytes});
  return e;
}

extern "C" {

const char* bx_last_error(void) { return g_err.c_str(); }

int bx_device_count(int* n) {
  int c = 0;
  hipError_t err = hipGetDeviceCount(&c);
  if (err != hipSuccess) c = 0;
  *n = c;
  return BX_OK;
}

int bx_engine_create(const bx_config* cfg, bx_engine** out) {
  if (!cfg || !out) return set_err(BX_ERR_INVALID, "null argument");
  *out = nullptr;
  if (cfg->kind != BX_BYTETRACK && cfg->kind != BX_BOTSORT)
    return set_err(BX_ERR_INVALID, "unknown tracker kind");
  if (cfg->n_seq <= 0 || cfg->track_cap <= 0 || cfg->det_cap <= 0 || cfg->track_cap > 32767 ||
      cfg->det_cap > 32767)
    return set_err(BX_ERR_INVALID, "n_seq/track_cap/det_cap out of range");
  const bool reid = cfg->kind == BX_BOTSORT && cfg->with_reid;
  if (reid && cfg->emb_dim <= 0) return set_err(BX_ERR_INVALID, "with_reid needs emb_dim > 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return set_err(BX_ERR_NO_DEVICE, "no HIP device visible");
  auto* e = new bx_engine();
  e->cfg = *cfg;
  HIPCHK(hipGetDevice(&e->device));
  const int S = cfg->n_seq, T = cfg->track_cap, D = cfg->det_cap;
  const int F = reid ? cfg->emb_dim : 0;
  const size_t fs = cfg->emb_f64 ? 8 : 4;
  Dev& d = e->dev;
  d.S = S; d.T = T; d.D = D; d.F = F; d.kind = cfg->kind; d.emb_f64 = cfg->emb_f64;
  d.with_reid = reid; d.fuse_first = cfg->fuse_first_associate;
  d.elds = ELDS_DEFAULT;
  d.lap_stats = 0;
  d.jvs_stride = (jv_bytes(T + D) + 255) & ~size_t(255);
  d.match_thresh = cfg->match_thresh;
  d.max_time_lost = (int)(cfg->frame_rate / 30.0 * cfg->track_buffer);
  if (cfg->kind == BX_BYTETRACK) {
    d.low = cfg->min_conf; d.high = cfg->track_thresh; d.new_thresh = cfg->track_thresh;
  } else {
    d.low = cfg->track_low_thresh; d.high = cfg->track_high_thresh;
    d.new_thresh = cfg->new_track_thresh;
  }
  d.prox = cfg->proximity_thresh;
  d.app = cfg->appearance_thresh;
  const size_t ST = (size_t)S * T;
  const size_t SD = (size_t)S * D, FF = F ? F : 1;
  const size_t FS = F > REG_F ? F : 1;  // twice-normalised det rows kept only for wide features
  // carve the arena twice: once from a null base to size it, once for real
  auto layout = [&](char* p) {
    char* p0 = p;
    d.seq = carve<int>(p, (size_t)S * SQ_STRIDE);
    d.act = carve<uint16_t>(p, ST);
    d.lost = carve<uint16_t>(p, ST);
    d.act2 = carve<uint16_t>(p, ST);
    d.lost2 = carve<uint16_t>(p, ST);
    d.flags = carve<uint32_t>(p, ST);
    d.frame_id = carve<int>(p, ST);
    d.start = carve<int>(p, ST);
    d.id = carve<int>(p, ST);
    d.tlen = carve<int>(p, ST);
    d.detind = carve<int>(p, ST);
    d.conf = carve<double>(p, ST);
    d.cls = carve<double>(p, ST);
    d.kf = carve<double>(p, ST * KF_STRIDE);
    d.feat = carve<char>(p, fs * ST * FF);
    d.clsh = carve<double>(p, ST * CLS_HIST * 2);
    d.ncls = carve<int>(p, ST);
    d.gcol = carve<uint16_t>(p, ST * D);
    d.gcost = carve<double>(p, ST * D);
    d.rec = carve<int2>(p, SD);
    d.dnrm = carve<double>(p, 2 * SD * 4);
    d.tdn = carve<float>(p, reid ? ST : 1);
    d.pairs = carve<uint32_t>(p, reid ? ST * D : 1);
    d.npair = carve<int>(p, S);
    d.etab = carve<double>(p, reid ? ST * D : 1);
    d.jvs = carve<unsigned char>(p, (size_t)S * d.jvs_stride);
    d.fscr = carve<char>(p, fs * SD * FS);
    d.status = carve<int>(p, 16);
    return (size_t)(p - p0);
  };
  const size_t bytes = layout(nullptr);
  e->arena_bytes = bytes;
  if (hipMalloc(&e->arena, bytes) != hipSuccess) {
    delete e;
    return set_err(BX_ERR_HIP, "hipMalloc of the engine arena failed");
  }
  layout((char*)e->arena);
  d.dbg = nullptr;
#ifdef BX_PHASE_TIMING
  HIPCHK(hipMalloc(&d.dbg, sizeof(unsigned long long) * BX_DBG_STRIDE * S));
  HIPCHK(hipMemset(d.dbg, 0, sizeof(unsigned long long) * BX_DBG_STRIDE * S));
#endif
  HIPCHK(hipMemset(e->arena, 0, bytes));
  e->lds_assoc = LdsA(T, D, d.elds).total;
  e->lds_finish = LdsF(T).total;
  {
    const LdsA Lo(T, D, d.elds);  // the LAP helper scratch overlays tboxf .. dconf
    if (lap_helper_bytes((T + 7) & ~7, (D + 7) & ~7) > Lo.o_dconf - Lo.o_tboxf) {
      (void)hipFree(e->arena);
      delete e;
      return set_err(BX_ERR_INVALID, "LAP helper scratch does not fit its LDS overlay");
    }
  }
  if (e->lds_assoc > 160 * 1024 || e->lds_finish > 160 * 1024) {
    (void)hipFree(e->arena);
    delete e;
    return set_err(BX_ERR_INVALID, "track_cap/det_cap too large for one workgroup's LDS");
  }
  // host-path staging for one sequence
  HIPCHK(hipMalloc(&e->h_dets, sizeof(float) * 6 * D));
  HIPCHK(hipMalloc(&e->h_embs, fs * (size_t)D * (F ? F : 1)));
  HIPCHK(hipMalloc(&e->h_off, sizeof(int) * 2));
  HIPCHK(hipMalloc(&e->h_out, sizeof(double) * 8 * D));
  HIPCHK(hipMalloc(&e->h_cnt, sizeof(int)));
  HIPCHK(hipMalloc(&e->h_warp, sizeof(double) * 6));
  HIPCHK(hipHostMalloc(&e->p_dets, sizeof(float) * 6 * D));
  HIPCHK(hipHostMalloc(&e->p_embs, fs * (size_t)D * (F ? F : 1)));
  HIPCHK(hipHostMalloc(&e->p_off, sizeof(int) * 2));
  HIPCHK(hipHostMalloc(&e->p_warp, sizeof(double) * 6));
  HIPCHK(hipHostMalloc(&e->p_out, sizeof(double) * 8 * D));
  HIPCHK(hipHostMalloc(&e->p_cnt, sizeof(int) * 2));
  HIPCHK(hipHostMalloc(&e->p_seq, sizeof(int) * SQ_STRIDE));
  // the LAPs' helper-wave cue, written by the association kernel, read by the host at launch
  HIPCHK(hipHostMalloc(&e->h_lapmark, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *e->h_lapmark = (int)(0u - (BX_HELP_WINDOW + 1u));  // "long ago" on the wrapping clock
  HIPCHK(hipHostGetDevicePointer((void**)&e->dev.lapmark, e->h_lapmark, 0));
  *out = e;
  return BX_OK;
}

int bx_engine_destroy(bx_engine* e) {
  if (!e) return BX_OK;
  if (e->side) {
    (void)hipStreamSynchronize(e->side);
    (void)hipStreamDestroy(e->side);
    for (int k = 0; k < 2; k++) {
      (void)hipEventDestroy(e->ev_fork[k]);
      (void)hipEventDestroy(e->ev_join[k]);
    }
  }
  if (e->k1s) {
    (void)hipStreamSynchronize(e->k1s);
    (void)hipStreamDestroy(e->k1s);
    (void)hipEventDestroy(e->ev_k1);
    for (int k = 0; k < 2; k++) (void)hipEventDestroy(e->ev_k5[k]);
  }
  for (auto& ev : e->probe_ev) {
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  (void)hipFree(e->arena);
  (void)hipFree(e->h_dets);
  (void)hipFree(e->h_embs);
  (void)hipFree(e->h_off);
  (void)hipFree(e->h_out);
  (void)hipFree(e->h_cnt);
  (void)hipFree(e->h_warp);
  (void)hipHostFree(e->p_dets);
  if (e->h_lapmark) (void)hipHostFree(e->h_lapmark);
  (void)hipHostFree(e->p_embs);
  (void)hipHostFree(e->p_off);
  (void)hipHostFree(e->p_warp);
  (void)hipHostFree(e->p_out);
  (void)hipHostFree(e->p_cnt);
  (void)hipHostFree(e->p_seq);
  for (char* p : e->park) (void)hipFree(p);
  (void)hipFree(e->h_coff);
  (void)hipFree(e->h_ccnt);
  (void)hipFree(e->h_cwarp);
  delete e;
  return BX_OK;
}

int bx_engine_reset(bx_engine* e, int seq0, int nseq, void* stream) {
  if (int rc = settle(e)) return rc;
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S)
    return set_err(BX_ERR_INVALID, "bad sequence range");
  e->cache_seq = -1;
  hipLaunchKernelGGL(reset_kernel, dim3(nseq), dim3(256), 0, (hipStream_t)stream, e->dev.seq,
                     e->dev.flags, e->dev.T, seq0, nseq);
  HIPCHK(hipGetLastError());
  for (int s = seq0; s < seq0 + nseq && e->n_classes; s++)
    if (e->park[s]) {  // parked class lists are gone with the tracks
      HIPCHK(hipMemsetAsync(e->park[s] + park_npark_off(e), 0, sizeof(int) * (e->n_classes + 1),
                            (hipStream_t)stream));
      e->cur_cls[s] = 0;
    }
  return BX_OK;
}

int bx_engine_step(bx_engine* e, int seq0, int nseq, const float* dets, const int32_t* det_off,
                   const void* embs, const double* warps, double* out, int32_t* out_count,
                   void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_step");
  if (e->dev.with_reid && !embs) return set_err(BX_ERR_SHAPE, "BoT-SORT with_reid needs embs");
  hipStream_t st = (hipStream_t)stream;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  e->cache_seq = -1;
  if (e->dev.kind == BX_BYTETRACK)
    return launch_frame<KIND_BYTE, float, true>(e, seq0, nseq, dets, det_off, embs, warps, out,
                                                out_count, st);
  const bool npf = np_wave_exact(e->dev.F);
  if (e->dev.emb_f64)
    return npf ? launch_frame<KIND_BOT, double, true>(e, seq0, nseq, dets, det_off, embs, warps,
                                                      out, out_count, st)
               : launch_frame<KIND_BOT, double, false>(e, seq0, nseq, dets, det_off, embs, warps,
                                                       out, out_count, st);
  return npf ? launch_frame<KIND_BOT, float, true>(e, seq0, nseq, dets, det_off, embs, warps, out,
                                                   out_count, st)
             : launch_frame<KIND_BOT, float, false>(e, seq0, nseq, dets, det_off, embs, warps,
                                                    out, out_count, st);
}

int bx_engine_update_host(bx_engine* e, int seq, const float* dets, int n, const void* embs,
                          const double* warp, double* out, int* n_out, void* stream) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || !n_out)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_update_host");
  if (n > e->dev.D) return set_err(BX_ERR_CAPACITY, "detections exceed det_cap");
  if (e->dev.with_reid && n > 0 && !embs)
    return set_err(BX_ERR_SHAPE, "BoT-SORT with_reid needs embs");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  hipStream_t st = (hipStream_t)stream;
  const size_t fs = e->cfg.emb_f64 ? 8 : 4;
  // inputs through pinned mirrors (asynchronous DMA), the frame, then the rows (at most n), the
  // count and the status back in one go: a single synchronisation per frame
  const bool ecopy = n && e->dev.with_reid;
  if (n) memcpy(e->p_dets, dets, sizeof(float) * 6 * n);
  if (ecopy) memcpy(e->p_embs, embs, fs * (size_t)n * e->dev.F);
  e->p_off[0] = 0;
  e->p_off[1] = n;
  if (warp) memcpy(e->p_warp, warp, sizeof(double) * 6);
  if (n) HIPCHK(hipMemcpyAsync(e->h_dets, e->p_dets, sizeof(float) * 6 * n, hipMemcpyHostToDevice, st));
  if (ecopy)
    HIPCHK(hipMemcpyAsync(e->h_embs, e->p_embs, fs * (size_t)n * e->dev.F, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(e->h_off, e->p_off, sizeof(int) * 2, hipMemcpyHostToDevice, st));
  if (warp) HIPCHK(hipMemcpyAsync(e->h_warp, e->p_warp, sizeof(double) * 6, hipMemcpyHostToDevice, st));
  int rc = bx_engine_step(e, seq, 1, e->h_dets, e->h_off, e->h_embs, warp ? e->h_warp : nullptr,
                          e->h_out, e->h_cnt, stream);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(e->p_cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(e->p_cnt + 1, e->dev.status, sizeof(int), hipMemcpyDeviceToHost, st));
  if (n) HIPCHK(hipMemcpyAsync(e->p_out, e->h_out, sizeof(double) * 8 * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(e->p_seq, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(int) * SQ_STRIDE,
                        hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  e->cache_seq = seq;  // bx_engine_counters_host answers from it until the next device change
  const int cnt = e->p_cnt[0], status = e->p_cnt[1];
  if (cnt && out) memcpy(out, e->p_out, sizeof(double) * 8 * cnt);
  *n_out = cnt;
  if (status & (1 << BX_ERR_TRACK_OVERFLOW))
    return set_err(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

// per_class=True (BaseTracker.per_class_decorator, basetracker.py:155-201) for one sequence:
// the update runs once per class id 0..C-1 on that class's detections (`dets[:, 5] == cls_id` on
// the float32 array; rows keep their input order; det_ind indexes the class's subset), with the
// class's active list swapped in (class_swap_kernel) and the frame counter held; outputs are
// stacked in class order.  All C class calls are enqueued back to back on `stream` (no host sync
// between them); one synchronisation at the end.
int bx_engine_update_classes_host(bx_engine* e, int seq, const float* dets, int n,
                                  const void* embs, const double* warps, int n_classes,
                                  double* out, int* n_out, void* stream) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !dets) || !n_out || n_classes <= 0 ||
      n_classes > 4096)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_update_classes_host");
  if (n > e->dev.D) return set_err(BX_ERR_CAPACITY, "detections exceed det_cap");
  const bool reid = e->dev.with_reid;
  if (reid && n > 0 && !embs) return set_err(BX_ERR_SHAPE, "BoT-SORT with_reid needs embs");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  hipStream_t st = (hipStream_t)stream;
  const int C = n_classes, F = e->dev.F;
  if (e->n_classes && e->n_classes != C)
    return set_err(BX_ERR_INVALID, "n_classes differs from the engine's first per-class call");
  if (!e->n_classes) {
    e->n_classes = C;
    e->park.assign(e->dev.S, nullptr);
    e->cur_cls.assign(e->dev.S, 0);
    HIPCHK(hipMalloc(&e->h_coff, sizeof(int) * 2 * C));
    HIPCHK(hipMalloc(&e->h_ccnt, sizeof(int) * C));
    HIPCHK(hipMalloc(&e->h_cwarp, sizeof(double) * 6 * C));
  }
  if (!e->park[seq]) {
    const size_t bytes = park_npark_off(e) + sizeof(int) * (C + 1);
    HIPCHK(hipMalloc(&e->park[seq], bytes));
    HIPCHK(hipMemset(e->park[seq], 0, bytes));
  }
  uint16_t* park = (uint16_t*)e->park[seq];
  int* npark = (int*)(e->park[seq] + park_npark_off(e));
  // class split, stable within a class
  std::vector<int> cnt(C + 1, 0), order;
  order.reserve(n);
  auto cls_of = [&](int i) -> int {
    const float v = dets[6 * i + 5];
    return (v >= 0.f && v < (float)C && v == (float)(int)v) ? (int)v : -1;
  };
  for (int i = 0; i < n; i++) {
    const int c = cls_of(i);
    if (c >= 0) cnt[c + 1]++;
  }
  for (int c = 0; c < C; c++) cnt[c + 1] += cnt[c];
  std::vector<int> fill(cnt.begin(), cnt.end() - 1);
  order.assign(cnt[C], 0);
  for (int i = 0; i < n; i++) {
    const int c = cls_of(i);
    if (c >= 0) order[fill[c]++] = i;
  }
  const int m = cnt[C];
  const size_t fs = e->cfg.emb_f64 ? 8 : 4;
  std::vector<float> hd((size_t)6 * (m ? m : 1));
  std::vector<char> he(reid ? fs * (size_t)(m ? m : 1) * F : 1);
  for (int k = 0; k < m; k++) {
    memcpy(&hd[6 * (size_t)k], dets + 6 * (size_t)order[k], 6 * sizeof(float));
    if (reid) memcpy(&he[fs * F * (size_t)k], (const char*)embs + fs * F * (size_t)order[k], fs * F);
  }
  std::vector<int> hoff(2 * C);
  for (int c = 0; c < C; c++) { hoff[2 * c] = 0; hoff[2 * c + 1] = cnt[c + 1] - cnt[c]; }
  if (m) HIPCHK(hipMemcpyAsync(e->h_dets, hd.data(), sizeof(float) * 6 * m, hipMemcpyHostToDevice, st));
  if (m && reid) HIPCHK(hipMemcpyAsync(e->h_embs, he.data(), fs * (size_t)m * F, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(e->h_coff, hoff.data(), sizeof(int) * 2 * C, hipMemcpyHostToDevice, st));
  if (warps) HIPCHK(hipMemcpyAsync(e->h_cwarp, warps, sizeof(double) * 6 * C, hipMemcpyHostToDevice, st));
  for (int c = 0; c < C; c++) {
    hipLaunchKernelGGL(class_swap_kernel, dim3(1), dim3(WG), 0, st, e->dev, seq, park, npark, C,
                       e->cur_cls[seq], c, c == 0 ? 1 : 0);
    HIPCHK(hipGetLastError());
    e->cur_cls[seq] = c;
    const char* ep = reid ? (const char*)e->h_embs + fs * F * (size_t)cnt[c] : nullptr;
    // class call c's warp (an identity warp is no warp, as in bx_engine_update_host's callers)
    const bool wc = warps && !is_identity_warp(warps + 6 * (size_t)c);
    int rc = bx_engine_step(e, seq, 1, e->h_dets + 6 * (size_t)cnt[c], e->h_coff + 2 * c, ep,
                            wc ? e->h_cwarp + 6 * (size_t)c : nullptr,
                            e->h_out + 8 * (size_t)cnt[c], e->h_ccnt + c, stream);
    if (rc) return rc;
  }
  std::vector<int> oc(C);
  HIPCHK(hipMemcpyAsync(oc.data(), e->h_ccnt, sizeof(int) * C, hipMemcpyDeviceToHost, st));
  std::vector<double> ho((size_t)8 * (m ? m : 1));
  if (m) HIPCHK(hipMemcpyAsync(ho.data(), e->h_out, sizeof(double) * 8 * m, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  int k = 0;
  for (int c = 0; c < C; c++)
    for (int j = 0; j < oc[c]; j++, k++)
      if (out) memcpy(out + 8 * (size_t)k, &ho[8 * ((size_t)cnt[c] + j)], 8 * sizeof(double));
  *n_out = k;
  int status = 0;
  HIPCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status & (1 << BX_ERR_TRACK_OVERFLOW))
    return set_err(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

#ifdef BX_PHASE_TIMING
// diagnostic only: copy the [S][32] phase stamps of the last launch to the host
int bx_debug_stamps_host(bx_engine* e, unsigned long long* out) {
  if (int rc = settle(e)) return rc;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, e->dev.dbg, sizeof(unsigned long long) * BX_DBG_STRIDE * e->dev.S,
                   hipMemcpyDeviceToHost));
  return BX_OK;
}
#endif

int bx_engine_status(bx_engine* e, int* status) {
  if (int rc = settle(e)) return rc;
  if (!e || !status) return set_err(BX_ERR_INVALID, "null argument");
  int s = 0;
  HIPCHK(hipMemcpy(&s, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  *status = (s & (1 << BX_ERR_TRACK_OVERFLOW)) ? BX_ERR_TRACK_OVERFLOW
            : (s & (1 << BX_ERR_CAPACITY))     ? BX_ERR_CAPACITY
                                               : BX_OK;
  return BX_OK;
}

int bx_engine_frame_stats_host(bx_engine* e, int seq0, int nseq, int64_t* sums) {
  if (int rc = settle(e)) return rc;
  if (!e || !sums || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_frame_stats_host");
  std::vector<int> v((size_t)nseq * SQ_STRIDE);
  HIPCHK(hipMemcpy(v.data(), e->dev.seq + (size_t)seq0 * SQ_STRIDE, sizeof(int) * v.size(),
                   hipMemcpyDeviceToHost));
  const int idx[7] = {SQ_NDET, SQ_NHIGH, SQ_NA, SQ_NL, SQ_NREC, SQ_NPAIR, SQ_FC};
  for (int k = 0; k < 7; k++) {
    int64_t t = 0;
    for (int q = 0; q < nseq; q++) t += v[(size_t)q * SQ_STRIDE + idx[k]];
    sums[k] = t;
  }
  return BX_OK;
}

int bx_engine_lap_ties_host(bx_engine* e, int seq0, int nseq, int64_t* total) {
  if (int rc = settle(e)) return rc;
  if (!e || !total || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_lap_ties_host");
  std::vector<int> v((size_t)nseq * SQ_STRIDE);
  HIPCHK(hipMemcpy(v.data(), e->dev.seq + (size_t)seq0 * SQ_STRIDE, sizeof(int) * v.size(),
                   hipMemcpyDeviceToHost));
  int64_t t = 0;
  for (int q = 0; q < nseq; q++) t += v[(size_t)q * SQ_STRIDE + SQ_NTIE];
  *total = t;
  return BX_OK;
}

int bx_engine_lap_components_host(bx_engine* e, int seq0, int nseq, int64_t* sums) {
  if (int rc = settle(e)) return rc;
  if (!e || !sums || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_lap_components_host");
  std::vector<int> v((size_t)nseq * SQ_STRIDE);
  HIPCHK(hipMemcpy(v.data(), e->dev.seq + (size_t)seq0 * SQ_STRIDE, sizeof(int) * v.size(),
                   hipMemcpyDeviceToHost));
  sums[0] = sums[1] = sums[2] = 0;
  for (int q = 0; q < nseq; q++) {
    sums[0] += v[(size_t)q * SQ_STRIDE + SQ_NCOMP17];
    sums[1] += v[(size_t)q * SQ_STRIDE + SQ_NCOMPW];
    sums[2] += v[(size_t)q * SQ_STRIDE + SQ_NCOMPH];
  }
  return BX_OK;
}

int bx_engine_probe(bx_engine* e, int stage) {
  if (!e || stage >= BX_STAGE_COUNT) return set_err(BX_ERR_INVALID, "bad probe stage");
  e->probe_stage = stage < 0 ? -1 : stage;
  e->probe_used = 0;
  return BX_OK;
}

int bx_engine_probe_read(bx_engine* e, double* total_ms, int* count) {
  if (int rc = settle(e)) return rc;
  if (!e || !total_ms || !count) return set_err(BX_ERR_INVALID, "null argument");
  double t = 0.0;
  for (size_t k = 0; k < e->probe_used; k++) {
    HIPCHK(hipEventSynchronize(e->probe_ev[k].second));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e->probe_ev[k].first, e->probe_ev[k].second));
    t += ms;
  }
  *total_ms = t;
  *count = (int)e->probe_used;
  e->probe_used = 0;
  return BX_OK;
}

int bx_engine_counters_host(bx_engine* e, int seq, int* frame_count, int* id_count, int* n_active,
                            int* n_lost) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  int v[SQ_STRIDE];
  if (seq == e->cache_seq)
    memcpy(v, e->p_seq, sizeof(v));
  else
    HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  if (frame_count) *frame_count = v[SQ_FC];
  if (id_count) *id_count = v[SQ_IDC];
  if (n_active) *n_active = v[SQ_NA];
  if (n_lost) *n_lost = v[SQ_NL];
  return BX_OK;
}

int bx_engine_set_id_count(bx_engine* e, int seq, int id_count, void* stream) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  e->cache_seq = -1;
  hipLaunchKernelGGL(set_id_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, e->dev.seq, seq,
                     id_count);
  HIPCHK(hipGetLastError());
  return BX_OK;
}

namespace {
// host copy of the listed slots' track fields (bx_engine_tracks_host / _class_tracks_host);
// pending covariance predicts are materialised first
int snapshot_slots(bx_engine* e, int seq, const std::vector<int>& slots, int32_t* ids,
                   int32_t* state, int32_t* is_activated, int32_t* frame_id, int32_t* start_frame,
                   double* mean, double* cov) {
  const int T = e->dev.T;
  if (cov) {  // the covariance of tracks without an update since their last predicts
    if (e->cfg.kind == BX_BYTETRACK)
      hipLaunchKernelGGL(materialize_kernel<KIND_BYTE>, dim3((T + WG - 1) / WG), dim3(WG), 0, 0,
                         e->dev, seq);
    else
      hipLaunchKernelGGL(materialize_kernel<KIND_BOT>, dim3((T + WG - 1) / WG), dim3(WG), 0, 0,
                         e->dev, seq);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
  }
  std::vector<uint32_t> fl(T);
  std::vector<int> id(T), fid(T), st(T);
  std::vector<double> kf((size_t)KF_STRIDE * T);
  const size_t sT = (size_t)seq * T;
  HIPCHK(hipMemcpy(fl.data(), e->dev.flags + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(id.data(), e->dev.id + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(fid.data(), e->dev.frame_id + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(st.data(), e->dev.start + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(kf.data(), e->dev.kf + sT * KF_STRIDE, 8 * KF_STRIDE * (size_t)T,
                   hipMemcpyDeviceToHost));
  for (size_t k = 0; k < slots.size(); k++) {
    const int slot = slots[k];
    if (ids) ids[k] = id[slot];
    if (state) state[k] = (int)(fl[slot] & F_STATE);
    if (is_activated) is_activated[k] = (fl[slot] & F_ACT) ? 1 : 0;
    if (frame_id) frame_id[k] = fid[slot];
    if (start_frame) start_frame[k] = st[slot];
    for (int q = 0; q < 8 && mean; q++) mean[8 * k + q] = kf[(size_t)slot * KF_STRIDE + q];
    for (int q = 0; q < 64 && cov; q++) cov[64 * k + q] = kf[(size_t)slot * KF_STRIDE + 8 + q];
  }
  return BX_OK;
}
}  // namespace

int bx_engine_tracks_host(bx_engine* e, int seq, int cap, int32_t* ids, int32_t* state,
                          int32_t* is_activated, int32_t* frame_id, int32_t* start_frame,
                          double* mean, double* cov, int* n_active, int* n_lost) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIPCHK(hipDeviceSynchronize());
  const int T = e->dev.T;
  int v[SQ_STRIDE];
  HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  const int na = v[SQ_NA], nl = v[SQ_NL];
  if (n_active) *n_active = na;
  if (n_lost) *n_lost = nl;
  if (na + nl > cap) return set_err(BX_ERR_CAPACITY, "cap too small for the live tracks");
  std::vector<uint16_t> act(T), lost(T);
  const size_t sT = (size_t)seq * T;
  HIPCHK(hipMemcpy(act.data(), e->dev.act + sT, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lost.data(), e->dev.lost + sT, 2 * T, hipMemcpyDeviceToHost));
  std::vector<int> slots(na + nl);
  for (int k = 0; k < na + nl; k++) slots[k] = k < na ? act[k] : lost[k - na];
  return snapshot_slots(e, seq, slots, ids, state, is_activated, frame_id, start_frame, mean, cov);
}

int bx_engine_class_tracks_host(bx_engine* e, int seq, int n_classes, int cap, int32_t* cls_off,
                                int32_t* ids, int32_t* state, int32_t* is_activated,
                                int32_t* frame_id, int32_t* start_frame, double* mean,
                                double* cov) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S || n_classes <= 0 || !cls_off)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_class_tracks_host");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (e->n_classes && e->n_classes != n_classes)
    return set_err(BX_ERR_INVALID, "n_classes differs from the engine's per-class calls");
  const int T = e->dev.T, C = n_classes;
  std::vector<int> slots;
  for (int c = 0; c <= C; c++) cls_off[c] = 0;
  if (!e->n_classes || !e->park[seq]) return BX_OK;  // no per-class call yet: every list empty
  HIPCHK(hipDeviceSynchronize());
  int v[SQ_STRIDE];
  HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  std::vector<uint16_t> act(T), park((size_t)C * T);
  std::vector<int> npark(C);
  HIPCHK(hipMemcpy(act.data(), e->dev.act + (size_t)seq * T, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(park.data(), e->park[seq], 2 * (size_t)C * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(npark.data(), e->park[seq] + park_npark_off(e), sizeof(int) * C,
                   hipMemcpyDeviceToHost));
  // the class that ran last holds the engine's active list, every other class its parked one
  const int cur = e->cur_cls[seq];
  for (int c = 0; c < C; c++) {
    const int n = c == cur ? v[SQ_NA] : npark[c];
    for (int k = 0; k < n; k++) slots.push_back(c == cur ? act[k] : park[(size_t)c * T + k]);
    cls_off[c + 1] = (int)slots.size();
  }
  if ((int)slots.size() > cap) return set_err(BX_ERR_CAPACITY, "cap too small for the class lists");
  return snapshot_slots(e, seq, slots, ids, state, is_activated, frame_id, start_frame, mean, cov);
}

int bx_engine_state_set_host(bx_engine* e, int seq, int n, const int32_t* ids, const double* mean,
                             const double* cov) {
  if (int rc = settle(e)) return rc;
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || (n && !ids))
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_state_set_host");
  HIPCHK(hipDeviceSynchronize());
  const int T = e->dev.T;
  const size_t sT = (size_t)seq * T;
  int v[SQ_STRIDE];
  HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  const int na = v[SQ_NA], nl = v[SQ_NL];
  std::vector<uint16_t> act(T), lost(T);
  std::vector<int> id(T);
  HIPCHK(hipMemcpy(act.data(), e->dev.act + sT, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lost.data(), e->dev.lost + sT, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(id.data(), e->dev.id + sT, 4 * T, hipMemcpyDeviceToHost));
  for (int j = 0; j < n; j++) {
    int slot = -1;
    for (int k = 0; k < na + nl && slot < 0; k++) {
      const int sl = k < na ? act[k] : lost[k - na];
      if (id[sl] == ids[j]) slot = sl;
    }
    if (slot < 0) return set_err(BX_ERR_INVALID, "state_set: no live track with that id");
    double* kf = e->dev.kf + (sT + slot) * KF_STRIDE;
    uint32_t f;
    HIPCHK(hipMemcpy(&f, e->dev.flags + sT + slot, 4, hipMemcpyDeviceToHost));
    if (cov && pend_of(f)) {  // the set covariance is current: its pending predicts are void
      f &= ~F_PEND_MASK;
      HIPCHK(hipMemcpy(e->dev.flags + sT + slot, &f, 4, hipMemcpyHostToDevice));
    } else if (pend_of(f)) {  // keep the covariance: apply its pending predicts (with the
      // operands of the mean they were made from) before the mean changes
      if (e->cfg.kind == BX_BYTETRACK)
        hipLaunchKernelGGL(materialize_kernel<KIND_BYTE>, dim3((T + WG - 1) / WG), dim3(WG), 0,
                           0, e->dev, seq);
      else
        hipLaunchKernelGGL(materialize_kernel<KIND_BOT>, dim3((T + WG - 1) / WG), dim3(WG), 0,
                           0, e->dev, seq);
      HIPCHK(hipGetLastError());
      HIPCHK(hipDeviceSynchronize());
    }
    if (mean) HIPCHK(hipMemcpy(kf, mean + 8 * j, 8 * 8, hipMemcpyHostToDevice));
    if (cov) HIPCHK(hipMemcpy(kf + 8, cov + 64 * j, 64 * 8, hipMemcpyHostToDevice));
  }
  HIPCHK(hipDeviceSynchronize());
  return BX_OK;
}

int bx_engine_set_lap_stats(bx_engine* e, int on) {
  if (!e) return set_err(BX_ERR_INVALID, "null engine");
  if (int rc = settle(e)) return rc;
  e->dev.lap_stats = on != 0;
  return BX_OK;
}

int bx_engine_force_assoc_build(bx_engine* e, int mode) {
  if (!e || mode < -1 || mode > 1) return set_err(BX_ERR_INVALID, "bad assoc build mode");
  if (int rc = settle(e)) return rc;
  e->force_help = mode;
  return BX_OK;
}

int bx_engine_set_early_features(bx_engine* e, int on) {
  if (!e) return set_err(BX_ERR_INVALID, "null engine");
  if (int rc = settle(e)) return rc;
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (e->k1s) HIPCHK(hipStreamSynchronize(e->k1s));
  e->early = on != 0;
  return BX_OK;
}

int bx_engine_set_overlap(bx_engine* e, int on) {
  if (!e) return set_err(BX_ERR_INVALID, "null engine");
  if (int rc = settle(e)) return rc;
  e->overlap = on != 0;
  return BX_OK;
}

// copy S rows of `row_bytes` (src pitch sp, dst pitch dp) — a per-slot array [S][T][...] into a
// larger [S][T'][...]
static int copy_rows(void* dst, size_t dp, const void* src, size_t sp, size_t row_bytes, int S) {
  if (!row_bytes || !S) return BX_OK;
  HIPCHK(hipMemcpy2D(dst, dp, src, sp, row_bytes, S, hipMemcpyDeviceToDevice));
  return BX_OK;
}

int bx_engine_copy_state(bx_engine* dst, bx_engine* src) {
  if (!dst || !src) return set_err(BX_ERR_INVALID, "null engine");
  if (int rc = settle(src)) return rc;
  if (int rc = settle(dst)) return rc;
  const Dev &a = src->dev, &b = dst->dev;
  if (a.S != b.S || a.kind != b.kind || a.F != b.F || a.emb_f64 != b.emb_f64 ||
      a.with_reid != b.with_reid || b.T < a.T || b.D < a.D)
    return set_err(BX_ERR_INVALID,
                   "bx_engine_copy_state: destination must match the source's sequences, kind and "
                   "features and have at least its capacities");
  std::lock_guard<std::recursive_mutex> l1(src->mu), l2(dst->mu);
  HIPCHK(hipDeviceSynchronize());
  const int S = a.S;
  const size_t Ta = a.T, Tb = b.T, fs = a.emb_f64 ? 8 : 4;
  auto rows = [&](void* d, const void* s_, size_t per_slot) {
    return copy_rows(d, Tb * per_slot, s_, Ta * per_slot, Ta * per_slot, S);
  };
  int rc = BX_OK;
  const std::pair<std::pair<void*, const void*>, size_t> slot_arrays[] = {
      {{b.act, a.act}, 2}, {{b.lost, a.lost}, 2}, {{b.act2, a.act2}, 2},
      {{b.lost2, a.lost2}, 2}, {{b.flags, a.flags}, 4}, {{b.frame_id, a.frame_id}, 4},
      {{b.start, a.start}, 4}, {{b.id, a.id}, 4}, {{b.tlen, a.tlen}, 4},
      {{b.detind, a.detind}, 4}, {{b.conf, a.conf}, 8}, {{b.cls, a.cls}, 8},
      {{b.kf, a.kf}, 8 * KF_STRIDE}, {{b.clsh, a.clsh}, 8 * CLS_HIST * 2}, {{b.ncls, a.ncls}, 4},
  };
  for (auto& x : slot_arrays)
    if ((rc = rows(x.first.first, x.first.second, x.second))) return rc;
  if (a.with_reid) {
    if ((rc = rows(b.feat, a.feat, fs * a.F))) return rc;
    if ((rc = rows(b.tdn, a.tdn, 4))) return rc;
  }
  HIPCHK(hipMemcpy(b.seq, a.seq, sizeof(int) * SQ_STRIDE * S, hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(b.npair, a.npair, sizeof(int) * S, hipMemcpyDeviceToDevice));
  HIPCHK(hipMemcpy(b.status, a.status, sizeof(int) * 16, hipMemcpyDeviceToDevice));
  dst->overlap = src->overlap;
  dst->cache_seq = -1;
  // per_class state: parked class lists [C][T] (+ their lengths and the held frame counter)
  if (src->n_classes) {
    const int C = src->n_classes;
    if (dst->n_classes && dst->n_classes != C)
      return set_err(BX_ERR_INVALID, "bx_engine_copy_state: n_classes differs");
    if (!dst->n_classes) {
      dst->n_classes = C;
      dst->park.assign(S, nullptr);
      dst->cur_cls.assign(S, 0);
      HIPCHK(hipMalloc(&dst->h_coff, sizeof(int) * 2 * C));
      HIPCHK(hipMalloc(&dst->h_ccnt, sizeof(int) * C));
      HIPCHK(hipMalloc(&dst->h_cwarp, sizeof(double) * 6 * C));
    }
    for (int q = 0; q < S; q++) {
      dst->cur_cls[q] = src->cur_cls[q];
      if (!src->park[q]) continue;
      if (!dst->park[q]) {
        const size_t bytes = park_npark_off(dst) + sizeof(int) * (C + 1);
        HIPCHK(hipMalloc(&dst->park[q], bytes));
        HIPCHK(hipMemset(dst->park[q], 0, bytes));
      }
      if ((rc = copy_rows(dst->park[q], Tb * 2, src->park[q], Ta * 2, Ta * 2, C))) return rc;
      HIPCHK(hipMemcpy(dst->park[q] + park_npark_off(dst), src->park[q] + park_npark_off(src),
                       sizeof(int) * (C + 1), hipMemcpyDeviceToDevice));
    }
  }
  HIPCHK(hipDeviceSynchronize());
  return BX_OK;
}

int bx_engine_slots_used_host(bx_engine* e, int seq, int* used) {
  if (int rc = settle(e)) return rc;
  if (!e || !used || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  std::vector<uint32_t> f(e->dev.T);
  HIPCHK(hipMemcpy(f.data(), e->dev.flags + (size_t)seq * e->dev.T, sizeof(uint32_t) * f.size(),
                   hipMemcpyDeviceToHost));
  int n = 0;
  for (uint32_t x : f) n += (x & F_INUSE) != 0;
  *used = n;
  return BX_OK;
}

int bx_engine_inputs_released(bx_engine* e, void* stream) {
  if (!e) return set_err(BX_ERR_INVALID, "null engine");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (!e->side_pending) return BX_OK;
  // the last step's K5 is the last reader of its dets / det_off / embs: order `stream` after it
  HIPCHK(hipEventRecord(e->ev_join[1], e->side));
  HIPCHK(hipStreamWaitEvent((hipStream_t)stream, e->ev_join[1], 0));
  return BX_OK;
}

}  // extern "C"
