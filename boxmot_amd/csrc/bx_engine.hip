// bx_engine.hip — the per-frame association engine: ONE kernel launch advances one frame of
// many independent sequences, one 256-thread workgroup per sequence.
//
// Everything the reference's ByteTrack.update (trackers/bytetrack/bytetrack.py:158-302) and
// BotSort.update (trackers/botsort/botsort.py:94-411) do for a frame runs inside that
// workgroup: detection split, list bookkeeping (joint/sub/remove_duplicate_stracks), batched
// Kalman predict (+ CMC warp), IoU / score-fusion / re-ID cosine costs, three lapx-semantics
// assignments, Kalman updates, feature EMA, new-track initiation and output rows.  Track state
// stays resident in HBM between frames (SoA per sequence); lists, dets and the assignment
// workspace live in LDS for the frame.
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int CLS_HIST = 8;  // BoT-SORT per-track class-history entries (update_cls)
constexpr int ELDS_DEFAULT = 1024;  // LAP edges kept in LDS; the rest spill to global scratch
constexpr int REG_F = 512;   // feature rows up to this width live in registers: 8 per lane
constexpr int REG_EPL = REG_F / 64;

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
      if (lane + 64 * r < F) { double d = (double)v[r]; s += d * d; }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if constexpr (sizeof(FT) == 4) return sqrtf((float)s);
    else return sqrt(s);
  }
  __device__ void div(FT n) {
#pragma unroll
    for (int r = 0; r < REG_EPL; r++) v[r] = v[r] / n;
  }
  // numpy float32 norm of the float32-cast row (+1e-8 as embedding_distance adds it), staged
  // through this wave's LDS row so lanes can read numpy's accumulator layout
  __device__ float np_dn(float* wbuf, int F) const {
    store(wbuf, F);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float dn = sqrtf(np_sumsq_wave((const float*)wbuf, F)) + 1e-8f;
    __builtin_amdgcn_wave_barrier();
    return dn;
  }
};

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

// Device-side view of an engine (passed by value to the frame kernel).
struct Dev {
  int S, T, D, F, kind, emb_f64, with_reid, fuse_first, max_time_lost, elds;
  double low, high, new_thresh, match_thresh, prox, app;
  int* seq;           // [S][8]: n_active, n_lost, frame_count, id_count, status
  uint16_t* act;      // [S][T]
  uint16_t* lost;     // [S][T]
  uint32_t* flags;    // [S][T]
  int* frame_id;      // [S][T]
  int* start;         // [S][T]
  int* id;            // [S][T]
  int* tlen;          // [S][T]
  int* detind;        // [S][T]
  double* conf;       // [S][T]
  double* cls;        // [S][T]
  double* mean;       // [S][8][T]
  double* cov;        // [S][64][T]
  void* feat;         // [S][T][F]
  double* clsh;       // [S][T][CLS_HIST][2]
  int* ncls;          // [S][T]
  uint16_t* gcol;     // [S][T*D] LAP edge overflow
  double* gcost;      // [S][T*D]
  void* df2;          // [S][D][F] frame scratch: detection features after STrack.__init__
  float* dB;          // [S][D][F] frame scratch: det rows as embedding_distance normalises them
  float* tA;          // [S][T][F] frame scratch: track rows as embedding_distance normalises them
  int* status;        // [1] latched engine status
  unsigned long long* dbg;  // [S][32] phase stamps (diagnostic builds only, else null)
};

// Diagnostic phase stamps (build with -DBX_PHASE_TIMING; never in the shipped library).
#ifdef BX_PHASE_TIMING
#define BX_STAMP(k)                                                                   \
  do {                                                                                \
    __syncthreads();                                                                  \
    if (threadIdx.x == 0 && P.dbg) P.dbg[(size_t)s * 32 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define BX_STAMP(k) \
  do {              \
  } while (0)
#endif

enum { SQ_NA = 0, SQ_NL = 1, SQ_FC = 2, SQ_IDC = 3, SQ_STATUS = 4, SQ_STRIDE = 8 };

// LDS carve-out (host and device agree on it).
struct Lds {
  size_t o_act, o_lost, o_tracked, o_unconf, o_pool, o_rtr, o_lostl, o_refind, o_fa, o_fl,
      o_newt, o_flags, o_fid, o_mark, o_rowptr, o_c4r, o_u, o_srl, o_r4c, o_v, o_spc, o_path,
      o_colf, o_touch, o_dbox, o_dconf, o_dkind, o_hd, o_sd, o_rem, o_ecol, o_ecost, o_tdn,
      o_tna, o_ddn, o_dnb, o_ints, o_cdeg, o_wbuf, o_tbox, o_dboxf, o_tboxf, total;
  __host__ __device__ Lds(int T, int D, int elds, int F) {
    size_t o = 0;
    auto take = [&](size_t bytes) {
      size_t r = o;
      o += (bytes + 15) & ~size_t(15);
      return r;
    };
    int R = T > D ? T : D;  // assignment rows/cols never exceed these
    o_dbox = take(sizeof(double) * 4 * D);
    o_tbox = take(sizeof(double) * 4 * T);  // row boxes of the current association / dedup
    o_dconf = take(sizeof(double) * D);
    o_dboxf = take(sizeof(float) * 4 * D);  // outward-rounded fp32 copy for candidate tests
    o_tboxf = take(sizeof(float) * 4 * T);  // same for the rows of the current association
    o_u = take(sizeof(double) * T);
    o_v = take(sizeof(double) * D);
    o_spc = take(sizeof(double) * D);
    o_ecost = take(sizeof(double) * elds);
    o_tna = take(sizeof(double) * T);
    o_dnb = take(sizeof(double) * D);
    o_flags = take(sizeof(uint32_t) * T);
    o_fid = take(sizeof(int) * T);
    o_rowptr = take(sizeof(int) * (T + 1));
    o_tdn = o_ddn = 0;  // (unused: the norms are folded into the dB/tA rows)
    o_ints = take(sizeof(int) * 64);
    o_act = take(2 * T);
    o_lost = take(2 * T);
    o_tracked = take(2 * T);
    o_unconf = take(2 * T);
    o_pool = take(2 * T);
    o_rtr = take(2 * T);
    o_lostl = take(2 * T);
    o_refind = take(2 * T);
    o_fa = take(2 * T);
    o_fl = take(2 * T);
    o_newt = take(2 * D);
    o_c4r = take(2 * T);
    o_srl = take(2 * T);
    o_r4c = take(2 * D);
    o_path = take(2 * D);
    o_touch = take(2 * D);
    o_cdeg = take(4 * D);
    // per-wave float32 staging row for numpy's pairwise norm (register fast path, F <= 512)
    o_wbuf = take(F > 0 && F <= REG_F ? sizeof(float) * 4 * F : 0);
    o_hd = take(2 * D);
    o_sd = take(2 * D);
    o_rem = take(2 * D);
    o_ecol = take(2 * elds);
    o_mark = take(T);
    o_colf = take(D);
    o_dkind = take(D);
    (void)R;
    total = o;
  }
};

// mark bits (per slot, per frame)
enum : uint8_t { M_POOL = 1, M_ACT2 = 2, M_REMNOW = 4, M_DUP = 8, M_KEEP = 16, M_TMP = 32 };
// ints[] scratch slots
enum {
  I_NA = 0, I_NL, I_FC, I_IDC, I_N, I_DH, I_DS, I_NTR, I_NUN, I_NPOOL, I_NRTR, I_NLOSTL,
  I_NREF, I_NREM, I_NNEW, I_NFA, I_NFL, I_E, I_ERR, I_NACT0, I_NOUT, I_NFREE, I_SCAN = 32
};

template <typename FT>
struct FeatView {
  const FT* p;
  __device__ double operator()(int i) const { return (double)p[i]; }
};

// Normalised-float32 view used by matching.embedding_distance: x / (||x||_np + 1e-8) in f32.
template <typename FT>
struct NormF32View {
  const FT* p;
  float dn;
  __device__ double operator()(int i) const { return (double)((float)p[i] / dn); }
};

struct F32Row {
  const float* p;
  __device__ double operator()(int i) const { return (double)p[i]; }
};

// scipy cdist-cosine of two already-normalised float32 rows (matching.py:283-287), max(0, .)
__device__ inline double cosine_rows(const float* a, double na, const float* b, double nb,
                                     int F) {
  F32Row A{a}, B{b};
  double c = dot2(A, B, F) / (na * nb);
  if (fabs(c) > 1.0) c = copysign(1.0, c);
  double d = 1.0 - c;
  return d < 0.0 ? 0.0 : d;
}

// ------------------------------------------------------------------------------------------
template <int KIND, typename FT>
__global__ __launch_bounds__(WG) void frame_kernel(Dev P, int seq0, const float* __restrict__ dets,
                                                   const int* __restrict__ det_off,
                                                   const FT* __restrict__ embs,
                                                   const double* __restrict__ warps,
                                                   double* __restrict__ out,
                                                   int* __restrict__ out_count) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int T = P.T, D = P.D, F = P.F;
  const Lds Lo(T, D, P.elds, F);
  float* s_wbuf = (float*)(smem + Lo.o_wbuf) + (size_t)wave_id() * (F <= REG_F ? F : 0);
  uint16_t* s_act = (uint16_t*)(smem + Lo.o_act);
  uint16_t* s_lost = (uint16_t*)(smem + Lo.o_lost);
  uint16_t* s_tracked = (uint16_t*)(smem + Lo.o_tracked);
  uint16_t* s_unconf = (uint16_t*)(smem + Lo.o_unconf);
  uint16_t* s_pool = (uint16_t*)(smem + Lo.o_pool);
  uint16_t* s_rtr = (uint16_t*)(smem + Lo.o_rtr);
  uint16_t* s_lostl = (uint16_t*)(smem + Lo.o_lostl);
  uint16_t* s_refind = (uint16_t*)(smem + Lo.o_refind);
  uint16_t* s_fa = (uint16_t*)(smem + Lo.o_fa);
  uint16_t* s_fl = (uint16_t*)(smem + Lo.o_fl);
  uint16_t* s_newt = (uint16_t*)(smem + Lo.o_newt);
  uint32_t* s_flags = (uint32_t*)(smem + Lo.o_flags);
  int* s_fid = (int*)(smem + Lo.o_fid);
  uint8_t* s_mark = (uint8_t*)(smem + Lo.o_mark);
  int* s_rowptr = (int*)(smem + Lo.o_rowptr);
  int16_t* s_c4r = (int16_t*)(smem + Lo.o_c4r);
  double* s_u = (double*)(smem + Lo.o_u);
  uint16_t* s_srl = (uint16_t*)(smem + Lo.o_srl);
  int16_t* s_r4c = (int16_t*)(smem + Lo.o_r4c);
  double* s_v = (double*)(smem + Lo.o_v);
  double* s_spc = (double*)(smem + Lo.o_spc);
  int16_t* s_path = (int16_t*)(smem + Lo.o_path);
  uint8_t* s_colf = (uint8_t*)(smem + Lo.o_colf);
  uint16_t* s_touch = (uint16_t*)(smem + Lo.o_touch);
  double* s_dbox = (double*)(smem + Lo.o_dbox);
  float4* s_dboxf = (float4*)(smem + Lo.o_dboxf);
  double* s_dconf = (double*)(smem + Lo.o_dconf);
  uint8_t* s_dkind = (uint8_t*)(smem + Lo.o_dkind);
  uint16_t* s_hd = (uint16_t*)(smem + Lo.o_hd);
  uint16_t* s_sd = (uint16_t*)(smem + Lo.o_sd);
  uint16_t* s_rem = (uint16_t*)(smem + Lo.o_rem);
  uint16_t* s_ecol = (uint16_t*)(smem + Lo.o_ecol);
  double* s_ecost = (double*)(smem + Lo.o_ecost);
  double* s_tna = (double*)(smem + Lo.o_tna);
  double* s_dnb = (double*)(smem + Lo.o_dnb);
  int* I = (int*)(smem + Lo.o_ints);
  int* scan_tmp = I + I_SCAN;

  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const int s = seq0 + b;
  const size_t sT = (size_t)s * T;
  int* seq = P.seq + (size_t)s * SQ_STRIDE;
  uint32_t* g_flags = P.flags + sT;
  int* g_fid = P.frame_id + sT;
  int* g_start = P.start + sT;
  int* g_id = P.id + sT;
  int* g_tlen = P.tlen + sT;
  int* g_detind = P.detind + sT;
  double* g_conf = P.conf + sT;
  double* g_cls = P.cls + sT;
  double* g_mean = P.mean + (size_t)s * 8 * T;
  double* g_cov = P.cov + (size_t)s * 64 * T;
  FT* g_feat = (FT*)P.feat + (size_t)s * T * F;
  FT* g_df2 = (FT*)P.df2 + (size_t)s * D * F;
  double* g_clsh = P.clsh + sT * CLS_HIST * 2;
  int* g_ncls = P.ncls + sT;
  const int kf = KIND;  // KIND_BYTE → XYAH, KIND_BOT → XYWH
  const bool REID = (KIND == KIND_BOT) && P.with_reid;

  const int d0 = det_off[b], N = det_off[b + 1] - det_off[b];
  const float* fdets = dets + (size_t)d0 * 6;
  const FT* fembs = REID ? embs + (size_t)d0 * F : nullptr;

  BX_STAMP(0);
  // ---------------- P0: sequence state → LDS
  if (tid == 0) {
    I[I_NA] = seq[SQ_NA];
    I[I_NL] = seq[SQ_NL];
    I[I_FC] = seq[SQ_FC] + 1;
    I[I_IDC] = seq[SQ_IDC];
    I[I_N] = N;
    I[I_ERR] = 0;
  }
  __syncthreads();
  const int na = I[I_NA], nl = I[I_NL], fc = I[I_FC];
  if (N > D) {  // host checks det_cap; never trust it blindly
    if (tid == 0) { out_count[b] = 0; atomicOr(P.status, 1 << BX_ERR_CAPACITY); }
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

  // BoT-SORT: STrack(det, feat) → update_features: f1 = f/|f|, f2 = f1/|f1| (curr == smooth),
  // plus the float32 norms embedding_distance will need for the det side.
  if (REID) {
    // one wave per detection row (lane-strided, coalesced)
    if (F <= REG_F) {  // whole row in registers: one load, two stores; next row prefetched
      const int lane = lane_id();
      int p = wave_id();
      RegRow<FT> x;
      if (p < Dh) x.load(fembs + (size_t)s_hd[p] * F, F);
      for (; p < Dh; p += WG / WAVE) {
        const int k = s_hd[p], pn = p + WG / WAVE;
        RegRow<FT> nx;
        if (pn < Dh) nx.load(fembs + (size_t)s_hd[pn] * F, F);
        x.div(x.norm(F));
        x.div(x.norm(F));
        x.store(g_df2 + (size_t)k * F, F);
        const float dn = x.np_dn(s_wbuf, F);
        float* Bk = P.dB + ((size_t)s * D + k) * F;
#pragma unroll
        for (int r = 0; r < REG_EPL; r++) {
          const int q = lane + 64 * r;
          if (q < F) Bk[q] = (float)x.v[r] / dn;
        }
        x = nx;
      }
    }
    for (int p = wave_id(); p < (F <= REG_F ? 0 : Dh); p += WG / WAVE) {
      const int k = s_hd[p], lane = lane_id();
      const FT* f = fembs + (size_t)k * F;
      FT* f2 = g_df2 + (size_t)k * F;
      const FT n1 = wave_norm(f, F);
      for (int q = lane; q < F; q += WAVE) f2[q] = f[q] / n1;
      const FT n2 = wave_norm((const FT*)f2, F);  // same lane mapping: reads own writes
      for (int q = lane; q < F; q += WAVE) f2[q] = f2[q] / n2;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // other lanes read f2 next
      const float dn = sqrtf(np_sumsq_wave(f2, F)) + 1e-8f;
      float* Bk = P.dB + ((size_t)s * D + k) * F;
      for (int q = lane; q < F; q += WAVE) Bk[q] = (float)f2[q] / dn;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __syncthreads();
    // scipy cdist's norm of each normalised row: its own two-accumulator sequential order
    for (int p = tid; p < Dh; p += WG) {
      const int k = s_hd[p];
      const float* Bk = P.dB + ((size_t)s * D + k) * F;
      F32Row B{Bk};
      s_dnb[k] = sqrt(dot2(B, B, F));
    }
  }

  BX_STAMP(1);
  // ---------------- P2: tracked / unconfirmed / strack_pool = joint(tracked, lost)
  const int ntr = block_compact(na, [&](int k) { return (s_flags[s_act[k]] & F_ACT) != 0; },
                                [&](int k, int p) { s_tracked[p] = s_act[k]; }, scan_tmp);
  const int nun = block_compact(na, [&](int k) { return (s_flags[s_act[k]] & F_ACT) == 0; },
                                [&](int k, int p) { s_unconf[p] = s_act[k]; }, scan_tmp);
  for (int k = tid; k < ntr; k += WG) {
    s_pool[k] = s_tracked[k];
    s_mark[s_tracked[k]] |= M_POOL;
  }
  __syncthreads();
  const int npl = block_compact(nl, [&](int k) { return !(s_mark[s_lost[k]] & M_POOL); },
                                [&](int k, int p) { s_pool[ntr + p] = s_lost[k]; }, scan_tmp);
  const int npool = ntr + npl;
  for (int k = tid; k < npool; k += WG) s_mark[s_pool[k]] &= ~M_POOL;

  BX_STAMP(2);
  // ---------------- P3: multi_predict (+ BoT-SORT multi_gmc on pool and unconfirmed)
  const double* H = (KIND == KIND_BOT && warps) ? warps + 6 * (size_t)b : nullptr;
  for (int k = tid; k < npool + ((KIND == KIND_BOT) ? nun : 0); k += WG) {
    const bool is_pool = k < npool;
    const int slot = is_pool ? s_pool[k] : s_unconf[k - npool];
    double* m = g_mean + slot;
    double* c = g_cov + slot;
    if (is_pool) {
      if (st_of(s_flags[slot]) != ST_TRACKED) {
        if (KIND == KIND_BOT) m[6 * T] = 0.0;
        m[7 * T] = 0.0;
      }
      kf_predict_soa(kf, m, c, T);
    }
    if (H) {  // R8 = kron(I4, R): mean = R8·mean + t, cov = R8·cov·R8ᵀ
      double mm[8];
      for (int q = 0; q < 8; q++) mm[q] = m[q * T];
      for (int q = 0; q < 4; q++) {
        double a0 = H[0] * mm[2 * q] + H[1] * mm[2 * q + 1];
        double a1 = H[3] * mm[2 * q] + H[4] * mm[2 * q + 1];
        mm[2 * q] = a0;
        mm[2 * q + 1] = a1;
      }
      mm[0] += H[2];
      mm[1] += H[5];
      for (int q = 0; q < 8; q++) m[q * T] = mm[q];
      double RP[64];
      for (int bq = 0; bq < 4; bq++)
        for (int cc = 0; cc < 8; cc++) {
          double x0 = c[(8 * (2 * bq) + cc) * T], x1 = c[(8 * (2 * bq + 1) + cc) * T];
          RP[8 * (2 * bq) + cc] = H[0] * x0 + H[1] * x1;
          RP[8 * (2 * bq + 1) + cc] = H[3] * x0 + H[4] * x1;
        }
      for (int r = 0; r < 8; r++)
        for (int bq = 0; bq < 4; bq++) {
          double y0 = RP[8 * r + 2 * bq], y1 = RP[8 * r + 2 * bq + 1];
          c[(8 * r + 2 * bq) * T] = y0 * H[0] + y1 * H[1];
          c[(8 * r + 2 * bq + 1) * T] = y0 * H[3] + y1 * H[4];
        }
    }
  }
  __syncthreads();

  // track box (STrack.xyxy) from the current mean
  auto track_box = [&](int slot, double* box) {
    double r[4] = {g_mean[slot], g_mean[T + slot], g_mean[2 * T + slot], g_mean[3 * T + slot]};
    if (KIND == KIND_BYTE) r[2] *= r[3];
    xywh2xyxy(r, box);
  };

  // LAP workspace (rows use s_c4r/s_u/s_srl, columns s_r4c/s_v/s_spc/...)
  LapWS W;
  W.row_ptr = s_rowptr; W.ecol = s_ecol; W.ecost = s_ecost;
  W.gcol = P.gcol + (size_t)s * T * D; W.gcost = P.gcost + (size_t)s * T * D;
  W.elds = P.elds; W.col4row = s_c4r; W.row4col = s_r4c; W.u = s_u; W.v = s_v;
  W.spc = s_spc; W.path = s_path; W.colflag = s_colf; W.touched = s_touch; W.srlist = s_srl;
  W.coldeg = (int*)(smem + Lo.o_cdeg);
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
    // non-overlapping pairs have IoU 0: cost >= 1, never admissible, never gated (prox < 1)
    const bool prefilter = L <= 1.0 && (!reid || P.prox < 1.0);
    auto pair_cost = [&](const double* tb, int dk, bool& gated, bool& cand) -> double {
      double c = 1 - iou_pair(tb, s_dbox + 4 * dk);
      gated = false;
      if (mode == 1) {
        c = fuse_one(c, s_dconf[dk]);
      } else if (mode >= 2) {
        gated = reid && !(c > P.prox);
        if (mode == 3 || P.fuse_first) c = fuse_one(c, s_dconf[dk]);
      }
      cand = c < L || gated;
      return c;
    };
    // Candidates: one wave per row, lanes over columns, a conservative fp32 intersection test on
    // outward-rounded boxes (never misses an fp64-intersecting pair); a row's candidates keep
    // column order (ballot prefix).  Exact fp64 costs are then computed once per candidate with
    // every lane busy; candidates that turn out inadmissible stay in the CSR with cost INF,
    // which the solver treats as absent.  Row boxes are gathered into LDS first.
    // Lanes own columns: a lane keeps the boxes of its columns j = lane + 64k (k < 4, i.e.
    // C <= 256) in registers for the whole row sweep, so a row costs one broadcast LDS read.
    double* s_tbox = (double*)(smem + Lo.o_tbox);
    float4* s_tboxf = (float4*)(smem + Lo.o_tboxf);
    for (int i = tid; i < R; i += WG) {
      double* t = s_tbox + 4 * i;
      track_box(rows[i], t);
      s_tboxf[i] = make_float4(__double2float_rd(t[0]), __double2float_rd(t[1]),
                               __double2float_ru(t[2]), __double2float_ru(t[3]));
      s_srl[i] = 0;  // "row has a gated edge" flag; the LAP reuses s_srl afterwards
    }
    __syncthreads();
    const int lane = lane_id();
    constexpr int MAXCH = 4;
    const int nch = (C + WAVE - 1) / WAVE;
    const bool regcols = nch <= MAXCH;
    const float4 empty = make_float4(INFINITY, INFINITY, -INFINITY, -INFINITY);
    float4 cb[MAXCH];
#pragma unroll
    for (int k = 0; k < MAXCH; k++) {
      const int j = lane + WAVE * k;
      cb[k] = (regcols && j < C) ? s_dboxf[cols[j]] : empty;
    }
    auto hit = [&](const float4& tb, const float4& db, int j) -> bool {
      if (!prefilter) return j < C;
      return (fminf(tb.z, db.z) > fmaxf(tb.x, db.x)) & (fminf(tb.w, db.w) > fmaxf(tb.y, db.y));
    };
    auto chunk_mask = [&](const float4& tb, int k) -> unsigned long long {  // runtime k
      const int j = lane + WAVE * k;
      return __ballot(j < C && hit(tb, j < C ? s_dboxf[cols[j]] : empty, j));
    };
    // pass 1: count candidates per row
    for (int i = wave_id(); i < R; i += WG / WAVE) {
      const float4 tb = s_tboxf[i];
      int cnt = 0;
      if (regcols) {
#pragma unroll
        for (int k = 0; k < MAXCH; k++)
          if (k < nch) cnt += __popcll(__ballot(hit(tb, cb[k], lane + WAVE * k)));
      } else {
        for (int k = 0; k < nch; k++) cnt += __popcll(chunk_mask(tb, k));
      }
      if (lane == 0) s_rowptr[i] = cnt;
    }
    __syncthreads();
    wave0_exclusive_scan(s_rowptr, R);
    __syncthreads();
    // pass 2: write candidate columns in column order; the row index is parked in the cost slot
    for (int i = wave_id(); i < R; i += WG / WAVE) {
      const float4 tb = s_tboxf[i];
      int e = s_rowptr[i];
      auto emit = [&](unsigned long long m, int k) {
        if ((m >> lane) & 1ull)
          put_edge(e + __popcll(m & ((1ull << lane) - 1ull)), lane + WAVE * k, (double)i);
        e += __popcll(m);
      };
      if (regcols) {
#pragma unroll
        for (int k = 0; k < MAXCH; k++)
          if (k < nch) emit(__ballot(hit(tb, cb[k], lane + WAVE * k)), k);
      } else {
        for (int k = 0; k < nch; k++) emit(chunk_mask(tb, k), k);
      }
    }
    __syncthreads();
    // pass 3: exact fp64 cost per candidate (gated ones flagged in the column's top bit)
    for (int e = tid; e < s_rowptr[R]; e += WG) {
      int j;
      double ri;
      get_edge(e, j, ri);
      const int i = (int)ri;
      bool g, cand;
      const double c = pair_cost(s_tbox + 4 * i, cols[j], g, cand);
      put_edge(e, (g && cand) ? (j | 0x8000) : j, cand ? c : INF);
      if (g && cand) s_srl[i] = 1;
    }
    __syncthreads();
    if (reid) {
      // track rows as embedding_distance sees them: float32 smooth_feat / (np norm + 1e-8)
      for (int i = wave_id(); i < R; i += WG / WAVE) {
        if (!s_srl[i]) continue;  // wave-uniform
        const int slot = rows[i], lane = lane_id();
        const FT* tf = g_feat + (size_t)slot * F;
        float* A = P.tA + ((size_t)s * T + slot) * F;
        if (F <= REG_F) {
          RegRow<FT> x;
          x.load(tf, F);
          const float dn = x.np_dn(s_wbuf, F);
#pragma unroll
          for (int r = 0; r < REG_EPL; r++) {
            const int q = lane + 64 * r;
            if (q < F) A[q] = (float)x.v[r] / dn;
          }
          continue;
        }
        const float dn = sqrtf(np_sumsq_wave(tf, F)) + 1e-8f;
        for (int q = lane; q < F; q += WAVE) A[q] = (float)tf[q] / dn;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      __syncthreads();
      for (int i = tid; i < R; i += WG) {
        if (!s_srl[i]) continue;
        F32Row A{P.tA + ((size_t)s * T + rows[i]) * F};
        s_tna[rows[i]] = sqrt(dot2(A, A, F));
      }
      __syncthreads();
      // emb_dists = cdist/2; > appearance_thresh → 1; (not gated → 1); dists = min(iou, emb)
      const int E = s_rowptr[R];
      // thread per edge: find its row by binary search over row_ptr
      for (int e = tid; e < E; e += WG) {
        int col;
        double c;
        get_edge(e, col, c);
        if (!(col & 0x8000)) continue;
        int lo = 0, hi = R;  // row_ptr[lo] <= e < row_ptr[lo+1]
        while (hi - lo > 1) {
          int mid = (lo + hi) >> 1;
          if (s_rowptr[mid] <= e) lo = mid; else hi = mid;
        }
        const int slot = rows[lo], j = col & 0x7fff, dk = cols[j];
        double ed = cosine_rows(P.tA + ((size_t)s * T + slot) * F, s_tna[slot],
                                P.dB + ((size_t)s * D + dk) * F, s_dnb[dk], F) / 2.0;
        if (ed > P.app) ed = 1.0;
        double cm = c < ed ? c : ed;  // np.minimum(ious_dists, emb_dists)
        put_edge(e, j, cm < L ? cm : INF);
      }
      __syncthreads();
    }
    BX_STAMP(stamp);
    if (wave_id() == 0) lap_solve_wave(R, C, L, W);
    __syncthreads();
  };

  // ---------------- P4/P5: first association: pool x high dets
  BX_STAMP(3);
  associate(s_pool, npool, s_hd, Dh, P.match_thresh, KIND == KIND_BYTE ? 1 : 2, 4);
  BX_STAMP(5);

  // per-track matched update (STrack.update / re_activate)
  // botsort_track.py:40-49 update_features(det.curr_feat) on one track — one wave, lane-strided:
  // feat /= |feat|; smooth = 0.9 smooth + 0.1 feat; smooth /= |smooth|
  auto feature_update_wave = [&](int slot, int dk) {
    const int lane = lane_id();
    FT* sm = g_feat + (size_t)slot * F;
    const FT* f2 = g_df2 + (size_t)dk * F;
    const FT a = (FT)0.9, bb = (FT)(1.0 - 0.9);
    if (F <= REG_F) {
      RegRow<FT> g, m;
      g.load(f2, F);
      m.load(sm, F);
      const FT n3 = g.norm(F);
#pragma unroll
      for (int r = 0; r < REG_EPL; r++) {
        FT g3 = g.v[r] / n3;
        m.v[r] = a * m.v[r] + bb * g3;
      }
      m.div(m.norm(F));
      m.store(sm, F);
      return;
    }
    const FT n3 = wave_norm(f2, F);
    for (int q = lane; q < F; q += WAVE) {
      FT g3 = f2[q] / n3;
      sm[q] = a * sm[q] + bb * g3;
    }
    const FT ns = wave_norm((const FT*)sm, F);  // same lane mapping: reads own writes
    for (int q = lane; q < F; q += WAVE) sm[q] = sm[q] / ns;
  };
  // feature updates for the rows of the last solve that matched (rows[i] ↔ cols[c4r[i]]):
  // the matched pairs are compacted into the (now idle) LAP scratch, then one wave per pair
  // with the next pair's two rows prefetched into registers while this one computes.
  auto feature_updates = [&](const uint16_t* rows, int R, const uint16_t* cols) {
    uint16_t* ms = s_touch;
    int16_t* md = s_path;
    const int nm = block_compact(R, [&](int i) { return s_c4r[i] >= 0; },
                                 [&](int i, int p) {
                                   ms[p] = rows[i];
                                   md[p] = (int16_t)cols[s_c4r[i]];
                                 },
                                 scan_tmp);
    if (F > REG_F) {
      for (int p = wave_id(); p < nm; p += WG / WAVE) feature_update_wave(ms[p], md[p]);
      return;
    }
    const FT a = (FT)0.9, bb = (FT)(1.0 - 0.9);
    int p = wave_id();
    RegRow<FT> g, m;
    if (p < nm) {
      g.load(g_df2 + (size_t)md[p] * F, F);
      m.load(g_feat + (size_t)ms[p] * F, F);
    }
    for (; p < nm; p += WG / WAVE) {
      const int pn = p + WG / WAVE;
      RegRow<FT> ng, nm_;
      if (pn < nm) {
        ng.load(g_df2 + (size_t)md[pn] * F, F);
        nm_.load(g_feat + (size_t)ms[pn] * F, F);
      }
      const FT n3 = g.norm(F);
#pragma unroll
      for (int r = 0; r < REG_EPL; r++) {
        FT g3 = g.v[r] / n3;
        m.v[r] = a * m.v[r] + bb * g3;
      }
      m.div(m.norm(F));
      m.store(g_feat + (size_t)ms[p] * F, F);
      g = ng;
      m = nm_;
    }
  };

  auto apply_update = [&](int slot, int dk, bool reactivate, bool with_feat) {
    (void)with_feat;  // features: feature_updates() after the scalar pass
    const float* r = fdets + 6 * dk;
    double xyxy[4] = {(double)r[0], (double)r[1], (double)r[2], (double)r[3]};
    double xywh[4], meas[4];
    xyxy2xywh(xyxy, xywh);
    if (KIND == KIND_BYTE) {
      double tlwh[4];
      xywh2tlwh(xywh, tlwh);
      tlwh2xyah(tlwh, meas);
    } else {
      for (int q = 0; q < 4; q++) meas[q] = xywh[q];
    }
    kf_update_soa(kf, g_mean + slot, g_cov + slot, T, meas, 0.0);
    uint32_t fl = s_flags[slot];
    fl = (fl & ~F_STATE) | ST_TRACKED | F_ACT;
    s_flags[slot] = fl;
    s_fid[slot] = fc;
    g_tlen[slot] = reactivate ? 0 : g_tlen[slot] + 1;
    const double conf = (double)r[4], cls = (double)r[5];
    g_conf[slot] = conf;
    g_cls[slot] = cls;
    g_detind[slot] = dk;
    if (KIND == KIND_BOT) {  // update_cls (botsort_track.py:51-64)
      double* h = g_clsh + (size_t)slot * CLS_HIST * 2;
      int nh = g_ncls[slot];
      double max_freq = 0.0, out_cls = cls;
      bool found = false;
      for (int q = 0; q < nh; q++) {
        if (cls == h[2 * q]) { h[2 * q + 1] += conf; found = true; }
        if (h[2 * q + 1] > max_freq) { max_freq = h[2 * q + 1]; out_cls = h[2 * q]; }
      }
      if (!found) {
        if (nh < CLS_HIST) { h[2 * nh] = cls; h[2 * nh + 1] = conf; g_ncls[slot] = nh + 1; }
        else atomicOr(P.status, 1 << BX_ERR_TRACK_OVERFLOW);
        out_cls = cls;
      }
      g_cls[slot] = out_cls;
    }
  };

  // ---------------- P6: apply first-association matches (row order)
  for (int i = tid; i < npool; i += WG) {
    const int j = s_c4r[i];
    if (j < 0) continue;
    const int slot = s_pool[i];
    const bool tracked = st_of(s_flags[slot]) == ST_TRACKED;
    apply_update(slot, s_hd[j], !tracked, REID);
    if (!tracked) s_mark[slot] |= M_TMP;  // refind
  }
  if (REID) feature_updates(s_pool, npool, s_hd);
  __syncthreads();
  const int nref = block_compact(npool, [&](int k) { return (s_mark[s_pool[k]] & M_TMP) != 0; },
                                 [&](int k, int p) { s_refind[p] = s_pool[k]; }, scan_tmp);
  // remaining high dets (u_detection, ascending) — saved before the next solve reuses r4c
  const int nrem = block_compact(Dh, [&](int j) { return s_r4c[j] < 0; },
                                 [&](int j, int p) { s_rem[p] = s_hd[j]; }, scan_tmp);
  for (int k = tid; k < nref; k += WG) s_mark[s_refind[k]] &= ~M_TMP;
  // r_tracked = unmatched pool rows still Tracked
  const int nrtr = block_compact(
      npool, [&](int k) { return s_c4r[k] < 0 && st_of(s_flags[s_pool[k]]) == ST_TRACKED; },
      [&](int k, int p) { s_rtr[p] = s_pool[k]; }, scan_tmp);

  BX_STAMP(6);
  // ---------------- P7: second association: r_tracked x low-confidence dets (IoU, 0.5)
  associate(s_rtr, nrtr, s_sd, Ds, 0.5, 0, 7);
  for (int i = tid; i < nrtr; i += WG) {
    const int j = s_c4r[i];
    if (j < 0) continue;
    apply_update(s_rtr[i], s_sd[j], false, false);  // second dets carry no features
  }
  __syncthreads();
  const int nlostl = block_compact(
      nrtr, [&](int k) { return s_c4r[k] < 0; },
      [&](int k, int p) {
        const int slot = s_rtr[k];
        s_lostl[p] = (uint16_t)slot;
        s_flags[slot] = (s_flags[slot] & ~F_STATE) | ST_LOST;  // mark_lost
      },
      scan_tmp);

  // ---------------- P8: unconfirmed x remaining high dets (fused, 0.7)
  BX_STAMP(8);
  associate(s_unconf, nun, s_rem, nrem, 0.7, KIND == KIND_BYTE ? 1 : 3, 9);
  BX_STAMP(10);
  for (int i = tid; i < nun; i += WG) {
    const int j = s_c4r[i];
    const int slot = s_unconf[i];
    if (j >= 0) {
      apply_update(slot, s_rem[j], false, REID);
    } else {
      s_flags[slot] = (s_flags[slot] & ~F_STATE) | ST_REMOVED;  // mark_removed
      s_mark[slot] |= M_REMNOW;
    }
  }
  if (REID) feature_updates(s_unconf, nun, s_rem);
  __syncthreads();

  // ---------------- P9: new tracks from the detections left over (conf >= det/new thresh)
  const int nnew = block_compact(
      nrem, [&](int k) { return s_r4c[k] < 0 && s_dconf[s_rem[k]] >= P.new_thresh; },
      [&](int k, int p) { s_newt[p] = s_rem[k]; /* det index for now */ }, scan_tmp);
  // allocate the first nnew free slots (ascending)
  if (tid == 0) I[I_NFREE] = 0;
  __syncthreads();
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
  for (int p = tid; p < nnew_ok; p += WG) {
    const int dk = s_newt[p], slot = s_rtr[p];
    const float* r = fdets + 6 * dk;
    double xyxy[4] = {(double)r[0], (double)r[1], (double)r[2], (double)r[3]};
    double xywh[4], meas[4], m8[8], c64[64];
    xyxy2xywh(xyxy, xywh);
    if (KIND == KIND_BYTE) {
      double tlwh[4];
      xywh2tlwh(xywh, tlwh);
      tlwh2xyah(tlwh, meas);
    } else {
      for (int q = 0; q < 4; q++) meas[q] = xywh[q];
    }
    kf_initiate(kf, meas, m8, c64);
    for (int q = 0; q < 8; q++) g_mean[q * T + slot] = m8[q];
    for (int q = 0; q < 64; q++) g_cov[q * T + slot] = c64[q];
    g_id[slot] = idc0 + 1 + p;
    g_tlen[slot] = 0;
    g_conf[slot] = (double)r[4];
    g_cls[slot] = (double)r[5];
    g_detind[slot] = dk;
    s_flags[slot] = ST_TRACKED | F_INUSE | (fc == 1 ? F_ACT : 0u);
    s_fid[slot] = fc;
    g_start[slot] = fc;
    if (KIND == KIND_BOT) {
      double* h = g_clsh + (size_t)slot * CLS_HIST * 2;
      h[0] = (double)r[5];
      h[1] = (double)r[4];
      g_ncls[slot] = 1;
    }
    s_newt[p] = (uint16_t)slot;
  }
  if (tid == 0) I[I_IDC] = idc0 + nnew_ok;
  __syncthreads();
  if (REID) {  // smooth_feat of a new track = the detection's (already twice-normalised) feature
    for (int p = wave_id(); p < nnew_ok; p += WG / WAVE) {
      const int slot = s_newt[p], dk = g_detind[slot];
      FT* sm = g_feat + (size_t)slot * F;
      const FT* f2 = g_df2 + (size_t)dk * F;
      for (int q = lane_id(); q < F; q += WAVE) sm[q] = f2[q];
    }
  }

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

  // ---------------- P11: list rebuild (bytetrack.py:278-289 / botsort.py:392-403)
  // act2 = [t in active if Tracked] ++ new tracks ++ refind    (joint_stracks x2)
  int nact2 = block_compact(na, [&](int k) { return st_of(s_flags[s_act[k]]) == ST_TRACKED; },
                            [&](int k, int p) { s_fa[p] = s_act[k]; }, scan_tmp);
  for (int k = tid; k < nact2; k += WG) s_mark[s_fa[k]] |= M_ACT2;
  __syncthreads();
  for (int k = tid; k < nnew_ok; k += WG) { s_fa[nact2 + k] = s_newt[k]; s_mark[s_newt[k]] |= M_ACT2; }
  nact2 += nnew_ok;
  __syncthreads();
  {
    const int add = block_compact(nref, [&](int k) { return !(s_mark[s_refind[k]] & M_ACT2); },
                                  [&](int k, int p) { s_fa[nact2 + p] = s_refind[k]; }, scan_tmp);
    for (int k = tid; k < add; k += WG) s_mark[s_fa[nact2 + k]] |= M_ACT2;
    nact2 += add;
  }
  __syncthreads();
  // lost = sub(lost, active) ++ lost_local, then sub(., removed_stracks) (flag from earlier frames)
  int nlost1 = block_compact(nl, [&](int k) { return !(s_mark[s_lost[k]] & M_ACT2); },
                             [&](int k, int p) { s_fl[p] = s_lost[k]; }, scan_tmp);
  for (int k = tid; k < nlostl; k += WG) s_fl[nlost1 + k] = s_lostl[k];
  nlost1 += nlostl;
  __syncthreads();
  const int nlost2 = block_compact(nlost1, [&](int k) { return !(s_flags[s_fl[k]] & F_INREM); },
                                   [&](int k, int p) { s_tracked[p] = s_fl[k]; }, scan_tmp);
  // removed_stracks.extend(removed_local)
  for (int k = tid; k < T; k += WG)
    if (s_mark[k] & M_REMNOW) s_flags[k] |= F_INREM;
  __syncthreads();
  // remove_duplicate_stracks(act2, lost2): iou distance < 0.15 → drop the younger track
  {
    double* lbox = s_ecost;  // the LAP edge store is dead by now: lost boxes + ages live there
    const bool in_lds = nlost2 * 5 <= P.elds;
    double* abox = (double*)(smem + Lo.o_tbox);
    if (in_lds)
      for (int q = tid; q < nlost2; q += WG) {
        const int sb = s_tracked[q];
        track_box(sb, lbox + 4 * q);
        lbox[4 * nlost2 + q] = (double)(s_fid[sb] - g_start[sb]);
      }
    for (int p = tid; p < nact2; p += WG) track_box(s_fa[p], abox + 4 * p);
    __syncthreads();
    const int lane = lane_id();
    for (int p = wave_id(); p < nact2; p += WG / WAVE) {  // wave per active track
      const int sa = s_fa[p];
      const double* ba = abox + 4 * p;
      const int ta = s_fid[sa] - g_start[sa];
      bool dupa = false;
      for (int q = lane; q < nlost2; q += WAVE) {
        const int sb = s_tracked[q];
        double bb[4];
        if (in_lds) for (int k = 0; k < 4; k++) bb[k] = lbox[4 * q + k];
        else track_box(sb, bb);
        if (!boxes_intersect(ba, bb)) continue;
        if (1 - iou_pair(ba, bb) < 0.15) {
          const int tb = in_lds ? (int)lbox[4 * nlost2 + q] : s_fid[sb] - g_start[sb];
          if (ta > tb) atomicOr((unsigned*)&s_flags[sb], 0x80000000u);  // dupb (transient bit)
          else dupa = true;                                             // dupa
        }
      }
      if (__ballot(dupa) != 0ull && lane == 0) s_mark[sa] |= M_DUP;
    }
  }
  __syncthreads();
  const int nfa = block_compact(nact2, [&](int k) { return !(s_mark[s_fa[k]] & M_DUP); },
                                [&](int k, int p) { s_unconf[p] = s_fa[k]; }, scan_tmp);
  const int nfl = block_compact(
      nlost2, [&](int k) { return !(s_flags[s_tracked[k]] & 0x80000000u); },
      [&](int k, int p) { s_pool[p] = s_tracked[k]; }, scan_tmp);
  for (int k = tid; k < nlost2; k += WG) s_flags[s_tracked[k]] &= ~0x80000000u;
  __syncthreads();

  BX_STAMP(12);
  // ---------------- P12: outputs [x1,y1,x2,y2,id,conf,cls,det_ind] for activated tracks
  const int nout = block_compact(
      nfa, [&](int k) { return (s_flags[s_unconf[k]] & F_ACT) != 0; },
      [&](int k, int p) {
        const int slot = s_unconf[k];
        double box[4];
        track_box(slot, box);
        double* o = out + (size_t)(d0 + p) * 8;
        o[0] = box[0]; o[1] = box[1]; o[2] = box[2]; o[3] = box[3];
        o[4] = (double)g_id[slot];
        o[5] = g_conf[slot];
        o[6] = g_cls[slot];
        o[7] = (double)g_detind[slot];
      },
      scan_tmp);

  // ---------------- P13: free slots that left both lists; write back
  for (int k = tid; k < T; k += WG) s_mark[k] = 0;
  __syncthreads();
  for (int k = tid; k < nfa; k += WG) s_mark[s_unconf[k]] = M_KEEP;
  for (int k = tid; k < nfl; k += WG) s_mark[s_pool[k]] = M_KEEP;
  __syncthreads();
  for (int k = tid; k < T; k += WG) {
    uint32_t f = s_flags[k];
    if (!(s_mark[k] & M_KEEP)) f = 0;  // slot free (track unreachable from here on)
    g_flags[k] = f;
    g_fid[k] = s_fid[k];
  }
  for (int k = tid; k < nfa; k += WG) P.act[sT + k] = s_unconf[k];
  for (int k = tid; k < nfl; k += WG) P.lost[sT + k] = s_pool[k];
  if (tid == 0) {
    seq[SQ_NA] = nfa;
    seq[SQ_NL] = nfl;
    seq[SQ_FC] = fc;
    seq[SQ_IDC] = I[I_IDC];
    if (I[I_ERR]) seq[SQ_STATUS] |= 1 << BX_ERR_TRACK_OVERFLOW;
    out_count[b] = nout;
  }
  BX_STAMP(13);
}

// ------------------------------------------------------------------------------------------
__global__ void reset_kernel(int* seq, uint32_t* flags, int T, int seq0, int nseq) {
  const int s = seq0 + blockIdx.x;
  if (blockIdx.x >= nseq) return;
  for (int k = threadIdx.x; k < SQ_STRIDE; k += blockDim.x) seq[(size_t)s * SQ_STRIDE + k] = 0;
  for (int k = threadIdx.x; k < T; k += blockDim.x) flags[(size_t)s * T + k] = 0;
}

__global__ void set_id_kernel(int* seq, int s, int v) { seq[(size_t)s * SQ_STRIDE + SQ_IDC] = v; }

}  // namespace

struct bx_engine {
  bx_config cfg;
  Dev dev;
  int device;
  size_t lds_bytes;
  void* arena;
  size_t arena_bytes;
  // host-path staging (device)
  float* h_dets;
  void* h_embs;
  int* h_off;
  double* h_out;
  int* h_cnt;
  double* h_warp;
  std::mutex mu;
};

namespace {

template <typename T>
T* carve(char*& p, size_t n) {
  size_t bytes = (sizeof(T) * n + 255) & ~size_t(255);
  T* r = (T*)p;
  p += bytes;
  return r;
}

template <int KIND, typename FT>
int launch_frame(bx_engine* e, int seq0, int nseq, const float* dets, const int* det_off,
                 const void* embs, const double* warps, double* out, int* out_count,
                 hipStream_t st) {
  auto kern = frame_kernel<KIND, FT>;
  static thread_local size_t attr_set = 0;
  if (e->lds_bytes > 65536 && attr_set < e->lds_bytes) {
    HIPCHK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)e->lds_bytes));
    attr_set = e->lds_bytes;
  }
  hipLaunchKernelGGL(kern, dim3(nseq), dim3(WG), e->lds_bytes, st, e->dev, seq0, dets, det_off,
                     (const FT*)embs, warps, out, out_count);
  HIPCHK(hipGetLastError());
  return BX_OK;
}

}  // namespace

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
  size_t bytes = 0;
  auto acc = [&](size_t b) { bytes += (b + 255) & ~size_t(255); };
  acc(sizeof(int) * S * SQ_STRIDE); acc(2 * ST); acc(2 * ST); acc(4 * ST); acc(4 * ST);
  acc(4 * ST); acc(4 * ST); acc(4 * ST); acc(4 * ST); acc(8 * ST); acc(8 * ST);
  acc(8 * ST * 8); acc(8 * ST * 64); acc(fs * ST * (F ? F : 1)); acc(8 * ST * CLS_HIST * 2);
  acc(4 * ST); acc(2 * ST * D); acc(8 * ST * D); acc(fs * (size_t)S * D * (F ? F : 1)); acc(64);
  acc(4 * (size_t)S * D * (F ? F : 1)); acc(4 * ST * (F ? F : 1));
  e->arena_bytes = bytes;
  if (hipMalloc(&e->arena, bytes) != hipSuccess) {
    delete e;
    return set_err(BX_ERR_HIP, "hipMalloc of the engine arena failed");
  }
  char* p = (char*)e->arena;
  d.seq = carve<int>(p, (size_t)S * SQ_STRIDE);
  d.act = carve<uint16_t>(p, ST);
  d.lost = carve<uint16_t>(p, ST);
  d.flags = carve<uint32_t>(p, ST);
  d.frame_id = carve<int>(p, ST);
  d.start = carve<int>(p, ST);
  d.id = carve<int>(p, ST);
  d.tlen = carve<int>(p, ST);
  d.detind = carve<int>(p, ST);
  d.conf = carve<double>(p, ST);
  d.cls = carve<double>(p, ST);
  d.mean = carve<double>(p, ST * 8);
  d.cov = carve<double>(p, ST * 64);
  d.feat = carve<char>(p, fs * ST * (F ? F : 1));
  d.clsh = carve<double>(p, ST * CLS_HIST * 2);
  d.ncls = carve<int>(p, ST);
  d.gcol = carve<uint16_t>(p, ST * D);
  d.gcost = carve<double>(p, ST * D);
  d.df2 = carve<char>(p, fs * (size_t)S * D * (F ? F : 1));
  d.status = carve<int>(p, 16);
  d.dB = carve<float>(p, (size_t)S * D * (F ? F : 1));
  d.tA = carve<float>(p, ST * (F ? F : 1));
  d.dbg = nullptr;
#ifdef BX_PHASE_TIMING
  HIPCHK(hipMalloc(&d.dbg, sizeof(unsigned long long) * 32 * S));
  HIPCHK(hipMemset(d.dbg, 0, sizeof(unsigned long long) * 32 * S));
#endif
  HIPCHK(hipMemset(e->arena, 0, bytes));
  e->lds_bytes = Lds(T, D, d.elds, F).total;
  if (e->lds_bytes > 160 * 1024) {
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
  *out = e;
  return BX_OK;
}

int bx_engine_destroy(bx_engine* e) {
  if (!e) return BX_OK;
  (void)hipFree(e->arena);
  (void)hipFree(e->h_dets);
  (void)hipFree(e->h_embs);
  (void)hipFree(e->h_off);
  (void)hipFree(e->h_out);
  (void)hipFree(e->h_cnt);
  (void)hipFree(e->h_warp);
  delete e;
  return BX_OK;
}

int bx_engine_reset(bx_engine* e, int seq0, int nseq, void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S)
    return set_err(BX_ERR_INVALID, "bad sequence range");
  hipLaunchKernelGGL(reset_kernel, dim3(nseq), dim3(256), 0, (hipStream_t)stream, e->dev.seq,
                     e->dev.flags, e->dev.T, seq0, nseq);
  HIPCHK(hipGetLastError());
  return BX_OK;
}

int bx_engine_step(bx_engine* e, int seq0, int nseq, const float* dets, const int32_t* det_off,
                   const void* embs, const double* warps, double* out, int32_t* out_count,
                   void* stream) {
  if (!e || seq0 < 0 || nseq <= 0 || seq0 + nseq > e->dev.S || !det_off || !out || !out_count)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_step");
  if (e->dev.with_reid && !embs) return set_err(BX_ERR_SHAPE, "BoT-SORT with_reid needs embs");
  hipStream_t st = (hipStream_t)stream;
  if (e->dev.kind == BX_BYTETRACK)
    return launch_frame<KIND_BYTE, float>(e, seq0, nseq, dets, det_off, embs, warps, out,
                                          out_count, st);
  if (e->dev.emb_f64)
    return launch_frame<KIND_BOT, double>(e, seq0, nseq, dets, det_off, embs, warps, out,
                                          out_count, st);
  return launch_frame<KIND_BOT, float>(e, seq0, nseq, dets, det_off, embs, warps, out, out_count,
                                       st);
}

int bx_engine_update_host(bx_engine* e, int seq, const float* dets, int n, const void* embs,
                          const double* warp, double* out, int* n_out, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S || n < 0 || !n_out)
    return set_err(BX_ERR_INVALID, "bad arguments to bx_engine_update_host");
  if (n > e->dev.D) return set_err(BX_ERR_CAPACITY, "detections exceed det_cap");
  if (e->dev.with_reid && n > 0 && !embs)
    return set_err(BX_ERR_SHAPE, "BoT-SORT with_reid needs embs");
  std::lock_guard<std::mutex> lk(e->mu);
  hipStream_t st = (hipStream_t)stream;
  const size_t fs = e->cfg.emb_f64 ? 8 : 4;
  int off[2] = {0, n};
  if (n) HIPCHK(hipMemcpyAsync(e->h_dets, dets, sizeof(float) * 6 * n, hipMemcpyHostToDevice, st));
  if (n && e->dev.with_reid)
    HIPCHK(hipMemcpyAsync(e->h_embs, embs, fs * (size_t)n * e->dev.F, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(e->h_off, off, sizeof(off), hipMemcpyHostToDevice, st));
  if (warp) HIPCHK(hipMemcpyAsync(e->h_warp, warp, sizeof(double) * 6, hipMemcpyHostToDevice, st));
  int rc = bx_engine_step(e, seq, 1, e->h_dets, e->h_off, e->h_embs, warp ? e->h_warp : nullptr,
                          e->h_out, e->h_cnt, stream);
  if (rc) return rc;
  int cnt = 0;
  HIPCHK(hipMemcpyAsync(&cnt, e->h_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (cnt && out)
    HIPCHK(hipMemcpy(out, e->h_out, sizeof(double) * 8 * cnt, hipMemcpyDeviceToHost));
  *n_out = cnt;
  int status = 0;
  HIPCHK(hipMemcpy(&status, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  if (status & (1 << BX_ERR_TRACK_OVERFLOW))
    return set_err(BX_ERR_TRACK_OVERFLOW, "a sequence ran out of track slots (raise track_cap)");
  return BX_OK;
}

#ifdef BX_PHASE_TIMING
// diagnostic only: copy the [S][32] phase stamps of the last launch to the host
int bx_debug_stamps_host(bx_engine* e, unsigned long long* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, e->dev.dbg, sizeof(unsigned long long) * 32 * e->dev.S,
                   hipMemcpyDeviceToHost));
  return BX_OK;
}
#endif

int bx_engine_status(bx_engine* e, int* status) {
  if (!e || !status) return set_err(BX_ERR_INVALID, "null argument");
  int s = 0;
  HIPCHK(hipMemcpy(&s, e->dev.status, sizeof(int), hipMemcpyDeviceToHost));
  *status = (s & (1 << BX_ERR_TRACK_OVERFLOW)) ? BX_ERR_TRACK_OVERFLOW
            : (s & (1 << BX_ERR_CAPACITY))     ? BX_ERR_CAPACITY
                                               : BX_OK;
  return BX_OK;
}

int bx_engine_counters_host(bx_engine* e, int seq, int* frame_count, int* id_count, int* n_active,
                            int* n_lost) {
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  int v[SQ_STRIDE];
  HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  if (frame_count) *frame_count = v[SQ_FC];
  if (id_count) *id_count = v[SQ_IDC];
  if (n_active) *n_active = v[SQ_NA];
  if (n_lost) *n_lost = v[SQ_NL];
  return BX_OK;
}

int bx_engine_set_id_count(bx_engine* e, int seq, int id_count, void* stream) {
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  hipLaunchKernelGGL(set_id_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, e->dev.seq, seq,
                     id_count);
  HIPCHK(hipGetLastError());
  return BX_OK;
}

int bx_engine_tracks_host(bx_engine* e, int seq, int cap, int32_t* ids, int32_t* state,
                          int32_t* is_activated, int32_t* frame_id, int32_t* start_frame,
                          double* mean, double* cov, int* n_active, int* n_lost) {
  if (!e || seq < 0 || seq >= e->dev.S) return set_err(BX_ERR_INVALID, "bad sequence");
  HIPCHK(hipDeviceSynchronize());
  const int T = e->dev.T;
  int v[SQ_STRIDE];
  HIPCHK(hipMemcpy(v, e->dev.seq + (size_t)seq * SQ_STRIDE, sizeof(v), hipMemcpyDeviceToHost));
  const int na = v[SQ_NA], nl = v[SQ_NL];
  if (n_active) *n_active = na;
  if (n_lost) *n_lost = nl;
  if (na + nl > cap) return set_err(BX_ERR_CAPACITY, "cap too small for the live tracks");
  std::vector<uint16_t> act(T), lost(T);
  std::vector<uint32_t> fl(T);
  std::vector<int> id(T), fid(T), st(T);
  std::vector<double> m((size_t)8 * T), c((size_t)64 * T);
  const size_t sT = (size_t)seq * T;
  HIPCHK(hipMemcpy(act.data(), e->dev.act + sT, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(lost.data(), e->dev.lost + sT, 2 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(fl.data(), e->dev.flags + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(id.data(), e->dev.id + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(fid.data(), e->dev.frame_id + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(st.data(), e->dev.start + sT, 4 * T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(m.data(), e->dev.mean + sT * 8, 8 * 8 * (size_t)T, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(c.data(), e->dev.cov + sT * 64, 8 * 64 * (size_t)T, hipMemcpyDeviceToHost));
  for (int k = 0; k < na + nl; k++) {
    const int slot = k < na ? act[k] : lost[k - na];
    if (ids) ids[k] = id[slot];
    if (state) state[k] = (int)(fl[slot] & F_STATE);
    if (is_activated) is_activated[k] = (fl[slot] & F_ACT) ? 1 : 0;
    if (frame_id) frame_id[k] = fid[slot];
    if (start_frame) start_frame[k] = st[slot];
    for (int q = 0; q < 8 && mean; q++) mean[8 * k + q] = m[(size_t)q * T + slot];
    for (int q = 0; q < 64 && cov; q++) cov[64 * k + q] = c[(size_t)q * T + slot];
  }
  return BX_OK;
}

}  // extern "C"
