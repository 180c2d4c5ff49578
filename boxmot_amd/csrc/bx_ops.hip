// bx_ops.hip — op-level kernels of the C ABI (stateless, device pointers).  They share the
// device functions of the frame kernel (bx_device.h) and exist so every building block can be
// parity-checked on its own against the oracle and the reference's golden vectors.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/bxassoc.h"
#include "bx_device.h"

hipError_t bx_lds_attr(const void* kern, size_t bytes);  // bx_engine.hip (never lowers a limit)

using namespace bx;

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)

namespace {

int op_err(int code, const char* msg) { return bx_record_error(code, msg); }
#define OPCHK(x)                                                  \
  do {                                                            \
    hipError_t _e = (x);                                          \
    if (_e != hipSuccess) return op_err(BX_ERR_HIP, hipGetErrorString(_e)); \
  } while (0)

__global__ void iou_kernel(const double* a, int na, const double* b, int nb, double* out) {
  const size_t n = (size_t)na * nb;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(k / nb), j = (int)(k % nb);
    out[k] = iou_pair(a + 4 * i, b + 4 * j);
  }
}

__global__ void pairwise_kernel(int kind, const double* a, int na, int lda, const double* b,
                                int nb, int ldb, double fw, double fh, double* out) {
  const size_t n = (size_t)na * nb;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(k / nb), j = (int)(k % nb);
    out[k] = asso_pair(kind, a + (size_t)lda * i, b + (size_t)ldb * j, fw, fh);
  }
}

// compute_aw_max_metric (utils/association.py:320-374): one workgroup; thread per row, then per
// column, for the weights (LDS), then the grid of products in ((w * rw) * cw) * emb order
constexpr int AW_MAX = 4096;
__device__ double aw_weight(const double* v, int n, int stride, double bottom, bool* apply) {
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
  const double ex = m2 / m1 - bottom;
  return 1 - (ex > 0 ? ex : 0.0) / (1 - bottom);
}
__global__ void __launch_bounds__(1024) aw_kernel(const double* emb, int nr, int nc, double w0,
                                                  double bottom, double* out) {
  __shared__ double rw[AW_MAX], cw[AW_MAX];
  __shared__ bool ra[AW_MAX], ca[AW_MAX];
  for (int i = threadIdx.x; i < nr; i += blockDim.x)
    rw[i] = aw_weight(emb + (size_t)i * nc, nc, 1, bottom, &ra[i]);
  for (int j = threadIdx.x; j < nc; j += blockDim.x)
    cw[j] = aw_weight(emb + j, nr, nc, bottom, &ca[j]);
  __syncthreads();
  const size_t n = (size_t)nr * nc;
  for (size_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int i = (int)(k / nc), j = (int)(k % nc);
    double w = w0;
    if (ra[i]) w *= rw[i];
    if (ca[j]) w *= cw[j];
    out[k] = w * emb[k];
  }
}

__global__ void fuse_kernel(double* c, int nr, int nc, const double* conf) {
  const size_t n = (size_t)nr * nc;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x)
    c[k] = fuse_one(c[k], conf[k % nc]);
}

// per-row float32 norm (numpy pairwise) and the fp64 norm cdist computes of the normalised row
__global__ void row_norms_kernel(const float* x, int n, int f, float* dn, double* nrm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = x + (size_t)i * f;
  float d = sqrtf(np_pairwise_sumsq_f32(r, f)) + 1e-8f;
  struct V {
    const float* p;
    float d;
    __device__ double operator()(int k) const { return (double)(p[k] / d); }
  } A{r, d};
  dn[i] = d;
  nrm[i] = sqrt(dot2(A, A, f));
}

__global__ void cosine_kernel(const float* a, int na, const float* b, int nb, int f,
                              const float* adn, const double* anr, const float* bdn,
                              const double* bnr, double* out) {
  const size_t n = (size_t)na * nb;
  for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < n;
       k += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(k / nb), j = (int)(k % nb);
    struct V {
      const float* p;
      float d;
      __device__ double operator()(int q) const { return (double)(p[q] / d); }
    } A{a + (size_t)i * f, adn[i]}, B{b + (size_t)j * f, bdn[j]};
    double c = dot2(A, B, f) / (anr[i] * bnr[j]);
    if (fabs(c) > 1.0) c = copysign(1.0, c);
    double d = 1.0 - c;
    out[k] = d < 0.0 ? 0.0 : d;
  }
}

__global__ void kf_init_kernel(int kind, int n, const double* meas, double* mean, double* cov) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  kf_initiate(kind, meas + 4 * t, mean + 8 * t, cov + 64 * t);
}
__global__ void kf_predict_kernel(int kind, int n, double* mean, double* cov) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  double m[8], c[64];
  for (int k = 0; k < 8; k++) m[k] = mean[8 * t + k];
  for (int k = 0; k < 64; k++) c[k] = cov[64 * t + k];
  kf_predict_soa(kind, m, c, 1);
  for (int k = 0; k < 8; k++) mean[8 * t + k] = m[k];
  for (int k = 0; k < 64; k++) cov[64 * t + k] = c[k];
}
__global__ void kf_update_kernel(int kind, int n, double* mean, double* cov, const double* z,
                                 const double* conf) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  kf_update_soa(kind, mean + 8 * t, cov + 64 * t, 1, z + 4 * t, conf ? conf[t] : 0.0);
}
__global__ void kf_gate_kernel(int kind, int n, const double* mean, const double* cov,
                               const double* z, int nz, double* out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  kf_gating_soa(kind, mean + 8 * t, cov + 64 * t, 1, z, nz, out + (size_t)t * nz);
}

#include "bx_jv.h"

// One dense problem: CSR of admissible edges (cost < thresh) in LDS, then the wave LAP.  When
// the optimum is not unique (lap_tied_block) the problem is re-solved by lapx's own lapjv on the
// (nr+nc)^2 extension (matching.py:54-61: lap.lapjv(extend_cost=True, cost_limit=thresh)), read
// through an accessor, so ties resolve as lapx's do — its state in the kernel's LDS (the sparse
// solve's CSR and workspace are dead by then) when the launch sized it for that (jv_lds), else in
// `jvs` (global memory).
// Outputs: x[i] = column, -1 unmatched, -3 assigned by lapx to a real column above thresh (the
// reference neither matches nor lists such a row: matching.py:56-61); y likewise.
__global__ __launch_bounds__(WG) void lap_dense_kernel(const double* cost, int nr, int nc,
                                                       double thr, int elds, uint16_t* gcol,
                                                       double* gcost, unsigned char* jvs,
                                                       int jv_lds, int cls_lds, int32_t* x,
                                                       int32_t* y, int32_t* tied) {
  extern __shared__ __align__(16) unsigned char smem[];
  size_t o = 0;
  auto take = [&](size_t bytes) {
    unsigned char* p = smem + o;
    o += (bytes + 15) & ~size_t(15);
    return p;
  };
  double* u = (double*)take(8 * nr);
  double* v = (double*)take(8 * nc);
  double* spc = (double*)take(8 * nc);
  double* ecost = (double*)take(8 * elds);
  int* rowptr = (int*)take(4 * (nr + 1));
  int16_t* c4r = (int16_t*)take(2 * nr);
  uint16_t* srl = (uint16_t*)take(2 * nr);
  int16_t* r4c = (int16_t*)take(2 * nc);
  int16_t* path = (int16_t*)take(2 * nc);
  uint16_t* touch = (uint16_t*)take(2 * nc);
  uint16_t* ecol = (uint16_t*)take(2 * elds);
  uint8_t* colf = (uint8_t*)take(nc);
  int* cdeg = (int*)take(4 * nc);
  uint16_t* roots = (uint16_t*)take(2 * nr);
  int* rlab = (int*)take(4 * nr);
  int* caux = (int*)take(4 * nc);
  int* cmin = (int*)take(4 * nc);
  int* scan_tmp = (int*)take(4 * 8);
  const int tid = threadIdx.x;
  bool pre = false;  // a cost within BX_TIE_EPS of the limit: gain 0, a tie by itself
  for (int i = tid; i < nr; i += WG) {
    int cnt = 0;
    for (int j = 0; j < nc; j++) {
      const double c = cost[(size_t)i * nc + j];
      cnt += c < thr;
      pre |= fabs(c - thr) <= BX_TIE_EPS;
    }
    rowptr[i] = cnt;
  }
  __syncthreads();
  wave0_exclusive_scan(rowptr, nr);
  __syncthreads();
  for (int i = tid; i < nr; i += WG) {
    int e = rowptr[i];
    for (int j = 0; j < nc; j++) {
      double c = cost[(size_t)i * nc + j];
      if (!(c < thr)) continue;
      if (e < elds) { ecol[e] = (uint16_t)j; ecost[e] = c; }
      else { gcol[e - elds] = (uint16_t)j; gcost[e - elds] = c; }
      e++;
    }
  }
  __syncthreads();
  LapWS W;
  W.row_ptr = lds_ptr<int>(rowptr); W.ecol = lds_ptr<uint16_t>(ecol);
  W.ecost = lds_ptr<double>(ecost); W.gcol = gcol; W.gcost = gcost;
  W.elds = elds; W.col4row = lds_ptr<int16_t>(c4r); W.row4col = lds_ptr<int16_t>(r4c);
  W.u = lds_ptr<double>(u); W.v = lds_ptr<double>(v); W.spc = lds_ptr<double>(spc);
  W.path = lds_ptr<int16_t>(path); W.colflag = lds_ptr<uint8_t>(colf);
  W.touched = lds_ptr<uint16_t>(touch); W.srlist = lds_ptr<uint16_t>(srl);
  W.coldeg = lds_ptr<int>(cdeg);
  W.roots = lds_ptr<uint16_t>(roots);
  W.rlab = lds_ptr<int>(rlab);
  W.colaux = lds_ptr<int>(caux);
  W.colmin = lds_ptr<int>(cmin);
  lap_solve_block(nr, nc, thr, W, scan_tmp);
  const bool tie = lap_tied_block(nr, nc, thr, W, scan_tmp, pre);
  if (!tie) {
    for (int i = tid; i < nr; i += WG) x[i] = c4r[i];
    for (int j = tid; j < nc; j += WG) y[j] = r4c[j];
    if (tid == 0) *tied = 0;
    return;
  }
  const int n = nr + nc;
  __syncthreads();  // every wave is done with the CSR before the LDS is rebound
  JvLds jw = jv_bind(jv_lds ? smem : jvs, n);
  // row classes for the solver's scan skip (jv_wave_t): dummy rows 0; real rows whose every cost
  // equals the first constant row's 1 (flags in the LDS past the state when the launch sized it)
  unsigned char* cls = cls_lds ? smem + ((jv_bytes(n) + 15) & ~size_t(15)) : nullptr;
  if (cls) {
    for (int i = tid; i < nr; i += WG) {
      const double c0 = cost[(size_t)i * nc];
      bool cst = isfinite(c0);
      for (int j = 1; j < nc && cst; j++) cst = cost[(size_t)i * nc + j] == c0;
      cls[i] = cst ? 1 : 0;
    }
    __syncthreads();
    int i0 = 0;
    while (i0 < nr && !cls[i0]) i0++;
    const double K = i0 < nr ? cost[(size_t)i0 * nc] : 0.0;
    __syncthreads();
    for (int i = tid; i < nr; i += WG) cls[i] = cls[i] && cost[(size_t)i * nc] == K ? 1 : 0;
    __syncthreads();
  }
  if (wave_id() == 0) {
    const double half = thr / 2.;
    const JvExt cf{cost, nr, nc, half};
    auto rk = [&](int i) { return i >= nr ? 0 : (cls && cls[i] ? 1 : -1); };
    if (jv_lds) jv_wave_t(cf, n, jw, SyncWaveL{}, rk);
    else jv_wave_t(cf, n, jw, SyncWaveG{}, rk);
  }
  __syncthreads();
  for (int i = tid; i < nr; i += WG) {
    const int j = jw.x[i];
    x[i] = j >= nc ? -1 : (cost[(size_t)i * nc + j] <= thr ? j : -3);
  }
  for (int j = tid; j < nc; j += WG) {
    const int i = jw.y[j];
    y[j] = i >= nr ? -1 : (cost[(size_t)i * nc + j] <= thr ? i : -3);
  }
  if (tid == 0) *tied = 1;
}

int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

// lapx.lapjv(cost, extend_cost, cost_limit) on one dense problem, one wave: mode 0 = square,
// 1 = extend_cost (zero padding to max(nr, nc), read through cget), 2 = cost_limit (the
// (nr+nc)^2 extension with cost_limit / 2 off the diagonal blocks, read through an accessor).
// State in LDS when gst is null, else in global memory at gst.
// The legacy association.linear_assignment both ways on one matrix (n <= 64): lapx's lapjv
// (legacy_lap) and the shortest-augmenting-path solve with its uniqueness certificate
// (legacy_lap_ssp, lapjv only on a tie), for the op-level test that they agree.
__global__ __launch_bounds__(OW) void legacy_lap_pair_kernel(const double* cost, int nr, int nc,
                                                             int32_t* a, int32_t* b,
                                                             int32_t* info) {
  extern __shared__ __align__(16) unsigned char smem[];
  JvLds w = jv_bind(smem, nr > nc ? nr : nc);
  const int na = legacy_lap(cost, nr, nc, w, a);
  __syncthreads();
  bool ran = false;
  const int nb = legacy_lap_ssp(cost, nr, nc, w, b, SyncBlock{}, ran);
  if (threadIdx.x == 0) info[0] = na, info[1] = nb, info[2] = ran ? 1 : 0;
}

__global__ __launch_bounds__(OW) void lapjv_kernel(const double* cost, int nr, int nc, int mode,
                                                   double lim, unsigned char* gst, int32_t* x,
                                                   int32_t* y) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = mode == 2 ? nr + nc : (nr > nc ? nr : nc);
  JvLds w = jv_bind(gst ? gst : smem, n);
  // state past the LDS lives in global memory: the solver's atomics (column ownership) run in
  // L2, so their results are read back through an invalidated L1 (SyncWaveG)
  auto solve = [&](auto sync) {
    if (mode == 2) {
      const double half = lim / 2.;
      jv_wave_t(JvExt{cost, nr, nc, half}, n, w, sync,
                [&](int i) { return i >= nr ? 0 : -1; });  // dummy rows: one class
    } else if (n <= OW) {
      jv_wave64(cost, nr, nc, w);
    } else {
      jv_wave(cost, nr, nc, w, sync);
    }
  };
  if (gst)
    solve(SyncWaveG{});
  else
    solve(SyncBlock{});
  const bool cut = mode != 0;  // lapx: x >= n_cols -> -1, y >= n_rows -> -1, then [:nr] / [:nc]
  for (int i = threadIdx.x; i < nr; i += OW) x[i] = (cut && w.x[i] >= nc) ? -1 : w.x[i];
  for (int j = threadIdx.x; j < nc; j += OW) y[j] = (cut && w.y[j] >= nr) ? -1 : w.y[j];
}

}  // namespace

extern "C" {

int bx_iou_batch(const double* a, int na, const double* b, int nb, double* out, void* stream) {
  if (na < 0 || nb < 0) return op_err(BX_ERR_INVALID, "negative size");
  if (!na || !nb) return BX_OK;
  hipLaunchKernelGGL(iou_kernel, dim3(grid_for((size_t)na * nb)), dim3(256), 0,
                     (hipStream_t)stream, a, na, b, nb, out);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_pairwise_cost(int kind, const double* a, int na, int lda, const double* b, int nb,
                     int ldb, double w, double h, double* out, void* stream) {
  if (kind < BX_ASSO_IOU || kind > BX_ASSO_CENTROID)
    return op_err(BX_ERR_INVALID, "unknown association kind");
  if (na < 0 || nb < 0) return op_err(BX_ERR_INVALID, "negative size");
  if (!na || !nb) return BX_OK;
  if (lda < 4 || ldb < 4) return op_err(BX_ERR_INVALID, "row stride below 4");
  hipLaunchKernelGGL(pairwise_kernel, dim3(grid_for((size_t)na * nb)), dim3(256), 0,
                     (hipStream_t)stream, kind, a, na, lda, b, nb, ldb, w, h, out);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_aw_max_metric(const double* emb, int nr, int nc, double w_assoc, double bottom,
                     double* out, void* stream) {
  if (nr < 0 || nc < 0 || nr > AW_MAX || nc > AW_MAX)
    return op_err(BX_ERR_INVALID, "aw_max_metric: sizes out of range (0..4096)");
  if (!nr || !nc) return BX_OK;
  hipLaunchKernelGGL(aw_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, emb, nr, nc, w_assoc,
                     bottom, out);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_fuse_score(double* cost, int nr, int nc, const double* confs, void* stream) {
  if (nr < 0 || nc < 0) return op_err(BX_ERR_INVALID, "negative size");
  if (!nr || !nc) return BX_OK;
  hipLaunchKernelGGL(fuse_kernel, dim3(grid_for((size_t)nr * nc)), dim3(256), 0,
                     (hipStream_t)stream, cost, nr, nc, confs);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_embedding_distance(const float* trk, int nt, const float* det, int nd, int f, double* out,
                          void* stream) {
  if (nt < 0 || nd < 0 || f <= 0) return op_err(BX_ERR_INVALID, "bad sizes");
  if (!nt || !nd) return BX_OK;
  hipStream_t st = (hipStream_t)stream;
  void* ws = nullptr;
  const size_t bytes = (size_t)(nt + nd) * (sizeof(float) + sizeof(double)) + 64;
  OPCHK(hipMallocAsync(&ws, bytes, st));
  float* adn = (float*)ws;
  float* bdn = adn + nt;
  double* anr = (double*)(((uintptr_t)(bdn + nd) + 15) & ~uintptr_t(15));
  double* bnr = anr + nt;
  hipLaunchKernelGGL(row_norms_kernel, dim3((nt + 127) / 128), dim3(128), 0, st, trk, nt, f, adn,
                     anr);
  hipLaunchKernelGGL(row_norms_kernel, dim3((nd + 127) / 128), dim3(128), 0, st, det, nd, f, bdn,
                     bnr);
  hipLaunchKernelGGL(cosine_kernel, dim3(grid_for((size_t)nt * nd)), dim3(256), 0, st, trk, nt,
                     det, nd, f, adn, anr, bdn, bnr, out);
  OPCHK(hipGetLastError());
  OPCHK(hipFreeAsync(ws, st));
  return BX_OK;
}

int bx_kf_initiate(int kind, int n, const double* meas, double* mean, double* cov, void* stream) {
  if ((kind != 0 && kind != 1) || n < 0) return op_err(BX_ERR_INVALID, "bad kind/size");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_init_kernel, dim3((n + 127) / 128), dim3(128), 0, (hipStream_t)stream,
                     kind, n, meas, mean, cov);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_kf_multi_predict(int kind, int n, double* mean, double* cov, void* stream) {
  if ((kind != 0 && kind != 1) || n < 0) return op_err(BX_ERR_INVALID, "bad kind/size");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_predict_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     kind, n, mean, cov);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_kf_update(int kind, int n, double* mean, double* cov, const double* z, const double* conf,
                 void* stream) {
  if ((kind != 0 && kind != 1) || n < 0) return op_err(BX_ERR_INVALID, "bad kind/size");
  if (!n) return BX_OK;
  hipLaunchKernelGGL(kf_update_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                     kind, n, mean, cov, z, conf);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_kf_gating_distance(int kind, int n, const double* mean, const double* cov,
                          const double* z, int nz, double* out, void* stream) {
  if ((kind != 0 && kind != 1) || n < 0 || nz < 0) return op_err(BX_ERR_INVALID, "bad args");
  if (!n || !nz) return BX_OK;
  hipLaunchKernelGGL(kf_gate_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, kind,
                     n, mean, cov, z, nz, out);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_linear_assignment(const double* cost, int nr, int nc, double thresh, int32_t* x,
                         int32_t* y, void* stream) {
  return bx_linear_assignment_ex(cost, nr, nc, thresh, x, y, nullptr, stream);
}

int bx_linear_assignment_ex(const double* cost, int nr, int nc, double thresh, int32_t* x,
                            int32_t* y, int32_t* tied_out, void* stream) {
  if (nr < 0 || nc < 0 || nr > 8192 || nc > 8192)
    return op_err(BX_ERR_INVALID, "nr/nc out of range (0..8192)");
  hipStream_t st = (hipStream_t)stream;
  if (!nr || !nc) {
    if (nr) OPCHK(hipMemsetAsync(x, 0xff, sizeof(int32_t) * nr, st));
    if (nc) OPCHK(hipMemsetAsync(y, 0xff, sizeof(int32_t) * nc, st));
    return BX_OK;
  }
  int elds = 2048;
  auto lds_for = [&](int e) {
    size_t o = 0;
    auto take = [&](size_t b) { o += (b + 15) & ~size_t(15); };
    take(8 * nr); take(8 * nc); take(8 * nc); take(8 * e); take(4 * (nr + 1)); take(2 * nr);
    take(2 * nr); take(2 * nc); take(2 * nc); take(2 * nc); take(2 * e); take(nc); take(4 * nc);
    take(2 * nr);
    take(4 * nr);
    take(4 * nc);
    take(4 * nc);
    take(4 * 8);
    return o;
  };
  while (elds > 0 && lds_for(elds) > 160 * 1024) elds /= 2;
  size_t lds = lds_for(elds);
  if (lds > 160 * 1024) return op_err(BX_ERR_INVALID, "problem too large for LDS");
  // the tie re-solve's lapjv state in LDS too when it fits (n = nr + nc up to ~4000)
  const int jv_lds = jv_bytes(nr + nc) <= 160 * 1024;
  if (jv_lds && jv_bytes(nr + nc) > lds) lds = jv_bytes(nr + nc);
  // and the row-class flags of its scan skip past that state
  const size_t jvc = ((jv_bytes(nr + nc) + 15) & ~size_t(15)) + (size_t)nr;
  const int cls_lds = jv_lds && jvc <= 160 * 1024;
  if (cls_lds && jvc > lds) lds = jvc;
  void* ws = nullptr;
  const size_t ne = (size_t)nr * nc;
  const size_t jvb = (jv_bytes(nr + nc) + 255) & ~size_t(255);
  OPCHK(hipMallocAsync(&ws, jvb + 64 + ne * 10 + 64, st));
  unsigned char* jvs = (unsigned char*)ws;
  int32_t* tied = (int32_t*)(jvs + jvb);
  double* gcost = (double*)(jvs + jvb + 64);
  uint16_t* gcol = (uint16_t*)(gcost + ne);
  // (never lowers the limit a concurrent call on another thread or stream launches with)
  if (lds > 65536) OPCHK(bx_lds_attr((const void*)lap_dense_kernel, lds));
  hipLaunchKernelGGL(lap_dense_kernel, dim3(1), dim3(WG), lds, st, cost, nr, nc, thresh, elds,
                     gcol, gcost, jvs, jv_lds, cls_lds, x, y, tied);
  OPCHK(hipGetLastError());
  if (tied_out) OPCHK(hipMemcpyAsync(tied_out, tied, sizeof(int32_t), hipMemcpyDeviceToDevice, st));
  OPCHK(hipFreeAsync(ws, st));
  return BX_OK;
}

int bx_legacy_lap_pair(const double* cost, int nr, int nc, int32_t* pairs_jv, int32_t* pairs_ssp,
                       int32_t* info, void* stream) {
  if (nr < 0 || nc < 0 || (nr > nc ? nr : nc) > OW || !info)
    return op_err(BX_ERR_INVALID, "bx_legacy_lap_pair: 0 <= nr, nc <= 64");
  hipStream_t st = (hipStream_t)stream;
  if (!nr || !nc) {
    const int32_t z[3] = {0, 0, 0};
    OPCHK(hipMemcpyAsync(info, z, sizeof(z), hipMemcpyHostToDevice, st));
    return BX_OK;
  }
  const size_t lds = jv_bytes(nr > nc ? nr : nc);
  hipLaunchKernelGGL(legacy_lap_pair_kernel, dim3(1), dim3(OW), lds, st, cost, nr, nc, pairs_jv,
                     pairs_ssp, info);
  OPCHK(hipGetLastError());
  return BX_OK;
}

int bx_lapjv(const double* cost, int nr, int nc, int extend_cost, double cost_limit, int32_t* x,
             int32_t* y, void* stream) {
  const bool lim = cost_limit < INFINITY;  // NaN compares false: no limit, as lapx's `< np.inf`
  if (nr < 0 || nc < 0) return op_err(BX_ERR_INVALID, "negative size");
  if (!extend_cost && nr != nc)  // lapx checks this before the cost_limit extension
    return op_err(BX_ERR_INVALID,
                  "Square cost array expected. If cost is intentionally non-square, pass "
                  "extend_cost=True.");
  const int mode = lim ? 2 : (extend_cost ? 1 : 0);
  const int n = mode == 2 ? nr + nc : (nr > nc ? nr : nc);
  if (n > 32768) return op_err(BX_ERR_INVALID, "lapjv: extended size above 32768");
  hipStream_t st = (hipStream_t)stream;
  if (!nr || !nc) {
    if (nr) OPCHK(hipMemsetAsync(x, 0xff, sizeof(int32_t) * nr, st));
    if (nc) OPCHK(hipMemsetAsync(y, 0xff, sizeof(int32_t) * nc, st));
    return BX_OK;
  }
  const size_t lds = jv_bytes(n);
  unsigned char* gst = nullptr;
  if (lds > 160 * 1024) OPCHK(hipMallocAsync((void**)&gst, lds, st));
  const size_t dyn = gst ? 0 : lds;
  if (dyn > 65536) OPCHK(bx_lds_attr((const void*)lapjv_kernel, dyn));
  hipLaunchKernelGGL(lapjv_kernel, dim3(1), dim3(OW), dyn, st, cost, nr, nc, mode, cost_limit,
                     gst, x, y);
  OPCHK(hipGetLastError());
  if (gst) OPCHK(hipFreeAsync(gst, st));
  return BX_OK;
}

}  // extern "C"
