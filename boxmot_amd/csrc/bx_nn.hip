// bx_nn.hip — StrongSort's appearance metric on MI355X: the nearest-neighbour cosine distance of
// every detection to every target's gallery of samples.
//
// Reference: NearestNeighborDistanceMetric.distance (boxmot/trackers/strongsort/sort/
// linear_assignment.py:595-618) -> _nn_cosine_distance (:468-497) -> _cosine_distance (:382-413):
//   x̂ = x / (np.linalg.norm(x, axis=1) + 1e-8) for samples and detection features (float64),
//   dist(t, d) = min over the samples s of target t of 1 - clip(ŝ·d̂, -1, 1); 1e5 without samples.
//
// The contraction is a (samples x F) · (F x dets) fp64 GEMM on the matrix cores
// (v_mfma_f64_16x16x4_f64, measured to be a k-ordered fma chain -> bitwise equal to
// oracle/bxo_ops.c:bxo_nn_cosine_distance, which restates np.dot's unpinned BLAS order this way).
// min over samples of 1 - clip(x) = 1 - clip(max over samples of x) exactly (monotone rounding),
// so the epilogue keeps a per-(target, detection) maximum of the raw dot product as an
// order-preserving 64-bit key updated with atomicMax; a last pass maps it to the distance.
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/bxassoc.h"
#include "bx_device.h"

int bx_record_error(int code, const char* msg);  // bx_engine.hip (shared bx_last_error)

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- row normalisation (numpy's float64 pairwise sum of squares, PW_BLOCKSIZE 128) ----------
__device__ double np_pairwise_sumsq_f64(const double* x, int n) {
  double acc[24];
  int ap = 0;
  int stk_off[24], stk_n[24], stk_state[24], top = 1;
  stk_off[0] = 0;
  stk_n[0] = n;
  stk_state[0] = 0;
  while (top > 0) {
    const int t = top - 1;
    const int off = stk_off[t], m = stk_n[t];
    if (m <= 128) {
      double res;
      if (m < 8) {
        res = 0.0;
        for (int i = 0; i < m; i++) {
          const double v = x[off + i];
          res += v * v;
        }
      } else {
        double r[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const double v = x[off + k];
          r[k] = v * v;
        }
        int i;
        for (i = 8; i < m - (m % 8); i += 8)
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const double v = x[off + i + k];
            r[k] += v * v;
          }
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < m; i++) {
          const double v = x[off + i];
          res += v * v;
        }
      }
      acc[ap++] = res;
      top--;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (stk_state[t] == 0) {
      stk_state[t] = 1;
      stk_off[top] = off;
      stk_n[top] = n2;
      stk_state[top] = 0;
      top++;
    } else if (stk_state[t] == 1) {
      stk_state[t] = 2;
      stk_off[top] = off + n2;
      stk_n[top] = m - n2;
      stk_state[top] = 0;
      top++;
    } else {
      const double b = acc[--ap], a = acc[--ap];
      acc[ap++] = a + b;
      top--;
    }
  }
  return acc[0];
}

// thread per row: the norm denominator sqrt(sum) + 1e-8
__global__ void nn_norm_kernel(const double* __restrict__ x, int n, int F, double* __restrict__ den) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) den[i] = sqrt(np_pairwise_sumsq_f64(x + (size_t)i * F, F)) + 1e-8;
}

// x̂ = x / den, a block-stride pass over [n][F] (coalesced)
__global__ void nn_scale_kernel(const double* __restrict__ x, const double* __restrict__ den,
                                size_t total, int F, double* __restrict__ y) {
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < total;
       q += (size_t)gridDim.x * blockDim.x)
    y[q] = x[q] / den[q / F];
}

__global__ void nn_row_target_kernel(const int* __restrict__ off, int T, int* __restrict__ tgt) {
  const int t = blockIdx.x;
  if (t >= T) return;
  for (int r = off[t] + threadIdx.x; r < off[t + 1]; r += blockDim.x) tgt[r] = t;
}

// order-preserving map of a double onto uint64 (key(a) < key(b) <=> a < b; -0 < +0)
__device__ __forceinline__ unsigned long long dkey(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double dval(unsigned long long k) {
  const unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)u);
}

// ---- the contraction ------------------------------------------------------------------------
// Workgroup tile: BM = 128 sample rows x BN = 256 detections, 8 waves (wave w: rows
// 32 (w & 3) .. +31, detections 128 (w >> 2) .. +127 = 2 x 8 tiles of 16 x 16 fp64 MFMA
// accumulators).  K advances in chunks of 16 through double-buffered LDS images stored k-major
// ([k][row], [k][det]; 16-double padding keeps the four k rows of one operand read on distinct
// bank halves).
constexpr int BM = 128, BN = 256, KC = 16, NT = 512;
constexpr int LDA = BM + 16, LDB = BN + 16;
constexpr int LDS_STAGE = KC * (LDA + LDB);  // doubles per buffer

__global__ void __launch_bounds__(NT)
    nn_cosine_mfma_kernel(const double* __restrict__ S, int G, const double* __restrict__ Dm,
                          int D, int F, const int* __restrict__ tgt,
                          unsigned long long* __restrict__ keys) {
  extern __shared__ __align__(16) double lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rg = w & 3, cg = w >> 2;
  // column blocks fastest: the sample rows of a row block stay hot while its column blocks run
  const int ncb = (D + BN - 1) / BN;
  const int row0 = (blockIdx.x / ncb) * BM, col0 = (blockIdx.x % ncb) * BN;

  // staging assignment: A 128 rows x 16 k = 4 doubles per thread; B 256 dets x 16 k = 8
  const int ar = tid >> 2, aq = tid & 3;
  const int bc = tid >> 1, bh = tid & 1;
  const bool a_ok = row0 + ar < G, b_ok = col0 + bc < D;
  const double* ap = S + (size_t)(row0 + ar) * F + 4 * aq;
  const double* bp = Dm + (size_t)(col0 + bc) * F + 8 * bh;

  double ra[4], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; j++) ra[j] = (a_ok && k0 + 4 * aq + j < F) ? ap[k0 + j] : 0.0;
#pragma unroll
    for (int j = 0; j < 8; j++) rb[j] = (b_ok && k0 + 8 * bh + j < F) ? bp[k0 + j] : 0.0;
  };
  auto store = [&](double* buf) {
    double* As = buf;
    double* Bs = buf + KC * LDA;
#pragma unroll
    for (int j = 0; j < 4; j++) As[(4 * aq + j) * LDA + ar] = ra[j];
#pragma unroll
    for (int j = 0; j < 8; j++) Bs[(8 * bh + j) * LDB + bc] = rb[j];
  };

  d4 acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 8; j++) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  const int nk = (F + KC - 1) / KC;
  load(0);
  store(lds);
  __syncthreads();
  for (int kc = 0; kc < nk; kc++) {
    double* cur = lds + (kc & 1) * LDS_STAGE;
    if (kc + 1 < nk) load((kc + 1) * KC);  // next chunk's global loads overlap the MFMAs
    const double* As = cur;
    const double* Bs = cur + KC * LDA;
#pragma unroll
    for (int ks = 0; ks < KC / 4; ks++) {
      const int kr = ks * 4 + (lane >> 4);
      double a[2], bq[8];
#pragma unroll
      for (int i = 0; i < 2; i++) a[i] = As[kr * LDA + rg * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 8; j++) bq[j] = Bs[kr * LDB + cg * 128 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 8; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], bq[j], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) store(lds + ((kc + 1) & 1) * LDS_STAGE);
    __syncthreads();
  }

  // epilogue: lane holds column (lane & 15) of each tile, rows (lane >> 4) + 4 m, m = 0..7 in
  // increasing order across (i, r); runs of one target are reduced before the atomic
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int col = col0 + cg * 128 + j * 16 + (lane & 15);
    if (col >= D) continue;
    int cur_t = -1;
    double cur = 0.0;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + rg * 32 + i * 16 + (lane >> 4) + 4 * r;
        if (row >= G) continue;
        const int t = tgt[row];
        const double v = acc[i][j][r];
        if (t != cur_t) {
          if (cur_t >= 0) atomicMax(&keys[(size_t)cur_t * D + col], dkey(cur));
          cur_t = t;
          cur = v;
        } else if (dkey(v) > dkey(cur)) {
          cur = v;
        }
      }
    if (cur_t >= 0) atomicMax(&keys[(size_t)cur_t * D + col], dkey(cur));
  }
}

// dist = 1 - clip(max dot, -1, 1); a target without samples costs INFTY_COST = 1e5
__global__ void nn_finish_kernel(const unsigned long long* __restrict__ keys,
                                 const int* __restrict__ off, int T, int D,
                                 double* __restrict__ out) {
  const size_t n = (size_t)T * D;
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < n;
       q += (size_t)gridDim.x * blockDim.x) {
    const int t = (int)(q / D);
    if (off[t + 1] <= off[t]) {
      out[q] = 1e5;
    } else {
      double c = dval(keys[q]);
      c = c < -1.0 ? -1.0 : (c > 1.0 ? 1.0 : c);
      out[q] = 1.0 - c;
    }
  }
}

int grid_for(size_t n, int per = 256) {
  size_t g = (n + per - 1) / per;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

#define NCHK(x)                                                                          \
  do {                                                                                   \
    hipError_t _e = (x);                                                                 \
    if (_e != hipSuccess)                                                                \
      return bx_record_error(BX_ERR_HIP, (std::string(#x) + ": " + hipGetErrorString(_e)).c_str()); \
  } while (0)

}  // namespace

extern "C" {

int bx_nn_cosine_distance(const double* samples, int G, const int32_t* off, int T,
                          const double* feats, int D, int F, int flags, double* out, void* stream) {
  if (T < 0 || D < 0 || F <= 0 || G < 0 || (T && !off) || (T && D && (!out || !feats)) ||
      (G && !samples))
    return bx_record_error(BX_ERR_INVALID, "bad arguments to bx_nn_cosine_distance");
  if (!T || !D) return BX_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool pre = (flags & BX_NN_SAMPLES_NORMALIZED) != 0;
  // workspace: normalised samples (unless given so) and features, their denominators, the
  // row -> target map and the max keys
  const size_t b_sh = pre ? 0 : (size_t)G * F * 8, b_dh = (size_t)D * F * 8;
  const size_t b_den = (size_t)(G + D) * 8, b_tgt = (size_t)(G ? G : 1) * 4,
               b_key = (size_t)T * D * 8;
  char* ws = nullptr;
  NCHK(hipMallocAsync((void**)&ws, b_sh + b_dh + b_den + b_tgt + b_key + 1024, st));
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  double* sh = (double*)ws;
  double* dh = (double*)(ws + al(b_sh));
  double* den = (double*)(ws + al(b_sh) + al(b_dh));
  int* tgt = (int*)(ws + al(b_sh) + al(b_dh) + al(b_den));
  unsigned long long* keys = (unsigned long long*)(ws + al(b_sh) + al(b_dh) + al(b_den) + al(b_tgt));
  const double* S = samples;
  if (G && !pre) {
    hipLaunchKernelGGL(nn_norm_kernel, dim3((G + 255) / 256), dim3(256), 0, st, samples, G, F, den);
    hipLaunchKernelGGL(nn_scale_kernel, dim3(grid_for((size_t)G * F)), dim3(256), 0, st, samples,
                       den, (size_t)G * F, F, sh);
    S = sh;
  }
  hipLaunchKernelGGL(nn_norm_kernel, dim3((D + 255) / 256), dim3(256), 0, st, feats, D, F, den + G);
  hipLaunchKernelGGL(nn_scale_kernel, dim3(grid_for((size_t)D * F)), dim3(256), 0, st, feats,
                     den + G, (size_t)D * F, F, dh);
  NCHK(hipMemsetAsync(keys, 0, b_key, st));
  if (G) {
    hipLaunchKernelGGL(nn_row_target_kernel, dim3(T), dim3(256), 0, st, off, T, tgt);
    const size_t lds = sizeof(double) * 2 * LDS_STAGE;
    static bool attr = false;
    if (!attr) {
      NCHK(hipFuncSetAttribute((const void*)nn_cosine_mfma_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr = true;
    }
    const int nrb = (G + BM - 1) / BM, ncb = (D + BN - 1) / BN;
    hipLaunchKernelGGL(nn_cosine_mfma_kernel, dim3(nrb * ncb), dim3(NT), lds, st, S, G, dh, D, F,
                       tgt, keys);
  }
  hipLaunchKernelGGL(nn_finish_kernel, dim3(grid_for((size_t)T * D)), dim3(256), 0, st, keys, off,
                     T, D, out);
  NCHK(hipGetLastError());
  NCHK(hipFreeAsync(ws, st));
  return BX_OK;
}

}  // extern "C"
