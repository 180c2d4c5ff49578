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
hipError_t bx_lds_attr(const void* kern, size_t bytes);  // bx_engine.hip (never lowers a limit)

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- row normalisation (numpy's float64 pairwise sum of squares, PW_BLOCKSIZE 128) ----------
// Wave per row: the norm denominator sqrt(sum) + 1e-8 with numpy's pairwise tree.  The tree's
// leaves (<= 128 elements, found by the same halving numpy does) are summed by 8 lanes each —
// lane k keeps numpy's accumulator r[k] over elements k, k+8, ... — combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) by butterfly, the leaf tail added in order; lane 0 then
// folds the leaf sums in the tree's order.  Bitwise numpy's sequential pairwise_sum
// (restated in oracle/bxo_ops.c:pairwise_sum_f64).
constexpr int NN_MAX_LEAVES = 256;  // leaves hold > 56 elements: F <= 8192 needs < 147

__device__ int nn_leaves(int n, int* lo, int* ln) {
  int cnt = 0, stk_o[24], stk_n[24], top = 1;
  stk_o[0] = 0;
  stk_n[0] = n;
  while (top > 0) {  // pre-order, left first: leaves come out in element order
    const int o = stk_o[--top], m = stk_n[top];
    if (m <= 128) {
      lo[cnt] = o;
      ln[cnt] = m;
      cnt++;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    stk_o[top] = o + n2;  // right pushed first, popped last
    stk_n[top] = m - n2;
    top++;
    stk_o[top] = o;
    stk_n[top] = n2;
    top++;
  }
  return cnt;
}

// fold the leaf sums in the tree's combine order (post-order over the same halving)
__device__ double nn_fold_iter(int n, const double* leaf) {
  double acc[24];
  int ap = 0, li = 0, stk_n[24], stk_state[24], top = 1;
  stk_n[0] = n;
  stk_state[0] = 0;
  while (top > 0) {
    const int t = top - 1, m = stk_n[t];
    if (m <= 128) {
      acc[ap++] = leaf[li++];
      top--;
      continue;
    }
    int n2 = m / 2;
    n2 -= n2 % 8;
    if (stk_state[t] == 0) {
      stk_state[t] = 1;
      stk_n[top] = n2;
      stk_state[top] = 0;
      top++;
    } else if (stk_state[t] == 1) {
      stk_state[t] = 2;
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

__global__ void __launch_bounds__(256)
    nn_norm_kernel(const double* __restrict__ x, int n, int F, double* __restrict__ den) {
  __shared__ int lo[NN_MAX_LEAVES], ln[NN_MAX_LEAVES];
  __shared__ double leaf[4][NN_MAX_LEAVES];
  __shared__ int nleaf;
  if (threadIdx.x == 0) nleaf = nn_leaves(F, lo, ln);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  const bool live = row < n;  // no early exit: the block meets the barrier below
  const double* xr = x + (size_t)(live ? row : 0) * F;
  const int nl = nleaf;
  for (int base = 0; base < nl && live; base += 8) {
    const int li = base + (lane >> 3), k = lane & 7;
    double r = 0.0;
    int m = 0, o = 0;
    if (li < nl) {
      m = ln[li];
      o = lo[li];
      if (m >= 8) {
        const int full = m - (m % 8);
        const double v0 = xr[o + k];
        r = v0 * v0;
        for (int i = 8 + k; i < full; i += 8) {
          const double v = xr[o + i];
          r += v * v;
        }
      }
    }
    // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) within each group of 8 lanes
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (li < nl && k == 0) {
      double res;
      if (m < 8) {
        res = 0.0;
        for (int i = 0; i < m; i++) {
          const double v = xr[o + i];
          res += v * v;
        }
      } else {
        res = r;
        for (int i = m - (m % 8); i < m; i++) {
          const double v = xr[o + i];
          res += v * v;
        }
      }
      leaf[w][li] = res;
    }
  }
  __syncthreads();
  if (live && lane == 0) den[row] = sqrt(nn_fold_iter(F, leaf[w])) + 1e-8;
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
// Workgroup = WR x WC waves; wave (wr, wc) owns RT x CT tiles of 16 x 16 fp64 MFMA accumulators,
// i.e. a (16 RT) x (16 CT) block at rows 16 RT wr, detections 16 CT wc of the workgroup tile
// BM = 16 RT WR sample rows x BN = 16 CT WC detections.  K advances in chunks of 16 through
// double-buffered LDS images stored k-major ([k][row], [k][det]; 16-double padding puts the four
// k rows one MFMA operand reads on distinct bank halves).  Two shapes: 128 x 256 (8 waves, the
// full-gallery case) and 64 x 64 (4 waves) when the large tiles would not fill the CUs.
constexpr int KC = 16;

template <int RT, int CT, int WR, int WC>
struct NnTile {
  static constexpr int BM = 16 * RT * WR, BN = 16 * CT * WC, NT = 64 * WR * WC;
  static constexpr int LDA = BM + 16, LDB = BN + 16;
  static constexpr int STAGE = KC * (LDA + LDB);  // doubles per buffer
  static constexpr int APT = BM * KC / NT, BPT = BN * KC / NT;  // staged doubles per thread
  static_assert(APT >= 1 && BPT >= 1 && KC % APT == 0 && KC % BPT == 0, "staging split");
};

template <int RT, int CT, int WR, int WC>
__global__ void __launch_bounds__(64 * WR * WC)
    nn_cosine_mfma_kernel(const double* __restrict__ S, int G, const double* __restrict__ Dm,
                          int D, int F, const int* __restrict__ tgt,
                          unsigned long long* __restrict__ keys) {
  using P = NnTile<RT, CT, WR, WC>;
  extern __shared__ __align__(16) double lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w % WR, wc = w / WR;
  // column blocks fastest: a row block's samples stay hot in L2 while its column blocks run
  const int ncb = (D + P::BN - 1) / P::BN;
  const int row0 = (blockIdx.x / ncb) * P::BM, col0 = (blockIdx.x % ncb) * P::BN;

  constexpr int ATR = KC / P::APT, BTR = KC / P::BPT;  // threads per staged row
  const int ar = tid / ATR, aq = tid % ATR, bc = tid / BTR, bq_ = tid % BTR;
  const bool a_ok = row0 + ar < G, b_ok = col0 + bc < D;
  const double* ap = S + (size_t)(a_ok ? row0 + ar : 0) * F + P::APT * aq;
  const double* bp = Dm + (size_t)(b_ok ? col0 + bc : 0) * F + P::BPT * bq_;

  double ra[P::APT], rb[P::BPT];
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < P::APT; j++)
      ra[j] = (a_ok && k0 + P::APT * aq + j < F) ? ap[k0 + j] : 0.0;
#pragma unroll
    for (int j = 0; j < P::BPT; j++)
      rb[j] = (b_ok && k0 + P::BPT * bq_ + j < F) ? bp[k0 + j] : 0.0;
  };
  auto store = [&](double* buf) {
    double* As = buf;
    double* Bs = buf + KC * P::LDA;
#pragma unroll
    for (int j = 0; j < P::APT; j++) As[(P::APT * aq + j) * P::LDA + ar] = ra[j];
#pragma unroll
    for (int j = 0; j < P::BPT; j++) Bs[(P::BPT * bq_ + j) * P::LDB + bc] = rb[j];
  };

  d4 acc[RT][CT];
#pragma unroll
  for (int i = 0; i < RT; i++)
#pragma unroll
    for (int j = 0; j < CT; j++) acc[i][j] = (d4){0.0, 0.0, 0.0, 0.0};

  const int nk = (F + KC - 1) / KC;
  load(0);
  store(lds);
  __syncthreads();
  for (int kc = 0; kc < nk; kc++) {
    const double* cur = lds + (kc & 1) * P::STAGE;
    if (kc + 1 < nk) load((kc + 1) * KC);  // the next chunk's global loads overlap the MFMAs
    const double* As = cur;
    const double* Bs = cur + KC * P::LDA;
#pragma unroll
    for (int ks = 0; ks < KC / 4; ks++) {
      const int kr = ks * 4 + (lane >> 4);
      double a[RT], b[CT];
#pragma unroll
      for (int i = 0; i < RT; i++) a[i] = As[kr * P::LDA + (wr * RT + i) * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < CT; j++) b[j] = Bs[kr * P::LDB + (wc * CT + j) * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < RT; i++)
#pragma unroll
        for (int j = 0; j < CT; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kc + 1 < nk) store(lds + ((kc + 1) & 1) * P::STAGE);
    __syncthreads();
  }

  // epilogue: the lane holds column (lane & 15) of each tile at rows (lane >> 4) + 4 r, in
  // increasing order over (i, r); runs of one target are reduced before the atomic
#pragma unroll
  for (int j = 0; j < CT; j++) {
    const int col = col0 + (wc * CT + j) * 16 + (lane & 15);
    if (col >= D) continue;
    int cur_t = -1;
    double cur = 0.0;
#pragma unroll
    for (int i = 0; i < RT; i++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + (wr * RT + i) * 16 + (lane >> 4) + 4 * r;
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

using NnBig = NnTile<2, 8, 4, 2>;    // 128 x 256, 8 waves
using NnSmall = NnTile<2, 2, 2, 2>;  // 64 x 64, 4 waves

template <int RT, int CT, int WR, int WC>
int nn_launch(const double* S, int G, const double* Dm, int D, int F, const int* tgt,
              unsigned long long* keys, hipStream_t st) {
  using P = NnTile<RT, CT, WR, WC>;
  const size_t lds = sizeof(double) * 2 * P::STAGE;
  // (per device, never lowered: bx_lds_attr)
  if (bx_lds_attr((const void*)nn_cosine_mfma_kernel<RT, CT, WR, WC>, lds) != hipSuccess)
    return bx_record_error(BX_ERR_HIP, "hipFuncSetAttribute(nn_cosine_mfma_kernel)");
  const int nrb = (G + P::BM - 1) / P::BM, ncb = (D + P::BN - 1) / P::BN;
  hipLaunchKernelGGL((nn_cosine_mfma_kernel<RT, CT, WR, WC>), dim3(nrb * ncb), dim3(P::NT), lds,
                     st, S, G, Dm, D, F, tgt, keys);
  return BX_OK;
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
  if (T < 0 || D < 0 || F <= 0 || F > 8192 || G < 0 || (T && !off) || (T && D && (!out || !feats)) ||
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
    hipLaunchKernelGGL(nn_norm_kernel, dim3((G + 3) / 4), dim3(256), 0, st, samples, G, F, den);
    hipLaunchKernelGGL(nn_scale_kernel, dim3(grid_for((size_t)G * F)), dim3(256), 0, st, samples,
                       den, (size_t)G * F, F, sh);
    S = sh;
  }
  hipLaunchKernelGGL(nn_norm_kernel, dim3((D + 3) / 4), dim3(256), 0, st, feats, D, F, den + G);
  hipLaunchKernelGGL(nn_scale_kernel, dim3(grid_for((size_t)D * F)), dim3(256), 0, st, feats,
                     den + G, (size_t)D * F, F, dh);
  NCHK(hipMemsetAsync(keys, 0, b_key, st));
  if (G) {
    hipLaunchKernelGGL(nn_row_target_kernel, dim3(T), dim3(256), 0, st, off, T, tgt);
    // the 128 x 256 tile when its grid covers the CUs (one 8-wave workgroup each), else 64 x 64
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const long big = (long)((G + NnBig::BM - 1) / NnBig::BM) * ((D + NnBig::BN - 1) / NnBig::BN);
    const int rc = big >= cus ? nn_launch<2, 8, 4, 2>(S, G, dh, D, F, tgt, keys, st)
                              : nn_launch<2, 2, 2, 2>(S, G, dh, D, F, tgt, keys, st);
    if (rc) return rc;
  }
  hipLaunchKernelGGL(nn_finish_kernel, dim3(grid_for((size_t)T * D)), dim3(256), 0, st, keys, off,
                     T, D, out);
  NCHK(hipGetLastError());
  NCHK(hipFreeAsync(ws, st));
  return BX_OK;
}

}  // extern "C"
