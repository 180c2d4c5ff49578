// bx_jv.h — wave-cooperative building blocks shared by the one-wave-per-sequence trackers
// (OCSort, BoostTrack) and the op-level bx_lapjv: lapx's dense lapjv with lapx's own tie order
// (oracle/bxo_ops.c bxo_lapjv: _ccrrt_dense, up to two _carr_dense passes, _ca_dense), and a
// wave-order-preserving compaction.  Include inside a translation unit's anonymous namespace
// after bx_device.h (uses bx::INF); a workgroup is exactly one wave64.
#pragma once

constexpr int OW = 64;                    // threads per workgroup: one wave per sequence
constexpr double LAPX_LARGE = 1000000.0;  // lapx's LARGE sentinel (lapjv.h)
constexpr int JV_IMAX = 0x7fffffff;

// Wave-cooperative lapx lapjv on the zero-padded square max(nr, nc) of a row-major nr x nc
// matrix (legacy linear_assignment, association.py:105-114; boosttrack/assoc.py:106-114).
struct JvLds {
  double *v, *d;
  int *x, *y, *matches, *freer, *pred, *col;
  int* sc;  // >= 8 ints of broadcast scratch
  double* sd;
  unsigned long long* dc;  // diagnostic counters (timing builds) or null
};

// JvLds state of an n-column problem carved from `p` (LDS or global), jv_bytes(n) bytes.
__host__ __device__ constexpr size_t jv_ints_bytes(int n) { return (((size_t)n * 4 + 7) / 8) * 8; }
__host__ __device__ constexpr size_t jv_bytes(int n) {
  return 2 * 8 * (size_t)n + 16 + 6 * jv_ints_bytes(n) + 32;
}
__device__ inline JvLds jv_bind(unsigned char* p, int n) {
  JvLds w;
  size_t o = 0;
  auto takeD = [&](int k) { double* q = (double*)(p + o); o += (size_t)k * 8; return q; };
  auto takeI = [&](int k) { int* q = (int*)(p + o); o += jv_ints_bytes(k); return q; };
  w.v = takeD(n);
  w.d = takeD(n);
  w.sd = takeD(2);
  w.x = takeI(n);
  w.y = takeI(n);
  w.matches = takeI(n);
  w.freer = takeI(n);
  w.pred = takeI(n);
  w.col = takeI(n);
  w.sc = takeI(8);
  w.dc = nullptr;
  return w;
}

// The same state split over three buffers (the doubles v, d, sd in pd: 16 n + 16 bytes; x, y,
// matches, freer in pa: 4 jv_ints_bytes(n); pred, col, sc in pb: 2 jv_ints_bytes(n) + 32) — for
// a caller whose free LDS is not one contiguous block.
__host__ __device__ constexpr size_t jv_split_d_bytes(int n) { return 16 * (size_t)n + 16; }
__host__ __device__ constexpr size_t jv_split_a_bytes(int n) { return 4 * jv_ints_bytes(n); }
__host__ __device__ constexpr size_t jv_split_b_bytes(int n) { return 2 * jv_ints_bytes(n) + 32; }
__device__ inline JvLds jv_bind_split(unsigned char* pd, unsigned char* pa, unsigned char* pb,
                                      int n) {
  JvLds w;
  w.v = (double*)pd;
  w.d = w.v + n;
  w.sd = w.d + n;
  size_t o = 0;
  auto takeA = [&](int k) { int* q = (int*)(pa + o); o += jv_ints_bytes(k); return q; };
  w.x = takeA(n);
  w.y = takeA(n);
  w.matches = takeA(n);
  w.freer = takeA(n);
  w.pred = (int*)pb;
  w.col = (int*)(pb + jv_ints_bytes(n));
  w.sc = (int*)(pb + 2 * jv_ints_bytes(n));
  w.dc = nullptr;
  return w;
}

__device__ __forceinline__ double cget(const double* C, int nr, int nc, int i, int j) {
  return (i < nr && j < nc) ? C[i * nc + j] : 0.0;
}

__device__ __forceinline__ int rl_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ double rl_d(double v, int k) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_i(int src, int old) {
  return __builtin_amdgcn_update_dpp(old, src, CTRL, RM, BM, false);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_d(double src, double old) {
  const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffll), (int)(s & 0xffffffffll),
                                             CTRL, RM, BM, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), CTRL, RM, BM, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double scan_min_d(double r) {  // no NaNs
  r = fmin(r, dpp_d<0x111, 0xf, 0xf>(r, INF));
  r = fmin(r, dpp_d<0x112, 0xf, 0xf>(r, INF));
  r = fmin(r, dpp_d<0x114, 0xf, 0xf>(r, INF));
  r = fmin(r, dpp_d<0x118, 0xf, 0xf>(r, INF));
  r = fmin(r, dpp_d<0x142, 0xa, 0xf>(r, INF));
  r = fmin(r, dpp_d<0x143, 0xc, 0xf>(r, INF));
  return r;
}
__device__ __forceinline__ int scan_min_i(int r) {
  constexpr int BIG = 0x7fffffff;
  r = min(r, dpp_i<0x111, 0xf, 0xf>(r, BIG));
  r = min(r, dpp_i<0x112, 0xf, 0xf>(r, BIG));
  r = min(r, dpp_i<0x114, 0xf, 0xf>(r, BIG));
  r = min(r, dpp_i<0x118, 0xf, 0xf>(r, BIG));
  r = min(r, dpp_i<0x142, 0xa, 0xf>(r, BIG));
  r = min(r, dpp_i<0x143, 0xc, 0xf>(r, BIG));
  return r;
}
__device__ __forceinline__ int wave_min_i(int a) { return __builtin_amdgcn_readlane(scan_min_i(a), 63); }
__device__ __forceinline__ int first_lane(bool p) {
  const unsigned long long m = __ballot(p);
  return m ? __ffsll((long long)m) - 1 : -1;
}
__device__ __forceinline__ int last_lane(bool p) {
  const unsigned long long m = __ballot(p);
  return m ? 63 - __clzll((long long)m) : -1;
}
// send each lane's value to lane `dst` (a permutation)
__device__ __forceinline__ int perm_i(int v, int dst) {
  return __builtin_amdgcn_ds_permute(dst << 2, v);
}
__device__ __forceinline__ double perm_d(double v, int dst) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_permute(dst << 2, (int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_ds_permute(dst << 2, (int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// (compare-select steps instead of fmin measured slower: C5 22.4 vs 23.0 k frames/s)
__device__ __forceinline__ double wave_min_dpp(double a) {  // no NaNs (fmin drops them anyway)
  return rl_d(scan_min_d(a), 63);
}
// the wave minimum in every lane (DPP row shifts and a readlane, no LDS permutes); NaNs dropped
// as fmin drops them (no caller feeds one: their running minima start from INF / LARGE)
__device__ __forceinline__ double wave_min_d(double a) { return wave_min_dpp(a); }

// (value, index) argmin across the wave: the smallest value, the smallest index among equal
// values — what a sequential ascending `<` scan keeps.  No NaNs.
__device__ __forceinline__ void wave_argmin(double& m, int& j) {
  for (int o = 32; o >= 1; o >>= 1) {
    const double om = __shfl_xor(m, o);
    const int oj = __shfl_xor(j, o);
    if (om < m || (om == m && oj < j)) {
      m = om;
      j = oj;
    }
  }
}

// Cross-lane hand-off points of the wave solvers: the whole (one-wave) workgroup, or only the
// calling wave of a larger one with its state in global memory (workgroup-scope fence: the
// stores are complete and visible to the wave's later loads through the CU's L1).
// after_atomics(): global atomics are performed in L2 and need not update a line the CU's L1
// still holds, so a global-state solver invalidates L1 (agent-scope fence) before reading what
// its atomics wrote; plain stores and loads of one wave meet in the same L1.
struct SyncBlock {
  __device__ void operator()() const { __syncthreads(); }
  __device__ void after_atomics() const {}
};
// Only the calling wave of a larger workgroup, its state in LDS (LDS atomics are performed in
// the LDS itself: the workgroup-scope fence, i.e. the wait for the wave's LDS operations, is all).
struct SyncWaveL {
  __device__ void operator()() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  __device__ void after_atomics() const { (*this)(); }
};
// SyncWaveL or SyncWaveG chosen at run time (one instantiation of the solver for both homes of
// its state: the engine's rare tie path must not add a second inlined copy to its kernel)
struct SyncWaveLG {
  bool global;
  __device__ void operator()() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  __device__ void after_atomics() const {
    if (global) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
  }
};
struct SyncWaveG {
  __device__ void operator()() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  }
  __device__ void after_atomics() const {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
  }
};

// Wave-order-preserving compaction: emit(k, pos) for k < n with pred(k); returns the count.
template <class P, class E, class SY>
__device__ __forceinline__ int wave_compact_s(int n, P pred, E emit, SY sync) {
  const int lane = threadIdx.x & 63;
  int base = 0;
  for (int c = 0; c < n; c += OW) {
    const int k = c + lane;
    const bool f = k < n && pred(k);
    const unsigned long long m = __ballot(f);
    if (f) emit(k, base + __popcll(m & ((1ull << lane) - 1ull)));
    base += __popcll(m);
  }
  sync();
  return base;
}
template <class P, class E>
__device__ int wave_compact(int n, P pred, E emit) {
  return wave_compact_s(n, pred, emit, SyncBlock{});
}

// 64-position chunks of one scan's relaxation loaded together (two: a scan's TODO range is
// usually one or two chunks, and the unrolled group is issued whole — 8 measured 25 % slower on
// the crowd solve, profiles/r06/tie_path_r06.txt), and the find's register copy of at most
// JV_FR chunks
#ifndef BX_JV_CH
#define BX_JV_CH 2
#endif
constexpr int JV_CH = BX_JV_CH;
constexpr int JV_FR = 8;

// a value every lane holds alike (an LDS word all lanes read), made wave-uniform for the compiler
// (scalar registers: branches on it are scalar, not exec-mask juggling)
__device__ __forceinline__ int ufl_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double ufl_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// BX_JV_CLOCK (diagnostic builds only, tools/dbg/jv_clock.hip): wall-clock ticks per phase of
// jv_wave_t added to w.dc[8..15] by lane 0 (8 ccrrt, 9 carr, 10 find, 11 scan, 12 augment,
// 13 scan steps, 14 scans of a row below w.dc[7] (the caller stores R there), 15 skipped scans)
#ifdef BX_JV_CLOCK
#define JV_T0(t) unsigned long long t = wall_clock64()
#define JV_ACC(q, t) do { if (lane == 0 && w.dc) w.dc[q] += wall_clock64() - t; } while (0)
#define JV_CNT(q, k) do { if (lane == 0 && w.dc) w.dc[q] += (k); } while (0)
#else
#define JV_T0(t) do {} while (0)
#define JV_ACC(q, t) do {} while (0)
#define JV_CNT(q, k) do {} while (0)
#endif

// lapx's cost_limit extension of a row-major nr x nc cost (matching.py:54-61): the real block,
// limit / 2 off the diagonal blocks, 0 in the dummy block — read with the row index uniform (a
// scalar branch) and the column clamped into the row, so a chunk's lanes load without masking.
struct JvExt {
  const double* M;
  int nr, nc;
  double half;
  __device__ __forceinline__ double operator()(int i, int j) const {
    if (i < nr) {
      const double c = M[(size_t)i * nc + min(max(j, 0), nc - 1)];
      return j < nc ? c : half;
    }
    return j < nc ? half : 0.0;
  }
};

// Row classes for the scan skip of jv_wave_t: rk(i) = 0 or 1 when row i belongs to that class of
// rows with IDENTICAL finite cost rows (the cost_limit extension's dummy rows; real rows whose
// every real cost equals one constant), -1 otherwise.
struct JvNoClass {
  __device__ int operator()(int) const { return -1; }
};

// ------------------------------------------------------------------------------------------
// Any n, state in `w` (LDS, or global memory with a SyncWaveG); the cost of (i, j) from cf(i, j)
// and every cross-lane hand-off through sync() (the whole workgroup when it is one wave, else
// the calling wave only).
//
// Scan skip (exact): within one shortest-path search v is fixed, d only falls and the TODO set
// only shrinks, so after a row of class c was scanned with h = c(i, j1) - v[j1] - mind every
// TODO column has d[j] <= c(i, j) - v[j] - h.  A later scan of a row i' of the same class (the
// same cost row) with h' <= h computes c(i, j) - v[j] - h' >= d[j] everywhere: no update, no
// swap, no end of path — it is skipped.  (lapx scans it to no effect.)  Only finite h count.
template <class CF, class SY, class RK = JvNoClass>
__device__ __forceinline__ void jv_wave_t(const CF& cf, int n, JvLds& w, SY sync,
                                          const RK& rk = RK{}) {
  const int lane = threadIdx.x & 63;
  JV_T0(tc0);
  // ---- _ccrrt_dense.  Column minima from LARGE, first row on ties (lane per column) ...
  for (int j = lane; j < n; j += OW) {
    double mn = LAPX_LARGE;
    int im = 0;
#pragma unroll 8
    for (int i = 0; i < n; i++) {
      const double c = cf(i, j);
      if (c < mn) mn = c, im = i;
    }
    w.v[j] = mn;
    w.y[j] = im;
    w.x[j] = -1;
    w.matches[j] = 0;
  }
  sync();
  // ... the sweep j = n-1..0 leaves each row the LARGEST column whose minimum it holds and
  // releases the others; `matches` counts them (lapx's unique[] is a count of one)
  for (int j = lane; j < n; j += OW) {
    atomicMax(&w.x[w.y[j]], j);
    atomicAdd(&w.matches[w.y[j]], 1);
  }
  sync();
  sync.after_atomics();
  for (int j = lane; j < n; j += OW)
    if (w.x[w.y[j]] != j) w.y[j] = -1;
  int nfree = wave_compact_s(
      n, [&](int i) { return w.x[i] < 0; }, [&](int i, int p) { w.freer[p] = i; }, sync);
  // reduction transfer, uniquely-assigned rows in order (each lowers v[x[i]], which the rows
  // after it read)
  for (int i = 0; i < n; i++) {
    const int j1 = ufl_i(w.x[i]);
    if (j1 < 0 || ufl_i(w.matches[i]) != 1) continue;
    double mn = LAPX_LARGE;
#pragma unroll 4
    for (int j = lane; j < n; j += OW) {
      const double h = cf(i, j) - w.v[j];
      if (j != j1 && h < mn) mn = h;
    }
    mn = wave_min_d(mn);
    sync();
    if (lane == 0) w.v[j1] = w.v[j1] - mn;
    sync();
  }
  JV_ACC(8, tc0);
  JV_T0(tc1);
  // ---- _carr_dense, at most two passes over the free rows (lapjv_internal)
  for (int pass = 0; pass < 2 && nfree > 0; pass++) {
    unsigned current = 0, rr_cnt = 0;
    int nnew = 0;
    while (current < (unsigned)nfree) {
      rr_cnt++;
      const int fi = ufl_i(w.freer[current++]);
      // the cheapest column j1 (first on ties) and the cheapest other one j2 (first on ties):
      // exactly lapx's running pair whenever every reduced cost is below LARGE
      // (one pass: each lane's two smallest (value, index) pairs, merged over the wave)
      double m1 = INF, m2 = INF;
      int k1 = JV_IMAX, k2 = JV_IMAX;
      bool odd = false;
#pragma unroll 4
      for (int j = lane; j < n; j += OW) {
        const double h = cf(fi, j) - w.v[j];
        odd |= !(h < LAPX_LARGE);
        if (h < m1) {
          m2 = m1, k2 = k1;
          m1 = h, k1 = j;
        } else if (h < m2) {
          m2 = h, k2 = j;
        }
      }
      int j1, j2;
      double v1, v2;
      if (!__any(odd)) {
        auto lt = [](double a, int ia, double b, int ib) { return a < b || (a == b && ia < ib); };
        for (int o = 32; o >= 1; o >>= 1) {
          const double b1 = __shfl_xor(m1, o), b2 = __shfl_xor(m2, o);
          const int c1 = __shfl_xor(k1, o), c2 = __shfl_xor(k2, o);
          if (lt(b1, c1, m1, k1)) {  // partner's first leads: second = min(own first, its second)
            if (lt(m1, k1, b2, c2)) m2 = m1, k2 = k1;
            else m2 = b2, k2 = c2;
            m1 = b1, k1 = c1;
          } else if (lt(b1, c1, m2, k2)) {
            m2 = b1, k2 = c1;
          }
        }
        j1 = ufl_i(k1);
        v1 = ufl_d(cf(fi, j1) - w.v[j1]);
        if (n >= 2) {
          j2 = ufl_i(k2);
          v2 = ufl_d(cf(fi, j2) - w.v[j2]);
        } else {
          j2 = -1;
          v2 = LAPX_LARGE;
        }
      } else {  // NaN or huge reduced costs: lapx's scan as written
        j1 = 0;
        j2 = -1;
        v1 = cf(fi, 0) - w.v[0];
        v2 = LAPX_LARGE;
        for (int j = 1; j < n; j++) {
          const double h = cf(fi, j) - w.v[j];
          if (h < v2) {
            if (h >= v1) {
              v2 = h;
              j2 = j;
            } else {
              v2 = v1;
              v1 = h;
              j2 = j1;
              j1 = j;
            }
          }
        }
      }
      int i0 = ufl_i(w.y[j1]);
      const double vj1 = ufl_d(w.v[j1]);
      const double v1_new = vj1 - (v2 - v1);
      const bool lowers = v1_new < vj1;
      if (rr_cnt < current * (unsigned)n) {
        if (lowers) {
          if (lane == 0) w.v[j1] = v1_new;
        } else if (i0 >= 0 && j2 >= 0) {
          j1 = j2;
          i0 = ufl_i(w.y[j2]);
        }
        if (i0 >= 0) {
          if (lowers) {
            --current;
            if (lane == 0) w.freer[current] = i0;
          } else {
            if (lane == 0) w.freer[nnew] = i0;
            nnew++;
          }
        }
      } else if (i0 >= 0) {
        if (lane == 0) w.freer[nnew] = i0;
        nnew++;
      }
      sync();
      if (lane == 0) {
        w.x[fi] = j1;
        w.y[j1] = fi;
      }
      sync();
    }
    nfree = nnew;
  }
#ifdef BX_PHASE_TIMING
  if (lane == 0 && w.dc) w.dc[0] += nfree;
#endif
  JV_ACC(9, tc1);
  // ---- _ca_dense: one shortest augmenting path per remaining free row
  for (int f = 0; f < nfree; f++) {
    const int start = ufl_i(w.freer[f]);
#pragma unroll 4
    for (int j = lane; j < n; j += OW) {
      w.d[j] = cf(start, j) - w.v[j];
      w.pred[j] = start;
      w.col[j] = j;
    }
    sync();
    int low = 0, up = 0, last = 0, endofpath = -1, found = 0;
    double mn = 0.0;
    double hmax0 = -INF, hmax1 = -INF;  // the largest finite h scanned per row class
    do {
#ifdef BX_PHASE_TIMING
      if (lane == 0 && w.dc) w.dc[up == low ? 1 : 2] += 1;
#endif
      if (up == low) {
        JV_T0(tf);
        // _find_dense.  It gathers, in position order, every TODO column at the minimum into
        // col[low..up) and the path ends at the LAST unassigned one.  When one exists the search
        // ends here and the rest of the permutation is never read again (col is rebuilt for the
        // next free row), so the lane-parallel path finds it directly; otherwise (or with NaN
        // distances) the scan runs as written — over a register copy of the positions when at
        // most JV_FR * 64 remain, else over LDS on lane 0.
        if (n - low <= JV_FR * OW) {
          int cq[JV_FR];
          double dq[JV_FR];
          double m = INF;
          bool bad = false;
#pragma unroll
          for (int q = 0; q < JV_FR; q++) {
            const int k = low + q * OW + lane;
            cq[q] = -1;
            dq[q] = INF;
            if (k < n) {
              cq[q] = w.col[k];
              dq[q] = w.d[cq[q]];
              m = fmin(m, dq[q]);
              bad |= isnan(dq[q]);
            }
          }
          m = wave_min_d(m);
          bad = __any(bad) || !(m < INF);
          int kg = -1, ke = -1;
          if (!bad) {
#pragma unroll
            for (int q = 0; q < JV_FR; q++) {
              const int base = low + q * OW;
              if (base >= n) break;
              const bool G = base + lane < n && dq[q] == m;
              const bool E = G && w.y[cq[q]] < 0;
              const unsigned long long gm = __ballot(G), em = __ballot(E);
              if (kg < 0 && gm) kg = base + __ffsll((long long)gm) - 1;
              if (em) ke = base + 63 - __clzll((long long)em);
            }
          }
#ifdef BX_PHASE_TIMING
          if (lane == 0 && w.dc && ke < 0) w.dc[3] += 1;
#endif
          if (ke >= 0) {
            last = low - 1;
            mn = m;  // d[cols[lo]] after the scan: the first column at the minimum
            endofpath = w.col[ke];
            found = 1;
          } else {
            // lapx's sequential loop, every lane in step: position k's own entry is read before
            // any swap writes it (a swap writes positions <= k), so the registers hold what the
            // loop reads there; col[up] is read back from LDS (lane 0 swaps in place).  Only
            // positions at or below the running minimum when their chunk starts can act (the
            // minimum only falls), so each chunk visits its ballot's lanes.
            last = low - 1;
            double mnv = rl_d(dq[0], 0);
            int upl = low + 1;
#pragma unroll
            for (int q = 0; q < JV_FR; q++) {
              const int base = low + q * OW;
              if (base >= n) break;
              unsigned long long cm = __ballot(base + lane < n && dq[q] <= mnv);
              if (q == 0) cm &= ~1ull;
              while (cm) {
                const int t = __ffsll((long long)cm) - 1;
                cm &= cm - 1;
                const double h = rl_d(dq[q], t);
                if (h <= mnv) {
                  if (h < mnv) {
                    upl = low;
                    mnv = h;
                  }
                  const int j = rl_i(cq[q], t);
                  if (lane == 0) {
                    w.col[base + t] = w.col[upl];
                    w.col[upl] = j;
                  }
                  upl++;
                }
              }
            }
            sync();
            for (int base = low; base < upl; base += OW) {
              const int k = base + lane;
              int j = -1;
              bool E = false;
              if (k < upl) {
                j = w.col[k];
                E = w.y[j] < 0;
              }
              const unsigned long long em = __ballot(E);
              if (em) {
                endofpath = __shfl(j, 63 - __clzll((long long)em));
                found = 1;
              }
            }
            up = upl;
            mn = mnv;
          }
        } else {
          double m = INF;
          bool bad = false;
          for (int k = low + lane; k < n; k += OW) {
            const double h = w.d[w.col[k]];
            m = fmin(m, h);
            bad |= isnan(h);
          }
          m = wave_min_d(m);
          bad = __any(bad) || !(m < INF);
          int kg = -1, ke = -1;
          if (!bad) {
            for (int base = low; base < n; base += OW) {
              const int k = base + lane;
              bool G = false, E = false;
              if (k < n) {
                const int j = w.col[k];
                G = w.d[j] == m;
                E = G && w.y[j] < 0;
              }
              const unsigned long long gm = __ballot(G), em = __ballot(E);
              if (kg < 0 && gm) kg = base + __ffsll((long long)gm) - 1;
              if (em) ke = base + 63 - __clzll((long long)em);
            }
          }
#ifdef BX_PHASE_TIMING
          if (lane == 0 && w.dc && ke < 0) w.dc[3] += 1;
#endif
          if (ke >= 0) {
            last = low - 1;
            mn = w.d[w.col[kg]];
            endofpath = w.col[ke];
            found = 1;
          } else {
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
                }
              w.sc[0] = last;
              w.sc[1] = up;
              w.sc[2] = endofpath;
              w.sc[3] = found;
              w.sd[0] = mn;
            }
            sync();
            last = w.sc[0];
            up = w.sc[1];
            endofpath = w.sc[2];
            found = w.sc[3];
            mn = w.sd[0];
            sync();
          }
        }
        JV_ACC(10, tf);
      }
      if (!found) {
        // batch skip: the SCAN positions from low on whose scans the skip rule below passes over
        // (with the class maxima as they stand — a skipped scan changes nothing, so they stand up
        // to the first position that is scanned) are passed over 64 at a time — entered only
        // when position low itself skips (a scanned row pays one test, not a batch)
        bool skip0 = false;
        {
          const int j = ufl_i(w.col[low]);
          const int ii = ufl_i(w.y[j]);
          const int c = rk(ii);
          if (c >= 0) {
            const double hh = cf(ii, j) - w.v[j] - w.d[j];
            skip0 = isfinite(hh) && hh <= (c == 0 ? hmax0 : hmax1);
          }
        }
        while (skip0 && low < up) {
          const int p = low + lane;
          bool sk = false;
          if (p < up) {
            const int j = w.col[p];
            const int ii = w.y[j];
            const int c = rk(ii);
            if (c >= 0) {
              const double hh = cf(ii, j) - w.v[j] - w.d[j];
              sk = isfinite(hh) && hh <= (c == 0 ? hmax0 : hmax1);
            }
          }
          const unsigned long long ns = __ballot(p < up && !sk);
          const int adv = ns ? __ffsll((long long)ns) - 1 : min(OW, up - low);
          JV_CNT(15, adv);
          low += adv;
          if (ns) break;
        }
        if (low < up) {
        // _scan_dense from SCAN column j1 = col[low]: relax the TODO columns col[up..n) in
        // chunks of 64 positions; the first column lowered to the minimum that is unassigned
        // ends the path.  Every operand of every chunk is loaded up front: a swap writes only
        // positions up to the chunk in flight, and each column appears once, so later chunks
        // read what the sequential loop would.
        JV_T0(ts);
        const int j1 = ufl_i(w.col[low++]);
        const int i = ufl_i(w.y[j1]);
        JV_CNT(13, 1);
        JV_CNT(14, i < (int)w.dc[7] ? 1 : 0);
        const double mind = ufl_d(w.d[j1]);
        const double h = cf(i, j1) - w.v[j1] - mind;
        const int cls = rk(i);
        bool skip = false;
        if (cls >= 0 && isfinite(h)) {
          double& hm = cls == 0 ? hmax0 : hmax1;
          skip = h <= hm;
          if (!skip) hm = h;
        }
        JV_CNT(15, skip ? 1 : 0);
        // groups of JV_CH chunks (a swap only writes positions up to the chunk in flight, so a
        // later group's operands are still the sequential loop's)
        for (int g0 = up; g0 < n && !found && !skip; g0 += JV_CH * OW) {
          int jc[JV_CH];
          double v2c[JV_CH], dc[JV_CH];
          bool yc[JV_CH];
#pragma unroll
          for (int c = 0; c < JV_CH; c++) {
            const int k = g0 + c * OW + lane;
            jc[c] = -1;
            if (k < n) {
              const int j = w.col[k];
              jc[c] = j;
              v2c[c] = cf(i, j) - w.v[j] - h;
              dc[c] = w.d[j];
              yc[c] = w.y[j] < 0;
            }
          }
#pragma unroll
          for (int c = 0; c < JV_CH; c++) {
            const int base = g0 + c * OW;
            if (base >= n || found) break;
            const int j = jc[c];
            const double v2 = v2c[c];
            bool A = false, B = false, E = false;
            if (j >= 0) {
              A = v2 < dc[c];
              B = A && v2 == mind;
              E = B && yc[c];
            }
            const unsigned long long em = __ballot(E);
            int kE = OW;
            if (em) kE = __ffsll((long long)em) - 1;
            if (A && lane <= kE) {
              w.pred[j] = i;
              w.d[j] = v2;
            }
            unsigned long long hm = __ballot(B && !E && lane < kE);
            if (hm) {
              while (hm) {  // the swaps, in position order (lane 0 owns col)
                const int bb = __ffsll((long long)hm) - 1;
                hm &= hm - 1;
                const int jb = __shfl(j, bb);
                if (lane == 0) {
                  w.col[base + bb] = w.col[up];
                  w.col[up] = jb;
                }
                up++;
              }
            }
            if (em) {
              endofpath = __shfl(j, kE);
              found = 1;
            }
          }
        }
        sync();
        JV_ACC(11, ts);
        }
      }
    } while (!found);
    JV_T0(ta);
    for (int k = lane; k <= last; k += OW) {
      const int j1 = w.col[k];
      w.v[j1] = w.v[j1] + (w.d[j1] - mn);  // lapx: v[j] += d[j] - mind
    }
    sync();
    if (lane == 0) {
      int i;
      do {
        i = w.pred[endofpath];
        w.y[endofpath] = i;
        const int j1 = endofpath;
        endofpath = w.x[i];
        w.x[i] = j1;
      } while (i != start);
    }
    sync();
    JV_ACC(12, ta);
  }
}

// sync: SyncBlock when `w` is in LDS (or the workgroup is this one wave and the state is in
// LDS); SyncWaveG when the state is in global memory (its atomics' results are read back
// through an invalidated L1)
template <class SY = SyncBlock>
__device__ void jv_wave(const double* C, int nr, int nc, JvLds& w, SY sync = SY{}) {
  jv_wave_t([&](int i, int j) { return cget(C, nr, nc, i, j); }, nr > nc ? nr : nc, w, sync);
}

// ------------------------------------------------------------------------------------------
// The same lapjv for n <= 64, register-resident.  Setup (_ccrrt_dense, _carr_dense): lane j owns
// column j (v, y) and row j (x, the free-row list entry j).  Augmentation: lane k holds the
// column at POSITION k of lapx's `cols` permutation with its v, d, y and pred, so
// position-ordered choices (the first / last column at the minimum, the first unassigned one the
// scan lowers) are single ballots and the swaps cols[k] <-> cols[hi] exchange two lanes'
// registers (readlane); rows keep x in lane i.  Every comparison, arithmetic operation and tie
// is lapx's.
// DPP inclusive min-scan across the wave (row_shr 1/2/4/8 within rows of 16, then row_bcast 15
// and 31 — the gfx9 wave64 scan sequence); lanes whose source is outside the row keep the
// identity.  Lane 63 holds the wave minimum.
// at least three bits set (scalar ops only: a popcount compare became a VALU 64-bit compare)
__device__ __forceinline__ bool ge3(unsigned long long m) {
  const unsigned long long a = m & (m - 1);
  return (a & (a - 1)) != 0;
}
// The wave minimum in every lane, returned uniform: a butterfly — row rotations by 8/4/2/1 within
// rows of 16 (every lane stays valid, no identity to preload), then gfx950's row-pair and half
// swaps.  fmin ignores NaNs (an all-NaN wave gives NaN).
__device__ __forceinline__ double swap_min(double r, bool half) {
  const long long b = __double_as_longlong(r);
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
  const double x = __longlong_as_double(((long long)h0 << 32) | a0);
  const double y = __longlong_as_double(((long long)h1 << 32) | a1);
  return fmin(x, y);
}
// a row rotation of an fp64 within rows of 16: every lane's source is valid, so no old value is
// needed (mov_dpp: the compiler does not copy the destination first)
template <int CTRL>
__device__ __forceinline__ double ror_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_min_bfly(double r) {
  r = fmin(r, ror_d<0x128>(r));
  r = fmin(r, ror_d<0x124>(r));
  r = fmin(r, ror_d<0x122>(r));
  r = fmin(r, ror_d<0x121>(r));
  r = swap_min(r, false);
  r = swap_min(r, true);
  return rl_d(r, 0);
}
// two independent wave minima, level by level (the two chains interleave)
__device__ __forceinline__ void wave_min_bfly2(double& a, double& b) {
  a = fmin(a, ror_d<0x128>(a));
  b = fmin(b, ror_d<0x128>(b));
  a = fmin(a, ror_d<0x124>(a));
  b = fmin(b, ror_d<0x124>(b));
  a = fmin(a, ror_d<0x122>(a));
  b = fmin(b, ror_d<0x122>(b));
  a = fmin(a, ror_d<0x121>(a));
  b = fmin(b, ror_d<0x121>(b));
  a = swap_min(a, false);
  b = swap_min(b, false);
  a = swap_min(a, true);
  b = swap_min(b, true);
  a = rl_d(a, 0);
  b = rl_d(b, 0);
}

// Cost loads of the register-resident solver from address space AS (0: generic, 1: global,
// 3: LDS — a generic pointer into LDS would be read by flat loads, which wait on both counters).
template <int AS>
__device__ __forceinline__ double cget_as(const double* C, int nr, int nc, int i, int j) {
  if (!(i < nr && j < nc)) return 0.0;
  if constexpr (AS == 3)
    return ((const __attribute__((address_space(3))) double*)C)[i * nc + j];
  else if constexpr (AS == 1)
    return ((const __attribute__((address_space(1))) double*)C)[i * nc + j];
  else
    return C[i * nc + j];
}

template <class SY = SyncBlock, int AS = 0>
__device__ void jv_wave64(const double* C, int nr, int nc, JvLds& w, SY sync = SY{}) {
  const int n = nr > nc ? nr : nc;
  const int lane = threadIdx.x & 63;
  auto cget = [&](const double*, int, int, int i, int j) { return cget_as<AS>(C, nr, nc, i, j); };
  // row i (wave-uniform) at this lane's column j: a scalar branch on the row (rows past nr are
  // zero) and a clamped, unconditional load for the column (no exec-masked region)
  auto crow_at = [&](int i, int j) -> double {
    double c = 0.0;
    if (i < nr && nc > 0) {
      const double t = cget_as<AS>(C, nr, nc, i, j < nc ? j : nc - 1);
      c = j < nc ? t : 0.0;
    }
    return c;
  };
  const bool own = lane < n;
#ifdef BX_PHASE_TIMING
  // cycles per slot and event counters kept in registers, added to w.dc once at the end (a
  // global read-modify-write per step would put its latency into the next wait it meets)
  unsigned long long jt0 = __builtin_amdgcn_s_memtime(), jt1 = 0, jacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long jcnt[16] = {0};
#define JCNT(k, v) (jcnt[k] += (unsigned long long)(v))
#define JVT(slot)                                                             \
  do {                                                                        \
    jt1 = __builtin_amdgcn_s_memtime();                                       \
    jacc[slot] += jt1 - jt0;                                                  \
    jt0 = jt1;                                                                \
  } while (0)
#else
#define JVT(slot) \
  do {            \
  } while (0)
#define JCNT(k, v) ((void)0)
#endif
  // ---- _ccrrt_dense.  Column minima from LARGE (first row on ties) ...
  double v = LAPX_LARGE, d = 0.0;
  int y = 0, pred = 0, col = lane, xr = -1;
  if (own) {
    for (int i = 0; i < n; i++) {
      const double c = cget(C, nr, nc, i, lane);
      if (c < v) v = c, y = i;
    }
    w.x[lane] = -1;
    w.matches[lane] = 0;
  }
  sync();
  // ... each row keeps the largest column whose minimum it holds (the j = n-1..0 sweep's first)
  if (own) {
    atomicMax(&w.x[y], lane);
    atomicAdd(&w.matches[y], 1);
  }
  sync();
  sync.after_atomics();
  bool uniq = false;
  if (own) {
    xr = w.x[lane];
    uniq = w.matches[lane] == 1;
    if (w.x[y] != lane) y = -1;
  }
  // reduction transfer, uniquely-assigned rows in order
  {
    unsigned long long rt = __ballot(own && xr >= 0 && uniq);
    while (rt) {
      const int i = __ffsll((long long)rt) - 1;
      rt &= rt - 1;
      const int j1 = rl_i(xr, i);
      double h = LAPX_LARGE;
      if (own && lane != j1) {
        const double t = cget(C, nr, nc, i, lane) - v;
        if (t < h) h = t;
      }
      h = wave_min_dpp(h);
      if (lane == j1) v = v - h;
    }
  }
  // free rows in row order: lane k holds the k-th
  int fr = -1, nfree;
  {
    const unsigned long long fm = __ballot(own && xr < 0);
    nfree = __popcll(fm);
    if (own && xr < 0) w.freer[__popcll(fm & ((1ull << lane) - 1ull))] = lane;
    sync();
    if (lane < nfree) fr = w.freer[lane];
  }
  // ---- _carr_dense, at most two passes
  for (int pass = 0; pass < 2 && nfree > 0; pass++) {
    unsigned current = 0, rr_cnt = 0;
    int nnew = 0;
    while (current < (unsigned)nfree) {
      rr_cnt++;
      const int fi = rl_i(fr, (int)current);
      current++;
      const double h = own ? crow_at(fi, lane) - v : INF;
      int j1, j2;
      double v1, v2;
      if (!__any(own && !(h < LAPX_LARGE))) {
        const double m1 = wave_min_dpp(own ? h : INF);
        j1 = first_lane(own && h == m1);
        v1 = rl_d(h, j1);
        if (n >= 2) {
          const bool o2 = own && lane != j1;
          const double m2 = wave_min_dpp(o2 ? h : INF);
          j2 = first_lane(o2 && h == m2);
          v2 = rl_d(h, j2);
        } else {
          j2 = -1;
          v2 = LAPX_LARGE;
        }
      } else {  // NaN or huge reduced costs: lapx's scan as written
        j1 = 0;
        j2 = -1;
        v1 = rl_d(h, 0);
        v2 = LAPX_LARGE;
        for (int j = 1; j < n; j++) {
          const double t = rl_d(h, j);
          if (t < v2) {
            if (t >= v1) {
              v2 = t;
              j2 = j;
            } else {
              v2 = v1;
              v1 = t;
              j2 = j1;
              j1 = j;
            }
          }
        }
      }
      int i0 = rl_i(y, j1);
      const double vj1 = rl_d(v, j1);
      const double v1_new = vj1 - (v2 - v1);
      const bool lowers = v1_new < vj1;
      if (rr_cnt < current * (unsigned)n) {
        if (lowers) {
          if (lane == j1) v = v1_new;
        } else if (i0 >= 0 && j2 >= 0) {
          j1 = j2;
          i0 = rl_i(y, j2);
        }
        if (i0 >= 0) {
          if (lowers) {
            --current;
            if (lane == (int)current) fr = i0;
          } else {
            if (lane == nnew) fr = i0;
            nnew++;
          }
        }
      } else if (i0 >= 0) {
        if (lane == nnew) fr = i0;
        nnew++;
      }
      if (lane == fi) xr = j1;
      if (lane == j1) y = fi;
    }
    JCNT(11, rr_cnt);
    nfree = nnew;
  }
  JCNT(0, nfree);
  JVT(4);
  // exchange the registers of positions a and b (cols[a] <-> cols[b])
  auto swap_pos = [&](int a, int b) {
    if (a == b) return;
    const int ca = rl_i(col, a), cb = rl_i(col, b);
    const int ya = rl_i(y, a), yb = rl_i(y, b);
    const int pa = rl_i(pred, a), pb = rl_i(pred, b);
    const double va = rl_d(v, a), vb = rl_d(v, b);
    const double da = rl_d(d, a), db = rl_d(d, b);
    if (lane == a) col = cb, y = yb, pred = pb, v = vb, d = db;
    if (lane == b) col = ca, y = ya, pred = pa, v = va, d = da;
  };
  // A run of swaps replayed on one index register (perm: the lane whose registers end at this
  // position) and applied once, by one gather per register, when it is long: a swap then costs
  // one or two readlanes instead of fourteen.  (The runs below only swap a position k with one at
  // or before it, so a later position still holds its own registers while the run is replayed.)
  auto swap_perm = [&](int& perm, int a, int b) {
    if (a == b) return;
    const int pa = rl_i(perm, a), pb = rl_i(perm, b);
    perm = lane == a ? pb : (lane == b ? pa : perm);
  };
  auto apply_perm = [&](int perm) {
    col = __shfl(col, perm);
    y = __shfl(y, perm);
    pred = __shfl(pred, perm);
    v = __shfl(v, perm);
    d = __shfl(d, perm);
  };
  // (a run of three or more swaps pays for the gather: ge3)
  // ---- _ca_dense
  for (int f = 0; f < nfree; f++) {
    const int start = rl_i(fr, f);
    if (col != lane) {  // find_path_dense restarts from cols[j] = j: every column back to its lane
      const int c0 = col;
      v = perm_d(v, c0);
      y = perm_i(y, c0);
      col = lane;
    }
    const double cs = crow_at(start, lane);
    if (own) {
      d = cs - v;
      pred = start;
    }
    int low = 0, up = 0, last = 0, endofpath = -1;
    bool found = false;
    double mn = 0.0;
    JVT(0);
    do {
      if (up == low)
        JCNT(1, 1);
      else
        JCNT(2, 1);
      JVT(3);
      if (up == low) {
        last = low - 1;
        const bool cand = own && lane >= low;
        const bool nanb = __any(cand && isnan(d));
        // inclusive prefix minimum of d over the TODO positions (lanes below lo hold INF): its
        // lane 63 is the minimum, and shifted by one lane (DPP wave_shr, lane 0 INF) the
        // exclusive one the sequential find below compares against
        const double pm = nanb ? INF : scan_min_d(cand ? d : INF);
        const double m = nanb ? INF : rl_d(pm, 63);
        const bool bad = nanb || !(m < INF);
        const int ke = bad ? -1 : last_lane(cand && d == m && y < 0);
        if (ke >= 0) {
          // _find_dense's SCAN set = the TODO columns at the minimum in position order; the path
          // ends at the LAST unassigned one (the rest of the permutation is never read again)
          mn = rl_d(d, first_lane(cand && d == m));
          endofpath = rl_i(col, ke);
          found = true;
        } else {
          JCNT(3, 1);
          // _find_dense on the position lanes: mind runs from d[cols[lo]], and the positions
          // k > lo whose d is <= the minimum of d over [lo, k) are its events — those with d
          // strictly below it reset up to lo — found by ballots against the exclusive prefix
          // minimum, then replayed in order (a swap only exchanges k with a position <= k, so a
          // later position still holds its own registers: position k's own are k's at its event)
          mn = rl_d(d, low);
          up = low + 1;
          if (!nanb) {
            const double ex = dpp_d<0x138, 0xf, 0xf>(pm, INF);  // wave_shr:1
            const bool evk = own && lane > low && d <= ex;
            unsigned long long ev = __ballot(evk);
            const unsigned long long st = __ballot(evk && d < ex);
            JCNT(8, __popcll(ev));
            if (st) mn = rl_d(d, 63 - __clzll((long long)st));  // the last reset's d
            if (ge3(ev)) {
              int perm = lane;  // the lane whose registers end at this position
              while (ev) {
                const int k = __ffsll((long long)ev) - 1;
                ev &= ev - 1;
                if ((st >> k) & 1ull) up = low;
                const int pu = rl_i(perm, up);
                perm = lane == up ? k : (lane == k ? pu : perm);
                up++;
              }
              apply_perm(perm);
            } else {
              while (ev) {
                const int k = __ffsll((long long)ev) - 1;
                ev &= ev - 1;
                if ((st >> k) & 1ull) up = low;
                swap_pos(k, up);
                up++;
              }
            }
          } else {
            for (int k = up; k < n; k++) {
              const double h = rl_d(d, k);
              if (h <= mn) {
                if (h < mn) {
                  up = low;
                  mn = h;
                }
                swap_pos(k, up);
                up++;
              }
            }
          }
          const int ke2 = last_lane(own && lane >= low && lane < up && y < 0);
          if (ke2 >= 0) {
            endofpath = rl_i(col, ke2);
            found = true;
          }
        }
      }
      JVT(5);
      if (!found) {
        // _scan_dense from the SCAN column at position lo
        // (the next scan's row prefetched at the end of this one measured slower: C5 scan cycles
        // +8%, the load's wait lands at the loop head)
        const int i = rl_i(y, low);
        const double crow = crow_at(i, col);  // lanes past n: column >= nc, 0
        const double mind = rl_d(d, low);
        const double h = rl_d(crow, low) - rl_d(v, low) - mind;  // lane lo holds column cols[lo]
        low++;
        const bool R = own && lane >= up;
        const double v2 = crow - v - h;  // every lane (no masked region); used where R
        const bool A = R && v2 < d;
        const bool B = A && v2 == mind;
        const bool E = B && y < 0;
        int pe = first_lane(E);  // _scan_dense's early return
        if (pe < 0) pe = OW;
        const bool act = R && lane <= pe;
        if (act && A) {
          pred = i;
          d = v2;
        }
        if (pe < OW) {
          endofpath = rl_i(col, pe);
          found = true;
        }
        // columns lowered to the minimum join the SCAN set, in position order (all before pe)
        unsigned long long bits = __ballot(act && B && lane < pe);
        JCNT(9, __popcll(bits));
        if (!bits) {
        } else if (ge3(bits)) {
          int perm = lane;
          while (bits) {
            const int k = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            swap_perm(perm, k, up);
            up++;
          }
          apply_perm(perm);
        } else {
          while (bits) {
            const int k = __ffsll((long long)bits) - 1;
            bits &= bits - 1;
            swap_pos(k, up);
            up++;
          }
        }
      }
      JVT(6);
    } while (!found);
    if (own && lane <= last) v = v + (d - mn);  // lapx: v[j] += d[j] - mind
    JVT(1);
    int i;
    do {
      const int le = first_lane(own && col == endofpath);
      i = rl_i(pred, le);
      if (lane == le) y = i;
      const int j1 = endofpath;
      endofpath = rl_i(xr, i);
      if (lane == i) xr = j1;
      JCNT(10, 1);
    } while (i != start);
    JVT(2);
  }
  JVT(7);
  if (own) {
    w.x[lane] = xr;
    w.y[col] = y;
    w.v[col] = v;
  }
  sync();
  JVT(7);
#undef JVT
#ifdef BX_PHASE_TIMING
  if (lane == 0 && w.dc) {
    for (int q = 0; q < 16; q++) w.dc[q] += jcnt[q];
    for (int q = 4; q < 8; q++) w.dc[q] += jacc[q];
    for (int q = 0; q < 4; q++) w.dc[12 + q] += jacc[q];
  }
#endif
#undef JCNT
}

// lapx's lapjv(extend_cost=True) answer on the real rows when that answer is the ONLY optimum,
// found without lapjv: scipy's shortest-augmenting-path LSAP (Crouse; rows in order, a Dijkstra
// over the columns per row, column j on lane j, row i's duals on lane i) on the zero-padded
// n x n problem lapx solves (n = max(nr, nc) <= 64), then a uniqueness test.  Any optimal
// assignment uses only edges that are tight (zero reduced cost) under ANY optimal duals, so a
// second optimum exists iff the tight graph (row i -> the row matched to a tight column of i)
// has a cycle; one through a real row could change lapx's pairs.  Tight = reduced cost <=
// LSAP_TIE_TOL, far above the two solvers' rounding (n * eps * |C| ~ 1e-14 at these costs), so a
// near-tie is treated as a tie.  Returns true with w.x (row -> column, >= nc: unmatched) when
// the real rows' optimum is unique; false when tied or degenerate (NaN / infinite costs, a
// dual infeasibility) — the caller then runs lapjv itself.  One wave; sync as jv_wave64's.
constexpr double LSAP_TIE_TOL = 1e-9;
template <class SY = SyncBlock, int AS = 0>
__device__ bool lsap_unique64(const double* C, int nr, int nc, JvLds& w, SY sync = SY{}) {
  const int n = nr > nc ? nr : nc;
  const int lane = threadIdx.x & 63;
  const bool own = lane < n;
  auto crow_at = [&](int i, int j) -> double {  // row i uniform, column j per lane
    double c = 0.0;
    if (i < nr && nc > 0) {
      const double t = cget_as<AS>(C, nr, nc, i, j < nc ? j : nc - 1);
      c = j < nc ? t : 0.0;
    }
    return c;
  };
  double u = 0.0, v = 0.0, spc = INF;
  int r4c = -1, c4r = -1, path = -1;  // column lane: its row; row lane: its column
  bool bad = false;
  for (int cur = 0; cur < n && !bad; cur++) {
    spc = INF;
    path = -1;
    bool sc = false, sr = false;
    int i = cur, sink = -1;
    double minv = 0.0;
    while (sink < 0) {
      if (lane == i) sr = true;
      const double ui = rl_d(u, i);
      const double r = minv + crow_at(i, lane) - ui - v;
      if (own && !sc && r < spc) {
        spc = r;
        path = i;
      }
      const double lowest = wave_min_bfly(own && !sc ? spc : INF);
      if (!(lowest < INF)) {  // NaN / infinite costs: lapjv's own handling
        bad = true;
        break;
      }
      const bool cand = own && !sc && spc == lowest;
      int j = first_lane(cand && r4c < 0);  // scipy's tie rule: an unassigned column first
      if (j < 0) j = first_lane(cand);
      minv = lowest;
      if (lane == j) sc = true;
      const int r4 = rl_i(r4c, j);
      if (r4 < 0) sink = j;
      else i = r4;
    }
    if (bad) break;
    // duals: u[cur] += minv; the other rows of SR u[i] += minv - spc[col4row[i]]; SC columns
    // v[j] -= minv - spc[j]
    const double sp4 = __shfl(spc, c4r >= 0 ? c4r : 0);
    if (lane == cur) u += minv;
    else if (sr) u += minv - sp4;
    if (sc) v -= minv - spc;
    // augment along path[] from the sink back to cur
    int j = sink;
    while (true) {
      const int pi = rl_i(path, j);
      if (lane == j) r4c = pi;
      const int old = rl_i(c4r, pi);
      if (lane == pi) c4r = j;
      if (pi == cur) break;
      j = old;
    }
  }
  if (bad) return false;
  // the tight graph: row lane i's successors (the rows matched to its tight unmatched columns)
  if (own) {
    w.v[lane] = v;
    w.y[lane] = r4c;
  }
  sync();
  unsigned long long A = 0;
  bool infeasible = false;
  if (own)
    for (int j = 0; j < n; j++) {
      double c = 0.0;
      if (lane < nr && j < nc) c = cget_as<AS>(C, nr, nc, lane, j);
      const double rc = c - u - w.v[j];
      if (!(rc >= -LSAP_TIE_TOL)) infeasible = true;  // (NaN included)
      if (j != c4r && rc <= LSAP_TIE_TOL) A |= 1ull << w.y[j];
    }
  if (__any(infeasible)) return false;
  // cycle test: reachability closure by repeated squaring (masks in w.d), then a real row on a
  // cycle is a tie
  unsigned long long* M = (unsigned long long*)w.d;
  bool tied = false;
  if (__any(A != 0ull)) {
    unsigned long long R = A;
    for (int it = 0; it < 7; it++) {
      sync();
      if (own) M[lane] = R;
      sync();
      unsigned long long nR = R, m = R;
      while (m) {
        const int k = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        nR |= M[k];
      }
      const bool grew = __any(nR != R);
      R = nR;
      if (!grew) break;
    }
    tied = __any(own && lane < nr && ((R >> lane) & 1ull));
  }
  if (tied) return false;
  sync();
  if (own) w.x[lane] = c4r;
  sync();
  return true;
}

// legacy linear_assignment of the nr x nc matrix C: pairs (row, col) in row order into out
// (interleaved), returns the count (uniform).  SY: the whole one-wave workgroup, or SyncWaveL
// when one wave of a larger workgroup solves alone.
// cas: the address space C is known to be in (3: LDS, 1: global, 0: either), for n <= 64.
template <class SY = SyncBlock>
__device__ int legacy_lap(const double* C, int nr, int nc, JvLds& jv, int* out, SY sync = SY{},
                          int cas = 0) {
  if ((nr > nc ? nr : nc) <= OW) {
    if (cas == 3)
      jv_wave64<SY, 3>(C, nr, nc, jv, sync);
    else if (cas == 1)
      jv_wave64<SY, 1>(C, nr, nc, jv, sync);
    else
      jv_wave64<SY, 0>(C, nr, nc, jv, sync);
  } else
    jv_wave(C, nr, nc, jv, sync);
  return wave_compact_s(
      nr, [&](int i) { return jv.x[i] < nc; },
      [&](int i, int p) {
        out[2 * p] = i;
        out[2 * p + 1] = jv.x[i];
      },
      sync);
}

// legacy_lap with the shortest-augmenting-path solve first (lsap_unique64): lapjv itself only
// when the real rows' optimum is tied (or n > 64).  `jv_ran` tells the caller which it was.
template <class SY = SyncBlock>
__device__ int legacy_lap_ssp(const double* C, int nr, int nc, JvLds& jv, int* out, SY sync,
                              bool& jv_ran) {
  if ((nr > nc ? nr : nc) <= OW && lsap_unique64<SY, 0>(C, nr, nc, jv, sync)) {
    jv_ran = false;
    return wave_compact_s(
        nr, [&](int i) { return jv.x[i] < nc; },
        [&](int i, int p) {
          out[2 * p] = i;
          out[2 * p + 1] = jv.x[i];
        },
        sync);
  }
  jv_ran = true;
  return legacy_lap(C, nr, nc, jv, out, sync);
}
