// bx_jv.h — wave-cooperative building blocks shared by the one-wave-per-sequence trackers
// (OCSort, BoostTrack): lapx's dense Jonker-Volgenant with the oracle's tie order, and a
// wave-order-preserving compaction.  Include inside a translation unit's anonymous namespace
// after bx_device.h (uses bx::INF); a workgroup is exactly one wave64.
#pragma once

constexpr int OW = 64;  // threads per workgroup: one wave per sequence

// Wave-cooperative lapx lapjv (oracle/bxo_ops.c bxo_lapjv) on the zero-padded square
// max(nr, nc) of a row-major nr x nc matrix (legacy linear_assignment, association.py:105-114).
struct JvLds {
  double *v, *d;
  int *x, *y, *matches, *freer, *pred, *col;
  int* sc;  // >= 8 ints of broadcast scratch
  double* sd;
  unsigned long long* dc;  // diagnostic counters (timing builds) or null
};

__device__ __forceinline__ double cget(const double* C, int nr, int nc, int i, int j) {
  return (i < nr && j < nc) ? C[i * nc + j] : 0.0;
}

__device__ double wave_min_d(double a) {
  for (int o = 32; o >= 1; o >>= 1) a = fmin(a, __shfl_xor(a, o));
  return a;
}

constexpr int JV_CH = 8;  // 64-position chunks of one relaxation (assignment sizes <= 512)

__device__ void jv_wave(const double* C, int nr, int nc, JvLds& w) {
  const int n = nr > nc ? nr : nc;
  const int lane = threadIdx.x;
  // column reduction: minima (first row index on ties) lane-parallel ...
  for (int j = lane; j < n; j += OW) {
    double mn = cget(C, nr, nc, 0, j);
    int imin = 0;
    for (int i = 1; i < n; i++) {
      const double c = cget(C, nr, nc, i, j);
      if (c < mn) mn = c, imin = i;
    }
    w.d[j] = mn;
    w.pred[j] = imin;
    w.x[j] = -1;
    w.matches[j] = 0;
  }
  __syncthreads();
  // ... and the sweep j = n-1..0 that settles them in the oracle's order
  if (lane == 0) {
    for (int j = n - 1; j >= 0; j--) {
      const int imin = w.pred[j];
      w.v[j] = w.d[j];
      if (++w.matches[imin] == 1) {
        w.x[imin] = j;
        w.y[j] = imin;
      } else if (w.v[j] < w.v[w.x[imin]]) {
        const int j1 = w.x[imin];
        w.x[imin] = j;
        w.y[j] = imin;
        w.y[j1] = -1;
      } else {
        w.y[j] = -1;
      }
    }
  }
  __syncthreads();
  // reduction transfer (rows in order: each changes v[x[i]], read by the rows after it)
  int nfree = 0;
  for (int i = 0; i < n; i++) {
    const int m = w.matches[i];
    if (m == 0) {
      if (lane == 0) w.freer[nfree] = i;
      nfree++;
    } else if (m == 1) {
      const int j1 = w.x[i];
      double mn = DBL_MAX;
      for (int j = lane; j < n; j += OW) {
        const double h = cget(C, nr, nc, i, j) - w.v[j];
        if (j != j1 && h < mn) mn = h;
      }
      mn = wave_min_d(mn);
      __syncthreads();
      if (lane == 0 && mn < DBL_MAX) w.v[j1] = w.v[j1] - mn;
      __syncthreads();
    }
  }
  __syncthreads();
#ifdef BX_PHASE_TIMING
  if (lane == 0 && w.dc) w.dc[0] += nfree;
#endif
  // augmentation
  for (int f = 0; f < nfree; f++) {
    const int fr = w.freer[f];
    for (int j = lane; j < n; j += OW) {
      w.d[j] = cget(C, nr, nc, fr, j) - w.v[j];
      w.pred[j] = fr;
      w.col[j] = j;
    }
    __syncthreads();
    int low = 0, up = 0, last = 0, endofpath = -1, found = 0;
    double mn = 0.0;
    do {
#ifdef BX_PHASE_TIMING
      if (lane == 0 && w.dc) w.dc[up == low ? 1 : 2] += 1;
#endif
      if (up == low) {
        // Minimum scan.  The oracle's sequential scan gathers, in position order, every column
        // at the minimum distance into col[low..up) and takes the first unassigned one as the
        // path end.  When one exists the search ends here and the rest of the permutation it
        // built is never read again (col is rebuilt for the next free row), so the lane-parallel
        // path finds it directly; otherwise (or with NaN distances) the scan runs as written.
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
          for (int base = low; base < n && ke < 0; base += OW) {
            const int k = base + lane;
            bool G = false, E = false;
            if (k < n) {
              const int j = w.col[k];
              G = w.d[j] == m;
              E = G && w.y[j] < 0;
            }
            const unsigned long long gm = __ballot(G), em = __ballot(E);
            if (kg < 0 && gm) kg = base + __ffsll((long long)gm) - 1;
            if (em) ke = base + __ffsll((long long)em) - 1;
          }
        }
#ifdef BX_PHASE_TIMING
        if (lane == 0 && w.dc && ke < 0) w.dc[3] += 1;
#endif
        if (ke >= 0) {
          last = low - 1;
          mn = w.d[w.col[kg]];  // the first minimum, exactly as the sequential scan keeps it
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
                break;
              }
            w.sc[0] = last;
            w.sc[1] = up;
            w.sc[2] = endofpath;
            w.sc[3] = found;
            w.sd[0] = mn;
          }
          __syncthreads();
          last = w.sc[0];
          up = w.sc[1];
          endofpath = w.sc[2];
          found = w.sc[3];
          mn = w.sd[0];
          __syncthreads();
        }
      }
      if (!found) {
        const int j1 = w.col[low++];
        const int i = w.y[j1];
        const double h = cget(C, nr, nc, i, j1) - w.v[j1] - mn;
        // relaxation from row i over col[up..n) in chunks of 64 positions; the first column
        // reached at distance mn that is unassigned ends the path (the oracle's break).  Every
        // operand of every chunk is loaded up front: a swap writes only positions up to the
        // chunk in flight, and each column appears once, so later chunks read what the
        // sequential loop would.
        const int up0 = up;
        int jc[JV_CH];
        double v2c[JV_CH], dc[JV_CH];
        bool yc[JV_CH];
#pragma unroll
        for (int c = 0; c < JV_CH; c++) {
          const int k = up0 + c * OW + lane;
          jc[c] = -1;
          if (k < n) {
            const int j = w.col[k];
            jc[c] = j;
            v2c[c] = cget(C, nr, nc, i, j) - w.v[j] - h;
            dc[c] = w.d[j];
            yc[c] = w.y[j] < 0;
          }
        }
#pragma unroll
        for (int c = 0; c < JV_CH; c++) {
          const int base = up0 + c * OW;
          if (base >= n || found) break;
          const int j = jc[c];
          const double v2 = v2c[c];
          bool A = false, B = false, E = false;
          if (j >= 0) {
            A = v2 < dc[c];
            B = A && v2 == mn;
            E = B && yc[c];
          }
          const unsigned long long em = __ballot(E);
          int kE = OW;
          if (em) kE = __ffsll((long long)em) - 1;
          if (A && lane < kE) {
            w.pred[j] = i;
            w.d[j] = v2;
          }
          if (em && lane == kE) w.pred[j] = i;
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
        __syncthreads();
      }
    } while (!found);
    for (int k = lane; k <= last; k += OW) {
      const int j1 = w.col[k];
      w.v[j1] = w.v[j1] + w.d[j1] - mn;
    }
    __syncthreads();
    if (lane == 0) {
      int i;
      do {
        i = w.pred[endofpath];
        w.y[endofpath] = i;
        const int j1 = endofpath;
        endofpath = w.x[i];
        w.x[i] = j1;
      } while (i != fr);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// The same lapjv for n <= 64, register-resident.  Setup (column reduction, reduction transfer):
// lane j owns column j and row j.  Augmentation: lane k holds the column at POSITION k of the
// oracle's `col` permutation with its v, d, y and pred, so position-ordered choices (first column
// at the minimum, first unassigned, the oracle's break) are single ballots and the swaps
// col[k] <-> col[up] exchange two lanes' registers (readlane); rows keep x in lane i.  Every
// comparison, arithmetic operation and tie is the oracle's.
// DPP inclusive min-scan across the wave (row_shr 1/2/4/8 within rows of 16, then row_bcast 15
// and 31 — the gfx9 wave64 scan sequence); lanes whose source is outside the row keep the
// identity.  Lane 63 holds the wave minimum.
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
__device__ __forceinline__ int rl_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ double rl_d(double v, int k) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ int first_lane(bool p) {
  const unsigned long long m = __ballot(p);
  return m ? __ffsll((long long)m) - 1 : -1;
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

__device__ __forceinline__ double wave_min_dpp(double a) {  // no NaNs (fmin drops them anyway)
  return rl_d(scan_min_d(a), 63);
}

__device__ void jv_wave64(const double* C, int nr, int nc, JvLds& w) {
  const int n = nr > nc ? nr : nc;
  const int lane = threadIdx.x;
  const bool own = lane < n;
#ifdef BX_PHASE_TIMING
  unsigned long long jt0 = __builtin_amdgcn_s_memtime(), jt1 = 0, jacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
#endif
  double v = 0.0, d = 0.0;
  int y = -1, pred = 0, col = lane, xr = -1, matches = 0;
  // column reduction: the column minima (first row on ties) ...
  int imin = 0;
  if (own) {
    double mn = cget(C, nr, nc, 0, lane);
    for (int i = 1; i < n; i++) {
      const double c = cget(C, nr, nc, i, lane);
      if (c < mn) mn = c, imin = i;
    }
    v = mn;
  }
  // ... settled j = n-1..0 as the oracle does
  for (int j = n - 1; j >= 0; j--) {
    const int im = rl_i(imin, j);
    const double vj = rl_d(v, j);
    const int mc = rl_i(matches, im);
    const int xi = rl_i(xr, im);
    const double vx = rl_d(v, xi < 0 ? 0 : xi);
    if (mc == 0 || vj < vx) {
      if (lane == im) xr = j;
      if (lane == j) y = im;
      if (mc != 0 && lane == xi) y = -1;
    } else if (lane == j) {
      y = -1;
    }
    if (lane == im) matches++;
  }
  // reduction transfer, rows in order
  int nfree = 0;
  for (int i = 0; i < n; i++) {
    const int m = rl_i(matches, i);
    if (m == 0) {
      if (lane == 0) w.freer[nfree] = i;
      nfree++;
    } else if (m == 1) {
      const int j1 = rl_i(xr, i);
      double h = DBL_MAX;
      if (own && lane != j1) {
        const double t = cget(C, nr, nc, i, lane) - v;
        if (t < h) h = t;
      }
      h = wave_min_dpp(h);
      if (h < DBL_MAX && lane == j1) v = v - h;
    }
  }
  __syncthreads();
#ifdef BX_PHASE_TIMING
  if (lane == 0 && w.dc) w.dc[0] += nfree;
#endif
  JVT(4);
  // exchange the registers of positions a and b (col[a] <-> col[b])
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
  // augmentation
  for (int f = 0; f < nfree; f++) {
    const int fr = w.freer[f];
    if (col != lane) {  // the oracle restarts from col[j] = j: every column back to its lane
      const int c0 = col;
      v = perm_d(v, c0);
      y = perm_i(y, c0);
      col = lane;
    }
    if (own) {
      d = cget(C, nr, nc, fr, lane) - v;
      pred = fr;
    }
    int low = 0, up = 0, last = 0, endofpath = -1;
    bool found = false;
    double mn = 0.0;
    do {
#ifdef BX_PHASE_TIMING
      if (lane == 0 && w.dc) w.dc[up == low ? 1 : 2] += 1;
#endif
      JVT(7);
      if (up == low) {
        last = low - 1;
        const bool cand = own && lane >= low;
        bool bad = __any(cand && isnan(d));
        double m = bad ? INF : wave_min_dpp(cand ? d : INF);
        bad = bad || !(m < INF);
        const int ke = bad ? -1 : first_lane(cand && d == m && y < 0);
        if (ke >= 0) {
          // the columns at the minimum form the new TODO set in position order; the first
          // unassigned one ends the path (the rest of the permutation is never read again)
          mn = m;
          endofpath = rl_i(col, ke);
          found = true;
        } else {
#ifdef BX_PHASE_TIMING
          if (lane == 0 && w.dc) w.dc[3] += 1;
#endif
          // the oracle's scan, on the position lanes: mn runs from d[col[low]], and the
          // positions k > low whose d is <= the minimum of d over [low, k) are its events (a
          // swap only exchanges k with a position <= k, so later positions still hold their
          // columns) — found by a prefix minimum across the lanes, then replayed in order
          mn = rl_d(d, low);
          up = low + 1;
          if (!__any(own && lane >= low && isnan(d))) {
            const double pm = scan_min_d((own && lane >= low) ? d : INF);
            double ex = __shfl_up(pm, 1);
            if (lane == 0) ex = INF;
            unsigned long long ev = __ballot(own && lane > low && d <= ex);
            while (ev) {
              const int k = __ffsll((long long)ev) - 1;
              ev &= ev - 1;
              const double h = rl_d(d, k);
              if (h < mn) {
                up = low;
                mn = h;
              }
              swap_pos(k, up);
              up++;
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
          const int ke2 = first_lane(own && lane >= low && lane < up && y < 0);
          if (ke2 >= 0) {
            endofpath = rl_i(col, ke2);
            found = true;
          }
        }
      }
      JVT(5);
      if (!found) {
        const int j1 = rl_i(col, low);
        const int i = rl_i(y, low);
        const double h = cget(C, nr, nc, i, j1) - rl_d(v, low) - mn;
        low++;
        const bool R = own && lane >= up;
        double v2 = 0.0;
        bool A = false, B = false, E = false;
        if (R) {
          v2 = cget(C, nr, nc, i, col) - v - h;
          A = v2 < d;
          B = A && v2 == mn;
          E = B && y < 0;
        }
        int pe = first_lane(E);  // the oracle's break
        if (pe < 0) pe = OW;
        const bool act = R && lane < pe;
        if (act && A) {
          pred = i;
          d = v2;
        }
        if (lane == pe) pred = i;
        if (pe < OW) {
          endofpath = rl_i(col, pe);
          found = true;
        }
        // columns reaching the minimum join the TODO set, in position order (all before pe)
        unsigned long long bits = __ballot(act && B);
        while (bits) {
          const int k = __ffsll((long long)bits) - 1;
          bits &= bits - 1;
          swap_pos(k, up);
          up++;
        }
      }
      JVT(6);
    } while (!found);
    if (own && lane <= last) v = v + d - mn;
    int i;
    do {
      const int le = first_lane(own && col == endofpath);
      i = rl_i(pred, le);
      if (lane == le) y = i;
      const int j1 = endofpath;
      endofpath = rl_i(xr, i);
      if (lane == i) xr = j1;
    } while (i != fr);
  }
  if (own) {
    w.x[lane] = xr;
    w.y[col] = y;
    w.v[col] = v;
  }
  __syncthreads();
  JVT(7);
#undef JVT
#ifdef BX_PHASE_TIMING
  if (lane == 0 && w.dc)
    for (int q = 4; q < 8; q++) w.dc[q] += jacc[q];
#endif
}

// ------------------------------------------------------------------------------------------
// Wave-order-preserving compaction: emit(k, pos) for k < n with pred(k); returns the count.
template <class P, class E>
__device__ int wave_compact(int n, P pred, E emit) {
  const int lane = threadIdx.x;
  int base = 0;
  for (int c = 0; c < n; c += OW) {
    const int k = c + lane;
    const bool f = k < n && pred(k);
    const unsigned long long m = __ballot(f);
    if (f) emit(k, base + __popcll(m & ((1ull << lane) - 1ull)));
    base += __popcll(m);
  }
  __syncthreads();
  return base;
}

// legacy linear_assignment of the nr x nc matrix C: pairs (row, col) in row order into out
// (interleaved), returns the count (uniform)
__device__ int legacy_lap(const double* C, int nr, int nc, JvLds& jv, int* out) {
  if ((nr > nc ? nr : nc) <= OW)
    jv_wave64(C, nr, nc, jv);
  else
    jv_wave(C, nr, nc, jv);
  return wave_compact(
      nr, [&](int i) { return jv.x[i] < nc; },
      [&](int i, int p) {
        out[2 * p] = i;
        out[2 * p + 1] = jv.x[i];
      });
}
