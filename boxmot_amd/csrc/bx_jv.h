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
  jv_wave(C, nr, nc, jv);
  return wave_compact(
      nr, [&](int i) { return jv.x[i] < nc; },
      [&](int i, int p) {
        out[2 * p] = i;
        out[2 * p + 1] = jv.x[i];
      });
}
