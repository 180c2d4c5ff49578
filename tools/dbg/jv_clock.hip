// Diagnostic: lapx's JV (jv_wave_t) on the cost_limit extension of a matrix read from a file,
// state in LDS, with BX_JV_CLOCK phase clocks.  Usage: jv_clock <file: int32 nr, nc; f64 cost>
// <limit>.  Prints the per-phase microseconds and the step counts.
#define BX_JV_CLOCK 1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../boxmot_amd/csrc/bx_device.h"
using namespace bx;
namespace {
#include "../../boxmot_amd/csrc/bx_jv.h"
__global__ __launch_bounds__(64) void k(const double* cost, int nr, int nc, double lim,
                                        unsigned long long* dc, int* x, int lcost,
                                        const unsigned char* cls, int skip, int eng,
                                        unsigned char* gst) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int n = nr + nc;
  JvLds w = jv_bind(smem, n);
  if (lcost) {  // the real block copied into LDS after the state: the accessor reads LDS
    double* lc = (double*)(smem + ((jv_bytes(n) + 15) & ~size_t(15)));
    for (int k = threadIdx.x; k < nr * nc; k += 64) lc[k] = cost[k];
    __syncthreads();
    cost = lc;
  }
  w.dc = dc;
  const double half = lim / 2.;
  unsigned long long t0 = wall_clock64();
  const JvExt cf{cost, nr, nc, half};
  auto rk = [&](int i) { return i >= nr ? 0 : (cls[i] ? 1 : -1); };
  if (eng) {
    if (skip) jv_wave_t(cf, n, w, SyncWaveLG{eng == 2}, rk);
    else jv_wave_t(cf, n, w, SyncWaveLG{eng == 2});
  } else {
    if (skip) jv_wave_t(cf, n, w, SyncBlock{}, rk);
    else jv_wave_t(cf, n, w, SyncBlock{});
  }
  if (threadIdx.x == 0) dc[6] = wall_clock64() - t0;
  for (int i = threadIdx.x; i < n; i += 64) x[i] = w.x[i];
}
}  // namespace
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  int nr, nc;
  if (fread(&nr, 4, 1, f) != 1 || fread(&nc, 4, 1, f) != 1) return 1;
  std::vector<double> c((size_t)nr * nc);
  if (fread(c.data(), 8, c.size(), f) != c.size()) return 1;
  fclose(f);
  const double lim = atof(argv[2]);
  const int lcost = argc > 3 ? atoi(argv[3]) : 0;
  const int skip = argc > 4 ? atoi(argv[4]) : 0;
  const int eng = argc > 5 ? atoi(argv[5]) : 0;
  unsigned char* gst;
  hipMalloc(&gst, jv_bytes(nr + nc) + 256);
  // class 1: real rows constant over the real columns at the first constant row's value
  std::vector<unsigned char> cl(nr, 0);
  double K = 0; bool haveK = false;
  for (int i = 0; i < nr; i++) {
    bool cst = true;
    for (int j = 1; j < nc; j++) cst &= c[(size_t)i * nc + j] == c[(size_t)i * nc];
    if (cst && !haveK) { K = c[(size_t)i * nc]; haveK = true; }
    cl[i] = cst && c[(size_t)i * nc] == K;
  }
  unsigned char* dcl; hipMalloc(&dcl, nr);
  hipMemcpy(dcl, cl.data(), nr, hipMemcpyHostToDevice);
  double* dcost; unsigned long long* ddc; int* dx;
  hipMalloc(&dcost, c.size() * 8); hipMalloc(&ddc, 16 * 8); hipMalloc(&dx, 4 * (nr + nc));
  hipMemcpy(dcost, c.data(), c.size() * 8, hipMemcpyHostToDevice);
  int khz = 0;
  hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  const double tpu = khz / 1000.0;  // ticks per microsecond
  const size_t lds = ((jv_bytes(nr + nc) + 15) & ~size_t(15)) + (lcost ? c.size() * 8 : 0);
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  for (int rep = 0; rep < 2; rep++) {
    unsigned long long h[16] = {0};
    h[7] = nr;
    hipMemcpy(ddc, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), lds, 0, dcost, nr, nc, lim, ddc, dx, lcost, dcl, skip, eng, gst);
    hipMemcpy(h, ddc, sizeof(h), hipMemcpyDeviceToHost);
    std::vector<int> hx(nr + nc);
    hipMemcpy(hx.data(), dx, 4 * (nr + nc), hipMemcpyDeviceToHost);
    unsigned long long ck = 0;
    for (int i = 0; i < nr + nc; i++) ck = ck * 1000003ull + (unsigned)hx[i];
    printf("eng=%d x_hash=%016llx skip=%d lcost=%d nr=%d nc=%d total=%.1fus ccrrt=%.1f carr=%.1f find=%.1f scan=%.1f aug=%.1f "
           "scans=%llu real_row_scans=%llu skipped=%llu nfree=%llu finds=%llu serial_finds=%llu\n",
           eng, ck, skip, lcost, nr, nc, h[6] / tpu, h[8] / tpu, h[9] / tpu, h[10] / tpu, h[11] / tpu,
           h[12] / tpu, h[13], h[14], h[15], h[0], h[1], h[3]);
  }
  return 0;
}
