// Development micro-benchmark (not part of the library): the blocked inverse's 128-tile trailing
// update with C0 read in the epilogue (launch_trail128_band, C = C0 - A B) against the variant whose
// accumulators start from C0 (launch_trail128_pre) and the same tile grid with no C0 at all
// (launch_gemm EPI_STORE), and C0 folded in during the K loop (launch_trail128, the library's update at B2 = 256),
// hipEvent-timed.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMIDAGMA_EXPERIMENTS
//          -I../../midagma_amd/csrc trail_micro.hip ../../midagma_amd/csrc/gemm.hip -o trail_micro
//   run  : ./trail_micro [D ...]   (default 2048 3072 5120; B2 = 256, outer step g = 1)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "launch.h"

using namespace midagma;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void fill_kernel(double* p, int64_t n, uint64_t seed, double scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = scale * ((double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5);
  }
}

__global__ void reldiff_kernel(const double* a, const double* b, int64_t n, unsigned long long* out) {
  double m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmax(m, fabs(a[i] - b[i]) / fmax(1e-300, fabs(b[i])));
  atomicMax(out, (unsigned long long)__double_as_longlong(m));
}

static double reldiff(const double* a, const double* b, int64_t n) {
  unsigned long long* d;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(reldiff_kernel, dim3(4096), dim3(256), 0, 0, a, b, n, d);
  unsigned long long h = 0;
  CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  double r;
  memcpy(&r, &h, 8);
  return r;
}

template <class F>
static double time_us(F&& f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return 1e3 * ms / reps;
}

int main(int argc, char** argv) {
  std::vector<int64_t> Ds;
  for (int i = 1; i < argc; ++i) Ds.push_back(atoll(argv[i]));
  if (Ds.empty()) Ds = {2048, 3072, 5120};
  gemm_setup_attributes();
  const int64_t B2 = 256, g = 1;
  const int reps = 50;
  for (int64_t D : Ds) {
    double *Ain, *Aout, *Aout2, *Aout3, *C;
    CK(hipMalloc(&Ain, sizeof(double) * D * D));
    CK(hipMalloc(&Aout, sizeof(double) * D * D));
    CK(hipMalloc(&Aout2, sizeof(double) * D * D));
    CK(hipMalloc(&Aout3, sizeof(double) * D * D));
    CK(hipMalloc(&C, sizeof(double) * D * D));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, Ain, D * D, 1, 2.0);
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, Aout, D * D, 2, 2.0);
    CK(hipMemcpy(Aout2, Aout, sizeof(double) * D * D, hipMemcpyDeviceToDevice));
    CK(hipMemcpy(Aout3, Aout, sizeof(double) * D * D, hipMemcpyDeviceToDevice));
    CK(hipDeviceSynchronize());
    const int64_t t = D - B2;
    const double f = 2.0 * t * t * B2;
    const double us_lib = time_us([&] { launch_trail128_band(Ain, Aout, D, B2, g, false, nullptr, 0); }, reps);
    const double us_pre = time_us([&] { launch_trail128_pre(Ain, Aout2, D, B2, g, false, nullptr, 0); }, reps);
    CK(hipDeviceSynchronize());
    const double us_mid = time_us([&] { launch_trail128(Ain, Aout3, D, B2, g, false, nullptr, 0); }, reps);
    CK(hipDeviceSynchronize());
    const double rd = reldiff(Aout2, Aout, D * D);
    const double rd_mid = reldiff(Aout3, Aout, D * D);
    const double us_st = time_us([&] {
      launch_gemm(t, t, B2, Ain, D, false, Aout, D, B_PLAIN, C, D, EPI_STORE, 1, 0, nullptr, 0, 0, nullptr, 0);
    }, reps);
    // in place (Aout = Ain: the whole matrix is one 8 D^2-byte buffer, which fits the 256 MB
    // Infinity Cache up to D ~ 5600; timing only: the column band is read while other tiles write)
    const double us_ip = time_us([&] { launch_trail128_band(Aout2, Aout2, D, B2, g, false, nullptr, 0); }, reps);
    const double us_ip_pre = time_us([&] { launch_trail128_pre(Aout2, Aout2, D, B2, g, false, nullptr, 0); }, reps);
    // in place with C0 folded in during the K loop (the product's tile body; timing only)
    const double us_ip_mid = time_us([&] { launch_trail128(Aout2, Aout2, D, B2, g, false, nullptr, 0); }, reps);
    printf("D=%5ld in place, C0 folded (mid) %8.2f us (ping-pong mid above)\n", (long)D, us_ip_mid);
    // persistent workgroups (launch_trail128_persist): static round robin and a claimed-tile queue
    double* Aout4;
    int* ctr;
    CK(hipMalloc(&Aout4, sizeof(double) * D * D));
    CK(hipMalloc(&ctr, sizeof(int)));
    CK(hipMemcpy(Aout4, Aout3, sizeof(double) * D * D, hipMemcpyDeviceToDevice));
    double us_ps[3], us_pd[3], rd_ps = 0, rd_pd = 0;
    const int nwgs[3] = {256, 512, 1024};
    for (int k = 0; k < 3; ++k) {
      us_ps[k] = time_us([&] { launch_trail128_persist(Ain, Aout4, D, g, false, nullptr, nwgs[k], nullptr, 0); }, reps);
      CK(hipDeviceSynchronize());
      rd_ps = fmax(rd_ps, reldiff(Aout4, Aout3, D * D));
      us_pd[k] = time_us([&] {
        CK(hipMemsetAsync(ctr, 0, sizeof(int), 0));
        launch_trail128_persist(Ain, Aout4, D, g, false, nullptr, nwgs[k], ctr, 0);
      }, reps);
      CK(hipDeviceSynchronize());
      rd_pd = fmax(rd_pd, reldiff(Aout4, Aout3, D * D));
    }
    const double us_memset = time_us([&] { CK(hipMemsetAsync(ctr, 0, sizeof(int), 0)); }, reps);
    // stream-K remainder: dp = whole rounds of 512 tiles, the rest over nsk workgroups
    const int ntl = (int)(((D - B2) / 128) * ((D - B2) / 128));
    double* ws;
    int* flg;
    CK(hipMalloc(&ws, sizeof(double) * 2 * 1024 * 16384));
    CK(hipMalloc(&flg, sizeof(int) * 1024));
    CK(hipMemset(flg, 0, sizeof(int) * 1024));
    double us_sk[3], rd_sk = 0;
    const int nsks[3] = {256, 512, 1024};
    for (int q = 0; q < 3; ++q) {
      const int dp = (ntl / 512) * 512;
      us_sk[q] = time_us([&] { launch_trail128_sk(Ain, Aout4, D, g, false, nullptr, dp, nsks[q], ws, flg, 0); }, reps);
      CK(hipDeviceSynchronize());
      rd_sk = fmax(rd_sk, reldiff(Aout4, Aout3, D * D));
    }
    const double us_sk0 = time_us([&] { launch_trail128_sk(Ain, Aout4, D, g, false, nullptr, ntl, 512, ws, flg, 0); },
                                  reps);
    printf("D=%5ld stream-K remainder (dp %d of %d tiles) over 256/512/1024 wgs %8.2f %8.2f %8.2f us | dp only "
           "%8.2f us | max rel diff vs mid %.1e\n", (long)D, (ntl / 512) * 512, ntl, us_sk[0], us_sk[1], us_sk[2],
           us_sk0, rd_sk);
    CK(hipFree(ws));
    CK(hipFree(flg));
    printf("D=%5ld persistent static 256/512/1024 wgs %8.2f %8.2f %8.2f us | claimed %8.2f %8.2f %8.2f us (incl. "
           "a %.2f us memset) | rel diff vs mid %.1e %.1e\n", (long)D, us_ps[0], us_ps[1], us_ps[2], us_pd[0],
           us_pd[1], us_pd[2], us_memset, rd_ps, rd_pd);
    CK(hipFree(Aout4));
    CK(hipFree(ctr));
    const int tiles = (int)((t / 128) * (t / 128));
    printf("D=%5ld tiles=%5d (%.2f rounds of 512)  lib %8.2f us %5.1f TF | pre %8.2f us %5.1f TF | "
           "mid %8.2f us %5.1f TF | no-C0 store %8.2f us %5.1f TF | in place %8.2f / pre %8.2f us | max rel diff "
           "pre %.2e mid %.2e vs lib\n",
           (long)D, tiles, tiles / 512.0, us_lib, f / us_lib / 1e6, us_pre, f / us_pre / 1e6, us_mid, f / us_mid / 1e6,
           us_st, f / us_st / 1e6, us_ip, us_ip_pre, rd, rd_mid);
    fflush(stdout);
    CK(hipFree(Ain));
    CK(hipFree(Aout));
    CK(hipFree(Aout2));
    CK(hipFree(Aout3));
    CK(hipFree(C));
  }
  return 0;
}
