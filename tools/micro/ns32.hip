// Microbenchmark: cycle cost of the pieces of the GJ diagonal-owner chain on ONE
// workgroup (256 threads) of an otherwise idle GPU.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off ns32.hip -o ns32 && ./ns32
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int NB = 32, ST = 34, REPS = 64;

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ int q_m0() { return (threadIdx.x >> 7) * 16; }
__device__ __forceinline__ int q_n0() { return ((threadIdx.x >> 6) & 1) * 16; }

__device__ __forceinline__ void mma32(const double* Ls, const double* Rs, dbl4& acc) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4;
  const double* La = Ls + (q_m0() + r) * ST + kq;
  const double* Rb = Rs + kq * ST + q_n0() + r;
#pragma unroll
  for (int k0 = 0; k0 < NB; k0 += 4)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(La[k0], Rb[k0 * ST], acc, 0, 0, 0);
}
// operands already in registers: pure MFMA chain
__device__ __forceinline__ void mma32_reg(const double* a, const double* b, dbl4& acc) {
#pragma unroll
  for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  const long long b = __double_as_longlong(v);
  double m = v;
#pragma unroll
  for (int row = 0; row < 4; ++row) {
    const int lo = __builtin_amdgcn_readlane((int)b, row * 16);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), row * 16);
    const double r = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    m = row == 0 ? r : fmax(m, r);
  }
  return m;
}

__global__ __launch_bounds__(256) void bench(const double* in, double* sink, unsigned long long* out) {
  __shared__ double A[NB * ST], B[NB * ST], C[NB * ST];
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * ST; e += 256) {
    A[e] = in[e % 1024] * 1e-3;
    B[e] = in[(e + 7) % 1024] * 1e-3;
    C[e] = 0.0;
  }
  __syncthreads();
  dbl4 acc = {0, 0, 0, 0};
  unsigned long long t0, t1;
  // 1: dependent MFMA chains, operands in registers
  double a[8], b[8];
  for (int q = 0; q < 8; ++q) { a[q] = in[(tid + q) & 1023]; b[q] = in[(tid * 3 + q) & 1023]; }
  t0 = now();
  for (int r = 0; r < REPS; ++r) mma32_reg(a, b, acc);
  t1 = now();
  if (tid == 0) out[0] = (t1 - t0) / REPS;
  // 2: mma32 from LDS, dependent through acc
  __syncthreads();
  t0 = now();
  for (int r = 0; r < REPS; ++r) mma32(A, B, acc);
  t1 = now();
  if (tid == 0) out[1] = (t1 - t0) / REPS;
  // 3: barrier alone
  __syncthreads();
  t0 = now();
  for (int r = 0; r < REPS; ++r) __syncthreads();
  t1 = now();
  if (tid == 0) out[2] = (t1 - t0) / REPS;
  // 4: wave_max alone (dependent)
  double v = acc[0];
  t0 = now();
  for (int r = 0; r < REPS; ++r) v = wave_max(v) * 0.5 + acc[r & 3];
  t1 = now();
  if (tid == 0) out[3] = (t1 - t0) / REPS;
  // 5: shuffle max (ds_bpermute)
  t0 = now();
  for (int r = 0; r < REPS; ++r) {
    double m = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmax(m, __shfl_xor(m, off));
    v = m * 0.5 + acc[r & 3];
  }
  t1 = now();
  if (tid == 0) out[4] = (t1 - t0) / REPS;
  // 6: one NS-like half iteration: mma32 + write C + barrier
  __syncthreads();
  t0 = now();
  for (int r = 0; r < REPS; ++r) {
    dbl4 s = {0, 0, 0, 0};
    mma32(A, B, s);
    const int lane = tid & 63;
#pragma unroll
    for (int t = 0; t < 4; ++t) C[(q_m0() + (lane >> 4) + 4 * t) * ST + q_n0() + (lane & 15)] = s[t];
    __syncthreads();
    acc += s;
  }
  t1 = now();
  if (tid == 0) out[5] = (t1 - t0) / REPS;
  // 7: full NS iteration pattern: mma(A,B)->C, reduce, barrier, mma(B,C) -> B', barrier
  __syncthreads();
  t0 = now();
  for (int r = 0; r < REPS; ++r) {
    dbl4 s = {0, 0, 0, 0};
    mma32(A, B, s);
    const int lane = tid & 63;
    double am = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      C[(q_m0() + (lane >> 4) + 4 * t) * ST + q_n0() + (lane & 15)] = s[t];
      am = fmax(am, fabs(s[t]));
    }
    am = wave_max(am);
    __syncthreads();
    dbl4 x = {0, 0, 0, 0};
    mma32(B, C, x);
#pragma unroll
    for (int t = 0; t < 4; ++t) A[(q_m0() + (lane >> 4) + 4 * t) * ST + q_n0() + (lane & 15)] = x[t] * 1e-3 + am * 1e-30;
    __syncthreads();
  }
  t1 = now();
  if (tid == 0) out[6] = (t1 - t0) / REPS;
  // 8: s_memtime vs s_memrealtime calibration over the whole kernel so far
  sink[tid] = acc[0] + acc[1] + acc[2] + acc[3] + v + A[tid];
}

__global__ void calib(unsigned long long* out) {
  unsigned long long t0, r0, t1, r1;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0)::"memory");
  double x = 1.0;
  for (int i = 0; i < 200000; ++i) x = x * 1.0000001 + 1e-9;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
  out[0] = t1 - t0;
  out[1] = r1 - r0;
  out[2] = (unsigned long long)x;
}

int main() {
  double *in, *sink;
  unsigned long long* out;
  hipMalloc(&in, 1024 * sizeof(double));
  hipMalloc(&sink, 256 * sizeof(double));
  hipMalloc(&out, 64 * sizeof(unsigned long long));
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (i % 17) * 0.01 - 0.08;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(out, 0, 64 * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep) bench<<<1, 256>>>(in, sink, out);
  hipDeviceSynchronize();
  unsigned long long o[64];
  hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  const char* names[] = {"mma32 regs (8 dep MFMA)", "mma32 from LDS", "barrier", "wave_max dpp",
                         "shfl max (bpermute)", "mma32+write+barrier", "NS iteration (2 mma, 2 bar)"};
  for (int i = 0; i < 7; ++i) printf("%-32s %llu cycles\n", names[i], o[i]);
  calib<<<1, 64>>>(out);
  hipDeviceSynchronize();
  hipMemcpy(o, out, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  printf("calib: memtime %llu ticks, memrealtime %llu ticks (100 MHz) -> %.3f GHz\n", o[0], o[1],
         o[0] / (o[1] / 100e6) / 1e9);
  return 0;
}
