#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <set>
__global__ void k(unsigned* out) {
  unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID (id 4), offset 0, size 32
  unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID (id 20), 16 bits
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
  __builtin_amdgcn_s_sleep(100);
}
int main() {
  const int n = 4096;
  unsigned* d; hipMalloc(&d, n * 8);
  hipLaunchKernelGGL(k, dim3(n), dim3(256), 0, 0, d);
  unsigned h[2 * n]; hipMemcpy(h, d, n * 8, hipMemcpyDeviceToHost);
  std::map<unsigned, std::set<unsigned>> cus;  // xcc -> set of (se,sh,cu)
  std::map<unsigned,int> cuid_hist, se_hist, sh_hist;
  for (int i = 0; i < n; ++i) {
    unsigned hw = h[2*i], x = h[2*i+1] & 0xF;
    unsigned cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cus[x].insert((se << 8) | (sh << 4) | cu);
    cuid_hist[cu]++; se_hist[se]++; sh_hist[sh]++;
  }
  for (auto& [x, s] : cus) { printf("xcc %u: %zu CUs:", x, s.size()); for (auto v : s) printf(" %u.%u.%u", v >> 8, (v >> 4) & 1, v & 15); printf("\n"); }
  printf("cu_id hist:"); for (auto& [a,b]: cuid_hist) printf(" %u:%d", a, b); printf("\nse hist:"); for (auto& [a,b]: se_hist) printf(" %u:%d", a, b);
  printf("\nsh hist:"); for (auto& [a,b]: sh_hist) printf(" %u:%d", a, b); printf("\nblock0 xcc %u block1 xcc %u block8 xcc %u\n", h[1]&15, h[3]&15, h[17]&15);
  return 0;
}
