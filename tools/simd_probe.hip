// Where the dispatcher puts the waves of 4-wave workgroups (the search kernels' helper layout):
// 1024 workgroups x 4 waves, LDS sized so 4 workgroups share a CU; each wave records its hardware id
// (XCC, SE, CU, SIMD).  Prints, for the first CUs, which (workgroup, wave) runs on which SIMD.
// build: hipcc --offload-arch=gfx950 -O2 tools/simd_probe.hip -o tools/simd_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned *out, int spin) {
  extern __shared__ unsigned char smem[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  if ((threadIdx.x & 63) == 0) {
    smem[threadIdx.x >> 6] = 1;
    out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = hw;
    out[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = xcc;
  }
  // keep every workgroup resident until all have started (so the 4 per CU are concurrent)
  for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(10);
}

int main() {
  const int grid = 1024;
  unsigned *d = nullptr;
  hipMalloc(&d, grid * 4 * 2 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 38 * 1024, 0, d, 2000);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<unsigned> h(grid * 4 * 2);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::map<unsigned, std::vector<std::pair<int, int>>> cu;  // (xcc, se, sh, cu) -> (block, wave, simd)
  int same_simd_wave0 = 0, cus = 0;
  std::map<unsigned, std::vector<int>> simd_of;
  for (int b = 0; b < grid; ++b)
    for (int w = 0; w < 4; ++w) {
      const unsigned hw = h[2 * (b * 4 + w)], xcc = h[2 * (b * 4 + w) + 1] & 0xf;
      const unsigned simd = (hw >> 4) & 3, cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cuid;
      cu[key].push_back({b, static_cast<int>(w * 4 + simd)});
      if (w == 0) simd_of[key].push_back(static_cast<int>(simd));
    }
  for (auto &kv : simd_of) {
    ++cus;
    std::map<int, int> c;
    for (int s : kv.second) c[s]++;
    if (c.size() == 1 && kv.second.size() > 1) ++same_simd_wave0;
  }
  printf("CUs seen %d; CUs where every workgroup's wave 0 is on one SIMD: %d\n", cus, same_simd_wave0);
  int shown = 0;
  for (auto &kv : cu) {
    if (shown++ >= 6) break;
    printf("xcc %u se %u sh %u cu %u:", kv.first >> 16, (kv.first >> 8) & 0xff, (kv.first >> 4) & 0xf, kv.first & 0xf);
    for (auto &p : kv.second) printf(" b%d.w%d@simd%d", p.first, p.second / 4, p.second % 4);
    printf("\n");
  }
  return 0;
}
