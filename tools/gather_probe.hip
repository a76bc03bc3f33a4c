// Random-row gather ceilings per row size (roofline context for DESIGN.md; not part of the product).
// Each wave gathers uniformly random rows with the search kernel's load shape for that row size:
//   sift  -- 512 B f32 rows (d 128):   8 lanes per row, 4 x dwordx4 per lane, 16 rows per pass
//   sq8   -- 768 B code rows (d 768):  8 lanes per row, 24 x dword per lane,  16 rows per pass
//   gist  -- 3840 B f32 rows (d 960):  8 lanes per row, 30 x dwordx4 per lane, 24 rows per pass
// at 4, 8 and 16 waves per CU, every load of a pass in flight before the first use (as in the
// search's issue_rows / sq8_issue).  Prints GB/s of row bytes per configuration.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__device__ __forceinline__ float fold(float4 v) { return v.x + v.y + v.z + v.w; }
__device__ __forceinline__ float fold(uint32_t v) { return static_cast<float>(v & 0xffu); }

// T: the per-lane load type; kPerLane loads of T per lane per row (lane m of the row's 8 lanes reads
// elements m, m+8, ...); kRPL rows per lane group per pass.
template <typename T, int kPerLane, int kRPL>
__global__ void __launch_bounds__(64) gather_rows(const T *base, const uint32_t *ids, int rows_per_task,
                                                  int tasks, float *sink) {
  constexpr size_t kRowElems = 8 * kPerLane;
  const int lane = threadIdx.x;
  const int g = lane >> 3, m = lane & 7;
  float acc = 0.f;
  for (int t = blockIdx.x; t < tasks; t += gridDim.x) {
    const uint32_t *tid = ids + static_cast<size_t>(t) * rows_per_task;
    for (int r0 = 0; r0 < rows_per_task; r0 += 8 * kRPL) {
      T v[kRPL][kPerLane];
#pragma unroll
      for (int k = 0; k < kRPL; ++k) {
        const T *row = base + static_cast<size_t>(tid[r0 + g + 8 * k]) * kRowElems;
#pragma unroll
        for (int c = 0; c < kPerLane; ++c) v[k][c] = row[c * 8 + m];
      }
#pragma unroll
      for (int k = 0; k < kRPL; ++k)
#pragma unroll
        for (int c = 0; c < kPerLane; ++c) acc += fold(v[k][c]);
    }
  }
  if (acc == -1.2345f) *sink = acc;
}

template <typename T, int kPerLane, int kRPL>
void run(const char *name, size_t n_rows, int cus) {
  constexpr size_t row_bytes = 8 * kPerLane * sizeof(T);
  const size_t bytes = n_rows * row_bytes;
  T *base = nullptr;
  float *sink = nullptr;
  CHECK(hipMalloc(&base, bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(base, 1, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int rows_per_task = 8 * kRPL * 16;
  for (int waves_per_cu : {4, 8, 16}) {
    const int tasks = cus * waves_per_cu * 4;
    std::vector<uint32_t> h(static_cast<size_t>(tasks) * rows_per_task);
    uint64_t s = 88172645463325252ull;
    for (auto &x : h) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      x = static_cast<uint32_t>(s % n_rows);
    }
    uint32_t *ids = nullptr;
    CHECK(hipMalloc(&ids, h.size() * 4));
    CHECK(hipMemcpy(ids, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    for (int it = 0; it < 3; ++it) {
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL((gather_rows<T, kPerLane, kRPL>), dim3(cus * waves_per_cu), dim3(64), 0, 0, base, ids,
                         rows_per_task, tasks, sink);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double gb = static_cast<double>(h.size()) * row_bytes / 1e9;
      std::printf("%-5s rows=%zu row_bytes=%zu rows/pass=%d waves/CU=%2d  %.1f GB/s (%.3f ms, %.2f GB)\n", name,
                  n_rows, row_bytes, 8 * kRPL, waves_per_cu, gb * 1e3 / ms, ms, gb);
      std::fflush(stdout);
    }
    CHECK(hipFree(ids));
  }
  CHECK(hipFree(base));
  CHECK(hipFree(sink));
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  run<float4, 4, 2>("sift", 1000000, cus);      // 1M x 128 f32
  run<uint32_t, 24, 2>("sq8", 10000000, cus);   // 10M x 768 codes (config 5)
  run<float4, 30, 3>("gist", 1000000, cus);     // 1M x 960 f32
  return 0;
}
