// HBM calibration probe for the roofline discussion in DESIGN.md (not part of the product).
// (1) sequential stream read of a large buffer, (2) random gathers of whole rows of `row_bytes`
// with the search kernel's load shape (8 lanes per row, dwordx4, all rows of a pass in flight).
// Prints GB/s for each.  Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void __launch_bounds__(256) stream_read(const float4 *p, size_t n4, float *sink) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += static_cast<size_t>(gridDim.x) * 256) {
    const float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == -1.2345f) *sink = acc;
}

// one wave per task; each pass gathers 24 rows (8 lanes per row, kRPL rows per lane group)
template <int kVecPerRow>
__global__ void __launch_bounds__(64) gather_rows(const float4 *base, const uint32_t *ids, int rows_per_task,
                                                  int tasks, size_t row_vecs, float *sink) {
  const int lane = threadIdx.x;
  const int g = lane >> 3, m = lane & 7;
  float acc = 0.f;
  for (int t = blockIdx.x; t < tasks; t += gridDim.x) {
    const uint32_t *tid = ids + static_cast<size_t>(t) * rows_per_task;
    for (int r0 = 0; r0 < rows_per_task; r0 += 24) {
      float4 v[3][kVecPerRow / 8];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float4 *row = base + static_cast<size_t>(tid[r0 + g + 8 * k]) * row_vecs;
#pragma unroll
        for (int c = 0; c < kVecPerRow / 8; ++c) v[k][c] = row[c * 8 + m];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int c = 0; c < kVecPerRow / 8; ++c) acc += v[k][c].x + v[k][c].y + v[k][c].z + v[k][c].w;
    }
  }
  if (acc == -1.2345f) *sink = acc;
}

int main(int argc, char **argv) {
  const size_t n_rows = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  constexpr int kVec = 240;  // 960 floats = 3840 B
  const size_t row_vecs = kVec;
  const size_t bytes = n_rows * row_vecs * 16;
  float4 *base = nullptr;
  float *sink = nullptr;
  CHECK(hipMalloc(&base, bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(base, 0, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // (1) stream
  for (int it = 0; it < 3; ++it) {
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(stream_read, dim3(cus * 8), dim3(256), 0, 0, base, bytes / 16, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::printf("stream_read   %.1f GB/s (%.3f ms, %.2f GB)\n", bytes / (ms * 1e6), ms, bytes / 1e9);
  }
  // (2) random row gathers: tasks x 24*P rows each
  const int rows_per_task = 24 * 16;
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
      hipLaunchKernelGGL(gather_rows<kVec>, dim3(cus * waves_per_cu), dim3(64), 0, 0, base, ids, rows_per_task,
                         tasks, row_vecs, sink);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double gb = static_cast<double>(h.size()) * row_vecs * 16 / 1e9;
      std::printf("gather_rows   waves/CU=%2d  %.1f GB/s (%.3f ms, %.2f GB)\n", waves_per_cu, gb * 1e3 / ms, ms, gb);
    }
    CHECK(hipFree(ids));
  }
  CHECK(hipFree(base));
  return 0;
}
