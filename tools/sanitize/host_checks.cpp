// Host-side sanitizer driver (SURVEY §5 "race detection / sanitizers"): exercises the engine's host
// C++ -- the multi-threaded HNSW builder, the graph file writer/reader, the C ABI's host-only entry
// points, SQ8 training/encoding and the update job's bookkeeping -- in a binary built with
// -fsanitize=address (or thread) for the host translation units (tools/run_sanitizers.sh).  The HIP
// kernels are linked uninstrumented; no GPU is touched except alaya_device_count / index_create's
// "no device" path in the ASAN run.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/alaya_hip.h"
#include "../../alayalite_amd/csrc/graph_update.h"
#include "../../alayalite_amd/csrc/hnsw_build.h"

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                  \
    }                                                                \
  } while (0)

static std::vector<float> rows(uint64_t n, uint32_t d, uint32_t seed) {
  std::mt19937 g(seed);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  std::vector<float> v(n * d);
  for (auto &x : v) x = u(g);
  return v;
}

int main(int argc, char **argv) {
  const bool touch_hip = argc > 1 && std::string(argv[1]) == "--hip";
  const std::string tmp = argc > 2 ? argv[2] : "/tmp";
  const uint64_t n = 4000;
  const uint32_t d = 24;
  std::vector<float> data = rows(n, d, 7);

  // 1. the builder, sequential and on 8 threads (per-node locks, shared entry point), via the ABI
  for (uint32_t threads : {1u, 8u}) {
    for (int metric : {ALAYA_METRIC_L2, ALAYA_METRIC_IP, ALAYA_METRIC_L2 | ALAYA_DIST_GENERIC}) {
      alaya_graph *g = nullptr;
      CHECK(alaya_graph_build_hnsw(data.data(), n, d, metric, 32, 64, threads, 100, &g) == ALAYA_OK);
      uint64_t gn = 0, nue = 0;
      uint32_t R = 0, ur = 0, ep = 0, ml = 0, ne = 0;
      int ov = 0;
      CHECK(alaya_graph_info(g, &gn, &R, &ov, &ur, &ep, &ml, &nue, &ne) == ALAYA_OK);
      CHECK(gn == n && R == 32 && ov == 1 && ep < n);
      std::vector<uint32_t> l0(gn * R), lv(gn), ue(nue + 1), eps(1);
      std::vector<uint64_t> off(gn);
      CHECK(alaya_graph_export(g, l0.data(), lv.data(), off.data(), ue.data(), eps.data()) == ALAYA_OK);
      for (uint64_t i = 0; i < gn; ++i)
        for (uint32_t j = 0; j < R; ++j) CHECK(l0[i * R + j] == 0xffffffffu || l0[i * R + j] < gn);
      // 2. file round trip, 32- and 64-bit ids, with a validity bitmap
      std::vector<uint8_t> valid((n + 7) / 8, 0xff);
      valid[3] = 0x7f;
      for (int ib : {4, 8}) {
        const std::string path = tmp + "/san_graph_" + std::to_string(ib) + ".index";
        CHECK(alaya_graph_save(g, path.c_str(), ib, n + 100, valid.data()) == ALAYA_OK);
        alaya_graph *h = nullptr;
        CHECK(alaya_graph_load(path.c_str(), ib, &h) == ALAYA_OK);
        std::vector<uint32_t> l0b(gn * R);
        CHECK(alaya_graph_export(h, l0b.data(), nullptr, nullptr, nullptr, nullptr) == ALAYA_OK);
        CHECK(l0b == l0);
        alaya_graph_free(h);
        std::remove(path.c_str());
      }
      // 3. import of the exported arrays
      alaya_graph *imp = nullptr;
      CHECK(alaya_graph_import(gn, R, l0.data(), lv.data(), off.data(), ue.data(), nue, ur, ep, nullptr, 0, &imp) ==
            ALAYA_OK);
      alaya_graph_free(imp);
      alaya_graph_free(g);
    }
  }
  // error paths leave a message and no leak
  alaya_graph *bad = nullptr;
  CHECK(alaya_graph_load("/nonexistent/x.index", 4, &bad) != ALAYA_OK && std::strlen(alaya_last_error()) > 0);
  CHECK(alaya_graph_build_hnsw(data.data(), n, d, 7, 32, 64, 1, 100, &bad) == ALAYA_ERR_ARG);

  // 4. SQ8 training and threaded encoding
  std::vector<float> mn(d), mx(d);
  CHECK(alaya_sq8_train(data.data(), n, d, mn.data(), mx.data()) == ALAYA_OK);
  std::vector<uint8_t> codes(n * d), codes1(n * d);
  CHECK(alaya_sq8_encode(data.data(), n, d, mn.data(), mx.data(), codes.data(), 8) == ALAYA_OK);
  CHECK(alaya_sq8_encode(data.data(), n, d, mn.data(), mx.data(), codes1.data(), 1) == ALAYA_OK);
  CHECK(codes == codes1);

  // 5. the update job's host bookkeeping on a built graph
  {
    alaya_amd::HostGraph hg = alaya_amd::build_hnsw(data.data(), 600, d, 0, 32, 64, 4, 100);
    alaya_amd::RowMirror m;
    m.dim = d;
    m.rows.assign(data.begin(), data.begin() + 600 * d);
    m.valid.assign(600 / 8 + 1, 0xff);
    alaya_amd::UpdateContext ctx;
    for (uint32_t u : {3u, 40u, 41u}) {
      alaya_amd::record_remove(hg, ctx, u);
      m.valid[u >> 3] &= static_cast<uint8_t>(~(1u << (u & 7)));
    }
    ctx.inserted_edges[5].push_back(599);
    for (uint32_t u = 0; u < 600; u += 7) {
      std::vector<uint32_t> e = alaya_amd::update_edges(hg, m, ctx, u);
      CHECK(e.size() == hg.R);
    }
  }

  // 6. the device index without a device: a clean error, nothing leaked
  if (touch_hip) {
    int count = -1;
    CHECK(alaya_device_count(&count) == ALAYA_OK && count >= 0);
    alaya_index *ix = nullptr;
    if (count == 0) CHECK(alaya_index_create(0, &ix) == ALAYA_ERR_DEVICE && ix == nullptr);
  }
  std::printf("host sanitizer checks passed\n");
  return 0;
}
