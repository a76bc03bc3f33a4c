// Host-side HNSW graph (the index the device search traverses) and its builder.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace alaya_amd {

// Flattened HNSW graph in the layout uploaded to HBM.
//  * l0:           n x R uint32, -1 padded (Graph<>, include/index/graph/graph.hpp:65-68)
//  * levels:       per-node top level (OverlayGraph::levels_, overlay_graph.hpp:37)
//  * upper_off:    start of node u's upper lists in upper_edges; level l (>=1) list is
//                  upper_edges[upper_off[u] + (l-1)*upper_R ... + upper_R), -1 padded
//                  (OverlayGraph::lists_, overlay_graph.hpp:38-40, edges() :93-96)
//  * ep:           overlay entry point (OverlayGraph::ep_)
//  * has_overlay:  false -> NSG-style entry points `eps` (Graph::initialize_search :153-156)
struct HostGraph {
  uint64_t n = 0;          // rows stored (Graph::max_nodes_ = capacity in the reference file)
  uint32_t R = 32;
  std::vector<uint32_t> l0;
  bool has_overlay = false;
  uint32_t upper_R = 32;
  uint32_t ep = 0;
  std::vector<uint32_t> levels;
  std::vector<uint64_t> upper_off;
  std::vector<uint32_t> upper_edges;
  std::vector<uint32_t> eps;
  uint32_t max_level() const;
};

// HNSW construction with hnswlib semantics as the reference restates them
// (include/index/graph/hnsw/hnswlib.hpp:87-751, hnsw_builder.hpp:68-194): M = R/2 upper-layer
// degree, 2M level-0 degree, ef_construction = max(efc, M), std::default_random_engine seeded
// with `seed` (100 in the reference) for levels, mult = 1/ln(M), heuristic neighbour selection.
// num_threads == 1 reproduces the sequential add_point order exactly; more threads run the
// same algorithm concurrently with per-node locks (like the reference, not deterministic).
// `data` is n x dim row-major float32 (already normalised for COS).
HostGraph build_hnsw(const float *data, uint64_t n, uint32_t dim, int metric, uint32_t R,
                     uint32_t ef_construction, uint32_t num_threads, uint64_t seed);

// Per-node top levels in label order: std::default_random_engine seeded with `seed`, level =
// floor(-ln(U[0,1)) / ln(M)) (get_random_level, hnswlib.hpp:182-186).
std::vector<uint32_t> hnsw_levels(uint64_t n, uint32_t M, uint64_t seed);

// Reference on-disk format (graph.hpp:165-238 + overlay_graph.hpp:151-194 +
// sequential_storage.hpp:110-142), IDType = uint32 or uint64 (id_bytes 4 or 8).
// valid: the graph storage bitmap (bit i%8 of byte i/8; NULL = every stored node valid)
void save_graph(const HostGraph &g, const std::string &path, int id_bytes, uint64_t capacity,
                const uint8_t *valid = nullptr);
HostGraph load_graph(const std::string &path, int id_bytes);

}  // namespace alaya_amd
