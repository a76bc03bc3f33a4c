#include "graph_update.h"

#include <cfloat>

#include "host_distance.h"

namespace alaya_amd {
namespace {

constexpr uint32_t kNone = 0xffffffffu;

// LinearPool insert path (include/utils/query_utils.hpp:250-268): sorted by distance, equal
// distances after existing entries, reject when full and d >= last, a full pool drops its last.
struct SmallPool {
  explicit SmallPool(uint32_t cap) : cap(cap) {}
  uint32_t cap;
  std::vector<float> d;
  std::vector<uint32_t> id;
  void insert(uint32_t u, float dist) {
    if (d.size() == cap && dist >= d.back()) return;
    size_t lo = 0, hi = d.size();
    while (lo < hi) {  // find_bsearch: first position with d > dist
      const size_t mid = (lo + hi) / 2;
      if (d[mid] > dist) hi = mid;
      else lo = mid + 1;
    }
    d.insert(d.begin() + lo, dist);
    id.insert(id.begin() + lo, u);
    if (d.size() > cap) {
      d.pop_back();
      id.pop_back();
    }
  }
};

}  // namespace

std::vector<uint32_t> update_edges(const HostGraph &g, const RowMirror &m, const UpdateContext &ctx,
                                   uint32_t node) {
  std::unordered_set<uint32_t> candidate_nbrs;
  const uint32_t *cur = &g.l0[static_cast<size_t>(node) * g.R];
  for (uint32_t i = 0; i < g.R; ++i) {
    const uint32_t nbr = cur[i];
    if (nbr == kNone) break;
    if (ctx.removed_vertices.count(nbr)) {
      for (uint32_t second_hop : ctx.removed_node_nbrs.at(nbr)) candidate_nbrs.insert(second_hop);
    }
    candidate_nbrs.insert(nbr);
  }
  auto it = ctx.inserted_edges.find(node);
  if (it != ctx.inserted_edges.end()) {
    for (uint32_t inserted : it->second) candidate_nbrs.insert(inserted);
  }
  // QueryComputer(space, id): the node's stored row as the query, no normalisation
  const float *q = m.row(node);
  SmallPool pool(g.R);
  for (uint32_t nbr : candidate_nbrs) {
    const float dist = m.is_valid(nbr) ? host_dist(m.metric, q, m.row(nbr), m.dim) : FLT_MAX;
    pool.insert(nbr, dist);
  }
  std::vector<uint32_t> edges(g.R, 0u);
  for (size_t i = 0; i < pool.id.size() && i < g.R; ++i) edges[i] = pool.id[i];
  return edges;
}

void record_remove(const HostGraph &g, UpdateContext &ctx, uint32_t node) {
  const uint32_t *nbrs = &g.l0[static_cast<size_t>(node) * g.R];
  auto &rec = ctx.removed_node_nbrs[node];
  for (uint32_t i = 0; i < g.R; ++i) {
    if (nbrs[i] == kNone) break;
    rec.push_back(nbrs[i]);
  }
  ctx.removed_vertices.insert(node);
}

}  // namespace alaya_amd
