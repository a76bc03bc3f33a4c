// Online updates of a device-resident HNSW index: the host half (graph bookkeeping) of
// GraphUpdateJob (include/executor/jobs/graph_update_job.hpp:49-137).  The device half is the
// search that picks a new node's edges (search_solo, graph_search_job.hpp:302-335, run by the
// search kernel) and the patches that mirror each change into HBM (capi.cpp).
#pragma once
#include <cstdint>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "hnsw_build.h"

namespace alaya_amd {

// JobContext (include/executor/jobs/job_context.hpp:25-29).  The same libstdc++ containers with
// the same insertion sequences as the reference, so every iteration order -- and therefore the
// LinearPool tie order in update() -- is the reference's.
struct UpdateContext {
  std::unordered_map<uint32_t, std::vector<uint32_t>> inserted_edges;
  std::unordered_set<uint32_t> removed_vertices;
  std::unordered_map<uint32_t, std::vector<uint32_t>> removed_node_nbrs;
};

// Host mirror of what the updates read: rows (n x dim f32, as RawSpace stores them) and the
// validity bitmap (SequentialStorage::bitmap_, bit i%8 of byte i/8).
struct RowMirror {
  std::vector<float> rows;
  std::vector<uint8_t> valid;
  uint32_t dim = 0;
  int metric = 0;
  bool is_valid(uint32_t id) const { return (valid[id >> 3] >> (id & 7)) & 1u; }
  const float *row(uint32_t id) const { return rows.data() + static_cast<size_t>(id) * dim; }
};

// GraphUpdateJob::update(node_id) (graph_update_job.hpp:105-137): candidates = current edges,
// plus the stored neighbours of removed neighbours, plus edges inserted towards the node; each
// scored from the node's own row (RawSpace::QueryComputer(id), FLT_MAX for removed rows) into a
// LinearPool of capacity R.  Returns the new R edges: the pool ids, then zeros (the reference's
// value-initialised updated_edges vector, not -1).
std::vector<uint32_t> update_edges(const HostGraph &g, const RowMirror &m, const UpdateContext &ctx,
                                   uint32_t node);

// GraphUpdateJob::remove(node_id) bookkeeping (:91-103): record the node's edges up to the first
// -1 and mark it removed.  The caller clears the validity bit (RawSpace::remove).
void record_remove(const HostGraph &g, UpdateContext &ctx, uint32_t node);

}  // namespace alaya_amd
