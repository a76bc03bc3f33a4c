// Launch interface of the device HNSW construction kernels (build_kernels.hip).
//
// The device build inserts points in label order in batches.  For one batch and one level L, the
// host (capi.cpp, alaya_index_build_graph) launches:
//   1. build_search   -- per inserted point: greedy descent from the entry point through the levels
//                        above L (hnswlib.hpp:684-705), then a best-first search of level L with a
//                        pool of ef_construction (searchBaseLayer, :373-489) -> candidate pool;
//   2. build_select   -- getNeighborsByHeuristic2 (:291-354) keeps M of the candidates; the point's
//                        list at L is written in the heap's pop order (farthest first, :523-530) and
//                        one reverse edge (neighbour, point, distance) is emitted per selection;
//   3. sort_edges     -- radix sort of the reverse edges by (neighbour, point);
//   4. build_apply    -- per neighbour: append the incoming points while the list has room, else
//                        prune (existing + incoming) with the same heuristic to Mmax (:561-628).
// Points of one batch do not see each other during these searches.  A refine pass then repeats
// 1-4 on level 0 for the batch: the batch's points are now in the graph (reverse edges of step 4),
// so each point re-selects its neighbours among old points and batch mates alike; apply skips
// edges a list already holds.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "search_kernels.h"

namespace alaya_amd {

struct BuildParams {
  // rows, adjacency (l0 / overlay with upper_off + upper_R), ep, ef = ef_construction, visited-set
  // sizing and scratch: the same fields a search launch uses.  s.nq = number of active points.
  SearchParams s;
  uint32_t *l0w;             // writable views of s.l0 / s.upper_edges
  uint32_t *upw;
  const uint32_t *pts;       // active points of this level (row ids)
  uint32_t batch_first;      // first row id of the batch (index into next[])
  int level;                 // level searched / connected by this launch
  int max_level;             // graph's max level before the batch (descent starts at s.ep)
  int refine;                // refine pass: every point starts from next[] (its closest neighbour)
  uint32_t *next;            // batch-local: closest selected neighbour = entry for the next level
  uint32_t *cand_ids;        // nq x ef candidate pool (ascending distance)
  float *cand_d;
  uint32_t *cand_n;          // nq pool sizes
  uint32_t M;                // neighbours selected for a new point (M_)
  uint32_t Mmax;             // list capacity at this level (maxM0_ on level 0, maxM_ above)
  uint64_t *edge_keys;       // nq x M: (neighbour << 32) | point, ~0 = unused (sorted in place)
  float *edge_d;             // nq x M: dist(point, neighbour)
  uint64_t n_edges;          // apply: edge slots (nq x M)
  unsigned long long *counters;  // optional: [0] prunes, [1] appends, [2] heuristic distances
};

size_t build_lds_bytes(uint32_t stride, uint32_t ef, uint32_t hash_log2, bool compact);
hipError_t build_search_occupancy(const BuildParams &p, size_t lds, int *blocks_per_cu);
hipError_t launch_build_search(const BuildParams &p, int grid, size_t lds, hipStream_t stream);
hipError_t launch_build_select(const BuildParams &p, int grid, hipStream_t stream);
hipError_t launch_build_apply(const BuildParams &p, int grid, hipStream_t stream);
// Radix sort of (key, dist) pairs, keys ascending.  tmp == nullptr: *tmp_bytes = scratch needed.
hipError_t sort_edges(void *tmp, size_t *tmp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                      const float *d_in, float *d_out, uint64_t n, hipStream_t stream);

}  // namespace alaya_amd
