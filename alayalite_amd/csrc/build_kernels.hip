// MI355X (gfx950) device code for HNSW construction (batched insertion; see build_kernels.h).
//
// The distance, visited set and candidate pool are the search kernel's (search_device.h): one wave
// per inserted point, the pool is a LinearPool of capacity ef_construction, so a build search is
// hnswlib's searchBaseLayer (include/index/graph/hnsw/hnswlib.hpp:373-489) with the pool standing
// in for its (candidates, top_candidates) heap pair -- both stop once no unexpanded candidate is
// closer than the ef-th best.  Ties on the distance are ordered by arrival (the reference leaves
// them to its heap).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <cstdint>

#include "build_kernels.h"
#include "search_device.h"

namespace alaya_amd {

namespace {

constexpr uint64_t kNoEdge = ~0ull;
constexpr uint32_t kApplyCap = 128;  // candidates held at once when a list is pruned

__device__ __forceinline__ uint32_t level_width(const SearchParams &p, int level) {
  return level == 0 ? p.R : p.upper_R;
}

// adjacency row of u at `level` (level 0: Graph rows; above: OverlayGraph lists)
__device__ __forceinline__ uint64_t adj_offset(const SearchParams &p, uint32_t u, int level) {
  return level == 0 ? static_cast<uint64_t>(u) * p.R
                    : p.upper_off[u] + static_cast<uint64_t>(level - 1) * p.upper_R;
}

__device__ __forceinline__ const uint32_t *adj_row(const SearchParams &p, uint32_t u, int level) {
  return (level == 0 ? p.l0 : p.upper_edges) + adj_offset(p, u, level);
}

__device__ __forceinline__ uint32_t *adj_row_w(const BuildParams &bp, uint32_t u, int level) {
  return (level == 0 ? bp.l0w : bp.upw) + adj_offset(bp.s, u, level);
}

// number of ids before the first -1 of a row of width w (w <= 64)
__device__ __forceinline__ uint32_t row_count(uint32_t v, uint32_t w) {
  const int lane = lane_id();
  const uint64_t endm = ballot(lane < static_cast<int>(w) && v == kEmpty);
  return endm ? static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(endm)) - 1) : w;
}

// copy base row `id` into the LDS vector q (rows are zero padded to the stride)
__device__ __forceinline__ void stage_row(const SearchParams &p, uint32_t id, float *q) {
  const float4 *src = reinterpret_cast<const float4 *>(p.base + static_cast<uint64_t>(id) * p.stride);
  float4 *dst = reinterpret_cast<float4 *>(q);
  for (uint32_t e = lane_id(); e < p.stride / 4; e += 64) dst[e] = src[e];
  wave_sync();
}

// getNeighborsByHeuristic2 (hnswlib.hpp:291-354) over candidates sorted by ascending distance to
// the base point: keep a candidate unless an already kept one is closer to it than the base point
// is (dist(kept, cand) < dist(base, cand)); stop at m kept.  Fewer than m candidates: keep all
// (:296-298).  Returns the number kept; sel_i/sel_d (LDS, >= m entries) hold them in ascending
// order.  tmp is an LDS scratch of >= m floats.
template <bool kIP, int kChunks>
__device__ uint32_t heuristic(const SearchParams &p, const uint32_t *ci, const float *cd, uint32_t C,
                              uint32_t m, uint32_t *sel_i, float *sel_d, float *tmp, uint32_t *n_dist) {
  const int lane = lane_id();
  if (C < m) {
    for (uint32_t j = lane; j < C; j += 64) {
      sel_i[j] = ci[j];
      sel_d[j] = cd[j];
    }
    wave_sync();
    return C;
  }
  uint32_t nsel = 0;
  for (uint32_t i = 0; i < C && nsel < m; ++i) {
    const uint32_t c = ci[i];
    const float dc = cd[i];
    bool good = true;
    if (nsel > 0) {
      // the candidate's row is read straight from global memory (L2) by every row group, issued
      // together with the kept rows' loads: one round trip per candidate instead of a staging
      // copy into LDS first
      row_distances<kIP, kChunks>(p, p.base + static_cast<uint64_t>(c) * p.stride, sel_i, static_cast<int>(nsel), tmp);
      good = ballot(lane < static_cast<int>(nsel) && tmp[lane] < dc) == 0;
      *n_dist += nsel;
      wave_sync();
    }
    if (good) {
      if (lane == 0) {
        sel_i[nsel] = c;
        sel_d[nsel] = dc;
      }
      ++nsel;
      wave_sync();
    }
  }
  return nsel;
}

// ---------------------------------------------------------------------------------------------
// 1. candidate search for every active point (persistent one-wave workgroups)
// ---------------------------------------------------------------------------------------------
template <bool kIP, int kChunks>
__global__ void __launch_bounds__(64) build_search_kernel(BuildParams bp) {
  const SearchParams &p = bp.s;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  Lds L;
  {
    unsigned char *ptr = smem;
    L.q = reinterpret_cast<float *>(ptr);
    ptr += static_cast<size_t>(p.stride) * 4;
    L.cid = reinterpret_cast<uint32_t *>(ptr);
    ptr += 64 * 4;
    L.cd = reinterpret_cast<float *>(ptr);
    ptr += 64 * 4;
    L.sd = reinterpret_cast<float *>(ptr);
    ptr += 64 * 4;
    L.pd = reinterpret_cast<float *>(ptr);
    ptr += ((p.ef + 1) * 4 + 15) / 16 * 16;
    L.pi = reinterpret_cast<uint32_t *>(ptr);
    ptr += ((p.ef + 1) * 4 + 15) / 16 * 16;
    L.hash = reinterpret_cast<uint32_t *>(ptr);
    L.sq_scale = nullptr;
    L.sq_min = nullptr;
  }
  const uint32_t hsize = 1u << p.hash_log2;
  const uint64_t bit_words = (p.n + 31) / 32;
  uint32_t *slot_bits = p.overflow_bits + static_cast<uint64_t>(blockIdx.x) * bit_words;
  uint32_t *slot_dirty = p.dirty_words + static_cast<uint64_t>(blockIdx.x) * p.dirty_cap;
  const uint32_t W = level_width(p, bp.level);

  for (;;) {
    uint32_t qi = 0;
    if (lane == 0) qi = atomicAdd(p.work_counter, 1u);
    qi = read_lane(qi, 0);
    if (qi >= p.nq) break;
    const uint32_t pt = bp.pts[qi];
    stage_row(p, pt, L.q);
    {
      const bool wide = p.vis_rbits == kVisWide;
      const uint32_t words = wide ? hsize : hsize / 2;
      for (uint32_t e = lane; e < words; e += 64) L.hash[e] = wide ? kEmpty : 0u;
    }
    for (uint32_t e = lane; e <= p.ef; e += 64) {
      L.pd[e] = 0.f;
      L.pi[e] = 0u;
    }
    wave_sync();
    Visited vs = make_visited(p, L.hash, slot_bits, slot_dirty);
    PoolState ps{0u, 0u, p.ef};

    // entry: the point's first searched level starts from the greedy descent, lower levels from
    // the closest neighbour selected one level up (hnswlib.hpp:694-737)
    const int top = min(static_cast<int>(p.levels[pt]), bp.max_level);
    const bool descend = top == bp.level && !bp.refine;
    uint32_t u = descend ? p.ep : bp.next[pt - bp.batch_first];
    if (lane == 0) L.cid[0] = u;
    wave_sync();
    row_distances<kIP, kChunks>(p, L.q, L.cid, 1, L.cd);
    float cur = L.cd[0];
    if (descend) {
      for (int level = bp.max_level; level > bp.level; --level) {
        bool changed = true;
        while (changed) {
          changed = false;
          const uint32_t *list = adj_row(p, u, level);
          const uint32_t v = lane < static_cast<int>(p.upper_R) ? list[lane] : kEmpty;
          const int cnt = static_cast<int>(row_count(v, p.upper_R));
          wave_sync();
          if (lane < cnt) L.cid[lane] = v;
          wave_sync();
          row_distances<kIP, kChunks>(p, L.q, L.cid, cnt, L.cd);
          // first index of the minimum == the sequential strict-'<' scan (hnswlib.hpp:705-712)
          const bool has = lane < cnt;
          const float dl = has ? L.cd[lane] : FLT_MAX;
          float mn = dl;
          for (int off = 32; off > 0; off >>= 1) mn = fminf(mn, __shfl_xor(mn, off));
          const uint64_t at = ballot(has && dl == mn);
          if (at && mn < cur) {
            u = read_lane(v, __ffsll(static_cast<unsigned long long>(at)) - 1);
            cur = mn;
            changed = true;
          }
          wave_sync();
        }
      }
    }
    if (lane == 0) {
      L.pd[0] = cur;
      L.pi[0] = u;
    }
    ps.size = 1;
    visit(vs, u, lane == 0);
    // the point itself is reachable in a refine pass: never a candidate of its own
    if (u != pt) visit(vs, pt, lane == 0);
    wave_sync();

    while (ps.cur < ps.size) {
      const uint32_t x = pool_pop(ps, L);
      const uint32_t *row = adj_row(p, x, bp.level);
      const uint32_t v = lane < static_cast<int>(W) ? row[lane] : kEmpty;
      const int cnt = static_cast<int>(row_count(v, W));
      const bool act = lane < cnt;
      if (!vs.spilled && vs.count + 64 > vs.limit) spill_begin(vs);
      const bool fresh = visit(vs, v, act);
      const uint64_t fm = ballot(fresh);
      const int nf = __popcll(fm);
      if (nf == 0) continue;
      const uint32_t slot = __popcll(fm & ((1ull << lane) - 1ull));
      if (fresh) L.cid[slot] = v;
      wave_sync();
      row_distances<kIP, kChunks>(p, L.q, L.cid, nf, L.cd);
      const bool has = lane < nf;
      const uint32_t cid = has ? L.cid[lane] : 0u;
      const float cd = has ? L.cd[lane] : 0.f;
      wave_sync();
      pool_merge(ps, L, has, cid, cd);
    }
    for (uint32_t i = lane; i < ps.size; i += 64) {
      bp.cand_ids[static_cast<uint64_t>(qi) * p.ef + i] = L.pi[i] & kIdMask;
      bp.cand_d[static_cast<uint64_t>(qi) * p.ef + i] = L.pd[i];
    }
    if (lane == 0) bp.cand_n[qi] = ps.size;
    visit_end(vs);
    wave_sync();
  }
}

// ---------------------------------------------------------------------------------------------
// 2. neighbour selection for the new points + reverse edges
// ---------------------------------------------------------------------------------------------
template <bool kIP, int kChunks>
__global__ void __launch_bounds__(64) build_select_kernel(BuildParams bp) {
  const SearchParams &p = bp.s;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *sel_i = reinterpret_cast<uint32_t *>(smem);
  float *sel_d = reinterpret_cast<float *>(sel_i + 64);
  float *tmp = sel_d + 64;
  const int lane = lane_id();
  const uint32_t W = level_width(p, bp.level);
  uint32_t n_dist = 0;
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    const uint32_t pt = bp.pts[qi];
    const uint32_t C = bp.cand_n[qi];
    const uint32_t nsel = heuristic<kIP, kChunks>(p, bp.cand_ids + qi * p.ef, bp.cand_d + qi * p.ef, C, bp.M,
                                                  sel_i, sel_d, tmp, &n_dist);
    // own list in the max-heap pop order: farthest first (hnswlib.hpp:527-551)
    uint32_t *row = adj_row_w(bp, pt, bp.level);
    for (uint32_t j = lane; j < W; j += 64) row[j] = j < nsel ? sel_i[nsel - 1 - j] : kEmpty;
    if (lane == 0) bp.next[pt - bp.batch_first] = nsel ? sel_i[0] : p.ep;
    for (uint32_t j = lane; j < bp.M; j += 64) {
      bp.edge_keys[qi * bp.M + j] = j < nsel ? (static_cast<uint64_t>(sel_i[j]) << 32) | pt : kNoEdge;
      bp.edge_d[qi * bp.M + j] = j < nsel ? sel_d[j] : 0.f;
    }
    wave_sync();
  }
  if (bp.counters && lane == 0 && n_dist) atomicAdd(&bp.counters[2], static_cast<unsigned long long>(n_dist));
}

// ---------------------------------------------------------------------------------------------
// 3. reverse edges: one wave per destination segment of the sorted edge list
// ---------------------------------------------------------------------------------------------
template <bool kIP, int kChunks>
__device__ void apply_segment(const BuildParams &bp, uint64_t s, unsigned char *smem, uint32_t *n_dist,
                              uint32_t *n_prune, uint32_t *n_append) {
  const SearchParams &p = bp.s;
  const int lane = lane_id();
  uint32_t *li = reinterpret_cast<uint32_t *>(smem);  // list in row order
  float *ld = reinterpret_cast<float *>(li + kApplyCap);
  uint32_t *si = reinterpret_cast<uint32_t *>(ld + kApplyCap);  // sorted candidates
  float *sdd = reinterpret_cast<float *>(si + kApplyCap);
  uint32_t *sel_i = reinterpret_cast<uint32_t *>(sdd + kApplyCap);
  float *sel_d = reinterpret_cast<float *>(sel_i + 64);
  float *tmp = sel_d + 64;

  const uint32_t v = static_cast<uint32_t>(bp.edge_keys[s] >> 32);
  uint64_t e = s;  // segment end
  for (;;) {
    const uint64_t i = e + lane;
    const bool same = i < bp.n_edges && bp.edge_keys[i] != kNoEdge &&
                      static_cast<uint32_t>(bp.edge_keys[i] >> 32) == v;
    const uint64_t m = ballot(same);
    if (~m == 0ull) {
      e += 64;
      continue;
    }
    e += static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(~m)) - 1);
    break;
  }
  uint32_t *row = adj_row_w(bp, v, bp.level);
  const uint32_t W = level_width(p, bp.level);
  const uint32_t rv = lane < static_cast<int>(W) ? row[lane] : kEmpty;
  uint32_t c = row_count(rv, W);
  if (lane < static_cast<int>(c)) li[lane] = rv;
  wave_sync();
  // distances of the existing list to v, needed once a prune is possible
  if (c + (e - s) > bp.Mmax) {
    row_distances<kIP, kChunks>(p, p.base + static_cast<uint64_t>(v) * p.stride, li, static_cast<int>(c), ld);
    *n_dist += c;
  }
  bool pruned = false;
  uint32_t appended = 0;
  for (uint64_t pos = s; pos < e; pos += 64) {
    // incoming points not already listed (a refine pass re-proposes edges), appended in point order
    const uint64_t i = pos + lane;
    const bool in = i < e;
    const uint32_t u = in ? static_cast<uint32_t>(bp.edge_keys[i]) : kEmpty;
    bool fresh = in;
    for (uint32_t k = 0; k < c && fresh; ++k) fresh = li[k] != u;
    const uint64_t fm = ballot(fresh);
    const uint32_t slot = c + __popcll(fm & ((1ull << lane) - 1ull));
    wave_sync();
    if (fresh) {
      li[slot] = u;
      ld[slot] = bp.edge_d[i];
    }
    wave_sync();
    c += __popcll(fm);
    appended += __popcll(fm);
    if (c <= bp.Mmax) continue;
    // prune (hnswlib.hpp:590-626): rank sort by (distance, id) -- ids are distinct -- then the heuristic
    for (uint32_t j = lane; j < c; j += 64) {
      const float dj = ld[j];
      const uint32_t ij = li[j];
      uint32_t r = 0;
      for (uint32_t k = 0; k < c; ++k) {
        const float dk = ld[k];
        r += (dk < dj || (dk == dj && li[k] < ij)) ? 1u : 0u;
      }
      si[r] = ij;
      sdd[r] = dj;
    }
    wave_sync();
    const uint32_t nsel = heuristic<kIP, kChunks>(p, si, sdd, c, bp.Mmax, sel_i, sel_d, tmp, n_dist);
    // pruned list in the max-heap pop order: farthest first (hnswlib.hpp:617-626)
    for (uint32_t j = lane; j < nsel; j += 64) {
      li[j] = sel_i[nsel - 1 - j];
      ld[j] = sel_d[nsel - 1 - j];
    }
    wave_sync();
    c = nsel;
    pruned = true;
  }
  if (appended) {
    for (uint32_t j = lane; j < W; j += 64) row[j] = j < c ? li[j] : kEmpty;
  }
  if (lane == 0) {
    *n_prune += pruned ? 1u : 0u;
    *n_append += pruned ? 0u : appended;
  }
  wave_sync();
}

template <bool kIP, int kChunks>
__global__ void __launch_bounds__(64) build_apply_kernel(BuildParams bp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = lane_id();
  uint32_t n_dist = 0, n_prune = 0, n_append = 0;
  for (uint64_t b = static_cast<uint64_t>(blockIdx.x) * 64; b < bp.n_edges; b += static_cast<uint64_t>(gridDim.x) * 64) {
    const uint64_t i = b + lane;
    const uint64_t key = i < bp.n_edges ? bp.edge_keys[i] : kNoEdge;
    const uint64_t prev = (i > 0 && i < bp.n_edges) ? bp.edge_keys[i - 1] : kNoEdge;
    const bool head = key != kNoEdge && (i == 0 || (prev >> 32) != (key >> 32) || prev == kNoEdge);
    uint64_t heads = ballot(head);
    while (heads) {
      const int h = __ffsll(static_cast<unsigned long long>(heads)) - 1;
      heads &= heads - 1;
      apply_segment<kIP, kChunks>(bp, b + h, smem, &n_dist, &n_prune, &n_append);
    }
  }
  if (bp.counters && lane == 0) {
    if (n_prune) atomicAdd(&bp.counters[0], static_cast<unsigned long long>(n_prune));
    if (n_append) atomicAdd(&bp.counters[1], static_cast<unsigned long long>(n_append));
    if (n_dist) atomicAdd(&bp.counters[2], static_cast<unsigned long long>(n_dist));
  }
}

// d = 128 / 768 / 960 specialised (the benchmark shapes), every other d runs the generic kernel
#define ALAYA_BUILD_CHUNKS(X) X(4) X(24) X(30)

template <bool kIP, int kChunks>
const void *search_ptr() { return reinterpret_cast<const void *>(&build_search_kernel<kIP, kChunks>); }
template <bool kIP, int kChunks>
const void *select_ptr() { return reinterpret_cast<const void *>(&build_select_kernel<kIP, kChunks>); }
template <bool kIP, int kChunks>
const void *apply_ptr() { return reinterpret_cast<const void *>(&build_apply_kernel<kIP, kChunks>); }

enum class Which { kSearch, kSelect, kApply };

template <int C>
const void *sym(Which w, bool ip) {
  switch (w) {
    case Which::kSearch: return ip ? search_ptr<true, C>() : search_ptr<false, C>();
    case Which::kSelect: return ip ? select_ptr<true, 0>() : select_ptr<false, 0>();
    default: return ip ? apply_ptr<true, 0>() : apply_ptr<false, 0>();
  }
}

// The search kernel is specialised on d (all row chunks of a pass in flight); the selection and
// apply kernels compare a row with <= 32 others per step and are latency-bound, so they take the
// generic distance loop (~100 VGPRs instead of ~400) for more resident waves.
const void *kernel_for(Which w, const SearchParams &p) {
  const uint32_t chunks = (!p.generic && p.dim % 32 == 0) ? p.dim / 32 : 0;
#define ALAYA_CASE(C) \
  if (chunks == C) return sym<C>(w, p.ip);
  ALAYA_BUILD_CHUNKS(ALAYA_CASE)
#undef ALAYA_CASE
  return sym<0>(w, p.ip);
}

size_t select_lds(uint32_t) { return 3 * 64 * 4; }
size_t apply_lds(uint32_t) { return 4 * kApplyCap * 4 + 3 * 64 * 4; }

hipError_t launch(Which w, const BuildParams &p, int grid, size_t lds, hipStream_t stream) {
  BuildParams arg = p;
  void *args[] = {&arg};
  return hipLaunchKernel(kernel_for(w, p.s), dim3(grid), dim3(64), args, lds, stream);
}

}  // namespace

size_t build_lds_bytes(uint32_t stride, uint32_t ef, uint32_t hash_log2, bool compact) {
  return search_wave_lds_bytes(stride, ef, hash_log2, compact);
}

hipError_t build_search_occupancy(const BuildParams &p, size_t lds, int *blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, kernel_for(Which::kSearch, p.s), 64, lds);
}

hipError_t launch_build_search(const BuildParams &p, int grid, size_t lds, hipStream_t stream) {
  return launch(Which::kSearch, p, grid, lds, stream);
}

hipError_t launch_build_select(const BuildParams &p, int grid, hipStream_t stream) {
  return launch(Which::kSelect, p, grid, select_lds(p.s.stride), stream);
}

hipError_t launch_build_apply(const BuildParams &p, int grid, hipStream_t stream) {
  return launch(Which::kApply, p, grid, apply_lds(p.s.stride), stream);
}

hipError_t sort_edges(void *tmp, size_t *tmp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                      const float *d_in, float *d_out, uint64_t n, hipStream_t stream) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys_in, keys_out, d_in, d_out,
                                            static_cast<int>(n), 0, 64, stream);
}

}  // namespace alaya_amd
