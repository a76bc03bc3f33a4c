// Launch interface between the C-ABI layer (capi.cpp) and the device code (search_kernels.hip).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace alaya_amd {

// Everything one search launch reads or writes.  All pointers are device pointers.
struct SearchParams {
  // base rows (RawSpace storage): n rows of `stride` floats, first `dim` used, zero padded
  const float *base;
  uint64_t n;
  uint32_t dim;
  uint32_t stride;        // multiple of 32 floats (128 B rows, 16 B aligned float4 loads)
  const uint32_t *valid;  // SequentialStorage validity bitmap as 32-bit words; nullptr = all valid
  bool ip;                // IP / COS (negated inner product) vs L2
  bool generic;           // non-float DataType: generic l2_sqr<T>/ip_sqr<T> order (one accumulator,
                          // elements in order; distance_l2.ipp:735-741), not the AVX2 float order
  // level-0 adjacency (Graph), n x R, -1 padded
  const uint32_t *l0;
  uint32_t R;
  bool dedup_edges;       // some row repeats an id: drop later occurrences in-kernel
  // overlay (OverlayGraph); levels == nullptr -> NSG-style entry points
  const uint32_t *levels;
  const uint64_t *upper_off;
  const uint32_t *upper_edges;
  uint32_t upper_R;
  uint32_t ep;
  const uint32_t *eps;
  uint32_t n_eps;
  // batch
  const float *queries;   // nq rows of q_stride floats
  uint64_t nq;
  uint32_t q_stride;
  uint32_t k;
  uint32_t ef;
  uint32_t *out_ids;      // nq x k
  float *out_dists;       // nq x k (nullable)
  uint32_t *out_counters; // nq x 4 (n_dist, n_expand, n_dist_upper, n_hops_upper), nullable
  uint32_t fill_id;       // id written for result slots past the pool (0 = reference behaviour, with
                          // distance 0.0; 0xffffffff = empty slot, with distance FLT_MAX)
  // scratch
  uint32_t *work_counter; // zeroed before each launch
  uint32_t *overflow_bits;// grid x ceil(n/32) words: visited-set spill area, all zero between queries
  uint32_t *dirty_words;  // slots x dirty_cap: per-slot list of the spill-area words a query set
  uint32_t dirty_cap;
  uint32_t wave_lds;      // bytes of one wave's LDS region (search_wave_lds_bytes)
  uint32_t hash_log2;     // LDS visited table = 1 << hash_log2 slots
  // visited-table layout: kVisWide = 32-bit id slots; otherwise 16-bit compact slots holding
  // (probe distance, low vis_rbits bits of a vis_lbits-bit bijective hash) -- exact either way
  uint32_t vis_rbits;
  uint32_t vis_lbits;
  uint32_t vis_max_disp;  // compact: largest probe distance an entry may sit at (<= 0xffff >> rbits - 1)
  uint32_t vis_limit;     // LDS table entries before a query spills to the second level (0 = the
                          // layout's default: half the slots wide, 11/16 compact); <= slots - 64
  // Spill table (stab_log2 != 0): the second level is a per-slot hash table of 2^stab_log2 16-bit
  // entries in buckets of 8 (16 B), all zero between queries, instead of the N-bit bitset; the bitset
  // stays as a third level for the (rare) ids whose home bucket is full.  An entry is 1 + the low
  // stab_rbits bits of the vis_lbits-bit bijective hash, whose top bits are the bucket.
  uint16_t *spill_table;  // slots x 2^stab_log2 entries
  uint32_t stab_log2;
  uint32_t stab_rbits;    // <= 15
  uint32_t spill_flags;   // diagnostics (ALAYA_SPILL_FLAGS): bit 0 = no second-level prefetch, bit 2 =
                          // prefetch after the rows land, bit 8 = the prefetch-check kernel (kDiag 2)
  uint64_t *stamps;       // nullable: diagnostic per-phase cycle counts, nq x 8
  // SQ8 search space (SQ8Space, space/sq8_space.hpp): traversal distances on uint8 codes
  int sq8_order;          // 0 = f32 RawSpace search; 2 = AVX-512 SQ8 order; 1 = AVX2 SQ8 order
  const uint8_t *codes;   // n rows of code_stride bytes (16 B aligned)
  uint32_t code_stride;
  const float *sq_min;    // per-dimension min / max of SQ8Quantizer (sq8.hpp:99-113)
  const float *sq_max;
  // distance helpers (search_has_helpers): 1 = a wave with no query left computes its workgroup
  // siblings' next distances into an LDS memo (kHelpBoardBytes after the wave regions); help_flags
  // are diagnostics (ALAYA_HELP_FLAGS bit 0 = no visited hint: helpers compute every claimed row;
  // bit 1 = the hint in the f32 kernels too -- by default only the SQ8 kernels use it)
  uint32_t help;
  uint32_t help_flags;
  uint32_t memo_off;      // byte offset of a helper's memo in its wave region (0: the query vector)
  uint32_t two_waves;     // 1 = the wide-row f32 kernel at two waves per SIMD (one row per lane group):
                          // twice the resident searchers, each with half the rows in flight
  uint32_t *help_stats;   // nullable: per searcher, (fresh distances it took from a memo, expansions
                          // with every fresh distance from the memo, rows it computed as a helper)
};

// PyIndex::rerank inputs (python/include/index.hpp:450-488).  Per query the kernel rescores
// search_ids[0 .. n_take) (row stride n_src; kEmpty entries are skipped) plus `zeros` entries of id 0
// -- the reference's res_pool slots [k, ef) that batch_search leaves zero (index.hpp:301) -- and
// returns the k smallest pair<dist, id>.
//   reference mode:  n_take = min(k, ef), zeros = ef - k, fill_id = 0
//   corrected mode:  n_take = ef (the whole pool, kEmpty past it), zeros = 0, fill_id = 0
//   shard mode:      n_take = min(k, ef); zeros = ef - k only on the shard that holds global row 0,
//                    else 0; fill_id = kEmpty (see alaya_index_shard_search_sq8_device)
struct RerankParams {
  const uint32_t *search_ids;  // nq x n_src ids written by the SQ8 search
  uint32_t k;
  uint32_t n_src;              // ids per query row of search_ids
  uint32_t n_take;             // ids rescored per query (<= n_src)
  uint32_t zeros;              // multiplicity of the extra id-0 entry (0 = none)
  uint32_t fill_id;            // output slots without a candidate: 0 -> (0, 0.0), kEmpty -> (kEmpty, FLT_MAX)
  uint32_t *out_ids;           // nq x k
  float *out_dists;            // nq x k (nullable)
};

constexpr uint32_t kVisWide = 0xffffffffu;
constexpr size_t kHelpBoardBytes = 256;  // the helpers' request board (search kernel, kMode 4)
#ifndef ALAYA_HELP_DEPTH
#define ALAYA_HELP_DEPTH 1
#endif
constexpr size_t kHelpMemoSlots = ALAYA_HELP_DEPTH + 1;  // memo rows (requests) per searcher
constexpr uint32_t kStabBucket = 8;  // spill-table entries per bucket (16 B: one prefetch per lane)
// bytes of the LDS visited table / of one wave's LDS region / of a workgroup's shared region
// (SQ8: the quantizer's per-dimension scale and min); a workgroup of W waves takes
// shared + W * wave bytes
inline size_t visited_table_bytes(uint32_t hash_log2, bool compact) {
  return (static_cast<size_t>(compact ? 2 : 4)) << hash_log2;
}
size_t search_wave_lds_bytes(uint32_t stride, uint32_t ef, uint32_t hash_log2, bool compact = false,
                             int sq8_order = 0);
// bytes of a wave's query region: stride f32 terms, or the query's codes (AVX-512-order SQ8 kernels
// built with ALAYA_SQ8_QCODES)
size_t search_query_lds_bytes(uint32_t stride, int sq8_order);
__host__ __device__ inline size_t search_shared_lds_bytes(uint32_t stride, bool sq8) {
  return sq8 ? 2 * static_cast<size_t>(stride) * 4 : 0;
}
// rerank: p.base/p.queries are the raw f32 rows and the (normalised) f32 queries
hipError_t launch_rerank(const SearchParams &p, const RerankParams &r, hipStream_t stream);
hipError_t search_occupancy(const SearchParams &p, int waves, size_t lds, int *blocks_per_cu);
// whether a search of this shape has a helper kernel (SearchParams::help)
bool search_has_helpers(uint32_t dim, int sq8_order, bool generic);
// whether a search of this shape has a two-waves-per-SIMD kernel (SearchParams::two_waves)
bool search_has_two_waves(uint32_t dim, int sq8_order, bool generic);
hipError_t launch_search(const SearchParams &p, int grid, int waves, size_t lds, hipStream_t stream);
// out[q * n + i] = dist(queries[q], base[ids[i]]) for q < nq (bit-exact device distance)
hipError_t launch_row_distances(const SearchParams &p, const uint32_t *ids, uint32_t n,
                                uint32_t nq, float *out, hipStream_t stream);

// streaming read of `bytes` (multiple of 16) for the measured-bandwidth calibration
hipError_t launch_stream_read(const void *buf, uint64_t bytes, int grid, int shape, float *sink,
                              hipStream_t stream);

}  // namespace alaya_amd
