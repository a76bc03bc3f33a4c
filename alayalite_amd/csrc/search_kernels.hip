// MI355X (gfx950) device code for the HNSW best-first search hot path.
//
// One wavefront (64 lanes) owns one query at a time; workgroups are single waves that pull query
// indices from a device work counter until the batch is drained (persistent blocks).  Per query:
//   * query vector staged in LDS, zero-padded to the row stride;
//   * the candidate pool (the reference's LinearPool, include/utils/query_utils.hpp:236-312) is a
//     sorted LDS array of (dist, id|checked) with capacity ef;
//   * the visited set (DynamicBitset, query_utils.hpp:69-115) is an exact LDS open-addressing hash
//     table that spills to a per-slot global bitset when it fills;
//   * one expansion = read a 128 B adjacency row, filter visited ids in adjacency order, compute all
//     new distances at once (8 lanes per row, 8 rows per wave pass, 128 B-coalesced row chunks), then
//     merge the batch into the pool with a wave-parallel stable merge that is provably identical to
//     inserting the neighbours one by one (graph_search_job.hpp:237-251 + LinearPool::insert).
// The distance reproduces l2_sqr_avx2 / ip_sqr_avx2 (include/simd/distance_l2.ipp:54-116,
// distance_ip.ipp:56-111) bit for bit: lane m of a row group owns partial sums acc[4m..4m+3]
// (element 32t+j -> acc[j]), the 8-lane combine follows the AVX2 horizontal tree exactly.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "search_kernels.h"
#include "search_device.h"

// Minimum waves per SIMD the compiler must leave room for, per search-kernel shape (the register
// budget: 512 / waves VGPRs).  0 = no constraint.  Diagnostics builds override with
// -DALAYA_MIN_WAVES_SQ8=... / -DALAYA_MIN_WAVES_NARROW=....
#ifndef ALAYA_MIN_WAVES_SQ8
// The AVX-512-order SQ8 kernels (config 5 on an AVX-512 host) are held to 4 waves per SIMD (128
// VGPRs): with the spill table the 768-d IP kernel needs 129 and would drop to 3; at 128 the
// allocator spills one 8-byte value that is live across the whole query loop (a store at kernel
// entry, a load after the loop), nothing per expansion.  The AVX2-order kernels would spill inside
// the expansion loop (32-136 B of scratch) and keep their natural budget.
#define ALAYA_MIN_WAVES_SQ8 -1
#endif
#ifndef ALAYA_MIN_WAVES_NARROW
#define ALAYA_MIN_WAVES_NARROW 0
#endif
#ifndef ALAYA_MIN_WAVES_WIDE
#define ALAYA_MIN_WAVES_WIDE 0  // diagnostics: waves per SIMD for the f32 kernels with d > 256
#endif
// kSpace: 0 = f32 rows, 1 = SQ8 codes in the AVX2 order, 2 = SQ8 codes in the AVX-512 order (the
// kernels that run on the spill table).  f32 rows on the spill table were measured and dropped:
// SIFT 1M at 10k queries 1.19 -> 1.47 ms, at 1k 0.55 -> 0.68 ms
// (profiles/r04/search_experiments/sift_spill_table_rejected.log).
template <int kSpace>
constexpr bool space_sq8() { return kSpace == 1 || kSpace == 2; }
template <int kSpace>
constexpr bool space_tab() { return kSpace == 2; }

template <int kChunks, int kSpace, int kMode = 0>
constexpr int search_min_waves() {
  if constexpr ((kMode & 8) != 0) return 2;  // the two-waves-per-SIMD wide-row kernels
  if constexpr (space_sq8<kSpace>()) {
    if (ALAYA_MIN_WAVES_SQ8 >= 0) return ALAYA_MIN_WAVES_SQ8;
    return kSpace == 2 && kChunks > 0 ? 4 : 0;
  }
  return kChunks > 0 && kChunks <= 8 ? ALAYA_MIN_WAVES_NARROW : (kChunks > 8 ? ALAYA_MIN_WAVES_WIDE : 0);
}

namespace alaya_amd {

namespace {

// LDS layout of a search workgroup of W waves: a shared region (SQ8: the per-index scale and min
// of SQ8Space's quantizer, identical for every query, stored once per workgroup) followed by one
// region of p.wave_lds bytes per wave (query, candidate batch, pool, visited table).
template <int kSpace>
__device__ __forceinline__ Lds carve_lds(const SearchParams &p, unsigned char *smem, int wave) {
  Lds L;
  unsigned char *ptr = smem + search_shared_lds_bytes(p.stride, space_sq8<kSpace>()) + static_cast<size_t>(wave) * p.wave_lds;
  L.q = reinterpret_cast<float *>(ptr);
  ptr += sq8_query_codes<kSpace>() ? (static_cast<size_t>(p.stride) + 15) / 16 * 16 : static_cast<size_t>(p.stride) * 4;
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
  L.sq_scale = space_sq8<kSpace>() ? reinterpret_cast<float *>(smem) : nullptr;
  L.sq_min = space_sq8<kSpace>() ? reinterpret_cast<float *>(smem) + p.stride : nullptr;
  return L;
}

// SQ8: the workgroup's waves fill the shared scale / min once (SQ8Quantizer, sq8.hpp:99-130:
// scale = (max - min) * (1/255)), before any wave starts a query.
template <int kSpace>
__device__ __forceinline__ void fill_shared(const SearchParams &p, const Lds &L) {
  if constexpr (space_sq8<kSpace>()) {
    const float kInv255 = 1.0f / 255.0f;
    for (uint32_t e = threadIdx.x; e < p.stride; e += blockDim.x) {
      float sc = 0.f, mn = 0.f;
      if (e < p.dim) {
        mn = p.sq_min[e];
        sc = (p.sq_max[e] - mn) * kInv255;
      }
      L.sq_scale[e] = sc;
      L.sq_min[e] = mn;
    }
    __syncthreads();
  }
}

// Per-query setup shared by the search kernels: the query staged in LDS (SQ8: encoded with the
// quantizer), visited table and pool cleared, then Graph::initialize_search (graph.hpp:148-158).
template <bool kIP, int kChunks, int kSpace, int kRows = 0>
__device__ __forceinline__ void query_begin(const SearchParams &p, const Lds &L, uint32_t qi, uint32_t *slot_bits,
                                            uint32_t *slot_dirty, uint16_t *slot_stab, Visited &vs, PoolState &ps,
                                            uint32_t &n_dist_up, uint32_t &n_hops_up) {
  const int lane = lane_id();
  const uint32_t hsize = 1u << p.hash_log2;
  // ---- per-query init ------------------------------------------------------------------
  const float *qsrc = p.queries + static_cast<uint64_t>(qi) * p.q_stride;
  if constexpr (!space_sq8<kSpace>()) {
    for (uint32_t e = lane; e < p.stride; e += 64) L.q[e] = e < p.dim ? qsrc[e] : 0.f;
  } else {
    // SQ8Space::QueryComputer encodes the query with the quantizer (sq8_space.hpp:266-271,
    // SQ8Quantizer::quantize sq8.hpp:118-130), then every distance uses its codes.
    // (the per-index scale and min are the workgroup's shared LDS copy, fill_shared)
    for (uint32_t e = lane; e < p.stride; e += 64) {
      float xq = 0.f;
      uint32_t code = 0;
      if (e < p.dim) {
        const float v = qsrc[e];
        const float mn = p.sq_min[e];
        const float mx = p.sq_max[e];
        if (mx == mn) code = 0;
        else if (v >= mx) code = 255;
        else if (v <= mn) code = 0;
        else code = static_cast<uint8_t>(((v - mn) / (mx - mn)) * 255);
        const float xf = static_cast<float>(code);
        xq = kIP ? fmaf(xf, L.sq_scale[e], mn) : xf;
      }
      if constexpr (sq8_query_codes<kSpace>()) {
        reinterpret_cast<uint8_t *>(L.q)[e] = static_cast<uint8_t>(code);  // the term is rebuilt per chunk
      } else {
        L.q[e] = xq;
      }
    }
  }
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
  vs = make_visited(p, L.hash, slot_bits, slot_dirty, slot_stab);
  ps = PoolState{0u, 0u, p.ef};
  constexpr bool kTab = space_tab<kSpace>();  // the kernels that may run on the spill table

  // ---- Graph::initialize_search (graph.hpp:148-158) ---------------------------------------
  if (p.levels != nullptr) {
    // OverlayGraph::initialize (overlay_graph.hpp:122-144): greedy descent, strict '<'.
    uint32_t u = p.ep;
    uint64_t off_u = p.upper_off[u];  // u's upper-level lists, kept while u stays
    if (lane == 0) L.cid[0] = u;
    wave_sync();
    space_distances<kIP, kChunks, kSpace, false, kRows>(p, L, L.cid, 1, L.cd);
    float cur = L.cd[0];
    ++n_dist_up;
    for (int level = static_cast<int>(p.levels[u]); level > 0; --level) {
      bool changed = true;
      while (changed) {
        changed = false;
        const uint32_t *list = p.upper_edges + off_u + static_cast<uint64_t>(level - 1) * p.upper_R;
        const uint32_t v = lane < static_cast<int>(p.upper_R) ? list[lane] : kEmpty;
        const uint64_t endm = ballot(lane < static_cast<int>(p.upper_R) && v == kEmpty);
        const int cnt = endm ? __ffsll(static_cast<unsigned long long>(endm)) - 1
                             : static_cast<int>(p.upper_R);
        ++n_hops_up;
        const bool has = lane < cnt;
        // every candidate's list offset is loaded beside its row: the hop to the winner then needs
        // one dependent load (its list), not two
        uint64_t off_v = 0;
        if (has) off_v = p.upper_off[v];
        wave_sync();
        if (has) L.cid[lane] = v;
        wave_sync();
        space_distances<kIP, kChunks, kSpace, false, kRows>(p, L, L.cid, cnt, L.cd);
        n_dist_up += cnt;
        // first index of the minimum == the sequential strict-'<' scan's final choice (the minimum
        // is order-free: DPP / swizzle steps within each 32-lane half, then the two halves)
        const float dl = has ? L.cd[lane] : FLT_MAX;
        float mn = dl;
        mn = fminf(mn, lane_xor<1>(mn));
        mn = fminf(mn, lane_xor<2>(mn));
        mn = fminf(mn, lane_xor<4>(mn));
        mn = fminf(mn, lane_xor<8>(mn));
        mn = fminf(mn, lane_xor<16>(mn));
        mn = fminf(read_lane(mn, 0), read_lane(mn, 32));
        const uint64_t at = ballot(has && dl == mn);
        if (at && mn < cur) {
          const int w = __ffsll(static_cast<unsigned long long>(at)) - 1;
          u = read_lane(v, w);
          off_u = (static_cast<uint64_t>(read_lane(static_cast<uint32_t>(off_v >> 32), w)) << 32) |
                  read_lane(static_cast<uint32_t>(off_v), w);
          cur = mn;
          changed = true;
        }
        wave_sync();
      }
    }
    // pool.insert(u, cur); vis.set(u)
    if (lane == 0) {
      L.pd[0] = cur;
      L.pi[0] = u;
    }
    ps.size = 1;
    ps.cur = 0;
    visit<kTab>(vs, u, lane == 0);
    wave_sync();
  } else {
    // NSG-style entry points: insert each ep, then mark it visited (graph.hpp:153-156)
    for (uint32_t b = 0; b < p.n_eps; b += 64) {
      const uint32_t cnt = min(64u, p.n_eps - b);
      const bool has = static_cast<uint32_t>(lane) < cnt;
      uint32_t v = has ? p.eps[b + lane] : 0u;
      if (has) L.cid[lane] = v;
      wave_sync();
      for (uint32_t c = 0; c < cnt; c += 8) {
        space_distances<kIP, kChunks, kSpace, false, kRows>(p, L, L.cid + c, min(8u, cnt - c), L.cd + c);
      }
      n_dist_up += cnt;
      const float d = has ? L.cd[lane] : 0.f;
      wave_sync();
      pool_merge(ps, L, has, v, d);
      // duplicates among eps are all inserted (no visited check in the reference loop)
      for (uint32_t j = 0; j < cnt; ++j) {
        const uint32_t vj = read_lane(v, j);
        if (!vs.spilled && vs.count + 64 > vs.limit) spill_begin<kTab>(vs);
        visit<kTab>(vs, vj, lane == 0);
      }
      wave_sync();
    }
  }
}

// Results (ids[i] = pool.id(i), distances[i] = pool.dist(i), graph_search_job.hpp:254-256) and the
// per-query counters.
__device__ __forceinline__ void query_end(const SearchParams &p, const Lds &L, const PoolState &ps, uint32_t qi,
                                          uint32_t n_dist, uint32_t n_expand, uint32_t n_dist_up,
                                          uint32_t n_hops_up) {
  const int lane = lane_id();
  for (uint32_t i = lane; i < p.k; i += 64) {
    uint32_t id = p.fill_id;
    float d = p.fill_id == kEmpty ? FLT_MAX : 0.f;  // kEmpty fill (shard / corrected rerank) sorts last
    if (i < ps.size) {
      id = L.pi[i] & kIdMask;
      d = L.pd[i];
    }
    p.out_ids[static_cast<uint64_t>(qi) * p.k + i] = id;
    if (p.out_dists) p.out_dists[static_cast<uint64_t>(qi) * p.k + i] = d;
  }
  if (p.out_counters && lane == 0) {
    uint32_t *c = p.out_counters + static_cast<uint64_t>(qi) * 4;
    c[0] = n_dist;
    c[1] = n_expand;
    c[2] = n_dist_up;
    c[3] = n_hops_up;
  }
}

// --------------------------------------------------------------------------------------------
// Distance helpers.  A searcher with no query left (the batch counter ran out) computes distances
// for the siblings of its workgroup that are still searching.  Each searcher keeps three requests on
// the workgroup's board: the node it is expanding (until it has read the memo) and the nodes it will
// most likely expand next -- the pool's first two unchecked entries right after each pop, and the
// merge's new next pop when it changes (the prediction holds ~99.8 % of the time for the next
// expansion).  Helpers claim 16 adjacency
// positions of a request at a time (older requests first: the nearer expansion), compute those
// rows' distances against the sibling's query and store (request seq, distance) per position in
// one memo, held in the region of the first wave that became a helper.  When the searcher expands
// a requested node it takes the memo's distance for every fresh neighbour whose entry carries the
// request's seq, and computes the rest itself -- none when the helpers kept up, so the expansion has
// no row gather at all.  The distances are deterministic (same function, same query vector, same
// row) and the searcher still does every visit, merge and pop itself, so ids, distances and
// counters are those of the search without helpers; a helper that falls behind or answers a stale
// request only costs work.  The reference keeps every worker busy to the end with its coroutine
// interleave (include/executor/worker.hpp:47,111-136); here the batch tail's idle waves (and, in
// batches smaller than the resident searchers, the spare ones) shorten the remaining searchers'
// expansions instead.
// LDS: a kHelpBoardBytes (256-byte) board after the workgroup's wave regions; the memo (W x kHelpSlots
// x R entries of 8 bytes) at byte p.memo_off of the memo wave's region -- its query vector or its pool
// and visited table, unused once it has no query.
// --------------------------------------------------------------------------------------------
// How far ahead a searcher asks: 1 = the next expansion, 2 = the next two (diagnostics builds:
// -DALAYA_HELP_DEPTH=2).  One slot more than the depth keeps the expanding node's request alive
// until its memo entries are read.
#ifndef ALAYA_HELP_DEPTH
#define ALAYA_HELP_DEPTH 1
#endif
// Issue priority (s_setprio) of a searcher with helpers present: a helper shares its SIMD with up to
// three waves of other workgroups, which may still be searching; the searchers' expansion chains run
// at this priority and helpers at 0, so a helper's distance work fills issue slots the chains leave
// free instead of delaying them.  0 = no priorities (diagnostics builds: -DALAYA_HELP_PRIO=0).
#ifndef ALAYA_HELP_PRIO
#define ALAYA_HELP_PRIO 2
#endif
constexpr int kHelpDepth = ALAYA_HELP_DEPTH;
static_assert(kHelpDepth == 1 || kHelpDepth == 2, "help depth 1 or 2");
constexpr int kHelpSlots = kHelpDepth + 1;  // requests per searcher
constexpr uint32_t kHelpClaim = 16;         // adjacency positions per claim (one row pass)
struct HelpOwner {                          // one searcher's requests
  uint64_t req[kHelpSlots];                 // (seq << 32) | node per slot; node kEmpty = none; seq only grows
  uint32_t claim[kHelpSlots];               // (seq mod 2^24) << 8 | next adjacency position to hand out
  uint32_t hits;                            // fresh distances taken from the memo (help_stats)
  uint32_t skips;                           // expansions whose fresh distances all came from the memo
  uint32_t rows;                            // as a helper: rows whose distances it computed
};
struct HelpBoard {
  HelpOwner own[4];
  uint32_t mask;  // bits 0-3: waves with no query left (helpers); bits 8-15: 1 + the memo wave
  uint32_t pad[3];
};
static_assert(sizeof(HelpBoard) <= kHelpBoardBytes, "board size");

__device__ __forceinline__ HelpBoard *help_board(const SearchParams &p, unsigned char *smem, int W) {
  return reinterpret_cast<HelpBoard *>(smem + search_shared_lds_bytes(p.stride, p.sq8_order != 0) +
                                       static_cast<size_t>(W) * p.wave_lds);
}

__device__ __forceinline__ void help_board_init(HelpBoard *b) {
  for (int i = 0; i < 4; ++i) {
    for (int s = 0; s < kHelpSlots; ++s) {
      b->own[i].req[s] = static_cast<uint64_t>(kEmpty);
      b->own[i].claim[s] = 0u;
    }
    b->own[i].hits = 0u;
    b->own[i].skips = 0u;
    b->own[i].rows = 0u;
  }
  b->mask = 0u;
}

__device__ __forceinline__ uint32_t help_word(HelpBoard *b) {
  return read_lane(__hip_atomic_load(&b->mask, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), 0);
}

// A searcher's requests as (node, seq) pairs (wave-uniform; each pair is one 8-byte LDS word)
struct HelpReqs {
  uint32_t node[kHelpSlots];
  uint32_t seq[kHelpSlots];
};
__device__ __forceinline__ HelpReqs help_reqs(HelpBoard *b, int t) {
  HelpReqs q;
#pragma unroll
  for (int s = 0; s < kHelpSlots; ++s) {
    const uint64_t r = __hip_atomic_load(&b->own[t].req[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    q.node[s] = read_lane(static_cast<uint32_t>(r), 0);
    q.seq[s] = read_lane(static_cast<uint32_t>(r >> 32), 0);
  }
  return q;
}

// A new query: no request of the previous one may match again (memo entries are tagged with a seq
// that only grows; emptied slots are skipped by the helpers).
__device__ __forceinline__ void help_reset(HelpBoard *b, int wave) {
  if (lane_id() < kHelpSlots)
    __hip_atomic_store(&b->own[wave].req[lane_id()], static_cast<uint64_t>(kEmpty), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The searcher has read the memo for slot s: no helper should start more work on that request.
__device__ __forceinline__ void help_retire(HelpBoard *b, int wave, int s, uint32_t seq) {
  if (lane_id() == 0)
    __hip_atomic_store(&b->own[wave].claim[s], ((seq & 0xffffffu) << 8) | 0xffu, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The searcher's side of the board, kept in (scalar) registers so that an expansion pays no LDS
// round trip for it: its requests, its seq counter and the memo wave (-1 while it has no helper).
struct HelpMine {
  uint32_t node[kHelpSlots];
  uint32_t seq[kHelpSlots];
  uint32_t next_seq;
  int memo_wave;
};

// A new request for `node` in slot s (lane 0: the claim word first, then the request, so a helper
// that sees the request finds its claim reset).
__device__ __forceinline__ void mine_publish(HelpBoard *b, int wave, HelpMine &m, int s, uint32_t node) {
  const uint32_t seq = ++m.next_seq;
  m.node[s] = node;
  m.seq[s] = seq;
  if (lane_id() == 0) {
    HelpOwner &o = b->own[wave];
    // the LDS performs one wave's operations in order: a compiler barrier keeps the claim before the
    // request without the release's wait for every outstanding LDS and scalar load
    __hip_atomic_store(&o.claim[s], (seq & 0xffffffu) << 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    __hip_atomic_store(&o.req[s], (static_cast<uint64_t>(seq) << 32) | node, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// Requests for the next expansions c1 (and, at depth 2, c2; kEmpty: none), keeping the slot of the
// node being expanded (u) until its memo entries are read: slots holding u, c1 or c2 stay, the others
// take the missing ones (with depth + 1 slots there is always room).
__device__ __forceinline__ void mine_request(HelpBoard *b, int wave, HelpMine &m, uint32_t u, uint32_t c1,
                                             uint32_t c2) {
  if (kHelpDepth < 2) c2 = kEmpty;
  bool need1 = c1 != kEmpty, need2 = c2 != kEmpty && c2 != c1;
#pragma unroll
  for (int s = 0; s < kHelpSlots; ++s) {
    need1 = need1 && m.node[s] != c1;
    need2 = need2 && m.node[s] != c2;
  }
  if (!need1 && !need2) return;
#pragma unroll
  for (int s = 0; s < kHelpSlots; ++s) {
    const uint32_t x = m.node[s];
    if (x != kEmpty && (x == u || x == c1 || x == c2)) continue;  // a slot to keep
    if (need1) {
      mine_publish(b, wave, m, s, c1);
      need1 = false;
    } else if (need2) {
      mine_publish(b, wave, m, s, c2);
      need2 = false;
    }
  }
}

__device__ __forceinline__ void mine_reset(HelpBoard *b, int wave, HelpMine &m) {
#pragma unroll
  for (int s = 0; s < kHelpSlots; ++s) m.node[s] = kEmpty;
  help_reset(b, wave);
}

// The memo: W x kHelpSlots x R entries (seq << 32 | distance bits) at p.memo_off of the memo wave's
// region.
template <int kSpace>
__device__ __forceinline__ uint64_t *help_memo(const SearchParams &p, unsigned char *smem, int memo_wave) {
  return reinterpret_cast<uint64_t *>(reinterpret_cast<unsigned char *>(carve_lds<kSpace>(p, smem, memo_wave).q) +
                                      p.memo_off);
}

// Whether sibling t has probably visited v already (a hint: read while the sibling writes, so it may
// be stale either way): its LDS first level, and -- SQ8 on the spill table -- its spill-table bucket.
template <int kSpace>
__device__ __forceinline__ bool sibling_visited(const SearchParams &p, const Lds &Lt, int t, uint32_t v, bool want) {
  Visited vt = make_visited(p, Lt.hash, nullptr, nullptr, nullptr);
  bool seen = want && table_lookup<true>(vt, v);
  if constexpr (space_tab<kSpace>()) {
    if (p.spill_table != nullptr) {
      const uint64_t slot = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + t;
      vt.stab = p.spill_table + (slot << p.stab_log2);
      vt.stab_bmask = (1u << (p.stab_log2 - 3)) - 1u;
      uint32_t home, code;
      stab_key(vt, v, home, code);
      uint64_t lo = 0ull, hi = 0ull;
      if (want && !seen) stab_load(vt, home, lo, hi);
      bool found;
      uint32_t occ;
      stab_scan(lo, hi, code, found, occ);
      seen = seen || (want && found);
    }
  }
  return seen;
}

// A wave whose batch counter ran out helps its siblings until every wave of the workgroup has none
// left (then all exit: no wave ever waits for another).
template <bool kIP, int kChunks, int kSpace>
__device__ void help_siblings(const SearchParams &p, unsigned char *smem, const Lds &L, HelpBoard *b, int wave,
                              int W) {
  const int lane = lane_id();
  const uint32_t R = p.R;
  const uint32_t full = (1u << W) - 1u;
  if constexpr (ALAYA_HELP_PRIO > 0) __builtin_amdgcn_s_setprio(0);  // helpers yield to searchers
  // the visited hint (skip rows the sibling has already visited): by default where a stale read costs
  // a global round trip less than the rows it saves -- SQ8 on the spill table (config 5, 1k queries:
  // 3.47 ms with it, 3.62 without); the f32 rows of the SIFT shape are cheaper to compute than to
  // filter (10k queries: 1.138 ms without, 1.153 with).  ALAYA_HELP_FLAGS bit 0 / 1 force it off / on.
  const bool hint = (p.help_flags & 2u) || (space_sq8<kSpace>() && !(p.help_flags & 1u));
  uint32_t *exhausted = reinterpret_cast<uint32_t *>(L.sd);  // per (sibling, slot): a request fully claimed
  if (lane < 4 * kHelpSlots) exhausted[lane] = 0u;
  // Leave the searchers first: retire this wave's last requests and set its helper bit, so no helper
  // that reads the board from now on picks this wave as a sibling.  Only then may its region be
  // overwritten by the memo clear below (with memo_off > 0 it covers the pool and the visited
  // table, which another helper's visited hint reads; a helper that read the board just before
  // still probes a bounded lap, table_lookup<true>).
  help_reset(b, wave);
  wave_sync();
  if (lane == 0) __hip_atomic_fetch_or(&b->mask, 1u << wave, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  wave_sync();
  // the first helper's region holds the memo: clear this wave's (seq 0 = no entry), then claim the
  // role (no helper reads the memo before some wave has claimed it: each claims or finds it claimed
  // before its own loop, and a searcher looks only once the role is set)
  {
    uint64_t *mine = help_memo<kSpace>(p, smem, wave);
    for (uint32_t e = lane; e < static_cast<uint32_t>(W) * kHelpSlots * R; e += 64)
      __hip_atomic_store(mine + e, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  wave_sync();
  if (lane == 0) {
    uint32_t cur = __hip_atomic_load(&b->mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while ((cur >> 8) == 0u) {
      const uint32_t want = cur | (static_cast<uint32_t>(wave + 1) << 8);
      if (__hip_atomic_compare_exchange_strong(&b->mask, &cur, want, __ATOMIC_RELEASE, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP))
        break;
    }
  }
  wave_sync();
  int t = wave;
  for (;;) {
    const uint32_t hw = help_word(b);
    const uint32_t mask = hw & 0xffu;
    if (mask == full) break;  // every sibling is done
    uint64_t *memo = help_memo<kSpace>(p, smem, static_cast<int>(hw >> 8) - 1);
    do {
      t = t + 1 == W ? 0 : t + 1;
    } while ((mask >> t) & 1u);
    const HelpReqs r = help_reqs(b, t);
    // the oldest open request first (the nearest expansion)
    uint32_t order = 0u;  // slot indices, 2 bits each, oldest first
    if constexpr (kHelpSlots == 2) {
      order = r.seq[1] < r.seq[0] ? (1u | (0u << 2)) : (0u | (1u << 2));
    } else {
      const uint32_t a = r.seq[0], b1 = r.seq[1], c = r.seq[kHelpSlots - 1];
      const int s0 = (a <= b1 && a <= c) ? 0 : (b1 <= c ? 1 : 2);
      const int sa = (s0 + 1) % 3, sb = (s0 + 2) % 3;
      const bool swap = r.seq[sb] < r.seq[sa];
      order = static_cast<uint32_t>(s0) | (static_cast<uint32_t>(swap ? sb : sa) << 2) |
              (static_cast<uint32_t>(swap ? sa : sb) << 4);
    }
    bool worked = false;
    for (int k = 0; k < kHelpSlots && !worked; ++k) {
      const int s = static_cast<int>((order >> (2 * k)) & 3u);
      const uint32_t node = r.node[s], seq = r.seq[s];
      if (node == kEmpty || seq == 0u || exhausted[t * kHelpSlots + s] == seq) continue;
      uint32_t old = 0u;
      if (lane == 0) old = atomicAdd(&b->own[t].claim[s], kHelpClaim);
      old = read_lane(old, 0);
      if ((old >> 8) != (seq & 0xffffffu)) continue;  // replaced by a newer request meanwhile
      const uint32_t pos = old & 0xffu;
      const uint32_t v = lane < static_cast<int>(R) ? p.l0[static_cast<uint64_t>(node) * R + lane] : kEmpty;
      const uint64_t endm = ballot(lane < static_cast<int>(R) && v == kEmpty);
      const uint32_t cnt = endm ? static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(endm)) - 1) : R;
      if (pos >= cnt) {
        if (lane == 0) exhausted[t * kHelpSlots + s] = seq;
        wave_sync();
        continue;
      }
      worked = true;
      const Lds Lt = carve_lds<kSpace>(p, smem, t);
      bool want = static_cast<uint32_t>(lane) >= pos && static_cast<uint32_t>(lane) < min(pos + kHelpClaim, cnt);
      if (hint) want = want && !sibling_visited<kSpace>(p, Lt, t, v, want);
      const uint64_t wm = ballot(want);
      const int n = __popcll(wm);
      if (n == 0) continue;
      const uint32_t slot = __popcll(wm & ((1ull << lane) - 1ull));
      if (want) L.cid[slot] = v;
      wave_sync();
      space_distances<kIP, kChunks, kSpace>(p, Lt, L.cid, n, L.cd);
      if (lane == 0) b->own[wave].rows += static_cast<uint32_t>(n);
      if (want) {
        const uint64_t e = (static_cast<uint64_t>(seq) << 32) | __float_as_uint(L.cd[slot]);
        __hip_atomic_store(memo + (static_cast<uint32_t>(t) * kHelpSlots + s) * R + lane, e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      wave_sync();
    }
    if (!worked) __builtin_amdgcn_s_sleep(4);  // ~256 cycles: polls stay off the searchers' LDS
  }
}

// --------------------------------------------------------------------------------------------
// The search kernel.
// --------------------------------------------------------------------------------------------
// kMode bits: 1 = diagnostic build that accumulates s_memtime cycles per phase into p.stamps
// (nq x 8): [0] init + overlay descent, [1] pop, [2] adjacency load + visited set, [3] distances,
// [4] merge, [5] expansions after the visited table spilled, [6] whole query, [7] prefetch hits;
// 2 = the spill-table prefetch check (ALAYA_SPILL_FLAGS bit 8: every bucket read one expansion ahead
// is compared with a re-read at its use, and a stale one marks the query's counters);
// 4 = distance helpers (SearchParams::help): a wave with no query left computes the distances of a
// sibling's next expansion into a memo the sibling reads (help_siblings below);
// 8 = two waves per SIMD for wide f32 rows (one row per lane group, SearchParams::two_waves).
// A workgroup holds blockDim.x / 64 waves (1 for wide f32 rows; 4 for SQ8, which share the
// quantizer's scale / min, and for searches with helpers); each wave is an independent persistent
// searcher with its own visited spill slot.  After fill_shared the waves never wait on each other.
template <bool kIP, int kChunks, int kMode, int kSpace = 0>
__global__ void __launch_bounds__(256)
    __attribute__((amdgpu_waves_per_eu(search_min_waves<kChunks, kSpace, kMode>() ? search_min_waves<kChunks, kSpace, kMode>() : 1,
                                       8))) hnsw_search_kernel(SearchParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kStamp = (kMode & 1) != 0;
  constexpr bool kCheck = (kMode & 2) != 0;
  constexpr bool kHelp = (kMode & 4) != 0;
  constexpr int kRows = (kMode & 8) != 0 ? 1 : 0;
  const int lane = lane_id();
  const int wave = static_cast<int>(threadIdx.x >> 6);
  const int W = static_cast<int>(blockDim.x >> 6);
  const Lds L = carve_lds<kSpace>(p, smem, wave);
  fill_shared<kSpace>(p, L);
  HelpBoard *board = kHelp ? help_board(p, smem, W) : nullptr;
  HelpMine mine;
  if constexpr (kHelp) {
    if constexpr (ALAYA_HELP_PRIO > 0) __builtin_amdgcn_s_setprio(ALAYA_HELP_PRIO);
    if (threadIdx.x == 0) help_board_init(board);
    __syncthreads();
    for (int s = 0; s < kHelpSlots; ++s) mine.node[s] = kEmpty, mine.seq[s] = 0u;
    mine.next_seq = 0u;
    mine.memo_wave = -1;
  }
  const uint64_t bit_words = (p.n + 31) / 32;
  const uint64_t slot = static_cast<uint64_t>(blockIdx.x) * (blockDim.x >> 6) + wave;
  uint32_t *slot_bits = p.overflow_bits + slot * bit_words;
  uint32_t *slot_dirty = p.dirty_words + slot * p.dirty_cap;
  // spill tables only in the AVX-512-order SQ8 kernels (a compile-time null elsewhere: the f32
  // kernels carry none of it)
  uint16_t *slot_stab = (space_tab<kSpace>() && p.spill_table) ? p.spill_table + (slot << p.stab_log2) : nullptr;

  bool first_round = true;
  for (;;) {
    uint32_t qi = 0;
    if (kHelp && first_round) {
      // first round assigned wave-major over the workgroups, so a batch smaller than the resident
      // searchers leaves every workgroup a mix of searchers and helpers; then the work counter
      qi = static_cast<uint32_t>(wave) * gridDim.x + blockIdx.x;
    } else {
      if (lane == 0) qi = atomicAdd(p.work_counter, 1u);
      qi = read_lane(qi, 0) + (kHelp ? static_cast<uint32_t>(W) * gridDim.x : 0u);
    }
    first_round = false;
    if (qi >= p.nq) break;
    // a memo entry belongs to the query it was requested in: requests of an earlier query never
    // match again (the seq only grows, and the requests are dropped here)
    if constexpr (kHelp) mine_reset(board, wave, mine);

    uint64_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = kStamp ? __builtin_readcyclecounter() : 0;
    const uint64_t t_begin = t_prev;
    auto stamp = [&](int slot) {
      if constexpr (kStamp) {
        const uint64_t now = __builtin_readcyclecounter();
        st[slot] += now - t_prev;
        t_prev = now;
      }
    };
    Visited vs;
    PoolState ps;
    uint32_t n_dist = 0, n_expand = 0, n_dist_up = 0, n_hops_up = 0;
    query_begin<kIP, kChunks, kSpace, kRows>(p, L, qi, slot_bits, slot_dirty, slot_stab, vs, ps, n_dist_up, n_hops_up);

    // ---- best-first expansion (graph_search_job.hpp:228-252 / 310-330) -----------------------
    stamp(0);
    // Adjacency prefetch (no semantic effect): after a pop, the first unchecked entry is the next
    // expansion unless the merge puts a closer candidate in front of it.  Its 128 B row is loaded
    // into registers while this expansion runs and used only if the next pop returns that id.
    uint32_t pred = kEmpty, pred_v = kEmpty;
    // Second-level state of the predicted next expansion's neighbours (spilled queries,
    // spill_prefetch: spill-table buckets or bitset words): the SQ8 kernels only, where config 5's
    // 10k-query batch spills almost every query (its 10M ids fit only a few hundred LDS slots at full
    // residency): 10.43 -> 9.76 ms with the bitset.  The f32 shapes rarely spill at their table
    // sizes and measured 0.8 % slower with it (profiles/r03/search_experiments/).
    constexpr bool kSpillPrefetch = kSpace != 0;
    // Register merge (pool_merge, pools of <= 128 entries) in the small-row f32 kernels, whose ef
    // at recall 0.95 is ~70 (SIFT-shaped); the SQ8 / wide-row kernels run ef ~370 and keep their
    // registers for the row pass.
    constexpr bool kRegMerge = kSpace == 0 && kChunks > 0 && kChunks <= 8;
    uint32_t pre_u = kEmpty;
    uint64_t pre_lo = 0ull, pre_hi = 0ull;
    while (ps.cur < ps.size) {
      uint32_t c1 = kEmpty, c2 = kEmpty;
      const uint32_t u = pool_pop<kHelp>(ps, L, &c1, &c2);
      ++n_expand;
      // helpers present: the request for this node (if any; its memo is read in the distance phase)
      // and requests for the next two expansions as the pool stands now
      uint32_t look = 0u;  // (seq << 2) | slot
      if constexpr (kHelp) {
        if (mine.memo_wave < 0 && (n_expand & 3u) == 1u) {  // (a helper appears at most once)
          const uint32_t hw = help_word(board);
          if ((hw >> 8) != 0u) mine.memo_wave = static_cast<int>(hw >> 8) - 1;
        }
        if (mine.memo_wave >= 0) {
#pragma unroll
          for (int hs = 0; hs < kHelpSlots; ++hs)
            if (mine.node[hs] == u) look = (mine.seq[hs] << 2) | static_cast<uint32_t>(hs);
          mine_request(board, wave, mine, u, c1, c2);
        }
      }
#ifndef ALAYA_FINE_STAMPS
      if (kStamp && vs.spilled) st[5]++;
#endif
      stamp(1);
      uint32_t v;
      if (u == pred) {
        v = pred_v;
#ifndef ALAYA_FINE_STAMPS
        if (kStamp) st[7]++;
#endif
      } else {
        v = lane < static_cast<int>(p.R) ? p.l0[static_cast<uint64_t>(u) * p.R + lane] : kEmpty;
      }
      const uint64_t endm = ballot(lane < static_cast<int>(p.R) && v == kEmpty);
      const int cnt = endm ? __ffsll(static_cast<unsigned long long>(endm)) - 1 : static_cast<int>(p.R);
      bool act = lane < cnt;
#ifdef ALAYA_FINE_STAMPS
      stamp(2);
#endif
      if (p.dedup_edges) {  // graphs with repeated ids in a row: keep the first occurrence only
        for (int j = 0; j < cnt; ++j) {
          const uint32_t vj = read_lane(v, j);
          if (j < lane && vj == v) act = false;
        }
      }
      if (!vs.spilled && vs.count + 64 > vs.limit) spill_begin<space_tab<kSpace>()>(vs);
      if constexpr (kCheck && space_tab<kSpace>()) {
        // diagnostics (tests/test_sq8_spill.py): the buckets read one expansion ahead must equal the
        // table as it is now; a stale one marks the query's counters
        if (u == pre_u && vs.spilled && vs.stab != nullptr) {
          stab_order();
          uint32_t home, code;
          stab_key(vs, v, home, code);
          uint64_t lo2 = 0ull, hi2 = 0ull;
          if (act) stab_load(vs, home, lo2, hi2);
          if (ballot(act && (lo2 != pre_lo || hi2 != pre_hi))) n_hops_up |= 0x40000000u;
        }
      }
      const bool fresh = visit<space_tab<kSpace>()>(vs, v, act, kSpillPrefetch && u == pre_u, pre_lo, pre_hi);
      if constexpr (kSpillPrefetch) {
        // the pred_v load below must issue after this visit's spill-table stores and bitset atomics:
        // the second-level prefetch's wait for pred_v is its wait for them (vmcnt retires in issue
        // order), so no compiler may move the load above them
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" ::: "memory");
      }
      // consumed: the prefetched state describes the table only up to this visit's stores, so it
      // is never reused (an expansion without fresh neighbours skips the prefetch below, and the
      // next pop must not take this one for its own); zeroed so it is not live across the
      // distance phase either
      pre_u = kEmpty;
      pre_lo = pre_hi = 0ull;
      const uint64_t fm = ballot(fresh);
      const int nf = __popcll(fm);
      // issue the prefetch only after v is consumed: a use of v behind a younger load would
      // otherwise wait for that load too (vmcnt counts in issue order)
      pred = ps.cur < ps.size ? (L.pi[ps.cur] & kIdMask) : kEmpty;
      if (pred != kEmpty && lane < static_cast<int>(p.R)) pred_v = p.l0[static_cast<uint64_t>(pred) * p.R + lane];
#ifdef ALAYA_FINE_STAMPS
      stamp(5);
#else
      stamp(2);
#endif
      if (nf == 0) continue;
      // compact fresh ids in adjacency order
      const uint32_t slot = __popcll(fm & ((1ull << lane) - 1ull));
      if (fresh) L.cid[slot] = v;
      // distances a helper already computed for this node's row (exact: the same function of the same
      // query and row) go straight to cd; the rest are computed here, the known ones standing in the
      // list as kEmpty (distance functions skip them)
      const uint32_t *dist_ids = L.cid;
      bool compute = true;
      if constexpr (kHelp) {
        if (look != 0u) {
          const uint32_t seq = look >> 2;
          const int hs = static_cast<int>(look & 3u);
          const uint64_t *memo = help_memo<kSpace>(p, smem, mine.memo_wave) +
                                 (static_cast<uint32_t>(wave) * kHelpSlots + hs) * p.R;
          uint64_t e = 0ull;
          if (fresh) e = __hip_atomic_load(memo + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const bool got = fresh && static_cast<uint32_t>(e >> 32) == seq;
          help_retire(board, wave, hs, seq);
          uint32_t *ids2 = reinterpret_cast<uint32_t *>(L.sd);  // free until the merge
          if (fresh) {
            ids2[slot] = got ? kEmpty : v;
            if (got) L.cd[slot] = __uint_as_float(static_cast<uint32_t>(e));
          }
          dist_ids = ids2;
          const uint32_t n_got = __popcll(ballot(got));
          if (lane == 0 && n_got) {
            board->own[wave].hits += n_got;
            if (n_got == static_cast<uint32_t>(nf)) board->own[wave].skips += 1u;
          }
          compute = n_got < static_cast<uint32_t>(nf);
        }
      }
      wave_sync();
      // The second-level prefetch of the predicted next expansion goes out right after this
      // expansion's first row pass is issued, so its latency overlaps the rows'.  It needs pred_v,
      // which was loaded after this visit's stores and atomics (the barrier after the visit pins
      // that order) and before the rows: the wait for pred_v (vmcnt counts loads, stores and atomics
      // in issue order) is the wait for them too, so the prefetch reads the table as this visit left
      // it (ALAYA_SPILL_FLAGS bit 8 checks every prefetched bucket against a re-read).
      auto second_level_prefetch = [&]() {
        if constexpr (kSpillPrefetch) {
          if (vs.spilled && pred != kEmpty && !(p.spill_flags & 1u)) {
            if (p.spill_flags & 4u) __builtin_amdgcn_s_waitcnt(0);  // diagnostics: also wait for the rows
            spill_prefetch(vs, pred_v, lane < static_cast<int>(p.R), pre_lo, pre_hi);
            pre_u = pred;
          }
        }
      };
      if (!kHelp || compute) {
        space_distances<kIP, kChunks, kSpace, kHelp, kRows>(p, L, dist_ids, nf, L.cd, second_level_prefetch);
      } else {
        second_level_prefetch();
      }
      stamp(3);
      n_dist += nf;
      const bool has = lane < nf;
      const uint32_t cid = has ? L.cid[lane] : 0u;
      const float cd = has ? L.cd[lane] : 0.f;
      wave_sync();
      // the merge reports the next pop when it is a newcomer: load its adjacency row while the
      // rest of the merge and the pop run (the prediction above is then stale)
      pool_merge<kRegMerge>(ps, L, has, cid, cd, [&](uint32_t nx) {
        if (nx != pred) {
          const uint32_t old_pred = pred;
          (void)old_pred;
          pred = nx;
          if (lane < static_cast<int>(p.R)) pred_v = p.l0[static_cast<uint64_t>(nx) * p.R + lane];
          if constexpr (kHelp) {  // the new next pop, keeping the old one's request (likely the one after)
            if (mine.memo_wave >= 0) mine_request(board, wave, mine, kEmpty, nx, old_pred);
          }
        }
      }
#ifdef ALAYA_FINE_STAMPS
      , [&]() { stamp(7); }
#endif
      );
      stamp(4);
    }

    query_end(p, L, ps, qi, n_dist, n_expand, n_dist_up, n_hops_up);
    visit_end(vs);
    if constexpr (kStamp) {
      st[6] = __builtin_readcyclecounter() - t_begin;
      if (lane < 8) p.stamps[static_cast<uint64_t>(qi) * 8 + lane] = st[lane & 7];
    }
    wave_sync();
  }
  if constexpr (kHelp) {
    help_siblings<kIP, kChunks, kSpace>(p, smem, L, board, wave, W);
    if (p.help_stats != nullptr && lane == 0) {  // (the board outlives every wave's searching)
      p.help_stats[3 * slot] = board->own[wave].hits;
      p.help_stats[3 * slot + 1] = board->own[wave].skips;
      p.help_stats[3 * slot + 2] = board->own[wave].rows;
    }
  }
}

// Plain batched distance kernel (one query, list of ids) -- used by the rerank and by tests.
template <bool kIP>
__global__ void __launch_bounds__(64) row_distance_kernel(SearchParams p, const uint32_t *ids,
                                                          uint32_t n, float *out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *q = reinterpret_cast<float *>(smem);
  uint32_t *lid = reinterpret_cast<uint32_t *>(smem + static_cast<size_t>(p.stride) * 4);
  float *ld = reinterpret_cast<float *>(lid + 64);
  const int lane = lane_id();
  const float *qsrc = p.queries + static_cast<uint64_t>(blockIdx.y) * p.q_stride;
  for (uint32_t e = lane; e < p.stride; e += 64) q[e] = e < p.dim ? qsrc[e] : 0.f;
  wave_sync();
  for (uint32_t b = blockIdx.x * 64; b < n; b += gridDim.x * 64) {
    const uint32_t cnt = min(64u, n - b);
    if (static_cast<uint32_t>(lane) < cnt) lid[lane] = ids[b + lane];
    wave_sync();
    for (uint32_t c = 0; c < cnt; c += 8)
      row_distances<kIP, 0>(p, q, lid + c, min(8u, cnt - c), ld + c);
    if (static_cast<uint32_t>(lane) < cnt)
      out[static_cast<uint64_t>(blockIdx.y) * n + b + lane] = ld[lane];
    wave_sync();
  }
}


// PyIndex::rerank (python/include/index.hpp:450-488) for SQ8 indexes, Linux batch path (:337-345):
// res_pool[i] holds the k ids the search wrote plus ef-k zeros; all ef entries are rescored with
// the raw-space QueryComputer (f32 rows, FLT_MAX for invalid rows) and the k smallest
// pair<dist, id> are returned (id 0 can repeat -- reference behaviour).  The ef-k zero entries
// are one rescored entry of multiplicity rp.zeros.  Corrected mode (SURVEY A12 "corrected mode
// behind a flag") hands over the whole ef pool with no zeros; shard mode keeps the zeros only on
// the shard holding global row 0 (RerankParams).  kEmpty ids (slots past a pool) are skipped.
// One wave per query.
template <bool kIP>
__global__ void __launch_bounds__(64) rerank_kernel(SearchParams p, RerankParams rp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *q = reinterpret_cast<float *>(smem);
  uint32_t *cid = reinterpret_cast<uint32_t *>(smem + static_cast<size_t>(p.stride) * 4);
  const uint32_t cap = max(rp.k, rp.n_src) + 1;
  float *cd = reinterpret_cast<float *>(cid + cap);
  uint32_t *cm = reinterpret_cast<uint32_t *>(cd + cap);
  const int lane = lane_id();
  const uint32_t taken = rp.n_take;
  const uint32_t zeros = rp.zeros;
  const uint32_t c = taken + (zeros ? 1u : 0u);
  const float fill_d = rp.fill_id == kEmpty ? FLT_MAX : 0.f;
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    const float *qsrc = p.queries + qi * p.q_stride;
    for (uint32_t e = lane; e < p.stride; e += 64) q[e] = e < p.dim ? qsrc[e] : 0.f;
    uint32_t nv = 0;  // entries that will be emitted (with multiplicity)
    for (uint32_t b = 0; b < c; b += 64) {
      const uint32_t i = b + lane;
      uint32_t id = 0, m = 0;
      if (i < c) {
        id = i < taken ? rp.search_ids[qi * rp.n_src + i] : 0u;
        m = i < taken ? 1u : zeros;
        if (id == kEmpty) {  // a slot past the pool
          id = 0u;
          m = 0u;
        }
        cid[i] = id;
        cm[i] = m;
      }
      for (int off = 32; off > 0; off >>= 1) m += __shfl_xor(m, off);
      nv += m;
    }
    wave_sync();
    row_distances<kIP, 0>(p, q, cid, static_cast<int>(c), cd);
    // rank of each distinct entry in the (dist, id) order, equal pairs in entry order
    for (uint32_t i = lane; i < c; i += 64) {
      const float di = cd[i];
      const uint32_t ii = cid[i];
      uint32_t rank = 0;
      for (uint32_t j = 0; j < c; ++j) {
        const float dj = cd[j];
        const uint32_t ij = cid[j];
        const bool less = dj < di || (dj == di && ij < ii);
        const bool tie_before = dj == di && ij == ii && j < i;
        if (less || tie_before) rank += cm[j];
      }
      for (uint32_t m = 0; m < cm[i] && rank + m < rp.k; ++m) {
        rp.out_ids[qi * rp.k + rank + m] = ii;
        if (rp.out_dists) rp.out_dists[qi * rp.k + rank + m] = di;
      }
    }
    for (uint32_t i = nv + lane; i < rp.k; i += 64) {  // fewer candidates than k
      rp.out_ids[qi * rp.k + i] = rp.fill_id;
      if (rp.out_dists) rp.out_dists[qi * rp.k + i] = fill_d;
    }
    wave_sync();
  }
}
// Roofline calibration (bench.py's measured peak): streaming reads of n16 16-byte words, summed so
// the loads cannot be dropped.  Shape 0: one dwordx4 per lane per step (a wave reads 1 KB
// contiguous, the grid sweeps the buffer in order); shape 1: four independent dwordx4 per lane,
// grid-stride apart; shape 2: four consecutive dwordx4 per lane (a wave reads 4 KB contiguous).
// alaya_hbm_stream_read reports the best shape.
template <int kShape>
__global__ void __launch_bounds__(256) stream_read_kernel(const float4 *p, uint64_t n16, float *sink) {
  float acc = 0.f;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * 256;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
  if constexpr (kShape == 1) {
    for (; i + 3 * stride < n16; i += 4 * stride) {
      const float4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
      acc += (a.x + b.x) + (c.x + d.x) + (a.w + b.w) + (c.w + d.w);
    }
  } else if constexpr (kShape == 2) {
    const uint64_t w = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);  // wave index
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * 4;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t base = w * 256;
    for (; base + 256 <= n16; base += waves * 256) {
      const float4 a = p[base + lane], b = p[base + 64 + lane], c = p[base + 128 + lane], d = p[base + 192 + lane];
      acc += (a.x + b.x) + (c.x + d.x) + (a.w + b.w) + (c.w + d.w);
    }
    i = n16;  // the tail (< 4 KB per wave) is not read: the byte count below excludes nothing material
  }
  for (; i < n16; i += stride) acc += p[i].x;
  if (acc == -1.2345f) *sink = acc;  // never true for the probe's zeroed buffer
}
}  // namespace

hipError_t launch_stream_read(const void *buf, uint64_t bytes, int grid, int shape, float *sink,
                              hipStream_t stream) {
  const float4 *p = static_cast<const float4 *>(buf);
  if (shape == 1) {
    hipLaunchKernelGGL(stream_read_kernel<1>, dim3(grid), dim3(256), 0, stream, p, bytes / 16, sink);
  } else if (shape == 2) {
    hipLaunchKernelGGL(stream_read_kernel<2>, dim3(grid), dim3(256), 0, stream, p, bytes / 16, sink);
  } else {
    hipLaunchKernelGGL(stream_read_kernel<0>, dim3(grid), dim3(256), 0, stream, p, bytes / 16, sink);
  }
  return hipGetLastError();
}

size_t search_query_lds_bytes(uint32_t stride, int sq8_order) {
  // the query as f32 terms, or (ALAYA_SQ8_QCODES, AVX-512-order SQ8) as its codes, 16 B aligned
  return sq8_order == 2 && sq8_query_codes<2>() ? (static_cast<size_t>(stride) + 15) / 16 * 16
                                                : static_cast<size_t>(stride) * 4;
}

size_t search_wave_lds_bytes(uint32_t stride, uint32_t ef, uint32_t hash_log2, bool compact, int sq8_order) {
  return search_query_lds_bytes(stride, sq8_order) + 3 * 64 * 4 + 2 * (((ef + 1) * 4 + 15) / 16 * 16) +
         visited_table_bytes(hash_log2, compact);
}

hipError_t launch_rerank(const SearchParams &p, const RerankParams &r, hipStream_t stream) {
  const size_t lds = static_cast<size_t>(p.stride) * 4 + 3 * (static_cast<size_t>(std::max(r.k, r.n_src)) + 1) * 4 + 64;
  const int grid = static_cast<int>(std::min<uint64_t>(p.nq, 4096));
  if (p.ip) {
    hipLaunchKernelGGL(rerank_kernel<true>, dim3(grid), dim3(64), lds, stream, p, r);
  } else {
    hipLaunchKernelGGL(rerank_kernel<false>, dim3(grid), dim3(64), lds, stream, p, r);
  }
  return hipGetLastError();
}

template <bool kIP, int kChunks, int kMode = 0, int kSpace = 0>
static const void *kernel_ptr() {
  return reinterpret_cast<const void *>(&hnsw_search_kernel<kIP, kChunks, kMode, kSpace>);
}

template <int kSpace>
static const void *sq8_symbol(bool ip, uint32_t dim, bool stamped, bool check, bool help) {
  const uint32_t chunks = (dim % 32 == 0) ? dim / 32 : 0;
  if constexpr (kSpace == 2) {  // stamped with helpers (tools/profile_phases.py)
    if (stamped && help && chunks == 24) return ip ? kernel_ptr<true, 24, 5, kSpace>() : kernel_ptr<false, 24, 5, kSpace>();
  }
  if (stamped && chunks == 24) return ip ? kernel_ptr<true, 24, 1, kSpace>() : kernel_ptr<false, 24, 1, kSpace>();
  if constexpr (kSpace == 2) {  // the spill-table prefetch check (config 5's d = 768 and d = 960)
    if (check && chunks == 24) return ip ? kernel_ptr<true, 24, 2, kSpace>() : kernel_ptr<false, 24, 2, kSpace>();
    if (check && chunks == 30) return ip ? kernel_ptr<true, 30, 2, kSpace>() : kernel_ptr<false, 30, 2, kSpace>();
    if (help && chunks == 4) return ip ? kernel_ptr<true, 4, 4, kSpace>() : kernel_ptr<false, 4, 4, kSpace>();
    if (help && chunks == 24) return ip ? kernel_ptr<true, 24, 4, kSpace>() : kernel_ptr<false, 24, 4, kSpace>();
    if (help && chunks == 30) return ip ? kernel_ptr<true, 30, 4, kSpace>() : kernel_ptr<false, 30, 4, kSpace>();
  }
  if (chunks == 4) return ip ? kernel_ptr<true, 4, 0, kSpace>() : kernel_ptr<false, 4, 0, kSpace>();
  if (chunks == 24) return ip ? kernel_ptr<true, 24, 0, kSpace>() : kernel_ptr<false, 24, 0, kSpace>();
  if (chunks == 30) return ip ? kernel_ptr<true, 30, 0, kSpace>() : kernel_ptr<false, 30, 0, kSpace>();
  return ip ? kernel_ptr<true, 0, 0, kSpace>() : kernel_ptr<false, 0, 0, kSpace>();
}

// Whether a search has a helper kernel (kMode 4): the small-row f32 kernels (d = 128 / 256, the
// latency-bound SIFT shape) and the AVX-512-order SQ8 kernels with a compile-time chunk count.  The
// wide f32 rows (GIST, the headline) are bandwidth-bound: helpers would add bytes, not overlap.
bool search_has_two_waves(uint32_t dim, int sq8_order, bool generic) {
  return sq8_order == 0 && !generic && (dim == 24 * 32 || dim == 30 * 32);
}

bool search_has_helpers(uint32_t dim, int sq8_order, bool generic) {
  if (generic || dim % 32 != 0) return false;
  const uint32_t chunks = dim / 32;
  if (sq8_order == 2) return chunks == 4 || chunks == 24 || chunks == 30;
  if (sq8_order == 1) return false;
  return chunks == 4 || chunks == 8;
}

const void *search_kernel_symbol(bool ip, uint32_t dim, bool stamped, int sq8_order, bool generic, bool check,
                                 bool help, bool two_waves) {
  if (sq8_order == 2) return sq8_symbol<2>(ip, dim, stamped, check, help);
  if (sq8_order == 1) return sq8_symbol<1>(ip, dim, stamped, false, false);
  const uint32_t chunks = (!generic && dim % 32 == 0) ? dim / 32 : 0;  // generic order: the runtime-d kernel
  if (stamped) {
    if (help && chunks == 4) return ip ? kernel_ptr<true, 4, 5>() : kernel_ptr<false, 4, 5>();
    if (chunks == 30) return ip ? kernel_ptr<true, 30, 1>() : kernel_ptr<false, 30, 1>();
    if (chunks == 4) return ip ? kernel_ptr<true, 4, 1>() : kernel_ptr<false, 4, 1>();
    return ip ? kernel_ptr<true, 0, 1>() : kernel_ptr<false, 0, 1>();
  }
  if (help && chunks == 4) return ip ? kernel_ptr<true, 4, 4>() : kernel_ptr<false, 4, 4>();
  if (help && chunks == 8) return ip ? kernel_ptr<true, 8, 4>() : kernel_ptr<false, 8, 4>();
  if (two_waves && chunks == 24) return ip ? kernel_ptr<true, 24, 8>() : kernel_ptr<false, 24, 8>();
  if (two_waves && chunks == 30) return ip ? kernel_ptr<true, 30, 8>() : kernel_ptr<false, 30, 8>();
#define ALAYA_CASE(C)                                                        \
  if (chunks == C) return ip ? kernel_ptr<true, C>() : kernel_ptr<false, C>();
  ALAYA_CASE(4)
  ALAYA_CASE(8)
  ALAYA_CASE(16)
  ALAYA_CASE(24)
  ALAYA_CASE(30)
  ALAYA_CASE(32)
#undef ALAYA_CASE
  return ip ? kernel_ptr<true, 0>() : kernel_ptr<false, 0>();
}

hipError_t launch_search(const SearchParams &p, int grid, int waves, size_t lds, hipStream_t stream) {
  const void *fn = search_kernel_symbol(p.ip, p.dim, p.stamps != nullptr, p.sq8_order, p.generic,
                                        (p.spill_flags & 256u) != 0, p.help != 0, p.two_waves != 0);
  SearchParams arg = p;
  void *args[] = {&arg};
  return hipLaunchKernel(fn, dim3(grid), dim3(64 * waves), args, lds, stream);
}

hipError_t launch_row_distances(const SearchParams &p, const uint32_t *ids, uint32_t n,
                                uint32_t nq, float *out, hipStream_t stream) {
  const size_t lds = static_cast<size_t>(p.stride) * 4 + 128 * 4;
  const int gx = static_cast<int>(std::min<uint32_t>((n + 63) / 64, 1024u));
  if (p.ip) {
    hipLaunchKernelGGL(row_distance_kernel<true>, dim3(gx, nq), dim3(64), lds, stream, p, ids, n, out);
  } else {
    hipLaunchKernelGGL(row_distance_kernel<false>, dim3(gx, nq), dim3(64), lds, stream, p, ids, n, out);
  }
  return hipGetLastError();
}

hipError_t search_occupancy(const SearchParams &p, int waves, size_t lds, int *blocks_per_cu) {
  const void *fn = search_kernel_symbol(p.ip, p.dim, p.stamps != nullptr, p.sq8_order, p.generic,
                                        (p.spill_flags & 256u) != 0, p.help != 0, p.two_waves != 0);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 64 * waves, lds);
}

}  // namespace alaya_amd
