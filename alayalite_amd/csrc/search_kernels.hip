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

namespace alaya_amd {

namespace {

constexpr uint32_t kEmpty = 0xffffffffu;
constexpr uint32_t kChecked = 0x80000000u;
constexpr uint32_t kIdMask = 0x7fffffffu;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_sync() {
  // One workgroup == one wave.  LDS instructions of a wave execute in order, so a lane's ds_write
  // is seen by a later ds_read of any lane; this fence only stops the compiler from reordering LDS
  // accesses across it and, unlike __syncthreads(), does not drain outstanding global loads.
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t hash_slot(uint32_t v, uint32_t log2h) {
  return (v * 0x9E3779B1u) >> (32 - log2h);
}

struct Lds {
  float *q;          // stride floats
  float *pd;         // ef + 1 pool distances
  uint32_t *pi;      // ef + 1 pool ids (bit 31 = checked)
  uint32_t *hash;    // 1 << hash_log2 visited slots
  uint32_t *cid;     // 64 candidate ids (adjacency order)
  float *cd;         // 64 candidate distances
  float *sd;         // 64 sorted accepted distances
  float *sq_scale;   // SQ8: per-dimension scale (nullptr for f32 search)
  float *sq_min;     // SQ8: per-dimension min
};

// Distance of the query to candidate rows in the index's search space.
template <bool kIP, int kChunks, int kSpace>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out);

template <bool kIP>
__device__ __forceinline__ void accumulate(const float4 x, const float4 y, float &a0, float &a1,
                                           float &a2, float &a3) {
  if (kIP) {  // acc = fma(x, y, acc)              (distance_ip.ipp:82-85)
    a0 = fmaf(x.x, y.x, a0); a1 = fmaf(x.y, y.y, a1);
    a2 = fmaf(x.z, y.z, a2); a3 = fmaf(x.w, y.w, a3);
  } else {    // diff = x - y; acc = fma(diff, diff, acc)  (distance_l2.ipp:74-83)
    const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
    a0 = fmaf(d0, d0, a0); a1 = fmaf(d1, d1, a1);
    a2 = fmaf(d2, d2, a2); a3 = fmaf(d3, d3, a3);
  }
}

// --------------------------------------------------------------------------------------------
// Distance of the query (LDS) to `n` rows listed in ids[0..n) -> out[0..n).
// 8 lanes per row (lane m of the group owns partial sums acc[4m..4m+3]); each lane group of a
// pass handles kRPL rows, so one pass covers 8*kRPL rows and issues every 128 B row chunk of
// the pass before the first FMA (all loads of the pass in flight at once).
// --------------------------------------------------------------------------------------------
template <bool kIP>
__device__ __forceinline__ float finish_row(float a0, float a1, float a2, float a3) {
  // (acc0+acc1) + (acc2+acc3) per lane of the 8-wide vector: lanes m^2 then m^4.
  a0 += __shfl_xor(a0, 2); a1 += __shfl_xor(a1, 2); a2 += __shfl_xor(a2, 2); a3 += __shfl_xor(a3, 2);
  a0 += __shfl_xor(a0, 4); a1 += __shfl_xor(a1, 4); a2 += __shfl_xor(a2, 4); a3 += __shfl_xor(a3, 4);
  // lane m==0 holds v[0..3], lane m==1 holds v[4..7]: s[j] = v[j] + v[j+4]; r = (s0+s1)+(s2+s3)
  const float s0 = a0 + __shfl_xor(a0, 1), s1 = a1 + __shfl_xor(a1, 1);
  const float s2 = a2 + __shfl_xor(a2, 1), s3 = a3 + __shfl_xor(a3, 1);
  return (s0 + s1) + (s2 + s3);
}

template <bool kIP>
__device__ __forceinline__ float finish_tail(const SearchParams &p, const float *q, const float *row,
                                             int tail_begin, float res, uint32_t id) {
  for (int e = tail_begin; e < static_cast<int>(p.dim); ++e) {
    if (kIP) {
      res = fmaf(q[e], row[e], res);
    } else {
      const float d = q[e] - row[e];
      res = fmaf(d, d, res);
    }
  }
  if (kIP) res = -res;
  if (p.valid != nullptr && !((p.valid[id >> 5] >> (id & 31)) & 1u)) res = FLT_MAX;
  return res;
}

// rows per lane group per pass for a compile-time chunk count: keep the hoisted row chunks
// within ~96 float4 (384 VGPRs) -- one wave per SIMD has the whole 512-entry register file.
template <int kChunks>
constexpr int rows_per_group() {
  return kChunks <= 0 ? 1 : (96 / kChunks >= 4 ? 4 : (96 / kChunks < 1 ? 1 : 96 / kChunks));
}

template <bool kIP, int kChunks>
__device__ __forceinline__ void row_distances(const SearchParams &p, const float *q,
                                              const uint32_t *ids, int n, float *out) {
  const int lane = lane_id();
  const int g = lane >> 3, m = lane & 7;
  const int T = kChunks > 0 ? kChunks : static_cast<int>(p.dim >> 5);
  const int rem = static_cast<int>(p.dim) - 32 * T;
  const int nb8 = rem >> 3;
  const int tail_begin = 32 * T + 8 * nb8;
  if constexpr (kChunks > 0) {
    constexpr int kRPL = rows_per_group<kChunks>();
    for (int base = 0; base < n; base += 8 * kRPL) {
      uint32_t id[kRPL];
      bool act[kRPL];
      const float *row[kRPL];
      float4 y[kRPL][kChunks];
#pragma unroll
      for (int r = 0; r < kRPL; ++r) {
        const int idx = base + g + 8 * r;
        act[r] = idx < n;
        id[r] = act[r] ? ids[idx] : 0u;
        row[r] = p.base + static_cast<uint64_t>(id[r]) * p.stride;
      }
#pragma unroll
      for (int r = 0; r < kRPL; ++r) {
        const float4 *rp = reinterpret_cast<const float4 *>(row[r]) + m;
        if (act[r]) {
#pragma unroll
          for (int t = 0; t < kChunks; ++t) y[r][t] = rp[8 * t];
        } else {
#pragma unroll
          for (int t = 0; t < kChunks; ++t) y[r][t] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      float a[kRPL][4];
#pragma unroll
      for (int r = 0; r < kRPL; ++r) a[r][0] = a[r][1] = a[r][2] = a[r][3] = 0.f;
      const float4 *qp = reinterpret_cast<const float4 *>(q) + m;
#pragma unroll
      for (int t = 0; t < kChunks; ++t) {
        const float4 x = qp[8 * t];
#pragma unroll
        for (int r = 0; r < kRPL; ++r) accumulate<kIP>(x, y[r][t], a[r][0], a[r][1], a[r][2], a[r][3]);
      }
#pragma unroll
      for (int r = 0; r < kRPL; ++r) {
        if (m < 2) {  // trailing 8-element blocks feed acc[0..7] (lanes m = 0, 1)
          for (int b = 0; b < nb8; ++b) {
            const int e = 32 * T + 8 * b + 4 * m;
            if (act[r]) {
              accumulate<kIP>(*reinterpret_cast<const float4 *>(q + e),
                              *reinterpret_cast<const float4 *>(row[r] + e), a[r][0], a[r][1], a[r][2], a[r][3]);
            }
          }
        }
        const float res = finish_row<kIP>(a[r][0], a[r][1], a[r][2], a[r][3]);
        if (act[r] && m == 0) out[base + g + 8 * r] = finish_tail<kIP>(p, q, row[r], tail_begin, res, id[r]);
      }
    }
  } else {
    for (int base = 0; base < n; base += 8) {
      const int r = base + g;
      const bool act = r < n;
      const uint32_t id = act ? ids[r] : 0u;
      const float *row = p.base + static_cast<uint64_t>(id) * p.stride;
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      if (act) {
        const float4 *rp = reinterpret_cast<const float4 *>(row) + m;
        const float4 *qp = reinterpret_cast<const float4 *>(q) + m;
#pragma unroll 8
        for (int t = 0; t < T; ++t) accumulate<kIP>(qp[8 * t], rp[8 * t], a0, a1, a2, a3);
        if (m < 2) {
          for (int b = 0; b < nb8; ++b) {
            const int e = 32 * T + 8 * b + 4 * m;
            accumulate<kIP>(*reinterpret_cast<const float4 *>(q + e),
                            *reinterpret_cast<const float4 *>(row + e), a0, a1, a2, a3);
          }
        }
      }
      const float res = finish_row<kIP>(a0, a1, a2, a3);
      if (act && m == 0) out[r] = finish_tail<kIP>(p, q, row, tail_begin, res, id);
    }
  }
  wave_sync();
}

// --------------------------------------------------------------------------------------------
// SQ8 distances (SQ8Space::QueryComputer over l2_sqr_sq8 / ip_sqr_sq8).  The reference picks the
// AVX-512 kernel when the host has AVX-512F, else AVX2 (distance_l2.ipp:694-708,
// distance_ip.ipp:703-716).  Both are "P partial sums, element P*t+j -> acc[j]":
//   AVX-512 (:334-408 / :292-366): P = 32 (sum0 = acc[0..15], sum1 = acc[16..31]); a trailing
//     16-block feeds acc[0..15]; combine a = sum0+sum1, then GCC 11 _mm512_reduce_add_ps:
//     T3[j] = a[8+j]+a[j], T6[j] = T3[4+j]+T3[j], r = (T6[0]+T6[2]) + (T6[1]+T6[3]).
//   AVX2 (:244-329 / :198-287): P = 16 (sum0 = acc[0..7], sum1 = acc[8..15]); a trailing 8-block
//     feeds acc[0..7]; combine v = sum0+sum1, s[j] = v[j]+v[j+4], r = (s0+s1)+(s2+s3).
// Per element: scale = (max-min)*(1/255); L2: d = (x-y)*scale, acc = fma(d,d,acc);
// IP: xv = fma(x,scale,min), yv = fma(y,scale,min), acc = fma(xv,yv,acc).  Scalar tail the same.
// Two lanes per row (lane h owns acc[h*P/2 ...]): one pass covers 32 rows.  LDS holds, per
// dimension, the query term (x for L2, xv for IP), scale and min.
// --------------------------------------------------------------------------------------------
template <bool kIP>
__device__ __forceinline__ float sq8_term(float xq, float scale, float mn, float yf, float acc) {
  if (kIP) return fmaf(xq, fmaf(yf, scale, mn), acc);
  const float d = (xq - yf) * scale;
  return fmaf(d, d, acc);
}

template <bool kIP, int kOrder, int kFull>
__device__ __forceinline__ void sq8_distances(const SearchParams &p, const float *xq,
                                              const float *sc, const float *mnv,
                                              const uint32_t *ids, int n, float *out) {
  constexpr int P = kOrder == 2 ? 32 : 16;
  constexpr int H = P / 2;
  constexpr int W = H / 4;  // 32-bit words per lane per chunk
  const int lane = lane_id();
  const int g = lane >> 1, h = lane & 1;
  const int T = kFull > 0 ? kFull : static_cast<int>(p.dim) / P;
  const int rem = static_cast<int>(p.dim) - P * T;
  const bool half = rem >= H;
  const int tail_begin = P * T + (half ? H : 0);
  for (int base = 0; base < n; base += 32) {
    const int r = base + g;
    const bool act = r < n;
    const uint32_t id = act ? ids[r] : 0u;
    const uint8_t *row = p.codes + static_cast<uint64_t>(id) * p.code_stride;
    float acc[H];
#pragma unroll
    for (int l = 0; l < H; ++l) acc[l] = 0.f;
    auto chunk = [&](int t, const uint32_t *w, int hh) {
#pragma unroll
      for (int l = 0; l < H; ++l) {
        const int e = P * t + H * hh + l;
        const float yf = static_cast<float>((w[l >> 2] >> (8 * (l & 3))) & 0xffu);
        acc[l] = sq8_term<kIP>(xq[e], sc[e], mnv[e], yf, acc[l]);
      }
    };
    if (act) {
      if constexpr (kFull > 0) {
        uint32_t w[kFull][W];
#pragma unroll
        for (int t = 0; t < kFull; ++t) {
          const uint32_t *src = reinterpret_cast<const uint32_t *>(row + P * t + H * h);
#pragma unroll
          for (int q = 0; q < W; ++q) w[t][q] = src[q];
        }
#pragma unroll
        for (int t = 0; t < kFull; ++t) chunk(t, w[t], h);
      } else {
        for (int t = 0; t < T; ++t) {
          uint32_t w[W];
          const uint32_t *src = reinterpret_cast<const uint32_t *>(row + P * t + H * h);
#pragma unroll
          for (int q = 0; q < W; ++q) w[q] = src[q];
          chunk(t, w, h);
        }
      }
      if (half && h == 0) {  // trailing half block -> sum0
        uint32_t w[W];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(row + P * T);
#pragma unroll
        for (int q = 0; q < W; ++q) w[q] = src[q];
        chunk(T, w, 0);
      }
    }
    float res;
#pragma unroll
    for (int l = 0; l < H; ++l) acc[l] += __shfl_xor(acc[l], 1);  // sum0 + sum1
    if constexpr (kOrder == 2) {
      float t3[8], t6[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) t3[j] = acc[8 + j] + acc[j];
#pragma unroll
      for (int j = 0; j < 4; ++j) t6[j] = t3[4 + j] + t3[j];
      res = (t6[0] + t6[2]) + (t6[1] + t6[3]);
    } else {
      float s4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) s4[j] = acc[j] + acc[j + 4];
      res = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
    if (act && h == 0) {
      for (int e = tail_begin; e < static_cast<int>(p.dim); ++e)
        res = sq8_term<kIP>(xq[e], sc[e], mnv[e], static_cast<float>(row[e]), res);
      out[r] = kIP ? -res : res;  // no validity check in SQ8Space::QueryComputer
    }
  }
  wave_sync();
}

template <bool kIP, int kChunks, int kSpace>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out) {
  if constexpr (kSpace == 0) {
    row_distances<kIP, kChunks>(p, L.q, ids, n, out);
  } else {
    sq8_distances<kIP, kSpace, kSpace == 2 ? kChunks : 2 * kChunks>(p, L.q, L.sq_scale, L.sq_min, ids, n, out);
  }
}

// --------------------------------------------------------------------------------------------
// Visited set: exact (DynamicBitset semantics, query_utils.hpp:69-115).  First level: an LDS
// open-addressing table with linear probing.  Two layouts:
//   wide    -- 32-bit slots holding the id (kEmpty = free);
//   compact -- 16-bit slots.  h = (v * C) mod 2^L is a bijection on [0, 2^L) (C odd,
//              L = vis_lbits >= log2 n); the home slot is the top log2h bits of h and the slot
//              stores 1 + (probe distance << rbits | low rbits bits of h), so (slot, entry)
//              identifies v exactly in half the bytes: twice the entries per LDS byte.
// When the table passes its load limit (or a compact probe would exceed the encodable distance)
// the query spills: a per-slot global N-bit bitset becomes the second level (atomicOr).
// --------------------------------------------------------------------------------------------
struct Visited {
  uint32_t *tab;
  uint32_t log2h;
  uint32_t count;        // wave-uniform number of entries in the LDS table
  uint32_t limit;        // switch to the global bitset above this many entries
  bool spilled;          // wave-uniform
  uint32_t *bits;        // per-slot global bitset (valid when spilled)
  uint32_t rbits;        // compact: remainder bits; kVisWide: 32-bit slots
  uint32_t lmask;        // compact: 2^L - 1
  uint32_t lshift;       // compact, L < log2h: home = h << lshift
  uint32_t max_disp;     // compact: largest encodable probe distance
};

__device__ __forceinline__ Visited make_visited(const SearchParams &p, uint32_t *tab, uint32_t *bits) {
  Visited vs;
  vs.tab = tab;
  vs.log2h = p.hash_log2;
  vs.count = 0u;
  vs.spilled = false;
  vs.bits = bits;
  vs.rbits = p.vis_rbits;
  const uint32_t hsize = 1u << p.hash_log2;
  if (p.vis_rbits == kVisWide) {
    vs.limit = hsize / 2;
    vs.lmask = vs.lshift = vs.max_disp = 0u;
  } else {
    vs.limit = hsize - hsize / 4 - hsize / 16;  // load factor 0.69
    vs.lmask = p.vis_lbits >= 32 ? 0xffffffffu : (1u << p.vis_lbits) - 1u;
    vs.lshift = p.vis_lbits < p.hash_log2 ? p.hash_log2 - p.vis_lbits : 0u;
    vs.max_disp = p.vis_max_disp;
  }
  return vs;
}

__device__ __forceinline__ void compact_key(const Visited &vs, uint32_t v, uint32_t &home, uint32_t &rem) {
  const uint32_t h = (v * 0x9E3779B1u) & vs.lmask;
  if (vs.rbits) {
    home = h >> vs.rbits;
    rem = h & ((1u << vs.rbits) - 1u);
  } else {
    home = h << vs.lshift;
    rem = 0u;
  }
}

__device__ __forceinline__ bool table_lookup(const Visited &vs, uint32_t v) {
  const uint32_t mask = (1u << vs.log2h) - 1u;
  if (vs.rbits == kVisWide) {
    uint32_t h = hash_slot(v, vs.log2h);
    for (;;) {
      const uint32_t e = vs.tab[h];
      if (e == v) return true;
      if (e == kEmpty) return false;
      h = (h + 1) & mask;
    }
  }
  uint32_t home, rem;
  compact_key(vs, v, home, rem);
  const uint16_t *t16 = reinterpret_cast<const uint16_t *>(vs.tab);
  for (uint32_t i = 0;; ++i) {
    const uint32_t e = t16[(home + i) & mask];
    if (e == 0u) return false;
    if (e == 1u + ((i << vs.rbits) | rem)) return true;
    if (i == vs.max_disp) return false;  // inserts never go further
  }
}

// Insert into the LDS table.  Returns 1 = inserted (fresh), 0 = already present, 2 = compact probe
// ran past max_disp (not present, not inserted: the caller spills).
__device__ __forceinline__ int table_insert(const Visited &vs, uint32_t v) {
  const uint32_t mask = (1u << vs.log2h) - 1u;
  if (vs.rbits == kVisWide) {
    uint32_t h = hash_slot(v, vs.log2h);
    for (;;) {
      const uint32_t old = atomicCAS(&vs.tab[h], kEmpty, v);
      if (old == kEmpty) return 1;
      if (old == v) return 0;
      h = (h + 1) & mask;
    }
  }
  uint32_t home, rem;
  compact_key(vs, v, home, rem);
  for (uint32_t i = 0; i <= vs.max_disp; ++i) {
    const uint32_t slot = (home + i) & mask;
    uint32_t *w = &vs.tab[slot >> 1];
    const uint32_t sh = (slot & 1u) * 16u;
    const uint32_t mine = 1u + ((i << vs.rbits) | rem);
    uint32_t cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
      const uint32_t e = (cur >> sh) & 0xffffu;
      if (e == mine) return 0;
      if (e != 0u) break;  // occupied by another key: next slot
      const uint32_t old = atomicCAS(w, cur, cur | (mine << sh));
      if (old == cur) return 1;
      cur = old;  // the other half of the word (or this slot) changed: re-examine
    }
  }
  return 2;
}

__device__ void spill_begin(Visited &vs, uint64_t n_words) {
  // zero this slot's global bitset once, then keep the LDS table as a read-only first level.
  const int lane = lane_id();
  for (uint64_t w = lane; w < n_words; w += 64) vs.bits[w] = 0u;
  __threadfence_block();
  wave_sync();
  vs.spilled = true;
}

__device__ __forceinline__ bool global_visit(const Visited &vs, uint32_t v) {
  const uint32_t bit = 1u << (v & 31);
  const uint32_t old = atomicOr(&vs.bits[v >> 5], bit);
  return (old & bit) == 0u;
}

// All lanes with `act` insert their v; duplicates among lanes must have been removed.
__device__ __forceinline__ bool visit(Visited &vs, uint32_t v, bool act, uint64_t n_words) {
  bool fresh = false;
  if (!vs.spilled) {
    int r = 0;
    if (act) r = table_insert(vs, v);
    fresh = r == 1;
    vs.count += __popcll(ballot(fresh));
    if (ballot(r == 2)) {  // a compact probe ran out of encodable distance: spill now
      spill_begin(vs, n_words);
      if (r == 2) fresh = global_visit(vs, v);
    }
  } else if (act) {
    if (!table_lookup(vs, v)) fresh = global_visit(vs, v);
  }
  return fresh;
}

// --------------------------------------------------------------------------------------------
// Pool (LinearPool).  size/cur are wave-uniform.  Checked flag lives in bit 31 of the id.
// --------------------------------------------------------------------------------------------
struct PoolState {
  uint32_t size;
  uint32_t cur;
  uint32_t ef;
};

// number of pool entries with dist <= d (find_bsearch, strict '>' keeps equal ones first)
__device__ __forceinline__ uint32_t pool_upper_bound(const float *pd, uint32_t size, float d) {
  uint32_t lo = 0, hi = size;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pd[mid] > d) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// number of sorted batch distances strictly below d
__device__ __forceinline__ uint32_t batch_lower_bound(const float *sd, uint32_t n, float d) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sd[mid] < d) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Merge candidates held by lanes 0..nb-1 (arrival order = lane order, nb <= 64) into the pool.
// Equivalent to calling LinearPool::insert(id_i, d_i) for i = 0..nb-1 in order.
__device__ void pool_merge(PoolState &ps, const Lds &L, bool has, uint32_t id, float d) {
  const int lane = lane_id();
  const bool full = ps.size == ps.ef;
  const float last = full ? L.pd[ps.size - 1] : 0.f;
  const bool acc = has && !(full && d >= last);
  const uint64_t amask = ballot(acc);
  const uint32_t n_acc = __popcll(amask);
  if (n_acc == 0) return;
  // stable rank of this candidate among accepted ones, ordered by (dist, arrival)
  uint32_t rank = 0;
  uint64_t rest = amask;
  while (rest) {
    const int j = __ffsll(static_cast<unsigned long long>(rest)) - 1;
    rest &= rest - 1;
    const float dj = __shfl(d, j);
    rank += (dj < d || (dj == d && j < lane)) ? 1u : 0u;
  }
  if (acc) L.sd[rank] = d;
  uint32_t pos = 0;
  if (acc) pos = pool_upper_bound(L.pd, ps.size, d) + rank;
  // first insertion position = position of the rank-0 element
  const uint32_t first_pos = __shfl(pos, __ffsll(static_cast<unsigned long long>(ballot(acc && rank == 0))) - 1);
  wave_sync();
  // shift pool entries [first_pos, size) up by #accepted strictly smaller, top chunk first.
  for (int hi = static_cast<int>(ps.size); hi > static_cast<int>(first_pos); hi -= 64) {
    const int j = hi - 64 + lane;
    const bool mv = j >= static_cast<int>(first_pos);
    float pdj = 0.f;
    uint32_t pij = 0;
    uint32_t dest = 0;
    if (mv) {
      pdj = L.pd[j];
      pij = L.pi[j];
      dest = static_cast<uint32_t>(j) + batch_lower_bound(L.sd, n_acc, pdj);
    }
    wave_sync();
    if (mv && dest < ps.ef) {
      L.pd[dest] = pdj;
      L.pi[dest] = pij;
    }
    wave_sync();
  }
  if (acc && pos < ps.ef) {
    L.pd[pos] = d;
    L.pi[pos] = id;
  }
  wave_sync();
  ps.size = min(ps.size + n_acc, ps.ef);
  if (first_pos < ps.cur) ps.cur = first_pos;
}

// LinearPool::pop: mark cur checked, advance to the next unchecked entry.
__device__ __forceinline__ uint32_t pool_pop(PoolState &ps, const Lds &L) {
  const int lane = lane_id();
  const uint32_t raw = L.pi[ps.cur];
  wave_sync();
  if (lane == 0) L.pi[ps.cur] = raw | kChecked;
  uint32_t next = ps.size;
  for (uint32_t b = ps.cur + 1; b < ps.size; b += 64) {
    const uint32_t j = b + lane;
    const bool un = j < ps.size && !(L.pi[j] & kChecked);
    const uint64_t mk = ballot(un);
    if (mk) {
      next = b + __ffsll(static_cast<unsigned long long>(mk)) - 1;
      break;
    }
  }
  wave_sync();
  ps.cur = next;
  return raw & kIdMask;
}

// --------------------------------------------------------------------------------------------
// The search kernel.
// --------------------------------------------------------------------------------------------
// kStamp: diagnostic build that accumulates s_memtime cycles per phase into p.stamps (nq x 8):
// [0] init + overlay descent, [1] pop, [2] adjacency load + visited set, [3] distances,
// [4] merge, [5] expansions after the visited table spilled, [6] whole query, [7] prefetch hits.
template <bool kIP, int kChunks, bool kStamp, int kSpace = 0>
__global__ void __launch_bounds__(64) hnsw_search_kernel(SearchParams p) {
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
    ptr += static_cast<size_t>(p.vis_rbits != kVisWide ? 2 : 4) << p.hash_log2;
    L.sq_scale = kSpace ? reinterpret_cast<float *>(ptr) : nullptr;
    ptr += kSpace ? static_cast<size_t>(p.stride) * 4 : 0;
    L.sq_min = kSpace ? reinterpret_cast<float *>(ptr) : nullptr;
  }
  const uint32_t hsize = 1u << p.hash_log2;
  const uint64_t bit_words = (p.n + 31) / 32;
  uint32_t *slot_bits = p.overflow_bits + static_cast<uint64_t>(blockIdx.x) * bit_words;

  for (;;) {
    uint32_t qi = 0;
    if (lane == 0) qi = atomicAdd(p.work_counter, 1u);
    qi = __shfl(qi, 0);
    if (qi >= p.nq) break;

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
    // ---- per-query init ------------------------------------------------------------------
    const float *qsrc = p.queries + static_cast<uint64_t>(qi) * p.q_stride;
    if constexpr (kSpace == 0) {
      for (uint32_t e = lane; e < p.stride; e += 64) L.q[e] = e < p.dim ? qsrc[e] : 0.f;
    } else {
      // SQ8Space::QueryComputer encodes the query with the quantizer (sq8_space.hpp:266-271,
      // SQ8Quantizer::quantize sq8.hpp:118-130), then every distance uses its codes.
      const float kInv255 = 1.0f / 255.0f;
      for (uint32_t e = lane; e < p.stride; e += 64) {
        float xq = 0.f, sc = 0.f, mn = 0.f;
        if (e < p.dim) {
          const float v = qsrc[e];
          mn = p.sq_min[e];
          const float mx = p.sq_max[e];
          uint32_t code;
          if (mx == mn) code = 0;
          else if (v >= mx) code = 255;
          else if (v <= mn) code = 0;
          else code = static_cast<uint8_t>(((v - mn) / (mx - mn)) * 255);
          sc = (mx - mn) * kInv255;
          const float xf = static_cast<float>(code);
          xq = kIP ? fmaf(xf, sc, mn) : xf;
        }
        L.q[e] = xq;
        L.sq_scale[e] = sc;
        L.sq_min[e] = mn;
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
    Visited vs = make_visited(p, L.hash, slot_bits);
    PoolState ps{0u, 0u, p.ef};
    uint32_t n_dist = 0, n_expand = 0, n_dist_up = 0, n_hops_up = 0;

    // ---- Graph::initialize_search (graph.hpp:148-158) ---------------------------------------
    if (p.levels != nullptr) {
      // OverlayGraph::initialize (overlay_graph.hpp:122-144): greedy descent, strict '<'.
      uint32_t u = p.ep;
      if (lane == 0) L.cid[0] = u;
      wave_sync();
      space_distances<kIP, kChunks, kSpace>(p, L, L.cid, 1, L.cd);
      float cur = L.cd[0];
      ++n_dist_up;
      for (int level = static_cast<int>(p.levels[u]); level > 0; --level) {
        bool changed = true;
        while (changed) {
          changed = false;
          const uint32_t *list = p.upper_edges + p.upper_off[u] +
                                 static_cast<uint64_t>(level - 1) * p.upper_R;
          const uint32_t v = lane < static_cast<int>(p.upper_R) ? list[lane] : kEmpty;
          const uint64_t endm = ballot(lane < static_cast<int>(p.upper_R) && v == kEmpty);
          const int cnt = endm ? __ffsll(static_cast<unsigned long long>(endm)) - 1
                               : static_cast<int>(p.upper_R);
          ++n_hops_up;
          wave_sync();
          if (lane < cnt) L.cid[lane] = v;
          wave_sync();
          space_distances<kIP, kChunks, kSpace>(p, L, L.cid, cnt, L.cd);
          n_dist_up += cnt;
          // first index of the minimum == the sequential strict-'<' scan's final choice
          float dl = lane < cnt ? L.cd[lane] : FLT_MAX;
          bool has = lane < cnt;
          float mn = has ? dl : FLT_MAX;
          for (int off = 32; off > 0; off >>= 1) mn = fminf(mn, __shfl_xor(mn, off));
          const uint64_t at = ballot(has && dl == mn);
          if (at && mn < cur) {
            const int w = __ffsll(static_cast<unsigned long long>(at)) - 1;
            u = __shfl(v, w);
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
      visit(vs, u, lane == 0, bit_words);
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
          space_distances<kIP, kChunks, kSpace>(p, L, L.cid + c, min(8u, cnt - c), L.cd + c);
        }
        n_dist_up += cnt;
        const float d = has ? L.cd[lane] : 0.f;
        wave_sync();
        pool_merge(ps, L, has, v, d);
        // duplicates among eps are all inserted (no visited check in the reference loop)
        for (uint32_t j = 0; j < cnt; ++j) {
          const uint32_t vj = __shfl(v, j);
          if (!vs.spilled && vs.count + 64 > vs.limit) spill_begin(vs, bit_words);
          visit(vs, vj, lane == 0, bit_words);
        }
        wave_sync();
      }
    }

    // ---- best-first expansion (graph_search_job.hpp:228-252 / 310-330) -----------------------
    stamp(0);
    // Adjacency prefetch (no semantic effect): after a pop, the first unchecked entry is the next
    // expansion unless the merge puts a closer candidate in front of it.  Its 128 B row is loaded
    // into registers while this expansion runs and used only if the next pop returns that id.
    uint32_t pred = kEmpty, pred_v = kEmpty;
    while (ps.cur < ps.size) {
      const uint32_t u = pool_pop(ps, L);
      ++n_expand;
      if (kStamp && vs.spilled) st[5]++;
      stamp(1);
      uint32_t v;
      if (u == pred) {
        v = pred_v;
        if (kStamp) st[7]++;
      } else {
        v = lane < static_cast<int>(p.R) ? p.l0[static_cast<uint64_t>(u) * p.R + lane] : kEmpty;
      }
      pred = ps.cur < ps.size ? (L.pi[ps.cur] & kIdMask) : kEmpty;
      if (pred != kEmpty && lane < static_cast<int>(p.R)) pred_v = p.l0[static_cast<uint64_t>(pred) * p.R + lane];
      const uint64_t endm = ballot(lane < static_cast<int>(p.R) && v == kEmpty);
      const int cnt = endm ? __ffsll(static_cast<unsigned long long>(endm)) - 1 : static_cast<int>(p.R);
      bool act = lane < cnt;
      if (p.dedup_edges) {  // graphs with repeated ids in a row: keep the first occurrence only
        for (int j = 0; j < cnt; ++j) {
          const uint32_t vj = __shfl(v, j);
          if (j < lane && vj == v) act = false;
        }
      }
      if (!vs.spilled && vs.count + 64 > vs.limit) spill_begin(vs, bit_words);
      const bool fresh = visit(vs, v, act, bit_words);
      const uint64_t fm = ballot(fresh);
      const int nf = __popcll(fm);
      stamp(2);
      if (nf == 0) continue;
      // compact fresh ids in adjacency order
      const uint32_t slot = __popcll(fm & ((1ull << lane) - 1ull));
      if (fresh) L.cid[slot] = v;
      wave_sync();
      space_distances<kIP, kChunks, kSpace>(p, L, L.cid, nf, L.cd);
      stamp(3);
      n_dist += nf;
      const bool has = lane < nf;
      const uint32_t cid = has ? L.cid[lane] : 0u;
      const float cd = has ? L.cd[lane] : 0.f;
      wave_sync();
      pool_merge(ps, L, has, cid, cd);
      stamp(4);
    }

    // ---- results (ids[i] = pool.id(i), distances[i] = pool.dist(i)) --------------------------
    for (uint32_t i = lane; i < p.k; i += 64) {
      uint32_t id = p.fill_id;
      float d = 0.f;
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
    if constexpr (kStamp) {
      st[6] = __builtin_readcyclecounter() - t_begin;
      if (lane < 8) p.stamps[static_cast<uint64_t>(qi) * 8 + lane] = st[lane & 7];
    }
    wave_sync();
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
// pair<dist, id> are returned (id 0 can repeat -- reference behaviour).  Corrected mode (SURVEY
// A12 "corrected mode behind a flag"): the search hands over its whole ef pool (slots past the pool
// hold kEmpty and are skipped), so every rescored entry is a real candidate.  One wave per query.
template <bool kIP>
__global__ void __launch_bounds__(64) rerank_kernel(SearchParams p, RerankParams rp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *q = reinterpret_cast<float *>(smem);
  uint32_t *cid = reinterpret_cast<uint32_t *>(smem + static_cast<size_t>(p.stride) * 4);
  const uint32_t cap = max(rp.k, rp.n_src) + 1;
  float *cd = reinterpret_cast<float *>(cid + cap);
  uint32_t *cm = reinterpret_cast<uint32_t *>(cd + cap);
  const int lane = lane_id();
  const uint32_t taken = rp.corrected ? rp.n_src : min(rp.k, rp.ef);
  const uint32_t zeros = (!rp.corrected && rp.ef > rp.k) ? rp.ef - rp.k : 0u;
  const uint32_t c = taken + (zeros ? 1u : 0u);
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
        if (id == kEmpty) {  // corrected mode: slot past the pool
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
      rp.out_ids[qi * rp.k + i] = 0u;
      if (rp.out_dists) rp.out_dists[qi * rp.k + i] = 0.f;
    }
    wave_sync();
  }
}
}  // namespace

size_t search_lds_bytes(uint32_t stride, uint32_t ef, uint32_t hash_log2, bool sq8, bool compact) {
  return static_cast<size_t>(stride) * 4 + 3 * 64 * 4 + 2 * (((ef + 1) * 4 + 15) / 16 * 16) +
         visited_table_bytes(hash_log2, compact) + (sq8 ? 2 * static_cast<size_t>(stride) * 4 : 0);
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

template <bool kIP, int kChunks, bool kStamp = false, int kSpace = 0>
static const void *kernel_ptr() {
  return reinterpret_cast<const void *>(&hnsw_search_kernel<kIP, kChunks, kStamp, kSpace>);
}

template <int kSpace>
static const void *sq8_symbol(bool ip, uint32_t dim) {
  const uint32_t chunks = (dim % 32 == 0) ? dim / 32 : 0;
  if (chunks == 4) return ip ? kernel_ptr<true, 4, false, kSpace>() : kernel_ptr<false, 4, false, kSpace>();
  if (chunks == 24) return ip ? kernel_ptr<true, 24, false, kSpace>() : kernel_ptr<false, 24, false, kSpace>();
  if (chunks == 30) return ip ? kernel_ptr<true, 30, false, kSpace>() : kernel_ptr<false, 30, false, kSpace>();
  return ip ? kernel_ptr<true, 0, false, kSpace>() : kernel_ptr<false, 0, false, kSpace>();
}

const void *search_kernel_symbol(bool ip, uint32_t dim, bool stamped, int sq8_order) {
  if (sq8_order == 2) return sq8_symbol<2>(ip, dim);
  if (sq8_order == 1) return sq8_symbol<1>(ip, dim);
  const uint32_t chunks = (dim % 32 == 0) ? dim / 32 : 0;
  if (stamped) {
    if (chunks == 30) return ip ? kernel_ptr<true, 30, true>() : kernel_ptr<false, 30, true>();
    if (chunks == 4) return ip ? kernel_ptr<true, 4, true>() : kernel_ptr<false, 4, true>();
    return ip ? kernel_ptr<true, 0, true>() : kernel_ptr<false, 0, true>();
  }
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

hipError_t launch_search(const SearchParams &p, int grid, size_t lds, hipStream_t stream) {
  const void *fn = search_kernel_symbol(p.ip, p.dim, p.stamps != nullptr, p.sq8_order);
  SearchParams arg = p;
  void *args[] = {&arg};
  return hipLaunchKernel(fn, dim3(grid), dim3(64), args, lds, stream);
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

hipError_t search_occupancy(const SearchParams &p, size_t lds, int *blocks_per_cu) {
  const void *fn = search_kernel_symbol(p.ip, p.dim, p.stamps != nullptr, p.sq8_order);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, 64, lds);
}

}  // namespace alaya_amd
