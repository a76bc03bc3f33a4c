// Device-side building blocks shared by the search kernels (search_kernels.hip) and the graph
// construction kernels (build_kernels.hip): the bit-exact row distances, the exact visited set and
// the LinearPool-equivalent candidate pool.  Everything lives in an anonymous namespace, so each
// translation unit gets its own copy (no relocatable device code).
#pragma once
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

// Lane exchanges without the LDS crossbar: xor 1 / xor 2 are quad-permute DPP moves (VALU), xor 4
// is a bit-mode ds_swizzle (32-lane groups, no LDS access); a read of one uniform lane is a
// v_readlane.  __shfl/__shfl_xor compile to ds_bpermute, an LDS-pipe round trip each.
template <int kXor>
__device__ __forceinline__ float lane_xor(float v) {
  const int x = __builtin_bit_cast(int, v);
  int r;
  // quad permutes read a lane of the same quad, so every lane is written: no "old" operand (a
  // zeroed register per move with update_dpp(0, ...))
  if constexpr (kXor == 1) {
    r = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  } else if constexpr (kXor == 2) {
    r = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  } else {
    static_assert(kXor == 4 || kXor == 8 || kXor == 16, "lane_xor: 1, 2, 4, 8 or 16");
    r = __builtin_amdgcn_ds_swizzle(x, (kXor << 10) | 0x1F);        // and 0x1f, xor kXor
  }
  return __builtin_bit_cast(float, r);
}

__device__ __forceinline__ float read_lane(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ uint32_t read_lane(uint32_t v, int l) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), l));
}

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
// kSkip: the id list may hold kEmpty entries -- rows whose distance the caller already has (a helper's
// memo, search kernel kMode 4); they take a row slot but load nothing new and write no output.
// kRows: rows per lane group of an f32 row pass (0 = rows_per_group: the pass that fills one wave
// per SIMD's registers; 1 = the two-waves-per-SIMD wide-row kernels, search kernel kMode 8).
template <bool kIP, int kChunks, int kSpace, bool kSkip = false, int kRows = 0>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out);
template <bool kIP, int kChunks, int kSpace, bool kSkip = false, int kRows = 0, typename Hook>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out, Hook after_issue);

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
  a0 += lane_xor<2>(a0); a1 += lane_xor<2>(a1); a2 += lane_xor<2>(a2); a3 += lane_xor<2>(a3);
  a0 += lane_xor<4>(a0); a1 += lane_xor<4>(a1); a2 += lane_xor<4>(a2); a3 += lane_xor<4>(a3);
  // lane m==0 holds v[0..3], lane m==1 holds v[4..7]: s[j] = v[j] + v[j+4]; r = (s0+s1)+(s2+s3)
  const float s0 = a0 + lane_xor<1>(a0), s1 = a1 + lane_xor<1>(a1);
  const float s2 = a2 + lane_xor<1>(a2), s3 = a3 + lane_xor<1>(a3);
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
// Small rows (d <= 256): 2 rows per group = 16 rows per pass, which covers the ~10 fresh
// neighbours of a typical expansion in one pass and leaves registers for more resident waves.
#ifndef ALAYA_NARROW_RPL
#define ALAYA_NARROW_RPL 2  // diagnostics builds: -DALAYA_NARROW_RPL=1 (8-row passes, fewer VGPRs)
#endif
#ifndef ALAYA_WIDE_RPL
#define ALAYA_WIDE_RPL 0  // diagnostics builds: rows per lane group of the wide-row kernels (0 = 96 / chunks)
#endif
template <int kChunks>
constexpr int rows_per_group() {
  return kChunks <= 0 ? 1
         : kChunks <= 8 ? ALAYA_NARROW_RPL
         : ALAYA_WIDE_RPL > 0 ? ALAYA_WIDE_RPL
                        : (96 / kChunks >= 4 ? 4 : (96 / kChunks < 1 ? 1 : 96 / kChunks));
}

// One pass of row loads in registers: lane group g (8 lanes) takes rows base + g + 8r, r < kR.
template <int kChunks, int kRows = 0>
struct RowPass {
  static constexpr int kR = kRows > 0 ? kRows : rows_per_group<kChunks>();
  uint32_t id[kR];
  bool act[kR];
  float4 y[kR][kChunks];
};

// The row a lane group loads in place of a missing one (past n, or a kSkip kEmpty entry): the pass's
// first id, or row 0 when that one is kEmpty too -- a load whose result is dropped.
template <bool kSkip>
__device__ __forceinline__ uint32_t stand_in_row(uint32_t first) {
  if constexpr (kSkip) return first == kEmpty ? 0u : first;
  return first;
}

// Issue every row chunk of the pass (all loads in flight before the first FMA).  Branch-free: a
// lane group past n loads the pass's first row again (its result is dropped), and a whole slot
// past n is skipped wave-uniformly -- per-load exec-mask branches would serialise the issue.
// Requires base < n.
template <int kChunks, bool kSkip = false, int kRows = 0>
__device__ __forceinline__ void issue_rows(const SearchParams &p, const uint32_t *ids, int n, int base,
                                           RowPass<kChunks, kRows> &P) {
  constexpr int kRPL = RowPass<kChunks, kRows>::kR;
  const int lane = lane_id();
  const int g = lane >> 3, m = lane & 7;
  const uint32_t id0 = stand_in_row<kSkip>(ids[base]);
#pragma unroll
  for (int r = 0; r < kRPL; ++r) {
    const int idx = base + g + 8 * r;
    if constexpr (kSkip) {
      const uint32_t id = idx < n ? ids[idx] : kEmpty;
      P.act[r] = id != kEmpty;
      P.id[r] = P.act[r] ? id : id0;
    } else {
      P.act[r] = idx < n;
      P.id[r] = P.act[r] ? ids[idx] : id0;
    }
  }
#pragma unroll
  for (int r = 0; r < kRPL; ++r) {
    const float4 *rp = reinterpret_cast<const float4 *>(p.base + static_cast<uint64_t>(P.id[r]) * p.stride) + m;
    if (base + 8 * r < n) {  // wave-uniform; a skipped slot is never read (finish_rows' `live`)
#pragma unroll
      for (int t = 0; t < kChunks; ++t) P.y[r][t] = rp[8 * t];
    }
  }
}

// Distances of an issued pass -> out[base + g + 8r].  The kChunks > 0 kernels run only for
// dim == 32 * kChunks (search_kernel_symbol / the build's dispatch pick them from dim % 32 == 0), so
// there is no 8-block or scalar tail.  Row slots past n (wave-uniform) are skipped whole.
template <bool kIP, int kChunks, int kRows = 0>
__device__ __forceinline__ void finish_rows(const SearchParams &p, const float *q, int n, int base,
                                            RowPass<kChunks, kRows> &P, float *out) {
  constexpr int kRPL = RowPass<kChunks, kRows>::kR;
  const int lane = lane_id();
  const int g = lane >> 3, m = lane & 7;
  int live = 0;  // wave-uniform number of row slots in use
  float a[kRPL][4];
#pragma unroll
  for (int r = 0; r < kRPL; ++r) {
    a[r][0] = a[r][1] = a[r][2] = a[r][3] = 0.f;
    live += base + 8 * r < n ? 1 : 0;
  }
  const float4 *qp = reinterpret_cast<const float4 *>(q) + m;
#pragma unroll
  for (int t = 0; t < kChunks; ++t) {
    const float4 x = qp[8 * t];
#pragma unroll
    for (int r = 0; r < kRPL; ++r) {
      if (r >= live) break;
      accumulate<kIP>(x, P.y[r][t], a[r][0], a[r][1], a[r][2], a[r][3]);
    }
  }
#pragma unroll
  for (int r = 0; r < kRPL; ++r) {
    if (r >= live) break;
    float res = finish_row<kIP>(a[r][0], a[r][1], a[r][2], a[r][3]);
    if (P.act[r] && m == 0) {
      if (kIP) res = -res;
      const uint32_t id = P.id[r];
      if (p.valid != nullptr && !((p.valid[id >> 5] >> (id & 31)) & 1u)) res = FLT_MAX;
      out[base + g + 8 * r] = res;
    }
  }
}

// The generic branch of l2_sqr<T> / ip_sqr<T> for non-float DataType (distance_l2.ipp:735-741,
// distance_ip.ipp:744-750): elements cast to float, one accumulator over the elements in order,
// diff*diff (x*y) rounded before the add (-ffp-contract=off).  The reference builds it with -Ofast,
// which leaves the order to the compiler; the source order is the restatement's (oracle generic_l2),
// and every order agrees while the partial sums stay integers below 2^24.  One lane per row.
template <bool kIP, bool kSkip = false>
__device__ __forceinline__ void generic_distances(const SearchParams &p, const float *q,
                                                  const uint32_t *ids, int n, float *out) {
  const int lane = lane_id();
  for (int base = 0; base < n; base += 64) {
    const int r = base + lane;
    if (r < n) {
      const uint32_t id = ids[r];
      if (kSkip && id == kEmpty) continue;  // known to the caller
      const float *row = p.base + static_cast<uint64_t>(id) * p.stride;
      float sum = 0.f;
      for (uint32_t e = 0; e < p.dim; ++e) {
        if (kIP) {
          sum += q[e] * row[e];
        } else {
          const float d = q[e] - row[e];
          sum += d * d;
        }
      }
      float res = kIP ? -sum : sum;
      if (p.valid != nullptr && !((p.valid[id >> 5] >> (id & 31)) & 1u)) res = FLT_MAX;
      out[r] = res;
    }
  }
  wave_sync();
}

template <bool kIP, int kChunks, bool kSkip = false, int kRows = 0>
__device__ __forceinline__ void row_distances(const SearchParams &p, const float *q,
                                              const uint32_t *ids, int n, float *out) {
  if constexpr (kChunks == 0) {
    if (p.generic) {  // wave-uniform; the host selects the kChunks == 0 kernels for generic rows
      generic_distances<kIP, kSkip>(p, q, ids, n, out);
      return;
    }
  }
  const int lane = lane_id();
  const int g = lane >> 3, m = lane & 7;
  const int T = kChunks > 0 ? kChunks : static_cast<int>(p.dim >> 5);
  const int rem = static_cast<int>(p.dim) - 32 * T;
  const int nb8 = rem >> 3;
  const int tail_begin = 32 * T + 8 * nb8;
  if constexpr (kChunks > 0) {
    constexpr int kStep = 8 * RowPass<kChunks, kRows>::kR;
    for (int base = 0; base < n; base += kStep) {
      RowPass<kChunks, kRows> P;
      issue_rows<kChunks, kSkip, kRows>(p, ids, n, base, P);
      finish_rows<kIP, kChunks, kRows>(p, q, n, base, P, out);
    }
    (void)g; (void)m; (void)tail_begin;
  } else {
    for (int base = 0; base < n; base += 8) {
      const int r = base + g;
      const uint32_t rid = r < n ? ids[r] : kEmpty;
      const bool act = r < n && (!kSkip || rid != kEmpty);
      const uint32_t id = act ? rid : 0u;
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
// P/4 lanes per row (8 for AVX-512, 4 for AVX2): lane m owns acc[4m..4m+3], i.e. one code dword
// per P-byte chunk, so every partial sum stays one sequential chain as on the host.  The combine
// is a shuffle tree inside the row's lanes (xor 4 / 2 / 1).  Each lane group takes kRPL rows per
// pass; row slices past n are skipped wave-uniformly.  LDS holds, per dimension, the query term
// (x for L2, xv for IP), scale and min, read as float4 for the lane's 4 dimensions.
// --------------------------------------------------------------------------------------------
template <bool kIP>
__device__ __forceinline__ float sq8_term(float xq, float scale, float mn, float yf, float acc) {
  if (kIP) return fmaf(xq, fmaf(yf, scale, mn), acc);
  const float d = (xq - yf) * scale;
  return fmaf(d, d, acc);
}

// The query's term per dimension: x = float(code) (L2) or xv = fma(float(code), scale, min) (IP), read
// from LDS as f32 (kCodes = false), or rebuilt from the query's one-byte codes (kCodes: the
// AVX-512-order kernels with ALAYA_SQ8_QCODES, a quarter of the LDS) with the same operations as the
// encoder, so the value -- and every distance -- is bit-identical.
#ifndef ALAYA_SQ8_QCODES
#define ALAYA_SQ8_QCODES 0
#endif
template <int kOrder>
constexpr bool sq8_query_codes() { return ALAYA_SQ8_QCODES != 0 && kOrder == 2; }

template <bool kIP, bool kCodes>
__device__ __forceinline__ float4 sq8_qterm4(const float *xq, const float4 &s, const float4 &mn, int e) {
  if constexpr (!kCodes) {
    return *reinterpret_cast<const float4 *>(xq + e);
  } else {
    const uint32_t w = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(xq) + e);
    const float c0 = static_cast<float>(w & 0xffu), c1 = static_cast<float>((w >> 8) & 0xffu);
    const float c2 = static_cast<float>((w >> 16) & 0xffu), c3 = static_cast<float>(w >> 24);
    if (kIP) return make_float4(fmaf(c0, s.x, mn.x), fmaf(c1, s.y, mn.y), fmaf(c2, s.z, mn.z), fmaf(c3, s.w, mn.w));
    return make_float4(c0, c1, c2, c3);
  }
}
template <bool kIP, bool kCodes>
__device__ __forceinline__ float sq8_qterm(const float *xq, const float *sc, const float *mnv, int e) {
  if constexpr (!kCodes) return xq[e];
  const float c = static_cast<float>(reinterpret_cast<const uint8_t *>(xq)[e]);
  return kIP ? fmaf(c, sc[e], mnv[e]) : c;
}

template <bool kIP, bool kCodes = false>
__device__ __forceinline__ void sq8_chunk(const float *xq, const float *sc, const float *mnv, int e,
                                          uint32_t w, float *acc) {
  const float4 s = *reinterpret_cast<const float4 *>(sc + e);
  float4 mn = make_float4(0.f, 0.f, 0.f, 0.f);
  if (kIP) mn = *reinterpret_cast<const float4 *>(mnv + e);
  const float4 x = sq8_qterm4<kIP, kCodes>(xq, s, mn, e);
  acc[0] = sq8_term<kIP>(x.x, s.x, mn.x, static_cast<float>(w & 0xffu), acc[0]);
  acc[1] = sq8_term<kIP>(x.y, s.y, mn.y, static_cast<float>((w >> 8) & 0xffu), acc[1]);
  acc[2] = sq8_term<kIP>(x.z, s.z, mn.z, static_cast<float>((w >> 16) & 0xffu), acc[2]);
  acc[3] = sq8_term<kIP>(x.w, s.w, mn.w, static_cast<float>(w >> 24), acc[3]);
}

#ifndef ALAYA_PAIR_LOOPS
// lane loops over ballot masks take two lanes per trip (pool_merge's LDS path, stab_visit): config 5
// 1k queries 3.60 -> 3.53 ms, 10k 9.51 -> 9.47 ms, GIST unchanged (profiles/r05/pair/)
#define ALAYA_PAIR_LOOPS 1
#endif
#ifndef ALAYA_SQ8_DW
#define ALAYA_SQ8_DW 48  // code dwords in flight per lane (rows per lane group = DW / chunks)
#endif
// rows per lane group per pass: <= 48 code dwords in flight per lane (the per-chunk float4 LDS
// reads are hoisted too; more rows spill at d = 768)
template <int kOrder, int kFull>
constexpr int sq8_rows_per_group() {
  return kFull <= 0 ? 1 : (ALAYA_SQ8_DW / kFull >= 4 ? 4 : (ALAYA_SQ8_DW / kFull < 1 ? 1 : ALAYA_SQ8_DW / kFull));
}

// One pass of SQ8 code loads in registers (compile-time chunk count): lane group g takes rows
// base + g + G r, r < kR.  Issued branch-free like issue_rows (a group past n reloads the pass's
// first row, a whole slot past n is skipped wave-uniformly).
template <int kOrder, int kFull>
struct Sq8Pass {
  static constexpr int P = kOrder == 2 ? 32 : 16;
  static constexpr int LPR = P / 4;
  static constexpr int G = 64 / LPR;
  static constexpr int kR = sq8_rows_per_group<kOrder, kFull>();
  static constexpr int kStep = G * kR;
  uint32_t id[kR];
  bool act[kR];
  uint32_t w[kR][kFull > 0 ? kFull : 1];
};

template <int kOrder, int kFull, bool kSkip = false>
__device__ __forceinline__ void sq8_issue(const SearchParams &p, const uint32_t *ids, int n, int base,
                                          Sq8Pass<kOrder, kFull> &S) {
  static_assert(kFull > 0, "compile-time chunk count only");
  using SP = Sq8Pass<kOrder, kFull>;
  const int lane = lane_id();
  const int g = lane / SP::LPR, m = lane % SP::LPR;
  const uint32_t id0 = stand_in_row<kSkip>(ids[base]);
#pragma unroll
  for (int r = 0; r < SP::kR; ++r) {
    const int idx = base + g + SP::G * r;
    if constexpr (kSkip) {
      const uint32_t id = idx < n ? ids[idx] : kEmpty;
      S.act[r] = id != kEmpty;
      S.id[r] = S.act[r] ? id : id0;
    } else {
      S.act[r] = idx < n;
      S.id[r] = S.act[r] ? ids[idx] : id0;
    }
  }
#pragma unroll
  for (int r = 0; r < SP::kR; ++r) {
    const uint8_t *row = p.codes + static_cast<uint64_t>(S.id[r]) * p.code_stride + 4 * m;
    if (base + SP::G * r < n) {  // wave-uniform
#pragma unroll
      for (int t = 0; t < kFull; ++t) S.w[r][t] = *reinterpret_cast<const uint32_t *>(row + SP::P * t);
    } else {
#pragma unroll
      for (int t = 0; t < kFull; ++t) S.w[r][t] = 0u;
    }
  }
}

template <bool kIP, int kOrder, int kFull>
__device__ __forceinline__ void sq8_finish(const SearchParams &p, const float *xq, const float *sc,
                                           const float *mnv, int n, int base, Sq8Pass<kOrder, kFull> &S,
                                           float *out) {
  using SP = Sq8Pass<kOrder, kFull>;
  constexpr int P = SP::P, LPR = SP::LPR, G = SP::G;
  const int lane = lane_id();
  const int g = lane / LPR, m = lane % LPR;
  // kFull > 0 kernels run only for dim == P * kFull (dim / 32 chunks of 32 codes, or twice as many
  // of 16), so rem == 0: no half block, no scalar tail.  The AVX-512 order drops the dead tail code;
  // the AVX2 order keeps it, because without it the compiler schedules the 48-chunk loop into
  // 186-235 VGPRs (2 waves per SIMD) instead of 121-144.
  constexpr bool kTail = kOrder == 1;
  constexpr bool kCodes = sq8_query_codes<kOrder>();
  const int rem = kTail ? static_cast<int>(p.dim) - P * kFull : 0;
  const bool half = kTail && rem >= P / 2;
  const int tail_begin = P * kFull + (half ? P / 2 : 0);
  float acc[SP::kR][4];
  int live = 0;  // wave-uniform number of row slots in use
#pragma unroll
  for (int r = 0; r < SP::kR; ++r) {
    acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0.f;
    live += base + G * r < n ? 1 : 0;
  }
  // chunk-major: a chunk's query / scale / min values feed every row slot, then die
#pragma unroll
  for (int t = 0; t < kFull; ++t) {
#ifndef ALAYA_SQ8_NO_FENCE
    // keep the scheduler from hoisting later chunks' LDS reads (and their registers) above this
    // chunk's FMAs: 199 -> 131 VGPRs at d = 768 (IP), i.e. 3 instead of 2 waves per SIMD (config
    // 5 at 10k queries 12.2 -> 10.5 ms; with one row per lane group 123 VGPRs, but slower at 1k
    // queries: profiles/r03/sweeps)
    __builtin_amdgcn_sched_barrier(0);
#endif
    const int e = P * t + 4 * m;
    const float4 s = *reinterpret_cast<const float4 *>(sc + e);
    float4 mn = make_float4(0.f, 0.f, 0.f, 0.f);
    if (kIP) mn = *reinterpret_cast<const float4 *>(mnv + e);
    const float4 x = sq8_qterm4<kIP, kCodes>(xq, s, mn, e);
#pragma unroll
    for (int r = 0; r < SP::kR; ++r) {
      if (r >= live) break;
      const uint32_t w = S.w[r][t];
      float *a = acc[r];
      a[0] = sq8_term<kIP>(x.x, s.x, mn.x, static_cast<float>(w & 0xffu), a[0]);
      a[1] = sq8_term<kIP>(x.y, s.y, mn.y, static_cast<float>((w >> 8) & 0xffu), a[1]);
      a[2] = sq8_term<kIP>(x.z, s.z, mn.z, static_cast<float>((w >> 16) & 0xffu), a[2]);
      a[3] = sq8_term<kIP>(x.w, s.w, mn.w, static_cast<float>(w >> 24), a[3]);
    }
  }
#pragma unroll
  for (int r = 0; r < SP::kR; ++r) {
    if (r >= live) break;
    const uint8_t *rw = p.codes + static_cast<uint64_t>(S.id[r]) * p.code_stride;
    if (half && m < LPR / 2 && S.act[r])  // trailing half block -> acc[0 .. P/2)
      sq8_chunk<kIP, kCodes>(xq, sc, mnv, P * kFull + 4 * m,
                             *reinterpret_cast<const uint32_t *>(rw + P * kFull + 4 * m), acc[r]);
    float a0 = acc[r][0], a1 = acc[r][1], a2 = acc[r][2], a3 = acc[r][3];
    if constexpr (kOrder == 2) {
      a0 += lane_xor<4>(a0); a1 += lane_xor<4>(a1); a2 += lane_xor<4>(a2); a3 += lane_xor<4>(a3);
    }
    a0 += lane_xor<2>(a0); a1 += lane_xor<2>(a1); a2 += lane_xor<2>(a2); a3 += lane_xor<2>(a3);
    a0 += lane_xor<1>(a0); a1 += lane_xor<1>(a1); a2 += lane_xor<1>(a2); a3 += lane_xor<1>(a3);
    float res = kOrder == 2 ? (a0 + a2) + (a1 + a3) : (a0 + a1) + (a2 + a3);
    if (S.act[r] && m == 0) {
      if constexpr (kTail) {
        for (int e = tail_begin; e < static_cast<int>(p.dim); ++e)
          res = sq8_term<kIP>(sq8_qterm<kIP, kCodes>(xq, sc, mnv, e), sc[e], mnv[e], static_cast<float>(rw[e]), res);
      }
      out[base + g + G * r] = kIP ? -res : res;  // no validity check in SQ8Space::QueryComputer
    }
  }
}

struct NoHook {
  __device__ void operator()() const {}
};

// after_issue() runs once, right after the first pass's row loads are issued (the search kernel
// issues its second-level prefetch there, so it overlaps the rows' latency)
template <bool kIP, int kOrder, int kFull, bool kSkip = false, typename Hook = NoHook>
__device__ __forceinline__ void sq8_distances(const SearchParams &p, const float *xq,
                                              const float *sc, const float *mnv,
                                              const uint32_t *ids, int n, float *out, Hook after_issue = Hook()) {
  constexpr int P = kOrder == 2 ? 32 : 16;
  constexpr int LPR = P / 4;    // lanes per row
  constexpr int G = 64 / LPR;   // row groups per wave
  constexpr int kRPL = sq8_rows_per_group<kOrder, kFull>();
  constexpr bool kCodes = sq8_query_codes<kOrder>();
  if constexpr (kFull > 0) {
    for (int base = 0; base < n; base += G * kRPL) {
      Sq8Pass<kOrder, kFull> S;
      sq8_issue<kOrder, kFull, kSkip>(p, ids, n, base, S);
      if (base == 0) after_issue();
      sq8_finish<kIP, kOrder, kFull>(p, xq, sc, mnv, n, base, S, out);
    }
    wave_sync();
    return;
  }
  after_issue();
  const int lane = lane_id();
  const int g = lane / LPR, m = lane % LPR;
  const int T = kFull > 0 ? kFull : static_cast<int>(p.dim) / P;
  const int rem = static_cast<int>(p.dim) - P * T;
  const bool half = rem >= P / 2;
  const int tail_begin = P * T + (half ? P / 2 : 0);
  for (int base = 0; base < n; base += G * kRPL) {
    uint32_t id[kRPL];
    bool act[kRPL];
    const uint8_t *row[kRPL];
    float acc[kRPL][4];
#pragma unroll
    for (int r = 0; r < kRPL; ++r) {
      const int idx = base + g + G * r;
      const uint32_t rid = idx < n ? ids[idx] : kEmpty;
      act[r] = idx < n && (!kSkip || rid != kEmpty);
      id[r] = act[r] ? rid : 0u;
      row[r] = p.codes + static_cast<uint64_t>(id[r]) * p.code_stride;
      acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0.f;
    }
    if constexpr (kFull > 0) {
      uint32_t w[kRPL][kFull];
#pragma unroll
      for (int r = 0; r < kRPL; ++r) {
        if (base + G * r >= n) break;  // wave-uniform
#pragma unroll
        for (int t = 0; t < kFull; ++t)
          w[r][t] = act[r] ? *reinterpret_cast<const uint32_t *>(row[r] + P * t + 4 * m) : 0u;
      }
#pragma unroll
      for (int r = 0; r < kRPL; ++r) {
        if (base + G * r >= n) break;
#pragma unroll
        for (int t = 0; t < kFull; ++t) sq8_chunk<kIP, kCodes>(xq, sc, mnv, P * t + 4 * m, w[r][t], acc[r]);
      }
    } else {
      if (act[0]) {
        for (int t = 0; t < T; ++t)
          sq8_chunk<kIP, kCodes>(xq, sc, mnv, P * t + 4 * m,
                                 *reinterpret_cast<const uint32_t *>(row[0] + P * t + 4 * m), acc[0]);
      }
    }
#pragma unroll
    for (int r = 0; r < kRPL; ++r) {
      if (base + G * r >= n) break;
      if (half && m < LPR / 2 && act[r])  // trailing half block -> acc[0 .. P/2)
        sq8_chunk<kIP, kCodes>(xq, sc, mnv, P * T + 4 * m, *reinterpret_cast<const uint32_t *>(row[r] + P * T + 4 * m),
                               acc[r]);
      float a0 = acc[r][0], a1 = acc[r][1], a2 = acc[r][2], a3 = acc[r][3];
      if constexpr (kOrder == 2) {  // a = sum0 + sum1 (lanes m, m+4)
        a0 += lane_xor<4>(a0); a1 += lane_xor<4>(a1); a2 += lane_xor<4>(a2); a3 += lane_xor<4>(a3);
      }
      // AVX-512: T3 = a[8+j] + a[j]; AVX2: v = sum0 + sum1 (lanes m, m+2)
      a0 += lane_xor<2>(a0); a1 += lane_xor<2>(a1); a2 += lane_xor<2>(a2); a3 += lane_xor<2>(a3);
      // AVX-512: T6 = T3[4+j] + T3[j]; AVX2: s = v[j] + v[j+4] (lanes m, m+1)
      a0 += lane_xor<1>(a0); a1 += lane_xor<1>(a1); a2 += lane_xor<1>(a2); a3 += lane_xor<1>(a3);
      float res = kOrder == 2 ? (a0 + a2) + (a1 + a3) : (a0 + a1) + (a2 + a3);
      if (act[r] && m == 0) {
        const uint8_t *rw = row[r];
        for (int e = tail_begin; e < static_cast<int>(p.dim); ++e)
          res = sq8_term<kIP>(sq8_qterm<kIP, kCodes>(xq, sc, mnv, e), sc[e], mnv[e], static_cast<float>(rw[e]), res);
        out[base + g + G * r] = kIP ? -res : res;  // no validity check in SQ8Space::QueryComputer
      }
    }
  }
  wave_sync();
}

template <bool kIP, int kChunks, int kSpace, bool kSkip, int kRows, typename Hook>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out, Hook after_issue) {
  if constexpr (kSpace == 0) {
    row_distances<kIP, kChunks, kSkip, kRows>(p, L.q, ids, n, out);
    after_issue();
  } else {
    sq8_distances<kIP, kSpace, kSpace == 2 ? kChunks : 2 * kChunks, kSkip>(p, L.q, L.sq_scale, L.sq_min, ids, n,
                                                                             out, after_issue);
  }
}

template <bool kIP, int kChunks, int kSpace, bool kSkip, int kRows>
__device__ __forceinline__ void space_distances(const SearchParams &p, const Lds &L,
                                                const uint32_t *ids, int n, float *out) {
  space_distances<kIP, kChunks, kSpace, kSkip, kRows>(p, L, ids, n, out, NoHook());
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
// the query spills: a per-slot global N-bit bitset becomes the second level (atomicOr), and the
// LDS table stays as a read-only first level.
// The bitset is clean (all zero) whenever no query owns the slot, and is cleared lazily: the
// atomicOr that sets the first bit of a word returns 0, and that lane appends the word's index to
// the slot's dirty list (one append per touched word, ballot + prefix count).  At the query's end
// the wave zeroes exactly the listed words -- O(words touched), not the N/8 bytes of the whole
// bitset (1.25 MB at 10M rows) that a spilling query used to clear first.  A list that outgrows
// its capacity falls back to clearing the whole bitset.  No extra round trip per visit.
// --------------------------------------------------------------------------------------------
struct Visited {
  uint32_t *tab;
  uint32_t log2h;
  uint32_t count;        // wave-uniform number of entries in the LDS table
  uint32_t limit;        // switch to the global bitset above this many entries
  bool spilled;          // wave-uniform
  uint32_t *bits;        // per-slot global bitset (clean on entry, cleaned by visit_end)
  uint32_t *dirty;       // per-slot list of the bitset words this query set (dirty_cap entries)
  uint32_t dirty_cap;
  uint32_t ndirty;       // wave-uniform number of words appended (may exceed dirty_cap)
  uint64_t n_words;      // bitset words (ceil(n / 32))
  uint32_t rbits;        // compact: remainder bits; kVisWide: 32-bit slots
  uint32_t lmask;        // 2^L - 1 (compact slots and the spill table hash with it)
  uint32_t lshift;       // compact, L < log2h: home = h << lshift
  uint32_t max_disp;     // compact: largest encodable probe distance
  // spill table (SQ8 kernels, SearchParams::spill_table): nullptr = the bitset is the second level
  uint16_t *stab;
  uint32_t stab_bmask;   // buckets - 1
  uint32_t stab_rbits;
};

__device__ __forceinline__ Visited make_visited(const SearchParams &p, uint32_t *tab, uint32_t *bits,
                                                uint32_t *dirty, uint16_t *stab = nullptr) {
  Visited vs;
  vs.tab = tab;
  vs.log2h = p.hash_log2;
  vs.count = 0u;
  vs.spilled = false;
  vs.bits = bits;
  vs.dirty = dirty;
  vs.dirty_cap = p.dirty_cap;
  vs.ndirty = 0u;
  vs.n_words = (p.n + 31) / 32;
  vs.stab = stab;
  vs.stab_bmask = stab ? (1u << (p.stab_log2 - 3)) - 1u : 0u;
  vs.stab_rbits = p.stab_rbits;
  vs.rbits = p.vis_rbits;
  const uint32_t hsize = 1u << p.hash_log2;
  vs.lmask = p.vis_lbits >= 32 ? 0xffffffffu : (1u << p.vis_lbits) - 1u;  // compact slots, spill table
  if (p.vis_rbits == kVisWide) {
    vs.limit = hsize / 2;
    vs.lshift = vs.max_disp = 0u;
  } else {
    vs.limit = hsize - hsize / 4 - hsize / 16;  // load factor 0.69
    vs.lshift = p.vis_lbits < p.hash_log2 ? p.hash_log2 - p.vis_lbits : 0u;
    vs.max_disp = p.vis_max_disp;
  }
  if (p.vis_limit != 0u) vs.limit = p.vis_limit;
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

// kShared: the table belongs to another wave that may be writing it (the distance helpers' visited
// hint, search_kernels.hip): its slots are read as relaxed workgroup-scope atomics, and the answer is
// a hint that may be stale either way.  The owner's own probe ends because a table holds at most
// vis_limit + 64 < slots entries (a wide probe meets an empty slot) and a compact probe stops at
// max_disp.  A shared wide probe is also bounded by the table size: the region may be overwritten
// under it (a sibling that just ran out of queries clears its memo area over its table, and a zeroed
// wide table has no kEmpty slot), so it gives up after one lap.
template <bool kShared = false>
__device__ __forceinline__ bool table_lookup(const Visited &vs, uint32_t v) {
  const uint32_t mask = (1u << vs.log2h) - 1u;
  if (vs.rbits == kVisWide) {
    uint32_t h = hash_slot(v, vs.log2h);
    for (uint32_t i = 0;; ++i) {
      const uint32_t e = kShared ? __hip_atomic_load(&vs.tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                                 : vs.tab[h];
      if (e == v) return true;
      if (e == kEmpty) return false;
      if (kShared && i == mask) return false;
      h = (h + 1) & mask;
    }
  }
  uint32_t home, rem;
  compact_key(vs, v, home, rem);
  const uint16_t *t16 = reinterpret_cast<const uint16_t *>(vs.tab);
  for (uint32_t i = 0;; ++i) {
    const uint32_t e = kShared ? __hip_atomic_load(&t16[(home + i) & mask], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP)
                               : t16[(home + i) & mask];
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

// The lane that set a bitset word's first bit records the word on the slot's dirty list (visit_end
// clears exactly those words).  Wave-uniform.
__device__ __forceinline__ void dirty_append(Visited &vs, bool first, uint32_t word) {
  const uint64_t fm = ballot(first);
  if (fm) {
    const uint32_t pos = vs.ndirty + __popcll(fm & ((1ull << lane_id()) - 1ull));
    if (first && pos < vs.dirty_cap) vs.dirty[pos] = word;
    vs.ndirty += __popcll(fm);
  }
}

// --------------------------------------------------------------------------------------------
// Spill table: the second level of the SQ8 kernels (config 5: 10M ids fit only a few hundred LDS
// slots at full residency, so ~90 % of a query's expansions run spilled).  Per slot, 2^s 16-bit
// entries in buckets of 8 (16 B), zero = empty, clean between queries.  h = (v * C) mod 2^L is a
// bijection (L = vis_lbits >= log2 n, C odd); the home bucket is h's top s - 3 bits and an entry
// stores 1 + h's low rbits bits, so (bucket, entry) identifies v.  An id
// goes into its home bucket's first free entry, or -- when the bucket is full -- into the bitset
// (third level).  Buckets fill in entry order and nothing is removed during a query, so a bucket
// that is not full has never been full: v is visited iff its home bucket holds it, or the bucket is
// full and the bitset holds it.
// At 32 KB per slot (config 5: 2^14 entries for ~2.7k visited ids, load 0.16) every table of a
// launch fits the Infinity Cache, where the N-bit bitsets took 1.25 MB per slot (3.8 GB) and every
// visit was a scattered line in HBM.  The wave is the slot's only writer: entries are plain 16-bit
// stores, no atomics.  Reads are agent-scope (L2, never a stale vector-L1 line).
// --------------------------------------------------------------------------------------------
__device__ __forceinline__ void stab_key(const Visited &vs, uint32_t v, uint32_t &home, uint32_t &code) {
  const uint32_t h = (v * 0x9E3779B1u) & vs.lmask;
  home = h >> vs.stab_rbits;  // the host keeps buckets <= 2^L: rbits >= 0
  code = 1u + (h & ((1u << vs.stab_rbits) - 1u));
}

// Scope of every spill-table access (diagnostics builds: -DALAYA_STAB_SCOPE=__HIP_MEMORY_SCOPE_WORKGROUP
// keeps the table's lines in the XCD's L2 -- a slot's table is only ever touched by the one wave that
// owns the slot during a launch, and kernel boundaries order launches)
#ifndef ALAYA_STAB_SCOPE
#define ALAYA_STAB_SCOPE __HIP_MEMORY_SCOPE_AGENT
#endif
__device__ __forceinline__ void stab_load(const Visited &vs, uint32_t bucket, uint64_t &lo, uint64_t &hi) {
  uint64_t *b = reinterpret_cast<uint64_t *>(vs.stab + static_cast<size_t>(bucket) * kStabBucket);
  lo = __hip_atomic_load(b, __ATOMIC_RELAXED, ALAYA_STAB_SCOPE);
  hi = __hip_atomic_load(b + 1, __ATOMIC_RELAXED, ALAYA_STAB_SCOPE);
}

// Stores are agent-scope too: a plain (CU-scope) store may be acknowledged before it reaches L2, where
// the wave's next agent-scope read of the bucket looks (measured: duplicate visits with plain stores).
__device__ __forceinline__ void stab_store(const Visited &vs, uint32_t entry, uint32_t code) {
  __hip_atomic_store(vs.stab + entry, static_cast<uint16_t>(code), __ATOMIC_RELAXED, ALAYA_STAB_SCOPE);
}

// Order the wave's earlier spill-table stores (and bitset atomics) before its later bucket reads.
// Every access to a slot's table comes from the one wave that owns the slot, from one CU, so the
// order needed is the workgroup's: the seq_cst workgroup fence is the language-level guarantee (no
// compiler may move a load above it; in LLVM's AMDGPU memory model the CU then performs the wave's
// memory operations in order, so gfx950 emits no instruction for it), and s_waitcnt(0) makes the
// stores complete at L2 -- where the agent-scope reads look -- before the reads are issued.  An
// agent-scope fence would be wrong here: on gfx950 it writes back and invalidates the whole L2
// (buffer_wbl2 / buffer_inv sc1) for an order that never leaves the wave.
__device__ __forceinline__ void stab_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// found: the bucket holds `code`; occ: entries in use (= the first free position)
__device__ __forceinline__ void stab_scan(uint64_t lo, uint64_t hi, uint32_t code, bool &found, uint32_t &occ) {
  found = false;
  occ = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t a = static_cast<uint32_t>(lo >> (16 * j)) & 0xffffu;
    const uint32_t b = static_cast<uint32_t>(hi >> (16 * j)) & 0xffffu;
    found |= (a == code) | (b == code);
    occ += (a != 0u ? 1u : 0u) + (b != 0u ? 1u : 0u);
  }
}

// Visit on the spill table.  Lanes with `act` hold distinct ids.  pre_ok (wave-uniform): (lo, hi)
// hold each lane's home bucket as it is now (stab_prefetch after the previous expansion's stores had
// landed; nothing is stored in between); otherwise the buckets are loaded here.
__device__ __forceinline__ bool stab_visit(Visited &vs, uint32_t v, bool act, bool pre_ok, uint64_t lo, uint64_t hi) {
  const int lane = lane_id();
  uint32_t home = 0, code = 0;
  stab_key(vs, v, home, code);
  if (!pre_ok) {
    stab_order();
    if (act) stab_load(vs, home, lo, hi);
  }
  bool found;
  uint32_t occ;
  stab_scan(lo, hi, code, found, occ);
  // home bucket with room and v not in it: v is nowhere (not in the bitset either) -> fresh; it
  // takes position occ + (fresh lanes below it with the same home bucket)
  const bool fast = act && !found && occ < kStabBucket;
  const uint64_t fm = ballot(fast);
  uint32_t rank = 0;
#if ALAYA_PAIR_LOOPS
  for (uint64_t r = fm; r;) {  // two fast lanes per trip (see pool_merge)
    const int j = __ffsll(static_cast<unsigned long long>(r)) - 1;
    r &= r - 1;
    const bool t2 = r != 0ull;
    const int j2 = t2 ? __ffsll(static_cast<unsigned long long>(r)) - 1 : j;
    r &= t2 ? r - 1 : r;
    const uint32_t h1 = read_lane(home, j), h2 = read_lane(home, j2);
    rank += (j < lane && h1 == home) ? 1u : 0u;
    rank += (t2 && j2 < lane && h2 == home) ? 1u : 0u;
  }
#else
  for (uint64_t r = fm; r; r &= r - 1) {
    const int j = __ffsll(static_cast<unsigned long long>(r)) - 1;
    rank += (j < lane && read_lane(home, j) == home) ? 1u : 0u;
  }
#endif
  const bool placed = fast && occ + rank < kStabBucket;
  if (placed) stab_store(vs, home * kStabBucket + occ + rank, code);
  // rare: the home bucket is full (v may be in the bitset) or filled up within this visit (v is
  // fresh): the bitset, one returning atomic per such lane
  const bool third = act && !found && !placed;
  if (ballot(third)) {
    const uint32_t bit = 1u << (v & 31);
    uint32_t old = bit;
    if (third) old = atomicOr(&vs.bits[v >> 5], bit);
    dirty_append(vs, third && old == 0u, v >> 5);
    return placed || (third && (old & bit) == 0u);
  }
  return placed;
}

// After an expansion's distances (its visits are complete: the wave waited for its row loads, which
// were issued after them, and for its stores), read the spill-table home buckets of the predicted
// next expansion's neighbours (`row_v`, lane-aligned as the next visit will see them).  Used only if
// the prediction holds.
__device__ __forceinline__ void stab_prefetch(const Visited &vs, uint32_t row_v, bool lane_in_row, uint64_t &lo,
                                              uint64_t &hi) {
  lo = hi = 0ull;
  if (lane_in_row && row_v != kEmpty) {
    uint32_t home, code;
    stab_key(vs, row_v, home, code);
    stab_load(vs, home, lo, hi);
  }
}

// Spill with the table as the second level: every id the LDS table holds goes into the spill table
// (compact slots decode back to ids: (slot, probe distance, remainder) gives the hash h, and h times
// the inverse of the multiplicative constant mod 2^L gives v), so a spilled visit never consults
// the LDS table again.  Wave-uniform; table sizes are multiples of 64 slots.
__device__ void stab_flush(Visited &vs) {
  vs.spilled = true;
  const int lane = lane_id();
  const uint32_t hsize = 1u << vs.log2h;
  const uint32_t mask = hsize - 1u;
  wave_sync();
  for (uint32_t b = 0; b < hsize; b += 64) {
    const uint32_t slot = b + static_cast<uint32_t>(lane);
    uint32_t v = kEmpty;
    if (vs.rbits == kVisWide) {
      v = vs.tab[slot];
    } else {
      const uint32_t e = reinterpret_cast<const uint16_t *>(vs.tab)[slot];
      if (e != 0u) {
        const uint32_t x = e - 1u;
        const uint32_t i = x >> vs.rbits;
        const uint32_t rem = x & ((1u << vs.rbits) - 1u);
        const uint32_t home = (slot - i) & mask;
        const uint32_t h = vs.rbits ? ((home << vs.rbits) | rem) : (home >> vs.lshift);
        v = (h * 0x0E8B2F51u) & vs.lmask;  // 0x9E3779B1 * 0x0E8B2F51 == 1 (mod 2^32)
      }
    }
    const bool has = v != kEmpty;
    if (ballot(has)) stab_visit(vs, v, has, false, 0ull, 0ull);
  }
}

// The second level takes over (the bitset is already clean; the spill table gets the LDS entries).
template <bool kTab = false>
__device__ __forceinline__ void spill_begin(Visited &vs) {
  if (kTab && vs.stab != nullptr) {
    stab_flush(vs);
  } else {
    vs.spilled = true;
  }
}

// All lanes with `act` insert their v; duplicates among lanes must have been removed.
// pre_ok (wave-uniform): (pre_lo, pre_hi) hold the lane's second-level state for its v, read one
// expansion ahead (spill_prefetch below, issued for exactly this adjacency row after the previous
// expansion's visits had completed; the wave is the slot's only writer and nothing is visited in
// between).  Spill table: the v's home bucket (stab_visit).  Bitset: pre_lo's low word is v's bitset
// word -- a set bit means visited without a round trip, and a clear one means fresh unless the
// (read-only) first level holds v: its bit is set by an atomic whose result nobody waits for.
template <bool kTab = false>
__device__ __forceinline__ bool visit(Visited &vs, uint32_t v, bool act, bool pre_ok, uint64_t pre_lo,
                                      uint64_t pre_hi) {
  if (kTab && vs.spilled && vs.stab != nullptr) return stab_visit(vs, v, act, pre_ok, pre_lo, pre_hi);
  const uint32_t pre_w = static_cast<uint32_t>(pre_lo);
  bool fresh = false;
  bool global = false;
  if (!vs.spilled) {
    int r = 0;
    if (act) r = table_insert(vs, v);
    fresh = r == 1;
    vs.count += __popcll(ballot(fresh));
    if (ballot(r == 2)) {  // a compact probe ran out of encodable distance: spill now
      if (kTab && vs.stab != nullptr) {
        stab_flush(vs);  // this visit's LDS inserts included; the lanes that failed go to the table
        const bool f2 = stab_visit(vs, v, r == 2, false, 0ull, 0ull);
        return fresh || f2;
      }
      spill_begin(vs);
      global = r == 2;
    }
  } else if (act) {
    global = !(pre_ok && ((pre_w >> (v & 31)) & 1u)) && !table_lookup(vs, v);
  }
  if (vs.spilled) {  // wave-uniform
    const uint32_t bit = 1u << (v & 31);
    uint32_t old = bit;
    if (global && pre_ok) {
      __hip_atomic_fetch_or(&vs.bits[v >> 5], bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      old = pre_w;  // exact: the word as it is now (two lanes of one word may both see it empty;
      fresh = true; // the dirty list then names the word twice, which only clears it twice)
    } else if (global) {
      old = atomicOr(&vs.bits[v >> 5], bit);
      fresh = (old & bit) == 0u;
    }
    // the lane that set a word's first bit records the word (at most one lane per word: the
    // atomics of one wave to one word are serialised, the later ones see the earlier bits)
    dirty_append(vs, global && old == 0u, v >> 5);
  }
  return fresh;
}

template <bool kTab = false>
__device__ __forceinline__ bool visit(Visited &vs, uint32_t v, bool act) {
  return visit<kTab>(vs, v, act, false, 0ull, 0ull);
}

// After an expansion's distances (its visits are complete: the wave waited for its row loads, which
// were issued after them), read the second-level state of the predicted next expansion's adjacency
// row (`row`, lane-aligned as the next visit will see it): the spill table's home buckets, or the
// bitset words.  The loads are agent-scope so they read L2, where the wave's own stores and atomics
// landed, not a stale vector-L1 copy.  Used only if the prediction holds.
__device__ __forceinline__ void spill_prefetch(const Visited &vs, uint32_t row_v, bool lane_in_row, uint64_t &lo,
                                               uint64_t &hi) {
  if (vs.stab != nullptr) {
    stab_prefetch(vs, row_v, lane_in_row, lo, hi);
    return;
  }
  lo = hi = 0ull;
  if (lane_in_row && row_v != kEmpty)
    lo = __hip_atomic_load(&vs.bits[row_v >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// End of a query: leave the slot's second level clean for the next one -- the spill table whole, and
// the bitset's words on the dirty list (or the whole bitset when the list overflowed).  Wave-uniform.
// The spill table is cleared whole on purpose: at its sizing (32 * ef entries, spill_table_log2) a
// query's ~2.7k visited ids land in 1 - exp(-ids / buckets) of the buckets, ~73 % at config 5 (2^14
// entries = 2,048 buckets, ef 368), so a dirty-bucket list would skip at most a quarter of a 32 KB
// clear -- ~0.4 % of the launch's 21.6 GB -- and add a list store per first touch of a bucket plus
// its SGPR state to an expansion loop that is at its register budget.  The clear is full 128-B lines
// of coalesced stores (no read for ownership).
__device__ __forceinline__ void visit_end(Visited &vs) {
  if (!vs.spilled) return;
  const int lane = lane_id();
  __threadfence_block();  // this wave's dirty-list stores are visible to its own loads below
  if (vs.stab != nullptr) {  // agent-scope stores: the next query's agent-scope reads see the zeros
    uint64_t *t = reinterpret_cast<uint64_t *>(vs.stab);
    const uint32_t n8 = 2u * (vs.stab_bmask + 1u);  // two 8-byte halves per bucket
    for (uint32_t i = lane; i < n8; i += 64) __hip_atomic_store(t + i, 0ull, __ATOMIC_RELAXED, ALAYA_STAB_SCOPE);
  }
  // agent-scope stores: the next query's atomics (performed in L2) must find them there
  if (vs.ndirty <= vs.dirty_cap) {
    for (uint32_t i = lane; i < vs.ndirty; i += 64)
      __hip_atomic_store(&vs.bits[vs.dirty[i]], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    for (uint64_t w = lane; w < vs.n_words; w += 64)
      __hip_atomic_store(&vs.bits[w], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the clearing stores land before the slot's next query sets bits (and before its agent-scope
  // spill-table reads)
  stab_order();
  vs.spilled = false;
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
struct NoNext {
  __device__ void operator()(uint32_t) const {}
};

// on_next(id) is called (wave-uniformly, before the shift) when the closest accepted candidate
// lands at or before the first unchecked entry, i.e. when it is the next pop.
struct NoMark {
  __device__ void operator()() const {}
};

template <bool kRegMerge = false, typename OnNext = NoNext, typename Mark = NoMark>
__device__ void pool_merge(PoolState &ps, const Lds &L, bool has, uint32_t id, float d,
                           OnNext on_next = OnNext(), Mark mark = Mark()) {
  const int lane = lane_id();
  const bool full = ps.size == ps.ef;
  const float last = full ? L.pd[ps.size - 1] : 0.f;
  const bool acc = has && !(full && d >= last);
  const uint64_t amask = ballot(acc);
  const uint32_t n_acc = __popcll(amask);
  if (n_acc == 0) return;
  if (kRegMerge && ps.ef <= 128) {
    // Pools of up to 128 entries (ef <= 128: SIFT-shaped searches) merge from registers: lane l
    // holds entries l and 64 + l, and one pass over the accepted lanes yields every candidate's
    // rank, its upper bound in the pool (a ballot count, == the binary search on a sorted pool)
    // and every entry's shift (#accepted strictly below it, == batch_lower_bound) -- no dependent
    // LDS round trips.  A NaN anywhere (pool or batch) takes the binary-search path below, whose
    // answers on such input are the oracle's.
    const uint32_t size = ps.size;
    const bool v0 = static_cast<uint32_t>(lane) < size;
    const bool v1 = static_cast<uint32_t>(lane) + 64 < size;
    const float p0 = v0 ? L.pd[lane] : 0.f;
    const float p1 = v1 ? L.pd[lane + 64] : 0.f;
    const uint32_t i0 = v0 ? L.pi[lane] : 0u;
    const uint32_t i1 = v1 ? L.pi[lane + 64] : 0u;
    if (!ballot((acc && d != d) || (v0 && p0 != p0) || (v1 && p1 != p1))) {
      uint32_t rank = 0, pos = 0, s0 = 0, s1 = 0;
      uint64_t rest = amask;
      // (one lane per trip: the paired loop of the LDS path below was 4-5 % slower here, SIFT-shaped
      // 1M at 10k / 1k queries, profiles/r05/pair/)
      while (rest) {
        const int j = __ffsll(static_cast<unsigned long long>(rest)) - 1;
        rest &= rest - 1;
        const float dj = read_lane(d, j);
        rank += (dj < d || (dj == d && j < lane)) ? 1u : 0u;
        const uint32_t ub = __popcll(ballot(v0 && p0 <= dj)) + __popcll(ballot(v1 && p1 <= dj));
        if (lane == j) pos = ub;
        s0 += dj < p0 ? 1u : 0u;
        s1 += dj < p1 ? 1u : 0u;
      }
      pos += rank;
      const int lane0 = __ffsll(static_cast<unsigned long long>(ballot(acc && rank == 0))) - 1;
      const uint32_t first_pos = read_lane(pos, lane0);
      if (first_pos <= ps.cur) on_next(read_lane(id, lane0));
      mark();
      wave_sync();
      // an entry with a nonzero shift sits at or after first_pos; destinations are distinct
      if (v0 && s0 != 0 && lane + s0 < ps.ef) {
        L.pd[lane + s0] = p0;
        L.pi[lane + s0] = i0;
      }
      if (v1 && s1 != 0 && lane + 64 + s1 < ps.ef) {
        L.pd[lane + 64 + s1] = p1;
        L.pi[lane + 64 + s1] = i1;
      }
      if (acc && pos < ps.ef) {
        L.pd[pos] = d;
        L.pi[pos] = id;
      }
      wave_sync();
      ps.size = min(size + n_acc, ps.ef);
      if (first_pos < ps.cur) ps.cur = first_pos;
      return;
    }
  }
  // stable rank of this candidate among accepted ones, ordered by (dist, arrival)
  uint32_t rank = 0;
  uint64_t rest = amask;
#if ALAYA_PAIR_LOOPS
  while (rest) {  // two accepted lanes per trip (see the register merge above)
    const int j = __ffsll(static_cast<unsigned long long>(rest)) - 1;
    rest &= rest - 1;
    const bool t2 = rest != 0ull;
    const int j2 = t2 ? __ffsll(static_cast<unsigned long long>(rest)) - 1 : j;
    rest &= t2 ? rest - 1 : rest;
    const float dj = read_lane(d, j);
    const float dj2 = read_lane(d, j2);
    rank += (dj < d || (dj == d && j < lane)) ? 1u : 0u;
    rank += (t2 && (dj2 < d || (dj2 == d && j2 < lane))) ? 1u : 0u;
  }
#else
  while (rest) {
    const int j = __ffsll(static_cast<unsigned long long>(rest)) - 1;
    rest &= rest - 1;
    const float dj = read_lane(d, j);
    rank += (dj < d || (dj == d && j < lane)) ? 1u : 0u;
  }
#endif
  if (acc) L.sd[rank] = d;
  uint32_t pos = 0;
  if (acc) pos = pool_upper_bound(L.pd, ps.size, d) + rank;
  // first insertion position = position of the rank-0 element
  const int lane0 = __ffsll(static_cast<unsigned long long>(ballot(acc && rank == 0))) - 1;
  const uint32_t first_pos = read_lane(pos, lane0);
  if (first_pos <= ps.cur) on_next(read_lane(id, lane0));
  mark();  // diagnostics: end of the rank / position phase
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

// LinearPool::pop: mark cur checked, advance to the next unchecked entry.  kNext: also report the
// ids of the first two unchecked entries after the pop (c1 = the new cur; c2 only from the same
// 64-entry scan, else kEmpty) -- the distance helpers' requests.
template <bool kNext = false>
__device__ __forceinline__ uint32_t pool_pop(PoolState &ps, const Lds &L, uint32_t *c1 = nullptr,
                                             uint32_t *c2 = nullptr) {
  const int lane = lane_id();
  const uint32_t raw = L.pi[ps.cur];
  wave_sync();
  if (lane == 0) L.pi[ps.cur] = raw | kChecked;
  uint32_t next = ps.size;
  if constexpr (kNext) *c1 = *c2 = kEmpty;
  for (uint32_t b = ps.cur + 1; b < ps.size; b += 64) {
    const uint32_t j = b + lane;
    const uint32_t pij = j < ps.size ? L.pi[j] : kChecked;
    const bool un = !(pij & kChecked);
    const uint64_t mk = ballot(un);
    if (mk) {
      const int f = __ffsll(static_cast<unsigned long long>(mk)) - 1;
      next = b + f;
      if constexpr (kNext) {
        *c1 = read_lane(pij & kIdMask, f);
        const uint64_t mk2 = mk & (mk - 1ull);
        if (mk2) *c2 = read_lane(pij & kIdMask, __ffsll(static_cast<unsigned long long>(mk2)) - 1);
      }
      break;
    }
  }
  wave_sync();
  ps.cur = next;
  return raw & kIdMask;
}

}  // namespace
}  // namespace alaya_amd
