// Flat (brute-force) exact k-NN on gfx950: the MFMA contraction -2 Q B^T + |b|^2 with a fused
// per-query shortlist, then an exact rescoring pass.  The reference has no FLAT index
// (IndexType::FLAT is enum-only, include/index/index_type.hpp:28); its brute-force analogues are
// find_exact_gt (include/utils/evaluate.hpp:29-62) and calc_gt (python/src/alayalite/utils.py:99-105).
// Result contract: the k nearest rows by the reference metric function (l2_sqr_avx2 order, the same
// device function as the graph search) with ties broken by id, plus a per-query flag that is set
// when the shortlist cannot be proven to contain them (error bound below) -- the host then
// recomputes that query exhaustively.
//
// flat_scan_kernel: 256 threads = 4 waves, 128 queries per block (32 per wave), one base chunk per
// block.  Each wave holds its 32 queries as MFMA A fragments in VGPRs: lane l owns query (l & 31),
// k in [h*K/2, (h+1)*K/2) with h = l >> 5 (the k order is free -- the GEMM only ranks candidates).
// Base rows stream through a double-buffered LDS tile of 32 rows.  Default contraction: each f32 is
// split into bf16 hi + lo when the tile is staged, and a 32-row tile costs 3 K/16
// v_mfma_f32_32x32x16_bf16 (qh.bh + qh.bl + ql.bh); the f32 form (ALAYA_FLAT_F32) issues K/2
// v_mfma_f32_32x32x2f32.  Both fill one 32x32 accumulator (C[query][row]: row = lane & 31, query =
// (r&3) + 8(r>>2) + 4h for accumulator register r).  Approximate distance a = |b|^2 - 2 C.
// Candidates below the query's running threshold are appended to a per-query LDS buffer (a stack).
// The shortlists themselves live in registers laid out like the accumulator (register r, half h
// <-> query (r&3) + 8(r>>2) + 4h, entry = lane & 31), so 32 buffered candidates at a time are
// folded in by a 32-lane bitonic sort + merge on DPP / ds_swizzle lane exchanges, without leaving
// the half-wave that owns the query.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <cstdlib>

#include "flat_kernels.h"

namespace alaya_amd {
namespace {

constexpr int kL = 32;       // shortlist per (query, chunk)
constexpr int kBuf = 96;     // candidate buffer per query
constexpr int kTile = 32;    // base rows per LDS tile
constexpr int kPad = 4;      // LDS row pitch padding (floats)
constexpr int kWideTiles = 4;  // row tiles per super-chunk of the wide scan
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Split contraction (kSplit): x = hi + lo + r with hi = bf16(x), lo = bf16(x - hi) (x - hi is exact
// in f32), |r| <= 2^-16 |x|.  q.b ~= qh.bh + qh.bl + ql.bh: three v_mfma_f32_32x32x16_bf16 per 16 k
// (products exact in f32) instead of eight v_mfma_f32_32x32x2f32 -- 768 vs 4096 MFMA cycles per
// 32x32x128 tile.  The dropped terms are bounded by ~3 * 2^-16 |q||b| (flat_merge_kernel's eps).
__device__ __forceinline__ void split_bf16(float x, __bf16 &hi, __bf16 &lo) {
  hi = static_cast<__bf16>(x);
  lo = static_cast<__bf16>(x - static_cast<float>(hi));
}

// Single-pass f16 contraction (FlatParams::single, the warp-specialised scan): one
// v_mfma_f32_32x32x16_f16 per 16 k on operands scaled by powers of two into f16's range -- rows by
// 2^s (base_exp, from the largest row norm: max|b| 2^s < 2^15), each query by its own 2^t (its
// largest element, t = f16_exp(max|q|)) -- so C = 2^-(s+t) (q 2^t).(b 2^s) with exact scaling.
// f16 keeps 11 significant bits: each operand is within 2^-11 relative (plus 2^-14 absolute, in
// scaled units, should a tiny element flush to zero) of its f32 value, so the dropped terms are
// bounded by ~2^-10 |q||b| (flat_merge_kernel's eps) -- 8x the split's bound, still far inside the
// 10th-to-32nd distance gap of real data, at a third of the MFMAs and half the tile bytes.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr int kF16Top = 15;    // scaled operands stay below 2^15 (f16 max 65504)
constexpr int kF16MaxExp = 100;  // |s + t| beyond this: the query is flagged (its scale-back leaves f32's range)
// 2^t with |x| 2^t < 2^kF16Top for every |x| <= maxabs (0 for a zero or non-finite maxabs)
__device__ __host__ __forceinline__ int f16_exp(float maxabs) {
  if (!(maxabs > 0.f) || !(maxabs < 3.0e38f)) return 0;
  int e = 0;
  (void)frexpf(maxabs, &e);  // maxabs < 2^e
  return kF16Top - e;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// (d, tie) total order used by every selection below: smaller distance first, then smaller tie key
__device__ __forceinline__ bool before(float da, uint32_t ta, float db, uint32_t tb) {
  return da < db || (da == db && ta < tb);
}

// Lane xor within each 32-lane half.  xor 1/2: DPP quad_perm; xor 8: DPP row_ror:8 (rows of 16);
// xor 4: row_ror:12 or row_ror:4 by lane bit 2 (row_ror:n reads lane (l - n) mod 16 of the row) -- all VALU, no LDS-pipeline round trip.  xor 16 and
// the 31-reversal: bit-mode ds_swizzle (source lane = ((l & 0x1f) | or) ^ xor, inside the half).
template <int kXor>
__device__ __forceinline__ int xor_lane(int v) {
  if constexpr (kXor == 1) {
    return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (kXor == 2) {
    return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (kXor == 8) {
    return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (kXor == 4) {
    const int up = __builtin_amdgcn_update_dpp(0, v, 0x12C, 0xF, 0xF, false);    // row_ror:12 (l + 4)
    const int down = __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4  (l - 4)
    return (__lane_id() & 4) ? down : up;
  } else {
    return __builtin_amdgcn_ds_swizzle(v, 0x1f | (kXor << 10));
  }
}
template <int kXor>
__device__ __forceinline__ float swz_f(float v) {
  return __int_as_float(xor_lane<kXor>(__float_as_int(v)));
}
template <int kXor>
__device__ __forceinline__ uint32_t swz_u(uint32_t v) {
  return static_cast<uint32_t>(xor_lane<kXor>(static_cast<int>(v)));
}
__device__ __forceinline__ float lane31_of_half(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 31 << 5));
}

// One compare-exchange of a bitonic network over the 32 lanes of a half (block size K, distance J).
template <int K, int J>
__device__ __forceinline__ void cmpx(float &d, uint32_t &i, int col) {
  const bool take_min = ((col & K) == 0) == ((col & J) == 0);
  const float od = swz_f<J>(d);
  const uint32_t oi = swz_u<J>(i);
  // branch-free (d, id) comparison: short-circuit forms compile to nested exec-mask branches
  const bool eq = od == d;
  const bool o_first = (od < d) | (eq & (oi < i));
  const bool m_first = (d < od) | (eq & (i < oi));
  const bool sw = (take_min & o_first) | (!take_min & m_first);
  d = sw ? od : d;
  i = sw ? oi : i;
}
// bitonic sequence -> ascending
__device__ __forceinline__ void bitonic_merge32(float &d, uint32_t &i, int col) {
  cmpx<32, 16>(d, i, col);
  cmpx<32, 8>(d, i, col);
  cmpx<32, 4>(d, i, col);
  cmpx<32, 2>(d, i, col);
  cmpx<32, 1>(d, i, col);
}
__device__ __forceinline__ void bitonic_sort32(float &d, uint32_t &i, int col) {
  cmpx<2, 1>(d, i, col);
  cmpx<4, 2>(d, i, col);
  cmpx<4, 1>(d, i, col);
  cmpx<8, 4>(d, i, col);
  cmpx<8, 2>(d, i, col);
  cmpx<8, 1>(d, i, col);
  cmpx<16, 8>(d, i, col);
  cmpx<16, 4>(d, i, col);
  cmpx<16, 2>(d, i, col);
  cmpx<16, 1>(d, i, col);
  bitonic_merge32(d, i, col);
}
// Fold 32 candidates (one per lane of the half, any order) into the ascending list (L, Li):
// sort them, pair list[c] with candidate[31-c] (the min of each pair is a bitonic sequence holding
// the 32 smallest of the union), re-sort.
__device__ __forceinline__ void fold32_sorted(float &L, uint32_t &Li, float cd, uint32_t ci, int col) {
  const float rd = swz_f<31>(cd);
  const uint32_t ri = swz_u<31>(ci);
  const bool take = (rd < L) | ((rd == L) & (ri < Li));
  L = take ? rd : L;
  Li = take ? ri : Li;
  bitonic_merge32(L, Li, col);
}
__device__ __forceinline__ void fold32(float &L, uint32_t &Li, float cd, uint32_t ci, int col) {
  bitonic_sort32(cd, ci, col);
  fold32_sorted(L, Li, cd, ci, col);
}

// Shortlists of one wave (32 queries) in registers with the accumulator's layout: register r of
// half h holds the ascending list of query (r & 3) + 8 (r >> 2) + 4h, entry (lane & 31).  cnt[r] =
// buffered candidates of that query (uniform over the half), tau[r] = its current 32nd distance;
// full / nonempty: registers whose buffer holds >= kTile / > 0 candidates (uniform).
// (vector values, not arrays: the fold picks a register by value, which the compiler turns into a
// dynamic index -- on an array that means scratch memory, on a vector a register move)
// A consumer may own only part of an accumulator: NR registers starting at register R0 (the
// two-consumer scan splits the 16 between two waves); register r of the part is accumulator
// register R0 + r.
template <int N>
using f32xN = float __attribute__((ext_vector_type(N)));
template <int N>
using u32xN = uint32_t __attribute__((ext_vector_type(N)));
template <int N>
using i32xN = int __attribute__((ext_vector_type(N)));
template <int NR = 16>
struct ShortlistsT {
  f32xN<NR> ld, tau;
  u32xN<NR> li;
  i32xN<NR> cnt;
  uint32_t full, nonempty;
};
using Shortlists = ShortlistsT<16>;

// wave-local query of accumulator register r (half h of the wave)
__device__ __forceinline__ constexpr int reg_query(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

template <int NR = 16, int R0 = 0>
__device__ __forceinline__ void init_shortlists(const FlatParams &p, uint64_t q0, int h, ShortlistsT<NR> &S) {
  S.full = S.nonempty = 0;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    S.ld[r] = FLT_MAX;
    S.li[r] = 0xffffffffu;
    const uint64_t qi = q0 + reg_query(R0 + r, h);
    // a slot past the last query takes no candidates (-FLT_MAX: no `d < tau` holds), so a partial
    // query group does no append or fold work for its empty slots
    S.tau[r] = qi < p.nq ? (p.tau_init ? p.tau_init[qi] : FLT_MAX) : -FLT_MAX;
    S.cnt[r] = 0;
  }
}

// write the per-(chunk, query) shortlist
template <int NR = 16, int R0 = 0>
__device__ __forceinline__ void store_shortlists(const FlatParams &p, uint64_t q0, int chunk, const ShortlistsT<NR> &S) {
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const uint64_t qi = q0 + reg_query(R0 + r, h);
    if (qi < p.nq) {
      const uint64_t o = (static_cast<uint64_t>(chunk) * p.nq + qi) * kL + col;
      p.cand_d[o] = S.ld[r];
      p.cand_i[o] = S.li[r];
    }
  }
}

template <int kB, int NR, int R0>
__device__ __forceinline__ void fold_rounds(const FlatParams &p, uint32_t need, bool last, ShortlistsT<NR> &S,
                                            float *bd, uint32_t *bi);

// Candidate handling of one 32-row tile: approximate distances a = |b|^2 - 2 c[r] below the
// query's threshold are appended to its LDS buffer (bd/bi, a stack per query), then the fold
// rounds that became due run.  last: the wave's final tile (every buffer is drained).  kDv: c
// already holds the approximate distances (the single-role f16 scan computes them first to test
// the whole tile at once); bn is then unused.
template <int kB = kBuf, int NR = 16, int R0 = 0, bool kDv = false>
__device__ __forceinline__ void tile_candidates(const FlatParams &p, const f32xN<NR> &c, float bn, uint32_t rid,
                                                uint64_t live_mask, bool last, ShortlistsT<NR> &S, float *bd,
                                                uint32_t *bi, uint64_t &t_app, uint64_t &t_fold) {
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  // append candidates below each query's threshold (counts stay in registers).  The common case
  // per register is fma, compare, one uniform branch: the bookkeeping for folds (`S.full`,
  // `S.nonempty`, `need`) changes only when a register takes an append, so it lives inside that
  // branch, in scalar masks carried across tiles.
  const uint64_t ta = p.merge_count ? __builtin_amdgcn_s_memtime() : 0;
  uint32_t need = 0;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int qloc = reg_query(R0 + r, h);  // wave-local query of register r, half h
    const float dv = kDv ? c[r] : fmaf(-2.0f, c[r], bn);
    // the compare's lane mask straight from v_cmp (llvm.amdgcn.fcmp, predicate OLT = 4), no
    // bool round trip through a VGPR
    const uint64_t mk = __builtin_amdgcn_fcmpf(dv, S.tau[r], 4) & live_mask;
    const bool pass = (mk >> lane) & 1;
    if (mk) {
      const uint32_t hm = h ? static_cast<uint32_t>(mk >> 32) : static_cast<uint32_t>(mk);
      if (pass) {
        const int pos = S.cnt[r] + __popc(hm & ((1u << col) - 1u));
        bd[qloc * kB + pos] = dv;
        bi[qloc * kB + pos] = rid;
      }
      S.cnt[r] += __popc(hm);
      S.nonempty |= 1u << r;
      if (__builtin_amdgcn_ballot_w64(S.cnt[r] >= kTile)) {
        S.full |= 1u << r;
        if (__builtin_amdgcn_ballot_w64(S.cnt[r] > kB - kTile)) need |= 1u << r;  // could overflow next tile
      }
    }
  }
  // A fold round takes the newest 32 entries of a buffer (it is a stack), so a round costs the
  // same wherever it happens.  Due rounds: buffers that could overflow on the next tile (one round
  // brings > 64 down to <= 64).  Smoothing: otherwise one round of a buffer holding a S.full batch.
  // At most ~one round per wave per tile keeps the four waves level between barriers.  The last
  // tile drains every buffer.
  if (last) need |= S.nonempty;
  if (need == 0 && S.full) need = 1u << __builtin_ctz(S.full);
  if (p.ablate == 2) {  // diagnostics: appends only, buffers dropped instead of folded
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (need & (1u << r)) S.cnt[r] = 0;
    S.full &= ~need;
    S.nonempty &= ~need;
    need = 0;
  }
  const uint64_t tf = p.merge_count ? __builtin_amdgcn_s_memtime() : 0;
  t_app += tf - ta;
  fold_rounds<kB, NR, R0>(p, need, last, S, bd, bi);
  t_fold += (p.merge_count ? __builtin_amdgcn_s_memtime() : 0) - tf;
}

// Fold rounds for the registers in `need` (each: the newest 32 buffered entries of its two queries,
// one per half; last: repeated until the buffer is empty).  One copy of the fold body (a uniform
// loop over `need`, the register picked by value): unrolling it per register would put ~48 KB of
// code in the loop and thrash the instruction cache.
template <int kB, int NR, int R0>
__device__ __forceinline__ void fold_rounds(const FlatParams &p, uint32_t need, bool last, ShortlistsT<NR> &S,
                                            float *bd, uint32_t *bi) {
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  if (need) {
    wave_fence();
    do {
      const int r = __builtin_ctz(need);
      need &= need - 1;
      float L = S.ld[0];
      uint32_t Li = S.li[0];
      int cr = S.cnt[0];
#pragma unroll
      for (int r2 = 1; r2 < NR; ++r2) {
        if (r2 == r) {
          L = S.ld[r2];
          Li = S.li[r2];
          cr = S.cnt[r2];
        }
      }
      const int qloc = reg_query(R0 + r, h);
      do {  // one round; the last tile repeats until the buffer is empty
        const int start = max(cr - 32, 0);  // uniform per half
        float cd = FLT_MAX;
        uint32_t ci = 0xffffffffu;
        if (start + col < cr) {
          cd = bd[qloc * kB + start + col];
          ci = bi[qloc * kB + start + col];
        }
        fold32(L, Li, cd, ci, col);
        cr = start;
      } while (last && __builtin_amdgcn_ballot_w64(cr > 0));
      if (__builtin_amdgcn_ballot_w64(cr >= kTile)) S.full |= 1u << r;
      else S.full &= ~(1u << r);
      if (!__builtin_amdgcn_ballot_w64(cr > 0)) S.nonempty &= ~(1u << r);
      const float th = lane31_of_half(L);
#pragma unroll
      for (int r2 = 0; r2 < NR; ++r2) {
        if (r2 == r) {
          S.ld[r2] = L;
          S.li[r2] = Li;
          S.cnt[r2] = cr;
          S.tau[r2] = th;
        }
      }
      if (lane == 0 && p.merge_count) atomicAdd(p.merge_count + blockIdx.x, 1u);
    } while (need);
    wave_fence();
  }
}

// fold_rounds with static register indices (an unrolled loop, one fold body per register): the
// single-role scan folds rarely, and picking the register by value made the compiler copy all 64
// shortlist registers on every record of the hot loop; the 16 bodies cost code size instead.
// The single-role scan's shortlist state as plain arrays with static indices only (scalars after
// SROA): a whole-vector value would be copied at every control-flow join of the hot loop.
struct TilesLists {
  float tau[16];
  uint32_t nonempty;
  float *ld;     // LDS: this wave's 32 queries x kL shortlist distances (ascending)
  uint32_t *li;  // and ids
  uint32_t *cnt;  // LDS: buffered candidates per query
};

template <int kB>
__device__ __forceinline__ void fold_rounds_static(const FlatParams &p, uint32_t need, bool last, TilesLists &S,
                                                   const uint64_t *gb) {
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  // this wave's appends (global stores) have completed before it reads them back, past L1
  __builtin_amdgcn_s_waitcnt(0x70);  // vmcnt(0) lgkmcnt(0)
  wave_fence();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (!(need & (1u << r))) continue;
    const int qloc = reg_query(r, h);
    float L = S.ld[qloc * kL + col];
    uint32_t Li = S.li[qloc * kL + col];
    // an append past kB was counted but not stored: the buffer holds min(count, kB)
    int cr = min(static_cast<int>(S.cnt[qloc]), kB);
    do {  // one round; the last record repeats until the buffer is empty
      const int start = max(cr - 32, 0);  // uniform per half
      float cd = FLT_MAX;
      uint32_t ci = 0xffffffffu;
      if (start + col < cr) {
        const uint64_t v = __hip_atomic_load(gb + qloc * kB + start + col, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cd = __uint_as_float(static_cast<uint32_t>(v));
        ci = static_cast<uint32_t>(v >> 32);
      }
      fold32(L, Li, cd, ci, col);
      cr = start;
    } while (last && __builtin_amdgcn_ballot_w64(cr > 0));
    S.ld[qloc * kL + col] = L;
    S.li[qloc * kL + col] = Li;
    if (col == 0) S.cnt[qloc] = static_cast<uint32_t>(cr);
    if (!__builtin_amdgcn_ballot_w64(cr > 0)) S.nonempty &= ~(1u << r);
    S.tau[r] = lane31_of_half(L);
    if (lane == 0 && p.merge_count) atomicAdd(p.merge_count + blockIdx.x, 1u);
  }
  wave_fence();
}

// OR of a per-lane mask over the wave
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
  v |= __shfl_xor(v, 1);
  v |= __shfl_xor(v, 2);
  v |= __shfl_xor(v, 4);
  v |= __shfl_xor(v, 8);
  v |= __shfl_xor(v, 16);
  v |= __shfl_xor(v, 32);
  return __builtin_amdgcn_readfirstlane(v);
}

template <int K, bool kSplit>
__global__ void __launch_bounds__(256) flat_scan_kernel(FlatParams p) {
  static_assert(K % 16 == 0 && K <= 256, "K must be a multiple of 16, at most 256");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // f32: row pitch K+4 floats.  split: a hi and a lo half-tile of bf16 rows with pitch K+8 (2K+16
  // bytes, so the 16 rows of a ds_read_b128 group start on distinct 16-byte bank quads).
  constexpr int kPitch = K + kPad;
  constexpr int kBPitch = K + 8;
  constexpr int kTileWords = kSplit ? kTile * kBPitch : kTile * kPitch;  // 4-byte words per buffer
  float *tile = reinterpret_cast<float *>(smem);                       // 2 x kTileWords
  float *nrm = tile + 2 * kTileWords;                                   // 2 x kTile
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  float *bd = tile + 2 * kTileWords + 2 * kTile + wave * 32 * kBuf * 2;  // 32 queries x kBuf
  uint32_t *bi = reinterpret_cast<uint32_t *>(bd + 32 * kBuf);

  // XCD-aware block -> (query group, chunk): the query groups of one chunk share an XCD label.
  const int nqg = static_cast<int>((p.nq + 127) / 128);
  const int b = blockIdx.x;
  const int qg = (b / 8) % nqg;
  const int chunk = (b % 8) + 8 * (b / (8 * nqg));
  if (chunk >= p.n_chunks) return;
  const uint64_t rows_per_chunk = (p.n + p.n_chunks - 1) / p.n_chunks;
  const uint64_t r0 = chunk * rows_per_chunk;
  const uint64_t r1 = min(p.n, r0 + rows_per_chunk);

  // A fragments: query q0 + col, k in [h*K/2, h*K/2 + K/2)
  const uint64_t q0 = static_cast<uint64_t>(qg) * 128 + wave * 32;
  float a[K / 2];
  {
    const uint64_t qi = q0 + col;
    // elements past dim are zero (the query rows are dim apart, not stride apart: reading past dim
    // would take the next query's values or, for the last query, bytes past the buffer -- finite or
    // not, and Inf/NaN times the base's zero padding is NaN); scalar loads, once per kernel
    const uint32_t e0 = h * (K / 2);
    const float *qp = p.queries + qi * p.q_stride;
#pragma unroll
    for (int s = 0; s < K / 2; ++s) a[s] = (qi < p.nq && e0 + s < p.dim) ? qp[e0 + s] : 0.f;
  }
  // split: k-step s of lane (col, h) holds query elements h*K/2 + 8s + j, j < 8 (the base fragment
  // below uses the same map, so the MFMA's k = 8h + j pairs equal elements)
  bf16x8 ah[kSplit ? K / 16 : 1], al[kSplit ? K / 16 : 1];
  if constexpr (kSplit) {
#pragma unroll
    for (int s = 0; s < K / 16; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        __bf16 hi, lo;
        split_bf16(a[8 * s + j], hi, lo);
        ah[s][j] = hi;
        al[s][j] = lo;
      }
  }
  Shortlists S;
  init_shortlists(p, q0, h, S);

  // cooperative tile load: 32 rows x K floats, 256 threads, float4 each
  constexpr int kVecPerRow = K / 4;
  constexpr int kVecs = kTile * kVecPerRow;
  constexpr int kPerThread = (kVecs + 255) / 256;
  auto load_tile = [&](uint64_t row0, float4 (&reg)[kPerThread], float (&nr)[1]) {
#pragma unroll
    for (int v = 0; v < kPerThread; ++v) {
      const int idx = threadIdx.x + v * 256;
      reg[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (idx < kVecs) {
        const uint64_t row = row0 + idx / kVecPerRow;
        if (row < r1)
          reg[v] = *reinterpret_cast<const float4 *>(p.base + row * p.row_step * p.stride + (idx % kVecPerRow) * 4);
      }
    }
    nr[0] = 0.f;
    if (threadIdx.x < kTile) {
      const uint64_t row = row0 + threadIdx.x;
      nr[0] = row < r1 ? p.norms[row * p.row_step] : FLT_MAX;
    }
  };
  auto store_tile = [&](int buf, const float4 (&reg)[kPerThread], const float (&nr)[1]) {
    float *t = tile + buf * kTileWords;
#pragma unroll
    for (int v = 0; v < kPerThread; ++v) {
      const int idx = threadIdx.x + v * 256;
      if (idx < kVecs) {
        if constexpr (kSplit) {
          // split once per tile here, not per wave at the fragment reads
          __bf16 *th = reinterpret_cast<__bf16 *>(t) + (idx / kVecPerRow) * kBPitch + (idx % kVecPerRow) * 4;
          bf16x4 hv, lv;
          __bf16 hi, lo;
          split_bf16(reg[v].x, hi, lo); hv[0] = hi; lv[0] = lo;
          split_bf16(reg[v].y, hi, lo); hv[1] = hi; lv[1] = lo;
          split_bf16(reg[v].z, hi, lo); hv[2] = hi; lv[2] = lo;
          split_bf16(reg[v].w, hi, lo); hv[3] = hi; lv[3] = lo;
          *reinterpret_cast<bf16x4 *>(th) = hv;
          *reinterpret_cast<bf16x4 *>(th + kTile * kBPitch) = lv;
        } else {
          *reinterpret_cast<float4 *>(t + (idx / kVecPerRow) * kPitch + (idx % kVecPerRow) * 4) = reg[v];
        }
      }
    }
    if (threadIdx.x < kTile) nrm[buf * kTile + threadIdx.x] = nr[0];
  };

  float4 stage[kPerThread];
  float stage_n[1];
  load_tile(r0, stage, stage_n);
  store_tile(0, stage, stage_n);
  __syncthreads();
  int buf = 0;
  uint64_t t_fold = 0, t_bar = 0, t_app = 0;
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  for (uint64_t row0 = r0; row0 < r1; row0 += kTile) {
    const bool more = row0 + kTile < r1;
    if (more) load_tile(row0 + kTile, stage, stage_n);  // next tile in flight during the MFMAs
    f32x16 c = {};
    if constexpr (kSplit) {
      const __bf16 *tb = reinterpret_cast<const __bf16 *>(tile + buf * kTileWords) + col * kBPitch + h * (K / 2);
#pragma unroll
      for (int s = 0; s < K / 16; ++s) {
        const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(tb + 8 * s);
        const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(tb + kTile * kBPitch + 8 * s);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bh, c, 0, 0, 0);
      }
    } else {
      const float *t = tile + buf * kTile * kPitch + col * kPitch + h * (K / 2);
#pragma unroll
      for (int s = 0; s < K / 2; s += 4) {
        const float4 bv = *reinterpret_cast<const float4 *>(t + s);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bv.x, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s + 1], bv.y, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s + 2], bv.z, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s + 3], bv.w, c, 0, 0, 0);
      }
    }
    const float bn = nrm[buf * kTile + col];
    const uint32_t rid = static_cast<uint32_t>((row0 + col) * p.row_step);
    bool live = row0 + col < r1;
    if (p.valid != nullptr && live) live = (p.valid[rid >> 5] >> (rid & 31)) & 1u;
    const uint64_t live_mask = __builtin_amdgcn_ballot_w64(live);
    if (p.ablate == 1) {  // diagnostics: keep the accumulator live, skip the candidate path
      float sink = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sink += c[r];
      if (sink == -1.2345f) p.flags[0] = 7;
      if (more) {
        store_tile(buf ^ 1, stage, stage_n);
        buf ^= 1;
      }
      __syncthreads();
      continue;
    }
    tile_candidates(p, c, bn, rid, live_mask, !more, S, bd, bi, t_app, t_fold);
    const uint64_t tb = p.merge_count ? __builtin_amdgcn_s_memtime() : 0;
    if (more) {
      store_tile(buf ^ 1, stage, stage_n);
      buf ^= 1;
    }
    __syncthreads();
    if (p.merge_count) t_bar += __builtin_amdgcn_s_memtime() - tb;
  }
  if (p.merge_count && lane == 0) {
    // diagnostics: per-wave cycle split (s_memtime ticks) after the per-block merge counters
    unsigned long long *st = reinterpret_cast<unsigned long long *>(p.merge_count + 4096) + (blockIdx.x * 4 + wave) * 4;
    st[0] = __builtin_amdgcn_s_memtime() - t_start;
    st[1] = t_app;
    st[2] = t_fold;
    st[3] = t_bar;
  }
  store_shortlists(p, q0, chunk, S);
}

// --------------------------------------------------------------------------------------------
// Narrow rows, warp-specialised (the default for stride <= 224, split contraction): 512 threads
// = 4 producer waves + 4 consumer waves.  Producer wave w holds the A fragments of queries
// 32w .. 32w+31, stages the block's 32-row tiles and turns each tile into its 32x32 contraction,
// written to slot t % kD of an LDS ring; consumer wave 4 + w runs the candidate handling (appends,
// fold rounds, register shortlists -- tile_candidates, unchanged) on the contractions in order.
// The waves of a pair share a SIMD, so the consumer's VALU work issues in the gaps of the
// producer's MFMA chain.  No block-wide barrier per tile: a pair hands tiles over through LDS
// flags (producer w publishes tile t, consumer w acknowledges it), and only the four producers
// meet per tile (an LDS counter) because they stage the shared tile together.  A consumer that
// draws a fold round falls up to kD - 1 tiles behind its producer instead of stalling all eight
// waves at a barrier (the fold rounds of the four consumers fall on different tiles).
// --------------------------------------------------------------------------------------------
// Default poll limit (p.spin_limit): ~0.1 s of polling, so a protocol error ends the scan, not the
// GPU.  ALAYA_FLAT_SPIN_LIMIT overrides it (tests force aborts with a tiny limit).
// Wait until *a >= v (wave-uniform).  False when the block aborted (a wait ran past the limit):
// every later wait then returns at once, the loops end and the shortlists are written as
// unprovable (see flat_scan_ws_kernel), so the merge flags the queries for the exhaustive redo.
__device__ __forceinline__ bool lds_wait_ge(uint32_t *a, uint32_t v, uint32_t *abort, uint32_t limit) {
  for (uint32_t n = 0;; ++n) {
    if (__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) break;
    if (__hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u) return false;
    if (n >= limit) {
      if (__lane_id() == 0) __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");  // later LDS reads after the flag
  return true;
}
// Publish v in *a after this wave's earlier LDS writes (LDS operations of a wave complete in order).
__device__ __forceinline__ void lds_publish(uint32_t *a, uint32_t v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (__lane_id() == 0) __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The consumer side of flat_scan_ws_kernel: wave `cw` of the pair w handles accumulator registers
// [R0, R0 + NR) of its producer's tiles -- all 16 with one consumer per producer, 8 each with two.
template <int kB, int kD, int kCons, int NR, int R0, bool kOne>
__device__ __forceinline__ void ws_consume(const FlatParams &p, const float *cx, uint32_t *published,
                                           uint32_t *consumed, uint32_t *abort, float *bd, uint32_t *bi, int w,
                                           int half, uint64_t q0, int chunk, int ntiles, uint64_t r0, uint64_t r1,
                                           const int *qexp) {
  const int lane = lane_id();
  const int h = lane >> 5;
  ShortlistsT<NR> S;
  init_shortlists<NR, R0>(p, q0, h, S);
  uint64_t t_app = 0, t_fold = 0;
  __syncthreads();
  // single-pass f16: the contraction comes in scaled units; 2^-(s + t) per register's query (the
  // producers wrote each query's t before the barrier)
  f32xN<NR> unscale;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    unscale[r] = kOne ? ldexpf(1.0f, -(p.base_exp + qexp[w * 32 + reg_query(R0 + r, h)])) : 1.0f;
  const bool diag = p.merge_count != nullptr;
  uint64_t t_wait = 0;
  const uint64_t t_start = diag ? __builtin_amdgcn_s_memtime() : 0;
  int slot = 0;
  bool ok = true;
  const int col = lane & 31;
  for (int t = 0; t < ntiles; ++t) {
    const uint64_t tw = diag ? __builtin_amdgcn_s_memtime() : 0;
    if (!lds_wait_ge(&published[w], static_cast<uint32_t>(t + 1), abort, p.spin_limit)) {
      ok = false;
      break;
    }
    if (diag) t_wait += __builtin_amdgcn_s_memtime() - tw;
    const uint64_t row0 = r0 + static_cast<uint64_t>(kTile) * t;
    const uint64_t row = row0 + col;
    const uint32_t rid = static_cast<uint32_t>(row * p.row_step);
    bool live = row < r1;
    const float bn = p.norms[(live ? row : r0) * p.row_step];
    if (p.valid != nullptr && live) live = (p.valid[rid >> 5] >> (rid & 31)) & 1u;
    const uint64_t live_mask = __builtin_amdgcn_ballot_w64(live);
    const float *in = cx + ((slot * 4 + w) * 16 + R0) * 64 + lane;
    f32xN<NR> c;
#pragma unroll
    for (int r = 0; r < NR; ++r) c[r] = in[r * 64];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slot's reads are done before it is released
    if constexpr (kOne) {
#pragma unroll
      for (int r = 0; r < NR; ++r) c[r] *= unscale[r];  // a power of two: exact
    }
    lds_publish(&consumed[w * kCons + half], static_cast<uint32_t>(t + 1));
    slot = slot + 1 == kD ? 0 : slot + 1;
    tile_candidates<kB, NR, R0>(p, c, bn, rid, live_mask, t == ntiles - 1, S, bd, bi, t_app, t_fold);
  }
  if (!ok) {
    // aborted: an unprovable shortlist (cutoff -FLT_MAX, no ids) makes the merge flag every query
    // of the group, and the flagged queries are recomputed exhaustively
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      S.ld[r] = -FLT_MAX;
      S.li[r] = 0xffffffffu;
    }
  }
  if (diag && lane == 0) {  // diagnostics: total, appends, fold rounds, waiting for the producer
    unsigned long long *st =
        reinterpret_cast<unsigned long long *>(p.merge_count + 4096) + (blockIdx.x * 4 * kCons + w * kCons + half) * 4;
    st[0] = __builtin_amdgcn_s_memtime() - t_start;
    st[1] = t_app;
    st[2] = t_fold;
    st[3] = t_wait;
  }
  store_shortlists<NR, R0>(p, q0, chunk, S);
}

// kOne: the single-pass f16 contraction (one MFMA per 16 k, an f16 tile); else the bf16 hi/lo split.
template <int K, int kB, int kD, int kCons, bool kOne>
__global__ void __launch_bounds__(256 * (1 + kCons)) flat_scan_ws_kernel(FlatParams p) {
  static_assert(K % 16 == 0 && K <= 224, "narrow rows");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kBPitch = K + 8;
  // 4-byte words per tile buffer: hi + lo bf16 half-tiles (split), one f16 tile (single pass)
  constexpr int kTileWords = kOne ? kTile * kBPitch / 2 : kTile * kBPitch;
  float *tile = reinterpret_cast<float *>(smem);                   // 2 x kTileWords
  float *cx = tile + 2 * kTileWords;                                // kD x 4 waves x 16 regs x 64 lanes
  uint32_t *sync = reinterpret_cast<uint32_t *>(cx + kD * 4 * 16 * 64 + 4 * 32 * kB * 2);
  uint32_t *published = sync;                // [w]: tiles pair w's producer has written
  uint32_t *consumed = sync + 4;             // [w * kCons + c]: tiles pair w's consumer c has read
  uint32_t *staged = sync + 4 + 4 * kCons;   // producer arrivals (4 per tile)
  uint32_t *abort = staged + 1;
  int *qexp = reinterpret_cast<int *>(sync + 16);  // single pass: each query's scale exponent t (128)
  const int wave = threadIdx.x >> 6;
  const int w = wave & 3;
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;

  const int nqg = static_cast<int>((p.nq + 127) / 128);
  const int b = blockIdx.x;
  const int qg = (b / 8) % nqg;
  const int chunk = (b % 8) + 8 * (b / (8 * nqg));
  if (chunk >= p.n_chunks) return;
  const uint64_t rows_per_chunk = (p.n + p.n_chunks - 1) / p.n_chunks;
  const uint64_t r0 = chunk * rows_per_chunk;
  const uint64_t r1 = min(p.n, r0 + rows_per_chunk);
  const int ntiles = r1 > r0 ? static_cast<int>((r1 - r0 + kTile - 1) / kTile) : 0;
  const uint64_t q0 = static_cast<uint64_t>(qg) * 128 + w * 32;
  if (threadIdx.x < 16) sync[threadIdx.x] = 0u;

  if (wave < 4) {
    // ---- producer ------------------------------------------------------------------------
    bf16x8 ah[kOne ? 1 : K / 16], al[kOne ? 1 : K / 16];
    f16x8 aq[kOne ? K / 16 : 1];
    {
      const uint64_t qi = q0 + col;
      const uint32_t e0 = h * (K / 2);
      const float *qp = p.queries + qi * p.q_stride;
      if constexpr (kOne) {
        // the query's scale 2^t from its largest element (both halves of the wave hold it)
        float mx = 0.f;
#pragma unroll
        for (int s = 0; s < K / 16; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t e = e0 + 8 * s + j;
            mx = fmaxf(mx, fabsf((qi < p.nq && e < p.dim) ? qp[e] : 0.f));
          }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const int t = f16_exp(mx);
        if (h == 0) qexp[w * 32 + col] = t;
#pragma unroll
        for (int s = 0; s < K / 16; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t e = e0 + 8 * s + j;
            const float x = (qi < p.nq && e < p.dim) ? qp[e] : 0.f;
            aq[s][j] = static_cast<_Float16>(ldexpf(x, t));
          }
      } else {
#pragma unroll
        for (int s = 0; s < K / 16; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t e = e0 + 8 * s + j;
            const float x = (qi < p.nq && e < p.dim) ? qp[e] : 0.f;
            __bf16 hi, lo;
            split_bf16(x, hi, lo);
            ah[s][j] = hi;
            al[s][j] = lo;
          }
      }
    }
    constexpr int kVecPerRow = K / 4;
    constexpr int kVecs = kTile * kVecPerRow;
    constexpr int kPerThread = (kVecs + 255) / 256;
    auto load_tile = [&](uint64_t row0, float4 (&reg)[kPerThread]) {
#pragma unroll
      for (int v = 0; v < kPerThread; ++v) {
        const int idx = threadIdx.x + v * 256;
        reg[v] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < kVecs) {
          const uint64_t row = row0 + idx / kVecPerRow;
          if (row < r1)
            reg[v] = *reinterpret_cast<const float4 *>(p.base + row * p.row_step * p.stride + (idx % kVecPerRow) * 4);
        }
      }
    };
    auto store_tile = [&](int buf, const float4 (&reg)[kPerThread]) {
      float *t = tile + buf * kTileWords;
#pragma unroll
      for (int v = 0; v < kPerThread; ++v) {
        const int idx = threadIdx.x + v * 256;
        if (idx < kVecs && kOne) {
          _Float16 *th = reinterpret_cast<_Float16 *>(t) + (idx / kVecPerRow) * kBPitch + (idx % kVecPerRow) * 4;
          f16x4 v4;
          v4[0] = static_cast<_Float16>(ldexpf(reg[v].x, p.base_exp));
          v4[1] = static_cast<_Float16>(ldexpf(reg[v].y, p.base_exp));
          v4[2] = static_cast<_Float16>(ldexpf(reg[v].z, p.base_exp));
          v4[3] = static_cast<_Float16>(ldexpf(reg[v].w, p.base_exp));
          *reinterpret_cast<f16x4 *>(th) = v4;
        } else if (idx < kVecs) {
          __bf16 *th = reinterpret_cast<__bf16 *>(t) + (idx / kVecPerRow) * kBPitch + (idx % kVecPerRow) * 4;
          bf16x4 hv, lv;
          __bf16 hi, lo;
          split_bf16(reg[v].x, hi, lo); hv[0] = hi; lv[0] = lo;
          split_bf16(reg[v].y, hi, lo); hv[1] = hi; lv[1] = lo;
          split_bf16(reg[v].z, hi, lo); hv[2] = hi; lv[2] = lo;
          split_bf16(reg[v].w, hi, lo); hv[3] = hi; lv[3] = lo;
          *reinterpret_cast<bf16x4 *>(th) = hv;
          *reinterpret_cast<bf16x4 *>(th + kTile * kBPitch) = lv;
        }
      }
    };
    // K <= 128: row tiles are loaded two ahead (tile s + 2 while tile s is contracted, tile s + 1
    // waits in registers), so a tile's loads have a whole step plus the staging wait to land; wider
    // rows load one ahead (the registers of a second tile would spill)
    constexpr bool kDeep = K <= 128;
    float4 stage_a[kPerThread], stage_b[kDeep ? kPerThread : 1];
    load_tile(r0, stage_a);
    store_tile(0, stage_a);
    if (kDeep && ntiles > 1) load_tile(r0 + kTile, stage_a);
    __syncthreads();  // the only block-wide barrier: tile 0 staged, sync words zeroed
    const bool diag = p.merge_count != nullptr;
    uint64_t t_slot = 0, t_staged = 0;
    const uint64_t t_start = diag ? __builtin_amdgcn_s_memtime() : 0;
    int slot = 0;
    // one step: contract tile s (LDS buffer s & 1), publish it, stage tile s + 1 from `next` (kDeep:
    // while tile s + 2 loads into `ahead`); false = aborted
    auto step = [&](int s, float4 (&next)[kPerThread], float4 (&ahead)[kPerThread]) -> bool {
      const int buf = s & 1;
      if (kDeep && s + 2 < ntiles) load_tile(r0 + static_cast<uint64_t>(kTile) * (s + 2), ahead);
      if (!kDeep && s + 1 < ntiles) load_tile(r0 + static_cast<uint64_t>(kTile) * (s + 1), next);
      f32x16 c = {};
      if constexpr (kOne) {
        const _Float16 *tq = reinterpret_cast<const _Float16 *>(tile + buf * kTileWords) + col * kBPitch + h * (K / 2);
#pragma unroll
        for (int st = 0; st < K / 16; ++st)
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(aq[st], *reinterpret_cast<const f16x8 *>(tq + 8 * st), c, 0, 0, 0);
      } else {
        const __bf16 *tb = reinterpret_cast<const __bf16 *>(tile + buf * kTileWords) + col * kBPitch + h * (K / 2);
#pragma unroll
        for (int st = 0; st < K / 16; ++st) {
          const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(tb + 8 * st);
          const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(tb + kTile * kBPitch + 8 * st);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[st], bh, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[st], bl, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[st], bh, c, 0, 0, 0);
        }
      }
      // ring slot s % kD is free once the consumers have read tile s - kD
      const uint64_t tw = diag ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
      for (int c2 = 0; c2 < kCons; ++c2)
        if (s >= kD && !lds_wait_ge(&consumed[w * kCons + c2], static_cast<uint32_t>(s + 1 - kD), abort, p.spin_limit))
          return false;
      if (diag) t_slot += __builtin_amdgcn_s_memtime() - tw;
      float *out = cx + ((slot * 4 + w) * 16) * 64 + lane;
#pragma unroll
      for (int r = 0; r < 16; ++r) out[r * 64] = c[r];
      lds_publish(&published[w], static_cast<uint32_t>(s + 1));
      slot = slot + 1 == kD ? 0 : slot + 1;
      if (s + 1 < ntiles) {
        // every producer has finished this step's MFMAs on `buf` before any stages tile s + 2 into
        // it, and tile s + 1 is complete before any reads it
        store_tile(buf ^ 1, next);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) __hip_atomic_fetch_add(staged, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t tb2 = diag ? __builtin_amdgcn_s_memtime() : 0;
        if (!lds_wait_ge(staged, static_cast<uint32_t>(4 * (s + 1)), abort, p.spin_limit)) return false;
        if (diag) t_staged += __builtin_amdgcn_s_memtime() - tb2;
      }
      return true;
    };
    if constexpr (kDeep) {
      for (int s = 0; s < ntiles; s += 2) {
        if (!step(s, stage_a, stage_b)) break;
        if (s + 1 < ntiles && !step(s + 1, stage_b, stage_a)) break;
      }
    } else {
      for (int s = 0; s < ntiles; ++s)
        if (!step(s, stage_a, stage_a)) break;
    }
    if (diag && lane == 0) {  // diagnostics: producer rows after the consumers' (tools/flat_diag.py)
      unsigned long long *st =
          reinterpret_cast<unsigned long long *>(p.merge_count + 4096) + (1024 * kCons + blockIdx.x * 4 + w) * 4;
      st[0] = __builtin_amdgcn_s_memtime() - t_start;
      st[1] = t_slot;
      st[2] = t_staged;
      st[3] = 0;
    }
  } else {
    // ---- consumer(s) ---------------------------------------------------------------------
    float *bd = cx + kD * 4 * 16 * 64 + w * 32 * kB * 2;  // 32 queries x kB (each consumer its own queries)
    uint32_t *bi = reinterpret_cast<uint32_t *>(bd + 32 * kB);
    const int half = (wave - 4) / 4;
    if constexpr (kCons == 1) {
      ws_consume<kB, kD, 1, 16, 0, kOne>(p, cx, published, consumed, abort, bd, bi, w, 0, q0, chunk, ntiles, r0, r1,
                                         qexp);
    } else {
      if (half == 0)
        ws_consume<kB, kD, 2, 8, 0, kOne>(p, cx, published, consumed, abort, bd, bi, w, 0, q0, chunk, ntiles, r0, r1,
                                          qexp);
      else
        ws_consume<kB, kD, 2, 8, 8, kOne>(p, cx, published, consumed, abort, bd, bi, w, 1, q0, chunk, ntiles, r0, r1,
                                          qexp);
    }
  }
}

// --------------------------------------------------------------------------------------------
// Single-role single-pass scan over prebuilt f16 tile records (round 6, the default for narrow rows
// in the single-pass contraction).  The warp-specialised scan above converts every f32 row tile
// to f16 in each of the 8 blocks that scan it and hands each 32x32 contraction from a producer to
// a consumer through LDS flags; the tile records below are converted once per base (cached on the
// index) and laid out as the MFMA's B fragments in lane order, so a block stages a record with one
// lane-linear global->LDS DMA per 1 KB piece and every wave reads its fragments with conflict-free
// ds_read_b128.  512 threads = 8 waves (two per SIMD), each holding 32 queries as A fragments,
// 256 queries per block sharing every staged record; each wave contracts the record (K/16 MFMAs),
// forms the 1,024 approximate distances and tests them against its queries' thresholds in one
// pass, and only a record with a candidate enters the append path (LDS atomic slots in 32-entry
// buffers, folds into LDS-resident shortlists only on overflow and at the end), so the merge and
// its error bound (the single pass's) are those of the other scans.  One raw s_barrier per group
// of kG records orders the slots: after it, every wave's pieces of the group have landed (each
// wave waited for its own DMA) and every wave has finished the previous group, whose slots are
// then refilled with the next.  A prescan launch of the same kernel (kMin) over a sample of the
// records gives every query a starting threshold (flat_group_threshold_kernel).
// --------------------------------------------------------------------------------------------
// Tile record T (rows 32T .. 32T+31): K/16 pieces of 64 lanes x 8 f16 -- lane l: row 32T + (l & 31),
// k = (l >> 5) K/2 + 8 st + j, the k map of the other scans' A fragments -- each element
// f16(x 2^base_exp) exactly as the warp-specialised scan stages it; then a 256-byte tail: the 32
// rows' |b|^2 (+inf for a row past n or cleared in the validity bitmap: its approximate distance
// is +inf and fails every `d < tau`, so the scan reads no bitmap) and 32 zero words.
template <int K>
constexpr int tiles_rec() { return K / 16 * 1024 + 256; }

template <int K>
__global__ void flat_tiles_kernel(const float *base, uint64_t n, uint32_t stride, const float *norms,
                                  const uint32_t *valid, int base_exp, uint64_t n_tiles, unsigned char *out) {
  constexpr int kSteps = K / 16;
  constexpr int kPer = kSteps * 64 + 64;  // threads per record: one per 16-byte piece lane, 64 for the tail
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t T = g / kPer;
  if (T >= n_tiles) return;
  const int w = static_cast<int>(g % kPer);
  unsigned char *rec = out + T * tiles_rec<K>();
  if (w < kSteps * 64) {
    const int st = w >> 6, l = w & 63;
    const uint64_t row = T * 32 + (l & 31);
    const uint32_t e0 = (l >> 5) * (K / 2) + 8 * st;
    f16x8 v;
    if (row < n) {
      const float4 a = *reinterpret_cast<const float4 *>(base + row * stride + e0);
      const float4 b = *reinterpret_cast<const float4 *>(base + row * stride + e0 + 4);
      v[0] = static_cast<_Float16>(ldexpf(a.x, base_exp));
      v[1] = static_cast<_Float16>(ldexpf(a.y, base_exp));
      v[2] = static_cast<_Float16>(ldexpf(a.z, base_exp));
      v[3] = static_cast<_Float16>(ldexpf(a.w, base_exp));
      v[4] = static_cast<_Float16>(ldexpf(b.x, base_exp));
      v[5] = static_cast<_Float16>(ldexpf(b.y, base_exp));
      v[6] = static_cast<_Float16>(ldexpf(b.z, base_exp));
      v[7] = static_cast<_Float16>(ldexpf(b.w, base_exp));
    } else {
      for (int j = 0; j < 8; ++j) v[j] = static_cast<_Float16>(0.f);
    }
    *reinterpret_cast<f16x8 *>(rec + st * 1024 + l * 16) = v;
  } else {
    const int l = w - kSteps * 64;
    float x = 0.f;
    if (l < 32) {
      const uint64_t row = T * 32 + l;
      const bool live = row < n && (valid == nullptr || ((valid[row >> 5] >> (row & 31)) & 1u));
      x = live ? norms[row] : __builtin_inff();
    }
    reinterpret_cast<float *>(rec + kSteps * 1024)[l] = x;
  }
}

// Candidate buffers: kB = 32 entries per query in global memory (L2: p.tiles_buf, written with
// plain stores, read back past L1 by the rare folds); an append that finds its buffer full is
// retried after that buffer is folded -- exact for any data and any kB.  The shortlists (32
// entries per query) and the counts live in LDS, the thresholds in registers; the LDS the buffers
// would take holds records instead (barrier groups of up to 4 records).
constexpr int kTilesBuf = 32;
constexpr int kTilesWaveLds = 32 * (kL * 8 + 4);  // shortlists, counts
// Records per barrier group: the block meets once per kG records (the pieces of group g landed,
// group g - 1 read by every wave, its slots refilled with group g + 1), so a wave's candidate work
// on one record overlaps the other waves' contractions instead of holding all of them at a
// per-record barrier.  2 kG slots (two groups) beside the 8 waves' candidate buffers in 160 KB,
// at most ALAYA_FLAT_TILES_GROUP (diagnostics builds).
#ifndef ALAYA_FLAT_TILES_GROUP
#define ALAYA_FLAT_TILES_GROUP 4
#endif
template <int K>
constexpr int tiles_group() {
  constexpr int fit = static_cast<int>((160 * 1024 - 8 * kTilesWaveLds) / (2 * (K / 16 * 1024 + 256)));
  return fit < ALAYA_FLAT_TILES_GROUP ? fit : ALAYA_FLAT_TILES_GROUP;
}
// dynamic LDS of a launch: the record slots (the lists and counts are a static LDS object)
template <int K>
constexpr size_t tiles_lds() {
  return static_cast<size_t>(2 * tiles_group<K>()) * tiles_rec<K>();
}
template <int K>
constexpr bool tiles_fits() {
  return tiles_lds<K>() + static_cast<size_t>(8) * kTilesWaveLds <= 160 * 1024 && tiles_group<K>() >= 1;
}
static_assert(tiles_fits<32>() && tiles_fits<64>() && tiles_fits<96>() && tiles_fits<128>() && tiles_fits<160>() &&
                  tiles_fits<192>() && tiles_fits<224>(),
              "single-role f16 scan: tile groups / candidate buffers");

// this wave's DMA pieces of one record: pieces w, w + 8, ... of K/16 fragment pieces (16 B per lane)
// and the tail (4 B per lane)
template <int K>
__device__ __forceinline__ void tiles_issue(const unsigned char *src, unsigned char *slot, int wave, int lane) {
  constexpr int kSteps = K / 16;
#pragma unroll
  for (int pc = 0; pc < kSteps + 1; pc += 8) {
    const int piece = pc + wave;
    if (piece < kSteps) {
      __builtin_amdgcn_global_load_lds(static_cast<const void *>(src + piece * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void *)(slot + piece * 1024), 16, 0, 0);
    } else if (piece == kSteps) {
      __builtin_amdgcn_global_load_lds(static_cast<const void *>(src + kSteps * 1024 + lane * 4),
                                       (__attribute__((address_space(3))) void *)(slot + kSteps * 1024), 4, 0, 0);
    }
  }
}

// kMin: the prescan's form -- no shortlists: each block is one group of sampled records, and each
// query's smallest approximate distance over the group is written to cand_d[group * nq + query]
// (flat_group_threshold_kernel then takes the 32nd smallest of the groups' minima per query).
template <int K, bool kMin>
__global__ void __launch_bounds__(512) flat_scan_tiles_kernel(FlatParams p) {
  static_assert(K % 16 == 0 && K <= 224, "narrow rows");
  constexpr int kW = 8;
  constexpr int kSteps = K / 16;
  constexpr int kRec = tiles_rec<K>();
  constexpr int kB = kTilesBuf;
  constexpr int kG = tiles_group<K>();
  constexpr int kD = 2 * kG;
  constexpr bool kPre = true;  // fold before an overflowing append (kB = 32)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // uniform: scalar branches on it
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  // the lists and counts in an LDS object of their own: the compiler then knows the record DMA
  // (into smem) cannot alias them and does not drain it (vmcnt(0)) before each append's atomic
  __shared__ __attribute__((aligned(16))) unsigned char lists_lds[kMin ? 16 : 8 * kTilesWaveLds];
  unsigned char *wl = lists_lds + (kMin ? 0 : wave * kTilesWaveLds);  // this wave's lists, counts
  float *ldL = reinterpret_cast<float *>(wl);                       // 32 queries x kL
  uint32_t *liL = reinterpret_cast<uint32_t *>(ldL + 32 * kL);
  uint32_t *cntL = liL + 32 * kL;                                   // 32

  // XCD-aware: the query groups of a chunk are consecutive multiples of 8 apart (one XCD)
  const int nqg = static_cast<int>((p.nq + 32 * kW - 1) / (32 * kW));
  const int b = blockIdx.x;
  const int qg = (b / 8) % nqg;
  const int chunk = (b % 8) + 8 * (b / (8 * nqg));
  if (chunk >= p.n_chunks) return;  // the whole block
  const uint64_t per = (p.n_scan_tiles + p.n_chunks - 1) / p.n_chunks;
  const uint64_t j0 = chunk * per;
  const uint64_t j1 = min(p.n_scan_tiles, j0 + per);
  const int ntiles = j1 > j0 ? static_cast<int>(j1 - j0) : 0;
  const uint64_t q0 = static_cast<uint64_t>(qg) * (32 * kW) + wave * 32;
  // this wave's candidate buffers: 32 queries x kB (distance bits | id << 32)
  uint64_t *gb = kMin ? nullptr : p.tiles_buf + (static_cast<uint64_t>(blockIdx.x) * kW + wave) * 32 * kB;

  // A fragments of the wave's 32 queries, each scaled by its own 2^t (the ws scan's producer code).
  // The loads are unconditional (a clamped row and column, the value selected afterwards): a load
  // under a per-element condition makes the compiler wait for each one in turn, which a prescan
  // block of 16 records cannot amortise.
  f16x8 aq[kSteps];
  int t_own = 0;
  {
    const uint64_t qi = q0 + col;
    const bool qok = qi < p.nq;
    const uint32_t e0 = h * (K / 2);
    const float *qp = p.queries + (qok ? qi : 0) * p.q_stride;
    float x[kSteps * 8];
#pragma unroll
    for (int s = 0; s < kSteps; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t e = e0 + 8 * s + j;
        const float v = qp[e < p.dim ? e : p.dim - 1];
        x[8 * s + j] = (qok && e < p.dim) ? v : 0.f;
      }
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < kSteps * 8; ++i) mx = fmaxf(mx, fabsf(x[i]));
    // one scale 2^t for the wave's 32 queries, from their largest element (every scaled operand stays
    // below 2^15); flat_merge_kernel's bound takes this t from p.tiles_qexp
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    t_own = f16_exp(mx);
    if (!kMin && p.tiles_qexp && qok && h == 0) p.tiles_qexp[qi] = t_own;
#pragma unroll
    for (int s = 0; s < kSteps; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) aq[s][j] = static_cast<_Float16>(ldexpf(x[8 * s + j], t_own));
  }
  // -2 x the scale-back 2^-(s + t), one value for the wave: a = fma(m2s, C~, |b|^2)
  const float m2s = ldexpf(-2.0f, -(p.base_exp + t_own));
  TilesLists S;
  S.nonempty = 0;
  S.ld = ldL;
  S.li = liL;
  S.cnt = cntL;
  if (!kMin) {
    for (int e = lane; e < 32 * kL; e += 64) {
      ldL[e] = FLT_MAX;
      liL[e] = 0xffffffffu;
    }
    if (lane < 32) cntL[lane] = 0u;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint64_t qi = q0 + reg_query(r, h);
    S.tau[r] = qi < p.nq ? (p.tau_init ? p.tau_init[qi] : FLT_MAX) : -FLT_MAX;  // empty slots: no candidates
  }
  // the thresholds' loads complete here, not at their first use inside the loop (a vmcnt(0) there
  // would also wait out the record DMA in flight on every record)
#pragma unroll
  for (int r = 0; r < 16; ++r) asm volatile("" ::"v"(S.tau[r]));
  f32xN<16> rmin;  // kMin: running minimum of register r's query over the group
#pragma unroll
  for (int r = 0; r < 16; ++r) rmin[r] = __builtin_inff();

  const unsigned char *recs = p.tiles;
  auto rec_of = [&](int jj) { return recs + (j0 + jj) * p.tile_step * kRec; };
  // record t lives in slot (t / kG % 2) kG + t % kG: group g in one half of the ring, g + 1 in the other
  auto slot_of = [&](int t) { return smem + (((t / kG) & 1) * kG + t % kG) * kRec; };
#pragma unroll
  for (int jj = 0; jj < kG; ++jj)
    if (jj < ntiles) tiles_issue<K>(rec_of(jj), slot_of(jj), wave, lane);
  // diagnostics (p.merge_count): per-wave s_memtime totals of the wait + barrier, the contraction
  // and threshold test, and the candidate handling; p.ablate 1 skips the candidate handling, 3 the
  // contraction too (the DMA ring and the barriers alone)
  const bool diag = p.merge_count != nullptr;
  uint64_t t_wait = 0, t_mm = 0, t_cand = 0, sink = 0;
  uint32_t n_ctile = 0, n_app = 0;  // diagnostics: records with a candidate, appended candidates
  const uint64_t t_start = diag ? __builtin_amdgcn_s_memtime() : 0;
  // Software pipeline (the scan proper): record jj's MFMAs are issued between the distance forms
  // and threshold compares of record jj - 1, so the matrix pipe and the VALU overlap inside the
  // wave; record jj - 1's candidates follow.  cp/bnp/ridp: the previous record (|b|^2 = +inf
  // before the first, so it yields no candidate).
  f32x16 cp = {};
  float bnp = __builtin_inff();
  uint64_t ridp = 0;
  for (int jj = 0; jj <= ntiles; ++jj) {
    // the extra trip (jj == ntiles) only finishes the last record: its test, candidates and drain
    if (jj == ntiles && (kMin || ntiles == 0)) break;
    const uint64_t tw = diag ? __builtin_amdgcn_s_memtime() : 0;
    if (jj % kG == 0 && jj < ntiles) {
      // group start: this wave's pieces of the group have landed and its LDS reads of the previous
      // group are done; after the barrier every wave's are, and the previous group's slots take
      // the next group
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(0x70);  // vmcnt(0) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < kG; ++i)
        if (jj + kG + i < ntiles) tiles_issue<K>(rec_of(jj + kG + i), slot_of(jj + kG + i), wave, lane);
    }
    const uint64_t tm = diag ? __builtin_amdgcn_s_memtime() : 0;
    if (diag) t_wait += tm - tw;
    const unsigned char *tl = slot_of(jj < ntiles ? jj : 0);
    if (p.ablate == 3) continue;
    // every B fragment of the tile in flight at once (one LDS latency, not one per MFMA pair)
    // (the extra trip reads a settled slot and contracts it unused: no branch splits the block
    // that interleaves these MFMAs with the previous record's compares)
    f16x8 bf[kSteps];
#pragma unroll
    for (int st = 0; st < kSteps; ++st) bf[st] = *reinterpret_cast<const f16x8 *>(tl + st * 1024 + lane * 16);
    const float bn = reinterpret_cast<const float *>(tl + kSteps * 1024)[col];
    // all reads issued before the first MFMA waits on one (K <= 128; wider rows would spill)
    if constexpr (kSteps <= 8) __builtin_amdgcn_sched_barrier(0);
    f32x16 c = {};
    // the previous record's distances and compares, interleaved with this record's MFMAs
    f32xN<16> dv;
    uint64_t any = 0;
    if constexpr (!kMin) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dv[r] = fmaf(m2s, cp[r], bnp);
        any |= __builtin_amdgcn_fcmpf(dv[r], S.tau[r], 4);
      }
    }
#pragma unroll
    for (int st = 0; st < kSteps; ++st) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(aq[st], bf[st], c, 0, 0, 0);
    if constexpr (kMin) {
#pragma unroll
      for (int r = 0; r < 16; ++r) rmin[r] = fminf(rmin[r], fmaf(m2s, c[r], bn));
      continue;
    }
    const uint64_t rid = ridp;  // the previous record's rows
    cp = c;
    bnp = bn;
    ridp = ((j0 + jj) * p.tile_step) * 32 + col;
    const bool last = jj == ntiles;
    const uint64_t tc = diag ? __builtin_amdgcn_s_memtime() : 0;
    if (diag) t_mm += tc - tm;
    if (p.ablate == 1) {
      sink += any;
      continue;
    }
    // Candidates are rare once the prescan threshold is in (~10 per query and chunk): a record with
    // one builds each lane's 16-bit pass mask, and only the passing (lane, register) pairs do any
    // work -- a buffer slot from an LDS atomic add on the query's count, the (distance, id) store.
    // An append that finds its buffer full (kB = 32) is retried after the buffers it overfilled
    // are folded (against their tightened thresholds).  The last record drains every buffer.
    if (any) {
      if (diag) ++n_ctile;
      uint32_t pm = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) pm |= dv[r] < S.tau[r] ? (1u << r) : 0u;
      for (;;) {
        uint32_t ne = 0, over = 0;
        for (uint32_t m = pm; m; m &= m - 1) {
          const int r = __builtin_ctz(m);
          float d = dv[0];
#pragma unroll
          for (int r2 = 1; r2 < 16; ++r2) d = r2 == r ? dv[r2] : d;
          const int q = reg_query(r, h);
          // the slot: an LDS atomic add on the query's count, in asm -- the compiler cannot tell this
          // address from the record DMA's and would otherwise drain that DMA (vmcnt(0)) first
          uint32_t pos;
          const uint32_t one = 1u;
          const uint32_t at = static_cast<uint32_t>(
              reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint32_t *)(cntL + q)));
          asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(pos) : "v"(at), "v"(one) : "memory");
          if (pos < static_cast<uint32_t>(kB)) {
            gb[q * kB + pos] = static_cast<uint64_t>(__float_as_uint(d)) | (static_cast<uint64_t>(rid) << 32);
            ne |= 1u << r;
            if (diag) ++n_app;
          } else {
            over |= 1u << r;
          }
        }
        (void)ne;
        if (!__builtin_amdgcn_ballot_w64(over != 0u)) break;  // the common case: no buffer overflowed
        const uint32_t fold = wave_or(over);
        if (p.ablate == 4) {  // diagnostics: overflowing candidates dropped instead of folded
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if ((fold & (1u << r)) && col == 0) cntL[reg_query(r, h)] = 0u;
          break;
        }
        fold_rounds_static<kB>(p, fold, false, S, gb);
        // retry the overflowed candidates that still pass the tightened thresholds
        uint32_t retry = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          retry |= ((over & (1u << r)) && dv[r] < S.tau[r]) ? (1u << r) : 0u;
        pm = retry;
      }
    }
    if (last && p.ablate != 4) {
      // drain: every register with a buffered candidate in either half (counts from LDS)
      const int c0 = static_cast<int>(cntL[col]);  // lane l: query l & 31
      uint32_t ne = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qa = reg_query(r, 0), qb = reg_query(r, 1);
        const uint64_t m = __builtin_amdgcn_ballot_w64(c0 > 0 && (col == qa || col == qb));
        ne |= m ? (1u << r) : 0u;
      }
      S.nonempty = ne;
      if (ne) fold_rounds_static<kB>(p, ne, true, S, gb);
    }
    if (diag) t_cand += __builtin_amdgcn_s_memtime() - tc;
  }
  if constexpr (kMin) {
    // the group's minimum of each query: over the 32 rows (lanes) of its half
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = rmin[r];
      v = fminf(v, swz_f<1>(v));
      v = fminf(v, swz_f<2>(v));
      v = fminf(v, swz_f<4>(v));
      v = fminf(v, swz_f<8>(v));
      v = fminf(v, swz_f<16>(v));
      const uint64_t qi = q0 + reg_query(r, h);
      if (col == 0 && qi < p.nq) p.cand_d[static_cast<uint64_t>(chunk) * p.nq + qi] = v;
    }
    return;
  }
  if (diag && lane == 0) {  // diagnostics rows (tools/ab_flat.py --diag): total, wait, contraction, candidates
    unsigned long long *st = reinterpret_cast<unsigned long long *>(p.merge_count + 4096) + (blockIdx.x * kW + wave) * 8;
    st[0] = __builtin_amdgcn_s_memtime() - t_start;
    st[1] = t_wait;
    st[2] = t_mm;
    st[3] = t_cand + (sink == 0xffffffffffffffffull ? 1 : 0);
    st[4] = n_ctile;
    st[5] = n_app;
    st[6] = ntiles;
    st[7] = 0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const uint64_t qi = q0 + reg_query(r, h);
    if (qi < p.nq) {
      const uint64_t o = (static_cast<uint64_t>(chunk) * p.nq + qi) * kL + col;
      p.cand_d[o] = ldL[reg_query(r, h) * kL + col];
      p.cand_i[o] = liL[reg_query(r, h) * kL + col];
    }
  }
}

// --------------------------------------------------------------------------------------------
// Wide rows (stride > 224): the queries' A fragments no longer fit in registers, so K is cut into
// slabs of KS columns.  A super-chunk of TT row tiles keeps TT 32x32 accumulators; for each slab
// the wave converts its 32 queries' KS-column A fragments (prefetched one slab ahead from a
// zero-padded copy of the queries) and streams the super-chunk's (slab, tile) units through the
// double-buffered LDS tile, slab-major.  After the last slab every tile of the super-chunk goes
// through the same candidate handling (tile_candidates) as the narrow kernel, so shortlists, the
// merge and its error bound are unchanged (the bound's gamma uses the padded length).
// --------------------------------------------------------------------------------------------
template <int KS, int TT, bool kSplit>
__global__ void __launch_bounds__(256) flat_scan_wide_kernel(FlatParams p) {
  static_assert(KS % 16 == 0 && KS <= 128, "slab width: a multiple of 16, at most 128");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kPitch = KS + kPad;
  constexpr int kBPitch = KS + 8;
  constexpr int kTileWords = kSplit ? kTile * kBPitch : kTile * kPitch;
  float *tile = reinterpret_cast<float *>(smem);  // 2 x kTileWords
  const int wave = threadIdx.x >> 6;
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  float *bd = tile + 2 * kTileWords + wave * 32 * kBuf * 2;
  uint32_t *bi = reinterpret_cast<uint32_t *>(bd + 32 * kBuf);

  const int nqg = static_cast<int>((p.nq + 127) / 128);
  const int b = blockIdx.x;
  const int qg = (b / 8) % nqg;
  const int chunk = (b % 8) + 8 * (b / (8 * nqg));
  if (chunk >= p.n_chunks) return;
  const uint64_t rows_per_chunk = (p.n + p.n_chunks - 1) / p.n_chunks;
  const uint64_t r0 = chunk * rows_per_chunk;
  const uint64_t r1 = min(p.n, r0 + rows_per_chunk);
  const int nslab = static_cast<int>((p.stride + KS - 1) / KS);
  const uint32_t qwidth = static_cast<uint32_t>(nslab) * KS;  // padded query row (zeros past dim)

  const uint64_t q0 = static_cast<uint64_t>(qg) * 128 + wave * 32;
  // A prefetch: lane (col, h) holds query q0 + col, columns [s KS + h KS/2, + KS/2).  Queries past
  // nq read the last query (their shortlists are never stored).
  const uint64_t qa = min<uint64_t>(q0 + col, p.nq - 1);
  const float4 *qrow = reinterpret_cast<const float4 *>(p.queries + qa * qwidth + h * (KS / 2));
  float4 an[KS / 8];
  auto load_a = [&](int s) {
#pragma unroll
    for (int j = 0; j < KS / 8; ++j) an[j] = qrow[s * (KS / 4) + j];
  };

  Shortlists S;
  init_shortlists(p, q0, h, S);

  // cooperative unit load: 32 rows x KS columns, 256 threads, float4 each; rows past n read row
  // n-1 (dead columns of the accumulator), columns past stride are zeroed when stored
  constexpr int kVecPerRow = KS / 4;
  constexpr int kPerThread = kTile * kVecPerRow / 256;
  static_assert(kTile * kVecPerRow % 256 == 0, "whole float4s per thread");
  auto load_unit = [&](uint64_t row0, uint32_t c0, float4 (&reg)[kPerThread]) {
#pragma unroll
    for (int v = 0; v < kPerThread; ++v) {
      const int idx = threadIdx.x + v * 256;
      const uint64_t row = min<uint64_t>(row0 + idx / kVecPerRow, p.n - 1);
      const uint32_t c = min<uint32_t>(c0 + (idx % kVecPerRow) * 4, p.stride - 4);
      reg[v] = *reinterpret_cast<const float4 *>(p.base + row * p.stride + c);
    }
  };
  auto store_unit = [&](int buf, uint32_t c0, const float4 (&reg)[kPerThread]) {
    float *t = tile + buf * kTileWords;
#pragma unroll
    for (int v = 0; v < kPerThread; ++v) {
      const int idx = threadIdx.x + v * 256;
      const bool in = c0 + (idx % kVecPerRow) * 4 < p.stride;
      const float4 x = in ? reg[v] : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (kSplit) {
        __bf16 *th = reinterpret_cast<__bf16 *>(t) + (idx / kVecPerRow) * kBPitch + (idx % kVecPerRow) * 4;
        bf16x4 hv, lv;
        __bf16 hi, lo;
        split_bf16(x.x, hi, lo); hv[0] = hi; lv[0] = lo;
        split_bf16(x.y, hi, lo); hv[1] = hi; lv[1] = lo;
        split_bf16(x.z, hi, lo); hv[2] = hi; lv[2] = lo;
        split_bf16(x.w, hi, lo); hv[3] = hi; lv[3] = lo;
        *reinterpret_cast<bf16x4 *>(th) = hv;
        *reinterpret_cast<bf16x4 *>(th + kTile * kBPitch) = lv;
      } else {
        *reinterpret_cast<float4 *>(t + (idx / kVecPerRow) * kPitch + (idx % kVecPerRow) * 4) = x;
      }
    }
  };

  float4 stage[kPerThread];
  load_a(0);
  load_unit(r0, 0, stage);
  store_unit(0, 0, stage);
  __syncthreads();
  int buf = 0;
  uint64_t t_app = 0, t_fold = 0;
  for (uint64_t sup = r0; sup < r1; sup += kTile * TT) {
    const int ntiles = static_cast<int>(min<uint64_t>(TT, (r1 - sup + kTile - 1) / kTile));
    const bool last_sup = sup + kTile * TT >= r1;
    float bn[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) bn[t] = p.norms[min<uint64_t>(sup + kTile * t + col, p.n - 1)];
    f32x16 c[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) c[t] = f32x16{};
    for (int s = 0; s < nslab; ++s) {
      // this slab's A fragments (k order as in the narrow kernel: k-step st of lane (col, h) holds
      // columns s KS + h KS/2 + 8 st + j)
      bf16x8 ah[kSplit ? KS / 16 : 1], al[kSplit ? KS / 16 : 1];
      float a[kSplit ? 1 : KS / 2];
      if constexpr (kSplit) {
#pragma unroll
        for (int st = 0; st < KS / 16; ++st) {
          const float4 u = an[2 * st], w = an[2 * st + 1];
          const float v8[8] = {u.x, u.y, u.z, u.w, w.x, w.y, w.z, w.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            __bf16 hi, lo;
            split_bf16(v8[j], hi, lo);
            ah[st][j] = hi;
            al[st][j] = lo;
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < KS / 8; ++j) {
          a[4 * j] = an[j].x; a[4 * j + 1] = an[j].y; a[4 * j + 2] = an[j].z; a[4 * j + 3] = an[j].w;
        }
      }
      const bool more_a = s + 1 < nslab || !last_sup;
      if (more_a) load_a(s + 1 < nslab ? s + 1 : 0);  // next slab's fragments in flight
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        if (t < ntiles) {  // wave-uniform
          // the unit after (s, t): (s, t+1), else (s+1, 0), else the next super-chunk's (0, 0)
          uint64_t nrow = 0;
          uint32_t ncol = 0;
          bool next = true;
          if (t + 1 < ntiles) {
            nrow = sup + kTile * (t + 1);
            ncol = s * KS;
          } else if (s + 1 < nslab) {
            nrow = sup;
            ncol = (s + 1) * KS;
          } else if (!last_sup) {
            nrow = sup + kTile * TT;
            ncol = 0;
          } else {
            next = false;
          }
          if (next) load_unit(nrow, ncol, stage);
          if constexpr (kSplit) {
            const __bf16 *tb = reinterpret_cast<const __bf16 *>(tile + buf * kTileWords) + col * kBPitch + h * (KS / 2);
#pragma unroll
            for (int st = 0; st < KS / 16; ++st) {
              const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(tb + 8 * st);
              const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(tb + kTile * kBPitch + 8 * st);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[st], bh, c[t], 0, 0, 0);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[st], bl, c[t], 0, 0, 0);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[st], bh, c[t], 0, 0, 0);
            }
          } else {
            const float *tp = tile + buf * kTileWords + col * kPitch + h * (KS / 2);
#pragma unroll
            for (int k = 0; k < KS / 2; k += 4) {
              const float4 bv = *reinterpret_cast<const float4 *>(tp + k);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k], bv.x, c[t], 0, 0, 0);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k + 1], bv.y, c[t], 0, 0, 0);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k + 2], bv.z, c[t], 0, 0, 0);
              c[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[k + 3], bv.w, c[t], 0, 0, 0);
            }
          }
          if (next) {
            store_unit(buf ^ 1, ncol, stage);
            buf ^= 1;
          }
          __syncthreads();
        }
      }
    }
    // candidate handling of the super-chunk's tiles
#pragma unroll
    for (int t = 0; t < TT; ++t) {
      if (t < ntiles) {
        const uint64_t row0 = sup + kTile * t;
        const uint32_t rid = static_cast<uint32_t>(row0 + col);
        bool live = row0 + col < r1;
        if (p.valid != nullptr && live) live = (p.valid[rid >> 5] >> (rid & 31)) & 1u;
        const uint64_t live_mask = __builtin_amdgcn_ballot_w64(live);
        tile_candidates(p, c[t], bn[t], rid, live_mask, last_sup && t == ntiles - 1, S, bd, bi, t_app, t_fold);
      }
    }
  }
  store_shortlists(p, q0, chunk, S);
}

// zero-padded copy of the queries for the wide scan: dst[q][e] = src[q][e] for e < dim, else 0
__global__ void pad_queries_kernel(const float *src, uint64_t nq, uint32_t dim, uint32_t width, float *dst) {
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nq * width) return;
  const uint64_t q = i / width;
  const uint32_t e = static_cast<uint32_t>(i % width);
  dst[i] = e < dim ? src[q * dim + e] : 0.f;
}

// Exact rescoring (l2_sqr_avx2 order, 8 lanes per row) of one query's shortlist.
__device__ float exact_l2(const FlatParams &p, const float *q, uint32_t id, int m) {
  const float *row = p.base + static_cast<uint64_t>(id) * p.stride;
  const int T = static_cast<int>(p.dim >> 5);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int t = 0; t < T; ++t) {
    const float4 x = *reinterpret_cast<const float4 *>(q + 32 * t + 4 * m);
    const float4 y = *reinterpret_cast<const float4 *>(row + 32 * t + 4 * m);
    const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
    a0 = fmaf(d0, d0, a0); a1 = fmaf(d1, d1, a1); a2 = fmaf(d2, d2, a2); a3 = fmaf(d3, d3, a3);
  }
  const int nb8 = (static_cast<int>(p.dim) - 32 * T) >> 3;
  if (m < 2) {
    for (int bb = 0; bb < nb8; ++bb) {
      const float4 x = *reinterpret_cast<const float4 *>(q + 32 * T + 8 * bb + 4 * m);
      const float4 y = *reinterpret_cast<const float4 *>(row + 32 * T + 8 * bb + 4 * m);
      const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
      a0 = fmaf(d0, d0, a0); a1 = fmaf(d1, d1, a1); a2 = fmaf(d2, d2, a2); a3 = fmaf(d3, d3, a3);
    }
  }
  a0 += __shfl_xor(a0, 2); a1 += __shfl_xor(a1, 2); a2 += __shfl_xor(a2, 2); a3 += __shfl_xor(a3, 2);
  a0 += __shfl_xor(a0, 4); a1 += __shfl_xor(a1, 4); a2 += __shfl_xor(a2, 4); a3 += __shfl_xor(a3, 4);
  const float s0 = a0 + __shfl_xor(a0, 1), s1 = a1 + __shfl_xor(a1, 1);
  const float s2 = a2 + __shfl_xor(a2, 1), s3 = a3 + __shfl_xor(a3, 1);
  float res = (s0 + s1) + (s2 + s3);
  for (int e = 32 * T + 8 * nb8; e < static_cast<int>(p.dim); ++e) {
    const float d = q[e] - row[e];
    res = fmaf(d, d, res);
  }
  return res;
}

// The shortlist bound's slack on one query: rows outside the shortlist have true distance >=
// cutoff + |q|^2 - eps, and the exact k-th result is within gam of its f32 value.  The shortlist
// GEMM error is <= gam * (|q|^2 + max|b|^2 + 2|q| max|b|), gam = 2 k_acc u (u = 2^-24, conservative);
// split contraction: the f32 accumulation covers 3K terms of total magnitude <= 1.02 |q||b|
// (gam x 3.1), and the dropped terms (ql.bl and the two split residuals) add <= 3.02 * 2^-16 |q||b|
// to C, i.e. twice that to the distance; 1e-30 covers bf16 lo parts flushed as denormals.
// Single-pass f16 (operands scaled by 2^s, 2^t): every scaled operand is within 2^-11 relative plus
// 2^-14 absolute (a flushed denormal) of its f32 value, so with a_b = 2^(-14-s), a_q = 2^(-14-t)
// |C~ - C| <= (2^-10 + 2^-22) |q||b| + (1 + 2^-11) sqrt(K) (a_b |q| + a_q |b|) + K a_q a_b,
// twice that on the distance (gam x 1.01 for the slightly larger rounded operands).  A query whose
// scale-back 2^-(s+t) would leave f32's range is not provable: ok = false.
__device__ __forceinline__ float shortlist_eps(const FlatParams &p, float qn, float qmax, float &gam, bool &ok,
                                              uint64_t qi) {
  const float qnorm = sqrtf(qn);
  const float bmax = p.max_norm;
  ok = true;
  gam = 2.0f * static_cast<float>(p.k_acc) * 5.9604645e-8f * (p.split ? 3.1f : (p.single ? 1.01f : 1.0f));
  float eps = gam * (qn + bmax * bmax + 2.0f * qnorm * bmax);
  if (p.single) {
    // the scale the scan used: the single-role scan's is per wave of 32 queries (p.tiles_qexp)
    const int t = p.tiles_qexp ? p.tiles_qexp[qi] : f16_exp(qmax);
    if (abs(p.base_exp + t) > kF16MaxExp || !(qn < 3.0e38f)) ok = false;
    const float ab = ldexpf(1.0f, -14 - p.base_exp), aq = ldexpf(1.0f, -14 - t);
    const float rk = sqrtf(static_cast<float>(p.k_acc));
    const float ec = (9.7680283e-4f + 2.4e-7f) * qnorm * bmax + 1.0005f * rk * (ab * qnorm + aq * bmax) +
                     static_cast<float>(p.k_acc) * aq * ab;
    eps += 2.0f * 1.0001f * ec;
  } else if (p.split) {
    eps += 2.0f * 3.05f * 1.5258789e-5f * qnorm * bmax + 1e-30f;
  }
  return eps;
}

// One wave per query: merge the chunk shortlists (approximate distances), rescore the best kL
// exactly, sort by (exact distance, id), emit k, flag the query if the bound does not hold.
__global__ void __launch_bounds__(64) flat_merge_kernel(FlatParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *q = reinterpret_cast<float *>(smem);
  float *ld = q + p.stride;
  uint32_t *li = reinterpret_cast<uint32_t *>(ld + kL);
  float *ed = reinterpret_cast<float *>(li + kL);
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    const float *qs = p.queries + qi * p.q_stride;
    float qn = 0.f, qmax = 0.f;
    for (uint32_t e = lane; e < p.stride; e += 64) {
      const float v = e < p.dim ? qs[e] : 0.f;
      q[e] = v;
      qn = fmaf(v, v, qn);
      qmax = fmaxf(qmax, fabsf(v));
    }
    for (int off = 32; off > 0; off >>= 1) {
      qn += __shfl_xor(qn, off);
      qmax = fmaxf(qmax, __shfl_xor(qmax, off));
    }
    // chunk shortlists (each ascending): half h folds chunks h, h+2, ...; then the halves swap
    float L = FLT_MAX;
    uint32_t Li = 0xffffffffu;
    for (int c0 = 0; c0 < p.n_chunks; c0 += 2) {
      const int chunk = c0 + h;
      float cd = FLT_MAX;
      uint32_t ci = 0xffffffffu;
      if (chunk < p.n_chunks) {
        const uint64_t o = (static_cast<uint64_t>(chunk) * p.nq + qi) * kL + col;
        cd = p.cand_d[o];
        ci = p.cand_i[o];
      }
      fold32_sorted(L, Li, cd, ci, col);
    }
    fold32_sorted(L, Li, __shfl_xor(L, 32), __shfl_xor(Li, 32), col);
    if (lane < kL) {
      ld[lane] = L;
      li[lane] = Li;
    }
    wave_fence();
    // Every row outside the shortlist has approx >= cutoff: it was either displaced by 32 closer
    // entries of its chunk or rejected against a threshold that never dropped below
    // min(its chunk's final 32nd, the prescan threshold).
    const float cutoff = fminf(ld[kL - 1], p.tau_init ? p.tau_init[qi] : FLT_MAX);
    // exact distances of the shortlist (8 lanes per row, 8 rows per pass)
    const int g = lane >> 3, m = lane & 7;
    for (int base = 0; base < kL; base += 8) {
      const uint32_t id = li[base + g];
      const bool ok = id != 0xffffffffu;
      const float d = exact_l2(p, q, ok ? id : 0u, m);
      if (m == 0) ed[base + g] = ok ? d : FLT_MAX;
    }
    wave_fence();
    // rank by (exact distance, id)
    float dv = FLT_MAX;
    uint32_t iv = 0xffffffffu;
    if (lane < kL) {
      dv = ed[lane];
      iv = li[lane];
    }
    uint32_t rank = 0;
    for (int f = 0; f < kL; ++f) {
      const float df = __shfl(dv, f);
      const uint32_t tf = __shfl(iv, f);
      // equal (distance, id) pairs (only the empty entries of a short list) rank by lane
      rank += (before(df, tf, dv, iv) || (df == dv && tf == iv && f < lane)) ? 1u : 0u;
    }
    if (lane < kL && rank < p.k) {
      p.out_ids[qi * p.k + rank] = iv;
      if (p.out_dists) p.out_dists[qi * p.k + rank] = dv;
    }
    // bound (shortlist_eps): rows outside the shortlist have true distance >= cutoff + |q|^2 - eps
    float kth_d = 0.f;
    {
      const uint64_t mk = __ballot(lane < kL && rank == p.k - 1);
      kth_d = mk ? __shfl(dv, __ffsll(static_cast<unsigned long long>(mk)) - 1) : FLT_MAX;
    }
    float gam = 0.f;
    bool ok = true;
    const float eps = shortlist_eps(p, qn, qmax, gam, ok, qi);
    const bool exact = ok && (kth_d * (1.0f + gam) < cutoff + qn - eps || cutoff == FLT_MAX);
    if (lane == 0 && p.flags) p.flags[qi] = exact ? 0u : 1u;
    wave_fence();
  }
}

// --------------------------------------------------------------------------------------------
// Merge for k > kL - 8: the chunk shortlists are folded into a sorted list of M = 64R entries held
// in registers (entry e = r * 64 + lane), by bitonic networks over (distance, id).  Every row
// outside the list has approx >= cutoff = min(list[M-1], min over chunks of the chunk's 32nd, the
// prescan threshold): a row outside its chunk's shortlist is at or above that chunk's 32nd, and a
// listed row that lost the fold is at or above list[M-1].  The list is rescored exactly, sorted by
// (exact distance, id), and the bound check of flat_merge_kernel runs on the k-th result.
// --------------------------------------------------------------------------------------------
// register-held lists of the big merge (vectors, so a computed index never becomes scratch)
template <int R>
using VF = float __attribute__((ext_vector_type(R)));
template <int R>
using VU = uint32_t __attribute__((ext_vector_type(R)));

template <int R>
__device__ __forceinline__ void cmpx_regs(VF<R> &d, VU<R> &ix, int r, int r2, bool up) {
  // entries r (lower index) and r2 of the same lane; ascending when up
  const bool sw = up ? before(d[r2], ix[r2], d[r], ix[r]) : before(d[r], ix[r], d[r2], ix[r2]);
  const float td = d[r];
  const uint32_t ti = ix[r];
  d[r] = sw ? d[r2] : d[r];
  ix[r] = sw ? ix[r2] : ix[r];
  d[r2] = sw ? td : d[r2];
  ix[r2] = sw ? ti : ix[r2];
}

// one stage (block size K, distance J) of a bitonic network over the 64R entries
template <int R>
__device__ __forceinline__ void bitonic_stage(VF<R> &d, VU<R> &ix, int K, int J) {
  const int lane = lane_id();
  if (J >= 64) {
    const int rj = J >> 6;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if ((r & rj) == 0) cmpx_regs<R>(d, ix, r, r | rj, ((r * 64) & K) == 0);
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int e = r * 64 + lane;
      const bool up = (e & K) == 0;
      const bool lower = (lane & J) == 0;
      const float od = __shfl_xor(d[r], J);
      const uint32_t oi = __shfl_xor(ix[r], J);
      const bool o_first = before(od, oi, d[r], ix[r]);
      const bool take = (up == lower) ? o_first : !o_first;  // lower slot of an ascending pair keeps the min
      d[r] = take ? od : d[r];
      ix[r] = take ? oi : ix[r];
    }
  }
}

template <int R>
__device__ __forceinline__ void bitonic_sort_big(VF<R> &d, VU<R> &ix) {
#pragma unroll
  for (int K = 2; K <= 64 * R; K <<= 1)
#pragma unroll
    for (int J = K >> 1; J > 0; J >>= 1) bitonic_stage<R>(d, ix, K, J);
}

// list (ascending) absorbs a sorted batch c: pair list[e] with c[M-1-e], keep the min (a bitonic
// sequence holding the M smallest of both), then a bitonic merge
template <int R>
__device__ __forceinline__ void fold_big(VF<R> &L, VU<R> &Li, const VF<R> &c, const VU<R> &ci) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float rd = __shfl_xor(c[R - 1 - r], 63);
    const uint32_t ri = __shfl_xor(ci[R - 1 - r], 63);
    const bool take = before(rd, ri, L[r], Li[r]);
    L[r] = take ? rd : L[r];
    Li[r] = take ? ri : Li[r];
  }
#pragma unroll
  for (int J = 32 * R; J > 0; J >>= 1) bitonic_stage<R>(L, Li, 64 * R, J);
}

template <int R>
__global__ void __launch_bounds__(64) flat_merge_big_kernel(FlatParams p) {
  constexpr int M = 64 * R;
  constexpr int kPerFold = M / kL;  // chunk lists per fold
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float *q = reinterpret_cast<float *>(smem);
  uint32_t *lid = reinterpret_cast<uint32_t *>(q + max(p.stride, p.q_stride));
  float *led = reinterpret_cast<float *>(lid + M);
  const int lane = lane_id();
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    const float *qs = p.queries + qi * p.q_stride;
    float qn = 0.f, qmax = 0.f;
    for (uint32_t e = lane; e < p.stride; e += 64) {
      const float v = e < p.dim ? qs[e] : 0.f;
      q[e] = v;
      qn = fmaf(v, v, qn);
      qmax = fmaxf(qmax, fabsf(v));
    }
    for (int off = 32; off > 0; off >>= 1) {
      qn += __shfl_xor(qn, off);
      qmax = fmaxf(qmax, __shfl_xor(qmax, off));
    }
    VF<R> L;
    VU<R> Li;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      L[r] = FLT_MAX;
      Li[r] = 0xffffffffu;
    }
    float cmin = FLT_MAX;  // min over chunks of the chunk list's 32nd entry
    for (int c0 = 0; c0 < p.n_chunks; c0 += kPerFold) {
      VF<R> cd;
      VU<R> ci;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int chunk = c0 + 2 * r + (lane >> 5);
        cd[r] = FLT_MAX;
        ci[r] = 0xffffffffu;
        if (chunk < p.n_chunks) {
          const uint64_t o = (static_cast<uint64_t>(chunk) * p.nq + qi) * kL + (lane & 31);
          cd[r] = p.cand_d[o];
          ci[r] = p.cand_i[o];
          if ((lane & 31) == kL - 1) cmin = fminf(cmin, cd[r]);
        }
      }
      bitonic_sort_big<R>(cd, ci);
      fold_big<R>(L, Li, cd, ci);
    }
    for (int off = 32; off > 0; off >>= 1) cmin = fminf(cmin, __shfl_xor(cmin, off));
    const float lastv = __shfl(L[R - 1], 63);
    const float cutoff = fminf(fminf(lastv, cmin), p.tau_init ? p.tau_init[qi] : FLT_MAX);
#pragma unroll
    for (int r = 0; r < R; ++r) lid[r * 64 + lane] = Li[r];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // exact distances of the list (8 lanes per row, 8 rows per pass)
    const int g = lane >> 3, m = lane & 7;
    for (int base = 0; base < M; base += 8) {
      const uint32_t id = lid[base + g];
      const bool ok = id != 0xffffffffu;
      const float dd = exact_l2(p, q, ok ? id : 0u, m);
      if (m == 0) led[base + g] = ok ? dd : FLT_MAX;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    VF<R> E;
#pragma unroll
    for (int r = 0; r < R; ++r) E[r] = led[r * 64 + lane];
    bitonic_sort_big<R>(E, Li);  // by (exact distance, id)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t e = r * 64 + lane;
      if (e < p.k) {
        p.out_ids[qi * p.k + e] = Li[r];
        if (p.out_dists) p.out_dists[qi * p.k + e] = E[r];
      }
    }
    float kth_d = FLT_MAX;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if ((p.k - 1) / 64 == static_cast<uint32_t>(r)) kth_d = __shfl(E[r], (p.k - 1) & 63);
    float gam = 0.f;
    bool ok = true;
    const float eps = shortlist_eps(p, qn, qmax, gam, ok, qi);
    const bool exact = ok && (kth_d * (1.0f + gam) < cutoff + qn - eps || cutoff == FLT_MAX);
    if (lane == 0 && p.flags) p.flags[qi] = exact ? 0u : 1u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// Prescan threshold: one wave per query folds the chunk shortlists of a scan over a row sample and
// keeps the 32nd-best approximate distance T, written as nextafter(T, +inf): the scan's strict
// `d < tau` then admits every row with d <= T, so the sample's 32 best rows re-enter the full scan
// and the merged shortlist always holds 32 entries at or below T.
__global__ void __launch_bounds__(64) flat_threshold_kernel(FlatParams p) {
  const int lane = lane_id();
  const int h = lane >> 5, col = lane & 31;
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    float L = FLT_MAX;
    uint32_t Li = 0xffffffffu;
    for (int c0 = 0; c0 < p.n_chunks; c0 += 2) {
      const int chunk = c0 + h;
      float cd = FLT_MAX;
      uint32_t ci = 0xffffffffu;
      if (chunk < p.n_chunks) {
        const uint64_t o = (static_cast<uint64_t>(chunk) * p.nq + qi) * kL + col;
        cd = p.cand_d[o];
        ci = p.cand_i[o];
      }
      fold32_sorted(L, Li, cd, ci, col);
    }
    fold32_sorted(L, Li, __shfl_xor(L, 32), __shfl_xor(Li, 32), col);
    const float th = __shfl(L, kL - 1);
    if (lane == 0) p.tau_out[qi] = th == FLT_MAX ? FLT_MAX : nextafterf(th, FLT_MAX);
  }
}

// Prescan threshold of the single-role scan: one wave per query takes the 32nd smallest of the
// n_chunks group minima (each a distinct row's approximate distance) as T and writes
// nextafter(T, +inf): at least 32 rows then pass the full scan's strict `d < tau` and reach the
// merged shortlist, which is all flat_merge_kernel's bound needs (cutoff = min(list 32nd, T)).
// Fewer than 32 groups, or minima that are not finite: FLT_MAX (no threshold).
__global__ void __launch_bounds__(64) flat_group_threshold_kernel(FlatParams p) {
  const int lane = lane_id();
  const int G = p.n_chunks;
  for (uint64_t qi = blockIdx.x; qi < p.nq; qi += gridDim.x) {
    // rank of each minimum by (value, group): the entry of rank kL - 1 is the 32nd smallest
    float th = FLT_MAX;
    for (int g0 = 0; g0 < G; g0 += 64) {
      const int g = g0 + lane;
      const float v = g < G ? p.cand_d[static_cast<uint64_t>(g) * p.nq + qi] : FLT_MAX;
      int rank = 0;
      for (int o = 0; o < G; ++o) {
        const float w = p.cand_d[static_cast<uint64_t>(o) * p.nq + qi];
        rank += (w < v || (w == v && o < g)) ? 1 : 0;
      }
      const uint64_t m = __ballot(g < G && rank == kL - 1);
      if (m) th = __shfl(v, __ffsll(static_cast<unsigned long long>(m)) - 1);
    }
    if (lane == 0)
      p.tau_out[qi] = (G < kL || !(th < FLT_MAX)) ? FLT_MAX : nextafterf(th, FLT_MAX);
  }
}

__global__ void row_norms_kernel(const float *base, uint64_t n, uint32_t stride, float *norms) {
  const uint64_t row = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  float s = 0.f;
  for (uint32_t e = lane; e < stride; e += 64) {
    const float v = base[row * stride + e];
    s = fmaf(v, v, s);
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) norms[row] = s;
}

template <int K>
size_t scan_lds() {
  // the split tile (hi + lo bf16 rows, pitch K+8) is 4 bytes per row larger than the f32 tile
  return (2 * kTile * (K + 8) + 2 * kTile) * 4 + 4 * (32 * kBuf * 8);
}

template <int K>
constexpr int ws_buf() { return 64; }  // consumer buffers shrink to fit 160 KB
#ifndef ALAYA_FLAT_F16_RING
#define ALAYA_FLAT_F16_RING 4  // diagnostics builds: ring slots of the single-pass scan
#endif
// contraction slots per producer/consumer pair (the single pass's half-size tile leaves room for more:
// 4 slots against 3, config 2 1.301 -> 1.267 ms, profiles/r06/flat/ab_ring_*.log)
template <int K, bool kOne = false>
constexpr int ws_ring() { return kOne ? ALAYA_FLAT_F16_RING : (K <= 160 ? 3 : 2); }

// tile buffers (split: hi + lo bf16; single pass: one f16 tile), the ring, the candidate buffers, the
// sync words and the queries' scale exponents
template <int K, bool kOne = false>
constexpr size_t ws_lds() {
  return static_cast<size_t>(2 * kTile * (K + 8)) * (kOne ? 2 : 4) + ws_ring<K, kOne>() * 4 * 16 * 64 * 4 +
         4 * (32 * ws_buf<K>() * 8) + 16 * 4 + 128 * 4;
}
// every narrow-row instantiation fits one block's 160 KB of LDS, and a candidate buffer holds a
// whole tile of appends on top of the 32 a due fold leaves (tile_candidates' `need` rule)
template <int K, bool kOne = false>
constexpr bool ws_fits() {
  return ws_lds<K, kOne>() <= 160 * 1024 && ws_buf<K>() >= 2 * kTile;
}
static_assert(ws_fits<32>() && ws_fits<64>() && ws_fits<96>() && ws_fits<128>() && ws_fits<160>() &&
                  ws_fits<192>() && ws_fits<224>(),
              "warp-specialised scan: LDS ring / candidate buffers");
static_assert(ws_fits<32, true>() && ws_fits<64, true>() && ws_fits<96, true>() && ws_fits<128, true>() &&
                  ws_fits<160, true>() && ws_fits<192, true>() && ws_fits<224, true>(),
              "warp-specialised single-pass scan: LDS ring / candidate buffers");

template <int KS>
size_t wide_lds() {
  return (2 * kTile * (KS + 8)) * 4 + 4 * (32 * kBuf * 8);
}

}  // namespace

int flat_shortlist() { return kL; }

bool flat_ws_available(int ablate) { return ablate == 0 && std::getenv("ALAYA_FLAT_WS0") == nullptr; }

int flat_base_exp(float max_norm) { return f16_exp(max_norm); }

hipError_t launch_row_norms(const float *base, uint64_t n, uint32_t stride, float *norms, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(row_norms_kernel, dim3(static_cast<unsigned>((n + 3) / 4)), dim3(256), 0, s, base, n, stride, norms);
  return hipGetLastError();
}

uint32_t flat_slab(uint32_t stride) {
  if (stride <= 224) return 0;  // narrow kernel: the whole row's A fragments stay in registers
  // the slab width with the least zero padding, larger slabs first on ties
  uint32_t best = 128;
  uint64_t waste = ~0ull;
  for (uint32_t ks : {128u, 96u, 64u}) {
    const uint64_t w = (stride + ks - 1) / ks * ks - stride;
    if (w < waste) {
      waste = w;
      best = ks;
    }
  }
  return best;
}

size_t flat_scan_lds(uint32_t stride) {
  switch (flat_slab(stride)) {
    case 128: return wide_lds<128>();
    case 96: return wide_lds<96>();
    case 64: return wide_lds<64>();
    default: break;
  }
  switch (stride) {
    case 32: return scan_lds<32>();
    case 64: return scan_lds<64>();
    case 96: return scan_lds<96>();
    case 128: return scan_lds<128>();
    case 160: return scan_lds<160>();
    case 192: return scan_lds<192>();
    case 224: return scan_lds<224>();
    default: return 0;
  }
}

uint32_t flat_query_width(uint32_t stride) {
  const uint32_t ks = flat_slab(stride);
  return ks ? (stride + ks - 1) / ks * ks : 0;
}

hipError_t launch_pad_queries(const float *src, uint64_t nq, uint32_t dim, uint32_t width, float *dst,
                              hipStream_t s) {
  const uint64_t total = nq * width;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(pad_queries_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, s, src, nq,
                     dim, width, dst);
  return hipGetLastError();
}

size_t flat_tiles_bytes(uint32_t stride, uint64_t n) {
  if (stride == 0 || stride > 224 || stride % 32 != 0) return 0;
  return static_cast<size_t>((n + 31) / 32) * (stride / 16 * 1024 + 256);
}

int flat_tiles_queries() { return 256; }
int flat_tiles_buf() { return kTilesBuf; }

hipError_t launch_flat_tiles(const float *base, uint64_t n, uint32_t stride, const float *norms, const uint32_t *valid,
                             int base_exp, unsigned char *out, hipStream_t s) {
  const uint64_t n_tiles = (n + 31) / 32;
  if (n_tiles == 0) return hipSuccess;
  const uint64_t threads = n_tiles * (stride / 16 * 64 + 64);
  const dim3 grid(static_cast<unsigned>((threads + 255) / 256));
  switch (stride) {
#define ALAYA_TILES(K)                                                                                        \
  case K:                                                                                                     \
    hipLaunchKernelGGL(flat_tiles_kernel<K>, grid, dim3(256), 0, s, base, n, stride, norms, valid, base_exp, \
                       n_tiles, out);                                                                         \
    break;
    ALAYA_TILES(32) ALAYA_TILES(64) ALAYA_TILES(96) ALAYA_TILES(128) ALAYA_TILES(160) ALAYA_TILES(192)
    ALAYA_TILES(224)
#undef ALAYA_TILES
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_flat_scan(const FlatParams &p, int blocks, hipStream_t s) {
  if (p.tiles != nullptr) {
    // p.tau_out set: the prescan's group minima (ring only in LDS, no candidate buffers)
    switch (p.stride) {
#define ALAYA_TILES(K)                                                                                          \
  case K:                                                                                                       \
    if (p.tau_out)                                                                                              \
      hipLaunchKernelGGL((flat_scan_tiles_kernel<K, true>), dim3(blocks), dim3(512),                           \
                         (static_cast<size_t>(2 * tiles_group<K>()) * tiles_rec<K>()), s, p);                 \
    else                                                                                                        \
      hipLaunchKernelGGL((flat_scan_tiles_kernel<K, false>), dim3(blocks), dim3(512), (tiles_lds<K>()), s, p); \
    break;
      ALAYA_TILES(32) ALAYA_TILES(64) ALAYA_TILES(96) ALAYA_TILES(128) ALAYA_TILES(160) ALAYA_TILES(192)
      ALAYA_TILES(224)
#undef ALAYA_TILES
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const size_t lds = flat_scan_lds(p.stride);
  if (lds == 0) return hipErrorInvalidValue;
  constexpr int TT = kWideTiles;
  switch (flat_slab(p.stride)) {
#define ALAYA_WIDE(KS)                                                                                  \
  case KS:                                                                                              \
    if (p.split)                                                                                        \
      hipLaunchKernelGGL((flat_scan_wide_kernel<KS, TT, true>), dim3(blocks), dim3(256), lds, s, p);    \
    else                                                                                                \
      hipLaunchKernelGGL((flat_scan_wide_kernel<KS, TT, false>), dim3(blocks), dim3(256), lds, s, p);   \
    return hipGetLastError();
    ALAYA_WIDE(128) ALAYA_WIDE(96) ALAYA_WIDE(64)
#undef ALAYA_WIDE
    default: break;
  }
  // the warp-specialised kernel for the single-pass f16 and the split contraction; the single-role
  // kernel for the f32 contraction and the diagnostics (ablation, per-phase stamps)
  const bool ws = (p.split || p.single) && flat_ws_available(p.ablate);
  // two consumer waves per producer (default): config 2 566k -> 617k QPS (scan 1.76 -> 1.61 ms,
  // profiles/r04/flat/); ALAYA_FLAT_WS2=0 keeps one
  const char *ws2 = std::getenv("ALAYA_FLAT_WS2");
  const bool two = !(ws2 && ws2[0] == '0');
#define ALAYA_FLAT(K)                                                                          \
  case K:                                                                                      \
    if (ws && p.single && two)                                                                 \
      hipLaunchKernelGGL((flat_scan_ws_kernel<K, ws_buf<K>(), ws_ring<K, true>(), 2, true>), dim3(blocks), dim3(768), \
                         (ws_lds<K, true>()), s, p);                                             \
    else if (ws && p.single)                                                                   \
      hipLaunchKernelGGL((flat_scan_ws_kernel<K, ws_buf<K>(), ws_ring<K, true>(), 1, true>), dim3(blocks), dim3(512), \
                         (ws_lds<K, true>()), s, p);                                             \
    else if (ws && two)                                                                        \
      hipLaunchKernelGGL((flat_scan_ws_kernel<K, ws_buf<K>(), ws_ring<K>(), 2, false>), dim3(blocks), dim3(768), \
                         ws_lds<K>(), s, p);                                                   \
    else if (ws)                                                                               \
      hipLaunchKernelGGL((flat_scan_ws_kernel<K, ws_buf<K>(), ws_ring<K>(), 1, false>), dim3(blocks), dim3(512), \
                         ws_lds<K>(), s, p);                                                   \
    else if (p.split)                                                                          \
      hipLaunchKernelGGL((flat_scan_kernel<K, true>), dim3(blocks), dim3(256), lds, s, p);     \
    else                                                                                       \
      hipLaunchKernelGGL((flat_scan_kernel<K, false>), dim3(blocks), dim3(256), lds, s, p);    \
    break;
  switch (p.stride) {
    ALAYA_FLAT(32) ALAYA_FLAT(64) ALAYA_FLAT(96) ALAYA_FLAT(128) ALAYA_FLAT(160) ALAYA_FLAT(192)
    ALAYA_FLAT(224)
    default: return hipErrorInvalidValue;
  }
#undef ALAYA_FLAT
  return hipGetLastError();
}

hipError_t launch_flat_threshold(const FlatParams &p, hipStream_t s) {
  const int grid = static_cast<int>(p.nq < 4096 ? p.nq : 4096);
  if (p.tiles != nullptr)
    hipLaunchKernelGGL(flat_group_threshold_kernel, dim3(grid), dim3(64), 0, s, p);
  else
    hipLaunchKernelGGL(flat_threshold_kernel, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}

int flat_max_k() { return 4 * 64 - 32; }

hipError_t launch_flat_merge(const FlatParams &p, hipStream_t s) {
  const int grid = static_cast<int>(p.nq < 4096 ? p.nq : 4096);
  if (p.k <= static_cast<uint32_t>(kL - 8)) {
    const size_t lds = (static_cast<size_t>(std::max(p.stride, p.q_stride)) + 3 * kL + 2 * kBuf) * 4 + 64;
    hipLaunchKernelGGL(flat_merge_kernel, dim3(grid), dim3(64), lds, s, p);
  } else if (p.k <= 128 - 28) {
    const size_t lds = (static_cast<size_t>(std::max(p.stride, p.q_stride)) + 2 * 128) * 4 + 64;
    hipLaunchKernelGGL(flat_merge_big_kernel<2>, dim3(grid), dim3(64), lds, s, p);
  } else if (p.k <= static_cast<uint32_t>(flat_max_k())) {
    const size_t lds = (static_cast<size_t>(std::max(p.stride, p.q_stride)) + 2 * 256) * 4 + 64;
    hipLaunchKernelGGL(flat_merge_big_kernel<4>, dim3(grid), dim3(64), lds, s, p);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace alaya_amd
