// C-ABI implementation (include/alaya_hip.h): device-resident index state, uploads, launches.
#include "../../include/alaya_hip.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "build_kernels.h"
#include "graph_update.h"
#include "hnsw_build.h"
#include "flat_kernels.h"
#include <cstdlib>
#include "search_kernels.h"

using alaya_amd::HostGraph;
using alaya_amd::SearchParams;

struct alaya_graph {
  HostGraph g;
};

namespace {

thread_local std::string g_last_error;

struct ArgError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct DeviceError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename F>
int guarded(F &&f) {
  try {
    f();
    return ALAYA_OK;
  } catch (const ArgError &e) {
    g_last_error = e.what();
    return ALAYA_ERR_ARG;
  } catch (const DeviceError &e) {
    g_last_error = e.what();
    return ALAYA_ERR_DEVICE;
  } catch (const std::exception &e) {
    g_last_error = e.what();
    return ALAYA_ERR_RUNTIME;
  }
}

// Grow-only device buffer.
struct DevBuf {
  void *ptr = nullptr;
  size_t bytes = 0;
  void reserve(size_t n) {
    if (n <= bytes) return;
    release();
    hip_check(hipMalloc(&ptr, std::max<size_t>(n, 256)), "hipMalloc");
    bytes = std::max<size_t>(n, 256);
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
  template <typename T>
  T *as() const {
    return static_cast<T *>(ptr);
  }
  ~DevBuf() { release(); }
};

uint32_t round_up32(uint32_t d) { return (d + 31u) / 32u * 32u; }

uint32_t ceil_log2(uint64_t v) {
  uint32_t l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}

}  // namespace

struct alaya_index {
  int device = 0;
  std::mutex mu;
  // base
  uint64_t n = 0;
  uint32_t dim = 0, stride = 0;
  int metric = ALAYA_METRIC_L2;
  bool generic = false;  // ALAYA_DIST_GENERIC: non-float DataType rows, generic distance order
  DevBuf base, valid;
  bool has_valid = false;
  // graph
  bool has_graph = false;
  uint32_t R = 0, upper_R = 0, ep = 0, n_eps = 0;
  bool has_overlay = false, dedup = false;
  DevBuf l0, levels, upper_off, upper_edges, eps;
  uint64_t graph_n = 0;
  // SQ8 search space
  bool has_sq8 = false;
  int sq8_order = 2;
  uint32_t code_stride = 0;
  DevBuf codes, sq_min, sq_max, rr_q_buf, sq_ids, sq_d;
  // flat path
  DevBuf norms, cand_d, cand_i, flat_tau, flag_buf, iota, flat_q;
  int flat_contraction = -1;  // the last flat search's: 0 = f32, 1 = bf16 hi/lo split, 2 = single-pass f16
  bool norms_ready = false;
  // single-role f16 flat scan: the base's tile records (alaya_amd::launch_flat_tiles), built at the
  // first flat search after any change to the rows, their count or the validity bitmap
  DevBuf flat_tiles, tiles_cand, tiles_qexp;  // the records; the scan's candidate buffers, query scales
  bool tiles_ready = false;
  int tiles_exp = 0;
  float max_norm = 0.f;
  // scratch
  DevBuf work, overflow, dirty, stab, q_buf, id_buf, dist_buf, cnt_buf, dlist_buf, dout_buf;
  size_t overflow_clean = 0;  // leading bytes of `overflow` known to be zero (kernels leave it clean)
  size_t stab_clean = 0;      // the same for the spill tables
  uint32_t hash_log2_override = 0;
  int helpers_mode = -1;          // distance helpers: -1 automatic, 0 off, 1 on (alaya_index_set_helpers)
  DevBuf help_stats;              // per searcher of the last helper launch: (memo distances, memo expansions)
  uint64_t help_stats_slots = 0;
  uint32_t last_grid = 0, last_waves = 0;  // the last search launch's workgroups and waves per workgroup
  int visited_mode_override = 0;  // 0 auto, 1 compact 16-bit slots, 2 wide 32-bit slots,
                                  // 3 compact with probes capped at 2 (exercises the probe spill)
  int num_cus = 0;
  // online updates (alaya_index_enable_updates): host mirror + JobContext, device capacity
  uint64_t capacity = 0;
  std::unique_ptr<alaya_amd::HostGraph> upd_graph;
  std::unique_ptr<alaya_amd::RowMirror> upd_rows;
  std::unique_ptr<alaya_amd::UpdateContext> upd_ctx;
  hipStream_t stream = nullptr;
  // Per-index scratch (work counter, visited spill area, flat candidates, SQ8 id buffer) is shared
  // by every launch; `scratch_ev` marks the end of the last launch that used it, on
  // `scratch_stream`.  A launch on another stream waits for it first (scratch_acquire), and calls
  // that replace or free device buffers drain it (scratch_drain).
  hipEvent_t scratch_ev = nullptr;
  hipStream_t scratch_stream = nullptr;
  bool scratch_used = false;
  uint64_t device_bytes() const {
    return base.bytes + valid.bytes + l0.bytes + levels.bytes + upper_off.bytes +
           upper_edges.bytes + eps.bytes + overflow.bytes + dirty.bytes + stab.bytes + codes.bytes + sq_min.bytes +
           sq_max.bytes;
  }
};

namespace {

void set_device(const alaya_index *ix) { hip_check(hipSetDevice(ix->device), "hipSetDevice"); }

// Order this call's launches on `s` after every earlier launch that used the index's scratch.
void scratch_acquire(alaya_index *ix, hipStream_t s) {
  if (ix->scratch_used && ix->scratch_stream != s)
    hip_check(hipStreamWaitEvent(s, ix->scratch_ev, 0), "hipStreamWaitEvent");
}
// Mark the end of this call's launches on `s`.
void scratch_release(alaya_index *ix, hipStream_t s) {
  hip_check(hipEventRecord(ix->scratch_ev, s), "hipEventRecord");
  ix->scratch_stream = s;
  ix->scratch_used = true;
}
// The visited spill areas (bitsets, spill tables) are zeroed once and then kept clean by every
// query that finishes.  A launch or sync that reports an error may have left a query half done, so
// the next launch zeroes them again.
void scratch_suspect(alaya_index *ix) {
  ix->overflow_clean = 0;
  ix->stab_clean = 0;
}
// Wait (host side) until no launch can still read or write the index's device buffers.
void scratch_drain(alaya_index *ix) {
  if (!ix->scratch_used) return;
  const hipError_t e = hipEventSynchronize(ix->scratch_ev);
  if (e != hipSuccess) scratch_suspect(ix);
  hip_check(e, "hipEventSynchronize");
}
// guarded() for the entry points that launch searches on the index's scratch: a device error marks
// the spill areas for re-zeroing.  This covers errors the call itself sees (launch failures, and the
// synchronous entry points' syncs, scratch_drain).  A stream-async *_device call returns before its
// kernel ends; a fault surfacing later (at a torch sync) is not seen here.  HIP errors from a device
// fault are sticky -- the context is unusable and every later call of this index throws -- so no
// later launch runs on tables a half-finished query left dirty.
template <typename F>
int guarded_scratch(alaya_index *ix, F &&f) {
  return guarded([&] {
    try {
      f();
    } catch (const DeviceError &) {
      if (ix) scratch_suspect(ix);
      throw;
    }
  });
}

SearchParams base_params(alaya_index *ix) {
  SearchParams p{};
  p.base = ix->base.as<float>();
  p.n = ix->n;
  p.dim = ix->dim;
  p.stride = ix->stride;
  p.valid = ix->has_valid ? ix->valid.as<uint32_t>() : nullptr;
  p.ip = ix->metric != ALAYA_METRIC_L2;
  p.generic = ix->generic;
  return p;
}

constexpr size_t kLdsPerCu = 160 * 1024;
constexpr uint32_t kDirtyCap = 16384;  // per-slot dirty-word list (64 KB): words a spilled query set

// Spill table size (log2 entries per slot) for an AVX-512-order SQ8 search, 0 = the bitset is the
// second level.
// ~32 ef entries (config 5, ef 340: 2^14 = 32 KB per slot for ~2.7k visited ids, load 0.16, so a
// full bucket of 8 -- the bitset fallback -- is rare); at least 2^(L - 12) so an entry (1 + the
// hash's low L - (s - 3) bits) fits 16 bits; at most 2^16 (128 KB per slot; ids wider than 28 bits
// keep the bitset).  ALAYA_SPILL_TABLE=0 keeps the bitset, a value 6..16 forces the size (tests: tiny
// tables fill their buckets and exercise the bitset fallback).
uint32_t spill_table_log2(int sq8_order, uint32_t L, uint32_t ef) {
  // f32 kernels keep the LDS first level and the bitset (their tables rarely spill; on the spill
  // table SIFT ran 23 % slower); so do the AVX2-order SQ8 kernels (hosts without AVX-512), whose
  // SGPR budget the table's state would overrun (65-116 restores per expansion)
  if (sq8_order != 2) return 0;
  uint32_t s = std::max<uint32_t>({6u, ceil_log2(32ull * ef), L > 12 ? L - 12 : 0u});
  if (const char *e = std::getenv("ALAYA_SPILL_TABLE")) {
    const uint32_t v = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
    if (v == 0) return 0;
    if (v >= 6 && v <= 16) s = v;
  }
  s = std::min<uint32_t>(s, L + 3);  // buckets <= 2^L: the bucket index is the hash's top bits
  if (s > 16 || s < 6 || L - (s - 3) > 15) return 0;
  return s;
}

// The visited set's second level for `slots` persistent searchers over ix->n rows: one clean N-bit
// bitset per slot (zeroed once when allocated; every query leaves it clean) and a dirty-word list,
// plus (SQ8 searches, spill_table_log2) one clean spill table per slot.
void prepare_spill(alaya_index *ix, SearchParams &p, uint64_t slots, hipStream_t stream) {
  const uint64_t words = (ix->n + 31) / 32;
  const size_t bytes = static_cast<size_t>(std::max<uint64_t>(slots, 1)) * words * 4;
  if (bytes > ix->overflow.bytes) {
    ix->overflow.reserve(bytes);
    ix->overflow_clean = 0;
  }
  if (ix->overflow_clean < ix->overflow.bytes) {
    hip_check(hipMemsetAsync(ix->overflow.ptr, 0, ix->overflow.bytes, stream), "hipMemsetAsync");
    ix->overflow_clean = ix->overflow.bytes;
  }
  uint32_t cap = kDirtyCap;
  if (const char *e = std::getenv("ALAYA_DIRTY_CAP")) cap = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));  // tests
  ix->dirty.reserve(static_cast<size_t>(std::max<uint64_t>(slots, 1)) * std::max<uint32_t>(cap, 1) * 4);
  p.overflow_bits = ix->overflow.as<uint32_t>();
  p.dirty_words = ix->dirty.as<uint32_t>();
  p.dirty_cap = cap;
  p.spill_table = nullptr;
  p.stab_rbits = 0;
  p.spill_flags = 0;
  if (const char *e = std::getenv("ALAYA_SPILL_FLAGS")) p.spill_flags = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  if (const uint32_t st = p.stab_log2) {
    const size_t tbytes = static_cast<size_t>(std::max<uint64_t>(slots, 1)) * (2ull << st);
    if (tbytes > ix->stab.bytes) {
      ix->stab.reserve(tbytes);
      ix->stab_clean = 0;
    }
    if (ix->stab_clean < ix->stab.bytes) {
      hip_check(hipMemsetAsync(ix->stab.ptr, 0, ix->stab.bytes, stream), "hipMemsetAsync");
      ix->stab_clean = ix->stab.bytes;
    }
    const uint32_t rbits = p.vis_lbits - (st - 3);
    p.spill_table = ix->stab.as<uint16_t>();
    p.stab_log2 = st;
    p.stab_rbits = rbits;
  }
}

// Waves per search workgroup: SQ8 searchers share the quantizer's per-dimension scale and min
// (search_shared_lds_bytes) across 4 waves, one per SIMD; f32 searchers have nothing to share.
// ALAYA_SEARCH_WAVES overrides (1, 2 or 4; diagnostics).
int search_waves(const SearchParams &p) {
  if (const char *e = std::getenv("ALAYA_SEARCH_WAVES")) {
    const int w = std::atoi(e);
    if (w == 1 || w == 2 || w == 4) return w;
  }
  return p.sq8_order != 0 ? 4 : 1;
}

// Size the LDS visited table for residency: the batch wants ceil(nq / CUs) resident queries
// (waves) per CU; the register file caps that.  With more queries than resident slots the launch
// runs as many waves as the registers admit -- a spill to the global second level is one atomicOr
// per visit and no clearing beyond the words set (visit_end), so residency beats table size
// (config 5, 10k queries: 4 -> 8 -> 12 waves per CU with 16 / 8 / 4 KB tables took 20.3 / 13.3 /
// 11.1 ms; profiles/r03/sweeps) -- and the table takes what LDS is left per wave at that count
// (workgroups of W waves plus the shared region), never below 256 slots, never more than ~2x the
// expected visited count (48 ef).  Layout: compact 16-bit slots (twice the entries per byte)
// whenever the ids' hash remainder fits (log2 n - log2 slots <= 11), else 32-bit id slots.
// Returns log2 slots; sets p.vis_*.
constexpr uint32_t kMaxCompactRbits = 11;
// At most 4 searchers per SIMD: a 5th wave (the 96-VGPR d = 128 L2 kernel admits 5) halves every
// table and costs more in probes than it hides -- SIFT 1M, 10k queries, ef 70: 16 waves per CU with
// 4096-slot tables 1.198 ms, 20 with 2048-slot tables 1.513 ms (profiles/r03/sift_c3/residency_sweep_tree.log);
// config 5 measured 12 and 16 per CU equal.
constexpr uint64_t kMaxSearchWavesPerCu = 16;
uint64_t max_search_waves_per_cu() {
  if (const char *e = std::getenv("ALAYA_MAX_WAVES_PER_CU"))  // diagnostics (tools/shape_sweep.py)
    return std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
  return kMaxSearchWavesPerCu;
}

// Distance helpers (search kernel kMode 4, search_has_helpers): with helpers every search runs 4-wave
// workgroups, and a batch smaller than the resident searchers still fills the CUs, so each workgroup
// has idle waves to help from the start.  Automatic policy, from the measurements in DESIGN.md
// (round 5, "distance helpers"): on for the SQ8 kernels (config 5: 1k queries 3.75 -> 3.54 ms, 10k
// 9.60 -> 9.53 ms); for the small-row f32 kernels only when the batch outnumbers the resident
// searchers, i.e. for its tail (SIFT-shaped 10k 1.192 -> 1.138 ms; at 1k the helper layout costs more
// than it saves: 0.536 -> 0.583 ms).  alaya_index_set_helpers and ALAYA_HELPERS=0/1 override it.
bool helpers_requested(const alaya_index *ix, const SearchParams &p, uint64_t nq, uint64_t cus) {
  if (const char *e = std::getenv("ALAYA_HELPERS")) return std::atoi(e) != 0;  // A/B override
  if (ix->helpers_mode >= 0) return ix->helpers_mode > 0;
  if (std::getenv("ALAYA_SEARCH_WAVES")) return false;  // a forced workgroup shape (diagnostics, tests)
  if (p.sq8_order == 2) return true;
  return nq > max_search_waves_per_cu() * cus;
}

uint32_t size_visited(alaya_index *ix, SearchParams &p, uint64_t nq, uint32_t ef, int W = 1) {
  const uint32_t lbits = std::max<uint32_t>(1, ceil_log2(std::max<uint64_t>(ix->n, 2)));
  const int mode = ix->visited_mode_override;  // 0 auto, 1 compact, 2 wide, 3 compact + short probes
  auto set_mode = [&](uint32_t l, bool compact) {
    p.vis_lbits = lbits;
    p.vis_rbits = compact ? (lbits > l ? lbits - l : 0u) : alaya_amd::kVisWide;
    p.vis_max_disp = compact ? (0xffffu >> p.vis_rbits) - 1u : 0u;
    if (compact && mode == 3) p.vis_max_disp = std::min<uint32_t>(p.vis_max_disp, 2u);
    p.vis_limit = 0u;
    if (const char *e = std::getenv("ALAYA_VIS_LIMIT_PCT")) {  // diagnostics: spill threshold in % of slots
      const uint64_t slots = 1ull << l;
      const uint64_t lim = slots * std::min<uint64_t>(100, std::strtoull(e, nullptr, 10)) / 100;
      // exact at any threshold up to slots - 64: one visit inserts at most 64 ids, and a compact
      // probe past max_disp spills by itself
      p.vis_limit = static_cast<uint32_t>(std::max<uint64_t>(64, std::min<uint64_t>(lim, slots - 64)));
    }
    if (const char *e = std::getenv("ALAYA_VIS_LIMIT")) {  // diagnostics: spill threshold in entries (1 = at the
      const uint64_t lim = std::strtoull(e, nullptr, 10);  // first expansion); exact up to slots - 64
      if (lim > 0) p.vis_limit = static_cast<uint32_t>(std::min<uint64_t>(lim, (1ull << l) - 64));
    }
    return l;
  };
  auto fits_compact = [&](uint32_t l) { return (lbits > l ? lbits - l : 0u) <= kMaxCompactRbits; };
  if (ix->hash_log2_override) {
    const uint32_t l = ix->hash_log2_override;
    const bool compact = mode == 1 || mode == 3 || (mode == 0 && fits_compact(l));
    if (compact && !fits_compact(l)) throw ArgError("compact visited table cannot encode ids of this index");
    return set_mode(l, compact);
  }
  if (p.stab_log2 != 0 && mode != 1 && mode != 3) {
    // The spill table is the second level: a query spills at its first expansion into a 128-slot
    // first level, then every visit is prefetched bucket reads (config 5: 10k queries 9.30 ->
    // 9.20 ms, 1k queries 3.89 -> 3.69 ms against first levels sized for LDS;
    // profiles/r04/spill_table/c5_first_level_size_threshold.log).  LDS then bounds nothing.
    return set_mode(7, false);
  }
  const size_t shared = alaya_amd::search_shared_lds_bytes(ix->stride, p.sq8_order != 0) +
                        (p.help ? alaya_amd::kHelpBoardBytes : 0);
  const size_t wave_fixed = alaya_amd::search_wave_lds_bytes(ix->stride, ef, 0, false, p.sq8_order) - 4;
  // the register-bound residency, probed with a 4 KB table.  The 1 KB probe applies only to the
  // forced compact modes (1, 3) with a spill table: every other mode with a spill table returned
  // set_mode(7) above.
  const bool stab = p.stab_log2 != 0;  // set by do_search (spill_table_log2)
  int vgpr_blocks = 0;
  hip_check(alaya_amd::search_occupancy(p, W, shared + W * (wave_fixed + (stab ? 1024 : 4096)), &vgpr_blocks),
            "occupancy");
  const uint64_t vgpr_waves = static_cast<uint64_t>(std::max(1, vgpr_blocks)) * W;
  const uint64_t max_waves = std::max<uint64_t>(W, max_search_waves_per_cu());
  // with helpers a small batch still fills the CUs (the waves without a query help)
  const uint64_t want = p.help ? max_waves : (nq + ix->num_cus - 1) / std::max(1, ix->num_cus);
  uint64_t waves = std::max<uint64_t>(1, std::min<uint64_t>({vgpr_waves, want, max_waves}));
  const uint32_t cap = ceil_log2(48ull * ef);
  // table bytes per wave when `w` waves share a CU in workgroups of W
  auto table_budget = [&](uint64_t w) -> size_t {
    const uint64_t blocks = std::max<uint64_t>(1, w / W);
    const size_t per_block = kLdsPerCu / blocks;
    if (per_block <= shared) return 0;
    const size_t per_wave = (per_block - shared) / W;
    return per_wave > wave_fixed ? per_wave - wave_fixed : 0;
  };
  const size_t min_table = (mode == 2 || !fits_compact(9)) ? (4u << 8) : (2u << 9);  // 256 wide / 512 compact slots
  while (waves > static_cast<uint64_t>(W) && table_budget(waves) < min_table) waves -= W;
  const size_t budget = table_budget(waves);
  auto pick = [&](size_t slot_bytes, uint32_t lmax) {
    uint32_t l = 8;
    while (l < lmax && (slot_bytes << (l + 1)) <= budget) ++l;
    return std::max<uint32_t>(8, std::min<uint32_t>(l, cap));
  };
  if (mode == 0) {
    // a 32-bit id table of >= 32 ef slots (load <= ~0.3 at the usual 10-24 visited ids per ef)
    // costs one LDS atomic per probe instead of a load and a compare-and-swap: where it fits (the
    // 1k-query SIFT shape) it is 11 % faster; a compact table stays the choice when LDS is short
    const uint32_t wl = std::max<uint32_t>(10, ceil_log2(32ull * ef));
    if (wl <= 15 && (static_cast<size_t>(4) << wl) <= budget) return set_mode(wl, false);
  }
  if (mode != 2) {
    const uint32_t l = pick(2, 16);
    if (fits_compact(l)) return set_mode(l, true);
    if (mode == 1 || mode == 3) throw ArgError("compact visited table cannot encode ids of this index");
  }
  return set_mode(pick(4, 15), false);
}

// CUs a launch on `s` may use: all of the device's, unless the stream carries a CU mask
// (alaya_stream_create_reserving: the persistent grid is sized to the CUs left to it, so none of its
// workgroups waits for a CU that another stream's kernels -- the shard exchange's -- keep).
int stream_cus(const alaya_index *ix, hipStream_t s) {
  if (s == nullptr) return ix->num_cus;
  uint32_t mask[32] = {};
  const uint32_t words = static_cast<uint32_t>((ix->num_cus + 31) / 32);
  if (words > 32 || hipExtStreamGetCUMask(s, words, mask) != hipSuccess) {
    (void)hipGetLastError();
    return ix->num_cus;
  }
  int c = 0;
  for (uint32_t w = 0; w < words; ++w) c += __builtin_popcount(mask[w]);
  return c > 0 && c <= ix->num_cus ? c : ix->num_cus;
}

void do_search(alaya_index *ix, const float *d_q, uint64_t nq, uint32_t k, uint32_t ef,
               uint32_t *d_ids, float *d_dists, uint32_t *d_cnt, hipStream_t stream,
               uint64_t *d_stamps = nullptr, bool sq8 = false, uint32_t fill_id = 0) {
  if (!ix->base.ptr) throw ArgError("index has no base vectors");
  if (!ix->has_graph) throw ArgError("index has no graph");
  if (ef == 0) throw ArgError("ef must be >= 1");
  if (k == 0 || nq == 0) return;
  if (ix->graph_n > ix->n) throw ArgError("graph has more nodes than base vectors");
  SearchParams p = base_params(ix);
  p.l0 = ix->l0.as<uint32_t>();
  p.R = ix->R;
  p.dedup_edges = ix->dedup;
  p.levels = ix->has_overlay ? ix->levels.as<uint32_t>() : nullptr;
  p.upper_off = ix->upper_off.as<uint64_t>();
  p.upper_edges = ix->upper_edges.as<uint32_t>();
  p.upper_R = ix->upper_R;
  p.ep = ix->ep;
  p.eps = ix->eps.as<uint32_t>();
  p.n_eps = ix->n_eps;
  p.queries = d_q;
  p.nq = nq;
  p.q_stride = ix->dim;
  p.k = k;
  p.ef = ef;
  p.out_ids = d_ids;
  p.out_dists = d_dists;
  p.out_counters = d_cnt;
  p.stamps = d_stamps;
  p.fill_id = fill_id;
  if (sq8) {
    if (!ix->has_sq8) throw ArgError("index has no SQ8 codes");
    p.sq8_order = ix->sq8_order;
    p.codes = ix->codes.as<uint8_t>();
    p.code_stride = ix->code_stride;
    p.sq_min = ix->sq_min.as<float>();
    p.sq_max = ix->sq_max.as<float>();
  }
  // diagnostics flags (read again by prepare_spill); bit 8 selects the prefetch-check kernel, so it
  // must be known before the occupancy probes
  if (const char *e = std::getenv("ALAYA_SPILL_FLAGS")) p.spill_flags = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  // the visited second level: spill table or bitset
  p.stab_log2 = spill_table_log2(p.sq8_order, std::max<uint32_t>(1, ceil_log2(std::max<uint64_t>(ix->n, 2))), ef);
  // distance helpers (4-wave workgroups; a helper's memo of 4 x R entries lives in its pool and
  // visited table, checked below)
  p.help = (helpers_requested(ix, p, nq, static_cast<uint64_t>(stream_cus(ix, stream))) && ix->R <= 64 &&
            alaya_amd::search_has_helpers(ix->dim, p.sq8_order, ix->generic)) ? 1u : 0u;
  if (const char *e = std::getenv("ALAYA_HELP_FLAGS")) p.help_flags = static_cast<uint32_t>(std::strtoul(e, nullptr, 10));
  // Wide f32 rows (d = 768 / 960) run one searcher per SIMD; a batch a little larger than that
  // (config 4's S = 1 layout: 1,250 queries per rank on 1,024 searchers) would leave most of a
  // second round idle, so it runs the two-waves-per-SIMD kernel instead (one row per lane group):
  // GIST-shaped 1M, ef 373, 1,250 queries 8.92 -> 7.44 ms, <= 1,024 queries equal, 2,048 and more
  // slower (profiles/r05/gist_rounds/).  ALAYA_TWO_WAVES = 0 / 1 forces it off / on.
  p.two_waves = 0;
  if (!p.help && d_stamps == nullptr && alaya_amd::search_has_two_waves(ix->dim, p.sq8_order, ix->generic)) {
    const char *e = std::getenv("ALAYA_TWO_WAVES");
    const int force = e ? std::atoi(e) : -1;
    if (force == 1) {
      p.two_waves = 1;
    } else if (force != 0) {
      int b1 = 0;
      const size_t probe = alaya_amd::search_wave_lds_bytes(ix->stride, ef, 12, true);
      hip_check(alaya_amd::search_occupancy(p, 1, probe, &b1), "occupancy");
      const uint64_t resident1 = static_cast<uint64_t>(std::max(1, b1)) * static_cast<uint64_t>(stream_cus(ix, stream));
      p.two_waves = (nq > resident1 && 2 * nq <= 3 * resident1) ? 1u : 0u;
    }
  }
  // waves per workgroup: never more than the batch needs (helpers: always 4).  A plan with helpers
  // that does not fit (the memo, or four waves' LDS with a forced large visited table) falls back
  // to the search without them.
  int W = 1;
  size_t lds = 0;
  for (;;) {
    W = p.help ? 4 : search_waves(p);
    while (!p.help && W > 1 && static_cast<uint64_t>(W) > nq) W /= 2;
    p.hash_log2 = size_visited(ix, p, nq, ef, W);
    const bool compact = p.vis_rbits != alaya_amd::kVisWide;
    p.wave_lds = static_cast<uint32_t>(alaya_amd::search_wave_lds_bytes(ix->stride, ef, p.hash_log2, compact,
                                                                        p.sq8_order));
    bool fits = true;
    if (p.help) {
      // the memo (W searchers x kHelpMemoSlots requests x R entries of 8 bytes) overlays the memo
      // wave's query vector, or else its pool and visited table (past the query and the three
      // 64-entry lists the helper still uses)
      const size_t need = static_cast<size_t>(W) * alaya_amd::kHelpMemoSlots * ix->R * 8;
      const size_t q_bytes = alaya_amd::search_query_lds_bytes(ix->stride, p.sq8_order);
      if (q_bytes >= need) {
        p.memo_off = 0;
      } else if (p.wave_lds >= q_bytes + 3 * 64 * 4 + need) {
        p.memo_off = static_cast<uint32_t>(q_bytes + 3 * 64 * 4);
      } else {
        fits = false;
      }
    }
    lds = alaya_amd::search_shared_lds_bytes(ix->stride, sq8) + static_cast<size_t>(W) * p.wave_lds +
          (p.help ? alaya_amd::kHelpBoardBytes : 0);
    if (p.help && (!fits || lds > kLdsPerCu)) {
      p.help = 0;
      continue;
    }
    break;
  }
  if (lds > kLdsPerCu) throw ArgError("ef / dim too large for the LDS budget");
  int per_cu = 0;
  hip_check(alaya_amd::search_occupancy(p, W, lds, &per_cu), "occupancy");
  per_cu = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(per_cu, max_search_waves_per_cu() / W)));
  // with helpers the grid fills the CUs whatever the batch (idle waves help from the start)
  const uint64_t cus = static_cast<uint64_t>(stream_cus(ix, stream));
  const uint64_t blocks_needed = p.help ? static_cast<uint64_t>(per_cu) * cus : (nq + W - 1) / W;
  const uint64_t grid64 = std::min<uint64_t>(blocks_needed, static_cast<uint64_t>(per_cu) * cus);
  const int grid = static_cast<int>(std::max<uint64_t>(1, grid64));
  scratch_acquire(ix, stream);
  prepare_spill(ix, p, static_cast<uint64_t>(grid) * W, stream);
  ix->last_grid = static_cast<uint32_t>(grid);
  ix->last_waves = static_cast<uint32_t>(W);
  ix->help_stats_slots = 0;
  if (p.help) {
    ix->help_stats_slots = static_cast<uint64_t>(grid) * W;
    ix->help_stats.reserve(ix->help_stats_slots * 12);
    p.help_stats = ix->help_stats.as<uint32_t>();
  }
  ix->work.reserve(4);
  p.work_counter = ix->work.as<uint32_t>();
  hip_check(hipMemsetAsync(p.work_counter, 0, 4, stream), "hipMemsetAsync");
  hip_check(alaya_amd::launch_search(p, grid, W, lds, stream), "search launch");
  scratch_release(ix, stream);
}

void ensure_norms(alaya_index *ix, hipStream_t stream) {
  if (ix->norms_ready) return;
  ix->norms.reserve(std::max<uint64_t>(ix->n, 1) * 4);
  hip_check(alaya_amd::launch_row_norms(ix->base.as<float>(), ix->n, ix->stride, ix->norms.as<float>(), stream),
            "row norms");
  std::vector<float> h(ix->n);
  hip_check(hipMemcpyAsync(h.data(), ix->norms.ptr, ix->n * 4, hipMemcpyDeviceToHost, stream), "D2H");
  hip_check(hipStreamSynchronize(stream), "norms");
  float mx = 0.f;
  for (float v : h) mx = std::max(mx, v);
  ix->max_norm = std::sqrt(mx) * 1.0001f;
  ix->norms_ready = true;
}

// Base chunks per query group: enough blocks to cover the CUs, each chunk >= 64 rows.
int flat_chunks(alaya_index *ix, int nqg, uint64_t rows) {
  int chunks = (ix->num_cus + nqg - 1) / nqg;
  chunks = std::max(8, (chunks + 7) / 8 * 8);
  const uint64_t max_chunks = std::max<uint64_t>(8, (rows / 64) / 8 * 8);
  return static_cast<int>(std::min<uint64_t>(chunks, max_chunks));
}

// Chunks per query group of the single-role f16 scan (256 queries per block, one block per CU): the
// fewest chunks that give every CU a block; past that, the chunk count in 8..64 whose blocks fill
// whole rounds of the CUs best (fewer chunks on ties -- each chunk adds ~32 ln(rows) appends per
// query).  Every chunk keeps >= 4 records.
int flat_tiles_chunks(alaya_index *ix, uint64_t nq, uint64_t scan_tiles) {
  const uint64_t qpb = alaya_amd::flat_tiles_queries();
  const uint64_t nqg = (nq + qpb - 1) / qpb;
  const uint64_t cus = static_cast<uint64_t>(std::max(1, ix->num_cus));
  const uint64_t cap = std::max<uint64_t>(8, std::min<uint64_t>(256, (scan_tiles / 4) / 8 * 8));
  if (nqg * 8 < cus) return static_cast<int>(std::min<uint64_t>(cap, (cus + nqg - 1) / nqg + 7) / 8 * 8);
  uint64_t best = 8;
  double best_eff = 0.0;
  for (uint64_t c = 8; c <= std::min<uint64_t>(64, cap); c += 8) {
    const uint64_t b = nqg * c;
    const double eff = static_cast<double>(b) / static_cast<double>((b + cus - 1) / cus * cus);
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = c;
    }
  }
  return static_cast<int>(best);
}

void ensure_tiles(alaya_index *ix, int base_exp, hipStream_t stream) {
  if (ix->tiles_ready && ix->tiles_exp == base_exp) return;
  const size_t bytes = alaya_amd::flat_tiles_bytes(ix->stride, ix->n);
  ix->flat_tiles.reserve(std::max<size_t>(bytes, 256));
  hip_check(alaya_amd::launch_flat_tiles(ix->base.as<float>(), ix->n, ix->stride, ix->norms.as<float>(),
                                         ix->has_valid ? ix->valid.as<uint32_t>() : nullptr, base_exp,
                                         ix->flat_tiles.as<unsigned char>(), stream),
            "flat tile records");
  ix->tiles_ready = true;
  ix->tiles_exp = base_exp;
}

// Prescan: the same scan over rows 0, S, 2S, ... (S = ALAYA_FLAT_PRESCAN; default 0 = off: on
// config 2 it cuts fold rounds 846 -> 302 per block but costs more than it saves),
// then per query the sample's 32nd-best approximate distance as every chunk's starting threshold.
// The sample's 32nd is about the whole base's (32 S)-th, so the full scan appends ~S candidates
// per (query, chunk) instead of ~32 (1 + ln(chunk rows / 32)).  Results are unchanged: the
// threshold only rejects rows that cannot reach the merged 32, and the merge's bound uses it.
void flat_prescan(alaya_index *ix, alaya_amd::FlatParams &p, int *blocks, hipStream_t s) {
  const char *env = std::getenv("ALAYA_FLAT_PRESCAN");
  const uint64_t step = env ? std::strtoull(env, nullptr, 10) : 0;
  if (p.tiles != nullptr) {
    // The single-role scan's prescan: group minima over a sample of whole tile records (every S-th;
    // default S = records / 4096, on when the base has >= 8192 records, ALAYA_FLAT_PRESCAN=S forces S,
    // 1 turns it off), one block per (query group, group of sampled records); the 32nd smallest
    // of a query's group minima is its starting threshold (flat_group_threshold_kernel).
    const uint64_t nt = p.n_scan_tiles;
    const char *genv = std::getenv("ALAYA_FLAT_PRESCAN_GROUPS");  // diagnostics: groups (default 64)
    const char *senv = std::getenv("ALAYA_FLAT_PRESCAN_SAMPLE");  // diagnostics: sampled records (4096)
    const uint64_t want_sample = senv ? std::max<uint64_t>(32, std::strtoull(senv, nullptr, 10)) : 4096;
    uint64_t S = env ? step : (nt >= 2 * want_sample ? nt / want_sample : 0);
    if (S < 1 || (env && S < 2)) return;
    const uint64_t sample = (nt + S - 1) / S;
    // groups of >= 1 sampled record (64+ at the defaults); the minima (groups x nq floats) fit the
    // candidate buffers (n_chunks >= 8 lists of 32 per query)
    const uint64_t want_groups = genv ? std::strtoull(genv, nullptr, 10) : 64;
    const uint64_t groups = std::min<uint64_t>(std::min<uint64_t>(256, want_groups), sample) / 8 * 8;
    if (groups < static_cast<uint64_t>(alaya_amd::flat_shortlist())) return;
    alaya_amd::FlatParams q = p;
    q.tile_step = static_cast<uint32_t>(S);
    q.n_scan_tiles = sample;
    q.n_chunks = static_cast<int>(groups);
    q.tau_init = nullptr;
    q.out_ids = nullptr;
    q.out_dists = nullptr;
    q.flags = nullptr;
    q.merge_count = nullptr;
    q.ablate = 0;
    ix->flat_tau.reserve(p.nq * 4);
    q.tau_out = ix->flat_tau.as<float>();
    const int qpb = alaya_amd::flat_tiles_queries();
    const int nqg = static_cast<int>((p.nq + qpb - 1) / qpb);
    hip_check(alaya_amd::launch_flat_scan(q, nqg * q.n_chunks, s), "flat prescan");
    hip_check(alaya_amd::launch_flat_threshold(q, s), "flat threshold");
    p.tau_init = q.tau_out;
    return;
  }
  if (step < 2 || p.n / step < 1024) return;
  // the slabbed wide scan (rows past 224 floats) reads contiguous rows and has no row_step: its
  // "sample" would be the first n/S rows, so the prescan is off there
  if (alaya_amd::flat_query_width(ix->stride) != 0) return;
  alaya_amd::FlatParams q = p;
  q.n = (p.n + step - 1) / step;
  q.row_step = static_cast<uint32_t>(step);
  const int nqg = static_cast<int>((p.nq + 127) / 128);
  q.n_chunks = flat_chunks(ix, nqg, q.n);  // <= p.n_chunks: the candidate buffers fit
  q.tau_init = nullptr;
  q.out_ids = nullptr;
  q.out_dists = nullptr;
  q.flags = nullptr;
  q.merge_count = nullptr;
  q.ablate = 0;
  ix->flat_tau.reserve(p.nq * 4);
  q.tau_out = ix->flat_tau.as<float>();
  hip_check(alaya_amd::launch_flat_scan(q, nqg * q.n_chunks, s), "flat prescan");
  hip_check(alaya_amd::launch_flat_threshold(q, s), "flat threshold");
  p.tau_init = q.tau_out;
  (void)blocks;
}

alaya_amd::FlatParams flat_params(alaya_index *ix, const float *d_q, uint64_t nq, uint32_t k, uint32_t *d_ids,
                                  float *d_dists, uint32_t *d_flags, int *blocks, hipStream_t stream,
                                  bool no_single = false) {
  if (!ix->base.ptr) throw ArgError("index has no base vectors");
  if (ix->metric != ALAYA_METRIC_L2) throw ArgError("the flat MFMA path supports the L2 metric");
  if (ix->generic) throw ArgError("the flat MFMA path ranks float32 rows (not the generic non-float order)");
  if (alaya_amd::flat_scan_lds(ix->stride) == 0) throw ArgError("no flat MFMA scan for this row stride");
  if (k == 0 || k > static_cast<uint32_t>(alaya_amd::flat_max_k()))
    throw ArgError("flat search needs 1 <= k <= " + std::to_string(alaya_amd::flat_max_k()));
  alaya_amd::FlatParams p{};
  p.base = ix->base.as<float>();
  p.n = ix->n;
  p.dim = ix->dim;
  p.stride = ix->stride;
  p.norms = ix->norms.as<float>();
  p.valid = ix->has_valid ? ix->valid.as<uint32_t>() : nullptr;
  p.max_norm = ix->max_norm;
  // The contraction that ranks the shortlist (all three feed the same exact rescoring and proof):
  //  * single-pass f16 (default for rows of <= 224 floats, the warp-specialised scan): one MFMA per
  //    16 k on power-of-two-scaled operands; needs the row scale 2^s in range (|s| <= 60);
  //  * bf16 hi/lo split (wide rows, or rows out of the f16 scale's range, or
  //    ALAYA_FLAT_CONTRACTION=bf16x3), unless the rows are large enough for bf16(x) to overflow;
  //  * f32 MFMA (ALAYA_FLAT_CONTRACTION=f32 or ALAYA_FLAT_F32).
  const char *fc = std::getenv("ALAYA_FLAT_CONTRACTION");
  const std::string want = fc ? fc : (std::getenv("ALAYA_FLAT_F32") ? "f32" : "auto");
  if (want != "auto" && want != "f16" && want != "bf16x3" && want != "f32")
    throw ArgError("ALAYA_FLAT_CONTRACTION must be f16, bf16x3 or f32");
  p.base_exp = alaya_amd::flat_base_exp(ix->max_norm);
  const bool narrow = alaya_amd::flat_query_width(ix->stride) == 0;
  p.single = !no_single && (want == "auto" || want == "f16") && narrow && alaya_amd::flat_ws_available(0) &&
             std::abs(p.base_exp) <= 60 && ix->max_norm > 0.f && std::isfinite(ix->max_norm);
  p.split = !p.single && want != "f32" && ix->max_norm < 1e18f;
  ix->flat_contraction = p.single ? 2 : (p.split ? 1 : 0);
  p.queries = d_q;
  p.nq = nq;
  p.q_stride = ix->dim;
  p.k_acc = ix->stride;
  if (const uint32_t width = alaya_amd::flat_query_width(ix->stride)) {
    // wide rows: the scan reads the queries as zero-padded rows of the slabbed width
    ix->flat_q.reserve(nq * width * 4);
    hip_check(alaya_amd::launch_pad_queries(d_q, nq, ix->dim, width, ix->flat_q.as<float>(), stream), "pad queries");
    p.queries = ix->flat_q.as<float>();
    p.q_stride = width;
    p.k_acc = width;
  }
  // the single pass runs the single-role scan over the cached tile records (ALAYA_FLAT_TILES=0 keeps
  // the warp-specialised scan, which converts the f32 rows itself)
  const char *tenv = std::getenv("ALAYA_FLAT_TILES");
  const bool tiles = p.single && !(tenv && tenv[0] == '0') && alaya_amd::flat_tiles_bytes(ix->stride, ix->n) > 0;
  int nqg = 0, chunks = 0;
  if (tiles) {
    ensure_tiles(ix, p.base_exp, stream);
    p.tiles = ix->flat_tiles.as<unsigned char>();
    p.n_scan_tiles = (ix->n + 31) / 32;
    p.tile_step = 1;
    const int qpb = alaya_amd::flat_tiles_queries();
    nqg = static_cast<int>((nq + qpb - 1) / qpb);
    chunks = flat_tiles_chunks(ix, nq, p.n_scan_tiles);
    ix->tiles_cand.reserve(static_cast<size_t>(nqg) * chunks * qpb * alaya_amd::flat_tiles_buf() * 8);
    p.tiles_buf = ix->tiles_cand.as<uint64_t>();
    ix->tiles_qexp.reserve(nq * 4);
    p.tiles_qexp = ix->tiles_qexp.as<int>();
  } else {
    nqg = static_cast<int>((nq + 127) / 128);
    chunks = flat_chunks(ix, nqg, ix->n);
  }
  p.n_chunks = chunks;
  p.row_step = 1;
  const char *spin = std::getenv("ALAYA_FLAT_SPIN_LIMIT");  // debug override (tests force an abort)
  p.spin_limit = spin ? static_cast<uint32_t>(std::strtoul(spin, nullptr, 10)) : (1u << 20);
  const size_t cand = static_cast<size_t>(chunks) * nq * alaya_amd::flat_shortlist();
  ix->cand_d.reserve(cand * 4);
  ix->cand_i.reserve(cand * 4);
  p.cand_d = ix->cand_d.as<float>();
  p.cand_i = ix->cand_i.as<uint32_t>();
  p.k = k;
  p.out_ids = d_ids;
  p.out_dists = d_dists;
  p.flags = d_flags;
  *blocks = nqg * chunks;
  return p;
}

}  // namespace

extern "C" {

const char *alaya_last_error(void) { return g_last_error.c_str(); }

#ifndef ALAYA_BUILD_INFO
#define ALAYA_BUILD_INFO "source=unknown"
#endif
const char *alaya_build_info(void) { return ALAYA_BUILD_INFO; }

int alaya_device_count(int *count) {
  return guarded([&] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
  });
}

// ---- graphs ---------------------------------------------------------------------------------
int alaya_hbm_stream_read(int device, uint64_t bytes, int iters, double *gbs) {
  return guarded([&] {
    if (!gbs || bytes < (1u << 20) || iters < 1) throw ArgError("invalid arguments");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) throw DeviceError("no HIP device available");
    if (device < 0 || device >= count) throw ArgError("device ordinal out of range");
    hip_check(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    bytes = bytes / 16 * 16;
    DevBuf buf, sink;
    buf.reserve(bytes);
    sink.reserve(4);
    hipStream_t s = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(hipEventCreate(&a), "hipEventCreate");
    hip_check(hipEventCreate(&b), "hipEventCreate");
    double best = 0.0;
    try {
      hip_check(hipMemsetAsync(buf.ptr, 0, bytes, s), "memset");
      for (int shape = 0; shape < 3; ++shape) {
        for (int occ : {8, 16}) {  // 256-thread workgroups per CU
          const int grid = prop.multiProcessorCount * occ;
          hip_check(alaya_amd::launch_stream_read(buf.ptr, bytes, grid, shape, sink.as<float>(), s), "stream read");
          for (int it = 0; it < iters; ++it) {
            hip_check(hipEventRecord(a, s), "hipEventRecord");
            hip_check(alaya_amd::launch_stream_read(buf.ptr, bytes, grid, shape, sink.as<float>(), s), "stream read");
            hip_check(hipEventRecord(b, s), "hipEventRecord");
            hip_check(hipEventSynchronize(b), "hipEventSynchronize");
            float ms = 0.f;
            hip_check(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
            best = std::max(best, static_cast<double>(bytes) / (ms * 1e6));
          }
        }
      }
    } catch (...) {
      (void)hipStreamSynchronize(s);
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
      (void)hipStreamDestroy(s);
      throw;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipStreamDestroy(s);
    *gbs = best;
  });
}

int alaya_graph_build_hnsw(const float *data, uint64_t n, uint32_t dim, int metric, uint32_t R,
                           uint32_t ef_construction, uint32_t num_threads, uint64_t seed,
                           alaya_graph **out) {
  return guarded([&] {
    if (!out || (n && !data) || dim == 0) throw ArgError("invalid arguments");
    if ((metric & ~ALAYA_DIST_GENERIC) < ALAYA_METRIC_L2 || (metric & ~ALAYA_DIST_GENERIC) > ALAYA_METRIC_COS)
      throw ArgError("unknown metric");
    if (n >= (1ull << 31)) throw ArgError("ids must stay below 2^31 (LinearPool checked bit)");
    auto g = std::make_unique<alaya_graph>();
    g->g = alaya_amd::build_hnsw(data, n, dim, metric, R, ef_construction, num_threads, seed);
    *out = g.release();
  });
}

int alaya_graph_load(const char *path, int id_bytes, alaya_graph **out) {
  return guarded([&] {
    if (!out || !path) throw ArgError("invalid arguments");
    auto g = std::make_unique<alaya_graph>();
    g->g = alaya_amd::load_graph(path, id_bytes);
    *out = g.release();
  });
}

int alaya_graph_save(const alaya_graph *g, const char *path, int id_bytes, uint64_t capacity,
                     const uint8_t *valid_bitmap) {
  return guarded([&] {
    if (!g || !path) throw ArgError("invalid arguments");
    alaya_amd::save_graph(g->g, path, id_bytes, capacity, valid_bitmap);
  });
}

int alaya_graph_info(const alaya_graph *g, uint64_t *n, uint32_t *R, int *has_overlay,
                     uint32_t *upper_R, uint32_t *ep, uint32_t *max_level,
                     uint64_t *n_upper_edges, uint32_t *n_eps) {
  return guarded([&] {
    if (!g) throw ArgError("null graph");
    if (n) *n = g->g.n;
    if (R) *R = g->g.R;
    if (has_overlay) *has_overlay = g->g.has_overlay ? 1 : 0;
    if (upper_R) *upper_R = g->g.upper_R;
    if (ep) *ep = g->g.ep;
    if (max_level) *max_level = g->g.max_level();
    if (n_upper_edges) *n_upper_edges = g->g.upper_edges.size();
    if (n_eps) *n_eps = static_cast<uint32_t>(g->g.eps.size());
  });
}

int alaya_graph_export(const alaya_graph *g, uint32_t *l0, uint32_t *levels, uint64_t *upper_off,
                       uint32_t *upper_edges, uint32_t *eps) {
  return guarded([&] {
    if (!g) throw ArgError("null graph");
    const HostGraph &h = g->g;
    if (l0) std::memcpy(l0, h.l0.data(), h.l0.size() * 4);
    if (levels && !h.levels.empty()) std::memcpy(levels, h.levels.data(), h.levels.size() * 4);
    if (upper_off && !h.upper_off.empty()) std::memcpy(upper_off, h.upper_off.data(), h.upper_off.size() * 8);
    if (upper_edges && !h.upper_edges.empty())
      std::memcpy(upper_edges, h.upper_edges.data(), h.upper_edges.size() * 4);
    if (eps && !h.eps.empty()) std::memcpy(eps, h.eps.data(), h.eps.size() * 4);
  });
}

int alaya_graph_import(uint64_t n, uint32_t R, const uint32_t *l0, const uint32_t *levels,
                       const uint64_t *upper_off, const uint32_t *upper_edges,
                       uint64_t n_upper_edges, uint32_t upper_R, uint32_t ep, const uint32_t *eps,
                       uint32_t n_eps, alaya_graph **out) {
  return guarded([&] {
    if (!out || (n && !l0) || R == 0 || R > 64) throw ArgError("invalid graph arrays (R must be 1..64)");
    auto g = std::make_unique<alaya_graph>();
    HostGraph &h = g->g;
    h.n = n;
    h.R = R;
    h.l0.assign(l0, l0 + n * R);
    if (levels) {
      if (!upper_off || (n_upper_edges && !upper_edges) || upper_R == 0 || upper_R > 64)
        throw ArgError("invalid overlay arrays (upper_R must be 1..64)");
      if (n && ep >= n) throw ArgError("entry point out of range");
      h.has_overlay = true;
      h.levels.assign(levels, levels + n);
      h.upper_off.assign(upper_off, upper_off + n);
      h.upper_edges.assign(upper_edges, upper_edges + n_upper_edges);
      h.upper_R = upper_R;
      h.ep = ep;
      for (uint64_t i = 0; i < n; ++i)
        if (h.levels[i] && h.upper_off[i] + static_cast<uint64_t>(h.levels[i]) * upper_R > n_upper_edges)
          throw ArgError("upper_off/levels exceed upper_edges");
    } else {
      if (n_eps == 0 && n) throw ArgError("graph without overlay needs entry points");
      h.eps.assign(eps, eps + n_eps);
    }
    *out = g.release();
  });
}

void alaya_graph_free(alaya_graph *g) { delete g; }

// ---- device index ----------------------------------------------------------------------------
int alaya_index_create(int device, alaya_index **out) {
  return guarded([&] {
    if (!out) throw ArgError("null out");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
      throw DeviceError("no HIP device available (the MI355X search path has no CPU fallback)");
    if (device < 0 || device >= count) throw ArgError("device ordinal out of range");
    auto ix = std::make_unique<alaya_index>();
    ix->device = device;
    set_device(ix.get());
    hipDeviceProp_t prop;
    hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    ix->num_cus = prop.multiProcessorCount;
    hip_check(hipStreamCreateWithFlags(&ix->stream, hipStreamNonBlocking), "hipStreamCreate");
    hip_check(hipEventCreateWithFlags(&ix->scratch_ev, hipEventDisableTiming), "hipEventCreate");
    *out = ix.release();
  });
}

void alaya_index_destroy(alaya_index *ix) {
  if (!ix) return;
  (void)hipSetDevice(ix->device);
  if (ix->scratch_used) (void)hipEventSynchronize(ix->scratch_ev);
  if (ix->scratch_ev) (void)hipEventDestroy(ix->scratch_ev);
  if (ix->stream) (void)hipStreamDestroy(ix->stream);
  delete ix;
}

int alaya_index_set_base(alaya_index *ix, const float *rows, uint64_t n, uint32_t dim, int metric,
                         const uint8_t *valid_bitmap) {
  return guarded([&] {
    if (!ix || (n && !rows) || dim == 0) throw ArgError("invalid arguments");
    const bool generic = (metric & ALAYA_DIST_GENERIC) != 0;
    metric &= ~ALAYA_DIST_GENERIC;
    if (metric < ALAYA_METRIC_L2 || metric > ALAYA_METRIC_COS) throw ArgError("unknown metric");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    scratch_drain(ix);
    const uint32_t stride = round_up32(dim);
    if (ix->has_sq8) {  // new rows: the codes describe the old ones, whatever the shape
      ix->has_sq8 = false;
      ix->codes.release();
      ix->sq_min.release();
      ix->sq_max.release();
    }
    ix->base.release();
    ix->base.reserve(std::max<uint64_t>(n, 1) * stride * 4);
    if (n) {
      hip_check(hipMemset2DAsync(ix->base.ptr, static_cast<size_t>(stride) * 4, 0,
                                 static_cast<size_t>(stride) * 4, n, ix->stream), "memset");
      hip_check(hipMemcpy2DAsync(ix->base.ptr, static_cast<size_t>(stride) * 4, rows,
                                 static_cast<size_t>(dim) * 4, static_cast<size_t>(dim) * 4, n,
                                 hipMemcpyHostToDevice, ix->stream), "upload base");
    }
    ix->has_valid = valid_bitmap != nullptr;
    ix->valid.release();
    if (valid_bitmap) {
      const size_t words = (n + 31) / 32;
      std::vector<uint32_t> w(std::max<size_t>(words, 1), 0);
      std::memcpy(w.data(), valid_bitmap, (n + 7) / 8);
      ix->valid.reserve(w.size() * 4);
      hip_check(hipMemcpyAsync(ix->valid.ptr, w.data(), w.size() * 4, hipMemcpyHostToDevice,
                               ix->stream), "upload bitmap");
      hip_check(hipStreamSynchronize(ix->stream), "sync");
    }
    hip_check(hipStreamSynchronize(ix->stream), "sync");
    ix->n = n;
    ix->dim = dim;
    ix->stride = stride;
    ix->metric = metric;
    ix->generic = generic;
    ix->overflow.release();
    ix->overflow_clean = 0;
    ix->norms_ready = false;
    ix->tiles_ready = false;
    ix->capacity = n;
    ix->upd_graph.reset();
    ix->upd_rows.reset();
    ix->upd_ctx.reset();
  });
}

int alaya_index_set_graph(alaya_index *ix, const alaya_graph *g) {
  return guarded([&] {
    if (!ix || !g) throw ArgError("invalid arguments");
    const HostGraph &h = g->g;
    if (h.R == 0 || h.R > 64) throw ArgError("max_nbrs must be 1..64 for the device search");
    if (h.has_overlay && (h.upper_R == 0 || h.upper_R > 64)) throw ArgError("overlay degree must be 1..64");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    scratch_drain(ix);
    auto up = [&](DevBuf &b, const void *src, size_t bytes) {
      b.release();
      b.reserve(std::max<size_t>(bytes, 4));
      if (bytes)
        hip_check(hipMemcpyAsync(b.ptr, src, bytes, hipMemcpyHostToDevice, ix->stream), "upload graph");
    };
    // rows of a HNSW adjacency list never repeat an id; scan once so the kernel can skip dedup.
    bool dup = false;
    for (uint64_t i = 0; i < h.n && !dup; ++i) {
      const uint32_t *r = &h.l0[i * h.R];
      for (uint32_t a = 0; a < h.R && r[a] != 0xffffffffu && !dup; ++a)
        for (uint32_t b = 0; b < a; ++b)
          if (r[a] == r[b]) {
            dup = true;
            break;
          }
    }
    up(ix->l0, h.l0.data(), h.l0.size() * 4);
    up(ix->levels, h.levels.data(), h.levels.size() * 4);
    up(ix->upper_off, h.upper_off.data(), h.upper_off.size() * 8);
    up(ix->upper_edges, h.upper_edges.data(), h.upper_edges.size() * 4);
    up(ix->eps, h.eps.data(), h.eps.size() * 4);
    hip_check(hipStreamSynchronize(ix->stream), "sync");
    ix->R = h.R;
    ix->upper_R = h.upper_R;
    ix->ep = h.ep;
    ix->n_eps = static_cast<uint32_t>(h.eps.size());
    ix->has_overlay = h.has_overlay;
    ix->dedup = dup;
    ix->graph_n = h.n;
    ix->has_graph = true;
    ix->upd_graph.reset();
    ix->upd_rows.reset();
    ix->upd_ctx.reset();
  });
}

// ---- device mirror patches (online updates) ------------------------------------------------
namespace {

// Grow a device buffer to `bytes`, keeping its first `keep` bytes.
void grow_keep(alaya_index *ix, DevBuf &b, size_t bytes, size_t keep) {
  if (bytes <= b.bytes) return;
  DevBuf nb;
  nb.reserve(bytes);
  hip_check(hipMemsetAsync(nb.ptr, 0, nb.bytes, ix->stream), "memset");
  if (keep && b.ptr) hip_check(hipMemcpyAsync(nb.ptr, b.ptr, keep, hipMemcpyDeviceToDevice, ix->stream), "copy");
  hip_check(hipStreamSynchronize(ix->stream), "sync");
  std::swap(b.ptr, nb.ptr);
  std::swap(b.bytes, nb.bytes);
}

void reserve_locked(alaya_index *ix, uint64_t capacity) {
  if (!ix->base.ptr) throw ArgError("index has no base vectors");
  if (capacity < ix->n) throw ArgError("capacity below the stored rows");
  const size_t row = static_cast<size_t>(ix->stride) * 4;
  grow_keep(ix, ix->base, std::max<uint64_t>(capacity, 1) * row, ix->n * row);
  const size_t words = (std::max<uint64_t>(capacity, 1) + 31) / 32;
  if (!ix->has_valid) {  // all stored rows valid: materialise the bitmap so rows can be removed
    std::vector<uint32_t> w(words, 0u);
    for (uint64_t i = 0; i < ix->n; ++i) w[i >> 5] |= 1u << (i & 31);
    ix->valid.release();
    ix->valid.reserve(words * 4);
    hip_check(hipMemcpyAsync(ix->valid.ptr, w.data(), words * 4, hipMemcpyHostToDevice, ix->stream), "bitmap");
    hip_check(hipStreamSynchronize(ix->stream), "sync");
    ix->has_valid = true;
  } else {
    grow_keep(ix, ix->valid, words * 4, (ix->n + 31) / 32 * 4);
  }
  if (ix->has_graph) {
    grow_keep(ix, ix->l0, std::max<uint64_t>(capacity, 1) * ix->R * 4, ix->graph_n * ix->R * 4);
    grow_keep(ix, ix->levels, std::max<uint64_t>(capacity, 1) * 4, ix->graph_n * 4);
    grow_keep(ix, ix->upper_off, std::max<uint64_t>(capacity, 1) * 8, ix->graph_n * 8);
  }
  ix->capacity = std::max(ix->capacity, capacity);
}

// The three patch helpers below change buffers an in-flight search reads (rows, adjacency, the
// validity bitmap), so each first waits for every earlier launch on the index (alaya_hip.h's
// stream contract: a call is ordered after the launches before it).
void write_rows_locked(alaya_index *ix, uint64_t first, const float *rows, uint64_t count) {
  scratch_drain(ix);
  const size_t row = static_cast<size_t>(ix->stride) * 4;
  if (first + count > ix->capacity || (first + count) * row > ix->base.bytes)
    throw ArgError("rows beyond the reserved capacity");
  char *dst = static_cast<char *>(ix->base.ptr) + first * row;
  hip_check(hipMemset2DAsync(dst, row, 0, row, count, ix->stream), "memset");
  hip_check(hipMemcpy2DAsync(dst, row, rows, static_cast<size_t>(ix->dim) * 4, static_cast<size_t>(ix->dim) * 4,
                             count, hipMemcpyHostToDevice, ix->stream), "write rows");
  hip_check(hipStreamSynchronize(ix->stream), "sync");
  ix->n = std::max(ix->n, first + count);
  ix->norms_ready = false;
  ix->tiles_ready = false;
}

void write_edges_locked(alaya_index *ix, const uint32_t *ids, const uint32_t *edges, uint64_t count) {
  if (!ix->has_graph) throw ArgError("index has no graph");
  scratch_drain(ix);
  for (uint64_t i = 0; i < count; ++i) {
    if (ids[i] >= ix->capacity || ids[i] >= ix->n || (static_cast<uint64_t>(ids[i]) + 1) * ix->R * 4 > ix->l0.bytes ||
        (ix->has_overlay && (static_cast<uint64_t>(ids[i]) + 1) * 4 > ix->levels.bytes))
      throw ArgError("edge row id out of range (reserve capacity first)");
    const uint32_t *r = edges + i * ix->R;
    for (uint32_t a = 0; a < ix->R && r[a] != 0xffffffffu; ++a) {
      for (uint32_t b = 0; b < a; ++b)
        if (r[a] == r[b]) ix->dedup = true;  // e.g. the zero padding update() writes
    }
    hip_check(hipMemcpyAsync(ix->l0.as<uint32_t>() + static_cast<uint64_t>(ids[i]) * ix->R, r, ix->R * 4,
                             hipMemcpyHostToDevice, ix->stream), "write edges");
    ix->graph_n = std::max<uint64_t>(ix->graph_n, static_cast<uint64_t>(ids[i]) + 1);
  }
  hip_check(hipStreamSynchronize(ix->stream), "sync");
}

void set_valid_locked(alaya_index *ix, uint64_t id, bool valid) {
  if (!ix->has_valid || id >= ix->capacity || (id / 32 + 1) * 4 > ix->valid.bytes)
    throw ArgError("id out of range (reserve capacity first)");
  scratch_drain(ix);
  uint32_t w = 0;
  uint32_t *dw = ix->valid.as<uint32_t>() + (id >> 5);
  hip_check(hipMemcpy(&w, dw, 4, hipMemcpyDeviceToHost), "read bitmap");
  w = valid ? (w | (1u << (id & 31))) : (w & ~(1u << (id & 31)));
  hip_check(hipMemcpy(dw, &w, 4, hipMemcpyHostToDevice), "write bitmap");
  ix->tiles_ready = false;  // the records carry +inf norms for cleared rows
}

}  // namespace

int alaya_index_reserve(alaya_index *ix, uint64_t capacity) {
  return guarded([&] {
    if (!ix) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    scratch_drain(ix);
    reserve_locked(ix, capacity);
  });
}

int alaya_index_write_rows(alaya_index *ix, uint64_t first, const float *rows, uint64_t count) {
  return guarded([&] {
    if (!ix || (count && !rows)) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    write_rows_locked(ix, first, rows, count);
  });
}

int alaya_index_write_edges(alaya_index *ix, const uint32_t *ids, const uint32_t *edges, uint64_t count) {
  return guarded([&] {
    if (!ix || (count && (!ids || !edges))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    write_edges_locked(ix, ids, edges, count);
  });
}

int alaya_index_set_valid(alaya_index *ix, uint64_t id, int valid) {
  return guarded([&] {
    if (!ix) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    set_valid_locked(ix, id, valid != 0);
  });
}

int alaya_index_enable_updates(alaya_index *ix, const alaya_graph *g, const float *rows, uint64_t n,
                               uint64_t capacity, const uint8_t *valid_bitmap) {
  return guarded([&] {
    if (!ix || !g || (n && !rows)) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (g->g.n != n || ix->n != n || ix->graph_n != n) throw ArgError("graph, rows and device index sizes differ");
    if (capacity < n) throw ArgError("capacity below the stored rows");
    scratch_drain(ix);
    auto m = std::make_unique<alaya_amd::RowMirror>();
    m->dim = ix->dim;
    m->metric = ix->metric | (ix->generic ? ALAYA_DIST_GENERIC : 0);
    m->rows.assign(rows, rows + n * ix->dim);
    m->valid.assign((capacity + 7) / 8 + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
      const bool v = valid_bitmap ? ((valid_bitmap[i >> 3] >> (i & 7)) & 1) : true;
      if (v) m->valid[i >> 3] |= static_cast<uint8_t>(1u << (i & 7));
    }
    ix->upd_graph = std::make_unique<alaya_amd::HostGraph>(g->g);
    ix->upd_rows = std::move(m);
    ix->upd_ctx = std::make_unique<alaya_amd::UpdateContext>();
    reserve_locked(ix, capacity);
  });
}

int alaya_index_insert(alaya_index *ix, const float *search_query, const float *row, uint32_t ef,
                       uint64_t *new_id) {
  return guarded_scratch(ix, [&] {
    if (!ix || !search_query || !row || !new_id) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (!ix->upd_graph) throw ArgError("updates are not enabled on this index");
    alaya_amd::HostGraph &g = *ix->upd_graph;
    alaya_amd::RowMirror &m = *ix->upd_rows;
    alaya_amd::UpdateContext &ctx = *ix->upd_ctx;
    const uint32_t R = g.R;
    // search_solo(query, max_nbrs, results, ef) on the current index (graph_update_job.hpp:67-69)
    std::vector<uint32_t> results(R, 0u);
    ix->q_buf.reserve(static_cast<size_t>(ix->dim) * 4);
    ix->id_buf.reserve(static_cast<size_t>(R) * 4);
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, search_query, ix->dim * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    do_search(ix, ix->q_buf.as<float>(), 1, R, std::max(ef, 1u), ix->id_buf.as<uint32_t>(), nullptr, nullptr,
              ix->stream);
    hip_check(hipMemcpyAsync(results.data(), ix->id_buf.ptr, R * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipStreamSynchronize(ix->stream), "insert search");
    // graph_->insert: -1 when the storage is full (then nothing else happens, :70-73)
    if (g.n >= ix->capacity) {
      *new_id = UINT64_MAX;
      return;
    }
    const uint32_t id = static_cast<uint32_t>(g.n);
    g.l0.insert(g.l0.end(), results.begin(), results.end());
    if (g.has_overlay) {  // Graph::insert adds a level-0 node; the overlay is not touched
      g.levels.push_back(0);
      g.upper_off.push_back(g.upper_edges.size());
    }
    g.n += 1;
    // space_->insert (RawSpace::insert: row stored, validity bit set)
    m.rows.insert(m.rows.end(), row, row + ix->dim);
    m.valid[id >> 3] |= static_cast<uint8_t>(1u << (id & 7));
    for (uint32_t i = 0; i < R; ++i)
      if (results[i] != 0xffffffffu) ctx.inserted_edges[results[i]].push_back(id);
    // update every node that gained an edge (:80-83), in the map's iteration order
    std::vector<uint32_t> touched{id};
    std::vector<uint32_t> edges(results);
    for (const auto &kv : ctx.inserted_edges) {
      std::vector<uint32_t> e = alaya_amd::update_edges(g, m, ctx, kv.first);
      std::copy(e.begin(), e.end(), g.l0.begin() + static_cast<size_t>(kv.first) * R);
      touched.push_back(kv.first);
      edges.insert(edges.end(), e.begin(), e.end());
    }
    ctx.inserted_edges.clear();
    // mirror into HBM: the row, its validity bit, the new and the updated adjacency rows
    write_rows_locked(ix, id, row, 1);
    set_valid_locked(ix, id, true);
    write_edges_locked(ix, touched.data(), edges.data(), touched.size());
    *new_id = id;
  });
}

int alaya_index_remove(alaya_index *ix, uint64_t id) {
  return guarded([&] {
    if (!ix) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (!ix->upd_graph) throw ArgError("updates are not enabled on this index");
    if (id >= ix->upd_graph->n) throw ArgError("id out of range");
    alaya_amd::record_remove(*ix->upd_graph, *ix->upd_ctx, static_cast<uint32_t>(id));
    ix->upd_rows->valid[id >> 3] &= static_cast<uint8_t>(~(1u << (id & 7)));
    set_valid_locked(ix, id, false);
  });
}

int alaya_index_export_graph(alaya_index *ix, alaya_graph **out) {
  return guarded([&] {
    if (!ix || !out) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    if (!ix->upd_graph) throw ArgError("updates are not enabled on this index");
    *out = new alaya_graph{*ix->upd_graph};
  });
}

int alaya_index_export_rows(alaya_index *ix, float *rows, uint8_t *valid_bitmap, uint64_t *n) {
  return guarded([&] {
    if (!ix || !n) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    if (!ix->upd_rows) throw ArgError("updates are not enabled on this index");
    *n = ix->upd_graph->n;
    if (rows) std::memcpy(rows, ix->upd_rows->rows.data(), ix->upd_rows->rows.size() * 4);
    if (valid_bitmap) std::memcpy(valid_bitmap, ix->upd_rows->valid.data(), (*n + 7) / 8);
  });
}

}  // extern "C"

// ---- device graph construction ----------------------------------------------------------------
namespace {

// One launch group of the batched build: the points of batch [first, ...) active at `level`.
struct BuildStep {
  uint32_t first;
  int level;
  int max_level;  // graph max level before the batch
  uint32_t ep;    // graph entry point before the batch
  uint64_t off;   // active points: act[off, off + cnt)
  uint32_t cnt;
  int refine;     // level-0 refine pass of the batch
};

// Batch schedule (label order): batch size max(1, min(max_batch, inserted / batch_div)); a point
// whose level exceeds the graph's max level closes its batch, so the entry point / max level a
// batch sees are exactly the sequential ones (hnswlib.hpp:740-748).
std::vector<BuildStep> build_schedule(const std::vector<uint32_t> &lv, uint32_t batch_div, uint32_t max_batch,
                                      uint32_t refine, std::vector<uint32_t> &act, uint32_t *final_ep,
                                      int *final_max) {
  std::vector<BuildStep> steps;
  const uint64_t n = lv.size();
  uint32_t ep = 0;
  int maxl = n ? static_cast<int>(lv[0]) : 0;
  uint64_t i = 1;
  while (i < n) {
    const uint64_t b = std::max<uint64_t>(1, std::min<uint64_t>(max_batch, i / batch_div));
    uint64_t end = std::min<uint64_t>(n, i + b);
    int top = 0;
    for (uint64_t j = i; j < end; ++j) {
      top = std::max(top, std::min(static_cast<int>(lv[j]), maxl));
      if (static_cast<int>(lv[j]) > maxl) {
        end = j + 1;
        break;
      }
    }
    for (int L = top; L >= 0; --L) {
      BuildStep st{static_cast<uint32_t>(i), L, maxl, ep, act.size(), 0, 0};
      for (uint64_t j = i; j < end; ++j)
        if (std::min(static_cast<int>(lv[j]), maxl) >= L) act.push_back(static_cast<uint32_t>(j));
      st.cnt = static_cast<uint32_t>(act.size() - st.off);
      steps.push_back(st);
    }
    // refine passes over level 0 (single-point batches have no batch mates to find)
    for (uint32_t r = 0; r < refine && end - i > 1; ++r) {
      BuildStep st = steps.back();
      st.refine = 1;
      steps.push_back(st);
    }
    if (static_cast<int>(lv[end - 1]) > maxl) {
      ep = static_cast<uint32_t>(end - 1);
      maxl = static_cast<int>(lv[end - 1]);
    }
    i = end;
  }
  *final_ep = ep;
  *final_max = maxl;
  return steps;
}

}  // namespace

extern "C" {

int alaya_index_build_graph(alaya_index *ix, uint32_t R, uint32_t ef_construction, uint64_t seed,
                            uint32_t batch_div, uint32_t max_batch, uint32_t refine, alaya_graph **out,
                            uint64_t *stats) {
  return guarded_scratch(ix, [&] {
    if (!ix) throw ArgError("invalid arguments");
    if (R < 2 || R > 64 || R % 2) throw ArgError("max_nbrs must be even and in 2..64 for the device build");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    scratch_drain(ix);
    if (!ix->base.ptr || ix->n == 0) throw ArgError("index has no base vectors");
    if (ix->n >= (1ull << 31)) throw ArgError("ids must stay below 2^31 (LinearPool checked bit)");
    const uint64_t n = ix->n;
    const uint32_t M = R / 2;                            // hnsw_builder.hpp:71-72: M = R/2, M0 = R
    const uint32_t ef = std::max(ef_construction, M);    // hnswlib.hpp:104
    batch_div = batch_div ? batch_div : 16;
    max_batch = max_batch ? max_batch : 65536;
    hipStream_t st = ix->stream;
    hipEvent_t e0, e1;
    hip_check(hipEventCreate(&e0), "event");
    hip_check(hipEventCreate(&e1), "event");

    // levels and overlay offsets are known up front (upper lists R wide, HNSWBuilder's export)
    const std::vector<uint32_t> lv = alaya_amd::hnsw_levels(n, M, seed);
    std::vector<uint64_t> off(n);
    uint64_t n_upper = 0;
    for (uint64_t i = 0; i < n; ++i) {
      off[i] = n_upper;
      n_upper += static_cast<uint64_t>(lv[i]) * R;
    }
    std::vector<uint32_t> act;
    uint32_t ep = 0;
    int maxl = 0;
    const std::vector<BuildStep> steps = build_schedule(lv, batch_div, max_batch, refine, act, &ep, &maxl);
    uint32_t bmax = 1;
    for (const BuildStep &s : steps) bmax = std::max(bmax, s.cnt);

    // device graph (installed as the index's search graph) + scratch
    ix->has_graph = false;
    ix->upd_graph.reset();
    ix->upd_rows.reset();
    ix->upd_ctx.reset();
    ix->l0.release();
    ix->l0.reserve(n * R * 4);
    ix->levels.release();
    ix->levels.reserve(n * 4);
    ix->upper_off.release();
    ix->upper_off.reserve(n * 8);
    ix->upper_edges.release();
    ix->upper_edges.reserve(std::max<uint64_t>(n_upper, 1) * 4);
    hip_check(hipMemsetAsync(ix->l0.ptr, 0xff, n * R * 4, st), "memset");
    if (n_upper) hip_check(hipMemsetAsync(ix->upper_edges.ptr, 0xff, n_upper * 4, st), "memset");
    hip_check(hipMemcpyAsync(ix->levels.ptr, lv.data(), n * 4, hipMemcpyHostToDevice, st), "H2D");
    hip_check(hipMemcpyAsync(ix->upper_off.ptr, off.data(), n * 8, hipMemcpyHostToDevice, st), "H2D");
    DevBuf d_act, d_next, c_ids, c_d, c_n, k_in, k_out, dd_in, dd_out, sort_tmp, cnt;
    d_act.reserve(std::max<size_t>(act.size(), 1) * 4);
    if (!act.empty())
      hip_check(hipMemcpyAsync(d_act.ptr, act.data(), act.size() * 4, hipMemcpyHostToDevice, st), "H2D");
    d_next.reserve(static_cast<size_t>(max_batch) * 4);
    c_ids.reserve(static_cast<size_t>(bmax) * ef * 4);
    c_d.reserve(static_cast<size_t>(bmax) * ef * 4);
    c_n.reserve(static_cast<size_t>(bmax) * 4);
    const size_t n_edge_max = static_cast<size_t>(bmax) * M;
    k_in.reserve(n_edge_max * 8);
    k_out.reserve(n_edge_max * 8);
    dd_in.reserve(n_edge_max * 4);
    dd_out.reserve(n_edge_max * 4);
    size_t tmp_bytes = 0;
    hip_check(alaya_amd::sort_edges(nullptr, &tmp_bytes, nullptr, nullptr, nullptr, nullptr, n_edge_max, st), "sort size");
    sort_tmp.reserve(tmp_bytes);
    cnt.reserve(8 * 8);
    hip_check(hipMemsetAsync(cnt.ptr, 0, 8 * 8, st), "memset");
    ix->work.reserve(4);

    alaya_amd::BuildParams bp{};
    bp.s = base_params(ix);
    bp.s.valid = nullptr;
    bp.s.l0 = ix->l0.as<uint32_t>();
    bp.s.R = R;
    bp.s.levels = ix->levels.as<uint32_t>();
    bp.s.upper_off = ix->upper_off.as<uint64_t>();
    bp.s.upper_edges = ix->upper_edges.as<uint32_t>();
    bp.s.upper_R = R;
    bp.s.queries = nullptr;
    bp.s.ef = ef;
    bp.s.work_counter = ix->work.as<uint32_t>();
    bp.l0w = ix->l0.as<uint32_t>();
    bp.upw = ix->upper_edges.as<uint32_t>();
    bp.next = d_next.as<uint32_t>();
    bp.cand_ids = c_ids.as<uint32_t>();
    bp.cand_d = c_d.as<float>();
    bp.cand_n = c_n.as<uint32_t>();
    bp.M = M;
    bp.counters = cnt.as<unsigned long long>();
    // visited-set sizing and the spill area for the largest batch (sized once: kernels in flight)
    {
      SearchParams probe = bp.s;
      const uint32_t hl = size_visited(ix, probe, bmax, ef);
      const size_t lds = alaya_amd::build_lds_bytes(ix->stride, ef, hl, probe.vis_rbits != alaya_amd::kVisWide);
      bp.s.hash_log2 = hl;
      bp.s.vis_rbits = probe.vis_rbits;
      bp.s.vis_lbits = probe.vis_lbits;
      bp.s.vis_max_disp = probe.vis_max_disp;
      bp.s.vis_limit = probe.vis_limit;
      if (lds > kLdsPerCu) throw ArgError("ef_construction / dim too large for the LDS budget");
    }
    const size_t lds = alaya_amd::build_lds_bytes(ix->stride, ef, bp.s.hash_log2, bp.s.vis_rbits != alaya_amd::kVisWide);
    int per_cu = 0;
    hip_check(alaya_amd::build_search_occupancy(bp, lds, &per_cu), "occupancy");
    per_cu = std::max(1, per_cu);
    const uint64_t grid_max = static_cast<uint64_t>(per_cu) * ix->num_cus;
    prepare_spill(ix, bp.s, std::min<uint64_t>(grid_max, bmax), st);

    hip_check(hipEventRecord(e0, st), "event");
    uint64_t launches = 0;
    for (const BuildStep &s : steps) {
      bp.s.nq = s.cnt;
      bp.s.ep = s.ep;
      bp.pts = d_act.as<uint32_t>() + s.off;
      bp.batch_first = s.first;
      bp.level = s.level;
      bp.max_level = s.max_level;
      bp.refine = s.refine;
      bp.Mmax = s.level == 0 ? R : M;
      bp.edge_keys = k_in.as<uint64_t>();
      bp.edge_d = dd_in.as<float>();
      const int grid = static_cast<int>(std::min<uint64_t>(s.cnt, grid_max));
      const int wide = static_cast<int>(std::min<uint64_t>(s.cnt, static_cast<uint64_t>(ix->num_cus) * 16));
      hip_check(hipMemsetAsync(bp.s.work_counter, 0, 4, st), "memset");
      hip_check(alaya_amd::launch_build_search(bp, grid, lds, st), "build search");
      hip_check(alaya_amd::launch_build_select(bp, wide, st), "build select");
      const uint64_t ne = static_cast<uint64_t>(s.cnt) * M;
      size_t tb = tmp_bytes;
      hip_check(alaya_amd::sort_edges(sort_tmp.ptr, &tb, k_in.as<uint64_t>(), k_out.as<uint64_t>(), dd_in.as<float>(),
                                      dd_out.as<float>(), ne, st), "sort edges");
      bp.edge_keys = k_out.as<uint64_t>();
      bp.edge_d = dd_out.as<float>();
      bp.n_edges = ne;
      const int agrid = static_cast<int>(std::min<uint64_t>((ne + 63) / 64, static_cast<uint64_t>(ix->num_cus) * 16));
      hip_check(alaya_amd::launch_build_apply(bp, agrid, st), "build apply");
      launches += 4;
    }
    hip_check(hipEventRecord(e1, st), "event");
    HostGraph g;
    g.n = n;
    g.R = R;
    g.l0.resize(n * R);
    g.has_overlay = true;
    g.upper_R = R;
    g.ep = ep;
    g.levels = lv;
    g.upper_off = off;
    g.upper_edges.resize(n_upper);
    hip_check(hipMemcpyAsync(g.l0.data(), ix->l0.ptr, n * R * 4, hipMemcpyDeviceToHost, st), "D2H");
    if (n_upper)
      hip_check(hipMemcpyAsync(g.upper_edges.data(), ix->upper_edges.ptr, n_upper * 4, hipMemcpyDeviceToHost, st), "D2H");
    unsigned long long hc[8] = {0};
    hip_check(hipMemcpyAsync(hc, cnt.ptr, sizeof(hc), hipMemcpyDeviceToHost, st), "D2H");
    hip_check(hipStreamSynchronize(st), "device build");
    float ms = 0.f;
    hip_check(hipEventElapsedTime(&ms, e0, e1), "event");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    ix->R = R;
    ix->upper_R = R;
    ix->ep = ep;
    ix->n_eps = 0;
    ix->has_overlay = true;
    ix->dedup = false;
    ix->graph_n = n;
    ix->has_graph = true;
    if (stats) {
      stats[0] = steps.empty() ? 0 : 1;
      for (size_t i = 1; i < steps.size(); ++i) stats[0] += steps[i].first != steps[i - 1].first ? 1 : 0;
      stats[1] = launches;
      stats[2] = hc[0];
      stats[3] = hc[1];
      stats[4] = hc[2];
      stats[5] = static_cast<uint64_t>(ms * 1000.0);
      stats[6] = bmax;
      stats[7] = static_cast<uint64_t>(maxl);
    }
    if (out) *out = new alaya_graph{std::move(g)};
  });
}

int alaya_index_batch_search_device(alaya_index *ix, const float *d_queries, uint64_t nq,
                                    uint32_t k, uint32_t ef, uint32_t *d_ids, float *d_dists,
                                    uint32_t *d_counters, void *stream) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!d_queries || !d_ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    do_search(ix, d_queries, nq, k, ef, d_ids, d_dists, d_counters,
              static_cast<hipStream_t>(stream));
  });
}

int alaya_index_shard_search_device(alaya_index *ix, const float *d_queries, uint64_t nq, uint32_t k,
                                    uint32_t ef, uint32_t *d_ids, float *d_dists, uint32_t *d_counters,
                                    void *stream) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!d_queries || !d_ids || !d_dists))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    do_search(ix, d_queries, nq, k, ef, d_ids, d_dists, d_counters, static_cast<hipStream_t>(stream), nullptr,
              false, 0xffffffffu);
  });
}

int alaya_index_batch_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                             uint32_t ef, uint32_t *ids, float *dists, uint32_t *counters) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!queries || !ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (nq == 0 || k == 0) return;
    ix->q_buf.reserve(nq * ix->dim * 4);
    ix->id_buf.reserve(nq * k * 4);
    ix->dist_buf.reserve(nq * k * 4);
    ix->cnt_buf.reserve(nq * 16);
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, queries, nq * ix->dim * 4, hipMemcpyHostToDevice,
                             ix->stream), "upload queries");
    do_search(ix, ix->q_buf.as<float>(), nq, k, ef, ix->id_buf.as<uint32_t>(),
              ix->dist_buf.as<float>(), ix->cnt_buf.as<uint32_t>(), ix->stream);
    hip_check(hipMemcpyAsync(ids, ix->id_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    if (dists)
      hip_check(hipMemcpyAsync(dists, ix->dist_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    if (counters)
      hip_check(hipMemcpyAsync(counters, ix->cnt_buf.ptr, nq * 16, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipStreamSynchronize(ix->stream), "search");
  });
}

int alaya_index_profile_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                               uint32_t ef, int space, uint32_t *ids, uint32_t *counters, uint64_t *stamps) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!queries || !ids || !stamps))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (nq == 0 || k == 0) return;
    ix->q_buf.reserve(nq * ix->dim * 4);
    ix->id_buf.reserve(nq * k * 4);
    ix->cnt_buf.reserve(nq * 16);
    DevBuf st;
    st.reserve(nq * 64);
    hip_check(hipMemsetAsync(st.ptr, 0, nq * 64, ix->stream), "memset");
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, queries, nq * ix->dim * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    do_search(ix, ix->q_buf.as<float>(), nq, k, ef, ix->id_buf.as<uint32_t>(), nullptr,
              ix->cnt_buf.as<uint32_t>(), ix->stream, st.as<uint64_t>(), space == 1);
    hip_check(hipMemcpyAsync(ids, ix->id_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    if (counters)
      hip_check(hipMemcpyAsync(counters, ix->cnt_buf.ptr, nq * 16, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipMemcpyAsync(stamps, st.ptr, nq * 64, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipStreamSynchronize(ix->stream), "profile search");
  });
}

int alaya_index_distances(alaya_index *ix, const float *queries, uint64_t nq, const uint32_t *ids,
                          uint32_t n, float *out) {
  return guarded([&] {
    if (!ix || (nq && (!queries || !out)) || (n && !ids)) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (!ix->base.ptr) throw ArgError("index has no base vectors");
    if (nq == 0 || n == 0) return;
    if (nq > 65535) throw ArgError("at most 65535 queries per call");
    for (uint32_t i = 0; i < n; ++i)
      if (ids[i] >= ix->n) throw ArgError("id out of range");
    ix->q_buf.reserve(nq * ix->dim * 4);
    ix->dlist_buf.reserve(static_cast<size_t>(n) * 4);
    ix->dout_buf.reserve(nq * n * 4);
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, queries, nq * ix->dim * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    hip_check(hipMemcpyAsync(ix->dlist_buf.ptr, ids, static_cast<size_t>(n) * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    SearchParams p = base_params(ix);
    p.queries = ix->q_buf.as<float>();
    p.q_stride = ix->dim;
    hip_check(alaya_amd::launch_row_distances(p, ix->dlist_buf.as<uint32_t>(), n,
                                              static_cast<uint32_t>(nq), ix->dout_buf.as<float>(),
                                              ix->stream), "distance launch");
    hip_check(hipMemcpyAsync(out, ix->dout_buf.ptr, nq * n * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipStreamSynchronize(ix->stream), "distances");
  });
}

// ---- SQ8 (space/quant/sq8.hpp:78-143, space/sq8_space.hpp) --------------------------------
int alaya_sq8_train(const float *data, uint64_t n, uint32_t dim, float *min_v, float *max_v) {
  return guarded([&] {
    if ((n && !data) || !min_v || !max_v || dim == 0) throw ArgError("invalid arguments");
    for (uint32_t j = 0; j < dim; ++j) {  // SQ8Quantizer ctor: min = max(), max = lowest()
      min_v[j] = std::numeric_limits<float>::max();
      max_v[j] = std::numeric_limits<float>::lowest();
    }
    for (uint64_t i = 0; i < n; ++i) {
      const float *r = data + i * dim;
      for (uint32_t j = 0; j < dim; ++j) {
        if (r[j] < min_v[j]) min_v[j] = r[j];
        if (r[j] > max_v[j]) max_v[j] = r[j];
      }
    }
  });
}

int alaya_sq8_encode(const float *data, uint64_t n, uint32_t dim, const float *min_v,
                     const float *max_v, uint8_t *codes, uint32_t num_threads) {
  return guarded([&] {
    if ((n && (!data || !codes)) || !min_v || !max_v) throw ArgError("invalid arguments");
    auto work = [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i) {
        for (uint32_t j = 0; j < dim; ++j) {  // SQ8Quantizer::quantize (sq8.hpp:118-130)
          const float v = data[i * dim + j], mn = min_v[j], mx = max_v[j];
          uint8_t c;
          if (mx == mn) c = 0;
          else if (v >= mx) c = 255;
          else if (v <= mn) c = 0;
          else c = static_cast<uint8_t>(((v - mn) / (mx - mn)) * 255);
          codes[i * dim + j] = c;
        }
      }
    };
    const uint32_t nt = std::max(1u, std::min<uint32_t>(num_threads, 64));
    std::vector<std::thread> ts;
    const uint64_t per = (n + nt - 1) / nt;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint64_t lo = t * per, hi = std::min(n, lo + per);
      if (lo < hi) ts.emplace_back(work, lo, hi);
    }
    for (auto &t : ts) t.join();
  });
}

int alaya_index_set_sq8(alaya_index *ix, const uint8_t *codes, uint64_t n, uint32_t dim,
                        const float *min_v, const float *max_v, int order) {
  return guarded([&] {
    if (!ix || (n && !codes) || !min_v || !max_v) throw ArgError("invalid arguments");
    if (order != 1 && order != 2) throw ArgError("SQ8 order must be 1 (AVX2) or 2 (AVX-512)");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (ix->base.ptr && (dim != ix->dim || n != ix->n)) throw ArgError("SQ8 codes do not match the base rows");
    scratch_drain(ix);
    const uint32_t cs = (dim + 63) / 64 * 64;
    ix->codes.release();
    ix->codes.reserve(std::max<uint64_t>(n, 1) * cs);
    if (n) {
      hip_check(hipMemsetAsync(ix->codes.ptr, 0, n * cs, ix->stream), "memset");
      hip_check(hipMemcpy2DAsync(ix->codes.ptr, cs, codes, dim, dim, n, hipMemcpyHostToDevice, ix->stream),
                "upload codes");
    }
    ix->sq_min.release();
    ix->sq_max.release();
    ix->sq_min.reserve(dim * 4);
    ix->sq_max.reserve(dim * 4);
    hip_check(hipMemcpyAsync(ix->sq_min.ptr, min_v, dim * 4, hipMemcpyHostToDevice, ix->stream), "upload");
    hip_check(hipMemcpyAsync(ix->sq_max.ptr, max_v, dim * 4, hipMemcpyHostToDevice, ix->stream), "upload");
    hip_check(hipStreamSynchronize(ix->stream), "sync");
    ix->code_stride = cs;
    ix->sq8_order = order;
    ix->has_sq8 = true;
  });
}

// SQ8 graph search (+ optional rerank) on device buffers.  The search writes its ks = k (reference
// rerank) or ef (corrected rerank) ids into ix->sq_ids; the rerank reads them and writes d_ids.
// shard >= 0: shard mode (alaya_index_shard_search_sq8_device) with the reference rerank, the id-0
// zero entries only when shard == 1 (this shard holds global row 0), empty slots (kEmpty, FLT_MAX).
static void sq8_search_dev(alaya_index *ix, const float *d_q, const float *d_rq, uint64_t nq, uint32_t k,
                           uint32_t ef, int rerank, uint32_t *d_ids, float *d_dists, uint32_t *d_cnt,
                           hipStream_t s, int shard = -1) {
  if (rerank < 0 || rerank > 2) throw ArgError("rerank must be 0 (none), 1 (reference) or 2 (corrected)");
  if (nq == 0 || k == 0) return;
  if (!rerank) {
    do_search(ix, d_q, nq, k, ef, d_ids, d_dists, d_cnt, s, nullptr, true, shard >= 0 ? 0xffffffffu : 0u);
    return;
  }
  const bool corrected = rerank == 2;
  const uint32_t ks = corrected ? ef : k;  // corrected: the whole ef pool, kEmpty past the pool
  ix->sq_ids.reserve(nq * ks * 4);
  ix->sq_d.reserve(nq * ks * 4);
  // search fill: the reference's zero-initialised pool slots (rescored as row 0) on a single index
  // and on the shard holding global row 0; empty elsewhere (skipped by the rerank)
  const uint32_t search_fill = (corrected || shard == 0) ? 0xffffffffu : 0u;
  do_search(ix, d_q, nq, ks, ef, ix->sq_ids.as<uint32_t>(), ix->sq_d.as<float>(), d_cnt, s, nullptr, true,
            search_fill);
  SearchParams p = base_params(ix);
  p.queries = d_rq ? d_rq : d_q;
  p.nq = nq;
  p.q_stride = ix->dim;
  alaya_amd::RerankParams r{};
  r.search_ids = ix->sq_ids.as<uint32_t>();
  r.k = k;
  r.n_src = ks;
  r.n_take = corrected ? ef : std::min(k, ef);
  r.zeros = (!corrected && shard != 0 && ef > k) ? ef - k : 0u;
  r.fill_id = shard >= 0 ? 0xffffffffu : 0u;
  r.out_ids = d_ids;
  r.out_dists = d_dists;
  hip_check(alaya_amd::launch_rerank(p, r, s), "rerank launch");
  scratch_release(ix, s);  // the rerank read the search's ids from the index's sq_ids buffer
}

int alaya_index_batch_search_sq8(alaya_index *ix, const float *queries, const float *rerank_queries,
                                 uint64_t nq, uint32_t k, uint32_t ef, int rerank, uint32_t *ids,
                                 float *dists, uint32_t *counters) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!queries || !ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (nq == 0 || k == 0) return;
    ix->q_buf.reserve(nq * ix->dim * 4);
    ix->id_buf.reserve(nq * k * 4);
    ix->dist_buf.reserve(nq * k * 4);
    ix->cnt_buf.reserve(nq * 16);
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, queries, nq * ix->dim * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    const float *d_rq = nullptr;
    if (rerank && rerank_queries && rerank_queries != queries) {
      ix->rr_q_buf.reserve(nq * ix->dim * 4);
      hip_check(hipMemcpyAsync(ix->rr_q_buf.ptr, rerank_queries, nq * ix->dim * 4, hipMemcpyHostToDevice,
                               ix->stream), "H2D");
      d_rq = ix->rr_q_buf.as<float>();
    }
    sq8_search_dev(ix, ix->q_buf.as<float>(), d_rq, nq, k, ef, rerank, ix->id_buf.as<uint32_t>(),
                   ix->dist_buf.as<float>(), ix->cnt_buf.as<uint32_t>(), ix->stream);
    hip_check(hipMemcpyAsync(ids, ix->id_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    if (dists) hip_check(hipMemcpyAsync(dists, ix->dist_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
    if (counters)
      hip_check(hipMemcpyAsync(counters, ix->cnt_buf.ptr, nq * 16, hipMemcpyDeviceToHost, ix->stream), "D2H");
    hip_check(hipStreamSynchronize(ix->stream), "sq8 search");
  });
}

int alaya_index_batch_search_sq8_device(alaya_index *ix, const float *d_queries, const float *d_rerank_queries,
                                        uint64_t nq, uint32_t k, uint32_t ef, int rerank, uint32_t *d_ids,
                                        float *d_dists, uint32_t *d_counters, void *stream) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!d_queries || !d_ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    sq8_search_dev(ix, d_queries, d_rerank_queries, nq, k, ef, rerank, d_ids, d_dists, d_counters,
                   static_cast<hipStream_t>(stream));
  });
}

int alaya_index_shard_search_sq8_device(alaya_index *ix, const float *d_queries, const float *d_rerank_queries,
                                        uint64_t nq, uint32_t k, uint32_t ef, int holds_row0, uint32_t *d_ids,
                                        float *d_dists, uint32_t *d_counters, void *stream) {
  return guarded_scratch(ix, [&] {
    if (!ix || (nq && (!d_queries || !d_ids || !d_dists))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    sq8_search_dev(ix, d_queries, d_rerank_queries, nq, k, ef, 1, d_ids, d_dists, d_counters,
                   static_cast<hipStream_t>(stream), holds_row0 ? 1 : 0);
  });
}

// ---- flat exact k-NN (MFMA shortlist + exact rescoring) ---------------------------------------
int alaya_index_flat_diag(alaya_index *ix, const float *d_queries, uint64_t nq, uint32_t k, int ablate,
                          uint32_t *d_ids, float *d_dists, uint32_t *d_flags, uint32_t *d_merge_count,
                          void *stream) {
  return guarded([&] {
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    hipStream_t s = static_cast<hipStream_t>(stream);
    scratch_acquire(ix, s);
    ensure_norms(ix, s);
    int blocks = 0;
    alaya_amd::FlatParams p = flat_params(ix, d_queries, nq, k, d_ids, d_dists, d_flags, &blocks, s);
    flat_prescan(ix, p, &blocks, s);
    p.ablate = ablate;
    p.merge_count = d_merge_count;
    hip_check(alaya_amd::launch_flat_scan(p, blocks, s), "flat scan");
    scratch_release(ix, s);
  });
}

int alaya_index_flat_search_device(alaya_index *ix, const float *d_queries, uint64_t nq, uint32_t k,
                                   uint32_t *d_ids, float *d_dists, uint32_t *d_flags, void *stream) {
  return guarded([&] {
    if (!ix || (nq && (!d_queries || !d_ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (nq == 0) return;
    hipStream_t s = static_cast<hipStream_t>(stream);
    scratch_acquire(ix, s);
    ensure_norms(ix, s);
    int blocks = 0;
    alaya_amd::FlatParams p = flat_params(ix, d_queries, nq, k, d_ids, d_dists, d_flags, &blocks, s);
    flat_prescan(ix, p, &blocks, s);
    hip_check(alaya_amd::launch_flat_scan(p, blocks, s), "flat scan");
    hip_check(alaya_amd::launch_flat_merge(p, s), "flat merge");
    scratch_release(ix, s);
  });
}

int alaya_index_flat_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                            uint32_t *ids, float *dists, uint32_t *n_recomputed) {
  return guarded([&] {
    if (!ix || (nq && (!queries || !ids))) throw ArgError("invalid arguments");
    std::lock_guard<std::mutex> lk(ix->mu);
    set_device(ix);
    if (n_recomputed) *n_recomputed = 0;
    if (nq == 0) return;
    scratch_acquire(ix, ix->stream);
    ensure_norms(ix, ix->stream);
    ix->q_buf.reserve(nq * ix->dim * 4);
    ix->id_buf.reserve(nq * k * 4);
    ix->dist_buf.reserve(nq * k * 4);
    ix->flag_buf.reserve(nq * 4);
    hip_check(hipMemcpyAsync(ix->q_buf.ptr, queries, nq * ix->dim * 4, hipMemcpyHostToDevice, ix->stream), "H2D");
    int blocks = 0;
    alaya_amd::FlatParams p = flat_params(ix, ix->q_buf.as<float>(), nq, k, ix->id_buf.as<uint32_t>(),
                                          ix->dist_buf.as<float>(), ix->flag_buf.as<uint32_t>(), &blocks, ix->stream);
    flat_prescan(ix, p, &blocks, ix->stream);
    std::vector<uint32_t> flags(nq);
    std::vector<float> dv(nq * k);
    auto run = [&]() {
      hip_check(alaya_amd::launch_flat_scan(p, blocks, ix->stream), "flat scan");
      hip_check(alaya_amd::launch_flat_merge(p, ix->stream), "flat merge");
      hip_check(hipMemcpyAsync(ids, ix->id_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
      hip_check(hipMemcpyAsync(dv.data(), ix->dist_buf.ptr, nq * k * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
      hip_check(hipMemcpyAsync(flags.data(), ix->flag_buf.ptr, nq * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
      hip_check(hipStreamSynchronize(ix->stream), "flat search");
    };
    run();
    if (p.single) {
      // the single pass's bound is ~8x the split's: on data whose 10th and 32nd distances are that
      // close, more than 1 % of the queries flagged reruns the launch with the bf16 hi/lo split
      // before any exhaustive redo
      uint64_t nflag = 0;
      for (uint64_t q = 0; q < nq; ++q) nflag += flags[q] ? 1 : 0;
      if (nflag * 100 > nq) {
        p = flat_params(ix, ix->q_buf.as<float>(), nq, k, ix->id_buf.as<uint32_t>(), ix->dist_buf.as<float>(),
                        ix->flag_buf.as<uint32_t>(), &blocks, ix->stream, /*no_single=*/true);
        flat_prescan(ix, p, &blocks, ix->stream);
        run();
      }
    }
    scratch_release(ix, ix->stream);
    // queries whose shortlist bound did not hold: exhaustive exact distances on the device, over
    // the valid rows only (the scan never returns a row cleared in the validity bitmap)
    uint32_t redo = 0;
    std::vector<uint32_t> vbits;
    for (uint64_t q = 0; q < nq; ++q) {
      if (!flags[q]) continue;
      ++redo;
      if (!ix->iota.ptr || ix->iota.bytes < ix->n * 4) {
        std::vector<uint32_t> io(ix->n);
        for (uint64_t i = 0; i < ix->n; ++i) io[i] = static_cast<uint32_t>(i);
        ix->iota.reserve(ix->n * 4);
        hip_check(hipMemcpy(ix->iota.ptr, io.data(), ix->n * 4, hipMemcpyHostToDevice), "H2D");
      }
      if (ix->has_valid && vbits.empty()) {
        vbits.assign((ix->n + 31) / 32, 0u);
        hip_check(hipMemcpy(vbits.data(), ix->valid.ptr, vbits.size() * 4, hipMemcpyDeviceToHost), "D2H");
      }
      ix->dout_buf.reserve(ix->n * 4);
      SearchParams sp = base_params(ix);
      sp.queries = ix->q_buf.as<float>() + q * ix->dim;
      sp.q_stride = ix->dim;
      hip_check(alaya_amd::launch_row_distances(sp, ix->iota.as<uint32_t>(), static_cast<uint32_t>(ix->n), 1,
                                                ix->dout_buf.as<float>(), ix->stream), "exhaustive");
      std::vector<float> all(ix->n);
      hip_check(hipMemcpyAsync(all.data(), ix->dout_buf.ptr, ix->n * 4, hipMemcpyDeviceToHost, ix->stream), "D2H");
      hip_check(hipStreamSynchronize(ix->stream), "exhaustive");
      std::vector<uint32_t> order;
      order.reserve(ix->n);
      for (uint64_t i = 0; i < ix->n; ++i)
        if (vbits.empty() || ((vbits[i >> 5] >> (i & 31)) & 1u)) order.push_back(static_cast<uint32_t>(i));
      const uint64_t kk = std::min<uint64_t>(k, order.size());
      std::partial_sort(order.begin(), order.begin() + kk, order.end(), [&](uint32_t a, uint32_t b) {
        return all[a] < all[b] || (all[a] == all[b] && a < b);
      });
      for (uint64_t j = 0; j < k; ++j) {  // slots past the valid rows: (0xffffffff, FLT_MAX), as the scan
        ids[q * k + j] = j < kk ? order[j] : 0xffffffffu;
        dv[q * k + j] = j < kk ? all[order[j]] : FLT_MAX;
      }
    }
    if (dists) std::memcpy(dists, dv.data(), nq * k * 4);
    if (n_recomputed) *n_recomputed = redo;
  });
}

int alaya_index_flat_last_contraction(const alaya_index *ix, int *contraction) {
  return guarded([&] {
    if (!ix || !contraction) throw ArgError("invalid arguments");
    *contraction = ix->flat_contraction;
  });
}

int alaya_index_set_hash_log2(alaya_index *ix, uint32_t log2_slots) {
  return guarded([&] {
    if (!ix) throw ArgError("null index");
    if (log2_slots != 0 && (log2_slots < 6 || log2_slots > 16)) throw ArgError("log2_slots must be 0 or 6..16");
    ix->hash_log2_override = log2_slots;
  });
}

int alaya_stream_create_reserving(int device, uint32_t reserved_cus, void **stream) {
  return guarded([&] {
    if (!stream) throw ArgError("null stream pointer");
    hip_check(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    const uint32_t n = static_cast<uint32_t>(prop.multiProcessorCount);
    if (reserved_cus >= n) throw ArgError("reserved_cus must leave at least one CU");
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (uint32_t c = 0; c < n; ++c) mask[c / 32] |= 1u << (c % 32);
    // The reserved CUs go one per XCD in turn.  Which XCD a CU-mask bit names is not documented
    // (the bits may interleave, CU i on XCD i mod X, or run in blocks, CU i on XCD i / (n / X)), so
    // reserved CU r is chosen on XCD r mod X under both numberings: c = x * (n / X) + ((x + X k) mod
    // (n / X)) with x = r mod X, k = r / X (c mod X = x when X divides n / X).  A CU already taken
    // (more than n / X reserved) moves to the next free one.
    int xcds = 1;
    if (hipDeviceGetAttribute(&xcds, hipDeviceAttributeNumberOfXccs, device) != hipSuccess || xcds < 1) {
      (void)hipGetLastError();
      xcds = 1;
    }
    const uint32_t X = static_cast<uint32_t>(xcds);
    const uint32_t per = (n % X == 0) ? n / X : n;  // CUs per XCD (1 block when X does not divide n)
    const uint32_t xs = (n % X == 0) ? X : 1u;
    for (uint32_t r = 0; r < reserved_cus; ++r) {
      const uint32_t x = r % xs, k = r / xs;
      uint32_t c = x * per + (x + xs * k) % per;
      while (!(mask[c / 32] & (1u << (c % 32)))) c = (c + 1) % n;  // reserved_cus < n: a free CU exists
      mask[c / 32] &= ~(1u << (c % 32));
    }
    hipStream_t s = nullptr;
    hip_check(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()),
              "hipExtStreamCreateWithCUMask");
    *stream = s;
  });
}

int alaya_stream_destroy(void *stream) {
  return guarded([&] {
    if (stream) hip_check(hipStreamDestroy(static_cast<hipStream_t>(stream)), "hipStreamDestroy");
  });
}

int alaya_index_last_launch(const alaya_index *ix, uint32_t *workgroups, uint32_t *waves_per_group) {
  return guarded([&] {
    if (!ix) throw ArgError("null index");
    if (workgroups) *workgroups = ix->last_grid;
    if (waves_per_group) *waves_per_group = ix->last_waves;
  });
}

int alaya_index_set_helpers(alaya_index *ix, int mode) {
  return guarded([&] {
    if (!ix) throw ArgError("null index");
    if (mode < -1 || mode > 1) throw ArgError("helpers mode must be -1 (automatic), 0 (off) or 1 (on)");
    ix->helpers_mode = mode;
  });
}

int alaya_index_help_stats(alaya_index *ix, uint64_t *memo_dists, uint64_t *memo_expansions, uint64_t *helper_rows) {
  return guarded_scratch(ix, [&] {
    if (!ix) throw ArgError("null index");
    uint64_t m = 0, x = 0, r = 0;
    if (ix->help_stats_slots) {
      set_device(ix);
      scratch_drain(ix);
      std::vector<uint32_t> h(3 * ix->help_stats_slots);
      hip_check(hipMemcpy(h.data(), ix->help_stats.ptr, h.size() * 4, hipMemcpyDeviceToHost), "D2H");
      for (uint64_t i = 0; i < ix->help_stats_slots; ++i) {
        m += h[3 * i];
        x += h[3 * i + 1];
        r += h[3 * i + 2];
      }
    }
    if (memo_dists) *memo_dists = m;
    if (memo_expansions) *memo_expansions = x;
    if (helper_rows) *helper_rows = r;
  });
}

int alaya_index_set_visited_mode(alaya_index *ix, int mode) {
  return guarded([&] {
    if (!ix) throw ArgError("null index");
    if (mode < 0 || mode > 3) throw ArgError("visited mode must be 0 (auto), 1 (compact), 2 (wide) or 3 (test)");
    ix->visited_mode_override = mode;
  });
}

int alaya_index_info(const alaya_index *ix, uint64_t *n, uint32_t *dim, uint32_t *stride,
                     int *metric, uint64_t *device_bytes) {
  return guarded([&] {
    if (!ix) throw ArgError("null index");
    if (n) *n = ix->n;
    if (dim) *dim = ix->dim;
    if (stride) *stride = ix->stride;
    if (metric) *metric = ix->metric;
    if (device_bytes) *device_bytes = ix->device_bytes();
  });
}

}  // extern "C"
