// Flat (exhaustive) exact k-NN: MFMA shortlist + exact rescoring (flat_kernels.hip).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace alaya_amd {

struct FlatParams {
  const float *base;   // n x stride f32 rows (zero padded)
  uint64_t n;
  uint32_t dim;
  uint32_t stride;     // multiple of 32
  const float *norms;  // |b|^2 per row
  const uint32_t *valid;  // validity bitmap (bit i of word i/32), nullable = all rows valid;
                          // removed / invalid rows are never returned
  float max_norm;      // max |b|
  const float *queries;   // wide scan (flat_slab(stride) != 0): nq x flat_query_width(stride), zero padded
  uint64_t nq;
  uint32_t q_stride;
  uint32_t k_acc;         // columns the scan accumulates over (stride, or the padded width)
  int n_chunks;        // base chunks (multiple of 8)
  float *cand_d;       // n_chunks x nq x shortlist approximate distances
  uint32_t *cand_i;
  uint32_t k;
  uint32_t *out_ids;   // nq x k
  float *out_dists;    // nq x k, nullable
  uint32_t *flags;     // nq: 1 = shortlist bound not proven, recompute exhaustively
  uint32_t row_step;   // scan rows 0, row_step, 2*row_step, ... (n counts scanned rows); 1 = all
  const float *tau_init;  // nq per-query starting thresholds (nullable = FLT_MAX): the prescan's
                          // 32nd-best over a row sample, nudged up one ulp (see flat_kernels.hip)
  float *tau_out;      // threshold kernel output (nq)
  int split;           // 1 = bf16 hi/lo split contraction (3 bf16 MFMAs), 0 = f32 MFMA (or single)
  int single;          // 1 = single-pass f16 contraction (warp-specialised narrow scan only): rows scaled
                       // by 2^base_exp, each query by its own power of two (flat_kernels.hip)
  int base_exp;        // single pass: s with max|b| 2^s < 2^15 (flat_base_exp(max_norm))
  int ablate;          // diagnostics only: 1 = skip candidate handling (MFMA + tile stream only)
  uint32_t *merge_count;  // diagnostics only (nullable): merges per block
  uint32_t spin_limit; // warp-specialised scan: LDS-flag polls before a block aborts (its queries are
                       // then flagged for the exhaustive redo); 1 << 20 unless ALAYA_FLAT_SPIN_LIMIT
  const unsigned char *tiles;  // single-role f16 scan (non-null selects it): the base's tile records
                               // (launch_flat_tiles), rows already scaled by 2^base_exp
  uint64_t n_scan_tiles;       // records the scan visits: 0, tile_step, 2 tile_step, ... (split over the chunks)
  uint32_t tile_step;          // 1 = every record; the prescan's sample takes every tile_step-th
  uint64_t *tiles_buf;         // its candidate buffers: blocks x flat_tiles_queries() x flat_tiles_buf() entries
  int *tiles_qexp;             // its scale exponent t per query (one per wave of 32 queries), for the merge's bound
};

int flat_shortlist();
// whether the warp-specialised narrow scan runs (not the diagnostics' single-role kernel)
bool flat_ws_available(int ablate);
// the single pass's row scale exponent s for rows of largest norm max_norm (max|b| 2^s < 2^15)
int flat_base_exp(float max_norm);
// largest k of the flat path (merged list of 256 with a margin of 32)
int flat_max_k();
// slab width of the wide scan for rows of `stride` floats (0: the narrow kernel, stride <= 224)
uint32_t flat_slab(uint32_t stride);
uint32_t flat_query_width(uint32_t stride);
size_t flat_scan_lds(uint32_t stride);
hipError_t launch_pad_queries(const float *src, uint64_t nq, uint32_t dim, uint32_t width, float *dst,
                              hipStream_t s);
hipError_t launch_row_norms(const float *base, uint64_t n, uint32_t stride, float *norms, hipStream_t s);
hipError_t launch_flat_scan(const FlatParams &p, int blocks, hipStream_t s);
// Tile records of the single-role f16 scan for rows of `stride` floats: bytes for n rows (0: that
// scan does not cover this stride); built from the f32 rows, their |b|^2 and the validity bitmap
size_t flat_tiles_bytes(uint32_t stride, uint64_t n);
hipError_t launch_flat_tiles(const float *base, uint64_t n, uint32_t stride, const float *norms, const uint32_t *valid,
                             int base_exp, unsigned char *out, hipStream_t s);
// queries per block of the single-role f16 scan, and candidate buffer entries per query
int flat_tiles_queries();
int flat_tiles_buf();
hipError_t launch_flat_merge(const FlatParams &p, hipStream_t s);
hipError_t launch_flat_threshold(const FlatParams &p, hipStream_t s);

}  // namespace alaya_amd
