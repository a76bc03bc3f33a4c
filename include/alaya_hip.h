/*
 * alaya_hip.h -- C ABI of the MI355X search engine (libalaya_hip.so).
 *
 * This is the drop-in boundary for AlayaLite's search hot path.  Plain pointers and sizes only;
 * every call returns an int status (ALAYA_OK == 0) and alaya_last_error() gives the message of
 * the last failure on the calling thread.  Host buffers are copied; *_device variants take device
 * pointers and a hipStream_t (passed as void*) and are asynchronous on that stream.
 *
 * Streams: an index keeps per-index scratch (work counter, visited-set spill area, flat and SQ8
 * candidate buffers).  Every launching call orders itself after the previous launching call on the
 * index (a hipStreamWaitEvent when the streams differ), so calls on different streams serialise on
 * the device instead of racing; calls that replace device buffers (set_base, set_graph, set_sq8,
 * build_graph, reserve, enable_updates, destroy) first wait for those launches to finish.  Calls on
 * one index from several host threads are serialised by the index's lock.
 *
 * Reference interfaces each group replaces (paths relative to the AlayaLite repo root):
 *   alaya_index_*            PyIndex<HNSWBuilder<RawSpace>, Space> state and lifetime
 *                            (python/include/index.hpp:85-506, PyIndexInterface :508-587)
 *   alaya_index_set_base     RawSpace ctor/fit + SequentialStorage (include/space/raw_space.hpp:81-140,
 *                            include/storage/sequential_storage.hpp:53-84) -- rows moved to HBM
 *   alaya_index_set_graph    Graph + OverlayGraph (include/index/graph/graph.hpp:44-158,
 *                            overlay_graph.hpp:26-144) -- adjacency moved to HBM
 *   alaya_index_batch_search PyIndex::batch_search / batch_search_with_distance
 *                            (python/include/index.hpp:289-451) -> GraphSearchJob::search
 *                            (include/executor/jobs/graph_search_job.hpp:221-299) on the device
 *   alaya_index_search       PyIndex::search (index.hpp:236-258) -> search_solo (:302-371)
 *   alaya_index_distances    RawSpace::QueryComputer::operator() (raw_space.hpp:297-304) over
 *                            simd::l2_sqr / ip_sqr (include/simd/distance_l2.ipp:729-742,
 *                            distance_ip.ipp:739-751) -- the metric plugin surface
 *                            (include/space/space_concepts.hpp:31-73)
 *   alaya_graph_*            HNSWBuilder::build_graph (include/index/graph/hnsw/hnsw_builder.hpp:98-194)
 *                            and Graph::save/load (graph.hpp:165-238)
 */
#ifndef ALAYA_HIP_H_
#define ALAYA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ALAYA_OK 0
#define ALAYA_ERR_ARG 1      /* invalid argument (Python: ValueError)            */
#define ALAYA_ERR_RUNTIME 2  /* runtime failure (Python: RuntimeError)           */
#define ALAYA_ERR_DEVICE 3   /* HIP error / no device (Python: RuntimeError)     */

/* MetricType values of include/utils/metric_type.hpp */
#define ALAYA_METRIC_L2 0
#define ALAYA_METRIC_IP 1
#define ALAYA_METRIC_COS 2
/* OR-ed into the metric of alaya_index_set_base / alaya_graph_build_hnsw: the rows are a non-float
 * DataType (int8, uint8, int32, uint32, double) cast to float, and distances follow the generic
 * branch of l2_sqr<T> / ip_sqr<T> (include/simd/distance_l2.ipp:735-741, distance_ip.ipp:744-750:
 * one float accumulator over the elements in order) instead of the AVX2 float kernel. */
#define ALAYA_DIST_GENERIC 0x100

typedef struct alaya_index alaya_index;
typedef struct alaya_graph alaya_graph;

const char *alaya_last_error(void);
/* Build provenance (no reference counterpart): "source=<16 hex digits of sha256 over the library's
 * sources and headers> arch=gfx950 hipcc=<compiler> built=<UTC time>", fixed when the library was
 * compiled (alayalite_amd/_build.py).  bench.py and smoke() compare the source hash with the tree. */
const char *alaya_build_info(void);
/* Number of visible HIP devices (0 when none). */
int alaya_device_count(int *count);
/* Roofline calibration (no reference counterpart): the best of `iters` streaming reads of a
 * `bytes`-byte device buffer (>= 1 MiB) over three load shapes and two occupancies, in GB/s -- the
 * measured bandwidth ceiling bench.py reports beside the 8 TB/s HBM3E figure. */
int alaya_hbm_stream_read(int device, uint64_t bytes, int iters, double *gbs);
/* A HIP stream whose launches may use every CU of `device` but `reserved_cus` (spread over the CU
 * numbering), so kernels of other streams -- the shard exchange's RCCL all_gather -- find free CUs
 * while a persistent search runs; searches launched on it size their grid to the CUs left.  No
 * reference counterpart (the reference is single-process CPU code). */
int alaya_stream_create_reserving(int device, uint32_t reserved_cus, void **stream);
int alaya_stream_destroy(void *stream);

/* ---- host graph (builder + reference on-disk format) --------------------------------------- */
/* data: n x dim float32 row-major (normalised already for COS).  seed 100 = reference default. */
int alaya_graph_build_hnsw(const float *data, uint64_t n, uint32_t dim, int metric, uint32_t R,
                           uint32_t ef_construction, uint32_t num_threads, uint64_t seed,
                           alaya_graph **out);
int alaya_graph_load(const char *path, int id_bytes, alaya_graph **out);
/* valid_bitmap (nullable): the graph storage bitmap, ceil(n/8) bytes; a node removed with
 * GraphUpdateJob::remove has its bit cleared in the reference's file (sequential_storage.hpp:94-100). */
int alaya_graph_save(const alaya_graph *g, const char *path, int id_bytes, uint64_t capacity,
                     const uint8_t *valid_bitmap);
/* sizes: n, R, has_overlay, upper_R, ep, max_level, n_upper_edges, n_eps */
int alaya_graph_info(const alaya_graph *g, uint64_t *n, uint32_t *R, int *has_overlay,
                     uint32_t *upper_R, uint32_t *ep, uint32_t *max_level,
                     uint64_t *n_upper_edges, uint32_t *n_eps);
/* copy out: l0[n*R], levels[n], upper_off[n], upper_edges[n_upper_edges], eps[n_eps]; any NULL skipped */
int alaya_graph_export(const alaya_graph *g, uint32_t *l0, uint32_t *levels, uint64_t *upper_off,
                       uint32_t *upper_edges, uint32_t *eps);
/* build a graph object from host arrays (levels == NULL -> NSG-style eps) */
int alaya_graph_import(uint64_t n, uint32_t R, const uint32_t *l0, const uint32_t *levels,
                       const uint64_t *upper_off, const uint32_t *upper_edges,
                       uint64_t n_upper_edges, uint32_t upper_R, uint32_t ep, const uint32_t *eps,
                       uint32_t n_eps, alaya_graph **out);
void alaya_graph_free(alaya_graph *g);

/* ---- device index ---------------------------------------------------------------------------- */
int alaya_index_create(int device, alaya_index **out);
void alaya_index_destroy(alaya_index *ix);
/* rows: n x dim float32 host array (row pitch dim).  valid_bitmap: ceil(n/8) bytes in the
 * SequentialStorage layout (bit i%8 of byte i/8 set = valid) or NULL for all valid. */
int alaya_index_set_base(alaya_index *ix, const float *rows, uint64_t n, uint32_t dim, int metric,
                         const uint8_t *valid_bitmap);
int alaya_index_set_graph(alaya_index *ix, const alaya_graph *g);
/* Batched search on host buffers.  ids: nq x k; dists (nullable): nq x k; counters (nullable):
 * nq x 4 uint32 = (n_dist, n_expand, n_dist_upper, n_hops_upper). */
int alaya_index_batch_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                             uint32_t ef, uint32_t *ids, float *dists, uint32_t *counters);
/* Same on device buffers, asynchronous on `stream` (hipStream_t; NULL = default stream). */
int alaya_index_batch_search_device(alaya_index *ix, const float *d_queries, uint64_t nq,
                                    uint32_t k, uint32_t ef, uint32_t *d_ids, float *d_dists,
                                    uint32_t *d_counters, void *stream);
/* The per-shard search of a base-range sharded index (no reference counterpart): as
 * alaya_index_batch_search_device, except that result slots past the pool (shard rows < k, or
 * ef < k) hold (0xffffffff, FLT_MAX) instead of the reference's (0, 0.0), so they sort after every
 * real candidate in the cross-shard merge.  d_dists is required. */
int alaya_index_shard_search_device(alaya_index *ix, const float *d_queries, uint64_t nq, uint32_t k,
                                    uint32_t ef, uint32_t *d_ids, float *d_dists, uint32_t *d_counters,
                                    void *stream);
/* ---- device graph construction (Index.fit on the MI355X) ------------------------------------
 * Replaces HNSWBuilder::build_graph (include/index/graph/hnsw/hnsw_builder.hpp:98-194) over hnswlib
 * add_point (include/index/graph/hnsw/hnswlib.hpp:652-751), from the index's own rows
 * (alaya_index_set_base; COS rows already normalised).  M = R/2, M0 = R, ef = max(ef_construction,
 * M), levels drawn exactly as the reference draws them from `seed` (100 in the reference).  Points
 * are inserted in label order in batches of max(1, min(max_batch, inserted / batch_div)) (0 ->
 * defaults 16 / 65536); within a batch every point runs searchBaseLayer + the neighbour heuristic
 * on the device against the graph as it stood before the batch, then reverse edges are merged per
 * destination (append, or prune with the heuristic).  `refine` extra level-0 passes per batch let
 * the batch's points re-select among each other once they are linked in (2 recommended; with
 * batch_div = max_batch = 1 and refine = 0 the insertion is sequential, as the reference's).  The result is installed as the index's
 * search graph and a host copy is returned in *out (nullable).  stats (nullable, 8 x u64):
 * batches, kernel launches, list prunes, appended edges, heuristic distances, device time (us),
 * largest batch, max level. */
int alaya_index_build_graph(alaya_index *ix, uint32_t R, uint32_t ef_construction, uint64_t seed,
                            uint32_t batch_div, uint32_t max_batch, uint32_t refine, alaya_graph **out,
                            uint64_t *stats);
/* ---- online updates (Index.insert / Index.remove) ------------------------------------------
 * Device-mirror primitives, for a host that keeps its own graph and update job (the reference's
 * GraphUpdateJob, include/executor/jobs/graph_update_job.hpp:49-137) and patches HBM after each
 * change:  reserve capacity (rows, validity, adjacency; contents kept), write rows at [first,
 * first+count), overwrite level-0 adjacency rows, set or clear a validity bit
 * (SequentialStorage::insert/remove, sequential_storage.hpp:77-100). */
int alaya_index_reserve(alaya_index *ix, uint64_t capacity);
int alaya_index_write_rows(alaya_index *ix, uint64_t first, const float *rows, uint64_t count);
int alaya_index_write_edges(alaya_index *ix, const uint32_t *ids, const uint32_t *edges, uint64_t count);
int alaya_index_set_valid(alaya_index *ix, uint64_t id, int valid);
/* Or let the engine run the update job: enable_updates copies the graph, rows and bitmap into a
 * host mirror (capacity = the index capacity, IndexParams.capacity_).  insert = PyIndex::insert ->
 * insert_and_update (graph_update_job.hpp:65-89): search_solo for R neighbours at ef on the device,
 * append the node, update() every node that gained an edge, patch HBM.  search_query is the query
 * as search_solo sees it and row the vector as RawSpace::insert stores it (they differ only for COS,
 * which normalises at both steps).  new_id = UINT64_MAX when the index is full.  remove =
 * GraphUpdateJob::remove (:91-103): record the node's edges, clear its validity bit.  export_*
 * return the mirror (for save). */
int alaya_index_enable_updates(alaya_index *ix, const alaya_graph *g, const float *rows, uint64_t n,
                               uint64_t capacity, const uint8_t *valid_bitmap);
int alaya_index_insert(alaya_index *ix, const float *search_query, const float *row, uint32_t ef,
                       uint64_t *new_id);
int alaya_index_remove(alaya_index *ix, uint64_t id);
int alaya_index_export_graph(alaya_index *ix, alaya_graph **out);
/* rows: n x dim (nullable), valid_bitmap: (n+7)/8 bytes (nullable); *n = stored rows. */
int alaya_index_export_rows(alaya_index *ix, float *rows, uint8_t *valid_bitmap, uint64_t *n);
/* out[q*n + i] = metric distance(queries[q], row ids[i]), bit-exact with the search kernel. */
int alaya_index_distances(alaya_index *ix, const float *queries, uint64_t nq, const uint32_t *ids,
                          uint32_t n, float *out);
/* Diagnostic build of the search kernel: also returns per-query s_memtime cycles per phase,
 * stamps[nq*8] = (init+descent, pop, adjacency+visited, distances, merge, expansions after the
 * visited table spilled, whole query, adjacency-prefetch hits).  space 0 = f32 rows (same ids as
 * alaya_index_batch_search), 1 = the SQ8 codes (no rerank; d = 768 is stamped, others run plain). */
int alaya_index_profile_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                               uint32_t ef, int space, uint32_t *ids, uint32_t *counters, uint64_t *stamps);
/* ---- SQ8 search space (SQ8Space: include/space/sq8_space.hpp, quant/sq8.hpp) --------------------
 * Per-dimension min/max (SQ8Quantizer::fit, sq8.hpp:99-113) and codes (quantize, :118-130). */
int alaya_sq8_train(const float *data, uint64_t n, uint32_t dim, float *min_v, float *max_v);
int alaya_sq8_encode(const float *data, uint64_t n, uint32_t dim, const float *min_v,
                     const float *max_v, uint8_t *codes, uint32_t num_threads);
/* Attach SQ8 codes (n x dim) to an index whose f32 rows are set.  order: the reduction order of
 * the reference kernel the host would pick -- 2 = l2/ip_sqr_sq8_avx512 (AVX-512F hosts),
 * 1 = the AVX2 variants (distance_l2.ipp:694-708, distance_ip.ipp:703-716). */
int alaya_index_set_sq8(alaya_index *ix, const uint8_t *codes, uint64_t n, uint32_t dim,
                        const float *min_v, const float *max_v, int order);
/* PyIndex::batch_search with SearchSpace = SQ8Space (index.hpp:289-346): graph search on the SQ8
 * codes (queries encoded in-kernel), then a rerank on the f32 rows with rerank_queries (NULL =
 * queries).  rerank: 0 = none (the SQ8 ids and distances), 1 = PyIndex::rerank as the reference
 * runs it, including its ef-k zero entries (index.hpp:450-488), 2 = corrected: the whole ef pool
 * is rescored (no id-0 duplicates); result slots beyond the candidates hold (0, 0.0). */
int alaya_index_batch_search_sq8(alaya_index *ix, const float *queries, const float *rerank_queries,
                                 uint64_t nq, uint32_t k, uint32_t ef, int rerank, uint32_t *ids,
                                 float *dists, uint32_t *counters);
/* Same on device buffers, asynchronous on `stream`; d_rerank_queries NULL = d_queries. */
int alaya_index_batch_search_sq8_device(alaya_index *ix, const float *d_queries, const float *d_rerank_queries,
                                        uint64_t nq, uint32_t k, uint32_t ef, int rerank, uint32_t *d_ids,
                                        float *d_dists, uint32_t *d_counters, void *stream);
/* The per-shard search of a base-range sharded SQ8 index (no reference
 * counterpart): the SQ8 graph search plus PyIndex::rerank (index.hpp:337-345, 450-488) on this
 * shard's rows.  The reference's id-0 quirk (the ef - k zero-filled res_pool slots, :301, rescored
 * as row 0) belongs to global row 0 only: with holds_row0 != 0 (the shard whose local row 0 is
 * global row 0) the rerank is exactly alaya_index_batch_search_sq8_device's rerank = 1; otherwise
 * only the k search ids are rescored.  Result slots without a candidate hold (0xffffffff, FLT_MAX),
 * so they sort after every real candidate in the cross-shard merge.  With one shard the merged
 * result equals the reference's batch_search.  d_dists is required. */
int alaya_index_shard_search_sq8_device(alaya_index *ix, const float *d_queries, const float *d_rerank_queries,
                                        uint64_t nq, uint32_t k, uint32_t ef, int holds_row0, uint32_t *d_ids,
                                        float *d_dists, uint32_t *d_counters, void *stream);
/* ---- flat (exhaustive) exact k-NN, L2, any dim, 1 <= k <= 224 -----------------------------------
 * No reference implementation (IndexType::FLAT is enum-only, include/index/index_type.hpp:28); the
 * analogue is find_exact_gt (include/utils/evaluate.hpp:29-62).  An MFMA pass ranks every row
 * by |b|^2 - 2 q.b and keeps a shortlist -- q.b from a single-pass f16 contraction on power-of-two
 * scaled operands (rows of <= 224 floats) or a bf16 hi/lo split (3 bf16 MFMAs; wider rows), each
 * error bounded and folded into the proof below (alaya_index_flat_last_contraction; environment
 * ALAYA_FLAT_CONTRACTION selects one, ALAYA_FLAT_F32=1 the f32 MFMA form); rows wider than 224
 * floats are scanned in K slabs.  The single-pass scan reads f16 tile records of the rows that the
 * index builds at its first flat search and keeps (K/16 KB + 256 B per 32 rows: 264.5 MB for
 * 1M x 128), rebuilding them after any change to the rows, their count or the validity bitmap;
 * a prescan over a sample of them seeds every query's threshold.  The shortlist (32 per row chunk,
 * folded into a 128/256-entry list for k > 24) is rescored with the exact device metric
 * (l2_sqr_avx2 order) and sorted by (distance, id).  A query whose shortlist cannot be proven to
 * hold the exact top-k (error bound in flat_kernels.hip) is flagged; the host API recomputes it
 * exhaustively and reports how many it did.  The device variant is asynchronous on `stream` and
 * only writes d_flags[q] = 1 for such a query (its d_ids row is then not proven exact): the caller
 * recomputes it, e.g. through alaya_index_flat_search. */
int alaya_index_flat_search(alaya_index *ix, const float *queries, uint64_t nq, uint32_t k,
                            uint32_t *ids, float *dists, uint32_t *n_recomputed);
int alaya_index_flat_search_device(alaya_index *ix, const float *d_queries, uint64_t nq, uint32_t k,
                                   uint32_t *d_ids, float *d_dists, uint32_t *d_flags, void *stream);
/* The contraction the last flat search ranked its shortlist with (introspection): 2 = single-pass f16
 * (the default for rows of <= 224 floats: one f16 MFMA per 16 k on operands scaled by powers of two,
 * error bound ~2^-10 |q||b|; the host API reruns a launch with the split if more than 1 % of its
 * queries are flagged), 1 = bf16 hi/lo split (3 bf16 MFMAs; wide rows and out-of-range scales),
 * 0 = f32 MFMA; -1 before any flat search.  Environment ALAYA_FLAT_CONTRACTION = f16 | bf16x3 | f32
 * selects one. */
int alaya_index_flat_last_contraction(const alaya_index *ix, int *contraction);
/* Tuning / introspection: LDS visited-table size (log2 slots, 6..16; 0 = automatic) and layout
 * (0 = automatic, 1 = compact 16-bit slots, 2 = 32-bit id slots, 3 = compact with probe distance
 * capped at 2, a test hook for the spill-on-long-probe path).  Results never depend on either:
 * the visited set is exact (DynamicBitset, include/utils/query_utils.hpp:69-115). */
int alaya_index_set_hash_log2(alaya_index *ix, uint32_t log2_slots);
int alaya_index_set_visited_mode(alaya_index *ix, int mode);
/* Distance helpers (-1 automatic, 0 off, 1 on; environment ALAYA_HELPERS overrides): a searcher
 * whose batch has no query left computes the distances of a sibling searcher's predicted next
 * expansion (same workgroup) into an LDS memo the sibling reads.  Replaces nothing in the reference:
 * its coroutine scheduler keeps every worker busy to the end of a batch
 * (include/executor/worker.hpp:47,111-136); results never depend on it (the searcher still does
 * every visit, merge and pop; memo distances are the same function of the same inputs).
 * alaya_index_help_stats: of the last search with helpers, how many of its fresh distances
 * (the n_dist counters) the searchers took from a memo, in how many expansions every fresh distance
 * came from it, and how many rows the helpers computed (waits for that search; 0 without helpers). */
int alaya_index_set_helpers(alaya_index *ix, int mode);
int alaya_index_help_stats(alaya_index *ix, uint64_t *memo_dists, uint64_t *memo_expansions,
                           uint64_t *helper_rows);
/* The last graph search's launch shape: persistent workgroups and searchers (waves) per workgroup --
 * workgroups x waves is the number of queries the launch runs at once (introspection). */
int alaya_index_last_launch(const alaya_index *ix, uint32_t *workgroups, uint32_t *waves_per_group);
int alaya_index_info(const alaya_index *ix, uint64_t *n, uint32_t *dim, uint32_t *stride,
                     int *metric, uint64_t *device_bytes);

#ifdef __cplusplus
}
#endif
#endif /* ALAYA_HIP_H_ */
