/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement ("oracle") of the AlayaLite HNSW search hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * The product (alayalite_amd/) never links, imports or calls anything under oracle/.
 *
 * Every function restates a reference routine (paths relative to the reference repo root):
 *   orc_l2_f32 / orc_ip_f32         include/simd/distance_l2.ipp:54-116 (l2_sqr_avx2, chosen by
 *                                   get_l2_sqr_func :678-692 on every AVX2/AVX-512 host) and
 *                                   include/simd/distance_ip.ipp:56-111 (ip_sqr_avx2, :687-700)
 *   orc_l2_generic / orc_ip_generic non-float branch of l2_sqr<T>/ip_sqr<T>
 *                                   (distance_l2.ipp:735-741, distance_ip.ipp:744-750)
 *   orc_normalize                   include/utils/data_utils.hpp:36-46
 *   orc_pool_*                      LinearPool, include/utils/query_utils.hpp:236-312
 *   orc_search                      GraphSearchJob::search_solo, graph_search_job.hpp:302-371,
 *                                   with Graph::initialize_search graph.hpp:148-158 and
 *                                   OverlayGraph::initialize overlay_graph.hpp:122-144
 *   orc_batch_search_coro           PyIndex::batch_search python/include/index.hpp:289-336 driving
 *                                   GraphSearchJob::search (coroutine) graph_search_job.hpp:221-299
 *                                   on the Scheduler/Worker runtime (executor/scheduler.hpp:113-203,
 *                                   executor/worker.hpp:111-136, 4 local tasks per worker)
 *   orc_updater_*                   GraphUpdateJob insert_and_update / update / remove
 *                                   (executor/jobs/graph_update_job.hpp:49-137) with JobContext
 *                                   (job_context.hpp:25-29), Graph/RawSpace insert + remove
 *   orc_hnsw_*                      HNSWBuilder::build_graph, one thread (oracle_build.cpp:
 *                                   hnsw_builder.hpp:98-194, hnswlib.hpp:87-751)
 *   orc_sq8_*                       SQ8Quantizer (space/quant/sq8.hpp:99-143) and the AVX-512 /
 *                                   AVX2 SQ8 kernels (distance_l2.ipp:244-408, distance_ip.ipp:198-366)
 *
 * Parity status: pinned by the reference's own known-answer tests (tests/space/raw_space_test.cpp,
 * tests/space/sq8_space_test.cpp, tests/simd/l2_sqr_test.cpp, tests/utils/query_utils_test.cpp) --
 * see tests/test_oracle.py.  The reference binary itself cannot be run here.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* metric codes (match include/utils/metric_type.hpp: L2=0, IP=1, COS=2) */
enum { ORC_L2 = 0, ORC_IP = 1, ORC_COS = 2 };

/* ---- distances --------------------------------------------------------------------------- */
float orc_l2_f32(const float *x, const float *y, size_t dim);        /* portable, exact AVX2 order */
float orc_ip_f32(const float *x, const float *y, size_t dim);        /* returns -<x,y>            */
float orc_l2_f32_avx2(const float *x, const float *y, size_t dim);   /* intrinsics, same order    */
float orc_ip_f32_avx2(const float *x, const float *y, size_t dim);
/* generic (non-float DataType) scalar branch; dtype: 0=f32 1=i8 2=u8 3=f64 4=i32 5=u32 */
float orc_l2_generic(const void *x, const void *y, size_t dim, int dtype);
float orc_ip_generic(const void *x, const void *y, size_t dim, int dtype);
void orc_normalize(float *v, size_t dim);
int orc_cpu_has_avx2_fma(void);
int orc_cpu_has_avx512f(void);

/* ---- LinearPool (opaque, float distances, uint32 ids) ------------------------------------- */
typedef struct orc_pool orc_pool;
orc_pool *orc_pool_new(uint32_t n, int capacity);
void orc_pool_free(orc_pool *p);
int orc_pool_insert(orc_pool *p, uint32_t id, float dist);
uint32_t orc_pool_pop(orc_pool *p);
uint32_t orc_pool_top(orc_pool *p);
int orc_pool_has_next(const orc_pool *p);
size_t orc_pool_size(const orc_pool *p);
uint32_t orc_pool_id(const orc_pool *p, size_t i);
float orc_pool_dist(const orc_pool *p, size_t i);

/* ---- graph + space view ------------------------------------------------------------------- */
typedef struct {
  const float *base;          /* n rows, row stride `stride` floats                            */
  uint64_t n;                 /* get_data_num()                                                 */
  uint32_t dim;
  uint32_t stride;
  const uint8_t *valid;       /* SequentialStorage bitmap, bit (i%8) of byte i/8; NULL=all valid*/
  int metric;                 /* ORC_L2 / ORC_IP / ORC_COS (COS: data already normalised)      */
  const uint32_t *l0;         /* n x R level-0 adjacency, -1 padded                            */
  uint32_t R;
  const uint32_t *levels;     /* NULL => no overlay (NSG-style eps)                             */
  const uint64_t *upper_off;  /* node u, level l: upper_edges[upper_off[u] + (l-1)*upper_R ...] */
  const uint32_t *upper_edges;
  uint32_t upper_R;
  uint32_t ep;
  /* SQ8 search space (SQ8Space, space/sq8_space.hpp:255-298); used when space == 1 */
  int space;                  /* 0 = RawSpace (f32 rows), 1 = SQ8Space                          */
  const uint8_t *codes;       /* n rows of code_stride bytes                                    */
  uint32_t code_stride;
  const float *sq_min, *sq_max;
  int sq8_variant;            /* 0 generic, 1 AVX2, 2 AVX-512 (get_*_sq8_func host choice)       */
  int generic;                /* 1: non-float DataType -- the rows (cast to float) are compared with
                                 the generic branch of l2_sqr<T>/ip_sqr<T> (distance_l2.ipp:735-741,
                                 distance_ip.ipp:744-750) instead of the AVX2 float kernel          */
} orc_index;

typedef struct {
  uint64_t n_dist;        /* level-0 QueryComputer calls                                        */
  uint64_t n_expand;      /* pool pops                                                          */
  uint64_t n_dist_upper;  /* distance calls during the overlay descent (incl. the entry point)  */
  uint64_t n_hops_upper;  /* adjacency lists scanned during the overlay descent                 */
} orc_counters;

/* One query (search_solo).  ids/dists must hold k entries; dists may be NULL. */
void orc_search(const orc_index *ix, const float *query, uint32_t k, uint32_t ef, uint32_t *ids,
                float *dists, orc_counters *cnt);

/* nq queries on num_threads workers running the coroutine restatement.  Returns the seconds
 * between Scheduler::begin and Scheduler::join (the region index.hpp:300,328 times). */
double orc_batch_search_coro(const orc_index *ix, const float *queries, uint64_t nq, uint32_t k,
                             uint32_t ef, uint32_t num_threads, uint32_t *ids, float *dists,
                             orc_counters *cnt);

/* PyIndex::rerank (python/include/index.hpp:450-488) as the Linux batch path calls it (:337-345):
 * src = the k ids search_job wrote into a zero-initialised ef-sized res_pool (so ef-k extra zeros),
 * rescored with the raw-space QueryComputer (metric on f32 rows of ix, FLT_MAX for invalid rows),
 * top-k by a min-heap on pair<dist, id>.  Writes k ids and their distances. */
void orc_rerank(const orc_index *ix, const float *query, const uint32_t *search_ids, uint32_t k,
                uint32_t ef, uint32_t *ids, float *dists);
/* The batch path's rerank loop (index.hpp:337-345), single-threaded over nq queries; returns seconds. */
double orc_batch_rerank(const orc_index *ix, const float *queries, uint64_t nq, const uint32_t *search_ids,
                        uint32_t k, uint32_t ef, uint32_t *ids, float *dists);

/* ---- online updates ------------------------------------------------------------------------
 * An updater copies the index (rows, l0, validity, overlay) into growable storage with room for
 * `capacity` nodes; insert = insert_and_update (search_solo for R ids at ef, append, update every
 * node that gained an edge), returns the new id or -1 when full; remove = GraphUpdateJob::remove.
 * orc_updater_view() is the current index (pointers change after an insert). */
typedef struct orc_updater orc_updater;
orc_updater *orc_updater_new(const orc_index *ix, uint64_t capacity);
void orc_updater_free(orc_updater *u);
const orc_index *orc_updater_view(orc_updater *u);
int64_t orc_updater_insert(orc_updater *u, const float *search_query, const float *row, uint32_t ef);
void orc_updater_remove(orc_updater *u, uint32_t id);

/* ---- HNSW construction (oracle_build.cpp) ------------------------------------------------------
 * HNSWBuilder::build_graph with one thread (hnsw_builder.hpp:98-194 over hnswlib.hpp:87-751):
 * M = R/2, M0 = R, ef = max(ef_construction, M), levels from default_random_engine(seed).
 * export: l0[n*R] (-1 padded), levels[n], upper_off[n], upper_edges[upper_slots] (R per level,
 * -1 padded), ep.  generic = 1: the non-float DataType distance branch. */
typedef struct orc_hnsw orc_hnsw;
orc_hnsw *orc_hnsw_build(const float *rows, uint64_t n, uint32_t dim, int metric, int generic, uint32_t R,
                         uint32_t ef_construction, uint64_t seed);
uint64_t orc_hnsw_upper_slots(const orc_hnsw *o);
void orc_hnsw_export(const orc_hnsw *o, uint32_t *l0, uint32_t *levels, uint64_t *upper_off,
                     uint32_t *upper_edges, uint32_t *ep);
void orc_hnsw_free(orc_hnsw *o);

/* ---- SQ8 ---------------------------------------------------------------------------------- */
/* find_exact_gt (include/utils/evaluate.hpp:29-62): per query, l2_sqr to every row, std::sort of
 * (id, dist) by dist, the first k ids.  Queries split over num_threads threads (the reference loops
 * them on one thread).  Returns the seconds spent (CPU baseline of the flat path, config 2). */
double orc_exact_gt(const float *base, uint64_t n, uint32_t dim, const float *queries, uint64_t nq,
                    uint32_t k, uint32_t num_threads, uint32_t *ids);
void orc_sq8_fit(const float *data, uint64_t n, uint32_t dim, float *min_v, float *max_v);
void orc_sq8_encode(const float *row, uint32_t dim, const float *min_v, const float *max_v,
                    uint8_t *code);
/* variant: 0 = generic, 1 = AVX2 order, 2 = AVX-512 order (GCC 11 _mm512_reduce_add_ps tree) */
float orc_sq8_l2(const uint8_t *x, const uint8_t *y, size_t dim, const float *min_v,
                 const float *max_v, int variant);
float orc_sq8_ip(const uint8_t *x, const uint8_t *y, size_t dim, const float *min_v,
                 const float *max_v, int variant);

#ifdef __cplusplus
}
#endif
