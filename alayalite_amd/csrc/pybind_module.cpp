// _alayalitepy: pybind11 module with the reference binding's surface (python/src/pybind.cpp:37-147)
// -- IndexType / MetricType / QuantizationType enums, IndexParams, PyIndexInterface -- implemented
// over the C ABI of libalaya_hip.so (include/alaya_hip.h).  All search work runs on the MI355X;
// there is no CPU search path: construction fails loudly when no HIP device is present.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <queue>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/alaya_hip.h"

extern "C" int alaya_index_flat_diag(alaya_index *, const float *, uint64_t, uint32_t, int, uint32_t *, float *,
                                     uint32_t *, uint32_t *, void *);
#include "host_distance.h"

namespace py = pybind11;

namespace alaya_py {

// include/index/index_type.hpp:27-33, include/utils/metric_type.hpp, quantization_type.hpp
enum class IndexType { FLAT = 0, HNSW = 1, NSG = 2, FUSION = 3, QG = 4 };
enum class MetricType { L2 = 0, IP = 1, COS = 2, NONE = 3 };
enum class QuantizationType { NONE = 0, SQ8 = 1, SQ4 = 2, RABITQ = 3 };

// python/include/params.hpp:29-52 (max_nbrs_ is not exposed by the reference binding either)
struct IndexParams {
  IndexType index_type_ = IndexType::HNSW;
  py::dtype data_type_ = py::dtype::of<float>();
  py::dtype id_type_ = py::dtype::of<uint32_t>();
  QuantizationType quantization_type_ = QuantizationType::NONE;
  MetricType metric_ = MetricType::L2;
  uint32_t capacity_ = 100000;
  uint32_t max_nbrs_ = 32;
};

void check(int rc) {
  if (rc == ALAYA_OK) return;
  const std::string msg = alaya_last_error();
  if (rc == ALAYA_ERR_ARG) throw py::value_error(msg);
  throw std::runtime_error(msg);
}

enum DType { kF32 = 0, kI8, kU8, kF64, kI32, kU32 };

DType dtype_code(const py::dtype &dt) {
  if (dt.is(py::dtype::of<float>())) return kF32;
  if (dt.is(py::dtype::of<int8_t>())) return kI8;
  if (dt.is(py::dtype::of<uint8_t>())) return kU8;
  if (dt.is(py::dtype::of<double>())) return kF64;
  if (dt.is(py::dtype::of<int32_t>())) return kI32;
  if (dt.is(py::dtype::of<uint32_t>())) return kU32;
  throw std::runtime_error("Unsupported data type");  // dispatch.hpp: "Unsupported data type"
}

size_t dtype_size(DType t) {
  switch (t) {
    case kF32: case kI32: case kU32: return 4;
    case kI8: case kU8: return 1;
    case kF64: return 8;
  }
  return 4;
}

// DataType -> float as the reference's generic l2_sqr<T>/ip_sqr<T> casts each element
// (distance_l2.ipp:735-741).  For float32 data this is the identity.
void to_float(const void *src, DType t, size_t count, float *dst) {
  switch (t) {
    case kF32: std::memcpy(dst, src, count * 4); break;
    case kI8: for (size_t i = 0; i < count; ++i) dst[i] = static_cast<const int8_t *>(src)[i]; break;
    case kU8: for (size_t i = 0; i < count; ++i) dst[i] = static_cast<const uint8_t *>(src)[i]; break;
    case kF64: for (size_t i = 0; i < count; ++i) dst[i] = static_cast<float>(static_cast<const double *>(src)[i]); break;
    case kI32: for (size_t i = 0; i < count; ++i) dst[i] = static_cast<float>(static_cast<const int32_t *>(src)[i]); break;
    case kU32: for (size_t i = 0; i < count; ++i) dst[i] = static_cast<float>(static_cast<const uint32_t *>(src)[i]); break;
  }
}

// get_l2_sqr_sq8_func / get_ip_sqr_sq8_func pick the AVX-512 kernel on AVX-512F hosts, else AVX2
// (distance_l2.ipp:694-708): the device reproduces the order this host's reference build uses.
int host_sq8_order() { return __builtin_cpu_supports("avx512f") ? 2 : 1; }

class PyIndexInterface {
 public:
  explicit PyIndexInterface(const IndexParams &params) : params_(params) {
    dtype_ = dtype_code(params_.data_type_);
    if (params_.id_type_.is(py::dtype::of<uint32_t>())) {
      id_bytes_ = 4;
    } else if (params_.id_type_.is(py::dtype::of<uint64_t>())) {
      id_bytes_ = 8;
    } else {
      throw std::runtime_error("Unsupported id type");
    }
    if (params_.quantization_type_ == QuantizationType::SQ4 ||
        params_.quantization_type_ == QuantizationType::RABITQ)
      throw std::runtime_error("quantization type not supported by the MI355X engine (SQ4/RaBitQ are out of scope)");
    if (params_.metric_ == MetricType::COS && dtype_ != kF32 && dtype_ != kF64) {
      throw std::runtime_error("COS metric only support float or double");  // raw_space.hpp:88-93
    }
    // SQ8 over a non-float DataType takes the reference's generic SQ8 branch (distance_l2.ipp:750-763,
    // quantize in double arithmetic for double data, sq8.hpp:118-130), which the device does not
    // implement: refuse rather than return different neighbours.
    if (params_.quantization_type_ == QuantizationType::SQ8 && dtype_ != kF32)
      throw std::runtime_error("SQ8 quantization of non-float32 data is not supported by the MI355X engine");
    check(alaya_index_create(0, &ix_));
  }
  ~PyIndexInterface() {
    if (graph_) alaya_graph_free(graph_);
    if (ix_) alaya_index_destroy(ix_);
  }
  PyIndexInterface(const PyIndexInterface &) = delete;
  PyIndexInterface &operator=(const PyIndexInterface &) = delete;

  std::string to_string() const { return "PyIndexInterface"; }

  // PyIndex::fit (index.hpp:177-227)
  // builder: "host" = HNSWBuilder restated on the host (num_threads == 1 reproduces the reference's
  // sequential graph exactly); "gpu" = batched insertion on the device (alaya_index_build_graph).
  void fit(py::array vectors, uint32_t ef_construction, uint32_t num_threads, const std::string &builder) {
    if (builder != "host" && builder != "gpu") throw py::value_error("builder must be 'host' or 'gpu'");
    if (vectors.ndim() != 2) throw std::runtime_error("Array must be 2D");
    check_dtype(vectors);
    py::array arr = py::array::ensure(vectors, py::array::c_style);
    const uint64_t n = arr.shape(0);
    dim_ = static_cast<uint32_t>(arr.shape(1));
    // RawSpace::fit silently stops storing past capacity (sequential_storage.hpp:77-80); the
    // builder (and the search bitset) still see n items.  Keep it defined: refuse instead.
    if (n > params_.capacity_) throw std::runtime_error("number of vectors exceeds the index capacity");
    // COS normalises the caller's rows in place (raw_space.hpp:131-140) -- done identically here.
    if (params_.metric_ == MetricType::COS) normalize_in_place(arr, n);
    raw_.assign(static_cast<const char *>(arr.data()),
                static_cast<const char *>(arr.data()) + n * dim_ * dtype_size(dtype_));
    n_ = n;
    delete_cnt_ = 0;
    valid_.clear();
    rows_f32_.resize(n * dim_);
    to_float(raw_.data(), dtype_, n * dim_, rows_f32_.data());
    if (graph_) alaya_graph_free(graph_);
    graph_ = nullptr;
    if (builder == "gpu") {
      {
        py::gil_scoped_release nogil;
        check(alaya_index_set_base(ix_, rows_f32_.data(), n, dim_, dist_code(), nullptr));
        check(alaya_index_build_graph(ix_, params_.max_nbrs_, ef_construction, 100, 0, 0, 2, &graph_, nullptr));
      }
      if (params_.quantization_type_ == QuantizationType::SQ8) {
        train_sq8(num_threads);
        check(alaya_index_set_sq8(ix_, sq_codes_.data(), n_, dim_, sq_min_.data(), sq_max_.data(), host_sq8_order()));
      }
      updates_enabled_ = false;
      graph_dirty_ = false;
      return;
    }
    {
      py::gil_scoped_release nogil;
      check(alaya_graph_build_hnsw(rows_f32_.data(), n, dim_, dist_code(), params_.max_nbrs_,
                                   ef_construction, num_threads, 100, &graph_));
    }
    if (params_.quantization_type_ == QuantizationType::SQ8) train_sq8(num_threads);
    upload();
  }

  py::array search(py::array query, uint32_t topk, uint32_t ef) {
    if (query.ndim() != 1) throw std::runtime_error("query must be 1D");
    py::array q2 = query.attr("reshape")(1, query.shape(0));
    auto r = run(q2, topk, ef, false);
    return r.first.attr("reshape")(topk);
  }

  py::array batch_search(py::array queries, uint32_t topk, uint32_t ef, uint32_t /*num_threads*/) {
    return run(queries, topk, ef, false).first;
  }

  py::object batch_search_with_distance(py::array queries, uint32_t topk, uint32_t ef,
                                        uint32_t /*num_threads*/) {
    auto r = run(queries, topk, ef, true);
    return py::make_tuple(r.first, r.second);
  }

  py::array get_data_by_id(uint32_t id) {
    if (n_ == 0) throw std::runtime_error("space is nullptr");
    if (id >= n_) throw std::runtime_error("id out of range");
    const size_t es = dtype_size(dtype_);
    py::array out(params_.data_type_, std::vector<py::ssize_t>{static_cast<py::ssize_t>(dim_)});
    std::memcpy(out.mutable_data(), raw_.data() + static_cast<size_t>(id) * dim_ * es, dim_ * es);
    return out;
  }

  // PyIndex::insert -> GraphUpdateJob::insert_and_update (index.hpp:229-232,
  // graph_update_job.hpp:65-89): device search_solo for R neighbours, host update job, HBM patch.
  py::object insert(py::array insert_data, uint32_t ef) {
    if (!graph_) throw std::runtime_error("Index is not init yet");
    if (params_.quantization_type_ != QuantizationType::NONE)
      throw std::runtime_error("insert on quantized indexes is not supported by the MI355X engine");
    check_dtype(insert_data);
    if (insert_data.ndim() != 1 || static_cast<uint32_t>(insert_data.shape(0)) != dim_)
      throw std::runtime_error("vector dimension mismatch");
    py::array arr = py::array::ensure(insert_data, py::array::c_style);
    ensure_updates();
    // COS: search_solo's QueryComputer normalises the caller's vector in place (raw_space.hpp:
    // 267-269), then RawSpace::insert normalises it again (:146-150).
    std::vector<float> q(dim_), row(dim_);
    if (params_.metric_ == MetricType::COS) normalize_in_place(arr, 1);
    to_float(arr.data(), dtype_, dim_, q.data());
    if (params_.metric_ == MetricType::COS) normalize_in_place(arr, 1);
    to_float(arr.data(), dtype_, dim_, row.data());
    uint64_t id = 0;
    {
      py::gil_scoped_release nogil;
      check(alaya_index_insert(ix_, q.data(), row.data(), ef, &id));
    }
    if (id == UINT64_MAX) return py::int_(id_bytes_ == 4 ? uint64_t{0xffffffffu} : UINT64_MAX);
    const size_t es = dtype_size(dtype_);
    raw_.insert(raw_.end(), static_cast<const char *>(arr.data()), static_cast<const char *>(arr.data()) + dim_ * es);
    rows_f32_.insert(rows_f32_.end(), row.begin(), row.end());
    n_ += 1;
    if (!valid_.empty()) {
      valid_.resize((n_ + 7) / 8, 0);
      valid_[id / 8] |= static_cast<uint8_t>(1u << (id % 8));
    }
    graph_dirty_ = true;
    return py::int_(id);
  }

  // PyIndex::remove -> GraphUpdateJob::remove (index.hpp:234, graph_update_job.hpp:91-103)
  void remove(uint32_t id) {
    if (!graph_) throw std::runtime_error("Index is not init yet");
    if (params_.quantization_type_ != QuantizationType::NONE)
      throw std::runtime_error("remove on quantized indexes is not supported by the MI355X engine");
    if (id >= n_) throw std::runtime_error("id out of range");
    ensure_updates();
    check(alaya_index_remove(ix_, id));
    if (valid_.empty()) {
      valid_.assign((n_ + 7) / 8, 0);
      for (uint64_t i = 0; i < n_; ++i) valid_[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
    }
    valid_[id / 8] &= static_cast<uint8_t>(~(1u << (id % 8)));
    delete_cnt_ += 1;  // RawSpace::remove counts every call (raw_space.hpp:160-163)
  }

  // PyIndex::save (index.hpp:113-130): graph file + raw data file (+ quant file)
  void save(const std::string &index_path, const std::string &data_path, const std::string &quant_path) {
    if (!graph_) throw std::runtime_error("index is not fitted");
    sync_graph();
    check(alaya_graph_save(graph_, index_path.c_str(), id_bytes_, std::max<uint64_t>(params_.capacity_, n_),
                           valid_.empty() ? nullptr : valid_.data()));
    if (!data_path.empty()) save_raw(data_path);
    if (!quant_path.empty()) {
      if (params_.quantization_type_ != QuantizationType::SQ8) throw std::runtime_error("no quantized space to save");
      save_sq8(quant_path);
    }
  }

  void load(const std::string &index_path, const std::string &data_path, const std::string &quant_path) {
    if (graph_) alaya_graph_free(graph_);
    graph_ = nullptr;
    check(alaya_graph_load(index_path.c_str(), id_bytes_, &graph_));
    if (data_path.empty()) throw std::runtime_error("the MI355X engine needs the raw data file");
    load_raw(data_path);
    if (params_.quantization_type_ == QuantizationType::SQ8) {
      if (quant_path.empty()) throw std::runtime_error("SQ8 index needs its quant file");
      load_sq8(quant_path);
    }
    upload();
  }

  uint32_t get_data_dim() const { return dim_; }

  // --- extra (not in the reference binding): device counters of the last search ---
  py::array last_counters() const {
    py::array_t<uint32_t> out({static_cast<py::ssize_t>(last_counters_.size() / 4), static_cast<py::ssize_t>(4)});
    std::memcpy(out.mutable_data(), last_counters_.data(), last_counters_.size() * 4);
    return out;
  }
  void set_hash_log2(uint32_t v) { check(alaya_index_set_hash_log2(ix_, v)); }
  void set_visited_mode(int m) { check(alaya_index_set_visited_mode(ix_, m)); }
  void set_helpers(int m) { check(alaya_index_set_helpers(ix_, m)); }
  py::tuple last_launch() {
    uint32_t g = 0, w = 0;
    check(alaya_index_last_launch(ix_, &g, &w));
    return py::make_tuple(g, w);
  }
  py::tuple help_stats() {
    uint64_t m = 0, x = 0, r = 0;
    check(alaya_index_help_stats(ix_, &m, &x, &r));
    return py::make_tuple(m, x, r);
  }
  // SQ8 batch_search rerank: 1 = the reference's PyIndex::rerank (default), 2 = corrected (whole ef pool)
  void set_rerank_mode(int m) {
    if (m != 1 && m != 2) throw std::invalid_argument("rerank mode must be 1 (reference) or 2 (corrected)");
    rerank_mode_ = m;
  }
  int rerank_mode() const { return rerank_mode_; }
  py::array device_distances(py::array queries, py::array_t<uint32_t> ids) {
    py::array q = prepare_queries(queries);
    py::array_t<uint32_t, py::array::c_style | py::array::forcecast> idc(ids);
    const uint64_t nq = q.shape(0);
    const uint32_t n = static_cast<uint32_t>(idc.size());
    py::array_t<float> out({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(n)});
    check(alaya_index_distances(ix_, static_cast<const float *>(q.data()), nq, idc.data(), n,
                                out.mutable_data()));
    return out;
  }
  // graph arrays (n x R l0, levels, upper_off, upper_edges, ep, upper_R) for tests/tools
  py::tuple graph_arrays() {
    if (!graph_) throw std::runtime_error("index is not fitted");
    sync_graph();
    uint64_t n, nue;
    uint32_t R, upper_R, ep, max_level, n_eps;
    int has_overlay;
    check(alaya_graph_info(graph_, &n, &R, &has_overlay, &upper_R, &ep, &max_level, &nue, &n_eps));
    py::array_t<uint32_t> l0({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(R)});
    py::array_t<uint32_t> levels(static_cast<py::ssize_t>(has_overlay ? n : 0));
    py::array_t<uint64_t> off(static_cast<py::ssize_t>(has_overlay ? n : 0));
    py::array_t<uint32_t> ue(static_cast<py::ssize_t>(nue));
    py::array_t<uint32_t> eps(static_cast<py::ssize_t>(n_eps));
    check(alaya_graph_export(graph_, l0.mutable_data(), levels.mutable_data(), off.mutable_data(),
                             ue.mutable_data(), eps.mutable_data()));
    return py::make_tuple(l0, has_overlay ? py::object(levels) : py::none(),
                          has_overlay ? py::object(off) : py::none(), ue, ep, upper_R, eps);
  }

 private:
  int metric_code() const {
    switch (params_.metric_) {
      case MetricType::L2: return ALAYA_METRIC_L2;
      case MetricType::IP: return ALAYA_METRIC_IP;
      case MetricType::COS: return ALAYA_METRIC_COS;
      default: throw std::runtime_error("unsupported metric");
    }
  }

  // the metric plus ALAYA_DIST_GENERIC for non-float DataType: l2_sqr<T>/ip_sqr<T> take their generic
  // branch for every DataType but float (distance_l2.ipp:735-741, distance_ip.ipp:744-750)
  int dist_code() const { return metric_code() | (dtype_ != kF32 ? ALAYA_DIST_GENERIC : 0); }

  void check_dtype(const py::array &a) const {
    if (dtype_code(a.dtype()) != dtype_) throw std::runtime_error("Unsupported data type");
  }

  void normalize_in_place(py::array &arr, uint64_t rows) {
    if (!arr.writeable()) throw std::runtime_error("COS metric normalises the input in place; array is read-only");
    if (dtype_ == kF32) {
      float *p = static_cast<float *>(arr.mutable_data());
      for (uint64_t i = 0; i < rows; ++i) alaya_amd::normalize_row(p + i * dim_, dim_);
    } else {  // float64 rows (data_utils.hpp normalize<double>)
      double *p = static_cast<double *>(arr.mutable_data());
      for (uint64_t i = 0; i < rows; ++i) {
        float sum = 0.0f;
        for (uint32_t j = 0; j < dim_; ++j) sum += static_cast<float>(p[i * dim_ + j] * p[i * dim_ + j]);
        sum = static_cast<float>(1.0 / std::sqrt(static_cast<double>(sum)));
        for (uint32_t j = 0; j < dim_; ++j) p[i * dim_ + j] *= sum;
      }
    }
  }

  py::array prepare_queries(py::array queries) {
    if (queries.ndim() != 2) throw std::runtime_error("queries must be 2D");
    check_dtype(queries);
    if (static_cast<uint32_t>(queries.shape(1)) != dim_) throw py::value_error("query dimension mismatch");
    py::array arr = py::array::ensure(queries, py::array::c_style);
    const uint64_t nq = arr.shape(0);
    raw_queries_.clear();
    if (params_.quantization_type_ == QuantizationType::SQ8 && params_.metric_ == MetricType::COS) {
      raw_queries_.resize(nq * dim_);
      to_float(arr.data(), dtype_, nq * dim_, raw_queries_.data());
    }
    if (params_.metric_ == MetricType::COS) normalize_in_place(arr, nq);  // raw_space.hpp:267-269
    py::array_t<float> qf({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(dim_)});
    to_float(arr.data(), dtype_, nq * dim_, qf.mutable_data());
    return qf;
  }

  std::pair<py::array, py::array> run(py::array queries, uint32_t topk, uint32_t ef, bool want_dist) {
    if (!graph_) throw std::runtime_error("Index is not init yet");
    py::array q = prepare_queries(queries);
    const uint64_t nq = q.shape(0);
    std::vector<uint32_t> ids32(nq * topk);
    py::array_t<float> dists({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(topk)});
    last_counters_.assign(nq * 4, 0);
    if (params_.quantization_type_ == QuantizationType::SQ8) {
      // SQ8Space::QueryComputer encodes the query as given (no COS normalisation), the rerank's
      // RawSpace::QueryComputer normalises it (raw_space.hpp:267-269): keep both forms.
      const float *rq = static_cast<const float *>(q.data());
      const float *sq = raw_queries_.empty() ? rq : raw_queries_.data();
      // batch_search reranks (index.hpp:337-345); batch_search_with_distance does not and returns
      // an empty distance array for SQ spaces (index.hpp:391-418, get_topk_array of no rows).
      const int rerank = want_dist ? 0 : rerank_mode_;
      {
        py::gil_scoped_release nogil;
        check(alaya_index_batch_search_sq8(ix_, sq, rq, nq, topk, ef, rerank, ids32.data(),
                                           dists.mutable_data(), last_counters_.data()));
      }
      if (want_dist) dists = py::array_t<float>(std::vector<py::ssize_t>{0, static_cast<py::ssize_t>(topk)});
    } else {
      py::gil_scoped_release nogil;
      check(alaya_index_batch_search(ix_, static_cast<const float *>(q.data()), nq, topk, ef,
                                     ids32.data(), dists.mutable_data(), last_counters_.data()));
    }
    py::array ids(params_.id_type_, std::vector<py::ssize_t>{static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(topk)});
    if (id_bytes_ == 4) {
      std::memcpy(ids.mutable_data(), ids32.data(), ids32.size() * 4);
    } else {
      auto *o = static_cast<uint64_t *>(ids.mutable_data());
      for (size_t i = 0; i < ids32.size(); ++i) o[i] = ids32[i];
    }
    return {ids, want_dist ? py::array(dists) : py::array()};
  }

  // first insert/remove: hand the device index a host mirror of the graph, rows and bitmap
  void ensure_updates() {
    if (updates_enabled_) return;
    const uint64_t cap = std::max<uint64_t>(params_.capacity_, n_);
    check(alaya_index_enable_updates(ix_, graph_, rows_f32_.data(), n_, cap, valid_.empty() ? nullptr : valid_.data()));
    updates_enabled_ = true;
  }
  // replace the (stale) fitted graph with the updated mirror
  void sync_graph() {
    if (!graph_dirty_) return;
    alaya_graph *g = nullptr;
    check(alaya_index_export_graph(ix_, &g));
    alaya_graph_free(graph_);
    graph_ = g;
    graph_dirty_ = false;
  }

  void upload() {
    updates_enabled_ = false;
    graph_dirty_ = false;
    if (!graph_) return;
    uint64_t gn = 0;
    check(alaya_graph_info(graph_, &gn, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr));
    py::gil_scoped_release nogil;
    check(alaya_index_set_base(ix_, rows_f32_.data(), n_, dim_, dist_code(),
                               valid_.empty() ? nullptr : valid_.data()));
    check(alaya_index_set_graph(ix_, graph_));
    if (!sq_codes_.empty())
      check(alaya_index_set_sq8(ix_, sq_codes_.data(), n_, dim_, sq_min_.data(), sq_max_.data(), host_sq8_order()));
  }

  void train_sq8(uint32_t num_threads) {
    if (params_.metric_ == MetricType::COS && dtype_ != kF32) throw std::runtime_error("COS metric only support float or double");
    sq_min_.assign(dim_, 0.f);
    sq_max_.assign(dim_, 0.f);
    sq_codes_.assign(n_ * dim_, 0);
    check(alaya_sq8_train(rows_f32_.data(), n_, dim_, sq_min_.data(), sq_max_.data()));
    check(alaya_sq8_encode(rows_f32_.data(), n_, dim_, sq_min_.data(), sq_max_.data(), sq_codes_.data(),
                           std::max(1u, num_threads)));
  }

  // RawSpace save/load (raw_space.hpp:219-250) + SequentialStorage (sequential_storage.hpp:110-142)
  void save_raw(const std::string &path) const {
    std::ofstream w(path, std::ios::binary);
    if (!w.is_open()) throw std::runtime_error("Cannot open file " + path);
    const int32_t metric = static_cast<int32_t>(params_.metric_);
    const size_t es = dtype_size(dtype_);
    const uint32_t data_size = static_cast<uint32_t>(dim_ * es);
    const uint64_t cap = std::max<uint64_t>(params_.capacity_, n_);
    w.write(reinterpret_cast<const char *>(&metric), 4);
    w.write(reinterpret_cast<const char *>(&data_size), 4);
    w.write(reinterpret_cast<const char *>(&dim_), 4);
    auto put_id = [&](uint64_t v) {
      if (id_bytes_ == 4) {
        uint32_t x = static_cast<uint32_t>(v);
        w.write(reinterpret_cast<const char *>(&x), 4);
      } else {
        w.write(reinterpret_cast<const char *>(&v), 8);
      }
    };
    put_id(n_);   // item_cnt_
    put_id(delete_cnt_);  // delete_cnt_
    put_id(cap);  // capacity_
    const uint64_t item = data_size, aligned = (item + 63) / 64 * 64, align = 64;
    w.write(reinterpret_cast<const char *>(&item), 8);
    w.write(reinterpret_cast<const char *>(&aligned), 8);
    w.write(reinterpret_cast<const char *>(&cap), 8);
    w.write(reinterpret_cast<const char *>(&n_), 8);
    w.write(reinterpret_cast<const char *>(&align), 8);
    std::vector<char> row(aligned, 0);
    for (uint64_t i = 0; i < cap; ++i) {
      std::fill(row.begin(), row.end(), 0);
      if (i < n_) std::memcpy(row.data(), raw_.data() + i * item, item);
      w.write(row.data(), static_cast<std::streamsize>(aligned));
    }
    std::vector<uint8_t> bitmap((cap + 7) / 8, 0);
    for (uint64_t i = 0; i < n_; ++i)
      if (valid_.empty() || (valid_[i / 8] >> (i % 8)) & 1) bitmap[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
    w.write(reinterpret_cast<const char *>(bitmap.data()), static_cast<std::streamsize>(bitmap.size()));
    if (!w) throw std::runtime_error("write failed: " + path);
  }

  void load_raw(const std::string &path) {
    std::ifstream r(path, std::ios::binary);
    if (!r.is_open()) throw std::runtime_error("Cannot open file " + path);
    int32_t metric;
    uint32_t data_size, dim;
    r.read(reinterpret_cast<char *>(&metric), 4);
    r.read(reinterpret_cast<char *>(&data_size), 4);
    r.read(reinterpret_cast<char *>(&dim), 4);
    auto get_id = [&]() -> uint64_t {
      if (id_bytes_ == 4) {
        uint32_t x;
        r.read(reinterpret_cast<char *>(&x), 4);
        return x;
      }
      uint64_t x;
      r.read(reinterpret_cast<char *>(&x), 8);
      return x;
    };
    const uint64_t item_cnt = get_id();
    delete_cnt_ = get_id();
    (void)get_id();
    uint64_t hdr[5];
    r.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
    if (!r) throw std::runtime_error("truncated raw data file");
    const uint64_t item = hdr[0], aligned = hdr[1], cap = hdr[2], pos = hdr[3];
    const size_t es = dtype_size(dtype_);
    if (item != static_cast<uint64_t>(dim) * es || data_size != item || aligned < item)
      throw std::runtime_error("raw data file does not match the index data type");
    dim_ = dim;
    n_ = item_cnt;
    if (pos < n_) n_ = pos;
    raw_.assign(n_ * item, 0);
    std::vector<char> row(aligned);
    for (uint64_t i = 0; i < cap; ++i) {
      r.read(row.data(), static_cast<std::streamsize>(aligned));
      if (!r) throw std::runtime_error("truncated raw data file");
      if (i < n_) std::memcpy(raw_.data() + i * item, row.data(), item);
    }
    std::vector<uint8_t> bitmap((cap + 7) / 8);
    r.read(reinterpret_cast<char *>(bitmap.data()), static_cast<std::streamsize>(bitmap.size()));
    valid_.assign((n_ + 7) / 8, 0);
    bool all = true;
    for (uint64_t i = 0; i < n_; ++i) {
      const bool v = (bitmap[i / 8] >> (i % 8)) & 1;
      if (v) valid_[i / 8] |= static_cast<uint8_t>(1u << (i % 8)); else all = false;
    }
    if (all) valid_.clear();
    rows_f32_.resize(n_ * dim_);
    to_float(raw_.data(), dtype_, n_ * dim_, rows_f32_.data());
  }

  // SQ8Space save/load (sq8_space.hpp:213-251) + SQ8Quantizer (sq8.hpp:161-177)
  void save_sq8(const std::string &path) const {
    std::ofstream w(path, std::ios::binary);
    if (!w.is_open()) throw std::runtime_error("Cannot open file " + path);
    const int32_t metric = static_cast<int32_t>(params_.metric_);
    const uint32_t data_size = dim_;
    const uint64_t cap = std::max<uint64_t>(params_.capacity_, n_);
    w.write(reinterpret_cast<const char *>(&metric), 4);
    w.write(reinterpret_cast<const char *>(&data_size), 4);
    w.write(reinterpret_cast<const char *>(&dim_), 4);
    auto put_id = [&](uint64_t v) {
      if (id_bytes_ == 4) {
        uint32_t x = static_cast<uint32_t>(v);
        w.write(reinterpret_cast<const char *>(&x), 4);
      } else {
        w.write(reinterpret_cast<const char *>(&v), 8);
      }
    };
    put_id(n_);
    put_id(0);
    put_id(cap);
    const uint64_t item = dim_, aligned = (item + 63) / 64 * 64, align = 64;
    w.write(reinterpret_cast<const char *>(&item), 8);
    w.write(reinterpret_cast<const char *>(&aligned), 8);
    w.write(reinterpret_cast<const char *>(&cap), 8);
    w.write(reinterpret_cast<const char *>(&n_), 8);
    w.write(reinterpret_cast<const char *>(&align), 8);
    std::vector<char> row(aligned, 0);
    for (uint64_t i = 0; i < cap; ++i) {
      std::fill(row.begin(), row.end(), 0);
      if (i < n_) std::memcpy(row.data(), sq_codes_.data() + i * item, item);
      w.write(row.data(), static_cast<std::streamsize>(aligned));
    }
    std::vector<uint8_t> bitmap((cap + 7) / 8, 0);
    for (uint64_t i = 0; i < n_; ++i) bitmap[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
    w.write(reinterpret_cast<const char *>(bitmap.data()), static_cast<std::streamsize>(bitmap.size()));
    w.write(reinterpret_cast<const char *>(&dim_), 4);
    w.write(reinterpret_cast<const char *>(sq_min_.data()), dim_ * 4);
    w.write(reinterpret_cast<const char *>(sq_max_.data()), dim_ * 4);
    if (!w) throw std::runtime_error("write failed: " + path);
  }
  void load_sq8(const std::string &path) {
    std::ifstream r(path, std::ios::binary);
    if (!r.is_open()) throw std::runtime_error("Cannot open file " + path);
    int32_t metric;
    uint32_t data_size, dim;
    r.read(reinterpret_cast<char *>(&metric), 4);
    r.read(reinterpret_cast<char *>(&data_size), 4);
    r.read(reinterpret_cast<char *>(&dim), 4);
    r.ignore(3 * id_bytes_);
    uint64_t hdr[5];
    r.read(reinterpret_cast<char *>(hdr), sizeof(hdr));
    if (!r || dim != dim_ || hdr[0] != dim) throw std::runtime_error("SQ8 file does not match the raw data");
    const uint64_t aligned = hdr[1], cap = hdr[2];
    sq_codes_.assign(n_ * dim_, 0);
    std::vector<char> row(aligned);
    for (uint64_t i = 0; i < cap; ++i) {
      r.read(row.data(), static_cast<std::streamsize>(aligned));
      if (!r) throw std::runtime_error("truncated SQ8 file");
      if (i < n_) std::memcpy(sq_codes_.data() + i * dim_, row.data(), dim_);
    }
    r.ignore(static_cast<std::streamsize>((cap + 7) / 8));
    uint32_t qd = 0;
    r.read(reinterpret_cast<char *>(&qd), 4);
    if (qd != dim_) throw std::runtime_error("SQ8 quantizer dimension mismatch");
    sq_min_.resize(dim_);
    sq_max_.resize(dim_);
    r.read(reinterpret_cast<char *>(sq_min_.data()), dim_ * 4);
    r.read(reinterpret_cast<char *>(sq_max_.data()), dim_ * 4);
    if (!r) throw std::runtime_error("truncated SQ8 file");
  }

  IndexParams params_;
  DType dtype_ = kF32;
  int id_bytes_ = 4;
  alaya_index *ix_ = nullptr;
  alaya_graph *graph_ = nullptr;
  uint64_t n_ = 0;
  uint32_t dim_ = 0;
  std::vector<char> raw_;          // original-dtype rows (get_data_by_id, save)
  std::vector<float> rows_f32_;    // float rows uploaded to HBM
  std::vector<uint8_t> valid_;     // empty = all valid
  uint64_t delete_cnt_ = 0;        // RawSpace::delete_cnt_
  bool updates_enabled_ = false;   // the device index holds an update mirror (alaya_index_enable_updates)
  bool graph_dirty_ = false;       // graph_ predates inserts (sync_graph refreshes it)
  std::vector<uint32_t> last_counters_;
  int rerank_mode_ = 1;
  std::vector<float> raw_queries_;   // SQ8 + COS: the un-normalised queries the SQ8 search encodes
  std::vector<uint8_t> sq_codes_;
  std::vector<float> sq_min_, sq_max_;
};


// ---- engine-level objects (beyond the reference binding): host graph + raw device index -----
class Graph {
 public:
  Graph() = default;
  explicit Graph(alaya_graph *g) : g_(g) {}
  ~Graph() {
    if (g_) alaya_graph_free(g_);
  }
  Graph(const Graph &) = delete;
  Graph &operator=(const Graph &) = delete;

  static std::shared_ptr<Graph> build(py::array_t<float, py::array::c_style | py::array::forcecast> data,
                                      int metric, uint32_t R, uint32_t efc, uint32_t threads,
                                      uint64_t seed) {
    if (data.ndim() != 2) throw py::value_error("data must be 2D");
    alaya_graph *g = nullptr;
    const float *ptr = data.data();
    const uint64_t n = data.shape(0);
    const uint32_t d = static_cast<uint32_t>(data.shape(1));
    {
      py::gil_scoped_release nogil;
      check(alaya_graph_build_hnsw(ptr, n, d, metric, R, efc, threads, seed, &g));
    }
    return std::make_shared<Graph>(g);
  }
  static std::shared_ptr<Graph> load(const std::string &path, int id_bytes) {
    alaya_graph *g = nullptr;
    check(alaya_graph_load(path.c_str(), id_bytes, &g));
    return std::make_shared<Graph>(g);
  }
  static std::shared_ptr<Graph> from_arrays(py::array_t<uint32_t, py::array::c_style | py::array::forcecast> l0,
                                            py::object levels, py::object upper_off, py::object upper_edges,
                                            uint32_t upper_R, uint32_t ep, py::object eps) {
    alaya_graph *g = nullptr;
    const uint64_t n = l0.shape(0);
    const uint32_t R = static_cast<uint32_t>(l0.shape(1));
    if (!levels.is_none()) {
      auto lv = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>(levels);
      auto off = py::array_t<uint64_t, py::array::c_style | py::array::forcecast>(upper_off);
      auto ue = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>(upper_edges);
      check(alaya_graph_import(n, R, l0.data(), lv.data(), off.data(), ue.data(), ue.size(), upper_R, ep,
                               nullptr, 0, &g));
    } else {
      auto e = py::array_t<uint32_t, py::array::c_style | py::array::forcecast>(eps);
      check(alaya_graph_import(n, R, l0.data(), nullptr, nullptr, nullptr, 0, 0, 0, e.data(),
                               static_cast<uint32_t>(e.size()), &g));
    }
    return std::make_shared<Graph>(g);
  }
  void save(const std::string &path, int id_bytes, uint64_t capacity) const {
    check(alaya_graph_save(g_, path.c_str(), id_bytes, capacity, nullptr));
  }
  py::tuple arrays() const {
    uint64_t n, nue;
    uint32_t R, upper_R, ep, max_level, n_eps;
    int has_overlay;
    check(alaya_graph_info(g_, &n, &R, &has_overlay, &upper_R, &ep, &max_level, &nue, &n_eps));
    py::array_t<uint32_t> l0({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(R)});
    py::array_t<uint32_t> levels(static_cast<py::ssize_t>(has_overlay ? n : 0));
    py::array_t<uint64_t> off(static_cast<py::ssize_t>(has_overlay ? n : 0));
    py::array_t<uint32_t> ue(static_cast<py::ssize_t>(nue));
    py::array_t<uint32_t> eps(static_cast<py::ssize_t>(n_eps));
    check(alaya_graph_export(g_, l0.mutable_data(), levels.mutable_data(), off.mutable_data(),
                             ue.mutable_data(), eps.mutable_data()));
    return py::make_tuple(l0, has_overlay ? py::object(levels) : py::none(),
                          has_overlay ? py::object(off) : py::none(), ue, ep, upper_R, eps);
  }
  alaya_graph *get() const { return g_; }

 private:
  alaya_graph *g_ = nullptr;
};

// Raw device index: rows + graph in HBM, batch search on host arrays or device pointers.
class DeviceIndex {
 public:
  explicit DeviceIndex(int device) { check(alaya_index_create(device, &ix_)); }
  ~DeviceIndex() {
    if (ix_) alaya_index_destroy(ix_);
  }
  DeviceIndex(const DeviceIndex &) = delete;
  DeviceIndex &operator=(const DeviceIndex &) = delete;
  void set_base(py::array_t<float, py::array::c_style | py::array::forcecast> rows, int metric,
                py::object valid) {
    const uint8_t *vp = nullptr;
    py::array_t<uint8_t, py::array::c_style | py::array::forcecast> v;
    if (!valid.is_none()) {
      v = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>(valid);
      vp = v.data();
    }
    const float *ptr = rows.data();
    const uint64_t n = rows.shape(0);
    const uint32_t d = static_cast<uint32_t>(rows.shape(1));
    py::gil_scoped_release nogil;
    check(alaya_index_set_base(ix_, ptr, n, d, metric, vp));
  }
  void set_graph(const Graph &g) { check(alaya_index_set_graph(ix_, g.get())); }
  // device HNSW build from the rows set by set_base; the graph becomes this index's search graph
  py::tuple build_graph(uint32_t R, uint32_t efc, uint64_t seed, uint32_t batch_div, uint32_t max_batch,
                        uint32_t refine) {
    alaya_graph *g = nullptr;
    uint64_t st[8] = {0};
    {
      py::gil_scoped_release nogil;
      check(alaya_index_build_graph(ix_, R, efc, seed, batch_div, max_batch, refine, &g, st));
    }
    py::dict stats;
    stats["batches"] = st[0];
    stats["launches"] = st[1];
    stats["prunes"] = st[2];
    stats["appends"] = st[3];
    stats["heuristic_dists"] = st[4];
    stats["device_ms"] = static_cast<double>(st[5]) / 1000.0;
    stats["max_batch"] = st[6];
    stats["max_level"] = st[7];
    return py::make_tuple(std::make_shared<Graph>(g), stats);
  }
  py::tuple search(py::array_t<float, py::array::c_style | py::array::forcecast> q, uint32_t k, uint32_t ef) {
    const uint64_t nq = q.shape(0);
    py::array_t<uint32_t> ids({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<float> d({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<uint32_t> c({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(4)});
    const float *qp = q.data();
    uint32_t *ip = ids.mutable_data();
    float *dp = d.mutable_data();
    uint32_t *cp = c.mutable_data();
    {
      py::gil_scoped_release nogil;
      check(alaya_index_batch_search(ix_, qp, nq, k, ef, ip, dp, cp));
    }
    return py::make_tuple(ids, d, c);
  }
  void search_device(uintptr_t q, uint64_t nq, uint32_t k, uint32_t ef, uintptr_t ids, uintptr_t dists,
                     uintptr_t counters, uintptr_t stream) {
    check(alaya_index_batch_search_device(ix_, reinterpret_cast<const float *>(q), nq, k, ef,
                                          reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                          reinterpret_cast<uint32_t *>(counters), reinterpret_cast<void *>(stream)));
  }
  void shard_search_device(uintptr_t q, uint64_t nq, uint32_t k, uint32_t ef, uintptr_t ids, uintptr_t dists,
                           uintptr_t counters, uintptr_t stream) {
    check(alaya_index_shard_search_device(ix_, reinterpret_cast<const float *>(q), nq, k, ef,
                                          reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                          reinterpret_cast<uint32_t *>(counters), reinterpret_cast<void *>(stream)));
  }
  py::array distances(py::array_t<float, py::array::c_style | py::array::forcecast> q,
                      py::array_t<uint32_t, py::array::c_style | py::array::forcecast> ids) {
    const uint64_t nq = q.shape(0);
    const uint32_t n = static_cast<uint32_t>(ids.size());
    py::array_t<float> out({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(n)});
    check(alaya_index_distances(ix_, q.data(), nq, ids.data(), n, out.mutable_data()));
    return out;
  }
  void set_sq8(py::array_t<uint8_t, py::array::c_style | py::array::forcecast> codes,
               py::array_t<float, py::array::c_style | py::array::forcecast> mn,
               py::array_t<float, py::array::c_style | py::array::forcecast> mx, int order) {
    check(alaya_index_set_sq8(ix_, codes.data(), codes.shape(0), static_cast<uint32_t>(codes.shape(1)),
                              mn.data(), mx.data(), order));
  }
  py::tuple search_sq8(py::array_t<float, py::array::c_style | py::array::forcecast> q, uint32_t k,
                       uint32_t ef, int rerank, py::object rerank_queries) {
    const uint64_t nq = q.shape(0);
    py::array_t<float, py::array::c_style | py::array::forcecast> rq;
    const float *rqp = nullptr;
    if (!rerank_queries.is_none()) {
      rq = py::array_t<float, py::array::c_style | py::array::forcecast>(rerank_queries);
      rqp = rq.data();
    }
    py::array_t<uint32_t> ids({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<float> d({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<uint32_t> c({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(4)});
    check(alaya_index_batch_search_sq8(ix_, q.data(), rqp, nq, k, ef, rerank, ids.mutable_data(),
                                       d.mutable_data(), c.mutable_data()));
    return py::make_tuple(ids, d, c);
  }
  void search_sq8_device(uintptr_t q, uintptr_t rq, uint64_t nq, uint32_t k, uint32_t ef, int rerank,
                         uintptr_t ids, uintptr_t dists, uintptr_t counters, uintptr_t stream) {
    check(alaya_index_batch_search_sq8_device(ix_, reinterpret_cast<const float *>(q),
                                              reinterpret_cast<const float *>(rq), nq, k, ef, rerank,
                                              reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                              reinterpret_cast<uint32_t *>(counters),
                                              reinterpret_cast<void *>(stream)));
  }
  void shard_search_sq8_device(uintptr_t q, uintptr_t rq, uint64_t nq, uint32_t k, uint32_t ef, bool holds_row0,
                               uintptr_t ids, uintptr_t dists, uintptr_t counters, uintptr_t stream) {
    check(alaya_index_shard_search_sq8_device(ix_, reinterpret_cast<const float *>(q),
                                              reinterpret_cast<const float *>(rq), nq, k, ef, holds_row0 ? 1 : 0,
                                              reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                              reinterpret_cast<uint32_t *>(counters),
                                              reinterpret_cast<void *>(stream)));
  }
  py::tuple flat_search(py::array_t<float, py::array::c_style | py::array::forcecast> q, uint32_t k) {
    const uint64_t nq = q.shape(0);
    py::array_t<uint32_t> ids({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<float> d({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    uint32_t redo = 0;
    const float *qp = q.data();
    uint32_t *ip = ids.mutable_data();
    float *dp = d.mutable_data();
    {
      py::gil_scoped_release nogil;
      check(alaya_index_flat_search(ix_, qp, nq, k, ip, dp, &redo));
    }
    return py::make_tuple(ids, d, redo);
  }
  void flat_search_device(uintptr_t q, uint64_t nq, uint32_t k, uintptr_t ids, uintptr_t dists,
                          uintptr_t flags, uintptr_t stream) {
    check(alaya_index_flat_search_device(ix_, reinterpret_cast<const float *>(q), nq, k,
                                         reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                         reinterpret_cast<uint32_t *>(flags), reinterpret_cast<void *>(stream)));
  }
  int flat_contraction() const {
    int c = -1;
    check(alaya_index_flat_last_contraction(ix_, &c));
    return c;
  }
  void flat_diag(uintptr_t q, uint64_t nq, uint32_t k, int ablate, uintptr_t ids, uintptr_t dists,
                 uintptr_t flags, uintptr_t mc, uintptr_t stream) {
    check(alaya_index_flat_diag(ix_, reinterpret_cast<const float *>(q), nq, k, ablate,
                                reinterpret_cast<uint32_t *>(ids), reinterpret_cast<float *>(dists),
                                reinterpret_cast<uint32_t *>(flags), reinterpret_cast<uint32_t *>(mc),
                                reinterpret_cast<void *>(stream)));
  }
  void set_hash_log2(uint32_t v) { check(alaya_index_set_hash_log2(ix_, v)); }
  void set_visited_mode(int m) { check(alaya_index_set_visited_mode(ix_, m)); }
  void set_helpers(int m) { check(alaya_index_set_helpers(ix_, m)); }
  py::tuple last_launch() {
    uint32_t g = 0, w = 0;
    check(alaya_index_last_launch(ix_, &g, &w));
    return py::make_tuple(g, w);
  }
  py::tuple help_stats() {
    uint64_t m = 0, x = 0, r = 0;
    check(alaya_index_help_stats(ix_, &m, &x, &r));
    return py::make_tuple(m, x, r);
  }
  py::tuple profile_search(py::array_t<float, py::array::c_style | py::array::forcecast> q, uint32_t k,
                           uint32_t ef, int space) {
    const uint64_t nq = q.shape(0);
    py::array_t<uint32_t> ids({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(k)});
    py::array_t<uint32_t> c({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(4)});
    py::array_t<uint64_t> st({static_cast<py::ssize_t>(nq), static_cast<py::ssize_t>(8)});
    check(alaya_index_profile_search(ix_, q.data(), nq, k, ef, space, ids.mutable_data(), c.mutable_data(),
                                     st.mutable_data()));
    return py::make_tuple(ids, c, st);
  }
  uint64_t device_bytes() const {
    uint64_t b = 0;
    check(alaya_index_info(ix_, nullptr, nullptr, nullptr, nullptr, &b));
    return b;
  }

 private:
  alaya_index *ix_ = nullptr;
};

}  // namespace alaya_py

PYBIND11_MODULE(_alayalitepy, m) {
  using namespace alaya_py;
  m.doc() = "AlayaLite MI355X engine";
  m.attr("__version__") = "0.1.0-mi355x";

  py::enum_<IndexType>(m, "IndexType")
      .value("FLAT", IndexType::FLAT)
      .value("HNSW", IndexType::HNSW)
      .value("NSG", IndexType::NSG)
      .value("FUSION", IndexType::FUSION)
      .export_values();
  py::enum_<MetricType>(m, "MetricType")
      .value("L2", MetricType::L2)
      .value("IP", MetricType::IP)
      .value("COS", MetricType::COS)
      .export_values();
  py::enum_<QuantizationType>(m, "QuantizationType")
      .value("NONE", QuantizationType::NONE)
      .value("SQ8", QuantizationType::SQ8)
      .value("SQ4", QuantizationType::SQ4)
      .value("RABITQ", QuantizationType::RABITQ)
      .export_values();

  py::class_<IndexParams>(m, "IndexParams")
      .def(py::init<>())
      .def(py::init([](IndexType it, py::dtype dt, py::dtype idt, QuantizationType qt, MetricType mt,
                       uint32_t cap) {
             IndexParams p;
             p.index_type_ = it;
             p.data_type_ = std::move(dt);
             p.id_type_ = std::move(idt);
             p.quantization_type_ = qt;
             p.metric_ = mt;
             p.capacity_ = cap;
             return p;
           }),
           py::arg("index_type_") = IndexType::HNSW, py::arg("data_type_") = py::dtype::of<float>(),
           py::arg("id_type_") = py::dtype::of<uint32_t>(),
           py::arg("quantization_type_") = QuantizationType::NONE,
           py::arg("metric_") = MetricType::L2, py::arg("capacity_") = 100000u)
      .def_readwrite("index_type_", &IndexParams::index_type_)
      .def_readwrite("data_type_", &IndexParams::data_type_)
      .def_readwrite("id_type_", &IndexParams::id_type_)
      .def_readwrite("quantization_type_", &IndexParams::quantization_type_)
      .def_readwrite("metric_", &IndexParams::metric_)
      .def_readwrite("capacity_", &IndexParams::capacity_);

  py::class_<PyIndexInterface, std::shared_ptr<PyIndexInterface>>(m, "PyIndexInterface")
      .def(py::init<IndexParams>(), py::arg("params"))
      .def("to_string", &PyIndexInterface::to_string)
      .def("fit", &PyIndexInterface::fit, py::arg("vectors"), py::arg("ef_construction"), py::arg("num_threads"),
           py::arg("builder") = "host")
      .def("search", &PyIndexInterface::search, py::arg("query"), py::arg("topk"), py::arg("ef"))
      .def("get_data_by_id", &PyIndexInterface::get_data_by_id, py::arg("id"))
      .def("insert", &PyIndexInterface::insert, py::arg("insert_data"), py::arg("ef"))
      .def("remove", &PyIndexInterface::remove, py::arg("id"))
      .def("batch_search", &PyIndexInterface::batch_search, py::arg("queries"), py::arg("topk"),
           py::arg("ef"), py::arg("num_threads"))
      .def("batch_search_with_distance", &PyIndexInterface::batch_search_with_distance,
           py::arg("queries"), py::arg("topk"), py::arg("ef"), py::arg("num_threads"))
      .def("save", &PyIndexInterface::save, py::arg("index_path"), py::arg("data_path"),
           py::arg("quant_path") = std::string())
      .def("load", &PyIndexInterface::load, py::arg("index_path"), py::arg("data_path"),
           py::arg("quant_path") = std::string())
      .def("get_data_dim", &PyIndexInterface::get_data_dim)
      .def("last_counters", &PyIndexInterface::last_counters)
      .def("set_hash_log2", &PyIndexInterface::set_hash_log2)
      .def("set_visited_mode", &PyIndexInterface::set_visited_mode)
      .def("set_helpers", &PyIndexInterface::set_helpers)
      .def("last_launch", &PyIndexInterface::last_launch)
      .def("help_stats", &PyIndexInterface::help_stats)
      .def("set_rerank_mode", &PyIndexInterface::set_rerank_mode)
      .def("rerank_mode", &PyIndexInterface::rerank_mode)
      .def("device_distances", &PyIndexInterface::device_distances)
      .def("graph_arrays", &PyIndexInterface::graph_arrays);


  py::class_<Graph, std::shared_ptr<Graph>>(m, "Graph")
      .def_static("build", &Graph::build, py::arg("data"), py::arg("metric") = 0, py::arg("R") = 32u,
                  py::arg("ef_construction") = 100u, py::arg("num_threads") = 1u, py::arg("seed") = 100u)
      .def_static("load", &Graph::load, py::arg("path"), py::arg("id_bytes") = 4)
      .def_static("from_arrays", &Graph::from_arrays, py::arg("l0"), py::arg("levels"), py::arg("upper_off"),
                  py::arg("upper_edges"), py::arg("upper_R"), py::arg("ep"), py::arg("eps") = py::none())
      .def("save", &Graph::save, py::arg("path"), py::arg("id_bytes") = 4, py::arg("capacity") = 0u)
      .def("arrays", &Graph::arrays);
  py::class_<DeviceIndex, std::shared_ptr<DeviceIndex>>(m, "DeviceIndex")
      .def(py::init<int>(), py::arg("device") = 0)
      .def("set_base", &DeviceIndex::set_base, py::arg("rows"), py::arg("metric") = 0, py::arg("valid") = py::none())
      .def("set_graph", &DeviceIndex::set_graph)
      .def("build_graph", &DeviceIndex::build_graph, py::arg("R") = 32, py::arg("ef_construction") = 100,
           py::arg("seed") = 100, py::arg("batch_div") = 0, py::arg("max_batch") = 0, py::arg("refine") = 2)
      .def("search", &DeviceIndex::search, py::arg("queries"), py::arg("k"), py::arg("ef"))
      .def("search_device", &DeviceIndex::search_device)
      .def("shard_search_device", &DeviceIndex::shard_search_device)
      .def("distances", &DeviceIndex::distances)
      .def("set_hash_log2", &DeviceIndex::set_hash_log2)
      .def("set_visited_mode", &DeviceIndex::set_visited_mode)
      .def("set_helpers", &DeviceIndex::set_helpers)
      .def("last_launch", &DeviceIndex::last_launch)
      .def("help_stats", &DeviceIndex::help_stats)
      .def("flat_search", &DeviceIndex::flat_search, py::arg("queries"), py::arg("k"))
      .def("flat_search_device", &DeviceIndex::flat_search_device)
      .def("flat_diag", &DeviceIndex::flat_diag)
      .def("flat_contraction", &DeviceIndex::flat_contraction)
      .def("search_sq8_device", &DeviceIndex::search_sq8_device)
      .def("shard_search_sq8_device", &DeviceIndex::shard_search_sq8_device)
      .def("set_sq8", &DeviceIndex::set_sq8, py::arg("codes"), py::arg("min"), py::arg("max"), py::arg("order") = 2)
      .def("search_sq8", &DeviceIndex::search_sq8, py::arg("queries"), py::arg("k"), py::arg("ef"),
           py::arg("rerank") = 1, py::arg("rerank_queries") = py::none())
      .def("profile_search", &DeviceIndex::profile_search, py::arg("q"), py::arg("k"), py::arg("ef"),
           py::arg("space") = 0)
      .def("device_bytes", &DeviceIndex::device_bytes);
  m.def("sq8_train", [](py::array_t<float, py::array::c_style | py::array::forcecast> data) {
    const uint32_t d = static_cast<uint32_t>(data.shape(1));
    py::array_t<float> mn(d), mx(d);
    check(alaya_sq8_train(data.data(), data.shape(0), d, mn.mutable_data(), mx.mutable_data()));
    return py::make_tuple(mn, mx);
  });
  m.def("sq8_encode", [](py::array_t<float, py::array::c_style | py::array::forcecast> data,
                         py::array_t<float, py::array::c_style | py::array::forcecast> mn,
                         py::array_t<float, py::array::c_style | py::array::forcecast> mx, uint32_t threads) {
    py::array_t<uint8_t> codes({data.shape(0), data.shape(1)});
    check(alaya_sq8_encode(data.data(), data.shape(0), static_cast<uint32_t>(data.shape(1)), mn.data(), mx.data(),
                           codes.mutable_data(), threads));
    return codes;
  }, py::arg("data"), py::arg("min"), py::arg("max"), py::arg("num_threads") = 1u);
  m.def("host_sq8_order", &host_sq8_order);
  m.def("build_info", [] { return std::string(alaya_build_info()); });
  m.def("device_count", [] {
    int c = 0;
    check(alaya_device_count(&c));
    return c;
  });
  m.def("hbm_stream_read", [](int device, uint64_t bytes, int iters) {
    double gbs = 0.0;
    check(alaya_hbm_stream_read(device, bytes, iters, &gbs));
    return gbs;
  }, py::arg("device") = 0, py::arg("bytes") = 4ull << 30, py::arg("iters") = 5);
  // a CU-masked stream (handle as an int, for torch.cuda.ExternalStream) and its release
  m.def("stream_create_reserving", [](int device, uint32_t reserved_cus) {
    void *s = nullptr;
    check(alaya_stream_create_reserving(device, reserved_cus, &s));
    return reinterpret_cast<uintptr_t>(s);
  }, py::arg("device"), py::arg("reserved_cus"));
  m.def("stream_destroy", [](uintptr_t s) { check(alaya_stream_destroy(reinterpret_cast<void *>(s))); });
}
