/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's HNSW construction, the checker for
 * the engine's graph builders (alayalite_amd/csrc/hnsw_build.cpp, build_kernels.hip).  Written from
 * the reference, sharing no code with the product:
 *
 *   HNSWImpl (include/index/graph/hnsw/hnswlib.hpp)
 *     ctor                          :87-121   M, M0 = 2M, ef = max(efc, M), seed, mult = 1/ln(M)
 *     CompareByFirst                :129-136  heap order on the distance only
 *     get_random_level              :182-186  -ln(U(0,1)) * mult, truncated
 *     get_neighbors_by_heuristic2   :291-354
 *     search_base_layer             :373-489
 *     mutually_connect_new_element  :509-628  (isUpdate == false)
 *     add_point                     :652-751
 *   HNSWBuilder::build_graph (include/index/graph/hnsw/hnsw_builder.hpp:98-194), thread_num = 1:
 *     add_point(0), add_point(1 .. n-1) in label order; level-0 lists copied into R-wide rows
 *     padded with -1; upper lists into R-wide per-level slots padded with -1; ep = enterpoint.
 *
 * Single-threaded, so internal id == label and the level draws happen in label order.  The heaps are
 * the same std::priority_queue instantiations as the reference, so equal-distance candidates leave
 * them in the same order.  Distances: RawSpace::get_distance (raw_space.hpp:178-180) = the float
 * kernel in the l2_sqr_avx2 / ip_sqr_avx2 order (oracle.cpp), or, for non-float DataType, the
 * generic branch (distance_l2.ipp:735-741, distance_ip.ipp:744-750) over the rows cast to float.
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <queue>
#include <random>
#include <utility>
#include <vector>

#include "oracle.h"

namespace {

using Pair = std::pair<float, uint32_t>;
struct CompareByFirst {  // hnswlib.hpp:129-136
  bool operator()(const Pair &a, const Pair &b) const noexcept { return a.first < b.first; }
};
using TopHeap = std::priority_queue<Pair, std::vector<Pair>, CompareByFirst>;

class Hnsw {
 public:
  Hnsw(const float *rows, uint64_t n, uint32_t dim, int metric, int generic, size_t M, size_t efc, uint64_t seed)
      : rows_(rows), n_(n), dim_(dim), metric_(metric), generic_(generic), M_(M), M0_(2 * M),
        ef_(efc > M ? efc : M), level_of_(n, 0), l0_(n * (M0_ + 1), 0), upper_(n), visit_(n, 0) {
    gen_.seed(seed);
    mult_ = 1.0 / std::log(1.0 * static_cast<double>(M_));
  }

  void add_point(uint32_t label) {  // hnswlib.hpp:652-751 (one thread: internal id == label)
    const int level = random_level();
    level_of_[label] = level;
    const int maxlevel_copy = maxlevel_;
    uint32_t cur = enterpoint_;
    if (level != 0) upper_[label].assign(static_cast<size_t>(level) * (M_ + 1), 0u);
    if (cur != kNone) {
      if (level < maxlevel_copy) {
        float curdist = dist(label, cur);
        for (int l = maxlevel_copy; l > level; --l) {
          bool changed = true;
          while (changed) {
            changed = false;
            const uint32_t *ll = list(cur, l);
            for (uint32_t i = 0; i < ll[0]; ++i) {
              const uint32_t cand = ll[1 + i];
              const float d = dist(label, cand);
              if (d < curdist) {
                curdist = d;
                cur = cand;
                changed = true;
              }
            }
          }
        }
      }
      for (int l = level < maxlevel_copy ? level : maxlevel_copy; l >= 0; --l) {
        TopHeap top = search_layer(cur, label, l);
        cur = connect(label, top, l);
      }
    } else {
      enterpoint_ = 0;
      maxlevel_ = level;
    }
    if (level > maxlevel_copy) {
      enterpoint_ = label;
      maxlevel_ = level;
    }
  }

  // HNSWBuilder::build_graph's copy into Graph + OverlayGraph (hnsw_builder.hpp:145-192)
  void export_graph(uint32_t R, uint32_t *l0, uint32_t *levels, uint64_t *upper_off, uint32_t *upper_edges,
                    uint32_t *ep) const {
    uint64_t off = 0;
    for (uint64_t i = 0; i < n_; ++i) {
      const uint32_t *ll = list(static_cast<uint32_t>(i), 0);
      for (uint32_t j = 0; j < R; ++j) l0[i * R + j] = j < ll[0] ? ll[1 + j] : 0xffffffffu;
      levels[i] = static_cast<uint32_t>(level_of_[i]);
      upper_off[i] = off;
      for (int l = 1; l <= level_of_[i]; ++l) {
        const uint32_t *ul = list(static_cast<uint32_t>(i), l);
        for (uint32_t j = 0; j < R; ++j) upper_edges[off + j] = j < ul[0] ? ul[1 + j] : 0xffffffffu;
        off += R;
      }
    }
    *ep = n_ ? enterpoint_ : 0;
  }

  uint64_t upper_slots(uint32_t R) const {
    uint64_t s = 0;
    for (int l : level_of_) s += static_cast<uint64_t>(l) * R;
    return s;
  }

 private:
  static constexpr uint32_t kNone = 0xffffffffu;

  int random_level() {  // hnswlib.hpp:182-186, called with mult_ (:679)
    std::uniform_real_distribution<double> u(0.0, 1.0);
    const double r = -std::log(u(gen_)) * mult_;
    return static_cast<int>(static_cast<size_t>(r));
  }

  float dist(uint32_t a, uint32_t b) const {
    const float *x = rows_ + static_cast<uint64_t>(a) * dim_;
    const float *y = rows_ + static_cast<uint64_t>(b) * dim_;
    if (generic_) return metric_ == ORC_L2 ? orc_l2_generic(x, y, dim_, 0) : orc_ip_generic(x, y, dim_, 0);
    return metric_ == ORC_L2 ? orc_l2_f32(x, y, dim_) : orc_ip_f32(x, y, dim_);
  }

  // link list of node u at level l: [count, id_0 .. id_{cap-1}]
  uint32_t *list(uint32_t u, int l) {
    return l == 0 ? &l0_[static_cast<uint64_t>(u) * (M0_ + 1)] : &upper_[u][static_cast<size_t>(l - 1) * (M_ + 1)];
  }
  const uint32_t *list(uint32_t u, int l) const {
    return l == 0 ? &l0_[static_cast<uint64_t>(u) * (M0_ + 1)] : &upper_[u][static_cast<size_t>(l - 1) * (M_ + 1)];
  }

  TopHeap search_layer(uint32_t ep, uint32_t q, int layer) {  // hnswlib.hpp:373-489
    if (++tag_ == 0) {  // VisitedList::reset (visited_list_pool.hpp:39-44)
      std::fill(visit_.begin(), visit_.end(), 0u);
      tag_ = 1;
    }
    TopHeap top, candidates;
    const float d0 = dist(q, ep);
    top.emplace(d0, ep);
    float lower_bound = d0;
    candidates.emplace(-d0, ep);
    visit_[ep] = tag_;
    while (!candidates.empty()) {
      const Pair cur = candidates.top();
      if (-cur.first > lower_bound && top.size() == ef_) break;
      candidates.pop();
      const uint32_t *ll = list(cur.second, layer);
      for (uint32_t j = 0; j < ll[0]; ++j) {
        const uint32_t c = ll[1 + j];
        if (visit_[c] == tag_) continue;
        visit_[c] = tag_;
        const float d = dist(q, c);
        if (top.size() < ef_ || lower_bound > d) {
          candidates.emplace(-d, c);
          top.emplace(d, c);
          if (top.size() > ef_) top.pop();
          if (!top.empty()) lower_bound = top.top().first;
        }
      }
    }
    return top;
  }

  void heuristic(TopHeap &top, size_t m) const {  // hnswlib.hpp:291-354
    if (top.size() < m) return;
    std::priority_queue<Pair> closest;
    std::vector<Pair> kept;
    while (!top.empty()) {
      closest.emplace(-top.top().first, top.top().second);
      top.pop();
    }
    while (!closest.empty()) {
      if (kept.size() >= m) break;
      const Pair cur = closest.top();
      const float to_query = -cur.first;
      closest.pop();
      bool good = true;
      for (const Pair &s : kept) {
        if (dist(s.second, cur.second) < to_query) {
          good = false;
          break;
        }
      }
      if (good) kept.push_back(cur);
    }
    for (const Pair &s : kept) top.emplace(-s.first, s.second);
  }

  uint32_t connect(uint32_t c, TopHeap &top, int level) {  // hnswlib.hpp:509-628, isUpdate false
    const size_t cap = level != 0 ? M_ : M0_;
    heuristic(top, M_);
    std::vector<uint32_t> chosen;
    chosen.reserve(M_);
    while (!top.empty()) {
      chosen.push_back(top.top().second);
      top.pop();
    }
    const uint32_t next = chosen.back();
    uint32_t *own = list(c, level);
    own[0] = static_cast<uint32_t>(chosen.size());
    for (size_t i = 0; i < chosen.size(); ++i) own[1 + i] = chosen[i];
    for (uint32_t nb : chosen) {
      uint32_t *ll = list(nb, level);
      const size_t sz = ll[0];
      if (sz < cap) {
        ll[1 + sz] = c;
        ll[0] = static_cast<uint32_t>(sz + 1);
        continue;
      }
      TopHeap cand;
      cand.emplace(dist(c, nb), c);
      for (size_t j = 0; j < sz; ++j) cand.emplace(dist(ll[1 + j], nb), ll[1 + j]);
      heuristic(cand, cap);
      uint32_t idx = 0;
      while (!cand.empty()) {
        ll[1 + idx] = cand.top().second;
        cand.pop();
        ++idx;
      }
      ll[0] = idx;
    }
    return next;
  }

  const float *rows_;
  uint64_t n_;
  uint32_t dim_;
  int metric_, generic_;
  size_t M_, M0_, ef_;
  double mult_ = 0.0;
  std::default_random_engine gen_;
  std::vector<int> level_of_;
  std::vector<uint32_t> l0_;
  std::vector<std::vector<uint32_t>> upper_;
  std::vector<uint32_t> visit_;
  uint32_t tag_ = 0;
  uint32_t enterpoint_ = kNone;
  int maxlevel_ = -1;
};

}  // namespace

struct orc_hnsw {
  Hnsw h;
  uint32_t R;
};

extern "C" {

orc_hnsw *orc_hnsw_build(const float *rows, uint64_t n, uint32_t dim, int metric, int generic, uint32_t R,
                         uint32_t ef_construction, uint64_t seed) {
  auto *o = new orc_hnsw{Hnsw(rows, n, dim, metric, generic, R / 2, ef_construction, seed), R};
  for (uint64_t i = 0; i < n; ++i) o->h.add_point(static_cast<uint32_t>(i));
  return o;
}

uint64_t orc_hnsw_upper_slots(const orc_hnsw *o) { return o->h.upper_slots(o->R); }

void orc_hnsw_export(const orc_hnsw *o, uint32_t *l0, uint32_t *levels, uint64_t *upper_off,
                     uint32_t *upper_edges, uint32_t *ep) {
  o->h.export_graph(o->R, l0, levels, upper_off, upper_edges, ep);
}

void orc_hnsw_free(orc_hnsw *o) { delete o; }

}  // extern "C"
