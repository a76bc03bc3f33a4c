// HNSW builder (host C++) -- hnswlib semantics as restated by the reference
// (include/index/graph/hnsw/hnswlib.hpp:87-751, hnsw_builder.hpp:98-194).  Produces the HostGraph
// that is uploaded to HBM for the device search.
#include "hnsw_build.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <queue>
#include <random>
#include <stdexcept>
#include <thread>

#include "host_distance.h"

namespace alaya_amd {

uint32_t HostGraph::max_level() const {
  return has_overlay && !levels.empty() ? levels[ep] : 0;
}

std::vector<uint32_t> hnsw_levels(uint64_t n, uint32_t M, uint64_t seed) {
  // Levels are drawn in label order exactly as sequential add_point(0..n-1) draws them
  // (get_random_level, hnswlib.hpp:182-186; mult_ = 1/ln(M), :118).
  std::vector<uint32_t> levels(n);
  std::default_random_engine gen;
  gen.seed(seed);
  const double mult = 1.0 / std::log(1.0 * M);
  for (uint64_t i = 0; i < n; ++i) {
    std::uniform_real_distribution<double> distribution(0.0, 1.0);
    double r = -std::log(distribution(gen)) * mult;
    levels[i] = static_cast<uint32_t>(static_cast<size_t>(r));
  }
  return levels;
}

namespace {

using DistId = std::pair<float, uint32_t>;
struct CompareByFirst {  // hnswlib.hpp:129-136: ties on the distance are left to the heap
  bool operator()(const DistId &a, const DistId &b) const noexcept { return a.first < b.first; }
};
using MaxHeap = std::priority_queue<DistId, std::vector<DistId>, CompareByFirst>;

class Builder {
 public:
  Builder(const float *data, uint64_t n, uint32_t dim, int metric, uint32_t M, uint32_t efc,
          uint64_t seed)
      : data_(data), n_(n), dim_(dim), metric_(metric), M_(M), M0_(2 * M),
        efc_(std::max<size_t>(efc, M)), locks_(n), levels_(n, 0), links0_(n * (1 + 2 * M), 0),
        upper_(n) {
    const std::vector<uint32_t> lv = hnsw_levels(n_, static_cast<uint32_t>(M_), seed);
    for (uint64_t i = 0; i < n_; ++i) levels_[i] = static_cast<int>(lv[i]);
  }

  // The reference holds the new node's lock for the whole insertion (hnswlib.hpp:670); here every
  // lock is taken one node at a time (own list written under its lock in connect()), which keeps
  // the sequential result identical and rules out lock-order cycles between concurrent inserts.
  void add_point(uint32_t id, std::vector<uint32_t> &visited, uint32_t &tag) {  // :652-751
    const int cur_level = levels_[id];
    if (cur_level > 0) {
      std::unique_lock<std::mutex> lock(locks_[id]);
      upper_[id].assign(static_cast<size_t>(cur_level) * (1 + M_), 0);
    }

    std::unique_lock<std::mutex> templock(global_);
    const int maxlevel_copy = maxlevel_;
    uint32_t curr = enterpoint_;
    if (cur_level <= maxlevel_copy) templock.unlock();

    if (curr != kNone) {
      if (cur_level < maxlevel_copy) {
        float curdist = dist(id, curr);
        for (int level = maxlevel_copy; level > cur_level; --level) {
          bool changed = true;
          while (changed) {
            changed = false;
            std::unique_lock<std::mutex> lock(locks_[curr]);
            const uint32_t *ll = list(curr, level);
            const uint32_t size = ll[0];
            for (uint32_t i = 0; i < size; ++i) {
              uint32_t cand = ll[1 + i];
              float d = dist(id, cand);
              if (d < curdist) {
                curdist = d;
                curr = cand;
                changed = true;
              }
            }
          }
        }
      }
      for (int level = std::min(cur_level, maxlevel_copy); level >= 0; --level) {
        MaxHeap top = search_base_layer(curr, id, level, visited, tag);
        curr = connect(id, top, level);
      }
    } else {
      enterpoint_ = 0;
      maxlevel_ = cur_level;
    }
    if (cur_level > maxlevel_copy) {
      enterpoint_ = id;
      maxlevel_ = cur_level;
    }
  }

  HostGraph export_graph(uint32_t R) const {  // hnsw_builder.hpp:145-192
    HostGraph g;
    g.n = n_;
    g.R = R;
    g.l0.assign(n_ * R, 0xffffffffu);
    for (uint64_t i = 0; i < n_; ++i) {
      const uint32_t *ll = &links0_[i * (1 + M0_)];
      for (uint32_t j = 0; j < ll[0] && j < R; ++j) g.l0[i * R + j] = ll[1 + j];
    }
    g.has_overlay = true;
    g.upper_R = R;
    g.ep = n_ ? enterpoint_ : 0;
    g.levels.resize(n_);
    g.upper_off.assign(n_, 0);
    uint64_t off = 0;
    for (uint64_t i = 0; i < n_; ++i) {
      g.levels[i] = static_cast<uint32_t>(levels_[i]);
      g.upper_off[i] = off;
      off += static_cast<uint64_t>(levels_[i]) * R;
    }
    g.upper_edges.assign(off, 0xffffffffu);
    for (uint64_t i = 0; i < n_; ++i) {
      for (int l = 1; l <= levels_[i]; ++l) {
        const uint32_t *ll = list(static_cast<uint32_t>(i), l);
        for (uint32_t k = 0; k < ll[0]; ++k) g.upper_edges[g.upper_off[i] + (l - 1) * R + k] = ll[1 + k];
      }
    }
    return g;
  }

  uint64_t size() const { return n_; }

 private:
  static constexpr uint32_t kNone = 0xffffffffu;

  float dist(uint32_t a, uint32_t b) const {
    return host_dist(metric_, data_ + static_cast<uint64_t>(a) * dim_,
                     data_ + static_cast<uint64_t>(b) * dim_, dim_);
  }
  uint32_t *list(uint32_t u, int level) {
    return level == 0 ? &links0_[static_cast<uint64_t>(u) * (1 + M0_)]
                      : &upper_[u][static_cast<size_t>(level - 1) * (1 + M_)];
  }
  const uint32_t *list(uint32_t u, int level) const {
    return level == 0 ? &links0_[static_cast<uint64_t>(u) * (1 + M0_)]
                      : &upper_[u][static_cast<size_t>(level - 1) * (1 + M_)];
  }

  // search_base_layer (hnswlib.hpp:373-489)
  MaxHeap search_base_layer(uint32_t ep, uint32_t q, int layer, std::vector<uint32_t> &visited,
                            uint32_t &tag) {
    if (++tag == 0) {
      std::fill(visited.begin(), visited.end(), 0);
      tag = 1;
    }
    MaxHeap top, cand;
    float d = dist(q, ep);
    top.emplace(d, ep);
    float lower_bound = d;
    cand.emplace(-d, ep);
    visited[ep] = tag;
    while (!cand.empty()) {
      DistId cur = cand.top();
      if (-cur.first > lower_bound && top.size() == efc_) break;
      cand.pop();
      const uint32_t node = cur.second;
      std::unique_lock<std::mutex> lock(locks_[node]);
      const uint32_t *ll = list(node, layer);
      const uint32_t size = ll[0];
      for (uint32_t j = 0; j < size; ++j) {
        uint32_t c = ll[1 + j];
        if (visited[c] == tag) continue;
        visited[c] = tag;
        float d1 = dist(q, c);
        if (top.size() < efc_ || lower_bound > d1) {
          cand.emplace(-d1, c);
          top.emplace(d1, c);
          if (top.size() > efc_) top.pop();
          if (!top.empty()) lower_bound = top.top().first;
        }
      }
    }
    return top;
  }

  // get_neighbors_by_heuristic2 (hnswlib.hpp:291-354)
  void heuristic(MaxHeap &top, size_t m) const {
    if (top.size() < m) return;
    std::priority_queue<DistId> closest;
    std::vector<DistId> ret;
    while (!top.empty()) {
      closest.emplace(-top.top().first, top.top().second);
      top.pop();
    }
    while (!closest.empty()) {
      if (ret.size() >= m) break;
      DistId cur = closest.top();
      float dq = -cur.first;
      closest.pop();
      bool good = true;
      for (const DistId &sel : ret) {
        if (dist(sel.second, cur.second) < dq) {
          good = false;
          break;
        }
      }
      if (good) ret.push_back(cur);
    }
    for (const DistId &p : ret) top.emplace(-p.first, p.second);
  }

  // mutually_connect_new_element (hnswlib.hpp:509-628), isUpdate == false
  uint32_t connect(uint32_t cur_c, MaxHeap &top, int level) {
    const size_t mcurmax = level ? M_ : M0_;
    heuristic(top, M_);
    std::vector<uint32_t> selected;
    selected.reserve(M_);
    while (!top.empty()) {
      selected.push_back(top.top().second);
      top.pop();
    }
    const uint32_t next = selected.back();
    {
      std::unique_lock<std::mutex> lock(locks_[cur_c]);
      uint32_t *ll = list(cur_c, level);
      ll[0] = static_cast<uint32_t>(selected.size());
      for (size_t i = 0; i < selected.size(); ++i) ll[1 + i] = selected[i];
    }
    for (uint32_t other : selected) {
      std::unique_lock<std::mutex> lock(locks_[other]);
      uint32_t *ll = list(other, level);
      const size_t sz = ll[0];
      if (sz < mcurmax) {
        ll[1 + sz] = cur_c;
        ll[0] = static_cast<uint32_t>(sz + 1);
      } else {
        MaxHeap cands;
        cands.emplace(dist(cur_c, other), cur_c);
        for (size_t j = 0; j < sz; ++j) cands.emplace(dist(ll[1 + j], other), ll[1 + j]);
        heuristic(cands, mcurmax);
        uint32_t idx = 0;
        while (!cands.empty()) {
          ll[1 + idx] = cands.top().second;
          cands.pop();
          ++idx;
        }
        ll[0] = idx;
      }
    }
    return next;
  }

  const float *data_;
  uint64_t n_;
  uint32_t dim_;
  int metric_;
  size_t M_, M0_, efc_;
  std::vector<std::mutex> locks_;
  std::mutex global_;
  std::vector<int> levels_;
  std::vector<uint32_t> links0_;
  std::vector<std::vector<uint32_t>> upper_;
  uint32_t enterpoint_ = kNone;
  int maxlevel_ = -1;
};

}  // namespace

HostGraph build_hnsw(const float *data, uint64_t n, uint32_t dim, int metric, uint32_t R,
                     uint32_t ef_construction, uint32_t num_threads, uint64_t seed) {
  if (R < 2) throw std::runtime_error("max_nbrs must be >= 2");
  HostGraph g;
  if (n == 0) {
    g.R = R;
    g.has_overlay = true;
    return g;
  }
  Builder b(data, n, dim, metric, R / 2, ef_construction, seed);
  {
    std::vector<uint32_t> visited(n, 0);
    uint32_t tag = 0;
    b.add_point(0, visited, tag);
  }
  std::atomic<uint64_t> next{1};
  auto work = [&]() {
    std::vector<uint32_t> visited(n, 0);
    uint32_t tag = 0;
    for (;;) {
      uint64_t i = next.fetch_add(1);
      if (i >= n) break;
      b.add_point(static_cast<uint32_t>(i), visited, tag);
    }
  };
  const uint32_t nt = std::max(1u, num_threads);
  if (nt == 1) {
    work();
  } else {
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < nt; ++t) ts.emplace_back(work);
    for (auto &t : ts) t.join();
  }
  return b.export_graph(R);
}

// ---------------------------------------------------------------------------------------------
// Reference on-disk format.
// ---------------------------------------------------------------------------------------------
namespace {
template <typename T>
void put(std::ofstream &w, T v) {
  w.write(reinterpret_cast<const char *>(&v), sizeof(T));
}
template <typename T>
T get(std::ifstream &r) {
  T v{};
  r.read(reinterpret_cast<char *>(&v), sizeof(T));
  if (!r) throw std::runtime_error("truncated graph file");
  return v;
}
}  // namespace

void save_graph(const HostGraph &g, const std::string &path, int id_bytes, uint64_t capacity,
                const uint8_t *valid) {
  if (id_bytes != 4 && id_bytes != 8) throw std::runtime_error("id_bytes must be 4 or 8");
  capacity = std::max<uint64_t>(capacity, g.n);
  std::ofstream w(path, std::ios::binary);
  if (!w.is_open()) throw std::runtime_error("Cannot open file " + path);
  // graph.hpp:176-183: nep, eps, max_nodes_, max_nbrs_ (written with sizeof(IDType) bytes).
  const std::vector<uint32_t> eps = g.has_overlay ? std::vector<uint32_t>{} : g.eps;
  put<int32_t>(w, static_cast<int32_t>(eps.size()));
  for (uint32_t e : eps) id_bytes == 4 ? put<uint32_t>(w, e) : put<uint64_t>(w, e);
  if (id_bytes == 4) {
    put<uint32_t>(w, static_cast<uint32_t>(capacity));
    put<uint32_t>(w, g.R);
  } else {
    put<uint64_t>(w, capacity);
    put<uint64_t>(w, g.R);
  }
  // SequentialStorage::save (sequential_storage.hpp:110-119)
  const uint64_t item = static_cast<uint64_t>(g.R) * id_bytes;
  const uint64_t aligned = (item + 63) / 64 * 64;
  put<uint64_t>(w, item);
  put<uint64_t>(w, aligned);
  put<uint64_t>(w, capacity);
  put<uint64_t>(w, g.n);
  put<uint64_t>(w, 64);
  std::vector<char> row(aligned, static_cast<char>(0xff));
  for (uint64_t i = 0; i < capacity; ++i) {
    std::fill(row.begin(), row.end(), static_cast<char>(0xff));
    if (i < g.n) {
      for (uint32_t j = 0; j < g.R; ++j) {
        uint32_t v = g.l0[i * g.R + j];
        if (id_bytes == 4) {
          std::memcpy(&row[j * 4], &v, 4);
        } else {
          uint64_t v64 = v == 0xffffffffu ? ~0ull : v;
          std::memcpy(&row[j * 8], &v64, 8);
        }
      }
    }
    w.write(row.data(), aligned);
  }
  // Graph::insert sets a node's bit, Graph::remove (GraphUpdateJob::remove,
  // graph_update_job.hpp:91-103 -> sequential_storage.hpp:94-100) clears it again.
  std::vector<uint8_t> bitmap((capacity + 7) / 8, 0);
  for (uint64_t i = 0; i < g.n; ++i)
    if (valid == nullptr || ((valid[i / 8] >> (i % 8)) & 1)) bitmap[i / 8] |= static_cast<uint8_t>(1u << (i % 8));
  w.write(reinterpret_cast<const char *>(bitmap.data()), bitmap.size());
  if (g.has_overlay) {  // overlay_graph.hpp:183-194
    // node_num_ and ep_ are IDType but written with 4 bytes (the low half on little-endian hosts);
    // each node's list is levels * max_nbrs IDType entries written with `cur * 4` bytes, so for
    // 64-bit ids only the first cur / 2 entries reach the file (the reference's own width quirk).
    put<uint32_t>(w, static_cast<uint32_t>(capacity));
    put<uint32_t>(w, g.upper_R);
    put<uint32_t>(w, g.ep);
    std::vector<uint64_t> wide;
    for (uint64_t i = 0; i < capacity; ++i) {
      const uint32_t lvl = i < g.n ? g.levels[i] : 0;
      const uint64_t cur = static_cast<uint64_t>(lvl) * g.upper_R;
      put<int32_t>(w, static_cast<int32_t>(cur));
      if (!cur) continue;
      const uint32_t *src = &g.upper_edges[g.upper_off[i]];
      if (id_bytes == 4) {
        w.write(reinterpret_cast<const char *>(src), static_cast<std::streamsize>(cur) * 4);
      } else {
        wide.assign(cur, 0);
        for (uint64_t j = 0; j < cur; ++j) wide[j] = src[j] == 0xffffffffu ? ~0ull : src[j];
        w.write(reinterpret_cast<const char *>(wide.data()), static_cast<std::streamsize>(cur) * 4);
      }
    }
  }
  if (!w) throw std::runtime_error("write failed: " + path);
}

HostGraph load_graph(const std::string &path, int id_bytes) {
  if (id_bytes != 4 && id_bytes != 8) throw std::runtime_error("id_bytes must be 4 or 8");
  std::ifstream r(path, std::ios::binary);
  if (!r.is_open()) throw std::runtime_error("Cannot open file " + path);
  HostGraph g;
  const int32_t nep = get<int32_t>(r);
  if (nep < 0) throw std::runtime_error("corrupt graph file");
  for (int32_t i = 0; i < nep; ++i)
    g.eps.push_back(id_bytes == 4 ? get<uint32_t>(r) : static_cast<uint32_t>(get<uint64_t>(r)));
  uint64_t max_nodes;
  if (id_bytes == 4) {
    max_nodes = get<uint32_t>(r);
    g.R = get<uint32_t>(r);
  } else {
    max_nodes = get<uint64_t>(r);
    g.R = static_cast<uint32_t>(get<uint64_t>(r));
  }
  const uint64_t item = get<uint64_t>(r);
  const uint64_t aligned = get<uint64_t>(r);
  const uint64_t capacity = get<uint64_t>(r);
  const uint64_t pos = get<uint64_t>(r);
  (void)get<uint64_t>(r);  // alignment
  if (item != static_cast<uint64_t>(g.R) * id_bytes || aligned < item || capacity != max_nodes ||
      pos > capacity)
    throw std::runtime_error("corrupt graph file (storage header)");
  g.n = pos;
  g.l0.assign(pos * g.R, 0xffffffffu);
  std::vector<char> row(aligned);
  for (uint64_t i = 0; i < capacity; ++i) {
    r.read(row.data(), static_cast<std::streamsize>(aligned));
    if (!r) throw std::runtime_error("truncated graph file");
    if (i >= pos) continue;
    for (uint32_t j = 0; j < g.R; ++j) {
      if (id_bytes == 4) {
        std::memcpy(&g.l0[i * g.R + j], &row[j * 4], 4);
      } else {
        uint64_t v;
        std::memcpy(&v, &row[j * 8], 8);
        g.l0[i * g.R + j] = v == ~0ull ? 0xffffffffu : static_cast<uint32_t>(v);
      }
    }
  }
  r.ignore(static_cast<std::streamsize>((capacity + 7) / 8));
  if (r.peek() != EOF) {  // graph.hpp:233-236
    g.has_overlay = true;
    const uint32_t node_num = get<uint32_t>(r);
    g.upper_R = get<uint32_t>(r);
    g.ep = get<uint32_t>(r);
    if (g.upper_R == 0) throw std::runtime_error("corrupt overlay");
    g.levels.assign(g.n, 0);
    g.upper_off.assign(g.n, 0);
    for (uint32_t i = 0; i < node_num; ++i) {
      const int32_t cur = get<int32_t>(r);
      if (cur < 0) throw std::runtime_error("corrupt overlay");
      // OverlayGraph::load reads cur * 4 bytes into a list of cur IDType entries pre-filled with -1
      // (overlay_graph.hpp:151-170): for 64-bit ids the first cur / 2 entries, the rest stay -1
      std::vector<uint32_t> buf(cur, 0xffffffffu);
      if (cur && id_bytes == 4) {
        r.read(reinterpret_cast<char *>(buf.data()), static_cast<std::streamsize>(cur) * 4);
      } else if (cur) {
        std::vector<uint64_t> wide(cur, ~0ull);
        r.read(reinterpret_cast<char *>(wide.data()), static_cast<std::streamsize>(cur) * 4);
        for (int32_t j = 0; j < cur; ++j) buf[j] = wide[j] == ~0ull ? 0xffffffffu : static_cast<uint32_t>(wide[j]);
      }
      if (!r) throw std::runtime_error("truncated overlay");
      if (i < g.n) {
        g.levels[i] = static_cast<uint32_t>(cur) / g.upper_R;
        g.upper_off[i] = g.upper_edges.size();
        g.upper_edges.insert(g.upper_edges.end(), buf.begin(), buf.end());
      }
    }
  }
  return g;
}

}  // namespace alaya_amd
