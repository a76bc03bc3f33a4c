// TEST INFRASTRUCTURE ONLY -- CPU restatement of the AlayaLite search hot path (see oracle.h).
// Written from the reference's source text; no reference code is compiled, linked or copied.
// Built with -O2 -ffp-contract=off (no -ffast-math): every multiply-add below is an explicit fmaf
// and every add is a separate rounding, so the arithmetic order is exactly the one written here.
#include "oracle.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <unordered_map>
#include <unordered_set>
#include <cmath>
#include <coroutine>
#include <cstring>
#include <deque>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

namespace {

// ------------------------------------------------------------------------------------------
// Distances.  l2_sqr_avx2 (distance_l2.ipp:54-116): 4 accumulators x 8 lanes; element 32t+8a+l
// feeds acc[a][l] by fma(diff, diff, acc); remaining 8-blocks feed acc[0][l]; combine
// v[l] = (acc0+acc1)[l] + (acc2+acc3)[l]; s[j] = v[j] + v[j+4]; r = (s0+s1) + (s2+s3)
// (movehdup/movehl/add_ss, :100-108); scalar tail r = fma(diff, diff, r) (-Ofast + target fma
// contracts `result += diff*diff`, :111-114).  Here acc[j], j = 8a+l.
// ------------------------------------------------------------------------------------------
template <bool kIP>
inline float avx2_order(const float *x, const float *y, size_t dim) {
  float acc[32];
  for (float &a : acc) a = 0.0f;
  size_t i = 0;
  for (; i + 32 <= dim; i += 32) {
    for (int j = 0; j < 32; ++j) {
      if (kIP) {
        acc[j] = fmaf(x[i + j], y[i + j], acc[j]);
      } else {
        float d = x[i + j] - y[i + j];
        acc[j] = fmaf(d, d, acc[j]);
      }
    }
  }
  for (; i + 8 <= dim; i += 8) {
    for (int l = 0; l < 8; ++l) {
      if (kIP) {
        acc[l] = fmaf(x[i + l], y[i + l], acc[l]);
      } else {
        float d = x[i + l] - y[i + l];
        acc[l] = fmaf(d, d, acc[l]);
      }
    }
  }
  float v[8];
  for (int l = 0; l < 8; ++l) {
    float a01 = acc[l] + acc[8 + l];
    float a23 = acc[16 + l] + acc[24 + l];
    v[l] = a01 + a23;
  }
  float s[4];
  for (int j = 0; j < 4; ++j) s[j] = v[j] + v[j + 4];
  float r = (s[0] + s[1]) + (s[2] + s[3]);
  for (; i < dim; ++i) {
    if (kIP) {
      r = fmaf(x[i], y[i], r);
    } else {
      float d = x[i] - y[i];
      r = fmaf(d, d, r);
    }
  }
  return kIP ? -r : r;
}

// Same order with AVX2 intrinsics -- used by the CPU baseline (speed) and cross-checked
// bit-for-bit against avx2_order by tests/test_oracle.py.
template <bool kIP>
__attribute__((target("avx2,fma"))) float avx2_intrin(const float *x, const float *y,
                                                      size_t dim) {
  __m256 a0 = _mm256_setzero_ps(), a1 = _mm256_setzero_ps();
  __m256 a2 = _mm256_setzero_ps(), a3 = _mm256_setzero_ps();
  size_t i = 0;
  for (; i + 32 <= dim; i += 32) {
    __m256 x0 = _mm256_loadu_ps(x + i), y0 = _mm256_loadu_ps(y + i);
    __m256 x1 = _mm256_loadu_ps(x + i + 8), y1 = _mm256_loadu_ps(y + i + 8);
    __m256 x2 = _mm256_loadu_ps(x + i + 16), y2 = _mm256_loadu_ps(y + i + 16);
    __m256 x3 = _mm256_loadu_ps(x + i + 24), y3 = _mm256_loadu_ps(y + i + 24);
    if (kIP) {
      a0 = _mm256_fmadd_ps(x0, y0, a0);
      a1 = _mm256_fmadd_ps(x1, y1, a1);
      a2 = _mm256_fmadd_ps(x2, y2, a2);
      a3 = _mm256_fmadd_ps(x3, y3, a3);
    } else {
      __m256 d0 = _mm256_sub_ps(x0, y0), d1 = _mm256_sub_ps(x1, y1);
      __m256 d2 = _mm256_sub_ps(x2, y2), d3 = _mm256_sub_ps(x3, y3);
      a0 = _mm256_fmadd_ps(d0, d0, a0);
      a1 = _mm256_fmadd_ps(d1, d1, a1);
      a2 = _mm256_fmadd_ps(d2, d2, a2);
      a3 = _mm256_fmadd_ps(d3, d3, a3);
    }
  }
  for (; i + 8 <= dim; i += 8) {
    __m256 xv = _mm256_loadu_ps(x + i), yv = _mm256_loadu_ps(y + i);
    if (kIP) {
      a0 = _mm256_fmadd_ps(xv, yv, a0);
    } else {
      __m256 d = _mm256_sub_ps(xv, yv);
      a0 = _mm256_fmadd_ps(d, d, a0);
    }
  }
  __m256 v = _mm256_add_ps(_mm256_add_ps(a0, a1), _mm256_add_ps(a2, a3));
  __m128 s = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
  __m128 h = _mm_movehdup_ps(s);
  s = _mm_add_ps(s, h);
  h = _mm_movehl_ps(h, s);
  s = _mm_add_ss(s, h);
  float r = _mm_cvtss_f32(s);
  for (; i < dim; ++i) {
    if (kIP) {
      r = fmaf(x[i], y[i], r);
    } else {
      float d = x[i] - y[i];
      r = fmaf(d, d, r);
    }
  }
  return kIP ? -r : r;
}

template <typename T>
float generic_l2(const T *x, const T *y, size_t dim) {
  float sum = 0.0f;
  for (size_t i = 0; i < dim; ++i) {
    float d = static_cast<float>(x[i]) - static_cast<float>(y[i]);
    sum += d * d;
  }
  return sum;
}

template <typename T>
float generic_ip(const T *x, const T *y, size_t dim) {
  float sum = 0.0f;
  for (size_t i = 0; i < dim; ++i) sum += static_cast<float>(x[i]) * static_cast<float>(y[i]);
  return -sum;
}

bool g_has_avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");

inline float fast_dist(int metric, const float *x, const float *y, size_t dim) {
  if (g_has_avx2) {
    return metric == ORC_L2 ? avx2_intrin<false>(x, y, dim) : avx2_intrin<true>(x, y, dim);
  }
  return metric == ORC_L2 ? avx2_order<false>(x, y, dim) : avx2_order<true>(x, y, dim);
}

// ------------------------------------------------------------------------------------------
// LinearPool (query_utils.hpp:236-312).  Storage capacity+1 value-initialised Neighbors; bit 31
// of the id is the "checked" flag; insert = reject-if-full-and-d>=last, upper_bound, memmove.
// ------------------------------------------------------------------------------------------
struct Nb {
  uint32_t id;
  float dist;
};

struct Pool {
  size_t size = 0, cur = 0, cap;
  std::vector<Nb> data;
  std::vector<uint64_t> vis;  // DynamicBitset (query_utils.hpp:69-115)

  Pool(uint64_t n, int capacity) : cap(capacity), data(capacity + 1, Nb{0, 0.0f}),
                                   vis((n + 63) / 64, 0) {}

  size_t upper_bound(float d) const {  // find_bsearch :240-252
    size_t l = 0, r = size;
    while (l < r) {
      size_t mid = (l + r) / 2;
      if (data[mid].dist > d) r = mid; else l = mid + 1;
    }
    return l;
  }
  bool insert(uint32_t u, float d) {  // :254-272
    if (size == cap && d >= data[size - 1].dist) return false;
    size_t lo = upper_bound(d);
    std::memmove(&data[lo + 1], &data[lo], (size - lo) * sizeof(Nb));
    data[lo] = Nb{u, d};
    if (size < cap) size++;
    if (lo < cur) cur = lo;
    return true;
  }
  static bool checked(uint32_t id) { return (id >> 31) & 1u; }
  uint32_t pop() {  // :284-293
    data[cur].id |= 1u << 31;
    size_t pre = cur;
    while (cur < size && checked(data[cur].id)) cur++;
    return data[pre].id & 0x7fffffffu;
  }
  bool has_next() const { return cur < size; }
  uint32_t id(size_t i) const { return data[i].id & 0x7fffffffu; }
  bool vis_get(uint32_t v) const { return (vis[v >> 6] >> (v & 63)) & 1ull; }
  void vis_set(uint32_t v) { vis[v >> 6] |= 1ull << (v & 63); }
};

// ------------------------------------------------------------------------------------------
// QueryComputer (raw_space.hpp:255-305): FLT_MAX for invalid rows, else dist(query, row).
// COS queries are normalised by the caller (the reference normalises the caller's buffer).
// ------------------------------------------------------------------------------------------
float sq8_dist_any(int metric, const uint8_t *x, const uint8_t *y, size_t dim, const float *mn,
                   const float *mx, int variant);
void sq8_encode_row(const float *row, uint32_t dim, const float *mn, const float *mx, uint8_t *code);

struct QC {
  const orc_index *ix;
  const float *q;
  std::vector<uint8_t> qcode;  // SQ8 QueryComputer encodes the query (sq8_space.hpp:266-271)
  QC(const orc_index *i, const float *query) : ix(i), q(query) {
    if (ix->space == 1) {
      qcode.resize(ix->dim);
      sq8_encode_row(query, ix->dim, ix->sq_min, ix->sq_max, qcode.data());
    }
  }
  float operator()(uint32_t u) const {
    if (ix->space == 1)  // no validity check in SQ8Space::QueryComputer (sq8_space.hpp:290-297)
      return sq8_dist_any(ix->metric, qcode.data(), ix->codes + static_cast<uint64_t>(u) * ix->code_stride,
                          ix->dim, ix->sq_min, ix->sq_max, ix->sq8_variant);
    if (ix->valid && !((ix->valid[u >> 3] >> (u & 7)) & 1)) return FLT_MAX;
    const float *row = ix->base + static_cast<uint64_t>(u) * ix->stride;
    if (ix->generic)
      return ix->metric == ORC_L2 ? generic_l2(q, row, ix->dim) : generic_ip(q, row, ix->dim);
    return fast_dist(ix->metric, q, row, ix->dim);
  }
};

inline const uint32_t *upper_list(const orc_index *ix, uint32_t u, uint32_t level) {
  return ix->upper_edges + ix->upper_off[u] + static_cast<uint64_t>(level - 1) * ix->upper_R;
}

// Graph::initialize_search (graph.hpp:148-158) -> OverlayGraph::initialize
// (overlay_graph.hpp:122-144): greedy descent, strict <, only the final node is marked visited.
void initialize_search(const orc_index *ix, Pool &pool, const QC &qc, orc_counters *cnt) {
  if (ix->levels == nullptr) {
    pool.insert(ix->ep, qc(ix->ep));
    pool.vis_set(ix->ep);
    if (cnt) cnt->n_dist_upper++;
    return;
  }
  uint32_t u = ix->ep;
  float cur = qc(u);
  if (cnt) cnt->n_dist_upper++;
  for (int level = static_cast<int>(ix->levels[u]); level > 0; --level) {
    bool changed = true;
    while (changed) {
      changed = false;
      const uint32_t *list = upper_list(ix, u, level);
      if (cnt) cnt->n_hops_upper++;
      for (uint32_t i = 0; i < ix->upper_R && list[i] != 0xffffffffu; ++i) {
        uint32_t v = list[i];
        float d = qc(v);
        if (cnt) cnt->n_dist_upper++;
        if (d < cur) {
          cur = d;
          u = v;
          changed = true;
        }
      }
    }
  }
  pool.insert(u, cur);
  pool.vis_set(u);
}

// ------------------------------------------------------------------------------------------
// Coroutine plumbing for the batch baseline (own minimal task type; the reference uses
// libcoro's coro::task<>, which only provides the handle -- results do not depend on it).
// ------------------------------------------------------------------------------------------
struct Task {
  struct promise_type {
    Task get_return_object() { return Task{std::coroutine_handle<promise_type>::from_promise(*this)}; }
    std::suspend_always initial_suspend() noexcept { return {}; }
    std::suspend_always final_suspend() noexcept { return {}; }
    void return_void() {}
    void unhandled_exception() { std::terminate(); }
  };
  std::coroutine_handle<promise_type> h;
};

// GraphSearchJob::search (graph_search_job.hpp:221-299): same algorithm as search_solo with a
// suspension after each pop (edge-list prefetch) and before each distance (row prefetch).
Task search_coro(const orc_index *ix, const float *query, uint32_t k, uint32_t ef, uint32_t *ids,
                 float *dists, orc_counters *cnt) {
  QC qc(ix, query);
  Pool pool(ix->n, static_cast<int>(ef));
  initialize_search(ix, pool, qc, cnt);
  while (pool.has_next()) {
    uint32_t u = pool.pop();
    if (cnt) cnt->n_expand++;
    const uint32_t *adj = ix->l0 + static_cast<uint64_t>(u) * ix->R;
    _mm_prefetch(reinterpret_cast<const char *>(adj), _MM_HINT_T0);
    co_await std::suspend_always{};
    for (uint32_t i = 0; i < ix->R; ++i) {
      uint32_t v = adj[i];
      if (v == 0xffffffffu) break;
      if (pool.vis_get(v)) continue;
      pool.vis_set(v);
      const char *row = reinterpret_cast<const char *>(ix->base + static_cast<uint64_t>(v) * ix->stride);
      for (uint32_t off = 0; off < ix->dim * 4; off += 64) _mm_prefetch(row + off, _MM_HINT_T0);
      co_await std::suspend_always{};
      float d = qc(v);
      if (cnt) cnt->n_dist++;
      pool.insert(v, d);
    }
  }
  for (uint32_t i = 0; i < k; ++i) {
    ids[i] = pool.id(i);
    if (dists) dists[i] = pool.data[i].dist;
  }
  co_return;
}

// Scheduler + Worker (scheduler.hpp:113-203, worker.hpp:111-136): a shared queue guarded by a
// lock, N workers each round-robin over 4 local handles, exit when finished == total.
struct TaskQueue {
  std::mutex mu;
  std::deque<std::coroutine_handle<>> q;
  bool pop(std::coroutine_handle<> &h) {
    std::lock_guard<std::mutex> g(mu);
    if (q.empty()) return false;
    h = q.front();
    q.pop_front();
    return true;
  }
};

// SQ8 kernels.  Per element: scale = (max-min)*(1/255); L2: diff = (xf-yf)*scale,
// acc = fma(diff,diff,acc); IP: xv = fma(xf,scale,min), yv = fma(yf,scale,min), acc = fma(xv,yv,acc).
// AVX-512 (distance_l2.ipp:334-408): sum0 <- 32t+l, sum1 <- 32t+16+l (l<16), a remaining 16-block
// -> sum0; combine sum0+sum1, then GCC 11 _mm512_reduce_add_ps (avx512fintrin.h:16112-16127).
// AVX2 (distance_l2.ipp:244-329): sum0 <- 16t+l, sum1 <- 16t+8+l, remaining 8-block -> sum0,
// combine + the AVX2 horizontal tree.  Generic: sequential.
template <bool kIP>
inline float sq8_term(uint8_t xc, uint8_t yc, float mn, float mx, float acc) {
  const float kInv255 = 1.0f / 255.0f;
  float scale = (mx - mn) * kInv255;
  float xf = static_cast<float>(xc), yf = static_cast<float>(yc);
  if (kIP) {
    float xv = fmaf(xf, scale, mn);
    float yv = fmaf(yf, scale, mn);
    return fmaf(xv, yv, acc);
  }
  float d = (xf - yf) * scale;
  return fmaf(d, d, acc);
}

template <bool kIP>
float sq8_dist(const uint8_t *x, const uint8_t *y, size_t dim, const float *mn, const float *mx,
               int variant) {
  size_t i = 0;
  float r;
  if (variant == 2) {
    float s0[16] = {0}, s1[16] = {0};
    for (; i + 32 <= dim; i += 32) {
      for (int l = 0; l < 16; ++l) s0[l] = sq8_term<kIP>(x[i + l], y[i + l], mn[i + l], mx[i + l], s0[l]);
      for (int l = 0; l < 16; ++l)
        s1[l] = sq8_term<kIP>(x[i + 16 + l], y[i + 16 + l], mn[i + 16 + l], mx[i + 16 + l], s1[l]);
    }
    for (; i + 16 <= dim; i += 16)
      for (int l = 0; l < 16; ++l) s0[l] = sq8_term<kIP>(x[i + l], y[i + l], mn[i + l], mx[i + l], s0[l]);
    float a[16];
    for (int l = 0; l < 16; ++l) a[l] = s0[l] + s1[l];
    float t3[8], t6[4];
    for (int j = 0; j < 8; ++j) t3[j] = a[8 + j] + a[j];
    for (int j = 0; j < 4; ++j) t6[j] = t3[4 + j] + t3[j];
    float t80 = t6[0] + t6[2], t81 = t6[1] + t6[3];
    r = t80 + t81;
  } else if (variant == 1) {
    float s0[8] = {0}, s1[8] = {0};
    for (; i + 16 <= dim; i += 16) {
      for (int l = 0; l < 8; ++l) s0[l] = sq8_term<kIP>(x[i + l], y[i + l], mn[i + l], mx[i + l], s0[l]);
      for (int l = 0; l < 8; ++l)
        s1[l] = sq8_term<kIP>(x[i + 8 + l], y[i + 8 + l], mn[i + 8 + l], mx[i + 8 + l], s1[l]);
    }
    for (; i + 8 <= dim; i += 8)
      for (int l = 0; l < 8; ++l) s0[l] = sq8_term<kIP>(x[i + l], y[i + l], mn[i + l], mx[i + l], s0[l]);
    float v[8];
    for (int l = 0; l < 8; ++l) v[l] = s0[l] + s1[l];
    float s[4];
    for (int j = 0; j < 4; ++j) s[j] = v[j] + v[j + 4];
    r = (s[0] + s[1]) + (s[2] + s[3]);
  } else {
    r = 0.0f;
    const float kInv255 = 1.0f / 255.0f;
    for (; i < dim; ++i) {
      float scale = (mx[i] - mn[i]) * kInv255;
      if (kIP) {
        float xv = mn[i] + static_cast<float>(x[i]) * scale;
        float yv = mn[i] + static_cast<float>(y[i]) * scale;
        r += xv * yv;
      } else {
        float d = (static_cast<float>(x[i]) - static_cast<float>(y[i])) * scale;
        r += d * d;
      }
    }
    return kIP ? -r : r;
  }
  for (; i < dim; ++i) r = sq8_term<kIP>(x[i], y[i], mn[i], mx[i], r);
  return kIP ? -r : r;
}

float sq8_dist_any(int metric, const uint8_t *x, const uint8_t *y, size_t dim, const float *mn,
                   const float *mx, int variant) {
  return metric == ORC_L2 ? sq8_dist<false>(x, y, dim, mn, mx, variant)
                          : sq8_dist<true>(x, y, dim, mn, mx, variant);
}

void sq8_encode_row(const float *row, uint32_t dim, const float *mn, const float *mx, uint8_t *code) {
  for (uint32_t j = 0; j < dim; ++j) {  // SQ8Quantizer::quantize (sq8.hpp:118-130)
    float v = row[j], lo = mn[j], hi = mx[j];
    uint8_t c;
    if (hi == lo) c = 0;
    else if (v >= hi) c = 255;
    else if (v <= lo) c = 0;
    else c = static_cast<uint8_t>(((v - lo) / (hi - lo)) * 255);
    code[j] = c;
  }
}

}  // namespace

extern "C" {

float orc_l2_f32(const float *x, const float *y, size_t dim) { return avx2_order<false>(x, y, dim); }
float orc_ip_f32(const float *x, const float *y, size_t dim) { return avx2_order<true>(x, y, dim); }
float orc_l2_f32_avx2(const float *x, const float *y, size_t dim) {
  return avx2_intrin<false>(x, y, dim);
}
float orc_ip_f32_avx2(const float *x, const float *y, size_t dim) {
  return avx2_intrin<true>(x, y, dim);
}
int orc_cpu_has_avx2_fma(void) { return g_has_avx2 ? 1 : 0; }
int orc_cpu_has_avx512f(void) { return __builtin_cpu_supports("avx512f") ? 1 : 0; }

float orc_l2_generic(const void *x, const void *y, size_t dim, int dtype) {
  switch (dtype) {
    case 0: return generic_l2(static_cast<const float *>(x), static_cast<const float *>(y), dim);
    case 1: return generic_l2(static_cast<const int8_t *>(x), static_cast<const int8_t *>(y), dim);
    case 2: return generic_l2(static_cast<const uint8_t *>(x), static_cast<const uint8_t *>(y), dim);
    case 3: return generic_l2(static_cast<const double *>(x), static_cast<const double *>(y), dim);
    case 4: return generic_l2(static_cast<const int32_t *>(x), static_cast<const int32_t *>(y), dim);
    case 5: return generic_l2(static_cast<const uint32_t *>(x), static_cast<const uint32_t *>(y), dim);
    default: return NAN;
  }
}
float orc_ip_generic(const void *x, const void *y, size_t dim, int dtype) {
  switch (dtype) {
    case 0: return generic_ip(static_cast<const float *>(x), static_cast<const float *>(y), dim);
    case 1: return generic_ip(static_cast<const int8_t *>(x), static_cast<const int8_t *>(y), dim);
    case 2: return generic_ip(static_cast<const uint8_t *>(x), static_cast<const uint8_t *>(y), dim);
    case 3: return generic_ip(static_cast<const double *>(x), static_cast<const double *>(y), dim);
    case 4: return generic_ip(static_cast<const int32_t *>(x), static_cast<const int32_t *>(y), dim);
    case 5: return generic_ip(static_cast<const uint32_t *>(x), static_cast<const uint32_t *>(y), dim);
    default: return NAN;
  }
}

// data_utils.hpp:36-46: float sum of squares, 1.0/sqrt in double, rounded to float, then scale.
void orc_normalize(float *v, size_t dim) {
  float sum = 0.0f;
  for (size_t i = 0; i < dim; ++i) sum += v[i] * v[i];
  sum = static_cast<float>(1.0 / std::sqrt(static_cast<double>(sum)));
  for (size_t i = 0; i < dim; ++i) v[i] *= sum;
}

struct orc_pool {
  Pool p;
};
orc_pool *orc_pool_new(uint32_t n, int capacity) { return new orc_pool{Pool(n, capacity)}; }
void orc_pool_free(orc_pool *p) { delete p; }
int orc_pool_insert(orc_pool *p, uint32_t id, float dist) { return p->p.insert(id, dist) ? 1 : 0; }
uint32_t orc_pool_pop(orc_pool *p) { return p->p.pop(); }
uint32_t orc_pool_top(orc_pool *p) { return p->p.data[p->p.cur].id; }
int orc_pool_has_next(const orc_pool *p) { return p->p.has_next() ? 1 : 0; }
size_t orc_pool_size(const orc_pool *p) { return p->p.size; }
uint32_t orc_pool_id(const orc_pool *p, size_t i) { return p->p.id(i); }
float orc_pool_dist(const orc_pool *p, size_t i) { return p->p.data[i].dist; }

// GraphSearchJob::search_solo (graph_search_job.hpp:302-371).
void orc_search(const orc_index *ix, const float *query, uint32_t k, uint32_t ef, uint32_t *ids,
                float *dists, orc_counters *cnt) {
  QC qc(ix, query);
  Pool pool(ix->n, static_cast<int>(ef));
  initialize_search(ix, pool, qc, cnt);
  while (pool.has_next()) {
    uint32_t u = pool.pop();
    if (cnt) cnt->n_expand++;
    const uint32_t *adj = ix->l0 + static_cast<uint64_t>(u) * ix->R;
    for (uint32_t i = 0; i < ix->R; ++i) {
      uint32_t v = adj[i];
      if (v == 0xffffffffu) break;
      if (pool.vis_get(v)) continue;
      pool.vis_set(v);
      float d = qc(v);
      if (cnt) cnt->n_dist++;
      pool.insert(v, d);
    }
  }
  for (uint32_t i = 0; i < k; ++i) {
    ids[i] = pool.id(i);
    if (dists) dists[i] = pool.data[i].dist;
  }
}

double orc_batch_search_coro(const orc_index *ix, const float *queries, uint64_t nq, uint32_t k,
                             uint32_t ef, uint32_t num_threads, uint32_t *ids, float *dists,
                             orc_counters *cnt) {
  std::vector<Task> tasks;
  tasks.reserve(nq);
  TaskQueue queue;
  for (uint64_t i = 0; i < nq; ++i) {
    tasks.push_back(search_coro(ix, queries + i * ix->dim, k, ef, ids + i * k,
                                dists ? dists + i * k : nullptr, cnt ? cnt + i : nullptr));
    queue.q.push_back(tasks.back().h);
  }
  const size_t total = nq;
  std::atomic<size_t> finished{0};
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> workers;
  for (uint32_t w = 0; w < std::max(1u, num_threads); ++w) {
    workers.emplace_back([&] {
      constexpr uint32_t kLocal = 4;  // worker.hpp:47
      std::coroutine_handle<> local[kLocal] = {};
      uint32_t nav = 0;
      while (true) {
        auto &h = local[nav++ % kLocal];
        if (!h) {
          if (!queue.pop(h)) {
            if (finished.load() == total) break;
            continue;
          }
        }
        h.resume();
        if (h.done()) {
          h = nullptr;
          finished.fetch_add(1);
        }
      }
    });
  }
  for (auto &t : workers) t.join();
  double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (auto &t : tasks) t.h.destroy();
  return sec;
}

// ---- SQ8 (space/quant/sq8.hpp:78-143) ------------------------------------------------------
void orc_sq8_fit(const float *data, uint64_t n, uint32_t dim, float *min_v, float *max_v) {
  for (uint32_t j = 0; j < dim; ++j) {
    min_v[j] = FLT_MAX;
    max_v[j] = -FLT_MAX;
  }
  for (uint64_t i = 0; i < n; ++i) {
    for (uint32_t j = 0; j < dim; ++j) {
      float v = data[i * dim + j];
      if (v < min_v[j]) min_v[j] = v;
      if (v > max_v[j]) max_v[j] = v;
    }
  }
}

void orc_sq8_encode(const float *row, uint32_t dim, const float *min_v, const float *max_v,
                    uint8_t *code) {
  sq8_encode_row(row, dim, min_v, max_v, code);
}

void orc_rerank(const orc_index *ix, const float *query, const uint32_t *search_ids, uint32_t k,
                uint32_t ef, uint32_t *ids, float *dists) {
  orc_index raw = *ix;
  raw.space = 0;
  QC qc(&raw, query);
  std::vector<uint32_t> src(std::max(ef, k), 0u);  // res_pool(ef): zeros past the k written ids
  for (uint32_t i = 0; i < k; ++i) src[i] = search_ids[i];
  std::priority_queue<std::pair<float, uint32_t>, std::vector<std::pair<float, uint32_t>>,
                      std::greater<>> pq;
  for (uint32_t i = 0; i < ef; ++i) pq.push({qc(src[i]), src[i]});
  for (uint32_t i = 0; i < k; ++i) {
    if (pq.empty()) {
      ids[i] = 0;
      dists[i] = 0.0f;
      continue;
    }
    dists[i] = pq.top().first;
    ids[i] = pq.top().second;
    pq.pop();
  }
}

// The Linux batch path's rerank loop after Scheduler::join (index.hpp:337-345): one thread, query
// by query.  Returns its seconds (outside the reference's Timer, but part of batch_search).
double orc_exact_gt(const float *base, uint64_t n, uint32_t dim, const float *queries, uint64_t nq,
                    uint32_t k, uint32_t num_threads, uint32_t *ids) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool avx2 = orc_cpu_has_avx2_fma() != 0;
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<std::pair<uint32_t, float>> dists;
    dists.reserve(n);
    for (;;) {
      const uint64_t i = next.fetch_add(1);
      if (i >= nq) break;
      dists.clear();
      const float *q = queries + i * dim;
      for (uint64_t j = 0; j < n; ++j) {
        const float *row = base + j * dim;
        dists.emplace_back(static_cast<uint32_t>(j), avx2 ? orc_l2_f32_avx2(q, row, dim) : orc_l2_f32(q, row, dim));
      }
      std::sort(dists.begin(), dists.end(), [](const auto &a, const auto &b) { return a.second < b.second; });
      for (uint32_t j = 0; j < k && j < dists.size(); ++j) ids[i * k + j] = dists[j].first;
    }
  };
  std::vector<std::thread> ts;
  for (uint32_t t = 0; t < std::max(1u, num_threads); ++t) ts.emplace_back(work);
  for (auto &t : ts) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

double orc_batch_rerank(const orc_index *ix, const float *queries, uint64_t nq, const uint32_t *search_ids,
                        uint32_t k, uint32_t ef, uint32_t *ids, float *dists) {
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 0; i < nq; ++i)
    orc_rerank(ix, queries + i * ix->dim, search_ids + i * k, k, ef, ids + i * k, dists + i * k);
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

float orc_sq8_l2(const uint8_t *x, const uint8_t *y, size_t dim, const float *min_v,
                 const float *max_v, int variant) {
  return sq8_dist<false>(x, y, dim, min_v, max_v, variant);
}
float orc_sq8_ip(const uint8_t *x, const uint8_t *y, size_t dim, const float *min_v,
                 const float *max_v, int variant) {
  return sq8_dist<true>(x, y, dim, min_v, max_v, variant);
}


// ---- online updates: GraphUpdateJob (include/executor/jobs/graph_update_job.hpp:49-137) ------
// JobContext (job_context.hpp:25-29) with the reference's container types, so iteration orders
// (and the LinearPool tie order in update()) follow the same libstdc++ sequences.
struct orc_updater {
  orc_index view;
  uint64_t capacity;
  std::vector<float> base;
  std::vector<uint32_t> l0;
  std::vector<uint8_t> valid;
  std::vector<uint32_t> levels;
  std::vector<uint64_t> upper_off;
  std::vector<uint32_t> upper_edges;
  std::unordered_map<uint32_t, std::vector<uint32_t>> inserted_edges;
  std::unordered_set<uint32_t> removed_vertices;
  std::unordered_map<uint32_t, std::vector<uint32_t>> removed_node_nbrs;

  void refresh() {
    view.base = base.data();
    view.stride = view.dim;
    view.l0 = l0.data();
    view.valid = valid.data();
    view.levels = levels.empty() ? nullptr : levels.data();
    view.upper_off = upper_off.empty() ? nullptr : upper_off.data();
    view.upper_edges = upper_edges.empty() ? nullptr : upper_edges.data();
  }
  float dist_by_id(uint32_t q, uint32_t u) const {  // QueryComputer(space, id) (raw_space.hpp:276-281)
    if (!((valid[u >> 3] >> (u & 7)) & 1)) return FLT_MAX;
    const float *x = base.data() + static_cast<size_t>(q) * view.dim;
    const float *y = base.data() + static_cast<size_t>(u) * view.dim;
    if (view.generic) return view.metric == ORC_L2 ? generic_l2(x, y, view.dim) : generic_ip(x, y, view.dim);
    return view.metric == ORC_L2 ? orc_l2_f32(x, y, view.dim) : orc_ip_f32(x, y, view.dim);
  }
  void update(uint32_t node) {  // :105-137
    std::unordered_set<uint32_t> candidate_nbrs;
    const uint32_t R = view.R;
    for (uint32_t i = 0; i < R; ++i) {
      uint32_t nbr = l0[static_cast<size_t>(node) * R + i];
      if (nbr == 0xffffffffu) break;
      if (removed_vertices.count(nbr)) {
        for (auto &second_hop_nbr : removed_node_nbrs.at(nbr)) candidate_nbrs.insert(second_hop_nbr);
      }
      candidate_nbrs.insert(nbr);
    }
    if (inserted_edges.count(node)) {
      for (auto inserted_nbr : inserted_edges.at(node)) candidate_nbrs.insert(inserted_nbr);
    }
    Pool pool(view.n, static_cast<int>(R));
    for (auto &nbr : candidate_nbrs) pool.insert(nbr, dist_by_id(node, nbr));
    std::vector<uint32_t> updated_edges(R);  // value-initialised: zeros past the pool
    for (uint32_t i = 0; i < R && i < pool.size; i++) updated_edges[i] = pool.id(i);
    std::memcpy(&l0[static_cast<size_t>(node) * R], updated_edges.data(), R * 4);
  }
};

orc_updater *orc_updater_new(const orc_index *ix, uint64_t capacity) {
  auto *u = new orc_updater();
  u->view = *ix;
  u->capacity = capacity;
  const uint64_t n = ix->n;
  u->base.resize(n * ix->dim);
  for (uint64_t i = 0; i < n; ++i)
    std::memcpy(&u->base[i * ix->dim], ix->base + i * ix->stride, ix->dim * sizeof(float));
  u->l0.assign(ix->l0, ix->l0 + n * ix->R);
  u->valid.assign((capacity + 7) / 8 + 1, 0);
  for (uint64_t i = 0; i < n; ++i) {
    const bool v = ix->valid ? ((ix->valid[i >> 3] >> (i & 7)) & 1) : true;
    if (v) u->valid[i >> 3] |= static_cast<uint8_t>(1u << (i & 7));
  }
  if (ix->levels) {
    u->levels.assign(ix->levels, ix->levels + n);
    u->upper_off.assign(ix->upper_off, ix->upper_off + n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i)
      if (ix->levels[i] > 0) total = std::max<uint64_t>(total, ix->upper_off[i] + uint64_t(ix->levels[i]) * ix->upper_R);
    u->upper_edges.assign(ix->upper_edges, ix->upper_edges + total);
  }
  u->refresh();
  return u;
}

void orc_updater_free(orc_updater *u) { delete u; }
const orc_index *orc_updater_view(orc_updater *u) { return &u->view; }

int64_t orc_updater_insert(orc_updater *u, const float *search_query, const float *row, uint32_t ef) {
  const uint32_t R = u->view.R;
  std::vector<uint32_t> search_results(R, 0xffffffffu);
  orc_search(&u->view, search_query, R, ef, search_results.data(), nullptr, nullptr);
  if (u->view.n >= u->capacity) return -1;  // Graph::insert fails: nothing else happens
  const uint32_t node_id = static_cast<uint32_t>(u->view.n);
  u->l0.insert(u->l0.end(), search_results.begin(), search_results.end());
  if (!u->levels.empty()) {
    u->levels.push_back(0);
    u->upper_off.push_back(u->upper_edges.size());
  }
  u->base.insert(u->base.end(), row, row + u->view.dim);  // RawSpace::insert
  u->valid[node_id >> 3] |= static_cast<uint8_t>(1u << (node_id & 7));
  u->view.n += 1;
  u->refresh();
  for (uint32_t i = 0; i < R; i++) {
    auto invert_node = search_results[i];
    if (invert_node != 0xffffffffu) u->inserted_edges[invert_node].push_back(node_id);
  }
  for (const auto &kv : u->inserted_edges) u->update(kv.first);
  u->inserted_edges.clear();
  return node_id;
}

void orc_updater_remove(orc_updater *u, uint32_t node_id) {  // :91-103
  const uint32_t R = u->view.R;
  auto &rec = u->removed_node_nbrs[node_id];
  for (uint32_t i = 0; i < R; i++) {
    auto nbr = u->l0[static_cast<size_t>(node_id) * R + i];
    if (nbr == 0xffffffffu) break;
    rec.push_back(nbr);
  }
  u->removed_vertices.insert(node_id);
  u->valid[node_id >> 3] &= static_cast<uint8_t>(~(1u << (node_id & 7)));
}

}  // extern "C"
