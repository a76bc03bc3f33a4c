// Host-side distance functions used by the graph builder and the SQ8 rerank.
//
// They compute exactly what the device kernels compute (same float reduction order), which is the
// order of the reference's AVX2 kernels: include/simd/distance_l2.ipp:54-116 (l2_sqr_avx2, picked
// by get_l2_sqr_func :678-692 on AVX2 and AVX-512 hosts alike) and distance_ip.ipp:56-111.
// 32 partial sums: element 32t+j feeds acc[j] by fma; a trailing 8-block feeds acc[0..7];
// combine v[l] = (acc[l]+acc[8+l]) + (acc[16+l]+acc[24+l]), s[j] = v[j]+v[j+4],
// r = (s0+s1)+(s2+s3); scalar tail r = fma(.,.,r).
#pragma once
#include <immintrin.h>

#include <cmath>
#include <cstddef>
#include <cstdint>

namespace alaya_amd {

enum Metric : int { kL2 = 0, kIP = 1, kCOS = 2 };

template <bool kInner>
__attribute__((target("avx2,fma"))) inline float dist_avx2(const float *x, const float *y,
                                                           size_t dim) {
  __m256 a0 = _mm256_setzero_ps(), a1 = _mm256_setzero_ps();
  __m256 a2 = _mm256_setzero_ps(), a3 = _mm256_setzero_ps();
  size_t i = 0;
  for (; i + 32 <= dim; i += 32) {
    __m256 x0 = _mm256_loadu_ps(x + i), y0 = _mm256_loadu_ps(y + i);
    __m256 x1 = _mm256_loadu_ps(x + i + 8), y1 = _mm256_loadu_ps(y + i + 8);
    __m256 x2 = _mm256_loadu_ps(x + i + 16), y2 = _mm256_loadu_ps(y + i + 16);
    __m256 x3 = _mm256_loadu_ps(x + i + 24), y3 = _mm256_loadu_ps(y + i + 24);
    if (kInner) {
      a0 = _mm256_fmadd_ps(x0, y0, a0);
      a1 = _mm256_fmadd_ps(x1, y1, a1);
      a2 = _mm256_fmadd_ps(x2, y2, a2);
      a3 = _mm256_fmadd_ps(x3, y3, a3);
    } else {
      x0 = _mm256_sub_ps(x0, y0);
      x1 = _mm256_sub_ps(x1, y1);
      x2 = _mm256_sub_ps(x2, y2);
      x3 = _mm256_sub_ps(x3, y3);
      a0 = _mm256_fmadd_ps(x0, x0, a0);
      a1 = _mm256_fmadd_ps(x1, x1, a1);
      a2 = _mm256_fmadd_ps(x2, x2, a2);
      a3 = _mm256_fmadd_ps(x3, x3, a3);
    }
  }
  for (; i + 8 <= dim; i += 8) {
    __m256 xv = _mm256_loadu_ps(x + i), yv = _mm256_loadu_ps(y + i);
    if (kInner) {
      a0 = _mm256_fmadd_ps(xv, yv, a0);
    } else {
      xv = _mm256_sub_ps(xv, yv);
      a0 = _mm256_fmadd_ps(xv, xv, a0);
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
    if (kInner) {
      r = std::fma(x[i], y[i], r);
    } else {
      float d = x[i] - y[i];
      r = std::fma(d, d, r);
    }
  }
  return kInner ? -r : r;
}

// Portable restatement of the same order (hosts without AVX2+FMA).
template <bool kInner>
inline float dist_portable(const float *x, const float *y, size_t dim) {
  float acc[32] = {};
  size_t i = 0;
  for (; i + 32 <= dim; i += 32)
    for (int j = 0; j < 32; ++j) {
      float d = kInner ? x[i + j] : x[i + j] - y[i + j];
      acc[j] = std::fma(d, kInner ? y[i + j] : d, acc[j]);
    }
  for (; i + 8 <= dim; i += 8)
    for (int l = 0; l < 8; ++l) {
      float d = kInner ? x[i + l] : x[i + l] - y[i + l];
      acc[l] = std::fma(d, kInner ? y[i + l] : d, acc[l]);
    }
  float v[8];
  for (int l = 0; l < 8; ++l) v[l] = (acc[l] + acc[8 + l]) + (acc[16 + l] + acc[24 + l]);
  float r = ((v[0] + v[4]) + (v[1] + v[5])) + ((v[2] + v[6]) + (v[3] + v[7]));
  for (; i < dim; ++i) {
    float d = kInner ? x[i] : x[i] - y[i];
    r = std::fma(d, kInner ? y[i] : d, r);
  }
  return kInner ? -r : r;
}

inline bool host_has_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}

// Generic branch of l2_sqr<T> / ip_sqr<T> for non-float DataType (distance_l2.ipp:735-741,
// distance_ip.ipp:744-750), the same order as the device's generic_distances: one float
// accumulator, elements in order, no contraction (the library is built -ffp-contract=off).
template <bool kInner>
inline float dist_generic(const float *x, const float *y, size_t dim) {
  float sum = 0.0f;
  for (size_t i = 0; i < dim; ++i) {
    if (kInner) {
      sum += x[i] * y[i];
    } else {
      const float d = x[i] - y[i];
      sum += d * d;
    }
  }
  return kInner ? -sum : sum;
}

// flag OR-ed into a metric code: the rows are a non-float DataType (ALAYA_DIST_GENERIC,
// include/alaya_hip.h)
constexpr int kDistGeneric = 0x100;

inline float host_dist(int metric, const float *x, const float *y, size_t dim) {
  if (metric & kDistGeneric) return (metric & 0xff) == kL2 ? dist_generic<false>(x, y, dim) : dist_generic<true>(x, y, dim);
  if (host_has_avx2()) return metric == kL2 ? dist_avx2<false>(x, y, dim) : dist_avx2<true>(x, y, dim);
  return metric == kL2 ? dist_portable<false>(x, y, dim) : dist_portable<true>(x, y, dim);
}

// data_utils.hpp:36-46 (COS): float sum of squares, 1/sqrt in double, scale in float.
inline void normalize_row(float *v, size_t dim) {
  float sum = 0.0f;
  for (size_t i = 0; i < dim; ++i) sum += v[i] * v[i];
  sum = static_cast<float>(1.0 / std::sqrt(static_cast<double>(sum)));
  for (size_t i = 0; i < dim; ++i) v[i] *= sum;
}

}  // namespace alaya_amd
