// vc_dual.hpp -- forward-mode dual numbers (value + K tangents) for the device models.
//
// The reference differentiates its models symbolically with CasADi inside IPOPT
// ("expand": True, controllers/mpc/cascaded_mpc.py:65).  The build instead runs the
// same templated model code (vc_models.hpp) on Dual<K>: one evaluation returns the
// value and K directional derivatives, so every Jacobian the SQP needs comes from the
// restated model itself rather than from a second, hand-derived formula set.  The
// oracle uses complex-step differentiation of its numpy model (oracle/dyn_sqp.py), an
// independent method.
#pragma once
#include <hip/hip_runtime.h>

#include "vc_models.hpp"

namespace vc {

template <int K>
struct Dual {
  float v;
  float d[K];
  __host__ __device__ Dual() : v(0.f) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = 0.f;
  }
  __host__ __device__ Dual(double c) : v(float(c)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = 0.f;
  }
  __host__ __device__ Dual(float c) : v(c) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = 0.f;
  }
  __host__ __device__ Dual(int c) : v(float(c)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = 0.f;
  }
};

// unary map: value f(v), derivative scale f'(v)
template <int K>
__device__ __forceinline__ Dual<K> dmap(const Dual<K>& a, float fv, float dfv) {
  Dual<K> r;
  r.v = fv;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = dfv * a.d[i];
  return r;
}

template <int K>
__device__ __forceinline__ Dual<K> operator+(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator-(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] - b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator-(const Dual<K>& a) {
  Dual<K> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = -a.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator*(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
template <int K>
__device__ __forceinline__ Dual<K> operator/(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  const float ib = 1.0f / b.v;
  r.v = a.v * ib;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
  return r;
}
template <int K>
__device__ __forceinline__ bool operator<(const Dual<K>& a, const Dual<K>& b) { return a.v < b.v; }
template <int K>
__device__ __forceinline__ bool operator>(const Dual<K>& a, const Dual<K>& b) { return a.v > b.v; }
template <int K>
__device__ __forceinline__ bool operator<=(const Dual<K>& a, const Dual<K>& b) { return a.v <= b.v; }

template <int K>
__device__ __forceinline__ Dual<K> vsin(const Dual<K>& a) { return dmap(a, vsin(a.v), vcos(a.v)); }
template <int K>
__device__ __forceinline__ Dual<K> vcos(const Dual<K>& a) { return dmap(a, vcos(a.v), -vsin(a.v)); }
template <int K>
__device__ __forceinline__ Dual<K> vtan(const Dual<K>& a) {
  const float t = vtan(a.v);
  return dmap(a, t, 1.0f + t * t);
}
template <int K>
__device__ __forceinline__ Dual<K> vatan(const Dual<K>& a) { return dmap(a, vatan(a.v), 1.0f / (1.0f + a.v * a.v)); }
template <int K>
__device__ __forceinline__ Dual<K> vtanh(const Dual<K>& a) {
  const float t = vtanh(a.v);
  return dmap(a, t, 1.0f - t * t);
}
template <int K>
__device__ __forceinline__ Dual<K> vsqrt(const Dual<K>& a) {
  const float r = vsqrt(a.v);
  return dmap(a, r, 0.5f / r);
}
template <int K>
__device__ __forceinline__ Dual<K> vfabs(const Dual<K>& a) { return a.v < 0.f ? -a : a; }

}  // namespace vc
