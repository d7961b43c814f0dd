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

template <int K, typename S = float>
struct Dual {
  S v;
  S d[K];
  __host__ __device__ Dual() : v(S(0)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = S(0);
  }
  __host__ __device__ Dual(double c) : v(S(c)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = S(0);
  }
  __host__ __device__ Dual(float c) : v(S(c)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = S(0);
  }
  __host__ __device__ Dual(int c) : v(S(c)) {
#pragma unroll
    for (int i = 0; i < K; ++i) d[i] = S(0);
  }
};

// unary map: value f(v), derivative scale f'(v)
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> dmap(const Dual<K, S>& a, S fv, S dfv) {
  Dual<K, S> r;
  r.v = fv;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = dfv * a.d[i];
  return r;
}

template <int K, typename S>
__device__ __forceinline__ Dual<K, S> operator+(const Dual<K, S>& a, const Dual<K, S>& b) {
  Dual<K, S> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> operator-(const Dual<K, S>& a, const Dual<K, S>& b) {
  Dual<K, S> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] - b.d[i];
  return r;
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> operator-(const Dual<K, S>& a) {
  Dual<K, S> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = -a.d[i];
  return r;
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> operator*(const Dual<K, S>& a, const Dual<K, S>& b) {
  Dual<K, S> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> operator/(const Dual<K, S>& a, const Dual<K, S>& b) {
  Dual<K, S> r;
  const S ib = S(1) / b.v;
  r.v = a.v * ib;
#pragma unroll
  for (int i = 0; i < K; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
  return r;
}
template <int K, typename S>
__device__ __forceinline__ bool operator<(const Dual<K, S>& a, const Dual<K, S>& b) { return a.v < b.v; }
template <int K, typename S>
__device__ __forceinline__ bool operator>(const Dual<K, S>& a, const Dual<K, S>& b) { return a.v > b.v; }
template <int K, typename S>
__device__ __forceinline__ bool operator<=(const Dual<K, S>& a, const Dual<K, S>& b) { return a.v <= b.v; }

template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vsin(const Dual<K, S>& a) { return dmap(a, S(vsin(a.v)), S(vcos(a.v))); }
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vcos(const Dual<K, S>& a) { return dmap(a, S(vcos(a.v)), S(-vsin(a.v))); }
template <int K, typename S>
__device__ __forceinline__ void vsincos(const Dual<K, S>& a, Dual<K, S>& s, Dual<K, S>& c) {
  S sv, cv;
  vsincos(a.v, sv, cv);
  s = dmap(a, sv, cv);
  c = dmap(a, cv, S(-sv));
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vtan(const Dual<K, S>& a) {
  const S t = vtan(a.v);
  return dmap(a, t, S(1) + t * t);
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vatan(const Dual<K, S>& a) { return dmap(a, S(vatan(a.v)), S(1) / (S(1) + a.v * a.v)); }
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vtanh(const Dual<K, S>& a) {
  const S t = vtanh(a.v);
  return dmap(a, t, S(1) - t * t);
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vsqrt(const Dual<K, S>& a) {
  const S r = vsqrt(a.v);
  return dmap(a, r, S(0.5) / r);
}
template <int K, typename S>
__device__ __forceinline__ Dual<K, S> vfabs(const Dual<K, S>& a) { return a.v < S(0) ? -a : a; }

}  // namespace vc
