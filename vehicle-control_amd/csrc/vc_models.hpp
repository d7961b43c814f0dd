// vc_models.hpp -- device-side vehicle models for the batched MPC path (gfx950).
//
// Each function restates one reference model function; citations are relative to
// the reference checkout (neverorfrog/vehicle-control @ 2024-12-20).
#pragma once
#include <hip/hip_runtime.h>

#include "vcmpc.h"

namespace vc {

// Transcendental entry points of the models.  double: libm precision (the fp64 paths
// are pinned to the reference traces at 1e-12).  float on the device: gfx950's native
// forms (v_sin_f32 / v_cos_f32 / v_exp_f32 based, ~1e-6 absolute error on the
// angles and forces here) -- the fp32 SQP path is compared with the fp64 oracle at a
// scaled 1e-4 and its rollouts were a quarter of its time with the libm versions.
__host__ __device__ inline double vsin(double x) { return sin(x); }
__host__ __device__ inline double vcos(double x) { return cos(x); }
__host__ __device__ inline double vtan(double x) { return tan(x); }
__host__ __device__ inline double vatan(double x) { return atan(x); }
__host__ __device__ inline double vtanh(double x) { return tanh(x); }
__host__ __device__ inline double vsqrt(double x) { return sqrt(x); }
__host__ __device__ inline double vfabs(double x) { return fabs(x); }
// sin and cos of one argument from one range reduction: bit-identical to sin(x), cos(x)
// (scripts/ubench/model.hip: 0 of 4.2 M inputs differ) at 409 instead of 691 cycles of latency
__host__ __device__ inline void vsincos(double x, double& s, double& c) { sincos(x, &s, &c); }
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline float vsin(float x) { return __sinf(x); }
__device__ inline float vcos(float x) { return __cosf(x); }
__device__ inline float vtan(float x) { return __sinf(x) / __cosf(x); }
__device__ inline float vtanh(float x) { return 1.0f - 2.0f / (1.0f + __expf(2.0f * x)); }
#else
inline float vsin(float x) { return sinf(x); }
inline float vcos(float x) { return cosf(x); }
inline float vtan(float x) { return tanf(x); }
inline float vtanh(float x) { return tanhf(x); }
#endif
__host__ __device__ inline float vatan(float x) { return atanf(x); }
__host__ __device__ inline float vsqrt(float x) { return sqrtf(x); }
__host__ __device__ inline float vfabs(float x) { return fabsf(x); }
__host__ __device__ inline void vsincos(float x, float& s, float& c) {
  s = vsin(x);
  c = vcos(x);
}

constexpr int KIN_NX = 6, KIN_NU = 2;
constexpr int DYN_NX = 8, DYN_NU = 2;
constexpr double GRAVITY = 9.88;  // models/dynamic_car.py:61

// ---------------------------------------------------------------------------
// Kinematic bicycle, x = [v, delta, s, ey, epsi, t], u = [a, w]
// ---------------------------------------------------------------------------

// Temporal ODE -- models/kinematic_car.py:34-41.
template <typename T>
__host__ __device__ inline void kin_temporal_ode(const T* x, const T* u, T kappa, T L, T* f) {
  const T v = x[0], delta = x[1], ey = x[3], epsi = x[4];
  const T s_dot = (v * cos(epsi)) / (T(1) - ey * kappa);
  f[0] = u[0];
  f[1] = u[1];
  f[2] = s_dot;
  f[3] = v * sin(epsi);
  f[4] = v * (tan(delta) / L) - s_dot * kappa;
  f[5] = T(1);
}

// Spatial ODE (d/ds) -- models/kinematic_car.py:47-60:
// rho = 1 - ey kappa, q = rho / (v cos epsi),
// f' = [q a, q w, 1, rho tan epsi, tan(delta)/L * rho / cos(epsi) - kappa, q].
template <typename T>
__host__ __device__ inline void kin_spatial_ode(const T* x, const T* u, T kappa, T L, T* f) {
  const T v = x[0], delta = x[1], ey = x[3], epsi = x[4];
  const T rho = T(1) - ey * kappa;
  const T c = cos(epsi);
  const T q = rho / (v * c);
  f[0] = q * u[0];
  f[1] = q * u[1];
  f[2] = T(1);
  f[3] = rho * tan(epsi);
  f[4] = (tan(delta) / L) * (rho / c) - kappa;
  f[5] = q;
}

// Euler step (utils/integrators.py:15-23): x+ = x + h f.
template <typename T, int NX>
__host__ __device__ inline void euler_apply(const T* x, const T* f, T h, T* xn) {
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h * f[i];
}

// Jacobian data of the kinematic spatial Euler step at (x, u, kappa): the nonzeros of
// J = d f'/d x (A = I + ds J, B = ds q [e_v e_a' + e_delta e_w']).  Derived by hand
// from kinematic_car.py:48-60 (CasADi AD does this inside IPOPT in the reference).
//   q, dq/dv, dq/dey, dq/depsi, d(ey')/dey, d(ey')/depsi,
//   d(epsi')/ddelta, d(epsi')/dey, d(epsi')/depsi
struct KinJac {
  double q, qv, qey, qep, J33, J34, J41, J43, J44;
};

__host__ __device__ inline KinJac kin_spatial_jac(const double* x, double kappa, double L) {
  const double v = x[0], delta = x[1], ey = x[3], epsi = x[4];
  const double rho = 1.0 - ey * kappa;
  const double c = cos(epsi);
  const double te = tan(epsi);
  const double td = tan(delta);
  KinJac j;
  j.q = rho / (v * c);
  j.qv = -j.q / v;
  j.qey = -kappa / (v * c);
  j.qep = j.q * te;
  j.J33 = -kappa * te;
  j.J34 = rho / (c * c);
  j.J41 = (1.0 + td * td) * rho / (L * c);
  j.J43 = -kappa * td / (L * c);
  j.J44 = td * rho * te / (L * c);
  return j;
}

// ---------------------------------------------------------------------------
// Dynamic bicycle, x = [Ux, Uy, r, delta, s, ey, epsi, t], u = [Fx, w]
// ---------------------------------------------------------------------------

// Dynamic-bicycle coefficients in the arithmetic type R, precomputed once on the host
// from vc_dyn_car (double) so the kernels never evaluate parameter expressions (or
// doubles) in their inner loops.  Every combination keeps the reference's evaluation
// order (dynamic_car.py:78-151), e.g. (b / l) * m is the left factor of
// (b / l) * m * (g cos(theta) cos(phi) + Av2 Ux^2) as Python evaluates it.
template <typename R>
struct DynCoef {
  R m, Izz, a, b, h, l, eps, Peng, Caf, Car, Cd, muf, mur, Av2, Frr;
  R xf_a, xf_b, xr_a, xr_b;  // (Xdf - Xbf)/2, (Xdf + Xbf)/2, (Xbr - Xdr)/2, (Xdr + Xbr)/2
  R gz0;                     // g cos(theta) cos(phi)
  R fzf_m, fzr_m;            // (b / l) m, (a / l) m
  // extra constants of the algebraic-slip form (dyn_*_alg, fp32 SQP kernel only)
  R h_l, inv_m, inv_Izz;     // h / l, 1 / m, 1 / Izz
  R tamf_k, tamr_k;          // 3 eps / Caf, 3 eps / Car   (tan alphamod = Fymax * tam_k)
  R fi1, fi2;                // 1 - 2 eps + eps^2, 3 eps^2 - 2 eps^3  (Fiala sliding branch)
  int tyre;
};

template <typename R>
__host__ __device__ inline DynCoef<R> make_dyn_coef(const vc_dyn_car& p) {
  DynCoef<R> c;
  c.m = R(p.m); c.Izz = R(p.Izz); c.a = R(p.a); c.b = R(p.b); c.h = R(p.h); c.l = R(p.l);
  c.eps = R(p.eps); c.Peng = R(p.Peng); c.Caf = R(p.Caf); c.Car = R(p.Car); c.Cd = R(p.Cd);
  c.muf = R(p.muf); c.mur = R(p.mur); c.Av2 = R(p.Av2); c.Frr = R(p.Frr);
  c.xf_a = R((p.Xdf - p.Xbf) / 2); c.xf_b = R((p.Xdf + p.Xbf) / 2);
  c.xr_a = R((p.Xbr - p.Xdr) / 2); c.xr_b = R((p.Xdr + p.Xbr) / 2);
  c.gz0 = R(GRAVITY * cos(p.theta) * cos(p.phi));
  c.fzf_m = R(p.b / p.l * p.m);
  c.fzr_m = R(p.a / p.l * p.m);
  c.h_l = R(p.h / p.l);
  c.inv_m = R(1.0 / p.m);
  c.inv_Izz = R(1.0 / p.Izz);
  c.tamf_k = R(3.0 * p.eps / p.Caf);
  c.tamr_k = R(3.0 * p.eps / p.Car);
  c.fi1 = R(1.0 - 2.0 * p.eps + p.eps * p.eps);
  c.fi2 = R(3.0 * p.eps * p.eps - 2.0 * p.eps * p.eps * p.eps);
  c.tyre = p.tyre;
  return c;
}

// Modified Fiala / brush tyre -- models/dynamic_car.py:119-142.
template <typename T>
__host__ __device__ inline T fiala_fy(T alpha, T Ca, T Fymax, T eps) {
  const T ta = vtan(alpha);
  const T alphamod = vatan((T(3) * Fymax * eps) / Ca);
  if (vfabs(alpha) <= alphamod) {
    return -Ca * ta + Ca * Ca * vfabs(ta) * ta / (T(3) * Fymax) -
           (Ca * Ca * Ca * ta * ta * ta) / (T(27) * Fymax * Fymax);
  }
  const T sgn = alpha > T(0) ? T(1) : (alpha < T(0) ? T(-1) : T(0));
  return -Ca * (T(1) - T(2) * eps + eps * eps) * ta - Fymax * (T(3) * eps * eps - T(2) * eps * eps * eps) * sgn;
}

// Tyre/load intermediates shared by the ODE and the NLP's stage terms (dynamic_car.py:78-115).
template <typename T, typename R>
struct DynForces {
  T Fx_f, Fx_r, Fz_f, Fz_r, alpha_f, alpha_r;
  __host__ __device__ DynForces(T Ux, T Uy, T r, T delta, T Fx, const DynCoef<R>& c) {
    // drive/brake split (dynamic_car.py:78-86)
    const T Xf = T(c.xf_a) * vtanh(T(2) * (Fx / T(1000) + T(0.5))) + T(c.xf_b);
    Fx_f = Fx * Xf;
    const T Xr = T(c.xr_a) * vtanh(T(-2) * (Fx / T(1000) + T(0.5))) + T(c.xr_b);
    Fx_r = Fx * Xr;
    // loads (dynamic_car.py:98-102); l = car.l
    const T gz = T(c.gz0) + T(c.Av2) * (Ux * Ux);
    Fz_f = T(c.fzf_m) * gz - T(c.h) * Fx / T(c.l);
    Fz_r = T(c.fzr_m) * gz + T(c.h) * Fx / T(c.l);
    // slip angles (dynamic_car.py:111-115)
    alpha_f = vatan((Uy + T(c.a) * r) / Ux) - delta;
    alpha_r = vatan((Uy - T(c.b) * r) / Ux);
  }
  // friction-ellipse lateral capacity (dynamic_car.py:107-108)
  __host__ __device__ T fymax_f(const DynCoef<R>& c) const {
    return vsqrt((T(c.muf) * Fz_f) * (T(c.muf) * Fz_f) - (T(0.99) * Fx_f) * (T(0.99) * Fx_f));
  }
  __host__ __device__ T fymax_r(const DynCoef<R>& c) const {
    return vsqrt((T(c.mur) * Fz_r) * (T(c.mur) * Fz_r) - (T(0.99) * Fx_r) * (T(0.99) * Fx_r));
  }
};

// Temporal ODE -- models/dynamic_car.py:66-163 (Fb = 0).  tyre: VC_TYRE_FIALA or the
// build-defined VC_TYRE_LINEAR (Fy = -C_alpha tan alpha, first term of :123).
template <typename T, typename R>
__host__ __device__ inline void dyn_temporal_ode(const T* x, const T* u, T kappa, const DynCoef<R>& c, T* f) {
  const T Ux = x[0], Uy = x[1], r = x[2], delta = x[3], ey = x[5], epsi = x[6];
  const T Fx = u[0], w = u[1];
  const DynForces<T, R> F(Ux, Uy, r, delta, Fx, c);
  T Fy_f, Fy_r;
  if (c.tyre == VC_TYRE_LINEAR) {
    Fy_f = -T(c.Caf) * vtan(F.alpha_f);
    Fy_r = -T(c.Car) * vtan(F.alpha_r);
  } else {
    Fy_f = fiala_fy(F.alpha_f, T(c.Caf), F.fymax_f(c), T(c.eps));
    Fy_r = fiala_fy(F.alpha_r, T(c.Car), F.fymax_r(c), T(c.eps));
  }
  const T Fd = T(c.Frr) + T(c.Cd) * (Ux * Ux);
  T sd, cd;
  vsincos(delta, sd, cd);
  const T m = T(c.m);
  f[0] = (F.Fx_f * cd - Fy_f * sd + F.Fx_r - Fd) / m + r * Uy;
  f[1] = (Fy_f * cd + F.Fx_f * sd + Fy_r) / m - r * Ux;
  f[2] = (T(c.a) * (Fy_f * cd + F.Fx_f * sd) - T(c.b) * Fy_r) / T(c.Izz);
  f[3] = w;
  T se, ce;
  vsincos(epsi, se, ce);
  const T s_dot = (Ux * ce - Uy * se) / (T(1) - kappa * ey);
  f[4] = s_dot;
  f[5] = Ux * se + Uy * ce;
  f[6] = r - kappa * s_dot;
  f[7] = T(1);
}

// Spatial ODE = temporal / s_dot with s' = 1, t' = 1/s_dot -- dynamic_car.py:169-187.
template <typename T, typename R>
__host__ __device__ inline void dyn_spatial_ode(const T* x, const T* u, T kappa, const DynCoef<R>& c, T* f) {
  dyn_temporal_ode(x, u, kappa, c, f);
  const T s_dot = f[4];
#pragma unroll
  for (int i = 0; i < DYN_NX; ++i) f[i] = f[i] / s_dot;
  f[4] = T(1);
  f[7] = T(1) / s_dot;
}

// Per-stage nonlinear terms of the single-track NLP at (Ux, Uy, r, delta, Fx):
//   out[0] slip_f = |tan alpha_f| - vtan(alphamod_f)   (slip cost, cascaded_mpc.py:155-159)
//   out[1] slip_r                                     (cascaded_mpc.py:161-165)
//   out[2] peng   = Fx - Peng / Ux  <= 0              (power limit, cascaded_mpc.py:110)
//   out[3] Fx_f - mu_f Fz_f vcos(alpha_f) <= 0,  out[4] -Fx_f - mu_f Fz_f vcos(alpha_f) <= 0
//   out[5] Fx_r - mu_r Fz_r vcos(alpha_r) <= 0,  out[6] -Fx_r - mu_r Fz_r vcos(alpha_r) <= 0
//                                                     (tyre force bounds, cascaded_mpc.py:124-128)
// with Fz, Fymax, alpha, alphamod as in dynamic_car.py:78-132.
template <typename T, typename R>
__host__ __device__ inline void dyn_stage_terms(const T* X5, const DynCoef<R>& c, T* out) {
  const T Ux = X5[0], Fx = X5[4];
  const DynForces<T, R> F(Ux, X5[1], X5[2], X5[3], Fx, c);
  const T amod_f = vatan((T(3) * F.fymax_f(c) * T(c.eps)) / T(c.Caf));
  const T amod_r = vatan((T(3) * F.fymax_r(c) * T(c.eps)) / T(c.Car));
  out[0] = vfabs(vtan(F.alpha_f)) - vtan(amod_f);
  out[1] = vfabs(vtan(F.alpha_r)) - vtan(amod_r);
  out[2] = Fx - T(c.Peng) / Ux;
  const T bound_f = T(c.muf) * F.Fz_f * vcos(F.alpha_f);
  const T bound_r = T(c.mur) * F.Fz_r * vcos(F.alpha_r);
  out[3] = F.Fx_f - bound_f;
  out[4] = -F.Fx_f - bound_f;
  out[5] = F.Fx_r - bound_r;
  out[6] = -F.Fx_r - bound_r;
}

// ---------------------------------------------------------------------------
// Algebraic-slip form of the same model, for the fp32 SQP kernel (dyn_sqp.hip).
//
// The slip angles enter the model only through tan(alpha), the comparison
// |alpha| <= alphamod, sign(alpha) and cos(alpha), and alphamod = atan(3 Fymax eps / Ca)
// only through tan(alphamod).  With z_f = (Uy + a r) / Ux, z_r = (Uy - b r) / Ux:
//   tan(alpha_f) = tan(atan z_f - delta) = (z_f - tan delta) / (1 + z_f tan delta)
//   tan(alpha_r) = z_r,            tan(alphamod) = 3 Fymax eps / Ca
//   |alpha| <= alphamod  <=>  |tan alpha| <= tan alphamod,  sgn alpha = sgn tan alpha
//   cos(alpha) = 1 / sqrt(1 + tan^2 alpha)          (|alpha| < pi/2)
// so an evaluation needs no atan/tan and one sin/cos pair less, and divisions by
// constants become products.  Same function as dyn_temporal_ode / dyn_stage_terms
// (identities exact for |alpha| < pi/2); the fp64 plant and the oracle keep the
// reference's literal form.
// ---------------------------------------------------------------------------
// the input-only transcendental of the algebraic model: the front / rear Fx split
// tanh(2 (Fx / 1000 + 1/2)) (tanh(-y) = -tanh(y) gives the rear share)
template <typename T>
__host__ __device__ inline T dyn_fx_split(T Fx) {
  return vtanh(T(2) * (Fx * T(1e-3) + T(0.5)));
}

template <typename T, typename R>
struct DynForcesAlg {
  T Fx_f, Fx_r, Fz_f, Fz_r, ta_f, ta_r, cd, sd, iU;
  __host__ __device__ DynForcesAlg(T Ux, T Uy, T r, T delta, T Fx, const DynCoef<R>& c)
      : DynForcesAlg(Ux, Uy, r, delta, Fx, dyn_fx_split(Fx), c) {}
  // th = dyn_fx_split(Fx), precomputed by callers that evaluate one input several times (RK4)
  __host__ __device__ DynForcesAlg(T Ux, T Uy, T r, T delta, T Fx, T th, const DynCoef<R>& c) {
    Fx_f = Fx * (T(c.xf_a) * th + T(c.xf_b));
    Fx_r = Fx * (T(c.xr_b) - T(c.xr_a) * th);
    const T gz = T(c.gz0) + T(c.Av2) * (Ux * Ux);
    Fz_f = T(c.fzf_m) * gz - T(c.h_l) * Fx;
    Fz_r = T(c.fzr_m) * gz + T(c.h_l) * Fx;
    iU = T(1) / Ux;
    const T zf = (Uy + T(c.a) * r) * iU;
    ta_r = (Uy - T(c.b) * r) * iU;
    vsincos(delta, sd, cd);
    // tan(atan zf - delta) = (zf cd - sd) / (cd + zf sd)
    ta_f = (zf * cd - sd) / (cd + zf * sd);
  }
  __host__ __device__ T fymax_f(const DynCoef<R>& c) const {
    return vsqrt((T(c.muf) * Fz_f) * (T(c.muf) * Fz_f) - (T(0.99) * Fx_f) * (T(0.99) * Fx_f));
  }
  __host__ __device__ T fymax_r(const DynCoef<R>& c) const {
    return vsqrt((T(c.mur) * Fz_r) * (T(c.mur) * Fz_r) - (T(0.99) * Fx_r) * (T(0.99) * Fx_r));
  }
};

// Modified Fiala in tan(alpha) (dynamic_car.py:119-142): Ca ta (-1 + |q|/3 - q^2/27),
// q = Ca ta / Fymax, inside |ta| <= tan alphamod; -Ca fi1 ta - Fymax fi2 sgn(ta) outside.
template <typename T, typename R>
__host__ __device__ inline T fiala_fy_alg(T ta, R Ca, T Fymax, R tam_k, R fi1, R fi2) {
  const T q = (T(Ca) * ta) / Fymax;
  const T inside = T(Ca) * ta * (T(-1) + vfabs(q) * T(R(1) / R(3)) - q * q * T(R(1) / R(27)));
  const T sg = ta > T(0) ? T(1) : (ta < T(0) ? T(-1) : T(0));
  const T outside = -T(Ca * fi1) * ta - Fymax * T(fi2) * sg;
  return vfabs(ta) <= Fymax * T(tam_k) ? inside : outside;
}

template <typename T, typename R>
__host__ __device__ inline void dyn_temporal_ode_alg(const T* x, const T* u, T th, T kappa, const DynCoef<R>& c,
                                                     T* f) {
  const T Ux = x[0], Uy = x[1], r = x[2], ey = x[5], epsi = x[6];
  const T Fx = u[0], w = u[1];
  const DynForcesAlg<T, R> F(Ux, Uy, r, x[3], Fx, th, c);
  T Fy_f, Fy_r;
  if (c.tyre == VC_TYRE_LINEAR) {
    Fy_f = -T(c.Caf) * F.ta_f;
    Fy_r = -T(c.Car) * F.ta_r;
  } else {
    Fy_f = fiala_fy_alg(F.ta_f, c.Caf, F.fymax_f(c), c.tamf_k, c.fi1, c.fi2);
    Fy_r = fiala_fy_alg(F.ta_r, c.Car, F.fymax_r(c), c.tamr_k, c.fi1, c.fi2);
  }
  const T Fd = T(c.Frr) + T(c.Cd) * (Ux * Ux);
  const T lat_f = Fy_f * F.cd + F.Fx_f * F.sd;
  f[0] = (F.Fx_f * F.cd - Fy_f * F.sd + F.Fx_r - Fd) * T(c.inv_m) + r * Uy;
  f[1] = (lat_f + Fy_r) * T(c.inv_m) - r * Ux;
  f[2] = (T(c.a) * lat_f - T(c.b) * Fy_r) * T(c.inv_Izz);
  f[3] = w;
  T se, ce;
  vsincos(epsi, se, ce);
  const T s_dot = (Ux * ce - Uy * se) / (T(1) - kappa * ey);
  f[4] = s_dot;
  f[5] = Ux * se + Uy * ce;
  f[6] = r - kappa * s_dot;
  f[7] = T(1);
}

template <typename T, typename R>
__host__ __device__ inline void dyn_temporal_ode_alg(const T* x, const T* u, T kappa, const DynCoef<R>& c, T* f) {
  dyn_temporal_ode_alg(x, u, dyn_fx_split(u[0]), kappa, c, f);
}

// spatial form; th = dyn_fx_split(u[0]) (the RK4 steps compute it once for their 4 evaluations:
// the same value, so the same result as the plain form)
template <typename T, typename R>
__host__ __device__ inline void dyn_spatial_ode_alg_th(const T* x, const T* u, T th, T kappa, const DynCoef<R>& c,
                                                       T* f) {
  dyn_temporal_ode_alg(x, u, th, kappa, c, f);
  const T inv = T(1) / f[4];
#pragma unroll
  for (int i = 0; i < DYN_NX; ++i) f[i] = f[i] * inv;
  f[4] = T(1);
  f[7] = inv;
}

template <typename T, typename R>
__host__ __device__ inline void dyn_spatial_ode_alg(const T* x, const T* u, T kappa, const DynCoef<R>& c, T* f) {
  dyn_temporal_ode_alg(x, u, kappa, c, f);
  const T inv = T(1) / f[4];
#pragma unroll
  for (int i = 0; i < DYN_NX; ++i) f[i] = f[i] * inv;
  f[4] = T(1);
  f[7] = inv;
}

template <typename T, typename R>
__host__ __device__ inline void dyn_stage_terms_alg(const T* X5, const DynCoef<R>& c, T* out) {
  const T Ux = X5[0], Fx = X5[4];
  const DynForcesAlg<T, R> F(Ux, X5[1], X5[2], X5[3], Fx, c);
  out[0] = vfabs(F.ta_f) - F.fymax_f(c) * T(c.tamf_k);
  out[1] = vfabs(F.ta_r) - F.fymax_r(c) * T(c.tamr_k);
  out[2] = Fx - T(c.Peng) * F.iU;
  const T bound_f = T(c.muf) * F.Fz_f / vsqrt(T(1) + F.ta_f * F.ta_f);
  const T bound_r = T(c.mur) * F.Fz_r / vsqrt(T(1) + F.ta_r * F.ta_r);
  out[3] = F.Fx_f - bound_f;
  out[4] = -F.Fx_f - bound_f;
  out[5] = F.Fx_r - bound_r;
  out[6] = -F.Fx_r - bound_r;
}

// Dynamic point mass, the cascaded controller's tail (models/dynamic_point_mass.py:76-100):
// x = [V, s, ey, epsi, t], u = [Fx, Fy]; spatial ODE = temporal / s_dot, s' = 1, t' = 1/s_dot.
// Same car coefficients as the bicycle (simulation/racing.py:44-46 builds both from carconfig).
template <typename T, typename R>
__host__ __device__ inline void pm_spatial_ode(const T* x, const T* u, T kappa, const DynCoef<R>& c, T* f) {
  const T V = x[0], ey = x[2], epsi = x[3];
  const T Fd = T(c.Frr) + T(c.Cd) * (V * V);
  T se, ce;
  vsincos(epsi, se, ce);
  const T s_dot = (V * ce) / (T(1) - kappa * ey);
  const T V_dot = (u[0] - Fd) / T(c.m);
  const T ey_dot = V * se;
  const T epsi_dot = u[1] / (T(c.m) * V) - kappa * s_dot;
  f[0] = V_dot / s_dot;
  f[1] = T(1);
  f[2] = ey_dot / s_dot;
  f[3] = epsi_dot / s_dot;
  f[4] = T(1) / s_dot;
}

// Switching map of the cascaded controller (cascaded_mpc.py:256-277): point-mass state
// from the last single-track state.
template <typename T>
__host__ __device__ inline void st_to_pm(const T* x, T* p) {
  p[0] = vsqrt(x[0] * x[0] + x[1] * x[1]);
  p[1] = x[4];
  p[2] = x[5];
  p[3] = vatan(x[1] / x[0]) + x[6];
  p[4] = x[7];
}

// Lateral tyre forces Fy_f + Fy_r at (Ux, Uy, r, delta, Fx) (dynamic_car.py:117-142), the
// switching cost's lateral residual (cascaded_mpc.py:241-255).
template <typename T, typename R>
__host__ __device__ inline T dyn_lateral_sum(const T* X5, const DynCoef<R>& c) {
  const DynForces<T, R> F(X5[0], X5[1], X5[2], X5[3], X5[4], c);
  if (c.tyre == VC_TYRE_LINEAR) return -T(c.Caf) * vtan(F.alpha_f) + -T(c.Car) * vtan(F.alpha_r);
  return fiala_fy(F.alpha_f, T(c.Caf), F.fymax_f(c), T(c.eps)) + fiala_fy(F.alpha_r, T(c.Car), F.fymax_r(c), T(c.eps));
}

// RK4 (utils/integrators.py:26-37): x + h (1/6) (k1 + 2k2 + 2k3 + k4).
// The stage sum is accumulated left to right, ((k1 + 2k2) + 2k3) + k4, the evaluation
// order of the reference expression, so only four stage vectors are live at once.
template <typename T, int NX, typename F>
__host__ __device__ inline void rk4_apply(const T* x, T h, F&& f, T* xn) {
  T k[NX], acc[NX], xs[NX];
  f(x, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    acc[i] = k[i];
    xs[i] = x[i] + T(0.5) * h * k[i];
  }
  f(xs, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    acc[i] = acc[i] + T(2) * k[i];
    xs[i] = x[i] + T(0.5) * h * k[i];
  }
  f(xs, k);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    acc[i] = acc[i] + T(2) * k[i];
    xs[i] = x[i] + h * k[i];
  }
  f(xs, k);
  const T sixth = T(1.0 / 6.0);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h * sixth * (acc[i] + k[i]);
}

}  // namespace vc
