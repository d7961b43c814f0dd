// vc_models.hpp -- device-side vehicle models for the batched MPC path (gfx950).
//
// Each function restates one reference model function; citations are relative to
// the reference checkout (neverorfrog/vehicle-control @ 2024-12-20).
#pragma once
#include <hip/hip_runtime.h>

#include "vcmpc.h"

namespace vc {

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

// Modified Fiala / brush tyre -- models/dynamic_car.py:119-142.
template <typename T>
__host__ __device__ inline T fiala_fy(T alpha, T Ca, T Fymax, T eps) {
  const T ta = tan(alpha);
  const T alphamod = atan((T(3) * Fymax * eps) / Ca);
  if (fabs(alpha) <= alphamod) {
    return -Ca * ta + Ca * Ca * fabs(ta) * ta / (T(3) * Fymax) -
           (Ca * Ca * Ca * ta * ta * ta) / (T(27) * Fymax * Fymax);
  }
  const T sgn = alpha > T(0) ? T(1) : (alpha < T(0) ? T(-1) : T(0));
  return -Ca * (T(1) - T(2) * eps + eps * eps) * ta - Fymax * (T(3) * eps * eps - T(2) * eps * eps * eps) * sgn;
}

// Temporal ODE -- models/dynamic_car.py:66-163 (Fb = 0).  tyre: VC_TYRE_FIALA or the
// build-defined VC_TYRE_LINEAR (Fy = -C_alpha tan alpha, first term of :123).
template <typename T>
__host__ __device__ inline void dyn_temporal_ode(const T* x, const T* u, T kappa, const vc_dyn_car& p, T* f) {
  const T Ux = x[0], Uy = x[1], r = x[2], delta = x[3], ey = x[5], epsi = x[6];
  const T Fx = u[0], w = u[1];
  // drive/brake split (dynamic_car.py:78-86)
  const T Xf = T((p.Xdf - p.Xbf) / 2) * tanh(T(2) * (Fx / T(1000) + T(0.5))) + T((p.Xdf + p.Xbf) / 2);
  const T Fx_f = Fx * Xf;
  const T Xr = T((p.Xbr - p.Xdr) / 2) * tanh(T(-2) * (Fx / T(1000) + T(0.5))) + T((p.Xdr + p.Xbr) / 2);
  const T Fx_r = Fx * Xr;
  // loads (dynamic_car.py:98-102); l = car.l
  const T gz = T(GRAVITY) * T(cos(p.theta)) * T(cos(p.phi)) + T(p.Av2) * Ux * Ux;
  const T Fz_f = T(p.b / p.l) * T(p.m) * gz - T(p.h) * Fx / T(p.l);
  const T Fz_r = T(p.a / p.l) * T(p.m) * gz + T(p.h) * Fx / T(p.l);
  // slip angles (dynamic_car.py:111-115)
  const T alpha_f = atan((Uy + T(p.a) * r) / Ux) - delta;
  const T alpha_r = atan((Uy - T(p.b) * r) / Ux);
  T Fy_f, Fy_r;
  if (p.tyre == VC_TYRE_LINEAR) {
    Fy_f = -T(p.Caf) * tan(alpha_f);
    Fy_r = -T(p.Car) * tan(alpha_r);
  } else {
    // friction-ellipse lateral capacity (dynamic_car.py:107-108)
    const T Fymax_f = sqrt((T(p.muf) * Fz_f) * (T(p.muf) * Fz_f) - (T(0.99) * Fx_f) * (T(0.99) * Fx_f));
    const T Fymax_r = sqrt((T(p.mur) * Fz_r) * (T(p.mur) * Fz_r) - (T(0.99) * Fx_r) * (T(0.99) * Fx_r));
    Fy_f = fiala_fy(alpha_f, T(p.Caf), Fymax_f, T(p.eps));
    Fy_r = fiala_fy(alpha_r, T(p.Car), Fymax_r, T(p.eps));
  }
  const T Fd = T(p.Frr) + T(p.Cd) * Ux * Ux;
  const T cd = cos(delta), sd = sin(delta);
  const T m = T(p.m);
  f[0] = (Fx_f * cd - Fy_f * sd + Fx_r - Fd) / m + r * Uy;
  f[1] = (Fy_f * cd + Fx_f * sd + Fy_r) / m - r * Ux;
  f[2] = (T(p.a) * (Fy_f * cd + Fx_f * sd) - T(p.b) * Fy_r) / T(p.Izz);
  f[3] = w;
  const T s_dot = (Ux * cos(epsi) - Uy * sin(epsi)) / (T(1) - kappa * ey);
  f[4] = s_dot;
  f[5] = Ux * sin(epsi) + Uy * cos(epsi);
  f[6] = r - kappa * s_dot;
  f[7] = T(1);
}

// Spatial ODE = temporal / s_dot with s' = 1, t' = 1/s_dot -- dynamic_car.py:169-187.
template <typename T>
__host__ __device__ inline void dyn_spatial_ode(const T* x, const T* u, T kappa, const vc_dyn_car& p, T* f) {
  dyn_temporal_ode(x, u, kappa, p, f);
  const T s_dot = f[4];
#pragma unroll
  for (int i = 0; i < DYN_NX; ++i) f[i] = f[i] / s_dot;
  f[4] = T(1);
  f[7] = T(1) / s_dot;
}

// RK4 (utils/integrators.py:26-37): x + h (1/6) (k1 + 2k2 + 2k3 + k4).
template <typename T, int NX, typename F>
__host__ __device__ inline void rk4_apply(const T* x, T h, F&& f, T* xn) {
  T k1[NX], k2[NX], k3[NX], k4[NX], xs[NX];
  f(x, k1);
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = x[i] + T(0.5) * h * k1[i];
  f(xs, k2);
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = x[i] + T(0.5) * h * k2[i];
  f(xs, k3);
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = x[i] + h * k3[i];
  f(xs, k4);
  const T sixth = T(1.0 / 6.0);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[i] = x[i] + h * sixth * (k1[i] + T(2) * k2[i] + T(2) * k3[i] + k4[i]);
}

}  // namespace vc
