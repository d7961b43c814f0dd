// Latency of the single-lane model evaluations on gfx950 (s_memtime cycles per dependent step):
// the SQP kernels' predict phase is lane 0 rolling the spatial model out stage by stage, so its
// time is the dependent latency of these calls.  (a) sin, (b) cos, (c) sin + cos of one argument,
// (d) tanh, (e) IEEE 1/x, (f) sqrt, (g) dyn_spatial_ode_alg linear tyre, (h) Fiala, (i) one RK4
// step (4 evaluations), linear.
// build: hipcc -O3 --offload-arch=gfx950 -I../../vehicle-control_amd/csrc -I../../include model.hip -o model
#include <hip/hip_runtime.h>

#include <cstdio>

#include "vc_kernels.hpp"
#include "vc_models.hpp"

#define STEPS 64
#define T0() __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#define T1(slot, n) __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); out[slot] = double(t1 - t0) / (n);

__global__ void k_model(double* out, vc::DynCoef<double> c, double seed) {
  if (threadIdx.x != 0) return;
  uint64_t t0, t1;
  double x = 0.1 + seed, y = 0.0;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 0.1 + 1e-3 * sin(x);
  T1(0, STEPS);
  y += x;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 0.1 + 1e-3 * cos(x);
  T1(1, STEPS);
  y += x;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 0.1 + 1e-3 * (sin(x) + cos(x));
  T1(2, STEPS);
  y += x;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 0.1 + 1e-3 * tanh(x);
  T1(3, STEPS);
  y += x;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 1.0 + 1e-3 / x;
  T1(4, STEPS);
  y += x;
  T0();
  for (int i = 0; i < STEPS; ++i) x = 1.0 + 1e-3 * sqrt(x);
  T1(5, STEPS);
  y += x;
  double xs[8] = {10.0 + seed, 0.1, 0.05, 0.02, 0.0, 0.3, 0.05, 0.0}, u[2] = {500.0, 0.01}, f[8];
  for (int tyre = 0; tyre < 2; ++tyre) {
    vc::DynCoef<double> cc = c;
    cc.tyre = tyre == 0 ? VC_TYRE_LINEAR : VC_TYRE_FIALA;
    T0();
    for (int i = 0; i < STEPS; ++i) {
      vc::dyn_spatial_ode_alg<double, double>(xs, u, 0.01, cc, f);
      xs[0] = 10.0 + 1e-6 * f[0];
      xs[1] = 0.1 + 1e-6 * f[1];
    }
    T1(6 + tyre, STEPS);
    y += xs[0];
  }
  {
    vc::DynCoef<double> cc = c;
    cc.tyre = VC_TYRE_LINEAR;
    double xn[8];
    T0();
    for (int i = 0; i < STEPS / 4; ++i) {
      vc::rk4_apply<double, 8>(xs, 0.5, [&](const double* xx, double* ff) { vc::dyn_spatial_ode_alg<double, double>(xx, u, 0.01, cc, ff); }, xn);
      for (int j = 0; j < 8; ++j) xs[j] = j == 4 ? 0.0 : xn[j];
    }
    T1(8, STEPS / 4);
    y += xs[0];
  }
  T0();
  for (int i = 0; i < STEPS; ++i) {
    double s, cs;
    sincos(x, &s, &cs);
    x = 0.1 + 1e-3 * (s + cs);
  }
  T1(9, STEPS);
  y += x;
  out[15] = y;
}

// sincos(x) vs sin(x), cos(x): count of inputs whose bits differ (n log-spaced + signed inputs)
__global__ void k_sincos_bits(unsigned long long* bad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = double(i) / n;
  const double x = (i & 1 ? -1.0 : 1.0) * exp2(-30.0 + 40.0 * t) * (1.0 + 0.37 * t);
  double s, c;
  sincos(x, &s, &c);
  const double s1 = sin(x), c1 = cos(x);
  if (__double_as_longlong(s) != __double_as_longlong(s1) || __double_as_longlong(c) != __double_as_longlong(c1))
    atomicAdd(bad, 1ull);
}

int main() {
  double* d;
  hipMalloc(&d, 16 * sizeof(double));
  vc::DynCoef<double> c{};
  // plausible coefficients (values only set the data path, not the instruction count)
  c.a = 1.2; c.b = 1.4; c.m = 1500; c.inv_m = 1.0 / 1500; c.inv_Izz = 1.0 / 2500; c.Caf = 8e4; c.Car = 9e4;
  c.muf = 1.0; c.mur = 1.0; c.gz0 = 9.81 * 1500; c.Av2 = 1.0; c.fzf_m = 0.5; c.fzr_m = 0.5; c.h_l = 0.2;
  c.xf_a = 0.25; c.xf_b = 0.25; c.xr_a = 0.25; c.xr_b = 0.75; c.Frr = 200; c.Cd = 0.4; c.tamf_k = 0.1; c.tamr_k = 0.1;
  c.fi1 = 0.1; c.fi2 = 0.9; c.eps = 0.1;
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k_model, dim3(1), dim3(64), 0, 0, d, c, 0.0);
  double h[16];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[10] = {"sin", "cos", "sin+cos", "tanh", "1/x", "sqrt", "ode linear", "ode fiala", "rk4 step linear",
                        "sincos"};
  for (int i = 0; i < 10; ++i) printf("%-18s %8.1f cycles\n", nm[i], h[i]);
  unsigned long long* bad;
  hipMalloc(&bad, 8);
  hipMemset(bad, 0, 8);
  const int n = 1 << 22;
  hipLaunchKernelGGL(k_sincos_bits, dim3(n / 256), dim3(256), 0, 0, bad, n);
  unsigned long long nb = 0;
  hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
  printf("sincos vs sin/cos: %llu of %d inputs differ in some bit\n", nb, n);
  hipFree(d);
  return 0;
}
