// models.hip -- batched model kernels behind vc_plant_step / vc_spatial_step /
// vc_rollout / vc_linearize.  One thread per problem (or per problem-stage).
// These are the reference's per-vehicle CasADi Function calls
// (RacingCar.drive -> transition, racing_car.py:34-46; spatial_transition,
// kinematic_car.py:70-72 / dynamic_car.py:197-199) evaluated for a whole batch.
#include <hip/hip_runtime.h>

#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

namespace vc {


template <typename T>
__device__ inline void temporal_step(const ModelArgs& m, const T* x, const T* u, T kappa, T dt, T* xn) {
  if (m.model == VC_MODEL_KINEMATIC) {
    T f[KIN_NX];
    kin_temporal_ode(x, u, kappa, T(m.L), f);   // Euler, kinematic_car.py:42-45
    euler_apply<T, KIN_NX>(x, f, dt, xn);
  } else {
    rk4_apply<T, DYN_NX>(x, dt, [&](const T* xs, T* f) { dyn_temporal_ode(xs, u, kappa, dyn_coef<T>(m), f); }, xn);
  }
}

template <typename T>
__device__ inline void spatial_step(const ModelArgs& m, const T* x, const T* u, T kappa, T ds, T* xn) {
  if (m.model == VC_MODEL_KINEMATIC) {
    T f[KIN_NX];
    kin_spatial_ode(x, u, kappa, T(m.L), f);    // Euler, kinematic_car.py:61-64
    euler_apply<T, KIN_NX>(x, f, ds, xn);
  } else {
    rk4_apply<T, DYN_NX>(x, ds, [&](const T* xs, T* f) { dyn_spatial_ode(xs, u, kappa, dyn_coef<T>(m), f); }, xn);
  }
}

// the continuous vector field f(x, u, kappa): temporal (kinematic_car.py:34-40, dynamic_car.py:153-167)
// or spatial (kinematic_car.py:47-60, dynamic_car.py:169-191) -- the `f` CasADi Function the
// reference's integrators wrap (utils/integrators.py:18,29)
template <typename T, int NX>
__global__ void ode_kernel(ModelArgs m, const T* x, const T* u, const T* kappa, int space, T* fo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  T xl[NX], ul[2], f[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xl[i] = x[(size_t)b * NX + i];
  ul[0] = u[(size_t)b * 2];
  ul[1] = u[(size_t)b * 2 + 1];
  if (m.model == VC_MODEL_KINEMATIC) {
    if (space) kin_spatial_ode(xl, ul, kappa[b], T(m.L), f);
    else kin_temporal_ode(xl, ul, kappa[b], T(m.L), f);
  } else {
    if (space) dyn_spatial_ode(xl, ul, kappa[b], dyn_coef<T>(m), f);
    else dyn_temporal_ode(xl, ul, kappa[b], dyn_coef<T>(m), f);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) fo[(size_t)b * NX + i] = f[i];
}

template <typename T, int NX>
__global__ void plant_step_kernel(ModelArgs m, const T* x, const T* u, const T* kappa, T dt, T* xn) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  T xl[NX], ul[2], out[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xl[i] = x[(size_t)b * NX + i];
  ul[0] = u[(size_t)b * 2];
  ul[1] = u[(size_t)b * 2 + 1];
  temporal_step<T>(m, xl, ul, kappa[b], dt, out);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[(size_t)b * NX + i] = out[i];
}

template <typename T, int NX>
__global__ void spatial_step_kernel(ModelArgs m, const T* x, const T* u, const T* kappa, const T* ds, T* xn) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  T xl[NX], ul[2], out[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xl[i] = x[(size_t)b * NX + i];
  ul[0] = u[(size_t)b * 2];
  ul[1] = u[(size_t)b * 2 + 1];
  spatial_step<T>(m, xl, ul, kappa[b], ds[b], out);
#pragma unroll
  for (int i = 0; i < NX; ++i) xn[(size_t)b * NX + i] = out[i];
}

template <typename T, int NX>
__global__ void rollout_kernel(ModelArgs m, const T* x0, const T* ubar, const T* kappa, const T* ds, T* xbar) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  const int N = m.N;
  T x[NX];
  T* out = xbar + (size_t)b * (N + 1) * NX;
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    x[i] = x0[(size_t)b * NX + i];
    out[i] = x[i];
  }
  for (int k = 0; k < N; ++k) {
    T ul[2] = {ubar[((size_t)b * N + k) * 2], ubar[((size_t)b * N + k) * 2 + 1]};
    T xn[NX];
    spatial_step<T>(m, x, ul, kappa[(size_t)b * N + k], ds[(size_t)b * N + k], xn);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      x[i] = xn[i];
      out[(k + 1) * NX + i] = xn[i];
    }
  }
}

// Kinematic A_k = I + ds J, B_k = ds q [e_v e_a' + e_delta e_w'] per (problem, stage).
__global__ void kin_linearize_kernel(ModelArgs m, const double* xbar, const double* ubar, const double* kappa,
                                     const double* ds, double* Aout, double* Bout) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m.B * m.N) return;
  const int b = idx / m.N, k = idx % m.N;
  const double* x = xbar + ((size_t)b * (m.N + 1) + k) * KIN_NX;
  const double h = ds[idx];
  const double a = ubar[(size_t)idx * 2], w = ubar[(size_t)idx * 2 + 1];
  const KinJac J = kin_spatial_jac(x, kappa[idx], m.L);
  double Jm[KIN_NX][KIN_NX] = {};
  const double rowmul[3] = {a, w, 1.0};
  const int rows[3] = {0, 1, 5};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    Jm[rows[t]][0] = J.qv * rowmul[t];
    Jm[rows[t]][3] = J.qey * rowmul[t];
    Jm[rows[t]][4] = J.qep * rowmul[t];
  }
  Jm[3][3] = J.J33; Jm[3][4] = J.J34;
  Jm[4][1] = J.J41; Jm[4][3] = J.J43; Jm[4][4] = J.J44;
  double* Ao = Aout + (size_t)idx * KIN_NX * KIN_NX;
#pragma unroll
  for (int i = 0; i < KIN_NX; ++i)
#pragma unroll
    for (int j = 0; j < KIN_NX; ++j) Ao[i * KIN_NX + j] = (i == j ? 1.0 : 0.0) + h * Jm[i][j];
  double* Bo = Bout + (size_t)idx * KIN_NX * KIN_NU;
#pragma unroll
  for (int i = 0; i < KIN_NX * KIN_NU; ++i) Bo[i] = 0.0;
  Bo[0 * KIN_NU + 0] = h * J.q;
  Bo[1 * KIN_NU + 1] = h * J.q;
}

static inline dim3 grid1(int n, int bs) { return dim3((n + bs - 1) / bs); }

template <typename T>
hipError_t launch_plant_step_t(const ModelArgs& m, const void* x, const void* u, const void* kappa, double dt,
                               void* xn, hipStream_t st) {
  if (m.model == VC_MODEL_KINEMATIC)
    hipLaunchKernelGGL((plant_step_kernel<T, KIN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x,
                       (const T*)u, (const T*)kappa, T(dt), (T*)xn);
  else
    hipLaunchKernelGGL((plant_step_kernel<T, DYN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x,
                       (const T*)u, (const T*)kappa, T(dt), (T*)xn);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_spatial_step_t(const ModelArgs& m, const void* x, const void* u, const void* kappa, const void* ds,
                                 void* xn, hipStream_t st) {
  if (m.model == VC_MODEL_KINEMATIC)
    hipLaunchKernelGGL((spatial_step_kernel<T, KIN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x,
                       (const T*)u, (const T*)kappa, (const T*)ds, (T*)xn);
  else
    hipLaunchKernelGGL((spatial_step_kernel<T, DYN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x,
                       (const T*)u, (const T*)kappa, (const T*)ds, (T*)xn);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_rollout_t(const ModelArgs& m, const void* x0, const void* ubar, const void* kappa, const void* ds,
                            void* xbar, hipStream_t st) {
  if (m.model == VC_MODEL_KINEMATIC)
    hipLaunchKernelGGL((rollout_kernel<T, KIN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x0,
                       (const T*)ubar, (const T*)kappa, (const T*)ds, (T*)xbar);
  else
    hipLaunchKernelGGL((rollout_kernel<T, DYN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x0,
                       (const T*)ubar, (const T*)kappa, (const T*)ds, (T*)xbar);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_ode_t(const ModelArgs& m, const void* x, const void* u, const void* kappa, int space, void* f,
                        hipStream_t st) {
  if (m.model == VC_MODEL_KINEMATIC)
    hipLaunchKernelGGL((ode_kernel<T, KIN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x, (const T*)u,
                       (const T*)kappa, space, (T*)f);
  else
    hipLaunchKernelGGL((ode_kernel<T, DYN_NX>), grid1(m.B, 128), dim3(128), 0, st, m, (const T*)x, (const T*)u,
                       (const T*)kappa, space, (T*)f);
  return hipGetLastError();
}

hipError_t launch_ode(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa, int space,
                      void* f, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  return dtype == VC_F32 ? launch_ode_t<float>(m, x, u, kappa, space, f, st)
                         : launch_ode_t<double>(m, x, u, kappa, space, f, st);
}
hipError_t launch_plant_step(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa, double dt,
                             void* xn, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  return dtype == VC_F32 ? launch_plant_step_t<float>(m, x, u, kappa, dt, xn, st)
                         : launch_plant_step_t<double>(m, x, u, kappa, dt, xn, st);
}
hipError_t launch_spatial_step(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa,
                               const void* ds, void* xn, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  return dtype == VC_F32 ? launch_spatial_step_t<float>(m, x, u, kappa, ds, xn, st)
                         : launch_spatial_step_t<double>(m, x, u, kappa, ds, xn, st);
}
hipError_t launch_rollout(const ModelArgs& m, int dtype, const void* x0, const void* ubar, const void* kappa,
                          const void* ds, void* xbar, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  return dtype == VC_F32 ? launch_rollout_t<float>(m, x0, ubar, kappa, ds, xbar, st)
                         : launch_rollout_t<double>(m, x0, ubar, kappa, ds, xbar, st);
}
hipError_t launch_kin_linearize(const ModelArgs& m, const void* xbar, const void* ubar, const void* kappa,
                                const void* ds, void* A, void* Bm, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  hipLaunchKernelGGL(kin_linearize_kernel, grid1(m.B * m.N, 128), dim3(128), 0, st, m, (const double*)xbar,
                     (const double*)ubar, (const double*)kappa, (const double*)ds, (double*)A, (double*)Bm);
  return hipGetLastError();
}

}  // namespace vc
