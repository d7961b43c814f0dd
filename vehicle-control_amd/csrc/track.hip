// track.hip -- curvature table k(s) and the closed-loop kernels behind vc_track_k /
// vc_horizon / vc_drive / vc_simulate.
//
// The reference evaluates k(s) with one CasADi bspline call per vehicle per step
// (track.py:162-166 via RacingCar.drive, racing_car.py:38, and _init_horizon,
// kinematic_mpc.py:187 / cascaded_mpc.py:330).  Here the bspline is a table of
// cubic pieces on the uniform 0.05 m grid (~6.3K pieces x 32 B = 200 KB for
// ippodromo): it stays resident in L2, every lookup is one 32-byte read.
//
// All three kernels are one thread per vehicle and trivially HBM/latency bound
// (a few hundred bytes per vehicle); they exist so that the closed loop never
// leaves the device.  Arithmetic is fp64 with FMA contraction off so that the
// results follow numpy's operation order exactly (parity is bit-level for the
// horizon sums and ~1 ulp for the table evaluation).
#include <hip/hip_runtime.h>

#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

namespace vc {

#pragma clang fp contract(off)

__device__ inline double track_k(const TrackTable& tt, double s) {
  const double sw = fmod(s, tt.length);
  double q = floor(sw / tt.h);
  q = q < 0.0 ? 0.0 : (q > double(tt.n - 1) ? double(tt.n - 1) : q);
  const int i = int(q);
  const double t = sw - double(i) * tt.h;
  const double4 c = reinterpret_cast<const double4*>(tt.coef)[i];
  return ((c.w * t + c.z) * t + c.y) * t + c.x;
}

template <typename T>
__global__ void track_k_kernel(TrackTable tt, int B, const T* s, T* k) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  k[b] = T(track_k(tt, double(s[b])));
}

// _init_horizon.  XT is the type of x0 (double inside vc_simulate, where the kernel
// also emits the context-dtype copy x0_out for the solve).
template <typename T, typename XT, int MODEL>
__global__ void horizon_kernel(TrackTable tt, int B, int N, int M, double ds_pm, const XT* x0, const T* xbar,
                               double mpc_dt, T* kappa, T* ds, T* x0_out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  constexpr int NX = MODEL == VC_MODEL_KINEMATIC ? KIN_NX : DYN_NX;
  constexpr int IS = MODEL == VC_MODEL_KINEMATIC ? 2 : 4;  // s  (kinematic_car.py:81, dynamic_car.py:209)
  constexpr int IV = 0;                                     // v / Ux
  const int H = N + (MODEL == VC_MODEL_CASCADED ? M : 0);   // stages of the kappa / ds arrays
  const int NS = MODEL == VC_MODEL_KINEMATIC ? N + 1 : H;
  const XT* xb0 = x0 + (size_t)b * NX;
  const double s0 = double(xb0[IS]);
  if (x0_out) {
#pragma unroll
    for (int i = 0; i < NX; ++i) x0_out[(size_t)b * NX + i] = T(xb0[i]);
  }
  const T* xp = xbar + (size_t)b * NS * NX;
  T* kap = kappa + (size_t)b * H;
  T* dsb = ds + (size_t)b * H;
  if (MODEL == VC_MODEL_KINEMATIC) {
    // ds_traj = mpc_dt * v + 0.5 (N+1 values); ds = ds_traj[:N]; ds_traj[0] = 0;
    // s = cumsum(ds_traj) + s0; kappa = k(s[:N])   (kinematic_mpc.py:178-187)
    double c = 0.0;
    for (int k = 0; k < N; ++k) {
      const double d = mpc_dt * double(xp[(size_t)k * NX + IV]) + 0.5;
      dsb[k] = T(d);
      if (k > 0) c = c + d;
      kap[k] = T(track_k(tt, c + s0));
    }
  } else {
    // ds = mpc_dt * Ux[:N]; s = cumsum(ds) - ds[0] + s0; kappa = k(s)  (cascaded_mpc.py:323-330)
    double c = 0.0, d0 = 0.0;
    for (int k = 0; k < N; ++k) {
      const double d = mpc_dt * double(xp[(size_t)k * NX + IV]);
      dsb[k] = T(d);
      if (k == 0) {
        d0 = d;
        c = d;
      } else {
        c = c + d;
      }
      kap[k] = T(track_k(tt, (c - d0) + s0));
    }
    if (MODEL == VC_MODEL_CASCADED) {
      // point mass: ds = ds_pm, s = cumsum(ds_pm) - ds[N-1] + s_traj[N-1]  (cascaded_mpc.py:332-338)
      const double d_last = mpc_dt * double(xp[(size_t)(N - 1) * NX + IV]);
      const double s_last = (c - d0) + s0;
      double cp = 0.0;
      for (int j = 0; j < M; ++j) {
        cp = cp + ds_pm;
        dsb[N + j] = T(ds_pm);
        kap[N + j] = T(track_k(tt, (cp - d_last) + s_last));
      }
    }
  }
}

// RacingCar.drive (racing_car.py:34-46) in fp64 with k(s) from the table, plus the
// closed-loop bookkeeping of vc_simulate (failure restart, logging).
template <typename T, int MODEL>
__global__ void drive_kernel(ModelArgs m, TrackTable tt, double* x64, const T* u0, double dt, T* x_ctx,
                             const int32_t* status, T* xbar, T* ubar, int32_t* nfail, double* log_x, T* log_u,
                             const T* kappa) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= m.B) return;
  constexpr int NX = MODEL == VC_MODEL_KINEMATIC ? KIN_NX : DYN_NX;
  constexpr int IS = MODEL == VC_MODEL_KINEMATIC ? 2 : 4;
  double x[NX], u[2], xn[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) x[i] = x64[(size_t)b * NX + i];
  u[0] = double(u0[(size_t)b * 2]);
  u[1] = double(u0[(size_t)b * 2 + 1]);
  // a non-solved step applies the neutral plan's input (zero: the restart below re-plans
  // from ubar = 0), not the unconverged iterate -- the failures are almost all infeasible
  // linearised QPs (scripts/kin_fail_modes.py), whose iterates diverge
  const bool failed = status && status[b] != VC_SOLVED;
  if (failed) u[0] = u[1] = 0.0;
  const double kap = track_k(tt, x[IS]);
  if (MODEL == VC_MODEL_KINEMATIC) {
    double f[KIN_NX];
    kin_temporal_ode(x, u, kap, m.L, f);  // kinematic_car.py:34-45, Euler (integrators.py:15-23)
    euler_apply<double, KIN_NX>(x, f, dt, xn);
  } else {                                // dynamic_car.py:144-167, RK4 (integrators.py:26-37)
    rk4_apply<double, DYN_NX>(x, dt, [&](const double* xs, double* f) { dyn_temporal_ode(xs, u, kap, m.dyn64, f); },
                              xn);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    x64[(size_t)b * NX + i] = xn[i];
    if (x_ctx) x_ctx[(size_t)b * NX + i] = T(xn[i]);
    if (log_x) log_x[(size_t)b * NX + i] = xn[i];
  }
  if (log_u) {
    log_u[(size_t)b * 2] = T(u[0]);
    log_u[(size_t)b * 2 + 1] = T(u[1]);
  }
  if (failed) {
    if (nfail) nfail[b] += 1;
    const int N = m.N, H = N + (MODEL == VC_MODEL_CASCADED ? m.M : 0), NS = MODEL == VC_MODEL_KINEMATIC ? N + 1 : H;
    for (int k = 0; k < H; ++k) ubar[((size_t)b * H + k) * 2] = ubar[((size_t)b * H + k) * 2 + 1] = T(0);
    if (MODEL == VC_MODEL_CASCADED && kappa) {
      // the neutral point-mass tail (controllers/cascaded_mpc.py BatchedCascadedMPC._neutral):
      // Fx = the drag at the current speed, Fy = m V^2 kappa (steady cornering)
      const DynCoef<double>& c = m.dyn64;
      const double V = fmax(sqrt(x[0] * x[0] + x[1] * x[1]), 3.0);
      for (int k = N; k < H; ++k) {
        ubar[((size_t)b * H + k) * 2] = T(c.Frr + c.Cd * (V * V));
        ubar[((size_t)b * H + k) * 2 + 1] = T(c.m * (V * V) * double(kappa[(size_t)b * H + k]));
      }
    }
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int i = 0; i < NX; ++i) xbar[((size_t)b * NS + k) * NX + i] = T(xn[i]);
  } else if (m.shift && MODEL != VC_MODEL_CASCADED) {
    // shifted warm start: the plan one stage on (single shooting re-rolls the warm-start inputs
    // from the new state; unshifted, they lag one step and over a 40 m kinematic horizon the
    // rollout crosses the spatial model's eps = +-pi/2 singularity, scripts/kin_shift_test.py)
    const int N = m.N, NS = MODEL == VC_MODEL_KINEMATIC ? N + 1 : N;
    for (int k = 0; k + 1 < N; ++k) {
      ubar[((size_t)b * N + k) * 2] = ubar[((size_t)b * N + k + 1) * 2];
      ubar[((size_t)b * N + k) * 2 + 1] = ubar[((size_t)b * N + k + 1) * 2 + 1];
    }
    for (int k = 0; k + 1 < NS; ++k)
#pragma unroll
      for (int i = 0; i < NX; ++i) xbar[((size_t)b * NS + k) * NX + i] = xbar[((size_t)b * NS + k + 1) * NX + i];
  }
}

static inline dim3 grid1(int n, int bs) { return dim3((n + bs - 1) / bs); }

template <typename T>
hipError_t launch_track_k_t(const TrackTable& tt, int B, const void* s, void* k, hipStream_t st) {
  hipLaunchKernelGGL(track_k_kernel<T>, grid1(B, 256), dim3(256), 0, st, tt, B, (const T*)s, (T*)k);
  return hipGetLastError();
}

hipError_t launch_track_k(const TrackTable& tt, int dtype, int B, const void* s, void* k, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  return dtype == VC_F32 ? launch_track_k_t<float>(tt, B, s, k, st) : launch_track_k_t<double>(tt, B, s, k, st);
}

template <typename T, typename XT>
hipError_t launch_horizon_t(const TrackTable& tt, int model, int B, int N, int M, double ds_pm, const void* x0,
                            const void* xbar, double mpc_dt, void* kappa, void* ds, void* x0_out, hipStream_t st) {
#define VC_HZ(MD)                                                                                                   \
  hipLaunchKernelGGL((horizon_kernel<T, XT, MD>), grid1(B, 128), dim3(128), 0, st, tt, B, N, M, ds_pm, (const XT*)x0, \
                     (const T*)xbar, mpc_dt, (T*)kappa, (T*)ds, (T*)x0_out)
  if (model == VC_MODEL_KINEMATIC) VC_HZ(VC_MODEL_KINEMATIC);
  else if (model == VC_MODEL_CASCADED) VC_HZ(VC_MODEL_CASCADED);
  else VC_HZ(VC_MODEL_DYNAMIC);
#undef VC_HZ
  return hipGetLastError();
}

hipError_t launch_horizon(const TrackTable& tt, int model, int dtype, int B, int N, int M, double ds_pm,
                          const void* x0, bool x0_fp64, const void* xbar, double mpc_dt, void* kappa, void* ds,
                          void* x0_out, hipStream_t st) {
  if (B <= 0) return hipSuccess;
  if (dtype == VC_F32)
    return x0_fp64 ? launch_horizon_t<float, double>(tt, model, B, N, M, ds_pm, x0, xbar, mpc_dt, kappa, ds, x0_out, st)
                   : launch_horizon_t<float, float>(tt, model, B, N, M, ds_pm, x0, xbar, mpc_dt, kappa, ds, x0_out, st);
  return launch_horizon_t<double, double>(tt, model, B, N, M, ds_pm, x0, xbar, mpc_dt, kappa, ds, x0_out, st);
}

template <typename T>
hipError_t launch_drive_t(const ModelArgs& m, const TrackTable& tt, double* x64, const void* u0, double dt,
                          void* x_ctx, const int32_t* status, void* xbar, void* ubar, int32_t* nfail, double* log_x,
                          void* log_u, const void* kappa, hipStream_t st) {
#define VC_DR(MD)                                                                                                   \
  hipLaunchKernelGGL((drive_kernel<T, MD>), grid1(m.B, 128), dim3(128), 0, st, m, tt, x64, (const T*)u0, dt,      \
                     (T*)x_ctx, status, (T*)xbar, (T*)ubar, nfail, log_x, (T*)log_u, (const T*)kappa)
  if (m.model == VC_MODEL_KINEMATIC) VC_DR(VC_MODEL_KINEMATIC);
  else if (m.model == VC_MODEL_CASCADED) VC_DR(VC_MODEL_CASCADED);
  else VC_DR(VC_MODEL_DYNAMIC);
#undef VC_DR
  return hipGetLastError();
}

hipError_t launch_drive(const ModelArgs& m, int dtype, const TrackTable& tt, double* x64, const void* u0, double dt,
                        void* x_ctx, const int32_t* status, void* xbar, void* ubar, int32_t* nfail, double* log_x,
                        void* log_u, const void* kappa, hipStream_t st) {
  if (m.B <= 0) return hipSuccess;
  return dtype == VC_F32
             ? launch_drive_t<float>(m, tt, x64, u0, dt, x_ctx, status, xbar, ubar, nfail, log_x, log_u, kappa, st)
             : launch_drive_t<double>(m, tt, x64, u0, dt, x_ctx, status, xbar, ubar, nfail, log_x, log_u, kappa, st);
}

}  // namespace vc
