// kin_merit.hip -- merit line search of the kinematic SQP step (fp64), one wavefront per problem.
//
// The kinematic LTV-QP contract takes one convexified QP step per control step; with the
// obstacle barrier of kinematic_mpc.py:130-133 the build globalises it (vc_qp.kin_sqp > 0):
// kin_sqp times { QP step dz at ubar (kin_ltv.hip / kin_ric.hip); this kernel: Armijo
// backtracking on the exact NLP cost + an L1 penalty on the state rows; ubar += alpha dz }.
// Contract and operation order: oracle/kin_sqp.py (merit, line_search).
//
// Lanes 0..LS-1 evaluate phi(u_prev + 2^-j dz), lane LS phi(u_prev + EPS dz) (the one-sided
// directional derivative), lane LS+1 phi(u_prev) -- 26 of the wave's 64 lanes, so the 24 step
// sizes cost one evaluation's latency; each lane rolls its candidate out with the
// spatial Euler model (kinematic_car.py:47-64) and sums the cost terms stage by stage -- a few
// thousand flops per lane, negligible next to the QP.  Lane 0 picks the first candidate with
// sufficient decrease (none, or a failed QP: alpha = 0; the full step when the decrease is at the
// merit's rounding level and phi does not rise, noise_step), then the wavefront writes the
// accepted inputs, lane 0 their rollout x* and u0, and the solve status / iteration count
// accumulate over the SQP iterations (status: the first QP's -- a later QP's failure only
// refuses its step; iterations: summed).  A first QP without a solution restarts the iterate
// from the neutral guess, and the next QP's status becomes the step's (kin_sqp > 1).
// With multiple shooting (vc_qp.ms) the iterate is the pair (x, u): the candidates are
// (x_prev, u_prev) + alpha (x* - x_prev, u* - u_prev), the terms are evaluated on the state
// candidate instead of a rollout (s = s0 + sum ds, s' = 1), plus RHO_DEF |F(x_n, u_n) - x_{n+1}|_1
// on the defects (oracle/kin_sqp.py merit(..., x=)), and the accepted state iterate is x_out --
// or the rollout of the accepted inputs when its (defect-free) merit is no larger.
#include <hip/hip_runtime.h>

#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

namespace vc {
namespace {

constexpr int LS = 24;           // alpha = 1 .. 2^-23  (oracle/kin_sqp.py LS_STEPS)
constexpr double ARMIJO = 1e-4;  // sufficient-decrease constant
constexpr double EPS_FD = 1e-7;  // directional-derivative step
constexpr double RHO = 1e3;      // L1 penalty on the state rows
constexpr double RHO_DEF = 1e3;  // L1 penalty on the multiple-shooting defects
// noise-level steps (oracle/kin_sqp.py noise_step): |D| at its own rounding level, full step
// taken when it raises phi by no more than NOISE_PHI (both x max(1, |phi0|))
constexpr double NOISE_D = 8.0 * 2.220446049250313e-16 / 1e-7;
constexpr double NOISE_PHI = 1e-13;
constexpr double V_DOM = 0.5;      // merit domain: v > V_DOM, |epsi| < EPSI_DOM, rho > 0 (oracle V_DOM)
constexpr double EPSI_DOM = 1.2;
constexpr double TIE = 1e-9;     // the rollout wins unless the state iterate's merit is lower by more
constexpr int32_t RESTART_PENDING = -1;  // st_acc: the iterate restarted, the next QP's status is the step's

__device__ __forceinline__ double bcast(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// b(m): 1/m above m0, the quadratic Taylor extension of 1/m at m0 below (oracle barrier_ext)
__device__ __forceinline__ double barrier_ext(double m, double m0) {
  if (m >= m0) return 1.0 / m;
  const double dm = m - m0;
  return 1.0 / m0 - dm / (m0 * m0) + dm * dm / (m0 * m0 * m0);
}

// p + al (q - p), or p itself for a refused step (al = 0): a failed QP's output may be
// non-finite, and 0 * NaN would carry it into the accepted iterate
__device__ __forceinline__ double step_to(double p, double q, double al) {
  return al == 0.0 ? p : p + al * (q - p);
}

// phi(u), u = up + alpha (uq - up), for one problem (oracle/kin_sqp.py merit)
__device__ double merit(const KinMeritArgs& A, int b, double alpha, bool msm) {
  const int N = A.N;
  const vc_kin_mpc& W = A.w;
  const double* x0 = A.x0 + (size_t)b * KIN_NX;
  const double* kap = A.kappa + (size_t)b * N;
  const double* dsv = A.ds + (size_t)b * N;
  const double* up = A.u_prev + (size_t)b * N * 2;
  const double* uq = A.ubar + (size_t)b * N * 2;
  const double* xq = A.x_out + (size_t)b * (N + 1) * KIN_NX;  // multiple shooting: QP's x*
  const double* xp = A.x_prev + (size_t)b * (N + 1) * KIN_NX;
  double x[KIN_NX];
#pragma unroll
  for (int i = 0; i < KIN_NX; ++i) x[i] = x0[i];
  double blo = 0.0, bhi = 0.0, dev = 0.0, obs = 0.0, ww = 0.0, wa = 0.0, pen = 0.0, a_prev = 0.0, pdef = 0.0;
  bool inside = true;  // the spatial model's domain on stages 0..N-1 (oracle/kin_sqp.py merit)
  const double m0 = A.obs.margin_min;
  for (int n = 0; n < N; ++n) {
    const double u[2] = {step_to(up[2 * n], uq[2 * n], alpha), step_to(up[2 * n + 1], uq[2 * n + 1], alpha)};
    const double ds = dsv[n];
    if (n >= 1) {  // stage terms on x_n (n = 0 is the fixed initial state)
      const double ey = x[3];
      if (ey < W.ey_min) blo += W.w_b * ds * (ey - W.ey_min) * (ey - W.ey_min);
      if (ey > W.ey_max) bhi += W.w_b * ds * (ey - W.ey_max) * (ey - W.ey_max);
      dev += W.w_dev * ds * ey * ey;
      for (int j = 0; j < A.obs.n; ++j) {
        const double a = x[2] - A.obs.s[j], e = ey - A.obs.ey[j];
        const double d = sqrt(a * a + e * e);
        obs += W.w_obs * ds * barrier_ext(d - (A.obs.radius[j] + 0.1), m0);
      }
      pen += fmax(W.v_min - x[0], 0.0) + fmax(x[1] - W.delta_max, 0.0) + fmax(W.delta_min - x[1], 0.0);
      wa += W.w_a * (u[0] - a_prev) * (u[0] - a_prev);
    }
    ww += W.w_w * u[1] * u[1];
    a_prev = u[0];
    inside = inside && x[0] > V_DOM && fabs(x[4]) < EPSI_DOM && 1.0 - x[3] * kap[n] > 0.0;
    double f[KIN_NX];
    kin_spatial_ode<double>(x, u, kap[n], A.L, f);
    if (msm) {
      const int o = (n + 1) * KIN_NX;
#pragma unroll
      for (int i = 0; i < KIN_NX; ++i) {
        const double xn = i == 2 ? x[2] + ds : step_to(xp[o + i], xq[o + i], alpha);
        pdef += fabs(x[i] + ds * f[i] - xn);
        x[i] = xn;
      }
    } else {
#pragma unroll
      for (int i = 0; i < KIN_NX; ++i) x[i] = x[i] + ds * f[i];
    }
  }
  double phi = blo + bhi + dev + obs + ww + wa + RHO_DEF * pdef;
  if (x[0] >= W.v_max) phi += W.w_v * (x[0] - W.v_max) * (x[0] - W.v_max);
  phi += W.w_time * x[5] + W.w_ey * x[3] * x[3] + W.w_epsi * x[4] * x[4];
  return inside ? phi + RHO * pen : __builtin_huge_val();
}

__global__ __launch_bounds__(64) void kin_merit_kernel(KinMeritArgs A) {
  const int b = xcd_problem(blockIdx.x, A.B);
  const int l = threadIdx.x;
  const int N = A.N;
  // candidate of this lane
  double alpha = 0.0;
  if (l < LS) alpha = ldexp(1.0, -l);
  else if (l == LS) alpha = EPS_FD;
  // multiple shooting: both merits per candidate; the single-shooting one governs where the
  // rollout of the current inputs has no larger merit than the state iterate ("roll" mode,
  // oracle/kin_sqp.py line_search_ms), the multiple-shooting one elsewhere
  double phs = 0.0, phm = 0.0;
  if (l <= LS + 1) {
    phs = merit(A, b, alpha, false);
    if (A.ms) phm = merit(A, b, alpha, true);
  }
  const double ps0 = bcast(phs, LS + 1), pm0 = bcast(phm, LS + 1);
  const bool roll = !A.ms || (isfinite(ps0) && ps0 <= pm0 + TIE * fabs(pm0));
  const double phi = roll ? phs : phm;
  const double phi0 = roll ? ps0 : pm0;
  const double D = (bcast(phi, LS) - phi0) / EPS_FD;
  const bool qp_ok = A.qp_status[b] == VC_SOLVED;
  // a first QP without a solution (infeasible, or linearised where the model is near-singular)
  // cannot be fixed by further SQP iterations from the same iterate: the iterate restarts from
  // the neutral guess (u = 0, the state iterate the current state at every stage, the plan
  // vc_simulate's failure restart would give) and the remaining iterations solve from there
  const bool restart = A.restart && A.first && !qp_ok;
  // lane 0..LS-1: sufficient decrease?  the first such lane (largest alpha) wins.  From an iterate
  // outside the model's domain (phi0 = inf): the largest step back inside it
  const bool restore = !isfinite(phi0);
  const bool good = l < LS && qp_ok && isfinite(phi) && (restore || (D < 0.0 && phi <= phi0 + ARMIJO * alpha * D));
  const uint64_t mask = __ballot(good);
  const double sc = fmax(1.0, fabs(phi0));
  const double p1 = bcast(phi, 0);
  // no Armijo step: near a KKT point the promised decrease is below the merit's resolution
  // (finite merits only: from outside the domain, phi0 = inf, the comparisons below hold for any p1,
  // an infinite one included, and the full step would leave the domain again)
  const bool noise = !mask && qp_ok && isfinite(phi0) && isfinite(p1) && fabs(D) <= NOISE_D * sc &&
                     p1 <= phi0 + NOISE_PHI * sc;
  const int pick = mask ? __builtin_ctzll(mask) : (noise ? 0 : -1);
  const double al = pick >= 0 ? ldexp(1.0, -pick) : 0.0;
  const double phia = pick >= 0 ? bcast(phi, pick) : phi0;
  const double* up = A.u_prev + (size_t)b * N * 2;
  double* ub = A.ubar + (size_t)b * N * 2;
  // multiple shooting: the accepted state iterate is reset to the rollout of the accepted inputs
  // when that has no larger merit (no defects; e.g. the reference's placeholder first guess)
  const int src = pick >= 0 ? pick : LS + 1;
  const double phr = bcast(phs, src), pma = bcast(phm, src);
  const bool reset = A.ms && isfinite(phr) && phr <= pma + TIE * fabs(pma);
  __syncthreads();  // every lane's merit reads of x* have completed
  if (A.ms && !reset) {  // multiple shooting: the state iterate moves with the inputs, x_prev + al (x* - x_prev)
    double* xo = A.x_out + (size_t)b * (N + 1) * KIN_NX;
    const double* xp = A.x_prev + (size_t)b * (N + 1) * KIN_NX;
    for (int e = l; e < (N + 1) * KIN_NX; e += 64)
      if (e < KIN_NX) xo[e] = A.x0[(size_t)b * KIN_NX + e];  // x_0 = x0
      else if (e % KIN_NX != 2) xo[e] = step_to(xp[e], xo[e], al);  // s stays s0 + sum ds
  }
  if (l == 0) {  // rollout of the accepted inputs (read before the wavefront overwrites u*)
    double x[KIN_NX];
    double* xo = (A.ms && !reset) ? nullptr : A.x_out + (size_t)b * (N + 1) * KIN_NX;
#pragma unroll
    for (int i = 0; i < KIN_NX; ++i) {
      x[i] = A.x0[(size_t)b * KIN_NX + i];
      if (xo) xo[i] = x[i];
    }
    for (int n = 0; n < N; ++n) {
      const double u[2] = {step_to(up[2 * n], ub[2 * n], al), step_to(up[2 * n + 1], ub[2 * n + 1], al)};
      if (n == 0) {
        A.u0[(size_t)b * 2] = u[0];
        A.u0[(size_t)b * 2 + 1] = u[1];
      }
      double f[KIN_NX];
      kin_spatial_ode<double>(x, u, A.kappa[(size_t)b * N + n], A.L, f);
#pragma unroll
      for (int i = 0; i < KIN_NX; ++i) {
        x[i] = x[i] + A.ds[(size_t)b * N + n] * f[i];
        if (xo) xo[(n + 1) * KIN_NX + i] = x[i];
      }
    }
    // the step's status is the first QP's: a later QP that fails only stops the progress (its
    // step is refused, alpha = 0), the accepted iterate never has a larger merit than the start.
    // A failed first QP restarts the iterate (below): then the next QP's status is the step's.
    const int32_t st = (A.first || A.st_acc[b] == RESTART_PENDING) ? A.qp_status[b] : A.st_acc[b];
    const int32_t it = (A.first ? 0 : A.it_acc[b]) + A.qp_iters[b];
    A.st_acc[b] = restart ? RESTART_PENDING : st;
    A.it_acc[b] = it;
    A.status[b] = st;
    A.iters[b] = it;
    if (A.ls_diag) {
      A.ls_diag[(size_t)b * 4 + 0] = al;
      A.ls_diag[(size_t)b * 4 + 1] = phi0;
      A.ls_diag[(size_t)b * 4 + 2] = phia;
      A.ls_diag[(size_t)b * 4 + 3] = D;
    }
  }
  __syncthreads();  // lane 0's reads of u* have completed
  for (int e = l; e < 2 * N; e += 64) ub[e] = restart ? 0.0 : step_to(up[e], ub[e], al);
  if (restart && A.ms) {
    double* xo = A.x_out + (size_t)b * (N + 1) * KIN_NX;
    for (int e = l; e < (N + 1) * KIN_NX; e += 64) xo[e] = A.x0[(size_t)b * KIN_NX + e % KIN_NX];
  }
}

// a QP that failed with non-finite output (the case kin_ric reports as VC_NONFINITE)
__global__ __launch_bounds__(64) void kin_qp_fault_kernel(KinLtvArgs a, int N, int b) {
  const double nan = __builtin_nan("");
  for (int e = threadIdx.x; e < 2 * N; e += 64) a.u_out[(size_t)b * 2 * N + e] = nan;
  for (int e = threadIdx.x; e < 6 * (N + 1); e += 64) a.x_out[(size_t)b * 6 * (N + 1) + e] = nan;
  if (threadIdx.x < 2) a.u0[(size_t)b * 2 + threadIdx.x] = nan;
  if (threadIdx.x == 0) a.status[b] = VC_NONFINITE;
}

}  // namespace

hipError_t launch_kin_qp_fault(const KinLtvArgs& a, int N, int b, hipStream_t stream) {
  hipLaunchKernelGGL(kin_qp_fault_kernel, dim3(1), dim3(64), 0, stream, a, N, b);
  return hipGetLastError();
}

hipError_t launch_kin_merit(const KinMeritArgs& a, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  hipLaunchKernelGGL(kin_merit_kernel, dim3(a.B), dim3(64), 0, stream, a);
  return hipGetLastError();
}

}  // namespace vc
