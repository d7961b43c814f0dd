// kin_ltv.hip -- fused batched kinematic LTV-MPC step for gfx950 (fp64).
//
// One 64-lane wavefront (= one workgroup) owns one problem and runs, without
// leaving the CU:  predict -> linearize -> condense -> Mehrotra primal-dual
// interior point -> active-set polish -> output.  This replaces, per control
// step and vehicle, KinematicMPC.command (controllers/mpc/kinematic_mpc.py:160-168),
// i.e. the IPOPT + HSL MA27 solve of the NLP built at kinematic_mpc.py:15-30.
// The QP solved is the build's LTV-QP contract (oracle/ltv_qp.py).
//
// Lane roles (n = 2N decision variables, NC = 2(N-1) state-constraint rows):
//   lane j < n   owns decision variable dz_j: column j of the condensed
//                sensitivity G, row j of the Hessian H (registers), row j of the
//                KKT matrix and of its Cholesky factor (registers), and the two
//                box inequalities of u_j.
//   lane r < NC  owns state-constraint row r: r < N-1 -> v_{r+1} >= v_min,
//                else delta_{r-N+2} in [delta_min, delta_max].
// LDS holds the constraint rows of G (read as broadcasts), the Cholesky factor
// for the transposed solve, and small broadcast vectors.  HBM traffic is only
// the compulsory per-problem inputs and outputs (roofline).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

namespace vc {


// ---- wave-level helpers ----------------------------------------------------
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
// value of `v` in lane `src` (src a compile-time constant in the unrolled loops)
__device__ inline double lane_bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}
__device__ inline void wave_sync() { __syncthreads(); }  // one-wave workgroup: cheap

// largest a in (0,1] keeping v + a dv >= 0
__device__ inline double step_bound(double v, double dv) { return dv < 0.0 ? -v / dv : 1.0; }

template <int N>
struct KinDims {
  static constexpr int n = 2 * N;        // decision variables
  static constexpr int NC = 2 * (N - 1); // state-constraint rows
  static constexpr int LD = n + 1;       // padded LDS row stride (conflict-free column reads)
  static_assert(n <= 64, "one wavefront per problem needs 2N <= 64");
};

template <int N>
struct __align__(16) KinShared {
  using D = KinDims<N>;
  double G[D::NC][D::LD];     // constraint rows of the condensed sensitivity
  double Lm[D::n][D::LD];     // Cholesky factor rows (for the transposed solve)
  double xb[N + 1][KIN_NX];   // predicted trajectory
  double jac[N][9];           // Jacobian data per stage (KinJac)
  double ub[D::n];            // warm-start inputs
  double kap[N], ds[N];
  double vz[64];              // broadcast: a length-n vector (z, dz, fixed values, ...)
  double vc[64];              // broadcast: a length-NC vector (weights, residual terms)
  double col[2][64];          // broadcast: one Cholesky column / one G row
  double dinv[64];            // 1 / L_kk
};

// ---- dense kernels on register-resident rows -------------------------------

// In-place Cholesky of the SPD matrix whose row `lane` is Mr[0..n).  On return
// Mr holds row `lane` of L (lower part), s.Lm the same rows, s.dinv = 1/diag.
// Returns false if a pivot is not positive (uniform).
template <int N>
__device__ bool chol_rows(double (&Mr)[KinDims<N>::n], KinShared<N>& s, int lane) {
  constexpr int n = KinDims<N>::n;
  bool ok = true;
  double mydiag = 1.0;
#pragma unroll
  for (int k = 0; k < n; ++k) {
    const double dkk = lane_bcast(Mr[k], k);
    ok = ok && (dkk > 0.0);
    const double d = sqrt(dkk);
    const double inv = 1.0 / d;
    const double lik = (lane == k) ? d : Mr[k] * inv;
    if (lane == k) mydiag = d;
    Mr[k] = lik;
    double* cb = s.col[k & 1];
    cb[lane] = lik;
    wave_sync();
#pragma unroll
    for (int j = k + 1; j < n; ++j) Mr[j] -= lik * cb[j];
  }
  if (lane < n) {
#pragma unroll
    for (int j = 0; j < n; ++j) s.Lm[lane][j] = Mr[j];
    s.dinv[lane] = 1.0 / mydiag;
  }
  wave_sync();
  return ok;
}

// Solve (L L') x = b, lane j holding b_j; returns x_j.  Runtime loops over the
// factor in LDS (s.Lm rows, s.dinv): the substitution chain is inherently serial,
// so unrolling it only inflates register pressure.
template <int N>
__device__ double chol_solve(const KinShared<N>& s, double b, int lane) {
  constexpr int n = KinDims<N>::n;
  const int row = lane < n ? lane : 0;
  double acc = b, y = 0.0;
#pragma unroll 2
  for (int k = 0; k < n; ++k) {  // forward: L y = b  (lane i reads L[i][k])
    const double yk = lane_bcast(acc, k) * s.dinv[k];
    if (lane == k) y = yk;
    acc -= s.Lm[row][k] * yk;
  }
  acc = y;
  double x = 0.0;
#pragma unroll 2
  for (int k = n - 1; k >= 0; --k) {  // backward: L' x = y  (lane i reads L[k][i])
    const double xk = lane_bcast(acc, k) * s.dinv[k];
    if (lane == k) x = xk;
    acc -= s.Lm[k][row] * xk;
  }
  return x;
}

// stage index (1..N-1) of constraint row r
template <int N>
__host__ __device__ constexpr int crow_stage(int r) {
  return r < N - 1 ? r + 1 : r - (N - 1) + 1;
}

// y_r = G_r . v for lane r (v broadcast in s.vz)
template <int N>
__device__ double grow_dot(const KinShared<N>& s, int lane) {
  constexpr int n = KinDims<N>::n, NC = KinDims<N>::NC;
  if (lane >= NC) return 0.0;
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < n - 2; ++i) acc += s.G[lane][i] * s.vz[i];  // rows have <= 2(N-1) nonzeros
  return acc;
}

// (G' v)_j for lane j (v broadcast in s.vc)
template <int N>
__device__ double gt_dot(const KinShared<N>& s, int lane) {
  constexpr int n = KinDims<N>::n, NC = KinDims<N>::NC;
  if (lane >= n) return 0.0;
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < NC; ++r) acc += s.G[r][lane] * s.vc[r];
  return acc;
}

// (H v)_j with H row j in registers (v broadcast in s.vz)
template <int N>
__device__ double h_dot(const double (&Hr)[KinDims<N>::n], const KinShared<N>& s) {
  constexpr int n = KinDims<N>::n;
  double acc = 0.0;
#pragma unroll
  for (int i = 0; i < n; ++i) acc += Hr[i] * s.vz[i];
  return acc;
}

// inequality side data of one lane role (box or state row)
struct Side {
  double lo, hi, slo, shi, llo, lhi;
  bool hasLo, hasHi;
};

template <int N>
__global__ __launch_bounds__(64) void kin_ltv_kernel(KinLtvArgs A) {
  using D = KinDims<N>;
  constexpr int n = D::n, NC = D::NC;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  KinShared<N>& s = *reinterpret_cast<KinShared<N>*>(smem_raw);
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= A.B) return;
  const vc_kin_mpc& W = A.w;

  // ---- load inputs (coalesced) -------------------------------------------
  if (lane < n) s.ub[lane] = A.ubar[(size_t)b * n + lane];
  if (lane < N) {
    s.kap[lane] = A.kappa[(size_t)b * N + lane];
    s.ds[lane] = A.ds[(size_t)b * N + lane];
  }
  if (lane < KIN_NX) s.xb[0][lane] = A.x0[(size_t)b * KIN_NX + lane];
  wave_sync();

  // ---- predict + linearize + condense (fused, one pass over the horizon) ---
  // Trajectory values are uniform across lanes; lane j also carries column j of
  // the sensitivity (dv, ddelta, dey, depsi, dt) w.r.t. dz_j.
  double x[KIN_NX];
#pragma unroll
  for (int i = 0; i < KIN_NX; ++i) x[i] = s.xb[0][i];
  double cv = 0, cd = 0, cey = 0, cep = 0, ct = 0;
  double Hr[n];
#pragma unroll
  for (int i = 0; i < n; ++i) Hr[i] = 0.0;
  double gj = 0.0;
  bool finite = true;

  for (int k = 0; k < N; ++k) {
    const double a = s.ub[2 * k], w = s.ub[2 * k + 1], kk = s.kap[k], h = s.ds[k];
    const KinJac J = kin_spatial_jac(x, kk, A.L);
    double u2[2] = {a, w}, f[KIN_NX], xn[KIN_NX];
    kin_spatial_ode(x, u2, kk, A.L, f);
    euler_apply<double, KIN_NX>(x, f, h, xn);
    // column update: c_{k+1} = A_k c_k + B_k e_j
    const double dq = J.qv * cv + J.qey * cey + J.qep * cep;
    const double ncv = cv + h * a * dq + (lane == 2 * k ? h * J.q : 0.0);
    const double ncd = cd + h * w * dq + (lane == 2 * k + 1 ? h * J.q : 0.0);
    const double ncey = cey + h * (J.J33 * cey + J.J34 * cep);
    const double ncep = cep + h * (J.J41 * cd + J.J43 * cey + J.J44 * cep);
    ct += h * dq;
    cv = ncv; cd = ncd; cey = ncey; cep = ncep;
#pragma unroll
    for (int i = 0; i < KIN_NX; ++i) {
      x[i] = xn[i];
      finite = finite && isfinite(xn[i]);
    }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < KIN_NX; ++i) s.xb[k + 1][i] = xn[i];
      s.jac[k][0] = J.q; s.jac[k][1] = J.qv; s.jac[k][2] = J.qey; s.jac[k][3] = J.qep;
      s.jac[k][4] = J.J33; s.jac[k][5] = J.J34; s.jac[k][6] = J.J41; s.jac[k][7] = J.J43;
      s.jac[k][8] = J.J44;
    }
    const int st = k + 1;  // stage of the updated column
    if (st <= N - 1 && lane < n) {
      s.G[st - 1][lane] = cv;            // row v_st
      s.G[(N - 1) + st - 1][lane] = cd;  // row delta_st
    }
    // ey_st cost: stage (deviation + boundary, kinematic_mpc.py:110-122) or terminal (:152-154)
    double cw, lin;
    const double ey = x[3];
    if (st < N) {
      const double hs = s.ds[st];
      cw = W.w_dev * hs;
      lin = W.w_dev * hs * ey;
      if (ey < W.ey_min) { cw += W.w_b * hs; lin += W.w_b * hs * (ey - W.ey_min); }
      if (ey > W.ey_max) { cw += W.w_b * hs; lin += W.w_b * hs * (ey - W.ey_max); }
    } else {
      cw = W.w_ey;
      lin = W.w_ey * ey;
    }
    double* cb = s.col[k & 1];
    cb[lane] = (lane < n) ? cey : 0.0;
    wave_sync();
    const double t2 = 2.0 * cw * cey;
#pragma unroll
    for (int i = 0; i < n; ++i) Hr[i] += t2 * cb[i];
    gj += 2.0 * lin * cey;
  }
  // terminal rows on v_N (kinematic_mpc.py:144-148), epsi_N (:155-157), t_N (:149-151)
  {
    const double vN = x[0];
    const double cw = (vN >= W.v_max) ? W.w_v : 0.0;
    double* cb = s.col[0];
    cb[lane] = (lane < n) ? cv : 0.0;
    wave_sync();
    const double t2 = 2.0 * cw * cv;
#pragma unroll
    for (int i = 0; i < n; ++i) Hr[i] += t2 * cb[i];
    gj += 2.0 * cw * (vN - W.v_max) * cv;
    double* cb1 = s.col[1];
    cb1[lane] = (lane < n) ? cep : 0.0;
    wave_sync();
    const double t3 = 2.0 * W.w_epsi * cep;
#pragma unroll
    for (int i = 0; i < n; ++i) Hr[i] += t3 * cb1[i];
    gj += 2.0 * W.w_epsi * x[4] * cep;
    gj += W.w_time * ct;
  }
  // input costs: w_w w^2 (kinematic_mpc.py:124), slew w_a (a_{n+1}-a_n)^2 (:126-128), prox
  {
    const int kq = lane >> 1;
    double dself = 2.0 * A.qp.prox, dm2 = 0.0, dp2 = 0.0;
    if (lane < n) {
      if (lane & 1) {
        dself += 2.0 * W.w_w;
        gj += 2.0 * W.w_w * s.ub[lane];
      } else {
        if (kq >= 1) {
          dself += 2.0 * W.w_a; dm2 = -2.0 * W.w_a;
          gj += 2.0 * W.w_a * (s.ub[lane] - s.ub[lane - 2]);
        }
        if (kq <= N - 2) {
          dself += 2.0 * W.w_a; dp2 = -2.0 * W.w_a;
          gj -= 2.0 * W.w_a * (s.ub[lane + 2] - s.ub[lane]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < n; ++i) {
      if (i == lane) Hr[i] += dself;
      if (i == lane - 2) Hr[i] += dm2;
      if (i == lane + 2) Hr[i] += dp2;
    }
  }
  if (lane >= n) gj = 0.0;
  wave_sync();
  if (A.mode == 1) {  // vc_condense: expose the QP data of the fused kernel
    if (lane < n) {
#pragma unroll
      for (int i = 0; i < n; ++i) A.H_out[((size_t)b * n + lane) * n + i] = Hr[i];
      A.g_out[(size_t)b * n + lane] = gj;
    }
    return;
  }

  // ---- inequality data ------------------------------------------------------
  Side bx, cs;  // box side (lane j < n), state-row side (lane r < NC)
  {
    const bool isw = lane & 1;
    const double u = (lane < n) ? s.ub[lane] : 0.0;
    bx.lo = (isw ? W.w_min : W.a_min) - u;
    bx.hi = (isw ? W.w_max : W.a_max) - u;
    bx.hasLo = bx.hasHi = (lane < n);
    const int st = crow_stage<N>(lane < NC ? lane : 0);
    if (lane < N - 1) {
      cs.lo = W.v_min - s.xb[st][0];
      cs.hi = 0.0;
      cs.hasLo = true; cs.hasHi = false;
    } else if (lane < NC) {
      cs.lo = W.delta_min - s.xb[st][1];
      cs.hi = W.delta_max - s.xb[st][1];
      cs.hasLo = cs.hasHi = true;
    } else {
      cs.lo = cs.hi = 0.0;
      cs.hasLo = cs.hasHi = false;
    }
  }
  const double mtot = double(4 * N + 3 * (N - 1));
  double scale, hdiag_max;
  {
    double m = fabs(gj);
    if (bx.hasLo) m = fmax(m, fabs(bx.lo));
    if (bx.hasHi) m = fmax(m, fabs(bx.hi));
    if (cs.hasLo) m = fmax(m, fabs(cs.lo));
    if (cs.hasHi) m = fmax(m, fabs(cs.hi));
    scale = 1.0 + wave_max(m);
    double dg = 0.0;
#pragma unroll
    for (int i = 0; i < n; ++i)
      if (i == lane) dg = Hr[i];
    hdiag_max = fmax(wave_max(dg), 1.0);
  }
  // start point dz = 0, slacks max(d, 1), multipliers 1 (oracle/qp.py uses the same rule)
  double z = 0.0;
  bx.slo = bx.hasLo ? fmax(-bx.lo, 1.0) : 1.0;
  bx.shi = bx.hasHi ? fmax(bx.hi, 1.0) : 1.0;
  bx.llo = bx.hasLo ? 1.0 : 0.0;
  bx.lhi = bx.hasHi ? 1.0 : 0.0;
  cs.slo = cs.hasLo ? fmax(-cs.lo, 1.0) : 1.0;
  cs.shi = cs.hasHi ? fmax(cs.hi, 1.0) : 1.0;
  cs.llo = cs.hasLo ? 1.0 : 0.0;
  cs.lhi = cs.hasHi ? 1.0 : 0.0;

  // ---- solver state machine ---------------------------------------------------
  // Phase PDIP: Mehrotra predictor-corrector on the normal equations
  //   (H + C'WC) dz = -rd - C'e.
  // Phase POLISH: crossover to the active set the interior point identified:
  //   box-active inputs are fixed (identity rows), active state rows are imposed
  //   with an augmented Lagrangian (P + rho C_A'C_A), whose multiplier update
  //   converges in a few solves with one factorisation; the set is repaired
  //   until primal and dual feasible (oracle/qp.py:polish does the same with a
  //   direct KKT solve).  Every phase shares one matrix build, one Cholesky and
  //   one solve site, keeping the unrolled code and register footprint small.
  enum { PH_PDIP = 0, PH_POLISH = 1, PH_DONE = 2 };
  constexpr double AL_RHO = 100.0;
  constexpr int AL_MAX = 8;
  const int max_iter = A.qp.max_iter;
  const double tol = A.qp.tol * scale;
  const double ptol = 1e-11 * scale;
  int phase = finite ? PH_PDIP : PH_DONE;
  int it = 0, rounds = 0;
  bool converged = false, polished = false;
  double Mr[n];
  // polish state
  bool alo_b = false, ahi_b = false, alo_c = false, ahi_c = false;
  bool fixed = false;
  double zfix = 0.0, rho_c = 0.0, nu_c = 0.0, bnd_c = 0.0, base = 0.0;
  uint64_t fmask = 0ull;
  // PDIP per-iteration quantities
  double rd = 0, rlo_b = 0, rhi_b = 0, rlo_c = 0, rhi_c = 0, mu = 0;
  double wlo_b = 0, whi_b = 0, wlo_c = 0, whi_c = 0;
  double pa1 = 0, pa2 = 0, pa3 = 0, pa4 = 0, pc1 = 0, pc2 = 0, pc3 = 0, pc4 = 0;  // predictor directions

  while (phase != PH_DONE) {
    double wb = 0.0, wc = 0.0;
    if (phase == PH_PDIP) {
      wave_sync();
      if (lane < n) s.vz[lane] = z;
      s.vc[lane] = (lane < NC) ? (cs.lhi - cs.llo) : 0.0;
      wave_sync();
      const double yc = grow_dot<N>(s, lane);
      rd = (lane < n) ? (h_dot<N>(Hr, s) + gj + (bx.lhi - bx.llo) + gt_dot<N>(s, lane)) : 0.0;
      rlo_b = bx.hasLo ? (z - bx.lo - bx.slo) : 0.0;
      rhi_b = bx.hasHi ? (bx.hi - z - bx.shi) : 0.0;
      rlo_c = cs.hasLo ? (yc - cs.lo - cs.slo) : 0.0;
      rhi_c = cs.hasHi ? (cs.hi - yc - cs.shi) : 0.0;
      mu = wave_sum(bx.slo * bx.llo + bx.shi * bx.lhi + cs.slo * cs.llo + cs.shi * cs.lhi) / mtot;
      const double res =
          wave_max(fmax(fmax(fabs(rd), fmax(fabs(rlo_b), fabs(rhi_b))), fmax(fabs(rlo_c), fabs(rhi_c))));
      const bool stop = (res <= tol && mu <= tol) || it >= max_iter || !isfinite(res) || !isfinite(mu);
      if (stop) {
        converged = (res <= tol && mu <= tol);
        if (A.qp.polish > 0 && isfinite(res) && isfinite(mu)) {
          phase = PH_POLISH;
          alo_b = bx.hasLo && bx.llo > bx.slo;
          ahi_b = bx.hasHi && bx.lhi > bx.shi;
          alo_c = cs.hasLo && cs.llo > cs.slo;
          ahi_c = cs.hasHi && cs.lhi > cs.shi;
        } else {
          phase = PH_DONE;
        }
        continue;
      }
      ++it;
      wlo_b = bx.hasLo ? bx.llo / bx.slo : 0.0;
      whi_b = bx.hasHi ? bx.lhi / bx.shi : 0.0;
      wlo_c = cs.hasLo ? cs.llo / cs.slo : 0.0;
      whi_c = cs.hasHi ? cs.lhi / cs.shi : 0.0;
      wb = wlo_b + whi_b;
      wc = wlo_c + whi_c;
      fmask = 0ull;
      fixed = false;
    } else {  // PH_POLISH: set up the reduced problem of this round
      if (rounds >= A.qp.polish) { phase = PH_DONE; continue; }
      ++rounds;
      fixed = (lane < n) && (alo_b || ahi_b);
      zfix = alo_b ? bx.lo : (ahi_b ? bx.hi : 0.0);
      if (!fixed) zfix = 0.0;
      fmask = __ballot(fixed);
      const bool act = (lane < NC) && (alo_c || ahi_c);
      bnd_c = alo_c ? cs.lo : cs.hi;
      wave_sync();
      if (lane < n) s.vz[lane] = zfix;
      wave_sync();
      // fixed-variable part of each active row, and its free-part norm for rho
      const double gfix = grow_dot<N>(s, lane);
      double gn2 = 0.0;
      if (lane < NC) {
#pragma unroll
        for (int i = 0; i < n - 2; ++i) {
          const double gi = ((fmask >> i) & 1ull) ? 0.0 : s.G[lane][i];
          gn2 += gi * gi;
        }
      }
      rho_c = act ? AL_RHO * hdiag_max / fmax(gn2, 1e-300) : 0.0;
      if (act && gn2 <= 1e-28) { rho_c = 0.0; }  // row fully determined by fixed inputs
      nu_c = 0.0;
      bnd_c = act ? (bnd_c - gfix) : 0.0;  // b' = b - G_X zfix
      base = (lane < n) ? -(gj + h_dot<N>(Hr, s)) : 0.0;
      wb = 0.0;
      wc = rho_c;
    }

    // ---- matrix build: Mr = row `lane` of H + diag(wb) + sum_r wc_r g_r g_r' ----
    wave_sync();
    s.vc[lane] = wc;
    wave_sync();
#pragma unroll
    for (int i = 0; i < n; ++i) Mr[i] = Hr[i] + (i == lane ? wb : 0.0);
#pragma unroll
    for (int r = 0; r < NC; ++r) {
      const double t = s.vc[r] * ((lane < n) ? s.G[r][lane] : 0.0);
      const int nz = 2 * crow_stage<N>(r);
#pragma unroll
      for (int i = 0; i < nz; ++i) Mr[i] += t * s.G[r][i];
    }
    if (fmask) {  // reduced matrix: fixed rows/cols -> identity
#pragma unroll
      for (int i = 0; i < n; ++i) {
        const bool fi = (fmask >> i) & 1ull;
        Mr[i] = fixed ? (i == lane ? 1.0 : 0.0) : (fi ? 0.0 : Mr[i]);
      }
    }
    if (lane >= n) {
#pragma unroll
      for (int i = 0; i < n; ++i) Mr[i] = 0.0;
    }
    if (!chol_rows<N>(Mr, s, lane)) { phase = PH_DONE; continue; }

    // ---- solve passes ----------------------------------------------------------
    const int npass = (phase == PH_PDIP) ? 2 : AL_MAX;
    double zp = 0.0;
#pragma unroll 1
    for (int pass = 0; pass < npass; ++pass) {
      double rhs;
      double rclo_b = 0, rchi_b = 0, rclo_c = 0, rchi_c = 0;
      if (phase == PH_PDIP) {
        if (pass == 0) {  // predictor (affine scaling)
          rclo_b = bx.slo * bx.llo; rchi_b = bx.shi * bx.lhi;
          rclo_c = cs.slo * cs.llo; rchi_c = cs.shi * cs.lhi;
        } else {          // Mehrotra corrector
          const double aa = wave_min(fmin(
              fmin(fmin(step_bound(bx.slo, pa1), step_bound(bx.llo, pa2)),
                   fmin(step_bound(bx.shi, pa3), step_bound(bx.lhi, pa4))),
              fmin(fmin(step_bound(cs.slo, pc1), step_bound(cs.llo, pc2)),
                   fmin(step_bound(cs.shi, pc3), step_bound(cs.lhi, pc4)))));
          const double mua =
              wave_sum((bx.slo + aa * pa1) * (bx.llo + aa * pa2) + (bx.shi + aa * pa3) * (bx.lhi + aa * pa4) +
                       (cs.slo + aa * pc1) * (cs.llo + aa * pc2) + (cs.shi + aa * pc3) * (cs.lhi + aa * pc4)) /
              mtot;
          const double sr = mua / mu;
          const double sm = sr * sr * sr * mu;  // sigma * mu with sigma = (mu_aff / mu)^3
          rclo_b = bx.slo * bx.llo + pa1 * pa2 - sm;
          rchi_b = bx.shi * bx.lhi + pa3 * pa4 - sm;
          rclo_c = cs.slo * cs.llo + pc1 * pc2 - sm;
          rchi_c = cs.shi * cs.lhi + pc3 * pc4 - sm;
        }
        const double eb = (bx.hasHi ? (-rchi_b / bx.shi - whi_b * rhi_b) : 0.0) +
                          (bx.hasLo ? (rclo_b / bx.slo + wlo_b * rlo_b) : 0.0);
        const double ec = (cs.hasHi ? (-rchi_c / cs.shi - whi_c * rhi_c) : 0.0) +
                          (cs.hasLo ? (rclo_c / cs.slo + wlo_c * rlo_c) : 0.0);
        wave_sync();
        s.vc[lane] = (lane < NC) ? ec : 0.0;
        wave_sync();
        rhs = (lane < n) ? (-rd - eb - gt_dot<N>(s, lane)) : 0.0;
      } else {  // augmented-Lagrangian pass on the active set
        wave_sync();
        s.vc[lane] = (lane < NC) ? (nu_c - rho_c * bnd_c) : 0.0;
        wave_sync();
        rhs = (lane < n) ? (fixed ? zfix : (base - gt_dot<N>(s, lane))) : 0.0;
      }

      const double dz = chol_solve<N>(s, rhs, lane);  // the one solve site

      wave_sync();
      if (lane < n) s.vz[lane] = dz;
      wave_sync();
      const double dyc = grow_dot<N>(s, lane);
      if (phase == PH_PDIP) {
        const double dyb = dz;
        const double d1 = bx.hasLo ? dyb + rlo_b : 0.0;
        const double d2 = bx.hasLo ? (-rclo_b / bx.slo - wlo_b * (dyb + rlo_b)) : 0.0;
        const double d3 = bx.hasHi ? rhi_b - dyb : 0.0;
        const double d4 = bx.hasHi ? (-rchi_b / bx.shi - whi_b * (rhi_b - dyb)) : 0.0;
        const double e1 = cs.hasLo ? dyc + rlo_c : 0.0;
        const double e2 = cs.hasLo ? (-rclo_c / cs.slo - wlo_c * (dyc + rlo_c)) : 0.0;
        const double e3 = cs.hasHi ? rhi_c - dyc : 0.0;
        const double e4 = cs.hasHi ? (-rchi_c / cs.shi - whi_c * (rhi_c - dyc)) : 0.0;
        if (pass == 0) {
          pa1 = d1; pa2 = d2; pa3 = d3; pa4 = d4;
          pc1 = e1; pc2 = e2; pc3 = e3; pc4 = e4;
        } else {
          const double al = 0.99 * wave_min(fmin(
                                       fmin(fmin(step_bound(bx.slo, d1), step_bound(bx.llo, d2)),
                                            fmin(step_bound(bx.shi, d3), step_bound(bx.lhi, d4))),
                                       fmin(fmin(step_bound(cs.slo, e1), step_bound(cs.llo, e2)),
                                            fmin(step_bound(cs.shi, e3), step_bound(cs.lhi, e4)))));
          if (lane < n) z += al * dz;
          bx.slo += al * d1; bx.llo += al * d2; bx.shi += al * d3; bx.lhi += al * d4;
          cs.slo += al * e1; cs.llo += al * e2; cs.shi += al * e3; cs.lhi += al * e4;
        }
      } else {
        zp = dz;
        // dyc = G_r . zp (zp carries zfix on fixed lanes): multiplier update
        const bool act = (lane < NC) && (alo_c || ahi_c) && rho_c > 0.0;
        const double e = act ? (dyc - (alo_c ? cs.lo : cs.hi)) : 0.0;
        nu_c += rho_c * e;
        if (wave_max(fabs(e)) <= 1e-14 * scale) break;
      }
    }
    if (phase == PH_PDIP) continue;

    // ---- polish: KKT check of zp and active-set repair --------------------------
    wave_sync();
    if (lane < n) s.vz[lane] = zp;
    s.vc[lane] = (lane < NC) ? nu_c : 0.0;
    wave_sync();
    const double grad = (lane < n) ? (h_dot<N>(Hr, s) + gj + gt_dot<N>(s, lane)) : 0.0;
    const double ypc = grow_dot<N>(s, lane);
    bool ok = true;
    bool n_alo_b = alo_b, n_ahi_b = ahi_b, n_alo_c = alo_c, n_ahi_c = ahi_c;
    if (lane < n) {
      if (ahi_b && -grad < -ptol) { ok = false; n_ahi_b = false; }
      if (alo_b && grad < -ptol) { ok = false; n_alo_b = false; }
      if (!fixed) {
        if (zp < bx.lo - ptol) { ok = false; n_alo_b = true; }
        if (zp > bx.hi + ptol) { ok = false; n_ahi_b = true; }
      }
    }
    if (lane < NC) {
      if (ahi_c && nu_c < -ptol) { ok = false; n_ahi_c = false; }
      if (alo_c && -nu_c < -ptol) { ok = false; n_alo_c = false; }
      if (!(alo_c || ahi_c)) {
        if (cs.hasLo && ypc < cs.lo - ptol) { ok = false; n_alo_c = true; }
        if (cs.hasHi && ypc > cs.hi + ptol) { ok = false; n_ahi_c = true; }
      } else if (fabs(ypc - (alo_c ? cs.lo : cs.hi)) > ptol) {
        ok = false;  // equality not met (e.g. a row left fully fixed by the inputs)
        n_alo_c = n_ahi_c = false;
      }
    }
    if (__ballot(!ok) == 0ull) {
      z = zp;
      polished = true;
      phase = PH_DONE;
    } else {
      alo_b = n_alo_b; ahi_b = n_ahi_b; alo_c = n_alo_c; ahi_c = n_ahi_c;
    }
  }

  // ---- outputs -------------------------------------------------------------------
  int32_t st;
  if (!finite) st = VC_NONFINITE;
  else if (polished || (converged && A.qp.polish <= 0)) st = VC_SOLVED;
  else st = VC_MAX_ITER;
  if (!finite) z = 0.0;
  wave_sync();
  if (lane < n) {
    s.vz[lane] = z;
    A.u_out[(size_t)b * n + lane] = s.ub[lane] + z;
  }
  wave_sync();
  if (lane < 2) A.u0[(size_t)b * 2 + lane] = s.ub[lane] + s.vz[lane];
  if (lane == 0) {
    A.status[b] = st;
    A.iters[b] = it;
  }
  // x* = xbar + G dz via the linearised recursion, lanes 0..5 own components
  double dx[KIN_NX] = {0, 0, 0, 0, 0, 0};
  double* xo = A.x_out + (size_t)b * (N + 1) * KIN_NX;
  if (lane < KIN_NX) xo[lane] = s.xb[0][lane];
  for (int k = 0; k < N; ++k) {
    const double q = s.jac[k][0], qv = s.jac[k][1], qey = s.jac[k][2], qep = s.jac[k][3];
    const double h = s.ds[k], a = s.ub[2 * k], w = s.ub[2 * k + 1];
    const double da = s.vz[2 * k], dw = s.vz[2 * k + 1];
    const double dq = qv * dx[0] + qey * dx[3] + qep * dx[4];
    double nx[KIN_NX];
    nx[0] = dx[0] + h * (a * dq + q * da);
    nx[1] = dx[1] + h * (w * dq + q * dw);
    nx[2] = dx[2];
    nx[3] = dx[3] + h * (s.jac[k][4] * dx[3] + s.jac[k][5] * dx[4]);
    nx[4] = dx[4] + h * (s.jac[k][6] * dx[1] + s.jac[k][7] * dx[3] + s.jac[k][8] * dx[4]);
    nx[5] = dx[5] + h * dq;
    double mine = 0.0;
#pragma unroll
    for (int i = 0; i < KIN_NX; ++i) {
      dx[i] = nx[i];
      if (i == lane) mine = nx[i];
    }
    if (lane < KIN_NX) xo[(k + 1) * KIN_NX + lane] = s.xb[k + 1][lane] + mine;
  }
}

}  // namespace vc

// ---- host launcher ---------------------------------------------------------------
namespace vc {
size_t kin_ltv_smem_bytes(int N) {
  switch (N) {
    case 20: return sizeof(KinShared<20>);
    default: return 0;
  }
}

hipError_t launch_kin_ltv(const KinLtvArgs& a, int N, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  switch (N) {
    case 20:
      hipLaunchKernelGGL(kin_ltv_kernel<20>, dim3(a.B), dim3(64), sizeof(KinShared<20>), stream, a);
      return hipGetLastError();
    default:
      return hipErrorInvalidValue;
  }
}
}  // namespace vc
