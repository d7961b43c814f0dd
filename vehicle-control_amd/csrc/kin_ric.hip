// kin_ric.hip -- fused kinematic LTV-MPC step, fp64, one wavefront per problem, with a
// stagewise Riccati interior point: any horizon N <= 63.
//
// Replaces the IPOPT solve of KinematicMPC.command (controllers/mpc/kinematic_mpc.py:
// 160-168; NLP :71-158) at the reference's own horizon (config/controllers/kinematic.yaml
// N = 50), where the condensed kernel kin_ltv.hip (n = 2N decision variables, an O(n^3)
// factorisation per iteration, one lane per variable) does not fit.  Contract: the LTV-QP
// of oracle/ltv_qp.py (the same QP kin_ltv.hip solves), restated stage by stage as in
// scripts/kin_riccati_proto.py:
//   QP state xt_k = (dv, ddelta, dey, depsi, p_k), p_k = da_{k-1} (the slew w_a (a_{k+1} -
//   a_k)^2 couples neighbouring inputs), input u_k = (da, dw), stages k = 0..N (stage N has
//   no input).  s is fixed (s' = 1) and t only enters the terminal w_time t_N, which becomes
//   a linear stage term through each step's t-row.  Every constraint row is a bound on one
//   stage variable (input boxes k < N, v / delta rows 1 <= k <= N-1), so the barrier
//   Hessian is diagonal and the stage Hessians keep the pattern diag + (p, da).
// Per problem:
//   predict    lane 0: spatial Euler rollout (vc_models.hpp kin_spatial_ode)
//   linearize  lane k: analytic Jacobian of step k (kin_spatial_jac) -> [A4 | B4], t-row
//   QP         Mehrotra predictor-corrector; each Newton step is an LQ problem solved by a
//              backward Riccati recursion over the 5-state / 2-input stages and a forward
//              rollout.  Lane k owns stage k's rows, slacks and multipliers in registers.
//   polish     once mu <= 1e-7 (again at 1e-10, or when the recursion fails): the active set (lam > s) is imposed by an augmented
//              Lagrangian (rho = 1e4, one factorisation, <= 16 multiplier passes until the
//              active rows hold to 1e-13) and certified (inactive rows feasible, multipliers >= 0) -- the crossover of
//              kin_ltv.hip restated stagewise.  The Riccati recursion of the interior
//              point itself loses accuracy once barrier weights reach ~1e10 (cancellation
//              in P = Hxx - Hxu Huu^-1 Hux), so the exact answer comes from the polish.
//   output     u* = ubar + du, x* = xbar + dx (t from the t-rows), u0, status, iterations.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vc_kernels.hpp"

namespace vc {
namespace {

constexpr int WTH = 64;
constexpr int NXT = 5;  // QP state (dv, ddelta, dey, depsi, p)
constexpr int NV = 7;   // stage vector (xt, da, dw)
constexpr int NRW = 7;  // one-sided rows per stage
// Stage Hessian slots: the diagonal D0..D6 and the slew coupling (p, da).
enum { D0 = 0, O45 = 7, NQK = 8 };
constexpr double RHO_AL = 1e4;     // augmented-Lagrangian weight of the polish
constexpr int AL_PASSES = 16;
constexpr double MU_POLISH = 1e-7;  // complementarity at which the polish is first tried
constexpr double TOL_CERT = 1e-9;   // feasibility / multiplier sign tolerance of the certificate
constexpr double EPS_T = 1e-8;      // elastic slacks' quadratic cost (oracle/ltv_qp.py ELASTIC_EPS_T)

// Row i: sign * v[var] <= d:  da <=, -da <=, dw <=, -dw <=, -dv <=, ddelta <=, -ddelta <=
__host__ __device__ constexpr int row_var(int i) { return i < 2 ? 5 : (i < 4 ? 6 : (i == 4 ? 0 : 1)); }
__host__ __device__ constexpr double row_sgn(int i) { return (i == 0 || i == 2 || i == 5) ? 1.0 : -1.0; }
// stage vector index -> column of [A4 | B4] (-1 for p: no dynamics enters through it)
__host__ __device__ constexpr int fcol(int j) { return j < 4 ? j : (j == 4 ? -1 : j - 1); }

template <int N>
struct KrSmem {
  double xs[N + 1][6];  // prediction (becomes x* at the end)
  double ew[N + 1][5];  // multiple shooting: their linear rollout e over (v, delta, ey, epsi | t)
  double ub[N][2];
  double kap[N], dsv[N];
  double F[N][4][6];    // [A4 | B4]: rows (v, delta, ey, epsi), cols (v, delta, ey, epsi | a, w)
  double tr[N][4];      // t-row of step k over (v, delta, ey, epsi)
  double Qt[N + 1][NQK];
  double gr[N + 1][NV];
  // the LQ right-hand side h lives in the interior point / polish only; before it, in the
  // multiple-shooting setup, the same space holds the defects -- at N = 50 this keeps the block
  // at <= 39,936 B, four workgroups per CU instead of three (rocprofv3 LDS_Block_Size)
  union {
    double cdef[N][6];  // multiple shooting: defects F(xs_k, ub_k) - xs_{k+1} (setup only)
    double h[N + 1][NV];
  };
  double v[N + 1][NV];
  double dv[N + 1][NV];
  double K[N][2][NXT];
  double Hi[N][3];
  double kk[N][2];
  double P[NXT][NXT];
  double T[NXT][NV];
  double Hm[NV][NV];
  int flag;
};

#ifndef KR_RES_RECUR
#define KR_RES_RECUR 1  // dual residual carried by the steps (0: adjoint sweep every iteration)
#endif

#define WSYNC()                          \
  do {                                   \
    asm volatile("" ::: "memory");       \
    __builtin_amdgcn_wave_barrier();     \
    asm volatile("" ::: "memory");       \
  } while (0)

__device__ __forceinline__ double bcast(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double step_to_bound(double x, double dx) { return dx < 0.0 ? -x / dx : 1e300; }

// out = Qc v for the diag + (p, da) pattern
__device__ __forceinline__ void qmul(const double* Q, const double* v, double* o) {
#pragma unroll
  for (int e = 0; e < NV; ++e) o[e] = Q[D0 + e] * v[e];
  o[4] += Q[O45] * v[5];
  o[5] += Q[O45] * v[4];
}

template <int N>
__global__ __launch_bounds__(WTH) void kin_ric_kernel(KinLtvArgs A) {
  static_assert(N >= 2 && N + 1 <= WTH, "one lane per stage");
  __shared__ KrSmem<N> s;
  const int l = threadIdx.x;
  const int b = blockIdx.x;  // identity placement: xcd_problem measured 21 % slower at N = 50
  // elastic-on-failure pass (qp.elastic < 0, launched by vc_solve after the hard-row pass): only
  // the problems that pass left non-solved are solved again, with elastic rows at -qp.elastic
  if (A.qp.elastic < 0.0 && A.status[b] == VC_SOLVED) return;
  const vc_kin_mpc& W = A.w;
  const bool stl = l <= N;   // lane owns stage l = 0..N
  const int k = stl ? l : N;

  for (int i = l; i < N; i += WTH) {
    s.kap[i] = A.kappa[(size_t)b * N + i];
    s.dsv[i] = A.ds[(size_t)b * N + i];
    s.ub[i][0] = A.ubar[((size_t)b * N + i) * 2];
    s.ub[i][1] = A.ubar[((size_t)b * N + i) * 2 + 1];
  }
  if (l < 6) s.xs[0][l] = A.x0[(size_t)b * 6 + l];
  if (l == 0) s.flag = VC_SOLVED;
  WSYNC();

  const bool ms = A.qp.ms != 0;
  if (ms) {  // multiple shooting: the warm-start states, x0 in column 0, s = s0 + sum ds (s' = 1)
    for (int e = l; e < 6 * N; e += WTH) s.xs[1 + e / 6][e % 6] = A.x_in[(size_t)b * 6 * (N + 1) + 6 + e];
    WSYNC();
    if (l == 0) {
      double sa = s.xs[0][2];
      bool fin = true;
      for (int kk = 0; kk < N; ++kk) {
        sa += s.dsv[kk];
        s.xs[kk + 1][2] = sa;
#pragma unroll
        for (int i = 0; i < 6; ++i) fin = fin && isfinite(s.xs[kk + 1][i]);
      }
      if (!fin) s.flag = VC_NONFINITE;
    }
  }
  // ---------------- predict (lane 0, serial spatial Euler) ----------------
  if (!ms && l == 0) {
    double x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = s.xs[0][i];
    bool fin = true;
    for (int kk = 0; kk < N; ++kk) {
      const double u2[2] = {s.ub[kk][0], s.ub[kk][1]};
      double f[6], xn[6];
      kin_spatial_ode<double>(x, u2, s.kap[kk], A.L, f);
      euler_apply<double, 6>(x, f, s.dsv[kk], xn);
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        x[i] = xn[i];
        s.xs[kk + 1][i] = xn[i];
        fin = fin && isfinite(xn[i]);
      }
    }
    if (!fin) s.flag = VC_NONFINITE;
  }
  WSYNC();
  const bool finite_pred = s.flag != VC_NONFINITE;

  // ---------------- linearize (lane k < N) ----------------
  if (l < N) {
    double xk[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) xk[i] = s.xs[l][i];
    const KinJac J = kin_spatial_jac(xk, s.kap[l], A.L);
    const double ds = s.dsv[l], a = s.ub[l][0], w = s.ub[l][1];
    // A = I + ds d f'/dx, B = ds d f'/du (kinematic_car.py:48-60; vc_models.hpp KinJac)
    const double r0[6] = {1.0 + ds * (J.qv * a), 0.0, ds * (J.qey * a), ds * (J.qep * a), ds * J.q, 0.0};
    const double r1[6] = {ds * (J.qv * w), 1.0, ds * (J.qey * w), ds * (J.qep * w), 0.0, ds * J.q};
    const double r2[6] = {0.0, 0.0, 1.0 + ds * J.J33, ds * J.J34, 0.0, 0.0};
    const double r3[6] = {0.0, ds * J.J41, ds * J.J43, 1.0 + ds * J.J44, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      s.F[l][0][c] = r0[c];
      s.F[l][1][c] = r1[c];
      s.F[l][2][c] = r2[c];
      s.F[l][3][c] = r3[c];
    }
    s.tr[l][0] = ds * J.qv;
    s.tr[l][1] = 0.0;
    s.tr[l][2] = ds * J.qey;
    s.tr[l][3] = ds * J.qep;
    if (ms) {  // defect of step l
      const double u2[2] = {a, w};
      double f[6];
      kin_spatial_ode<double>(xk, u2, s.kap[l], A.L, f);
#pragma unroll
      for (int i = 0; i < 6; ++i) s.cdef[l][i] = xk[i] + ds * f[i] - s.xs[l + 1][i];
    }
  }
  WSYNC();
  if (ms && l == 0) {  // e_0 = 0, e_{k+1} = A_k e_k + c_k over (v, delta, ey, epsi) and t
    double e[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    constexpr int ix[4] = {0, 1, 3, 4};
#pragma unroll
    for (int a = 0; a < 5; ++a) s.ew[0][a] = 0.0;
    for (int kk = 0; kk < N; ++kk) {
      double en[5];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double acc = s.cdef[kk][ix[r]];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc += s.F[kk][r][c] * e[c];
        en[r] = acc;
      }
      double et = e[4] + s.cdef[kk][5];
#pragma unroll
      for (int c = 0; c < 4; ++c) et += s.tr[kk][c] * e[c];
      en[4] = et;
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        e[a] = en[a];
        s.ew[kk + 1][a] = en[a];
      }
    }
  }
  WSYNC();

  // ---------------- stage QP data (lane k, registers) ----------------
  double Qc[NQK], qc[NV], d[NRW], m[NRW];
#pragma unroll
  for (int e = 0; e < NQK; ++e) Qc[e] = 0.0;
#pragma unroll
  for (int e = 0; e < NV; ++e) qc[e] = 0.0;
  {
    const double ey = s.xs[k][3];
    if (k >= 1 && k < N) {  // stage costs on ey (kinematic_mpc.py:110-122), obstacles (:130-133)
      const double ds = s.dsv[k];
      const double cdev = W.w_dev * ds;
      const double blo = ey < W.ey_min ? W.w_b * ds : 0.0, bhi = ey > W.ey_max ? W.w_b * ds : 0.0;
      Qc[D0 + 2] += 2.0 * (cdev + blo + bhi);
      qc[2] += 2.0 * (cdev * ey + blo * (ey - W.ey_min) + bhi * (ey - W.ey_max));
      if (A.obs.n > 0) {
        double po, qo;
        obstacle_ey_model<double>(A.obs, s.xs[k][2], ey, W.w_obs * ds, po, qo);
        Qc[D0 + 2] += qo;
        qc[2] += po;
      }
    }
    if (k < N) {
      // w_w w^2 (:124), prox on both inputs
      Qc[D0 + 6] += 2.0 * W.w_w + 2.0 * A.qp.prox;
      qc[6] += 2.0 * W.w_w * s.ub[k][1];
      Qc[D0 + 5] += 2.0 * A.qp.prox;
      // slew w_a (a_k - a_{k-1})^2 (:126-128) in (p_k, da_k)
      if (k >= 1) {
        const double c2 = 2.0 * W.w_a, r0 = s.ub[k][0] - s.ub[k - 1][0];
        Qc[D0 + 4] += c2;
        Qc[D0 + 5] += c2;
        Qc[O45] -= c2;
        qc[4] -= c2 * r0;
        qc[5] += c2 * r0;
      }
      // w_time t_N = sum_k t-row_k . y_k (:152)
#pragma unroll
      for (int a = 0; a < 4; ++a) qc[a] += W.w_time * s.tr[k][a];
    } else {  // terminal (:144-157)
      const double vN = s.xs[N][0];
      if (vN >= W.v_max) {
        Qc[D0] += 2.0 * W.w_v;
        qc[0] += 2.0 * W.w_v * (vN - W.v_max);
      }
      Qc[D0 + 2] += 2.0 * W.w_ey;
      qc[2] += 2.0 * W.w_ey * ey;
      Qc[D0 + 3] += 2.0 * W.w_epsi;
      qc[3] += 2.0 * W.w_epsi * s.xs[N][4];
    }
    // rows (:80-93; the optional trust region tightens the input boxes)
    const double mi = (stl && k < N) ? 1.0 : 0.0, mx = (stl && k >= 1 && k < N) ? 1.0 : 0.0;
    const double ab = k < N ? s.ub[k][0] : 0.0, wb = k < N ? s.ub[k][1] : 0.0;
    double upa = W.a_max - ab, dna = ab - W.a_min, upw = W.w_max - wb, dnw = wb - W.w_min;
    if (A.qp.trust_a > 0) {
      upa = fmin(upa, A.qp.trust_a);
      dna = fmin(dna, A.qp.trust_a);
    }
    if (A.qp.trust_w > 0) {
      upw = fmin(upw, A.qp.trust_w);
      dnw = fmin(dnw, A.qp.trust_w);
    }
    d[0] = upa;
    d[1] = dna;
    d[2] = upw;
    d[3] = dnw;
    d[4] = s.xs[k][0] - W.v_min;
    d[5] = W.delta_max - s.xs[k][1];
    d[6] = s.xs[k][1] - W.delta_min;
    if (ms) {  // v = e + w: linear terms q + Q e, row bounds d - C e (all stage-local)
#pragma unroll
      for (int a = 0; a < 4; ++a) qc[a] += Qc[D0 + a] * s.ew[k][a];
      d[4] += s.ew[k][0];
      d[5] -= s.ew[k][1];
      d[6] += s.ew[k][1];
    }
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      m[i] = i < 4 ? mi : mx;
      if (m[i] == 0.0) d[i] = 1.0;
    }
  }
  double qmax = 0.0;
#pragma unroll
  for (int e = 0; e < NV; ++e) qmax = fmax(qmax, fabs(qc[e]));
  qmax = wmax(stl ? qmax : 0.0);
  double sl[NRW], la[NRW];
#pragma unroll
  for (int i = 0; i < NRW; ++i) {
    sl[i] = m[i] > 0.0 ? fmax(d[i], 1.0) : 1.0;
    la[i] = m[i];
  }
  // elastic state rows (vc_qp.elastic = rho > 0): the slack t >= 0 of row 4 + j and its
  // multiplier le; me = 1 where the row is present and elastic
  const double rho_el = fabs(A.qp.elastic);
  double me[3], te[3], le[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    me[j] = rho_el > 0.0 ? m[4 + j] : 0.0;
    // start on the t-stationarity (la + le = rho): from le = 1 the multipliers have to grow
    // three decades through the fraction to the boundary (45 iterations instead of 18 in the
    // dense restatement of this elimination)
    te[j] = 1.0;
    le[j] = me[j] * fmax(rho_el - 1.0, 0.5 * rho_el);
  }
  double mc = 0.0;
#pragma unroll
  for (int i = 0; i < NRW; ++i) mc += m[i];
#pragma unroll
  for (int j = 0; j < 3; ++j) mc += me[j];
  const double mcount = fmax(wsum(mc), 1.0);
  if (stl) {
#pragma unroll
    for (int e = 0; e < NV; ++e) s.v[k][e] = 0.0;
  }
  WSYNC();

  // ---- LQ machinery (stage loops branch-free in their lanes; operands of the next stage
  // loaded before the current stage's dependent chain) -------------------------------
  // Riccati lane roles: T = P F (lanes 0..34, (ta, tj)), H = Qt + F' T (lanes 0..27,
  // (hi, hj), hi <= hj), P' (lanes 0..14), K (lanes 15..24), Huu^-1 (lane 25).
  const int ta = l < 35 ? l / 7 : 0, tj = l < 35 ? l % 7 : 0;
  const int tcol = fcol(tj) < 0 ? 0 : fcol(tj);
  const double tmsk = (l < 35 && fcol(tj) >= 0) ? 1.0 : 0.0, tpa = (l < 35 && tj == 5) ? 1.0 : 0.0;
  int hi = 0, hj = 0;
  {
    int q = l < 28 ? l : 0, i = 0;
    while (q >= NV - i) { q -= NV - i; ++i; }
    hi = i;
    hj = i + q;
  }
  const int hci = fcol(hi) < 0 ? 0 : fcol(hi);
  const double hdyn = (l < 28 && fcol(hi) >= 0) ? 1.0 : 0.0, hpa = (l < 28 && hi == 5) ? 1.0 : 0.0;
  const int hslot = hi == hj ? D0 + hi : ((hi == 4 && hj == 5) ? O45 : 0);
  const double hq = (l < 28 && (hi == hj || (hi == 4 && hj == 5))) ? 1.0 : 0.0;
  int pi = 0, pj = 0;
  {
    int q = l < 15 ? l : 0, i = 0;
    while (q >= NXT - i) { q -= NXT - i; ++i; }
    pi = i;
    pj = i + q;
  }
  struct FacOps {
    double FT[4], FH[4], qv;
  };
  auto fac_load = [&](int kk, FacOps& o) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o.FT[e] = s.F[kk][e][tcol];
      o.FH[e] = s.F[kk][e][hci];
    }
    o.qv = s.Qt[kk][hslot];
  };
  auto fac_stage = [&](int kk, const FacOps& o) -> bool {
    {
      // T[a][j] = sum_e P[a][e] F[e][j] + [j = da] P[a][p]   (column j = p is zero)
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += s.P[ta][e] * o.FT[e];
      if (l < 35) s.T[ta][tj] = tmsk * acc + tpa * s.P[ta][4];
    }
    WSYNC();
    double hv = hq * o.qv + hpa * s.T[4][hj];
#pragma unroll
    for (int e = 0; e < 4; ++e) hv += hdyn * o.FH[e] * s.T[e][hj];
    if (l < 28) {
      s.Hm[hi][hj] = hv;
      s.Hm[hj][hi] = hv;
    }
    WSYNC();
    const double h00 = s.Hm[5][5], h01 = s.Hm[5][6], h11 = s.Hm[6][6];
    const double det = h00 * h11 - h01 * h01;
    // reciprocal bit-identical to IEEE 1/x on every class (asserted: tests/test_gpu_numerics.py): the plain v_rcp_f64 + Newton form turns
    // det = +inf (h00 h11 overflowing at barrier weights ~1e154) into NaN where 1/det = 0
#ifdef VC_KIN_RIC_RAW_RCP  // diagnostic build only (scripts/: the round-2 inverse)
    double id = __builtin_amdgcn_rcp(det);
    id = id * (2.0 - det * id);
    id = id * (2.0 - det * id);
#else
    const double id = rcp_nr(det);
#endif
    const double i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
    {
      const int kc = l >= 15 && l < 25 ? (l - 15) / NXT : 0, ki = l >= 15 && l < 25 ? (l - 15) % NXT : 0;
      const int ci = l < 15 ? pi : ki;
      const double x0 = s.Hm[5][ci], x1 = s.Hm[6][ci], y0 = s.Hm[5][pj], y1 = s.Hm[6][pj];
      const double hpp = s.Hm[pi][pj];
      if (l < 15) {
        const double pv = hpp - (x0 * (i00 * y0 + i01 * y1) + x1 * (i01 * y0 + i11 * y1));
        s.P[pi][pj] = pv;
        s.P[pj][pi] = pv;
      } else if (l < 25) {
        s.K[kk][kc][ki] = kc == 0 ? -(i00 * x0 + i01 * x1) : -(i01 * x0 + i11 * x1);
      } else if (l == 25) {
        s.Hi[kk][0] = i00;
        s.Hi[kk][1] = i01;
        s.Hi[kk][2] = i11;
      }
    }
    WSYNC();
    // det = +inf (h00 h11 overflowing: a diverging barrier) is a failed factorisation: its exact
    // reciprocal 0 would silently drop the input block (Hi = K = 0) from the Newton step
    return h00 > 0.0 && det >= 0x1p-1022 && isfinite(det);  // (and a subnormal det)
  };
  // Riccati factorisation of the stage Hessians s.Qt (backward from P_N = Qt_N on xt)
  auto factor = [&]() -> bool {
    if (l < NXT * NXT) {
      const int a = l / NXT, e = l % NXT;
      s.P[a][e] = a == e ? s.Qt[N][D0 + a] : 0.0;
    }
    WSYNC();
    bool ok = true;
    FacOps A0, B0;
    fac_load(N - 1, A0);
#pragma unroll 1
    for (int kk = N - 1; kk >= 0; kk -= 2) {
      const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
      fac_load(k1, B0);
      ok = fac_stage(kk, A0) && ok;
      if (kk >= 1) {  // uniform
        fac_load(k2, A0);
        ok = fac_stage(kk - 1, B0) && ok;
      }
    }
    return ok;
  };

  // Sweep lanes 0..6 own the stage-vector components v = (y0..y3, p, da, dw).
  const int sl7 = l < NV ? l : NV - 1;
  const int scol = fcol(sl7) < 0 ? 0 : fcol(sl7);
  const double smsk = (l < NV && fcol(sl7) >= 0) ? 1.0 : 0.0;  // p (l = 4) has no dynamics column
  const double spa = (l == 5) ? 1.0 : 0.0;                      // da picks up the p costate
  const int bl5 = l < NXT ? l : 0;
  const bool fu = l == 5 || l == 6;                              // input lanes
  const int fr = l < 4 ? l : 0, fc = l == 6 ? 1 : 0;

  struct BwdOps {
    double F4[4], h, a, b;
  };
  auto bwd_load = [&](int kk, const double (*vec)[NV], BwdOps& o) {
#pragma unroll
    for (int e = 0; e < 4; ++e) o.F4[e] = s.F[kk][e][scol];
    o.h = vec[kk][sl7];
    // lanes 0..4 read K[kk][.][l]; lanes 5, 6 the Huu^-1 pair of their component
    const double* pa = l < NXT ? &s.K[kk][0][bl5] : &s.Hi[kk][l == 5 ? 0 : 1];
    const double* pb = l < NXT ? &s.K[kk][1][bl5] : &s.Hi[kk][l == 5 ? 1 : 2];
    o.a = *pa;
    o.b = *pb;
  };
  // g = vec_k + F_k' p_{k+1} on lanes 0..6
  auto bwd_g = [&](const BwdOps& o, double pv) -> double {
    double pb[NXT];
#pragma unroll
    for (int a = 0; a < NXT; ++a) pb[a] = bcast(pv, a);
    double acc = spa * pb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += o.F4[e] * pb[e];
    return o.h + smsk * acc;
  };
  struct FwdOps {
    double w[6];
  };
  auto fwd_load = [&](int kk, FwdOps& o) {
    const double* src = fu ? &s.K[kk][fc][0] : &s.F[kk][fr][0];
    const double* src5 = fu ? &s.kk[kk][fc] : &s.F[kk][fr][5];
#pragma unroll
    for (int e = 0; e < 5; ++e) o.w[e] = src[e];
    o.w[5] = *src5;
  };
  // one forward stage: writes dv[kk], returns xt_{k+1} (lanes 0..4)
  auto fwd_stage = [&](int kk, const FwdOps& o, double X) -> double {
    double xb[NXT];
#pragma unroll
    for (int a = 0; a < NXT; ++a) xb[a] = bcast(X, a);
    double acc = 0.0;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc += o.w[e] * xb[e];
    const double uk = acc + o.w[4] * xb[4] + o.w[5];  // lanes 5, 6: u_c = K_c xt + kk_c
    const double u0 = bcast(uk, 5), u1 = bcast(uk, 6);
    if (l < NV) s.dv[kk][l] = fu ? uk : X;
    const double xn = acc + o.w[4] * u0 + o.w[5] * u1;  // lanes 0..3
    return l < 4 ? xn : (l == 4 ? u0 : 0.0);
  };

  // LQ solve with linear terms s.h -> direction s.dv (stage N: xt only)
  auto lq_solve = [&]() {
    double pv = l < NXT ? s.h[N][l] : 0.0;  // lanes 0..4: p_N
    BwdOps A1, B1;
    bwd_load(N - 1, s.h, A1);
    auto bstage = [&](int kk, const BwdOps& o) {
      const double g = bwd_g(o, pv);
      const double gu0 = bcast(g, 5), gu1 = bcast(g, 6);
      const double t2 = o.a * gu0 + o.b * gu1;
      pv = g + t2;
      if (fu) s.kk[kk][l - 5] = -t2;
    };
#pragma unroll 1
    for (int kk = N - 1; kk >= 0; kk -= 2) {
      const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
      bwd_load(k1, s.h, B1);
      bstage(kk, A1);
      if (kk >= 1) {
        bwd_load(k2, s.h, A1);
        bstage(kk - 1, B1);
      }
    }
    WSYNC();
    FwdOps A2, B2;
    fwd_load(0, A2);
    double X = 0.0;  // lanes 0..4: xt_k
#pragma unroll 1
    for (int kk = 0; kk < N; kk += 2) {
      const int k1 = kk + 1 < N ? kk + 1 : kk, k2 = kk + 2 < N ? kk + 2 : kk;
      fwd_load(k1, B2);
      X = fwd_stage(kk, A2, X);
      if (kk + 1 < N) {
        fwd_load(k2, A2);
        X = fwd_stage(kk + 1, B2, X);
      }
    }
    if (l < NV) s.dv[N][l] = l < NXT ? X : 0.0;
    WSYNC();
  };

  // condensed dual residual max |d/du (sum_k gr_k . v_k)| through the dynamics (adjoint sweep)
  auto dual_residual = [&]() -> double {
    double rho = l < NXT ? s.gr[N][l] : 0.0, rmax = 0.0;
    BwdOps A3, B3;
    bwd_load(N - 1, s.gr, A3);
    auto rstage = [&](const BwdOps& o) {
      const double g = bwd_g(o, rho);
      rmax = fu ? fmax(rmax, fabs(g)) : rmax;
      rho = g;
    };
#pragma unroll 1
    for (int kk = N - 1; kk >= 0; kk -= 2) {
      const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
      bwd_load(k1, s.gr, B3);
      rstage(A3);
      if (kk >= 1) {
        bwd_load(k2, s.gr, A3);
        rstage(B3);
      }
    }
    return wmax(rmax);
  };

  // ---------------- active-set polish ----------------
  // true when certified; the polished stage vectors are then in s.v.  Elastic rows (el) have a
  // third state besides active / inactive: violated at the penalty, t = sgn v - d > 0 at cost
  // rho t + EPS_T t^2 (a stage-local quadratic in v, no multiplier to find).
  int rounds_used = 0;
  bool pol_fact_fail = false;
  auto polish = [&]() -> bool {
    bool act[NRW], elr[3];
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      // lambda > s (the Tapia-indicator guess of kin_ltv.hip was measured here in round 5: polish rounds
      // mean 1.60 -> 1.05 but max 4 -> 11 at N = 50, B = 1024, and the launch is its slowest problem --
      // the round-4 2.2x slowdown, with unchanged resources: profiles/r05/kr_tapia_ab_r05c.log)
      act[i] = m[i] > 0.0 && la[i] > sl[i];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      elr[j] = me[j] > 0.0 && te[j] > le[j];
      act[4 + j] = act[4 + j] && !elr[j];
    }
#pragma unroll 1
    for (int r = 0; r < A.qp.polish; ++r) {
      ++rounds_used;
      if (stl) {
        double Qt[NQK];
#pragma unroll
        for (int e = 0; e < NQK; ++e) Qt[e] = Qc[e];
#pragma unroll
        for (int i = 0; i < NRW; ++i) Qt[D0 + row_var(i)] += act[i] ? RHO_AL : 0.0;
#pragma unroll
        for (int j = 0; j < 3; ++j) Qt[D0 + row_var(4 + j)] += elr[j] ? 2.0 * EPS_T : 0.0;
#pragma unroll
        for (int e = 0; e < NQK; ++e) s.Qt[k][e] = Qt[e];
      }
      WSYNC();
      if (!factor()) {
        pol_fact_fail = true;
        return false;
      }
      double lm[NRW], cv[NRW];
      bool al_conv = false;
#pragma unroll
      for (int i = 0; i < NRW; ++i) lm[i] = act[i] ? la[i] : 0.0;
#pragma unroll 1
      for (int p = 0; p < AL_PASSES; ++p) {
        // min 1/2 v'Qv + q'v + lm'(C_A v - d_A) + rho/2 |C_A v - d_A|^2 (+ the elastic rows' penalty)
        if (stl) {
          double hk[NV];
#pragma unroll
          for (int e = 0; e < NV; ++e) hk[e] = qc[e];
#pragma unroll
          for (int i = 0; i < NRW; ++i) hk[row_var(i)] += act[i] ? row_sgn(i) * (lm[i] - RHO_AL * d[i]) : 0.0;
#pragma unroll
          for (int j = 0; j < 3; ++j)
            hk[row_var(4 + j)] += elr[j] ? row_sgn(4 + j) * (rho_el - 2.0 * EPS_T * d[4 + j]) : 0.0;
#pragma unroll
          for (int e = 0; e < NV; ++e) s.h[k][e] = hk[e];
        }
        WSYNC();
        lq_solve();
        double dmax = 0.0;
#pragma unroll
        for (int i = 0; i < NRW; ++i) {
          cv[i] = row_sgn(i) * s.dv[k][row_var(i)];
          const double r = act[i] ? cv[i] - d[i] : 0.0;
          lm[i] += RHO_AL * r;
          dmax = fmax(dmax, fabs(r));
        }
        al_conv = wmax(stl ? dmax : 0.0) <= 1e-13 * (1.0 + qmax);
        if (al_conv) break;
      }
      // certificate: inactive rows feasible, multipliers of the active ones >= 0 (and <= rho on
      // elastic rows), elastic rows violated
      bool bad = false;
      bool viol[NRW], neg[NRW], over[3], under[3];
#pragma unroll
      for (int i = 0; i < NRW; ++i) {
        const bool free_row = i < 4 || !elr[i >= 4 ? i - 4 : 0];
        viol[i] = stl && m[i] > 0.0 && !act[i] && free_row && cv[i] - d[i] > TOL_CERT * (1.0 + fabs(d[i]));
        neg[i] = stl && act[i] && lm[i] < -TOL_CERT * (1.0 + qmax);
        bad = bad || viol[i] || neg[i];
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        over[j] = stl && me[j] > 0.0 && act[4 + j] && lm[4 + j] > rho_el + TOL_CERT * (1.0 + qmax);
        under[j] = stl && elr[j] && cv[4 + j] - d[4 + j] < -TOL_CERT * (1.0 + fabs(d[4 + j]));
        bad = bad || over[j] || under[j];
      }
      const bool good = al_conv && __all(bad ? 0 : 1) != 0;
      if (good) {
        if (stl) {
#pragma unroll
          for (int e = 0; e < NV; ++e) s.v[k][e] = s.dv[k][e];
        }
        WSYNC();
        return true;
      }
#pragma unroll
      for (int i = 0; i < NRW; ++i) act[i] = (act[i] || viol[i]) && !neg[i];
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        act[4 + j] = (act[4 + j] || under[j]) && !over[j];
        elr[j] = (elr[j] || over[j]) && !under[j];
      }
    }
    return false;
  };

  // ---------------- interior point (Mehrotra predictor-corrector) ----------------
  // Elastic row i = 4 + j (el): sgn v - t + s = d, t >= 0, cost rho t + EPS_T t^2, multipliers
  // la (row) and le (t >= 0).  The slack t is eliminated stage-locally: with w1 = la / s,
  // w2 = le / t, D = 2 EPS_T + w1 + w2 the row enters the Newton system like a hard row with
  // weight weff = w1 (2 EPS_T + w2) / D and the complementarity term
  //   rco = (rc1 / s) (2 EPS_T + w2) / D - (w1 / D) (rc2 / t + rt),   rt = rho + 2 EPS_T t - la - le,
  // and after the solve  dt = (w1 (C dv + rp) - rc1 / s - rc2 / t - rt) / D,  ds = -rp - C dv + dt,
  // dla = weff (C dv + rp) - rco,  dle = -rc2 / t - w2 dt.
  const double tol_r = A.qp.tol * (1.0 + qmax), tol_mu = 1e-13;
  int it = 0;
  bool conv = false, fail = false, polished = false, tried_polish = false;
  double mu_next_polish = MU_POLISH;
  double last_res = 0.0, last_mu = 0.0;
  // dual residual carried by the steps (KR_RES_RECUR): the LQ direction solves the linearised
  // stationarity exactly, so a step of length alpha scales the condensed gradient by (1 - alpha);
  // the adjoint sweep runs at the first iteration and wherever the carried value would end the loop
  double rd_carry = 0.0;
  bool have_rd = false;
#pragma unroll 1
  for (; finite_pred && it < A.qp.max_iter; ++it) {
    // (a) residuals, stage gradients, barrier-augmented stage Hessians
    double vk[NV], rp[NRW], wg[NRW], grk[NV], rt[3], fE[3], gE[3], ieD[3], w2[3];
    double rpm = 0.0, mus = 0.0;
#pragma unroll
    for (int e = 0; e < NV; ++e) vk[e] = s.v[k][e];
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      rp[i] = m[i] * (row_sgn(i) * vk[row_var(i)] + sl[i] - d[i]) - (i >= 4 ? me[i - 4] * te[i - 4] : 0.0);
      wg[i] = m[i] * la[i] / sl[i];
      rpm = fmax(rpm, fabs(rp[i]));
      mus += m[i] * sl[i] * la[i];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      rt[j] = me[j] * (rho_el + 2.0 * EPS_T * te[j] - la[4 + j] - le[j]);
      rpm = fmax(rpm, fabs(rt[j]));
      mus += me[j] * te[j] * le[j];
      w2[j] = me[j] * le[j] / te[j];
      ieD[j] = me[j] / (2.0 * EPS_T + wg[4 + j] + w2[j]);
      fE[j] = me[j] > 0.0 ? (2.0 * EPS_T + w2[j]) * ieD[j] : 1.0;
      gE[j] = wg[4 + j] * ieD[j];
    }
    double wgE[NRW];  // the rows' weights in the Newton system (effective on elastic rows)
#pragma unroll
    for (int i = 0; i < NRW; ++i) wgE[i] = i < 4 ? wg[i] : wg[i] * fE[i - 4];
    qmul(Qc, vk, grk);
#pragma unroll
    for (int e = 0; e < NV; ++e) grk[e] += qc[e];
#pragma unroll
    for (int i = 0; i < NRW; ++i) grk[row_var(i)] += row_sgn(i) * m[i] * la[i];
    if (stl) {
#pragma unroll
      for (int e = 0; e < NV; ++e) s.gr[k][e] = grk[e];
      double Qt[NQK];
#pragma unroll
      for (int e = 0; e < NQK; ++e) Qt[e] = Qc[e];
#pragma unroll
      for (int i = 0; i < NRW; ++i) Qt[D0 + row_var(i)] += wgE[i];
#pragma unroll
      for (int e = 0; e < NQK; ++e) s.Qt[k][e] = Qt[e];
    } else {
      rpm = 0.0;
      mus = 0.0;
    }
    WSYNC();
    rpm = wmax(rpm);
    const double mu = wsum(mus) / mcount;
    double rdm = (KR_RES_RECUR && have_rd) ? rd_carry : dual_residual();
    last_res = fmax(rdm, rpm);
    last_mu = mu;
    if (!(last_res == last_res) || !(mu == mu) || last_res > 1e300) { fail = true; break; }
    if (KR_RES_RECUR && have_rd && mu <= 1e2 * tol_mu && fmax(rdm, rpm) <= 1e3 * tol_r) {
      // the carried value would end the loop here: take the sweep's
      rdm = dual_residual();
      have_rd = false;
      last_res = fmax(rdm, rpm);
      if (!(last_res == last_res) || last_res > 1e300) { fail = true; break; }
    }
    if (last_res <= tol_r && mu <= tol_mu) { conv = true; break; }
    // polish attempts at mu <= 1e-7 and, if that active set does not certify, at 1e-10
    if (A.qp.polish > 0 && mu <= mu_next_polish) {
      tried_polish = true;
      mu_next_polish *= 1e-3;
      if (polish()) { polished = true; break; }
      if (pol_fact_fail) break;
    }

    // (b) Riccati factorisation of Q + C'WC (the polish may have overwritten s.Qt)
    if (tried_polish && stl) {
      double Qt[NQK];
#pragma unroll
      for (int e = 0; e < NQK; ++e) Qt[e] = Qc[e];
#pragma unroll
      for (int i = 0; i < NRW; ++i) Qt[D0 + row_var(i)] += wgE[i];
#pragma unroll
      for (int e = 0; e < NQK; ++e) s.Qt[k][e] = Qt[e];
    }
    WSYNC();
    if (!factor()) {
      // the barrier-augmented recursion lost definiteness (weights ~1e10 near the end): the
      // polish takes the active set from this iterate if it is close enough
      fail = true;
      if (A.qp.polish > 0 && mu <= 1e2 * MU_POLISH) {
        tried_polish = true;
        polished = polish();
      }
      break;
    }

    // (c) predictor: h = gr + C'(W rp - rco), rco = lam on hard rows (rc = s lam)
    auto set_h = [&](const double* rc_over_s) {
      if (stl) {
        double hk[NV];
#pragma unroll
        for (int e = 0; e < NV; ++e) hk[e] = grk[e];
#pragma unroll
        for (int i = 0; i < NRW; ++i) hk[row_var(i)] += row_sgn(i) * m[i] * (wgE[i] * rp[i] - rc_over_s[i]);
#pragma unroll
        for (int e = 0; e < NV; ++e) s.h[k][e] = hk[e];
      }
      WSYNC();
    };
    double rco[NRW], rc2t[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) rc2t[j] = me[j] * le[j];  // rc2 / t with rc2 = t le
#pragma unroll
    for (int i = 0; i < NRW; ++i) rco[i] = i < 4 ? la[i] : la[i] * fE[i - 4] - gE[i - 4] * (rc2t[i - 4] + rt[i - 4]);
    set_h(rco);
    lq_solve();
    double dsa[NRW], dla[NRW], cdv[NRW], dvk[NV], dta[3], dlea[3];
    double amin = 1.0;
#pragma unroll
    for (int e = 0; e < NV; ++e) dvk[e] = s.dv[k][e];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int i = 4 + j;
      const double c = row_sgn(i) * dvk[row_var(i)];
      dta[j] = ieD[j] * (wg[i] * (c + rp[i]) - la[i] - rc2t[j] - rt[j]);
      dlea[j] = me[j] * (-rc2t[j] - w2[j] * dta[j]);
      if (stl && me[j] > 0.0) amin = fmin(amin, fmin(step_to_bound(te[j], dta[j]), step_to_bound(le[j], dlea[j])));
    }
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      cdv[i] = row_sgn(i) * dvk[row_var(i)];
      dsa[i] = m[i] * (-rp[i] - cdv[i]) + (i >= 4 ? dta[i - 4] : 0.0);
      dla[i] = m[i] * (wgE[i] * (cdv[i] + rp[i]) - rco[i]);
      if (stl && m[i] > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
    }
    amin = wmin(amin);
    double mua = 0.0;
    if (stl) {
#pragma unroll
      for (int i = 0; i < NRW; ++i) mua += m[i] * (sl[i] + amin * dsa[i]) * (la[i] + amin * dla[i]);
#pragma unroll
      for (int j = 0; j < 3; ++j) mua += me[j] * (te[j] + amin * dta[j]) * (le[j] + amin * dlea[j]);
    }
    mua = wsum(mua) / mcount;
    const double ratio = mu > 0.0 ? fmin(1.0, mua / mu) : 0.0;
    const double smu = ratio * ratio * ratio * mu;

    // (d) corrector: rc = s lam + ds_a dl_a - sigma mu (and t le + dt_a dle_a - sigma mu)
    double rcs[NRW];
#pragma unroll
    for (int i = 0; i < NRW; ++i) rcs[i] = m[i] * (sl[i] * la[i] + dsa[i] * dla[i] - smu) / sl[i];
#pragma unroll
    for (int j = 0; j < 3; ++j) rc2t[j] = me[j] * (te[j] * le[j] + dta[j] * dlea[j] - smu) / te[j];
#pragma unroll
    for (int i = 0; i < NRW; ++i) rco[i] = i < 4 ? rcs[i] : rcs[i] * fE[i - 4] - gE[i - 4] * (rc2t[i - 4] + rt[i - 4]);
    set_h(rco);
    lq_solve();
#pragma unroll
    for (int e = 0; e < NV; ++e) dvk[e] = s.dv[k][e];
    amin = 1.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int i = 4 + j;
      const double c = row_sgn(i) * dvk[row_var(i)];
      dta[j] = ieD[j] * (wg[i] * (c + rp[i]) - rcs[i] - rc2t[j] - rt[j]);
      dlea[j] = me[j] * (-rc2t[j] - w2[j] * dta[j]);
      if (stl && me[j] > 0.0) amin = fmin(amin, fmin(step_to_bound(te[j], dta[j]), step_to_bound(le[j], dlea[j])));
    }
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      cdv[i] = row_sgn(i) * dvk[row_var(i)];
      dsa[i] = m[i] * (-rp[i] - cdv[i]) + (i >= 4 ? dta[i - 4] : 0.0);
      dla[i] = m[i] * (wgE[i] * (cdv[i] + rp[i]) - rco[i]);
      if (stl && m[i] > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
    }
    const double alpha = fmin(1.0, 0.99 * wmin(amin));
    rd_carry = (1.0 - alpha) * rdm;
    have_rd = true;
    if (stl) {
#pragma unroll
      for (int i = 0; i < NRW; ++i) {
        if (m[i] > 0.0) {
          sl[i] = fmax(sl[i] + alpha * dsa[i], 1e-300);
          la[i] = fmax(la[i] + alpha * dla[i], 1e-300);
        }
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (me[j] > 0.0) {
          te[j] = fmax(te[j] + alpha * dta[j], 1e-300);
          le[j] = fmax(le[j] + alpha * dlea[j], 1e-300);
        }
      }
#pragma unroll
      for (int e = 0; e < NV; ++e) s.v[k][e] = vk[e] + alpha * dvk[e];
    }
    WSYNC();
  }
  const bool solved = finite_pred && (polished || conv);

  // ---------------- outputs: u* = ubar + du, x* = xbar + dx, u0, status ----------------
  {
    // t: dt_{k+1} = sum_{j <= k} t-row_j . y_j (exclusive scan over the stage lanes)
    double c = 0.0;
    if (l < N) {
#pragma unroll
      for (int a = 0; a < 4; ++a) c += s.tr[l][a] * s.v[l][a];
    }
    double incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double t = __shfl_up(incl, o, 64);
      incl += l >= o ? t : 0.0;
    }
    const double dt = incl - c;  // sum over j < l
    if (stl) {
      const double e0 = ms ? s.ew[k][0] : 0.0, e1 = ms ? s.ew[k][1] : 0.0, e2 = ms ? s.ew[k][2] : 0.0,
                   e3 = ms ? s.ew[k][3] : 0.0, e4 = ms ? s.ew[k][4] : 0.0;
      s.xs[k][0] += s.v[k][0] + e0;
      s.xs[k][1] += s.v[k][1] + e1;
      s.xs[k][3] += s.v[k][2] + e2;
      s.xs[k][4] += s.v[k][3] + e3;
      s.xs[k][5] += dt + e4;
      if (k < N) {
        s.ub[k][0] += s.v[k][5];
        s.ub[k][1] += s.v[k][6];
      }
    }
  }
  WSYNC();
  bool finite = true;
  for (int e = l; e < 2 * N; e += WTH) {
    const double v = s.ub[e >> 1][e & 1];
    finite = finite && isfinite(v);
    A.u_out[(size_t)b * 2 * N + e] = v;
  }
  for (int e = l; e < 6 * (N + 1); e += WTH) {
    const double v = s.xs[e / 6][e % 6];
    finite = finite && isfinite(v);
    A.x_out[(size_t)b * 6 * (N + 1) + e] = v;
  }
  finite = __all(finite ? 1 : 0) != 0;
  if (l < 2) A.u0[(size_t)b * 2 + l] = s.ub[0][l];
  if (l == 0) {
    constexpr size_t DS = VC_DIAG_COLS;  // the ABI's row stride (no section counters here)
    int32_t st;
    if (!finite || !finite_pred) st = VC_NONFINITE;
    else if (solved) st = VC_SOLVED;
    else st = VC_MAX_ITER;
    A.status[b] = st;
    // the elastic-on-failure pass adds its iterations to the hard-row pass's (read before overwriting)
    A.iters[b] = it + (A.qp.elastic < 0.0 ? A.iters[b] : 0);
    if (A.diag) {
      A.diag[(size_t)b * DS + 0] = last_res;
      A.diag[(size_t)b * DS + 1] = last_mu;
      A.diag[(size_t)b * DS + 2] =
          double((fail ? 1 : 0) | (conv ? 2 : 0) | (polished ? 4 : 0) | (pol_fact_fail ? 8 : 0));
      A.diag[(size_t)b * DS + 3] = double(rounds_used);
    }
  }
}

}  // namespace

// ---- host launcher ---------------------------------------------------------------
#define VC_KR_HORIZONS(X) X(10) X(20) X(30) X(40) X(50) X(60)

bool kin_ric_built(int N) {
  switch (N) {
#define VC_CASE(n) case n:
    VC_KR_HORIZONS(VC_CASE)
#undef VC_CASE
    return true;
    default:
      return false;
  }
}

hipError_t launch_kin_ric(const KinLtvArgs& a, int N, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  switch (N) {
#define VC_CASE(n)                                                                 \
  case n:                                                                          \
    hipLaunchKernelGGL((kin_ric_kernel<n>), dim3(a.B), dim3(WTH), 0, stream, a);  \
    return hipGetLastError();
    VC_KR_HORIZONS(VC_CASE)
#undef VC_CASE
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vc
