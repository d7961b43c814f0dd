// casc_ric.hip -- fused cascaded (single-track + point-mass) SQP step, fp64, one wavefront
// per problem, with a stagewise Riccati interior point: any tail length M with
// H = N + M <= 64 stages.
//
// Replaces the IPOPT solve of CascadedMPC with horizon_pm > 0 (controllers/mpc/
// cascaded_mpc.py:17-39,91-304; config/controllers/cascaded.yaml N = 20 + M = 40, and the
// recorded runs' M = 15 / 25 / 35, experiments/data/*/cascaded_config.yaml).  Contract:
// oracle/casc_sqp.py, the same QPs the condensed kernel casc_sqp.hip solves.  The QP is
// restated stage by stage (the single-track part exactly as st_sqp.hip):
//   stage vector v_k (9) = (y_k, p_k, u_k), QP state xt_k = (y_k, p_k), p_k = dFx_{k-1} (the Fx
//   slews and the switching Fx term couple neighbouring inputs)
//     single-track k < N:  y = (dUx, dUy, dr, ddelta, dey, depsi), u = (dFx / S, dw)
//     point mass  k >= N:  y = (dV, dey, depsi, c, 0, 0),           u = (dFx / S, dFy / S)
//   where c = dFy_{k-1} / S for k > N (the Fy slew) and, at the first point-mass stage k = N,
//   the linearised change of the lateral tyre forces Fy_f + Fy_r of stage N-1 (the switching
//   cost's lateral residual, cascaded_mpc.py:241-255) -- so every cost term is stage-local.
//   Transitions xt_{k+1} = [A6 | 0 | B6; 0 | 0 | e_Fx] v_k: single-track RK4 Jacobians; the
//   switching map (cascaded_mpc.py:256-277) at k = N-1 (V, ey, epsi from (Ux, Uy, ey, epsi),
//   c from the lateral-force gradient); point-mass Euler Jacobians (dynamic_point_mass.py:
//   76-100) for k >= N.  s is fixed (s' = 1 in both models); t enters only the terminal
//   w_time t_{H-1}, a linear stage term through each step's t-row (the switch copies t).
//   Stage Hessians share one 21-slot pattern; the 12 one-sided rows of a stage touch
//   (y0..y3, dFx, u1) only (point mass: V >= V_min, Fx <= Peng / V, the trust region).
// Per SQP iteration: predict (lane 0: RK4, switch, Euler), linearize (one lane per (stage,
// seed pair), dual numbers), then the Mehrotra predictor-corrector whose Newton steps are LQ
// problems solved by a backward Riccati recursion over the H stages (O(H) per iteration;
// the condensed kernel pays O(H^3)) and a forward rollout; lane k owns stage k's rows,
// slacks and multipliers in registers.
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "vc_dual.hpp"
#include "vc_kernels.hpp"

namespace vc {
namespace {

constexpr int WTH = 64;
constexpr int NQ = 21;  // nonzeros of a stage Hessian over v = (y0..y5, p, u0, u1)
constexpr int NR = 12;  // one-sided rows per stage
enum { Q00, Q01, Q02, Q03, Q07, Q11, Q12, Q13, Q17, Q22, Q23, Q27, Q33, Q37, Q77, Q44, Q55, Q66, Q67, Q88, Q38 };

__host__ __device__ constexpr int qslot(int i, int j) {
  if (i > j) { const int t = i; i = j; j = t; }
  const int a = i == 7 ? 4 : (i < 4 ? i : -1), b = j == 7 ? 4 : (j < 4 ? j : -1);
  if (a >= 0 && b >= 0) {
    constexpr int blk[5][5] = {{Q00, Q01, Q02, Q03, Q07}, {Q01, Q11, Q12, Q13, Q17}, {Q02, Q12, Q22, Q23, Q27},
                               {Q03, Q13, Q23, Q33, Q37}, {Q07, Q17, Q27, Q37, Q77}};
    return blk[a][b];
  }
  if (i == 4 && j == 4) return Q44;
  if (i == 5 && j == 5) return Q55;
  if (i == 6 && j == 6) return Q66;
  if (i == 6 && j == 7) return Q67;
  if (i == 8 && j == 8) return Q88;
  if (i == 3 && j == 8) return Q38;
  return -1;
}
// Swizzled lane-per-stage arrays (round 4): lane k reads row k of trow[.][8] and st[.][42] at a
// fixed column, and those even strides put lanes k and k + 4 (trow: 8-way over a 32-lane
// ds_read_b64 group) or k and k + 16 (st: 2-way) on the same banks.  Instead of padding (no LDS to
// spare at N = 60) each row is permuted: trow column a of row k sits in slot (a + k / 4) mod 8,
// st element e = 6 r + j of row k in slot e ^ (k / 16 mod 2) -- every lane of a group then reads
// a distinct bank pair, and the layout stays a permutation within each row.
__device__ __forceinline__ int tsw(int k, int a) { return (a + (k >> 2)) & 7; }
__device__ __forceinline__ int stx(int k, int r, int j) { return (6 * r + j) ^ ((k >> 4) & 1); }
// stage vector index -> column of [A6 | B6] (-1 for p: no dynamics enters through it)
__host__ __device__ constexpr int vcol(int i) { return i < 6 ? i : (i == 6 ? -1 : i - 1); }

// Strides (round 4): a lane-per-stage phase reads row k of xs / ub / J in lane k; an even stride
// of 8 doubles put lanes k and k + 4 on the same banks (ds_read_b64: bank (a/4) mod 64 over 32
// lanes -> 8-way on xs, 16-way on J's 48-double stages, 2-way on ub).  J, the array every
// Riccati sweep reads, gets the odd stride 49: the 32 lanes of a ds_read_b64 group then hit 32
// distinct bank pairs and the 16 of a ds_write_b64 / ds_read2_b64 group 16 ((a/4) mod 32).  xs
// and ub keep 8 / 2, and the model coefficients are read from the kernel arguments instead of
// LDS: with odd xs / ub strides too the M = 40 block reached 54,312 B, which rocprofv3 allocates
// as 54,272 B -- two workgroups per CU instead of three (cascaded 201 K -> 143 K solves/s,
// r04c/d); three need <= 53,248 B.
struct CrJ {  // [A6 | B6 diag(S, 1 or S)] of one transition + 1 pad (49 doubles)
  double m[6][8];
  double pad;
  __device__ __forceinline__ double* operator[](int r) { return m[r]; }
  __device__ __forceinline__ const double* operator[](int r) const { return m[r]; }
};
// Round 5: where the LDS copy of J (49 doubles per stage) would cost a workgroup per CU (M = 35 / 40:
// 48.7 / 53.1 KB, three per CU) it lives in a per-problem global workspace (CascSqpArgs.jws, 384 B
// per stage; written once per SQP iteration, read by the Riccati passes one stage ahead of use):
// 29.6 / 31.7 KB, four per CU -- the ceiling, the kernel holds ~480 VGPRs + AGPRs (one wave per SIMD)
template <int N, int M>
constexpr bool cr_j_global_ok() { return N + M >= 55; }  // (cr_jg_pick)
template <bool JG>
using CrJP = std::conditional_t<JG, double*, CrJ*>;  // workspace base (GBuf) or LDS
struct CrNone {};  // (global: 48 doubles = 384 B per stage, [6][8] row-major)

template <int N, int M, bool JG>
struct CrSmem {
  static constexpr int H = N + M;
  StageRows8<H> xs;   // prediction: single-track states k < N, point-mass (V, s, ey, epsi, t) k >= N (rotated rows)
  double ub[H][2];    // current ubar (stride 2: the odd stride 3 cost M = 40 its third workgroup per CU)
  double kap[H], dsv[H];
  // J[k][row][col]: [A6 | B6 diag(S, 1 or S)] of the transition out of stage k (LDS unless JG)
  std::conditional_t<JG, CrNone, CrJ[H]> J;
  union {
    struct {
      double Qt[H][NQ];  // stage Hessian + barrier, this iteration
      // stage vector, three lives per interior-point iteration: the gradient Q v + q + C' lam
      // (residuals -> dual residual sweep), the LQ right-hand side h (set_h -> backward pass),
      // the direction dv (forward pass -> step); after the QP: the pre-step iterate uo in
      // [0..1] and the step dz in [2..3] (SQP update -> domain cut-back).  The QP iterate v
      // itself lives in its lane's registers.  During the Riccati factorisation (between the
      // dual residual sweep and set_h: g dead) the same space holds the factorisation's
      // scratch f: cost-to-go P, T = P [A B], stage Hessian Hm.  (At M = 40 the block drops from
      // 68 KB to 52 KB: three one-wave workgroups per CU instead of two.)
      union {
        double g[H][9];
        struct {
          double P[7][7];
          double T[7][8];
          double Hm[9][9];
        } f;
      };
      double K[H][2][7];
      double Hi[H][3];   // Huu^-1 (00, 01, 11)
      double kk[H][2];
    } q;
    struct {
      double trow[H][8];     // t-row of the transition out of stage k over (y | u)
      double st[N][42];    // single-track stage functions: value + gradient over (Ux, Uy, r, delta, Fx)
      double gfy[6];         // Fy_f + Fy_r at stage N-1: value + gradient over (Ux, Uy, r, delta, Fx)
    } l;
  } u;
  // weights and QP options: each phase loads its own register copy from here (held in registers
  // across the SQP loop they were spilled to scratch); the model coefficients are re-read from
  // the kernel arguments (kargs), which keeps the M = 40 block at three workgroups per CU
  vc_dyn_mpc w;
  vc_casc_mpc cw;
  vc_qp qp;
  int flag[4];
};


constexpr int kCrPolish = 3;  // active-set polish rounds after each converged QP (0: off, the round-4 kernel)
constexpr double kCrAlRho = 1e2;  // polish: augmented-Lagrangian weight of an active row, x (1 + max diag Q) / |c|^2
constexpr int kCrAlPasses = 16;
constexpr double kCrCertPtol = 1e-11;  // polish certificate: inactive-row violation, x (1 + max |q|)
constexpr double kCrCertDtol = 1e-12;  // polish certificate: wrong-signed multiplier, x (1 + max |q|)


#define WSYNC()                          \
  do {                                   \
    asm volatile("" ::: "memory");       \
    __builtin_amdgcn_wave_barrier();     \
    asm volatile("" ::: "memory");       \
  } while (0)

// the kernel-argument block through an opaque scalar pointer: every read is a fresh scalar load
// at its point of use (K$ hit), so nothing derived from it is held -- spilled -- across a phase
template <typename T>
__device__ __forceinline__ const T* kargs() {
  const T* p = (const T*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
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

// Stage k's one-sided rows C v <= d (lane-owned):
//   0: -y0 <= ..   (Ux >= Ux_min, point mass V >= V_min)
//   1: y3 <= ..   2: -y3 <= ..   (delta bounds, single track)
//   3..7: c_r . (y0, y1, y2, y3, u0) <= d_r   (power limit, tyre force bounds; point mass: Peng / V)
//   8: u1 <= ..   9: -u1 <= ..   (w box, point mass: the Fy trust region)   10, 11: |u0| trust
struct Rows {
  double c[5][5];
  double d[NR];
  uint32_t mb;  // bit i: row i is present (a 1.0 / 0.0 mask as 12 doubles would hold 24 VGPRs)
  __device__ __forceinline__ double m(int i) const { return ((mb >> i) & 1u) ? 1.0 : 0.0; }
  __device__ __forceinline__ void set(int i, bool on) { mb = on ? (mb | (1u << i)) : (mb & ~(1u << i)); }
};

__device__ __forceinline__ void row_values(const Rows& R, const double* v, double* o) {
  o[0] = -v[0];
  o[1] = v[3];
  o[2] = -v[3];
#pragma unroll
  for (int r = 0; r < 5; ++r)
    o[3 + r] = R.c[r][0] * v[0] + R.c[r][1] * v[1] + R.c[r][2] * v[2] + R.c[r][3] * v[3] + R.c[r][4] * v[7];
  o[8] = v[8];
  o[9] = -v[8];
  o[10] = v[7];
  o[11] = -v[7];
}
// out += C' y
__device__ __forceinline__ void row_adjoint(const Rows& R, const double* y, double* out) {
  out[0] -= y[0];
  out[3] += y[1] - y[2];
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    out[0] += R.c[r][0] * y[3 + r];
    out[1] += R.c[r][1] * y[3 + r];
    out[2] += R.c[r][2] * y[3 + r];
    out[3] += R.c[r][3] * y[3 + r];
    out[7] += R.c[r][4] * y[3 + r];
  }
  out[8] += y[8] - y[9];
  out[7] += y[10] - y[11];
}
// out = Q v (symmetric, 21 slots)
__device__ __forceinline__ void qmul(const double* Q, const double* v, double* o) {
  o[0] = Q[Q00] * v[0] + Q[Q01] * v[1] + Q[Q02] * v[2] + Q[Q03] * v[3] + Q[Q07] * v[7];
  o[1] = Q[Q01] * v[0] + Q[Q11] * v[1] + Q[Q12] * v[2] + Q[Q13] * v[3] + Q[Q17] * v[7];
  o[2] = Q[Q02] * v[0] + Q[Q12] * v[1] + Q[Q22] * v[2] + Q[Q23] * v[3] + Q[Q27] * v[7];
  o[3] = Q[Q03] * v[0] + Q[Q13] * v[1] + Q[Q23] * v[2] + Q[Q33] * v[3] + Q[Q37] * v[7] + Q[Q38] * v[8];
  o[4] = Q[Q44] * v[4];
  o[5] = Q[Q55] * v[5];
  o[6] = Q[Q66] * v[6] + Q[Q67] * v[7];
  o[7] = Q[Q07] * v[0] + Q[Q17] * v[1] + Q[Q27] * v[2] + Q[Q37] * v[3] + Q[Q67] * v[6] + Q[Q77] * v[7];
  o[8] = Q[Q88] * v[8] + Q[Q38] * v[3];
}

// stage-Jacobian element (k, r, c): the LDS array, or the global workspace through a buffer
// resource (GBuf: one offset VGPR per access, bounds-checked to the problem's (N + M) stages)
template <int N, int M, bool JG>
__device__ __forceinline__ double cr_jld(CrJP<JG> J, int k, int r, int c) {
  if constexpr (JG) return GBuf(J, (N + M) * 384).ld((uint32_t)(((k * 6 + r) * 8 + c) * 8));
  else return J[k].m[r][c];
}
template <int N, int M, bool JG>
__device__ __forceinline__ void cr_jst(CrJP<JG> J, int k, int r, int c, double v) {
  if constexpr (JG) GBuf(J, (N + M) * 384).st((uint32_t)(((k * 6 + r) * 8 + c) * 8), v);
  else J[k].m[r][c] = v;
}
// columns c, c + 1 (c even) of one row: global J as one 16-byte store (GBuf::st2)
template <int N, int M, bool JG>
__device__ __forceinline__ void cr_jst2(CrJP<JG> J, int k, int r, int c, double v0, double v1) {
  if constexpr (JG) GBuf(J, (N + M) * 384).st2((uint32_t)(((k * 6 + r) * 8 + c) * 8), v0, v1);
  else {
    J[k].m[r][c] = v0;
    J[k].m[r][c + 1] = v1;
  }
}
#define JLD(k, r, c) cr_jld<N, M, JG>(J, (k), (r), (c))
#define JST(k, r, c, v) cr_jst<N, M, JG>(J, (k), (r), (c), (v))
#define JST2(k, r, c, v0, v1) cr_jst2<N, M, JG>(J, (k), (r), (c), (v0), (v1))

// global J: the linearisation's stores visible to every lane of the wave before they are read
template <bool JG>
__device__ __forceinline__ void cr_jfence() {
  if constexpr (JG) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}
template <int N, int M, bool JG>
__device__ __forceinline__ CrJP<JG> cr_jac(CrSmem<N, M, JG>& s, int b) {
  if constexpr (JG) return GBuf::uniform(kargs<CascSqpArgs>()->jws + (size_t)b * (N + M) * 48);
  else return s.J;
}

template <int N, int M, int TYRE, bool JG>
__global__ __launch_bounds__(WTH) void casc_ric_kernel(CascSqpArgs A) {
  constexpr int H = N + M;
  static_assert(N >= 2 && M >= 2 && H <= WTH, "one lane per stage");
  // occupancy guard (rocprofv3 LDS_Block_Size: 53,248 B ran three one-wave workgroups per CU --
  // r03, 201 K solves/s at M = 40 --, 54,272 B two -- r04c/d, 143-147 K);
  // four (one per SIMD: the register file allows no more) need <= 40,960 B
  static_assert(!JG || sizeof(CrSmem<N, M, JG>) <= 40960, "global-J casc_ric must fit four workgroups per CU");
  static_assert(JG || M != 40 || sizeof(CrSmem<N, M, JG>) <= 53248, "LDS-J casc_ric<20, 40> must fit three per CU");
  __shared__ CrSmem<N, M, JG> s;
  const int l = threadIdx.x;
  const int b = xcd_problem(blockIdx.x, A.B);
  const double S = A.w.fx_scale;
  const bool stl = l < H;
  const int k = stl ? l : 0;  // this lane's stage
  const bool pm = k >= N;     // point-mass stage

  for (int i = l; i < H; i += WTH) {
    s.kap[i] = A.kappa[(size_t)b * H + i];
    s.dsv[i] = A.ds[(size_t)b * H + i];
    s.ub[i][0] = A.ubar[((size_t)b * H + i) * 2];
    s.ub[i][1] = A.ubar[((size_t)b * H + i) * 2 + 1];
  }
  if (l < 8) s.xs.at(0, l) = A.x0[(size_t)b * 8 + l];
  if (l >= N && l < H) {  // point-mass slots 5..7 are reported as 0 (free in the reference's NLP)
    s.xs.at(l, 5) = s.xs.at(l, 6) = s.xs.at(l, 7) = 0.0;
  }
  if (l == 0) {
    s.flag[0] = VC_SOLVED;
    s.w = A.w;
    s.cw = A.cw;
    s.qp = A.qp;
  }
  WSYNC();

  int it_total = 0, it_max = 0;
  bool all_conv = true, any_fail = false, stopped = false;  // stopped: a later QP ended the SQP early
  bool all_pol = true;  // every converged QP's answer certified by the active-set polish
  double last_res = 0.0, last_mu = 0.0;
  const double tol_r = 1e-10, tol_mu = 1e-13;

  // SQP update state: a step under test (tries > 0) is ub = uo + 2^-(tries-1) du (uo, du in
  // u.q.g[k][0..3], untouched by the rollout), the last try the unchanged iterate
  // (oracle/casc_sqp.py, oracle/dyn_sqp.py domain_step)
  int tries = 0, sq = 0;
  bool first = true, test = false;  // test: the iterate's own rollout is inside the domain
  const int l_out = l, k_out = k;
  for (;;) {
    // lane coordinates re-laundered every SQP iteration: lane masks derived from them are
    // recomputed inside the loop instead of being hoisted out of it and spilled
    int l = l_out, k = k_out;
    asm volatile("" : "+v"(l), "+v"(k));
    const CrJP<JG> J = cr_jac<N, M, JG>(s, b);
    const bool stl = l < H;
    const bool pm = k >= N;
    // ---------------- predict (lane 0: RK4, switch, point-mass Euler) ----------------
    // the only rollout site; flag[2]: finite and inside both models' domain (casc_in_domain)
    if (l == 0) {
      DynCoef<double> c = kargs<CascSqpArgs>()->car;
      c.tyre = TYRE;
      double x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = s.xs.at(0, i);
      bool fin = true, dom = dyn_in_domain(x, s.kap[0]);
      for (int kk = 0; kk < N - 1; ++kk) {
        const double u2[2] = {s.ub[kk][0], s.ub[kk][1]};
        const double kp = s.kap[kk];
        double xn[8];
        const double th = dyn_fx_split(u2[0]);  // one tanh per step, not per evaluation
        rk4_apply<double, 8>(x, s.dsv[kk], [&](const double* xx, double* f) { dyn_spatial_ode_alg_th<double, double>(xx, u2, th, kp, c, f); }, xn);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          x[i] = xn[i];
          s.xs.at(kk + 1, i) = xn[i];
          fin = fin && isfinite(xn[i]);
        }
        dom = dom && dyn_in_domain(x, s.kap[kk + 1]);
      }
      double p[5];
      st_to_pm<double>(x, p);  // cascaded_mpc.py:256-277
#pragma unroll
      for (int i = 0; i < 5; ++i) s.xs.at(N, i) = p[i];
      dom = dom && pm_in_domain(p, s.kap[N]);
      for (int j = N; j < H - 1; ++j) {  // dynamic_point_mass.py:76-100, Euler
        const double u2[2] = {s.ub[j][0], s.ub[j][1]};
        double f[5];
        pm_spatial_ode<double, double>(p, u2, s.kap[j], c, f);
        const double h = s.dsv[j];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          p[i] = p[i] + h * f[i];
          s.xs.at(j + 1, i) = p[i];
          fin = fin && isfinite(p[i]);
        }
        dom = dom && pm_in_domain(p, s.kap[j + 1]);
      }
      s.flag[2] = (fin && dom) ? 1 : 0;
      if (first && !fin) s.flag[0] = VC_NONFINITE;
    }
    WSYNC();
    first = false;
    if (tries > 0) {
      // ---------------- SQP update: cut the step back while its rollout leaves the domain ----------------
      if (test && s.flag[2] == 0 && tries <= DOM_HALVINGS) {
        const double a = tries < DOM_HALVINGS ? ldexp(1.0, -tries) : 0.0;
        if (stl) {
          const double u0v = s.u.q.g[k][0], u1v = s.u.q.g[k][1];  // uo
          const double d0 = s.u.q.g[k][2], d1 = s.u.q.g[k][3];
          s.ub[k][0] = a > 0.0 ? u0v + a * (d0 * S) : u0v;
          if (pm) s.ub[k][1] = a > 0.0 ? u1v + a * (d1 * S) : u1v;
          else s.ub[k][1] = a > 0.0 ? fmin(fmax(u1v + a * d1, s.w.w_min), s.w.w_max) : u1v;
        }
        ++tries;
        WSYNC();
        continue;
      }
      tries = 0;
      ++sq;
    }
    if (sq == s.w.sqp_iters || s.flag[0] == VC_NONFINITE) break;

    // ---------------- linearize + stage functions ----------------
    {
      DynCoef<double> c = kargs<CascSqpArgs>()->car;
      c.tyre = TYRE;
      constexpr int NLIN = 8 * (N - 1), NSTF = 5 * N, NPM = 3 * (M - 1);
      using D2 = Dual<2, double>;
      using D1 = Dual<1, double>;
      // three task loops (one kind of work per loop: no divergent mix of the dual-number
      // evaluations in one iteration)
#pragma unroll 1
      for (int task = l; task < NLIN; task += WTH) {
        {  // single-track RK4 step k -> k + 1 (k < N - 1): one column of [A6 | B6] per task
          // (one dual seed: half the registers of a seed pair, which made the Fiala build spill)
          const int kk = task >> 3, col = task & 7;
          // column -> seeded variable: (Ux, Uy, r, delta, ey, epsi | Fx, w)
          const int a0 = col < 4 ? col : (col < 6 ? col + 1 : -1);
          D1 x[8], u2[2], xn[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            x[i] = D1(s.xs.at(kk, i));
            x[i].d[0] = i == a0 ? 1.0 : 0.0;
          }
          u2[0] = D1(s.ub[kk][0]);
          u2[1] = D1(s.ub[kk][1]);
          u2[0].d[0] = col == 6 ? 1.0 : 0.0;
          u2[1].d[0] = col == 7 ? 1.0 : 0.0;
          const D1 kp(s.kap[kk]);
          const D1 th = dyn_fx_split(u2[0]);
          rk4_apply<D1, 8>(x, D1(s.dsv[kk]), [&](const D1* xx, D1* f) { dyn_spatial_ode_alg_th<D1, double>(xx, u2, th, kp, c, f); }, xn);
          const double s0 = col == 6 ? S : 1.0;
          const int yr[6] = {0, 1, 2, 3, 5, 6};
#pragma unroll
          for (int r = 0; r < 6; ++r) JST(kk, r, col, xn[yr[r]].d[0] * s0);
          s.u.l.trow[kk][tsw(kk, col)] = xn[7].d[0] * s0;
        }
      }
#pragma unroll 1
      for (int task = l; task < NSTF; task += WTH) {
        {  // single-track stage functions (cascaded_mpc.py:110-128,155-165)
          const int q = task, kk = q / 5, j = q % 5;
          D1 X5[5], o[7];
#pragma unroll
          for (int i = 0; i < 4; ++i) X5[i] = D1(s.xs.at(kk, i));
          X5[4] = D1(s.ub[kk][0]);
#pragma unroll
          for (int i = 0; i < 5; ++i) X5[i].d[0] = i == j ? 1.0 : 0.0;
          dyn_stage_terms_alg<D1, double>(X5, c, o);
#pragma unroll
          for (int r = 0; r < 7; ++r) {
            s.u.l.st[kk][stx(kk, r, 1 + j)] = o[r].d[0];
            if (j == 0) s.u.l.st[kk][stx(kk, r, 0)] = o[r].v;
          }
        }
      }
#pragma unroll 1
      for (int task = l; task < NPM; task += WTH) {
        {  // point-mass Euler step j -> j + 1: seed pairs (V, ey), (epsi, -), (Fx, Fy)
          const int q = task, j = N + q / 3, pr = q % 3;
          D2 x[5], u2[2], f[5];
          const int a0 = pr == 0 ? 0 : (pr == 1 ? 3 : -1), a1 = pr == 0 ? 2 : -1;
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            x[i] = D2(s.xs.at(j, i));
            x[i].d[0] = i == a0 ? 1.0 : 0.0;
            x[i].d[1] = i == a1 ? 1.0 : 0.0;
          }
          u2[0] = D2(s.ub[j][0]);
          u2[1] = D2(s.ub[j][1]);
          u2[0].d[0] = pr == 2 ? 1.0 : 0.0;
          u2[1].d[1] = pr == 2 ? 1.0 : 0.0;
          pm_spatial_ode<D2, double>(x, u2, D2(s.kap[j]), c, f);
          const double h = s.dsv[j];
          // rows (V, ey, epsi) of I + h df/dx at y slots (0, 1, 2); inputs scaled by S; the
          // Fy slew's c row (3) = e_u1; t-row over (V, ey, epsi).  Each task owns one column pair
          // of rows 0..2 -- (0, 1), (2, 3) with column 3 zero, (6, 7) -- stored by one 16-byte store
          // per row after the seed branches (the three tasks of a stage are adjacent lanes: one
          // store instruction per row); the constant entries (columns 4, 5 of rows 0..2, rows 3..5)
          // are written by the first linearisation of the launch only
          const int yi[3] = {0, 2, 3};
          double cv0[3], cv1[3];
          if (pr == 0) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              cv0[r] = (r == 0 ? 1.0 : 0.0) + h * f[yi[r]].d[0];
              cv1[r] = (r == 1 ? 1.0 : 0.0) + h * f[yi[r]].d[1];
            }
            s.u.l.trow[j][tsw(j, 0)] = h * f[4].d[0];
            s.u.l.trow[j][tsw(j, 1)] = h * f[4].d[1];
          } else if (pr == 1) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              cv0[r] = (r == 2 ? 1.0 : 0.0) + h * f[yi[r]].d[0];
              cv1[r] = 0.0;
            }
            s.u.l.trow[j][tsw(j, 2)] = h * f[4].d[0];
#pragma unroll
            for (int cc = 3; cc < 6; ++cc) s.u.l.trow[j][tsw(j, cc)] = 0.0;
            if (sq == 0) {
#pragma unroll
              for (int r = 0; r < 3; ++r) JST2(j, r, 4, 0.0, 0.0);
#pragma unroll
              for (int r = 3; r < 6; ++r)
#pragma unroll
                for (int cc = 0; cc < 8; cc += 2) JST2(j, r, cc, 0.0, (r == 3 && cc == 6) ? 1.0 : 0.0);
            }
          } else {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              cv0[r] = h * f[yi[r]].d[0] * S;
              cv1[r] = h * f[yi[r]].d[1] * S;
            }
            s.u.l.trow[j][tsw(j, 6)] = h * f[4].d[0] * S;
            s.u.l.trow[j][tsw(j, 7)] = h * f[4].d[1] * S;
          }
          const int cp = pr == 0 ? 0 : (pr == 1 ? 2 : 6);
#pragma unroll
          for (int r = 0; r < 3; ++r) JST2(j, r, cp, cv0[r], cv1[r]);
        }
      }
    }
    WSYNC();
    // the switching map out of stage N - 1 (cascaded_mpc.py:241-277): lanes 0..4 the lateral
    // tyre forces Fy_f + Fy_r and their gradient (one dual seed each), lane 5 the Jacobian rows
    // (V, ey, epsi); t passes through unchanged
    if (l < 5) {
      using D1 = Dual<1, double>;
      DynCoef<double> c = kargs<CascSqpArgs>()->car;
      c.tyre = TYRE;
      D1 X5[5];
#pragma unroll
      for (int i = 0; i < 4; ++i) X5[i] = D1(s.xs.at(N - 1, i));
      X5[4] = D1(s.ub[N - 1][0]);
#pragma unroll
      for (int i = 0; i < 5; ++i) X5[i].d[0] = i == l ? 1.0 : 0.0;
      const D1 fy = dyn_lateral_sum<D1, double>(X5, c);
      s.u.l.gfy[1 + l] = fy.d[0];
      if (l == 0) s.u.l.gfy[0] = fy.v;
    } else if (l == 5) {
      const double Ux = s.xs.at(N - 1, 0), Uy = s.xs.at(N - 1, 1);
      const double q2 = Ux * Ux + Uy * Uy, V = sqrt(q2);
      // every element stored once (row 3's entries 0..3 and 6 by lanes 0..4 below)
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          if (r == 3 && (cc < 4 || cc == 6)) continue;
          double v = 0.0;
          if (r == 0 && cc == 0) v = Ux / V;
          if (r == 0 && cc == 1) v = Uy / V;
          if (r == 1 && cc == 4) v = 1.0;
          if (r == 2 && cc == 0) v = -Uy / q2;
          if (r == 2 && cc == 1) v = Ux / q2;
          if (r == 2 && cc == 5) v = 1.0;
          JST(N - 1, r, cc, v);
        }
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) s.u.l.trow[N - 1][tsw(N - 1, cc)] = 0.0;
    }
    WSYNC();
    // the switch's c row: the lateral-force gradient over (Ux, Uy, r, delta | dFx / S)
    if (l < 4) JST(N - 1, 3, l, s.u.l.gfy[1 + l]);
    if (l == 4) JST(N - 1, 3, 6, s.u.l.gfy[5] * S);
    cr_jfence<JG>();
    WSYNC();

    // ---------------- stage QP data (lane k, registers) ----------------
    double Qc[NQ], qc[9];
    Rows R;
    R.mb = 0u;
#pragma unroll
    for (int e = 0; e < NQ; ++e) Qc[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) qc[e] = 0.0;
    {
      const vc_dyn_mpc W = s.w;
      const vc_casc_mpc CW = s.cw;
      const vc_qp QP = s.qp;
      const double Peng = kargs<CascSqpArgs>()->car.Peng;
      const double ds = s.dsv[k];
      // ey / s slots of this stage's state
      const double ey = pm ? s.xs.at(k, 2) : s.xs.at(k, 5), sa = pm ? s.xs.at(k, 1) : s.xs.at(k, 4);
      const double wdev = pm ? CW.w_dev_pm : W.w_dev, eylo = pm ? CW.ey_min_pm : W.ey_min,
                   eyhi = pm ? CW.ey_max_pm : W.ey_max;
      // boundary + deviation (cascaded_mpc.py:139-151, point mass :204-219), obstacles (:173-176)
      const double cdev = wdev * ds;
      const double blo = ey < eylo ? W.w_b * ds : 0.0, bhi = ey > eyhi ? W.w_b * ds : 0.0;
      const double cey = 2.0 * (cdev + blo + bhi), qey = 2.0 * (cdev * ey + blo * (ey - eylo) + bhi * (ey - eyhi));
      double po = 0.0, qo = 0.0;
      if (A.obs.n > 0) obstacle_ey_model<double>(A.obs, sa, ey, W.w_obs * ds, po, qo);
      if (pm) {
        Qc[Q11] += cey + qo;
        qc[1] += qey + po;
      } else {
        Qc[Q44] += cey + qo;
        qc[4] += qey + po;
      }
      // prox on the scaled step, w^2 on the single track (:153)
      Qc[Q77] += 2.0 * QP.prox;
      Qc[Q88] += 2.0 * QP.prox;
      if (!pm) {
        Qc[Q88] += 2.0 * W.w_w;
        qc[8] += 2.0 * W.w_w * s.ub[k][1];
        // slip-angle penalties when active at the prediction (:155-165)
#pragma unroll
        for (int sr = 0; sr < 2; ++sr) {
          const double fv = s.u.l.st[k][stx(k, sr, 0)];
          const double wsl = fv >= 0.0 ? 2.0 * W.w_slip : 0.0;
          const double a5[5] = {s.u.l.st[k][stx(k, sr, 1)], s.u.l.st[k][stx(k, sr, 2)], s.u.l.st[k][stx(k, sr, 3)], s.u.l.st[k][stx(k, sr, 4)],
                                s.u.l.st[k][stx(k, sr, 5)] * S};
          constexpr int ix[5] = {0, 1, 2, 3, 7};
#pragma unroll
          for (int a = 0; a < 5; ++a) {
            qc[ix[a]] += wsl * fv * a5[a];
#pragma unroll
            for (int e = a; e < 5; ++e) Qc[qslot(ix[a], ix[e])] += wsl * a5[a] * a5[e];
          }
        }
      }
      // Fx slew with the previous stage (:167-171, point mass :226-232), the switching Fx term at
      // k = N (:244-249): c (dFx_k - p_k + (Fx_k - Fx_{k-1}) / S)^2 S^2, c = w / ds_{k-1}
      if (k >= 1) {
        const double wfx = k == N ? CW.w_switch : W.w_Fx;
        const double cs = 2.0 * wfx / s.dsv[k - 1] * S * S;
        const double r0 = (s.ub[k][0] - s.ub[k - 1][0]) / S;
        Qc[Q66] += cs;
        Qc[Q67] -= cs;
        Qc[Q77] += cs;
        qc[6] -= cs * r0;
        qc[7] += cs * r0;
      }
      if (k == N) {  // switching lateral term (:250-255): csw (dFy S - c + Fy_N - (Fy_f + Fy_r))^2
        const double csw = 2.0 * CW.w_switch / s.dsv[N - 1];
        const double r1 = s.ub[N][1] - s.u.l.gfy[0];
        Qc[Q33] += csw;
        Qc[Q38] -= csw * S;
        Qc[Q88] += csw * S * S;
        qc[3] -= csw * r1;
        qc[8] += csw * r1 * S;
      } else if (k > N) {  // Fy slew (:233-239): c (dFy_k - c_k + (Fy_k - Fy_{k-1}) / S)^2 S^2
        const double cf = 2.0 * CW.w_Fy / s.dsv[k - 1] * S * S;
        const double r0 = (s.ub[k][1] - s.ub[k - 1][1]) / S;
        Qc[Q33] += cf;
        Qc[Q38] -= cf;
        Qc[Q88] += cf;
        qc[3] -= cf * r0;
        qc[8] += cf * r0;
      }
      // w_time t_{H-1} = sum_k t-row_k . (y_k, u_k): linear stage terms (:292)
      if (k < H - 1) {
        constexpr int iy[8] = {0, 1, 2, 3, 4, 5, 7, 8};
#pragma unroll
        for (int a = 0; a < 8; ++a) qc[iy[a]] += W.w_time * s.u.l.trow[k][tsw(k, a)];
      }
      // terminal on the last point-mass state (:279-304)
      if (k == H - 1) {
        const double V = s.xs.at(k, 0);
        if (V >= W.max_speed) {
          Qc[Q00] += 2.0 * W.w_speed;
          qc[0] += 2.0 * W.w_speed * (V - W.max_speed);
        }
        Qc[Q11] += 2.0 * W.w_ey;
        qc[1] += 2.0 * W.w_ey * ey;
        Qc[Q22] += 2.0 * W.w_epsi;
        qc[2] += 2.0 * W.w_epsi * s.xs.at(k, 3);
      }
      // rows (:101-128, point mass :190-195, trust region)
      const double on = stl ? 1.0 : 0.0;
#pragma unroll
      for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int a = 0; a < 5; ++a) R.c[r][a] = 0.0;
      if (!pm) {
        const double mk = (stl && k >= 1) ? 1.0 : 0.0;
        R.d[0] = s.xs.at(k, 0) - W.Ux_min;
        R.d[1] = W.delta_max - s.xs.at(k, 3);
        R.d[2] = s.xs.at(k, 3) - W.delta_min;
        R.set(0, mk > 0.0); R.set(1, mk > 0.0); R.set(2, mk > 0.0);
#pragma unroll
        for (int r = 0; r < 5; ++r) {
          const int fn = 2 + r;
#pragma unroll
          for (int a = 0; a < 4; ++a) R.c[r][a] = s.u.l.st[k][stx(k, fn, 1 + a)] / S;
          R.c[r][4] = s.u.l.st[k][stx(k, fn, 5)];
          R.d[3 + r] = -s.u.l.st[k][stx(k, fn, 0)] / S;
          R.set(3 + r, on > 0.0);
        }
        const double wv = s.ub[k][1];
        double up = W.w_max - wv, dn = wv - W.w_min;
        if (QP.trust_w > 0) {
          up = fmin(up, QP.trust_w);
          dn = fmin(dn, QP.trust_w);
        }
        R.d[8] = up;
        R.d[9] = dn;
        R.set(8, on > 0.0); R.set(9, on > 0.0);
      } else {
        const double V = s.xs.at(k, 0);
        R.d[0] = V - CW.V_min;
        R.set(0, on > 0.0);
        R.d[1] = R.d[2] = 1.0;
        R.set(1, false); R.set(2, false);
        // Fx - Peng / V <= 0 (divided by S), linearised in (V, Fx)
        R.c[0][0] = Peng / (V * V) / S;
        R.c[0][4] = 1.0;
        R.d[3] = -(s.ub[k][0] - Peng / V) / S;
        R.set(3, on > 0.0);
#pragma unroll
        for (int r = 4; r < 8; ++r) {
          R.d[r] = 1.0;
          R.set(r, false);
        }
        R.d[8] = R.d[9] = W.trust_Fx / S;
        R.set(8, stl && W.trust_Fx > 0); R.set(9, stl && W.trust_Fx > 0);
      }
      R.d[10] = R.d[11] = W.trust_Fx / S;
      R.set(10, stl && W.trust_Fx > 0); R.set(11, stl && W.trust_Fx > 0);
#pragma unroll
      for (int i = 0; i < NR; ++i)
        if (R.m(i) == 0.0) R.d[i] = 1.0;
    }
    double sl[NR], la[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      sl[i] = R.m(i) > 0.0 ? fmax(R.d[i], 1.0) : 1.0;
      la[i] = R.m(i);
    }
    double mc = 0.0;
#pragma unroll
    for (int i = 0; i < NR; ++i) mc += R.m(i);
    const double mcount = wsum(mc);
    // the residual floor grows with the data (|q| up to ~1e3 in the scaled units): the
    // stopping test is relative to it
    double qm = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) qm = fmax(qm, fabs(qc[e]));
    const double rtol = tol_r * (1.0 + wmax(stl ? qm : 0.0));
    WSYNC();  // the linearisation scratch is dead from here: the QP arrays alias it
    double vk[9];  // the QP iterate (xt, u) of this lane's stage
#pragma unroll
    for (int e = 0; e < 9; ++e) vk[e] = 0.0;

    // ---- LQ machinery (st_sqp.hip's, over H stages) -----------------------------------
    // Riccati lane roles: H entry (hi, hj), hi <= hj, for lanes < 45; P entry (pi, pj) for
    // lanes < 28.  Recomputed here each SQP iteration (a few integer ops) rather than held
    // across the linearisation, whose dual-number evaluations need every register.
    int hi = 0, hj = 0;
    {
      int q = l < 45 ? l : 0, i = 0;
      while (q >= 9 - i) { q -= 9 - i; ++i; }
      hi = i;
      hj = i + q;
    }
    const int hslot = qslot(hi, hj), hci = vcol(hi), hcj = vcol(hj);
    int pi = 0, pj = 0;
    {
      int q = l < 28 ? l : 0, i = 0;
      while (q >= 7 - i) { q -= 7 - i; ++i; }
      pi = i;
      pj = i + q;
    }
    const int ta = l < 56 ? (l >> 3) : 0, tj = l & 7;
    const double tpm = tj == 6 ? 1.0 : 0.0;
    const int hcic = hci < 0 ? 0 : hci, hcjc = hcj < 0 ? 0 : hcj;
    const double hdyn = (l < 45 && hci >= 0 && hcj >= 0) ? 1.0 : 0.0, hpm = hci == 6 ? 1.0 : 0.0;
    const int hsc = hslot < 0 ? 0 : hslot;
    const double hq = (l < 45 && hslot >= 0) ? 1.0 : 0.0;
    struct FacOps {
      double JT[6], JH[6], qv;
    };
    auto fac_load = [&](int kk, FacOps& o) {
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        o.JT[e] = JLD(kk, e, tj);
        o.JH[e] = JLD(kk, e, hcic);
      }
      o.qv = s.u.q.Qt[kk][hsc];
    };
    auto fac_stage = [&](int kk, const FacOps& o) -> bool {
      double hv = hq * o.qv;
      if (kk < H - 1) {  // uniform
        double acc = tpm * s.u.q.f.P[ta][6];
#pragma unroll
        for (int e = 0; e < 6; ++e) acc += s.u.q.f.P[ta][e] * o.JT[e];
        if (l < 56) s.u.q.f.T[ta][tj] = acc;
        WSYNC();
        double a2 = hpm * s.u.q.f.T[6][hcjc];
#pragma unroll
        for (int e = 0; e < 6; ++e) a2 += o.JH[e] * s.u.q.f.T[e][hcjc];
        hv += hdyn * a2;
      }
      if (l < 45) {
        s.u.q.f.Hm[hi][hj] = hv;
        s.u.q.f.Hm[hj][hi] = hv;
      }
      WSYNC();
      const double h00 = s.u.q.f.Hm[7][7], h01 = s.u.q.f.Hm[7][8], h11 = s.u.q.f.Hm[8][8];
      const double det = h00 * h11 - h01 * h01;
      // reciprocal bit-identical to IEEE 1/x on every class (asserted: tests/test_gpu_numerics.py): the plain v_rcp_f64 + Newton form turns
      // det = +inf (h00 h11 overflowing at barrier weights ~1e154) into NaN where 1/det = 0
      const double id = rcp_nr(det);
      const double i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
      {
        const int kc = l >= 28 && l < 42 ? (l - 28) / 7 : 0, ki = l >= 28 && l < 42 ? (l - 28) % 7 : 0;
        const int ci = l < 28 ? pi : ki;
        const double x0 = s.u.q.f.Hm[7][ci], x1 = s.u.q.f.Hm[8][ci], y0 = s.u.q.f.Hm[7][pj], y1 = s.u.q.f.Hm[8][pj];
        const double hpp = s.u.q.f.Hm[pi][pj];
        if (l < 28) {
          const double pv = hpp - (x0 * (i00 * y0 + i01 * y1) + x1 * (i01 * y0 + i11 * y1));
          s.u.q.f.P[pi][pj] = pv;
          s.u.q.f.P[pj][pi] = pv;
        } else if (l < 42) {
          s.u.q.K[kk][kc][ki] = kc == 0 ? -(i00 * x0 + i01 * x1) : -(i01 * x0 + i11 * x1);
        } else if (l == 42) {
          s.u.q.Hi[kk][0] = i00;
          s.u.q.Hi[kk][1] = i01;
          s.u.q.Hi[kk][2] = i11;
        }
      }
      WSYNC();
      // det = +inf (h00 h11 overflowing: a diverging barrier) is a failed factorisation: its exact
      // reciprocal 0 would silently drop the input block (Hi = K = 0) from the Newton step
      return h00 > 0.0 && det >= 0x1p-1022 && isfinite(det);  // (and a subnormal det)
    };
    auto factor = [&]() -> bool {
      bool ok = true;
      FacOps A0, B0;
      fac_load(H - 1, A0);
#pragma unroll 1
      for (int kk = H - 1; kk >= 0; kk -= 2) {
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

    const int sl9 = l < 9 ? l : 8;
    const int scol = vcol(sl9) < 0 ? 0 : vcol(sl9);
    const double smsk = (l < 9 && vcol(sl9) >= 0) ? 1.0 : 0.0;
    const double spm = (l < 9 && vcol(sl9) == 6) ? 1.0 : 0.0;
    const int bl7 = l < 7 ? l : 0;
    const int fr = l < 6 ? l : 0, fc = l == 8 ? 1 : 0;
    const bool fk = l == 7 || l == 8;

    struct BwdOps {
      double J6[6], h, a, b;
    };
    auto bwd_load = [&](int kk, const double (*vec)[9], BwdOps& o) {
#pragma unroll
      for (int e = 0; e < 6; ++e) o.J6[e] = JLD(kk, e, scol);
      o.h = vec[kk][sl9];
      const double* pa = l < 7 ? &s.u.q.K[kk][0][bl7] : &s.u.q.Hi[kk][l == 7 ? 0 : 1];
      const double* pb = l < 7 ? &s.u.q.K[kk][1][bl7] : &s.u.q.Hi[kk][l == 7 ? 1 : 2];
      o.a = *pa;
      o.b = *pb;
    };
    auto bwd_g = [&](int kk, const BwdOps& o, double pv) -> double {
      double g = o.h;
      if (kk < H - 1) {  // uniform
        double pb[7];
#pragma unroll
        for (int a = 0; a < 7; ++a) pb[a] = bcast(pv, a);
        double acc = spm * pb[6];
#pragma unroll
        for (int e = 0; e < 6; ++e) acc += o.J6[e] * pb[e];
        g += smsk * acc;
      }
      return g;
    };
    struct FwdOps {
      double w[8];
    };
    auto fwd_load = [&](int kk, FwdOps& o) {
      if constexpr (JG) {  // (no pointer select across address spaces: it would go flat)
#pragma unroll
        for (int e = 0; e < 7; ++e) {
          const double kv = s.u.q.K[kk][fc][e], jv = JLD(kk, fr, e);
          o.w[e] = fk ? kv : jv;
        }
        const double k7 = s.u.q.kk[kk][fc], j7 = JLD(kk, fr, 7);
        o.w[7] = fk ? k7 : j7;
      } else {
        const double* src = fk ? &s.u.q.K[kk][fc][0] : &J[kk].m[fr][0];
        const double* src7 = fk ? &s.u.q.kk[kk][fc] : &J[kk].m[fr][7];
#pragma unroll
        for (int e = 0; e < 7; ++e) o.w[e] = src[e];
        o.w[7] = *src7;
      }
    };
    auto fwd_stage = [&](int kk, const FwdOps& o, double X) -> double {
      double xb[7];
#pragma unroll
      for (int a = 0; a < 7; ++a) xb[a] = bcast(X, a);
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < 6; ++e) acc += o.w[e] * xb[e];
      const double uk = acc + o.w[6] * xb[6] + o.w[7];
      const double u0 = bcast(uk, 7), u1 = bcast(uk, 8);
      if (l < 9) s.u.q.g[kk][l] = fk ? uk : X;
      const double xn = acc + o.w[6] * u0 + o.w[7] * u1;
      return l < 6 ? xn : (l == 6 ? u0 : 0.0);
    };
    auto lq_solve = [&]() {
      BwdOps A1, B1;
      bwd_load(H - 1, s.u.q.g, A1);
      double pv = 0.0;
      auto bstage = [&](int kk, const BwdOps& o) {
        const double g = bwd_g(kk, o, pv);
        const double gu0 = bcast(g, 7), gu1 = bcast(g, 8);
        const double t2 = o.a * gu0 + o.b * gu1;
        pv = g + t2;
        if (fk) s.u.q.kk[kk][l - 7] = -t2;
      };
#pragma unroll 1
      for (int kk = H - 1; kk >= 0; kk -= 2) {
        const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
        bwd_load(k1, s.u.q.g, B1);
        bstage(kk, A1);
        if (kk >= 1) {
          bwd_load(k2, s.u.q.g, A1);
          bstage(kk - 1, B1);
        }
      }
      WSYNC();
      double X = 0.0;
      FwdOps A2, B2;
      fwd_load(0, A2);
#pragma unroll 1
      for (int kk = 0; kk < H; kk += 2) {
        const int k1 = kk + 1 < H ? kk + 1 : kk, k2 = kk + 2 < H ? kk + 2 : kk;
        fwd_load(k1, B2);
        X = fwd_stage(kk, A2, X);
        if (kk + 1 < H) {
          fwd_load(k2, A2);
          X = fwd_stage(kk + 1, B2, X);
        }
      }
      WSYNC();
    };
    // condensed dual residual through the dynamics (adjoint sweep); cl: through the closed-loop
    // A + B K of the last Riccati factorisation, as in st_sqp.hip (the open-loop sweep amplifies
    // rounding through the RK4 step's unstable lateral mode at low speed)
    auto dual_residual = [&](bool cl) -> double {
      BwdOps A3, B3;
      bwd_load(H - 1, s.u.q.g, A3);
      double rho = 0.0, rmax = 0.0;
      auto rstage = [&](int kk, const BwdOps& o) {
        const double g = bwd_g(kk, o, rho);
        rmax = fk ? fmax(rmax, fabs(g)) : rmax;
        rho = cl ? g + o.a * bcast(g, 7) + o.b * bcast(g, 8) : g;  // lanes 0..6: + K' g_u
      };
#pragma unroll 1
      for (int kk = H - 1; kk >= 0; kk -= 2) {
        const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
        bwd_load(k1, s.u.q.g, B3);
        rstage(kk, A3);
        if (kk >= 1) {
          bwd_load(k2, s.u.q.g, A3);
          rstage(kk - 1, B3);
        }
      }
      return wmax(rmax);
    };

    // stage lanes: s.u.q.Qt[k] = Qc + sum_i w_i c_i c_i' (the barrier weights of the interior
    // point, or the augmented-Lagrangian weights of the polish)
    auto put_qt = [&](const double* w) {
      double Qt[NQ];
#pragma unroll
      for (int e = 0; e < NQ; ++e) Qt[e] = Qc[e];
      Qt[Q00] += w[0];
      Qt[Q33] += w[1] + w[2];
      Qt[Q88] += w[8] + w[9];
      Qt[Q77] += w[10] + w[11];
      constexpr int ix[5] = {0, 1, 2, 3, 7};
#pragma unroll
      for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int a = 0; a < 5; ++a)
#pragma unroll
          for (int e = a; e < 5; ++e) Qt[qslot(ix[a], ix[e])] += w[3 + r] * R.c[r][a] * R.c[r][e];
#pragma unroll
      for (int e = 0; e < NQ; ++e) s.u.q.Qt[k][e] = Qt[e];
    };

    // ---------------- interior point (Mehrotra predictor-corrector) ----------------
    int it = 0;
    bool conv = false, fail = false;
    // dual residual carried by the steps: the LQ direction solves the linearised
    // stationarity exactly, so a step of length alpha scales the condensed gradient by
    // (1 - alpha); the adjoint sweep runs at the first iteration and wherever the carried value
    // would end the loop (convergence, or acceptance at a factorisation failure)
    double rd_carry = 0.0;
    bool have_rd = false;
    bool kvalid = false;  // s.u.q.K holds this IPM's factorisation (the linearisation aliases it)
#pragma unroll 1
    for (; it < s.qp.max_iter; ++it) {
      double rp[NR], wg[NR], grk[9], val[NR];
      double rpm = 0.0, mus = 0.0;
      row_values(R, vk, val);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        rp[i] = R.m(i) * (val[i] + sl[i] - R.d[i]);
        wg[i] = R.m(i) * la[i] / sl[i];
        rpm = fmax(rpm, fabs(rp[i]));
        mus += R.m(i) * sl[i] * la[i];
      }
      qmul(Qc, vk, grk);
#pragma unroll
      for (int e = 0; e < 9; ++e) grk[e] += qc[e];
      {
        double ml[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) ml[i] = R.m(i) * la[i];
        row_adjoint(R, ml, grk);
      }
      if (stl) {
#pragma unroll
        for (int e = 0; e < 9; ++e) s.u.q.g[k][e] = grk[e];
        put_qt(wg);
      } else {
        rpm = 0.0;
        mus = 0.0;
      }
      WSYNC();
      rpm = wmax(rpm);
      const double mu = wsum(mus) / mcount;
      const bool carried = have_rd;
      double rdm = carried ? rd_carry : dual_residual(kvalid);
      bool rd_cl = carried || kvalid;
      last_res = fmax(rdm, rpm);
      last_mu = mu;
      if (!(last_res == last_res) || !(mu == mu) || last_res > 1e300) { fail = true; break; }
      if (have_rd && mu <= 1e2 * tol_mu && fmax(rdm, rpm) <= 1e3 * rtol) {
        // the carried value would end the loop here or below: take the sweep's
        rdm = dual_residual(kvalid);
        rd_cl = kvalid;
        have_rd = false;
        last_res = fmax(rdm, rpm);
        if (!(last_res == last_res) || last_res > 1e300) { fail = true; break; }
      }
      if (last_res <= rtol && mu <= tol_mu) { conv = true; break; }

      const bool fok = factor();
      kvalid = kvalid || fok;
      if (!fok) {
        // the barrier-augmented recursion lost definiteness at the numerical floor (weights
        // ~1e13, cancellation in P = Hxx - Hxu Huu^-1 Hux): a near-converged iterate stands
        if (mu <= 1e2 * tol_mu && last_res <= 1e3 * rtol) conv = true;
        else fail = true;
        break;
      }

      auto set_h = [&](const double* rc_over_s) {
        if (stl) {
          double y[NR], hk[9];
#pragma unroll
          for (int i = 0; i < NR; ++i) y[i] = R.m(i) * (wg[i] * rp[i] - rc_over_s[i]);
#pragma unroll
          for (int e = 0; e < 9; ++e) hk[e] = grk[e];
          row_adjoint(R, y, hk);
#pragma unroll
          for (int e = 0; e < 9; ++e) s.u.q.g[k][e] = hk[e];
        }
        WSYNC();
      };
      set_h(la);
      lq_solve();
      double dsa[NR], dla[NR], cdv[NR], dvk[9];
      double amin = 1.0;
#pragma unroll
      for (int e = 0; e < 9; ++e) dvk[e] = s.u.q.g[k][e];
      row_values(R, dvk, cdv);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        dsa[i] = R.m(i) * (-rp[i] - cdv[i]);
        dla[i] = R.m(i) * (wg[i] * (cdv[i] + rp[i]) - la[i]);
        if (stl && R.m(i) > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
      }
      amin = wmin(amin);
      double ms = 0.0;
      if (stl) {
#pragma unroll
        for (int i = 0; i < NR; ++i) ms += R.m(i) * (sl[i] + amin * dsa[i]) * (la[i] + amin * dla[i]);
      }
      ms = wsum(ms) / mcount;
      const double ratio = mu > 0.0 ? fmin(1.0, ms / mu) : 0.0;
      const double smu = ratio * ratio * ratio * mu;

      double rcs[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) rcs[i] = R.m(i) * (sl[i] * la[i] + dsa[i] * dla[i] - smu) / sl[i];
      set_h(rcs);
      lq_solve();
#pragma unroll
      for (int e = 0; e < 9; ++e) dvk[e] = s.u.q.g[k][e];
      row_values(R, dvk, cdv);
      amin = 1.0;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        dsa[i] = R.m(i) * (-rp[i] - cdv[i]);
        dla[i] = R.m(i) * (wg[i] * (cdv[i] + rp[i]) - rcs[i]);
        if (stl && R.m(i) > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
      }
      const double alpha = fmin(1.0, 0.99 * wmin(amin));
      rd_carry = (1.0 - alpha) * rdm;
      have_rd = rd_cl;  // only closed-loop values are carried
      if (stl) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          if (R.m(i) > 0.0) {
            sl[i] = fmax(sl[i] + alpha * dsa[i], 1e-300);
            la[i] = fmax(la[i] + alpha * dla[i], 1e-300);
          }
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) vk[e] += alpha * dvk[e];
      }
      WSYNC();
    }
    it_total += it;
    it_max = max(it_max, it);

    // ---------------- active-set polish (round 5; st_sqp.hip has the same) ----------------
    // The interior point's iterate is only as close to the QP's optimum as its weakly active rows
    // allow (tests/test_gpu_certify.py: up to 1e-6 in the scaled units on the bench batch, 1e-3 N).
    // The QP on the active set it identified (lambda > s) is solved exactly by an augmented
    // Lagrangian (one Riccati factorisation of Q + sum_A rho_i c_i c_i') whose passes are Newton
    // steps from the current point (the gradient recomputed stage-locally, so the factor's rounding
    // is refined away) with multiplier updates, then certified (inactive rows feasible, active
    // multipliers nonnegative); otherwise the violated rows join and the negative ones leave.
    bool pol_qp = false;
    if (kCrPolish > 0 && conv) {
      double hs = 0.0, qs = 0.0;
      if (stl) {
        hs = fmax(fmax(fmax(Qc[Q00], Qc[Q11]), fmax(Qc[Q22], Qc[Q33])),
                  fmax(fmax(Qc[Q44], Qc[Q55]), fmax(fmax(Qc[Q66], Qc[Q77]), Qc[Q88])));
#pragma unroll
        for (int e = 0; e < 9; ++e) qs = fmax(qs, fabs(qc[e]));
      }
      hs = 1.0 + wmax(hs);
      qs = 1.0 + wmax(qs);
      // row i's weight (recomputed where used: an array of 12 would stay live across the polish)
      const double rho_h = kCrAlRho * hs;
      auto rho = [&](int i) -> double {
        double cn2 = 1.0;
        if (i >= 3 && i < 8) {
          cn2 = 0.0;
#pragma unroll
          for (int a = 0; a < 5; ++a) cn2 += R.c[i - 3][a] * R.c[i - 3][a];
        }
        return rho_h / fmax(cn2, 1e-30);
      };
      uint32_t act = 0;  // bit i: row i active
#pragma unroll
      for (int i = 0; i < NR; ++i) act |= (stl && R.m(i) > 0.0 && la[i] > sl[i]) ? (1u << i) : 0u;
#pragma unroll 1
      for (int round = 0; round < kCrPolish; ++round) {
        // the interior point's slacks / multipliers are dead from here: sl holds the polish's
        // iterate and la its multipliers (a later round starts from the last round's)
        double w[NR], val[NR] = {};
        double* const lm = la;
        double* const vp = sl;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const bool ai = (act >> i) & 1u;
          w[i] = ai ? rho(i) : 0.0;
          lm[i] = ai ? lm[i] : 0.0;
        }
        if (stl) put_qt(w);
        WSYNC();
        if (!factor()) break;  // keep the interior point's iterate
#pragma unroll
        for (int e = 0; e < 9; ++e) vp[e] = vk[e];
        bool al_conv = false;
        int held = 0;
#pragma unroll 1
        for (int p = 0; p < kCrAlPasses; ++p) {
          if (stl) {
            double g9[9], y[NR];
            row_values(R, vp, val);
#pragma unroll
            for (int i = 0; i < NR; ++i) y[i] = ((act >> i) & 1u) ? lm[i] + rho(i) * (val[i] - R.d[i]) : 0.0;
            qmul(Qc, vp, g9);
#pragma unroll
            for (int e = 0; e < 9; ++e) g9[e] += qc[e];
            row_adjoint(R, y, g9);
#pragma unroll
            for (int e = 0; e < 9; ++e) s.u.q.g[k][e] = g9[e];
          }
          WSYNC();
          lq_solve();
          double emax = 0.0;
          if (stl) {
#pragma unroll
            for (int e = 0; e < 9; ++e) vp[e] += s.u.q.g[k][e];
            row_values(R, vp, val);
#pragma unroll
            for (int i = 0; i < NR; ++i) {
              const double r = ((act >> i) & 1u) ? val[i] - R.d[i] : 0.0;
              lm[i] += rho(i) * r;
              emax = fmax(emax, fabs(r));
            }
          }
          WSYNC();
          // converged: the active rows held on two passes in a row -- the second is a pure refinement
          // step (the first pass that meets the rows still carries the factor's error, ~cond x eps in v:
          // r05 certified N = 60 problem 2531 at a stationarity of 2e-9 x scale without it)
          held = wmax(emax) <= 1e-14 * qs ? held + 1 : 0;
          if (held >= 2) {
            al_conv = true;
            break;
          }
        }
        // certificate: inactive rows feasible, active multipliers nonnegative (the row values
        // recomputed here keep val out of the pass loop's live set)
        if (stl) row_values(R, vp, val);
        uint32_t viol = 0, neg = 0;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          const bool ai = (act >> i) & 1u;
          viol |= (stl && R.m(i) > 0.0 && !ai && val[i] - R.d[i] > kCrCertPtol * qs) ? (1u << i) : 0u;
          neg |= (ai && lm[i] < -kCrCertDtol * qs) ? (1u << i) : 0u;
        }
        if (al_conv && __all((viol | neg) ? 0 : 1) != 0) {
          if (stl) {
#pragma unroll
            for (int e = 0; e < 9; ++e) vk[e] = vp[e];
          }
          pol_qp = true;
          break;
        }
        act = (act | viol) & ~neg;
      }
      WSYNC();
    }
    all_pol = all_pol && (pol_qp || !conv);
    // a QP after the first without a solution (an infeasible linearisation: the interior point
    // diverges) refuses its own step and ends the SQP at the current iterate, whose rollout is
    // s.xs; the step's status is then that of the QPs before it -- the kinematic SQP's rule
    // (kin_merit.hip) and oracle/dyn_sqp.py alike.  (Applying the unconverged iterate and
    // reporting the whole step non-solved threw away a plan from converged QPs: the
    // single-track N = 60 obstacle run on the shoe track lost the car, scripts/band_trace.py.)
    if (sq > 0 && !conv) {
      stopped = true;
      break;
    }
    all_conv = all_conv && conv;
    any_fail = any_fail || fail;

    // ---------------- SQP update: ubar += dz (Fx, and the point mass's Fy, scaled by S) ----------------
    // tested by the next rollout (domain cut-back above)
    if (stl) {
      const double u0v = s.ub[k][0], u1v = s.ub[k][1];
      s.u.q.g[k][0] = u0v;
      s.u.q.g[k][1] = u1v;
      s.u.q.g[k][2] = vk[7];
      s.u.q.g[k][3] = vk[8];
      s.ub[k][0] = u0v + vk[7] * S;
      if (pm) s.ub[k][1] = u1v + vk[8] * S;
      else s.ub[k][1] = fmin(fmax(u1v + vk[8], s.w.w_min), s.w.w_max);
    }
    test = s.flag[2] != 0;  // from an iterate outside the domain: the full step, untested
    tries = 1;
    WSYNC();
  }

  // ---------------- outputs: u*, x* = rollout(u*), u0, status ----------------
  bool finite = true;
  for (int e = l; e < 2 * H; e += WTH) {
    const double v = s.ub[e >> 1][e & 1];
    finite = finite && isfinite(v);
    A.u_out[(size_t)b * 2 * H + e] = v;
  }
  for (int e = l; e < 8 * H; e += WTH) {
    const double v = s.xs.at(e >> 3, e & 7);
    finite = finite && isfinite(v);
    A.x_out[(size_t)b * 8 * H + e] = v;
  }
  finite = __all(finite ? 1 : 0) != 0;
  if (l < 2) A.u0[(size_t)b * 2 + l] = s.ub[0][l];
  if (l == 0) {
    int32_t st;
    if (!finite || s.flag[0] == VC_NONFINITE) st = VC_NONFINITE;
    else if (s.flag[2] == 0) st = VC_OUT_OF_DOMAIN;  // x* (the last rollout) outside the models' domain
    else if (all_conv) st = VC_SOLVED;
    else st = VC_MAX_ITER;
    A.status[b] = st;
    A.iters[b] = it_total;
    if (A.diag) {
      constexpr size_t DS = VC_CASC_DIAG_COLS;  // the ABI's row stride (no section counters here)
      A.diag[(size_t)b * DS + 0] = last_res;
      A.diag[(size_t)b * DS + 1] = last_mu;
      A.diag[(size_t)b * DS + 2] =
          double((any_fail ? 1 : 0) | (all_conv ? 2 : 0) | (all_pol ? 4 : 0) | (stopped ? 16 : 0));
      A.diag[(size_t)b * DS + 3] = double(it_max);
    }
  }
}

}  // namespace

// ---- host launcher ---------------------------------------------------------------
// N = 20 single-track stages (cascaded.yaml) x the recorded tails M = 15, 25, 35, 40
#define VC_CR_SHAPES(X) X(20, 15) X(20, 25) X(20, 35) X(20, 40)

bool casc_ric_built(int N, int M) {
#define VC_CASE(n, m) \
  if (N == n && M == m) return true;
  VC_CR_SHAPES(VC_CASE)
#undef VC_CASE
  return false;
}

// J placement per launch (st_sqp.hip st_jg_pick): the LDS-J kernel while the batch fits the machine
// at its occupancy, the four-per-CU global-J kernel beyond
template <int N, int M>
bool cr_jg_pick(int B) {
  if constexpr (!cr_j_global_ok<N, M>()) return false;
  else return B > wg_per_cu(sizeof(CrSmem<N, M, false>)) * device_cus();
}

// doubles of J workspace per problem a launch of B problems needs (nonzero only where cr_jg_pick
// takes the global-J kernel)
size_t casc_ric_jws_doubles(int N, int M, int B) {
#define VC_CASE(n, m) \
  if (N == n && M == m) return cr_jg_pick<n, m>(B) ? (size_t)(n + m) * 48 : 0;
  VC_CR_SHAPES(VC_CASE)
#undef VC_CASE
  return 0;
}

template <int N, int M, int TYRE>
void cr_launch(const CascSqpArgs& a, hipStream_t stream) {
  if constexpr (cr_j_global_ok<N, M>()) {
    if (cr_jg_pick<N, M>(a.B)) {
      hipLaunchKernelGGL((casc_ric_kernel<N, M, TYRE, true>), dim3(a.B), dim3(WTH), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((casc_ric_kernel<N, M, TYRE, false>), dim3(a.B), dim3(WTH), 0, stream, a);
}

hipError_t launch_casc_ric(const CascSqpArgs& a, int N, int M, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  if (casc_ric_jws_doubles(N, M, a.B) && !a.jws) return hipErrorInvalidValue;  // the workspace the kernel needs
  const bool lin = a.car.tyre == VC_TYRE_LINEAR;
#define VC_CASE(n, m)                                \
  if (N == n && M == m) {                           \
    if (lin) cr_launch<n, m, VC_TYRE_LINEAR>(a, stream); \
    else cr_launch<n, m, VC_TYRE_FIALA>(a, stream);      \
    return hipGetLastError();                       \
  }
  VC_CR_SHAPES(VC_CASE)
#undef VC_CASE
  return hipErrorInvalidValue;
}

}  // namespace vc
