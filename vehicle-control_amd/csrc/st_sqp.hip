// st_sqp.hip -- fused single-track SQP step, fp64, one wavefront per problem, with a
// stagewise Riccati interior point.
//
// Replaces the IPOPT solve of CascadedMPC in single-track mode (controllers/mpc/
// cascaded_mpc.py:17-39,91-179,279-314, horizon_pm = 0) for the reference's own horizons
// (config/controllers/singletrack.yaml N = 60; recorded runs N = 50 / 60) and BASELINE's
// N = 40.  Contract: oracle/dyn_sqp.py (the same QP as the fp32 condensed kernel
// dyn_sqp.hip, solved to fp64 accuracy).  Per SQP iteration:
//   predict    lane 0: RK4 spatial rollout (vc_models.hpp dyn_spatial_ode_alg)
//   linearize  one lane per (stage, seed pair): Dual<2> RK4 step -> two columns of
//              [A B] and of the t-row; one lane per (stage, seed) for the stage terms
//              (slip residuals, power and tyre-force rows) with Dual<1>
//   QP         restated stage by stage (scripts/riccati_proto.py): QP state
//              xt_k = (dUx, dUy, dr, ddelta, dey, depsi, p_k), p_k = dz_{k-1,Fx} (the Fx
//              slew couples neighbouring stages), input u_k = dz_k = (dFx/S, dw); s is
//              fixed (s' = 1) and t only enters w_time t_{N-1}, which becomes linear stage
//              terms through each step's t-row.  Stage Hessians have 20 nonzeros; the 12
//              one-sided rows of a stage touch (Ux, Uy, r, delta, dFx, dw) only.
//              Mehrotra predictor-corrector; each Newton step is an LQ problem solved by
//              a backward Riccati recursion (7 states + 2 inputs per stage: O(N) work per
//              iteration, where the condensed form pays O(N^3)), then forward sweeps.
//              Lane k owns stage k's rows, slacks and multipliers in registers; the
//              recursions run on lanes 0..44 with the stage matrices in LDS.
//   update     ubar += dz (Fx scaled back by fx_scale)
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "vc_dual.hpp"
#include "vc_kernels.hpp"

namespace vc {
namespace {

constexpr int WTH = 64;
constexpr int NQ = 20;  // nonzeros of a stage Hessian over v = (Ux, Uy, r, delta, ey, epsi, p, dFx, dw)
constexpr int NR = 12;  // one-sided rows per stage
// slots of the stage Hessian's nonzeros (block {Ux, Uy, r, delta, dFx} + five diagonal-ish)
enum { Q00, Q01, Q02, Q03, Q07, Q11, Q12, Q13, Q17, Q22, Q23, Q27, Q33, Q37, Q77, Q44, Q55, Q66, Q67, Q88 };

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

// LDS layout.  Strides: every array a lane-per-stage phase reads or writes (residuals, stage
// data, linearisation) has an odd number of doubles per stage (or per matrix row read across
// lanes), so the 32 lanes of a ds_read_b64 group land on 32 distinct bank pairs ((a/4) mod 64)
// and the 16 lanes of a ds_write_b64 group on 16 ((a/4) mod 32); pad slots are never touched.
// Size: one stage vector g carries the dual-residual gradient, the LQ right-hand side, the
// Newton direction and the SQP cut-back's data in turn, and the Riccati scratch between them
// (disjoint live ranges, below); the QP iterate stays in registers.  N = 40 then fits 4 one-wave
// workgroups per CU (one per SIMD; 48.5 KB before left one SIMD idle), N = 60 fits 3 (was 2).
// [A6 | B6 diag(S, 1)] of one step, rows Ux, Uy, r, delta, ey, epsi; + 1 pad.  The forward LQ pass
// reads rows 0..5 of one stage in lanes 0..5: a row stride of 8 doubles puts rows r and r + 4 on
// the same banks, 9 does not -- used where the extra 6 doubles per stage keep the workgroups per
// CU (N = 20, 40, 50; N = 30 / 60 would lose one)
template <int JW>
struct StJT {
  double m[6][JW];
  double pad;
  __device__ __forceinline__ double* operator[](int r) { return m[r]; }
  __device__ __forceinline__ const double* operator[](int r) const { return m[r]; }
};
template <int N>
using StJ = StJT<(N == 30 || N == 60) ? 8 : 9>;
// Round 5: [A6 | B6] in LDS costs 49 doubles per stage (23.5 KB at N = 60) and kept st_sqp<60> at three
// workgroups per CU.  From N = 45 on it lives in a per-problem global workspace instead
// (StSqpArgs.jws, 384 B = three 128 B lines per stage; written once per SQP iteration by the
// linearisation, read by the Riccati passes one stage ahead of use, so the L2 latency overlaps the
// current stage's chain).
// whether the global-J instantiation exists for horizon N (the launcher picks it per batch: st_jg_pick)
template <int N>
constexpr bool st_j_global_ok() { return N >= 45; }
template <int N, bool JG>
using StJP = std::conditional_t<JG, double*, StJ<N>*>;  // workspace base (GBuf) or LDS
struct StNone {};  // (global: 48 doubles = 384 B per stage, [6][8] row-major)
// Row stride of ub: odd (3; conflict-free lane-per-stage reads) where the LDS allows, N = 60 takes
// 2 -- a block above 53,248 B leaves two workgroups per CU instead of three (measured: rocprofv3
// LDS_Block_Size 53,248 ran three per CU, 54,272 two; r04).  xs: rotated rows of 8 (StageRows8)
template <int N>
constexpr int st_ub_w() { return N == 60 ? 2 : 3; }
template <int N, bool JG>
struct StSmem {
  StageRows8<N> xs;   // prediction (N columns, dynamics for k < N-1), rotated rows (vc_kernels.hpp)
  double ub[N][st_ub_w<N>()];  // current ubar; [2] pad where 3
  double kap[N], dsv[N];
  // J[k][row][col], cols Ux, Uy, r, delta, ey, epsi | dFx, dw (LDS unless JG)
  std::conditional_t<JG, StNone, StJ<N>[N]> J;
  union {
    struct {
      double Qt[N][NQ + 1];  // stage Hessian + barrier, this iteration; [NQ] pad
      // stage vector, three lives per interior-point iteration: the gradient Q v + q + C' lam
      // (residuals -> dual residual sweep), the LQ right-hand side h (set_h -> backward pass),
      // the direction dv (forward pass -> step); after the QP: the pre-step iterate uo in
      // [0..1] and the step dz in [2..3] (SQP update -> domain cut-back).  The QP iterate v
      // itself lives in its lane's registers.  During the Riccati factorisation (between the
      // dual residual sweep and set_h: g dead) the same space holds the factorisation's
      // scratch f: cost-to-go P, T = P [A B], stage Hessian Hm.
      union {
        double g[N][9];
        struct {
          double P[7][7];
          double T[7][8];
          double Hm[9][9];
        } f;
      };
      double K[N][2][7];
      double Hi[N][3];   // Huu^-1 (00, 01, 11)
      double kk[N][2];
    } q;
    struct {
      // (unpadded: this member sets the union's size; its reads are once per SQP iteration)
      double trow[N - 1][8];  // t-row of step k < N-1 over (y | dFx, dw)
      double st[N][42];    // stage functions: value + gradient over (Ux, Uy, r, delta, Fx)
    } l;
  } u;
  int flag[4];
};

// Workgroup = one wavefront: LDS operations of a wave execute in order, so a sync only has to
// stop the compiler from moving memory operations across it (no s_barrier, and no wait for
// outstanding loads other than the ones actually used).
constexpr double kStNewtonTol = 1e-14;  // accepted defect, relative to 1 + |y|
constexpr int kStNewtonMax = 12;
// below ~6 m/s the reference's RK4 step (mpc_dt 0.03 s) is expansive in the lateral mode (|eig A_k| 3-5
// at 4 m/s), so a stage defect the chord iteration accepts at 1e-14 grows through the stages
// and x* drifts from rollout(u*): there the serial rollout runs
constexpr double kStNewtonUxMin = 8.0;

constexpr int kStPolish = 3;  // active-set polish rounds after each converged QP (0: off, the round-4 kernel)
constexpr double kStAlRho = 1e2;  // polish: augmented-Lagrangian weight of an active row, x (1 + max diag Q) / |c|^2
constexpr int kStAlPasses = 16;
constexpr double kStCertPtol = 1e-11;  // polish certificate: inactive-row violation, x (1 + max |q|)
constexpr double kStCertDtol = 1e-12;  // polish certificate: wrong-signed multiplier, x (1 + max |q|)


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

// Section timing (debug builds only, -DVC_TIMING, `make timing`): lane 0's s_memtime stamps,
// accumulated per section and written to diag[b][4 + slot] (scripts/st_section_timing.py).
enum { ST_PRED = 0, ST_LIN, ST_SETUP, ST_RESID, ST_DUAL, ST_FACT, ST_SOLVE, ST_STEP, ST_TOTAL, ST_NSLOT };
#ifdef VC_TIMING
#define ST_STAMP(var)                                \
  __builtin_amdgcn_sched_barrier(0);                 \
  const uint64_t var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0);
#define ST_ACC(slot, t0)                               \
  {                                                    \
    __builtin_amdgcn_sched_barrier(0);                 \
    tacc[slot] += __builtin_amdgcn_s_memtime() - (t0); \
    __builtin_amdgcn_sched_barrier(0);                 \
  }
#else
#define ST_STAMP(var)
#define ST_ACC(slot, t0)
#endif

// Stage k's one-sided rows C v <= d (lane-owned):
//   0: -Ux <= Ux - Ux_min          1: delta <= delta_max - delta   2: -delta <= delta - delta_min
//   3..7: c_r . (Ux, Uy, r, delta, dFx) <= d_r   (power limit, tyre force bounds front / rear)
//   8: dw <= ..   9: -dw <= ..   10: dFx <= trust   11: -dFx <= trust
struct Rows {
  double c[5][5];
  double d[NR];
  double m[NR];
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
// out = Q v (symmetric, 20 slots)
__device__ __forceinline__ void qmul(const double* Q, const double* v, double* o) {
  o[0] = Q[Q00] * v[0] + Q[Q01] * v[1] + Q[Q02] * v[2] + Q[Q03] * v[3] + Q[Q07] * v[7];
  o[1] = Q[Q01] * v[0] + Q[Q11] * v[1] + Q[Q12] * v[2] + Q[Q13] * v[3] + Q[Q17] * v[7];
  o[2] = Q[Q02] * v[0] + Q[Q12] * v[1] + Q[Q22] * v[2] + Q[Q23] * v[3] + Q[Q27] * v[7];
  o[3] = Q[Q03] * v[0] + Q[Q13] * v[1] + Q[Q23] * v[2] + Q[Q33] * v[3] + Q[Q37] * v[7];
  o[4] = Q[Q44] * v[4];
  o[5] = Q[Q55] * v[5];
  o[6] = Q[Q66] * v[6] + Q[Q67] * v[7];
  o[7] = Q[Q07] * v[0] + Q[Q17] * v[1] + Q[Q27] * v[2] + Q[Q37] * v[3] + Q[Q67] * v[6] + Q[Q77] * v[7];
  o[8] = Q[Q88] * v[8];
}

// stage-Jacobian element (k, r, c): the LDS array, or the global workspace through a buffer
// resource (GBuf: one offset VGPR per access, bounds-checked to the problem's N stages)
// (round 6: the stage offset k * 384 as the loads' SGPR soffset instead, per-lane offsets loop-invariant,
// was 2.8 % slower at N = 60 -- profiles/r06/kin_ab/sqp_ab_soffset_r06j.log)
template <int N, bool JG>
__device__ __forceinline__ double st_jld(StJP<N, JG> J, int k, int r, int c) {
  if constexpr (JG) return GBuf(J, N * 384).ld((uint32_t)(((k * 6 + r) * 8 + c) * 8));
  else return J[k].m[r][c];
}
template <int N, bool JG>
__device__ __forceinline__ void st_jst(StJP<N, JG> J, int k, int r, int c, double v) {
  if constexpr (JG) GBuf(J, N * 384).st((uint32_t)(((k * 6 + r) * 8 + c) * 8), v);
  else J[k].m[r][c] = v;
}
// columns c, c + 1 (c even) of one row: global J as one 16-byte store
template <int N, bool JG>
__device__ __forceinline__ void st_jst2(StJP<N, JG> J, int k, int r, int c, double v0, double v1) {
  if constexpr (JG) GBuf(J, N * 384).st2((uint32_t)(((k * 6 + r) * 8 + c) * 8), v0, v1);
  else {
    J[k].m[r][c] = v0;
    J[k].m[r][c + 1] = v1;
  }
}
#define JLD(k, r, c) st_jld<N, JG>(J, (k), (r), (c))
#define JST(k, r, c, v) st_jst<N, JG>(J, (k), (r), (c), (v))
#define JST2(k, r, c, v0, v1) st_jst2<N, JG>(J, (k), (r), (c), (v0), (v1))

template <int N, bool JG>
__device__ __forceinline__ StJP<N, JG> st_jac(StSmem<N, JG>& s, const StSqpArgs& A, int b) {
  if constexpr (JG) return GBuf::uniform(A.jws + (size_t)b * N * 48);
  else return s.J;
}

template <int N, int TYRE, bool JG>
__global__ __launch_bounds__(WTH) void st_sqp_kernel(StSqpArgs A) {
  static_assert(N >= 2 && N <= WTH, "one lane per stage");
  // occupancy guard (rocprofv3 LDS_Block_Size: 53,248 B ran three one-wave workgroups per CU,
  // 54,272 B two; four need <= 40,960 B)
  // (the kernel holds ~450 VGPRs + AGPRs: one wave per SIMD, so four workgroups per CU is the ceiling)
  static_assert(!JG || sizeof(StSmem<N, JG>) <= 40960, "global-J st_sqp must fit four workgroups per CU");
  static_assert(JG || N != 60 || sizeof(StSmem<N, JG>) <= 53248, "LDS-J st_sqp<60> must fit three workgroups per CU");
  __shared__ StSmem<N, JG> s;
  const int l = threadIdx.x;
  const int b = xcd_problem(blockIdx.x, A.B);
  DynCoef<double> c = A.car;
  c.tyre = TYRE;
  const vc_dyn_mpc& W = A.w;
  const double S = W.fx_scale;
  const bool stl = l < N;
  const int k = stl ? l : 0;  // this lane's stage

  for (int i = l; i < N; i += WTH) {
    s.kap[i] = A.kappa[(size_t)b * N + i];
    s.dsv[i] = A.ds[(size_t)b * N + i];
    s.ub[i][0] = A.ubar[((size_t)b * N + i) * 2];
    s.ub[i][1] = A.ubar[((size_t)b * N + i) * 2 + 1];
  }
  if (l < 8) s.xs.at(0, l) = A.x0[(size_t)b * 8 + l];
  if (l == 0) s.flag[0] = VC_SOLVED;
#ifdef VC_TIMING
  uint64_t tacc[ST_NSLOT] = {};
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
  WSYNC();

  // Riccati lane roles (fixed per lane): H entry (hi, hj), hi <= hj, for lanes < 45
  int hi = 0, hj = 0;
  {
    int q = l < 45 ? l : 0, i = 0;
    while (q >= 9 - i) { q -= 9 - i; ++i; }
    hi = i;
    hj = i + q;
  }
  // P entry (pi, pj) for lanes < 28
  int pi = 0, pj = 0;
  {
    int q = l < 28 ? l : 0, i = 0;
    while (q >= 7 - i) { q -= 7 - i; ++i; }
    pi = i;
    pj = i + q;
  }

  int it_total = 0, it_max = 0;
  bool all_conv = true, any_fail = false, stopped = false;  // stopped: a later QP ended the SQP early
  bool all_pol = true;  // every converged QP's answer certified by the active-set polish
  double last_res = 0.0, last_mu = 0.0;
  const double tol_r = 1e-10, tol_mu = 1e-13;

  // SQP update state: a step under test (tries > 0) is ub = u + 2^-(tries-1) du, the last try
  // the unchanged iterate (oracle/dyn_sqp.py domain_step)
  // (the iterate uo in u.q.g[k][0..1], the scaled step in u.q.g[k][2..3], untouched by the rollout)
  int tries = 0, sq = 0;
  bool first = true, test = false;  // test: the iterate's own rollout is inside the domain
  const int l_out = l, k_out = k, hi_out = hi, hj_out = hj, pi_out = pi, pj_out = pj;
  for (;;) {
    // The lane coordinates, lane roles and the kernel-argument pointer are re-laundered every
    // SQP iteration: whatever the body derives from them (lane masks, scaled weights, ...) is
    // then recomputed inside the loop instead of being hoisted out of it and held -- spilled --
    // across the linearisation (528 B/lane of scratch for the Fiala tyre before).
    int l = l_out, k = k_out, hi = hi_out, hj = hj_out, pi = pi_out, pj = pj_out;
    asm volatile("" : "+v"(l), "+v"(k), "+v"(hi), "+v"(hj), "+v"(pi), "+v"(pj));
    const bool stl = l < N;
    const int hslot = qslot(hi, hj), hci = vcol(hi), hcj = vcol(hj);
    const StSqpArgs* Ap = (const StSqpArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(Ap));
    const StSqpArgs& A = *Ap;
    const vc_dyn_mpc& W = A.w;
    DynCoef<double> c = A.car;
    c.tyre = TYRE;
    const StJP<N, JG> J = st_jac<N, JG>(s, A, b);
    // ---------------- predict: xs = rollout(ubar) ----------------
    // Serial: lane 0 walks the stages (RK4, algebraic tan-alpha form).  After a QP step
    // (tries == 1, from the second QP step, linear tyre) the new rollout is found instead by chord-Newton
    // sweeps from the pre-step trajectory, whose Jacobians A_k are still in s.J: every lane
    // evaluates its own stage, F(x_k, u_k) -> defect c_k = F_y - y_{k+1} (6 lateral/longitudinal
    // states; s and t do not enter F and are prefix sums of their increments), then lanes 0..5
    // sweep delta_{k+1} = c_k + A_k delta_k, y_{k+1} += delta_{k+1}.  Accepted when every defect is
    // below kStNewtonTol (1 + |y|): the serial rollout's trajectory up to those defects carried
    // through the dynamics (measured <= 3e-10 relative at 1e-13, tests/test_gpu_st_sqp.py), at the
    // cost of one RK4 step per sweep instead of N - 1; otherwise (not converged in kStNewtonMax sweeps,
    // non-finite) the serial rollout runs.  The chord iteration converges linearly at a rate set by
    // the step's size (scripts/newton_rollout_study.py: 3-10 sweeps for the linear tyre's SQP
    // steps; the Fiala tyre's saturation often needs more, so it keeps the serial rollout).
    // One RK4 call site for both modes (a second one makes the compiler outline it and spill).
    // flag[1]: finite, flag[2]: inside the spatial model's domain (Ux > 0, s' > 0)
    ST_STAMP(t_p0)
    {
      bool newton = TYRE == VC_TYRE_LINEAR && tries == 1 && sq >= 1;  // from the second QP step on
      if (newton) {  // uniform: only where the RK4 step's lateral mode is stable along the pre-step plan
        const double ux = stl ? s.xs.at(k, 0) : 1e300;
        newton = wmin(ux) >= kStNewtonUxMin;
      }
      double* scr = &s.u.l.trow[0][0];  // defects / increments [N-1][8]: dead between the IPM and the linearisation
      for (int nit = 0;; ++nit) {
        double x[8];
        bool fin = true, dom = true;
        double err = 0.0;
        const bool act = newton ? (l < N - 1) : (l == 0);
        const int kk0 = newton ? (l < N - 1 ? l : 0) : 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = s.xs.at(kk0, i);
        if (!newton) dom = dyn_in_domain(x, s.kap[0]);
        const int nsteps = newton ? 1 : N - 1;
        if (act) {
          for (int st = 0; st < nsteps; ++st) {
            const int kk = newton ? kk0 : st;
            const double u2[2] = {s.ub[kk][0], s.ub[kk][1]};
            const double kp = s.kap[kk];
            double xn[8];
            const double th = dyn_fx_split(u2[0]);  // one tanh per step, not per evaluation
            rk4_apply<double, 8>(x, s.dsv[kk], [&](const double* xx, double* f) { dyn_spatial_ode_alg_th<double, double>(xx, u2, th, kp, c, f); }, xn);
            if (newton) {
              constexpr int yr[6] = {0, 1, 2, 3, 5, 6};
#pragma unroll
              for (int r = 0; r < 6; ++r) {
                const double yn = s.xs.at(kk + 1, yr[r]);
                const double cd = xn[yr[r]] - yn;
                scr[kk * 8 + r] = cd;
                err = fmax(err, fabs(cd) / (1.0 + fabs(yn)));
              }
              scr[kk * 8 + 6] = xn[4] - x[4];
              scr[kk * 8 + 7] = xn[7] - x[7];
#pragma unroll
              for (int i = 0; i < 8; ++i) fin = fin && isfinite(xn[i]);
            } else {
#pragma unroll
              for (int i = 0; i < 8; ++i) {
                x[i] = xn[i];
                s.xs.at(kk + 1, i) = xn[i];
                fin = fin && isfinite(xn[i]);
              }
              dom = dom && dyn_in_domain(x, s.kap[kk + 1]);
            }
          }
        }
        if (!newton) {
          if (l == 0) {
            s.flag[1] = fin ? 1 : 0;
            s.flag[2] = (fin && dom) ? 1 : 0;
            if (first && !fin) s.flag[0] = VC_NONFINITE;
          }
          break;
        }
        WSYNC();
        const bool allfin = __all(fin ? 1 : 0) != 0;
        err = wmax(err);
        if (allfin && err <= kStNewtonTol) {
          // converged: s and t as prefix sums of the stage increments, domain test in parallel
          if (l == 0) {
            double sv = s.xs.at(0, 4), tv = s.xs.at(0, 7);
            for (int kk = 0; kk < N - 1; ++kk) {
              sv += scr[kk * 8 + 6];
              tv += scr[kk * 8 + 7];
              s.xs.at(kk + 1, 4) = sv;
              s.xs.at(kk + 1, 7) = tv;
            }
          }
          WSYNC();
          bool ok = true, fn = true;
          if (l < N) {
            double xk[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              xk[i] = s.xs.at(l, i);
              fn = fn && isfinite(xk[i]);
            }
            ok = fn && dyn_in_domain(xk, s.kap[l]);
          }
          const bool allf = __all(fn ? 1 : 0) != 0, allok = __all(ok ? 1 : 0) != 0;
          if (l == 0) {
            s.flag[1] = allf ? 1 : 0;
            s.flag[2] = (allf && allok) ? 1 : 0;
          }
          break;
        }
        if (!allfin || nit + 1 >= kStNewtonMax) {
          newton = false;  // the serial rollout (from state 0, which the sweeps never change)
          continue;
        }
        // chord sweep over the stages, lanes 0..5 own the six y-components of delta
        {
          constexpr int yr[6] = {0, 1, 2, 3, 5, 6};
          const int r = l < 6 ? l : 0;
          // rows kk + 1 (LDS) or kk + 1, kk + 2 (global J) loaded ahead of use
          constexpr int AH = 1;
          double d = 0.0, jn[AH][6];
#pragma unroll
          for (int a = 0; a < AH; ++a)
#pragma unroll
            for (int cc = 0; cc < 6; ++cc) jn[a][cc] = JLD(a < N - 2 ? a : N - 2, r, cc);
          for (int kk = 0; kk < N - 1; ++kk) {
            double jc[6];
#pragma unroll
            for (int cc = 0; cc < 6; ++cc) jc[cc] = jn[0][cc];
#pragma unroll
            for (int a = 0; a + 1 < AH; ++a)
#pragma unroll
              for (int cc = 0; cc < 6; ++cc) jn[a][cc] = jn[a + 1][cc];
            const int kn = kk + AH < N - 1 ? kk + AH : N - 2;
#pragma unroll
            for (int cc = 0; cc < 6; ++cc) jn[AH - 1][cc] = JLD(kn, r, cc);
            double acc = scr[kk * 8 + r];
#pragma unroll
            for (int cc = 0; cc < 6; ++cc) acc += jc[cc] * bcast(d, cc);
            d = acc;
            if (l < 6) s.xs.at(kk + 1, yr[r]) += d;
          }
        }
        WSYNC();
      }
    }
    WSYNC();
    ST_ACC(ST_PRED, t_p0)
    first = false;
    if (tries > 0) {
      // ---------------- SQP update: the step's rollout left the domain? ----------------
      // alpha = the first of 1, 1/2, ... whose rollout stays in the model's domain, 0 if none
      // (IPOPT cuts its step back alike on evaluation errors)
      if (test && s.flag[2] == 0 && tries <= DOM_HALVINGS) {
        const double a = tries < DOM_HALVINGS ? ldexp(1.0, -tries) : 0.0;
        if (stl) {
          const double uF = s.u.q.g[k][0], uW = s.u.q.g[k][1];  // uo: the pre-step iterate
          const double d0 = s.u.q.g[k][2], d1 = s.u.q.g[k][3];
          s.ub[k][0] = a > 0.0 ? uF + a * (d0 * S) : uF;
          s.ub[k][1] = a > 0.0 ? fmin(fmax(uW + a * d1, W.w_min), W.w_max) : uW;
        }
        ++tries;
        WSYNC();
        continue;
      }
      tries = 0;
      ++sq;
    }
    if (sq == W.sqp_iters || s.flag[0] == VC_NONFINITE) break;

    // ---------------- linearize + stage functions ----------------
    ST_STAMP(t_l0)
    {
      constexpr int NLIN = 4 * (N - 1), NTASK = NLIN + 5 * N;
      using D2 = Dual<2, double>;
      using D1 = Dual<1, double>;
#pragma unroll 1
      for (int task = l; task < NTASK; task += WTH) {
        if (task < NLIN) {
          const int kk = task >> 2, pr = task & 3;
          // seed pairs: (Ux, Uy), (r, delta), (ey, epsi), (Fx, w)
          const int a0 = pr == 0 ? 0 : (pr == 1 ? 2 : (pr == 2 ? 5 : -1));
          const int a1 = pr == 0 ? 1 : (pr == 1 ? 3 : (pr == 2 ? 6 : -1));
          D2 x[8], u2[2], xn[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            x[i] = D2(s.xs.at(kk, i));
            x[i].d[0] = i == a0 ? 1.0 : 0.0;
            x[i].d[1] = i == a1 ? 1.0 : 0.0;
          }
          u2[0] = D2(s.ub[kk][0]);
          u2[1] = D2(s.ub[kk][1]);
          u2[0].d[0] = pr == 3 ? 1.0 : 0.0;
          u2[1].d[1] = pr == 3 ? 1.0 : 0.0;
          const D2 kp(s.kap[kk]);
          const D2 th = dyn_fx_split(u2[0]);
          rk4_apply<D2, 8>(x, D2(s.dsv[kk]), [&](const D2* xx, D2* f) { dyn_spatial_ode_alg_th<D2, double>(xx, u2, th, kp, c, f); }, xn);
          // columns of [A6 | B6] (y index of the seeds) and the t-row; the four tasks of a stage
          // are adjacent lanes, so each row store covers the stage's whole 64-byte row (global J)
          const int c0 = pr < 3 ? 2 * pr : 6, c1 = c0 + 1;
          const double s0 = pr == 3 ? S : 1.0;
          const int yr[6] = {0, 1, 2, 3, 5, 6};
#pragma unroll
          for (int r = 0; r < 6; ++r) JST2(kk, r, c0, xn[yr[r]].d[0] * s0, xn[yr[r]].d[1]);
          s.u.l.trow[kk][tsw(kk, c0)] = xn[7].d[0] * s0;
          s.u.l.trow[kk][tsw(kk, c1)] = xn[7].d[1];
        } else {
          const int q = task - NLIN, kk = q / 5, j = q % 5;
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
    }
    if constexpr (JG) {
      // the stage Jacobians went to global memory: visible to every lane before the passes read them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    WSYNC();
    ST_ACC(ST_LIN, t_l0)
    ST_STAMP(t_s0)

    // ---------------- stage QP data (lane k, registers) ----------------
    double Qc[NQ], qc[9];
    Rows R;
#pragma unroll
    for (int e = 0; e < NQ; ++e) Qc[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) qc[e] = 0.0;
    {
      const double ds = s.dsv[k];
      const double ey = s.xs.at(k, 5);
      // boundary + deviation (cascaded_mpc.py:139-151), obstacle barrier (:173-176) in ey
      const double cdev = W.w_dev * ds;
      const double blo = ey < W.ey_min ? W.w_b * ds : 0.0, bhi = ey > W.ey_max ? W.w_b * ds : 0.0;
      Qc[Q44] += 2.0 * (cdev + blo + bhi);
      qc[4] += 2.0 * (cdev * ey + blo * (ey - W.ey_min) + bhi * (ey - W.ey_max));
      if (A.obs.n > 0) {
        double po, qo;
        obstacle_ey_model<double>(A.obs, s.xs.at(k, 4), ey, W.w_obs * ds, po, qo);
        Qc[Q44] += qo;
        qc[4] += po;
      }
      // w^2 (:153), prox on the scaled step
      Qc[Q88] += 2.0 * W.w_w + 2.0 * A.qp.prox;
      qc[8] += 2.0 * W.w_w * s.ub[k][1];
      Qc[Q77] += 2.0 * A.qp.prox;
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
      // Fx slew with the previous stage (:167-171): c (dFx_k - p_k + (Fx_k - Fx_{k-1}) / S)^2 S^2
      if (k >= 1) {
        const double cs = 2.0 * W.w_Fx / s.dsv[k - 1] * S * S;
        const double r0 = (s.ub[k][0] - s.ub[k - 1][0]) / S;
        Qc[Q66] += cs;
        Qc[Q67] -= cs;
        Qc[Q77] += cs;
        qc[6] -= cs * r0;
        qc[7] += cs * r0;
      }
      // w_time t_{N-1} = sum_k t-row_k . (y_k, u_k): linear stage terms (:292)
      if (k < N - 1) {
        constexpr int iy[8] = {0, 1, 2, 3, 4, 5, 7, 8};
#pragma unroll
        for (int a = 0; a < 8; ++a) qc[iy[a]] += W.w_time * s.u.l.trow[k][tsw(k, a)];
      }
      // terminal (:290-303)
      if (k == N - 1) {
        const double Ux = s.xs.at(k, 0);
        if (Ux >= W.max_speed) {
          Qc[Q00] += 2.0 * W.w_speed;
          qc[0] += 2.0 * W.w_speed * (Ux - W.max_speed);
        }
        Qc[Q44] += 2.0 * W.w_ey;
        qc[4] += 2.0 * W.w_ey * ey;
        Qc[Q55] += 2.0 * W.w_epsi;
        qc[5] += 2.0 * W.w_epsi * s.xs.at(k, 6);
      }
      // rows (:101-128, trust region)
      const double mk = (stl && k >= 1) ? 1.0 : 0.0;
      R.d[0] = s.xs.at(k, 0) - W.Ux_min;
      R.d[1] = W.delta_max - s.xs.at(k, 3);
      R.d[2] = s.xs.at(k, 3) - W.delta_min;
      R.m[0] = R.m[1] = R.m[2] = mk;
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        const int fn = 2 + r;
#pragma unroll
        for (int a = 0; a < 4; ++a) R.c[r][a] = s.u.l.st[k][stx(k, fn, 1 + a)] / S;
        R.c[r][4] = s.u.l.st[k][stx(k, fn, 5)];
        R.d[3 + r] = -s.u.l.st[k][stx(k, fn, 0)] / S;
        R.m[3 + r] = stl ? 1.0 : 0.0;
      }
      const double wv = s.ub[k][1];
      double up = W.w_max - wv, dn = wv - W.w_min;
      if (A.qp.trust_w > 0) {
        up = fmin(up, A.qp.trust_w);
        dn = fmin(dn, A.qp.trust_w);
      }
      R.d[8] = up;
      R.d[9] = dn;
      R.m[8] = R.m[9] = stl ? 1.0 : 0.0;
      R.d[10] = R.d[11] = W.trust_Fx / S;
      R.m[10] = R.m[11] = (stl && W.trust_Fx > 0) ? 1.0 : 0.0;
#pragma unroll
      for (int i = 0; i < NR; ++i)
        if (R.m[i] == 0.0) R.d[i] = 1.0;
    }
    double sl[NR], la[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      sl[i] = R.m[i] > 0.0 ? fmax(R.d[i], 1.0) : 1.0;
      la[i] = R.m[i];
    }
    double mc = 0.0;
#pragma unroll
    for (int i = 0; i < NR; ++i) mc += R.m[i];
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
    ST_ACC(ST_SETUP, t_s0)

    // ---- LQ machinery -----------------------------------------------------------------
    // Every stage loop below is branch-free in its lanes (clamped addresses, 0/1 masks) and
    // loads the next stage's operands before the current stage's dependent chain, so LDS
    // latency stays off the recursion; cross-lane values move by v_readlane.
    //
    // Riccati factorisation of the stage Hessians s.u.q.Qt (backward): K, Hi per stage.
    //   T = P [A6 B6 ; 0 e_Fx]      lanes 0..55  (a, j) = (l / 8, l % 8)
    //   H = Qt + [..]' T            lanes 0..44  (hi, hj)
    //   P' = Hxx - Hux' Huu^-1 Hux  lanes 0..27, K = -Huu^-1 Hux lanes 28..41, Huu^-1 lane 42
    const int ta = l < 56 ? (l >> 3) : 0, tj = l & 7;
    const double tpm = tj == 6 ? 1.0 : 0.0;
    const int hcic = hci < 0 ? 0 : hci, hcjc = hcj < 0 ? 0 : hcj;
    const double hdyn = (l < 45 && hci >= 0 && hcj >= 0) ? 1.0 : 0.0, hpm = hci == 6 ? 1.0 : 0.0;
    const int hsc = hslot < 0 ? 0 : hslot;
    const double hq = (l < 45 && hslot >= 0) ? 1.0 : 0.0;
    // The stage loops are unrolled by two with ping-pong operand buffers (A for kk, B for
    // the next stage): no register rotation at the loop latch, so the next stage's loads
    // stay in flight across the current stage's chain.
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
      if (kk < N - 1) {  // uniform
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
      // 1 / det: v_rcp_f64 + two Newton steps (full fp64 accuracy, no IEEE divide sequence)
      // reciprocal bit-identical to IEEE 1/x on every class (asserted: tests/test_gpu_numerics.py): the plain v_rcp_f64 + Newton form turns
      // det = +inf (h00 h11 overflowing at barrier weights ~1e154) into NaN where 1/det = 0
      const double id = rcp_nr(det);
      const double i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
      {
        // lanes 0..27: P entry (pi, pj); lanes 28..41: K entry; lane 42: Huu^-1
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
    // Riccati factorisation of the stage Hessians s.u.q.Qt (backward): K, Hi per stage.
    auto factor = [&]() -> bool {
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

    // Sweep lanes 0..8 own the stage-vector components v = (y0..y5, p, dFx, dw).
    const int sl9 = l < 9 ? l : 8;
    const int scol = vcol(sl9) < 0 ? 0 : vcol(sl9);                 // column of [A6 | B6]
    const double smsk = (l < 9 && vcol(sl9) >= 0) ? 1.0 : 0.0;      // p (l = 6) has no dynamics column
    const double spm = (l < 9 && vcol(sl9) == 6) ? 1.0 : 0.0;       // dFx picks up the p costate
    // backward pass extras: lanes 0..6 read K[kk][0][l], K[kk][1][l]; lanes 7, 8 read the
    // Huu^-1 pair of their kk component -> one formula t = a gu0 + b gu1 for both
    const int bl7 = l < 7 ? l : 0;
    // forward pass: lanes 0..5 read J row l; lanes 7, 8 read K row (l - 7) and kk
    const int fr = l < 6 ? l : 0, fc = l == 8 ? 1 : 0;
    const bool fk = l == 7 || l == 8;

    struct BwdOps {
      double J6[6], h, a, b;
    };
    // vec: s.u.q.g, the right-hand side h (solve) or the gradient gr (dual residual)
    auto bwd_load = [&](int kk, const double (*vec)[9], BwdOps& o) {
#pragma unroll
      for (int e = 0; e < 6; ++e) o.J6[e] = JLD(kk, e, scol);
      o.h = vec[kk][sl9];
      // lane-selected addresses, one unconditional load each (a value select would make
      // the compiler predicate the loads and wait on the whole prefetch)
      const double* pa = l < 7 ? &s.u.q.K[kk][0][bl7] : &s.u.q.Hi[kk][l == 7 ? 0 : 1];
      const double* pb = l < 7 ? &s.u.q.K[kk][1][bl7] : &s.u.q.Hi[kk][l == 7 ? 1 : 2];
      o.a = *pa;
      o.b = *pb;
    };
    // g = vec_k + [A6 | B6 ; 0 e_Fx]' p_{k+1} on lanes 0..8
    auto bwd_g = [&](int kk, const BwdOps& o, double pv) -> double {
      double g = o.h;
      if (kk < N - 1) {  // uniform
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
    // one forward stage: writes dv[kk], returns xt_{k+1} (lanes 0..6)
    auto fwd_stage = [&](int kk, const FwdOps& o, double X) -> double {
      double xb[7];
#pragma unroll
      for (int a = 0; a < 7; ++a) xb[a] = bcast(X, a);
      double acc = 0.0;
#pragma unroll
      for (int e = 0; e < 6; ++e) acc += o.w[e] * xb[e];
      const double uk = acc + o.w[6] * xb[6] + o.w[7];  // lanes 7, 8: u_c = K_c xt + kk_c
      const double u0 = bcast(uk, 7), u1 = bcast(uk, 8);
      if (l < 9) s.u.q.g[kk][l] = fk ? uk : X;
      const double xn = acc + o.w[6] * u0 + o.w[7] * u1;  // lanes 0..5
      return l < 6 ? xn : (l == 6 ? u0 : 0.0);
    };

    // LQ solve with linear terms h -> direction dv (backward vector pass with the factor, then
    // the forward rollout u = K xt + kk); both live in s.u.q.g: the forward pass overwrites h
    // once the backward pass is done with it
    auto lq_solve = [&]() {
      BwdOps A1, B1;
      bwd_load(N - 1, s.u.q.g, A1);
      double pv = 0.0;  // lanes 0..6: p_{k+1}
      auto bstage = [&](int kk, const BwdOps& o) {
        const double g = bwd_g(kk, o, pv);
        const double gu0 = bcast(g, 7), gu1 = bcast(g, 8);
        const double t2 = o.a * gu0 + o.b * gu1;
        pv = g + t2;
        if (fk) s.u.q.kk[kk][l - 7] = -t2;
      };
#pragma unroll 1
      for (int kk = N - 1; kk >= 0; kk -= 2) {
        const int k1 = kk >= 1 ? kk - 1 : 0, k2 = kk >= 2 ? kk - 2 : 0;
        bwd_load(k1, s.u.q.g, B1);
        bstage(kk, A1);
        if (kk >= 1) {
          bwd_load(k2, s.u.q.g, A1);
          bstage(kk - 1, B1);
        }
      }
      WSYNC();
      double X = 0.0;  // lanes 0..6: xt_k
      FwdOps A2, B2;
      fwd_load(0, A2);
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
      WSYNC();
    };

    // condensed dual residual max |d/du (sum_k gr_k . v_k)| through the dynamics (adjoint sweep).
    // cl: through the closed-loop dynamics A + B K of the last Riccati factorisation, i.e. the
    // gradient over v in u = K x + v -- zero exactly where the open-loop one is (an invertible
    // change of the input variables), but without the open-loop sweep's growth: at low speed the
    // reference's RK4 step (mpc_dt 0.03 s) is unstable in the lateral mode (|eig A_k| 3-5 at
    // Ux = 4 m/s, Fx = 0), so over 60 stages the open-loop adjoint amplifies rounding by ~1e30 and
    // the interior point never meets its tolerance once anything excites that mode (an obstacle's
    // barrier gradient: scripts/st_obs_shoe_diag.py, the N = 60 obstacle runs of test_gpu_bands).
    auto dual_residual = [&](bool cl) -> double {
      BwdOps A3, B3;
      bwd_load(N - 1, s.u.q.g, A3);
      double rho = 0.0, rmax = 0.0;
      auto rstage = [&](int kk, const BwdOps& o) {
        const double g = bwd_g(kk, o, rho);
        rmax = fk ? fmax(rmax, fabs(g)) : rmax;
        // lanes 0..6: + K' g_u (the lq_solve backward pass's pv); lanes 7, 8 are not read on
        rho = cl ? g + o.a * bcast(g, 7) + o.b * bcast(g, 8) : g;
      };
#pragma unroll 1
      for (int kk = N - 1; kk >= 0; kk -= 2) {
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
    for (; it < A.qp.max_iter; ++it) {
      // (a) residuals, stage gradients, barrier-augmented stage Hessians
      ST_STAMP(t_r0)
      double rp[NR], wg[NR], grk[9], val[NR];
      double rpm = 0.0, mus = 0.0;
      row_values(R, vk, val);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        rp[i] = R.m[i] * (val[i] + sl[i] - R.d[i]);
        wg[i] = R.m[i] * la[i] / sl[i];
        rpm = fmax(rpm, fabs(rp[i]));
        mus += R.m[i] * sl[i] * la[i];
      }
      qmul(Qc, vk, grk);
#pragma unroll
      for (int e = 0; e < 9; ++e) grk[e] += qc[e];
      {
        double ml[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) ml[i] = R.m[i] * la[i];
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
      ST_ACC(ST_RESID, t_r0)
      ST_STAMP(t_d0)
      const bool carried = have_rd;
      double rdm = carried ? rd_carry : dual_residual(kvalid);
      bool rd_cl = carried || kvalid;
      ST_ACC(ST_DUAL, t_d0)
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

      // (b) Riccati factorisation of H + C'WC
      ST_STAMP(t_f0)
      const bool fok = factor();
      kvalid = kvalid || fok;
      ST_ACC(ST_FACT, t_f0)
      if (!fok) {
        // the barrier-augmented recursion lost definiteness at the numerical floor (weights
        // ~1e13, cancellation in P = Hxx - Hxu Huu^-1 Hux): a near-converged iterate stands
        if (mu <= 1e2 * tol_mu && last_res <= 1e3 * rtol) conv = true;
        else fail = true;
        break;
      }

      // (c) predictor: h = gr + C'(W rp - lam)
      auto set_h = [&](const double* rc_over_s) {
        if (stl) {
          double y[NR], hk[9];
#pragma unroll
          for (int i = 0; i < NR; ++i) y[i] = R.m[i] * (wg[i] * rp[i] - rc_over_s[i]);
#pragma unroll
          for (int e = 0; e < 9; ++e) hk[e] = grk[e];
          row_adjoint(R, y, hk);
#pragma unroll
          for (int e = 0; e < 9; ++e) s.u.q.g[k][e] = hk[e];
        }
        WSYNC();
      };
      ST_STAMP(t_q0)
      set_h(la);
      ST_ACC(ST_STEP, t_q0)
      ST_STAMP(t_q1)
      lq_solve();
      ST_ACC(ST_SOLVE, t_q1)
      ST_STAMP(t_q2)
      double dsa[NR], dla[NR], cdv[NR], dvk[9];
      double amin = 1.0;
#pragma unroll
      for (int e = 0; e < 9; ++e) dvk[e] = s.u.q.g[k][e];
      row_values(R, dvk, cdv);
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        dsa[i] = R.m[i] * (-rp[i] - cdv[i]);
        dla[i] = R.m[i] * (wg[i] * (cdv[i] + rp[i]) - la[i]);
        if (stl && R.m[i] > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
      }
      amin = wmin(amin);
      double ms = 0.0;
      if (stl) {
#pragma unroll
        for (int i = 0; i < NR; ++i) ms += R.m[i] * (sl[i] + amin * dsa[i]) * (la[i] + amin * dla[i]);
      }
      ms = wsum(ms) / mcount;
      const double ratio = mu > 0.0 ? fmin(1.0, ms / mu) : 0.0;
      const double smu = ratio * ratio * ratio * mu;

      // (d) corrector: rc = s lam + ds_a dl_a - sigma mu
      double rcs[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) rcs[i] = R.m[i] * (sl[i] * la[i] + dsa[i] * dla[i] - smu) / sl[i];
      set_h(rcs);
      ST_ACC(ST_STEP, t_q2)
      ST_STAMP(t_q3)
      lq_solve();
      ST_ACC(ST_SOLVE, t_q3)
      ST_STAMP(t_q4)
#pragma unroll
      for (int e = 0; e < 9; ++e) dvk[e] = s.u.q.g[k][e];
      row_values(R, dvk, cdv);
      amin = 1.0;
#pragma unroll
      for (int i = 0; i < NR; ++i) {
        dsa[i] = R.m[i] * (-rp[i] - cdv[i]);
        dla[i] = R.m[i] * (wg[i] * (cdv[i] + rp[i]) - rcs[i]);
        if (stl && R.m[i] > 0.0) amin = fmin(amin, fmin(step_to_bound(sl[i], dsa[i]), step_to_bound(la[i], dla[i])));
      }
      const double alpha = fmin(1.0, 0.99 * wmin(amin));
      rd_carry = (1.0 - alpha) * rdm;
      have_rd = rd_cl;  // only closed-loop values are carried
      if (stl) {
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          if (R.m[i] > 0.0) {
            sl[i] = fmax(sl[i] + alpha * dsa[i], 1e-300);
            la[i] = fmax(la[i] + alpha * dla[i], 1e-300);
          }
        }
#pragma unroll
        for (int e = 0; e < 9; ++e) vk[e] += alpha * dvk[e];
      }
      WSYNC();
      ST_ACC(ST_STEP, t_q4)
    }
    it_total += it;
    it_max = max(it_max, it);

    // ---------------- active-set polish (round 5) ----------------
    // The interior point stops at mu <= 1e-13 with a floor acceptance near the end, and its
    // iterate is then as far from the QP's optimum as its weakly active rows allow: up to 1e-6 in
    // the scaled units on the bench's C3 / N = 60 batches, i.e. 1e-3 N (tests/test_gpu_certify.py,
    // every QP of every problem against the oracle-built QP).  The polish solves the QP on the
    // active set the interior point identified (lambda > s) exactly: an augmented Lagrangian
    // (Q + sum_A rho_i c_i c_i', one Riccati factorisation) whose passes are Newton steps from the
    // current point -- the gradient Q v + q + sum_A c_i (lm_i + rho_i (c_i v - d_i)) is recomputed
    // stage-locally each pass, so the factor's rounding is refined away instead of entering the
    // answer -- with multiplier updates lm_i += rho_i (c_i v - d_i) until the active rows hold.
    // Certified when the inactive rows are feasible and the active multipliers nonnegative;
    // otherwise the violated rows join and the negative ones leave (kStPolish rounds), and an
    // uncertified polish keeps the interior point's iterate.
    bool pol_qp = false;
    if (kStPolish > 0 && conv) {
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
      const double rho_h = kStAlRho * hs;
      auto rho = [&](int i) -> double {
        double cn2 = 1.0;
        if (i >= 3 && i < 8) {
          cn2 = 0.0;
#pragma unroll
          for (int a = 0; a < 5; ++a) cn2 += R.c[i - 3][a] * R.c[i - 3][a];
        }
        return rho_h / fmax(cn2, 1e-30);
      };
      bool act[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) act[i] = stl && R.m[i] > 0.0 && la[i] > sl[i];
#pragma unroll 1
      for (int round = 0; round < kStPolish; ++round) {
        // the interior point's slacks / multipliers are dead from here: sl holds the polish's
        // iterate and la its multipliers (a later round starts from the last round's)
        double w[NR], val[NR] = {};
        double* const lm = la;
        double* const vp = sl;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          w[i] = act[i] ? rho(i) : 0.0;
          lm[i] = act[i] ? lm[i] : 0.0;
        }
        if (stl) put_qt(w);
        WSYNC();
        if (!factor()) break;  // keep the interior point's iterate
#pragma unroll
        for (int e = 0; e < 9; ++e) vp[e] = vk[e];
        bool al_conv = false;
        int held = 0;
#pragma unroll 1
        for (int p = 0; p < kStAlPasses; ++p) {
          if (stl) {
            double g9[9], y[NR];
            row_values(R, vp, val);
#pragma unroll
            for (int i = 0; i < NR; ++i) y[i] = act[i] ? lm[i] + rho(i) * (val[i] - R.d[i]) : 0.0;
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
              const double r = act[i] ? val[i] - R.d[i] : 0.0;
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
        bool viol[NR], neg[NR], bad = false;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
          viol[i] = stl && R.m[i] > 0.0 && !act[i] && val[i] - R.d[i] > kStCertPtol * qs;
          neg[i] = act[i] && lm[i] < -kStCertDtol * qs;
          bad = bad || viol[i] || neg[i];
        }
        if (al_conv && __all(bad ? 0 : 1) != 0) {
          if (stl) {
#pragma unroll
            for (int e = 0; e < 9; ++e) vk[e] = vp[e];
          }
          pol_qp = true;
          break;
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) act[i] = (act[i] || viol[i]) && !neg[i];
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

    // ---------------- SQP update: ubar += dz, tested by the next rollout ----------------
    // w is projected onto its box: exact at a converged QP (|violation| <= tol_r), and it
    // keeps a non-converged iterate (infeasible-start interior point) from leaving it
    if (stl) {
      const double uF = s.ub[k][0], uW = s.ub[k][1];
      s.u.q.g[k][0] = uF;
      s.u.q.g[k][1] = uW;
      s.u.q.g[k][2] = vk[7];
      s.u.q.g[k][3] = vk[8];
      s.ub[k][0] = uF + vk[7] * S;
      s.ub[k][1] = fmin(fmax(uW + vk[8], W.w_min), W.w_max);
    }
    test = s.flag[2] != 0;  // from an iterate outside the domain: the full step, untested
    tries = 1;
    WSYNC();
  }

  // ---------------- outputs: u*, x* = rollout(u*), u0, status ----------------
  bool finite = true;
  for (int e = l; e < 2 * N; e += WTH) {
    const double v = s.ub[e >> 1][e & 1];
    finite = finite && isfinite(v);
    A.u_out[(size_t)b * 2 * N + e] = v;
  }
  for (int e = l; e < 8 * N; e += WTH) {
    const double v = s.xs.at(e >> 3, e & 7);
    finite = finite && isfinite(v);
    A.x_out[(size_t)b * 8 * N + e] = v;
  }
  finite = __all(finite ? 1 : 0) != 0;
  if (l < 2) A.u0[(size_t)b * 2 + l] = s.ub[0][l];
  if (l == 0) {
    int32_t st;
    if (!finite || s.flag[0] == VC_NONFINITE) st = VC_NONFINITE;
    else if (s.flag[2] == 0) st = VC_OUT_OF_DOMAIN;  // x* (the last rollout) outside the model's domain
    else if (all_conv) st = VC_SOLVED;
    else st = VC_MAX_ITER;
    A.status[b] = st;
    A.iters[b] = it_total;
    if (A.diag) {
#ifdef VC_TIMING
      constexpr size_t DS = 4 + ST_NSLOT;
      tacc[ST_TOTAL] = __builtin_amdgcn_s_memtime() - t_start;
      for (int i = 0; i < ST_NSLOT; ++i) A.diag[(size_t)b * DS + 4 + i] = double(tacc[i]);
#else
      constexpr size_t DS = 4;
#endif
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
#define VC_ST_HORIZONS(X) X(20) X(30) X(40) X(50) X(60)

bool st_sqp_built(int N) {
  switch (N) {
#define VC_CASE(n) case n:
    VC_ST_HORIZONS(VC_CASE)
#undef VC_CASE
    return true;
    default:
      return false;
  }
}

// J placement per launch (round 5): the LDS-J kernel runs its waves ~10 % faster (no L2 latency in
// the LQ sweeps), the global-J kernel fits more workgroups per CU (N = 50 / 60: four instead of
// three).  A batch the LDS-J kernel holds resident at once (wg_per_cu x CUs problems) takes it; a
// larger one the global-J kernel, which then needs fewer rounds of the machine
// (scripts/st_jg_ab.sh).
template <int N>
bool st_jg_pick(int B) {
  if constexpr (!st_j_global_ok<N>()) return false;
  else return B > wg_per_cu(sizeof(StSmem<N, false>)) * device_cus();
}
// doubles of J workspace per problem a launch of B problems needs: nonzero only where st_jg_pick
// takes the global-J kernel (a large max_batch no longer allocates it for LDS-J launches)
size_t st_sqp_jws_doubles(int N, int B) {
  switch (N) {
#define VC_CASE(n) \
  case n:          \
    return st_jg_pick<n>(B) ? (size_t)n * 48 : 0;
    VC_ST_HORIZONS(VC_CASE)
#undef VC_CASE
    default:
      return 0;
  }
}
template <int N, int TYRE>
void st_launch(const StSqpArgs& a, hipStream_t stream) {
  if constexpr (st_j_global_ok<N>()) {
    if (st_jg_pick<N>(a.B)) {
      hipLaunchKernelGGL((st_sqp_kernel<N, TYRE, true>), dim3(a.B), dim3(WTH), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((st_sqp_kernel<N, TYRE, false>), dim3(a.B), dim3(WTH), 0, stream, a);
}

hipError_t launch_st_sqp(const StSqpArgs& a, int N, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  if (st_sqp_jws_doubles(N, a.B) && !a.jws) return hipErrorInvalidValue;  // the workspace the kernel needs
  const bool lin = a.car.tyre == VC_TYRE_LINEAR;
  switch (N) {
#define VC_CASE(n)                                        \
  case n:                                                \
    if (lin) st_launch<n, VC_TYRE_LINEAR>(a, stream);    \
    else st_launch<n, VC_TYRE_FIALA>(a, stream);         \
    return hipGetLastError();
    VC_ST_HORIZONS(VC_CASE)
#undef VC_CASE
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vc
