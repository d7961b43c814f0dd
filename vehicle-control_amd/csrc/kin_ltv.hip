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
//                sensitivity G during the forward sweep, row j of the normal
//                matrix and of its Cholesky factor (registers Mr), and the two
//                box inequalities of u_j.
//   lane r < NC  owns state-constraint row r: r < N-1 -> v_{r+1} >= v_min,
//                else delta_{r-N+2} in [delta_min, delta_max].
// LDS holds the Hessian H, the constraint rows of G (broadcast reads), the
// packed columns of the Cholesky factor (pivot-column broadcast during the
// factorisation and the transposed solve), and small broadcast vectors:
// 37.8 KB at N = 20, so four problems fit a CU (B = 1024 fills 256 CUs once).  HBM traffic is only the
// compulsory per-problem inputs and outputs (roofline).
//
// Register discipline (checked with `make resources`: no scratch): Mr[n] is the
// only register array in the solver loops and is indexed with compile-time
// indices only (fully unrolled loops); lane-dependent stores are branch-free
// (dummy LDS slots) because divergent ifs inside the unrolled factorisation make
// the register allocator spill; sched_barrier fences bound how far the
// scheduler hoists LDS broadcast reads; LDS is static so every address folds
// into the ds instruction's offset field.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

#ifndef KIN_NU_TOL
#define KIN_NU_TOL 1e-10  // CG also runs until the multiplier step R e is below this x scale (0: off)
#endif
#ifndef KIN_EARLY_F
#define KIN_EARLY_F 100.0  // first polish attempt at this x the interior point's tolerance (0: only at it)
#endif
#ifndef KIN_EARLY_ROUNDS
#define KIN_EARLY_ROUNDS 2  // active-set rounds of that attempt before the interior point resumes
#endif
#ifndef KIN_TAPIA_F
#define KIN_TAPIA_F 1.02  // ratio gap that makes the indicators decisive (else lambda > s)
#endif
#ifndef KIN_DUAL_TOL
// polish: a multiplier of the wrong sign is accepted up to this x scale.  The cost is nearly flat
// along the acceleration directions (curvature 2 prox = 2e-4), so a wrong-signed multiplier
// lam moves the answer by ~lam / 2e-4: at 1e-9 scale (the round-4 value) C4 problem 33696 kept
// a box bound whose multiplier was -2e-7 and landed 4e-4 off the optimum (tests/test_gpu_certify.py)
#define KIN_DUAL_TOL 1e-12
#endif
#ifndef KIN_AL_RHO
#define KIN_AL_RHO 1e1  // polish: augmented-Lagrangian weight of an active row, x max diag(H) / |free part|^2 (1e4 in
                        // round 4: the factored matrix's condition number left C4 problems 6e-6 off the optimum;
                        // 1e1 keeps every C4 problem within 5e-9 at the same cost, profiles/r05/alrho_r05a.log)
#endif
#ifndef KIN_DOT_CH
#define KIN_DOT_CH 8  // terms per chunk of the residual dot products
#endif
#ifndef KIN_UPDATE
#define KIN_UPDATE 1  // polish rounds after the first update the factor by rank one where they can (0: refactor)
#endif
#ifndef KIN_RSQ_HALLEY
#define KIN_RSQ_HALLEY 1  // pivots' 1/sqrt by one third-order step (0: two Newton steps; C2 -0.8 %, C4 -1.2 %)
#endif
#ifndef KIN_STAT_CHECK
#define KIN_STAT_CHECK 0  // 1: the polish certificate also checks the free variables' stationarity (same time,
                          // same certification at the shipped settings: profiles/r06/kin_ab/kin_polish_cert_st1_r06zj.log)
#endif
#ifndef KIN_STEP_F
// interior point: fraction of the step to the boundary.  0.98 costs +0.6 iterations; 0.995 / 0.998 are
// slower at C2 (+7 / +13 %) and expose two C4 problems (c4_shard seed 31: 9204 reported solved from an
// unpolished interior point 3e-5 off, 6021 polish-certified 6.0 off the oracle's optimum along a flat
// direction) that the oracle certificate catches (scripts/kin_hole_diag.py, profiles/r06/kin_ab/*_r06z[ijk].*)
#define KIN_STEP_F 0.99
#endif
#ifndef KIN_SOLVE_CH
#define KIN_SOLVE_CH 8  // backward-sweep steps per prefetched chunk of the triangular solves (divides 2N;
                        // 4 / 10 within noise of 8, as KIN_DOT_CH 4 / 12: profiles/r06/kin_ab/kin_polish_ab_c2_r06zg.log)
#endif
#ifndef KIN_PANEL_CH
#define KIN_PANEL_CH 6  // columns per in-panel update chunk of factor_blocked, loaded one chunk ahead (2 / 4 / 8:
                        // C2 +1.2 / +1.0 / +0.8 %, bit-identical; profiles/r06/kin_ab/kin_polish_ab_c2_r06ze.log)
#endif

namespace vc {
namespace {

// ---- wave-level helpers ----------------------------------------------------
// value of `v` in lane `src` (src wave-uniform)
__device__ __forceinline__ double lane_bcast(double v, int src) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
  return __hiloint2double(hi, lo);
}
// `old` with lane `dst` replaced by the wave-uniform v (v_writelane: no lane-mask compare,
// whose 40 per-sweep SGPR masks the compiler hoists and spills)
__device__ int amdgcn_writelane(int v, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ double lane_put(double old, double v, int dst) {
  const int lo = amdgcn_writelane(__double2loint(v), dst, __double2loint(old));
  const int hi = amdgcn_writelane(__double2hiint(v), dst, __double2hiint(old));
  return __hiloint2double(hi, lo);
}
// v of lane (i - K) within each 16-lane DPP row, `ident` where that leaves the row
template <int K>
__device__ __forceinline__ double dpp_row_shr(double v, double ident) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(ident), __double2loint(v), 0x110 + K, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(ident), __double2hiint(v), 0x110 + K, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// Wave-wide reductions: a DPP prefix within each 16-lane row (VALU latency, no
// LDS round trip), then the four row totals combined from SGPR readlanes.
template <typename Op>
__device__ __forceinline__ double wave_reduce(double v, double ident, Op op) {
  v = op(v, dpp_row_shr<1>(v, ident));
  v = op(v, dpp_row_shr<2>(v, ident));
  v = op(v, dpp_row_shr<4>(v, ident));
  v = op(v, dpp_row_shr<8>(v, ident));
  return op(op(lane_bcast(v, 15), lane_bcast(v, 31)), op(lane_bcast(v, 47), lane_bcast(v, 63)));
}
__device__ __forceinline__ double wave_sum(double v) {
  return wave_reduce(v, 0.0, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wave_max(double v) {
  return wave_reduce(v, -__builtin_inf(), [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wave_min(double v) {
  return wave_reduce(v, __builtin_inf(), [](double a, double b) { return fmin(a, b); });
}
// one-wave workgroup: LDS ordering point.  The LDS operations of one wave execute in issue
// order, so a store followed by another lane's load of the same address needs no wait: only
// the compiler must not move memory operations across this point (a __syncthreads here made
// every column step of the factorisation wait for its own store, s_waitcnt lgkmcnt(0)).
__device__ __forceinline__ void wave_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
// the lane index through an opaque register: LDS addresses derived from it are recomputed
// where they are used instead of being hoisted out of the solver loop (and spilled)
__device__ __forceinline__ int lane_opaque(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}
// compiler-only memory barrier: stops LICM from hoisting the (loop-invariant) LDS
// reads of G / the factor out of the solver loops into thousands of live registers
__device__ __forceinline__ void no_hoist() { asm volatile("" ::: "memory"); }

// LDS pointer the compiler cannot see through: re-derived from an opaque
// register at the point of use, it stops the address arithmetic of the
// (thousands of) constant-address broadcast reads in the unrolled matrix build
// from being hoisted out of the solver loop into live registers, which spills.
using lds_cdouble = const __attribute__((address_space(3))) double;
__device__ __forceinline__ lds_cdouble* lds_opaque(const double* p) {
  uint32_t a = (uint32_t)(uintptr_t)(lds_cdouble*)p;
  asm volatile("" : "+v"(a));
  return (lds_cdouble*)(uintptr_t)a;
}

// Section timing (debug builds only, -DVC_TIMING, `make timing`): wave-uniform
// s_memtime stamps accumulated per section and written to diag[b][4..].
#ifdef VC_TIMING
#define VC_TSTAMP(var) \
  fence();              \
  const uint64_t var = __builtin_amdgcn_s_memtime(); \
  fence();
#define VC_TACC(slot, t0) \
  {                      \
    fence();             \
    tacc[slot] += __builtin_amdgcn_s_memtime() - (t0); \
    fence();             \
  }
#else
#define VC_TSTAMP(var)
#define VC_TACC(slot, t0)
#endif
// T_SWEEP = the serial rollout S1; T_S2 / T_S3 / T_S4 the sweep's other three parts
// T_UPDATE: the polish's matrix build + factorisation (part of T_POLISH); T_PAL its augmented-
// Lagrangian passes (cycles), T_PPASS their count; T_NUPD the rounds whose factor came from
// factor_update, T_UCYC those updates' cycles, T_NDROP the rounds ended by dropping a bound or row;
// T_CFAIL 1 after a failed early attempt, T_CRM / T_CADD how many bounds and rows the final attempt's
// first set drops / adds against the early attempt's last factored one (a study of carrying that factor);
// T_R0CHG the early attempt's first change: 1 + (0 box add, 1 row add, 2 drop) + 3 x its side's Tapia state
enum { T_SWEEP = 0, T_SETUP, T_RESID, T_BUILD, T_CHOL, T_SOLVE, T_UPDATE, T_POLISH, T_OUT, T_S2, T_S3, T_S4, T_PAL, T_PPASS, T_NUPD, T_UCYC, T_NDROP, T_CFAIL, T_CRM, T_CADD, T_R0CHG, T_NSLOT };


template <int N>
struct Dims {
  static constexpr int n = 2 * N;         // decision variables
  static constexpr int NC = 2 * (N - 1);  // state-constraint rows
  static constexpr int LD = n + 1;        // odd LDS row stride: lane-varying-row reads are conflict-free
  static_assert(n <= 64 && N >= 2, "one wavefront per problem needs 2 <= N <= 32");
};

// Column k of the Cholesky factor, L[j][k] for j = k..n-1, is stored at Lc[lc_base(k) + j].
// lc_base(k) is even, so the entry pairs (j, j+1) with j even sit on 16-byte boundaries: both
// columns of a trailing-update chunk load as ds_read_b128 at immediate offsets (a packed layout
// left every other column odd, and its pairs became ds_read2_b64 behind a v_mov of the address).
// Closed form (n even; a loop here became a divergent runtime loop where k is a lane's row):
// column k starts at lc_start(k) = lc_base(k) + k, one padding slot after every even column.
template <int n>
__host__ __device__ constexpr int lc_base(int k) {
  static_assert(n % 2 == 0, "even n");
  return k * (n - 1) - k * (k - 1) / 2 + (k + 1) / 2;
}
template <int n>
__host__ __device__ constexpr int lc_start(int k) {
  return lc_base<n>(k) + k;
}

template <int N>
struct Smem {
  using D = Dims<N>;
  static constexpr int LC_DUMMY = lc_start<D::n>(D::n);  // branch-free stores of inactive lanes
  static constexpr int LC_ZERO = LC_DUMMY + 1;           // always 0.0 (solve reads above the factor)
  // constraint rows of the condensed sensitivity (row r: stage crow_stage(r)); rows NC, NC+1 are
  // zero (the normal-matrix build's last k-step), row NC+2 takes the sweep's dummy stores;
  // column n is zero in every row
  double G[D::NC + 3][D::LD];
  double H[D::n + 1][D::LD];  // condensed Hessian (constant over the solve); row n: dummy
  alignas(16) double Lc[LC_ZERO + 1];  // columns of the Cholesky factor (lc_base), dummy, zero
  alignas(16) double zrow[48];  // zeros: the normal-matrix transpose reads it for other block rows
  double xb[N + 1][KIN_NX + 1];  // predicted trajectory (+1: dummy column for branch-free stores)
  double jac[N + 1][9];     // Jacobian data per stage (KinJac); row N: dummy
  double ub[D::n];          // warm-start inputs, interleaved (a_0, w_0, a_1, ...)
  double kap[N], ds[N];
  union {
    struct {
      double vz[64];        // broadcast: a length-n vector (z, dz, ...)
      double vc[64];        // broadcast: a length-NC vector (weights, residual terms)
    };
    alignas(16) double tb2[128];  // factor_blocked: last panel's transpose buffer (vz, vc are scratch then)
  };
  double dinv[64];          // inverse pivots 1/L_kk of the current factor (uniform reads)
};

// stage index (1..N-1) of constraint row r
template <int N>
__host__ __device__ constexpr int crow_stage(int r) {
  return r < N - 1 ? r + 1 : r - (N - 1) + 1;
}

// sum_{i<LEN} a[i*SA] b[i*SB] over LDS operands, loaded one CH-chunk ahead of their FMAs
// (one scheduling fence per chunk) so the LDS latency is paid about once per call
template <int LEN, int SA, int SB, int CH = KIN_DOT_CH>
__device__ __forceinline__ double lds_dot(lds_cdouble* a, lds_cdouble* b) {
  constexpr int NCH = (LEN + CH - 1) / CH;
  double ca[2][CH], cb[2][CH];
  auto fetch = [&](int c, int buf) {
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const int i = c * CH + q;
      ca[buf][q] = (i < LEN) ? a[i * SA] : 0.0;
      cb[buf][q] = (i < LEN) ? b[i * SB] : 0.0;
    }
  };
  double a0 = 0.0, a1 = 0.0;
  fetch(0, 0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) fetch(c + 1, (c + 1) & 1);
    fence();
#pragma unroll
    for (int q = 0; q < CH; q += 2) {
      a0 += ca[c & 1][q] * cb[c & 1][q];
      a1 += ca[c & 1][q + 1] * cb[c & 1][q + 1];
    }
  }
  fence();
  return a0 + a1;
}

// y_r = G_r . v for lane r (v broadcast in s.vz); rows have <= 2(N-1) nonzeros
template <int N>
__device__ double grow_dot(const Smem<N>& s, int lane) {
  constexpr int NC = Dims<N>::NC;
  const int r = lane < NC ? lane : 0;
  const double a = lds_dot<2 * (N - 1), 1, 1>(lds_opaque(&s.G[r][0]), lds_opaque(&s.vz[0]));
  return lane < NC ? a : 0.0;
}

// (G' v)_j for lane j (v broadcast in s.vc)
template <int N>
__device__ double gt_dot(const Smem<N>& s, int lane) {
  constexpr int n = Dims<N>::n, NC = Dims<N>::NC, LD = Dims<N>::LD;
  const int j = lane < n ? lane : 0;
  const double a = lds_dot<NC, LD, 1>(lds_opaque(&s.G[0][j]), lds_opaque(&s.vc[0]));
  return lane < n ? a : 0.0;
}


// (H v)_j for lane j (v broadcast in s.vz)
template <int N>
__device__ double h_dot(const Smem<N>& s, int lane) {
  constexpr int n = Dims<N>::n;
  const int j = lane < n ? lane : 0;
  return lds_dot<n, 1, 1>(lds_opaque(&s.H[j][0]), lds_opaque(&s.vz[0]));
}

// sin and cos of a small angle (the rollout's heading error and steering angle, |x| ~ 1): one
// Cody-Waite step by pi/2 (a 33-bit head, exact in the fma for |n| < 2^20, and a 53-bit tail) and
// fdlibm's kernels on [-pi/4, pi/4] (< 1 ulp), no large-argument path -- the library sincos
// carries a Payne-Hanek branch and a three-part reduction on S1's serial chain.  With the quotients
// below as num * rcp_nr(den): S1 26.6 K -> 22.1 K cycles, C2 -1.0 %, C4 -1.4 %, u* within 2.2e-10
// (profiles/r06/kin_ab/kin_polish_ab_c2_r06y.log, kin_polish_sec_ft1_r06y.txt)
__device__ __forceinline__ void kin_sincos(double x, double& sn, double& cs) {
  const double n = __builtin_rint(x * 6.36619772367581382433e-01);
  const double y = fma(-n, 6.07710050650619224932e-11, fma(-n, 1.57079632673412561417e+00, x));
  const double z = y * y;
  const double rs = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                      2.75573137070700676789e-06), -1.98412698298579493134e-04),
                        8.33333333332248946124e-03);
  const double sk = fma(z * y, fma(z, rs, -1.66666666666666324348e-01), y);
  const double rc = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                  -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                   -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double ck = w + (((1.0 - w) - hz) + z * rc);
  const int q = int(n) & 3;
  const double a = (q & 1) ? ck : sk, b = (q & 1) ? sk : ck;
  sn = (q & 2) ? -a : a;
  cs = ((q + 1) & 2) ? -b : b;
}

// 1/sqrt(d): hardware v_rsq_f64 + two Newton steps (full fp64 accuracy, a much shorter
// dependent chain than IEEE sqrt followed by IEEE divide)
__device__ __forceinline__ double rsq_nr(double d) {
  double inv = __builtin_amdgcn_rsq(d);
#if KIN_RSQ_HALLEY
  // one third-order step: with e = 1 - d y^2, 1/sqrt(d) = y (1 - e)^-1/2 = y (1 + e/2 + 3e^2/8 + O(e^3)):
  // four dependent operations instead of two Newton steps' eight
  const double e = fma(-d, inv * inv, 1.0);
  return fma(inv * e, fma(0.375, e, 0.5), inv);
#else
  inv = inv * (1.5 - 0.5 * d * inv * inv);
  inv = inv * (1.5 - 0.5 * d * inv * inv);
  return inv;
#endif
}

// After a factorisation: row k of L (entries i < k) to Lc[k (k-1)/2 + i], packed rows, for the
// backward sweep -- its lanes i then read L[k][i] at consecutive addresses (the column layout put
// them one column apart: 4-6 way bank conflicts on every read, ~75 % of the kernel's conflict
// cycles, r04 PMC).  Lane j stores entries i < j; the others go to the dummy slot (branch-free:
// the compiler may reorder one lane's stores, so no store may land on another lane's entry).  The
// factorisation's own column reads were issued before (LDS executes a wave's operations in order).
template <int N>
__device__ __forceinline__ void store_rows(const double (&Mr)[Dims<N>::n], Smem<N>& s, int lane) {
}

// Solve (L L') x = b, lane j holding b_j; returns x_j.  Forward sweep: y_k = acc_k / L_kk is
// broadcast from lane k, and every lane subtracts L[lane][k] y_k from its accumulator with the
// row registers zero on and above the diagonal (factor_blocked), so lane k's accumulator stops
// changing once y_k is taken and y = acc / L_kk at the end -- no per-step select (a finite
// factor times 0 subtracts exactly 0: the same values as collecting y_k per step).  Backward
// sweep: lane i reads L[k][i] (row k of the packed rows, store_rows; or column i of the factor)
// from LDS at immediate offsets of one per-lane base, prefetched one 8-step chunk ahead, and x_i
// is written into lane i at step i by v_writelane (entries k <= i of the read are other rows'
// storage: after step i they no longer matter) -- cheaper than a zero-or-entry address select
// per element.  (A four-unknown blocked variant
// was 13 % slower: the sweeps are bound by instruction issue, profiles/r03/section_cycles_r03g.txt.)
template <int N>
__device__ double chol_solve(const double (&Lr)[Dims<N>::n], const Smem<N>& s, double b, int lane) {
  constexpr int n = Dims<N>::n;
  constexpr int CH = KIN_SOLVE_CH;
  static_assert(n % CH == 0, "backward prefetch chunks");
  const int row = lane < n ? lane : 0;
  lds_cdouble* col = lds_opaque(&s.Lc[lc_base<n>(row)]);  // col[k] = L[k][row] for k > row
  const double dj = s.dinv[row];
  double acc = b;
#pragma unroll
  for (int k = 0; k < n; ++k) acc -= Lr[k] * lane_bcast(acc * dj, k);  // L y = b
  acc *= dj;                                                           // y
  double x = 0.0;
  double lk[2][CH];
  lds_cdouble* zero = lds_opaque(&s.zrow[0]);
  auto fetch = [&](int c, int buf) {  // L[k][row] for k = n-1-c*CH ... n-CH-c*CH
    // a lane whose row is at or below every k of the chunk reads zeros at one shared address
    // (broadcast) instead of the previous columns' storage (distinct addresses: bank conflicts)
    lds_cdouble* src = row < n - 1 - c * CH ? col : zero;
#pragma unroll
    for (int q = 0; q < CH; ++q) lk[buf][q] = src[n - 1 - c * CH - q];
  };
  fetch(0, 0);
#pragma unroll
  for (int c = 0; c < n / CH; ++c) {  // L' x = y: lane i < k needs L[k][i]
    if (c + 1 < n / CH) fetch(c + 1, (c + 1) & 1);
    fence();
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const int k = n - 1 - c * CH - q;
      const double xk = lane_bcast(acc * dj, k);
      x = lane_put(x, xk, k);
      acc -= lk[c & 1][q] * xk;
    }
    fence();
  }
  return x;
}

// Nonzero extent of row r of the two LDS row sets the matrix cores take Gram matrices of:
// ROWS_G, the constraint rows of G (row r is zero beyond column 2 crow_stage(r): stage k's
// sensitivity sees only the inputs of stages < k; rows NC, NC+1 are the zero rows), and
// ROWS_E, the ey cost rows E[k] (ey_{k+1}, zero beyond column 2 (k+1)) plus the terminal v_N /
// epsi_N rows and two zero rows.
enum { ROWS_G = 0, ROWS_E = 1 };
template <int N, int KIND>
__host__ __device__ constexpr int row_extent(int r) {
  if (KIND == ROWS_G) return r < Dims<N>::NC ? 2 * crow_stage<N>(r) : 0;
  return r < N ? 2 * (r + 1) : (r < N + 2 ? 2 * N : 0);
}
template <int N, int KIND>
__host__ __device__ constexpr int gram_rows() {
  return KIND == ROWS_G ? Dims<N>::NC : N + 2;
}
// Does MFMA k-step ks (rows 4 ks .. 4 ks + 3) touch block-row I of the lower block triangle?
// A k-step whose four rows all end at or before column 16 I adds exact zeros to every tile
// (I, J <= I) and is skipped.  N = 20, G: 33 of the 60 tile-steps remain (block-row 0: 10
// k-steps, 1: 7, 2: 3); E: 20 of 36.
template <int N, int KIND>
__host__ __device__ constexpr bool kstep_hits(int ks, int I) {
  for (int q = 0; q < 4; ++q)
    if (row_extent<N, KIND>(4 * ks + q) > 16 * I) return true;
  return false;
}

using d4 = __attribute__((ext_vector_type(4))) double;
using d2 = __attribute__((ext_vector_type(2))) double;
template <int N>
struct Tiles {
  // BLD even: the buffer rows are 16-byte aligned, so the row reads of tiles_to_rows pair up as
  // ds_read_b128 (conflict-free: row starts 100 dwords apart spread over the 64 banks)
  static constexpr int n = Dims<N>::n, NB = (n + 15) / 16, NT = NB * (NB + 1) / 2, BLD = 16 * NB + 2;
  static constexpr int count(bool full) { return full ? NB * NB : NT; }
};

// acc += (W R)' R over the rows R of one LDS row set (row stride LD, column n zero, rows up to
// 4 KS - 1 readable) with weights w[r]: 16x16 tiles of v_mfma_f64_16x16x4_f64, K = 4 rows per
// step, the lower block triangle (tile t of row I, column J <= I in order) or, FULL, every
// tile (t = NB I + J).  Operands are loaded up front (the LDS latency paid once): lane l
// holds row 4 ks + (l >> 4), column 16 J + (l & 15).
template <int N, int KIND, bool FULL>
__device__ __forceinline__ void gram_mfma(d4 (&acc)[Tiles<N>::count(FULL)], const double* rows, const double* w,
                                          int lane) {
  constexpr int n = Dims<N>::n, LD = Dims<N>::LD, NB = Tiles<N>::NB;
  constexpr int KS = (gram_rows<N, KIND>() + 3) / 4;
  lane = lane_opaque(lane);
  const int lr = lane >> 4, lc = lane & 15;
  lds_cdouble* R = lds_opaque(rows);
  lds_cdouble* W = lds_opaque(w);
  double gk[KS][NB], wk[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int r = 4 * ks + lr;
    wk[ks] = W[r];
#pragma unroll
    for (int J = 0; J < NB; ++J) {
      const int c = 16 * J + lc;
      gk[ks][J] = R[r * LD + (c < n ? c : n)];
    }
  }
  fence();
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int I = 0, t = 0; I < NB; ++I) {
      const double a = wk[ks] * gk[ks][I];
#pragma unroll
      for (int J = 0; J < (FULL ? NB : I + 1); ++J, ++t)
        if (kstep_hits<N, KIND>(ks, I > J ? I : J))
          acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, gk[ks][J], acc[t], 0, 0, 0);
    }
  }
}

// Accumulator tiles (lane l, element q of tile (I, J): row 16 I + (l >> 4) + 4 q, column
// 16 J + (l & 15)) to row `lane` in Mr -- its lower block triangle, or the whole row (FULL) --
// one 16-row block at a time through a 16 x 50 LDS buffer aliasing the (not yet written)
// factor storage.  Select-free: lanes outside the block row being moved read the zero row.
template <int N, bool FULL>
__device__ __forceinline__ void tiles_to_rows(double (&Mr)[Dims<N>::n], const d4 (&acc)[Tiles<N>::count(FULL)],
                                              Smem<N>& s, int lane) {
  constexpr int n = Dims<N>::n, NB = Tiles<N>::NB, BLD = Tiles<N>::BLD;
  static_assert(16 * BLD <= Smem<N>::LC_DUMMY, "transpose buffer must fit the factor storage");
  static_assert(16 * NB <= 48, "zero row length");
  lane = lane_opaque(lane);
  const int lr = lane >> 4, lc = lane & 15;
  double* buf = &s.Lc[0];
  const int myI = lane >> 4;
#pragma unroll
  for (int I = 0, t0 = 0; I < NB; ++I, t0 += FULL ? NB : I) {
    wave_sync();  // previous block-row consumed
#pragma unroll
    for (int J = 0; J < (FULL ? NB : I + 1); ++J) {
#pragma unroll
      for (int q = 0; q < 4; ++q) buf[(lr + 4 * q) * BLD + 16 * J + lc] = acc[t0 + J][q];
    }
    wave_sync();
    // 16-byte pair reads (BLD even; the laundered pointer hides the alignment from the compiler)
    using lds_cd2 = const __attribute__((address_space(3))) d2;
    lds_cd2* brow = (lds_cd2*)lds_opaque(myI == I ? &buf[lc * BLD] : &s.zrow[0]);
#pragma unroll
    for (int i = 0; i < n; i += 2) {
      const int iend = FULL ? n : 16 * (I + 1);
      if (i < iend) {
        const d2 p = brow[i / 2];
        if (I == 0) { Mr[i] = p.x; Mr[i + 1] = p.y; }
        else { Mr[i] += p.x; Mr[i + 1] += p.y; }
      } else if (I == 0) {
        Mr[i] = 0.0;
        Mr[i + 1] = 0.0;
      }
    }
  }
  wave_sync();  // buffer reads done before the factorisation overwrites it
}

// The normal matrix M = H + diag(wb) + (W G)' G, row `lane` into Mr: the constraint part on
// the matrix cores (gram_mfma over the G rows, weights s.vc), accumulated onto H + diag(wb)
// loaded in the accumulator layout, then moved to rows (tiles_to_rows).  Select-free (every
// VALU instruction costs the same ~5 ticks as an fp64 FMA here): diag(wb) enters through
// lane j's own H[j][j] slot (written before the tile loads, restored after), padding comes
// from zero rows / columns in LDS (G rows NC, NC+1, H column n).  hjj: this lane's H[j][j].
template <int N>
__device__ __forceinline__ void build_normal_acc(d4 (&acc)[Tiles<N>::NT], Smem<N>& s, double wb, double hjj, int lane) {
  constexpr int n = Dims<N>::n, LD = Dims<N>::LD, NB = Tiles<N>::NB;
  static_assert(4 * ((Dims<N>::NC + 3) / 4) <= Dims<N>::NC + 2, "G zero rows cover the last k-step");
  lane = lane_opaque(lane);
  const int lr = lane >> 4, lc = lane & 15;
  const int jd = lane < n ? lane : n;  // lanes >= n: the dummy row's padding slot
  s.H[jd][jd] = hjj + wb;
  wave_sync();
  {
    lds_cdouble* H = lds_opaque(&s.H[0][0]);
#pragma unroll
    for (int I = 0, t = 0; I < NB; ++I) {
#pragma unroll
      for (int J = 0; J <= I; ++J, ++t) {
        const int c = 16 * J + lc < n ? 16 * J + lc : n;  // column n of H is zero
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r0 = 16 * I + 4 * q;  // row r0 + lr: every lane of this q is padding when r0 >= n
          acc[t][q] = r0 < n ? H[(r0 + lr) * LD + c] : 0.0;
        }
      }
    }
  }
  s.H[jd][jd] = hjj;  // LDS executes in issue order: the loads above saw hjj + wb
  gram_mfma<N, ROWS_G, false>(acc, &s.G[0][0], &s.vc[0], lane);
}

template <int N>
__device__ __forceinline__ void build_normal_mfma(double (&Mr)[Dims<N>::n], Smem<N>& s, double wb, double hjj,
                                                  int lane) {
  d4 acc[Tiles<N>::NT];
  build_normal_acc<N>(acc, s, wb, hjj, lane);
  tiles_to_rows<N, false>(Mr, acc, s, lane);
}

// Blocked factorisation of the normal matrix straight from the build's accumulator tiles:
// panels of 16 columns (the last one 8); for each, the panel's tiles (I, p), I >= p, are moved
// to this lane's row registers (tile by tile through a 16 x 18 LDS buffer, select-free: lanes
// outside block row I read the zero row), the panel is factored by the two-column pivot steps
// described below with the trailing update kept inside the panel, and the tiles to the right,
// (I, J) with p < J <= I, take the panel's rank-16 update on the matrix cores
// (v_mfma_f64_16x16x4_f64, operands = the just-stored factor columns from LDS): the trailing
// update, 880 VALU FMAs + 380 broadcast reads in the row-per-lane factorisation, becomes
// 16 MFMAs.  Output: s.Lc columns, s.dinv (inverse pivots), Mr = row `lane` of L strictly
// below the diagonal.  Buffers: panels 0, 1 use the factor storage of columns >= 16 (written
// only by panel 1's own steps, after its transposes), panel 2 the broadcast vectors (tb2).
// Returns false (uniform) if a pivot is not positive.
// Pivot steps: two columns per step -- the 2x2 diagonal block comes from lanes k, k+1 by
// readlane, both pivots are taken in registers (rsq_nr), both columns published to LDS, and one
// LDS round trip serves the rank-2 update.  Software-pipelined: the pivot block k+2, k+3 depends
// only on the lookahead columns (chunk 0 of step k's update), so its chain -- readlanes, two
// rsq, the column scaling and its stores -- is split in three parts placed in the fence regions
// of step k's update chunks 1, 2, 3, where the scheduler interleaves it with independent FMAs.
// (A row-per-lane unblocked version of the same steps was the round-2/3 factorisation; the
// second pivot from the block's determinant, both rsq chains in parallel, measured no gain in
// round 6: the steps are bound by issue, not by the pivot chain.)
template <int N>
__device__ bool factor_blocked(double (&Mr)[Dims<N>::n], d4 (&acc)[Tiles<N>::NT], Smem<N>& s, int lane) {
  constexpr int n = Dims<N>::n, NB = Tiles<N>::NB;
  constexpr int DUMMY = Smem<N>::LC_DUMMY;
  static_assert(NB == 3 && n > 32 && n <= 40, "three panels, the last one at most 8 wide");
  static_assert(lc_start<n>(16) + 16 * 18 <= DUMMY, "panel 0/1 transpose buffer inside the factor storage");
  static_assert((lc_start<n>(16) & 1) == 0, "16-byte aligned transpose buffer");
  lane = lane_opaque(lane);
  const int lr = lane >> 4, lc = lane & 15, myI = lane >> 4;
  bool ok = true;
  double pa, pb, pc, pi1, pl21, pi2;  // chain state of the pending pivot block
  auto part = [&](int p, int k) {
    if (p == 0) {
      pa = lane_bcast(Mr[k], k);
      pb = lane_bcast(Mr[k], k + 1);
      pc = lane_bcast(Mr[k + 1], k + 1);
      pi1 = rsq_nr(pa);
    } else if (p == 1) {
      pl21 = pb * pi1;
      const double d2 = fma(-pl21, pl21, pc);
      pi2 = rsq_nr(d2);
      ok = ok && (pa > 0.0) && (d2 > 0.0);
    } else {
      const double x = Mr[k] * pi1;
      const double y = fma(-x, pl21, Mr[k + 1]) * pi2;
      Mr[k] = x;
      Mr[k + 1] = y;
      s.Lc[lane >= k && lane < n ? lc_base<n>(k) + lane : DUMMY] = x;
      s.Lc[lane >= k + 1 && lane < n ? lc_base<n>(k + 1) + lane : DUMMY] = y;
      s.dinv[k] = pi1;
      s.dinv[k + 1] = pi2;
    }
  };
  using lds_cd2 = const __attribute__((address_space(3))) d2;
#pragma unroll
  for (int p = 0; p < NB; ++p) {
    const int c0 = 16 * p, c1 = (16 * p + 16 < n) ? 16 * p + 16 : n, W = c1 - c0;
    // ---- panel columns of this lane's row from tiles (I, p), I >= p
    double* tb = p < 2 ? &s.Lc[lc_start<n>(16)] : &s.tb2[0];
    const int TS = p < 2 ? 18 : 10;  // even stride: 16-byte rows, conflict-free row reads
#pragma unroll
    for (int i = c0; i < c1; ++i) Mr[i] = 0.0;
#pragma unroll
    for (int I = p; I < NB; ++I) {
      const int t = I * (I + 1) / 2 + p;
      wave_sync();  // previous tile consumed
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = lr + 4 * q;
        if (4 * q < W)  // panel 2: rows 8..15 of its tile are padding
          tb[(lc < W ? r * TS + lc : 8 * TS + lc)] = acc[t][q];  // lc >= W: dummy slots past the rows
      }
      wave_sync();
      lds_cd2* src = (lds_cd2*)lds_opaque(myI == I && lc < W ? &tb[lc * TS] : &s.zrow[0]);
#pragma unroll
      for (int i = 0; i < W; i += 2) {
        const d2 v = src[i / 2];
        Mr[c0 + i] += v.x;
        Mr[c0 + i + 1] += v.y;
      }
    }
    wave_sync();  // buffer reads done before the panel's factor stores
    // ---- the panel: two-column pivot steps, trailing update inside the panel
    part(0, c0);
    part(1, c0);
    part(2, c0);
#pragma unroll
    for (int k = c0; k + 2 < c1; k += 2) {
      wave_sync();  // columns k, k+1 visible
      fence();
      const double x = Mr[k], y = Mr[k + 1];
      Mr[k] = lane > k ? x : 0.0;
      Mr[k + 1] = lane > k + 1 ? y : 0.0;
      const double* cA = &s.Lc[lc_base<n>(k)];
      const double* cB = &s.Lc[lc_base<n>(k + 1)];
      constexpr int CH = KIN_PANEL_CH;
      const int J0 = k + 2, NCH = (c1 - J0 + CH - 1) / CH;
      double u0[2][CH], u1[2][CH];
      auto load = [&](int ch, int buf) {
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const int j = J0 + ch * CH + q;
          u0[buf][q] = j < c1 ? cA[j] : 0.0;
          u1[buf][q] = j < c1 ? cB[j] : 0.0;
        }
      };
      load(0, 0);
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (ch + 1 < NCH) load(ch + 1, (ch + 1) & 1);
        fence();
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const int j = J0 + ch * CH + q;
          if (j < c1) Mr[j] = fma(-y, u1[ch & 1][q], fma(-x, u0[ch & 1][q], Mr[j]));
        }
        if (ch >= 1 && ch <= 3) part(ch - 1, k + 2);
        fence();
      }
#pragma unroll
      for (int pp = NCH - 1; pp < 3; ++pp) {
        part(pp < 0 ? 0 : pp, k + 2);
        fence();
      }
    }
    Mr[c1 - 2] = lane > c1 - 2 ? Mr[c1 - 2] : 0.0;
    Mr[c1 - 1] = lane > c1 - 1 ? Mr[c1 - 1] : 0.0;
    wave_sync();  // the panel's factor columns visible
    // ---- rank-W update of the tiles right of the panel on the matrix cores
    if (p + 1 < NB) {
      lds_cdouble* Lc = lds_opaque(&s.Lc[0]);
      lds_cdouble* Z = lds_opaque(&s.zrow[0]);
#pragma unroll
      for (int ks = 0; ks < W / 4; ++ks) {
        // operand of block row I: lane l holds L[16 I + (l & 15)][c0 + 4 ks + (l >> 4)]
        const int kk = c0 + 4 * ks + lr;
        double op[NB];
#pragma unroll
        for (int I = p + 1; I < NB; ++I) {
          const int jj = 16 * I + lc;
          op[I] = jj < n ? Lc[lc_base<n>(kk) + jj] : Z[0];
        }
#pragma unroll
        for (int I = p + 1; I < NB; ++I) {
#pragma unroll
          for (int J = p + 1; J <= I; ++J) {
            const int t = I * (I + 1) / 2 + J;
            acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-op[I], op[J], acc[t], 0, 0, 0);
          }
        }
      }
    }
  }
  store_rows<N>(Mr, s, lane);
  wave_sync();  // factor and inverse pivots visible to the solves
  return ok;
}

// Inclusive prefix sum over the wave (lane i: sum of v over lanes <= i): a DPP prefix within each
// 16-lane row, then the earlier rows' totals from three readlanes.
__device__ __forceinline__ double wave_prefix(double v, int lane) {
  v += dpp_row_shr<1>(v, 0.0);
  v += dpp_row_shr<2>(v, 0.0);
  v += dpp_row_shr<4>(v, 0.0);
  v += dpp_row_shr<8>(v, 0.0);
  const double r0 = lane_bcast(v, 15), r1 = lane_bcast(v, 31), r2 = lane_bcast(v, 47);
  return v + (lane >= 16 ? r0 : 0.0) + (lane >= 32 ? r1 : 0.0) + (lane >= 48 ? r2 : 0.0);
}

// The polish's next factor from the current one when a round changed the reduced matrix by a
// rank-one term (KIN_UPDATE), instead of a build + factor_blocked (~17 K cycles per round):
//   upd 1: variable j became fixed.  Its row / column turn into the identity; with
//          M = [M11 . M13; . . .; M31 . M33] the new factor keeps L11 and L31, and its trailing
//          block satisfies L33' L33'^T = L33 L33^T + z z^T, z = L[j+1:, j] -- a rank-one update
//          of the columns after j (the state rows keep their weights, see the polish);
//   upd 2: state row j became active with weight rho: M' = M + z z^T, z = sqrt(rho) g_F.
// Both are updates (a dropped bound or row, a downdate, takes the full path).  The update is
// Gill, Golub, Murray & Saunders' method C1 (Math. Comp. 28, 1974), stable for positive
// updates, in the form that maps onto lanes: with y = L^-1 z (one forward sweep) and the prefix
// sums t_k = 1 + sum_{i<=k} y_i^2 (one wave scan), column k of the new factor is
//     L'_rk = (L_rk + c_k w_r) s_k,   w_r <- w_r - y_k L_rk (before),   c_k = y_k / t_k,
//     s_k = sqrt(t_k / t_{k-1}),   L'_kk = L_kk s_k,
// where w starts at z: the recurrence that sets every coefficient is the scan, and the column sweep
// is lane-local (lane r runs along its own row), so no step waits on the previous one's pivot
// (a textbook rotation sweep, one pivot chain per column, measured ~450 cycles per column).  Lane k's
// w is zeroed at column k, so the entries on and above the diagonal stay 0.  (numpy check of both
// cases against a fresh Cholesky: <= 9e-15 relative.)
template <int N>
__device__ bool factor_update(double (&Mr)[Dims<N>::n], Smem<N>& s, int upd, int j, bool fixed, double sqrho,
                              int lane) {
  constexpr int n = Dims<N>::n;
  constexpr int DUMMY = Smem<N>::LC_DUMMY, ZERO = Smem<N>::LC_ZERO;
  lane = lane_opaque(lane);
  const int row = lane < n ? lane : 0;
  // slot of L[lane][k] strictly below the diagonal, else the zero slot (loads) / the dummy (stores)
  auto below = [&](int k, int other) { return lane > k && lane < n ? lc_base<n>(k) + lane : other; };
  double z;
  if (upd == 1) {  // uniform
    z = s.Lc[below(j, ZERO)];  // column j below the diagonal, then the identity row / column j
    wave_sync();
    s.Lc[below(j, DUMMY)] = 0.0;
    s.Lc[lane < j ? lc_base<n>(lane) + j : DUMMY] = 0.0;
    s.Lc[lc_start<n>(j)] = 1.0;
    s.dinv[j] = 1.0;
  } else {
    z = (lane < n && !fixed) ? sqrho * s.G[j][lane < n ? lane : n] : 0.0;
  }
  wave_sync();
  // the rows from the stored columns (Mr is dead between rounds: the KKT check needs its registers)
  {
    lds_cdouble* L = lds_opaque(&s.Lc[0]);
#pragma unroll
    for (int k = 0; k < n; ++k) Mr[k] = L[below(k, ZERO)];
  }
  // y = L^-1 z (chol_solve's forward sweep)
  const double dj = s.dinv[row];
  double acc = z;
#pragma unroll
  for (int k = 0; k < n; ++k) acc -= Mr[k] * lane_bcast(acc * dj, k);
  const double y = lane < n ? acc * dj : 0.0;
  const double t = 1.0 + wave_prefix(y * y, lane);
  const double sk = sqrt(t / (t - y * y)), ck = y / t;
  const bool ok = __ballot(!(sk > 0.5 && sk < 1e150)) == 0ull;  // uniform: finite scalings (s_k >= 1 in exact arithmetic)
  wave_sync();
  if (lane < n) {
    s.Lc[lc_start<n>(row)] *= sk;
    s.dinv[row] = dj / sk;
  }
  s.tb2[2 * lane] = ck;  // (c_k, s_k) pairs: one 16-byte broadcast read per column
  s.tb2[2 * lane + 1] = sk;
  wave_sync();
  {
    using lds_cd2 = const __attribute__((address_space(3))) d2;
    lds_cd2* cs = (lds_cd2*)lds_opaque(&s.tb2[0]);
    double w = z;
#pragma unroll
    for (int k = 0; k < n - 1; ++k) {
      const double yk = lane_bcast(y, k);
      const d2 c = cs[k];
      w = lane_put(w, 0.0, k);
      const double l = Mr[k];
      w = fma(-yk, l, w);
      Mr[k] = fma(c.x, w, l) * c.y;
    }
  }
#pragma unroll
  for (int k = 0; k < n - 1; ++k) s.Lc[below(k, DUMMY)] = Mr[k];
  wave_sync();  // factor and inverse pivots visible to the solves
  return ok;
}

// inequality data of one lane role (box or state row): bounds lo <= y <= hi,
// slacks slo = y - lo, shi = hi - y, multipliers llo, lhi.
struct Side {
  double lo, hi, slo, shi, llo, lhi;
  bool hasLo, hasHi;
};

}  // namespace

template <int N>
__global__ __launch_bounds__(64) void kin_ltv_kernel(KinLtvArgs A) {
  using D = Dims<N>;
  constexpr int n = D::n, NC = D::NC;
  // static LDS: every address is a compile-time constant folded into the ds
  // instruction's offset field (a dynamic extern buffer makes the compiler
  // materialise each address in an SGPR and spill them)
  __shared__ Smem<N> s;
  const int lane = threadIdx.x;
  const int b = xcd_problem(blockIdx.x, A.B);
  if (b >= A.B) return;
  const vc_kin_mpc& W = A.w;

  // ---- load inputs (coalesced) -------------------------------------------
  if (lane < n) s.ub[lane] = A.ubar[(size_t)b * n + lane];
  if (lane < N) {
    s.kap[lane] = A.kappa[(size_t)b * N + lane];
    s.ds[lane] = A.ds[(size_t)b * N + lane];
  }
  if (lane < KIN_NX) s.xb[0][lane] = A.x0[(size_t)b * KIN_NX + lane];
  for (int i = lane; i < 2 * D::LD; i += 64) (&s.G[NC][0])[i] = 0.0;  // zero rows NC, NC+1
  if (lane < 48) s.zrow[lane] = 0.0;
  if (lane == 0) s.Lc[Smem<N>::LC_ZERO] = 0.0;
  wave_sync();

#ifdef VC_TIMING
  uint64_t tacc[T_NSLOT] = {};
#endif
  VC_TSTAMP(t_sweep0)
  // ---- predict + linearize + condense ------------------------------------------
  // S1 serial rollout (uniform across lanes; the only serial transcendental
  // chain), S2 Jacobians of all stages in parallel (lane k: stage k), S3 the
  // sensitivity sweep (lane j carries column j of G: dv, ddelta, dey, depsi, dt
  // w.r.t. dz_j) writing the v / delta constraint rows and the ey cost rows to
  // LDS, S4 the Hessian from the ey rows (rank-1 updates, each row's broadcast
  // operands preloaded at once).  No LDS round trip sits inside S1/S3's chains
  // except the one-stage-ahead Jacobian prefetch.
  constexpr int LD = Dims<N>::LD;
  double* E = &s.H[0][0];  // ey rows E[k][j] (k < N) + 2 terminal rows, scratch until H is written
  bool finite = true;
  {  // S1
    double x[KIN_NX];
#pragma unroll
    for (int i = 0; i < KIN_NX; ++i) x[i] = s.xb[0][i];
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
      const double u2[2] = {s.ub[2 * k], s.ub[2 * k + 1]};
      const double h = s.ds[k];
      double f[KIN_NX];
      // kin_spatial_ode (kinematic_car.py:47-64) with its transcendentals and divides taken in
      // parallel lanes (S1 is the sweep's only serial chain): lane 0 sincos(epsi), lane 1
      // sincos(delta) -- one range reduction each instead of cos(epsi), tan(epsi), tan(delta)
      // one after another -- then the four quotients tan(epsi) = sin/cos, tan(delta) / L,
      // rho / cos(epsi) and q = rho / (v cos(epsi)) as one divide in lanes 0..3
      {
        double sn, cs;
        kin_sincos((lane & 1) ? x[1] : x[4], sn, cs);
        const double se = lane_bcast(sn, 0), ce = lane_bcast(cs, 0);
        const double sd = lane_bcast(sn, 1), cd = lane_bcast(cs, 1);
        const double kap = s.kap[k];
        const double rho = 1.0 - x[3] * kap;
        const int r4 = lane & 3;
        const double num = r4 == 0 ? se : (r4 == 1 ? sd : rho);
        const double den = r4 == 0 ? ce : (r4 == 1 ? cd * A.L : (r4 == 2 ? ce : x[0] * ce));
        const double quo = num * rcp_nr(den);  // correctly rounded 1/den, then one rounding more
        const double te = lane_bcast(quo, 0), tdl = lane_bcast(quo, 1);
        const double rc = lane_bcast(quo, 2), q = lane_bcast(quo, 3);
        f[0] = q * u2[0];
        f[1] = q * u2[1];
        f[2] = 1.0;
        f[3] = rho * te;
        f[4] = tdl * rc - kap;
        f[5] = q;
      }
      double mine = 0.0;
#pragma unroll
      for (int i = 0; i < KIN_NX; ++i) {
        x[i] += h * f[i];
        finite = finite && isfinite(x[i]);
        mine = (i == lane) ? x[i] : mine;
      }
      s.xb[k + 1][lane < KIN_NX ? lane : KIN_NX] = mine;  // xb rows padded: col KIN_NX is a dummy
      // ey_{k+1} cost weight and linear term: stage (deviation + boundary,
      // kinematic_mpc.py:110-122) or terminal (:152-154)
      const double ey = x[3];
      double cw, lin;
      if (k + 1 < N) {
        const double hs = s.ds[k + 1];
        cw = W.w_dev * hs;
        lin = W.w_dev * hs * ey;
        if (ey < W.ey_min) { cw += W.w_b * hs; lin += W.w_b * hs * (ey - W.ey_min); }
        if (ey > W.ey_max) { cw += W.w_b * hs; lin += W.w_b * hs * (ey - W.ey_max); }
      } else {
        cw = W.w_ey;
        lin = W.w_ey * ey;
      }
      s.vc[k] = 2.0 * cw;
      s.vz[k] = 2.0 * lin;
    }
  }
  wave_sync();
  VC_TACC(T_SWEEP, t_sweep0)
  VC_TSTAMP(t_s20)
  {  // S2: lane k < N linearises stage k
    const int k = lane < N ? lane : 0;
    double xk[KIN_NX];
#pragma unroll
    for (int i = 0; i < KIN_NX; ++i) xk[i] = s.xb[k][i];
    const KinJac J = kin_spatial_jac(xk, s.kap[k], A.L);
    double* jr = s.jac[lane < N ? lane : N];  // row N: dummy
    jr[0] = J.q; jr[1] = J.qv; jr[2] = J.qey; jr[3] = J.qep;
    jr[4] = J.J33; jr[5] = J.J34; jr[6] = J.J41; jr[7] = J.J43; jr[8] = J.J44;
    // obstacle barrier of stage k = 1..N-1 (kinematic_mpc.py:130-133) as a convexified
    // quadratic in ey_k: adds to the ey_k weight / linear term S1 left in vc/vz[k-1]
    if (A.obs.n > 0 && lane >= 1 && lane < N) {
      double p, q;
      obstacle_ey_model<double>(A.obs, xk[2], xk[3], W.w_obs * s.ds[k], p, q);
      s.vc[k - 1] += q;
      s.vz[k - 1] += p;
    }
  }
  wave_sync();
  VC_TACC(T_S2, t_s20)
  VC_TSTAMP(t_s30)
  double gj = 0.0;
  double cv = 0, cd = 0, cey = 0, cep = 0, ct = 0;
  {  // S3
    const int jcol = lane < n ? lane : n;  // lanes >= n write the padding column
    double jn[9], hn, an, wn;
    auto fetch = [&](int k) {
#pragma unroll
      for (int q = 0; q < 9; ++q) jn[q] = s.jac[k][q];
      hn = s.ds[k]; an = s.ub[2 * k]; wn = s.ub[2 * k + 1];
    };
    fetch(0);
#pragma unroll 1
    for (int k = 0; k < N; ++k) {
      double J[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) J[q] = jn[q];
      const double h = hn, a = an, w = wn;
      const double lin2 = s.vz[k];
      if (k + 1 < N) fetch(k + 1);
      // c_{k+1} = A_k c_k + B_k e_j
      const double dq = J[1] * cv + J[2] * cey + J[3] * cep;
      const double ncv = cv + h * a * dq + (lane == 2 * k ? h * J[0] : 0.0);
      const double ncd = cd + h * w * dq + (lane == 2 * k + 1 ? h * J[0] : 0.0);
      const double ncey = cey + h * (J[4] * cey + J[5] * cep);
      const double ncep = cep + h * (J[6] * cd + J[7] * cey + J[8] * cep);
      ct += h * dq;
      cv = ncv; cd = ncd; cey = ncey; cep = ncep;
      // rows of stage k+1: v and delta constraint rows (k+1 <= N-1), ey cost row
      const bool has = k + 1 <= N - 1;  // stage N has no constraint rows: dummy row
      s.G[has ? k : NC + 2][jcol] = cv;
      s.G[has ? (N - 1) + k : NC + 2][jcol] = cd;
      E[k * LD + jcol] = cey;
      gj += lin2 * cey;
    }
    // terminal rows on v_N (kinematic_mpc.py:144-148) and epsi_N (:155-157)
    E[N * LD + jcol] = cv;
    E[(N + 1) * LD + jcol] = cep;
  }
  wave_sync();
  VC_TACC(T_S3, t_s30)
  VC_TSTAMP(t_s40)
  double Hr[n];
  double hjj;  // this lane's H[j][j]
  {  // S4: H = E' diag(w) E on the matrix cores (gram_mfma over the ey rows and the terminal rows)
    const double vN = s.xb[N][0];
    const double cwv = (vN >= W.v_max) ? W.w_v : 0.0;
    gj += 2.0 * cwv * (vN - W.v_max) * cv;
    gj += 2.0 * W.w_epsi * s.xb[N][4] * cep;
    gj += W.w_time * ct;  // t_N (:149-151)
    // weights of the terminal v_N (:144-148) and epsi_N (:155-157) rows, then two zero rows
    if (lane < 4) s.vc[N + lane] = lane == 0 ? 2.0 * cwv : (lane == 1 ? 2.0 * W.w_epsi : 0.0);
    for (int i = lane; i < 2 * LD; i += 64) E[(N + 2) * LD + i] = 0.0;
    wave_sync();
    // every tile: H is kept whole in LDS (the residual's H z reads full rows)
    d4 acc[Tiles<N>::count(true)];
#pragma unroll
    for (int t = 0; t < Tiles<N>::count(true); ++t) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
    gram_mfma<N, ROWS_E, true>(acc, E, &s.vc[0], lane);
    tiles_to_rows<N, true>(Hr, acc, s, lane);
  }
  // input costs: w_w w^2 (kinematic_mpc.py:124), slew w_a (a_{n+1}-a_n)^2 (:126-128), prox
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
  gj = (lane < n) ? gj : 0.0;
  {
    const int j = lane < n ? lane : n;  // lanes >= n write the dummy row
#pragma unroll
    for (int i = 0; i < n; ++i) s.H[j][i] = Hr[i];
    s.H[j][n] = 0.0;  // zero column (normal-matrix padding)
    // the input-cost band through this lane's own row in LDS (in issue order after the row
    // store; a register add would need a lane-index select on all n entries); 0 where absent
    s.H[j][j] += dself;
    s.H[j][j >= 2 ? j - 2 : j] += dm2;
    s.H[j][j + 2 < n ? j + 2 : j] += dp2;
    hjj = lane < n ? s.H[j][j] : 0.0;
  }
  wave_sync();
  if (A.mode == 1) {  // vc_condense: expose the QP data of the fused kernel
    if (lane < n) {
#pragma unroll
      for (int i = 0; i < n; ++i) A.H_out[((size_t)b * n + lane) * n + i] = s.H[lane][i];
      A.g_out[(size_t)b * n + lane] = gj;
    }
    return;
  }

  VC_TACC(T_S4, t_s40)
  VC_TSTAMP(t_setup0)
  // ---- inequality data ------------------------------------------------------
  Side bx, cs;  // box side (lane j < n), state-row side (lane r < NC)
  {
    const bool isw = lane & 1;
    const double u = (lane < n) ? s.ub[lane] : 0.0;
    bx.lo = (isw ? W.w_min : W.a_min) - u;
    bx.hi = (isw ? W.w_max : W.a_max) - u;
    const double tr = isw ? A.qp.trust_w : A.qp.trust_a;  // trust region (SQP globalisation), 0 = off
    if (tr > 0.0) {
      bx.lo = fmax(bx.lo, -tr);
      bx.hi = fmin(bx.hi, tr);
    }
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
    hdiag_max = fmax(wave_max(hjj), 1.0);
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

  VC_TACC(T_SETUP, t_setup0)
  // ---- Phase 1: Mehrotra predictor-corrector interior point ------------------
  // Normal equations (H + diag(wb) + G'diag(wc)G) dz = rhs, one factorisation and
  // two solves (predictor, corrector) per iteration.
  const int max_iter = A.qp.max_iter;
  const double tol = A.qp.tol * scale;
  int it = 0;
  bool converged = false, chol_fail = false, near = false;
  double last_res = 0.0, last_mu = 0.0;
  double Mr[n];
  // Residuals: dual rd = H z + g + C' lambda (lane j < n), primal r = C z + s - d per row side.
  // Computed once at the start point and then carried by the step -- the
  // direction solves the linearised KKT system, whose dual and primal rows are linear, so a step
  // of length al scales every residual by (1 - al) exactly (H dz + wb dz + eb + G'(wc G dz + ec)
  // = -rd by the normal equations; d1 = dz + rlo_b etc. by construction).  That replaces three
  // matrix-vector products per iteration (G z, H z, G' lambda) by five multiplies; the oracle's
  // Mehrotra iteration with the same recursion takes the same iterations on the C2 batch and its
  // true residuals end at the same 9.4e-11 / 3.5e-12 (scaled), polish certifying all 1,024.
  // The carried values never end the loop on their own: once they pass the stopping test the
  // true residuals are recomputed from z, lambda and decide (the normal-equation solves are not
  // exact, so the true residual stalls at a level set by the condition number, and a carried
  // value that drifted below it must not certify convergence -- nor land in diag[0]).
  double rd = 0.0, rlo_b = 0.0, rhi_b = 0.0, rlo_c = 0.0, rhi_c = 0.0;
  auto true_residuals = [&]() {
    wave_sync();
    s.vz[lane] = (lane < n) ? z : 0.0;
    s.vc[lane] = (lane < NC) ? (cs.lhi - cs.llo) : 0.0;
    wave_sync();
    const double yc = grow_dot<N>(s, lane);
    rd = (lane < n) ? (h_dot<N>(s, lane) + gj + (bx.lhi - bx.llo) + gt_dot<N>(s, lane)) : 0.0;
    rlo_b = bx.hasLo ? (z - bx.lo - bx.slo) : 0.0;
    rhi_b = bx.hasHi ? (bx.hi - z - bx.shi) : 0.0;
    rlo_c = cs.hasLo ? (yc - cs.lo - cs.slo) : 0.0;
    rhi_c = cs.hasHi ? (cs.hi - yc - cs.shi) : 0.0;
  };
  auto max_residual = [&]() {
    return wave_max(fmax(fmax(fabs(rd), fmax(fabs(rlo_b), fabs(rhi_b))), fmax(fabs(rlo_c), fabs(rhi_c))));
  };
  int tapb = 0;  // Tapia indicators: two bits per constraint side (1 active, 2 inactive, 0 undecided)
  // KIN_EARLY_F: the polish is first tried once the interior point reaches tol_early; if that
  // attempt does not certify within KIN_EARLY_ROUNDS rounds the interior point resumes from its
  // iterate (the polish changes none of its state) to tol and the polish runs again.  With the
  // Tapia guess 99.6 % of the C2 problems certify at 100 x tol, 1.15 interior-point iterations
  // earlier on average (scripts/early_polish_study.py).
  const double tol_early = KIN_EARLY_F > 0.0 ? fmax(tol, KIN_EARLY_F * tol) : tol;
  int e_set = 0;  // per lane: 256 | the early attempt's last set (bits 0..3) | that set changed (bits 4..7)
#ifdef VC_TIMING
  uint64_t e_fmask = 0;
  bool e_row = false, e_have = false;
#endif
  double tol_cur = tol_early;
  bool polished = false, pchol_fail = false;
  int rounds = 0;
#pragma unroll 1
  for (;;) {
  if (finite) {
#pragma unroll 1
    for (;;) {
      no_hoist();
      VC_TSTAMP(t_res0)
      if (it == 0) true_residuals();
      const double mu = wave_sum(bx.slo * bx.llo + bx.shi * bx.lhi + cs.slo * cs.llo + cs.shi * cs.lhi) / mtot;
      double res = max_residual();
      if (it > 0 && res <= tol_cur && mu <= tol_cur) {
        true_residuals();  // the carried residual would stop here: the true one decides
        res = max_residual();
      }
      converged = res <= tol_cur && mu <= tol_cur;
      last_res = res;
      last_mu = mu;
      if (converged || it >= max_iter || !isfinite(res) || !isfinite(mu)) break;
      ++it;
      const double wlo_b = bx.hasLo ? bx.llo / bx.slo : 0.0;
      const double whi_b = bx.hasHi ? bx.lhi / bx.shi : 0.0;
      const double wlo_c = cs.hasLo ? cs.llo / cs.slo : 0.0;
      const double whi_c = cs.hasHi ? cs.lhi / cs.shi : 0.0;
      wave_sync();
      s.vc[lane] = (lane < NC) ? wlo_c + whi_c : 0.0;
      wave_sync();
      VC_TACC(T_RESID, t_res0)
      VC_TSTAMP(t_build0)
      d4 nacc[Tiles<N>::NT];
      build_normal_acc<N>(nacc, s, wlo_b + whi_b, hjj, lane);
      VC_TACC(T_BUILD, t_build0)
      VC_TSTAMP(t_chol0)
      const bool chol_ok = factor_blocked<N>(Mr, nacc, s, lane);
      VC_TACC(T_CHOL, t_chol0)
      if (!chol_ok) {
        // The barrier weights lambda/s of the active set (~1/mu) have made the
        // normal matrix numerically indefinite.  This happens only at the very
        // end (mu ~ 1e-14); the iterate is then accurate enough for the
        // active-set polish to identify and solve the exact optimum.
        chol_fail = true;
        near = res <= 1e-6 * scale && mu <= tol;
        break;
      }
      // inverse slacks / multipliers of this iteration (0 on absent sides): the two passes
      // divide by them 16 times, and the fraction to the boundary min over -v/dv (dv < 0)
      // is 1 / max over -dv (1/v)
      const double islo_b = bx.hasLo ? rcp_nr(bx.slo) : 0.0, ishi_b = bx.hasHi ? rcp_nr(bx.shi) : 0.0;
      const double islo_c = cs.hasLo ? rcp_nr(cs.slo) : 0.0, ishi_c = cs.hasHi ? rcp_nr(cs.shi) : 0.0;
      const double illo_b = bx.hasLo ? rcp_nr(bx.llo) : 0.0, ilhi_b = bx.hasHi ? rcp_nr(bx.lhi) : 0.0;
      const double illo_c = cs.hasLo ? rcp_nr(cs.llo) : 0.0, ilhi_c = cs.hasHi ? rcp_nr(cs.lhi) : 0.0;
      double sm = 0.0, pp1 = 0.0, pp2 = 0.0, pp3 = 0.0, pp4 = 0.0;
#pragma unroll 1
      for (int pass = 0; pass < 2; ++pass) {
        no_hoist();
        // complementarity residuals: affine (pass 0), Mehrotra corrector (pass 1)
        const double rclo_b = bx.slo * bx.llo + pp1 - sm, rchi_b = bx.shi * bx.lhi + pp2 - sm;
        const double rclo_c = cs.slo * cs.llo + pp3 - sm, rchi_c = cs.shi * cs.lhi + pp4 - sm;
        const double eb = (bx.hasHi ? (-rchi_b * ishi_b - whi_b * rhi_b) : 0.0) +
                          (bx.hasLo ? (rclo_b * islo_b + wlo_b * rlo_b) : 0.0);
        const double ec = (cs.hasHi ? (-rchi_c * ishi_c - whi_c * rhi_c) : 0.0) +
                          (cs.hasLo ? (rclo_c * islo_c + wlo_c * rlo_c) : 0.0);
        wave_sync();
        s.vc[lane] = (lane < NC) ? ec : 0.0;
        wave_sync();
        const double rhs = (lane < n) ? (-rd - eb - gt_dot<N>(s, lane)) : 0.0;
        VC_TSTAMP(t_sol0)
        const double dz = chol_solve<N>(Mr, s, rhs, lane);
        VC_TACC(T_SOLVE, t_sol0)
        wave_sync();
        s.vz[lane] = (lane < n) ? dz : 0.0;
        wave_sync();
        const double dyc = grow_dot<N>(s, lane);
        const double d1 = bx.hasLo ? dz + rlo_b : 0.0;
        const double d2 = bx.hasLo ? (-rclo_b * islo_b - wlo_b * (dz + rlo_b)) : 0.0;
        const double d3 = bx.hasHi ? rhi_b - dz : 0.0;
        const double d4 = bx.hasHi ? (-rchi_b * ishi_b - whi_b * (rhi_b - dz)) : 0.0;
        const double e1 = cs.hasLo ? dyc + rlo_c : 0.0;
        const double e2 = cs.hasLo ? (-rclo_c * islo_c - wlo_c * (dyc + rlo_c)) : 0.0;
        const double e3 = cs.hasHi ? rhi_c - dyc : 0.0;
        const double e4 = cs.hasHi ? (-rchi_c * ishi_c - whi_c * (rhi_c - dyc)) : 0.0;
        const double tmax = wave_max(fmax(fmax(fmax(-d1 * islo_b, -d2 * illo_b), fmax(-d3 * ishi_b, -d4 * ilhi_b)),
                                          fmax(fmax(-e1 * islo_c, -e2 * illo_c), fmax(-e3 * ishi_c, -e4 * ilhi_c))));
        const double amax = 1.0 / fmax(1.0, tmax);  // largest a in (0, 1] keeping every v + a dv >= 0
        if (pass == 0) {
          const double mua = wave_sum((bx.slo + amax * d1) * (bx.llo + amax * d2) +
                                      (bx.shi + amax * d3) * (bx.lhi + amax * d4) +
                                      (cs.slo + amax * e1) * (cs.llo + amax * e2) +
                                      (cs.shi + amax * e3) * (cs.lhi + amax * e4)) / mtot;
          const double sr = mua / mu;
          sm = sr * sr * sr * mu;  // sigma * mu with sigma = (mu_aff / mu)^3
          pp1 = d1 * d2; pp2 = d3 * d4; pp3 = e1 * e2; pp4 = e3 * e4;
        } else {
          const double al = KIN_STEP_F * amax;
          {
            // Tapia indicators of this step (El-Bakry, Tapia, Tsuchiya, Zhang 1996): near the
            // solution an active side's slack shrinks by a factor the multiplier does not, an
            // inactive side's multiplier the other way round -- with the interior point's loose
            // stopping rule (mu <= 1e-10 scale) weakly active bounds still have slacks ~1e-3 above
            // their multipliers, and lambda > s misses them (122 of the 1,024 C2 problems, each a
            // polish round; scripts/polish_cg_study.py).  il, is: 1 / the pre-step values.
            auto tap = [&](double dl, double il, double dsv, double is) -> int {
              const double lr = fma(al * dl, il, 1.0), sr = fma(al * dsv, is, 1.0);
              return lr > KIN_TAPIA_F * sr ? 1 : (sr > KIN_TAPIA_F * lr ? 2 : 0);
            };
            tapb = tap(d2, illo_b, d1, islo_b) | (tap(d4, ilhi_b, d3, ishi_b) << 2) |
                   (tap(e2, illo_c, e1, islo_c) << 4) | (tap(e4, ilhi_c, e3, ishi_c) << 6);
          }
          z = (lane < n) ? z + al * dz : z;
          bx.slo += al * d1; bx.llo += al * d2; bx.shi += al * d3; bx.lhi += al * d4;
          cs.slo += al * e1; cs.llo += al * e2; cs.shi += al * e3; cs.lhi += al * e4;
          const double om = 1.0 - al;
          rd *= om; rlo_b *= om; rhi_b *= om; rlo_c *= om; rhi_c *= om;
        }
      }
    }
  }

  VC_TSTAMP(t_pol0)
  // ---- Phase 2: active-set polish --------------------------------------------
  // Crossover to the active set the interior point identified (lambda > s):
  // box-active inputs are fixed (identity rows), active state rows are imposed
  // with an augmented Lagrangian (P + rho C_A'C_A) whose multiplier update
  // converges in a few solves with one factorisation.  The candidate is accepted
  // when it is primal and dual feasible to ptol; otherwise ONE constraint is
  // changed per round -- the most negative multiplier dropped, else the most
  // violated constraint added (oracle/qp.py:polish uses the same rule with a
  // direct KKT solve).  If no candidate certifies within qp.polish rounds, the
  // converged interior-point iterate is kept.
  if ((converged || near) && A.qp.polish > 0) {
    constexpr double AL_RHO = KIN_AL_RHO;
    constexpr int AL_MAX = 16;
    const double ptol = 1e-9 * scale, dtol = KIN_DUAL_TOL * scale;
    // decisive indicators first, lambda > s where the last step left them undecided
    auto guess = [&](bool has, double l, double sv, int t) { return has && (t == 1 || (t == 0 && l > sv)); };
    bool alo_b = guess(bx.hasLo, bx.llo, bx.slo, tapb & 3);
    bool ahi_b = guess(bx.hasHi, bx.lhi, bx.shi, (tapb >> 2) & 3);
    bool alo_c = guess(cs.hasLo, cs.llo, cs.slo, (tapb >> 4) & 3);
    bool ahi_c = guess(cs.hasHi, cs.lhi, cs.shi, (tapb >> 6) & 3);
    auto pack = [&]() { return int(alo_b) | (int(ahi_b) << 1) | (int(alo_c) << 2) | (int(ahi_c) << 3); };
    // The final attempt's guess repeats the set the failed early attempt factored last (problems 153
    // and 855 of the C2 batch): that round's outcome is known -- the equality-constrained optimum of
    // a set does not depend on the interior-point iterate -- so start from the set it changed to
    // (153: 388 K -> 360 K cycles, 855: 377 K -> 358 K; C2 -0.6 %; profiles/r06/kin_ab/kin_polish_*_r06za.*)
    if (tol_cur <= tol && __ballot(e_set != 0 && pack() != (e_set & 15)) == 0ull && __ballot(e_set != 0) != 0ull) {
      const int t = e_set >> 4;
      alo_b = t & 1; ahi_b = (t >> 1) & 1; alo_c = (t >> 2) & 1; ahi_c = (t >> 3) & 1;
    }
    // (more early rounds, now that most rounds after the first are rank-one updates, lose: up to 3 / 4 / 6
    // while each further round is an update, C2 +7 %, problem 260 adds a wrong bound and drops it again;
    // profiles/r06/kin_ab/kin_polish_ab_c2_r06u.log)
    const int max_rounds = tol_cur > tol ? min(A.qp.polish, KIN_EARLY_ROUNDS) : A.qp.polish;
    // KIN_UPDATE: the weight the current factor holds for state row `lane` (0: none), and how the
    // last round changed the active set (uniform; 1: variable upd_j fixed, 2: row upd_j added,
    // 0: anything else -- a dropped bound or row, or no factor yet -- which refactors)
    double rho_k = 0.0;
    int upd = 0, upd_j = 0;
#pragma unroll 1
    for (int round = 0; round < max_rounds; ++round) {
      no_hoist();
      const int set0 = pack();  // this round's set (bits 0..3), for the carry above
#ifdef VC_TIMING
      if (round == 0 && tol_cur <= tol && e_have) {
        const bool fx = (lane < n) && (alo_b || ahi_b);
        const uint64_t fm = __ballot(fx);
        const bool ract = (lane < NC) && (alo_c || ahi_c);
        tacc[T_CFAIL] = 1;
        tacc[T_CRM] = __builtin_popcountll(e_fmask & ~fm) + __builtin_popcountll(__ballot(e_row && !ract));
        tacc[T_CADD] = __builtin_popcountll(fm & ~e_fmask) + __builtin_popcountll(__ballot(ract && !e_row));
      }
#endif
      ++rounds;  // over both attempts (diag[3]; bench.py prices each round as an iteration)
      const bool fixed = (lane < n) && (alo_b || ahi_b);
      const double zfix = fixed ? (alo_b ? bx.lo : bx.hi) : 0.0;
      const uint64_t fmask = __ballot(fixed);
      const bool act = (lane < NC) && (alo_c || ahi_c);
      wave_sync();
      s.vz[lane] = (lane < n) ? zfix : 0.0;
      wave_sync();
      // fixed-variable part of each active row, and its free-part norm for rho
      const double gfix = grow_dot<N>(s, lane);
      double gn2 = 0.0;
      {
        const int r = lane < NC ? lane : 0;
#pragma unroll 2
        for (int i = 0; i < 2 * (N - 1); ++i) {
          const double gi = ((fmask >> i) & 1ull) ? 0.0 : s.G[r][i];
          gn2 += gi * gi;
        }
      }
      const double rho_new = (act && gn2 > 1e-28) ? AL_RHO * hdiag_max / gn2 : 0.0;
      // a row the factor already holds keeps its weight (any positive weight has the same fixed
      // point), so fixing a variable leaves the matrix one rank-one update away (factor_update)
      const double rho_c = (KIN_UPDATE && rho_k > 0.0 && rho_new > 0.0) ? rho_k : rho_new;
      const double bnd_c = act ? ((alo_c ? cs.lo : cs.hi) - gfix) : 0.0;  // b' = b - G_X zfix
      const double base = (lane < n) ? -(gj + h_dot<N>(s, lane)) : 0.0;
      wave_sync();
      s.vc[lane] = rho_c;
      wave_sync();
      VC_TSTAMP(t_pf0)
      bool updated = false;
      if (KIN_UPDATE && upd != 0) {  // uniform
        // every row but the added one kept its weight (else refactor)
        const bool same = __ballot(lane < NC && rho_c != rho_k && !(upd == 2 && lane == upd_j)) == 0ull;
        VC_TSTAMP(t_u0)
        if (same) updated = factor_update<N>(Mr, s, upd, upd_j, fixed, sqrt(lane_bcast(rho_c, upd_j)), lane);
#ifdef VC_TIMING
        if (updated) tacc[T_NUPD] += 1;
#endif
        VC_TACC(T_UCYC, t_u0)
      }
      rho_k = rho_c;
      if (!updated) {
        // the interior point's path: H + G' diag(rho_c) G in the accumulator tiles (s.vc =
        // rho_c; zero weights where no row is active), fixed rows / columns set to the identity
        // in the tiles -- D (H + G'WG) D + (I - D) with D the free-variable mask equals the
        // reduced matrix H_FF + G_F' W G_F -- and the blocked factorisation (matrix-core panel
        // updates) instead of the row-per-lane one
        d4 pacc[Tiles<N>::NT];
        build_normal_acc<N>(pacc, s, 0.0, hjj, lane);
        const int pl = lane_opaque(lane), plr = pl >> 4, plc = pl & 15;  // not hoisted out of the rounds
#pragma unroll
        for (int I = 0, t = 0; I < Tiles<N>::NB; ++I) {
#pragma unroll
          for (int J = 0; J <= I; ++J, ++t) {
            const int c = 16 * J + plc;
            const bool fc = (fmask >> c) & 1ull;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = 16 * I + plr + 4 * q;
              const bool fr = (fmask >> r) & 1ull;
              pacc[t][q] = (fr || fc) ? (r == c ? 1.0 : 0.0) : pacc[t][q];
            }
          }
        }
        if (!factor_blocked<N>(Mr, pacc, s, lane)) {
          pchol_fail = true;
          break;
        }
      }
      VC_TACC(T_UPDATE, t_pf0)
      VC_TSTAMP(t_pal0)
      // multiplier estimate: the interior point's own (lambda_hi - lambda_lo of an active row,
      // the sign convention of the check below), so the augmented-Lagrangian passes start next
      // to the fixed point instead of at 0 (the fixed point does not depend on
      // the start: same certified z).  Rows the AL does not enforce (rho_c = 0) keep 0.
      double nu_c = (act && rho_c > 0.0) ? ((ahi_c ? cs.lhi : 0.0) - (alo_c ? cs.llo : 0.0)) : 0.0;

      // The passes are Richardson's iteration nu += R e on S dnu = e(nu), S = G_A M^-1 G_A' (M the
      // factored matrix, R = diag(rho_c)): it contracts by 1 - min eig(R S) per pass, up to 14 passes
      // on the slowest C2 problems (profiles/r04/sec_r04f.txt).  Conjugate gradients solve the same
      // system by conjugate gradients preconditioned with R -- same cost per iteration (one
      // triangular solve pair, one G' and one G product), same fixed point, and R S has its
      // eigenvalues clustered below 1, so CG needs a few.  z follows nu exactly: dz = -M^-1 G' dnu.
      const bool al_act = act && rho_c > 0.0;
      const double bnd_al = alo_c ? cs.lo : cs.hi;
      double zp = 0.0, emax = 0.0;
      {
        wave_sync();
        s.vc[lane] = (lane < NC) ? (nu_c - rho_c * bnd_c) : 0.0;
        wave_sync();
        const double rhs = (lane < n) ? (fixed ? zfix : (base - gt_dot<N>(s, lane))) : 0.0;
        zp = chol_solve<N>(Mr, s, rhs, lane);
        wave_sync();
        s.vz[lane] = (lane < n) ? zp : 0.0;
        wave_sync();
        const double yr = grow_dot<N>(s, lane);
        double rr = al_act ? (yr - bnd_al) : 0.0;  // e(nu), the active rows' violation
        // stop when the violation is below 1e-14 scale and (KIN_NU_TOL) the multiplier step R e
        // below KIN_NU_TOL scale: rho_c reaches 1e10 on rows with a small free part, and a
        // violation at rounding level then still leaves multipliers off by more than the dual
        // check's 1e-9 scale -- the active set cycled (two C2-like problems of 4,096, seed 7)
        const double ie = 1.0 / (1e-14 * scale), inu = KIN_NU_TOL > 0.0 ? 1.0 / (KIN_NU_TOL * scale) : 0.0;
        auto crit = [&](double r) { return wave_max(fmax(fabs(r) * ie, fabs(rho_c * r) * inu)); };
#ifdef VC_TIMING
        tacc[T_PPASS] += 1;
#endif
        if (crit(rr) > 1.0) {
          double pd = rho_c * rr;  // preconditioned residual = first direction
          double rz = wave_sum(rr * pd);
#pragma unroll 1
          for (int it = 1; it < AL_MAX; ++it) {
            no_hoist();
            wave_sync();
            s.vc[lane] = (lane < NC) ? pd : 0.0;
            wave_sync();
            const double gtp = gt_dot<N>(s, lane);
            const double zq = chol_solve<N>(Mr, s, (lane < n && !fixed) ? gtp : 0.0, lane);  // M^-1 G' p
            wave_sync();
            s.vz[lane] = (lane < n) ? zq : 0.0;
            wave_sync();
            const double gq = grow_dot<N>(s, lane);
            const double q = al_act ? gq : 0.0;  // S p on the active rows
            const double pq = wave_sum(pd * q);
#ifdef VC_TIMING
            tacc[T_PPASS] += 1;
#endif
            if (!(pq > 0.0)) break;  // uniform: a direction S does not see (the KKT check decides)
            const double al = rz / pq;
            nu_c = fma(al, pd, nu_c);
            zp = fma(-al, zq, zp);
            rr = fma(-al, q, rr);
            if (crit(rr) <= 1.0) break;
            const double zt = rho_c * rr;
            const double rzn = wave_sum(rr * zt);
            pd = fma(rzn / rz, pd, zt);
            rz = rzn;
          }
        }
      }
      VC_TACC(T_PAL, t_pal0)
      // KKT check of zp
      wave_sync();
      s.vz[lane] = (lane < n) ? zp : 0.0;
      s.vc[lane] = (lane < NC) ? nu_c : 0.0;
      wave_sync();
      const double grad = (lane < n) ? (h_dot<N>(s, lane) + gj + gt_dot<N>(s, lane)) : 0.0;
      const double ypc = grow_dot<N>(s, lane);
      // the true violation, not CG's recurrence -- and, with KIN_STAT_CHECK, the free variables'
      // stationarity (the solves are trusted to make it ~0; a factor gone inaccurate must not certify)
#if KIN_STAT_CHECK
      emax = wave_max(fmax(al_act ? fabs(ypc - bnd_al) : 0.0, (lane < n && !fixed) ? fabs(grad) : 0.0));
#else
      emax = wave_max(al_act ? fabs(ypc - bnd_al) : 0.0);
#endif
      // dual violations (> 0 is wrong-signed): box multiplier of an active bound is
      // -grad (upper) / grad (lower); state-row multiplier is nu (upper) / -nu (lower)
      const double dv_b = (lane < n) ? (ahi_b ? grad : (alo_b ? -grad : -1.0)) : -1.0;
      const double dv_c = (lane < NC) ? (ahi_c ? -nu_c : (alo_c ? nu_c : -1.0)) : -1.0;
      // primal violations of the inactive constraints
      const double pv_b = (lane < n && !fixed) ? fmax(bx.lo - zp, zp - bx.hi) : -1.0;
      // every row the equality solve does not enforce is checked against its bounds: the inactive
      // ones, and active ones without a free variable (rho_c = 0: fixed inputs alone decide them --
      // unchecked, an early attempt's guess certified a point 9e-3 off the optimum, C4 problem 23921)
      const double pv_c = (lane < NC && !(act && rho_c > 0.0))
                              ? fmax(cs.hasLo ? cs.lo - ypc : -1.0, cs.hasHi ? ypc - cs.hi : -1.0)
                              : -1.0;
      const double dmax = wave_max(fmax(dv_b, dv_c));
      const double pmax = wave_max(fmax(pv_b, pv_c));
      if (dmax <= dtol && pmax <= ptol) {
        if (emax <= ptol) {
          z = (lane < n) ? zp : z;
          polished = true;
        }
        break;  // certified, or the equality solve did not converge: keep the IPM iterate
      }
      // change one constraint: the lowest lane holding the worst violation
      const bool dual = dmax > dtol;
      const double worst = dual ? dmax : pmax;
      const double vb = dual ? dv_b : pv_b, vcr = dual ? dv_c : pv_c;
      const uint64_t who = __ballot(fmax(vb, vcr) == worst);
      const int sel = __builtin_ffsll((long long)who) - 1;
      const bool sel_box = (__ballot(vb >= vcr) >> sel) & 1ull;
      upd = dual ? 0 : (sel_box ? 1 : 2);  // an added bound fixes variable sel, an added row is row sel
      upd_j = sel;
#ifdef VC_TIMING
      if (dual) tacc[T_NDROP] += 1;
#endif
      if (lane == sel) {
        if (vb >= vcr) {  // box constraint of input `lane`
          if (dual) { alo_b = false; ahi_b = false; }
          else if (zp < bx.lo) alo_b = true;
          else ahi_b = true;
        } else {          // state row `lane`
          if (dual) { alo_c = false; ahi_c = false; }
          else if (ypc < cs.lo) alo_c = true;
          else ahi_c = true;
        }
      }
#ifdef VC_TIMING
      int r0code = 0;
      if (tol_cur > tol && round == 0) {
        int tside = 0;
        if (vb >= vcr) tside = (dual ? (ahi_b ? (tapb >> 2) : tapb) : (zp < bx.lo ? tapb : (tapb >> 2))) & 3;
        else tside = (dual ? (ahi_c ? (tapb >> 6) : (tapb >> 4)) : (ypc < cs.lo ? (tapb >> 4) : (tapb >> 6))) & 3;
        const int code = 1 + (dual ? 2 : (vb >= vcr ? 0 : 1)) + 3 * tside;
        r0code = __builtin_amdgcn_readlane(code, sel);
#ifdef VC_TIMING
        tacc[T_R0CHG] = (uint64_t)r0code;
#endif
      }
#endif
      if (tol_cur > tol) e_set = 256 | set0 | (pack() << 4);  // early attempt: this round's set and its change
      // (ending the early attempt after its first change by the change's kind and the changed side's
      // Tapia state does not separate the attempts that fail: C2 +1 / +5 / +3 % for undecided adds / all
      // adds / drops, profiles/r06/kin_ab/kin_polish_ab_c2_r06zd.log; on 16,384 problems 262 of 282
      // first changes "box add, Tapia inactive" certify in the next round, kin_polish_sec16k_r06zd.txt)
#ifdef VC_TIMING
      if (tol_cur > tol) {  // the early attempt's last factored set (this round's)
        e_fmask = fmask;
        e_row = rho_k > 0.0;
        e_have = true;
      }
#endif
    }
  }

  VC_TACC(T_POLISH, t_pol0)
  // (a polish factorisation that fails also resumes: the interior point's state is intact)
  if (polished || !converged || chol_fail || tol_cur <= tol) break;
  tol_cur = tol;  // the early attempt did not certify: back to the interior point
  converged = false;
  pchol_fail = false;
  }
  VC_TSTAMP(t_out0)
  // ---- outputs -------------------------------------------------------------------
  int32_t st;
  if (!finite) st = VC_NONFINITE;
  else if (polished || converged) st = VC_SOLVED;
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
    if (A.diag) {
#ifdef VC_TIMING
      constexpr size_t DS = 4 + T_NSLOT;
#else
      constexpr size_t DS = 4;
#endif
      A.diag[(size_t)b * DS + 0] = last_res / scale;
      A.diag[(size_t)b * DS + 1] = last_mu / scale;
      A.diag[(size_t)b * DS + 2] = double((chol_fail ? 1 : 0) | (converged ? 2 : 0) | (polished ? 4 : 0) |
                                          (pchol_fail ? 8 : 0));
      A.diag[(size_t)b * DS + 3] = double(rounds);
    }
  }
  // x* = xbar + G dz via the linearised recursion, lanes 0..5 own components
  double dx[KIN_NX] = {0, 0, 0, 0, 0, 0};
  double* xo = A.x_out + (size_t)b * (N + 1) * KIN_NX;
  if (lane < KIN_NX) xo[lane] = s.xb[0][lane];
#pragma unroll 1
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
  // (reading each step's LDS operands a step ahead, S3's pattern, measured equal: C2 0.2090 vs
  // 0.2097 ms, profiles/r06/kin_ab/kin_polish_ab_c2_r06z.log -- the section is not LDS-latency bound)
  VC_TACC(T_OUT, t_out0)
#ifdef VC_TIMING
  // timing builds: diag is [B][4 + T_NSLOT]
  if (A.diag && lane < T_NSLOT) {
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < T_NSLOT; ++i) v = (i == lane) ? double(tacc[i]) : v;
    A.diag[(size_t)b * (4 + T_NSLOT) + 4 + lane] = v;
  }
#endif
}

// ---- host launcher ---------------------------------------------------------------
size_t kin_ltv_smem_bytes(int N) {
  switch (N) {
    case 20: return sizeof(Smem<20>);
    default: return 0;
  }
}

hipError_t launch_kin_ltv(const KinLtvArgs& a, int N, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  switch (N) {
    case 20:
      hipLaunchKernelGGL(kin_ltv_kernel<20>, dim3(a.B), dim3(64), 0, stream, a);
      return hipGetLastError();
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vc
