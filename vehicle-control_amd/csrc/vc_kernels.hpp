// vc_kernels.hpp -- kernel argument blocks and launchers shared by the .hip units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "vc_models.hpp"
#include "vcmpc.h"

// Columns of vc_solve_diag's diag rows, per kernel family: 4 diagnostics, plus the
// section-cycle counters in the VC_TIMING build (make timing).
#ifdef VC_TIMING
#define VC_DIAG_COLS 16      // 4 diagnostics + 12 section-cycle counters (kin_ltv.hip T_*)
#define VC_DYN_DIAG_COLS 19  // 4 diagnostics + 15 section-cycle counters (dyn_sqp.hip DT_*)
#define VC_CASC_DIAG_COLS 17 // 4 diagnostics + 13 section-cycle counters (casc_sqp.hip CT_*)
#define VC_ST_DIAG_COLS 13   // 4 diagnostics + 9 section-cycle counters (st_sqp.hip ST_*)
#else
#define VC_DIAG_COLS 4
#define VC_DYN_DIAG_COLS 4
#define VC_CASC_DIAG_COLS 4
#define VC_ST_DIAG_COLS 4
#endif

// Default floor of the obstacle barrier margin dist - (r + 0.1) [m] (vc_obstacles.margin_min).
#define VC_OBS_MARGIN_MIN 0.05

namespace vc {

// Problem owned by workgroup g of a one-workgroup-per-problem launch (grid = B).
// Workgroups are dealt round-robin over the 8 XCDs (g and g + 8 share one L2), so the
// identity mapping puts neighbouring problems -- whose rows of x0 / kappa / ds / the warm
// start share 128-B lines -- on different XCDs, and every shared line is fetched into
// (and written back from) two L2s.  This mapping gives XCD slot g % 8 the contiguous
// problem range [(g % 8) q, (g % 8 + 1) q), q = B / 8; the B % 8 tail keeps the identity.
// A bijection on [0, B); placement is a speed hint only (correctness never depends on it).
__device__ __forceinline__ int xcd_problem(int g, int B) {
  const int q = B >> 3;
  return g < 8 * q ? (g & 7) * q + (g >> 3) : g;
}

// Compute units of the current device (host side; the occupancy-driven kernel choices).
inline int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 256;
  return n > 0 ? n : 256;
}
// One-wave workgroups of an lds-byte block resident per CU (160 KB of LDS allocated in 512 B
// granules -- rocprofv3 LDS_Block_Size --, and at most one per SIMD: the solve kernels hold more
// than 256 VGPRs + AGPRs per lane).
constexpr int wg_per_cu(size_t lds) {
  const size_t g = (lds + 511) / 512 * 512, n = 163840 / (g ? g : 1);
  return n < 4 ? (int)n : 4;
}

// fp64 array in global memory addressed through a buffer resource: SGPR base + 32-bit VGPR byte
// offset (one VGPR per access instead of a 64-bit address pair -- the Riccati kernels have no
// registers to spare), and an offset at or past `bytes` reads 0 / drops the store instead of
// faulting.  (A pointer read out of the kernel-argument block has no known address space: plain
// loads through it become flat loads, which count against lgkmcnt too, so every LDS wait after
// them would also wait for global memory.)
struct GBuf {
  __amdgpu_buffer_rsrc_t r;
  // a base the compiler cannot prove uniform (read through a laundered kernel-argument pointer)
  // would put the descriptor in VGPRs and wrap every access in a readfirstlane loop: callers
  // pass it through uniform() first
  static __device__ __forceinline__ double* uniform(double* p) {
    const uint64_t u = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return (double*)(((uint64_t)hi << 32) | lo);
  }
  __device__ __forceinline__ GBuf(double* base, uint32_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000)) {}  // gfx9 raw buffer
  __device__ __forceinline__ double ld(uint32_t off) const {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  }

  __device__ __forceinline__ void st(uint32_t off, double v) const {
    typedef __attribute__((ext_vector_type(2))) unsigned u2;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, off, 0, 0);
  }
  // two adjacent doubles as one 16-byte store (off 16-byte aligned): where the lanes of one store
  // instruction cover whole 64-byte rows this way, each row leaves the CU as one full write instead
  // of several partial ones (the memory side counts a request per partial write: st_sqp's J went out
  // ~4x its size as 8-byte column stores, r05 PMC)
  __device__ __forceinline__ void st2(uint32_t off, double v0, double v1) const {
    typedef __attribute__((ext_vector_type(4))) unsigned u4;
    typedef __attribute__((ext_vector_type(2))) double d2v;
    const d2v v = {v0, v1};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, off, 0, 0);
  }
};

// 1/x to full fp64 accuracy: hardware v_rcp_f64 + two Newton steps (five VALU ops against
// the ~11-op div_scale / div_fmas / div_fixup sequence of an IEEE divide).  x = +-inf or 0
// (an unbounded row's slack, a zero step component) makes the Newton residual NaN; the
// hardware reciprocal is then the IEEE 1/x (0 or inf) and is returned as is, so products
// such as la * rcp_nr(sl) behave exactly like la / sl.  Used by kin_ltv only, whose interior
// slacks and multipliers are never floored: the Riccati kernels floor theirs at 1e-300,
// and the same substitution there made every step of st_sqp's Fiala closed loop fail
// (DESIGN 3.1), so they keep the IEEE divide (whose div_scale pre-scaling covers the
// full exponent range).
__device__ __forceinline__ double rcp_nr(double x) {
  const double r0 = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r0, 1.0);
  double r = fma(r0, e, r0);
  e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  return isfinite(r) ? r : r0;
}

// Domain of the spatial single-track model at one state (oracle/dyn_sqp.py in_domain): Ux > 0
// and s' = (Ux cos epsi - Uy sin epsi) / (1 - kappa ey) > 0 (dynamic_car.py:169-191 divides by
// s', the slip angles by Ux).  False for non-finite states.  The SQP kernels cut a step back
// (DOM_HALVINGS halvings, then no step) when its rollout leaves the domain.
constexpr int DOM_HALVINGS = 8;
template <typename T>
__device__ __forceinline__ bool dyn_in_domain(const T* x, T kappa) {
  const T sdot = (x[0] * cos(x[6]) - x[1] * sin(x[6])) / (T(1) - kappa * x[5]);
  return x[0] > T(0) && sdot > T(0);
}

// ... and of the point-mass tail (oracle/casc_sqp.py casc_in_domain): V > 0 and
// s' = V cos(epsi) / (1 - kappa ey) > 0 (dynamic_point_mass.py:90-100), p = (V, s, ey, epsi, t)
template <typename T>
__device__ __forceinline__ bool pm_in_domain(const T* p, T kappa) {
  const T sdot = p[0] * cos(p[3]) / (T(1) - kappa * p[2]);
  return p[0] > T(0) && sdot > T(0);
}

// Obstacle barrier of one stage as a convexified quadratic in ey:
//   phi(ey) = sum_j w ds / (d_j - (r_j + 0.1)),  d_j = |(s, ey) - (s_j, ey_j)|
// (kinematic_mpc.py:130-133, cascaded_mpc.py:173-176).  s is not a decision function
// (s' = 1 in both spatial models), so the term is one-dimensional in ey.  Returns the
// slope p = phi'(ey) and the curvature q = max(phi''(ey), 0), with the margin floored at
// margin_min.  Operation order mirrored by oracle/obstacles.py.
template <typename T>
__device__ __forceinline__ void obstacle_ey_model(const vc_obstacles& o, T s, T ey, T wds, T& p, T& q) {
  T ps = T(0), qs = T(0);
  const T mmin = T(o.margin_min);
  for (int j = 0; j < o.n; ++j) {
    const T a = s - T(o.s[j]);
    const T e = ey - T(o.ey[j]);
    const T d2 = a * a + e * e;
    const T d = sqrt(d2);
    const T dc = d > T(1e-6) ? d : T(1e-6);
    const T m0 = d - (T(o.radius[j]) + T(0.1));
    // floored at margin_min; with o.inside the reference's own (negative) barrier beyond the
    // band |m0| <= margin_min inside the obstacle (the slope w ds / m^2 is continuous at -mmin)
    const T m = (o.inside && m0 < -mmin) ? m0 : (m0 > mmin ? m0 : mmin);
    const T d1 = e / dc;                  // d'(ey)
    const T dd = (a * a) / (dc * dc * dc);  // d''(ey)
    const T im = T(1) / m;
    const T c1 = wds * im * im;           // w ds / m^2
    ps -= c1 * d1;
    qs += c1 * (T(2) * d1 * d1 * im - dd);
  }
  p = ps;
  q = qs > T(0) ? qs : T(0);
}

// Per-stage state rows of the Riccati SQP kernels (st_sqp.hip, casc_ric.hip): 8 doubles a row, row k
// rotated by k / 4 (element i of row k in slot (i + k / 4) mod 8).  A lane-per-stage read of one
// element then hits 32 distinct bank pairs over a 32-lane ds_read_b64 group (dword address
// 16 k + 2 ((i + k / 4) mod 8) mod 64: k mod 4 and k / 4 mod 8 both vary), where the plain stride of
// 8 doubles put lanes k and k + 4 on the same banks (8-way) and an odd stride of 9 costs a ninth
// double per stage -- at N = 60 / the cascaded H = 60 the difference between three workgroups per
// CU and two.
template <int R>
struct StageRows8 {
  double m[R][8];
  __device__ __forceinline__ double& at(int k, int i) { return m[k][(i + (k >> 2)) & 7]; }
  __device__ __forceinline__ const double& at(int k, int i) const { return m[k][(i + (k >> 2)) & 7]; }
};

// Fused kinematic LTV-MPC step (kin_ltv.hip, condensed, N = 20; kin_ric.hip, stagewise).
struct KinLtvArgs {
  const double* x0;     // [B][6]
  const double* kappa;  // [B][N]
  const double* ds;     // [B][N]
  const double* ubar;   // [B][N][2]  warm start (may alias u_out)
  double* u_out;        // [B][N][2]  u*
  double* x_out;        // [B][N+1][6] x*
  const double* x_in;   // [B][N+1][6] warm-start states (multiple shooting, qp.ms; may alias x_out)
  double* u0;           // [B][2]
  int32_t* status;      // [B]
  int32_t* iters;       // [B]
  double* diag;         // [B][4] optional solver diagnostics (vc_solve_diag), may be null
  double* H_out;        // [B][2N][2N]  (mode 1 only)
  double* g_out;        // [B][2N]      (mode 1 only)
  int mode;             // 0 = full solve, 1 = stop after condensing and write H, g
  int B;
  double L;             // wheelbase
  vc_kin_mpc w;
  vc_qp qp;
  vc_obstacles obs;
};

// Merit line search of the kinematic SQP step (kin_merit.hip; vc_qp.kin_sqp > 0).
struct KinMeritArgs {
  const double* x0;        // [B][6]
  const double* kappa;     // [B][N]
  const double* ds;        // [B][N]
  const double* u_prev;    // [B][N][2]  iterate before this QP step
  double* ubar;            // [B][N][2]  in: the QP's u*; out: u_prev + alpha (u* - u_prev)
  double* x_out;           // [B][N+1][6] rollout of the accepted iterate (multiple shooting: in: the
                           // QP's x*, out: x_prev + alpha (x* - x_prev))
  const double* x_prev;    // [B][N+1][6] states before this QP step (multiple shooting only)
  double* u0;              // [B][2]
  const int32_t* qp_status;  // [B] this iteration's QP status (aliases status)
  const int32_t* qp_iters;   // [B] this iteration's QP iterations (aliases iters)
  int32_t* status;         // [B] the first QP's status (later failures refuse their step)
  int32_t* iters;          // [B] accumulated interior-point iterations
  int32_t* st_acc;         // [B] scratch accumulators
  int32_t* it_acc;         // [B]
  double* ls_diag;         // [B][4] optional: alpha, phi(u_prev), phi(accepted), directional derivative
  int B, N;
  int first;               // 1 on the first SQP iteration
  int restart;             // 1: a failed first QP restarts the iterate from the neutral guess
  int ms;                  // multiple shooting (vc_qp.ms)
  double L;
  vc_kin_mpc w;
  vc_obstacles obs;
};

// Fused dynamic-bicycle SQP step (dyn_sqp.hip), fp32.
struct DynSqpArgs {
  const float* x0;     // [B][8]
  const float* kappa;  // [B][N]
  const float* ds;     // [B][N]
  const float* ubar;   // [B][N][2]  warm start (may alias u_out)
  float* u_out;        // [B][N][2]  u*
  float* x_out;        // [B][N][8]  x* = rollout(u*)
  float* u0;           // [B][2]
  int32_t* status;     // [B]
  int32_t* iters;      // [B]
  float* diag;         // [B][4] optional diagnostics, may be null
  float* dbg;          // [B][dyn_sqp_debug_stride()] first-QP dump (vc_solve_debug), may be null
  int B;
  DynCoef<float> car;
  vc_dyn_mpc w;
  vc_qp qp;
  vc_obstacles obs;
};

// Fused single-track SQP step with a stagewise Riccati interior point (st_sqp.hip), fp64.
struct StSqpArgs {
  const double* x0;     // [B][8]
  const double* kappa;  // [B][N]
  const double* ds;     // [B][N]
  const double* ubar;   // [B][N][2]  warm start (may alias u_out)
  double* u_out;        // [B][N][2]  u*
  double* x_out;        // [B][N][8]  x* = rollout(u*)
  double* u0;           // [B][2]
  int32_t* status;      // [B]
  int32_t* iters;       // [B]
  double* diag;         // [B][4] optional diagnostics, may be null
  double* jws;          // [B][st_sqp_jws_doubles(N, B)] stage Jacobians kept out of LDS (null: none needed)
  int B;
  DynCoef<double> car;
  vc_dyn_mpc w;
  vc_qp qp;
  vc_obstacles obs;
};

// Fused cascaded (single-track + point-mass) SQP step (casc_sqp.hip), fp64.
struct CascSqpArgs {
  const double* x0;     // [B][8]
  const double* kappa;  // [B][H]
  const double* ds;     // [B][H]
  const double* ubar;   // [B][H][2]  warm start (may alias u_out)
  double* u_out;        // [B][H][2]  u*
  double* x_out;        // [B][H][8]  x* = rollout(u*), point-mass states in slots 0..4
  double* u0;           // [B][2]
  int32_t* status;      // [B]
  int32_t* iters;       // [B]
  double* diag;         // [B][4] optional diagnostics, may be null
  double* jws;          // [B][casc_ric_jws_doubles(N, M, B)] stage Jacobians kept out of LDS (null: none needed)
  double* H_out;        // [B][2H][2H]  (mode 1 only)
  double* g_out;        // [B][2H]      (mode 1 only)
  int mode;             // 0 = full solve, 1 = first QP's H, g only
  int B;
  DynCoef<double> car;
  vc_dyn_mpc w;
  vc_casc_mpc cw;
  vc_qp qp;
  vc_obstacles obs;
};

// Elementwise model kernels (models.hip).
struct ModelArgs {
  int model;  // vc_model
  int B, N;
  int M;      // point-mass stages of a cascaded context (0 otherwise)
  int shift;  // vc_qp.shift: advance a solved vehicle's warm start one stage after the step
  double L;   // kinematic wheelbase
  DynCoef<double> dyn64;
  DynCoef<float> dyn32;
};
template <typename T>
__host__ __device__ inline const DynCoef<T>& dyn_coef(const ModelArgs& m);
template <>
__host__ __device__ inline const DynCoef<double>& dyn_coef<double>(const ModelArgs& m) { return m.dyn64; }
template <>
__host__ __device__ inline const DynCoef<float>& dyn_coef<float>(const ModelArgs& m) { return m.dyn32; }

// Curvature table k(s) (track.hip, vc_track_set): n cubic pieces on a uniform grid h,
// coef[n][4] = (c0, c1, c2, c3) in the local coordinate t = s - i h, lap length `length`.
struct TrackTable {
  const double* coef;
  int n;
  double h, length;
};

hipError_t launch_track_k(const TrackTable& tt, int dtype, int B, const void* s, void* k, hipStream_t st);
// M, ds_pm: the point-mass tail of a cascaded context (M = 0 otherwise)
hipError_t launch_horizon(const TrackTable& tt, int model, int dtype, int B, int N, int M, double ds_pm,
                          const void* x0, bool x0_fp64, const void* xbar, double mpc_dt, void* kappa, void* ds,
                          void* x0_out, hipStream_t st);
// kappa: this step's horizon curvature (cascaded restart: the neutral point-mass tail), may be null
hipError_t launch_drive(const ModelArgs& m, int dtype, const TrackTable& tt, double* x64, const void* u0, double dt,
                        void* x_ctx, const int32_t* status, void* xbar, void* ubar, int32_t* nfail, double* log_x,
                        void* log_u, const void* kappa, hipStream_t st);
hipError_t launch_kin_ltv(const KinLtvArgs& a, int N, hipStream_t stream);
// Stagewise-Riccati kinematic LTV-MPC step (kin_ric.hip): the same contract, any built N
// (KinLtvArgs.mode / H_out / g_out are not read).
hipError_t launch_kin_ric(const KinLtvArgs& a, int N, hipStream_t stream);
hipError_t launch_kin_merit(const KinMeritArgs& a, hipStream_t stream);
// Test hook (vc_debug_rcp): the reciprocal forms of the solve kernels on n inputs, out[n][4].
hipError_t launch_rcp_probe(int n, const double* x, double* out, hipStream_t st);
// Test hook (vc_debug_qp_fault): overwrite problem b's QP output with NaN, status VC_NONFINITE.
hipError_t launch_kin_qp_fault(const KinLtvArgs& a, int N, int b, hipStream_t stream);
bool kin_ric_built(int N);
hipError_t launch_dyn_sqp(const DynSqpArgs& a, int N, hipStream_t stream);
hipError_t launch_casc_sqp(const CascSqpArgs& a, int N, int M, hipStream_t stream);
// Stagewise-Riccati cascaded SQP step (casc_ric.hip): the same contract (CascSqpArgs.mode /
// H_out / g_out are not read), N + M <= 64.
hipError_t launch_casc_ric(const CascSqpArgs& a, int N, int M, hipStream_t stream);
bool casc_ric_built(int N, int M);
// doubles per problem of CascSqpArgs.jws for shape (N, M) (0: the kernel keeps its Jacobians in LDS)
size_t casc_ric_jws_doubles(int N, int M, int B);  // 0: the launch of B problems keeps J in LDS
hipError_t launch_st_sqp(const StSqpArgs& a, int N, hipStream_t stream);
bool st_sqp_built(int N);
// doubles per problem of StSqpArgs.jws for horizon N (0: the kernel keeps its Jacobians in LDS)
size_t st_sqp_jws_doubles(int N, int B);  // 0: the launch of B problems keeps J in LDS
bool casc_sqp_built(int N, int M);
size_t dyn_sqp_smem_bytes(int N);
int dyn_sqp_debug_stride();
size_t kin_ltv_smem_bytes(int N);
hipError_t launch_ode(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa, int space,
                      void* f, hipStream_t st);
hipError_t launch_plant_step(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa, double dt,
                             void* xn, hipStream_t st);
hipError_t launch_spatial_step(const ModelArgs& m, int dtype, const void* x, const void* u, const void* kappa,
                               const void* ds, void* xn, hipStream_t st);
hipError_t launch_rollout(const ModelArgs& m, int dtype, const void* x0, const void* ubar, const void* kappa,
                          const void* ds, void* xbar, hipStream_t st);
hipError_t launch_kin_linearize(const ModelArgs& m, const void* xbar, const void* ubar, const void* kappa,
                                const void* ds, void* A, void* Bm, hipStream_t st);

}  // namespace vc
