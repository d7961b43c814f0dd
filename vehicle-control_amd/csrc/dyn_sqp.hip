// dyn_sqp.hip -- fused batched dynamic-bicycle SQP-MPC step for gfx950 (fp32).
//
// One 256-thread workgroup (4 wavefronts, one per SIMD of a CU) owns one problem and
// runs, without leaving the CU, `sqp_iters` rounds of
//     predict -> linearize -> condense -> QP (Mehrotra interior point) -> update,
// then the rollout of u*.  This replaces, per control step and vehicle,
// CascadedMPC.command in single-track mode (controllers/mpc/cascaded_mpc.py:306-314,
// horizon_pm = 0), i.e. the IPOPT + HSL MA27 solve of the NLP built at
// cascaded_mpc.py:17-39,91-179,279-304.  The contract (what is solved, in which
// variables) is restated by oracle/dyn_sqp.py; DESIGN.md section 3.3.
//
// Decision variable dz (n = 2N = 80): dz_{2k} = dFx_k / S, dz_{2k+1} = dw_k (S = fx_scale).
// Condensed sensitivities G_k (dx_k = G_k dz) of the rows the cost/constraints touch
// are kept in LDS per stage k = 1..N-1 in a triangular layout (stage k has nonzeros in
// columns < 2k; its storage is padded to vw(k) = 16 (1 + k/8) columns):
//     Vg[.]  float4 (Ux, Uy, r, delta) rows,   Vey[.] ey row,   Vep[n] terminal epsi row.
// Every per-stage quadratic form of the QP (Gauss-Newton cost + interior-point barrier
// weights of the stage's constraint rows) is a 7x7 block W_k over the stage basis
// (Ux, Uy, r, delta, ey, Fx_k, epsi), so the interior-point normal matrix is
//     M = sum_k V_k' W_k V_k + D        (V_k = the basis rows of stage k),
// built on the matrix cores (v_mfma_f32_16x16x4_f32, one K = 8 block per stage): this is
// the condensing GEMM G'QG of the north star.  M is factorised by a blocked (16x16)
// right-looking Cholesky whose augmented identity rows produce Y = L^-T in place, so
// each Newton solve is two triangular mat-vecs  dz = Y (Y' rhs).
//
// Thread roles: stage owner = thread k < N (wave 0) holds stage k's 12 constraint rows
// (slacks, multipliers, linearised coefficients) in registers; column threads t < n own
// decision variable t; the forward (V z) and adjoint (V' v) passes and the tile GEMMs use
// all 256 threads.  HBM traffic is only the compulsory per-problem inputs and outputs.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "vc_dual.hpp"
#include "vc_kernels.hpp"
#include "vc_models.hpp"
#include "vcmpc.h"

namespace vc {
namespace {

using f4 = __attribute__((ext_vector_type(4))) float;

constexpr int NTH = 256;   // threads per problem
// debug dump layout (vc_solve_debug, first QP of the first SQP iteration)
constexpr int DBG_G = 0, DBG_M = 80, DBG_Y = 80 + 6400, DBG_RHS = 80 + 12800, DBG_DZ = 160 + 12800;
constexpr int DBG_STRIDE = 240 + 12800;
constexpr int NROW = 12;   // one-sided constraint rows per stage (owner lane)
constexpr int TS = 16;     // tile size

// stage storage width and offset (columns) of the triangular G layout
__host__ __device__ constexpr int vw(int k) { return k == 0 ? 0 : 16 * (1 + k / 8); }
__host__ __device__ constexpr int voff(int k) {
  // sum_{i=1}^{k-1} 16 (1 + i/8)
  const int m = k - 1;
  if (m <= 0) return 0;
  const int q = m / 8, r = m - 8 * q;
  return 16 * (m + 4 * q * (q - 1) + q * (r + 1));
}
static_assert(voff(9) == 144 && voff(2) == 16 && voff(1) == 0, "voff");

template <int N>
struct DD {
  static constexpr int n = 2 * N;
  static constexpr int NTL = n / TS;
  static constexpr int LDM = n + 1;  // odd stride: conflict-free column reads
  static constexpr int VC = voff(N);
  static_assert(n % TS == 0 && NTL == 5, "tile schedule is built for N = 40");
};

template <int N>
struct DynSmem {
  using D = DD<N>;
  float4 Vg[D::VC];
  float Vey[D::VC];
  float Vep[D::n];
  union {
    float M[D::n][D::LDM];   // normal matrix; lower tiles -> L (transient); upper + diag -> Y = L^-T
    float AB[N - 1][7][8];   // Jacobians [stage][row Ux,Uy,r,dlt,ey,eps,t][col Ux,Uy,r,dlt,ey,eps,Fx*S,w]
  } u;
  float W[N][32];            // per-stage weight block: 5x5 over (Ux,Uy,r,dlt,Fx) at row stride 6, [30] q_ey, [31] q_ep
  float xb[N][8];
  float ub[N][2];
  float uo[N][2];  // the iterate before the SQP step under test (domain cut-back)
  float kap[N], dsv[N];
  float y[N][8];             // forward pass: (Ux,Uy,r,dlt,ey) of V_k z, [5] terminal epsi
  float va[2][N][8];         // adjoint inputs: (Ux,Uy,r,dlt,ey, Fx-unit, w-direct, epsi(N-1))
  float part[2][3][D::n];    // adjoint / mat-vec partial sums
  float vz[D::n], vd[D::n], vr[D::n], vg[D::n], vt[D::n], vp[D::n];
  float ddw[N];              // barrier weight on w_k (box rows)
  float red[16];
  int flag[4];
};

// ---- wave helpers --------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_quad(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_quad<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_quad<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float rl(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ float step_bound(float v, float dv) { return dv < 0.f ? -v / dv : 1.f; }
// compiler-only memory barrier: keeps the loop-invariant LDS reads of G (constant over an
// interior-point solve) inside the loops instead of hoisted into hundreds of live VGPRs
__device__ __forceinline__ void no_hoist() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- phase 1: predict (wave 0; every lane redundantly, lane 0 stores) ------------------
template <int N>
__device__ __forceinline__ void predict(DynSmem<N>& s, const DynCoef<float>& p, int lane) {
  float x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = s.xb[0][i];
  bool dom = dyn_in_domain(x, s.kap[0]);
#pragma unroll 1
  for (int k = 0; k < N - 1; ++k) {
    const float u[2] = {s.ub[k][0], s.ub[k][1]};
    const float kap = s.kap[k];
    float xn[8];
    const float th = dyn_fx_split(u[0]);  // one tanh per step, not per evaluation
    rk4_apply<float, 8>(x, s.dsv[k], [&](const float* xs, float* f) { dyn_spatial_ode_alg_th(xs, u, th, kap, p, f); }, xn);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = xn[i];
    dom = dom && dyn_in_domain(x, s.kap[k + 1]);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) s.xb[k + 1][i] = x[i];
    }
  }
  // flag[2]: the rollout is inside the spatial model's domain (oracle/dyn_sqp.py in_domain)
  if (lane == 0) s.flag[2] = dom ? 1 : 0;
}

// ---- phase 2: Jacobians of the RK4 spatial step by dual numbers (task = stage x seed pair)
// seeds 0..7 = (Ux, Uy, r, dlt, ey, eps, Fx, w); output rows (Ux, Uy, r, dlt, ey, eps, t)
template <int N>
__device__ __forceinline__ void linearize(DynSmem<N>& s, const DynCoef<float>& p, float S, int task) {
  const int k = task >> 2, pr = task & 3;
  using T = Dual<2>;
  T x[8], u[2];
  constexpr int xi_of_seed[6] = {0, 1, 2, 3, 5, 6};
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = T(s.xb[k][i]);
  u[0] = T(s.ub[k][0]);
  u[1] = T(s.ub[k][1]);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int sd = 2 * pr + e;
#pragma unroll
    for (int q = 0; q < 6; ++q)
      if (sd == q) x[xi_of_seed[q]].d[e] = 1.f;
    if (sd == 6) u[0].d[e] = 1.f;
    if (sd == 7) u[1].d[e] = 1.f;
  }
  const T kap(s.kap[k]);
  const T h(s.dsv[k]);
  T xn[8];
  const T th = dyn_fx_split(u[0]);
  rk4_apply<T, 8>(x, h, [&](const T* xs, T* f) { dyn_spatial_ode_alg_th(xs, u, th, kap, p, f); }, xn);
  constexpr int row_of[7] = {0, 1, 2, 3, 5, 6, 7};
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int sd = 2 * pr + e;
      s.u.AB[k][r][sd] = xn[row_of[r]].d[e] * (sd == 6 ? S : 1.f);
    }
}

// ---- phase 3: condensing, thread j = column j -----------------------------------------
// G_{k0+1}[:, j] = B_{k0}[:, j&1] (k0 = j/2), G_{k+1} = A_k G_k; rows stored per stage.
// Returns the terminal t-row entry G_t[N-1][j] (the time cost is linear in it).
template <int N>
__device__ __forceinline__ float condense(DynSmem<N>& s, int j) {
  float g[7] = {0, 0, 0, 0, 0, 0, 0};  // Ux, Uy, r, dlt, ey, eps, t
  const int k0 = j >> 1;
#pragma unroll 1
  for (int k = 1; k < N; ++k) {
    const int km = k - 1;
    if (km == k0) {
#pragma unroll
      for (int r = 0; r < 7; ++r) g[r] = s.u.AB[km][r][6 + (j & 1)];
    } else if (km > k0) {
      float ng[7];
#pragma unroll
      for (int r = 0; r < 7; ++r) {
        float a = (r == 6) ? g[6] : 0.f;
#pragma unroll
        for (int c = 0; c < 6; ++c) a += s.u.AB[km][r][c] * g[c];
        ng[r] = a;
      }
#pragma unroll
      for (int r = 0; r < 7; ++r) g[r] = ng[r];
    }
    if (j < vw(k)) {
      const int o = voff(k) + j;
      s.Vg[o] = make_float4(g[0], g[1], g[2], g[3]);
      s.Vey[o] = g[4];
    }
  }
  s.Vep[j] = g[5];
  return g[6];
}

// ---- forward pass: y_k = V_k z (Ux, Uy, r, dlt, ey), y[N-1][5] = epsi row --------------
template <int N>
__device__ __forceinline__ void fwd_pass(DynSmem<N>& s, const float* z, int t) {
  constexpr int NK = 4 * (N - 1);
  no_hoist();  // G is invariant over an interior-point solve: keep its reads inside this pass
  if (t < NK) {
    const int k = 1 + (t >> 2), q = t & 3;
    const int len = 2 * k, per = (len + 3) >> 2;
    const int j0 = q * per, j1 = min(len, j0 + per);
    const float4* g = &s.Vg[voff(k)];
    const float* e = &s.Vey[voff(k)];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
    for (int j = j0; j < j1; ++j) {
      const float4 v = g[j];
      const float zj = z[j];
      a0 += v.x * zj;
      a1 += v.y * zj;
      a2 += v.z * zj;
      a3 += v.w * zj;
      a4 += e[j] * zj;
    }
    a0 = quad_sum(a0);
    a1 = quad_sum(a1);
    a2 = quad_sum(a2);
    a3 = quad_sum(a3);
    a4 = quad_sum(a4);
    if (q == 0) {
      s.y[k][0] = a0;
      s.y[k][1] = a1;
      s.y[k][2] = a2;
      s.y[k][3] = a3;
      s.y[k][4] = a4;
    }
  } else if (t == NK) {
    float a = 0.f;
    for (int j = 0; j < 2 * N; ++j) a += s.Vep[j] * z[j];
    s.y[N - 1][5] = a;
  }
}

// ---- adjoint pass: out_j = (V' v)_j for NV stage-vector sets s.va[v] ---------------------
// Stage ranges [1,23), [23,33), [33,N) split the triangular work in thirds.  Valid in
// threads t < n after the call (the call contains one barrier).
template <int N, int NV>
__device__ __forceinline__ void adj_pass(DynSmem<N>& s, int t, float* out, int v0 = 0) {
  constexpr int n = 2 * N;
  constexpr int lo[3] = {1, 23, 33}, hi[3] = {23, 33, N};
  no_hoist();
  if (t < 3 * n) {
    const int j = t % n, gp = t / n;
    float acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.f;
    int off = voff(lo[gp]);
#pragma unroll 1
    for (int k = lo[gp]; k < hi[gp]; ++k) {
      const int w = vw(k);
      if (j < w) {
        const float4 g = s.Vg[off + j];
        const float e = s.Vey[off + j];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const float* a = s.va[v0 + v][k];
          acc[v] += g.x * a[0] + g.y * a[1] + g.z * a[2] + g.w * a[3] + e * a[4];
        }
      }
      off += w;
    }
    if (gp == 0) {  // direct terms: Fx-unit / w entries of stage j/2, terminal epsi row
#pragma unroll
      for (int v = 0; v < NV; ++v)
        acc[v] += s.va[v0 + v][j >> 1][5 + (j & 1)] + s.Vep[j] * s.va[v0 + v][N - 1][7];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) s.part[v][gp][j] = acc[v];
  }
  __syncthreads();
  if (t < n) {
#pragma unroll
    for (int v = 0; v < NV; ++v) out[v] = s.part[v][0][t] + s.part[v][1][t] + s.part[v][2][t];
  }
}

// ---- normal matrix on the matrix cores ---------------------------------------------------
// M = sum_k V_k' W_k V_k over stages k >= 1, lower 16x16 tiles (I, J), one K = 8 block per
// stage: rows (Ux, Uy, r, dlt) and (ey, Fx-unit, epsi [k = N-1], 0).  Stage k contributes to
// row block I iff k >= 8 I (its G rows are zero in columns >= 2k).  Each wave owns a fixed
// tile list (balanced by contributing stages) and walks the stages once, reusing a stage's
// operands across its tiles; operand selection by the lane's K row is branch-free.
// W layout per stage: rows (Ux, Uy, r, dlt, Fx) of the 5x5 block at 6-float stride, then
// q_ey at [30] and q_ep at [31].
constexpr int WROW = 6;

// lane-row selection as an arithmetic blend (m[i] = [kk == i]): a select on a lane-varying
// index otherwise becomes exec-masked control flow around the operand loads
__device__ __forceinline__ float blend4(const float* m, float a, float b, float c, float d) {
  return m[0] * a + m[1] * b + m[2] * c + m[3] * d;
}

template <int N, int I0, int J0, int I1, int J1, int I2, int J2, int I3, int J3>
__device__ __forceinline__ void build_wave(DynSmem<N>& s, int lane) {
  constexpr int TI[4] = {I0, I1, I2, I3}, TJ[4] = {J0, J1, J2, J3};
  const int i16 = lane & 15, kk = lane >> 4;
  const float km[4] = {kk == 0 ? 1.f : 0.f, kk == 1 ? 1.f : 0.f, kk == 2 ? 1.f : 0.f, kk == 3 ? 1.f : 0.f};
  f4 acc0[4], acc1[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    acc0[tt] = f4{0.f, 0.f, 0.f, 0.f};
    acc1[tt] = f4{0.f, 0.f, 0.f, 0.f};
  }
  no_hoist();
#pragma unroll 1
  for (int k = 1; k < N; ++k) {
    const int off = voff(k);
    const float* w = s.W[k];
    const float* wr = w + WROW * kk;  // W row kk (kk < 4) for K block 0
    const float wk0 = wr[0], wk1 = wr[1], wk2 = wr[2], wk3 = wr[3], wk4 = wr[4];
    const float wf0 = w[24], wf1 = w[25], wf2 = w[26], wf3 = w[27], wf4 = w[28];
    const float qey = w[30], qep = w[31];
    const bool last = (k == N - 1);
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int I = TI[tt], J = TJ[tt];
      if (I < 0 || k < (I == 0 ? 1 : 8 * I)) continue;  // wave-uniform
      const int ci = TS * I + i16, cj = TS * J + i16;
      const float4 vi = s.Vg[off + ci], vj = s.Vg[off + cj];
      const float eyi = s.Vey[off + ci], eyj = s.Vey[off + cj];
      const float lm = last ? 1.f : 0.f;  // Vep is read every stage (no load under a branch)
      const float epi = lm * s.Vep[ci], epj = lm * s.Vep[cj];
      const float fi = (ci == 2 * k) ? 1.f : 0.f, fj = (cj == 2 * k) ? 1.f : 0.f;
      const float a0 = blend4(km, vi.x, vi.y, vi.z, vi.w);
      const float b0 = wk0 * vj.x + wk1 * vj.y + wk2 * vj.z + wk3 * vj.w + wk4 * fj;
      acc0[tt] = mfma4(a0, b0, acc0[tt]);
      const float bF = wf0 * vj.x + wf1 * vj.y + wf2 * vj.z + wf3 * vj.w + wf4 * fj;
      const float a1 = blend4(km, eyi, fi, epi, 0.f);
      const float b1 = blend4(km, qey * eyj, bF, qep * epj, 0.f);
      acc1[tt] = mfma4(a1, b1, acc1[tt]);
    }
  }
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    const int I = TI[tt], J = TJ[tt];
    if (I < 0) continue;
    const f4 acc = acc0[tt] + acc1[tt];
#pragma unroll
    for (int r = 0; r < 4; ++r) s.u.M[TS * I + 4 * kk + r][TS * J + i16] = acc[r];
  }
}

// tile lists per wave: 71 / 72 / 72 / 64 contributing (tile, stage) pairs at N = 40
template <int N>
__device__ __forceinline__ void build_normal(DynSmem<N>& s, int wv, int lane) {
  switch (wv) {
    case 0: build_wave<N, 0, 0, 3, 0, 4, 0, 4, 1>(s, lane); break;
    case 1: build_wave<N, 1, 0, 1, 1, 4, 2, -1, -1>(s, lane); break;
    case 2: build_wave<N, 2, 0, 2, 1, 3, 1, 4, 3>(s, lane); break;
    default: build_wave<N, 2, 2, 3, 2, 3, 3, 4, 4>(s, lane); break;
  }
}

// ---- blocked Cholesky with augmented identity rows: M -> Y = L^-T ----------------------
// C (+/-)= A . B for 16x16 tiles: A[i][k] = pa[i*sai + k*sak], B[k][j] = pb[k*sbk + j*sbj]
__device__ __forceinline__ f4 tile_mma(f4 acc, const float* pa, int sai, int sak, const float* pb, int sbk, int sbj,
                                       int lane, float sign) {
  const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int k = 4 * st + kq;
    acc = mfma4(sign * pa[i16 * sai + k * sak], pb[k * sbk + i16 * sbj], acc);
  }
  return acc;
}

template <int N>
__device__ __forceinline__ f4 load_tile(const DynSmem<N>& s, int R, int C, int lane) {
  const int i16 = lane & 15, kq = lane >> 4;
  f4 c;
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = s.u.M[TS * R + 4 * kq + r][TS * C + i16];
  return c;
}
template <int N>
__device__ __forceinline__ void store_tile(DynSmem<N>& s, int R, int C, int lane, f4 c) {
  const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) s.u.M[TS * R + 4 * kq + r][TS * C + i16] = c[r];
}

// factor the diagonal tile (J,J) in one wave and overwrite it with Y_JJ = L_JJ^-T
// (upper triangular, zeros below).  Returns false if a pivot is not positive/finite.
template <int N>
__device__ __forceinline__ bool diag_block(DynSmem<N>& s, int J, int lane) {
  constexpr int LDM = DD<N>::LDM;
  float* T0 = &s.u.M[TS * J][TS * J];
  const int j = lane & 15;
  float a[TS];
#pragma unroll
  for (int i = 0; i < TS; ++i) a[i] = T0[i * LDM + j];  // lane j: column j (= row j, symmetric)
  bool ok = true;
#pragma unroll
  for (int c = 0; c < TS; ++c) {
    const float piv = rl(a[c], c);
    ok = ok && (piv > 0.f) && (piv < 3.0e38f);
    const float d = rsqrtf(piv);
    const float f = a[c] * d * d;  // l_jc d  (lane j)
#pragma unroll
    for (int i = c + 1; i < TS; ++i) a[i] = fmaf(-rl(a[i], c), f, a[i]);
    a[c] = a[c] * d;  // lane j now holds L[j][c] in register c (row-per-lane factor)
    __builtin_amdgcn_sched_barrier(0);  // one step at a time: bounds the live readlane SGPRs
  }
  // X = L^-1, lane p computes column p: X[i][p] = (delta_ip - sum_{m<i} L[i][m] X[m][p]) / L[i][i].
  // L goes through the tile (row j written by lane j) and is read back as wave-uniform
  // broadcasts; the reads of a row are issued before that row of Y is written.
  if (lane < TS) {
#pragma unroll
    for (int c = 0; c < TS; ++c) T0[j * LDM + c] = (c <= j) ? a[c] : 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS stores are done
  __builtin_amdgcn_wave_barrier();
  float x[TS];
#pragma unroll
  for (int i = 0; i < TS; ++i) {
    float acc = (i == j) ? 1.f : 0.f;
#pragma unroll
    for (int m = 0; m < i; ++m) acc = fmaf(-T0[i * LDM + m], x[m], acc);
    x[i] = acc / T0[i * LDM + i];
    __builtin_amdgcn_sched_barrier(0);  // row i's broadcast reads stay with row i
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  if (lane < TS) {
    // Y_JJ[p][i] = X[i][p]: lane p writes row p
#pragma unroll
    for (int i = 0; i < TS; ++i) T0[j * LDM + i] = (i >= j) ? x[i] : 0.f;
  }
  return ok;
}

template <int N>
__device__ __forceinline__ bool chol_inverse(DynSmem<N>& s, int wv, int lane, int t) {
  constexpr int NT = DD<N>::NTL, LDM = DD<N>::LDM;
  if (t == 0) s.flag[0] = 1;
#pragma unroll 1
  for (int J = 0; J < NT; ++J) {
    if (wv == (J & 3)) {
      const bool ok = diag_block(s, J, lane);
      if (lane == 0 && !ok) s.flag[0] = 0;
    }
    __syncthreads();
    // panel: (R,J), R > J: L_RJ = M_RJ Y_JJ ; (P,J), P < J: Y_PJ <- Y_PJ Y_JJ   (NT-1 tiles)
    {
      const int q = wv;  // one tile per wave (NT - 1 = 4)
      const int R = (q < NT - 1 - J) ? J + 1 + q : q - (NT - 1 - J);
      const float* Y = &s.u.M[TS * J][TS * J];
      const float* A = &s.u.M[TS * R][TS * J];
      f4 c = {0.f, 0.f, 0.f, 0.f};
      c = tile_mma(c, A, LDM, 1, Y, LDM, 1, lane, 1.f);
      store_tile(s, R, J, lane, c);
    }
    __syncthreads();
    // trailing: original (R,K), J < K <= R: M_RK -= L_RJ L_KJ' ; augmented (P,K), P <= J < K:
    // Y_PK -= Y_PJ L_KJ'
    {
      const int nK = NT - 1 - J;
      const int nOrig = nK * (nK + 1) / 2;
      const int nAug = (J + 1) * nK;
#pragma unroll 1
      for (int q = wv; q < nOrig + nAug; q += 4) {
        int R, K;
        if (q < nOrig) {  // enumerate K = J+1.., R = K..NT-1
          int rem = q;
          K = J + 1;
          while (rem >= NT - K) { rem -= NT - K; ++K; }
          R = K + rem;
        } else {
          const int r = q - nOrig;
          R = r / nK;           // P = 0..J
          K = J + 1 + r % nK;
        }
        const float* A = &s.u.M[TS * R][TS * J];   // L_RJ (R > J) or Y_RJ (R <= J)
        const float* Bt = &s.u.M[TS * K][TS * J];  // L_KJ, read transposed
        f4 c = load_tile(s, R, K, lane);
        c = tile_mma(c, A, LDM, 1, Bt, 1, LDM, lane, -1.f);
        store_tile(s, R, K, lane, c);
      }
    }
    __syncthreads();
  }
  return s.flag[0] != 0;
}

// dz = Y (Y' rhs) with Y = L^-T in the upper triangle of M (rows split in thirds)
template <int N>
__device__ __forceinline__ void solve(DynSmem<N>& s, const float* rhs, float* out, int t) {
  constexpr int n = 2 * N, CH = (n + 2) / 3;
  if (t < 3 * n) {  // u_j = sum_{i <= j} Y[i][j] rhs_i
    const int j = t % n, gp = t / n;
    const int i0 = gp * CH, i1 = min(j + 1, min(n, i0 + CH));
    float a = 0.f;
    for (int i = i0; i < i1; ++i) a += s.u.M[i][j] * rhs[i];
    s.part[0][gp][j] = a;
  }
  __syncthreads();
  if (t < n) s.vt[t] = s.part[0][0][t] + s.part[0][1][t] + s.part[0][2][t];
  __syncthreads();
  if (t < 3 * n) {  // out_i = sum_{j >= i} Y[i][j] u_j
    const int i = t % n, gp = t / n;
    const int j0 = max(i, gp * CH), j1 = min(n, gp * CH + CH);
    float a = 0.f;
    for (int j = j0; j < j1; ++j) a += s.u.M[i][j] * s.vt[j];
    s.part[1][gp][i] = a;
  }
  __syncthreads();
  if (t < n) out[t] = s.part[1][0][t] + s.part[1][1][t] + s.part[1][2][t];
  __syncthreads();
}

// ---- stage lanes ------------------------------------------------------------------------
// Thread t < 4N serves stage k = t / 4 as lane q = t % 4 of a DPP quad.  Each lane owns three
// one-sided rows of its stage, each a dense coefficient vector over the stage basis
// b = (dUx, dUy, dr, ddlt, zFx, zw) (zFx = dFx / S):
//   q = 0: -Ux <= Ux - Ux_min, dlt <= dlt_max - dlt, -dlt <= dlt - dlt_min  (k >= 1)
//   q = 1: power limit, front tyre upper, front tyre lower                 (linearised)
//   q = 2: rear tyre upper, rear tyre lower, w <= min(w_max - w, trust_w)
//   q = 3: -w <= min(w - w_min, trust_w), +-zFx <= trust_Fx / S             (if trust_Fx > 0)
// Lane q = 0 also carries the stage's Gauss-Newton cost block (wc over Ux..dlt, Fx).
struct StageRows {
  float c[3][6];
  float d[3], m[3];  // rhs, validity mask
  float sl[3], la[3];
};

__device__ __forceinline__ float row_val(const float* c, const float* bx) {
  return c[0] * bx[0] + c[1] * bx[1] + c[2] * bx[2] + c[3] * bx[3] + c[4] * bx[4] + c[5] * bx[5];
}
template <int CTRL>
__device__ __forceinline__ float quad_bcast(float v) { return dpp_quad<CTRL>(v); }
// sym 5x5 packed index
__host__ __device__ constexpr int sym5(int a, int c) {
  return a <= c ? a * 5 - a * (a - 1) / 2 + (c - a) : c * 5 - c * (c - 1) / 2 + (a - c);
}

// block-wide reductions through s.red (one barrier each)
template <int N>
__device__ __forceinline__ float block_max(DynSmem<N>& s, float v, int wv, int lane, int slot) {
  v = wave_max(v);
  if (lane == 0) s.red[slot + wv] = v;
  __syncthreads();
  return fmaxf(fmaxf(s.red[slot], s.red[slot + 1]), fmaxf(s.red[slot + 2], s.red[slot + 3]));
}
template <int N>
__device__ __forceinline__ float block_min(DynSmem<N>& s, float v, int wv, int lane, int slot) {
  v = wave_min(v);
  if (lane == 0) s.red[slot + wv] = v;
  __syncthreads();
  return fminf(fminf(s.red[slot], s.red[slot + 1]), fminf(s.red[slot + 2], s.red[slot + 3]));
}
template <int N>
__device__ __forceinline__ float block_sum(DynSmem<N>& s, float v, int wv, int lane, int slot) {
  v = wave_sum(v);
  if (lane == 0) s.red[slot + wv] = v;
  __syncthreads();
  return (s.red[slot] + s.red[slot + 1]) + (s.red[slot + 2] + s.red[slot + 3]);
}

// stage basis values bx = (V_k v)(Ux,Uy,r,dlt), v[2k], v[2k+1] after a forward pass of v
template <int N>
__device__ __forceinline__ void stage_basis(const DynSmem<N>& s, const float* v, int k, float* bx) {
  bx[0] = s.y[k][0];
  bx[1] = s.y[k][1];
  bx[2] = s.y[k][2];
  bx[3] = s.y[k][3];
  bx[4] = v[2 * k];
  bx[5] = v[2 * k + 1];
}

// q == 0 lane writes the stage's adjoint input vector (quad-summed 6-vector + extras)
template <int N>
__device__ __forceinline__ void write_adj(DynSmem<N>& s, int slot, int k, int q, float* v6, float ey, float ep) {
#pragma unroll
  for (int i = 0; i < 6; ++i) v6[i] = quad_sum(v6[i]);
  if (q == 0) {
    float* va = s.va[slot][k];
    va[0] = v6[0];
    va[1] = v6[1];
    va[2] = v6[2];
    va[3] = v6[3];
    va[4] = ey;
    va[5] = v6[4];
    va[6] = v6[5];
    va[7] = ep;
  }
}

// Section timing (debug builds only, -DVC_TIMING, `make timing`): thread 0's s_memtime
// stamps between barriers, accumulated per section and written to diag[b][4 + slot].
enum { DT_PRED = 0, DT_LIN, DT_COND, DT_SETUP, DT_RESID, DT_BUILD, DT_CHOL, DT_PREDICTOR, DT_CORRECTOR,
       DT_POLISH, DT_OUT, DT_TOTAL, DT_BW, DT_BMFMA, DT_BDIAG, DT_NSLOT };
#ifdef VC_TIMING
#define DT_STAMP(var)                               \
  __builtin_amdgcn_sched_barrier(0);                \
  const uint64_t var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0);
#define DT_ACC(slot, t0)                                  \
  {                                                       \
    __builtin_amdgcn_sched_barrier(0);                    \
    tacc[slot] += __builtin_amdgcn_s_memtime() - (t0);    \
    __builtin_amdgcn_sched_barrier(0);                    \
  }
#else
#define DT_STAMP(var)
#define DT_ACC(slot, t0)
#endif

// ---- the fused kernel ---------------------------------------------------------------------
template <int N, int TYRE>
__global__ __launch_bounds__(NTH, 1) void dyn_sqp_kernel(DynSqpArgs A) {
  constexpr int n = 2 * N;
  constexpr int NS = 4 * N;  // stage lanes
  __shared__ DynSmem<N> s;
  const int b = xcd_problem(blockIdx.x, A.B);
  // Thread coordinates are re-laundered (asm "+v") at the top of every solver loop so the
  // hundreds of LDS addresses derived from them are recomputed per iteration instead of
  // being hoisted out of the loops into live registers (which spilled to scratch).
  int t = threadIdx.x, lane = t & 63;
  int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // wave-uniform (scalar branches)
  int k = t >> 2, q = t & 3;  // stage lane role (t < NS)
  const bool stl = t < NS;
  DynCoef<float> p = A.car;
  p.tyre = TYRE;  // compile-time tyre model: the other branch of the ODE is not generated
  const vc_dyn_mpc& W = A.w;
  const float S = float(W.fx_scale);
  const float prox2 = float(2.0 * A.qp.prox);
  const float tol = float(A.qp.tol);
  const float Tw = float(A.qp.trust_w), TF = float(W.trust_Fx);

  // ---- inputs ----
  if (t < 8) s.xb[0][t] = A.x0[(size_t)b * 8 + t];
  if (t < N) {
    s.kap[t] = A.kappa[(size_t)b * N + t];
    s.dsv[t] = A.ds[(size_t)b * N + t];
  }
  if (t < n) s.ub[t >> 1][t & 1] = A.ubar[(size_t)b * n + t];
  if (t < 8) s.y[0][t] = 0.f;
  for (int e = t; e < 2 * N * 8; e += NTH) (&s.va[0][0][0])[e] = 0.f;
  __syncthreads();

  int it_total = 0, it_max = 0, n_polished = 0;
#ifdef VC_TIMING
  uint64_t tacc[DT_NSLOT] = {};
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
  bool all_conv = true, any_fail = false;
  float last_res = 0.f, last_mu = 0.f;

  // SQP update state: a step under test (tries > 0) is ub = uo + 2^-(tries-1) du (du = the QP
  // iterate vz, untouched by the rollout), the last try the unchanged iterate; the loop's one
  // rollout site also makes the output rollout x* = rollout(u*)
  int tries = 0, sq = 0;
  bool test = false;  // the iterate's own rollout is inside the domain (else the full step, untested)
#pragma unroll 1
  for (;;) {
    asm volatile("" : "+v"(t), "+v"(lane), "+v"(k), "+v"(q));
    asm volatile("" : "+s"(wv));
    // ---------------- predict ----------------
    DT_STAMP(t_p0)
    if (wv == 0) predict(s, p, lane);
    __syncthreads();
    DT_ACC(DT_PRED, t_p0)
    if (tries > 0) {
      // ---------------- SQP update: cut the step back while its rollout leaves the domain ----------------
      // (oracle/dyn_sqp.py domain_step; IPOPT cuts its step back alike on evaluation errors)
      if (test && s.flag[2] == 0 && tries <= DOM_HALVINGS) {
        const float a = tries < DOM_HALVINGS ? ldexpf(1.f, -tries) : 0.f;
        if (t < n) {
          const float uo = s.uo[t >> 1][t & 1];
          s.ub[t >> 1][t & 1] = a > 0.f ? uo + a * (s.vz[t] * ((t & 1) ? 1.f : S)) : uo;
        }
        ++tries;
        __syncthreads();
        continue;
      }
      tries = 0;
      ++sq;
    }
    if (sq == W.sqp_iters) break;
    DT_STAMP(t_l0)

    // ---------------- linearize (waves 1-3) | stage terms (stage lanes of wave 0-2) ----------
    if (t >= 64 && t < 64 + 4 * (N - 1)) linearize(s, p, S, t - 64);
    __syncthreads();
    // stage functions with tangents (X_q, Fx): lane q gets d/dX_q and d/dFx of all 7
    float fv[7], fgq[7], fgF[7];
    if (stl) {
      using T2 = Dual<2>;
      T2 X5[5];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        X5[i] = T2(s.xb[k][i]);
        X5[i].d[0] = (i == q) ? 1.f : 0.f;
      }
      X5[4] = T2(s.ub[k][0]);
      X5[4].d[1] = 1.f;
      T2 o[7];
      dyn_stage_terms_alg(X5, p, o);
#pragma unroll
      for (int r = 0; r < 7; ++r) {
        fv[r] = o[r].v;
        fgq[r] = o[r].d[0];
        fgF[r] = o[r].d[1];
      }
    }
    // gather the full gradient (Ux, Uy, r, dlt, Fx) of every stage function inside the quad
    float gr[7][5];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      gr[r][0] = quad_bcast<0x00>(fgq[r]);
      gr[r][1] = quad_bcast<0x55>(fgq[r]);
      gr[r][2] = quad_bcast<0xAA>(fgq[r]);
      gr[r][3] = quad_bcast<0xFF>(fgq[r]);
      gr[r][4] = fgF[r];
    }

    DT_ACC(DT_LIN, t_l0)
    // ---------------- condense ----------------
    DT_STAMP(t_c0)
    float gt = 0.f;
    if (t < n) gt = condense(s, t);
    __syncthreads();
    DT_ACC(DT_COND, t_c0)
    DT_STAMP(t_s0)

    // ---------------- QP setup (branch-free in q: selects, not divergent ifs) ----------------
    StageRows R;
    float wc[15], qey, qep;
    {
      const float invS = 1.f / S;
      const float ds = s.dsv[k];
      const float Ux = s.xb[k][0], dl = s.xb[k][3], ey = s.xb[k][5], ep = s.xb[k][6];
      const float wb = s.ub[k][1];
      const float c0 = (q == 0 && stl) ? 1.f : 0.f;        // lane carries the cost
      const float term = (k == N - 1) ? 1.f : 0.f;          // terminal stage
      // ---- Gauss-Newton cost (cascaded_mpc.py:139-171, 279-304), nonzero on q == 0 only ----
      const float blo = ey < float(W.ey_min) ? float(W.w_b) : 0.f;
      const float bhi = ey > float(W.ey_max) ? float(W.w_b) : 0.f;
      // obstacle barrier (cascaded_mpc.py:173-176), convexified quadratic in ey_k
      float po = 0.f, qo = 0.f;
      if (A.obs.n > 0) obstacle_ey_model<float>(A.obs, s.xb[k][4], ey, float(W.w_obs) * ds, po, qo);
      qey = c0 * (2.f * ds * (float(W.w_dev) + blo + bhi) + term * 2.f * float(W.w_ey) + qo);
      const float gey = c0 * (2.f * ds * (float(W.w_dev) * ey + blo * (ey - float(W.ey_min)) +
                                          bhi * (ey - float(W.ey_max))) +
                              term * 2.f * float(W.w_ey) * ey + po);
      qep = c0 * term * 2.f * float(W.w_epsi);
      const float gep = c0 * term * 2.f * float(W.w_epsi) * ep;
      float gv[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 15; ++e) wc[e] = 0.f;
#pragma unroll
      for (int sr = 0; sr < 2; ++sr) {  // slip front / rear
        const float act = fv[sr] >= 0.f ? c0 * 2.f * float(W.w_slip) : 0.f;
        const float c5[5] = {gr[sr][0], gr[sr][1], gr[sr][2], gr[sr][3], gr[sr][4] * S};
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          gv[a] += act * fv[sr] * c5[a];
#pragma unroll
          for (int c = a; c < 5; ++c) wc[sym5(a, c)] += act * c5[a] * c5[c];
        }
      }
      const float spd = (Ux >= float(W.max_speed)) ? c0 * term * 2.f * float(W.w_speed) : 0.f;
      wc[sym5(0, 0)] += spd;
      gv[0] += spd * (Ux - float(W.max_speed));
      if (q == 0 && stl) {
        float* va = s.va[0][k];
        va[0] = gv[0];
        va[1] = gv[1];
        va[2] = gv[2];
        va[3] = gv[3];
        va[4] = gey;
        va[5] = gv[4];
        va[6] = 2.f * float(W.w_w) * wb;
        va[7] = gep;
      }
      // ---- rows: dense linearised rows (q = 1: f = 2,3,4; q = 2: f = 5,6) + unit rows ----
      const float isd = (q == 1) ? 1.f : 0.f, isr = (q == 2) ? 1.f : 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        float g5[5], v;
        if (i < 2) {
#pragma unroll
          for (int c = 0; c < 5; ++c) g5[c] = q == 1 ? gr[2 + i][c] : gr[5 + i][c];
          v = q == 1 ? fv[2 + i] : fv[5 + i];
        } else {
#pragma unroll
          for (int c = 0; c < 5; ++c) g5[c] = gr[4][c];
          v = fv[4];
        }
        const float dm = (i < 2) ? isd + isr : isd;  // dense row present
#pragma unroll
        for (int c = 0; c < 4; ++c) R.c[i][c] = dm * g5[c] * invS;
        R.c[i][4] = dm * g5[4];
        R.c[i][5] = 0.f;
        R.d[i] = dm > 0.f ? -v * invS : 1.f;
        R.m[i] = dm;
      }
      const float st = (q == 0 && k >= 1) ? 1.f : 0.f;
      float wup = float(W.w_max) - wb, wdn = wb - float(W.w_min);
      if (Tw > 0.f) { wup = fminf(wup, Tw); wdn = fminf(wdn, Tw); }
      const float q3 = (q == 3) ? 1.f : 0.f, tm = (q == 3 && TF > 0.f) ? 1.f : 0.f;
      // q == 0: state rows
      R.c[0][0] += -st;   R.d[0] = st > 0.f ? Ux - float(W.Ux_min) : R.d[0];          R.m[0] += st;
      R.c[1][3] += st;    R.d[1] = st > 0.f ? float(W.delta_max) - dl : R.d[1];       R.m[1] += st;
      R.c[2][3] += -st;   R.d[2] = st > 0.f ? dl - float(W.delta_min) : R.d[2];       R.m[2] += st;
      // q == 2 slot 2: w upper;  q == 3: w lower, +-dFx trust region
      R.c[2][5] += isr;   R.d[2] = isr > 0.f ? wup : R.d[2];                          R.m[2] += isr;
      R.c[0][5] += -q3;   R.d[0] = q3 > 0.f ? wdn : R.d[0];                           R.m[0] += q3;
      R.c[1][4] += tm;    R.d[1] = q3 > 0.f ? TF * invS : R.d[1];                     R.m[1] += tm;
      R.c[2][4] += -tm;   R.d[2] = q3 > 0.f ? TF * invS : R.d[2];                     R.m[2] += tm;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (!stl) R.m[i] = 0.f;
        R.sl[i] = R.m[i] > 0.f ? fmaxf(R.d[i], 1.f) : 1.f;
        R.la[i] = R.m[i];
      }
    }
    __syncthreads();
    // gradient g = V' va0 + direct terms (w_time G_t, Fx slew)
    float gj = 0.f;
    {
      float o[1];
      adj_pass<N, 1>(s, t, o);
      if (t < n) {
        const int kc = t >> 1;
        gj = o[0] + float(W.w_time) * gt;
        if ((t & 1) == 0) {  // (w_Fx / ds_k) (Fx_{k+1} - Fx_k)^2, cascaded_mpc.py:167-171
          if (kc < N - 1) gj -= 2.f * float(W.w_Fx) / s.dsv[kc] * (s.ub[kc + 1][0] - s.ub[kc][0]) * S;
          if (kc >= 1) gj += 2.f * float(W.w_Fx) / s.dsv[kc - 1] * (s.ub[kc][0] - s.ub[kc - 1][0]) * S;
        }
        s.vg[t] = gj;
        s.vz[t] = 0.f;
        if (A.dbg && sq == 0) A.dbg[(size_t)b * DBG_STRIDE + DBG_G + t] = gj;
      }
    }
    float scale, mcount;
    {
      float m = (t < n) ? fabsf(gj) : 0.f, c = 0.f;
      if (stl) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          m = fmaxf(m, R.m[i] * fabsf(R.d[i]));
          c += R.m[i];
        }
      }
      scale = 1.f + block_max(s, m, wv, lane, 0);
      mcount = fmaxf(block_sum(s, c, wv, lane, 4), 1.f);
    }
    DT_ACC(DT_SETUP, t_s0)
    // Hessian direct part: prox, w_w, Fx slew (tridiagonal in the Fx columns)
    int kc = t >> 1;
    const float slew_here = (t < n && (t & 1) == 0 && kc < N - 1) ? 2.f * float(W.w_Fx) / s.dsv[kc] * S * S : 0.f;
    const float slew_prev = (t < n && (t & 1) == 0 && kc >= 1) ? 2.f * float(W.w_Fx) / s.dsv[kc - 1] * S * S : 0.f;
    const float hdiag = prox2 + ((t & 1) ? 2.f * float(W.w_w) : slew_here + slew_prev);

    // M = H + C' diag(w) C on the stage blocks (+ direct part), ready for chol_inverse.
    // w[3]: this stage lane's row weights (barrier weights, or rho on the polish's active set)
    auto assemble = [&](const float* w) {
      DT_STAMP(t_a0)
      if (stl) {
        float w15[15], dw = 0.f;
#pragma unroll
        for (int e = 0; e < 15; ++e) w15[e] = wc[e];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int c = a; c < 5; ++c) w15[sym5(a, c)] += w[i] * R.c[i][a] * R.c[i][c];
          dw += w[i] * R.c[i][5] * R.c[i][5];
        }
#pragma unroll
        for (int e = 0; e < 15; ++e) w15[e] = quad_sum(w15[e]);
        dw = quad_sum(dw);
        if (q == 0) {
#pragma unroll
          for (int a = 0; a < 5; ++a)
#pragma unroll
            for (int c = 0; c < 5; ++c) s.W[k][WROW * a + c] = w15[sym5(a, c)];
          s.W[k][30] = qey;
          s.W[k][31] = qep;
          s.ddw[k] = dw;
        }
      }
      __syncthreads();
      DT_ACC(DT_BW, t_a0)
      DT_STAMP(t_a1)
      build_normal(s, wv, lane);
      for (int e = t; e < 10 * TS * TS; e += NTH) {  // upper tiles start at 0 (augmented rows)
        int rem = e >> 8, P = 0;
        while (rem >= DD<N>::NTL - 1 - P) { rem -= DD<N>::NTL - 1 - P; ++P; }
        const int K = P + 1 + rem;
        s.u.M[TS * P + ((e & 255) >> 4)][TS * K + (e & 15)] = 0.f;
      }
      __syncthreads();
      DT_ACC(DT_BMFMA, t_a1)
      DT_STAMP(t_a2)
      if (t < n) {
        float d = hdiag;
        if (t & 1) d += s.ddw[kc];
        else if (kc == 0) d += s.W[0][WROW * 4 + 4];
        s.u.M[t][t] += d;
        if ((t & 1) == 0 && kc >= 1) {
          s.u.M[t][t - 2] -= slew_prev;
          if ((t & 15) >= 2) s.u.M[t - 2][t] -= slew_prev;  // same diagonal tile: keep it symmetric
        }
      }
      __syncthreads();
      DT_ACC(DT_BDIAG, t_a2)
    };

    // ---------------- interior point (Mehrotra predictor-corrector) ----------------
    int it = 0;
    bool conv = false, fail = false;
    float rhsp = 0.f;
#pragma unroll 1
    for (; it < A.qp.max_iter; ++it) {
      no_hoist();
      asm volatile("" : "+v"(t), "+v"(lane), "+v"(k), "+v"(q), "+v"(kc));
      asm volatile("" : "+s"(wv));

      // (a) residuals at z: rp = C z + s - d (stage lanes), rd = H z + g + C' lam (columns)
      DT_STAMP(t_r0)
      fwd_pass(s, s.vz, t);
      __syncthreads();
      float rp[3], wg[3];
      float rpmax = 0.f, musum = 0.f;
      if (stl) {
        float bx[6];
        stage_basis(s, s.vz, k, bx);
        float v6[6], u6[6];
#pragma unroll
        for (int a = 0; a < 5; ++a) {  // cost part of H z (wc is zero off q == 0)
          float acc = 0.f;
#pragma unroll
          for (int c = 0; c < 5; ++c) acc += wc[sym5(a, c)] * bx[c];
          v6[a] = acc;
          u6[a] = acc;  // H z enters both rd and the predictor rhs
        }
        v6[5] = 0.f;
        u6[5] = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          rp[i] = R.m[i] * (row_val(R.c[i], bx) + R.sl[i] - R.d[i]);
          wg[i] = R.m[i] * R.la[i] / R.sl[i];
          rpmax = fmaxf(rpmax, fabsf(rp[i]));
          musum += R.m[i] * R.sl[i] * R.la[i];
          const float al = R.m[i] * R.la[i], au = wg[i] * rp[i];
#pragma unroll
          for (int c = 0; c < 6; ++c) {
            v6[c] += al * R.c[i][c];  // C' lam
            u6[c] += au * R.c[i][c];  // C' (w rp)
          }
        }
        // va0 -> H z + C' lam (rd);  va1 -> H z + C' (w rp) (predictor rhs = -g - va1 adjoint)
        const float hey = qey * s.y[k][4], hep = (k == N - 1) ? qep * s.y[N - 1][5] : 0.f;
        write_adj(s, 0, k, q, v6, hey, hep);
        write_adj(s, 1, k, q, u6, hey, hep);
      }
      const float rpm = block_max(s, rpmax, wv, lane, 0);
      const float mu = block_sum(s, musum, wv, lane, 4) / mcount;
      float o[2];
      adj_pass<N, 2>(s, t, o);
      float rdmax = 0.f;
      if (t < n) {
        float hz = hdiag * s.vz[t];
        if ((t & 1) == 0) {
          if (kc < N - 1) hz -= slew_here * s.vz[t + 2];
          if (kc >= 1) hz -= slew_prev * s.vz[t - 2];
        }
        const float rd = o[0] + s.vg[t] + hz;
        rhsp = -s.vg[t] - hz - o[1];  // = -rd - C'(w rp - lam)
        s.vr[t] = rhsp;
        rdmax = fabsf(rd);
      }
      const float rdm = block_max(s, rdmax, wv, lane, 8);
      last_res = fmaxf(rdm, rpm) / scale;
      last_mu = mu / scale;
      DT_ACC(DT_RESID, t_r0)
      if (!(rdm == rdm) || !(rpm == rpm) || !(mu == mu) || rdm > 3.0e38f) { fail = true; break; }
      if (rdm <= tol * scale && rpm <= tol * scale && mu <= tol * scale) { conv = true; break; }

      // (b) normal matrix M = sum_k V_k' W_k V_k + D, blocked Cholesky, Y = L^-T
      DT_STAMP(t_b0)
      assemble(wg);
      DT_ACC(DT_BUILD, t_b0)
      DT_STAMP(t_ch0)
      const bool dump = A.dbg && sq == 0 && it == 0;
      if (dump)
        for (int e = t; e < n * n; e += NTH) A.dbg[(size_t)b * DBG_STRIDE + DBG_M + e] = s.u.M[e / n][e % n];
      if (!chol_inverse(s, wv, lane, t)) { fail = true; break; }
      if (dump) {
        for (int e = t; e < n * n; e += NTH) A.dbg[(size_t)b * DBG_STRIDE + DBG_Y + e] = s.u.M[e / n][e % n];
        if (t < n) A.dbg[(size_t)b * DBG_STRIDE + DBG_RHS + t] = s.vr[t];
      }

      DT_ACC(DT_CHOL, t_ch0)
      // (c) predictor (affine-scaling) direction
      DT_STAMP(t_pr0)
      solve(s, s.vr, s.vd, t);
      if (dump && t < n) A.dbg[(size_t)b * DBG_STRIDE + DBG_DZ + t] = s.vd[t];
      fwd_pass(s, s.vd, t);
      __syncthreads();
      float ds_a[3], dl_a[3], amin = 1.f;
      if (stl) {
        float bx[6];
        stage_basis(s, s.vd, k, bx);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float cz = R.m[i] * row_val(R.c[i], bx);
          ds_a[i] = -rp[i] - cz;
          dl_a[i] = wg[i] * (cz + rp[i]) - R.m[i] * R.la[i];
          if (R.m[i] > 0.f) amin = fminf(amin, fminf(step_bound(R.sl[i], ds_a[i]), step_bound(R.la[i], dl_a[i])));
        }
      }
      amin = block_min(s, amin, wv, lane, 0);
      float ms = 0.f;
      if (stl) {
#pragma unroll
        for (int i = 0; i < 3; ++i) ms += R.m[i] * (R.sl[i] + amin * ds_a[i]) * (R.la[i] + amin * dl_a[i]);
      }
      ms = block_sum(s, ms, wv, lane, 4) / mcount;
      const float ratio = mu > 0.f ? fminf(1.f, ms / mu) : 0.f;
      const float smu = ratio * ratio * ratio * mu;  // sigma mu, sigma = (mu_aff / mu)^3
      float rc[3];
      if (stl) {
        float u6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          rc[i] = R.m[i] * (R.sl[i] * R.la[i] + ds_a[i] * dl_a[i] - smu);
          // corrector rhs = predictor rhs + C' ((ds_a dl_a - sigma mu) / s)
          const float au = R.m[i] * (ds_a[i] * dl_a[i] - smu) / R.sl[i];
#pragma unroll
          for (int c = 0; c < 6; ++c) u6[c] += au * R.c[i][c];
        }
        write_adj(s, 1, k, q, u6, 0.f, 0.f);
      }
      __syncthreads();
      {
        float o1[1];
        adj_pass<N, 1>(s, t, o1, 1);
        if (t < n) s.vr[t] = rhsp + o1[0];
      }
      __syncthreads();

      DT_ACC(DT_PREDICTOR, t_pr0)
      // (d) corrector direction, step to the boundary, update
      DT_STAMP(t_co0)
      solve(s, s.vr, s.vd, t);
      fwd_pass(s, s.vd, t);
      __syncthreads();
      float dsr[3], dlr[3];
      amin = 1.f;
      if (stl) {
        float bx[6];
        stage_basis(s, s.vd, k, bx);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const float cz = R.m[i] * row_val(R.c[i], bx);
          dsr[i] = -rp[i] - cz;
          dlr[i] = wg[i] * (cz + rp[i]) - rc[i] / R.sl[i];
          if (R.m[i] > 0.f) amin = fminf(amin, fminf(step_bound(R.sl[i], dsr[i]), step_bound(R.la[i], dlr[i])));
        }
      }
      const float alpha = fminf(1.f, 0.99f * block_min(s, amin, wv, lane, 8));
      if (stl) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (R.m[i] > 0.f) {
            R.sl[i] = fmaxf(R.sl[i] + alpha * dsr[i], 1e-30f);
            R.la[i] = fmaxf(R.la[i] + alpha * dlr[i], 1e-30f);
          }
        }
      }
      if (t < n) s.vz[t] += alpha * s.vd[t];
      __syncthreads();
      DT_ACC(DT_CORRECTOR, t_co0)
    }
    it_total += it;
    it_max = max(it_max, it);

    // ---------------- active-set polish (augmented Lagrangian on the identified set) ------------
    // The interior point stops at mu ~ tol * scale, which leaves O(mu / lambda) errors along
    // weakly active rows.  Fix the active set it identified (lambda > s), solve
    //   min 1/2 z'Hz + g'z  s.t.  C_A z = d_A
    // by augmented-Lagrangian passes on one factorisation of H + rho C_A'C_A (multipliers
    // warm-started from the interior point), then certify: inactive rows feasible, active
    // multipliers >= 0.  A failed certificate adds every violated row and drops every
    // negative multiplier for the next round (the oracle changes one row per round);
    // after A.qp.polish rounds without a certificate the interior-point iterate is kept.
    bool polished = false;
    DT_STAMP(t_po0)
    if (!fail && A.qp.polish > 0) {
      const float rho = 1.0e4f;  // AL converges in ~4 passes; H + rho C_A'C_A stays ~1e5-conditioned
      // tolerances on the O(1) rows (scaled units), not on the gradient-inflated `scale`
      float dm = 0.f;
      if (stl) {
#pragma unroll
        for (int i = 0; i < 3; ++i) dm = fmaxf(dm, R.m[i] * fabsf(R.d[i]));
      }
      const float dscale = 1.f + block_max(s, dm, wv, lane, 8);
      const float eps_r = 5.0e-7f * dscale, eps_p = 1.0e-5f * dscale;
      if (t < n) s.vp[t] = s.vz[t];  // interior-point solution (restored if not certified)
      float act[3], nu[3], res[3];
      if (stl) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          act[i] = (R.m[i] > 0.f && R.la[i] > R.sl[i]) ? 1.f : 0.f;
          nu[i] = act[i] * R.la[i];
          res[i] = 0.f;
        }
      }
#pragma unroll 1
      for (int round = 0; round < A.qp.polish; ++round) {
        asm volatile("" : "+v"(t), "+v"(lane), "+v"(k), "+v"(q), "+v"(kc));
        asm volatile("" : "+s"(wv));

        float w3[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) w3[i] = stl ? rho * act[i] : 0.f;
        assemble(w3);
        if (!chol_inverse(s, wv, lane, t)) break;
        float rlast = 0.f;
#pragma unroll 1
        for (int pass = 0; pass < 12; ++pass) {
          // rhs = -g - C' (nu - rho a d)
          if (stl) {
            float u6[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              const float cf = nu[i] - rho * act[i] * R.d[i];
#pragma unroll
              for (int c = 0; c < 6; ++c) u6[c] += cf * R.c[i][c];
            }
            write_adj(s, 1, k, q, u6, 0.f, 0.f);
          }
          __syncthreads();
          {
            float o1[1];
            adj_pass<N, 1>(s, t, o1, 1);
            if (t < n) s.vr[t] = -s.vg[t] - o1[0];
          }
          __syncthreads();
          solve(s, s.vr, s.vz, t);
          fwd_pass(s, s.vz, t);
          __syncthreads();
          float rmax = 0.f;
          if (stl) {
            float bx[6];
            stage_basis(s, s.vz, k, bx);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              res[i] = R.m[i] * (row_val(R.c[i], bx) - R.d[i]);
              nu[i] += rho * act[i] * res[i];
              rmax = fmaxf(rmax, act[i] * fabsf(res[i]));
            }
          }
          rlast = block_max(s, rmax, wv, lane, 0);
          if (rlast <= eps_r) break;
        }
        // certificate
        float bad = 0.f;
        if (stl) {
          const float nscale = 1e-5f * (1.f + fmaxf(fabsf(nu[0]), fmaxf(fabsf(nu[1]), fabsf(nu[2]))));
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const bool viol = act[i] == 0.f && R.m[i] > 0.f && res[i] > eps_p;
            const bool neg = act[i] > 0.f && nu[i] < -nscale;
            if (viol || neg) bad = 1.f;
            if (viol) act[i] = 1.f;
            if (neg) { act[i] = 0.f; nu[i] = 0.f; }
          }
        }
        // certified only with the equality-constrained solve converged as well
        if (block_max(s, bad, wv, lane, 8) == 0.f && rlast <= 10.f * eps_r) { polished = true; break; }
      }
      if (!polished && t < n) s.vz[t] = s.vp[t];
      __syncthreads();
    }
    DT_ACC(DT_POLISH, t_po0)
    all_conv = all_conv && (conv || polished);
    any_fail = any_fail || fail;
    n_polished += polished ? 1 : 0;

    // ---------------- SQP update: ubar += du, tested by the next rollout ----------------
    if (t < n) {
      const float uo = s.ub[t >> 1][t & 1];
      s.uo[t >> 1][t & 1] = uo;
      s.ub[t >> 1][t & 1] = uo + s.vz[t] * ((t & 1) ? 1.f : S);
    }
    test = s.flag[2] != 0;
    tries = 1;
    __syncthreads();
  }

  // ---------------- outputs: u*, x* = rollout(u*) (the loop's last predict), u0, status ----------------
  DT_STAMP(t_o0)
  DT_ACC(DT_OUT, t_o0)
  bool finite = true;
  if (t < n) {
    const float v = s.ub[t >> 1][t & 1];
    finite = (v == v) && fabsf(v) < 3.0e38f;
    A.u_out[(size_t)b * n + t] = v;
  }
  for (int e = t; e < N * 8; e += NTH) {
    const float v = s.xb[e >> 3][e & 7];
    finite = finite && (v == v) && fabsf(v) < 3.0e38f;
    A.x_out[(size_t)b * N * 8 + e] = v;
  }
  const bool all_finite = __syncthreads_and(finite ? 1 : 0) != 0;
  if (t < 2) A.u0[(size_t)b * 2 + t] = s.ub[0][t];
  if (t == 0) {
    int32_t st;
    if (!all_finite) st = VC_NONFINITE;
    else if (s.flag[2] == 0) st = VC_OUT_OF_DOMAIN;  // x* (the last rollout) outside the model's domain
    else if (all_conv) st = VC_SOLVED;
    else st = VC_MAX_ITER;
    A.status[b] = st;
    A.iters[b] = it_total;
    if (A.diag) {
#ifdef VC_TIMING
      constexpr size_t DS = 4 + DT_NSLOT;
      tacc[DT_TOTAL] = __builtin_amdgcn_s_memtime() - t_start;
      for (int i = 0; i < DT_NSLOT; ++i) A.diag[(size_t)b * DS + 4 + i] = float(tacc[i]);
#else
      constexpr size_t DS = 4;
#endif
      A.diag[(size_t)b * DS + 0] = last_res;
      A.diag[(size_t)b * DS + 1] = last_mu;
      A.diag[(size_t)b * DS + 2] =
          float((any_fail ? 1 : 0) | (all_conv ? 2 : 0) | (n_polished == W.sqp_iters ? 4 : 0) | (n_polished << 4));
      A.diag[(size_t)b * DS + 3] = float(it_max);
    }
  }
}

}  // namespace

// ---- host launcher ---------------------------------------------------------------
int dyn_sqp_debug_stride() { return DBG_STRIDE; }

size_t dyn_sqp_smem_bytes(int N) {
  switch (N) {
    case 40: return sizeof(DynSmem<40>);
    default: return 0;
  }
}

hipError_t launch_dyn_sqp(const DynSqpArgs& a, int N, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  switch (N) {
    case 40:
      if (a.car.tyre == VC_TYRE_LINEAR)
        hipLaunchKernelGGL((dyn_sqp_kernel<40, VC_TYRE_LINEAR>), dim3(a.B), dim3(NTH), 0, stream, a);
      else
        hipLaunchKernelGGL((dyn_sqp_kernel<40, VC_TYRE_FIALA>), dim3(a.B), dim3(NTH), 0, stream, a);
      return hipGetLastError();
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vc
