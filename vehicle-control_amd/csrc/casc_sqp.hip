// casc_sqp.hip -- fused cascaded (single-track + point-mass) SQP step, fp64, one
// 256-thread workgroup per problem.
//
// Replaces the IPOPT solve of CascadedMPC with horizon_pm > 0
// (controllers/mpc/cascaded_mpc.py:17-39,91-304, config/controllers/cascaded.yaml: N = 20
// single-track stages, M = 40 point-mass stages every ds_pm = 3 m).  Contract:
// oracle/casc_sqp.py.  Per SQP iteration:
//   predict    thread 0: single-track RK4 (vc_models.hpp dyn_spatial_ode_alg: the same model
//              in tan(alpha), no atan / tan), switching map
//              st_to_pm, point-mass Euler (pm_spatial_ode)
//   linearize  one thread per (stage, seed): Dual<1, double> evaluation of the same step
//              code gives one column of [A B]; the switch Jacobian analytically; the
//              switching cost's lateral residual Fy_f + Fy_r and its gradient by duals
//   condense   one thread per decision column j: the column's sensitivity is carried
//              through the stages and the rows the QP reads are stored in LDS, triangular
//              (single-track stage k: Ux, Uy, r, delta, ey over columns < 2k; point-mass
//              stage j: V, ey over columns < 2j; terminal epsi, t; the lateral row)
//   QP         every cost and constraint term is local to a stage's vector
//              v_k = (Ux, Uy, r, delta | V, ey, dFx, dw | dFy) = V_k dz, plus input slews,
//              the switching residuals and the terminal epsi row.  Four lanes per stage
//              hold its 12 one-sided rows (3 each); the normal matrix
//                  M = P + sum_k V_k' (Q_k + C_k' D_k C_k) V_k
//              is built in LDS (packed lower triangle) from 4x4 register tiles,
//              factorised by a blocked right-looking Cholesky (8-column blocks, 3
//              barriers per block), and each Mehrotra predictor / corrector solve is
//              two single-wave triangular sweeps in register-prefetched 8-column blocks.
//   update     ubar += dz (scaled back: Fx and the point mass's Fy by fx_scale)
// LDS: packed normal matrix 58 KB (aliased by the linearisation scratch before the QP),
// condensed rows 68 KB, stage blocks 13 KB, trajectory and vectors 18 KB.
#include <hip/hip_runtime.h>

#include <cmath>

#include "vc_dual.hpp"
#include "vc_kernels.hpp"

namespace vc {
namespace {

constexpr int CTH = 256;

template <int N, int M>
struct CL {
  static constexpr int H = N + M, n = 2 * H, NP = n * (n + 1) / 2;
  static constexpr int P0 = 5 * N * (N - 1);                          // first point-mass row
  static constexpr int T0 = P0 + 4 * (M * N + M * (M - 1) / 2);       // terminal epsi, t rows
  static constexpr int SW0 = T0 + 4 * (H - 1);                        // switch lateral row
  static constexpr int NG = SW0 + 2 * N + 2;
  // single-track stage k (1..N-1): rows (Ux, Uy, r, delta, ey), each of length 2k
  __device__ static constexpr int gst(int k) { return 5 * k * (k - 1); }
  // point-mass stage m (global stage N + m): rows (V, ey), each of length 2(N + m)
  __device__ static constexpr int gpm(int m) { return P0 + 4 * (m * N + m * (m - 1) / 2); }
  // packed lower triangle, column-major: (i >= j)
  __device__ static constexpr int pidx(int i, int j) { return j * n - (j * (j - 1)) / 2 + (i - j); }
};

template <int N, int M>
struct CascSmem {
  using L = CL<N, M>;
  union {
    double Mp[L::NP];
    struct {
      double As[N - 1][8][10];  // [A B] of the single-track RK4 steps
      double Ap[M - 1][5][7];   // [A B] of the point-mass Euler steps
      double Sw[5][8];          // switching map Jacobian
    } lin;
  } u;
  double G[L::NG];
  double W[L::H][28];           // stage normal blocks, packed symmetric 7x7
  double xs[N][8];
  double xp[M][5];
  double ub[L::H][2];
  double uo[L::H][2];  // the iterate before the SQP step under test (domain cut-back)
  double kap[L::H], dsv[L::H];
  double z[L::n], dz[L::n], rhs[L::n], gp[L::n], invd[L::n];
  double Y[L::H][8], R[L::H][8];
  double ex[4];                 // a_sw . x, g_epsi . x (extra dense rows)
  double sc[8];                 // lateral residual value + gradient (Ux, Uy, r, delta, Fx)
  double red[8];
  int flag[4];
  int dom;             // the last rollout is inside both models' domain (casc_in_domain)
};

__device__ __forceinline__ int sym7(int a, int b) {  // a <= b
  return a * 7 - (a * (a - 1)) / 2 + (b - a);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
template <int OP>  // 0 sum, 1 max, 2 min
__device__ __forceinline__ double block_reduce(double v, double* red) {
  v = OP == 0 ? wave_sum(v) : (OP == 1 ? wave_max(v) : wave_min(v));
  const int t = threadIdx.x;
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  const double a = red[0], b = red[1], c = red[2], d = red[3];
  return OP == 0 ? (a + b) + (c + d) : (OP == 1 ? fmax(fmax(a, b), fmax(c, d)) : fmin(fmin(a, b), fmin(c, d)));
}

// one-sided constraint rows of a stage: coefficients over the stage vector, rhs, activity
struct Rows3 {
  double c[3][7];
  double d[3];
  double act[3];
};


// normal matrix (see the kernel's comment at its call); out of line so its register tiles do not
// compete with the interior point's live row state
// normal matrix: M = P + sum_k V_k' W_k V_k (W_k in s.W), one pass, no read-modify-write.
// Thread-owned 4x4 register tiles of the lower triangle (465 tiles; thread t takes tile t
// and its mirror 464 - t so heavy and light tiles pair up).  Entry (i, j), i >= j, sums
// the stages k >= i / 2; past the tile's first two stages every column is below 2k, so
// only the condensed rows enter (5 for a single-track stage, 2 for a point-mass stage).
template <int N, int M>
__device__ __forceinline__ void casc_build(CascSmem<N, M>& s, double csw, double w_epsi, double prox, double w_Fx,
                                        double w_Fy, double w_switch, double S) {
  using L = CL<N, M>;
  constexpr int H = L::H, n = L::n;
  const int t = threadIdx.x;
  auto pair_w = [&](int a) -> double {
    const int k = a >> 1, cc = a & 1;
    if (k > H - 2) return 0.0;
    double w;
    if (cc == 0) w = (k == N - 1 ? w_switch : w_Fx) / s.dsv[k];
    else if (k >= N) w = w_Fy / s.dsv[k];
    else return 0.0;
    return 2.0 * w * S * S;
  };
  auto vcol = [&](int k, int col, double* v) {
    if (k < N) {
      const int len = 2 * k, base = L::gst(k);
      const bool in = col < len;
#pragma unroll
      for (int r = 0; r < 5; ++r) v[r] = in ? s.G[base + r * len + (in ? col : 0)] : 0.0;
    } else {
      const int m = k - N, len = 2 * k, base = L::gpm(m);
      const bool in = col < len;
      v[0] = in ? s.G[base + (in ? col : 0)] : 0.0;
      v[1] = v[2] = v[3] = 0.0;
      v[4] = in ? s.G[base + len + (in ? col : 0)] : 0.0;
    }
    v[5] = col == 2 * k ? 1.0 : 0.0;
    v[6] = col == 2 * k + 1 ? 1.0 : 0.0;
  };
      constexpr int NT = n / 4, NTILES = NT * (NT + 1) / 2;
#pragma unroll 1
      for (int pass = 0; pass < 2; ++pass) {
        const int tile = pass == 0 ? t : NTILES - 1 - t;
        if (tile >= NTILES || (pass == 1 && tile < CTH)) continue;
        int I = (int)((sqrtf(8.f * tile + 1.f) - 1.f) * 0.5f);  // fp32 guess, fixed up below
        while ((I + 1) * (I + 2) / 2 <= tile) ++I;
        while (I * (I + 1) / 2 > tile) --I;
        const int J = tile - I * (I + 1) / 2;
        const int i0 = 4 * I, j0 = 4 * J;
        double acc[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            const int i = i0 + r, j = j0 + cc;
            double v = 0.0;
            if (i < 2 * N + 2 && j < 2 * N + 2) v += 2.0 * csw * s.G[L::SW0 + i] * s.G[L::SW0 + j];
            if (i < 2 * (H - 1) && j < 2 * (H - 1)) v += 2.0 * w_epsi * s.G[L::T0 + i] * s.G[L::T0 + j];
            if (i == j) v += 2.0 * prox + pair_w(j) + (j >= 2 ? pair_w(j - 2) : 0.0);
            if (i == j + 2) v -= pair_w(j);
            acc[r][cc] = v;
          }
        // the tile's first two stages: general stage vectors (unit input slots); one column
        // at a time to keep the register footprint small (these are 2 of up to 60 stages)
#pragma unroll 1
        for (int kk = 2 * I; kk < 2 * I + 2 && kk < H; ++kk) {
          const double* Wf = s.W[kk];
#pragma unroll 1
          for (int cc = 0; cc < 4; ++cc) {
            double vj[7], hv[7];
            vcol(kk, j0 + cc, vj);
#pragma unroll
            for (int a = 0; a < 7; ++a) {
              double x = 0.0;
#pragma unroll
              for (int e = 0; e < 7; ++e) x += Wf[a <= e ? sym7(a, e) : sym7(e, a)] * vj[e];
              hv[a] = x;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              double vi[7];
              vcol(kk, i0 + r, vi);
              double x = 0.0;
#pragma unroll
              for (int a = 0; a < 7; ++a) x += vi[a] * hv[a];
#pragma unroll
              for (int c2 = 0; c2 < 4; ++c2) acc[r][c2] += (c2 == cc) ? x : 0.0;
            }
          }
        }
        // single-track bulk stages: 5 condensed rows
#pragma unroll 1
        for (int kk = 2 * I + 2; kk < N; ++kk) {
          const int len = 2 * kk;
          const double* g = &s.G[L::gst(kk)];
          // W_k entries straight from LDS (one broadcast address for the whole workgroup)
          // rather than a 25-double register copy: the build runs inside the interior
          // point, whose per-lane row state is live across it
          const double* Wk = s.W[kk];
          auto Wg = [&](int a, int e) -> double { return Wk[a <= e ? sym7(a, e) : sym7(e, a)]; };
          double hv[4][5];
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            double vj[5];
#pragma unroll
            for (int a = 0; a < 5; ++a) vj[a] = g[a * len + j0 + cc];
#pragma unroll
            for (int a = 0; a < 5; ++a) {
              double x = 0.0;
#pragma unroll
              for (int e = 0; e < 5; ++e) x += Wg(a, e) * vj[e];
              hv[cc][a] = x;
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            double vi[5];
#pragma unroll
            for (int a = 0; a < 5; ++a) vi[a] = g[a * len + i0 + r];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
              double x = 0.0;
#pragma unroll
              for (int a = 0; a < 5; ++a) x += vi[a] * hv[cc][a];
              acc[r][cc] += x;
            }
          }
        }
        // point-mass bulk stages: rows V (slot 0) and ey (slot 4)
#pragma unroll 1
        for (int kk = (2 * I + 2 > N ? 2 * I + 2 : N); kk < H; ++kk) {
          const int len = 2 * kk;
          const double* g = &s.G[L::gpm(kk - N)];
          const double w00 = s.W[kk][sym7(0, 0)], w04 = s.W[kk][sym7(0, 4)], w44 = s.W[kk][sym7(4, 4)];
          double h0[4], h4[4];
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) {
            const double a = g[j0 + cc], e = g[len + j0 + cc];
            h0[cc] = w00 * a + w04 * e;
            h4[cc] = w04 * a + w44 * e;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double a = g[i0 + r], e = g[len + i0 + r];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) acc[r][cc] += a * h0[cc] + e * h4[cc];
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc)
            if (i0 + r >= j0 + cc) s.u.Mp[L::pidx(i0 + r, j0 + cc)] = acc[r][cc];
      }
      __syncthreads();
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Blocked right-looking Cholesky of the packed normal matrix, in place (L in the lower
// triangle, 1 / L_jj in s.invd), 8-column blocks, 3 barriers per block:
//   A  wave 0 factors the 8x8 diagonal block in registers (lane p owns column p);
//   B  one thread per row below the block solves its 8 panel entries against L_D;
//   C  4x4 register tiles of the trailing triangle take the rank-8 update.
// s.flag[3] = 1 on a non-positive pivot.
template <int N, int M>
__device__ __forceinline__ void casc_cholesky(CascSmem<N, M>& s) {
  using L = CL<N, M>;
  constexpr int n = L::n, NB = 8;
  static_assert(n % NB == 0, "block size");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) s.flag[3] = 0;
#pragma unroll 1
  for (int j0 = 0; j0 < n; j0 += NB) {
    // A: diagonal block
    if (wave == 0) {
      const int p = lane < NB ? lane : 0;
      double a[NB];
#pragma unroll
      for (int r = 0; r < NB; ++r) a[r] = s.u.Mp[L::pidx(j0 + (r >= p ? r : p), j0 + p)];  // no branch
#pragma unroll
      for (int r = 0; r < NB; ++r) a[r] = r >= p ? a[r] : 0.0;
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const double d = readlane_d(a[q], q);
        bad = bad || !(d > 1e-300);
        // 1 / sqrt(d): v_rsq_f64 + two Newton steps (full fp64 accuracy; a much shorter
        // dependent chain than IEEE sqrt then IEEE divide, on every block's serial path)
        const double dd = d > 1e-300 ? d : 1e-300;
        double il = __builtin_amdgcn_rsq(dd);
        il = il * (1.5 - 0.5 * dd * il * il);
        il = il * (1.5 - 0.5 * dd * il * il);
        const double l = dd * il;
        if (p == q) {
#pragma unroll
          for (int r = 0; r < NB; ++r) a[r] = r == q ? l : (r > q ? a[r] * il : a[r]);
        }
        double lq[NB];  // column q of L (rows > q), read from lane q after its scaling
#pragma unroll
        for (int r = q + 1; r < NB; ++r) lq[r] = readlane_d(a[r], q);
        // lanes p > q: a[r] -= L[r][q] L[p][q] for r >= p
#pragma unroll
        for (int r = q + 1; r < NB; ++r) {
          const double lrq = lq[r];
          double lp = 0.0;
#pragma unroll
          for (int c = q + 1; c < NB; ++c) lp = (p == c) ? lq[c] : lp;
          if (p > q && r >= p) a[r] -= lrq * lp;
        }
        if (lane == 0) s.invd[j0 + q] = il;
      }
      if (lane < NB) {
#pragma unroll
        for (int r = 0; r < NB; ++r)
          if (r >= p) s.u.Mp[L::pidx(j0 + r, j0 + p)] = a[r];
      }
      if (lane == 0 && bad) s.flag[3] = 1;
    }
    __syncthreads();
    // B: panel rows i >= j0 + NB
    {
      const int i = j0 + NB + t;
      if (i < n) {
        double x[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          double v = s.u.Mp[L::pidx(i, j0 + q)];
#pragma unroll
          for (int r = 0; r < q; ++r) v -= x[r] * s.u.Mp[L::pidx(j0 + q, j0 + r)];
          x[q] = v * s.invd[j0 + q];
        }
#pragma unroll
        for (int q = 0; q < NB; ++q) s.u.Mp[L::pidx(i, j0 + q)] = x[q];
      }
    }
    __syncthreads();
    // C: trailing update of rows / columns >= j0 + NB, 4x4 tiles
    {
      const int b0 = j0 + NB, nt = (n - b0) / 4, ntiles = nt * (nt + 1) / 2;
#pragma unroll 1
      for (int tile = t; tile < ntiles; tile += CTH) {
        int I = (int)((sqrtf(8.f * tile + 1.f) - 1.f) * 0.5f);  // fp32 guess, fixed up below
        while ((I + 1) * (I + 2) / 2 <= tile) ++I;
        while (I * (I + 1) / 2 > tile) --I;
        const int Jt = tile - I * (I + 1) / 2;
        const int i0 = b0 + 4 * I, c0 = b0 + 4 * Jt;
        double acc[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[r][c] = 0.0;
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          double li[4], lc[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) li[r] = s.u.Mp[L::pidx(i0 + r, j0 + q)];
#pragma unroll
          for (int c = 0; c < 4; ++c) lc[c] = s.u.Mp[L::pidx(c0 + c, j0 + q)];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] += li[r] * lc[c];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (i0 + r >= c0 + c) s.u.Mp[L::pidx(i0 + r, c0 + c)] -= acc[r][c];
      }
    }
    __syncthreads();
  }
}

// Solve M x = s.rhs with the factor of casc_cholesky -> s.dz.  Wave 0 alone (no barriers):
// lanes own rows lane and lane + 64.  The sweeps run in 8-column blocks whose factor
// entries sit in registers, and the NEXT block's 16 entries per lane are loaded before the
// current block's 8 dependent steps, so LDS latency stays off the pivot chain; each pivot
// is broadcast with v_readlane.  Blocks never straddle the lane / lane + 64 split.
template <int N, int M>
__device__ __forceinline__ void casc_tri_solve(CascSmem<N, M>& s) {
  using L = CL<N, M>;
  constexpr int n = L::n, NB = 8;
  static_assert(n % NB == 0 && 64 % NB == 0 && n > 64 && n <= 128, "tri solve layout");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (wave == 0) {
    const int i0 = lane, i1 = lane + 64 < n ? lane + 64 : n - 1;
    const bool has1 = lane + 64 < n;
    double y0 = s.rhs[i0], y1 = has1 ? s.rhs[i1] : 0.0;
    const double d0 = s.invd[i0], d1 = s.invd[i1];
    // addresses: column j starts at the wave-uniform pidx(j, j); row j of column i (i < j)
    // is at rb_i + j with the lane constant rb_i = pidx(i, i) - i -- one add per load
    // raw loads at clamped (always valid) addresses, no control flow and no select, so the
    // next block's 16 loads stay in flight; the structural zeros are applied at the use
    auto lowc = [&](int i, int j) -> double {  // L[i][j] where i > j
      const int d = i - j;
      return s.u.Mp[L::pidx(j, j) + (d > 0 ? d : 0)];
    };
    const int rb0 = L::pidx(i0, i0) - i0, rb1 = L::pidx(i1, i1) - i1;
    auto uppc0 = [&](int j) -> double { return s.u.Mp[j > i0 ? rb0 + j : 0]; };  // L[j][i0] where j > i0
    auto uppc1 = [&](int j) -> double { return s.u.Mp[j > i1 ? rb1 + j : 0]; };  // L[j][i1] where j > i1
    double c0[NB], c1[NB], n0[NB], n1[NB];
    // L y = b: step j scales y_j by 1 / L_jj, then y_i -= L[i][j] y_j for i > j
#pragma unroll
    for (int q = 0; q < NB; ++q) { c0[q] = lowc(i0, q); c1[q] = lowc(i1, q); }
#pragma unroll 1
    for (int j0 = 0; j0 < n; j0 += NB) {
      const int jn = j0 + NB < n ? j0 + NB : j0;
#pragma unroll
      for (int q = 0; q < NB; ++q) { n0[q] = lowc(i0, jn + q); n1[q] = lowc(i1, jn + q); }
      if (j0 < 64) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double l0 = i0 > j0 + q ? c0[q] : 0.0, l1 = i1 > j0 + q ? c1[q] : 0.0;
          y0 = (i0 == j0 + q) ? y0 * d0 : y0;
          const double yj = readlane_d(y0, j0 + q);
          y0 -= l0 * yj;
          y1 -= l1 * yj;
        }
      } else {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double l1 = i1 > j0 + q ? c1[q] : 0.0;  // rows i0 < 64 <= j: nothing
          y1 = (i1 == j0 + q && has1) ? y1 * d1 : y1;
          const double yj = readlane_d(y1, j0 + q - 64);
          y1 -= l1 * yj;
        }
      }
#pragma unroll
      for (int q = 0; q < NB; ++q) { c0[q] = n0[q]; c1[q] = n1[q]; }
    }
    // L' x = y: descending j, x_j = y_j / L_jj, then y_i -= L[j][i] x_j for i < j
#pragma unroll
    for (int q = 0; q < NB; ++q) { c0[q] = uppc0(n - 1 - q); c1[q] = uppc1(n - 1 - q); }
#pragma unroll 1
    for (int j0 = n - 1; j0 > 0; j0 -= NB) {  // block covers j0, j0 - 1, ..., j0 - NB + 1
      const int jn = j0 - NB > 0 ? j0 - NB : j0;
#pragma unroll
      for (int q = 0; q < NB; ++q) { n0[q] = uppc0(jn - q); n1[q] = uppc1(jn - q); }
      if (j0 >= 64) {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double l0 = c0[q], l1 = j0 - q > i1 ? c1[q] : 0.0;  // rows i0 < 64 <= j: all
          y1 = (i1 == j0 - q && has1) ? y1 * d1 : y1;
          const double xj = readlane_d(y1, j0 - q - 64);
          y0 -= l0 * xj;
          y1 -= l1 * xj;
        }
      } else {
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const double l0 = j0 - q > i0 ? c0[q] : 0.0;  // rows i1 >= 64 > j: nothing
          y0 = (i0 == j0 - q) ? y0 * d0 : y0;
          const double xj = readlane_d(y0, j0 - q);
          y0 -= l0 * xj;
        }
      }
#pragma unroll
      for (int q = 0; q < NB; ++q) { c0[q] = n0[q]; c1[q] = n1[q]; }
    }
    s.dz[i0] = y0;
    if (has1) s.dz[i1] = y1;
  }
  __syncthreads();
}

// Section timing (debug builds only, -DVC_TIMING, `make timing`): thread 0's s_memtime stamps,
// accumulated per section and written to diag[b][4 + slot] (scripts/casc_phase_timing.py).
enum { CT_PRED = 0, CT_LIN, CT_COND, CT_SETUP, CT_LOCAL, CT_RD, CT_WASM, CT_BUILD, CT_CHOL, CT_SOLVE, CT_DIR,
       CT_UPD, CT_TOTAL, CT_NSLOT };
#ifdef VC_TIMING
#define CT_STAMP(var)                                \
  __builtin_amdgcn_sched_barrier(0);                 \
  const uint64_t var = __builtin_amdgcn_s_memtime(); \
  __builtin_amdgcn_sched_barrier(0);
#define CT_ACC(slot, t0)                               \
  {                                                    \
    __builtin_amdgcn_sched_barrier(0);                 \
    tacc[slot] += __builtin_amdgcn_s_memtime() - (t0); \
    __builtin_amdgcn_sched_barrier(0);                 \
  }
#else
#define CT_STAMP(var)
#define CT_ACC(slot, t0)
#endif

template <int N, int M, int TYRE>
__global__ __launch_bounds__(CTH, 1) void casc_sqp_kernel(CascSqpArgs A) {
  using L = CL<N, M>;
  constexpr int H = L::H, n = L::n;
  __shared__ CascSmem<N, M> s;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b = xcd_problem(blockIdx.x, A.B);
  DynCoef<double> c = A.car;
  c.tyre = TYRE;
  const vc_dyn_mpc& W = A.w;
  const vc_casc_mpc& CW = A.cw;
  const double S = W.fx_scale;
  using D1 = Dual<1, double>;
  using D2 = Dual<2, double>;

  for (int i = t; i < H; i += CTH) {
    s.kap[i] = A.kappa[(size_t)b * H + i];
    s.dsv[i] = A.ds[(size_t)b * H + i];
    s.ub[i][0] = A.ubar[((size_t)b * H + i) * 2];
    s.ub[i][1] = A.ubar[((size_t)b * H + i) * 2 + 1];
  }
  if (t < 8) s.xs[0][t] = A.x0[(size_t)b * 8 + t];
#ifdef VC_TIMING
  uint64_t tacc[CT_NSLOT] = {};
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
  if (t == 0) {
    s.flag[0] = VC_SOLVED;
    s.flag[1] = 0;  // interior-point iterations, summed
    s.flag[2] = 2;  // diag flags: 2 = every QP converged
  }
  __syncthreads();

  bool first = true;  // the warm start's rollout: non-finite -> VC_NONFINITE
  auto predict = [&]() {
    if (t == 0) {
      double x[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = s.xs[0][i];
      bool fin = true, dom = dyn_in_domain(x, s.kap[0]);
      for (int k = 0; k < N - 1; ++k) {
        const double u2[2] = {s.ub[k][0], s.ub[k][1]};
        const double kp = s.kap[k];
        double xn[8];
        const double th = dyn_fx_split(u2[0]);  // one tanh per step, not per evaluation
        rk4_apply<double, 8>(x, s.dsv[k], [&](const double* xx, double* f) { dyn_spatial_ode_alg_th<double, double>(xx, u2, th, kp, c, f); }, xn);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          x[i] = xn[i];
          s.xs[k + 1][i] = xn[i];
          fin = fin && isfinite(xn[i]);
        }
        dom = dom && dyn_in_domain(x, s.kap[k + 1]);
      }
      double p[5];
      st_to_pm<double>(x, p);
#pragma unroll
      for (int i = 0; i < 5; ++i) s.xp[0][i] = p[i];
      dom = dom && pm_in_domain(p, s.kap[N]);
      for (int m = 0; m < M - 1; ++m) {
        const int j = N + m;
        const double u2[2] = {s.ub[j][0], s.ub[j][1]};
        double f[5];
        pm_spatial_ode<double, double>(p, u2, s.kap[j], c, f);
        const double h = s.dsv[j];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          p[i] = p[i] + h * f[i];
          s.xp[m + 1][i] = p[i];
          fin = fin && isfinite(p[i]);
        }
        dom = dom && pm_in_domain(p, s.kap[j + 1]);
      }
      s.dom = (fin && dom) ? 1 : 0;
      if (first && !fin) s.flag[0] = VC_NONFINITE;
    }
  };

  // stage vector V_k[:, col] (slots 0..6)
  auto vcol = [&](int k, int col, double* v) {
    if (k < N) {
      const int len = 2 * k, base = L::gst(k);
      const bool in = col < len;
#pragma unroll
      for (int r = 0; r < 5; ++r) v[r] = in ? s.G[base + r * len + (in ? col : 0)] : 0.0;
    } else {
      const int m = k - N, len = 2 * k, base = L::gpm(m);
      const bool in = col < len;
      v[0] = in ? s.G[base + (in ? col : 0)] : 0.0;
      v[1] = v[2] = v[3] = 0.0;
      v[4] = in ? s.G[base + len + (in ? col : 0)] : 0.0;
    }
    v[5] = col == 2 * k ? 1.0 : 0.0;
    v[6] = col == 2 * k + 1 ? 1.0 : 0.0;
  };

  // Y_k = V_k x for every stage, and the extra dense rows' dots (ex[0] a_sw.x, ex[1] g_epsi.x)
  auto stage_local = [&](const double* x) {
    if (t < 5 * (N - 1)) {
      const int k = 1 + t / 5, r = t % 5, len = 2 * k;
      const double* g = &s.G[L::gst(k) + r * len];
      double acc = 0.0;
      for (int j = 0; j < len; ++j) acc += g[j] * x[j];
      s.Y[k][r] = acc;
    } else if (t < 5 * (N - 1) + 2 * M) {
      const int q = t - 5 * (N - 1), m = q >> 1, r = q & 1, len = 2 * (N + m);
      const double* g = &s.G[L::gpm(m) + r * len];
      double acc = 0.0;
      for (int j = 0; j < len; ++j) acc += g[j] * x[j];
      s.Y[N + m][r ? 4 : 0] = acc;
    } else if (t < 5 * (N - 1) + 2 * M + 2) {
      const int q = t - 5 * (N - 1) - 2 * M;
      const int len = q == 0 ? 2 * N + 2 : 2 * (H - 1);
      const double* g = &s.G[q == 0 ? L::SW0 : L::T0];
      double acc = 0.0;
      for (int j = 0; j < len; ++j) acc += g[j] * x[j];
      s.ex[q] = acc;
    }
    if (t >= CTH - H) {  // inputs and structural zeros
      const int k = t - (CTH - H);
      s.Y[k][5] = x[2 * k];
      s.Y[k][6] = x[2 * k + 1];
      if (k == 0) {
#pragma unroll
        for (int r = 0; r < 5; ++r) s.Y[0][r] = 0.0;
      }
      if (k >= N) s.Y[k][1] = s.Y[k][2] = s.Y[k][3] = 0.0;
    }
    __syncthreads();
  };

  // out_j = sum_k V_k[:, j]' R_k  (thread j < n)
  auto adjoint = [&](int j) -> double {
    const int kj = j >> 1;
    double acc = s.R[kj][5 + (j & 1)];
    if (kj < N) {
      for (int k = kj + 1; k < N; ++k) {
        const int len = 2 * k, base = L::gst(k) + j;
#pragma unroll
        for (int r = 0; r < 5; ++r) acc += s.G[base + r * len] * s.R[k][r];
      }
    }
    for (int m = (kj < N ? 0 : kj - N + 1); m < M; ++m) {
      const int len = 2 * (N + m), base = L::gpm(m) + j;
      acc += s.G[base] * s.R[N + m][0] + s.G[base + len] * s.R[N + m][4];
    }
    return acc;
  };

  // slew pairs between columns a and a + 2: weight c2 (H entries) for the pair starting at a
  auto pair_w = [&](int a) -> double {  // 2 * w / ds * S^2, 0 if no pair
    const int k = a >> 1, cc = a & 1;
    if (k > H - 2) return 0.0;
    double w;
    if (cc == 0) w = (k == N - 1 ? CW.w_switch : W.w_Fx) / s.dsv[k];
    else if (k >= N) w = CW.w_Fy / s.dsv[k];
    else return 0.0;
    return 2.0 * w * S * S;
  };

  // one predict call site (the final pass is the output rollout x* = rollout(u*)): a second
  // call site made the compiler outline the rollout, and the call spilled ~400 VGPRs
  // SQP update state: a step under test (tries > 0) is ub = uo + 2^-(tries-1) du (du = the QP
  // solution z, untouched by the rollout), the last try the unchanged iterate (oracle/casc_sqp.py)
  int sqp_done = 0, tries = 0, it = 0;
  bool test = false;  // the iterate's own rollout is inside the domain (else the full step, untested)
  for (;;) {
    CT_STAMP(t_p0)
    predict();
    __syncthreads();
    first = false;
    CT_ACC(CT_PRED, t_p0)
    if (tries > 0) {  // cut the step back while its rollout leaves the domain
      if (test && s.dom == 0 && tries <= DOM_HALVINGS) {
        const double a = tries < DOM_HALVINGS ? ldexp(1.0, -tries) : 0.0;
        if (t < n) {
          const int kk = t >> 1, cc = t & 1;
          const double scl = (cc == 0 || kk >= N) ? S : 1.0;
          s.ub[kk][cc] = a > 0.0 ? s.uo[kk][cc] + a * (s.z[t] * scl) : s.uo[kk][cc];
        }
        ++tries;
        __syncthreads();
        continue;
      }
      tries = 0;
      ++it;
    }
    CT_STAMP(t_l0)
    if (it == W.sqp_iters || s.flag[0] == VC_NONFINITE) break;

    // ---------------- linearize ----------------
    if (t < (N - 1) * 10) {
      const int k = t / 10, q = t % 10;
      D1 x[8], u2[2], xn[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = D1(s.xs[k][i]);
      u2[0] = D1(s.ub[k][0]);
      u2[1] = D1(s.ub[k][1]);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i].d[0] = (i == q) ? 1.0 : 0.0;
      u2[0].d[0] = (q == 8) ? 1.0 : 0.0;
      u2[1].d[0] = (q == 9) ? 1.0 : 0.0;
      const D1 kp(s.kap[k]);
      rk4_apply<D1, 8>(x, D1(s.dsv[k]), [&](const D1* xx, D1* f) { dyn_spatial_ode<D1, double>(xx, u2, kp, c, f); }, xn);
#pragma unroll
      for (int i = 0; i < 8; ++i) s.u.lin.As[k][i][q] = xn[i].d[0];
    }
    for (int t2 = t; t2 < (M - 1) * 7; t2 += CTH) {
      const int m = t2 / 7, q = t2 % 7, j = N + m;
      D1 x[5], u2[2], f[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) x[i] = D1(s.xp[m][i]);
      u2[0] = D1(s.ub[j][0]);
      u2[1] = D1(s.ub[j][1]);
#pragma unroll
      for (int i = 0; i < 5; ++i) x[i].d[0] = (i == q) ? 1.0 : 0.0;
      u2[0].d[0] = (q == 5) ? 1.0 : 0.0;
      u2[1].d[0] = (q == 6) ? 1.0 : 0.0;
      pm_spatial_ode<D1, double>(x, u2, D1(s.kap[j]), c, f);
      const double h = s.dsv[j];
#pragma unroll
      for (int i = 0; i < 5; ++i) s.u.lin.Ap[m][i][q] = x[i].d[0] + h * f[i].d[0];
    }
    if (t == CTH - 1) {  // switching map Jacobian (cascaded_mpc.py:256-277)
      const double Ux = s.xs[N - 1][0], Uy = s.xs[N - 1][1];
      const double V = sqrt(Ux * Ux + Uy * Uy), q2 = Ux * Ux + Uy * Uy;
#pragma unroll
      for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) s.u.lin.Sw[r][i] = 0.0;
      s.u.lin.Sw[0][0] = Ux / V;
      s.u.lin.Sw[0][1] = Uy / V;
      s.u.lin.Sw[1][4] = 1.0;
      s.u.lin.Sw[2][5] = 1.0;
      s.u.lin.Sw[3][0] = -Uy / q2;
      s.u.lin.Sw[3][1] = Ux / q2;
      s.u.lin.Sw[3][6] = 1.0;
      s.u.lin.Sw[4][7] = 1.0;
    }
    if (t >= CTH - 6 && t < CTH - 1) {  // lateral residual Fy_f + Fy_r at stage N-1 (cascaded_mpc.py:250-255)
      const int q = t - (CTH - 6);
      D1 X5[5];
#pragma unroll
      for (int i = 0; i < 4; ++i) X5[i] = D1(s.xs[N - 1][i]);
      X5[4] = D1(s.ub[N - 1][0]);
#pragma unroll
      for (int i = 0; i < 5; ++i) X5[i].d[0] = (i == q) ? 1.0 : 0.0;
      const D1 fy = dyn_lateral_sum<D1, double>(X5, c);
      s.sc[1 + q] = fy.d[0];
      if (q == 0) s.sc[0] = fy.v;
    }
    __syncthreads();
    CT_ACC(CT_LIN, t_l0)
    CT_STAMP(t_c0)

    // ---------------- condense (thread j = decision column) ----------------
    if (t < n) {
      const int j = t, kj = j >> 1, cj = j & 1;
      double c8[8], c5[5];
#pragma unroll
      for (int i = 0; i < 8; ++i) c8[i] = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i) c5[i] = 0.0;
      int m0;
      if (kj < N) {
        const double scl = cj ? 1.0 : S;
        if (kj < N - 1) {
#pragma unroll
          for (int i = 0; i < 8; ++i) c8[i] = scl * s.u.lin.As[kj][i][8 + cj];
        }
        for (int k = kj + 1; k < N; ++k) {
          const int len = 2 * k, base = L::gst(k) + j;
          s.G[base] = c8[0];
          s.G[base + len] = c8[1];
          s.G[base + 2 * len] = c8[2];
          s.G[base + 3 * len] = c8[3];
          s.G[base + 4 * len] = c8[5];
          if (k < N - 1) {
            double nx[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              double a = 0.0;
#pragma unroll
              for (int q = 0; q < 8; ++q) a += s.u.lin.As[k][i][q] * c8[q];
              nx[i] = a;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) c8[i] = nx[i];
          }
        }
        // switching cost's lateral row (the sensitivity at stage N-1 is c8 now)
        double a = -(s.sc[1] * c8[0] + s.sc[2] * c8[1] + s.sc[3] * c8[2] + s.sc[4] * c8[3]);
        if (j == 2 * (N - 1)) a -= s.sc[5] * S;
        s.G[L::SW0 + j] = a;
#pragma unroll
        for (int r = 0; r < 5; ++r) {
          double v = 0.0;
#pragma unroll
          for (int q = 0; q < 8; ++q) v += s.u.lin.Sw[r][q] * c8[q];
          c5[r] = v;
        }
        m0 = 0;
      } else {
        const int mj = kj - N;
        if (mj < M - 1) {
#pragma unroll
          for (int i = 0; i < 5; ++i) c5[i] = S * s.u.lin.Ap[mj][i][5 + cj];
        }
        if (j < 2 * N + 2) s.G[L::SW0 + j] = (j == 2 * N + 1) ? S : 0.0;
        m0 = mj + 1;
      }
      for (int m = m0; m < M; ++m) {
        const int len = 2 * (N + m), base = L::gpm(m) + j;
        s.G[base] = c5[0];
        s.G[base + len] = c5[2];
        if (m < M - 1) {
          double nx[5];
#pragma unroll
          for (int i = 0; i < 5; ++i) {
            double a = 0.0;
#pragma unroll
            for (int q = 0; q < 5; ++q) a += s.u.lin.Ap[m][i][q] * c5[q];
            nx[i] = a;
          }
#pragma unroll
          for (int i = 0; i < 5; ++i) c5[i] = nx[i];
        }
      }
      if (j < 2 * (H - 1)) {
        s.G[L::T0 + j] = c5[3];
        s.G[L::T0 + 2 * (H - 1) + j] = c5[4];
      }
    }
    __syncthreads();
    CT_ACC(CT_COND, t_c0)
    CT_STAMP(t_s0)

    // ---------------- QP setup ----------------
    // rows and stage costs: 4 lanes per stage k = t / 4 (t < 4H), lane q = t % 4
    Rows3 R3;
    double Qp[28], qv[7];
    const bool stl = t < 4 * H;
    const int k = stl ? (t >> 2) : 0, q = t & 3;
#pragma unroll
    for (int e = 0; e < 28; ++e) Qp[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 7; ++e) qv[e] = 0.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      R3.d[i] = 1.0;
      R3.act[i] = 0.0;
#pragma unroll
      for (int e = 0; e < 7; ++e) R3.c[i][e] = 0.0;
    }
    {
      // obstacle barrier (cascaded_mpc.py:173-176, 233-237), convexified in ey
      auto ey_cost = [&](double ey, double sv, double ds, double lo, double hi, double wdev) {
        const double blo = ey < lo ? W.w_b : 0.0, bhi = ey > hi ? W.w_b : 0.0;
        double qo = 0.0, po = 0.0;
        if (A.obs.n > 0) obstacle_ey_model<double>(A.obs, sv, ey, W.w_obs * ds, po, qo);
        Qp[sym7(4, 4)] += 2.0 * ds * (wdev + blo + bhi) + qo;
        qv[4] += 2.0 * ds * (wdev * ey + blo * (ey - lo) + bhi * (ey - hi)) + po;
      };
      if (k < N) {
        // stage functions with duals: d[0] along this lane's state (Ux, Uy, r, delta), d[1] along Fx
        D2 X5[5];
#pragma unroll
        for (int i = 0; i < 4; ++i) X5[i] = D2(s.xs[k][i]);
        X5[4] = D2(s.ub[k][0]);
#pragma unroll
        for (int i = 0; i < 4; ++i) X5[i].d[0] = (i == q) ? 1.0 : 0.0;
        X5[4].d[1] = 1.0;
        D2 o[7];
        dyn_stage_terms<D2, double>(X5, c, o);
        double fv[7], gr[7][5];
        const int qb = lane & ~3;
#pragma unroll
        for (int r = 0; r < 7; ++r) {
          fv[r] = o[r].v;
#pragma unroll
          for (int a = 0; a < 4; ++a) gr[r][a] = __shfl(o[r].d[0], qb | a, 64);
          gr[r][4] = o[r].d[1];
        }
        const double ds = s.dsv[k];
        if (q == 0 && stl) {
          // Gauss-Newton cost (cascaded_mpc.py:130-171)
          ey_cost(s.xs[k][5], s.xs[k][4], ds, W.ey_min, W.ey_max, W.w_dev);
          Qp[sym7(6, 6)] += 2.0 * W.w_w;
          qv[6] += 2.0 * W.w_w * s.ub[k][1];
#pragma unroll
          for (int sr = 0; sr < 2; ++sr) {
            if (fv[sr] >= 0.0) {
              const double a7[7] = {gr[sr][0], gr[sr][1], gr[sr][2], gr[sr][3], 0.0, gr[sr][4] * S, 0.0};
#pragma unroll
              for (int a = 0; a < 7; ++a) {
                qv[a] += 2.0 * W.w_slip * fv[sr] * a7[a];
#pragma unroll
                for (int e = a; e < 7; ++e) Qp[sym7(a, e)] += 2.0 * W.w_slip * a7[a] * a7[e];
              }
            }
          }
        }
        // rows (slot 3q + i)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int sl = 3 * q + i;
          double* cr = R3.c[i];
          double d = 1.0, act = 1.0;
          if (sl == 0) { cr[0] = -1.0; d = s.xs[k][0] - W.Ux_min; act = k >= 1; }
          else if (sl == 1) { cr[3] = 1.0; d = W.delta_max - s.xs[k][3]; act = k >= 1; }
          else if (sl == 2) { cr[3] = -1.0; d = s.xs[k][3] - W.delta_min; act = k >= 1; }
          else if (sl <= 7) {
            const int r = sl - 1;  // stage functions 2..6: peng, tyre f up / lo, r up / lo
#pragma unroll
            for (int rr = 2; rr < 7; ++rr) {
              if (rr == r) {
                cr[0] = gr[rr][0] / S; cr[1] = gr[rr][1] / S; cr[2] = gr[rr][2] / S; cr[3] = gr[rr][3] / S;
                cr[5] = gr[rr][4];
                d = -fv[rr] / S;
              }
            }
          } else if (sl == 8) {
            cr[6] = 1.0;
            d = W.w_max - s.ub[k][1];
            if (A.qp.trust_w > 0) d = fmin(d, A.qp.trust_w);
          } else if (sl == 9) {
            cr[6] = -1.0;
            d = s.ub[k][1] - W.w_min;
            if (A.qp.trust_w > 0) d = fmin(d, A.qp.trust_w);
          } else {
            cr[5] = sl == 10 ? 1.0 : -1.0;
            d = W.trust_Fx / S;
            act = W.trust_Fx > 0;
          }
          R3.d[i] = d;
          R3.act[i] = stl ? act : 0.0;
          if (!(act > 0)) {
#pragma unroll
            for (int e = 0; e < 7; ++e) cr[e] = 0.0;
            R3.d[i] = 1.0;
          }
        }
      } else {
        const int m = k - N;
        const double V = s.xp[m][0];
        if (q == 0 && stl) {
          // point-mass stage cost (cascaded_mpc.py:204-239) and the terminal cost (:279-304)
          ey_cost(s.xp[m][2], s.xp[m][1], s.dsv[k], CW.ey_min_pm, CW.ey_max_pm, CW.w_dev_pm);
          if (m == M - 1) {
            if (V >= W.max_speed) {
              Qp[sym7(0, 0)] += 2.0 * W.w_speed;
              qv[0] += 2.0 * W.w_speed * (V - W.max_speed);
            }
            Qp[sym7(4, 4)] += 2.0 * W.w_ey;
            qv[4] += 2.0 * W.w_ey * s.xp[m][2];
          }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int sl = 3 * q + i;
          double* cr = R3.c[i];
          double d = 1.0, act = 1.0;
          if (sl == 0) { cr[0] = -1.0; d = V - CW.V_min; }
          else if (sl == 1) {  // Fx <= Peng / V (cascaded_mpc.py:193), divided by S
            cr[0] = c.Peng / (V * V) / S;
            cr[5] = 1.0;
            d = -(s.ub[k][0] - c.Peng / V) / S;
          } else if (sl <= 5) {
            cr[sl <= 3 ? 5 : 6] = (sl & 1) ? -1.0 : 1.0;
            d = W.trust_Fx / S;
            act = W.trust_Fx > 0;
          } else {
            act = 0.0;
          }
          R3.d[i] = d;
          R3.act[i] = stl ? act : 0.0;
          if (!(act > 0)) {
#pragma unroll
            for (int e = 0; e < 7; ++e) cr[e] = 0.0;
            R3.d[i] = 1.0;
          }
        }
      }
    }
    // distribute the stage cost Hessian over the quad: lane q keeps packed entries 7q..7q+6
    double Qd[7];
    {
      const int qb = lane & ~3;
#pragma unroll
      for (int e = 0; e < 28; ++e) {
        const double v = __shfl(Qp[e], qb, 64);
        if (e / 7 == q) Qd[e % 7] = v;
      }
    }
    // constant gradient part gp (slews, switching residuals, terminal epsi and time)
    const double csw = CW.w_switch / s.dsv[N - 1];
    const double r_lat = s.ub[N][1] - s.sc[0];
    const double ep_end = s.xp[M - 1][3];
    if (t < n) {
      const int j = t;
      double g = 0.0;
      auto lin = [&](int a) -> double {  // 2 w r0 S of the pair starting at column a
        const double c2 = pair_w(a);
        return c2 == 0.0 ? 0.0 : c2 / S * (s.ub[(a >> 1) + 1][a & 1] - s.ub[a >> 1][a & 1]);
      };
      if (j >= 2) g += lin(j - 2);
      g -= lin(j);
      if (j < 2 * N + 2) g += 2.0 * csw * r_lat * s.G[L::SW0 + j];
      if (j < 2 * (H - 1)) {
        g += 2.0 * W.w_epsi * ep_end * s.G[L::T0 + j];
        g += W.w_time * s.G[L::T0 + 2 * (H - 1) + j];
      }
      s.gp[j] = g;
      s.z[j] = 0.0;
    }
    // P x (prox, slews, switching lateral and terminal epsi rank-1 terms); ex[] must hold the dots
    auto px = [&](const double* x, int j) -> double {
      double v = 2.0 * A.qp.prox * x[j];
      const double cf = pair_w(j);
      if (cf != 0.0) v += cf * (x[j] - x[j + 2]);
      if (j >= 2) {
        const double cb = pair_w(j - 2);
        if (cb != 0.0) v += cb * (x[j] - x[j - 2]);
      }
      if (j < 2 * N + 2) v += 2.0 * csw * s.G[L::SW0 + j] * s.ex[0];
      if (j < 2 * (H - 1)) v += 2.0 * W.w_epsi * s.G[L::T0 + j] * s.ex[1];
      return v;
    };
    auto build = [&]() { casc_build<N, M>(s, csw, W.w_epsi, A.qp.prox, W.w_Fx, CW.w_Fy, CW.w_switch, S); };

    if (A.mode == 1) {  // first QP's H and g (vc_condense)
      if (stl && q == 0) {
#pragma unroll
        for (int e = 0; e < 28; ++e) s.W[k][e] = __shfl(Qp[e], lane & ~3, 64);
#pragma unroll
        for (int e = 0; e < 7; ++e) s.R[k][e] = qv[e];
      }
      __syncthreads();
      build();
      for (int e = t; e < n * n; e += CTH) {
        const int i = e / n, j = e % n;
        A.H_out[(size_t)b * n * n + e] = s.u.Mp[i >= j ? L::pidx(i, j) : L::pidx(j, i)];
      }
      if (t < n) A.g_out[(size_t)b * n + t] = adjoint(t) + s.gp[t];
      return;
    }

    // ---------------- interior point (Mehrotra predictor-corrector) ----------------
    double sl3[3], lm3[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      sl3[i] = R3.act[i] > 0 ? fmax(R3.d[i], 0.0) + 1.0 : 1.0;
      lm3[i] = R3.act[i] > 0 ? 1.0 : 0.0;
    }
    const double m_act = block_reduce<0>(R3.act[0] + R3.act[1] + R3.act[2], s.red);
    CT_ACC(CT_SETUP, t_s0)
    int ipm_it = 0;
    bool conv = false, fail = false;
    __syncthreads();
    for (ipm_it = 0; ipm_it < A.qp.max_iter; ++ipm_it) {
      CT_STAMP(t_i0)
      stage_local(s.z);
      double pxj = 0.0;
      if (t < n) pxj = px(s.z, t);
      double Yk[7];
#pragma unroll
      for (int e = 0; e < 7; ++e) Yk[e] = s.Y[k][e];
      double qy[7];
      {
        double pq[7];
#pragma unroll
        for (int a = 0; a < 7; ++a) pq[a] = 0.0;
#pragma unroll
        for (int a = 0; a < 7; ++a)
#pragma unroll
          for (int e = a; e < 7; ++e) {
            const int id = sym7(a, e);
            const double v = (id / 7 == q) ? Qd[id % 7] : 0.0;
            pq[a] += v * Yk[e];
            if (e != a) pq[e] += v * Yk[a];
          }
#pragma unroll
        for (int a = 0; a < 7; ++a) {
          double v = pq[a];
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          qy[a] = v + qv[a];  // qv is nonzero on lane 0 only: stage_vec's quad sum must not add it again
        }
      }
      double rp3[3], Dg3[3];
      double smu = 0.0, rpm = 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        double cy = 0.0;
#pragma unroll
        for (int e = 0; e < 7; ++e) cy += R3.c[i][e] * Yk[e];
        rp3[i] = R3.act[i] > 0 ? cy + sl3[i] - R3.d[i] : 0.0;
        Dg3[i] = R3.act[i] > 0 ? lm3[i] / sl3[i] : 0.0;
        smu += R3.act[i] * sl3[i] * lm3[i];
        rpm = fmax(rpm, fabs(rp3[i]));
      }
      const double mu = block_reduce<0>(smu, s.red) / fmax(m_act, 1.0);
      const double rp_inf = block_reduce<1>(rpm, s.red);
      // dual residual r_d = H z + g + C' lambda
      auto stage_vec = [&](const double* wv) {  // R_k = Q_k Y_k + q_k + sum_i wv_i c_i (quad-reduced)
        double v[7];
#pragma unroll
        for (int e = 0; e < 7; ++e) {
          double a = 0.0;
#pragma unroll
          for (int i = 0; i < 3; ++i) a += wv[i] * R3.c[i][e];
          a += __shfl_xor(a, 1, 64);
          a += __shfl_xor(a, 2, 64);
          v[e] = a + qy[e];
        }
        if (stl && q == 0) {
#pragma unroll
          for (int e = 0; e < 7; ++e) s.R[k][e] = v[e];
        }
        __syncthreads();
      };
      CT_ACC(CT_LOCAL, t_i0)
      CT_STAMP(t_r0)
      stage_vec(lm3);
      double rdm = 0.0;
      if (t < n) rdm = fabs(adjoint(t) + pxj + s.gp[t]);
      const double rd_inf = block_reduce<1>(rdm, s.red);
      if (!(mu == mu) || !(rd_inf == rd_inf)) { fail = true; break; }
      CT_ACC(CT_RD, t_r0)
      // mu carries the accuracy (tol = 1e-13); the residuals only need to be small in the
      // scaled units (|dz| ~ 1), a 1e-12 absolute dual residual is below fp64 resolution of
      // adjoint sums of magnitude ~1e3 and left 1 % of problems at max_iter
      if (mu <= A.qp.tol && rp_inf <= 1e-9 && rd_inf <= 1e-9) { conv = true; break; }
      CT_STAMP(t_w0)
      // W_k = Q_k + sum_i D_i c_i c_i'
#pragma unroll
      for (int a = 0; a < 7; ++a)
#pragma unroll
        for (int e = a; e < 7; ++e) {
          const int id = sym7(a, e);
          double v = 0.0;
#pragma unroll
          for (int i = 0; i < 3; ++i) v += Dg3[i] * R3.c[i][a] * R3.c[i][e];
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          if (stl && id / 7 == q) s.W[k][id] = v + Qd[id % 7];
        }
      __syncthreads();
      CT_ACC(CT_WASM, t_w0)
      CT_STAMP(t_b0)
      build();
      CT_ACC(CT_BUILD, t_b0)
      CT_STAMP(t_h0)
      casc_cholesky<N, M>(s);
      CT_ACC(CT_CHOL, t_h0)
      if (s.flag[3]) { fail = true; break; }

      // solve M dz = rhs (in s.rhs) -> s.dz; wave 0, lanes own rows lane and lane + 64
      auto chol_solve = [&]() { casc_tri_solve<N, M>(s); };
      // Newton direction for a given w (per row): rhs = -(adjoint(QY + q + sum (lam + w) c) + Px + gp)
      auto direction = [&](const double* w3, double* dsl, double* dlm) {
        double lw[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) lw[i] = lm3[i] + w3[i];
        stage_vec(lw);
        if (t < n) s.rhs[t] = -(adjoint(t) + pxj + s.gp[t]);
        __syncthreads();
        CT_STAMP(t_v0)
        chol_solve();
        CT_ACC(CT_SOLVE, t_v0)
        stage_local(s.dz);
        double Yd[7];
#pragma unroll
        for (int e = 0; e < 7; ++e) Yd[e] = s.Y[k][e];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          double cy = 0.0;
#pragma unroll
          for (int e = 0; e < 7; ++e) cy += R3.c[i][e] * Yd[e];
          dsl[i] = R3.act[i] > 0 ? -rp3[i] - cy : 0.0;
          dlm[i] = R3.act[i] > 0 ? w3[i] + Dg3[i] * cy : 0.0;
        }
      };
      auto max_step = [&](const double* dsl, const double* dlm) -> double {
        double a = 1.0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (R3.act[i] > 0) {
            if (dsl[i] < 0.0) a = fmin(a, -sl3[i] / dsl[i]);
            if (dlm[i] < 0.0) a = fmin(a, -lm3[i] / dlm[i]);
          }
        }
        return block_reduce<2>(a, s.red);
      };
      CT_STAMP(t_d0)
      // predictor (affine)
      double w3[3], dsa[3], dla[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) w3[i] = R3.act[i] > 0 ? (-sl3[i] * lm3[i] + lm3[i] * rp3[i]) / sl3[i] : 0.0;
      direction(w3, dsa, dla);
      const double aa = max_step(dsa, dla);
      double mua = 0.0;
#pragma unroll
      for (int i = 0; i < 3; ++i) mua += R3.act[i] * (sl3[i] + aa * dsa[i]) * (lm3[i] + aa * dla[i]);
      mua = block_reduce<0>(mua, s.red) / fmax(m_act, 1.0);
      const double sg = mu > 0 ? (mua / mu) * (mua / mu) * (mua / mu) : 0.0;
      // corrector
#pragma unroll
      for (int i = 0; i < 3; ++i)
        w3[i] = R3.act[i] > 0 ? (sg * mu - sl3[i] * lm3[i] - dsa[i] * dla[i] + lm3[i] * rp3[i]) / sl3[i] : 0.0;
      double dsc[3], dlc[3];
      direction(w3, dsc, dlc);
      const double al = fmin(1.0, 0.995 * max_step(dsc, dlc));
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (R3.act[i] > 0) {
          sl3[i] += al * dsc[i];
          lm3[i] += al * dlc[i];
        }
      }
      if (t < n) s.z[t] += al * s.dz[t];
      __syncthreads();
      CT_ACC(CT_DIR, t_d0)
    }
    if (t == 0) {
      s.flag[1] += ipm_it;
      if (fail) { s.flag[0] = VC_NONFINITE; s.flag[2] = 1; }
      else if (!conv) { if (s.flag[0] == VC_SOLVED) s.flag[0] = VC_MAX_ITER; s.flag[2] &= ~2; }

    }
    if (fail) { __syncthreads(); break; }
    // update ubar (scaled back)
    if (t < n) {
      const int kk = t >> 1, cc = t & 1;
      const double scl = (cc == 0 || kk >= N) ? S : 1.0;
      s.uo[kk][cc] = s.ub[kk][cc];
      s.ub[kk][cc] += s.z[t] * scl;
    }
    test = s.dom != 0;
    tries = 1;
    __syncthreads();
    ++sqp_done;
  }

  // outputs: u*, x* = rollout(u*) (the loop's last predict), u0, status, iterations
  for (int i = t; i < H; i += CTH) {
    A.u_out[((size_t)b * H + i) * 2] = s.ub[i][0];
    A.u_out[((size_t)b * H + i) * 2 + 1] = s.ub[i][1];
  }
  for (int e = t; e < H * 8; e += CTH) {
    const int kk = e >> 3, i = e & 7;
    double v;
    if (kk < N) v = s.xs[kk][i];
    else v = i < 5 ? s.xp[kk - N][i] : 0.0;
    A.x_out[(size_t)b * H * 8 + e] = v;
  }
  if (t == 0) {
    A.u0[(size_t)b * 2] = s.ub[0][0];
    A.u0[(size_t)b * 2 + 1] = s.ub[0][1];
    // x* (the last rollout) outside the models' domain: not a solution (VC_OUT_OF_DOMAIN)
    A.status[b] = (s.flag[0] == VC_NONFINITE || s.dom != 0) ? s.flag[0] : VC_OUT_OF_DOMAIN;
    A.iters[b] = s.flag[1];
    if (A.diag) {
#ifdef VC_TIMING
      constexpr int DS = 4 + CT_NSLOT;
      tacc[CT_TOTAL] = __builtin_amdgcn_s_memtime() - t_start;
      for (int i = 0; i < CT_NSLOT; ++i) A.diag[(size_t)b * DS + 4 + i] = double(tacc[i]);
#else
      constexpr int DS = 4;
#endif
      A.diag[(size_t)b * DS + 0] = 0.0;
      A.diag[(size_t)b * DS + 1] = 0.0;
      A.diag[(size_t)b * DS + 2] = s.flag[2];
      A.diag[(size_t)b * DS + 3] = sqp_done;
    }
  }
}

}  // namespace

bool casc_sqp_built(int N, int M) { return N == 20 && M == 40; }

hipError_t launch_casc_sqp(const CascSqpArgs& a, int N, int M, hipStream_t stream) {
  if (a.B <= 0) return hipSuccess;
  if (!casc_sqp_built(N, M)) return hipErrorInvalidValue;
  if (a.car.tyre == VC_TYRE_LINEAR)
    hipLaunchKernelGGL((casc_sqp_kernel<20, 40, VC_TYRE_LINEAR>), dim3(a.B), dim3(CTH), 0, stream, a);
  else
    hipLaunchKernelGGL((casc_sqp_kernel<20, 40, VC_TYRE_FIALA>), dim3(a.B), dim3(CTH), 0, stream, a);
  return hipGetLastError();
}

}  // namespace vc
