// vcmpc_abi.hip -- the C ABI of libvcmpc.so (declared in include/vcmpc.h).
//
// Context management, argument validation, host<->device staging for
// VC_HOST_PTRS calls, and dispatch to the HIP kernels.  No compute happens on
// the host: every numeric result comes from a gfx950 kernel.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "vc_kernels.hpp"
#include "vcmpc.h"


struct vc_ctx {
  int device = 0, model = 0, N = 0, max_batch = 0, dtype = 0;
  vc_params p{};
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  void* arena = nullptr;
  size_t arena_bytes = 0;
  void* track = nullptr;  // vc_track_set: [n][4] fp64 curvature pieces
  int track_n = 0;
  double track_h = 0.0, track_len = 0.0;
  void* sim = nullptr;    // vc_simulate scratch (kappa, ds, x, u0, status, iters)
  size_t sim_bytes = 0;
  void* ls = nullptr;     // kinematic SQP scratch (vc_qp.kin_sqp > 0): u_prev, status / iteration sums
  size_t ls_bytes = 0;
  void* jw = nullptr;     // single-track / cascaded SQP: stage Jacobians of the kernels that keep them out of LDS
  size_t jw_bytes = 0;
  int fault_iter = -1, fault_problem = -1;  // vc_debug_qp_fault (tests only)
  std::string err;
};

namespace {
thread_local std::string g_create_err;

int fail(vc_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  else g_create_err = buf;
  return code;
}

#define VC_HIP(ctx, call)                                                                         \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) return fail((ctx), VC_E_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

size_t esize(const vc_ctx* c) { return c->dtype == VC_F32 ? 4 : 8; }

// Grow-only device scratch owned by the context (freed once the stream has drained).
int ensure_scratch(vc_ctx* c, void** p, size_t* have, size_t need) {
  if (need <= *have) return 0;
  VC_HIP(c, hipStreamSynchronize(c->stream));
  if (*p) VC_HIP(c, hipFree(*p));
  *p = nullptr;
  *have = 0;
  VC_HIP(c, hipMalloc(p, need));
  *have = need;
  return 0;
}
int nx_of(const vc_ctx* c) { return c->model == VC_MODEL_KINEMATIC ? 6 : 8; }

int ensure_arena(vc_ctx* c, size_t bytes) {
  if (bytes <= c->arena_bytes) return 0;
  VC_HIP(c, hipSetDevice(c->device));
  if (c->arena) VC_HIP(c, hipFree(c->arena));
  c->arena = nullptr;
  c->arena_bytes = 0;
  VC_HIP(c, hipMalloc(&c->arena, bytes));
  c->arena_bytes = bytes;
  return 0;
}

// Staging plan for a host-pointer call: each buffer gets an aligned arena slice.
struct Slot {
  const void* host_in;  // copied H2D before the launch (may be null)
  void* host_out;       // copied D2H after the launch (may be null)
  size_t bytes;
  void* dev;
};

int stage(vc_ctx* c, std::vector<Slot>& slots) {
  size_t total = 0;
  for (auto& s : slots) total += (s.bytes + 255) & ~size_t(255);
  if (int r = ensure_arena(c, total ? total : 256)) return r;
  size_t off = 0;
  for (auto& s : slots) {
    s.dev = static_cast<char*>(c->arena) + off;
    off += (s.bytes + 255) & ~size_t(255);
    if (s.host_in && s.bytes) VC_HIP(c, hipMemcpyAsync(s.dev, s.host_in, s.bytes, hipMemcpyHostToDevice, c->stream));
  }
  return 0;
}

int unstage(vc_ctx* c, const std::vector<Slot>& slots) {
  for (auto& s : slots)
    if (s.host_out && s.bytes) VC_HIP(c, hipMemcpyAsync(s.host_out, s.dev, s.bytes, hipMemcpyDeviceToHost, c->stream));
  VC_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

int check_common(vc_ctx* c, int B, int flags) {
  if (!c) return VC_E_ARG;
  if (B < 0 || B > c->max_batch) return fail(c, VC_E_ARG, "batch %d outside [0, max_batch=%d]", B, c->max_batch);
  if (flags != VC_HOST_PTRS && flags != VC_DEVICE_PTRS) return fail(c, VC_E_ARG, "bad flags %d", flags);
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return fail(c, VC_E_HIP, "hipSetDevice: %s", hipGetErrorString(e));
  return 0;
}

vc::ModelArgs model_args(const vc_ctx* c, int B) {
  vc::ModelArgs m{};
  m.model = c->model;
  m.B = B;
  m.N = c->N;
  m.M = c->model == VC_MODEL_CASCADED ? c->p.casc.horizon_pm : 0;
  m.shift = c->p.qp.shift;
  m.L = c->p.kin_car.l;
  m.dyn64 = vc::make_dyn_coef<double>(c->p.dyn_car);
  m.dyn32 = vc::make_dyn_coef<float>(c->p.dyn_car);
  return m;
}

// stages of the solve arrays: kappa / ds / ubar span H (= N, or N + horizon_pm for a
// cascaded context); xbar has N + 1 (kinematic) or H state columns
int nh_of(const vc_ctx* c) { return c->N + (c->model == VC_MODEL_CASCADED ? c->p.casc.horizon_pm : 0); }
int ns_of(const vc_ctx* c) { return c->model == VC_MODEL_KINEMATIC ? c->N + 1 : nh_of(c); }
size_t al256(size_t b) { return (b + 255) & ~size_t(255); }
vc::TrackTable track_table(const vc_ctx* c) {
  return vc::TrackTable{static_cast<const double*>(c->track), c->track_n, c->track_h, c->track_len};
}

// The condensed kernel (kin_ltv.hip) where it is built (N = 20, the bench's C2/C4 shape),
// the stagewise Riccati kernel (kin_ric.hip) for the other horizons (kinematic.yaml: 50).
// the condensed kernel for the one-step contract only: the globalised step's QPs (obstacle
// barriers, condition numbers ~1e6) need the stagewise factorisation's accuracy (kin_ric.hip
// matches the oracle to 1e-8 there, the condensed normal equations to 8e-5; scripts/kin_sqp_debug.py)
bool kin_condensed(const vc_ctx* c) {
  // elastic rows (qp.elastic) and multiple shooting are built in the stagewise kernel only
  return vc::kin_ltv_smem_bytes(c->N) > 0 && c->p.qp.solver == 0 && c->p.qp.kin_sqp <= 0 && !c->p.qp.ms &&
         c->p.qp.elastic == 0.0;
}
bool kin_solve_built(const vc_ctx* c) {
  return c->model == VC_MODEL_KINEMATIC && c->dtype == VC_F64 && (kin_condensed(c) || vc::kin_ric_built(c->N));
}
bool dyn_solve_built(const vc_ctx* c) {
  if (c->model != VC_MODEL_DYNAMIC) return false;
  if (c->dtype == VC_F32) return vc::dyn_sqp_smem_bytes(c->N) > 0;
  return vc::st_sqp_built(c->N);
}
// Cascaded: the stagewise Riccati kernel (casc_ric.hip; M = 15, 25, 35, 40) unless
// qp.solver = 2 asks for the condensed one (casc_sqp.hip, M = 40).
bool casc_stagewise(const vc_ctx* c) {
  return c->p.qp.solver != 2 && vc::casc_ric_built(c->N, c->p.casc.horizon_pm);
}
bool casc_solve_built(const vc_ctx* c) {
  return c->model == VC_MODEL_CASCADED && c->dtype == VC_F64 &&
         (casc_stagewise(c) || vc::casc_sqp_built(c->N, c->p.casc.horizon_pm));
}

// Cascaded single-track + point-mass SQP (casc_sqp.hip), fp64: arrays span H = N + M stages.
// mode 0: solve (xbar, ubar, u0, status, iters, diag); mode 1: first QP's H, g (H_out, g_out).
int casc_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar, void* u0,
               int32_t* status, int32_t* iters, void* diag, int flags, int mode = 0, void* H_out = nullptr,
               void* g_out = nullptr) {
  const int Hs = c->N + c->p.casc.horizon_pm, n = 2 * Hs, nx = 8, nu = 2;
  const vc_dyn_mpc& w = c->p.dyn_mpc;
  if (w.sqp_iters < 1 || w.sqp_iters > 64) return fail(c, VC_E_ARG, "dyn_mpc.sqp_iters=%d outside [1,64]", w.sqp_iters);
  if (!(w.fx_scale > 0)) return fail(c, VC_E_ARG, "dyn_mpc.fx_scale must be > 0");
  if (c->p.qp.max_iter < 1) return fail(c, VC_E_ARG, "qp.max_iter must be >= 1");
  if (!(c->p.casc.ds_pm > 0)) return fail(c, VC_E_ARG, "casc.ds_pm must be > 0");
  vc::CascSqpArgs a{};
  a.B = B;
  a.mode = mode;
  a.car = vc::make_dyn_coef<double>(c->p.dyn_car);
  a.w = w;
  a.cw = c->p.casc;
  a.qp = c->p.qp;
  a.obs = c->p.obs;
  std::vector<Slot> slots;
  if (flags == VC_HOST_PTRS) {
    if (mode == 0) {
      slots = {{x0, nullptr, (size_t)B * nx * 8, nullptr},
               {kappa, nullptr, (size_t)B * Hs * 8, nullptr},
               {ds, nullptr, (size_t)B * Hs * 8, nullptr},
               {ubar, ubar, (size_t)B * Hs * nu * 8, nullptr},
               {nullptr, xbar, (size_t)B * Hs * nx * 8, nullptr},
               {nullptr, u0, (size_t)B * nu * 8, nullptr},
               {nullptr, status, (size_t)B * 4, nullptr},
               {nullptr, iters, (size_t)B * 4, nullptr},
               {nullptr, diag, diag ? (size_t)B * VC_CASC_DIAG_COLS * 8 : 0, nullptr}};
    } else {
      slots = {{x0, nullptr, (size_t)B * nx * 8, nullptr},
               {kappa, nullptr, (size_t)B * Hs * 8, nullptr},
               {ds, nullptr, (size_t)B * Hs * 8, nullptr},
               {ubar, nullptr, (size_t)B * Hs * nu * 8, nullptr},
               {nullptr, H_out, (size_t)B * n * n * 8, nullptr},
               {nullptr, g_out, (size_t)B * n * 8, nullptr}};
    }
    if (int r = stage(c, slots)) return r;
    a.x0 = (const double*)slots[0].dev;
    a.kappa = (const double*)slots[1].dev;
    a.ds = (const double*)slots[2].dev;
    a.ubar = (const double*)slots[3].dev;
    if (mode == 0) {
      a.u_out = (double*)slots[3].dev;
      a.x_out = (double*)slots[4].dev;
      a.u0 = (double*)slots[5].dev;
      a.status = (int32_t*)slots[6].dev;
      a.iters = (int32_t*)slots[7].dev;
      a.diag = diag ? (double*)slots[8].dev : nullptr;
    } else {
      a.H_out = (double*)slots[4].dev;
      a.g_out = (double*)slots[5].dev;
    }
  } else {
    a.x0 = (const double*)x0;
    a.kappa = (const double*)kappa;
    a.ds = (const double*)ds;
    a.ubar = (const double*)ubar;
    a.u_out = (double*)ubar;
    a.x_out = (double*)xbar;
    a.u0 = (double*)u0;
    a.status = status;
    a.iters = iters;
    a.diag = (double*)diag;
    a.H_out = (double*)H_out;
    a.g_out = (double*)g_out;
  }
  if (mode == 0 && casc_stagewise(c)) {
    if (const size_t jd = vc::casc_ric_jws_doubles(c->N, c->p.casc.horizon_pm, B)) {
      if (int r = ensure_scratch(c, &c->jw, &c->jw_bytes, (size_t)B * jd * 8)) return r;
      a.jws = (double*)c->jw;
    }
    VC_HIP(c, vc::launch_casc_ric(a, c->N, c->p.casc.horizon_pm, c->stream));
  }
  else VC_HIP(c, vc::launch_casc_sqp(a, c->N, c->p.casc.horizon_pm, c->stream));
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}

// Dynamic single-track SQP, fp64 (st_sqp.hip, stagewise Riccati interior point): xbar has
// N state columns.
int st_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar, void* u0,
             int32_t* status, int32_t* iters, void* diag, int flags) {
  const int N = c->N, nx = 8, nu = 2;
  const vc_dyn_mpc& w = c->p.dyn_mpc;
  vc::StSqpArgs a{};
  a.B = B;
  a.car = vc::make_dyn_coef<double>(c->p.dyn_car);
  a.w = w;
  a.qp = c->p.qp;
  a.obs = c->p.obs;
  std::vector<Slot> slots;
  if (flags == VC_HOST_PTRS) {
    slots = {{x0, nullptr, (size_t)B * nx * 8, nullptr},
             {kappa, nullptr, (size_t)B * N * 8, nullptr},
             {ds, nullptr, (size_t)B * N * 8, nullptr},
             {ubar, ubar, (size_t)B * N * nu * 8, nullptr},
             {nullptr, xbar, (size_t)B * N * nx * 8, nullptr},
             {nullptr, u0, (size_t)B * nu * 8, nullptr},
             {nullptr, status, (size_t)B * 4, nullptr},
             {nullptr, iters, (size_t)B * 4, nullptr},
             {nullptr, diag, diag ? (size_t)B * VC_ST_DIAG_COLS * 8 : 0, nullptr}};
    if (int r = stage(c, slots)) return r;
    a.x0 = (const double*)slots[0].dev;
    a.kappa = (const double*)slots[1].dev;
    a.ds = (const double*)slots[2].dev;
    a.ubar = (const double*)slots[3].dev;
    a.u_out = (double*)slots[3].dev;
    a.x_out = (double*)slots[4].dev;
    a.u0 = (double*)slots[5].dev;
    a.status = (int32_t*)slots[6].dev;
    a.iters = (int32_t*)slots[7].dev;
    a.diag = diag ? (double*)slots[8].dev : nullptr;
  } else {
    a.x0 = (const double*)x0;
    a.kappa = (const double*)kappa;
    a.ds = (const double*)ds;
    a.ubar = (const double*)ubar;
    a.u_out = (double*)ubar;
    a.x_out = (double*)xbar;
    a.u0 = (double*)u0;
    a.status = status;
    a.iters = iters;
    a.diag = (double*)diag;
  }
  if (const size_t jd = vc::st_sqp_jws_doubles(N, B)) {
    if (int r = ensure_scratch(c, &c->jw, &c->jw_bytes, (size_t)B * jd * 8)) return r;
    a.jws = (double*)c->jw;
  }
  VC_HIP(c, vc::launch_st_sqp(a, N, c->stream));
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}

// Dynamic single-track SQP (dyn_sqp.hip), fp32: xbar has N state columns.
int dyn_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar, void* u0,
              int32_t* status, int32_t* iters, void* diag, int flags, void* dbg = nullptr) {
  const int N = c->N, nx = 8, nu = 2;
  const vc_dyn_mpc& w = c->p.dyn_mpc;
  if (w.sqp_iters < 1 || w.sqp_iters > 64) return fail(c, VC_E_ARG, "dyn_mpc.sqp_iters=%d outside [1,64]", w.sqp_iters);
  if (!(w.fx_scale > 0)) return fail(c, VC_E_ARG, "dyn_mpc.fx_scale must be > 0");
  if (c->p.qp.max_iter < 1) return fail(c, VC_E_ARG, "qp.max_iter must be >= 1");
  if (c->dtype == VC_F64) return st_solve(c, B, x0, kappa, ds, xbar, ubar, u0, status, iters, diag, flags);
  vc::DynSqpArgs a{};
  a.B = B;
  a.car = vc::make_dyn_coef<float>(c->p.dyn_car);
  a.w = w;
  a.qp = c->p.qp;
  a.obs = c->p.obs;
  std::vector<Slot> slots;
  if (flags == VC_HOST_PTRS) {
    slots = {{x0, nullptr, (size_t)B * nx * 4, nullptr},
             {kappa, nullptr, (size_t)B * N * 4, nullptr},
             {ds, nullptr, (size_t)B * N * 4, nullptr},
             {ubar, ubar, (size_t)B * N * nu * 4, nullptr},
             {nullptr, xbar, (size_t)B * N * nx * 4, nullptr},
             {nullptr, u0, (size_t)B * nu * 4, nullptr},
             {nullptr, status, (size_t)B * 4, nullptr},
             {nullptr, iters, (size_t)B * 4, nullptr},
             {nullptr, diag, diag ? (size_t)B * VC_DYN_DIAG_COLS * 4 : 0, nullptr},
             {nullptr, dbg, dbg ? (size_t)B * vc::dyn_sqp_debug_stride() * 4 : 0, nullptr}};
    if (int r = stage(c, slots)) return r;
    a.dbg = dbg ? (float*)slots[9].dev : nullptr;
    a.x0 = (const float*)slots[0].dev;
    a.kappa = (const float*)slots[1].dev;
    a.ds = (const float*)slots[2].dev;
    a.ubar = (const float*)slots[3].dev;
    a.u_out = (float*)slots[3].dev;
    a.x_out = (float*)slots[4].dev;
    a.u0 = (float*)slots[5].dev;
    a.status = (int32_t*)slots[6].dev;
    a.iters = (int32_t*)slots[7].dev;
    a.diag = diag ? (float*)slots[8].dev : nullptr;
  } else {
    a.x0 = (const float*)x0;
    a.kappa = (const float*)kappa;
    a.ds = (const float*)ds;
    a.ubar = (const float*)ubar;
    a.u_out = (float*)ubar;
    a.x_out = (float*)xbar;
    a.u0 = (float*)u0;
    a.status = status;
    a.iters = iters;
    a.diag = (float*)diag;
    a.dbg = (float*)dbg;
  }
  VC_HIP(c, vc::launch_dyn_sqp(a, N, c->stream));
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}
}  // namespace

extern "C" {

int vc_abi_version(void) { return VCMPC_ABI_VERSION; }
int vc_params_sizeof(void) { return (int)sizeof(vc_params); }

// Shared by vc_create and vc_set_obstacles: NULL when the set is usable, else the reason.
static const char* obstacles_invalid(const vc_obstacles& o) {
  static thread_local char msg[96];
  if (o.n < 0 || o.n > VC_MAX_OBSTACLES) {
    snprintf(msg, sizeof msg, "n=%d obstacles outside [0,%d]", o.n, VC_MAX_OBSTACLES);
    return msg;
  }
  for (int j = 0; j < o.n; ++j)
    if (!std::isfinite(o.s[j]) || !std::isfinite(o.ey[j]) || !std::isfinite(o.radius[j])) {
      snprintf(msg, sizeof msg, "obstacle %d is not finite", j);
      return msg;
    }
  return nullptr;
}

vc_ctx* vc_create(int device, int model, int N, int max_batch, int dtype, const vc_params* params) {
  g_create_err.clear();
  if (!params) { fail(nullptr, VC_E_ARG, "params is NULL"); return nullptr; }
  if (model != VC_MODEL_KINEMATIC && model != VC_MODEL_DYNAMIC && model != VC_MODEL_CASCADED) {
    fail(nullptr, VC_E_ARG, "bad model %d", model);
    return nullptr;
  }
  if (model == VC_MODEL_CASCADED && (params->casc.horizon_pm < 1 || params->casc.horizon_pm > 4096)) {
    fail(nullptr, VC_E_ARG, "cascaded context needs casc.horizon_pm >= 1 (got %d)", params->casc.horizon_pm);
    return nullptr;
  }
  if (dtype != VC_F64 && dtype != VC_F32) { fail(nullptr, VC_E_ARG, "bad dtype %d", dtype); return nullptr; }
  if (N < 1 || N > 4096) { fail(nullptr, VC_E_ARG, "bad horizon N=%d", N); return nullptr; }
  if (max_batch < 1) { fail(nullptr, VC_E_ARG, "bad max_batch %d", max_batch); return nullptr; }
  // obs.inside (ABI 11) is a switch, and only the SQP models' QP and merit use it: the kinematic
  // merit keeps its C1 extension inside the margin floor, so an inside-mode kinematic QP would
  // disagree with its own line search
  if (params->obs.inside != 0 && params->obs.inside != 1) {
    fail(nullptr, VC_E_ARG, "obs.inside=%d must be 0 or 1", params->obs.inside);
    return nullptr;
  }
  if (model == VC_MODEL_KINEMATIC && params->obs.inside) {
    fail(nullptr, VC_E_ARG, "obs.inside=1 is not supported by the kinematic model (dynamic / cascaded only)");
    return nullptr;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    fail(nullptr, VC_E_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (device < 0 || device >= ndev) { fail(nullptr, VC_E_ARG, "device %d not in [0,%d)", device, ndev); return nullptr; }
  e = hipSetDevice(device);
  if (e != hipSuccess) { fail(nullptr, VC_E_HIP, "hipSetDevice: %s", hipGetErrorString(e)); return nullptr; }
  // the obstacle set is validated by the same rule as vc_set_obstacles, before any allocation
  if (const char* why = obstacles_invalid(params->obs)) {
    fail(nullptr, VC_E_ARG, "params->obs: %s", why);
    return nullptr;
  }
  vc_ctx* c = new vc_ctx();
  c->device = device;
  c->model = model;
  c->N = N;
  c->max_batch = max_batch;
  c->dtype = dtype;
  c->p = *params;
  if (!(c->p.obs.margin_min > 0)) c->p.obs.margin_min = VC_OBS_MARGIN_MIN;
  e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
  if (e != hipSuccess) {
    fail(nullptr, VC_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    delete c;
    return nullptr;
  }
  c->stream = c->own;
  return c;
}

void vc_destroy(vc_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->arena) (void)hipFree(c->arena);
  if (c->track) (void)hipFree(c->track);
  if (c->sim) (void)hipFree(c->sim);
  if (c->ls) (void)hipFree(c->ls);
  if (c->jw) (void)hipFree(c->jw);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

const char* vc_last_error(const vc_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

int vc_set_stream(vc_ctx* c, void* stream) {
  if (!c) return VC_E_ARG;
  c->stream = stream ? static_cast<hipStream_t>(stream) : c->own;
  return 0;
}

int vc_set_obstacles(vc_ctx* c, int n, const double* s, const double* ey, const double* radius, double margin_min) {
  if (!c) return VC_E_ARG;
  if (n < 0 || n > VC_MAX_OBSTACLES) return fail(c, VC_E_ARG, "n=%d obstacles outside [0,%d]", n, VC_MAX_OBSTACLES);
  if (n > 0 && (!s || !ey || !radius)) return fail(c, VC_E_ARG, "null pointer");
  vc_obstacles o{};
  o.n = n;
  o.inside = c->p.obs.inside;  // the barrier mode is the context's (vc_create's params)
  o.margin_min = margin_min > 0 ? margin_min : c->p.obs.margin_min;
  for (int j = 0; j < n; ++j) {
    o.s[j] = s[j];
    o.ey[j] = ey[j];
    o.radius[j] = radius[j];
  }
  if (const char* why = obstacles_invalid(o)) return fail(c, VC_E_ARG, "%s", why);
  c->p.obs = o;
  return 0;
}

int vc_synchronize(vc_ctx* c) {
  if (!c) return VC_E_ARG;
  VC_HIP(c, hipSetDevice(c->device));
  VC_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int kin_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar,
                     const void* ubar_in, void* u_out, void* u0, int32_t* status, int32_t* iters, void* diag,
                     int flags);

int vc_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar, void* u0,
             int32_t* status, int32_t* iters, int flags) {
  return vc_solve_diag(c, B, x0, kappa, ds, xbar, ubar, u0, status, iters, nullptr, flags);
}

int vc_solve_from(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, const void* ubar_in,
                  void* xbar, void* u_out, void* u0, int32_t* status, int32_t* iters, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!ubar_in || !u_out) return fail(c, VC_E_ARG, "null pointer");
  if (ubar_in == u_out) return vc_solve(c, B, x0, kappa, ds, xbar, u_out, u0, status, iters, flags);
  if (c->model == VC_MODEL_KINEMATIC && kin_solve_built(c)) {
    if (!x0 || !kappa || !ds || !xbar || !u0 || !status || !iters) return fail(c, VC_E_ARG, "null pointer");
    if (B == 0) return 0;
    return kin_solve(c, B, x0, kappa, ds, xbar, ubar_in, u_out, u0, status, iters, nullptr, flags);
  }
  // the SQP contexts iterate in place: u_out <- ubar_in, then vc_solve on u_out
  const int H = c->N + (c->model == VC_MODEL_CASCADED ? c->p.casc.horizon_pm : 0);
  const size_t bytes = (size_t)B * H * 2 * (c->dtype == VC_F32 ? 4 : 8);
  if (flags == VC_HOST_PTRS) std::memcpy(u_out, ubar_in, bytes);
  else VC_HIP(c, hipMemcpyAsync(u_out, ubar_in, bytes, hipMemcpyDeviceToDevice, c->stream));
  return vc_solve(c, B, x0, kappa, ds, xbar, u_out, u0, status, iters, flags);
}

int vc_solve_diag(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar,
                  void* u0, int32_t* status, int32_t* iters, void* diag, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!kin_solve_built(c) && !dyn_solve_built(c) && !casc_solve_built(c))
    return fail(c, VC_E_UNSUPPORTED,
                "vc_solve: model=%d dtype=%d N=%d not built (kinematic fp64 N=10..60 step 10, dynamic fp64 "
                "N=20..60 step 10, dynamic fp32 N=40, cascaded fp64 N=20 + 40 are)", c->model, c->dtype, c->N);
  if (!x0 || !kappa || !ds || !xbar || !ubar || !u0 || !status || !iters) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  if (c->model == VC_MODEL_DYNAMIC) return dyn_solve(c, B, x0, kappa, ds, xbar, ubar, u0, status, iters, diag, flags);
  if (c->model == VC_MODEL_CASCADED) return casc_solve(c, B, x0, kappa, ds, xbar, ubar, u0, status, iters, diag, flags);
  return kin_solve(c, B, x0, kappa, ds, xbar, ubar, ubar, u0, status, iters, diag, flags);
}

// The kinematic solve with the warm start read through ubar_in and u* written through u_out
// (vc_solve: both the caller's ubar; vc_solve_from: two buffers).
static int kin_solve(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar,
                     const void* ubar_in, void* u_out, void* u0, int32_t* status, int32_t* iters, void* diag,
                     int flags) {
  if (c->p.qp.elastic < 0.0 && c->p.qp.kin_sqp <= 0)
    return fail(c, VC_E_ARG, "vc_qp.elastic < 0 (elastic on failure) needs kin_sqp > 0; rho > 0 for one QP step");
  const int N = c->N, nx = 6, nu = 2;
  vc::KinLtvArgs a{};
  a.mode = 0;
  a.B = B;
  a.L = c->p.kin_car.l;
  a.w = c->p.kin_mpc;
  a.qp = c->p.qp;
  a.obs = c->p.obs;
  std::vector<Slot> slots;
  if (flags == VC_HOST_PTRS) {
    slots = {{x0, nullptr, (size_t)B * nx * 8, nullptr},
             {kappa, nullptr, (size_t)B * N * 8, nullptr},
             {ds, nullptr, (size_t)B * N * 8, nullptr},
             {ubar_in, u_out, (size_t)B * N * nu * 8, nullptr},
             {c->p.qp.ms ? xbar : nullptr, xbar, (size_t)B * (N + 1) * nx * 8, nullptr},
             {nullptr, u0, (size_t)B * nu * 8, nullptr},
             {nullptr, status, (size_t)B * 4, nullptr},
             {nullptr, iters, (size_t)B * 4, nullptr},
             {nullptr, diag, diag ? (size_t)B * VC_DIAG_COLS * 8 : 0, nullptr}};
    if (int r = stage(c, slots)) return r;
    a.x0 = (const double*)slots[0].dev;
    a.kappa = (const double*)slots[1].dev;
    a.ds = (const double*)slots[2].dev;
    a.ubar = (const double*)slots[3].dev;
    a.u_out = (double*)slots[3].dev;
    a.x_out = (double*)slots[4].dev;
    a.u0 = (double*)slots[5].dev;
    a.status = (int32_t*)slots[6].dev;
    a.iters = (int32_t*)slots[7].dev;
    a.diag = diag ? (double*)slots[8].dev : nullptr;
  } else {
    a.x0 = (const double*)x0;
    a.kappa = (const double*)kappa;
    a.ds = (const double*)ds;
    a.ubar = (const double*)ubar_in;
    a.u_out = (double*)u_out;
    a.x_out = (double*)xbar;
    a.u0 = (double*)u0;
    a.status = status;
    a.iters = iters;
    a.diag = (double*)diag;
  }
  a.x_in = a.x_out;  // multiple shooting (qp.ms): the warm-start states arrive in xbar
  const int S = c->p.qp.kin_sqp;
  if (S > 0 && (const void*)a.ubar != (const void*)a.u_out) {
    // the SQP iterates in place: start it on u_out
    VC_HIP(c, hipMemcpyAsync(a.u_out, a.ubar, (size_t)B * N * nu * 8, hipMemcpyDeviceToDevice, c->stream));
    a.ubar = a.u_out;
  }
  if (S <= 0) {  // the LTV-QP contract: one QP step
    if (kin_condensed(c)) VC_HIP(c, vc::launch_kin_ltv(a, N, c->stream));
    else VC_HIP(c, vc::launch_kin_ric(a, N, c->stream));
  } else {
    // globalised step (oracle/kin_sqp.py): S x { QP step at ubar; merit line search }
    const size_t o_up = 0, o_st = al256((size_t)B * N * nu * 8), o_it = o_st + al256((size_t)B * 4),
                 o_xp = o_it + al256((size_t)B * 4), total = o_xp + al256((size_t)B * (N + 1) * nx * 8);
    if (total > c->ls_bytes) {
      VC_HIP(c, hipStreamSynchronize(c->stream));
      if (c->ls) VC_HIP(c, hipFree(c->ls));
      c->ls = nullptr;
      c->ls_bytes = 0;
      VC_HIP(c, hipMalloc(&c->ls, total));
      c->ls_bytes = total;
    }
    char* base = static_cast<char*>(c->ls);
    vc::KinMeritArgs m{};
    m.x0 = a.x0;
    m.kappa = a.kappa;
    m.ds = a.ds;
    m.u_prev = (const double*)(base + o_up);
    m.ubar = a.u_out;
    m.x_out = a.x_out;
    m.u0 = a.u0;
    m.qp_status = a.status;
    m.qp_iters = a.iters;
    m.status = a.status;
    m.iters = a.iters;
    m.st_acc = (int32_t*)(base + o_st);
    m.it_acc = (int32_t*)(base + o_it);
    m.ls_diag = nullptr;
    m.ms = c->p.qp.ms;
    m.restart = S > 1;
    m.x_prev = (const double*)(base + o_xp);
    m.B = B;
    m.N = N;
    m.L = a.L;
    m.w = a.w;
    m.obs = a.obs;
    // qp.elastic < 0: hard rows first, elastic rows only where those fail (stagewise kernel only)
    const bool elastic_retry = c->p.qp.elastic < 0.0 && !kin_condensed(c);
    if (c->p.qp.elastic < 0.0) a.qp.elastic = 0.0;
    for (int i = 0; i < S; ++i) {
      VC_HIP(c, hipMemcpyAsync(base + o_up, a.u_out, (size_t)B * N * nu * 8, hipMemcpyDeviceToDevice, c->stream));
      if (m.ms)
        VC_HIP(c, hipMemcpyAsync(base + o_xp, a.x_out, (size_t)B * (N + 1) * nx * 8, hipMemcpyDeviceToDevice,
                                 c->stream));
      if (kin_condensed(c)) VC_HIP(c, vc::launch_kin_ltv(a, N, c->stream));
      else VC_HIP(c, vc::launch_kin_ric(a, N, c->stream));
      if (elastic_retry) {
        // elastic on failure: the QPs the hard-row pass left non-solved, again from the same
        // iterate (the pre-step copies: the first pass has overwritten ubar / xbar in place)
        vc::KinLtvArgs e = a;
        e.qp.elastic = c->p.qp.elastic;
        e.ubar = (const double*)(base + o_up);
        if (m.ms) e.x_in = (const double*)(base + o_xp);
        VC_HIP(c, vc::launch_kin_ric(e, N, c->stream));
      }
      if (i == c->fault_iter && c->fault_problem >= 0 && c->fault_problem < B)
        VC_HIP(c, vc::launch_kin_qp_fault(a, N, c->fault_problem, c->stream));
      m.first = i == 0;
      VC_HIP(c, vc::launch_kin_merit(m, c->stream));
    }
  }
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}

int vc_solve_debug(vc_ctx* c, int B, const void* x0, const void* kappa, const void* ds, void* xbar, void* ubar,
                   void* u0, int32_t* status, int32_t* iters, void* dbg, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!dyn_solve_built(c)) return fail(c, VC_E_UNSUPPORTED, "vc_solve_debug: dynamic fp32 N=40 contexts only");
  if (!x0 || !kappa || !ds || !xbar || !ubar || !u0 || !status || !iters || !dbg)
    return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  return dyn_solve(c, B, x0, kappa, ds, xbar, ubar, u0, status, iters, nullptr, flags, dbg);
}

int vc_debug_stride(void) { return vc::dyn_sqp_debug_stride(); }

int vc_debug_rcp(vc_ctx* c, int n, const void* x, void* out, int flags) {
  if (!c) return VC_E_ARG;
  if (n < 0 || n > c->max_batch) return fail(c, VC_E_ARG, "n %d outside [0, max_batch=%d]", n, c->max_batch);
  if (int r = check_common(c, 0, flags)) return r;
  if (!x || !out) return fail(c, VC_E_ARG, "null pointer");
  if (n == 0) return 0;
  if (flags == VC_DEVICE_PTRS) {
    VC_HIP(c, vc::launch_rcp_probe(n, (const double*)x, (double*)out, c->stream));
    return 0;
  }
  std::vector<Slot> slots = {{x, nullptr, (size_t)n * 8, nullptr}, {nullptr, out, (size_t)n * 32, nullptr}};
  if (int r = stage(c, slots)) return r;
  VC_HIP(c, vc::launch_rcp_probe(n, (const double*)slots[0].dev, (double*)slots[1].dev, c->stream));
  return unstage(c, slots);
}

int vc_debug_qp_fault(vc_ctx* c, int sqp_iter, int problem) {
  if (!c) return VC_E_ARG;
  c->fault_iter = sqp_iter;
  c->fault_problem = problem;
  return 0;
}

int vc_condense(vc_ctx* c, int B, const void* x0, const void* ubar, const void* kappa, const void* ds, void* H,
                void* g, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  const bool casc_cond = c->model == VC_MODEL_CASCADED && c->dtype == VC_F64 &&
                         vc::casc_sqp_built(c->N, c->p.casc.horizon_pm);
  if (!(kin_solve_built(c) && kin_condensed(c)) && !casc_cond)
    return fail(c, VC_E_UNSUPPORTED, "vc_condense: model=%d dtype=%d N=%d not built", c->model, c->dtype, c->N);
  if (!x0 || !kappa || !ds || !ubar || !H || !g) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  if (c->model == VC_MODEL_CASCADED)
    return casc_solve(c, B, x0, kappa, ds, nullptr, const_cast<void*>(ubar), nullptr, nullptr, nullptr, nullptr, flags,
                      1, H, g);
  const int N = c->N, n = 2 * N;
  vc::KinLtvArgs a{};
  a.mode = 1;
  a.B = B;
  a.L = c->p.kin_car.l;
  a.w = c->p.kin_mpc;
  a.qp = c->p.qp;
  a.obs = c->p.obs;
  std::vector<Slot> slots;
  if (flags == VC_HOST_PTRS) {
    slots = {{x0, nullptr, (size_t)B * 6 * 8, nullptr},
             {kappa, nullptr, (size_t)B * N * 8, nullptr},
             {ds, nullptr, (size_t)B * N * 8, nullptr},
             {ubar, nullptr, (size_t)B * n * 8, nullptr},
             {nullptr, H, (size_t)B * n * n * 8, nullptr},
             {nullptr, g, (size_t)B * n * 8, nullptr}};
    if (int r = stage(c, slots)) return r;
    a.x0 = (const double*)slots[0].dev;
    a.kappa = (const double*)slots[1].dev;
    a.ds = (const double*)slots[2].dev;
    a.ubar = (const double*)slots[3].dev;
    a.H_out = (double*)slots[4].dev;
    a.g_out = (double*)slots[5].dev;
  } else {
    a.x0 = (const double*)x0;
    a.kappa = (const double*)kappa;
    a.ds = (const double*)ds;
    a.ubar = (const double*)ubar;
    a.H_out = (double*)H;
    a.g_out = (double*)g;
  }
  VC_HIP(c, vc::launch_kin_ltv(a, N, c->stream));
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}

int vc_rollout(vc_ctx* c, int B, const void* x0, const void* ubar, const void* kappa, const void* ds, void* xbar,
               int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x0 || !ubar || !kappa || !ds || !xbar) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  const int N = c->N, nx = nx_of(c);
  const size_t es = esize(c);
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x0, nullptr, (size_t)B * nx * es, nullptr},
                               {ubar, nullptr, (size_t)B * N * 2 * es, nullptr},
                               {kappa, nullptr, (size_t)B * N * es, nullptr},
                               {ds, nullptr, (size_t)B * N * es, nullptr},
                               {nullptr, xbar, (size_t)B * (N + 1) * nx * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_rollout(m, c->dtype, slots[0].dev, slots[1].dev, slots[2].dev, slots[3].dev, slots[4].dev,
                                 c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_rollout(m, c->dtype, x0, ubar, kappa, ds, xbar, c->stream));
  return 0;
}

int vc_linearize(vc_ctx* c, int B, const void* xbar, const void* ubar, const void* kappa, const void* ds, void* A,
                 void* Bm, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (c->model != VC_MODEL_KINEMATIC || c->dtype != VC_F64)
    return fail(c, VC_E_UNSUPPORTED, "vc_linearize: only the kinematic fp64 model is built");
  if (!xbar || !ubar || !kappa || !ds || !A || !Bm) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  const int N = c->N;
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{xbar, nullptr, (size_t)B * (N + 1) * 6 * 8, nullptr},
                               {ubar, nullptr, (size_t)B * N * 2 * 8, nullptr},
                               {kappa, nullptr, (size_t)B * N * 8, nullptr},
                               {ds, nullptr, (size_t)B * N * 8, nullptr},
                               {nullptr, A, (size_t)B * N * 36 * 8, nullptr},
                               {nullptr, Bm, (size_t)B * N * 12 * 8, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_kin_linearize(m, slots[0].dev, slots[1].dev, slots[2].dev, slots[3].dev, slots[4].dev,
                                       slots[5].dev, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_kin_linearize(m, xbar, ubar, kappa, ds, A, Bm, c->stream));
  return 0;
}

int vc_plant_step(vc_ctx* c, int B, const void* x, const void* u, const void* kappa, double dt, void* x_next,
                  int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x || !u || !kappa || !x_next) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  const int nx = nx_of(c);
  const size_t es = esize(c);
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x, nullptr, (size_t)B * nx * es, nullptr},
                               {u, nullptr, (size_t)B * 2 * es, nullptr},
                               {kappa, nullptr, (size_t)B * es, nullptr},
                               {nullptr, x_next, (size_t)B * nx * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_plant_step(m, c->dtype, slots[0].dev, slots[1].dev, slots[2].dev, dt, slots[3].dev,
                                    c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_plant_step(m, c->dtype, x, u, kappa, dt, x_next, c->stream));
  return 0;
}

int vc_ode(vc_ctx* c, int B, const void* x, const void* u, const void* kappa, int space, void* f, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x || !u || !kappa || !f) return fail(c, VC_E_ARG, "null pointer");
  if (space != 0 && space != 1) return fail(c, VC_E_ARG, "vc_ode: space must be 0 (temporal) or 1 (spatial)");
  if (B == 0) return 0;
  const int nx = nx_of(c);
  const size_t es = esize(c);
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x, nullptr, (size_t)B * nx * es, nullptr},
                               {u, nullptr, (size_t)B * 2 * es, nullptr},
                               {kappa, nullptr, (size_t)B * es, nullptr},
                               {nullptr, f, (size_t)B * nx * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_ode(m, c->dtype, slots[0].dev, slots[1].dev, slots[2].dev, space, slots[3].dev, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_ode(m, c->dtype, x, u, kappa, space, f, c->stream));
  return 0;
}

int vc_spatial_step(vc_ctx* c, int B, const void* x, const void* u, const void* kappa, const void* ds, void* x_next,
                    int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x || !u || !kappa || !ds || !x_next) return fail(c, VC_E_ARG, "null pointer");
  if (B == 0) return 0;
  const int nx = nx_of(c);
  const size_t es = esize(c);
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x, nullptr, (size_t)B * nx * es, nullptr},
                               {u, nullptr, (size_t)B * 2 * es, nullptr},
                               {kappa, nullptr, (size_t)B * es, nullptr},
                               {ds, nullptr, (size_t)B * es, nullptr},
                               {nullptr, x_next, (size_t)B * nx * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_spatial_step(m, c->dtype, slots[0].dev, slots[1].dev, slots[2].dev, slots[3].dev,
                                      slots[4].dev, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_spatial_step(m, c->dtype, x, u, kappa, ds, x_next, c->stream));
  return 0;
}

int vc_track_set(vc_ctx* c, int n_pieces, double h, double length, const double* coef) {
  if (!c) return VC_E_ARG;
  if (n_pieces < 1 || !(h > 0) || !(length > 0) || !coef)
    return fail(c, VC_E_ARG, "vc_track_set: need n_pieces >= 1, h > 0, length > 0, coef");
  for (int i = 0; i < 4 * n_pieces; ++i)
    if (!std::isfinite(coef[i])) return fail(c, VC_E_ARG, "vc_track_set: coef[%d] not finite", i);
  VC_HIP(c, hipSetDevice(c->device));
  VC_HIP(c, hipStreamSynchronize(c->stream));  // no kernel may still read the old table
  if (c->track) VC_HIP(c, hipFree(c->track));
  c->track = nullptr;
  c->track_n = 0;
  VC_HIP(c, hipMalloc(&c->track, (size_t)n_pieces * 4 * sizeof(double)));
  VC_HIP(c, hipMemcpy(c->track, coef, (size_t)n_pieces * 4 * sizeof(double), hipMemcpyHostToDevice));
  c->track_n = n_pieces;
  c->track_h = h;
  c->track_len = length;
  return 0;
}

int vc_track_k(vc_ctx* c, int B, const void* s, void* k, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!s || !k) return fail(c, VC_E_ARG, "null pointer");
  if (!c->track) return fail(c, VC_E_ARG, "vc_track_k: no track table (vc_track_set)");
  if (B == 0) return 0;
  const size_t es = esize(c);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{s, nullptr, B * es, nullptr}, {nullptr, k, B * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_track_k(track_table(c), c->dtype, B, slots[0].dev, slots[1].dev, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_track_k(track_table(c), c->dtype, B, s, k, c->stream));
  return 0;
}

int vc_horizon(vc_ctx* c, int B, const void* x0, const void* xbar, double mpc_dt, void* kappa, void* ds,
               int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x0 || !xbar || !kappa || !ds) return fail(c, VC_E_ARG, "null pointer");
  if (!c->track) return fail(c, VC_E_ARG, "vc_horizon: no track table (vc_track_set)");
  if (B == 0) return 0;
  const int N = c->N, nx = nx_of(c), NS = ns_of(c), NH = nh_of(c), M = NH - N;
  const double ds_pm = c->p.casc.ds_pm;
  const size_t es = esize(c);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x0, nullptr, (size_t)B * nx * es, nullptr},
                               {xbar, nullptr, (size_t)B * NS * nx * es, nullptr},
                               {nullptr, kappa, (size_t)B * NH * es, nullptr},
                               {nullptr, ds, (size_t)B * NH * es, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_horizon(track_table(c), c->model, c->dtype, B, N, M, ds_pm, slots[0].dev, c->dtype == VC_F64,
                                 slots[1].dev, mpc_dt, slots[2].dev, slots[3].dev, nullptr, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_horizon(track_table(c), c->model, c->dtype, B, N, M, ds_pm, x0, c->dtype == VC_F64, xbar,
                               mpc_dt, kappa, ds, nullptr, c->stream));
  return 0;
}

int vc_drive(vc_ctx* c, int B, double* x64, const void* u0, double dt, void* x_ctx, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x64 || !u0) return fail(c, VC_E_ARG, "null pointer");
  if (!c->track) return fail(c, VC_E_ARG, "vc_drive: no track table (vc_track_set)");
  if (B == 0) return 0;
  const int nx = nx_of(c);
  const size_t es = esize(c);
  vc::ModelArgs m = model_args(c, B);
  if (flags == VC_HOST_PTRS) {
    std::vector<Slot> slots = {{x64, x64, (size_t)B * nx * 8, nullptr},
                               {u0, nullptr, (size_t)B * 2 * es, nullptr},
                               {nullptr, x_ctx, x_ctx ? (size_t)B * nx * es : 0, nullptr}};
    if (int r = stage(c, slots)) return r;
    VC_HIP(c, vc::launch_drive(m, c->dtype, track_table(c), (double*)slots[0].dev, slots[1].dev, dt,
                               x_ctx ? slots[2].dev : nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr, c->stream));
    return unstage(c, slots);
  }
  VC_HIP(c, vc::launch_drive(m, c->dtype, track_table(c), x64, u0, dt, x_ctx, nullptr, nullptr, nullptr, nullptr,
                             nullptr, nullptr, nullptr, c->stream));
  return 0;
}

int vc_simulate(vc_ctx* c, int B, int steps, double mpc_dt, double dt, double* x64, void* xbar, void* ubar,
                double* log_x, void* log_u, int32_t* nfail, int flags) {
  if (int r = check_common(c, B, flags)) return r;
  if (!x64 || !xbar || !ubar) return fail(c, VC_E_ARG, "null pointer");
  if (steps < 0) return fail(c, VC_E_ARG, "steps %d < 0", steps);
  if (!c->track) return fail(c, VC_E_ARG, "vc_simulate: no track table (vc_track_set)");
  if (!kin_solve_built(c) && !dyn_solve_built(c) && !casc_solve_built(c))
    return fail(c, VC_E_UNSUPPORTED, "vc_simulate: model=%d dtype=%d N=%d has no built vc_solve", c->model, c->dtype,
                c->N);
  if (B == 0 || steps == 0) return 0;
  const int N = c->N, nx = nx_of(c), NS = ns_of(c), NH = nh_of(c), M = NH - N;
  const double ds_pm = c->p.casc.ds_pm;
  const size_t es = esize(c);
  std::vector<Slot> slots;
  double* dx = x64;
  void *dxbar = xbar, *dubar = ubar, *dlu = log_u;
  double* dlx = log_x;
  int32_t* dnf = nfail;
  if (flags == VC_HOST_PTRS) {
    slots = {{x64, x64, (size_t)B * nx * 8, nullptr},
             {xbar, xbar, (size_t)B * NS * nx * es, nullptr},
             {ubar, ubar, (size_t)B * NH * 2 * es, nullptr},
             {nullptr, log_x, log_x ? (size_t)(steps + 1) * B * nx * 8 : 0, nullptr},
             {nullptr, log_u, log_u ? (size_t)steps * B * 2 * es : 0, nullptr},
             {nfail, nfail, nfail ? (size_t)B * 4 : 0, nullptr}};
    if (int r = stage(c, slots)) return r;
    dx = (double*)slots[0].dev;
    dxbar = slots[1].dev;
    dubar = slots[2].dev;
    dlx = log_x ? (double*)slots[3].dev : nullptr;
    dlu = log_u ? slots[4].dev : nullptr;
    dnf = nfail ? (int32_t*)slots[5].dev : nullptr;
  }
  // scratch: kappa[B][NH], ds[B][NH], x[B][nx], u0[B][2] (context dtype), status[B], iters[B]
  const size_t o_kap = 0, o_ds = o_kap + al256((size_t)B * NH * es), o_x = o_ds + al256((size_t)B * NH * es),
               o_u0 = o_x + al256((size_t)B * nx * es), o_st = o_u0 + al256((size_t)B * 2 * es),
               o_it = o_st + al256((size_t)B * 4), total = o_it + al256((size_t)B * 4);
  if (total > c->sim_bytes) {
    VC_HIP(c, hipStreamSynchronize(c->stream));
    if (c->sim) VC_HIP(c, hipFree(c->sim));
    c->sim = nullptr;
    c->sim_bytes = 0;
    VC_HIP(c, hipMalloc(&c->sim, total));
    c->sim_bytes = total;
  }
  char* base = static_cast<char*>(c->sim);
  void *kap = base + o_kap, *dsv = base + o_ds, *xc = base + o_x, *u0 = base + o_u0;
  int32_t *st = (int32_t*)(base + o_st), *it = (int32_t*)(base + o_it);
  const vc::TrackTable tt = track_table(c);
  vc::ModelArgs m = model_args(c, B);
  if (dlx) VC_HIP(c, hipMemcpyAsync(dlx, dx, (size_t)B * nx * 8, hipMemcpyDeviceToDevice, c->stream));
  for (int step = 0; step < steps; ++step) {
    VC_HIP(c, vc::launch_horizon(tt, c->model, c->dtype, B, N, M, ds_pm, dx, true, dxbar, mpc_dt, kap, dsv, xc,
                                 c->stream));
    if (int r = vc_solve_diag(c, B, xc, kap, dsv, dxbar, dubar, u0, st, it, nullptr, VC_DEVICE_PTRS)) return r;
    VC_HIP(c, vc::launch_drive(m, c->dtype, tt, dx, u0, dt, nullptr, st, dxbar, dubar, dnf,
                               dlx ? dlx + (size_t)(step + 1) * B * nx : nullptr,
                               dlu ? (char*)dlu + (size_t)step * B * 2 * es : nullptr, kap, c->stream));
  }
  if (flags == VC_HOST_PTRS) return unstage(c, slots);
  return 0;
}

}  // extern "C"
