// Host-side AddressSanitizer check of the C-ABI shim (optional ASan build): links
// build/libvcmpc_asan.so -- vcmpc_abi.hip's host code built with -fsanitize=address (device code is
// not sanitised: GPU ASan is not available on this pool) -- and drives the entry points' argument
// validation and error paths.  Without a GPU vc_create fails loudly; with one the driver also runs
// a context through its bad-argument returns, a track upload and destroy.  `make asan` builds both.
#include <cstdio>
#include <cstring>

#include "vcmpc.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

int main() {
  CHECK(vc_abi_version() == 13);
  CHECK(vc_params_sizeof() == (int)sizeof(vc_params));
  vc_params p;
  std::memset(&p, 0, sizeof(p));
  // bad arguments never reach the device
  CHECK(vc_create(0, 99, 20, 64, VC_F64, &p) == nullptr);
  CHECK(vc_last_error(nullptr) && std::strlen(vc_last_error(nullptr)) > 0);
  CHECK(vc_create(0, VC_MODEL_KINEMATIC, 0, 64, VC_F64, &p) == nullptr);
  CHECK(vc_create(0, VC_MODEL_KINEMATIC, 20, 0, VC_F64, &p) == nullptr);
  CHECK(vc_create(0, VC_MODEL_KINEMATIC, 20, 64, VC_F64, nullptr) == nullptr);
  p.obs.inside = 1;   // the inside-mode barrier is an SQP-model feature (ABI 12)
  CHECK(vc_create(0, VC_MODEL_KINEMATIC, 20, 64, VC_F64, &p) == nullptr);
  p.obs.inside = 2;   // a switch: 0 or 1
  CHECK(vc_create(0, VC_MODEL_DYNAMIC, 40, 64, VC_F64, &p) == nullptr);
  p.obs.inside = 0;
  vc_destroy(nullptr);
  vc_ctx* c = vc_create(0, VC_MODEL_KINEMATIC, 20, 64, VC_F64, &p);
  if (!c) {
    std::printf("no device: %s\n", vc_last_error(nullptr));
  } else {
    double x[64 * 6] = {0}, k[64 * 20] = {0}, ds[64 * 20] = {0}, u[64 * 20 * 2] = {0}, xb[64 * 21 * 6] = {0};
    double u0[64 * 2] = {0};
    int st[64] = {0}, it[64] = {0};
    CHECK(vc_solve(c, 65, x, k, ds, xb, u, u0, st, it, VC_HOST_PTRS) != 0);  // B > max_batch
    CHECK(vc_solve(c, -1, x, k, ds, xb, u, u0, st, it, VC_HOST_PTRS) != 0);
    double uo[64 * 20 * 2] = {0};
    CHECK(vc_solve_from(c, 65, x, k, ds, u, xb, uo, u0, st, it, VC_HOST_PTRS) != 0);  // ABI 13
    CHECK(vc_solve_from(c, 4, x, k, ds, nullptr, xb, uo, u0, st, it, VC_HOST_PTRS) != 0);
    CHECK(vc_solve_from(c, 4, x, k, ds, u, xb, nullptr, u0, st, it, VC_HOST_PTRS) != 0);
    CHECK(std::strlen(vc_last_error(c)) > 0);
    CHECK(vc_set_obstacles(c, -1, nullptr, nullptr, nullptr, 0.0) != 0);
    const double coef[4 * 4] = {0.0, 0.0, 0.0, 0.01, 0.0, 0.0, 0.0, 0.01, 0.0, 0.0, 0.0, 0.01, 0.0, 0.0, 0.0, 0.01};
    CHECK(vc_track_set(c, 4, 1.0, 4.0, coef) == 0);
    CHECK(vc_track_set(c, 0, 1.0, 4.0, coef) != 0);
    vc_destroy(c);
  }
  std::printf(fails ? "asan driver FAILED\n" : "asan driver ok\n");
  return fails ? 1 : 0;
}
