// numerics.hip -- device probe of the reciprocal forms the solve kernels use (test diagnostics,
// vc_debug_rcp; tests/test_gpu_numerics.py).
//
//   out[i][0] = 1.0 / x          IEEE fp64 divide (div_scale / div_fmas / div_fixup)
//   out[i][1] = rcp_nr(x)        vc_kernels.hpp: v_rcp_f64 + two fma Newton steps, falling back
//                                to the raw estimate when the refinement is not finite
//                                (kin_ltv.hip's inverse slacks / multipliers)
//   out[i][2] = r2(x)            v_rcp_f64 + two Newton steps r (2 - x r), no fallback (the 2x2
//                                input-block inverse of st_sqp / kin_ric / casc_ric, det > 0)
//   out[i][3] = v_rcp_f64(x)     the raw hardware estimate
#include <hip/hip_runtime.h>

#include "vc_kernels.hpp"

namespace vc {
namespace {

__global__ void rcp_probe_kernel(int n, const double* x, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double id = __builtin_amdgcn_rcp(v);
  id = id * (2.0 - v * id);
  id = id * (2.0 - v * id);
  out[4 * (size_t)i + 0] = 1.0 / v;
  out[4 * (size_t)i + 1] = rcp_nr(v);
  out[4 * (size_t)i + 2] = id;
  out[4 * (size_t)i + 3] = __builtin_amdgcn_rcp(v);
}

}  // namespace

hipError_t launch_rcp_probe(int n, const double* x, double* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rcp_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, st, n, x, out);
  return hipGetLastError();
}

}  // namespace vc
