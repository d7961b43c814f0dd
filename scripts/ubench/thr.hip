// Throughput micro-benchmarks on gfx950 (one wave; s_memtime ticks per instruction), with
// inline asm so the compiler cannot fold the loops: v_fma_f64 (8 independent chains),
// v_readlane_b32, ds_read_b64 / ds_read_b128 broadcast (all lanes one address) and
// lane-strided, v_cndmask_b32, v_mfma_f64_16x16x4_f64 (4 independent accumulators).
// build: hipcc -O3 --offload-arch=gfx950 thr.hip -o thr ; run: ./thr [waves_per_block]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define T0() (__builtin_amdgcn_sched_barrier(0), __builtin_amdgcn_s_memtime())
__global__ void k_thr(double* out, double seed) {
  __shared__ double buf[2048];
  const int l = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) buf[i] = seed + i;
  __syncthreads();
  double c0 = seed, c1 = seed + 1, c2 = seed + 2, c3 = seed + 3, c4 = seed + 4, c5 = seed + 5, c6 = seed + 6, c7 = seed + 7;
  const double a = 0.999, b = 1e-9;
  uint64_t t0, t1;
  const int REP = 64;
  // fma
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "v_fma_f64 %0, %8, %9, %0\n v_fma_f64 %1, %8, %9, %1\n v_fma_f64 %2, %8, %9, %2\n v_fma_f64 %3, %8, %9, %3\n"
        "v_fma_f64 %4, %8, %9, %4\n v_fma_f64 %5, %8, %9, %5\n v_fma_f64 %6, %8, %9, %6\n v_fma_f64 %7, %8, %9, %7\n"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[0] = double(t1 - t0) / (REP * 8);
  // readlane
  int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int vv = l;
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "v_readlane_b32 %0, %4, 1\n v_readlane_b32 %1, %4, 2\n v_readlane_b32 %2, %4, 3\n v_readlane_b32 %3, %4, 4\n"
        "v_readlane_b32 %0, %4, 5\n v_readlane_b32 %1, %4, 6\n v_readlane_b32 %2, %4, 7\n v_readlane_b32 %3, %4, 8\n"
        : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3)
        : "v"(vv));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[1] = double(t1 - t0) / (REP * 8);
  // ds_read_b64 broadcast
  double r0, r1, r2, r3;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) double*)buf;
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "ds_read_b64 %0, %4 offset:0\n ds_read_b64 %1, %4 offset:64\n ds_read_b64 %2, %4 offset:128\n ds_read_b64 %3, %4 offset:192\n"
        "ds_read_b64 %0, %4 offset:256\n ds_read_b64 %1, %4 offset:320\n ds_read_b64 %2, %4 offset:384\n ds_read_b64 %3, %4 offset:448\n"
        "s_waitcnt lgkmcnt(0)\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(base));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[2] = double(t1 - t0) / (REP * 8);
  // ds_read_b128 broadcast
  typedef double d2 __attribute__((ext_vector_type(2)));
  d2 q0, q1, q2, q3;
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "ds_read_b128 %0, %4 offset:0\n ds_read_b128 %1, %4 offset:64\n ds_read_b128 %2, %4 offset:128\n ds_read_b128 %3, %4 offset:192\n"
        "ds_read_b128 %0, %4 offset:256\n ds_read_b128 %1, %4 offset:320\n ds_read_b128 %2, %4 offset:384\n ds_read_b128 %3, %4 offset:448\n"
        "s_waitcnt lgkmcnt(0)\n"
        : "=v"(q0), "=v"(q1), "=v"(q2), "=v"(q3)
        : "v"(base));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[3] = double(t1 - t0) / (REP * 8);
  // ds_read_b64 lane-strided (stride 41 doubles: the kernels' odd row pitch)
  const unsigned sb = base + (unsigned)(l * 41 * 8 % 8192);
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "ds_read_b64 %0, %4 offset:0\n ds_read_b64 %1, %4 offset:8\n ds_read_b64 %2, %4 offset:16\n ds_read_b64 %3, %4 offset:24\n"
        "ds_read_b64 %0, %4 offset:32\n ds_read_b64 %1, %4 offset:40\n ds_read_b64 %2, %4 offset:48\n ds_read_b64 %3, %4 offset:56\n"
        "s_waitcnt lgkmcnt(0)\n"
        : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
        : "v"(sb));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[4] = double(t1 - t0) / (REP * 8);
  // v_cndmask_b32
  int m0 = l, m1 = l + 1, m2 = l + 2, m3 = l + 3;
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %0, vcc\n"
        "v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %0, vcc\n"
        : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[5] = double(t1 - t0) / (REP * 8);
  // mfma f64 16x16x4, 4 independent accumulators
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  double ma = seed + l, mb = seed - l;
  t0 = T0();
  for (int r = 0; r < REP / 4; ++r) {
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc3, 0, 0, 0);
  }
  asm volatile("" ::"v"(acc0), "v"(acc1), "v"(acc2), "v"(acc3));
  t1 = T0();
  if (threadIdx.x == 0) out[6] = double(t1 - t0) / REP;
  // v_mul_f64 + v_add_f64 (non-fma) throughput check
  t0 = T0();
  for (int r = 0; r < REP; ++r) {
    asm volatile(
        "v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n v_mul_f64 %3, %3, %8\n"
        "v_add_f64 %4, %4, %9\n v_add_f64 %5, %5, %9\n v_add_f64 %6, %6, %9\n v_add_f64 %7, %7, %9\n"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b));
  }
  t1 = T0();
  if (threadIdx.x == 0) out[7] = double(t1 - t0) / (REP * 8);
  out[64 + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + s0 + s1 + s2 + s3 + r0 + r1 + r2 + r3 + q0.x + q1.y +
                          q2.x + q3.y + m0 + m1 + m2 + m3;
}

int main(int argc, char** argv) {
  const int wpb = argc > 1 ? atoi(argv[1]) : 1;
  double* d;
  hipMalloc(&d, 4096 * sizeof(double));
  double h[8];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_thr, dim3(1), dim3(64 * wpb), 0, 0, d, 1.0);
    hipMemcpy(h, d, 8 * sizeof(double), hipMemcpyDeviceToHost);
  }
  const char* nm[8] = {"v_fma_f64", "v_readlane_b32", "ds_read_b64 broadcast", "ds_read_b128 broadcast",
                       "ds_read_b64 stride-41 rows", "v_cndmask_b32", "v_mfma_f64_16x16x4 (4 acc)", "v_mul/add_f64"};
  printf("waves per block: %d\n", wpb);
  for (int i = 0; i < 8; ++i) printf("%-32s %7.2f ticks / instruction\n", nm[i], h[i]);
  // tick rate: a long fma loop timed by events
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(k_thr, dim3(1), dim3(64 * wpb), 0, 0, d, 1.0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("200 launches: %.3f ms\n", ms);
  return 0;
}
