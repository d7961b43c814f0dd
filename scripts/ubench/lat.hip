// Latency micro-benchmarks on gfx950, one wave: s_memtime cycles per dependent step of
//  (a) fp64 FMA chain, (b) v_rcp/rsq + 2 Newton chain, (c) LDS write -> read round trip by another
//  lane (single wave, in-order LDS), (d) same with s_barrier, (e) v_readlane of a just-written VGPR
//  feeding the next FMA, (f) DPP row_shr:1 chain, (g) ds_bpermute chain.
// build: hipcc -O3 --offload-arch=gfx950 lat.hip -o lat ; run: ./lat
#include <hip/hip_runtime.h>
#include <cstdio>

#define STEPS 256
__device__ __forceinline__ double rl(double v, int l) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), l), hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

__global__ void k_lat(double* out, double seed, int src) {
  __shared__ double buf[256];
  const int l = threadIdx.x;
  double x = seed + l * 1e-3, y = 0.0;
  uint64_t t0, t1;
  // (a) fma chain
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 64
  for (int i = 0; i < STEPS; ++i) x = fma(x, 0.999999, 1e-9);
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[0] = double(t1 - t0) / STEPS;
  y += x;
  // (b) rsq + 2 Newton chain
  x = 1.5 + l * 1e-3;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < STEPS / 4; ++i) {
    double r = __builtin_amdgcn_rsq(x);
    r = r * (1.5 - 0.5 * x * r * r);
    r = r * (1.5 - 0.5 * x * r * r);
    x = 1.0 + r * 1e-3;
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[1] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (c) LDS round trip: lane l writes, all lanes read lane (src) -- dependent chain
  x = seed + l;
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 8
  for (int i = 0; i < STEPS / 4; ++i) {
    buf[l] = x;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    x = buf[(src + i) & 63] + 1e-9;
    asm volatile("" ::: "memory");
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[2] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (d) the same with __syncthreads (s_waitcnt + s_barrier)
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 8
  for (int i = 0; i < STEPS / 4; ++i) {
    buf[l] = x;
    __syncthreads();
    x = buf[(src + i) & 63] + 1e-9;
    __syncthreads();
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[3] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (e) readlane chain: x_{i+1} = fma(readlane(x_i, src), c, lane term)
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < STEPS / 4; ++i) x = fma(rl(x, src), 0.999999, l * 1e-12);
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[4] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (f) DPP row_shr:1 chain (update_dpp on both halves)
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < STEPS / 4; ++i) {
    int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x111, 0xf, 0xf, false);
    int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x111, 0xf, 0xf, false);
    x = fma(__hiloint2double(hi, lo), 0.999999, 1e-9);
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[5] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (g) ds_bpermute chain (lane (l+src)&63)
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 16
  for (int i = 0; i < STEPS / 4; ++i) {
    const int a = ((l + src) & 63) << 2;
    int lo = __builtin_amdgcn_ds_bpermute(a, __double2loint(x));
    int hi = __builtin_amdgcn_ds_bpermute(a, __double2hiint(x));
    x = fma(__hiloint2double(hi, lo), 0.999999, 1e-9);
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[6] = double(t1 - t0) / (STEPS / 4);
  y += x;
  // (h) throughput: 256 independent fp64 FMAs (8 chains)
  double c0 = x, c1 = x + 1, c2 = x + 2, c3 = x + 3, c4 = x + 4, c5 = x + 5, c6 = x + 6, c7 = x + 7;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 32
  for (int i = 0; i < STEPS / 8; ++i) {
    c0 = fma(c0, 0.9999, 1e-9); c1 = fma(c1, 0.9999, 1e-9); c2 = fma(c2, 0.9999, 1e-9); c3 = fma(c3, 0.9999, 1e-9);
    c4 = fma(c4, 0.9999, 1e-9); c5 = fma(c5, 0.9999, 1e-9); c6 = fma(c6, 0.9999, 1e-9); c7 = fma(c7, 0.9999, 1e-9);
  }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[7] = double(t1 - t0) / STEPS;
  y += c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  // (i) throughput: 256 independent LDS broadcast reads
  __syncthreads();
  double acc = 0.0;
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
#pragma unroll 64
  for (int i = 0; i < STEPS; ++i) acc += buf[(i * 7) & 255];
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[8] = double(t1 - t0) / STEPS;
  // (j) throughput: readlanes (pairs) into FMAs
  __builtin_amdgcn_sched_barrier(0); t0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  double s0 = 0.0, s1 = 0.0;
#pragma unroll 32
  for (int i = 0; i < STEPS / 2; ++i) { s0 = fma(rl(c0 + i, i & 63), 1.0, s0); s1 = fma(rl(c1 + i, (i + 5) & 63), 1.0, s1); }
  __builtin_amdgcn_sched_barrier(0); t1 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0);
  if (l == 0) out[9] = double(t1 - t0) / STEPS;
  out[16 + l] = y + acc + s0 + s1;
}

int main() {
  double* d;
  hipMalloc(&d, 128 * sizeof(double));
  double h[16];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, 1.0, 3);
    hipMemcpy(h, d, 16 * sizeof(double), hipMemcpyDeviceToHost);
  }
  const char* nm[10] = {"fma chain", "rsq+2 Newton chain", "LDS write->read (wave_barrier)", "LDS write->read (__syncthreads x2)",
                        "readlane -> fma chain", "DPP row_shr -> fma chain", "ds_bpermute pair -> fma chain",
                        "fma throughput (per instr)", "LDS bcast read throughput (per read+add)", "readlane pair + fma throughput (per pair)"};
  for (int i = 0; i < 10; ++i) printf("%-45s %8.1f s_memtime ticks\n", nm[i], h[i]);
  // s_memtime frequency: compare with a wall-clock timed loop
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 100; ++rep) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, 1.0, 3);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("100 launches: %.3f ms\n", ms);
  return 0;
}
