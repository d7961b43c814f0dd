#!/bin/bash
# C2 kernel time against the batch (kin_ltv_kernel<20>, one 64-lane workgroup per problem):
# 256 CUs x 4 SIMDs hold 1,024 problems at one wave per SIMD (256 VGPRs + 226 AGPRs per lane,
# 38.9 KB of LDS per problem).  If a second wave could share a SIMD, B = 2,048 would overlap
# with B = 1,024 instead of taking a second round.  B = 8,192 is C4's per-rank shard at 8 GPUs and
# B = 65,536 the whole C4 set on one GPU: their kernel-time ratio is the strong-scaling ceiling of
# C4 over 1 -> 8 GPUs (the ranks share nothing on the data path; launch-tail effects included).
# usage: bash scripts/kin_occupancy_sweep.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/kinocc_$TAG
mkdir -p "$OUT"
LEGS="--no-c3 --no-c4 --no-c5 --no-casc --no-kin-legs --no-latency --no-cpu-baseline"
for B in 256 512 1024 1536 2048 4096 8192 65536; do
  timeout -k 10 300 python "$ROOT/bench.py" --batch $B $LEGS > "$OUT/b$B.log" 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
res = {}
for B in (256, 512, 1024, 1536, 2048, 4096, 8192, 65536):
    d = json.loads([l for l in open(f"{out}/b{B}.log") if l.startswith("{")][-1])
    print(f"B={B:5d}: kernel {d['roofline']['kernel_ms']:.4f} ms, {d['value'] / 1e6:.3f} M solves/s, "
          f"IPM iterations mean {d['solver']['iters_mean']:.2f} max {d['solver']['iters_max']}")
    res[B] = d['roofline']['kernel_ms']
print(f"C4 strong-scaling ceiling 1 -> 8 GPUs (kernel time B = 65,536 / B = 8,192): {res[65536] / res[8192]:.2f}x "
      f"(ideal 8; B = 8,192 is {8192 // 1024} rounds of the machine at one problem per SIMD)")
PY
