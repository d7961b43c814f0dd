#!/bin/bash
# A/B of the kin_ltv polish's dual tolerance: certification of the C4 sets + C2/C4 kernel time
set -e
L=vehicle-control_amd/vcmpc
for t in "$@"; do
  for s in c4_bench c4_seed31; do
    VCMPC_LIB=$L/libvcmpc_$t.so timeout -k 10 200 python -u scripts/cert_diag.py $s --top 3 2>&1 | grep -v amdgpu.ids | sed "s/^/[$t] /"
  done
done
libs=""; for t in "$@"; do libs="$libs $L/libvcmpc_$t.so"; done
timeout -k 10 300 python -u scripts/kin_ab.py --batch 1024 --reps 40 $libs
timeout -k 10 300 python -u scripts/kin_ab.py --batch 65536 --reps 5 $libs
