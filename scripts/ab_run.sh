set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/kin_ab.py vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_pch2.so vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_pch2.so > gpurun_out/ab12.log 2>&1 || exit $?
VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_timing_pch2.so timeout -k 10 120 python -u scripts/section_timing.py > gpurun_out/ab12_sec_pch2.log 2>&1
