set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/kin_ab.py vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_piv2.so vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_piv2.so > gpurun_out/ab11.log 2>&1 || exit $?
VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_piv2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kin_sqp.py tests/test_gpu_obstacles.py -k 'not closed_loop' > gpurun_out/ab11_parity_piv2.log 2>&1 || exit $?
VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_timing_piv2.so timeout -k 10 120 python -u scripts/section_timing.py > gpurun_out/ab11_sec_piv2.log 2>&1
