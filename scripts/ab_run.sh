set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/kin_ab.py vehicle-control_amd/vcmpc/libvcmpc_head.so vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_blk.so vehicle-control_amd/vcmpc/libvcmpc_head.so vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_blk.so > gpurun_out/ab10.log 2>&1 || exit $?
VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_blk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kin_sqp.py > gpurun_out/ab10_parity_blk.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kin_sqp.py > gpurun_out/ab10_parity.log 2>&1 || exit $?
VCMPC_LIB=vehicle-control_amd/vcmpc/libvcmpc_timing_blk.so timeout -k 10 120 python -u scripts/section_timing.py > gpurun_out/ab10_sec_blk.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/kin_ab.py --batch 65536 --reps 5 vehicle-control_amd/vcmpc/libvcmpc_head.so vehicle-control_amd/vcmpc/libvcmpc.so vehicle-control_amd/vcmpc/libvcmpc_blk.so > gpurun_out/ab10_c4.log 2>&1
