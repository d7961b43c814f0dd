"""FETCH_SIZE / WRITE_SIZE calibration for 8-byte-per-lane accesses (the guide's factor-2 rule for
FETCH_SIZE is calibrated on 16 B/lane streams only; kin_ltv's input and output accesses are one
double per lane).  Runs the rcp probe kernel (csrc/numerics.hip: lane i reads x[i], 8 B, and
writes out[4 i .. 4 i + 3], four 8 B stores) over n = 2^24 doubles from HBM-resident device
buffers: 128 MiB read, 512 MiB written per launch.  Under
    rocprofv3 --kernel-trace --pmc FETCH_SIZE WRITE_SIZE -d <dir> -o run -f csv -- python3 scripts/pmc_calibrate.py
the counters per launch, divided by these byte counts, are the correction factors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vehicle-control_amd"))
import torch  # noqa: E402

from vcmpc import Context, _abi  # noqa: E402

n = 1 << 24
x = torch.rand(n, dtype=torch.float64, device="cuda") + 0.5
out = torch.empty(4 * n, dtype=torch.float64, device="cuda")
with Context(model=_abi.VC_MODEL_KINEMATIC, N=20, max_batch=n) as c:  # (vc_debug_rcp: n <= max_batch)
    for _ in range(4):
        c._check(c.lib.vc_debug_rcp(c._h, n, x.data_ptr(), out.data_ptr(), _abi.VC_DEVICE_PTRS))
    torch.cuda.synchronize()
print(f"rcp probe: n = {n}, read {8 * n} B, written {32 * n} B per launch, 4 launches")
