"""Fixture: the seven problems of the bench's N = 60 single-track leg (vcmpc.workload.dynamic_batch
(4096, N=60, seed=31)) that round 2's st_sqp kernel left non-solved (profiles/r02/
pytest_casc_st_r02w.log).  Inputs only (x0, kappa, ds, ubar); the oracle computes the rest.

    python tests/golden/make_st_n60_cases.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.join(os.path.dirname(os.path.dirname(HERE)),
                                                                   "vehicle-control_amd")]
IDX = [418, 828, 1847, 2334, 2499, 2697, 3255]

if __name__ == "__main__":
    from vcmpc.workload import dynamic_batch
    d = dynamic_batch(4096, N=60, seed=31)
    np.savez_compressed(os.path.join(HERE, "st_n60_cases.npz"), idx=np.array(IDX),
                        **{k: np.ascontiguousarray(v[IDX].astype(np.float64)) for k, v in d.items()})
