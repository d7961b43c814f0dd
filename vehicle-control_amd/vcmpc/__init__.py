"""vcmpc -- MI355X-native batched MPC solve path for neverorfrog/vehicle-control.

Python surface of the reference (controllers/, models/, utils/) over the C ABI
of libvcmpc.so (include/vcmpc.h); all arithmetic runs in gfx950 HIP kernels.
"""
from . import _abi  # noqa: F401
from .config import AttrDict, load_config, make_params  # noqa: F401
from .solver import Context  # noqa: F401

__all__ = ["Context", "load_config", "make_params", "AttrDict"]
