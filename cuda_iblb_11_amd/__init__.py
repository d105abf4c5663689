"""MI355X-native (gfx950) immersed-boundary lattice-Boltzmann hot path of ptheywood/CUDA_IBLB_11.

The compute lives in libiblb.so (hand-written HIP kernels behind the C ABI of include/iblb.h).
This package is the host-side mirror of that boundary: `Lattice` (fused context API),
`LocalGroup` / `Lattice.attach_rccl` (x-slab decomposition) and `kernels` (reference-named
drop-in kernels on device tensors).  There is no CPU fallback.
"""
from ._lib import IBLB_ERR_ARG, IBLB_ERR_COMM, IBLB_ERR_STATE, IblbError, device_count, load
from .lattice import (Lattice, LocalGroup, RefParams, plan_slabs, rccl_unique_id, reference_taus,
                      split_populations, split_state)

__all__ = [
    "IBLB_ERR_ARG", "IBLB_ERR_COMM", "IBLB_ERR_STATE", "IblbError", "device_count", "load", "Lattice", "LocalGroup", "RefParams", "plan_slabs",
    "rccl_unique_id", "reference_taus", "split_populations", "split_state",
]
