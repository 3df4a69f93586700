"""mceik_amd -- MI355X-native hot path of the mceik MCMC travel-time tomography
sampler: batched 3D fast-sweeping eikonal solves (HIP, gfx950), L2 misfit with
analytic origin time, Metropolis accept/reject, behind the reference's
mceik.h / mceik_struct.h driver API.
"""
from . import _lib  # noqa: F401  (ctypes binding; raises if the HIP library is missing)

__all__ = ["_lib", "eikonal", "mcmc"]
