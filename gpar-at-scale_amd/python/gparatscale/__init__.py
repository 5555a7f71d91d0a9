"""gparatscale -- MI355X-native GPAR-at-scale hot path (Python mirror of the Julia API).

Mirrors the reference module `GPARatScale` (src/GPARatScale.jl) for the per-output GP
regression hot path; all arithmetic runs in the gfx950 kernels of libgparhip.so.
"""
from ._lib import (  # noqa: F401
    Context, DomainError, GparError, PosDefException, Unsupported, context, load, LIB_PATH,
    EXPORTED, NelderMead, nelder_mead, debug_counter,
)
from .api import *  # noqa: F401,F403
