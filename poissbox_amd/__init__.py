"""poissbox_amd -- MI355X-native (gfx950) KSPSolve hot path of 3decomp/poissbox.

Host side mirrors the reference's Fortran/PETSc interface (see api.py); compute runs in the
in-tree HIP library libpoissbox_gpu.so through the C ABI of include/poissbox_gpu.h.
"""
from ._lib import PbError, build, load  # noqa: F401
from .api import *  # noqa: F401,F403
from .api import (ASSEMBLED27, COMPACT, DA, KSP, PC_JACOBI, PC_NONE, REASONS, STAR7,  # noqa: F401
                  Context, Mat, Vec, comm_unique_id, ksp_options, slab_partition)

__version__ = "0.1.0"
