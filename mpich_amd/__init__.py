"""mpich_amd -- MI355X-native local reduction for MPICH.

The hot path of MPI_Reduce / MPI_Allreduce / MPI_Reduce_scatter: the
per-chunk element-wise combine MPIR_Reduce_local, rebuilt as hand-written
gfx950 HIP kernels behind MPICH's own C call surface
(include/mpix_redop.h, libmpix_redop.so), plus the recursive-halving
reduce-scatter schedule that feeds it across GPUs (mpich_amd.coll).
"""
from . import handles  # noqa: F401
from .handles import *  # noqa: F401,F403

__all__ = ['handles', 'redop', 'coll']


def __getattr__(name):
    # redop/coll import torch; load them lazily
    if name in ('redop', 'coll'):
        import importlib
        return importlib.import_module('.' + name, __name__)
    raise AttributeError(name)
