"""ompi_amd -- an MI355X-native MPI derived-datatype pack/unpack engine.

The product is ``libddt_hip.so`` (C ABI in ``include/ddt_hip.h``): hand-written gfx950
gather/scatter kernels driven by a host plan compiler, sitting behind Open MPI's
datatype + convertor interface.  This package is the Python mirror of that interface.
"""
from ._lib import DDTError, LIB_PATH, lib  # noqa: F401
from . import datatype, convertor  # noqa: F401
from .datatype import MPI, Datatype  # noqa: F401
from .convertor import (Convertor, pack, unpack, pack_size, pack_external,  # noqa: F401
                        unpack_external, pack_external_size)

__all__ = ["lib", "LIB_PATH", "DDTError", "datatype", "convertor", "MPI", "Datatype",
           "Convertor", "pack", "unpack", "pack_size", "pack_external", "unpack_external",
           "pack_external_size"]
