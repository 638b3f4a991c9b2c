"""modulations_amd -- MI355X-native DVB-RCS2 turbo-decode hot path.

Drop-in for the decode side of poriya219/modulations:
``from modulations_amd import dvb_rcs2_turbo`` exposes the reference module's
API with every SISO / decode / demap running in hand-written gfx950 HIP
(modulations_amd/lib/libtdec.so, C ABI in include/tdec.h).
"""
from . import tables  # noqa: F401

__all__ = ["dvb_rcs2_turbo", "demap", "tables"]
