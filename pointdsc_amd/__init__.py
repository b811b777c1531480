"""pointdsc_amd -- MI355X-native (gfx950) PointDSC spatial-consistency + NSM hot path.

``pointdsc_amd.PointDSC.PointDSC`` is the drop-in for the reference's
``models.PointDSC.PointDSC``; ``pointdsc_amd.kernels`` exposes each hot-path op;
the C ABI is ``include/pdsc.h`` / ``pointdsc_amd/libpdsc.so``.
"""
__version__ = "0.1.0"
