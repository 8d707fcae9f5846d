"""MI355X-native multi-camera stitch hot path (drop-in for kiwicampus/multicamera_stitching).

The public surface is the reference's own: ``multicamera_stitching_amd.StitcherClass`` (also
importable as ``StitcherClass``) with ``Stitcher`` / ``StitcherBase``.  Pixels go through the
HIP library libmcs.so (include/mcs.h); see DESIGN.md.
"""
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("Stitcher", "StitcherBase"):
        from . import StitcherClass
        return getattr(StitcherClass, name)
    raise AttributeError(name)
