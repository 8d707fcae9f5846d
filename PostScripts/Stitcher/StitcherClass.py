# PYTHONPATH entry point kept from the reference layout (MediaPlayer/visionsystem:8-9,
# TestTrackVision/config/start_MotionTestTrack:20-23): `from StitcherClass import Stitcher`
# resolves here and gets the MI355X implementation.
import os as _os
import sys as _sys

_root = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
if _root not in _sys.path:
    _sys.path.insert(0, _root)

from multicamera_stitching_amd.StitcherClass import *  # noqa: E402,F401,F403
from multicamera_stitching_amd.StitcherClass import Stitcher, StitcherBase  # noqa: E402,F401
