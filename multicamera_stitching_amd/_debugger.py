"""Stand-in for extended_rospylogs' Debugger mixin (imported at StitcherClass.py:16-17).

The reference only ever calls ``self.debugger(level, msg, log_type=...)`` and never runs the
mixin's __init__ (Stitcher/StitcherBase do not call super().__init__), so the shim keeps no
per-instance state.  Messages go to the stdlib logger ``multicamera_stitching_amd``; levels above
$MCS_DEBUG_LEVEL (default 0) are dropped, mirroring the ROS debug-level parameter
(video_mapping_node.py:63).
"""
from __future__ import annotations

import logging
import os

DEBUG_LEVEL_0 = 0
DEBUG_LEVEL_1 = 1
DEBUG_LEVEL_2 = 2
DEBUG_LEVEL_3 = 3
DEBUG_LEVEL_4 = 4

_log = logging.getLogger("multicamera_stitching_amd")
_LEVELS = {
    "info": logging.INFO,
    "warn": logging.WARNING,
    "warning": logging.WARNING,
    "err": logging.ERROR,
    "error": logging.ERROR,
    "debug": logging.DEBUG,
}


def _threshold() -> int:
    try:
        return int(os.environ.get("MCS_DEBUG_LEVEL", "0"))
    except ValueError:
        return 0


class Debugger(object):
    def debugger(self, level, msg, log_type="info"):
        if level > _threshold():
            return
        _log.log(_LEVELS.get(log_type, logging.INFO), msg)


def update_debuggers(*args, **kwargs):
    return None


def loginfo_cond(cond, msg):
    if cond:
        _log.info(msg)


def logerr_cond(cond, msg):
    if cond:
        _log.error(msg)
