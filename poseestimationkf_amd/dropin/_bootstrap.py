"""Make the poseestimationkf_amd package importable when only this directory is on sys.path.

The reference's driver imports its modules by bare name from the script directory
(Python Kalman Filter/main_file.py:1-6).  A user points sys.path (or PYTHONPATH) at
this ``dropin/`` directory instead; the shims then reach the engine through here.
"""
import os
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.append(_ROOT)

from poseestimationkf_amd import engine  # noqa: E402,F401
from poseestimationkf_amd import _fastcall as fastcall  # noqa: E402,F401  (n = 1 calls, CPython binding)
