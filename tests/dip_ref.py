"""Re-export of oracle/dip_ref.py (the plain-torch DIP restatement lives with the rest of the oracle)."""
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _REPO not in sys.path:
    sys.path.insert(0, _REPO)

from oracle.dip_ref import *  # noqa: E402,F401,F403
from oracle.dip_ref import CONV, BN, CONCAT, EarlyStopRef, RefTrainer  # noqa: E402,F401
