"""Python handle over the MI355X PPE decode + ACL classify engine (libppe_hip.so, C ABI in include/ppe_hip.h).

Plumbing for tests and bench.py only: every classification runs in the HIP kernels of libppe_hip.so.
"""
from . import abi, synth  # noqa: F401
from .abi import RULE_DTYPE, ST, ST_NAME, COUNTERS, build_image  # noqa: F401
from .engine import Defrag, Engine, PPEError, decode_verdict  # noqa: F401
