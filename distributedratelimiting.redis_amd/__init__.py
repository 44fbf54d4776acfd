"""MI355X-native batched token-bucket engine (drop-in for the Redis script path of
ReubenBond/DistributedRateLimiting.Redis).

The decision path is HIP (``csrc/``) behind the C ABI in ``include/tbe.h``; this
Python package only binds that ABI (``_capi``) and moves buffers (``engine``).
Importing it does not load the shared library; the first engine does, and fails
loudly if ``libtbe.so`` has not been built (see ``build.py``).
"""
from .engine import (ApproximateEngine, QueueingTokenBucketEngine, TokenBucketEngine,  # noqa: F401
                     fill_rate)
from ._capi import TbeError  # noqa: F401

__all__ = ["TokenBucketEngine", "QueueingTokenBucketEngine", "ApproximateEngine", "TbeError", "fill_rate"]
