#!/usr/bin/env python3
"""HBM-counter calibration run (rocprofv3 --pmc over this script): each k_calib<mode>
dispatch of libtbe.so moves a known byte count with one access shape of the engine's
kernels (include/tbe_tools.h tbe_calib_device).  tools/pmc_summary.py turns the counters
of these dispatches into the per-request-size scale it applies to the engine's kernels
(MI355X_MICROARCH.md, HBM section: calibrate on a known byte count)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from distributedratelimiting.redis_amd import _capi  # noqa: E402

BYTES = 4 << 30          # 4 GiB: far beyond the 256 MiB Infinity Cache
STREAM = 1 << 30         # streamed bytes per streaming pattern
GATHER_N = 1 << 23       # scattered accesses per gather / scatter pattern
WIDTH = {0: 16, 1: 8, 2: 4, 3: 16, 4: 8, 5: 4, 6: 16, 7: 4, 8: 16, 9: 1}


def expected():
    """Bytes each pattern moves: streams their span; gathers/scatters n * width bytes of
    payload in n distinct-ish 128-byte lines (the summary reports counters per access)."""
    out = {}
    for m, w in WIDTH.items():
        streaming = m in (0, 1, 2, 6, 7)
        n = STREAM // w if streaming else GATHER_N
        out[m] = {"n": n, "width": w, "kind": ("read" if m <= 5 else "write"),
                  "pattern": "stream" if streaming else "scatter", "payload_bytes": n * w}
    return out


def main():
    lib = _capi.load()
    lib.tbe_calib_device.restype = ctypes.c_int
    lib.tbe_calib_device.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]
    torch.cuda.set_device(0)
    buf = torch.zeros(BYTES, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for rep in range(3):
        for m, e in expected().items():
            rc = lib.tbe_calib_device(m, buf.data_ptr(), BYTES, e["n"], sink.data_ptr(), None)
            assert rc == 0, (m, rc)
            torch.cuda.synchronize()
    print(json.dumps(expected()))


if __name__ == "__main__":
    main()
