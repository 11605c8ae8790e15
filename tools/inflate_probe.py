"""tools/inflate_probe.py BAM [max_bytes] [check] -- the GPU BGZF inflater on a
BAM (grom_inflate_device_selftest): blocks, inflated bytes, the kernel's time
(HIP events, second of two launches) and GB/s of output; check=1 also
compares every block with zlib on the host."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import grom_amd  # noqa: E402

path = sys.argv[1]
max_bytes = int(float(sys.argv[2])) if len(sys.argv) > 2 else 0
check = int(sys.argv[3]) if len(sys.argv) > 3 else 0
f = grom_amd.lib().grom_inflate_device_selftest
f.restype = ctypes.c_int64
f.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
ms, nb, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64()
bad = f(path.encode(), 0, max_bytes, check, ctypes.byref(ms), ctypes.byref(nb), ctypes.byref(by))
print(json.dumps({"bam": path, "blocks": nb.value, "inflated_bytes": by.value, "bad_blocks": bad, "checked": bool(check),
                  "kernel_ms": round(ms.value, 3),
                  "output_gb_per_s": round(by.value / (ms.value / 1e3) / 1e9, 1) if ms.value > 0 else None}))
