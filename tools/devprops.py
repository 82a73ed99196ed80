"""Print the HIP device attributes that bound occupancy (diagnostic)."""
import ctypes

import torch

torch.cuda.init()
lib = ctypes.CDLL("libamdhip64.so")
v = ctypes.c_int()
for name, enum in (("max_blocks_per_cu", 25),):
    rc = lib.hipDeviceGetAttribute(ctypes.byref(v), enum, 0)
    print(name, v.value, "rc", rc)
print(torch.cuda.get_device_properties(0))
