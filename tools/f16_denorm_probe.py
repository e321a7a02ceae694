"""Does gfx950 keep f16 subnormals in an MFMA operand, a conversion and a native f16
multiply? (r04 drift diagnostic; tools/ubench ub_f16_denorm). Prints the four values; each
of the first three is 2^-20 = 9.5367e-07 when subnormals are kept, 0 when flushed."""

import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "atmospheric-neural-rendering_amd"))

import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libanr_ubench.so"))
out = torch.zeros(4, device="cuda:0")
rc = lib.ub_f16_denorm(ctypes.c_void_p(out.data_ptr()),
                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print({"rc": rc, "mfma": out[0].item(), "cvt": out[1].item(), "mul_f16": out[2].item(),
       "expected": out[3].item()})
