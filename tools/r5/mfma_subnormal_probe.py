"""Which f16 subnormal operands does v_mfma_f32_16x16x32_f16 keep exactly? (r05 probe)
One nonzero product per output: A[r][0] = k * 2^-24 (k = 1..1023, the f16 subnormals),
B[0][c] = 1, everything else 0; prints the k whose product comes back inexact."""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libanr_ubench.so"))
ks = np.arange(1, 1024)
n = len(ks)
a = np.zeros((n, 2, 64, 8), np.float16)
b = np.zeros((n, 2, 64, 8), np.float16)
# lane l < 16: A row l, k = 0..7; put the subnormal at (row 0, k 0) and B[0][col 0] = 1
a[:, 0, 0, 0] = (ks * 2.0 ** -24).astype(np.float16)
b[:, 0, 0, 0] = 1.0
for scale_b in (1.0, 3.0, 0.5):
    b[:, 0, 0, 0] = scale_b
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    tc = torch.zeros(n, 64, 4, device="cuda")
    assert lib.ub_mfma_dot(ctypes.c_void_p(ta.data_ptr()), ctypes.c_void_p(tb.data_ptr()),
                           ctypes.c_void_p(tc.data_ptr()), n,
                           ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    got = tc[:, 0, 0].cpu().numpy().astype(np.float64)  # C[row 0][col 0]
    want = ks * 2.0 ** -24 * scale_b
    bad = ks[got != want]
    print(f"b={scale_b}: inexact for {len(bad)} of {n} subnormal a; first {bad[:12].tolist()}; "
          f"got/want at those {[(float(got[k-1] / want[k-1])) for k in bad[:6]]}", flush=True)
