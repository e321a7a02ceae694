"""How does v_mfma_f32_16x16x32_f16 round its sums? (r05 PSNR-drift probe; needs the GPU)

Random f16 operands, C = A0 B0 + A1 B1 (K = 64 in two chained MFMAs, the field backward's
input-gradient shape). Against the exact f64 sum: signed error in f32 ulps (bias and
spread), and how often f16(C) differs from f16(exact) -- beside the same figures for an
f32 sum in sequential k order with round-to-nearest-even (what a CPU f32 loop does).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libanr_ubench.so"))


def run(scale_a, scale_b, n_mats=4096, seed=0, shift_b=0):
    """shift_b: b is multiplied by 2^shift_b in f16 (exact: no overflow) before the MFMA
    and the result by 2^-shift_b after it -- the exponent shift that keeps f16 subnormal
    operands out of the MFMA."""
    rng = np.random.default_rng(seed)
    a = (rng.standard_normal((n_mats, 2, 64, 8)) * scale_a).astype(np.float16)
    b = (rng.standard_normal((n_mats, 2, 64, 8)) * scale_b).astype(np.float16)
    bs = (b.astype(np.float64) * 2.0 ** shift_b).astype(np.float16)
    assert np.array_equal(bs.astype(np.float64) * 2.0 ** -shift_b, b.astype(np.float64))
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(bs).cuda()
    tc = torch.zeros(n_mats, 64, 4, device="cuda")
    rc = lib.ub_mfma_dot(ctypes.c_void_p(ta.data_ptr()), ctypes.c_void_p(tb.data_ptr()),
                         ctypes.c_void_p(tc.data_ptr()), n_mats,
                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    c = tc.cpu().numpy().astype(np.float64) * 2.0 ** -shift_b
    # A[mat][row][k], B[mat][k][col] from the lane layout
    A = np.zeros((n_mats, 16, 64), np.float64)
    Bm = np.zeros((n_mats, 64, 16), np.float64)
    for kb in range(2):
        for l in range(64):
            r, kk = l % 16, 32 * kb + 8 * (l // 16)
            A[:, r, kk:kk + 8] = a[:, kb, l, :]
            Bm[:, kk:kk + 8, r] = b[:, kb, l, :]
    exact = A @ Bm  # f64: products of f16 are exact, sums of 64 near-exact
    C = np.zeros((n_mats, 16, 16), np.float64)
    for l in range(64):
        for i in range(4):
            C[:, 4 * (l // 16) + i, l % 16] = c[:, l, i]
    prods = (A[:, :, :, None] * Bm[:, None, :, :]).astype(np.float32)  # exact in f32
    seq = np.zeros((n_mats, 16, 16), np.float32)
    for k in range(64):
        seq = (seq + prods[:, :, k, :]).astype(np.float32)
    ulp = np.spacing(np.abs(exact).astype(np.float32)).astype(np.float64)
    out = {}
    for name, v in (("mfma", C), ("f32seq", seq.astype(np.float64))):
        e = (v - exact) / ulp
        h_v = v.astype(np.float32).astype(np.float16)
        h_x = exact.astype(np.float32).astype(np.float16)
        # toward-zero bias: signed error times sign(exact)
        tz = np.mean(e * np.sign(exact))
        out[name] = {"max_abs_ulp": float(np.max(np.abs(e))), "mean_ulp": float(np.mean(e)),
                     "mean_toward_larger_magnitude_ulp": float(tz),
                     "rms_ulp": float(np.sqrt(np.mean(e ** 2))),
                     "f16_differs_frac": float(np.mean(h_v != h_x)),
                     "exact_match_frac": float(np.mean(v == exact.astype(np.float32)))}
    return out


if __name__ == "__main__":
    for sa, sb, sh in ((1.0, 1.0, 0), (1e-3, 1e-2, 0), (1.0, 1e-6, 0), (1.0, 1e-6, 12),
                       (1e-6, 1.0, 0), (1e-2, 1e-4, 0), (1e-2, 3e-5, 0), (1e-2, 3e-5, 8)):
        r = run(sa, sb, shift_b=sh)
        print(f"scale a {sa} b {sb} shift_b {sh}:",
              {k: {x: round(v[x], 6) for x in ("rms_ulp", "mean_toward_larger_magnitude_ulp",
                                               "f16_differs_frac")} for k, v in r.items()},
              flush=True)
