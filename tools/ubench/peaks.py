"""Measured MI355X ceilings for the rooflines (tools/ubench/ubench.hip).

``measure(dev)`` runs each microbenchmark on the current stream a few times, times it with
HIP events and returns the best rate:

* ``hbm_copy_gbs``  float4 copy of 2 x 1 GiB (bytes read + written / time)
* ``hbm_read_gbs``  float4 read of 2 GiB
* ``mfma_f16_tfs`` / ``mfma_bf16_tfs`` / ``mfma_f32_tfs``  back-to-back
  v_mfma_f32_16x16x32_{f16,bf16} / v_mfma_f32_16x16x4_f32 on random operands, best of
  1, 2 and 8 waves per SIMD, every CU
* ``atomic_seg16_greq_s``  f32 atomic wave-instructions cut into 16 segments of 4 lanes
  (16 B) at random 16-B-aligned addresses of a 49 MB table: the hash-grid backward's
  shape (one segment per level); G segment requests / s. ``atomic_seg64_greq_s`` (4 x
  64 B) and ``atomic_seg256_greq_s`` (one contiguous 256 B instruction) for comparison,
  as 64-B requests / s.

Measurement infrastructure (bench.py's untimed phase, tools/), never on the product path.
"""

from __future__ import annotations

import ctypes
import os

import torch

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libanr_ubench.so")


def _lib():
    lib = ctypes.CDLL(LIB)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    lib.ub_copy.argtypes = [vp, vp, i64, i32, vp]
    lib.ub_read.argtypes = [vp, i64, vp, i32, vp]
    lib.ub_mfma.argtypes = [i32, i32, i32, vp, vp]
    lib.ub_atomic.argtypes = [vp, i64, i32, i32, i32, ctypes.c_uint32, vp]
    return lib


def _time(fn, reps: int) -> float:
    """Best of ``reps`` launches, seconds (HIP events on torch's current stream)."""
    fn()  # warm
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e-3)
    return best


def measure(dev: torch.device, reps: int = 5) -> dict:
    lib = _lib()
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    out = {"cus": n_cu}

    n4 = (1 << 30) // 16  # 1 GiB of float4
    src = torch.empty(n4 * 4, device=dev).uniform_()
    dst = torch.empty_like(src)
    sink = torch.zeros(256, device=dev)

    def chk(rc):
        if rc != 0:
            raise RuntimeError(f"ubench launch failed ({rc})")

    # best over grid shapes: 8 / 32 resident blocks per CU (grid-stride) and one float4
    # per lane over the whole array
    grids = (n_cu * 8, n_cu * 32, -(-n4 // 256))
    t = min(_time(lambda: chk(lib.ub_copy(src.data_ptr(), dst.data_ptr(), n4, g, st)), reps)
            for g in grids)
    out["hbm_copy_gbs"] = round(2 * n4 * 16 / t / 1e9, 1)
    t = min(_time(lambda: chk(lib.ub_read(src.data_ptr(), n4, sink.data_ptr(), g, st)), reps)
            for g in grids)
    out["hbm_read_gbs"] = round(n4 * 16 / t / 1e9, 1)
    del src, dst

    # best of 1, 2 and 8 waves per SIMD (256-thread blocks, one per CU per wave slot)
    iters = 4096
    res = torch.empty(n_cu * 8 * 256, device=dev)
    for name, bf in (("mfma_f16_tfs", 0), ("mfma_bf16_tfs", 1), ("mfma_f32_tfs", 2)):
        best = 0.0
        for wps in (1, 2, 8):
            mblocks = n_cu * wps
            flops = mblocks * 4 * iters * 4 * (2 * 16 * 16 * (4 if bf == 2 else 32))
            t = _time(lambda: chk(lib.ub_mfma(bf, iters, mblocks, res.data_ptr(), st)), reps)
            best = max(best, flops / t / 1e12)
        out[name] = round(best, 1)

    n_floats = 12_196_240  # the T = 2^19 hash table's f32 gradient (49 MB)
    table = torch.zeros(n_floats, device=dev)
    ablocks, aiters = n_cu * 8, 256
    waves = ablocks * 4
    for seg_lanes, key in ((4, "atomic_seg16_greq_s"), (16, "atomic_seg64_greq_s"),
                           (64, "atomic_seg256_greq_s")):
        nreq = waves * aiters * (64 // seg_lanes) if seg_lanes < 16 else \
            waves * aiters * 4  # 64-B memory-side requests
        t = _time(lambda: chk(lib.ub_atomic(table.data_ptr(), n_floats, seg_lanes, aiters,
                                            ablocks, 12345, st)), reps)
        out[key] = round(nreq / t / 1e9, 3)
        if seg_lanes == 4:
            out["atomic_seg16_gbs_added"] = round(waves * aiters * 256 / t / 1e9, 1)
    torch.cuda.synchronize(dev)
    return out


if __name__ == "__main__":
    import json

    print(json.dumps(measure(torch.device("cuda", 0))))
