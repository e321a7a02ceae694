"""Static MFMA hazard check of the built device code (tools/mfma_hazards.py; CPU only).

The fused field kernels issue MFMAs and a ReLU mask from inline asm, where hipcc pads no
wait states, so the required ones are hand-placed s_nops (one missing
pair in r02 made dW differ from launch to launch). The checker reads the library's gfx950
code back and verifies every VALU -> MFMA operand and MFMA result -> reader distance.
Validated on the real kernels (r04): with the `s_nop 1` of `mma32_acc_v` deleted, the
rebuilt field_fused.o gives VALU -> MFMA violations at 0 and 1 wait states in the
register-transposed backward (`v_cvt_pk_f16_f32` feeding an AGPR-accumulating MFMA);
restored, none.
"""

import os
import shutil

import pytest

from tools import mfma_hazards as mh

SNIPPET_BAD = """
0000000000001000 <k>:
	v_pk_mul_lo_u16 v1, v8, v1
	v_mfma_f32_16x16x32_f16 a[0:3], v[0:3], v[4:7], a[0:3]
	v_mfma_f32_16x16x32_f16 v[10:13], v[0:3], v[4:7], 0
	v_add_f32_e32 v20, v10, v21
"""

SNIPPET_OK = """
0000000000001000 <k>:
	v_pk_mul_lo_u16 v1, v8, v1
	s_nop 1
	v_mfma_f32_16x16x32_f16 a[0:3], v[0:3], v[4:7], a[0:3]
	v_mfma_f32_16x16x32_f16 a[0:3], v[0:3], v[4:7], a[0:3]
	v_mfma_f32_16x16x32_f16 v[10:13], v[0:3], v[4:7], 0
	s_nop 7
	s_nop 2
	v_add_f32_e32 v20, v10, v21
"""


NEED = {"v_mfma_f32_16x16x32_f16": 8}  # what hipcc keeps on gfx950 (tools/mfma_hazards.py)


def test_checker_flags_the_r02_hazard_class():
    bad = mh.check(SNIPPET_BAD, NEED)
    assert any("VALU write -> MFMA read after 0" in b for b in bad), bad
    assert any("MFMA result -> VALU after 0" in b for b in bad), bad
    # two wait states after the VALU write, 11 after the 16x16 MFMA result, and an
    # accumulating MFMA chaining on its own SrcC: clean
    assert mh.check(SNIPPET_OK, NEED) == []


@pytest.mark.skipif(not shutil.which(f"{mh.LLVM}/llvm-objdump"), reason="no ROCm llvm tools")
def test_library_device_code_has_no_mfma_hazards():
    objs = [os.path.join(mh.ROOT, "atmospheric-neural-rendering_amd", "csrc", "build", o)
            for o in mh.OBJS]
    if not all(os.path.exists(o) for o in objs):
        pytest.skip("library objects not built (run __graft_entry__.build())")
    asms = [mh.device_asm(o) for o in objs]
    need = mh.compiler_minimum([b for a in asms for b in mh.blocks(a)])
    # the compiler's own distances for the field's opcodes: the gfx950 figure (4 passes
    # + 4); a smaller value would mean the calibration picked up a non-reader
    assert need.get("v_mfma_f32_16x16x32_f16", 0) >= 8, need
    assert sum(a.count("v_mfma") for a in asms) > 10000
    bad = [b for a in asms for b in mh.check(a, need)]
    assert bad == [], bad[:10]
