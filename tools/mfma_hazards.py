"""Static check of the MFMA data hazards that hand-written inline asm must cover itself.

The fused field kernels (csrc/field_fused.hip) issue some MFMAs from inline asm (the dW
accumulators in AGPRs, `mma32_acc*`) and a ReLU mask from asm; hipcc's hazard recognizer
pads nothing inside an asm statement, so the kernels carry hand-placed `s_nop`s. r02
shipped one missing pair (a VALU-written MFMA operand read at once: launch-to-launch
different dW). This tool reads the built device code back and checks,
per kernel, in program order (straight-line; a label, a branch target or an
unconditional branch restarts the window):

* VALU write of a VGPR -> MFMA reading it as SrcA / SrcB / SrcC: >= 2 wait states between;
* MFMA write of a VGPR / AGPR -> VALU (incl. v_accvgpr_read / _mov) reading it as a
  source, or MFMA SrcA / SrcB reading it (or a different SrcC range overlapping it): >= R(opcode) wait states, where
  R is the smallest distance hipcc's own hazard recognizer keeps between that opcode's
  result and a VALU reader anywhere in the same objects (8 for the gfx950 16x16 f16 /
  bf16 MFMAs; 12 for an opcode the compiler never emits). Hand-written asm must keep at
  least what the compiler keeps. An MFMA chaining on the previous MFMA's result as its own
  SrcC with the same range is the hardware's forwarding case and needs none.

A wait state is one instruction issue; `s_nop N` is N + 1.

    python tools/mfma_hazards.py [objects...]   (default: the library's MFMA objects)

Exit status 1 and one line per violation when any is found. tests/test_mfma_hazards.py
runs it on the built objects (no GPU needed).
"""

from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OBJS = ["field_fused.o", "mlp_fused.o", "mlp.o"]
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def device_asm(obj: str) -> str:
    """Disassembly of the gfx950 code object embedded in a hipcc host object."""
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                        os.path.join(td, "junk.o")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", f"--targets={TARGET}", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co],
                              check=True, capture_output=True, text=True).stdout


def regs(tok: str) -> set:
    out = set()
    for m in _REG.finditer(tok):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def parse(line: str):
    """(mnemonic, [operand strings]) of a disassembly line, or None."""
    line = line.split("//")[0].strip()
    if not line or line.endswith(":") or line.startswith("<"):
        return None
    parts = line.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def is_mfma(mn: str) -> bool:
    return mn.startswith("v_mfma") or mn.startswith("v_smfmac")


def is_valu(mn: str) -> bool:
    return mn.startswith("v_") and not is_mfma(mn)


def waits(mn: str, ops) -> int:
    if mn == "s_nop":
        return int(ops[0], 0) + 1
    return 1


_ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
_ENDS = ("s_branch", "s_setpc_b64", "s_endpgm")


def blocks(asm: str):
    """(kernel, [(mnemonic, operands, text)]) straight-line blocks in program order. A
    block ends at a label, at an unconditional branch / return, and before any address a
    branch jumps to (llvm-objdump prints no labels for those: the targets are read from
    the branches' `<kernel+0x...>` annotations); code after an `s_branch` is reached only
    by a jump, so an MFMA's result window never runs across it."""
    starts, targets = {}, set()
    for raw in asm.splitlines():
        s = raw.strip()
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", s)
        if m:
            starts[m.group(2)] = int(m.group(1), 16)
    for raw in asm.splitlines():
        t = _TARGET.search(raw)
        if t and t.group(1) in starts and raw.strip().startswith("s_"):
            targets.add(starts[t.group(1)] + int(t.group(2), 16))
    out, kernel, block = [], "?", []

    def flush():
        nonlocal block
        if block:
            out.append((kernel, block))
        block = []

    for raw in asm.splitlines():
        s = raw.strip()
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", s)
        if m or s.endswith(":") or s.startswith("<"):
            flush()
            if m:
                kernel = m.group(1)
            continue  # a label restarts the window
        a = _ADDR.search(s)
        if a and int(a.group(1), 16) in targets:
            flush()  # a branch target restarts the window
        p = parse(s)
        if p:
            block.append((p[0], p[1], s.split("//")[0].strip()))
            if p[0] in _ENDS:
                flush()
    flush()
    return out


def _first_reader(block, i, horizon=64):
    """(index, wait states, kind) of the first instruction after block[i] (an MFMA) that
    reads or overwrites its result, within ``horizon`` wait states; None if none."""
    mn, ops, _ = block[i]
    dst = regs(ops[0])
    w = 0
    for j in range(i + 1, len(block)):
        if w >= horizon:
            return None
        nmn, nops, _ = block[j]
        if is_mfma(nmn) and len(nops) >= 4:
            same_c = nops[3] == ops[0]
            if (regs(nops[1]) | regs(nops[2])) & dst or (regs(nops[3]) & dst and not same_c):
                return j, w, "MFMA"
            if same_c:
                return None  # the accumulation chain continues: the next link is checked
        elif is_valu(nmn) and nops and any(regs(o) & dst for o in nops[1:]):
            return j, w, "VALU"  # a VALU source (RAW); an overwrite alone is not a read
        w += waits(nmn, nops)
    return None


def compiler_minimum(all_blocks) -> dict:
    """Smallest MFMA -> VALU-reader distance per opcode over the given code."""
    need: dict = {}
    for _, block in all_blocks:
        for i, (mn, ops, _) in enumerate(block):
            if is_mfma(mn) and len(ops) >= 4:
                r = _first_reader(block, i)
                if r and r[2] == "VALU":
                    need[mn] = min(need.get(mn, 99), r[1])
    return need


def check(asm: str, need: dict | None = None) -> list[str]:
    """Violations in ``asm``; ``need``: per-opcode MFMA result distance (default: the
    compiler's own minimum in ``asm``)."""
    bs = blocks(asm)
    need = compiler_minimum(bs) if need is None else need
    bad = []
    for kernel, block in bs:
        for i, (mn, ops, text) in enumerate(block):
            if not (is_mfma(mn) and len(ops) >= 4):
                continue
            srcs = regs(ops[1]) | regs(ops[2]) | regs(ops[3])
            w = 0
            for j in range(i - 1, -1, -1):
                if w >= 2:
                    break
                pmn, pops, ptext = block[j]
                if is_valu(pmn) and pops and regs(pops[0]) & srcs:
                    bad.append(f"{kernel}: VALU write -> MFMA read after {w} wait "
                               f"state(s): '{ptext}' -> '{text}'")
                    break
                w += waits(pmn, pops)
            r = _first_reader(block, i)
            n = need.get(mn, 12)
            if r and r[1] < n:
                bad.append(f"{kernel}: MFMA result -> {r[2]} after {r[1]} wait state(s) "
                           f"(needs {n}): '{text}' -> '{block[r[0]][2]}'")
    return bad


def main(argv):
    objs = argv or [os.path.join(ROOT, "atmospheric-neural-rendering_amd", "csrc", "build", o)
                    for o in OBJS]
    asms = {o: device_asm(o) for o in objs}
    need = compiler_minimum([b for a in asms.values() for b in blocks(a)])
    bad = []
    for o, asm in asms.items():
        bad += [f"{os.path.basename(o)}: {b}" for b in check(asm, need)]
    for b in bad:
        print(b)
    n_mfma = sum(a.count("v_mfma") for a in asms.values())
    print(f"{len(objs)} objects, {n_mfma} MFMA instructions, required MFMA result "
          f"distances {need}, {len(bad)} hazard(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
