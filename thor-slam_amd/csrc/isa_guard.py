#!/usr/bin/env python3
"""Build guard for libtslam_hip.so: fail the build when the gfx950 code of any kernel

1. spills VGPRs (``.vgpr_spill_count`` > 0) or uses private (scratch) memory at all
   (``.private_segment_fixed_size`` > 0: spills, and private arrays indexed at run time), or
2. contains an MFMA whose destination shares registers with a source other than an exact
   accumulate (srcC == vdst): vdst overlapping srcA / srcB, or srcC partially overlapping vdst, or
3. is an in-launch hand-off kernel (``HANDOFF``: blocks publish data, count themselves in, the last
   block to arrive reads everything) whose machine code does not follow the hardware rule the
   hand-off relies on instead of an agent-scope release / acquire pair ("the BA
   hand-off and the memory model"): every global store before the counter atomic carries ``sc1``
   (agent scope: written through the XCD's L2), an ``s_waitcnt vmcnt(0)`` separates the last of
   them from the counter atomic (the stores have reached memory before the count is visible), and
   the last block reads the published data with at least the listed number of ``sc1`` loads
   (agent scope: not served from a stale line of its own XCD's L2).

Why ("k_match and the MFMA operand rule"): the toolchain keeps the destination of a
>128-bit MFMA apart from its sources by an early-clobber constraint, and its assembler rejects a
partial srcC overlap ("source 2 operand must not partially overlap with dst") — but neither holds
for the block-scaled ``v_mfma_scale_*`` instructions k_match uses.  A k_match build forced to 4
waves/SIMD spilled 43 VGPRs, and under that register pressure the allocator emitted
``v_mfma_scale_f32_32x32x64_f8f6f4 v[16:31], v[20:23], v[0:3], v[4:19]``: srcC v[4:19] half inside
vdst v[16:31], srcA too — the build that gave wrong stereo matches.  Nothing in the compiler stops
that, so the build checks the machine code itself.

SGPR spills are not counted: with no private segment they go to VGPR lanes (``v_writelane`` /
``v_readlane``), which changes neither memory traffic nor results; ``--verbose`` lists them.

The device code is read from each host object's ``.hip_fatbin`` (llvm-objcopy →
clang-offload-bundler → llvm-readelf --notes / llvm-objdump -d).  Usage::

    isa_guard.py [--verbose] OBJ.o|CODE_OBJECT [...]      # exit 1 and one line per violation
"""

from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path(os.environ.get("ROCM_LLVM_BIN", "/opt/rocm/lib/llvm/bin"))
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
_REG = re.compile(r"^([va])(?:\[(\d+):(\d+)\]|(\d+))$")
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")
_BASE = re.compile(r"^_Z(\d+)")

# hand-off kernel -> the agent-scope loads its last block must issue for the published data
# (k_ba_reduce_solve: C as 4096 / 512 threads = 8 loads per thread, and the camera blocks: 1)
HANDOFF = {"k_ba_reduce_solve": 9, "k_ba_reduce_solve_ine": 9, "k_ba_reduce_solve_rec": 9, "k_ba_reduce_solve_ine_rec": 9}


def _run(*args: str) -> str:
    return subprocess.run(args, check=True, capture_output=True, text=True).stdout


def code_object(path: Path, tmp: Path) -> Path | None:
    """The gfx950 code object inside a host object (None: no device code), or ``path`` itself
    when it already is one (an ELF for AMDGPU)."""
    with open(path, "rb") as f:
        head = f.read(20)
    if head[:4] == b"\x7fELF" and int.from_bytes(head[18:20], "little") == 0xE0:   # EM_AMDGPU
        return path
    sections = _run(str(LLVM / "llvm-readelf"), "-S", str(path))
    if ".hip_fatbin" not in sections:
        return None
    fat = tmp / (path.name + ".fatbin")
    _run(str(LLVM / "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", str(path), str(fat))
    out = tmp / (path.name + ".co")
    _run(str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
         f"--targets={TARGET}", f"--output={out}")
    return out


def kernel_resources(co: Path) -> list[dict]:
    """Per kernel of the code object: name, spill counts, private segment bytes (metadata note)."""
    kernels: list[dict] = []
    for line in _run(str(LLVM / "llvm-readelf"), "--notes", str(co)).splitlines():
        if line.startswith("  - ."):
            kernels.append({})
        m = re.match(r"^    \.(name|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|vgpr_count):\s+(\S+)", line)
        if m and kernels:
            kernels[-1][m.group(1)] = m.group(2) if m.group(1) == "name" else int(m.group(2))
    return kernels


def _regs(tok: str):
    m = _REG.match(tok.strip())
    if not m:
        return None   # an inline constant or a literal
    lo = int(m.group(2) if m.group(2) is not None else m.group(4))
    hi = int(m.group(3)) if m.group(3) is not None else lo
    return m.group(1), lo, hi


def _overlap(a, b) -> bool:
    return a is not None and b is not None and a[0] == b[0] and not (a[2] < b[1] or b[2] < a[1])


def mfma_violations(co: Path) -> list[str]:
    """MFMAs whose vdst overlaps srcA / srcB, or whose srcC overlaps vdst without being equal."""
    bad, func = [], "?"
    for line in _run(str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", str(co)).splitlines():
        m = _FUNC.match(line.strip())
        if m:
            func = m.group(1)
            continue
        s = line.split("//")[0].strip()
        if not s.startswith("v_mfma"):
            continue
        mnem, _, rest = s.partition(" ")
        ops = [o.strip() for o in rest.split(",")]
        if len(ops) < 4:
            continue
        d, a, b, c = (_regs(o.split()[0]) if o else None for o in ops[:4])
        why = [n for n, r in (("srcA", a), ("srcB", b)) if _overlap(d, r)]
        if _overlap(d, c) and d != c:
            why.append("srcC (partial)")
        if why:
            bad.append(f"{func}: {s}  [vdst overlaps {', '.join(why)}]")
    return bad


def _base_name(mangled: str) -> str:
    m = _BASE.match(mangled)
    return mangled[m.end():m.end() + int(m.group(1))] if m else mangled


def _functions(co: Path) -> dict[str, list[str]]:
    """Instruction lines (comments stripped) per function of the code object's disassembly."""
    funcs: dict[str, list[str]] = {}
    cur: list[str] | None = None
    for line in _run(str(LLVM / "llvm-objdump"), "-d", "--mcpu=gfx950", "--no-show-raw-insn", str(co)).splitlines():
        m = _FUNC.match(line.strip())
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        s = line.split("//")[0].strip()
        if cur is not None and s:
            cur.append(s)
    return funcs


def handoff_violations(co: Path, table: dict[str, int] | None = None, found: set | None = None) -> list[str]:
    """Rule 3 over every kernel of ``table`` (default ``HANDOFF``) found in the code object (their
    names are added to ``found``)."""
    table = HANDOFF if table is None else table
    bad = []
    for func, ins in _functions(co).items():
        name = _base_name(func)
        if name not in table:
            continue
        if found is not None:
            found.add(name)
        # the counter: the first returning (sc0) global atomic
        at = next((i for i, s in enumerate(ins) if s.startswith("global_atomic") and " sc0" in f" {s} "), None)
        if at is None:
            bad.append(f"{func}: hand-off kernel without a returning counter atomic")
            continue
        stores = [i for i in range(at) if ins[i].startswith("global_store")]
        if not stores:
            bad.append(f"{func}: hand-off kernel publishes nothing before its counter atomic")
        for i in stores:
            if "sc1" not in ins[i].split():
                bad.append(f"{func}: {ins[i]}  [published store without sc1 (agent scope) before the counter]")
        if stores and not any(s.startswith("s_waitcnt") and "vmcnt(0)" in s for s in ins[stores[-1] + 1:at]):
            bad.append(f"{func}: no s_waitcnt vmcnt(0) between the last published store and the counter atomic")
        loads = sum(1 for s in ins[at + 1:] if s.startswith("global_load") and "sc1" in s.split())
        if loads < table[name]:
            bad.append(f"{func}: {loads} sc1 (agent-scope) loads after the counter, the hand-off needs {table[name]}")
    return bad


def check(paths: list[Path], notes: list[str] | None = None, handoff: dict[str, int] | None = None) -> list[str]:
    """Every violation of the two rules over the given objects, as printable lines (SGPR spills
    into VGPR lanes go to ``notes`` when given)."""
    errors: list[str] = []
    found: set = set()
    with tempfile.TemporaryDirectory() as d:
        for p in paths:
            co = code_object(Path(p), Path(d))
            if co is None:
                continue
            for k in kernel_resources(co):
                name = k.get("name", "?")
                if k.get("vgpr_spill_count", 0):
                    errors.append(f"{Path(p).name}: {name} spills {k['vgpr_spill_count']} VGPRs")
                if k.get("sgpr_spill_count", 0) and notes is not None:
                    notes.append(f"{Path(p).name}: {name} spills {k['sgpr_spill_count']} SGPRs into VGPR lanes")
                if k.get("private_segment_fixed_size", 0):
                    errors.append(f"{Path(p).name}: {name} uses {k['private_segment_fixed_size']} B/lane of scratch")
            errors += [f"{Path(p).name}: {v}" for v in mfma_violations(co)]
            errors += [f"{Path(p).name}: {v}" for v in handoff_violations(co, handoff, found)]
    # a hand-off kernel that vanished from the library (renamed, or the objects incomplete) would
    # pass unchecked: the library's own objects must hold every HANDOFF kernel
    table = HANDOFF if handoff is None else handoff
    if any(Path(p).name == "k_ba.hip.o" for p in paths) or handoff is not None:
        errors += [f"{m}: hand-off kernel not found in the checked objects" for m in sorted(set(table) - found)]
    return errors


def main(argv: list[str]) -> int:
    notes: list[str] | None = [] if "--verbose" in argv else None
    errors = check([Path(a) for a in argv if a != "--verbose"], notes)
    for n in notes or []:
        print(f"isa_guard: note: {n}", file=sys.stderr)
    for e in errors:
        print(f"isa_guard: {e}", file=sys.stderr)
    if errors:
        print(f"isa_guard: {len(errors)} violation(s); see thor-slam_amd/csrc/isa_guard.py", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
