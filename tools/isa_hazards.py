"""Scan the built gfx950 code objects for an MFMA result read by a non-MFMA instruction too soon after the MFMA
(the RAW hazard behind round 5's mha_block wrong results, verdict item 7; DESIGN.md §5 "Compiler hazards").

tools/probe/mfma_war.hip measured on MI355X: a v_accvgpr_read of a v_mfma_f32_16x16x32_bf16 result (8 passes)
with fewer than 7-8 wait states in between returns the stale register, and the hardware has no interlock for it;
the compiler must insert the wait states.  In the bad mha_block schedule it did so only on the fall-through
path of a uniform branch:
    v_mfma_f32_16x16x32_bf16 a[4:7], v[12:15], v[106:109], a[4:7]
    s_cbranch_vccnz .LBB3_116          ; taken: wave with two row tiles
    ...                                ; fall-through: 10 instructions (the third tile's MFMA + AGPR copies)
  .LBB3_116:
    v_accvgpr_read_b32 v39, a7         ; 1 wait state after the MFMA on the taken edge -> stale a7

This checker follows every path (fall-through and branch targets) from each MFMA and reports a read of any of its
destination registers by a VALU / memory instruction before that register's measured wait states (each
instruction counts one, s_nop N counts N + 1; need_for()), unless the register was overwritten first -- and, as
a write-after-write hazard, a VALU write of a destination register inside the same window (the MFMA's own late
write-back would land on top of it; the RAW thresholds are used for it, the WAW ones were not probed).
    python tools/isa_hazards.py [object files ...]      (default: speaker_diarization_amd/lib/obj/*.o)
Exit status 1 if any hazard is found."""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
REG = re.compile(r"\b([av])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def need_for(mnemonic: str, k: int) -> int:
    """Wait states destination register k (0-based within the MFMA's dst range) needs before a VALU may read it,
    as measured on MI355X (tools/probe/mfma_war.hip, profiles/r06/hazards/mfma_hazard.txt): 16x16 shapes (4 dst
    registers) 7, 7, 8, 8; 32x32 shapes (16 dst registers, written 4 at a time) 6 + 2 * (k // 4)."""
    m = re.search(r"_(\d+)x(\d+)x(\d+)", mnemonic)
    big = m is not None and int(m.group(1)) == 32
    if big:
        return 6 + 2 * (k // 4)
    return 7 if k < 2 else 8


def regs(text: str):
    out = set()
    for kind, lo, hi, one in REG.findall(text):
        if one:
            out.add((kind, int(one)))
        else:
            out.update((kind, r) for r in range(int(lo), int(hi) + 1))
    return out


def disassemble(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True,
                       capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--symbolize-operands",
                            "--no-show-raw-insn", co], check=True, capture_output=True, text=True)
        return r.stdout


def parse(dis: str):
    """-> list of functions: (name, instrs [(mnemonic, operands)], labels {label: index})."""
    funcs = []
    cur = None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            name = m.group(1)
            if re.match(r"^L\d+$", name):
                cur[2][name] = len(cur[1])
            else:
                cur = (name, [], {})
                funcs.append(cur)
            continue
        if cur is None or not line.startswith("\t"):
            continue
        ins = line.split("//")[0].strip()
        if not ins:
            continue
        parts = ins.split(None, 1)
        cur[1].append((parts[0], parts[1] if len(parts) > 1 else ""))
    return funcs


def wait_states(mn: str, ops: str) -> int:
    if mn == "s_nop":
        return int(ops.strip(), 0) + 1
    return 1


def is_reader(mn: str) -> bool:
    """Instructions whose register reads are subject to the XDL-write hazard (VALU, LDS / memory data)."""
    if mn.startswith("v_mfma") or mn.startswith("s_"):
        return False
    return mn.startswith(("v_", "ds_", "global_", "buffer_", "scratch_", "flat_"))


def sources(mn: str, ops: str):
    parts = [p.strip() for p in ops.split(",")]
    if mn.startswith(("ds_write", "ds_store", "global_store", "buffer_store", "scratch_store", "flat_store")):
        return regs(ops)
    if mn.startswith(("ds_", "global_", "buffer_", "scratch_", "flat_")):
        return regs(",".join(parts[1:]))      # loads: the address operands
    return regs(",".join(parts[1:]))


def dests(mn: str, ops: str):
    if mn.startswith(("ds_write", "ds_store", "global_store", "buffer_store", "scratch_store", "flat_store", "s_")):
        return set()
    parts = [p.strip() for p in ops.split(",")]
    return regs(parts[0]) if parts and parts[0] else set()


def check_function(name, ins, labels, max_paths=20000):
    found = []
    for i, (mn, ops) in enumerate(ins):
        if not mn.startswith("v_mfma"):
            continue
        dst = regs(ops.split(",")[0])
        base = min(r for _, r in dst) if dst else 0
        need_of = {reg: need_for(mn, reg[1] - base) for reg in dst}
        need = max(need_of.values()) if dst else 0
        # DFS over (index, wait states so far, live destination registers)
        stack = [(i + 1, 0, frozenset(dst))]
        seen = set()
        n = 0
        while stack and n < max_paths:
            j, ws, live = stack.pop()
            n += 1
            while j < len(ins) and ws < need and live:
                key = (j, ws, live)
                if key in seen:
                    break
                seen.add(key)
                mj, oj = ins[j]
                if is_reader(mj):
                    hit = [r for r in sources(mj, oj) & live if ws < need_of[r]]
                    if not hit and mj.startswith("v_"):   # WAW: a VALU overwrite inside the MFMA's window
                        hit = [r for r in dests(mj, oj) & live if ws < need_of[r]]
                    if hit:
                        found.append((name, i, mn, ops, j, mj, oj, ws))
                        break
                live = live - dests(mj, oj)
                if mj == "s_endpgm":
                    break
                if mj == "s_branch":
                    t = labels.get(oj.strip())
                    if t is None:
                        break
                    ws += 1
                    j = t
                    continue
                if mj.startswith("s_cbranch"):
                    t = labels.get(oj.strip())
                    if t is not None:
                        stack.append((t, ws + 1, live))
                ws += wait_states(mj, oj)
                j += 1
    return found


def main(argv):
    objs = argv or sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                 "speaker_diarization_amd", "lib", "obj", "*.hip.*.o")))
    total, kernels = [], 0
    for obj in objs:
        for name, ins, labels in parse(disassemble(obj)):
            kernels += 1
            total += check_function(name, ins, labels)
    for name, i, mn, ops, j, mj, oj, ws in total:
        print(f"HAZARD {name}: [{i}] {mn} {ops}  ->  [{j}] {mj} {oj}  after {ws} wait states")
    print(f"{len(objs)} objects, {kernels} functions, {len(total)} MFMA-result reads / overwrites below the measured wait states")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
