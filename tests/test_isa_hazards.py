"""CPU-side guard for the compiler hazard behind round 5's mha_block wrong results (DESIGN.md §5 "Compiler
hazards"): an MFMA result read by a VALU / memory instruction before the MFMA has written it.  gfx950 has no
interlock for it (tools/probe/mfma_war.hip on MI355X: a v_accvgpr_read of a 16x16x32 bf16 result needs >= 8
wait states), and hipcc (ROCm 7.2) placed the wait states only on the fall-through side of a uniform branch.
tools/isa_hazards.py walks every path from every MFMA in the disassembled gfx950 code objects.

1. The shipped objects (speaker_diarization_amd/lib/obj) carry no such read.
2. The checker finds the round-5 pattern: mha_block.hip with the third tile's MFMA behind the uniform branch
   (`if (ntile > 2)` instead of `if (W == 4 || ntile > 2)`), compiled with the build's flags, reports hazards in
   the 4-wave layouts only -- the same build that gives wrong results on the GPU (profiles/r06/hazards/)."""
import glob
import os
import re
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import isa_hazards  # noqa: E402

CSRC = os.path.join(REPO, "speaker_diarization_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
needs_llvm = pytest.mark.skipif(not os.path.exists(os.path.join(isa_hazards.LLVM, "llvm-objdump")),
                                reason="ROCm LLVM tools absent")


@needs_llvm
def test_built_objects_have_no_early_mfma_result_reads():
    objs = sorted(glob.glob(os.path.join(REPO, "speaker_diarization_amd", "lib", "obj", "*.hip.*.o")))
    if not objs:
        pytest.skip("library not built")
    found = []
    for o in objs:
        for name, ins, labels in isa_hazards.parse(isa_hazards.disassemble(o)):
            found += isa_hazards.check_function(name, ins, labels)
    assert not found, found[:5]


@needs_llvm
@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc absent")
def test_checker_finds_the_round5_branch_pattern(tmp_path):
    src = open(os.path.join(CSRC, "mha_block.hip")).read()
    bad = src.replace("if (W == 4 || ntile > 2) acc[2]", "if (ntile > 2) acc[2]")
    assert bad != src, "mha_block.hip no longer holds the guarded third-tile MFMA this test rewrites"
    for h in glob.glob(os.path.join(CSRC, "*.h")):
        shutil.copy(h, tmp_path)
    p = tmp_path / "mha_block.hip"
    p.write_text(bad)
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics"]
    obj = str(tmp_path / "mha_block.o")
    r = subprocess.run([HIPCC, *flags, "-x", "hip", "-c", str(p), "-o", obj], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    found = []
    for name, ins, labels in isa_hazards.parse(isa_hazards.disassemble(obj)):
        found += isa_hazards.check_function(name, ins, labels)
    assert found, "the branch-guarded MFMA no longer produces an early read (compiler changed?)"
    # every hazard sits in a 4-wave layout (mha_block_kernel<SEQ, 4, ...>), none in the 8-wave ones
    assert all(re.search(r"mha_block_kernelILi\d+ELi4E", f[0]) for f in found), {f[0] for f in found}
    # and it is the taken-edge read the round-5 schedule had: an AGPR read a few wait states after the MFMA
    assert any(f[5] == "v_accvgpr_read_b32" and f[7] <= 2 for f in found)


def test_checker_flags_write_after_write_and_taken_edges():
    """Synthetic instruction lists: a VALU overwrite of an MFMA destination inside its window is reported (the
    MFMA's later write-back would clobber it), a far one is not, and a read on a branch target is followed."""
    mf = ("v_mfma_f32_16x16x32_bf16", "v[0:3], v[4:7], v[8:11], v[0:3]")
    waw = [mf, ("v_mov_b32_e32", "v2, 0xff800000"), ("s_endpgm", "")]
    assert isa_hazards.check_function("waw", waw, {})
    late = [mf, ("s_nop", "7"), ("v_mov_b32_e32", "v2, 0xff800000"), ("s_endpgm", "")]
    assert not isa_hazards.check_function("late", late, {})
    taken = [mf, ("s_cbranch_vccnz", "L1"), ("s_nop", "7"), ("s_endpgm", ""), ("v_add_f32_e32", "v12, v3, v3"),
             ("s_endpgm", "")]
    assert isa_hazards.check_function("taken", taken, {"L1": 4})
