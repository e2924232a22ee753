"""ISA lint of the shipped gfx950 code objects (tools/isa_lint.py).

CPU-only: the objects the library is linked from (build/csrc/*.o, brought up to date by make)
are unbundled and disassembled here, and the MFMA operand / opaque LDS-DMA rules are asserted
over every kernel.  The assembler facts the rules rest on are pinned with llvm-mc."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_lint as I  # noqa: E402

LLVM_MC = os.path.join(I.LLVM, "llvm-mc")
pytestmark = pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="ROCm LLVM tools not installed")


@pytest.fixture(scope="module")
def linted():
    subprocess.run(["make", "-C", os.path.join(ROOT, "cat-seg_amd", "csrc"), "-j8", "-s"], check=True,
                   capture_output=True)
    objs = I.default_objects()
    assert len(objs) >= 14, objs
    return I.lint(objs)


def _assemble(src: str, tmp_path):
    s = tmp_path / "t.s"
    s.write_text(src)
    return subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-filetype=obj", str(s), "-o",
                           str(tmp_path / "t.o")], capture_output=True, text=True)


def test_assembler_overlap_rule(tmp_path):
    """LLVM's gfx950 rule (AMDGPUAsmParser): a destination wider than 4 VGPRs must not partially
    overlap srcC; 16x16 (4-VGPR) destinations may overlap any source partially."""
    ok = _assemble("v_mfma_f32_16x16x32_bf16 v[28:31], v[4:7], v[26:29], v[30:33]\n"
                   "v_mfma_f32_16x16x16_bf16 v[74:77], v[76:77], v[66:67], v[82:85]\n", tmp_path)
    assert ok.returncode == 0, ok.stderr
    bad = _assemble("v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[8:23]\n", tmp_path)
    assert bad.returncode != 0 and "must not partially overlap with dst" in bad.stderr


def test_lint_rules_fire(tmp_path):
    """The lint flags what it claims to (so a clean run is not vacuous)."""
    r = _assemble("v_mfma_f32_16x16x16_bf16 v[0:3], v[4:5], v[6:7], v[8:11]\n"
                  "v_mfma_f32_32x32x16_bf16 v[0:15], v[12:15], v[20:23], v[32:47]\n"
                  "s_endpgm\n", tmp_path)
    assert r.returncode == 0, r.stderr
    text = subprocess.run([os.path.join(I.LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", str(tmp_path / "t.o")],
                          capture_output=True, text=True, check=True).stdout
    funcs = I.parse(text)
    assert funcs and sum(len(f.insns) for f in funcs) == 3
    found = [x for f in funcs for x in I.check_mfma(f)[0]]
    assert {x.rule for x in found} == {"R1", "R2"}
    # R3 on a synthetic stream: a DMA, 2 stores, a loop back-edge to a vmcnt(3) wait
    f = I.Func("swin_win5_kernel_synthetic", [
        I.Insn(0, "s_waitcnt", "vmcnt(3)"),
        I.Insn(4, "s_mov_b32", "m0, s4"), I.Insn(8, "s_nop", "0"), I.Insn(12, "global_load_lds_dwordx4", "v[2:3], off"),
        I.Insn(20, "global_store_dwordx2", "v[0:1], v[4:5], off"),
        I.Insn(28, "global_store_dwordx2", "v[0:1], v[6:7], off"),
        I.Insn(36, "s_cbranch_scc1", "", target=0),
        I.Insn(40, "s_endpgm", "")])
    bad = I.check_dma(f, (3,))[0]
    assert len(bad) == 1 and "only 2 younger" in bad[0].text
    f.insns.insert(6, I.Insn(32, "global_store_dwordx2", "v[0:1], v[8:9], off"))
    assert I.check_dma(f, (3,))[0] == []


def test_shipped_kernels_have_no_k16_mfma(linted):
    findings, report = linted
    assert sum(s["mfma"] for s in report.values()) > 10000
    r1 = [str(x) for x in findings if x.rule == "R1"]
    assert not r1, "\n".join(r1[:20])


def test_shipped_kernels_no_wide_partial_overlap(linted):
    findings, _ = linted
    r2 = [str(x) for x in findings if x.rule == "R2"]
    assert not r2, "\n".join(r2[:20])


def test_swin_opaque_dma_counted_waits(linted):
    """swin_win5 (default) and swin_win3 retire the window's LDS-DMA with a counted vmcnt: every
    path from a DMA to that wait carries at least that many younger vector-memory instructions, and
    M0 is touched only by the DMA asm."""
    findings, report = linted
    r3 = [str(x) for x in findings if x.rule == "R3"]
    assert not r3, "\n".join(r3[:20])
    win5 = {k: v for k, v in report.items() if "swin_win5_kernel" in k}
    assert len(win5) == 4          # shifted / unshifted, plain / write-through output stores
    for k, v in win5.items():
        assert v["opaque_dma"] >= 1 and v["counted_waits"] == 1, (k, v)
        assert v["min_younger_vmem"] >= 18, (k, v)

