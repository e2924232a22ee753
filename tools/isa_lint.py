"""ISA lint over the shipped gfx950 code objects (build/csrc/*.o -> libcatseg_hip.so).

Why: two hand-written kernels returned intermittently wrong tiles on the box while every
instruction they issue is legal to the assembler.  The rules below are the
properties those investigations rest on; they are checked on the disassembly of the objects the
library is linked from, so a source edit or a compiler update that breaks one fails a CPU test
instead of a GPU run.

  R1  no K=16 bf16/f16 MFMA (`v_mfma_f32_16x16x16_{bf16,f16}`, `v_mfma_f32_32x32x8_{bf16,f16}`)
      in any kernel: the instruction form behind both observed wrong-output defects (§8).
  R2  no MFMA whose destination PARTIALLY overlaps one of its sources when the destination is
      wider than 4 VGPRs (the assembler's own rule, `source 2 operand must not partially overlap
      with dst`, extended to srcA / srcB).  16x16 destinations (4 VGPRs) may overlap a source
      partially: LLVM accepts it and the shipped K=32 kernels rely on it (§8).
  R3  opaque LDS-DMA (inline-asm `s_mov_b32 m0` / `global_load_lds_dwordx4`, invisible to the
      compiler's waitcnt pass): M0 is written only by that asm and read only by its DMA, and each
      hand-counted `s_waitcnt vmcnt(N)` the kernel relies on is reached from every DMA only along
      paths that issue >= N younger vector-memory instructions (or pass a vmcnt(0)), so the wait
      retires every DMA.  Control-flow aware: basic blocks from the branch targets.

Usage: python tools/isa_lint.py [objects...]   (default build/csrc/*.o); exits 1 on a violation.
"""
from __future__ import annotations

import glob
import os
import re
import subprocess
import sys
import tempfile
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

K16_MFMA = re.compile(r"^v_mfma_f32_(16x16x16|32x32x8)_(bf16|f16)$")
VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")


@dataclass
class Insn:
    addr: int
    op: str
    args: str
    target: Optional[int] = None      # branch target address


@dataclass
class Func:
    name: str
    insns: List[Insn] = field(default_factory=list)


def _run(cmd: List[str]) -> str:
    return subprocess.run(cmd, check=True, capture_output=True, text=True).stdout


def disassemble(obj: str, tmpdir: str) -> str:
    """gfx950 disassembly of the device code object bundled in a host object file."""
    base = os.path.join(tmpdir, os.path.basename(obj))
    if ".hip_fatbin" not in _run([f"{LLVM}/llvm-readelf", "-S", "-W", obj]):
        return ""                    # host-only object (no kernels)
    _run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={base}.fatbin", obj, f"{base}.tmp"])
    _run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
          f"--input={base}.fatbin", f"--output={base}.co"])
    return _run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f"{base}.co"])


_FUNC = re.compile(r"^([0-9a-f]+) <([^>]+)>:$")
_INSN = re.compile(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_TGT = re.compile(r"<([^>+]+)\+0x([0-9a-f]+)>\s*$")


def parse(text: str) -> List[Func]:
    funcs: List[Func] = []
    bases: Dict[str, int] = {}
    cur: Optional[Func] = None
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = Func(m.group(2))
            bases[cur.name] = int(m.group(1), 16)
            funcs.append(cur)
            continue
        if cur is None:
            continue
        m = _INSN.match(line)
        if not m:
            continue
        ins = Insn(int(m.group(3), 16), m.group(1), m.group(2))
        if ins.op.startswith(("s_branch", "s_cbranch")):
            t = _TGT.search(line)
            if t and t.group(1) in bases:
                ins.target = bases[t.group(1)] + int(t.group(2), 16)
        cur.insns.append(ins)
    return funcs


# ---------------------------------------------------------------- registers
_VR = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+))")


def regs(operand: str) -> Tuple[str, int, int]:
    """('v'|'a', first, last) of a VGPR / AGPR operand; ('', 0, -1) otherwise."""
    m = _VR.match(operand.strip())
    if not m:
        return "", 0, -1
    if m.group(4) is not None:
        n = int(m.group(4))
        return m.group(1), n, n
    return m.group(1), int(m.group(2)), int(m.group(3))


def split_operands(args: str) -> List[str]:
    return [a.strip() for a in args.split(",")]


def partial_overlap(a: Tuple[str, int, int], b: Tuple[str, int, int]) -> bool:
    if not a[0] or a[0] != b[0]:
        return False
    lo, hi = max(a[1], b[1]), min(a[2], b[2])
    return lo <= hi and (a[1], a[2]) != (b[1], b[2])


@dataclass
class Finding:
    rule: str
    func: str
    addr: int
    text: str

    def __str__(self):
        return f"{self.rule} {self.func} @0x{self.addr:x}: {self.text}"


def check_mfma(f: Func) -> Tuple[List[Finding], Dict[str, int]]:
    """R1 + R2; also counts the 4-VGPR partial overlaps R2 admits (reported, not findings)."""
    out: List[Finding] = []
    stats = {"mfma": 0, "dst4_partial_srcA": 0, "dst4_partial_srcB": 0, "dst4_partial_srcC": 0}
    for ins in f.insns:
        if not ins.op.startswith("v_mfma"):
            continue
        stats["mfma"] += 1
        if K16_MFMA.match(ins.op):
            out.append(Finding("R1", f.name, ins.addr, f"{ins.op} {ins.args}"))
        ops = split_operands(ins.args)
        dst = regs(ops[0])
        width = dst[2] - dst[1] + 1
        for name, o in zip(("srcA", "srcB", "srcC"), ops[1:4]):
            if partial_overlap(dst, regs(o)):
                if width > 4:
                    out.append(Finding("R2", f.name, ins.addr, f"{ins.op} {ins.args} (dst partially overlaps {name})"))
                else:
                    stats[f"dst4_partial_{name}"] += 1
    return out, stats


# ---------------------------------------------------------------- R3: opaque LDS-DMA
def is_opaque_dma(insns: List[Insn], i: int) -> bool:
    """The inline-asm DMA signature: s_mov_b32 m0, sN ; s_nop 0 ; global_load_lds_dwordx4."""
    return (insns[i].op == "global_load_lds_dwordx4" and i >= 2 and insns[i - 1].op == "s_nop"
            and insns[i - 1].args == "0" and insns[i - 2].op == "s_mov_b32" and insns[i - 2].args.startswith("m0,"))


def _vmcnt(ins: Insn) -> Optional[int]:
    if ins.op != "s_waitcnt":
        return None
    m = re.search(r"vmcnt\((\d+)\)", ins.args)
    return int(m.group(1)) if m else None


def _blocks(f: Func):
    """Basic blocks: start index list and successor lists (by instruction index)."""
    idx = {ins.addr: i for i, ins in enumerate(f.insns)}
    starts = {0}
    for i, ins in enumerate(f.insns):
        if ins.target is not None:
            if ins.target in idx:
                starts.add(idx[ins.target])
            if i + 1 < len(f.insns):
                starts.add(i + 1)
        elif ins.op in ("s_endpgm", "s_setpc_b64") and i + 1 < len(f.insns):
            starts.add(i + 1)
    order = sorted(starts)
    end_of = {s: (order[k + 1] if k + 1 < len(order) else len(f.insns)) for k, s in enumerate(order)}
    succ: Dict[int, List[int]] = {}
    for s in order:
        last = f.insns[end_of[s] - 1]
        nxt: List[int] = []
        if last.target is not None and last.target in idx:
            nxt.append(idx[last.target])
        if last.op != "s_branch" and last.op not in ("s_endpgm", "s_setpc_b64") and end_of[s] < len(f.insns):
            nxt.append(end_of[s])
        succ[s] = nxt
    return order, end_of, succ


def min_vmem_before(f: Func, wait_i: int, cap: int) -> Tuple[Optional[int], Optional[int]]:
    """Fewest vector-memory instructions issued between an opaque DMA and instruction `wait_i`
    over every CFG path from the DMA to it that does not pass a vmcnt(0) wait (capped at `cap`).
    Returns (count, dma_index) of the worst path, or (None, None) if no DMA reaches the wait."""
    order, end_of, succ = _blocks(f)
    pred: Dict[int, List[int]] = {s: [] for s in order}
    for s, ns in succ.items():
        for n in ns:
            pred[n].append(s)
    block_of = {}
    for s in order:
        for i in range(s, end_of[s]):
            block_of[i] = s
    insns = f.insns
    worst: Tuple[Optional[int], Optional[int]] = (None, None)
    # walk backwards from the wait: state = (VMEM ops between the position and the wait, block,
    # last instruction index still to inspect in that block)
    import heapq
    s0 = block_of[wait_i]
    heap = [(0, s0, wait_i - 1)]
    seen: Dict[Tuple[int, int], int] = {}
    while heap:
        cnt, s, i = heapq.heappop(heap)
        if cnt >= cap or seen.get((s, i), cap + 1) <= cnt:
            continue
        seen[(s, i)] = cnt
        stopped = False
        j = i
        while j >= s:
            ins = insns[j]
            if _vmcnt(ins) == 0:
                stopped = True
                break
            if is_opaque_dma(insns, j):
                # the youngest DMA on this path: every older one has more VMEM ops behind it
                if worst[0] is None or cnt < worst[0]:
                    worst = (cnt, j)
                stopped = True
                break
            if VMEM.match(ins.op):
                cnt += 1
                if cnt >= cap:
                    stopped = True
                    break
            j -= 1
        if stopped:
            continue
        for p in pred[s]:
            heapq.heappush(heap, (cnt, p, end_of[p] - 1))
    return worst


def check_dma(f: Func, counted: Iterable[int]) -> Tuple[List[Finding], Dict[str, int]]:
    out: List[Finding] = []
    insns = f.insns
    if not counted:               # only the kernels whose source issues the DMA from inline asm
        return out, {"opaque_dma": 0, "counted_waits": 0}
    dmas = [i for i in range(len(insns)) if is_opaque_dma(insns, i)]
    stats = {"opaque_dma": len(dmas), "counted_waits": 0}
    if not dmas:
        return out, stats
    dma_m0 = {i - 2 for i in dmas}
    for i, ins in enumerate(insns):
        if "m0" in re.split(r"[\s,]+", ins.args) and i not in dma_m0:
            out.append(Finding("R3", f.name, ins.addr, f"M0 used outside the DMA asm: {ins.op} {ins.args}"))
    for i, ins in enumerate(insns):
        v = _vmcnt(ins)
        if v is None or v == 0 or v not in counted:
            continue
        stats["counted_waits"] += 1
        cnt, d = min_vmem_before(f, i, v + 64)
        if cnt is not None:
            stats["min_younger_vmem"] = min(stats.get("min_younger_vmem", 1 << 30), cnt)
        if cnt is not None and cnt < v:
            out.append(Finding("R3", f.name, ins.addr,
                               f"s_waitcnt vmcnt({v}) is reached from the DMA @0x{insns[d].addr:x} "
                               f"with only {cnt} younger vector-memory instructions"))
    return out, stats


# counted waits each opaque-DMA kernel relies on (swin_window.hip): the window-start wait
COUNTED = {"swin_win5_kernel": (18,), "swin_win3_kernel": (8,)}


def lint(objs: List[str]):
    findings: List[Finding] = []
    report: Dict[str, Dict[str, int]] = {}
    with tempfile.TemporaryDirectory() as td:
        for obj in objs:
            for f in parse(disassemble(obj, td)):
                fl, st = check_mfma(f)
                counted = next((v for k, v in COUNTED.items() if k in f.name), ())
                dl, ds = check_dma(f, counted)
                findings += fl + dl
                report[f"{os.path.basename(obj)}:{f.name}"] = {**st, **ds}
    return findings, report


def default_objects() -> List[str]:
    return sorted(glob.glob(os.path.join(ROOT, "build", "csrc", "*.o")))


if __name__ == "__main__":
    objs = sys.argv[1:] or default_objects()
    if not objs:
        raise SystemExit("no objects (build first: make -C cat-seg_amd/csrc)")
    findings, report = lint(objs)
    tot = {}
    for st in report.values():
        for k, v in st.items():
            tot[k] = tot.get(k, 0) + v
    print(f"{len(report)} functions, totals: {tot}")
    for f in findings:
        print(f)
    sys.exit(1 if findings else 0)
