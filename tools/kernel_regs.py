"""VGPR count, spills and scratch of the gfx950 kernels in a built object (code-object metadata).
usage: python tools/kernel_regs.py <object under build/csrc, e.g. rowpersist> [kernel-name substring]"""
import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_lint as I  # noqa: E402

obj = sys.argv[1]
if not obj.endswith(".o"):
    obj = os.path.join(I.ROOT, "build", "csrc", obj + ".o")
sub = sys.argv[2] if len(sys.argv) > 2 else ""
with tempfile.TemporaryDirectory() as td:
    base = os.path.join(td, os.path.basename(obj))
    I._run([f"{I.LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={base}.fatbin", obj, f"{base}.tmp"])
    I._run([f"{I.LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={I.TARGET}",
            f"--input={base}.fatbin", f"--output={base}.co"])
    notes = I._run([f"{I.LLVM}/llvm-readelf", "--notes", f"{base}.co"])
cur = {}
rows = []
for line in notes.splitlines():
    m = re.match(r"\s+\.(name|vgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size|group_segment_fixed_size):\s+(\S+)", line)
    if not m:
        continue
    cur[m.group(1)] = m.group(2)
    if m.group(1) == "name":
        rows.append(cur)
for r in rows:
    pass
# metadata keys of one kernel precede or follow its name; regroup by scanning blocks
blocks = re.split(r"\n\s+- \.", notes)
for b in blocks:
    m = re.search(r"\.name:\s+(\S+)", b)
    if not m or sub not in m.group(1) or m.group(1).endswith(".kd"):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", b) or [None, "?"])[1]
    print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>3} vspill {g('vgpr_spill_count'):>3} "
          f"scratch {g('private_segment_fixed_size'):>4} lds {g('group_segment_fixed_size'):>6}  {m.group(1)[:110]}")
