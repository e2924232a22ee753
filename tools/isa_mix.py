"""Static instruction mix of the gfx950 kernels in a built object: per kernel and per loop body
(the instructions between a backward branch's target and the branch), counted by class.

usage: python tools/isa_mix.py <object under build/csrc, e.g. conv_ring> [kernel-name substring]
"""
import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_lint as I  # noqa: E402


def klass(op):
    if op.startswith("v_mfma") or op.startswith("v_smfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    obj = sys.argv[1]
    if not obj.endswith(".o"):
        obj = os.path.join(I.ROOT, "build", "csrc", obj + ".o")
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as td:
        text = I.disassemble(obj, td)
    funcs, cur = [], None
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <([^>]+)>:$", line)
        if m:
            cur = [m.group(2), []]
            funcs.append(cur)
            continue
        m = re.match(r"^\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$", line)
        if m and cur is not None:
            cur[1].append((int(m.group(3), 16), m.group(1), m.group(2) + " " + m.group(4)))
    for name, ins in funcs:
        if sub not in name or not ins:
            continue
        tot = {}
        for _, op, _ in ins:
            tot[klass(op)] = tot.get(klass(op), 0) + 1
        print(f"== {name[:150]}\n   total {tot}")
        addr = {a: i for i, (a, _, _) in enumerate(ins)}
        for i, (a, op, args) in enumerate(ins):
            if not op.startswith("s_cbranch") and op != "s_branch":
                continue
            m = re.search(r"<[^>+]+\+0x([0-9a-f]+)>", args)
            if not m:
                continue
            tgt = ins[0][0] + int(m.group(1), 16)
            j = addr.get(tgt)
            if j is None or j > i:
                continue
            body = {}
            for _, op2, _ in ins[j:i + 1]:
                body[klass(op2)] = body.get(klass(op2), 0) + 1
            mf = body.get("mfma", 0)
            ratio = f"  valu/mfma {body.get('valu', 0) / mf:.2f}" if mf else ""
            print(f"   loop [{j}:{i}] {i - j + 1} insns {body}{ratio}")


if __name__ == "__main__":
    main()
