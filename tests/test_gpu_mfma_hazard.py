"""The gfx950 MFMA operand cases the shipped kernels rely on, on the device:
tools/probe_mfma_overlap.hip (built by `make -C cat-seg_amd/csrc probe`, which __graft_entry__.build() runs) compares every case with the same
products on disjoint, generously padded registers, bit for bit, alone and beside partner waves that
saturate the matrix pipe.  Every K=32 case -- destination partially over srcA / srcB / srcC, the
chained-srcC LDS write-after-read pattern -- and the K=16 cases without a pending srcC dependency must
match exactly; the K=16 chained-srcC case (the defect behind the round-2/3 wrong tiles, which is why no
kernel issues the K=16 form: tools/isa_lint.py R1) is reported, not asserted."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
PROBE = os.path.join(ROOT, "tools", "bin", "probe_mfma_overlap")


def test_mfma_operand_cases_the_kernels_use():
    if not os.path.exists(PROBE):
        pytest.fail("tools/bin/probe_mfma_overlap missing: build with make -C cat-seg_amd/csrc probe")
    out = subprocess.run([PROBE, "4"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = re.findall(r"^(plain|hammer)\s+(.+?)\s+mismatching words (\d+) of (\d+)$", out.stdout, re.M)
    assert len(rows) == 36, out.stdout
    for mode, case, bad, total in rows:
        assert int(total) > 0, (mode, case)
        if case.startswith("k16 chained"):
            print(f"{mode} {case}: {bad} of {total} words wrong (known K=16 hazard)")
            continue
        assert int(bad) == 0, f"{mode} {case}: {bad} of {total} words differ"
