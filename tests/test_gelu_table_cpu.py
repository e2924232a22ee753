"""The persistent MLPs' segment-table GELU (rowpersist.hip kGeluSeg / gelu_seg): the
table in the source is the one tools/gelu_table_fit.py fits, and evaluated in fp32 the way the
kernel does (segment from fma + clamp, fract, cubic by Horner, times x) it stays within 5e-6 of the
exact erf GELU, against 3.0e-5 for the degree-8 polynomial it replaced."""
import math
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gelu_table_fit as G  # noqa: E402


def source_table():
    src = open(os.path.join(ROOT, "cat-seg_amd", "csrc", "rowpersist.hip")).read()
    body = src[src.index("kGeluSeg[GSEG][4] = {"):]
    body = body[:body.index("};")]
    rows = re.findall(r"\{([^{}]+)\}", body)
    return np.array([[float(v.strip().rstrip("f")) for v in r.split(",")] for r in rows], np.float32)


def test_source_table_is_the_fit():
    tab = source_table()
    assert tab.shape == (G.NSEG, 4)
    np.testing.assert_array_equal(tab, G.fit())


def test_gelu_table_error():
    tab = source_table()
    x = np.linspace(-12, 12, 200001)
    exact = x * 0.5 * (1 + np.vectorize(math.erf)(x / math.sqrt(2)))
    err = np.abs(G.gelu_fp32(x, tab).astype(np.float64) - exact)
    assert err.max() < 5e-6, err.max()
    # saturation: far left ~0, far right ~x
    assert abs(G.gelu_fp32(np.array([-40.0]), tab)[0]) < 1e-4
    assert abs(G.gelu_fp32(np.array([40.0]), tab)[0] - 40.0) < 1e-4
