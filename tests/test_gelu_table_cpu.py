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


# ---- the 7-VALU form (rowpersist.hip kGeluX7 / gelu_x7, the default gelu_form 1)
import gelu_x7_fit as G7  # noqa: E402


def source_table_x7():
    src = open(os.path.join(ROOT, "cat-seg_amd", "csrc", "rowpersist.hip")).read()
    body = src[src.index("kGeluX7[GSEG7][4] = {"):]
    body = body[:body.index("};")]
    rows = re.findall(r"\{([^{}]+)\}", body)
    return np.array([[float(v.strip().rstrip("f")) for v in r.split(",")] for r in rows], np.float32)


def test_x7_source_table_is_the_fit():
    tab = source_table_x7()
    assert tab.shape == (G7.NSEG, 4)
    np.testing.assert_array_equal(tab, G7.fit())


def test_x7_segment_from_fp32_bits():
    """The kernel's segment index: fma(x, 3.2, 2^23 + 16) in fp32 rounds to an integer whose bit pattern
    is 0x4B000000 + round(3.2 x + 16); med3 to [2^23, 2^23 + 32] clamps it (as np.float32 arithmetic)."""
    x = np.concatenate([np.linspace(-20, 20, 100001), [-1e30, 1e30, -5.15625, 5.15625, 0.0]]).astype(np.float32)
    t = (x.astype(np.float64) * np.float64(np.float32(3.2)) + 8388624.0).astype(np.float32)   # fma: one rounding
    t = np.clip(t, np.float32(8388608.0), np.float32(8388640.0))
    k = t.view(np.uint32).astype(np.int64) - 0x4B000000
    want = np.clip(np.round(x.astype(np.float64) * np.float64(np.float32(3.2)) + 16), 0, 32)
    assert k.min() >= 0 and k.max() <= 32
    # ties (exact .5 after the fma) may round either way: the neighbouring cubics agree there
    assert np.all((k == want) | (np.abs(x.astype(np.float64) * np.float64(np.float32(3.2)) + 16 - np.round(
        x.astype(np.float64) * np.float64(np.float32(3.2)) + 16)) > 0.49))


def test_x7_gelu_error():
    tab = source_table_x7()
    x = np.linspace(-12, 12, 200001)
    exact = x * 0.5 * (1 + np.vectorize(math.erf)(x / math.sqrt(2)))
    err = np.abs(G7.gelu_fp32(x, tab) - exact)
    assert err.max() < 4e-6, err.max()
    assert abs(G7.gelu_fp32(np.array([-40.0]), tab)[0]) < 1e-4
    assert abs(G7.gelu_fp32(np.array([40.0]), tab)[0] - 40.0) < 1e-4
