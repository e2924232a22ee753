"""Fit the segment table of the persistent MLP's GELU (rowpersist.hip gelu_seg): Phi(x) = 0.5 (1 + erf(x / sqrt 2))
on [-R, R] as NSEG cubics in the in-segment position f in [0, 1) (u = (x + R) NSEG / 2R, segment floor(u),
f = fract(u)); GELU(x) = x * P_seg(f), x clamped to the table's range for the segment choice only.
Prints the coefficient table (c0, c1, c2, c3 per segment, P = c0 + f (c1 + f (c2 + f c3))) and the
max |GELU error| over a dense grid, evaluated in fp32 the way the kernel does.
usage: python tools/gelu_table_fit.py"""
import math
import numpy as np

R, NSEG = 5.0, 32


def phi(x):
    return 0.5 * (1.0 + np.vectorize(math.erf)(x / math.sqrt(2.0)))


def fit():
    h = 2 * R / NSEG
    tab = []
    for k in range(NSEG):
        f = 0.5 - 0.5 * np.cos(np.linspace(0, np.pi, 400))        # Chebyshev-spaced in [0, 1]
        y = phi(-R + (k + f) * h)
        A = np.stack([f ** p for p in range(4)], 1)
        c = np.linalg.lstsq(A, y, rcond=None)[0]
        tab.append(c.astype(np.float32))
    return np.array(tab, np.float32)


def gelu_fp32(x, tab):
    x = x.astype(np.float32)
    S, O = np.float32(NSEG / (2 * R)), np.float32(NSEG / 2)
    u = np.clip(x * S + O, np.float32(0), np.float32(NSEG) - np.float32(2 ** -18)).astype(np.float32)
    i = np.floor(u).astype(np.int64)
    f = (u - np.floor(u)).astype(np.float32)
    c = tab[i]
    p = c[:, 3] * f + c[:, 2]
    p = (p * f + c[:, 1]).astype(np.float32)
    p = (p * f + c[:, 0]).astype(np.float32)
    return x * p


if __name__ == "__main__":
    tab = fit()
    x = np.linspace(-12, 12, 400001)
    ex = x * phi(x)
    err = np.abs(gelu_fp32(x, tab).astype(np.float64) - ex)
    print(f"// R = {R}, {NSEG} cubic segments: max |GELU error| {err.max():.3e} on [-12, 12] "
          f"({err[np.abs(x) <= 4].max():.3e} on [-4, 4])")
    for k, c in enumerate(tab):
        print("    {" + ", ".join(f"{v:.9e}f" for v in c) + "},")
