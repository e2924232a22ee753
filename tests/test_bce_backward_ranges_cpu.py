"""Host check of the gather ranges catseg_bce_onehot_loss_backward walks (evaluate.hip
bce_first_src / bce_lin): for every logit index j, the loop's start index lies at or below the
first target index whose bilinear taps (align_corners=False, F.interpolate's source-index rule)
reach j, and the contributing targets form one contiguous run -- so the gather sees every
contribution the scatter form (torch's interpolate backward) would add.  fp32 arithmetic as on
the device."""
import numpy as np
import pytest

f32 = np.float32


def lin(dst, in_size, scale):
    src = max(f32(scale) * (f32(dst) + f32(0.5)) - f32(0.5), f32(0))
    i0 = int(src)
    i1 = i0 + (1 if i0 < in_size - 1 else 0)
    return i0, i1, f32(src - f32(i0))


def first_src(j, in_size, out_size):
    s = int(np.floor((f32(j) - f32(1.5)) * f32(out_size) / f32(in_size))) - 2
    return max(s, 0)


@pytest.mark.parametrize("n_in,n_out", [(24, 96), (24, 50), (24, 37), (96, 384), (96, 512), (17, 17), (40, 20),
                                        (30, 45), (96, 640), (7, 1000), (100, 33)])
def test_gather_ranges_cover_every_tap(n_in, n_out):
    scale = f32(n_in) / f32(n_out)
    taps = [lin(x, n_in, scale) for x in range(n_out)]
    for j in range(n_in):
        contrib = [x for x, (i0, i1, _) in enumerate(taps) if i0 == j or i1 == j]
        if not contrib:
            continue
        assert first_src(j, n_in, n_out) <= contrib[0]
        assert contrib == list(range(contrib[0], contrib[-1] + 1))
        # the loop's stop rule (x0 > j) is never hit before the last contributor
        assert all(taps[x][0] <= j for x in contrib)
    # every target's weight lands on its taps: total weight per target is 1
    for i0, i1, l1 in taps:
        w = {}
        w[i0] = w.get(i0, 0) + (1 - l1)
        w[i1] = w.get(i1, 0) + l1
        assert abs(sum(w.values()) - 1) < 1e-6
