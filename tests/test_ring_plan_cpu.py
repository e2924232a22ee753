"""The decoder ring convs' pixel-granular ring plan (conv_ring.hip ring_plan_ok).

A chunk of CH output pixels needs input pixels up to the bottom-right neighbour of its last pixel;
the ring (NR row slots, row y in slot (y + 1) % NR) is filled CH pixels at a time, one chunk ahead.
The launch refuses a plan in which a written slot could alias a row still being read; this restates
that rule and checks it holds for every (width, chunk, ring) combination the dispatcher can pick,
and that it rejects an undersized ring."""


def ring_plan_ok(H, W, CH, NR, OB):
    n = H * W // CH
    for c in range(n):
        p0 = c * CH
        first = p0 // W - 1                       # top halo row of chunk c
        if (p0 + CH + W) // W - first + 1 > NR:   # the band prime's rows
            return False
        if c + 1 == n:
            break
        wr_last = (p0 + 2 * CH + W) // W          # row of the prefetch's last pixel
        oldest = first if OB else (p0 + CH) // W - 1
        if wr_last - oldest + 1 > NR:
            return False
    return True


def dispatched_plans(W):
    """(CH, NR, OB) of the conv3x3 ring variants ring_variant() can pick at width W (48 <= W <= 96)."""
    plans = [(128, 6 if W < 64 else 5, False)]
    if W == 96:
        plans.append((128, 7, True))
    if W <= 50:
        plans += [(128, 9, True), (128, 6, False), (64, 5, False)]
    return plans


def test_every_dispatched_plan_is_valid():
    for W in range(48, 97):
        for H in range(8, 160):
            if (H * W) % 128:
                continue
            for CH, NR, OB in dispatched_plans(W):
                if (H * W) % CH == 0:
                    assert ring_plan_ok(H, W, CH, NR, OB), (H, W, CH, NR, OB)


def test_upconv_plans_are_valid():
    # catseg_upconv3x3: 64-pixel chunks, Up2 at W = 48 (NR 7 one-barrier, 5 two-barrier), Up1 at W = 24 (9 / 6)
    for W, NR, OB in ((48, 7, True), (48, 5, False), (24, 9, True), (24, 6, False)):
        for H in range(4, 160):
            if (H * W) % 64 == 0:
                assert ring_plan_ok(H, W, 64, NR, OB), (H, W, NR, OB)


def test_undersized_rings_are_rejected():
    assert not ring_plan_ok(96, 96, 128, 5, True)      # one-barrier 96-wide: 6 rows suffice (7 ship), 5 do not
    assert not ring_plan_ok(48, 48, 128, 5, False)     # 48-wide 128-pixel chunks need 6
    assert not ring_plan_ok(24, 24, 64, 8, True)       # Up1's one-barrier ring needs 9
