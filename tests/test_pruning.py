"""CPU checks of the exactness arguments behind build_grid's candidate lists
(hq_search.hip), restated in numpy float32 with the kernel's expression order:

- the box-bound candidate test dmin^2(B, k) <= T(B) (1 + 1e-5), T = min_j dmax^2;
- the dominance pruning: a is dropped when f_min = min over the box of
  |p - a|^2 - |p - b*|^2 exceeds 1e-5 (dmax^2(B, a) + S);
- for lists still longer than an 8-B level-2 entry holds (7), the same test
  against every other listed colour (build_grid's prune_long_lists).

Each is checked against the reference's own argmin (CL:179-192: its distance
as compiled for gfx950, oracle.ref_len; first minimum in ascending index) over dense pixel sets
inside the box -- every u8/255 value of the box, its corners and faces, and
points one ulp inside -- for random and adversarial palettes: a colour the
tests drop never wins, ties included.  No GPU needed.
"""

import numpy as np

import oracle as o

f32 = np.float32


def ax_min2(c, lo, hi):
    d = np.maximum(np.maximum(f32(lo - c), f32(c - hi)), f32(0))
    return f32(d * d)


def ax_max2(c, lo, hi):
    d = np.maximum(f32(c - lo), f32(hi - c))
    return f32(d * d)


def box_bounds(pal, lo, hi):
    dmin = f32(f32(ax_min2(pal[:, 0], lo[0], hi[0]) + ax_min2(pal[:, 1], lo[1], hi[1])) +
               ax_min2(pal[:, 2], lo[2], hi[2]))
    dmax = f32(f32(ax_max2(pal[:, 0], lo[0], hi[0]) + ax_max2(pal[:, 1], lo[1], hi[1])) +
               ax_max2(pal[:, 2], lo[2], hi[2]))
    return dmin, dmax


def dominated(a, b, lo, hi):
    """prune_dominated's test, one (a, b) pair, float32 like the kernel."""
    dmax2a = f32(f32(ax_max2(a[0], lo[0], hi[0]) + ax_max2(a[1], lo[1], hi[1])) + ax_max2(a[2], lo[2], hi[2]))
    na = f32(f32(a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])
    nb = f32(f32(b[0] * b[0] + b[1] * b[1]) + b[2] * b[2])
    fmin = f32(na - nb)
    S = f32(f32(na + nb) + dmax2a)
    for ax in range(3):
        cc = f32(f32(2) * f32(b[ax] - a[ax]))
        tl, th = f32(cc * lo[ax]), f32(cc * hi[ax])
        fmin = f32(fmin + min(tl, th))
        S = f32(S + max(abs(tl), abs(th)))
    return fmin > f32(1e-5) * S


def box_pixels(lo, hi, rng):
    """u8/255 values inside the box per axis, the faces and one ulp inside, all combinations
    (capped), plus random floats."""
    axes = []
    for a in range(3):
        u8 = np.arange(256, dtype=np.float32) / f32(255)
        v = u8[(u8 >= lo[a]) & (u8 <= hi[a])]
        extra = np.array([lo[a], hi[a], np.nextafter(f32(lo[a]), f32(2)), np.nextafter(f32(hi[a]), f32(-1))],
                         np.float32)
        axes.append(np.unique(np.concatenate([v, extra])))
    g = np.stack(np.meshgrid(*axes, indexing="ij"), -1).reshape(-1, 3)
    r = lo + (hi - lo) * rng.random((2000, 3), dtype=np.float32)
    return np.concatenate([g, r.astype(np.float32)])


def ref_argmin(px, pal):
    """CL:179-192 over all colours: the reference's distance on gfx950
    (oracle.ref_len: fma-chain d^2, its square root), first minimum."""
    return o.assign(px, pal)[0]


def check_palette(pal, G2, rng, cells=60, long_cap=7):
    pal = pal.astype(np.float32)
    inv = f32(1) / f32(G2)
    kept_total = dropped_total = 0
    for _ in range(cells):
        c = rng.integers(0, G2, 3)
        lo = (c * inv).astype(np.float32)
        hi = ((c + 1) * inv).astype(np.float32)
        dmin, dmax = box_bounds(pal, lo, hi)
        T = dmax.min()
        cand = np.nonzero(dmin <= T * f32(1 + 1e-5))[0]
        bstar = cand[np.argmin(dmax[cand])]
        keep = [k for k in cand if k == bstar or not dominated(pal[k], pal[bstar], lo, hi)]
        if len(keep) > long_cap:  # build_grid's second pass (prune_long_lists): every pair
            keep = [k for k in keep if not any(j != k and dominated(pal[k], pal[j], lo, hi) for j in keep)]
        kept_total += len(keep)
        dropped_total += len(cand) - len(keep)
        win = np.unique(ref_argmin(box_pixels(lo, hi, rng), pal))
        assert set(win) <= set(keep), (lo, hi, set(win) - set(keep))
    return kept_total, dropped_total


def test_pruning_never_drops_a_winner_random():
    rng = np.random.default_rng(5)
    dropped = 0
    for G2 in (16, 32, 64):
        pal = o.synthetic_palette(256, 11 + G2)[:, :3]
        kept, d = check_palette(pal, G2, rng)
        dropped += d
    assert dropped > 0  # the test does prune on random palettes


def test_pairwise_pruning_of_long_lists_never_drops_a_winner():
    """The pairwise pass on every list (long_cap 0), clustered palettes whose
    cells list many colours: a colour dominated by any listed colour never wins."""
    rng = np.random.default_rng(21)
    for G2 in (16, 32):
        centres = rng.random((8, 3), dtype=np.float32)
        pal = (centres[rng.integers(0, 8, 256)] + rng.normal(0, 0.03, (256, 3))).astype(np.float32)
        pal = np.clip(pal, 0, 1)
        kept, dropped = check_palette(pal, G2, rng, cells=40, long_cap=0)
        assert dropped > 0


def test_pruning_never_drops_a_winner_adversarial():
    """Colours mirrored across cell faces (exact ties on the face), colours one
    ulp apart, colours on corners."""
    rng = np.random.default_rng(8)
    for G2 in (16, 32):
        faces = (np.arange(G2 + 1) / G2).astype(np.float32)
        pal = np.zeros((256, 3), np.float32)
        for i in range(128):
            ax = i % 3
            f = faces[rng.integers(1, G2)]
            d = np.float32(rng.integers(1, 8)) / np.float32(4 * G2)
            base = rng.choice(faces, 3)
            a, b = base.copy(), base.copy()
            a[ax], b[ax] = f - d, f + d
            pal[2 * i], pal[2 * i + 1] = np.clip(a, 0, 1), np.clip(b, 0, 1)
        pal[200:220] = np.nextafter(pal[0:20], np.float32(2))
        check_palette(pal, G2, rng, cells=80)
