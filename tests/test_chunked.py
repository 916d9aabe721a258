"""CPU check of the chunked argmin behind 256 < K <= 4096 (hq_assign.hip,
assign_pipe_kernel with CMB > 1; hq_runtime.hip pack_chunks):

a palette of K colours becomes nch = 2, 4, 8 or 16 sub-palettes of 256
(colours 256 c .. 256 c + 255; past K, copies of colour 0).  Each chunk's
winner is that chunk's own reference argmin (CL:179-193: the reference's
distance, oracle.ref_len; first minimum in ascending index), and the winners are compared in
ascending chunk order by the same distance with a strict <, nch / 4 chunks at a
time when nch > 4 (the passes keep the best distance so far).  The result must
be the reference argmin over all K colours, for palettes with exact ties across
chunks (duplicates, pixels equal to colours in two chunks, colours mirrored
about pixels) and padding.  Restated in numpy float32 with the oracle's
expression order; no GPU needed.
"""

import numpy as np
import pytest

import oracle as o

f32 = np.float32


def chunk_count(K):
    n = 1
    while 256 * n < K:
        n <<= 1
    return n


def chunked_argmin(px, pal):
    K = pal.shape[0]
    nch = chunk_count(K)
    padded = np.concatenate([pal, np.repeat(pal[:1], nch * 256 - K, axis=0)])  # pack_chunks
    win = []
    for c in range(nch):
        idx, _ = o.assign(px[:, :3], padded[256 * c:256 * (c + 1)])
        win.append(256 * c + idx)
    best = ref_dist_at(px, padded, win[0])
    out = win[0].copy()
    for c in range(1, nch):  # ascending chunks, strict <
        d = ref_dist_at(px, padded, win[c])
        lt = d < best
        best = np.where(lt, d, best)
        out = np.where(lt, win[c], out)
    return out


def ref_dist_at(px, pal, idx):
    """The reference's distance (CL:186 as compiled for gfx950: oracle.ref_len)."""
    d = (px[:, :3] - pal[idx, :3]).astype(f32)
    return o.ref_len(d[:, 0], d[:, 1], d[:, 2])


@pytest.mark.parametrize("K", [257, 300, 512, 600, 1000, 1500, 2048, 4096])
def test_chunked_argmin_equals_reference(K):
    rng = np.random.default_rng(K)
    n = 3000
    px = np.zeros((n, 4), f32)
    px[:, :3] = (rng.integers(0, 256, (n, 3)) / f32(255)).astype(f32)
    pal = o.synthetic_palette(K, 7 + K).copy()
    nch = chunk_count(K)
    # ties across chunks: exact duplicates at the same offset of every chunk
    for c in range(1, (K - 1) // 256 + 1):
        if 256 * c + 5 < K:
            pal[256 * c + 5] = pal[5]
    # pixels equal to a colour of chunk 0 and of the last real chunk
    last = ((K - 1) // 256) * 256
    pal[10, :3] = px[0, :3]
    pal[min(K - 1, last + 1), :3] = px[0, :3]
    pal[11, :3] = px[1, :3]
    pal[min(K - 1, last + 2), :3] = px[1, :3]
    # two colours mirrored about a pixel, in different chunks (equal distances)
    e = f32(3.0 / 255)
    pal[20, :3] = px[2, :3] + e
    pal[min(K - 1, 256 + 20), :3] = px[2, :3] - e
    # the padding colour (colour 0) nearest for some pixels
    px[3, :3] = pal[0, :3]
    ref, _ = o.assign(px[:, :3], pal)
    got = chunked_argmin(px, pal)
    assert nch >= 2
    np.testing.assert_array_equal(got, ref)
    assert (got < K).all()  # a padding colour never wins
