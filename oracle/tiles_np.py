"""numpy restatement of the image-tile layout (TEST INFRASTRUCTURE ONLY):
rank r owns tiles t = r, r+P, ...; its slab holds them in that order as
16x16 row-major pixel blocks (librtamd k_trace PACKED and
k_unpack follow the same layout)."""
import numpy as np

TILE = 16


def pack(img: np.ndarray, w: int, h: int, rank: int, nranks: int, slab_tiles: int) -> np.ndarray:
    """img: (h*w,) uint32 -> slab (slab_tiles*256,) uint32 (padding zero)."""
    tx = (w + TILE - 1) // TILE
    nt = tx * ((h + TILE - 1) // TILE)
    slab = np.zeros(slab_tiles * 256, np.uint32)
    im = img.reshape(h, w)
    for b, t in enumerate(range(rank, nt, nranks)):
        x0, y0 = (t % tx) * TILE, (t // tx) * TILE
        blk = np.zeros((TILE, TILE), np.uint32)
        ys, xs = min(TILE, h - y0), min(TILE, w - x0)
        blk[:ys, :xs] = im[y0:y0 + ys, x0:x0 + xs]
        slab[b * 256:(b + 1) * 256] = blk.reshape(-1)
    return slab


def unpack(slabs: np.ndarray, w: int, h: int, nranks: int, slab_tiles: int) -> np.ndarray:
    tx = (w + TILE - 1) // TILE
    nt = tx * ((h + TILE - 1) // TILE)
    img = np.zeros((h, w), np.uint32)
    s = slabs.reshape(nranks, slab_tiles, TILE, TILE)
    for r in range(nranks):
        for b, t in enumerate(range(r, nt, nranks)):
            x0, y0 = (t % tx) * TILE, (t // tx) * TILE
            ys, xs = min(TILE, h - y0), min(TILE, w - x0)
            img[y0:y0 + ys, x0:x0 + xs] = s[r, b, :ys, :xs]
    return img.reshape(-1)
