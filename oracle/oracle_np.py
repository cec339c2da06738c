"""Independent numpy restatement of the hot-path contract.

TEST INFRASTRUCTURE ONLY (same rules as oracle/rt_oracle.c).  It shares no
code with the C oracle: it is written from the contract text, vectorised over
elements/rays, and exists to cross-check the C oracle and to regenerate the
committed golden fixtures under tests/golden/ (container-side; small sizes).

Every fp32 step is a numpy float32 ufunc (one IEEE rounding per op, no FMA),
in the exact operation order SURVEY.md §9.1 fixes.
"""
from __future__ import annotations

import numpy as np

SENTINEL = np.uint32(0xFFFFFFFF)
f32 = np.float32


# -- §9.1 min/max: NaN-ignoring, -0 < +0 (device v_min_f32/v_max_f32 semantics)
def fmin(a, b):
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    r = np.where(a < b, a, np.where(b < a, b, np.where(np.signbit(a), a, b)))
    r = np.where(np.isnan(b), a, r)
    return np.where(np.isnan(a), b, r).astype(f32)


def fmax(a, b):
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    r = np.where(a > b, a, np.where(b > a, b, np.where(np.signbit(a), b, a)))
    r = np.where(np.isnan(b), a, r)
    return np.where(np.isnan(a), b, r).astype(f32)


def dot(a, b):  # a, b: (...,3)
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1).astype(f32)


# -- §9.9 generators -------------------------------------------------------
_M64 = (1 << 64) - 1


def splitmix64_stream(seed: int, count: int) -> np.ndarray:
    out = np.empty(count, np.uint64)
    s = seed & _M64
    for i in range(count):
        s = (s + 0x9E3779B97F4A7C15) & _M64
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        out[i] = z ^ (z >> 31)
    return out


def soup(n: int, seed: int = 1) -> np.ndarray:
    z = splitmix64_stream(seed, 12 * n).reshape(n, 12)
    u = (z >> np.uint64(40)).astype(f32) * f32(2.0 ** -24)
    r = f32(1.0 / np.cbrt(np.float64(n))) if n else f32(0)
    c = u[:, 0:3]
    off = u[:, 3:12].reshape(n, 3, 3)
    tris = c[:, None, :] + (f32(2) * off - f32(1)) * r
    return tris.reshape(n, 9).astype(f32)


# -- §9.7 camera ----------------------------------------------------------
def camera_look_at(eye, at, up, vfov_deg, w, h):
    eye = np.asarray(eye, np.float64)
    f = np.asarray(at, np.float64) - eye
    f = f / np.sqrt(np.sum(f * f))
    r = np.cross(f, np.asarray(up, np.float64))
    r = r / np.sqrt(np.sum(r * r))
    u = np.cross(r, f)
    th = np.tan(vfov_deg * np.pi / 360.0)
    aspect = w / h
    w00 = f + u * th - r * th * aspect
    du = r * (2.0 * th * aspect / w)
    dv = -u * (2.0 * th / h)
    return np.stack([eye, w00, du, dv]).astype(f32)


# -- §9.2/§9.3 ------------------------------------------------------------
def tri_bounds(tris):
    v = tris.reshape(-1, 3, 3)
    return fmin(fmin(v[:, 0], v[:, 1]), v[:, 2]), fmax(fmax(v[:, 0], v[:, 1]), v[:, 2])


def centroid_bounds(tris):
    bmin, bmax = tri_bounds(tris)
    c = (bmin + bmax) * f32(0.5)
    lo = np.full(3, np.inf, f32)
    hi = np.full(3, -np.inf, f32)
    for row in c:  # order-independent (exact); plain loop keeps fmin semantics
        lo = fmin(lo, row)
        hi = fmax(hi, row)
    inv = np.where(hi > lo, f32(1) / np.where(hi > lo, hi - lo, f32(1)), f32(0)).astype(f32)
    return lo, hi, inv, c


def expand10(v):
    v = np.asarray(v, np.uint64)
    m = np.uint64(0xFFFFFFFF)
    v = ((v * np.uint64(0x00010001)) & m) & np.uint64(0xFF0000FF)
    v = ((v * np.uint64(0x00000101)) & m) & np.uint64(0x0F00F00F)
    v = ((v * np.uint64(0x00000011)) & m) & np.uint64(0xC30C30C3)
    v = ((v * np.uint64(0x00000005)) & m) & np.uint64(0x49249249)
    return v.astype(np.uint32)


def morton(tris, lo, inv):
    bmin, bmax = tri_bounds(tris)
    c = (bmin + bmax) * f32(0.5)
    x = ((c - lo) * inv) * f32(1024.0)
    q = fmin(fmax(x, f32(0)), f32(1023)).astype(np.uint32)
    keys = (expand10(q[:, 0]).astype(np.uint64) * 4 + expand10(q[:, 1]).astype(np.uint64) * 2
            + expand10(q[:, 2]).astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    return keys.astype(np.uint32), np.arange(len(keys), dtype=np.uint32)


def sort(keys, vals):
    # §9.4: the unique stable order -- ascending key, ties by original position
    o = np.argsort(keys, kind="stable")
    return keys[o], vals[o]


# -- §9.5 Karras ----------------------------------------------------------
def _clz32(x):
    x = np.asarray(x, np.uint64)
    out = np.full(x.shape, 32, np.int64)
    nz = x != 0
    out[nz] = 31 - np.floor(np.log2(x[nz].astype(np.float64))).astype(np.int64)
    return out


def delta(keys, i, j):
    n = len(keys)
    i = np.asarray(i, np.int64)
    j = np.asarray(j, np.int64)
    valid = (j >= 0) & (j <= n - 1)
    jj = np.clip(j, 0, max(n - 1, 0))
    ki = keys[i].astype(np.uint64)
    kj = keys[jj].astype(np.uint64)
    same = ki == kj
    d = np.where(same, 32 + _clz32((i ^ jj) & 0xFFFFFFFF), _clz32(ki ^ kj))
    return np.where(valid, d, -1)


def karras(keys):
    n = len(keys)
    m = n - 1
    parent = np.zeros(max(2 * n - 1, 0), np.uint32)
    if n == 0:
        return (np.zeros(0, np.uint32),) * 4 + (parent,)
    parent[0] = SENTINEL
    if m == 0:
        return (np.zeros(0, np.uint32),) * 4 + (parent,)
    i = np.arange(m, dtype=np.int64)
    d = np.where(delta(keys, i, i + 1) - delta(keys, i, i - 1) > 0, 1, -1)
    dmin = delta(keys, i, i - d)
    lmax = np.full(m, 2, np.int64)
    act = delta(keys, i, i + lmax * d) > dmin
    while act.any():
        lmax = np.where(act, lmax * 2, lmax)
        act = act & (delta(keys, i, i + lmax * d) > dmin)
    l = np.zeros(m, np.int64)
    t = lmax // 2
    while (t >= 1).any():
        ok = t >= 1
        cond = ok & (delta(keys, i, i + (l + t) * d) > dmin)
        l = np.where(cond, l + t, l)
        t = t // 2
    j = i + l * d
    dnode = delta(keys, i, j)
    s = np.zeros(m, np.int64)
    t = l.copy()
    run = np.ones(m, bool)
    while run.any():
        t = np.where(run, (t + 1) >> 1, t)
        cond = run & (delta(keys, i, i + (s + t) * d) > dnode)
        s = np.where(cond, s + t, s)
        run = run & (t > 1)
    g = i + s * d + np.minimum(d, 0)
    mn = np.minimum(i, j)
    mx = np.maximum(i, j)
    left = np.where(mn == g, m + g, g).astype(np.uint32)
    right = np.where(mx == g + 1, m + g + 1, g + 1).astype(np.uint32)
    parent[left] = i
    parent[right] = i
    return left, right, mn.astype(np.uint32), mx.astype(np.uint32), parent


def escape(n, left, right, parent):
    tot = 2 * n - 1
    if n == 0:
        return np.zeros(0, np.uint32)
    esc = np.full(tot, SENTINEL, np.uint32)
    cur = np.arange(tot, dtype=np.int64)
    pending = np.ones(tot, bool)
    while pending.any():
        p = parent[cur]
        root = p == SENTINEL
        pending &= ~root
        if not pending.any():
            break
        pp = np.where(pending, p, 0).astype(np.int64)
        is_left = pending & (left[pp] == cur)
        esc[is_left] = right[pp[is_left]]
        pending &= ~is_left
        cur = np.where(pending, pp, cur)
    return esc


def refit(tris, n, vals, left, right, parent):
    tot = 2 * n - 1
    lo = np.zeros((tot, 3), f32)
    hi = np.zeros((tot, 3), f32)
    if n == 0:
        return lo, hi
    bmin, bmax = tri_bounds(tris[vals])
    lo[n - 1:] = bmin
    hi[n - 1:] = bmax
    if n == 1:
        return lo, hi
    depth = np.zeros(tot, np.int64)
    cur = np.arange(tot, dtype=np.int64)
    while True:
        p = parent[cur]
        live = p != SENTINEL
        if not live.any():
            break
        depth += live
        cur = np.where(live, p, cur).astype(np.int64)
    internal = np.arange(n - 1)
    for dep in range(int(depth[: n - 1].max()), -1, -1):
        sel = internal[depth[: n - 1] == dep]
        lo[sel] = fmin(lo[left[sel]], lo[right[sel]])
        hi[sel] = fmax(hi[left[sel]], hi[right[sel]])
    return lo, hi


def build(tris):
    tris = np.asarray(tris, f32).reshape(-1, 9)
    n = len(tris)
    lo, hi, inv, _ = centroid_bounds(tris) if n else (np.full(3, np.inf, f32), np.full(3, -np.inf, f32), np.zeros(3, f32), None)
    keys, vals = morton(tris, lo, inv) if n else (np.zeros(0, np.uint32),) * 2
    skeys, svals = sort(keys, vals)
    left, right, rlo, rhi, parent = karras(skeys)
    esc = escape(n, left, right, parent)
    nlo, nhi = refit(tris, n, svals, left, right, parent)
    a = np.concatenate([left, svals]).astype(np.uint32) if n else np.zeros(0, np.uint32)
    return dict(keys=keys, vals=vals, skeys=skeys, svals=svals, left=left, right=right,
                rlo=rlo, rhi=rhi, parent=parent, esc=esc, lo=nlo, hi=nhi, a=a,
                blo=lo, bhi=hi, inv=inv)


# -- §9.7 rays + traversal ------------------------------------------------
def pcg_hash(x):
    x = np.asarray(x, np.uint64)
    m = np.uint64(0xFFFFFFFF)
    st = (x * np.uint64(747796405) + np.uint64(2891336453)) & m
    w = (((st >> ((st >> np.uint64(28)) + np.uint64(4))) ^ st) * np.uint64(277803737)) & m
    return ((w >> np.uint64(22)) ^ w).astype(np.uint32)


def rays(cam, w, h, spp):
    eye, w00, du, dv = cam
    y, x, s = np.meshgrid(np.arange(h), np.arange(w), np.arange(spp), indexing="ij")
    x = x.ravel(); y = y.ravel(); s = s.ravel()
    sidx = ((y.astype(np.uint64) * np.uint64(w) + x.astype(np.uint64)) * np.uint64(spp) + s.astype(np.uint64)) & np.uint64(0xFFFFFFFF)
    hh = pcg_hash(sidx)
    jx = np.where(s == 0, f32(0.5), (hh >> 8).astype(f32) * f32(2.0 ** -24)).astype(f32)
    jy = np.where(s == 0, f32(0.5), (pcg_hash(hh) >> 8).astype(f32) * f32(2.0 ** -24)).astype(f32)
    px = x.astype(f32) + jx
    py = y.astype(f32) + jy
    d = (w00[None, :] + px[:, None] * du[None, :]) + py[:, None] * dv[None, :]
    return np.broadcast_to(eye, d.shape).astype(f32), d.astype(f32)


def trace(b, tris, cam, w, h, spp=1):
    """Vectorised over rays.  Returns (t, u, v, prim, nodes_fetched, tris_tested)."""
    tris = np.asarray(tris, f32).reshape(-1, 9)
    n = len(tris)
    o, d = rays(np.asarray(cam, f32), w, h, spp)
    R = len(d)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        invd = f32(1) / d
    tb = np.full(R, np.inf, f32)
    hu = np.zeros(R, f32)
    hv = np.zeros(R, f32)
    hp = np.full(R, SENTINEL, np.uint32)
    idx = np.zeros(R, np.int64) if n else np.full(R, -1, np.int64)
    nn = np.zeros(R, np.int64)
    nt = np.zeros(R, np.int64)
    lo, hi, a, esc = b["lo"], b["hi"], b["a"], b["esc"]
    V = tris.reshape(-1, 3, 3)
    L0 = n - 1
    act = idx >= 0
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        while act.any():
            r = np.nonzero(act)[0]
            k = idx[r]
            nn[r] += 1
            t0 = (lo[k] - o[r]) * invd[r]
            t1 = (hi[k] - o[r]) * invd[r]
            mn = fmin(t0, t1)
            mx = fmax(t0, t1)
            tn = fmax(fmax(fmax(mn[:, 0], mn[:, 1]), mn[:, 2]), f32(0))
            tf = fmin(fmin(fmin(mx[:, 0], mx[:, 1]), mx[:, 2]), tb[r])
            hitbox = tn <= tf
            nxt = np.where(esc[k] == SENTINEL, -1, esc[k].astype(np.int64))
            leaf = hitbox & (k >= L0)
            inner = hitbox & (k < L0)
            new = np.where(inner, a[k].astype(np.int64), nxt)
            lr = r[leaf]
            if len(lr):
                nt[lr] += 1
                prim = a[k[leaf]]
                v0, v1, v2 = V[prim, 0], V[prim, 1], V[prim, 2]
                dd, oo = d[lr], o[lr]
                e1 = v1 - v0
                e2 = v2 - v0
                p = cross(dd, e2)
                det = dot(e1, p)
                inv = f32(1) / det
                s_ = oo - v0
                u = dot(s_, p) * inv
                q = cross(s_, e1)
                v = dot(dd, q) * inv
                t = dot(e2, q) * inv
                ok = (det != 0) & ~((u < 0) | (u > 1)) & ~((v < 0) | (u + v > 1)) & ~(t <= 0) & (t < tb[lr])
                w_ = lr[ok]
                tb[w_] = t[ok]; hu[w_] = u[ok]; hv[w_] = v[ok]; hp[w_] = prim[ok]
            idx[r] = new
            act = idx >= 0
    return tb, hu, hv, hp, nn, nt


def shade(tb, hu, hv, hp, w, h, spp):
    hit = hp != SENTINEL
    r = np.where(hit, hu, f32(0)).reshape(-1, spp)
    g = np.where(hit, hv, f32(0)).reshape(-1, spp)
    bl = np.where(hit, (f32(1) - hu) - hv, f32(0)).reshape(-1, spp)
    acc = [np.zeros(r.shape[0], f32) for _ in range(3)]
    for s in range(spp):
        acc[0] = acc[0] + r[:, s]
        acc[1] = acc[1] + g[:, s]
        acc[2] = acc[2] + bl[:, s]
    sc = f32(1) / f32(spp)
    out = np.empty((r.shape[0], 4), np.uint8)
    for c in range(3):
        out[:, c] = fmin(fmax(acc[c] * sc * f32(255) + f32(0.5), f32(0)), f32(255)).astype(np.uint8)
    out[:, 3] = 255
    return out.reshape(-1)
