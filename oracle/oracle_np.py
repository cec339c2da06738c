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
    o, d = rays(np.asarray(cam, f32), w, h, spp)
    return trace_rays(b, tris, o, d)


def trace_rays(b, tris, o, d, tmax=np.inf, any_hit=False):
    """§9.7 escape-link traversal of arbitrary rays over (0, tmax); any_hit
    ends a ray at its first hit (shadow rays)."""
    tris = np.asarray(tris, f32).reshape(-1, 9)
    n = len(tris)
    o = np.asarray(o, f32)
    d = np.asarray(d, f32)
    R = len(d)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        invd = f32(1) / d
    tb = np.full(R, tmax, f32)
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
                if any_hit:
                    new[np.nonzero(leaf)[0][ok]] = -1
            idx[r] = new
            act = idx >= 0
    return tb, hu, hv, hp, nn, nt


def _q8(x):
    return fmin(fmax(x * f32(255) + f32(0.5), f32(0)), f32(255)).astype(np.uint8)


def _surface(tris, prim, o, d, t, light):
    """Shading frame of hits (DESIGN.md shadow/path modes): unit geometric
    normal facing the ray, S = P + 1e-4 N, D = light - S, cos to the light."""
    V = np.asarray(tris, f32).reshape(-1, 3, 3)[prim]
    P = o + t[:, None] * d
    e1 = V[:, 1] - V[:, 0]
    e2 = V[:, 2] - V[:, 0]
    nrm = cross(e1, e2)
    nl = np.sqrt(dot(nrm, nrm))
    with np.errstate(divide="ignore", invalid="ignore"):
        N = np.where((nl > 0)[:, None], nrm / nl[:, None], f32(0)).astype(f32)
    N = np.where((dot(N, d) > 0)[:, None], -N, N).astype(f32)
    S = P + N * f32(1e-4)
    D = np.asarray(light, f32)[None, :] - S
    dl = np.sqrt(dot(D, D))
    with np.errstate(divide="ignore", invalid="ignore"):
        cosl = np.where(dl > 0, dot(N, D) / dl, f32(0)).astype(f32)
    return N, S, D, cosl


def render_shadow(b, tris, cam, w, h, spp, light, ambient):
    """Shadow mode: (t, u, v, prim, rgba)."""
    o, d = rays(np.asarray(cam, f32), w, h, spp)
    t, u, v, p, _, _ = trace_rays(b, tris, o, d)
    hit = np.nonzero(p != SENTINEL)[0]
    f = np.zeros(len(d), f32)
    if len(hit):
        N, S, D, cosl = _surface(tris, p[hit], o[hit], d[hit], t[hit], light)
        _, _, _, sp, _, _ = trace_rays(b, tris, S, D, f32(1), True)
        lit = np.where(sp != SENTINEL, f32(0), fmax(cosl, f32(0)))
        f[hit] = f32(ambient) + (f32(1) - f32(ambient)) * lit
    rgb = np.stack([u * f, v * f, ((f32(1) - u) - v) * f], 1).astype(f32)
    rgb[p == SENTINEL] = 0
    return t, u, v, p, _mean_q8(rgb, spp)


def _mean_q8(rgb, spp):
    rgb = rgb.reshape(-1, spp, 3)
    acc = np.zeros((rgb.shape[0], 3), f32)
    for s in range(spp):
        acc = acc + rgb[:, s]
    out = np.empty((rgb.shape[0], 4), np.uint8)
    out[:, :3] = _q8(acc * (f32(1) / f32(spp)))
    out[:, 3] = 255
    return out.reshape(-1)


def render_path(b, tris, cam, w, h, spp, light, sky, max_depth):
    """Path mode, advanced as a wavefront: every live path traces
    its next segment together.  Returns (t, u, v, prim of the primary rays,
    rgba, rays traced)."""
    o, d = rays(np.asarray(cam, f32), w, h, spp)
    R = len(d)
    st = pcg_hash(np.arange(R, dtype=np.uint64) ^ np.uint64(0x5BD1E995))
    L = np.zeros((R, 3), f32)
    beta = np.ones((R, 3), f32)
    live = np.arange(R)
    nrays = 0
    sky = f32(sky)
    for depth in range(max_depth + 1):
        t, u, v, p, _, _ = trace_rays(b, tris, o[live], d[live])
        nrays += len(live)
        if depth == 0:
            prim0 = (t, u, v, p)
        miss = p == SENTINEL
        if depth > 0:
            L[live[miss]] = L[live[miss]] + beta[live[miss]] * sky
        hm = ~miss
        live, t, p = live[hm], t[hm], p[hm]
        if not len(live):
            break
        N, S, D, cosl = _surface(tris, p, o[live], d[live], t, light)
        ha = pcg_hash(p.astype(np.uint64) ^ np.uint64(0x27D4EB2F))
        alb = np.stack([f32(0.25) + ((ha >> np.uint32(8 * c)) & np.uint32(255)).astype(f32) * f32(2.0 ** -9)
                        for c in range(3)], 1).astype(f32)
        sh = cosl > 0
        if sh.any():
            _, _, _, sp, _, _ = trace_rays(b, tris, S[sh], D[sh], f32(1), True)
            nrays += int(sh.sum())
            vis = np.nonzero(sh)[0][sp == SENTINEL]
            r = live[vis]
            L[r] = L[r] + (beta[r] * alb[vis]) * cosl[vis][:, None]
        if depth == max_depth:
            break
        beta[live] = beta[live] * alb
        sl = st[live]
        px = np.zeros(len(live), f32); py = np.zeros(len(live), f32); r2 = np.zeros(len(live), f32)
        todo = np.ones(len(live), bool)
        for _k in range(16):
            i = np.nonzero(todo)[0]
            if not len(i):
                break
            sl[i] = pcg_hash(sl[i])
            qx = (sl[i] >> np.uint32(8)).astype(f32) * f32(2.0 ** -24) * f32(2) - f32(1)
            sl[i] = pcg_hash(sl[i])
            qy = (sl[i] >> np.uint32(8)).astype(f32) * f32(2.0 ** -24) * f32(2) - f32(1)
            q2 = qx * qx + qy * qy
            acc = q2 < f32(1)
            px[i[acc]] = qx[acc]; py[i[acc]] = qy[acc]; r2[i[acc]] = q2[acc]
            todo[i[acc]] = False
        st[live] = sl
        z = np.sqrt(f32(1) - r2)
        sg = np.where(N[:, 2] >= 0, f32(1), f32(-1)).astype(f32)
        ia = f32(-1) / (sg + N[:, 2])
        ib = (N[:, 0] * N[:, 1]) * ia
        T = np.stack([f32(1) + ((sg * N[:, 0]) * N[:, 0]) * ia, sg * ib, -(sg * N[:, 0])], 1).astype(f32)
        B = np.stack([ib, sg + (N[:, 1] * N[:, 1]) * ia, -N[:, 1]], 1).astype(f32)
        d[live] = (px[:, None] * T + py[:, None] * B) + z[:, None] * N
        o[live] = S
    return prim0 + (_mean_q8(L, spp), nrays)


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
