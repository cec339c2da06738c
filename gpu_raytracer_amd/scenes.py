"""Scene presets for the five BASELINE.json configs.

| config | scene                                   | image        | spp | where            |
|--------|-----------------------------------------|--------------|-----|------------------|
| 1      | Cornell box, 32 tris (committed below)  | 256x256      | 1   | CPU oracle       |
| 2      | Bunny-class substitute, 70,000 tris     | 1920x1080    | 1   | 1 GPU            |
| 3      | random soup, 1M tris (splitmix64 seed 1)| 1920x1080    | 1   | 1 GPU (headline) |
| 4      | Sponza-class substitute, 262,144 tris   | 1920x1080    | 16  | image-tiled, 8 GPU|
| 5      | random soup, 10M tris                   | 3840x2160    | 4   | 8 GPU + gather   |

The Stanford Bunny and Crytek Sponza meshes are not in the container and cannot
be fetched; configs 2 and 4 use the procedural substitutes of
SURVEY.md §9.9 unless a user OBJ is given (Scene.load_obj).  Geometry here is
plain data generation (numpy, float64 -> float32); no compute on the hot path.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class View:
    eye: tuple
    at: tuple
    up: tuple
    vfov: float


def _quad(a, b, c, d):
    """Two triangles (a,b,c), (a,c,d)."""
    return [a + b + c, a + c + d]


def cornell_tris() -> np.ndarray:
    """32-triangle Cornell-style box: 5 walls + light + 2 blocks, 2 tris/quad."""
    X, Y, Z = 556.0, 548.8, 559.2
    q = []
    q += _quad((0, 0, 0), (X, 0, 0), (X, 0, Z), (0, 0, Z))                  # floor
    q += _quad((0, Y, 0), (0, Y, Z), (X, Y, Z), (X, Y, 0))                  # ceiling
    q += _quad((0, 0, Z), (X, 0, Z), (X, Y, Z), (0, Y, Z))                  # back wall
    q += _quad((X, 0, 0), (X, Y, 0), (X, Y, Z), (X, 0, Z))                  # left wall (red, +x)
    q += _quad((0, 0, 0), (0, 0, Z), (0, Y, Z), (0, Y, 0))                  # right wall (green)
    q += _quad((213, Y - 0.1, 227), (343, Y - 0.1, 227), (343, Y - 0.1, 332), (213, Y - 0.1, 332))  # light

    def block(x0, x1, z0, z1, h):
        out = []
        out += _quad((x0, h, z0), (x1, h, z0), (x1, h, z1), (x0, h, z1))    # top
        out += _quad((x0, 0, z0), (x1, 0, z0), (x1, h, z0), (x0, h, z0))    # front
        out += _quad((x1, 0, z0), (x1, 0, z1), (x1, h, z1), (x1, h, z0))    # +x side
        out += _quad((x0, 0, z1), (x0, 0, z0), (x0, h, z0), (x0, h, z1))    # -x side
        out += _quad((x1, 0, z1), (x0, 0, z1), (x0, h, z1), (x1, h, z1))    # back
        return out

    q += block(82.0, 240.0, 65.0, 225.0, 165.0)
    q += block(265.0, 430.0, 272.0, 440.0, 330.0)
    t = np.asarray(q, dtype=np.float64).astype(np.float32)
    assert t.shape == (32, 9)
    return t


CORNELL_VIEW = View((278.0, 273.0, -800.0), (278.0, 273.0, 0.0), (0.0, 1.0, 0.0), 39.3077)
SOUP_VIEW = View((0.5, 0.5, -1.5), (0.5, 0.5, 0.5), (0.0, 1.0, 0.0), 45.0)
BUNNY_VIEW = View((0.0, 0.3, -3.2), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 45.0)
SPONZA_VIEW = View((128.0, 22.0, -24.0), (128.0, 8.0, 300.0), (0.0, 1.0, 0.0), 60.0)


def bunny_substitute_tris(M: int = 200, L: int = 176) -> np.ndarray:
    """Closed lat-long sphere, 2*M*(L-1) tris (70,000 at M=200, L=176),
    radius 1 + 0.1*sin(5 theta)*cos(7 phi)."""
    th = np.pi * np.arange(1, L) / L                 # ring polar angles (L-1 rings)
    ph = 2.0 * np.pi * np.arange(M) / M
    T, P = np.meshgrid(th, ph, indexing="ij")
    R = 1.0 + 0.1 * np.sin(5.0 * T) * np.cos(7.0 * P)
    ring = np.stack([R * np.sin(T) * np.cos(P), R * np.cos(T), R * np.sin(T) * np.sin(P)], axis=-1)  # (L-1, M, 3)
    top = np.array([0.0, 1.0, 0.0])
    bot = np.array([0.0, -1.0, 0.0])
    j = np.arange(M)
    jn = (j + 1) % M
    tris = [np.concatenate([np.broadcast_to(top, (M, 3)), ring[0, jn], ring[0, j]], axis=1)]
    for i in range(L - 2):
        a, b = ring[i, j], ring[i, jn]
        c, d = ring[i + 1, jn], ring[i + 1, j]
        tris.append(np.concatenate([a, b, c], axis=1))
        tris.append(np.concatenate([a, c, d], axis=1))
    tris.append(np.concatenate([np.broadcast_to(bot, (M, 3)), ring[-1, j], ring[-1, jn]], axis=1))
    t = np.concatenate(tris, axis=0).astype(np.float32)
    assert t.shape == (2 * M * (L - 1), 9)
    return t


def sponza_substitute_tris(nx: int = 256, nz: int = 512) -> np.ndarray:
    """Heightfield 'canyon' of nx*nz quads (262,144 tris at 256x512)."""
    x = np.arange(nx + 1, dtype=np.float64)
    z = np.arange(nz + 1, dtype=np.float64)
    Xg, Zg = np.meshgrid(x, z, indexing="ij")
    wall = 60.0 * np.clip(np.abs(Xg - nx / 2) / (nx / 2), 0, 1) ** 4
    ripple = 2.0 * np.sin(0.11 * Zg) * np.cos(0.17 * Xg) + 1.5 * np.sin(0.031 * Zg + 0.05 * Xg)
    Yg = wall + ripple
    V = np.stack([Xg, Yg, Zg], axis=-1)
    a = V[:-1, :-1].reshape(-1, 3)
    b = V[1:, :-1].reshape(-1, 3)
    c = V[1:, 1:].reshape(-1, 3)
    d = V[:-1, 1:].reshape(-1, 3)
    t = np.concatenate([np.concatenate([a, b, c], 1), np.concatenate([a, c, d], 1)], 0).astype(np.float32)
    assert t.shape == (2 * nx * nz, 9)
    return t


@dataclass(frozen=True)
class Config:
    name: str
    scene: str
    n: int
    w: int
    h: int
    spp: int
    gpus: int


CONFIGS = {
    1: Config("cornell", "cornell", 32, 256, 256, 1, 0),
    2: Config("bunny-substitute", "bunny", 70000, 1920, 1080, 1, 1),
    3: Config("soup-1M", "soup", 1_000_000, 1920, 1080, 1, 1),
    4: Config("sponza-substitute", "sponza", 262144, 1920, 1080, 16, 8),
    5: Config("soup-10M", "soup", 10_000_000, 3840, 2160, 4, 8),
}

VIEWS = {"cornell": CORNELL_VIEW, "soup": SOUP_VIEW, "bunny": BUNNY_VIEW, "sponza": SPONZA_VIEW}

# Point lights of the shadow mode (DESIGN.md "Shadow mode"), per preset, and
# its ambient floor.
LIGHTS = {"cornell": (278.0, 540.0, 279.5), "soup": (2.0, 3.0, -2.0), "bunny": (2.0, 3.0, -3.0),
          "sponza": (128.0, 120.0, 150.0)}
AMBIENT = 0.2


def tris_for(scene: str, n: int = 0, seed: int = 1) -> np.ndarray | None:
    """Host triangles for a preset (None for 'soup': generated inside the library)."""
    if scene == "cornell":
        return cornell_tris()
    if scene == "bunny":
        return bunny_substitute_tris()
    if scene == "sponza":
        return sponza_substitute_tris()
    if scene == "soup":
        return None
    raise ValueError(scene)
