"""Perlin (simplex fBm) terrain (reference terrain/perlin.py:8-74).

The reference evaluates `noise.snoise2(i/scale, j/scale, octaves, persistence,
lacunarity, repeatx=1024, repeaty=1024, base=seed)` per grid point and maps
[-1, 1] -> [0, 1] * amplitude, clipped.  `noise` (caseman/noise 1.2.x, C
extension `_simplex.c`) is NOT installed here and not vendored in the
reference, so this module restates its published algorithm:

* tiled 2-D noise is 4-D simplex noise on a torus: each tiled axis u with
  period R maps to (sin(2 pi u/R), cos(2 pi u/R)) * R / (2 pi), the cosine
  part added to the 'base' coordinate (z for x, w for y).  The library takes
  sine and cosine from its polynomial fast_sin/fast_cos (_noise.h: input
  u2 = u*2/R in [0, 2] <-> [0, 2 pi]; wrap by the 1.5*2^24 round trick;
  y = u2 - u2|u2|; y*(3.1 + 3.6|y|); cos(u2) = sin(u2 + 0.5)), so this
  restatement does too -- the approximation error (~1e-3) moves points by
  O(0.1) noise units, well above float rounding;
* fBm: total = sum_o noise(p * lacunarity^o) * persistence^o / sum_o persistence^o;
* simplex corners by coordinate ranking (Gustavson), Perlin's permutation,
  the 32 4-D gradients, radius 0.6, scale 27 (4-D) / 32 (3-D);
* float32 arithmetic throughout, like the C code.

PARITY UNPINNED: without the library no reference output exists to compare
against; tests pin the properties the reference's own tests check
(shape, range, same seed -> same field, different seeds -> different fields;
test_terrains.py:22-44) plus value ranges and smoothness.
"""
from __future__ import annotations

import numpy as np

from ballbot_gym.terrain._common import check_odd

_PERM = np.array([
    151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142, 8, 99, 37,
    240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117, 35, 11, 32, 57, 177,
    33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71, 134, 139, 48, 27, 166, 77, 146,
    158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41, 55, 46, 245, 40, 244, 102, 143, 54, 65, 25,
    63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89, 18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100,
    109, 198, 173, 186, 3, 64, 52, 217, 226, 250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206,
    59, 227, 47, 16, 58, 17, 182, 189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153,
    101, 155, 167, 43, 172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218, 246,
    97, 228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239, 107, 49, 192,
    214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254, 138, 236, 205, 93, 222, 114,
    67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180], dtype=np.int64)
PERM = np.concatenate([_PERM, _PERM])

GRAD3 = np.array([[1, 1, 0], [-1, 1, 0], [1, -1, 0], [-1, -1, 0], [1, 0, 1], [-1, 0, 1], [1, 0, -1], [-1, 0, -1],
                  [0, 1, 1], [0, -1, 1], [0, 1, -1], [0, -1, -1]], dtype=np.float32)
_g4 = []  # the 32 edge midpoints of the 4-cube: one zero component, the rest +-1
for zero in (0, 1, 2, 3):  # position of the zero component: x, y, z, w
    for signs in ((1, 1, 1), (1, 1, -1), (1, -1, 1), (1, -1, -1), (-1, 1, 1), (-1, 1, -1), (-1, -1, 1), (-1, -1, -1)):
        v = list(signs)
        v.insert(zero, 0)
        _g4.append(v)
GRAD4 = np.array(_g4, dtype=np.float32)

f32 = np.float32
F3, G3 = f32(1.0 / 3.0), f32(1.0 / 6.0)
F4 = f32((np.sqrt(5.0) - 1.0) / 4.0)
G4 = f32((5.0 - np.sqrt(5.0)) / 20.0)


def _floor_i(v):
    return np.floor(v).astype(np.int64)


def noise3(x, y, z):
    """3-D simplex noise, float32 arrays of one shape."""
    x, y, z = (np.asarray(a, np.float32) for a in (x, y, z))
    s = (x + y + z) * F3
    i, j, k = np.floor(x + s), np.floor(y + s), np.floor(z + s)
    t = (i + j + k) * G3
    p0 = np.stack([x - (i - t), y - (j - t), z - (k - t)])
    X, Y, Z = p0
    xy, yz, xz = X >= Y, Y >= Z, X >= Z
    # corner offsets by the ordering of the coordinates (Gustavson's 6 cases)
    o1 = np.zeros((3,) + X.shape, np.int64)
    o2 = np.zeros((3,) + X.shape, np.int64)
    c1 = xy & yz                      # X>=Y>=Z
    c2 = xy & ~yz & xz                # X>=Z>Y
    c3 = xy & ~yz & ~xz               # Z>X>=Y
    c4 = ~xy & ~yz                    # Y>X, Y<Z -> Z>Y>X
    c5 = ~xy & yz & ~xz               # Y>X, Y>=Z, X<Z -> Y>=Z>X
    c6 = ~xy & yz & xz                # Y>X>=Z
    for cond, a, b in ((c1, (1, 0, 0), (1, 1, 0)), (c2, (1, 0, 0), (1, 0, 1)), (c3, (0, 0, 1), (1, 0, 1)),
                       (c4, (0, 0, 1), (0, 1, 1)), (c5, (0, 1, 0), (0, 1, 1)), (c6, (0, 1, 0), (1, 1, 0))):
        for d in range(3):
            o1[d] = np.where(cond, a[d], o1[d])
            o2[d] = np.where(cond, b[d], o2[d])
    p1 = p0 - o1.astype(np.float32) + G3
    p2 = p0 - o2.astype(np.float32) + f32(2.0) * G3
    p3 = p0 - f32(1.0) + f32(3.0) * G3
    I, J, K = _floor_i(i) & 255, _floor_i(j) & 255, _floor_i(k) & 255
    g = [PERM[I + PERM[J + PERM[K]]] % 12,
         PERM[I + o1[0] + PERM[J + o1[1] + PERM[o1[2] + K]]] % 12,
         PERM[I + o2[0] + PERM[J + o2[1] + PERM[o2[2] + K]]] % 12,
         PERM[I + 1 + PERM[J + 1 + PERM[K + 1]]] % 12]
    total = np.zeros_like(X)
    for p, gi in zip((p0, p1, p2, p3), g):
        f = f32(0.6) - p[0] * p[0] - p[1] * p[1] - p[2] * p[2]
        gr = GRAD3[gi]
        dot = gr[..., 0] * p[0] + gr[..., 1] * p[1] + gr[..., 2] * p[2]
        total = total + np.where(f > 0, f * f * f * f * dot, f32(0))
    return total * f32(32.0)


def noise4(x, y, z, w):
    """4-D simplex noise, float32 arrays of one shape."""
    x, y, z, w = (np.asarray(a, np.float32) for a in (x, y, z, w))
    s = (x + y + z + w) * F4
    i, j, k, l_ = np.floor(x + s), np.floor(y + s), np.floor(z + s), np.floor(w + s)
    t = (i + j + k + l_) * G4
    p0 = np.stack([x - (i - t), y - (j - t), z - (k - t), w - (l_ - t)])
    X, Y, Z, Wc = p0
    rank = np.stack([
        (X > Y).astype(np.int64) + (X > Z) + (X > Wc),
        (Y >= X).astype(np.int64) + (Y > Z) + (Y > Wc),
        (Z >= X).astype(np.int64) + (Z >= Y) + (Z > Wc),
        (Wc >= X).astype(np.int64) + (Wc >= Y) + (Wc >= Z)])
    o1, o2, o3 = (rank >= 3), (rank >= 2), (rank >= 1)
    corners = [p0,
               p0 - o1.astype(np.float32) + G4,
               p0 - o2.astype(np.float32) + f32(2.0) * G4,
               p0 - o3.astype(np.float32) + f32(3.0) * G4,
               p0 - f32(1.0) + f32(4.0) * G4]
    offs = [np.zeros_like(rank), o1.astype(np.int64), o2.astype(np.int64), o3.astype(np.int64), np.ones_like(rank)]
    I, J, K, L = (_floor_i(a) & 255 for a in (i, j, k, l_))
    total = np.zeros_like(X)
    for p, o in zip(corners, offs):
        gi = PERM[I + o[0] + PERM[J + o[1] + PERM[K + o[2] + PERM[L + o[3]]]]] & 0x1F
        f = f32(0.6) - p[0] * p[0] - p[1] * p[1] - p[2] * p[2] - p[3] * p[3]
        gr = GRAD4[gi]
        dot = gr[..., 0] * p[0] + gr[..., 1] * p[1] + gr[..., 2] * p[2] + gr[..., 3] * p[3]
        total = total + np.where(f > 0, (f * f) * (f * f) * dot, f32(0))
    return total * f32(27.0)


def fast_sin(u2):
    """noise/_noise.h fast_sin on float32: sin(pi * u2) by a wrapped parabola."""
    x = np.asarray(u2, np.float32)
    z = x + f32(25165824.0)
    x = x - (z - f32(25165824.0))
    y = x - x * np.abs(x)
    return y * (f32(3.1) + f32(3.6) * np.abs(y))


def snoise2_grid(xs, ys, octaves=1, persistence=0.5, lacunarity=2.0, base=0.0, repeat=1024.0):
    """snoise2 over the grid xs[i] x ys[j] ('ij'), float32; repeat=None -> untiled (3-D, z = base)."""
    X, Y = np.meshgrid(np.asarray(xs, np.float32), np.asarray(ys, np.float32), indexing="ij")
    pers, lac = f32(persistence), f32(lacunarity)
    if repeat is None:
        z = np.full_like(X, f32(base))
        total, amp, freq, mx = np.zeros_like(X), f32(1.0), f32(1.0), f32(0.0)
        for _ in range(int(octaves)):
            total = total + noise3(X * freq, Y * freq, z) * amp
            mx = mx + amp
            freq = freq * lac
            amp = amp * pers
        return (total / mx).astype(np.float32)
    R = float(np.float32(repeat))
    r = f32(R * (1.0 / np.pi) * 0.5)                      # repeat * M_1_PI * 0.5
    u_x = (X.astype(np.float64) * 2.0 / R).astype(np.float32)  # x * 2.0 / repeatx
    u_y = (Y.astype(np.float64) * 2.0 / R).astype(np.float32)
    x4, z4 = fast_sin(u_x) * r, f32(base) + fast_sin(u_x + f32(0.5)) * r
    y4, w4 = fast_sin(u_y) * r, f32(base) + fast_sin(u_y + f32(0.5)) * r
    total = noise4(x4, y4, z4, w4)
    amp, freq, mx = f32(1.0), f32(1.0), f32(1.0)
    for _ in range(1, int(octaves)):
        freq = freq * lac
        amp = amp * pers
        mx = mx + amp
        total = total + noise4(x4 * freq, y4 * freq, z4 * freq, w4 * freq) * amp
    return (total / mx).astype(np.float32)


def generate_perlin_terrain(n: int, scale: float = 25.0, octaves: int = 4, persistence: float = 0.2,
                            lacunarity: float = 2.0, amplitude: float = 1.0, seed: int = 0) -> np.ndarray:
    """(snoise2(i/scale, j/scale, ...) + 1) / 2 * amplitude, clipped to [0, 1], float64[n*n]."""
    check_odd(n)
    g = np.arange(n, dtype=np.float64) / scale
    noise = snoise2_grid(g, g, octaves=octaves, persistence=persistence, lacunarity=lacunarity,
                         base=float(seed), repeat=1024.0).astype(np.float64)
    t = (noise + 1.0) / 2.0 * amplitude
    return np.clip(t, 0.0, 1.0).flatten()
