"""Dynamics fields (environment.py:59-95 set_dynamics), generated without `perlin_noise`.

The reference builds its speed field from three PerlinNoise(octaves=5/10/20, seed=RANDOM_SEED)
functions (weights 1, .5, .25) sampled at (col/100, row/100), min-max normalises, then stretches
with sigmoid(10 (x - .5)); the angle field is one octave-5 function, min-max normalised. The
third-party `perlin_noise` package is absent from this image and unpinned by the reference, so the
exact field values are PARITY UNPINNED: this module reproduces the construction (octave mix,
normalisation, sigmoid stretch, x-major float32 [100][100]) with its own seeded gradient noise.
Fields are an input of every kernel; tests inject fixed fields.
"""
import numpy as np


def _gradient_noise(rng, octaves, n=100):
    """Classic 2-D Perlin gradient noise with `octaves` lattice cells across [0,1)."""
    g = rng.standard_normal((octaves + 1, octaves + 1, 2))
    g /= np.linalg.norm(g, axis=-1, keepdims=True) + 1e-12
    u = np.arange(n) / n * octaves
    x, y = np.meshgrid(u, u, indexing="ij")  # [col][row] like environment.py:69-75
    x0, y0 = np.floor(x).astype(int), np.floor(y).astype(int)
    fx, fy = x - x0, y - y0

    def dot(ix, iy, dx, dy):
        v = g[ix, iy]
        return v[..., 0] * dx + v[..., 1] * dy

    fade = lambda t: t * t * t * (t * (t * 6 - 15) + 10)  # noqa: E731
    n00 = dot(x0, y0, fx, fy)
    n10 = dot(x0 + 1, y0, fx - 1, fy)
    n01 = dot(x0, y0 + 1, fx, fy - 1)
    n11 = dot(x0 + 1, y0 + 1, fx - 1, fy - 1)
    wx, wy = fade(fx), fade(fy)
    return (n00 * (1 - wx) + n10 * wx) * (1 - wy) + (n01 * (1 - wx) + n11 * wx) * wy


def make_fields(seed):
    """(speed, angle) float32 [100][100], x-major, value ranges as set_dynamics produces."""
    rng = np.random.default_rng(seed)
    cells = (_gradient_noise(rng, 5) + 0.5 * _gradient_noise(rng, 10)
             + 0.25 * _gradient_noise(rng, 20)).astype(np.float32)
    mn, mx = np.min(cells), np.max(cells)
    norm = (cells - mn) / (mx - mn)
    speed = (1 / (1 + np.exp(-10 * (norm - 0.5)))).astype(np.float32)
    cells = _gradient_noise(rng, 5).astype(np.float32)
    mn, mx = np.min(cells), np.max(cells)
    angle = ((cells - mn) / (mx - mn)).astype(np.float32)
    return speed, angle
