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


def _gradient_table(rng, octaves):
    """the unit lattice gradients [octaves+1][octaves+1][2] of one noise function"""
    g = rng.standard_normal((octaves + 1, octaves + 1, 2))
    g /= np.linalg.norm(g, axis=-1, keepdims=True) + 1e-12
    return g


def gradient_tables(seed):
    """(g5, g10, g20): make_fields' gradient tables, drawn in its order."""
    rng = np.random.default_rng(seed)
    return tuple(_gradient_table(rng, o) for o in (5, 10, 20))


def _gradient_noise(g, octaves, n=100):
    """Classic 2-D Perlin gradient noise with `octaves` lattice cells across [0,1), f64."""
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


def noise_terms(seed):
    """(noise5, noise10, noise20): the three f64 [100][100] noise functions sampled at
    (col/100, row/100) — PerlinNoise(octaves=5/10/20, seed) of environment.py:62-64."""
    return tuple(_gradient_noise(g, o) for g, o in zip(gradient_tables(seed), (5, 10, 20)))


def minmax(cells):
    """environment.py:77-79 / :92-94 on a float32 table (float32 arithmetic, NEP 50)."""
    mn, mx = np.min(cells), np.max(cells)
    return (cells - mn) / (mx - mn)


def make_fields(seed):
    """(speed, angle) float32 [100][100], x-major, value ranges as set_dynamics produces."""
    n5, n10, n20 = noise_terms(seed)
    # environment.py:72-75: the cell sum in Python floats, stored float32
    norm = minmax(((n5 + 0.5 * n10) + 0.25 * n20).astype(np.float32))
    speed = (1 / (1 + np.exp(-10 * (norm - 0.5)))).astype(np.float32)
    # environment.py:85-95: the SAME octave-5 function as the speed's first term
    angle = minmax(n5.astype(np.float32)).astype(np.float32)
    return speed, angle


def make_field_device(seed, device="cuda", stream=None):
    """make_fields on the device (nav_fields_generate): the [100][100][2] (speed, angle) float32
    table the kernels read, from the same gradient tables (tests/test_gpu_env.py compares)."""
    import torch
    from ._lib import lib, ptr, stream_handle
    g = [torch.as_tensor(np.ascontiguousarray(t), dtype=torch.float64).to(device)
         for t in gradient_tables(seed)]
    field = torch.empty(100, 100, 2, dtype=torch.float32, device=device)
    lib().nav_fields_generate(*[ptr(t) for t in g], ptr(field), stream_handle(stream))
    return field
