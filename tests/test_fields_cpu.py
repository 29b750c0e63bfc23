"""set_dynamics' structure (environment.py:59-95), CPU. The Perlin VALUES are parity unpinned
(`perlin_noise` is absent), but the reference source alone fixes one relation: the angle field's
noise (:85) is PerlinNoise(octaves=5, seed=RANDOM_SEED), the very function whose values are the
speed field's first term (:62, :72). So angle == minmax(float32(noise5)) bit for bit, and the
speed cells are built on the same noise5 values."""
import numpy as np
import pytest

SEEDS = (1707366464, 0, 12345)


@pytest.mark.parametrize("seed", SEEDS)
def test_angle_is_minmax_of_the_speed_first_octave(seed):
    from nav.fields import gradient_tables, make_fields, minmax, noise_terms
    assert len(gradient_tables(seed)) == 3  # octaves 5, 10, 20: no independent angle table
    n5, n10, n20 = noise_terms(seed)
    speed, angle = make_fields(seed)
    assert angle.dtype == np.float32 and angle.shape == (100, 100)
    # environment.py:85-95 with noise == noise_1 of :62
    want = minmax(n5.astype(np.float32))
    assert np.array_equal(angle, want)
    # environment.py:72-83: the cell sum starts from those same noise5 values
    cells = ((n5 + 0.5 * n10) + 0.25 * n20).astype(np.float32)
    norm = minmax(cells)
    assert np.array_equal(speed, (1 / (1 + np.exp(-10 * (norm - 0.5)))).astype(np.float32))
    # value ranges set_dynamics produces
    assert angle.min() == 0.0 and angle.max() == 1.0
    assert 0.0 < speed.min() < 0.01 and 0.99 < speed.max() < 1.0


def test_fields_are_seed_deterministic_and_seed_dependent():
    from nav.fields import make_fields
    a = make_fields(SEEDS[0])
    b = make_fields(SEEDS[0])
    c = make_fields(SEEDS[1])
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not np.array_equal(a[1], c[1])
