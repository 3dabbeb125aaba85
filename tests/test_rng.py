"""Host mirror of the kernel's Philox4x32-10 reset RNG: Random123 known answers."""
import numpy as np

import pybulletgym_amd  # noqa: F401
from pybulletgym_amd import rng


def test_philox_known_answers():
    z = rng.philox4x32_10(np.zeros((1, 4), np.uint32), (0, 0))[0]
    assert [int(v) for v in z] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = rng.philox4x32_10(np.full((1, 4), 0xFFFFFFFF, np.uint32), (0xFFFFFFFF, 0xFFFFFFFF))[0]
    assert [int(v) for v in f] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_reset_noise_range_and_independence_of_sharding():
    a = rng.reset_noise(7, np.arange(100), 0, 17)
    assert a.dtype == np.float32 and a.shape == (100, 17)
    assert a.min() >= -0.1 and a.max() < 0.1
    b = rng.reset_noise(7, np.arange(50, 100), 0, 17)
    np.testing.assert_array_equal(a[50:], b)
    c = rng.reset_noise(7, np.arange(100), 1, 17)
    assert not np.array_equal(a, c)
