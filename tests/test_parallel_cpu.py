"""Host logic of pynbodyext.parallel that needs no device: 64-aligned range
cuts (whole walk waves per rank)."""
import pytest

from pynbodyext.parallel import align_ranges


@pytest.mark.parametrize("n", [1000, 64 * 4688, 4_000_000])
def test_align_ranges(n):
    import numpy as np

    rng = np.random.default_rng(n)
    for world in (2, 3, 8):
        cuts = np.sort(rng.integers(0, n, world - 1))
        bounds = [0, *cuts.tolist(), n]
        ranges = [(a, b - a) for a, b in zip(bounds[:-1], bounds[1:])]
        out = align_ranges(ranges, n, 64)
        assert len(out) == world
        assert out[0][0] == 0 and sum(c for _, c in out) == n
        for (f0, c0), (f1, _) in zip(out[:-1], out[1:]):
            assert f0 + c0 == f1 and c0 >= 0
            assert f1 % 64 == 0 or f1 == n
        for (f, _), (g, _) in zip(ranges[1:], out[1:]):
            assert abs(f - g) <= 32 or g == out[0][1]  # nearest multiple (or clamped monotone)
