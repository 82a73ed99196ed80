"""A lane-level model of k_tile_ranges' empty-tile fill (wave_fill_runs in
gsplat_mi355x.hip), run on the CPU: 64-lane waves, the last wave partial
(lanes past num_pairs leave the kernel first), gaps longer than 32 tiles
written by the wave's active lanes together.  Every tile's range must be
written and equal to the bisection of the sorted keys (empty tiles: start ==
end).  The first GPU version strode by 64 regardless of the active lanes and
left ranges unwritten behind a partial wave (a GPU fault on the sparse-frame
test); the model of that stride is checked to fail the same way."""
import bisect
import random

import pytest

WAVE, BLOCK, RUN = 64, 256, 32


def model_tile_ranges(keys, num_tiles, stride_active=True):
    T = len(keys)
    ranges = [None] * (2 * num_tiles)
    nthreads = ((T + 1 + BLOCK - 1) // BLOCK) * BLOCK
    for w0 in range(0, nthreads, WAVE):
        lanes = [p for p in range(w0, w0 + WAVE) if p <= T]  # `if (p > num_pairs) return;`
        if not lanes:
            continue
        state = {}
        for p in lanes:
            prev = keys[p - 1] if p > 0 else -1
            cur = keys[p] if p < T else num_tiles
            edge = cur != prev
            if edge and prev >= 0:
                ranges[2 * prev + 1] = p
            if edge and cur < num_tiles:
                ranges[2 * cur] = p
            t0 = prev + 1
            t1 = cur if edge else t0
            wide = t1 > t0 + RUN
            if not wide:
                for t in range(t0, t1):
                    ranges[2 * t] = ranges[2 * t + 1] = p
            state[p] = (wide, t0, t1)
        stride = len(lanes) if stride_active else WAVE
        for owner in (p for p in lanes if state[p][0]):
            _, lo, hi = state[owner]
            for rank, p in enumerate(lanes):
                o = lo + (rank if stride_active else p - w0)
                while o < hi:
                    ranges[2 * o] = ranges[2 * o + 1] = owner
                    o += stride
    return ranges


def check(keys, num_tiles, ranges):
    for t in range(num_tiles):
        a, b = ranges[2 * t], ranges[2 * t + 1]
        assert a is not None and b is not None, f"tile {t} unwritten"
        lo, hi = bisect.bisect_left(keys, t), bisect.bisect_right(keys, t)
        if lo != hi:
            assert (a, b) == (lo, hi), t
        else:
            assert a == b, t


@pytest.mark.parametrize("num_tiles", [1, 5, 40, 300, 19200])
@pytest.mark.parametrize("T", [0, 1, 3, 20, 63, 64, 65, 200, 700])
def test_every_range_written(num_tiles, T):
    rng = random.Random(num_tiles * 1000 + T)
    keys = sorted(rng.randrange(num_tiles) for _ in range(T))
    check(keys, num_tiles, model_tile_ranges(keys, num_tiles))


def test_stride_of_64_leaves_holes_behind_a_partial_wave():
    rng = random.Random(7)
    keys = sorted(rng.randrange(19200) for _ in range(20))
    ranges = model_tile_ranges(keys, 19200, stride_active=False)
    assert any(v is None for v in ranges)
