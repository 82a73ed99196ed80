"""The fused loss kernels' XCD-aware tile order (gs_loss.hip, Tiles::of_block):
block b takes tile (b mod 8) * floor(n/8) + min(b mod 8, n mod 8) + floor(b/8).
Every tile must be taken exactly once for every tile count (a missed tile
would leave its loss partial and its gradient unwritten), and the blocks an
XCD runs (b = x, x + 8, ...) must take one contiguous run of tiles."""
import pytest


def of_block(b, n):
    x, per, rem = b & 7, n >> 3, n & 7
    return x * per + min(x, rem) + (b >> 3)


@pytest.mark.parametrize("n", list(range(1, 70)) + [2500, 6120, 8160 * 3, 123457])
def test_bijection_and_contiguous_runs(n):
    tiles = [of_block(b, n) for b in range(n)]
    assert sorted(tiles) == list(range(n))
    for x in range(8):
        run = [of_block(b, n) for b in range(x, n, 8)]
        assert run == list(range(run[0], run[0] + len(run))) if run else True
