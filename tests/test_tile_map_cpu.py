"""The leaf-dot kernels' block -> tile map (xcd_tile, csrc/pp2_pbvi_dots.hip and
pp2_pbvi_host.hip), restated: a launch is sized for every row (the host does
not know how many children were kept) and the device counts the live tiles;
block b runs on XCD b % 8 and takes tile (b % 8) * per + b // 8 with
per = ceil(live / 8).  Every live tile must be taken by exactly one block that
exists in the launch, and no XCD may take more than ceil(live / 8) of them
(the grid-wide numbering put ~96 live tiles of a 144-row launch on 3 XCDs)."""
import pytest


def xcd_tile(b, ntiles):
    per = (ntiles + 7) // 8
    k = b // 8
    return (b % 8) * per + k if k < per else None


@pytest.mark.parametrize("rows_max", [16, 144, 300])
@pytest.mark.parametrize("nb", [1, 16, 53, 500])
def test_live_tiles_each_taken_once(rows_max, nb):
    alpha_tiles = (nb + 15) // 16
    tiles_max = (rows_max + 15) // 16 * alpha_tiles
    grid = (tiles_max + 7) // 8 * 8
    for kept in range(0, rows_max + 1, 7):
        live = (kept + 15) // 16 * alpha_tiles
        taken = [t for b in range(grid) if (t := xcd_tile(b, live)) is not None and t < live]
        assert sorted(taken) == list(range(live)), (rows_max, nb, kept)
        per_xcd = [0] * 8
        for b in range(grid):
            t = xcd_tile(b, live)
            if t is not None and t < live:
                per_xcd[b % 8] += 1
        assert max(per_xcd) == (live + 7) // 8, (rows_max, nb, kept)
