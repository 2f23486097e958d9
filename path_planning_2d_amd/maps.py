"""Occupancy-grid loading, as PathPlanning2dBase::loadMapFromFile does it
(src/pomdp/path_planning_2d.cu:243-257, src/mdp/path_planning_2d.cu:191-205):
``imread(path, IMREAD_GRAYSCALE)`` then ``threshold(img, 250, 1,
THRESH_BINARY_INV)`` -- a pixel <= 250 is occupied (1), otherwise free (0).
"""
from __future__ import annotations

import numpy as np


def threshold_map(gray: np.ndarray) -> np.ndarray:
    gray = np.asarray(gray)
    return (gray <= 250).astype(np.uint8)


def load_map(path: str) -> np.ndarray:
    """Decode a map image to an (H, W) uint8 grid (1 = occupied)."""
    if path.endswith(".npy"):
        return np.ascontiguousarray(np.load(path, allow_pickle=False), np.uint8)
    from PIL import Image  # only needed for image maps
    with Image.open(path) as im:
        gray = np.array(im.convert("L"))
    return threshold_map(gray)


def tile_map(grid: np.ndarray, height: int, width: int) -> np.ndarray:
    """Periodic tiling of a map to (height, width) -- SURVEY.md §8(d)'s
    'realistic-structure' synthetic grids (e.g. a 64x64 tile of
    sparse_map_100x40)."""
    H, W = grid.shape
    ys = np.arange(height) % H
    xs = np.arange(width) % W
    return np.ascontiguousarray(grid[np.ix_(ys, xs)], np.uint8)
