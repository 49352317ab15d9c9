"""Render one env state to an RGB image (numpy), the headless counterpart of the
reference's pygame drawing (renderer.py, game.py:440-456, entities.py:37-58, 86-88).

Screen coordinates follow pygame's: x right, y down, y_screen = 600 - y_world.
"""
from __future__ import annotations

import numpy as np

W, H = 800, 600
FIELD = (0, 100, 0)
LINE = (255, 255, 255)
BLUE = (0, 0, 255)
RED = (255, 0, 0)
MARKER = (255, 255, 0)


def _yy_xx():
    yy, xx = np.mgrid[0:H, 0:W]
    return xx.astype(np.float32) + 0.5, (H - (yy.astype(np.float32) + 0.5))


_GRID = None


def render_state(st) -> np.ndarray:
    """st: one ms_env_state record (marlsoccer._native.ENV_STATE_DTYPE)."""
    global _GRID
    if _GRID is None:
        _GRID = _yy_xx()
    X, Y = _GRID
    img = np.empty((H, W, 3), np.uint8)
    img[:] = FIELD
    # field lines (game.py:443-448)
    img[:, 399:401] = LINE
    r = np.hypot(X - 400, Y - 300)
    img[(r > 69) & (r < 71)] = LINE
    img[(Y > 225) & (Y < 375) & (X < 10)] = LINE
    img[(Y > 225) & (Y < 375) & (X > 790)] = LINE
    body = st["body"]
    for i in range(4):
        px, py, a = float(body["px"][i]), float(body["py"][i]), float(body["angle"][i])
        c, s = np.cos(a), np.sin(a)
        lx = (X - px) * c + (Y - py) * s
        ly = -(X - px) * s + (Y - py) * c
        img[(np.abs(lx) <= 15) & (np.abs(ly) <= 15)] = BLUE if i < 2 else RED
        # orientation marker triangle (entities.py:44-57): (15,0), (7.5,-7.5), (7.5,7.5)
        tri = (lx >= 7.5) & (lx <= 15) & (np.abs(ly) <= (15 - lx))
        img[tri] = MARKER
    bx, by = float(body["px"][4]), float(body["py"][4])
    img[np.hypot(X - bx, Y - by) <= 10] = LINE
    return img
