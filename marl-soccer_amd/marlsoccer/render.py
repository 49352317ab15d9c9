"""Raster the field from env state: the headless counterpart of the reference's pygame drawing
(renderer.py:22-44 `_draw_field` / `draw`, entities.py:37-58 `Agent.draw`, :86-88 `Ball.draw`,
constants.py:2-10). pygame is not a dependency: images are uint8 RGB arrays, written as PNG by
`write_png` (stdlib zlib).

`render_batch` rasters many envs at once on the device that holds them (torch ops over the
exported state, no host round trip until the caller asks for the pixels); `render_state`
rasters one host-side `ms_env_state` record. Screen coordinates follow pygame's: x right,
y down, y_screen = 600 - y_world; pixel centres are sampled.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np
import torch

W, H = 800, 600                      # SCREEN_WIDTH, SCREEN_HEIGHT
FIELD_MARGIN, GOAL_HEIGHT = 10, 150
AGENT_HALF, BALL_RADIUS = 15.0, 10.0
FIELD = (0, 100, 0)
LINE = (255, 255, 255)
BLUE = (0, 0, 255)
RED = (255, 0, 0)
MARKER = (255, 255, 0)


def _grid(device, scale: int):
    """World coordinates of the pixel centres of a (H*scale, W*scale) image."""
    ys = (torch.arange(H * scale, device=device, dtype=torch.float32) + 0.5) / scale
    xs = (torch.arange(W * scale, device=device, dtype=torch.float32) + 0.5) / scale
    return xs.view(1, -1), ys.view(-1, 1)  # screen x, screen y


def _paint(img, mask, color):
    img[mask] = torch.tensor(color, dtype=torch.uint8, device=img.device)


def _field(device, scale: int) -> torch.Tensor:
    """renderer.py `_draw_field`: green, halfway line, centre circle, two penalty boxes
    (2-px outlines) and the two goal mouths (filled)."""
    X, Y = _grid(device, scale)
    img = torch.empty((H * scale, W * scale, 3), dtype=torch.uint8, device=device)
    img[:] = torch.tensor(FIELD, dtype=torch.uint8, device=device)
    cx, cy = W / 2, H / 2
    line = ((X >= cx - 1) & (X < cx + 1)) & (Y >= FIELD_MARGIN) & (Y <= H - FIELD_MARGIN)
    r = torch.sqrt((X - cx) ** 2 + (Y - cy) ** 2)
    circle = (r > 68.0) & (r <= 70.0)

    def outline(x0, y0, w, h, t=2):
        inside = (X >= x0) & (X < x0 + w) & (Y >= y0) & (Y < y0 + h)
        core = (X >= x0 + t) & (X < x0 + w - t) & (Y >= y0 + t) & (Y < y0 + h - t)
        return inside & ~core

    box_l = outline(FIELD_MARGIN, cy - 150, 120, 300)
    box_r = outline(W - FIELD_MARGIN - 120, cy - 150, 120, 300)
    gy = (Y >= cy - GOAL_HEIGHT / 2) & (Y < cy + GOAL_HEIGHT / 2)
    goal_l = (X >= FIELD_MARGIN - 10) & (X < FIELD_MARGIN) & gy
    goal_r = (X >= W - FIELD_MARGIN) & (X < W - FIELD_MARGIN + 10) & gy
    _paint(img, line | circle | box_l | box_r | goal_l | goal_r, LINE)
    return img


def _draw_bodies(img, px, py, ang, scale: int) -> None:
    """Agents (filled 30x30 boxes, blue team 0-1, red 2-3, yellow orientation triangle
    (15,0),(7.5,-7.5),(7.5,7.5) in body coordinates) and the ball (white disc r=10)."""
    X, Y = _grid(img.device, scale)
    Xw, Yw = X, H - Y  # world coordinates of the pixel centres
    for i in range(4):
        c, s = torch.cos(ang[i]), torch.sin(ang[i])
        dx, dy = Xw - px[i], Yw - py[i]
        lx = dx * c + dy * s
        ly = -dx * s + dy * c
        _paint(img, (lx.abs() <= AGENT_HALF) & (ly.abs() <= AGENT_HALF), BLUE if i < 2 else RED)
        _paint(img, (lx >= 7.5) & (lx <= 15.0) & (ly.abs() <= 15.0 - lx), MARKER)
    # Ball.draw rounds the centre to whole pixels: (int(x), SCREEN_HEIGHT - int(y))
    bx, by = torch.trunc(px[4]), H - torch.trunc(py[4])
    _paint(img, (X - bx) ** 2 + (Y - by) ** 2 <= BALL_RADIUS ** 2, LINE)


def body_poses(state_bytes: torch.Tensor):
    """(px, py, angle) of the 5 bodies, each (N, 5), from exported ms_env_state records held as
    raw bytes (N, itemsize) on any device (the body array leads the record)."""
    f = state_bytes.view(torch.float32).view(state_bytes.shape[0], -1)
    body = f[:, :45].reshape(-1, 5, 9)
    return body[..., 0], body[..., 1], body[..., 4]


def render_poses(px, py, ang, scale: int = 1) -> torch.Tensor:
    """Images (K, H*scale, W*scale, 3) uint8 for K envs' body poses (tensors (K, 5))."""
    base = _field(px.device, scale)
    out = base.unsqueeze(0).repeat(px.shape[0], 1, 1, 1)
    for k in range(px.shape[0]):
        _draw_bodies(out[k], px[k], py[k], ang[k], scale)
    return out


def render_batch(batch, env_ids=None, scale: int = 1) -> torch.Tensor:
    """Raster envs of a SoccerBatch on its own device (no host copy): (K, H, W, 3) uint8."""
    raw = batch.export_state_raw()
    if env_ids is not None:
        raw = raw[torch.as_tensor(env_ids, device=raw.device, dtype=torch.long)]
    px, py, ang = body_poses(raw)
    return render_poses(px, py, ang, scale)


def render_state(st) -> np.ndarray:
    """One host-side ms_env_state record (marlsoccer._native.ENV_STATE_DTYPE) -> (600, 800, 3)."""
    b = st["body"]
    px = torch.tensor(np.asarray(b["px"], np.float32))
    py = torch.tensor(np.asarray(b["py"], np.float32))
    ang = torch.tensor(np.asarray(b["angle"], np.float32))
    return render_poses(px[None], py[None], ang[None])[0].numpy()


def tile(images, cols: int) -> np.ndarray:
    """Grid of equally sized images (K, h, w, 3) -> (rows*h, cols*w, 3), unused cells black."""
    imgs = images.cpu().numpy() if isinstance(images, torch.Tensor) else np.asarray(images)
    k, h, w, _ = imgs.shape
    rows = (k + cols - 1) // cols
    out = np.zeros((rows * h, cols * w, 3), np.uint8)
    for i in range(k):
        r, c = divmod(i, cols)
        out[r * h:(r + 1) * h, c * w:(c + 1) * w] = imgs[i]
    return out


def write_png(path: str, img) -> None:
    """8-bit RGB PNG of an (h, w, 3) uint8 array (stdlib zlib; no imaging dependency)."""
    a = np.ascontiguousarray(img.cpu().numpy() if isinstance(img, torch.Tensor) else img, dtype=np.uint8)
    h, w, _ = a.shape
    raw = b"".join(b"\x00" + a[y].tobytes() for y in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def read_png(path: str) -> np.ndarray:
    """Inverse of write_png for its own files (filter type 0, RGB8) — used by the tests."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[y * (3 * w + 1) + 1:(y + 1) * (3 * w + 1)] for y in range(h)]
    return np.frombuffer(b"".join(rows), np.uint8).reshape(h, w, 3)
