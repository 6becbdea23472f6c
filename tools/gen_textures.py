"""Deterministic PNG textures for the `bitmap` texture tests and scenes.

PNG files are written from the published format (RFC 2083): IHDR, optional
PLTE / gAMA / sRGB chunks, one zlib IDAT stream whose scanlines cycle through
all five filter types (so the reader's unfiltering is exercised), IEND.

    python3 tools/gen_textures.py [outdir]   (default: scenes/)

Outputs (all pure functions of their size, no RNG state):
    tex_checker.png   96 x 64 8-bit RGB, colored checker + gradients (no colour chunk: sRGB)
    tex_rgba.png      50 x 50 8-bit RGBA with an sRGB chunk
    tex_gray16.png    40 x 30 16-bit gray with gAMA 0.45455
    tex_palette.png   33 x 17 4-bit palette
"""
import os
import struct
import sys
import zlib

import numpy as np


def _chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def _filter_rows(raw: np.ndarray, bpp: int) -> bytes:
    """raw: (h, rowbytes) uint8; row y uses filter y % 5."""
    out = bytearray()
    prev = np.zeros(raw.shape[1], np.int32)
    for y in range(raw.shape[0]):
        cur = raw[y].astype(np.int32)
        ft = y % 5
        line = np.zeros_like(cur)
        for i in range(len(cur)):
            a = cur[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
            line[i] = (cur[i] - pred) & 0xFF
        out.append(ft)
        out += bytes(line.astype(np.uint8))
        prev = cur
    return bytes(out)


def write_png(path: str, samples: np.ndarray, color_type: int, depth: int, palette=None, gama=None, srgb=False):
    """samples: (h, w, ch) integers (palette indices for color type 3)."""
    h, w = samples.shape[:2]
    ch = samples.shape[2]
    if depth == 16:
        raw = samples.astype(">u2").reshape(h, w * ch).view(np.uint8).reshape(h, -1)
        bpp = 2 * ch
    elif depth == 8:
        raw = samples.astype(np.uint8).reshape(h, w * ch)
        bpp = ch
    else:   # packed sub-byte samples (one channel)
        per = 8 // depth
        rb = (w * depth + 7) // 8
        raw = np.zeros((h, rb), np.uint8)
        for x in range(w):
            raw[:, x // per] |= (samples[:, x, 0].astype(np.uint8) << (8 - depth * (x % per + 1))).astype(np.uint8)
        bpp = 1
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, color_type, 0, 0, 0))
    if srgb:
        data += _chunk(b"sRGB", b"\x00")
    if gama is not None:
        data += _chunk(b"gAMA", struct.pack(">I", int(round(gama * 100000))))
    if palette is not None:
        data += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).ravel()))
    data += _chunk(b"IDAT", zlib.compress(_filter_rows(raw, bpp), 9)) + _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


def checker(w=96, h=64):
    y, x = np.mgrid[0:h, 0:w]
    c = ((x // 8 + y // 8) % 2).astype(np.float64)
    r = 40 + 180 * c + 30 * np.sin(x / 7.0)
    g = 30 + 150 * (1 - c) + 60 * (y / h)
    b = 20 + 200 * (x / w) * (y / h)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def rgba(w=50, h=50):
    y, x = np.mgrid[0:h, 0:w]
    ring = ((np.hypot(x - 25, y - 25) // 5) % 2).astype(np.float64)
    r = 30 + 200 * ring
    g = 60 + 150 * (x / w)
    b = 200 - 150 * ring
    a = 255 - 3 * x
    return np.clip(np.stack([r, g, b, a], -1), 0, 255).astype(np.uint8)


def gray16(w=40, h=30):
    y, x = np.mgrid[0:h, 0:w]
    v = 65535 * (0.5 + 0.45 * np.sin(x / 3.0) * np.cos(y / 4.0))
    return np.clip(v, 0, 65535).astype(np.uint16)[..., None]


def palette4(w=33, h=17):
    y, x = np.mgrid[0:h, 0:w]
    idx = ((x // 3) + 2 * (y // 4)) % 11
    pal = np.array([[int(255 * ((i * 37) % 11) / 10), int(255 * ((i * 53) % 11) / 10), int(255 * i / 10)] for i in range(11)])
    return idx.astype(np.uint8)[..., None], pal


def main(out="scenes"):
    os.makedirs(out, exist_ok=True)
    write_png(os.path.join(out, "tex_checker.png"), checker(), 2, 8)
    write_png(os.path.join(out, "tex_rgba.png"), rgba(), 6, 8, srgb=True)
    write_png(os.path.join(out, "tex_gray16.png"), gray16(), 0, 16, gama=0.45455)
    idx, pal = palette4()
    write_png(os.path.join(out, "tex_palette.png"), idx, 3, 4, palette=pal)


if __name__ == "__main__":
    main(*sys.argv[1:])
