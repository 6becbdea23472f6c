#!/usr/bin/env python3
"""Synthetic HDR lat-long environment map (PFM) for the envmap emitter.

The reference's own test map, data/tests/envmap.exr, is PIZ-compressed
OpenEXR; there is no EXR decoder in this image, so the envmap scenes use this
deterministic stand-in (sky gradient, ground, a sun disk and a few coloured
patches that exercise the bilinear / EWA filters and the importance
sampler).  Values stay below the half-precision maximum (65504) because
Mitsuba stores MIP levels as half.

usage: python tools/gen_envmap.py OUT.pfm [width height]"""
import sys

import numpy as np


def make(w=512, h=256):
    v = (np.arange(h) + 0.5) / h                      # 0 = zenith (top row)
    u = (np.arange(w) + 0.5) / w
    theta = v * np.pi
    phi = u * 2 * np.pi
    T, P = np.meshgrid(theta, phi, indexing="ij")
    y = np.cos(T)                                       # up = +y (envmap.cpp:380-395)
    img = np.zeros((h, w, 3), np.float64)
    sky = np.clip(y, 0, 1)[..., None]
    img += (1 - sky) * np.array([0.9, 0.95, 1.2]) + sky * np.array([0.25, 0.45, 1.0])
    ground = y < 0
    img[ground] = np.array([0.30, 0.25, 0.20]) * (0.6 + 0.4 * np.cos(8 * P[ground]) ** 2)[:, None]
    # sun: small bright disk
    sun_t, sun_p = np.radians(35.0), np.radians(60.0)
    cosang = np.sin(T) * np.sin(sun_t) * np.cos(P - sun_p) + np.cos(T) * np.cos(sun_t)
    img[cosang > np.cos(np.radians(2.0))] = np.array([3000.0, 2600.0, 2000.0])
    # coloured patches (filter / sampler structure)
    for (pt, pp, col) in [(70, 200, (8, 0.5, 0.5)), (80, 300, (0.5, 6, 0.5)), (60, 20, (0.5, 0.5, 10))]:
        c = np.sin(T) * np.sin(np.radians(pt)) * np.cos(P - np.radians(pp)) + np.cos(T) * np.cos(np.radians(pt))
        img[c > np.cos(np.radians(6.0))] = col
    return img.astype(np.float32)


def write_pfm(path, img):
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(img[::-1]).astype("<f4").tobytes())   # rows bottom-up


if __name__ == "__main__":
    out = sys.argv[1]
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    write_pfm(out, make(w, h))
