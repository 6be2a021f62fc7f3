"""Write the image maps of tests/scenes/imagemap.pbrt (data made for this repository's tests):
TGA files in the layouts ReadImageTGA decodes (imageio.cpp:443-533: uncompressed true colour
24 / 32 bit and 8-bit grey, origin bits 0x10 / 0x20) and PFM files of both channel counts and
byte orders (imageio.cpp:574-650).  Deterministic: rerunning rewrites the same bytes.

usage: python tools/make_images.py [outdir (default tests/scenes/textures)]
"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tga(path, img, attr=0):
    """img: uint8 [h][w][c] (c = 1 grey, 3 RGB, 4 RGBA) in FILE row order (first row first)."""
    h, w, c = img.shape
    itype = 3 if c == 1 else 2
    hdr = struct.pack("<BBB", 0, 0, itype) + struct.pack("<hhB", 0, 0, 0) + struct.pack("<hhhhBB", 0, 0, w, h, 8 * c, attr)
    px = img.copy()
    if c >= 3:
        px[..., 0], px[..., 2] = img[..., 2], img[..., 0]   # RGB(A) -> BGR(A)
    with open(path, "wb") as f:
        f.write(hdr + px.astype(np.uint8).tobytes())


def pfm(path, img, scale):
    """img: float32 [h][w][c] (c = 1 or 3); scale < 0: little-endian data, > 0: big-endian."""
    h, w, c = img.shape
    data = img.astype("<f4" if scale < 0 else ">f4").tobytes()
    with open(path, "wb") as f:
        f.write(("%s\n%d %d\n%f\n" % ("Pf" if c == 1 else "PF", w, h, scale)).encode() + data)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "scenes", "textures")
    os.makedirs(out, exist_ok=True)
    y, x = np.mgrid[0:7, 0:13]
    rgb = np.stack([(x * 19 + y * 7) % 256, (255 - x * 17) % 256, ((x ^ y) * 37) % 256], -1)
    tga(os.path.join(out, "rgb13x7.tga"), rgb)                         # 24 bit, bottom-left origin, non-power-of-2
    y, x = np.mgrid[0:5, 0:6]
    tga(os.path.join(out, "grey6x5.tga"), ((x * 40 + y * 23) % 256)[..., None], attr=0x20)   # 8-bit grey, top-left
    y, x = np.mgrid[0:4, 0:4]
    rgba = np.stack([x * 60 + 15, y * 70 + 5, ((x + y) % 2) * 200 + 30, np.full_like(x, 255)], -1)
    tga(os.path.join(out, "rgba4x4.tga"), rgba, attr=0x08 | 0x10)     # 32 bit, 8 alpha bits, right-to-left
    y, x = np.mgrid[0:3, 0:5]
    prgb = np.stack([0.1 + 0.35 * x, 0.2 + 0.4 * y, 1.5 - 0.2 * x * y], -1).astype(np.float32)
    pfm(os.path.join(out, "rgb5x3.pfm"), prgb, -1.0)                   # PF, little-endian
    y, x = np.mgrid[0:2, 0:8]
    pfm(os.path.join(out, "grey8x2.pfm"), (0.05 * x + 0.3 * y)[..., None].astype(np.float32), 2.0)   # Pf, big-endian, x2
    # a tangent-space normal map (RGB = (n + 1) / 2): a bumpy grid of tilted normals, one texel (1/2, 1/2, 1)
    y, x = np.mgrid[0:8, 0:8]
    nx, ny = 0.45 * np.sin(x * 1.3 + y * 0.4), 0.45 * np.cos(y * 1.1 - x * 0.7)
    nx[3, 5], ny[3, 5] = 0.0, 0.0
    nz = np.sqrt(np.maximum(0.0, 1.0 - nx * nx - ny * ny))
    nrm = np.stack([(nx + 1) * 127.5, (ny + 1) * 127.5, (nz + 1) * 127.5], -1).round().clip(0, 255)
    tga(os.path.join(out, "normal8x8.tga"), nrm)
    # tests/scenes/textured.pbrt: a glass index map (Pf, values 1.25 - 1.75) and a roughness map
    y, x = np.mgrid[0:4, 0:6]
    pfm(os.path.join(out, "index6x4.pfm"), (1.25 + 0.08 * x + 0.05 * y)[..., None].astype(np.float32), -1.0)
    y, x = np.mgrid[0:3, 0:7]
    pfm(os.path.join(out, "rough7x3.pfm"), (0.01 + 0.04 * ((x * 3 + y * 5) % 7))[..., None].astype(np.float32), 1.0)
    # an environment map (lat-long PF RGB, 16 x 8): a bright warm patch over a blue-grey sky (the
    # InfiniteAreaLight's radiance MIPMap and Distribution2D, infinite.cpp:60-114)
    y, x = np.mgrid[0:8, 0:16]
    sky = np.stack([0.2 + 0.02 * x, 0.25 + 0.03 * y, 0.45 + 0.01 * (x + y)], -1)
    sky[1:3, 4:7] = [6.0, 5.0, 3.5]
    sky[6, 12] = [0.0, 0.0, 0.0]
    pfm(os.path.join(out, "env16x8.pfm"), sky.astype(np.float32), -1.0)


if __name__ == "__main__":
    main()
