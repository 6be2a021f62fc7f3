"""Whole-frame fixtures of BASELINE.json's configs at their real size and sample count, from the
reference harness (oracle/_ref, the unmodified reference TUs).  Build container only: the frame
is rendered as horizontal strips by parallel harness processes, each strip's sample window one
row larger on each side (a film pixel receives samples of its own and its neighbouring sample
pixels only, spectralImage.cpp:77-152), so every pixel of a strip holds all of its contributions
in the reference's order.  The committed fixture is small:

  tests/golden/<name>.npz   hash[nty, ntx] uint64   blake2b-64 of each 16x16 tile's float32 bits
                            sum[nty, ntx] float64    the tile's sum of every band of every pixel
                            absmax[nty, ntx] float32 the tile's largest |value|
                            config [W, H, spp, seed, maxdepth, bands, tile]

tests/test_frame_golden.py renders the same frame on the GPU and compares every tile's hash.

Usage: python tools/make_frame_golden.py [c1|c2|c4|c5|c3 ...] [--jobs 8]
"""
import hashlib
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from make_golden import HARNESS, HARNESS60, HARNESSRGB, SCENES, OUT  # noqa: E402

TILE = 16
# name, scene file, W, H, spp, bands
# bands 3 = the reference's RGBSpectrum build (C1, BASELINE configs[0]; oracle/_ref/brgb)
FRAMES = {"c1": ("killeroo_rgb_frame_c1_400x400s64", "killeroo-simple.pbrt", 400, 400, 64, 3),
          "c2": ("killeroo_frame_c2_700x700s256", "killeroo-simple.pbrt", 700, 700, 256, 32),
          "c3": ("bunny_frame_c3_1920x1080s1024", "bunny.pbrt", 1920, 1080, 1024, 32),
          "c4": ("metal_frame_c4_400x400s4096", "metal.pbrt", 400, 400, 4096, 60),
          "c5": ("anim_frame_c5_600x600s512", "anim-killeroos-moving.pbrt", 600, 600, 512, 32)}


def tile_digest(film, tile=TILE):
    """per-tile blake2b-64 of the float32 bits, sum (float64) and max |value| (shared with the test)"""
    H, W = film.shape[:2]
    nty, ntx = (H + tile - 1) // tile, (W + tile - 1) // tile
    hs = np.zeros((nty, ntx), np.uint64)
    sm = np.zeros((nty, ntx), np.float64)
    mx = np.zeros((nty, ntx), np.float32)
    for ty in range(nty):
        for tx in range(ntx):
            t = np.ascontiguousarray(film[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile], dtype=np.float32)
            hs[ty, tx] = int.from_bytes(hashlib.blake2b(t.tobytes(), digest_size=8).digest(), "little")
            sm[ty, tx] = t.astype(np.float64).sum()
            mx[ty, tx] = np.abs(t).max() if t.size else 0.0
    return hs, sm, mx


def render_frame(scene, W, H, spp, bands, jobs, tmp):
    exe = {60: HARNESS60, 3: HARNESSRGB}.get(bands, HARNESS)
    strips = np.linspace(0, H, jobs + 1).astype(int)
    procs = []
    for j in range(jobs):
        y0, y1 = int(strips[j]), int(strips[j + 1])
        fn = os.path.join(tmp, "strip%d.f32" % j)
        args = [exe, os.path.join(SCENES, scene), "--res", str(W), str(H), "--spp", str(spp), "--seed", "0",
                "--maxdepth", "5", "--window", "0", str(W + 1), str(y0 - 1), str(y1 + 1), "--raw", fn]
        # sample pixels [0, W + 1) x [y0 - 1, y1 + 1) (end-exclusive; x0 < 0 would mean no window): the
        # sample extent ends at W + 1 (film.cpp GetSampleExtent), and samples at exactly x = W land on
        # film pixel W - 1
        procs.append((y0, y1, fn, subprocess.Popen(args, cwd=SCENES, stdout=subprocess.DEVNULL)))
    film = None
    for y0, y1, fn, p in procs:
        if p.wait() != 0:
            raise SystemExit("harness failed on rows %d-%d" % (y0, y1))
        raw = np.fromfile(fn, dtype=np.int32)
        FW, FH, N = raw[:3]
        f = raw[3:].view(np.float32).reshape(FH, FW, N)
        if film is None:
            film = np.zeros_like(f)
        film[y0:y1] = f[y0:y1]
    return film


def main():
    jobs = 8
    argv = sys.argv[1:]
    if "--jobs" in argv:
        i = argv.index("--jobs")
        jobs = int(argv[i + 1])
        del argv[i:i + 2]
    for cfg in argv or ["c2", "c5"]:
        name, scene, W, H, spp, bands = FRAMES[cfg]
        t = time.time()
        with tempfile.TemporaryDirectory() as tmp:
            film = render_frame(scene, W, H, spp, bands, jobs, tmp)
        hs, sm, mx = tile_digest(film)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), hash=hs, sum=sm, absmax=mx,
                            config=np.array([W, H, spp, 0, 5, bands, TILE], np.int32))
        print("%s: %d tiles, film sum %.6e, %.0f s" % (name, hs.size, sm.sum(), time.time() - t), flush=True)


if __name__ == "__main__":
    main()
