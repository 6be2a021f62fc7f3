"""tools/make_packs.py -- build scene packs (scenes/*.pack) from the reference scene files.

Run in the build container (needs /root/reference).  The packs are the flattened scenes
produced by this repository's own front end (pbrt-v2-spectral_amd/host) from the unchanged
pbrt scene files, so the GPU box -- which has no /root/reference -- can render the config
scenes.  Resolution / spp / maxdepth stay overridable at load time.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg  # noqa: E402

REF = "/root/reference/scenes"
# (pack name, scene file, bands, xres, yres, spp) -- SURVEY App. B overrides
PACKS = [
    ("killeroo-simple", "killeroo-simple.pbrt", 32, 700, 700, 256),
    ("anim-killeroos-moving", "anim-killeroos-moving.pbrt", 32, 600, 600, 512),
    ("bunny", "bunny.pbrt", 32, 1920, 1080, 1024),
    ("metal", "metal.pbrt", 60, 400, 400, 4096),
    ("coverage", os.path.join(ROOT, "tests", "scenes", "coverage.pbrt"), 32, 64, 48, 8),
    # C1: the reference's RGB build (Spectrum = RGBSpectrum), 400x400 at 64 spp
    ("killeroo-simple-rgb", "killeroo-simple.pbrt", 3, 400, 400, 64),
    # the upstream 30-band, 400-700 nm sampling (spectrum.h.original:36-38; BASELINE's "30 bands")
    ("killeroo-simple-b30", "killeroo-simple.pbrt", 30, 700, 700, 256),
    ("coverage-b30", os.path.join(ROOT, "tests", "scenes", "coverage.pbrt"), 30, 64, 48, 8),
    # C2's scene in the 60-band build (C4's band count): the 60-band kernels of the plain variants
    ("killeroo-simple-b60", "killeroo-simple.pbrt", 60, 700, 700, 256),
    # decoded TGA / PFM image maps in MIPMap pyramids (tests/scenes/textures, tools/make_images.py)
    ("imagemap", os.path.join(ROOT, "tests", "scenes", "imagemap.pbrt"), 32, 64, 48, 4),
    # an animated camera (coverage.pbrt's world)
    ("animcam", os.path.join(ROOT, "tests", "scenes", "animcam.pbrt"), 32, 64, 48, 4),
    # every material parameter as a texture (two textured spectra, textured floats, raw metal eta / k)
    ("textured", os.path.join(ROOT, "tests", "scenes", "textured.pbrt"), 32, 64, 48, 4),
    # an image-based infinite light (decoded lat-long PFM: radiance MIPMap + Distribution2D)
    ("envmap", os.path.join(ROOT, "tests", "scenes", "envmap.pbrt"), 32, 64, 48, 4),
    # spot and distant lights beside an area light
    ("lights", os.path.join(ROOT, "tests", "scenes", "lights.pbrt"), 32, 64, 48, 4),
    # the orthographic camera
    ("ortho", os.path.join(ROOT, "tests", "scenes", "ortho.pbrt"), 32, 64, 48, 4),
    # heightfield shapes
    ("heightfield", os.path.join(ROOT, "tests", "scenes", "heightfield.pbrt"), 32, 64, 48, 4),
    # cylinders
    ("cylinder", os.path.join(ROOT, "tests", "scenes", "cylinder.pbrt"), 32, 64, 48, 4),
    # the fork's anisotropic Ward material
    ("anisoward", os.path.join(ROOT, "tests", "scenes", "anisoward.pbrt"), 32, 64, 48, 4),
    # shinymetal
    ("shinymetal", os.path.join(ROOT, "tests", "scenes", "shinymetal.pbrt"), 32, 64, 48, 4),
    # spherical / cylindrical / planar texture mappings
    ("mappings", os.path.join(ROOT, "tests", "scenes", "mappings.pbrt"), 32, 64, 48, 4),
    # Checkerboard2DTexture
    ("checker", os.path.join(ROOT, "tests", "scenes", "checker.pbrt"), 32, 64, 48, 4),
    # NURBS surfaces
    ("nurbs", os.path.join(ROOT, "tests", "scenes", "nurbs.pbrt"), 32, 64, 48, 4),
]


def main():
    out = os.path.join(ROOT, "scenes")
    os.makedirs(out, exist_ok=True)
    only = sys.argv[2:] if len(sys.argv) > 2 and sys.argv[1] == "--only" else None   # --only NAME ...
    for name, fn, bands, xr, yr, spp in PACKS:
        if only and name not in only:
            continue
        # the configs render with "path" (SURVEY App. B); load a pack with integrator="directlighting"
        # to render it with the DirectLightingIntegrator the scene files name
        s = pg.Scene.load(os.path.join(REF, fn), xres=xr, yres=yr, spp=spp, maxdepth=-1 if name.startswith(("coverage", "imagemap", "animcam", "textured", "envmap", "lights", "ortho", "heightfield", "cylinder", "anisoward", "shinymetal", "nurbs", "mappings", "checker")) else 5,
                          bands=bands, integrator="path")
        path = os.path.join(out, name + ".pack")
        s.save_pack(path)
        print(name, s.info(), os.path.getsize(path))


if __name__ == "__main__":
    main()
