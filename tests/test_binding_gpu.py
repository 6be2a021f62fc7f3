"""The reference-side binding's call sequence on the GPU: tests/cpp/render_dat.cpp replays
GpuPathRenderer::Render (integration/gpupathrenderer.cpp:37-92) -- context per device,
pbrthost_load, pbrtgpu_scene_upload, pbrtgpu_render_multi over 16x16 tiles, then
pbrthost_write_dat_scene -- as a C++ program over the C ABI, and its .dat is compared with the
.dat the reference's own spectral film wrote for the same render
(tests/golden/killeroo_dat_40x32s4.npz, tools/make_golden.py --only dat)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PACKS, ROOT

EXE = os.path.join(ROOT, "pbrt-v2-spectral_amd", "lib", "render_dat")


def _payload(raw):
    """line 1 and the float64 planes of a .dat (the reference film has no lens line 2)"""
    l1 = raw.index(b"\n") + 1
    W, H, N = [int(v) for v in raw[:l1].split()]
    body = raw[l1:]
    if len(body) != W * H * N * 8:
        l2 = body.index(b"\n") + 1
        assert body[:l2] == b"0 0 -nan\n"
        body = body[l2:]
    return raw[:l1], np.frombuffer(body, np.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("slices", [1, 2])
def test_binding_call_sequence_writes_reference_dat(tmp_path, slices):
    assert os.path.exists(EXE), "build first: make -C pbrt-v2-spectral_amd"
    g = np.load(os.path.join(GOLDEN, "killeroo_dat_40x32s4.npz"))
    H, W, N = g["film"].shape
    out = str(tmp_path / "k.dat")
    r = subprocess.run([EXE, os.path.join(PACKS, "killeroo-simple.pack"), out, str(W), str(H), "4", "1", str(slices)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    h_ref, ref = _payload(g["dat"].tobytes())
    h_mine, mine = _payload(open(out, "rb").read())
    assert h_mine == h_ref == b"%d %d %d\n" % (W, H, N)
    assert mine.shape == ref.shape
    # image L-inf relative error (BASELINE.json north star); most values bit for bit (a pixel
    # differs when one of its 4 paths meets a last-ulp transcendental difference)
    assert np.abs(mine - ref).max() / np.abs(ref).max() < 1e-4
    assert (mine == ref).mean() >= 0.9
