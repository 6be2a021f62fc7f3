"""INTEGRATION.md's C example is compiled and linked against include/ and both product
libraries here, then run: the host front end loads the scene pack, and without a GPU the context
creation fails with a message (exit 2) -- never a silent CPU fallback; with one, it renders."""
import os
import re
import subprocess

from conftest import ROOT


def test_c_example_compiles_links_and_runs(tmp_path):
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. C usage"):doc.index("## 3.")]
    src = re.search(r"```c\n(.*?)```", sec, re.S).group(1)
    c = tmp_path / "example.c"
    c.write_text(src)
    lib = os.path.join(ROOT, "pbrt-v2-spectral_amd", "lib")
    exe = str(tmp_path / "example")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o", exe,
                    "-L" + lib, "-lpbrtgpu", "-lpbrthost", "-Wl,-rpath," + lib, "-Wl,-rpath-link,/opt/rocm/lib"],
                   check=True)
    r = subprocess.run([exe, os.path.join(ROOT, "scenes", "killeroo-simple.pack")], capture_output=True, text=True,
                       timeout=300, cwd=str(tmp_path))
    if r.returncode == 0:    # a GPU is visible: the whole C2 frame rendered and written
        assert os.path.getsize(str(tmp_path / "killeroo.dat")) > 700 * 700 * 32 * 8
    else:
        assert r.returncode == 2 and r.stderr.strip(), (r.returncode, r.stderr)
