"""Port-vs-reference CPU calibration (BASELINE.md plan step 2; TEST INFRASTRUCTURE, build
container only): the reference's own path (oracle/_ref harness, unmodified reference TUs,
one thread) and the C restatement (oracle/liboracle.so, one thread) render the same windows
of the same frame (C2: killeroo-simple 700x700@256, 32 bands).  The harness's parse + BVH
build time (an empty window) is subtracted.  Writes profiles/cpu_calibration.json.
Usage: python tools/calibrate_cpu.py"""
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "b32", "pbrt_ref_harness")
SCENES = "/root/reference/scenes"
WINDOWS = [(300, 332, 300, 332), (100, 132, 500, 532), (500, 532, 200, 232)]   # x0 x1 y0 y1 (sample pixels)


def harness(win):
    t = time.perf_counter()
    subprocess.run([HARNESS, os.path.join(SCENES, "killeroo-simple.pbrt"), "--res", "700", "700", "--spp", "256",
                    "--window"] + [str(v) for v in win], check=True, cwd=SCENES, capture_output=True)
    return time.perf_counter() - t


def main():
    setup = min(harness((0, 0, 0, 0)) for _ in range(3))
    scene = pg.Scene.load(os.path.join(ROOT, "scenes", "killeroo-simple.pack"))
    o = pg.oracle(libm_float=True)
    rows = []
    for w in WINDOWS:
        n = (w[1] - w[0]) * (w[3] - w[2]) * 256
        tr = harness(w) - setup
        t = time.perf_counter()
        o.render(scene, window=w, threads=1)
        tp = time.perf_counter() - t
        rows.append({"window": w, "paths": n, "reference_s": round(tr, 3), "port_s": round(tp, 3),
                     "reference_Mpaths_s": round(n / tr / 1e6, 4), "port_Mpaths_s": round(n / tp / 1e6, 4)})
    ref = sum(r["paths"] for r in rows) / sum(r["reference_s"] for r in rows) / 1e6
    port = sum(r["paths"] for r in rows) / sum(r["port_s"] for r in rows) / 1e6
    cpu = "unknown"
    for ln in open("/proc/cpuinfo"):
        if ln.startswith("model name"):
            cpu = ln.split(":", 1)[1].strip()
            break
    out = {"what": "one-thread Mpaths/s of the reference harness (unmodified reference TUs, -O2) and of the C restatement "
                   "(liboracle_libm.so, -O2) on the same windows of C2 (killeroo-simple 700x700@256, 32 bands); harness "
                   "parse + BVH build (%.2f s) subtracted" % setup,
           "host": cpu, "nproc": os.cpu_count(), "python": platform.python_version(),
           "reference_Mpaths_s_per_core": round(ref, 4), "port_Mpaths_s_per_core": round(port, 4),
           "port_over_reference": round(port / ref, 3), "windows": rows}
    json.dump(out, open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
