"""Writes tests/golden/killeroo_control.npz: the Loop-subdivision control mesh of the
reference's killeroo (scenes/geometry/killeroo.pbrt: its "integer indices" and "point P",
parsed as the pbrt parser does -- decimal -> double -> float) and its "nlevels".  Input data of
the GPU subdivider's timing and parity test (tests/test_loop.py); run in the build container."""
import os
import re
import sys

import numpy as np

SRC = "/root/reference/scenes/geometry/killeroo.pbrt"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "killeroo_control.npz")


def main():
    s = open(SRC).read()
    vi = np.array(re.search(r'"integer indices"\s*\[([^\]]*)\]', s).group(1).split(), dtype=np.int64).astype(np.int32)
    P = np.array([np.float32(float(t)) for t in re.search(r'"point P"\s*\[([^\]]*)\]', s).group(1).split()], np.float32)
    levels = int(re.search(r'"integer nlevels"\s*\[([^\]]*)\]', s).group(1))
    np.savez_compressed(OUT, vi=vi.reshape(-1, 3), P=P.reshape(-1, 3), levels=np.int32(levels))
    print("wrote", OUT, vi.size // 3, "faces", P.size // 3, "vertices", levels, "levels")


if __name__ == "__main__":
    sys.exit(main())
