"""The float transcendentals (include/pbrt_libmf.h): the reference calls glibc's sinf, cosf,
powf, expf, logf, acosf, atan2f, atanf and tanf; the GPU kernels and the oracle evaluate a
restatement of those glibc 2.35 routines.

CPU: tools/libmf_check.c compares the restatement with the system libm -- its tables byte for
byte against libm's data, a strided sweep of the float inputs for the unary functions (the full
2^32 sweep is a tool run: profiles/r04/libmf_exhaustive.txt) and random / structured pairs for
powf and atan2f -- and the two oracle builds agree through their eval hooks.
GPU: the device functions (pbrtgpu_libmf_eval, the entry points k_shade calls) against glibc on
the box, bit for bit (NaN as NaN).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

UNARY = ["sinf", "cosf", "sincosf", "expf", "logf", "acosf", "atanf", "tanf"]
BINARY = ["powf", "atan2f"]


def _same(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def _inputs(fn, n, seed):
    """n float bit patterns spread over all of them, plus the renderer's own argument ranges"""
    rng = np.random.RandomState(seed)
    stride = (1 << 32) // (n // 2)   # stratified: one pattern drawn below the stride in each stratum
    bits = ((np.arange(n // 2, dtype=np.uint64) * np.uint64(stride)
             + rng.randint(0, stride, n // 2).astype(np.uint64)) & np.uint64(0xffffffff)).astype(np.uint32)
    x = bits.view(np.float32)
    dom = {"acosf": (-1.0, 1.0), "atanf": (-50.0, 50.0), "tanf": (0.0, np.pi / 2), "expf": (-104.0, 0.0),
           "logf": (0.0, 4.0)}.get(fn, (-7.0, 7.0))
    x2 = rng.uniform(dom[0], dom[1], n - n // 2).astype(np.float32)
    if fn in BINARY:
        y = rng.randint(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
        if fn == "powf":      # Blinn / microfacet: cos in [0, 1] to exponents up to 1e4
            x2 = rng.uniform(0, 1, len(x2)).astype(np.float32)
            y[n // 2:] = rng.uniform(0, 1e4, n - n // 2).astype(np.float32)
        else:                 # directions
            y[n // 2:] = rng.uniform(-1, 1, n - n // 2).astype(np.float32)
        return np.concatenate([x, x2]), y
    return np.concatenate([x, x2]), None


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("libmf") / "libmf_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tools", "libmf_check.c"), "-o", exe, "-lm", "-lpthread", "-ldl"], check=True)
    return exe


def _glibc_version():
    import ctypes
    f = ctypes.CDLL(None).gnu_get_libc_version
    f.restype = ctypes.c_char_p
    return f().decode()


def test_restatement_matches_system_libm(checker):
    """the restatement is glibc 2.35's (include/pbrt_libmf.h): compared with the running libm only
    where that is the glibc it restates"""
    if _glibc_version() != "2.35":
        pytest.skip("system glibc %s is not the 2.35 that include/pbrt_libmf.h restates" % _glibc_version())
    r = subprocess.run([checker, "--stride", "4099", "--pairs", str(1 << 22), "--threads", str(min(8, os.cpu_count() or 1))],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert r.stdout.count("found in") == 6 and r.stdout.count(" 0 differ") == 10


@pytest.mark.parametrize("fn", UNARY + BINARY)
def test_oracle_builds_agree(pg, fn):
    x, y = _inputs(fn, 1 << 16, 7)
    a = pg.oracle().libmf_eval(fn, x, y)
    b = pg.oracle(libm_float=True).libmf_eval(fn, x, y)
    assert _same(a, b).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fn", UNARY + BINARY)
def test_gpu_transcendentals_bit_exact_vs_glibc(pg, fn):
    x, y = _inputs(fn, 1 << 22, 11)
    with pg.Device(0) as d:
        g = d.libmf_eval(fn, x, y)
    ref = pg.oracle(libm_float=True).libmf_eval(fn, x, y)
    ok = _same(g, ref)
    assert ok.all(), "%s: %d of %d differ, first x %r" % (fn, (~ok).sum(), ok.size, x[np.nonzero(~ok.reshape(len(x), -1).all(1))[0][:3]])
