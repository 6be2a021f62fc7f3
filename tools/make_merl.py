"""Write a synthetic MERL-format measured BRDF (the RegularHalfangleBRDF file format read by
materials/measured.cpp:133-175): three int32 dimensions whose product is 90 x 90 x 180,
then, per RGB channel, 90*90*180 float64 samples with delta-phi the minor index, then delta
theta, then sqrt(theta_h) (the major index).  The MERL database itself is not in the
reference tree, so the tests use this deterministic table: a smooth specular-plus-diffuse
lobe per channel, with a band of negative samples that the loader clamps to 0.
Usage: python tools/make_merl.py OUT.merl  (35 MB; written by the tests into a temp dir)"""
import sys

import numpy as np

NTH, NTD, NPD = 90, 90, 180


def table():
    th = (np.arange(NTH) + .5) / NTH                   # sqrt(theta_h / (pi/2))
    td = (np.arange(NTD) + .5) / NTD * (np.pi / 2)     # theta_d
    pd = (np.arange(NPD) + .5) / NPD * np.pi           # phi_d
    TH, TD, PD = np.meshgrid(th, td, pd, indexing="ij")
    out = []
    for c, (kd, ks, n) in enumerate([(0.35, 1800.0, 9.0), (0.22, 1500.0, 12.0), (0.10, 1200.0, 16.0)]):
        spec = ks * np.exp(-n * TH * TH) * (1.0 + 0.3 * np.cos(PD)) * np.cos(TD) ** 2
        v = 1500.0 * kd + spec + 40.0 * np.sin(7.0 * TD + c) * np.cos(3.0 * PD)
        v[:, :, 170:] -= 3000.0                          # negative samples: clamped by the loader
        out.append(v.reshape(-1))
    return out


def write(path):
    chans = table()
    with open(path, "wb") as f:
        np.array([NPD, NTD, NTH], np.int32).tofile(f)
        for v in chans:
            v.astype("<f8").tofile(f)


if __name__ == "__main__":
    write(sys.argv[1])
