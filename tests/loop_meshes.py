"""Synthetic Loop-subdivision control meshes covering every vertex rule of
shapes/loopsubdiv.cpp: closed meshes with interior valences 3, 4, 5, 6 and 7 (regular and
irregular one-ring weights, loopsubdiv.cpp:245-259), open meshes with boundary valences 2, 3, 4
and > 4 (the boundary rule and every branch of the boundary tangent, :361-389)."""
import numpy as np


def icosahedron():
    t = (1 + 5 ** .5) / 2
    P = np.array([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
                  [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], np.float32)
    F = [[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2], [10, 7, 6],
         [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5], [2, 4, 11], [6, 2, 10],
         [8, 6, 7], [9, 8, 1]]
    return np.array(F, np.int32), P


def tetrahedron():
    P = np.array([[1, 1, 1], [-1, -1, 1], [-1, 1, -1], [1, -1, -1]], np.float32)
    return np.array([[0, 1, 2], [0, 3, 1], [0, 2, 3], [1, 3, 2]], np.int32), P


def bipyramid(k=7):
    """closed: a k-gon ring (valence 4) between two apexes of valence k"""
    a = 2 * np.pi * np.arange(k) / k
    P = np.concatenate([np.stack([np.cos(a), np.sin(a), 0.1 * np.sin(3 * a)], 1), [[0, 0, 1.3], [0, 0, -0.9]]]).astype(np.float32)
    F = [[i, (i + 1) % k, k] for i in range(k)] + [[(i + 1) % k, i, k + 1] for i in range(k)]
    return np.array(F, np.int32), P


def grid(n=5, seed=1):
    """open n x n vertex patch: corners of boundary valence 2 / 3, edges 4, interior 6"""
    rng = np.random.RandomState(seed)
    ys, xs = np.mgrid[0:n, 0:n]
    P = np.stack([xs.ravel(), ys.ravel(), 0.2 * rng.rand(n * n)], 1).astype(np.float32)
    F = []
    for y in range(n - 1):
        for x in range(n - 1):
            a, b, c, d = y * n + x, y * n + x + 1, (y + 1) * n + x, (y + 1) * n + x + 1
            F += [[a, b, d], [a, d, c]]
    return np.array(F, np.int32), P


def fan(k=6):
    """open fan: centre of boundary valence k + 1 (> 4), rim vertices of valence 2 / 3"""
    a = np.pi * np.arange(k + 1) / k
    P = np.concatenate([[[0, 0, 0.3]], np.stack([np.cos(a), np.sin(a), 0 * a], 1)]).astype(np.float32)
    F = [[0, i + 1, i + 2] for i in range(k)]
    return np.array(F, np.int32), P


MESHES = {"icosahedron": icosahedron, "tetrahedron": tetrahedron, "bipyramid": bipyramid, "grid": grid, "fan": fan}
