// loopsubdiv.hip -- Loop subdivision on the GPU (the host front end's
// setup cost; shapes/loopsubdiv.cpp).  LoopSubdiv::Refine (loopsubdiv.cpp:222-437) runs level
// by level over a pointer mesh (SDVertex / SDFace) with a std::map of edge vertices; here one
// level is five data-parallel steps over index arrays, each vertex or face written by one
// thread, with every float operation in the reference's order, so the refined mesh is the
// front end's (host/frontend.cpp LoopRefine) bit for bit apart from the last-ulp cases of
// cosf / sinf in the limit normals:
//
//   k_loop_flags  boundary / regular per control vertex (loopsubdiv.cpp:181-196)
//   k_even        even vertex j of the next level: weightOneRing / weightBoundary of vertex
//                 j (loopsubdiv.cpp:245-259), its start face child (:300-305)
//   k_edge_own    the first (face, edge) in the reference's loop order to meet an edge owns
//                 its odd vertex: face j owns edge k unless its neighbour there is a face
//                 with a smaller index; an exclusive scan of the owner flags numbers the odd
//                 vertices in the order the reference's map first sees them (:262-295)
//   k_odd         the owners' odd vertices (edge rule, boundary midpoint)
//   k_children    the four children of face j: neighbour and vertex pointers (:306-337)
//
// Vertices and faces are renumbered per level in the reference's list order (its newVertices
// / newFaces), which keeps every index comparison and every sum order.  After the levels,
// k_limit (limit positions, :340-351) and k_normals (tangents -> Cross(S, T), :352-395).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <chrono>
#include <string>
#include <unordered_map>
#include <vector>
#include "device.h"

namespace pgd {

static const int kLoopBlock = 256;
#define LNEXT(i) (((i) + 1) % 3)
#define LPREV(i) (((i) + 2) % 3)
enum { LV_BOUNDARY = 1, LV_REGULAR = 2 };

struct LoopTopo {   // one level: faces' vertices / neighbours, vertices' start face and flags
    const int *fv, *ff;
    const int *start;
    const uint32_t *flags;
    const float *P;   // [nv][3]
};

__device__ __forceinline__ int lvnum(const LoopTopo &T, int f, int v) {
    return T.fv[3 * f] == v ? 0 : (T.fv[3 * f + 1] == v ? 1 : 2);
}
__device__ __forceinline__ int lnext_face(const LoopTopo &T, int f, int v) { return T.ff[3 * f + lvnum(T, f, v)]; }
__device__ __forceinline__ int lprev_face(const LoopTopo &T, int f, int v) { return T.ff[3 * f + LPREV(lvnum(T, f, v))]; }
__device__ __forceinline__ int lnext_vert(const LoopTopo &T, int f, int v) { return T.fv[3 * f + LNEXT(lvnum(T, f, v))]; }
__device__ __forceinline__ int lprev_vert(const LoopTopo &T, int f, int v) { return T.fv[3 * f + LPREV(lvnum(T, f, v))]; }
__device__ __forceinline__ V lP(const LoopTopo &T, int v) { return v3(T.P[3 * v], T.P[3 * v + 1], T.P[3 * v + 2]); }
// P += f * Q  (Point operator* then operator+=)
__device__ __forceinline__ void lacc(V &p, float f, V q) { p.x += f * q.x; p.y += f * q.y; p.z += f * q.z; }

// SDVertex::valence (loopsubdiv.cpp:121-143)
__device__ int lvalence(const LoopTopo &T, int v, bool boundary) {
    int f = T.start[v];
    int nf = 1;
    if (!boundary) {
        while ((f = lnext_face(T, f, v)) != T.start[v]) ++nf;
        return nf;
    }
    while ((f = lnext_face(T, f, v)) != -1) ++nf;
    f = T.start[v];
    while ((f = lprev_face(T, f, v)) != -1) ++nf;
    return nf + 1;
}
// the one ring's k-th vertex (SDVertex::oneRing, loopsubdiv.cpp:451-470) is visited in order
// by these walkers: interior -- next vertex of each face around from the start face;
// boundary -- from the last face forward, its next vertex, then each face's previous vertex
struct LRing {
    int face, k;
    bool boundary;
};
__device__ __forceinline__ LRing lring_begin(const LoopTopo &T, int v, bool boundary) {
    LRing r{T.start[v], 0, boundary};
    if (boundary) {
        int f2;
        while ((f2 = lnext_face(T, r.face, v)) != -1) r.face = f2;
    }
    return r;
}
__device__ __forceinline__ int lring_next(const LoopTopo &T, int v, LRing &r) {
    int out;
    if (!r.boundary) {
        out = lnext_vert(T, r.face, v);
        r.face = lnext_face(T, r.face, v);
    } else if (r.k == 0) {
        out = lnext_vert(T, r.face, v);
    } else {
        out = lprev_vert(T, r.face, v);
        r.face = lprev_face(T, r.face, v);
    }
    ++r.k;
    return out;
}
__device__ __forceinline__ float lbeta(int valence) { return valence == 3 ? 3.f / 16.f : 3.f / (8.f * valence); }
__device__ __forceinline__ float lgamma(int valence) { return 1.f / (valence + 3.f / (8.f * lbeta(valence))); }

// LoopSubdiv::weightOneRing (loopsubdiv.cpp:440-449)
__device__ V lweight_ring(const LoopTopo &T, int v, bool boundary, int valence, float beta) {
    V P = vmul(lP(T, v), 1 - valence * beta);
    LRing r = lring_begin(T, v, boundary);
    for (int i = 0; i < valence; ++i) lacc(P, beta, lP(T, lring_next(T, v, r)));
    return P;
}
// LoopSubdiv::weightBoundary (loopsubdiv.cpp:473-482): ring[0] and ring[valence - 1]
__device__ V lweight_boundary(const LoopTopo &T, int v, int valence, float beta) {
    V P = vmul(lP(T, v), 1 - 2 * beta);
    LRing r = lring_begin(T, v, true);
    int first = lring_next(T, v, r), last = first;
    for (int i = 1; i < valence; ++i) last = lring_next(T, v, r);
    lacc(P, beta, lP(T, first));
    lacc(P, beta, lP(T, last));
    return P;
}

__global__ void k_loop_flags(int nv, LoopTopo T, uint32_t *__restrict__ flags) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    int f = T.start[v];
    do { f = lnext_face(T, f, v); } while (f != -1 && f != T.start[v]);
    const bool boundary = f == -1;
    const int val = lvalence(T, v, boundary);
    const bool regular = boundary ? val == 4 : val == 6;
    flags[v] = (boundary ? LV_BOUNDARY : 0u) | (regular ? LV_REGULAR : 0u);
}

__global__ void k_even(int nv, LoopTopo T, float *__restrict__ P1, uint32_t *__restrict__ flags1, int *__restrict__ start1) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const uint32_t fl = T.flags[v];
    const bool boundary = fl & LV_BOUNDARY;
    const int val = lvalence(T, v, boundary);
    V P;
    if (!boundary) P = lweight_ring(T, v, false, val, (fl & LV_REGULAR) ? 1.f / 16.f : lbeta(val));
    else P = lweight_boundary(T, v, val, 1.f / 8.f);
    P1[3 * v] = P.x; P1[3 * v + 1] = P.y; P1[3 * v + 2] = P.z;
    flags1[v] = fl;
    const int sf = T.start[v];
    start1[v] = 4 * sf + lvnum(T, sf, v);
}

__global__ void k_edge_own(int nf, LoopTopo T, uint32_t *__restrict__ own) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 3 * nf) return;
    const int f2 = T.ff[e];
    own[e] = (f2 == -1 || e / 3 < f2) ? 1u : 0u;
}

// the odd vertex id of edge k of face f (owned by f or by its neighbour there)
__device__ __forceinline__ int lodd_id(const LoopTopo &T, const uint32_t *rank, int nv, int f, int k) {
    const int f2 = T.ff[3 * f + k];
    if (f2 == -1 || f < f2) return nv + (int)rank[3 * f + k];
    const int a = T.fv[3 * f + k], b = T.fv[3 * f + LNEXT(k)];
    int k2 = 0;
    for (int i = 0; i < 3; ++i) {
        const int c = T.fv[3 * f2 + i], d = T.fv[3 * f2 + LNEXT(i)];
        if ((c == a && d == b) || (c == b && d == a)) k2 = i;
    }
    return nv + (int)rank[3 * f2 + k2];
}

__global__ void k_odd(int nf, int nv, LoopTopo T, const uint32_t *__restrict__ rank, float *__restrict__ P1,
                      uint32_t *__restrict__ flags1, int *__restrict__ start1) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 3 * nf) return;
    const int f = e / 3, k = e % 3, f2 = T.ff[e];
    if (!(f2 == -1 || f < f2)) return;
    const int id = nv + (int)rank[e];
    const int e0 = T.fv[e], e1 = T.fv[3 * f + LNEXT(k)];
    const int a = min(e0, e1), b = max(e0, e1);
    V P;
    if (f2 == -1) {
        P = vmul(lP(T, a), 0.5f);
        lacc(P, 0.5f, lP(T, b));
    } else {
        P = vmul(lP(T, a), 3.f / 8.f);
        lacc(P, 3.f / 8.f, lP(T, b));
        int c = -1, d = -1;   // otherVert of this face, of the neighbour
        for (int i = 0; i < 3; ++i) {
            if (T.fv[3 * f + i] != a && T.fv[3 * f + i] != b) c = T.fv[3 * f + i];
            if (T.fv[3 * f2 + i] != a && T.fv[3 * f2 + i] != b) d = T.fv[3 * f2 + i];
        }
        lacc(P, 1.f / 8.f, lP(T, c));
        lacc(P, 1.f / 8.f, lP(T, d));
    }
    P1[3 * id] = P.x; P1[3 * id + 1] = P.y; P1[3 * id + 2] = P.z;
    flags1[id] = LV_REGULAR | (f2 == -1 ? LV_BOUNDARY : 0u);
    start1[id] = 4 * f + 3;
}

__global__ void k_children(int nf, int nv, LoopTopo T, const uint32_t *__restrict__ rank, int *__restrict__ fv1,
                           int *__restrict__ ff1) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    int cv[4][3], cf[4][3];
    for (int k = 0; k < 3; ++k) {
        cf[3][k] = 4 * f + LNEXT(k);
        cf[k][LNEXT(k)] = 4 * f + 3;
        int f2 = T.ff[3 * f + k];
        cf[k][k] = f2 != -1 ? 4 * f2 + lvnum(T, f2, T.fv[3 * f + k]) : -1;
        f2 = T.ff[3 * f + LPREV(k)];
        cf[k][LPREV(k)] = f2 != -1 ? 4 * f2 + lvnum(T, f2, T.fv[3 * f + k]) : -1;
    }
    for (int k = 0; k < 3; ++k) {
        cv[k][k] = T.fv[3 * f + k];   // the even child keeps the vertex's index
        const int vert = lodd_id(T, rank, nv, f, k);
        cv[k][LNEXT(k)] = vert;
        cv[LNEXT(k)][k] = vert;
        cv[3][k] = vert;
    }
    for (int c = 0; c < 4; ++c)
        for (int k = 0; k < 3; ++k) {
            fv1[3 * (4 * f + c) + k] = cv[c][k];
            ff1[3 * (4 * f + c) + k] = cf[c][k];
        }
}

__global__ void k_limit(int nv, LoopTopo T, float *__restrict__ Pl) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const bool boundary = T.flags[v] & LV_BOUNDARY;
    const int val = lvalence(T, v, boundary);
    const V P = boundary ? lweight_boundary(T, v, val, 1.f / 5.f) : lweight_ring(T, v, false, val, lgamma(val));
    Pl[3 * v] = P.x; Pl[3 * v + 1] = P.y; Pl[3 * v + 2] = P.z;
}

// T.P = the limit positions here (the reference assigns them before the tangents)
__global__ void k_normals(int nv, LoopTopo T, float *__restrict__ N) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const bool boundary = T.flags[v] & LV_BOUNDARY;
    const int val = lvalence(T, v, boundary);
    V S = v3(0.f, 0.f, 0.f), Tg = v3(0.f, 0.f, 0.f);
    LRing r = lring_begin(T, v, boundary);
    if (!boundary) {
        for (int k = 0; k < val; ++k) {
            const V q = lP(T, lring_next(T, v, r));
            lacc(S, COSF(2.f * kPi * k / val), q);
            lacc(Tg, SINF(2.f * kPi * k / val), q);
        }
    } else {
        // ring[0 .. 3] and ring[valence - 1]; larger valences walk the ring again below
        V p[4];
        V last = v3(0.f, 0.f, 0.f);
        for (int k = 0; k < val; ++k) {
            const V q = lP(T, lring_next(T, v, r));
            if (k < 4) p[k] = q;
            last = q;
        }
        const V c = lP(T, v);
        S = vsub(last, p[0]);
        if (val == 2) Tg = vsub(vadd(p[0], p[1]), vmul(c, 2.f));
        else if (val == 3) Tg = vsub(p[1], c);
        else if (val == 4)
            Tg = vadd(vadd(vadd(vadd(vmul(p[0], -1.f), vmul(p[1], 2.f)), vmul(p[2], 2.f)), vmul(p[3], -1.f)), vmul(c, -2.f));
        else {
            const float theta = kPi / float(val - 1);
            Tg = vmul(vadd(p[0], last), SINF(theta));
            LRing r2 = lring_begin(T, v, true);
            (void)lring_next(T, v, r2);
            for (int k = 1; k < val - 1; ++k) {
                const float wt = (2 * COSF(theta) - 2) * SINF((k) * theta);
                lacc(Tg, wt, lP(T, lring_next(T, v, r2)));
            }
            Tg = vneg(Tg);
        }
    }
    const V n = vcross(S, Tg);
    N[3 * v] = n.x; N[3 * v + 1] = n.y; N[3 * v + 2] = n.z;
}

#define LSCHK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { *err = std::string(#x) + ": " + hipGetErrorString(e_); rc = -(1000 + (int)e_); goto done; } \
    } while (0)

// LoopSubdiv (loopsubdiv.cpp:147-198) control mesh -> Refine's limit mesh (object space).
// Sizes only when P_out is null.  Returns 0 or a negative error (err set).
int loop_subdivide(hipStream_t stream, int nf, int nv, const int32_t *vi, const float *P, int levels, int32_t *nv_out,
                   float *P_out, float *N_out, int32_t *vi_out, double *ms_out, std::string *err) {
    const auto w0 = std::chrono::steady_clock::now();
    // the constructor's topology (host): start faces, neighbours by edge pairing
    std::vector<int> fv(vi, vi + 3 * (size_t)nf), ff(3 * (size_t)nf, -1), start(nv, -1);
    for (int i = 0; i < nf; ++i)
        for (int j = 0; j < 3; ++j) {
            const int v = fv[3 * i + j];
            if (v < 0 || v >= nv) { *err = "vertex index out of range"; return -1; }
            start[v] = i;
        }
    for (int v = 0; v < nv; ++v)
        if (start[v] < 0) { *err = "vertex used by no face (the reference's LoopSubdiv cannot refine it)"; return -1; }
    {
        std::unordered_map<uint64_t, int> edges;   // (min, max) -> first face edge 3 f + k
        edges.reserve(3 * (size_t)nf);
        for (int i = 0; i < nf; ++i)
            for (int k = 0; k < 3; ++k) {
                const int a = fv[3 * i + k], b = fv[3 * i + LNEXT(k)];
                const uint64_t key = ((uint64_t)(uint32_t)std::min(a, b) << 32) | (uint32_t)std::max(a, b);
                auto it = edges.find(key);
                if (it == edges.end()) edges.emplace(key, 3 * i + k);
                else {
                    ff[it->second] = i;
                    ff[3 * i + k] = it->second / 3;
                    edges.erase(it);
                }
            }
    }
    // sizes per level: odd vertices = owned edges = (3 nf + boundary edges) / 2
    long long nb = 0;
    for (int e = 0; e < 3 * nf; ++e) nb += ff[e] == -1;
    long long NF = nf, NV = nv, B = nb;
    std::vector<long long> lnf(levels + 1), lnv(levels + 1);
    lnf[0] = NF; lnv[0] = NV;
    for (int l = 0; l < levels; ++l) {
        NV += (3 * NF + B) / 2;
        NF *= 4;
        B *= 2;
        lnf[l + 1] = NF; lnv[l + 1] = NV;
    }
    if (NF > (1ll << 28) || NV > (1ll << 28)) { *err = "refined mesh too large"; return -1; }
    *nv_out = (int32_t)NV;
    if (!P_out) return 0;
    int rc = 0;
    int *dfv[2] = {}, *dff[2] = {}, *dst[2] = {};
    uint32_t *dfl[2] = {}, *dOwn = nullptr, *dRank = nullptr;
    float *dP[2] = {}, *dN = nullptr;
    void *dTmp = nullptr;
    size_t tmpBytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int cur = 0;
    const size_t mf = (size_t)NF, mv = (size_t)NV;
    LSCHK(hipEventCreate(&e0));
    LSCHK(hipEventCreate(&e1));
    for (int b = 0; b < 2; ++b) {
        LSCHK(hipMalloc(&dfv[b], 12 * mf));
        LSCHK(hipMalloc(&dff[b], 12 * mf));
        LSCHK(hipMalloc(&dst[b], 4 * mv));
        LSCHK(hipMalloc(&dfl[b], 4 * mv));
        LSCHK(hipMalloc(&dP[b], 12 * mv));
    }
    LSCHK(hipMalloc(&dN, 12 * mv));
    LSCHK(hipMalloc(&dOwn, 12 * mf / 4 + 4));
    LSCHK(hipMalloc(&dRank, 12 * mf / 4 + 4));
    LSCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmpBytes, dOwn, dRank, (int)std::max<long long>(1, 3 * lnf[std::max(0, levels - 1)]), stream));
    LSCHK(hipMalloc(&dTmp, std::max<size_t>(tmpBytes, 16)));
    LSCHK(hipMemcpyAsync(dfv[0], fv.data(), 12 * (size_t)nf, hipMemcpyHostToDevice, stream));
    LSCHK(hipMemcpyAsync(dff[0], ff.data(), 12 * (size_t)nf, hipMemcpyHostToDevice, stream));
    LSCHK(hipMemcpyAsync(dst[0], start.data(), 4 * (size_t)nv, hipMemcpyHostToDevice, stream));
    LSCHK(hipMemcpyAsync(dP[0], P, 12 * (size_t)nv, hipMemcpyHostToDevice, stream));
    LSCHK(hipEventRecord(e0, stream));
    {
        LoopTopo T{dfv[0], dff[0], dst[0], nullptr, dP[0]};
        hipLaunchKernelGGL(k_loop_flags, dim3((nv + kLoopBlock - 1) / kLoopBlock), dim3(kLoopBlock), 0, stream, nv, T, dfl[0]);
        LSCHK(hipGetLastError());
    }
    for (int l = 0; l < levels; ++l) {
        const int n = cur ^ 1, F = (int)lnf[l], Vn = (int)lnv[l];
        LoopTopo T{dfv[cur], dff[cur], dst[cur], dfl[cur], dP[cur]};
        const int gv = (Vn + kLoopBlock - 1) / kLoopBlock, ge = (3 * F + kLoopBlock - 1) / kLoopBlock,
                  gf = (F + kLoopBlock - 1) / kLoopBlock;
        hipLaunchKernelGGL(k_even, dim3(gv), dim3(kLoopBlock), 0, stream, Vn, T, dP[n], dfl[n], dst[n]);
        LSCHK(hipGetLastError());
        hipLaunchKernelGGL(k_edge_own, dim3(ge), dim3(kLoopBlock), 0, stream, F, T, dOwn);
        LSCHK(hipGetLastError());
        LSCHK(hipcub::DeviceScan::ExclusiveSum(dTmp, tmpBytes, dOwn, dRank, 3 * F, stream));
        hipLaunchKernelGGL(k_odd, dim3(ge), dim3(kLoopBlock), 0, stream, F, Vn, T, dRank, dP[n], dfl[n], dst[n]);
        LSCHK(hipGetLastError());
        hipLaunchKernelGGL(k_children, dim3(gf), dim3(kLoopBlock), 0, stream, F, Vn, T, dRank, dfv[n], dff[n]);
        LSCHK(hipGetLastError());
        cur = n;
    }
    {
        const int Vn = (int)NV, n = cur ^ 1, gv = (Vn + kLoopBlock - 1) / kLoopBlock;
        LoopTopo T{dfv[cur], dff[cur], dst[cur], dfl[cur], dP[cur]};
        hipLaunchKernelGGL(k_limit, dim3(gv), dim3(kLoopBlock), 0, stream, Vn, T, dP[n]);
        LSCHK(hipGetLastError());
        T.P = dP[n];
        hipLaunchKernelGGL(k_normals, dim3(gv), dim3(kLoopBlock), 0, stream, Vn, T, dN);
        LSCHK(hipGetLastError());
        LSCHK(hipEventRecord(e1, stream));
        LSCHK(hipMemcpyAsync(P_out, dP[n], 12 * mv, hipMemcpyDeviceToHost, stream));
        LSCHK(hipMemcpyAsync(N_out, dN, 12 * mv, hipMemcpyDeviceToHost, stream));
        LSCHK(hipMemcpyAsync(vi_out, dfv[cur], 12 * mf, hipMemcpyDeviceToHost, stream));
        LSCHK(hipStreamSynchronize(stream));
    }
    if (ms_out) {
        float m = 0.f;
        LSCHK(hipEventElapsedTime(&m, e0, e1));
        ms_out[0] = m;
        ms_out[1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    }
done:
    for (int b = 0; b < 2; ++b)
        for (void *p : {(void *)dfv[b], (void *)dff[b], (void *)dst[b], (void *)dfl[b], (void *)dP[b]})
            if (p) (void)hipFree(p);
    for (void *p : {(void *)dN, (void *)dOwn, (void *)dRank, dTmp})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

}  // namespace pgd
