/* oracle/pathtrace.c -- TEST INFRASTRUCTURE: CPU restatement of the reference hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (libpbrtgpu.so) never
 * links or calls it.
 *
 * Parity pinning: compiled with -DORACLE_LIBM_FLOAT (calls into glibc's float transcendentals,
 * as the reference build does) it reproduces the reference harness (oracle/_ref, which runs
 * the reference's own PathIntegrator/BVH/BSDF/light/camera code) bit for bit; compiled
 * without it, sinf/cosf/powf/expf/logf/acosf/atan2f/tanf/atanf are include/pbrt_libmf.h, the
 * restatement of those glibc routines the HIP kernels compile from the same header (pinned to
 * the system libm over every float input by tools/libmf_check.c), see DESIGN.md §3.2.  The
 * lens camera's double-precision diffraction terms use include/pbrt_fmath.h in that build.
 *
 * It consumes the flattened scene of include/pbrtgpu.h and follows, function by function:
 *   samplerrenderer.cpp:60-164,225-247  render loop, NaN/inf guard, SamplerRenderer::Li
 *   path.cpp:44-115                     PathIntegrator::Li
 *   integrator.cpp:74-166               UniformSampleOneLight / EstimateDirect
 *   bvh.cpp:118-140,380-481             slab test, Intersect, IntersectP
 *   trianglemesh.cpp:119-360            Triangle::Intersect/IntersectP/GetShadingGeometry
 *   sphere.cpp, disk.cpp, shape.cpp     quadric intersection / sampling / pdf
 *   material.cpp:39-81                  Material::Bump (constant displacement)
 *   matte.cpp, plastic.cpp, mirror.cpp, substrate.cpp   per-hit BSDF assembly
 *   reflection.cpp:52-618               BSDF and BxDFs
 *   light.cpp, diffuse.cpp, point.cpp   lights
 *   perspective.cpp:73-106              camera rays
 *   spectralImage.cpp:77-152            film accumulation (box filter)
 *   rng.cpp                             MT19937
 *   montecarlo.{h,cpp}                  sampling helpers
 * Compile with -ffp-contract=off (the reference x86-64 build has no FMA contraction).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>
#include "pbrtgpu.h"

#define MAXB PBRTGPU_MAX_BANDS
#define PI_F 3.14159265358979323846f
#define INV_PI_F 0.31830988618379067154f
#define INV_TWOPI_F 0.15915494309189533577f
#define ONE_MINUS_EPS 0x1.fffffep-1f

#include "pbrt_fmath.h"
#ifdef ORACLE_LIBM_FLOAT
#define SINF sinf
#define COSF cosf
#define POWF powf
#define EXPF expf
#define ACOSF acosf
#define ATAN2F atan2f
#define TANF tanf
#define ATANF atanf
#define DSIN sin   /* double: the lens camera's diffraction (realisticDiffraction.cpp:1057-1150) */
#define DCOS cos
#define DACOS acos
#define DATAN atan
#define DLOG log
#else
/* the definition shared with the GPU: glibc's float routines restated, include/pbrt_libmf.h */
#include "pbrt_libmf.h"
static inline float SINF(float x) { return libmf_sinf(x); }
static inline float COSF(float x) { return libmf_cosf(x); }
static inline float POWF(float x, float y) { return libmf_powf(x, y); }
static inline float EXPF(float x) { return libmf_expf(x); }
static inline float ACOSF(float x) { return libmf_acosf(x); }
static inline float ATAN2F(float y, float x) { return libmf_atan2f(y, x); }
static inline float TANF(float x) { return libmf_tanf(x); }
static inline float ATANF(float x) { return libmf_atanf(x); }
#define DSIN pbrt_fm_sin
#define DCOS pbrt_fm_cos
#define DACOS pbrt_fm_acos
#define DATAN pbrt_fm_atan
#define DLOG pbrt_fm_log
#endif

/* ------------------------------------------------------------------ vector math */
typedef struct { float x, y, z; } V;
static inline V v3(float x, float y, float z) { V r; r.x = x; r.y = y; r.z = z; return r; }
static inline V vadd(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V vsub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V vneg(V a) { return v3(-a.x, -a.y, -a.z); }
static inline V vmul(V a, float f) { return v3(f * a.x, f * a.y, f * a.z); }
static inline V vdiv(V a, float f) { float inv = 1.f / f; return v3(a.x * inv, a.y * inv, a.z * inv); }
static inline float vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float vlen2(V a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float vlen(V a) { return sqrtf(vlen2(a)); }
static inline V vnorm(V a) { return vdiv(a, vlen(a)); }
static inline V vcross(V a, V b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return v3((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx)));
}
static inline float vcomp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline float fminf_(float a, float b) { return (b < a) ? b : a; }   /* std::min */
static inline float fmaxf_(float a, float b) { return (a < b) ? b : a; }   /* std::max */
static inline float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline float lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }
static inline V faceforward(V n, V v) { return (vdot(n, v) < 0.f) ? vneg(n) : n; }
static inline void coordsys(V v1, V *v2, V *v3_) {
    if (fabsf(v1.x) > fabsf(v1.y)) {
        float invLen = 1.f / sqrtf(v1.x * v1.x + v1.z * v1.z);
        *v2 = v3(-v1.z * invLen, 0.f, v1.x * invLen);
    } else {
        float invLen = 1.f / sqrtf(v1.y * v1.y + v1.z * v1.z);
        *v2 = v3(0.f, v1.z * invLen, -v1.y * invLen);
    }
    *v3_ = vcross(v1, *v2);
}
/* Transform::operator()(Point) (transform.h:184-194) */
static inline V xpoint(const float *m, V p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1.) return v3(xp, yp, zp);
    return vdiv(v3(xp, yp, zp), wp);
}
static inline V xvec(const float *m, V v) {
    return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
static inline V xnormal(const float *minv, V n) {
    return v3(minv[0] * n.x + minv[4] * n.y + minv[8] * n.z, minv[1] * n.x + minv[5] * n.y + minv[9] * n.z,
              minv[2] * n.x + minv[6] * n.y + minv[10] * n.z);
}

typedef struct { V o, d; float mint, maxt, time; } Ray;
static inline V rayat(const Ray *r, float t) { return vadd(r->o, vmul(r->d, t)); }

/* ------------------------------------------------------------------ sampling */
static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
static inline uint32_t pixel_hash(uint32_t seed, int px, int py) {
    uint32_t h = mix32(seed + 0x9E3779B9U);
    h = mix32(h ^ (uint32_t)px);
    h = mix32(h ^ ((uint32_t)py * 0x85EBCA6BU));
    return h;
}
static inline uint32_t dim_scramble(uint32_t hp, uint32_t d) { return mix32(hp ^ (0x9E3779B9U * (d + 1U))); }
static inline uint32_t perm_index(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp) {
    return s ^ (mix32(dim_scramble(hp, d) ^ 0x5BD1E995U) & (spp - 1U));
}
static inline uint32_t path_seed(uint32_t hp, uint32_t s) { return mix32(hp ^ mix32(s + 0x7F4A7C15U)); }
static inline float vdc(uint32_t n, uint32_t scramble) {   /* montecarlo.h:269-278 */
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ff) << 8) | ((n & 0xff00ff00) >> 8);
    n = ((n & 0x0f0f0f0f) << 4) | ((n & 0xf0f0f0f0) >> 4);
    n = ((n & 0x33333333) << 2) | ((n & 0xcccccccc) >> 2);
    n = ((n & 0x55555555) << 1) | ((n & 0xaaaaaaaa) >> 1);
    n ^= scramble;
    return fminf_(((n >> 8) & 0xffffff) / (float)(1 << 24), ONE_MINUS_EPS);
}
static inline float sobol2(uint32_t n, uint32_t scramble) {   /* montecarlo.h:281-285 */
    for (uint32_t v = 1u << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 0x1) scramble ^= v;
    return fminf_(((scramble >> 8) & 0xffffff) / (float)(1 << 24), ONE_MINUS_EPS);
}
static inline float s1d(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp) {
    return vdc(perm_index(hp, d, s, spp), dim_scramble(hp, d));
}
static inline void s2d(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp, float *u) {
    uint32_t sp = perm_index(hp, d, s, spp), sc = dim_scramble(hp, d);
    u[0] = vdc(sp, sc);
    u[1] = sobol2(sp, mix32(sc ^ 0x68BC21EBU));
}
/* sample slots of PathIntegrator::RequestSamples (path.cpp:33-41) + emission (2x1D):
 * 1D slot j -> dim 3+j (bounce b: lightComp 4b, lightNum 4b+1, bsdfComp 4b+2, pathComp 4b+3)
 * 2D slot k -> dim 17+k (bounce b: lightPos 3b, bsdfDir 3b+1, pathDir 3b+2) */
#define N1D 14
#define DIM_1D(j) (3u + (uint32_t)(j))
#define DIM_2D(k) (3u + N1D + (uint32_t)(k))

/* MT19937 (rng.cpp:35-100) */
typedef struct { uint32_t mt[624]; int mti; } RNG;
static void rng_seed(RNG *r, uint32_t seed) {
    r->mt[0] = seed;
    for (r->mti = 1; r->mti < 624; r->mti++) r->mt[r->mti] = (1812433253U * (r->mt[r->mti - 1] ^ (r->mt[r->mti - 1] >> 30)) + r->mti);
}
static uint32_t rng_uint(RNG *r) {
    static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
    uint32_t y;
    if (r->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (r->mt[kk] & 0x80000000U) | (r->mt[kk + 1] & 0x7fffffffU);
            r->mt[kk] = r->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        for (; kk < 623; kk++) {
            y = (r->mt[kk] & 0x80000000U) | (r->mt[kk + 1] & 0x7fffffffU);
            r->mt[kk] = r->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 0x1U];
        }
        y = (r->mt[623] & 0x80000000U) | (r->mt[0] & 0x7fffffffU);
        r->mt[623] = r->mt[396] ^ (y >> 1) ^ mag01[y & 0x1U];
        r->mti = 0;
    }
    y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}
static inline float rng_float(RNG *r) { return (rng_uint(r) & 0xffffff) / (float)(1 << 24); }

/* montecarlo.cpp:298-340 */
static void concentric_disk(float u1, float u2, float *dx, float *dy) {
    float r, theta;
    float sx = 2 * u1 - 1;
    float sy = 2 * u2 - 1;
    if (sx == 0.0 && sy == 0.0) { *dx = 0.0; *dy = 0.0; return; }
    if (sx >= -sy) {
        if (sx > sy) { r = sx; if (sy > 0.0) theta = sy / r; else theta = 8.0f + sy / r; }
        else { r = sy; theta = 2.0f - sx / r; }
    } else {
        if (sx <= sy) { r = -sx; theta = 4.0f - sy / r; }
        else { r = -sy; theta = 6.0f + sx / r; }
    }
    theta *= PI_F / 4.f;
    *dx = r * COSF(theta);
    *dy = r * SINF(theta);
}
static inline V cosine_hemisphere(float u1, float u2) {
    V r;
    concentric_disk(u1, u2, &r.x, &r.y);
    r.z = sqrtf(fmaxf_(0.f, 1.f - r.x * r.x - r.y * r.y));
    return r;
}
static inline V uniform_sphere(float u1, float u2) {
    float z = 1.f - 2.f * u1;
    float r = sqrtf(fmaxf_(0.f, 1.f - z * z));
    float phi = 2.f * PI_F * u2;
    return v3(r * COSF(phi), r * SINF(phi), z);
}
static inline float power_heuristic(int nf, float fPdf, int ng, float gPdf) {
    float f = nf * fPdf, g = ng * gPdf;
    return (f * f) / (f * f + g * g);
}

/* ------------------------------------------------------------------ scene access */
typedef struct {
    const pbrtgpu_flat_scene *s;
    int nb;
} Ctx;
static inline const float *SPEC(const Ctx *c, int off) { return c->s->spectra + off; }
static inline float spec_y(const Ctx *c, const float *v) {
    float yy = 0.f;
    for (int i = 0; i < c->nb; ++i) yy += c->s->band_Y[i] * v[i];
    return yy / c->s->y_int;
}
static inline int spec_black(const Ctx *c, const float *v) {
    for (int i = 0; i < c->nb; ++i) if (v[i] != 0.) return 0;
    return 1;
}

/* ------------------------------------------------------------------ shapes */
typedef struct {   /* DifferentialGeometry (diffgeom.h) subset */
    V p, nn, dpdu, dpdv, dndu, dndv;
    float u, v;
} DG;
static void dg_init(DG *dg, V p, V dpdu, V dpdv, V dndu, V dndv, float u, float v, int flip) {
    dg->p = p; dg->dpdu = dpdu; dg->dpdv = dpdv; dg->dndu = dndu; dg->dndv = dndv;
    dg->nn = vnorm(vcross(dpdu, dpdv));
    dg->u = u; dg->v = v;
    if (flip) dg->nn = vmul(dg->nn, -1.f);
}
static void tri_uvs(const Ctx *c, const pbrtgpu_triangle *t, float uv[3][2]) {
    const pbrtgpu_mesh *m = &c->s->meshes[t->mesh];
    if (m->has_uvs) {
        for (int k = 0; k < 3; ++k) { uv[k][0] = c->s->vert_uv[2 * t->v[k]]; uv[k][1] = c->s->vert_uv[2 * t->v[k] + 1]; }
    } else {
        uv[0][0] = 0.; uv[0][1] = 0.; uv[1][0] = 1.; uv[1][1] = 0.; uv[2][0] = 1.; uv[2][1] = 1.;
    }
}
static inline V vert(const Ctx *c, int i) { const float *p = c->s->vert_p + 3 * i; return v3(p[0], p[1], p[2]); }
static inline V vnormal(const Ctx *c, int i) { const float *p = c->s->vert_n + 3 * i; return v3(p[0], p[1], p[2]); }

/* Triangle::Intersect / IntersectP (trianglemesh.cpp:119-273) */
static int tri_intersect(const Ctx *c, int ti, const Ray *ray, float *tHit, float *rayEps, DG *dg) {
    const pbrtgpu_triangle *t = &c->s->tris[ti];
    V p1 = vert(c, t->v[0]), p2 = vert(c, t->v[1]), p3 = vert(c, t->v[2]);
    V e1 = vsub(p2, p1), e2 = vsub(p3, p1);
    V s1 = vcross(ray->d, e2);
    float divisor = vdot(s1, e1);
    if (divisor == 0.) return 0;
    float invDivisor = 1.f / divisor;
    V d = vsub(ray->o, p1);
    float b1 = vdot(d, s1) * invDivisor;
    if (b1 < 0. || b1 > 1.) return 0;
    V s2 = vcross(d, e1);
    float b2 = vdot(ray->d, s2) * invDivisor;
    if (b2 < 0. || b1 + b2 > 1.) return 0;
    float tt = vdot(e2, s2) * invDivisor;
    if (tt < ray->mint || tt > ray->maxt) return 0;
    if (!dg) { *tHit = tt; return 1; }
    float uvs[3][2];
    tri_uvs(c, t, uvs);
    float du1 = uvs[0][0] - uvs[2][0], du2 = uvs[1][0] - uvs[2][0];
    float dv1 = uvs[0][1] - uvs[2][1], dv2 = uvs[1][1] - uvs[2][1];
    V dp1 = vsub(p1, p3), dp2 = vsub(p2, p3);
    float determinant = du1 * dv2 - dv1 * du2;
    V dpdu, dpdv;
    if (determinant == 0.f) coordsys(vnorm(vcross(e2, e1)), &dpdu, &dpdv);
    else {
        float invdet = 1.f / determinant;
        dpdu = vmul(vsub(vmul(dp1, dv2), vmul(dp2, dv1)), invdet);
        dpdv = vmul(vadd(vmul(dp1, -du2), vmul(dp2, du1)), invdet);
    }
    float b0 = 1 - b1 - b2;
    float tu = b0 * uvs[0][0] + b1 * uvs[1][0] + b2 * uvs[2][0];
    float tv = b0 * uvs[0][1] + b1 * uvs[1][1] + b2 * uvs[2][1];
    const pbrtgpu_mesh *m = &c->s->meshes[t->mesh];
    dg_init(dg, rayat(ray, tt), dpdu, dpdv, v3(0, 0, 0), v3(0, 0, 0), tu, tv, m->reverse_orientation ^ m->swaps_handedness);
    *tHit = tt;
    *rayEps = 1e-3f * *tHit;
    return 1;
}
/* transform.cpp:30-40 */
static int solve2x2(const float A[2][2], const float B[2], float *x0, float *x1) {
    float det = A[0][0] * A[1][1] - A[0][1] * A[1][0];
    if (fabsf(det) < 1e-10f) return 0;
    *x0 = (A[1][1] * B[0] - A[0][1] * B[1]) / det;
    *x1 = (A[0][0] * B[1] - A[1][0] * B[0]) / det;
    if (isnan(*x0) || isnan(*x1)) return 0;
    return 1;
}
/* Triangle::GetShadingGeometry (trianglemesh.cpp:285-360) */
/* obj2wMinv: mInv of the ObjectToWorld passed to GetShadingGeometry (the mesh's, or the
 * instance-composed one set by TransformedPrimitive::Intersect) */
static void tri_shading(const Ctx *c, int ti, const float *obj2wMinv, const DG *dg, DG *dgs) {
    const pbrtgpu_triangle *t = &c->s->tris[ti];
    const pbrtgpu_mesh *m = &c->s->meshes[t->mesh];
    if (!m->has_normals) { *dgs = *dg; return; }
    float b[3];
    float uv[3][2];
    tri_uvs(c, t, uv);
    float A[2][2] = {{uv[1][0] - uv[0][0], uv[2][0] - uv[0][0]}, {uv[1][1] - uv[0][1], uv[2][1] - uv[0][1]}};
    float C[2] = {dg->u - uv[0][0], dg->v - uv[0][1]};
    if (!solve2x2(A, C, &b[1], &b[2])) b[0] = b[1] = b[2] = 1.f / 3.f;
    else b[0] = 1.f - b[1] - b[2];
    V n0 = vnormal(c, t->v[0]), n1 = vnormal(c, t->v[1]), n2 = vnormal(c, t->v[2]);
    /* b[0] * n[v0] + b[1] * n[v1] + b[2] * n[v2]  (Normal operator*(float, Normal) = (f*x,...)) */
    V ni = vadd(vadd(vmul(n0, b[0]), vmul(n1, b[1])), vmul(n2, b[2]));
    V ns = vnorm(xnormal(obj2wMinv, ni));
    V ss = vnorm(dg->dpdu);
    V ts = vcross(ss, ns);
    if (vlen2(ts) > 0.f) { ts = vnorm(ts); ss = vcross(ts, ns); }
    else coordsys(ns, &ss, &ts);
    V dndu, dndv;
    {
        float du1 = uv[0][0] - uv[2][0], du2 = uv[1][0] - uv[2][0];
        float dv1 = uv[0][1] - uv[2][1], dv2 = uv[1][1] - uv[2][1];
        V dn1 = vsub(n0, n2), dn2 = vsub(n1, n2);
        float determinant = du1 * dv2 - dv1 * du2;
        if (determinant == 0.f) dndu = dndv = v3(0, 0, 0);
        else {
            float invdet = 1.f / determinant;
            /* Normal ops: (dv2 * dn1 - dv1 * dn2) * invdet */
            dndu = vmul(vsub(vmul(dn1, dv2), vmul(dn2, dv1)), invdet);
            dndv = vmul(vadd(vmul(dn1, -du2), vmul(dn2, du1)), invdet);
        }
    }
    dg_init(dgs, dg->p, ss, ts, xnormal(obj2wMinv, dndu), xnormal(obj2wMinv, dndv), dg->u, dg->v,
            m->reverse_orientation ^ m->swaps_handedness);
}

/* pbrt.h:297-311 */
static int quadratic(float A, float B, float C, float *t0, float *t1) {
    float discrim = B * B - 4.f * A * C;
    if (discrim <= 0.) return 0;
    float rootDiscrim = sqrtf(discrim);
    float q;
    if (B < 0) q = -.5f * (B - rootDiscrim);
    else q = -.5f * (B + rootDiscrim);
    *t0 = q / A;
    *t1 = C / q;
    if (*t0 > *t1) { float tmp = *t0; *t0 = *t1; *t1 = tmp; }
    return 1;
}
/* WorldToObject(r) with WorldToObject = (o2w.mInv, o2w.m): Ray transform (transform.h:253-262) */
static Ray to_object(const pbrtgpu_quadric *q, const Ray *r) {
    Ray o = *r;
    /* 2-arg point form: *ptrans /= w if w != 1 */
    const float *m = q->o2w_minv;
    V p = r->o;
    float x = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float y = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float z = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    o.o = v3(x, y, z);
    if (w != 1.) o.o = vdiv(o.o, w);
    o.d = xvec(m, r->d);
    return o;
}
/* Sphere::Intersect (sphere.cpp:50-150); dg may be NULL (IntersectP) */
static int sphere_intersect(const pbrtgpu_quadric *q, const Ray *r, float *tHit, float *rayEps, DG *dg) {
    float phi;
    V phit;
    Ray ray = to_object(q, r);
    float A = ray.d.x * ray.d.x + ray.d.y * ray.d.y + ray.d.z * ray.d.z;
    float B = 2 * (ray.d.x * ray.o.x + ray.d.y * ray.o.y + ray.d.z * ray.o.z);
    float C = ray.o.x * ray.o.x + ray.o.y * ray.o.y + ray.o.z * ray.o.z - q->radius * q->radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return 0;
    if (t0 > ray.maxt || t1 < ray.mint) return 0;
    float thit = t0;
    if (t0 < ray.mint) { thit = t1; if (thit > ray.maxt) return 0; }
    phit = rayat(&ray, thit);
    if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * q->radius;
    phi = ATAN2F(phit.y, phit.x);
    if (phi < 0.) phi += 2.f * PI_F;
    if ((q->zmin > -q->radius && phit.z < q->zmin) || (q->zmax < q->radius && phit.z > q->zmax) || phi > q->phi_max) {
        if (thit == t1) return 0;
        if (t1 > ray.maxt) return 0;
        thit = t1;
        phit = rayat(&ray, thit);
        if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * q->radius;
        phi = ATAN2F(phit.y, phit.x);
        if (phi < 0.) phi += 2.f * PI_F;
        if ((q->zmin > -q->radius && phit.z < q->zmin) || (q->zmax < q->radius && phit.z > q->zmax) || phi > q->phi_max)
            return 0;
    }
    if (!dg) { if (tHit) *tHit = thit; return 1; }
    float u = phi / q->phi_max;
    float theta = ACOSF(clampf(phit.z / q->radius, -1.f, 1.f));
    float v = (theta - q->theta_min) / (q->theta_max - q->theta_min);
    float zradius = sqrtf(phit.x * phit.x + phit.y * phit.y);
    float invzradius = 1.f / zradius;
    float cosphi = phit.x * invzradius, sinphi = phit.y * invzradius;
    V dpdu = v3(-q->phi_max * phit.y, q->phi_max * phit.x, 0);
    V dpdv = vmul(v3(phit.z * cosphi, phit.z * sinphi, -q->radius * SINF(theta)), q->theta_max - q->theta_min);
    V d2Pduu = vmul(v3(phit.x, phit.y, 0), -q->phi_max * q->phi_max);
    V d2Pduv = vmul(v3(-sinphi, cosphi, 0.), (q->theta_max - q->theta_min) * phit.z * q->phi_max);
    V d2Pdvv = vmul(v3(phit.x, phit.y, phit.z), -(q->theta_max - q->theta_min) * (q->theta_max - q->theta_min));
    float E = vdot(dpdu, dpdu), F = vdot(dpdu, dpdv), G = vdot(dpdv, dpdv);
    V N = vnorm(vcross(dpdu, dpdv));
    float e = vdot(N, d2Pduu), f = vdot(N, d2Pduv), g = vdot(N, d2Pdvv);
    float invEGF2 = 1.f / (E * G - F * F);
    V dndu = vadd(vmul(dpdu, (f * F - e * G) * invEGF2), vmul(dpdv, (e * F - f * E) * invEGF2));
    V dndv = vadd(vmul(dpdu, (g * F - f * G) * invEGF2), vmul(dpdv, (f * F - g * E) * invEGF2));
    dg_init(dg, xpoint(q->o2w_m, phit), xvec(q->o2w_m, dpdu), xvec(q->o2w_m, dpdv), xnormal(q->o2w_minv, dndu),
            xnormal(q->o2w_minv, dndv), u, v, q->reverse_orientation ^ q->swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return 1;
}
/* Disk::Intersect (disk.cpp:48-96) */
static int disk_intersect(const pbrtgpu_quadric *q, const Ray *r, float *tHit, float *rayEps, DG *dg) {
    Ray ray = to_object(q, r);
    if (fabsf(ray.d.z) < 1e-7) return 0;
    float thit = (q->height - ray.o.z) / ray.d.z;
    if (thit < ray.mint || thit > ray.maxt) return 0;
    V phit = rayat(&ray, thit);
    float dist2 = phit.x * phit.x + phit.y * phit.y;
    if (dist2 > q->radius * q->radius || dist2 < q->inner_radius * q->inner_radius) return 0;
    float phi = ATAN2F(phit.y, phit.x);
    if (phi < 0) phi = (float)((double)phi + 2. * (double)PI_F);
    if (phi > q->phi_max) return 0;
    if (!dg) { if (tHit) *tHit = thit; return 1; }
    float u = phi / q->phi_max;
    float oneMinusV = ((sqrtf(dist2) - q->inner_radius) / (q->radius - q->inner_radius));
    float invOneMinusV = (oneMinusV > 0.f) ? (1.f / oneMinusV) : 0.f;
    float v = 1.f - oneMinusV;
    V dpdu = v3(-q->phi_max * phit.y, q->phi_max * phit.x, 0.);
    V dpdv = v3(-phit.x * invOneMinusV, -phit.y * invOneMinusV, 0.);
    dpdu = v3(dpdu.x * (q->phi_max * INV_TWOPI_F), dpdu.y * (q->phi_max * INV_TWOPI_F), dpdu.z * (q->phi_max * INV_TWOPI_F));
    float sc = (q->radius - q->inner_radius) / q->radius;
    dpdv = v3(dpdv.x * sc, dpdv.y * sc, dpdv.z * sc);
    V zero = v3(0, 0, 0);
    dg_init(dg, xpoint(q->o2w_m, phit), xvec(q->o2w_m, dpdu), xvec(q->o2w_m, dpdv), xnormal(q->o2w_minv, zero),
            xnormal(q->o2w_minv, zero), u, v, q->reverse_orientation ^ q->swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return 1;
}
/* Cylinder::Intersect (cylinder.cpp:48-111); dg may be NULL (IntersectP, :113-176) */
static int cylinder_intersect(const pbrtgpu_quadric *q, const Ray *r, float *tHit, float *rayEps, DG *dg) {
    Ray ray = to_object(q, r);
    float A = ray.d.x * ray.d.x + ray.d.y * ray.d.y;
    float B = 2 * (ray.d.x * ray.o.x + ray.d.y * ray.o.y);
    float C = ray.o.x * ray.o.x + ray.o.y * ray.o.y - q->radius * q->radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return 0;
    if (t0 > ray.maxt || t1 < ray.mint) return 0;
    float thit = t0;
    if (t0 < ray.mint) { thit = t1; if (thit > ray.maxt) return 0; }
    V phit = rayat(&ray, thit);
    float phi = ATAN2F(phit.y, phit.x);
    if (phi < 0.) phi += 2.f * PI_F;
    if (phit.z < q->zmin || phit.z > q->zmax || phi > q->phi_max) {
        if (thit == t1) return 0;
        thit = t1;
        if (t1 > ray.maxt) return 0;
        phit = rayat(&ray, thit);
        phi = ATAN2F(phit.y, phit.x);
        if (phi < 0.) phi += 2.f * PI_F;
        if (phit.z < q->zmin || phit.z > q->zmax || phi > q->phi_max) return 0;
    }
    if (!dg) { if (tHit) *tHit = thit; return 1; }
    float u = phi / q->phi_max, v = (phit.z - q->zmin) / (q->zmax - q->zmin);
    V dpdu = v3(-q->phi_max * phit.y, q->phi_max * phit.x, 0), dpdv = v3(0, 0, q->zmax - q->zmin);
    V d2Pduu = vmul(v3(phit.x, phit.y, 0), -q->phi_max * q->phi_max), d2Pduv = v3(0, 0, 0), d2Pdvv = v3(0, 0, 0);
    float E = vdot(dpdu, dpdu), F = vdot(dpdu, dpdv), G = vdot(dpdv, dpdv);
    V N = vnorm(vcross(dpdu, dpdv));
    float e = vdot(N, d2Pduu), f = vdot(N, d2Pduv), g = vdot(N, d2Pdvv);
    float invEGF2 = 1.f / (E * G - F * F);
    V dndu = vadd(vmul(dpdu, (f * F - e * G) * invEGF2), vmul(dpdv, (e * F - f * E) * invEGF2));
    V dndv = vadd(vmul(dpdu, (g * F - f * G) * invEGF2), vmul(dpdv, (f * F - g * E) * invEGF2));
    dg_init(dg, xpoint(q->o2w_m, phit), xvec(q->o2w_m, dpdu), xvec(q->o2w_m, dpdv), xnormal(q->o2w_minv, dndu),
            xnormal(q->o2w_minv, dndv), u, v, q->reverse_orientation ^ q->swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return 1;
}
static float shape_area(const Ctx *c, int type, int idx) {
    if (type == PBRTGPU_SHAPE_TRIANGLE) {
        const pbrtgpu_triangle *t = &c->s->tris[idx];
        V p1 = vert(c, t->v[0]), p2 = vert(c, t->v[1]), p3 = vert(c, t->v[2]);
        return 0.5f * vlen(vcross(vsub(p2, p1), vsub(p3, p1)));
    }
    const pbrtgpu_quadric *q = &c->s->quadrics[idx];
    if (type == PBRTGPU_SHAPE_SPHERE) return q->phi_max * q->radius * (q->zmax - q->zmin);
    if (type == PBRTGPU_SHAPE_CYLINDER) return (q->zmax - q->zmin) * q->phi_max * q->radius;   /* cylinder.cpp:180-182 */
    return q->phi_max * 0.5f * (q->radius * q->radius - q->inner_radius * q->inner_radius);
}
static int shape_intersect(const Ctx *c, int type, int idx, const Ray *r, float *tHit, float *eps, DG *dg) {
    if (type == PBRTGPU_SHAPE_TRIANGLE) return tri_intersect(c, idx, r, tHit, eps, dg);
    if (type == PBRTGPU_SHAPE_SPHERE) return sphere_intersect(&c->s->quadrics[idx], r, tHit, eps, dg);
    if (type == PBRTGPU_SHAPE_CYLINDER) return cylinder_intersect(&c->s->quadrics[idx], r, tHit, eps, dg);
    return disk_intersect(&c->s->quadrics[idx], r, tHit, eps, dg);
}

/* ------------------------------------------------------------------ BVH */
static inline int bbox_hit(const pbrtgpu_bvh_node *n, const Ray *ray, V invDir, const int dirIsNeg[3]) {
    const float *b0 = n->bmin, *b1 = n->bmax;
    float tmin = ((dirIsNeg[0] ? b1 : b0)[0] - ray->o.x) * invDir.x;
    float tmax = ((dirIsNeg[0] ? b0 : b1)[0] - ray->o.x) * invDir.x;
    float tymin = ((dirIsNeg[1] ? b1 : b0)[1] - ray->o.y) * invDir.y;
    float tymax = ((dirIsNeg[1] ? b0 : b1)[1] - ray->o.y) * invDir.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = ((dirIsNeg[2] ? b1 : b0)[2] - ray->o.z) * invDir.z;
    float tzmax = ((dirIsNeg[2] ? b0 : b1)[2] - ray->o.z) * invDir.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return (tmin < ray->maxt) && (tmax > ray->mint);
}
typedef struct { int prim; float t; } Hit;

/* ---- Matrix4x4 / Transform / Quaternion / AnimatedTransform (transform.cpp, quaternion.cpp) */
static void m4_mul(const float *a, const float *b, float *r) {   /* Matrix4x4::Mul */
    float t[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            t[4 * i + j] = a[4 * i + 0] * b[0 * 4 + j] + a[4 * i + 1] * b[1 * 4 + j] + a[4 * i + 2] * b[2 * 4 + j] +
                           a[4 * i + 3] * b[3 * 4 + j];
    memcpy(r, t, sizeof(t));
}
static void m4_identity(float *m) { memset(m, 0, 64); m[0] = m[5] = m[10] = m[15] = 1.f; }
static void m4_inverse(const float *m, float *out) {   /* transform.cpp:68-130, Gauss-Jordan, full pivoting */
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    float minv[4][4];
    memcpy(minv, m, 64);
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0.;
        for (int j = 0; j < 4; j++)
            if (ipiv[j] != 1)
                for (int k = 0; k < 4; k++)
                    if (ipiv[k] == 0 && fabsf(minv[j][k]) >= big) { big = (float)fabsf(minv[j][k]); irow = j; icol = k; }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) { float t = minv[irow][k]; minv[irow][k] = minv[icol][k]; minv[icol][k] = t; }
        indxr[i] = irow;
        indxc[i] = icol;
        float pivinv = 1.f / minv[icol][icol];
        minv[icol][icol] = 1.f;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++)
            if (j != icol) {
                float save = minv[j][icol];
                minv[j][icol] = 0;
                for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
            }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) { float t = minv[k][indxr[j]]; minv[k][indxr[j]] = minv[k][indxc[j]]; minv[k][indxc[j]] = t; }
    memcpy(out, minv, 64);
}
typedef struct { float x, y, z, w; } Quat;
static float qdot(Quat a, Quat b) { return (a.x * b.x + a.y * b.y + a.z * b.z) + a.w * b.w; }
static Quat qnormalize(Quat q) {   /* q / sqrtf(Dot(q, q)): Vector operator/ (reciprocal), w / d */
    float d = sqrtf(qdot(q, q));
    float inv = 1.f / d;
    Quat r = {q.x * inv, q.y * inv, q.z * inv, q.w / d};
    return r;
}
static Quat qscale(Quat q, float f) { Quat r = {q.x * f, q.y * f, q.z * f, q.w * f}; return r; }
static Quat qadd(Quat a, Quat b) { Quat r = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; return r; }
static Quat qsub(Quat a, Quat b) { Quat r = {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; return r; }
static Quat slerp(float t, Quat q1, Quat q2) {   /* quaternion.cpp:39-49 */
    float cosTheta = qdot(q1, q2);
    if (cosTheta > .9995f) return qnormalize(qadd(qscale(q1, 1.f - t), qscale(q2, t)));
    float theta = ACOSF(clampf(cosTheta, -1.f, 1.f));
    float thetap = theta * t;
    Quat qperp = qnormalize(qsub(q2, qscale(q1, cosTheta)));
    return qadd(qscale(q1, COSF(thetap)), qscale(qperp, SINF(thetap)));
}
/* Quaternion::ToTransform (quaternion.cpp:52-70): m = Transpose(M), mInv = M */
static void quat_to_m(Quat q, float *m, float *minv) {
    float xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    float xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z;
    float wx = q.x * q.w, wy = q.y * q.w, wz = q.z * q.w;
    float M[16];
    m4_identity(M);
    M[0] = 1.f - 2.f * (yy + zz); M[1] = 2.f * (xy + wz); M[2] = 2.f * (xz - wy);
    M[4] = 2.f * (xy - wz); M[5] = 1.f - 2.f * (xx + zz); M[6] = 2.f * (yz + wx);
    M[8] = 2.f * (xz + wy); M[9] = 2.f * (yz - wx); M[10] = 1.f - 2.f * (xx + yy);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) m[4 * i + j] = M[4 * j + i];
    if (minv) memcpy(minv, M, 64);
}
/* AnimatedTransform::Interpolate (transform.cpp:356-381): world->primitive (m, mInv) */
static void inst_interp(const pbrtgpu_instance *I, float time, float *m, float *minv) {
    if (!I->animated || time <= I->start_time) { memcpy(m, I->start_m, 64); if (minv) memcpy(minv, I->start_minv, 64); return; }
    if (time >= I->end_time) { memcpy(m, I->end_m, 64); if (minv) memcpy(minv, I->end_minv, 64); return; }
    float dt = (time - I->start_time) / (I->end_time - I->start_time);
    /* Vector trans = (1-dt) * T[0] + dt * T[1] */
    float tr[3];
    for (int k = 0; k < 3; ++k) tr[k] = (1.f - dt) * I->T[0][k] + dt * I->T[1][k];
    Quat r0 = {I->R[0][0], I->R[0][1], I->R[0][2], I->R[0][3]}, r1 = {I->R[1][0], I->R[1][1], I->R[1][2], I->R[1][3]};
    Quat rot = slerp(dt, r0, r1);
    float S[16];
    m4_identity(S);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) S[4 * i + j] = lerpf(dt, I->S[0][4 * i + j], I->S[1][4 * i + j]);
    /* Translate(trans) * rotate.ToTransform() * Transform(scale) */
    float T[16], Tinv[16], R[16], Rinv[16], TR[16];
    m4_identity(T); T[3] = tr[0]; T[7] = tr[1]; T[11] = tr[2];
    quat_to_m(rot, R, Rinv);
    m4_mul(T, R, TR);
    m4_mul(TR, S, m);
    if (minv) {
        float Sinv[16], RiTi[16];
        m4_identity(Tinv); Tinv[3] = -tr[0]; Tinv[7] = -tr[1]; Tinv[11] = -tr[2];
        m4_inverse(S, Sinv);
        m4_mul(Rinv, Tinv, RiTi);
        m4_mul(Sinv, RiTi, minv);
    }
}
static int m4_is_identity(const float *m) {
    for (int i = 0; i < 16; ++i)
        if (m[i] != ((i % 5 == 0) ? 1.f : 0.f)) return 0;
    return 1;
}
static Ray xray(const float *m, const Ray *r) {   /* Transform::operator()(Ray) */
    Ray o = *r;
    o.o = xpoint(m, r->o);
    o.d = xvec(m, r->d);
    return o;
}

/* BVHAccel::Intersect (bvh.cpp:380-432) from node `root`; prims of shape_type INSTANCE run
 * TransformedPrimitive::Intersect (primitive.cpp:87-116) on their nested BVH.  Updates
 * ray->maxt like GeometricPrimitive; anyhit = IntersectP (bvh.cpp:435-481). */
static int bvh_walk(const Ctx *c, uint32_t root, Ray *ray, Hit *hit, int anyhit);
static int prim_test(const Ctx *c, int pi, Ray *ray, Hit *hit, int anyhit) {
    const pbrtgpu_prim *pr = &c->s->prims[pi];
    if (pr->shape_type == PBRTGPU_SHAPE_INSTANCE) {
        const pbrtgpu_instance *I = &c->s->instances[pr->shape_index];
        float m[16];
        inst_interp(I, ray->time, m, NULL);
        Ray r = xray(m, ray);
        int found;
        if (I->single_prim >= 0) found = prim_test(c, I->single_prim, &r, hit, anyhit);
        else found = bvh_walk(c, (uint32_t)I->root, &r, hit, anyhit);
        if (found && !anyhit) ray->maxt = r.maxt;
        return found;
    }
    float t, eps;
    if (!shape_intersect(c, pr->shape_type, pr->shape_index, ray, &t, &eps, NULL)) return 0;
    if (!anyhit) { ray->maxt = t; hit->prim = pi; hit->t = t; }
    return 1;
}
static int bvh_walk(const Ctx *c, uint32_t root, Ray *ray, Hit *hit, int anyhit) {
    const pbrtgpu_bvh_node *nodes = c->s->nodes;
    V invDir = v3(1.f / ray->d.x, 1.f / ray->d.y, 1.f / ray->d.z);
    int dirIsNeg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    uint32_t todo[64];
    int todoOffset = 0;
    uint32_t nodeNum = root;
    int found = 0;
    for (;;) {
        const pbrtgpu_bvh_node *node = &nodes[nodeNum];
        if (bbox_hit(node, ray, invDir, dirIsNeg)) {
            uint32_t np = node->meta & 0xff;
            if (np > 0) {
                for (uint32_t i = 0; i < np; ++i)
                    if (prim_test(c, (int)(node->offset + i), ray, hit, anyhit)) {
                        if (anyhit) return 1;
                        found = 1;
                    }
                if (todoOffset == 0) break;
                nodeNum = todo[--todoOffset];
            } else {
                uint32_t axis = (node->meta >> 8) & 0xff;
                if (dirIsNeg[axis]) { todo[todoOffset++] = nodeNum + 1; nodeNum = node->offset; }
                else { todo[todoOffset++] = node->offset; nodeNum = nodeNum + 1; }
            }
        } else {
            if (todoOffset == 0) break;
            nodeNum = todo[--todoOffset];
        }
    }
    return found;
}
static int bvh_intersect(const Ctx *c, Ray *ray, Hit *hit) { return bvh_walk(c, 0, ray, hit, 0); }
static int bvh_intersectP(const Ctx *c, const Ray *ray) {
    Ray r = *ray;
    Hit h;
    return bvh_walk(c, 0, &r, &h, 1);
}
/* full intersection record for a recorded closest hit; for primitives of a transformed
 * instance the object-space record is moved to world space as TransformedPrimitive does */
typedef struct { DG dg; float rayEps; int prim; int inst; float nmat[16]; } Isect;
static void isect_fill(const Ctx *c, const Ray *ray, const Hit *h, Isect *is) {
    const pbrtgpu_prim *pr = &c->s->prims[h->prim];
    int inst = c->s->prim_instance ? c->s->prim_instance[h->prim] : -1;
    Ray r = *ray;
    r.maxt = h->t;
    float t;
    is->prim = h->prim;
    is->inst = -1;
    if (inst < 0) {
        shape_intersect(c, pr->shape_type, pr->shape_index, &r, &t, &is->rayEps, &is->dg);
        return;
    }
    const pbrtgpu_instance *I = &c->s->instances[inst];
    float m[16], minv[16];
    inst_interp(I, ray->time, m, minv);
    Ray ro = xray(m, &r);
    shape_intersect(c, pr->shape_type, pr->shape_index, &ro, &t, &is->rayEps, &is->dg);
    if (m4_is_identity(m)) return;
    /* WorldToObject = Identity * w2p ; ObjectToWorld = Inverse(that): normals use Mul(I, w2p.m) */
    float id[16];
    m4_identity(id);
    m4_mul(id, m, is->nmat);
    is->inst = inst;
    /* PrimitiveToWorld = Inverse(w2p): points/vectors with w2p.mInv, normals with w2p.m */
    DG *g = &is->dg;
    g->p = xpoint(minv, g->p);
    g->nn = vnorm(xnormal(m, g->nn));
    g->dpdu = xvec(minv, g->dpdu);
    g->dpdv = xvec(minv, g->dpdv);
    g->dndu = xnormal(m, g->dndu);
    g->dndv = xnormal(m, g->dndv);
}

/* ------------------------------------------------------------------ BSDF */
enum { BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16,
       BSDF_ALL = 31 };
enum { BX_LAMBERT, BX_OREN, BX_MICRO_BLINN_DIEL, BX_SPEC_REFL_NOOP, BX_FRESNEL_BLEND_ANISO, BX_MEASURED_IRREG,
       BX_MICRO_BLINN_COND, BX_SPEC_REFL_DIEL, BX_SPEC_TRANS,    /* eta_t = index of refraction for these two */
       BX_MEASURED_HALF,                                          /* RegularHalfangleBRDF: merl = its table */
       BX_ANISOWARD,                                              /* AnisoWardBrdf: R = Rs, a = Ax, b = Ay */
       BX_SPEC_REFL_COND };                                       /* SpecularReflection(1, FresnelConductor(eta, 0)) */
typedef struct {
    int kind, type;
    const float *R;      /* reflectance spectrum */
    const float *R2;     /* second spectrum (FresnelBlend Rs) */
    float a, b;          /* OrenNayar A,B ; Blinn exponent ; Aniso ex,ey */
    float eta_i, eta_t;  /* FresnelDielectric */
    const float *eta, *k;   /* FresnelConductor */
    const pbrtgpu_kdnode *kd;   /* IrregIsotropicBRDF: kd-tree nodes */
    int nkd;
    const float *merl;          /* RegularHalfangleBRDF: RGB table (90 x 90 x 180 texels) */
} BxDF;
typedef struct {
    V nn, ng, sn, tn;
    int n;
    BxDF bx[4];
    float texbuf[2][MAXB];   /* the material's textured spectra evaluated at this hit (slots 0, 1) */
    float eta;               /* BSDF::eta: the glass material's index, 1 otherwise (glass.cpp:47-48) */
} BSDF;
static inline int matches(const BxDF *b, int flags) { return (b->type & flags) == b->type; }
static inline V to_local(const BSDF *b, V v) { return v3(vdot(v, b->sn), vdot(v, b->tn), vdot(v, b->nn)); }
static inline V to_world(const BSDF *b, V v) {
    return v3(b->sn.x * v.x + b->tn.x * v.y + b->nn.x * v.z, b->sn.y * v.x + b->tn.y * v.y + b->nn.y * v.z,
              b->sn.z * v.x + b->tn.z * v.y + b->nn.z * v.z);
}
static inline float costh(V w) { return w.z; }
static inline float abscos(V w) { return fabsf(w.z); }
static inline float sin2(V w) { return fmaxf_(0.f, 1.f - costh(w) * costh(w)); }
static inline float sinth(V w) { return sqrtf(sin2(w)); }
static inline float cosphi(V w) { float s = sinth(w); if (s == 0.f) return 1.f; return clampf(w.x / s, -1.f, 1.f); }
static inline float sinphi(V w) { float s = sinth(w); if (s == 0.f) return 0.f; return clampf(w.y / s, -1.f, 1.f); }
static inline int samehemi(V w, V wp) { return w.z * wp.z > 0.f; }

/* FresnelDielectric::Evaluate + FrDiel (reflection.cpp:52-58,112-127); all bands equal */
static float fr_dielectric(float cosi, float eta_i, float eta_t) {
    cosi = clampf(cosi, -1.f, 1.f);
    int entering = cosi > 0.;
    float ei = eta_i, et = eta_t;
    if (!entering) { float t = ei; ei = et; et = t; }
    float sint = ei / et * sqrtf(fmaxf_(0.f, 1.f - cosi * cosi));
    if (sint >= 1.) return 1.f;
    float cost = sqrtf(fmaxf_(0.f, 1.f - sint * sint));
    float ci = fabsf(cosi);
    float Rparl = ((et * ci) - (ei * cost)) / ((et * ci) + (ei * cost));
    float Rperp = ((ei * ci) - (et * cost)) / ((ei * ci) + (et * cost));
    return (Rparl * Rparl + Rperp * Rperp) / 2.f;
}
/* FrCond (reflection.cpp:62-71) for one band */
static inline float fr_cond(float cosi, float eta, float k) {
    float tmp = ((eta * eta + k * k) * cosi) * cosi;
    float Rparl2 = ((tmp - ((2.f * eta) * cosi)) + 1.f) / ((tmp + ((2.f * eta) * cosi)) + 1.f);
    float tmp_f = eta * eta + k * k;
    float Rperp2 = ((tmp_f - ((2.f * eta) * cosi)) + cosi * cosi) / ((tmp_f + ((2.f * eta) * cosi)) + cosi * cosi);
    return (Rparl2 + Rperp2) / 2.f;
}
static inline float blinn_D(float e, V wh) { return (e + 2) * INV_TWOPI_F * POWF(abscos(wh), e); }
static inline float micro_G(V wo, V wi, V wh) {
    float NdotWh = abscos(wh), NdotWo = abscos(wo), NdotWi = abscos(wi), WOdotWh = fabsf(vdot(wo, wh));
    return fminf_(1.f, fminf_((2.f * NdotWh * NdotWo / WOdotWh), (2.f * NdotWh * NdotWi / WOdotWh)));
}
static float blinn_pdf(float e, V wo, V wi) {
    V wh = vnorm(vadd(wo, wi));
    float costheta = abscos(wh);
    float p = ((e + 1.f) * POWF(costheta, e)) / (2.f * PI_F * 4.f * vdot(wo, wh));
    if (vdot(wo, wh) <= 0.f) p = 0.f;
    return p;
}
static void blinn_sample(float e, V wo, V *wi, float u1, float u2, float *pdf) {
    float costheta = POWF(u1, 1.f / (e + 1));
    float sintheta = sqrtf(fmaxf_(0.f, 1.f - costheta * costheta));
    float phi = u2 * 2.f * PI_F;
    V wh = v3(sintheta * COSF(phi), sintheta * SINF(phi), costheta);
    if (!samehemi(wo, wh)) wh = vneg(wh);
    *wi = vadd(vneg(wo), vmul(wh, 2.f * vdot(wo, wh)));
    float p = ((e + 1.f) * POWF(costheta, e)) / (2.f * PI_F * 4.f * vdot(wo, wh));
    if (vdot(wo, wh) <= 0.f) p = 0.f;
    *pdf = p;
}
/* Anisotropic (reflection.cpp:369-435) */
static inline float aniso_D(float ex, float ey, V wh) {
    float costhetah = abscos(wh);
    float d = 1.f - costhetah * costhetah;
    if (d == 0.f) return 0.f;
    float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / d;
    return sqrtf((ex + 2.f) * (ey + 2.f)) * INV_TWOPI_F * POWF(costhetah, e);
}
static float aniso_pdf(float ex, float ey, V wo, V wi) {
    V wh = vnorm(vadd(wo, wi));
    float costhetah = abscos(wh);
    float ds = 1.f - costhetah * costhetah;
    float p = 0.f;
    if (ds > 0.f && vdot(wo, wh) > 0.f) {
        float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / ds;
        float d = sqrtf((ex + 1.f) * (ey + 1.f)) * INV_TWOPI_F * POWF(costhetah, e);
        p = d / (4.f * vdot(wo, wh));
    }
    return p;
}
static void aniso_first_quadrant(float ex, float ey, float u1, float u2, float *phi, float *costheta) {
    if (ex == ey) *phi = PI_F * u1 * 0.5f;
    else *phi = ATANF(sqrtf((ex + 1.f) / (ey + 1.f)) * TANF(PI_F * u1 * 0.5f));
    float cp = COSF(*phi), sp = SINF(*phi);
    *costheta = POWF(u2, 1.f / (ex * cp * cp + ey * sp * sp + 1));
}
static void aniso_sample(float ex, float ey, V wo, V *wi, float u1, float u2, float *pdf) {
    float phi, costheta;
    if (u1 < .25f) aniso_first_quadrant(ex, ey, 4.f * u1, u2, &phi, &costheta);
    else if (u1 < .5f) { u1 = 4.f * (.5f - u1); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi = PI_F - phi; }
    else if (u1 < .75f) { u1 = 4.f * (u1 - .5f); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi += PI_F; }
    else { u1 = 4.f * (1.f - u1); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi = 2.f * PI_F - phi; }
    float sintheta = sqrtf(fmaxf_(0.f, 1.f - costheta * costheta));
    V wh = v3(sintheta * COSF(phi), sintheta * SINF(phi), costheta);
    if (!samehemi(wo, wh)) wh = vneg(wh);
    *wi = vadd(vneg(wo), vmul(wh, 2.f * vdot(wo, wh)));
    float costhetah = abscos(wh);
    float ds = 1.f - costhetah * costhetah;
    float p = 0.f;
    if (ds > 0.f && vdot(wo, wh) > 0.f) {
        float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / ds;
        float d = sqrtf((ex + 1.f) * (ey + 1.f)) * INV_TWOPI_F * POWF(costhetah, e);
        p = d / (4.f * vdot(wo, wh));
    }
    *pdf = p;
}

/* BxDF::f for one bxdf, accumulated band-wise into out (out += f) */
/* BRDFRemap (reflection.cpp:239-248); pbrt.h defines M_PI as a float literal, so every
 * operation here is single precision */
static V brdf_remap(V wo, V wi) {
    float cosi = wi.z, coso = wo.z;
    float sini = sinth(wi), sino = sinth(wo);
    float pi_ = ATAN2F(wi.y, wi.x), po_ = ATAN2F(wo.y, wo.x);
    float phii = (pi_ < 0.f) ? pi_ + 2.f * PI_F : pi_;   /* SphericalPhi (geometry.h:647-650) */
    float phio = (po_ < 0.f) ? po_ + 2.f * PI_F : po_;
    float dphi = phii - phio;
    if (dphi < 0.) dphi += 2.f * PI_F;
    if (dphi > 2.f * PI_F) dphi -= 2.f * PI_F;
    if (dphi > PI_F) dphi = 2.f * PI_F - dphi;
    return v3(sini * sino, dphi / PI_F, cosi * coso);
}
typedef struct { float *v; float sumWeights; int nFound; } IrregProc;
/* KdTree::privateLookup (kdtree.h:160-185) with IrregIsoProc (reflection.cpp:34-47) */
static void kd_lookup(const Ctx *c, const pbrtgpu_kdnode *nodes, int nNodes, uint32_t nodeNum, V p, IrregProc *pr,
                      float maxD2) {
    const pbrtgpu_kdnode *node = &nodes[nodeNum];
    int axis = node->split_axis;
    if (axis != 3) {
        float pa = vcomp(p, axis);
        float dist2 = (pa - node->split_pos) * (pa - node->split_pos);
        if (pa <= node->split_pos) {
            if (node->has_left) kd_lookup(c, nodes, nNodes, nodeNum + 1, p, pr, maxD2);
            if (dist2 < maxD2 && node->right_child < nNodes) kd_lookup(c, nodes, nNodes, (uint32_t)node->right_child, p, pr, maxD2);
        } else {
            if (node->right_child < nNodes) kd_lookup(c, nodes, nNodes, (uint32_t)node->right_child, p, pr, maxD2);
            if (dist2 < maxD2 && node->has_left) kd_lookup(c, nodes, nNodes, nodeNum + 1, p, pr, maxD2);
        }
    }
    V d = vsub(v3(node->p[0], node->p[1], node->p[2]), p);   /* DistanceSquared = LengthSquared(p1 - p2) */
    float dist2 = vlen2(d);
    if (dist2 < maxD2) {
        float weight = EXPF(-100.f * dist2);
        const float *sv = SPEC(c, node->spec);
        for (int i = 0; i < c->nb; ++i) pr->v[i] += weight * sv[i];
        pr->sumWeights += weight;
        ++pr->nFound;
    }
}
/* IrregIsotropicBRDF::f (reflection.cpp:251-264) */
static void irreg_f(const Ctx *c, const BxDF *b, V wo, V wi, float *f) {
    V m = brdf_remap(wo, wi);
    float lastMaxDist2 = .001f;
    float v[PBRTGPU_MAX_BANDS];
    for (;;) {
        IrregProc pr;
        for (int i = 0; i < c->nb; ++i) v[i] = 0.f;
        pr.v = v; pr.sumWeights = 0.f; pr.nFound = 0;
        float maxDist2 = lastMaxDist2;
        if (b->nkd > 0) kd_lookup(c, b->kd, b->nkd, 0, m, &pr, maxDist2);
        if (pr.nFound > 2 || lastMaxDist2 > 1.5f) {
            for (int i = 0; i < c->nb; ++i) f[i] = clampf(v[i], 0.f, INFINITY) / pr.sumWeights;
            return;
        }
        lastMaxDist2 *= 2.f;
    }
}
static void from_rgb(const Ctx *c, const float rgb[3], int illum, float *r);
static inline int clampi_(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
/* RegularHalfangleBRDF::f (reflection.cpp:267-300); M_PI is a float literal (pbrt.h:179),
 * REMAP = Clamp(int(V / MAX * COUNT), 0, COUNT - 1) */
static void halfangle_f(const Ctx *c, const BxDF *b, V WO, V WI, float *f) {
    V wo = WO, wi = WI, wh = vadd(wo, wi);
    for (int i = 0; i < c->nb; ++i) f[i] = 0.f;
    if (wh.z < 0.f) { wo = vneg(wo); wi = vneg(wi); wh = vneg(wh); }
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return;
    wh = vnorm(wh);
    float whTheta = ACOSF(clampf(wh.z, -1.f, 1.f));
    float whCosPhi = cosphi(wh), whSinPhi = sinphi(wh);
    float whCosTheta = wh.z, whSinTheta = sinth(wh);
    V whx = v3(whCosPhi * whCosTheta, whSinPhi * whCosTheta, -whSinTheta);
    V why = v3(-whSinPhi, whCosPhi, 0.f);
    V wd = v3(vdot(wi, whx), vdot(wi, why), vdot(wi, wh));
    float wdTheta = ACOSF(clampf(wd.z, -1.f, 1.f));
    float wdPhi = ATAN2F(wd.y, wd.x);
    wdPhi = (wdPhi < 0.f) ? wdPhi + 2.f * PI_F : wdPhi;
    if (wdPhi > PI_F) wdPhi -= PI_F;
    int whThetaIndex = clampi_((int)(sqrtf(fmaxf_(0.f, whTheta / (PI_F / 2.f))) / 1.f * (float)90), 0, 89);
    int wdThetaIndex = clampi_((int)(wdTheta / (PI_F / 2.f) * (float)90), 0, 89);
    int wdPhiIndex = clampi_((int)(wdPhi / PI_F * (float)180), 0, 179);
    int index = wdPhiIndex + 180 * (wdThetaIndex + whThetaIndex * 90);
    from_rgb(c, &b->merl[3 * index], 0, f);
}
static void bx_f_add(const Ctx *c, const BxDF *b, V wo, V wi, float *out) {
    int nb = c->nb;
    switch (b->kind) {
        case BX_MEASURED_HALF: {
            float f[PBRTGPU_MAX_BANDS];
            halfangle_f(c, b, wo, wi, f);
            for (int i = 0; i < nb; ++i) out[i] += f[i];
            break;
        }
        case BX_MEASURED_IRREG: {
            float f[PBRTGPU_MAX_BANDS];
            irreg_f(c, b, wo, wi, f);
            for (int i = 0; i < nb; ++i) out[i] += f[i];
            break;
        }
        case BX_LAMBERT:
            for (int i = 0; i < nb; ++i) out[i] += b->R[i] * INV_PI_F;
            break;
        case BX_OREN: {   /* reflection.cpp:170-193 */
            float sinthetai = sinth(wi), sinthetao = sinth(wo);
            float maxcos = 0.f;
            if (sinthetai > 1e-4 && sinthetao > 1e-4) {
                float sinphii = sinphi(wi), cosphii = cosphi(wi), sinphio = sinphi(wo), cosphio = cosphi(wo);
                float dcos = cosphii * cosphio + sinphii * sinphio;
                maxcos = fmaxf_(0.f, dcos);
            }
            float sinalpha, tanbeta;
            if (abscos(wi) > abscos(wo)) { sinalpha = sinthetao; tanbeta = sinthetai / abscos(wi); }
            else { sinalpha = sinthetai; tanbeta = sinthetao / abscos(wo); }
            float s = (b->a + b->b * maxcos * sinalpha * tanbeta);
            for (int i = 0; i < nb; ++i) out[i] += (b->R[i] * INV_PI_F) * s;
            break;
        }
        case BX_MICRO_BLINN_DIEL: {   /* Microfacet::f (reflection.cpp:203-214) */
            float cosThetaO = abscos(wo), cosThetaI = abscos(wi);
            if (cosThetaI == 0.f || cosThetaO == 0.f) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            V wh = vadd(wi, wo);
            if (wh.x == 0. && wh.y == 0. && wh.z == 0.) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            wh = vnorm(wh);
            float cosThetaH = vdot(wi, wh);
            float F = fr_dielectric(cosThetaH, b->eta_i, b->eta_t);
            float D = blinn_D(b->a, wh), G = micro_G(wo, wi, wh);
            float den = 4.f * cosThetaI * cosThetaO;
            for (int i = 0; i < nb; ++i) out[i] += (((b->R[i] * D) * G) * F) / den;
            break;
        }
        case BX_MICRO_BLINN_COND: {   /* Microfacet::f with FresnelConductor (reflection.cpp:62-71, 102-104) */
            float cosThetaO = abscos(wo), cosThetaI = abscos(wi);
            if (cosThetaI == 0.f || cosThetaO == 0.f) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            V wh = vadd(wi, wo);
            if (wh.x == 0. && wh.y == 0. && wh.z == 0.) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            wh = vnorm(wh);
            float cosi = fabsf(vdot(wi, wh));
            float D = blinn_D(b->a, wh), G = micro_G(wo, wi, wh);
            float den = 4.f * cosThetaI * cosThetaO;
            for (int i = 0; i < nb; ++i) out[i] += (((1.f * D) * G) * fr_cond(cosi, b->eta[i], b->k[i])) / den;
            break;
        }
        case BX_SPEC_REFL_NOOP:
        case BX_SPEC_REFL_DIEL:
        case BX_SPEC_REFL_COND:
        case BX_SPEC_TRANS:
            for (int i = 0; i < nb; ++i) out[i] += 0.f;
            break;
        case BX_ANISOWARD: {   /* AnisoWardBrdf::f (AnisoWardBrdf.cpp:10-23) */
            V wh = vadd(wi, wo);
            if (wh.z == 0.0f) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            float cosi_coso = wi.z * wo.z;
            if (cosi_coso <= 0.0f) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            float invAx2 = 1.0f / (b->a * b->a), invAy2 = 1.0f / (b->b * b->b);
            float fourPiAxAy = (4.0f * PI_F * b->a * b->b);
            float expTerm = EXPF(-1.0f * (wh.x * wh.x * invAx2 + wh.y * wh.y * invAy2) / (wh.z * wh.z));
            cosi_coso = sqrtf(cosi_coso);
            float den = cosi_coso * fourPiAxAy;
            for (int i = 0; i < nb; ++i) out[i] += (b->R[i] * expTerm) / den;
            break;
        }
        case BX_FRESNEL_BLEND_ANISO: {   /* FresnelBlend::f (reflection.cpp:224-236) */
            float cd = (28.f / (23.f * PI_F));
            float ta = (1.f - POWF(1.f - .5f * abscos(wi), 5)), tb = (1.f - POWF(1.f - .5f * abscos(wo), 5));
            V wh = vadd(wi, wo);
            if (wh.x == 0. && wh.y == 0. && wh.z == 0.) { for (int i = 0; i < nb; ++i) out[i] += 0.f; break; }
            wh = vnorm(wh);
            float D = aniso_D(b->a, b->b, wh);
            float den = (4.f * fabsf(vdot(wi, wh)) * fmaxf_(abscos(wi), abscos(wo)));
            float schl = POWF(1 - vdot(wi, wh), 5.f);
            for (int i = 0; i < nb; ++i) {
                float diffuse = ((((cd * b->R[i]) * (1.f - b->R2[i])) * ta) * tb);
                float schlick = b->R2[i] + schl * (1.f - b->R2[i]);
                float specular = (D / den) * schlick;
                out[i] += diffuse + specular;
            }
            break;
        }
    }
}
static float bx_pdf(const BxDF *b, V wo, V wi) {
    switch (b->kind) {
        case BX_MICRO_BLINN_DIEL:
        case BX_MICRO_BLINN_COND:
            if (!samehemi(wo, wi)) return 0.f;
            return blinn_pdf(b->a, wo, wi);
        case BX_SPEC_REFL_NOOP:
        case BX_SPEC_REFL_DIEL:
        case BX_SPEC_REFL_COND:
        case BX_SPEC_TRANS: return 0.;
        case BX_FRESNEL_BLEND_ANISO:
            if (!samehemi(wo, wi)) return 0.f;
            return .5f * (abscos(wi) * INV_PI_F + aniso_pdf(b->a, b->b, wo, wi));
        default: return samehemi(wo, wi) ? abscos(wi) * INV_PI_F : 0.f;
    }
}
/* BxDF::Sample_f; returns f into fout (overwritten) */
static void bx_sample_f(const Ctx *c, const BxDF *b, V wo, V *wi, float u1, float u2, float *pdf, float *fout) {
    int nb = c->nb;
    for (int i = 0; i < nb; ++i) fout[i] = 0.f;
    switch (b->kind) {
        case BX_MICRO_BLINN_DIEL:
        case BX_MICRO_BLINN_COND:
            blinn_sample(b->a, wo, wi, u1, u2, pdf);
            if (!samehemi(wo, *wi)) return;
            bx_f_add(c, b, wo, *wi, fout);
            return;
        case BX_SPEC_REFL_NOOP: {   /* SpecularReflection::Sample_f with FresnelNoOp */
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            float d = abscos(*wi);
            for (int i = 0; i < nb; ++i) fout[i] = (1.f * b->R[i]) / d;
            return;
        }
        case BX_SPEC_REFL_DIEL: {   /* SpecularReflection::Sample_f (reflection.cpp:130-136), FresnelDielectric(1, ior) */
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            float F = fr_dielectric(costh(wo), 1.f, b->eta_t), d = abscos(*wi);
            for (int i = 0; i < nb; ++i) fout[i] = (F * b->R[i]) / d;
            return;
        }
        case BX_SPEC_REFL_COND: {   /* SpecularReflection::Sample_f, FresnelConductor(eta, 0) (reflection.cpp:102-104) */
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            float ci = fabsf(costh(wo)), d = abscos(*wi);
            for (int i = 0; i < nb; ++i) fout[i] = (fr_cond(ci, b->eta[i], 0.f) * 1.f) / d;
            return;
        }
        case BX_SPEC_TRANS: {   /* SpecularTransmission::Sample_f (reflection.cpp:139-162) */
            int entering = costh(wo) > 0.;
            float ei = 1.f, et = b->eta_t;
            if (!entering) { float t = ei; ei = et; et = t; }
            float sini2 = sin2(wo);
            float eta = ei / et;
            float sint2 = eta * eta * sini2;
            if (sint2 >= 1.) return;
            float cost = sqrtf(fmaxf_(0.f, 1.f - sint2));
            if (entering) cost = -cost;
            float sintOverSini = eta;
            *wi = v3(sintOverSini * -wo.x, sintOverSini * -wo.y, cost);
            *pdf = 1.f;
            float F = fr_dielectric(costh(wo), 1.f, b->eta_t), d = abscos(*wi);
            for (int i = 0; i < nb; ++i) fout[i] = ((1.f - F) * b->R[i]) / d;
            return;
        }
        case BX_FRESNEL_BLEND_ANISO:
            if (u1 < .5) {
                u1 = 2.f * u1;
                *wi = cosine_hemisphere(u1, u2);
                if (wo.z < 0.) wi->z *= -1.f;
            } else {
                u1 = 2.f * (u1 - .5f);
                aniso_sample(b->a, b->b, wo, wi, u1, u2, pdf);
                if (!samehemi(wo, *wi)) return;
            }
            *pdf = bx_pdf(b, wo, *wi);
            bx_f_add(c, b, wo, *wi, fout);
            return;
        default:
            *wi = cosine_hemisphere(u1, u2);
            if (wo.z < 0.) wi->z *= -1.f;
            *pdf = bx_pdf(b, wo, *wi);
            bx_f_add(c, b, wo, *wi, fout);
            return;
    }
}
/* BSDF::f (reflection.cpp:604-618) */
static void bsdf_f(const Ctx *c, const BSDF *bs, V woW, V wiW, int flags, float *f) {
    V wi = to_local(bs, wiW), wo = to_local(bs, woW);
    if (vdot(wiW, bs->ng) * vdot(woW, bs->ng) > 0) flags &= ~BSDF_TRANSMISSION;
    else flags &= ~BSDF_REFLECTION;
    for (int i = 0; i < c->nb; ++i) f[i] = 0.f;
    for (int k = 0; k < bs->n; ++k)
        if (matches(&bs->bx[k], flags)) bx_f_add(c, &bs->bx[k], wo, wi, f);
}
/* BSDF::Pdf (reflection.cpp:575-590) */
static float bsdf_pdf(const BSDF *bs, V woW, V wiW, int flags) {
    if (bs->n == 0.) return 0.;
    V wo = to_local(bs, woW), wi = to_local(bs, wiW);
    float pdf = 0.f;
    int m = 0;
    for (int k = 0; k < bs->n; ++k)
        if (matches(&bs->bx[k], flags)) { ++m; pdf += bx_pdf(&bs->bx[k], wo, wi); }
    return m > 0 ? pdf / m : 0.f;
}
/* BSDF::Sample_f (reflection.cpp:514-572) */
static void bsdf_sample_f(const Ctx *c, const BSDF *bs, V woW, V *wiW, float u0, float u1, float uc, float *pdf,
                          int flags, int *sampledType, float *f) {
    int nb = c->nb;
    int matching = 0;
    for (int k = 0; k < bs->n; ++k) if (matches(&bs->bx[k], flags)) ++matching;
    if (matching == 0) { *pdf = 0.f; *sampledType = 0; for (int i = 0; i < nb; ++i) f[i] = 0.f; return; }
    int which = (int)floorf(uc * matching);
    if (which > matching - 1) which = matching - 1;
    const BxDF *bx = NULL;
    int count = which;
    for (int k = 0; k < bs->n; ++k)
        if (matches(&bs->bx[k], flags) && count-- == 0) { bx = &bs->bx[k]; break; }
    V wo = to_local(bs, woW), wi;
    *pdf = 0.f;
    bx_sample_f(c, bx, wo, &wi, u0, u1, pdf, f);
    if (*pdf == 0.f) { *sampledType = 0; for (int i = 0; i < nb; ++i) f[i] = 0.f; return; }
    *sampledType = bx->type;
    *wiW = to_world(bs, wi);
    if (!(bx->type & BSDF_SPECULAR) && matching > 1)
        for (int k = 0; k < bs->n; ++k)
            if (&bs->bx[k] != bx && matches(&bs->bx[k], flags)) *pdf += bx_pdf(&bs->bx[k], wo, wi);
    if (matching > 1) *pdf /= matching;
    if (!(bx->type & BSDF_SPECULAR)) {
        for (int i = 0; i < nb; ++i) f[i] = 0.f;
        if (vdot(*wiW, bs->ng) * vdot(woW, bs->ng) > 0) flags &= ~BSDF_TRANSMISSION;
        else flags &= ~BSDF_REFLECTION;
        for (int k = 0; k < bs->n; ++k)
            if (matches(&bs->bx[k], flags)) bx_f_add(c, &bs->bx[k], wo, wi, f);
    }
}

/* ------------------------------------------------------------------ RGB spectra, textures */
#ifdef ORACLE_LIBM_FLOAT
#define LOGF logf
#else
static inline float LOGF(float x) { return libmf_logf(x); }
#endif
/* Log2 (pbrt.h:243-246) */
static inline float log2_(float x) { float invLog2 = 1.f / LOGF(2.f); return LOGF(x) * invLog2; }

/* SampledSpectrum::FromRGB (spectrum.cpp:93-178), basis tables from the flattened scene; the RGB
 * build's RGBSpectrum::FromRGB is the triple itself */
static void add_scaled(float *r, int nb, float a, const float *B) { for (int i = 0; i < nb; ++i) r[i] += B[i] * a; }
static void from_rgb(const Ctx *c, const float rgb[3], int illum, float *r) {
    int nb = c->nb;
    if (nb == 3) { r[0] = rgb[0]; r[1] = rgb[1]; r[2] = rgb[2]; return; }   /* RGBSpectrum::FromRGB (spectrum.h:463-470) */
    const float *base = c->s->rgb_basis + (size_t)(illum ? 7 : 0) * nb;
    const float *W = base, *Cy = base + nb, *Mg = base + 2 * nb, *Ye = base + 3 * nb, *Rd = base + 4 * nb,
                *Gr = base + 5 * nb, *Bl = base + 6 * nb;
    for (int i = 0; i < nb; ++i) r[i] = 0.f;
    if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        add_scaled(r, nb, rgb[0], W);
        if (rgb[1] <= rgb[2]) { add_scaled(r, nb, rgb[1] - rgb[0], Cy); add_scaled(r, nb, rgb[2] - rgb[1], Bl); }
        else { add_scaled(r, nb, rgb[2] - rgb[0], Cy); add_scaled(r, nb, rgb[1] - rgb[2], Gr); }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        add_scaled(r, nb, rgb[1], W);
        if (rgb[0] <= rgb[2]) { add_scaled(r, nb, rgb[0] - rgb[1], Mg); add_scaled(r, nb, rgb[2] - rgb[0], Bl); }
        else { add_scaled(r, nb, rgb[2] - rgb[1], Mg); add_scaled(r, nb, rgb[0] - rgb[2], Rd); }
    } else {
        add_scaled(r, nb, rgb[2], W);
        if (rgb[0] <= rgb[1]) { add_scaled(r, nb, rgb[0] - rgb[2], Ye); add_scaled(r, nb, rgb[1] - rgb[0], Gr); }
        else { add_scaled(r, nb, rgb[1] - rgb[2], Ye); add_scaled(r, nb, rgb[0] - rgb[1], Rd); }
    }
    float sc = illum ? .86445f : (float).94;
    for (int i = 0; i < nb; ++i) r[i] = clampf(r[i] * sc, 0.f, INFINITY);
}

/* The environment light's one-texel MIPMap (mipmap.h): Texel with the wrap mode (:197-222),
 * triangle (:263-274); nc = 3 (RGB) or 1 (float) */
static inline float texel_c(const float *T, int wrap, int s, int t, int k) {
    if (wrap == PBRTGPU_WRAP_BLACK && (s != 0 || t != 0)) return 0.f;
    return T[k];
}
static void mip_triangle(const float *T, int nc, int wrap, float s, float t, float *out) {
    s = s * 1.f - 0.5f;
    t = t * 1.f - 0.5f;
    int s0 = (int)floorf(s), t0 = (int)floorf(t);
    float ds = s - s0, dt = t - t0;
    float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
    for (int k = 0; k < nc; ++k)
        out[k] = ((w00 * texel_c(T, wrap, s0, t0, k) + w01 * texel_c(T, wrap, s0, t0 + 1, k)) +
                  w10 * texel_c(T, wrap, s0 + 1, t0, k)) + w11 * texel_c(T, wrap, s0 + 1, t0 + 1, k);
}
/* MIPMap (mipmap.h:119-375) of an IMAGE texture: its pyramid in texels[] from texel_off, level l
 * max(1, width >> l) x max(1, height >> l) texels of nc floats */
typedef struct { const float *T; int w, h; } MipLv;
static MipLv mip_lv(const Ctx *c, const pbrtgpu_texture *tx, int nc, int l) {
    size_t off = (size_t)tx->texel_off;
    int w = tx->width, h = tx->height;
    for (int i = 0; i < l; ++i) {
        off += (size_t)w * h * nc;
        w = w > 1 ? w >> 1 : 1;
        h = h > 1 ? h >> 1 : 1;
    }
    MipLv r = {c->s->texels + off, w, h};
    return r;
}
static int mod_i(int a, int b) { int n = a / b; a -= n * b; if (a < 0) a += b; return a; }   /* pbrt.h Mod */
/* Texel(level, s, t) with the wrap mode (mipmap.h:197-222) */
static void mip_texel(const MipLv *L, int nc, int wrap, int s, int t, float *out) {
    if (wrap == PBRTGPU_WRAP_REPEAT) { s = mod_i(s, L->w); t = mod_i(t, L->h); }
    else if (wrap == PBRTGPU_WRAP_CLAMP) { s = s < 0 ? 0 : (s > L->w - 1 ? L->w - 1 : s); t = t < 0 ? 0 : (t > L->h - 1 ? L->h - 1 : t); }
    else if (s < 0 || s >= L->w || t < 0 || t >= L->h) { for (int k = 0; k < nc; ++k) out[k] = 0.f; return; }
    for (int k = 0; k < nc; ++k) out[k] = L->T[((size_t)t * L->w + s) * nc + k];
}
/* MIPMap::triangle (mipmap.h:263-274) */
static void mip_tri(const Ctx *c, const pbrtgpu_texture *tx, int nc, int level, float s, float t, float *out) {
    level = level < 0 ? 0 : (level > tx->levels - 1 ? tx->levels - 1 : level);
    const MipLv L = mip_lv(c, tx, nc, level);
    s = s * (float)(uint32_t)L.w - 0.5f;
    t = t * (float)(uint32_t)L.h - 0.5f;
    int s0 = (int)floorf(s), t0 = (int)floorf(t);
    float ds = s - s0, dt = t - t0;
    float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
    float a[3], b[3], cc[3], d[3];
    mip_texel(&L, nc, tx->wrap, s0, t0, a);
    mip_texel(&L, nc, tx->wrap, s0, t0 + 1, b);
    mip_texel(&L, nc, tx->wrap, s0 + 1, t0, cc);
    mip_texel(&L, nc, tx->wrap, s0 + 1, t0 + 1, d);
    for (int k = 0; k < nc; ++k) out[k] = ((w00 * a[k] + w01 * b[k]) + w10 * cc[k]) + w11 * d[k];
}
/* MIPMap::EWA (mipmap.h:320-375) */
static void mip_ewa(const Ctx *c, const pbrtgpu_texture *tx, int nc, int level, float s, float t, float ds0, float dt0,
                    float ds1, float dt1, float *out) {
    if (level >= tx->levels) {
        const MipLv Lt = mip_lv(c, tx, nc, tx->levels - 1);
        mip_texel(&Lt, nc, tx->wrap, 0, 0, out);
        return;
    }
    const MipLv L = mip_lv(c, tx, nc, level);
    const float fw = (float)(uint32_t)L.w, fh = (float)(uint32_t)L.h;
    s = s * fw - 0.5f;
    t = t * fh - 0.5f;
    ds0 *= fw; dt0 *= fh; ds1 *= fw; dt1 *= fh;
    float A = dt0 * dt0 + dt1 * dt1 + 1;
    float B = -2.f * (ds0 * dt0 + ds1 * dt1);
    float C = ds0 * ds0 + ds1 * ds1 + 1;
    float invF = 1.f / (A * C - B * B * 0.25f);
    A *= invF; B *= invF; C *= invF;
    float det = -B * B + 4.f * A * C;
    float invDet = 1.f / det;
    float uSqrt = sqrtf(det * C), vSqrt = sqrtf(A * det);
    int s0 = (int)ceilf(s - 2.f * invDet * uSqrt), s1 = (int)floorf(s + 2.f * invDet * uSqrt);
    int t0 = (int)ceilf(t - 2.f * invDet * vSqrt), t1 = (int)floorf(t + 2.f * invDet * vSqrt);
    float sum[3] = {0.f, 0.f, 0.f}, sumWts = 0.f;
    for (int it = t0; it <= t1; ++it) {
        float tt = it - t;
        for (int is = s0; is <= s1; ++is) {
            float ss = is - s;
            float r2 = A * ss * ss + B * ss * tt + C * tt * tt;
            if (r2 < 1.) {
                int li = (int)(r2 * 128);
                float weight = c->s->ewa_lut[li < 127 ? li : 127], tv[3];
                mip_texel(&L, nc, tx->wrap, is, it, tv);
                for (int k = 0; k < nc; ++k) sum[k] += tv[k] * weight;
                sumWts += weight;
            }
        }
    }
    for (int k = 0; k < nc; ++k) out[k] = sum[k] / sumWts;
}
/* MIPMap::Lookup(s, t, width) (mipmap.h:226-259) with the fork's noFiltering nearest texel */
static void mip_lookup_w(const Ctx *c, const pbrtgpu_texture *tx, int nc, float s, float t, float width, float *out) {
    if (tx->nofilter) {
        const MipLv L = mip_lv(c, tx, nc, 0);
        s = s * (float)(uint32_t)L.w - 0.5f;
        t = t * (float)(uint32_t)L.h - 0.5f;
        mip_texel(&L, nc, tx->wrap, (int)floorf(s + 0.5f), (int)floorf(t + 0.5f), out);   /* Round2Int */
        return;
    }
    float level = (float)(uint32_t)(tx->levels - 1) + log2_(fmaxf_(width, 1e-8f));
    if (level < 0) mip_tri(c, tx, nc, 0, s, t, out);
    else if (level >= (float)(uint32_t)(tx->levels - 1)) {
        const MipLv Lt = mip_lv(c, tx, nc, tx->levels - 1);
        mip_texel(&Lt, nc, tx->wrap, 0, 0, out);
    } else {
        int iLevel = (int)floorf(level);
        float delta = level - iLevel, a[3], b[3];
        mip_tri(c, tx, nc, iLevel, s, t, a);
        mip_tri(c, tx, nc, iLevel + 1, s, t, b);
        for (int k = 0; k < nc; ++k) out[k] = (1.f - delta) * a[k] + delta * b[k];
    }
}
/* MIPMap::Lookup(s, t, ds0, dt0, ds1, dt1) (mipmap.h:278-318) */
static void mip_lookup(const Ctx *c, const pbrtgpu_texture *tx, int nc, float s, float t, float ds0, float dt0, float ds1,
                       float dt1, float *out) {
    if (tx->trilinear) {
        mip_lookup_w(c, tx, nc, s, t, 2.f * fmaxf_(fmaxf_(fabsf(ds0), fabsf(dt0)), fmaxf_(fabsf(ds1), fabsf(dt1))), out);
        return;
    }
    if (ds0 * ds0 + dt0 * dt0 < ds1 * ds1 + dt1 * dt1) {
        float a = ds0; ds0 = ds1; ds1 = a;
        a = dt0; dt0 = dt1; dt1 = a;
    }
    float majorLength = sqrtf(ds0 * ds0 + dt0 * dt0);
    float minorLength = sqrtf(ds1 * ds1 + dt1 * dt1);
    if (minorLength * tx->max_aniso < majorLength && minorLength > 0.f) {
        float scale = majorLength / (minorLength * tx->max_aniso);
        ds1 *= scale; dt1 *= scale; minorLength *= scale;
    }
    if (minorLength == 0.f) { mip_tri(c, tx, nc, 0, s, t, out); return; }
    float lod = fmaxf_(0.f, (float)(uint32_t)tx->levels - 1.f + log2_(minorLength));
    int ilod = (int)floorf(lod);
    float d = lod - (float)(uint32_t)ilod;
    float e0[3], e1[3];
    mip_ewa(c, tx, nc, ilod, s, t, ds0, dt0, ds1, dt1, e0);
    mip_ewa(c, tx, nc, ilod + 1, s, t, ds0, dt0, ds1, dt1, e1);
    for (int k = 0; k < nc; ++k) out[k] = (1.f - d) * e0[k] + d * e1[k];
}
/* texture-space position and screen-space derivatives of the hit (dgs.u, v, dudx, ...), and its
 * world-space point with the ray-differential offsets dpdx, dpdy (the non-uv mappings) */
typedef struct { float u, v, dudx, dvdx, dudy, dvdy; V p, dpdx, dpdy; } TexPt;
/* SphericalMapping2D::sphere (texture.cpp:104-110), CylindricalMapping2D::cylinder (texture.h);
 * M_PI is a float in pbrt (pbrt.h:176-179) */
static void map_dir(const pbrtgpu_texture *tx, V p, float *s, float *t) {
    V vec = vnorm(xpoint(tx->map, p));
    if (tx->mapping == PBRTGPU_MAP_SPHERICAL) {
        float theta = ACOSF(clampf(vec.z, -1.f, 1.f));
        float pp = ATAN2F(vec.y, vec.x);
        float phi = (pp < 0.f) ? pp + 2.f * PI_F : pp;
        *s = theta * INV_PI_F;
        *t = phi * INV_TWOPI_F;
    } else {
        *s = (PI_F + ATAN2F(vec.y, vec.x)) / (2.f * PI_F);
        *t = vec.z;
    }
}
/* TextureMapping2D::Map: UVMapping2D (texture.cpp:80-90), SphericalMapping2D (:93-110, delta
 * .1f), CylindricalMapping2D (:113-131, delta .01f), PlanarMapping2D (:134-144) */
static void tex_map(const pbrtgpu_texture *tx, const TexPt *q, float *s, float *t, float *dsdx, float *dtdx,
                    float *dsdy, float *dtdy) {
    if (tx->mapping == PBRTGPU_MAP_UV) {
        *s = tx->su * q->u + tx->du; *t = tx->sv * q->v + tx->dv;
        *dsdx = tx->su * q->dudx; *dtdx = tx->sv * q->dvdx; *dsdy = tx->su * q->dudy; *dtdy = tx->sv * q->dvdy;
    } else if (tx->mapping == PBRTGPU_MAP_PLANAR) {
        V vs = v3(tx->map[0], tx->map[1], tx->map[2]), vt = v3(tx->map[3], tx->map[4], tx->map[5]);
        V vec = vsub(q->p, v3(0.f, 0.f, 0.f));
        *s = tx->du + vdot(vec, vs); *t = tx->dv + vdot(vec, vt);
        *dsdx = vdot(q->dpdx, vs); *dtdx = vdot(q->dpdx, vt); *dsdy = vdot(q->dpdy, vs); *dtdy = vdot(q->dpdy, vt);
    } else {
        const float delta = tx->mapping == PBRTGPU_MAP_SPHERICAL ? .1f : .01f;
        float sx, tx_, sy, ty;
        map_dir(tx, q->p, s, t);
        map_dir(tx, vadd(q->p, vmul(q->dpdx, delta)), &sx, &tx_);
        *dsdx = (sx - *s) / delta;
        *dtdx = (tx_ - *t) / delta;
        if (*dtdx > .5) *dtdx = 1.f - *dtdx;
        else if (*dtdx < -.5f) *dtdx = -(*dtdx + 1);
        map_dir(tx, vadd(q->p, vmul(q->dpdy, delta)), &sy, &ty);
        *dsdy = (sy - *s) / delta;
        *dtdy = (ty - *t) / delta;
        if (*dtdy > .5) *dtdy = 1.f - *dtdy;
        else if (*dtdy < -.5f) *dtdy = -(*dtdy + 1);
    }
}
/* ImageTexture::Evaluate (imagemap.cpp:84-101) */
static void tex_image(const Ctx *c, const pbrtgpu_texture *tx, int nc, const TexPt *q, float *out) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    mip_lookup(c, tx, nc, s, t, dsdx, dtdx, dsdy, dtdy, out);
}
/* Perlin noise (texture.cpp:163-250): NoisePerm, Grad, NoiseWeight, Noise, FBm, Turbulence */
static const int kNoisePerm[512] = {
#include "pbrt_noise_perm.inc"
};
static float noise_grad(int x, int y, int z, float dx, float dy, float dz) {
    int h = kNoisePerm[kNoisePerm[kNoisePerm[x] + y] + z];
    h &= 15;
    float u = h < 8 || h == 12 || h == 13 ? dx : dy;
    float v = h < 4 || h == 12 || h == 13 ? dy : dz;
    return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}
static float noise_weight(float t) { float t3 = t * t * t; float t4 = t3 * t; return 6.f * t4 * t - 15.f * t4 + 10.f * t3; }
static float noise3(float x, float y, float z) {
    int ix = (int)floorf(x), iy = (int)floorf(y), iz = (int)floorf(z);
    float dx = x - ix, dy = y - iy, dz = z - iz;
    ix &= 255; iy &= 255; iz &= 255;
    float w000 = noise_grad(ix, iy, iz, dx, dy, dz);
    float w100 = noise_grad(ix + 1, iy, iz, dx - 1, dy, dz);
    float w010 = noise_grad(ix, iy + 1, iz, dx, dy - 1, dz);
    float w110 = noise_grad(ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    float w001 = noise_grad(ix, iy, iz + 1, dx, dy, dz - 1);
    float w101 = noise_grad(ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    float w011 = noise_grad(ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    float w111 = noise_grad(ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    float wx = noise_weight(dx), wy = noise_weight(dy), wz = noise_weight(dz);
    float x00 = lerpf(wx, w000, w100), x10 = lerpf(wx, w010, w110);
    float x01 = lerpf(wx, w001, w101), x11 = lerpf(wx, w011, w111);
    float y0 = lerpf(wy, x00, x10), y1 = lerpf(wy, x01, x11);
    return lerpf(wz, y0, y1);
}
static float smoothstep_(float a, float b, float value) {
    float v = clampf((value - a) / (b - a), 0.f, 1.f);
    return v * v * (-2.f * v + 3.f);
}
static float fbm_turb(V P, V dpdx, V dpdy, float omega, int maxOctaves, int turb) {
    float s2 = fmaxf_(vdot(dpdx, dpdx), vdot(dpdy, dpdy));
    float foctaves = fminf_((float)maxOctaves, 1.f - .5f * log2_(s2));
    int octaves = (int)floorf(foctaves);
    float sum = 0., lambda = 1., o = 1.;
    for (int i = 0; i < octaves; ++i) {
        float n = noise3(P.x * lambda, P.y * lambda, P.z * lambda);
        sum += o * (turb ? fabsf(n) : n);
        lambda *= 1.99f;
        o *= omega;
    }
    float partialOctave = foctaves - octaves;
    float n = noise3(P.x * lambda, P.y * lambda, P.z * lambda);
    sum += o * smoothstep_(.3f, .7f, partialOctave) * (turb ? fabsf(n) : n);
    if (turb) sum += (maxOctaves - foctaves) * 0.2f;
    return sum;
}
/* DotsTexture::Evaluate (dots.h:47-66): 1 = tex2 (insideDot, the "outside" parameter), 0 = tex1 */
static int dots_pick(const pbrtgpu_texture *tx, const TexPt *q) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    int sCell = (int)floorf(s + .5f), tCell = (int)floorf(t + .5f);
    if (noise3(sCell + .5f, tCell + .5f, .5f) > 0) {
        float radius = .35f;
        float maxShift = 0.5f - radius;
        float sCenter = sCell + maxShift * noise3(sCell + 1.5f, tCell + 2.8f, .5f);
        float tCenter = tCell + maxShift * noise3(sCell + 4.5f, tCell + 9.8f, .5f);
        float ds = s - sCenter, dt = t - tCenter;
        if (ds * ds + dt * dt < radius * radius) return 1;
    }
    return 0;
}
/* FBmTexture / WrinkledTexture / WindyTexture (fbm.h, wrinkled.h, windy.h) over IdentityMapping3D */
static float tex_noise(const pbrtgpu_texture *tx, const TexPt *q) {
    V P = xpoint(tx->map, q->p), dpdx = xvec(tx->map, q->dpdx), dpdy = xvec(tx->map, q->dpdy);
    if (tx->type == PBRTGPU_TEX_WINDY) {
        float windStrength = fbm_turb(vmul(P, .1f), vmul(dpdx, .1f), vmul(dpdy, .1f), .5f, 3, 0);
        float waveHeight = fbm_turb(P, dpdx, dpdy, .5f, 6, 0);
        return fabsf(windStrength) * waveHeight;
    }
    if (tx->type == PBRTGPU_TEX_MARBLE) {   /* MarbleTexture::Evaluate (marble.h:45-49): the spline's t */
        float sc = tx->su;
        V Ps = vmul(P, sc);
        float marble = Ps.y + tx->sv * fbm_turb(Ps, vmul(dpdx, sc), vmul(dpdy, sc), tx->value, tx->levels, 0);
        return .5f + .5f * SINF(marble);
    }
    return fbm_turb(P, dpdx, dpdy, tx->value, tx->levels, tx->type == PBRTGPU_TEX_WRINKLED);
}
/* UVTexture::Evaluate / EvaluateMemory (uv.h:38-51): the RGB (s - Floor2Int(s), t - Floor2Int(t), 0) */
static void uv_rgb(const pbrtgpu_texture *tx, const TexPt *q, float rgb[3]) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    rgb[0] = s - (float)(int)floorf(s);
    rgb[1] = t - (float)(int)floorf(t);
    rgb[2] = 0.f;
}
/* Checkerboard2DTexture::Evaluate (checkerboard.h:84-125) without its operands: 0 = tex1, 1 = tex2,
 * 2 = (1 - area2) * tex1 + area2 * tex2 */
static float bumpint(float x) { int f = (int)floorf(x / 2); return (float)f + 2.f * fmaxf_((x / 2) - (float)f - .5f, 0.f); }
static int checker_pick(const pbrtgpu_texture *tx, const TexPt *q, float *area2) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    int point = (((int)floorf(s) + (int)floorf(t)) % 2 == 0) ? 0 : 1;
    if (tx->aamode == 1) return point;
    float ds = fmaxf_(fabsf(dsdx), fabsf(dsdy)), dt = fmaxf_(fabsf(dtdx), fabsf(dtdy));
    float s0 = s - ds, s1 = s + ds, t0 = t - dt, t1 = t + dt;
    if ((int)floorf(s0) == (int)floorf(s1) && (int)floorf(t0) == (int)floorf(t1)) return point;
    float sint = (bumpint(s1) - bumpint(s0)) / (2.f * ds);
    float tint = (bumpint(t1) - bumpint(t0)) / (2.f * dt);
    float a = sint + tint - 2.f * sint * tint;
    if (ds > 1.f || dt > 1.f) a = .5f;
    *area2 = a;
    return 2;
}
static float tex_float(const Ctx *c, int id, const TexPt *q) {
    const pbrtgpu_texture *tx = &c->s->textures[id];
    switch (tx->type) {
        case PBRTGPU_TEX_CONST: return tx->value;
        case PBRTGPU_TEX_IMAGE: { float v; tex_image(c, tx, 1, q, &v); return v; }
        case PBRTGPU_TEX_CHECKER: {
            float a2 = 0.f;
            int k = checker_pick(tx, q, &a2);
            if (k < 2) return tex_float(c, k == 0 ? tx->tex1 : tx->tex2, q);
            return (1.f - a2) * tex_float(c, tx->tex1, q) + a2 * tex_float(c, tx->tex2, q);
        }
        case PBRTGPU_TEX_FBM: case PBRTGPU_TEX_WRINKLED: case PBRTGPU_TEX_WINDY: return tex_noise(tx, q);
        case PBRTGPU_TEX_DOTS: return tex_float(c, dots_pick(tx, q) ? tx->tex2 : tx->tex1, q);
        case PBRTGPU_TEX_BILERP: {   /* BilerpTexture::Evaluate (bilerp.h:38-44) */
            float s, t, dsdx, dtdx, dsdy, dtdy;
            tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
            const float *v = &c->s->texels[tx->texel_off];
            return (1 - s) * (1 - t) * v[0] + (1 - s) * (t) * v[1] + (s) * (1 - t) * v[2] + (s) * (t) * v[3];
        }
        case PBRTGPU_TEX_MIX: {   /* MixTexture::Evaluate (mix.h:38-43) */
            float amt = tex_float(c, tx->amount, q);
            return (1.f - amt) * tex_float(c, tx->tex1, q) + amt * tex_float(c, tx->tex2, q);
        }
        default: return tex_float(c, tx->tex1, q) * tex_float(c, tx->tex2, q);   /* ScaleTexture */
    }
}
static void tex_spec(const Ctx *c, int id, const TexPt *q, float *out) {
    const pbrtgpu_texture *tx = &c->s->textures[id];
    int nb = c->nb;
    switch (tx->type) {
        case PBRTGPU_TEX_CONST: memcpy(out, SPEC(c, tx->spec), sizeof(float) * nb); return;
        case PBRTGPU_TEX_IMAGE: { float rgb[3]; tex_image(c, tx, 3, q, rgb); from_rgb(c, rgb, 0, out); return; }
        case PBRTGPU_TEX_UV: { float rgb[3]; uv_rgb(tx, q, rgb); from_rgb(c, rgb, 0, out); return; }
        case PBRTGPU_TEX_DOTS: tex_spec(c, dots_pick(tx, q) ? tx->tex2 : tx->tex1, q, out); return;
        case PBRTGPU_TEX_FBM: case PBRTGPU_TEX_WRINKLED: case PBRTGPU_TEX_WINDY: {   /* Spectrum(FBm(...)) */
            float v = tex_noise(tx, q);
            for (int i = 0; i < nb; ++i) out[i] = v;
            return;
        }
        case PBRTGPU_TEX_MARBLE: {   /* marble.h:50-66; first clamped to 0..5 (6 reads past the table) */
            float t = tex_noise(tx, q) * 6.f;
            float ff = floorf(t);
            int first = ff >= 5.f ? 5 : (ff >= 0.f ? (int)ff : 0);
            t = t - (float)first;
            float u = 1.f - t;
            const float *c0 = SPEC(c, tx->spec + first * nb), *c1 = c0 + nb, *c2 = c1 + nb, *c3 = c2 + nb;
            for (int i = 0; i < nb; ++i) {
                float s0 = c0[i] * u + c1[i] * t, s1 = c1[i] * u + c2[i] * t, s2 = c2[i] * u + c3[i] * t;
                s0 = s0 * u + s1 * t;
                s1 = s1 * u + s2 * t;
                out[i] = (s0 * u + s1 * t) * 1.5f;
            }
            return;
        }
        case PBRTGPU_TEX_BILERP: {
            float s, t, dsdx, dtdx, dsdy, dtdy;
            tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
            const float w00 = (1 - s) * (1 - t), w01 = (1 - s) * (t), w10 = (s) * (1 - t), w11 = (s) * (t);
            const float *v00 = SPEC(c, tx->spec), *v01 = SPEC(c, tx->spec + nb), *v10 = SPEC(c, tx->spec + 2 * nb),
                        *v11 = SPEC(c, tx->spec + 3 * nb);
            for (int i = 0; i < nb; ++i) out[i] = ((v00[i] * w00 + v01[i] * w01) + v10[i] * w10) + v11[i] * w11;
            return;
        }
        case PBRTGPU_TEX_MIX: {
            float a[MAXB], b[MAXB];
            tex_spec(c, tx->tex1, q, a);
            tex_spec(c, tx->tex2, q, b);
            float amt = tex_float(c, tx->amount, q);
            for (int i = 0; i < nb; ++i) out[i] = (a[i] * (1.f - amt)) + (b[i] * amt);
            return;
        }
        case PBRTGPU_TEX_CHECKER: {
            float a2 = 0.f;
            int k = checker_pick(tx, q, &a2);
            if (k < 2) { tex_spec(c, k == 0 ? tx->tex1 : tx->tex2, q, out); return; }
            float a[MAXB], b[MAXB];
            tex_spec(c, tx->tex1, q, a);
            tex_spec(c, tx->tex2, q, b);
            for (int i = 0; i < nb; ++i) out[i] = (a[i] * (1.f - a2)) + (b[i] * a2);   /* s * a, then the sum */
            return;
        }
        default: {
            float a[MAXB], b[MAXB];
            tex_spec(c, tx->tex1, q, a);
            tex_spec(c, tx->tex2, q, b);
            for (int i = 0; i < nb; ++i) out[i] = a[i] * b[i];
        }
    }
}
/* camera ray differentials (perspective.cpp:98-104 + RayDifferential::ScaleDifferentials) */
typedef struct { V rxo, rxd, ryo, ryd; int has; } RayDiff;
/* DifferentialGeometry::ComputeDifferentials (diffgeom.cpp:50-105): out = dudx, dvdx, dudy, dvdy;
 * dpdx / dpdy (may be NULL) = px - p, py - p, zero where the reference zeroes them */
static void compute_differentials2(const DG *dg, const RayDiff *rd, float out[4], V *dpdx, V *dpdy) {
    out[0] = out[1] = out[2] = out[3] = 0.f;
    if (dpdx) *dpdx = v3(0.f, 0.f, 0.f);
    if (dpdy) *dpdy = v3(0.f, 0.f, 0.f);
    if (!rd || !rd->has) return;
    float d = -vdot(dg->nn, dg->p);
    float tx = -(vdot(dg->nn, rd->rxo) + d) / vdot(dg->nn, rd->rxd);
    if (isnan(tx)) return;
    V px = vadd(rd->rxo, vmul(rd->rxd, tx));
    float ty = -(vdot(dg->nn, rd->ryo) + d) / vdot(dg->nn, rd->ryd);
    if (isnan(ty)) return;
    V py = vadd(rd->ryo, vmul(rd->ryd, ty));
    if (dpdx) *dpdx = vsub(px, dg->p);
    if (dpdy) *dpdy = vsub(py, dg->p);
    int a0, a1;
    if (fabsf(dg->nn.x) > fabsf(dg->nn.y) && fabsf(dg->nn.x) > fabsf(dg->nn.z)) { a0 = 1; a1 = 2; }
    else if (fabsf(dg->nn.y) > fabsf(dg->nn.z)) { a0 = 0; a1 = 2; }
    else { a0 = 0; a1 = 1; }
    float A[2][2] = {{vcomp(dg->dpdu, a0), vcomp(dg->dpdv, a0)}, {vcomp(dg->dpdu, a1), vcomp(dg->dpdv, a1)}};
    float Bx[2] = {vcomp(px, a0) - vcomp(dg->p, a0), vcomp(px, a1) - vcomp(dg->p, a1)};
    float By[2] = {vcomp(py, a0) - vcomp(dg->p, a0), vcomp(py, a1) - vcomp(dg->p, a1)};
    if (!solve2x2(A, Bx, &out[0], &out[1])) out[0] = out[1] = 0.f;
    if (!solve2x2(A, By, &out[2], &out[3])) out[2] = out[3] = 0.f;
}
/* out = dudx, dvdx, dudy, dvdy, dpdx.xyz, dpdy.xyz (zero where the reference leaves them zero) */
static void compute_differentials(const DG *dg, const RayDiff *rd, float out[10]) {
    for (int i = 0; i < 10; ++i) out[i] = 0.f;
    if (!rd || !rd->has) return;
    float d = -vdot(dg->nn, dg->p);
    float tx = -(vdot(dg->nn, rd->rxo) + d) / vdot(dg->nn, rd->rxd);
    if (isnan(tx)) return;
    V px = vadd(rd->rxo, vmul(rd->rxd, tx));
    float ty = -(vdot(dg->nn, rd->ryo) + d) / vdot(dg->nn, rd->ryd);
    if (isnan(ty)) return;
    V py = vadd(rd->ryo, vmul(rd->ryd, ty));
    V dpx = vsub(px, dg->p), dpy = vsub(py, dg->p);
    out[4] = dpx.x; out[5] = dpx.y; out[6] = dpx.z; out[7] = dpy.x; out[8] = dpy.y; out[9] = dpy.z;
    int a0, a1;
    if (fabsf(dg->nn.x) > fabsf(dg->nn.y) && fabsf(dg->nn.x) > fabsf(dg->nn.z)) { a0 = 1; a1 = 2; }
    else if (fabsf(dg->nn.y) > fabsf(dg->nn.z)) { a0 = 0; a1 = 2; }
    else { a0 = 0; a1 = 1; }
    float A[2][2] = {{vcomp(dg->dpdu, a0), vcomp(dg->dpdv, a0)}, {vcomp(dg->dpdu, a1), vcomp(dg->dpdv, a1)}};
    float Bx[2] = {vcomp(px, a0) - vcomp(dg->p, a0), vcomp(px, a1) - vcomp(dg->p, a1)};
    float By[2] = {vcomp(py, a0) - vcomp(dg->p, a0), vcomp(py, a1) - vcomp(dg->p, a1)};
    if (!solve2x2(A, Bx, &out[0], &out[1])) out[0] = out[1] = 0.f;
    if (!solve2x2(A, By, &out[2], &out[3])) out[2] = out[3] = 0.f;
}

/* Texture<Spectrum>::EvaluateMemory of a leaf (the fork's RGB before FromRGB): an image map's
 * MIPMap lookup, RGB 0 for a constant (constant.h:45-47) */
static void tex_memory_leaf(const Ctx *c, int id, const TexPt *q, float rgb[3]) {
    const pbrtgpu_texture *tx = &c->s->textures[id];
    if (tx->type == PBRTGPU_TEX_IMAGE) tex_image(c, tx, 3, q, rgb);
    else if (tx->type == PBRTGPU_TEX_UV) uv_rgb(tx, q, rgb);
    else rgb[0] = rgb[1] = rgb[2] = 0.f;
}
/* Material::NormalMap (material.cpp:82-126), taken by every material where the map's Evaluate is
 * not black (e.g. matte.cpp:40-47); returns 0 when it is black (Bump then), else the rotated
 * shading normal in *nOut (before the orientation flip and Faceforward) */
static int normal_map(const Ctx *c, int id, const TexPt *q, V nn, V *nOut) {
    float sp[MAXB];
    tex_spec(c, id, q, sp);
    if (spec_black(c, sp)) return 0;
    const pbrtgpu_texture *tx = &c->s->textures[id];
    float rgb[3];
    if (tx->type == PBRTGPU_TEX_SCALE) {   /* ScaleTexture::EvaluateMemory: tex1 * tex2 (scale.h:47-49) */
        float a[3], b[3];
        tex_memory_leaf(c, tx->tex1, q, a);
        tex_memory_leaf(c, tx->tex2, q, b);
        for (int k = 0; k < 3; ++k) rgb[k] = a[k] * b[k];
    } else tex_memory_leaf(c, id, q, rgb);
    for (int k = 0; k < 3; ++k) rgb[k] = rgb[k] * 2 - 1;
    V n = vnorm(v3(rgb[0], rgb[1], rgb[2]));
    V axis = vcross(v3(0.f, 0.f, 1.f), n);
    float angle = (180.f / (float)M_PI) * ACOSF(vdot(v3(0.f, 0.f, 1.f), n));   /* Degrees */
    /* Rotate (transform.cpp:197-224), then Transform::operator()(Normal) with mInv = Transpose(m) */
    V a = vnorm(axis);
    float s = SINF(((float)M_PI / 180.f) * angle), co = COSF(((float)M_PI / 180.f) * angle);
    float m[3][3] = {{a.x * a.x + (1.f - a.x * a.x) * co, a.x * a.y * (1.f - co) - a.z * s, a.x * a.z * (1.f - co) + a.y * s},
                     {a.x * a.y * (1.f - co) + a.z * s, a.y * a.y + (1.f - a.y * a.y) * co, a.y * a.z * (1.f - co) - a.x * s},
                     {a.x * a.z * (1.f - co) - a.y * s, a.y * a.z * (1.f - co) + a.x * s, a.z * a.z + (1.f - a.z * a.z) * co}};
    *nOut = v3(m[0][0] * nn.x + m[0][1] * nn.y + m[0][2] * nn.z, m[1][0] * nn.x + m[1][1] * nn.y + m[1][2] * nn.z,
               m[2][0] * nn.x + m[2][1] * nn.y + m[2][2] * nn.z);
    return 1;
}

/* Intersection::GetBSDF -> GetShadingGeometry -> Material::GetBSDF (with Bump or NormalMap) */
static void get_bsdf(const Ctx *c, const Isect *is, const float diff[10], BSDF *bs, DG *dgsOut) {
    const pbrtgpu_prim *pr = &c->s->prims[is->prim];
    const pbrtgpu_material *mt = &c->s->materials[pr->material];
    DG dgs;
    int ro, swaps;
    if (pr->shape_type == PBRTGPU_SHAPE_TRIANGLE) {
        const pbrtgpu_mesh *m = &c->s->meshes[c->s->tris[pr->shape_index].mesh];
        tri_shading(c, pr->shape_index, is->inst >= 0 ? is->nmat : m->o2w_minv, &is->dg, &dgs);
        ro = m->reverse_orientation; swaps = m->swaps_handedness;
    } else {
        dgs = is->dg;
        const pbrtgpu_quadric *q = &c->s->quadrics[pr->shape_index];
        ro = q->reverse_orientation; swaps = q->swaps_handedness;
    }
    const TexPt q = {dgs.u, dgs.v, diff[0], diff[1], diff[2], diff[3], dgs.p, {diff[4], diff[5], diff[6]},
                     {diff[7], diff[8], diff[9]}};
    DG b = dgs;
    V nmapN;
    const int nmap = mt->normal_tex >= 0 && normal_map(c, mt->normal_tex, &q, dgs.nn, &nmapN);
    if (nmap) {
        /* dgBump = dgs with the rotated normal */
    } else if (mt->bump_tex < 0) {
        /* Material::Bump with constant displacement d (material.cpp:39-81); du = dv = .01f
         * gives the identical result for any positive du because (d - d) == 0 */
        float d = mt->f[7];
        float du = .01f, dv = .01f;
        b.dpdu = vadd(vadd(dgs.dpdu, vmul(dgs.nn, (d - d) / du)), vmul(dgs.dndu, d));
        b.dpdv = vadd(vadd(dgs.dpdv, vmul(dgs.nn, (d - d) / dv)), vmul(dgs.dndv, d));
    } else {
        /* Material::Bump with a displacement texture: u- and v-shifted evaluations */
        float du = .5f * (fabsf(q.dudx) + fabsf(q.dudy));
        if (du == 0.f) du = .01f;
        TexPt qu = q; qu.u = dgs.u + du; qu.p = vadd(dgs.p, vmul(dgs.dpdu, du));   /* dgEval.p (material.cpp:49) */
        float uDisplace = tex_float(c, mt->bump_tex, &qu);
        float dv = .5f * (fabsf(q.dvdx) + fabsf(q.dvdy));
        if (dv == 0.f) dv = .01f;
        TexPt qv = q; qv.v = dgs.v + dv; qv.p = vadd(dgs.p, vmul(dgs.dpdv, dv));
        float vDisplace = tex_float(c, mt->bump_tex, &qv);
        float displace = tex_float(c, mt->bump_tex, &q);
        b.dpdu = vadd(vadd(dgs.dpdu, vmul(dgs.nn, (uDisplace - displace) / du)), vmul(dgs.dndu, displace));
        b.dpdv = vadd(vadd(dgs.dpdv, vmul(dgs.nn, (vDisplace - displace) / dv)), vmul(dgs.dndv, displace));
    }
    b.nn = nmap ? nmapN : vnorm(vcross(b.dpdu, b.dpdv));
    if (ro ^ swaps) b.nn = vmul(b.nn, -1.f);
    b.nn = faceforward(b.nn, is->dg.nn);
    /* BSDF ctor (reflection.cpp:593-601) */
    bs->ng = is->dg.nn;
    bs->nn = b.nn;
    bs->sn = vnorm(b.dpdu);
    bs->tn = vcross(bs->nn, bs->sn);
    bs->n = 0;
    *dgsOut = b;
    /* material spectra (slots 0, 1): constants, or textures evaluated here -- .Clamp()ed, except
       metal's eta and k (metal.cpp:64-65: Evaluate(dgs) as is; black_mask bit 4 + k) */
    const float *K[2];
    int black[2];
    for (int k = 0; k < 2; ++k) {
        if (mt->tex[k] >= 0) {
            tex_spec(c, mt->tex[k], &q, bs->texbuf[k]);
            if (!((mt->black_mask >> (4 + k)) & 1))
                for (int i = 0; i < c->nb; ++i) bs->texbuf[k][i] = clampf(bs->texbuf[k][i], 0.f, INFINITY);
            K[k] = bs->texbuf[k];
            black[k] = spec_black(c, bs->texbuf[k]);
        } else {
            K[k] = mt->spec[k] >= 0 ? SPEC(c, mt->spec[k]) : NULL;
            black[k] = (mt->black_mask >> k) & 1;
        }
    }
    /* float parameters f[0], f[1]: constants or float textures at the shading geometry (matte's
       sigma clamped to [0, 90], matte.cpp:54; plastic / metal roughness, substrate u / v roughness,
       glass index: Evaluate(dgs) as is) */
    float fp[2];
    for (int j = 0; j < 2; ++j) {
        fp[j] = mt->f[j];
        if (mt->ftex[j] >= 0) {
            fp[j] = tex_float(c, mt->ftex[j], &q);
            if (mt->type == PBRTGPU_MAT_MATTE) fp[j] = clampf(fp[j], 0.f, 90.f);
        }
    }
    bs->eta = mt->type == PBRTGPU_MAT_GLASS ? fp[0] : 1.f;
    switch (mt->type) {
        case PBRTGPU_MAT_MATTE: {
            BxDF *x = &bs->bx[bs->n++];
            x->R = K[0];
            x->type = BSDF_REFLECTION | BSDF_DIFFUSE;
            float sig = fp[0];
            if (sig == 0.) x->kind = BX_LAMBERT;
            else {
                x->kind = BX_OREN;
                float sigma = (PI_F / 180.f) * sig;
                float sigma2 = sigma * sigma;
                x->a = 1.f - (sigma2 / (2.f * (sigma2 + 0.33f)));
                x->b = 0.45f * sigma2 / (sigma2 + 0.09f);
            }
            break;
        }
        case PBRTGPU_MAT_PLASTIC: {   /* plastic.cpp:34-61 */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_LAMBERT; x->type = BSDF_REFLECTION | BSDF_DIFFUSE; x->R = K[0];
            x = &bs->bx[bs->n++];
            x->kind = BX_MICRO_BLINN_DIEL; x->type = BSDF_REFLECTION | BSDF_GLOSSY; x->R = K[1];
            float e = 1.f / fp[0];
            if (e > 10000.f || isnan(e)) e = 10000.f;   /* Blinn ctor */
            x->a = e; x->eta_i = 1.5f; x->eta_t = 1.f;
            break;
        }
        case PBRTGPU_MAT_METAL: {   /* metal.cpp:44-62: Microfacet(1, FresnelConductor(eta, k), Blinn(1/rough)) */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_MICRO_BLINN_COND; x->type = BSDF_REFLECTION | BSDF_GLOSSY;
            x->eta = K[0]; x->k = K[1];
            float e = 1.f / fp[0];
            if (e > 10000.f || isnan(e)) e = 10000.f;
            x->a = e;
            break;
        }
        case PBRTGPU_MAT_SHINYMETAL: {   /* shinymetal.cpp:45-68 */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_MICRO_BLINN_COND; x->type = BSDF_REFLECTION | BSDF_GLOSSY;
            x->eta = K[0]; x->k = SPEC(c, mt->spec[2]);
            float e = 1.f / fp[0];
            if (e > 10000.f || isnan(e)) e = 10000.f;
            x->a = e;
            x = &bs->bx[bs->n++];
            x->kind = BX_SPEC_REFL_COND; x->type = BSDF_REFLECTION | BSDF_SPECULAR;
            x->eta = SPEC(c, mt->spec[1]);
            break;
        }
        case PBRTGPU_MAT_MIRROR: {
            if (!black[0]) {
                BxDF *x = &bs->bx[bs->n++];
                x->kind = BX_SPEC_REFL_NOOP; x->type = BSDF_REFLECTION | BSDF_SPECULAR; x->R = K[0];
            }
            break;
        }
        case PBRTGPU_MAT_GLASS: {   /* glass.cpp:34-57 */
            if (!black[0]) {
                BxDF *x = &bs->bx[bs->n++];
                x->kind = BX_SPEC_REFL_DIEL; x->type = BSDF_REFLECTION | BSDF_SPECULAR; x->R = K[0]; x->eta_t = fp[0];
            }
            if (!black[1]) {
                BxDF *x = &bs->bx[bs->n++];
                x->kind = BX_SPEC_TRANS; x->type = BSDF_TRANSMISSION | BSDF_SPECULAR; x->R = K[1]; x->eta_t = fp[0];
            }
            break;
        }
        case PBRTGPU_MAT_MEASURED: {   /* measured.cpp:182-206: one IrregIsotropicBRDF */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_MEASURED_IRREG; x->type = BSDF_REFLECTION | BSDF_GLOSSY;
            x->kd = c->s->kdnodes + mt->aux; x->nkd = mt->aux2;
            break;
        }
        case PBRTGPU_MAT_MEASURED_HALFANGLE: {   /* measured.cpp:196-198: RegularHalfangleBRDF, none without data */
            if (mt->aux < 0) break;
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_MEASURED_HALF; x->type = BSDF_REFLECTION | BSDF_GLOSSY;
            x->merl = c->s->merl + 3 * (size_t)mt->aux;
            break;
        }
        case PBRTGPU_MAT_ANISOWARD: {   /* anisoward.cpp:35-60: Lambertian(Kd) + AnisoWardBrdf(Ks, alphaU, alphaV) */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_LAMBERT; x->type = BSDF_REFLECTION | BSDF_DIFFUSE; x->R = K[0];
            x = &bs->bx[bs->n++];
            x->kind = BX_ANISOWARD; x->type = BSDF_REFLECTION | BSDF_GLOSSY; x->R = K[1];
            x->a = fp[0]; x->b = fp[1];
            break;
        }
        case PBRTGPU_MAT_SUBSTRATE: {   /* substrate.cpp:34-56 */
            BxDF *x = &bs->bx[bs->n++];
            x->kind = BX_FRESNEL_BLEND_ANISO; x->type = BSDF_REFLECTION | BSDF_GLOSSY;
            x->R = K[0]; x->R2 = K[1];
            float ex = 1.f / fp[0], ey = 1.f / fp[1];
            if (ex > 10000.f || isnan(ex)) ex = 10000.f;
            if (ey > 10000.f || isnan(ey)) ey = 10000.f;
            x->a = ex; x->b = ey;
            break;
        }
        default: break;
    }
}

/* ------------------------------------------------------------------ lights */
/* Sphere::Sample(p,u1,u2) (sphere.cpp:228-254) */
static V sphere_sample_p(const pbrtgpu_quadric *q, V p, float u1, float u2, V *ns) {
    V Pcenter = xpoint(q->o2w_m, v3(0, 0, 0));
    V wc = vnorm(vsub(Pcenter, p));
    V wcX, wcY;
    coordsys(wc, &wcX, &wcY);
    if (vlen2(vsub(p, Pcenter)) - q->radius * q->radius < 1e-4f) {
        V pp = vadd(v3(0, 0, 0), vmul(uniform_sphere(u1, u2), q->radius));
        *ns = vnorm(xnormal(q->o2w_minv, v3(pp.x, pp.y, pp.z)));
        if (q->reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q->o2w_m, pp);
    }
    float sinThetaMax2 = q->radius * q->radius / vlen2(vsub(p, Pcenter));
    float cosThetaMax = sqrtf(fmaxf_(0.f, 1.f - sinThetaMax2));
    /* UniformSampleCone(u1,u2,cosThetaMax,wcX,wcY,wc) (montecarlo.cpp:381-388) */
    float costheta = lerpf(u1, cosThetaMax, 1.f);
    float sintheta = sqrtf(1.f - costheta * costheta);
    float phi = u2 * 2.f * PI_F;
    V dir = vadd(vadd(vmul(wcX, COSF(phi) * sintheta), vmul(wcY, SINF(phi) * sintheta)), vmul(wc, costheta));
    Ray r; r.o = p; r.d = dir; r.mint = 1e-3f; r.maxt = INFINITY; r.time = 0.f;
    float thit, eps;
    DG dgs;
    if (!sphere_intersect(q, &r, &thit, &eps, &dgs)) thit = vdot(vsub(Pcenter, p), vnorm(r.d));
    V ps = rayat(&r, thit);
    *ns = vnorm(vsub(ps, Pcenter));
    if (q->reverse_orientation) *ns = vmul(*ns, -1.f);
    return ps;
}
/* Shape::Pdf(p, wi) (shape.cpp:78-91) */
static float shape_pdf_generic(const Ctx *c, int type, int idx, V p, V wi) {
    Ray ray; ray.o = p; ray.d = wi; ray.mint = 1e-3f; ray.maxt = INFINITY; ray.time = 0.f;
    float thit, eps;
    DG dg;
    if (!shape_intersect(c, type, idx, &ray, &thit, &eps, &dg)) return 0.;
    float pdf = vlen2(vsub(p, rayat(&ray, thit))) / (fabsf(vdot(dg.nn, vneg(wi))) * shape_area(c, type, idx));
    if (isinf(pdf)) pdf = 0.f;
    return pdf;
}
static float shape_pdf(const Ctx *c, int type, int idx, V p, V wi) {
    if (type == PBRTGPU_SHAPE_SPHERE) {   /* sphere.cpp:256-266 */
        const pbrtgpu_quadric *q = &c->s->quadrics[idx];
        V Pcenter = xpoint(q->o2w_m, v3(0, 0, 0));
        if (vlen2(vsub(p, Pcenter)) - q->radius * q->radius < 1e-4f) return shape_pdf_generic(c, type, idx, p, wi);
        float sinThetaMax2 = q->radius * q->radius / vlen2(vsub(p, Pcenter));
        float cosThetaMax = sqrtf(fmaxf_(0.f, 1.f - sinThetaMax2));
        return 1.f / (2.f * PI_F * (1.f - cosThetaMax));
    }
    return shape_pdf_generic(c, type, idx, p, wi);
}
/* Shape::Sample(p, u1, u2) for triangle / disk = Sample(u1, u2) */
static V shape_sample_p(const Ctx *c, int type, int idx, V p, float u1, float u2, V *ns) {
    if (type == PBRTGPU_SHAPE_SPHERE) return sphere_sample_p(&c->s->quadrics[idx], p, u1, u2, ns);
    if (type == PBRTGPU_SHAPE_CYLINDER) {   /* cylinder.cpp:195-203 */
        const pbrtgpu_quadric *q = &c->s->quadrics[idx];
        float z = lerpf(u1, q->zmin, q->zmax), t = u2 * q->phi_max;
        V pp = v3(q->radius * COSF(t), q->radius * SINF(t), z);
        *ns = vnorm(xnormal(q->o2w_minv, v3(pp.x, pp.y, 0.f)));
        if (q->reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q->o2w_m, pp);
    }
    if (type == PBRTGPU_SHAPE_DISK) {   /* disk.cpp:140-150 */
        const pbrtgpu_quadric *q = &c->s->quadrics[idx];
        V pp;
        concentric_disk(u1, u2, &pp.x, &pp.y);
        pp.x *= q->radius; pp.y *= q->radius; pp.z = q->height;
        *ns = vnorm(xnormal(q->o2w_minv, v3(0, 0, 1)));
        if (q->reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q->o2w_m, pp);
    }
    /* Triangle::Sample (trianglemesh.cpp:436-448) */
    const pbrtgpu_triangle *t = &c->s->tris[idx];
    const pbrtgpu_mesh *m = &c->s->meshes[t->mesh];
    float su1 = sqrtf(u1);
    float b1 = 1.f - su1, b2 = u2 * su1;
    V p1 = vert(c, t->v[0]), p2 = vert(c, t->v[1]), p3 = vert(c, t->v[2]);
    V pp = vadd(vadd(vmul(p1, b1), vmul(p2, b2)), vmul(p3, (1.f - b1 - b2)));
    V n = vcross(vsub(p2, p1), vsub(p3, p1));
    *ns = vnorm(n);
    if (m->reverse_orientation) *ns = vmul(*ns, -1.f);
    return pp;
}
/* Distribution1D::SampleDiscrete (montecarlo.h:83-91) over cdf[1..n] (cdf[0] = 0) */
static int sample_discrete(const pbrtgpu_light_shape *ls, int n, float u) {
    /* upper_bound(cdf, cdf+n+1, u) with cdf[0]=0 */
    int lo = 0, count = n + 1;
    while (count > 0) {
        int step = count / 2, it = lo + step;
        float cv = it == 0 ? 0.f : ls[it - 1].cdf;
        if (!(u < cv)) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    int off = lo - 1;
    return off < 0 ? 0 : off;
}
typedef struct { V o, d; float mint, maxt; } Seg;
/* InfiniteAreaLight (lights/infinite.cpp): a one-texel radiance map, or a decoded image's MIPMap
   (map_tex) with its Distribution2D (in the texel pool from dist_off) */
static inline float spherical_theta(V v) { return ACOSF(clampf(v.z, -1.f, 1.f)); }   /* geometry.h:642-650 */
static inline float spherical_phi(V v) { float p = ATAN2F(v.y, v.x); return (p < 0.f) ? p + 2.f * PI_F : p; }
static void inf_radiance(const Ctx *c, const pbrtgpu_light *L, float s, float t, float *out) {
    float rgb[3];
    if (L->map_tex >= 0) mip_lookup_w(c, &c->s->textures[L->map_tex], 3, s, t, 0.f, rgb);   /* MIPMap::Lookup(s, t) */
    else mip_triangle(L->texel, 3, L->wrap, s, t, rgb);   /* MIPMap::Lookup(s, t), width 0 */
    from_rgb(c, rgb, 1, out);                          /* Spectrum(rgb, SPECTRUM_ILLUMINANT) */
}
/* Distribution1D::SampleContinuous (montecarlo.h:68-84) of {funcInt, func[n], cdf[n + 1]} */
static float dist1d_sample(const float *D, int n, float u, float *pdf, int *off) {
    const float *cdf = D + 1 + n;
    int lo = 0, count = n + 1;   /* std::upper_bound(cdf, cdf + n + 1, u) */
    while (count > 0) {
        int step = count / 2, it = lo + step;
        if (!(u < cdf[it])) { lo = it + 1; count -= step + 1; }
        else count = step;
    }
    int offset = lo - 1 > 0 ? lo - 1 : 0;
    *off = offset;
    float du = (u - cdf[offset]) / (cdf[offset + 1] - cdf[offset]);
    *pdf = D[1 + offset] / D[0];
    return (offset + du) / n;
}
/* Distribution2D::SampleContinuous / Pdf (montecarlo.h:137-152) */
static void dist2d_sample(const Ctx *c, const pbrtgpu_light *L, float u0, float u1, float uv[2], float *pdf) {
    const int nu = L->dist_nu, nv = L->dist_nv;
    const float *M = c->s->texels + L->dist_off;
    float pdfs[2];
    int v, o;
    uv[1] = dist1d_sample(M, nv, u1, &pdfs[1], &v);
    uv[0] = dist1d_sample(M + (2 + 2 * nv) + (size_t)v * (2 + 2 * nu), nu, u0, &pdfs[0], &o);
    *pdf = pdfs[0] * pdfs[1];
}
static float dist2d_pdf(const Ctx *c, const pbrtgpu_light *L, float u, float v) {
    const int nu = L->dist_nu, nv = L->dist_nv;
    const float *M = c->s->texels + L->dist_off;
    int iu = (int)(u * nu), iv = (int)(v * nv);   /* Clamp(Float2Int(.), 0, count - 1) */
    iu = iu < 0 ? 0 : (iu > nu - 1 ? nu - 1 : iu);
    iv = iv < 0 ? 0 : (iv > nv - 1 ? nv - 1 : iv);
    const float *R = M + (2 + 2 * nv) + (size_t)iv * (2 + 2 * nu);
    if (R[0] * M[0] == 0.f) return 0.f;
    return (R[1 + iu] * M[1 + iv]) / (R[0] * M[0]);
}
/* InfiniteAreaLight::Le (infinite.cpp:84-89) */
static void inf_Le(const Ctx *c, const pbrtgpu_light *L, V d, float *out) {
    V wh = vnorm(xvec(L->l2w_minv, d));
    inf_radiance(c, L, spherical_phi(wh) * INV_TWOPI_F, spherical_theta(wh) * INV_PI_F, out);
}
/* InfiniteAreaLight::Pdf (infinite.cpp:188-197); Distribution2D::Pdf of one texel is dist_pdf */
static float inf_pdf(const Ctx *c, const pbrtgpu_light *L, V w) {
    V wi = xvec(L->l2w_minv, w);
    float theta = spherical_theta(wi);
    float sintheta = SINF(theta);
    if (sintheta == 0.f) return 0.f;
    float dp = L->map_tex >= 0 ? dist2d_pdf(c, L, spherical_phi(wi) * INV_TWOPI_F, theta * INV_PI_F) : L->dist_pdf;
    return dp / (2.f * PI_F * PI_F * sintheta);
}
/* Light::Sample_L (diffuse.cpp:61-74, point.cpp:42-49, spot.cpp:41-48, distant.cpp:39-46,
 * infinite.cpp:155-185); returns Li into Li[] */
static void light_sample_L(const Ctx *c, const pbrtgpu_light *L, V p, float pEps, const float u[3], float time,
                           V *wi, float *pdf, Seg *vis, float *Li) {
    int nb = c->nb;
    const float *Ls = SPEC(c, L->spec);
    (void)time;
    if (L->type == PBRTGPU_LIGHT_INFINITE) {
        /* Distribution2D::SampleContinuous; of one texel it returns (u0, u1) with pdf map_pdf */
        float uv0 = u[0], uv1 = u[1], mapPdf = L->map_pdf;
        if (L->map_tex >= 0) {
            float uv[2];
            dist2d_sample(c, L, u[0], u[1], uv, &mapPdf);
            uv0 = uv[0]; uv1 = uv[1];
        }
        if (mapPdf == 0.f) { *pdf = 0.f; for (int i = 0; i < nb; ++i) Li[i] = 0.f; return; }
        float theta = uv1 * PI_F, phi = uv0 * 2.f * PI_F;
        float costheta = COSF(theta), sintheta = SINF(theta);
        float sinphi = SINF(phi), cosphi = COSF(phi);
        *wi = xvec(L->l2w_m, v3(sintheta * cosphi, sintheta * sinphi, costheta));
        *pdf = mapPdf / (2.f * PI_F * PI_F * sintheta);
        if (sintheta == 0.f) *pdf = 0.f;
        vis->o = p; vis->d = *wi; vis->mint = pEps; vis->maxt = INFINITY;   /* VisibilityTester::SetRay */
        inf_radiance(c, L, uv0, uv1, Li);
        return;
    }
    if (L->type == PBRTGPU_LIGHT_POINT) {
        V lp = v3(L->pos[0], L->pos[1], L->pos[2]);
        *wi = vnorm(vsub(lp, p));
        *pdf = 1.f;
        float dist = vlen(vsub(p, lp));
        vis->o = p; vis->d = vdiv(vsub(lp, p), dist); vis->mint = pEps; vis->maxt = dist * (1.f - 0.f);
        float d2 = vlen2(vsub(lp, p));
        for (int i = 0; i < nb; ++i) Li[i] = Ls[i] / d2;
        return;
    }
    if (L->type == PBRTGPU_LIGHT_SPOT) {   /* spot.cpp:41-48: Intensity * Falloff(-wi) / DistanceSquared */
        V lp = v3(L->pos[0], L->pos[1], L->pos[2]);
        *wi = vnorm(vsub(lp, p));
        *pdf = 1.f;
        float dist = vlen(vsub(p, lp));
        vis->o = p; vis->d = vdiv(vsub(lp, p), dist); vis->mint = pEps; vis->maxt = dist * (1.f - 0.f);
        /* Falloff (spot.cpp:51-60): wl = Normalize(WorldToLight(w)) */
        V wl = vnorm(xvec(L->l2w_minv, vneg(*wi)));
        float fo;
        if (wl.z < L->texel[0]) fo = 0.f;
        else if (wl.z > L->texel[1]) fo = 1.f;
        else {
            float delta = (wl.z - L->texel[0]) / (L->texel[1] - L->texel[0]);
            fo = delta * delta * delta * delta;
        }
        float d2 = vlen2(vsub(lp, p));
        for (int i = 0; i < nb; ++i) Li[i] = (Ls[i] * fo) / d2;
        return;
    }
    if (L->type == PBRTGPU_LIGHT_DISTANT) {   /* distant.cpp:39-46: L, toward lightDir */
        *wi = v3(L->pos[0], L->pos[1], L->pos[2]);
        *pdf = 1.f;
        vis->o = p; vis->d = *wi; vis->mint = pEps; vis->maxt = INFINITY;   /* VisibilityTester::SetRay */
        for (int i = 0; i < nb; ++i) Li[i] = Ls[i];
        return;
    }
    /* area: ShapeSet::Sample(p, ls, &ns) (light.cpp:137-151) */
    const pbrtgpu_light_shape *shs = c->s->light_shapes + L->shape_offset;
    int sn = sample_discrete(shs, L->n_shapes, u[2]);
    V ns;
    V pt = shape_sample_p(c, shs[sn].shape_type, shs[sn].shape_index, p, u[0], u[1], &ns);
    Ray r; r.o = p; r.d = vsub(pt, p); r.mint = 1e-3f; r.maxt = INFINITY; r.time = 0.f;
    float rayEps, thit = 1.f;
    int anyHit = 0;
    DG dg;
    for (int i = 0; i < L->n_shapes; ++i) {
        float th, e;
        DG d2;
        if (shape_intersect(c, shs[i].shape_type, shs[i].shape_index, &r, &th, &e, &d2)) { anyHit = 1; thit = th; rayEps = e; dg = d2; }
    }
    (void)rayEps;
    if (anyHit) ns = dg.nn;
    V ps = rayat(&r, thit);
    *wi = vnorm(vsub(ps, p));
    /* ShapeSet::Pdf(p, wi) (light.cpp:159-165) */
    float pp = 0.f;
    for (int i = 0; i < L->n_shapes; ++i) pp += shs[i].area * shape_pdf(c, shs[i].shape_type, shs[i].shape_index, p, *wi);
    *pdf = pp / L->sum_area;
    /* VisibilityTester::SetSegment(p, pEps, ps, 1e-3f) */
    float dist = vlen(vsub(p, ps));
    vis->o = p; vis->d = vdiv(vsub(ps, p), dist); vis->mint = pEps; vis->maxt = dist * (1.f - 1e-3f);
    /* DiffuseAreaLight::L(ps, ns, -wi) */
    if (vdot(ns, vneg(*wi)) > 0.f) for (int i = 0; i < nb; ++i) Li[i] = Ls[i];
    else for (int i = 0; i < nb; ++i) Li[i] = 0.f;
}
static float light_pdf(const Ctx *c, const pbrtgpu_light *L, V p, V wi) {
    if (L->type == PBRTGPU_LIGHT_POINT || L->type == PBRTGPU_LIGHT_SPOT || L->type == PBRTGPU_LIGHT_DISTANT) return 0.;
    if (L->type == PBRTGPU_LIGHT_INFINITE) return inf_pdf(c, L, wi);
    const pbrtgpu_light_shape *shs = c->s->light_shapes + L->shape_offset;
    float pp = 0.f;
    for (int i = 0; i < L->n_shapes; ++i) pp += shs[i].area * shape_pdf(c, shs[i].shape_type, shs[i].shape_index, p, wi);
    return pp / L->sum_area;
}
static inline int light_is_delta(const pbrtgpu_light *L) {   /* Light::IsDeltaLight: point, spot, distant */
    return L->type == PBRTGPU_LIGHT_POINT || L->type == PBRTGPU_LIGHT_SPOT || L->type == PBRTGPU_LIGHT_DISTANT;
}
/* AreaLight::L via Intersection::Le (intersection.cpp:53-57, diffuse.h:43-45) */
static void isect_Le(const Ctx *c, const Isect *is, V w, float *out) {
    int al = c->s->prims[is->prim].area_light;
    if (al < 0) { for (int i = 0; i < c->nb; ++i) out[i] = 0.f; return; }
    const pbrtgpu_light *L = &c->s->lights[al];
    const float *Ls = SPEC(c, L->spec);
    if (vdot(is->dg.nn, w) > 0.f) for (int i = 0; i < c->nb; ++i) out[i] = Ls[i];
    else for (int i = 0; i < c->nb; ++i) out[i] = 0.f;
}

/* ------------------------------------------------------------------ integrator */
typedef struct {
    uint32_t hp, s, spp;
    RNG rng;
} PathSampler;
/* EstimateDirect (integrator.cpp:109-166) */
static void estimate_direct(const Ctx *c, int lightNum, V p, V n, V wo, float rayEps, float time, const BSDF *bs,
                            const float ul[3], const float ub[3], float *Ld) {
    int nb = c->nb;
    const pbrtgpu_light *L = &c->s->lights[lightNum];
    int flags = BSDF_ALL & ~BSDF_SPECULAR;
    float Li[MAXB], f[MAXB];
    for (int i = 0; i < nb; ++i) Ld[i] = 0.f;
    V wi;
    float lightPdf, bsdfPdf;
    Seg vis;
    light_sample_L(c, L, p, rayEps, ul, time, &wi, &lightPdf, &vis, Li);
    if (lightPdf > 0. && !spec_black(c, Li)) {
        bsdf_f(c, bs, wo, wi, flags, f);
        Ray sr; sr.o = vis.o; sr.d = vis.d; sr.mint = vis.mint; sr.maxt = vis.maxt; sr.time = time;
        if (!spec_black(c, f) && !bvh_intersectP(c, &sr)) {
            if (light_is_delta(L)) {
                float s = fabsf(vdot(wi, n)) / lightPdf;
                for (int i = 0; i < nb; ++i) Ld[i] += (f[i] * Li[i]) * s;
            } else {
                bsdfPdf = bsdf_pdf(bs, wo, wi, flags);
                float weight = power_heuristic(1, lightPdf, 1, bsdfPdf);
                float s = fabsf(vdot(wi, n)) * weight / lightPdf;
                for (int i = 0; i < nb; ++i) Ld[i] += (f[i] * Li[i]) * s;
            }
        }
    }
    if (!light_is_delta(L)) {
        int sampledType;
        bsdf_sample_f(c, bs, wo, &wi, ub[0], ub[1], ub[2], &bsdfPdf, flags, &sampledType, f);
        if (!spec_black(c, f) && bsdfPdf > 0.) {
            float weight = 1.f;
            if (!(sampledType & BSDF_SPECULAR)) {
                lightPdf = light_pdf(c, L, p, wi);
                if (lightPdf == 0.) return;
                weight = power_heuristic(1, bsdfPdf, 1, lightPdf);
            }
            Ray ray; ray.o = p; ray.d = wi; ray.mint = rayEps; ray.maxt = INFINITY; ray.time = time;
            Hit h;
            for (int i = 0; i < nb; ++i) Li[i] = 0.f;
            if (bvh_intersect(c, &ray, &h)) {
                if (L->type == PBRTGPU_LIGHT_AREA && c->s->prims[h.prim].area_light == lightNum) {
                    Isect is;
                    isect_fill(c, &ray, &h, &is);
                    isect_Le(c, &is, vneg(wi), Li);
                }
            } else if (L->type == PBRTGPU_LIGHT_INFINITE)
                inf_Le(c, L, ray.d, Li);   /* Li = light->Le(ray) (0 for area lights) */
            if (!spec_black(c, Li)) {
                float ad = fabsf(vdot(wi, n));
                for (int i = 0; i < nb; ++i) Ld[i] += (((f[i] * Li[i]) * ad) * weight) / bsdfPdf;
            }
        }
    }
}
/* PathIntegrator::Li (path.cpp:44-115) + SamplerRenderer::Li (samplerrenderer.cpp:225-247) */
static void radiance(const Ctx *c, Ray ray, const RayDiff *rd, PathSampler *ps, float *Lout) {
    int nb = c->nb;
    float L[MAXB], beta[MAXB], tmp[MAXB], Ld[MAXB], f[MAXB];
    for (int i = 0; i < nb; ++i) { L[i] = 0.f; beta[i] = 1.f; }
    Hit h;
    Isect is;
    if (!bvh_intersect(c, &ray, &h)) {
        /* miss: Li = sum of the lights' Le (area/point: 0) */
        for (int k = 0; k < c->s->n_lights; ++k)
            if (c->s->lights[k].type == PBRTGPU_LIGHT_INFINITE) {
                inf_Le(c, &c->s->lights[k], ray.d, tmp);
                for (int i = 0; i < nb; ++i) L[i] += tmp[i];
            }
        for (int i = 0; i < nb; ++i) Lout[i] = (1.f * L[i]) + 0.f;
        return;
    }
    isect_fill(c, &ray, &h, &is);
    int specularBounce = 0;
    int nLights = c->s->n_lights;
    for (int bounces = 0;; ++bounces) {
        if (bounces == 0 || specularBounce) {
            isect_Le(c, &is, vneg(ray.d), tmp);
            for (int i = 0; i < nb; ++i) L[i] += beta[i] * tmp[i];
        }
        BSDF bs;
        DG dgs;
        float diff[10];   /* only the camera ray carries differentials (path.cpp:107) */
        compute_differentials(&is.dg, bounces == 0 ? rd : NULL, diff);
        get_bsdf(c, &is, diff, &bs, &dgs);
        V p = dgs.p, n = dgs.nn;
        V wo = vneg(ray.d);
        /* UniformSampleOneLight (integrator.cpp:74-106) */
        if (nLights > 0) {
            float ul[3], ub[3], ulnum;
            if (bounces < 3) {
                float u2[2];
                ulnum = s1d(ps->hp, DIM_1D(4 * bounces + 1), ps->s, ps->spp);
                s2d(ps->hp, DIM_2D(3 * bounces + 0), ps->s, ps->spp, u2); ul[0] = u2[0]; ul[1] = u2[1];
                ul[2] = s1d(ps->hp, DIM_1D(4 * bounces + 0), ps->s, ps->spp);
                s2d(ps->hp, DIM_2D(3 * bounces + 1), ps->s, ps->spp, u2); ub[0] = u2[0]; ub[1] = u2[1];
                ub[2] = s1d(ps->hp, DIM_1D(4 * bounces + 2), ps->s, ps->spp);
            } else {
                ulnum = rng_float(&ps->rng);
                ul[0] = rng_float(&ps->rng); ul[1] = rng_float(&ps->rng); ul[2] = rng_float(&ps->rng);
                ub[0] = rng_float(&ps->rng); ub[1] = rng_float(&ps->rng); ub[2] = rng_float(&ps->rng);
            }
            int lightNum = (int)floorf(ulnum * nLights);
            if (lightNum > nLights - 1) lightNum = nLights - 1;
            estimate_direct(c, lightNum, p, n, wo, is.rayEps, ray.time, &bs, ul, ub, Ld);
            for (int i = 0; i < nb; ++i) L[i] += beta[i] * ((float)nLights * Ld[i]);
        } else {
            for (int i = 0; i < nb; ++i) L[i] += beta[i] * 0.f;
        }
        /* BSDF sample for the path direction */
        float up[3];
        if (bounces < 3) {
            float u2[2];
            s2d(ps->hp, DIM_2D(3 * bounces + 2), ps->s, ps->spp, u2); up[0] = u2[0]; up[1] = u2[1];
            up[2] = s1d(ps->hp, DIM_1D(4 * bounces + 3), ps->s, ps->spp);
        } else {
            up[0] = rng_float(&ps->rng); up[1] = rng_float(&ps->rng); up[2] = rng_float(&ps->rng);
        }
        V wi;
        float pdf;
        int flags;
        bsdf_sample_f(c, &bs, wo, &wi, up[0], up[1], up[2], &pdf, BSDF_ALL, &flags, f);
        if (spec_black(c, f) || pdf == 0.) break;
        specularBounce = (flags & BSDF_SPECULAR) != 0;
        float ad = fabsf(vdot(wi, n));
        for (int i = 0; i < nb; ++i) beta[i] *= (f[i] * ad) / pdf;
        Ray nray; nray.o = p; nray.d = wi; nray.mint = is.rayEps; nray.maxt = INFINITY; nray.time = ray.time;
        ray = nray;
        if (bounces > 3) {
            float cp = fminf_(.5f, spec_y(c, beta));
            if (rng_float(&ps->rng) > cp) break;
            for (int i = 0; i < nb; ++i) beta[i] /= cp;
        }
        if (bounces == c->s->max_depth) break;
        if (!bvh_intersect(c, &ray, &h)) {
            if (specularBounce)
                for (int k = 0; k < nLights; ++k) {
                    if (c->s->lights[k].type == PBRTGPU_LIGHT_INFINITE) inf_Le(c, &c->s->lights[k], ray.d, tmp);
                    else for (int i = 0; i < nb; ++i) tmp[i] = 0.f;   /* area/point Le == 0 */
                    for (int i = 0; i < nb; ++i) L[i] += beta[i] * tmp[i];
                }
            break;
        }
        isect_fill(c, &ray, &h, &is);
        /* pathThroughput *= Transmittance (== 1) */
        for (int i = 0; i < nb; ++i) beta[i] *= 1.f;
    }
    for (int i = 0; i < nb; ++i) Lout[i] = (1.f * L[i]) + 0.f;   /* T * Li + Lvi */
}

/* ------------------------------------------------------------------ DirectLightingIntegrator */
/* Sample layout of DirectLightingIntegrator::RequestSamples (directlighting.cpp:46-70) + the
 * emission integrator's 2 x 1D: strategy "all": per light i 1D [lightComp 2i, bsdfComp 2i+1],
 * 2D [lightPos 2i, bsdfDir 2i+1], each with RoundUpPow2(nSamples) values; "one": 1D
 * [lightComp 0, lightNum 1, bsdfComp 2], 2D [lightPos 0, bsdfDir 1].  Value k of a slot of
 * count n is sample index s * n + k of a sequence of length spp * n. */
static uint32_t pow2_up(uint32_t v) { v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; return v + 1; }
static int dl_n1d(const Ctx *c) { return c->s->dl_strategy == PBRTGPU_DL_ONE ? 5 : 2 * c->s->n_lights + 2; }
static int dl_count(const Ctx *c, int i) { int n = c->s->lights[i].n_samples; return (int)pow2_up((uint32_t)(n > 1 ? n : 1)); }
static void dl_light_sample(const Ctx *c, const PathSampler *ps, int i, int j, float ul[3], float ub[3], float *ulnum) {
    uint32_t n1 = (uint32_t)dl_n1d(c), u2i[2];
    float u2[2];
    (void)u2i;
    if (c->s->dl_strategy == PBRTGPU_DL_ONE) {
        *ulnum = s1d(ps->hp, 3u + 1u, ps->s, ps->spp);
        s2d(ps->hp, 3u + n1 + 0u, ps->s, ps->spp, u2); ul[0] = u2[0]; ul[1] = u2[1];
        ul[2] = s1d(ps->hp, 3u + 0u, ps->s, ps->spp);
        s2d(ps->hp, 3u + n1 + 1u, ps->s, ps->spp, u2); ub[0] = u2[0]; ub[1] = u2[1];
        ub[2] = s1d(ps->hp, 3u + 2u, ps->s, ps->spp);
        return;
    }
    uint32_t n = (uint32_t)dl_count(c, i), k = ps->s * n + (uint32_t)j, len = ps->spp * n;
    s2d(ps->hp, 3u + n1 + 2u * i, k, len, u2); ul[0] = u2[0]; ul[1] = u2[1];
    ul[2] = s1d(ps->hp, 3u + 2u * i, k, len);
    s2d(ps->hp, 3u + n1 + 2u * i + 1u, k, len, u2); ub[0] = u2[0]; ub[1] = u2[1];
    ub[2] = s1d(ps->hp, 3u + 2u * i + 1u, k, len);
    *ulnum = 0.f;
}
/* DirectLightingIntegrator::Li (directlighting.cpp:73-109) for a ray of depth `depth`, via
 * SamplerRenderer::Li (samplerrenderer.cpp:225-247: miss -> sum of the lights' Le), with
 * SpecularReflect / SpecularTransmit (integrator.cpp:169-250) and their ray differentials */
static void dl_radiance(const Ctx *c, Ray ray, const RayDiff *rd, int depth, PathSampler *ps, float *Lout) {
    int nb = c->nb, nLights = c->s->n_lights;
    float L[MAXB], tmp[MAXB], Ld[MAXB], ed[MAXB], f[MAXB], Lc[MAXB];
    for (int i = 0; i < nb; ++i) L[i] = 0.f;
    Hit h;
    Isect is;
    if (!bvh_intersect(c, &ray, &h)) {
        for (int k = 0; k < nLights; ++k)
            if (c->s->lights[k].type == PBRTGPU_LIGHT_INFINITE) {
                inf_Le(c, &c->s->lights[k], ray.d, tmp);
                for (int i = 0; i < nb; ++i) L[i] += tmp[i];
            }
        for (int i = 0; i < nb; ++i) Lout[i] = (1.f * L[i]) + 0.f;
        return;
    }
    isect_fill(c, &ray, &h, &is);
    float diff[10];
    V dpdx, dpdy;
    compute_differentials2(&is.dg, rd, diff, &dpdx, &dpdy);
    diff[4] = dpdx.x; diff[5] = dpdx.y; diff[6] = dpdx.z; diff[7] = dpdy.x; diff[8] = dpdy.y; diff[9] = dpdy.z;
    BSDF bs;
    DG dgs;
    get_bsdf(c, &is, diff, &bs, &dgs);
    V wo = vneg(ray.d), p = dgs.p, n = dgs.nn;
    isect_Le(c, &is, wo, tmp);
    for (int i = 0; i < nb; ++i) L[i] += tmp[i];
    if (nLights > 0) {
        float ul[3], ub[3], ulnum;
        if (c->s->dl_strategy == PBRTGPU_DL_ONE) {   /* UniformSampleOneLight (integrator.cpp:74-106) */
            dl_light_sample(c, ps, 0, 0, ul, ub, &ulnum);
            int lightNum = (int)floorf(ulnum * nLights);
            if (lightNum > nLights - 1) lightNum = nLights - 1;
            estimate_direct(c, lightNum, p, n, wo, is.rayEps, ray.time, &bs, ul, ub, ed);
            for (int i = 0; i < nb; ++i) L[i] += ed[i] * (float)nLights;
        } else {                                       /* UniformSampleAllLights (integrator.cpp:39-71) */
            float La[MAXB];                            /* its own sum, added to L once */
            for (int i = 0; i < nb; ++i) La[i] = 0.f;
            for (int li = 0; li < nLights; ++li) {
                int ns = dl_count(c, li);
                for (int i = 0; i < nb; ++i) Ld[i] = 0.f;
                for (int j = 0; j < ns; ++j) {
                    dl_light_sample(c, ps, li, j, ul, ub, &ulnum);
                    estimate_direct(c, li, p, n, wo, is.rayEps, ray.time, &bs, ul, ub, ed);
                    for (int i = 0; i < nb; ++i) Ld[i] += ed[i];
                }
                for (int i = 0; i < nb; ++i) La[i] += Ld[i] / (float)ns;
            }
            for (int i = 0; i < nb; ++i) L[i] += La[i];
        }
    }
    if (depth + 1 < c->s->max_depth) {
        float bsdfEta = bs.eta;   /* BSDF::eta (glass.cpp:47-48) */
        for (int pass = 0; pass < 2; ++pass) {   /* SpecularReflect, then SpecularTransmit */
            float u0 = rng_float(&ps->rng), u1 = rng_float(&ps->rng), uc = rng_float(&ps->rng);   /* BSDFSample(rng) */
            int flags = BSDF_SPECULAR | (pass ? BSDF_TRANSMISSION : BSDF_REFLECTION), st;
            V wi;
            float pdf;
            bsdf_sample_f(c, &bs, wo, &wi, u0, u1, uc, &pdf, flags, &st, f);
            float ad = fabsf(vdot(wi, n));
            if (!(pdf > 0.f) || spec_black(c, f) || ad == 0.f) continue;
            Ray cr; cr.o = p; cr.d = wi; cr.mint = is.rayEps; cr.maxt = INFINITY; cr.time = ray.time;
            RayDiff crd;
            crd.has = 0;
            if (rd && rd->has) {
                crd.has = 1;
                crd.rxo = vadd(p, dpdx);
                crd.ryo = vadd(p, dpdy);
                V dndx = vadd(vmul(dgs.dndu, diff[0]), vmul(dgs.dndv, diff[1]));
                V dndy = vadd(vmul(dgs.dndu, diff[2]), vmul(dgs.dndv, diff[3]));
                V dwodx = vsub(vneg(rd->rxd), wo), dwody = vsub(vneg(rd->ryd), wo);
                float dDNdx = vdot(dwodx, n) + vdot(wo, dndx);
                float dDNdy = vdot(dwody, n) + vdot(wo, dndy);
                if (pass == 0) {
                    float won = vdot(wo, n);
                    crd.rxd = vadd(vsub(wi, dwodx), vmul(vadd(vmul(dndx, won), vmul(n, dDNdx)), 2.f));
                    crd.ryd = vadd(vsub(wi, dwody), vmul(vadd(vmul(dndy, won), vmul(n, dDNdy)), 2.f));
                } else {
                    float eta = bsdfEta;
                    V w = vneg(wo);
                    if (vdot(wo, n) < 0) eta = 1.f / eta;
                    float mu = eta * vdot(w, n) - vdot(wi, n);
                    float dmudx = (eta - (eta * eta * vdot(w, n)) / vdot(wi, n)) * dDNdx;
                    float dmudy = (eta - (eta * eta * vdot(w, n)) / vdot(wi, n)) * dDNdy;
                    crd.rxd = vsub(vadd(wi, vmul(dwodx, eta)), vadd(vmul(dndx, mu), vmul(n, dmudx)));
                    crd.ryd = vsub(vadd(wi, vmul(dwody, eta)), vadd(vmul(dndy, mu), vmul(n, dmudy)));
                }
            }
            dl_radiance(c, cr, &crd, depth + 1, ps, Lc);
            for (int i = 0; i < nb; ++i) L[i] += ((f[i] * Lc[i]) * ad) / pdf;
        }
    }
    for (int i = 0; i < nb; ++i) Lout[i] = (1.f * L[i]) + 0.f;
}

/* MetadataIntegrator::Li (metadata.cpp:41-80) via SamplerRenderer::Li (samplerrenderer.cpp:225-247):
 * first hit -> Spectrum(primitiveId), Spectrum(materialId) or Spectrum(|p - ray.o|); a miss ->
 * the lights' Le */
static void meta_radiance(const Ctx *c, Ray ray, float *Lout) {
    int nb = c->nb;
    float L[MAXB], tmp[MAXB];
    for (int i = 0; i < nb; ++i) L[i] = 0.f;
    Hit h;
    if (!bvh_intersect(c, &ray, &h)) {
        for (int k = 0; k < c->s->n_lights; ++k)
            if (c->s->lights[k].type == PBRTGPU_LIGHT_INFINITE) {
                inf_Le(c, &c->s->lights[k], ray.d, tmp);
                for (int i = 0; i < nb; ++i) L[i] += tmp[i];
            }
    } else {
        float v;
        if (c->s->meta_strategy == PBRTGPU_META_DEPTH) {
            Isect is;
            isect_fill(c, &ray, &h, &is);
            V d = vsub(is.dg.p, ray.o);
            v = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        } else {
            const uint32_t *m = c->s->prim_meta;
            v = m ? (float)m[2 * h.prim + (c->s->meta_strategy == PBRTGPU_META_MATERIAL)] : 0.f;
        }
        for (int i = 0; i < nb; ++i) L[i] = v;
    }
    for (int i = 0; i < nb; ++i) Lout[i] = (1.f * L[i]) + 0.f;
}

/* camera sample -> world ray (perspective.cpp:73-106, orthographic.cpp:42-102, transform.h:253-262) */
static Ray camera_ray(const Ctx *c, float imageX, float imageY, float lensU, float lensV, float timeU, RayDiff *rd) {
    const pbrtgpu_camera *cam = &c->s->camera;
    const float *m = cam->raster_to_camera;
    float x = imageX, y = imageY, z = 0;
    V Pc;
    Pc.x = m[0] * x + m[1] * y + m[2] * z + m[3];
    Pc.y = m[4] * x + m[5] * y + m[6] * z + m[7];
    Pc.z = m[8] * x + m[9] * y + m[10] * z + m[11];
    float w = m[12] * x + m[13] * y + m[14] * z + m[15];
    if (w != 1.) Pc = vdiv(Pc, w);
    Ray r;
    if (cam->ortho) {   /* orthographic.cpp:42-65: from Pcamera along +z */
        r.o = Pc;
        r.d = v3(0.f, 0.f, 1.f);
    } else {
        r.o = v3(0, 0, 0);
        r.d = vnorm(v3(Pc.x, Pc.y, Pc.z));
    }
    r.mint = 0.f; r.maxt = INFINITY;
    if (cam->lens_radius > 0.) {
        float lu, lv;
        concentric_disk(lensU, lensV, &lu, &lv);
        lu *= cam->lens_radius; lv *= cam->lens_radius;
        float ft = cam->focal_distance / r.d.z;
        V Pfocus = rayat(&r, ft);
        r.o = v3(lu, lv, 0.f);
        r.d = vnorm(vsub(Pfocus, r.o));
    }
    /* Sample::time = Lerp(u, open, close) (LDPixelSample, montecarlo.cpp:229), lerped again by the camera
     * (perspective.cpp:67, 102; realisticDiffraction.cpp:1157) */
    r.time = lerpf(lerpf(timeU, cam->shutter_open, cam->shutter_close), cam->shutter_open, cam->shutter_close);
    /* CameraToWorld at the ray's time: AnimatedTransform's start / end transform or
     * Interpolate (transform.cpp:356-381, 427-455) for an animated camera */
    float cwb[16];
    const float *cw = cam->cam2world_m;
    if (c->s->camera_motion) {
        inst_interp(c->s->camera_motion, r.time, cwb, NULL);
        cw = cwb;
    }
    Ray o = r;
    {
        V p = r.o;
        float xp = cw[0] * p.x + cw[1] * p.y + cw[2] * p.z + cw[3];
        float yp = cw[4] * p.x + cw[5] * p.y + cw[6] * p.z + cw[7];
        float zp = cw[8] * p.x + cw[9] * p.y + cw[10] * p.z + cw[11];
        float wp = cw[12] * p.x + cw[13] * p.y + cw[14] * p.z + cw[15];
        o.o = v3(xp, yp, zp);
        if (wp != 1.) o.o = vdiv(o.o, wp);
    }
    o.d = xvec(cw, r.d);
    if (rd) {   /* rx/ry rays in camera space, CameraToWorld, ScaleDifferentials(1/sqrt(spp)) */
        const float *dx = cam->dx_camera, *dy = cam->dy_camera;
        V rxd = vnorm(vadd(Pc, v3(dx[0], dx[1], dx[2]))), ryd = vnorm(vadd(Pc, v3(dy[0], dy[1], dy[2])));
        V owx = o.o, owy = o.o;   /* rxOrigin = ryOrigin = ray->o, transformed like o */
        if (cam->ortho) {   /* orthographic.cpp:95-98: o + dxCamera / dyCamera, direction d */
            owx = xpoint(cw, vadd(r.o, v3(dx[0], dx[1], dx[2])));
            owy = xpoint(cw, vadd(r.o, v3(dy[0], dy[1], dy[2])));
            rxd = ryd = r.d;
        }
        rxd = xvec(cw, rxd); ryd = xvec(cw, ryd);
        float sc = 1.f / sqrtf((float)c->s->spp);
        rd->rxo = vadd(o.o, vmul(vsub(owx, o.o), sc));
        rd->ryo = vadd(o.o, vmul(vsub(owy, o.o), sc));
        rd->rxd = vadd(o.d, vmul(vsub(rxd, o.d), sc));
        rd->ryd = vadd(o.d, vmul(vsub(ryd, o.d), sc));
        rd->has = 1;
    }
    return o;
}

/* ---- RealisticDiffractionCamera (cameras/realisticDiffraction.cpp).
 * PARITY UNPINNED: the camera's TU includes GSL headers this image lacks, so the reference
 * harness cannot run it; this restatement and the GPU's are checked against each other. */

/* Diffraction's Gaussian draws (realisticDiffraction.cpp:1091, gsl_ran_bivariate_gaussian over
 * one GSL generator shared by the render threads): here each camera sample has its own
 * counter-based stream, uniform number n = top 32 bits of
 * splitmix64(key + n * 0x9E3779B97F4A7C15) / 2^32, n = 1, 2, ... */
typedef struct { uint64_t key; uint32_t n; } DiffStream;
static double diff_next(DiffStream *st) {
    st->n += 1;
    uint64_t z = st->key + (uint64_t)st->n * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (double)(uint32_t)(z >> 32) / 4294967296.0;
}
/* GSL randist/bigauss.c, rho = 0: polar Box-Muller, at most 64 tries (then no noise) */
static void diff_bigauss(DiffStream *st, double sigma_x, double sigma_y, double *x, double *y) {
    int tries;
    *x = 0.0;
    *y = 0.0;
    for (tries = 0; tries < 64; ++tries) {
        double u = -1 + 2 * diff_next(st);
        double v = -1 + 2 * diff_next(st);
        double r2 = u * u + v * v;
        if (r2 > 1.0 || r2 == 0) continue;
        double scale = sqrt(-2.0 * DLOG(r2) / r2);
        *x = sigma_x * u * scale;
        *y = sigma_y * (0.0 * u + 1.0 * v) * scale;   /* rho u + sqrt(1 - rho^2) v */
        return;
    }
}
/* realisticDiffraction.cpp:1057-1150 after an element: p its intersection point, ap its aperture,
 * wl the ray's wavelength; the radius is measured from (cx, cy) -- the axis for the main lens, the
 * microlens centre for the microlens elements (:790-872).  C++'s float overloads (sqrt of a float
 * expression) are sqrtf here.  nan_out (main lens): a NaN direction returns 0 (the ray's weight is
 * 0); the microlens step normalises whatever it got (no check there). */
static int lens_diffraction(DiffStream *st, V p, float cx, float cy, float ap, float wl, V *dir_io, int nan_out) {
    double radius = sqrtf((p.x - cx) * (p.x - cx) + (p.y - cy) * (p.y - cy));
    V ea = v3(p.x, p.y, 0.f), eb = v3(-p.y, p.x, 0.f);
    double a = ap / 2 - radius;
    double b = sqrt(ap / 2 * ap / 2 - radius * radius);
    double pi = 3.14159265359;
    double lambda = wl * 1e-9;
    double sigma_x = DATAN(1 / (sqrt(2.0) * a * .001 * 2 * pi / lambda));
    double sigma_y = DATAN(1 / (sqrt(2.0) * b * .001 * 2 * pi / lambda));
    double gx, gy;
    diff_bigauss(st, sigma_x, sigma_y, &gx, &gy);
    ea = vnorm(ea);
    eb = vnorm(eb);
    float noiseA = (float)gx, noiseB = (float)gy;
    V d = *dir_io;
    double projA = (d.x * ea.x + d.y * ea.y) / sqrtf(ea.x * ea.x + ea.y * ea.y);
    double projB = (d.x * eb.x + d.y * eb.y) / sqrtf(eb.x * eb.x + eb.y * eb.y);
    double projC = d.z;
    double rA = sqrt(projA * projA + projC * projC);
    double rB = sqrt(projB * projB + projC * projC);
    double thetaA = DACOS(projA / rA) + noiseA;
    double thetaB = DACOS(projB / rB) + noiseB;   /* recomputed below without the noise */
    double newA = DCOS(thetaA) * rA;
    d.z = (float)(DSIN(thetaA) * rA);
    projC = d.z;
    rB = sqrt(projB * projB + projC * projC);
    thetaB = DACOS(projB / rB);
    double newB = DCOS(thetaB) * rB;
    d.z = (float)(DSIN(thetaB) * rB);
    d.x = (float)(ea.x * newA + eb.x * newB);
    d.y = (float)(ea.y * newA + eb.y * newB);
    if (nan_out && (isnan(d.x) || isnan(d.y) || isnan(d.z))) {
        *dir_io = v3(0.f, 0.f, 0.f);
        return 0;
    }
    *dir_io = vnorm(d);
    return 1;
}
/* IntersectLensEl (realisticDiffraction.cpp:412-468) */
static int lens_el_hit(const Ray *r, float radius, V dist, float *tHit, V *nrm) {
    float m[16] = {1.f, 0.f, 0.f, dist.x, 0.f, 1.f, 0.f, dist.y, 0.f, 0.f, 1.f, dist.z, 0.f, 0.f, 0.f, 1.f};
    V o = xpoint(m, r->o), d = xvec(m, r->d);
    if (radius < 0) radius = -radius;
    float A = d.x * d.x + d.y * d.y + d.z * d.z;
    float B = 2 * (d.x * o.x + d.y * o.y + d.z * o.z);
    float C = o.x * o.x + o.y * o.y + o.z * o.z - radius * radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return 0;
    if (t0 > r->maxt || t1 < r->mint) return 0;
    float th = t0;
    if (t0 < r->mint) {
        th = t1;
        if (th > r->maxt) return 0;
    }
    *tHit = th;
    *nrm = vnorm(v3(d.x * th + o.x, d.y * th + o.y, d.z * th + o.z));
    return 1;
}
/* Spectrum::GetValueAtWavelength (spectrum.h:384-405): the band interval of wl (int step), Lerp of
 * its two band values, 0 outside every interval (the front end refuses band wavelengths in the
 * last interval, which would read c[N]) */
static float value_at_wavelength(const float *c, int N, float wl) {
    const int l0 = N == 30 ? 400 : 395, l1 = N == 30 ? 700 : 715;
    const float step = (float)((l1 - l0) / N);
    for (int i = 0; i < N; ++i) {
        const float w0 = l0 + i * step, w1 = l0 + (i + 1) * step;
        if (wl >= w0 && wl < w1) return lerpf((wl - w0) / (w1 - w0), c[i], c[i + 1]);
    }
    return 0.f;
}
/* applySnellsLaw (realisticDiffraction.cpp:347-410): with IORforEyeEnabled and a wavelength, the
 * ocular medium is recognised by the lens file's n (vitreous 1.336, lens 1.42, aqueous 1.3374,
 * cornea 1.3771; |n1 - n| < .001 in double) and both indices come from the eye IOR spectra
 * (cornea, aqueous, lens, vitreous) at the wavelength; otherwise the chromatic model, in double
 * (-.04) */
static void lens_snell(const pbrtgpu_lens *Ls, int N, float n1, float n2, float lensRadius, V nrm, Ray *ray, float wl) {
    if (Ls->ior_eye && wl != 0) {
        const float *cornea = Ls->eye_ior, *aqueous = cornea + N, *lensI = cornea + 2 * N, *vitreous = cornea + 3 * N;
        if (fabs((double)n1 - 1.336) < 0.001) {
            n1 = value_at_wavelength(vitreous, N, wl);
            n2 = value_at_wavelength(lensI, N, wl);
        } else if (fabs((double)n1 - 1.42) < 0.001) {
            n1 = value_at_wavelength(lensI, N, wl);
            n2 = value_at_wavelength(aqueous, N, wl);
        } else if (fabs((double)n1 - 1.3374) < 0.001) {
            n1 = value_at_wavelength(aqueous, N, wl);
            n2 = value_at_wavelength(cornea, N, wl);
        } else if (fabs((double)n1 - 1.3771) < 0.001) {
            n1 = value_at_wavelength(cornea, N, wl);
            n2 = 1;
        }
    } else if (Ls->chromatic) {
        if (n1 != 1) n1 = (float)((double)(wl - 550) * -.04 / (300) + (double)n1);
        if (n2 != 1) n2 = (float)((double)(wl - 550) * -.04 / (300) + (double)n2);
    }
    V s1 = ray->d;
    if (lensRadius > 0) nrm = vneg(nrm);
    V cr = vcross(nrm, s1);
    float radicand = 1 - (n1 / n2) * (n1 / n2) * vdot(cr, cr);
    if (radicand < 0) { ray->d = v3(0.f, 0.f, 0.f); return; }
    V s2 = vsub(vmul(vcross(nrm, vcross(vmul(nrm, -1.f), s1)), n1 / n2), vmul(nrm, sqrtf(radicand)));
    ray->d = vnorm(s2);
}
/* GenerateRay (realisticDiffraction.cpp:478-1164): returns the weight (0: blocked) */
static float lens_ray(const Ctx *c, float imageX, float imageY, float lensU, float lensV, float timeU, float wl,
                      DiffStream *st, Ray *out) {
    const pbrtgpu_camera *cam = &c->s->camera;
    const pbrtgpu_lens *Ls = &c->s->lens;
    const float xr2 = (float)cam->xres / 2.f, yr2 = (float)cam->yres / 2.f;
    V sp;
    sp.x = (float)(-((double)(imageX - xr2) - .25) / (double)xr2);
    sp.y = (float)(((double)(imageY - yr2) - .25) / (double)yr2);
    sp.z = -Ls->film_distance;
    float aspect = (float)cam->xres / (float)cam->yres;
    float width = Ls->film_diag / sqrtf((1.f + 1.f / (aspect * aspect)));
    float height = width / aspect;
    sp.x = sp.x * width / 2.f + Ls->film_center[0];
    sp.y = sp.y * height / 2.f + Ls->film_center[1];
    if (Ls->curve_radius != 0) {
        float R = Ls->curve_radius, th = sp.x / R, ph = sp.y / R;
        sp.x = R * COSF(ph) * SINF(th);
        sp.z = R * COSF(ph) * COSF(th);
        sp.y = R * SINF(ph);
        float sc = (-Ls->film_distance - R);
        sp.z = sc + sp.z;
    }
    float lu, lv;
    concentric_disk(lensU, lensV, &lu, &lv);
    const int n = Ls->n_elements;
    const float *E = Ls->elements;
    float firstAp = E[4 * (n - 1) + 3] / 2, firstR = E[4 * (n - 1)];
    float zI = firstR == 0 ? 0.f : (-firstR - sqrtf(firstR * firstR - firstAp * firstAp));
    const float luNoScale = lu, lvNoScale = lv;
    float pitch = 0.f;   /* superpixelPitch */
    int xp = 0, yp = 0;  /* the pinhole under the film point */
    const int nW = Ls->num_pinholes_w, nH = Ls->num_pinholes_h, pinholes = nW > 0 && nH > 0;
    lu *= firstAp;
    lv *= firstAp;
    V pol = v3(lu, lv, zI);
    if (Ls->pinhole_exit[0] != -1 && Ls->pinhole_exit[1] != -1 && Ls->pinhole_exit[2] != -1)
        pol = v3(Ls->pinhole_exit[0], Ls->pinhole_exit[1], Ls->pinhole_exit[2]);
    else if (pinholes) {
        /* the pinhole array (:560-629): the superpixel under the film point, clamped */
        const int ppW = cam->xres / nW, ppH = cam->yres / nH;
        xp = (int)(((double)imageX - .25) / ppW);
        yp = (int)(((double)imageY - .25) / ppH);
        if (xp > nW - 1) xp = nW - 1;
        else if (xp < 0) xp = 0;
        if (yp > nH - 1) yp = nH - 1;
        else if (yp < 0) yp = 0;
        const float *ph = Ls->pinholes + 3 * ((size_t)xp * nH + yp);
        if (Ls->microlens) {
            /* the microlens's entrance square (:614-623) */
            pitch = width / nW;
            pol = v3(luNoScale * pitch / 2.f + ph[0], lvNoScale * pitch / 2.f + ph[1], ph[2]);
        } else pol = v3(ph[0], ph[1], ph[2]);
    }
    Ray r;
    r.o = sp;
    r.d = vnorm(vsub(pol, r.o));
    r.mint = 0.f; r.maxt = INFINITY; r.time = 0.f;
    if (Ls->microlens && pinholes) {
        /* two spherical microlens surfaces (:634-876): radius from the thick-lens focal length */
        const float *ph = Ls->pinholes + 3 * ((size_t)xp * nH + yp);
        const float ap = pitch;
        const float thick = (float).01;
        const float mFilmDist = Ls->film_distance + pol.z;
        const float mFocal = mFilmDist + thick / 2;
        const float mN = (float)1.67;
        const double nm1 = (double)(mN - 1);
        const float oneOverR = (float)((-2 * (mN - 1) + sqrt(4 * (nm1 * nm1) + 4 * (nm1 * nm1) * thick / (mN * mFocal))) /
                                       (2 * (nm1 * nm1) * thick / mN));
        float mRad = 1 / oneOverR;
        float mDist = -Ls->film_distance + mFilmDist;
        for (int k = 0; k < 2; ++k) {
            const float cx = ph[0], cy = ph[1];
            float tHit = 0.f;
            V nrm = v3(0.f, 0.f, 1.f), ip = v3(0.f, 0.f, 0.f);
            mRad = -mRad;
            r.o = sp;
            if (lens_el_hit(&r, mRad, v3(-cx, -cy, mRad - mDist), &tHit, &nrm)) {
                ip = v3(tHit * r.d.x + r.o.x, tHit * r.d.y + r.o.y, tHit * r.d.z + r.o.z);
                if ((ip.x - cx) * (ip.x - cx) + (ip.y - cy) * (ip.y - cy) >= (ap * ap) / (2 * 2)) return 0.f;
                float n1 = 1, n2 = 1;
                if (k == 0) {
                    n2 = mN;
                    mDist += thick;
                } else n1 = mN;
                lens_snell(Ls, c->nb, n1, n2, mRad, nrm, &r, wl);
                sp = ip;
            }
            if (Ls->diffraction) lens_diffraction(st, ip, cx, cy, ap, wl, &r.d, 0);
        }
    }
    float lensDist = 0.f;
    for (int i = n - 1; i >= 0; --i) {
        float rad = E[4 * i], ap = E[4 * i + 3];
        lensDist += E[4 * i + 1];
        r.o = sp;
        if (rad == 0) {
            float tA = (i == n - 1) ? Ls->film_distance / r.d.z : (lensDist - r.o.z) / (r.d.z);
            V ai = v3(r.o.x + r.d.x * tA, r.o.y + r.d.y * tA, r.o.z + r.d.z * tA);
            float dx = ai.x - Ls->aperture_offset[0], dy = ai.y - Ls->aperture_offset[1];
            if ((double)(dx * dx + dy * dy) > (double)(ap * ap) * .25) return 0.f;
            sp = ai;
            if (Ls->diffraction && !lens_diffraction(st, ai, 0.f, 0.f, ap, wl, &r.d, 1)) return 0.f;
        } else {
            float tHit = 0.f;
            V nrm = v3(0.f, 0.f, 1.f);
            if (!lens_el_hit(&r, rad, v3(0.f, 0.f, rad - lensDist), &tHit, &nrm)) return 0.f;
            V ip = v3(tHit * r.d.x + r.o.x, tHit * r.d.y + r.o.y, tHit * r.d.z + r.o.z);
            if (ip.x * ip.x + ip.y * ip.y >= ap * ap / 4.f) return 0.f;
            float n1 = E[4 * i + 2], n2 = 1;
            if (i - 1 >= 0) {
                n2 = E[4 * (i - 1) + 2];
                if (n2 == 0) n2 = E[4 * (i - 2) + 2];
            }
            lens_snell(Ls, c->nb, n1, n2, rad, nrm, &r, wl);
            sp = ip;
            if (Ls->diffraction && !lens_diffraction(st, ip, 0.f, 0.f, ap, wl, &r.d, 1)) return 0.f;
        }
    }
    r.o = sp;
    /* Sample::time = Lerp(u, open, close) (LDPixelSample, montecarlo.cpp:229), lerped again by the camera
     * (perspective.cpp:67, 102; realisticDiffraction.cpp:1157) */
    r.time = lerpf(lerpf(timeU, cam->shutter_open, cam->shutter_close), cam->shutter_open, cam->shutter_close);
    /* CameraToWorld(*ray, ray) at the ray's time (realisticDiffraction.cpp:1158): the static
     * matrix, or the animated camera's start / end transform or Interpolate */
    float cwb[16];
    const float *cw = cam->cam2world_m;
    if (c->s->camera_motion) {
        inst_interp(c->s->camera_motion, r.time, cwb, NULL);
        cw = cwb;
    }
    out->o = xpoint(cw, r.o);
    out->d = vnorm(xvec(cw, r.d));
    out->mint = r.mint; out->maxt = r.maxt; out->time = r.time;
    return 1.f;
}
/* Camera::GenerateRayDifferential (camera.cpp:52-81) + ScaleDifferentials(1 / sqrtf(spp)) */
static float lens_ray_diff(const Ctx *c, float imageX, float imageY, float lensU, float lensV, float timeU, float wl,
                           uint64_t dkey, Ray *ray, RayDiff *rd) {
    DiffStream st;
    st.key = dkey;
    st.n = 0;
    float wt = lens_ray(c, imageX, imageY, lensU, lensV, timeU, wl, &st, ray);
    Ray rx, ry;
    float sx = imageX + 1.f;
    float wtx = lens_ray(c, sx, imageY, lensU, lensV, timeU, wl, &st, &rx);
    sx = sx - 1.f;
    float wty = lens_ray(c, sx, imageY + 1.f, lensU, lensV, timeU, wl, &st, &ry);
    if (wtx == 0.f || wty == 0.f) return 0.f;
    float sc = 1.f / sqrtf((float)c->s->spp);
    rd->rxo = vadd(ray->o, vmul(vsub(rx.o, ray->o), sc));
    rd->ryo = vadd(ray->o, vmul(vsub(ry.o, ray->o), sc));
    rd->rxd = vadd(ray->d, vmul(vsub(rx.d, ray->d), sc));
    rd->ryd = vadd(ray->d, vmul(vsub(ry.d, ray->d), sc));
    rd->has = 1;
    return wt;
}

/* One camera path: sample -> ray -> rayWeight * Li (samplerrenderer.cpp:86-110), the path
 * drawing from RNG(path_seed(hp, rngIdx)); wl is the ray's wavelength (0 under the
 * SamplerRenderer, Ray() in geometry.h:317) */
static void camera_path(const Ctx *c, int px, int py, uint32_t s, uint32_t rngIdx, float wl, float *L, float *imgX,
                        float *imgY) {
    uint32_t spp = (uint32_t)c->s->spp;
    PathSampler ps;
    ps.hp = pixel_hash(c->s->seed, px, py);
    ps.s = s;
    ps.spp = spp;
    float u[2], lens[2];
    s2d(ps.hp, 0, s, spp, u);
    float imageX = px + u[0], imageY = py + u[1];
    s2d(ps.hp, 1, s, spp, lens);
    float timeU = s1d(ps.hp, 2, s, spp);
    rng_seed(&ps.rng, path_seed(ps.hp, rngIdx));
    ps.rng.mti = 624;   /* RNG ctor: Seed() leaves mti == N, first draw regenerates */
    RayDiff rd;
    Ray r;
    float Lr[MAXB];
    if (c->s->camera_type == PBRTGPU_CAMERA_REALISTIC &&
        lens_ray_diff(c, imageX, imageY, lens[0], lens[1], timeU, wl, ((uint64_t)ps.hp << 32) | rngIdx, &r, &rd) == 0.f) {
        for (int i = 0; i < c->nb; ++i) L[i] = 0.f;   /* rayWeight 0: L = 0, nothing traced */
        if (imgX) *imgX = imageX;
        if (imgY) *imgY = imageY;
        return;
    }
    if (c->s->camera_type != PBRTGPU_CAMERA_REALISTIC) r = camera_ray(c, imageX, imageY, lens[0], lens[1], timeU, &rd);
    if (c->s->integrator == PBRTGPU_INTEGRATOR_DIRECT) dl_radiance(c, r, &rd, 0, &ps, Lr);
    else if (c->s->integrator == PBRTGPU_INTEGRATOR_METADATA) meta_radiance(c, r, Lr);
    else radiance(c, r, &rd, &ps, Lr);
    for (int i = 0; i < c->nb; ++i) L[i] = 1.f * Lr[i];   /* rayWeight * Li */
    if (imgX) *imgX = imageX;
    if (imgY) *imgY = imageY;
}

/* SamplerRenderer: the path and the NaN / negative / infinite luminance guard
 * (samplerrenderer.cpp:111-128) */
static int sampler_sample(const Ctx *c, int px, int py, uint32_t s, float *L, float *imgX, float *imgY) {
    camera_path(c, px, py, s, s, 0.f, L, imgX, imgY);
    int nb = c->nb, bad = 0;
    int nan = 0;
    for (int i = 0; i < nb; ++i) if (isnan(L[i])) nan = 1;
    if (nan) bad = 1;
    else {
        float yv = spec_y(c, L);
        if (yv < -1e-5) bad = 1;
        else if (isinf(yv)) bad = 1;
    }
    if (bad) for (int i = 0; i < nb; ++i) L[i] = 0.f;
    return bad;
}

/* sampledLambdaStart / End (ints): 395 / 715 in the 32- and 60-band builds (spectrum.h:41-42),
 * 400 / 700 in the upstream 30-band one (spectrum.h.original:36-38) */
static inline int lambda_start(int N) { return N == 30 ? 400 : 395; }
static inline int lambda_end(int N) { return N == 30 ? 700 : 715; }

/* SpectralRenderer: one camera sample of SpectralRendererTask::Run (spectralrenderer.cpp:
 * 98-190).  sampledLambdaStart / End are ints, so deltaWave = float((end - start) / nWaveBands)
 * and GetValueAtWavelength's step float((end - start) / N).
 * singleDirection: band b = 0 .. nWaveBands-1 traces the sample's camera path with
 * RNG(path_seed(hp, s nWaveBands + b)); samplerDirection: band s % nWaveBands only, with
 * RNG(path_seed(hp, s)).  A band's radiance: NaN -> 0; the luminance guard on the sample's
 * spectrum as assigned so far (it starts at 0 per sample); its value at the band's
 * wavelength (spectrum.h:384-405, Lerp(t, c[i], c[i+1])) into indices
 * [dI b, min(dI (b+1), N-1)), dI = round(N / nWaveBands).  Returns the bands zeroed. */
static int spectral_sample(const Ctx *c, int px, int py, uint32_t s, float *L, float *imgX, float *imgY) {
    const int N = c->nb, nWB = c->s->wave_bands;
    const int single = c->s->spectral_sampling == PBRTGPU_SPECTRAL_SINGLE;
    const int mm = single ? nWB : 1;
    const int dI = (int)round(N / nWB), l0 = lambda_start(N), l1 = lambda_end(N);
    const float dW = (float)((l1 - l0) / nWB), step = (float)((l1 - l0) / N);
    int bad = 0;
    for (int i = 0; i < N; ++i) L[i] = 0.f;
    for (int sb = 0; sb < mm; ++sb) {
        const int b = single ? sb : (int)(s % (uint32_t)nWB);
        float Lr[MAXB];
        const float wl = l0 + dW * b + (dW / 2);
        camera_path(c, px, py, s, single ? s * (uint32_t)nWB + (uint32_t)b : s, wl, Lr, imgX, imgY);
        int nan = 0;
        for (int i = 0; i < N; ++i) if (isnan(Lr[i])) nan = 1;
        int zero = nan;
        if (!nan) {
            float yv = spec_y(c, L);
            if (yv < -1e-5) zero = 1;
            else if (isinf(yv)) zero = 1;
        }
        if (zero) { for (int i = 0; i < N; ++i) Lr[i] = 0.f; ++bad; }
        const int lo = dI * b, hi = (dI * (b + 1) < N - 1) ? dI * (b + 1) : N - 1;
        if (hi <= lo) continue;
        float v = 0.f;
        for (int i = 0; i < N; ++i) {
            const float w0 = l0 + i * step, w1 = l0 + (i + 1) * step;
            if (wl >= w0 && wl < w1) {
                if (i + 1 >= N) abort();   /* c[N]: rejected by oracle_spectral_ok */
                v = lerpf((wl - w0) / (w1 - w0), Lr[i], Lr[i + 1]);
                break;
            }
        }
        for (int k = lo; k < hi; ++k) L[k] = v;
    }
    return bad;
}

/* a SpectralRenderer band whose indices need c[N] reads past the spectrum: such scenes are
 * rejected (as by pbrtgpu_scene_upload) */
static int spectral_ok(const pbrtgpu_flat_scene *s) {
    if (s->renderer != PBRTGPU_RENDERER_SPECTRAL) return 1;
    const int N = s->n_bands, nWB = s->wave_bands;
    if (nWB < 1) return 0;
    const int dI = (int)round(N / nWB), l0 = lambda_start(N), l1 = lambda_end(N);
    const float dW = (float)((l1 - l0) / nWB), step = (float)((l1 - l0) / N);
    for (int b = 0; b < nWB; ++b) {
        const int lo = dI * b, hi = (dI * (b + 1) < N - 1) ? dI * (b + 1) : N - 1;
        if (hi <= lo) continue;
        const float wl = l0 + dW * b + (dW / 2);
        if (wl >= l0 + (N - 1) * step) return 0;
    }
    /* the eye IOR lookups read every traced band's interval (spectrum.h:397) */
    if (s->camera_type == PBRTGPU_CAMERA_REALISTIC && s->lens.ior_eye)
        for (int b = 0; b < nWB; ++b) {
            const float wl = l0 + dW * b + (dW / 2);
            if (wl >= l0 + (N - 1) * step) return 0;
        }
    return 1;
}

static int trace_path(const Ctx *c, int px, int py, uint32_t s, float *L, float *imgX, float *imgY) {
    if (c->s->renderer == PBRTGPU_RENDERER_SPECTRAL) return spectral_sample(c, px, py, s, L, imgX, imgY);
    return sampler_sample(c, px, py, s, L, imgX, imgY);
}

/* ------------------------------------------------------------------ exported API */
int oracle_abi_version(void) { return PBRTGPU_ABI_VERSION; }
int oracle_libm_float(void) {
#ifdef ORACLE_LIBM_FLOAT
    return 1;
#else
    return 0;
#endif
}

/* per-path radiance for keys [n][3] = (x, y, s) */
/* first n outputs of MT19937 seeded with seed (RNG::Seed + RandomUInt, rng.cpp:35-100) */
int oracle_mt_first(uint32_t seed, int n, uint32_t *out) {
    RNG r;
    rng_seed(&r, seed);
    for (int i = 0; i < n; ++i) out[i] = rng_uint(&r);
    return 0;
}
int oracle_trace_paths(const pbrtgpu_flat_scene *s, const int32_t *keys, int32_t n, float *out) {
    Ctx c = {s, s->n_bands};
    if (!spectral_ok(s)) return -1;
    for (int k = 0; k < n; ++k) trace_path(&c, keys[3 * k], keys[3 * k + 1], (uint32_t)keys[3 * k + 2], out + (size_t)k * s->n_bands, NULL, NULL);
    return 0;
}

/* closest / any hit queries: rays [n][8] (o, d, mint, maxt); hits [n][4] (t, b1, b2, prim) */
int oracle_intersect(const pbrtgpu_flat_scene *s, const float *rays, int32_t n, float *hits, int32_t *occluded) {
    Ctx c = {s, s->n_bands};
    for (int k = 0; k < n; ++k) {
        const float *q = rays + 8 * k;
        Ray r; r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]); r.mint = q[6]; r.maxt = q[7]; r.time = 0.f;
        Ray r2 = r;
        Hit h;
        if (bvh_intersect(&c, &r, &h)) { hits[4 * k] = h.t; hits[4 * k + 1] = 0.f; hits[4 * k + 2] = 0.f; int32_t p = h.prim; memcpy(&hits[4 * k + 3], &p, 4); }
        else { hits[4 * k] = INFINITY; hits[4 * k + 1] = 0.f; hits[4 * k + 2] = 0.f; int32_t p = -1; memcpy(&hits[4 * k + 3], &p, 4); }
        if (occluded) occluded[k] = bvh_intersectP(&c, &r2);
    }
    return 0;
}

/* Film render over a window of sample pixels [x0,x1)x[y0,y1) (clamped to the sample
 * extent), all samples [0,spp).  film: [py_count][px_count][nb] float32.
 * The reference harness adds samples in sample-pixel row-major order, samples ascending
 * (SamplerRendererTask::Run + SpectralImageFilm::AddSample).  A sample whose imageX or
 * imageY rounds to an integer also lands on a neighbouring pixel ("spill"); for a film
 * pixel T the contribution order is therefore: spills from earlier sample pixels, T's own
 * samples, spills from later sample pixels.  Spill samples are found from
 * the sampler alone (no tracing) and traced first. */
typedef struct {
    const Ctx *c;
    int x0, x1, y0, y1, spp;
    float *film;
    int nextRow;
    pthread_mutex_t mu;
    long zeroed;
    int phase;                 /* 0: spill scan, 1: trace spills, 2: own accumulation */
    int32_t *spillKeys;        /* [n][3] x, y, s */
    long nSpill, capSpill, nextSpill;
    float *spillL;             /* [n][nb] */
} Job;

static inline void footprint(const pbrtgpu_camera *cam, float ix, float iy, int *fx0, int *fx1, int *fy0, int *fy1) {
    float dx = ix - 0.5f, dy = iy - 0.5f;   /* spectralImage.cpp:80-91, box filter width .5 */
    *fx0 = (int)ceilf(dx - 0.5f); *fx1 = (int)floorf(dx + 0.5f);
    *fy0 = (int)ceilf(dy - 0.5f); *fy1 = (int)floorf(dy + 0.5f);
    if (*fx0 < cam->px_start) *fx0 = cam->px_start;
    if (*fx1 > cam->px_start + cam->px_count - 1) *fx1 = cam->px_start + cam->px_count - 1;
    if (*fy0 < cam->py_start) *fy0 = cam->py_start;
    if (*fy1 > cam->py_start + cam->py_count - 1) *fy1 = cam->py_start + cam->py_count - 1;
}
static inline void image_xy(const Ctx *c, int x, int y, uint32_t s, float *ix, float *iy) {
    uint32_t hp = pixel_hash(c->s->seed, x, y);
    float u[2];
    s2d(hp, 0, s, (uint32_t)c->s->spp, u);
    *ix = x + u[0];
    *iy = y + u[1];
}
static void *worker(void *arg) {
    Job *j = (Job *)arg;
    const Ctx *c = j->c;
    const pbrtgpu_camera *cam = &c->s->camera;
    int nb = c->nb;
    float L[MAXB];
    if (j->phase == 1) {
        for (;;) {
            pthread_mutex_lock(&j->mu);
            long k = j->nextSpill++;
            pthread_mutex_unlock(&j->mu);
            if (k >= j->nSpill) break;
            const int32_t *key = j->spillKeys + 3 * k;
            trace_path(c, key[0], key[1], (uint32_t)key[2], j->spillL + (size_t)k * nb, NULL, NULL);
        }
        return NULL;
    }
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int y = j->nextRow++;
        pthread_mutex_unlock(&j->mu);
        if (y >= j->y1) break;
        for (int x = j->x0; x < j->x1; ++x) {
            int own = x >= cam->px_start && x < cam->px_start + cam->px_count && y >= cam->py_start &&
                      y < cam->py_start + cam->py_count;
            for (int s = 0; s < j->spp; ++s) {
                float ix, iy;
                int fx0, fx1, fy0, fy1;
                if (j->phase == 0) {
                    image_xy(c, x, y, (uint32_t)s, &ix, &iy);
                    footprint(cam, ix, iy, &fx0, &fx1, &fy0, &fy1);
                    if (fx1 - fx0 < 0 || fy1 - fy0 < 0) continue;
                    if (fx0 == x && fx1 == x && fy0 == y && fy1 == y) continue;
                    pthread_mutex_lock(&j->mu);
                    if (j->nSpill == j->capSpill) {
                        j->capSpill = j->capSpill ? 2 * j->capSpill : 256;
                        j->spillKeys = (int32_t *)realloc(j->spillKeys, sizeof(int32_t) * 3 * j->capSpill);
                    }
                    int32_t *k = j->spillKeys + 3 * j->nSpill++;
                    k[0] = x; k[1] = y; k[2] = s;
                    pthread_mutex_unlock(&j->mu);
                    continue;
                }
                if (!own) continue;
                memset(L, 0, sizeof(L));
                int bad = trace_path(c, x, y, (uint32_t)s, L, &ix, &iy);
                if (bad) { pthread_mutex_lock(&j->mu); j->zeroed++; pthread_mutex_unlock(&j->mu); }
                float *pix = j->film + ((size_t)(y - cam->py_start) * cam->px_count + (x - cam->px_start)) * nb;
                for (int i = 0; i < nb; ++i) pix[i] += 1.f * L[i];
            }
        }
    }
    return NULL;
}
typedef struct { int32_t target, src, s, idx; } Contrib;
static int cmp_contrib(const void *a, const void *b) {
    const Contrib *x = (const Contrib *)a, *y = (const Contrib *)b;
    if (x->target != y->target) return x->target < y->target ? -1 : 1;
    if (x->src != y->src) return x->src < y->src ? -1 : 1;
    return x->s < y->s ? -1 : (x->s > y->s);
}
static void run_phase(Job *j, int phase, int nthreads) {
    j->phase = phase;
    j->nextRow = j->y0;
    j->nextSpill = 0;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, j);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
}
int oracle_render(const pbrtgpu_flat_scene *s, int x0, int x1, int y0, int y1, float *film, int nthreads,
                  double *stats) {
    Ctx c = {s, s->n_bands};
    if (!spectral_ok(s)) return -1;
    const pbrtgpu_camera *cam = &s->camera;
    int nb = s->n_bands;
    Job j;
    memset(&j, 0, sizeof(j));
    j.c = &c;
    j.x0 = x0 < cam->sx_start ? cam->sx_start : x0; j.x1 = x1 > cam->sx_end ? cam->sx_end : x1;
    j.y0 = y0 < cam->sy_start ? cam->sy_start : y0; j.y1 = y1 > cam->sy_end ? cam->sy_end : y1;
    j.spp = s->spp;
    j.film = film;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    run_phase(&j, 0, nthreads);            /* find spill samples */
    j.spillL = (float *)malloc(sizeof(float) * nb * (j.nSpill + 1));
    run_phase(&j, 1, nthreads);            /* trace them */
    /* contributions of spill samples to pixels other than their own */
    long nc = 0, cap = 4 * j.nSpill + 1;
    Contrib *cs = (Contrib *)malloc(sizeof(Contrib) * cap);
    int ew = cam->sx_end - cam->sx_start;
    for (long k = 0; k < j.nSpill; ++k) {
        const int32_t *key = j.spillKeys + 3 * k;
        float ix, iy;
        int fx0, fx1, fy0, fy1;
        image_xy(&c, key[0], key[1], (uint32_t)key[2], &ix, &iy);
        footprint(cam, ix, iy, &fx0, &fx1, &fy0, &fy1);
        for (int fy = fy0; fy <= fy1; ++fy)
            for (int fx = fx0; fx <= fx1; ++fx) {
                if (fx == key[0] && fy == key[1]) continue;
                Contrib *q = &cs[nc++];
                q->target = (fy - cam->py_start) * cam->px_count + (fx - cam->px_start);
                q->src = (key[1] - cam->sy_start) * ew + (key[0] - cam->sx_start);
                q->s = key[2];
                q->idx = (int32_t)k;
            }
    }
    qsort(cs, nc, sizeof(Contrib), cmp_contrib);
    /* pre-spills: sources earlier (row-major) than the target's own sample pixel */
    for (long k = 0; k < nc; ++k) {
        int tx = cs[k].target % cam->px_count + cam->px_start, ty = cs[k].target / cam->px_count + cam->py_start;
        int ownIdx = (ty - cam->sy_start) * ew + (tx - cam->sx_start);
        if (cs[k].src < ownIdx) {
            float *pix = film + (size_t)cs[k].target * nb;
            const float *L = j.spillL + (size_t)cs[k].idx * nb;
            for (int i = 0; i < nb; ++i) pix[i] += 1.f * L[i];
        }
    }
    run_phase(&j, 2, nthreads);            /* own samples, in order */
    for (long k = 0; k < nc; ++k) {         /* post-spills */
        int tx = cs[k].target % cam->px_count + cam->px_start, ty = cs[k].target / cam->px_count + cam->py_start;
        int ownIdx = (ty - cam->sy_start) * ew + (tx - cam->sx_start);
        if (cs[k].src > ownIdx) {
            float *pix = film + (size_t)cs[k].target * nb;
            const float *L = j.spillL + (size_t)cs[k].idx * nb;
            for (int i = 0; i < nb; ++i) pix[i] += 1.f * L[i];
        }
    }
    if (stats) {
        stats[0] = (double)(j.x1 - j.x0) * (j.y1 - j.y0) * j.spp;
        stats[1] = (double)j.zeroed;
        stats[2] = (double)j.nSpill;
    }
    free(cs);
    free(j.spillKeys);
    free(j.spillL);
    pthread_mutex_destroy(&j.mu);
    return 0;
}

/* Throughput helper for the CPU baseline: trace a bounded list of paths over the
 * sample extent (every path traced fully, no film), returns paths traced. */
typedef struct { const Ctx *c; long n0, n1; long next; pthread_mutex_t mu; int W, H; } TJob;
static void *tworker(void *arg) {
    TJob *t = (TJob *)arg;
    float L[MAXB];
    for (;;) {
        pthread_mutex_lock(&t->mu);
        long k = t->next; t->next += 64;
        pthread_mutex_unlock(&t->mu);
        if (k >= t->n1) break;
        long e = k + 64 < t->n1 ? k + 64 : t->n1;
        for (long q = k; q < e; ++q) {
            /* all samples of pseudo-randomly spread pixels: a representative sample of the frame */
            long npix = (long)t->W * t->H;
            long pix = (long)(((unsigned long long)(q / t->c->s->spp) * 2654435761ull) % (unsigned long long)npix);
            int s = (int)(q % t->c->s->spp);
            int x = t->c->s->camera.px_start + (int)(pix % t->W), y = t->c->s->camera.py_start + (int)(pix / t->W);
            trace_path(t->c, x, y, (uint32_t)s, L, NULL, NULL);
        }
    }
    return NULL;
}
long oracle_trace_range(const pbrtgpu_flat_scene *s, long first, long count, int nthreads) {
    Ctx c = {s, s->n_bands};
    if (!spectral_ok(s)) return -1;
    TJob t;
    t.c = &c; t.n0 = first; t.n1 = first + count; t.next = first; t.W = s->camera.px_count; t.H = s->camera.py_count;
    pthread_mutex_init(&t.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, tworker, &t);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    free(th);
    pthread_mutex_destroy(&t.mu);
    return count;
}

/* test hook: IrregIsotropicBRDF::f of material `mat` for local directions wo, wi */
int oracle_measured_f(const pbrtgpu_flat_scene *s, int mat, const float *wo, const float *wi, float *out) {
    Ctx c;
    memset(&c, 0, sizeof(c));
    c.s = s;
    c.nb = s->n_bands;
    const pbrtgpu_material *mt = &s->materials[mat];
    if (mt->type != PBRTGPU_MAT_MEASURED) return -1;
    BxDF b;
    memset(&b, 0, sizeof(b));
    b.kind = BX_MEASURED_IRREG;
    b.kd = s->kdnodes + mt->aux;
    b.nkd = mt->aux2;
    irreg_f(&c, &b, v3(wo[0], wo[1], wo[2]), v3(wi[0], wi[1], wi[2]), out);
    return 0;
}

/* test hook: the float transcendentals of this build (fn: PBRTGPU_LIBMF_*; powf / atan2f take
 * y; sincosf writes (sin, cos) pairs) -- glibc's own in liboracle_libm.so, include/pbrt_libmf.h
 * in liboracle.so; tests/test_libmf.py compares the GPU's with both */
int oracle_libmf_eval(int fn, int64_t n, const float *x, const float *y, float *out) {
    for (int64_t i = 0; i < n; ++i) {
        const float a = x[i];
        switch (fn) {
        case PBRTGPU_LIBMF_SINF: out[i] = SINF(a); break;
        case PBRTGPU_LIBMF_COSF: out[i] = COSF(a); break;
        case PBRTGPU_LIBMF_SINCOSF: out[2 * i] = SINF(a); out[2 * i + 1] = COSF(a); break;
        case PBRTGPU_LIBMF_EXPF: out[i] = EXPF(a); break;
        case PBRTGPU_LIBMF_LOGF: out[i] = LOGF(a); break;
        case PBRTGPU_LIBMF_ACOSF: out[i] = ACOSF(a); break;
        case PBRTGPU_LIBMF_ATANF: out[i] = ATANF(a); break;
        case PBRTGPU_LIBMF_TANF: out[i] = TANF(a); break;
        case PBRTGPU_LIBMF_POWF: out[i] = POWF(a, y[i]); break;
        case PBRTGPU_LIBMF_ATAN2F: out[i] = ATAN2F(a, y[i]); break;
        default: return -1;
        }
    }
    return 0;
}
