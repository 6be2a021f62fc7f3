// device.h -- CDNA4 (gfx950) device code of the spectral path tracer.
//
// Every function restates the reference arithmetic exactly (same operand order, float vs
// double promotion, correctly-rounded div/sqrt, no FMA contraction: build with
// -ffp-contract=off).  Float transcendentals are the reference's own libm routines restated
// bit for bit (include/pbrt_libmf.h, shared with the CPU oracle).
//
// GPU-specific structure (not in the reference):
//   * BVH nodes are read as two 16-byte loads; the traversal stack lives in LDS, one
//     column per lane (bank = lane), depth sized from the BVH depth at launch.
//   * triangle vertices are pre-gathered per primitive in BVH leaf order (48 B, 3 loads).
//   * spectra are NB-wide register arrays (NB = 32 or 60 template parameter); material,
//     light and band-Y spectra are read from the scene spectrum pool.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "pbrtgpu.h"
#include "pbrt_fmath.h"
#include "pbrt_libmf.h"

// Timing-ablation switches that knowingly change the radiance (PGD_EXP_* / PGD_EXPERIMENT_*,
// DESIGN.md §4.2, §5) compile only in experiment builds (tools/build_exp*.sh -> lib/exp/, which
// define PGD_EXPERIMENT_BUILD); the product library refuses them
#if !defined(PGD_EXPERIMENT_BUILD) &&                                                                   \
    (defined(PGD_EXPERIMENT_FASTMATH) || defined(PGD_EXPERIMENT_NO_MIS) || defined(PGD_EXPERIMENT_NO_NEE) ||  \
     defined(PGD_EXP_KD_FIXED) || defined(PGD_EXP_MEAS_CHEAP) || defined(PGD_EXP_MT_CHEAP) ||              \
     defined(PGD_EXP_NOBETA) || defined(PGD_EXP_NOSPEC) || defined(PGD_EXP_NO_AB) ||                        \
     defined(PGD_EXP_NO_MT_LIST) || defined(PGD_EXP_NO_OUT) || defined(PGD_EXP_NO_ABLOOP) ||                  \
     defined(PGD_EXP_NB_HALF))
#error "PGD_EXP* / PGD_EXPERIMENT_* switches change the radiance: experiment builds only (tools/build_exp.sh)"
#endif

namespace pgd {

#define PGD_INLINE __device__ __forceinline__
// large shading routines with several call sites: one out-of-line copy each keeps the shade
// kernel's code (instruction-cache footprint) small
#ifdef PGD_OUTLINE
#define PGD_HEAVY __device__ __attribute__((noinline))
#else
#define PGD_HEAVY __device__ __forceinline__
#endif
#define PGD_HD __host__ __device__ __forceinline__
// the global address space, spelled out where an out-of-line function receives a pointer (its
// accesses would be generic: flat loads / stores, which also count on the LDS counter); the host
// replay of tools/hostsan defines it empty
#ifndef PGD_GLOBAL_AS
#define PGD_GLOBAL_AS __attribute__((address_space(1)))
#endif
static constexpr float kPi = 3.14159265358979323846f;
static constexpr float kInvPi = 0.31830988618379067154f;
static constexpr float kInvTwoPi = 0.15915494309189533577f;
static constexpr float kOneMinusEps = 0x1.fffffep-1f;

// float transcendentals: the reference's glibc routines restated bit for bit (include/
// pbrt_libmf.h, shared with the CPU oracle).  On the GPU each one is a single
// out-of-line copy: inlined at every call site they grew the shade kernel's code and register
// budget (shade 379 -> 361 ms/frame on C2 when outlined, r01f ablation)
#ifdef PGD_TRANS_INLINE
#define PGD_TFN PGD_INLINE
#else
#define PGD_TFN __device__ __attribute__((noinline))
#endif
#ifndef PGD_EXPERIMENT_FASTMATH
PGD_TFN float SINF(float x) { return libmf_sinf(x); }
PGD_TFN float COSF(float x) { return libmf_cosf(x); }
PGD_TFN float POWF(float x, float y) { return libmf_powf(x, y); }
PGD_TFN float EXPF(float x) { return libmf_expf(x); }
PGD_TFN float ACOSF(float x) { return libmf_acosf(x); }
PGD_TFN float ATAN2F(float y, float x) { return libmf_atan2f(y, x); }
PGD_TFN float TANF(float x) { return libmf_tanf(x); }
PGD_TFN float ATANF(float x) { return libmf_atanf(x); }
PGD_TFN float LOGF(float x) { return libmf_logf(x); }
// (SINF(x), COSF(x)) from one argument reduction -- glibc's sincosf, the same two values
PGD_TFN float2 SINCOSF(float x) {
    float s, c;
    libmf_sincosf(x, &s, &c);
    return make_float2(s, c);
}
#else
PGD_INLINE float2 SINCOSF(float x) { return make_float2(__sinf(x), __cosf(x)); }
PGD_INLINE float LOGF(float x) { return __logf(x); }   // timing experiment only (not the parity definition): float library functions
PGD_INLINE float SINF(float x) { return __sinf(x); }
PGD_INLINE float COSF(float x) { return __cosf(x); }
PGD_INLINE float POWF(float x, float y) { return __powf(x, y); }
PGD_INLINE float ACOSF(float x) { return acosf(x); }
PGD_INLINE float ATAN2F(float y, float x) { return atan2f(y, x); }
PGD_INLINE float TANF(float x) { return __tanf(x); }
PGD_INLINE float ATANF(float x) { return atanf(x); }
#endif

// Scene and slot arrays are addressed through a 32-bit element index from their base: the base
// is a kernel argument (wave-uniform, in SGPRs) and the byte offset a 32-bit value, so a load or
// store takes one VGPR of address (global saddr mode) instead of a 64-bit per-lane pointer --
// fewer registers live across the kernels and no 64-bit address arithmetic.  Every array
// addressed this way is < 4 GiB (scene_build.h and pbrtgpu.hip ensure_slots check it).
template <class T> PGD_INLINE T *sa(T *base, uint32_t i) {
    return reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (uint32_t)(i * (uint32_t)sizeof(T)));
}
template <class T> PGD_INLINE const T *sa(const T *base, uint32_t i) {
    return reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (uint32_t)(i * (uint32_t)sizeof(T)));
}

// ------------------------------------------------------------------ vectors
struct V { float x, y, z; };
PGD_INLINE V v3(float x, float y, float z) { V r; r.x = x; r.y = y; r.z = z; return r; }
PGD_INLINE V vadd(V a, V b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PGD_INLINE V vsub(V a, V b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PGD_INLINE V vneg(V a) { return v3(-a.x, -a.y, -a.z); }
PGD_INLINE V vmul(V a, float f) { return v3(f * a.x, f * a.y, f * a.z); }
PGD_INLINE V vdiv(V a, float f) { float inv = 1.f / f; return v3(a.x * inv, a.y * inv, a.z * inv); }
PGD_INLINE float vdot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PGD_INLINE float vlen2(V a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
PGD_INLINE float vlen(V a) { return sqrtf(vlen2(a)); }
PGD_INLINE V vnorm(V a) { return vdiv(a, vlen(a)); }
// geometry.h:461-468: products exact in double, one rounding per component.  A product of two floats
// is exact in double (48 significant bits), so (p - q) rounded once equals fma(a, b, -q) rounded
// once: one DMUL and one DFMA per component instead of two DMULs and a DADD, the same bits
PGD_INLINE V vcross(V a, V b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
#ifdef PGD_AB_VCROSS_DFMA
    return v3((float)fma(ay, bz, -(az * by)), (float)fma(az, bx, -(ax * bz)), (float)fma(ax, by, -(ay * bx)));
#else
    return v3((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx)));
#endif
}
PGD_HD float pmin(float a, float b) { return (b < a) ? b : a; }
PGD_HD float pmax(float a, float b) { return (a < b) ? b : a; }
PGD_INLINE float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
PGD_INLINE float lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }
PGD_INLINE V faceforward(V n, V v) { return (vdot(n, v) < 0.f) ? vneg(n) : n; }
PGD_INLINE void coordsys(V v1, V *v2, V *v3_) {
    if (fabsf(v1.x) > fabsf(v1.y)) {
        float invLen = 1.f / sqrtf(v1.x * v1.x + v1.z * v1.z);
        *v2 = v3(-v1.z * invLen, 0.f, v1.x * invLen);
    } else {
        float invLen = 1.f / sqrtf(v1.y * v1.y + v1.z * v1.z);
        *v2 = v3(0.f, v1.z * invLen, -v1.y * invLen);
    }
    *v3_ = vcross(v1, *v2);
}
PGD_INLINE V xpoint(const float *m, V p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1.) return v3(xp, yp, zp);
    return vdiv(v3(xp, yp, zp), wp);
}
PGD_INLINE V xvec(const float *m, V v) {
    return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
PGD_INLINE V xnormal(const float *mi, V n) {
    return v3(mi[0] * n.x + mi[4] * n.y + mi[8] * n.z, mi[1] * n.x + mi[5] * n.y + mi[9] * n.z,
              mi[2] * n.x + mi[6] * n.y + mi[10] * n.z);
}
struct Ray { V o, d; float mint, maxt, time; };
PGD_INLINE V rayat(const Ray &r, float t) { return vadd(r.o, vmul(r.d, t)); }

// ------------------------------------------------------------------ sampler
PGD_HD uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
PGD_HD uint32_t pixel_hash(uint32_t seed, int px, int py) {
    uint32_t h = mix32(seed + 0x9E3779B9U);
    h = mix32(h ^ (uint32_t)px);
    h = mix32(h ^ ((uint32_t)py * 0x85EBCA6BU));
    return h;
}
PGD_HD uint32_t dim_scramble(uint32_t hp, uint32_t d) { return mix32(hp ^ (0x9E3779B9U * (d + 1U))); }
PGD_HD uint32_t perm_index(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp) {
    return s ^ (mix32(dim_scramble(hp, d) ^ 0x5BD1E995U) & (spp - 1U));
}
PGD_HD uint32_t path_seed(uint32_t hp, uint32_t s) { return mix32(hp ^ mix32(s + 0x7F4A7C15U)); }
PGD_HD float vdc(uint32_t n, uint32_t scramble) {   // montecarlo.h:269-278
    n = __builtin_bitreverse32(n);
    n ^= scramble;
    return pmin(((n >> 8) & 0xffffff) / (float)(1 << 24), kOneMinusEps);
}
PGD_HD float sobol2(uint32_t n, uint32_t scramble) {   // montecarlo.h:281-285
    for (uint32_t v = 1u << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 0x1) scramble ^= v;
    return pmin(((scramble >> 8) & 0xffffff) / (float)(1 << 24), kOneMinusEps);
}
PGD_HD float s1d(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp) { return vdc(perm_index(hp, d, s, spp), dim_scramble(hp, d)); }
PGD_HD void s2d(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp, float *u) {
    uint32_t sp = perm_index(hp, d, s, spp), sc = dim_scramble(hp, d);
    u[0] = vdc(sp, sc);
    u[1] = sobol2(sp, mix32(sc ^ 0x68BC21EBU));
}
#define PGD_N1D 14
#define DIM_1D(j) (3u + (uint32_t)(j))
#define DIM_2D(k) (3u + PGD_N1D + (uint32_t)(k))

// MT19937 first-generation stream (rng.cpp:35-100).  A path draws at most 32 values
// (3 bounces x 10 + 2 roulette draws at maxdepth 5), all from the first 227-word block,
// whose outputs depend only on the seed recurrence: out_k = temper(mt[k+397] ^
// twist(mt[k], mt[k+1])).  State: the recurrence at positions k, k+1 and k+397.
struct MT {
    uint32_t k;        // next output index
    uint32_t a, b;     // mt[k], mt[k+1]
    uint32_t m;        // mt[k+397]
    bool init;
    uint32_t seed;
    uint32_t *ext;     // the slot's full 624-word state for outputs k >= 227, or null (mt_ext)
};
PGD_INLINE uint32_t mt_next_word(uint32_t prev, uint32_t idx) { return 1812433253U * (prev ^ (prev >> 30)) + idx; }
PGD_INLINE void mt_begin(MT &r, uint32_t seed) { r.seed = seed; r.init = false; r.k = 0; r.ext = nullptr; }
// the seed recurrence up to mt[397]: once per path, before its first draw (one copy; a
// fully unrolled 396-step loop at every draw site would dominate the shade kernel's code).
// Scalars in and out: an MT passed by reference to an out-of-line function would live in
// scratch memory at every draw site.
__device__ __attribute__((noinline)) uint32_t mt_word397(uint32_t w) {
#ifdef PGD_EXP_MT_CHEAP   // timing experiment only: the recurrence's cost (wrong MT values)
    for (uint32_t i = 2; i <= 5; ++i) w = mt_next_word(w, i);
    return w;
#endif
#pragma unroll 4
    for (uint32_t i = 2; i <= 397; ++i) w = mt_next_word(w, i);
    return w;
}
PGD_INLINE void mt_init(MT &r) {
    r.a = r.seed;
    r.b = mt_next_word(r.a, 1);
    r.m = mt_word397(r.b);
    r.init = true;
}
PGD_INLINE uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}
PGD_INLINE uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {   // one twist step (rng.cpp:68-78)
    const uint32_t y = (a & 0x80000000U) | (b & 0x7fffffffU);
    return m ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
}
// Outputs k >= 227 of RNG (rng.cpp:60-100): from there on a twist step reads words the same
// generation already rewrote, so the 5-word window no longer suffices.  The path's full state
// lives in its slot's ext row (PathSoA::mtExt, allocated when maxdepth allows so many draws):
// at k = 227 it is rebuilt from the seed (Seed + the first twist of the whole array), at
// k = 624 j (j >= 1) twisted in place, exactly as RNG::RandomUInt regenerates; output k is
// the tempered word k mod 624.  Out of line, scalars in and out (no MT in private memory at
// the draw sites): paths get here only beyond ~20 bounces.
__device__ __attribute__((noinline)) uint32_t mt_ext_draw(uint32_t k, uint32_t seed, uint32_t *mt) {
    if (k == 227 || k % 624 == 0) {
        if (k == 227) {
            mt[0] = seed;
            for (uint32_t i = 1; i < 624; ++i) mt[i] = mt_next_word(mt[i - 1], i);
        }
        int kk = 0;
        for (; kk < 624 - 397; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + 397]);
        for (; kk < 623; ++kk) mt[kk] = mt_mix(mt[kk], mt[kk + 1], mt[kk + (397 - 624)]);
        mt[623] = mt_mix(mt[623], mt[0], mt[396]);
    }
    return mt_temper(mt[k % 624]);
}
PGD_INLINE uint32_t mt_uint(MT &r) {   // requires r.init (mt_init)
    if (__builtin_expect(r.k >= 227, 0)) {
        // without an ext row (run_wavefront allocates them when the integrator's maxdepth can get
        // here) the draw is 0 and mt_store flags the run (CNT_ERR -> PBRTGPU_E_STATE)
        const uint32_t y = r.ext ? mt_ext_draw(r.k, r.seed, r.ext) : 0u;
        r.k++;
        return y;
    }
    uint32_t y = mt_mix(r.a, r.b, r.m);
    // advance the recurrence windows
    r.a = r.b;
    r.b = mt_next_word(r.b, r.k + 2);
    r.m = mt_next_word(r.m, r.k + 398);
    r.k++;
    return mt_temper(y);
}
PGD_INLINE float mt_float(MT &r) { return (mt_uint(r) & 0xffffff) / (float)(1 << 24); }

// montecarlo.cpp:298-340
PGD_INLINE void concentric_disk(float u1, float u2, float *dx, float *dy) {
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
    theta *= kPi / 4.f;
    const float2 sc = SINCOSF(theta);
    *dx = r * sc.y;
    *dy = r * sc.x;
}
PGD_INLINE V cosine_hemisphere(float u1, float u2) {
    V r;
    concentric_disk(u1, u2, &r.x, &r.y);
    r.z = sqrtf(pmax(0.f, 1.f - r.x * r.x - r.y * r.y));
    return r;
}
PGD_INLINE V uniform_sphere(float u1, float u2) {
    float z = 1.f - 2.f * u1;
    float r = sqrtf(pmax(0.f, 1.f - z * z));
    float phi = 2.f * kPi * u2;
    const float2 sc = SINCOSF(phi);
    return v3(r * sc.y, r * sc.x, z);
}
PGD_INLINE float power_heuristic(float fPdf, float gPdf) {
    float f = 1 * fPdf, g = 1 * gPdf;
    return (f * f) / (f * f + g * g);
}

// ------------------------------------------------------------------ device scene
// p1.xyz, shape | p2.xyz, pad | p3.xyz, pad -- `shape` (bits of a.w) the primitive's shape type
// (PBRTGPU_SHAPE_TRIANGLE = 0, the vertices meaningful), so a leaf's primitive test loads this one
// record first and the pbrtgpu_prim only for the other shapes
struct DevTri { float4 a, b, c; };
struct DevScene {
    int nb, maxDepth, spp, stackDepth;
    uint32_t seed;
    float yint;
    const float *bandY;
    pbrtgpu_camera cam;
    const float4 *nodes;              // 2 x float4 per node (the flattened scene's BVH; roots are tested here)
    const float4 *wnodes;             // child-in-parent BVH: 4 x float4 per interior node (wide_bvh)
    const uint32_t *nodeRef;          // per node: its wide-node index, or a leaf reference (WREF_*)
    int nTop;                         // wide nodes [0, nTop): the BVH's top levels, breadth-first (LDS in k_trace_pt)
    const float4 *w4nodes;            // 4-wide copy for the shadow queries (wide4_bvh): 8 x float4 per node
    int w4N, w4Stack;                 // its nodes (0: none) and the any-hit stack bound (3 per level + 1)
    const uint4 *w4q;                 // its quantized copy (scene_build.h quant_w4): 4 x uint4 per node, or null
    const int *leafOf;                // per first primitive of a leaf: the binary leaf node (quant_w4)
    const pbrtgpu_prim *prims;
    const DevTri *primTri;            // per prim (triangles only meaningful)
    const float4 *primRec;            // per prim: its shading record, 8 float4 (PrimRec below)
    const pbrtgpu_triangle *tris;
    const pbrtgpu_mesh *meshes;
    const float *vertP, *vertN, *vertUV;
    const pbrtgpu_quadric *quads;
    const pbrtgpu_material *mats;
    const pbrtgpu_light *lights;
    int nLights;
    const pbrtgpu_light_shape *lightShapes;
    const float *spectra;
    const pbrtgpu_instance *insts;    // TransformedPrimitive records (may be empty)
    const int *primInst;              // per prim: owning instance or -1
    int nInsts;
    const pbrtgpu_kdnode *kd;         // measured BRDF kd-trees
    const float4 *kdPack;             // kd nodes packed for the lookup walk (kd_lookup, wavefront.h)
    int nKd, kdInLds;                 // kd nodes in all trees; 1: k_shade copies them to LDS
    const float *merl;                // RegularHalfangleBRDF RGB tables (3 floats per texel)
    const pbrtgpu_texture *tex;       // texture nodes (image maps, scale, constants)
    const float *ewa;                 // [128] MIPMap::weightLut
    const float *texels;              // the image maps' MIPMap pyramids (pbrtgpu_texture::texel_off)
    const pbrtgpu_instance *camMotion;   // an animated camera's CameraToWorld, or null (cam.cam2world_m)
    const float *basis;               // [14][nbp] FromRGB basis spectra, band-quad padded
    int nbp;                          // padded band count (multiple of 4)
    int nInf;                         // infinite lights among lights[]
    int integrator, dlStrategy;       // PBRTGPU_INTEGRATOR_*, PBRTGPU_DL_*
    int dlK;                          // DirectLighting light samples per vertex (sum of RoundUpPow2(nSamples))
    int metaStrategy;                 // PBRTGPU_META_* (MetadataIntegrator)
    const uint32_t *primMeta;         // [prims][2]: primitiveId, materialId a hit reports
    // SpectralRenderer (spectralrenderer.cpp:60-223): specItems paths per camera sample
    // (nWaveBands for singleDirection, 1 for samplerDirection and the SamplerRenderer)
    int specMode;                     // 0: SamplerRenderer, 1: singleDirection, 2: samplerDirection
    int specBands;                    // nWaveBands
    int specItems;
    const int4 *specTab;              // [nWaveBands]: assigned indices [x, y), interval z (-1: none), t (bits)
    const float *specWl;              // [nWaveBands]: the band's ray wavelength
    int camType;                      // PBRTGPU_CAMERA_*
    int lensN, lensChromatic;         // RealisticDiffractionCamera: elements, chromaticAberrationEnabled
    int lensDiffraction;              // diffractionEnabled
    float lensFilmDist, lensFilmDiag, lensCurveR, lensApOff[2], lensFilmC[2], lensPinhole[3];
    const float4 *lensEl;             // [lensN]: radius, separation, n, aperture
    int lensPinW, lensPinH;           // pinhole array (both > 0), its microlenses, the eye IOR curves
    int lensMicro, lensEye;
    const float *lensPinholes;        // [lensPinW][lensPinH][3]
    const float *lensEyeIor;          // [4][NB]: cornea, aqueous, lens, vitreous
};

// scene features a shade kernel is specialised for (k_shade<NB, FEAT>): a scene without
// them runs a variant with that code compiled out
enum { FEAT_MEAS = 1, FEAT_TEX = 2, FEAT_INF = 4, FEAT_ALL = 7, FEAT_BASIC = 8, FEAT_NOSPEC = 16 };
// FEAT_BASIC: a scene without textures or infinite / spot / distant lights whose materials are all
// matte or plastic, or also measured with FEAT_MEAS (C2 and C5's killeroos: FEAT_BASIC; C3's bunny:
// FEAT_MEAS | FEAT_BASIC).  Its shading objects (shade.hip built with SHADE_FEAT 8 or 9) compile
// the Lambertian, Oren-Nayar, dielectric-Blinn (and measured) BxDFs only: the other kinds' sample,
// pdf and band code is never reached there (pbrtgpu.hip path_shade_variant)
#if defined(SHADE_FEAT) && (SHADE_FEAT & 8)
#define PGD_BASIC_MATS 1
#define PGD_BASIC_MEAS (SHADE_FEAT & 1)
#else
#define PGD_BASIC_MATS 0
#define PGD_BASIC_MEAS 0
#endif
// FEAT_NOSPEC: likewise for a scene without measured BRDFs whose materials are all matte, plastic,
// metal or substrate (C4's): its objects (SHADE_FEAT | 16) compile no specular, measured or Ward kind
#if defined(SHADE_FEAT) && (SHADE_FEAT & 16)
#define PGD_NOSPEC_MATS 1
#else
#define PGD_NOSPEC_MATS 0
#endif

struct DG { V p, nn, dpdu, dpdv, dndu, dndv; float u, v; };
PGD_INLINE void dg_init(DG &dg, V p, V dpdu, V dpdv, V dndu, V dndv, float u, float v, int flip) {
    dg.p = p; dg.dpdu = dpdu; dg.dpdv = dpdv; dg.dndu = dndu; dg.dndv = dndv;
    dg.nn = vnorm(vcross(dpdu, dpdv));
    dg.u = u; dg.v = v;
    if (flip) dg.nn = vmul(dg.nn, -1.f);
}
PGD_INLINE V ldv(const float *p) { return v3(p[0], p[1], p[2]); }

// Triangle::Intersect hit test (trianglemesh.cpp:119-157), vertices from primTri
PGD_INLINE bool tri_hit(const DevTri &t, const Ray &ray, float *tHit) {
    V p1 = v3(t.a.x, t.a.y, t.a.z), p2 = v3(t.b.x, t.b.y, t.b.z), p3 = v3(t.c.x, t.c.y, t.c.z);
    V e1 = vsub(p2, p1), e2 = vsub(p3, p1);
    V s1 = vcross(ray.d, e2);
    float divisor = vdot(s1, e1);
    if (divisor == 0.) return false;
    float invDivisor = 1.f / divisor;
    V d = vsub(ray.o, p1);
    float b1 = vdot(d, s1) * invDivisor;
    if (b1 < 0. || b1 > 1.) return false;
    V s2 = vcross(d, e1);
    float b2 = vdot(ray.d, s2) * invDivisor;
    if (b2 < 0. || b1 + b2 > 1.) return false;
    float tt = vdot(e2, s2) * invDivisor;
    if (tt < ray.mint || tt > ray.maxt) return false;
    *tHit = tt;
    return true;
}
PGD_INLINE void tri_uvs(const DevScene &S, const pbrtgpu_triangle &t, float uv[3][2]) {
    const pbrtgpu_mesh &m = (*sa(S.meshes, (uint32_t)(t.mesh)));
    if (m.has_uvs) {
        for (int k = 0; k < 3; ++k) { uv[k][0] = (*sa(S.vertUV, (uint32_t)(2 * t.v[k]))); uv[k][1] = (*sa(S.vertUV, (uint32_t)(2 * t.v[k] + 1))); }
    } else {
        uv[0][0] = 0.; uv[0][1] = 0.; uv[1][0] = 1.; uv[1][1] = 0.; uv[2][0] = 1.; uv[2][1] = 1.;
    }
}
// full Triangle::Intersect (dg + rayEpsilon) for a known-hit triangle
PGD_INLINE bool tri_intersect(const DevScene &S, int ti, const Ray &ray, float *tHit, float *rayEps, DG *dg) {
    const pbrtgpu_triangle t = (*sa(S.tris, (uint32_t)(ti)));
    V p1 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[0]))), p2 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[1]))), p3 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[2])));
    V e1 = vsub(p2, p1), e2 = vsub(p3, p1);
    V s1 = vcross(ray.d, e2);
    float divisor = vdot(s1, e1);
    if (divisor == 0.) return false;
    float invDivisor = 1.f / divisor;
    V d = vsub(ray.o, p1);
    float b1 = vdot(d, s1) * invDivisor;
    if (b1 < 0. || b1 > 1.) return false;
    V s2 = vcross(d, e1);
    float b2 = vdot(ray.d, s2) * invDivisor;
    if (b2 < 0. || b1 + b2 > 1.) return false;
    float tt = vdot(e2, s2) * invDivisor;
    if (tt < ray.mint || tt > ray.maxt) return false;
    if (!dg) { *tHit = tt; return true; }
    float uvs[3][2];
    tri_uvs(S, t, uvs);
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
    const pbrtgpu_mesh &m = (*sa(S.meshes, (uint32_t)(t.mesh)));
    dg_init(*dg, rayat(ray, tt), dpdu, dpdv, v3(0, 0, 0), v3(0, 0, 0), tu, tv, m.reverse_orientation ^ m.swaps_handedness);
    *tHit = tt;
    *rayEps = 1e-3f * *tHit;
    return true;
}
PGD_INLINE bool solve2x2(const float A[2][2], const float B[2], float *x0, float *x1) {
    float det = A[0][0] * A[1][1] - A[0][1] * A[1][0];
    if (fabsf(det) < 1e-10f) return false;
    *x0 = (A[1][1] * B[0] - A[0][1] * B[1]) / det;
    *x1 = (A[0][0] * B[1] - A[1][0] * B[0]) / det;
    if (isnan(*x0) || isnan(*x1)) return false;
    return true;
}
// Triangle::GetShadingGeometry (trianglemesh.cpp:285-360)
// nmat: mInv of the ObjectToWorld handed to GetShadingGeometry (the mesh's, or the instance-
// composed one of TransformedPrimitive::Intersect)
PGD_INLINE void tri_shading(const DevScene &S, int ti, const float *nmat, const DG &dg, DG &dgs) {
    const pbrtgpu_triangle t = (*sa(S.tris, (uint32_t)(ti)));
    const pbrtgpu_mesh &m = (*sa(S.meshes, (uint32_t)(t.mesh)));
    if (!m.has_normals) { dgs = dg; return; }
    float b[3];
    float uv[3][2];
    tri_uvs(S, t, uv);
    float A[2][2] = {{uv[1][0] - uv[0][0], uv[2][0] - uv[0][0]}, {uv[1][1] - uv[0][1], uv[2][1] - uv[0][1]}};
    float C[2] = {dg.u - uv[0][0], dg.v - uv[0][1]};
    if (!solve2x2(A, C, &b[1], &b[2])) b[0] = b[1] = b[2] = 1.f / 3.f;
    else b[0] = 1.f - b[1] - b[2];
    V n0 = ldv(sa(S.vertN, (uint32_t)(3 * t.v[0]))), n1 = ldv(sa(S.vertN, (uint32_t)(3 * t.v[1]))), n2 = ldv(sa(S.vertN, (uint32_t)(3 * t.v[2])));
    V ni = vadd(vadd(vmul(n0, b[0]), vmul(n1, b[1])), vmul(n2, b[2]));
    V ns = vnorm(xnormal(nmat, ni));
    V ss = vnorm(dg.dpdu);
    V ts = vcross(ss, ns);
    if (vlen2(ts) > 0.f) { ts = vnorm(ts); ss = vcross(ts, ns); }
    else coordsys(ns, &ss, &ts);
    V dndu, dndv;
    float du1 = uv[0][0] - uv[2][0], du2 = uv[1][0] - uv[2][0];
    float dv1 = uv[0][1] - uv[2][1], dv2 = uv[1][1] - uv[2][1];
    V dn1 = vsub(n0, n2), dn2 = vsub(n1, n2);
    float determinant = du1 * dv2 - dv1 * du2;
    if (determinant == 0.f) dndu = dndv = v3(0, 0, 0);
    else {
        float invdet = 1.f / determinant;
        dndu = vmul(vsub(vmul(dn1, dv2), vmul(dn2, dv1)), invdet);
        dndv = vmul(vadd(vmul(dn1, -du2), vmul(dn2, du1)), invdet);
    }
    dg_init(dgs, dg.p, ss, ts, xnormal(nmat, dndu), xnormal(nmat, dndv), dg.u, dg.v,
            m.reverse_orientation ^ m.swaps_handedness);
}

// Per-primitive shading record (scene_build.h, built at upload from the flattened scene): what
// isect_fill and get_bsdf read of a hit, in one 128-byte line per primitive instead of the chain
// prim -> triangle -> 3 vertices, 3 uvs, the mesh -> 3 normals (about 15 divergent cache-line
// requests per lane over three dependent levels).  The values are the flattened scene's, so every
// result is bit-identical:
//   r[0..2]  {p_k.xyz, w}   the triangle's vertices; w = u0, v0, u1
//   r[3..5]  {n_k.xyz, w}   its shading normals (mesh without normals: 0); w = v1, u2, v2
//            (the uvs are the mesh's, or Triangle::GetUVs's defaults (0,0) (1,0) (1,1))
//   r[6]     {shape_type, shape_index, material, area_light}   the pbrtgpu_prim
//   r[7]     {flags, mesh, 0, 0}   flags: REC_NORMALS the mesh has normals, REC_FLIP reverse ^ swaps
enum { REC_NORMALS = 2, REC_FLIP = 4 };
PGD_INLINE const float4 *prim_rec(const DevScene &S, int prim) { return sa(S.primRec, (uint32_t)(8 * prim)); }
PGD_INLINE int4 rec_prim(const float4 *rec) {
    const float4 v = rec[6];
    return make_int4(__float_as_int(v.x), __float_as_int(v.y), __float_as_int(v.z), __float_as_int(v.w));
}
// Triangle::Intersect (trianglemesh.cpp:119-199) of a known-hit triangle from its record:
// tri_intersect's arithmetic, operand for operand
PGD_INLINE bool tri_intersect_rec(const float4 *rec, const Ray &ray, float *tHit, float *rayEps, DG *dg) {
    const float4 a = rec[0], b = rec[1], cc = rec[2];
    V p1 = v3(a.x, a.y, a.z), p2 = v3(b.x, b.y, b.z), p3 = v3(cc.x, cc.y, cc.z);
    V e1 = vsub(p2, p1), e2 = vsub(p3, p1);
    V s1 = vcross(ray.d, e2);
    float divisor = vdot(s1, e1);
    if (divisor == 0.) return false;
    float invDivisor = 1.f / divisor;
    V d = vsub(ray.o, p1);
    float b1 = vdot(d, s1) * invDivisor;
    if (b1 < 0. || b1 > 1.) return false;
    V s2 = vcross(d, e1);
    float b2 = vdot(ray.d, s2) * invDivisor;
    if (b2 < 0. || b1 + b2 > 1.) return false;
    float tt = vdot(e2, s2) * invDivisor;
    if (tt < ray.mint || tt > ray.maxt) return false;
    if (!dg) { *tHit = tt; return true; }
    const float4 n0 = rec[3], n1 = rec[4], n2 = rec[5];
    const float uvs[3][2] = {{a.w, b.w}, {cc.w, n0.w}, {n1.w, n2.w}};
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
    dg_init(*dg, rayat(ray, tt), dpdu, dpdv, v3(0, 0, 0), v3(0, 0, 0), tu, tv, (__float_as_int(rec[7].x) & REC_FLIP) != 0);
    *tHit = tt;
    *rayEps = 1e-3f * *tHit;
    return true;
}
// Triangle::GetShadingGeometry (trianglemesh.cpp:285-360) from the record: tri_shading's arithmetic
PGD_INLINE void tri_shading_rec(const float4 *rec, const float *nmat, const DG &dg, DG &dgs) {
    const int flags = __float_as_int(rec[7].x);
    if (!(flags & REC_NORMALS)) { dgs = dg; return; }
    const float4 a = rec[0], b4 = rec[1], cc = rec[2], r3 = rec[3], r4 = rec[4], r5 = rec[5];
    const float uv[3][2] = {{a.w, b4.w}, {cc.w, r3.w}, {r4.w, r5.w}};
    float b[3];
    float A[2][2] = {{uv[1][0] - uv[0][0], uv[2][0] - uv[0][0]}, {uv[1][1] - uv[0][1], uv[2][1] - uv[0][1]}};
    float C[2] = {dg.u - uv[0][0], dg.v - uv[0][1]};
    if (!solve2x2(A, C, &b[1], &b[2])) b[0] = b[1] = b[2] = 1.f / 3.f;
    else b[0] = 1.f - b[1] - b[2];
    V n0 = v3(r3.x, r3.y, r3.z), n1 = v3(r4.x, r4.y, r4.z), n2 = v3(r5.x, r5.y, r5.z);
    V ni = vadd(vadd(vmul(n0, b[0]), vmul(n1, b[1])), vmul(n2, b[2]));
    V ns = vnorm(xnormal(nmat, ni));
    V ss = vnorm(dg.dpdu);
    V ts = vcross(ss, ns);
    if (vlen2(ts) > 0.f) { ts = vnorm(ts); ss = vcross(ts, ns); }
    else coordsys(ns, &ss, &ts);
    V dndu, dndv;
    float du1 = uv[0][0] - uv[2][0], du2 = uv[1][0] - uv[2][0];
    float dv1 = uv[0][1] - uv[2][1], dv2 = uv[1][1] - uv[2][1];
    V dn1 = vsub(n0, n2), dn2 = vsub(n1, n2);
    float determinant = du1 * dv2 - dv1 * du2;
    if (determinant == 0.f) dndu = dndv = v3(0, 0, 0);
    else {
        float invdet = 1.f / determinant;
        dndu = vmul(vsub(vmul(dn1, dv2), vmul(dn2, dv1)), invdet);
        dndv = vmul(vadd(vmul(dn1, -du2), vmul(dn2, du1)), invdet);
    }
    dg_init(dgs, dg.p, ss, ts, xnormal(nmat, dndu), xnormal(nmat, dndv), dg.u, dg.v, (flags & REC_FLIP) != 0);
}

PGD_INLINE bool quadratic(float A, float B, float C, float *t0, float *t1) {
    float discrim = B * B - 4.f * A * C;
    if (discrim <= 0.) return false;
    float rootDiscrim = sqrtf(discrim);
    float q;
    if (B < 0) q = -.5f * (B - rootDiscrim);
    else q = -.5f * (B + rootDiscrim);
    *t0 = q / A;
    *t1 = C / q;
    if (*t0 > *t1) { float tmp = *t0; *t0 = *t1; *t1 = tmp; }
    return true;
}
PGD_INLINE Ray to_object(const pbrtgpu_quadric &q, const Ray &r) {
    Ray o = r;
    const float *m = q.o2w_minv;
    V p = r.o;
    float x = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float y = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float z = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    o.o = v3(x, y, z);
    if (w != 1.) o.o = vdiv(o.o, w);
    o.d = xvec(m, r.d);
    return o;
}
// Sphere::Intersect (sphere.cpp:50-150)
// nnOnly: the caller uses only dg->nn (light sampling / pdf / MIS facing tests); nn is
// computed exactly as dg_init would, the rest of the differential geometry is skipped
PGD_INLINE bool sphere_intersect(const pbrtgpu_quadric &q, const Ray &r, float *tHit, float *rayEps, DG *dg,
                                 bool nnOnly = false) {
    float phi;
    V phit;
    Ray ray = to_object(q, r);
    float A = ray.d.x * ray.d.x + ray.d.y * ray.d.y + ray.d.z * ray.d.z;
    float B = 2 * (ray.d.x * ray.o.x + ray.d.y * ray.o.y + ray.d.z * ray.o.z);
    float C = ray.o.x * ray.o.x + ray.o.y * ray.o.y + ray.o.z * ray.o.z - q.radius * q.radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return false;
    if (t0 > ray.maxt || t1 < ray.mint) return false;
    float thit = t0;
    if (t0 < ray.mint) { thit = t1; if (thit > ray.maxt) return false; }
    // phi <= 2.f * kPi always (atan2 in [-pi, pi], + 2pi in float), so with phi_max >= that
    // bound the phi test cannot fail and a hit-only query (no dg) skips the atan2
    const bool needPhi = dg || !(q.phi_max >= 2.f * kPi);
    phit = rayat(ray, thit);
    if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * q.radius;
    phi = 0.f;
    if (needPhi) {
        phi = ATAN2F(phit.y, phit.x);
        if (phi < 0.) phi += 2.f * kPi;
    }
    if ((q.zmin > -q.radius && phit.z < q.zmin) || (q.zmax < q.radius && phit.z > q.zmax) || phi > q.phi_max) {
        if (thit == t1) return false;
        if (t1 > ray.maxt) return false;
        thit = t1;
        phit = rayat(ray, thit);
        if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * q.radius;
        if (needPhi) {
            phi = ATAN2F(phit.y, phit.x);
            if (phi < 0.) phi += 2.f * kPi;
        }
        if ((q.zmin > -q.radius && phit.z < q.zmin) || (q.zmax < q.radius && phit.z > q.zmax) || phi > q.phi_max)
            return false;
    }
    if (!dg) { *tHit = thit; return true; }
    if (nnOnly) {
        const float theta = ACOSF(clampf(phit.z / q.radius, -1.f, 1.f));
        const float zradius = sqrtf(phit.x * phit.x + phit.y * phit.y);
        const float invzradius = 1.f / zradius;
        const float cosphi = phit.x * invzradius, sinphi = phit.y * invzradius;
        const V dpdu = v3(-q.phi_max * phit.y, q.phi_max * phit.x, 0);
        const V dpdv = vmul(v3(phit.z * cosphi, phit.z * sinphi, -q.radius * SINF(theta)), q.theta_max - q.theta_min);
        dg->nn = vnorm(vcross(xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv)));
        if (q.reverse_orientation ^ q.swaps_handedness) dg->nn = vmul(dg->nn, -1.f);
        *tHit = thit;
        *rayEps = 5e-4f * *tHit;
        return true;
    }
    float u = phi / q.phi_max;
    float theta = ACOSF(clampf(phit.z / q.radius, -1.f, 1.f));
    float v = (theta - q.theta_min) / (q.theta_max - q.theta_min);
    float zradius = sqrtf(phit.x * phit.x + phit.y * phit.y);
    float invzradius = 1.f / zradius;
    float cosphi = phit.x * invzradius, sinphi = phit.y * invzradius;
    V dpdu = v3(-q.phi_max * phit.y, q.phi_max * phit.x, 0);
    V dpdv = vmul(v3(phit.z * cosphi, phit.z * sinphi, -q.radius * SINF(theta)), q.theta_max - q.theta_min);
    V d2Pduu = vmul(v3(phit.x, phit.y, 0), -q.phi_max * q.phi_max);
    V d2Pduv = vmul(v3(-sinphi, cosphi, 0.), (q.theta_max - q.theta_min) * phit.z * q.phi_max);
    V d2Pdvv = vmul(v3(phit.x, phit.y, phit.z), -(q.theta_max - q.theta_min) * (q.theta_max - q.theta_min));
    float E = vdot(dpdu, dpdu), F = vdot(dpdu, dpdv), G = vdot(dpdv, dpdv);
    V N = vnorm(vcross(dpdu, dpdv));
    float e = vdot(N, d2Pduu), f = vdot(N, d2Pduv), g = vdot(N, d2Pdvv);
    float invEGF2 = 1.f / (E * G - F * F);
    V dndu = vadd(vmul(dpdu, (f * F - e * G) * invEGF2), vmul(dpdv, (e * F - f * E) * invEGF2));
    V dndv = vadd(vmul(dpdu, (g * F - f * G) * invEGF2), vmul(dpdv, (f * F - g * E) * invEGF2));
    dg_init(*dg, xpoint(q.o2w_m, phit), xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv), xnormal(q.o2w_minv, dndu),
            xnormal(q.o2w_minv, dndv), u, v, q.reverse_orientation ^ q.swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return true;
}
// Disk::Intersect (disk.cpp:48-96)
PGD_INLINE bool disk_intersect(const pbrtgpu_quadric &q, const Ray &r, float *tHit, float *rayEps, DG *dg,
                               bool nnOnly = false) {
    Ray ray = to_object(q, r);
    if (fabsf(ray.d.z) < 1e-7) return false;
    float thit = (q.height - ray.o.z) / ray.d.z;
    if (thit < ray.mint || thit > ray.maxt) return false;
    V phit = rayat(ray, thit);
    float dist2 = phit.x * phit.x + phit.y * phit.y;
    if (dist2 > q.radius * q.radius || dist2 < q.inner_radius * q.inner_radius) return false;
    // phi <= (float)(2pi) always: with phi_max >= that bound the phi test cannot fail, and a
    // hit-only (or nn-only) query skips the atan2
    const bool phiFree = q.phi_max >= 2.f * kPi;
    if (!dg && phiFree) { *tHit = thit; return true; }
    if (nnOnly) {
        if (!phiFree) {
            float phi = ATAN2F(phit.y, phit.x);
            if (phi < 0) phi = (float)((double)phi + 2. * (double)kPi);
            if (phi > q.phi_max) return false;
        }
        const float oneMinusV = ((sqrtf(dist2) - q.inner_radius) / (q.radius - q.inner_radius));
        const float invOneMinusV = (oneMinusV > 0.f) ? (1.f / oneMinusV) : 0.f;
        V dpdu = v3(-q.phi_max * phit.y, q.phi_max * phit.x, 0.);
        V dpdv = v3(-phit.x * invOneMinusV, -phit.y * invOneMinusV, 0.);
        const float su = q.phi_max * kInvTwoPi;
        dpdu = v3(dpdu.x * su, dpdu.y * su, dpdu.z * su);
        const float sc = (q.radius - q.inner_radius) / q.radius;
        dpdv = v3(dpdv.x * sc, dpdv.y * sc, dpdv.z * sc);
        dg->nn = vnorm(vcross(xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv)));
        if (q.reverse_orientation ^ q.swaps_handedness) dg->nn = vmul(dg->nn, -1.f);
        *tHit = thit;
        *rayEps = 5e-4f * *tHit;
        return true;
    }
    float phi = ATAN2F(phit.y, phit.x);
    if (phi < 0) phi = (float)((double)phi + 2. * (double)kPi);
    if (phi > q.phi_max) return false;
    if (!dg) { *tHit = thit; return true; }
    float u = phi / q.phi_max;
    float oneMinusV = ((sqrtf(dist2) - q.inner_radius) / (q.radius - q.inner_radius));
    float invOneMinusV = (oneMinusV > 0.f) ? (1.f / oneMinusV) : 0.f;
    float v = 1.f - oneMinusV;
    V dpdu = v3(-q.phi_max * phit.y, q.phi_max * phit.x, 0.);
    V dpdv = v3(-phit.x * invOneMinusV, -phit.y * invOneMinusV, 0.);
    float su = q.phi_max * kInvTwoPi;
    dpdu = v3(dpdu.x * su, dpdu.y * su, dpdu.z * su);
    float sc = (q.radius - q.inner_radius) / q.radius;
    dpdv = v3(dpdv.x * sc, dpdv.y * sc, dpdv.z * sc);
    V zero = v3(0, 0, 0);
    dg_init(*dg, xpoint(q.o2w_m, phit), xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv), xnormal(q.o2w_minv, zero),
            xnormal(q.o2w_minv, zero), u, v, q.reverse_orientation ^ q.swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return true;
}
// Cylinder::Intersect / IntersectP (cylinder.cpp:48-176); nnOnly as for the sphere
PGD_INLINE bool cylinder_intersect(const pbrtgpu_quadric &q, const Ray &r, float *tHit, float *rayEps, DG *dg,
                                   bool nnOnly = false) {
    Ray ray = to_object(q, r);
    float A = ray.d.x * ray.d.x + ray.d.y * ray.d.y;
    float B = 2 * (ray.d.x * ray.o.x + ray.d.y * ray.o.y);
    float C = ray.o.x * ray.o.x + ray.o.y * ray.o.y - q.radius * q.radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return false;
    if (t0 > ray.maxt || t1 < ray.mint) return false;
    float thit = t0;
    if (t0 < ray.mint) { thit = t1; if (thit > ray.maxt) return false; }
    V phit = rayat(ray, thit);
    float phi = ATAN2F(phit.y, phit.x);
    if (phi < 0.) phi += 2.f * kPi;
    if (phit.z < q.zmin || phit.z > q.zmax || phi > q.phi_max) {
        if (thit == t1) return false;
        thit = t1;
        if (t1 > ray.maxt) return false;
        phit = rayat(ray, thit);
        phi = ATAN2F(phit.y, phit.x);
        if (phi < 0.) phi += 2.f * kPi;
        if (phit.z < q.zmin || phit.z > q.zmax || phi > q.phi_max) return false;
    }
    if (!dg) { *tHit = thit; return true; }
    const V dpdu = v3(-q.phi_max * phit.y, q.phi_max * phit.x, 0), dpdv = v3(0, 0, q.zmax - q.zmin);
    if (nnOnly) {
        dg->nn = vnorm(vcross(xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv)));
        if (q.reverse_orientation ^ q.swaps_handedness) dg->nn = vmul(dg->nn, -1.f);
        *tHit = thit;
        *rayEps = 5e-4f * *tHit;
        return true;
    }
    const float u = phi / q.phi_max, v = (phit.z - q.zmin) / (q.zmax - q.zmin);
    const V d2Pduu = vmul(v3(phit.x, phit.y, 0), -q.phi_max * q.phi_max), d2Pduv = v3(0, 0, 0), d2Pdvv = v3(0, 0, 0);
    const float E = vdot(dpdu, dpdu), F = vdot(dpdu, dpdv), G = vdot(dpdv, dpdv);
    const V N = vnorm(vcross(dpdu, dpdv));
    const float e = vdot(N, d2Pduu), f = vdot(N, d2Pduv), g = vdot(N, d2Pdvv);
    const float invEGF2 = 1.f / (E * G - F * F);
    const V dndu = vadd(vmul(dpdu, (f * F - e * G) * invEGF2), vmul(dpdv, (e * F - f * E) * invEGF2));
    const V dndv = vadd(vmul(dpdu, (g * F - f * G) * invEGF2), vmul(dpdv, (f * F - g * E) * invEGF2));
    dg_init(*dg, xpoint(q.o2w_m, phit), xvec(q.o2w_m, dpdu), xvec(q.o2w_m, dpdv), xnormal(q.o2w_minv, dndu),
            xnormal(q.o2w_minv, dndv), u, v, q.reverse_orientation ^ q.swaps_handedness);
    *tHit = thit;
    *rayEps = 5e-4f * *tHit;
    return true;
}
PGD_INLINE float shape_area(const DevScene &S, int type, int idx) {
    if (type == PBRTGPU_SHAPE_TRIANGLE) {
        const pbrtgpu_triangle t = (*sa(S.tris, (uint32_t)(idx)));
        V p1 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[0]))), p2 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[1]))), p3 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[2])));
        return 0.5f * vlen(vcross(vsub(p2, p1), vsub(p3, p1)));
    }
    const pbrtgpu_quadric &q = (*sa(S.quads, (uint32_t)(idx)));
    if (type == PBRTGPU_SHAPE_SPHERE) return q.phi_max * q.radius * (q.zmax - q.zmin);
    if (type == PBRTGPU_SHAPE_CYLINDER) return (q.zmax - q.zmin) * q.phi_max * q.radius;   // cylinder.cpp:180-182
    return q.phi_max * 0.5f * (q.radius * q.radius - q.inner_radius * q.inner_radius);
}
PGD_HEAVY bool shape_intersect(const DevScene &S, int type, int idx, const Ray &r, float *tHit, float *eps, DG *dg,
                               bool nnOnly = false) {
    if (type == PBRTGPU_SHAPE_TRIANGLE) return tri_intersect(S, idx, r, tHit, eps, dg);
    if (type == PBRTGPU_SHAPE_SPHERE) return sphere_intersect((*sa(S.quads, (uint32_t)(idx))), r, tHit, eps, dg, nnOnly);
    if (type == PBRTGPU_SHAPE_CYLINDER) return cylinder_intersect((*sa(S.quads, (uint32_t)(idx))), r, tHit, eps, dg, nnOnly);
    return disk_intersect((*sa(S.quads, (uint32_t)(idx))), r, tHit, eps, dg, nnOnly);
}

// ------------------------------------------------------------------ BVH traversal
// child references in the child-in-parent BVH: an interior child is its wide-node index,
// a leaf is WREF_LEAF | nPrims << 24 | first primitive
enum : uint32_t { WREF_LEAF = 0x80000000u, WREF_NP_SHIFT = 24, WREF_NP_MASK = 0x7fu, WREF_OFF_MASK = 0xffffffu };
// slab test (bvh.cpp:118-140); node = {bmin.xyz, bmax.x} {bmax.yz, offset, meta}
PGD_INLINE bool bbox_hit(float4 n0, float4 n1, const Ray &ray, V invDir, const int neg[3]) {
    float bminx = n0.x, bminy = n0.y, bminz = n0.z, bmaxx = n0.w, bmaxy = n1.x, bmaxz = n1.y;
    float tmin = ((neg[0] ? bmaxx : bminx) - ray.o.x) * invDir.x;
    float tmax = ((neg[0] ? bminx : bmaxx) - ray.o.x) * invDir.x;
    float tymin = ((neg[1] ? bmaxy : bminy) - ray.o.y) * invDir.y;
    float tymax = ((neg[1] ? bminy : bmaxy) - ray.o.y) * invDir.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = ((neg[2] ? bmaxz : bminz) - ray.o.z) * invDir.z;
    float tzmax = ((neg[2] ? bminz : bmaxz) - ray.o.z) * invDir.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return (tmin < ray.maxt) && (tmax > ray.mint);
}
// the same slab test with its parts split for a child box tested at its parent: returns
// whether the maxt-independent part passes (the slab intervals overlap and tmax > mint) and
// the entry distance tmin; the box is hit for a ray extent [mint, maxt] iff that holds and
// tmin < maxt, exactly as bbox_hit decides it
PGD_INLINE bool slab_enter(float4 lo, float4 hi, const Ray &ray, V invDir, const int neg[3], float *tEnter) {
    float tmin = ((neg[0] ? hi.x : lo.x) - ray.o.x) * invDir.x;
    float tmax = ((neg[0] ? lo.x : hi.x) - ray.o.x) * invDir.x;
    float tymin = ((neg[1] ? hi.y : lo.y) - ray.o.y) * invDir.y;
    float tymax = ((neg[1] ? lo.y : hi.y) - ray.o.y) * invDir.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = ((neg[2] ? hi.z : lo.z) - ray.o.z) * invDir.z;
    float tzmax = ((neg[2] ? lo.z : hi.z) - ray.o.z) * invDir.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    *tEnter = tmin;
    return tmax > ray.mint;
}
// slab_enter as one straight-line sequence (every plane distance computed, the early exits folded
// into the result): the same answer and, where it passes, the same entry distance.  In the 4-wide
// walks the four child tests then run as value selects rather than divergent branches under exec
// masks (the short-circuit && of four tests per node compiled to a branch each)
PGD_INLINE bool slab_enter_bf(float4 lo, float4 hi, const Ray &ray, V invDir, const int neg[3], float *tEnter) {
    float tmin = ((neg[0] ? hi.x : lo.x) - ray.o.x) * invDir.x;
    float tmax = ((neg[0] ? lo.x : hi.x) - ray.o.x) * invDir.x;
    const float tymin = ((neg[1] ? hi.y : lo.y) - ray.o.y) * invDir.y;
    const float tymax = ((neg[1] ? lo.y : hi.y) - ray.o.y) * invDir.y;
    const bool ok1 = !(tmin > tymax) & !(tymin > tmax);
    tmin = (tymin > tmin) ? tymin : tmin;
    tmax = (tymax < tmax) ? tymax : tmax;
    const float tzmin = ((neg[2] ? hi.z : lo.z) - ray.o.z) * invDir.z;
    const float tzmax = ((neg[2] ? lo.z : hi.z) - ray.o.z) * invDir.z;
    const bool ok2 = !(tmin > tzmax) & !(tzmin > tmax);
    tmin = (tzmin > tmin) ? tzmin : tmin;
    tmax = (tzmax < tmax) ? tzmax : tmax;
    *tEnter = tmin;
    return ok1 & ok2 & (tmax > ray.mint);
}
// LDS stack: column per lane
struct Stack {
    uint32_t *base;   // &lds[lane]: child refs
    float *tbase;     // &lds[depth * stride + lane]: entry distance of each pushed child (closest-hit only)
    int stride;       // threads per block
    // work counters; only the stats kernel reads them, elsewhere they are dead and removed
    uint32_t cRays = 0, cNodes = 0, cTris = 0, cQuads = 0, cHits = 0, cShadow = 0;
    PGD_INLINE void set(int i, uint32_t v) { base[i * stride] = v; }
    PGD_INLINE uint32_t get(int i) const { return base[i * stride]; }
    PGD_INLINE void setT(int i, float v) { tbase[i * stride] = v; }
    PGD_INLINE float getT(int i) const { return tbase[i * stride]; }
};
// quadric hit test kept out of line: its double-precision transcendentals would otherwise
// set the register budget of every traversal loop.  Scalars in, t out (-inf: miss), so
// the call passes everything in VGPRs and the traversal kernels need no private memory.
#ifndef PGD_QUAD_ATTR   // quadric hit test out of line (traversal register budget); experiments may inline it
#define PGD_QUAD_ATTR __attribute__((noinline))
#endif
// hit-only Sphere / Cylinder::IntersectP in one body (sphere.cpp:153-202, cylinder.cpp:113-176): the
// cylinder drops the z terms of A, B, C, the sphere's phit.x nudge and the sphere's "clipped at all"
// guards of its z tests; the operations and their order are each shape's own.  One body keeps the
// traversal kernels' registers where the sphere test alone put them (a separate cylinder test cost
// k_trace_c4 94 -> 103 VGPRs inlined, and scratch out of line)
PGD_INLINE bool sphere_cyl_hit(const pbrtgpu_quadric &q, const Ray &r, bool cyl, float *tHit) {
    Ray ray = to_object(q, r);
    const float dz2 = ray.d.z * ray.d.z, dozz = ray.d.z * ray.o.z, oz2 = ray.o.z * ray.o.z;
    const float A = cyl ? ray.d.x * ray.d.x + ray.d.y * ray.d.y : ray.d.x * ray.d.x + ray.d.y * ray.d.y + dz2;
    const float B = 2 * (cyl ? ray.d.x * ray.o.x + ray.d.y * ray.o.y : ray.d.x * ray.o.x + ray.d.y * ray.o.y + dozz);
    const float C = (cyl ? ray.o.x * ray.o.x + ray.o.y * ray.o.y : ray.o.x * ray.o.x + ray.o.y * ray.o.y + oz2) -
                    q.radius * q.radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return false;
    if (t0 > ray.maxt || t1 < ray.mint) return false;
    float thit = t0;
    if (t0 < ray.mint) { thit = t1; if (thit > ray.maxt) return false; }
    // phi <= 2.f * kPi always (atan2 in [-pi, pi], + 2pi in float): with phi_max >= that bound
    // the phi test cannot fail and the atan2 is skipped
    const bool needPhi = !(q.phi_max >= 2.f * kPi);
    const bool zLo = cyl || q.zmin > -q.radius, zHi = cyl || q.zmax < q.radius;
    for (int k = 0; k < 2; ++k) {
        V phit = rayat(ray, thit);
        if (!cyl && phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * q.radius;
        float phi = 0.f;
        if (needPhi) {
            phi = ATAN2F(phit.y, phit.x);
            if (phi < 0.) phi += 2.f * kPi;
        }
        if (!((zLo && phit.z < q.zmin) || (zHi && phit.z > q.zmax) || phi > q.phi_max)) { *tHit = thit; return true; }
        if (k == 1 || thit == t1 || t1 > ray.maxt) return false;
        thit = t1;
    }
    return false;
}
PGD_INLINE float quadric_hit_inl(const pbrtgpu_quadric *quads, int type, int idx, float ox, float oy, float oz, float dx,
                                 float dy, float dz, float mint, float maxt, float time) {
    Ray ray;
    ray.o = v3(ox, oy, oz); ray.d = v3(dx, dy, dz); ray.mint = mint; ray.maxt = maxt; ray.time = time;
    float t, e;
    const bool hit = type == PBRTGPU_SHAPE_DISK ? disk_intersect(quads[idx], ray, &t, &e, nullptr)
                                                : sphere_cyl_hit(quads[idx], ray, type == PBRTGPU_SHAPE_CYLINDER, &t);
    return hit ? t : -INFINITY;   // a hit has t >= mint >= 0 (or NaN)
}
__device__ PGD_QUAD_ATTR float quadric_hit(const pbrtgpu_quadric *quads, int type, int idx, float ox, float oy, float oz,
                                           float dx, float dy, float dz, float mint, float maxt, float time) {
    // the record through global loads (not flat), as whole float4s
    typedef float Q4 __attribute__((ext_vector_type(4)));
    static_assert(sizeof(pbrtgpu_quadric) % 16 == 0, "quadric records are whole float4s");
    constexpr int NW = (int)(sizeof(pbrtgpu_quadric) / 16);
    const PGD_GLOBAL_AS Q4 *src = (const PGD_GLOBAL_AS Q4 *)(quads + idx);
    Q4 w[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k) w[k] = src[k];
    pbrtgpu_quadric q;
    memcpy(&q, w, sizeof(q));
    return quadric_hit_inl(&q, type, 0, ox, oy, oz, dx, dy, dz, mint, maxt, time);
}
// INL: the persistent traversal kernels inline the hit-only test (fewer VGPRs than the call
// there); the shading kernel calls it (inlined, it costs k_shade registers)
template <bool INL = false>
PGD_INLINE bool quadric_test(const DevScene &S, int type, int idx, const Ray &r, float *t) {
    const float th = INL ? quadric_hit_inl(S.quads, type, idx, r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.mint, r.maxt, r.time)
                         : quadric_hit(S.quads, type, idx, r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, r.mint, r.maxt, r.time);
    *t = th;
    return th != -INFINITY;
}
PGD_INLINE bool prim_hit(const DevScene &S, Stack &st, int pi, const Ray &ray, float *t) {
    const DevTri tr = (*sa(S.primTri, (uint32_t)(pi)));
    if (__float_as_int(tr.a.w) == PBRTGPU_SHAPE_TRIANGLE) { st.cTris++; return tri_hit(tr, ray, t); }
    const pbrtgpu_prim pr = (*sa(S.prims, (uint32_t)(pi)));
    st.cQuads++;
    return quadric_test(S, pr.shape_type, pr.shape_index, ray, t);
}
// ---- Matrix4x4 / Quaternion / AnimatedTransform (transform.cpp, quaternion.cpp) for
// TransformedPrimitive instances
PGD_INLINE void m4_mul(const float *a, const float *b, float *r) {   // Matrix4x4::Mul
    float t[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            t[4 * i + j] = a[4 * i + 0] * b[j] + a[4 * i + 1] * b[4 + j] + a[4 * i + 2] * b[8 + j] + a[4 * i + 3] * b[12 + j];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = t[i];
}
PGD_INLINE void m4_identity(float *m) {
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f;
}
// transform.cpp:68-130, Gauss-Jordan with full pivoting
PGD_INLINE void m4_inverse(const float *m, float *out) {
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    float minv[16];
    for (int i = 0; i < 16; ++i) minv[i] = m[i];
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0.;
        for (int j = 0; j < 4; j++)
            if (ipiv[j] != 1)
                for (int k = 0; k < 4; k++)
                    if (ipiv[k] == 0 && fabsf(minv[4 * j + k]) >= big) { big = fabsf(minv[4 * j + k]); irow = j; icol = k; }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) { float t = minv[4 * irow + k]; minv[4 * irow + k] = minv[4 * icol + k]; minv[4 * icol + k] = t; }
        indxr[i] = irow;
        indxc[i] = icol;
        float pivinv = 1.f / minv[4 * icol + icol];
        minv[4 * icol + icol] = 1.f;
        for (int j = 0; j < 4; j++) minv[4 * icol + j] *= pivinv;
        for (int j = 0; j < 4; j++)
            if (j != icol) {
                float save = minv[4 * j + icol];
                minv[4 * j + icol] = 0;
                for (int k = 0; k < 4; k++) minv[4 * j + k] -= minv[4 * icol + k] * save;
            }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) {
                float t = minv[4 * k + indxr[j]]; minv[4 * k + indxr[j]] = minv[4 * k + indxc[j]]; minv[4 * k + indxc[j]] = t;
            }
    for (int i = 0; i < 16; ++i) out[i] = minv[i];
}
// m4_inverse of the scale factor S of an AnimatedTransform's decomposition.  Gauss-Jordan over
// dynamic pivot indices compiles to select chains over all 16 entries per access; when S is
// diagonal (every off-diagonal entry +0) with positive normal-range entries -- an animation
// without scaling has S = I -- every pivot is a diagonal entry (the first candidate of each step
// is one, an off-diagonal +0 never beats it, so no row is swapped), each row is scaled by its own
// 1/d, and the eliminations subtract +0 products: the result is diag(1/d) with +0 elsewhere, the
// general routine's bits (checked against it by the host replay, tests/test_hostsan.py)
PGD_INLINE void m4_inverse_scale(const float *S, float *out) {
    bool diag = true;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i % 5 == 0) diag = diag && S[i] >= 0x1p-100f && S[i] <= 0x1p100f;
        else diag = diag && __float_as_uint(S[i]) == 0u;
    }
    if (!diag) { m4_inverse(S, out); return; }
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1.f / S[i] : 0.f;
}
struct Quat { float x, y, z, w; };
PGD_INLINE float qdot(Quat a, Quat b) { return (a.x * b.x + a.y * b.y + a.z * b.z) + a.w * b.w; }
PGD_INLINE Quat qmk(float x, float y, float z, float w) { Quat q; q.x = x; q.y = y; q.z = z; q.w = w; return q; }
PGD_INLINE Quat qnormalize(Quat q) {
    float d = sqrtf(qdot(q, q));
    float inv = 1.f / d;
    return qmk(q.x * inv, q.y * inv, q.z * inv, q.w / d);
}
PGD_INLINE Quat qscale(Quat q, float f) { return qmk(q.x * f, q.y * f, q.z * f, q.w * f); }
PGD_INLINE Quat qadd(Quat a, Quat b) { return qmk(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
PGD_INLINE Quat qsub(Quat a, Quat b) { return qmk(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
PGD_INLINE Quat slerp(float t, Quat q1, Quat q2) {   // quaternion.cpp:39-49
    float cosTheta = qdot(q1, q2);
    if (cosTheta > .9995f) return qnormalize(qadd(qscale(q1, 1.f - t), qscale(q2, t)));
    float theta = ACOSF(clampf(cosTheta, -1.f, 1.f));
    float thetap = theta * t;
    Quat qperp = qnormalize(qsub(q2, qscale(q1, cosTheta)));
    const float2 sc = SINCOSF(thetap);
    return qadd(qscale(q1, sc.y), qscale(qperp, sc.x));
}
// AnimatedTransform::Interpolate (transform.cpp:356-381): world->primitive m (and mInv)
PGD_INLINE void inst_interp(const pbrtgpu_instance &I, float time, float *m, float *minv) {
    if (!I.animated || time <= I.start_time) {
        for (int i = 0; i < 16; ++i) m[i] = I.start_m[i];
        if (minv) for (int i = 0; i < 16; ++i) minv[i] = I.start_minv[i];
        return;
    }
    if (time >= I.end_time) {
        for (int i = 0; i < 16; ++i) m[i] = I.end_m[i];
        if (minv) for (int i = 0; i < 16; ++i) minv[i] = I.end_minv[i];
        return;
    }
    float dt = (time - I.start_time) / (I.end_time - I.start_time);
    float tr[3];
    for (int k = 0; k < 3; ++k) tr[k] = (1.f - dt) * I.T[0][k] + dt * I.T[1][k];
    Quat rot = slerp(dt, qmk(I.R[0][0], I.R[0][1], I.R[0][2], I.R[0][3]), qmk(I.R[1][0], I.R[1][1], I.R[1][2], I.R[1][3]));
    float Sm[16];
    m4_identity(Sm);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Sm[4 * i + j] = lerpf(dt, I.S[0][4 * i + j], I.S[1][4 * i + j]);
    // Quaternion::ToTransform: m = Transpose(M), mInv = M
    float xx = rot.x * rot.x, yy = rot.y * rot.y, zz = rot.z * rot.z;
    float xy = rot.x * rot.y, xz = rot.x * rot.z, yz = rot.y * rot.z;
    float wx = rot.x * rot.w, wy = rot.y * rot.w, wz = rot.z * rot.w;
    float M[16];
    m4_identity(M);
    M[0] = 1.f - 2.f * (yy + zz); M[1] = 2.f * (xy + wz); M[2] = 2.f * (xz - wy);
    M[4] = 2.f * (xy - wz); M[5] = 1.f - 2.f * (xx + zz); M[6] = 2.f * (yz + wx);
    M[8] = 2.f * (xz + wy); M[9] = 2.f * (yz - wx); M[10] = 1.f - 2.f * (xx + yy);
    float R[16], T[16], TR[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) R[4 * i + j] = M[4 * j + i];
    m4_identity(T); T[3] = tr[0]; T[7] = tr[1]; T[11] = tr[2];
    m4_mul(T, R, TR);   // Translate(trans) * rotate.ToTransform() * Transform(scale)
    m4_mul(TR, Sm, m);
    if (minv) {
        float Ti[16], Si[16], RiTi[16];
        m4_identity(Ti); Ti[3] = -tr[0]; Ti[7] = -tr[1]; Ti[11] = -tr[2];
        m4_inverse_scale(Sm, Si);
        m4_mul(M, Ti, RiTi);
        m4_mul(Si, RiTi, minv);
    }
}
PGD_INLINE Ray xray(const float *m, const Ray &r) {   // Transform::operator()(Ray)
    Ray o = r;
    o.o = xpoint(m, r.o);
    o.d = xvec(m, r.d);
    return o;
}
PGD_INLINE bool m4_is_identity(const float *m) {
    bool id = true;
    for (int i = 0; i < 16; ++i) id = id && (m[i] == ((i % 5 == 0) ? 1.f : 0.f));
    return id;
}

// BVHAccel::Intersect / IntersectP (bvh.cpp:380-481) from node `root`, LDS stack entries
// from `base`.  Closest hit: ray.maxt shrinks on every accepted hit.  With INST, prims of
// shape_type INSTANCE run TransformedPrimitive::Intersect/IntersectP (primitive.cpp:87-116):
// the ray is moved to primitive space at ray.time and the nested BVH is walked with the
// stack entries above this level's.
template <bool ANY, bool INST>
PGD_INLINE bool bvh_walk(const DevScene &S, Stack &st, int base, uint32_t root, Ray &ray, int *hitPrim, float *hitT);

template <bool ANY, bool INST>
PGD_INLINE bool prim_test(const DevScene &S, Stack &st, int base, int pi, Ray &ray, int *hitPrim, float *hitT) {
    // Any-hit walks read the shape type from the triangle record (DevTri a.w): one dependent load
    // per triangle test.  The closest walk reads the primitive record first: holding the triangle
    // record across the type test takes it past 96 VGPRs (4 waves/SIMD instead of 5)
    float t;
    DevTri tr;
    bool isTri;
    if constexpr (ANY) {
        tr = (*sa(S.primTri, (uint32_t)(pi)));
        isTri = __float_as_int(tr.a.w) == PBRTGPU_SHAPE_TRIANGLE;
    } else {
        isTri = (*sa(S.prims, (uint32_t)(pi))).shape_type == PBRTGPU_SHAPE_TRIANGLE;
        if (isTri) tr = (*sa(S.primTri, (uint32_t)(pi)));
    }
    if (isTri) {
        st.cTris++;
        if (!tri_hit(tr, ray, &t)) return false;
        if (!ANY) { ray.maxt = t; *hitPrim = pi; *hitT = t; }
        return true;
    }
    const pbrtgpu_prim pr = (*sa(S.prims, (uint32_t)(pi)));
    if (!INST || pr.shape_type != PBRTGPU_SHAPE_INSTANCE) {
        st.cQuads++;
        if (!quadric_test<true>(S, pr.shape_type, pr.shape_index, ray, &t)) return false;
    } else {
        if constexpr (INST) {
            const pbrtgpu_instance &I = (*sa(S.insts, (uint32_t)(pr.shape_index)));
            float m[16];
            inst_interp(I, ray.time, m, nullptr);
            Ray r = xray(m, ray);
            bool f;
            if (I.single_prim >= 0) f = prim_test<ANY, false>(S, st, base, I.single_prim, r, hitPrim, hitT);
            else f = bvh_walk<ANY, false>(S, st, base, (uint32_t)I.root, r, hitPrim, hitT);
            if (f && !ANY) ray.maxt = r.maxt;
            return f;
        }
        return false;
    }
    if (!ANY) { ray.maxt = t; *hitPrim = pi; *hitT = t; }
    return true;
}

// The walk runs on the child-in-parent copy of the BVH (DevScene::wnodes): one 64-byte
// record per interior node holds both children's boxes, so a visit tests both children
// at once.  Visiting order and culling are the reference's: the children are taken in its
// dirIsNeg[axis] order, a near child whose box passes is entered at once (bvh.cpp:417-425
// visits it next with the same maxt), and a pushed far child carries its entry distance,
// re-checked against the then-current maxt when popped -- the slab test's only
// maxt-dependent part (bbox_hit == slab_enter && tmin < maxt).  So the primitives tested,
// and their order, are identical to BVHAccel::Intersect / IntersectP.
template <bool ANY, bool INST>
PGD_INLINE bool bvh_walk(const DevScene &S, Stack &st, int base, uint32_t root, Ray &ray, int *hitPrim, float *hitT) {
    V invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    if (ANY) st.cShadow += INST ? 1u : 0u; else st.cRays += INST ? 1u : 0u;
    {
        const float4 n0 = (*sa(S.nodes, (uint32_t)(2 * root))), n1 = (*sa(S.nodes, (uint32_t)(2 * root + 1)));
        st.cNodes++;
        if (!bbox_hit(n0, n1, ray, invDir, neg)) return false;
    }
    int todo = base;
    uint32_t ref = (*sa(S.nodeRef, (uint32_t)(root)));
    bool found = false;
    for (;;) {
        if (ref & WREF_LEAF) {
            const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
            for (uint32_t i = 0; i < np; ++i)
                if (prim_test<ANY, INST>(S, st, todo, (int)(off + i), ray, hitPrim, hitT)) {
                    if (ANY) return true;
                    found = true;
                }
        } else {
            const float4 *w = sa(S.wnodes, (uint32_t)(4 * (size_t)ref));
            const float4 l0 = w[0], l1 = w[1], r0 = w[2], r1 = w[3];
            st.cNodes++;
            float tl = 0.f, tr = 0.f;
            const bool hl = slab_enter(l0, l1, ray, invDir, neg, &tl) && tl < ray.maxt;
            const bool hr = slab_enter(r0, r1, ray, invDir, neg, &tr) && tr < ray.maxt;
            const uint32_t refL = __float_as_uint(l0.w), refR = __float_as_uint(l1.w);
            // bvh.cpp:420-425: dirIsNeg[axis] -> second child first
            const bool swap = neg[__float_as_uint(r0.w)] != 0;
            const bool hn = swap ? hr : hl, hf = swap ? hl : hr;
            const uint32_t rn = swap ? refR : refL, rf = swap ? refL : refR;
            if (hn) {
                if (hf) {
                    st.set(todo, rf);
                    if (!ANY) st.setT(todo, swap ? tl : tr);
                    ++todo;
                }
                ref = rn;
                continue;
            }
            if (hf) { ref = rf; continue; }
        }
        // pop the next far child whose box is still entered before maxt
        for (;;) {
            if (todo == base) return found;
            --todo;
            ref = st.get(todo);
            if (ANY || st.getT(todo) < ray.maxt) break;
        }
    }
}
template <bool INST = true>
PGD_INLINE bool bvh_intersect(const DevScene &S, Stack &st, Ray &ray, int *hitPrim, float *hitT) {
    if (!INST) st.cRays++;
    bool f = bvh_walk<false, INST>(S, st, 0, 0u, ray, hitPrim, hitT);
    st.cHits += f ? 1u : 0u;
    return f;
}
template <bool INST = true>
PGD_INLINE bool bvh_intersectP(const DevScene &S, Stack &st, const Ray &ray) {
    if (!INST) st.cShadow++;
    Ray r = ray;
    int hp;
    float ht;
    return bvh_walk<true, INST>(S, st, 0, 0u, r, &hp, &ht);
}
// The binary walk's visiting order of a 4-wide node's slots (scene_build.h wide4_bvh): the near
// child's part first by the parent's split axis (bvh.cpp:420-425: dirIsNeg[axis] -> second child
// first), within each part the near grandchild first by that child's axis (a leaf child: its one
// slot, the empty one skipped).  negMask: dirIsNeg as bits; meta: the node's axes (2 bits each).
PGD_INLINE uint32_t w4_order(uint32_t meta, uint32_t negMask) {
    const uint32_t aP = meta & 3u, aA = (meta >> 2) & 3u, aB = (meta >> 4) & 3u;
    const uint32_t sP = (negMask >> aP) & 1u, sA = aA < 3u ? (negMask >> aA) & 1u : 0u, sB = aB < 3u ? (negMask >> aB) & 1u : 0u;
    const uint32_t a0 = sA, a1 = 1u - sA, b0 = 2u + sB, b1 = 3u - sB;
    // slot of position k in bits 2k..2k+1
    return sP ? (b0 | b1 << 2 | a0 << 4 | a1 << 6) : (a0 | a1 << 2 | b0 << 4 | b1 << 6);
}
// The closest-hit query on the 4-wide copy as one plain walk (host replay and tests; the GPU runs
// k_trace_c4): the root box, then per node the four child boxes in w4_order, the first passing
// child next and the others pushed (entry distances re-checked against maxt when popped) -- the
// primitives tested and their order are bvh_walk's.  st.base / st.tbase must hold S.w4Stack entries.
PGD_INLINE bool bvh_intersect4(const DevScene &S, Stack &st, Ray &ray, int *hitPrim, float *hitT) {
    const V invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    const int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    const uint32_t negMask = (uint32_t)neg[0] | ((uint32_t)neg[1] << 1) | ((uint32_t)neg[2] << 2);
    st.cRays++;
    if (!bbox_hit((*sa(S.nodes, 0u)), (*sa(S.nodes, 1u)), ray, invDir, neg)) return false;
    int todo = 0;
    bool found = false;
    uint32_t ref = 0u;
    for (;;) {
        if (ref & WREF_LEAF) {
            const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
            for (uint32_t i = 0; i < np; ++i)
                if (prim_test<false, false>(S, st, todo, (int)(off + i), ray, hitPrim, hitT)) found = true;
        } else {
            const float4 *w = sa(S.w4nodes, (uint32_t)(8 * (size_t)ref));
            const uint32_t ord = w4_order(__float_as_uint(w[1].w), negMask);
            uint32_t rs[4];
            float ts[4];
            bool hs[4];
            for (int k = 0; k < 4; ++k) {
                const int sl = (int)((ord >> (2 * k)) & 3u);
                rs[k] = __float_as_uint(w[2 * sl].w);
                ts[k] = 0.f;
                hs[k] = rs[k] != 0xffffffffu && slab_enter(w[2 * sl], w[2 * sl + 1], ray, invDir, neg, &ts[k]) &&
                        ts[k] < ray.maxt;
            }
            int first = 4;
            for (int k = 3; k >= 0; --k)
                if (hs[k]) first = k;
            for (int k = 3; k > first; --k)
                if (hs[k]) {
                    st.set(todo, rs[k]);
                    st.setT(todo, ts[k]);
                    ++todo;
                }
            if (first < 4) {
                ref = rs[first];
                continue;
            }
        }
        for (;;) {
            if (todo == 0) return found;
            --todo;
            ref = st.get(todo);
            if (st.getT(todo) < ray.maxt) break;
        }
    }
}
// The shadow query on the 4-wide BVH copy (scene_build.h wide4_bvh) as one plain walk: the root box,
// then per node the child boxes k_trace_s4 tests and the same leaves (host replay and tests; the
// GPU runs k_trace_s4).  st.base must hold S.w4Stack entries.
PGD_INLINE bool bvh_intersectP4(const DevScene &S, Stack &st, const Ray &ray0) {
    Ray ray = ray0;
    const V invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    const int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    if (!bbox_hit((*sa(S.nodes, 0u)), (*sa(S.nodes, 1u)), ray, invDir, neg)) return false;
    int todo = 0, prim = -1;
    float thit = INFINITY;
    st.set(todo++, 0u);
    while (todo > 0) {
        const uint32_t ref = st.get(--todo);
        if (ref & WREF_LEAF) {
            const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
            for (uint32_t i = 0; i < np; ++i)
                if (prim_test<true, false>(S, st, todo, (int)(off + i), ray, &prim, &thit)) return true;
            continue;
        }
        const float4 *w = sa(S.w4nodes, (uint32_t)(8 * (size_t)ref));
        for (int k = 0; k < 4; ++k) {
            const uint32_t r = __float_as_uint(w[2 * k].w);
            float t = 0.f;
            if (r != 0xffffffffu && slab_enter(w[2 * k], w[2 * k + 1], ray, invDir, neg, &t) && t < ray.maxt)
                st.set(todo++, r);
        }
    }
    return false;
}
// ---- the quantized 4-wide copy (scene_build.h quant_w4) for the shadow queries
// the stack entries of a quantized walk carry a "certain" bit: every box on the path to them passed
// its inner (contained) test, so the reference's exact walk reaches them too
enum : uint32_t { WQ_CERT = 0x40000000u };
// slot k's boxes of a quantized node: outer (containing the exact box) and inner (contained in it;
// empty -- lo > hi -- where the quantization has no step inside)
PGD_INLINE void wq_boxes(const uint4 &q0, const uint4 &q1, const uint4 &q2, const uint4 &q3, int k, float4 *olo,
                         float4 *ohi, float4 *ilo, float4 *ihi) {
    const uint32_t pk[6] = {q1.x, q1.y, q1.z, q1.w, q2.x, q2.y};
    const float o[3] = {__uint_as_float(q0.x), __uint_as_float(q0.y), __uint_as_float(q0.z)};
    float lo[3], hi[3], li[3], hj[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float sc = __uint_as_float(((q0.w >> (8 * a)) & 0xffu) << 23);   // 2^e
        const int bl = 6 * k + a, bh = 6 * k + 3 + a;
        const uint32_t ql = (pk[bl >> 2] >> (8 * (bl & 3))) & 0xffu, qh = (pk[bh >> 2] >> (8 * (bh & 3))) & 0xffu;
        const uint32_t el = (q3.z >> bl) & 1u, eh = (q3.z >> bh) & 1u;
        lo[a] = o[a] + (float)ql * sc;
        hi[a] = o[a] + (float)qh * sc;
        li[a] = el ? lo[a] : o[a] + (float)(ql + 1u) * sc;
        hj[a] = eh ? hi[a] : o[a] + (float)(qh - 1u) * sc;   // qh >= 1 wherever it is not exact (qh = 0 is exact)
    }
    *olo = make_float4(lo[0], lo[1], lo[2], 0.f);
    *ohi = make_float4(hi[0], hi[1], hi[2], 0.f);
    *ilo = make_float4(li[0], li[1], li[2], 0.f);
    *ihi = make_float4(hj[0], hj[1], hj[2], 0.f);
}
// BBox::IntersectP of the exact boxes of binary leaf `leaf`'s ancestors and itself, from the root
// (the nodes the reference's IntersectP tests on its way to the leaf: bvh.cpp:435-481), found by
// descending the depth-first node order (the right child of node i is nodes[i].offset, every node
// of i's left subtree below it)
PGD_INLINE bool leaf_reached(const DevScene &S, const Ray &ray, V invDir, const int neg[3], int leaf) {
    int i = 0;
    for (;;) {
        const float4 n0 = (*sa(S.nodes, (uint32_t)(2 * i))), n1 = (*sa(S.nodes, (uint32_t)(2 * i + 1)));
        if (!bbox_hit(n0, n1, ray, invDir, neg)) return false;
        if (i == leaf) return true;
        if (__float_as_uint(n1.w) & 0xffu) return false;   // another leaf: not an ancestor (corrupt leafOf)
        const int right = (int)__float_as_uint(n1.z);
        i = leaf >= right ? right : i + 1;
    }
}
// The shadow query on the quantized copy as one plain walk (host replay and tests; the GPU runs
// k_trace_s4q): outer boxes to descend, inner boxes to keep the "certain" bit, an uncertain leaf's
// hit confirmed by leaf_reached.  Same answer as bvh_intersectP (quant_w4).
PGD_INLINE bool bvh_intersectP4q(const DevScene &S, Stack &st, const Ray &ray0) {
    Ray ray = ray0;
    const V invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
    const int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
    if (!bbox_hit((*sa(S.nodes, 0u)), (*sa(S.nodes, 1u)), ray, invDir, neg)) return false;
    int todo = 0, prim = -1;
    float thit = INFINITY;
    st.set(todo++, 0u | WQ_CERT);   // the root box passed its exact test
    while (todo > 0) {
        const uint32_t e = st.get(--todo), ref = e & ~WQ_CERT;
        const bool cert = (e & WQ_CERT) != 0;
        if (ref & WREF_LEAF) {
            const uint32_t np = (ref >> WREF_NP_SHIFT) & 0x3fu, off = ref & WREF_OFF_MASK;
            for (uint32_t i = 0; i < np; ++i)
                if (prim_test<true, false>(S, st, todo, (int)(off + i), ray, &prim, &thit)) {
                    if (cert || leaf_reached(S, ray, invDir, neg, (*sa(S.leafOf, off)))) return true;
                    break;   // the reference never tests this leaf
                }
            continue;
        }
        const uint4 *q = sa(S.w4q, (uint32_t)(4 * (size_t)ref));
        const uint4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
        const uint32_t refs[4] = {q2.z, q2.w, q3.x, q3.y};
        for (int k = 0; k < 4; ++k) {
            if (refs[k] == 0xffffffffu) continue;
            float4 olo, ohi, ilo, ihi;
            wq_boxes(q0, q1, q2, q3, k, &olo, &ohi, &ilo, &ihi);
            float t = 0.f, ti = 0.f;
            if (slab_enter(olo, ohi, ray, invDir, neg, &t) && t < ray.maxt) {
                const bool c = cert && slab_enter(ilo, ihi, ray, invDir, neg, &ti) && ti < ray.maxt;
                st.set(todo++, refs[k] | (c ? WQ_CERT : 0u));
            }
        }
    }
    return false;
}
// im: the path's instance transforms (PathSoA::instM, per instance 8 float4: world->primitive
// m rows, then its inverse), or null in scenes without instances
// mat, al: the hit primitive's material and area light (its record, filled by isect_fill)
struct Isect { DG dg; float rayEps; int prim; int inst; float time; const float4 *im; int mat, al; };
// instance transforms of a path, computed once at path start (every ray of a path carries
// the camera sample's time, so AnimatedTransform::Interpolate gives the same matrices for all
// of them): m (and mInv) of instance i from the path's record
PGD_INLINE void inst_load(const float4 *im, int i, float *m, float *minv) {
    for (int k = 0; k < 4; ++k) {
        const float4 a = im[8 * i + k];
        m[4 * k] = a.x; m[4 * k + 1] = a.y; m[4 * k + 2] = a.z; m[4 * k + 3] = a.w;
        if (minv) {
            const float4 b = im[8 * i + 4 + k];
            minv[4 * k] = b.x; minv[4 * k + 1] = b.y; minv[4 * k + 2] = b.z; minv[4 * k + 3] = b.w;
        }
    }
}
PGD_HEAVY void isect_fill(const DevScene &S, const Ray &ray, int prim, float t, Isect &is, const float4 *im);
// geometric normal dg.nn of a recorded closest hit (the field isect_fill would produce)
PGD_INLINE V isect_nn(const DevScene &S, const Ray &ray, int prim, float t, const float4 *im) {
    if (!S.nInsts || (*sa(S.primInst, (uint32_t)(prim))) < 0) {
        const pbrtgpu_prim pr = (*sa(S.prims, (uint32_t)(prim)));
        Ray r = ray;
        r.maxt = t;
        float th, e;
        DG dg;
        shape_intersect(S, pr.shape_type, pr.shape_index, r, &th, &e, &dg, true);
        return dg.nn;
    }
    Isect is;
    isect_fill(S, ray, prim, t, is, im);
    return is.dg.nn;
}
// full intersection record for a recorded closest hit; primitives of a transformed instance
// are intersected in primitive space and moved to world space (primitive.cpp:94-110)
PGD_HEAVY void isect_fill(const DevScene &S, const Ray &ray, int prim, float t, Isect &is, const float4 *im) {
    const float4 *rec = prim_rec(S, prim);
    const int4 pr = rec_prim(rec);   // shape_type, shape_index, material, area_light
    Ray r = ray;
    r.maxt = t;
    float th;
    is.prim = prim;
    is.inst = -1;
    is.time = ray.time;
    is.im = im;
    is.mat = pr.z;
    is.al = pr.w;
    const int inst = S.nInsts ? (*sa(S.primInst, (uint32_t)(prim))) : -1;
#ifdef PGD_AB_NO_PRIMREC   // A/B timing build only: the triangle from the prim -> triangle -> vertex chain
    const bool useRec = false;
#else
    const bool useRec = true;
#endif
    if (inst < 0) {
        if (useRec && pr.x == PBRTGPU_SHAPE_TRIANGLE) tri_intersect_rec(rec, r, &th, &is.rayEps, &is.dg);
        else shape_intersect(S, pr.x, pr.y, r, &th, &is.rayEps, &is.dg);
        return;
    }
    float m[16], minv[16];
    inst_load(im, inst, m, minv);
    Ray ro = xray(m, r);
    if (useRec && pr.x == PBRTGPU_SHAPE_TRIANGLE) tri_intersect_rec(rec, ro, &th, &is.rayEps, &is.dg);
    else shape_intersect(S, pr.x, pr.y, ro, &th, &is.rayEps, &is.dg);
    if (m4_is_identity(m)) return;
    is.inst = inst;
    DG &g = is.dg;   // PrimitiveToWorld = Inverse(w2p): points/vectors with mInv, normals with m
    g.p = xpoint(minv, g.p);
    g.nn = vnorm(xnormal(m, g.nn));
    g.dpdu = xvec(minv, g.dpdu);
    g.dpdv = xvec(minv, g.dpdv);
    g.dndu = xnormal(m, g.dndu);
    g.dndv = xnormal(m, g.dndv);
}

// ------------------------------------------------------------------ BSDF
enum { BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16, BSDF_ALL = 31 };
enum { BX_LAMBERT, BX_OREN, BX_MICRO_BLINN_DIEL, BX_SPEC_REFL_NOOP, BX_FRESNEL_BLEND_ANISO, BX_MEASURED_IRREG,
       BX_MICRO_BLINN_COND, BX_SPEC_REFL_DIEL, BX_SPEC_TRANS,    // a = index of refraction for these two
       BX_MEASURED_HALF,                                          // RegularHalfangleBRDF: R = first texel
       BX_ANISOWARD,                                              // AnisoWardBrdf: R = Rs, a = Ax, b = Ay
       BX_SPEC_REFL_COND };                                       // SpecularReflection(1, FresnelConductor(R, 0))
// R, R2: offsets into DevScene::spectra, or -1 for the per-slot textured spectrum (K bands)
struct BxDF { int kind, type; int R, R2; float a, b; };
// the BxDF kinds a shading object compiles (FEAT_BASIC objects: the basic materials' kinds only)
PGD_INLINE bool bx_kind_on(int k) {
    if (PGD_NOSPEC_MATS) return k <= BX_MICRO_BLINN_DIEL || k == BX_FRESNEL_BLEND_ANISO || k == BX_MICRO_BLINN_COND;
    return !PGD_BASIC_MATS || k <= BX_MICRO_BLINN_DIEL || (PGD_BASIC_MEAS && (k == BX_MEASURED_IRREG || k == BX_MEASURED_HALF));
}
// eta: BSDF::eta, the glass material's index (glass.cpp:47-48), 1 otherwise (DirectLighting's
// SpecularTransmit differentials read it, integrator.cpp:219-247)
struct BSDF { V nn, ng, sn, tn; int n; BxDF bx[2]; float eta; };
PGD_INLINE bool matches(const BxDF &b, int flags) { return (b.type & flags) == b.type; }
PGD_INLINE V to_local(const BSDF &b, V v) { return v3(vdot(v, b.sn), vdot(v, b.tn), vdot(v, b.nn)); }
PGD_INLINE V to_world(const BSDF &b, V v) {
    return v3(b.sn.x * v.x + b.tn.x * v.y + b.nn.x * v.z, b.sn.y * v.x + b.tn.y * v.y + b.nn.y * v.z,
              b.sn.z * v.x + b.tn.z * v.y + b.nn.z * v.z);
}
PGD_INLINE float abscos(V w) { return fabsf(w.z); }
PGD_INLINE float sin2(V w) { return pmax(0.f, 1.f - w.z * w.z); }
PGD_INLINE float sinth(V w) { return sqrtf(sin2(w)); }
PGD_INLINE float cosphi(V w) { float s = sinth(w); if (s == 0.f) return 1.f; return clampf(w.x / s, -1.f, 1.f); }
PGD_INLINE float sinphi(V w) { float s = sinth(w); if (s == 0.f) return 0.f; return clampf(w.y / s, -1.f, 1.f); }
PGD_INLINE bool samehemi(V w, V wp) { return w.z * wp.z > 0.f; }
// FresnelDielectric(1.5, 1) + FrDiel (reflection.cpp:52-58, 112-127); equal in every band
PGD_INLINE float fr_dielectric(float cosi, float eta_i, float eta_t) {
    cosi = clampf(cosi, -1.f, 1.f);
    bool entering = cosi > 0.;
    float ei = eta_i, et = eta_t;
    if (!entering) { float t = ei; ei = et; et = t; }
    float sint = ei / et * sqrtf(pmax(0.f, 1.f - cosi * cosi));
    if (sint >= 1.) return 1.f;
    float cost = sqrtf(pmax(0.f, 1.f - sint * sint));
    float ci = fabsf(cosi);
    float Rparl = ((et * ci) - (ei * cost)) / ((et * ci) + (ei * cost));
    float Rperp = ((ei * ci) - (et * cost)) / ((ei * ci) + (et * cost));
    return (Rparl * Rparl + Rperp * Rperp) / 2.f;
}
// The microfacet distribution D(wh) and the matching pdf raise the same |cos theta_h| to the
// same exponent when BSDF::f and BSDF::Pdf (or Sample_f's other-component pdf) look at one
// (wo, wi); a one-entry memo per vertex returns the identical powf instead of recomputing it
struct PowMemo {
    uint32_t x = 0xffffffffu, e = 0xffffffffu;   // a NaN key: never matches
    float r = 0.f;
};
PGD_INLINE float dpow(PowMemo &m, float x, float e) {
    const uint32_t xb = __float_as_uint(x), eb = __float_as_uint(e);
    if (xb == m.x && eb == m.e) return m.r;
    const float r = POWF(x, e);
    m.x = xb; m.e = eb; m.r = r;
    return r;
}
PGD_INLINE float blinn_D(PowMemo &pm, float e, V wh) { return (e + 2) * kInvTwoPi * dpow(pm, abscos(wh), e); }
PGD_INLINE float micro_G(V wo, V wi, V wh) {
    float NdotWh = abscos(wh), NdotWo = abscos(wo), NdotWi = abscos(wi), WOdotWh = fabsf(vdot(wo, wh));
    return pmin(1.f, pmin((2.f * NdotWh * NdotWo / WOdotWh), (2.f * NdotWh * NdotWi / WOdotWh)));
}
PGD_INLINE float blinn_pdf(PowMemo &pm, float e, V wo, V wi) {
    V wh = vnorm(vadd(wo, wi));
    float costheta = abscos(wh);
    float p = ((e + 1.f) * dpow(pm, costheta, e)) / (2.f * kPi * 4.f * vdot(wo, wh));
    if (vdot(wo, wh) <= 0.f) p = 0.f;
    return p;
}
PGD_INLINE void blinn_sample(float e, V wo, V *wi, float u1, float u2, float *pdf) {
    float costheta = POWF(u1, 1.f / (e + 1));
    float sintheta = sqrtf(pmax(0.f, 1.f - costheta * costheta));
    float phi = u2 * 2.f * kPi;
    const float2 sc = SINCOSF(phi);
    V wh = v3(sintheta * sc.y, sintheta * sc.x, costheta);
    if (!samehemi(wo, wh)) wh = vneg(wh);
    *wi = vadd(vneg(wo), vmul(wh, 2.f * vdot(wo, wh)));
    float p = ((e + 1.f) * POWF(costheta, e)) / (2.f * kPi * 4.f * vdot(wo, wh));
    if (vdot(wo, wh) <= 0.f) p = 0.f;
    *pdf = p;
}
PGD_INLINE float aniso_D(PowMemo &pm, float ex, float ey, V wh) {
    float costhetah = abscos(wh);
    float d = 1.f - costhetah * costhetah;
    if (d == 0.f) return 0.f;
    float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / d;
    return sqrtf((ex + 2.f) * (ey + 2.f)) * kInvTwoPi * dpow(pm, costhetah, e);
}
PGD_INLINE float aniso_pdf(PowMemo &pm, float ex, float ey, V wo, V wi) {
    V wh = vnorm(vadd(wo, wi));
    float costhetah = abscos(wh);
    float ds = 1.f - costhetah * costhetah;
    float p = 0.f;
    if (ds > 0.f && vdot(wo, wh) > 0.f) {
        float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / ds;
        float d = sqrtf((ex + 1.f) * (ey + 1.f)) * kInvTwoPi * dpow(pm, costhetah, e);
        p = d / (4.f * vdot(wo, wh));
    }
    return p;
}
PGD_INLINE void aniso_first_quadrant(float ex, float ey, float u1, float u2, float *phi, float *costheta) {
    if (ex == ey) *phi = kPi * u1 * 0.5f;
    else *phi = ATANF(sqrtf((ex + 1.f) / (ey + 1.f)) * TANF(kPi * u1 * 0.5f));
    const float2 scp = SINCOSF(*phi);
    float cp = scp.y, sp = scp.x;
    *costheta = POWF(u2, 1.f / (ex * cp * cp + ey * sp * sp + 1));
}
PGD_INLINE void aniso_sample(float ex, float ey, V wo, V *wi, float u1, float u2, float *pdf) {
    float phi, costheta;
    if (u1 < .25f) aniso_first_quadrant(ex, ey, 4.f * u1, u2, &phi, &costheta);
    else if (u1 < .5f) { u1 = 4.f * (.5f - u1); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi = kPi - phi; }
    else if (u1 < .75f) { u1 = 4.f * (u1 - .5f); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi += kPi; }
    else { u1 = 4.f * (1.f - u1); aniso_first_quadrant(ex, ey, u1, u2, &phi, &costheta); phi = 2.f * kPi - phi; }
    float sintheta = sqrtf(pmax(0.f, 1.f - costheta * costheta));
    const float2 sc = SINCOSF(phi);
    V wh = v3(sintheta * sc.y, sintheta * sc.x, costheta);
    if (!samehemi(wo, wh)) wh = vneg(wh);
    *wi = vadd(vneg(wo), vmul(wh, 2.f * vdot(wo, wh)));
    float costhetah = abscos(wh);
    float ds = 1.f - costhetah * costhetah;
    float p = 0.f;
    if (ds > 0.f && vdot(wo, wh) > 0.f) {
        float e = (ex * wh.x * wh.x + ey * wh.y * wh.y) / ds;
        float d = sqrtf((ex + 1.f) * (ey + 1.f)) * kInvTwoPi * POWF(costhetah, e);
        p = d / (4.f * vdot(wo, wh));
    }
    *pdf = p;
}

// A BSDF value is a spectrum f_i(wo, wi).  Instead of materialising it as a float[NB]
// array, evaluation produces the per-direction scalars once (FTerm) and the spectrum is
// evaluated band by band where it is consumed (fval).  fval reproduces the reference's
// accumulation exactly: f = 0; for each matching BxDF: f += term_i  (reflection.cpp:
// 478-512), with every term's operand order as in BxDF::f (reflection.cpp, microfacet.h).
// T_MEAS: IrregIsotropicBRDF at BRDFRemap point (s0, s1, s2), kd-tree nodes [R, R + R2);
// once looked up (measured_prepare) it becomes T_BUF: the spectrum in the slot's scratch bands
// T_BLINNC: Microfacet with FresnelConductor, eta = R, k = R2, s2 = |cos theta_h|
// T_MERL: RegularHalfangleBRDF texel R + R2 of DevScene::merl, FromRGB'd into the slot's scratch
// bands (fval_prepare, like T_MEAS)
enum { T_ZERO = 0, T_LAMB, T_OREN, T_BLINN, T_FB, T_MEAS, T_BUF, T_BLINNC, T_MERL };
struct FTerm { int kind; int R, R2; float s0, s1, s2, s3; };
enum { FV_SUM = 0, FV_SPEC = 1, FV_SPEC_COND = 2 };
// FV_SPEC: a specular BxDF's sampled value (fs * R_i) / d (reflection.cpp:130-162)
// FV_SPEC_COND: SpecularReflection(1, FresnelConductor(eta = R, k = 0)): (FrCond(fs, eta_i, 0) * 1) / d
// The two terms are named members, not an array: any access through a runtime index (or an
// address the compiler selects between them) keeps the whole FVal in scratch memory, and the
// band loops then reload its terms from there (r03: 3 x 64 scratch loads in k_shade's band loops)
struct FVal { int mode, n; FTerm t0, t1; float d, fs; int R; };   // FV_SUM with n == 0: zero spectrum

PGD_INLINE void fval_zero(FVal &F) { F.mode = FV_SUM; F.n = 0; }
// Field by field, as value selects: `if (F.n == 0) F.t[0] = t; else F.t[1] = t;` was folded into
// a store through a selected address, a dynamic index that kept every FVal in scratch memory (and
// the band loops reloading its terms from there)
PGD_INLINE FTerm fterm_sel(bool c, const FTerm &a, const FTerm &b) {
    FTerm r;
    r.kind = c ? a.kind : b.kind; r.R = c ? a.R : b.R; r.R2 = c ? a.R2 : b.R2;
    r.s0 = c ? a.s0 : b.s0; r.s1 = c ? a.s1 : b.s1; r.s2 = c ? a.s2 : b.s2; r.s3 = c ? a.s3 : b.s3;
    return r;
}
PGD_INLINE void fval_push(FVal &F, const FTerm &t) {
    const bool first = F.n == 0;
    F.t1 = fterm_sel(first, F.t1, t);
    F.t0 = fterm_sel(first, t, F.t0);
    F.n++;
}

// BxDF::f(wo, wi) as a term (scalars per direction pair)
// BRDFRemap (reflection.cpp:239-248); pbrt.h:179 defines M_PI as a float literal
PGD_INLINE V brdf_remap(V wo, V wi) {
    float cosi = wi.z, coso = wo.z;
    float sini = sinth(wi), sino = sinth(wo);
    float pi_ = ATAN2F(wi.y, wi.x), po_ = ATAN2F(wo.y, wo.x);
    float phii = (pi_ < 0.f) ? pi_ + 2.f * kPi : pi_;   // SphericalPhi (geometry.h:647-650)
    float phio = (po_ < 0.f) ? po_ + 2.f * kPi : po_;
    float dphi = phii - phio;
    if (dphi < 0.) dphi += 2.f * kPi;
    if (dphi > 2.f * kPi) dphi -= 2.f * kPi;
    if (dphi > kPi) dphi = 2.f * kPi - dphi;
    return v3(sini * sino, dphi / kPi, cosi * coso);
}
PGD_INLINE int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }   // Clamp(int) (pbrt.h)
// RegularHalfangleBRDF::f (reflection.cpp:267-300) up to the table lookup: the texel index
// of (wo, wi) in the 90 x 90 x 180 (sqrt thetaH, thetaD, phiD) table, or -1 when wo + wi == 0
// (Spectrum(0.)).  M_PI is a float literal in this reference (pbrt.h:179); REMAP truncates
// V / MAX * COUNT to int and clamps to [0, COUNT - 1].
PGD_INLINE int halfangle_index(V WO, V WI) {
    V wo = WO, wi = WI, wh = vadd(wo, wi);
    if (wh.z < 0.f) { wo = vneg(wo); wi = vneg(wi); wh = vneg(wh); }
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return -1;
    wh = vnorm(wh);
    const float whTheta = ACOSF(clampf(wh.z, -1.f, 1.f));   // SphericalTheta
    const float whCosPhi = cosphi(wh), whSinPhi = sinphi(wh);
    const float whCosTheta = wh.z, whSinTheta = sinth(wh);
    const V whx = v3(whCosPhi * whCosTheta, whSinPhi * whCosTheta, -whSinTheta);
    const V why = v3(-whSinPhi, whCosPhi, 0.f);
    const V wd = v3(vdot(wi, whx), vdot(wi, why), vdot(wi, wh));
    const float wdTheta = ACOSF(clampf(wd.z, -1.f, 1.f));
    float wdPhi = ATAN2F(wd.y, wd.x);                        // SphericalPhi
    wdPhi = (wdPhi < 0.f) ? wdPhi + 2.f * kPi : wdPhi;
    if (wdPhi > kPi) wdPhi -= kPi;
    auto remap = [](float v, float mx, int count) { return clampi((int)(v / mx * (float)count), 0, count - 1); };
    const int whThetaIndex = remap(sqrtf(pmax(0.f, whTheta / (kPi / 2.f))), 1.f, 90);
    const int wdThetaIndex = remap(wdTheta, kPi / 2.f, 90);
    const int wdPhiIndex = remap(wdPhi, kPi, 180);
    return wdPhiIndex + 180 * (wdThetaIndex + whThetaIndex * 90);
}
PGD_INLINE FTerm bx_term(PowMemo &pm, const BxDF &b, V wo, V wi) {
    FTerm t;
    t.kind = T_ZERO; t.R = b.R; t.R2 = b.R2; t.s0 = t.s1 = t.s2 = t.s3 = 0.f;
    switch (bx_kind_on(b.kind) ? b.kind : -1) {
        case BX_LAMBERT: t.kind = T_LAMB; break;
        case BX_OREN: {
            float sinthetai = sinth(wi), sinthetao = sinth(wo);
            float maxcos = 0.f;
            if (sinthetai > 1e-4 && sinthetao > 1e-4) {
                float sinphii = sinphi(wi), cosphii = cosphi(wi), sinphio = sinphi(wo), cosphio = cosphi(wo);
                float dcos = cosphii * cosphio + sinphii * sinphio;
                maxcos = pmax(0.f, dcos);
            }
            float sinalpha, tanbeta;
            if (abscos(wi) > abscos(wo)) { sinalpha = sinthetao; tanbeta = sinthetai / abscos(wi); }
            else { sinalpha = sinthetai; tanbeta = sinthetao / abscos(wo); }
            t.kind = T_OREN;
            t.s0 = (b.a + b.b * maxcos * sinalpha * tanbeta);
            break;
        }
        case BX_MICRO_BLINN_DIEL:
        case BX_MICRO_BLINN_COND: {
            float cosThetaO = abscos(wo), cosThetaI = abscos(wi);
            if (cosThetaI == 0.f || cosThetaO == 0.f) break;
            V wh = vadd(wi, wo);
            if (wh.x == 0. && wh.y == 0. && wh.z == 0.) break;
            wh = vnorm(wh);
            float cosThetaH = vdot(wi, wh);
            if (b.kind == BX_MICRO_BLINN_DIEL) { t.kind = T_BLINN; t.s2 = fr_dielectric(cosThetaH, 1.5f, 1.f); }
            else { t.kind = T_BLINNC; t.s2 = fabsf(cosThetaH); }   // FresnelConductor::Evaluate
            t.s0 = blinn_D(pm, b.a, wh);
            t.s1 = micro_G(wo, wi, wh);
            t.s3 = 4.f * cosThetaI * cosThetaO;
            break;
        }
        case BX_FRESNEL_BLEND_ANISO: {
            float ta = (1.f - POWF(1.f - .5f * abscos(wi), 5)), tb = (1.f - POWF(1.f - .5f * abscos(wo), 5));
            V wh = vadd(wi, wo);
            if (wh.x == 0. && wh.y == 0. && wh.z == 0.) break;
            wh = vnorm(wh);
            float D = aniso_D(pm, b.a, b.b, wh);
            float den = (4.f * fabsf(vdot(wi, wh)) * pmax(abscos(wi), abscos(wo)));
            t.kind = T_FB;
            t.s0 = ta; t.s1 = tb;
            t.s2 = POWF(1 - vdot(wi, wh), 5.f);
            t.s3 = D / den;
            break;
        }
        case BX_MEASURED_IRREG: {
            V m = brdf_remap(wo, wi);
            t.kind = T_MEAS;
            t.s0 = m.x; t.s1 = m.y; t.s2 = m.z;
            break;
        }
        case BX_MEASURED_HALF: {
            const int idx = halfangle_index(wo, wi);
            if (idx >= 0) { t.kind = T_MERL; t.R2 = idx; }
            break;
        }
        case BX_ANISOWARD: {   // AnisoWardBrdf::f (AnisoWardBrdf.cpp:10-23): Rs * expTerm / (sqrt(cos cos) 4 pi Ax Ay)
            const V wh = vadd(wi, wo);
            if (wh.z == 0.f) break;
            float cc = wi.z * wo.z;
            if (cc <= 0.f) break;
            const float invAx2 = 1.0f / (b.a * b.a), invAy2 = 1.0f / (b.b * b.b);
            const float fourPiAxAy = (4.0f * kPi * b.a * b.b);
            const float expTerm = libmf_expf(-1.0f * (wh.x * wh.x * invAx2 + wh.y * wh.y * invAy2) / (wh.z * wh.z));
            cc = sqrtf(cc);
            // ((Rs * expTerm) * 1 * 1) / den: T_BLINN's band operation with unit G and F
            t.kind = T_BLINN;
            t.s0 = expTerm; t.s1 = 1.f; t.s2 = 1.f; t.s3 = cc * fourPiAxAy;
            break;
        }
        default: break;   // SpecularReflection::f == 0
    }
    return t;
}
PGD_INLINE float bx_pdf(PowMemo &pm, const BxDF &b, V wo, V wi) {
    switch (bx_kind_on(b.kind) ? b.kind : -1) {
        case BX_MICRO_BLINN_DIEL:
        case BX_MICRO_BLINN_COND: if (!samehemi(wo, wi)) return 0.f; return blinn_pdf(pm, b.a, wo, wi);
        case BX_SPEC_REFL_NOOP:
        case BX_SPEC_REFL_DIEL:
        case BX_SPEC_REFL_COND:
        case BX_SPEC_TRANS: return 0.;
        case BX_FRESNEL_BLEND_ANISO:
            if (!samehemi(wo, wi)) return 0.f;
            return .5f * (abscos(wi) * kInvPi + aniso_pdf(pm, b.a, b.b, wo, wi));
        default: return samehemi(wo, wi) ? abscos(wi) * kInvPi : 0.f;
    }
}
// the specular BxDFs' Sample_f (reflection.cpp SpecularReflection / SpecularTransmission::Sample_f)
PGD_INLINE void bx_sample_specular(const BxDF &b, V wo, V *wi, float *pdf, FVal &F) {
    switch ((PGD_BASIC_MATS || PGD_NOSPEC_MATS) ? -1 : b.kind) {
        case BX_SPEC_REFL_NOOP:    // SpecularReflection with FresnelNoOp: Spectrum(1) * R / |cos|
        case BX_SPEC_REFL_DIEL:    // ... with FresnelDielectric(1, ior)
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            F.mode = FV_SPEC; F.R = b.R; F.d = abscos(*wi);
            F.fs = b.kind == BX_SPEC_REFL_NOOP ? 1.f : fr_dielectric(wo.z, 1.f, b.a);
            return;
        case BX_SPEC_REFL_COND:    // ... with FresnelConductor(eta, 0): Evaluate(CosTheta(wo)) * 1 / |cos|
            *wi = v3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            F.mode = FV_SPEC_COND; F.R = b.R; F.d = abscos(*wi);
            F.fs = fabsf(wo.z);    // FresnelConductor::Evaluate takes |cosi| (reflection.cpp:102-104)
            return;
        case BX_SPEC_TRANS: {      // SpecularTransmission(T, 1, ior): (Spectrum(1) - F) * T / |cos|
            const bool entering = wo.z > 0.;
            float ei = 1.f, et = b.a;
            if (!entering) { float t = ei; ei = et; et = t; }
            const float sini2 = sin2(wo);
            const float eta = ei / et;
            const float sint2 = eta * eta * sini2;
            if (sint2 >= 1.) return;   // total internal reflection: pdf stays 0
            float cost = sqrtf(pmax(0.f, 1.f - sint2));
            if (entering) cost = -cost;
            const float sintOverSini = eta;
            *wi = v3(sintOverSini * -wo.x, sintOverSini * -wo.y, cost);
            *pdf = 1.f;
            F.mode = FV_SPEC; F.R = b.R; F.d = abscos(*wi);
            F.fs = 1.f - fr_dielectric(wo.z, 1.f, b.a);
            return;
        }
        default: return;
    }
}
// BxDF::Sample_f: direction + pdf; f as a one-term sum (or the specular spectrum)
PGD_INLINE void bx_sample_f(PowMemo &pm, const BxDF &b, V wo, V *wi, float u1, float u2, float *pdf, FVal &F) {
    fval_zero(F);
    switch (bx_kind_on(b.kind) ? b.kind : -1) {
        case BX_MICRO_BLINN_DIEL:
        case BX_MICRO_BLINN_COND:
            blinn_sample(b.a, wo, wi, u1, u2, pdf);
            if (!samehemi(wo, *wi)) return;
            F.n = 1; F.t0 = bx_term(pm, b, wo, *wi);
            return;
        case BX_SPEC_REFL_NOOP:
        case BX_SPEC_REFL_DIEL:
        case BX_SPEC_REFL_COND:
        case BX_SPEC_TRANS:
            bx_sample_specular(b, wo, wi, pdf, F);
            return;
        case BX_FRESNEL_BLEND_ANISO:
            if (u1 < .5) {
                u1 = 2.f * u1;
                *wi = cosine_hemisphere(u1, u2);
                if (wo.z < 0.) wi->z *= -1.f;
            } else {
                u1 = 2.f * (u1 - .5f);
                aniso_sample(b.a, b.b, wo, wi, u1, u2, pdf);
                if (!samehemi(wo, *wi)) return;
            }
            *pdf = bx_pdf(pm, b, wo, *wi);
            F.n = 1; F.t0 = bx_term(pm, b, wo, *wi);
            return;
        default:
            *wi = cosine_hemisphere(u1, u2);
            if (wo.z < 0.) wi->z *= -1.f;
            *pdf = bx_pdf(pm, b, wo, *wi);
            F.n = 1; F.t0 = bx_term(pm, b, wo, *wi);
            return;
    }
}
// BSDF::f (reflection.cpp:478-494)
PGD_INLINE void bsdf_f(PowMemo &pm, const BSDF &bs, V woW, V wiW, int flags, FVal &F) {
    V wi = to_local(bs, wiW), wo = to_local(bs, woW);
    if (vdot(wiW, bs.ng) * vdot(woW, bs.ng) > 0) flags &= ~BSDF_TRANSMISSION;
    else flags &= ~BSDF_REFLECTION;
    fval_zero(F);
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (k < bs.n && matches(bs.bx[k], flags)) fval_push(F, bx_term(pm, bs.bx[k], wo, wi));
}
PGD_INLINE float bsdf_pdf(PowMemo &pm, const BSDF &bs, V woW, V wiW, int flags) {
    if (bs.n == 0.) return 0.;
    V wo = to_local(bs, woW), wi = to_local(bs, wiW);
    float pdf = 0.f;
    int m = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (k < bs.n && matches(bs.bx[k], flags)) { ++m; pdf += bx_pdf(pm, bs.bx[k], wo, wi); }
    return m > 0 ? pdf / m : 0.f;
}
// BSDF::Sample_f (reflection.cpp:514-568)
// BSDF::Sample_f (reflection.cpp:555-611) in two steps: bsdf_sample_dir picks the component
// and samples the direction (pdf of that component, F of a specular one); bsdf_sample_rest
// adds the other matching components' pdfs and, for a non-specular sample, the BSDF value.
// Callers that may discard the direction (the MIS ray, mis_may_reach) run the second step
// only when they keep it; bsdf_sample_f runs both.
struct BSDFSampleState { int sel, matching; V wo, wi; };
PGD_HEAVY bool bsdf_sample_dir(PowMemo &pm, const BSDF &bs, V woW, V *wiW, float u0, float u1, float uc, float *pdf,
                               int flags, int *sampledType, FVal &F, BSDFSampleState &st) {
    int matching = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) if (k < bs.n && matches(bs.bx[k], flags)) ++matching;
    if (matching == 0) {
        *pdf = 0.f; *sampledType = 0;
        fval_zero(F);
        return false;
    }
    int which = (int)floorf(uc * matching);
    if (which > matching - 1) which = matching - 1;
    int sel = -1, count = which;
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (sel < 0 && k < bs.n && matches(bs.bx[k], flags) && count-- == 0) sel = k;
    const BxDF bx = sel == 0 ? bs.bx[0] : bs.bx[1];
    V wo = to_local(bs, woW), wi;
    *pdf = 0.f;
    bx_sample_f(pm, bx, wo, &wi, u0, u1, pdf, F);
    if (*pdf == 0.f) {
        *sampledType = 0;
        fval_zero(F);
        return false;
    }
    *sampledType = bx.type;
    *wiW = to_world(bs, wi);
    st.sel = sel; st.matching = matching; st.wo = wo; st.wi = wi;
    return true;
}
PGD_HEAVY void bsdf_sample_rest(PowMemo &pm, const BSDF &bs, V woW, V wiW, const BSDFSampleState &st, float *pdf,
                                int flags, int sampledType, FVal &F) {
    const int sel = st.sel, matching = st.matching;
    const V wo = st.wo, wi = st.wi;
    if (!(sampledType & BSDF_SPECULAR) && matching > 1)
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (k < bs.n && k != sel && matches(bs.bx[k], flags)) *pdf += bx_pdf(pm, bs.bx[k], wo, wi);
    if (matching > 1) *pdf /= matching;
    if (!(sampledType & BSDF_SPECULAR)) {
        fval_zero(F);
        if (vdot(wiW, bs.ng) * vdot(woW, bs.ng) > 0) flags &= ~BSDF_TRANSMISSION;
        else flags &= ~BSDF_REFLECTION;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (k < bs.n && matches(bs.bx[k], flags)) fval_push(F, bx_term(pm, bs.bx[k], wo, wi));
    }
}
PGD_INLINE void bsdf_sample_f(PowMemo &pm, const BSDF &bs, V woW, V *wiW, float u0, float u1, float uc, float *pdf,
                              int flags, int *sampledType, FVal &F) {
    BSDFSampleState st;
    if (bsdf_sample_dir(pm, bs, woW, wiW, u0, u1, uc, pdf, flags, sampledType, F, st))
        bsdf_sample_rest(pm, bs, woW, *wiW, st, pdf, flags, *sampledType, F);
}
// BSDF::Sample_f for flags that select specular BxDFs only (SpecularReflect / SpecularTransmit,
// integrator.cpp:169-250): bsdf_sample_f's arithmetic for the components such flags can match
// (the microfacet / diffuse cases compiled out).  pdf 0: nothing sampled (wi not set).
PGD_INLINE void bsdf_sample_specular(const BSDF &bs, V woW, V *wiW, float uc, float *pdf, int flags, FVal &F) {
    int matching = 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) if (k < bs.n && matches(bs.bx[k], flags)) ++matching;
    fval_zero(F);
    *pdf = 0.f;
    if (matching == 0) return;
    int which = (int)floorf(uc * matching);
    if (which > matching - 1) which = matching - 1;
    int sel = -1, count = which;
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (sel < 0 && k < bs.n && matches(bs.bx[k], flags) && count-- == 0) sel = k;
    const BxDF bx = sel == 0 ? bs.bx[0] : bs.bx[1];
    const V wo = to_local(bs, woW);
    V wi;
    bx_sample_specular(bx, wo, &wi, pdf, F);
    if (*pdf == 0.f) { fval_zero(F); return; }
    *wiW = to_world(bs, wi);
    if (matching > 1) *pdf /= matching;   // a specular sample adds no other pdfs (bsdf_sample_rest)
}


// ------------------------------------------------------------------ RGB spectra and textures
// SampledSpectrum::FromRGB (spectrum.cpp:93-178) for band quad q: the branch picks three basis
// spectra and weights; every band is r = ((0 + B0*a0) + B1*a1) + B2*a2, then *0.94 / *0.86445
// and Clamp(0, inf), exactly the reference's per-band operation sequence.  The RGB build
// (S.nb == 3) is RGBSpectrum::FromRGB (rgb.h): the triple itself, no basis, scale or clamp (k0 < 0)
struct RGBPick { int k0, k1, k2; float a0, a1, a2; };
PGD_INLINE RGBPick rgb_pick(const DevScene &S, const float rgb[3]) {
    enum { W = 0, Cy, Mg, Ye, Rd, Gr, Bl };
    RGBPick p;
    if (S.nb == 3) {
        p.k0 = p.k1 = p.k2 = -1; p.a0 = rgb[0]; p.a1 = rgb[1]; p.a2 = rgb[2];
    } else if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        p.k0 = W; p.a0 = rgb[0];
        if (rgb[1] <= rgb[2]) { p.k1 = Cy; p.a1 = rgb[1] - rgb[0]; p.k2 = Bl; p.a2 = rgb[2] - rgb[1]; }
        else { p.k1 = Cy; p.a1 = rgb[2] - rgb[0]; p.k2 = Gr; p.a2 = rgb[1] - rgb[2]; }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        p.k0 = W; p.a0 = rgb[1];
        if (rgb[0] <= rgb[2]) { p.k1 = Mg; p.a1 = rgb[0] - rgb[1]; p.k2 = Bl; p.a2 = rgb[2] - rgb[0]; }
        else { p.k1 = Mg; p.a1 = rgb[2] - rgb[1]; p.k2 = Rd; p.a2 = rgb[0] - rgb[2]; }
    } else {
        p.k0 = W; p.a0 = rgb[2];
        if (rgb[0] <= rgb[1]) { p.k1 = Ye; p.a1 = rgb[0] - rgb[2]; p.k2 = Gr; p.a2 = rgb[1] - rgb[0]; }
        else { p.k1 = Ye; p.a1 = rgb[1] - rgb[2]; p.k2 = Rd; p.a2 = rgb[0] - rgb[1]; }
    }
    return p;
}
PGD_INLINE float4 from_rgb4(const DevScene &S, const RGBPick &p, bool illum, int q) {
    if (p.k0 < 0) return make_float4(p.a0, p.a1, p.a2, 0.f);
    const float *b = sa(S.basis, (uint32_t)((illum ? 7 : 0) * S.nbp + 4 * q));
    const float4 x = *reinterpret_cast<const float4 *>(b + p.k0 * S.nbp);
    const float4 y = *reinterpret_cast<const float4 *>(b + p.k1 * S.nbp);
    const float4 z = *reinterpret_cast<const float4 *>(b + p.k2 * S.nbp);
    const float sc = illum ? .86445f : (float).94;
    float4 r;
    r.x = clampf((((0.f + x.x * p.a0) + y.x * p.a1) + z.x * p.a2) * sc, 0.f, INFINITY);
    r.y = clampf((((0.f + x.y * p.a0) + y.y * p.a1) + z.y * p.a2) * sc, 0.f, INFINITY);
    r.z = clampf((((0.f + x.z * p.a0) + y.z * p.a1) + z.z * p.a2) * sc, 0.f, INFINITY);
    r.w = clampf((((0.f + x.w * p.a0) + y.w * p.a1) + z.w * p.a2) * sc, 0.f, INFINITY);
    return r;
}

// The environment light's one-texel MIPMap (mipmap.h): Texel with wrap (:197-222), triangle
// (:263-274).  NC = 3 (RGB) or 1 (float).
PGD_INLINE float log2_(float x) { float invLog2 = 1.f / LOGF(2.f); return LOGF(x) * invLog2; }   // pbrt.h:243-246
PGD_INLINE float texel_c(const float *T, int wrap, int s, int t, int k) {
    if (wrap == PBRTGPU_WRAP_BLACK && (s != 0 || t != 0)) return 0.f;
    return T[k];
}
template <int NC>
PGD_INLINE void mip_triangle(const float *T, int wrap, float s, float t, float *out) {
    s = s * 1.f - 0.5f;
    t = t * 1.f - 0.5f;
    int s0 = (int)floorf(s), t0 = (int)floorf(t);
    float ds = s - s0, dt = t - t0;
    float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
#pragma unroll
    for (int k = 0; k < NC; ++k)
        out[k] = ((w00 * texel_c(T, wrap, s0, t0, k) + w01 * texel_c(T, wrap, s0, t0 + 1, k)) +
                  w10 * texel_c(T, wrap, s0 + 1, t0, k)) + w11 * texel_c(T, wrap, s0 + 1, t0 + 1, k);
}
// MIPMap (mipmap.h:119-375) of an IMAGE texture: its pyramid in S.texels from texel_off,
// level l max(1, width >> l) x max(1, height >> l) texels of NC floats (3: RGB, 1: float)
struct MipLv { const float *T; int w, h; };
template <int NC>
PGD_INLINE MipLv mip_lv(const DevScene &S, const pbrtgpu_texture &tx, int l) {
    uint32_t off = (uint32_t)tx.texel_off;
    int w = tx.width, h = tx.height;
    for (int i = 0; i < l; ++i) {
        off += (uint32_t)(w * h * NC);
        w = w > 1 ? w >> 1 : 1;
        h = h > 1 ? h >> 1 : 1;
    }
    MipLv r;
    r.T = S.texels + off; r.w = w; r.h = h;
    return r;
}
PGD_INLINE int mod_i(int a, int b) { int n = int(a / b); a -= n * b; if (a < 0) a += b; return a; }   // pbrt.h Mod
// Texel(level, s, t) with the wrap mode (mipmap.h:197-222)
template <int NC>
PGD_INLINE void mip_texel(const MipLv &L, int wrap, int s, int t, float *out) {
    if (wrap == PBRTGPU_WRAP_REPEAT) { s = mod_i(s, L.w); t = mod_i(t, L.h); }
    else if (wrap == PBRTGPU_WRAP_CLAMP) { s = clampi(s, 0, L.w - 1); t = clampi(t, 0, L.h - 1); }
    else if (s < 0 || s >= L.w || t < 0 || t >= L.h) {
#pragma unroll
        for (int k = 0; k < NC; ++k) out[k] = 0.f;
        return;
    }
    const float *p = L.T + (size_t)(t * L.w + s) * NC;
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = p[k];
}
// MIPMap::triangle (mipmap.h:263-274)
template <int NC>
PGD_INLINE void mip_tri(const DevScene &S, const pbrtgpu_texture &tx, int level, float s, float t, float *out) {
    level = clampi(level, 0, tx.levels - 1);
    const MipLv L = mip_lv<NC>(S, tx, level);
    s = s * (float)(uint32_t)L.w - 0.5f;
    t = t * (float)(uint32_t)L.h - 0.5f;
    const int s0 = (int)floorf(s), t0 = (int)floorf(t);
    const float ds = s - s0, dt = t - t0;
    const float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
    float a[NC], b[NC], c[NC], d[NC];
    mip_texel<NC>(L, tx.wrap, s0, t0, a);
    mip_texel<NC>(L, tx.wrap, s0, t0 + 1, b);
    mip_texel<NC>(L, tx.wrap, s0 + 1, t0, c);
    mip_texel<NC>(L, tx.wrap, s0 + 1, t0 + 1, d);
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = ((w00 * a[k] + w01 * b[k]) + w10 * c[k]) + w11 * d[k];
}
// MIPMap::EWA (mipmap.h:320-375)
template <int NC>
PGD_INLINE void mip_ewa(const DevScene &S, const pbrtgpu_texture &tx, int level, float s, float t, float ds0, float dt0,
                        float ds1, float dt1, float *out) {
    if (level >= tx.levels) {
        mip_texel<NC>(mip_lv<NC>(S, tx, tx.levels - 1), tx.wrap, 0, 0, out);
        return;
    }
    const MipLv L = mip_lv<NC>(S, tx, level);
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
    float sum[NC], sumWts = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) sum[k] = 0.f;
    for (int it = t0; it <= t1; ++it) {
        float tt = it - t;
        for (int is = s0; is <= s1; ++is) {
            float ss = is - s;
            float r2 = A * ss * ss + B * ss * tt + C * tt * tt;
            if (r2 < 1.) {
                int li = (int)(r2 * 128);
                float weight = (*sa(S.ewa, (uint32_t)(li < 127 ? li : 127)));
                float tv[NC];
                mip_texel<NC>(L, tx.wrap, is, it, tv);
#pragma unroll
                for (int k = 0; k < NC; ++k) sum[k] += tv[k] * weight;
                sumWts += weight;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = sum[k] / sumWts;
}
// MIPMap::Lookup(s, t, width) (mipmap.h:226-259), with the fork's noFiltering nearest texel
template <int NC>
PGD_INLINE void mip_lookup_w(const DevScene &S, const pbrtgpu_texture &tx, float s, float t, float width, float *out) {
    if (tx.nofilter) {
        const MipLv L = mip_lv<NC>(S, tx, 0);
        s = s * (float)(uint32_t)L.w - 0.5f;
        t = t * (float)(uint32_t)L.h - 0.5f;
        mip_texel<NC>(L, tx.wrap, (int)floorf(s + 0.5f), (int)floorf(t + 0.5f), out);   // Round2Int
        return;
    }
    const float level = (float)(uint32_t)(tx.levels - 1) + log2_(pmax(width, 1e-8f));
    if (level < 0) mip_tri<NC>(S, tx, 0, s, t, out);
    else if (level >= (float)(uint32_t)(tx.levels - 1)) mip_texel<NC>(mip_lv<NC>(S, tx, tx.levels - 1), tx.wrap, 0, 0, out);
    else {
        const int iLevel = (int)floorf(level);
        const float delta = level - iLevel;
        float a[NC], b[NC];
        mip_tri<NC>(S, tx, iLevel, s, t, a);
        mip_tri<NC>(S, tx, iLevel + 1, s, t, b);
#pragma unroll
        for (int k = 0; k < NC; ++k) out[k] = (1.f - delta) * a[k] + delta * b[k];
    }
}
// MIPMap::Lookup(s, t, ds0, dt0, ds1, dt1) (mipmap.h:278-318)
template <int NC>
PGD_INLINE void mip_lookup(const DevScene &S, const pbrtgpu_texture &tx, float s, float t, float ds0, float dt0,
                           float ds1, float dt1, float *out) {
    if (tx.trilinear) {
        mip_lookup_w<NC>(S, tx, s, t, 2.f * pmax(pmax(fabsf(ds0), fabsf(dt0)), pmax(fabsf(ds1), fabsf(dt1))), out);
        return;
    }
    if (ds0 * ds0 + dt0 * dt0 < ds1 * ds1 + dt1 * dt1) {
        float a = ds0; ds0 = ds1; ds1 = a;
        a = dt0; dt0 = dt1; dt1 = a;
    }
    float majorLength = sqrtf(ds0 * ds0 + dt0 * dt0);
    float minorLength = sqrtf(ds1 * ds1 + dt1 * dt1);
    if (minorLength * tx.max_aniso < majorLength && minorLength > 0.f) {
        float scale = majorLength / (minorLength * tx.max_aniso);
        ds1 *= scale; dt1 *= scale; minorLength *= scale;
    }
    if (minorLength == 0.f) { mip_tri<NC>(S, tx, 0, s, t, out); return; }
    float lod = pmax(0.f, (float)(uint32_t)tx.levels - 1.f + log2_(minorLength));
    int ilod = (int)floorf(lod);
    float d = lod - (float)(uint32_t)ilod;
    float e0[NC], e1[NC];
    mip_ewa<NC>(S, tx, ilod, s, t, ds0, dt0, ds1, dt1, e0);
    mip_ewa<NC>(S, tx, ilod + 1, s, t, ds0, dt0, ds1, dt1, e1);
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = (1.f - d) * e0[k] + d * e1[k];
}
// hit position in texture space with its screen-space derivatives, and the world-space point with
// its ray-differential offsets (dpdx, dpdy) for the non-uv mappings
struct TexPt { float u, v, dudx, dvdx, dudy, dvdy; V p, dpdx, dpdy; };
// SphericalMapping2D::sphere / CylindricalMapping2D::cylinder (texture.cpp:104-110, texture.h):
// the direction of the point in texture space (pbrt.h:176-179 makes M_PI a float)
PGD_INLINE void map_dir(const pbrtgpu_texture &tx, V p, float *s, float *t) {
    const V vec = vnorm(xpoint(tx.map, p));
    if (tx.mapping == PBRTGPU_MAP_SPHERICAL) {
        const float theta = ACOSF(clampf(vec.z, -1.f, 1.f));
        const float pp = ATAN2F(vec.y, vec.x);
        const float phi = (pp < 0.f) ? pp + 2.f * kPi : pp;
        *s = theta * kInvPi;
        *t = phi * kInvTwoPi;
    } else {
        *s = (kPi + ATAN2F(vec.y, vec.x)) / (2.f * kPi);
        *t = vec.z;
    }
}
// TextureMapping2D::Map (texture.cpp:80-150): (s, t) and their screen-space derivatives
PGD_INLINE void tex_map(const pbrtgpu_texture &tx, const TexPt &q, float *s, float *t, float *dsdx, float *dtdx,
                        float *dsdy, float *dtdy) {
    if (tx.mapping == PBRTGPU_MAP_UV) {   // UVMapping2D
        *s = tx.su * q.u + tx.du; *t = tx.sv * q.v + tx.dv;
        *dsdx = tx.su * q.dudx; *dtdx = tx.sv * q.dvdx; *dsdy = tx.su * q.dudy; *dtdy = tx.sv * q.dvdy;
    } else if (tx.mapping == PBRTGPU_MAP_PLANAR) {   // PlanarMapping2D
        const V vs = v3(tx.map[0], tx.map[1], tx.map[2]), vt = v3(tx.map[3], tx.map[4], tx.map[5]);
        *s = tx.du + vdot(q.p, vs); *t = tx.dv + vdot(q.p, vt);
        *dsdx = vdot(q.dpdx, vs); *dtdx = vdot(q.dpdx, vt); *dsdy = vdot(q.dpdy, vs); *dtdy = vdot(q.dpdy, vt);
    } else {   // spherical (delta .1) / cylindrical (delta .01): forward differences
        const float delta = tx.mapping == PBRTGPU_MAP_SPHERICAL ? .1f : .01f;
        float sx, tx_, sy, ty;
        map_dir(tx, q.p, s, t);
        map_dir(tx, vadd(q.p, vmul(q.dpdx, delta)), &sx, &tx_);
        *dsdx = (sx - *s) / delta;
        *dtdx = (tx_ - *t) / delta;
        if (*dtdx > .5f) *dtdx = 1.f - *dtdx;
        else if (*dtdx < -.5f) *dtdx = -(*dtdx + 1.f);
        map_dir(tx, vadd(q.p, vmul(q.dpdy, delta)), &sy, &ty);
        *dsdy = (sy - *s) / delta;
        *dtdy = (ty - *t) / delta;
        if (*dtdy > .5f) *dtdy = 1.f - *dtdy;
        else if (*dtdy < -.5f) *dtdy = -(*dtdy + 1.f);
    }
}
// ImageTexture::Evaluate (imagemap.cpp:84-101): the mapping, then the MIPMap lookup
template <int NC>
PGD_INLINE void tex_image(const DevScene &S, const pbrtgpu_texture &tx, const TexPt &q, float *out) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    mip_lookup<NC>(S, tx, s, t, dsdx, dtdx, dsdy, dtdy, out);
}
// the RGB of a spectrum leaf before FromRGB: an image map's MIPMap lookup, or UVTexture's
// (s - Floor2Int(s), t - Floor2Int(t), 0) (uv.h:38-44)
PGD_INLINE void leaf_rgb(const DevScene &S, const pbrtgpu_texture &tx, const TexPt &q, float rgb[3]) {
    if (tx.type == PBRTGPU_TEX_UV) {
        float s, t, dsdx, dtdx, dsdy, dtdy;
        tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
        rgb[0] = s - (float)(int)floorf(s);
        rgb[1] = t - (float)(int)floorf(t);
        rgb[2] = 0.f;
    } else tex_image<3>(S, tx, q, rgb);
}
PGD_HEAVY float tex_noise_leaf(const pbrtgpu_texture &tx, const TexPt &q);
PGD_INLINE float tex_leaf_float(const DevScene &S, int id, const TexPt &q) {
    const pbrtgpu_texture &tx = (*sa(S.tex, (uint32_t)(id)));
    if (tx.type == PBRTGPU_TEX_CONST) return tx.value;
    if (tx.type >= PBRTGPU_TEX_FBM && tx.type <= PBRTGPU_TEX_WINDY) return tex_noise_leaf(tx, q);
    float v;
    tex_image<1>(S, tx, q, &v);
    return v;
}
PGD_HEAVY float noise3(V P);
// DotsTexture::Evaluate (dots.h:47-66) without its operands: 1 = tex2 (insideDot: the "outside"
// parameter, as the reference's constructor stores them), 0 = tex1
PGD_INLINE int dots_pick(const pbrtgpu_texture &tx, const TexPt &q) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    const int sCell = (int)floorf(s + .5f), tCell = (int)floorf(t + .5f);
    if (noise3(v3(sCell + .5f, tCell + .5f, .5f)) > 0) {
        const float radius = .35f, maxShift = 0.5f - radius;
        const float sCenter = sCell + maxShift * noise3(v3(sCell + 1.5f, tCell + 2.8f, .5f));
        const float tCenter = tCell + maxShift * noise3(v3(sCell + 4.5f, tCell + 9.8f, .5f));
        const float ds = s - sCenter, dt = t - tCenter;
        if (ds * ds + dt * dt < radius * radius) return 1;
    }
    return 0;
}
// Checkerboard2DTexture::Evaluate (checkerboard.h:84-125) without its operands: 0 = tex1 alone,
// 1 = tex2 alone, 2 = (1 - area2) * tex1 + area2 * tex2 (*area2 set)
PGD_INLINE int checker_pick(const pbrtgpu_texture &tx, const TexPt &q, float *area2) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    const int point = ((int)floorf(s) + (int)floorf(t)) % 2 == 0 ? 0 : 1;   // Floor2Int
    if (tx.aamode == 1) return point;
    const float ds = pmax(fabsf(dsdx), fabsf(dsdy)), dt = pmax(fabsf(dtdx), fabsf(dtdy));   // std::max
    const float s0 = s - ds, s1 = s + ds, t0 = t - dt, t1 = t + dt;
    if ((int)floorf(s0) == (int)floorf(s1) && (int)floorf(t0) == (int)floorf(t1)) return point;
    // BUMPINT(x) = Floor2Int(x / 2) + 2 * max(x / 2 - Floor2Int(x / 2) - .5, 0)
    auto bumpint = [](float x) {
        const int f = (int)floorf(x / 2);
        return (float)f + 2.f * pmax((x / 2) - (float)f - .5f, 0.f);
    };
    const float sint = (bumpint(s1) - bumpint(s0)) / (2.f * ds);
    const float tint = (bumpint(t1) - bumpint(t0)) / (2.f * dt);
    float a = sint + tint - 2.f * sint * tint;
    if (ds > 1.f || dt > 1.f) a = .5f;
    *area2 = a;
    return 2;
}
// Texture<float>: CONST, IMAGE, ScaleTexture, Checkerboard2DTexture or MixTexture of leaves (the
// front end guarantees the depth); the leaves are looked up in one loop (one copy of the MIPMap
// lookup code per call site)
// Perlin noise (texture.cpp:163-250): NoisePerm, Grad, NoiseWeight, Noise, FBm, Turbulence
__constant__ int pgd_noise_perm[512] = {
#include "pbrt_noise_perm.inc"
};
PGD_INLINE float noise_grad(int x, int y, int z, float dx, float dy, float dz) {
    int h = pgd_noise_perm[pgd_noise_perm[pgd_noise_perm[x] + y] + z];
    h &= 15;
    const float u = h < 8 || h == 12 || h == 13 ? dx : dy;
    const float v = h < 4 || h == 12 || h == 13 ? dy : dz;
    return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}
PGD_INLINE float noise_weight(float t) {
    const float t3 = t * t * t, t4 = t3 * t;
    return 6.f * t4 * t - 15.f * t4 + 10.f * t3;
}
PGD_HEAVY float noise3(V P) {
    int ix = (int)floorf(P.x), iy = (int)floorf(P.y), iz = (int)floorf(P.z);
    const float dx = P.x - ix, dy = P.y - iy, dz = P.z - iz;
    ix &= 255; iy &= 255; iz &= 255;
    const float w000 = noise_grad(ix, iy, iz, dx, dy, dz), w100 = noise_grad(ix + 1, iy, iz, dx - 1, dy, dz);
    const float w010 = noise_grad(ix, iy + 1, iz, dx, dy - 1, dz), w110 = noise_grad(ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    const float w001 = noise_grad(ix, iy, iz + 1, dx, dy, dz - 1), w101 = noise_grad(ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    const float w011 = noise_grad(ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    const float w111 = noise_grad(ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    const float wx = noise_weight(dx), wy = noise_weight(dy), wz = noise_weight(dz);
    const float x00 = lerpf(wx, w000, w100), x10 = lerpf(wx, w010, w110), x01 = lerpf(wx, w001, w101),
                x11 = lerpf(wx, w011, w111);
    const float y0 = lerpf(wy, x00, x10), y1 = lerpf(wy, x01, x11);
    return lerpf(wz, y0, y1);
}
// FBm (turb = false) / Turbulence (turb = true), texture.cpp:214-250
PGD_HEAVY float fbm_turb(V P, V dpdx, V dpdy, float omega, int maxOctaves, bool turb) {
    const float s2 = pmax(vlen2(dpdx), vlen2(dpdy));
    const float foctaves = pmin((float)maxOctaves, 1.f - .5f * log2_(s2));
    const int octaves = (int)floorf(foctaves);
    float sum = 0.f, lambda = 1.f, o = 1.f;
    for (int i = 0; i < octaves; ++i) {
        const float n = noise3(vmul(P, lambda));
        sum += o * (turb ? fabsf(n) : n);
        lambda *= 1.99f;
        o *= omega;
    }
    const float partialOctave = foctaves - octaves;
    const float v = clampf((partialOctave - .3f) / (.7f - .3f), 0.f, 1.f);   // SmoothStep(.3, .7, x)
    const float n = noise3(vmul(P, lambda));
    sum += o * (v * v * (-2.f * v + 3.f)) * (turb ? fabsf(n) : n);
    if (turb) sum += (maxOctaves - foctaves) * 0.2f;
    return sum;
}
// FBmTexture / WrinkledTexture / WindyTexture::Evaluate (fbm.h, wrinkled.h, windy.h) with
// IdentityMapping3D::Map (texture.cpp:155-160: tex2world applied to p, dpdx, dpdy)
PGD_INLINE float tex_noise(const pbrtgpu_texture &tx, const TexPt &q) {
    const V P = xpoint(tx.map, q.p), dpdx = xvec(tx.map, q.dpdx), dpdy = xvec(tx.map, q.dpdy);
    if (tx.type == PBRTGPU_TEX_WINDY) {
        const float windStrength = fbm_turb(vmul(P, .1f), vmul(dpdx, .1f), vmul(dpdy, .1f), .5f, 3, false);
        const float waveHeight = fbm_turb(P, dpdx, dpdy, .5f, 6, false);
        return fabsf(windStrength) * waveHeight;
    }
    if (tx.type == PBRTGPU_TEX_MARBLE) {   // MarbleTexture::Evaluate (marble.h:45-49): its spline parameter t
        const float sc = tx.su;
        const V Ps = vmul(P, sc);
        const float marble = Ps.y + tx.sv * fbm_turb(Ps, vmul(dpdx, sc), vmul(dpdy, sc), tx.value, tx.levels, false);
        return .5f + .5f * SINF(marble);
    }
    return fbm_turb(P, dpdx, dpdy, tx.value, tx.levels, tx.type == PBRTGPU_TEX_WRINKLED);
}
PGD_HEAVY float tex_noise_leaf(const pbrtgpu_texture &tx, const TexPt &q) { return tex_noise(tx, q); }
// BilerpTexture's weights (bilerp.h:38-44): (1-s)(1-t), (1-s)t, s(1-t), st
PGD_INLINE void bilerp_w(const pbrtgpu_texture &tx, const TexPt &q, float w[4]) {
    float s, t, dsdx, dtdx, dsdy, dtdy;
    tex_map(tx, q, &s, &t, &dsdx, &dtdx, &dsdy, &dtdy);
    w[0] = (1.f - s) * (1.f - t); w[1] = (1.f - s) * t; w[2] = s * (1.f - t); w[3] = s * t;
}
PGD_HEAVY float tex_float(const DevScene &S, int id, const TexPt &q) {
    const pbrtgpu_texture &tx = (*sa(S.tex, (uint32_t)(id)));
    if (tx.type == PBRTGPU_TEX_BILERP) {
        float w[4];
        bilerp_w(tx, q, w);
        const float *v = sa(S.texels, (uint32_t)tx.texel_off);
        return ((w[0] * v[0] + w[1] * v[1]) + w[2] * v[2]) + w[3] * v[3];
    }
    int l0 = id, l1 = -1, l2 = -1;
    float a2 = 0.f;
    int kind = 0;   // 0 the leaf, 1 product, 2 checker blend, 3 mix
    if (tx.type == PBRTGPU_TEX_CHECKER) {
        const int k = checker_pick(tx, q, &a2);
        if (k < 2) l0 = k == 0 ? tx.tex1 : tx.tex2;
        else { l0 = tx.tex1; l1 = tx.tex2; kind = 2; }
    } else if (tx.type == PBRTGPU_TEX_DOTS) l0 = dots_pick(tx, q) ? tx.tex2 : tx.tex1; else if (tx.type == PBRTGPU_TEX_MIX) { l0 = tx.amount; l1 = tx.tex1; l2 = tx.tex2; kind = 3; }
    else if (tx.type == PBRTGPU_TEX_SCALE) { l0 = tx.tex1; l1 = tx.tex2; kind = 1; }
    float v0 = 0.f, v1 = 0.f, v2 = 0.f;
#pragma unroll 1
    for (int l = 0; l < 3; ++l) {
        const int lid = l == 0 ? l0 : (l == 1 ? l1 : l2);
        if (lid < 0) break;
        const float v = tex_leaf_float(S, lid, q);
        if (l == 0) v0 = v; else if (l == 1) v1 = v; else v2 = v;
    }
    if (kind == 1) return v0 * v1;                            // ScaleTexture: tex1 * tex2
    if (kind == 2) return (1.f - a2) * v0 + a2 * v1;           // checkerboard.h:120-121
    if (kind == 3) return (1.f - v0) * v1 + v0 * v2;           // mix.h:38-43 (v0 = amount)
    return v0;
}
// Texture<Spectrum> in device form: FromRGB(image lookup) [times a constant spectrum, in the
// ScaleTexture operand order]; SpecTex carries the per-hit part, spec4 evaluates a band quad
// A Checkerboard2DTexture becomes one of its leaves (CONST: constOnly) or a blend of both: the
// second leaf in pick2 / constOff2 and the weights w1 = 1 - area2, w2 = area2 (blend)
// (a BilerpTexture: its four spectra from constOff at one spectrum's stride, weights in w1, w2, w3, w4)
// (a spectrum noise texture, Spectrum(value) of its float: every band w1, uniform)
// (a MarbleTexture: the spline's four colours from constOff at one spectrum's stride, t in w1)
struct SpecTex { RGBPick pick; int constOff; bool constFirst, constOnly, blend, bilerp, uniform, marble; RGBPick pick2; int constOff2; float w1, w2, w3, w4; };
// one leaf of a checkerboard (CONST or IMAGE) into pick / constOff (constant: constOff >= 0)
PGD_INLINE void spec_leaf(const DevScene &S, int id, const TexPt &q, RGBPick *pick, int *constOff) {
    const pbrtgpu_texture &lf = (*sa(S.tex, (uint32_t)(id)));
    if (lf.type == PBRTGPU_TEX_CONST) { *constOff = lf.spec; pick->k0 = pick->k1 = pick->k2 = -1; pick->a0 = pick->a1 = pick->a2 = 0.f; return; }
    float rgb[3];
    leaf_rgb(S, lf, q, rgb);
    *pick = rgb_pick(S, rgb);
    *constOff = -1;
}
PGD_HEAVY SpecTex tex_spec_prepare(const DevScene &S, int id, const TexPt &q) {
    SpecTex r;
    r.constOff = -1; r.constFirst = false; r.constOnly = false; r.blend = false; r.bilerp = false; r.uniform = false;
    r.marble = false; r.constOff2 = -1;
    r.w1 = r.w2 = r.w3 = r.w4 = 0.f;
    const pbrtgpu_texture &tx = (*sa(S.tex, (uint32_t)(id)));
    if (tx.type >= PBRTGPU_TEX_FBM && tx.type <= PBRTGPU_TEX_WINDY) {   // T(FBm(...)) for T = Spectrum
        r.uniform = true;
        r.w1 = tex_noise_leaf(tx, q);
        return r;
    }
    if (tx.type == PBRTGPU_TEX_MARBLE) {   // marble.h:50-57: the segment (Floor2Int(t * NSEG)) and its t
        const float t6 = tex_noise_leaf(tx, q) * 6.f;
        // first is 0..6 in the reference; 6 (t == 1) reads one colour past its table -- 5 with t = 1
        // gives the same colour (c[6] == c[8]) without that read; NaN takes segment 0
        const float ff = floorf(t6);
        const int first = ff >= 5.f ? 5 : (ff >= 0.f ? (int)ff : 0);
        r.marble = true; r.constOff = tx.spec + first * S.nbp; r.w1 = t6 - (float)first;
        return r;
    }
    if (tx.type == PBRTGPU_TEX_BILERP) {
        float w[4];
        bilerp_w(tx, q, w);
        r.bilerp = true; r.constOff = tx.spec; r.w1 = w[0]; r.w2 = w[1]; r.w3 = w[2]; r.w4 = w[3];
        return r;
    }
    // the leaves to look up (one copy of the lookup code below): leaf[0], and leaf[1] for a blend
    int leaf0 = id, leaf1 = -1;
    const bool two = tx.type == PBRTGPU_TEX_MIX || tx.type == PBRTGPU_TEX_CHECKER || tx.type == PBRTGPU_TEX_DOTS;   // leaves: CONST / IMAGE / UV
    if (tx.type == PBRTGPU_TEX_MIX) {   // MixTexture::Evaluate: always the blend (mix.h:38-43)
        const float amt = tex_leaf_float(S, tx.amount, q);
        leaf0 = tx.tex1; leaf1 = tx.tex2;
        r.blend = true; r.w1 = 1.f - amt; r.w2 = amt;
    } else if (tx.type == PBRTGPU_TEX_CHECKER) {
        float a2 = 0.f;
        const int k = checker_pick(tx, q, &a2);
        leaf0 = k == 1 ? tx.tex2 : tx.tex1;
        if (k == 2) { leaf1 = tx.tex2; r.blend = true; r.w1 = 1.f - a2; r.w2 = a2; }
    } else if (tx.type == PBRTGPU_TEX_DOTS) {
        leaf0 = dots_pick(tx, q) ? tx.tex2 : tx.tex1;
    } else if (tx.type == PBRTGPU_TEX_SCALE) {   // one image / uv leaf times a constant spectrum
        const bool firstConst = (*sa(S.tex, (uint32_t)(tx.tex1))).type == PBRTGPU_TEX_CONST;
        leaf0 = firstConst ? tx.tex2 : tx.tex1;
        r.constOff = (*sa(S.tex, (uint32_t)(firstConst ? tx.tex1 : tx.tex2))).spec;
        r.constFirst = firstConst;
    }
#pragma unroll 1
    for (int l = 0; l < 2; ++l) {
        const int lid = l == 0 ? leaf0 : leaf1;
        if (lid < 0) break;
        RGBPick p;
        int co;
        spec_leaf(S, lid, q, &p, &co);
        if (l == 0) {
            r.pick = p;
            if (two) { r.constOff = co; r.constOnly = co >= 0; }
        } else { r.pick2 = p; r.constOff2 = co; }
    }
    return r;
}
PGD_INLINE float4 tex_spec4(const DevScene &S, const SpecTex &t, int q) {
    if (t.uniform) return make_float4(t.w1, t.w1, t.w1, t.w1);
    if (t.marble) {   // de Casteljau over c0..c3 (marble.h:58-66), per band, then * 1.5
        const uint32_t st = (uint32_t)S.nbp;
        const float tt = t.w1, u = 1.f - tt;
        float r[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float c0 = *sa(S.spectra, (uint32_t)(t.constOff + 4 * q + b));
            const float c1 = *sa(S.spectra, (uint32_t)(t.constOff + st + 4 * q + b));
            const float c2 = *sa(S.spectra, (uint32_t)(t.constOff + 2 * st + 4 * q + b));
            const float c3 = *sa(S.spectra, (uint32_t)(t.constOff + 3 * st + 4 * q + b));
            float s0 = c0 * u + c1 * tt, s1 = c1 * u + c2 * tt;
            const float s2 = c2 * u + c3 * tt;
            s0 = s0 * u + s1 * tt;
            s1 = s1 * u + s2 * tt;
            r[b] = (s0 * u + s1 * tt) * 1.5f;
        }
        return make_float4(r[0], r[1], r[2], r[3]);
    }
    if (t.bilerp) {   // ((v00 w00 + v01 w01) + v10 w10) + v11 w11 per band (Spectrum * float: c * w)
        const uint32_t st = (uint32_t)S.nbp;
        const float4 a = *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + 4 * q)));
        const float4 b = *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + st + 4 * q)));
        const float4 c = *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + 2 * st + 4 * q)));
        const float4 d = *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + 3 * st + 4 * q)));
        return make_float4(((a.x * t.w1 + b.x * t.w2) + c.x * t.w3) + d.x * t.w4,
                           ((a.y * t.w1 + b.y * t.w2) + c.y * t.w3) + d.y * t.w4,
                           ((a.z * t.w1 + b.z * t.w2) + c.z * t.w3) + d.z * t.w4,
                           ((a.w * t.w1 + b.w * t.w2) + c.w * t.w3) + d.w * t.w4);
    }
    if (t.constOnly || t.blend) {   // a checkerboard: leaf 1 [blended with leaf 2]
        const float4 a = t.constOnly ? *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + 4 * q)))
                                     : from_rgb4(S, t.pick, false, q);
        if (!t.blend) return a;
        const float4 b = t.constOff2 >= 0 ? *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff2 + 4 * q)))
                                          : from_rgb4(S, t.pick2, false, q);
        // (1 - area2) * tex1 + area2 * tex2: CoefficientSpectrum's s * a, then the sum
        return make_float4((a.x * t.w1) + (b.x * t.w2), (a.y * t.w1) + (b.y * t.w2), (a.z * t.w1) + (b.z * t.w2),
                           (a.w * t.w1) + (b.w * t.w2));
    }
    float4 a = from_rgb4(S, t.pick, false, q);
    if (t.constOff < 0) return a;
    float4 b = *reinterpret_cast<const float4 *>(sa(S.spectra, (uint32_t)(t.constOff + 4 * q)));
    return t.constFirst ? make_float4(b.x * a.x, b.y * a.y, b.z * a.z, b.w * a.w)
                        : make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
// Texture<Spectrum>::EvaluateMemory (the fork's RGB of a texture before FromRGB): an image map's
// MIPMap lookup, RGB 0 for a constant (constant.h:45-47), the product for a scale (scale.h:47-49)
PGD_INLINE void tex_memory_leaf(const DevScene &S, int id, const TexPt &q, float rgb[3]) {
    const pbrtgpu_texture &tx = (*sa(S.tex, (uint32_t)(id)));
    if (tx.type == PBRTGPU_TEX_IMAGE || tx.type == PBRTGPU_TEX_UV) leaf_rgb(S, tx, q, rgb);   // uv.h:46-51
    else rgb[0] = rgb[1] = rgb[2] = 0.f;
}
// Material::NormalMap (material.cpp:82-126) where the map's spectrum (Evaluate, FromRGB of its
// texel) is not black (the materials' `!normalSpectrum.IsBlack()`); *nOut = the rotated shading
// normal before the orientation flip and Faceforward.  false: not black -> Bump instead
PGD_HEAVY bool normal_map(const DevScene &S, int id, const TexPt &q, V nn, V *nOut) {
    const pbrtgpu_texture &tx = (*sa(S.tex, (uint32_t)(id)));
    bool black = true;
    if (tx.type == PBRTGPU_TEX_CONST) {
        for (int i = 0; i < S.nb; ++i) black = black && (*sa(S.spectra, (uint32_t)(tx.spec + i))) == 0.f;
    } else {
        const SpecTex st = tex_spec_prepare(S, id, q);
        for (int qq = 0; qq < S.nbp / 4; ++qq) {
            const float4 v = tex_spec4(S, st, qq);
            black = black && v.x == 0.f && (4 * qq + 1 >= S.nb || v.y == 0.f) && (4 * qq + 2 >= S.nb || v.z == 0.f) &&
                    (4 * qq + 3 >= S.nb || v.w == 0.f);
        }
    }
    if (black) return false;
    float c[3];
    if (tx.type == PBRTGPU_TEX_SCALE) {
        float a[3], b[3];
        tex_memory_leaf(S, tx.tex1, q, a);
        tex_memory_leaf(S, tx.tex2, q, b);
        for (int k = 0; k < 3; ++k) c[k] = a[k] * b[k];
    } else tex_memory_leaf(S, id, q, c);
    for (int k = 0; k < 3; ++k) c[k] = c[k] * 2.f - 1.f;
    const V n = vnorm(v3(c[0], c[1], c[2]));
    const V axis = vcross(v3(0.f, 0.f, 1.f), n);
    const float angle = (180.f / kPi) * ACOSF(vdot(v3(0.f, 0.f, 1.f), n));   // Degrees(acosf(Dot))
    // Rotate(angle, axis) (transform.cpp:197-224) applied to the normal: m . nn
    const V a = vnorm(axis);
    const float2 sc = SINCOSF((kPi / 180.f) * angle);   // sinf / cosf (Radians)
    const float s = sc.x, co = sc.y;
    const float m00 = a.x * a.x + (1.f - a.x * a.x) * co, m01 = a.x * a.y * (1.f - co) - a.z * s,
                m02 = a.x * a.z * (1.f - co) + a.y * s;
    const float m10 = a.x * a.y * (1.f - co) + a.z * s, m11 = a.y * a.y + (1.f - a.y * a.y) * co,
                m12 = a.y * a.z * (1.f - co) - a.x * s;
    const float m20 = a.x * a.z * (1.f - co) - a.y * s, m21 = a.y * a.z * (1.f - co) + a.x * s,
                m22 = a.z * a.z + (1.f - a.z * a.z) * co;
    *nOut = v3(m00 * nn.x + m01 * nn.y + m02 * nn.z, m10 * nn.x + m11 * nn.y + m12 * nn.z,
               m20 * nn.x + m21 * nn.y + m22 * nn.z);
    return true;
}
// DifferentialGeometry::ComputeDifferentials (diffgeom.cpp:50-105) for the camera ray's
// offset rays; out = dudx, dvdx, dudy, dvdy
struct RayDiff { V rxo, rxd, ryo, ryd; };
PGD_INLINE float vcomp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// dpdx / dpdy (optional) = px - p, py - p, zero where the reference leaves them zero
PGD_HEAVY void compute_differentials(const DG &dg, const RayDiff &rd, float out[4], V *dpdx = nullptr,
                                     V *dpdy = nullptr) {
    out[0] = out[1] = out[2] = out[3] = 0.f;
    if (dpdx) { *dpdx = v3(0.f, 0.f, 0.f); *dpdy = v3(0.f, 0.f, 0.f); }
    float d = -vdot(dg.nn, dg.p);
    float tx = -(vdot(dg.nn, rd.rxo) + d) / vdot(dg.nn, rd.rxd);
    if (isnan(tx)) return;
    V px = vadd(rd.rxo, vmul(rd.rxd, tx));
    float ty = -(vdot(dg.nn, rd.ryo) + d) / vdot(dg.nn, rd.ryd);
    if (isnan(ty)) return;
    V py = vadd(rd.ryo, vmul(rd.ryd, ty));
    if (dpdx) { *dpdx = vsub(px, dg.p); *dpdy = vsub(py, dg.p); }
    int a0, a1;
    if (fabsf(dg.nn.x) > fabsf(dg.nn.y) && fabsf(dg.nn.x) > fabsf(dg.nn.z)) { a0 = 1; a1 = 2; }
    else if (fabsf(dg.nn.y) > fabsf(dg.nn.z)) { a0 = 0; a1 = 2; }
    else { a0 = 0; a1 = 1; }
    float A[2][2] = {{vcomp(dg.dpdu, a0), vcomp(dg.dpdv, a0)}, {vcomp(dg.dpdu, a1), vcomp(dg.dpdv, a1)}};
    float Bx[2] = {vcomp(px, a0) - vcomp(dg.p, a0), vcomp(px, a1) - vcomp(dg.p, a1)};
    float By[2] = {vcomp(py, a0) - vcomp(dg.p, a0), vcomp(py, a1) - vcomp(dg.p, a1)};
    if (!solve2x2(A, Bx, &out[0], &out[1])) out[0] = out[1] = 0.f;
    if (!solve2x2(A, By, &out[2], &out[3])) out[2] = out[3] = 0.f;
}

// Intersection::GetBSDF -> GetShadingGeometry -> Material::GetBSDF (+ Bump, material.cpp:39-81)
// diff: dudx, dvdx, dudy, dvdy of the hit (zero without ray differentials); the material's
// textured spectra (at most two) are evaluated in slot order into the slot's K band buffers j = 0,
// 1 (kb[(j * NQ + q) * c], clamped unless the material uses them raw) and its BxDFs refer to
// buffer j with offset -1 - j * NQ (spec4)
// dnOut (optional): dndu, dndv of the shading geometry (SpecularReflect / SpecularTransmit ray
// differentials, integrator.cpp:190-192)
template <int FEAT>
PGD_HEAVY void get_bsdf(const DevScene &S, const Isect &is, const float diff[10], float4 *kb, size_t c, BSDF &bs,
                        V *pOut, V *nOut, V *dnOut = nullptr) {
    const float4 *rec = prim_rec(S, is.prim);
    const pbrtgpu_material &mt = (*sa(S.mats, (uint32_t)(is.mat)));
    DG dgs;
    int ro, swaps;
    if (__float_as_int(rec[6].x) == PBRTGPU_SHAPE_TRIANGLE) {
        if (is.inst < 0) {
            const pbrtgpu_mesh &m = (*sa(S.meshes, (uint32_t)__float_as_int(rec[7].y)));
#ifdef PGD_AB_NO_PRIMREC
            tri_shading(S, __float_as_int(rec[6].y), m.o2w_minv, is.dg, dgs);
#else
            tri_shading_rec(rec, m.o2w_minv, is.dg, dgs);
#endif
        } else {
            // ObjectToWorld = Inverse(Identity * w2p): its mInv is Mul(Identity, w2p.m)
            float w[16], id[16], nm[16];
            inst_load(is.im, is.inst, w, nullptr);
            m4_identity(id);
            m4_mul(id, w, nm);
            tri_shading_rec(rec, nm, is.dg, dgs);
        }
        ro = (__float_as_int(rec[7].x) & REC_FLIP) ? 1 : 0; swaps = 0;   // only reverse ^ swaps is used
    } else {
        dgs = is.dg;
        const pbrtgpu_quadric &q = (*sa(S.quads, (uint32_t)__float_as_int(rec[6].y)));
        ro = q.reverse_orientation; swaps = q.swaps_handedness;
    }
    TexPt tq;
    tq.u = dgs.u; tq.v = dgs.v; tq.dudx = diff[0]; tq.dvdx = diff[1]; tq.dudy = diff[2]; tq.dvdy = diff[3];
    tq.p = dgs.p; tq.dpdx = v3(diff[4], diff[5], diff[6]); tq.dpdy = v3(diff[7], diff[8], diff[9]);
    V bdpdu, bdpdv;
    V nmapN;
    const bool nmap = (FEAT & FEAT_TEX) && mt.normal_tex >= 0 && normal_map(S, mt.normal_tex, tq, dgs.nn, &nmapN);
    if (nmap) {   // dgBump = dgs with the rotated normal (material.cpp:113-114)
        bdpdu = dgs.dpdu;
        bdpdv = dgs.dpdv;
    } else if (!(FEAT & FEAT_TEX) || mt.bump_tex < 0) {
        float d = mt.f[7];
        const float du = .01f, dv = .01f;   // (d - d) / du == +0 for every positive du
        bdpdu = vadd(vadd(dgs.dpdu, vmul(dgs.nn, (d - d) / du)), vmul(dgs.dndu, d));
        bdpdv = vadd(vadd(dgs.dpdv, vmul(dgs.nn, (d - d) / dv)), vmul(dgs.dndv, d));
    } else {
        float du = .5f * (fabsf(tq.dudx) + fabsf(tq.dudy));
        if (du == 0.f) du = .01f;
        float dv = .5f * (fabsf(tq.dvdx) + fabsf(tq.dvdy));
        if (dv == 0.f) dv = .01f;
        // the u-shifted, v-shifted and unshifted evaluations (dgEval, material.cpp:47-62), in one
        // loop: one copy of the texture code
        float uDisplace = 0.f, vDisplace = 0.f, displace = 0.f;
#pragma unroll 1
        for (int l = 0; l < 3; ++l) {
            TexPt qe = tq;
            if (l == 0) { qe.u = dgs.u + du; qe.p = vadd(dgs.p, vmul(dgs.dpdu, du)); }
            else if (l == 1) { qe.v = dgs.v + dv; qe.p = vadd(dgs.p, vmul(dgs.dpdv, dv)); }
            const float dsp = tex_float(S, mt.bump_tex, qe);
            if (l == 0) uDisplace = dsp; else if (l == 1) vDisplace = dsp; else displace = dsp;
        }
        bdpdu = vadd(vadd(dgs.dpdu, vmul(dgs.nn, (uDisplace - displace) / du)), vmul(dgs.dndu, displace));
        bdpdv = vadd(vadd(dgs.dpdv, vmul(dgs.nn, (vDisplace - displace) / dv)), vmul(dgs.dndv, displace));
    }
    V nn = nmap ? nmapN : vnorm(vcross(bdpdu, bdpdv));
    if (ro ^ swaps) nn = vmul(nn, -1.f);
    nn = faceforward(nn, is.dg.nn);
    bs.ng = is.dg.nn;
    bs.nn = nn;
    bs.sn = vnorm(bdpdu);
    bs.tn = vcross(bs.nn, bs.sn);
    bs.n = 0;
    *pOut = dgs.p;
    *nOut = nn;
    if (dnOut) { dnOut[0] = dgs.dndu; dnOut[1] = dgs.dndv; }
    // material spectra: constant offsets, or the textured slots materialised in K (every material's
    // spectrum parameters are slots 0 and 1)
    int off[2];
    bool black0 = (mt.black_mask & 1) != 0, black1 = (mt.black_mask & 2) != 0;
    off[0] = mt.spec[0];
    off[1] = mt.spec[1];
    float fp0 = mt.f[0], fp1 = mt.f[1];
    if (FEAT & FEAT_TEX) {
        const int nq = S.nbp / 4;
        int j = 0;   // K buffer of the next textured slot
        // one copy of the lookup code for both slots (unrolled, the inlined texture lookups
        // doubled and k_shade's register peak with them)
#pragma unroll 1
        for (int k = 0; k < 2; ++k) {
            const int tid = k == 0 ? mt.tex[0] : mt.tex[1];
            if (tid < 0) continue;
            SpecTex st = tex_spec_prepare(S, tid, tq);
            const bool raw = (mt.black_mask >> (4 + k)) & 1;   // metal eta / k: Evaluate(dgs), no .Clamp()
            bool black = true;
            float4 *kj = kb + (size_t)j * nq * c;
            for (int q = 0; q < nq; ++q) {
                float4 v = tex_spec4(S, st, q);
                if (!raw)
                    v = make_float4(clampf(v.x, 0.f, INFINITY), clampf(v.y, 0.f, INFINITY), clampf(v.z, 0.f, INFINITY),
                                    clampf(v.w, 0.f, INFINITY));
                kj[q * c] = v;
                black = black && v.x == 0.f && (4 * q + 1 >= S.nb || v.y == 0.f) && (4 * q + 2 >= S.nb || v.z == 0.f) &&
                        (4 * q + 3 >= S.nb || v.w == 0.f);
            }
            if (k == 0) { off[0] = -1 - j * nq; black0 = black; }
            else { off[1] = -1 - j * nq; black1 = black; }
            ++j;
        }
        // float parameters f[0], f[1]: the constants, or float textures at the shading geometry
        // (matte's sigma clamped to [0, 90], matte.cpp:54; the constant was clamped on the host)
#pragma unroll 1
        for (int k = 0; k < 2; ++k) {
            const int tid = k == 0 ? mt.ftex[0] : mt.ftex[1];
            if (tid < 0) continue;
            float v = tex_float(S, tid, tq);
            if (mt.type == PBRTGPU_MAT_MATTE) v = clampf(v, 0.f, 90.f);
            if (k == 0) fp0 = v; else fp1 = v;
        }
    }
    const float f0 = fp0;
    bs.eta = mt.type == PBRTGPU_MAT_GLASS ? f0 : 1.f;
    // (the material switch itself is left whole in FEAT_BASIC objects: pruned, it moved k_shade's
    // register allocation from 9 to 31 spilled VGPRs, r06q)
    switch (mt.type) {
        case PBRTGPU_MAT_MATTE: {
            BxDF &x = bs.bx[bs.n++];
            x.R = off[0]; x.R2 = x.R;
            x.type = BSDF_REFLECTION | BSDF_DIFFUSE;
            float sig = f0;
            if (sig == 0.) { x.kind = BX_LAMBERT; x.a = x.b = 0.f; }
            else {
                x.kind = BX_OREN;
                float sigma = (kPi / 180.f) * sig;
                float sigma2 = sigma * sigma;
                x.a = 1.f - (sigma2 / (2.f * (sigma2 + 0.33f)));
                x.b = 0.45f * sigma2 / (sigma2 + 0.09f);
            }
            break;
        }
        case PBRTGPU_MAT_PLASTIC: {
            BxDF &x0 = bs.bx[bs.n++];
            x0.kind = BX_LAMBERT; x0.type = BSDF_REFLECTION | BSDF_DIFFUSE; x0.R = off[0]; x0.R2 = x0.R;
            x0.a = x0.b = 0.f;
            BxDF &x1 = bs.bx[bs.n++];
            x1.kind = BX_MICRO_BLINN_DIEL; x1.type = BSDF_REFLECTION | BSDF_GLOSSY; x1.R = off[1]; x1.R2 = x1.R;
            float e = 1.f / f0;
            if (e > 10000.f || isnan(e)) e = 10000.f;
            x1.a = e; x1.b = 0.f;
            break;
        }
        case PBRTGPU_MAT_METAL: {   // metal.cpp:44-62: Microfacet(1, FresnelConductor(eta, k), Blinn(1/rough))
            BxDF &x = bs.bx[bs.n++];
            x.kind = BX_MICRO_BLINN_COND; x.type = BSDF_REFLECTION | BSDF_GLOSSY;
            x.R = off[0]; x.R2 = off[1];
            float e = 1.f / f0;
            if (e > 10000.f || isnan(e)) e = 10000.f;
            x.a = e; x.b = 0.f;
            break;
        }
        case PBRTGPU_MAT_MIRROR: {
            if (!black0) {
                BxDF &x = bs.bx[bs.n++];
                x.kind = BX_SPEC_REFL_NOOP; x.type = BSDF_REFLECTION | BSDF_SPECULAR; x.R = off[0]; x.R2 = x.R;
                x.a = x.b = 0.f;
            }
            break;
        }
        case PBRTGPU_MAT_GLASS: {   // glass.cpp:34-57: each specular lobe if its spectrum is not black
            if (!black0) {
                BxDF &x = bs.bx[bs.n++];
                x.kind = BX_SPEC_REFL_DIEL; x.type = BSDF_REFLECTION | BSDF_SPECULAR; x.R = off[0]; x.R2 = x.R;
                x.a = f0; x.b = 0.f;
            }
            if (!black1) {
                BxDF &x = bs.bx[bs.n++];
                x.kind = BX_SPEC_TRANS; x.type = BSDF_TRANSMISSION | BSDF_SPECULAR; x.R = off[1]; x.R2 = x.R;
                x.a = f0; x.b = 0.f;
            }
            break;
        }
        case PBRTGPU_MAT_MEASURED: {   // measured.cpp:182-206: one IrregIsotropicBRDF
            BxDF &x = bs.bx[bs.n++];
            x.kind = BX_MEASURED_IRREG; x.type = BSDF_REFLECTION | BSDF_GLOSSY;
            x.R = mt.aux; x.R2 = mt.aux2;
            x.a = x.b = 0.f;
            break;
        }
        case PBRTGPU_MAT_MEASURED_HALFANGLE: {   // measured.cpp:196-198: one RegularHalfangleBRDF, none without data
            if (mt.aux < 0) break;
            BxDF &x = bs.bx[bs.n++];
            x.kind = BX_MEASURED_HALF; x.type = BSDF_REFLECTION | BSDF_GLOSSY;
            x.R = mt.aux; x.R2 = 0;
            x.a = x.b = 0.f;
            break;
        }
        case PBRTGPU_MAT_ANISOWARD: {   // anisoward.cpp:35-60: Lambertian(Kd) + AnisoWardBrdf(Ks, alphaU, alphaV)
            BxDF &x0 = bs.bx[bs.n++];
            x0.kind = BX_LAMBERT; x0.type = BSDF_REFLECTION | BSDF_DIFFUSE; x0.R = off[0]; x0.R2 = x0.R;
            x0.a = x0.b = 0.f;
            BxDF &x1 = bs.bx[bs.n++];
            x1.kind = BX_ANISOWARD; x1.type = BSDF_REFLECTION | BSDF_GLOSSY; x1.R = off[1]; x1.R2 = x1.R;
            x1.a = f0; x1.b = fp1;   // sampled and weighed by BxDF's cosine defaults (reflection.cpp:303-315)
            break;
        }
        case PBRTGPU_MAT_SHINYMETAL: {   // shinymetal.cpp:45-68: Microfacet(1, FresnelConductor(etaKs, 0), Blinn(1/rough))
            BxDF &x0 = bs.bx[bs.n++];     // + SpecularReflection(1, FresnelConductor(etaKr, 0))
            x0.kind = BX_MICRO_BLINN_COND; x0.type = BSDF_REFLECTION | BSDF_GLOSSY;
            x0.R = off[0]; x0.R2 = mt.spec[2];
            float e = 1.f / f0;
            if (e > 10000.f || isnan(e)) e = 10000.f;
            x0.a = e; x0.b = 0.f;
            BxDF &x1 = bs.bx[bs.n++];
            x1.kind = BX_SPEC_REFL_COND; x1.type = BSDF_REFLECTION | BSDF_SPECULAR; x1.R = mt.spec[1]; x1.R2 = x1.R;
            x1.a = x1.b = 0.f;
            break;
        }
        case PBRTGPU_MAT_SUBSTRATE: {
            BxDF &x = bs.bx[bs.n++];
            x.kind = BX_FRESNEL_BLEND_ANISO; x.type = BSDF_REFLECTION | BSDF_GLOSSY;
            x.R = off[0]; x.R2 = off[1];
            float ex = 1.f / f0, ey = 1.f / fp1;
            if (ex > 10000.f || isnan(ex)) ex = 10000.f;
            if (ey > 10000.f || isnan(ey)) ey = 10000.f;
            x.a = ex; x.b = ey;
            break;
        }
        default: break;
    }
}

// ------------------------------------------------------------------ lights
PGD_INLINE V sphere_sample_p(const pbrtgpu_quadric &q, V p, float u1, float u2, V *ns) {
    V Pcenter = xpoint(q.o2w_m, v3(0, 0, 0));
    V wc = vnorm(vsub(Pcenter, p));
    V wcX, wcY;
    coordsys(wc, &wcX, &wcY);
    if (vlen2(vsub(p, Pcenter)) - q.radius * q.radius < 1e-4f) {
        V pp = vadd(v3(0, 0, 0), vmul(uniform_sphere(u1, u2), q.radius));
        *ns = vnorm(xnormal(q.o2w_minv, v3(pp.x, pp.y, pp.z)));
        if (q.reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q.o2w_m, pp);
    }
    float sinThetaMax2 = q.radius * q.radius / vlen2(vsub(p, Pcenter));
    float cosThetaMax = sqrtf(pmax(0.f, 1.f - sinThetaMax2));
    float costheta = lerpf(u1, cosThetaMax, 1.f);
    float sintheta = sqrtf(1.f - costheta * costheta);
    float phi = u2 * 2.f * kPi;
    const float2 sc = SINCOSF(phi);
    V dir = vadd(vadd(vmul(wcX, sc.y * sintheta), vmul(wcY, sc.x * sintheta)), vmul(wc, costheta));
    Ray r; r.o = p; r.d = dir; r.mint = 1e-3f; r.maxt = INFINITY; r.time = 0.f;
    float thit, eps;   // sphere.cpp:245-247 uses only thit of the intersection
    if (!sphere_intersect(q, r, &thit, &eps, nullptr)) thit = vdot(vsub(Pcenter, p), vnorm(r.d));
    V ps = rayat(r, thit);
    *ns = vnorm(vsub(ps, Pcenter));
    if (q.reverse_orientation) *ns = vmul(*ns, -1.f);
    return ps;
}
PGD_INLINE float shape_pdf_generic(const DevScene &S, int type, int idx, V p, V wi) {
    Ray ray; ray.o = p; ray.d = wi; ray.mint = 1e-3f; ray.maxt = INFINITY; ray.time = 0.f;
    float thit, eps;
    DG dg;
    if (!shape_intersect(S, type, idx, ray, &thit, &eps, &dg, true)) return 0.;
    float pdf = vlen2(vsub(p, rayat(ray, thit))) / (fabsf(vdot(dg.nn, vneg(wi))) * shape_area(S, type, idx));
    if (isinf(pdf)) pdf = 0.f;
    return pdf;
}
PGD_INLINE float shape_pdf(const DevScene &S, int type, int idx, V p, V wi) {
    if (type == PBRTGPU_SHAPE_SPHERE) {
        const pbrtgpu_quadric &q = (*sa(S.quads, (uint32_t)(idx)));
        V Pcenter = xpoint(q.o2w_m, v3(0, 0, 0));
        if (vlen2(vsub(p, Pcenter)) - q.radius * q.radius < 1e-4f) return shape_pdf_generic(S, type, idx, p, wi);
        float sinThetaMax2 = q.radius * q.radius / vlen2(vsub(p, Pcenter));
        float cosThetaMax = sqrtf(pmax(0.f, 1.f - sinThetaMax2));
        return 1.f / (2.f * kPi * (1.f - cosThetaMax));
    }
    return shape_pdf_generic(S, type, idx, p, wi);
}
PGD_INLINE V shape_sample_p(const DevScene &S, int type, int idx, V p, float u1, float u2, V *ns) {
    if (type == PBRTGPU_SHAPE_SPHERE) return sphere_sample_p((*sa(S.quads, (uint32_t)(idx))), p, u1, u2, ns);
    if (type == PBRTGPU_SHAPE_CYLINDER) {   // Cylinder::Sample (cylinder.cpp:195-203)
        const pbrtgpu_quadric &q = (*sa(S.quads, (uint32_t)(idx)));
        const float z = lerpf(u1, q.zmin, q.zmax), t = u2 * q.phi_max;
        const V pp = v3(q.radius * COSF(t), q.radius * SINF(t), z);
        *ns = vnorm(xnormal(q.o2w_minv, v3(pp.x, pp.y, 0.f)));
        if (q.reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q.o2w_m, pp);
    }
    if (type == PBRTGPU_SHAPE_DISK) {
        const pbrtgpu_quadric &q = (*sa(S.quads, (uint32_t)(idx)));
        V pp;
        concentric_disk(u1, u2, &pp.x, &pp.y);
        pp.x *= q.radius; pp.y *= q.radius; pp.z = q.height;
        *ns = vnorm(xnormal(q.o2w_minv, v3(0, 0, 1)));
        if (q.reverse_orientation) *ns = vmul(*ns, -1.f);
        return xpoint(q.o2w_m, pp);
    }
    const pbrtgpu_triangle t = (*sa(S.tris, (uint32_t)(idx)));
    const pbrtgpu_mesh &m = (*sa(S.meshes, (uint32_t)(t.mesh)));
    float su1 = sqrtf(u1);
    float b1 = 1.f - su1, b2 = u2 * su1;
    V p1 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[0]))), p2 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[1]))), p3 = ldv(sa(S.vertP, (uint32_t)(3 * t.v[2])));
    V pp = vadd(vadd(vmul(p1, b1), vmul(p2, b2)), vmul(p3, (1.f - b1 - b2)));
    *ns = vnorm(vcross(vsub(p2, p1), vsub(p3, p1)));
    if (m.reverse_orientation) *ns = vmul(*ns, -1.f);
    return pp;
}
PGD_INLINE int sample_discrete(const pbrtgpu_light_shape *ls, int n, float u) {
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
struct Seg { V o, d; float mint, maxt; };
// The radiance a light sample or a missed ray brings: a pool spectrum (divided by `div` for a
// point light's 1/d^2), FromRGB(illuminant) of an environment-map lookup, or black
enum { EM_BLACK = 0, EM_POOL = 1, EM_RGB = 2 };
// point (a delta light: PointLight, SpotLight, DistantLight): the pool spectrum times mul (the
// spot's Falloff) divided by div (the squared distance; 1 for the distant light)
struct Emit { int mode; int off; float div; bool point; RGBPick pick; float mul = 1.f; };
// InfiniteAreaLight (lights/infinite.cpp): its radiance map is one texel (an unreadable or
// non-TGA / PFM mapname, or none) or a decoded image's MIPMap (map_tex) with its Distribution2D
PGD_INLINE float spherical_theta(V v) { return ACOSF(clampf(v.z, -1.f, 1.f)); }   // geometry.h:642-650
PGD_INLINE float spherical_phi(V v) { float p = ATAN2F(v.y, v.x); return (p < 0.f) ? p + 2.f * kPi : p; }
PGD_INLINE Emit inf_radiance(const DevScene &S, const pbrtgpu_light &L, float s, float t) {
    float rgb[3];
    if (L.map_tex >= 0) mip_lookup_w<3>(S, (*sa(S.tex, (uint32_t)L.map_tex)), s, t, 0.f, rgb);   // MIPMap::Lookup(s, t)
    else mip_triangle<3>(L.texel, L.wrap, s, t, rgb);   // the one texel: MIPMap::Lookup(s, t), width 0
    Emit e;
    e.mode = EM_RGB; e.off = -1; e.div = 1.f; e.point = false;
    e.pick = rgb_pick(S, rgb);
    return e;
}
// InfiniteAreaLight::Le (infinite.cpp:84-89)
PGD_HEAVY Emit inf_Le(const DevScene &S, const pbrtgpu_light &L, V d) {
    V wh = vnorm(xvec(L.l2w_minv, d));
    return inf_radiance(S, L, spherical_phi(wh) * kInvTwoPi, spherical_theta(wh) * kInvPi);
}
// Distribution1D::SampleContinuous (montecarlo.h:68-84) of a record {funcInt, func[n], cdf[n + 1]}:
// std::upper_bound over the cdf (the first entry > u), the offset along its segment, the pdf
PGD_INLINE float dist1d_sample(const float *D, int n, float u, float *pdf, int *off) {
    const float *cdf = D + 1 + n;
    int lo = 0, len = n + 1;   // upper_bound: first i in [0, n + 1) with cdf[i] > u
    while (len > 0) {
        const int half = len >> 1;
        if (!(u < cdf[lo + half])) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    const int offset = lo - 1 > 0 ? lo - 1 : 0;
    *off = offset;
    const float du = (u - cdf[offset]) / (cdf[offset + 1] - cdf[offset]);
    *pdf = D[1 + offset] / D[0];
    return (offset + du) / n;
}
// Distribution2D::SampleContinuous (montecarlo.h:137-143) of a decoded environment map
PGD_INLINE void dist2d_sample(const DevScene &S, const pbrtgpu_light &L, float u0, float u1, float uv[2], float *pdf) {
    const int nu = L.dist_nu, nv = L.dist_nv;
    const float *M = sa(S.texels, (uint32_t)L.dist_off);
    float pdfs[2];
    int v;
    uv[1] = dist1d_sample(M, nv, u1, &pdfs[1], &v);
    const float *R = M + (2 + 2 * nv) + (size_t)v * (2 + 2 * nu);
    int o;
    uv[0] = dist1d_sample(R, nu, u0, &pdfs[0], &o);
    *pdf = pdfs[0] * pdfs[1];
}
// Distribution2D::Pdf (montecarlo.h:144-152)
PGD_INLINE float dist2d_pdf(const DevScene &S, const pbrtgpu_light &L, float u, float v) {
    const int nu = L.dist_nu, nv = L.dist_nv;
    const float *M = sa(S.texels, (uint32_t)L.dist_off);
    const int iu = clampi((int)(u * nu), 0, nu - 1), iv = clampi((int)(v * nv), 0, nv - 1);   // Float2Int
    const float *R = M + (2 + 2 * nv) + (size_t)iv * (2 + 2 * nu);
    if (R[0] * M[0] == 0.f) return 0.f;
    return (R[1 + iu] * M[1 + iv]) / (R[0] * M[0]);
}
// SpotLight::Falloff (spot.cpp:51-60): 0 outside the cone, 1 inside the falloff start, a quartic between
PGD_INLINE float spot_falloff(const pbrtgpu_light &L, V w) {
    const V wl = vnorm(xvec(L.l2w_minv, w));   // Normalize(WorldToLight(w))
    const float costheta = wl.z, cosTotal = L.texel[0], cosFalloff = L.texel[1];
    if (costheta < cosTotal) return 0.f;
    if (costheta > cosFalloff) return 1.f;
    const float delta = (costheta - cosTotal) / (cosFalloff - cosTotal);
    return delta * delta * delta * delta;
}
// Light::Sample_L (diffuse.cpp:61-74, point.cpp:42-49, spot.cpp:41-48, distant.cpp:39-46,
// infinite.cpp:155-185)
template <int FEAT>
PGD_HEAVY void light_sample_L(const DevScene &S, const pbrtgpu_light &L, V p, float pEps, const float u[3], V *wi,
                              float *pdf, Seg *vis, Emit *em) {
    em->mode = EM_BLACK; em->off = L.spec; em->div = 1.f; em->point = false;
    if ((FEAT & FEAT_INF) && L.type == PBRTGPU_LIGHT_INFINITE) {
        // Distribution2D::SampleContinuous: of one texel it returns (u0, u1) with pdf map_pdf
        float uv0 = u[0], uv1 = u[1], mapPdf = L.map_pdf;
        if (L.map_tex >= 0) {
            float uv[2];
            dist2d_sample(S, L, u[0], u[1], uv, &mapPdf);
            uv0 = uv[0]; uv1 = uv[1];
        }
        if (mapPdf == 0.f) { *pdf = 0.f; return; }
        float theta = uv1 * kPi, phi = uv0 * 2.f * kPi;
        const float2 st = SINCOSF(theta), sp = SINCOSF(phi);
        float costheta = st.y, sintheta = st.x;
        float sinphi = sp.x, cosphi = sp.y;
        *wi = xvec(L.l2w_m, v3(sintheta * cosphi, sintheta * sinphi, costheta));
        *pdf = mapPdf / (2.f * kPi * kPi * sintheta);
        if (sintheta == 0.f) *pdf = 0.f;
        vis->o = p; vis->d = *wi; vis->mint = pEps; vis->maxt = INFINITY;   // VisibilityTester::SetRay
        *em = inf_radiance(S, L, uv0, uv1);
        return;
    }
    if (L.type == PBRTGPU_LIGHT_POINT || ((FEAT & FEAT_INF) && L.type == PBRTGPU_LIGHT_SPOT)) {
        V lp = v3(L.pos[0], L.pos[1], L.pos[2]);
        *wi = vnorm(vsub(lp, p));
        *pdf = 1.f;
        float dist = vlen(vsub(p, lp));
        vis->o = p; vis->d = vdiv(vsub(lp, p), dist); vis->mint = pEps; vis->maxt = dist * (1.f - 0.f);
        em->mode = EM_POOL; em->point = true;
        em->div = vlen2(vsub(lp, p));   // Intensity / DistanceSquared
        if ((FEAT & FEAT_INF) && L.type == PBRTGPU_LIGHT_SPOT) em->mul = spot_falloff(L, vneg(*wi));   // spot.cpp:41-48
        return;
    }
    if ((FEAT & FEAT_INF) && L.type == PBRTGPU_LIGHT_DISTANT) {   // distant.cpp:39-46: L toward lightDir
        *wi = v3(L.pos[0], L.pos[1], L.pos[2]);
        *pdf = 1.f;
        vis->o = p; vis->d = *wi; vis->mint = pEps; vis->maxt = INFINITY;   // VisibilityTester::SetRay
        em->mode = EM_POOL; em->point = true;
        return;
    }
    const pbrtgpu_light_shape *shs = sa(S.lightShapes, (uint32_t)(L.shape_offset));
    int sn = sample_discrete(shs, L.n_shapes, u[2]);
    V ns;
    V pt = shape_sample_p(S, shs[sn].shape_type, shs[sn].shape_index, p, u[0], u[1], &ns);
    Ray r; r.o = p; r.d = vsub(pt, p); r.mint = 1e-3f; r.maxt = INFINITY; r.time = 0.f;
    float thit = 1.f;
    bool anyHit = false;
    V hitNN = v3(0, 0, 0);
    for (int i = 0; i < L.n_shapes; ++i) {
        float th, e;
        DG d2;
        if (shape_intersect(S, shs[i].shape_type, shs[i].shape_index, r, &th, &e, &d2, true)) { anyHit = true; thit = th; hitNN = d2.nn; }
    }
    if (anyHit) ns = hitNN;
    V ps = rayat(r, thit);
    *wi = vnorm(vsub(ps, p));
    float pp = 0.f;
    for (int i = 0; i < L.n_shapes; ++i) pp += shs[i].area * shape_pdf(S, shs[i].shape_type, shs[i].shape_index, p, *wi);
    *pdf = pp / L.sum_area;
    float dist = vlen(vsub(p, ps));
    vis->o = p; vis->d = vdiv(vsub(ps, p), dist); vis->mint = pEps; vis->maxt = dist * (1.f - 1e-3f);
    if (vdot(ns, vneg(*wi)) > 0.f && !L.is_black) em->mode = EM_POOL;   // DiffuseAreaLight::L
}
template <int FEAT>
PGD_HEAVY float light_pdf(const DevScene &S, const pbrtgpu_light &L, V p, V wi) {
    if (L.type == PBRTGPU_LIGHT_POINT) return 0.;
    if ((FEAT & FEAT_INF) && (L.type == PBRTGPU_LIGHT_SPOT || L.type == PBRTGPU_LIGHT_DISTANT)) return 0.;
    if ((FEAT & FEAT_INF) && L.type == PBRTGPU_LIGHT_INFINITE) {   // infinite.cpp:188-197
        V w = xvec(L.l2w_minv, wi);
        const float theta = spherical_theta(w);
        float sintheta = SINF(theta);
        if (sintheta == 0.f) return 0.f;
        // Distribution2D::Pdf(phi / 2pi, theta / pi); of one texel the constant dist_pdf
        const float dp = L.map_tex >= 0 ? dist2d_pdf(S, L, spherical_phi(w) * kInvTwoPi, theta * kInvPi) : L.dist_pdf;
        return dp / (2.f * kPi * kPi * sintheta);
    }
    const pbrtgpu_light_shape *shs = sa(S.lightShapes, (uint32_t)(L.shape_offset));
    float pp = 0.f;
    for (int i = 0; i < L.n_shapes; ++i) pp += shs[i].area * shape_pdf(S, shs[i].shape_type, shs[i].shape_index, p, wi);
    return pp / L.sum_area;
}

// camera sample -> camera-space ray before CameraToWorld, and Pcamera (perspective.cpp:73-97;
// orthographic.cpp:42-65: the ray starts at Pcamera along +z)
PGD_INLINE Ray camera_local(const pbrtgpu_camera &cam, float imageX, float imageY, float lensU, float lensV,
                            float timeU, V *PcOut) {
    const float *m = cam.raster_to_camera;
    float x = imageX, y = imageY, z = 0;
    V Pc;
    Pc.x = m[0] * x + m[1] * y + m[2] * z + m[3];
    Pc.y = m[4] * x + m[5] * y + m[6] * z + m[7];
    Pc.z = m[8] * x + m[9] * y + m[10] * z + m[11];
    float w = m[12] * x + m[13] * y + m[14] * z + m[15];
    if (w != 1.) Pc = vdiv(Pc, w);
    Ray r;
    if (cam.ortho) {
        r.o = Pc;
        r.d = v3(0.f, 0.f, 1.f);
    } else {
        r.o = v3(0, 0, 0);
        r.d = vnorm(v3(Pc.x, Pc.y, Pc.z));
    }
    r.mint = 0.f; r.maxt = INFINITY;
    if (cam.lens_radius > 0.) {
        float lu, lv;
        concentric_disk(lensU, lensV, &lu, &lv);
        lu *= cam.lens_radius; lv *= cam.lens_radius;
        float ft = cam.focal_distance / r.d.z;
        V Pfocus = rayat(r, ft);
        r.o = v3(lu, lv, 0.f);
        r.d = vnorm(vsub(Pfocus, r.o));
    }
    // the sampler's Sample::time is already Lerp(u, shutterOpen, shutterClose) (LDPixelSample,
    // montecarlo.cpp:229) and the camera lerps it again (perspective.cpp:67, 102;
    // realisticDiffraction.cpp:1157): the identity only for the default shutter [0, 1]
    r.time = lerpf(lerpf(timeU, cam.shutter_open, cam.shutter_close), cam.shutter_open, cam.shutter_close);
    *PcOut = Pc;
    return r;
}
PGD_INLINE V cam_point(const float *cw, V p) {   // Transform::operator()(Point), divide if w != 1
    float xp = cw[0] * p.x + cw[1] * p.y + cw[2] * p.z + cw[3];
    float yp = cw[4] * p.x + cw[5] * p.y + cw[6] * p.z + cw[7];
    float zp = cw[8] * p.x + cw[9] * p.y + cw[10] * p.z + cw[11];
    float wp = cw[12] * p.x + cw[13] * p.y + cw[14] * p.z + cw[15];
    V o = v3(xp, yp, zp);
    if (wp != 1.) o = vdiv(o, wp);
    return o;
}
// the camera ray's offset rays (perspective.cpp:98-104) in world space, after
// RayDifferential::ScaleDifferentials(1 / sqrtf(spp)) (samplerrenderer.cpp:91)
// CameraToWorld at the ray's time: the static matrix, or AnimatedTransform's start / end
// transform or Interpolate(time) (transform.cpp:356-381, 427-455) of an animated camera
PGD_INLINE const float *cam_xform(const pbrtgpu_camera &cam, const pbrtgpu_instance *cm, float time, float *buf) {
    if (!cm) return cam.cam2world_m;
    inst_interp(*cm, time, buf, nullptr);
    return buf;
}
PGD_INLINE RayDiff camera_diff(const pbrtgpu_camera &cam, int spp, float imageX, float imageY, float lensU, float lensV,
                               float timeU, const pbrtgpu_instance *cm = nullptr) {
    V Pc;
    Ray r = camera_local(cam, imageX, imageY, lensU, lensV, timeU, &Pc);
    float cwb[16];
    const float *cw = cam_xform(cam, cm, r.time, cwb);
    V o = cam_point(cw, r.o), d = xvec(cw, r.d);
    const V dx = v3(cam.dx_camera[0], cam.dx_camera[1], cam.dx_camera[2]), dy = v3(cam.dy_camera[0], cam.dy_camera[1], cam.dy_camera[2]);
    float sc = 1.f / sqrtf((float)spp);
    RayDiff rd;
    if (cam.ortho) {   // orthographic.cpp:95-98: origins one pixel over, the ray's own direction
        rd.rxo = vadd(o, vmul(vsub(cam_point(cw, vadd(r.o, dx)), o), sc));
        rd.ryo = vadd(o, vmul(vsub(cam_point(cw, vadd(r.o, dy)), o), sc));
        rd.rxd = vadd(d, vmul(vsub(d, d), sc));
        rd.ryd = rd.rxd;
        return rd;
    }
    V rxd = xvec(cw, vnorm(vadd(Pc, dx)));
    V ryd = xvec(cw, vnorm(vadd(Pc, dy)));
    rd.rxo = vadd(o, vmul(vsub(o, o), sc));
    rd.ryo = rd.rxo;
    rd.rxd = vadd(d, vmul(vsub(rxd, d), sc));
    rd.ryd = vadd(d, vmul(vsub(ryd, d), sc));
    return rd;
}
// camera sample -> world ray (perspective.cpp:73-106)
PGD_INLINE Ray camera_ray(const pbrtgpu_camera &cam, float imageX, float imageY, float lensU, float lensV, float timeU,
                          const pbrtgpu_instance *cm = nullptr) {
    V Pc;
    Ray r = camera_local(cam, imageX, imageY, lensU, lensV, timeU, &Pc);
    float cwb[16];
    const float *cw = cam_xform(cam, cm, r.time, cwb);
    Ray o = r;
    o.o = cam_point(cw, r.o);
    o.d = xvec(cw, r.d);
    return o;
}

// ---- RealisticDiffractionCamera (cameras/realisticDiffraction.cpp), diffraction off
// IntersectLensEl (realisticDiffraction.cpp:412-468): the sphere of |radius| centred by
// Translate(dist); tHit, and the normalised hit point (in the shifted frame) as the normal
PGD_INLINE bool lens_el_hit(const Ray &r, float radius, V dist, float *tHit, V *nrm) {
    const float m[16] = {1.f, 0.f, 0.f, dist.x, 0.f, 1.f, 0.f, dist.y, 0.f, 0.f, 1.f, dist.z, 0.f, 0.f, 0.f, 1.f};
    const V o = cam_point(m, r.o), d = xvec(m, r.d);
    if (radius < 0) radius = -radius;
    const float A = d.x * d.x + d.y * d.y + d.z * d.z;
    const float B = 2 * (d.x * o.x + d.y * o.y + d.z * o.z);
    const float C = o.x * o.x + o.y * o.y + o.z * o.z - radius * radius;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return false;
    if (t0 > r.maxt || t1 < r.mint) return false;
    float th = t0;
    if (t0 < r.mint) {
        th = t1;
        if (th > r.maxt) return false;
    }
    *tHit = th;
    *nrm = vnorm(v3(d.x * th + o.x, d.y * th + o.y, d.z * th + o.z));
    return true;
}
// Spectrum::GetValueAtWavelength (spectrum.h:384-405) of a spectrum of N bands: the band interval
// of wl (integer step), Lerp of its two values; 0 outside every interval (band wavelengths in the
// last interval, which would read c[N], are refused at upload)
PGD_INLINE float value_at_wavelength(const float *c, int N, float wl) {
    const int l0 = N == 30 ? 400 : 395, l1 = N == 30 ? 700 : 715;
    const float step = (float)((l1 - l0) / N);
    for (int i = 0; i < N; ++i) {
        const float w0 = l0 + i * step, w1 = l0 + (i + 1) * step;
        if (wl >= w0 && wl < w1) return lerpf((wl - w0) / (w1 - w0), *sa(c, (uint32_t)i), *sa(c, (uint32_t)(i + 1)));
    }
    return 0.f;
}
// applySnellsLaw (realisticDiffraction.cpp:347-410).  IORforEyeEnabled with a wavelength: the
// ocular medium is recognised by the lens file's n (|n1 - n| < .001 in double: vitreous 1.336,
// lens 1.42, aqueous 1.3374, cornea 1.3771) and both indices come from the eye IOR spectra at the
// wavelength; otherwise the chromatic model, whose arithmetic is double (the -.04 literal)
PGD_INLINE void lens_snell(const DevScene &S, float n1, float n2, float lensRadius, V nrm, Ray *ray, float wl) {
    if (S.lensEye && wl != 0) {
        const int N = S.nb;
        const float *cornea = S.lensEyeIor, *aqueous = cornea + N, *lensI = cornea + 2 * N, *vitreous = cornea + 3 * N;
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
    } else if (S.lensChromatic) {
        if (n1 != 1) n1 = (float)((double)(wl - 550) * -.04 / (300) + (double)n1);
        if (n2 != 1) n2 = (float)((double)(wl - 550) * -.04 / (300) + (double)n2);
    }
    const V s1 = ray->d;
    if (lensRadius > 0) nrm = vneg(nrm);
    const V c = vcross(nrm, s1);
    const float radicand = 1 - (n1 / n2) * (n1 / n2) * vdot(c, c);
    if (radicand < 0) {
        ray->d = v3(0.f, 0.f, 0.f);
        return;
    }
    const V s2 = vsub(vmul(vcross(nrm, vcross(vmul(nrm, -1.f), s1)), n1 / n2), vmul(nrm, sqrtf(radicand)));
    ray->d = vnorm(s2);
}
// ---- diffraction (realisticDiffraction.cpp:1057-1150).  PARITY UNPINNED: the reference draws
// the Gaussian from one GSL generator (gsl_rng_default, mt19937) shared by every render thread,
// so which values a ray receives depends on thread scheduling, and GSL is absent here (the
// reference camera cannot be built).  The oracle restates the same stream; GPU = oracle.
// The camera sample's stream: each camera sample (and SpectralRenderer band) draws from its own
// counter-based stream, uniform j = (top 32 bits of splitmix64(key + (j + 1) * golden)) / 2^32
// (gsl_rng_uniform's 32-bit resolution), key = pixel hash << 32 | the path's RNG index.  Being
// counter based, the camera differentials re-derived at the first hit (path_camera_diff) see
// the same values as the camera ray.
struct DiffStream {
    uint64_t key;
    uint32_t j;
};
PGD_INLINE double diff_uniform(DiffStream *st) {
    uint64_t z = st->key + (uint64_t)(++st->j) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(uint32_t)(z >> 32) / 4294967296.0;
}
// gsl_ran_bivariate_gaussian (GSL randist/bigauss.c, the polar Box-Muller method) with rho = 0:
// (u, v) uniform in the square [-1, 1)^2 until 0 < r2 = u^2 + v^2 <= 1, s = sqrt(-2 ln r2 / r2),
// x = sigma_x u s, y = sigma_y (rho u + sqrt(1 - rho^2) v) s.  The rejection loop is bounded
// (64 tries, each accepted with probability pi / 4): after that, no noise.
PGD_INLINE void diff_gaussian(DiffStream *st, double sx, double sy, double *x, double *y) {
    *x = 0.0;
    *y = 0.0;
    for (int k = 0; k < 64; ++k) {
        const double u = -1 + 2 * diff_uniform(st);
        const double v = -1 + 2 * diff_uniform(st);
        const double r2 = u * u + v * v;
        if (r2 > 1.0 || r2 == 0) continue;
        const double scale = __builtin_sqrt(-2.0 * pbrt_fm_log(r2) / r2);
        *x = sx * u * scale;
        *y = sy * (0.0 * u + 1.0 * v) * scale;
        return;
    }
}
// The perturbation after element i (aperture stop or lens surface): ip the element's
// intersection point, ap its aperture, wl the ray's wavelength (0 under the SamplerRenderer:
// sigma = atan(1 / inf) = 0, the draws are still made); the radius is measured from (cx, cy):
// the axis for the main lens, the microlens centre for a microlens surface (:790-872, whose
// direction vectors still come from the absolute hit point).  The expressions keep the
// reference's float / double mix (float Vector arithmetic and sqrtf where its operands are
// float).  nanOut (main lens): a NaN direction returns false (weight 0, realisticDiffraction.cpp:
// 1141-1147); the microlens step normalises whatever it got.  Out of line: its double arithmetic
// is not inlined into the element steps of a camera differential.
__device__ __attribute__((noinline)) bool lens_diffract(DiffStream *st, V ip, float cx, float cy, float ap, float wl, V *dp,
                                                        bool nanOut) {
    const double radius = (double)sqrtf((ip.x - cx) * (ip.x - cx) + (ip.y - cy) * (ip.y - cy));
    V dir = v3(ip.x, ip.y, 0.f), orth = v3(-ip.y, ip.x, 0.f);
    const double a = (double)(ap / 2) - radius;
    const double b = __builtin_sqrt((double)(ap / 2 * ap / 2) - radius * radius);
    const double pi = 3.14159265359;
    const double lambda = (double)wl * 1e-9;
    const double sqrt2 = 1.4142135623730951;   // sqrt(2)
    const double sigx = pbrt_fm_atan(1 / (sqrt2 * a * .001 * 2 * pi / lambda));
    const double sigy = pbrt_fm_atan(1 / (sqrt2 * b * .001 * 2 * pi / lambda));
    double nx, ny;
    diff_gaussian(st, sigx, sigy, &nx, &ny);
    dir = vnorm(dir);
    orth = vnorm(orth);
    const float noiseA = (float)nx, noiseB = (float)ny;
    V d = *dp;
    const double projA = (double)((d.x * dir.x + d.y * dir.y) / sqrtf(dir.x * dir.x + dir.y * dir.y));
    const double projB = (double)((d.x * orth.x + d.y * orth.y) / sqrtf(orth.x * orth.x + orth.y * orth.y));
    double projC = (double)d.z;
    const double rA = __builtin_sqrt(projA * projA + projC * projC);
    double rB = __builtin_sqrt(projB * projB + projC * projC);
    double thetaA = pbrt_fm_acos(projA / rA);
    double thetaB = pbrt_fm_acos(projB / rB);
    thetaA = thetaA + (double)noiseA;
    thetaB = thetaB + (double)noiseB;   // overwritten below, as in the reference
    const double newProjA = pbrt_fm_cos(thetaA) * rA;
    d.z = (float)(pbrt_fm_sin(thetaA) * rA);
    projC = (double)d.z;
    rB = __builtin_sqrt(projB * projB + projC * projC);
    thetaB = pbrt_fm_acos(projB / rB);
    const double newProjB = pbrt_fm_cos(thetaB) * rB;
    d.z = (float)(pbrt_fm_sin(thetaB) * rB);
    d.x = (float)((double)dir.x * newProjA + (double)orth.x * newProjB);
    d.y = (float)((double)dir.y * newProjA + (double)orth.y * newProjB);
    if (nanOut && (d.x != d.x || d.y != d.y || d.z != d.z)) {
        *dp = v3(0.f, 0.f, 0.f);
        return false;
    }
    *dp = vnorm(d);
    return true;
}
// RealisticDiffractionCamera::GenerateRay (realisticDiffraction.cpp:478-1164): film point ->
// toward the sampled point of the last element's aperture disk (or the pinhole exit point, or
// the pinhole of the film point's superpixel, or a point of its microlens's entrance square) ->
// the two microlens surfaces -> every element, last first; a blocked or missed element returns
// weight 0.  The ray ends in world space with a normalised direction.
PGD_INLINE float lens_ray(const DevScene &S, float imageX, float imageY, float lensU, float lensV, float timeU, float wl,
                          DiffStream *st, Ray *out) {
    const pbrtgpu_camera &cam = S.cam;
    const float xr2 = (float)cam.xres / 2.f, yr2 = (float)cam.yres / 2.f;
    V sp;
    sp.x = (float)(-((double)(imageX - xr2) - .25) / (double)xr2);
    sp.y = (float)(((double)(imageY - yr2) - .25) / (double)yr2);
    sp.z = -S.lensFilmDist;
    const float aspect = (float)cam.xres / (float)cam.yres;
    const float width = S.lensFilmDiag / sqrtf((1.f + 1.f / (aspect * aspect)));
    const float height = width / aspect;
    sp.x = sp.x * width / 2.f + S.lensFilmC[0];
    sp.y = sp.y * height / 2.f + S.lensFilmC[1];
    if (S.lensCurveR != 0) {   // curved sensor
        const float R = S.lensCurveR, th = sp.x / R, ph = sp.y / R;
        sp.x = R * COSF(ph) * SINF(th);
        sp.z = R * COSF(ph) * COSF(th);
        sp.y = R * SINF(ph);
        const float sc = (-S.lensFilmDist - R);
        sp.z = sc + sp.z;
    }
    float lu, lv;
    concentric_disk(lensU, lensV, &lu, &lv);
    const float4 last = (*sa(S.lensEl, (uint32_t)(S.lensN - 1)));
    const float firstAp = last.w / 2, firstR = last.x;
    const float zI = firstR == 0 ? 0.f : (-firstR - sqrtf(firstR * firstR - firstAp * firstAp));
    const float luNoScale = lu, lvNoScale = lv;
    float pitch = 0.f;                  // superpixelPitch
    int xp = 0, yp = 0;                 // the pinhole under the film point
    const int nW = S.lensPinW, nH = S.lensPinH;
    const bool pinholes = nW > 0 && nH > 0;
    lu *= firstAp;
    lv *= firstAp;
    V pol = v3(lu, lv, zI);
    if (S.lensPinhole[0] != -1 && S.lensPinhole[1] != -1 && S.lensPinhole[2] != -1)
        pol = v3(S.lensPinhole[0], S.lensPinhole[1], S.lensPinhole[2]);
    else if (pinholes) {
        // the pinhole array (:560-629): the superpixel under the film point, clamped
        const int ppW = cam.xres / nW, ppH = cam.yres / nH;
        xp = (int)(((double)imageX - .25) / ppW);
        yp = (int)(((double)imageY - .25) / ppH);
        xp = xp > nW - 1 ? nW - 1 : (xp < 0 ? 0 : xp);
        yp = yp > nH - 1 ? nH - 1 : (yp < 0 ? 0 : yp);
        const float *ph = sa(S.lensPinholes, (uint32_t)(3 * (xp * nH + yp)));
        if (S.lensMicro) {   // the microlens's entrance square (:614-623)
            pitch = width / nW;
            pol = v3(luNoScale * pitch / 2.f + ph[0], lvNoScale * pitch / 2.f + ph[1], ph[2]);
        } else pol = v3(ph[0], ph[1], ph[2]);
    }
    Ray r;
    r.o = sp;
    r.d = vnorm(vsub(pol, r.o));
    r.mint = 0.f;
    r.maxt = INFINITY;
    r.time = 0.f;
    // The surfaces in tracing order: with microlenses first their two spherical surfaces (:634-876;
    // the radius from the thick-lens focal length, centred on the superpixel's pinhole, a miss
    // passes unrefracted, diffraction around the microlens centre without the NaN check), then
    // the lens elements, last first (a miss or a blocked ray has weight 0).  One loop body
    // serves both, so the kernels that start lens paths carry one copy of it.
    const int nMicro = (S.lensMicro && pinholes) ? 2 : 0;
    float mRad = 0.f, mDist = 0.f, mN = 1.f, cx = 0.f, cy = 0.f;
    const float thick = (float).01;
    if (nMicro) {
        const float *ph = sa(S.lensPinholes, (uint32_t)(3 * (xp * nH + yp)));
        const float mFilmDist = S.lensFilmDist + pol.z;
        const float mFocal = mFilmDist + thick / 2;
        mN = (float)1.67;
        const double nm1 = (double)(mN - 1);   // pow(microlensN - 1, 2): the exact square in double
        const float oneOverR = (float)((-2 * (mN - 1) + __builtin_sqrt(4 * (nm1 * nm1) + 4 * (nm1 * nm1) * thick / (mN * mFocal))) /
                                       (2 * (nm1 * nm1) * thick / mN));
        mRad = 1 / oneOverR;
        mDist = -S.lensFilmDist + mFilmDist;
        cx = ph[0];
        cy = ph[1];
    }
    float lensDist = 0.f;
    for (int k = 0; k < nMicro + S.lensN; ++k) {
        const bool micro = k < nMicro;
        const int i = S.lensN - 1 - (k - nMicro);   // the lens element (when !micro)
        float rad, ap;
        if (micro) {
            mRad = -mRad;
            rad = mRad;
            ap = pitch;
        } else {
            const float4 e = (*sa(S.lensEl, (uint32_t)(i)));
            rad = e.x;
            ap = e.w;
            lensDist += e.y;
            cx = 0.f;
            cy = 0.f;
        }
        r.o = sp;
        if (!micro && rad == 0) {   // aperture stop
            const float tA = (i == S.lensN - 1) ? S.lensFilmDist / r.d.z : (lensDist - r.o.z) / (r.d.z);
            const V ai = v3(r.o.x + r.d.x * tA, r.o.y + r.d.y * tA, r.o.z + r.d.z * tA);
            const float dx = ai.x - S.lensApOff[0], dy = ai.y - S.lensApOff[1];
            if ((double)(dx * dx + dy * dy) > (double)(ap * ap) * .25) return 0.f;
            sp = ai;
            if (S.lensDiffraction && !lens_diffract(st, ai, 0.f, 0.f, ap, wl, &r.d, true)) return 0.f;
            continue;
        }
        float tHit = 0.f;
        V nrm = v3(0.f, 0.f, 1.f), ip = v3(0.f, 0.f, 0.f);
        const bool hit = lens_el_hit(r, rad, v3(-cx, -cy, rad - (micro ? mDist : lensDist)), &tHit, &nrm);
        if (!hit && !micro) return 0.f;
        if (hit) {
            ip = v3(tHit * r.d.x + r.o.x, tHit * r.d.y + r.o.y, tHit * r.d.z + r.o.z);
            // (centre 0: (x - 0) (x - 0) is the main lens's x x; (ap ap) / (2 2) its ap ap / 4.f)
            if ((ip.x - cx) * (ip.x - cx) + (ip.y - cy) * (ip.y - cy) >= (ap * ap) / 4.f) return 0.f;
            float n1, n2 = 1;
            if (micro) {
                n1 = k == 0 ? 1.f : mN;
                n2 = k == 0 ? mN : 1.f;
                if (k == 0) mDist += thick;
            } else {
                n1 = (*sa(S.lensEl, (uint32_t)(i))).z;
                if (i - 1 >= 0) {
                    n2 = (*sa(S.lensEl, (uint32_t)(i - 1))).z;
                    if (n2 == 0) n2 = (*sa(S.lensEl, (uint32_t)(i - 2))).z;
                }
            }
            lens_snell(S, n1, n2, rad, nrm, &r, wl);
            sp = ip;
        }
        if (S.lensDiffraction && !lens_diffract(st, ip, cx, cy, ap, wl, &r.d, !micro)) return 0.f;
    }
    r.o = sp;
    // the sampler's Sample::time is already Lerp(u, shutterOpen, shutterClose) (LDPixelSample,
    // montecarlo.cpp:229) and the camera lerps it again (perspective.cpp:67, 102;
    // realisticDiffraction.cpp:1157): the identity only for the default shutter [0, 1]
    r.time = lerpf(lerpf(timeU, cam.shutter_open, cam.shutter_close), cam.shutter_open, cam.shutter_close);
    float cwb[16];   // CameraToWorld(*ray, ray) at the ray's time (realisticDiffraction.cpp:1158)
    const float *cw = cam_xform(cam, S.camMotion, r.time, cwb);
    out->o = cam_point(cw, r.o);
    out->d = vnorm(xvec(cw, r.d));
    out->mint = r.mint;
    out->maxt = r.maxt;
    out->time = r.time;
    return 1.f;
}
// Camera::GenerateRayDifferential (camera.cpp:52-81) for the lens camera: the ray, then the
// rays one pixel over in x and in y (the sample's imageX restored as (x + 1) - 1), weight 0
// if any of them is blocked; the offsets scaled by 1 / sqrtf(spp) (samplerrenderer.cpp:91)
// (the three rays draw from the sample's diffraction stream in that order)
PGD_INLINE float lens_ray_diff(const DevScene &S, float imageX, float imageY, float lensU, float lensV, float timeU,
                               float wl, uint64_t diffKey, Ray *ray, RayDiff *rd) {
    DiffStream st = {diffKey, 0u};
    const float wt = lens_ray(S, imageX, imageY, lensU, lensV, timeU, wl, &st, ray);
    Ray rx, ry;
    float sx = imageX + 1.f;
    const float wtx = lens_ray(S, sx, imageY, lensU, lensV, timeU, wl, &st, &rx);
    sx = sx - 1.f;
    const float wty = lens_ray(S, sx, imageY + 1.f, lensU, lensV, timeU, wl, &st, &ry);
    if (wtx == 0.f || wty == 0.f) return 0.f;
    const float sc = 1.f / sqrtf((float)S.spp);
    rd->rxo = vadd(ray->o, vmul(vsub(rx.o, ray->o), sc));
    rd->ryo = vadd(ray->o, vmul(vsub(ry.o, ray->o), sc));
    rd->rxd = vadd(ray->d, vmul(vsub(rx.d, ray->d), sc));
    rd->ryd = vadd(ray->d, vmul(vsub(ry.d, ray->d), sc));
    return wt;
}
// the ray wavelength of a path: the SpectralRenderer band's, 0 under the SamplerRenderer
// (its RayDifferentials start from Ray(), geometry.h:317)
PGD_INLINE float path_wavelength(const DevScene &S, int item, uint32_t smp) {
    if (!S.specMode) return 0.f;
    const int band = S.specMode == 1 ? item % S.specItems : (int)(smp % (uint32_t)S.specBands);
    return (*sa(S.specWl, (uint32_t)(band)));
}
// the RNG index of a path (path_seed's): its sample, or under the SpectralRenderer's
// singleDirection method sample * nWaveBands + band
PGD_INLINE uint32_t path_rng_index(const DevScene &S, uint32_t item, uint32_t smp) {
    return S.specItems > 1 ? smp * (uint32_t)S.specItems + item % (uint32_t)S.specItems : smp;
}
// the key of a camera sample's diffraction stream
PGD_INLINE uint64_t diff_key(uint32_t hp, uint32_t rngIdx) { return ((uint64_t)hp << 32) | rngIdx; }
// the camera ray's differentials for a path (first-hit texture filtering)
PGD_INLINE RayDiff path_camera_diff(const DevScene &S, int item, uint32_t hp, uint32_t smp, float imageX, float imageY,
                                    float lensU, float lensV, float timeU) {
    if (S.camType == PBRTGPU_CAMERA_REALISTIC) {
        Ray r;
        RayDiff rd;
        (void)lens_ray_diff(S, imageX, imageY, lensU, lensV, timeU, path_wavelength(S, item, smp),
                            diff_key(hp, path_rng_index(S, (uint32_t)item, smp)), &r, &rd);
        return rd;
    }
    return camera_diff(S.cam, S.spp, imageX, imageY, lensU, lensV, timeU, S.camMotion);
}

}  // namespace pgd
