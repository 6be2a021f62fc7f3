// directlighting.h -- DirectLightingIntegrator::Li (directlighting.cpp:73-109) as a wavefront
// shading step: k_shade<NB, FEAT, DL = true> calls shade_slot_dl once per live slot and pass.
//
// The reference recurses: a vertex adds its emission and its direct light (strategy "all":
// UniformSampleAllLights, integrator.cpp:39-71, RoundUpPow2(nSamples) samples per light;
// "one": UniformSampleOneLight, integrator.cpp:74-106), then, while depth + 1 < maxDepth,
// SpecularReflect and SpecularTransmit (integrator.cpp:169-250) trace a child ray each and add
// (f * Li_child) * |wi . n| / pdf.  Here a slot keeps that recursion as an explicit stack of
// frames in HBM (PathSoA::f*, frame d = the vertex at ray depth d) and advances it one ray
// round trip per pass:
//   - a light sample of the top vertex queues its shadow / MIS rays (estimate_direct, the
//     path integrator's EstimateDirect) and the next pass adds (0 [+ A]) [+ B] to the sums;
//   - a specular child queues its continuation ray; the pass that receives its hit pushes a
//     frame, the pass that completes the child pops it into the parent.
// Every other step (several zero-contribution light samples, a child that misses, a chain of
// completed frames) is done within one pass.  The vertex's BSDF is rebuilt from the frame's
// incoming ray whenever a pass needs it (isect_fill + get_bsdf are pure functions of the ray,
// the hit and the differentials).  The specular samples draw BSDFSample(rng) from the path's
// MT19937 stream in the reference's order (reflect, its subtree, transmit).
#pragma once
#include "wavefront.h"

namespace pgd {

template <int NB> PGD_INLINE float4 *dl_L(const PathSoA &P, int d, int slot) {
    return P.fL + (size_t)d * Bands<NB>::NQ * P.cap + slot;
}
template <int NB> PGD_INLINE float4 *dl_F(const PathSoA &P, int d, int slot) {
    return P.fF + (size_t)d * Bands<NB>::NQ * P.cap + slot;
}
PGD_INLINE void dl_vec_store(float *b, size_t c, V v) { b[0] = v.x; b[c] = v.y; b[2 * c] = v.z; }
PGD_INLINE V dl_vec_load(const float *b, size_t c) { return v3(b[0], b[c], b[2 * c]); }

// RoundUpPow2(max(1, nSamples)) samples of light i (directlighting.cpp:53-55)
PGD_INLINE int dl_count(const DevScene &S, int i) {
    uint32_t v = (uint32_t)max(1, (*sa(S.lights, (uint32_t)(i))).n_samples) - 1u;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return (int)(v + 1u);
}

// strategy "all": light-sample k of a vertex is sample j of light i (of n)
PGD_INLINE void dl_cursor(const DevScene &S, int k, int *i, int *j, int *n) {
    int li = 0, jj = k, nn = dl_count(S, 0);
    while (jj >= nn) { jj -= nn; ++li; nn = dl_count(S, li); }
    *i = li; *j = jj; *n = nn;
}

// sample values of light-sample k of a vertex (DirectLightingIntegrator::RequestSamples,
// directlighting.cpp:46-70 + the emission integrator's two 1D values): "all": per light i 1D
// [lightComp 2i, bsdfComp 2i+1], 2D [lightPos 2i, bsdfDir 2i+1], RoundUpPow2(nSamples) values
// each (value j of a count-n slot = sample s * n + j of a length spp * n sequence); "one":
// 1D [lightComp 0, lightNum 1, bsdfComp 2], 2D [lightPos 0, bsdfDir 1].  Returns the light.
PGD_INLINE int dl_sample(const DevScene &S, uint32_t hp, uint32_t s, int k, float ul[3], float ub[3], int *jOut,
                         int *nsOut) {
    const uint32_t spp = (uint32_t)S.spp;
    float u2[2];
    if (S.dlStrategy == PBRTGPU_DL_ONE) {
        const uint32_t n1 = 5u;
        const float ulnum = s1d(hp, 3u + 1u, s, spp);
        s2d(hp, 3u + n1 + 0u, s, spp, u2); ul[0] = u2[0]; ul[1] = u2[1];
        ul[2] = s1d(hp, 3u + 0u, s, spp);
        s2d(hp, 3u + n1 + 1u, s, spp, u2); ub[0] = u2[0]; ub[1] = u2[1];
        ub[2] = s1d(hp, 3u + 2u, s, spp);
        int ln = (int)floorf(ulnum * S.nLights);
        if (ln > S.nLights - 1) ln = S.nLights - 1;
        *jOut = 0; *nsOut = 1;
        return ln;
    }
    const uint32_t n1 = 2u * (uint32_t)S.nLights + 2u;
    int i, j, n;
    dl_cursor(S, k, &i, &j, &n);
    const uint32_t kk = s * (uint32_t)n + (uint32_t)j, len = spp * (uint32_t)n;
    s2d(hp, 3u + n1 + 2u * i, kk, len, u2); ul[0] = u2[0]; ul[1] = u2[1];
    ul[2] = s1d(hp, 3u + 2u * i, kk, len);
    s2d(hp, 3u + n1 + 2u * i + 1u, kk, len, u2); ub[0] = u2[0]; ub[1] = u2[1];
    ub[2] = s1d(hp, 3u + 2u * i + 1u, kk, len);
    *jOut = j; *nsOut = n;
    return i;
}

// the top vertex rebuilt from its frame: intersection, differentials, BSDF (col: the column of
// the textured-spectrum scratch PathSoA::K it uses -- the slot, or k_dl_nee's list row)
struct DLVertex {
    Ray ray;
    RayDiff rd;
    Isect is;
    BSDF bs;
    V p, n, wo, dpdx, dpdy, dn[2];
    float diff[10];   // du/dv (x, y), dpdx, dpdy (get_bsdf's texture point)
};
// DIFF: the ray differentials at the vertex (the specular branches' child rays need them); the
// light samples read them only through textured BSDF parameters (FEAT_TEX), so k_dl_nee's FEAT 0
// build skips the camera re-derivation and the differential solve
template <int NB, int FEAT, bool DIFF = true>
PGD_INLINE void dl_vertex(const DevScene &S, const PathSoA &P, int slot, int d, DLVertex &v, int col) {
    const size_t c = P.cap;
    const float *fr = P.fRay + (size_t)d * 9 * c + slot;
    v.ray.o = dl_vec_load(fr, c);
    v.ray.d = dl_vec_load(fr + 3 * c, c);
    v.ray.mint = fr[6 * c]; v.ray.maxt = fr[7 * c]; v.ray.time = fr[8 * c];
    const int prim = P.fHit[(size_t)2 * d * c + slot];
    const float t = __int_as_float(P.fHit[(size_t)(2 * d + 1) * c + slot]);
    isect_fill(S, v.ray, prim, t, v.is, inst_rec(P, slot));
    if (!DIFF) {
        for (int i = 0; i < 10; ++i) v.diff[i] = 0.f;
        get_bsdf<FEAT>(S, v.is, v.diff, P.K + col, c, v.bs, &v.p, &v.n, v.dn);
        v.wo = vneg(v.ray.d);
        return;
    }
    if (d == 0 && S.camType != PBRTGPU_CAMERA_REALISTIC) {
        // the perspective camera's differentials are re-derived from its sample; the lens camera's
        // were stored in frame 0 by path_start (their lens trace stays out of these kernels)
        const uint32_t hp = P.hp[slot], s = P.smp[slot], spp = (uint32_t)S.spp, pxy = P.pix[slot];
        float u[2], lens[2];
        s2d(hp, 0, s, spp, u);
        s2d(hp, 1, s, spp, lens);
        const float timeU = s1d(hp, 2, s, spp);
        v.rd = path_camera_diff(S, P.item[slot], hp, s, (int)(pxy & 0xffffu) + u[0], (int)(pxy >> 16) + u[1], lens[0], lens[1],
                                timeU);
    } else {
        const float *fd = P.fDiff + (size_t)d * 12 * c + slot;
        v.rd.rxo = dl_vec_load(fd, c);
        v.rd.rxd = dl_vec_load(fd + 3 * c, c);
        v.rd.ryo = dl_vec_load(fd + 6 * c, c);
        v.rd.ryd = dl_vec_load(fd + 9 * c, c);
    }
    compute_differentials(v.is.dg, v.rd, v.diff, &v.dpdx, &v.dpdy);
    v.diff[4] = v.dpdx.x; v.diff[5] = v.dpdx.y; v.diff[6] = v.dpdx.z;
    v.diff[7] = v.dpdy.x; v.diff[8] = v.dpdy.y; v.diff[9] = v.dpdy.z;
    get_bsdf<FEAT>(S, v.is, v.diff, P.K + col, c, v.bs, &v.p, &v.n, v.dn);
    v.wo = vneg(v.ray.d);
}

// adds light sample kk's ED = (0 [+ A]) [+ B] of the top vertex (frame d): strategy one
// L += ED * nLights (UniformSampleOneLight); strategy all Ld += ED, La += Ld / nSamples after a
// light's last sample and L += La after the last light (UniformSampleAllLights), the sums in the
// slot's beta buffers 0 (La) and 1 (Ld)
template <int NB>
PGD_INLINE void dl_add(const DevScene &S, const PathSoA &P, int slot, int d, int kk, int K, bool all, bool useA,
                       bool useB, const float4 *A, const float4 *B) {
    constexpr int NQ = Bands<NB>::NQ;
    const size_t c = P.cap;
    float4 *La = P.beta + slot, *Ld = P.beta + (size_t)NQ * c + slot;
    float4 *Lv = dl_L<NB>(P, d, slot);
    int li = 0, j = 0, ns = 1;
    if (all) dl_cursor(S, kk, &li, &j, &ns);
    const bool last = kk == K - 1;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float4 a = useA ? A[q * c] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 bb = useB ? B[q * c] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 ed;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float e = 0.f;
            if (useA) e += cmp(a, i);
            if (useB) e += cmp(bb, i);
            cmp(ed, i) = e;
        }
        if (!all) {
            float4 l = Lv[q * c];
            const float nl = (float)S.nLights;
            l.x += ed.x * nl; l.y += ed.y * nl; l.z += ed.z * nl; l.w += ed.w * nl;
            Lv[q * c] = l;
        } else {
            float4 ld = j == 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : Ld[q * c];
            ld.x += ed.x; ld.y += ed.y; ld.z += ed.z; ld.w += ed.w;
            if (j == ns - 1) {
                float4 la = kk + 1 == ns ? make_float4(0.f, 0.f, 0.f, 0.f) : La[q * c];   // the first light
                const float fn = (float)ns;
                la.x += ld.x / fn; la.y += ld.y / fn; la.z += ld.z / fn; la.w += ld.w / fn;
                if (last) {
                    float4 l = Lv[q * c];
                    l.x += la.x; l.y += la.y; l.z += la.z; l.w += la.w;
                    Lv[q * c] = l;
                } else La[q * c] = la;
            } else Ld[q * c] = ld;
        }
    }
}

// DirectLighting slot states beside wavefront.h's PF_* (bits 10, 11 are free there)
enum {
    PF_DLNEE = 1u << 10,   // the top vertex's next light-sample batch is due (k_dl_nee, this pass)
    PF_DLSPEC = 1u << 11,  // its light samples are done: its specular branches (k_dl_spec, this pass)
};

// the light-sample batches of a slot marked PF_DLNEE, run by k_dl_nee right after k_shade in
// the same pass: the vertex, then batches [k, kEnd) until one queues a ray (PF_PEND: the next
// k_shade adds it) or the last one is added (PF_DLSPEC: k_dl_spec takes the slot next).
// row: the slot's entry in the light-sample list (PathSoA::dlList): the batch's A / B column,
// the K / M scratch column and (without instances) the ray slots row + j * cap
template <int NB, int FEAT>
PGD_INLINE void dl_light_batches(const DevScene &S, const PathSoA &P, int slot, int row, Pushes &out) {
    constexpr int NQ = Bands<NB>::NQ;
    const size_t c = P.cap;
    uint32_t fl = P.flags[slot] & ~PF_DLNEE;
    const int d = P.bounce[slot];
    const bool all = S.dlStrategy != PBRTGPU_DL_ONE;
    const int K = all ? S.dlK : 1;
    const uint32_t hp = P.hp[slot], s = P.smp[slot];
    int k = (int)P.dlk[slot];
    const int rb = P.nInst ? slot : row;   // ray slots: the trace of an instanced scene finds the slot from them
    BSDF bs;
    V vp, vn, vwo;
    float vEps, vTime;
    {   // the vertex (its record is filled through out-of-line calls, so it lives in scratch
        // memory); the light samples read register copies of the fields they use
        DLVertex vx;
        dl_vertex<NB, FEAT, (FEAT & FEAT_TEX) != 0>(S, P, slot, d, vx, row);
        bs = vx.bs; vp = vx.p; vn = vx.n; vwo = vx.wo; vEps = vx.is.rayEps; vTime = vx.ray.time;
    }
    for (;;) {
        const int kEnd = min(k + P.dlBatch, K);
        uint32_t mA = 0u, mB = 0u;
        int lnOne = 0;
        for (int kk = k; kk < kEnd; ++kk) {
            const int jb = kk - k;
            float ul[3], ub[3];
            int j, ns;
            const int ln = dl_sample(S, hp, s, kk, ul, ub, &j, &ns);
            PowMemo pm;
            FVal F;
            uint32_t f2 = 0u;
            Pushes o2 = {false, false, false, 0u, 0u};
            estimate_direct<NB, FEAT>(S, P, row, rb + jb * (int)c, Col<float4>{P.A, (uint32_t)(jb * NQ * c + row)},
                                      Col<float4>{P.B, (uint32_t)(jb * NQ * c + row)}, ln, bs, pm, vp, vn, vwo,
                                      vEps, vTime, ul, ub, F, f2, o2, nullptr, nullptr, RAY_M);
            if (f2 & PF_PA) mA |= 1u << jb;
            if (f2 & PF_PB) mB |= 1u << jb;
            lnOne = ln;
        }
        if (mA | mB) {   // the next k_shade adds the batch
            out.sMask = mA;
            out.mMask = mB;
            fl |= PF_PEND | (all ? 0u : (uint32_t)lnOne << PF_LIGHT_SHIFT);
            P.dlMask[slot] = mA | (mB << 16);
            P.dlRow[slot] = (uint32_t)row;
            break;
        }
        // nothing queued: every ED of the batch is 0, added now
        for (int kk = k; kk < kEnd; ++kk)
            dl_add<NB>(S, P, slot, d, kk, K, all, false, false, P.A + slot, P.B + slot);
        k = kEnd;
        if (k < K) continue;
        fl |= PF_DLSPEC;
        break;
    }
    P.dlk[slot] = (uint32_t)k;
    P.flags[slot] = fl;
}

// L of frame d += (f * ((1 * Lr) + 0)) * |wi . n| / pdf: the completed child frame's radiance Lr
// into its parent d (integrator.cpp:199-200, 243-244; f, |wi . n| and pdf kept with the frame)
template <int NB>
PGD_INLINE void dl_pop(const PathSoA &P, int d, int slot, const float4 (&Lr)[Bands<NB>::NQ]) {
    constexpr int NQ = Bands<NB>::NQ;
    const size_t c = P.cap;
    float4 *Lv = dl_L<NB>(P, d, slot);
    const float4 *Fo = dl_F<NB>(P, d, slot);
    const float ad = P.fS[(size_t)2 * d * c + slot], pdf = P.fS[(size_t)(2 * d + 1) * c + slot];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        float4 l = Lv[q * c];
        const float4 f = Fo[q * c];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float li = (1.f * cmp(Lr[q], i)) + 0.f;
            cmp(l, i) += ((cmp(f, i) * li) * ad) / pdf;
        }
        Lv[q * c] = l;
    }
}

// k_dl_spec body for a slot marked PF_DLSPEC: SpecularReflect, then SpecularTransmit
// (integrator.cpp:169-250) of the top frame d -- each draws BSDFSample(rng) (3 MT19937 values,
// in the reference's order: reflect, its whole subtree, transmit) and queues its child ray with
// the ray differentials -- and, once a frame has no branch left, its pop into the parent and the
// parent's remaining branches, down to the camera sample's output at depth 0.
// Returns the ray requests; *done when the sample's radiance is in Lout.
// SPAWN = false (k_shade): only frames that cannot sample a specular child (not mirror or glass,
// or at maxdepth) are completed and popped -- the common case, cheap enough to run inline -- and
// the first frame that could branch is left to k_dl_spec (PF_DLSPEC).
template <int NB, int FEAT, bool SPAWN = true>
PGD_INLINE Pushes dl_spec_step(const DevScene &S, const PathSoA &P, int slot, float *__restrict__ Lout, bool *done,
                               bool *zeroed) {
    constexpr int NQ = Bands<NB>::NQ;
    const size_t c = P.cap;
    const float *sp = S.spectra;
    uint32_t fl = P.flags[slot] & ~PF_DLSPEC;
    int d = P.bounce[slot];
    Pushes out = {false, false, false, 0u, 0u};
    *done = false;
    *zeroed = false;
    MT rng;
    bool rngLoaded = false;
    for (;;) {
        // ---- the specular branches of frame d
        uint32_t br = P.fBr[(size_t)d * c + slot];
        bool spawned = false;
        // only mirror, glass and shinymetal have specular BxDFs: elsewhere the two BSDFSample(rng) draws
        // still happen (the reference constructs them) but no child can be sampled, and the
        // vertex need not be rebuilt
        const int vprim = P.fHit[(size_t)2 * d * c + slot];
        const int vtype = (*sa(S.mats, (uint32_t)((*sa(S.prims, (uint32_t)(vprim))).material))).type;
        const bool canSpec = vtype == PBRTGPU_MAT_MIRROR || vtype == PBRTGPU_MAT_GLASS || vtype == PBRTGPU_MAT_SHINYMETAL;
        if (!SPAWN && canSpec && d + 1 < S.maxDepth && br < 2u) {
            fl |= PF_DLSPEC;
            break;
        }
        while (d + 1 < S.maxDepth && br < 2u) {
            if (!rngLoaded) {
                mt_load(P, slot, fl, rng);
                if (!rng.init) mt_init(rng);
                rngLoaded = true;
            }
            const float u0 = mt_float(rng), u1 = mt_float(rng), uc = mt_float(rng);   // BSDFSample(rng)
            const bool refl = br == 0u;
            ++br;
            if (!SPAWN || !canSpec) continue;
            DLVertex vx;
            dl_vertex<NB, FEAT>(S, P, slot, d, vx, slot);
            const int flags = BSDF_SPECULAR | (refl ? BSDF_REFLECTION : BSDF_TRANSMISSION);
            FVal F;
            V wi;
            float pdf;
            (void)u0; (void)u1;   // the specular BxDFs ignore the two direction values
            bsdf_sample_specular(vx.bs, vx.wo, &wi, uc, &pdf, flags, F);
            if (!(pdf > 0.f)) continue;   // no matching BxDF: wi is not set
            const float ad = fabsf(vdot(wi, vx.n));
            if (ad == 0.f || (F.mode == FV_SUM && F.n == 0)) continue;
            float4 *mb = P.M + slot, *kb = P.K + slot;
            fval_prepare<NB, FEAT>(S, F, mb, c);
            float4 *Fo = dl_F<NB>(P, d, slot);
            bool black = true;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const float4 f = fval4<FEAT>(sp, F, q, mb, kb, c);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (4 * q + i < NB) black = black && (cmp(f, i) == 0.);
                Fo[q * c] = f;
            }
            if (black) continue;
            P.fS[(size_t)2 * d * c + slot] = ad;
            P.fS[(size_t)(2 * d + 1) * c + slot] = pdf;
            // the child ray and its differentials (the camera's rays always carry them)
            Ray cr;
            cr.o = vx.p; cr.d = wi; cr.mint = vx.is.rayEps; cr.maxt = INFINITY; cr.time = vx.ray.time;
            ray_store(P, RAY_C, slot, cr);
            const V n = vx.n, wo = vx.wo;
            const V rxo = vadd(vx.p, vx.dpdx), ryo = vadd(vx.p, vx.dpdy);
            const V dndx = vadd(vmul(vx.dn[0], vx.diff[0]), vmul(vx.dn[1], vx.diff[1]));
            const V dndy = vadd(vmul(vx.dn[0], vx.diff[2]), vmul(vx.dn[1], vx.diff[3]));
            const V dwodx = vsub(vneg(vx.rd.rxd), wo), dwody = vsub(vneg(vx.rd.ryd), wo);
            const float dDNdx = vdot(dwodx, n) + vdot(wo, dndx);
            const float dDNdy = vdot(dwody, n) + vdot(wo, dndy);
            V rxd, ryd;
            if (refl) {
                const float won = vdot(wo, n);
                rxd = vadd(vsub(wi, dwodx), vmul(vadd(vmul(dndx, won), vmul(n, dDNdx)), 2.f));
                ryd = vadd(vsub(wi, dwody), vmul(vadd(vmul(dndy, won), vmul(n, dDNdy)), 2.f));
            } else {
                // BSDF::eta: the glass material's index (a constant or its texture at the hit), 1
                // otherwise (glass.cpp:47-48)
                float eta = vx.bs.eta;
                const V w = vneg(wo);
                if (vdot(wo, n) < 0) eta = 1.f / eta;
                const float mu = eta * vdot(w, n) - vdot(wi, n);
                const float dmudx = (eta - (eta * eta * vdot(w, n)) / vdot(wi, n)) * dDNdx;
                const float dmudy = (eta - (eta * eta * vdot(w, n)) / vdot(wi, n)) * dDNdy;
                rxd = vsub(vadd(wi, vmul(dwodx, eta)), vadd(vmul(dndx, mu), vmul(n, dmudx)));
                ryd = vsub(vadd(wi, vmul(dwody, eta)), vadd(vmul(dndy, mu), vmul(n, dmudy)));
            }
            float *fd = P.fDiff + (size_t)(d + 1) * 12 * c + slot;
            dl_vec_store(fd, c, rxo);
            dl_vec_store(fd + 3 * c, c, rxd);
            dl_vec_store(fd + 6 * c, c, ryo);
            dl_vec_store(fd + 9 * c, c, ryd);
            fl |= PF_CONT;
            out.c = true;
            spawned = true;
            break;
        }
        P.fBr[(size_t)d * c + slot] = br;
        if (spawned) break;
        // ---- frame d is complete: Li = (1 * L) + 0 goes to its parent, or is the sample's
        float4 Lr[NQ];
        const float4 *Lv = dl_L<NB>(P, d, slot);
#pragma unroll
        for (int q = 0; q < NQ; ++q) Lr[q] = Lv[q * c];
        if (d == 0) {
            *zeroed = path_output<NB>(S, Lr, Lout, P.item[slot], P.smp[slot]);   // rayWeight * ((1 * L) + 0), guarded
            *done = true;
            break;
        }
        --d;
        dl_pop<NB>(P, d, slot, Lr);
    }
    if (rngLoaded) {
        mt_store(P, slot, rng);
        if (rng.init) fl |= PF_MTINIT;
    }
    P.bounce[slot] = d;
    P.flags[slot] = fl;
    return out;
}

// k_shade body of the DirectLighting integrator for one slot (see the file comment): the
// answers of the last pass -- a light-sample batch's shadow / MIS rays (added in sample order),
// or the camera / specular child ray (a hit pushes its frame, a miss pops straight into the
// parent) -- then the slot is handed to this pass's k_dl_nee (PF_DLNEE: the next light-sample
// batch) or k_dl_spec (PF_DLSPEC: the specular branches).  The specular branches and the
// frame pops they lead to run in k_dl_spec, a kernel of their own: inlined here they raised this
// step's register peak from 162 to ~330 VGPRs (559 spilled at 3 waves/SIMD).
// Returns the ray requests (none: the step queues no rays); *done when the camera ray missed
// and the sample's radiance is in Lout.
template <int NB, int FEAT>
PGD_INLINE Pushes shade_slot_dl(const DevScene &S, const PathSoA &P, int slot, float *__restrict__ Lout, bool *done,
                                bool *zeroed) {
    constexpr int NQ = Bands<NB>::NQ;
    const size_t c = P.cap;
    const float *sp = S.spectra;
    uint32_t fl = P.flags[slot];
    int d = P.bounce[slot];   // depth of the top frame (-1: camera ray in flight)
    Pushes out = {false, false, false, 0u, 0u};
    *done = false;
    *zeroed = false;
    const int nLights = S.nLights;
    const bool all = S.dlStrategy != PBRTGPU_DL_ONE;
    const int K = all ? S.dlK : 1;
    int k = (int)P.dlk[slot];
    bool spec;   // next: the specular branches (k_dl_spec), else a light-sample batch (k_dl_nee)
#ifdef PGD_DL_TRACE_ITEM   // debugging aid: the step of one item per pass
    const bool trc = P.item[slot] == PGD_DL_TRACE_ITEM;
    if (trc) printf("[dl] slot %d d %d fl %x k %d K %d prim %d occ %u hitM %d\n", slot, d, fl, k, K, P.hitPrim[slot],
                    P.occ[slot], P.hitPrim[P.rcap + slot]);
#endif
    if (fl & PF_PEND) {
        // ---- the answered batch of light samples [k, kEnd): ED = (0 [+ A]) [+ B] each
        // (EstimateDirect), added in sample order
        const uint32_t msk = P.dlMask[slot];
        const int row = (int)P.dlRow[slot], rb = P.nInst ? slot : row;   // the batch's row (dl_light_batches)
        const int kEnd = min(k + P.dlBatch, K);
        const int lnOne = (int)(fl >> PF_LIGHT_SHIFT);
        fl &= ~(PF_PEND | PF_PA | PF_PB | (PF_LIGHT_MASK << PF_LIGHT_SHIFT));
        for (int kk = k; kk < kEnd; ++kk) {
            const int jb = kk - k, rs = rb + jb * (int)c;
            int ln = lnOne;
            if (all) { int j, ns; dl_cursor(S, kk, &ln, &j, &ns); }
            const bool useA = ((msk >> jb) & 1u) && !P.occ[rs];
            bool useB = false;
            if ((msk >> (16 + jb)) & 1u) {
                const int mp = P.hitPrim[P.rcap + rs];
                if ((FEAT & FEAT_INF) && (*sa(S.lights, (uint32_t)(ln))).type == PBRTGPU_LIGHT_INFINITE) useB = mp < 0;
                else if (mp >= 0 && (*sa(S.prims, (uint32_t)(mp))).area_light == ln) {
                    const Ray mr = ray_load(P, RAY_M, rs);
                    useB = vdot(isect_nn(S, mr, mp, P.hitT[P.rcap + rs], inst_rec(P, slot)), vneg(mr.d)) > 0.f;
                }
            }
            dl_add<NB>(S, P, slot, d, kk, K, all, useA, useB, P.A + (size_t)jb * NQ * c + row,
                       P.B + (size_t)jb * NQ * c + row);
        }
        k = kEnd;
        spec = k >= K;
    } else {
        // ---- the camera ray or a specular child ray was answered (PF_CONT)
        fl &= ~PF_CONT;
        const int prim = P.hitPrim[slot];
        const Ray ray = ray_load(P, RAY_C, slot);
        if (prim < 0) {
            // SamplerRenderer::Li (samplerrenderer.cpp:237-240): Li = sum of the lights' Le
            float4 Lr[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) Lr[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if ((FEAT & FEAT_INF) && S.nInf > 0)
                for (int l = 0; l < nLights; ++l)
                    if ((*sa(S.lights, (uint32_t)(l))).type == PBRTGPU_LIGHT_INFINITE) {
                        const Emit e = inf_Le(S, (*sa(S.lights, (uint32_t)(l))), ray.d);
#pragma unroll
                        for (int q = 0; q < NQ; ++q) {
                            const float4 v = emit4<FEAT>(S, e, q);
                            Lr[q].x += v.x; Lr[q].y += v.y; Lr[q].z += v.z; Lr[q].w += v.w;
                        }
                    }
            if (d < 0) {   // the camera ray: rayWeight * ((1 * L) + 0), guarded
                *zeroed = path_output<NB>(S, Lr, Lout, P.item[slot], P.smp[slot]);
                *done = true;
                P.flags[slot] = fl;
                return out;
            }
            dl_pop<NB>(P, d, slot, Lr);   // the missing child's frame, popped at once
            spec = true;                  // the parent's remaining branches
        } else {
            // push frame d + 1: its incoming ray and hit; L = 0 + Le(wo)
            d = d + 1;
            float *fr = P.fRay + (size_t)d * 9 * c + slot;
            dl_vec_store(fr, c, ray.o);
            dl_vec_store(fr + 3 * c, c, ray.d);
            fr[6 * c] = ray.mint; fr[7 * c] = ray.maxt; fr[8 * c] = ray.time;
            P.fHit[(size_t)2 * d * c + slot] = prim;
            P.fHit[(size_t)(2 * d + 1) * c + slot] = __float_as_int(P.hitT[slot]);
            P.fBr[(size_t)d * c + slot] = 0u;
            k = 0;
            Isect is0;   // the hit alone decides the emission
            isect_fill(S, ray, prim, P.hitT[slot], is0, inst_rec(P, slot));
            const int al = is0.al;
            const int eo = (al >= 0 && vdot(is0.dg.nn, vneg(ray.d)) > 0.f) ? (*sa(S.lights, (uint32_t)(al))).spec : -1;   // AreaLight::L
            float4 *Lv = dl_L<NB>(P, d, slot);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const float4 e = eo >= 0 ? ld4(sp + eo + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                Lv[q * c] = make_float4(0.f + e.x, 0.f + e.y, 0.f + e.z, 0.f + e.w);
            }
            spec = nLights == 0;
        }
    }
#ifdef PGD_DL_TRACE_ITEM
    if (trc) printf("[dl]   -> d %d fl %x k %d spec %d\n", d, fl, k, (int)spec);
#endif
    P.bounce[slot] = d;
    P.dlk[slot] = (uint32_t)k;
    if (!spec) {
        P.flags[slot] = fl | PF_DLNEE;
        out.t = true;   // k_shade lists the slot for k_dl_nee
        return out;
    }
    // the top frame's branches: completed here if it cannot branch, else in k_dl_spec
    P.flags[slot] = fl;
    return dl_spec_step<NB, FEAT, false>(S, P, slot, Lout, done, zeroed);
}

}  // namespace pgd
