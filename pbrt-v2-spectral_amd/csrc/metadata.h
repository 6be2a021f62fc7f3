// metadata.h -- MetadataIntegrator::Li (integrators/metadata.cpp:41-80) as a wavefront shading
// step: k_shade<NB, FEAT, MODE_METADATA> runs it on each slot whose camera ray came back.  A
// hit reports Spectrum(primitiveId), Spectrum(materialId) (the ids the front end replays from
// the reference's Primitive / Material constructor counters, DevScene::primMeta) or
// Spectrum(|hit point - ray origin|); a miss is SamplerRenderer::Li's sum of the lights' Le
// (samplerrenderer.cpp:237-240).  One pass per path.
#pragma once
#include "wavefront.h"

namespace pgd {

template <int NB, int FEAT>
PGD_INLINE Pushes shade_slot_meta(const DevScene &S, const PathSoA &P, int slot, float *__restrict__ Lout, bool *done,
                                  bool *zeroed) {
    constexpr int NQ = Bands<NB>::NQ;
    const int prim = P.hitPrim[slot];
    const Ray ray = ray_load(P, RAY_C, slot);
    float4 L[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) L[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (prim < 0) {
        if ((FEAT & FEAT_INF) && S.nInf > 0)
            for (int l = 0; l < S.nLights; ++l)
                if ((*sa(S.lights, (uint32_t)(l))).type == PBRTGPU_LIGHT_INFINITE) {
                    const Emit e = inf_Le(S, (*sa(S.lights, (uint32_t)(l))), ray.d);
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const float4 v = emit4<FEAT>(S, e, q);
                        L[q].x += v.x; L[q].y += v.y; L[q].z += v.z; L[q].w += v.w;
                    }
                }
    } else {
        float v;
        if (S.metaStrategy == PBRTGPU_META_DEPTH) {
            Isect is;
            isect_fill(S, ray, prim, P.hitT[slot], is, inst_rec(P, slot));
            const V d = vsub(is.dg.p, ray.o);
            v = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
        } else
            v = (float)(*sa(S.primMeta, (uint32_t)(2 * prim + (S.metaStrategy == PBRTGPU_META_MATERIAL ? 1 : 0))));
#pragma unroll
        for (int q = 0; q < NQ; ++q) L[q] = make_float4(v, v, v, v);
    }
    // rayWeight * ((1 * Li) + 0), guarded (samplerrenderer.cpp:111-128)
    *zeroed = path_output<NB>(S, L, Lout, P.item[slot], P.smp[slot]);
    *done = true;
    return Pushes{false, false, false};
}

}  // namespace pgd
