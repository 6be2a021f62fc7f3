// pbrtgpu.hip -- MI355X (gfx950) spectral path-tracing core behind the C ABI of
// include/pbrtgpu.h.  Replaces SamplerRenderer::Render's task loop
// (renderers/samplerrenderer.cpp:60-222) for the "path" SurfaceIntegrator.
//
// Pipeline per pbrtgpu_render_tiles call:
//   k_spill_scan   : every sample of the sample extent -> imageX/Y footprint; samples that
//                    land on a film pixel of this context other than their own are queued
//                    (integer + float sampler work only, no tracing)
//   wavefront(spill keys) -> radiance of the spill samples
//   k_apply        : adds "pre" spill contributions (sources earlier in row-major order)
//   for each spp batch: wavefront(pixels x batch samples) -> Lbuf, then
//     k_accum<NB>  : film[p][band] += L in sample order (one lane per (pixel, band))
//   k_apply        : adds "post" spill contributions
// wavefront(items): persistent SoA path slots (wavefront.h); per pass
//   k_trace_closest (camera/continuation + MIS rays), k_trace_shadow, k_shade (+ regeneration)
// until every item has produced its radiance.
// The film is the reference's raw sum (spectralImage.cpp:267-296 does not normalise).
#include <hip/hip_runtime.h>
#include <vector>
#include <string>
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <mutex>
#include <thread>
#include <chrono>
#include <atomic>
#include "pbrtgpu.h"
#include "device.h"
#include "wavefront.h"
#include "scene_build.h"

using namespace pgd;
#ifdef PGD_SECTIONS
// weak: an experiment build may compile only some shade variants with PGD_SECTIONS
extern "C" {
__attribute__((weak)) int pgd_sections_read_32_0(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_32_8(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_32_9(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_32_7(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_60_0(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_60_6(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_60_7(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_30_0(unsigned long long *, int);
__attribute__((weak)) int pgd_sections_read_30_7(unsigned long long *, int);
}
static int pgd_sections_read(unsigned long long *out, int reset) {
    for (int k = 0; k < SEC_N; ++k) out[k] = 0;
    int e = 0;
    for (auto f : {pgd_sections_read_32_0, pgd_sections_read_32_8, pgd_sections_read_32_9, pgd_sections_read_32_7, pgd_sections_read_60_0, pgd_sections_read_60_6, pgd_sections_read_60_7,
                   pgd_sections_read_30_0, pgd_sections_read_30_7})
        if (f) e |= f(out, reset);
    return e;
}
#endif

namespace pgd {
// GPU linear BVH build (lbvh.hip)
int lbvh_build(hipStream_t stream, int n, const float *bounds, pbrtgpu_bvh_node *nodes_out, int32_t *order_out,
               double *ms_out, std::string *err);
// GPU Loop subdivision (loopsubdiv.hip)
int loop_subdivide(hipStream_t stream, int nf, int nv, const int32_t *vi, const float *P, int levels, int32_t *nv_out,
                   float *P_out, float *N_out, int32_t *vi_out, double *ms_out, std::string *err);
}
using pgd::lbvh_build;
using pgd::loop_subdivide;

static thread_local std::string g_err;
static int fail(int code, const std::string &msg) { g_err = msg; return code; }
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(-(1000 + (int)e_), std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)


// ------------------------------------------------------------------ kernels
#ifndef PGD_PASS_BATCH   // wavefront passes enqueued per counter read-back (<= 8)
#define PGD_PASS_BATCH 8
#endif
static_assert(PGD_PASS_BATCH >= 1 && PGD_PASS_BATCH <= 8, "Lane::ev holds the events of at most 8 passes");
#ifndef PGD_LBUF_GIB   // default per-sample radiance buffer of one spp batch (GiB); PBRTGPU_LBUF_MB overrides
#define PGD_LBUF_GIB 16   // C2: one 256-spp batch per frame (one drain instead of four): 265 -> 288 Mpaths/s
#endif
#ifndef PGD_TRACE_BLOCK
#define PGD_TRACE_BLOCK 128
#endif
static const int kTraceBlock = PGD_TRACE_BLOCK;
#ifndef PGD_STACK_LDS
#define PGD_STACK_LDS 8   // C2: 8 -> closest 161 -> 145 ms/frame vs 16 (r01m ablation)
#endif
static const int kStackLDS = PGD_STACK_LDS;
#ifndef PGD_DL_BATCH
#define PGD_DL_BATCH 8
#endif
static const int kDlBatch = PGD_DL_BATCH;   // DirectLighting light samples issued per pass (<= 16)
static_assert(PGD_DL_BATCH >= 1 && PGD_DL_BATCH <= 16, "the batch masks hold 16 samples");
// k_trace_pt: top-level wide nodes held in LDS per block.  Off: measured on C2 (r02k), the
// top levels are L1/L2-resident already and the LDS tile costs occupancy -- closest-hit
// 82 ms/frame without, 91 with 128 nodes, 113 with 256
#ifndef PGD_TOP_NODES
#define PGD_TOP_NODES 0
#endif
static const int kTopNodes = PGD_TOP_NODES;   // k_trace_pt: traversal-stack entries per lane kept in LDS (power of two)
#ifndef PGD_TRACE_ATTR   // occupancy experiments (tools/build_exp.sh)
#define PGD_TRACE_ATTR
#endif
#ifndef PGD_TRACE_S4_ATTR   // k_trace_s4 alone (experiments; r05g forced every trace kernel to 6 / 8 waves)
#define PGD_TRACE_S4_ATTR PGD_TRACE_ATTR
#endif
#ifndef PGD_TRACE_INST_ATTR   // the two-level kernel: the instance transform's peak would give 148 VGPRs (3 waves)
#define PGD_TRACE_INST_ATTR __attribute__((amdgpu_waves_per_eu(4, 8)))
#endif

// closest-hit queries of one pass (BVHAccel::Intersect, bvh.cpp:380-432): persistent grid,
// one ray per lane per iteration, LDS traversal stack (column per lane)
template <bool STATS, bool INST>
__global__ __launch_bounds__(kTraceBlock) void k_trace_closest(DevScene S, PathSoA P, int q) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.tbase = reinterpret_cast<float *>(lds + (size_t)S.stackDepth * blockDim.x) + threadIdx.x;
    st.stride = blockDim.x;
    const uint32_t n = P.cnt[CNT_QC(q)];
    const uint32_t *Q = P.qC + (size_t)q * 2 * P.rcap;
    uint32_t nM = 0, hM = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t e = Q[i];
        const int slot = (int)(e >> 1), kind = (int)(e & 1);
        Ray r = ray_load(P, rec_kind(S, q, kind), slot);
        int prim = -1;
        float t = INFINITY;
        if (!bvh_intersect<INST>(S, st, r, &prim, &t)) prim = -1;
        P.hitPrim[(size_t)kind * P.rcap + slot] = prim;
        P.hitT[(size_t)kind * P.rcap + slot] = t;
        if (STATS && kind == RAY_M) { nM++; hM += prim >= 0 ? 1u : 0u; }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        atomicAdd(&w[W_RAYS], (unsigned long long)st.cRays);
        atomicAdd(&w[W_NODES_C], (unsigned long long)st.cNodes);
        atomicAdd(&w[W_TRIS_C], (unsigned long long)st.cTris);
        atomicAdd(&w[W_QUADS_C], (unsigned long long)st.cQuads);
        atomicAdd(&w[W_HITS], (unsigned long long)st.cHits);
        atomicAdd(&w[W_RAYS_M], (unsigned long long)nM);
        atomicAdd(&w[W_HITS_M], (unsigned long long)hM);
    }
}

// any-hit queries of one pass (BVHAccel::IntersectP, bvh.cpp:435-481)
template <bool STATS, bool INST>
__global__ __launch_bounds__(kTraceBlock) void k_trace_shadow(DevScene S, PathSoA P, int q) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.tbase = reinterpret_cast<float *>(lds + (size_t)S.stackDepth * blockDim.x) + threadIdx.x;
    st.stride = blockDim.x;
    const uint32_t n = P.cnt[CNT_QS(q)];
    const uint32_t *Q = P.qS + (size_t)q * P.rcap;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int slot = (int)Q[i];
        Ray r = ray_load(P, RAY_S, slot);
        P.occ[slot] = bvh_intersectP<INST>(S, st, r) ? 1u : 0u;
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        atomicAdd(&w[W_SHADOW], (unsigned long long)st.cShadow);
        atomicAdd(&w[W_NODES_S], (unsigned long long)st.cNodes);
        atomicAdd(&w[W_TRIS_S], (unsigned long long)st.cTris);
        atomicAdd(&w[W_QUADS_S], (unsigned long long)st.cQuads);
    }
}

// Ray queries of one pass without instanced primitives (BVHAccel::Intersect / IntersectP,
// bvh.cpp:380-481, on the child-in-parent BVH of bvh_walk): persistent waves, each owning a
// contiguous range of the queue, with per-lane ray replacement -- a lane whose ray has
// finished takes the next ray of the wave's range once `refill` lanes are idle, so lanes
// do not sit out the longest ray of a batch (SIMD efficiency of the incoherent secondary
// rays).  One loop trip is one traversal step: an interior node (both children tested) and
// then, if the lane stands on a leaf, that leaf's primitives.  Per ray the nodes visited,
// primitives tested and their order are bvh_walk's.
// The persistent trace waves own contiguous ranges of the queue, in wave order.  Blocks are dealt
// round-robin over the 8 XCDs (blocks b, b + 8, ... share one, MI355X_MICROARCH.md "Workgroup
// dispatch"), so with the plain order every XCD traces rays from every stretch of the queue and
// its 4 MiB L2 holds the BVH nodes and triangles of the whole image region the pass covers.  With
// xcdMap the blocks of one XCD take one contiguous eighth of the queue: queue order follows slot
// order, and slots follow the pixel order of the items they took, so an XCD's rays come from
// neighbouring pixels (and their paths) and share the part of the scene they see.  Speed only:
// any block-to-XCD placement gives the same answers.  Measured (r05b, C2, two interleaved rounds):
// L2 hits and misses of both trace kernels unchanged to 0.2 %, closest 76 -> 82 ms and shadow
// 40 -> 46 ms per frame (the blocks that share a CU get neighbouring ranges of correlated cost),
// 492 -> 471 Mpaths/s; so it is off unless PBRTGPU_XCD_MAP=1.
PGD_INLINE uint32_t trace_wave(int xcdMap) {
    uint32_t b = blockIdx.x;
    const uint32_t nb = gridDim.x;
    if (xcdMap && (nb & 7u) == 0u) b = (b & 7u) * (nb >> 3) + (b >> 3);
    return (b * blockDim.x + threadIdx.x) >> 6;
}

template <bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) PGD_TRACE_ATTR void k_trace_pt(DevScene S, PathSoA P, int q, int refill, int ring, uint2 *__restrict__ spill) {
    // traversal stack: the top kStackLDS entries of each lane in LDS (a ring, column per
    // lane: refs, then entry distances), deeper entries in the lane's spill area in HBM
    __shared__ uint32_t sref[kStackLDS * kTraceBlock];
    __shared__ float stm[ANY ? 1 : kStackLDS * kTraceBlock];
    // the top levels of the BVH (wide nodes [0, S.nTop), breadth-first), once per block
    __shared__ float4 stop[kTopNodes > 0 ? 4 * kTopNodes : 1];
    if (kTopNodes > 0) {
        for (int i = threadIdx.x; i < 4 * S.nTop; i += blockDim.x) stop[i] = (*sa(S.wnodes, (uint32_t)(i)));
        __syncthreads();
    }
    uint2 *gsp = spill + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * S.stackDepth;
    int bottom = 0;   // entries [0, bottom) live in gsp
    Stack st;         // work counters only
    const uint32_t n = ANY ? P.cnt[CNT_QS(q)] : P.cnt[CNT_QC(q)];
    const uint32_t *Q = ANY ? P.qS + (size_t)q * P.rcap : P.qC + (size_t)q * 2 * P.rcap;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = trace_wave(P.xcdMap), nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t next = (uint32_t)((uint64_t)n * wave / nw);
    const uint32_t end = (uint32_t)((uint64_t)n * (wave + 1) / nw);
    bool active = false;
    int slot = 0, kind = 0, todo = 0, prim = -1;
    uint32_t ref = 0;
    float thit = INFINITY;
    Ray ray;
    V invDir = v3(0.f, 0.f, 0.f);
    int neg[3] = {0, 0, 0};
    uint32_t negMask = 0;
    uint32_t nM = 0, hM = 0;
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nIdle = (uint32_t)__popcll(idle);
        if (next < end && (nIdle >= (uint32_t)refill || nIdle == 64u)) {
            if (!active) {
                const uint32_t i = next + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (i < end) {
                    const uint32_t e = Q[i];
                    slot = ANY ? (int)e : (int)(e >> 1);
                    kind = ANY ? RAY_S : (int)(e & 1);
                    ray = ray_load(P, rec_kind(S, q, kind), slot);
                    invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
                    neg[0] = invDir.x < 0; neg[1] = invDir.y < 0; neg[2] = invDir.z < 0;
                    negMask = (uint32_t)neg[0] | ((uint32_t)neg[1] << 1) | ((uint32_t)neg[2] << 2);
                    prim = -1;
                    thit = INFINITY;
                    todo = 0;
                    bottom = 0;
                    if (ANY) st.cShadow++; else st.cRays++;
                    st.cNodes++;
                    if (bbox_hit((*sa(S.nodes, (uint32_t)(0))), (*sa(S.nodes, (uint32_t)(1))), ray, invDir, neg)) {
                        ref = (*sa(S.nodeRef, (uint32_t)(0)));
                        active = true;
                    } else if (ANY) P.occ[slot] = 0u;
                    else {
                        P.hitPrim[(size_t)kind * P.rcap + slot] = -1;
                        P.hitT[(size_t)kind * P.rcap + slot] = INFINITY;
                        if (STATS && kind == RAY_M) nM++;
                    }
                }
            }
            next = min(end, next + nIdle);
        }
        if (!__ballot(active)) {
            if (next >= end) break;
            continue;
        }
        if (active) {
            bool done = false, occluded = false;
            if (!(ref & WREF_LEAF)) {
                float4 l0, l1, r0, r1;
                if (kTopNodes > 0 && ref < (uint32_t)S.nTop) {
                    const float4 *w = stop + 4 * ref;
                    l0 = w[0]; l1 = w[1]; r0 = w[2]; r1 = w[3];
                } else {
                    const float4 *w = sa(S.wnodes, (uint32_t)(4 * (size_t)ref));
                    l0 = w[0]; l1 = w[1]; r0 = w[2]; r1 = w[3];
                }
                st.cNodes++;
                float tl = 0.f, tr = 0.f;
                const bool hl = slab_enter_bf(l0, l1, ray, invDir, neg, &tl) & (tl < ray.maxt);
                const bool hr = slab_enter_bf(r0, r1, ray, invDir, neg, &tr) & (tr < ray.maxt);
                const uint32_t refL = __float_as_uint(l0.w), refR = __float_as_uint(l1.w);
                const bool swap = ((negMask >> __float_as_uint(r0.w)) & 1u) != 0;   // no indexed private array
                const bool hn = swap ? hr : hl, hf = swap ? hl : hr;
                const uint32_t rn = swap ? refR : refL, rf = swap ? refL : refR;
                if (hn) {
                    if (hf) {
                        if (todo - bottom == ring) {   // ring full: oldest entry to HBM
                            const int j = (bottom & (ring - 1)) * kTraceBlock + threadIdx.x;
                            gsp[bottom] = make_uint2(sref[j], ANY ? 0u : __float_as_uint(stm[j]));
                            ++bottom;
                        }
                        const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
                        sref[j] = rf;
                        if (!ANY) stm[j] = swap ? tl : tr;
                        ++todo;
                    }
                    ref = rn;
                } else if (hf) ref = rf;
                else ref = 0xffffffffu;   // pop below
            }
            if (ref != 0xffffffffu && (ref & WREF_LEAF)) {
                const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
                for (uint32_t i = 0; i < np; ++i)
                    if (prim_test<ANY, false>(S, st, todo, (int)(off + i), ray, &prim, &thit) && ANY) {
                        occluded = true;
                        break;
                    }
                ref = 0xffffffffu;
            }
            if (occluded) done = true;
            else if (ref == 0xffffffffu) {
                done = true;
                while (todo > 0) {
                    --todo;
                    uint32_t r;
                    float tm;
                    if (todo < bottom) {
                        const uint2 g = gsp[todo];
                        r = g.x; tm = __uint_as_float(g.y);
                        bottom = todo;
                    } else {
                        const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
                        r = sref[j]; tm = ANY ? 0.f : stm[j];
                    }
                    if (ANY || tm < ray.maxt) { ref = r; done = false; break; }
                }
            }
            if (done) {
                active = false;
                if (ANY) P.occ[slot] = occluded ? 1u : 0u;
                else {
                    P.hitPrim[(size_t)kind * P.rcap + slot] = prim;
                    P.hitT[(size_t)kind * P.rcap + slot] = prim >= 0 ? thit : INFINITY;
                    st.cHits += prim >= 0 ? 1u : 0u;
                    if (STATS && kind == RAY_M) { nM++; hM += prim >= 0 ? 1u : 0u; }
                }
            }
        }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        if (ANY) {
            atomicAdd(&w[W_SHADOW], (unsigned long long)st.cShadow);
            atomicAdd(&w[W_NODES_S], (unsigned long long)st.cNodes);
            atomicAdd(&w[W_TRIS_S], (unsigned long long)st.cTris);
            atomicAdd(&w[W_QUADS_S], (unsigned long long)st.cQuads);
        } else {
            atomicAdd(&w[W_RAYS], (unsigned long long)st.cRays);
            atomicAdd(&w[W_NODES_C], (unsigned long long)st.cNodes);
            atomicAdd(&w[W_TRIS_C], (unsigned long long)st.cTris);
            atomicAdd(&w[W_QUADS_C], (unsigned long long)st.cQuads);
            atomicAdd(&w[W_HITS], (unsigned long long)st.cHits);
            atomicAdd(&w[W_RAYS_M], (unsigned long long)nM);
            atomicAdd(&w[W_HITS_M], (unsigned long long)hM);
        }
    }
}

// Shadow queries of one pass on the 4-wide BVH copy (BVHAccel::IntersectP, bvh.cpp:435-481;
// scene_build.h wide4_bvh): k_trace_pt<true>'s persistent ray-replacement scheme, one 4-wide node
// per loop trip -- its up to four child boxes tested with the reference's slab test, the first hit
// child taken next and the others pushed -- then, on a leaf, its primitives until one is hit.  The
// answer (occluded or not) is the reference's: the primitives whose boxes all pass are the same
// (wide4_bvh), and any-hit does not depend on the order they are tested in.  Half as many
// dependent node loads per ray as the binary walk.
template <bool STATS>
__global__ __launch_bounds__(kTraceBlock) PGD_TRACE_S4_ATTR void k_trace_s4(DevScene S, PathSoA P, int q, int refill, int ring, uint2 *__restrict__ spill) {
    __shared__ uint32_t sref[kStackLDS * kTraceBlock];
    uint2 *gsp = spill + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * S.w4Stack;
    int bottom = 0;
    Stack st;
    const uint32_t n = P.cnt[CNT_QS(q)];
    const uint32_t *Q = P.qS + (size_t)q * P.rcap;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = trace_wave(P.xcdMap), nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t next = (uint32_t)((uint64_t)n * wave / nw);
    const uint32_t end = (uint32_t)((uint64_t)n * (wave + 1) / nw);
    bool active = false;
    int slot = 0, todo = 0, prim = -1;
    uint32_t ref = 0;
    float thit = INFINITY;
    Ray ray;
    V invDir = v3(0.f, 0.f, 0.f);
    int neg[3] = {0, 0, 0};
    const uint32_t NONE = 0xffffffffu;
    auto push = [&](uint32_t r) {
        if (todo - bottom == ring) {   // ring full: oldest entry to HBM
            gsp[bottom] = make_uint2(sref[(bottom & (ring - 1)) * kTraceBlock + threadIdx.x], 0u);
            ++bottom;
        }
        sref[(todo & (ring - 1)) * kTraceBlock + threadIdx.x] = r;
        ++todo;
    };
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nIdle = (uint32_t)__popcll(idle);
        if (next < end && (nIdle >= (uint32_t)refill || nIdle == 64u)) {
            if (!active) {
                const uint32_t i = next + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (i < end) {
                    slot = (int)Q[i];
                    ray = ray_load(P, RAY_S, slot);
                    invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
                    neg[0] = invDir.x < 0; neg[1] = invDir.y < 0; neg[2] = invDir.z < 0;
                    prim = -1;
                    thit = INFINITY;
                    todo = 0;
                    bottom = 0;
                    st.cShadow++;
                    st.cNodes++;
                    if (bbox_hit((*sa(S.nodes, (uint32_t)(0))), (*sa(S.nodes, (uint32_t)(1))), ray, invDir, neg)) {
                        ref = 0u;   // the 4-wide root (the root's grandchildren)
                        active = true;
                    } else P.occ[slot] = 0u;
                }
            }
            next = min(end, next + nIdle);
        }
        if (!__ballot(active)) {
            if (next >= end) break;
            continue;
        }
        if (active) {
            bool occluded = false;
            if (!(ref & WREF_LEAF)) {
                const float4 *w = sa(S.w4nodes, (uint32_t)(8 * (size_t)ref));
                float4 b[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) b[k] = w[k];
                st.cNodes++;
                uint32_t nxt = NONE;
                bool h[4];   // the four tests first, straight-line (slab_enter_bf)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float t = 0.f;
                    h[k] = (__float_as_uint(b[2 * k].w) != NONE) & slab_enter_bf(b[2 * k], b[2 * k + 1], ray, invDir, neg, &t) &
                           (t < ray.maxt);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t r = __float_as_uint(b[2 * k].w);
                    if (h[k]) {
                        if (nxt == NONE) nxt = r;
                        else push(r);
                    }
                }
                ref = nxt;
            }
            if (ref != NONE && (ref & WREF_LEAF)) {
                const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
                for (uint32_t i = 0; i < np; ++i)
                    if (prim_test<true, false>(S, st, todo, (int)(off + i), ray, &prim, &thit)) {
                        occluded = true;
                        break;
                    }
                ref = NONE;
            }
            bool done = occluded;
            if (!occluded && ref == NONE) {
                if (todo > 0) {
                    --todo;
                    if (todo < bottom) {
                        ref = gsp[todo].x;
                        bottom = todo;
                    } else ref = sref[(todo & (ring - 1)) * kTraceBlock + threadIdx.x];
                } else done = true;
            }
            if (done) {
                active = false;
                P.occ[slot] = occluded ? 1u : 0u;
            }
        }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        atomicAdd(&w[W_SHADOW], (unsigned long long)st.cShadow);
        atomicAdd(&w[W_NODES_S], (unsigned long long)st.cNodes);
        atomicAdd(&w[W_TRIS_S], (unsigned long long)st.cTris);
        atomicAdd(&w[W_QUADS_S], (unsigned long long)st.cQuads);
    }
}

// Shadow queries of one pass on the QUANTIZED 4-wide copy (scene_build.h quant_w4: 64 B per node,
// 8-bit child boxes relative to the node's origin): k_trace_s4's persistent ray-replacement walk,
// descending on the children's outer (containing) boxes; a stack entry keeps a "certain" bit while
// every box on its path passed its inner (contained) test too, which implies the exact box passes.
// A primitive hit in a certain leaf occludes; a hit in an uncertain leaf occludes only if the
// leaf's binary ancestors' exact boxes all pass (leaf_reached) -- then the reference's IntersectP,
// whose answer depends only on the leaves its exact box tests reach (maxt is fixed), reaches it.
template <bool STATS>
__global__ __launch_bounds__(kTraceBlock) PGD_TRACE_ATTR void k_trace_s4q(DevScene S, PathSoA P, int q, int refill, int ring, uint2 *__restrict__ spill) {
    __shared__ uint32_t sref[kStackLDS * kTraceBlock];
    uint2 *gsp = spill + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * S.w4Stack;
    int bottom = 0;
    Stack st;
    const uint32_t n = P.cnt[CNT_QS(q)];
    const uint32_t *Q = P.qS + (size_t)q * P.rcap;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = trace_wave(P.xcdMap), nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t next = (uint32_t)((uint64_t)n * wave / nw);
    const uint32_t end = (uint32_t)((uint64_t)n * (wave + 1) / nw);
    bool active = false;
    int slot = 0, todo = 0, prim = -1;
    uint32_t ref = 0;   // a stack entry: ref | WQ_CERT
    float thit = INFINITY;
    Ray ray;
    V invDir = v3(0.f, 0.f, 0.f);
    int neg[3] = {0, 0, 0};
    const uint32_t NONE = 0xffffffffu;
    auto push = [&](uint32_t r) {
        if (todo - bottom == ring) {   // ring full: oldest entry to HBM
            gsp[bottom] = make_uint2(sref[(bottom & (ring - 1)) * kTraceBlock + threadIdx.x], 0u);
            ++bottom;
        }
        sref[(todo & (ring - 1)) * kTraceBlock + threadIdx.x] = r;
        ++todo;
    };
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nIdle = (uint32_t)__popcll(idle);
        if (next < end && (nIdle >= (uint32_t)refill || nIdle == 64u)) {
            if (!active) {
                const uint32_t i = next + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (i < end) {
                    slot = (int)Q[i];
                    ray = ray_load(P, RAY_S, slot);
                    invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
                    neg[0] = invDir.x < 0; neg[1] = invDir.y < 0; neg[2] = invDir.z < 0;
                    prim = -1;
                    thit = INFINITY;
                    todo = 0;
                    bottom = 0;
                    st.cShadow++;
                    st.cNodes++;
                    if (bbox_hit((*sa(S.nodes, (uint32_t)(0))), (*sa(S.nodes, (uint32_t)(1))), ray, invDir, neg)) {
                        ref = 0u | WQ_CERT;   // the quantized root (the root's grandchildren); its box passed exactly
                        active = true;
                    } else P.occ[slot] = 0u;
                }
            }
            next = min(end, next + nIdle);
        }
        if (!__ballot(active)) {
            if (next >= end) break;
            continue;
        }
        if (active) {
            bool occluded = false;
            const bool cert = (ref & WQ_CERT) != 0u;
            const uint32_t r0 = ref & ~WQ_CERT;
            if (!(r0 & WREF_LEAF)) {
                const uint4 *w = sa(S.w4q, (uint32_t)(4 * (size_t)r0));
                const uint4 q0 = w[0], q1 = w[1], q2 = w[2], q3 = w[3];
                const uint32_t refs[4] = {q2.z, q2.w, q3.x, q3.y};
                st.cNodes++;
                uint32_t nxt = NONE;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float4 olo, ohi, ilo, ihi;
                    wq_boxes(q0, q1, q2, q3, k, &olo, &ohi, &ilo, &ihi);
                    float t = 0.f, ti = 0.f;
                    if (refs[k] != NONE && slab_enter(olo, ohi, ray, invDir, neg, &t) && t < ray.maxt) {
                        const bool c = cert && slab_enter(ilo, ihi, ray, invDir, neg, &ti) && ti < ray.maxt;
                        const uint32_t e = refs[k] | (c ? WQ_CERT : 0u);
                        if (nxt == NONE) nxt = e;
                        else push(e);
                    }
                }
                ref = nxt;
            }
            if (ref != NONE && (ref & WREF_LEAF)) {
                const bool lc = (ref & WQ_CERT) != 0u;
                const uint32_t lr = ref & ~WQ_CERT;
                const uint32_t np = (lr >> WREF_NP_SHIFT) & 0x3fu, off = lr & WREF_OFF_MASK;
                for (uint32_t i = 0; i < np; ++i)
                    if (prim_test<true, false>(S, st, todo, (int)(off + i), ray, &prim, &thit)) {
                        occluded = lc || leaf_reached(S, ray, invDir, neg, (*sa(S.leafOf, off)));
                        break;   // a hit in a leaf the reference never tests: the walk goes on
                    }
                ref = NONE;
            }
            bool done = occluded;
            if (!occluded && ref == NONE) {
                if (todo > 0) {
                    --todo;
                    if (todo < bottom) {
                        ref = gsp[todo].x;
                        bottom = todo;
                    } else ref = sref[(todo & (ring - 1)) * kTraceBlock + threadIdx.x];
                } else done = true;
            }
            if (done) {
                active = false;
                P.occ[slot] = occluded ? 1u : 0u;
            }
        }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        atomicAdd(&w[W_SHADOW], (unsigned long long)st.cShadow);
        atomicAdd(&w[W_NODES_S], (unsigned long long)st.cNodes);
        atomicAdd(&w[W_TRIS_S], (unsigned long long)st.cTris);
        atomicAdd(&w[W_QUADS_S], (unsigned long long)st.cQuads);
    }
}

// Closest-hit queries of one pass (camera / continuation and MIS rays) on the 4-wide BVH copy
// (BVHAccel::Intersect, bvh.cpp:380-434; scene_build.h wide4_bvh): k_trace_pt<false>'s persistent
// ray-replacement scheme, one 4-wide node per loop trip -- its child boxes tested, taken in the
// binary walk's order (w4_order), the first passing child next and the others pushed with their
// entry distances, re-checked against the then-current maxt when popped.  The primitives tested
// and their order are the binary walk's (bvh_intersect4 is the same walk, replayed on the host
// against the oracle), with half as many dependent node loads per ray.
template <bool STATS>
__global__ __launch_bounds__(kTraceBlock) PGD_TRACE_ATTR void k_trace_c4(DevScene S, PathSoA P, int q, int refill, int ring, uint2 *__restrict__ spill) {
    __shared__ uint32_t sref[kStackLDS * kTraceBlock];
    __shared__ float stm[kStackLDS * kTraceBlock];
    uint2 *gsp = spill + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * S.w4Stack;
    int bottom = 0;
    Stack st;
    const uint32_t n = P.cnt[CNT_QC(q)];
    const uint32_t *Q = P.qC + (size_t)q * 2 * P.rcap;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = trace_wave(P.xcdMap), nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t next = (uint32_t)((uint64_t)n * wave / nw);
    const uint32_t end = (uint32_t)((uint64_t)n * (wave + 1) / nw);
    bool active = false;
    int slot = 0, kind = 0, todo = 0, prim = -1;
    uint32_t ref = 0;
    float thit = INFINITY;
    Ray ray;
    V invDir = v3(0.f, 0.f, 0.f);
    int neg[3] = {0, 0, 0};
    uint32_t negMask = 0;
    uint32_t nM = 0, hM = 0;
    const uint32_t NONE = 0xffffffffu;
    auto push = [&](uint32_t r, float t) {
        if (todo - bottom == ring) {   // ring full: oldest entry to HBM
            const int j = (bottom & (ring - 1)) * kTraceBlock + threadIdx.x;
            gsp[bottom] = make_uint2(sref[j], __float_as_uint(stm[j]));
            ++bottom;
        }
        const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
        sref[j] = r;
        stm[j] = t;
        ++todo;
    };
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nIdle = (uint32_t)__popcll(idle);
        if (next < end && (nIdle >= (uint32_t)refill || nIdle == 64u)) {
            if (!active) {
                const uint32_t i = next + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (i < end) {
                    const uint32_t e = Q[i];
                    slot = (int)(e >> 1);
                    kind = (int)(e & 1);
                    ray = ray_load(P, rec_kind(S, q, kind), slot);
                    invDir = v3(1.f / ray.d.x, 1.f / ray.d.y, 1.f / ray.d.z);
                    neg[0] = invDir.x < 0; neg[1] = invDir.y < 0; neg[2] = invDir.z < 0;
                    negMask = (uint32_t)neg[0] | ((uint32_t)neg[1] << 1) | ((uint32_t)neg[2] << 2);
                    prim = -1;
                    thit = INFINITY;
                    todo = 0;
                    bottom = 0;
                    st.cRays++;
                    st.cNodes++;
                    if (bbox_hit((*sa(S.nodes, (uint32_t)(0))), (*sa(S.nodes, (uint32_t)(1))), ray, invDir, neg)) {
                        ref = 0u;   // the 4-wide root (the root's grandchildren)
                        active = true;
                    } else {
                        P.hitPrim[(size_t)kind * P.rcap + slot] = -1;
                        P.hitT[(size_t)kind * P.rcap + slot] = INFINITY;
                        if (STATS && kind == RAY_M) nM++;
                    }
                }
            }
            next = min(end, next + nIdle);
        }
        if (!__ballot(active)) {
            if (next >= end) break;
            continue;
        }
        if (active) {
            if (!(ref & WREF_LEAF)) {
                const float4 *w = sa(S.w4nodes, (uint32_t)(8 * (size_t)ref));
                const float4 b0 = w[0], b1 = w[1], b2 = w[2], b3 = w[3], b4 = w[4], b5 = w[5], b6 = w[6], b7 = w[7];
                st.cNodes++;
                // the four slots' tests, then their refs / hits / entries in the binary walk's order
                float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
                const uint32_t r0 = __float_as_uint(b0.w), r1 = __float_as_uint(b2.w), r2 = __float_as_uint(b4.w),
                               r3 = __float_as_uint(b6.w);
                // the four tests and the selections by slot as straight-line value selects (slab_enter_bf):
                // a hit flag per slot in a bit mask, refs and entry distances picked by index
                const bool h0 = (r0 != NONE) & slab_enter_bf(b0, b1, ray, invDir, neg, &e0) & (e0 < ray.maxt);
                const bool h1 = (r1 != NONE) & slab_enter_bf(b2, b3, ray, invDir, neg, &e1) & (e1 < ray.maxt);
                const bool h2 = (r2 != NONE) & slab_enter_bf(b4, b5, ray, invDir, neg, &e2) & (e2 < ray.maxt);
                const bool h3 = (r3 != NONE) & slab_enter_bf(b6, b7, ray, invDir, neg, &e3) & (e3 < ray.maxt);
                const uint32_t hm = (uint32_t)h0 | ((uint32_t)h1 << 1) | ((uint32_t)h2 << 2) | ((uint32_t)h3 << 3);
                const uint32_t ord = w4_order(__float_as_uint(b1.w), negMask);
                // slot sl's ref / entry distance by two bit selects (a compare chain compiled to branches)
                auto pr = [&](uint32_t sl) {
                    const uint32_t lo = (sl & 1u) ? r1 : r0, hi = (sl & 1u) ? r3 : r2;
                    return (sl & 2u) ? hi : lo;
                };
                auto ph = [&](uint32_t sl) { return ((hm >> sl) & 1u) != 0u; };
                auto pe = [&](uint32_t sl) {
                    const float lo = (sl & 1u) ? e1 : e0, hi = (sl & 1u) ? e3 : e2;
                    return (sl & 2u) ? hi : lo;
                };
                const uint32_t s0 = ord & 3u, s1 = (ord >> 2) & 3u, s2 = (ord >> 4) & 3u, s3 = (ord >> 6) & 3u;
                const bool k0 = ph(s0), k1 = ph(s1), k2 = ph(s2), k3 = ph(s3);
                const int first = k0 ? 0 : k1 ? 1 : k2 ? 2 : k3 ? 3 : 4;
                const uint32_t q1 = pr(s1), q2 = pr(s2), q3 = pr(s3);
                const float t1 = pe(s1), t2 = pe(s2), t3 = pe(s3);
                if (k3 & (first < 3)) push(q3, t3);
                if (k2 & (first < 2)) push(q2, t2);
                if (k1 & (first < 1)) push(q1, t1);
                const uint32_t f01 = first == 0 ? pr(s0) : q1, f23 = first == 2 ? q2 : (first == 3 ? q3 : NONE);
                ref = first < 2 ? f01 : f23;
            }
            if (ref != NONE && (ref & WREF_LEAF)) {
                const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
                for (uint32_t i = 0; i < np; ++i) prim_test<false, false>(S, st, todo, (int)(off + i), ray, &prim, &thit);
                ref = NONE;
            }
            bool done = false;
            if (ref == NONE) {
                done = true;
                while (todo > 0) {
                    --todo;
                    uint32_t r;
                    float tm;
                    if (todo < bottom) {
                        const uint2 g = gsp[todo];
                        r = g.x; tm = __uint_as_float(g.y);
                        bottom = todo;
                    } else {
                        const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
                        r = sref[j]; tm = stm[j];
                    }
                    if (tm < ray.maxt) { ref = r; done = false; break; }
                }
            }
            if (done) {
                active = false;
                P.hitPrim[(size_t)kind * P.rcap + slot] = prim;
                P.hitT[(size_t)kind * P.rcap + slot] = prim >= 0 ? thit : INFINITY;
                st.cHits += prim >= 0 ? 1u : 0u;
                if (STATS && kind == RAY_M) { nM++; hM += prim >= 0 ? 1u : 0u; }
            }
        }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        atomicAdd(&w[W_RAYS], (unsigned long long)st.cRays);
        atomicAdd(&w[W_NODES_C], (unsigned long long)st.cNodes);
        atomicAdd(&w[W_TRIS_C], (unsigned long long)st.cTris);
        atomicAdd(&w[W_QUADS_C], (unsigned long long)st.cQuads);
        atomicAdd(&w[W_HITS], (unsigned long long)st.cHits);
        atomicAdd(&w[W_RAYS_M], (unsigned long long)nM);
        atomicAdd(&w[W_HITS_M], (unsigned long long)hM);
    }
}

// Ray queries of one pass WITH instanced primitives (TransformedPrimitive over nested BVHs,
// primitive.cpp:87-116, C5): k_trace_pt's persistent ray-replacement scheme with a two-level
// walk per lane.  Level 0 walks the top-level BVH in world space; a top-level leaf's
// primitives are tested in order, and an instance among them moves the lane to level 1:
// the ray is transformed to primitive space at ray.time (AnimatedTransform::Interpolate) and
// the instance's nested BVH is walked with the stack entries above `ibase`.  When that walk
// runs out of entries the lane returns to level 0 with the shrunken maxt (closest hit) and
// resumes the leaf after the instance.  Per ray the nodes visited, the primitives tested and
// their order are bvh_walk<ANY, true>'s; entry distances are parametric t, the same in both
// spaces.
template <bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) PGD_TRACE_INST_ATTR void k_trace_inst(DevScene S, PathSoA P, int q, int refill, int ring, uint2 *__restrict__ spill) {
    __shared__ uint32_t sref[kStackLDS * kTraceBlock];
    __shared__ float stm[ANY ? 1 : kStackLDS * kTraceBlock];
    uint2 *gsp = spill + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * S.stackDepth;
    int bottom = 0;   // entries [0, bottom) live in gsp
    Stack st;         // work counters only
    const uint32_t n = ANY ? P.cnt[CNT_QS(q)] : P.cnt[CNT_QC(q)];
    const uint32_t *Q = ANY ? P.qS + (size_t)q * P.rcap : P.qC + (size_t)q * 2 * P.rcap;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = trace_wave(P.xcdMap), nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t next = (uint32_t)((uint64_t)n * wave / nw);
    const uint32_t end = (uint32_t)((uint64_t)n * (wave + 1) / nw);
    bool active = false;
    int slot = 0, kind = 0, todo = 0, prim = -1;
    uint32_t ref = 0;
    float thit = INFINITY;
    // the ray of the current level: the world ray at level 0, the instance-space ray at level
    // 1 (the world ray is reloaded from the slot's ray record when the instance is done; only
    // its maxt, wmaxt, is kept)
    Ray ray;
    V invDir = v3(0.f, 0.f, 0.f);
    uint32_t negMask = 0;
    float wmaxt = 0.f;
    int level = 0, ibase = 0;                     // level 1: inside an instance, its entries from ibase
    uint32_t leafOff = 0, leafN = 0, leafI = 0;   // top-level leaf under test (resumed after an instance)
    bool inLeaf = false;
    uint32_t nM = 0, hM = 0;
    const uint32_t NONE = 0xffffffffu;
    auto setRay = [&](const Ray &r) {
        ray = r;
        invDir = v3(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z);
        negMask = (uint32_t)(invDir.x < 0) | ((uint32_t)(invDir.y < 0) << 1) | ((uint32_t)(invDir.z < 0) << 2);
    };
    for (;;) {
        const unsigned long long idle = __ballot(!active);
        const uint32_t nIdle = (uint32_t)__popcll(idle);
        if (next < end && (nIdle >= (uint32_t)refill || nIdle == 64u)) {
            if (!active) {
                const uint32_t i = next + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
                if (i < end) {
                    const uint32_t e = Q[i];
                    slot = ANY ? (int)e : (int)(e >> 1);
                    kind = ANY ? RAY_S : (int)(e & 1);
                    setRay(ray_load(P, rec_kind(S, q, kind), slot));
                    prim = -1;
                    thit = INFINITY;
                    todo = 0;
                    bottom = 0;
                    level = 0;
                    inLeaf = false;
                    if (ANY) st.cShadow++; else st.cRays++;
                    st.cNodes++;
                    const int neg[3] = {(int)(negMask & 1u), (int)((negMask >> 1) & 1u), (int)(negMask >> 2)};
                    if (bbox_hit((*sa(S.nodes, (uint32_t)(0))), (*sa(S.nodes, (uint32_t)(1))), ray, invDir, neg)) {
                        ref = (*sa(S.nodeRef, (uint32_t)(0)));
                        active = true;
                    } else if (ANY) P.occ[slot] = 0u;
                    else {
                        P.hitPrim[(size_t)kind * P.rcap + slot] = -1;
                        P.hitT[(size_t)kind * P.rcap + slot] = INFINITY;
                        if (STATS && kind == RAY_M) nM++;
                    }
                }
            }
            next = min(end, next + nIdle);
        }
        if (!__ballot(active)) {
            if (next >= end) break;
            continue;
        }
        if (active) {
            bool occluded = false, done = false;
            const int neg[3] = {(int)(negMask & 1u), (int)((negMask >> 1) & 1u), (int)(negMask >> 2)};
            if (level == 1 || !inLeaf) {
                if (ref != NONE && !(ref & WREF_LEAF)) {
                    const float4 *w = sa(S.wnodes, (uint32_t)(4 * (size_t)ref));
                    const float4 l0 = w[0], l1 = w[1], r0 = w[2], r1 = w[3];
                    st.cNodes++;
                    float tl = 0.f, tr = 0.f;
                    const bool hl = slab_enter_bf(l0, l1, ray, invDir, neg, &tl) & (tl < ray.maxt);
                    const bool hr = slab_enter_bf(r0, r1, ray, invDir, neg, &tr) & (tr < ray.maxt);
                    const uint32_t refL = __float_as_uint(l0.w), refR = __float_as_uint(l1.w);
                    const bool swap = ((negMask >> __float_as_uint(r0.w)) & 1u) != 0;
                    const bool hn = swap ? hr : hl, hf = swap ? hl : hr;
                    const uint32_t rn = swap ? refR : refL, rf = swap ? refL : refR;
                    if (hn) {
                        if (hf) {
                            if (todo - bottom == ring) {   // ring full: oldest entry to HBM
                                const int j = (bottom & (ring - 1)) * kTraceBlock + threadIdx.x;
                                gsp[bottom] = make_uint2(sref[j], ANY ? 0u : __float_as_uint(stm[j]));
                                ++bottom;
                            }
                            const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
                            sref[j] = rf;
                            if (!ANY) stm[j] = swap ? tl : tr;
                            ++todo;
                        }
                        ref = rn;
                    } else if (hf) ref = rf;
                    else ref = NONE;
                }
                if (ref != NONE && (ref & WREF_LEAF)) {
                    const uint32_t np = (ref >> WREF_NP_SHIFT) & WREF_NP_MASK, off = ref & WREF_OFF_MASK;
                    if (level == 1) {   // nested BVH leaf: triangles / quadrics only
                        for (uint32_t i = 0; i < np; ++i)
                            if (prim_test<ANY, false>(S, st, todo, (int)(off + i), ray, &prim, &thit) && ANY) {
                                occluded = true;
                                break;
                            }
                        ref = NONE;
                    } else {
                        leafOff = off;
                        leafN = np;
                        leafI = 0;
                        inLeaf = true;
                    }
                }
            }
            if (level == 0 && inLeaf) {
                // the top-level leaf's primitives from leafI; an instance suspends the leaf
                bool entered = false;
                while (leafI < leafN && !occluded) {
                    const int pi = (int)(leafOff + leafI);
                    ++leafI;
                    const pbrtgpu_prim pr = (*sa(S.prims, (uint32_t)(pi)));
                    if (pr.shape_type != PBRTGPU_SHAPE_INSTANCE) {
                        if (prim_test<ANY, false>(S, st, todo, pi, ray, &prim, &thit) && ANY) occluded = true;
                        continue;
                    }
                    const pbrtgpu_instance &I = (*sa(S.insts, (uint32_t)(pr.shape_index)));
                    float m[16];
                    inst_load(inst_rec(P, slot_of_ray(P, slot)), pr.shape_index, m, nullptr);   // the path's transform
                    Ray ir = xray(m, ray);
                    if (I.single_prim >= 0) {
                        if (prim_test<ANY, false>(S, st, todo, I.single_prim, ir, &prim, &thit)) {
                            if (ANY) occluded = true;
                            else ray.maxt = ir.maxt;
                        }
                        continue;
                    }
                    // nested BVH (bvh_walk<ANY, false>): its root box, then its walk
                    wmaxt = ray.maxt;
                    setRay(ir);
                    st.cNodes++;
                    const uint32_t root = (uint32_t)I.root;
                    const int negI[3] = {(int)(negMask & 1u), (int)((negMask >> 1) & 1u), (int)(negMask >> 2)};
                    if (!bbox_hit((*sa(S.nodes, (uint32_t)(2 * root))), (*sa(S.nodes, (uint32_t)(2 * root + 1))), ray, invDir, negI)) {
                        Ray wr = ray_load(P, rec_kind(S, q, kind), slot);   // back to the world ray
                        wr.maxt = wmaxt;
                        setRay(wr);
                        continue;
                    }
                    level = 1;
                    ibase = todo;
                    ref = (*sa(S.nodeRef, (uint32_t)(root)));
                    entered = true;
                    break;
                }
                if (!entered && !occluded) {
                    inLeaf = false;
                    ref = NONE;
                }
            }
            done = occluded;
            if (!done && ref == NONE && !(level == 0 && inLeaf)) {
                // pop the next entry of this level whose box is still entered before maxt
                for (;;) {
                    if (todo == (level ? ibase : 0)) {
                        if (level == 0) { done = true; break; }
                        // instance walked: back to the world ray (maxt shrunk by its hits),
                        // resume the suspended leaf
                        Ray wr = ray_load(P, rec_kind(S, q, kind), slot);
                        wr.maxt = ANY ? wmaxt : ray.maxt;
                        setRay(wr);
                        level = 0;
                        break;
                    }
                    --todo;
                    uint32_t r;
                    float tm;
                    if (todo < bottom) {
                        const uint2 g = gsp[todo];
                        r = g.x; tm = __uint_as_float(g.y);
                        bottom = todo;
                    } else {
                        const int j = (todo & (ring - 1)) * kTraceBlock + threadIdx.x;
                        r = sref[j]; tm = ANY ? 0.f : stm[j];
                    }
                    if (ANY || tm < ray.maxt) { ref = r; break; }
                }
            }
            if (done) {
                active = false;
                if (ANY) P.occ[slot] = occluded ? 1u : 0u;
                else {
                    P.hitPrim[(size_t)kind * P.rcap + slot] = prim;
                    P.hitT[(size_t)kind * P.rcap + slot] = prim >= 0 ? thit : INFINITY;
                    st.cHits += prim >= 0 ? 1u : 0u;
                    if (STATS && kind == RAY_M) { nM++; hM += prim >= 0 ? 1u : 0u; }
                }
            }
        }
    }
    if (STATS) {
        unsigned long long *w = reinterpret_cast<unsigned long long *>(P.cnt + CNT_WORK);
        if (ANY) {
            atomicAdd(&w[W_SHADOW], (unsigned long long)st.cShadow);
            atomicAdd(&w[W_NODES_S], (unsigned long long)st.cNodes);
            atomicAdd(&w[W_TRIS_S], (unsigned long long)st.cTris);
            atomicAdd(&w[W_QUADS_S], (unsigned long long)st.cQuads);
        } else {
            atomicAdd(&w[W_RAYS], (unsigned long long)st.cRays);
            atomicAdd(&w[W_NODES_C], (unsigned long long)st.cNodes);
            atomicAdd(&w[W_TRIS_C], (unsigned long long)st.cTris);
            atomicAdd(&w[W_QUADS_C], (unsigned long long)st.cQuads);
            atomicAdd(&w[W_HITS], (unsigned long long)st.cHits);
            atomicAdd(&w[W_RAYS_M], (unsigned long long)nM);
            atomicAdd(&w[W_HITS_M], (unsigned long long)hM);
        }
    }
}

// SpectralRenderer singleDirection: band b's luminance guard (spectralrenderer.cpp:163-172)
// looks at the sample's spectrum as assigned by bands 0 .. b-1 (the rest still 0): its
// y() = sum_i Y_i c_i / yint (spectrum.h:417-422) < -1e-5 or infinite zeroes band b.  The
// bands' index ranges are contiguous from 0, so y() is the running sum over the indices
// already final.  One thread per sample row.
template <int NB>
__global__ void k_spec_guard(const DevScene S, float *__restrict__ Lout, uint32_t rows) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    float *o = Lout + (size_t)r * NB;
    float yy = 0.f;
    for (int b = 0; b < S.specBands; ++b) {
        const int4 tb = (*sa(S.specTab, (uint32_t)(b)));
        if (tb.y <= tb.x) continue;
        const float yv = yy / S.yint;
        const bool bad = (yv < -1e-5f) || isinf(yv);
        for (int i = tb.x; i < tb.y; ++i) {
            float v = o[i];
            if (bad) o[i] = v = 0.f;
            yy += (*sa(S.bandY, (uint32_t)(i))) * v;
        }
    }
}

// MT windows of the slots k_shade (path integrator) listed in qT set q, one lane per entry (the
// list is compacted, so every lane of a wave runs the recurrence for a path); clears set q ^ 1's
// count, which the previous pass's k_mt_init consumed and the next k_shade fills
__global__ __launch_bounds__(256) void k_mt_init(PathSoA P, int q) {
    const uint32_t n = P.cnt[CNT_QT(q)];
    const uint32_t *list = P.qT + (size_t)q * P.cap;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        mt_window_init(P, list[i]);
    if (blockIdx.x == 0 && threadIdx.x == 0) P.cnt[CNT_QT(q ^ 1)] = 0u;
}
// The drain's list of live slots (PathSoA::listMode): block b lists the live slots of
// [b * chunk, (b + 1) * chunk) in slot order, one device-scope atomic per block
__global__ __launch_bounds__(256) void k_live_list(PathSoA P, int chunk) {
    const int lo = blockIdx.x * chunk, hi = min(P.cap, lo + chunk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t cnt[4], base;
    uint32_t mine = 0u;
    for (int s = lo + (int)threadIdx.x; s < hi; s += 256) mine += P.item[s] >= 0 ? 1u : 0u;
    if (threadIdx.x == 0) base = 0u;
    __syncthreads();
    if (mine) atomicAdd(&base, mine);
    __syncthreads();
    if (threadIdx.x == 0) base = base ? atomicAdd(&P.cnt[CNT_LIVE], base) : 0u;
    __syncthreads();
    uint32_t off = base;
    for (int s0 = lo; s0 < hi; s0 += 256) {
        const int s = s0 + (int)threadIdx.x;
        const bool lv = s < hi && P.item[s] >= 0;
        const unsigned long long b = __ballot(lv);
        if (lane == 0) cnt[wave] = (uint32_t)__popcll(b);
        __syncthreads();
        uint32_t pre = 0u, tot = 0u;
        for (int w = 0; w < 4; ++w) { pre += w < wave ? cnt[w] : 0u; tot += cnt[w]; }
        if (lv) P.live[off + pre + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = (uint32_t)s;
        off += tot;
        __syncthreads();
    }
}
static const int kLiveChunk = 4096;
static const int kMtInitGrid = 1024;   // 4 blocks per CU; a pass lists ~1 M slots at most (C2)
static hipError_t launch_mt_init(hipStream_t s, const PathSoA &P, int q) {
    hipLaunchKernelGGL(k_mt_init, dim3(kMtInitGrid), dim3(256), 0, s, P, q);
    return hipGetLastError();
}

// film[filmIdx[p]][b] += L(p, s) for s in batch order (spectralImage.cpp:125-131)
template <int NB>
__global__ void k_accum(const float *__restrict__ Lbuf, const int *__restrict__ filmIdx, int nPix, int sb,
                        float *__restrict__ film) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nPix * NB) return;
    int p = (int)(t / NB), b = (int)(t - (long)p * NB);
    float acc = film[(long)filmIdx[p] * NB + b];
    const float *src = Lbuf + (long)p * sb * NB + b;
    // the sum stays in sample order; unrolled so that 16 independent loads are in flight per lane
#pragma unroll 16
    for (int s = 0; s < sb; ++s) acc += 1.f * src[(long)s * NB];
    film[(long)filmIdx[p] * NB + b] = acc;
}

// spill scan over the sample extent: queue samples that land on a masked film pixel
// other than their own sample pixel (spectralImage.cpp:80-92, box filter width 0.5)
// over the samples [s0, s1) of a render call.  One thread per sample pixel: a pixel none of
// whose 8 neighbours is masked (most of the frame when a call renders a tile slice) is skipped
// without evaluating its samples.
__global__ void k_spill_scan(pbrtgpu_camera cam, uint32_t seed, int spp, int s0, int s1, const uint8_t *__restrict__ mask,
                             int3 *__restrict__ keys, unsigned int *__restrict__ count, unsigned int cap) {
    const int ew = cam.sx_end - cam.sx_start, eh = cam.sy_end - cam.sy_start;
    const long n = (long)ew * eh;
    for (long pi = (long)blockIdx.x * blockDim.x + threadIdx.x; pi < n; pi += (long)gridDim.x * blockDim.x) {
        const int x = cam.sx_start + (int)(pi % ew), y = cam.sy_start + (int)(pi / ew);
        bool near = false;
        for (int fy = max(y - 1, cam.py_start); fy <= min(y + 1, cam.py_start + cam.py_count - 1); ++fy)
            for (int fx = max(x - 1, cam.px_start); fx <= min(x + 1, cam.px_start + cam.px_count - 1); ++fx)
                if (!(fx == x && fy == y) && mask[(long)(fy - cam.py_start) * cam.px_count + (fx - cam.px_start)]) near = true;
        if (!near) continue;
        const uint32_t hp = pixel_hash(seed, x, y);
        for (int s = s0; s < s1; ++s) {
            float u[2];
            s2d(hp, 0, (uint32_t)s, (uint32_t)spp, u);
            float ix = x + u[0], iy = y + u[1];
            float dx = ix - 0.5f, dy = iy - 0.5f;
            int fx0 = (int)ceilf(dx - 0.5f), fx1 = (int)floorf(dx + 0.5f);
            int fy0 = (int)ceilf(dy - 0.5f), fy1 = (int)floorf(dy + 0.5f);
            fx0 = max(fx0, cam.px_start); fx1 = min(fx1, cam.px_start + cam.px_count - 1);
            fy0 = max(fy0, cam.py_start); fy1 = min(fy1, cam.py_start + cam.py_count - 1);
            if (fx1 - fx0 < 0 || fy1 - fy0 < 0) continue;
            if (fx0 == x && fx1 == x && fy0 == y && fy1 == y) continue;
            bool any = false;
            for (int fy = fy0; fy <= fy1; ++fy)
                for (int fx = fx0; fx <= fx1; ++fx)
                    if (!(fx == x && fy == y) && mask[(long)(fy - cam.py_start) * cam.px_count + (fx - cam.px_start)]) any = true;
            if (!any) continue;
            unsigned int k = atomicAdd(count, 1u);
            if (k < cap) keys[k] = make_int3(x, y, s);
        }
    }
}

// ordered contribution lists: for target t, entries [start[t], start[t+1]) of src in order
__global__ void k_apply(int nTargets, const int *__restrict__ tgt, const int *__restrict__ start,
                        const int *__restrict__ src, const float *__restrict__ Lsp, int nb, float *__restrict__ film) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nTargets * nb) return;
    int q = (int)(t / nb), b = (int)(t - (long)q * nb);
    float acc = film[(long)tgt[q] * nb + b];
    for (int e = start[q]; e < start[q + 1]; ++e) acc += 1.f * Lsp[(long)src[e] * nb + b];
    film[(long)tgt[q] * nb + b] = acc;
}

// film gather: out[p][b] = film[fidx[p]][b] (the pixels of a tile list, packed for one copy)
__global__ void k_pack(const float *__restrict__ film, const int *__restrict__ fidx, int nPix, int nb,
                       float *__restrict__ out) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nPix * nb) return;
    int p = (int)(t / nb), b = (int)(t - (long)p * nb);
    out[t] = film[(long)fidx[p] * nb + b];
}

__global__ __launch_bounds__(kTraceBlock) void k_intersect(DevScene S, const float *__restrict__ rays, int n,
                                                       float *__restrict__ hits, int *__restrict__ occ) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.tbase = reinterpret_cast<float *>(lds + (size_t)S.stackDepth * blockDim.x) + threadIdx.x;
    st.stride = blockDim.x;
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float *q = rays + 8 * k;
    Ray r;
    r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]); r.mint = q[6]; r.maxt = q[7]; r.time = 0.f;
    Ray r2 = r;
    int prim = -1;
    float t = INFINITY;
    if (!bvh_intersect(S, st, r, &prim, &t)) { prim = -1; t = INFINITY; }
    hits[4 * k] = t; hits[4 * k + 1] = 0.f; hits[4 * k + 2] = 0.f; hits[4 * k + 3] = __int_as_float(prim);
    const int o = bvh_intersectP(S, st, r2) ? 1 : 0;
    // the shadow walks of the renders answer the same: the 4-wide copy's (k_trace_s4) and its
    // quantized copy's (k_trace_s4q); a disagreement is reported as -1, which no oracle answer is
    bool same = true;
    if (S.w4N > 0) {
        same = same && (bvh_intersectP4(S, st, r2) ? 1 : 0) == o;
        if (S.w4q) same = same && (bvh_intersectP4q(S, st, r2) ? 1 : 0) == o;
    }
    occ[k] = same ? o : -1;
}

// pbrtgpu_mt_sequence: one lane draws the RNG's first n outputs with the shading code's MT
__global__ void k_mt_sequence(uint32_t seed, int n, uint32_t *out, uint32_t *ext) {
    if (threadIdx.x != 0) return;
    MT r;
    mt_begin(r, seed);
    mt_init(r);
    r.ext = ext;
    for (int i = 0; i < n; ++i) out[i] = mt_uint(r);
}

// pbrtgpu_libmf_eval: the shading code's transcendental entry points over an input array
__global__ void k_libmf_eval(int fn, int64_t n, const float *x, const float *y, float *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = x[i];
    switch (fn) {
    case PBRTGPU_LIBMF_SINF: out[i] = SINF(a); break;
    case PBRTGPU_LIBMF_COSF: out[i] = COSF(a); break;
    case PBRTGPU_LIBMF_SINCOSF: { const float2 sc = SINCOSF(a); out[2 * i] = sc.x; out[2 * i + 1] = sc.y; break; }
    case PBRTGPU_LIBMF_EXPF: out[i] = EXPF(a); break;
    case PBRTGPU_LIBMF_LOGF: out[i] = LOGF(a); break;
    case PBRTGPU_LIBMF_ACOSF: out[i] = ACOSF(a); break;
    case PBRTGPU_LIBMF_ATANF: out[i] = ATANF(a); break;
    case PBRTGPU_LIBMF_TANF: out[i] = TANF(a); break;
    case PBRTGPU_LIBMF_POWF: out[i] = POWF(a, y[i]); break;
    default: out[i] = ATAN2F(a, y[i]); break;
    }
}

// ------------------------------------------------------------------ context
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

// Pinned host staging of the film read-back: the device-to-host copy of a step's film (C2:
// 62.7 MB) runs at PCIe speed into it, where a pageable destination goes through the runtime's
// bounce buffers; host threads then copy or scatter it into the caller's film (par_for)
struct PinnedBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr; n = 0;
        hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; n = 0; }
};
// f(lo, hi) over [0, n) split across up to 8 host threads (chunks of at least `grain`)
template <class F> static void par_for(size_t n, size_t grain, const F &f) {
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::max<size_t>(1, std::min<size_t>({(size_t)8, hw, n / std::max<size_t>(1, grain)}));
    if (nt == 1) { f((size_t)0, n); return; }
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back([&, t] { f(n * t / nt, n * (t + 1) / nt); });
    f((size_t)0, n / nt);
    for (auto &x : th) x.join();
}

enum { K_CLOSEST = 0, K_SHADOW = 1, K_SHADE = 2, K_ACCUM = 3, K_KINDS = 4 };

struct Timing {
    double ms[K_KINDS] = {0, 0, 0, 0};
    int launches[K_KINDS] = {0, 0, 0, 0};
    int passes = 0;
    uint64_t work[W_COUNT] = {0};
};

// One wavefront instance: path slots, queues and counters, its two streams (closest-hit
// queries + shading; shadow queries beside them) and the events of one batch of passes.
struct Lane {
    DevBuf slots;            // PathSoA storage
    DevBuf spill;            // k_trace_pt stack spill areas (closest, shadow)
    int slotCap = 0, slotNb = 0, slotInst = 0, slotFrames = 0, slotBatch = 0;
    bool slotMtExt = false;
    PathSoA P{};
    hipStream_t s = nullptr, s2 = nullptr;
    // two batch slots (run_wavefront keeps up to two batches of passes in flight): per slot the
    // passes' event pairs, the pinned mirror of the queue counters at the batch's end, and the
    // event recorded after that read-back (polled)
    hipEvent_t ev[2][2 + 6 * 8] = {};
    uint32_t *hostCnt[2] = {};
    hipEvent_t done[2] = {};
};
#ifndef PGD_LANES
#define PGD_LANES 2
#endif
static const int kLanes = PGD_LANES;

struct pbrtgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[8] = {};
    Lane lane[kLanes];       // lane[0].s is `stream`
    bool hasScene = false;
    DevScene S{};
    int nb = 0, spp = 0, stackDepth = 0;
    int feat = 0;   // FEAT_* of the uploaded scene: selects the k_shade variant
    pbrtgpu_camera cam{};
    std::vector<DevBuf> sceneBufs;
    DevBuf film, Lbuf, pix, filmIdx, mask, keys, counter, spillL, lists[4], scratch[3], gather[2];
    PinnedBuf stage;          // film read-back staging (pbrtgpu_film_read / _gather)
    // render_impl's per-call setup of the last call -- its pixel lists (on the device: pix,
    // filmIdx, mask), its exact-boundary samples (keys, sorted) and their contribution lists --
    // reused by a call with the same tiles, sample range and scene (repeated frames of one tile
    // set: the timed steps of a rank)
    struct CallSetup {
        bool valid = false;
        uint64_t gen = 0;
        int tw = 0, th = 0, s0 = 0, s1 = 0, nPix = 0, nSpill = 0;
        bool all = false;
        std::vector<int32_t> tiles;
        double spills = 0;
        std::vector<int> preT, preStart, preSrc, postT, postStart, postSrc;
    } setup;
    uint64_t sceneGen = 0;    // bumped by every scene upload (invalidates `setup`)
    int numCUs = 256;
    int ptBlocksPerCU = 0;    // occupancy of k_trace_pt closest (computed on first use)
    int ptBlocksPerCUS = 0;   // occupancy of k_trace_pt shadow
    int s4BlocksPerCU = 0;    // occupancy of k_trace_s4 (shadow queries on the 4-wide BVH)
    int s4qBlocksPerCU = 0;   // occupancy of k_trace_s4q (shadow queries on its quantized copy)
    int c4BlocksPerCU = 0;    // occupancy of k_trace_c4 (closest-hit queries on the 4-wide BVH)
    int instBlocksPerCU = 0, instBlocksPerCUS = 0;   // occupancy of k_trace_inst closest / shadow
    int ring = kStackLDS;     // LDS ring entries in use (PBRTGPU_STACK_LDS: tests force HBM spills)
    int refill = 16;          // idle lanes that trigger ray replacement in k_trace_pt (PBRTGPU_REFILL)
    Timing last;
};

template <class T> static hipError_t upload(pbrtgpu_ctx *c, const T *src, size_t count, const T **dst) {
    c->sceneBufs.emplace_back();
    DevBuf &b = c->sceneBufs.back();
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = b.ensure(bytes);
    if (e != hipSuccess) return e;
    if (count) e = hipMemcpy(b.p, src, count * sizeof(T), hipMemcpyHostToDevice);
    *dst = reinterpret_cast<const T *>(b.p);
    return e;
}

// path slots: PBRTGPU_SLOTS env override (tests use small capacities to exercise regeneration)
static int slot_target() {
    const char *e = getenv("PBRTGPU_SLOTS");
    int v = e ? atoi(e) : 0;
    // 16 M slots = 2 lanes x 8 M (C2 456-461 -> 467-468 Mpaths/s vs 2 x 4 M, C4 230 -> 233;
    // profiles/r03/slot_rule/target16m.txt); a lane's arrays stay below 4 GiB (max_slots_32bit:
    // 60 bands cap a lane at ~6 M)
    return v > 0 ? v : (1 << 24);
}
// A lane's slot pool: the slot target when the lane has more items than that (two or more slot
// generations), else half of its items (at least 1 M), so a small render still runs two
// generations.  Round 2 took a quarter of the items: a pool's drain then cost about a full pass
// per drain pass.  With the drain on the live-slot list, larger pools win down to two
// generations (one GPU, min of 3 renders, profiles/r03/slot_rule/rules.txt): C2's 1/8
// (7.9 M items per lane) 395 (quarter) -> 429 Mpaths/s at 4 M slots, 402 with all its items in
// slots; its 1/4 (15.9 M) 455 at the 8.4 M target, 394 at exactly half its items (7.9 M: same
// passes, k_shade 25 % slower, reproducibly -- not understood), 427 at 4 M.
// PBRTGPU_SLOT_DIV=d (experiments): items / d when the lane has at most the target.
static uint32_t slot_div() {
    const char *e = getenv("PBRTGPU_SLOT_DIV");
    const long v = e ? atol(e) : 0;
    return v > 0 ? (uint32_t)v : 2u;
}
static int lane_slots(uint32_t items, int nl) {
    const int t = std::max(64, slot_target() / nl);
    if (getenv("PBRTGPU_SLOTS")) return (int)std::min<uint32_t>(items, (uint32_t)t);
    const uint32_t want = items > (uint32_t)t ? (uint32_t)t : std::max<uint32_t>(1u << 20, items / slot_div());
    return (int)std::min<uint32_t>(items, want);
}
// per-sample radiance budget of one spp batch: PBRTGPU_LBUF_MB env override (tests force
// many batches per frame with a tiny budget)
static size_t lbuf_budget() {
    const char *e = getenv("PBRTGPU_LBUF_MB");
    long v = e ? atol(e) : 0;
    return v > 0 ? ((size_t)v << 20) : ((size_t)PGD_LBUF_GIB << 30);
}
// PBRTGPU_SERIAL=1: one lane, shadow queries on the lane's main stream -- no two kernels of
// a render overlap, so each kernel's event spans are its exclusive device time (roofline)
static bool legacy_inst_walk() {
    const char *e = getenv("PBRTGPU_INST_WALK");
    return e && !strcmp(e, "legacy");
}
// top-level wide BVH nodes k_trace_pt copies to LDS (PBRTGPU_TOP_NODES: fewer, for tests)
static int top_nodes() {
    const char *e = getenv("PBRTGPU_TOP_NODES");
    const int v = e ? atoi(e) : kTopNodes;
    return std::max(0, std::min(v, kTopNodes));
}
// PBRTGPU_PASS_LOG=1: per-pass kernel times and queue sizes on stderr (diagnostics)
static bool pass_log() {
    static const bool on = getenv("PBRTGPU_PASS_LOG") != nullptr;
    return on;
}
static bool mt_ext_forced() {
    const char *e = getenv("PBRTGPU_MT_EXT");
    return e && atoi(e) != 0;
}
static bool closest4_on() {
    const char *e = getenv("PBRTGPU_CLOSEST4");
    return !e || atoi(e) != 0;
}
// PBRTGPU_SHADOW4Q=1: the shadow queries on the quantized copy of the 4-wide tree instead of the
// exact one.  Exact either way; opt-in because it measured slower (r05d: C2 shadow 49.5 vs 40.4
// ms/frame, DirectLighting 236 vs 189; L2 misses -6 %): the walk is latency-bound, not byte-bound
static bool shadow4q_on() {
    const char *e = getenv("PBRTGPU_SHADOW4Q");
    return e && atoi(e) != 0;
}
static bool shadow4_on() {
    const char *e = getenv("PBRTGPU_SHADOW4");
    return !e || atoi(e) != 0;
}
// PBRTGPU_TAIL=<rays>: the drain's remaining paths run to their end in one k_tail launch once the
// queued rays of a lane (closest + shadow) are at most this many (path integrator, no instances,
// after three list-mode passes); 0: off
static uint32_t tail_rays() {
    const char *e = getenv("PBRTGPU_TAIL");
    return e ? (uint32_t)strtoul(e, nullptr, 0) : 131072u;
}
// passes per read-back in the drain (default 2) and within one slot pool of the lane's last item
// (default 4): PBRTGPU_DRAIN_BATCH / PBRTGPU_NEAR_BATCH (A/B; at least 1)
static int env_int(const char *name, int def) {
    const char *e = getenv(name);
    return e && *e ? std::max(1, atoi(e)) : def;
}
static int drain_batch() { static const int v = env_int("PBRTGPU_DRAIN_BATCH", 2); return v; }
static int near_batch() { static const int v = env_int("PBRTGPU_NEAR_BATCH", 4); return v; }
static int xcd_map_on() {
    const char *e = getenv("PBRTGPU_XCD_MAP");
    return (e && atoi(e) != 0) ? 1 : 0;
}
// Batches of passes in flight per lane (run_wavefront): PBRTGPU_PIPE=0 (default) one -- every
// decision from the last batch's counters, with the host's gap at each read-back; 2 two always (the
// decisions one batch late); 1 two while the lane has more than two slot pools of items left --
// decisions that far from the drain cannot change -- and one from there on.  Measured (r06c, one
// box, two runs each): C2 504-506 Mpaths/s with one, 486-487 with 1, 483-488 with 2; one GPU's 1/8
// slice 455-457 Mpaths/s either way with 0 and 1, 1/4 and 1/8 much worse with 2 (the drain's list
// mode and tail a batch late).  The read-back gaps are not what bounds the frame: with two
// batches queued, the two lanes' kernels fall into step and overlap less
static int pipe_mode() {
    const char *e = getenv("PBRTGPU_PIPE");
    const int v = e ? atoi(e) : 0;
    return v < 0 ? 0 : (v > 2 ? 2 : v);
}
static bool drain_list_on() {
    const char *e = getenv("PBRTGPU_DRAIN_LIST");
    return !e || atoi(e) != 0;
}
// before a k_shade pass: the drain's live-slot list and PathSoA::listMode (read by the launch)
static hipError_t drain_list(Lane &L, bool drain, int cap) {
    L.P.listMode = drain ? 1 : 0;
    if (!drain) return hipSuccess;
    if (hipError_t e = hipMemsetAsync(L.P.cnt + CNT_LIVE, 0, 4, L.s)) return e;
    hipLaunchKernelGGL(k_live_list, dim3((cap + kLiveChunk - 1) / kLiveChunk), dim3(256), 0, L.s, L.P, kLiveChunk);
    return hipGetLastError();
}
static bool serial_mode() {
    const char *e = getenv("PBRTGPU_SERIAL");
    return e && atoi(e) != 0;
}
// PBRTGPU_POISON=<byte> (debugging / tests): every path-slot array, the traversal stack spill
// area and a render's per-sample radiance buffer are filled with that byte before each wavefront run, so a read of state no pass wrote
// gives a result that changes with the byte; -1 (unset): left as they are
static int poison_byte() {
    const char *e = getenv("PBRTGPU_POISON");
    return e && *e ? (int)(strtol(e, nullptr, 0) & 0xff) : -1;
}

// DirectLighting frame bytes per slot and frame (PathSoA::f*)
static size_t frame_bytes(int NB) { return (size_t)8 * ((NB + 3) / 4 * 4) + 104; }
// DirectLighting bytes per slot and batched light sample: A, B terms and the ray records
static size_t batch_bytes(int NB) { return (size_t)8 * ((NB + 3) / 4 * 4) + 27 * 4 + 8 + 8 + 4 + 24; }
// ray record floats per ray slot: 9 per kind -- RAY_C, RAY_M, RAY_S, and RAY_M1 (the path
// integrator's second MIS record set, wavefront.h mis_kind; DirectLighting, batch > 1, has none)
static size_t ray_floats(int batch) { return batch == 1 ? 36 : 27; }
// The shading step addresses the slot arrays through 32-bit byte offsets (wavefront.h sa / Col):
// the largest of them -- A / B at max(2, batch) x padded bands, beta at 3 x, the ray records at
// ray_floats per ray slot -- must stay below 4 GiB, which bounds a lane's slots
static int max_slots_32bit(int NB, int batch) {
    const size_t NBP = (size_t)(NB + 3) / 4 * 4;
    const size_t per = std::max({(size_t)std::max(2, batch) * NBP * 4, 3 * NBP * 4, (size_t)batch * ray_floats(batch) * 4});
    return (int)std::min<size_t>(INT32_MAX / 2, (((size_t)1 << 32) - 1) / per);
}
// batch: ray slots per slot (light samples a DirectLighting pass issues; 1 for the other integrators)
static int ensure_slots(Lane *c, int cap, int NB, int nInst, int nFrames, int batch, bool mtExt) {
    if (c->slotCap == cap && c->slotNb == NB && c->slotInst == nInst && c->slotFrames == nFrames &&
        c->slotBatch == batch && c->slotMtExt == mtExt)
        return 0;
    if (cap > max_slots_32bit(NB, batch)) return fail(PBRTGPU_E_INVALID, "slot arrays beyond 32-bit offsets");
    const size_t C = (size_t)cap, R = C * (size_t)batch, AB = (size_t)std::max(2, batch);
    const int NBP = (NB + 3) / 4 * 4;   // bands padded to whole float4 quads
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    size_t oItem = take(C * 4), oHp = take(C * 4), oSmp = take(C * 4), oBounce = take(C * 4), oFlags = take(C * 4),
           oMt = take(C * 20), oBeta = take(C * 3 * NBP * 4), oL = take(C * NBP * 4), oA = take(C * AB * NBP * 4),
           oB = take(C * AB * NBP * 4), oM = take(C * NBP * 4), oK = take(C * 2 * NBP * 4) /* [2][NQ][cap]: two textured spectra */, oPix = take(C * 4),
           oRay = take(R * ray_floats(batch) * 4), oHitP = take(R * 8), oHitT = take(R * 8), oOcc = take(R * 4), oQC = take(R * 16),
           oQS = take(R * 8), oQT = take(C * 8), oLive = take(C * 4), oCnt = take(CNT_WORDS * 4), oInst = take(C * (size_t)nInst * 128),
           oMask = take(nFrames ? C * 4 : 0), oAMask = take(2 * ((C + 63) / 64) * 8),
           oBMask = take(3 * ((C + 63) / 64) * 8), oMMask = take(2 * ((C + 63) / 64) * 8);
    const size_t F = (size_t)nFrames;
    size_t oFL = take(C * F * NBP * 4), oFF = take(C * F * NBP * 4), oFRay = take(C * F * 36), oFDiff = take(C * F * 48),
           oFS = take(C * F * 8), oFHit = take(C * F * 8), oFBr = take(C * F * 4), oDlk = take(nFrames ? C * 4 : 0),
           oDlList = take(nFrames ? C * 4 : 0), oDlRow = take(nFrames ? C * 4 : 0),
           oMtExt = take(mtExt ? C * 624 * 4 : 0);
    HIPCHK(c->slots.ensure(off));
    char *base = (char *)c->slots.p;
    PathSoA &P = c->P;
    P.cap = cap;
    P.rcap = (int)R;
    P.dlBatch = batch;
    P.dlMask = nFrames ? (uint32_t *)(base + oMask) : nullptr;
    P.aMask = (unsigned long long *)(base + oAMask);
    P.bMask = (unsigned long long *)(base + oBMask);
    P.mMask = (unsigned long long *)(base + oMMask);
    P.pass = 0;
    P.item = (int *)(base + oItem); P.hp = (uint32_t *)(base + oHp); P.smp = (uint32_t *)(base + oSmp);
    P.bounce = (int *)(base + oBounce); P.flags = (uint32_t *)(base + oFlags); P.mt = (uint32_t *)(base + oMt);
    P.beta = (float4 *)(base + oBeta); P.L = (float4 *)(base + oL); P.A = (float4 *)(base + oA); P.B = (float4 *)(base + oB);
    P.M = (float4 *)(base + oM); P.K = (float4 *)(base + oK); P.pix = (uint32_t *)(base + oPix);
    P.ray = (float *)(base + oRay); P.hitPrim = (int *)(base + oHitP); P.hitT = (float *)(base + oHitT);
    P.occ = (uint32_t *)(base + oOcc); P.qC = (uint32_t *)(base + oQC); P.qS = (uint32_t *)(base + oQS);
    P.qT = (uint32_t *)(base + oQT);
    P.live = (uint32_t *)(base + oLive);
    P.listMode = 0;
    P.xcdMap = 0;
    P.cnt = (uint32_t *)(base + oCnt);
    P.nInst = nInst;
    P.instM = nInst ? (float4 *)(base + oInst) : nullptr;
    P.nFrames = nFrames;
    P.fL = nFrames ? (float4 *)(base + oFL) : nullptr;
    P.fF = nFrames ? (float4 *)(base + oFF) : nullptr;
    P.fRay = nFrames ? (float *)(base + oFRay) : nullptr;
    P.fDiff = nFrames ? (float *)(base + oFDiff) : nullptr;
    P.fS = nFrames ? (float *)(base + oFS) : nullptr;
    P.fHit = nFrames ? (int *)(base + oFHit) : nullptr;
    P.fBr = nFrames ? (uint32_t *)(base + oFBr) : nullptr;
    P.dlk = nFrames ? (uint32_t *)(base + oDlk) : nullptr;
    P.dlList = nFrames ? (uint32_t *)(base + oDlList) : nullptr;
    P.dlRow = nFrames ? (uint32_t *)(base + oDlRow) : nullptr;
    P.mtExt = mtExt ? (uint32_t *)(base + oMtExt) : nullptr;
    c->slotMtExt = mtExt;
    c->slotFrames = nFrames;
    c->slotBatch = batch;
    c->slotCap = cap;
    c->slotNb = NB;
    c->slotInst = nInst;
    return 0;
}

// Runs every item of src through the wavefront pipeline; radiance of item i -> Lout[i][NB].
// The items are split into kLanes independent halves, each run by its own lane (slots,
// queues, streams), so one lane's shading overlaps the other's ray queries.  Within a lane,
// passes are enqueued kPassBatch at a time between counter read-backs: the kernels read
// their queue sizes on the device, and passes after the queues have drained are empty
// launches.  The shadow queries run on the lane's second stream beside the closest-hit
// queries (their tails overlap); shade waits for both.
// The path integrator's shading variant for a scene's features: FEAT 0, FEAT_ALL, and three
// partial builds -- 32 (and 3: C1) bands with matte / plastic materials only (C2, C5: FEAT_BASIC, device.h), 32
// bands with those and measured BRDFs (C3: FEAT_MEAS | FEAT_BASIC, without the texture /
// environment-light code and the other materials' BxDFs) and 60 bands with textures and environment
// lights but no measured BRDFs (C4: FEAT_TEX | FEAT_INF, no kd-tree walk).  FEAT_BASIC is a
// restriction, not a feature: other band counts and integrators take (feat & FEAT_ALL)
template <int NB>
static auto path_shade_variant(int feat) -> decltype(&launch_shade<NB, 0>) {
    if constexpr (NB == 32) {
        if (feat == FEAT_BASIC) return launch_shade<32, FEAT_BASIC>;
        if (feat == (FEAT_MEAS | FEAT_BASIC)) return launch_shade<32, FEAT_MEAS | FEAT_BASIC>;
    }
    if constexpr (NB == 3)   // the RGB build (C1)
        if (feat == FEAT_BASIC) return launch_shade<3, FEAT_BASIC>;
    if constexpr (NB == 60) {
        if (feat == (FEAT_TEX | FEAT_INF | FEAT_NOSPEC) && !getenv("PGD_NO60_6"))   // C4
            return launch_shade<60, FEAT_TEX | FEAT_INF | FEAT_NOSPEC>;
        if ((feat & FEAT_ALL) == (FEAT_TEX | FEAT_INF) && !getenv("PGD_NO60_6")) return launch_shade<60, FEAT_TEX | FEAT_INF>;
    }
    return (feat & FEAT_ALL) ? launch_shade<NB, FEAT_ALL> : launch_shade<NB, 0>;
}
// the DirectLighting step's objects: FEAT_BASIC at 32 bands (C2's scene), else FEAT_ALL or FEAT 0
// (PBRTGPU_DL_BASIC=0: the FEAT 0 objects on FEAT_BASIC scenes, A/B)
template <int NB, class F>
static F dl_variant(int feat, F all, F lean, F basic) {
    static const bool on = !getenv("PBRTGPU_DL_BASIC") || atoi(getenv("PBRTGPU_DL_BASIC")) != 0;
    if (basic && feat == FEAT_BASIC && on) return basic;
    return (feat & FEAT_ALL) ? all : lean;
}
// the FEAT_BASIC DirectLighting objects built (Makefile SHADEVARS): 32 and 60 bands
template <int NB> static constexpr bool kDlBasic = NB == 32 || NB == 60;
template <int NB>
static auto path_tail_variant(int feat) -> decltype(&launch_tail<NB, 0>) {
    if constexpr (NB == 32) {
        if (feat == FEAT_BASIC) return launch_tail<32, FEAT_BASIC>;
        if (feat == (FEAT_MEAS | FEAT_BASIC)) return launch_tail<32, FEAT_MEAS | FEAT_BASIC>;
    }
    if constexpr (NB == 3)
        if (feat == FEAT_BASIC) return launch_tail<3, FEAT_BASIC>;
    if constexpr (NB == 60) {
        if (feat == (FEAT_TEX | FEAT_INF | FEAT_NOSPEC) && !getenv("PGD_NO60_6"))
            return launch_tail<60, FEAT_TEX | FEAT_INF | FEAT_NOSPEC>;
        if ((feat & FEAT_ALL) == (FEAT_TEX | FEAT_INF) && !getenv("PGD_NO60_6")) return launch_tail<60, FEAT_TEX | FEAT_INF>;
    }
    return (feat & FEAT_ALL) ? launch_tail<NB, FEAT_ALL> : launch_tail<NB, 0>;
}

template <int NB>
static int run_wavefront(pbrtgpu_ctx *c, const ItemSrc &src, float *Lout, bool countWork, Timing &T,
                         unsigned int *zeroedOut) {
    if (src.nItems == 0) return 0;
    static const int kPassBatch = PGD_PASS_BATCH;
    // LDS stack of the instanced-scene kernels: child refs and (closest-hit) entry distances
    const size_t ldsS = (size_t)c->stackDepth * kTraceBlock * sizeof(uint32_t), lds = 2 * ldsS;
    const int perCU = std::max(1, std::min(16, (int)(160 * 1024 / std::max<size_t>(lds, 1))));
    const int traceGrid = c->numCUs * perCU;
    const bool inst = c->S.nInsts > 0;
    if (!c->ptBlocksPerCU) {   // resident blocks of the persistent kernels (registers, LDS)
        int b0 = 0, b1 = 0, b2 = 0, b3 = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b0, k_trace_pt<false, false>, kTraceBlock, 0));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b1, k_trace_pt<true, false>, kTraceBlock, 0));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b2, k_trace_inst<false, false>, kTraceBlock, 0));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b3, k_trace_inst<true, false>, kTraceBlock, 0));
        int b4 = 0, b5 = 0, b6 = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b4, k_trace_s4<false>, kTraceBlock, 0));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b5, k_trace_c4<false>, kTraceBlock, 0));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b6, k_trace_s4q<false>, kTraceBlock, 0));
        c->s4BlocksPerCU = std::max(1, b4);
        c->s4qBlocksPerCU = std::max(1, b6);
        c->c4BlocksPerCU = std::max(1, b5);
        c->ptBlocksPerCU = std::max(1, b0);
        c->ptBlocksPerCUS = std::max(1, b1);
        c->instBlocksPerCU = std::max(1, b2);
        c->instBlocksPerCUS = std::max(1, b3);
    }
    // instanced scenes: the two-level persistent kernels (PBRTGPU_INST_WALK=legacy: the
    // one-ray-per-thread bvh_walk kernels, kept for A/B parity tests)
    const bool instPT = inst && !legacy_inst_walk();
    // closest-hit queries on the 4-wide BVH copy likewise (PBRTGPU_CLOSEST4=0: the binary walk)
    const bool c4 = !inst && c->S.w4N > 0 && closest4_on();
    const uint32_t ptGrid = (uint32_t)(c->numCUs * (instPT ? c->instBlocksPerCU : c4 ? c->c4BlocksPerCU : c->ptBlocksPerCU));
    // shadow queries on the 4-wide BVH copy (scenes without instances; PBRTGPU_SHADOW4=0: the binary walk)
    const bool s4 = !inst && c->S.w4N > 0 && shadow4_on();
    const bool s4q = s4 && c->S.w4q && shadow4q_on();   // ... on its quantized copy (quant_w4)
    const uint32_t ptGridS = (uint32_t)(c->numCUs * (instPT ? c->instBlocksPerCUS
                                                     : s4q ? c->s4qBlocksPerCU : s4 ? c->s4BlocksPerCU : c->ptBlocksPerCUS));
    const size_t spillLane = (size_t)std::max(ptGrid, ptGridS) * kTraceBlock *
                             (size_t)std::max(c->stackDepth, (s4 || c4) ? c->S.w4Stack : 0);   // uint2 per kernel
    // scenes without measured BRDFs, textures and environment lights run the variant with
    // that code compiled out (fewer registers, no kd-tree stack)
    // the DirectLighting integrator has its own step (all features compiled in)
    const bool dl = c->S.integrator == PBRTGPU_INTEGRATOR_DIRECT;
    auto kShade = dl ? dl_variant<NB>(c->feat, launch_shade_dl<NB, FEAT_ALL>, launch_shade_dl<NB, 0>,
                                      kDlBasic<NB> ? launch_shade_dl<kDlBasic<NB> ? NB : 32, FEAT_BASIC> : nullptr)
                  : c->S.integrator == PBRTGPU_INTEGRATOR_METADATA
                      ? ((c->feat & FEAT_ALL) ? launch_shade_meta<NB, FEAT_ALL> : launch_shade_meta<NB, 0>)
                  : path_shade_variant<NB>(c->feat);
    const int nFrames = dl ? std::max(1, c->S.maxDepth) : 0;
    // the path integrator's k_shade lists the slots about to make their first MT draws (k_mt_init)
    const bool mtList = c->S.integrator != PBRTGPU_INTEGRATOR_DIRECT && c->S.integrator != PBRTGPU_INTEGRATOR_METADATA;
    // the path and DirectLighting integrators' drain runs on the live slots' list
    // (PBRTGPU_DRAIN_LIST=0: off, A/B)
    const bool drainList = c->S.integrator != PBRTGPU_INTEGRATOR_METADATA && drain_list_on();
    auto kNee = dl_variant<NB>(c->feat, launch_dl_nee<NB, FEAT_ALL>, launch_dl_nee<NB, 0>,
                               kDlBasic<NB> ? launch_dl_nee<kDlBasic<NB> ? NB : 32, FEAT_BASIC> : nullptr);
    auto kSpec = dl_variant<NB>(c->feat, launch_dl_spec<NB, FEAT_ALL>, launch_dl_spec<NB, 0>,
                                kDlBasic<NB> ? launch_dl_spec<kDlBasic<NB> ? NB : 32, FEAT_BASIC> : nullptr);
    // DirectLighting issues up to kDlBatch light samples of a vertex per pass
    const int batch = dl ? std::max(1, std::min(c->S.dlStrategy == PBRTGPU_DL_ONE ? 1 : c->S.dlK, kDlBatch)) : 1;
    // passes one path can take: the camera ray + maxdepth + 1 vertices + 1 finish (path); per
    // vertex of the DirectLighting recursion (at most 2^maxdepth - 1) its hit + one pass per
    // light sample, + the output
    const int64_t pathPasses = dl ? (nFrames >= 40 ? ((int64_t)1 << 60) : (((int64_t)1 << nFrames) - 1) * (c->S.dlK + 1) + 2)
                                  : c->S.maxDepth + 3;
    // paths that may draw past the first 227 MT19937 outputs keep their full state in an ext row
    // (device.h mt_uint_ext): path integrator maxdepth > 20 (at most 11 draws per vertex beyond
    // the sampler's 3 bounces), DirectLighting maxdepth > 6 (6 per specular vertex, up to
    // 2^(maxdepth-1) - 1 of them); PBRTGPU_MT_EXT=1 forces the rows (tests)
    const bool mtExt = (dl ? c->S.maxDepth > 6 : c->S.maxDepth > 20) || mt_ext_forced();
    // drain: the run's items are all taken; its k_shade passes take the live slots' list
    // (PathSoA::listMode) on a grid of liveGrid blocks (live slots <= the queued rays at the last
    // read-back, as every live slot ends a pass with a ray queued)
    // One batch of passes between two counter read-backs, as enqueued.  A lane keeps up to two
    // batches in flight (slots 0 / 1 of Lane::ev / hostCnt / done): while the GPU runs batch k+1,
    // the host reads batch k's counters and enqueues batch k+2, so a read-back never leaves the
    // lane's streams idle (round 5: 15 such gaps, 5.6 ms of a 41 ms 1/8-slice timeline).  The
    // decisions batch k+2 takes from batch k's counters stay valid one batch late:
    //   * the drain's list mode: once every item is taken (CNT_NEXT) no slot regenerates, so the
    //     live slots only decrease and the queued rays of batch k bound them at k+2 (liveGrid);
    //   * the tail (k_tail): queued rays at batch k bound those at k+2, and the three list-mode
    //     passes before it are counted as enqueued;
    //   * the end: queues empty at batch k stay empty, and batch k+1 is then empty passes.
    // Every pass runs in the same stream order whatever the batching, so the radiance is unchanged.
    struct Batch { int n; bool single, drain; int liveGrid, qEnd; };
    struct Run { Lane *L; ItemSrc src; int cap, grid, q, passes, maxPasses; bool done, drain, ending, tailed; int liveGrid, listPasses;
                 Batch b[2]; int head, inflight; };
    // the drain's tail kernel (k_tail): path integrator, scenes without instances (the 4-wide walks),
    // not in work-counting runs (it counts no traversal work)
    const uint32_t tailMax = (!dl && c->S.integrator == PBRTGPU_INTEGRATOR_PATH && !inst && c->S.w4N > 0 && !countWork)
                                 ? tail_rays() : 0u;
    auto kTail = path_tail_variant<NB>(c->feat);
    Run R[kLanes];
    const bool serial = serial_mode();
    const int nl = (src.nItems >= 8192u && !serial) ? kLanes : 1;
    // batch `bi` of run r after its passes: the counters to the host, the completion event
    auto close_batch = [&](Run &r, int bi, const Batch &B) -> int {
        Lane &L = *r.L;
        HIPCHK(hipMemcpyAsync(L.hostCnt[bi], L.P.cnt, CNT_WORDS * 4, hipMemcpyDeviceToHost, L.s));
        HIPCHK(hipEventRecord(L.done[bi], L.s));
        r.b[bi] = B;
        r.inflight++;
        return 0;
    };
    // the next batch of run r from the counters `cnt` of its last completed batch (qc: that batch's
    // final queue set): the drain / tail decisions above, then the passes
    auto enqueue = [&](Run &r, const uint32_t *cnt, int qc) -> int {
        Lane &L = *r.L;
        const PathSoA &P = L.P;
        const int bi = r.inflight ? (r.head ^ 1) : r.head;
        const uint64_t queued = (uint64_t)cnt[CNT_QC(qc)] + cnt[CNT_QS(qc)];
        if (drainList && cnt[CNT_NEXT] >= r.src.nItems) {
            r.drain = true;
            const uint64_t bound = std::min<uint64_t>((uint64_t)r.cap, queued);
            r.liveGrid = (int)std::max<uint64_t>(1, (bound + kShadeBlock - 1) / kShadeBlock);
        }
        int q = r.q;
        hipEvent_t *ev = L.ev[bi];
        if (r.drain && r.listPasses >= 3 && tailMax && queued <= tailMax) {
            // the tail: the live list, then k_tail runs those paths to their end; the next queue
            // set stays empty, so the lane reads as drained at this batch's read-back (its time is
            // the batch's single event pair, a shade launch)
            const int nq = q ^ 1;
            HIPCHK(hipMemsetAsync(P.cnt + CNT_QC(nq), 0, 4, L.s));
            HIPCHK(hipMemsetAsync(P.cnt + CNT_QS(nq), 0, 4, L.s));
            HIPCHK(hipEventRecord(ev[0], L.s));
            HIPCHK(drain_list(L, true, r.cap));
            const uint64_t bound = std::min<uint64_t>((uint64_t)r.cap, queued);
            HIPCHK(kTail((int)std::max<uint64_t>(1, (bound + kTailBlock - 1) / kTailBlock), L.s, c->S, L.P, q, Lout,
                         (int)std::min<int64_t>(pathPasses, INT32_MAX)));
            HIPCHK(hipEventRecord(ev[1], L.s));
            r.q = nq;
            r.tailed = true;
            T.passes++;
            r.passes++;
            return close_batch(r, bi, Batch{0, true, true, r.liveGrid, nq});
        }
        uint2 *spillC = (uint2 *)L.spill.p, *spillS = spillC + spillLane;
        // serial mode: the shadow queries follow the closest-hit queries on the main stream
        hipStream_t s2 = serial ? L.s : L.s2;
        // passes per read-back: kPassBatch while the lane has items for more than one more
        // pool, then fewer, so that the switch to the drain's list mode and the lane's end
        // are seen within a few passes (2 in the drain, 4 before it)
        const int n = r.drain ? std::min(drain_batch(), kPassBatch)
                              : (uint64_t)cnt[CNT_NEXT] + (uint64_t)r.cap >= r.src.nItems ? std::min(near_batch(), kPassBatch)
                                                                                        : kPassBatch;
        for (int j = 0; j < n; ++j) {
            hipEvent_t *e = ev + 2 + 6 * j;
            const int nq = q ^ 1;
            HIPCHK(hipMemsetAsync(P.cnt + CNT_QC(nq), 0, 4, L.s));
            HIPCHK(hipMemsetAsync(P.cnt + CNT_QS(nq), 0, 4, L.s));
            if (dl) HIPCHK(hipMemsetAsync(P.cnt + CNT_DLN, 0, 4, L.s));   // this pass's light-sample list
            HIPCHK(hipEventRecord(e[0], L.s));
            if (serial) {   // closest-hit queries first, alone on the device
                if (instPT) {
                    if (countWork) hipLaunchKernelGGL((k_trace_inst<false, true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    else hipLaunchKernelGGL((k_trace_inst<false, false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                } else if (inst) {
                    if (countWork) hipLaunchKernelGGL((k_trace_closest<true, true>), dim3(traceGrid), dim3(kTraceBlock), lds, L.s, c->S, P, q);
                    else hipLaunchKernelGGL((k_trace_closest<false, true>), dim3(traceGrid), dim3(kTraceBlock), lds, L.s, c->S, P, q);
                } else if (c4 && countWork) hipLaunchKernelGGL((k_trace_c4<true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                else if (c4) hipLaunchKernelGGL((k_trace_c4<false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                else if (countWork) hipLaunchKernelGGL((k_trace_pt<false, true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                else hipLaunchKernelGGL((k_trace_pt<false, false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(e[1], L.s));
                HIPCHK(hipEventRecord(e[2], L.s));
                if (instPT) {
                    if (countWork) hipLaunchKernelGGL((k_trace_inst<true, true>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                    else hipLaunchKernelGGL((k_trace_inst<true, false>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                } else if (inst) {
                    if (countWork) hipLaunchKernelGGL((k_trace_shadow<true, true>), dim3(traceGrid), dim3(kTraceBlock), ldsS, L.s, c->S, P, q);
                    else hipLaunchKernelGGL((k_trace_shadow<false, true>), dim3(traceGrid), dim3(kTraceBlock), ldsS, L.s, c->S, P, q);
                } else if (s4q && countWork) hipLaunchKernelGGL((k_trace_s4q<true>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                else if (s4q) hipLaunchKernelGGL((k_trace_s4q<false>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                else if (s4 && countWork) hipLaunchKernelGGL((k_trace_s4<true>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                else if (s4) hipLaunchKernelGGL((k_trace_s4<false>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                else if (countWork) hipLaunchKernelGGL((k_trace_pt<true, true>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                else hipLaunchKernelGGL((k_trace_pt<true, false>), dim3(ptGridS), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillS);
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(e[3], L.s));
            } else {
                // shadow queries of queue set q on s2, after the counter resets
                HIPCHK(hipStreamWaitEvent(s2, e[0], 0));
                HIPCHK(hipEventRecord(e[2], s2));
                // persistent ray-replacement kernels over the whole (wave-partitioned) queue;
                // instanced scenes run the two-level variant (or, legacy, bvh_walk per thread)
                if (instPT) {
                    if (countWork) hipLaunchKernelGGL((k_trace_inst<false, true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    else hipLaunchKernelGGL((k_trace_inst<false, false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    HIPCHK(hipGetLastError());
                    if (countWork) hipLaunchKernelGGL((k_trace_inst<true, true>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else hipLaunchKernelGGL((k_trace_inst<true, false>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                } else if (inst) {
                    if (countWork) hipLaunchKernelGGL((k_trace_closest<true, true>), dim3(traceGrid), dim3(kTraceBlock), lds, L.s, c->S, P, q);
                    else hipLaunchKernelGGL((k_trace_closest<false, true>), dim3(traceGrid), dim3(kTraceBlock), lds, L.s, c->S, P, q);
                    HIPCHK(hipGetLastError());
                    if (countWork) hipLaunchKernelGGL((k_trace_shadow<true, true>), dim3(traceGrid), dim3(kTraceBlock), ldsS, L.s2, c->S, P, q);
                    else hipLaunchKernelGGL((k_trace_shadow<false, true>), dim3(traceGrid), dim3(kTraceBlock), ldsS, L.s2, c->S, P, q);
                } else {
                    if (c4 && countWork) hipLaunchKernelGGL((k_trace_c4<true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    else if (c4) hipLaunchKernelGGL((k_trace_c4<false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    else if (countWork) hipLaunchKernelGGL((k_trace_pt<false, true>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    else hipLaunchKernelGGL((k_trace_pt<false, false>), dim3(ptGrid), dim3(kTraceBlock), 0, L.s, c->S, P, q, c->refill, c->ring, spillC);
                    HIPCHK(hipGetLastError());
                    if (s4q && countWork) hipLaunchKernelGGL((k_trace_s4q<true>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else if (s4q) hipLaunchKernelGGL((k_trace_s4q<false>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else if (s4 && countWork) hipLaunchKernelGGL((k_trace_s4<true>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else if (s4) hipLaunchKernelGGL((k_trace_s4<false>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else if (countWork) hipLaunchKernelGGL((k_trace_pt<true, true>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                    else hipLaunchKernelGGL((k_trace_pt<true, false>), dim3(ptGridS), dim3(kTraceBlock), 0, s2, c->S, P, q, c->refill, c->ring, spillS);
                }
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(e[1], L.s));
                HIPCHK(hipEventRecord(e[3], s2));
                HIPCHK(hipStreamWaitEvent(L.s, e[3], 0));
            }
            T.launches[K_CLOSEST]++;
            T.launches[K_SHADOW]++;
            HIPCHK(hipEventRecord(e[4], L.s));
            L.P.pass = (L.P.pass + 1) % 3;
            HIPCHK(drain_list(L, r.drain, r.cap));
            HIPCHK(kShade(r.drain ? r.liveGrid : r.grid, L.s, c->S, P, r.src, nq, Lout));
            if (dl) {
                const int g = r.drain ? r.liveGrid : r.grid;
                HIPCHK(kNee(g, L.s, c->S, L.P, nq));
                HIPCHK(kSpec(g, L.s, c->S, L.P, r.src, nq, Lout));
            }
            if (mtList) HIPCHK(launch_mt_init(L.s, P, nq));
            T.launches[K_SHADE]++;
            HIPCHK(hipEventRecord(e[5], L.s));
            T.passes++;
            r.passes++;
            r.listPasses += r.drain ? 1 : 0;
            q = nq;
        }
        r.q = q;
        return close_batch(r, bi, Batch{n, false, r.drain, r.liveGrid, q});
    };
    // a second batch may be enqueued behind the one in flight (pipe_mode)
    const int pipe = pipe_mode();
    auto pipe_far = [&](const Run &r, const uint32_t *cnt) -> bool {
        return pipe == 2 || (pipe == 1 && (uint64_t)cnt[CNT_NEXT] + 2ull * (uint64_t)r.cap < r.src.nItems);
    };
    HIPCHK(hipEventRecord(c->ev[0], c->stream));   // the other lanes start after the work queued so far
    for (int l = 0; l < nl; ++l) {
        Run &r = R[l];
        Lane &L = c->lane[l];
        r.L = &L;
        r.src = src;
        const uint32_t lo = (uint32_t)((uint64_t)src.nItems * l / nl), hi = (uint32_t)((uint64_t)src.nItems * (l + 1) / nl);
        r.src.base = src.base + lo;
        r.src.nItems = hi - lo;
        r.cap = lane_slots(r.src.nItems, nl);
        if (dl)   // the frame stacks and light-sample batches: at most 24 GiB per lane
            r.cap = (int)std::max<size_t>(64, std::min<size_t>((size_t)r.cap, ((size_t)24 << 30) /
                                                               (frame_bytes(NB) * nFrames + batch_bytes(NB) * batch)));
        if (mtExt && !getenv("PBRTGPU_SLOTS")) r.cap = std::min(r.cap, 1 << 20);   // 2.5 KiB of MT state per slot
        r.cap = std::min(r.cap, max_slots_32bit(NB, batch));
        r.grid = (r.cap + kShadeBlock - 1) / kShadeBlock;
        r.q = 0;
        r.done = false;
        r.drain = false;
        r.ending = false;
        r.tailed = false;
        r.liveGrid = r.grid;
        r.listPasses = 0;
        r.head = 0;
        r.inflight = 0;
        L.P.listMode = 0;
        L.P.xcdMap = xcd_map_on();
        // drain bound of this run: a path lives at most pathPasses passes, so every slot
        // takes a new item at least once per pathPasses passes while items remain; twice
        // that, plus the overshoot of the enqueued batches, means the wavefront is stuck
        r.passes = 0;
        r.maxPasses = (int)std::min<int64_t>(INT32_MAX / 2, 2 * ((r.src.nItems + r.cap - 1) / r.cap + 1) * pathPasses) +
                      4 * kPassBatch;
        if (int e = ensure_slots(&L, r.cap, NB, c->S.nInsts, nFrames, batch, mtExt)) return e;
        HIPCHK(L.spill.ensure(2 * spillLane * sizeof(uint2)));
        if (l > 0) HIPCHK(hipStreamWaitEvent(L.s, c->ev[0], 0));
        if (const int pb = poison_byte(); pb >= 0) {
            HIPCHK(hipMemsetAsync(L.slots.p, pb, L.slots.n, L.s));
            HIPCHK(hipMemsetAsync(L.spill.p, pb, L.spill.n, L.s));
        }
        HIPCHK(hipMemsetAsync(L.P.item, 0xff, (size_t)r.cap * 4, L.s));
        HIPCHK(hipMemsetAsync(L.P.cnt, 0, CNT_WORDS * 4, L.s));
        {   // the per-wave writer masks start empty: k_shade loads a wave's masks before it knows
            // which of them its lanes will use (wave_masks), so none is read unwritten
            const size_t W = (size_t)((r.cap + 63) / 64) * 8;
            HIPCHK(hipMemsetAsync(L.P.aMask, 0, 2 * W, L.s));
            HIPCHK(hipMemsetAsync(L.P.bMask, 0, 3 * W, L.s));
            HIPCHK(hipMemsetAsync(L.P.mMask, 0, 2 * W, L.s));
        }
        // pass 0: every slot is free -> regeneration fills them with camera rays (queue 0)
        HIPCHK(hipEventRecord(L.ev[0][0], L.s));
        L.P.pass = 0;   // k_shade pass index (mod 3) of this run: the beta buffers rotate with it
        HIPCHK(kShade(r.grid, L.s, c->S, L.P, r.src, 0, Lout));
        HIPCHK(hipEventRecord(L.ev[0][1], L.s));
        if (int e = close_batch(r, 0, Batch{0, true, false, r.grid, 0})) return e;
        // ... and the first batch of passes right behind it when the lane is far from its drain:
        // after pass 0 the slots hold the first min(cap, items) items (every slot regenerated),
        // each with its camera ray queued
        uint32_t c0[CNT_WORDS] = {};
        c0[CNT_NEXT] = (uint32_t)std::min<uint64_t>((uint64_t)r.cap, r.src.nItems);
        c0[CNT_QC(0)] = (uint32_t)r.cap;
        if (pipe_far(r, c0))
            if (int e = enqueue(r, c0, 0)) return e;
    }
    int live = nl;
    float m;
    int rr = 0;   // round-robin start of the lane poll
    while (live > 0) {
        // the next lane whose oldest batch has completed: the host never blocks on one lane while
        // the other lane's queue has run dry (it would idle until that wait ended)
        int l = -1;
        int spins = 0;
        for (;;) {
            for (int k = 0; k < nl && l < 0; ++k) {
                const int i = (rr + k) % nl;
                if (R[i].done) continue;
                const hipError_t qe = hipEventQuery(R[i].L->done[R[i].head]);
                if (qe == hipSuccess) l = i;
                else if (qe != hipErrorNotReady) HIPCHK(qe);
            }
            if (l >= 0) break;
            // a few empty polls, then short sleeps: a batch of passes takes milliseconds, and a host
            // thread per device (render_multi) should not burn a core for the whole frame
            if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
            else std::this_thread::yield();
        }
        rr = l + 1;
        Run &r = R[l];
        Lane &L = *r.L;
        const int bi = r.head;
        const Batch B = r.b[bi];
        uint32_t cnt[CNT_WORDS];
        memcpy(cnt, L.hostCnt[bi], sizeof(cnt));
        r.head ^= 1;
        r.inflight--;
        if (B.single) {
            HIPCHK(hipEventElapsedTime(&m, L.ev[bi][0], L.ev[bi][1])); T.ms[K_SHADE] += m;
            T.launches[K_SHADE]++;
        }
        for (int j = 0; j < B.n; ++j) {
            hipEvent_t *e = L.ev[bi] + 2 + 6 * j;
            float mc, ms, mh;
            HIPCHK(hipEventElapsedTime(&mc, e[0], e[1])); T.ms[K_CLOSEST] += mc;
            HIPCHK(hipEventElapsedTime(&ms, e[2], e[3])); T.ms[K_SHADOW] += ms;
            HIPCHK(hipEventElapsedTime(&mh, e[4], e[5])); T.ms[K_SHADE] += mh;
            if (pass_log())   // diagnostics: per-pass device time of each lane
                fprintf(stderr, "pass_log lane %d closest %.3f shadow %.3f shade %.3f\n", l, mc, ms, mh);
        }
        if (pass_log())
            fprintf(stderr, "pass_log lane %d batch of %d%s: closest queue %u shadow queue %u items taken %u of %u%s\n", l,
                    B.n, B.single ? " (single launch)" : "", cnt[CNT_QC(B.qEnd)], cnt[CNT_QS(B.qEnd)], cnt[CNT_NEXT],
                    r.src.nItems, B.drain ? " (drain list)" : "");
        if (cnt[CNT_ERR] & 1u) return fail(PBRTGPU_E_STATE, "a path drew past 227 MT19937 outputs without its state row");
        if (cnt[CNT_ERR] & 2u) return fail(PBRTGPU_E_STATE, "drain: a pass's live list exceeded its shade grid");
        if (cnt[CNT_ERR] & 4u) return fail(PBRTGPU_E_STATE, "tail: the live list exceeded the tail kernel's grid");
        if (cnt[CNT_ERR] & 8u) return fail(PBRTGPU_E_STATE, "tail: a path was still live after the tail kernel's steps");
        // every live slot ends a pass with a ray queued, so the drain's list fits the grid sized
        // from the queue sizes of an earlier read-back; a longer list would leave slots unshaded
        // (their beta / A / B buffers then rotate under them): refuse instead
        if (B.drain && !B.single && (uint64_t)cnt[CNT_LIVE] > (uint64_t)B.liveGrid * kShadeBlock)
            return fail(PBRTGPU_E_STATE, "drain: more live slots than the shade grid covers");
        if (cnt[CNT_QC(B.qEnd)] == 0 && cnt[CNT_QS(B.qEnd)] == 0) r.ending = true;   // nothing queued: empty from here on
        if (r.ending || r.tailed) {
            if (r.inflight > 0) continue;   // the batch behind it (empty passes, or the tail) completes first
            if (!r.ending) return fail(PBRTGPU_E_STATE, "tail: paths left after the tail kernel");
            r.done = true;
            --live;
            uint64_t w[W_COUNT];
            HIPCHK(hipMemcpy(w, L.P.cnt + CNT_WORK, sizeof(w), hipMemcpyDeviceToHost));
            if (countWork)
                for (int i = 0; i < W_COUNT; ++i) T.work[i] += w[i];
            if (zeroedOut) *zeroedOut += cnt[CNT_ZEROED];
            continue;
        }
        if (r.passes > r.maxPasses) return fail(PBRTGPU_E_STATE, "wavefront did not drain");
        // a batch still in flight behind this one: enqueue behind it only far from the drain;
        // otherwise decide at its read-back, from its counters
        if (r.inflight > 0 && !pipe_far(r, cnt)) continue;
        if (int e = enqueue(r, cnt, B.qEnd)) return e;
    }
    if (c->S.specMode == 1) {   // the rows' luminance guard once every band of them is in
        for (int l = 1; l < nl; ++l) {
            HIPCHK(hipEventRecord(c->ev[1], c->lane[l].s));
            HIPCHK(hipStreamWaitEvent(c->stream, c->ev[1], 0));
        }
        const uint32_t rows = src.nItems / (uint32_t)c->S.specItems;
        hipLaunchKernelGGL(k_spec_guard<NB>, dim3((rows + 255) / 256), dim3(256), 0, c->stream, c->S, Lout, rows);
        HIPCHK(hipGetLastError());
    }
    return 0;
}


extern "C" {

int pbrtgpu_abi_version(void) { return PBRTGPU_ABI_VERSION; }
const char *pbrtgpu_last_error(void) { return g_err.c_str(); }

int pbrtgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pbrtgpu_context_create(int device, pbrtgpu_ctx **out) {
    if (!out) return fail(PBRTGPU_E_INVALID, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(PBRTGPU_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= n) return fail(PBRTGPU_E_INVALID, "bad device index");
    HIPCHK(hipSetDevice(device));
    pbrtgpu_ctx *c = new pbrtgpu_ctx();
    c->device = device;
    if (const char *e = getenv("PBRTGPU_REFILL")) c->refill = std::max(1, std::min(64, atoi(e)));
    if (const char *e = getenv("PBRTGPU_STACK_LDS")) {
        const int r = atoi(e);
        if (r >= 1 && r <= kStackLDS && (r & (r - 1)) == 0) c->ring = r;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->numCUs = prop.multiProcessorCount;
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; i < 8 && ok; ++i) ok = hipEventCreate(&c->ev[i]) == hipSuccess;
    for (int l = 0; l < kLanes && ok; ++l) {
        Lane &L = c->lane[l];
        if (l == 0) L.s = c->stream;
        else ok = hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking) == hipSuccess;
        ok = ok && hipStreamCreateWithFlags(&L.s2, hipStreamNonBlocking) == hipSuccess;
        for (int b = 0; b < 2; ++b) {
            for (int i = 0; i < 2 + 6 * 8 && ok; ++i) ok = hipEventCreate(&L.ev[b][i]) == hipSuccess;
            ok = ok && hipEventCreateWithFlags(&L.done[b], hipEventDisableTiming) == hipSuccess;
            ok = ok && hipHostMalloc((void **)&L.hostCnt[b], CNT_WORDS * 4, hipHostMallocDefault) == hipSuccess;
        }
    }
    if (!ok) {
        delete c;
        return fail(PBRTGPU_E_NODEVICE, "stream/event creation failed");
    }
    *out = c;
    return 0;
}

int pbrtgpu_context_destroy(pbrtgpu_ctx *c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto &b : c->sceneBufs) b.release();
    DevBuf *bufs[] = {&c->film, &c->Lbuf, &c->pix, &c->filmIdx, &c->mask, &c->keys, &c->counter, &c->spillL,
                      &c->lists[0], &c->lists[1], &c->lists[2], &c->lists[3], &c->scratch[0],
                      &c->scratch[1], &c->scratch[2], &c->gather[0], &c->gather[1]};
    for (DevBuf *b : bufs) b->release();
    c->stage.release();
    for (int i = 0; i < 8; ++i) if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    for (Lane &L : c->lane) {
        if (L.s && L.s != c->stream) (void)hipStreamSynchronize(L.s);
        if (L.s2) (void)hipStreamSynchronize(L.s2);
        L.slots.release();
        L.spill.release();
        for (int b = 0; b < 2; ++b) {
            for (hipEvent_t e : L.ev[b]) if (e) (void)hipEventDestroy(e);
            if (L.done[b]) (void)hipEventDestroy(L.done[b]);
            if (L.hostCnt[b]) (void)hipHostFree(L.hostCnt[b]);
        }
        if (L.s2) (void)hipStreamDestroy(L.s2);
        if (L.s && L.s != c->stream) (void)hipStreamDestroy(L.s);
    }
    (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}
int pbrtgpu_scene_upload(pbrtgpu_ctx *c, const pbrtgpu_flat_scene *s) {
    if (!c || !s) return fail(PBRTGPU_E_INVALID, "null argument");
    c->sceneGen++;               // the cached render setup belongs to the previous scene
    c->setup.valid = false;
    std::string err;
    if (int e = scene_check(s, &err)) return fail(e, err);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->hasScene = false;
    for (auto &b : c->sceneBufs) b.release();
    c->sceneBufs.clear();
    c->sceneBufs.reserve(64);
    DevScene &S = c->S;
    hipError_t he = hipSuccess;
    auto put = [&](auto *src, size_t count, auto **dst) -> int {
        he = upload(c, src, count, dst);
        return he == hipSuccess ? 0 : PBRTGPU_E_NODEVICE;
    };
    if (int e = scene_build(s, top_nodes(), S, &c->feat, put, &err)) {
        if (he != hipSuccess) return fail(-(1000 + (int)he), std::string("scene upload: ") + hipGetErrorString(he));
        return fail(e, err);
    }
    c->stackDepth = S.stackDepth;
    if (const char *e = getenv("PBRTGPU_KD_LDS"))   // tests: force the global-memory walk
        if (atoi(e) == 0) S.kdInLds = 0;
    if (const char *e = getenv("PBRTGPU_SHADE_FULL"))   // tests: run the full variant on any scene
        if (atoi(e) != 0) c->feat = FEAT_ALL;
    c->nb = s->n_bands;
    c->spp = s->spp;
    c->cam = s->camera;
    size_t filmFloats = (size_t)s->camera.px_count * s->camera.py_count * s->n_bands;
    HIPCHK(c->film.ensure(filmFloats * 4));
    HIPCHK(hipMemsetAsync(c->film.p, 0, filmFloats * 4, c->stream));
    HIPCHK(c->counter.ensure(16));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->hasScene = true;
    return 0;
}

int pbrtgpu_film_clear(pbrtgpu_ctx *c) {
    if (!c || !c->hasScene) return fail(PBRTGPU_E_STATE, "no scene");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(c->film.p, 0, (size_t)c->cam.px_count * c->cam.py_count * c->nb * 4, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int pbrtgpu_film_read(pbrtgpu_ctx *c, float *out, int64_t n) {
    if (!c || !c->hasScene || !out) return fail(PBRTGPU_E_STATE, "no scene / null out");
    size_t need = (size_t)c->cam.px_count * c->cam.py_count * c->nb;
    if ((size_t)n < need) return fail(PBRTGPU_E_INVALID, "film buffer too small");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->stage.ensure(need * 4));
    HIPCHK(hipMemcpyAsync(c->stage.p, c->film.p, need * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const char *src = (const char *)c->stage.p;
    par_for(need * 4, (size_t)4 << 20, [&](size_t lo, size_t hi) { memcpy((char *)out + lo, src + lo, hi - lo); });
    return 0;
}

}  // extern "C"

// Film pixels of a tile list.  Tiles are tile_w x tile_h blocks of the FILM pixel window
// (px_count x py_count, row-major tile ids, ragged last row / column); tile_ids == NULL
// means every tile.  fidx = film indices (y * px_count + x) in tile order without repeats,
// mask = 1 on those pixels.
static int tile_pixels(const pbrtgpu_camera &cam, int tile_w, int tile_h, const int32_t *tiles, int32_t ntiles,
                       std::vector<int> *fidx, std::vector<uint8_t> *mask) {
    const int tw = tile_w > 0 ? tile_w : 16, th = tile_h > 0 ? tile_h : 16;
    const int ntx = (cam.px_count + tw - 1) / tw, nty = (cam.py_count + th - 1) / th;
    mask->assign((size_t)cam.px_count * cam.py_count, 0);
    fidx->clear();
    auto addTile = [&](int t) {
        int tx = t % ntx, ty = t / ntx;
        for (int y = ty * th; y < std::min(cam.py_count, (ty + 1) * th); ++y)
            for (int x = tx * tw; x < std::min(cam.px_count, (tx + 1) * tw); ++x) {
                size_t fi = (size_t)y * cam.px_count + x;
                if ((*mask)[fi]) continue;
                (*mask)[fi] = 1;
                fidx->push_back((int)fi);
            }
    };
    if (!tiles) for (int t = 0; t < ntx * nty; ++t) addTile(t);
    else {
        if (ntiles < 0) return fail(PBRTGPU_E_INVALID, "negative tile count");
        for (int i = 0; i < ntiles; ++i) {
            if (tiles[i] < 0 || tiles[i] >= ntx * nty) return fail(PBRTGPU_E_INVALID, "tile id out of range");
            addTile(tiles[i]);
        }
    }
    return 0;
}

template <int NB>
static int render_impl(pbrtgpu_ctx *c, const pbrtgpu_render_desc *d, const int32_t *tiles, int32_t ntiles, double *stats) {
    const pbrtgpu_camera &cam = c->cam;
    const int spp = c->spp;
    int s0 = d->spp_begin, s1 = d->spp_end;
    if (s0 < 0 || s1 > spp || s0 >= s1) return fail(PBRTGPU_E_INVALID, "bad sample range");
    const bool countWork = (d->flags & PBRTGPU_F_COUNT_WORK) != 0;
    Timing T;
    double st[PBRTGPU_STAT_COUNT] = {0};
    if (!(d->flags & PBRTGPU_F_ACCUMULATE) && s0 == 0)
        HIPCHK(hipMemsetAsync(c->film.p, 0, (size_t)cam.px_count * cam.py_count * NB * 4, c->stream));
    pbrtgpu_ctx::CallSetup &cs = c->setup;
    const bool same = cs.valid && cs.gen == c->sceneGen && cs.tw == d->tile_w && cs.th == d->tile_h && cs.s0 == s0 &&
                      cs.s1 == s1 && (tiles ? (!cs.all && cs.tiles.size() == (size_t)std::max(0, ntiles) &&
                                               std::equal(cs.tiles.begin(), cs.tiles.end(), tiles))
                                            : cs.all);
    std::vector<int> fidx;
    std::vector<uint8_t> mask;
    if (!same) {
        cs.valid = false;
        // pixel list of the requested tiles (film pixels; own sample pixel == film pixel)
        if (int e = tile_pixels(cam, d->tile_w, d->tile_h, tiles, ntiles, &fidx, &mask)) return e;
        std::vector<int2> pix(fidx.size());
        for (size_t i = 0; i < fidx.size(); ++i)
            pix[i] = make_int2(cam.px_start + fidx[i] % cam.px_count, cam.py_start + fidx[i] / cam.px_count);
        cs.nPix = (int)pix.size();
        if (cs.nPix > 0) {
            HIPCHK(c->pix.ensure(pix.size() * sizeof(int2)));
            HIPCHK(c->filmIdx.ensure(fidx.size() * sizeof(int)));
            HIPCHK(hipMemcpyAsync(c->pix.p, pix.data(), pix.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(c->filmIdx.p, fidx.data(), fidx.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));   // the host vectors go out of scope
        }
    }
    const int nPix = cs.nPix;
    if (nPix == 0) { if (stats) memcpy(stats, st, sizeof(st)); c->last = T; return 0; }
    unsigned int zeroed = 0;

    // ---- spill samples of the call's sample range [s0, s1).  A frame rendered as one call
    // adds every pixel's contributions in the reference's order; a frame split into sample
    // ranges (F_ACCUMULATE) adds the same contributions, range by range, so its sums differ
    // from the one-call film only in float summation order
    std::vector<int> &preT = cs.preT, &preStart = cs.preStart, &preSrc = cs.preSrc, &postT = cs.postT,
                     &postStart = cs.postStart, &postSrc = cs.postSrc;
    if (!same) {
        preT.clear(); preStart.clear(); preSrc.clear(); postT.clear(); postStart.clear(); postSrc.clear();
        cs.nSpill = 0;
        cs.spills = 0;
        HIPCHK(c->mask.ensure(mask.size()));
        HIPCHK(hipMemcpyAsync(c->mask.p, mask.data(), mask.size(), hipMemcpyHostToDevice, c->stream));
        unsigned int cap = 1u << 20;
        HIPCHK(c->keys.ensure((size_t)cap * sizeof(int3)));
        HIPCHK(c->counter.ensure(16));
        HIPCHK(hipMemsetAsync(c->counter.p, 0, 16, c->stream));
        long npx = (long)(cam.sx_end - cam.sx_start) * (cam.sy_end - cam.sy_start);
        int grid = (int)std::min<long>((npx + 255) / 256, (long)c->numCUs * 16);
        hipLaunchKernelGGL(k_spill_scan, dim3(grid), dim3(256), 0, c->stream, cam, c->S.seed, spp, s0, s1,
                           (const uint8_t *)c->mask.p, (int3 *)c->keys.p, (unsigned int *)c->counter.p, cap);
        HIPCHK(hipGetLastError());
        unsigned int cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, c->counter.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (cnt > cap) return fail(PBRTGPU_E_UNSUPPORTED, "too many exact-boundary samples");
        const int nSpill = (int)cnt;
        cs.nSpill = nSpill;
        if (nSpill > 0) {
            std::vector<int3> keys(nSpill);
            HIPCHK(hipMemcpy(keys.data(), c->keys.p, nSpill * sizeof(int3), hipMemcpyDeviceToHost));
            // canonical order: (source row-major, sample)
            std::sort(keys.begin(), keys.end(), [](const int3 &a, const int3 &b) {
                if (a.y != b.y) return a.y < b.y;
                if (a.x != b.x) return a.x < b.x;
                return a.z < b.z;
            });
            HIPCHK(hipMemcpy(c->keys.p, keys.data(), nSpill * sizeof(int3), hipMemcpyHostToDevice));
            // the spill samples are traced with the first batch (items after its pixel
            // samples), so they cost no wavefront fill and drain of their own
            HIPCHK(c->spillL.ensure((size_t)nSpill * NB * 4));
            // contributions per target pixel, split into pre (source before the target's own
            // sample pixel in row-major order) and post
            const int ew = cam.sx_end - cam.sx_start;
            struct Cb { int target; long src; int s; int idx; };
            std::vector<Cb> cbs;
            for (int k = 0; k < nSpill; ++k) {
                int x = keys[k].x, y = keys[k].y, s = keys[k].z;
                uint32_t hp = pixel_hash(c->S.seed, x, y);
                float u[2];
                s2d(hp, 0, (uint32_t)s, (uint32_t)spp, u);   // same sampler as k_spill_scan
                float ix = x + u[0], iy = y + u[1];
                float dx = ix - 0.5f, dy = iy - 0.5f;
                int fx0 = (int)ceilf(dx - 0.5f), fx1 = (int)floorf(dx + 0.5f);
                int fy0 = (int)ceilf(dy - 0.5f), fy1 = (int)floorf(dy + 0.5f);
                fx0 = std::max(fx0, cam.px_start); fx1 = std::min(fx1, cam.px_start + cam.px_count - 1);
                fy0 = std::max(fy0, cam.py_start); fy1 = std::min(fy1, cam.py_start + cam.py_count - 1);
                for (int fy = fy0; fy <= fy1; ++fy)
                    for (int fx = fx0; fx <= fx1; ++fx) {
                        if (fx == x && fy == y) continue;
                        int target = (fy - cam.py_start) * cam.px_count + (fx - cam.px_start);
                        if (!mask[target]) continue;
                        cbs.push_back(Cb{target, (long)(y - cam.sy_start) * ew + (x - cam.sx_start), s, k});
                    }
            }
            std::sort(cbs.begin(), cbs.end(), [](const Cb &a, const Cb &b) {
                if (a.target != b.target) return a.target < b.target;
                if (a.src != b.src) return a.src < b.src;
                return a.s < b.s;
            });
            for (size_t i = 0; i < cbs.size(); ++i) {
                const Cb &q = cbs[i];
                int tx = q.target % cam.px_count + cam.px_start, ty = q.target / cam.px_count + cam.py_start;
                long own = (long)(ty - cam.sy_start) * ew + (tx - cam.sx_start);
                bool pre = q.src < own;
                std::vector<int> &Tg = pre ? preT : postT, &ST = pre ? preStart : postStart, &SR = pre ? preSrc : postSrc;
                if (Tg.empty() || Tg.back() != q.target) { Tg.push_back(q.target); ST.push_back((int)SR.size()); }
                SR.push_back(q.idx);
            }
            preStart.push_back((int)preSrc.size());
            postStart.push_back((int)postSrc.size());
            cs.spills = (double)cbs.size();
        }
        cs.valid = true;
        cs.gen = c->sceneGen;
        cs.tw = d->tile_w; cs.th = d->tile_h; cs.s0 = s0; cs.s1 = s1;
        cs.all = tiles == nullptr;
        if (tiles) cs.tiles.assign(tiles, tiles + std::max(0, ntiles));
        else cs.tiles.clear();
    }
    const int nSpill = cs.nSpill;
    st[PBRTGPU_STAT_SPILLS] = cs.spills;
    auto applyLists = [&](std::vector<int> &Tg, std::vector<int> &ST, std::vector<int> &SR) -> int {
        if (Tg.empty()) return 0;
        HIPCHK(c->lists[0].ensure(Tg.size() * 4));
        HIPCHK(c->lists[1].ensure(ST.size() * 4));
        HIPCHK(c->lists[2].ensure(SR.size() * 4));
        HIPCHK(hipMemcpyAsync(c->lists[0].p, Tg.data(), Tg.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->lists[1].p, ST.data(), ST.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->lists[2].p, SR.data(), SR.size() * 4, hipMemcpyHostToDevice, c->stream));
        long n = (long)Tg.size() * NB;
        hipLaunchKernelGGL(k_apply, dim3((n + 255) / 256), dim3(256), 0, c->stream, (int)Tg.size(), (const int *)c->lists[0].p,
                           (const int *)c->lists[1].p, (const int *)c->lists[2].p, (const float *)c->spillL.p, NB,
                           (float *)c->film.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->stream));   // host vectors are reused right after
        return 0;
    };

    // ---- main batches: per-sample radiance for (pixels x batch samples), then the ordered film sum
    const size_t lbudget = lbuf_budget();   // per-sample radiance per batch
    int sb = (int)std::max<long>(1, std::min<long>(s1 - s0, (long)(lbudget / ((size_t)nPix * NB * 4))));
    const uint64_t bi = (uint64_t)c->S.specItems;   // paths per camera sample (SpectralRenderer bands)
    if (((uint64_t)nPix * sb + nSpill) * bi > 0x7fffffffull) sb = (int)((0x7fffffffll / bi - nSpill) / nPix);
    if (sb < 1) return fail(PBRTGPU_E_UNSUPPORTED, "render call too large for 31-bit path items");
    HIPCHK(c->Lbuf.ensure(((size_t)nPix * sb + nSpill) * NB * 4));
    for (int b0 = s0; b0 < s1; b0 += sb) {
        int n = std::min(sb, s1 - b0);
        ItemSrc src{};
        src.pix = (const int2 *)c->pix.p;
        src.sb = n;
        src.s0 = b0;
        src.nItems = (uint32_t)((long)nPix * n);
        const bool withSpills = b0 == s0 && nSpill > 0;
        if (withSpills) {
            src.keys = (const int3 *)c->keys.p;
            src.keyBase = src.nItems;
            src.nItems += (uint32_t)nSpill;
        }
        src.nItems *= (uint32_t)bi;   // keyBase stays in samples
        if (const int pb = poison_byte(); pb >= 0)   // an item no path writes reads as the byte (not last batch's)
            HIPCHK(hipMemsetAsync(c->Lbuf.p, pb, (size_t)src.nItems * NB * 4, c->stream));
        if (int e = run_wavefront<NB>(c, src, (float *)c->Lbuf.p, countWork, T, &zeroed)) return e;
        if (withSpills) {   // keep the spill radiance (later batches reuse Lbuf), add the pre lists
            HIPCHK(hipMemcpyAsync(c->spillL.p, (const float *)c->Lbuf.p + (size_t)src.keyBase * NB,
                                  (size_t)nSpill * NB * 4, hipMemcpyDeviceToDevice, c->stream));
            if (int e = applyLists(preT, preStart, preSrc)) return e;
        }
        long na = (long)nPix * NB;
        HIPCHK(hipEventRecord(c->ev[6], c->stream));
        hipLaunchKernelGGL(k_accum<NB>, dim3((na + 255) / 256), dim3(256), 0, c->stream, (const float *)c->Lbuf.p,
                           (const int *)c->filmIdx.p, nPix, n, (float *)c->film.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->ev[7], c->stream));
        HIPCHK(hipEventSynchronize(c->ev[7]));
        float m2 = 0.f;
        HIPCHK(hipEventElapsedTime(&m2, c->ev[6], c->ev[7]));
        T.ms[K_ACCUM] += m2;
        T.launches[K_ACCUM]++;
        st[PBRTGPU_STAT_PATHS] += (double)((long)nPix * n) * (double)bi;
    }
    if (int e = applyLists(postT, postStart, postSrc)) return e;
    HIPCHK(hipStreamSynchronize(c->stream));
#ifdef PGD_SECTIONS
    {   // timing experiment: wave-cycles per k_shade section of this render
        unsigned long long sec[SEC_N];
        if (pgd_sections_read(sec, 1) == 0) {
            static const char *nm[] = {"load", "finish", "isect", "bsdf", "light", "mis", "cont", "out", "regen", "push",
                                       "[light: sample", "eval", "store]", "[cont: sample", "bands]"};
            unsigned long long tot = 0;
            for (int k = 0; k < SEC_PUSH + 1; ++k) tot += sec[k];
            fprintf(stderr, "sections:");
            for (int k = 0; k < SEC_CBAND + 1; ++k) fprintf(stderr, " %s %.1f%%", nm[k], 100.0 * sec[k] / std::max(1ull, tot));
            fprintf(stderr, "  (total %.3e wave-cycles)\n", (double)tot);
        }
    }
#endif
    st[PBRTGPU_STAT_KERNEL_MS] = T.ms[K_CLOSEST] + T.ms[K_SHADOW] + T.ms[K_SHADE];
    st[PBRTGPU_STAT_ACCUM_MS] = T.ms[K_ACCUM];
    st[PBRTGPU_STAT_ZEROED] = zeroed;
    st[PBRTGPU_STAT_PASSES] = T.passes;
    c->last = T;
    if (stats) memcpy(stats, st, sizeof(st));
    return 0;
}

extern "C" {

int pbrtgpu_render_tiles(pbrtgpu_ctx *c, const pbrtgpu_render_desc *d, const int32_t *tile_ids, int32_t ntiles,
                         double *stats) {
    if (!c || !c->hasScene || !d) return fail(PBRTGPU_E_STATE, "no scene / null desc");
    HIPCHK(hipSetDevice(c->device));
    switch (c->nb) {
        case 32: return render_impl<32>(c, d, tile_ids, ntiles, stats);
        case 60: return render_impl<60>(c, d, tile_ids, ntiles, stats);
        case 3: return render_impl<3>(c, d, tile_ids, ntiles, stats);
        case 30: return render_impl<30>(c, d, tile_ids, ntiles, stats);
    }
    return fail(PBRTGPU_E_UNSUPPORTED, "band count");
}

int pbrtgpu_film_gather(pbrtgpu_ctx *c, int32_t tile_w, int32_t tile_h, const int32_t *tile_ids, int32_t ntiles,
                        float *film_out, int64_t n_floats) {
    if (!c || !c->hasScene || !film_out) return fail(PBRTGPU_E_STATE, "no scene / null out");
    if (!tile_ids) return pbrtgpu_film_read(c, film_out, n_floats);
    const size_t need = (size_t)c->cam.px_count * c->cam.py_count * c->nb;
    if (n_floats < 0 || (size_t)n_floats < need) return fail(PBRTGPU_E_INVALID, "film buffer too small");
    std::vector<int> fidx;
    std::vector<uint8_t> mask;
    if (int e = tile_pixels(c->cam, tile_w, tile_h, tile_ids, ntiles, &fidx, &mask)) return e;
    if (fidx.empty()) return 0;
    HIPCHK(hipSetDevice(c->device));
    const int nb = c->nb, nPix = (int)fidx.size();
    HIPCHK(c->gather[0].ensure(fidx.size() * sizeof(int)));
    HIPCHK(c->gather[1].ensure((size_t)nPix * nb * 4));
    HIPCHK(hipMemcpyAsync(c->gather[0].p, fidx.data(), fidx.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    const long n = (long)nPix * nb;
    hipLaunchKernelGGL(k_pack, dim3((n + 255) / 256), dim3(256), 0, c->stream, (const float *)c->film.p,
                       (const int *)c->gather[0].p, nPix, nb, (float *)c->gather[1].p);
    HIPCHK(hipGetLastError());
    HIPCHK(c->stage.ensure((size_t)n * 4));
    HIPCHK(hipMemcpyAsync(c->stage.p, c->gather[1].p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const float *packed = (const float *)c->stage.p;
    par_for((size_t)nPix, (size_t)1 << 15, [&](size_t lo, size_t hi) {
        for (size_t p = lo; p < hi; ++p) memcpy(film_out + (size_t)fidx[p] * nb, packed + p * nb, (size_t)nb * 4);
    });
    return 0;
}

int pbrtgpu_render_multi(pbrtgpu_ctx *const *ctxs, int32_t n, const pbrtgpu_render_desc *desc, const int32_t *tile_ids,
                         int32_t ntiles, int32_t slices_per_ctx, float *film_out, int64_t n_floats, double *stats_out) {
    if (!ctxs || n <= 0 || !desc || !film_out) return fail(PBRTGPU_E_INVALID, "bad arguments");
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i] || !ctxs[i]->hasScene) return fail(PBRTGPU_E_STATE, "context without a scene");
        for (int j = 0; j < i; ++j)
            if (ctxs[j] == ctxs[i]) return fail(PBRTGPU_E_INVALID, "a context is listed twice");
        const pbrtgpu_camera &a = ctxs[0]->cam, &b = ctxs[i]->cam;
        if (ctxs[i]->nb != ctxs[0]->nb || ctxs[i]->spp != ctxs[0]->spp || a.px_count != b.px_count ||
            a.py_count != b.py_count || a.px_start != b.px_start || a.py_start != b.py_start)
            return fail(PBRTGPU_E_INVALID, "contexts hold different scenes / films");
    }
    const pbrtgpu_camera &cam = ctxs[0]->cam;
    if (n_floats < 0 || (size_t)n_floats < (size_t)cam.px_count * cam.py_count * ctxs[0]->nb)
        return fail(PBRTGPU_E_INVALID, "film buffer too small");
    // the frame's tile list, dealt into m interleaved slices (slice j = list[j], list[j + m], ...):
    // each slice spreads over the whole image, so slices cost about the same
    const int tw = desc->tile_w > 0 ? desc->tile_w : 16, th = desc->tile_h > 0 ? desc->tile_h : 16;
    const int ntx = (cam.px_count + tw - 1) / tw, nty = (cam.py_count + th - 1) / th;
    std::vector<int32_t> list;
    if (tile_ids) {
        if (ntiles < 0) return fail(PBRTGPU_E_INVALID, "negative tile count");
        list.assign(tile_ids, tile_ids + ntiles);
    } else
        for (int t = 0; t < ntx * nty; ++t) list.push_back(t);
    for (int32_t t : list)
        if (t < 0 || t >= ntx * nty) return fail(PBRTGPU_E_INVALID, "tile id out of range");
    const int m = n * std::max(1, (int)slices_per_ctx);
    std::atomic<int> next(0);
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    std::vector<double> st((size_t)n * PBRTGPU_STAT_COUNT, 0.0);
    auto worker = [&](int i) {
        pbrtgpu_ctx *c = ctxs[i];
        std::vector<int32_t> mine;
        bool first = true;
        for (int j; (j = next.fetch_add(1)) < m;) {
            std::vector<int32_t> slice;
            for (size_t k = (size_t)j; k < list.size(); k += (size_t)m) slice.push_back(list[k]);
            if (slice.empty()) continue;
            pbrtgpu_render_desc d = *desc;
            if (!first) d.flags |= PBRTGPU_F_ACCUMULATE;   // the slices of one context share its film
            double s8[PBRTGPU_STAT_COUNT] = {0};
            int e = pbrtgpu_render_tiles(c, &d, slice.data(), (int32_t)slice.size(), s8);
            if (e) { rc[i] = e; msg[i] = g_err; return; }
            for (int k = 0; k < PBRTGPU_STAT_COUNT; ++k) st[(size_t)i * PBRTGPU_STAT_COUNT + k] += s8[k];
            mine.insert(mine.end(), slice.begin(), slice.end());
            first = false;
        }
        if (mine.empty()) return;
        // host gather: this context's film pixels (disjoint from every other context's)
        int e = pbrtgpu_film_gather(c, tw, th, mine.data(), (int32_t)mine.size(), film_out, n_floats);
        if (e) { rc[i] = e; msg[i] = g_err; }
    };
    std::vector<std::thread> threads;
    for (int i = 1; i < n; ++i) threads.emplace_back(worker, i);
    worker(0);
    for (auto &t : threads) t.join();
    if (stats_out) memcpy(stats_out, st.data(), st.size() * sizeof(double));
    for (int i = 0; i < n; ++i)
        if (rc[i]) return fail(rc[i], "context " + std::to_string(i) + ": " + msg[i]);
    return 0;
}

}  // extern "C"

template <int NB>
static int trace_impl(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, float *out, bool countWork) {
    const pbrtgpu_camera &cam = c->cam;
    for (int32_t i = 0; i < n; ++i) {
        const int32_t *k = keys + 3 * i;
        if (k[0] < cam.sx_start || k[0] >= cam.sx_end || k[1] < cam.sy_start || k[1] >= cam.sy_end || k[2] < 0 ||
            k[2] >= c->spp)
            return fail(PBRTGPU_E_INVALID, "path key outside the sample extent / sample range");
    }
    HIPCHK(c->scratch[0].ensure((size_t)n * sizeof(int3)));
    HIPCHK(c->scratch[1].ensure((size_t)n * NB * 4));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, keys, (size_t)n * 12, hipMemcpyHostToDevice, c->stream));
    if ((uint64_t)n * (uint64_t)c->S.specItems > 0x7fffffffull) return fail(PBRTGPU_E_INVALID, "too many keys");
    ItemSrc ks{};
    ks.keys = (const int3 *)c->scratch[0].p;
    ks.nItems = (uint32_t)n * (uint32_t)c->S.specItems;
    Timing T;
    if (int e = run_wavefront<NB>(c, ks, (float *)c->scratch[1].p, countWork, T, nullptr)) return e;
    c->last = T;
    if (out) HIPCHK(hipMemcpyAsync(out, c->scratch[1].p, (size_t)n * NB * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" {

int pbrtgpu_trace_paths(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, float *out) {
    if (!c || !c->hasScene || !keys || !out || n < 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    switch (c->nb) {
        case 32: return trace_impl<32>(c, keys, n, out, false);
        case 60: return trace_impl<60>(c, keys, n, out, false);
        case 3: return trace_impl<3>(c, keys, n, out, false);
        case 30: return trace_impl<30>(c, keys, n, out, false);
    }
    return fail(PBRTGPU_E_UNSUPPORTED, "band count");
}

int pbrtgpu_path_stats(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, uint64_t *counters_out) {
    if (!c || !c->hasScene || !keys || !counters_out || n <= 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    HIPCHK(hipSetDevice(c->device));
    int e = PBRTGPU_E_UNSUPPORTED;
    switch (c->nb) {
        case 32: e = trace_impl<32>(c, keys, n, nullptr, true); break;
        case 60: e = trace_impl<60>(c, keys, n, nullptr, true); break;
        case 3: e = trace_impl<3>(c, keys, n, nullptr, true); break;
        case 30: e = trace_impl<30>(c, keys, n, nullptr, true); break;
    }
    if (e) return e;
    const uint64_t *w = c->last.work;
    counters_out[0] = w[W_RAYS]; counters_out[1] = w[W_SHADOW]; counters_out[2] = w[W_NODES_C] + w[W_NODES_S];
    counters_out[3] = w[W_TRIS_C] + w[W_TRIS_S]; counters_out[4] = w[W_QUADS_C] + w[W_QUADS_S]; counters_out[5] = w[W_HITS];
    return 0;
}

int pbrtgpu_build_bvh(pbrtgpu_ctx *c, int32_t n, const float *bounds, pbrtgpu_bvh_node *nodes_out, int32_t *order_out,
                      double *ms_out) {
    if (!c || !bounds || !nodes_out || !order_out || n < 1) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n > (1 << 24)) return fail(PBRTGPU_E_UNSUPPORTED, "BVH leaf beyond the 2^24-primitive reference range");
    HIPCHK(hipSetDevice(c->device));
    std::string err;
    const int e = lbvh_build(c->stream, n, bounds, nodes_out, order_out, ms_out, &err);
    return e ? fail(e, "pbrtgpu_build_bvh: " + err) : 2 * n - 1;
}

int pbrtgpu_loop_subdivide(pbrtgpu_ctx *c, int32_t nf, int32_t nv, const int32_t *vi, const float *P, int32_t levels,
                           int32_t *nv_out, float *P_out, float *N_out, int32_t *vi_out, double *ms_out) {
    if (!c || nf < 1 || nv < 1 || !vi || !P || !nv_out || levels < 0 || levels > 12 || (P_out && (!N_out || !vi_out)))
        return fail(PBRTGPU_E_INVALID, "bad arguments");
    HIPCHK(hipSetDevice(c->device));
    std::string err;
    const int e = loop_subdivide(c->stream, nf, nv, vi, P, levels, nv_out, P_out, N_out, vi_out, ms_out, &err);
    return e ? fail(e < -1 ? e : PBRTGPU_E_INVALID, "pbrtgpu_loop_subdivide: " + err) : 0;
}

int pbrtgpu_loop_subdivide_hook(void *ctx, int32_t nf, int32_t nv, const int32_t *vi, const float *P, int32_t levels,
                                int32_t *nv_out, float *P_out, float *N_out, int32_t *vi_out) {
    return pbrtgpu_loop_subdivide((pbrtgpu_ctx *)ctx, nf, nv, vi, P, levels, nv_out, P_out, N_out, vi_out, nullptr);
}

int pbrtgpu_mt_sequence(pbrtgpu_ctx *c, uint32_t seed, int32_t n, uint32_t *out) {
    if (!c || !out || n < 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->scratch[0].ensure((size_t)n * 4 + 624 * 4));
    uint32_t *d = (uint32_t *)c->scratch[0].p;
    hipLaunchKernelGGL(k_mt_sequence, dim3(1), dim3(64), 0, c->stream, seed, n, d, d + n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, d, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int pbrtgpu_libmf_eval(pbrtgpu_ctx *c, int32_t fn, int64_t n, const float *x, const float *y, float *out) {
    const bool two = fn == PBRTGPU_LIBMF_POWF || fn == PBRTGPU_LIBMF_ATAN2F;
    if (!c || !x || !out || n < 0 || fn < 0 || fn >= PBRTGPU_LIBMF_COUNT || (two && !y) || n > ((int64_t)1 << 30))
        return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    const size_t no = (size_t)n * (fn == PBRTGPU_LIBMF_SINCOSF ? 2 : 1);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->scratch[0].ensure((size_t)n * 4));
    HIPCHK(c->scratch[1].ensure((size_t)n * 4));
    HIPCHK(c->scratch[2].ensure(no * 4));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, x, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    if (two) HIPCHK(hipMemcpyAsync(c->scratch[1].p, y, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_libmf_eval, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, fn, n,
                       (const float *)c->scratch[0].p, (const float *)c->scratch[1].p, (float *)c->scratch[2].p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->scratch[2].p, no * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int pbrtgpu_intersect(pbrtgpu_ctx *c, const float *rays, int32_t n, float *hits, int32_t *occ) {
    if (!c || !c->hasScene || !rays || !hits || n < 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->scratch[0].ensure((size_t)n * 32));
    HIPCHK(c->scratch[1].ensure((size_t)n * 16));
    HIPCHK(c->scratch[2].ensure((size_t)n * 4));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, rays, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    size_t lds = 2 * (size_t)std::max(c->stackDepth, c->S.w4Stack + 1) * kTraceBlock * 4;
    hipLaunchKernelGGL(k_intersect, dim3((n + kTraceBlock - 1) / kTraceBlock), dim3(kTraceBlock), lds, c->stream, c->S,
                       (const float *)c->scratch[0].p, n, (float *)c->scratch[1].p, (int *)c->scratch[2].p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(hits, c->scratch[1].p, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    std::vector<int> o(n);
    HIPCHK(hipMemcpyAsync(o.data(), c->scratch[2].p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (occ) memcpy(occ, o.data(), (size_t)n * 4);
    return 0;
}

int pbrtgpu_last_timing(pbrtgpu_ctx *c, pbrtgpu_timing *out) {
    if (!c || !out) return fail(PBRTGPU_E_INVALID, "null argument");
    memset(out, 0, sizeof(*out));
    for (int k = 0; k < K_KINDS; ++k) { out->ms[k] = c->last.ms[k]; out->launches[k] = c->last.launches[k]; }
    out->passes = c->last.passes;
    out->shade_feat = c->feat;
    for (int i = 0; i < W_COUNT; ++i) out->work[i] = c->last.work[i];
    return 0;
}

}  // extern "C"
