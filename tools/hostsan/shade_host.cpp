// shade_host.cpp -- TEST INFRASTRUCTURE (never part of the product): the GPU wavefront's device
// code replayed on the CPU, so that it can run under the host sanitizers.
//
// The device shading steps (csrc/wavefront.h shade_slot / path_start, directlighting.h
// shade_slot_dl / dl_light_batches, metadata.h shade_slot_meta), the ray queries
// (device.h bvh_intersect / bvh_intersectP: the legacy one-ray walk, same primitives in the same
// order as the persistent kernels) and the DevScene layout (csrc/scene_build.h) are compiled as
// host C++ against tools/hostsan/hip/hip_runtime.h and driven pass by pass the way
// pbrtgpu.hip run_wavefront drives them: regeneration, closest-hit and shadow queries of the
// queued rays, one shading step per live slot (+ k_dl_nee's light batches for DirectLighting).
//   * Every path-slot array is its own heap block (ASan redzones per array) and is left as
//     malloc returns it (MSan tracks it as uninitialised) or filled with --poison BYTE, as the
//     GPU leaves hipMalloc memory unwritten: a read of state no pass wrote shows up as an MSan
//     report or as a radiance that changes with the poison byte.
//   * Each slot is lane 0 of its own 64-slot wave (slot = 64 i): the wave intrinsics of the
//     stand-in header then see one active lane.
//
// usage: shade_host SCENE [--xres N] [--yres N] [--spp N] [--maxdepth N] [--bands N]
//                         [--integrator path|directlighting|metadata] [--strategy all|one|mesh|material|depth]
//                         [--slots N] [--poison BYTE] [--keys FILE] --out FILE
//        shade_host SEED --mt-kat N --out FILE     (the device RNG's first N outputs, uint32)
// Items: every (x, y, s) of the camera's sample extent in row-major order, or the int32
// (x, y, s) triples of --keys.  Writes float32 [items][bands] radiance to --out.
#include <hip/hip_runtime.h>   // the stand-in of tools/hostsan/hip
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>
#include "pbrthost.h"
#include "scene_build.h"
#include "directlighting.h"
#include "metadata.h"

#if defined(__has_feature)
#if __has_feature(memory_sanitizer)
#include <sanitizer/msan_interface.h>
#define HS_MSAN 1
#endif
#endif
#ifndef HS_MSAN
#define HS_MSAN 0
#endif

namespace pgd {
float4 pgd_kd_lds[2 * kKdLdsNodes];   // k_shade's dynamic LDS (the measured-BRDF kd-trees)
}
using namespace pgd;

static std::vector<void *> g_blocks;
static int g_poison = -1;   // -1: leave heap blocks as allocated
static uint32_t g_maxDraws = 0;

static void *halloc(size_t bytes, bool poison) {
    const size_t n = std::max<size_t>(64, (bytes + 63) & ~(size_t)63);
    void *p = aligned_alloc(64, n);
    if (!p) { fprintf(stderr, "out of memory\n"); exit(2); }
    if (poison && g_poison >= 0) memset(p, g_poison, n);
    g_blocks.push_back(p);
    return p;
}
template <class T> static T *arr(size_t n) { return static_cast<T *>(halloc(n * sizeof(T), true)); }

#if HS_MSAN
// the flattened scene comes from libpbrthost (not instrumented): its arrays are initialised
static void unpoison_flat(const pbrtgpu_flat_scene *s) {
    auto u = [](const void *p, size_t b) { if (p && b) __msan_unpoison(p, b); };
    u(s, sizeof(*s));
    u(s->band_Y, 4 * (size_t)s->n_bands);
    u(s->nodes, sizeof(*s->nodes) * (size_t)s->n_nodes);
    u(s->prims, sizeof(*s->prims) * (size_t)s->n_prims);
    u(s->tris, sizeof(*s->tris) * (size_t)s->n_tris);
    u(s->meshes, sizeof(*s->meshes) * (size_t)s->n_meshes);
    u(s->vert_p, 12 * (size_t)s->n_verts);
    u(s->vert_n, 12 * (size_t)s->n_verts);
    u(s->vert_uv, 8 * (size_t)s->n_verts);
    u(s->quadrics, sizeof(*s->quadrics) * (size_t)s->n_quadrics);
    u(s->materials, sizeof(*s->materials) * (size_t)s->n_materials);
    u(s->lights, sizeof(*s->lights) * (size_t)s->n_lights);
    u(s->light_shapes, sizeof(*s->light_shapes) * (size_t)s->n_light_shapes);
    u(s->spectra, 4 * (size_t)s->n_spectra_floats);
    u(s->instances, sizeof(*s->instances) * (size_t)std::max(0, s->n_instances));
    u(s->camera_motion, sizeof(*s->camera_motion));
    if (s->n_instances > 0) u(s->prim_instance, 4 * (size_t)s->n_prims);
    u(s->kdnodes, sizeof(*s->kdnodes) * (size_t)std::max(0, s->n_kdnodes));
    u(s->textures, sizeof(*s->textures) * (size_t)std::max(0, s->n_textures));
    u(s->texels, 4 * (size_t)std::max(0, s->n_texel_floats));
    u(s->ewa_lut, 4 * 128);
    u(s->rgb_basis, 4 * 14 * (size_t)s->n_bands);
    u(s->merl, 4 * (size_t)std::max(0, s->n_merl_floats));
    u(s->prim_meta, 8 * (size_t)s->n_prims);
    u(s->lens.elements, 16 * (size_t)std::max(0, s->lens.n_elements));
    if (s->lens.num_pinholes_w > 0 && s->lens.num_pinholes_h > 0)
        u(s->lens.pinholes, 12 * (size_t)s->lens.num_pinholes_w * (size_t)s->lens.num_pinholes_h);
    if (s->lens.ior_eye) u(s->lens.eye_ior, 16 * (size_t)s->n_bands);
}
#endif

// PathSoA as pbrtgpu.hip ensure_slots lays it out, one heap block per array
static PathSoA make_soa(int cap, int NB, int nInst, int nFrames, int batch, bool mtExt) {
    const size_t C = (size_t)cap, R = C * (size_t)batch, AB = (size_t)std::max(2, batch), W = (C + 63) / 64;
    const size_t NQ = (size_t)(NB + 3) / 4, F = (size_t)nFrames;
    PathSoA P{};
    P.cap = cap;
    P.rcap = (int)R;
    P.dlBatch = batch;
    P.item = arr<int>(C); P.hp = arr<uint32_t>(C); P.smp = arr<uint32_t>(C); P.bounce = arr<int>(C);
    P.flags = arr<uint32_t>(C); P.mt = arr<uint32_t>(5 * C); P.pix = arr<uint32_t>(C);
    P.beta = arr<float4>(3 * NQ * C); P.L = arr<float4>(NQ * C);
    P.A = arr<float4>(AB * NQ * C); P.B = arr<float4>(AB * NQ * C);
    P.M = arr<float4>(NQ * C); P.K = arr<float4>(2 * NQ * C);
    P.aMask = arr<unsigned long long>(2 * W); P.bMask = arr<unsigned long long>(3 * W);
    P.mMask = arr<unsigned long long>(2 * W);
    P.ray = arr<float>(4 * 9 * R); P.hitPrim = arr<int>(2 * R); P.hitT = arr<float>(2 * R); P.occ = arr<uint32_t>(R);
    P.qC = arr<uint32_t>(2 * 2 * R); P.qS = arr<uint32_t>(2 * R);
    P.cnt = arr<uint32_t>(CNT_WORDS);
    memset(P.cnt, 0, CNT_WORDS * 4);
    P.nInst = nInst;
    P.instM = nInst ? arr<float4>(C * (size_t)nInst * 8) : nullptr;
    P.mtExt = mtExt ? arr<uint32_t>(C * 624) : nullptr;
    P.nFrames = nFrames;
    if (nFrames) {
        P.dlMask = arr<uint32_t>(C);
        P.dlList = arr<uint32_t>(C); P.dlRow = arr<uint32_t>(C);
        P.fL = arr<float4>(F * NQ * C); P.fF = arr<float4>(F * NQ * C);
        P.fRay = arr<float>(F * 9 * C); P.fDiff = arr<float>(F * 12 * C); P.fS = arr<float>(F * 2 * C);
        P.fHit = arr<int>(F * 2 * C); P.fBr = arr<uint32_t>(F * C); P.dlk = arr<uint32_t>(C);
    }
    for (size_t i = 0; i < C; ++i) P.item[i] = -1;   // run_wavefront: hipMemset(item, 0xff) and the masks' 0
    memset(P.aMask, 0, 2 * W * 8);
    memset(P.bMask, 0, 3 * W * 8);
    memset(P.mMask, 0, 2 * W * 8);
    return P;
}

struct Queues { std::vector<uint32_t> c, s; };

template <int NB, int FEAT, int MODE>
static int run(const DevScene &S, PathSoA &P, const ItemSrc &src, int nSlots, float *Lout, std::string *err) {
    enum { MODE_PATH = 0, MODE_DL = 1, MODE_META = 2 };
    const int cap = P.cap;
    uint32_t next = 0, finished = 0;
    Queues Q[2];
    std::vector<uint32_t> stk((size_t)std::max(S.stackDepth, S.w4Stack) + 1);
    std::vector<float> stkT((size_t)std::max(S.stackDepth, S.w4Stack) + 1);
    const int64_t pathPasses = MODE == MODE_DL ? (P.nFrames >= 40 ? ((int64_t)1 << 60) : (((int64_t)1 << P.nFrames) - 1) * (S.dlK + 1) + 2)
                                               : S.maxDepth + 3;
    const int64_t maxPasses = 2 * ((src.nItems + nSlots - 1) / nSlots + 1) * pathPasses + 8;
    // rb: the base of a DirectLighting batch's ray slots (k_dl_nee: its list row without instances)
    auto push = [&](int q, const Pushes &pu, int slot, int rb = -1) {
        if (pu.c) Q[q].c.push_back((uint32_t)slot << 1);
        if (MODE == MODE_DL) {
            if (rb < 0) rb = slot;
            for (uint32_t m = pu.mMask; m; m &= m - 1u) Q[q].c.push_back(((uint32_t)(rb + (__builtin_ctz(m)) * cap) << 1) | 1u);
            for (uint32_t m = pu.sMask; m; m &= m - 1u) Q[q].s.push_back((uint32_t)(rb + (__builtin_ctz(m)) * cap));
        } else {
            if (pu.m) Q[q].c.push_back(((uint32_t)(MODE == MODE_PATH ? pu.mIdx : slot) << 1) | 1u);
            if (pu.s) Q[q].s.push_back((uint32_t)(MODE == MODE_PATH ? pu.sIdx : slot));
        }
        if (MODE == MODE_PATH && pu.t) mt_window_init(P, (uint32_t)slot);   // k_mt_init (after the pass on the GPU)
    };
    // MT19937 outputs a finished path drew (the most of any path is reported: > 227 exercises mt_uint_ext)
    auto note_draws = [&](int slot) {
        if (P.flags[slot] & PF_MTINIT) g_maxDraws = std::max(g_maxDraws, P.mt[slot]);
    };
    // one k_shade pass (+ k_dl_nee): the per-thread body of shade.hip k_shade for every slot
    auto shade = [&](int qout) {
        Q[qout].c.clear();
        Q[qout].s.clear();
        P.cnt[CNT_DLN] = 0;
        for (int i = 0; i < nSlots; ++i) {
            const int slot = 64 * i;
            threadIdx.x = (unsigned)(slot & 63);
            Pushes pu = {false, false, false, 0u, 0u};
            bool freeSlot = P.item[slot] < 0, zeroed = false;
            if (!freeSlot) {
                bool done;
                if (P.bounce[slot] == -2) {
                    float4 Z[Bands<NB>::NQ];
                    for (int q = 0; q < Bands<NB>::NQ; ++q) Z[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                    (void)path_output<NB>(S, Z, Lout, P.item[slot], P.smp[slot]);
                    done = true;
                } else if (MODE == MODE_DL) pu = shade_slot_dl<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
                else if (MODE == MODE_META) pu = shade_slot_meta<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
                else pu = shade_slot<NB, FEAT>(S, P, slot, Lout, &done, &zeroed, qout);
                if (done) { P.item[slot] = -1; freeSlot = true; ++finished; note_draws(slot); }
            }
            push(qout, pu, slot);
            if (MODE == MODE_DL && pu.t) P.dlList[P.cnt[CNT_DLN]++] = (uint32_t)slot;   // the light-sample list
            if (freeSlot && next < src.nItems) {
                path_start<NB>(S, P, src, slot, next++);
                Q[qout].c.push_back((uint32_t)slot << 1);
            }
        }
        if (MODE == MODE_DL) {
            for (uint32_t i = 0; i < P.cnt[CNT_DLN]; ++i) {   // k_dl_nee: entry i of the list, row i
                const int slot = (int)P.dlList[i];
                threadIdx.x = (unsigned)(i & 63);
                Pushes pu = {false, false, false, 0u, 0u};
                if (P.item[slot] >= 0 && (P.flags[slot] & PF_DLNEE)) dl_light_batches<NB, FEAT>(S, P, slot, (int)i, pu);
                push(qout, pu, slot, P.nInst ? slot : (int)i);
            }
            for (int i = 0; i < nSlots; ++i) {   // k_dl_spec
                const int slot = 64 * i;
                threadIdx.x = (unsigned)(slot & 63);
                Pushes pu = {false, false, false, 0u, 0u};
                bool done = false, zeroed = false;
                if (P.item[slot] >= 0 && (P.flags[slot] & PF_DLSPEC)) {
                    pu = dl_spec_step<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
                    if (done) { P.item[slot] = -1; ++finished; note_draws(slot); }
                }
                push(qout, pu, slot);
            }
            for (int i = 0; i < nSlots; ++i) {   // k_regen
                const int slot = 64 * i;
                if (P.item[slot] < 0 && next < src.nItems) {
                    path_start<NB>(S, P, src, slot, next++);
                    Q[qout].c.push_back((uint32_t)slot << 1);
                }
            }
        }
    };
    // the ray queries of queue set q (k_trace_pt / k_trace_inst: hit or miss, t = inf on a miss)
    auto trace = [&](int q) {
        Stack st;
        st.base = stk.data();
        st.tbase = stkT.data();
        st.stride = 1;
        for (uint32_t e : Q[q].c) {
            const int rs = (int)(e >> 1), kind = (int)(e & 1u);
            Ray r = ray_load(P, rec_kind(S, q, kind), rs);
            int prim = -1;
            float t = INFINITY;
            const char *c4e = getenv("PBRTGPU_CLOSEST4");
            const bool c4 = S.nInsts == 0 && S.w4N > 0 && !(c4e && atoi(c4e) == 0);
            const bool hit = c4 ? bvh_intersect4(S, st, r, &prim, &t)
                           : S.nInsts > 0 ? bvh_intersect<true>(S, st, r, &prim, &t) : bvh_intersect<false>(S, st, r, &prim, &t);
            if (!hit) prim = -1;
            P.hitPrim[(size_t)kind * P.rcap + rs] = prim;
            P.hitT[(size_t)kind * P.rcap + rs] = prim >= 0 ? t : INFINITY;
        }
        // shadow queries: on the 4-wide copy where the GPU uses it (k_trace_s4; PBRTGPU_SHADOW4=0:
        // the binary walk), so the replay checks its boxes and leaves against the oracle too
        const char *s4e = getenv("PBRTGPU_SHADOW4"), *s4qe = getenv("PBRTGPU_SHADOW4Q");
        const bool s4 = S.nInsts == 0 && S.w4N > 0 && !(s4e && atoi(s4e) == 0);
        const bool s4q = s4 && S.w4q && !(s4qe && atoi(s4qe) == 0);   // k_trace_s4q's quantized copy
        for (uint32_t rs : Q[q].s) {
            const Ray r = ray_load(P, RAY_S, (int)rs);
            P.occ[rs] = (s4q ? bvh_intersectP4q(S, st, r) : s4 ? bvh_intersectP4(S, st, r)
                            : S.nInsts > 0 ? bvh_intersectP<true>(S, st, r) : bvh_intersectP<false>(S, st, r)) ? 1u : 0u;
        }
    };
    P.pass = 0;
    shade(0);
    int q = 0;
    for (int64_t pass = 0;; ++pass) {
        if (pass > maxPasses) { *err = "wavefront did not drain"; return 3; }
        if (P.cnt[CNT_ERR]) { *err = "a path drew past 227 MT19937 outputs without its state row"; return 3; }
        trace(q);
        const int nq = q ^ 1;
        P.pass = (P.pass + 1) % 3;
        // the drain's list mode (pbrtgpu.hip run_wavefront: once the items are all taken): the
        // identity compaction and per-lane mask loads of PathSoA::listMode, mixed with the passes
        // before it; the slot order is the list's (slot order)
        P.listMode = (MODE == MODE_PATH && next >= src.nItems && !getenv("PBRTGPU_DRAIN_LIST_OFF")) ? 1 : 0;
        shade(nq);
        q = nq;
        if (Q[q].c.empty() && Q[q].s.empty()) break;
    }
    if (finished != src.nItems || next != src.nItems) {
        *err = "items left unfinished: " + std::to_string(src.nItems - finished);
        return 3;
    }
    return 0;
}

template <int NB>
static int run_nb(const DevScene &S, PathSoA &P, const ItemSrc &src, int nSlots, int feat, float *Lout, std::string *err) {
    // the variant pbrtgpu.hip launches: FEAT_ALL when the scene uses a feature, else FEAT 0
    if (S.integrator == PBRTGPU_INTEGRATOR_DIRECT)
        return (feat & FEAT_ALL) ? run<NB, FEAT_ALL, 1>(S, P, src, nSlots, Lout, err) : run<NB, 0, 1>(S, P, src, nSlots, Lout, err);
    if (S.integrator == PBRTGPU_INTEGRATOR_METADATA)
        return (feat & FEAT_ALL) ? run<NB, FEAT_ALL, 2>(S, P, src, nSlots, Lout, err) : run<NB, 0, 2>(S, P, src, nSlots, Lout, err);
    return (feat & FEAT_ALL) ? run<NB, FEAT_ALL, 0>(S, P, src, nSlots, Lout, err) : run<NB, 0, 0>(S, P, src, nSlots, Lout, err);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s SCENE [--xres N] [--yres N] [--spp N] [--maxdepth N] [--bands N] [--integrator I] "
                        "[--strategy S] [--renderer R --wave_bands N --sampling M] [--slots N] [--poison BYTE] [--keys FILE] "
                        "--out FILE\n", argv[0]);
        return 2;
    }
    if (!strcmp(argv[1], "--m4inv-check")) {   // m4_inverse_scale (its diagonal fast path) against
        // the general Gauss-Jordan m4_inverse (transform.cpp:68-130): random diagonal scale factors,
        // identities, ties, and general / degenerate matrices (those take the general routine)
        uint64_t bad = 0, fast = 0;
        uint32_t x = 12345u;
        auto rnd = [&]() { x ^= x << 13; x ^= x >> 17; x ^= x << 5; return x; };
        auto chk = [&](const float *m) {
            float a[16], b[16];
            m4_inverse(m, a);
            m4_inverse_scale(m, b);
            bool d = true;
            for (int i = 0; i < 16; ++i) d = d && (i % 5 == 0 ? (m[i] >= 0x1p-100f && m[i] <= 0x1p100f) : __float_as_uint(m[i]) == 0u);
            fast += d;
            if (memcmp(a, b, sizeof(a))) ++bad;
        };
        const float pool[] = {1.f, 2.f, .5f, 3.f, 1e-3f, 7.25f, 1e30f, 0x1p-100f, 0x1p100f, 1.0000001f, 0.9999999f};
        for (int it = 0; it < 2000000; ++it) {
            float m[16];
            for (int i = 0; i < 16; ++i) m[i] = 0.f;
            for (int i = 0; i < 4; ++i)
                m[5 * i] = (rnd() & 3) ? __uint_as_float(0x3c000000u + rnd() % 0x0a000000u) : pool[rnd() % 11];
            if ((it & 7) == 0) m[5 * (rnd() & 3)] = m[5 * (rnd() & 3)];   // ties
            if ((it & 15) == 1) m[rnd() & 15] = -m[rnd() & 15];           // negative / -0 entries
            if ((it & 31) == 2) m[1 + 5 * (rnd() % 3)] = __uint_as_float(rnd() & 0x3fffffffu);   // off-diagonal
            chk(m);
        }
        printf("mismatches %llu fast %llu\n", (unsigned long long)bad, (unsigned long long)fast);
        return bad || fast < 1000000 ? 1 : 0;
    }
    if (!strcmp(argv[1], "--kd-radius-check")) {   // kd_radius_of (the device source) against the
        // reference retry loop's radius (measured.cpp, IrregIsotropicBRDF::f) over every non-negative float
        uint64_t bad = 0;
        for (uint64_t i = 0; i < 0x80000000ull; ++i) {
            const float d3 = __uint_as_float((uint32_t)i);
            float m = .001f;
            for (int k = 0; k < 11 && !(d3 < m); ++k) m *= 2.f;
            const float r = kd_radius_of(d3);
            if (__float_as_uint(r) != __float_as_uint(m)) ++bad;
        }
        printf("mismatches %llu\n", (unsigned long long)bad);
        return bad ? 1 : 0;
    }
    pbrthost_overrides ov = {PBRTHOST_ABI_VERSION, -1, -1, -1, -1, 0, PBRTHOST_KEEP_SEED, -1, -1, -1, -1, -1, -1};
    int nSlots = 256, mtKat = 0;
    const char *out = nullptr, *keyFile = nullptr, *strategy = nullptr;
    for (int i = 2; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        const char *v = argv[i + 1];
        if (a == "--xres") ov.xres = atoi(v);
        else if (a == "--yres") ov.yres = atoi(v);
        else if (a == "--spp") ov.spp = atoi(v);
        else if (a == "--maxdepth") ov.maxdepth = atoi(v);
        else if (a == "--bands") ov.bands = atoi(v);
        else if (a == "--slots") nSlots = std::max(1, atoi(v));
        else if (a == "--poison") g_poison = (int)strtol(v, nullptr, 0) & 0xff;
        else if (a == "--out") out = v;
        else if (a == "--keys") keyFile = v;
        else if (a == "--strategy") strategy = v;
        else if (a == "--mt-kat") mtKat = atoi(v);
        else if (a == "--renderer") ov.renderer = !strcmp(v, "spectral") ? PBRTGPU_RENDERER_SPECTRAL : PBRTGPU_RENDERER_SAMPLER;
        else if (a == "--wave_bands") ov.wave_bands = atoi(v);
        else if (a == "--sampling") ov.spectral_sampling = !strcmp(v, "sampler") ? PBRTGPU_SPECTRAL_SAMPLER : PBRTGPU_SPECTRAL_SINGLE;
        else if (a == "--integrator")
            ov.integrator = !strcmp(v, "directlighting") ? PBRTGPU_INTEGRATOR_DIRECT
                            : !strcmp(v, "metadata")     ? PBRTGPU_INTEGRATOR_METADATA
                                                         : PBRTGPU_INTEGRATOR_PATH;
        else { fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    if (strategy) {
        if (!strcmp(strategy, "all")) ov.dl_strategy = PBRTGPU_DL_ALL;
        else if (!strcmp(strategy, "one")) ov.dl_strategy = PBRTGPU_DL_ONE;
        else if (!strcmp(strategy, "mesh")) ov.meta_strategy = PBRTGPU_META_MESH;
        else if (!strcmp(strategy, "material")) ov.meta_strategy = PBRTGPU_META_MATERIAL;
        else if (!strcmp(strategy, "depth")) ov.meta_strategy = PBRTGPU_META_DEPTH;
    }
    if (!out) { fprintf(stderr, "--out FILE is required\n"); return 2; }
    if (mtKat) {   // the device RNG's first n outputs (mt_uint / mt_uint_ext) for seed = argv[1]
        const uint32_t seed = (uint32_t)strtoul(argv[1], nullptr, 0);
        std::vector<uint32_t> ext(624), seq((size_t)mtKat);
        MT r;
        mt_begin(r, seed);
        mt_init(r);
        r.ext = ext.data();
        for (int i = 0; i < mtKat; ++i) seq[(size_t)i] = mt_uint(r);
        FILE *f = fopen(out, "wb");
        if (!f || fwrite(seq.data(), 4, seq.size(), f) != seq.size()) { fprintf(stderr, "cannot write %s\n", out); return 1; }
        fclose(f);
        return 0;
    }
    char msg[512] = {0};
    pbrthost_scene *hs = nullptr;
    pbrtgpu_flat_scene fs;
#if HS_MSAN
    // libpbrthost and libz are not instrumented: no interceptor checks while they run (their
    // writes are not tracked), then their output counts as initialised
    __msan_scoped_disable_interceptor_checks();
#endif
    const int lrc = pbrthost_load(argv[1], &ov, &hs, msg, sizeof(msg));
    const int frc = lrc ? -1 : pbrthost_flat(hs, &fs);
#if HS_MSAN
    __msan_scoped_enable_interceptor_checks();
    __msan_unpoison(msg, sizeof(msg));
#endif
    if (lrc) { fprintf(stderr, "load: %s\n", msg); return 1; }
    if (frc) { fprintf(stderr, "flat scene failed\n"); return 1; }
#if HS_MSAN
    unpoison_flat(&fs);
#endif
    std::string err;
    if (int e = scene_check(&fs, &err)) { fprintf(stderr, "scene: %s (%d)\n", err.c_str(), e); return 1; }
    DevScene S{};
    int feat = 0;
    auto put = [&](auto *src, size_t count, auto **dst) -> int {
        using T = std::remove_const_t<std::remove_pointer_t<decltype(src)>>;
        T *p = static_cast<T *>(halloc(std::max<size_t>(count, 1) * sizeof(T), false));
        if (count) memcpy(p, src, count * sizeof(T));
        *dst = p;
        return 0;
    };
    if (int e = scene_build(&fs, 0, S, &feat, put, &err)) { fprintf(stderr, "scene: %s (%d)\n", err.c_str(), e); return 1; }
    if (S.kdInLds) memcpy(pgd_kd_lds, S.kdPack, (size_t)S.nKd * 32);
    // items
    std::vector<int3> keys;
    if (keyFile) {
        FILE *f = fopen(keyFile, "rb");
        if (!f) { fprintf(stderr, "cannot open %s\n", keyFile); return 1; }
        int3 k;
        while (fread(&k, 12, 1, f) == 1) keys.push_back(k);
        fclose(f);
    } else {
        const pbrtgpu_camera &c = fs.camera;
        for (int y = c.sy_start; y < c.sy_end; ++y)
            for (int x = c.sx_start; x < c.sx_end; ++x)
                for (int s = 0; s < fs.spp; ++s) keys.push_back(make_int3(x, y, s));
    }
    const uint32_t nItems = (uint32_t)keys.size() * (uint32_t)S.specItems;
    ItemSrc src{};
    src.pix = nullptr;
    src.sb = 1;
    src.s0 = 0;
    src.keys = keys.data();
    src.keyBase = 0;
    src.nItems = nItems;
    src.base = 0;
    const bool dl = S.integrator == PBRTGPU_INTEGRATOR_DIRECT;
    const int nFrames = dl ? std::max(1, S.maxDepth) : 0;
    const int batch = dl ? std::max(1, std::min(S.dlStrategy == PBRTGPU_DL_ONE ? 1 : S.dlK, 8)) : 1;
    const bool mtExt = dl ? S.maxDepth > 6 : S.maxDepth > 20;   // as pbrtgpu.hip run_wavefront
    PathSoA P = make_soa(64 * nSlots, S.nb, S.nInsts, nFrames, batch, mtExt);
    const size_t rows = S.specMode == 1 ? keys.size() : nItems;
    std::vector<float> Lout(rows * (size_t)S.nb, NAN);
    int rc;
    switch (S.nb) {
        case 32: rc = run_nb<32>(S, P, src, nSlots, feat, Lout.data(), &err); break;
        case 60: rc = run_nb<60>(S, P, src, nSlots, feat, Lout.data(), &err); break;
        case 30: rc = run_nb<30>(S, P, src, nSlots, feat, Lout.data(), &err); break;
        case 3: rc = run_nb<3>(S, P, src, nSlots, feat, Lout.data(), &err); break;
        default: err = "band count"; rc = 2;
    }
    if (rc) { fprintf(stderr, "replay: %s\n", err.c_str()); return rc; }
    FILE *f = fopen(out, "wb");
    if (!f || fwrite(Lout.data(), 4, Lout.size(), f) != Lout.size()) { fprintf(stderr, "cannot write %s\n", out); return 1; }
    fclose(f);
    printf("shade_host: %u items, %d bands, integrator %d, %d slots, poison %d, most MT draws of a path %u\n", nItems,
           S.nb, S.integrator, nSlots, g_poison, g_maxDraws);
    for (void *p : g_blocks) free(p);
    pbrthost_free(hs);
    return 0;
}
