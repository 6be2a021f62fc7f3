// scene_build.h -- host side of pbrtgpu_scene_upload (include/pbrtgpu.h): validation of the
// flattened scene and the layout of every DevScene array (the child-in-parent BVH copy, triangles
// pre-gathered per primitive, the spectrum pool in whole band quads, the packed kd-trees, the
// SpectralRenderer band table).  `put(src, count, &dst)` places one array where the shading code
// will read it: pbrtgpu.hip copies it to HBM; the host replay of the shading step
// (tools/hostsan/shade_host.cpp, test infrastructure) keeps it in host memory.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>
#include "pbrtgpu.h"
#include "wavefront.h"

namespace pgd {

#define SB_FAIL(code, msg)             \
    do {                               \
        if (err) *err = (msg);         \
        return (code);                 \
    } while (0)
// every array is < 4 GiB: the device addresses them through 32-bit byte offsets (device.h sa)
#define SB_PUT(src, n, dst)                                                                          \
    do {                                                                                             \
        if ((size_t)(n) * sizeof(*(src)) >= ((size_t)1 << 32)) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "scene array >= 4 GiB"); \
        if (int e_ = put((src), (size_t)(n), (dst))) return e_;                                      \
    } while (0)

// Child-in-parent copy of the flattened BVH (LinearBVHNode, bvh.cpp:105-115) for
// bvh_walk: wide node k of interior node i = {left box lo, ref(left)} {left box hi,
// ref(right)} {right box lo, axis} {right box hi, 0}, with left = i + 1 and right =
// secondChildOffset as in the reference's depth-first layout.  ref[] maps every node to its
// reference (wide index or WREF_LEAF record); the roots of the top-level and instance BVHs
// are looked up there.
static inline float sb_bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
// Wide indices: the first `top` interior nodes of the top-level BVH in breadth-first order
// (the top levels, which k_trace_pt keeps in LDS), then every other interior node in the
// reference's depth-first order.  Indices only name nodes: the traversal order is the same.
static inline int wide_bvh(const pbrtgpu_flat_scene *s, int top, std::vector<float4> *wn, std::vector<uint32_t> *ref,
                    int *nTopOut, std::string *err) {
    const int n = s->n_nodes;
    ref->assign(n, 0xffffffffu);
    uint32_t nw = 0;
    if (top > 0 && n > 0 && !(s->nodes[0].meta & 0xff)) {
        std::vector<int> bfs(1, 0);
        for (size_t h = 0; h < bfs.size() && (int)nw < top; ++h) {
            const int i = bfs[h];
            const pbrtgpu_bvh_node &b = s->nodes[i];
            if (b.meta & 0xff) continue;
            (*ref)[i] = nw++;
            if (i + 1 < n) bfs.push_back(i + 1);
            if (b.offset < (uint32_t)n) bfs.push_back((int)b.offset);
        }
    }
    *nTopOut = (int)nw;
    for (int i = 0; i < n; ++i) {
        const pbrtgpu_bvh_node &b = s->nodes[i];
        const uint32_t np = b.meta & 0xff;
        if (np == 0) { if ((*ref)[i] == 0xffffffffu) (*ref)[i] = nw++; }
        else {
            if (np > WREF_NP_MASK || b.offset > WREF_OFF_MASK)
                SB_FAIL(PBRTGPU_E_UNSUPPORTED, "BVH leaf beyond the 2^24-primitive reference range");
            (*ref)[i] = WREF_LEAF | (np << WREF_NP_SHIFT) | b.offset;
        }
    }
    if (nw >= WREF_LEAF) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "BVH too large");
    wn->assign((size_t)nw * 4, make_float4(0.f, 0.f, 0.f, 0.f));
    for (int i = 0; i < n; ++i) {
        const pbrtgpu_bvh_node &b = s->nodes[i];
        if (b.meta & 0xff) continue;
        const uint32_t L = (uint32_t)i + 1, R = b.offset;
        if (L >= (uint32_t)n || R >= (uint32_t)n) SB_FAIL(PBRTGPU_E_INVALID, "BVH child out of range");
        const pbrtgpu_bvh_node &l = s->nodes[L], &r = s->nodes[R];
        float4 *w = wn->data() + (size_t)(*ref)[i] * 4;
        w[0] = make_float4(l.bmin[0], l.bmin[1], l.bmin[2], sb_bits_f((*ref)[L]));
        w[1] = make_float4(l.bmax[0], l.bmax[1], l.bmax[2], sb_bits_f((*ref)[R]));
        w[2] = make_float4(r.bmin[0], r.bmin[1], r.bmin[2], sb_bits_f((b.meta >> 8) & 0xff));
        w[3] = make_float4(r.bmax[0], r.bmax[1], r.bmax[2], 0.f);
        if (((b.meta >> 8) & 0xff) > 2) SB_FAIL(PBRTGPU_E_INVALID, "BVH split axis");
    }
    return 0;
}

// 4-wide copy of the top-level BVH (k_trace_s4 / k_trace_c4, BVHAccel::Intersect / IntersectP,
// bvh.cpp:380-481): the node of binary interior node i holds i's grandchildren -- slots 0, 1: the
// left child's children (or the left child itself in slot 0, when it is a leaf), slots 2, 3: the
// right child's -- as {box lo, ref} {box hi, meta} pairs, refs as in wide_bvh (interior: 4-wide
// index, leaf: WREF_LEAF record, empty slot: ~0u); slot 0's meta holds the split axes of i, its left
// and its right child (2 bits each; 3: a leaf).  Testing a grandchild's box without its parent's
// tests the same primitives, because the slab test is monotonic in the box (a box inside another
// gets slab intervals inside the other's, entered no earlier: the float subtractions and products
// are monotonic), so a grandchild that passes implies its parent passes, then or at any later,
// smaller maxt.  The closest-hit walk visits the grandchildren in the binary walk's order (near
// child first by the parent's axis, each child's near child first by its own axis) and re-checks a
// pushed entry distance against the then-current maxt, as the binary walk re-checks the far child
// it pushed: the primitives tested, and their order, are the binary walk's.  The root's own box is
// still tested first (nodes[0]).  Returns the stack bound: at most 3 pushes per level.
static inline int wide4_bvh(const pbrtgpu_flat_scene *s, const std::vector<uint32_t> &ref2, std::vector<float4> *w4,
                            int *stackOut, std::string *err) {
    w4->clear();
    *stackOut = 0;
    const int n = s->n_nodes;
    if (n <= 0 || (s->nodes[0].meta & 0xff)) return 0;   // a single-leaf BVH: no 4-wide copy
    // (binary node, its level) of the 4-wide nodes to fill; DFS by an explicit stack
    std::vector<std::pair<int, int> > todo(1, std::make_pair(0, 0));
    std::vector<uint32_t> idx(n, 0xffffffffu);
    idx[0] = 0;
    w4->resize(8);
    int maxLevel = 0;
    auto axisOf = [&](int i) -> uint32_t { return (s->nodes[i].meta & 0xff) ? 3u : ((s->nodes[i].meta >> 8) & 0xff); };
    while (!todo.empty()) {
        const int i = todo.back().first, level = todo.back().second;
        todo.pop_back();
        maxLevel = std::max(maxLevel, level);
        const pbrtgpu_bvh_node &b = s->nodes[i];
        const int kids[2] = {i + 1, (int)b.offset};
        float4 w[8];
        for (int k = 0; k < 4; ++k) {
            w[2 * k] = make_float4(0.f, 0.f, 0.f, sb_bits_f(0xffffffffu));
            w[2 * k + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        for (int k = 0; k < 2; ++k)
            if (kids[k] < 0 || kids[k] >= n) SB_FAIL(PBRTGPU_E_INVALID, "BVH child out of range");
        const uint32_t meta = axisOf(i) | (axisOf(kids[0]) << 2) | (axisOf(kids[1]) << 4);
        if (axisOf(i) > 2) SB_FAIL(PBRTGPU_E_INVALID, "BVH split axis");
        for (int k = 0; k < 2; ++k) {
            const int c = kids[k];
            int slotc[2] = {c, -1};
            if (!(s->nodes[c].meta & 0xff)) {
                slotc[0] = c + 1;
                slotc[1] = (int)s->nodes[c].offset;
                if (slotc[1] < 0 || slotc[1] >= n || slotc[0] >= n) SB_FAIL(PBRTGPU_E_INVALID, "BVH child out of range");
                if (axisOf(c) > 2) SB_FAIL(PBRTGPU_E_INVALID, "BVH split axis");
            }
            for (int m = 0; m < 2; ++m) {
                const int g = slotc[m];
                if (g < 0) continue;
                const pbrtgpu_bvh_node &gn = s->nodes[g];
                uint32_t r;
                if (gn.meta & 0xff) r = ref2[g];
                else {
                    if (w4->size() / 8 >= WREF_LEAF) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "BVH too large");
                    r = idx[g] = (uint32_t)(w4->size() / 8);
                    w4->resize(w4->size() + 8);
                    todo.push_back(std::make_pair(g, level + 1));
                }
                const int sl = 2 * k + m;
                w[2 * sl] = make_float4(gn.bmin[0], gn.bmin[1], gn.bmin[2], sb_bits_f(r));
                w[2 * sl + 1] = make_float4(gn.bmax[0], gn.bmax[1], gn.bmax[2], 0.f);
            }
        }
        w[1].w = sb_bits_f(meta);
        std::copy(w, w + 8, w4->begin() + (size_t)idx[i] * 8);
    }
    *stackOut = 3 * (maxLevel + 1) + 1;
    return 0;
}

// Quantized copy of the 4-wide BVH for the shadow queries (k_trace_s4q): 64 B per node instead of
// 128, so the tree a shadow walk reads is half as large in L2 / MALL.  Per node (4 x uint4):
//   q0 = {origin.xyz (float bits), biased exponents ex | ey << 8 | ez << 16}
//   q1, q2.xy = per slot k the bytes qlo.x qlo.y qlo.z qhi.x qhi.y qhi.z at byte 6k
//   q2.zw, q3.xy = the slots' refs (as the 4-wide node's; ~0u empty)
//   q3.z = per slot 6 "exact" bits (bit 6k + c: bound c of slot k dequantizes to the box exactly)
// A bound dequantizes as origin + float(q) * 2^e in float arithmetic (the device repeats the same
// two operations): the lower bound takes the largest q whose value is <= the box's, the upper the
// smallest whose value is >= (the outer box, containing the exact one); the inner box takes q + 1 /
// q - 1 where the bound is not exact (contained in the exact box).  A slab test is monotonic in
// the box (see wide4_bvh), so: exact pass => outer pass, and inner pass => exact pass.  The walk
// (k_trace_s4q) descends on outer passes, marking a path "certain" while every box on it passes
// its inner test; a primitive hit in a certain leaf is a hit the reference's walk reaches.  A hit
// in an uncertain leaf is confirmed by re-testing the leaf's binary ancestors' exact boxes from the
// root (leaf_reached) -- IntersectP's answer depends only on which leaves its exact box tests
// reach, and maxt does not change during a shadow query.  leafOf[first primitive] = the binary
// leaf node.  Returns 0 without building when a leaf holds more than 63 primitives or the tree
// has 2^29 nodes or more (the walk keeps a "certain" bit at bit 30 of its stack entries).
static inline int quant_w4(const pbrtgpu_flat_scene *s, const std::vector<float4> &w4, std::vector<uint4> *wq,
                           std::vector<int32_t> *leafOf, std::string *err) {
    wq->clear();
    leafOf->clear();
    const size_t nw = w4.size() / 8;
    if (nw == 0 || nw >= (1u << 29)) return 0;
    for (int i = 0; i < s->n_nodes; ++i)
        if ((s->nodes[i].meta & 0xff) > 63) return 0;
    leafOf->assign((size_t)std::max(1, s->n_prims), -1);
    for (int i = 0; i < s->n_nodes; ++i) {
        const pbrtgpu_bvh_node &b = s->nodes[i];
        if ((b.meta & 0xff) && b.offset < (uint32_t)s->n_prims) (*leafOf)[b.offset] = i;
    }
    wq->assign(nw * 4, make_uint4(0u, 0u, 0u, 0u));
    auto fbits = [](float f) { uint32_t u; memcpy(&u, &f, 4); return u; };
    for (size_t n = 0; n < nw; ++n) {
        const float4 *w = &w4[n * 8];
        uint32_t refs[4];
        float lo[4][3], hi[4][3];
        int used = 0;
        for (int k = 0; k < 4; ++k) {
            uint32_t r;
            memcpy(&r, &w[2 * k].w, 4);
            refs[k] = r;
            lo[k][0] = w[2 * k].x; lo[k][1] = w[2 * k].y; lo[k][2] = w[2 * k].z;
            hi[k][0] = w[2 * k + 1].x; hi[k][1] = w[2 * k + 1].y; hi[k][2] = w[2 * k + 1].z;
            if (r != 0xffffffffu) ++used;
        }
        if (!used) SB_FAIL(PBRTGPU_E_INVALID, "4-wide node without children");
        uint8_t qb[24] = {0};
        uint32_t exactBits = 0, expBits = 0;
        float org[3];
        for (int a = 0; a < 3; ++a) {
            float o = INFINITY, top = -INFINITY;
            for (int k = 0; k < 4; ++k)
                if (refs[k] != 0xffffffffu) { o = std::min(o, lo[k][a]); top = std::max(top, hi[k][a]); }
            if (!(o <= top) || !std::isfinite(o) || !std::isfinite(top)) SB_FAIL(PBRTGPU_E_INVALID, "BVH box");
            org[a] = o;
            // the smallest exponent whose 255 steps reach the top bound from the origin
            int e = -126;
            const float span = top - o;
            if (span > 0.f) e = std::max(-126, (int)std::ceil(std::log2((double)span / 250.0)));
            auto deq = [&](int q, int ee) {
                const float sc = std::ldexp(1.f, ee);
                const float v = (float)q * sc;   // exact: q < 256, sc a power of two
                return o + v;                    // rounded as the device rounds it
            };
            while (e < 127 && deq(255, e) < top) ++e;
            if (e >= 127) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "BVH box too large to quantize");
            expBits |= (uint32_t)(e + 127) << (8 * a);
            for (int k = 0; k < 4; ++k) {
                if (refs[k] == 0xffffffffu) continue;
                int ql = 0;   // the largest q with deq(q) <= lo
                while (ql < 255 && deq(ql + 1, e) <= lo[k][a]) ++ql;
                int qh = 255;   // the smallest q with deq(q) >= hi
                while (qh > 0 && deq(qh - 1, e) >= hi[k][a]) --qh;
                if (!(deq(ql, e) <= lo[k][a]) || !(deq(qh, e) >= hi[k][a])) SB_FAIL(PBRTGPU_E_INVALID, "BVH quantization");
                qb[6 * k + a] = (uint8_t)ql;
                qb[6 * k + 3 + a] = (uint8_t)qh;
                if (deq(ql, e) == lo[k][a]) exactBits |= 1u << (6 * k + a);
                if (deq(qh, e) == hi[k][a]) exactBits |= 1u << (6 * k + 3 + a);
            }
        }
        uint32_t pk[6];
        memcpy(pk, qb, 24);
        uint4 *q = &(*wq)[n * 4];
        q[0] = make_uint4(fbits(org[0]), fbits(org[1]), fbits(org[2]), expBits);
        q[1] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        q[2] = make_uint4(pk[4], pk[5], refs[0], refs[1]);
        q[3] = make_uint4(refs[2], refs[3], exactBits, 0u);
    }
    return 0;
}

// SpectralRendererTask::Run's wave bands (spectralrenderer.cpp:99-100, 124, 180-188) in the
// reference's own int / float arithmetic (sampledLambdaStart / sampledLambdaEnd are ints:
// 395 / 715 in the 32- and 60-band builds, spectrum.h:41-42; 400 / 700 in the upstream 30-band
// one, spectrum.h.original:36-38): band b's wavelength start + dW b + dW / 2 with dW =
// float((end - start) / nWB), its interval i of GetValueAtWavelength (spectrum.h:384-405: step
// float((end - start) / N), first i with w0 <= wl < w1) and t = (wl - w0) / (w1 - w0), and its
// indices [dI b, min(dI (b+1), N-1)), dI = round(N / nWB).  A band with indices whose interval is
// the last reads c[N], past the spectrum: rejected.
static inline int spectral_table(int N, int nWB, std::vector<int4> *tab, std::vector<float> *wls, std::string *err) {
    const int lStart = N == 30 ? 400 : 395, lEnd = N == 30 ? 700 : 715;
    const int dI = (int)round(N / nWB);
    const float dW = (float)((lEnd - lStart) / nWB);
    const float step = (float)((lEnd - lStart) / N);
    tab->resize(nWB);
    wls->resize(nWB);
    for (int b = 0; b < nWB; ++b) {
        const float wl = lStart + dW * b + (dW / 2);
        (*wls)[b] = wl;
        int iv = -1;
        float t = 0.f;
        for (int i = 0; i < N; ++i) {
            const float w0 = lStart + i * step, w1 = lStart + (i + 1) * step;
            if (wl >= w0 && wl < w1) { iv = i; t = (wl - w0) / (w1 - w0); break; }
        }
        const int lo = dI * b, hi = std::max(lo, std::min(dI * (b + 1), N - 1));
        if (hi > lo && iv == N - 1) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "nWaveBands: a band reads past the spectrum (spectrum.h:397)");
        uint32_t tb;
        memcpy(&tb, &t, 4);
        (*tab)[b] = make_int4(lo, hi, iv, (int)tb);
    }
    return 0;
}

// The checks that need nothing placed: an invalid scene is refused before the context drops
// its current one.
static inline int scene_check(const pbrtgpu_flat_scene *s, std::string *err) {
    if (!s) SB_FAIL(PBRTGPU_E_INVALID, "null argument");
    if (s->abi_version != PBRTGPU_ABI_VERSION) SB_FAIL(PBRTGPU_E_INVALID, "ABI version mismatch");
    if (!(s->n_bands == 32 || s->n_bands == 60 || s->n_bands == 30 || s->n_bands == 3))
        SB_FAIL(PBRTGPU_E_UNSUPPORTED, "n_bands must be 30, 32, 60 or 3 (RGB)");
    // the RGB build (C1): image textures, the environment light and MERL tables take their RGB
    // as the spectrum (RGBSpectrum::FromRGB, device.h rgb_pick); the SpectralRenderer does not exist
    if (s->n_bands == 3 && s->renderer == PBRTGPU_RENDERER_SPECTRAL)
        SB_FAIL(PBRTGPU_E_UNSUPPORTED, "RGB build: the SpectralRenderer needs SampledSpectrum");
    if (s->spp <= 0 || (s->spp & (s->spp - 1))) SB_FAIL(PBRTGPU_E_INVALID, "spp must be a power of two");
    if (s->max_depth < 0 || s->max_depth > 100000) SB_FAIL(PBRTGPU_E_INVALID, "maxdepth out of range");
    if (s->n_nodes <= 0 || s->n_prims <= 0) SB_FAIL(PBRTGPU_E_INVALID, "empty scene");
    if (s->integrator != PBRTGPU_INTEGRATOR_PATH && s->integrator != PBRTGPU_INTEGRATOR_DIRECT &&
        s->integrator != PBRTGPU_INTEGRATOR_METADATA)
        SB_FAIL(PBRTGPU_E_INVALID, "unknown SurfaceIntegrator");
    if (s->integrator == PBRTGPU_INTEGRATOR_METADATA) {
        if (s->meta_strategy < PBRTGPU_META_MESH || s->meta_strategy > PBRTGPU_META_DEPTH)
            SB_FAIL(PBRTGPU_E_INVALID, "unknown metadata strategy");
        if (s->meta_strategy != PBRTGPU_META_DEPTH && !s->prim_meta)
            SB_FAIL(PBRTGPU_E_INVALID, "metadata mesh / material ids need prim_meta");
    }
    if (s->renderer != PBRTGPU_RENDERER_SAMPLER && s->renderer != PBRTGPU_RENDERER_SPECTRAL)
        SB_FAIL(PBRTGPU_E_INVALID, "unknown Renderer");
    std::vector<int4> specTab;
    std::vector<float> specWl;
    if (s->renderer == PBRTGPU_RENDERER_SPECTRAL) {
        if (s->spectral_sampling != PBRTGPU_SPECTRAL_SINGLE && s->spectral_sampling != PBRTGPU_SPECTRAL_SAMPLER)
            SB_FAIL(PBRTGPU_E_INVALID, "unknown spectral sampling method");
        if (s->wave_bands < 1 || s->wave_bands > 1024) SB_FAIL(PBRTGPU_E_INVALID, "nWaveBands must be 1..1024");
        if (int e = spectral_table(s->n_bands, s->wave_bands, &specTab, &specWl, err)) return e;
    }
    if (s->camera_type != PBRTGPU_CAMERA_PERSPECTIVE && s->camera_type != PBRTGPU_CAMERA_REALISTIC &&
        s->camera_type != PBRTGPU_CAMERA_ORTHOGRAPHIC)
        SB_FAIL(PBRTGPU_E_INVALID, "unknown camera type");
    if ((s->camera.ortho != 0) != (s->camera_type == PBRTGPU_CAMERA_ORTHOGRAPHIC))
        SB_FAIL(PBRTGPU_E_INVALID, "camera.ortho does not match camera_type");
    if (s->camera_type == PBRTGPU_CAMERA_REALISTIC) {
        const pbrtgpu_lens &L = s->lens;
        if (L.n_elements < 1 || L.n_elements > 4096 || !L.elements) SB_FAIL(PBRTGPU_E_INVALID, "lens camera without elements");
        // element 1 refracting into element 0 of n == 0 would read lensEls[-1] (realisticDiffraction.cpp:960-966)
        if (L.n_elements >= 2 && L.elements[2] == 0 && L.elements[4] != 0)
            SB_FAIL(PBRTGPU_E_INVALID, "lens element 0 has n == 0");
        if (s->camera.xres <= 0 || s->camera.yres <= 0) SB_FAIL(PBRTGPU_E_INVALID, "lens camera without film resolution");
        if (L.num_pinholes_w > 0 && L.num_pinholes_h > 0) {
            // GenerateRay divides by the pixels per superpixel (realisticDiffraction.cpp:566-570)
            if (L.num_pinholes_w > s->camera.xres || L.num_pinholes_h > s->camera.yres)
                SB_FAIL(PBRTGPU_E_INVALID, "more pinholes than film pixels");
            if (!L.pinholes) SB_FAIL(PBRTGPU_E_INVALID, "pinhole array missing");
        }
        if (L.ior_eye) {
            if (!L.eye_ior || s->n_bands == 3) SB_FAIL(PBRTGPU_E_INVALID, "IORforEyeEnabled without SampledSpectrum IOR curves");
            // a band wavelength in the last interval would read c[N] in GetValueAtWavelength (spectrum.h:397)
            if (s->renderer == PBRTGPU_RENDERER_SPECTRAL)
                for (size_t b = 0; b < specTab.size(); ++b)
                    if (specTab[b].z == s->n_bands - 1)
                        SB_FAIL(PBRTGPU_E_UNSUPPORTED, "IORforEyeEnabled: a wave band's wavelength reads past the IOR spectra");
        }
    }
    if (s->integrator == PBRTGPU_INTEGRATOR_DIRECT && s->dl_strategy != PBRTGPU_DL_ALL && s->dl_strategy != PBRTGPU_DL_ONE)
        SB_FAIL(PBRTGPU_E_INVALID, "unknown DirectLighting strategy");
    for (int i = 0; i < s->n_lights; ++i)
        if (s->lights[i].type < PBRTGPU_LIGHT_AREA || s->lights[i].type > PBRTGPU_LIGHT_DISTANT)
            SB_FAIL(PBRTGPU_E_INVALID, "bad light type");
    if (!s->rgb_basis || !s->ewa_lut) SB_FAIL(PBRTGPU_E_INVALID, "rgb_basis / ewa_lut missing");
    // texture graph: SCALE nodes combine CONST / IMAGE leaves; a material's spectrum slot is an
    // IMAGE or SCALE(IMAGE, CONST) spectrum texture, its bump a float texture
    // a leaf of a combining node (SCALE, MIX, CHECKER, DOTS): exactly the kinds the device evaluates
    // as leaves -- spectral: CONST / IMAGE / UV (spec_leaf -> leaf_rgb); float: CONST / IMAGE and the
    // noise textures (tex_leaf_float) -- with a valid mapping and octave count.  Checked against
    // this list rather than against refused kinds, so a node kind added later is refused as a leaf
    // until the device evaluates it there.
    auto leafOk = [&](int o, int spectral) -> bool {
        if (o < 0 || o >= s->n_textures || !s->textures) return false;
        const pbrtgpu_texture &l = s->textures[o];
        if (l.spectral != spectral) return false;
        const int ty = l.type;
        const bool noise = ty >= PBRTGPU_TEX_FBM && ty <= PBRTGPU_TEX_WINDY;
        const bool ok = ty == PBRTGPU_TEX_CONST || ty == PBRTGPU_TEX_IMAGE || (spectral ? ty == PBRTGPU_TEX_UV : noise);
        if (!ok) return false;
        if (noise && (l.levels < 0 || l.levels > 64)) return false;
        return l.mapping >= PBRTGPU_MAP_UV && l.mapping <= PBRTGPU_MAP_PLANAR;
    };
    auto texOk = [&](int id, int spectral, bool slot) -> bool {
        if (id < 0 || id >= s->n_textures || !s->textures) return false;
        const pbrtgpu_texture &t = s->textures[id];
        if (t.spectral != spectral || t.type < PBRTGPU_TEX_CONST || t.type > PBRTGPU_TEX_MARBLE) return false;
        if (t.type == PBRTGPU_TEX_MARBLE &&   // spectrum only; its nine spline colours in the pool
            (!spectral || t.levels < 0 || t.levels > 64 || t.spec < 0 ||
             (int64_t)t.spec + 9LL * s->n_bands > (int64_t)s->n_spectra_floats))
            return false;
        if (t.type >= PBRTGPU_TEX_FBM && t.type <= PBRTGPU_TEX_WINDY && (t.levels < 0 || t.levels > 64))
            return false;   // noise
        if (t.type == PBRTGPU_TEX_BILERP) {   // its four values: spectra in the pool / floats in texels[]
            if (spectral ? (t.spec < 0 || (int64_t)t.spec + 4LL * s->n_bands > (int64_t)s->n_spectra_floats)
                         : (t.texel_off < 0 || !s->texels || (int64_t)t.texel_off + 4 > (int64_t)s->n_texel_floats))
                return false;
        }
        if (t.type == PBRTGPU_TEX_MIX) {   // two CONST / IMAGE / UV leaves, a CONST / IMAGE float amount
            for (int o : {t.tex1, t.tex2})
                if (!leafOk(o, spectral) || s->textures[o].type > PBRTGPU_TEX_UV) return false;
            const int a = t.amount;
            if (a < 0 || a >= s->n_textures || s->textures[a].spectral ||
                (s->textures[a].type != PBRTGPU_TEX_CONST && s->textures[a].type != PBRTGPU_TEX_IMAGE))
                return false;
        }
        if (t.type == PBRTGPU_TEX_UV && !spectral) return false;   // UVTexture is Texture<Spectrum> only
        if (t.type == PBRTGPU_TEX_CHECKER || t.type == PBRTGPU_TEX_DOTS) {   // two CONST / IMAGE / UV leaves
            for (int o : {t.tex1, t.tex2})
                if (!leafOk(o, spectral) || s->textures[o].type > PBRTGPU_TEX_UV) return false;
            if (t.aamode < 0 || t.aamode > 1) return false;
        }
        if (t.type != PBRTGPU_TEX_IMAGE && t.type != PBRTGPU_TEX_CHECKER && t.type != PBRTGPU_TEX_UV &&
            t.type != PBRTGPU_TEX_BILERP && t.type != PBRTGPU_TEX_DOTS && t.mapping != PBRTGPU_MAP_UV)
            return false;
        if (t.mapping < PBRTGPU_MAP_UV || t.mapping > PBRTGPU_MAP_PLANAR) return false;
        if (t.type == PBRTGPU_TEX_SCALE) {
            for (int o : {t.tex1, t.tex2})
                if (!leafOk(o, spectral)) return false;
            if (spectral && (s->textures[t.tex1].type == PBRTGPU_TEX_CONST) == (s->textures[t.tex2].type == PBRTGPU_TEX_CONST))
                return false;
        }
        return !(slot && spectral && t.type == PBRTGPU_TEX_CONST);
    };
    // MIPMap pyramids: power-of-two level 0, nLevels = 1 + floor(log2(max(w, h))), every level
    // inside the texel pool (the lookups index texels[] without further checks)
    for (int i = 0; i < s->n_textures; ++i) {
        const pbrtgpu_texture &t = s->textures[i];
        if (t.type != PBRTGPU_TEX_IMAGE) continue;
        const int w = t.width, h = t.height, nc = t.spectral ? 3 : 1;
        int lv = 0;
        for (int m = w > h ? w : h; m > 1; m >>= 1) ++lv;
        if (w < 1 || h < 1 || w > (1 << 24) || h > (1 << 24) || (w & (w - 1)) || (h & (h - 1)) || t.levels != lv + 1 ||
            t.texel_off < 0 || !s->texels)
            SB_FAIL(PBRTGPU_E_INVALID, "image texture pyramid");
        int64_t n = 0;
        for (int l = 0; l < t.levels; ++l) n += (int64_t)(w >> l > 1 ? w >> l : 1) * (h >> l > 1 ? h >> l : 1) * nc;
        if ((int64_t)t.texel_off + n > (int64_t)s->n_texel_floats) SB_FAIL(PBRTGPU_E_INVALID, "image texture texels out of range");
    }
    for (int i = 0; i < s->n_materials; ++i) {
        const pbrtgpu_material &m = s->materials[i];
        if (m.type < PBRTGPU_MAT_MATTE || m.type > PBRTGPU_MAT_SHINYMETAL)
            SB_FAIL(PBRTGPU_E_UNSUPPORTED, "material type not yet supported on the GPU");
        // textured spectra in slots 0 and 1 only (device.h get_bsdf's two K buffers), textured float
        // parameters f[0], f[1]; the measured materials have none
        for (int k = 0; k < 4; ++k)
            if (m.tex[k] >= 0 && (k > 1 || !texOk(m.tex[k], 1, true) || m.type == PBRTGPU_MAT_MEASURED ||
                                  m.type == PBRTGPU_MAT_MEASURED_HALFANGLE))
                SB_FAIL(PBRTGPU_E_UNSUPPORTED, "material spectrum texture");
        for (int j = 0; j < 2; ++j)
            if (m.ftex[j] >= 0 && (!texOk(m.ftex[j], 0, false) || m.type == PBRTGPU_MAT_MEASURED ||
                                   m.type == PBRTGPU_MAT_MEASURED_HALFANGLE || m.type == PBRTGPU_MAT_MIRROR))
                SB_FAIL(PBRTGPU_E_INVALID, "material float texture");
        if (m.bump_tex >= 0 && !texOk(m.bump_tex, 0, false)) SB_FAIL(PBRTGPU_E_INVALID, "bump texture");
        if (m.normal_tex >= 0 && (!texOk(m.normal_tex, 1, false) || s->textures[m.normal_tex].type == PBRTGPU_TEX_MIX))
            SB_FAIL(PBRTGPU_E_INVALID, "normal map texture");
        if (m.type == PBRTGPU_MAT_MEASURED_HALFANGLE && m.aux >= 0 &&
            (!s->merl || s->n_merl_floats < 0 || (int64_t)m.aux * 3 + 3 * 90 * 90 * 180 > (int64_t)s->n_merl_floats))
            SB_FAIL(PBRTGPU_E_INVALID, "RegularHalfangle table out of range");
    }
    return 0;
}

// DevScene of a checked scene (scene_check); *feat: the FEAT_* of the k_shade variant it needs.
// topNodes: wide BVH nodes laid out first for k_trace_pt's LDS copy.
template <class Put>
static int scene_build(const pbrtgpu_flat_scene *s, int topNodes, DevScene &S, int *feat, Put put, std::string *err) {
    std::vector<int4> specTab;
    std::vector<float> specWl;
    if (s->renderer == PBRTGPU_RENDERER_SPECTRAL)
        if (int e = spectral_table(s->n_bands, s->wave_bands, &specTab, &specWl, err)) return e;
    S.nb = s->n_bands;
    S.maxDepth = s->max_depth;
    S.spp = s->spp;
    S.seed = s->seed;
    S.yint = s->y_int;
    S.cam = s->camera;
    S.nLights = s->n_lights;
    S.integrator = s->integrator;
    S.dlStrategy = s->dl_strategy;
    S.metaStrategy = s->meta_strategy;
    S.primMeta = nullptr;
    if (s->prim_meta) SB_PUT(s->prim_meta, (size_t)2 * s->n_prims, &S.primMeta);
    S.specMode = s->renderer != PBRTGPU_RENDERER_SPECTRAL ? 0 : s->spectral_sampling == PBRTGPU_SPECTRAL_SINGLE ? 1 : 2;
    S.specBands = S.specMode ? s->wave_bands : 1;
    S.specItems = S.specMode == 1 ? s->wave_bands : 1;
    S.specTab = nullptr;
    S.specWl = nullptr;
    if (S.specMode) {
        SB_PUT(specTab.data(), specTab.size(), &S.specTab);
        SB_PUT(specWl.data(), specWl.size(), &S.specWl);
    }
    S.camType = s->camera_type;
    S.lensN = 0;
    S.lensEl = nullptr;
    if (S.camType == PBRTGPU_CAMERA_REALISTIC) {
        const pbrtgpu_lens &L = s->lens;
        S.lensN = L.n_elements;
        S.lensChromatic = L.chromatic;
        S.lensDiffraction = L.diffraction;
        S.lensFilmDist = L.film_distance;
        S.lensFilmDiag = L.film_diag;
        S.lensCurveR = L.curve_radius;
        for (int k = 0; k < 2; ++k) { S.lensApOff[k] = L.aperture_offset[k]; S.lensFilmC[k] = L.film_center[k]; }
        for (int k = 0; k < 3; ++k) S.lensPinhole[k] = L.pinhole_exit[k];
        SB_PUT(reinterpret_cast<const float4 *>(L.elements), (size_t)L.n_elements, &S.lensEl);
        S.lensPinW = L.num_pinholes_w;
        S.lensPinH = L.num_pinholes_h;
        S.lensMicro = L.microlens;
        S.lensEye = L.ior_eye;
        S.lensPinholes = nullptr;
        S.lensEyeIor = nullptr;
        if (L.num_pinholes_w > 0 && L.num_pinholes_h > 0)
            SB_PUT(L.pinholes, (size_t)L.num_pinholes_w * L.num_pinholes_h * 3, &S.lensPinholes);
        if (L.ior_eye) SB_PUT(L.eye_ior, (size_t)4 * s->n_bands, &S.lensEyeIor);
    }
    S.dlK = 0;
    for (int i = 0; i < s->n_lights; ++i) {   // RoundUpPow2(max(1, nSamples)) per light
        uint32_t v = (uint32_t)std::max(1, s->lights[i].n_samples) - 1u;
        v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
        if (v + 1u > (1u << 16)) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "light nsamples > 65536");
        S.dlK += (int)(v + 1u);
    }
    // BVH: verify topology and measure the stack depth traversal needs (top level, plus the
    // deepest nested instance BVH whose walk stacks above it)
    if (s->n_instances < 0 || (s->n_instances > 0 && (!s->instances || !s->prim_instance)))
        SB_FAIL(PBRTGPU_E_INVALID, "instance arrays missing");
    auto walkDepth = [&](uint32_t root, int *depthOut) -> int {
        int maxD = 0;
        std::vector<std::pair<uint32_t, int> > todo;
        todo.push_back(std::make_pair(root, 0));
        while (!todo.empty()) {
            auto q = todo.back();
            todo.pop_back();
            if (q.first >= (uint32_t)s->n_nodes) SB_FAIL(PBRTGPU_E_INVALID, "BVH node index out of range");
            const pbrtgpu_bvh_node &n = s->nodes[q.first];
            maxD = std::max(maxD, q.second);
            if ((n.meta & 0xff) == 0) {
                if (q.second > 62) SB_FAIL(PBRTGPU_E_UNSUPPORTED, "BVH deeper than 63 levels");
                todo.push_back(std::make_pair(q.first + 1, q.second + 1));
                todo.push_back(std::make_pair(n.offset, q.second + 1));
            } else if (n.offset + (n.meta & 0xff) > (uint32_t)s->n_prims)
                SB_FAIL(PBRTGPU_E_INVALID, "BVH leaf out of range");
        }
        *depthOut = maxD;
        return 0;
    };
    int maxDepth = 0, instDepth = 0;
    if (int e = walkDepth(0, &maxDepth)) return e;
    for (int i = 0; i < s->n_instances; ++i) {
        const pbrtgpu_instance &I = s->instances[i];
        if (I.root >= 0) {
            int dd = 0;
            if (int e = walkDepth((uint32_t)I.root, &dd)) return e;
            instDepth = std::max(instDepth, dd + 1);
        } else if (I.single_prim < 0 || I.single_prim >= s->n_prims)
            SB_FAIL(PBRTGPU_E_INVALID, "instance without primitives");
    }
    for (int i = 0; i < s->n_prims; ++i)
        if (s->prims[i].shape_type == PBRTGPU_SHAPE_INSTANCE &&
            (s->prims[i].shape_index < 0 || s->prims[i].shape_index >= s->n_instances))
            SB_FAIL(PBRTGPU_E_INVALID, "bad instance index");
    maxDepth += instDepth;
    S.stackDepth = maxDepth + 1;
    SB_PUT(s->band_Y, (size_t)s->n_bands, &S.bandY);
    SB_PUT(reinterpret_cast<const float4 *>(s->nodes), (size_t)s->n_nodes * 2, &S.nodes);
    {
        std::vector<float4> wn;
        std::vector<uint32_t> ref;
        if (int e = wide_bvh(s, topNodes, &wn, &ref, &S.nTop, err)) return e;
        SB_PUT(wn.data(), wn.size(), &S.wnodes);
        SB_PUT(ref.data(), ref.size(), &S.nodeRef);
        // the 4-wide copy (scenes without instances)
        std::vector<float4> w4;
        S.w4nodes = nullptr;
        S.w4N = 0;
        S.w4Stack = 0;
        S.w4q = nullptr;
        S.leafOf = nullptr;
        if (s->n_instances == 0) {
            if (int e = wide4_bvh(s, ref, &w4, &S.w4Stack, err)) return e;
            if (!w4.empty()) {
                SB_PUT(w4.data(), w4.size(), &S.w4nodes);
                S.w4N = (int)(w4.size() / 8);
                std::vector<uint4> wq;
                std::vector<int32_t> leafOf;
                if (int e = quant_w4(s, w4, &wq, &leafOf, err)) return e;
                if (!wq.empty()) {
                    SB_PUT(wq.data(), wq.size(), &S.w4q);
                    SB_PUT(leafOf.data(), leafOf.size(), &S.leafOf);
                }
            }
        }
    }
    SB_PUT(s->prims, (size_t)s->n_prims, &S.prims);
    std::vector<DevTri> pt(s->n_prims);
    for (int i = 0; i < s->n_prims; ++i) {
        const pbrtgpu_prim &p = s->prims[i];
        DevTri t{};
        int32_t ty = p.shape_type;   // a.w: the shape type (device.h DevTri)
        memcpy(&t.a.w, &ty, 4);
        if (p.shape_type == PBRTGPU_SHAPE_INSTANCE) {
            pt[i] = t;
            continue;
        }
        if (p.shape_type == PBRTGPU_SHAPE_TRIANGLE) {
            if (p.shape_index < 0 || p.shape_index >= s->n_tris) SB_FAIL(PBRTGPU_E_INVALID, "bad triangle index");
            const pbrtgpu_triangle &tr = s->tris[p.shape_index];
            if (tr.mesh < 0 || tr.mesh >= s->n_meshes) SB_FAIL(PBRTGPU_E_INVALID, "bad triangle mesh");
            for (int k = 0; k < 3; ++k)
                if (tr.v[k] < 0 || tr.v[k] >= s->n_verts) SB_FAIL(PBRTGPU_E_INVALID, "bad triangle vertex");
            const float *a = s->vert_p + 3 * tr.v[0], *b = s->vert_p + 3 * tr.v[1], *cc = s->vert_p + 3 * tr.v[2];
            t.a = make_float4(a[0], a[1], a[2], 0.f);   // a.w = 0 = PBRTGPU_SHAPE_TRIANGLE
            t.b = make_float4(b[0], b[1], b[2], 0.f);
            t.c = make_float4(cc[0], cc[1], cc[2], 0.f);
        } else if (p.shape_index < 0 || p.shape_index >= s->n_quadrics)
            SB_FAIL(PBRTGPU_E_INVALID, "bad quadric index");
        pt[i] = t;
    }
    // the per-primitive shading records (device.h PrimRec): the hit's geometry, uvs, normals,
    // prim fields and mesh flags in one 128-byte line, values copied from the flattened scene
    std::vector<float4> rec((size_t)8 * s->n_prims, make_float4(0.f, 0.f, 0.f, 0.f));
    auto fi = [](int32_t v) { float f; memcpy(&f, &v, 4); return f; };
    for (int i = 0; i < s->n_prims; ++i) {
        const pbrtgpu_prim &p = s->prims[i];
        float4 *r = &rec[(size_t)8 * i];
        r[6] = make_float4(fi(p.shape_type), fi(p.shape_index), fi(p.material), fi(p.area_light));
        if (p.shape_type != PBRTGPU_SHAPE_TRIANGLE) continue;
        const pbrtgpu_triangle &tr = s->tris[p.shape_index];
        const pbrtgpu_mesh &m = s->meshes[tr.mesh];
        float uv[3][2] = {{0.f, 0.f}, {1.f, 0.f}, {1.f, 1.f}};   // Triangle::GetUVs without uvs
        if (m.has_uvs) {
            if (!s->vert_uv) SB_FAIL(PBRTGPU_E_INVALID, "mesh uvs missing");
            for (int k = 0; k < 3; ++k) { uv[k][0] = s->vert_uv[2 * tr.v[k]]; uv[k][1] = s->vert_uv[2 * tr.v[k] + 1]; }
        }
        if (m.has_normals && !s->vert_n) SB_FAIL(PBRTGPU_E_INVALID, "mesh normals missing");
        const float w[6] = {uv[0][0], uv[0][1], uv[1][0], uv[1][1], uv[2][0], uv[2][1]};
        for (int k = 0; k < 3; ++k) {
            const float *v = s->vert_p + 3 * tr.v[k];
            r[k] = make_float4(v[0], v[1], v[2], w[k]);
            const float *n = m.has_normals ? s->vert_n + 3 * tr.v[k] : nullptr;
            r[3 + k] = make_float4(n ? n[0] : 0.f, n ? n[1] : 0.f, n ? n[2] : 0.f, w[3 + k]);
        }
        const int flags = (m.has_normals ? 2 : 0) | ((m.reverse_orientation ^ m.swaps_handedness) ? 4 : 0);
        r[7] = make_float4(fi(flags), fi(tr.mesh), 0.f, 0.f);
    }
    SB_PUT(rec.data(), rec.size(), &S.primRec);
    // spectrum pool re-laid out with a stride of whole float4 quads (16-byte aligned band
    // quads for the shading loads); every offset in the flattened scene is a multiple of
    // n_bands (front end emits whole spectra)
    const int nbp = (s->n_bands + 3) / 4 * 4;
    if (s->n_spectra_floats % s->n_bands) SB_FAIL(PBRTGPU_E_INVALID, "spectrum pool is not whole spectra");
    auto remap = [&](int32_t off, int32_t *out) -> bool {
        if (off < 0) { *out = off; return true; }
        if (off % s->n_bands || off >= s->n_spectra_floats) return false;
        *out = off / s->n_bands * nbp;
        return true;
    };
    std::vector<float> pool((size_t)s->n_spectra_floats / s->n_bands * nbp, 0.f);
    for (int k = 0; k < s->n_spectra_floats / s->n_bands; ++k)
        for (int i = 0; i < s->n_bands; ++i) pool[(size_t)k * nbp + i] = s->spectra[(size_t)k * s->n_bands + i];
    std::vector<pbrtgpu_material> mats(s->materials, s->materials + s->n_materials);
    for (auto &m : mats)
        for (int k = 0; k < 4; ++k)
            if (!remap(m.spec[k], &m.spec[k])) SB_FAIL(PBRTGPU_E_INVALID, "material spectrum offset");
    std::vector<pbrtgpu_light> lts(s->lights, s->lights + s->n_lights);
    S.nInf = 0;
    int nSpotDistant = 0;
    for (auto &l : lts) {
        if (!remap(l.spec, &l.spec)) SB_FAIL(PBRTGPU_E_INVALID, "light spectrum offset");
        if (l.type == PBRTGPU_LIGHT_INFINITE) ++S.nInf;
        if (l.type == PBRTGPU_LIGHT_SPOT || l.type == PBRTGPU_LIGHT_DISTANT) ++nSpotDistant;
    }
    std::vector<pbrtgpu_texture> texs(s->textures, s->textures + std::max(0, s->n_textures));
    for (auto &t : texs)
        if ((t.type == PBRTGPU_TEX_CONST || t.type == PBRTGPU_TEX_BILERP || t.type == PBRTGPU_TEX_MARBLE) && t.spectral &&
            !remap(t.spec, &t.spec))
            SB_FAIL(PBRTGPU_E_INVALID, "texture spectrum offset");
    // FromRGB basis, each of the 14 spectra padded to whole quads
    std::vector<float> basis((size_t)14 * nbp, 0.f);
    for (int k = 0; k < 14; ++k)
        for (int i = 0; i < s->n_bands; ++i) basis[(size_t)k * nbp + i] = s->rgb_basis[(size_t)k * s->n_bands + i];
    S.nbp = nbp;
    SB_PUT(texs.data(), texs.size(), &S.tex);
    SB_PUT(basis.data(), basis.size(), &S.basis);
    SB_PUT(s->ewa_lut, (size_t)128, &S.ewa);
    S.texels = nullptr;
    if (s->n_texel_floats > 0) SB_PUT(s->texels, (size_t)s->n_texel_floats, &S.texels);
    S.camMotion = nullptr;
    if (s->camera_motion) SB_PUT(s->camera_motion, (size_t)1, &S.camMotion);
    SB_PUT(pt.data(), pt.size(), &S.primTri);
    SB_PUT(s->tris, (size_t)s->n_tris, &S.tris);
    SB_PUT(s->meshes, (size_t)s->n_meshes, &S.meshes);
    SB_PUT(s->vert_p, (size_t)s->n_verts * 3, &S.vertP);
    SB_PUT(s->vert_n, (size_t)s->n_verts * 3, &S.vertN);
    SB_PUT(s->vert_uv, (size_t)s->n_verts * 2, &S.vertUV);
    SB_PUT(s->quadrics, (size_t)s->n_quadrics, &S.quads);
    SB_PUT(mats.data(), mats.size(), &S.mats);
    SB_PUT(lts.data(), lts.size(), &S.lights);
    SB_PUT(s->light_shapes, (size_t)s->n_light_shapes, &S.lightShapes);
    S.nInsts = s->n_instances;
    SB_PUT(s->instances, (size_t)s->n_instances, &S.insts);
    {
        std::vector<int> pi(s->n_prims, -1);
        if (s->n_instances > 0) for (int i = 0; i < s->n_prims; ++i) pi[i] = s->prim_instance[i];
        SB_PUT(pi.data(), pi.size(), &S.primInst);
    }
    SB_PUT(pool.data(), pool.size(), &S.spectra);
    {
        std::vector<pbrtgpu_kdnode> kd(s->kdnodes, s->kdnodes + std::max(0, s->n_kdnodes));
        for (auto &k : kd)
            if (!remap(k.spec, &k.spec)) SB_FAIL(PBRTGPU_E_INVALID, "kd-tree spectrum offset");
        for (auto &m : mats)
            if (m.type == PBRTGPU_MAT_MEASURED && (m.aux < 0 || m.aux2 <= 0 || m.aux + m.aux2 > (int)kd.size()))
                SB_FAIL(PBRTGPU_E_INVALID, "measured material kd-tree range");
        SB_PUT(kd.data(), kd.size(), &S.kd);
        // packed nodes with parent links (relative indices; left child = node + 1) for the
        // stackless lookup walk (kd_lookup, wavefront.h)
        std::vector<float4> pack(2 * kd.size(), make_float4(0.f, 0.f, 0.f, 0.f));
        std::vector<int> par(kd.size(), -1);
        for (auto &m : mats) {
            if (m.type != PBRTGPU_MAT_MEASURED) continue;
            for (int i = 0; i < m.aux2; ++i) {
                const pbrtgpu_kdnode &k = kd[(size_t)m.aux + i];
                if (k.split_axis < 0 || k.split_axis > 3) SB_FAIL(PBRTGPU_E_INVALID, "kd-tree split axis");
                if (k.split_axis == 3) continue;
                if (k.has_left) {
                    if (i + 1 >= m.aux2) SB_FAIL(PBRTGPU_E_INVALID, "kd-tree left child out of range");
                    par[(size_t)m.aux + i + 1] = i;
                }
                if (k.right_child < m.aux2) {
                    if (k.right_child <= i) SB_FAIL(PBRTGPU_E_INVALID, "kd-tree right child order");
                    par[(size_t)m.aux + k.right_child] = i;
                }
            }
            for (int i = 0; i < m.aux2; ++i) {
                const pbrtgpu_kdnode &k = kd[(size_t)m.aux + i];
                const int rc = (k.split_axis != 3 && k.right_child < m.aux2) ? k.right_child : -1;
                const int meta = k.split_axis | (k.has_left && k.split_axis != 3 ? 4 : 0);
                pack[2 * ((size_t)m.aux + i)] = make_float4(k.p[0], k.p[1], k.p[2], k.split_pos);
                pack[2 * ((size_t)m.aux + i) + 1] =
                    make_float4(sb_bits_f((uint32_t)k.spec), sb_bits_f((uint32_t)rc), sb_bits_f((uint32_t)par[(size_t)m.aux + i]),
                                sb_bits_f((uint32_t)meta));
            }
        }
        SB_PUT(pack.data(), pack.size(), &S.kdPack);
        SB_PUT(s->merl, (size_t)std::max(0, s->n_merl_floats), &S.merl);
        S.nKd = (int)kd.size();
        S.kdInLds = (S.nKd > 0 && S.nKd <= kKdLdsNodes) ? 1 : 0;
    }
    // FEAT_INF: the light types beyond area and point (infinite, spot, distant) -- the kernels of
    // scenes with area and point lights only (C2, C3) carry none of their code
    *feat = (S.nInf > 0 || nSpotDistant > 0) ? FEAT_INF : 0;
    for (int i = 0; i < s->n_materials; ++i) {
        const pbrtgpu_material &m = s->materials[i];
        if (m.type == PBRTGPU_MAT_MEASURED || m.type == PBRTGPU_MAT_MEASURED_HALFANGLE) *feat |= FEAT_MEAS;
        if (m.type == PBRTGPU_MAT_SHINYMETAL) *feat |= FEAT_TEX;   // its conductor SpecularReflection (fval4)
        if (m.bump_tex >= 0 || m.normal_tex >= 0 || m.tex[0] >= 0 || m.tex[1] >= 0 || m.tex[2] >= 0 || m.tex[3] >= 0 ||
            m.ftex[0] >= 0 || m.ftex[1] >= 0)
            *feat |= FEAT_TEX;
    }
    // FEAT_BASIC (device.h): matte / plastic (and measured) materials only
    bool basic = (*feat & ~FEAT_MEAS) == 0;
    for (int i = 0; i < s->n_materials; ++i) {
        const int t = s->materials[i].type;
        basic = basic && (t == PBRTGPU_MAT_MATTE || t == PBRTGPU_MAT_PLASTIC ||
                          ((*feat & FEAT_MEAS) && (t == PBRTGPU_MAT_MEASURED || t == PBRTGPU_MAT_MEASURED_HALFANGLE)));
    }
    if (basic) *feat |= FEAT_BASIC;
    // FEAT_NOSPEC (device.h): otherwise matte / plastic / metal / substrate only, no measured BRDF
    bool nospec = !basic && (*feat & FEAT_MEAS) == 0;
    for (int i = 0; i < s->n_materials; ++i) {
        const int t = s->materials[i].type;
        nospec = nospec && (t == PBRTGPU_MAT_MATTE || t == PBRTGPU_MAT_PLASTIC || t == PBRTGPU_MAT_METAL ||
                            t == PBRTGPU_MAT_SUBSTRATE);
    }
    if (nospec) *feat |= FEAT_NOSPEC;
    return 0;
}

#undef SB_FAIL
#undef SB_PUT
}  // namespace pgd
