// pack.cpp -- binary snapshot of a HostScene ("scene pack").  The GPU box receives only
// this repository, not the reference's scene files, so the flattened scenes built here
// by the front end travel as packs.  Format: magic, version, then fixed scalar header,
// camera block, and length-prefixed arrays in a fixed order.  Little-endian.
#include "scene.h"
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <string>
#include <zlib.h>

namespace pbrtamd {

static const char kMagic[8] = {'P', 'B', 'R', 'T', 'P', 'A', 'C', 'K'};
static const uint32_t kVersion = 16;   // 6: + merl tables; 7: + metadata ids; 8: + Renderer; 9: + lens diffraction;
                                       // 10: + pinhole array / microlens / eye IOR; 11: image maps as MIPMap
                                       // pyramids (texture records + texel pool); 12: material normal maps
                                       // (normal_tex, a former pad word: -1 for older packs); 13: an animated
                                       // camera's CameraToWorld; 14: textured float parameters (ftex, the
                                       // former pad words: -1 for older packs); 15: decoded environment maps
                                       // (light map_tex / dist_off, former pad words: -1); 16: the texture
                                       // record's size ahead of the texture array.  The record grew
                                       // within v15 (amount, aamode, mapping + map[16]: ABI 16), so a
                                       // v11-v15 pack holding textures has an unknown record layout and is
                                       // refused (re-pack it); without textures v5-v15 still load

static const uint32_t kTexRecord = (uint32_t)sizeof(pbrtgpu_texture);   // v16: written ahead of the textures

// the texture record of packs before v11: one MIPMap texel inline (the one-texel maps they held)
struct TexV10 {
    int32_t type, spectral, tex1, tex2, spec, wrap, trilinear;
    float value, texel[3], su, sv, du, dv, max_aniso;
};

static bool W(gzFile f, const void *p, size_t n) {
    const char *c = (const char *)p;
    while (n) { unsigned k = (unsigned)std::min<size_t>(n, 1u << 30); if (gzwrite(f, c, k) != (int)k) return false; c += k; n -= k; }
    return true;
}
static bool R(gzFile f, void *p, size_t n) {
    char *c = (char *)p;
    while (n) { unsigned k = (unsigned)std::min<size_t>(n, 1u << 30); if (gzread(f, c, k) != (int)k) return false; c += k; n -= k; }
    return true;
}
template <class T> static bool WArr(gzFile f, const std::vector<T> &v) {
    uint64_t n = v.size();
    return W(f, &n, 8) && (n == 0 || W(f, v.data(), sizeof(T) * n));
}
template <class T> static bool RArr(gzFile f, std::vector<T> &v) {
    uint64_t n;
    if (!R(f, &n, 8)) return false;
    if (n > (1ull << 34) / sizeof(T)) return false;
    v.resize(n);
    return n == 0 || R(f, v.data(), sizeof(T) * n);
}

static bool WStr(gzFile f, const std::string &v) {
    uint64_t n = v.size();
    return W(f, &n, 8) && (n == 0 || W(f, v.data(), n));
}
static bool RStr(gzFile f, std::string &v) {
    uint64_t n;
    if (!R(f, &n, 8) || n > (1u << 20)) return false;
    v.assign(n, '\0');
    return n == 0 || R(f, &v[0], n);
}
typedef std::vector<std::pair<uint32_t, std::string> > IdList;
static bool WList(gzFile f, const IdList &v) {
    uint64_t n = v.size();
    bool ok = W(f, &n, 8);
    for (size_t i = 0; ok && i < v.size(); ++i) ok = W(f, &v[i].first, 4) && WStr(f, v[i].second);
    return ok;
}
static bool RList(gzFile f, IdList &v) {
    uint64_t n;
    if (!R(f, &n, 8) || n > (1u << 26)) return false;
    v.resize(n);
    bool ok = true;
    for (size_t i = 0; ok && i < n; ++i) ok = R(f, &v[i].first, 4) && RStr(f, v[i].second);
    return ok;
}

bool SavePack(const HostScene &s, const std::string &path, std::string *err) {
    gzFile f = gzopen(path.c_str(), "wb6");
    if (!f) { if (err) *err = "cannot write " + path; return false; }
    bool ok = W(f, kMagic, 8) && W(f, &kVersion, 4);
    int32_t hdr[4] = {s.nBands, s.maxDepth, s.spp, s.bvhMaxDepth};
    ok = ok && W(f, hdr, 16) && W(f, &s.seed, 4) && W(f, &s.yint, 4);
    ok = ok && W(f, &s.camParams, sizeof(s.camParams)) && W(f, &s.camera, sizeof(s.camera));
    ok = ok && WArr(f, s.bandY) && WArr(f, s.nodes) && WArr(f, s.prims) && WArr(f, s.tris) && WArr(f, s.meshes) &&
         WArr(f, s.vertP) && WArr(f, s.vertN) && WArr(f, s.vertUV) && WArr(f, s.quadrics) && WArr(f, s.materials) &&
         WArr(f, s.lights) && WArr(f, s.lightShapes) && WArr(f, s.spectra) && WArr(f, s.instances) &&
         WArr(f, s.primInstance) && WArr(f, s.kdnodes) && W(f, &kTexRecord, 4) && WArr(f, s.textures) && WArr(f, s.ewaLut) &&
         WArr(f, s.rgbBasis) && WArr(f, s.merl);
    int32_t integ[2] = {s.integrator, s.dlStrategy};
    ok = ok && W(f, integ, 8);
    // v7: metadata strategy, per-prim ids, the metadata text lists
    int32_t ms = s.metaStrategy;
    ok = ok && W(f, &ms, 4) && WStr(f, s.surfStrategy) && WArr(f, s.primMeta) && WList(f, s.metaMesh) &&
         WList(f, s.metaMaterials);
    // v8: the Renderer
    int32_t rnd[3] = {s.renderer, s.waveBands, s.spectralSampling};
    ok = ok && W(f, rnd, 12);
    // v8: the camera type and RealisticDiffractionCamera
    int32_t ct = s.cameraType;
    ok = ok && W(f, &ct, 4) && W(f, &s.lens, sizeof(s.lens)) && WArr(f, s.lensEl);
    // v10: the eye IOR spectra (the pinhole array is derived at the film resolution, Flat)
    ok = ok && WArr(f, s.eyeIor);
    // v11: the texel pool of the MIPMap pyramids
    ok = ok && WArr(f, s.texels);
    // v13: the animated camera
    ok = ok && WArr(f, s.cameraMotion);
    ok = (gzclose(f) == Z_OK) && ok;
    if (!ok && err) *err = "write error on " + path;
    return ok;
}

bool LoadPack(const std::string &path, HostScene *s, std::string *err) {
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) { if (err) *err = "cannot open " + path; return false; }
    char magic[8];
    uint32_t ver = 0;
    bool ok = R(f, magic, 8) && memcmp(magic, kMagic, 8) == 0 && R(f, &ver, 4) && ver >= 5 && ver <= kVersion;
    int32_t hdr[4];
    ok = ok && R(f, hdr, 16) && R(f, &s->seed, 4) && R(f, &s->yint, 4);
    if (ok) { s->nBands = hdr[0]; s->maxDepth = hdr[1]; s->spp = hdr[2]; s->bvhMaxDepth = hdr[3]; }
    ok = ok && R(f, &s->camParams, sizeof(s->camParams)) && R(f, &s->camera, sizeof(s->camera));
    ok = ok && RArr(f, s->bandY) && RArr(f, s->nodes) && RArr(f, s->prims) && RArr(f, s->tris) && RArr(f, s->meshes) &&
         RArr(f, s->vertP) && RArr(f, s->vertN) && RArr(f, s->vertUV) && RArr(f, s->quadrics) && RArr(f, s->materials) &&
         RArr(f, s->lights) && RArr(f, s->lightShapes) && RArr(f, s->spectra) && RArr(f, s->instances) &&
         RArr(f, s->primInstance) && RArr(f, s->kdnodes);
    std::vector<TexV10> oldTex;
    bool texLayout = true;
    if (ok && ver >= 16) {
        uint32_t rec = 0;
        ok = R(f, &rec, 4);
        texLayout = rec == kTexRecord;
    } else if (ok && ver >= 11) {   // v11-v15: the record's layout is not recorded; only an empty array is safe
        uint64_t n = 0;
        ok = R(f, &n, 8);
        texLayout = n == 0;
        s->textures.clear();
    }
    if (ok && !texLayout) {
        gzclose(f);
        if (err)
            *err = "scene pack " + path + " holds texture records of another layout (pack version " + std::to_string(ver) +
                   "; this build reads v16 records of " + std::to_string(kTexRecord) + " bytes): re-pack the scene";
        return false;
    }
    ok = ok && (ver >= 16 ? RArr(f, s->textures) : ver >= 11 ? true : RArr(f, oldTex));
    ok = ok && RArr(f, s->ewaLut) && RArr(f, s->rgbBasis);
    s->texels.clear();
    if (ok && ver < 11) {   // each one-texel map becomes a 1x1 pyramid in the texel pool
        s->textures.resize(oldTex.size());
        for (size_t i = 0; i < oldTex.size(); ++i) {
            const TexV10 &o = oldTex[i];
            pbrtgpu_texture &t = s->textures[i];
            memset(&t, 0, sizeof(t));
            t.type = o.type; t.spectral = o.spectral; t.tex1 = o.tex1; t.tex2 = o.tex2; t.spec = o.spec; t.wrap = o.wrap;
            t.trilinear = o.trilinear; t.value = o.value; t.su = o.su; t.sv = o.sv; t.du = o.du; t.dv = o.dv;
            t.max_aniso = o.max_aniso;
            if (t.type == PBRTGPU_TEX_IMAGE) {
                t.texel_off = (int32_t)s->texels.size();
                t.width = t.height = t.levels = 1;
                for (int k = 0; k < (o.spectral ? 3 : 1); ++k) s->texels.push_back(o.texel[k]);
            }
        }
    }
    s->merl.clear();
    s->integrator = 0;   // packs before v6: the configs' "path" 
    s->dlStrategy = 0;
    if (ok && ver >= 6) {
        int32_t integ[2];
        ok = RArr(f, s->merl) && R(f, integ, 8);
        if (ok) { s->integrator = integ[0]; s->dlStrategy = integ[1]; }
    }
    s->metaStrategy = PBRTGPU_META_DEPTH;
    s->surfStrategy.clear();
    s->primMeta.clear(); s->metaMesh.clear(); s->metaMaterials.clear();
    if (ok && ver >= 7) {
        int32_t ms;
        ok = R(f, &ms, 4) && RStr(f, s->surfStrategy) && RArr(f, s->primMeta) && RList(f, s->metaMesh) &&
             RList(f, s->metaMaterials);
        if (ok) s->metaStrategy = ms;
    }
    s->renderer = PBRTGPU_RENDERER_SAMPLER;
    s->cameraType = PBRTGPU_CAMERA_PERSPECTIVE;
    memset(&s->lens, 0, sizeof(s->lens));
    s->lensEl.clear();
    s->waveBands = 32;
    s->spectralSampling = PBRTGPU_SPECTRAL_SINGLE;
    if (ok && ver >= 8) {
        int32_t rnd[3];
        ok = R(f, rnd, 12);
        if (ok) { s->renderer = rnd[0]; s->waveBands = rnd[1]; s->spectralSampling = rnd[2]; }
        int32_t ct = 0;
        // v8's pbrtgpu_lens ended at fstop (56 bytes) + the elements pointer; v9's at the elements
        // pointer (72 bytes)
        const size_t lensBytes = ver >= 10 ? sizeof(s->lens) : ver >= 9 ? 72 : 64;
        char lensBuf[sizeof(s->lens) > 72 ? sizeof(s->lens) : 72];
        ok = ok && R(f, &ct, 4) && R(f, lensBuf, (unsigned)lensBytes) && RArr(f, s->lensEl);
        memcpy(&s->lens, lensBuf, ver >= 10 ? sizeof(s->lens) : ver >= 9 ? 64 : 56);
        if (ok) s->cameraType = ct;
        s->lens.elements = nullptr;
        s->lens.pinholes = nullptr;
        s->lens.eye_ior = nullptr;
    }
    s->eyeIor.clear();
    if (ok && ver >= 10) ok = RArr(f, s->eyeIor);
    if (ok && ver >= 11) ok = RArr(f, s->texels);
    if (ok && ver < 12)
        for (auto &m : s->materials) m.normal_tex = -1;
    if (ok && ver < 14)
        for (auto &m : s->materials) m.ftex[0] = m.ftex[1] = -1;
    if (ok && ver < 15)
        for (auto &l : s->lights) { l.map_tex = -1; l.dist_off = -1; l.dist_nu = l.dist_nv = 1; }
    s->cameraMotion.clear();
    if (ok && ver >= 13) ok = RArr(f, s->cameraMotion) && s->cameraMotion.size() <= 1;
    gzclose(f);
    if (!ok && err) *err = "bad or truncated scene pack " + path;
    return ok;
}

}  // namespace pbrtamd
