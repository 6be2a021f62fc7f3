// pack.cpp -- binary snapshot of a HostScene ("scene pack").  The GPU box receives only
// this repository, not the reference's scene files, so the flattened scenes built here
// by the front end travel as packs.  Format: magic, version, then fixed scalar header,
// camera block, and length-prefixed arrays in a fixed order.  Little-endian.
#include "scene.h"
#include <cstdio>
#include <cstring>

namespace pbrtamd {

static const char kMagic[8] = {'P', 'B', 'R', 'T', 'P', 'A', 'C', 'K'};
static const uint32_t kVersion = 1;

template <class T> static bool WArr(FILE *f, const std::vector<T> &v) {
    uint64_t n = v.size();
    if (fwrite(&n, 8, 1, f) != 1) return false;
    return n == 0 || fwrite(v.data(), sizeof(T), n, f) == n;
}
template <class T> static bool RArr(FILE *f, std::vector<T> &v) {
    uint64_t n;
    if (fread(&n, 8, 1, f) != 1) return false;
    if (n > (1ull << 34) / sizeof(T)) return false;
    v.resize(n);
    return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}

bool SavePack(const HostScene &s, const std::string &path, std::string *err) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { if (err) *err = "cannot write " + path; return false; }
    bool ok = fwrite(kMagic, 1, 8, f) == 8 && fwrite(&kVersion, 4, 1, f) == 1;
    int32_t hdr[4] = {s.nBands, s.maxDepth, s.spp, s.bvhMaxDepth};
    ok = ok && fwrite(hdr, 4, 4, f) == 4 && fwrite(&s.seed, 4, 1, f) == 1 && fwrite(&s.yint, 4, 1, f) == 1;
    ok = ok && fwrite(&s.camera, sizeof(s.camera), 1, f) == 1;
    ok = ok && WArr(f, s.bandY) && WArr(f, s.nodes) && WArr(f, s.prims) && WArr(f, s.tris) && WArr(f, s.meshes) &&
         WArr(f, s.vertP) && WArr(f, s.vertN) && WArr(f, s.vertUV) && WArr(f, s.quadrics) && WArr(f, s.materials) &&
         WArr(f, s.lights) && WArr(f, s.lightShapes) && WArr(f, s.spectra);
    fclose(f);
    if (!ok && err) *err = "write error on " + path;
    return ok;
}

bool LoadPack(const std::string &path, HostScene *s, std::string *err) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) { if (err) *err = "cannot open " + path; return false; }
    char magic[8];
    uint32_t ver = 0;
    bool ok = fread(magic, 1, 8, f) == 8 && memcmp(magic, kMagic, 8) == 0 && fread(&ver, 4, 1, f) == 1 && ver == kVersion;
    int32_t hdr[4];
    ok = ok && fread(hdr, 4, 4, f) == 4 && fread(&s->seed, 4, 1, f) == 1 && fread(&s->yint, 4, 1, f) == 1;
    if (ok) { s->nBands = hdr[0]; s->maxDepth = hdr[1]; s->spp = hdr[2]; s->bvhMaxDepth = hdr[3]; }
    ok = ok && fread(&s->camera, sizeof(s->camera), 1, f) == 1;
    ok = ok && RArr(f, s->bandY) && RArr(f, s->nodes) && RArr(f, s->prims) && RArr(f, s->tris) && RArr(f, s->meshes) &&
         RArr(f, s->vertP) && RArr(f, s->vertN) && RArr(f, s->vertUV) && RArr(f, s->quadrics) && RArr(f, s->materials) &&
         RArr(f, s->lights) && RArr(f, s->lightShapes) && RArr(f, s->spectra);
    fclose(f);
    if (!ok && err) *err = "bad or truncated scene pack " + path;
    return ok;
}

}  // namespace pbrtamd
