// capi.cpp -- C ABI of the host library (libpbrthost.so): scene loading (pbrt files or
// scene packs), flattening, and the reference's multispectral .dat writer.
// Declarations: include/pbrthost.h.
#include <sstream>
#include "pbrthost.h"
#include "scene.h"
#include <cstring>
#include <cstdio>
#include <vector>
#include <algorithm>

using namespace pbrtamd;

static void SetErr(char *err, int errlen, const std::string &msg) {
    if (err && errlen > 0) { strncpy(err, msg.c_str(), errlen - 1); err[errlen - 1] = 0; }
}

extern "C" {

int pbrthost_abi_version(void) { return PBRTHOST_ABI_VERSION; }

int pbrthost_load(const char *path, const pbrthost_overrides *ov, pbrthost_scene **out, char *err, int errlen) {
    if (!path || !out) { SetErr(err, errlen, "null argument"); return -1; }
    if (ov && ov->abi_version != PBRTHOST_ABI_VERSION) {
        SetErr(err, errlen, "pbrthost_overrides ABI version mismatch (caller built against another pbrthost.h)");
        return -1;
    }
    HostScene *s = new HostScene();
    std::string e, p(path);
    bool ok;
    if (p.size() > 5 && p.substr(p.size() - 5) == ".pack") ok = LoadPack(p, s, &e);
    else {
        RenderOverrides o;
        if (ov) {
            o.xres = ov->xres; o.yres = ov->yres; o.spp = ov->spp; o.maxdepth = ov->maxdepth;
            o.bands = ov->bands > 0 ? ov->bands : 32; o.seed = ov->seed;
            o.integrator = ov->integrator; o.dl_strategy = ov->dl_strategy; o.meta_strategy = ov->meta_strategy;
            o.renderer = ov->renderer; o.wave_bands = ov->wave_bands; o.spectral_sampling = ov->spectral_sampling;
        }
        ok = LoadPbrtScene(p, o, s, &e);
    }
    if (!ok) { delete s; SetErr(err, errlen, e); return -1; }
    // pack overrides that do not change geometry
    if (ov && p.size() > 5 && p.substr(p.size() - 5) == ".pack") {
        if (ov->xres > 0 || ov->yres > 0) {
            int xr = ov->xres > 0 ? ov->xres : s->camParams.xres, yr = ov->yres > 0 ? ov->yres : s->camParams.yres;
            ComputeCamera(s->camParams, xr, yr, &s->camera, s->cameraType);
        }
        if (ov->bands > 0 && ov->bands != s->nBands) { delete s; SetErr(err, errlen, "scene pack was built for a different band count"); return -1; }
        if (ov->spp > 0) { uint32_t v = ov->spp; v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; s->spp = v + 1; }
        if (ov->maxdepth >= 0) s->maxDepth = ov->maxdepth;
        if (ov->seed != PBRTHOST_KEEP_SEED) s->seed = ov->seed;
        if (ov->integrator >= 0) s->integrator = ov->integrator;
        if (ov->dl_strategy >= 0) s->dlStrategy = ov->dl_strategy;
        if (ov->meta_strategy >= 0) s->metaStrategy = ov->meta_strategy;
        if (ov->renderer >= 0) s->renderer = ov->renderer;
        if (ov->wave_bands > 0) s->waveBands = ov->wave_bands;
        if (ov->spectral_sampling >= 0) s->spectralSampling = ov->spectral_sampling;
    }
    *out = reinterpret_cast<pbrthost_scene *>(s);
    return 0;
}

int pbrthost_free(pbrthost_scene *h) { delete reinterpret_cast<HostScene *>(h); return 0; }

int pbrthost_flat(pbrthost_scene *h, pbrtgpu_flat_scene *out) {
    if (!h || !out) return -1;
    reinterpret_cast<HostScene *>(h)->Flat(out);
    return 0;
}

int pbrthost_save_pack(pbrthost_scene *h, const char *path, char *err, int errlen) {
    std::string e;
    if (!SavePack(*reinterpret_cast<HostScene *>(h), path, &e)) { SetErr(err, errlen, e); return -1; }
    return 0;
}

int pbrthost_set_render(pbrthost_scene *h, int spp, int maxdepth, uint32_t seed) {
    HostScene *s = reinterpret_cast<HostScene *>(h);
    if (spp > 0) { uint32_t v = spp; v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16; s->spp = v + 1; }
    if (maxdepth >= 0) s->maxDepth = maxdepth;
    s->seed = seed;
    return 0;
}

int pbrthost_info(pbrthost_scene *h, int64_t *info, int n) {
    HostScene *s = reinterpret_cast<HostScene *>(h);
    int64_t v[16] = {s->nBands, s->spp, s->maxDepth, (int64_t)s->nodes.size(), (int64_t)s->prims.size(),
                     (int64_t)s->tris.size(), (int64_t)s->meshes.size(), (int64_t)(s->vertP.size() / 3),
                     (int64_t)s->quadrics.size(), (int64_t)s->materials.size(), (int64_t)s->lights.size(),
                     s->bvhMaxDepth, s->camera.px_count, s->camera.py_count, (int64_t)s->warnings.size(), 0};
    for (int i = 0; i < n && i < 16; ++i) info[i] = v[i];
    return 0;
}

int pbrthost_write_metadata(pbrthost_scene *h, const char *image_file) {
    HostScene *s = reinterpret_cast<HostScene *>(h);
    if (!s || !image_file) return -1;
    // api.cpp:1235-1279: the output image name's stem + _mesh.txt / _materials.txt
    std::string fn(image_file);
    const std::string stem = fn.substr(0, fn.find_last_of("."));
    const std::vector<std::pair<uint32_t, std::string> > *list;
    std::string path;
    if (s->surfStrategy == "mesh") { list = &s->metaMesh; path = stem + "_mesh.txt"; }
    else if (s->surfStrategy == "material") { list = &s->metaMaterials; path = stem + "_materials.txt"; }
    else return 0;
    FILE *f = fopen(path.c_str(), "w");
    if (!f) return -1;
    for (auto &e : *list) fprintf(f, "%u %s\n", e.first, e.second.c_str());
    return fclose(f) == 0 ? 1 : -1;
}

// SpectralImageFilm::WriteImage (spectralImage.cpp:267-378), identity conversion matrix.
// film: [H][W][N] float32 raw sums; weight: [H][W] (filter weight sums, may be NULL = all 1).
// "focal fStop fov\n" with fov = 2 atan(sensorWidth / (2 focal)) / pi * 180 in the film's
// float / double mix, formatted by an ostream (default precision 6, "-nan" for the sign-set
// NaN x86 produces for 0 / 0)
static std::string dat_lens_line(float focal, float fStop, float sensorWidth) {
    volatile float den = 2 * focal;   // evaluated at run time, as in the reference
    const float fov = (float)(2 * atanf(sensorWidth / den) / 3.1415926539 * 180);
    std::ostringstream os;
    os << focal << " " << fStop << " " << fov << "\n";
    return os.str();
}

static int write_dat(const char *path, const float *film, const float *weight, int W, int H, int N,
                     const std::string &lensLine) {
    int nPix = W * H;
    std::vector<float> finalC((size_t)N * nPix);
    int offset = 0;
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) {
            for (int i = 0; i < N; ++i) finalC[(size_t)(y * W + x) * N + i] = film[((size_t)y * W + x) * N + i];
            float ws = weight ? weight[(size_t)y * W + x] : 1.f;
            if (ws != 0.f)
                for (int i = 0; i < N; ++i) finalC[(size_t)N * offset + i] = std::max(0.f, finalC[(size_t)N * offset + i]);
            for (int i = 0; i < N; ++i) finalC[(size_t)N * offset + i] += 1.f * 0.f;   // splatC[N] (pad) == 0
            ++offset;
        }
    std::vector<float> outv((size_t)N * nPix);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int row = 0; row < N; ++row) {
                float t = 0;
                for (int it = 0; it < N; ++it) t += (row == it ? 1.f : 0.f) * finalC[(size_t)N * (y * W + x) + it];
                outv[(size_t)N * (x * H + y) + row] = t;
            }
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "%d %d %d\n", W, H, N);
    // line 2: focalLength fStop fov as the film's ofstream formats them
    // (spectralImage.cpp:356-360).  CreateSpectralImageFilm leaves focal length, f-stop and
    // sensor width at 0 for every camera but RealisticDiffraction (:400-429), so the field
    // of view is 2 atan(0 / 0) ... = the x86 default NaN, printed "-nan"
    fputs(lensLine.c_str(), f);
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < nPix; ++j) { double r = outv[(size_t)N * j + i]; fwrite(&r, 8, 1, f); }
    fclose(f);
    return 0;
}

int pbrthost_write_dat(const char *path, const float *film, const float *weight, int W, int H, int N) {
    return write_dat(path, film, weight, W, H, N, dat_lens_line(0.f, 0.f, 0.f));
}

// the scene's film: its resolution and band count; line 2 from a RealisticDiffractionCamera's
// getFocalLength / getFStop / getSensorWidth (spectralImage.cpp:400-429, realisticDiffraction.cpp:
// 316-324, 470-476), zeros (and the NaN field of view) for every other camera
int pbrthost_write_dat_scene(const pbrthost_scene *h, const char *path, const float *film, const float *weight) {
    if (!h || !path || !film) return -1;
    const HostScene *s = reinterpret_cast<const HostScene *>(h);
    const int W = s->camera.px_count, H = s->camera.py_count;
    std::string line = dat_lens_line(0.f, 0.f, 0.f);
    if (s->cameraType == PBRTGPU_CAMERA_REALISTIC) {
        const float aspect = (float)s->camera.xres / (float)s->camera.yres;
        const float width = s->lens.film_diag / sqrtf((1.f + 1.f / (aspect * aspect)));
        line = dat_lens_line(s->lens.focal_length, s->lens.fstop, width);
    }
    return write_dat(path, film, weight, W, H, s->nBands, line);
}

int pbrthost_spectrum_from_rgb(int bands, const float rgb[3], int illuminant, float *out) {
    if (!rgb || !out || (bands != 32 && bands != 60 && bands != 30)) return -1;
    SpectrumCtx ctx(bands, bands == 30 ? 400 : 395, bands == 30 ? 700 : 715);
    Spec s = ctx.FromRGB(rgb, illuminant != 0);
    for (int i = 0; i < bands; ++i) out[i] = s[i];
    return 0;
}

}  // extern "C"
