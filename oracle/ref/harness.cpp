// oracle/ref/harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Drives the reference's own hot-path translation units (compiled unmodified from
// /root/reference/src by oracle/ref/Makefile) to produce golden vectors for the
// fixed-seed parity scheme described in DESIGN.md §3.
//
// What the reference would normally provide but cannot be compiled in this image:
//   * core/api.cpp        -- includes the GSL-dependent lens-camera headers
//                            (cameras/realisticDiffraction.h et al.); GSL is absent.
//   * core/parallel.cpp   -- includes <sys/sysctl.h>, absent from glibc 2.35.
//   * film/spectralImage.cpp -- includes cameras/realisticDiffraction.h (GSL).
//   * renderers/samplerrenderer.cpp -- needs parallel.cpp's task queue.
// This file therefore plays the part of the *application*: it implements the
// pbrt* scene-API entry points the reference parser calls (restating the subset of
// api.cpp:733-1330 the config scenes use, calling the reference factories
// Create*Shape/Material/Light/Texture, CreateBVHAccelerator, CreatePerspectiveCamera,
// CreatePathSurfaceIntegrator), a box-filter film restating
// SpectralImageFilm::AddSample/WriteImage (spectralImage.cpp:77-152, 267-378), and the
// render loop of SamplerRendererTask::Run (samplerrenderer.cpp:60-164) with the
// build's fixed per-path seeding instead of per-task RNG streams.
// No header or library is stubbed: everything it links is reference code or this file.
//
// --refdat additionally feeds every sample to the reference's own SpectralImageNoCameraFilm
// (film/spectralImageNoCamera.cpp, which builds here: it does not include the lens-camera
// headers).  Its AddSample c[] accumulation (:36-75 of that file) and WriteImage payload
// (clamp-index quirk, splat pad, identity conversion matrix, x-major band planes as float64)
// are those of SpectralImageFilm (spectralImage.cpp:77-152, 267-378); it writes header line
// 1 only (no "focal fStop fov" line) and attempts a _depth.exr side image, which this
// OpenEXR-less build cannot write.  So the .dat it writes pins the payload and line 1 of the
// spectral film's .dat with reference code.
// --keys traces an explicit (x, y, s) key list (int32 triples) at the scene's full
// resolution and sample count -- the configs' real spp -- without a film.

#include "stdafx.h"
#include "pbrt.h"
#include "api.h"
#include "parser.h"
#include "paramset.h"
#include "spectrum.h"
#include "scene.h"
#include "film.h"
#include "camera.h"
#include "sampler.h"
#include "integrator.h"
#include "intersection.h"
#include "primitive.h"
#include "light.h"
#include "renderer.h"
#include "volume.h"
#include "texture.h"
#include "montecarlo.h"
#include "reflection.h"
#include "accelerators/bvh.h"
#include "cameras/perspective.h"
#include "cameras/orthographic.h"
#include "filters/box.h"
#ifndef HARNESS_RGB
#include "film/spectralImageNoCamera.h"
#endif
#ifdef HARNESS_GPUPATH
#include "gpupathrenderer.h"   // integration/: the reference-side binding of the MI355X core
#endif
#include "integrators/path.h"
#include "integrators/directlighting.h"
#include "integrators/metadata.h"
#include "samplers/lowdiscrepancy.h"
#include "integrators/emission.h"
#include "lights/diffuse.h"
#include "lights/point.h"
#include "lights/infinite.h"
#include "lights/spot.h"
#include "lights/distant.h"
#include "materials/matte.h"
#include "materials/plastic.h"
#include "materials/anisoward.h"
#include "materials/shinymetal.h"
#include "materials/metal.h"
#include "materials/substrate.h"
#include "materials/measured.h"
#include "materials/mirror.h"
#include "materials/glass.h"
#include "shapes/sphere.h"
#include "shapes/heightfield.h"
#include "shapes/cylinder.h"
#include "shapes/nurbs.h"
// output channels of a radiance: the spectrum's bands, or RGB in the C1 build (HARNESS_RGB:
// Spectrum = RGBSpectrum, pbrt.h:144)
#ifdef HARNESS_RGB
static const int NOUT = 3;
static inline void spec_out(const Spectrum &L, float *c) { L.ToRGB(c); }
#else
static const int NOUT = nSpectralSamples;
static inline void spec_out(const Spectrum &L, float *c) { L.GetOrigC(c); }
#endif
#include "shapes/disk.h"
#include "shapes/trianglemesh.h"
#include "shapes/loopsubdiv.h"
#include "textures/constant.h"
#include "textures/imagemap.h"
#include "textures/checkerboard.h"
#include "textures/uv.h"
#include "textures/mix.h"
#include "textures/bilerp.h"
#include "textures/fbm.h"
#include "textures/wrinkled.h"
#include "textures/windy.h"
#include "textures/dots.h"
#include "textures/marble.h"
#include "textures/scale.h"

#include <map>
#include <vector>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <cstring>

Options PbrtOptions;   // normally defined by api.cpp:154; the application owns it here
// Terminal query used by error.cpp:64 for message wrapping; its home TU
// (progressreporter.cpp:110) needs parallel.cpp's Mutex.  The harness is non-interactive.
int TerminalWidth() { return 80; }

// ---------------------------------------------------------------------------------
// Fixed-seed sampler.  Integer-only; identical definition in
// oracle/pathtrace.c and pbrt-v2-spectral_amd/csrc/sampler.h.
// ---------------------------------------------------------------------------------
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
static float sample1D(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp) {
    return VanDerCorput(perm_index(hp, d, s, spp), dim_scramble(hp, d));
}
static void sample2D(uint32_t hp, uint32_t d, uint32_t s, uint32_t spp, float *u) {
    uint32_t sp = perm_index(hp, d, s, spp);
    uint32_t sc = dim_scramble(hp, d);
    u[0] = VanDerCorput(sp, sc);
    u[1] = Sobol2(sp, mix32(sc ^ 0x68BC21EBU));
}
// dimension ids: 0 image(2D) 1 lens(2D) 2 time(1D) 3+j 1-D slot j, 3+n1D+k 2-D slot k
static void FillSample(Sample *smp, int px, int py, uint32_t s, uint32_t spp, uint32_t seed,
                       float shutterOpen, float shutterClose) {
    uint32_t hp = pixel_hash(seed, px, py);
    float u[2];
    sample2D(hp, 0, s, spp, u);
    smp->imageX = px + u[0];
    smp->imageY = py + u[1];
    sample2D(hp, 1, s, spp, u);
    smp->lensU = u[0]; smp->lensV = u[1];
    smp->time = Lerp(sample1D(hp, 2, s, spp), shutterOpen, shutterClose);
    uint32_t n1 = smp->n1D.size(), n2 = smp->n2D.size();
    // a slot requested with count n (DirectLighting "all": a light's nSamples, rounded to a
    // power of two by LDSampler::RoundSize) holds the n values of sample index s * n + k of
    // the same dimension's sequence of length spp * n; with n == 1 that is (s, spp)
    for (uint32_t j = 0; j < n1; ++j)
        for (uint32_t k = 0; k < smp->n1D[j]; ++k)
            smp->oneD[j][k] = sample1D(hp, 3 + j, s * smp->n1D[j] + k, spp * smp->n1D[j]);
    for (uint32_t j = 0; j < n2; ++j)
        for (uint32_t k = 0; k < smp->n2D[j]; ++k)
            sample2D(hp, 3 + n1 + j, s * smp->n2D[j] + k, spp * smp->n2D[j], &smp->twoD[j][2 * k]);
}

// ---------------------------------------------------------------------------------
// Film: box-filter restatement of SpectralImageFilm (spectralImage.cpp:40-185,267-378)
// ---------------------------------------------------------------------------------
class HarnessFilm : public Film {
public:
    HarnessFilm(int xres, int yres, Filter *filt, const float crop[4], const string &fn)
        : Film(xres, yres, fn), filter(filt) {
        memcpy(cropWindow, crop, 4 * sizeof(float));
        xPixelStart = Ceil2Int(xResolution * cropWindow[0]);
        xPixelCount = max(1, Ceil2Int(xResolution * cropWindow[1]) - xPixelStart);
        yPixelStart = Ceil2Int(yResolution * cropWindow[2]);
        yPixelCount = max(1, Ceil2Int(yResolution * cropWindow[3]) - yPixelStart);
        c.assign((size_t)xPixelCount * yPixelCount * NOUT, 0.f);
        wsum.assign((size_t)xPixelCount * yPixelCount, 0.f);
        for (int y = 0; y < 16; ++y) {
            float fy = ((float)y + .5f) * filter->yWidth / 16;
            for (int x = 0; x < 16; ++x) {
                float fx = ((float)x + .5f) * filter->xWidth / 16;
                table[y * 16 + x] = filter->Evaluate(fx, fy);
            }
        }
    }
    void AddSample(const CameraSample &sample, const Spectrum &L, const Ray &) {
        float dimageX = sample.imageX - 0.5f;
        float dimageY = sample.imageY - 0.5f;
        int x0 = Ceil2Int(dimageX - filter->xWidth);
        int x1 = Floor2Int(dimageX + filter->xWidth);
        int y0 = Ceil2Int(dimageY - filter->yWidth);
        int y1 = Floor2Int(dimageY + filter->yWidth);
        x0 = max(x0, xPixelStart); x1 = min(x1, xPixelStart + xPixelCount - 1);
        y0 = max(y0, yPixelStart); y1 = min(y1, yPixelStart + yPixelCount - 1);
        if ((x1 - x0) < 0 || (y1 - y0) < 0) return;
        float origC[NOUT];
        spec_out(L, origC);
        for (int y = y0; y <= y1; ++y) {
            float fy = fabsf((y - dimageY) * filter->invYWidth * 16);
            int iy = min(Floor2Int(fy), 15);
            for (int x = x0; x <= x1; ++x) {
                float fx = fabsf((x - dimageX) * filter->invXWidth * 16);
                int ix = min(Floor2Int(fx), 15);
                float w = table[iy * 16 + ix];
                size_t pix = (size_t)(y - yPixelStart) * xPixelCount + (x - xPixelStart);
                for (int i = 0; i < NOUT; ++i) c[pix * NOUT + i] += w * origC[i];
                wsum[pix] += w;
            }
        }
    }
    void Splat(const CameraSample &, const Spectrum &) {}
    void GetSampleExtent(int *xs, int *xe, int *ys, int *ye) const {
        *xs = Floor2Int(xPixelStart + 0.5f - filter->xWidth);
        *xe = Floor2Int(xPixelStart + 0.5f + xPixelCount + filter->xWidth);
        *ys = Floor2Int(yPixelStart + 0.5f - filter->yWidth);
        *ye = Floor2Int(yPixelStart + 0.5f + yPixelCount + filter->yWidth);
    }
    void GetPixelExtent(int *xs, int *xe, int *ys, int *ye) const {
        *xs = xPixelStart; *xe = xPixelStart + xPixelCount;
        *ys = yPixelStart; *ye = yPixelStart + yPixelCount;
    }
    void WriteImage(float) {}
    // raw accumulator, [y][x][band] float32
    void WriteRaw(const char *fn) const {
        FILE *f = fopen(fn, "wb");
        int hdr[3] = { xPixelCount, yPixelCount, NOUT };
        fwrite(hdr, sizeof(int), 3, f);
        fwrite(&c[0], sizeof(float), c.size(), f);
        fclose(f);
    }
    // .dat exactly as SpectralImageFilm::WriteImage (identity conversion matrix)
    void WriteDat(const char *fn) const {
        int W = xPixelCount, H = yPixelCount, N = NOUT, nPix = W * H;
        std::vector<float> finalC((size_t)N * nPix);
        int offset = 0;
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < H; ++y) {
                for (int i = 0; i < N; ++i)
                    finalC[(size_t)(y * W + x) * N + i] = c[((size_t)y * W + x) * N + i];
                if (wsum[(size_t)y * W + x] != 0.f)
                    for (int i = 0; i < N; ++i)
                        finalC[(size_t)N * offset + i] = max(0.f, finalC[(size_t)N * offset + i]);
                for (int i = 0; i < N; ++i) finalC[(size_t)N * offset + i] += 1.f * 0.f;   // splatC[N] reads pad (0)
                ++offset;
            }
        std::vector<float> out((size_t)N * nPix);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x)
                for (int row = 0; row < N; ++row) {
                    float t = 0;
                    for (int it = 0; it < N; ++it)
                        t += (row == it ? 1.f : 0.f) * finalC[(size_t)N * (y * W + x) + it];
                    out[(size_t)N * (x * H + y) + row] = t;
                }
        FILE *f = fopen(fn, "w");
        fprintf(f, "%d %d %d\n", W, H, N);
        fprintf(f, "0 0 0\n");
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < nPix; ++j) { double r = out[(size_t)N * j + i]; fwrite(&r, 8, 1, f); }
        fclose(f);
    }
    Filter *filter;
    float cropWindow[4];
    int xPixelStart, yPixelStart, xPixelCount, yPixelCount;
    std::vector<float> c, wsum;
    float table[256];
};

// ---------------------------------------------------------------------------------
// Renderer: SamplerRenderer::Li / Transmittance semantics (samplerrenderer.cpp:225-257)
// ---------------------------------------------------------------------------------
class HarnessRenderer : public Renderer {
public:
    HarnessRenderer(SurfaceIntegrator *s, VolumeIntegrator *v) : surf(s), vol(v) {}
    void Render(const Scene *) {}
    Spectrum Li(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                MemoryArena &arena, Intersection *isect = NULL, Spectrum *T = NULL) const {
        Spectrum localT;
        if (!T) T = &localT;
        Intersection localIsect;
        if (!isect) isect = &localIsect;
        Spectrum Li = 0.f;
        if (scene->Intersect(ray, isect))
            Li = surf->Li(scene, this, ray, *isect, sample, rng, arena);
        else
            for (uint32_t i = 0; i < scene->lights.size(); ++i) Li += scene->lights[i]->Le(ray);
        Spectrum Lvi = vol->Li(scene, this, ray, sample, rng, T, arena);
        return *T * Li + Lvi;
    }
    Spectrum Transmittance(const Scene *scene, const RayDifferential &ray, const Sample *sample,
                           RNG &rng, MemoryArena &arena) const {
        return vol->Transmittance(scene, this, ray, sample, rng, arena);
    }
    SurfaceIntegrator *surf;
    VolumeIntegrator *vol;
};

// ---------------------------------------------------------------------------------
// Scene API: restatement of the api.cpp subset (api.cpp:146-330, 733-1330)
// ---------------------------------------------------------------------------------
#define MAX_TRANSFORMS 2
#define START_TRANSFORM_BITS (1 << 0)
#define END_TRANSFORM_BITS (1 << 1)
#define ALL_TRANSFORMS_BITS ((1 << MAX_TRANSFORMS) - 1)
struct TransformSet {
    Transform t[MAX_TRANSFORMS];
    Transform &operator[](int i) { return t[i]; }
    const Transform &operator[](int i) const { return t[i]; }
    bool IsAnimated() const { return t[0] != t[1]; }
};
static TransformSet Inv(const TransformSet &ts) {
    TransformSet r; for (int i = 0; i < MAX_TRANSFORMS; ++i) r.t[i] = Inverse(ts.t[i]); return r;
}
struct GState {
    std::map<string, Reference<Texture<float> > > floatTextures;
    std::map<string, Reference<Texture<Spectrum> > > spectrumTextures;
    ParamSet materialParams;
    string material = "matte";
    std::map<string, Reference<Material> > namedMaterials;
    string currentNamedMaterial;
    ParamSet areaLightParams;
    string areaLight;
    bool reverseOrientation = false;
};
struct TCache {
    std::map<Transform, std::pair<Transform *, Transform *> > cache;
    void Lookup(const Transform &t, Transform **tc, Transform **tci) {
        auto it = cache.find(t);
        if (it == cache.end()) {
            Transform *tr = new Transform(t);
            Transform *ti = new Transform(Inverse(t));
            cache[t] = std::make_pair(tr, ti);
            it = cache.find(t);
        }
        if (tc) *tc = it->second.first;
        if (tci) *tci = it->second.second;
    }
};
static TransformSet curT;
static int activeBits = ALL_TRANSFORMS_BITS;
static std::map<string, TransformSet> namedCS;
static GState gs;
static std::vector<GState> pushedGS;
static std::vector<TransformSet> pushedT;
static std::vector<int> pushedBits;
static TCache tcache;
static float tStart = 0.f, tEnd = 1.f;
static ParamSet filmParams, cameraParams, samplerParams, surfParams, accelParams, filterParams;
static string cameraName = "perspective", surfName = "directlighting";
static TransformSet cameraToWorld;
static std::vector<Light *> lights;
static std::vector<Reference<Primitive> > primitives;
// overrides from the command line
static int ovW = -1, ovH = -1, ovMaxDepth = -1;
static const char *surfOv = "path";   // --surf: the SurfaceIntegrator to create
static const char *dlStrategyOv = NULL;
static const char *metaStrategyOv = NULL;   // --meta-strategy: MetadataIntegrator "strategy" 
// --spectral N [single|sampler]: Renderer "spectralrenderer" with nWaveBands N and samplingMethod
// singleDirection / samplerDirection (api.cpp:1377-1403)
static int specBands = 0;
static bool specSampler = false;
// results of WorldEnd
static Scene *gScene = NULL;
static Camera *gCamera = NULL;
static HarnessFilm *gFilm = NULL;
static Film *gCameraFilm = NULL;   // --gpupath with --refdat: the camera's film is the reference's own
static Filter *gFilter = NULL;
static SurfaceIntegrator *gSurf = NULL;
static VolumeIntegrator *gVol = NULL;
static int gSppParam = 4;

#define FOR_ACTIVE(expr) for (int i = 0; i < MAX_TRANSFORMS; ++i) if (activeBits & (1 << i)) { expr }

void pbrtInit(const Options &opt) { PbrtOptions = opt; SampledSpectrum::Init(); }
void pbrtCleanup() {}
void pbrtIdentity() { FOR_ACTIVE(curT[i] = Transform();) }
void pbrtTranslate(float dx, float dy, float dz) { FOR_ACTIVE(curT[i] = curT[i] * Translate(Vector(dx, dy, dz));) }
void pbrtTransform(float tr[16]) {
    FOR_ACTIVE(curT[i] = Transform(Matrix4x4(tr[0], tr[4], tr[8], tr[12], tr[1], tr[5], tr[9], tr[13],
                                             tr[2], tr[6], tr[10], tr[14], tr[3], tr[7], tr[11], tr[15]));)
}
void pbrtConcatTransform(float tr[16]) {
    FOR_ACTIVE(curT[i] = curT[i] * Transform(Matrix4x4(tr[0], tr[4], tr[8], tr[12], tr[1], tr[5], tr[9], tr[13],
                                                       tr[2], tr[6], tr[10], tr[14], tr[3], tr[7], tr[11], tr[15]));)
}
void pbrtRotate(float a, float dx, float dy, float dz) { FOR_ACTIVE(curT[i] = curT[i] * Rotate(a, Vector(dx, dy, dz));) }
void pbrtScale(float sx, float sy, float sz) { FOR_ACTIVE(curT[i] = curT[i] * Scale(sx, sy, sz);) }
void pbrtLookAt(float ex, float ey, float ez, float lx, float ly, float lz, float ux, float uy, float uz) {
    FOR_ACTIVE(curT[i] = curT[i] * LookAt(Point(ex, ey, ez), Point(lx, ly, lz), Vector(ux, uy, uz));)
}
void pbrtCoordinateSystem(const string &n) { namedCS[n] = curT; }
void pbrtCoordSysTransform(const string &n) { if (namedCS.count(n)) curT = namedCS[n]; }
void pbrtActiveTransformAll() { activeBits = ALL_TRANSFORMS_BITS; }
void pbrtActiveTransformEndTime() { activeBits = END_TRANSFORM_BITS; }
void pbrtActiveTransformStartTime() { activeBits = START_TRANSFORM_BITS; }
void pbrtTransformTimes(float s, float e) { tStart = s; tEnd = e; }
void pbrtPixelFilter(const string &, const ParamSet &) {}   // api.cpp:858 stores only the name (box)
void pbrtFilm(const string &, const ParamSet &p) { filmParams = p; }
void pbrtSampler(const string &, const ParamSet &p) { samplerParams = p; }
void pbrtAccelerator(const string &, const ParamSet &p) { accelParams = p; }
void pbrtSurfaceIntegrator(const string &n, const ParamSet &p) { surfName = n; surfParams = p; }
void pbrtVolumeIntegrator(const string &, const ParamSet &) {}
void pbrtRenderer(const string &, const ParamSet &) {}
void pbrtCamera(const string &n, const ParamSet &p) {
    cameraName = n; cameraParams = p; cameraToWorld = Inv(curT); namedCS["camera"] = cameraToWorld;
}
void pbrtWorldBegin() {
    for (int i = 0; i < MAX_TRANSFORMS; ++i) curT[i] = Transform();
    activeBits = ALL_TRANSFORMS_BITS;
    namedCS["world"] = curT;
}
void pbrtAttributeBegin() { pushedGS.push_back(gs); pushedT.push_back(curT); pushedBits.push_back(activeBits); }
void pbrtAttributeEnd() {
    if (pushedGS.empty()) return;
    gs = pushedGS.back(); pushedGS.pop_back();
    curT = pushedT.back(); pushedT.pop_back();
    activeBits = pushedBits.back(); pushedBits.pop_back();
}
void pbrtTransformBegin() { pushedT.push_back(curT); pushedBits.push_back(activeBits); }
void pbrtTransformEnd() {
    if (pushedT.empty()) return;
    curT = pushedT.back(); pushedT.pop_back();
    activeBits = pushedBits.back(); pushedBits.pop_back();
}
static Reference<Texture<float> > MakeFloatTex(const string &n, const Transform &x, const TextureParams &tp) {
    if (n == "constant") return CreateConstantFloatTexture(x, tp);
    if (n == "scale") return CreateScaleFloatTexture(x, tp);
    if (n == "imagemap") return CreateImageFloatTexture(x, tp);
    if (n == "checkerboard") return CreateCheckerboardFloatTexture(x, tp);
    if (n == "mix") return CreateMixFloatTexture(x, tp);
    if (n == "bilerp") return CreateBilerpFloatTexture(x, tp);
    if (n == "fbm") return CreateFBmFloatTexture(x, tp);
    if (n == "wrinkled") return CreateWrinkledFloatTexture(x, tp);
    if (n == "windy") return CreateWindyFloatTexture(x, tp);
    if (n == "dots") return CreateDotsFloatTexture(x, tp);
    fprintf(stderr, "harness: float texture %s unsupported\n", n.c_str()); exit(2);
}
static Reference<Texture<Spectrum> > MakeSpecTex(const string &n, const Transform &x, const TextureParams &tp) {
    if (n == "constant") return CreateConstantSpectrumTexture(x, tp);
    if (n == "scale") return CreateScaleSpectrumTexture(x, tp);
    if (n == "imagemap") return CreateImageSpectrumTexture(x, tp);
    if (n == "checkerboard") return CreateCheckerboardSpectrumTexture(x, tp);
    if (n == "uv") return CreateUVSpectrumTexture(x, tp);
    if (n == "mix") return CreateMixSpectrumTexture(x, tp);
    if (n == "bilerp") return CreateBilerpSpectrumTexture(x, tp);
    if (n == "dots") return CreateDotsSpectrumTexture(x, tp);
    if (n == "marble") return CreateMarbleSpectrumTexture(x, tp);
    if (n == "fbm") return CreateFBmSpectrumTexture(x, tp);
    if (n == "wrinkled") return CreateWrinkledSpectrumTexture(x, tp);
    if (n == "windy") return CreateWindySpectrumTexture(x, tp);
    fprintf(stderr, "harness: spectrum texture %s unsupported\n", n.c_str()); exit(2);
}
void pbrtTexture(const string &name, const string &type, const string &texname, const ParamSet &params) {
    TextureParams tp(params, params, gs.floatTextures, gs.spectrumTextures);
    if (type == "float") gs.floatTextures[name] = MakeFloatTex(texname, curT[0], tp);
    else gs.spectrumTextures[name] = MakeSpecTex(texname, curT[0], tp);
}
static Reference<Material> MakeMat(const string &n, const Transform &x, const TextureParams &mp) {
    if (n == "matte") return CreateMatteMaterial(x, mp);
    if (n == "plastic") return CreatePlasticMaterial(x, mp);
    if (n == "metal") return CreateMetalMaterial(x, mp);
    if (n == "substrate") return CreateSubstrateMaterial(x, mp);
    if (n == "anisoward") return CreateAnisoWardMaterial(x, mp);
    if (n == "shinymetal") return CreateShinyMetalMaterial(x, mp);
    if (n == "measured") return CreateMeasuredMaterial(x, mp);
    if (n == "mirror") return CreateMirrorMaterial(x, mp);
    if (n == "glass") return CreateGlassMaterial(x, mp);
    fprintf(stderr, "harness: material %s unsupported\n", n.c_str()); exit(2);
}
void pbrtMaterial(const string &n, const ParamSet &p) { gs.material = n; gs.materialParams = p; gs.currentNamedMaterial = ""; }
void pbrtMakeNamedMaterial(const string &name, const ParamSet &params) {
    TextureParams mp(params, gs.materialParams, gs.floatTextures, gs.spectrumTextures);
    string mn = mp.FindString("type");
    if (mn != "") gs.namedMaterials[name] = MakeMat(mn, curT[0], mp);
}
void pbrtNamedMaterial(const string &n) { gs.currentNamedMaterial = n; }
void pbrtLightSource(const string &n, const ParamSet &p) {
    Light *lt = NULL;
    if (n == "point") lt = CreatePointLight(curT[0], p);
    else if (n == "infinite" || n == "exinfinite") lt = CreateInfiniteLight(curT[0], p);
    else if (n == "spot") lt = CreateSpotLight(curT[0], p);
    else if (n == "distant") lt = CreateDistantLight(curT[0], p);
    else { fprintf(stderr, "harness: light %s unsupported\n", n.c_str()); exit(2); }
    lights.push_back(lt);
}
void pbrtAreaLightSource(const string &n, const ParamSet &p) { gs.areaLight = n; gs.areaLightParams = p; }
static Reference<Shape> MakeShp(const string &n, const Transform *o2w, const Transform *w2o, bool ro,
                                const ParamSet &p) {
    if (n == "sphere") return CreateSphereShape(o2w, w2o, ro, p);
    if (n == "disk") return CreateDiskShape(o2w, w2o, ro, p);
    if (n == "trianglemesh") return CreateTriangleMeshShape(o2w, w2o, ro, p, &gs.floatTextures);
    if (n == "loopsubdiv") return CreateLoopSubdivShape(o2w, w2o, ro, p);
    if (n == "heightfield") return CreateHeightfieldShape(o2w, w2o, ro, p);
    if (n == "cylinder") return CreateCylinderShape(o2w, w2o, ro, p);
    if (n == "nurbs") return CreateNURBSShape(o2w, w2o, ro, p);
    fprintf(stderr, "harness: shape %s unsupported\n", n.c_str()); exit(2);
}
static Reference<Material> CreateMaterialFromState(const ParamSet &params) {
    TextureParams mp(params, gs.materialParams, gs.floatTextures, gs.spectrumTextures);
    Reference<Material> m;
    if (gs.currentNamedMaterial != "" && gs.namedMaterials.count(gs.currentNamedMaterial))
        m = gs.namedMaterials[gs.currentNamedMaterial];
    if (!m) m = MakeMat(gs.material, curT[0], mp);
    return m;
}
void pbrtShape(const string &name, const ParamSet &params) {
    Reference<Primitive> prim;
    AreaLight *area = NULL;
    if (!curT.IsAnimated()) {
        Transform *o2w, *w2o;
        tcache.Lookup(curT[0], &o2w, &w2o);
        Reference<Shape> shape = MakeShp(name, o2w, w2o, gs.reverseOrientation, params);
        if (!shape) return;
        Reference<Material> mtl = CreateMaterialFromState(params);
        if (gs.areaLight != "") area = CreateDiffuseAreaLight(curT[0], gs.areaLightParams, shape);
        prim = new GeometricPrimitive(shape, mtl, area);
    } else {
        Transform *identity;
        tcache.Lookup(Transform(), &identity, NULL);
        Reference<Shape> shape = MakeShp(name, identity, identity, gs.reverseOrientation, params);
        if (!shape) return;
        Reference<Material> mtl = CreateMaterialFromState(params);
        Transform *w2o[2];
        tcache.Lookup(curT[0], NULL, &w2o[0]);
        tcache.Lookup(curT[1], NULL, &w2o[1]);
        AnimatedTransform aw2o(w2o[0], tStart, w2o[1], tEnd);
        Reference<Primitive> base = new GeometricPrimitive(shape, mtl, NULL);
        if (!base->CanIntersect()) {
            std::vector<Reference<Primitive> > refined;
            base->FullyRefine(refined);
            if (refined.empty()) return;
            if (refined.size() > 1) base = new BVHAccel(refined);
            else base = refined[0];
        }
        prim = new TransformedPrimitive(base, aw2o);
    }
    primitives.push_back(prim);
    if (area) lights.push_back(area);
}
void pbrtReverseOrientation() { gs.reverseOrientation = !gs.reverseOrientation; }
void pbrtVolume(const string &, const ParamSet &) { fprintf(stderr, "harness: volumes unsupported\n"); exit(2); }
void pbrtObjectBegin(const string &) { fprintf(stderr, "harness: instancing unsupported\n"); exit(2); }
void pbrtObjectEnd() {}
void pbrtObjectInstance(const string &) {}
void pbrtWorldEnd() {
    while (pushedGS.size()) pbrtAttributeEnd();
    while (pushedT.size()) pbrtTransformEnd();
    // film (spectralImage.cpp:452-475 parameter handling) with resolution override
    if (ovW > 0) { int v = ovW; filmParams.AddInt("xresolution", &v, 1); }
    if (ovH > 0) { int v = ovH; filmParams.AddInt("yresolution", &v, 1); }
    int xres = filmParams.FindOneInt("xresolution", 640);
    int yres = filmParams.FindOneInt("yresolution", 480);
    float crop[4] = { 0, 1, 0, 1 };
    int cwi;
    const float *cr = filmParams.FindFloat("cropwindow", &cwi);
    if (cr && cwi == 4) {
        crop[0] = Clamp(min(cr[0], cr[1]), 0., 1.); crop[1] = Clamp(max(cr[0], cr[1]), 0., 1.);
        crop[2] = Clamp(min(cr[2], cr[3]), 0., 1.); crop[3] = Clamp(max(cr[2], cr[3]), 0., 1.);
    }
    Filter *filter = CreateBoxFilter(filterParams);
    gFilter = filter;
    gFilm = new HarnessFilm(xres, yres, filter, crop, "harness");
    Transform *c2w[2];
    tcache.Lookup(cameraToWorld[0], &c2w[0], NULL);
    tcache.Lookup(cameraToWorld[1], &c2w[1], NULL);
    AnimatedTransform ac2w(c2w[0], tStart, c2w[1], tEnd);
    if (cameraName == "orthographic")
        gCamera = CreateOrthographicCamera(cameraParams, ac2w, gCameraFilm ? gCameraFilm : (Film *)gFilm);
    else if (cameraName != "perspective") { fprintf(stderr, "harness: camera %s unsupported\n", cameraName.c_str()); exit(2); }
    else gCamera = CreatePerspectiveCamera(cameraParams, ac2w, gCameraFilm ? gCameraFilm : (Film *)gFilm);
    if (ovMaxDepth >= 0) { int v = ovMaxDepth; surfParams.AddInt("maxdepth", &v, 1); }
    // the configs override the scene's integrator to "path" (SURVEY App. B), the harness's
    // default; --surf directlighting creates the DirectLightingIntegrator from the scene's
    // SurfaceIntegrator parameters (maxdepth, strategy; --dl-strategy overrides the latter),
    // --surf scene the one the scene names (api.cpp:551-583)
    string sn = string(surfOv) == "scene" ? surfName : string(surfOv);
    if (sn == "directlighting") {
        if (dlStrategyOv) { string st(dlStrategyOv); surfParams.AddString("strategy", &st, 1); }
        gSurf = CreateDirectLightingIntegrator(surfParams);
    } else if (sn == "metadata") {   // integrators/metadata.cpp:83-97
        if (metaStrategyOv) { string st(metaStrategyOv); surfParams.AddString("strategy", &st, 1); }
        gSurf = CreateMetadataIntegrator(surfParams);
    } else if (sn == "path") gSurf = CreatePathSurfaceIntegrator(surfParams);
    else { fprintf(stderr, "harness: surface integrator %s unsupported\n", sn.c_str()); exit(2); }
    gVol = CreateEmissionVolumeIntegrator(ParamSet());
    gSppParam = samplerParams.FindOneInt("pixelsamples", 4);
    Primitive *accel = CreateBVHAccelerator(primitives, accelParams);
    gScene = new Scene(accel, lights, NULL);
}

// ---------------------------------------------------------------------------------
// MT19937 first-generation known-answer output (rng.cpp:35-100)
// ---------------------------------------------------------------------------------
static void KatMT(const char *fn) {
    FILE *f = fopen(fn, "wb");
    uint32_t seeds[6] = { 0u, 1u, 5489u, 12345u, 0xdeadbeefu, 0xffffffffu };
    for (int k = 0; k < 6; ++k) {
        RNG rng(seeds[k]);
        fwrite(&seeds[k], 4, 1, f);
        for (int i = 0; i < 64; ++i) { uint32_t v = (uint32_t)rng.RandomUInt(); fwrite(&v, 4, 1, f); }
    }
    fclose(f);
}

static void usage() {
    fprintf(stderr, "usage: harness scene.pbrt [--res W H] [--spp N] [--maxdepth D] [--seed S]\n"
                    "   [--window x0 x1 y0 y1] [--raw film.f32] [--dat film.dat] [--paths paths.bin]\n"
                    "   [--path-every K] [--kat-mt out.bin] [--spectra out.bin] [--tris out.bin]\n"
                    "   [--keys keys.i32 (with --paths)] [--refdat film.dat] [--gpupath]\n"
                    "   [--surf path|directlighting|metadata|scene] [--dl-strategy all|one]\n"
                    "   [--meta-strategy mesh|material|depth] [--spectral N single|sampler]\n");
    exit(1);
}

int main(int argc, char **argv) {
    if (argc < 2) usage();
    const char *scene = argv[1];
    int spp = -1, seed = 0, win[4] = { -1, -1, -1, -1 }, pathEvery = 0;
    const char *rawOut = NULL, *datOut = NULL, *pathsOut = NULL, *katMt = NULL, *specOut = NULL, *trisOut = NULL;
    const char *keysIn = NULL, *refDat = NULL;
    bool gpupath = false;
    for (int i = 2; i < argc; ++i) {
        string a = argv[i];
        if (a == "--res") { ovW = atoi(argv[++i]); ovH = atoi(argv[++i]); }
        else if (a == "--spp") spp = atoi(argv[++i]);
        else if (a == "--maxdepth") ovMaxDepth = atoi(argv[++i]);
        else if (a == "--seed") seed = atoi(argv[++i]);
        else if (a == "--window") for (int k = 0; k < 4; ++k) win[k] = atoi(argv[++i]);
        else if (a == "--raw") rawOut = argv[++i];
        else if (a == "--dat") datOut = argv[++i];
        else if (a == "--paths") pathsOut = argv[++i];
        else if (a == "--path-every") pathEvery = atoi(argv[++i]);
        else if (a == "--kat-mt") katMt = argv[++i];
        else if (a == "--spectra") specOut = argv[++i];
        else if (a == "--tris") trisOut = argv[++i];
        else if (a == "--keys") keysIn = argv[++i];
        else if (a == "--refdat") refDat = argv[++i];
        else if (a == "--gpupath") gpupath = true;
        else if (a == "--surf") surfOv = argv[++i];
        else if (a == "--dl-strategy") dlStrategyOv = argv[++i];
        else if (a == "--meta-strategy") metaStrategyOv = argv[++i];
        else if (a == "--spectral") { specBands = atoi(argv[++i]); specSampler = string(argv[++i]) == "sampler"; }
        else usage();
    }
    Options opt; opt.quiet = true;
    pbrtInit(opt);
    // the reference's own spectral film beside the restatement (--refdat).  WriteImage adds
    // splatScale * splatC[nSpectralSamples] -- the Pixel's `pad` member, which the Pixel
    // constructor never initialises (spectralImageNoCamera.h:72-82, spectralImage.h:74-84) --
    // to every band.  A config-size film (tens of MB) comes from fresh mmap pages, where pad
    // is 0; a small film allocated after the scene would reuse freed heap.  So the film is
    // created here, on the fresh heap, before the scene is parsed: the fixture sees the
    // config-size behaviour (pad == 0).  Film parameters: the --res override and the box
    // filter's defaults (the harness's film uses the same, pbrtPixelFilter keeps only the name).
    Film *refFilm = NULL;
#ifndef HARNESS_RGB
    if (refDat) {
        if (ovW <= 0) { fprintf(stderr, "harness: --refdat needs --res\n"); return 1; }
        ParamSet fp;
        int w = ovW, h = ovH;
        fp.AddInt("xresolution", &w, 1);
        fp.AddInt("yresolution", &h, 1);
        string fn(refDat);
        fp.AddString("filename", &fn, 1);
        refFilm = CreateSpectralImageNoCameraFilm(fp, CreateBoxFilter(ParamSet()));
    }
#else
    if (refDat) { fprintf(stderr, "harness: --refdat needs the SampledSpectrum build\n"); return 1; }
#endif
    if (katMt) KatMT(katMt);
#ifndef HARNESS_RGB
    if (specOut) {
        // 'color' parameters -> FromRGB(REFLECTANCE) (paramset.cpp:89-98); band table dump
        FILE *f = fopen(specOut, "wb");
        float rgbs[][3] = { {0.5f, 0.5f, 0.8f}, {.4f, .2f, .2f}, {.5f, .5f, .5f}, {.3f, .3f, .3f}, {.4f, .5f, .4f},
                            {2000, 2000, 2000}, {0, 0, 0}, {.4f, .42f, .4f}, {15, 15, 15}, {.7f, .7f, .7f}, {1, 1, 1},
                            {0.9f, 0.1f, 0.3f}, {0.2f, 0.7f, 0.1f}, {0.05f, 0.3f, 0.95f} };
        int n = sizeof(rgbs) / sizeof(rgbs[0]);
        fwrite(&n, 4, 1, f);
        for (int k = 0; k < n; ++k) {
            Spectrum r = Spectrum::FromRGB(rgbs[k]), il = Spectrum::FromRGB(rgbs[k], SPECTRUM_ILLUMINANT);
            float c[nSpectralSamples];
            fwrite(rgbs[k], 4, 3, f);
            r.GetOrigC(c); fwrite(c, 4, nSpectralSamples, f);
            il.GetOrigC(c); fwrite(c, 4, nSpectralSamples, f);
        }
        fclose(f);
    }
#else
    if (specOut) { fprintf(stderr, "harness: --spectra needs the SampledSpectrum build\n"); return 1; }
#endif
#ifdef HARNESS_GPUPATH
    if (gpupath && refFilm) gCameraFilm = refFilm;
#endif
    if (string(scene) == "-") return 0;
    if (!ParseFile(scene)) { fprintf(stderr, "harness: cannot parse %s\n", scene); return 1; }
    if (!gScene) { fprintf(stderr, "harness: no WorldEnd\n"); return 1; }
#ifdef HARNESS_GPUPATH
    if (gpupath) {
        // Renderer "gpupath" as the binding's MakeRenderer branch creates it (INTEGRATION.md
        // §1): the renderer owns the camera; Render() reports failures through Error()
        // With --refdat the camera's film is the reference's SpectralImageNoCameraFilm (created
        // before the scene, refFilm above): the renderer hands its frame to it and its own
        // WriteImage writes the .dat.  --spp / --maxdepth / --seed go to the renderer as its
        // parameters (the film's --res it reads from the film).
        GpuPathRenderer::SetSceneFile(scene);
        ParamSet rp;
        rp.AddInt("seed", &seed, 1);
        if (spp > 0) rp.AddInt("pixelsamples", &spp, 1);
        if (ovMaxDepth >= 0) { int md = ovMaxDepth; rp.AddInt("maxdepth", &md, 1); }
        GpuPathRenderer *r = CreateGpuPathRenderer(gCamera, rp);
        r->Render(gScene);
        fprintf(stderr, "harness: gpupath status %d\n", r->LastStatus());
        int st = r->LastStatus();
        delete r;
        return st == 0 ? 0 : 3;
    }
#else
    if (gpupath) { fprintf(stderr, "harness: built without the gpupath binding (make -C oracle/ref gpupath)\n"); return 1; }
#endif
#ifndef HARNESS_RGB
    if (specBands) {
        // bands whose assigned indices need GetValueAtWavelength's c[i + 1] past the last
        // sample (spectrum.h:397) read outside the spectrum: rejected, as the GPU core does
        const int dI = round(nSpectralSamples / specBands);
        const float dW = (sampledLambdaEnd - sampledLambdaStart) / specBands;
        const float step = (sampledLambdaEnd - sampledLambdaStart) / nSpectralSamples;
        for (int b = 0; specBands > 0 && b < specBands; ++b) {
            if (min(dI * (b + 1), nSpectralSamples - 1) <= dI * b) continue;
            float wl = sampledLambdaStart + dW * b + (dW / 2);
            if (wl >= sampledLambdaStart + (nSpectralSamples - 1) * step) {
                fprintf(stderr, "harness: nWaveBands %d reads past the spectrum\n", specBands);
                return 1;
            }
        }
        if (specBands < 1) { fprintf(stderr, "harness: nWaveBands must be >= 1\n"); return 1; }
    }
#else
    if (specBands) { fprintf(stderr, "harness: --spectral needs the SampledSpectrum build\n"); return 1; }
#endif
    if (spp <= 0) spp = gSppParam;
    spp = (int)RoundUpPow2(spp);   // LDSampler rounds up (lowdiscrepancy.cpp:33-39)

    if (trisOut) {
        // world-space vertices of every refined primitive in BVH-input order, through the
        // public Shape::Sample API (Sample(0,u)=p1, Sample(1,0)=p3, Sample(1,1)=p2)
        FILE *f = fopen(trisOut, "wb");
        for (size_t k = 0; k < primitives.size(); ++k) {
            std::vector<Reference<Primitive> > ref;
            primitives[k]->FullyRefine(ref);
            for (size_t j = 0; j < ref.size(); ++j) {
                BBox b = ref[j]->WorldBound();
                fwrite(&b, sizeof(float), 6, f);
            }
        }
        fclose(f);
    }

    int xs, xe, ys, ye;
    gFilm->GetSampleExtent(&xs, &xe, &ys, &ye);
    if (win[0] >= 0) { xs = max(xs, win[0]); xe = min(xe, win[1]); ys = max(ys, win[2]); ye = min(ye, win[3]); }
    // the renderer's sampler only sizes the request here (LDSampler::RoundSize rounds a
    // DirectLighting light's nSamples to a power of two, directlighting.cpp:51); the sample
    // values come from FillSample
    LDSampler sizer(xs, xe, ys, ye, spp, gCamera->shutterOpen, gCamera->shutterClose);
    Sample *smp = new Sample(&sizer, gSurf, gVol, gScene);
    HarnessRenderer renderer(gSurf, gVol);
    gSurf->Preprocess(gScene, gCamera, &renderer);
    gVol->Preprocess(gScene, gCamera, &renderer);
    FILE *pf = pathsOut ? fopen(pathsOut, "wb") : NULL;
    if (pf) { int hdr[4] = { NOUT, spp, seed, 0 }; fwrite(hdr, 4, 4, pf); }
    MemoryArena arena;
    long nPath = 0, nBad = 0;
    // one camera sample of SamplerRendererTask::Run (samplerrenderer.cpp:86-133) with the
    // fixed-seed sampler and per-path RNG
    auto trace = [&](int x, int y, int s, RayDifferential *ray) -> Spectrum {
        FillSample(smp, x, y, (uint32_t)s, (uint32_t)spp, (uint32_t)seed, gCamera->shutterOpen, gCamera->shutterClose);
        float rayWeight = gCamera->GenerateRayDifferential(*smp, ray);
        ray->ScaleDifferentials(1.f / sqrtf(spp));
        RNG rng(path_seed(pixel_hash((uint32_t)seed, x, y), (uint32_t)s));
        Spectrum L;
        Intersection isect;
        Spectrum T;
        if (rayWeight > 0.f) L = rayWeight * renderer.Li(gScene, *ray, smp, rng, arena, &isect, &T);
        else L = 0.f;
        if (L.HasNaNs()) { L = Spectrum(0.f); ++nBad; }
        else if (L.y() < -1e-5) { L = Spectrum(0.f); ++nBad; }
        else if (isinf(L.y())) { L = Spectrum(0.f); ++nBad; }
        return L;
    };
#ifndef HARNESS_RGB
    // one camera sample of SpectralRendererTask::Run (spectralrenderer.cpp:98-190): per wave
    // band b a ray of wavelength 395 + dW b + dW / 2 (integer dW = 320 / nWaveBands), its
    // radiance's value at that wavelength (Spectrum::GetValueAtWavelength, spectrum.h:384-405)
    // assigned to indices [dI b, min(dI (b+1), N-1)).  singleDirection traces every band of the
    // sample; samplerDirection only band s % nWaveBands.  Fixed-seed re-specification: the
    // sample's Ls starts at 0 (the reference reuses a per-batch-slot array across samples) and
    // band b's path draws from RNG(path_seed(hp, s nWaveBands + b)) (singleDirection) or
    // RNG(path_seed(hp, s)) (samplerDirection) instead of the task's shared stream.
    auto traceSpectral = [&](int x, int y, int s, RayDifferential *ray) -> Spectrum {
        const int nWaveBands = specBands;
        FillSample(smp, x, y, (uint32_t)s, (uint32_t)spp, (uint32_t)seed, gCamera->shutterOpen, gCamera->shutterClose);
        const int methodMultiplier = specSampler ? 1 : nWaveBands;
        int deltaIndex = round(nSpectralSamples / nWaveBands);
        float deltaWave = (sampledLambdaEnd - sampledLambdaStart) / nWaveBands;
        const uint32_t hp = pixel_hash((uint32_t)seed, x, y);
        Spectrum Ls(0.f);
        for (int sb = 0; sb < methodMultiplier; ++sb) {
            const int b = specSampler ? s % nWaveBands : sb;
            Spectrum Lr;
            ray->wavelength = sampledLambdaStart + deltaWave * b + (deltaWave / 2);
            const float wlSet = ray->wavelength;
            float rayWeight = gCamera->GenerateRayDifferential(*smp, ray);
            ray->ScaleDifferentials(1.f / sqrtf(spp));
            if (x == xs && y == ys && s == 0 && b == 0)
                fprintf(stderr, "harness: wavelength %g set, %g after GenerateRayDifferential\n", wlSet, ray->wavelength);
            // the camera may leave the wavelength indeterminate (the perspective camera's Ray
            // constructor does not set it, geometry.h:319-321); the band's wavelength is what
            // the renderer reads
            ray->wavelength = wlSet;
            RNG rng(path_seed(hp, specSampler ? (uint32_t)s : (uint32_t)s * (uint32_t)nWaveBands + (uint32_t)b));
            Intersection isect;
            Spectrum T;
            if (rayWeight > 0.f) {
                Lr = rayWeight * renderer.Li(gScene, *ray, smp, rng, arena, &isect, &T);
                if (Lr.HasNaNs()) { Lr = Spectrum(0.f); ++nBad; }
                else if (Ls.y() < -1e-5) { Lr = Spectrum(0.f); ++nBad; }
                else if (isinf(Ls.y())) { Lr = Spectrum(0.f); ++nBad; }
            }
            else Lr = 0.f;
            int bottomIndex = deltaIndex * b;
            int topIndex = min(deltaIndex * (b + 1), nSpectralSamples - 1);
            float v;
            if (topIndex > bottomIndex) {
                Lr.GetValueAtWavelength(ray->wavelength, &v);
                for (int k = bottomIndex; k < topIndex; ++k) Ls.AssignValueAtIndex(k, v);
            }
            arena.FreeAll();
        }
        return Ls;
    };
#else
    auto traceSpectral = [&](int x, int y, int s, RayDifferential *ray) -> Spectrum { return trace(x, y, s, ray); };
#endif
    auto emit = [&](int x, int y, int s, const Spectrum &L) {
        int key[3] = { x, y, s };
        float c[NOUT];
        spec_out(L, c);
        fwrite(key, 4, 3, pf);
        fwrite(c, 4, NOUT, pf);
    };
    if (keysIn) {
        if (!pf) { fprintf(stderr, "harness: --keys needs --paths\n"); return 1; }
        FILE *kf = fopen(keysIn, "rb");
        if (!kf) { fprintf(stderr, "harness: cannot open %s\n", keysIn); return 1; }
        int key[3];
        while (fread(key, 4, 3, kf) == 3) {
            int gx0, gx1, gy0, gy1;
            gFilm->GetSampleExtent(&gx0, &gx1, &gy0, &gy1);
            if (key[0] < gx0 || key[0] >= gx1 || key[1] < gy0 || key[1] >= gy1 || key[2] < 0 || key[2] >= spp) {
                fprintf(stderr, "harness: key (%d %d %d) outside the sample extent\n", key[0], key[1], key[2]);
                return 1;
            }
            RayDifferential ray;
            Spectrum L = specBands ? traceSpectral(key[0], key[1], key[2], &ray) : trace(key[0], key[1], key[2], &ray);
            emit(key[0], key[1], key[2], L);
            ++nPath;
            arena.FreeAll();
        }
        fclose(kf);
        fclose(pf);
        fprintf(stderr, "harness: %ld keyed paths traced (%d spp), %ld zeroed by NaN/inf guards\n", nPath, spp, nBad);
        return 0;
    }
    for (int y = ys; y < ye; ++y)
        for (int x = xs; x < xe; ++x)
            for (int s = 0; s < spp; ++s) {
                RayDifferential ray;
                Spectrum L = specBands ? traceSpectral(x, y, s, &ray) : trace(x, y, s, &ray);
                gFilm->AddSample(*smp, L, ray);
                if (refFilm) refFilm->AddSample(*smp, L, ray);
                if (pf && (pathEvery <= 1 || (nPath % pathEvery) == 0)) emit(x, y, s, L);
                ++nPath;
                arena.FreeAll();
            }
    if (pf) fclose(pf);
    if (rawOut) gFilm->WriteRaw(rawOut);
    if (datOut) gFilm->WriteDat(datOut);
    if (refFilm) refFilm->WriteImage(1.f);
    fprintf(stderr, "harness: %ld paths traced (%d spp), %ld zeroed by NaN/inf guards\n", nPath, spp, nBad);
    return 0;
}
