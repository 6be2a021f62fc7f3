// integration/gpupathrenderer.cpp -- see gpupathrenderer.h.
#include "stdafx.h"
#include "gpupathrenderer.h"
#include "camera.h"
#include "film.h"
#include "sampler.h"
#include "spectrum.h"
#include "pbrthost.h"
#include "pbrtgpu.h"
#include <vector>

static string gSceneFile;

void GpuPathRenderer::SetSceneFile(const string &file) { gSceneFile = file; }
const string &GpuPathRenderer::SceneFile() { return gSceneFile; }

GpuPathRenderer::GpuPathRenderer(Camera *c, const ParamSet &params)
    : camera(c), status(0) {
    ngpu = params.FindOneInt("gpus", 0);
    slices = params.FindOneInt("slices", 1);
    seed = (uint32_t)params.FindOneInt("seed", 0);
    sceneFile = params.FindOneString("scenefile", gSceneFile);
    spp = params.FindOneInt("pixelsamples", -1);
    maxDepth = params.FindOneInt("maxdepth", -1);
    // the SpectralRenderer's parameters (api.cpp:1378-1379): "integer nWaveBands" > 0 renders
    // as Renderer "spectralrenderer" would
    waveBands = params.FindOneInt("nWaveBands", 0);
    // "bool gpusetup": the front end refines the scene's loopsubdiv shapes on the first GPU
    // (positions bit-identical to the host refinement, normals up to last-ulp cosf / sinf cases)
    gpuSetup = params.FindOneBool("gpusetup", false);
    string sm = params.FindOneString("samplingMethod", "singleDirection");
    spectralSampling = sm == "samplerDirection" ? PBRTGPU_SPECTRAL_SAMPLER : PBRTGPU_SPECTRAL_SINGLE;
    // without a camera film (never from MakeRenderer) the .dat goes to <imageOutputName stem>.dat
    // through pbrthost_write_dat_scene, as the spectral film names it (spectralImage.cpp:348-350)
    const string &img = camera ? camera->film->imageOutputName : string("pbrt.exr");
    outFile = img.substr(0, img.find_last_of(".")) + ".dat";
}

// A Spectrum holding given coefficients: CoefficientSpectrum::c is protected (spectrum.h:97-250),
// and a derived class may set it.  Sized from c itself, so it serves SampledSpectrum and the RGB
// build's RGBSpectrum alike.
struct FilmPixelValue : public Spectrum {
    explicit FilmPixelValue(const float *v) {
        for (int i = 0; i < (int)(sizeof(c) / sizeof(c[0])); ++i) c[i] = v[i];
    }
};

// The GPU film into the camera's Film: one AddSample per pixel at its centre.  The film's box
// filter (width .5, BoxFilter::Evaluate = 1) then covers that one pixel with weight 1
// (spectralImage.cpp:77-152: x0 = Ceil2Int(x - .5), x1 = Floor2Int(x + .5), both x), and the
// pixel starts at 0, so its coefficients become 0 + 1 * v = v bit for bit (a -0 sum becomes +0,
// as in the reference's own film, which also starts at +0); weightSum becomes 1, and
// WriteImage only tests it against 0.  The core renders the box filter only (pbrthost refuses
// other PixelFilters), so the scene's film has that filter.
static bool AddToFilm(Film *f, const float *film, int px0, int py0, int W, int H, int N) {
    int fx0, fx1, fy0, fy1;
    f->GetPixelExtent(&fx0, &fx1, &fy0, &fy1);
    if (fx0 != px0 || fy0 != py0 || fx1 - fx0 != W || fy1 - fy0 != H || N != (int)(sizeof(Spectrum) / sizeof(float))) {
        Error("gpupath: the scene's film window [%d, %d) x [%d, %d) is not the camera film's [%d, %d) x [%d, %d)",
              px0, px0 + W, py0, py0 + H, fx0, fx1, fy0, fy1);
        return false;
    }
    const Ray none;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            CameraSample cs;
            cs.imageX = px0 + x + .5f;
            cs.imageY = py0 + y + .5f;
            cs.lensU = cs.lensV = .5f;
            cs.time = 0.f;
            f->AddSample(cs, FilmPixelValue(film + ((size_t)y * W + x) * N), none);
        }
    return true;
}

GpuPathRenderer::~GpuPathRenderer() { delete camera; }

void GpuPathRenderer::Render(const Scene *) {
    status = 0;
    if (sceneFile.empty()) {
        Error("gpupath: top-level scene file unknown (GpuPathRenderer::SetSceneFile or \"string scenefile\")");
        status = PBRTGPU_E_INVALID;
        return;
    }
    int ndev = pbrtgpu_device_count();
    if (ndev <= 0) {   // no CPU fallback: the core is the GPU path
        Error("gpupath: no MI355X device (pbrtgpu_device_count() == 0); nothing rendered");
        status = PBRTGPU_E_NODEVICE;
        return;
    }
    int n = ngpu > 0 ? min(ngpu, ndev) : ndev;
    // the scene's own integrator and camera; the SpectralRenderer if asked for
    // the camera film's resolution (the film is what MakeCamera sized), the scene's spp and
    // maxdepth unless overridden
    const int xres = camera ? camera->film->xResolution : -1, yres = camera ? camera->film->yResolution : -1;
    pbrthost_overrides ov = { PBRTHOST_ABI_VERSION, xres, yres, spp, maxDepth, nSpectralSamples, seed, -1, -1, -1,
                              waveBands > 0 ? PBRTGPU_RENDERER_SPECTRAL : -1, waveBands,
                              waveBands > 0 ? spectralSampling : -1 };
    pbrthost_scene *hs = NULL;
    char err[1024];
    std::vector<pbrtgpu_ctx *> ctx(n, (pbrtgpu_ctx *)NULL);
    for (int d = 0; d < n && status == 0; ++d) status = pbrtgpu_context_create(d, &ctx[d]);
    if (status == 0) {
        if (gpuSetup) pbrthost_set_loop_subdivider(pbrtgpu_loop_subdivide_hook, ctx[0]);
        status = pbrthost_load(sceneFile.c_str(), &ov, &hs, err, sizeof(err));
        if (gpuSetup) pbrthost_set_loop_subdivider(NULL, NULL);
        if (status != 0) Error("gpupath: %s", err);
    } else Error("gpupath: %s", pbrtgpu_last_error());
    if (status != 0) {
        for (int d = 0; d < n; ++d)
            if (ctx[d]) pbrtgpu_context_destroy(ctx[d]);
        return;
    }
    pbrtgpu_flat_scene fs;
    pbrthost_flat(hs, &fs);
    const int W = fs.camera.px_count, H = fs.camera.py_count, N = fs.n_bands;
    for (int d = 0; d < n && status == 0; ++d) status = pbrtgpu_scene_upload(ctx[d], &fs);
    std::vector<float> film((size_t)W * H * N, 0.f);
    if (status == 0) {
        // one host thread per GPU, interleaved 16x16 film tiles, host gather (no RCCL)
        pbrtgpu_render_desc rd = { 0, fs.spp, 16, 16, 0, { 0, 0, 0 } };
        status = pbrtgpu_render_multi(ctx.data(), n, &rd, NULL, 0, slices, film.data(), (int64_t)film.size(), NULL);
    }
    if (status != 0) Error("gpupath: %s", pbrtgpu_last_error());
    for (int d = 0; d < n; ++d)
        if (ctx[d]) pbrtgpu_context_destroy(ctx[d]);
    // (the metadata text file of a "metadata" SurfaceIntegrator is written by the reference's own
    // pbrtWorldEnd, api.cpp:1228-1282, before the renderer runs; pbrthost_write_metadata is that
    // writer for callers without api.cpp)
    if (status == 0 && camera && camera->film) {
        // the camera's Film writes the image: SpectralImageFilm::WriteImage (the .dat: header,
        // the lens camera's focal length / f-stop / field of view line, conversion matrix, payload)
        // as SamplerRenderer::Render ends (samplerrenderer.cpp:221)
        if (AddToFilm(camera->film, film.data(), fs.camera.px_start, fs.camera.py_start, W, H, N))
            camera->film->WriteImage();
        else status = PBRTGPU_E_INVALID;
    } else if (status == 0 && pbrthost_write_dat_scene(hs, outFile.c_str(), film.data(), NULL) != 0) {
        Error("gpupath: cannot write \"%s\"", outFile.c_str());
        status = PBRTGPU_E_INVALID;
    }
    pbrthost_free(hs);
}

Spectrum GpuPathRenderer::Li(const Scene *, const RayDifferential &, const Sample *, RNG &, MemoryArena &,
                             Intersection *, Spectrum *) const {
    Error("gpupath renders whole frames only (Renderer::Li is not available)");
    return Spectrum(0.f);
}

Spectrum GpuPathRenderer::Transmittance(const Scene *, const RayDifferential &, const Sample *, RNG &,
                                        MemoryArena &) const {
    return Spectrum(1.f);   // no participating media on this path (EmissionIntegrator: T = 1)
}

GpuPathRenderer *CreateGpuPathRenderer(Camera *camera, const ParamSet &params) {
    return new GpuPathRenderer(camera, params);
}
