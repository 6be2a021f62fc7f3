// integration/gpupathrenderer.cpp -- see gpupathrenderer.h.
#include "stdafx.h"
#include "gpupathrenderer.h"
#include "camera.h"
#include "film.h"
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
    // the SpectralRenderer's parameters (api.cpp:1378-1379): "integer nWaveBands" > 0 renders
    // as Renderer "spectralrenderer" would
    waveBands = params.FindOneInt("nWaveBands", 0);
    // "bool gpusetup": the front end refines the scene's loopsubdiv shapes on the first GPU
    // (positions bit-identical to the host refinement, normals up to last-ulp cosf / sinf cases)
    gpuSetup = params.FindOneBool("gpusetup", false);
    string sm = params.FindOneString("samplingMethod", "singleDirection");
    spectralSampling = sm == "samplerDirection" ? PBRTGPU_SPECTRAL_SAMPLER : PBRTGPU_SPECTRAL_SINGLE;
    // the spectral film writes <imageOutputName stem>.dat (spectralImage.cpp:348-350)
    const string &img = camera ? camera->film->imageOutputName : string("pbrt.exr");
    outFile = img.substr(0, img.find_last_of(".")) + ".dat";
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
    pbrthost_overrides ov = { PBRTHOST_ABI_VERSION, -1, -1, -1, -1, nSpectralSamples, seed, -1, -1, -1,
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
    // line 2 of the header: the lens camera's focal length, f-stop, field of view
    if (status == 0 && pbrthost_write_dat_scene(hs, outFile.c_str(), film.data(), NULL) != 0) {
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
