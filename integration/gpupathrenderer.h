// integration/gpupathrenderer.h -- the reference-side binding of the MI355X core: a
// Renderer (core/renderer.h:35-46) that renders a WorldBlock's frame on the GPUs of one node
// through the C ABIs include/pbrthost.h and include/pbrtgpu.h, and hands the rendered film to
// the camera's own Film, whose WriteImage writes it (film/spectralImage.cpp:267-378: the .dat).
//
// A maintainer adds this file and gpupathrenderer.cpp to the reference tree (e.g.
// src/renderers/), one branch to RenderOptions::MakeRenderer (core/api.cpp:1333-1420) and
// one line to main (main/pbrt.cpp:66-70); INTEGRATION.md §1 shows both.  tests/test_binding.py
// compiles the two files against the reference's own headers and links them into the
// reference harness (oracle/ref/Makefile, target gpupath).
//
// It renders what SamplerRenderer + PathIntegrator would: the core takes the scene from the
// scene file (its own front end builds a node-for-node identical BVH; the reference's BVH and
// mesh arrays are private, bvh.h:58-63, trianglemesh.h:51-59), not from the Scene* argument.
#ifndef PBRT_RENDERERS_GPUPATHRENDERER_H
#define PBRT_RENDERERS_GPUPATHRENDERER_H

#include "pbrt.h"
#include "renderer.h"
#include "paramset.h"

class GpuPathRenderer : public Renderer {
public:
    // camera: as MakeRenderer creates it for SamplerRenderer (the renderer owns it; its film
    // names the output, Film::imageOutputName).  params: the Renderer directive's
    //   "integer gpus" (0: every visible device), "integer seed" (fixed-seed sampler seed),
    //   "integer slices" (tile slices per GPU), "string scenefile" (overrides SceneFile()),
    //   "integer nWaveBands" / "string samplingMethod" (the SpectralRenderer's, api.cpp:1378-1379).
    //   "bool gpusetup" (refine loopsubdiv shapes on the GPU, pbrtgpu_loop_subdivide).
    //   "integer pixelsamples" / "integer maxdepth": override the scene file's Sampler /
    //   SurfaceIntegrator values (the harness's --spp / --maxdepth; default: the scene's).
    // The resolution is the camera film's (Film::xResolution / yResolution).
    GpuPathRenderer(Camera *camera, const ParamSet &params);
    ~GpuPathRenderer();
    // Renderer::Render: one frame over all GPUs, added to camera->film (one AddSample per
    // pixel, exact) and written by its WriteImage; on failure Error() and no file
    void Render(const Scene *scene);
    // per-ray queries stay on the CPU path: the core renders whole frames only
    Spectrum Li(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                MemoryArena &arena, Intersection *isect = NULL, Spectrum *T = NULL) const;
    Spectrum Transmittance(const Scene *scene, const RayDifferential &ray, const Sample *sample,
                           RNG &rng, MemoryArena &arena) const;

    // The top-level scene file.  The parser's current_file (core/parser.cpp:34-50) names the
    // file being parsed when WorldEnd runs -- an Include'd file if WorldEnd sits in one, and ""
    // once ParseFile returns -- so main records the file it hands to ParseFile instead.
    static void SetSceneFile(const string &file);
    static const string &SceneFile();

    // 0 after a successful Render, else the pbrtgpu / pbrthost error code (tests)
    int LastStatus() const { return status; }

private:
    Camera *camera;
    string sceneFile, outFile;
    int ngpu, slices, status;
    bool gpuSetup;   // "bool gpusetup": refine loopsubdiv shapes on the GPU (pbrtgpu_loop_subdivide)
    int waveBands, spectralSampling;   // "nWaveBands" (> 0: SpectralRenderer), "samplingMethod"
    int spp, maxDepth;                 // "pixelsamples", "maxdepth" overrides (-1: the scene's)
    uint32_t seed;
};

GpuPathRenderer *CreateGpuPathRenderer(Camera *camera, const ParamSet &params);

#endif // PBRT_RENDERERS_GPUPATHRENDERER_H
