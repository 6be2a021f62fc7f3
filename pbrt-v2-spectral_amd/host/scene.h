// scene.h -- host scene built by the pbrt front end and flattened for the device.
#pragma once
#include <string>
#include <vector>
#include <map>
#include "pbrtgpu.h"
#include "pmath.h"
#include "spectrum.h"

namespace pbrtamd {

struct RenderOverrides {
    int xres = -1, yres = -1;     // Film xresolution / yresolution
    int spp = -1;                 // Sampler pixelsamples (rounded up to a power of two)
    int maxdepth = -1;            // SurfaceIntegrator "path" maxdepth
    int bands = 32;               // nSpectralSamples (32 = reference build, 60 = C4 variant)
    uint32_t seed = 0;
    int integrator = -1;          // PBRTGPU_INTEGRATOR_* to force, -1: the scene's SurfaceIntegrator
    int dl_strategy = -1;         // PBRTGPU_DL_* to force, -1: the scene's "strategy"
    int meta_strategy = -1;       // PBRTGPU_META_* to force, -1: the scene's metadata "strategy"
    int renderer = -1;            // PBRTGPU_RENDERER_* to force, -1: the scene's Renderer
    int wave_bands = 0;           // SpectralRenderer nWaveBands to force, <= 0: the scene's
    int spectral_sampling = -1;   // PBRTGPU_SPECTRAL_* to force, -1: the scene's samplingMethod
};

// Resolution-independent camera description (perspective.cpp:110-147 parameters); the
// pbrtgpu_camera block is derived from it for a given film resolution.
struct CameraParams {
    float fov = 90.f, lensRadius = 0.f, focalDistance = 1e30f, shutterOpen = 0.f, shutterClose = 1.f;
    float frameAspect = 0.f;        // "frameaspectratio" if given (hasFrameAspect)
    int hasFrameAspect = 0;
    int hasScreenWindow = 0;
    float screenWindow[4] = {0, 0, 0, 0};
    float crop[4] = {0, 1, 0, 1};
    float cam2world[16];
    int xres = 640, yres = 480;     // film resolution the scene was built with
};
void ComputeCamera(const CameraParams &cp, int xres, int yres, pbrtgpu_camera *out, int cameraType);

// Host-owned storage behind a pbrtgpu_flat_scene.
struct HostScene {
    CameraParams camParams;
    int nBands = 32;
    int maxDepth = 5;
    int spp = 4;
    uint32_t seed = 0;
    std::vector<float> bandY;
    float yint = 0.f;
    pbrtgpu_camera camera{};
    std::vector<pbrtgpu_bvh_node> nodes;
    std::vector<pbrtgpu_prim> prims;          // BVH order
    std::vector<pbrtgpu_triangle> tris;
    std::vector<pbrtgpu_mesh> meshes;
    std::vector<float> vertP, vertN, vertUV;
    std::vector<pbrtgpu_quadric> quadrics;
    std::vector<pbrtgpu_material> materials;
    std::vector<pbrtgpu_light> lights;
    std::vector<pbrtgpu_light_shape> lightShapes;
    std::vector<float> spectra;
    std::vector<pbrtgpu_instance> instances;
    std::vector<int32_t> primInstance;        // per prim: owning instance or -1
    std::vector<pbrtgpu_kdnode> kdnodes;      // measured BRDF kd-trees
    std::vector<pbrtgpu_texture> textures;
    std::vector<float> texels;                // MIPMap pyramids of the IMAGE textures (pbrtgpu_texture)
    std::vector<pbrtgpu_instance> cameraMotion;   // 0 or 1: an animated camera's CameraToWorld
    std::vector<float> ewaLut;                // [128] MIPMap::weightLut
    std::vector<float> rgbBasis;              // [14][nBands] FromRGB basis spectra
    std::vector<float> merl;                  // RegularHalfangleBRDF RGB tables (pbrtgpu_flat_scene::merl)
    int integrator = 0;                       // PBRTGPU_INTEGRATOR_* (packs older than v6: path)
    int dlStrategy = 0;                       // PBRTGPU_DL_*
    int metaStrategy = PBRTGPU_META_DEPTH;    // PBRTGPU_META_*
    std::string surfStrategy;                 // the SurfaceIntegrator's "strategy" string (metadata files)
    int renderer = PBRTGPU_RENDERER_SAMPLER;  // PBRTGPU_RENDERER_* (packs older than v8: sampler)
    int waveBands = 32;                       // SpectralRenderer nWaveBands
    int spectralSampling = PBRTGPU_SPECTRAL_SINGLE;
    int cameraType = PBRTGPU_CAMERA_PERSPECTIVE;   // PBRTGPU_CAMERA_*
    pbrtgpu_lens lens = {};                   // RealisticDiffractionCamera (elements: lensEl)
    std::vector<float> lensEl;                // [elements][4]
    std::vector<float> eyeIor;                // [4][nBands] IORforEyeEnabled: cornea, aqueous, lens, vitreous
    mutable std::vector<float> lensPinholes;  // [w][h][3] pinhole array at the camera's film resolution (Flat)
    std::vector<uint32_t> primMeta;           // [prims][2]: primitiveId, materialId a hit reports
    std::vector<std::pair<uint32_t, std::string> > metaMesh;        // top-level primitives: id, shape name
    std::vector<std::pair<uint32_t, std::string> > metaMaterials;   // named materials: id, name (by name)
    // diagnostics
    std::vector<std::string> warnings;
    int bvhMaxDepth = 0;

    void Flat(pbrtgpu_flat_scene *out) const;     // pointers into this object
};

// Parse a pbrt-v2 scene file (Include resolved relative to its directory) and build the
// flattened scene with the reference's semantics (api.cpp subset, see frontend.cpp).
bool LoadPbrtScene(const std::string &path, const RenderOverrides &ov, HostScene *out, std::string *err);

// scene pack: a binary snapshot of a HostScene (so the GPU box needs no scene files)
bool SavePack(const HostScene &s, const std::string &path, std::string *err);
bool LoadPack(const std::string &path, HostScene *s, std::string *err);

}  // namespace pbrtamd
