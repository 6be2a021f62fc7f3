/* pbrthost.h -- C ABI of the host front end (libpbrthost.so).
 *
 * Replaces, for the hot path's inputs, the reference's parse + scene construction
 * (core/parser.cpp ParseFile -> core/api.cpp pbrt* -> RenderOptions::MakeScene /
 * MakeCamera, api.cpp:1215-1330) and the film output SpectralImageFilm::WriteImage
 * (film/spectralImage.cpp:267-378).  The flattened scene it produces is the input of
 * pbrtgpu_scene_upload (include/pbrtgpu.h).
 */
#ifndef PBRTHOST_H
#define PBRTHOST_H
#include <stdint.h>
#include "pbrtgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pbrthost_scene pbrthost_scene;

#define PBRTHOST_KEEP_SEED 0xffffffffu
/* Layout version of pbrthost_overrides: the caller writes it into abi_version, and
 * pbrthost_load refuses a struct of another layout (a caller built against an older header
 * passes a shorter struct) */
#define PBRTHOST_ABI_VERSION 2

/* Overrides of scene-file values: -1 keeps the file's value. */
typedef struct pbrthost_overrides {
    int32_t abi_version;  /* PBRTHOST_ABI_VERSION */
    int32_t xres, yres;   /* Film "xresolution"/"yresolution" */
    int32_t spp;          /* Sampler "pixelsamples" (rounded up to a power of two) */
    int32_t maxdepth;     /* SurfaceIntegrator "path" "maxdepth" */
    int32_t bands;        /* nSpectralSamples: 32 (reference build), 60 or 30; <= 0: the pack's own, or 32 */
    uint32_t seed;        /* fixed-seed sampler seed; PBRTHOST_KEEP_SEED keeps the pack's (0 for .pbrt) */
    int32_t integrator;   /* PBRTGPU_INTEGRATOR_* to force, or -1: the scene's own ("path" for packs
                           * built before integrators were recorded) */
    int32_t dl_strategy;  /* PBRTGPU_DL_* to force, or -1: the scene's "strategy" */
    int32_t meta_strategy;   /* PBRTGPU_META_* to force, or -1: the scene's metadata "strategy" */
    int32_t renderer;        /* PBRTGPU_RENDERER_* to force, or -1: the scene's Renderer */
    int32_t wave_bands;      /* SpectralRenderer nWaveBands to force, or <= 0: the scene's */
    int32_t spectral_sampling;   /* PBRTGPU_SPECTRAL_* to force, or -1: the scene's samplingMethod */
} pbrthost_overrides;

/* PBRTHOST_ABI_VERSION of the library */
int pbrthost_abi_version(void);
/* path: a .pbrt scene file or a .pack scene pack; ov may be NULL (the file's values) or must
 * carry abi_version == PBRTHOST_ABI_VERSION.  Returns 0 or -1 (message in err). */
int pbrthost_load(const char *path, const pbrthost_overrides *ov, pbrthost_scene **out, char *err, int errlen);
int pbrthost_free(pbrthost_scene *s);
int pbrthost_flat(pbrthost_scene *s, pbrtgpu_flat_scene *out);   /* pointers stay owned by s */
int pbrthost_save_pack(pbrthost_scene *s, const char *path, char *err, int errlen);
int pbrthost_set_render(pbrthost_scene *s, int spp, int maxdepth, uint32_t seed);
/* info[0..15]: bands, spp, maxdepth, nodes, prims, tris, meshes, verts, quadrics,
 * materials, lights, bvh depth, film W, film H, warnings, 0 */
int pbrthost_info(pbrthost_scene *s, int64_t *info, int n);
/* pbrtWorldEnd's metadata text file (api.cpp:1228-1282) for the scene's SurfaceIntegrator
 * "strategy": "mesh" -> <stem>_mesh.txt ("primitiveId shape-name" per top-level primitive, in
 * scene order), "material" -> <stem>_materials.txt ("materialId name" per named material, by
 * name); any other strategy writes nothing.  image_file: the film's output name (its stem is
 * kept).  Returns 1 if a file was written, 0 if none, -1 on error. */
int pbrthost_write_metadata(pbrthost_scene *s, const char *image_file);
/* reference .dat writer; film [H][W][N] float32 (raw sums), weight [H][W] or NULL */
int pbrthost_write_dat(const char *path, const float *film, const float *weight, int W, int H, int N);
/* the same for a scene's film (its crop window's W x H, its bands), line 2 holding the
 * RealisticDiffractionCamera's focal length, f-stop and field of view (spectralImage.cpp:356-360) */
int pbrthost_write_dat_scene(const pbrthost_scene *s, const char *path, const float *film, const float *weight);

/* SampledSpectrum::FromRGB (spectrum.cpp:93-178) at the given band count (32, 60 or 30);
 * illuminant != 0 selects SPECTRUM_ILLUMINANT.  out[bands]. */
/* Loop subdivision (shapes/loopsubdiv.cpp:147-437).  A subdivider refines a control mesh
 * (nf faces vi[nf][3] over nv vertices P[nv][3], object space) by `levels` levels to the
 * limit surface: *nv_out vertices, P_out / N_out [*nv_out][3] limit positions and normals,
 * vi_out [nf * 4^levels][3]; with P_out NULL it only sets *nv_out.  Returns 0 or an error.
 * pbrthost_set_loop_subdivider(fn, user) makes the front end refine loopsubdiv shapes with fn
 * (e.g. pbrtgpu_loop_subdivide_hook with user = a pbrtgpu context); NULL restores the host
 * refinement.  pbrthost_loop_refine is the host refinement itself (tests). */
typedef int (*pbrthost_loop_subdivider)(void *user, int32_t nf, int32_t nv, const int32_t *vi, const float *P,
                                        int32_t levels, int32_t *nv_out, float *P_out, float *N_out, int32_t *vi_out);
int pbrthost_set_loop_subdivider(pbrthost_loop_subdivider fn, void *user);
int pbrthost_loop_refine(int32_t nf, int32_t nv, const int32_t *vi, const float *P, int32_t levels, int32_t *nv_out,
                         float *P_out, float *N_out, int32_t *vi_out);
int pbrthost_spectrum_from_rgb(int bands, const float rgb[3], int illuminant, float *out);

#ifdef __cplusplus
}
#endif
#endif
