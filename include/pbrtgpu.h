/* pbrtgpu.h -- C ABI of the MI355X spectral path-tracing core (libpbrtgpu.so).
 *
 * Drop-in boundary: this library replaces the body of the reference's
 *   Renderer::Render(const Scene*)              core/renderer.h:35-46
 * as implemented by SamplerRenderer::Render + SamplerRendererTask::Run
 *   (renderers/samplerrenderer.cpp:60-222) driving PathIntegrator::Li
 *   (integrators/path.cpp:44-115), BVHAccel::Intersect/IntersectP
 *   (accelerators/bvh.cpp:380-481), BSDF::Sample_f/f/Pdf (core/reflection.cpp:514-618)
 *   and SpectralImageFilm::AddSample (film/spectralImage.cpp:77-152).
 * The host C++ side (pbrt-v2-spectral_amd/host, GpuPathRenderer) parses the unchanged
 * pbrt scene format, builds the BVH and hands the flattened scene below to
 * pbrtgpu_scene_upload.  All pointers are host pointers; sizes are element counts.
 * No torch / HIP types appear in this interface.
 *
 * Return codes: 0 = success; negative = error (PBRTGPU_E_*, or -(1000 + hipError_t)).
 * pbrtgpu_last_error() returns a thread-local message for the last failure.
 * Threading: one context per GPU, each driven by one host thread; calls on distinct
 * contexts may run concurrently.
 */
#ifndef PBRTGPU_H
#define PBRTGPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBRTGPU_ABI_VERSION 16
#define PBRTGPU_MAX_BANDS 64

#define PBRTGPU_E_INVALID   (-1)
#define PBRTGPU_E_NODEVICE  (-2)
#define PBRTGPU_E_NOMEM     (-3)
#define PBRTGPU_E_UNSUPPORTED (-4)
#define PBRTGPU_E_STATE     (-5)

/* ---- flattened scene ------------------------------------------------------------ */

/* LinearBVHNode (bvh.cpp:105-115): 32 bytes. leaf iff (meta & 0xff) != 0.
 * meta = nPrimitives | (axis << 8).  offset = primitivesOffset (leaf) or
 * secondChildOffset (interior); the first child of an interior node is node+1. */
typedef struct pbrtgpu_bvh_node {
    float bmin[3];
    float bmax[3];
    uint32_t offset;
    uint32_t meta;
} pbrtgpu_bvh_node;

enum { PBRTGPU_SHAPE_TRIANGLE = 0, PBRTGPU_SHAPE_SPHERE = 1, PBRTGPU_SHAPE_DISK = 2, PBRTGPU_SHAPE_INSTANCE = 3,
       PBRTGPU_SHAPE_CYLINDER = 4 };

/* one GeometricPrimitive, in BVH (orderedPrims) order */
typedef struct pbrtgpu_prim {
    int32_t shape_type;   /* PBRTGPU_SHAPE_* */
    int32_t shape_index;  /* triangle index or quadric index */
    int32_t material;     /* index into materials */
    int32_t area_light;   /* index into lights, or -1 */
} pbrtgpu_prim;

typedef struct pbrtgpu_triangle {
    int32_t mesh;         /* index into meshes */
    int32_t v[3];         /* global vertex indices (mesh->vertexIndex + mesh vert_offset) */
} pbrtgpu_triangle;

/* TriangleMesh (trianglemesh.cpp:33-63): positions are world space (P transformed at
 * construction), normals object space, uvs optional. */
typedef struct pbrtgpu_mesh {
    float o2w_m[16];      /* ObjectToWorld.m (row major) */
    float o2w_minv[16];   /* ObjectToWorld.mInv  (normals are transformed with this) */
    int32_t has_normals, has_uvs, reverse_orientation, swaps_handedness;
    int32_t vert_offset, nverts, pad0, pad1;
} pbrtgpu_mesh;

/* Sphere (sphere.cpp) / Disk (disk.cpp) / Cylinder (cylinder.cpp: radius, zmin, zmax, phi_max);
 * WorldToObject = (o2w_minv, o2w_m) */
typedef struct pbrtgpu_quadric {
    int32_t type;         /* PBRTGPU_SHAPE_SPHERE, _DISK or _CYLINDER */
    int32_t reverse_orientation, swaps_handedness, pad0;
    float o2w_m[16];
    float o2w_minv[16];
    float radius, zmin, zmax, theta_min, theta_max, phi_max, height, inner_radius;
} pbrtgpu_quadric;

enum {
    PBRTGPU_MAT_MATTE = 0,      /* spec[0]=Kd; f[0]=sigma (degrees) */
    PBRTGPU_MAT_PLASTIC = 1,    /* spec[0]=Kd, spec[1]=Ks; f[0]=roughness */
    PBRTGPU_MAT_METAL = 2,      /* spec[0]=eta, spec[1]=k; f[0]=roughness */
    PBRTGPU_MAT_SUBSTRATE = 3,  /* spec[0]=Kd, spec[1]=Ks; f[0]=uroughness, f[1]=vroughness */
    PBRTGPU_MAT_MIRROR = 4,     /* spec[0]=Kr */
    PBRTGPU_MAT_GLASS = 5,      /* spec[0]=Kr, spec[1]=Kt; f[0]=index */
    PBRTGPU_MAT_MEASURED = 6,   /* IrregIsotropicBRDF: aux = first kd-tree node, aux2 = node count */
    PBRTGPU_MAT_MEASURED_HALFANGLE = 7,  /* RegularHalfangleBRDF (.merl): aux = first texel of its
                                          * 90 x 90 x 180 RGB table in merl[] (3 floats per texel),
                                          * -1 when the file could not be read (no BxDF, as the
                                          * reference's MeasuredMaterial then adds none) */
    PBRTGPU_MAT_ANISOWARD = 8,  /* the fork's anisotropic Ward material (materials/anisoward.cpp,
                                 * AnisoWardBrdf.cpp): spec[0]=Kd, spec[1]=Ks; f[0]=alphaU, f[1]=alphaV */
    PBRTGPU_MAT_SHINYMETAL = 9  /* shinymetal.cpp: spec[0] = FresnelApproxEta(Ks.Clamp()), spec[1] =
                                 * FresnelApproxEta(Kr.Clamp()) (constant Ks / Kr), spec[2] = k = 0;
                                 * f[0]=roughness */
};

/* Texture<float> / Texture<Spectrum> (texture.h, textures/{constant,scale,imagemap}.cpp).
 * IMAGE textures are the reference's MIPMap (mipmap.h:119-193): the image ReadImage decodes
 * (TGA / PFM, imageio.cpp:443-650; a 1x1 RGB 0.5 image for other files, :45-66; the one-valued
 * powf(scale, gamma) map when a .tga / .pfm cannot be read, imagemap.cpp:64-70) after convertIn,
 * resampled to powers of two (Lanczos, clamped) and box-filtered into its pyramid; every level in
 * texels[] from texel_off (level l: max(1, width >> l) x max(1, height >> l) texels, row-major,
 * 3 floats (RGB) per texel for spectrum textures, 1 for float textures).  Lookups follow
 * MIPMap::Lookup (EWA, mipmap.h:278-375, or width-based / noFiltering, :232-259) with the
 * ImageWrap mode, texture coordinates from UVMapping2D (texture.cpp:80-90). */
enum { PBRTGPU_TEX_CONST = 0, PBRTGPU_TEX_IMAGE = 1, PBRTGPU_TEX_SCALE = 2, PBRTGPU_TEX_CHECKER = 3, PBRTGPU_TEX_UV = 4,
       PBRTGPU_TEX_MIX = 5, PBRTGPU_TEX_BILERP = 6 /* BilerpTexture: spectral v00, v01, v10, v11 at spec, spec + 1
       spectrum, ...; float at texels[texel_off .. + 3] */,
       /* float noise textures over IdentityMapping3D(tex2world) (map[16] = tex2world.m): FBmTexture,
          WrinkledTexture (octaves in levels, roughness / omega in value), WindyTexture */
       PBRTGPU_TEX_FBM = 7, PBRTGPU_TEX_WRINKLED = 8, PBRTGPU_TEX_WINDY = 9,
       /* DotsTexture (dots.h): tex1 = its "inside" parameter, tex2 = "outside" (the constructor
          stores them as outsideDot / insideDot), a 2D mapping; leaves as for CHECKER */
       PBRTGPU_TEX_DOTS = 10,
       /* MarbleTexture (marble.h, spectrum only): map = tex2world (IdentityMapping3D), levels =
          octaves, value = roughness, su = scale, sv = variation; spec = the first of the nine
          FromRGB spline colours, consecutive spectra */
       PBRTGPU_TEX_MARBLE = 11 };
enum { PBRTGPU_WRAP_REPEAT = 0, PBRTGPU_WRAP_BLACK = 1, PBRTGPU_WRAP_CLAMP = 2 };
typedef struct pbrtgpu_texture {
    int32_t type;          /* PBRTGPU_TEX_* */
    int32_t spectral;      /* 1: Texture<Spectrum> (value = FromRGB(reflectance) of the texel) */
    int32_t tex1, tex2;    /* SCALE operands (texture indices; CONST or IMAGE leaves) */
    int32_t spec;          /* CONST spectral: offset into spectra[] */
    int32_t wrap;          /* IMAGE: PBRTGPU_WRAP_* */
    int32_t trilinear;     /* IMAGE: doTrilinear || noFiltering (width-based lookup, no EWA) */
    int32_t nofilter;      /* IMAGE: noFiltering (the fork's nearest-texel lookup at level 0) */
    int32_t texel_off;     /* IMAGE: first float of level 0 in texels[] */
    int32_t width, height; /* IMAGE: level-0 resolution (powers of two) */
    int32_t levels;        /* IMAGE: nLevels = 1 + Log2Int(max(width, height)) */
    float value;           /* CONST float */
    float su, sv, du, dv;  /* UVMapping2D; PlanarMapping2D: du, dv are its ds, dt */
    float max_aniso;
    int32_t mapping;       /* IMAGE: PBRTGPU_MAP_* (the "mapping" parameter, imagemap.cpp:104-125) */
    float map[16];         /* SPHERICAL / CYLINDRICAL: WorldToTexture.m = Inverse(tex2world), row-major;
                              PLANAR: vs.xyz, vt.xyz (the "v1", "v2" parameters) */
    int32_t aamode;        /* CHECKER (Checkerboard2DTexture over tex1, tex2: CONST / IMAGE leaves, the
                              mapping above): 0 closedform box filter, 1 none (point sampled) */
    int32_t amount;        /* MIX ((1 - amount) * tex1 + amount * tex2, mix.h:38-43): the amount, a float
                              CONST / IMAGE texture */
} pbrtgpu_texture;
/* IMAGE and CHECKER nodes */
enum { PBRTGPU_MAP_UV = 0, PBRTGPU_MAP_SPHERICAL = 1, PBRTGPU_MAP_CYLINDRICAL = 2, PBRTGPU_MAP_PLANAR = 3 };

/* Material parameters.  A spectrum slot is either the constant spec[i] or, when
 * tex[i] >= 0, a spectrum texture evaluated per hit (at most two textured slots per material,
 * the most any reference material has: plastic / substrate Kd, Ks; glass Kr, Kt; metal eta, k).
 * The float parameters f[0], f[1] (matte sigma; plastic / metal roughness; substrate u / v
 * roughness; glass index) are the constants or, when ftex[j] >= 0, float textures evaluated per
 * hit (matte clamps sigma to [0, 90] as matte.cpp:54 does).  The bump displacement is the
 * constant f[7] or, when bump_tex >= 0, a float texture (Material::Bump, material.cpp:39-81, is
 * applied either way: bumpmap defaults to constant 0).
 * black_mask bit i: constant spec[i] IsBlack() (plastic/substrate/mirror skip such BxDFs);
 * bit 4 + i: textured slot i is used as evaluated, without the .Clamp() of the other materials
 * (metal eta and k, metal.cpp:64-65). */
typedef struct pbrtgpu_material {
    int32_t type;
    int32_t spec[4];      /* offsets (in floats) into spectra[] */
    int32_t aux, aux2;
    int32_t bump_tex;
    float f[8];
    int32_t tex[4];
    int32_t black_mask;
    int32_t normal_tex;   /* "normalmap" spectrum texture (Material::NormalMap, material.cpp:82-126, used
                           * where its value is not black), or -1 (the constant-0 default) */
    int32_t ftex[2];      /* float texture of f[0], f[1], or -1 (ABI 13; packs before v14 hold -1) */
} pbrtgpu_material;

/* area (DiffuseAreaLight), point (PointLight), infinite (InfiniteAreaLight), spot (SpotLight,
 * lights/spot.cpp), distant (DistantLight, lights/distant.cpp) */
enum { PBRTGPU_LIGHT_AREA = 0, PBRTGPU_LIGHT_POINT = 1, PBRTGPU_LIGHT_INFINITE = 2, PBRTGPU_LIGHT_SPOT = 3,
       PBRTGPU_LIGHT_DISTANT = 4 };

typedef struct pbrtgpu_light {
    int32_t type;
    int32_t spec;          /* Lemit (area) / intensity (point, spot) / L (infinite, distant), offset into spectra[] */
    int32_t shape_offset;  /* area: first entry in light_shapes[] (ShapeSet, light.cpp:114-135) */
    int32_t n_shapes;
    float sum_area;        /* ShapeSet::sumArea */
    float pos[3];          /* point / spot: the position LightToWorld(0,0,0); distant: lightDir =
                            * Normalize(LightToWorld(from - to)) */
    int32_t is_black;      /* emitted spectrum IsBlack() */
    int32_t n_samples;     /* Light::nSamples = max(1, "nsamples") (light.h:45); DirectLighting's
                            * strategy "all" takes RoundUpPow2 of it (LDSampler::RoundSize) */
    int32_t map_tex;       /* infinite, decoded environment image: its radiance MIPMap (an IMAGE
                            * texture of textures[], RGB, MIPMap defaults), or -1: the one texel below */
    int32_t dist_off;      /* infinite with map_tex: its Distribution2D in texels[] (infinite.cpp:93-109,
                            * montecarlo.h:134-160, montecarlo.cpp:350-362): marginal {funcInt,
                            * func[nv], cdf[nv + 1]}, then per row v {funcInt, func[nu], cdf[nu + 1]} */
    float l2w_m[16];
    float l2w_minv[16];
    /* infinite (InfiniteAreaLight, lights/infinite.cpp) without map_tex: the radiance MIPMap's
     * single texel (RGB, after L.ToRGBSpectrum()) with its wrap mode; Distribution2D of the
     * one-texel image: map_pdf = SampleContinuous's pdf, dist_pdf = Distribution2D::Pdf.  With
     * map_tex: dist_nu x dist_nv, the image's own resolution (before the MIPMap's resampling). */
    float texel[3];        /* spot: texel[0] = cosTotalWidth, texel[1] = cosFalloffStart (spot.cpp:35-36);
                            * l2w_m / l2w_minv its LightToWorld / WorldToLight */
    float map_pdf, dist_pdf;
    int32_t wrap, dist_nu, dist_nv;
} pbrtgpu_light;

typedef struct pbrtgpu_light_shape {
    int32_t shape_type, shape_index;
    float area;            /* Shape::Area() */
    float cdf;             /* Distribution1D cdf[i+1] of the area distribution */
} pbrtgpu_light_shape;

/* KdTree<IrregIsotropicBRDFSample> node (kdtree.h:37-55) with the sample stored at it:
 * p = BRDFRemap(wo, wi) of the measurement, spec = its spectrum (offset into spectra[]).
 * Nodes of one tree are contiguous; child indices are relative to the tree's first node. */
typedef struct pbrtgpu_kdnode {
    float p[3];
    float split_pos;
    int32_t split_axis;     /* 0..2, 3 = leaf */
    int32_t has_left;       /* left child = this node + 1 */
    int32_t right_child;    /* (1 << 29) - 1 if none */
    int32_t spec;
} pbrtgpu_kdnode;

/* TransformedPrimitive with an AnimatedTransform world->primitive (primitive.cpp:87-116,
 * transform.cpp:356-381): the top-level prim of shape_type PBRTGPU_SHAPE_INSTANCE points
 * here.  Its primitives (refined in object space) are prims[] entries whose prim_instance is
 * this index; they sit under the nested BVH rooted at node `root` (bvh.cpp, maxPrims 1),
 * or are the single primitive `single_prim` when refinement gave one primitive. */
typedef struct pbrtgpu_instance {
    int32_t root;             /* root node of the nested BVH, -1 if single_prim is used */
    int32_t single_prim;      /* the one primitive, -1 if root is used */
    int32_t animated;         /* AnimatedTransform::actuallyAnimated */
    int32_t pad0;
    float start_time, end_time, pad1, pad2;
    float start_m[16], start_minv[16];   /* world->primitive at start_time (m, mInv) */
    float end_m[16], end_minv[16];       /* ... at end_time */
    float T[2][4];            /* Decompose(): translation (xyz, 0) */
    float R[2][4];            /* Decompose(): rotation quaternion (x, y, z, w) */
    float S[2][16];           /* Decompose(): scale matrix */
} pbrtgpu_instance;

/* PerspectiveCamera (perspective.cpp, camera.cpp:84-103) + film/sample extent
 * (spectralImage.cpp:40-50, 176-185) */
typedef struct pbrtgpu_camera {
    float raster_to_camera[16];
    float cam2world_m[16];
    float lens_radius, focal_distance, shutter_open, shutter_close;
    int32_t xres, yres;
    int32_t px_start, px_count, py_start, py_count;   /* film pixel window */
    int32_t sx_start, sx_end, sy_start, sy_end;       /* sample extent (incl. border) */
    float dx_camera[3], dy_camera[3];                 /* dxCamera / dyCamera (perspective.cpp:45-48,
                                                       * orthographic.cpp:39-40) */
    int32_t ortho;        /* 1: OrthoCamera (cameras/orthographic.cpp): rays from Pcamera along +z,
                           * differentials from origins one pixel over */
    int32_t pad;
} pbrtgpu_camera;

/* RealisticDiffractionCamera (cameras/realisticDiffraction.cpp:32-94 parameters, 99-193
 * lens file, 347-468 Snell's law and element intersection, 478-1164 GenerateRay; ray
 * differentials by Camera::GenerateRayDifferential, camera.cpp:52-81): film rays traced from
 * the sensor through the lens elements, last element first; with "diffractionEnabled" each
 * element's exit direction is perturbed by a bivariate Gaussian (realisticDiffraction.cpp:
 * 1057-1150) drawn from the camera sample's own stream.  The light-field modes:
 * a pinhole array between lens and sensor (rays aim at the pinhole of their superpixel,
 * :248-304, 560-629), optionally with a two-surface microlens per pinhole (:614-876); and the
 * Gullstrand eye (IORforEyeEnabled, :196-205, 357-377): the ocular media's IOR spectra at the
 * ray's wavelength. */
typedef struct pbrtgpu_lens {
    int32_t n_elements;           /* lens-file elements, scene side first */
    int32_t chromatic;            /* chromaticAberrationEnabled: n + (lambda - 550) * -0.04 / 300 where n != 1 */
    float film_distance;          /* "filmdistance" */
    float film_diag;              /* "filmdiag" */
    float curve_radius;           /* "curveRadius" (0: flat sensor) */
    float aperture_offset[2];     /* "x_aperture_offset", "y_aperture_offset" */
    float film_center[2];         /* "film_center_x", "film_center_y" */
    float pinhole_exit[3];        /* "pinhole_exit_x/y/z": rays aim there unless one is -1 */
    float focal_length, fstop;    /* the lens file's first value; focal_length / "aperture_diameter" */
    int32_t diffraction;          /* "diffractionEnabled" (default true) */
    int32_t reserved;
    const float *elements;        /* [n_elements][4] radius, separation, n, aperture (an aperture stop,
                                   * radius 0, carries "aperture_diameter") */
    int32_t num_pinholes_w, num_pinholes_h;   /* "num_pinholes_w/h" (ints of the float parameters); both > 0:
                                               * the pinhole array */
    int32_t microlens;            /* "microlens_enabled": a microlens over every pinhole */
    int32_t ior_eye;              /* "IORforEyeEnabled" */
    const float *pinholes;        /* [num_pinholes_w][num_pinholes_h][3] the constructor's pinholeArray at the
                                   * film resolution (realisticDiffraction.cpp:248-304), or NULL */
    const float *eye_ior;         /* [4][n_bands] cornea, aqueous, lens, vitreous IOR spectra (Spectrum::
                                   * FromSampled of the camera's curves, :196-205), or NULL */
} pbrtgpu_lens;

typedef struct pbrtgpu_flat_scene {
    int32_t abi_version;
    int32_t n_bands;              /* nSpectralSamples */
    int32_t max_depth;            /* PathIntegrator maxdepth */
    int32_t spp;                  /* pixel samples (power of two) */
    uint32_t seed;                /* fixed-seed sampler seed */
    float y_int;                  /* SampledSpectrum::yint */
    const float *band_Y;          /* [n_bands] SampledSpectrum::Y */
    pbrtgpu_camera camera;
    int32_t n_nodes;   const pbrtgpu_bvh_node *nodes;
    int32_t n_prims;   const pbrtgpu_prim *prims;
    int32_t n_tris;    const pbrtgpu_triangle *tris;
    int32_t n_meshes;  const pbrtgpu_mesh *meshes;
    int32_t n_verts;   const float *vert_p;   /* [n_verts][3] world positions */
    const float *vert_n;                      /* [n_verts][3] object normals (0 if absent) */
    const float *vert_uv;                     /* [n_verts][2] (0 if absent) */
    int32_t n_quadrics; const pbrtgpu_quadric *quadrics;
    int32_t n_materials; const pbrtgpu_material *materials;
    int32_t n_lights;  const pbrtgpu_light *lights;
    int32_t n_light_shapes; const pbrtgpu_light_shape *light_shapes;
    int32_t n_spectra_floats; const float *spectra;   /* spectrum pool */
    int32_t n_instances; const pbrtgpu_instance *instances;
    const int32_t *prim_instance;                  /* [n_prims]: owning instance or -1 */
    int32_t n_kdnodes; const pbrtgpu_kdnode *kdnodes;   /* measured BRDF kd-trees */
    int32_t n_textures; const pbrtgpu_texture *textures;
    const float *ewa_lut;         /* [128] MIPMap::weightLut (mipmap.h:185-193) */
    const float *rgb_basis;       /* [14][n_bands] rgbRefl2Spect{White,Cyan,Magenta,Yellow,Red,
                                   * Green,Blue}, rgbIllum2Spect{...} (FromRGB, spectrum.cpp:93-178) */
    int32_t n_merl_floats;        /* RegularHalfangleBRDF tables: per texel RGB after the loader's
                                   * scale and clamp (measured.cpp:133-175), texel index
                                   * phiD + 180 * (thetaD + 90 * thetaH) */
    const float *merl;
    int32_t integrator;           /* PBRTGPU_INTEGRATOR_*: the scene's SurfaceIntegrator */
    int32_t dl_strategy;          /* DirectLighting "strategy": PBRTGPU_DL_ALL or PBRTGPU_DL_ONE */
    int32_t meta_strategy;        /* MetadataIntegrator "strategy": PBRTGPU_META_* */
    const uint32_t *prim_meta;    /* [n_prims][2]: the Intersection::primitiveId and ::materialId a hit
                                   * on the primitive reports (core/primitive.cpp:87-166; the
                                   * Primitive / Material constructor counters, primitive.h:40,
                                   * material.h:39), or NULL */
    int32_t renderer;             /* PBRTGPU_RENDERER_*: the scene's Renderer */
    int32_t wave_bands;           /* SpectralRenderer "nWaveBands" (api.cpp:1378, default 32) */
    int32_t spectral_sampling;    /* SpectralRenderer "samplingMethod": PBRTGPU_SPECTRAL_* */
    int32_t camera_type;          /* PBRTGPU_CAMERA_*: "perspective" / "orthographic" (camera) or "realisticDiffraction" (lens) */
    pbrtgpu_lens lens;
    int32_t n_texel_floats;       /* the MIPMap pyramids of the IMAGE textures (pbrtgpu_texture) */
    const float *texels;
    const pbrtgpu_instance *camera_motion;   /* an animated perspective camera's CameraToWorld
                                   * (AnimatedTransform, camera.cpp:84-103; start_m / end_m camera->world,
                                   * T / R / S their Decompose), or NULL: camera.cam2world_m */
} pbrtgpu_flat_scene;

/* SurfaceIntegrator of a flattened scene: "path" (integrators/path.cpp:44-115),
 * "directlighting" (integrators/directlighting.cpp:73-125, with the specular recursion of
 * core/integrator.cpp:169-250; max_depth is the integrator's "maxdepth" for both) or
 * "metadata" (integrators/metadata.cpp) */
enum { PBRTGPU_INTEGRATOR_PATH = 0, PBRTGPU_INTEGRATOR_DIRECT = 1, PBRTGPU_INTEGRATOR_METADATA = 2 };
enum { PBRTGPU_DL_ALL = 0, PBRTGPU_DL_ONE = 1 };
/* MetadataIntegrator (integrators/metadata.cpp:41-98): L = Spectrum(primitiveId),
 * Spectrum(materialId) or Spectrum(|hit point - ray origin|) at the camera ray's first hit */
enum { PBRTGPU_META_MESH = 0, PBRTGPU_META_MATERIAL = 1, PBRTGPU_META_DEPTH = 2 };
/* Renderer: "sampler" (renderers/samplerrenderer.cpp:60-247) or "spectralrenderer"
 * (renderers/spectralrenderer.cpp:60-223): per camera sample and wave band b of
 * nWaveBands, a path of wavelength 395 + dW b + dW / 2 (dW = 320 / nWaveBands, integer
 * division) whose radiance's value at that wavelength (Spectrum::GetValueAtWavelength,
 * spectrum.h:384-405) fills the sample's indices [dI b, min(dI (b + 1), N - 1)),
 * dI = N / nWaveBands.  singleDirection traces every band of every sample (nWaveBands paths
 * per sample, path b drawing from RNG(path_seed(hp, s nWaveBands + b))); samplerDirection
 * traces band s % nWaveBands of sample s only.  A sample's unassigned indices are 0. */
enum { PBRTGPU_RENDERER_SAMPLER = 0, PBRTGPU_RENDERER_SPECTRAL = 1 };
enum { PBRTGPU_CAMERA_PERSPECTIVE = 0, PBRTGPU_CAMERA_REALISTIC = 1, PBRTGPU_CAMERA_ORTHOGRAPHIC = 2 };
enum { PBRTGPU_SPECTRAL_SINGLE = 0, PBRTGPU_SPECTRAL_SAMPLER = 1 };

/* ---- render description ----------------------------------------------------------- */
/* Tiles are tile_w x tile_h blocks of the FILM pixel window (camera px_count x py_count;
 * the sample extent's half-pixel border belongs to no tile): tile id = ty * ntx + tx with
 * ntx = ceil(px_count / tile_w), nty = ceil(py_count / tile_h); the last row / column may be
 * ragged.  Rendering a tile renders the camera samples of its pixels, plus the samples of any
 * other sample pixel whose box footprint reaches one of them (spectralImage.cpp:80-92), so
 * films of disjoint tile sets are disjoint and sum to the full-frame film. */
typedef struct pbrtgpu_render_desc {
    int32_t spp_begin, spp_end;   /* sample index range [begin,end) of this call */
    int32_t tile_w, tile_h;       /* tile size in film pixels (<= 0: 16) */
    int32_t flags;                /* PBRTGPU_F_* */
    int32_t reserved[3];
} pbrtgpu_render_desc;

#define PBRTGPU_F_ACCUMULATE 1    /* add into the context film instead of clearing it */
#define PBRTGPU_F_COUNT_WORK 2    /* instrumented traversal kernels: fill pbrtgpu_timing.work */

/* stats_out layout (doubles) */
enum {
    PBRTGPU_STAT_PATHS = 0,       /* paths traced: camera samples x SpectralRenderer bands per sample */
    PBRTGPU_STAT_KERNEL_MS = 1,   /* device time of the path kernels (trace + shade) */
    PBRTGPU_STAT_ACCUM_MS = 2,    /* device time of the film accumulation */
    PBRTGPU_STAT_ZEROED = 3,      /* samples zeroed by the NaN/negative/inf guard */
    PBRTGPU_STAT_SPILLS = 4,      /* exact-boundary samples added to neighbour pixels */
    PBRTGPU_STAT_PASSES = 5,      /* wavefront passes */
    PBRTGPU_STAT_COUNT = 8
};

typedef struct pbrtgpu_ctx pbrtgpu_ctx;

int pbrtgpu_abi_version(void);
int pbrtgpu_device_count(void);
int pbrtgpu_context_create(int device, pbrtgpu_ctx **out);
int pbrtgpu_context_destroy(pbrtgpu_ctx *ctx);
const char *pbrtgpu_last_error(void);
/* copies the flattened scene into device memory owned by ctx */
int pbrtgpu_scene_upload(pbrtgpu_ctx *ctx, const pbrtgpu_flat_scene *scene);
/* Renders the listed tiles for samples [spp_begin, spp_end) into the context's film (the
 * film is cleared first unless PBRTGPU_F_ACCUMULATE is set or spp_begin > 0).
 * tile_ids == NULL means every tile. stats_out ([PBRTGPU_STAT_COUNT]) may be NULL.
 * One call over the whole sample range adds every pixel's samples in the reference's order
 * (SamplerRendererTask::Run + AddSample).  A frame split into sample ranges and accumulated
 * adds the same contributions range by range: its film equals the one-call film up to float
 * summation order.
 * Replaces SamplerRenderer::Render (renderers/samplerrenderer.cpp:188-222) for the tiles'
 * share of the frame; the tiles play the role of ComputeSubWindow's task windows
 * (core/sampler.cpp:47-67). */
int pbrtgpu_render_tiles(pbrtgpu_ctx *ctx, const pbrtgpu_render_desc *desc,
                         const int32_t *tile_ids, int32_t ntiles, double *stats_out);
/* Host gather of a tile list: writes the film pixels of the listed tiles (grid as in
 * pbrtgpu_render_desc) into film_out (float32 [py_count][px_count][n_bands], n_floats >= its
 * size); other pixels of film_out are left untouched.  tile_ids == NULL copies the whole film. */
int pbrtgpu_film_gather(pbrtgpu_ctx *ctx, int32_t tile_w, int32_t tile_h, const int32_t *tile_ids,
                        int32_t ntiles, float *film_out, int64_t n_floats);
/* One frame over n contexts (one per GPU, each holding the same uploaded scene; no RCCL, no
 * device-to-device traffic).  The tile list (tile_ids, or every tile when NULL) is dealt into
 * m = n * max(1, slices_per_ctx) interleaved slices (slice j = list[j], list[j + m], ...);
 * one host thread per context pulls slices from a shared atomic counter and renders each
 * with pbrtgpu_render_tiles (its first slice clears the context film unless desc asks to
 * accumulate), then gathers its tiles into film_out (pbrtgpu_film_gather).  Films of
 * different contexts cover disjoint pixels, so film_out is the full-frame film bit for bit.
 * stats_out ([n][PBRTGPU_STAT_COUNT], may be NULL): per-context sums.  Returns the first
 * context's error, if any. */
int pbrtgpu_render_multi(pbrtgpu_ctx *const *ctxs, int32_t n, const pbrtgpu_render_desc *desc,
                         const int32_t *tile_ids, int32_t ntiles, int32_t slices_per_ctx,
                         float *film_out, int64_t n_floats, double *stats_out);
/* Copies the film (float32 [py_count][px_count][n_bands], Σ L per pixel -- the
 * reference film does not normalise) to host memory. */
int pbrtgpu_film_read(pbrtgpu_ctx *ctx, float *film_out, int64_t n_floats);
int pbrtgpu_film_clear(pbrtgpu_ctx *ctx);
/* Per-path radiance for a list of path keys (x, y, s): debugging / parity hook.
 * keys: [n][3] int32; out: [n][n_bands] float32 (after the NaN/inf guard). */
int pbrtgpu_trace_paths(pbrtgpu_ctx *ctx, const int32_t *keys, int32_t n, float *out);
/* Closest-hit / any-hit queries for n rays (parity hook for BVHAccel::Intersect/IntersectP):
 * rays [n][8] = o.xyz, d.xyz, mint, maxt ; hits_out [n][4] = t, b1, b2, prim (as float bits),
 * prim = -1 on miss; occluded_out [n] (may be NULL). */
int pbrtgpu_intersect(pbrtgpu_ctx *ctx, const float *rays, int32_t n, float *hits_out,
                      int32_t *occluded_out);
/* The first n outputs of the path RNG as the device draws them (parity hook for RNG,
 * core/rng.cpp:35-100: Seed(seed) then n RandomUInt()): the 5-word window for outputs 0-226,
 * the full 624-word state rebuilt at output 227 and twisted every 624 after it (device.h
 * mt_uint_ext).  out [n] uint32.  Needs no scene. */
int pbrtgpu_mt_sequence(pbrtgpu_ctx *ctx, uint32_t seed, int32_t n, uint32_t *out);
/* Parity hook for the float transcendentals (include/pbrt_libmf.h, the reference's glibc routines
 * restated): out[i] = f(x[i]) -- or f(x[i], y[i]) for powf / atan2f -- evaluated by
 * the same device functions the shading kernels call.  fn: PBRTGPU_LIBMF_*; sincosf writes
 * (sin, cos) pairs (out [2n]).  Needs no scene. */
enum { PBRTGPU_LIBMF_SINF = 0, PBRTGPU_LIBMF_COSF, PBRTGPU_LIBMF_SINCOSF, PBRTGPU_LIBMF_EXPF, PBRTGPU_LIBMF_LOGF,
       PBRTGPU_LIBMF_ACOSF, PBRTGPU_LIBMF_ATANF, PBRTGPU_LIBMF_TANF, PBRTGPU_LIBMF_POWF, PBRTGPU_LIBMF_ATAN2F,
       PBRTGPU_LIBMF_COUNT };
int pbrtgpu_libmf_eval(pbrtgpu_ctx *ctx, int32_t fn, int64_t n, const float *x, const float *y, float *out);
/* GPU BVH build (the host front end's SAH build restates
 * accelerators/bvh.cpp:145-351 node for node and stays the default, since the bit-exact
 * traversal order rests on it).  A linear BVH (Morton codes, radix sort, Karras radix tree,
 * bottom-up bounds) over n primitives' world bounds [n][6] = bmin.xyz, bmax.xyz, returned in
 * the LinearBVHNode layout above with one primitive per leaf: nodes_out [2n-1];
 * order_out [n] = the original index of the primitive at leaf position j, i.e. the new
 * orderedPrims (prims[], prim_instance[] and prim_meta[] are permuted by it).  Deterministic.
 * ms_out [2] (may be NULL): device time of the build, wall time of the call.  Returns the
 * node count (2n - 1) or a negative error.  Scenes with instances keep the host build. */
int pbrtgpu_build_bvh(pbrtgpu_ctx *ctx, int32_t n, const float *bounds, pbrtgpu_bvh_node *nodes_out,
                      int32_t *order_out, double *ms_out);
/* GPU Loop subdivision (shapes/loopsubdiv.cpp:147-437): the control mesh
 * vi [nf][3] over P [nv][3] (object space) refined by n_levels levels to its limit surface,
 * with every float operation in the reference's order (csrc/loopsubdiv.hip): *n_verts_out
 * vertices, P_out / N_out [*n_verts_out][3] limit positions and normals (object space),
 * vi_out [nf * 4^n_levels][3]; with P_out NULL only *n_verts_out is set.  ms_out [2] (may be
 * NULL): device time, wall time of the call.  Every vertex must belong to a face. */
int pbrtgpu_loop_subdivide(pbrtgpu_ctx *ctx, int32_t nf, int32_t nv, const int32_t *vi, const float *P,
                           int32_t n_levels, int32_t *n_verts_out, float *P_out, float *N_out, int32_t *vi_out,
                           double *ms_out);
/* The same with pbrthost_set_loop_subdivider's signature (user = the pbrtgpu_ctx), so the
 * host front end refines its loopsubdiv shapes on the GPU. */
int pbrtgpu_loop_subdivide_hook(void *ctx, int32_t nf, int32_t nv, const int32_t *vi, const float *P,
                                int32_t n_levels, int32_t *n_verts_out, float *P_out, float *N_out, int32_t *vi_out);
/* Instrumented traversal statistics for a list of path keys (roofline model): counters_out
 * [6] = closest-hit rays, shadow rays, BVH nodes visited, triangle tests, quadric tests,
 * closest hits. */
int pbrtgpu_path_stats(pbrtgpu_ctx *ctx, const int32_t *keys, int32_t n, uint64_t *counters_out);
/* Per-kernel device time of the last render / trace call (HIP events on the context's
 * stream), for roofline reporting.  Index: 0 closest-hit trace, 1 shadow trace, 2 shade
 * (+ path regeneration), 3 film accumulation.  work[] (with PBRTGPU_F_COUNT_WORK, or after
 * pbrtgpu_path_stats): closest rays, shadow rays, BVH nodes visited by closest rays, by
 * shadow rays, triangle tests by closest rays, by shadow rays, quadric tests by closest
 * rays, by shadow rays, closest hits, MIS rays (among the closest rays), MIS hits, 0. */
typedef struct pbrtgpu_timing {
    double ms[4];
    int32_t launches[4];
    int32_t passes;
    int32_t shade_feat;   /* the scene's FEAT_* bits, which select the k_shade variant (csrc/scene_build.h,
                             pbrtgpu.hip path_shade_variant): 1 measured BRDFs, 2 textures, 4 infinite /
                             spot / distant lights, | 8 when every material is matte / plastic (or
                             measured), | 16 when otherwise matte / plastic / metal / substrate:
                             0 and 8 = lean, 7 = full */
    uint64_t work[12];
} pbrtgpu_timing;
int pbrtgpu_last_timing(pbrtgpu_ctx *ctx, pbrtgpu_timing *out);

#ifdef __cplusplus
}
#endif
#endif /* PBRTGPU_H */
