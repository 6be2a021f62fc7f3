// pbrtgpu.hip -- MI355X (gfx950) spectral path-tracing core behind the C ABI of
// include/pbrtgpu.h.  Replaces SamplerRenderer::Render's task loop
// (renderers/samplerrenderer.cpp:60-222) for the "path" SurfaceIntegrator.
//
// Pipeline per pbrtgpu_render_tiles call:
//   k_spill_scan   : every sample of the sample extent -> imageX/Y footprint; samples that
//                    land on a film pixel of this context other than their own are queued
//                    (integer + float sampler work only, no tracing)
//   k_trace_keys   : traces the queued spill samples (radiance kept for the film pass)
//   k_apply        : adds "pre" spill contributions (sources earlier in row-major order)
//   for each spp batch:
//     k_render<NB> : persistent grid; one camera path per lane per item, items
//                    (pixel, sample) interleaved with grid stride; the whole
//                    PathIntegrator::Li bounce loop runs in registers with the BVH
//                    traversal stack in LDS; writes L[NB] per item
//     k_accum<NB>  : film[p][band] += L in sample order (one lane per (pixel, band))
//   k_apply        : adds "post" spill contributions
// The film is the reference's raw sum (spectralImage.cpp:267-296 does not normalise).
#include <hip/hip_runtime.h>
#include <vector>
#include <string>
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <mutex>
#include "pbrtgpu.h"
#include "device.h"

using namespace pgd;

static thread_local std::string g_err;
static int fail(int code, const std::string &msg) { g_err = msg; return code; }
#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(-(1000 + (int)e_), std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

static const int kBlock = 128;

// ------------------------------------------------------------------ kernels
template <int NB>
__global__ __launch_bounds__(kBlock) void k_render(DevScene S, const int2 *__restrict__ pix, int nPix, int s0,
                                                    int sb, float *__restrict__ Lbuf, unsigned int *__restrict__ zeroed) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.stride = blockDim.x;
    const long nItems = (long)nPix * sb;
    unsigned int bad = 0;
    for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < nItems; it += (long)gridDim.x * blockDim.x) {
        int p = (int)(it / sb);
        int sl = (int)(it - (long)p * sb);
        int2 xy = pix[p];
        float L[NB];
        bad += trace_path<NB>(S, st, xy.x, xy.y, (uint32_t)(s0 + sl), L) ? 1u : 0u;
        float4 *o = reinterpret_cast<float4 *>(Lbuf + it * NB);
#pragma unroll
        for (int i = 0; i < NB / 4; ++i) o[i] = make_float4(L[4 * i], L[4 * i + 1], L[4 * i + 2], L[4 * i + 3]);
        if (NB % 4) {
#pragma unroll
            for (int i = (NB / 4) * 4; i < NB; ++i) Lbuf[it * NB + i] = L[i];
        }
    }
    if (bad) atomicAdd(zeroed, bad);
}

// film[filmIdx[p]][b] += L(p, s) for s in batch order (spectralImage.cpp:125-131)
template <int NB>
__global__ void k_accum(const float *__restrict__ Lbuf, const int *__restrict__ filmIdx, int nPix, int sb,
                        float *__restrict__ film) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nPix * NB) return;
    int p = (int)(t / NB), b = (int)(t - (long)p * NB);
    float acc = film[(long)filmIdx[p] * NB + b];
    const float *src = Lbuf + (long)p * sb * NB + b;
    for (int s = 0; s < sb; ++s) acc += 1.f * src[(long)s * NB];
    film[(long)filmIdx[p] * NB + b] = acc;
}

// spill scan over the sample extent: queue samples that land on a masked film pixel
// other than their own sample pixel (spectralImage.cpp:80-92, box filter width 0.5)
__global__ void k_spill_scan(pbrtgpu_camera cam, uint32_t seed, int spp, const uint8_t *__restrict__ mask,
                             int3 *__restrict__ keys, unsigned int *__restrict__ count, unsigned int cap) {
    const int ew = cam.sx_end - cam.sx_start, eh = cam.sy_end - cam.sy_start;
    const long n = (long)ew * eh * spp;
    for (long it = (long)blockIdx.x * blockDim.x + threadIdx.x; it < n; it += (long)gridDim.x * blockDim.x) {
        long pi = it / spp;
        int s = (int)(it - pi * spp);
        int x = cam.sx_start + (int)(pi % ew), y = cam.sy_start + (int)(pi / ew);
        uint32_t hp = pixel_hash(seed, x, y);
        float u[2];
        s2d(hp, 0, (uint32_t)s, (uint32_t)spp, u);
        float ix = x + u[0], iy = y + u[1];
        float dx = ix - 0.5f, dy = iy - 0.5f;
        int fx0 = (int)ceilf(dx - 0.5f), fx1 = (int)floorf(dx + 0.5f);
        int fy0 = (int)ceilf(dy - 0.5f), fy1 = (int)floorf(dy + 0.5f);
        fx0 = max(fx0, cam.px_start); fx1 = min(fx1, cam.px_start + cam.px_count - 1);
        fy0 = max(fy0, cam.py_start); fy1 = min(fy1, cam.py_start + cam.py_count - 1);
        if (fx1 - fx0 < 0 || fy1 - fy0 < 0) continue;
        if (fx0 == x && fx1 == x && fy0 == y && fy1 == y) continue;
        bool any = false;
        for (int fy = fy0; fy <= fy1; ++fy)
            for (int fx = fx0; fx <= fx1; ++fx)
                if (!(fx == x && fy == y) && mask[(long)(fy - cam.py_start) * cam.px_count + (fx - cam.px_start)]) any = true;
        if (!any) continue;
        unsigned int k = atomicAdd(count, 1u);
        if (k < cap) keys[k] = make_int3(x, y, s);
    }
}

template <int NB>
__global__ __launch_bounds__(kBlock) void k_trace_keys(DevScene S, const int3 *__restrict__ keys, int n,
                                                        float *__restrict__ out) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.stride = blockDim.x;
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int3 key = keys[k];
    float L[NB];
    trace_path<NB>(S, st, key.x, key.y, (uint32_t)key.z, L);
#pragma unroll
    for (int i = 0; i < NB; ++i) out[(long)k * NB + i] = L[i];
}

// instrumented variant: per-path work counters for the algorithmic-bytes model
template <int NB>
__global__ __launch_bounds__(kBlock) void k_stats(DevScene S, const int3 *__restrict__ keys, int n,
                                                   unsigned long long *__restrict__ counters) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.stride = blockDim.x;
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int3 key = keys[k];
    float L[NB];
    trace_path<NB>(S, st, key.x, key.y, (uint32_t)key.z, L);
    atomicAdd(&counters[0], (unsigned long long)st.cRays);
    atomicAdd(&counters[1], (unsigned long long)st.cShadow);
    atomicAdd(&counters[2], (unsigned long long)st.cNodes);
    atomicAdd(&counters[3], (unsigned long long)st.cTris);
    atomicAdd(&counters[4], (unsigned long long)st.cQuads);
    atomicAdd(&counters[5], (unsigned long long)st.cHits);
}

// ordered contribution lists: for target t, entries [start[t], start[t+1]) of src in order
__global__ void k_apply(int nTargets, const int *__restrict__ tgt, const int *__restrict__ start,
                        const int *__restrict__ src, const float *__restrict__ Lsp, int nb, float *__restrict__ film) {
    long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)nTargets * nb) return;
    int q = (int)(t / nb), b = (int)(t - (long)q * nb);
    float acc = film[(long)tgt[q] * nb + b];
    for (int e = start[q]; e < start[q + 1]; ++e) acc += 1.f * Lsp[(long)src[e] * nb + b];
    film[(long)tgt[q] * nb + b] = acc;
}

__global__ __launch_bounds__(kBlock) void k_intersect(DevScene S, const float *__restrict__ rays, int n,
                                                       float *__restrict__ hits, int *__restrict__ occ) {
    extern __shared__ uint32_t lds[];
    Stack st;
    st.base = lds + threadIdx.x;
    st.stride = blockDim.x;
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float *q = rays + 8 * k;
    Ray r;
    r.o = v3(q[0], q[1], q[2]); r.d = v3(q[3], q[4], q[5]); r.mint = q[6]; r.maxt = q[7]; r.time = 0.f;
    Ray r2 = r;
    int prim = -1;
    float t = INFINITY;
    if (!bvh_intersect(S, st, r, &prim, &t)) { prim = -1; t = INFINITY; }
    hits[4 * k] = t; hits[4 * k + 1] = 0.f; hits[4 * k + 2] = 0.f; hits[4 * k + 3] = __int_as_float(prim);
    occ[k] = bvh_intersectP(S, st, r2) ? 1 : 0;
}

// ------------------------------------------------------------------ context
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) n = bytes;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

struct pbrtgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool hasScene = false;
    DevScene S{};
    int nb = 0, spp = 0, stackDepth = 0;
    pbrtgpu_camera cam{};
    std::vector<DevBuf> sceneBufs;
    DevBuf film, Lbuf, pix, filmIdx, mask, keys, counter, spillL, zeroed, lists[4], scratch[3];
    int numCUs = 256;
    double lastKernelMs = 0.0;
    int lastLaunches = 0;
};

template <class T> static hipError_t upload(pbrtgpu_ctx *c, const T *src, size_t count, const T **dst) {
    c->sceneBufs.emplace_back();
    DevBuf &b = c->sceneBufs.back();
    size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = b.ensure(bytes);
    if (e != hipSuccess) return e;
    if (count) e = hipMemcpy(b.p, src, count * sizeof(T), hipMemcpyHostToDevice);
    *dst = reinterpret_cast<const T *>(b.p);
    return e;
}

extern "C" {

int pbrtgpu_abi_version(void) { return PBRTGPU_ABI_VERSION; }
const char *pbrtgpu_last_error(void) { return g_err.c_str(); }

int pbrtgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pbrtgpu_context_create(int device, pbrtgpu_ctx **out) {
    if (!out) return fail(PBRTGPU_E_INVALID, "null out");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(PBRTGPU_E_NODEVICE, "no HIP device");
    if (device < 0 || device >= n) return fail(PBRTGPU_E_INVALID, "bad device index");
    HIPCHK(hipSetDevice(device));
    pbrtgpu_ctx *c = new pbrtgpu_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->numCUs = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return fail(PBRTGPU_E_NODEVICE, "stream/event creation failed");
    }
    *out = c;
    return 0;
}

int pbrtgpu_context_destroy(pbrtgpu_ctx *c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto &b : c->sceneBufs) b.release();
    DevBuf *bufs[] = {&c->film, &c->Lbuf, &c->pix, &c->filmIdx, &c->mask, &c->keys, &c->counter, &c->spillL,
                      &c->zeroed, &c->lists[0], &c->lists[1], &c->lists[2], &c->lists[3], &c->scratch[0],
                      &c->scratch[1], &c->scratch[2]};
    for (DevBuf *b : bufs) b->release();
    (void)hipEventDestroy(c->ev0);
    (void)hipEventDestroy(c->ev1);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int pbrtgpu_scene_upload(pbrtgpu_ctx *c, const pbrtgpu_flat_scene *s) {
    if (!c || !s) return fail(PBRTGPU_E_INVALID, "null argument");
    if (s->abi_version != PBRTGPU_ABI_VERSION) return fail(PBRTGPU_E_INVALID, "ABI version mismatch");
    if (!(s->n_bands == 32 || s->n_bands == 60 || s->n_bands == 30))
        return fail(PBRTGPU_E_UNSUPPORTED, "n_bands must be 30, 32 or 60");
    if (s->spp <= 0 || (s->spp & (s->spp - 1))) return fail(PBRTGPU_E_INVALID, "spp must be a power of two");
    if (s->max_depth < 0 || s->max_depth > 20)
        return fail(PBRTGPU_E_UNSUPPORTED, "maxdepth > 20 exceeds the first MT19937 block (DESIGN.md §3.1)");
    if (s->n_nodes <= 0 || s->n_prims <= 0) return fail(PBRTGPU_E_INVALID, "empty scene");
    for (int i = 0; i < s->n_lights; ++i)
        if (s->lights[i].type == PBRTGPU_LIGHT_INFINITE) return fail(PBRTGPU_E_UNSUPPORTED, "infinite lights not yet supported");
    for (int i = 0; i < s->n_materials; ++i)
        if (s->materials[i].type > PBRTGPU_MAT_SUBSTRATE) return fail(PBRTGPU_E_UNSUPPORTED, "material type not yet supported on the GPU");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (auto &b : c->sceneBufs) b.release();
    c->sceneBufs.clear();
    c->sceneBufs.reserve(32);
    DevScene &S = c->S;
    S.nb = s->n_bands;
    S.maxDepth = s->max_depth;
    S.spp = s->spp;
    S.seed = s->seed;
    S.yint = s->y_int;
    S.cam = s->camera;
    S.nLights = s->n_lights;
    // BVH: verify topology and measure the stack depth traversal needs
    int maxDepth = 0;
    {
        std::vector<std::pair<uint32_t, int> > todo;
        todo.push_back(std::make_pair(0u, 0));
        while (!todo.empty()) {
            auto q = todo.back();
            todo.pop_back();
            if (q.first >= (uint32_t)s->n_nodes) return fail(PBRTGPU_E_INVALID, "BVH node index out of range");
            const pbrtgpu_bvh_node &n = s->nodes[q.first];
            maxDepth = std::max(maxDepth, q.second);
            if ((n.meta & 0xff) == 0) {
                if (q.second > 62) return fail(PBRTGPU_E_UNSUPPORTED, "BVH deeper than 63 levels");
                todo.push_back(std::make_pair(q.first + 1, q.second + 1));
                todo.push_back(std::make_pair(n.offset, q.second + 1));
            } else if (n.offset + (n.meta & 0xff) > (uint32_t)s->n_prims)
                return fail(PBRTGPU_E_INVALID, "BVH leaf out of range");
        }
    }
    c->stackDepth = maxDepth + 1;
    S.stackDepth = c->stackDepth;
    HIPCHK(upload(c, s->band_Y, (size_t)s->n_bands, &S.bandY));
    HIPCHK(upload(c, reinterpret_cast<const float4 *>(s->nodes), (size_t)s->n_nodes * 2, &S.nodes));
    HIPCHK(upload(c, s->prims, (size_t)s->n_prims, &S.prims));
    std::vector<DevTri> pt(s->n_prims);
    for (int i = 0; i < s->n_prims; ++i) {
        const pbrtgpu_prim &p = s->prims[i];
        DevTri t{};
        if (p.shape_type == PBRTGPU_SHAPE_TRIANGLE) {
            if (p.shape_index < 0 || p.shape_index >= s->n_tris) return fail(PBRTGPU_E_INVALID, "bad triangle index");
            const pbrtgpu_triangle &tr = s->tris[p.shape_index];
            const float *a = s->vert_p + 3 * tr.v[0], *b = s->vert_p + 3 * tr.v[1], *cc = s->vert_p + 3 * tr.v[2];
            t.a = make_float4(a[0], a[1], a[2], 0.f);
            t.b = make_float4(b[0], b[1], b[2], 0.f);
            t.c = make_float4(cc[0], cc[1], cc[2], 0.f);
        } else if (p.shape_index < 0 || p.shape_index >= s->n_quadrics)
            return fail(PBRTGPU_E_INVALID, "bad quadric index");
        pt[i] = t;
    }
    HIPCHK(upload(c, pt.data(), pt.size(), &S.primTri));
    HIPCHK(upload(c, s->tris, (size_t)s->n_tris, &S.tris));
    HIPCHK(upload(c, s->meshes, (size_t)s->n_meshes, &S.meshes));
    HIPCHK(upload(c, s->vert_p, (size_t)s->n_verts * 3, &S.vertP));
    HIPCHK(upload(c, s->vert_n, (size_t)s->n_verts * 3, &S.vertN));
    HIPCHK(upload(c, s->vert_uv, (size_t)s->n_verts * 2, &S.vertUV));
    HIPCHK(upload(c, s->quadrics, (size_t)s->n_quadrics, &S.quads));
    HIPCHK(upload(c, s->materials, (size_t)s->n_materials, &S.mats));
    HIPCHK(upload(c, s->lights, (size_t)s->n_lights, &S.lights));
    HIPCHK(upload(c, s->light_shapes, (size_t)s->n_light_shapes, &S.lightShapes));
    HIPCHK(upload(c, s->spectra, (size_t)s->n_spectra_floats, &S.spectra));
    c->nb = s->n_bands;
    c->spp = s->spp;
    c->cam = s->camera;
    size_t filmFloats = (size_t)s->camera.px_count * s->camera.py_count * s->n_bands;
    HIPCHK(c->film.ensure(filmFloats * 4));
    HIPCHK(hipMemsetAsync(c->film.p, 0, filmFloats * 4, c->stream));
    HIPCHK(c->zeroed.ensure(16));
    HIPCHK(c->counter.ensure(16));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->hasScene = true;
    return 0;
}

int pbrtgpu_film_clear(pbrtgpu_ctx *c) {
    if (!c || !c->hasScene) return fail(PBRTGPU_E_STATE, "no scene");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(c->film.p, 0, (size_t)c->cam.px_count * c->cam.py_count * c->nb * 4, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int pbrtgpu_film_read(pbrtgpu_ctx *c, float *out, int64_t n) {
    if (!c || !c->hasScene || !out) return fail(PBRTGPU_E_STATE, "no scene / null out");
    size_t need = (size_t)c->cam.px_count * c->cam.py_count * c->nb;
    if ((size_t)n < need) return fail(PBRTGPU_E_INVALID, "film buffer too small");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(out, c->film.p, need * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

}  // extern "C"

template <int NB>
static int render_impl(pbrtgpu_ctx *c, const pbrtgpu_render_desc *d, const int32_t *tiles, int32_t ntiles, double *stats) {
    const pbrtgpu_camera &cam = c->cam;
    const int spp = c->spp;
    int s0 = d->spp_begin, s1 = d->spp_end;
    if (s0 < 0 || s1 > spp || s0 >= s1) return fail(PBRTGPU_E_INVALID, "bad sample range");
    int tw = d->tile_w > 0 ? d->tile_w : 16, th = d->tile_h > 0 ? d->tile_h : 16;
    int ntx = (cam.px_count + tw - 1) / tw, nty = (cam.py_count + th - 1) / th;
    // pixel list of the requested tiles (film pixels; own sample pixel == film pixel)
    std::vector<int2> pix;
    std::vector<int> fidx;
    std::vector<uint8_t> mask((size_t)cam.px_count * cam.py_count, 0);
    auto addTile = [&](int t) {
        int tx = t % ntx, ty = t / ntx;
        for (int y = ty * th; y < std::min(cam.py_count, (ty + 1) * th); ++y)
            for (int x = tx * tw; x < std::min(cam.px_count, (tx + 1) * tw); ++x) {
                size_t fi = (size_t)y * cam.px_count + x;
                if (mask[fi]) continue;
                mask[fi] = 1;
                pix.push_back(make_int2(cam.px_start + x, cam.py_start + y));
                fidx.push_back((int)fi);
            }
    };
    if (!tiles) for (int t = 0; t < ntx * nty; ++t) addTile(t);
    else
        for (int i = 0; i < ntiles; ++i) {
            if (tiles[i] < 0 || tiles[i] >= ntx * nty) return fail(PBRTGPU_E_INVALID, "tile id out of range");
            addTile(tiles[i]);
        }
    const int nPix = (int)pix.size();
    double st[PBRTGPU_STAT_COUNT] = {0};
    if (!(d->flags & PBRTGPU_F_ACCUMULATE) && s0 == 0)
        HIPCHK(hipMemsetAsync(c->film.p, 0, (size_t)cam.px_count * cam.py_count * NB * 4, c->stream));
    if (nPix == 0) { if (stats) memcpy(stats, st, sizeof(st)); return 0; }
    HIPCHK(c->pix.ensure(pix.size() * sizeof(int2)));
    HIPCHK(c->filmIdx.ensure(fidx.size() * sizeof(int)));
    HIPCHK(hipMemcpyAsync(c->pix.p, pix.data(), pix.size() * sizeof(int2), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->filmIdx.p, fidx.data(), fidx.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    const size_t ldsBytes = (size_t)c->stackDepth * kBlock * sizeof(uint32_t);

    // ---- spill samples (only meaningful when the whole sample range is rendered)
    std::vector<int> preT, preStart, preSrc, postT, postStart, postSrc;
    int nSpill = 0;
    bool doSpills = (s0 == 0 && s1 == spp);
    if (doSpills) {
        HIPCHK(c->mask.ensure(mask.size()));
        HIPCHK(hipMemcpyAsync(c->mask.p, mask.data(), mask.size(), hipMemcpyHostToDevice, c->stream));
        unsigned int cap = 1u << 20;
        HIPCHK(c->keys.ensure((size_t)cap * sizeof(int3)));
        HIPCHK(hipMemsetAsync(c->counter.p, 0, 16, c->stream));
        long nsamp = (long)(cam.sx_end - cam.sx_start) * (cam.sy_end - cam.sy_start) * spp;
        int grid = (int)std::min<long>((nsamp + 255) / 256, (long)c->numCUs * 16);
        hipLaunchKernelGGL(k_spill_scan, dim3(grid), dim3(256), 0, c->stream, cam, c->S.seed, spp,
                           (const uint8_t *)c->mask.p, (int3 *)c->keys.p, (unsigned int *)c->counter.p, cap);
        HIPCHK(hipGetLastError());
        unsigned int cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, c->counter.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (cnt > cap) return fail(PBRTGPU_E_UNSUPPORTED, "too many exact-boundary samples");
        nSpill = (int)cnt;
        if (nSpill > 0) {
            std::vector<int3> keys(nSpill);
            HIPCHK(hipMemcpy(keys.data(), c->keys.p, nSpill * sizeof(int3), hipMemcpyDeviceToHost));
            // canonical order: (source row-major, sample)
            std::sort(keys.begin(), keys.end(), [](const int3 &a, const int3 &b) {
                if (a.y != b.y) return a.y < b.y;
                if (a.x != b.x) return a.x < b.x;
                return a.z < b.z;
            });
            HIPCHK(hipMemcpy(c->keys.p, keys.data(), nSpill * sizeof(int3), hipMemcpyHostToDevice));
            HIPCHK(c->spillL.ensure((size_t)nSpill * NB * 4));
            hipLaunchKernelGGL(k_trace_keys<NB>, dim3((nSpill + kBlock - 1) / kBlock), dim3(kBlock), ldsBytes, c->stream,
                               c->S, (const int3 *)c->keys.p, nSpill, (float *)c->spillL.p);
            HIPCHK(hipGetLastError());
            // contributions per target pixel, split into pre (source before the target's own
            // sample pixel in row-major order) and post
            const int ew = cam.sx_end - cam.sx_start;
            struct Cb { int target; long src; int s; int idx; };
            std::vector<Cb> cbs;
            for (int k = 0; k < nSpill; ++k) {
                int x = keys[k].x, y = keys[k].y, s = keys[k].z;
                uint32_t hp = pixel_hash(c->S.seed, x, y);
                float u[2];
                s2d(hp, 0, (uint32_t)s, (uint32_t)spp, u);   // same sampler as k_spill_scan
                float u0 = u[0], u1 = u[1];
                float ix = x + u0, iy = y + u1;
                float dx = ix - 0.5f, dy = iy - 0.5f;
                int fx0 = (int)ceilf(dx - 0.5f), fx1 = (int)floorf(dx + 0.5f);
                int fy0 = (int)ceilf(dy - 0.5f), fy1 = (int)floorf(dy + 0.5f);
                fx0 = std::max(fx0, cam.px_start); fx1 = std::min(fx1, cam.px_start + cam.px_count - 1);
                fy0 = std::max(fy0, cam.py_start); fy1 = std::min(fy1, cam.py_start + cam.py_count - 1);
                for (int fy = fy0; fy <= fy1; ++fy)
                    for (int fx = fx0; fx <= fx1; ++fx) {
                        if (fx == x && fy == y) continue;
                        int target = (fy - cam.py_start) * cam.px_count + (fx - cam.px_start);
                        if (!mask[target]) continue;
                        cbs.push_back(Cb{target, (long)(y - cam.sy_start) * ew + (x - cam.sx_start), s, k});
                    }
            }
            std::sort(cbs.begin(), cbs.end(), [](const Cb &a, const Cb &b) {
                if (a.target != b.target) return a.target < b.target;
                if (a.src != b.src) return a.src < b.src;
                return a.s < b.s;
            });
            for (size_t i = 0; i < cbs.size(); ++i) {
                const Cb &q = cbs[i];
                int tx = q.target % cam.px_count + cam.px_start, ty = q.target / cam.px_count + cam.py_start;
                long own = (long)(ty - cam.sy_start) * ew + (tx - cam.sx_start);
                bool pre = q.src < own;
                std::vector<int> &T = pre ? preT : postT, &ST = pre ? preStart : postStart, &SR = pre ? preSrc : postSrc;
                if (T.empty() || T.back() != q.target) { T.push_back(q.target); ST.push_back((int)SR.size()); }
                SR.push_back(q.idx);
            }
            preStart.push_back((int)preSrc.size());
            postStart.push_back((int)postSrc.size());
            st[PBRTGPU_STAT_SPILLS] = (double)cbs.size();
        }
    }
    auto applyLists = [&](std::vector<int> &T, std::vector<int> &ST, std::vector<int> &SR) -> int {
        if (T.empty()) return 0;
        HIPCHK(c->lists[0].ensure(T.size() * 4));
        HIPCHK(c->lists[1].ensure(ST.size() * 4));
        HIPCHK(c->lists[2].ensure(SR.size() * 4));
        HIPCHK(hipMemcpyAsync(c->lists[0].p, T.data(), T.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->lists[1].p, ST.data(), ST.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->lists[2].p, SR.data(), SR.size() * 4, hipMemcpyHostToDevice, c->stream));
        long n = (long)T.size() * NB;
        hipLaunchKernelGGL(k_apply, dim3((n + 255) / 256), dim3(256), 0, c->stream, (int)T.size(), (const int *)c->lists[0].p,
                           (const int *)c->lists[1].p, (const int *)c->lists[2].p, (const float *)c->spillL.p, NB,
                           (float *)c->film.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->stream));   // host vectors are reused right after
        return 0;
    };
    if (int e = applyLists(preT, preStart, preSrc)) return e;

    // ---- main batches
    const size_t lbudget = (size_t)1 << 30;   // 1 GiB of per-sample radiance per batch
    int sb = (int)std::max<long>(1, std::min<long>(s1 - s0, (long)(lbudget / ((size_t)nPix * NB * 4))));
    HIPCHK(c->Lbuf.ensure((size_t)nPix * sb * NB * 4));
    HIPCHK(hipMemsetAsync(c->zeroed.p, 0, 16, c->stream));
    float kms = 0.f, ams = 0.f;
    int launches = 0;
    hipEvent_t ea, eb, ec;
    HIPCHK(hipEventCreate(&ea)); HIPCHK(hipEventCreate(&eb)); HIPCHK(hipEventCreate(&ec));
    // persistent grid: resident blocks per CU from the LDS stack footprint (<= 8 per CU)
    int perCU = std::max(1, std::min(8, (int)(160 * 1024 / std::max<size_t>(ldsBytes, 1))));
    for (int b0 = s0; b0 < s1; b0 += sb) {
        int n = std::min(sb, s1 - b0);
        long items = (long)nPix * n;
        int grid = (int)std::min<long>((items + kBlock - 1) / kBlock, (long)c->numCUs * perCU);
        HIPCHK(hipEventRecord(ea, c->stream));
        hipLaunchKernelGGL(k_render<NB>, dim3(grid), dim3(kBlock), ldsBytes, c->stream, c->S, (const int2 *)c->pix.p, nPix,
                           b0, n, (float *)c->Lbuf.p, (unsigned int *)c->zeroed.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(eb, c->stream));
        long na = (long)nPix * NB;
        hipLaunchKernelGGL(k_accum<NB>, dim3((na + 255) / 256), dim3(256), 0, c->stream, (const float *)c->Lbuf.p,
                           (const int *)c->filmIdx.p, nPix, n, (float *)c->film.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ec, c->stream));
        HIPCHK(hipEventSynchronize(ec));
        float m1 = 0.f, m2 = 0.f;
        HIPCHK(hipEventElapsedTime(&m1, ea, eb));
        HIPCHK(hipEventElapsedTime(&m2, eb, ec));
        kms += m1; ams += m2; ++launches;
        st[PBRTGPU_STAT_PATHS] += (double)items;
    }
    (void)hipEventDestroy(ea); (void)hipEventDestroy(eb); (void)hipEventDestroy(ec);
    if (int e = applyLists(postT, postStart, postSrc)) return e;
    unsigned int z = 0;
    HIPCHK(hipMemcpyAsync(&z, c->zeroed.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    st[PBRTGPU_STAT_KERNEL_MS] = kms;
    st[PBRTGPU_STAT_ACCUM_MS] = ams;
    st[PBRTGPU_STAT_ZEROED] = z;
    c->lastKernelMs = launches ? kms / launches : 0.0;
    c->lastLaunches = launches;
    if (stats) memcpy(stats, st, sizeof(st));
    return 0;
}

extern "C" {

int pbrtgpu_render_tiles(pbrtgpu_ctx *c, const pbrtgpu_render_desc *d, const int32_t *tile_ids, int32_t ntiles,
                         double *stats) {
    if (!c || !c->hasScene || !d) return fail(PBRTGPU_E_STATE, "no scene / null desc");
    HIPCHK(hipSetDevice(c->device));
    switch (c->nb) {
        case 32: return render_impl<32>(c, d, tile_ids, ntiles, stats);
        case 60: return render_impl<60>(c, d, tile_ids, ntiles, stats);
        case 30: return render_impl<30>(c, d, tile_ids, ntiles, stats);
    }
    return fail(PBRTGPU_E_UNSUPPORTED, "band count");
}

}  // extern "C"

template <int NB>
static int trace_impl(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, float *out) {
    HIPCHK(c->scratch[0].ensure((size_t)n * sizeof(int3)));
    HIPCHK(c->scratch[1].ensure((size_t)n * NB * 4));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, keys, (size_t)n * 12, hipMemcpyHostToDevice, c->stream));
    size_t lds = (size_t)c->stackDepth * kBlock * 4;
    hipLaunchKernelGGL(k_trace_keys<NB>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), lds, c->stream, c->S,
                       (const int3 *)c->scratch[0].p, n, (float *)c->scratch[1].p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->scratch[1].p, (size_t)n * NB * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" {

int pbrtgpu_trace_paths(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, float *out) {
    if (!c || !c->hasScene || !keys || !out || n < 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    switch (c->nb) {
        case 32: return trace_impl<32>(c, keys, n, out);
        case 60: return trace_impl<60>(c, keys, n, out);
        case 30: return trace_impl<30>(c, keys, n, out);
    }
    return fail(PBRTGPU_E_UNSUPPORTED, "band count");
}

}  // extern "C"

template <int NB>
static int stats_impl(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, uint64_t *out) {
    HIPCHK(c->scratch[0].ensure((size_t)n * sizeof(int3)));
    HIPCHK(c->scratch[1].ensure(64));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, keys, (size_t)n * 12, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->scratch[1].p, 0, 64, c->stream));
    size_t lds = (size_t)c->stackDepth * kBlock * 4;
    hipLaunchKernelGGL(k_stats<NB>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), lds, c->stream, c->S,
                       (const int3 *)c->scratch[0].p, n, (unsigned long long *)c->scratch[1].p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->scratch[1].p, 6 * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

extern "C" {

int pbrtgpu_path_stats(pbrtgpu_ctx *c, const int32_t *keys, int32_t n, uint64_t *counters_out) {
    if (!c || !c->hasScene || !keys || !counters_out || n <= 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    HIPCHK(hipSetDevice(c->device));
    switch (c->nb) {
        case 32: return stats_impl<32>(c, keys, n, counters_out);
        case 60: return stats_impl<60>(c, keys, n, counters_out);
        case 30: return stats_impl<30>(c, keys, n, counters_out);
    }
    return fail(PBRTGPU_E_UNSUPPORTED, "band count");
}

int pbrtgpu_intersect(pbrtgpu_ctx *c, const float *rays, int32_t n, float *hits, int32_t *occ) {
    if (!c || !c->hasScene || !rays || !hits || n < 0) return fail(PBRTGPU_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(c->scratch[0].ensure((size_t)n * 32));
    HIPCHK(c->scratch[1].ensure((size_t)n * 16));
    HIPCHK(c->scratch[2].ensure((size_t)n * 4));
    HIPCHK(hipMemcpyAsync(c->scratch[0].p, rays, (size_t)n * 32, hipMemcpyHostToDevice, c->stream));
    size_t lds = (size_t)c->stackDepth * kBlock * 4;
    hipLaunchKernelGGL(k_intersect, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), lds, c->stream, c->S,
                       (const float *)c->scratch[0].p, n, (float *)c->scratch[1].p, (int *)c->scratch[2].p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(hits, c->scratch[1].p, (size_t)n * 16, hipMemcpyDeviceToHost, c->stream));
    std::vector<int> o(n);
    HIPCHK(hipMemcpyAsync(o.data(), c->scratch[2].p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (occ) memcpy(occ, o.data(), (size_t)n * 4);
    return 0;
}

int pbrtgpu_last_kernel_timing(pbrtgpu_ctx *c, double *avg_ms, int32_t *launches) {
    if (!c) return fail(PBRTGPU_E_INVALID, "null ctx");
    if (avg_ms) *avg_ms = c->lastKernelMs;
    if (launches) *launches = c->lastLaunches;
    return 0;
}

}  // extern "C"
