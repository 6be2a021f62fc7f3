// wavefront.h -- SoA path state and the per-vertex shading step of the wavefront path
// tracer.  PathIntegrator::Li (integrators/path.cpp:44-115) and
// EstimateDirect (core/integrator.cpp:109-166) are split at their three ray queries:
//
//   pass k:   k_trace_closest   continuation/camera rays + MIS rays  (BVHAccel::Intersect)
//             k_trace_shadow    light-sample visibility rays          (BVHAccel::IntersectP)
//             k_shade           per live path slot:
//                 1. finish the vertex whose direct light was pending:
//                      Ld = (0 [+ A if unoccluded]) [+ B if the MIS ray hit the light]
//                      L += beta_b * (nLights * Ld)
//                 2. if the continuation ray hit: the next vertex -- emission, BSDF, light
//                    sample (A + shadow ray), BSDF sample with MIS (B + MIS ray), path
//                    continuation (beta update, roulette, next ray)
//                 3. finished paths go through the NaN/negative/inf guard into Lout, and the
//                    slot takes the next camera sample (path regeneration)
//
// Every sampler / MT19937 draw, every float operation and its order are those of the
// single-path loop, so a path's radiance is identical to the oracle's; the split only
// defers the additions that need a ray answer.  Band data are stored as band quads,
// [band/4][slot] float4, so one 16-byte load per lane covers four bands and a wave's 64
// loads of one quad are a contiguous 1 KiB.
#pragma once
#include "device.h"

namespace pgd {

// Timing experiment only (-DPGD_SECTIONS, never in the product build): wave-cycles per
// section of k_shade, summed per block in LDS and written to a per-block array.
#ifdef PGD_SECTIONS
// Sub-sections of LIGHT (light_sample_L, the BSDF value / pdf, the A bands + shadow ray) and of
// CONT (the direction sample, the beta bands + roulette + continuation ray).  -DPGD_SECTIONS_DRAIN
// waits for every outstanding memory operation at each section's end, so a section is charged
// the latency of its own loads and stores (the total then exceeds an undrained run's).
enum { SEC_LOAD, SEC_FINISH, SEC_ISECT, SEC_BSDF, SEC_LIGHT, SEC_MIS, SEC_CONT, SEC_OUT, SEC_REGEN, SEC_PUSH,
       SEC_LSAMP, SEC_LEVAL, SEC_LSTORE, SEC_CSAMP, SEC_CBAND, SEC_N = 16 };
__shared__ unsigned long long pgd_secs[SEC_N];
#ifdef PGD_SECTIONS_DRAIN
#define PGD_SEC_DRAIN() __builtin_amdgcn_s_waitcnt(0)
#else
#define PGD_SEC_DRAIN() do {} while (0)
#endif
#define PGD_T0(k) const unsigned long long pgd_t_##k = clock64()
#define PGD_T1(k)                                                                                 \
    do {                                                                                          \
        PGD_SEC_DRAIN();                                                                          \
        const unsigned long long d_ = clock64() - pgd_t_##k;                                      \
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x) atomicAdd(&pgd_secs[SEC_##k], d_); \
    } while (0)
#else
#define PGD_T0(k) do {} while (0)
#define PGD_T1(k) do {} while (0)
#endif

enum {
    PF_CONT = 1,      // continuation / camera ray queued (answer in hit[0])
    PF_PEND = 2,      // direct lighting of vertex `bounce` not yet added to L
    PF_PA = 4,        // light-sample term A waits on the shadow ray
    PF_PB = 8,        // BSDF-sample term B waits on the MIS ray
    PF_SPEC = 16,     // specularBounce
    PF_MTINIT = 32,   // MT19937 recurrence window initialised
    PF_LZ = 64,       // L is still all zero (not stored yet)
    PF_NF0 = 128,     // bits 7..9: beta buffer k (PF_NF0 << k) holds a non-finite band
};
#define PF_LIGHT_SHIFT 12
#define PF_LIGHT_MASK 0xfffffu

enum { RAY_C = 0, RAY_M = 1, RAY_S = 2, RAY_M1 = 3 };
// The path integrator's MIS ray records alternate between two sets by the queue set of the pass
// that wrote them (RAY_M for set 0, RAY_M1 for set 1): a pass reads the records of the set the pass
// before wrote, at their compacted entries, while it writes its own at its entries.  With one set,
// the first pass of the drain's list mode (wavefront.h PathSoA::listMode: a 64-slot region's live
// slots may be shaded by two waves) could overwrite a record at its new identity entry before the
// slot that owned that compacted entry read it: an MIS term dropped, about 1 frame in 15 of C3
// (DESIGN.md §4.3).  DirectLighting indexes its records by light-sample row: RAY_M alone.
PGD_INLINE int mis_kind(int q) { return (q & 1) ? RAY_M1 : RAY_M; }
// the ray record of a closest-hit queue entry of queue set q (kind RAY_C or RAY_M)
PGD_INLINE int rec_kind(const DevScene &S, int q, int kind) {
    return (kind == RAY_M && S.integrator == PBRTGPU_INTEGRATOR_PATH) ? mis_kind(q) : kind;
}
// counters (u32 words), each on its own 128-byte line so that the per-block atomics of
// different queues do not serialise on one memory-side atomic unit; work = u64 at CNT_WORK
#define CNT_QC(q) (32 * (q))          // closest-hit queue size, queue set q = 0, 1
#define CNT_QS(q) (64 + 32 * (q))     // shadow queue size
#define CNT_QT(q) (224 + 32 * (q))    // MT-window list size (qT): k_mt_init of set q clears set q ^ 1
// CNT_ERR: bit 0 when a path drew past MT output 227 without its full-state row (mt_store), bit 1
// when a drain pass's live list was longer than its grid (k_shade LIST: slots left unshaded), which
// the host turns into PBRTGPU_E_STATE instead of a silently wrong radiance; k_tail (shade.hip): bit 2
// when its live list was longer than its grid, bit 3 when a path was still live after its steps; CNT_DLN: entries of
// the DirectLighting light-sample list (PathSoA::dlList) of this pass
enum { CNT_NEXT = 128, CNT_ZEROED = 160, CNT_WORK = 192, CNT_LIVE = 288, CNT_ERR = 320, CNT_DLN = 352, CNT_WORDS = 384 };
enum { W_RAYS = 0, W_SHADOW = 1, W_NODES_C = 2, W_NODES_S = 3, W_TRIS_C = 4, W_TRIS_S = 5, W_QUADS_C = 6, W_QUADS_S = 7,
       W_HITS = 8, W_RAYS_M = 9, W_HITS_M = 10, W_COUNT = 12 };

struct PathSoA {
    int cap;
    int *item;          // output index, -1 = free slot
    uint32_t *hp;       // pixel hash (sampler scramble key)
    uint32_t *pix;      // sample pixel (y << 16) | x  (camera ray differentials are re-derived)
    uint32_t *smp;      // sample index
    int *bounce;        // vertex index of the last processed vertex (-1: camera ray in flight)
    uint32_t *flags;
    uint32_t *mt;       // [5][cap]: k, a, b, m, seed
    uint32_t *mtExt;    // [cap][624]: the full MT19937 state of a path past 227 draws (device.h
                        // mt_uint_ext), or null when the scene's maxdepth cannot get there
    float4 *beta;       // [3][NQ][cap]: beta at vertex v in buffer v % 3
    float4 *L;          // [NQ][cap]
    float4 *A, *B;      // [2][NQ][cap]: pending direct-light terms of vertex v in buffer v & 1
                        // (path integrator: A of a pass in buffer qout, compacted per wave, see aMask)
    unsigned long long *aMask;   // [2][cap/64]: path integrator, the lanes of each wave that wrote
                                 // an A term in the pass with queue set q (A = wave region + rank)
    unsigned long long *mMask;   // [2][cap/64]: the same for the B (MIS) terms
    unsigned long long *bMask;   // [3][cap/64]: path integrator, the lanes of each wave that wrote
                                 // a beta in the pass with index pass % 3 (beta = wave region + rank)
    int pass;                    // index of this k_shade pass within the run (host counter)
    float4 *M;          // [NQ][cap]: measured-BRDF spectrum of the BSDF value being consumed
    float4 *K;          // [2][NQ][cap]: the material's textured spectra at the current vertex (device.h get_bsdf)
    // ray records are indexed by ray slot rs: the slot itself, or (DirectLighting, a batch of
    // light samples per pass) slot + j * cap for the batch's sample j; rcap = cap x batch
    int rcap;
    float *ray;         // [3 or 4][9][rcap]: o.xyz, d.xyz, mint, maxt, time  for RAY_C, RAY_M, RAY_S
                        // (and RAY_M1: the path integrator's second MIS record set, mis_kind)
    int *hitPrim;       // [2][rcap]  (RAY_C, RAY_M)
    float *hitT;        // [2][rcap]
    uint32_t *occ;      // [rcap]
    uint32_t *qC;       // [2][2*rcap]: (ray slot << 1) | kind
    uint32_t *qS;       // [2][rcap]: ray slot
    uint32_t *qT;       // [2][cap]: path integrator, slots whose MT window k_mt_init computes (mt_window_init)
    // The drain (path integrator, once the run's items are all taken): k_shade's threads take the
    // live slots listed in `live` (k_live_list, count at CNT_LIVE) instead of slot = thread, so the
    // last paths run in dense waves.  A wave then holds slots of many regions, and the per-wave
    // compaction degenerates to the identity: a writer stores at region + (slot & 63) and sets the
    // region's mask to all ones, so every reader (which ranks itself in the stored mask) finds it
    // there, whatever mode the writing pass ran in.
    int listMode;
    int xcdMap;         // the trace kernels' XCD-contiguous queue ranges (pbrtgpu.hip trace_wave)
    uint32_t *live;     // [cap]
    uint32_t *cnt;     // counters (CNT_*), work counters as u64 from word CNT_WORK
    float4 *instM;      // [cap][nInst][8]: the path's instance transforms (inst_load), or null
    int nInst;
    // DirectLightingIntegrator only (null for the path integrator): the slot's stack of the
    // SpecularReflect / SpecularTransmit recursion, frame d = the vertex at ray depth d
    int nFrames;
    float4 *fL;         // [nFrames][NQ][cap]: the vertex's radiance so far
    float4 *fF;         // [nFrames][NQ][cap]: BSDF value of its pending specular child
    float *fRay;        // [nFrames][9][cap]: its incoming ray
    float *fDiff;       // [nFrames][12][cap]: that ray's differentials rxo, rxd, ryo, ryd (depth >= 1)
    float *fS;          // [nFrames][2][cap]: |wi . n| and pdf of the pending child
    int *fHit;          // [nFrames][2][cap]: hit primitive, hit t (bits) of the incoming ray
    uint32_t *fBr;      // [nFrames][cap]: specular branches tried (0, 1 reflect, 2 transmit)
    uint32_t *dlk;      // [cap]: light-sample cursor of the top vertex (first sample of its batch)
    uint32_t *dlMask;   // [cap]: the batch's queued shadow rays (bits 0-15) and MIS rays (16-31)
    int dlBatch;        // light samples issued per pass (<= 16); A, B hold [dlBatch][NQ][cap]
    // the light-sample list: k_shade appends the slots it marks PF_DLNEE (in wave order, count at
    // CNT_DLN), k_dl_nee's thread i takes entry i, so its waves hold marked slots only.  Entry i is
    // the slot's batch row: its A / B terms sit in column i of [dlBatch][NQ][cap], its shadow / MIS
    // rays at ray slots i + j * cap (without instances), and dlRow[slot] = i tells the next
    // k_shade where to find them -- the rows of one k_shade wave's slots are contiguous, so
    // writers and readers touch whole lines instead of every other lane's
    uint32_t *dlList;   // [cap]
    uint32_t *dlRow;    // [cap]
};
// the slot a ray slot belongs to
PGD_INLINE int slot_of_ray(const PathSoA &P, int rs) { return rs < P.cap ? rs : rs % P.cap; }
// the path's instance-transform record (null without instances)
PGD_INLINE const float4 *inst_rec(const PathSoA &P, int slot) {
    return P.nInst ? P.instM + (size_t)slot * P.nInst * 8 : nullptr;
}

// where the camera samples of a pass come from
struct ItemSrc {
    const int2 *pix;    // film pixels (sample x, y) of the render call
    int sb;             // samples per pixel in this batch
    int s0;             // first sample index
    const int3 *keys;   // explicit (x, y, s) keys for items >= keyBase (trace_paths, spill samples), or null
    uint32_t keyBase;   // items [0, keyBase) are (pixel, sample) items, the rest keys[item - keyBase]
    uint32_t nItems;    // items of this run: global items base .. base + nItems - 1
    uint32_t base;
};

// a column of a slot array (32-bit addressing, device.h sa): element i (+ k) of base
template <class T> struct Col {
    T *base;
    uint32_t i;
    PGD_INLINE T &operator[](uint32_t k) const { return *sa(base, i + k); }
};
static constexpr uint32_t kNoCol = 0xffffffffu;

PGD_INLINE void ray_store(const PathSoA &P, int kind, int rs, const Ray &r) {
    const uint32_t c = (uint32_t)P.rcap, b = (uint32_t)kind * 9u * c + (uint32_t)rs;
    float *R = P.ray;
    *sa(R, b) = r.o.x; *sa(R, b + c) = r.o.y; *sa(R, b + 2 * c) = r.o.z;
    *sa(R, b + 3 * c) = r.d.x; *sa(R, b + 4 * c) = r.d.y; *sa(R, b + 5 * c) = r.d.z;
    *sa(R, b + 6 * c) = r.mint; *sa(R, b + 7 * c) = r.maxt; *sa(R, b + 8 * c) = r.time;
}
PGD_INLINE Ray ray_load(const PathSoA &P, int kind, int rs) {
    const uint32_t c = (uint32_t)P.rcap, b = (uint32_t)kind * 9u * c + (uint32_t)rs;
    const float *R = P.ray;
    Ray r;
    r.o = v3(*sa(R, b), *sa(R, b + c), *sa(R, b + 2 * c));
    r.d = v3(*sa(R, b + 3 * c), *sa(R, b + 4 * c), *sa(R, b + 5 * c));
    r.mint = *sa(R, b + 6 * c); r.maxt = *sa(R, b + 7 * c); r.time = *sa(R, b + 8 * c);
    return r;
}

PGD_INLINE void mt_load(const PathSoA &P, int slot, uint32_t fl, MT &r) {
    const uint32_t c = (uint32_t)P.cap, s = (uint32_t)slot;
    r.k = *sa(P.mt, s); r.a = *sa(P.mt, c + s); r.b = *sa(P.mt, 2 * c + s); r.m = *sa(P.mt, 3 * c + s);
    r.seed = *sa(P.mt, 4 * c + s);
    r.init = (fl & PF_MTINIT) != 0;
    r.ext = P.mtExt ? P.mtExt + (size_t)slot * 624 : nullptr;
}
PGD_INLINE void mt_store(const PathSoA &P, int slot, const MT &r) {
    const uint32_t c = (uint32_t)P.cap, s = (uint32_t)slot;
    if (__builtin_expect(r.k >= 227u && !r.ext, 0)) atomicOr(&P.cnt[CNT_ERR], 1u);   // (mt_uint returned 0s)
    *sa(P.mt, s) = r.k; *sa(P.mt, c + s) = r.a; *sa(P.mt, 2 * c + s) = r.b; *sa(P.mt, 3 * c + s) = r.m;
}
// The recurrence window of a path before its first MT draw (output 0: mt[0], mt[1], mt[397] of its
// seed), for a path integrator slot that shade_vertex queued in qT when it continued from vertex 2
// (vertex 3 draws first).  k_mt_init runs it over the pass's compacted list after k_shade: inline
// at the draw site, the 396 dependent steps of mt_word397 ran once per pass in nearly every wave
// (one lane in ~10 reaches vertex 3 in a given pass) and made up a large part of k_shade's VALU work
PGD_INLINE void mt_window_init(const PathSoA &P, uint32_t s) {
    const uint32_t c = (uint32_t)P.cap;
    MT r;
    mt_begin(r, *sa(P.mt, 4 * c + s));
    mt_init(r);
    *sa(P.mt, c + s) = r.a; *sa(P.mt, 2 * c + s) = r.b; *sa(P.mt, 3 * c + s) = r.m;
    *sa(P.flags, s) |= PF_MTINIT;
}

template <int NB> struct Bands { static constexpr int NQ = (NB + 3) / 4; };
// unrolling of the band loops that stream the light-sample and MIS terms A, B to memory: by 4
// quads (U=3 keeps every variant within the kernel budget; fully unrolled, all quads' loads were hoisted, and the FEAT 0 kernel reloaded a spilled
// BSDF parameter from scratch in every band: 213 scratch loads, 11 by 3 or 4 quads); the beta loop
// stays unrolled, its quads are kept for the roulette
#ifndef PGD_UNROLL_BANDS
#define PGD_UNROLL_BANDS _Pragma("unroll 3")
#endif
// path-state spectra: beta in three buffers, so that a pass can read beta_b (finishing vertex
// b), beta_{b+1} (shading it) and write beta_{b+2}; A, B in two
// Path integrator: beta of a vertex is written by the pass that samples its direction (buffer
// pass % 3, compacted per wave like A) and read by the next pass (shading the vertex) and the one
// after (finishing its direct light): ago = 1 or 2 passes.  Vertex 0 (beta = 1) is not stored.
PGD_INLINE int pass_buf(const PathSoA &P, int ago) { return (P.pass + 3 - ago) % 3; }
template <int NB> PGD_INLINE Col<float4> beta_reg(const PathSoA &P, int buf, int slot) {
    return Col<float4>{P.beta, (uint32_t)buf * Bands<NB>::NQ * (uint32_t)P.cap + ((uint32_t)slot & ~63u)};
}
PGD_INLINE unsigned long long *beta_mask(const PathSoA &P, int buf, int slot) {
    return P.bMask + (size_t)buf * ((P.cap + 63) >> 6) + (slot >> 6);
}
// the writer masks a k_shade wave reads, loaded once at the start of the slot's step (scalar
// loads: the wave index is uniform), so that no spectrum load waits on its mask
struct WaveMasks { unsigned long long a, b, b1, b2; };   // A, B of the last pass; beta 1, 2 passes back
PGD_INLINE WaveMasks wave_masks(const PathSoA &P, int qout, int slot) {
    const size_t W = (size_t)((P.cap + 63) >> 6);
    WaveMasks m;
    if (P.listMode) {   // the lanes' slots lie in different regions: per-lane loads
        const int w = slot >> 6;
        m.a = P.aMask[(size_t)(qout ^ 1) * W + w];
        m.b = P.mMask[(size_t)(qout ^ 1) * W + w];
        m.b1 = P.bMask[(size_t)pass_buf(P, 1) * W + w];
        m.b2 = P.bMask[(size_t)pass_buf(P, 2) * W + w];
        return m;
    }
    const int w = __builtin_amdgcn_readfirstlane(slot >> 6);
    m.a = P.aMask[(size_t)(qout ^ 1) * W + w];
    m.b = P.mMask[(size_t)(qout ^ 1) * W + w];
    m.b1 = P.bMask[(size_t)pass_buf(P, 1) * W + w];
    m.b2 = P.bMask[(size_t)pass_buf(P, 2) * W + w];
    return m;
}
PGD_INLINE int wave_rank(unsigned long long m, int slot) { return __popcll(m & ((1ull << (slot & 63)) - 1ull)); }
// the slot's beta written `ago` passes back (i = kNoCol for vertex 0: beta = 1, not stored);
// m = that pass's writer mask
template <int NB> PGD_INLINE Col<float4> beta_rd(const PathSoA &P, int v, int ago, int slot, unsigned long long m) {
    Col<float4> r = beta_reg<NB>(P, pass_buf(P, ago), slot);
    r.i = v == 0 ? kNoCol : r.i + (uint32_t)wave_rank(m, slot);
    return r;
}
#ifdef PGD_EXP_NOBETA   // timing experiment only: beta not loaded (wrong radiance)
PGD_INLINE float4 beta_q(const Col<float4> &bp, int q, uint32_t c) {
    return make_float4(1.f, 1.f, 1.f, bp.i != kNoCol ? 0.5f : 1.f);
}
#else
PGD_INLINE float4 beta_q(const Col<float4> &bp, int q, uint32_t c) {
    return bp.i != kNoCol ? bp[(uint32_t)q * c] : make_float4(1.f, 1.f, 1.f, 1.f);
}
#endif
// beta of vertex v has a non-finite band (then L += beta * 0 is NaN and cannot be skipped)
PGD_INLINE bool beta_nonfinite(uint32_t fl, int v) { return v > 0 && ((fl >> (7 + v % 3)) & 1u); }
// path integrator: the A region of slot's wave in the buffer of queue set q, and that wave's
// writer mask; the reader of the next pass finds its term at the region + its rank
template <int NB> PGD_INLINE Col<float4> A_reg(const PathSoA &P, int q, int slot) {
    return Col<float4>{P.A, (uint32_t)q * Bands<NB>::NQ * (uint32_t)P.cap + ((uint32_t)slot & ~63u)};
}
PGD_INLINE unsigned long long *A_mask(const PathSoA &P, int q, int slot) {
    return P.aMask + (size_t)q * ((P.cap + 63) >> 6) + (slot >> 6);
}
// the B (MIS) terms likewise
template <int NB> PGD_INLINE Col<float4> B_reg(const PathSoA &P, int q, int slot) {
    return Col<float4>{P.B, (uint32_t)q * Bands<NB>::NQ * (uint32_t)P.cap + ((uint32_t)slot & ~63u)};
}
PGD_INLINE unsigned long long *B_mask(const PathSoA &P, int q, int slot) {
    return P.mMask + (size_t)q * ((P.cap + 63) >> 6) + (slot >> 6);
}

#ifdef PGD_EXP_NOSPEC   // timing experiment only: scene spectra not loaded (wrong radiance)
PGD_INLINE float4 ld4(const float *p) { return make_float4(0.5f, 0.5f, 0.5f, (float)((uintptr_t)p & 1)); }
PGD_INLINE float4 ld4(const float *p, int off) { return make_float4(0.5f, 0.5f, 0.5f, (float)(off & 1)); }
#else
PGD_INLINE float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
// band quad at float offset off of the spectrum pool p (32-bit offset from the uniform base)
PGD_INLINE float4 ld4(const float *p, int off) { return *reinterpret_cast<const float4 *>(sa(p, (uint32_t)off)); }
#endif
PGD_INLINE float &cmp(float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
PGD_INLINE float cmp(const float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// FrCond (reflection.cpp:62-71) for one band
PGD_INLINE float fr_cond(float cosi, float eta, float k) {
    float tmp = ((eta * eta + k * k) * cosi) * cosi;
    float Rparl2 = ((tmp - ((2.f * eta) * cosi)) + 1.f) / ((tmp + ((2.f * eta) * cosi)) + 1.f);
    float tmp_f = eta * eta + k * k;
    float Rperp2 = ((tmp_f - ((2.f * eta) * cosi)) + cosi * cosi) / ((tmp_f + ((2.f * eta) * cosi)) + cosi * cosi);
    return (Rparl2 + Rperp2) / 2.f;
}
// BSDF value of one band of a term, with the reference's operand order per BxDF::f
PGD_INLINE float term_val(const FTerm &t, float r, float r2) {
    switch (t.kind) {
        case T_LAMB: return r * kInvPi;
        case T_OREN: return (r * kInvPi) * t.s0;
        case T_BLINN: return (((r * t.s0) * t.s1) * t.s2) / t.s3;
        case T_BLINNC: return (((1.f * t.s0) * t.s1) * fr_cond(t.s2, r, r2)) / t.s3;   // R = Spectrum(1.)
        case T_FB: {
            const float cd = (28.f / (23.f * kPi));
            float diffuse = ((((cd * r) * (1.f - r2)) * t.s0) * t.s1);
            float schlick = r2 + t.s2 * (1.f - r2);
            return diffuse + t.s3 * schlick;
        }
        default: return 0.f;
    }
}
// band quad q of a spectrum reference: pool offset, or -1 - j * NQ = the slot's K band buffer j
// (device.h get_bsdf)
PGD_INLINE float4 spec4(const float *sp, int off, int q, const float4 *kb, size_t c) {
    return off >= 0 ? ld4(sp, off + 4 * q) : kb[(size_t)(-1 - off + q) * c];
}
// one term's share of four bands (quad q), added to v
template <int FEAT>
PGD_INLINE void term4(const float *sp, const FTerm &t, int q, const float4 *mb, const float4 *kb, size_t c, float4 &v) {
    if ((FEAT & FEAT_MEAS) && t.kind == T_BUF) {
        const float4 m = mb[q * c];
        v.x += m.x; v.y += m.y; v.z += m.z; v.w += m.w;
        return;
    }
    float4 r, r2;
    if (PGD_BASIC_MATS) {   // Lambertian, Oren-Nayar, dielectric Blinn: one spectrum
        r = ld4(sp, t.R + 4 * q);
        r2 = r;
    } else if (FEAT & FEAT_TEX) {
        r = spec4(sp, t.R, q, kb, c);
        r2 = (t.kind == T_FB || t.kind == T_BLINNC) ? spec4(sp, t.R2, q, kb, c) : r;
    } else {
        r = ld4(sp, t.R + 4 * q);
        r2 = (t.kind == T_FB || t.kind == T_BLINNC) ? ld4(sp, t.R2 + 4 * q) : r;
    }
    // the kind is chosen once for the quad: a switch per band (term_val) had compiled to a branch
    // tree per band -- ~20 exec-mask instructions per band and term in every band loop
    float4 f;
    switch (t.kind) {
        case T_LAMB: f = make_float4(r.x * kInvPi, r.y * kInvPi, r.z * kInvPi, r.w * kInvPi); break;
        case T_OREN:
            f = make_float4((r.x * kInvPi) * t.s0, (r.y * kInvPi) * t.s0, (r.z * kInvPi) * t.s0, (r.w * kInvPi) * t.s0);
            break;
        case T_BLINN:
            f = make_float4((((r.x * t.s0) * t.s1) * t.s2) / t.s3, (((r.y * t.s0) * t.s1) * t.s2) / t.s3,
                            (((r.z * t.s0) * t.s1) * t.s2) / t.s3, (((r.w * t.s0) * t.s1) * t.s2) / t.s3);
            break;
        default:
            if (PGD_BASIC_MATS) { f = make_float4(0.f, 0.f, 0.f, 0.f); break; }
            f = make_float4(term_val(t, r.x, r2.x), term_val(t, r.y, r2.y), term_val(t, r.z, r2.z),
                            term_val(t, r.w, r2.w));
            break;
    }
    v.x += f.x;
    v.y += f.y;
    v.z += f.z;
    v.w += f.w;
}
// BSDF value of four bands (quad q): mb = measured scratch, kb = texture scratch of the slot
template <int FEAT>
PGD_INLINE float4 fval4(const float *sp, const FVal &F, int q, const float4 *mb, const float4 *kb, size_t c) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!PGD_BASIC_MATS && !PGD_NOSPEC_MATS && F.mode == FV_SPEC) {
        float4 r = (FEAT & FEAT_TEX) ? spec4(sp, F.R, q, kb, c) : ld4(sp, F.R + 4 * q);
        return make_float4((F.fs * r.x) / F.d, (F.fs * r.y) / F.d, (F.fs * r.z) / F.d, (F.fs * r.w) / F.d);
    }
    if (!PGD_NOSPEC_MATS && (FEAT & FEAT_TEX) && F.mode == FV_SPEC_COND) {   // shinymetal's mirror lobe (scenes with one run FEAT_TEX)
        const float4 e = ld4(sp, F.R + 4 * q);
        return make_float4((fr_cond(F.fs, e.x, 0.f) * 1.f) / F.d, (fr_cond(F.fs, e.y, 0.f) * 1.f) / F.d,
                           (fr_cond(F.fs, e.z, 0.f) * 1.f) / F.d, (fr_cond(F.fs, e.w, 0.f) * 1.f) / F.d);
    }
    if (F.n > 0) term4<FEAT>(sp, F.t0, q, mb, kb, c, v);
    if (F.n > 1) term4<FEAT>(sp, F.t1, q, mb, kb, c, v);
    return v;
}
// band quad q of an emitted radiance (Emit, device.h)
template <int FEAT>
PGD_INLINE float4 emit4(const DevScene &S, const Emit &e, int q) {
    if ((FEAT & FEAT_INF) && e.mode == EM_RGB) return from_rgb4(S, e.pick, true, q);
    if (e.mode == EM_BLACK) return make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = ld4(S.spectra, e.off + 4 * q);
    if (e.point) {
        if (FEAT & FEAT_INF) v = make_float4(v.x * e.mul, v.y * e.mul, v.z * e.mul, v.w * e.mul);   // spot Falloff
        v = make_float4(v.x / e.div, v.y / e.div, v.z / e.div, v.w / e.div);
    }
    return v;
}
template <int NB, int FEAT>
PGD_INLINE bool emit_black(const DevScene &S, const Emit &e) {
    if (e.mode == EM_BLACK) return true;
    if (e.mode == EM_POOL && !e.point) return false;   // area lights: is_black folded into the mode
    bool black = true;
#pragma unroll
    for (int q = 0; q < Bands<NB>::NQ; ++q) {
        float4 v = emit4<FEAT>(S, e, q);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * q + k < NB) black = black && (cmp(v, k) == 0.);
    }
    return black;
}

// IrregIsotropicBRDF::f (reflection.cpp:251-264): KdTree::Lookup (kdtree.h:160-185) with
// IrregIsoProc (reflection.cpp:34-47), retried with the radius doubled until more than 2
// samples are found (here: the final radius found first, kd_final_radius), in the reference's
// visiting order (children first, near child before
// far child, the far child only when the split plane is within reach, then the node).
//   * The walk is stackless: it climbs back over parent links, so there is no private stack
//     in scratch memory.
//   * Nodes are packed as 2 float4 (kd_pack, host-built): {p.xyz, splitPos},
//     {spec offset, rightChild, parent, axis | hasLeft << 2}; indices relative to the tree.
//   * When every tree of the scene fits (kKdLdsNodes), each shade block copies them to LDS
//     once and the walk's dependent node loads are LDS reads (~100 cycles) instead of L2
//     round trips -- the walk is a chain of ~100-200 dependent loads per lookup, and a wave
//     waits for its slowest lane (C3: lookups were 2/3 of the frame).
//   * The spectrum sum stays in registers and is written to the slot's M bands once.
// Out of line: the walk's registers do not add to the shade kernel's at its 3 call sites.
static const int kKdLdsNodes = 1536;            // 48 KB of LDS per shade block
extern __shared__ float4 pgd_kd_lds[];          // dynamic LDS of k_shade (FEAT_MEAS variants)
typedef float F4N __attribute__((ext_vector_type(4)));
#ifndef PGD_LDS_AS   // the LDS address space (the host replay of tools/hostsan defines it empty)
#define PGD_LDS_AS __attribute__((address_space(3)))
#endif
typedef PGD_LDS_AS const F4N LdsF4;   // an LDS float4 (ds_read_b128)
// The global address space, spelled out in the out-of-line kd-tree lookup: its pointer arguments
// (the spectrum pool, the slot's M bands) would otherwise be generic, and a generic (flat) access
// counts on the LDS counter as well -- every ds_read of the walk then waited (s_waitcnt lgkmcnt)
// for the candidate stores and spectrum loads still in flight
typedef PGD_GLOBAL_AS const F4N GlbF4c;
typedef PGD_GLOBAL_AS F4N GlbF4;
typedef PGD_GLOBAL_AS float GlbF;
PGD_INLINE float4 kd_node(const float4 *__restrict__ p, int i) { return p[i]; }
PGD_INLINE float4 kd_node(LdsF4 *p, int i) { const F4N v = p[i]; return make_float4(v.x, v.y, v.z, v.w); }

// One step of the walk from node cur (children first, near child before far child, the far child
// only when its split plane is within maxD2, then the node): the next node to visit, or -1 when
// the node itself is next.
PGD_INLINE int kd_next(const float4 &a, const float4 &b, int cur, int prev, bool down, float p0, float p1, float p2,
                       float maxD2) {
    const int meta = __float_as_int(b.w), axis = meta & 3;
    if (axis == 3) return -1;
    const float pa = axis == 0 ? p0 : (axis == 1 ? p1 : p2);
    const bool leftFirst = pa <= a.w;
    const float dist2s = (pa - a.w) * (pa - a.w);
    const int L = (meta & 4) ? cur + 1 : -1, R = __float_as_int(b.y);   // -1: no right child
    const int first = leftFirst ? L : R, second = leftFirst ? R : L;
    if (down && first >= 0) return first;
    if ((down || prev == first) && second >= 0 && dist2s < maxD2) return second;
    return -1;
}
// The radius the reference's retry loop ends at, without its retries: the loop walks at
// maxDist2 = .001f * 2^k for k = 0, 1, ... and stops at the first k with more than 2 samples
// strictly inside, or at k = 11 (maxDist2 = 2.048 > 1.5).  That k is the first with
// d3 < .001f * 2^k, d3 the third-smallest sample distance^2 (C3's points needed ~3-4 walks of
// growing radius each in the reference).
// Closed form of  m = .001f; for (k = 0; k < 11 && !(d3 < m); ++k) m *= 2.f;  -- the doublings
// are exact, so m = .001f * 2^k at the first k with d3 < m, found from d3's exponent and whether
// its mantissa is below .001f's (1.024); checked against the loop over every non-negative float
// (tests/test_hostsan.py).  No loop: its trip count diverged across a wave.
PGD_INLINE float kd_radius_of(float d3) {
    const uint32_t b = __float_as_uint(d3);
    int k = (int)(b >> 23) - 116 - ((b & 0x7fffffu) < 0x03126fu ? 1 : 0);
    k = min(max(k, 0), 11);
    return __uint_as_float(0x3a83126fu + ((uint32_t)k << 23));
}
// One walk finds d3 and the samples the reference's final walk accumulates, in its order:
//   * A node's own sample is compared on arrival (pre-order): d1 <= d2 <= d3 keep the three
//     smallest distances (capped at .001f * 1024, beyond which the radius is 2.048 regardless),
//     and the pruning bound is kd_radius_of(d3) -- never below the final radius, which it becomes
//     once d3 is final.  A pruned far child holds only samples at least its split plane's float
//     distance^2 away (the float subtraction and the sums of squares are monotonic), so pruning
//     at any bound >= the final radius loses none of them.
//   * The walk's order is the reference's (children first, near child before far child, then the
//     node; near / far fixed by the split), so its post-order visits of the nodes the final walk
//     visits come in the final walk's order; it visits more nodes early, while the bound is
//     looser, and every node it leaves within the bound of that moment is a candidate.  The
//     candidates are kept in the slot's M bands (4 NQ indices, the lookup's own output), then
//     re-tested against the final radius and accumulated in that order -- the reference's sum.
//   * More candidates than fit: the final walk is run as such at the final radius.
// Against a radius walk followed by the final walk, about half the node visits (C3: each visit a
// dependent LDS read, and a wave waits for its slowest lane).
template <int NB, class NodePtr>
PGD_INLINE void kd_accumulate(NodePtr nodes, const float *__restrict__ spectra, int node, float p0, float p1, float p2,
                              float maxD2, float4 *acc, float &sumWeights) {
    constexpr int NQ = Bands<NB>::NQ;
    const float4 a = kd_node(nodes, 2 * node), b = kd_node(nodes, 2 * node + 1);
    const V d = vsub(v3(a.x, a.y, a.z), v3(p0, p1, p2));
    const float dist2 = vlen2(d);
    if (dist2 < maxD2) {
        const float weight = libmf_expf(-100.f * dist2);   // glibc expf, inline
        const GlbF4c *sv = (const GlbF4c *)(spectra + __float_as_int(b.x));
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const F4N sq = sv[q];
            acc[q].x += weight * sq.x; acc[q].y += weight * sq.y;
            acc[q].z += weight * sq.z; acc[q].w += weight * sq.w;
        }
        sumWeights += weight;
    }
}
template <int NB, class NodePtr>
PGD_INLINE void kd_lookup(NodePtr nodes, const float *__restrict__ spectra, float p0, float p1, float p2,
                          float4 *__restrict__ mb, size_t c) {
    constexpr int NQ = Bands<NB>::NQ;
    float4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    float sumWeights = 0.f;
#ifdef PGD_KD_RETRY   // the reference's retry loop (timing comparison)
    float maxD2 = .001f;
    for (;;) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        sumWeights = 0.f;
        int nFound = 0, cur = 0, prev = -1;
        bool down = true;
        for (;;) {
            const float4 a = kd_node(nodes, 2 * cur), b = kd_node(nodes, 2 * cur + 1);
            const int nxt = kd_next(a, b, cur, prev, down, p0, p1, p2, maxD2);
            if (nxt >= 0) { prev = cur; cur = nxt; down = true; continue; }
            if (vlen2(vsub(v3(a.x, a.y, a.z), v3(p0, p1, p2))) < maxD2) ++nFound;
            kd_accumulate<NB>(nodes, spectra, cur, p0, p1, p2, maxD2, acc, sumWeights);
            if (cur == 0) break;
            prev = cur; cur = __float_as_int(b.z); down = false;
        }
        if (nFound > 2 || maxD2 > 1.5f) break;
        maxD2 *= 2.f;
    }
#else
    constexpr int CAP = 4 * NQ;
    // candidate j: component j & 3 of mb[(j >> 2) * c], a 32-bit offset (slot arrays < 4 GiB,
    // ensure_slots) from the slot's global pointer
    GlbF *cand = (GlbF *)mb;
    const uint32_t c4 = 4u * (uint32_t)c;
    const float capD2 = .001f * 1024.f;
    float d1 = capD2, d2 = capD2, d3 = capD2, bound = kd_radius_of(capD2);
    int n = 0, cur = 0, prev = -1;
    bool down = true;
    // one step per trip as value selects (the top-3 update, kd_next): the lanes of a wave take
    // different paths through the tree, and as branches each step ran every path under exec masks
    // (r06j: C3 476.7 -> 481.6 Mpaths/s)
    for (;;) {
        const float4 a = kd_node(nodes, 2 * cur), b = kd_node(nodes, 2 * cur + 1);
        const V d = vsub(v3(a.x, a.y, a.z), v3(p0, p1, p2));
        const float dist2 = vlen2(d);
        const bool upd = down & (dist2 < d3);
        const float n3 = fminf(fmaxf(dist2, d2), d3), n2 = fminf(fmaxf(dist2, d1), d2), n1 = fminf(dist2, d1);
        d3 = upd ? n3 : d3;
        d2 = upd ? n2 : d2;
        d1 = upd ? n1 : d1;
        const float nb = kd_radius_of(d3);
        bound = upd ? nb : bound;
        const int meta = __float_as_int(b.w), axis = meta & 3;   // kd_next, as selects
        const float pa = axis == 0 ? p0 : (axis == 1 ? p1 : p2);
        const bool leftFirst = pa <= a.w;
        const float dist2s = (pa - a.w) * (pa - a.w);
        const int L = (meta & 4) ? cur + 1 : -1, R = __float_as_int(b.y);
        const int first = leftFirst ? L : R, second = leftFirst ? R : L;
        const bool takeFirst = down & (first >= 0);
        const bool takeSecond = (down | (prev == first)) & (second >= 0) & (dist2s < bound);
        int nxt = takeFirst ? first : (takeSecond ? second : -1);
        nxt = axis == 3 ? -1 : nxt;
        const bool leave = nxt < 0;
        const bool isCand = leave & (dist2 < bound);   // post-order: a candidate of the final walk
        if (isCand & (n < CAP)) cand[(uint32_t)(n >> 2) * c4 + (uint32_t)(n & 3)] = __int_as_float(cur);
        n += isCand ? 1 : 0;
        if (leave & (cur == 0)) break;
        prev = cur;
        cur = leave ? __float_as_int(b.z) : nxt;
        down = !leave;
    }
    const float maxD2 = bound;
    if (n <= CAP) {
        for (int j = 0; j < n; ++j)
            kd_accumulate<NB>(nodes, spectra, __float_as_int(cand[(uint32_t)(j >> 2) * c4 + (uint32_t)(j & 3)]), p0, p1, p2,
                              maxD2, acc, sumWeights);
    } else {   // the final walk itself
        cur = 0; prev = -1; down = true;
        for (;;) {
            const float4 a = kd_node(nodes, 2 * cur), b = kd_node(nodes, 2 * cur + 1);
            const int nxt = kd_next(a, b, cur, prev, down, p0, p1, p2, maxD2);
            if (nxt >= 0) { prev = cur; cur = nxt; down = true; continue; }
            kd_accumulate<NB>(nodes, spectra, cur, p0, p1, p2, maxD2, acc, sumWeights);
            if (cur == 0) break;
            prev = cur; cur = __float_as_int(b.z); down = false;
        }
    }
#endif
    GlbF4 *mo = (GlbF4 *)mb;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const float4 v = acc[q];
        F4N o;
        o.x = clampf(v.x, 0.f, INFINITY) / sumWeights; o.y = clampf(v.y, 0.f, INFINITY) / sumWeights;
        o.z = clampf(v.z, 0.f, INFINITY) / sumWeights; o.w = clampf(v.w, 0.f, INFINITY) / sumWeights;
        mo[(uint32_t)q * (uint32_t)c] = o;
    }
}
template <int NB>
__device__ __attribute__((noinline)) void kd_lookup_lds(LdsF4 *nodes, const float *__restrict__ spectra, float p0,
                                                        float p1, float p2, float4 *__restrict__ mb, size_t c) {
    kd_lookup<NB>(nodes, spectra, p0, p1, p2, mb, c);
}
template <int NB>
__device__ __attribute__((noinline)) void kd_lookup_global(const float4 *__restrict__ nodes, const float *__restrict__ spectra,
                                                           float p0, float p1, float p2, float4 *__restrict__ mb, size_t c) {
    kd_lookup<NB>(nodes, spectra, p0, p1, p2, mb, c);
}
template <int NB>
PGD_INLINE void measured_lookup(const DevScene &S, const FTerm &t, float4 *mb, size_t c) {
#ifdef PGD_EXP_MEAS_CHEAP   // timing experiment only: the lookup's cost share (wrong radiance)
    for (int q = 0; q < Bands<NB>::NQ; ++q) mb[q * c] = ld4(sa(S.spectra, (uint32_t)((*sa(S.kd, (uint32_t)(t.R))).spec + 4 * q)));
    return;
#endif
    if (S.kdInLds) kd_lookup_lds<NB>((LdsF4 *)pgd_kd_lds + 2 * t.R, S.spectra, t.s0, t.s1, t.s2, mb, c);
    else kd_lookup_global<NB>(sa(S.kdPack, (uint32_t)(2 * t.R)), S.spectra, t.s0, t.s1, t.s2, mb, c);
}
// k_shade prologue of the FEAT_MEAS variants: the block's copy of the kd-trees in LDS
PGD_INLINE void kd_lds_fill(const DevScene &S) {
    if (!S.kdInLds) return;
    for (int i = threadIdx.x; i < 2 * S.nKd; i += blockDim.x) pgd_kd_lds[i] = (*sa(S.kdPack, (uint32_t)(i)));
    __syncthreads();
}
// materialise a measured term of F into the slot's M bands (T_MEAS -> T_BUF)
template <int NB>
PGD_INLINE void term_prepare(const DevScene &S, FTerm &t, float4 *mb, size_t c) {
    if (t.kind == T_MEAS) {
        measured_lookup<NB>(S, t, mb, c);
        t.kind = T_BUF;
    } else if (t.kind == T_MERL) {
        // Spectrum::FromRGB(&brdf[3 * index]) (reflection.cpp:299), reflectance
        const float *rgb = sa(S.merl, (uint32_t)(3 * ((size_t)t.R + (size_t)t.R2)));
        const float v[3] = {rgb[0], rgb[1], rgb[2]};
        const RGBPick pk = rgb_pick(S, v);
#pragma unroll
        for (int q = 0; q < Bands<NB>::NQ; ++q) mb[q * c] = from_rgb4(S, pk, false, q);
        t.kind = T_BUF;
    }
}
template <int NB, int FEAT>
PGD_INLINE void fval_prepare(const DevScene &S, FVal &F, float4 *mb, size_t c) {
    if (!(FEAT & FEAT_MEAS) || F.mode != FV_SUM) return;
    if (F.n > 0) term_prepare<NB>(S, F.t0, mb, c);
    if (F.n > 1) term_prepare<NB>(S, F.t1, mb, c);
}

// The BSDF-sampled term B of a vertex counts only if the MIS ray's closest hit is a
// primitive of light Lt (DiffuseAreaLight::L, integrator.cpp:150-160).  A ray that misses
// every shape of the light -- the hit test BVHAccel runs on them, with maxt = inf, whose
// hit set contains that of any shorter ray -- cannot reach it: B is never added, so that
// ray is not traced.  Lights with triangle shapes (or many shapes) are always traced.
template <int FEAT>
PGD_INLINE bool mis_may_reach(const DevScene &S, const pbrtgpu_light &Lt, const Ray &r) {
    if ((FEAT & FEAT_INF) && Lt.type == PBRTGPU_LIGHT_INFINITE) return true;
    if (Lt.n_shapes > 8) return true;
    const pbrtgpu_light_shape *shs = sa(S.lightShapes, (uint32_t)(Lt.shape_offset));
    for (int i = 0; i < Lt.n_shapes; ++i) {
        const int ty = shs[i].shape_type;
        if (ty == PBRTGPU_SHAPE_TRIANGLE) return true;
        float t;
        if (quadric_test(S, ty, shs[i].shape_index, r, &t)) return true;
    }
    return false;
}

// camera sample of an item -> fresh path in `slot` (SamplerRendererTask::Run,
// samplerrenderer.cpp:86-108 + the fixed-seed sampler of DESIGN.md §3.1).  With the
// SpectralRenderer's singleDirection method item = sample * nWaveBands + band: the band's
// path repeats the sample's camera ray and sample values and draws from its own RNG
// (spectralrenderer.cpp:116-151)
template <int NB>
PGD_INLINE void path_start(const DevScene &S, const PathSoA &P, const ItemSrc &src, int slot, uint32_t it) {
    const uint32_t item = src.base + it;
    const uint32_t sitem = S.specItems > 1 ? item / (uint32_t)S.specItems : item;
    int px, py;
    uint32_t s;
    if (src.keys && sitem >= src.keyBase) {
        const int3 k = src.keys[sitem - src.keyBase];
        px = k.x; py = k.y; s = (uint32_t)k.z;
    }
    else {
        uint32_t p = sitem / (uint32_t)src.sb;
        int2 xy = src.pix[p];
        px = xy.x; py = xy.y;
        s = (uint32_t)src.s0 + (sitem - p * (uint32_t)src.sb);
    }
    const uint32_t spp = (uint32_t)S.spp;
    uint32_t hp = pixel_hash(S.seed, px, py);
    float u[2], lens[2];
    s2d(hp, 0, s, spp, u);
    float imageX = px + u[0], imageY = py + u[1];
    s2d(hp, 1, s, spp, lens);
    float timeU = s1d(hp, 2, s, spp);
    Ray r;
    bool dead = false;   // rayWeight 0: the sample's radiance is 0 (samplerrenderer.cpp:105-110)
    if (S.camType == PBRTGPU_CAMERA_REALISTIC) {
        RayDiff rd;
        dead = lens_ray_diff(S, imageX, imageY, lens[0], lens[1], timeU, path_wavelength(S, (int)item, s),
                             diff_key(hp, path_rng_index(S, item, s)), &r, &rd) == 0.f;
        if (P.fDiff) {   // DirectLighting: frame 0's differentials (dl_vertex reads them there)
            const size_t c = (size_t)P.cap;
            float *fd = P.fDiff + slot;
            const V vs[4] = {rd.rxo, rd.rxd, rd.ryo, rd.ryd};
            for (int k = 0; k < 4; ++k) {
                fd[(3 * k) * c] = vs[k].x;
                fd[(3 * k + 1) * c] = vs[k].y;
                fd[(3 * k + 2) * c] = vs[k].z;
            }
        }
        if (dead) {   // a ray no traversal hits; k_shade writes the zero radiance
            r.o = v3(0.f, 0.f, 0.f);
            r.d = v3(0.f, 0.f, 1.f);
            r.mint = 1.f;
            r.maxt = 0.f;
        }
    }
    else r = camera_ray(S.cam, imageX, imageY, lens[0], lens[1], timeU, S.camMotion);
    ray_store(P, RAY_C, slot, r);
    // AnimatedTransform::Interpolate (transform.cpp:356-381) of every instance at the path's
    // time, once per path: all of the path's rays carry this time
    for (int i = 0; i < P.nInst; ++i) {
        float m[16], minv[16];
        inst_interp((*sa(S.insts, (uint32_t)(i))), r.time, m, minv);
        float4 *o = P.instM + ((size_t)slot * P.nInst + i) * 8;
        for (int k = 0; k < 4; ++k) {
            o[k] = make_float4(m[4 * k], m[4 * k + 1], m[4 * k + 2], m[4 * k + 3]);
            o[4 + k] = make_float4(minv[4 * k], minv[4 * k + 1], minv[4 * k + 2], minv[4 * k + 3]);
        }
    }
    const uint32_t us = (uint32_t)slot;
    *sa(P.item, us) = (int)item;
    *sa(P.hp, us) = hp;
    *sa(P.pix, us) = ((uint32_t)py << 16) | (uint32_t)px;
    *sa(P.smp, us) = s;
    *sa(P.bounce, us) = dead ? -2 : -1;
    *sa(P.flags, us) = PF_CONT | PF_LZ;   // L = 0 and beta_0 = 1 are implicit (not stored)
    *sa(P.mt, us) = 0;
    *sa(P.mt, 4 * (uint32_t)P.cap + us) = path_seed(hp, path_rng_index(S, item, s));
}

// SpectralRenderer output of one band's path (spectralrenderer.cpp:158-188): a NaN
// radiance -> 0; else the value at the band's wavelength, Lerp(t, c[i], c[i+1]), into the
// band's indices of the sample's row; samplerDirection rows (one band per sample) and the
// last band of a singleDirection row also write the unassigned indices' zeros.  The
// luminance guard on the partly assigned spectrum runs per row after the wavefront
// (k_spec_guard).  Returns "zeroed".
template <int NB>
PGD_INLINE bool spectral_output(const DevScene &S, const float4 (&L)[Bands<NB>::NQ], float *__restrict__ Lout, int item,
                                uint32_t smp) {
    const int bi = S.specItems;
    const int row = bi > 1 ? item / bi : item;
    const int band = S.specMode == 1 ? item - row * bi : (int)(smp % (uint32_t)S.specBands);
    const int4 tb = (*sa(S.specTab, (uint32_t)(band)));
    bool nan = false;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const float v = 1.f * ((1.f * cmp(L[i / 4], i % 4)) + 0.f);
        nan = nan || isnan(v);
        if (i == tb.z) a = v;
        if (i == tb.z + 1) b = v;
    }
    const float t = __int_as_float(tb.w);
    const float val = (nan || tb.z < 0) ? 0.f : (1.f - t) * a + t * b;
    float *o = Lout + (size_t)row * NB;
    const bool tail = S.specMode == 2 || band == S.specBands - 1;
    // the bands' index ranges are contiguous from 0 up to the last band's end
    const int tailLo = S.specMode == 2 ? 0 : (*sa(S.specTab, (uint32_t)(S.specBands - 1))).y;
    for (int i = tb.x; i < tb.y; ++i) o[i] = val;
    if (tail)
        for (int i = tailLo; i < NB; ++i)
            if (i < tb.x || i >= tb.y) o[i] = 0.f;
    return nan;
}

// finished path -> guard (samplerrenderer.cpp:111-128) -> Lout[item]; returns "zeroed"
template <int NB>
PGD_INLINE bool path_output(const DevScene &S, const float4 (&L)[Bands<NB>::NQ], float *__restrict__ Lout, int item,
                            uint32_t smp) {
    constexpr int NQ = Bands<NB>::NQ;
    if (S.specMode) return spectral_output<NB>(S, L, Lout, item, smp);
    bool nan = false;
    float yy = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        float v = 1.f * ((1.f * cmp(L[i / 4], i % 4)) + 0.f);
        nan = nan || isnan(v);
        yy += (*sa(S.bandY, (uint32_t)(i))) * v;
    }
    bool bad = nan;
    if (!bad) {
        float yv = yy / S.yint;
        bad = (yv < -1e-5) || isinf(yv);
    }
    float *o = Lout + (size_t)item * NB;
    if (NB % 4 == 0) {
        float4 *o4 = reinterpret_cast<float4 *>(o);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float4 v = L[q];
            o4[q] = bad ? make_float4(0.f, 0.f, 0.f, 0.f)
                        : make_float4(1.f * ((1.f * v.x) + 0.f), 1.f * ((1.f * v.y) + 0.f), 1.f * ((1.f * v.z) + 0.f),
                                      1.f * ((1.f * v.w) + 0.f));
        }
    } else {
#pragma unroll
        for (int i = 0; i < NB; ++i) o[i] = bad ? 0.f : 1.f * ((1.f * cmp(L[i / 4], i % 4)) + 0.f);
    }
    return bad;
}

// ray requests produced by one shade step (DirectLighting batches: the MIS / shadow rays of
// batch samples j at ray slots slot + j * cap, bit j of mMask / sMask)
// t (path integrator): the slot's MT window goes to k_mt_init's list (mt_window_init)
// (DirectLighting k_shade: t = the slot was marked PF_DLNEE, it joins the light-sample list)
struct Pushes { bool c, m, s; uint32_t mMask, sMask; int sIdx, mIdx; bool t; };   // the shadow / MIS ray's ray slot (path)

// Additions to L a vertex makes before its direct light is known, in order: emitted
// radiance (path.cpp:67-68; bounce 0 or after a specular bounce) and the zero direct light
// of a vertex with nothing pending (L += beta * (nLights * 0)).  Both scale beta of the
// vertex; they are applied with the rest of the pass's L updates (shade_slot).
struct LAdds {
    bool emit;      // L += beta * Le
    int emitOff;    // spectrum pool offset of Le, or -1: Le = 0 (L += beta * 0)
    bool zero;      // L += beta * (nLights * 0)
};

// EstimateDirect (integrator.cpp:109-166) of light lightNum at a vertex (point p, shading
// normal n, BSDF bs): the light-sample term goes to A_vb with its shadow ray (PF_PA), the
// BSDF-sample term with MIS to B_vb with its MIS ray (PF_PB); the caller adds (0 [+ A]) [+ B]
// when the rays are answered.  Sets PF_PEND and the light index in fl.
// A, B: the slot's term buffers for this sample; rs: the ray slot its shadow / MIS rays use.
template <int NB, int FEAT>
// aMask (path integrator): A is the wave's region of the pass's A buffer; the lanes that write
// a term take its entries in lane order (whole 64-B lines instead of the scattered lines of
// divergent lanes) and *aMask records them for the reader of the next pass.  With masks it must
// stay ONE call site per k_shade pass (shade_vertex): the first active lane overwrites the wave's
// mask, and the next pass's readers rank themselves in it (PF_PA / PF_PB are set in the same
// pass).  A second call site, or a persistent k_shade reusing a wave for other slots, would read
// another lane's entry.  (DirectLighting passes null masks: its batches are indexed by the slot's
// light-sample list row, passed as `slot` -- here only the column of the M / K scratch and A / B.)
PGD_INLINE void estimate_direct(const DevScene &S, const PathSoA &P, int slot, int rs, Col<float4> A, Col<float4> B,
                                int lightNum, const BSDF &bs, PowMemo &pm, V p, V n, V wo, float rayEps, float time,
                                const float ul[3], const float ub[3], FVal &F, uint32_t &fl, Pushes &out,
                                unsigned long long *aMask, unsigned long long *mMask, int mKind) {
    constexpr int NQ = Bands<NB>::NQ;
    const uint32_t c = (uint32_t)P.cap;
    const float *sp = S.spectra;
    float4 *mb = P.M + slot, *kb = P.K + slot;
    PGD_T0(LIGHT);
    const pbrtgpu_light &Lt = (*sa(S.lights, (uint32_t)(lightNum)));
    const int flags = BSDF_ALL & ~BSDF_SPECULAR;
    fl |= PF_PEND | ((uint32_t)lightNum << PF_LIGHT_SHIFT);
    // ---- light sample -> A (added if the shadow ray is unoccluded)
    V wi;
    float lightPdf, bsdfPdf;
    Seg vis;
    Emit em;
    PGD_T0(LSAMP);
    light_sample_L<FEAT>(S, Lt, p, rayEps, ul, &wi, &lightPdf, &vis, &em);
    PGD_T1(LSAMP);
    PGD_T0(LEVAL);
    if (lightPdf > 0. && !emit_black<NB, FEAT>(S, em)) bsdf_f(pm, bs, wo, wi, flags, F);
    // no matching BxDF (e.g. the light below the surface): f is black, A unused
    const bool withA = lightPdf > 0. && !emit_black<NB, FEAT>(S, em) && !(F.mode == FV_SUM && F.n == 0);
    int rsS = rs;   // the shadow ray's record: path integrator without instances, at A's compacted entry
    if (aMask) {
        int rank;
        if (P.listMode) {   // identity compaction (PathSoA::listMode)
            if (withA) *aMask = ~0ull;
            rank = slot & 63;
        } else {
            const unsigned long long m = __ballot(withA), act = __ballot(true);
            const int lane = threadIdx.x & 63;
            if (lane == __ffsll((long long)act) - 1) *aMask = m;
            rank = __popcll(m & ((1ull << lane) - 1ull));
        }
        A.i += (uint32_t)rank;
        if (!P.nInst) rsS = (slot & ~63) + rank;
    }
    if (withA) {
        fval_prepare<NB, FEAT>(S, F, mb, c);
        float sc;
        if (em.point) sc = fabsf(vdot(wi, n)) / lightPdf;
        else {
            bsdfPdf = bsdf_pdf(pm, bs, wo, wi, flags);
            float weight = power_heuristic(lightPdf, bsdfPdf);
            sc = fabsf(vdot(wi, n)) * weight / lightPdf;
        }
        PGD_T1(LEVAL);
        PGD_T0(LSTORE);
        // A_i = (f_i * Li_i) * sc ; written while testing f for black (A unused if black)
        bool black = true;
#ifdef PGD_EXP_NO_ABLOOP   // timing experiment only: the A / B band loops skipped (wrong radiance)
        black = sc == 12345.f;
        if (!black) {} else
#endif
PGD_UNROLL_BANDS
        for (int q = 0; q < NQ; ++q) {
            float4 f = fval4<FEAT>(sp, F, q, mb, kb, c), e = emit4<FEAT>(S, em, q), a;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                cmp(a, k) = (cmp(f, k) * cmp(e, k)) * sc;
                if (4 * q + k < NB) black = black && (cmp(f, k) == 0.);
            }
#ifdef PGD_EXP_NO_AB   // timing experiment only: the A / B band stores suppressed (wrong radiance)
            if (__float_as_uint(a.x) == 0x7fc01234u)
#endif
            A[(uint32_t)q * c] = a;
        }
        if (!black) {
            Ray sr;
            sr.o = vis.o; sr.d = vis.d; sr.mint = vis.mint; sr.maxt = vis.maxt; sr.time = time;
            ray_store(P, RAY_S, rsS, sr);
            fl |= PF_PA;
            out.s = true;
            out.sIdx = rsS;
        }
        PGD_T1(LSTORE);
    }
    PGD_T1(LIGHT);
    PGD_T0(MIS);
    // ---- BSDF sample with MIS -> B (added if the MIS ray reaches this light: hits it
    // facing, for an area light; escapes the scene, for the environment)
#ifdef PGD_EXPERIMENT_NO_MIS   // timing experiment only: the MIS section's cost (wrong radiance)
    if (false) {
#else
    if (!em.point) {
#endif
        int sampledType;
        BSDFSampleState sst;
        bool keep = bsdf_sample_dir(pm, bs, wo, &wi, ub[0], ub[1], ub[2], &bsdfPdf, flags, &sampledType, F, sst);
        Ray mr;
        mr.o = p; mr.d = wi; mr.mint = rayEps; mr.maxt = INFINITY; mr.time = time;
        // a direction whose MIS ray cannot reach the light contributes nothing (B unused)
        if (keep) keep = mis_may_reach<FEAT>(S, Lt, mr);
        if (keep) bsdf_sample_rest(pm, bs, wo, wi, sst, &bsdfPdf, flags, sampledType, F);
        if (keep && bsdfPdf > 0. && !(F.mode == FV_SUM && F.n == 0)) {
            fval_prepare<NB, FEAT>(S, F, mb, c);
            float weight = 1.f;
            bool go = true;
            if (!(sampledType & BSDF_SPECULAR)) {
                lightPdf = light_pdf<FEAT>(S, Lt, p, wi);
                if (lightPdf == 0.) go = false;
                else weight = power_heuristic(bsdfPdf, lightPdf);
            }
            Emit eb;
            if ((FEAT & FEAT_INF) && Lt.type == PBRTGPU_LIGHT_INFINITE) {
                if (go) eb = inf_Le(S, Lt, wi);
            } else {
                eb.mode = Lt.is_black ? EM_BLACK : EM_POOL; eb.off = Lt.spec; eb.div = 1.f; eb.point = false;
            }
            const bool withB = go && !emit_black<NB, FEAT>(S, eb);
            int rsM = rs;   // the MIS ray's record: without instances, at B's compacted entry
            if (mMask) {   // path integrator: B in the wave's compacted region (as A)
                int rank;
                if (P.listMode) {
                    if (withB) *mMask = ~0ull;
                    rank = slot & 63;
                } else {
                    const unsigned long long m = __ballot(withB), act = __ballot(true);
                    const int lane = threadIdx.x & 63;
                    if (lane == __ffsll((long long)act) - 1) *mMask = m;
                    rank = __popcll(m & ((1ull << lane) - 1ull));
                }
                B.i += (uint32_t)rank;
                if (!P.nInst) rsM = (slot & ~63) + rank;
            }
            if (withB) {
                const float ad = fabsf(vdot(wi, n));
                bool black = true;
#ifdef PGD_EXP_NO_ABLOOP
                black = ad == 12345.f;
                if (!black) {} else
#endif
PGD_UNROLL_BANDS
                for (int q = 0; q < NQ; ++q) {
                    float4 f = fval4<FEAT>(sp, F, q, mb, kb, c), e = emit4<FEAT>(S, eb, q), b;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        cmp(b, k) = (((cmp(f, k) * cmp(e, k)) * ad) * weight) / bsdfPdf;
                        if (4 * q + k < NB) black = black && (cmp(f, k) == 0.);
                    }
#ifdef PGD_EXP_NO_AB
                    if (__float_as_uint(b.x) == 0x7fc01234u)
#endif
                    B[(uint32_t)q * c] = b;
                }
                if (!black) {
                    ray_store(P, mKind, rsM, mr);
                    fl |= PF_PB;
                    out.m = true;
                    out.mIdx = rsM;
                }
            }
        }
    }
    PGD_T1(MIS);
}

// One vertex of PathIntegrator::Li at bounce `vb` for the path in `slot`, whose
// continuation ray `ray` hit primitive `prim` at `thit`.  L stays in HBM: the vertex's own
// additions to L are returned in *la.  beta_vb is beta_of(vb) in HBM.  BSDF values are
// evaluated lazily per band quad (fval4).  Updates fl.
template <int NB, int FEAT>
PGD_INLINE Pushes shade_vertex(const DevScene &S, const PathSoA &P, int slot, int vb, const Ray &ray, int prim,
                               float thit, uint32_t &fl, LAdds *la, int qout, unsigned long long mb1) {
    constexpr int NQ = Bands<NB>::NQ;
    const uint32_t c = (uint32_t)P.cap, us = (uint32_t)slot;
    const float *sp = S.spectra;
    Pushes out = {false, false, false};
    float4 *mb = P.M + slot;
    Isect is;
    PGD_T0(ISECT);
    isect_fill(S, ray, prim, thit, is, inst_rec(P, slot));
    PGD_T1(ISECT);
    la->emit = false;
    la->zero = false;
    if (vb == 0 || (fl & PF_SPEC)) {
        const int al = is.al;
        la->emit = true;
        la->emitOff = (al >= 0 && vdot(is.dg.nn, vneg(ray.d)) > 0.f) ? (*sa(S.lights, (uint32_t)(al))).spec : -1;
    }
    PGD_T0(BSDF);
    const uint32_t hp = *sa(P.hp, us), s = *sa(P.smp, us), spp = (uint32_t)S.spp;
    // only the camera ray carries differentials (path.cpp:107 drops them); they matter only
    // to textured materials
    float diff[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // du/dv (x, y), dpdx, dpdy
    if ((FEAT & FEAT_TEX) && vb == 0) {
        const pbrtgpu_material &mt = (*sa(S.mats, (uint32_t)(is.mat)));
        if (mt.bump_tex >= 0 || mt.normal_tex >= 0 || mt.tex[0] >= 0 || mt.tex[1] >= 0 || mt.tex[2] >= 0 || mt.tex[3] >= 0 ||
            mt.ftex[0] >= 0 || mt.ftex[1] >= 0) {
            const uint32_t pxy = P.pix[slot];
            float u[2], lens[2];
            s2d(hp, 0, s, spp, u);
            s2d(hp, 1, s, spp, lens);
            const float timeU = s1d(hp, 2, s, spp);
            RayDiff rd = path_camera_diff(S, P.item[slot], hp, s, (int)(pxy & 0xffffu) + u[0], (int)(pxy >> 16) + u[1],
                                          lens[0], lens[1], timeU);
            V dpdx, dpdy;
            compute_differentials(is.dg, rd, diff, &dpdx, &dpdy);
            diff[4] = dpdx.x; diff[5] = dpdx.y; diff[6] = dpdx.z; diff[7] = dpdy.x; diff[8] = dpdy.y; diff[9] = dpdy.z;
        }
    }
    float4 *kb = P.K + slot;
    BSDF bs;
    V p, n;
    get_bsdf<FEAT>(S, is, diff, kb, c, bs, &p, &n);
    PGD_T1(BSDF);
    const V wo = vneg(ray.d);
    PowMemo pm;   // powf memo of this vertex's BSDF evaluations
    MT rng;
    const bool useMT = vb >= 3;
    if (useMT) {
        mt_load(P, slot, fl, rng);
        if (!rng.init) mt_init(rng);
    }
    const int nLights = S.nLights;
    fl &= ~(PF_PEND | PF_PA | PF_PB | PF_CONT | (PF_LIGHT_MASK << PF_LIGHT_SHIFT));
    FVal F;
#ifdef PGD_EXPERIMENT_NO_NEE
    if (false) {
#else
    if (nLights > 0) {
#endif
        float ul[3], ub[3], ulnum;
        if (!useMT) {
            float u2[2];
            ulnum = s1d(hp, DIM_1D(4 * vb + 1), s, spp);
            s2d(hp, DIM_2D(3 * vb + 0), s, spp, u2); ul[0] = u2[0]; ul[1] = u2[1];
            ul[2] = s1d(hp, DIM_1D(4 * vb + 0), s, spp);
            s2d(hp, DIM_2D(3 * vb + 1), s, spp, u2); ub[0] = u2[0]; ub[1] = u2[1];
            ub[2] = s1d(hp, DIM_1D(4 * vb + 2), s, spp);
        } else {
            ulnum = mt_float(rng);
            ul[0] = mt_float(rng); ul[1] = mt_float(rng); ul[2] = mt_float(rng);
            ub[0] = mt_float(rng); ub[1] = mt_float(rng); ub[2] = mt_float(rng);
        }
        int lightNum = (int)floorf(ulnum * nLights);
        if (lightNum > nLights - 1) lightNum = nLights - 1;
        estimate_direct<NB, FEAT>(S, P, slot, slot, A_reg<NB>(P, qout, slot), B_reg<NB>(P, qout, slot), lightNum, bs, pm,
                                  p, n, wo, is.rayEps, ray.time, ul, ub, F, fl, out, A_mask(P, qout, slot),
                                  B_mask(P, qout, slot), mis_kind(qout));
        if (!(fl & (PF_PA | PF_PB))) {
            // nothing can add to Ld: finish now (L += beta * (nLights * 0), nLights * 0 == 0)
            la->zero = true;
            fl &= ~PF_PEND;
        }
    } else la->zero = true;   // L += beta * 0
    // ---- path continuation
    PGD_T0(CONT);
    float up[3];
    if (!useMT) {
        float u2[2];
        s2d(hp, DIM_2D(3 * vb + 2), s, spp, u2); up[0] = u2[0]; up[1] = u2[1];
        up[2] = s1d(hp, DIM_1D(4 * vb + 3), s, spp);
    } else {
        up[0] = mt_float(rng); up[1] = mt_float(rng); up[2] = mt_float(rng);
    }
    V wi;
    float pdf;
    int sflags;
    PGD_T0(CSAMP);
    bsdf_sample_f(pm, bs, wo, &wi, up[0], up[1], up[2], &pdf, BSDF_ALL, &sflags, F);
    PGD_T1(CSAMP);
    PGD_T0(CBAND);
    bool cont = pdf != 0. && !(F.mode == FV_SUM && F.n == 0);
    if (cont) {
        fval_prepare<NB, FEAT>(S, F, mb, c);
        const float ad = fabsf(vdot(wi, n));
        const Col<float4> bv = beta_rd<NB>(P, vb, 1, slot, mb1);
        float4 nb4[NQ];
        bool black = true;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float4 f = fval4<FEAT>(sp, F, q, mb, kb, c), b = beta_q(bv, q, c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                cmp(nb4[q], k) = cmp(b, k) * ((cmp(f, k) * ad) / pdf);
                if (4 * q + k < NB) black = black && (cmp(f, k) == 0.);
            }
        }
        cont = !black;
        if (cont) {
            if (sflags & BSDF_SPECULAR) fl |= PF_SPEC; else fl &= ~PF_SPEC;
            if (vb > 3) {
                float yy = 0.f;
#pragma unroll
                for (int i = 0; i < NB; ++i) yy += (*sa(S.bandY, (uint32_t)(i))) * cmp(nb4[i / 4], i % 4);
                float cp = pmin(.5f, yy / S.yint);
                if (mt_float(rng) > cp) cont = false;
                else {
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        nb4[q].x /= cp; nb4[q].y /= cp; nb4[q].z /= cp; nb4[q].w /= cp;
                    }
                }
            }
            if (vb == S.maxDepth) cont = false;
        }
        // beta_{vb+1}: the continuing lanes take the wave region's entries in lane order
        const int buf = pass_buf(P, 0);
        uint32_t bRank;
        if (P.listMode) {   // identity compaction (PathSoA::listMode)
            if (cont) *beta_mask(P, buf, slot) = ~0ull;
            bRank = (uint32_t)(slot & 63);
        } else {
            const unsigned long long bm = __ballot(cont), act = __ballot(true);
            const int lane = threadIdx.x & 63;
            if (lane == __ffsll((long long)act) - 1) *beta_mask(P, buf, slot) = bm;
            bRank = (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
        }
        if (cont) {
            Col<float4> bn = beta_reg<NB>(P, buf, slot);
            bn.i += bRank;
            bool nf = false;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                bn[(uint32_t)q * c] = nb4[q];
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (4 * q + k < NB) nf = nf || !(fabsf(cmp(nb4[q], k)) < INFINITY);
            }
            const uint32_t nfBit = (uint32_t)PF_NF0 << ((vb + 1) % 3);
            fl = nf ? (fl | nfBit) : (fl & ~nfBit);
            Ray nray;
            nray.o = p; nray.d = wi; nray.mint = is.rayEps; nray.maxt = INFINITY; nray.time = ray.time;
            ray_store(P, RAY_C, slot, nray);
            fl |= PF_CONT;
            out.c = true;
#ifndef PGD_EXP_NO_MT_LIST   // A/B experiment: the window computed inline at vertex 3 instead
            out.t = vb == 2 && !(fl & PF_MTINIT);   // vertex 3 makes the path's first MT draws
#endif
        }
    }
    if (useMT) {
        mt_store(P, slot, rng);
        if (rng.init) fl |= PF_MTINIT;
    }
    PGD_T1(CBAND);
    PGD_T1(CONT);
    return out;
}

// k_shade body for one slot: finish pending direct light, process the next vertex.
// Returns the ray requests; *done when the path has produced its radiance.  L is read and
// updated once, after the vertex: the finish of vertex b (beta_b, A_b, B_b), then the
// vertex's own additions -- the order of PathIntegrator::Li.  Keeping L out of registers
// through shade_vertex is what lets the kernel fit its occupancy target.
template <int NB, int FEAT>
PGD_INLINE Pushes shade_slot(const DevScene &S, const PathSoA &P, int slot, float *__restrict__ Lout, bool *done,
                             bool *zeroed, int qout) {
    constexpr int NQ = Bands<NB>::NQ;
    const uint32_t c = (uint32_t)P.cap, us = (uint32_t)slot, rc = (uint32_t)P.rcap;
    PGD_T0(LOAD);
    uint32_t fl = *sa(P.flags, us);
    const int b = *sa(P.bounce, us);
    const WaveMasks wm = wave_masks(P, qout, slot);
    Pushes out = {false, false, false};
    PGD_T1(LOAD);
    PGD_T0(FINISH);
    // which terms of vertex b's direct light arrived (decided before shade_vertex reuses the
    // slot's MIS ray)
    const bool fin = (fl & PF_PEND) != 0;
    bool useA = false, useB = false;
    if (fin) {
        // the shadow ray's answer: at A's compacted entry (path integrator without instances)
        useA = (fl & PF_PA) && !*sa(P.occ, P.nInst ? us : (us & ~63u) + (uint32_t)wave_rank(wm.a, slot));
        if (fl & PF_PB) {
            const int ln = (int)(fl >> PF_LIGHT_SHIFT);
            const int mi = P.nInst ? slot : (slot & ~63) + wave_rank(wm.b, slot);   // the MIS ray's record
            int mp = *sa(P.hitPrim, rc + (uint32_t)mi);
            if ((FEAT & FEAT_INF) && (*sa(S.lights, (uint32_t)(ln))).type == PBRTGPU_LIGHT_INFINITE) useB = mp < 0;   // Li = light->Le(ray)
            else if (mp >= 0 && (*sa(S.prims, (uint32_t)(mp))).area_light == ln) {
                Ray mr = ray_load(P, mis_kind(qout ^ 1), mi);   // written by the pass before
                useB = vdot(isect_nn(S, mr, mp, *sa(P.hitT, rc + (uint32_t)mi), inst_rec(P, slot)), vneg(mr.d)) > 0.f;   // DiffuseAreaLight::L
            }
        }
        fl &= ~(PF_PEND | PF_PA | PF_PB);
    }
    PGD_T1(FINISH);
    LAdds la = {false, -1, false};
    int esc = 0;   // continuation ray escaped: 1 camera ray (sum of Le), 2 after a specular bounce
    int vb = b;
    if (fl & PF_CONT) {
        vb = b + 1;
        const int prim = *sa(P.hitPrim, us);
        fl &= ~PF_CONT;
        if (prim < 0) esc = vb == 0 ? 1 : ((fl & PF_SPEC) ? 2 : 0);
        else {
            Ray ray = ray_load(P, RAY_C, slot);
            out = shade_vertex<NB, FEAT>(S, P, slot, vb, ray, prim, *sa(P.hitT, us), fl, &la, qout, wm.b1);
            *sa(P.bounce, us) = vb;
        }
    }
    PGD_T0(OUT);
#ifdef PGD_EXP_NO_OUT   // register-budget experiment only: the L update / output compiled out
    *sa(P.flags, us) = fl;
    *done = !(fl & (PF_CONT | PF_PEND));
    *zeroed = useA && useB;
    return out;
#endif
    // L += beta * 0 leaves L unchanged for a finite beta (up to the sign of a zero, which
    // path_output's "+ 0.f" erases), so those additions are skipped unless beta is
    // non-finite (NaN result); L is read and written only when something changes it
    const bool addFin = fin && (useA || useB || beta_nonfinite(fl, b));
    const bool addEmit = la.emit && (la.emitOff >= 0 || beta_nonfinite(fl, vb));
    const bool addZero = la.zero && beta_nonfinite(fl, vb);
    const bool infLe = (FEAT & FEAT_INF) && S.nInf > 0;
    const bool addEsc = esc == 1 ? infLe : (esc == 2 && (infLe || beta_nonfinite(fl, vb)));
    *done = !(fl & (PF_CONT | PF_PEND));
    *zeroed = false;
    if (!(addFin || addEmit || addZero || addEsc || *done)) {
        *sa(P.flags, us) = fl;
        PGD_T1(OUT);
        return out;
    }
    float4 L[NQ];
    const bool lz = (fl & PF_LZ) != 0;
#pragma unroll
    for (int q = 0; q < NQ; ++q) L[q] = lz ? make_float4(0.f, 0.f, 0.f, 0.f) : *sa(P.L, (uint32_t)q * c + us);
    if (addFin) {   // L += beta_b * (nLights * Ld), Ld = (0 [+ A]) [+ B]
        const float nl = (float)S.nLights;
        // A of vertex b: written by the previous pass (queue set qout ^ 1), compacted per wave
        Col<float4> A = A_reg<NB>(P, qout ^ 1, slot), B = B_reg<NB>(P, qout ^ 1, slot);
        A.i += (uint32_t)wave_rank(wm.a, slot);
        B.i += (uint32_t)wave_rank(wm.b, slot);
        const Col<float4> bb4 = beta_rd<NB>(P, b, 2, slot, wm.b2);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float4 bt = beta_q(bb4, q, c);
#ifdef PGD_EXP_NO_ABLOOP
            float4 a = make_float4(0.1f, 0.f, 0.f, 0.f), bb = a;
#else
            float4 a = useA ? A[(uint32_t)q * c] : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 bb = useB ? B[(uint32_t)q * c] : make_float4(0.f, 0.f, 0.f, 0.f);
#endif
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float Ld = 0.f;
                if (useA) Ld += cmp(a, k);
                if (useB) Ld += cmp(bb, k);
                cmp(L[q], k) += cmp(bt, k) * (nl * Ld);
            }
        }
    }
    if (addEmit || addZero) {   // vertex vb: L += beta * Le, then L += beta * (nLights * 0)
        const Col<float4> bv4 = beta_rd<NB>(P, vb, 1, slot, wm.b1);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float4 bt = beta_q(bv4, q, c);
            if (addEmit) {
                const float4 e = la.emitOff >= 0 ? ld4(S.spectra, la.emitOff + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
                L[q].x += bt.x * e.x; L[q].y += bt.y * e.y; L[q].z += bt.z * e.z; L[q].w += bt.w * e.w;
            }
            if (addZero) { L[q].x += bt.x * 0.f; L[q].y += bt.y * 0.f; L[q].z += bt.z * 0.f; L[q].w += bt.w * 0.f; }
        }
    }
    if (addEsc && esc == 1) {
        // SamplerRenderer::Li (samplerrenderer.cpp:237-240): Li = sum of the lights' Le, zero
        // for area and point lights
        if ((FEAT & FEAT_INF) && S.nInf > 0) {
            const Ray ray = ray_load(P, RAY_C, slot);
            for (int l = 0; l < S.nLights; ++l)
                if ((*sa(S.lights, (uint32_t)(l))).type == PBRTGPU_LIGHT_INFINITE) {
                    const Emit e = inf_Le(S, (*sa(S.lights, (uint32_t)(l))), ray.d);
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        float4 v = emit4<FEAT>(S, e, q);
                        L[q].x += v.x; L[q].y += v.y; L[q].z += v.z; L[q].w += v.w;
                    }
                }
        }
    } else if (addEsc && esc == 2) {
        // path.cpp:92-96: L += beta * Le(ray) for every light
        V d = v3(0.f, 0.f, 0.f);
        if ((FEAT & FEAT_INF) && S.nInf > 0) d = ray_load(P, RAY_C, slot).d;
        for (int l = 0; l < S.nLights; ++l) {
            Emit e;
            e.mode = EM_BLACK;
            if ((FEAT & FEAT_INF) && (*sa(S.lights, (uint32_t)(l))).type == PBRTGPU_LIGHT_INFINITE) e = inf_Le(S, (*sa(S.lights, (uint32_t)(l))), d);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                float4 bt = beta_q(beta_rd<NB>(P, vb, 1, slot, wm.b1), q, c), v = emit4<FEAT>(S, e, q);
                L[q].x += bt.x * v.x; L[q].y += bt.y * v.y; L[q].z += bt.z * v.z; L[q].w += bt.w * v.w;
            }
        }
    }
    if (*done) *zeroed = path_output<NB>(S, L, Lout, *sa(P.item, us), *sa(P.smp, us));
    else {
#pragma unroll
        for (int q = 0; q < NQ; ++q) *sa(P.L, (uint32_t)q * c + us) = L[q];
        fl &= ~PF_LZ;
    }
    *sa(P.flags, us) = fl;
    PGD_T1(OUT);
    return out;
}

#ifndef PGD_SHADE_BLOCK
#define PGD_SHADE_BLOCK 256
#endif
static const int kShadeBlock = PGD_SHADE_BLOCK;
// The per-wave compaction of A / B / beta and of the shadow / MIS ray records (wave region =
// slot & ~63, rank = lanes below that wrote) needs whole 64-lane waves with slot = block * blockDim
// + lane, every pass
static_assert(kShadeBlock % 64 == 0, "k_shade blocks must be whole waves");
static const int kTailBlock = 64;   // k_tail (shade.hip): one wave per block, its traversal stack in LDS
// k_shade<NB, FEAT> launch (defined in shade.hip, one translation unit per variant)
template <int NB, int FEAT>
hipError_t launch_shade(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                        float *Lout);
// k_shade with the DirectLightingIntegrator step (FEAT as for the path integrator)
template <int NB, int FEAT>
hipError_t launch_shade_dl(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src,
                           int qout, float *Lout);
// k_dl_nee: the light-sample batches of the DirectLighting slots k_shade marked (PF_DLNEE)
template <int NB, int FEAT>
hipError_t launch_dl_nee(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, int qout);
// k_dl_spec: their specular branches and frame pops (PF_DLSPEC), then k_regen: the slots it
// freed take the next camera samples
template <int NB, int FEAT>
hipError_t launch_dl_spec(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                          float *Lout);
// k_regen alone (instantiated once per band count, in the FEAT_ALL DirectLighting object)
template <int NB>
hipError_t launch_regen(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout);
// k_tail: the drain's last live paths run to their end in one launch (path integrator, no instances)
template <int NB, int FEAT>
hipError_t launch_tail(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, int q, float *Lout,
                       int maxSteps);
// k_shade with the MetadataIntegrator step
template <int NB, int FEAT>
hipError_t launch_shade_meta(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src,
                             int qout, float *Lout);

}  // namespace pgd
