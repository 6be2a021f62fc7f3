// shade.hip -- the k_shade kernel (one vertex of PathIntegrator::Li per live path slot plus
// path regeneration, wavefront.h) for one band count / feature set.  Compiled once per
// (SHADE_NB, SHADE_FEAT) so the large shading variants build in parallel; pbrtgpu.hip
// launches them through launch_shade<NB, FEAT>.
#include <hip/hip_runtime.h>
#include "pbrtgpu.h"
#include "device.h"
#include "wavefront.h"
#include "directlighting.h"
#include "metadata.h"

#if !defined(SHADE_NB) || !defined(SHADE_FEAT)
#error "compile with -DSHADE_NB=<3|30|32|60> -DSHADE_FEAT=<0|6|7|8|9> [-DSHADE_DL=1]"
#endif
#ifndef SHADE_DL
#define SHADE_DL 0
#endif

namespace pgd {

#ifdef PGD_SECTIONS
// per-section totals of this variant, each on its own 128-byte line, 8 copies striped by block
#define PGD_CAT2(a, b, c) a##b##_##c
#define PGD_CAT(a, b, c) PGD_CAT2(a, b, c)
static __device__ unsigned long long pgd_sec_total[8 * SEC_N * 16];
#if !SHADE_DL
extern "C" int PGD_CAT(pgd_sections_read_, SHADE_NB, SHADE_FEAT)(unsigned long long *out, int reset) {
    unsigned long long h[8 * SEC_N * 16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(pgd_sec_total), sizeof(h)) != hipSuccess) return -1;
    for (int k = 0; k < SEC_N; ++k)
        for (int c = 0; c < 8; ++c) out[k] += h[c * SEC_N * 16 + k * 16];
    if (reset) {
        for (auto &v : h) v = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(pgd_sec_total), h, sizeof(h)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
#endif

// inclusive prefix sum over the wave's 64 lanes
__device__ __forceinline__ uint32_t wave_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    return x;
}

// shading pass over every slot: finish / advance live paths, regenerate free slots, and
// queue the next pass's rays into queue set qout (block-aggregated queue pushes)
// occupancy target: 3 waves/SIMD (<= 168 VGPRs) for <= 32 bands costs a few spilled
// registers and beats the unconstrained 200-VGPR / 2-wave build (C2 shade 372 -> 335
// ms/frame, r01l ablation; 4 waves spills ~90 registers and loses); 60 bands: 2 waves
// The DirectLighting / metadata step at 3 waves/SIMD since its light-sample batches moved to
// k_dl_nee (C2 DL shade 409 -> 396 ms/frame; k_dl_nee itself is fastest at 2 waves: 3 waves 421,
// unconstrained 561).  Before the batches existed, a 3-wave build gave non-deterministic radiance
// on coverage.pbrt (tools/dbg/dl_debug4.py); every variant since passes
// tools/dbg/dl_determinism.py (3 identical runs, oracle bit for bit)
#ifndef PGD_SHADE_ATTR
#if SHADE_DL
#define PGD_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(3, 3)))
#else
#define PGD_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(SHADE_NB > 32 ? 2 : 3, SHADE_NB > 32 ? 2 : 3)))
#endif
#endif
// MODE: the SurfaceIntegrator's step -- PathIntegrator (wavefront.h), DirectLightingIntegrator
// (directlighting.h) or MetadataIntegrator (metadata.h)
enum { MODE_PATH = 0, MODE_DL = 1, MODE_META = 2 };
// LIST (path integrator): the drain's instantiation over the live slots' list (PathSoA::listMode);
// the other one has listMode constant 0, so its compaction code is the per-wave one alone
template <int NB, int FEAT, int MODE, bool LIST>
__global__ __launch_bounds__(kShadeBlock) PGD_SHADE_ATTR void k_shade(DevScene S, PathSoA P0, ItemSrc src, int qout,
                                                       float *__restrict__ Lout) {
    PathSoA P = P0;
    P.listMode = LIST ? 1 : 0;
#ifdef PGD_SECTIONS
    if (threadIdx.x < SEC_N) pgd_secs[threadIdx.x] = 0;
    __syncthreads();
#endif
    if (FEAT & FEAT_MEAS) kd_lds_fill(S);   // the measured-BRDF kd-trees, once per block
    int slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool inRange = slot < P.cap;
    if (LIST) {   // the drain: thread i takes the i-th live slot
        const uint32_t i = (uint32_t)slot;
        // every pass of a read-back batch checks its own list against its grid (the host sees
        // only the last pass's count): a longer list would leave slots unshaded
        if (i == 0 && P.cnt[CNT_LIVE] > gridDim.x * blockDim.x) atomicOr(&P.cnt[CNT_ERR], 2u);
        inRange = i < P.cnt[CNT_LIVE];
        slot = inRange ? (int)P.live[i] : 0;
    }
    Pushes pu = {false, false, false, 0u, 0u};
    bool freeSlot = inRange && P.item[slot] < 0;
    bool zeroed = false;
    if (inRange && !freeSlot) {
        bool done;
        if (P.bounce[slot] == -2) {   // a camera ray of weight 0 (lens camera): radiance 0
            float4 Z[Bands<NB>::NQ];
#pragma unroll
            for (int q = 0; q < Bands<NB>::NQ; ++q) Z[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            (void)path_output<NB>(S, Z, Lout, P.item[slot], P.smp[slot]);
            done = true;
        }
        else if (MODE == MODE_DL) pu = shade_slot_dl<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
        else if (MODE == MODE_META) pu = shade_slot_meta<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
        else pu = shade_slot<NB, FEAT>(S, P, slot, Lout, &done, &zeroed, qout);
        if (done) { P.item[slot] = -1; freeSlot = true; }
    }
    if (__ballot(zeroed)) {
        const unsigned long long m = __ballot(zeroed);
        if ((threadIdx.x & 63) == 0) atomicAdd(&P.cnt[CNT_ZEROED], (uint32_t)__popcll(m));
    }
    if (MODE == MODE_DL) {   // the slots marked for k_dl_nee join its list, in lane order
        const unsigned long long bN = __ballot(pu.t);
        if (bN) {
            uint32_t base = 0u;
            if ((threadIdx.x & 63) == __ffsll((long long)bN) - 1) base = atomicAdd(&P.cnt[CNT_DLN], (uint32_t)__popcll(bN));
            base = __shfl(base, __ffsll((long long)bN) - 1);
            if (pu.t) P.dlList[base + (uint32_t)__popcll(bN & ((1ull << (threadIdx.x & 63)) - 1ull))] = (uint32_t)slot;
        }
    }
    // Regeneration and the queue pushes of the block in one step -- one pair of barriers and at
    // most three atomics per block: free slots take the next camera samples; the closest-hit
    // queue gets the block's continuation / child rays, then the regenerated camera rays, then
    // the MIS rays; the shadow queue the shadow rays.  Entries are in block order.
    PGD_T0(PUSH);
    __shared__ uint32_t qsh[24];   // per wave [w][4]: want, C, M, S (totals -> offsets); bases
    __shared__ uint32_t qtw[5];    // path integrator: per wave the MT-window list entries -> offsets; base
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const bool want = freeSlot && *(volatile uint32_t *)&P.cnt[CNT_NEXT] < src.nItems;
    const unsigned long long bW = __ballot(want), bC = __ballot(pu.c);
    const unsigned long long bT = MODE == MODE_PATH ? __ballot(pu.t) : 0ull;
    if (MODE == MODE_PATH && lane == 0) qtw[wave] = (uint32_t)__popcll(bT);
    uint32_t pm, ps, tm, ts;   // this thread's prefix and the wave total, MIS / shadow entries
    if (MODE == MODE_DL) {   // a batch of light samples per slot: ray slots slot + j * cap
        const uint32_t nm = (uint32_t)__popc(pu.mMask), ns = (uint32_t)__popc(pu.sMask);
        const uint32_t im = wave_scan(nm), is = wave_scan(ns);
        pm = im - nm; ps = is - ns;
        tm = __shfl(im, 63); ts = __shfl(is, 63);
    } else {
        const unsigned long long bM = __ballot(pu.m), bS = __ballot(pu.s);
        pm = (uint32_t)__popcll(bM & lt); ps = (uint32_t)__popcll(bS & lt);
        tm = (uint32_t)__popcll(bM); ts = (uint32_t)__popcll(bS);
    }
    if (lane == 0) {
        qsh[4 * wave + 0] = (uint32_t)__popcll(bW); qsh[4 * wave + 1] = (uint32_t)__popcll(bC);
        qsh[4 * wave + 2] = tm; qsh[4 * wave + 3] = ts;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t[4] = {0u, 0u, 0u, 0u};
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
            for (int k = 0; k < 4; ++k) { const uint32_t v = qsh[4 * w + k]; qsh[4 * w + k] = t[k]; t[k] += v; }
        const uint32_t nb = t[0] ? atomicAdd(&P.cnt[CNT_NEXT], t[0]) : 0u;
        const uint32_t nReg = nb >= src.nItems ? 0u : min(t[0], src.nItems - nb);
        const uint32_t nQC = t[1] + nReg + t[2];
        qsh[16] = nb; qsh[17] = nReg; qsh[18] = nQC ? atomicAdd(&P.cnt[CNT_QC(qout)], nQC) : 0u;
        qsh[19] = t[3] ? atomicAdd(&P.cnt[CNT_QS(qout)], t[3]) : 0u;
        qsh[20] = t[1];
        if (MODE == MODE_PATH) {
            uint32_t tt = 0u;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { const uint32_t v = qtw[w]; qtw[w] = tt; tt += v; }
            qtw[4] = tt ? atomicAdd(&P.cnt[CNT_QT(qout)], tt) : 0u;
        }
    }
    __syncthreads();
    uint32_t *qC = P.qC + (size_t)qout * 2 * P.rcap, *qS = P.qS + (size_t)qout * P.rcap;
    const uint32_t qcBase = qsh[18], nC = qsh[20], nReg = qsh[17];
    if (pu.c) qC[qcBase + qsh[4 * wave + 1] + (uint32_t)__popcll(bC & lt)] = (uint32_t)slot << 1;
    if (MODE == MODE_PATH && pu.t) P.qT[(size_t)qout * P.cap + qtw[4] + qtw[wave] + (uint32_t)__popcll(bT & lt)] = (uint32_t)slot;
    if (want) {
        const uint32_t r = qsh[4 * wave + 0] + (uint32_t)__popcll(bW & lt);   // block order among free slots
        if (r < nReg) {
            path_start<NB>(S, P, src, slot, qsh[16] + r);
            qC[qcBase + nC + r] = (uint32_t)slot << 1;
        }
    }
    uint32_t km = qcBase + nC + nReg + qsh[4 * wave + 2] + pm, ks = qsh[19] + qsh[4 * wave + 3] + ps;
    if (MODE == MODE_DL) {
        for (uint32_t m = pu.mMask; m; m &= m - 1u) qC[km++] = ((uint32_t)(slot + (__ffs(m) - 1) * P.cap) << 1) | 1u;
        for (uint32_t m = pu.sMask; m; m &= m - 1u) qS[ks++] = (uint32_t)(slot + (__ffs(m) - 1) * P.cap);
    } else {
        if (pu.m) qC[km] = ((uint32_t)(MODE == MODE_PATH ? pu.mIdx : slot) << 1) | 1u;
        if (pu.s) qS[ks] = (uint32_t)(MODE == MODE_PATH ? pu.sIdx : slot);
    }
    PGD_T1(PUSH);
#ifdef PGD_SECTIONS
    __syncthreads();
    if (threadIdx.x < SEC_N) atomicAdd(&pgd_sec_total[(blockIdx.x & 7) * SEC_N * 16 + threadIdx.x * 16], pgd_secs[threadIdx.x]);
#endif
}

template <int NB, int FEAT, int MODE>
static hipError_t launch(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                         float *Lout) {
    const size_t lds = ((FEAT & FEAT_MEAS) && S.kdInLds) ? (size_t)S.nKd * 32 : 0;
    if constexpr (MODE == MODE_PATH || MODE == MODE_DL) {
        if (P.listMode) {
            hipLaunchKernelGGL((k_shade<NB, FEAT, MODE, true>), dim3(grid), dim3(kShadeBlock), lds, stream, S, P, src, qout, Lout);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_shade<NB, FEAT, MODE, false>), dim3(grid), dim3(kShadeBlock), lds, stream, S, P, src, qout, Lout);
    return hipGetLastError();
}
#if SHADE_DL
// The DirectLighting step's two kernels after k_shade in each pass, in kernels of their own so
// that no step carries another's registers (k_shade with the specular branches inlined peaked at
// ~330 VGPRs: 559 spilled at 3 waves/SIMD); their rays join the pass's queues.
//   k_dl_nee:  the light-sample batches of the slots k_shade marked PF_DLNEE
//              (directlighting.h dl_light_batches);
//   k_dl_spec: the specular branches and frame pops of the slots marked PF_DLSPEC by k_shade or
//              by k_dl_nee (dl_spec_step);
//   k_regen:   the slots whose sample completed in k_dl_spec take the next camera samples in the
//              same pass (as k_shade's regeneration does for the others), so a slot is not left
//              idle for a pass -- without it a C2 frame took 76 passes instead of 52.
// 2 waves/SIMD for <= 32 bands (k_dl_nee: 47 VGPRs spilled, k_dl_spec: 148) and for the 60-band
// FEAT 0 k_dl_nee since the light-sample list (90 spilled, 768 B of scratch per lane); the 60-band
// k_dl_spec and the all-features k_dl_nee stay at 1 wave/SIMD to keep within tools/kernel_budget.py
// (at 2 waves k_dl_nee<60, 7> spills 225 VGPRs, 1,300 B; k_dl_spec<60, 0> 160, 1,056 B once
// shinymetal's conductor mirror lobe joined the specular sampler); the all-features k_dl_spec at
// every band count runs at 1 wave since the noise textures (FBm / Turbulence inlined: 174 spilled at
// 2 waves, 1,040 B) -- the FEAT 0 builds of the benchmark configs are unaffected
#define PGD_NEE_WAVES ((SHADE_NB > 32 && (SHADE_FEAT & 7) != 0) ? 1 : 2)   // (FEAT_BASIC: as FEAT 0)
#define PGD_SPEC_WAVES ((SHADE_NB > 32 || (SHADE_FEAT & 7) != 0) ? 1 : 2)
#ifndef PGD_NEE_ATTR
#define PGD_NEE_ATTR __attribute__((amdgpu_waves_per_eu(PGD_NEE_WAVES, PGD_NEE_WAVES)))
#endif
#ifndef PGD_SPEC_ATTR
#define PGD_SPEC_ATTR __attribute__((amdgpu_waves_per_eu(PGD_SPEC_WAVES, PGD_SPEC_WAVES)))
#endif
// k_dl_nee: thread i takes entry i of the pass's light-sample list (PathSoA::dlList, CNT_DLN
// entries); blocks past its end return at once
template <int NB, int FEAT>
__global__ __launch_bounds__(kShadeBlock) PGD_NEE_ATTR void k_dl_nee(DevScene S, PathSoA P, int qout) {
    const uint32_t n = P.cnt[CNT_DLN], i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x * blockDim.x >= n) return;   // (block-uniform, before any barrier)
    if (FEAT & FEAT_MEAS) kd_lds_fill(S);   // measured-BRDF lookups read the LDS copy (as in k_shade)
    const int slot = i < n ? (int)P.dlList[i] : P.cap;
    const int rb = P.nInst ? slot : (int)i;   // the ray slots' base (dl_light_batches)
    Pushes pu = {false, false, false, 0u, 0u};
    if (slot < P.cap && P.item[slot] >= 0 && (P.flags[slot] & PF_DLNEE)) dl_light_batches<NB, FEAT>(S, P, slot, (int)i, pu);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t qsh[12];   // per wave: M, S totals -> offsets; bases
    const uint32_t nm = (uint32_t)__popc(pu.mMask), ns = (uint32_t)__popc(pu.sMask);
    const uint32_t im = wave_scan(nm), is = wave_scan(ns);
    if (lane == 63) { qsh[2 * wave] = im; qsh[2 * wave + 1] = is; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t[2] = {0u, 0u};
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
            for (int k = 0; k < 2; ++k) { const uint32_t v = qsh[2 * w + k]; qsh[2 * w + k] = t[k]; t[k] += v; }
        qsh[8] = t[0] ? atomicAdd(&P.cnt[CNT_QC(qout)], t[0]) : 0u;
        qsh[9] = t[1] ? atomicAdd(&P.cnt[CNT_QS(qout)], t[1]) : 0u;
    }
    __syncthreads();
    uint32_t *qC = P.qC + (size_t)qout * 2 * P.rcap, *qS = P.qS + (size_t)qout * P.rcap;
    uint32_t km = qsh[8] + qsh[2 * wave] + im - nm, ks = qsh[9] + qsh[2 * wave + 1] + is - ns;
    for (uint32_t m = pu.mMask; m; m &= m - 1u) qC[km++] = ((uint32_t)(rb + (__ffs(m) - 1) * P.cap) << 1) | 1u;
    for (uint32_t m = pu.sMask; m; m &= m - 1u) qS[ks++] = (uint32_t)(rb + (__ffs(m) - 1) * P.cap);
}
template <int NB, int FEAT>
__global__ __launch_bounds__(kShadeBlock) PGD_SPEC_ATTR void k_dl_spec(DevScene S, PathSoA P, int qout,
                                                                      float *__restrict__ Lout) {
    if (FEAT & FEAT_MEAS) kd_lds_fill(S);
    int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (P.listMode) slot = (uint32_t)slot < P.cnt[CNT_LIVE] ? (int)P.live[slot] : P.cap;   // the drain (k_shade)
    Pushes pu = {false, false, false, 0u, 0u};
    bool done = false, zeroed = false;
    if (slot < P.cap && P.item[slot] >= 0 && (P.flags[slot] & PF_DLSPEC)) {
        pu = dl_spec_step<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
        if (done) P.item[slot] = -1;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long bZ = __ballot(zeroed), bC = __ballot(pu.c);
    if (lane == 0 && bZ) atomicAdd(&P.cnt[CNT_ZEROED], (uint32_t)__popcll(bZ));
    __shared__ uint32_t qsh[8];   // per wave: child rays -> offsets; base
    if (lane == 0) qsh[wave] = (uint32_t)__popcll(bC);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0u;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { const uint32_t v = qsh[w]; qsh[w] = t; t += v; }
        qsh[7] = t ? atomicAdd(&P.cnt[CNT_QC(qout)], t) : 0u;
    }
    __syncthreads();
    if (pu.c) {
        uint32_t *qC = P.qC + (size_t)qout * 2 * P.rcap;
        qC[qsh[7] + qsh[wave] + (uint32_t)__popcll(bC & ((1ull << lane) - 1ull))] = (uint32_t)slot << 1;
    }
}
// regeneration of free slots (the tail of k_shade's queue step, for the slots k_dl_spec freed)
template <int NB>
__global__ __launch_bounds__(kShadeBlock) void k_regen(DevScene S, PathSoA P, ItemSrc src, int qout) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool want = slot < P.cap && P.item[slot] < 0 && *(volatile uint32_t *)&P.cnt[CNT_NEXT] < src.nItems;
    const unsigned long long bW = __ballot(want);
    __shared__ uint32_t qsh[8];   // per wave: wanting slots -> offsets; next item, regenerated, queue base
    if (lane == 0) qsh[wave] = (uint32_t)__popcll(bW);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0u;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { const uint32_t v = qsh[w]; qsh[w] = t; t += v; }
        const uint32_t nb = t ? atomicAdd(&P.cnt[CNT_NEXT], t) : 0u;
        const uint32_t nReg = nb >= src.nItems ? 0u : min(t, src.nItems - nb);
        qsh[4] = nb; qsh[5] = nReg; qsh[6] = nReg ? atomicAdd(&P.cnt[CNT_QC(qout)], nReg) : 0u;
    }
    __syncthreads();
    if (want) {
        const uint32_t r = qsh[wave] + (uint32_t)__popcll(bW & ((1ull << lane) - 1ull));   // block order
        if (r < qsh[5]) {
            path_start<NB>(S, P, src, slot, qsh[4] + r);
            P.qC[(size_t)qout * 2 * P.rcap + qsh[6] + r] = (uint32_t)slot << 1;
        }
    }
}
template <int NB, int FEAT>
hipError_t launch_dl_nee(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, int qout) {
    const size_t lds = ((FEAT & FEAT_MEAS) && S.kdInLds) ? (size_t)S.nKd * 32 : 0;
    hipLaunchKernelGGL((k_dl_nee<NB, FEAT>), dim3(grid), dim3(kShadeBlock), lds, stream, S, P, qout);
    return hipGetLastError();
}
#if SHADE_FEAT == FEAT_ALL   // one k_regen per band count
template <int NB>
hipError_t launch_regen(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout) {
    hipLaunchKernelGGL((k_regen<NB>), dim3(grid), dim3(kShadeBlock), 0, stream, S, P, src, qout);
    return hipGetLastError();
}
template hipError_t launch_regen<SHADE_NB>(int, hipStream_t, const DevScene &, const PathSoA &, const ItemSrc &, int);
#endif
template <int NB, int FEAT>
hipError_t launch_dl_spec(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                          float *Lout) {
    const size_t lds = ((FEAT & FEAT_MEAS) && S.kdInLds) ? (size_t)S.nKd * 32 : 0;
    hipLaunchKernelGGL((k_dl_spec<NB, FEAT>), dim3(grid), dim3(kShadeBlock), lds, stream, S, P, qout, Lout);
    if (hipError_t e = hipGetLastError()) return e;
    return launch_regen<NB>(grid, stream, S, P, src, qout);
}
template hipError_t launch_dl_nee<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &, int);
template hipError_t launch_dl_spec<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &,
                                                         const ItemSrc &, int, float *);
template <int NB, int FEAT>
hipError_t launch_shade_dl(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src,
                           int qout, float *Lout) {
    return launch<NB, FEAT, MODE_DL>(grid, stream, S, P, src, qout, Lout);
}
template <int NB, int FEAT>
hipError_t launch_shade_meta(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src,
                             int qout, float *Lout) {
    return launch<NB, FEAT, MODE_META>(grid, stream, S, P, src, qout, Lout);
}
template hipError_t launch_shade_dl<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &,
                                                          const ItemSrc &, int, float *);
template hipError_t launch_shade_meta<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &,
                                                            const ItemSrc &, int, float *);
#else
template <int NB, int FEAT>
hipError_t launch_shade(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                        float *Lout) {
#ifdef PGD_EXP_NB_HALF   // timing experiment only: a 32-band scene shaded by the 16-band kernel (wrong radiance)
    if constexpr (NB == 32) return launch<16, FEAT, MODE_PATH>(grid, stream, S, P, src, qout, Lout);
#endif
    return launch<NB, FEAT, MODE_PATH>(grid, stream, S, P, src, qout, Lout);
}
template hipError_t launch_shade<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &,
                                                       const ItemSrc &, int, float *);
#endif

#if !SHADE_DL
// The drain's tail (path integrator, scenes without instances).  Once a lane's items are all taken
// and the drain's list passes have left few live paths, each pass still costs its launches and a
// host read-back for a few thousand rays, and the last passes of a small render (one GPU's tile
// slice at 8 GPUs) are mostly that.  k_tail runs every live slot's path to its end in one launch,
// one thread per slot of the live list (k_live_list): the slot's pending queries of the last
// shading step -- continuation ray, MIS ray, shadow ray -- answered by the per-thread walks of the
// 4-wide BVH copy (bvh_intersect4 / bvh_intersectP4: the primitives and order k_trace_c4 / k_trace_s4
// test, replayed against the oracle on the host), then shade_slot as the next list-mode pass would
// run it, then the MT window where k_mt_init would compute it; until the path is done.
// Exact: a slot's pass-to-pass state is its own in list mode (every writer stores at the identity
// entry and sets its region's writer masks to all ones, wavefront.h PathSoA::listMode); the host
// starts k_tail only after three list-mode passes, so every entry a slot still reads (beta up to
// two passes back, A / B one) was written that way; each thread then advances its own pass index
// and queue set as the host would per pass.  Nothing is queued: the queues of the next set are
// left empty, and the lane reads as drained.
template <int NB, int FEAT>
__global__ __launch_bounds__(kTailBlock) void k_tail(DevScene S, PathSoA P0, int q0, float *__restrict__ Lout, int maxSteps) {
    PathSoA P = P0;
    P.listMode = 1;
    if (FEAT & FEAT_MEAS) kd_lds_fill(S);   // the measured-BRDF kd-trees, once per block (before any return)
    // the traversal stack after the kd-trees in the dynamic LDS: refs, then entry distances
    const int depth = (S.stackDepth > S.w4Stack ? S.stackDepth : S.w4Stack) + 1;
    uint32_t *stk = reinterpret_cast<uint32_t *>(pgd_kd_lds + (((FEAT & FEAT_MEAS) && S.kdInLds) ? 2 * S.nKd : 0));
    Stack st;
    st.base = stk + threadIdx.x;
    st.tbase = reinterpret_cast<float *>(stk + (size_t)depth * blockDim.x) + threadIdx.x;
    st.stride = blockDim.x;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    // a live list longer than the grid would leave paths unfinished (read as drained): CNT_ERR bit 2
    if (i == 0 && P.cnt[CNT_LIVE] > gridDim.x * blockDim.x) atomicOr(&P.cnt[CNT_ERR], 4u);
    if (i >= P.cnt[CNT_LIVE]) return;
    const int slot = (int)P.live[i];
    const uint32_t rc = (uint32_t)P.rcap;
    int qout = q0;
    for (int step = 0; step < maxSteps && P.item[slot] >= 0; ++step) {
        const uint32_t fl = P.flags[slot];
        if (fl & PF_CONT) {   // the continuation ray (list mode: every record at the slot)
            Ray r = ray_load(P, RAY_C, slot);
            int prim = -1;
            float t = INFINITY;
            if (!bvh_intersect4(S, st, r, &prim, &t)) prim = -1;
            P.hitPrim[slot] = prim;
            P.hitT[slot] = prim >= 0 ? t : INFINITY;
        }
        if (fl & PF_PB) {   // the MIS ray
            Ray r = ray_load(P, mis_kind(qout), slot);   // the set the last step wrote
            int prim = -1;
            float t = INFINITY;
            if (!bvh_intersect4(S, st, r, &prim, &t)) prim = -1;
            P.hitPrim[rc + (uint32_t)slot] = prim;
            P.hitT[rc + (uint32_t)slot] = prim >= 0 ? t : INFINITY;
        }
        if (fl & PF_PA) P.occ[slot] = bvh_intersectP4(S, st, ray_load(P, RAY_S, slot)) ? 1u : 0u;
        P.pass = (P.pass + 1) % 3;   // the next pass: beta buffers rotate, A / B take the other queue set
        qout ^= 1;
        bool done = false, zeroed = false;
        const Pushes pu = shade_slot<NB, FEAT>(S, P, slot, Lout, &done, &zeroed, qout);
        if (zeroed) atomicAdd(&P.cnt[CNT_ZEROED], 1u);
        if (done) P.item[slot] = -1;
        else if (pu.t) mt_window_init(P, (uint32_t)slot);   // vertex 3 draws first (k_mt_init's list)
    }
    // still live after maxSteps (a path lives at most maxdepth + 3 passes): its radiance would be
    // lost with nothing queued -- CNT_ERR bit 3, which the host turns into PBRTGPU_E_STATE
    if (P.item[slot] >= 0) atomicOr(&P.cnt[CNT_ERR], 8u);
}
template <int NB, int FEAT>
hipError_t launch_tail(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, int q, float *Lout,
                       int maxSteps) {
    const size_t kd = ((FEAT & FEAT_MEAS) && S.kdInLds) ? (size_t)S.nKd * 32 : 0;
    const int depth = (S.stackDepth > S.w4Stack ? S.stackDepth : S.w4Stack) + 1;
    const size_t lds = kd + (size_t)depth * kTailBlock * 8;
    hipLaunchKernelGGL((k_tail<NB, FEAT>), dim3(grid), dim3(kTailBlock), lds, stream, S, P, q, Lout, maxSteps);
    return hipGetLastError();
}
template hipError_t launch_tail<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &, int, float *, int);
#endif

}  // namespace pgd
