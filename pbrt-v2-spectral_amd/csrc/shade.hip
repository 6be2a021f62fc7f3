// shade.hip -- the k_shade kernel (one vertex of PathIntegrator::Li per live path slot plus
// path regeneration, wavefront.h) for one band count / feature set.  Compiled once per
// (SHADE_NB, SHADE_FEAT) so the large shading variants build in parallel; pbrtgpu.hip
// launches them through launch_shade<NB, FEAT>.
#include <hip/hip_runtime.h>
#include "pbrtgpu.h"
#include "device.h"
#include "wavefront.h"

#if !defined(SHADE_NB) || !defined(SHADE_FEAT)
#error "compile with -DSHADE_NB=<30|32|60> -DSHADE_FEAT=<0|7>"
#endif

namespace pgd {

// Block-wide exclusive prefix of a per-thread flag with ONE atomicAdd per block on
// *counter; returns this thread's index (valid where flag is set).  All threads of the
// block must call it (it contains barriers).
__device__ __forceinline__ uint32_t block_push(bool flag, uint32_t *counter, uint32_t *lds4) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(flag);
    const uint32_t before = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) lds4[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { uint32_t v = lds4[w]; lds4[w] = tot; tot += v; }
        lds4[15] = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    const uint32_t idx = lds4[15] + lds4[wave] + before;
    __syncthreads();   // lds4 is reused by the next call
    return idx;
}

// shading pass over every slot: finish / advance live paths, regenerate free slots, and
// queue the next pass's rays into queue set qout (block-aggregated queue pushes)
#ifndef PGD_SHADE_ATTR
#define PGD_SHADE_ATTR
#endif
template <int NB, int FEAT>
__global__ __launch_bounds__(kShadeBlock) PGD_SHADE_ATTR void k_shade(DevScene S, PathSoA P, ItemSrc src, int qout,
                                                       float *__restrict__ Lout) {
    __shared__ uint32_t lds4[16];
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    const bool inRange = slot < P.cap;
    Pushes pu = {false, false, false};
    bool freeSlot = inRange && P.item[slot] < 0;
    bool zeroed = false;
    if (inRange && !freeSlot) {
        bool done;
        pu = shade_slot<NB, FEAT>(S, P, slot, Lout, &done, &zeroed);
        if (done) { P.item[slot] = -1; freeSlot = true; }
    }
    if (__ballot(zeroed)) {
        const unsigned long long m = __ballot(zeroed);
        if ((threadIdx.x & 63) == 0) atomicAdd(&P.cnt[CNT_ZEROED], (uint32_t)__popcll(m));
    }
    // regeneration: free slots take the next camera samples
    const bool want = freeSlot && *(volatile uint32_t *)&P.cnt[CNT_NEXT] < src.nItems;
    if (__syncthreads_or(want)) {
        const uint32_t it = block_push(want, &P.cnt[CNT_NEXT], lds4);
        if (want && it < src.nItems) { path_start<NB>(S, P, src, slot, it); pu.c = true; }
    }
    const uint32_t kc = block_push(pu.c, &P.cnt[CNT_QC(qout)], lds4);
    if (pu.c) P.qC[(size_t)qout * 2 * P.cap + kc] = (uint32_t)slot << 1;
    const uint32_t km = block_push(pu.m, &P.cnt[CNT_QC(qout)], lds4);
    if (pu.m) P.qC[(size_t)qout * 2 * P.cap + km] = ((uint32_t)slot << 1) | 1u;
    const uint32_t ks = block_push(pu.s, &P.cnt[CNT_QS(qout)], lds4);
    if (pu.s) P.qS[(size_t)qout * P.cap + ks] = (uint32_t)slot;
}

template <int NB, int FEAT>
hipError_t launch_shade(int grid, hipStream_t stream, const DevScene &S, const PathSoA &P, const ItemSrc &src, int qout,
                        float *Lout) {
    hipLaunchKernelGGL((k_shade<NB, FEAT>), dim3(grid), dim3(kShadeBlock), 0, stream, S, P, src, qout, Lout);
    return hipGetLastError();
}
template hipError_t launch_shade<SHADE_NB, SHADE_FEAT>(int, hipStream_t, const DevScene &, const PathSoA &,
                                                       const ItemSrc &, int, float *);

}  // namespace pgd
