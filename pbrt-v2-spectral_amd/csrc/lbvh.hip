// lbvh.hip -- BVH construction on the GPU (the host front end's setup
// cost).  The reference builds its BVH on one CPU thread with the SAH splitter
// (accelerators/bvh.cpp:145-351); pbrthost restates that build node for node, because the
// reference traversal order (bvh.cpp:380-481) is what the bit-exact parity of §3 rests on.
// This file is the opt-in fast build: a linear BVH (Karras, "Maximizing parallelism in the
// construction of BVHs, octrees, and k-d trees", HPG 2012) over the primitives' world bounds,
//
//   k_morton   30-bit Morton code of each primitive's bound centroid in the centroid box
//   (sort)     hipcub radix sort of (code, primitive index) pairs -- stable, so primitives
//              with equal codes stay in index order and the build is deterministic
//   k_karras   one thread per interior node: its key range and split (radix tree)
//   k_refit    leaves upward, the second thread to reach a node forms its bound (min/max
//              only, so the bounds are exact whatever the arrival order) and leaf count
//   k_flatten  depth-first position of every node (a walk to the root summing left-sibling
//              subtree sizes), then the node in the reference's LinearBVHNode layout
//              (bvh.cpp:105-115): first child = next node, offset = second child or the
//              leaf's primitive position; one primitive per leaf; axis = largest extent
//
// A ray's closest hit is the same primitive at the same t under any BVH except for exact
// ties in t (the traversal visits them in another order), so a render over this BVH equals
// the reference's up to those ties (tests/test_lbvh.py measures it).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <chrono>
#include <string>
#include <vector>
#include "pbrtgpu.h"

namespace pgd {

static const int kLbvhBlock = 256;

// spread the low 10 bits of v to every third bit
__device__ __forceinline__ uint32_t morton_spread(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_morton(int n, const float *__restrict__ bounds, float3 lo, float3 scale, uint32_t *__restrict__ codes,
                         uint32_t *__restrict__ idx) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float *b = bounds + 6 * (size_t)i;
    const float c[3] = {.5f * b[0] + .5f * b[3], .5f * b[1] + .5f * b[4], .5f * b[2] + .5f * b[5]};
    const float l[3] = {lo.x, lo.y, lo.z}, s[3] = {scale.x, scale.y, scale.z};
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
        const float u = (c[k] - l[k]) * s[k];   // [0, 1024)
        q[k] = (uint32_t)fminf(fmaxf(u, 0.f), 1023.f);
    }
    codes[i] = (morton_spread(q[0]) << 2) | (morton_spread(q[1]) << 1) | morton_spread(q[2]);
    idx[i] = (uint32_t)i;
}

// common prefix length of sorted keys i and j (index bits break ties); -1 outside [0, n)
__device__ __forceinline__ int lb_delta(const uint32_t *__restrict__ codes, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = codes[i], b = codes[j];
    return a == b ? 32 + __clz((uint32_t)i ^ (uint32_t)j) : __clz(a ^ b);
}

// interior nodes 0 .. n-2, leaves n-1 .. 2n-2 (leaf k = sorted primitive k); root = node 0
__global__ void k_karras(int n, const uint32_t *__restrict__ codes, int2 *__restrict__ child, int *__restrict__ parent) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = lb_delta(codes, n, i, i + 1) - lb_delta(codes, n, i, i - 1) >= 0 ? 1 : -1;
    const int dmin = lb_delta(codes, n, i, i - d);
    int lmax = 2;
    while (lb_delta(codes, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (lb_delta(codes, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = lb_delta(codes, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (lb_delta(codes, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + (d < 0 ? -1 : 0);
    const int lft = min(i, j) == gamma ? (n - 1) + gamma : gamma;
    const int rgt = max(i, j) == gamma + 1 ? (n - 1) + gamma + 1 : gamma + 1;
    child[i] = make_int2(lft, rgt);
    parent[lft] = i;
    parent[rgt] = i;
}

template <class T> __device__ __forceinline__ T ld_dev(const T *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_refit(int n, const float *__restrict__ bounds, const uint32_t *__restrict__ idx,
                        const int2 *__restrict__ child, const int *__restrict__ parent, float *__restrict__ nb,
                        int *__restrict__ leaves, uint32_t *__restrict__ arrivals) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int x = (n - 1) + k;
    const float *b = bounds + 6 * (size_t)idx[k];
    for (int c = 0; c < 6; ++c) nb[6 * (size_t)x + c] = b[c];
    leaves[x] = 1;
    while (x != 0) {
        const int p = parent[x];
        __threadfence();
        if (atomicAdd(&arrivals[p], 1u) == 0u) return;   // the sibling's thread forms p
        __threadfence();
        const int2 ch = child[p];
        // the children were written by other threads: device-scope loads (past this CU's L1)
        const float *a = nb + 6 * (size_t)ch.x, *bb = nb + 6 * (size_t)ch.y;
        for (int c = 0; c < 3; ++c) {
            nb[6 * (size_t)p + c] = fminf(ld_dev(a + c), ld_dev(bb + c));
            nb[6 * (size_t)p + 3 + c] = fmaxf(ld_dev(a + 3 + c), ld_dev(bb + 3 + c));
        }
        leaves[p] = ld_dev(leaves + ch.x) + ld_dev(leaves + ch.y);
        x = p;
    }
}

__global__ void k_dfs(int n, const int2 *__restrict__ child, const int *__restrict__ parent, const int *__restrict__ leaves,
                      int *__restrict__ dfs) {
    const int x0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (x0 >= 2 * n - 1) return;
    int pos = 0, x = x0;
    while (x != 0) {
        const int p = parent[x];
        const int2 ch = child[p];
        pos += ch.x == x ? 1 : 1 + (2 * leaves[ch.x] - 1);
        x = p;
    }
    dfs[x0] = pos;
}

__global__ void k_flatten(int n, const int2 *__restrict__ child, const int *__restrict__ dfs, const float *__restrict__ nb,
                          pbrtgpu_bvh_node *__restrict__ out) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= 2 * n - 1) return;
    pbrtgpu_bvh_node o;
    const float *b = nb + 6 * (size_t)x;
    int axis = 0;
    float ext = -1.f;
    for (int c = 0; c < 3; ++c) {
        o.bmin[c] = b[c];
        o.bmax[c] = b[3 + c];
        if (b[3 + c] - b[c] > ext) { ext = b[3 + c] - b[c]; axis = c; }
    }
    if (x >= n - 1) {   // leaf: one primitive, at its sorted position
        o.offset = (uint32_t)(x - (n - 1));
        o.meta = 1u | ((uint32_t)axis << 8);
    } else {
        o.offset = (uint32_t)dfs[child[x].y];
        o.meta = (uint32_t)axis << 8;
    }
    out[dfs[x]] = o;
}

#define LBCHK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { *err = std::string(#x) + ": " + hipGetErrorString(e_); rc = -(1000 + (int)e_); goto done; } \
    } while (0)

// the build on `stream`; nodes_out [2n-1], order_out [n] (host); ms_out [2]: device time of the
// build kernels and sort (HIP events), wall time of the call including the copies
int lbvh_build(hipStream_t stream, int n, const float *bounds, pbrtgpu_bvh_node *nodes_out, int32_t *order_out,
               double *ms_out, std::string *err) {
    const auto w0 = std::chrono::steady_clock::now();
    int rc = 0;
    const int nn = 2 * n - 1;
    // centroid box (host: the bounds are host data anyway), scaled to the 10-bit grid
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n; ++i)
        for (int c = 0; c < 3; ++c) {
            const float v = .5f * bounds[6 * (size_t)i + c] + .5f * bounds[6 * (size_t)i + 3 + c];
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
        }
    float sc[3];
    for (int c = 0; c < 3; ++c) sc[c] = hi[c] > lo[c] ? 1024.f / (hi[c] - lo[c]) * (1.f - 1e-6f) : 0.f;
    float *dB = nullptr, *dNb = nullptr;
    uint32_t *dCode = nullptr, *dIdx = nullptr, *dCode2 = nullptr, *dIdx2 = nullptr, *dArr = nullptr;
    int2 *dChild = nullptr;
    int *dParent = nullptr, *dLeaves = nullptr, *dDfs = nullptr;
    pbrtgpu_bvh_node *dOut = nullptr;
    void *dTmp = nullptr;
    size_t tmpBytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int g1 = (n + kLbvhBlock - 1) / kLbvhBlock, g2 = (nn + kLbvhBlock - 1) / kLbvhBlock;
    LBCHK(hipEventCreate(&e0));
    LBCHK(hipEventCreate(&e1));
    LBCHK(hipMalloc(&dB, sizeof(float) * 6 * (size_t)n));
    LBCHK(hipMalloc(&dNb, sizeof(float) * 6 * (size_t)nn));
    LBCHK(hipMalloc(&dCode, 4 * (size_t)n));
    LBCHK(hipMalloc(&dIdx, 4 * (size_t)n));
    LBCHK(hipMalloc(&dCode2, 4 * (size_t)n));
    LBCHK(hipMalloc(&dIdx2, 4 * (size_t)n));
    LBCHK(hipMalloc(&dArr, 4 * (size_t)nn));
    LBCHK(hipMalloc(&dChild, sizeof(int2) * (size_t)n));
    LBCHK(hipMalloc(&dParent, 4 * (size_t)nn));
    LBCHK(hipMalloc(&dLeaves, 4 * (size_t)nn));
    LBCHK(hipMalloc(&dDfs, 4 * (size_t)nn));
    LBCHK(hipMalloc(&dOut, sizeof(pbrtgpu_bvh_node) * (size_t)nn));
    LBCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmpBytes, dCode, dCode2, dIdx, dIdx2, n, 0, 30, stream));
    LBCHK(hipMalloc(&dTmp, std::max<size_t>(tmpBytes, 16)));
    LBCHK(hipMemcpyAsync(dB, bounds, sizeof(float) * 6 * (size_t)n, hipMemcpyHostToDevice, stream));
    LBCHK(hipMemsetAsync(dArr, 0, 4 * (size_t)nn, stream));
    LBCHK(hipMemsetAsync(dParent, 0xff, 4 * (size_t)nn, stream));
    LBCHK(hipEventRecord(e0, stream));
    hipLaunchKernelGGL(k_morton, dim3(g1), dim3(kLbvhBlock), 0, stream, n, dB, make_float3(lo[0], lo[1], lo[2]),
                       make_float3(sc[0], sc[1], sc[2]), dCode, dIdx);
    LBCHK(hipGetLastError());
    LBCHK(hipcub::DeviceRadixSort::SortPairs(dTmp, tmpBytes, dCode, dCode2, dIdx, dIdx2, n, 0, 30, stream));
    if (n > 1) {
        hipLaunchKernelGGL(k_karras, dim3((n - 1 + kLbvhBlock - 1) / kLbvhBlock), dim3(kLbvhBlock), 0, stream, n, dCode2,
                           dChild, dParent);
        LBCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(k_refit, dim3(g1), dim3(kLbvhBlock), 0, stream, n, dB, dIdx2, dChild, dParent, dNb, dLeaves, dArr);
    LBCHK(hipGetLastError());
    hipLaunchKernelGGL(k_dfs, dim3(g2), dim3(kLbvhBlock), 0, stream, n, dChild, dParent, dLeaves, dDfs);
    LBCHK(hipGetLastError());
    hipLaunchKernelGGL(k_flatten, dim3(g2), dim3(kLbvhBlock), 0, stream, n, dChild, dDfs, dNb, dOut);
    LBCHK(hipGetLastError());
    LBCHK(hipEventRecord(e1, stream));
    LBCHK(hipMemcpyAsync(nodes_out, dOut, sizeof(pbrtgpu_bvh_node) * (size_t)nn, hipMemcpyDeviceToHost, stream));
    LBCHK(hipMemcpyAsync(order_out, dIdx2, 4 * (size_t)n, hipMemcpyDeviceToHost, stream));
    LBCHK(hipStreamSynchronize(stream));
    if (ms_out) {
        float m = 0.f;
        LBCHK(hipEventElapsedTime(&m, e0, e1));
        ms_out[0] = m;
        ms_out[1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
    }
done:
    for (void *p : {(void *)dB, (void *)dNb, (void *)dCode, (void *)dIdx, (void *)dCode2, (void *)dIdx2, (void *)dArr,
                    (void *)dChild, (void *)dParent, (void *)dLeaves, (void *)dDfs, (void *)dOut, dTmp})
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return rc;
}

}  // namespace pgd
