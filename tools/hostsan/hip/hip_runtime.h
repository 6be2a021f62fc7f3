// Host stand-in for <hip/hip_runtime.h> -- TEST INFRASTRUCTURE ONLY, never part of the product.
//
// tools/hostsan/shade_host.cpp compiles the device shading code (csrc/device.h, wavefront.h,
// directlighting.h, metadata.h, scene_build.h) as plain host C++ so that it can run under the
// host sanitizers (ASan, UBSan, MSan) and be compared with the oracle on the CPU.  This header
// is first on that build's include path; it supplies the few HIP names those headers use:
//   * qualifiers (__device__, __shared__, ...) as nothing;
//   * HIP's vector types as plain structs;
//   * wave intrinsics for a wave of ONE active lane: the replay runs each path slot as lane 0
//     of its own 64-slot wave (slot = 64 i), so a ballot is the lane's own predicate and every
//     per-wave rank is 0 -- the per-wave compaction of wavefront.h reduces to one entry per wave.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define __device__
#define __host__
#define __global__
#define __shared__
#define __constant__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define PGD_LDS_AS   // LDS address space qualifier of wavefront.h: ordinary memory here
#define PGD_GLOBAL_AS   // global address space qualifier of wavefront.h (kd lookup): ordinary memory here

typedef int hipError_t;
typedef void *hipStream_t;
enum { hipSuccess = 0 };

struct float2 { float x, y; };
struct float4 { float x, y, z, w; };
struct int2 { int x, y; };
struct int3 { int x, y, z; };
struct int4 { int x, y, z, w; };
struct uint2 { unsigned x, y; };
struct uint4 { unsigned x, y, z, w; };
inline uint4 make_uint4(unsigned x, unsigned y, unsigned z, unsigned w) { return uint4{x, y, z, w}; }
inline float2 make_float2(float x, float y) { return float2{x, y}; }
inline float4 make_float4(float x, float y, float z, float w) { return float4{x, y, z, w}; }
inline int2 make_int2(int x, int y) { return int2{x, y}; }
inline int3 make_int3(int x, int y, int z) { return int3{x, y, z}; }
inline int4 make_int4(int x, int y, int z, int w) { return int4{x, y, z, w}; }

struct pgd_host_dim3 { unsigned x, y, z; };
inline thread_local pgd_host_dim3 threadIdx = {0u, 0u, 0u};
inline thread_local pgd_host_dim3 blockIdx = {0u, 0u, 0u};
inline thread_local pgd_host_dim3 blockDim = {64u, 1u, 1u};
inline void __syncthreads() {}

inline unsigned long long __ballot(int p) { return p ? 1ull << (threadIdx.x & 63u) : 0ull; }
inline int __popc(unsigned v) { return __builtin_popcount(v); }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline int __ffs(unsigned v) { return __builtin_ffs((int)v); }
inline int __ffs(int v) { return __builtin_ffs(v); }
inline int __ffsll(long long v) { return __builtin_ffsll(v); }
inline int __ffsll(unsigned long long v) { return __builtin_ffsll((long long)v); }
#define __builtin_amdgcn_readfirstlane(x) (x)

inline int __float_as_int(float f) { int i; std::memcpy(&i, &f, 4); return i; }
inline unsigned __float_as_uint(float f) { unsigned i; std::memcpy(&i, &f, 4); return i; }
inline float __int_as_float(int i) { float f; std::memcpy(&f, &i, 4); return f; }
inline float __uint_as_float(unsigned i) { float f; std::memcpy(&f, &i, 4); return f; }
inline float __sinf(float x) { return std::sin(x); }
inline float __cosf(float x) { return std::cos(x); }
inline float __tanf(float x) { return std::tan(x); }
inline float __logf(float x) { return std::log(x); }
inline float __powf(float x, float y) { return std::pow(x, y); }

template <class T> inline T atomicAdd(T *p, T v) { const T o = *p; *p = o + v; return o; }
template <class T> inline T atomicOr(T *p, T v) { const T o = *p; *p = o | v; return o; }

// HIP's global min / max overloads
inline int min(int a, int b) { return a < b ? a : b; }
inline int max(int a, int b) { return a < b ? b : a; }
inline unsigned min(unsigned a, unsigned b) { return a < b ? a : b; }
inline unsigned max(unsigned a, unsigned b) { return a < b ? b : a; }
inline long long min(long long a, long long b) { return a < b ? a : b; }
inline long long max(long long a, long long b) { return a < b ? b : a; }
inline float min(float a, float b) { return std::fmin(a, b); }
inline float max(float a, float b) { return std::fmax(a, b); }
using std::isinf;
using std::isnan;
