// Shared device helpers for the DBA-on-MI355X kernel library (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC with a leading replica/job group dim: [G][N][H][W][C];
//   * bf16 tensors are passed as uint16_t (torch.bfloat16 bit pattern);
//   * every launcher is `extern "C"`, takes raw device pointers + the caller's hipStream_t
//     (torch's current stream, so launches are captured by HIP graphs) and returns the
//     hipError_t of the launch;
//   * per-group "valid rows" (nvalid[g] samples) gate every row reduction, so padded or
//     inactive client replicas cost nothing and never pollute statistics.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DBA_EXPORT extern "C" __attribute__((visibility("default")))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

static constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even float -> bf16 (NaN preserved as quiet NaN)
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t v) { return bf2f(v); }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t from_f<uint16_t>(float v) { return f2bf(v); }

// 8 consecutive elements (16-B bf16 / 32-B fp32 vector access) <-> float[8]
__device__ __forceinline__ void ld8(const uint16_t* __restrict__ p, float (&v)[8]) {
  const uint4 u = *(const uint4*)p;
  const uint16_t* q = (const uint16_t*)&u;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(q[e]);
}
__device__ __forceinline__ void ld8(const float* __restrict__ p, float (&v)[8]) {
  const float4 a = ((const float4*)p)[0], b = ((const float4*)p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(uint16_t* __restrict__ p, const float (&v)[8]) {
  uint4 u;
  uint16_t* q = (uint16_t*)&u;
#pragma unroll
  for (int e = 0; e < 8; ++e) q[e] = f2bf(v[e]);
  *(uint4*)p = u;
}
__device__ __forceinline__ void st8(float* __restrict__ p, const float (&v)[8]) {
  ((float4*)p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  ((float4*)p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

// lowbias32 — identical to dba_mod_amd/ops/rng.py and csrc/runtime/runtime.cpp
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash2(uint32_t seed, uint32_t ctr) {
  return lowbias32(ctr ^ lowbias32(seed));
}
__device__ __forceinline__ float uniform01(uint32_t seed, uint32_t ctr) {
  return ((float)(hash2(seed, ctr) >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// ---- operand max |x| slots of the fp16-pair split (csrc/kernels/xmfma.hpp HScale)
// A slot holds, per replica g, the max |x| (as non-negative float bits) spread over kAmaxSub
// sub-slots ld ints apart (ld >= 32: one 128-B line each): producers fold block maxima into
// sub-slot blockIdx.x % kAmaxSub with an integer atomicMax (exact, order-independent), so a
// launch's thousands of blocks contend on 16 lines instead of one; consumers take the max of
// the 16.  Slots are zeroed before their producer runs.
constexpr int kAmaxSub = 16;

// every thread of the block must call it (block-level reduction, then one atomic per block)
__device__ __forceinline__ void amax_fold(int* amax, int ld, int g, float m) {
  __shared__ float amax_red[16];   // up to 1024 threads
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) amax_red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (int)(blockDim.x + 63) >> 6;
    float b = amax_red[0];
    for (int w = 1; w < nw; ++w) b = fmaxf(b, amax_red[w]);
    if (b > 0.f) atomicMax(amax + (blockIdx.x % kAmaxSub) * ld + g, __float_as_int(b));
  }
}

// the slot's max for replica g (wave-uniform; every lane of the wave must call it)
__device__ __forceinline__ int amax_read(const int* amax, int ld, int g) {
  const int lane = threadIdx.x & 63;
  int v = lane < kAmaxSub ? amax[lane * ld + g] : 0;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, kWave));
  return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ int valid_rows(const int* nvalid, int g, int n_per_group) {
  return nvalid ? nvalid[g] : n_per_group;
}

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }
static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

#define DBA_LAUNCH_CHECK() return (int)hipGetLastError()
