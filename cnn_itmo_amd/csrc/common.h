// Shared device helpers for the CNN-ITMO HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cnn_itmo.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// Elements per 16-byte vector.
template <typename T> struct Vec16;
template <> struct Vec16<float> { static constexpr int N = 4; };
template <> struct Vec16<bf16> { static constexpr int N = 8; };

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

// 16-byte load/store of T elements as floats.
template <typename T> struct Pack16;
template <> struct Pack16<float> {
  static __device__ __forceinline__ void load(const float* p, float* v) {
    float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Pack16<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    bf16x8 q = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)q[i];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 q;
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = q;
  }
};

// Dropout keep test: splitmix64 finalizer of (seed*G1 + layer*G2 + idx).
// Bit-exact twin of oracle/unet_ref.py:dropout_keep.  Keep probability 0.5.
__device__ __forceinline__ bool dropout_keep(uint64_t base, uint64_t idx) {
  uint64_t x = base + idx;
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (x >> 63) == 0;
}
static inline uint64_t dropout_base(uint64_t seed, uint64_t layer) {
  return seed * 0x9E3779B97F4A7C15ull + layer * 0xD1B54A32D192ED03ull;
}

// Bijective XCD-aware remap of a 1-D block id: blocks that the dispatcher
// deals to the same XCD (b % 8 equal) get a contiguous range of logical ids.
__device__ __forceinline__ int xcd_remap(int b, int total) {
  const int q = total >> 3, r = total & 7;
  const int xcd = b & 7, idx = b >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Host-side error plumbing.
void cnnitmo_set_error(const char* fmt, ...);
int cnnitmo_check_launch(const char* what);

#define CNN_REQUIRE(cond, ...)                \
  do {                                        \
    if (!(cond)) {                            \
      cnnitmo_set_error(__VA_ARGS__);         \
      return CNNITMO_EINVAL;                  \
    }                                         \
  } while (0)
