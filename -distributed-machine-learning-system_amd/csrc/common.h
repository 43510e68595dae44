// Shared device-side types and helpers for the IDunno-MI355X HIP kernels.
//
// Everything here targets gfx950 (CDNA4) only: 64-lane wavefronts, MFMA
// f32_16x16x32_f16 matrix cores, 160 KiB LDS per CU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace idunno {

typedef _Float16 half_t;
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef _Float16 half4v __attribute__((ext_vector_type(4)));
typedef _Float16 half8v __attribute__((ext_vector_type(8)));
typedef float float4v __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// 16-byte vector used for raw global <-> LDS traffic.
struct alignas(16) vec16 {
  uint32_t x, y, z, w;
};
struct alignas(8) vec8 {
  uint32_t x, y;
};

__device__ __forceinline__ vec16 zero16() { return vec16{0u, 0u, 0u, 0u}; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming
// §5 "XCD swizzle must be bijective"): consecutive *logical* tiles land on
// the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd * 2) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd, idx = orig / nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace idunno
