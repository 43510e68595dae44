// Shared device-side types and helpers for the IDunno-MI355X HIP kernels.
//
// Everything here targets gfx950 (CDNA4) only: 64-lane wavefronts, MFMA
// f32_16x16x32_f16 matrix cores, 160 KiB LDS per CU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tile_math.h"

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


// ---- LDS reads the compiler does not see ------------------------------------------
// While a global_load_lds (LDS-DMA) is in flight, hipcc's wait-count pass puts
// an `s_waitcnt vmcnt(0)` in front of the next ds_read it emits (it cannot tell
// that the read does not touch the DMA's destination), draining the prefetch
// the kernel just issued.  Fragment reads issued from inline asm are invisible
// to that pass; the kernel then orders them itself: a counted
// `s_waitcnt lgkmcnt(N)` (lds_waitcnt) followed by lds_tie() of every fragment
// register it covers (volatile asm keeps its order, and each MFMA consumes the
// tied value, so none can be scheduled above the wait).
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ half8v lds_read_b128(uint32_t addr) {
  half8v v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// 16-byte-per-lane LDS-DMA through a buffer resource (buffer_load_dwordx4 ... lds):
// voff per lane, soff uniform; lanes past num_records land zeros.  A plain
// __device__ wrapper: called straight from a __global__ template's body, the
// target builtin made the host pass drop the kernel's launch stub without a
// diagnostic (every conv_glds instantiation became an undefined symbol).
__device__ __forceinline__ void dma_buf16(__amdgpu_buffer_rsrc_t rsrc, void* lds, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// 4-byte-per-lane LDS-DMA: an L2 prefetch whose data lands in a scratch LDS slot
__device__ __forceinline__ void dma_buf4(__amdgpu_buffer_rsrc_t rsrc, void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}

// ds_read_b128 at addr + OFF (OFF an immediate, < 64 KiB)
template <int OFF>
__device__ __forceinline__ half8v lds_read_b128_imm(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  half8v v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

// ds_read_b128 at addr + i * STEP for a compile-time-after-unrolling i < 16
template <int STEP>
__device__ __forceinline__ half8v lds_read_b128_step(uint32_t addr, int i) {
  switch (i) {
    case 0: return lds_read_b128_imm<0>(addr);
    case 1: return lds_read_b128_imm<STEP>(addr);
    case 2: return lds_read_b128_imm<2 * STEP>(addr);
    case 3: return lds_read_b128_imm<3 * STEP>(addr);
    case 4: return lds_read_b128_imm<4 * STEP>(addr);
    case 5: return lds_read_b128_imm<5 * STEP>(addr);
    case 6: return lds_read_b128_imm<6 * STEP>(addr);
    default: return lds_read_b128_imm<7 * STEP>(addr);
  }
}

template <int N>
__device__ __forceinline__ void lds_waitcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_tie(half8v& r) { asm volatile("" : "+v"(r)); }

// fp32 flavour (conv_f32.hip): 4 consecutive f32 of one LDS row per lane
__device__ __forceinline__ float4v lds_read_f4(uint32_t addr) {
  float4v v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

__device__ __forceinline__ void lds_tie(float4v& r) { asm volatile("" : "+v"(r)); }

// 8-byte global load the wait-count pass does not track (same reason as above:
// a tracked load beside an LDS-DMA prefetch gets a vmcnt(0) at its first use).
// The caller retires it with an explicit counted `s_waitcnt vmcnt(N)`.
__device__ __forceinline__ half4v gload_b64_untracked(const void* p) {
  half4v v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// 16-byte global load the wait-count pass does not track (see gload_b64_untracked).
__device__ __forceinline__ float4v gload_f4_untracked(const void* p) {
  float4v v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// ---- split fp16 (fp32-accurate) activations ------------------------------------
// A value v is two halfs hi = fp16(v), lo = fp16(v - hi); a pixel of C channels
// is 2C halfs, [hi x32][lo x32] per 32-channel block.  split_off(c) = offset of
// channel c's hi half within its pixel (lo at +32).
__device__ __forceinline__ int split_off(int c) { return ((c >> 5) << 6) + (c & 31); }

__device__ __forceinline__ void split_f16x4(const float4v v, half4v& h, half4v& l) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = (half_t)v[i];
    l[i] = (half_t)(v[i] - (float)h[i]);
  }
}

// Split range guard: a value with |v| >= 65504 has no
// finite hi half, so a split epilogue that meets one flags the forward.  The
// flag is an int in device memory owned by the runner (nullptr: unguarded);
// every lane that sees an out-of-range value stores 1 with a plain vector
// store (racing writers store the same value).  softmax_top1 then marks the
// batch, and the host reruns it on the all-f32 path, which has fp32's range.
__device__ __forceinline__ void split_guard(int* ovf, const float4v v) {
  constexpr float kMax = 65504.f;
  if (ovf != nullptr && !(fabsf(v[0]) < kMax && fabsf(v[1]) < kMax && fabsf(v[2]) < kMax && fabsf(v[3]) < kMax))
    *ovf = 1;
}

__device__ __forceinline__ void reg_tie(half4v& r) { asm volatile("" : "+v"(r)); }
__device__ __forceinline__ void reg_tie(float4v& r) { asm volatile("" : "+v"(r)); }

// ---- 16-byte split epilogue accesses (cdna_hip_programming T21) ------------------
// In the 16x16 C/D layout lane group q = lane >> 4 holds output channels
// nb + 4q .. nb + 4q + 3 of one pixel, as hi and lo half4s: two 8-byte accesses
// per lane.  One v_permlane16_swap per dword (rows 1/3 of the hi register trade
// with rows 0/2 of the lo register) leaves q even with the hi halfs of channels
// nb + 8(q/2) .. +7 and q odd with their lo halfs: ONE 16-byte access per lane at
// split_off_q(nb, q).  The inverse (split_swap_in) is the same swap.
typedef unsigned int u32x2_sw __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_sw __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int split_off_q(int nb, int q) { return split_off(nb + 8 * (q >> 1)) + 32 * (q & 1); }

__device__ __forceinline__ u32x4_sw split_swap_out(half4v h, half4v l) {
  const u32x2_sw hv = __builtin_bit_cast(u32x2_sw, h), lv = __builtin_bit_cast(u32x2_sw, l);
  const auto s0 = __builtin_amdgcn_permlane16_swap(hv[0], lv[0], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(hv[1], lv[1], false, false);
  return u32x4_sw{s0[0], s1[0], s0[1], s1[1]};
}

// fp16 outputs of two 16-channel fragments (lane group q: channels nb + 4q .. +3
// and nb + 16 + 4q .. +3): the same swap leaves lane q with 8 consecutive
// channels at f16_pair_off(nb, q) -> one 16-byte store per lane and pair.
__device__ __forceinline__ int f16_pair_off(int nb, int q) { return nb + 16 * (q & 1) + 8 * (q >> 1); }

__device__ __forceinline__ void split_swap_in(float4v r, half4v& h, half4v& l) {
  const u32x4_sw v = __builtin_bit_cast(u32x4_sw, r);
  const auto s0 = __builtin_amdgcn_permlane16_swap(v[0], v[2], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(v[1], v[3], false, false);
  h = __builtin_bit_cast(half4v, u32x2_sw{s0[0], s1[0]});
  l = __builtin_bit_cast(half4v, u32x2_sw{s0[1], s1[1]});
}

}  // namespace idunno
