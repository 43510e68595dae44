// Index math shared by the conv kernels and the host-side checker
// (csrc/tests/host_checks.cpp, built with host ASan + UBSan): block-id remaps and
// the LDS XOR swizzles.  __host__ __device__ so the checker exercises the exact
// functions the kernels inline, not a re-typed mirror.
#pragma once
#include <hip/hip_runtime.h>

namespace idunno {

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming
// §5 "XCD swizzle must be bijective"): consecutive *logical* tiles land on
// the same XCD so neighbouring tiles share that XCD's L2.
__host__ __device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd * 2) return orig;
  const int q = nwg / nxcd, r = nwg % nxcd;
  const int xcd = orig % nxcd, idx = orig / nxcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// conv_glds: 16-byte chunk XOR per LDS row; cpr = chunks per row (8: 128-byte
// rows, BK = 64; 4: 64-byte rows, BK = 32).
__host__ __device__ __forceinline__ int swz_r(int row, int cpr) {
  if (cpr == 8) return (row >> 1) & 7;
  const int q = (row >> 2) & 3;
  return (0x78 >> (2 * q)) & 3;
}

// conv_wino_f32: staged raw-input pixel p (64 bytes = 4 chunks of 4 channels) of
// one column-parity half row; a wave's 16 lanes of one channel group read 16
// consecutive pixels -> 16 distinct bank slots per ds_read_b128 lane group.
__host__ __device__ __forceinline__ int wino_raw_swz(int p) { return ((p >> 2) & 1) << 1; }

// conv3x3_c64: 128-byte rows (64 channels)
__host__ __device__ __forceinline__ int c64_swz(int row) { return row & 6; }

}  // namespace idunno
