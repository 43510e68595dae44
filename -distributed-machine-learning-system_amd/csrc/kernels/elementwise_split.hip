// Memory-bound kernels of the split-fp16 (fp32-accurate) path.
//
// Split layout (common.h split_off): a pixel of C channels is 2C halfs,
// [hi x32][lo x32] per 32-channel block, value = hi + lo, hi = fp16(v),
// lo = fp16(v - hi).  These kernels convert between fp32 NHWC and that layout
// and max-pool in it; every value goes through f32 and is re-split, so a
// round trip f32 -> split -> f32 is exact to 22 bits.
//   * split_from_f32   NHWC f32 [.., C]  -> split [.., 2C]
//   * f32_from_split   split [.., 2C]    -> NHWC f32 [.., C]
//   * maxpool_split    NHWC max pool, input f32 or split, output split
//                      (ResNet: the fp32 stem's output pooled straight into
//                      the split layer1 input)
#include "../kernels.h"

namespace idunno {

__device__ __forceinline__ float4v load_split4(const half_t* p) {
  const half4v h = *reinterpret_cast<const half4v*>(p);
  const half4v l = *reinterpret_cast<const half4v*>(p + 32);
  return float4v{(float)h[0] + (float)l[0], (float)h[1] + (float)l[1], (float)h[2] + (float)l[2],
                 (float)h[3] + (float)l[3]};
}

__device__ __forceinline__ void store_split4(half_t* p, const float4v v, int* ovf = nullptr) {
  split_guard(ovf, v);
  half4v h, l;
  split_f16x4(v, h, l);
  *reinterpret_cast<half4v*>(p) = h;
  *reinterpret_cast<half4v*>(p + 32) = l;
}

// one thread = 4 channels of one pixel
__global__ void split_from_f32_kernel(const float* __restrict__ x, half_t* __restrict__ y, long npix, int C,
                                      int* ovf) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = C / 4;
  if (t >= npix * cv) return;
  const long pix = t / cv;
  const int c = (int)(t - pix * cv) * 4;
  store_split4(y + pix * 2 * C + split_off(c), *reinterpret_cast<const float4v*>(x + pix * C + c), ovf);
}

__global__ void f32_from_split_kernel(const half_t* __restrict__ x, float* __restrict__ y, long npix, int C) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = C / 4;
  if (t >= npix * cv) return;
  const long pix = t / cv;
  const int c = (int)(t - pix * cv) * 4;
  *reinterpret_cast<float4v*>(y + pix * C + c) = load_split4(x + pix * 2 * C + split_off(c));
}

void split_from_f32_launch(const float* x, half_t* y, long npix, int C, int* ovf, hipStream_t st) {
  const long total = npix * (C / 4);
  hipLaunchKernelGGL(split_from_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, y, npix, C,
                     ovf);
}

void f32_from_split_launch(const half_t* x, float* y, long npix, int C, hipStream_t st) {
  const long total = npix * (C / 4);
  hipLaunchKernelGGL(f32_from_split_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x, y, npix, C);
}

// NHWC max pool -> split output; IN_SPLIT: input in the split layout too.
// Consecutive threads take consecutive 4-channel groups of one output pixel,
// so a wave reads whole 256-byte (f32) pixel rows.
template <bool IN_SPLIT>
__global__ void maxpool_split_kernel(const void* __restrict__ xv, half_t* __restrict__ y, int B, int H, int W,
                                     int C, int Ho, int Wo, int k, int s, int pad, int* ovf) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = C / 4;
  const long total = (long)B * Ho * Wo * cv;
  if (t >= total) return;
  const int c = (int)(t % cv) * 4;
  long pix = t / cv;
  const long opix = pix;
  const int ow = (int)(pix % Wo);
  pix /= Wo;
  const int oh = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  float4v m = float4v{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  const int ih0 = oh * s - pad, iw0 = ow * s - pad;
  for (int dy = 0; dy < k; ++dy) {
    const int ih = ih0 + dy;
    if ((unsigned)ih >= (unsigned)H) continue;
    for (int dx = 0; dx < k; ++dx) {
      const int iw = iw0 + dx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const size_t ip = ((size_t)b * H + ih) * W + iw;
      float4v v;
      if constexpr (IN_SPLIT)
        v = load_split4(static_cast<const half_t*>(xv) + ip * 2 * C + split_off(c));
      else
        v = *reinterpret_cast<const float4v*>(static_cast<const float*>(xv) + ip * C + c);
      m[0] = fmaxf(m[0], v[0]);
      m[1] = fmaxf(m[1], v[1]);
      m[2] = fmaxf(m[2], v[2]);
      m[3] = fmaxf(m[3], v[3]);
    }
  }
  // (a split input is already in range: only an fp32 input can leave it)
  store_split4(y + (size_t)opix * 2 * C + split_off(c), m, IN_SPLIT ? nullptr : ovf);
}

void maxpool_split_launch(const void* x, bool in_split, half_t* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                          int s, int pad, int* ovf, hipStream_t st) {
  const long total = (long)B * Ho * Wo * (C / 4);
  const dim3 grid((unsigned)((total + 255) / 256));
  if (in_split)
    hipLaunchKernelGGL(maxpool_split_kernel<true>, grid, dim3(256), 0, st, x, y, B, H, W, C, Ho, Wo, k, s, pad, ovf);
  else
    hipLaunchKernelGGL(maxpool_split_kernel<false>, grid, dim3(256), 0, st, x, y, B, H, W, C, Ho, Wo, k, s, pad, ovf);
}

}  // namespace idunno
