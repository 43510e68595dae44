// fp32 companions of conv_f32.hip (the reference-precision path):
//   * preprocess_f32  uint8 HWC -> normalised fp32 NHWC4 (4th channel 0), the
//                     reference's ToTensor + Normalize (alexnet_resnet.py:57-62)
//   * maxpool_f32     NHWC max pool, 4 channels (16 B) per lane
//   * avgpool_f32     NHWC global average pool -> [B][C] fp32
// The arithmetic is the same as the fp16 kernels in elementwise.hip, kept in f32.
#include "../kernels.h"

namespace idunno {

__constant__ float kMeanF[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStdF[3] = {0.229f, 0.224f, 0.225f};

__device__ __forceinline__ float4v norm_px_f32(uint32_t b0, uint32_t b1, uint32_t b2) {
  // (x/255 - mean)/std with a true division, as torchvision's Normalize
  float4v o;
  o[0] = ((float)b0 / 255.f - kMeanF[0]) / kStdF[0];
  o[1] = ((float)b1 / 255.f - kMeanF[1]) / kStdF[1];
  o[2] = ((float)b2 / 255.f - kMeanF[2]) / kStdF[2];
  o[3] = 0.f;
  return o;
}

// Four pixels per thread: 12 bytes in, 64 bytes (four 16-byte stores) out.
__global__ void preprocess_f32_kernel(const uint8_t* __restrict__ img, float* __restrict__ out, long npix,
                                      const long long* __restrict__ start_idx, long long start_off,
                                      long long max_start, long long sub, long pix_per_img) {
  const long p = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (p >= npix) return;
  if (start_idx != nullptr) {
    long long s0 = *start_idx - start_off;
    s0 = (s0 < 0 ? 0 : (s0 > max_start ? max_start : s0)) + sub;
    img += (size_t)s0 * pix_per_img * 3;
  }
  const uint8_t* s = img + p * 3;
  float4v* d = reinterpret_cast<float4v*>(out + p * 4);
  if (p + 4 <= npix && (reinterpret_cast<uintptr_t>(s) & 3) == 0) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    d[0] = norm_px_f32(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
    d[1] = norm_px_f32(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
    d[2] = norm_px_f32((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
    d[3] = norm_px_f32((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
    return;
  }
  const int n = (int)(npix - p < 4 ? npix - p : 4);
  for (int i = 0; i < n; ++i) d[i] = norm_px_f32(s[3 * i], s[3 * i + 1], s[3 * i + 2]);
}

// Packed-row stem input for conv_f32 mode 2 / conv_glds pack3 (T = float or
// half): out[b][y][c][wp].  Copy c holds the row R shifted left by c*g
// elements (g = E / nc, E = elements per 16-byte chunk: 4 floats / 8 halfs),
// where R[f] = channel f%3 of pixel f/3 - pad, normalised, and zero outside
// the image -- so the 3*KW contiguous elements a stride-s output pixel ox
// reads for one kernel row start 16-byte aligned in copy (3*s*ox mod E) / g,
// and the conv stages them with whole 16-byte DMA chunks (ResNet 7x7/2 fp32:
// K 176 instead of 224 for NHWC4).
// One thread = the 3-chunk group k (3E elements = E pixels) of EVERY copy of
// one row: copy c's group is R[3Ek + c*g ..], all inside the E+2 pixels
// Ek-pad .., loaded once (aligned dwords realigned with v_alignbyte away from
// the row ends) and normalised through an LDS table of the 256 x 3 byte values
// (same arithmetic as preprocess_f32, one division per table entry).
// SPLIT (T = half): split-fp16 stem input [b][y][2][c][wp]: plane 0 = hi =
// fp16(v), plane 1 = lo = fp16(v - hi) of the same copies (conv_glds P3+SPLIT).
template <typename T, int NC, bool SPLIT = false>
__global__ void __launch_bounds__(256) preprocess_pack3_kernel(
    const uint8_t* __restrict__ img, T* __restrict__ out, int B, int H, int W, int pad, int wp,
    const long long* __restrict__ start_idx, long long start_off, long long max_start, long long sub) {
  constexpr int E = 16 / (int)sizeof(T);               // elements per 16-byte chunk
  constexpr int G = E / NC;                            // copy shift (elements)
  constexpr int NPX = E + 2;                           // pixels loaded per group
  constexpr int NV = 3 * NPX;                          // their normalised values
  constexpr int NB = (NV + 3) / 4;                     // realigned dwords of their bytes
  constexpr int ND = NB + 1;                           // aligned dword loads
  __shared__ float lut[3][256];
  const int tid = threadIdx.x;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) lut[ch][tid] = ((float)tid / 255.f - kMeanF[ch]) / kStdF[ch];
  __syncthreads();
  const int ng = (wp + 3 * E - 1) / (3 * E);           // groups per copy row
  const long t = (long)blockIdx.x * blockDim.x + tid;
  const long total = (long)B * H * ng;
  if (t >= total) return;
  if (start_idx != nullptr) {
    long long s0 = *start_idx - start_off;
    s0 = (s0 < 0 ? 0 : (s0 > max_start ? max_start : s0)) + sub;
    img += (size_t)s0 * H * W * 3;
  }
  const int k = (int)(t % ng);
  const long r = t / ng;                               // b * H + y
  const uint8_t* row = img + (size_t)r * W * 3;
  const int px0 = E * k - pad;                         // first of the NPX pixels
  uint32_t bytes[NB];
  if (px0 >= 0 && 3 * px0 + 4 * ND <= 3 * W) {         // the aligned dwords stay inside the row
    const uint8_t* p = row + px0 * 3;
    const uint32_t* a = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    uint32_t d[ND];
#pragma unroll
    for (int i = 0; i < ND; ++i) d[i] = a[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) bytes[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
  } else {
#pragma unroll
    for (int i = 0; i < NB; ++i) bytes[i] = 0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int px = px0 + i / 3;
      if (px >= 0 && px < W) bytes[i >> 2] |= (uint32_t)row[px * 3 + i % 3] << (8 * (i & 3));
    }
  }
  float v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int px = px0 + i / 3;
    v[i] = (px >= 0 && px < W) ? lut[i % 3][(bytes[i >> 2] >> (8 * (i & 3))) & 255u] : 0.f;
  }
  const int nch = min(3, (wp - 3 * E * k) / E);        // chunks of this group inside the row
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if constexpr (SPLIT) {
      T* dst = out + (r * 2 * NC + c) * wp + 3 * E * k;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if (j >= nch) break;
        half8v h, l;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = v[c * G + 8 * j + e];
          h[e] = (half_t)x;
          l[e] = (half_t)(x - (float)h[e]);
        }
        *reinterpret_cast<half8v*>(dst + 8 * j) = h;
        *reinterpret_cast<half8v*>(dst + NC * wp + 8 * j) = l;
      }
      continue;
    }
    T* dst = out + (r * NC + c) * wp + 3 * E * k;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j >= nch) break;
      if constexpr (E == 4) {
        *reinterpret_cast<float4v*>(dst + 4 * j) = float4v{v[c * G + 4 * j], v[c * G + 4 * j + 1],
                                                           v[c * G + 4 * j + 2], v[c * G + 4 * j + 3]};
      } else {
        half8v o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (half_t)v[c * G + 8 * j + e];
        *reinterpret_cast<half8v*>(dst + 8 * j) = o;
      }
    }
  }
}

template <typename T>
static void pack3_launch(const uint8_t* img, T* out, int B, int H, int W, int pad, int nc, int wp,
                         const long long* start_idx, long long start_off, long long max_start, long long sub,
                         hipStream_t st) {
  constexpr int E = 16 / (int)sizeof(T);
  const int bs = 256;
  const long total = (long)B * H * ((wp + 3 * E - 1) / (3 * E));
  const long grid = (total + bs - 1) / bs;
  auto kern = nc == 4 ? preprocess_pack3_kernel<T, 4>
              : nc == 2 ? preprocess_pack3_kernel<T, 2> : preprocess_pack3_kernel<T, 1>;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(bs), 0, st, img, out, B, H, W, pad, wp, start_idx, start_off,
                     max_start, sub);
}

void preprocess_pack3_f32_launch(const uint8_t* img, float* out, int B, int H, int W, int pad, int nc, int wp,
                                 const long long* start_idx, long long start_off, long long max_start,
                                 long long sub, hipStream_t st) {
  pack3_launch<float>(img, out, B, H, W, pad, nc, wp, start_idx, start_off, max_start, sub, st);
}

void preprocess_pack3_split_launch(const uint8_t* img, half_t* out, int B, int H, int W, int pad, int nc, int wp,
                                   const long long* start_idx, long long start_off, long long max_start,
                                   long long sub, hipStream_t st) {
  const long total = (long)B * H * ((wp + 23) / 24);
  auto kern = nc == 4 ? preprocess_pack3_kernel<half_t, 4, true>
              : nc == 2 ? preprocess_pack3_kernel<half_t, 2, true> : preprocess_pack3_kernel<half_t, 1, true>;
  hipLaunchKernelGGL(kern, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, img, out, B, H, W, pad, wp,
                     start_idx, start_off, max_start, sub);
}

void preprocess_pack3_f16_launch(const uint8_t* img, half_t* out, int B, int H, int W, int pad, int nc, int wp,
                                 const long long* start_idx, long long start_off, long long max_start,
                                 long long sub, hipStream_t st) {
  pack3_launch<half_t>(img, out, B, H, W, pad, nc, wp, start_idx, start_off, max_start, sub, st);
}

void preprocess_f32_launch(const uint8_t* img, float* out, long npix, const long long* start_idx,
                           long long start_off, long long max_start, long long sub, long pix_per_img,
                           hipStream_t st) {
  const int bs = 256;
  const long grid = ((npix + 3) / 4 + bs - 1) / bs;
  hipLaunchKernelGGL(preprocess_f32_kernel, dim3((unsigned)grid), dim3(bs), 0, st, img, out, npix, start_idx,
                     start_off, max_start, sub, pix_per_img);
}

// NHWC max pool, C % 4 == 0: one thread = 4 channels of one output pixel.
__global__ void maxpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int H, int W,
                                   int C, int Ho, int Wo, int k, int s, int pad) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = C / 4;
  const long total = (long)B * Ho * Wo * cv;
  if (t >= total) return;
  const int c4 = (int)(t % cv);
  long pix = t / cv;
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
      const float4v v = *reinterpret_cast<const float4v*>(x + (((size_t)b * H + ih) * W + iw) * C + c4 * 4);
      m[0] = fmaxf(m[0], v[0]);
      m[1] = fmaxf(m[1], v[1]);
      m[2] = fmaxf(m[2], v[2]);
      m[3] = fmaxf(m[3], v[3]);
    }
  }
  *reinterpret_cast<float4v*>(y + (size_t)t * 4) = m;
}

void maxpool_f32_launch(const float* x, float* y, int B, int H, int W, int C, int Ho, int Wo, int k, int s,
                        int pad, hipStream_t st) {
  const long total = (long)B * Ho * Wo * (C / 4);
  const int bs = 256;
  hipLaunchKernelGGL(maxpool_f32_kernel, dim3((unsigned)((total + bs - 1) / bs)), dim3(bs), 0, st, x, y, B, H, W,
                     C, Ho, Wo, k, s, pad);
}

// NHWC global average pool -> [B][C] fp32.  One 256-thread workgroup per
// image; thread (g, c4) sums pixels g, g+G, ... of 4-channel chunk c4, the G
// partial sums meet in LDS (same decomposition as the fp16 avgpool_kernel).
// Global average pool, fp32 NHWC [B][HW][C] -> [B][C].  A workgroup takes one
// image and 32 channel quads (128 channels); its 8 pixel groups each sum every
// 8th pixel (independent 16-byte loads, unrolled), then one LDS pass adds the
// groups.  Grid B x C/128: at B = 50 (strong scaling) and C = 512 that is 200
// workgroups of ~6 loads per lane instead of 50 of ~25 (round 5: 8.3 us).
__global__ void __launch_bounds__(256) avgpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int B,
                                                          int HW, int C) {
  __shared__ float4v part[256];
  const int b = blockIdx.x;
  const int cv = C / 4;
  const int q = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int c4 = blockIdx.y * 32 + q;
  const float* p = x + (size_t)b * HW * C;
  float4v acc = float4v{0.f, 0.f, 0.f, 0.f};
  if (c4 < cv) {
    int i = g;
#pragma unroll 4
    for (; i < HW; i += 8) acc += *reinterpret_cast<const float4v*>(p + (size_t)i * C + c4 * 4);
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && c4 < cv) {
#pragma unroll
    for (int k = 1; k < 8; ++k) acc += part[k * 32 + q];
    *reinterpret_cast<float4v*>(y + (size_t)b * C + c4 * 4) = acc * (1.f / (float)HW);
  }
}

void avgpool_f32_launch(const float* x, float* y, int B, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_f32_kernel, dim3((unsigned)B, (unsigned)((C / 4 + 31) / 32)), dim3(256), 0, st, x, y, B,
                     HW, C);
}

}  // namespace idunno
