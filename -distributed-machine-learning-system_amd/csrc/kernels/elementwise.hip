// Memory-bound companions of the implicit-GEMM conv:
//   * preprocess      uint8 HWC images -> normalised fp16 NHWC (C padded to 4)
//                     (replaces ToTensor + Normalize, reference alexnet_resnet.py:57-62)
//   * resize_crop     bilinear resize (shorter side -> `resize`) + centre crop,
//                     fused with the normalisation (reference :57-59, Resize(256)
//                     + CenterCrop(224)) for real, non-224 inputs
//   * maxpool2d       NHWC 3x3 (any k/stride/pad), 8 channels per lane
//   * global_avgpool  NHWC [B][HW][C] -> [B][C]
//   * softmax_top1    row softmax + argmax fused, one wave per row
//                     (replaces softmax + topk(1), reference :80-84)
// All loads/stores are 8-16 bytes per lane (cdna_hip_programming Guideline 13).
#include "../kernels.h"

namespace idunno {

// ImageNet statistics (reference alexnet_resnet.py:61)
__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kInvStd[3] = {1.0f / 0.229f, 1.0f / 0.224f, 1.0f / 0.225f};

__device__ __forceinline__ half4v norm_px(uint32_t b0, uint32_t b1, uint32_t b2) {
  half4v o;
  o[0] = (half_t)(((float)b0 * (1.f / 255.f) - kMean[0]) * kInvStd[0]);
  o[1] = (half_t)(((float)b1 * (1.f / 255.f) - kMean[1]) * kInvStd[1]);
  o[2] = (half_t)(((float)b2 * (1.f / 255.f) - kMean[2]) * kInvStd[2]);
  o[3] = (half_t)0.f;
  return o;
}

// Four pixels per thread: 12 bytes in (three dword loads when the quad is
// 4-byte aligned -- always for 224x224 shards), 32 bytes (two 16-byte
// stores) out.  A ragged or unaligned quad falls back to byte loads.
// Optional device-side window: images start at *start_idx (clamped to
// [0, max_start]) of the shard `img`.
__global__ void preprocess_kernel(const uint8_t* __restrict__ img, half_t* __restrict__ out,
                                  long npix, const long long* __restrict__ start_idx, long long start_off,
                                  long long max_start, long long sub, long pix_per_img) {
  const long p = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (p >= npix) return;
  if (start_idx != nullptr) {
    long long s0 = *start_idx - start_off;
    s0 = (s0 < 0 ? 0 : (s0 > max_start ? max_start : s0)) + sub;
    img += (size_t)s0 * pix_per_img * 3;
  }
  const uint8_t* s = img + p * 3;
  half_t* d = out + p * 4;
  if (p + 4 <= npix && (reinterpret_cast<uintptr_t>(s) & 3) == 0 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    // bytes: w0 = r0 g0 b0 r1 | w1 = g1 b1 r2 g2 | w2 = b2 r3 g3 b3
    const half4v o0 = norm_px(w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u);
    const half4v o1 = norm_px(w0 >> 24, w1 & 255u, (w1 >> 8) & 255u);
    const half4v o2 = norm_px((w1 >> 16) & 255u, w1 >> 24, w2 & 255u);
    const half4v o3 = norm_px((w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24);
    half8v v0, v1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v0[i] = o0[i];
      v0[4 + i] = o1[i];
      v1[i] = o2[i];
      v1[4 + i] = o3[i];
    }
    reinterpret_cast<half8v*>(d)[0] = v0;
    reinterpret_cast<half8v*>(d)[1] = v1;
    return;
  }
  const int n = (int)(npix - p < 4 ? npix - p : 4);
  for (int i = 0; i < n; ++i)
    *reinterpret_cast<half4v*>(d + i * 4) = norm_px(s[3 * i], s[3 * i + 1], s[3 * i + 2]);
}

void preprocess_launch(const uint8_t* img, half_t* out, long npix, const long long* start_idx,
                       long long start_off, long long max_start, long long sub, long pix_per_img,
                       hipStream_t st) {
  const int bs = 256;
  const long grid = ((npix + 3) / 4 + bs - 1) / bs;
  hipLaunchKernelGGL(preprocess_kernel, dim3((unsigned)grid), dim3(bs), 0, st, img, out, npix, start_idx,
                     start_off, max_start, sub, pix_per_img);
}

// Bilinear resize of an (Hi x Wi) uint8 HWC image so that its shorter side is
// `rs`, then a centre crop of `crop` x `crop`, then normalisation.  Matches
// torchvision's Resize (bilinear, half-pixel centres, no antialias) + CenterCrop.
__global__ void resize_crop_kernel(const uint8_t* __restrict__ img, half_t* __restrict__ out,
                                   int B, int Hi, int Wi, int Hr, int Wr, int crop) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long npix = (long)B * crop * crop;
  if (p >= npix) return;
  const int b = (int)(p / (crop * crop));
  const int r = (int)(p - (long)b * crop * crop);
  const int oy = r / crop, ox = r - oy * crop;
  const int top = (Hr - crop + 1) / 2, left = (Wr - crop + 1) / 2;  // round((H-c)/2)
  const int y = oy + top, x = ox + left;
  const float sy = (float)Hi / (float)Hr, sx = (float)Wi / (float)Wr;
  float fy = ((float)y + 0.5f) * sy - 0.5f, fx = ((float)x + 0.5f) * sx - 0.5f;
  fy = fmaxf(fy, 0.f);
  fx = fmaxf(fx, 0.f);
  int y0 = (int)fy, x0 = (int)fx;
  y0 = min(y0, Hi - 1);
  x0 = min(x0, Wi - 1);
  const int y1 = min(y0 + 1, Hi - 1), x1 = min(x0 + 1, Wi - 1);
  const float wy = fy - (float)y0, wx = fx - (float)x0;
  const uint8_t* base = img + (size_t)b * Hi * Wi * 3;
  half4v o;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v00 = base[((size_t)y0 * Wi + x0) * 3 + c], v01 = base[((size_t)y0 * Wi + x1) * 3 + c];
    const float v10 = base[((size_t)y1 * Wi + x0) * 3 + c], v11 = base[((size_t)y1 * Wi + x1) * 3 + c];
    const float v = (v00 * (1.f - wx) + v01 * wx) * (1.f - wy) + (v10 * (1.f - wx) + v11 * wx) * wy;
    o[c] = (half_t)((v * (1.f / 255.f) - kMean[c]) * kInvStd[c]);
  }
  o[3] = (half_t)0.f;
  *reinterpret_cast<half4v*>(out + p * 4) = o;
}

void resize_crop_launch(const uint8_t* img, half_t* out, int B, int Hi, int Wi, int Hr, int Wr,
                        int crop, hipStream_t st) {
  const long npix = (long)B * crop * crop;
  const int bs = 256;
  hipLaunchKernelGGL(resize_crop_kernel, dim3((unsigned)((npix + bs - 1) / bs)), dim3(bs), 0, st,
                     img, out, B, Hi, Wi, Hr, Wr, crop);
}

// NHWC max-pool; C % 8 == 0.  One thread = 8 channels of one output pixel.
__global__ void maxpool_kernel(const half_t* __restrict__ x, half_t* __restrict__ y, int B, int H,
                               int W, int C, int Ho, int Wo, int k, int s, int pad) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = C / 8;
  const long total = (long)B * Ho * Wo * cv;
  if (t >= total) return;
  const int c8 = (int)(t % cv);
  long pix = t / cv;
  const int ow = (int)(pix % Wo);
  pix /= Wo;
  const int oh = (int)(pix % Ho);
  const int b = (int)(pix / Ho);
  half8v m;
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = (half_t)(-65504.f);
  const int ih0 = oh * s - pad, iw0 = ow * s - pad;
  for (int dy = 0; dy < k; ++dy) {
    const int ih = ih0 + dy;
    if ((unsigned)ih >= (unsigned)H) continue;
    for (int dx = 0; dx < k; ++dx) {
      const int iw = iw0 + dx;
      if ((unsigned)iw >= (unsigned)W) continue;
      const half8v v = *reinterpret_cast<const half8v*>(x + (((size_t)b * H + ih) * W + iw) * C + c8 * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = v[i] > m[i] ? v[i] : m[i];
    }
  }
  *reinterpret_cast<half8v*>(y + (size_t)t * 8) = m;
}

void maxpool_launch(const half_t* x, half_t* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                    int s, int pad, hipStream_t st) {
  const long total = (long)B * Ho * Wo * (C / 8);
  const int bs = 256;
  hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)((total + bs - 1) / bs)), dim3(bs), 0, st, x, y,
                     B, H, W, C, Ho, Wo, k, s, pad);
}

// NHWC global average pool -> [B][C] fp16.  One 256-thread workgroup per image:
// thread (g, c8) sums pixels g, g+G, ... of 8-channel chunk c8 (16-byte loads),
// the G partial sums meet in LDS.  (One thread per chunk over all HW pixels ran
// 400 workgroups' worth of work on 100 workgroups with a 49-long dependent
// chain: 17 us for the 20 MB ResNet18 layer4 output.)
__global__ void __launch_bounds__(256) avgpool_kernel(const half_t* __restrict__ x, half_t* __restrict__ y,
                                                      int B, int HW, int C) {
  __shared__ float part[256 * 8];
  const int b = blockIdx.x;
  const int cv = C / 8;
  const int G = cv >= 256 ? 1 : 256 / cv;          // pixel groups per chunk
  const half_t* p = x + (size_t)b * HW * C;
  const float inv = 1.f / (float)HW;
  for (int c8 = threadIdx.x % cv; c8 < cv; c8 += (cv >= 256 ? 256 : cv)) {
    const int g = cv >= 256 ? 0 : threadIdx.x / cv;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (g < G) {
      for (int i = g; i < HW; i += G) {
        const half8v v = *reinterpret_cast<const half8v*>(p + (size_t)i * C + c8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
      }
    }
    if (G == 1) {
      half8v o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)(acc[j] * inv);
      *reinterpret_cast<half8v*>(y + (size_t)b * C + c8 * 8) = o;
      continue;
    }
    if (g < G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) part[(g * cv + c8) * 8 + j] = acc[j];
    }
    __syncthreads();
    if (g == 0) {
      for (int k = 1; k < G; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += part[(k * cv + c8) * 8 + j];
      half8v o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (half_t)(acc[j] * inv);
      *reinterpret_cast<half8v*>(y + (size_t)b * C + c8 * 8) = o;
    }
    break;                                          // G > 1: every chunk handled in one pass
  }
}

void avgpool_launch(const half_t* x, half_t* y, int B, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_kernel, dim3((unsigned)B), dim3(256), 0, st, x, y, B, HW, C);
}

// Split-K combine: y[m][n] = act(sum_s part[s][m][n] + bias[n]), 4 outputs per
// thread (16-byte partial loads), fp16 or fp32 out.
__global__ void splitk_reduce_kernel(const float* __restrict__ part, int S, long MN, int N,
                                     const float* __restrict__ bias, int relu, void* __restrict__ y, int out_f32,
                                     int* ovf) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= MN) return;
  float4v v = *reinterpret_cast<const float4v*>(part + i);
  for (int s = 1; s < S; ++s) v += *reinterpret_cast<const float4v*>(part + (long)s * MN + i);
  const int n = (int)(i % N);
  v += *reinterpret_cast<const float4v*>(bias + n);
  if (relu) {
    v[0] = fmaxf(v[0], 0.f);
    v[1] = fmaxf(v[1], 0.f);
    v[2] = fmaxf(v[2], 0.f);
    v[3] = fmaxf(v[3], 0.f);
  }
  if (out_f32 == 2) {                     // split-fp16 layout [M][2N] (N % 32 == 0)
    split_guard(ovf, v);
    half4v h, l;
    split_f16x4(v, h, l);
    half_t* yp = static_cast<half_t*>(y) + (i / N) * 2 * N + split_off(n);
    *reinterpret_cast<half4v*>(yp) = h;
    *reinterpret_cast<half4v*>(yp + 32) = l;
  } else if (out_f32) {
    *reinterpret_cast<float4v*>(static_cast<float*>(y) + i) = v;
  } else {
    half4v o;
    o[0] = (half_t)v[0];
    o[1] = (half_t)v[1];
    o[2] = (half_t)v[2];
    o[3] = (half_t)v[3];
    *reinterpret_cast<half4v*>(static_cast<half_t*>(y) + i) = o;
  }
}

// Split-K combine for convs: y = act(sum_s part[s] + bias (+ split residual)), split
// [M][ldy] or fp32 [M][ldy] out, range-guarded (common.h split_guard).
// fmt: 0 split-fp16 residual and output, 1 split residual and fp32 output,
// 2 fp16 residual and fp16 output, 3 fp16 residual and fp32 output
__global__ void splitk_reduce_res_kernel(const float* __restrict__ part, int S, long MN, int N,
                                         const float* __restrict__ bias, const half_t* __restrict__ res, int ldr,
                                         int relu, void* __restrict__ y, int ldy, int fmt, int* ovf) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= MN) return;
  float4v v = *reinterpret_cast<const float4v*>(part + i);
  for (int s = 1; s < S; ++s) v += *reinterpret_cast<const float4v*>(part + (long)s * MN + i);
  const long m = i / N;
  const int n = (int)(i - m * N);
  v += *reinterpret_cast<const float4v*>(bias + n);
  if (res != nullptr && fmt < 2) {
    const half_t* rp = res + m * ldr + split_off(n);
    const half4v h = *reinterpret_cast<const half4v*>(rp), l = *reinterpret_cast<const half4v*>(rp + 32);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += (float)h[e] + (float)l[e];
  } else if (res != nullptr) {
    const half4v h = *reinterpret_cast<const half4v*>(res + m * ldr + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += (float)h[e];
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if (fmt == 1 || fmt == 3) {
    *reinterpret_cast<float4v*>(static_cast<float*>(y) + m * ldy + n) = v;
  } else if (fmt == 2) {
    half4v o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (half_t)v[e];
    *reinterpret_cast<half4v*>(static_cast<half_t*>(y) + m * ldy + n) = o;
  } else {
    split_guard(ovf, v);
    half4v h, l;
    split_f16x4(v, h, l);
    half_t* yp = static_cast<half_t*>(y) + m * ldy + split_off(n);
    *reinterpret_cast<half4v*>(yp) = h;
    *reinterpret_cast<half4v*>(yp + 32) = l;
  }
}

void splitk_reduce_res_launch(const float* part, int S, long MN, int N, const float* bias, const half_t* res,
                              int ldr, int relu, void* y, int ldy, int fmt, int* ovf, hipStream_t st) {
  const long threads = (MN + 3) / 4;
  hipLaunchKernelGGL(splitk_reduce_res_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, part, S,
                     MN, N, bias, res, ldr, relu, y, ldy, fmt, ovf);
}

void splitk_reduce_split_launch(const float* part, int S, long MN, int N, const float* bias, int relu, half_t* y,
                                int* ovf, hipStream_t st) {
  const long threads = (MN + 3) / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, part, S, MN, N,
                     bias, relu, (void*)y, 2, ovf);
}

void splitk_reduce_launch(const float* part, int S, long MN, int N, const float* bias, int relu, void* y,
                          bool out_f32, hipStream_t st) {
  const int bs = 256;
  const long threads = (MN + 3) / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((threads + bs - 1) / bs)), dim3(bs), 0, st, part, S, MN, N,
                     bias, relu, y, out_f32 ? 1 : 0, (int*)nullptr);
}

// Row softmax + top-1: one 64-lane wave per row of fp32 logits.
// prob(top1) = 1 / sum_j exp(x_j - x_max).  Ties resolve to the lowest index
// (torch.topk semantics on CPU).
__global__ void softmax_top1_kernel(const float* __restrict__ logits, int ld, int N, int rows,
                                    int* __restrict__ cls, float* __restrict__ prob, int* __restrict__ packed,
                                    const int* __restrict__ ovf) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= rows) return;
  if (ovf != nullptr && *ovf != 0) {        // split range exceeded somewhere in this forward
    if (lane == 0) {
      cls[wave] = -2;
      prob[wave] = 0.f;
      if (packed != nullptr) {
        packed[2 * wave] = -2;
        packed[2 * wave + 1] = 0;
      }
    }
    return;
  }
  const float* r = logits + (size_t)wave * ld;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  // N <= 1024 (every classifier here): the row's values land in registers from 16
  // independent loads per lane, read once for both the max and the sum (round 5 read
  // the row twice through two loop-carried load chains: 8.4 us at B = 50)
  constexpr int NR = 16;
  float vr[NR];
  const bool reg = N <= 64 * NR;
  if (reg) {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int j = lane + 64 * k;
      vr[k] = j < N ? r[j] : -INFINITY;
    }
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (vr[k] > best) {          // strict: the lowest index of a lane wins ties
        best = vr[k];
        bidx = lane + 64 * k;
      }
  } else {
    for (int j = lane; j < N; j += 64) {
      const float v = r[j];
      if (v > best) {
        best = v;
        bidx = j;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) {
      best = ov;
      bidx = oi;
    }
  }
  float s = 0.f;
  if (reg) {
#pragma unroll
    for (int k = 0; k < NR; ++k)
      if (lane + 64 * k < N) s += __expf(vr[k] - best);
  } else {
    for (int j = lane; j < N; j += 64) s += __expf(r[j] - best);
  }
  s = wave_sum(s);
  if (lane == 0) {
    const float p = 1.f / s;
    cls[wave] = bidx;
    prob[wave] = p;
    if (packed != nullptr) {   // (class, prob bits) pairs: the RCCL gather's send buffer
      packed[2 * wave] = bidx;
      packed[2 * wave + 1] = __float_as_int(p);
    }
  }
}

void softmax_top1_launch(const float* logits, int ld, int N, int rows, int* cls, float* prob, int* packed,
                         const int* ovf, hipStream_t st) {
  const int bs = 256;  // 4 rows per block
  const int grid = (rows + 3) / 4;
  hipLaunchKernelGGL(softmax_top1_kernel, dim3(grid), dim3(bs), 0, st, logits, ld, N, rows, cls,
                     prob, packed, ovf);
}

// Deterministic synthetic images: byte group g (8 bytes) of image `idx` is the
// little-endian splitmix64 hash of (seed << 32) ^ (idx * 18816 + g), where
// 18816 = 224*224*3 / 8.  The CPU generator (idunno.runtime.data) computes the
// same function with numpy, so any worker (GPU or CPU) produces bit-identical
// image `idx` without moving bytes - the synthetic stand-in for the
// reference's ./<model>/test_<i>.JPEG files.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void synth_images_kernel(uint64_t* __restrict__ out, uint64_t seed, long start, long n,
                                    long groups_per_img) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * groups_per_img) return;
  const long i = t / groups_per_img, g = t - i * groups_per_img;
  out[t] = splitmix64((seed << 32) ^ (uint64_t)((start + i) * groups_per_img + g));
}

void synth_images_launch(uint8_t* out, uint64_t seed, long start, long n, long bytes_per_img,
                         hipStream_t st) {
  const long gpi = bytes_per_img / 8;
  const long total = n * gpi;
  const int bs = 256;
  hipLaunchKernelGGL(synth_images_kernel, dim3((unsigned)((total + bs - 1) / bs)), dim3(bs), 0, st,
                     reinterpret_cast<uint64_t*>(out), seed, start, n, gpi);
}

}  // namespace idunno
