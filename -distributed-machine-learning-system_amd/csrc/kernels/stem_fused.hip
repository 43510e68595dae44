// Fused ResNet stem: uint8 images -> normalise -> conv 7x7/2 (3->64, BN folded)
// -> ReLU -> max-pool 3x3/2 -> fp16 NHWC [B][56][56][64], in ONE kernel.
//
// Replaces four separate passes of the unfused path (preprocess, the 7x7 conv,
// the 112x112x64 activation write + re-read, max-pool; reference op chain
// alexnet_resnet.py:57-75 -> torchvision resnet18.conv1/bn1/relu/maxpool).
// The 112x112x64 conv activation (642 MB at B=400) never touches HBM.
//
// One workgroup = one 8x8 tile of pooled outputs of one image:
//   * the 39x40 input patch it needs is read once as uint8, normalised, and
//     stored in LDS as [row][col][4] fp16 (channel 3 = 0), so every conv tap is
//     an LDS read;
//   * the 17x17 conv outputs under the tile's pool windows (289 pixels, padded
//     to 19 fragments of 16) are an implicit GEMM M=304, N=64, K=7x32 on
//     v_mfma_f32_16x16x32_f16: one K stage per kernel row kh = 8 taps x 4 ch
//     (taps 7 and channel 3 carry zero weights); each B fragment row is 16
//     contiguous, 16-byte-aligned bytes of the patch (two adjacent taps);
//   * conv outputs (+bias, ReLU; zero outside the image, which equals -inf
//     padding after ReLU) go to an LDS tile, then 9-way max per pooled pixel
//     with 16-byte LDS reads and 16-byte global stores.
#include "../kernels.h"

namespace idunno {

namespace stem {
constexpr int KH = 7, CS = 2, CP = 3;      // conv
constexpr int PK = 3, PS = 2, PP = 1;      // pool
constexpr int PT = 8;                       // pooled tile edge
constexpr int CR = (PT - 1) * PS + PK;      // 17 conv rows/cols under the tile
constexpr int NPIX = CR * CR;               // 289
constexpr int NFRAG = (NPIX + 15) / 16;     // 19
constexpr int IPR = (CR - 1) * CS + KH;     // 39 patch rows
constexpr int IPC = (CR - 1) * CS + 8;      // 40 patch cols (8th tap read, zero weight)
constexpr int PATCH_BYTES = IPR * IPC * 8;  // 12480
constexpr int W_BYTES = KH * 64 * 64;       // [kh][cout 64][32 halfs] = 28672
constexpr int CONV_BYTES = NPIX * 128;      // [pix][64 ch] fp16 = 36992
constexpr int LDS = PATCH_BYTES + W_BYTES + CONV_BYTES;
}  // namespace stem

__constant__ float kStemMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStemInvStd[3] = {1.0f / 0.229f, 1.0f / 0.224f, 1.0f / 0.225f};

__device__ __forceinline__ int swz64s(int row) {
  const int q = (row >> 2) & 3;
  return (0x78 >> (2 * q)) & 3;
}

__global__ void __launch_bounds__(256, 2)
stem_fused_kernel(const uint8_t* __restrict__ img, const half_t* __restrict__ w, const float* __restrict__ bias,
                  half_t* __restrict__ y, int B, int H, int W, int Hc, int Wc, int Hp, int Wp, int tiles_x,
                  int tiles_y) {
  using namespace stem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* patch = smem;
  char* wl = smem + PATCH_BYTES;
  char* conv = smem + PATCH_BYTES + W_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int per_img = tiles_x * tiles_y;
  const int b = blockIdx.x / per_img;
  const int t = blockIdx.x - b * per_img;
  const int py0 = (t / tiles_x) * PT, px0 = (t % tiles_x) * PT;
  const int oy0 = py0 * PS - PP, ox0 = px0 * PS - PP;       // first conv row/col of the tile
  const int iy0 = oy0 * CS - CP, ix0 = ox0 * CS - CP;       // first input row/col of the patch

  // ---- weights -> LDS [kh][cout][32] (swizzled 16-byte chunks) -------------
  for (int i = tid; i < 64 * KH * 4; i += 256) {
    const int ch = i & 3, kh = (i >> 2) % KH, co = i / (4 * KH);
    const vec16 v = *reinterpret_cast<const vec16*>(w + (size_t)co * (KH * 32) + kh * 32 + ch * 8);
    *reinterpret_cast<vec16*>(wl + kh * 4096 + co * 64 + ((ch ^ swz64s(co)) << 4)) = v;
  }
  // ---- uint8 patch -> normalised fp16 [row][col][4] ------------------------
  const uint8_t* ib = img + (size_t)b * H * W * 3;
  for (int i = tid; i < IPR * IPC; i += 256) {
    const int r = i / IPC, c = i - r * IPC;
    const int iy = iy0 + r, ix = ix0 + c;
    half4v o = {(half_t)0.f, (half_t)0.f, (half_t)0.f, (half_t)0.f};
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
      const uint8_t* p = ib + ((size_t)iy * W + ix) * 3;
      o[0] = (half_t)(((float)p[0] * (1.f / 255.f) - kStemMean[0]) * kStemInvStd[0]);
      o[1] = (half_t)(((float)p[1] * (1.f / 255.f) - kStemMean[1]) * kStemInvStd[1]);
      o[2] = (half_t)(((float)p[2] * (1.f / 255.f) - kStemMean[2]) * kStemInvStd[2]);
    }
    *reinterpret_cast<half4v*>(patch + i * 8) = o;
  }
  __syncthreads();

  // ---- A fragments (weights) for all 7 K stages, kept in registers -----------
  const int frow = lane & 15, fch = lane >> 4;
  half8v fa[KH][4];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = i * 16 + frow;
      fa[kh][i] = *reinterpret_cast<const half8v*>(wl + kh * 4096 + row * 64 + ((fch ^ swz64s(row)) << 4));
    }
  float bv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[i][r] = bias[i * 16 + fch * 4 + r];

  // ---- conv GEMM over the 19 pixel fragments, round-robin over 4 waves -------
  for (int f = wave; f < NFRAG; f += 4) {
    const int p = f * 16 + frow;
    const int pc = min(p, NPIX - 1);                    // padded rows read a valid address
    const int cy = pc / CR, cx = pc - cy * CR;
    const char* pb = patch + ((2 * cy) * IPC + 2 * cx + 2 * fch) * 8;
    float4v acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const half8v fb = *reinterpret_cast<const half8v*>(pb + kh * IPC * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[kh][i], fb, acc[i], 0, 0, 0);
    }
    // epilogue into the LDS conv tile: lane holds pixel (l&15), couts i*16+(l>>4)*4+r
    if (p < NPIX) {
      const int oy = oy0 + cy, ox = ox0 + cx;
      const bool valid = (unsigned)oy < (unsigned)Hc && (unsigned)ox < (unsigned)Wc;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        half4v o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (half_t)(valid ? fmaxf(acc[i][r] + bv[i][r], 0.f) : 0.f);
        *reinterpret_cast<half4v*>(conv + p * 128 + (i * 16 + fch * 4) * 2) = o;
      }
    }
  }
  __syncthreads();

  // ---- 3x3/2 max-pool from the LDS tile -> global -----------------------------
  for (int i = tid; i < PT * PT * 8; i += 256) {
    const int c8 = i & 7, pp = i >> 3;
    const int py = pp / PT, px = pp - py * PT;
    if (py0 + py >= Hp || px0 + px >= Wp) continue;
    half8v m = *reinterpret_cast<const half8v*>(conv + ((2 * py) * CR + 2 * px) * 128 + c8 * 16);
#pragma unroll
    for (int dy = 0; dy < PK; ++dy)
#pragma unroll
      for (int dx = 0; dx < PK; ++dx) {
        const half8v v = *reinterpret_cast<const half8v*>(conv + ((2 * py + dy) * CR + 2 * px + dx) * 128 + c8 * 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = v[j] > m[j] ? v[j] : m[j];
      }
    *reinterpret_cast<half8v*>(y + (((size_t)b * Hp + py0 + py) * Wp + px0 + px) * 64 + c8 * 8) = m;
  }
}

void stem_fused_launch(const uint8_t* img, const half_t* w, const float* bias, half_t* y, int B, int H, int W,
                       hipStream_t st) {
  using namespace stem;
  const int Hc = (H + 2 * CP - KH) / CS + 1, Wc = (W + 2 * CP - KH) / CS + 1;
  const int Hp = (Hc + 2 * PP - PK) / PS + 1, Wp = (Wc + 2 * PP - PK) / PS + 1;
  const int tx = (Wp + PT - 1) / PT, ty = (Hp + PT - 1) / PT;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fused_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL(stem_fused_kernel, dim3(B * tx * ty), dim3(256), LDS, st, img, w, bias, y, B, H, W, Hc, Wc,
                     Hp, Wp, tx, ty);
}

}  // namespace idunno
