// Fused ResNet stem: uint8 images -> normalise -> conv 7x7/2 (3->64, BN folded)
// -> ReLU -> max-pool 3x3/2 -> fp16 NHWC [B][Hp][Wp][64], in ONE persistent kernel.
//
// Replaces four separate passes of the unfused path (preprocess, the 7x7 conv,
// the 112x112x64 activation write + re-read, max-pool; reference op chain
// alexnet_resnet.py:57-75 -> torchvision resnet18.conv1/bn1/relu/maxpool).
// The conv activation (642 MB at B=400) never touches HBM.
//
// Work item = one 8x8 tile of pooled outputs of one image.  Workgroups are
// persistent (2 per CU): the 28 KB of packed weights are staged into LDS and
// the 7x4 MFMA A-fragments into registers ONCE, then every tile
//   * takes its 39x40 uint8 input patch from registers prefetched one tile
//     earlier (12-byte aligned pixel quads), normalises it into LDS as
//     [row][col][4] fp16 (channel 3 = 0);
//   * computes the 17x17 conv outputs under its pool windows (289 px, 19
//     fragments of 16) as an implicit GEMM M=304, N=64, K=7x32 on
//     v_mfma_f32_16x16x32_f16 — one K stage per kernel row (8 taps x 4 ch;
//     tap 7 and channel 3 have zero weights); each B-fragment row is 16
//     contiguous, 16-byte-aligned bytes of the patch;
//   * writes bias+ReLU outputs (zero outside the image == -inf padding after
//     ReLU) to an LDS tile, issues the global loads of the next-next patch,
//     then max-pools 3x3/2 with 16-byte LDS reads and 16-byte stores.
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
constexpr int QPR = 11;                     // 4-pixel quads per patch row (44 px cover 40)
constexpr int NQUAD = IPR * QPR;            // 429
constexpr int QPT = (NQUAD + 255) / 256;    // quads per thread (2)
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

// Byte offset of 16-byte channel chunk c (0..7) of conv pixel p in the LDS conv
// tile.  Rows are 128 B (64 fp16 channels); the chunk is XOR-swizzled by p & 7 so
// the epilogue's 16 lanes (16 consecutive pixels, one channel chunk) hit 8
// different 16-byte slots instead of one bank (16-way -> 2-way).
__device__ __forceinline__ int conv_off(int p, int c) { return p * 128 + ((c ^ (p & 7)) << 4); }

struct StemGeom {
  int B, H, W, Hc, Wc, Hp, Wp, tiles_x, tiles_y, ntiles;
  int ablate;   // profiling only (set_stem_ablation): 1 skip pool, 2 skip MFMAs, 4 skip patch normalise
};

static int g_stem_ablate = 0;
void set_stem_ablation(int mode) { g_stem_ablate = mode; }

struct Quads {
  uint32_t d[stem::QPT][3];
  bool ok[stem::QPT];
};

__device__ __forceinline__ void tile_coords(const StemGeom& g, int t, int& b, int& py0, int& px0) {
  const int per = g.tiles_x * g.tiles_y;
  b = t / per;
  const int r = t - b * per;
  py0 = (r / g.tiles_x) * stem::PT;
  px0 = (r % g.tiles_x) * stem::PT;
}

// global -> registers: this thread's quads of tile t's input patch
__device__ __forceinline__ void load_quads(const uint8_t* __restrict__ img, const StemGeom& g, int t, int tid,
                                           Quads& q) {
  using namespace stem;
  int b, py0, px0;
  tile_coords(g, t, b, py0, px0);
  const int iy0 = (py0 * PS - PP) * CS - CP;
  const int ixa = (px0 * PS - PP) * CS - CP - 3;     // 4px0 - 8: quad-aligned first column
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    q.ok[k] = false;
    q.d[k][0] = q.d[k][1] = q.d[k][2] = 0u;
    if (i >= NQUAD) continue;
    const int r = i / QPR, qc = i - r * QPR;
    const int iy = iy0 + r, ix = ixa + 4 * qc;
    if ((unsigned)iy >= (unsigned)g.H) continue;
    const uint8_t* p = img + (((size_t)b * g.H + iy) * g.W + ix) * 3;
    if (ix >= 0 && ix + 3 < g.W) {
      const uint32_t* pd = reinterpret_cast<const uint32_t*>(p);   // 12-byte quads are 4-byte aligned
      q.d[k][0] = pd[0];
      q.d[k][1] = pd[1];
      q.d[k][2] = pd[2];
      q.ok[k] = true;
    } else {                                           // ragged image edge: byte loads
      uint8_t v[12];
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const int x = ix + j / 3;
        v[j] = ((unsigned)x < (unsigned)g.W) ? p[j] : 0;
      }
      q.d[k][0] = v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
      q.d[k][1] = v[4] | (v[5] << 8) | (v[6] << 16) | ((uint32_t)v[7] << 24);
      q.d[k][2] = v[8] | (v[9] << 8) | (v[10] << 16) | ((uint32_t)v[11] << 24);
      q.ok[k] = true;
    }
  }
}

// registers -> normalised fp16 patch in LDS (invalid quads/pixels -> 0)
__device__ __forceinline__ void store_patch(char* patch, const StemGeom& g, int t, int tid, const Quads& q) {
  using namespace stem;
  int b, py0, px0;
  tile_coords(g, t, b, py0, px0);
  const int ixa = (px0 * PS - PP) * CS - CP - 3;
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    if (i >= NQUAD) continue;
    const int r = i / QPR, qc = i - r * QPR;
    half4v px[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      half4v o = {(half_t)0.f, (half_t)0.f, (half_t)0.f, (half_t)0.f};
      const int x = ixa + 4 * qc + j;
      if (q.ok[k] && (unsigned)x < (unsigned)g.W) {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const int byte = 3 * j + ch;
          const uint32_t u = (q.d[k][byte >> 2] >> (8 * (byte & 3))) & 0xFFu;
          o[ch] = (half_t)(((float)u * (1.f / 255.f) - kStemMean[ch]) * kStemInvStd[ch]);
        }
      }
      px[j] = o;
    }
    // write pixel (t + lane) & 3 in step t: neighbouring lanes' 8-byte stores are
    // then 40 B apart instead of 32 B, i.e. 16 distinct bank pairs (4-way -> none)
#pragma unroll
    for (int t2 = 0; t2 < 4; ++t2) {
      const int j = (t2 + tid) & 3;
      const half4v o = j == 0 ? px[0] : (j == 1 ? px[1] : (j == 2 ? px[2] : px[3]));
      const int c = 4 * qc + j - 3;                    // patch column of pixel j
      if (c < 0 || c >= IPC) continue;
      *reinterpret_cast<half4v*>(patch + (r * IPC + c) * 8) = o;
    }
  }
}

__global__ void __launch_bounds__(256, 2)
stem_fused_kernel(const uint8_t* __restrict__ img, const half_t* __restrict__ w, const float* __restrict__ bias,
                  half_t* __restrict__ y, const StemGeom g, const long long* __restrict__ start_idx,
                  long long start_off, long long max_start, long long sub) {
  using namespace stem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // device-side first-image index: a captured hipGraph reads any window of an
  // HBM-resident image shard without a host round trip or a staging copy
  if (start_idx != nullptr) {
    long long s = *start_idx - start_off;
    s = (s < 0 ? 0 : (s > max_start ? max_start : s)) + sub;   // sub: this launch's part of the window
    img += (size_t)s * g.H * g.W * 3;
  }
  char* patch = smem;
  char* wl = smem + PATCH_BYTES;
  char* conv = smem + PATCH_BYTES + W_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  int t = blockIdx.x;
  if (t >= g.ntiles) return;   // whole workgroup exits together (uniform)

  Quads q;
  load_quads(img, g, t, tid, q);

  // ---- weights -> LDS [kh][cout][32] (swizzled 16-byte chunks), once ---------
  for (int i = tid; i < 64 * KH * 4; i += 256) {
    const int ch = i & 3, kh = (i >> 2) % KH, co = i / (4 * KH);
    const vec16 v = *reinterpret_cast<const vec16*>(w + (size_t)co * (KH * 32) + kh * 32 + ch * 8);
    *reinterpret_cast<vec16*>(wl + kh * 4096 + co * 64 + ((ch ^ swz64s(co)) << 4)) = v;
  }
  store_patch(patch, g, t, tid, q);
  int tn = t + gridDim.x;
  if (tn < g.ntiles) load_quads(img, g, tn, tid, q);
  __syncthreads();

  const int frow = lane & 15, fch = lane >> 4;
  half8v fa[KH][4];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = i * 16 + frow;
      fa[kh][i] = *reinterpret_cast<const half8v*>(wl + kh * 4096 + row * 64 + ((fch ^ swz64s(row)) << 4));
    }
  // bias + ReLU are applied AFTER the max-pool (both commute with max:
  // relu(max(x) + b) == max(relu(x + b))), once per pooled output instead of once
  // per conv output (4.5x fewer); each thread pools one fixed 8-channel chunk
  half8v pb8;
#pragma unroll
  for (int j = 0; j < 8; ++j) pb8[j] = (half_t)bias[(tid & 7) * 8 + j];

  while (true) {
    int b, py0, px0;
    tile_coords(g, t, b, py0, px0);
    const int oy0 = py0 * PS - PP, ox0 = px0 * PS - PP;

    // ---- conv GEMM over the 19 pixel fragments, round-robin over 4 waves -----
    for (int f = wave; f < NFRAG; f += 4) {
      const int p = f * 16 + frow;
      const int pc = min(p, NPIX - 1);
      const int cy = pc / CR, cx = pc - cy * CR;
      const char* pb = patch + ((2 * cy) * IPC + 2 * cx + 2 * fch) * 8;
      float4v acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = float4v{0.f, 0.f, 0.f, 0.f};
      if (!(g.ablate & 2)) {
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          const half8v fb = *reinterpret_cast<const half8v*>(pb + kh * IPC * 8);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[kh][i], fb, acc[i], 0, 0, 0);
        }
      }
      if (p < NPIX) {
        const int oy = oy0 + cy, ox = ox0 + cx;
        const bool valid = (unsigned)oy < (unsigned)g.Hc && (unsigned)ox < (unsigned)g.Wc;
        // raw conv sums; outside the image -65504 (the pool's -inf padding)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          half4v o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = valid ? (half_t)acc[i][r] : (half_t)(-65504.f);
          *reinterpret_cast<half4v*>(conv + conv_off(p, i * 2 + (fch >> 1)) + (fch & 1) * 8) = o;
        }
      }
    }
    __syncthreads();   // conv tile complete; patch(t) no longer read

    const int tnext = tn;
    if (tnext < g.ntiles) {
      if (!(g.ablate & 4)) store_patch(patch, g, tnext, tid, q);   // uses the quads prefetched one tile ago
      tn = tnext + gridDim.x;
      if (tn < g.ntiles) load_quads(img, g, tn, tid, q);
    }

    // ---- 3x3/2 max-pool from the LDS tile -> global ---------------------------
    for (int i = tid; i < ((g.ablate & 1) ? 0 : PT * PT * 8); i += 256) {
      const int c8 = i & 7, pp = i >> 3;
      const int py = pp / PT, px = pp - py * PT;
      if (py0 + py >= g.Hp || px0 + px >= g.Wp) continue;
      half8v m = *reinterpret_cast<const half8v*>(conv + conv_off((2 * py) * CR + 2 * px, c8));
#pragma unroll
      for (int dy = 0; dy < PK; ++dy)
#pragma unroll
        for (int dx = 0; dx < PK; ++dx) {
          if (dy == 0 && dx == 0) continue;
          const half8v v = *reinterpret_cast<const half8v*>(conv + conv_off((2 * py + dy) * CR + 2 * px + dx, c8));
          m = __builtin_elementwise_max(m, v);
        }
      m = __builtin_elementwise_max(m + pb8, half8v{0, 0, 0, 0, 0, 0, 0, 0});
      *reinterpret_cast<half8v*>(y + (((size_t)b * g.Hp + py0 + py) * g.Wp + px0 + px) * 64 + c8 * 8) = m;
    }
    __syncthreads();   // conv tile reads done; patch(tnext) visible
    if (tnext >= g.ntiles) break;
    t = tnext;
  }
}

void stem_fused_launch(const uint8_t* img, const half_t* w, const float* bias, half_t* y, int B, int H, int W,
                       const long long* start_idx, long long start_off, long long max_start, long long sub,
                       hipStream_t st) {
  using namespace stem;
  StemGeom g;
  g.B = B;
  g.H = H;
  g.W = W;
  g.Hc = (H + 2 * CP - KH) / CS + 1;
  g.Wc = (W + 2 * CP - KH) / CS + 1;
  g.Hp = (g.Hc + 2 * PP - PK) / PS + 1;
  g.Wp = (g.Wc + 2 * PP - PK) / PS + 1;
  g.tiles_x = (g.Wp + PT - 1) / PT;
  g.tiles_y = (g.Hp + PT - 1) / PT;
  g.ntiles = B * g.tiles_x * g.tiles_y;
  g.ablate = g_stem_ablate;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_fused_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int grid = g.ntiles < 512 ? g.ntiles : 512;   // persistent: 2 workgroups per CU
  hipLaunchKernelGGL(stem_fused_kernel, dim3(grid), dim3(256), LDS, st, img, w, bias, y, g, start_idx, start_off, max_start, sub);
}

}  // namespace idunno
