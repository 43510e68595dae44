// Fused AlexNet stem in split fp16 (fp32-accurate): uint8 images -> normalise ->
// conv 11x11/4 pad 2 (3 -> 64) + bias -> ReLU -> max pool 3x3/2 -> split
// [B][27][27][128 halfs], in ONE persistent kernel (reference op chain:
// alexnet_resnet.py -> torchvision alexnet.features[0:3]).
//
// Replaces three passes of the round-5 split path: the packed-row preprocess
// (preprocess_pack3_split, 188 us at B = 500), the packed-row split conv
// (conv_glds P3, 482 us) and the max pool from its fp32 output (107 us) -- the
// 55x55x64 fp32 activation (387 MB at B = 500) and the ~800 MB packed-row
// operand never reach HBM (profiles/r6x_alexnet_b500_split_kernels.md).
//
// Exact-u8 form (as stem_split_kernel, stem_fused.hip): x = u * s_c + c_c with u
// the uint8 byte, so conv(x) = conv(w * s, u) + sum over the in-image taps of
// w * c.  u <= 255 is exact in fp16: the B operand has no lo part and every K
// step is two f16 MFMAs, w'_hi * u + w'_lo * u (w' = w * s scaled by 2^e, split
// into hi + lo halfs: 22-bit weights, exact products, f32 accumulation).  The c
// term of a conv output whose taps all lie inside the image is folded into the
// bias; the first and last conv row / column get a correction from 2D prefix
// sums of w * c over (kh, kw) (models/packed.py pack_alex_stem_split).
//
// K layout (17 steps of 32 = 8 pixels x 4 channels, channel 3 zero): step kh
// (0..10) holds taps kw 0..7 of kernel row kh; tail step 11 + t holds taps 8, 9
// and 10 (+ a zero tap) of rows 2t and 2t + 1 -- lane group q of a B fragment
// reads 16 contiguous bytes of ONE patch row (two pixels), so rows can be mixed
// within a step: 17 steps instead of 22 for 11 x 11 taps.
//
// Work item: a 4-row x 7-column tile of pooled outputs of one image = 9 conv rows
// x 15 conv columns.  Wave w owns couts 16w .. 16w+15 (A fragments of all 17
// steps, hi and lo, in 136 VGPRs for the whole launch) and computes all 9 conv
// rows as 9 independent accumulator chains (lane & 15 = conv column, lane 15 an
// unused column), so the pool is done in registers: horizontal 3-max by DPP row
// shifts, vertical 3-max across the accumulators.  The tile's uint8 patch
// (43 rows x 76 pixels) is prefetched into registers one tile ahead and staged in
// LDS as [row][pixel][4] fp16.
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

namespace astem {
constexpr int KH = 11, CS = 4, CP = 2;       // conv
constexpr int PK = 3, PS = 2;                // pool (no padding)
constexpr int PTX = 7, PTY = 4;              // pooled tile
constexpr int CRX = (PTX - 1) * PS + PK;     // 15 conv columns (lane 15 unused)
constexpr int CRY = (PTY - 1) * PS + PK;     // 9 conv rows
constexpr int IPR = (CRY - 1) * CS + KH;     // 43 patch rows
constexpr int XOFF = 2;                      // patch column of the first tap of conv column 0
constexpr int QPR = 19;                      // 4-pixel quads per patch row
constexpr int IPC = 4 * QPR;                 // 76 patch columns
constexpr int NQUAD = IPR * QPR;             // 817
constexpr int QPT = (NQUAD + 255) / 256;     // quads per thread (4)
constexpr int NKS = KH + (KH + 1) / 2;       // 17 K steps
constexpr int PATCH_BYTES = IPR * IPC * 8;   // 26144
static_assert(CRX <= 15, "one conv row per 16-lane fragment");
static_assert(4 * 15 + XOFF + 12 <= IPC, "every B read of lane 15 stays inside the patch row");
}  // namespace astem

struct AStemGeom {
  int B, H, W, Hc, Wc, Hp, Wp, tiles_x, tiles_y, ntiles;
  int aligned;                                 // W % 4 == 0 and a dword-aligned base: quads load as dwords
  int* ovf;
};

struct AQuads {
  uint32_t d[astem::QPT][3];
  bool ok[astem::QPT];
};

__device__ __forceinline__ void astem_tile(const AStemGeom& g, int t, int& b, int& py0, int& px0) {
  const int per = g.tiles_x * g.tiles_y;
  b = t / per;
  const int r = t - b * per;
  py0 = (r / g.tiles_x) * astem::PTY;
  px0 = (r % g.tiles_x) * astem::PTX;
}

// input patch origin of a tile: row of kernel row 0 of conv row 0, column of the
// patch's first pixel (a multiple of 4: 12-byte pixel quads are dword aligned)
__device__ __forceinline__ void astem_origin(int py0, int px0, int& iy0, int& ix0) {
  using namespace astem;
  iy0 = py0 * PS * CS - CP;
  ix0 = px0 * PS * CS - CP - XOFF;
}

__device__ __forceinline__ void astem_load(const uint8_t* __restrict__ img, const AStemGeom& g, int t, int tid,
                                           AQuads& q) {
  using namespace astem;
  int b, py0, px0, iy0, ix0;
  astem_tile(g, t, b, py0, px0);
  astem_origin(py0, px0, iy0, ix0);
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    q.ok[k] = false;
    q.d[k][0] = q.d[k][1] = q.d[k][2] = 0u;
    if (i >= NQUAD) continue;
    const int r = i / QPR, qc = i - r * QPR;
    const int iy = iy0 + r, ix = ix0 + 4 * qc;
    if ((unsigned)iy >= (unsigned)g.H || ix + 3 < 0 || ix >= g.W) continue;
    const uint8_t* p = img + (((size_t)b * g.H + iy) * g.W + ix) * 3;
    if (g.aligned && ix >= 0 && ix + 3 < g.W) {
      const uint32_t* pd = reinterpret_cast<const uint32_t*>(p);
      q.d[k][0] = pd[0];
      q.d[k][1] = pd[1];
      q.d[k][2] = pd[2];
    } else {                                           // ragged edge or unaligned rows: byte loads
      uint8_t v[12];
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const int x = ix + j / 3;
        v[j] = ((unsigned)x < (unsigned)g.W) ? p[j] : 0;
      }
      q.d[k][0] = v[0] | (v[1] << 8) | (v[2] << 16) | ((uint32_t)v[3] << 24);
      q.d[k][1] = v[4] | (v[5] << 8) | (v[6] << 16) | ((uint32_t)v[7] << 24);
      q.d[k][2] = v[8] | (v[9] << 8) | (v[10] << 16) | ((uint32_t)v[11] << 24);
    }
    q.ok[k] = true;
  }
}

// registers -> the patch in LDS as [row][pixel][r, g, b, 0] fp16 (bytes exact);
// pixels outside the image (and whole quads never loaded) are 0
__device__ __forceinline__ void astem_store(char* patch, int tid, const AQuads& q) {
  using namespace astem;
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    if (i >= NQUAD) continue;
    half8v o[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        const int byte = 3 * j + ch;
        o[j >> 1][4 * (j & 1) + ch] = (half_t)(float)((q.d[k][byte >> 2] >> (8 * (byte & 3))) & 0xFFu);
      }
      o[j >> 1][4 * (j & 1) + 3] = (half_t)0.f;
    }
    half8v* d = reinterpret_cast<half8v*>(patch + (size_t)i * 32);   // quad i = row r, pixels 4qc .. 4qc+3
    d[0] = o[0];
    d[1] = o[1];
  }
}

// the 9 B fragments of K step s: conv rows r = 0..8 (patch rows 4r + kh)
__device__ __forceinline__ void astem_read_b(const char* smem, int s, uint32_t mainb, uint32_t tailb, int trow,
                                             half8v* bf) {
  using namespace astem;
  int prow;
  uint32_t pcol;
  if (s < KH) {
    prow = s;
    pcol = mainb;
  } else {
    prow = min(2 * (s - KH) + trow, KH - 1);
    pcol = tailb;
  }
#pragma unroll
  for (int r = 0; r < CRY; ++r)
    bf[r] = *reinterpret_cast<const half8v*>(smem + (uint32_t)((CS * r + prow) * IPC) * 8u + pcol);
}

template <int N>
__device__ __forceinline__ float astem_shl(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x100 | N, 0xF, 0xF, true));
}

__global__ void __launch_bounds__(256, 1)
alex_stem_split_kernel(const uint8_t* __restrict__ img, const half_t* __restrict__ w, const float* __restrict__ bias,
                       const float* __restrict__ psum, float acc_scale, half_t* __restrict__ y, const AStemGeom g,
                       const long long* __restrict__ start_idx, long long start_off, long long max_start,
                       long long sub) {
  using namespace astem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (start_idx != nullptr) {                  // device-side window of an HBM-resident shard
    long long s = *start_idx - start_off;
    s = (s < 0 ? 0 : (s > max_start ? max_start : s)) + sub;
    img += (size_t)s * g.H * g.W * 3;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cx = lane & 15, fch = lane >> 4;
  int t = blockIdx.x;
  if (t >= g.ntiles) return;                   // uniform

  AQuads q;
  astem_load(img, g, t, tid, q);

  // A fragments: couts 16*wave + cx (rows of the fragment), K group fch, all steps
  half8v aH[NKS], aL[NKS];
  {
    const half_t* wr = w + (size_t)(16 * wave + cx) * (NKS * 32) + 8 * fch;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      aH[s] = *reinterpret_cast<const half8v*>(wr + s * 32);
      aL[s] = *reinterpret_cast<const half8v*>(wr + (size_t)64 * NKS * 32 + s * 32);
    }
  }
  const int c0 = 16 * wave + 4 * fch;          // this lane's 4 output channels
  const float4v bv = *reinterpret_cast<const float4v*>(bias + c0);
  const float inv_scale = 1.f / acc_scale;

  astem_store(smem, tid, q);
  __syncthreads();

  // per-lane patch byte offsets (conv row 0): main steps read pixels
  // 4cx + XOFF + 2fch (+1) of row kh; tail step t reads pixels 4cx + XOFF + 8 (fch 0, 2)
  // or + 10 (fch 1, 3) of row 2t (fch 0, 1) or 2t + 1 (fch 2, 3; row 11 holds zero
  // weights and reads row 10 instead, a finite value)
  const uint32_t mainb = (uint32_t)(4 * cx + XOFF + 2 * fch) * 8u;
  const uint32_t tailb = (uint32_t)(4 * cx + XOFF + 8 + 2 * (fch & 1)) * 8u;
  const int trow = fch >> 1;

  for (;;) {
    int b, py0, px0;
    astem_tile(g, t, b, py0, px0);
    float4v acc[CRY];
#pragma unroll
    for (int r = 0; r < CRY; ++r) acc[r] = float4v{0.f, 0.f, 0.f, 0.f};
    // B fragments double-buffered over K steps: step s + 1's 9 LDS reads are in flight
    // while step s's 18 MFMAs run (one wave per SIMD: nothing else hides their latency);
    // the hi products of all 9 rows go before the lo ones so no MFMA waits on the one before
    half8v bf[2][CRY];
    astem_read_b(smem, 0, mainb, tailb, trow, bf[0]);
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      if (s + 1 < NKS) astem_read_b(smem, s + 1, mainb, tailb, trow, bf[(s + 1) & 1]);
#pragma unroll
      for (int r = 0; r < CRY; ++r)
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aH[s], bf[s & 1][r], acc[r], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < CRY; ++r)
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aL[s], bf[s & 1][r], acc[r], 0, 0, 0);
      // keeps the scheduler from hoisting later steps' reads (it spilled when it did)
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();                           // every wave's patch reads of tile t are done
    // the next tile's patch loads go out now (not a tile ahead: the 136 A registers, 36
    // accumulators and 9 B fragments leave no room to hold them across the MFMA loop)
    // and land while this tile's epilogue runs
    const int tnext = t + gridDim.x;
    if (tnext < g.ntiles) astem_load(img, g, tnext, tid, q);

    // ---- epilogue of tile t, registers only ----
    const int cc = px0 * PS + cx;              // this lane's conv column
    int wlo = max(0, CP - CS * cc), whi = min(KH, g.W + CP - CS * cc);
#pragma unroll
    for (int r = 0; r < CRY; ++r) {
      const int cr = py0 * PS + r;
      const int hlo = max(0, CP - CS * cr), hhi = min(KH, g.H + CP - CS * cr);
      if ((hlo > 0 || hhi < KH || wlo > 0 || whi < KH) && cr < g.Hc && cc < g.Wc) {
        // border conv output: its out-of-image taps saw u = 0, not the zero of x:
        // add sum over the in-image taps of w * c minus the full sum in the bias
        const float4v s_hh = *reinterpret_cast<const float4v*>(psum + (hhi * 12 + whi) * 64 + c0);
        const float4v s_lh = *reinterpret_cast<const float4v*>(psum + (hlo * 12 + whi) * 64 + c0);
        const float4v s_hl = *reinterpret_cast<const float4v*>(psum + (hhi * 12 + wlo) * 64 + c0);
        const float4v s_ll = *reinterpret_cast<const float4v*>(psum + (hlo * 12 + wlo) * 64 + c0);
        const float4v s_ff = *reinterpret_cast<const float4v*>(psum + (KH * 12 + KH) * 64 + c0);
        acc[r] += (s_hh - s_lh - s_hl + s_ll - s_ff) * inv_scale;
      }
      // horizontal 3-max: lane cx holds max over conv columns cx .. cx+2
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = acc[r][e];
        acc[r][e] = fmaxf(v, fmaxf(astem_shl<1>(v), astem_shl<2>(v)));
      }
      __builtin_amdgcn_sched_barrier(0);       // one row's correction loads live at a time
    }
    const int px = cx >> 1;
    const int ox = px0 + px;
    const bool col_ok = !(cx & 1) && px < PTX && ox < g.Wp;
    bool bad = false;
#pragma unroll
    for (int py = 0; py < PTY; ++py) {
      const int oy = py0 + py;
      if (oy >= g.Hp) break;                   // uniform
      float4v m;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        m[e] = fmaxf(fmaxf(acc[2 * py][e], acc[2 * py + 1][e]), acc[2 * py + 2][e]);
        m[e] = fmaxf(m[e] * acc_scale + bv[e], 0.f);     // bias and ReLU commute with the max
      }
      if (col_ok) {
        constexpr float kMax = 65504.f;
        bad |= !(fabsf(m[0]) < kMax && fabsf(m[1]) < kMax && fabsf(m[2]) < kMax && fabsf(m[3]) < kMax);
        half4v h, l;
        split_f16x4(m, h, l);
        half_t* dst = y + (((size_t)b * g.Hp + oy) * g.Wp + ox) * 128 + split_off(c0);
        *reinterpret_cast<half4v*>(dst) = h;
        *reinterpret_cast<half4v*>(dst + 32) = l;
      }
    }
    if (bad && g.ovf != nullptr) *g.ovf = 1;
    if (tnext < g.ntiles) astem_store(smem, tid, q);
    __syncthreads();                           // tile tnext's patch is in LDS
    if (tnext >= g.ntiles) break;
    t = tnext;
  }
}

bool alex_stem_split_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum,
                            float acc_scale, half_t* y, int B, int H, int W, const long long* start_idx,
                            long long start_off, long long max_start, long long sub, int* ovf, hipStream_t st) {
  using namespace astem;
  AStemGeom g;
  g.ovf = ovf;
  g.B = B;
  g.H = H;
  g.W = W;
  g.aligned = W % 4 == 0 && (reinterpret_cast<uintptr_t>(img) & 3) == 0;
  g.Hc = (H + 2 * CP - KH) / CS + 1;
  g.Wc = (W + 2 * CP - KH) / CS + 1;
  g.Hp = (g.Hc - PK) / PS + 1;
  g.Wp = (g.Wc - PK) / PS + 1;
  if (g.Hp <= 0 || g.Wp <= 0) return false;
  g.tiles_x = (g.Wp + PTX - 1) / PTX;
  g.tiles_y = (g.Hp + PTY - 1) / PTY;
  g.ntiles = B * g.tiles_x * g.tiles_y;
  if (g.ntiles <= 0) return true;
  const int per = device_cu_count();          // one workgroup per CU (all 512 registers)
  const int grid = g.ntiles < per ? g.ntiles : per;
  hipLaunchKernelGGL(alex_stem_split_kernel, dim3(grid), dim3(256), PATCH_BYTES, st, img, w, bias, psum,
                     acc_scale, y, g, start_idx, start_off, max_start, sub);
  return true;
}

}  // namespace idunno
