// Fused ResNet stem: uint8 images -> normalise -> conv 7x7/2 (3->64, BN folded)
// -> ReLU -> max-pool 3x3/2 -> fp16 NHWC [B][Hp][Wp][64], in ONE persistent kernel.
//
// Replaces four separate passes of the unfused path (preprocess, the 7x7 conv,
// the 112x112x64 activation write + re-read, max-pool; reference op chain
// alexnet_resnet.py:57-75 -> torchvision resnet18.conv1/bn1/relu/maxpool).
// The conv activation (642 MB at B=400) never touches HBM.
//
// Work item = one 8-row x 7-column tile of pooled outputs of one image.  Its
// 17 x 15 conv outputs are 17 MFMA pixel fragments: fragment f = conv row f,
// lane&15 = conv column (lane 15 idle), so the C/D tile of
// v_mfma_f32_16x16x32_f16 has one conv row across each 16-lane DPP row.
// Workgroups are persistent (2 per CU); the 28 A-fragments (64 couts x K 7x32)
// are loaded into registers ONCE, then every tile
//   * takes its 39x38 uint8 input patch from registers prefetched one tile
//     earlier (12-byte aligned pixel quads), normalises it into LDS as
//     [row][col][4] fp16 (channel 3 = 0);
//   * runs the implicit GEMM M=17x16, N=64, K=7x32 — one K stage per kernel
//     row (8 taps x 4 ch; tap 7 and channel 3 have zero weights); each
//     B-fragment row is 16 contiguous, 16-byte-aligned bytes of the patch;
//   * does the pool's horizontal 3-max IN REGISTERS (two DPP row shifts of the
//     fp32 accumulators), so only the 7 pooled columns of each conv row are
//     written to LDS (2.2x fewer bytes than the full conv row);
//   * issues the global loads of the next-next patch, then finishes the pool
//     vertically (5 LDS rows per two pooled rows) with 16-byte stores.
// Bias + ReLU are applied after the max (both commute with it).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

namespace stem {
constexpr int KH = 7, CS = 2, CP = 3;       // conv
constexpr int PK = 3, PS = 2, PP = 1;       // pool
constexpr int PTX = 7, PTY = 8;             // pooled tile: 7 columns x 8 rows
constexpr int CRX = (PTX - 1) * PS + PK;    // 15 conv columns (<= 16 lanes)
constexpr int CRY = (PTY - 1) * PS + PK;    // 17 conv rows = pixel fragments
constexpr int IPR = (CRY - 1) * CS + KH;    // 39 patch rows
// LDS patch column of input-patch column c is c + PCO: every pixel of the 11
// loaded quads then has a slot (no range checks), the middle two pixels of a
// quad form one aligned 16-byte store, and B-fragment rows stay 16-byte aligned
constexpr int PCO = 4;
constexpr int IPC = 46;                     // >= 4*QPR + PCO - 3 + 1 and >= (16-1)*CS + 8 + PCO; even
constexpr int QPR = 11;                     // 4-pixel quads per patch row (44 px cover the 38 read)
constexpr int NQUAD = IPR * QPR;            // 429
constexpr int QPT = (NQUAD + 255) / 256;    // quads per thread (2)
constexpr int PATCH_BYTES = IPR * IPC * 8;  // 14352
constexpr int HP_BYTES = CRY * PTX * 128;   // [conv row][pooled col][64 ch] fp16 = 15232
constexpr int LDS = PATCH_BYTES + HP_BYTES;
constexpr int NVP = (PTY / 2) * PTX * 8;    // vertical-pool items: 2 pooled rows x 1 col x 8 ch (224)
static_assert(CRX <= 15, "one conv row per 16-lane fragment, lane 15 idle");
static_assert(NVP <= 256, "one vertical-pool item per thread");
static_assert(PCO >= 3 && 4 * (QPR - 1) + PCO < IPC, "every quad pixel has an LDS column");
static_assert((16 - 1) * CS + 8 + PCO <= IPC, "B-fragment rows stay inside the patch row");
static_assert(IPC % 2 == 0 && PCO % 2 == 0, "16-byte aligned B rows and middle-pair stores");
constexpr int NIW = 2;                      // 16-cout A fragments per wave (of 4)
constexpr int NCH = 4 / NIW;                // waves sharing each conv row
constexpr int WGS_MAX = 4;                  // workgroups per CU the registers allow
}  // namespace stem

// ToTensor + Normalize as x * s + c per channel: s = 1 / (255 std), c = -mean / std
typedef float float2v __attribute__((ext_vector_type(2)));
constexpr float kSR = 1.f / (255.f * 0.229f), kSG = 1.f / (255.f * 0.224f), kSB = 1.f / (255.f * 0.225f);
constexpr float kCR = -0.485f / 0.229f, kCG = -0.456f / 0.224f, kCB = -0.406f / 0.225f;
#define kScaleRG (float2v{kSR, kSG})
#define kShiftRG (float2v{kCR, kCG})
#define kScaleBB (float2v{kSB, kSB})
#define kShiftBB (float2v{kCB, kCB})

// Byte offset of 16-byte channel chunk c (0..7) of (conv row r, pooled col px)
// in the LDS tile.  Rows of 128 B; the chunk is XOR-swizzled by px so the
// epilogue's 8-byte writes (7 pooled columns of one chunk) spread over banks.
__device__ __forceinline__ int hp_off(int r, int px, int c) { return (r * stem::PTX + px) * 128 + ((c ^ px) << 4); }

struct StemGeom {
  int B, H, W, Hc, Wc, Hp, Wp, tiles_x, tiles_y, ntiles;
  int* ovf;     // stem_split: split range guard flag or nullptr (common.h split_guard)
};

// Round-1/2 ablation switches (tools/stem_ablate.py measurements, docs/KERNELS.md) are
// compiled out: the bit tests below fold to "no ablation".
constexpr int kStemAblate = 0;
// persistent workgroups per CU (A/B knob)

struct Quads {
  uint32_t d[stem::QPT][3];
  bool ok[stem::QPT];
};

__device__ __forceinline__ void tile_coords(const StemGeom& g, int t, int& b, int& py0, int& px0) {
  const int per = g.tiles_x * g.tiles_y;
  b = t / per;
  const int r = t - b * per;
  py0 = (r / g.tiles_x) * stem::PTY;
  px0 = (r % g.tiles_x) * stem::PTX;
}

// global -> registers: this thread's quads of tile t's input patch
__device__ __forceinline__ void load_quads(const uint8_t* __restrict__ img, const StemGeom& g, int t, int tid,
                                           Quads& q) {
  using namespace stem;
  int b, py0, px0;
  tile_coords(g, t, b, py0, px0);
  const int iy0 = (py0 * PS - PP) * CS - CP;
  const int ixa = (px0 * PS - PP) * CS - CP - 3;     // 4px0 - 8: a multiple of 4 -> 12-byte quads 4-byte aligned
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
      const uint32_t* pd = reinterpret_cast<const uint32_t*>(p);
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
    // byte -> f32 (v_cvt_f32_ubyteN), x * s + c on f32 pairs (v_pk_fma_f32),
    // pairs -> packed fp16: ~26 VALU per quad of 4 pixels
    float f[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) f[j] = (float)((q.d[k][j >> 2] >> (8 * (j & 3))) & 0xFFu);
    const float2v b01 = float2v{f[2], f[5]} * kScaleBB + kShiftBB;
    const float2v b23 = float2v{f[8], f[11]} * kScaleBB + kShiftBB;
    const float bl[4] = {b01[0], b01[1], b23[0], b23[1]};
    half4v px[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float2v rg = float2v{f[3 * j], f[3 * j + 1]} * kScaleRG + kShiftRG;
      const half2v lo = {(half_t)rg[0], (half_t)rg[1]};     // v_cvt_pk_f16_f32
      const half2v hi = {(half_t)bl[j], (half_t)0.f};
      px[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
    }
    const int x0 = ixa + 4 * qc;
    if (!(q.ok[k] && x0 >= 0 && x0 + 3 < g.W)) {       // image edge: zero the pixels outside
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (!q.ok[k] || (unsigned)(x0 + j) >= (unsigned)g.W) px[j] = half4v{0, 0, 0, 0};
    }
    // pixel j -> LDS column 4qc + j - 3 + PCO: 8 + 16 + 8 bytes
    char* d = patch + (r * IPC + 4 * qc + PCO - 3) * 8;
    *reinterpret_cast<half4v*>(d) = px[0];
    *reinterpret_cast<half8v*>(d + 8) = __builtin_shufflevector(px[1], px[2], 0, 1, 2, 3, 4, 5, 6, 7);
    *reinterpret_cast<half4v*>(d + 24) = px[3];
  }
}

// packed fp16 pair of lane l + N of the same 16-lane row (DPP row_shl:N; lanes
// past the row read 0 -- only lanes cx <= 12 are consumed)
template <int N>
__device__ __forceinline__ half2v row_shl_h2(half2v v) {
  return __builtin_bit_cast(half2v, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x100 | N, 0xF, 0xF, true));
}

__global__ void __launch_bounds__(256, stem::WGS_MAX)
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
  char* hp = smem + PATCH_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  int t = blockIdx.x;
  if (t >= g.ntiles) return;   // whole workgroup exits together (uniform)

  Quads q;
  load_quads(img, g, t, tid, q);

  // ---- A fragments (weights [cout][kh][32]) straight into registers, once ----
  const int frow = lane & 15, fch = lane >> 4;
  const int ch0 = (wave % NCH) * NIW;   // first 16-cout fragment of this wave
  half8v fa[KH][NIW];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int i = 0; i < NIW; ++i)
      fa[kh][i] = *reinterpret_cast<const half8v*>(w + (size_t)((ch0 + i) * 16 + frow) * (KH * 32) + kh * 32 + fch * 8);
  // bias + ReLU after the max-pool, once per pooled output; each pooling
  // thread owns one fixed 8-channel chunk
  half8v pb8;
#pragma unroll
  for (int j = 0; j < 8; ++j) pb8[j] = (half_t)bias[(tid & 7) * 8 + j];

  store_patch(patch, g, t, tid, q);
  int tn = t + gridDim.x;
  if (tn < g.ntiles) load_quads(img, g, tn, tid, q);
  __syncthreads();

  // vertical-pool item of this thread: chunk c8, pooled column vpx, pooled rows 2*vpy2 and 2*vpy2+1
  const int c8 = tid & 7, vpx = (tid >> 3) % PTX, vpy2 = tid / (8 * PTX);
  const int cx = frow;   // conv column of this lane in every fragment

  // nothing issued above may stay in flight into the tile loop: the waitcnt pass puts
  // the first-use waits of the A fragments / pool bias inside the loop, where from the
  // second tile on they wait for the next patch's loads and the last tile's output
  // stores instead (alex_stem.hip has the measurement)
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  while (true) {
    int b, py0, px0;
    tile_coords(g, t, b, py0, px0);
    const int oy0 = py0 * PS - PP, ox0 = px0 * PS - PP;
    const bool colv = cx < CRX && (unsigned)(ox0 + cx) < (unsigned)g.Wc;
    const bool interior = ox0 >= 0 && ox0 + CRX <= g.Wc;   // no column of this tile needs masking

    // ---- conv GEMM, one conv row per fragment, round-robin over 4 waves ------
    for (int f = wave / NCH; f < CRY; f += 4 / NCH) {
      const char* pb = patch + ((2 * f) * IPC + 2 * cx + 2 * fch + PCO) * 8;
      float4v acc[NIW];
#pragma unroll
      for (int i = 0; i < NIW; ++i) acc[i] = float4v{0.f, 0.f, 0.f, 0.f};
      if (!(kStemAblate & 2)) {
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          const half8v fb = *reinterpret_cast<const half8v*>(pb + kh * IPC * 8);
#pragma unroll
          for (int i = 0; i < NIW; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[kh][i], fb, acc[i], 0, 0, 0);
        }
      }
      // lane = (conv column cx; couts i*16 + fch*4 + r).  Outside the image the
      // conv output is the pool's -inf padding (-65504); the 3-wide horizontal
      // max takes lanes cx+1, cx+2 of the same DPP row, on packed fp16 pairs
      // (VALU issue is this phase's cost: 4 cycles per wave instruction).
      if (kStemAblate & 8) continue;
      half4v o[NIW];
      if ((unsigned)(oy0 + f) < (unsigned)g.Hc) {          // wave-uniform
#pragma unroll
        for (int i = 0; i < NIW; ++i) {
          half2v p0 = {(half_t)acc[i][0], (half_t)acc[i][1]};
          half2v p1 = {(half_t)acc[i][2], (half_t)acc[i][3]};
          if (!interior && !colv) p0 = p1 = half2v{(half_t)-65504.f, (half_t)-65504.f};
          // llvm.maximum (NaN-propagating) lowers to one v_pk_maximum3_f16 and
          // needs no canonicalising max(x, x) of the DPP results, unlike maxnum
          p0 = __builtin_elementwise_maximum(p0, __builtin_elementwise_maximum(row_shl_h2<1>(p0), row_shl_h2<2>(p0)));
          p1 = __builtin_elementwise_maximum(p1, __builtin_elementwise_maximum(row_shl_h2<1>(p1), row_shl_h2<2>(p1)));
          o[i] = half4v{p0[0], p0[1], p1[0], p1[1]};
        }
      } else {
#pragma unroll
        for (int i = 0; i < NIW; ++i) o[i] = half4v{(half_t)-65504.f, (half_t)-65504.f, (half_t)-65504.f, (half_t)-65504.f};
      }
      if (!(cx & 1) && cx < 2 * PTX) {
        const int px = cx >> 1;
#pragma unroll
        for (int i = 0; i < NIW; ++i)
          *reinterpret_cast<half4v*>(hp + hp_off(f, px, 2 * (ch0 + i) + (fch >> 1)) + (fch & 1) * 8) = o[i];
      }
    }
    __syncthreads();   // pooled-column tile complete; patch(t) no longer read

    const int tnext = tn;
    if (tnext < g.ntiles) {
      if (!(kStemAblate & 4)) store_patch(patch, g, tnext, tid, q);   // uses the quads prefetched one tile ago
      tn = tnext + gridDim.x;
      if (tn < g.ntiles && !(kStemAblate & 16)) load_quads(img, g, tn, tid, q);
    }

    // ---- vertical 3-max over conv rows 4*vpy2 .. 4*vpy2+4 -> 2 pooled rows ----
    if (tid < NVP && !(kStemAblate & 1)) {
      const int r0 = 4 * vpy2;
      const half8v a0 = *reinterpret_cast<const half8v*>(hp + hp_off(r0 + 0, vpx, c8));
      const half8v a1 = *reinterpret_cast<const half8v*>(hp + hp_off(r0 + 1, vpx, c8));
      const half8v a2 = *reinterpret_cast<const half8v*>(hp + hp_off(r0 + 2, vpx, c8));
      const half8v a3 = *reinterpret_cast<const half8v*>(hp + hp_off(r0 + 3, vpx, c8));
      const half8v a4 = *reinterpret_cast<const half8v*>(hp + hp_off(r0 + 4, vpx, c8));
      const half8v zero = {0, 0, 0, 0, 0, 0, 0, 0};
      half8v lo = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a0, a1), a2);
      half8v hi = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a2, a3), a4);
      lo = __builtin_elementwise_maximum(lo + pb8, zero);
      hi = __builtin_elementwise_maximum(hi + pb8, zero);
      const int ox = px0 + vpx, oy = py0 + 2 * vpy2;
      if (ox < g.Wp) {
        half_t* dst = y + (((size_t)b * g.Hp + oy) * g.Wp + ox) * 64 + c8 * 8;
        if (oy < g.Hp) *reinterpret_cast<half8v*>(dst) = lo;
        if (oy + 1 < g.Hp) *reinterpret_cast<half8v*>(dst + (size_t)g.Wp * 64) = hi;
      }
    }
    __syncthreads();   // tile reads done; patch(tnext) visible
    if (tnext >= g.ntiles) break;
    t = tnext;
  }
}

void stem_fused_launch(const uint8_t* img, const half_t* w, const float* bias, half_t* y, int B, int H, int W,
                       const long long* start_idx, long long start_off, long long max_start, long long sub,
                       hipStream_t st) {
  using namespace stem;
  StemGeom g{};
  g.B = B;
  g.H = H;
  g.W = W;
  g.Hc = (H + 2 * CP - KH) / CS + 1;
  g.Wc = (W + 2 * CP - KH) / CS + 1;
  g.Hp = (g.Hc + 2 * PP - PK) / PS + 1;
  g.Wp = (g.Wc + 2 * PP - PK) / PS + 1;
  g.tiles_x = (g.Wp + PTX - 1) / PTX;
  g.tiles_y = (g.Hp + PTY - 1) / PTY;
  g.ntiles = B * g.tiles_x * g.tiles_y;
  const int ncu = device_cu_count();   // per device (launch_util.h)
  const int per = stem::WGS_MAX * ncu;   // persistent: WGS_MAX workgroups per CU
  const int grid = g.ntiles < per ? g.ntiles : per;
  hipLaunchKernelGGL(stem_fused_kernel, dim3(grid), dim3(256), LDS, st, img, w, bias, y, g, start_idx, start_off,
                     max_start, sub);
}

// ============================================================================
// Split-fp16 (fp32-accurate) fused stem: same tiling as stem_fused_kernel, for
// the fp32 programs.  Exact-u8 formulation: the normalised input is
// x = u * s_c + c_c (u the uint8 byte, s_c = 1/(255 std_c), c_c = -mean_c/std_c),
// so conv(x) = conv'(u) + C(oy, ox) with w' = w * s_c and C the sum of
// w * c_c over the taps that fall inside the image.  u is an integer <= 255 and
// therefore EXACT in fp16: the B operand needs no lo part, and each K stage is
// w'_hi*u + w'_lo*u -- 2 f16 MFMAs instead of 3, one patch plane instead of two,
// and the patch store is a byte -> half conversion.  C(oy, ox) is the bias for
// interior pixels (host-folded) plus a border delta from a 2D prefix-sum table
// of w * c over (kh, kw), added to the accumulators before the max pool (it
// depends on the position).  Then as before: DPP horizontal 3-max on the f32
// accumulators, f32 LDS vertical 3-max, x 2^-e, + bias, ReLU, split store
// [B][Hp][Wp][128 halfs].  Replaces preprocess_pack3_split + conv2d_pack3_split
// + maxpool_split (three passes over ~3 GB at B = 400).
namespace stem_s {
constexpr int HP_BYTES = stem::CRY * stem::PTX * 256;     // [conv row][pooled col][64 ch] f32 = 30464
constexpr int LDS = stem::PATCH_BYTES + HP_BYTES;         // 44816
}  // namespace stem_s
// Stem variants measured and dropped (deleted in round 5): two 16-cout fragments per
// wave (461 vs 399 us at B = 400, profiles/r2_v28_stem_split_u8.md), one / three conv
// rows per pass (-0.86 % / -0.7 % whole graph vs two, profiles/r3_stem_split_rp2.md),
// a register-pooled kernel (-0.1 ... -0.5 %).

// f32 tile offset of 4-channel chunk c (0..15) of (conv row r, pooled col px),
// chunk XOR-swizzled by px
__device__ __forceinline__ int hp32_off(int r, int px, int c) { return (r * stem::PTX + px) * 256 + ((c ^ px) << 4); }

// registers -> u8 values as fp16 in LDS ([row][col][4], channel 3 and
// out-of-image pixels 0)
__device__ __forceinline__ void store_patch_u8(char* patch, const StemGeom& g, int t, int tid, const Quads& q) {
  using namespace stem;
  int b, py0, px0;
  tile_coords(g, t, b, py0, px0);
  const int ixa = (px0 * PS - PP) * CS - CP - 3;
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    if (i >= NQUAD) continue;
    const int r = i / QPR, qc = i - r * QPR;
    const int x0 = ixa + 4 * qc;
    const bool edge = !(q.ok[k] && x0 >= 0 && x0 + 3 < g.W);
    half4v px[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) px[j][ch] = (half_t)(float)((q.d[k][(3 * j + ch) >> 2] >> (8 * ((3 * j + ch) & 3))) & 0xFFu);
      px[j][3] = (half_t)0.f;
      if (edge && (!q.ok[k] || (unsigned)(x0 + j) >= (unsigned)g.W)) px[j] = half4v{0, 0, 0, 0};
    }
    char* d = patch + (r * IPC + 4 * qc + PCO - 3) * 8;
    *reinterpret_cast<half4v*>(d) = px[0];
    *reinterpret_cast<half8v*>(d + 8) = __builtin_shufflevector(px[1], px[2], 0, 1, 2, 3, 4, 5, 6, 7);
    *reinterpret_cast<half4v*>(d + 24) = px[3];
  }
}

// f32 of lane l + N of the same 16-lane row (DPP row_shl:N)
template <int N>
__device__ __forceinline__ float row_shl_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x100 | N, 0xF, 0xF, true));
}

// valid kernel-tap range [lo, hi) of conv output coordinate o (stride 2, pad 3)
__device__ __forceinline__ void tap_range(int o, int n, int& lo, int& hi) {
  lo = max(0, stem::CP - stem::CS * o);
  hi = min(stem::KH, n + stem::CP - stem::CS * o);
}

// NIWS: 16-cout A fragments per wave (2: two waves share a conv row, 2
// workgroups per CU by registers; 1: every wave takes all rows for its 16
// couts, half the A registers, 3 workgroups per CU)
// RP: conv rows per pass (2, 3: interleaved MFMA chains; NIWS 1 only)
// F16: the fp16 programs' stem in the same exact-u8 form -- only the hi
// MFMA (w' rounded to fp16 once; the input u is exact, unlike the normalised
// fp16 input of stem_fused_kernel) and a plain fp16 [B][Hp][Wp][64] output
template <int NIWS, int RP = 1, bool F16 = false, bool PREWAIT = true>
__global__ void __launch_bounds__(256, NIWS == 1 ? 3 : 2)
stem_split_kernel(const uint8_t* __restrict__ img, const half_t* __restrict__ w, const float* __restrict__ bias,
                  const float* __restrict__ psum, float acc_scale, half_t* __restrict__ y, const StemGeom g,
                  const long long* __restrict__ start_idx, long long start_off, long long max_start, long long sub) {
  using namespace stem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (start_idx != nullptr) {
    long long s = *start_idx - start_off;
    s = (s < 0 ? 0 : (s > max_start ? max_start : s)) + sub;
    img += (size_t)s * g.H * g.W * 3;
  }
  char* patch = smem;
  char* hp = smem + PATCH_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  int t = blockIdx.x;
  if (t >= g.ntiles) return;   // whole workgroup exits together (uniform)

  Quads q;
  load_quads(img, g, t, tid, q);

  // ---- A fragments: hi and lo of w' = w * s_c, [2][cout][kh][32], registers, once ----
  constexpr int NIW = NIWS, NCH = 4 / NIWS;
  static_assert(RP == 1 || NIWS == 1, "two rows per pass: one cout fragment per wave");
  static_assert(RP == 1 || ((2 * (RP * ((CRY + RP - 1) / RP) - 1) + KH - 1) * IPC + 2 * 15 + 2 * 3 + PCO) * 8 + 16 <=
                                stem_s::LDS, "dropped rows inside LDS");
  const int frow = lane & 15, fch = lane >> 4;
  const int ch0 = (wave % NCH) * NIW;
  half8v fah[KH][NIW], fal[KH][NIW];
#pragma unroll
  for (int kh = 0; kh < KH; ++kh)
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const size_t o = (size_t)((ch0 + i) * 16 + frow) * (KH * 32) + kh * 32 + fch * 8;
      fah[kh][i] = *reinterpret_cast<const half8v*>(w + o);
      if constexpr (!F16) fal[kh][i] = *reinterpret_cast<const half8v*>(w + 64 * KH * 32 + o);
    }
  const float inv_scale = 1.f / acc_scale;           // 2^e: border deltas in accumulator units

  store_patch_u8(patch, g, t, tid, q);
  int tn = t + gridDim.x;
  if (tn < g.ntiles) load_quads(img, g, tn, tid, q);
  __syncthreads();

  // vertical-pool item: 8-channel chunk c8, pooled column vpx, pooled rows 2*vpy2, 2*vpy2+1
  const int c8 = tid & 7, vpx = (tid >> 3) % PTX, vpy2 = tid / (8 * PTX);
  float4v pb0 = float4v{0.f, 0.f, 0.f, 0.f}, pb1 = pb0;
  if (tid < NVP) {
    pb0 = *reinterpret_cast<const float4v*>(bias + c8 * 8);
    pb1 = *reinterpret_cast<const float4v*>(bias + c8 * 8 + 4);
  }
  const int cx = frow;

  // nothing issued above may stay in flight into the tile loop: the waitcnt pass puts
  // the first-use waits of the A fragments / pool bias inside the loop, where from the
  // second tile on they wait for the next patch's loads and the last tile's output
  // stores instead (alex_stem.hip has the measurement)
  if (PREWAIT) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
  while (true) {
    int b, py0, px0;
    tile_coords(g, t, b, py0, px0);
    const int oy0 = py0 * PS - PP, ox0 = px0 * PS - PP;
    const bool colv = cx < CRX && (unsigned)(ox0 + cx) < (unsigned)g.Wc;
    const bool interior = ox0 >= 0 && ox0 + CRX <= g.Wc;
    // conv columns of this lane whose taps leave the image: border delta needed
    int wlo, whi;
    tap_range(ox0 + cx, g.W, wlo, whi);
    const bool colb = wlo > 0 || whi < KH;
    // the delta of an interior row (all 7 kh taps valid) depends on the column
    // only: S(7, whi) - S(7, wlo) - S(7, 7) (S(0, .) = 0), loaded once per tile
    // instead of 5 dependent global loads in every conv row of an edge tile
    float4v colcorr[NIW];
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      colcorr[i] = float4v{0.f, 0.f, 0.f, 0.f};
      if (colb) {
        const int co = (ch0 + i) * 16 + fch * 4;
        const float4v s_h = *reinterpret_cast<const float4v*>(psum + (7 * 8 + whi) * 64 + co);
        const float4v s_l = *reinterpret_cast<const float4v*>(psum + (7 * 8 + wlo) * 64 + co);
        const float4v s_f = *reinterpret_cast<const float4v*>(psum + (7 * 8 + 7) * 64 + co);
        colcorr[i] = (s_h - s_l - s_f) * inv_scale;
      }
    }

    // conv row f's epilogue: border delta, horizontal 3-max, f32 tile store
    auto row_epi = [&](int f, float4v (&acc)[NIW]) {
      const int oy = oy0 + f;
      const bool rowv = (unsigned)oy < (unsigned)g.Hc;    // wave-uniform
      int hlo, hhi;
      tap_range(oy, g.H, hlo, hhi);
      const bool rowb = hlo > 0 || hhi < KH;              // wave-uniform
      if (rowv && !rowb && colb) {
#pragma unroll
        for (int i = 0; i < NIW; ++i) acc[i] += colcorr[i];
      } else if (rowv && rowb) {
        // border pixel: add (sum of w*c over its valid taps) - (the full sum in
        // the bias), from the 2D prefix sums psum[kh][kw][64] (kh, kw in 0..7)
#pragma unroll
        for (int i = 0; i < NIW; ++i) {
          const int co = (ch0 + i) * 16 + fch * 4;
          const float4v s_hh = *reinterpret_cast<const float4v*>(psum + (hhi * 8 + whi) * 64 + co);
          const float4v s_lh = *reinterpret_cast<const float4v*>(psum + (hlo * 8 + whi) * 64 + co);
          const float4v s_hl = *reinterpret_cast<const float4v*>(psum + (hhi * 8 + wlo) * 64 + co);
          const float4v s_ll = *reinterpret_cast<const float4v*>(psum + (hlo * 8 + wlo) * 64 + co);
          const float4v s_ff = *reinterpret_cast<const float4v*>(psum + (7 * 8 + 7) * 64 + co);
          acc[i] += (s_hh - s_lh - s_hl + s_ll - s_ff) * inv_scale;
        }
      }
      // horizontal 3-max on the f32 accumulators; outside the image the conv
      // output is the pool's -inf padding
      float4v o[NIW];
#pragma unroll
      for (int i = 0; i < NIW; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[i][e];
          if (!rowv || (!interior && !colv)) v = -INFINITY;
          o[i][e] = fmaxf(v, fmaxf(row_shl_f32<1>(v), row_shl_f32<2>(v)));
        }
      }
      if (!(cx & 1) && cx < 2 * PTX) {
        const int px = cx >> 1;
#pragma unroll
        for (int i = 0; i < NIW; ++i)
          *reinterpret_cast<float4v*>(hp + hp32_off(f, px, 4 * (ch0 + i) + fch)) = o[i];
      }
    };
    if constexpr (RP > 1) {
      // RP conv rows per pass, their MFMA chains interleaved (each MFMA depends
      // on the one RP back, not the one before); rows past the tile (their patch
      // rows stay inside the LDS allocation) are computed and dropped
      for (int f = 0; f < CRY; f += RP) {
        const char* pa = patch + ((2 * f) * IPC + 2 * cx + 2 * fch + PCO) * 8;
        float4v acc[RP][1];
#pragma unroll
        for (int r = 0; r < RP; ++r) acc[r][0] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          if (kStemAblate & 2) break;
          half8v bq[RP];
#pragma unroll
          for (int r = 0; r < RP; ++r) bq[r] = *reinterpret_cast<const half8v*>(pa + (r * 2 * IPC + kh * IPC) * 8);
#pragma unroll
          for (int r = 0; r < RP; ++r) acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[kh][0], bq[r], acc[r][0], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < RP; ++r)
            if constexpr (!F16) acc[r][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[kh][0], bq[r], acc[r][0], 0, 0, 0);
        }
        if (kStemAblate & 8) continue;
        row_epi(f, acc[0]);
#pragma unroll
        for (int r = 1; r < RP; ++r)
          if (f + r < CRY) row_epi(f + r, acc[r]);
      }
    } else {
      for (int f = wave / NCH; f < CRY; f += 4 / NCH) {
        const char* pb = patch + ((2 * f) * IPC + 2 * cx + 2 * fch + PCO) * 8;
        float4v acc[NIW];
#pragma unroll
        for (int i = 0; i < NIW; ++i) acc[i] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          if (kStemAblate & 2) break;
          const half8v bu = *reinterpret_cast<const half8v*>(pb + kh * IPC * 8);
#pragma unroll
          for (int i = 0; i < NIW; ++i) {
            acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fah[kh][i], bu, acc[i], 0, 0, 0);
            if constexpr (!F16) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fal[kh][i], bu, acc[i], 0, 0, 0);
          }
        }
        if (kStemAblate & 8) continue;
        row_epi(f, acc);
      }
    }
    __syncthreads();   // pooled-column tile complete; patch(t) no longer read

    const int tnext = tn;
    if (tnext < g.ntiles) {
      if (!(kStemAblate & 4)) store_patch_u8(patch, g, tnext, tid, q);
      tn = tnext + gridDim.x;
      if (tn < g.ntiles && !(kStemAblate & 16)) load_quads(img, g, tn, tid, q);
    }

    // ---- vertical 3-max over conv rows 4*vpy2 .. 4*vpy2+4 -> 2 pooled rows ----
    if (tid < NVP && !(kStemAblate & 1)) {
      const int r0 = 4 * vpy2;
      float4v a[5][2];
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        a[r][0] = *reinterpret_cast<const float4v*>(hp + hp32_off(r0 + r, vpx, 2 * c8));
        a[r][1] = *reinterpret_cast<const float4v*>(hp + hp32_off(r0 + r, vpx, 2 * c8 + 1));
      }
      const int ox = px0 + vpx, oyp = py0 + 2 * vpy2;
      if (ox < g.Wp) {
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) {
          if (oyp + hr >= g.Hp) break;
          const int rr = 2 * hr;
          float4v m0, m1;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            m0[e] = fmaxf(fmaxf(a[rr][0][e], a[rr + 1][0][e]), a[rr + 2][0][e]);
            m1[e] = fmaxf(fmaxf(a[rr][1][e], a[rr + 1][1][e]), a[rr + 2][1][e]);
            m0[e] = fmaxf(m0[e] * acc_scale + pb0[e], 0.f);
            m1[e] = fmaxf(m1[e] * acc_scale + pb1[e], 0.f);
          }
          if constexpr (F16) {
            half8v o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              o[e] = (half_t)m0[e];
              o[4 + e] = (half_t)m1[e];
            }
            *reinterpret_cast<half8v*>(y + (((size_t)b * g.Hp + oyp + hr) * g.Wp + ox) * 64 + 8 * c8) = o;
          } else {
            split_guard(g.ovf, m0);
            split_guard(g.ovf, m1);
            half4v h0, l0, h1, l1;
            split_f16x4(m0, h0, l0);
            split_f16x4(m1, h1, l1);
            half_t* dst = y + (((size_t)b * g.Hp + oyp + hr) * g.Wp + ox) * 128 + split_off(8 * c8);
            *reinterpret_cast<half8v*>(dst) = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
            *reinterpret_cast<half8v*>(dst + 32) = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
          }
        }
      }
    }
    __syncthreads();   // tile reads done; patch(tnext) visible
    if (tnext >= g.ntiles) break;
    t = tnext;
  }
}

static int g_stem_prewait = 1;
void set_stem_prewait(bool on) { g_stem_prewait = on; }

void stem_split_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum, float acc_scale,
                       half_t* y, int B, int H, int W, const long long* start_idx, long long start_off,
                       long long max_start, long long sub, int* ovf, hipStream_t st) {
  using namespace stem;
  StemGeom g;
  g.ovf = ovf;
  g.B = B;
  g.H = H;
  g.W = W;
  g.Hc = (H + 2 * CP - KH) / CS + 1;
  g.Wc = (W + 2 * CP - KH) / CS + 1;
  g.Hp = (g.Hc + 2 * PP - PK) / PS + 1;
  g.Wp = (g.Wc + 2 * PP - PK) / PS + 1;
  g.tiles_x = (g.Wp + PTX - 1) / PTX;
  g.tiles_y = (g.Hp + PTY - 1) / PTY;
  g.ntiles = B * g.tiles_x * g.tiles_y;
  const int per = 3 * device_cu_count();
  const int grid = g.ntiles < per ? g.ntiles : per;
  auto k = g_stem_prewait ? stem_split_kernel<1, 2> : stem_split_kernel<1, 2, false, false>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), stem_s::LDS, st, img, w, bias,
                     psum, acc_scale, y, g, start_idx, start_off, max_start, sub);
}

// fp16 programs: the exact-u8 stem, hi MFMA only, fp16 [B][Hp][Wp][64] out
void stem_u8_f16_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum, float acc_scale,
                        half_t* y, int B, int H, int W, const long long* start_idx, long long start_off,
                        long long max_start, long long sub, hipStream_t st) {
  using namespace stem;
  StemGeom g;
  g.ovf = nullptr;
  g.B = B;
  g.H = H;
  g.W = W;
  g.Hc = (H + 2 * CP - KH) / CS + 1;
  g.Wc = (W + 2 * CP - KH) / CS + 1;
  g.Hp = (g.Hc + 2 * PP - PK) / PS + 1;
  g.Wp = (g.Wc + 2 * PP - PK) / PS + 1;
  g.tiles_x = (g.Wp + PTX - 1) / PTX;
  g.tiles_y = (g.Hp + PTY - 1) / PTY;
  g.ntiles = B * g.tiles_x * g.tiles_y;
  const int per = 3 * device_cu_count();
  const int grid = g.ntiles < per ? g.ntiles : per;
  hipLaunchKernelGGL(HIP_KERNEL_NAME(stem_split_kernel<1, 2, true>), dim3(grid), dim3(256), stem_s::LDS, st, img, w,
                     bias, psum, acc_scale, y, g, start_idx, start_off, max_start, sub);
}

}  // namespace idunno
