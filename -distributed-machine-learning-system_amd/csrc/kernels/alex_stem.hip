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
// x 15 conv columns.  Wave w owns couts 16w .. 16w+15 and computes all 9 conv rows
// as 9 independent accumulator chains (lane & 15 = conv column, lane 15 an unused
// column), so the pool is done in registers: horizontal 3-max by DPP row shifts,
// vertical 3-max across the accumulators.  The tile's uint8 patch (43 rows x 76
// pixels) is staged in LDS as [row][pixel][4] fp16; the border prefix sums live in
// LDS too.
//
// Two forms (set_astem_variant; B = 500, tools/astem_ablate.py):
//   alex_stem_split_kernel   one 256-thread workgroup per CU, A hi + lo in 136 VGPRs,
//                            accumulators in AGPRs, patch loads one tile ahead:
//                            MFMA loop, staging and epilogue run back to back
//                            (~305 us);
//   alex_stem_split_kernel2  (default) one 512-thread workgroup = two halves whose
//                            MFMA loops and epilogue/staging phases alternate, so
//                            each SIMD interleaves one wave's MFMAs with the other's
//                            VALU work (~230 us; AlexNet b500 forward -3.8 %).
//                            A lo moves to LDS to fit 256 registers a wave.
// The waitcnt lesson of both: nothing issued before the tile loop may stay in
// flight into it (vmcnt(0) ahead of the loop), or the loop's first-use waits on it
// turn into waits on the next patch's loads from the second tile on.
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
constexpr int PSUM_FLOATS = (KH + 1) * (KH + 1) * 64;   // border prefix sums [12][12][64] f32
constexpr int LDS_BYTES = PATCH_BYTES + PSUM_FLOATS * 4; // 62,1xx B: one workgroup per CU anyway
static_assert(PATCH_BYTES % 16 == 0, "float4 prefix-sum reads");
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

// two uint8 of a pixel quad -> two exact fp16 values: v_perm_b32 builds the halves
// 0x64XX = 1024 + XX (byte selectors 4..7 pick the 0x64 bytes of the constant, 0x0C a
// zero byte), one packed subtract of 1024 leaves XX exactly.  17 VALU per quad instead
// of a convert-to-f32, convert-to-f16 and pack per byte (~30)
typedef uint32_t uint4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t astem_h2(uint32_t v) {
  half2v h = __builtin_bit_cast(half2v, v) - half2v{(_Float16)1024.f, (_Float16)1024.f};
  return __builtin_bit_cast(uint32_t, h);
}

// registers -> the patch in LDS as [row][pixel][r, g, b, 0] fp16 (bytes exact);
// pixels outside the image (and whole quads never loaded) hold 0 bytes -> 0
__device__ __forceinline__ void astem_store(char* patch, int tid, const AQuads& q) {
  using namespace astem;
  constexpr uint32_t C = 0x64646464u;
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int i = tid + 256 * k;
    if (i >= NQUAD) continue;
    const uint32_t d0 = q.d[k][0], d1 = q.d[k][1], d2 = q.d[k][2];
    uint4v o0, o1;
    o0[0] = astem_h2(__builtin_amdgcn_perm(C, d0, 0x04010400u));                  // r0 g0
    o0[1] = astem_h2(__builtin_amdgcn_perm(C, d0, 0x040C0402u));                  // b0 0
    o0[2] = astem_h2(__builtin_amdgcn_perm(d1, d0, 0x0C040C03u) | 0x64006400u);   // r1 g1 (two dwords)
    o0[3] = astem_h2(__builtin_amdgcn_perm(C, d1, 0x040C0401u));                  // b1 0
    o1[0] = astem_h2(__builtin_amdgcn_perm(C, d1, 0x04030402u));                  // r2 g2
    o1[1] = astem_h2(__builtin_amdgcn_perm(C, d2, 0x040C0400u));                  // b2 0
    o1[2] = astem_h2(__builtin_amdgcn_perm(C, d2, 0x04020401u));                  // r3 g3
    o1[3] = astem_h2(__builtin_amdgcn_perm(C, d2, 0x040C0403u));                  // b3 0
    uint4v* d = reinterpret_cast<uint4v*>(patch + (size_t)i * 32);   // quad i = row r, pixels 4qc .. 4qc+3
    d[0] = o0;
    d[1] = o1;
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

// epilogue of one tile, registers only: border corrections, the 3x3/2 max pool (DPP
// row shifts across columns, the accumulators across rows), bias, ReLU, split store
// (F16: plain fp16 [B][Hp][Wp][64], the fp16 programs' stem)
template <bool F16 = false>
__device__ __forceinline__ void astem_epilogue(float4v (&acc)[astem::CRY], const AStemGeom& g, int b, int py0,
                                               int px0, int cx, int c0, const float* ps, float inv_scale,
                                               float acc_scale, float4v bv, half_t* __restrict__ y) {
  using namespace astem;
  // ---- epilogue of tile t, registers only ----
  // border conv outputs: their out-of-image taps saw u = 0, not the zero of x: add
  // the sum over the in-image taps of w * c minus the full sum in the bias, from the
  // 2D prefix sums S(kh, kw) (S(0, .) = S(., 0) = 0).  Rows with all 11 kernel rows
  // in the image (all but the first and last conv row) need only the column part,
  // S(11, whi) - S(11, wlo) - S(11, 11), computed once per tile
  const int cc = px0 * PS + cx;              // this lane's conv column
  const bool colv = cc < g.Wc;
  const int wlo = max(0, CP - CS * cc), whi = max(0, min(KH, g.W + CP - CS * cc));
  const bool colb = colv && (wlo > 0 || whi < KH);
  float4v colcorr = float4v{0.f, 0.f, 0.f, 0.f};
  if (colb) {
    const float4v s_h = *reinterpret_cast<const float4v*>(ps + (KH * 12 + whi) * 64 + c0);
    const float4v s_l = *reinterpret_cast<const float4v*>(ps + (KH * 12 + wlo) * 64 + c0);
    const float4v s_f = *reinterpret_cast<const float4v*>(ps + (KH * 12 + KH) * 64 + c0);
    colcorr = (s_h - s_l - s_f) * inv_scale;
  }
#pragma unroll
  for (int r = 0; r < CRY; ++r) {
    const int cr = py0 * PS + r;             // wave-uniform
    if (cr < g.Hc) {
      const int hlo = max(0, CP - CS * cr), hhi = min(KH, g.H + CP - CS * cr);
      if (hlo > 0 || hhi < KH) {
        if (colv) {
          const float4v s_hh = *reinterpret_cast<const float4v*>(ps + (hhi * 12 + whi) * 64 + c0);
          const float4v s_lh = *reinterpret_cast<const float4v*>(ps + (hlo * 12 + whi) * 64 + c0);
          const float4v s_hl = *reinterpret_cast<const float4v*>(ps + (hhi * 12 + wlo) * 64 + c0);
          const float4v s_ll = *reinterpret_cast<const float4v*>(ps + (hlo * 12 + wlo) * 64 + c0);
          const float4v s_ff = *reinterpret_cast<const float4v*>(ps + (KH * 12 + KH) * 64 + c0);
          acc[r] += (s_hh - s_lh - s_hl + s_ll - s_ff) * inv_scale;
        }
      } else {
        acc[r] += colcorr;
      }
    }
    // horizontal 3-max: lane cx holds max over conv columns cx .. cx+2
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = acc[r][e];
      acc[r][e] = fmaxf(v, fmaxf(astem_shl<1>(v), astem_shl<2>(v)));
    }
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
    if (col_ok && F16) {
      half4v o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (half_t)m[e];
      *reinterpret_cast<half4v*>(y + (((size_t)b * g.Hp + oy) * g.Wp + ox) * 64 + c0) = o;
    } else if (col_ok) {
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
}

// ABL: ablation bits for tools/astem_ablate.py (0 in production): 1 no MFMA loop,
// 2 no epilogue (accumulators kept alive by a never-taken store), 4 no patch staging
// F16: the fp16 programs' stem (hi MFMA only, fp16 out) at two workgroups per CU:
// without the A lo fragments a wave fits 256 registers, and with its MFMA loop half
// as long the epilogue/staging work dominates, which two independent workgroups
// overlap without phase barriers
template <bool AHEAD, int ABL = 0, bool F16 = false>
__global__ void __launch_bounds__(256, F16 ? 2 : 1)
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
      if constexpr (!F16) aL[s] = *reinterpret_cast<const half8v*>(wr + (size_t)64 * NKS * 32 + s * 32);
    }
  }
  const int c0 = 16 * wave + 4 * fch;          // this lane's 4 output channels
  const float4v bv = *reinterpret_cast<const float4v*>(bias + c0);
  const float inv_scale = 1.f / acc_scale;

  // the border prefix sums go to LDS once: the corrections of edge tiles then cost
  // LDS reads, not dependent L2 round trips inside the epilogue
  float* ps = reinterpret_cast<float*>(smem + PATCH_BYTES);
  for (int i = tid; i < PSUM_FLOATS / 4; i += 256)
    reinterpret_cast<float4v*>(ps)[i] = reinterpret_cast<const float4v*>(psum)[i];
  astem_store(smem, tid, q);
  int tn = t + gridDim.x;
  if (AHEAD && tn < g.ntiles) astem_load(img, g, tn, tid, q);   // one tile ahead (held in AGPRs)
  __syncthreads();

  // per-lane patch byte offsets (conv row 0): main steps read pixels
  // 4cx + XOFF + 2fch (+1) of row kh; tail step t reads pixels 4cx + XOFF + 8 (fch 0, 2)
  // or + 10 (fch 1, 3) of row 2t (fch 0, 1) or 2t + 1 (fch 2, 3; row 11 holds zero
  // weights and reads row 10 instead, a finite value)
  const uint32_t mainb = (uint32_t)(4 * cx + XOFF + 2 * fch) * 8u;
  const uint32_t tailb = (uint32_t)(4 * cx + XOFF + 8 + 2 * (fch & 1)) * 8u;
  const int trow = fch >> 1;
  // the A loads above must not stay in flight into the tile loop: the waitcnt pass
  // would put their vmcnt waits inside the loop, where from the second tile on they
  // wait for the next patch's global loads instead (a stall on every K step)
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)

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
      if (ABL & 1) break;
      if (s + 1 < NKS) astem_read_b(smem, s + 1, mainb, tailb, trow, bf[(s + 1) & 1]);
#pragma unroll
      for (int r = 0; r < CRY; ++r)
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aH[s], bf[s & 1][r], acc[r], 0, 0, 0);
      if constexpr (!F16) {
#pragma unroll
        for (int r = 0; r < CRY; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aL[s], bf[s & 1][r], acc[r], 0, 0, 0);
      }
      // keeps the scheduler from hoisting later steps' reads (it spilled when it did)
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();                           // every wave's patch reads of tile t are done
    // the next tile's patch loads go out now (not a tile ahead: the 136 A registers, 36
    // accumulators and 9 B fragments leave no room to hold them across the MFMA loop)
    // and land while this tile's epilogue runs
    const int tnext = tn;
    if constexpr (AHEAD) {
      if (!(ABL & 4) && tnext < g.ntiles) astem_store(smem, tid, q);
      tn = tnext + gridDim.x;
    } else {
      tn = tnext + gridDim.x;
      if (tnext < g.ntiles) astem_load(img, g, tnext, tid, q);
    }

    if constexpr ((ABL & 2) != 0) {
      if (g.B < 0) {                           // never: keeps the MFMA loop alive
#pragma unroll
        for (int r = 0; r < CRY; ++r) *reinterpret_cast<float4v*>(y + 8 * r) = acc[r];
      }
      if (AHEAD && !(ABL & 4) && tn < g.ntiles) astem_load(img, g, tn, tid, q);
      __syncthreads();
      if (tnext >= g.ntiles) break;
      t = tnext;
      continue;
    }
    astem_epilogue<F16>(acc, g, b, py0, px0, cx, c0, ps, inv_scale, acc_scale, bv, y);
    if (!AHEAD && tnext < g.ntiles) astem_store(smem, tid, q);
    // the loads of the tile after next go out behind this tile's border-correction
    // loads and output stores (vmcnt retires in order: those waits do not cover them)
    // and land during tile tnext's MFMA loop
    if (AHEAD && !(ABL & 4) && tn < g.ntiles) astem_load(img, g, tn, tid, q);
    __syncthreads();                           // tile tnext's patch is in LDS
    if (tnext >= g.ntiles) break;
    t = tnext;
  }
}

// Phased form: ONE workgroup of 512 threads per CU = two halves of 4 waves, each half
// on its own tiles (tile 2*blockIdx + h, then + 2*gridDim).  Phases alternate: while
// half 0 runs a tile's MFMA loop, half 1 runs its previous tile's epilogue and stages
// its next patch, then the roles swap (one workgroup barrier per phase).  SIMD k holds
// wave k of each half, so one wave's VALU/LDS/global work issues between the other's
// MFMAs instead of after them (the one-half form runs them back to back: MFMA loop
// 157 us + staging ~60 + epilogue ~90 at B = 500, tools/astem_ablate.py).  Two waves
// per SIMD leave 256 registers a wave: the A lo fragments move to LDS (one 16-byte read
// per K step, reused by 9 MFMAs) next to the two patches and the prefix sums.
namespace astem {
constexpr int PS_OFF = 2 * PATCH_BYTES;                  // border prefix sums
constexpr int AL_OFF = PS_OFF + PSUM_FLOATS * 4;         // A lo [64][17*32] fp16
constexpr int LDS2_BYTES = AL_OFF + 64 * NKS * 32 * 2;   // 158,784 B
static_assert(LDS2_BYTES <= 160 * 1024, "one workgroup per CU");
}  // namespace astem

// ABL: ablations (tools/astem_ablate.py): 1 no MFMA loop, 2 no E phase.  F16: the fp16
// programs' stem in the same exact-u8 form -- hi MFMA only (w' rounded to fp16 once,
// u exact), fp16 output
template <int ABL = 0, bool F16 = false>
__global__ void __launch_bounds__(512, 1)
alex_stem_split_kernel2(const uint8_t* __restrict__ img, const half_t* __restrict__ w, const float* __restrict__ bias,
                        const float* __restrict__ psum, float acc_scale, half_t* __restrict__ y, const AStemGeom g,
                        const long long* __restrict__ start_idx, long long start_off, long long max_start,
                        long long sub) {
  using namespace astem;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (start_idx != nullptr) {
    long long s = *start_idx - start_off;
    s = (s < 0 ? 0 : (s > max_start ? max_start : s)) + sub;
    img += (size_t)s * g.H * g.W * 3;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = wave >> 2, w4 = wave & 3, htid = tid & 255;
  const int cx = lane & 15, fch = lane >> 4;
  const int stride = 2 * gridDim.x;
  // tiles of half h: t0 + k * stride, k < nh; C(k) runs in phase 2k + h, E(k) in 2k + h + 1
  const int f0 = 2 * blockIdx.x, f1 = f0 + 1;
  const int n0 = f0 < g.ntiles ? (g.ntiles - 1 - f0) / stride + 1 : 0;
  const int n1 = f1 < g.ntiles ? (g.ntiles - 1 - f1) / stride + 1 : 0;
  if (n0 == 0) return;                          // uniform (n0 >= n1)
  const int t0 = h ? f1 : f0, nh = h ? n1 : n0;
  const int nphase = max(2 * n0 + 1, 2 * n1 + 2);
  char* patch = smem + h * PATCH_BYTES;
  float* ps = reinterpret_cast<float*>(smem + PS_OFF);
  const char* al = smem + AL_OFF;

  AQuads q;
  if (nh > 0) astem_load(img, g, t0, htid, q);
  half8v aH[NKS];
  const uint32_t aoff = (uint32_t)((16 * w4 + cx) * (NKS * 32) + 8 * fch) * 2u;   // bytes, hi and lo alike
#pragma unroll
  for (int s = 0; s < NKS; ++s) aH[s] = *reinterpret_cast<const half8v*>(reinterpret_cast<const char*>(w) + aoff + s * 64);
  for (int i = tid; i < PSUM_FLOATS / 4; i += 512)
    reinterpret_cast<float4v*>(ps)[i] = reinterpret_cast<const float4v*>(psum)[i];
  if constexpr (!F16)
    for (int i = tid; i < 64 * NKS * 32 / 8; i += 512)
      reinterpret_cast<half8v*>(smem + AL_OFF)[i] = reinterpret_cast<const half8v*>(w + 64 * NKS * 32)[i];
  const int c0 = 16 * w4 + 4 * fch;
  const float4v bv = *reinterpret_cast<const float4v*>(bias + c0);
  const float inv_scale = 1.f / acc_scale;
  if (nh > 0) astem_store(patch, htid, q);
  __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0): nothing of the prologue stays in flight
  if (nh > 1) astem_load(img, g, t0 + stride, htid, q);
  const uint32_t mainb = (uint32_t)(4 * cx + XOFF + 2 * fch) * 8u;
  const uint32_t tailb = (uint32_t)(4 * cx + XOFF + 8 + 2 * (fch & 1)) * 8u;
  const int trow = fch >> 1;
  __syncthreads();

  float4v acc[CRY];
#pragma unroll
  for (int r = 0; r < CRY; ++r) acc[r] = float4v{0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < nphase; ++p) {
    const int d = p - h;                        // wave-uniform
    if (d >= 0 && !(d & 1) && (d >> 1) < nh) {
      // ---- C(k): the MFMA loop of tile t0 + k * stride on this half's patch ----
#pragma unroll
      for (int r = 0; r < CRY; ++r) acc[r] = float4v{0.f, 0.f, 0.f, 0.f};
      if constexpr ((ABL & 1) != 0) {
#pragma unroll
        for (int r = 0; r < CRY; ++r) acc[r] = *reinterpret_cast<const float4v*>(patch + 64 * r + 16 * fch);
      } else {
      half8v bf[2][CRY];
      half8v al_s[2];
      astem_read_b(patch, 0, mainb, tailb, trow, bf[0]);
      if constexpr (!F16) al_s[0] = *reinterpret_cast<const half8v*>(al + aoff);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (s + 1 < NKS) {
          astem_read_b(patch, s + 1, mainb, tailb, trow, bf[(s + 1) & 1]);
          if constexpr (!F16) al_s[(s + 1) & 1] = *reinterpret_cast<const half8v*>(al + aoff + (s + 1) * 64);
        }
#pragma unroll
        for (int r = 0; r < CRY; ++r)
          acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aH[s], bf[s & 1][r], acc[r], 0, 0, 0);
        if constexpr (!F16) {
#pragma unroll
          for (int r = 0; r < CRY; ++r)
            acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al_s[s & 1], bf[s & 1][r], acc[r], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      }
    } else if (d >= 1 && (d & 1) && ((d - 1) >> 1) < nh) {
      // ---- E(k): stage tile k+1's patch, send tile k+2's loads, epilogue of tile k ----
      const int kk = (d - 1) >> 1;
      if constexpr ((ABL & 2) != 0) {
        if (g.B < 0) {                           // never: keeps the MFMA loop alive
#pragma unroll
          for (int r = 0; r < CRY; ++r) *reinterpret_cast<float4v*>(y + 8 * r) = acc[r];
        }
        __syncthreads();
        continue;
      }
      if (kk + 1 < nh) astem_store(patch, htid, q);
      if (kk + 2 < nh) astem_load(img, g, t0 + (kk + 2) * stride, htid, q);
      int b, py0, px0;
      astem_tile(g, t0 + kk * stride, b, py0, px0);
      astem_epilogue<F16>(acc, g, b, py0, px0, cx, c0, ps, inv_scale, acc_scale, bv, y);
    }
    __syncthreads();
  }
}

static bool astem_geom(AStemGeom& g, int B, int H, int W, const uint8_t* img, int* ovf) {
  using namespace astem;
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
  return true;
}

// fp16 form: two one-half workgroups per CU (default, AlexNet fp16 b500 +1.8 % over the
// phased halves: profiles/r6w_ab_alex_stem_f16_two_wg_b500.log) or the phased kernel
static int g_astem_f16_two_wg = 1;
void set_astem_f16_two_wg(bool on) { g_astem_f16_two_wg = on; }

// fp16 programs: the phased exact-u8 stem, hi MFMA only, fp16 [B][Hp][Wp][64] out
bool alex_stem_u8_f16_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum,
                             float acc_scale, half_t* y, int B, int H, int W, const long long* start_idx,
                             long long start_off, long long max_start, long long sub, hipStream_t st) {
  using namespace astem;
  AStemGeom g;
  if (!astem_geom(g, B, H, W, img, nullptr)) return false;
  if (g.ntiles <= 0) return true;
  const int per = device_cu_count();
  if (g_astem_f16_two_wg) {
    const int grid = g.ntiles < 2 * per ? g.ntiles : 2 * per;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(alex_stem_split_kernel<true, 0, true>), dim3(grid), dim3(256), LDS_BYTES, st,
                       img, w, bias, psum, acc_scale, y, g, start_idx, start_off, max_start, sub);
    return true;
  }
  const int grid2 = (g.ntiles + 1) / 2 < per ? (g.ntiles + 1) / 2 : per;
  auto k2 = alex_stem_split_kernel2<0, true>;
  ensure_lds_attr(reinterpret_cast<const void*>(k2), LDS2_BYTES);
  hipLaunchKernelGGL(k2, dim3(grid2), dim3(512), LDS2_BYTES, st, img, w, bias, psum, acc_scale, y, g, start_idx,
                     start_off, max_start, sub);
  return true;
}

static int g_astem_variant = 64;
void set_astem_ahead(bool on) { g_astem_variant = on ? 0 : 16; }
void set_astem_phased(bool on) { g_astem_variant = on ? 64 : 0; }
void set_astem_variant(int v) { g_astem_variant = v; }

bool alex_stem_split_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum,
                            float acc_scale, half_t* y, int B, int H, int W, const long long* start_idx,
                            long long start_off, long long max_start, long long sub, int* ovf, hipStream_t st) {
  using namespace astem;
  AStemGeom g;
  if (!astem_geom(g, B, H, W, img, ovf)) return false;
  if (g.ntiles <= 0) return true;
  const int per = device_cu_count();          // one workgroup per CU (all 512 registers)
  const int grid = g.ntiles < per ? g.ntiles : per;
  auto k = alex_stem_split_kernel<true>;
  switch (g_astem_variant) {
    case 16: k = alex_stem_split_kernel<false>; break;
    case 1: k = alex_stem_split_kernel<true, 1>; break;
    case 2: k = alex_stem_split_kernel<true, 2>; break;
    case 4: k = alex_stem_split_kernel<true, 4>; break;
    case 6: k = alex_stem_split_kernel<true, 6>; break;
    default: break;
  }
  if (g_astem_variant >= 64) {
    const int grid2 = (g.ntiles + 1) / 2 < per ? (g.ntiles + 1) / 2 : per;
    auto k2 = alex_stem_split_kernel2<0>;
    if (g_astem_variant == 65) k2 = alex_stem_split_kernel2<1>;
    if (g_astem_variant == 66) k2 = alex_stem_split_kernel2<2>;
    ensure_lds_attr(reinterpret_cast<const void*>(k2), LDS2_BYTES);
    hipLaunchKernelGGL(k2, dim3(grid2), dim3(512), LDS2_BYTES, st, img, w, bias, psum, acc_scale,
                       y, g, start_idx, start_off, max_start, sub);
    return true;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), LDS_BYTES, st, img, w, bias, psum, acc_scale, y, g, start_idx,
                     start_off, max_start, sub);
  return true;
}

}  // namespace idunno
