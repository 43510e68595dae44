// 3x3 / stride 1 / pad 1 convolution with an LDS-resident input patch.
//
// The implicit-GEMM kernels (conv_glds.hip) gather the im2col B operand once per
// tap: every input pixel row crosses L2 -> LDS nine times.  Here a workgroup owns
// a spatial tile of output pixels (TH rows x W cols of NI images, M <= 224) and
// 64 output channels.  For each 64-channel block `cb` of the input it DMAs the
// (TH+2) x (W+2) halo patch into LDS ONCE (global_load_lds_dwordx4, padding
// from a zero buffer) and runs all nine taps against it; only the 8 KiB weight
// slice of each tap streams through a 3-deep LDS ring.  Per barrier the block
// now does 224x64x64 MACs against 8 KiB of new bytes (vs 24 KiB for the
// 64x128 im2col tile): the B-operand traffic drops ~6x.
//
// MFMA: v_mfma_f32_16x16x32_f16, weights = A (rows = output channels), pixels =
// B.  A B fragment row for tap (kh, kw) is patch row
//   prow = (img*(TH+2) + oy + kh) * (W+2) + ox + kw
// i.e. the pixel's base row plus a wave-uniform tap offset.  Patch rows are
// 128 B (64 fp16 channels); chunks are XOR-swizzled by (prow >> 1) & 7 on the DMA
// source address and on the fragment read (as in conv_glds.hip).
//
// Workgroup = 4 waves (2 x 2): each wave 32 channels (2 A frags) x 7 pixel
// fragments (112 px) -> 14 MFMAs per 32-wide K step.  LDS <= ~68 KiB -> 2
// workgroups per CU.
#include "../../kernels.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_p;
typedef __attribute__((address_space(1))) void glb_void_p;

namespace c3 {
constexpr int WN = 2, WM = 2, NW = 4;
constexpr int FN = 2, FM = 7;          // per wave: 32 couts x 112 pixels
constexpr int MT = WM * FM * 16;       // 224 pixels per tile
constexpr int NT = WN * FN * 16;       // 64 couts per tile
constexpr int RING = 3;                // weight-slice ring depth
constexpr int A_BYTES = NT * 128;      // one tap x 64 ch x 64 couts = 8 KiB
constexpr int MAX_PATCH_INS = 48;      // <= 384 patch rows (49 KiB)
constexpr int PI_PER_WAVE = MAX_PATCH_INS / NW;
}  // namespace c3

struct C3Args {
  const half_t* x;     // NHWC [B][H][W][C]
  const half_t* w;     // [Cout][3][3][C]
  const float* bias;   // [Cout]
  const half_t* res;   // NHWC [B][H][W][Cout] or nullptr
  half_t* y;           // NHWC [B][H][W][Cout]
  const void* zero;
  int B, H, W, C, Cout;
  int TH, NI;          // tile: NI images x TH rows x W cols
  int tiles_y, groups, ctiles;
  int PR;              // patch rows = NI*(TH+2)*(W+2)
  int patch_ins;       // ceil(PR / 8) DMA instructions
  int relu;
};


template <bool HAS_RES>
__global__ void __launch_bounds__(256, 2) conv3x3_patch_kernel(const C3Args a) {
  using namespace c3;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  char* patch = smem;
  char* ring = smem + a.patch_ins * 1024;

  // block -> (cout tile, image group, row tile); cout tiles of one spatial tile
  // are consecutive so they share the XCD's L2 copy of the patch
  const int nwg = a.ctiles * a.groups * a.tiles_y;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int ct = lid % a.ctiles;
  const int sp = lid / a.ctiles;
  const int g = sp / a.tiles_y, ty = sp % a.tiles_y;
  const int n0 = ct * NT, oh0 = ty * a.TH, b0 = g * a.NI;
  const int Wp = a.W + 2, THp = a.TH + 2;
  const half_t* zero = reinterpret_cast<const half_t*>(a.zero);
  const int lrow = lane >> 3, lslot = lane & 7;

  // ---- patch DMA sources (fixed over cb): element offset incl. chunk, or -1 ----
  int poff[PI_PER_WAVE];
#pragma unroll
  for (int j = 0; j < PI_PER_WAVE; ++j) {
    const int i = wave + NW * j;
    const int row = i * 8 + lrow;
    poff[j] = -1;
    if (i < a.patch_ins && row < a.PR) {
      const int img = row / (THp * Wp), r = row - img * (THp * Wp);
      const int py = r / Wp, px = r - py * Wp;
      const int b = b0 + img, ih = oh0 + py - 1, iw = px - 1;
      if (b < a.B && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        poff[j] = ((b * a.H + ih) * a.W + iw) * a.C + ((lslot ^ swz8(row)) << 3);
    }
  }
  // ---- weight-slice DMA source: one instruction per wave per tap -------------
  const int arow = wave * 8 + lrow;                       // 0..31 (rows 32..63: second instr)
  int aoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = arow + 32 * j;
    const int co = n0 + row;
    aoff[j] = co < a.Cout ? co * 9 * a.C + ((lslot ^ swz8(row)) << 3) : -1;
  }

  const int ncb = a.C / 64;
  const int nS = ncb * 9;
  auto issue_a = [&](int s) {
    const int cb = s / 9, tap = s - cb * 9;
    char* dst = ring + (s % RING) * A_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const half_t* src = aoff[j] >= 0 ? a.w + aoff[j] + tap * a.C + cb * 64 : zero;
      __builtin_amdgcn_global_load_lds((glb_void_p*)src, (lds_void_p*)(dst + (wave + 4 * j) * 1024), 16, 0, 0);
    }
  };
  auto issue_patch = [&](int cb) {
#pragma unroll
    for (int j = 0; j < PI_PER_WAVE; ++j) {
      const int i = wave + NW * j;
      if (i < a.patch_ins) {
        const half_t* src = poff[j] >= 0 ? a.x + poff[j] + cb * 64 : zero;
        __builtin_amdgcn_global_load_lds((glb_void_p*)src, (lds_void_p*)(patch + i * 1024), 16, 0, 0);
      }
    }
  };

  // ---- per-lane B fragment bases (pixel -> patch row) -------------------------
  const int frow = lane & 15, fch = lane >> 4;
  int pbase[FM];
  bool pvalid[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int p = (wm * FM + f) * 16 + frow;
    const int per = a.TH * a.W;
    const int img = p / per, r = p - img * per;
    const int oy = r / a.W, ox = r - oy * a.W;
    pvalid[f] = p < a.NI * per;
    pbase[f] = pvalid[f] ? (img * THp + oy) * Wp + ox : 0;
  }

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[i][f] = float4v{0.f, 0.f, 0.f, 0.f};

  issue_a(0);
  if (nS > 1) issue_a(1);
  for (int s = 0; s < nS; ++s) {
    const int cb = s / 9, tap = s - cb * 9;
    if (tap == 0) {
      if (cb > 0) __builtin_amdgcn_s_barrier();          // everyone done with patch(cb-1)
      issue_patch(cb);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (s + 1 < nS) {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // A(s) landed; A(s+1) may fly
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nS) issue_a(s + 2);

    const int kh = tap / 3, kw = tap - kh * 3;
    const int toff = kh * Wp + kw;
    const char* abuf = ring + (s % RING) * A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = fch + 4 * kk;
      half8v fa[FN], fb[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * (FN * 16) + i * 16 + frow;
        fa[i] = *reinterpret_cast<const half8v*>(abuf + row * 128 + ((ch ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int row = pbase[f] + toff;
        fb[f] = *reinterpret_cast<const half8v*>(patch + row * 128 + ((ch ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f)
          acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[f], acc[i][f], 0, 0, 0);
    }
  }

  // ---- epilogue ------------------------------------------------------------------
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * (FN * 16) + i * 16 + fch * 4;
    if (n >= a.Cout) continue;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      if (!pvalid[f]) continue;
      const int p = (wm * FM + f) * 16 + frow;
      const int per = a.TH * a.W;
      const int img = p / per, r = p - img * per;
      const int oy = r / a.W, ox = r - oy * a.W;
      const int b = b0 + img, oh = oh0 + oy;
      if (b >= a.B || oh >= a.H) continue;
      const size_t m = ((size_t)b * a.H + oh) * a.W + ox;
      float4v v = acc[i][f] + bv;
      if constexpr (HAS_RES) {
        const half4v rr = *reinterpret_cast<const half4v*>(a.res + m * a.Cout + n);
        v[0] += (float)rr[0];
        v[1] += (float)rr[1];
        v[2] += (float)rr[2];
        v[3] += (float)rr[3];
      }
      if (a.relu) {
        v[0] = fmaxf(v[0], 0.f);
        v[1] = fmaxf(v[1], 0.f);
        v[2] = fmaxf(v[2], 0.f);
        v[3] = fmaxf(v[3], 0.f);
      }
      half4v o;
      o[0] = (half_t)v[0];
      o[1] = (half_t)v[1];
      o[2] = (half_t)v[2];
      o[3] = (half_t)v[3];
      *reinterpret_cast<half4v*>(a.y + m * a.Cout + n) = o;
    }
  }
}

// Tile geometry for an (H, W) plane: M = NI * TH * W <= 224 pixels.
static void c3_geometry(C3Args& a) {
  using namespace c3;
  if (a.W * a.H <= MT) {                   // whole images per tile
    a.TH = a.H;
    a.NI = MT / (a.W * a.H);
  } else {
    a.NI = 1;
    a.TH = MT / a.W;
    if (a.TH < 1) a.TH = 1;
  }
  a.tiles_y = (a.H + a.TH - 1) / a.TH;
  a.groups = (a.B + a.NI - 1) / a.NI;
  a.ctiles = (a.Cout + NT - 1) / NT;
  a.PR = a.NI * (a.TH + 2) * (a.W + 2);
  a.patch_ins = (a.PR + 7) / 8;
}

bool conv3x3_patch_supported(int H, int W, int C, int Cout) {
  if (C % 64 != 0 || Cout % 4 != 0 || W > c3::MT) return false;
  C3Args a{};
  a.B = 1;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  c3_geometry(a);
  return a.patch_ins <= c3::MAX_PATCH_INS;
}

void conv3x3_patch_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                          const void* zero, int B, int H, int W, int C, int Cout, int relu, hipStream_t st) {
  using namespace c3;
  C3Args a{};
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.B = B;
  a.H = H;
  a.W = W;
  a.C = C;
  a.Cout = Cout;
  a.relu = relu;
  c3_geometry(a);
  const size_t lds = (size_t)a.patch_ins * 1024 + RING * A_BYTES;
  const int grid = a.ctiles * a.groups * a.tiles_y;
  if (res) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_patch_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL(conv3x3_patch_kernel<true>, dim3(grid), dim3(256), lds, st, a);
  } else {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_patch_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL(conv3x3_patch_kernel<false>, dim3(grid), dim3(256), lds, st, a);
  }
}

}  // namespace idunno
