// EXPERIMENTAL (built only with IDUNNO_EXPERIMENTAL=1): measured -0.9 % in the
// whole graph, profiles/r2_v26_split_patch_c64_ab.md.
// 3x3 / stride-1 / pad-1 conv on split fp16 (fp32-accurate, conv_glds.hip SPLIT)
// with the B operand from a halo PATCH: ResNet layers 2-4 (C >= 128, 28x28 .. 7x7).
//
// As an implicit GEMM every input pixel is DMA'd from L2 once per tap: at B = 400
// the split 3x3 convs of layers 2-4 move ~10 TB/s L2 -> LDS at 42-48 % MFMA busy
// (profiles/r2_v25_pmc_split_forward.md).  Here a block (128 couts x 128
// consecutive output pixels, 8 waves, wave tile 64 x 32 as conv_glds tile 36)
// stages, per 32-channel block, ONE patch of every input pixel its 9 taps touch
// -- the tile's virtual rows +-1, all W+2 columns, where every image owns H+2
// virtual rows (its zero padding rows included), so a tile may span images --
// and reads the B fragments of all 9 taps from it at a pixel shift of
// (kh-1)*(W+2) + (kw-1).  At 28x28 a patch is <= 300 pixels against 9 x 128
// pixel rows per channel block for the im2col stream (3.8x less B traffic).
// The weights (A) stream per (tap, channel block) through an NSA-slot LDS-DMA
// ring (tiles 60 / 61 / 62 = NSA 2 / 3 / 4; LDS 72 / 88 / 104 KiB: two blocks
// per CU only at NSA 2).
// Pixel rows are 128 B (32 channels x (hi, lo)); chunk c of patch pixel pp sits
// in 16-byte slot c ^ (pp & 6): conflict-free for 16 consecutive pixels (a row
// wrap inside a fragment costs an occasional 2-way conflict).
#include "../../kernels.h"
#include "../../launch_util.h"

namespace idunno {

namespace pts {
constexpr int BN = 128, BM = 128, WN = 2, WM = 4, NW = WN * WM, NT = 64 * NW;
constexpr int TN = BN / WN, TM = BM / WM, FN = TN / 16, FM = TM / 16;
constexpr int RB = 128;                        // bytes per LDS row
constexpr int A_BYTES = BN * RB;               // 16 KiB per A slot
constexpr int GA = A_BYTES / 1024 / NW;        // A DMA instructions per wave and stage (2)
constexpr int GP = 5;                          // patch DMA instructions per wave and channel block
constexpr int PCAP = GP * NW * 1024 / RB;      // patch capacity in pixels (320)
constexpr int P_BYTES = PCAP * RB;             // 40 KiB
// LDS = NSA A slots + the patch: NSA 2 -> 72 KiB (two blocks per CU), 3 -> 88, 4 -> 104
constexpr int lds_bytes(int nsa) { return nsa * A_BYTES + P_BYTES; }
static_assert(GA * NW * 1024 == A_BYTES, "A DMA split");
}  // namespace pts

struct PatchSplitArgs {
  const half_t* x;      // split [B][H][W][C2]
  const half_t* w;      // split weights [Cout][9 * C2]
  const float* bias;    // [Cout]
  const half_t* res;    // split [B][H][W][2 Cout] or nullptr
  void* y;              // split [B][H][W][2 Cout], or fp32 [B][H][W][Cout] (OUT_F32)
  const void* zero;     // >= 16 zero bytes
  int B, H, W, C2, Cout, M, nK, relu, tiles_n, tiles_m;
  float acc_scale;
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

__device__ __forceinline__ int pts_key(int pp) { return pp & 6; }

template <bool HAS_RES, bool OUT_F32, int NSA>
__global__ void __launch_bounds__(pts::NT, 2) conv3x3_patch_split_kernel(const PatchSplitArgs a) {
  using namespace pts;
  constexpr int P_OFF = NSA * A_BYTES;            // A ring (NSA slots, NSA-1 stages in flight), then the patch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int nwg = a.tiles_n * a.tiles_m;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tm = lid / a.tiles_n, tn = lid % a.tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;
  const int HW = a.H * a.W, VR = a.H + 2, PW = a.W + 2;
  const half_t* zero = static_cast<const half_t*>(a.zero);
  const int Kpad = 9 * a.C2;

  // ---- virtual-row geometry of this tile: patch rows vr0-1 .. ----
  const int b0 = m0 / HW, oh0 = (m0 - b0 * HW) / a.W;
  const int vr0 = b0 * VR + oh0 + 1;             // virtual row of the tile's first pixel

  // A (weight) DMA sources: GA instructions of 8 rows x 128 B
  const int lrow = lane >> 3, lslot = lane & 7;
  const half_t* a_src[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int row = (wave + NW * j) * 8 + lrow;
    const int n = n0 + row;
    a_src[j] = n < a.Cout ? a.w + (size_t)n * Kpad + (lslot ^ swz_r(row, 8)) * 8 : nullptr;
  }
  // patch DMA sources: GP instructions of 8 pixels x 128 B; chunk i = pixel pp, slot
  int p_off[GP];
#pragma unroll
  for (int j = 0; j < GP; ++j) {
    const int i = (wave + NW * j) * 64 + lane;
    const int pp = i >> 3, slot = i & 7;
    const int vr = vr0 - 1 + pp / PW, col = pp - (pp / PW) * PW;
    const int b = vr / VR, ih = vr - b * VR - 1, iw = col - 1;
    const bool ok = b < a.B && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    p_off[j] = ok ? ((b * a.H + ih) * a.W + iw) * a.C2 + ((slot ^ pts_key(pp)) << 3) : -1;
  }
  auto issue_a = [&](int s, int buf) {
    const int tap = s % 9, cb = s / 9;
    const int koff = tap * a.C2 + cb * 64;
    char* base = smem + buf * A_BYTES;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const half_t* src = a_src[j] ? a_src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
  };
  auto issue_patch = [&](int cb) {
#pragma unroll
    for (int j = 0; j < GP; ++j) {
      const half_t* src = p_off[j] >= 0 ? a.x + p_off[j] + cb * 64 : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(smem + P_OFF + (wave + NW * j) * 1024), 16,
                                       0, 0);
    }
  };

  // B fragment pixels: patch index of each of this lane's FM pixels (tap centre)
  const int frow = lane & 15, fch = lane >> 4;
  int ppc[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = m0 + wm * TM + j * 16 + frow;
    int pp = PW + 1;                              // rows past M read a harmless in-patch pixel
    if (m < a.M) {
      const int b = m / HW, r = m - b * HW, oh = r / a.W, ow = r - oh * a.W;
      pp = (b * VR + oh + 1 - vr0 + 1) * PW + ow + 1;
    }
    ppc[j] = pp;
  }

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const uint32_t lds0 = lds_addr(smem);
  const int nK = a.nK;                            // 9 * C2 / 64 stages (tap, channel block)
#pragma unroll
  for (int p = 0; p < NSA - 1; ++p)
    if (p < nK) issue_a(p, p);
  for (int s = 0; s < nK; ++s) {
    const int tap = s % 9;
    if (tap == 0) {
      // new channel block: every wave is done with the previous patch; the
      // patch is the newest DMA, so this wait drains the A ring too
      __builtin_amdgcn_s_barrier();
      issue_patch(s / 9);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      // A(s) landed for this wave; up to NSA-2 newer A stages stay in flight
      const int ahead = min(NSA - 2, nK - 1 - s);
      if constexpr (NSA >= 4) {
        if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GA) : "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if constexpr (NSA == 3) {
        if (ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GA) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_barrier();                      // every wave's DMAs landed; slot (s-1) % NSA is free
    if (s + NSA - 1 < nK) issue_a(s + NSA - 1, (s + NSA - 1) % NSA);

    const uint32_t abase = lds0 + (s % NSA) * A_BYTES;
    const int kh = tap / 3, kw = tap - 3 * kh;
    const int dpp = (kh - 1) * PW + (kw - 1);
    half8v fa[2][FN], fb[2][FM];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {              // kk 0 = hi, 1 = lo
      const int ch = fch + 4 * kk;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * TN + i * 16 + frow;
        fa[kk][i] = lds_read_b128(abase + row * RB + ((ch ^ swz_r(row, 8)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int pp = ppc[j] + dpp;
        fb[kk][j] = lds_read_b128(lds0 + P_OFF + pp * RB + ((ch ^ pts_key(pp)) << 4));
      }
    }
    constexpr int NR = FN + FM;
    lds_waitcnt<NR>();
#pragma unroll
    for (int i = 0; i < FN; ++i) lds_tie(fa[0][i]);
#pragma unroll
    for (int j = 0; j < FM; ++j) lds_tie(fb[0][j]);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
    lds_waitcnt<0>();
#pragma unroll
    for (int i = 0; i < FN; ++i) lds_tie(fa[1][i]);
#pragma unroll
    for (int j = 0; j < FM; ++j) lds_tie(fb[1][j]);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
      }
  }

  // ---- epilogue (as conv_glds SPLIT): scale, bias (+ split residual), ReLU ----
  const int ldy = OUT_F32 ? a.Cout : 2 * a.Cout;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
    if (n >= a.Cout) continue;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + j * 16 + (lane & 15);
      if (m >= a.M) continue;
      float4v v = acc[i][j] * a.acc_scale + bv;
      if constexpr (HAS_RES) {
        const size_t off = (size_t)m * 2 * a.Cout + split_off(n);
        const half4v rh = *reinterpret_cast<const half4v*>(a.res + off);
        const half4v rl = *reinterpret_cast<const half4v*>(a.res + off + 32);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (float)rh[e] + (float)rl[e];
      }
      if (a.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4v*>(static_cast<float*>(a.y) + (size_t)m * ldy + n) = v;
      } else {
        half4v h, l;
        split_f16x4(v, h, l);
        half_t* yp = static_cast<half_t*>(a.y) + (size_t)m * ldy + split_off(n);
        *reinterpret_cast<half4v*>(yp) = h;
        *reinterpret_cast<half4v*>(yp + 32) = l;
      }
    }
  }
}

// Whether every 128-pixel tile's patch (its virtual rows +-1 x (W+2) columns)
// fits the LDS patch: checked exactly over the tiles on the host.
bool conv3x3_patch_split_supported(int B, int H, int W, int C, int Cout) {
  using namespace pts;
  if (C % 32 || Cout % 32 || H < 1 || W < 1) return false;
  const long M = (long)B * H * W, HW = (long)H * W;
  for (long m0 = 0; m0 < M; m0 += BM) {
    const long m1 = (m0 + BM < M ? m0 + BM : M) - 1;
    const long vr0 = (m0 / HW) * (H + 2) + (m0 % HW) / W + 1;
    const long vr1 = (m1 / HW) * (H + 2) + (m1 % HW) / W + 1;
    if ((vr1 - vr0 + 3) * (W + 2) > PCAP) return false;
  }
  return true;
}

template <int NSA>
static void patch_split_launch(const PatchSplitArgs& a, bool res, bool out_f32, hipStream_t st) {
  using namespace pts;
  const int grid = a.tiles_n * a.tiles_m;
  auto launch = [&](auto kern) {
    ensure_lds_attr(reinterpret_cast<const void*>(kern), lds_bytes(NSA));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds_bytes(NSA), st, a);
  };
  if (res) {
    if (out_f32) launch(conv3x3_patch_split_kernel<true, true, NSA>);
    else launch(conv3x3_patch_split_kernel<true, false, NSA>);
  } else {
    if (out_f32) launch(conv3x3_patch_split_kernel<false, true, NSA>);
    else launch(conv3x3_patch_split_kernel<false, false, NSA>);
  }
}

// nsa: A ring depth 2 (tile 60), 3 (61) or 4 (62)
void conv3x3_patch_split_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, void* y,
                                bool out_f32, const void* zero, int B, int H, int W, int C, int Cout, int relu,
                                float acc_scale, int nsa, hipStream_t st) {
  using namespace pts;
  PatchSplitArgs a;
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.B = B;
  a.H = H;
  a.W = W;
  a.C2 = 2 * C;
  a.Cout = Cout;
  a.M = B * H * W;
  a.nK = 9 * (2 * C) / 64;
  a.relu = relu;
  a.acc_scale = acc_scale;
  a.tiles_n = (Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  if (nsa >= 4) patch_split_launch<4>(a, res != nullptr, out_f32, st);
  else if (nsa == 3) patch_split_launch<3>(a, res != nullptr, out_f32, st);
  else patch_split_launch<2>(a, res != nullptr, out_f32, st);
}

}  // namespace idunno
