// Implicit-GEMM convolution, v3 main loop for the large ResNet layers: one
// 512-thread workgroup per CU, 64x64 (or 128x64) output tile per wave, and a
// loop where LDS fragment reads of one K-chunk run behind the MFMAs of the
// previous one (cdna_hip_programming §5 "Read a staged buffer one phase AFTER
// the wait that retires it").
//
// Why: the v2 kernel (conv_glds.hip, 128x128 tile, 64x32 per wave, 2 blocks
// per CU) re-reads 6 fragments per 8 MFMAs and has every wave of a block read
// its fragments at the same moment after each barrier; PMC (profiles/
// r1_v6_pmc_bench.md) shows mfma_busy 0.27-0.34 with waves parked at
// waitcnt/barrier half the time.  Here:
//   * a 64x64 wave tile reads 8 fragments per 16 MFMAs (0.5 LDS read cycles
//     per MFMA cycle instead of 0.75) and a 256-row block tile halves the DMA
//     bytes per FLOP of the 128x128 tile;
//   * each K stage (BK = 64) is two chunks of K = 32 with two fragment register
//     sets: chunk 1 is read while chunk 0's MFMAs issue, and chunk 0 of stage
//     s+1 is read (right after the barrier that publishes it) while chunk 1 of
//     stage s issues, so LDS latency hides behind MFMA issue even at 2 waves
//     per SIMD;
//   * one barrier per stage; the DMA of stage s+NS is issued right after it
//     and has NS-1 stages of MFMA time to land.
// Operand staging, swizzle and epilogue follow conv_glds.hip (weights = MFMA A,
// pixels = MFMA B, NHWC 8-byte epilogue stores).
#include "../../kernels.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_b;
typedef __attribute__((address_space(1))) void glb_void_b;

// 128-byte rows: chunk slot XOR (row >> 1) & 7 (conflict-free for the
// ds_read_b128 lane groups of a 16-row fragment, docs/KERNELS.md)

template <int N>
__device__ __forceinline__ void big_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BN, int BM, int WN, int WM, int NS, int MINB, bool HAS_RES, bool OUT_F32>
// second launch bound = waves per SIMD (HIP semantics): MINB workgroups of WN*WM waves per CU
__global__ void __launch_bounds__(64 * WN * WM, WN * WM / 4 * MINB) conv_big_kernel(const ConvArgs a) {
  constexpr int NW = WN * WM;
  static_assert(NW == 8 || NW == 16, "8 or 16 waves");
  constexpr int TN = BN / WN, TM = BM / WM;
  constexpr int FN = TN / 16, FM = TM / 16;
  constexpr int A_INS = BN / 8, B_INS = BM / 8;           // 1 KiB DMA instructions per stage
  static_assert(A_INS % NW == 0 && B_INS % NW == 0, "DMA instructions split evenly over waves");
  constexpr int GA = A_INS / NW, GB = B_INS / NW, G = GA + GB;
  constexpr int A_BYTES = BN * 128, STAGE = (BN + BM) * 128;
  constexpr int NR = FN + FM;                              // ds_read_b128 per K32 chunk
  static_assert(NR <= 15, "lgkmcnt immediate");
  static_assert(NS >= 2 && NS <= 3 && G * (NS - 2) < 64, "ring depth");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;

  const int nwg = a.tiles_n * a.tiles_m;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tm = lid / a.tiles_n, tn = lid % a.tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;

  const half_t* zero = reinterpret_cast<const half_t*>(a.zero);
  const int lrow = lane >> 3, lslot = lane & 7;

  // A (weights) DMA sources: row base per instruction, nullptr past Cout
  const half_t* a_src[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int row = (wave + NW * j) * 8 + lrow;
    const int n = n0 + row;
    a_src[j] = n < a.Cout ? a.w + (size_t)n * a.Kpad + ((lslot ^ swz8(row)) << 3) : nullptr;
  }
  // B (pixels) DMA sources: image base + top-left input coordinate per instruction
  int b_base[GB], b_ih0[GB], b_iw0[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = (wave + NW * j) * 8 + lrow;
    const int m = m0 + row;
    const int ch = (lslot ^ swz8(row)) << 3;
    if (m < a.M) {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw, r = m - b * hw;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      b_base[j] = b * a.H * a.W * a.C + ch;
      b_ih0[j] = oh * a.stride - a.pad;
      b_iw0[j] = ow * a.stride - a.pad;
    } else {
      b_base[j] = 0;
      b_ih0[j] = -100000;
      b_iw0[j] = -100000;
    }
  }

  // issue-side K coordinates: stage = (kh, kw, 64-channel block), cb fastest
  int i_s = 0, i_cb = 0, i_kw = 0, i_kh = 0;
  auto issue = [&](int buf) {
    char* base = smem + buf * STAGE;
    const int koff = i_s * 64;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const half_t* src = a_src[j] ? a_src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_b*)src, (lds_void_b*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
    const int coff = i_cb * 64;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int ih = b_ih0[j] + i_kh, iw = b_iw0[j] + i_kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const half_t* src = ok ? a.x + b_base[j] + (ih * a.W + iw) * a.C + coff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_b*)src, (lds_void_b*)(base + A_BYTES + (wave + NW * j) * 1024),
                                       16, 0, 0);
    }
    ++i_s;
    if (++i_cb == a.cblk) {
      i_cb = 0;
      if (++i_kw == a.KW) {
        i_kw = 0;
        ++i_kh;
      }
    }
  };

  // fragment reads (inline asm, common.h) of K32 chunk kk of LDS buffer `buf`
  const uint32_t lds0 = lds_addr(smem);
  const int frow = lane & 15, fch = lane >> 4;
  auto read_chunk = [&](int buf, int kk, half8v(&fa)[FN], half8v(&fb)[FM]) {
    const uint32_t base = lds0 + buf * STAGE;
    const int ch = fch + 4 * kk;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int row = wn * TN + i * 16 + frow;
      fa[i] = lds_read_b128(base + row * 128 + ((ch ^ swz8(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int row = wm * TM + j * 16 + frow;
      fb[j] = lds_read_b128(base + A_BYTES + row * 128 + ((ch ^ swz8(row)) << 4));
    }
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // the ties order the MFMAs after the preceding counted lgkmcnt wait; the
  // sched_barrier keeps them ahead of the next wait / barrier
  auto mfmas = [&](half8v(&fa)[FN], half8v(&fb)[FM]) {
#pragma unroll
    for (int i = 0; i < FN; ++i) lds_tie(fa[i]);
#pragma unroll
    for (int j = 0; j < FM; ++j) lds_tie(fb[j]);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nK = a.nK;
  // prologue: stages 0 .. NS-2 in flight, wait for stage 0, then issue stage NS-1
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nK) issue(p);
  if constexpr (NS == 3) {
    if (nK > 1) big_vmcnt<G>(); else big_vmcnt<0>();
  } else {
    big_vmcnt<0>();
  }
  __builtin_amdgcn_s_barrier();
  if (NS - 1 < nK) issue(NS - 1);

  half8v fa0[FN], fb0[FM], fa1[FN], fb1[FM];
  read_chunk(0, 0, fa0, fb0);
  int buf = 0;
  for (int s = 0; s < nK; ++s) {
    read_chunk(buf, 1, fa1, fb1);
    lds_waitcnt<NR>();                       // chunk 0 fragments landed
    mfmas(fa0, fb0);
    const int nbuf = buf + 1 == NS ? 0 : buf + 1;
    if (s + 1 < nK) {
      // stage s+1 landed (this wave's DMAs; a later stage may stay in flight)
      if constexpr (NS == 3) {
        if (s + 2 < nK) big_vmcnt<G>(); else big_vmcnt<0>();
      } else {
        big_vmcnt<0>();
      }
      lds_waitcnt<0>();                      // this wave's reads of stage s are done
      __builtin_amdgcn_s_barrier();          // stage s+1 visible to all; stage s free
      if (s + NS < nK) issue(buf);           // stage s+NS into the buffer of stage s
      read_chunk(nbuf, 0, fa0, fb0);
    } else {
      lds_waitcnt<0>();
    }
    mfmas(fa1, fb1);
    buf = nbuf;
  }

  // ---- epilogue: bias (+residual) (+ReLU), NHWC 8-byte stores ---------------------
  half4v rv[FN][FM];
  if constexpr (HAS_RES) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + i * 16 + fch * 4;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = m0 + wm * TM + j * 16 + frow;
        const size_t off = (m < a.M && n < a.Cout) ? (size_t)m * a.Cout + n : 0;
        rv[i][j] = *reinterpret_cast<const half4v*>(a.res + off);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * TN + i * 16 + fch * 4;
    if (n >= a.Cout) continue;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + j * 16 + frow;
      if (m >= a.M) continue;
      float4v v = acc[i][j] + bv;
      if constexpr (HAS_RES) {
        v[0] += (float)rv[i][j][0];
        v[1] += (float)rv[i][j][1];
        v[2] += (float)rv[i][j][2];
        v[3] += (float)rv[i][j][3];
      }
      if (a.relu) {
        v[0] = fmaxf(v[0], 0.f);
        v[1] = fmaxf(v[1], 0.f);
        v[2] = fmaxf(v[2], 0.f);
        v[3] = fmaxf(v[3], 0.f);
      }
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4v*>(static_cast<float*>(a.y) + (size_t)m * a.ldy + n) = v;
      } else {
        half4v o;
        o[0] = (half_t)v[0];
        o[1] = (half_t)v[1];
        o[2] = (half_t)v[2];
        o[3] = (half_t)v[3];
        *reinterpret_cast<half4v*>(static_cast<half_t*>(a.y) + (size_t)m * a.ldy + n) = o;
      }
    }
  }
}

template <int BN, int BM, int WN, int WM, int NS, int MINB, bool R, bool F>
static void big_cfg(ConvArgs a, hipStream_t st) {
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.cblk = a.C / 64;
  a.nK = a.KH * a.KW * a.cblk;
  const int grid = a.tiles_n * a.tiles_m;
  const size_t lds = (size_t)NS * (BN + BM) * 128;
  auto kern = conv_big_kernel<BN, BM, WN, WM, NS, MINB, R, F>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WN * WM), lds, st, a);
}

// Tile table (ids 60-67; 512 threads, BK = 64):
//   60: 256x128 (Cout x px), waves 4x2 (64x64 each), 2 stages  96 KiB, 1 block/CU
//   61: 128x256,             waves 2x4 (64x64),      2 stages  96 KiB
//   62: 256x128,             waves 4x2,              3 stages 144 KiB
//   63: 128x256,             waves 2x4,              3 stages 144 KiB
//   (a 256x256 tile, 128x64 per wave, needs > 256 registers at 2 waves/SIMD: spills)
//   65: 128x128,             waves 2x4 (64x32),      2 stages  64 KiB, 2 blocks/CU
//   66: 128x128,             waves 2x4 (64x32),      3 stages  96 KiB
//   67: 64x256,              waves 1x8 (64x32),      2 stages  80 KiB, 2 blocks/CU
//   68: 256x128, 16 waves 4x4 (64x32), 2 stages 96 KiB: the bytes per FLOP of a 256-row
//       tile (0.75x of 128x128) at the wave count of two 128x128 workgroups
//   69: 128x256, 16 waves 2x8 (64x32), 2 stages 96 KiB
template <bool R, bool F>
static bool big_dispatch(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 60: big_cfg<256, 128, 4, 2, 2, 1, R, F>(a, st); return true;
    case 61: big_cfg<128, 256, 2, 4, 2, 1, R, F>(a, st); return true;
    case 62: big_cfg<256, 128, 4, 2, 3, 1, R, F>(a, st); return true;
    case 63: big_cfg<128, 256, 2, 4, 3, 1, R, F>(a, st); return true;
    case 65: big_cfg<128, 128, 2, 4, 2, 2, R, F>(a, st); return true;
    case 66: big_cfg<128, 128, 2, 4, 3, 1, R, F>(a, st); return true;
    case 67: big_cfg<64, 256, 1, 8, 2, 2, R, F>(a, st); return true;
    case 68: big_cfg<256, 128, 4, 4, 2, 1, R, F>(a, st); return true;   // 16 waves (64x32 each)
    case 69: big_cfg<128, 256, 2, 8, 2, 1, R, F>(a, st); return true;   // 16 waves (64x32 each)
    default: return false;
  }
}

bool conv_big_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st) {
  const bool res = a.res != nullptr;
  if (res) return out_f32 ? big_dispatch<true, true>(a, tile, st) : big_dispatch<true, false>(a, tile, st);
  return out_f32 ? big_dispatch<false, true>(a, tile, st) : big_dispatch<false, false>(a, tile, st);
}

}  // namespace idunno
