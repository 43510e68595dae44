// Persistent implicit-GEMM convolution: each workgroup walks a strided list of
// output tiles, and the LDS-DMA ring runs straight across tile boundaries.
//
// Why: the per-layer sweep shows a large fixed cost per output tile in the
// one-tile-per-workgroup kernels (conv_glds.hip / conv_big.hip): at the same
// tile count, the 3x3/s2 layer2 conv with 9 K stages runs at 620 TF/s and the
// 3x3/s1 one with 18 stages at 820 TF/s; fitting time = tiles x (c0 + nK x c1)
// gives c0 ~ 10 stages (profiles/r1_v8_conv_big_sweep.log).  That cost is the
// exposed part of a tile's prologue (first DMA round trip, address set-up,
// workgroup launch) and epilogue (bias / residual loads, stores).  Here:
//   * the DMA of the next tile's first stages is issued while the current
//     tile's last stages compute (one global stage counter over (tile, stage));
//   * the epilogue operands (residual) are loaded one stage ahead with loads
//     the compiler does not track, and bias comes from LDS (staged once);
//   * epilogue stores are buffer stores issued by every lane unconditionally
//     (out-of-range lanes get an offset past the descriptor's size, so the
//     hardware drops them).  Every wave therefore issues exactly the same
//     number of vector-memory ops per stage, and each ring wait is a counted
//     `s_waitcnt vmcnt(N)` that leaves the younger stores / loads in flight:
//     no store or load latency is waited for in front of the MFMAs.
// Loop body per stage (BK = 64, two K32 chunks, two fragment register sets)
// as conv_big.hip; tiles and swizzles as conv_glds.hip.
#include "../../kernels.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_pp;
typedef __attribute__((address_space(1))) void glb_void_pp;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pers_swz(int row) { return (row >> 1) & 7; }

template <int N>
__device__ __forceinline__ void pers_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BN, int BM, int WN, int WM, int MINB, bool HAS_RES, bool OUT_F32>
// second launch bound = waves per SIMD (HIP semantics): MINB workgroups of 8 waves per CU
__global__ void __launch_bounds__(512, 2 * MINB) conv_pers_kernel(const ConvArgs a) {
  constexpr int NW = 8;
  static_assert(WN * WM == NW, "8 waves");
  constexpr int TN = BN / WN, TM = BM / WM;
  constexpr int FN = TN / 16, FM = TM / 16;
  constexpr int A_INS = BN / 8, B_INS = BM / 8;
  static_assert(A_INS % NW == 0 && B_INS % NW == 0, "DMA instructions split evenly over waves");
  constexpr int GA = A_INS / NW, GB = B_INS / NW, G = GA + GB;
  constexpr int A_BYTES = BN * 128, STAGE = (BN + BM) * 128;
  constexpr int NR = FN + FM;
  constexpr int NST = FN * FM;                      // epilogue stores per wave and tile
  constexpr int NRES = HAS_RES ? FN * FM : 0;       // residual loads per wave and tile
  // residual one stage ahead where registers allow (16 VGPRs for a 64x32 wave
  // tile would push the 2-workgroup configs past 128 and spill); otherwise
  // loaded in the epilogue, which then waits for it (and this stage's DMA)
  constexpr bool PREF = HAS_RES && (FN * FM <= 4 || MINB == 1);
  static_assert(NR <= 15 && NST < 64 && NRES < 64 && G < 64, "counter immediates");
  constexpr int OUT_BYTES = OUT_F32 ? 4 : 2;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* bias_lds = reinterpret_cast<float*>(smem + 2 * STAGE);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int lrow = lane >> 3, lslot = lane & 7;
  const int frow = lane & 15, fch = lane >> 4;

  const int nK = a.nK;
  const int ntiles = a.tiles_n * a.tiles_m;
  const int grid = gridDim.x;
  const int my_tiles = (ntiles - (int)blockIdx.x + grid - 1) / grid;
  if (my_tiles <= 0) return;
  const int total = my_tiles * nK;

  // bias -> LDS once (before any DMA is in flight)
  for (int i = tid; i < a.Cout; i += 512) bias_lds[i] = a.bias[i];
  __syncthreads();

  const half_t* zero = reinterpret_cast<const half_t*>(a.zero);
  // output descriptor: masked lanes store at an offset past its size (dropped)
  const unsigned out_bytes = (unsigned)a.M * (unsigned)a.ldy * OUT_BYTES;
  const auto out_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)out_bytes, 0x00020000);

  // ---- issue side: sources of the tile whose stages are being DMA'd ----------------
  const half_t* a_src[GA];
  int b_base[GB], b_ih0[GB], b_iw0[GB];
  int i_k = 0, i_s = 0, i_cb = 0, i_kw = 0, i_kh = 0;
  auto set_issue_tile = [&](int k) {
    const int lid = xcd_remap((int)blockIdx.x + k * grid, ntiles);
    const int tm = lid / a.tiles_n, tn = lid - (lid / a.tiles_n) * a.tiles_n;
    const int n0 = tn * BN, m0 = tm * BM;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int row = (wave + NW * j) * 8 + lrow;
      const int n = n0 + row;
      a_src[j] = n < a.Cout ? a.w + (size_t)n * a.Kpad + ((lslot ^ pers_swz(row)) << 3) : nullptr;
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = (wave + NW * j) * 8 + lrow;
      const int m = m0 + row;
      const int ch = (lslot ^ pers_swz(row)) << 3;
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
    i_s = i_cb = i_kw = i_kh = 0;
  };
  // DMA of the next stage in global (tile, stage) order into LDS buffer `buf`
  auto issue = [&](int buf) {
    if (i_s == nK) set_issue_tile(++i_k);
    char* base = smem + buf * STAGE;
    const int koff = i_s * 64;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const half_t* src = a_src[j] ? a_src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_pp*)src, (lds_void_pp*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
    const int coff = i_cb * 64;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int ih = b_ih0[j] + i_kh, iw = b_iw0[j] + i_kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const half_t* src = ok ? a.x + b_base[j] + (ih * a.W + iw) * a.C + coff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_pp*)src,
                                       (lds_void_pp*)(base + A_BYTES + (wave + NW * j) * 1024), 16, 0, 0);
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

  const uint32_t lds0 = lds_addr(smem);
  auto read_chunk = [&](int buf, int kk, half8v(&fa)[FN], half8v(&fb)[FM]) {
    const uint32_t base = lds0 + buf * STAGE;
    const int ch = fch + 4 * kk;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int row = wn * TN + i * 16 + frow;
      fa[i] = lds_read_b128(base + row * 128 + ((ch ^ pers_swz(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int row = wm * TM + j * 16 + frow;
      fb[j] = lds_read_b128(base + A_BYTES + row * 128 + ((ch ^ pers_swz(row)) << 4));
    }
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

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

  // ---- compute side ------------------------------------------------------------------
  int k = 0, s = 0;
  int c_n0 = 0, c_m0 = 0;
  auto set_compute_tile = [&](int kk) {
    const int lid = xcd_remap((int)blockIdx.x + kk * grid, ntiles);
    const int tm = lid / a.tiles_n, tn = lid - (lid / a.tiles_n) * a.tiles_n;
    c_n0 = tn * BN;
    c_m0 = tm * BM;
  };
  set_compute_tile(0);
  half4v rv[FN][FM];
  auto load_res = [&]() {   // residual of the compute tile, untracked, every lane issues
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = c_n0 + wn * TN + i * 16 + fch * 4;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = c_m0 + wm * TM + j * 16 + frow;
        const size_t off = (m < a.M && n < a.Cout) ? (size_t)m * a.Cout + n : 0;
        rv[i][j] = gload_b64_untracked(a.res + off);
      }
    }
  };

  // prologue: stage 0 landed and visible, stage 1 in flight
  set_issue_tile(0);
  issue(0);
  pers_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (total > 1) issue(1);

  half8v fa0[FN], fb0[FM], fa1[FN], fb1[FM];
  read_chunk(0, 0, fa0, fb0);
  int buf = 0;
  int young = 0;   // vector-memory ops this wave issued after the DMA of the next stage (0 / NRES / NST)
  for (int gc = 0; gc < total; ++gc) {
    read_chunk(buf, 1, fa1, fb1);
    lds_waitcnt<NR>();
    mfmas(fa0, fb0);
    const int nbuf = buf ^ 1;
    int young_now = 0;
    bool dma_now = false;
    if (gc + 1 < total) {
      // the DMA of stage gc+1 landed; the loads / stores issued after it may stay in flight
      if (young == 0) {
        pers_vmcnt<0>();
      } else if (PREF && young == NRES) {
        pers_vmcnt<(PREF ? NRES : 0)>();
      } else {
        pers_vmcnt<NST>();
      }
      lds_waitcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (gc + 2 < total) {
        issue(buf);
        dma_now = true;
      }
      if constexpr (PREF) {
        if (s == nK - 2) {        // epilogue operands one stage ahead
          load_res();
          young_now = NRES;
        }
      }
      read_chunk(nbuf, 0, fa0, fb0);
    } else {
      lds_waitcnt<0>();
    }
    mfmas(fa1, fb1);
    if (s == nK - 1) {
      // ---- epilogue of tile k: bias (LDS) + residual (+ReLU), buffer stores ----------
      if constexpr (HAS_RES) {
        if constexpr (PREF) {
          if (dma_now) pers_vmcnt<G>(); else pers_vmcnt<0>();
        } else {
          load_res();
          pers_vmcnt<0>();
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) reg_tie(rv[i][j]);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = c_n0 + wn * TN + i * 16 + fch * 4;
        const int nb = n < a.Cout ? n : 0;
        half8v braw = lds_read_b128(lds_addr(bias_lds + nb));
        lds_waitcnt<0>();
        lds_tie(braw);
        const float4v bv = __builtin_bit_cast(float4v, braw);
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int m = c_m0 + wm * TM + j * 16 + frow;
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
          const bool ok = m < a.M && n < a.Cout;
          const unsigned off = ok ? ((unsigned)m * (unsigned)a.ldy + (unsigned)n) * OUT_BYTES : 0x80000000u;
          if constexpr (OUT_F32) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), out_rsrc, off, 0, 0);
          } else {
            half4v o;
            o[0] = (half_t)v[0];
            o[1] = (half_t)v[1];
            o[2] = (half_t)v[2];
            o[3] = (half_t)v[3];
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), out_rsrc, off, 0, 0);
          }
          acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
        }
      }
      young_now = NST;
      ++k;
      s = 0;
      if (k < my_tiles) set_compute_tile(k);
    } else {
      ++s;
    }
    young = young_now;
    buf = nbuf;
  }
}

template <int BN, int BM, int WN, int WM, int MINB, bool R, bool F>
static void pers_cfg(ConvArgs a, hipStream_t st) {
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.cblk = a.C / 64;
  a.nK = a.KH * a.KW * a.cblk;
  const int ntiles = a.tiles_n * a.tiles_m;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int slots = MINB * cus;                     // co-resident workgroups
  const int grid = ntiles < slots ? ntiles : slots;
  const size_t lds = (size_t)2 * (BN + BM) * 128 + (size_t)a.Cout * 4;
  auto kern = conv_pers_kernel<BN, BM, WN, WM, MINB, R, F>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, st, a);
}

bool conv_pers_supported(const ConvArgs& a, bool out_f32) {
  const long out_bytes = (long)a.M * a.ldy * (out_f32 ? 4 : 2);
  return a.C % 64 == 0 && a.KH * a.KW * (a.C / 64) >= 2 && out_bytes < (1L << 31) && a.Cout <= 4096;
}

// Tile table (ids 70-73; 512 threads, BK = 64, 2-deep ring, persistent):
//   70: 128x128, waves 2x4 (64x32), 64 KiB + bias, 2 workgroups/CU
//   71: 128x64,  waves 2x4 (64x16), 48 KiB + bias, 2 workgroups/CU
//   72: 128x256, waves 2x4 (64x64), 96 KiB + bias, 1 workgroup/CU
//   73: 64x128,  waves 1x8 (64x16), 48 KiB + bias, 2 workgroups/CU
template <bool R, bool F>
static bool pers_dispatch(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 70: pers_cfg<128, 128, 2, 4, 2, R, F>(a, st); return true;
    case 71: pers_cfg<128, 64, 2, 4, 2, R, F>(a, st); return true;
    case 72: pers_cfg<128, 256, 2, 4, 1, R, F>(a, st); return true;
    case 73: pers_cfg<64, 128, 1, 8, 2, R, F>(a, st); return true;
    default: return false;
  }
}

bool conv_pers_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st) {
  if (!conv_pers_supported(a, out_f32)) return false;
  const bool res = a.res != nullptr;
  if (res) return out_f32 ? pers_dispatch<true, true>(a, tile, st) : pers_dispatch<true, false>(a, tile, st);
  return out_f32 ? pers_dispatch<false, true>(a, tile, st) : pers_dispatch<false, false>(a, tile, st);
}

}  // namespace idunno
