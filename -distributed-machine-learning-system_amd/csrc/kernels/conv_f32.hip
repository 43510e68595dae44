// Reference-precision (fp32) implicit-GEMM convolution on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulate -- bit-for-bit
// a k-ordered fmaf chain, cdna_hip_programming §3 "FP32-input MFMA").
//
// The reference classifies with torchvision models in fp32
// (/root/reference/alexnet_resnet.py:17-22, 74-75); this kernel is the conv /
// FC engine of the framework's fp32 path (HipRunner dtype "fp32").
//
// Shape of the problem: f32 MFMA runs at 1/16 of the f16 rate (64 FLOP/clk per
// SIMD, 157 TF chip peak), so unlike the fp16 kernels this loop is
// compute-bound: a 128x128 tile at BK=16 needs 32 FLOP per staged byte, i.e.
// ~4.9 TB/s of L2->LDS traffic at peak, well inside what the fp16 kernels
// already sustain.  The design goal is therefore MFMA issue density: every
// wave owns a 64x64 (or 64x32) output sub-tile = 16 (8) independent 16x16
// accumulators, so the 40-cycle dependent latency of the 32-cycle-issue MFMA
// never shows, and the LDS ring (global_load_lds DMA, counted vmcnt, raw
// s_barrier -- the conv_glds.hip recipe) keeps NS-1 stages in flight.
//
// Fragment trick: v_mfma_f32_16x16x4_f32 takes ONE f32 of A and B per lane
// (lane l: A[row l&15][k l>>4], B[k l>>4][col l&15]).  A ds_read_b128 gives a
// lane 4 consecutive k of its row, so lane group g = l>>4 reads k = 4g..4g+3
// and MFMA t (t = 0..3) consumes element t: MFMA t sums k = {t, 4+t, 8+t, 12+t}
// and the four MFMAs cover k = 0..15 exactly once.  The LDS bytes a lane reads
// are then the same (row, 16-byte chunk) pattern as the f16 16x16x32 kernel,
// so the same XOR swizzle (tile_math.h swz_r) is bank-conflict free.
//
// LDS image per stage: A (weights, BN rows) then B (pixels, BM rows), each row
// BK floats (16 -> 64 B, 32 -> 128 B) in 16-byte chunks XOR-swizzled per row.
// Two K decompositions:
//   big   (C % BK == 0): stage = (kh, kw, channel block), chunk c = channels
//         4c..4c+3 of one input pixel;
//   small (C == 4, the RGB(+0) stems): stage = (kh, tap block of BK/4 taps),
//         chunk c = all 4 channels of tap kw = blk*BK/4 + c (one pixel), so a
//         7x7/11x11 stem streams whole pixels; padding taps read the zero
//         buffer and have zero weights.
//   pack3 (mode 2, RGB stems from preprocess_pack3_f32): the 3*KW floats of one
//         kernel row are contiguous in a packed row copy in which they start
//         16-byte aligned; K = (kh, chunk of 4 floats), ceil(3*KW/4) chunks per
//         kh, 4 chunks per stage.  The 7x7/2 ResNet stem: K 168 (+8 pad) vs 224
//         for NHWC4, the 11x11/4 AlexNet conv1: 400 vs 528.
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `pending` stages (G DMA ops each) of this wave are in flight
template <int G, int NS>
__device__ __forceinline__ void wait_ring(int pending) {
  if constexpr (NS >= 4) {
    if (pending >= 2) { wait_vm<2 * G>(); return; }
  }
  if constexpr (NS >= 3) {
    if (pending >= 1) { wait_vm<G>(); return; }
  }
  wait_vm<0>();
}

}  // namespace

template <int BN, int BM, int BK, int WN, int WM, int NS, bool HAS_RES, int KM>
__global__ void __launch_bounds__(64 * WN * WM) conv_f32_kernel(const ConvF32Args a) {
  constexpr bool SMALL = KM == 1, P3 = KM == 2;
  constexpr int NW = WN * WM;
  constexpr int TN = BN / WN, TM = BM / WM;
  constexpr int FN = TN / 16, FM = TM / 16;
  constexpr int CPR = BK / 4;                 // 16-byte chunks per row
  constexpr int RB = BK * 4;                  // bytes per row
  constexpr int RPI = 64 / CPR;               // rows per DMA instruction (1 KiB)
  constexpr int A_INS = BN / RPI, B_INS = BM / RPI;
  static_assert(BK == 16 || BK == 32, "BK 16 or 32 floats");
  static_assert(A_INS % NW == 0 && B_INS % NW == 0, "DMA instructions must split evenly over waves");
  constexpr int GA = A_INS / NW, GB = B_INS / NW, G = GA + GB;
  constexpr int A_BYTES = BN * RB, STAGE = (BN + BM) * RB;
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(G * (NS - 2) < 64, "vmcnt immediate");
  static_assert(KM == 0 || BK == 16, "small-C / pack3 stages are 16 floats");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;

  const int nwg = a.tiles_n * a.tiles_m;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int lid_all = xcd_remap(blockIdx.x, nwg * nsplit);
  const int split = lid_all / nwg, lid = lid_all - split * nwg;
  const int tm = lid / a.tiles_n, tn = lid % a.tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;
  const float* const xin = a.x + (size_t)split * a.kslice;         // split-K: this block's K slice
  const float* const win = a.w + (size_t)split * a.kslice;
  float* const yout = a.y + (size_t)split * a.ysplit;

  const float* zero = reinterpret_cast<const float*>(a.zero);
  const int lrow = lane / CPR, lslot = lane % CPR;

  // A (weights): per DMA instruction j of this wave, a row base (nullptr: row >= Cout)
  const float* a_src[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int row = (wave + NW * j) * RPI + lrow;
    const int n = n0 + row;
    a_src[j] = n < a.Cout ? win + (size_t)n * a.Kpad + (lslot ^ swz_r(row, CPR)) * 4 : nullptr;
  }
  // B (pixels): image base, top-left input coordinate and the lane's chunk
  const int ldx = a.ldx ? a.ldx : a.C;
  int b_base[GB], b_ih0[GB], b_iw0[GB];
  // pack3: this lane's (kh, chunk) of the stage being issued (advanced by 4
  // chunks per stage; cpk >= 4 is checked on the host)
  int p_kh[P3 ? GB : 1], p_q[P3 ? GB : 1];
  const int prow = a.nc * a.wp;                        // pack3: floats per image row (all copies)
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = (wave + NW * j) * RPI + lrow;
    const int m = m0 + row;
    const int ch = lslot ^ swz_r(row, CPR);
    if constexpr (P3) {
      p_kh[j] = 0;
      p_q[j] = ch;
    }
    if (m < a.M) {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw, r = m - b * hw;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      if constexpr (P3) {
        const int r0 = 3 * a.stride * ow;               // first float of the pixel's kernel row in R
        const int sh = r0 & 3, g = 4 / a.nc;            // copy sh/g starts it 16-byte aligned
        b_base[j] = b * a.H * prow + (sh / g) * a.wp + r0 - sh;
      } else {
        b_base[j] = b * a.H * a.W * ldx + (SMALL ? 0 : ch * 4);
      }
      b_ih0[j] = oh * a.stride - a.pad;
      b_iw0[j] = ow * a.stride - a.pad + (SMALL ? ch : 0);   // small: chunk = tap offset
    } else {
      b_base[j] = 0;
      b_ih0[j] = -(1 << 28);
      b_iw0[j] = -(1 << 28);
    }
  }

  // issue-side K coordinates (NS-1 stages ahead of compute):
  //   big:   (kh, kw, cb) with cb fastest   == weight K order (kh, kw, c)
  //   small: (kh, kb)     with kb fastest   == weight K order (kh, tap, c4)
  int i_s = 0, i_c = 0, i_kw = 0, i_kh = 0;
  auto issue = [&](int buf) {
    char* base = smem + buf * STAGE;
    const int koff = i_s * BK;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const float* src = a_src[j] ? a_src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      if constexpr (P3) {
        const int ih = b_ih0[j] + p_kh[j];
        const bool ok = p_kh[j] < a.KH && (unsigned)ih < (unsigned)a.H;
        const float* src = ok ? xin + b_base[j] + ih * prow + 4 * p_q[j] : zero;
        __builtin_amdgcn_global_load_lds((glb_void_t*)src,
                                         (lds_void_t*)(base + A_BYTES + (wave + NW * j) * 1024), 16, 0, 0);
        p_q[j] += CPR;
        if (p_q[j] >= a.cpk) {
          p_q[j] -= a.cpk;
          ++p_kh[j];
        }
        continue;
      }
      int ih, iw, coff;
      if constexpr (SMALL) {
        ih = b_ih0[j] + i_kh;
        iw = b_iw0[j] + i_c * CPR;
        coff = 0;
      } else {
        ih = b_ih0[j] + i_kh;
        iw = b_iw0[j] + i_kw;
        coff = i_c * BK;
      }
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const float* src = ok ? xin + b_base[j] + (ih * a.W + iw) * ldx + coff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src,
                                       (lds_void_t*)(base + A_BYTES + (wave + NW * j) * 1024), 16, 0, 0);
    }
    ++i_s;
    if (++i_c == a.cblk) {
      i_c = 0;
      if constexpr (SMALL) {
        ++i_kh;
      } else if (++i_kw == a.KW) {
        i_kw = 0;
        ++i_kh;
      }
    }
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // residual tile -> registers ahead of the ring (untracked loads, retired by
  // the ring's counted waits long before the epilogue; conv_glds.hip)
  float4v rv[HAS_RES ? FN : 1][HAS_RES ? FM : 1];
  if constexpr (HAS_RES) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = m0 + wm * TM + j * 16 + (lane & 15);
        const size_t off = (m < a.M && n < a.Cout) ? (size_t)m * a.Cout + n : 0;
        rv[i][j] = gload_f4_untracked(a.res + off);
      }
    }
  }

  const int nK = a.nK;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nK) issue(p);

  const int frow = lane & 15, fch = lane >> 4;
  constexpr int KK = BK / 16, NR = FN + FM;
  for (int s = 0; s < nK; ++s) {
    const int ahead = min(NS - 2, nK - 1 - s);
    wait_ring<G, NS>(ahead);
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < nK) issue((s + NS - 1) % NS);

    // fragment reads through inline asm (see common.h): all reads of the
    // stage go out first, each 16-deep K chunk waits only for its own
    const uint32_t base = lds_addr(smem) + (s % NS) * STAGE;
    float4v fa[KK][FN], fb[KK][FM];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int ch = fch + 4 * kk;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * TN + i * 16 + frow;
        fa[kk][i] = lds_read_f4(base + row * RB + ((ch ^ swz_r(row, CPR)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int row = wm * TM + j * 16 + frow;
        fb[kk][j] = lds_read_f4(base + A_BYTES + row * RB + ((ch ^ swz_r(row, CPR)) << 4));
      }
    }
    auto mfma_chunk = [&](int kk) {
#pragma unroll
      for (int i = 0; i < FN; ++i) lds_tie(fa[kk][i]);
#pragma unroll
      for (int j = 0; j < FM; ++j) lds_tie(fb[kk][j]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[kk][i][t], fb[kk][j][t], acc[i][j], 0, 0, 0);
    };
    if constexpr (KK == 2) {
      lds_waitcnt<NR>();
      mfma_chunk(0);
    }
    lds_waitcnt<0>();
    mfma_chunk(KK - 1);
  }

  // ---- epilogue: bias (+residual) (+ReLU), NHWC f32 store (16 B per lane) ----
  if constexpr (HAS_RES) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) reg_tie(rv[i][j]);
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
    if (n >= a.Cout) continue;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + j * 16 + (lane & 15);
      if (m >= a.M) continue;
      float4v v = acc[i][j] + bv;
      if constexpr (HAS_RES) v += rv[i][j];
      if (a.relu) {
        v[0] = fmaxf(v[0], 0.f);
        v[1] = fmaxf(v[1], 0.f);
        v[2] = fmaxf(v[2], 0.f);
        v[3] = fmaxf(v[3], 0.f);
      }
      *reinterpret_cast<float4v*>(yout + (size_t)m * a.ldy + n) = v;
    }
  }
}

template <int BN, int BM, int BK, int WN, int WM, int NS, bool R, int S>
static void f32_cfg(ConvF32Args a, hipStream_t st) {
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  if constexpr (S == 2) {
    a.cblk = 1;
    a.nK = (a.KH * a.cpk + BK / 4 - 1) / (BK / 4);
  } else if constexpr (S == 1) {
    a.cblk = a.nsub;                 // tap blocks per kh row
    a.nK = a.KH * a.nsub;
  } else {
    a.cblk = a.C / BK;
    a.nK = a.KH * a.KW * a.cblk;
  }
  const int grid = a.tiles_n * a.tiles_m * (a.ksplit > 1 ? a.ksplit : 1);
  const int lds = NS * (BN + BM) * BK * 4;
  auto kern = conv_f32_kernel<BN, BM, BK, WN, WM, NS, R, S>;
  ensure_lds_attr(reinterpret_cast<const void*>(kern), lds);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WN * WM), lds, st, a);
}

// Tile table (id -> config).  Ids are stable: the GPU tests sweep all of them.
//   100: 128x128, BK 16, 4 waves (2x2, 64x64 per wave), 3 stages   48 KiB
//   101: 128x128, BK 32, 4 waves (2x2),                 3 stages   96 KiB
//   102:  64x256, BK 16, 4 waves (1x4, 64x64 per wave), 3 stages   60 KiB
//   103: 128x64,  BK 16, 4 waves (2x2, 64x32 per wave), 3 stages   36 KiB
//   104: 256x128, BK 16, 8 waves (4x2, 64x64 per wave), 3 stages   72 KiB
//   105:  64x128, BK 16, 4 waves (1x4, 64x32 per wave), 3 stages   36 KiB
//   106: 128x256, BK 16, 8 waves (2x4, 64x64 per wave), 3 stages   72 KiB
//   107:  64x64,  BK 16, 4 waves (2x2, 32x32 per wave), 3 stages   24 KiB
//   108: 128x128, BK 16, 4 waves (2x2),                 4 stages   64 KiB
//   109:  64x256, BK 16, 4 waves (1x4, 64x64 per wave), 4 stages   80 KiB
// The small-C and pack3 (stem) paths support every id (all are BK 16) except 101.
template <bool R, int S>
static bool f32_dispatch(ConvF32Args a, int tile, hipStream_t st) {
  switch (tile) {
    case 100: f32_cfg<128, 128, 16, 2, 2, 3, R, S>(a, st); return true;
    case 101:
      if constexpr (S) return false;
      else { f32_cfg<128, 128, 32, 2, 2, 3, R, S>(a, st); return true; }
    case 102: f32_cfg<64, 256, 16, 1, 4, 3, R, S>(a, st); return true;
    case 103: f32_cfg<128, 64, 16, 2, 2, 3, R, S>(a, st); return true;
    case 104: f32_cfg<256, 128, 16, 4, 2, 3, R, S>(a, st); return true;
    case 105: f32_cfg<64, 128, 16, 1, 4, 3, R, S>(a, st); return true;
    case 106: f32_cfg<128, 256, 16, 2, 4, 3, R, S>(a, st); return true;
    case 107: f32_cfg<64, 64, 16, 2, 2, 3, R, S>(a, st); return true;
    case 108: f32_cfg<128, 128, 16, 2, 2, 4, R, S>(a, st); return true;
    case 109: f32_cfg<64, 256, 16, 1, 4, 4, R, S>(a, st); return true;
    default: return false;
  }
}

bool conv_f32_launch(ConvF32Args a, int mode, int tile, hipStream_t st) {
  const bool res = a.res != nullptr;
  if (mode == 2) return res ? f32_dispatch<true, 2>(a, tile, st) : f32_dispatch<false, 2>(a, tile, st);
  if (mode == 1) return res ? f32_dispatch<true, 1>(a, tile, st) : f32_dispatch<false, 1>(a, tile, st);
  return res ? f32_dispatch<true, 0>(a, tile, st) : f32_dispatch<false, 0>(a, tile, st);
}

// Default tile per (M, Cout, K = KH*KW*C), from the per-layer sweep on MI355X
// (tools/bench_layers_f32.py, profiles/r2_v1_layers_f32.md): 64x128 for the RGB
// stems (K <= 4*...: C == 4), 64x64 for short-K 1x1 convs (prologue-bound),
// 64x256 for Cout 64, 128x128 where it fills >= 4 waves of 256 CUs, else 128x64.
int conv_f32_pick(int M, int Cout, int K, bool small) {
  const long tiles128 = (long)((M + 127) / 128) * ((Cout + 127) / 128);
  if (small) return 105;
  if (K <= 256) return 107;
  if (Cout <= 64) return M >= 256 * 256 ? 102 : 105;
  if (tiles128 >= 1024) return 100;
  return 103;
}

}  // namespace idunno
