// Implicit-GEMM convolution on CDNA4 matrix cores (v_mfma_f32_16x16x32_f16).
//
// Replaces the ATen conv2d / batch_norm / relu / add chain that the reference
// runs op-by-op at batch 1 (reference alexnet_resnet.py:67-75 via torch.hub
// models; op inventory in SURVEY.md §2.4).  Here one launch computes
//
//     y[m, n] = act( sum_k x_im2col[m, k] * w[n, k] + bias[n] (+ res[m, n]) )
//
// with BN already folded into (w, bias) on the host, ReLU and the residual add
// fused into the epilogue, activations in NHWC fp16 and fp32 accumulation.
//
// GEMM view: m = output pixel (b, oh, ow) [M = B*Ho*Wo], n = output channel,
// k = (kh, kw, c).  The MFMA is issued "transposed": weights are the MFMA A
// operand (rows = n) and pixels the B operand (cols = m), so each lane ends up
// holding 4 *consecutive output channels* of one pixel and the NHWC store is a
// packed 8-byte write instead of four scattered 2-byte writes.
//
// Two K-orderings:
//   * BIG  (C % 64 == 0): one K stage = 64 channels of a single (kh, kw) tap,
//          so each pixel row of the stage is one contiguous 128-byte run.
//   * SMALL (C == 4, the RGB(+pad) stems): one K stage = one kh row of 8 taps
//          x 4 channels = 32 halfs; taps beyond KW carry zero weights.  Each
//          16-byte chunk covers two taps, loaded as two 8-byte halves with
//          independent bounds checks.
//
// Pipeline: register-staged, double-buffered LDS.  Global loads for stage s+1
// are issued before the MFMAs of stage s and written to the other LDS buffer
// after them (async-STAGE split, cdna_hip_programming §5.5 T14), one barrier
// per stage.  LDS rows are XOR-swizzled at 16-byte granularity so the
// ds_read_b128 fragment reads are bank-conflict free (derivation in
// docs/KERNELS.md).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {


// g(q) for 64-byte rows, chosen so that every ds_read_b128 lane group of a
// 16x16x32 fragment read touches 16 distinct 16-byte bank slots.
__device__ __forceinline__ int swz64(int row) {
  const int q = (row >> 2) & 3;
  // q:0->0, 1->2, 2->3, 3->1   packed 2 bits each: 0b01'11'10'00 = 0x78
  return (0x78 >> (2 * q)) & 3;
}
__device__ __forceinline__ int swz128(int row) { return (row >> 1) & 7; }

template <int CPR>
__device__ __forceinline__ int swizzle(int row) {
  if constexpr (CPR == 8) return swz128(row);
  else return swz64(row);
}

template <int BN, int BM, int BK, int WN, int WM, bool SMALL, bool HAS_RES, bool OUT_F32>
__global__ void __launch_bounds__(256, 2) conv_igemm_kernel(const ConvArgs a) {
  static_assert(WN * WM == 4, "4 waves per workgroup");
  constexpr int TN = BN / WN, TM = BM / WM;       // wave tile
  constexpr int FN = TN / 16, FM = TM / 16;       // 16x16 fragments per wave
  constexpr int CPR = BK / 8;                     // 16-byte chunks per LDS row
  constexpr int RB = BK * 2;                      // bytes per LDS row
  constexpr int A_CHUNKS = BN * CPR / 256;        // per thread per stage
  constexpr int B_CHUNKS = BM * CPR / 256;
  static_assert(A_CHUNKS >= 1 && B_CHUNKS >= 1, "tile too small");
  static_assert(!SMALL || BK == 32, "small-C path uses 32-wide stages");
  constexpr int A_BYTES = BN * RB, B_BYTES = BM * RB;
  constexpr int STAGE_BYTES = A_BYTES + B_BYTES;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wn = wave / WM, wm = wave % WM;

  // Tile coordinates: n-tiles of one m-tile are consecutive logical ids so
  // they share an XCD (and its L2 copy of the activation panel).
  const int nwg = a.tiles_n * a.tiles_m;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tm = lid / a.tiles_n, tn = lid % a.tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;

  // ---- per-thread load descriptors (fixed over the K loop) ---------------
  // A (weights): chunk i = tid + 256*j -> row i / CPR, chunk i % CPR
  const half_t* a_src[A_CHUNKS];
  int a_lds[A_CHUNKS];
#pragma unroll
  for (int j = 0; j < A_CHUNKS; ++j) {
    const int i = tid + 256 * j;
    const int row = i / CPR, ch = i % CPR;
    const int n = n0 + row;
    a_src[j] = (n < a.Cout) ? a.w + (size_t)n * a.Kpad + ch * 8 : nullptr;
    a_lds[j] = row * RB + ((ch ^ swizzle<CPR>(row)) << 4);
  }
  // B (pixels)
  int b_base[B_CHUNKS];   // element offset of (b, 0, 0, 0) in x, or -1 if m >= M
  int b_ih0[B_CHUNKS], b_iw0[B_CHUNKS];
  int b_ch[B_CHUNKS], b_lds[B_CHUNKS];
#pragma unroll
  for (int j = 0; j < B_CHUNKS; ++j) {
    const int i = tid + 256 * j;
    const int row = i / CPR, ch = i % CPR;
    const int m = m0 + row;
    if (m < a.M) {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw, r = m - b * hw;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      b_base[j] = b * a.H * a.W * a.C;
      b_ih0[j] = oh * a.stride - a.pad;
      b_iw0[j] = ow * a.stride - a.pad;
    } else {
      b_base[j] = -1;
      b_ih0[j] = 0;
      b_iw0[j] = 0;
    }
    b_ch[j] = ch;
    b_lds[j] = A_BYTES + row * RB + ((ch ^ swizzle<CPR>(row)) << 4);
  }

  vec16 ra[A_CHUNKS], rb[B_CHUNKS];

  auto load_stage = [&](int s) {
#pragma unroll
    for (int j = 0; j < A_CHUNKS; ++j)
      ra[j] = a_src[j] ? *reinterpret_cast<const vec16*>(a_src[j] + s * BK) : zero16();
    if constexpr (!SMALL) {
      const int tap = s / a.cblk, cb = s - tap * a.cblk;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
#pragma unroll
      for (int j = 0; j < B_CHUNKS; ++j) {
        const int ih = b_ih0[j] + kh, iw = b_iw0[j] + kw;
        const bool ok = b_base[j] >= 0 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        rb[j] = ok ? *reinterpret_cast<const vec16*>(a.x + b_base[j] + (ih * a.W + iw) * a.C +
                                                     cb * BK + b_ch[j] * 8)
                   : zero16();
      }
    } else {
      const int kh = s / a.nsub, sub = s - kh * a.nsub;
#pragma unroll
      for (int j = 0; j < B_CHUNKS; ++j) {
        const int ih = b_ih0[j] + kh;
        const int iw = b_iw0[j] + sub * 8 + b_ch[j] * 2;
        const bool rok = b_base[j] >= 0 && (unsigned)ih < (unsigned)a.H;
        const half_t* p = a.x + b_base[j] + (ih * a.W + iw) * 4;
        vec8 lo{0u, 0u}, hi{0u, 0u};
        if (rok && (unsigned)iw < (unsigned)a.W) lo = *reinterpret_cast<const vec8*>(p);
        if (rok && (unsigned)(iw + 1) < (unsigned)a.W) hi = *reinterpret_cast<const vec8*>(p + 4);
        rb[j] = vec16{lo.x, lo.y, hi.x, hi.y};
      }
    }
  };
  auto store_stage = [&](int buf) {
    char* base = smem + buf * STAGE_BYTES;
#pragma unroll
    for (int j = 0; j < A_CHUNKS; ++j) *reinterpret_cast<vec16*>(base + a_lds[j]) = ra[j];
#pragma unroll
    for (int j = 0; j < B_CHUNKS; ++j) *reinterpret_cast<vec16*>(base + b_lds[j]) = rb[j];
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // Fragment read offsets (row = l & 15 within a 16-row fragment, chunk = l >> 4).
  const int frow = lane & 15, fch = lane >> 4;

  load_stage(0);
  store_stage(0);
  __syncthreads();

  for (int s = 0; s < a.nK; ++s) {
    const int cur = s & 1;
    const bool more = (s + 1) < a.nK;
    if (more) load_stage(s + 1);

    const char* base = smem + cur * STAGE_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = fch + 4 * kk;
      half8v fa[FN], fb[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * TN + i * 16 + frow;
        fa[i] = *reinterpret_cast<const half8v*>(base + row * RB + ((ch ^ swizzle<CPR>(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int row = wm * TM + j * 16 + frow;
        fb[j] = *reinterpret_cast<const half8v*>(base + A_BYTES + row * RB +
                                                 ((ch ^ swizzle<CPR>(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }

    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: bias (+residual) (+ReLU), NHWC store --------------------
  // acc[i][j] lane l: pixel col = l & 15, channels rows (l>>4)*4 + r.
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
      if constexpr (HAS_RES) {
        const half4v r = *reinterpret_cast<const half4v*>(a.res + (size_t)m * a.Cout + n);
        v[0] += (float)r[0];
        v[1] += (float)r[1];
        v[2] += (float)r[2];
        v[3] += (float)r[3];
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

// ---------------------------------------------------------------------------
// Host-side launch: tile table per layer shape (SURVEY.md §7.3 hard part 1:
// "a single tile config will not fit all of them").
// ---------------------------------------------------------------------------
template <int BN, int BM, int BK, int WN, int WM, bool SMALL, bool HAS_RES, bool OUT_F32>
static void launch_cfg(ConvArgs a, hipStream_t st) {
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  const int grid = a.tiles_n * a.tiles_m;
  const size_t lds = 2 * (size_t)(BN + BM) * BK * 2;
  // >64 KiB dynamic LDS needs an explicit opt-in, per (kernel, device): launch_util.h
  ensure_lds_attr(reinterpret_cast<const void*>(&conv_igemm_kernel<BN, BM, BK, WN, WM, SMALL, HAS_RES, OUT_F32>),
                  (int)lds);
  hipLaunchKernelGGL((conv_igemm_kernel<BN, BM, BK, WN, WM, SMALL, HAS_RES, OUT_F32>), dim3(grid),
                     dim3(256), lds, st, a);
}

template <bool SMALL, bool HAS_RES, bool OUT_F32>
static void launch_shape(ConvArgs a, int tile, hipStream_t st) {
  constexpr int BK = SMALL ? 32 : 64;
  switch (tile) {
    case 0: launch_cfg<64, 256, BK, 1, 4, SMALL, HAS_RES, OUT_F32>(a, st); break;
    case 1: launch_cfg<64, 128, BK, 1, 4, SMALL, HAS_RES, OUT_F32>(a, st); break;
    case 2: launch_cfg<128, 128, BK, 2, 2, SMALL, HAS_RES, OUT_F32>(a, st); break;
    default: launch_cfg<128, 64, BK, 2, 2, SMALL, HAS_RES, OUT_F32>(a, st); break;
  }
}

// Picks a tile so that the grid has enough workgroups to cover 256 CUs.
int conv_pick_tile(int M, int Cout) {
  auto blocks = [&](int bn, int bm) { return ((Cout + bn - 1) / bn) * ((M + bm - 1) / bm); };
  if (Cout % 128 == 0) {
    if (blocks(128, 128) >= 512) return 2;
    return 3;
  }
  if (blocks(64, 256) >= 1024) return 0;
  return 1;
}

void conv_igemm_launch(ConvArgs a, bool small, bool out_f32, int tile, hipStream_t st) {
  const bool res = a.res != nullptr;
  if (small) {
    if (res) launch_shape<true, true, false>(a, tile, st);
    else if (out_f32) launch_shape<true, false, true>(a, tile, st);
    else launch_shape<true, false, false>(a, tile, st);
  } else {
    if (res) {
      if (out_f32) launch_shape<false, true, true>(a, tile, st);
      else launch_shape<false, true, false>(a, tile, st);
    } else {
      if (out_f32) launch_shape<false, false, true>(a, tile, st);
      else launch_shape<false, false, false>(a, tile, st);
    }
  }
}

}  // namespace idunno
