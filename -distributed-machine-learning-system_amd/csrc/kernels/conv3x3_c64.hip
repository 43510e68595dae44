// 3x3 / stride 1 / pad 1 convolution, 64 -> 64 channels (ResNet layer1: every
// conv of ResNet18/34 layer1 and the 3x3 of each ResNet50 layer1 bottleneck).
//
// Why a dedicated kernel: with N = Cout = 64 the im2col kernels (conv_glds.hip)
// fetch 24 KiB per 1 MFLOP stage (64 weight rows + 128 pixel rows of 128 B)
// and run at the chip's L2->CU fetch rate (~20 B/clk/CU measured: 525 TF/s on
// layer1 vs ~800 TF/s at Cout >= 128, profiles/r1_v5_layer_sweep_persist.log).
// Here each CU keeps ALL 9 x 64 x 64 weights (72 KiB) resident in LDS for the
// whole launch (persistent, one workgroup per CU) and fetches each spatial
// tile's halo patch ONCE for all nine taps:
//   tile = 8 rows x 32 cols of one image (256 px), patch = 10 x 34 px x 128 B
//   = 42.5 KiB per 18.9 MFLOP  ->  ~430 FLOP per fetched byte (10x im2col).
// The patch of tile i+1 is DMA'd (global_load_lds_dwordx4, padding from a zero
// buffer) into the second buffer while tile i runs its 9 taps x 2 K-chunks.
//
// MFMA: v_mfma_f32_16x16x32_f16, weights = A (rows = output channels), pixels
// = B.  The B fragment row of output pixel (oy, ox) for tap (kh, kw) is patch
// row (oy + kh) * PW + ox + kw: a per-lane base plus a wave-uniform offset.
// A fragment's 16 pixels lie in one output row (TW = 32), so its B rows are 16
// CONSECUTIVE patch rows; 128-byte LDS rows (64 fp16 channels) with 16-byte
// chunks XOR-swizzled by (row & 6) make every such read, at any row offset,
// conflict-free for ds_read_b128's lane groups (searched exhaustively; the
// (row >> 1) & 7 swizzle of the im2col kernels is 2-way conflicted here).
// W = 56 leaves 8 of the second x-tile's 32 columns empty.  That tile (valid
// width 17..24) runs in PAIRED mode: 8 full fragments (row r, columns 0..15)
// plus 4 fragments that each take columns 16..23 of a row PAIR (lanes 0..7 row
// 2j, lanes 8..15 row 2j+1 at columns rotated by 6, which keeps every
// ds_read_b128 lane group on 8 distinct row residues, i.e. conflict-free):
// 12 fragments, 3 per wave, instead of 16 (-25 % MFMAs on half the tiles).
//
// Workgroup = 8 waves (2 x 4, two per SIMD): wave = 32 output channels (2 A
// frags) x 64 pixels (4 B frags) -> 8 MFMAs per K-chunk of 32, 144 per tile;
// the fragments of the next K-chunk are read while the current one's MFMAs
// run (register double buffer), so LDS latency hides behind MFMA issue.
// LDS = 72 KiB weights + 2 x 43 KiB patch buffers = 158 KiB (1 workgroup/CU).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_q;
typedef __attribute__((address_space(1))) void glb_void_q;

namespace c64 {
constexpr int C = 64, CO = 64;
constexpr int TH = 8, TW = 32;                 // output tile
constexpr int PH = TH + 2, PW = TW + 2;        // patch 10 x 34
constexpr int PROWS = PH * PW;                 // 340 patch rows
constexpr int NW = 8, WN = 2, WM = 4;
constexpr int FN = 2, FM = 4;                  // wave: 32 couts x 64 px
constexpr int P_TOT = (PROWS + 7) / 8;         // 43 patch DMA instructions (8 rows each)
constexpr int P_HI = P_TOT % NW;               // waves [0, P_HI) issue one more
constexpr int P_INS = (P_TOT + NW - 1) / NW;   // 6 (waves >= P_HI: 5)
constexpr int PBUF = P_TOT * 1024;             // 43 KiB per patch buffer
constexpr int W_BYTES = 9 * CO * C * 2;        // 72 KiB
constexpr int W_INS = W_BYTES / 1024 / NW;     // 9 weight DMA instructions per wave
constexpr int LDS = W_BYTES + 2 * PBUF;
static_assert(LDS <= 160 * 1024, "fits one CU's LDS");
static_assert(WM * FM * 16 == TH * TW && TW % 16 == 0, "pixel fragments cover the tile, one row each");
}  // namespace c64

struct C64Args {
  const half_t* x;     // NHWC [B][H][W][64]
  const half_t* w;     // [64][3][3][64]
  const float* bias;   // [64]
  const half_t* res;   // NHWC [B][H][W][64] or nullptr
  half_t* y;           // NHWC [B][H][W][64]
  const void* zero;
  int B, H, W;
  int tiles_x, tiles_y, ntiles;
  int relu;
  int pair_tx;         // x-tile run in paired mode (valid width 17..24), -1: none
};

// Tile-local pixel of lane `frow` of fragment f of wave wm: 4 fragments per
// wave (one row of 16 columns each), or (FMX 3) the paired map of the header.
template <int FMX>
__device__ __forceinline__ void c64_pix(int wm, int f, int frow, int& py, int& px) {
  using namespace c64;
  if constexpr (FMX == FM) {
    const int p = (wm * FM + f) * 16 + frow;
    py = p / TW;
    px = p % TW;
  } else {
    const int k = wm * FMX + f;
    if (k < TH) {
      py = k;
      px = frow;
    } else {
      py = 2 * (k - TH) + (frow >> 3);
      px = 16 + (frow < 8 ? frow : ((frow + 6) & 7));
    }
  }
}


// Patch DMA of tile t into dst: 8 patch rows per instruction, rows past the
// patch or outside the image load the zero buffer.
__device__ __forceinline__ void c64_issue_patch(const C64Args& a, int t, char* __restrict__ dst, int wave,
                                                int lrow, int lslot) {
  using namespace c64;
  const half_t* zero = reinterpret_cast<const half_t*>(a.zero);
  const int per = a.tiles_x * a.tiles_y;
  const int b = t / per, r = t - b * per;
  const int ih0 = (r / a.tiles_x) * TH - 1, iw0 = (r % a.tiles_x) * TW - 1;
#pragma unroll
  for (int j = 0; j < P_INS; ++j) {
    const int i = wave + NW * j;
    if (i >= P_TOT) break;                       // wave-uniform
    const int row = i * 8 + lrow;
    const int py = row / PW, px = row - py * PW;
    const int ih = ih0 + py, iw = iw0 + px;
    const bool ok = row < PROWS && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    const half_t* src = ok ? a.x + (((size_t)b * a.H + ih) * a.W + iw) * C + ((lslot ^ c64_swz(row)) << 3) : zero;
    __builtin_amdgcn_global_load_lds((glb_void_q*)src, (lds_void_q*)(dst + i * 1024), 16, 0, 0);
  }
}

// One output tile.  Fragment reads go through inline asm (lds_read_b128) and
// the residual through untracked asm loads issued one tile ahead: a ds_read or
// a load the compiler tracks itself gets an `s_waitcnt vmcnt(0)` in front of it
// (or of its first use) while the patch DMA of tile t+1 is in flight, and that
// prefetch would never overlap tile t's MFMAs.
// Residual of tile t -> registers (untracked asm loads; masked pixels read row 0).
// Branch-free over the tile's mode: an untracked load issued inside a branch
// has its result copied into the merged register at the join, before it lands.
__device__ __forceinline__ bool c64_paired(const C64Args& a, int t) {
  return (t % (a.tiles_x * a.tiles_y)) % a.tiles_x == a.pair_tx;
}

__device__ __forceinline__ void c64_load_res(const C64Args& a, int t, half4v (&rv)[c64::FN][c64::FM], int wn,
                                             int wm, int lane) {
  using namespace c64;
  const int frow = lane & 15, fch = lane >> 4;
  const int per = a.tiles_x * a.tiles_y;
  const int b = t / per, r = t - b * per;
  const int oh0 = (r / a.tiles_x) * TH, ow0 = (r % a.tiles_x) * TW;
  const bool paired = (r % a.tiles_x) == a.pair_tx;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const int n = wn * (FN * 16) + i * 16 + fch * 4;
      int py, px, qy = TH, qx = 0;                 // paired mode has FM - 1 fragments
      c64_pix<FM>(wm, f, frow, py, px);
      if (f < FM - 1) c64_pix<FM - 1>(wm, f, frow, qy, qx);
      const int oh = oh0 + (paired ? qy : py), ow = ow0 + (paired ? qx : px);
      const size_t m = (oh < a.H && ow < a.W) ? (((size_t)b * a.H + oh) * a.W + ow) : 0;
      rv[i][f] = gload_b64_untracked(a.res + m * CO + n);
    }
}

// Head of one tile: the barrier, then the patch DMA and residual of tile t+1.
// Kept out of the mode branch below (the untracked residual loads must not be
// merged at a join).
template <bool HAS_RES>
__device__ __forceinline__ void c64_tile_head(const C64Args& a, int t, bool prefetch, char* __restrict__ nxt,
                                              half4v (&rv_next)[c64::FN][c64::FM], int wave, int wn, int wm,
                                              int lane) {
  const int lrow = lane >> 3, lslot = lane & 7;
  // One barrier per tile.  Every wave reaches it after (a) its MFMAs of tile
  // t-1 (so `nxt`, tile t-1's patch, is free) and (b) its `vmcnt(0)` behind
  // those MFMAs (so its DMAs of tile t's patch, issued a whole tile earlier,
  // have landed).  The wait sits AFTER the MFMAs, not before them: vmcnt also
  // counts the epilogue stores of the previous tile, and a wait in front of
  // the MFMAs would expose their write latency on every tile.
  __builtin_amdgcn_s_barrier();
  if (prefetch) {
    c64_issue_patch(a, t + 1, nxt, wave, lrow, lslot);
    if constexpr (HAS_RES) c64_load_res(a, t + 1, rv_next, wn, wm, lane);
  }
}

// MFMAs and epilogue of one tile, FMX pixel fragments per wave (4, or 3 in the
// paired mode).
template <bool HAS_RES, int FMX>
__device__ __forceinline__ void c64_tile(const C64Args& a, int t, const char* __restrict__ wl,
                                         const char* __restrict__ cur, const float4v* bvr, const int* pbase,
                                         const half4v (&rv)[c64::FN][c64::FM], int wn, int wm, int lane) {
  using namespace c64;
  const int frow = lane & 15, fch = lane >> 4;
  float4v acc[FN][FMX];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FMX; ++f) acc[i][f] = float4v{0.f, 0.f, 0.f, 0.f};

  // 18 K-chunks (9 taps x 2 halves of 64 channels); fragments of chunk q+1 are
  // read (inline-asm ds_read_b128, common.h) into the other register set before
  // chunk q's MFMAs are issued; a counted lgkmcnt wait retires exactly chunk q
  constexpr int NR = FN + FMX;                   // ds_reads per chunk
  const uint32_t wl_a = lds_addr(wl), cur_a = lds_addr(cur);
  // keep the 72 per-(fragment, tap) B addresses from being hoisted out of the tile
  // loop into registers (they spill at 2 waves/SIMD); recomputing them is 3 VALU
  int pb[FMX];
#pragma unroll
  for (int f = 0; f < FMX; ++f) {
    pb[f] = pbase[f];
    asm volatile("" : "+v"(pb[f]));
  }
  half8v fa[2][FN], fb[2][FMX];
  auto load_frags = [&](int q, half8v* a_, half8v* b_) {
    const int tap = q >> 1, kk = q & 1;
    const int toff = (tap / 3) * PW + (tap % 3);
    const uint32_t wt = wl_a + tap * (CO * 128);
    const int ch = fch + 4 * kk;
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int row = wn * (FN * 16) + i * 16 + frow;
      a_[i] = lds_read_b128(wt + row * 128 + ((ch ^ c64_swz(row)) << 4));
    }
#pragma unroll
    for (int f = 0; f < FMX; ++f) {
      const int row = pb[f] + toff;
      b_[f] = lds_read_b128(cur_a + row * 128 + ((ch ^ c64_swz(row)) << 4));
    }
  };
  load_frags(0, fa[0], fb[0]);
#pragma unroll
  for (int q = 0; q < 18; ++q) {
    half8v* ca = fa[q & 1];
    half8v* cb = fb[q & 1];
    if (q + 1 < 18) {
      load_frags(q + 1, fa[(q + 1) & 1], fb[(q + 1) & 1]);
      lds_waitcnt<NR>();
    } else {
      lds_waitcnt<0>();
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) lds_tie(ca[i]);
#pragma unroll
    for (int f = 0; f < FMX; ++f) lds_tie(cb[f]);
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < FMX; ++f)
        acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ca[i], cb[f], acc[i][f], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  // patch and residual of tile t+1 (issued before the MFMAs), this tile's
  // residual and the previous tile's stores: all had a tile of MFMAs to land
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: bias (+residual) (+ReLU); the two 16-cout fragments of a
  // pixel fragment swap halves (f16_pair_off) -> one 16-byte NHWC store a lane
  const int per = a.tiles_x * a.tiles_y;
  const int b = t / per, r = t - b * per;
  const int oh0 = (r / a.tiles_x) * TH, ow0 = (r % a.tiles_x) * TW;
  static_assert(FN == 2, "fragment pair");
#pragma unroll
  for (int f = 0; f < FMX; ++f) {
    int py, px;
    c64_pix<FMX>(wm, f, frow, py, px);
    const int oh = oh0 + py, ow = ow0 + px;
    half4v o[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float4v v = acc[i][f] + bvr[i];
      if constexpr (HAS_RES) {
        const half4v rr = rv[i][f];
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
      o[i][0] = (half_t)v[0];
      o[i][1] = (half_t)v[1];
      o[i][2] = (half_t)v[2];
      o[i][3] = (half_t)v[3];
    }
    const u32x4_sw w = split_swap_out(o[0], o[1]);     // every lane swaps
    if (oh >= a.H || ow >= a.W) continue;
    const size_t m = ((size_t)b * a.H + oh) * a.W + ow;
    *reinterpret_cast<u32x4_sw*>(a.y + m * CO + f16_pair_off(wn * (FN * 16), fch)) = w;
  }
}

template <bool HAS_RES>
__global__ void __launch_bounds__(512, 1) conv3x3_c64_kernel(const C64Args a) {
  using namespace c64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int lrow = lane >> 3, lslot = lane & 7;

  // contiguous tile range per workgroup (neighbouring tiles share halo rows in L2)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int t_begin = (int)((long long)bid * a.ntiles / gridDim.x);
  const int t_end = (int)((long long)(bid + 1) * a.ntiles / gridDim.x);
  if (t_begin >= t_end) return;

  // bias -> registers before any DMA is in flight (no load to wait for later)
  const int fch = lane >> 4;
  float4v bvr[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) bvr[i] = *reinterpret_cast<const float4v*>(a.bias + wn * (FN * 16) + i * 16 + fch * 4);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(bvr[0]), "+v"(bvr[1])::"memory");

  // ---- all weights -> LDS, once: instruction i = (tap, 8 cout rows) ---------------
#pragma unroll
  for (int j = 0; j < W_INS; ++j) {
    const int i = wave + NW * j;                 // 0..71
    const int tap = i >> 3, row = (i & 7) * 8 + lrow;   // cout row within the tap slice
    const half_t* src = a.w + (size_t)row * (9 * C) + tap * C + ((lslot ^ c64_swz(row)) << 3);
    __builtin_amdgcn_global_load_lds((glb_void_q*)src, (lds_void_q*)(smem + i * 1024), 16, 0, 0);
  }

  // per-lane B fragment bases: output pixel -> patch row of tap (0, 0), for the
  // plain and the paired fragment map
  const int frow = lane & 15;
  int pbase[FM], pbase3[FM - 1];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    int py, px;
    c64_pix<FM>(wm, f, frow, py, px);
    pbase[f] = py * PW + px;
  }
#pragma unroll
  for (int f = 0; f < FM - 1; ++f) {
    int py, px;
    c64_pix<FM - 1>(wm, f, frow, py, px);
    pbase3[f] = py * PW + px;
  }

  char* p0 = smem + W_BYTES;
  char* p1 = p0 + PBUF;
  half4v rA[FN][FM], rB[FN][FM];                 // residual of the current / next tile
  c64_issue_patch(a, t_begin, p0, wave, lrow, lslot);
  if constexpr (HAS_RES) c64_load_res(a, t_begin, rA, wn, wm, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // weights + first patch (+ residual) landed
  // one tile in its mode (wave-uniform branch); two tiles per trip so the
  // buffers and residual registers swap statically
  auto tile = [&](int t, bool more, const char* cur, char* nxt, half4v(&rv)[FN][FM], half4v(&rvn)[FN][FM]) {
    c64_tile_head<HAS_RES>(a, t, more, nxt, rvn, wave, wn, wm, lane);
    if (c64_paired(a, t))
      c64_tile<HAS_RES, FM - 1>(a, t, smem, cur, bvr, pbase3, rv, wn, wm, lane);
    else
      c64_tile<HAS_RES, FM>(a, t, smem, cur, bvr, pbase, rv, wn, wm, lane);
  };
  for (int t = t_begin; t < t_end; t += 2) {
    tile(t, t + 1 < t_end, p0, p1, rA, rB);
    if (t + 1 < t_end) tile(t + 1, t + 2 < t_end, p1, p0, rB, rA);
  }
}

bool conv3x3_c64_supported(int C, int Cout) { return C == c64::C && Cout == c64::CO; }

void conv3x3_c64_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                        const void* zero, int B, int H, int W, int relu, hipStream_t st) {
  using namespace c64;
  C64Args a{};
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.B = B;
  a.H = H;
  a.W = W;
  a.relu = relu;
  a.tiles_x = (W + TW - 1) / TW;
  a.tiles_y = (H + TH - 1) / TH;
  a.ntiles = B * a.tiles_x * a.tiles_y;
  const int last_w = W - (a.tiles_x - 1) * TW;   // valid width of the last x-tile
  a.pair_tx = (last_w > 16 && last_w <= 24) ? a.tiles_x - 1 : -1;
  // LDS opt-in and CU count per (kernel, device), thread-safe (launch_util.h)
  ensure_lds_attr(reinterpret_cast<const void*>(&conv3x3_c64_kernel<true>), LDS);
  ensure_lds_attr(reinterpret_cast<const void*>(&conv3x3_c64_kernel<false>), LDS);
  const int cus = device_cu_count();
  const int grid = a.ntiles < cus ? a.ntiles : cus;   // persistent, one workgroup per CU
  if (res)
    hipLaunchKernelGGL(conv3x3_c64_kernel<true>, dim3(grid), dim3(64 * NW), LDS, st, a);
  else
    hipLaunchKernelGGL(conv3x3_c64_kernel<false>, dim3(grid), dim3(64 * NW), LDS, st, a);
}

}  // namespace idunno
