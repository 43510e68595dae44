// Persistent streaming 1x1 / stride-1 convolution (fp16 NHWC) for the
// memory-bound ResNet50 bottleneck layers (K = Cin 64 or 128).
//
// Why: at B = 1024 the 1x1 expansion convs (64 -> 256 with the residual, and
// the layer1 downsample) run at 47-60 % of HBM on the implicit-GEMM tiles
// (profiles/r3_resnet50_b1024_fp16_layer_roofline.md).  Their K loop is one or
// two stages, so each 128 x 128 block is a single memory round trip -- load,
// a few MFMAs, residual, store -- and with its epilogue traffic ablated the
// layer still takes 448 us for a 0.4 GB read (profiles/
// r3_resnet50_1x1_epilogue_ablation.log): the blocks are latency-bound.
// Here each workgroup stays resident and streams pixel tiles:
//   * its 4 waves each own 64 output channels and keep their weights in
//     REGISTERS for the whole launch (K = 64: 32 VGPRs);
//   * the 64-pixel input tile of the NEXT item is DMA'd (global_load_lds) into
//     the other half of a 2-tile LDS ring, and its residual is loaded into the
//     other half of a register double buffer, while the current item computes
//     and stores: every wait is a counted `s_waitcnt vmcnt(N)` that leaves the
//     younger loads and the previous item's stores in flight;
//   * epilogue stores are buffer stores issued by every lane (masked lanes
//     write past the descriptor's size and are dropped), so each wave issues
//     the same number of memory operations per item and the counts hold.
// Workgroup g takes cout slab g % nslab (256 channels) and every (G/nslab)-th
// pixel tile; the slabs of one tile are adjacent ids, placed on one XCD by
// xcd_remap so the second read of the tile hits that XCD's L2.
#include <type_traits>

#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_c1;
typedef __attribute__((address_space(1))) void glb_void_c1;
typedef unsigned int u32x2_c1 __attribute__((ext_vector_type(2)));

struct C1sArgs {
  const half_t* x;      // [M][K] (dual input: [M][K1])
  const half_t* x2;     // dual input: [B][H][W][K - K1] at stride `stride`, or nullptr
  const half_t* w;      // [N][K]
  const float* bias;    // [N]
  const half_t* res;    // [M][N] or nullptr
  half_t* y;            // [M][N]
  const void* zero;     // >= 16 zero bytes
  int M, N, relu;
  int nslab;            // cout slabs of NW * 64 channels
  int ntiles;           // ceil(M / BM)
  int G;                // workgroups (a multiple of nslab)
  int H, W, Wo, HWo, stride;   // stride 2: output pixel m reads input pixel (b, 2 oh, 2 ow)
  float acc_scale;      // SPLIT: accumulator multiplier 2^-e of the pre-scaled split weights
  int* ovf;             // SPLIT: range guard flag (common.h split_guard) or nullptr
  // N2 > 0 (fused next 1x1): z = relu(y . w2^T + b2), y the fp16 output tile
  const half_t* w2;     // [N2][N]
  const float* b2;      // [N2]
  half_t* z;            // [M][N2]
};

// ds_write_b64 outside the wait-count pass (a compiler LDS store after the
// next tile's LDS-DMA would get a vmcnt(0) in front of it)
__device__ __forceinline__ void c1_lds_write_b64(uint32_t addr, half4v v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

typedef int int4s __attribute__((ext_vector_type(4)));

// 8-byte buffer load (offen + SGPR soffset + immediate) that the wait-count pass
// does not track: the caller counts it in its own vmcnt waits and reg_tie()s
// the result after them
__device__ __forceinline__ half4v c1_lds_read_b64(uint32_t addr) {
  half4v v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
typedef unsigned int u32x4_c1 __attribute__((ext_vector_type(4)));

template <int IMM>
__device__ __forceinline__ half4v bload_b64_untracked(int4s rsrc, uint32_t voff, uint32_t soff) {
  half4v v;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen offset:%4"
               : "=v"(v) : "v"(voff), "s"(rsrc), "s"(soff), "n"(IMM) : "memory");
  return v;
}

// byte offset of cout fragment i (16 channels) from the wave's first channel:
// plain 32 i; split (pixel = [hi x32][lo x32] per 32 channels, the wave starting
// on a 32-channel boundary) 2 * (64 (i / 2) + 16 (i % 2)), lo 64 bytes further
template <bool SPLIT>
__host__ __device__ constexpr int c1_frag_off(int i) { return SPLIT ? 2 * (64 * (i >> 1) + 16 * (i & 1)) : 32 * i; }

template <int N_>
__device__ __forceinline__ void c1_vmcnt() {
  static_assert(N_ >= 0 && N_ < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// SPLIT: fp32-accurate split-fp16 operands (conv_glds.hip SPLIT): a pixel is 2K
// halfs, [hi x32][lo x32] per 32 channels, so one 128-byte LDS sub-row holds a
// channel chunk's hi and lo parts; 3 MFMAs per chunk (hi*hi + hi*lo + lo*hi);
// residual and output in the same layout, scaled by acc_scale, range-guarded.
// K1 > 0: TWO inputs concatenated along K -- channels [0, K1) from x (at the
// output resolution, stride 1) and [K1, K) from x2 (stride `stride`): a
// ResNet bottleneck's expansion 1x1 and its 1x1 downsample as one GEMM
// (W3 | Wds) . (y | x) + (b3 + bds): the downsample's output never reaches HBM.
// N2 > 0 (fp16, the whole output row N = NW * CW in one workgroup): the NEXT
// bottleneck block's reduce 1x1 (N -> N2, ReLU) runs on the output tile while
// it is on chip -- the tile is also written to LDS (fp16, exactly the values
// stored), and each wave computes N2 / NW of its channels -- so the next block
// never re-reads this block's 4x-wide output.
// LIO: the residual and the output go through per-wave LDS tiles, so every
// global access is 16 bytes per lane over whole 64-256-byte row segments (the
// C/D-fragment layout's 8-byte accesses over 16 rows kept the texture
// addresser 76-86 % busy on the ResNet50 tails: profiles/r3_pmc_r50_fp16.md).
template <int K, int NW, int BM, int CW, bool HAS_RES, bool SPLIT = false, int K1 = 0, int N2 = 0, bool LIO = false>
__global__ void __launch_bounds__(64 * NW, 2) conv1x1_stream_kernel   // 2nd: min waves per SIMD
(const C1sArgs a) {
  // BM pixels per tile: 64, or 32 for K = 128 (whose 64 A-fragment registers
  // plus a 64-pixel tile's accumulators and residual double buffer spill)
  // CW output channels per wave: 64, or 32 for K = 256 / 512 (A fragments: CW*K/128 VGPRs)
  constexpr int FN = CW / 16, FM = BM / 16;
  constexpr int KK = K / 32;             // MFMA K chunks
  constexpr int PXH = SPLIT ? 2 * K : K;  // halfs per input pixel
  constexpr int SP = SPLIT ? 2 : 1;       // (hi, lo) parts
  constexpr int KC = PXH / 64;            // 128-byte sub-rows per pixel (one LDS sub-tile each)
  constexpr int SUB = BM * 128;          // bytes per sub-tile
  constexpr int IPS = BM / 8;            // DMA instructions per sub-tile (8 rows of 128 B each)
  constexpr int TILE = KC * SUB;
  constexpr int NINS = TILE / 1024;      // DMA instructions per tile
  static_assert(NINS % NW == 0, "DMA instructions split evenly over the waves");
  constexpr int GX = NINS / NW;          // per wave
  constexpr int NY = NW * CW;             // output channels of a workgroup
  constexpr int CW2 = N2 / NW, FN2 = N2 ? CW2 / 16 : 1, KK2 = NY / 32;
  static_assert(N2 == 0 || (!SPLIT && CW2 % 16 == 0), "fused next 1x1: fp16, N2 a multiple of 16 * NW");
  constexpr int YROW = NY * 2;            // bytes per pixel row of the LDS output tile
  constexpr int ROWW = CW * 2 * SP;        // LIO: bytes of this wave's couts per pixel
  constexpr int RT = BM * ROWW;            // LIO: bytes of a wave's residual / output tile
  constexpr int CPRW = ROWW / 16;          // LIO: 16-byte chunks per pixel row (slot = chunk ^ (pixel % CPRW))
  constexpr int GLI = RT / 1024;           // LIO: 16-byte-per-lane instructions per wave tile
  // LIO + N2: y leaves from the block's LDS output tile (GLY whole-row
  // instructions per wave), z through the wave's tile (GLZ)
  constexpr int ROW2 = CW2 * 2, CPR2 = N2 ? ROW2 / 16 : 1;
  constexpr int GLY = N2 ? BM * NY * 2 / 1024 / NW : GLI;
  constexpr int GLZ = N2 ? BM * ROW2 / 1024 : 0;
  static_assert(!LIO || (RT % 1024 == 0 && (!SPLIT || CW % 32 == 0) && (CPRW & (CPRW - 1)) == 0),
                "LIO shapes: whole 1 KiB instructions, contiguous wave row segments");
  static_assert(!LIO || N2 == 0 || ((BM * NY * 2) % (1024 * NW) == 0 && (BM * ROW2) % 1024 == 0 && ROW2 <= ROWW &&
                                    (CPR2 & (CPR2 - 1)) == 0 && YROW == 512), "LIO + fused next shapes");
  // register-path stores are 16 bytes a lane (common.h split_swap_out): one per
  // fragment when split, one per fragment pair in fp16 (FN even)
  constexpr bool PAIR16 = !SPLIT && FN % 2 == 0;
  constexpr int GS = LIO ? GLY + GLZ : (PAIR16 ? FN / 2 : FN) * FM + (N2 ? FN2 * FM : 0);   // stores per wave and item
  constexpr int GR = HAS_RES ? (LIO ? GLI : FN * FM * SP) : 0;
  static_assert(GS + GX + GR < 64, "vmcnt immediate");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lid = xcd_remap((int)blockIdx.x, a.G);
  const int slab = lid % a.nslab;
  const int tstride = a.G / a.nslab;
  int t = lid / a.nslab;
  if (t >= a.ntiles) return;             // uniform
  const int frow = lane & 15, fch = lane >> 4;
  const int nw0 = slab * (NW * CW) + wave * CW;

  // ---- this wave's weights, resident: A fragments [cout frag][K chunk] ----
  half8v fa[FN][KK][SP];
  float4v bv[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int row = nw0 + i * 16 + frow;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int p = 0; p < SP; ++p)
        fa[i][kk][p] = row < a.N ? *reinterpret_cast<const half8v*>(a.w + (size_t)row * PXH + kk * (32 * SP) +
                                                                    p * 32 + fch * 8)
                                 : half8v{0, 0, 0, 0, 0, 0, 0, 0};
    const int n = nw0 + i * 16 + fch * 4;
    bv[i] = n < a.N ? *reinterpret_cast<const float4v*>(a.bias + n) : float4v{0.f, 0.f, 0.f, 0.f};
  }
  // fused next 1x1: this wave's N2/NW output channels, weights resident
  half8v fa2[N2 ? FN2 : 1][N2 ? KK2 : 1];
  float4v bv2[N2 ? FN2 : 1];
  if constexpr (N2 > 0) {
#pragma unroll
    for (int i = 0; i < FN2; ++i) {
      const int row = wave * CW2 + i * 16 + frow;
#pragma unroll
      for (int kk = 0; kk < KK2; ++kk) fa2[i][kk] = *reinterpret_cast<const half8v*>(a.w2 + (size_t)row * NY + kk * 32 + fch * 8);
      bv2[i] = *reinterpret_cast<const float4v*>(a.b2 + wave * CW2 + i * 16 + fch * 4);
    }
  }
  const half_t* zero = static_cast<const half_t*>(a.zero);
  constexpr int OPX = SPLIT ? 2 : 1;     // output / residual halfs per channel
  const unsigned out_bytes = (unsigned)a.M * (unsigned)a.N * (unsigned)(2 * OPX);
  const auto out_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)out_bytes, 0x00020000);
  // LIO: per-lane byte offset (from the tile's first pixel) of each 16-byte store
  uint32_t st_off[LIO ? GLY : 1], zst_off[LIO && N2 ? GLZ : 1];
  if constexpr (LIO && N2 > 0) {
#pragma unroll
    for (int j = 0; j < GLY; ++j) {        // this wave's rows of the block tile [BM][NY] (chunk ^ (pixel & 15))
      const int q = (wave * GLY + j) * 1024 + lane * 16;
      const int p = q / YROW, c = ((q % YROW) >> 4) ^ (p & 15);
      st_off[j] = (uint32_t)((p * a.N + c * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < GLZ; ++j) {
      const int q = j * 1024 + lane * 16;
      const int p = q / ROW2, c = ((q % ROW2) >> 4) ^ (p & (CPR2 - 1));
      zst_off[j] = (uint32_t)((p * N2 + wave * CW2 + c * 8) * 2);
    }
  } else if constexpr (LIO) {
#pragma unroll
    for (int j = 0; j < GLI; ++j) {
      const int q = j * 1024 + lane * 16;
      const int p = q / ROWW, c = ((q % ROWW) >> 4) ^ (p & (CPRW - 1));
      st_off[j] = (uint32_t)((p * a.N * OPX + (SPLIT ? split_off(nw0) : nw0) + c * 8) * 2);
    }
  }

  // DMA of tile tt into ring buffer buf: instruction ins covers rows 8*(ins%IPS).. of sub-tile ins/IPS;
  // lane l lands in row (l >> 3), slot (l & 7), and fetches chunk slot ^ swz_r(row)
  auto issue_x = [&](int tt, int buf) {   // buf: a constant at every call
#pragma unroll
    for (int j = 0; j < GX; ++j) {
      const int ins = wave + NW * j;
      const int sub = ins / IPS, r = (ins % IPS) * 8 + (lane >> 3);
      const int m = tt * BM + r;
      const int ch = (lane & 7) ^ swz_r(r, 8);
      constexpr int KC1 = K1 * SP / 64;       // sub-rows of the first input (0: single input)
      const half_t* src = zero;
      if (K1 > 0 && sub < KC1) {              // first input: output resolution, stride 1
        if (m < a.M) src = a.x + (size_t)m * (K1 * SP) + sub * 64 + ch * 8;
      } else {
        int pin = m;                          // input pixel of output pixel m
        if (a.stride != 1) {
          const int b = m / a.HWo, rr = m - b * a.HWo;
          const int oh = rr / a.Wo, ow = rr - oh * a.Wo;
          pin = (b * a.H + oh * a.stride) * a.W + ow * a.stride;
        }
        const half_t* xs = K1 > 0 ? a.x2 : a.x;
        if (m < a.M) src = xs + (size_t)pin * ((K - K1) * SP) + (sub - KC1) * 64 + ch * 8;
      }
      __builtin_amdgcn_global_load_lds((glb_void_c1*)src, (lds_void_c1*)(smem + buf * TILE + ins * 1024), 16, 0, 0);
    }
  };
  // residual and output addressing: byte offset of element (pixel m, cout n) =
  // lane part (frow*N + nw0 + 4*fch)*2 [VGPR] + tile / fragment-row part
  // (tt*BM + 16j)*N*2 [SGPR] + 32i [immediate]; rows past M fall outside the
  // descriptors (num_records = M*N*2): loads return 0, stores are dropped
  // (SPLIT: channel n sits at split_off(n) of a 2N-half pixel; nw0 % 32 == 0 or FN == 1,
  // so fragment i's offset from the lane part is the constant c1_frag_off(i))
  const uint32_t lane_off = (uint32_t)((frow * a.N * OPX + (SPLIT ? split_off(nw0) : nw0) + 4 * fch) * 2);
  // 16-byte stores after the lane swap: lane group fch holds channels 8 (fch >> 1)
  // .. +7 of the fragment's 16 (split: hi for fch even, lo for fch odd) or, fp16,
  // 16 (fch & 1) + 8 (fch >> 1) .. +7 of the fragment pair's 32
  const uint32_t lane_st = (uint32_t)((frow * a.N * OPX + (SPLIT ? split_off(nw0) + 8 * (fch >> 1) + 32 * (fch & 1)
                                                                   : nw0 + 16 * (fch & 1) + 8 * (fch >> 1))) * 2);
  int4s res_rsrc = {0, 0, 0, 0};
  if constexpr (HAS_RES) {
    const unsigned long long rp = reinterpret_cast<unsigned long long>(a.res);
    res_rsrc = int4s{(int)(rp & 0xffffffffu), (int)(rp >> 32), (int)out_bytes, 0x00020000};
  }
  // residual of tile tt (C/D layout: 4 consecutive couts of one pixel per
  // fragment): buffer loads the wait-count pass does not track (counted here)
  constexpr bool RREG = HAS_RES && !LIO;     // residual prefetched into registers
  half4v rv[2][RREG ? FN : 1][RREG ? FM : 1][SP];
  // LIO tiles of this wave: [residual ring 0][residual ring 1] (the current ring
  // half doubles as the output stage once its residual is in registers), or [output]
  char* const lio_p = smem + 2 * TILE + (N2 ? BM * NY * 2 : 0) + wave * (HAS_RES ? 2 : 1) * RT;
  const int colh = SPLIT ? split_off(nw0) : nw0;   // this wave's first half of a pixel row (LIO)
  auto load_res = [&](int tt, auto rb_c) {
    if constexpr (HAS_RES && LIO) {
      constexpr int rb = decltype(rb_c)::value;
#pragma unroll
      for (int j = 0; j < GLI; ++j) {
        const int q = j * 1024 + lane * 16;
        const int p = q / ROWW, c = ((q % ROWW) >> 4) ^ (p & (CPRW - 1));
        const int m = tt * BM + p;
        const half_t* src = m < a.M ? a.res + (size_t)m * ((size_t)a.N * OPX) + colh + c * 8 : zero;
        __builtin_amdgcn_global_load_lds((glb_void_c1*)src, (lds_void_c1*)(lio_p + rb * RT + j * 1024), 16, 0, 0);
      }
    } else if constexpr (HAS_RES) {
      constexpr int rb = decltype(rb_c)::value;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const uint32_t soff = (uint32_t)(tt * BM + j * 16) * (uint32_t)a.N * (uint32_t)(2 * OPX);
        rv[rb][0][j][0] = bload_b64_untracked<c1_frag_off<SPLIT>(0)>(res_rsrc, lane_off, soff);
        if constexpr (FN > 1) rv[rb][1][j][0] = bload_b64_untracked<c1_frag_off<SPLIT>(1)>(res_rsrc, lane_off, soff);
        if constexpr (FN > 2) rv[rb][2][j][0] = bload_b64_untracked<c1_frag_off<SPLIT>(2)>(res_rsrc, lane_off, soff);
        if constexpr (FN > 3) rv[rb][3][j][0] = bload_b64_untracked<c1_frag_off<SPLIT>(3)>(res_rsrc, lane_off, soff);
        if constexpr (SPLIT) {
          rv[rb][0][j][1] = bload_b64_untracked<c1_frag_off<SPLIT>(0) + 64>(res_rsrc, lane_off, soff);
          if constexpr (FN > 1) rv[rb][1][j][1] = bload_b64_untracked<c1_frag_off<SPLIT>(1) + 64>(res_rsrc, lane_off, soff);
          if constexpr (FN > 2) rv[rb][2][j][1] = bload_b64_untracked<c1_frag_off<SPLIT>(2) + 64>(res_rsrc, lane_off, soff);
          if constexpr (FN > 3) rv[rb][3][j][1] = bload_b64_untracked<c1_frag_off<SPLIT>(3) + 64>(res_rsrc, lane_off, soff);
        }
      }
    }
  };

  issue_x(t, 0);
  load_res(t, std::integral_constant<int, 0>{});
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t ytile = lds0 + 2 * TILE;    // fused next 1x1: the output tile (BM x NY fp16)
  const auto z_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.z, 0, (int)((unsigned)a.M * (unsigned)(N2 * 2)), 0x00020000);
  const uint32_t lane_off2 = (uint32_t)((frow * N2 + wave * CW2 + 4 * fch) * 2);
  bool first = true;
  // one item; BUF (the ring half and residual register set of tile t) is a
  // template constant so rv never needs runtime indexing (it went to scratch)
  auto item = [&](auto buf_c) -> bool {
    constexpr int buf = decltype(buf_c)::value;
    const int tn = t + tstride;
    const bool more = tn < a.ntiles;      // wave-uniform
    // tile t's DMA landed: younger are its residual loads and the previous item's stores
    if (first) c1_vmcnt<GR>(); else c1_vmcnt<GR + GS>();
    __builtin_amdgcn_s_barrier();         // everyone's DMA landed; the other buffer's reads are done
    if (more) {
      issue_x(tn, buf ^ 1);
      load_res(tn, std::integral_constant<int, buf ^ 1>{});
    }
    float4v acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    const uint32_t base = lds0 + buf * TILE;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      // chunk kk: plain -- sub-row kk/2, chunks 4(kk&1)+fch; SPLIT -- sub-row kk,
      // hi in chunks 0-3, lo in 4-7
      half8v fb[FM][SP];
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int r = j * 16 + frow;
#pragma unroll
        for (int p = 0; p < SP; ++p) {
          const int c = SPLIT ? 4 * p + fch : 4 * (kk & 1) + fch;
          fb[j][p] = lds_read_b128(base + (SPLIT ? kk : kk >> 1) * SUB + r * 128 + ((c ^ swz_r(r, 8)) << 4));
        }
      }
      lds_waitcnt<0>();
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int p = 0; p < SP; ++p) lds_tie(fb[j][p]);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][kk][0], fb[j][0], acc[i][j], 0, 0, 0);
      if constexpr (SPLIT) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][kk][0], fb[j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][kk][1], fb[j][0], acc[i][j], 0, 0, 0);
          }
      }
    }
    // ---- epilogue: bias (+ residual) (+ ReLU), fp16, buffer stores ----
    if constexpr (HAS_RES) {
      // this item's residual landed: younger are the previous stores and, with a
      // next item, its DMA and residual loads
      if (first) {
        if (more) c1_vmcnt<GX + GR>(); else c1_vmcnt<0>();
      } else {
        if (more) c1_vmcnt<GS + GX + GR>(); else c1_vmcnt<GS>();
      }
      if constexpr (RREG) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
#pragma unroll
            for (int p = 0; p < SP; ++p) reg_tie(rv[buf][i][j][p]);
      }
    }
    if constexpr (LIO) {
      // ---- LIO epilogue: residual fragments from LDS, output through LDS ----
      const uint32_t tile_l = lds0 + (uint32_t)(lio_p - smem) + (HAS_RES ? buf * RT : 0);
      auto frag_addr = [&](int j, int off) {   // byte `off` of the wave row of fragment-row pixel j*16+frow
        const int pp = j * 16 + frow;
        return tile_l + (uint32_t)(pp * ROWW + ((((off >> 4) ^ (pp & (CPRW - 1)))) << 4) + (off & 8));
      };
      half4v rl[HAS_RES ? FN : 1][HAS_RES ? FM : 1][SP];
      if constexpr (HAS_RES) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
#pragma unroll
            for (int p = 0; p < SP; ++p) rl[i][j][p] = c1_lds_read_b64(frag_addr(j, c1_frag_off<SPLIT>(i) + 8 * fch + 64 * p));
        lds_waitcnt<0>();
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
#pragma unroll
            for (int p = 0; p < SP; ++p) reg_tie(rl[i][j][p]);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          float4v v = SPLIT ? acc[i][j] * a.acc_scale + bv[i] : acc[i][j] + bv[i];
          if constexpr (HAS_RES) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] += (float)rl[i][j][0][e];
              if constexpr (SPLIT) v[e] += (float)rl[i][j][SP - 1][e];
            }
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          const int off = c1_frag_off<SPLIT>(i) + 8 * fch;
          if constexpr (SPLIT) {
            split_guard(a.ovf, v);
            half4v h, l;
            split_f16x4(v, h, l);
            c1_lds_write_b64(frag_addr(j, off), h);
            c1_lds_write_b64(frag_addr(j, off + 64), l);
          } else {
            half4v o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (half_t)v[e];
            if constexpr (N2 > 0) {
              // the block's output tile [pixel][NY], 16-byte chunk c of row p at c ^ (p & 15)
              const int pp = j * 16 + frow, c = (wave * CW + i * 16 + 4 * fch) >> 3;
              c1_lds_write_b64(ytile + pp * YROW + ((c ^ (pp & 15)) << 4) + (fch & 1) * 8, o);
            } else {
              c1_lds_write_b64(frag_addr(j, off), o);
            }
          }
        }
      lds_waitcnt<0>();
      if constexpr (N2 > 0) {
        __builtin_amdgcn_s_barrier();       // the whole output tile is in LDS
        // y: this wave's GLY KiB of the tile, whole rows, 16 bytes per lane
        half8v yb[GLY];
#pragma unroll
        for (int j = 0; j < GLY; ++j) yb[j] = lds_read_b128(ytile + (wave * GLY + j) * 1024 + lane * 16);
        // z = relu(y_tile . w2^T + b2)
        float4v acc2[FN2][FM];
#pragma unroll
        for (int i = 0; i < FN2; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc2[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
        lds_waitcnt<0>();
        const uint32_t soffy = (uint32_t)(t * BM) * (uint32_t)a.N * 2u;
#pragma unroll
        for (int j = 0; j < GLY; ++j) {
          lds_tie(yb[j]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c1, yb[j]), out_rsrc, (int)st_off[j],
                                                 (int)soffy, 0);
        }
#pragma unroll
        for (int kk = 0; kk < KK2; ++kk) {
          half8v fb2[FM];
#pragma unroll
          for (int j = 0; j < FM; ++j) {
            const int pp = j * 16 + frow, c = 4 * kk + fch;
            fb2[j] = lds_read_b128(ytile + pp * YROW + ((c ^ (pp & 15)) << 4));
          }
          lds_waitcnt<0>();
#pragma unroll
          for (int j = 0; j < FM; ++j) lds_tie(fb2[j]);
#pragma unroll
          for (int i = 0; i < FN2; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa2[i][kk], fb2[j], acc2[i][j], 0, 0, 0);
        }
        // z through this wave's tile (its residual is in registers already)
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
          for (int i = 0; i < FN2; ++i) {
            const float4v v = acc2[i][j] + bv2[i];
            half4v o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (half_t)fmaxf(v[e], 0.f);
            const int pp = j * 16 + frow, off = i * 32 + 8 * fch;
            c1_lds_write_b64(tile_l + pp * ROW2 + ((((off >> 4) ^ (pp & (CPR2 - 1)))) << 4) + (off & 8), o);
          }
        lds_waitcnt<0>();
        half8v zb[GLZ];
#pragma unroll
        for (int j = 0; j < GLZ; ++j) zb[j] = lds_read_b128(tile_l + j * 1024 + lane * 16);
        lds_waitcnt<0>();
        const uint32_t soffz = (uint32_t)(t * BM) * (uint32_t)(N2 * 2);
#pragma unroll
        for (int j = 0; j < GLZ; ++j) {
          lds_tie(zb[j]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c1, zb[j]), z_rsrc, (int)zst_off[j],
                                                 (int)soffz, 0);
        }
        t = tn;
        first = false;
        return more;
      }
      // whole row segments back out: lane-linear 16-byte LDS reads, one
      // 16-byte buffer store per lane (rows past M fall outside the descriptor)
      half8v ob[GLI];
#pragma unroll
      for (int j = 0; j < GLI; ++j) ob[j] = lds_read_b128(tile_l + j * 1024 + lane * 16);
      lds_waitcnt<0>();
      const uint32_t soff = (uint32_t)(t * BM) * (uint32_t)a.N * (uint32_t)(2 * OPX);
#pragma unroll
      for (int j = 0; j < GLI; ++j) {
        lds_tie(ob[j]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c1, ob[j]), out_rsrc, (int)st_off[j], (int)soff, 0);
      }
      t = tn;
      first = false;
      return more;
    } else {
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const uint32_t soff = (uint32_t)(t * BM + j * 16) * (uint32_t)a.N * (uint32_t)(2 * OPX);
      half4v op[PAIR16 ? FN : 1];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        float4v v = SPLIT ? acc[i][j] * a.acc_scale + bv[i] : acc[i][j] + bv[i];
        if constexpr (HAS_RES) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] += (float)rv[buf][i][j][0][e];
            if constexpr (SPLIT) v[e] += (float)rv[buf][i][j][SP - 1][e];
          }
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        const int voff = (int)lane_off + c1_frag_off<SPLIT>(i);
        if constexpr (SPLIT) {
          split_guard(a.ovf, v);
          half4v h, l;
          split_f16x4(v, h, l);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c1, split_swap_out(h, l)), out_rsrc,
                                                 (int)lane_st + c1_frag_off<SPLIT>(i), (int)soff, 0);
        } else {
          half4v o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (half_t)v[e];
          if constexpr (PAIR16) {
            op[i] = o;
            if (i & 1)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_c1, split_swap_out(op[i - 1], o)),
                                                     out_rsrc, (int)lane_st + 32 * (i - 1), (int)soff, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_c1, o), out_rsrc, voff, (int)soff, 0);
          }
          if constexpr (N2 > 0) {
            // output tile -> LDS [pixel][NY] fp16, 16-byte chunk c of pixel row p at c ^ (p & 15)
            const int p = j * 16 + frow, c = (wave * CW + i * 16 + 4 * fch) >> 3;
            c1_lds_write_b64(ytile + p * YROW + ((c ^ (p & 15)) << 4) + (fch & 1) * 8, o);
          }
        }
      }
    }
    if constexpr (N2 > 0) {
      // ---- fused next 1x1: z = relu(y_tile . w2^T + b2) ----
      lds_waitcnt<0>();
      __builtin_amdgcn_s_barrier();       // the whole output tile is in LDS
      float4v acc2[FN2][FM];
#pragma unroll
      for (int i = 0; i < FN2; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc2[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK2; ++kk) {
        half8v fb2[FM];
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int p = j * 16 + frow, c = 4 * kk + fch;
          fb2[j] = lds_read_b128(ytile + p * YROW + ((c ^ (p & 15)) << 4));
        }
        lds_waitcnt<0>();
#pragma unroll
        for (int j = 0; j < FM; ++j) lds_tie(fb2[j]);
#pragma unroll
        for (int i = 0; i < FN2; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa2[i][kk], fb2[j], acc2[i][j], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const uint32_t soff2 = (uint32_t)(t * BM + j * 16) * (uint32_t)(N2 * 2);
#pragma unroll
        for (int i = 0; i < FN2; ++i) {
          const float4v v = acc2[i][j] + bv2[i];
          half4v o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = (half_t)fmaxf(v[e], 0.f);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_c1, o), z_rsrc, (int)lane_off2 + 32 * i,
                                                (int)soff2, 0);
        }
      }
    }
    t = tn;
    first = false;
    return more;
    }
  };
  while (item(std::integral_constant<int, 0>{}) && item(std::integral_constant<int, 1>{})) {
  }
  c1_vmcnt<0>();
}

// Residual / output through per-wave LDS tiles (the LIO kernels) wherever the
// shape allows: ResNet50 b1024 fp16 +4.2 %, split +5.7 %, ResNet18 split +0.2 %,
// fused-next (N2) kernels ResNet50 fp16 +3.5 % (profiles/r3_ab_lio.md).  Two
// waves per SIMD (more resident workgroups measured no gain for fp16, +1 % split:
// not kept).
template <int K, int NW, int BM, int CW, bool R, bool SPLIT = false, int K1 = 0, int N2 = 0, bool LIO = false>
static void c1s_cfg(C1sArgs a, hipStream_t st) {
  constexpr int RT = BM * CW * 2 * (SPLIT ? 2 : 1), CPRW = RT / BM / 16;
  constexpr int ROW2 = N2 ? N2 / NW * 2 : 16;
  constexpr bool N2OK = N2 == 0 || ((BM * NW * CW * 2) % (1024 * NW) == 0 && (BM * ROW2) % 1024 == 0 &&
                                    ROW2 <= CW * 2 && NW * CW == 256);
  // (not K = 512: those tails are not addresser-bound, and the LDS round trip
  // spilled and cost 3-15 %: 258 -> 295 us, profiles/r3_resnet50_b1024_fp16_kernels_v2.md)
  if constexpr (!LIO && K != 512 && N2OK && RT % 1024 == 0 && (!SPLIT || CW % 32 == 0) && (CPRW & (CPRW - 1)) == 0) {
    c1s_cfg<K, NW, BM, CW, R, SPLIT, K1, N2, true>(a, st);
    return;
  }
  a.nslab = a.N / (NW * CW);
  constexpr int TILE = (SPLIT ? 2 : 1) * (K / 64) * BM * 128;
  constexpr int LDSB = 2 * TILE + (N2 ? BM * NW * CW * 2 : 0) + (LIO ? NW * (R ? 2 : 1) * RT : 0);
  a.ntiles = (a.M + BM - 1) / BM;
  auto kern = conv1x1_stream_kernel<K, NW, BM, CW, R, SPLIT, K1, N2, LIO>;
  ensure_lds_attr(reinterpret_cast<const void*>(kern), LDSB);
  const int per_cu = 8 / NW;                        // two waves per SIMD
  int G = per_cu * device_cu_count();
  G -= G % a.nslab;
  const long items = (long)a.ntiles * a.nslab;
  if (G > items) G = (int)items;
  a.G = G;
  hipLaunchKernelGGL(kern, dim3(G), dim3(64 * NW), LDSB, st, a);
}

bool conv1x1_stream_supported(int C, int Cout, long M) {
  // Cout 64 at C 64: one-wave workgroups, 8 per CU; C 256 / 512: 32 couts per
  // wave, slabs of 64 (two waves, C 256) or 128 channels
  const bool shape = (C == 64 && (Cout == 64 || Cout % 256 == 0)) || (C == 128 && Cout % 256 == 0) ||
                     (C == 256 && (Cout == 64 || Cout % 128 == 0)) || (C == 512 && Cout % 128 == 0);
  return shape && M > 0 && M * Cout * 2 < (1L << 31);
}

// Default for every eligible fp16 shape: ResNet50 b1024 fp16 whole forward 19.21 ->
// 17.80 ms (+7.9 %; Cin 256 +3.7 %, Cin 512 +1.7 %, stride 2 +1.0 % on top),
// profiles/r3_conv1x1_stream.md -- except fp16 stride 2 below ~100k output pixels
// (ResNet18's downsamples at B = 400: -0.4 % whole forward), which stay on the
// implicit-GEMM tiles.
bool conv1x1_stream_default(int C, int stride, long M) {
  (void)C;
  return stride == 1 || M >= 100000;
}

bool conv1x1_stream_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                           const void* zero, int M, int C, int Cout, int relu, int H, int W, int Wo, int HWo,
                           int stride, hipStream_t st) {
  if (!conv1x1_stream_supported(C, Cout, M)) return false;
  C1sArgs a{};
  a.H = H;
  a.W = W;
  a.Wo = Wo;
  a.HWo = HWo;
  a.stride = stride;
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.M = M;
  a.N = Cout;
  a.relu = relu;
  const bool r = res != nullptr;
  if (C == 64 && Cout == 64) {
    r ? c1s_cfg<64, 1, 64, 64, true>(a, st) : c1s_cfg<64, 1, 64, 64, false>(a, st);
  } else if (C == 64) {
    r ? c1s_cfg<64, 4, 64, 64, true>(a, st) : c1s_cfg<64, 4, 64, 64, false>(a, st);
  } else if (C == 128) {
    r ? c1s_cfg<128, 4, 32, 64, true>(a, st) : c1s_cfg<128, 4, 32, 64, false>(a, st);
  } else if (C == 256 && Cout == 64) {
    r ? c1s_cfg<256, 2, 32, 32, true>(a, st) : c1s_cfg<256, 2, 32, 32, false>(a, st);
  } else if (C == 256) {
    r ? c1s_cfg<256, 4, 32, 32, true>(a, st) : c1s_cfg<256, 4, 32, 32, false>(a, st);
  } else {
    r ? c1s_cfg<512, 4, 32, 32, true>(a, st) : c1s_cfg<512, 4, 32, 32, false>(a, st);
  }
  return true;
}

// split fp16 (fp32-accurate) 1x1 convs: 32-pixel tiles (16 where the A
// fragments, CW x K / 64 registers, leave no room for 32); 32 couts per wave,
// 16 for Cin 512 or Cout 64
bool conv1x1_stream_split_supported(int C, int Cout, long M) {
  const bool shape = ((C == 64 || C == 128 || C == 256) && (Cout % 128 == 0 || (Cout == 64 && C != 128))) ||
                     (C == 512 && Cout % 64 == 0);
  return shape && M > 0 && (M + 64) * Cout * 4 < (1L << 32);
}

// Default for every eligible split shape (ResNet50 b1024 split +9.4 %, ResNet18 b400
// split +0.5 %, profiles/r3_conv1x1_stream.md); Cin 64 / 128 with Cout % 256 == 0 use
// 64 couts per wave (ResNet50 b1024 split +2.5 %, profiles/r3_conv1x1_stream_ab_split.log).
bool conv1x1_stream_split_default(int C, int stride) {
  (void)C;
  (void)stride;
  return true;
}

bool conv1x1_stream_split_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                                 const void* zero, int M, int C, int Cout, int relu, float acc_scale, int* ovf, int H,
                                 int W, int Wo, int HWo, int stride, hipStream_t st) {
  if (!conv1x1_stream_split_supported(C, Cout, M)) return false;
  C1sArgs a{};
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.M = M;
  a.N = Cout;
  a.relu = relu;
  a.H = H;
  a.W = W;
  a.Wo = Wo;
  a.HWo = HWo;
  a.stride = stride;
  a.acc_scale = acc_scale;
  a.ovf = ovf;
  const bool r = res != nullptr;
  const bool narrow = C == 512 || Cout == 64;
  // wide: 64 couts per wave (256-channel slabs: 4x the bytes per item, the input
  // tile read once per 256 outputs) for Cin 64 / 128
  const bool wide = Cout % 256 == 0;
  switch (C) {
    case 64:
      if (narrow) r ? c1s_cfg<64, 4, 32, 16, true, true>(a, st) : c1s_cfg<64, 4, 32, 16, false, true>(a, st);
      else if (wide) r ? c1s_cfg<64, 4, 32, 64, true, true>(a, st) : c1s_cfg<64, 4, 32, 64, false, true>(a, st);
      else r ? c1s_cfg<64, 4, 32, 32, true, true>(a, st) : c1s_cfg<64, 4, 32, 32, false, true>(a, st);
      break;
    case 128:
      if (wide) r ? c1s_cfg<128, 4, 16, 64, true, true>(a, st) : c1s_cfg<128, 4, 16, 64, false, true>(a, st);
      else r ? c1s_cfg<128, 4, 32, 32, true, true>(a, st) : c1s_cfg<128, 4, 32, 32, false, true>(a, st);
      break;
    case 256:
      if (narrow) r ? c1s_cfg<256, 4, 32, 16, true, true>(a, st) : c1s_cfg<256, 4, 32, 16, false, true>(a, st);
      else r ? c1s_cfg<256, 4, 16, 32, true, true>(a, st) : c1s_cfg<256, 4, 16, 32, false, true>(a, st);
      break;
    default:
      r ? c1s_cfg<512, 4, 16, 16, true, true>(a, st) : c1s_cfg<512, 4, 16, 16, false, true>(a, st);
  }
  return true;
}

// dual input (ResNet bottleneck expansion + 1x1 downsample as one GEMM):
// (K1, K2) = (64, 64) [layer1] or (128, 256) [layer2, downsample stride 2]
bool conv1x1_dual_supported(int K1, int K2, int Cout, long M) {
  const bool shape = (K1 == 64 && K2 == 64 && Cout % 256 == 0) || (K1 == 128 && K2 == 256 && Cout % 128 == 0);
  return shape && M > 0 && (M + 64) * Cout * 2 < (1L << 31);
}

bool conv1x1_dual_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias, half_t* y,
                         const void* zero, int M, int K1, int K2, int Cout, int relu, int H, int W, int Wo, int HWo,
                         int stride, hipStream_t st) {
  if (!conv1x1_dual_supported(K1, K2, Cout, M)) return false;
  C1sArgs a{};
  a.x = x1;
  a.x2 = x2;
  a.w = w;
  a.bias = bias;
  a.y = y;
  a.zero = zero;
  a.M = M;
  a.N = Cout;
  a.relu = relu;
  a.H = H;
  a.W = W;
  a.Wo = Wo;
  a.HWo = HWo;
  a.stride = stride;
  if (K1 == 64) c1s_cfg<128, 4, 32, 64, false, false, 64>(a, st);
  else c1s_cfg<384, 4, 32, 32, false, false, 128>(a, st);
  return true;
}

// split (fp32-accurate) dual input: x1 [M][2 K1], x2 [..][2 K2] split layouts,
// w = pack_split_weight([W3 | Wds]) (one scale), split output
bool conv1x1_dual_split_supported(int K1, int K2, int Cout, long M) {
  const bool shape = (K1 == 64 && K2 == 64 && Cout % 128 == 0) || (K1 == 128 && K2 == 256 && Cout % 64 == 0);
  return shape && M > 0 && (M + 64) * Cout * 4 < (1L << 32);
}

bool conv1x1_dual_split_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias, half_t* y,
                               const void* zero, int M, int K1, int K2, int Cout, int relu, float acc_scale, int* ovf,
                               int H, int W, int Wo, int HWo, int stride, hipStream_t st) {
  if (!conv1x1_dual_split_supported(K1, K2, Cout, M)) return false;
  C1sArgs a{};
  a.x = x1;
  a.x2 = x2;
  a.w = w;
  a.bias = bias;
  a.y = y;
  a.zero = zero;
  a.M = M;
  a.N = Cout;
  a.relu = relu;
  a.H = H;
  a.W = W;
  a.Wo = Wo;
  a.HWo = HWo;
  a.stride = stride;
  a.acc_scale = acc_scale;
  a.ovf = ovf;
  if (K1 == 64 && Cout % 256 == 0) c1s_cfg<128, 4, 16, 64, false, true, 64>(a, st);
  else if (K1 == 64) c1s_cfg<128, 4, 32, 32, false, true, 64>(a, st);
  else c1s_cfg<384, 4, 16, 16, false, true, 128>(a, st);
  return true;
}

// ResNet50 layer1 bottleneck tail + the NEXT block's reduce 1x1, fp16, one pass:
//   y = relu(x1 . W^T + b (+ res)), or the dual form relu([x1 | x2 at stride] . W^T + b);
//   z = relu(y . w2^T + b2)  (N = 256, N2 = 64 or 128)
bool conv1x1_fused_next_supported(int K1, int K2, int N, int N2, long M) {
  // (the dual form with N2 = 128 spills and is no ResNet50 shape: layer1 block 0 feeds a 64-channel reduce)
  return N == 256 && M > 0 && (M + 64) * N * 2 < (1L << 31) && K1 == 64 &&
         ((K2 == 0 && (N2 == 64 || N2 == 128)) || (K2 == 64 && N2 == 64));
}

bool conv1x1_fused_next_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias,
                               const half_t* res, half_t* y, const half_t* w2, const float* b2, half_t* z,
                               const void* zero, int M, int K1, int K2, int N, int N2, int relu, int H, int W, int Wo,
                               int HWo, int stride, hipStream_t st) {
  if (!conv1x1_fused_next_supported(K1, K2, N, N2, M)) return false;
  C1sArgs a{};
  a.x = x1;
  a.x2 = x2;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.zero = zero;
  a.M = M;
  a.N = N;
  a.relu = relu;
  a.H = H;
  a.W = W;
  a.Wo = Wo;
  a.HWo = HWo;
  a.stride = stride;
  a.w2 = w2;
  a.b2 = b2;
  a.z = z;
  const bool r = res != nullptr;
  if (K2 == 0) {
    if (N2 == 64) r ? c1s_cfg<64, 4, 32, 64, true, false, 0, 64>(a, st) : c1s_cfg<64, 4, 32, 64, false, false, 0, 64>(a, st);
    else r ? c1s_cfg<64, 4, 32, 64, true, false, 0, 128>(a, st) : c1s_cfg<64, 4, 32, 64, false, false, 0, 128>(a, st);
  } else {
    c1s_cfg<128, 4, 32, 64, false, false, 64, 64>(a, st);
  }
  return true;
}

}  // namespace idunno
