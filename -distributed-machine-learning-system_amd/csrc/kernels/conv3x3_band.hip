// Band-staged split-fp16 3x3 / stride-1 / pad-1 convolution (ResNet layers 2-4).
//
// Why (docs/KERNELS.md "Where the ResNet18 split forward stands"): as an
// implicit GEMM (conv_glds SPLIT) every K stage DMAs its pixel operand from
// L2 again, once per tap, and a 128 x 128 tile needs ~43 B/clk/CU of LDS-DMA
// at full MFMA rate -- above the ~32 B/clk/CU the texture path moves (TA_busy
// 0.56 at mfma_busy 0.49).  Here the pixel operand is staged ONCE per 32-channel
// block and read for all nine taps at shifted LDS offsets, and a tile is
// 128 couts x up to 256 pixels, so weights are re-fetched half as often:
// ~16 B/clk/CU at full MFMA rate.
//
// Tile = 128 output channels x BM = 32*FM consecutive output pixels of the
// flattened (b, oh, ow) order.  8 waves: wave (wn, wm) owns couts
// 32wn..32wn+31 (2 fragments) x pixels wm*16FM .. (FM fragments).
//
// LDS (one 512-thread workgroup per CU, all 160 KiB):
//   [0, 64K)       patch buffer 0   }  channel block cb in buffer cb & 1
//   [64K, 128K)    patch buffer 1   }  (the next block lands while this one computes)
//   [128K, 160K)   weight ring, 2 slots of 128 rows x 128 B (one (cb, tap) stage each)
// A patch holds, for every image the tile touches, its rows oh_first-1 ..
// oh_last+1 (zero rows outside the image) x W+2 columns (zero columns 0 and
// W+1), 128 B per pixel (32 channels x (hi, lo)).  A tap (kh, kw) is then a
// uniform shift of kh*(W+2)+kw pixels: an immediate ds_read offset.
//
// Bank conflicts: chunk c of patch pixel t sits in slot c ^ (key(t) & 7) with
// key = row*(W+8) + col - 2W*segment (a compact address, a padded key): pixel
// pairs (t, t+8) of a fragment share a colour and fall in opposite halves of
// the lane groups, row wraps jump the key by a multiple of 8 and image
// segments are re-phased, so every ds_read_b128 of every tap is conflict-free
// for W = 56/28/14/7 (tests/test_band.py exhaustive check; the address costs 4
// VALU per fragment and tap: add, and-or, xor, xor).
//
// Pipeline (per stage = (cb, tap), 3 MFMAs per (cout fragment, pixel fragment)):
// the B fragment reads run R = 2 groups (pixel fragments) ahead of the MFMAs,
// across stage boundaries; the workgroup barrier of stage s+1 sits R groups
// before the end of stage s: there every wave has read stage s's A fragments
// (so weight slot s & 1 is free for stage s+2's DMA) and stage s+1's weights
// have landed.  The DMA ring runs across tile boundaries (persistent grid), so
// the next tile's first weights and patch are in flight during an epilogue.
// Every wait is counted: weight DMAs 2 per wave and stage, the next channel
// block's patch one DMA per wave at each of the first NPI stages (a 57 KiB burst
// per CU at one stage made the next in-order weight wait drain it), epilogue
// stores 2*2*FM per wave (buffer stores; rows past M fall outside the descriptor
// and are dropped, so the count is exact).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

typedef unsigned int u32x2_bd __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_bd __attribute__((ext_vector_type(4)));

struct BandArgs {
  const half_t* x;      // split input, pixel stride ldx halfs (2C used)
  const half_t* w;      // split weights [Cout][9 * 2C] (pack_split_weight)
  const float* bias;    // [Cout]
  const half_t* res;    // split residual, pixel stride ldr halfs, or nullptr
  void* y;              // split [M][ldy] halfs, or fp32 [M][ldy] (OUT_F32)
  int B, C, Cout, M;
  int ldx, ldr, ldy;
  int relu, ncb, tiles_n, ntiles;
  uint32_t wrow, wtap;  // weight row / one tap's bytes (split: 36C / 4C, fp16: 18C / 2C)
  float acc_scale;
  int* ovf;             // split range guard flag or nullptr
  int flags;            // profiling ablations (outputs wrong; tools/band_ab.py, tools/gpu/pmc_band.sh):
                        // bit 1 no epilogue stores, bit 2 no residual loads
};

namespace bnd {
constexpr int BN = 128;                        // couts per tile
constexpr int WN = 4;                          // wave groups along couts (32 couts each)
constexpr int FN = 2;                          // cout fragments per wave
constexpr int RB = 128;                        // bytes per LDS pixel / weight row
constexpr int WSLOT = BN * RB;                 // 16 KiB weight stage
constexpr uint32_t PB1 = 1u << 16;             // patch buffer 1 = buffer 0 | 64 KiB
constexpr uint32_t WB = 2u << 16;              // weight slots at 128 KiB and 144 KiB
constexpr uint32_t WS1 = 1u << 14;             // slot 1 = slot 0 | 16 KiB
constexpr int LDS = (2 << 16) + 2 * WSLOT;     // 160 KiB
constexpr uint32_t OOR = 0x80000000u;          // buffer offset past num_records: zeros / dropped
constexpr int R = 2;                           // B read groups in flight ahead of the MFMAs
}  // namespace bnd

template <int W, int FM, int WM>
struct BandGeom {
  static constexpr int NW = bnd::WN * WM;               // waves: 4 cout groups x WM pixel groups
  static constexpr int GW = bnd::WSLOT / 1024 / NW;     // weight DMA instructions per wave and stage
  static constexpr int HW = W * W;                      // square images (checked by the launcher)
  static constexpr int BM = 16 * FM * WM;
  static constexpr int WP = W + 2;                      // patch row: zero column, W pixels, zero column
  static constexpr int KS = W + 8;                      // swizzle-key row stride
  static constexpr int SPAN = (BM + W - 2) / W + 1;     // output rows BM consecutive pixels can touch
  static constexpr int NSEG = (BM + HW - 2) / HW + 1;   // images they can touch
  static constexpr int PROWS = SPAN + 2 * NSEG;         // + one zero/halo row above and below each image
  static constexpr int PPIX = PROWS * WP;
  static constexpr int NPI = (PPIX * 8 + 64 * NW - 1) / (64 * NW);   // patch DMAs per wave
  static_assert(NPI * NW * 1024 <= 65536, "a patch buffer is 64 KiB");
  static_assert(GW * NW * 1024 == bnd::WSLOT, "weight stage DMA split");
  static_assert((2 * WP + 2) * 128 + 65536 < 65536 * 2, "tap offsets");
};

struct BandTile {
  int m0, n0;           // first output pixel / channel
  int b0, oh0, b1, oh1; // first / last output pixel's image and row
  int nrows0;           // patch rows of the first image segment
  int rows;             // patch rows in use
};

template <int W, int FM, int WM>
__device__ __forceinline__ BandTile band_tile(const BandArgs& a, int T) {
  using G = BandGeom<W, FM, WM>;
  BandTile t;
  const int tm = T / a.tiles_n, tn = T - tm * a.tiles_n;
  t.m0 = tm * G::BM;
  t.n0 = tn * bnd::BN;
  const int ml = min(t.m0 + G::BM, a.M) - 1;
  t.b0 = t.m0 / G::HW;
  t.oh0 = (t.m0 - t.b0 * G::HW) / W;
  t.b1 = ml / G::HW;
  t.oh1 = (ml - t.b1 * G::HW) / W;
  t.nrows0 = (t.b0 == t.b1 ? t.oh1 : W - 1) - t.oh0 + 3;
  t.rows = t.b0 == t.b1 ? t.nrows0 : t.nrows0 + (t.b1 - t.b0 - 1) * (W + 2) + t.oh1 + 3;
  return t;
}

// Per-lane LDS-DMA source offsets of a tile's patch (valid = false: all zeros).
// Instruction i of wave w fills LDS chunks 64(w + 8i) .. +63: pixel t = chunk / 8,
// slot s = chunk % 8, which holds global chunk s ^ (key(t) & 7).
template <int W, int FM, int WM>
__device__ __forceinline__ void band_patch_offsets(const BandArgs& a, const BandTile& t, bool valid, int wave,
                                                   int lane, uint32_t (&pv)[BandGeom<W, FM, WM>::NPI]) {
  using G = BandGeom<W, FM, WM>;
#pragma unroll
  for (int i = 0; i < G::NPI; ++i) {
    const int J = (wave + G::NW * i) * 64 + lane;
    const int tt = J >> 3, s = J & 7;
    const int r = tt / G::WP, col = tt - r * G::WP;
    int seg, ih;
    if (r < t.nrows0) {
      seg = 0;
      ih = t.oh0 - 1 + r;
    } else {
      const int rr = r - t.nrows0;
      seg = 1 + rr / (W + 2);
      ih = rr - (seg - 1) * (W + 2) - 1;
    }
    const bool ok = valid && r < t.rows && (unsigned)ih < (unsigned)W && col >= 1 && col <= W;
    const int key = r * G::KS + col - 2 * W * seg;
    const int ch = s ^ (key & 7);
    const int pix = ((t.b0 + seg) * W + ih) * W + col - 1;
    pv[i] = ok ? (uint32_t)pix * (uint32_t)(a.ldx * 2) + (uint32_t)(ch << 4) : bnd::OOR;
  }
}

// Per-lane B-read bases of fragment j: bq = LDS byte address of the lane's
// tap-(0,0) pixel with its k-chunk q (bits 4-5), kb = (key & 7) << 4.
template <int W, int FM, int WM>
__device__ __forceinline__ void band_read_bases(const BandArgs& a, const BandTile& t, int wm, int frow, int q,
                                                uint32_t lds0, uint32_t (&bq)[FM], uint32_t (&kb)[FM]) {
  using G = BandGeom<W, FM, WM>;
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = min(t.m0 + wm * 16 * FM + 16 * j + frow, a.M - 1);
    const int b = m / G::HW, rr = m - b * G::HW;
    const int oh = rr / W, ow = rr - oh * W;
    const int seg = b - t.b0;
    const int rs = seg == 0 ? 0 : t.nrows0 + (seg - 1) * (W + 2);
    const int ohf = seg == 0 ? t.oh0 : 0;
    const int r = rs + oh - ohf;                          // patch row of tap kh = 0
    const int key = r * G::KS + ow - 2 * W * seg;         // key of tap (0, 0)
    bq[j] = lds0 + (uint32_t)((r * G::WP + ow) * 128 + (q << 4));
    kb[j] = (uint32_t)((key & 7) << 4);
  }
}

// B fragment read of tap `tap`: immediate offset (kh*(W+2) + kw) * 128
template <int W>
__device__ __forceinline__ half8v band_read(uint32_t addr, int tap) {
  constexpr int WP = W + 2;
  switch (tap) {
    case 0: return lds_read_b128_imm<0>(addr);
    case 1: return lds_read_b128_imm<128>(addr);
    case 2: return lds_read_b128_imm<256>(addr);
    case 3: return lds_read_b128_imm<WP * 128>(addr);
    case 4: return lds_read_b128_imm<(WP + 1) * 128>(addr);
    case 5: return lds_read_b128_imm<(WP + 2) * 128>(addr);
    case 6: return lds_read_b128_imm<2 * WP * 128>(addr);
    case 7: return lds_read_b128_imm<(2 * WP + 1) * 128>(addr);
    default: return lds_read_b128_imm<(2 * WP + 2) * 128>(addr);
  }
}

template <int N>
__device__ __forceinline__ void band_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue of one tile: x 2^-e, + bias (+ split residual), ReLU, split (or fp32)
// buffer stores -- exactly FN*FM store instructions per wave (16 B per lane when split)
// (rows past M get an offset past the descriptor and are dropped); clears acc.
template <int FM, bool HAS_RES, bool OUT_F32, bool F16, typename Rsrc>
__device__ __forceinline__ void band_epilogue(const BandArgs& a, const BandTile& cur, float4v (&acc)[bnd::FN][FM],
                                              int wn, int wm, int frow, int q, Rsrc y_rsrc, bool& bad) {
  using namespace bnd;
    const int mw = cur.m0 + wm * 16 * FM + frow;
    // split residual: one 16-byte load per lane and fragment (split_swap_in)
    half4v rh[HAS_RES ? FN : 1][HAS_RES ? FM : 1];
    float4v rw[HAS_RES && !F16 ? FN : 1][HAS_RES && !F16 ? FM : 1];
    if constexpr (HAS_RES) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = min(mw + 16 * j, a.M - 1);
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int nb = cur.n0 + wn * 32 + 16 * i;
          if constexpr (F16) {
            const half_t* p = a.res + (size_t)m * a.ldr + nb + 4 * q;
            rh[i][j] = (a.flags & 4) ? half4v{0, 0, 0, 0} : gload_b64_untracked(p);
          } else {
            const half_t* p = a.res + (size_t)m * a.ldr + split_off_q(nb, q);
            rw[i][j] = (a.flags & 4) ? float4v{0.f, 0.f, 0.f, 0.f} : gload_f4_untracked(p);
          }
        }
      }
    }
    float4v bv[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) bv[i] = *reinterpret_cast<const float4v*>(a.bias + cur.n0 + wn * 32 + 16 * i + 4 * q);
    band_vmcnt<0>();
    if constexpr (HAS_RES) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          if constexpr (F16) reg_tie(rh[i][j]);
          else reg_tie(rw[i][j]);
        }
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = mw + 16 * j;
      const bool mok = m < a.M;
      half4v o16[F16 ? FN : 1];                  // F16: the fragment pair, stored as one 16-byte lane
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = cur.n0 + wn * 32 + 16 * i + 4 * q;
        float4v v = acc[i][j] * a.acc_scale + bv[i];
        if constexpr (HAS_RES && F16) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)rh[i][j][e];
        } else if constexpr (HAS_RES) {
          half4v h, l;
          split_swap_in(rw[i][j], h, l);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)h[e] + (float)l[e];
        }
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (a.flags & 2) {
          if (v[0] == 12345.f) bad = true;           // keep the math alive
        } else if constexpr (F16) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o16[i][e] = (half_t)v[e];
        } else if constexpr (OUT_F32) {
          const uint32_t off = mok ? ((uint32_t)m * (uint32_t)a.ldy + (uint32_t)n) * 4u : OOR;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_bd, v), y_rsrc, (int)off, 0, 0);
        } else {
          constexpr float kMax = 65504.f;
          bad |= mok && !(fabsf(v[0]) < kMax && fabsf(v[1]) < kMax && fabsf(v[2]) < kMax && fabsf(v[3]) < kMax);
          half4v h, l;
          split_f16x4(v, h, l);
          // one 16-byte store per lane (split_swap_out: q even hi, q odd lo of 8 channels)
          const uint32_t off =
              mok ? ((uint32_t)m * (uint32_t)a.ldy + (uint32_t)split_off_q(n - 4 * q, q)) * 2u : OOR;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_bd, split_swap_out(h, l)), y_rsrc,
                                                 (int)off, 0, 0);
        }
        acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (F16) {
        static_assert(FN == 2, "fragment pair");
        if (!(a.flags & 2)) {
          const uint32_t off =
              mok ? ((uint32_t)m * (uint32_t)a.ldy + (uint32_t)f16_pair_off(cur.n0 + wn * 32, q)) * 2u : OOR;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_bd, split_swap_out(o16[0], o16[1])), y_rsrc,
                                                 (int)off, 0, 0);
        }
      }
    }
  }

// F16: plain fp16 operands (a 128-byte LDS row = 64 channels, two K = 32 halves:
// 2 MFMAs per fragment pair instead of the split's 3) and an fp16 epilogue.
template <int W, int FM, int WM, bool HAS_RES, bool OUT_F32, bool F16>
__global__ void __launch_bounds__(256 * WM, WM) conv3x3_band_kernel(const BandArgs a) {
  using G = BandGeom<W, FM, WM>;
  using namespace bnd;
  constexpr int NW = G::NW, GW = G::GW;
  constexpr int NPI = G::NPI;
  constexpr int NEPI = F16 ? FM : FN * FM;                           // epilogue stores per wave and tile
  static_assert(NEPI < 64 && NPI <= 8, "vmcnt immediates; patch chunks go out at taps 0 .. NPI-1");
  static_assert(!(F16 && OUT_F32), "fp16 band conv stores fp16");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;
  const int frow = lane & 15, q = lane >> 4;
  int T = blockIdx.x;
  if (T >= a.ntiles) return;                  // uniform
  const int GS = gridDim.x;
  const int ncb = a.ncb;
  const uint32_t lds0 = lds_addr(smem);

  const auto w_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, 0x7fffffff, 0x00020000);
  const auto x_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7fffffff, 0x00020000);
  const uint32_t ybytes = (uint32_t)a.M * (uint32_t)a.ldy * (OUT_F32 ? 4u : 2u);
  const auto y_rsrc = __builtin_amdgcn_make_buffer_rsrc(a.y, 0, (int)ybytes, 0x00020000);
  const uint32_t wrow = a.wrow;                     // weight row bytes (9 taps x K-row halfs)
  const uint32_t wtap = a.wtap;                     // one tap's bytes

  // weight DMA: instruction j of this wave fills rows (wave + 8j)*8 .. +7 of a slot
  uint32_t wv[GW];
#pragma unroll
  for (int j = 0; j < GW; ++j) {
    const int row = (wave + NW * j) * 8 + (lane >> 3);
    wv[j] = (uint32_t)row * wrow + (uint32_t)((((lane & 7) ^ swz_r(row, 8))) << 4);
  }
  // A fragment read (cout row 32wn + frow, k-chunk q; lo = ^64; fragment i = +2048)
  const int arow = wn * 32 + frow;
  const uint32_t fa = lds0 + WB + (uint32_t)(arow * 128 + ((q ^ swz_r(arow, 8)) << 4));

  BandTile cur = band_tile<W, FM, WM>(a, T);
  bool have_nxt = T + GS < a.ntiles;
  BandTile nxt = band_tile<W, FM, WM>(a, have_nxt ? T + GS : T);
  uint32_t pv[NPI];
  uint32_t bq[FM], kb[FM];
  band_patch_offsets<W, FM, WM>(a, cur, true, wave, lane, pv);
  band_read_bases<W, FM, WM>(a, cur, wm, frow, q, lds0, bq, kb);

  auto issue_w = [&](uint32_t slot, uint32_t soff) {
#pragma unroll
    for (int j = 0; j < GW; ++j) dma_buf16(w_rsrc, smem + WB + slot + (wave + NW * j) * 1024, wv[j], (int)soff);
  };
  auto issue_p = [&](uint32_t buf, int cb) {
#pragma unroll
    for (int i = 0; i < NPI; ++i) dma_buf16(x_rsrc, smem + buf + (wave + NW * i) * 1024, pv[i], cb * 128);
  };
  auto issue_p1 = [&](uint32_t buf, int cb, int i) {
    dma_buf16(x_rsrc, smem + buf + (wave + NW * i) * 1024, pv[i], cb * 128);
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  // A fragments [cout frag][hi, lo]: aN is read at the barrier of stage s+1
  // (R groups before the end of stage s) and copied to aC once it has landed
  // (the first wait of stage s+1), so stage s's last groups keep using aC
  half8v aC[FN][2], aN[FN][2];
  half8v bR[R + 1][2];                // B read ring [group % 3][hi, lo]
  bool bad = false;                   // split range guard, stored once at the end

  auto read_a = [&](uint32_t slot) {
    const uint32_t base = fa ^ slot;
    aN[0][0] = lds_read_b128_imm<0>(base);
    aN[1][0] = lds_read_b128_imm<2048>(base);
    aN[0][1] = lds_read_b128_imm<0>(base ^ 64u);
    aN[1][1] = lds_read_b128_imm<2048>(base ^ 64u);
  };
  auto read_b = [&](int ring, int j, int tap, uint32_t pbit) {
    const int kh = tap / 3, kw = tap - 3 * kh;
    const uint32_t dk16 = (uint32_t)(((kh * G::KS + kw) & 7) << 4);
    const uint32_t y = ((kb[j] + dk16) & 0x70u) | pbit;
    const uint32_t ah = bq[j] ^ y;
    bR[ring][0] = band_read<W>(ah, tap);
    bR[ring][1] = band_read<W>(ah ^ 64u, tap);
  };

  // ---- prologue: patch(cb 0) + weights of stages 0 and 1 ----
  issue_p(0u, 0);
  issue_w(0u, (uint32_t)cur.n0 * wrow);
  band_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  issue_w(WS1, (uint32_t)cur.n0 * wrow + wtap);
  read_a(0u);
#pragma unroll
  for (int g = 0; g < R; ++g) read_b(g, g, 0, 0u);
  bool first_tile = true;

  for (;;) {                                   // tiles of this workgroup
    for (int cb = 0; cb < ncb; ++cb) {
      // opaque per iteration: keeps the compiler from hoisting the 9 taps' B
      // addresses out of the loop (72 extra live registers)
#pragma unroll
      for (int j = 0; j < FM; ++j) asm volatile("" : "+v"(bq[j]), "+v"(kb[j]));
      const bool last_cb = cb == ncb - 1;
      const uint32_t pbit = (uint32_t)(cb & 1) << 16;    // patch buffer of this channel block
      const uint32_t slot0 = (uint32_t)(cb & 1) * WS1;   // weight slot of tap 0 (stage parity)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const uint32_t slot = (tap & 1) ? (slot0 ^ WS1) : slot0;
#pragma unroll
        for (int j = 0; j < FM; ++j) asm volatile("" : "+v"(bq[j]), "+v"(kb[j]));
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int gi = tap * FM + j;                   // group index; mod 3 is static (9 % 3 == 0)
          if (j == FM - R) {
            // ---- barrier of stage s+1 ----
            const bool new_tile = tap == 8 && last_cb;
            const bool has_next = !new_tile || have_nxt;
            if (has_next) {
              // w(s+1) landed; younger: the patch chunk issued behind it at the last
              // barrier (tap - 1 < NPI; at tap 8 the whole next patch must be in), or
              // at a tile's first stage the previous tile's epilogue stores
              if (tap >= 1 && tap <= NPI && tap != 8) band_vmcnt<1>();
              else if (tap == 0 && cb == 0 && !first_tile) band_vmcnt<NEPI>();
              else band_vmcnt<0>();
              __builtin_amdgcn_s_barrier();
              // weights of stage s+2 into this stage's slot (its A reads are done everywhere)
              int t2 = tap + 2, cbn = cb;
              bool nt2 = false;
              if (t2 >= 9) {
                t2 -= 9;
                if (++cbn == ncb) {
                  cbn = 0;
                  nt2 = true;
                }
              }
              if (!nt2 || have_nxt) {
                const int n0 = nt2 ? nxt.n0 : cur.n0;
                issue_w(slot, (uint32_t)n0 * wrow + (uint32_t)t2 * wtap + (uint32_t)cbn * 128u);
              }
              if (tap < NPI) {
                // chunk `tap` of the next channel block's patch (or the next tile's first)
                // into the other buffer: one DMA per wave and stage, not a burst
                if (last_cb && tap == 0) band_patch_offsets<W, FM, WM>(a, nxt, have_nxt, wave, lane, pv);
                issue_p1(pbit ^ PB1, last_cb ? 0 : cb + 1, tap);
              }
              if (new_tile) band_read_bases<W, FM, WM>(a, nxt, wm, frow, q, lds0, bq, kb);
            }
            read_a(slot ^ WS1);
          }
          // B reads of group gi + R (this stage, or the next one's first groups)
          if (j + R < FM) {
            read_b((gi + R) % (R + 1), j + R, tap, pbit);
          } else {
            const int ntap = tap == 8 ? 0 : tap + 1;
            const uint32_t npbit = tap == 8 ? (pbit ^ PB1) : pbit;
            read_b((gi + R) % (R + 1), j + R - FM, ntap, npbit);
          }
          if (j >= FM - R) lds_waitcnt<2 * R + 4>();
          else lds_waitcnt<2 * R>();
          const int rg = gi % (R + 1);
          lds_tie(bR[rg][0]);
          lds_tie(bR[rg][1]);
          if (j == 0) {
            // this stage's A (read before this group's B) has landed
#pragma unroll
            for (int i = 0; i < FN; ++i) {
              lds_tie(aN[i][0]);
              lds_tie(aN[i][1]);
              aC[i][0] = aN[i][0];
              aC[i][1] = aN[i][1];
            }
          }
          if constexpr (F16) {
            // channels 0-31 (chunks 0-3) and 32-63 (chunks 4-7) of the 64-channel block
#pragma unroll
            for (int i = 0; i < FN; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aC[i][0], bR[rg][0], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < FN; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aC[i][1], bR[rg][1], acc[i][j], 0, 0, 0);
          } else {
#pragma unroll
            for (int i = 0; i < FN; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aC[i][0], bR[rg][0], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < FN; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aC[i][0], bR[rg][1], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < FN; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aC[i][1], bR[rg][0], acc[i][j], 0, 0, 0);
          }
        }
      }
      // the next stage's A and first B groups are in flight and cross the loop
      // back-edge: land them before the compiler may move those registers
      lds_waitcnt<0>();
#pragma unroll
      for (int g = 0; g < R + 1; ++g) {
        lds_tie(bR[g][0]);
        lds_tie(bR[g][1]);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        lds_tie(aN[i][0]);
        lds_tie(aN[i][1]);
      }
    }

    band_epilogue<FM, HAS_RES, OUT_F32, F16>(a, cur, acc, wn, wm, frow, q, y_rsrc, bad);
    if (!have_nxt) break;
    first_tile = false;
    T += GS;
    cur = nxt;
    have_nxt = T + GS < a.ntiles;
    nxt = band_tile<W, FM, WM>(a, have_nxt ? T + GS : T);
  }
  lds_waitcnt<0>();
  band_vmcnt<0>();
  if (bad && a.ovf != nullptr) *a.ovf = 1;
}


// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

// (W, FM) configurations: FM pixel fragments per wave chosen so that the tile
// count at B = 400 is just under a whole number of waves of 256 workgroups
// (layer2: 1225 tiles of 256 pixels = 4.79 waves; layer3 980 = 3.83; layer4 492 = 1.92)
static int band_fm(int W) {
  switch (W) {
    case 28: return 8;
    case 14: return 5;
    case 7: return 5;
    default: return 0;
  }
}

bool conv3x3_band_supported(int H, int W, int C, int Cout) {
  return H == W && band_fm(W) > 0 && C % 64 == 0 && C >= 64 && Cout % bnd::BN == 0;
}

int conv3x3_band_tiles(int B, int W, int Cout);

// Auto selection: layer2 (W 28, 1225 tiles at B = 400) takes the band kernel; layer3
// (W 14) ties the 128 x 128 im2col tile and keeps it.  Layer4 (W 7) took it in round 5
// (4-5 % under the 128 x 160 im2col tile then), but after the round-5 16-byte epilogues
// the 128 x 160 tile wins the whole graph: ResNet18 b400 split +1.2 % same process
// without the band kernel at W 7, -1.1 % without it at W 28 (profiles/r6f_ab_route_*.log).
// Below one tile per CU (small per-GPU batches) the im2col tiles + split-K win.
bool conv3x3_band_default(int B, int W, int Cout) {
  if (W != 28) return false;
  return conv3x3_band_tiles(B, W, Cout) >= device_cu_count();
}

// fp16: with 8-byte epilogue stores the band kernel led the im2col tiles only
// at W 28 without a residual (profiles/r5_band_f16_layers.log).  With the
// 16-byte epilogue (f16_pair_off) it leads or ties per layer at every W
// (profiles/r5_band_f16_layers_b128.log), but in the whole graph only W 28 pays:
// W 28 with or without residual +1.0 % ResNet18 fp16 (ResNet50 -0.04 %), every W
// -2.0 % / -0.6 % (profiles/r5_ab_band_f16_rule_b128.log).
bool conv3x3_band_f16_default(int B, int W, int Cout, bool res) {
  (void)res;
  return W == 28 && conv3x3_band_tiles(B, W, Cout) >= device_cu_count();
}

int conv3x3_band_tiles(int B, int W, int Cout) {
  const int fm = band_fm(W);
  if (fm <= 0) return 0;
  const long M = (long)B * W * W;
  const int bm = 32 * fm;
  return (int)((M + bm - 1) / bm) * (Cout / bnd::BN);
}

template <int W, int FM, int WM, bool R, bool F, bool H>
static void band_cfg(const BandArgs& a, int grid, hipStream_t st) {
  auto kern = conv3x3_band_kernel<W, FM, WM, R, F, H>;
  ensure_lds_attr(reinterpret_cast<const void*>(kern), bnd::LDS);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256 * WM), bnd::LDS, st, a);
}

template <int W, int FM, int WM>
static bool band_dispatch(const BandArgs& a, bool res, bool out_f32, bool f16, int grid, hipStream_t st) {
  if (f16) {
    if (res) band_cfg<W, FM, WM, true, false, true>(a, grid, st);
    else band_cfg<W, FM, WM, false, false, true>(a, grid, st);
  } else if (res) {
    if (out_f32) band_cfg<W, FM, WM, true, true, false>(a, grid, st);
    else band_cfg<W, FM, WM, true, false, false>(a, grid, st);
  } else {
    if (out_f32) band_cfg<W, FM, WM, false, true, false>(a, grid, st);
    else band_cfg<W, FM, WM, false, false, false>(a, grid, st);
  }
  return true;
}

bool conv3x3_band_launch(const half_t* x, int ldx, const half_t* w, const float* bias, const half_t* res, int ldr,
                         void* y, int ldy, bool out_f32, int B, int H, int W, int C, int Cout, int relu,
                         float acc_scale, int* ovf, int max_grid, int flags, hipStream_t st, bool f16) {
  if (!conv3x3_band_supported(H, W, C, Cout)) return false;
  if (f16 && out_f32) return false;
  BandArgs a;
  a.x = x;
  a.w = w;
  a.bias = bias;
  a.res = res;
  a.y = y;
  a.B = B;
  a.C = C;
  a.Cout = Cout;
  a.M = B * H * W;
  a.ldx = ldx;
  a.ldr = ldr;
  a.ldy = ldy;
  a.relu = relu;
  // one 128-byte K block per stage: 32 split channels (hi, lo) or 64 fp16 channels
  a.ncb = f16 ? C / 64 : C / 32;
  a.wrow = (f16 ? 18u : 36u) * (uint32_t)C;
  a.wtap = (f16 ? 2u : 4u) * (uint32_t)C;
  a.tiles_n = Cout / bnd::BN;
  a.ntiles = conv3x3_band_tiles(B, W, Cout);
  a.acc_scale = acc_scale;
  a.ovf = ovf;
  a.flags = flags;
  // 32-bit buffer offsets: input pixels x stride, weights, output
  if ((long)B * H * W * ldx * 2 >= (1L << 31) || (long)Cout * (f16 ? 18 : 36) * C >= (1L << 31) ||
      (long)a.M * ldy * (out_f32 ? 4 : 2) >= (1L << 31))
    return false;
  if (a.ntiles <= 0) return true;
  // persistent: one workgroup per CU (max_grid > 0 caps it: tests run several tiles per workgroup)
  int grid = a.ntiles < device_cu_count() ? a.ntiles : device_cu_count();
  if (max_grid > 0 && grid > max_grid) grid = max_grid;
  switch (W) {
    case 28:
      return band_dispatch<28, 8, 2>(a, res != nullptr, out_f32, f16, grid, st);
    case 14: return band_dispatch<14, 5, 2>(a, res != nullptr, out_f32, f16, grid, st);
    case 7: return band_dispatch<7, 5, 2>(a, res != nullptr, out_f32, f16, grid, st);
    default: return false;
  }
}

}  // namespace idunno
