// Row-streaming 3x3 / stride-1 / pad-1 conv, 64 -> 64 channels, on split fp16
// (fp32-accurate, see conv_glds.hip SPLIT): ResNet layer1 (56x56x64).
//
// Why a kernel of its own: as an implicit GEMM (conv_glds SPLIT) every input
// pixel is DMA'd from L2 once per tap, 9x; at C = 64 the layer is bound by
// that L2 -> LDS stream (~11 TB/s at 28 % of the f16 MFMA peak).  Here
//   * the weights live in REGISTERS: wave w owns output channels 16w..16w+15
//     and holds their 9 taps x 2 channel blocks x (hi, lo) A fragments
//     (36 x half8v = 144 VGPRs) for the whole launch;
//   * the input streams through LDS one image row at a time: a 5-row ring
//     (rows y-2 .. y+1 in use, row y+2 landing by LDS-DMA while row y
//     computes), so each input row is fetched once per band of rows instead
//     of 9 times;
//   * an output row is 3 pixel fragments of 16 (columns 0..47) and every
//     second row adds one tail fragment with columns 48..W-1 of both rows of
//     the pair (49 <= W <= 56); per (tap, channel block, fragment) a wave reads
//     the hi and lo B fragments and issues 3 MFMAs (hi*hi + hi*lo + lo*hi),
//     the reads of the next two such groups in flight behind them (3-deep
//     register ring, counted lgkmcnt);
//   * the residual of the row is loaded into registers when the row starts.
// LDS pixel rows are 256 B (64 channels x (hi, lo) halfs: 16 chunks of 16 B);
// chunk c of LDS column col sits in slot c ^ ((2*col) & 15), which makes the
// B-fragment reads (lane = pixel col + 16 * k-group) conflict-free for every
// tap shift, the tail fragment's two-row lane split included (exhaustive
// checks in tests/test_split.py).
// Persistent: workgroup g takes the g-th equal share of the B * H output rows
// (flattened image-major), as one band per image it touches, so every
// workgroup finishes within a row of the others (round 4: 8-row bands, 2800
// items over 512 workgroups = 5.47 rounds, the last one half empty).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

namespace c64s {
constexpr int C = 64;              // channels in and out
constexpr int PIX = 2 * C;         // halfs per pixel (split)
constexpr int RC = 60;             // LDS columns per ring row (W + 2 <= 58 read; 60 = 3.75 whole DMA instructions)
constexpr int RB = RC * 256;       // bytes per ring row
constexpr int RING = 5;            // rows y-2 .. y+1 in use (a row pair's tail fragment) + row y+2 landing
constexpr int BIAS = RING * RB;    // the 64 biases (fp32), read by the epilogue: no VGPRs held for them
constexpr int LDS = BIAS + 256;    // 77,056 B: 2 workgroups per CU
constexpr int WMAX = 56;           // 3 full fragments + an 8-column tail per row
constexpr int NST = 3;             // epilogue stores per wave and row, at least (3 fragments, 16 B a lane)
}  // namespace c64s

struct C64sArgs {
  const half_t* x;      // split [B][H][W][128]
  const half_t* w;      // split weights [64][9 * 128] (pack_split_weight)
  const float* bias;    // [64]
  const half_t* res;    // split [B][H][W][128] or nullptr
  half_t* y;            // split [B][H][W][128]
  const void* zero;     // unused (padding comes from out-of-range buffer offsets)
  int B, H, W, relu, nrows;
  float acc_scale;
  int* ovf;             // split range guard flag or nullptr (common.h split_guard)
};

__device__ __forceinline__ int c64s_slot(int chunk, int col) { return chunk ^ ((2 * col) & 15); }

// ds_read_b128 with an immediate byte offset (invisible to the wait-count pass, see common.h)
template <int OFF>
__device__ __forceinline__ half8v lds_read_b128_off(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset range");
  half8v v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

// fragment f's read (f = 0..2 of the row: immediate offset 4096 * f; f = 3: the
// tail fragment, whose lanes carry their own row base)
__device__ __forceinline__ half8v lds_read_frag(uint32_t addr, int f) {
  switch (f) {
    case 0: return lds_read_b128_off<0>(addr);
    case 1: return lds_read_b128_off<4096>(addr);
    case 2: return lds_read_b128_off<8192>(addr);
    default: return lds_read_b128_off<0>(addr);
  }
}

// Per-lane buffer offsets of the row DMA (constant for the launch): chunk
// i = r * 256 + tid of an LDS ring row is column i / 16, slot i % 16, which holds
// global chunk c64s_slot(slot, col) of pixel col - 1; padding columns get an
// offset past the descriptor (zeros).
__device__ __forceinline__ void c64s_row_offsets(const C64sArgs& a, int tid, uint32_t (&voff)[4]) {
  using namespace c64s;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = r * 256 + tid;
    const int col = i >> 4, slot = i & 15;
    const int ix = col - 1;
    voff[r] = (unsigned)ix < (unsigned)a.W ? (uint32_t)(ix * 256 + (c64s_slot(slot, col) << 4)) : 0x80000000u;
  }
}

// DMA input row iy of image b into ring slot rs (zeros outside the image):
// RC * 16 = 960 chunks, so waves 0-2 issue 4 DMA instructions and wave 3 issues 3
// (a wave-uniform split: the counted waits below only need each wave's own DMAs
// to be older than its epilogue stores).  The row's base is the uniform soffset.
template <typename Rsrc>
__device__ __forceinline__ void c64s_load_row(const C64sArgs& a, char* ring, Rsrc x_rsrc, const uint32_t (&voff)[4],
                                              int b, int iy, int rs, int tid) {
  using namespace c64s;
  const bool rowv = (unsigned)iy < (unsigned)a.H;
  const int soff = rowv ? (b * a.H + iy) * a.W * 256 : 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r == 3 && (tid >> 6) == 3) break;       // chunks 960..1023: past the row (wave-uniform)
    dma_buf16(x_rsrc, ring + rs * RB + (r * 256 + (tid & ~63)) * 16, rowv ? voff[r] : 0x80000000u, soff);
  }
}

// D groups of B reads in the register ring: D - 1 groups in flight behind the
// group whose MFMAs issue
template <int N>
__device__ __forceinline__ void c64s_wait_groups() {
  lds_waitcnt<2 * N>();
}

template <int N>
struct c64s_nf {
  static constexpr int value = N;
};

// Output row y is fragments 0-2 (columns 0..47) plus, every second row, one
// TAIL fragment holding columns 48..W-1 of BOTH rows of the pair (lanes 0-7:
// row y-1, lanes 8-15: row y): 7 fragments per row pair instead of 8, so no
// MFMA work on the 8 columns past W = 56 (12.5 % of the round-4 kernel's).  A
// band's last row when the band has an odd count gets a tail of its own (lanes
// 8-15 masked).  The tail of the pair (y-1, y) reads input rows y-2 .. y+1: a
// 5-row ring holds them while row y+2 lands.
template <bool HAS_RES, int D>
__global__ void __launch_bounds__(256, 2) conv3x3_split_c64_kernel(const C64sArgs a) {
  using namespace c64s;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 15, q = lane >> 4;
  // this workgroup's rows [r_begin, r_end) of the B * H output rows
  const int r_begin = (int)((long long)blockIdx.x * a.nrows / gridDim.x);
  const int r_end = (int)((long long)(blockIdx.x + 1) * a.nrows / gridDim.x);
  if (r_begin >= r_end) return;              // uniform

  // ---- A fragments of this wave's 16 couts: [tap][block][hi|lo] ----
  half8v fa[9][2][2];
  {
    const half_t* wr = a.w + (size_t)(wave * 16 + frow) * (9 * PIX) + q * 8;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int p = 0; p < 2; ++p) fa[t][cb][p] = *reinterpret_cast<const half8v*>(wr + t * PIX + cb * 64 + p * 32);
  }
  const int n0 = wave * 16 + 4 * q;            // this lane's 4 output channels (C/D layout)
  if (tid < 16) *reinterpret_cast<float4v*>(smem + BIAS + 16 * tid) = *reinterpret_cast<const float4v*>(a.bias + 4 * tid);
  const uint32_t ring = lds_addr(smem);
  const auto x_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, 0x7fffffff, 0x00020000);
  uint32_t voff[4];
  c64s_row_offsets(a, tid, voff);
  // per-lane LDS byte offset of column col0 + kw, chunk 4c + q:
  //   col*256 + (slot << 4), slot = (4c + q) ^ x, x = (2*col) & 15
  // = off ^ (c << 6): bits 6-7 hold c ^ (x >> 2), bits 4-5 q ^ (x & 3)
  auto col_off = [&](int col) {
    const int x = (2 * col) & 15;
    return (uint32_t)(col * 256 + (((x >> 2) & 3) << 6) + (((q ^ x) & 3) << 4));
  };
  // fragments 0-2 read column frow + kw (+ 16 f by immediate offset); the tail
  // reads column 48 + frow % 8 + kw = frow + kw + (48 or 40), the same swizzle
  // (2 * col mod 16 does not change by a multiple of 8 columns): loff + tshift
  uint32_t loff[3];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) loff[kw] = col_off(frow + kw);
  const uint32_t tshift = frow < 8 ? 48u * 256u : 40u * 256u;
  const int tcol = 48 + (frow & 7);            // the tail fragment's output column
  const int tailn = a.W - 48;                  // valid tail columns per row (1..8)

  for (int r = r_begin; r < r_end;) {           // one band per image the range touches
    const int b = r / a.H;
    const int y0 = r - b * a.H;
    const int y1 = min(a.H, y0 + (r_end - r));
    r += y1 - y0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();              // previous item's ring reads are done
    c64s_load_row(a, smem, x_rsrc, voff, b, y0 - 1, (y0 + 4) % RING, tid);
    c64s_load_row(a, smem, x_rsrc, voff, b, y0, y0 % RING, tid);
    c64s_load_row(a, smem, x_rsrc, voff, b, y0 + 1, (y0 + 1) % RING, tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int y = y0; y < y1; ++y) {
      // row y+1 landed: its DMA (issued one row ago) is older than this wave's
      // last >= NST epilogue stores; then the barrier publishes everyone's DMA
      // and ends every wave's reads of row y-3, whose slot row y+2 now takes
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      __builtin_amdgcn_s_barrier();
      if (y + 2 <= y1) c64s_load_row(a, smem, x_rsrc, voff, b, y + 2, (y + 2) % RING, tid);
      const bool pair = ((y - y0) & 1) != 0;           // tail of rows (y-1, y)
      const bool single = !pair && y == y1 - 1;        // odd band: tail of row y alone
      // the tail's rows per lane: lanes 0-7 the pair's first row, 8-15 the second
      const int trow = (pair && frow < 8) ? y - 1 : y;
      const bool tok = (frow & 7) < tailn && (pair || frow < 8);
      // pixel indices: B*H*W*128 < 2^31 (checked by the launcher), 32-bit offsets
      const uint32_t rowpix = (uint32_t)((b * a.H + y) * a.W);
      const uint32_t tpix = (uint32_t)((b * a.H + trow) * a.W + min(tcol, a.W - 1));
      // ring rows of input rows y-2 .. y+1 (uniform); the tail's lanes 0-7 of a
      // pair read output row y-1's taps (rb4[kh]), every other lane row y's (rb4[kh + 1])
      uint32_t rb4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) rb4[i] = ring + (uint32_t)(((y - 2 + i + RING) % RING) * RB);
      const bool tprev = pair && frow < 8;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) asm volatile("" : "+v"(loff[kw]));

      auto body = [&](auto nft) {
        constexpr int NF = decltype(nft)::value;       // 3: fragments 0-2; 4: + the tail
        constexpr int NG = 18 * NF;                    // groups (tap, block, fragment)
        float4v rw[HAS_RES ? NF : 1];                   // 16-byte split residual (split_swap_in)
        // residual of the row's fragments -> registers when the row starts
        // (untracked loads, retired by the epilogue's vmcnt(0)): a load issued in
        // the epilogue exposed a full memory latency per row (+25 % on the residual
        // variant)
        auto load_res = [&]() {
          if constexpr (HAS_RES) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
              const uint32_t off = (f < 3 ? rowpix + 16 * f + frow : tpix) * PIX + split_off_q(n0 - 4 * q, q);
              rw[f] = gload_f4_untracked(a.res + off);
            }
          }
        };
        load_res();
        float4v acc[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) acc[f] = float4v{0.f, 0.f, 0.f, 0.f};
        // groups g = (tap t, block cb, pixel fragment F): 2 B reads (hi, lo), 3 MFMAs;
        // a D-deep register ring keeps the reads of groups g+1 .. g+D-1 in flight
        // behind group g's MFMAs (counted lgkmcnt)
        half8v bf[D][2];
        auto issue = [&](int g, int buf) {
          const int t = g / (2 * NF), cb = (g / NF) & 1, F = g % NF;
          const int kh = t / 3, kw = t - 3 * kh;
          uint32_t base;
          if (F < 3) {
            base = rb4[kh + 1] + loff[kw];
          } else {
            // opaque per read: the 9 tail addresses are not hoisted into live registers
            uint32_t ts = tshift;
            asm volatile("" : "+v"(ts));
            base = (tprev ? rb4[kh] : rb4[kh + 1]) + ts + loff[kw];
          }
#pragma unroll
          for (int p = 0; p < 2; ++p) bf[buf][p] = lds_read_frag(base ^ (uint32_t)((2 * cb + p) << 6), F);
        };
#pragma unroll
        for (int p = 0; p < D - 1; ++p) issue(p, p);
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const int buf = g % D;
          if (g + D - 1 < NG) {
            issue(g + D - 1, (g + D - 1) % D);
            c64s_wait_groups<D - 1>();
          } else {
            c64s_wait_groups<0>();
          }
          lds_tie(bf[buf][0]);
          lds_tie(bf[buf][1]);
          const int t = g / (2 * NF), cb = (g / NF) & 1, F = g % NF;
          float4v& c = acc[F];
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][cb][0], bf[buf][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][cb][0], bf[buf][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[t][cb][1], bf[buf][0], c, 0, 0, 0);
        }
        // ---- epilogue: scale, bias (+ residual), ReLU, split store ----
        if constexpr (HAS_RES) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int f = 0; f < NF; ++f) reg_tie(rw[f]);
        }
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          // one 16-byte store per lane (split_swap_out: q even hi, q odd lo of 8
          // channels); the lane swap runs on every lane, the tail's store only
          // where its column is < W (lane 0 always: every store instruction issues)
          const uint32_t off = (f < 3 ? rowpix + 16 * f + frow : tpix) * PIX + split_off_q(n0 - 4 * q, q);
          float4v v = acc[f] * a.acc_scale + *reinterpret_cast<const float4v*>(smem + BIAS + 4 * n0);
          if constexpr (HAS_RES) {
            half4v h, l;
            split_swap_in(rw[f], h, l);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)h[e] + (float)l[e];
          }
          if (a.relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          half4v h, l;
          split_f16x4(v, h, l);
          const u32x4_sw o = split_swap_out(h, l);
          if (f == 3 && !tok) continue;
          split_guard(a.ovf, v);
          *reinterpret_cast<u32x4_sw*>(a.y + off) = o;
        }
      };
      if (pair || single) body(c64s_nf<4>{});
      else body(c64s_nf<3>{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int D>
static void c64s_launch(const C64sArgs& a, bool res, int grid, hipStream_t st) {
  using namespace c64s;
  if (res) {
    ensure_lds_attr(reinterpret_cast<const void*>(conv3x3_split_c64_kernel<true, D>), LDS);
    hipLaunchKernelGGL((conv3x3_split_c64_kernel<true, D>), dim3(grid), dim3(256), LDS, st, a);
  } else {
    ensure_lds_attr(reinterpret_cast<const void*>(conv3x3_split_c64_kernel<false, D>), LDS);
    hipLaunchKernelGGL((conv3x3_split_c64_kernel<false, D>), dim3(grid), dim3(256), LDS, st, a);
  }
}

// Measured and dropped (round 3, profiles/r3_c64_split_variants.md, deleted in round 5):
// 32 couts per wave as one wave per SIMD holding all 64 input channels' A fragments
// (W32, -2.3 %) or as K-split wave pairs exchanging partial sums through LDS (-2.7 %).
// Round 5: W in [49, 56] (three full fragments and a tail of at most 8 columns per
// row; the round-4 kernel's fourth fragment per row also took W up to 62).
bool conv3x3_split_c64_supported(int H, int W, int C, int Cout) {
  return C == 64 && Cout == 64 && W >= 49 && W <= c64s::WMAX && H >= 1;
}

bool conv3x3_split_c64_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                              const void* zero, int B, int H, int W, int relu, float acc_scale, int* ovf,
                              hipStream_t st, int per_cu) {
  using namespace c64s;
  C64sArgs a;
  a.ovf = ovf;
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
  a.acc_scale = acc_scale;
  if ((long)B * H * W * c64s::PIX * 2 >= (1L << 31)) return false;   // 32-bit byte offsets
  // per_cu 0 = auto: two workgroups per CU, or one when two would leave each fewer than
  // 8 rows (B = 50 per GPU: 5.5 rows each, +1.0 % whole forward with one per CU,
  // profiles/r6b_route.md)
  if (per_cu <= 0) per_cu = B * H < 16 * device_cu_count() ? 1 : 2;
  const int per = per_cu * device_cu_count();
  // equal row shares over the resident workgroups, at least 4 rows each (a band
  // loads 2 halo rows and waits for its first 3 rows before computing)
  a.nrows = B * H;
  int grid = (a.nrows + 3) / 4;
  if (grid > per) grid = per;
  c64s_launch<3>(a, res != nullptr, grid, st);
  return true;
}

}  // namespace idunno
