// Implicit-GEMM convolution, v2 main loop: global->LDS DMA (global_load_lds_dwordx4)
// with an NS-deep LDS ring and counted vmcnt waits (cdna_hip_programming §5
// "Pipelining across barriers", T3/T4).  Used for every conv with C % 64 == 0
// (all ResNet / AlexNet convs after the stem, and the FC layers as 1x1 convs).
//
// Why: the v1 register-staged loop (conv_igemm.hip) keeps one K stage in
// flight; at 2-3 waves/SIMD the L2 latency of the im2col gathers is exposed
// every stage and the MFMA pipe idles (~20 % of peak on MI355X, see
// profiles/).  Here NS-1 stages are in flight while the MFMAs of the current
// one run, no VGPRs are spent on staging, and the LDS image is written by the
// DMA engine directly.
//
// LDS image: per stage, A (weights, BN rows) then B (pixels, BM rows), each
// row BK halfs, 16-byte chunks XOR-swizzled per row.  glds writes lane-linear
// (base + lane*16), so the swizzle is applied to the *source* address: the
// lane that lands in slot s of row r loads global chunk s ^ swz(r), and the
// fragment read uses the same XOR (rule 21).  Out-of-image taps (padding) and
// rows past M / Cout load from a 16-byte zero buffer instead of branching.
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;


template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most n (runtime, multiple of G) DMA ops of this wave are pending
template <int G, int NS>
__device__ __forceinline__ void wait_stages(int pending_stages) {
  if constexpr (NS >= 4) {
    if (pending_stages >= 2) { wait_vmcnt<2 * G>(); return; }
  }
  if constexpr (NS >= 3) {
    if (pending_stages >= 1) { wait_vmcnt<G>(); return; }
  }
  wait_vmcnt<0>();
}

// P3: RGB stem on packed rows (preprocess_pack3_f16, x = [B][H][nc][wp] halfs):
// the 3*KW halfs of one kernel row are contiguous in the row copy in which
// they start 16-byte aligned; K = (kh, 16-byte chunk), ceil(3*KW/8) chunks per
// kh (AlexNet 11x11/4: K 448 instead of 704 for NHWC4 on conv_igemm).
//
// SPLIT: fp32-accurate convolution on the f16 MFMA ("split fp16", the fp32
// programs' fast path).  Every fp32 value v is carried as two halfs,
// hi = fp16(v), lo = fp16(v - hi) (22 significant bits), laid out per 32
// channels as [hi x32][lo x32], so one BK = 64 stage holds 32 channels' hi
// and lo parts and the DMA / swizzle machinery is unchanged.  Per stage the
// products hi*hi + hi*lo + lo*hi are summed in f32 (lo*lo, ~2^-22 relative,
// is dropped): 3 f16 MFMAs per 32 channels = 5.3x the f32-MFMA rate.  Weights
// are pre-scaled by 2^e (max |w| ~ 2^14, so their lo parts stay normal) and
// the epilogue multiplies by a.acc_scale = 2^-e (exact).  Residual in, output
// out in the same split layout (or fp32 with OUT_F32).
//
// KS: conv split-K (small M) -- block s / tiles runs its own contiguous run of
// a.kstage K stages into fp32 partials; without it the prologue has no
// kstage / mid-tap start code (the B = 400 launches compile the plain loop).
template <int BN, int BM, int BK, int WN, int WM, int NS, bool HAS_RES, bool OUT_F32, bool P3 = false,
          bool SPLIT = false, bool KS = false>
__global__ void __launch_bounds__(64 * WN * WM, (BM % 64 != 0 && WN * WM == 8) ? 4 : 1)   // 2nd: min waves per SIMD
conv_glds_kernel(const ConvArgs a) {
  static_assert(!SPLIT || BK == 64, "split stages are 32 channels x (hi, lo)");
  static_assert(!KS || (OUT_F32 && !HAS_RES && !P3), "split-K writes fp32 partials");
  constexpr int NW = WN * WM;
  constexpr int NT = 64 * NW;
  constexpr int TN = BN / WN, TM = BM / WM;
  constexpr int FN = TN / 16, FM = TM / 16;
  constexpr int CPR = BK / 8;                 // 16-byte chunks per row
  constexpr int RB = BK * 2;                  // bytes per row
  constexpr int RPI = 64 / CPR;               // rows per DMA instruction (1 KiB)
  // B rows staged per stage: BM rounded up to whole DMA instructions per wave
  // (rows BM.. BMD-1 load zeros and are never read; e.g. BM 160 on 8 waves)
  constexpr int BMD = (BM + RPI * NW - 1) / (RPI * NW) * (RPI * NW);
  constexpr int A_INS = BN / RPI, B_INS = BMD / RPI;
  static_assert(A_INS % NW == 0 && B_INS % NW == 0, "DMA instructions must split evenly over waves");
  constexpr int GA = A_INS / NW, GB = B_INS / NW, G = GA + GB;
  constexpr int A_BYTES = BN * RB, STAGE = (BN + BMD) * RB;
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(G * (NS - 2) < 64, "vmcnt immediate");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave / WM, wm = wave % WM;

  const int nwg = a.tiles_n * a.tiles_m;
  const int nsplit = a.ksplit > 1 ? a.ksplit : 1;
  const int lid_all = xcd_remap(blockIdx.x, nwg * nsplit);
  const int split = lid_all / nwg, lid = lid_all - split * nwg;
  // m-major: an XCD's consecutive blocks share one pixel panel (n-major, sharing a
  // weight panel, was 0-6 % slower: profiles/r2_v26_split_tile_order.md)
  const int tm = lid / a.tiles_n, tn = lid - tm * a.tiles_n;
  const int n0 = tn * BN, m0 = tm * BM;
  // dual conv: this tile belongs to the second conv (see ConvArgs::nsplit_n)
  const bool second = a.nsplit_n > 0 && n0 >= a.nsplit_n;
  const half_t* const xin = a.x + (size_t)split * a.kslice;        // split-K: this block's K slice
  const half_t* const win = a.w + (size_t)split * a.kslice;

  const half_t* zero = reinterpret_cast<const half_t*>(a.zero);
  const int lrow = lane / CPR, lslot = lane % CPR;

  // A sources: per DMA instruction j of this wave, a row base pointer (or zero)
  const half_t* a_src[GA];
  int a_ch[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int row = (wave + NW * j) * RPI + lrow;
    const int n = n0 + row;
    a_ch[j] = (lslot ^ swz_r(row, CPR)) * 8;
    a_src[j] = n < a.Cout ? win + (size_t)n * a.Kpad + a_ch[j] : nullptr;
  }
  // B sources: pixel decomposition per instruction (pixel stride ldx: a K-slice
  // of wider rows when the caller splits K, e.g. linear_splitk)
  const int ldx = a.ldx ? a.ldx : a.C;
  int b_base[GB], b_ih0[GB], b_iw0[GB], b_ch[GB];
  const int prow = a.nc * a.wp * (SPLIT ? 2 : 1);     // P3: halfs per image row (all copies, both planes)
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = (wave + NW * j) * RPI + lrow;
    const int m = m0 + row;
    b_ch[j] = (lslot ^ swz_r(row, CPR)) * 8;
    if (row < BM && m < a.M) {
      const int hw = a.Ho * a.Wo;
      const int b = m / hw, r = m - b * hw;
      const int oh = r / a.Wo, ow = r - oh * a.Wo;
      if constexpr (P3) {
        const int r0 = 3 * a.stride * ow;              // first half of the pixel's kernel row in R
        const int sh = r0 & 7, g = 8 / a.nc;           // copy sh/g starts it 16-byte aligned
        b_base[j] = b * a.H * prow + (sh / g) * a.wp + r0 - sh;
      } else {
        b_base[j] = b * a.H * a.W * ldx + b_ch[j];
      }
      b_ih0[j] = oh * a.stride - a.pad;
      b_iw0[j] = ow * a.stride - a.pad;
    } else {
      b_base[j] = -1;
      b_ih0[j] = -100000;
      b_iw0[j] = -100000;
    }
  }

  // issue-side K coordinates (run NS-1 stages ahead of compute); the second
  // conv of a centre-only dual launch covers the centre tap's cblk stages
  int i_s = 0, i_cb = 0, i_kw = 0, i_kh = 0;
  int nK = a.nK;
  if (second && a.center_only) {
    i_kh = a.KH / 2;
    i_kw = a.KW / 2;
    i_s = (i_kh * a.KW + i_kw) * a.cblk;
    nK = a.cblk;
  }
  if constexpr (KS) {                          // conv split-K: this block's contiguous run of K stages
    i_s = split * a.kstage;
    i_cb = i_s % a.cblk;
    const int tap = i_s / a.cblk;
    i_kw = tap % a.KW;
    i_kh = tap / a.KW;
    nK = a.kstage;
  }
  // Buffer-resource DMA (every non-P3 conv; operands must fit 2 GiB, glds_cfg):
  // per-lane byte offsets are fixed -- A for the whole launch, B per kernel
  // tap (recomputed when the channel block wraps) -- and the stage's K offset
  // is the instruction's SGPR soffset, so a stage's DMA costs no VALU (the
  // global-pointer form spent ~28 VALU per stage on ih/iw/bounds/64-bit adds,
  // and the 128x128 split tile is issue-bound: profiles/r3_pmc_split_forward.md).
  // Padding taps and rows past M / Cout get an offset past num_records: the
  // hardware returns zeros.
  constexpr uint32_t OOR = 0x80000000u;
  const auto w_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)win, 0, 0x7fffffff, 0x00020000);
  const auto x_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)xin, 0, 0x7fffffff, 0x00020000);
  uint32_t a_voff[GA], b_voff[GB];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int n = n0 + (wave + NW * j) * RPI + lrow;
    a_voff[j] = n < a.Cout ? (uint32_t)((n * a.Kpad + a_ch[j]) * 2) : OOR;
  }
  auto set_tap = [&]() {
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int ih = b_ih0[j] + i_kh, iw = b_iw0[j] + i_kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      b_voff[j] = ok ? (uint32_t)((b_base[j] + (ih * a.W + iw) * ldx) * 2) : OOR;
    }
  };
  if constexpr (KS) {
    if (i_cb != 0) set_tap();                  // a split-K slice that starts inside a tap
  }
  auto issue_buf = [&](int buf) {
    char* base = smem + buf * STAGE;
    if (i_cb == 0) set_tap();
    const int koff = i_s * BK * 2, coff = i_cb * BK * 2;
#pragma unroll
    for (int j = 0; j < GA; ++j)
      dma_buf16(w_rsrc, base + (wave + NW * j) * 1024, a_voff[j], koff);
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      // padded B rows (BM .. BMD-1, e.g. 160 .. 191) are never read: no DMA for
      // them (wave-uniform; NS = 2 waits with vmcnt(0), so the counts need not match)
      if constexpr (BMD != BM) {
        static_assert(BMD == BM || (NS == 2 && BM % RPI == 0), "skipped padding instructions need vmcnt(0) waits");
        if ((wave + NW * j) * RPI >= BM) continue;
      }
      dma_buf16(x_rsrc, base + A_BYTES + (wave + NW * j) * 1024, b_voff[j], coff);
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
  auto issue_glb = [&](int buf) {
    char* base = smem + buf * STAGE;
    const int koff = i_s * BK;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const half_t* src = a_src[j] ? a_src[j] + koff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + (wave + NW * j) * 1024), 16, 0, 0);
    }
    const int coff = i_cb * BK;
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      if constexpr (P3) {
        // this lane's chunk of stage i_s: flat chunk q = i_s*CPR + ch over (kh, chunk)
        // SPLIT: chunks 0-3 of a stage are the hi plane's flat chunks
        // 4*i_s .. +3, chunks 4-7 the lo plane's same chunks
        int q, poff = 0;
        if constexpr (SPLIT) {
          const int cc = b_ch[j] / 8;
          q = i_s * 4 + (cc & 3);
          poff = (cc >> 2) * a.nc * a.wp;
        } else {
          q = i_s * CPR + b_ch[j] / 8;
        }
        const int kh = q / a.cpk, jj = q - kh * a.cpk;
        const int ih = b_ih0[j] + kh;
        const bool ok = kh < a.KH && (unsigned)ih < (unsigned)a.H;
        const half_t* src = ok ? xin + b_base[j] + ih * prow + 8 * jj + poff : zero;
        __builtin_amdgcn_global_load_lds((glb_void_t*)src,
                                         (lds_void_t*)(base + A_BYTES + (wave + NW * j) * 1024), 16, 0, 0);
        continue;
      }
      const int ih = b_ih0[j] + i_kh, iw = b_iw0[j] + i_kw;
      const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      const half_t* src = ok ? xin + b_base[j] + (ih * a.W + iw) * ldx + coff : zero;
      __builtin_amdgcn_global_load_lds((glb_void_t*)src,
                                       (lds_void_t*)(base + A_BYTES + (wave + NW * j) * 1024), 16, 0, 0);
    }
    // advance (cb fastest, then kw, then kh) == weight K order (kh, kw, c)
    ++i_s;
    if (++i_cb == a.cblk) {
      i_cb = 0;
      if (++i_kw == a.KW) {
        i_kw = 0;
        ++i_kh;
      }
    }
  };
  auto issue = [&](int buf) {
    if constexpr (P3) issue_glb(buf);
    else issue_buf(buf);
  };

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // residual of this tile -> registers before the ring's first DMA: untracked
  // loads (common.h) older than every DMA, so the ring's counted vmcnt waits
  // retire them long before the epilogue, whose own load would otherwise expose
  // a full memory latency per tile (30 us of 138 on ResNet layer2 conv2,
  // profiles/r1_v8_conv_big_sweep.log)
  //
  // SPLIT loads its residual (hi and lo: twice the registers) only after the
  // main loop instead: held across the loop it took the 128x128 8-wave tile
  // from 112 to 140 VGPRs, one block per CU instead of two, +25-50 % time.
  // The padded-B tiles (BMD > BM, e.g. 128 x 160) load it late too: their
  // register budget (>= 4 waves/SIMD) would spill the untracked preload, and a
  // spill of an asm load's destination before the load lands corrupts it.
  constexpr bool LATE_RES = SPLIT || BMD != BM;
  half4v rv[HAS_RES ? FN : 1][HAS_RES ? FM : 1];
  // SPLIT: the residual as one 16-byte load per lane and fragment (split_swap_in)
  float4v rw[HAS_RES && SPLIT ? FN : 1][HAS_RES && SPLIT ? FM : 1];
  if constexpr (HAS_RES && !LATE_RES) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = m0 + wm * TM + j * 16 + (lane & 15);
        const size_t off = (m < a.M && n < a.Cout) ? (size_t)m * (a.ldr ? a.ldr : a.Cout) + n : 0;
        rv[i][j] = gload_b64_untracked(a.res + off);
      }
    }
  }

  const int frow = lane & 15, fch = lane >> 4;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nK) issue(p);

  // per-lane LDS byte offsets (within a stage) of fragment 0 of each K chunk
  uint32_t frag_a[BK / 32], frag_b[BK / 32];
#pragma unroll
  for (int kk = 0; kk < BK / 32; ++kk) {
    const int ch = fch + 4 * kk;
    const int ra = wn * TN + frow, rb = wm * TM + frow;
    frag_a[kk] = (uint32_t)(ra * RB + ((ch ^ swz_r(ra, CPR)) << 4));
    frag_b[kk] = (uint32_t)(A_BYTES + rb * RB + ((ch ^ swz_r(rb, CPR)) << 4));
  }
  for (int s = 0; s < nK; ++s) {
    const int ahead = min(NS - 2, nK - 1 - s);
    wait_stages<G, NS>(ahead);
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < nK) issue((s + NS - 1) % NS);

    // fragment reads through inline asm (common.h lds_read_b128): a compiler-
    // emitted ds_read here gets an `s_waitcnt vmcnt(0)` in front of it that
    // drains the stage just issued above, and the ring never overlaps loads
    // with MFMAs.  All reads of the stage go out first; each K-chunk of 32 then
    // waits (counted lgkmcnt) only for its own fragments.
    const uint32_t base = lds_addr(smem) + (s % NS) * STAGE;
    constexpr int KK = BK / 32, NR = FN + FM;
    half8v fa[KK][FN], fb[KK][FM];
    // fragment rows 16 apart share the swizzle (swz_r(row) depends on row mod 16
    // for both row sizes), so fragment i of chunk kk is the lane's chunk-kk
    // address + i * 16 rows: one VGPR add per (operand, kk) and stage, the rest
    // immediate offsets (the per-read address adds were 16 VALU per stage)
    static_assert(16 * RB * (FN > FM ? FN : FM) <= 65536, "fragment offsets must fit the ds immediate");
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const uint32_t abase = base + frag_a[kk], bbase = base + frag_b[kk];
#pragma unroll
      for (int i = 0; i < FN; ++i) fa[kk][i] = lds_read_b128_step<16 * RB>(abase, i);
#pragma unroll
      for (int j = 0; j < FM; ++j) fb[kk][j] = lds_read_b128_step<16 * RB>(bbase, j);
    }
    auto mfma_chunk = [&](int kk) {
#pragma unroll
      for (int i = 0; i < FN; ++i) lds_tie(fa[kk][i]);
#pragma unroll
      for (int j = 0; j < FM; ++j) lds_tie(fb[kk][j]);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
    };
    static_assert(KK == 1 || KK == 2, "BK 32 or 64");
    if constexpr (SPLIT) {
      // chunk 0 = hi, chunk 1 = lo: hi*hi as soon as the hi fragments land,
      // then hi*lo + lo*hi
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
      // keep the hi*hi MFMAs above the second wait: without this barrier the
      // scheduler sank them below it, so no MFMA issued before every read landed
      __builtin_amdgcn_sched_barrier(0);
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
      continue;
    }
    if constexpr (KK == 2) {
      lds_waitcnt<NR>();                         // chunk 0 landed, chunk 1 may be in flight
      mfma_chunk(0);
      __builtin_amdgcn_sched_barrier(0);         // (as above: chunk 0's MFMAs stay above the wait)
    }
    lds_waitcnt<0>();
    mfma_chunk(KK - 1);
  }

  // ---- epilogue: bias (+residual) (+ReLU), NHWC store --------------------
  // late residual: the ring is drained (last wait was vmcnt(0)), so ordinary
  // tracked loads; all at once, or per cout fragment for the padded-B tiles
  // (whose epilogue would otherwise spill at their <= 128-VGPR budget)
  constexpr bool RES_PER_I = LATE_RES && BMD != BM;
  auto load_res = [&](int i) {
    const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + j * 16 + (lane & 15);
      const bool ok = m < a.M && n < a.Cout;
      if constexpr (SPLIT) {
        const int q = lane >> 4;
        const size_t off = ok ? (size_t)m * (a.ldr ? a.ldr : 2 * a.Cout) + split_off_q(n - 4 * q, q) : 0;
        rw[i][j] = *reinterpret_cast<const float4v*>(a.res + off);
      } else {
        const size_t off = ok ? (size_t)m * (a.ldr ? a.ldr : a.Cout) + n : 0;
        rv[i][j] = *reinterpret_cast<const half4v*>(a.res + off);
      }
    }
  };
  const float acc_scale = SPLIT ? (second ? a.acc_scale2 : a.acc_scale) : 1.f;
  const bool relu = a.relu && !second;
  if constexpr (HAS_RES && LATE_RES && !RES_PER_I) {
#pragma unroll
    for (int i = 0; i < FN; ++i) load_res(i);
  } else if constexpr (HAS_RES && !LATE_RES) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (already retired by the ring's last wait)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) reg_tie(rv[i][j]);
  }
  // fp16 output: the two 16-cout fragments of a pair swap halves (f16_pair_off),
  // one 16-byte store per lane and pair instead of two 8-byte ones
  constexpr bool PAIR_ST = !SPLIT && !OUT_F32 && FN % 2 == 0 && !(HAS_RES && RES_PER_I);
  if constexpr (PAIR_ST) {
    if (a.Cout % 32 == 0 && a.ldy % 8 == 0) {   // pairs never straddle Cout; 16-byte rows (uniform)
      const int q = lane >> 4;
#pragma unroll
      for (int i = 0; i < FN; i += 2) {
        const int nb = n0 + wn * TN + i * 16;
        if (nb >= a.Cout) continue;
        const float4v bv0 = *reinterpret_cast<const float4v*>(a.bias + nb + 4 * q);
        const float4v bv1 = *reinterpret_cast<const float4v*>(a.bias + nb + 16 + 4 * q);
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int m = m0 + wm * TM + j * 16 + (lane & 15);
          half4v o[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            float4v v = acc[i + k][j] + (k ? bv1 : bv0);
            if constexpr (HAS_RES) {
              const half4v r = rv[i + k][j];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += (float)r[e];
            }
            if (relu) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) o[k][e] = (half_t)v[e];
          }
          const u32x4_sw w = split_swap_out(o[0], o[1]);   // every lane swaps
          if (m < a.M)
            *reinterpret_cast<u32x4_sw*>(static_cast<half_t*>(a.y) + (size_t)m * a.ldy + f16_pair_off(nb, q)) = w;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * TN + i * 16 + (lane >> 4) * 4;
    if (n >= a.Cout) continue;
    if constexpr (HAS_RES && RES_PER_I) load_res(i);
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * TM + j * 16 + (lane & 15);
      if (m >= a.M) continue;
      float4v v;
      if constexpr (SPLIT) v = acc[i][j] * acc_scale + bv;
      else v = acc[i][j] + bv;
      if constexpr (HAS_RES) {
        const half4v r = rv[i][j];
        if constexpr (SPLIT) {
          half4v h, l;
          split_swap_in(rw[i][j], h, l);
          v[0] += (float)h[0] + (float)l[0];
          v[1] += (float)h[1] + (float)l[1];
          v[2] += (float)h[2] + (float)l[2];
          v[3] += (float)h[3] + (float)l[3];
        } else {
          v[0] += (float)r[0];
          v[1] += (float)r[1];
          v[2] += (float)r[2];
          v[3] += (float)r[3];
        }
      }
      if (relu) {
        v[0] = fmaxf(v[0], 0.f);
        v[1] = fmaxf(v[1], 0.f);
        v[2] = fmaxf(v[2], 0.f);
        v[3] = fmaxf(v[3], 0.f);
      }
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4v*>(static_cast<float*>(a.y) + (size_t)split * a.ysplit + (size_t)m * a.ldy + n) = v;
      } else if constexpr (SPLIT) {
        split_guard(a.ovf, v);
        half4v h, l;
        split_f16x4(v, h, l);
        // one 16-byte store per lane: q even the hi, q odd the lo halfs of 8 channels
        // (the lanes of one pixel share m, so a pixel's lanes swap together)
        const int q = lane >> 4;
        half_t* yp = static_cast<half_t*>(a.y) + (size_t)m * a.ldy + split_off_q(n - 4 * q, q);
        *reinterpret_cast<u32x4_sw*>(yp) = split_swap_out(h, l);
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

// the buffer-resource DMA addresses x and w with 32-bit byte offsets
static bool glds_fits(const ConvArgs& a) {
  const long xb = (long)a.B * a.H * a.W * (a.ldx ? a.ldx : a.C) * 2, wb = (long)a.Cout * a.Kpad * 2;
  return xb < (1L << 31) && wb < (1L << 31);
}

template <int BN, int BM, int BK, int WN, int WM, int NS, bool HAS_RES, bool OUT_F32, bool P3 = false,
          bool SPLIT = false, bool KS = false>
static void glds_cfg(ConvArgs a, hipStream_t st) {
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles_m = (a.M + BM - 1) / BM;
  if (P3) {
    a.cblk = 1;
    const int cps = SPLIT ? BK / 16 : BK / 8;          // input chunks per stage (SPLIT: hi + lo of 4)
    a.nK = (a.KH * a.cpk + cps - 1) / cps;
  } else {
    a.cblk = a.C / BK;
    a.nK = a.KH * a.KW * a.cblk;
  }
  const int grid = a.tiles_n * a.tiles_m * (a.ksplit > 1 ? a.ksplit : 1);
  constexpr int RPI_ = 64 / (BK / 8), NW_ = WN * WM;
  constexpr int BMD = (BM + RPI_ * NW_ - 1) / (RPI_ * NW_) * (RPI_ * NW_);
  const size_t lds = (size_t)NS * (BN + BMD) * BK * 2;
  auto kern = conv_glds_kernel<BN, BM, BK, WN, WM, NS, HAS_RES, OUT_F32, P3, SPLIT, KS>;
  ensure_lds_attr(reinterpret_cast<const void*>(kern), (int)lds);   // per (kernel, device), launch_util.h
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WN * WM), lds, st, a);
}

// Tile table (id -> config).  Exposed ids are stable: tests sweep all of them.
//   10: 128x128, BK 64, 4 waves (2x2), 3 stages   96 KiB LDS
//   11: 128x128, BK 32, 4 waves (2x2), 4 stages   64 KiB
//   12: 64x256,  BK 64, 4 waves (1x4), 3 stages   120 KiB
//   13: 64x256,  BK 32, 4 waves (1x4), 4 stages   80 KiB
//   14: 128x256, BK 64, 8 waves (2x4), 3 stages   144 KiB
//   15: 64x128,  BK 64, 4 waves (1x4), 3 stages   72 KiB
//   16: 128x64,  BK 64, 4 waves (2x2), 3 stages   72 KiB
//   17: 256x128, BK 64, 8 waves (4x2), 3 stages   144 KiB
//   18: 128x128, BK 32, 4 waves, 3 stages 48 KiB   19: 128x64, BK 32, 4 stages 48 KiB
//   20: 64x128,  BK 32, 4 stages 48 KiB            21: 256x128, BK 32, 8 waves, 4 stages 96 KiB
//   22: 128x256, BK 32, 8 waves, 4 stages 96 KiB   23: 64x64, BK 64, 4 waves (2x2), 3 stages 48 KiB
// The measured-and-dropped variants (32x32x16 MFMA tiles 55-59 / 90-92, deep pixel ring
// 60 / 61, input-footprint L2 prefetch) were deleted in round 5 (docs/KERNELS.md keeps
// their numbers; the code is in git history before commit "prune dropped conv variants").
template <bool R, bool F>
static bool glds_dispatch(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 10: glds_cfg<128, 128, 64, 2, 2, 3, R, F>(a, st); return true;
    case 11: glds_cfg<128, 128, 32, 2, 2, 4, R, F>(a, st); return true;
    case 12: glds_cfg<64, 256, 64, 1, 4, 3, R, F>(a, st); return true;
    case 13: glds_cfg<64, 256, 32, 1, 4, 4, R, F>(a, st); return true;
    case 14: glds_cfg<128, 256, 64, 2, 4, 3, R, F>(a, st); return true;
    case 15: glds_cfg<64, 128, 64, 1, 4, 3, R, F>(a, st); return true;
    case 16: glds_cfg<128, 64, 64, 2, 2, 3, R, F>(a, st); return true;
    case 17: glds_cfg<256, 128, 64, 4, 2, 3, R, F>(a, st); return true;
    case 18: glds_cfg<128, 128, 32, 2, 2, 3, R, F>(a, st); return true;
    case 19: glds_cfg<128, 64, 32, 2, 2, 4, R, F>(a, st); return true;
    case 20: glds_cfg<64, 128, 32, 1, 4, 4, R, F>(a, st); return true;
    case 21: glds_cfg<256, 128, 32, 4, 2, 4, R, F>(a, st); return true;
    case 22: glds_cfg<128, 256, 32, 2, 4, 4, R, F>(a, st); return true;
    case 23: glds_cfg<64, 64, 64, 2, 2, 3, R, F>(a, st); return true;
    case 24: glds_cfg<128, 128, 64, 2, 4, 3, R, F>(a, st); return true;   // 8 waves, 96 KiB
    case 25: glds_cfg<256, 128, 64, 4, 2, 2, R, F>(a, st); return true;   // 8 waves, 96 KiB, dbuf
    case 26: glds_cfg<128, 128, 64, 2, 2, 2, R, F>(a, st); return true;   // 64 KiB dbuf, 2 blk/CU
    case 27: glds_cfg<64, 128, 64, 1, 4, 2, R, F>(a, st); return true;    // 48 KiB dbuf, 3 blk/CU
    case 28: glds_cfg<64, 256, 32, 1, 4, 3, R, F>(a, st); return true;    // 60 KiB, 2 blk/CU
    case 29: glds_cfg<64, 256, 64, 1, 8, 3, R, F>(a, st); return true;    // 8 waves, 120 KiB
    case 30: glds_cfg<128, 256, 64, 2, 4, 2, R, F>(a, st); return true;   // 8 waves, 96 KiB dbuf
    case 31: glds_cfg<64, 128, 32, 1, 4, 3, R, F>(a, st); return true;    // 36 KiB, 4 blk/CU
    case 32: glds_cfg<128, 128, 32, 2, 2, 2, R, F>(a, st); return true;   // 32 KiB dbuf
    case 33: glds_cfg<64, 256, 64, 1, 4, 2, R, F>(a, st); return true;    // 80 KiB dbuf
    case 34: glds_cfg<128, 64, 64, 2, 2, 2, R, F>(a, st); return true;    // 48 KiB dbuf
    case 35: glds_cfg<64, 64, 64, 2, 2, 2, R, F>(a, st); return true;     // 32 KiB dbuf, 5 blk/CU
    case 36: glds_cfg<128, 128, 64, 2, 4, 2, R, F>(a, st); return true;   // 8 waves, 64 KiB dbuf
    case 37: glds_cfg<64, 128, 64, 1, 8, 2, R, F>(a, st); return true;    // 8 waves, 48 KiB dbuf
    case 38: glds_cfg<128, 64, 64, 2, 4, 2, R, F>(a, st); return true;    // 8 waves (32x16 wave tile)
    case 39: glds_cfg<128, 128, 32, 2, 4, 4, R, F>(a, st); return true;   // 8 waves, 64 KiB, 3 stages in flight
    case 42: glds_cfg<128, 160, 64, 4, 2, 2, R, F>(a, st); return true;   // 8 waves, B as 192 rows, 80 KiB (small M)
    default: return false;
  }
}

// split-K instantiations (fp32 partials, no residual): the auto-pickable BK-64 tiles
template <bool SPLIT>
static bool glds_dispatch_ks(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 27: glds_cfg<64, 128, 64, 1, 4, 2, false, true, false, SPLIT, true>(a, st); return true;
    case 36: glds_cfg<128, 128, 64, 2, 4, 2, false, true, false, SPLIT, true>(a, st); return true;
    case 42: glds_cfg<128, 160, 64, 4, 2, 2, false, true, false, SPLIT, true>(a, st); return true;
    default: return false;
  }
}

// pack3 stems: a few tile shapes (Cout 64: 64-row weight tiles)
template <bool F>
static bool glds_dispatch_p3(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 23: glds_cfg<64, 64, 64, 2, 2, 3, false, F, true>(a, st); return true;
    case 27: glds_cfg<64, 128, 64, 1, 4, 2, false, F, true>(a, st); return true;
    case 31: glds_cfg<64, 128, 32, 1, 4, 3, false, F, true>(a, st); return true;
    case 33: glds_cfg<64, 256, 64, 1, 4, 2, false, F, true>(a, st); return true;
    case 35: glds_cfg<64, 64, 64, 2, 2, 2, false, F, true>(a, st); return true;
    default: return false;
  }
}

// split fp16 (fp32-accurate) tiles: the BK = 64 shapes of the fp16 table that were
// measured useful: 36 / 42 / 27 are the defaults (conv_glds_split_pick), 26 / 34 / 38
// near-equal alternatives.  Measured and dropped (profiles/r2_v24..v29, r3, r4): 14/17/25/30
// (256-wide), 15/16/41 (3-stage rings), 24, 33, 35, 37, 43, 32x32x16 MFMA tiles, deep
// pixel ring -- 5-45 % slower on every ResNet layer.
template <bool R, bool F>
static bool glds_dispatch_split(ConvArgs a, int tile, hipStream_t st) {
  switch (tile) {
    case 26: glds_cfg<128, 128, 64, 2, 2, 2, R, F, false, true>(a, st); return true;
    case 27: glds_cfg<64, 128, 64, 1, 4, 2, R, F, false, true>(a, st); return true;
    case 34: glds_cfg<128, 64, 64, 2, 2, 2, R, F, false, true>(a, st); return true;
    case 36: glds_cfg<128, 128, 64, 2, 4, 2, R, F, false, true>(a, st); return true;
    case 38: glds_cfg<128, 64, 64, 2, 4, 2, R, F, false, true>(a, st); return true;
    // 128 x 160 (B staged as 192 rows): 0.96 waves of blocks on ResNet layer4
    // at B = 400 where 128 x 64 tiles make 1.6 (the partial last wave idles)
    case 42: glds_cfg<128, 160, 64, 4, 2, 2, R, F, false, true>(a, st); return true;    // 8 waves, 80 KiB
    default: return false;
  }
}

bool conv_glds_split_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st) {
  if (!glds_fits(a)) return false;
  if (a.kstage > 0) return out_f32 && a.res == nullptr && glds_dispatch_ks<true>(a, tile, st);
  const bool res = a.res != nullptr;
  if (res) return out_f32 ? glds_dispatch_split<true, true>(a, tile, st) : glds_dispatch_split<true, false>(a, tile, st);
  return out_f32 ? glds_dispatch_split<false, true>(a, tile, st) : glds_dispatch_split<false, false>(a, tile, st);
}

// Conv split-K for small M (strong scaling: a 400-image query over 8 GPUs is 50
// images per GPU, and ResNet layer4 then makes 64 blocks of tile 42 on 256 CUs):
// K slices of whole (kh, kw, cblk) stage runs in ONE launch into fp32 partials,
// then splitk_reduce_res adds bias (+ residual), ReLU and re-splits.
//   force < 0: auto (only for the auto-picked tile); 0 / 1: off; k > 1: k slices
//   (k must divide the K loop: 1 is returned otherwise).
static void ks_tile_dims(int tile, int& bn, int& bm) {
  switch (tile) {
    case 42: bn = 128; bm = 160; return;
    case 27: bn = 64; bm = 128; return;
    default: bn = 128; bm = 128; return;        // 36
  }
}
// target_blocks: the grid the doubling may reach; min_stages: K stages each slice keeps.
static int ksplit_rule(int force, int M, int Cout, int tile, int nk_total, long target_blocks, int min_stages) {
  if (tile != 27 && tile != 36 && tile != 42) return 1;   // split-K instantiations (glds_dispatch_ks)
  if (force == 0 || force == 1) return 1;
  if (force > 1) return nk_total % force == 0 ? force : 1;
  if (nk_total < 2 * min_stages) return 1;
  int bn, bm;
  ks_tile_dims(tile, bn, bm);
  const long blocks = (long)((M + bm - 1) / bm) * ((Cout + bn - 1) / bn);
  int s = 1;
  // double the slices while the grid stays within target_blocks, each slice keeps
  // >= min_stages stages and the slices divide the K loop evenly (at most 8:
  // capping at 4 lost 11 % at B = 8, profiles/r4_ab_ksplit_cap4_b8.log)
  while (s < 8 && blocks * s * 2 <= target_blocks && nk_total % (s * 2) == 0 && nk_total / (s * 2) >= min_stages)
    s *= 2;
  return s;
}
// Split convs (round 6, per-layer sweep at B = 50, profiles/r6a_b50_sweep.log): double
// only while the grid stays within ONE block per CU and every slice keeps >= 8 stages.
// The round-4 rule (two blocks per CU, >= 4 stages; legacy = true) split ResNet18
// layer2 at B = 50 in two (t42k2 49.0 vs t42k1 43.2 us on the residual conv) and the
// layer4 1x1 downsample (16.6 vs 11.5 us): the fp32 partials' round trip through
// splitk_reduce_res cost more than the half-empty wave it filled.
int conv_split_ksplit(int M, int Cout, int tile, int nk_total, int force, bool legacy) {
  if (legacy) return ksplit_rule(force, M, Cout, tile, nk_total, 2L * device_cu_count(), 4);
  return ksplit_rule(force, M, Cout, tile, nk_total, (long)device_cu_count(), 8);
}
int conv_f16_ksplit(int M, int Cout, int tile, int nk_total, int force) {
  // fp16's BK-64 tiles 27 / 42 keep the round-4 rule (fp16 small batches are bound by
  // the per-layer launch chain more than by occupancy, docs/KERNELS.md)
  return ksplit_rule(force, M, Cout, tile, nk_total, 2L * device_cu_count(), 4);
}

// Default split tile (a stage is 32 channels instead of 64, so a tile does 3x the
// MFMAs per byte staged): 128 x 128 8-wave tiles where M is large, 128 x 160 for
// layer4-sized GEMMs (~1 full wave of blocks where 128 x 64 made 1.6; whole-graph
// A/B profiles/r2_v29_split_wide_tile.md; 128 x 160 at every M: ResNet18 -2.9 %).
int conv_glds_split_pick(int M, int Cout) {
  if (Cout % 128 == 0) return M >= 50000 ? 36 : 42;
  return 27;
}

// Small-M 1x1 convs (the ResNet downsample at B = 50 per GPU: M 9800 / 2450) run on the
// 128 x 64 8-wave tile without split-K instead of the persistent streaming 1x1 kernel,
// whose register-resident weights and 2-tile ring do not amortise over a few tiles per
// CU (layer3 ds 13.2 -> 8.6 us, layer4 ds 12.4 -> 7.4 us, profiles/r6a_b50_sweep.log).
bool conv1x1_small_m(long M) { return M < 16384; }

bool conv_glds_split_p3_launch(ConvArgs a, int tile, hipStream_t st) {
  if (a.res != nullptr || a.cpk <= 0) return false;
  switch (tile) {
    case 23: glds_cfg<64, 64, 64, 2, 2, 3, false, true, true, true>(a, st); return true;
    case 27: glds_cfg<64, 128, 64, 1, 4, 2, false, true, true, true>(a, st); return true;
    case 33: glds_cfg<64, 256, 64, 1, 4, 2, false, true, true, true>(a, st); return true;
    case 35: glds_cfg<64, 64, 64, 2, 2, 2, false, true, true, true>(a, st); return true;
    case 37: glds_cfg<64, 128, 64, 1, 8, 2, false, true, true, true>(a, st); return true;
    default: return false;
  }
}

bool conv_glds_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st) {
  const bool res = a.res != nullptr;
  if (a.cpk > 0) {
    if (res) return false;
    return out_f32 ? glds_dispatch_p3<true>(a, tile, st) : glds_dispatch_p3<false>(a, tile, st);
  }
  if (!glds_fits(a)) return false;
  if (a.kstage > 0) return out_f32 && !res && glds_dispatch_ks<false>(a, tile, st);
  if (res) return out_f32 ? glds_dispatch<true, true>(a, tile, st) : glds_dispatch<true, false>(a, tile, st);
  return out_f32 ? glds_dispatch<false, true>(a, tile, st) : glds_dispatch<false, false>(a, tile, st);
}

// Default fp16 tile: 128 x 160 (8 waves, BK 64) for every 128-multiple Cout (after the
// buffer-DMA rewrite: ResNet18 b400 +4.2 %, ResNet50 b1024 +3.4 %, profiles/r3_ab_f16_wide_all.md),
// 64 x 128 otherwise.
int conv_glds_pick(int M, int Cout) {
  (void)M;
  return Cout % 128 == 0 ? 42 : 27;
}

}  // namespace idunno
