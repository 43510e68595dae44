// fp32 3x3 / stride-1 / pad-1 convolution by Winograd F(2x2, 3x3), fully fused
// (input transform -> 16 GEMMs on the f32-input MFMA -> output transform ->
// bias / residual / ReLU) in ONE kernel.  All arithmetic is fp32: this is the
// algorithm cuDNN / MIOpen use for fp32 3x3 convs, here written for gfx950.
//
// Why: the fp32 direct conv (conv_f32.hip) already runs at ~120 TF/s, i.e. at
// the f32-MFMA roofline (157 TF peak, 1/16 of f16), on every ResNet 3x3 layer
// (profiles/r2_v1_layers_f32.md).  The only way past that roofline at fp32 is
// fewer multiplications: F(2x2,3x3) computes a 2x2 output tile from a 4x4 input
// patch with 16 instead of 36 products per (cin, cout), 2.25x less MFMA work.
//
//   V = B^T d B  (4x4 input patch d, per channel)      B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   U = G g G^T  (3x3 filter g, precomputed on host)  G   = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]
//   M_e = sum_c U_e[cout][c] V_e[c][tile]   for the 16 elements e = (i, j)
//   Y = A^T M A  (2x2 output tile)                     A^T = [1 1 1 0; 0 1 -1 -1]
//
// Structure (one workgroup = 32 output channels x T = 16*NW tiles, all 16 e):
//   * the raw input region of the block's tiles (whole tile rows of one image,
//     or whole images when an image has few tiles) is staged once per
//     16-channel chunk by LDS-DMA (global_load_lds_dwordx4), deduplicated (a
//     4x4 patch per tile would be 4x the bytes);
//   * U for the 32 channels, 16 e and the chunk's 16 input channels (32 KiB)
//     is staged next to it; two stages, so chunk k+1 lands while k computes;
//   * every wave owns 16 tiles (the MFMA's 16 columns) x all 32 output
//     channels x all 16 e: 32 accumulators of 4 f32.  A lane reads the 4x4
//     patch of ITS tile for ITS 4 channels (16 ds_read_b128), transforms it in
//     registers, and the 16 results ARE its B operands of the 16 e-GEMMs (lane
//     l: tile l&15, channels 4(l>>4)..+3, the conv_f32.hip k-permutation), so V
//     never touches LDS or HBM;
//   * because a wave holds all 16 e of its (tile, channel) accumulators, the
//     output transform, bias, residual and ReLU run in registers and each lane
//     stores whole 16-byte channel quads of NHWC output.
// LDS raw layout: [image row][column parity][pixel][4 chunks of 4 channels],
// chunk XOR ((pixel >> 2) & 1) << 1: a wave's 16 lanes of one channel group
// read 16 consecutive even (or odd) pixels of one row -> 16 distinct 16-byte
// bank slots per ds_read_b128 lane group (conflict-free, checked offline).
#include "../kernels.h"
#include "../launch_util.h"

namespace idunno {

namespace {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int kRawMax = 40 * 1024;      // staged input region per stage (bytes)
constexpr int kUBytes = 16 * 32 * 64;   // 16 e x 32 couts x 16 channels x 4 B = 32 KiB
constexpr int kStage = kRawMax + kUBytes;
// variant 3 (one stage, two blocks per CU): 72 KiB per block (the rotated 7x7
// layout holds 4 images x 10 rows x 2 x 8 pixels x 64 B = 40 KiB)
constexpr int kRaw3 = 40 * 1024;

__device__ __forceinline__ int raw_swz(int p) { return wino_raw_swz(p); }   // tile_math.h

template <bool ASM>
__device__ __forceinline__ float4v ldsr(uint32_t addr) {
  if constexpr (ASM) return lds_read_f4(addr);
  else return *reinterpret_cast<const __attribute__((address_space(3))) float4v*>((size_t)addr);
}
template <bool ASM, int N>
__device__ __forceinline__ void lds_wait() {
  if constexpr (ASM) lds_waitcnt<N>();
}
template <bool ASM>
__device__ __forceinline__ void ldst(float4v& r) {
  if constexpr (ASM) lds_tie(r);
}

}  // namespace


// SINGLE: one LDS stage of 40 KiB raw + 32 KiB U (72 KiB) instead of two of
// 40 + 32 KiB, so TWO 4-wave blocks share a CU: each block's DMA wait,
// transform and epilogue (its output stores are 64 KiB) then overlap the other
// block's MFMAs -- with one 144-KiB block per CU they cannot (ablation:
// setup + epilogue alone took 16 % of the layer1 conv).
template <int NW, bool HAS_RES, bool PAIR, bool SINGLE = false, bool ABL = false>
__global__ void __launch_bounds__(64 * NW, SINGLE ? 2 : 1) conv_wino_f32_kernel(const WinoArgs a) {
  constexpr int T = 16 * NW;
  // single stage: no LDS-DMA is in flight while the chunk's LDS reads run, so
  // they are ordinary (compiler-scheduled, counted-wait) loads; with the
  // double-buffered ring they go through inline asm (common.h)
  constexpr bool ASMRD = !SINGLE;
  constexpr int RAWB = SINGLE ? kRaw3 : kRawMax;      // raw region bytes per stage
  constexpr int STG = RAWB + kUBytes;
  constexpr int RAW_INS = RAWB / 1024;                // DMA instructions (max) for the raw region
  constexpr int RAW_PER_WAVE = (RAW_INS + NW - 1) / NW;
  constexpr int U_PER_WAVE = (kUBytes / 1024) / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;                            // channel group of this lane (4 channels)

  // ---- block -> (tile block, output-channel block) ----------------------------
  const int nwg = a.nblk_t * a.nblk_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tb = lid / a.nblk_n, nb = lid - tb * a.nblk_n;
  const int n0 = nb * 32;
  const int rowb = 2 * a.NPP * 64;                    // bytes per staged image row
  int b0, ty0, imgs, rows;
  int t0 = 0, vr0 = 0, n_ins = a.raw_ins;             // LIN: first tile, first virtual row, DMA count
  const int per = a.TX * a.TY;
  if (a.LIN) {
    // virtual input rows: image b owns rows [b*RIN, (b+1)*RIN), row r = input row
    // r-1 (rows -1 and >= H are the zero padding), so the block's consecutive
    // tiles -- even across an image boundary -- read one contiguous row range
    t0 = tb * T;
    const int tl = min(t0 + T, a.B * per) - 1;
    const int bf = t0 / per, bl = tl / per;
    vr0 = bf * a.RIN + 2 * ((t0 - bf * per) / a.TX);
    const int vr_end = bl * a.RIN + 2 * ((tl - bl * per) / a.TX) + 4;
    n_ins = ((vr_end - vr0) * rowb + 1023) >> 10;
    b0 = ty0 = 0;
    imgs = rows = 0;
  } else if (a.IMG > 1) {
    b0 = tb * a.IMG;
    ty0 = 0;
    imgs = min(a.IMG, a.B - b0);
    rows = a.TY;
  } else {
    b0 = tb / a.bpi;
    ty0 = (tb - b0 * a.bpi) * a.R;
    imgs = 1;
    rows = min(a.R, a.TY - ty0);
  }
  const int per_img = a.R * a.TX;                     // tile slots per image in the block

  // ---- DMA sources (per lane, per instruction; + channel offset per stage) -----
  const float* zero = reinterpret_cast<const float*>(a.zero);
  int raw_off[RAW_PER_WAVE];
#pragma unroll
  for (int j = 0; j < RAW_PER_WAVE; ++j) {
    const int ins = wave + NW * j;
    const int L = ins * 64 + lane;
    raw_off[j] = -1;
    if (ins < n_ins) {
      const int qs = L & 3;
      int rest = L >> 2;
      const int pos = rest % a.NPP;                  // LDS pixel position in the half row
      rest /= a.NPP;
      const int half = rest & 1;
      const int lr = rest >> 1;
      // row rotation: staged row lr holds pixel p at position (p + f(lr)) mod NPP
      const int p = (pos + a.NPP - ((lr >> 1) * a.RMUL) % a.NPP) % a.NPP;
      const int ix = 2 * p + half - 1;
      const int q = qs ^ raw_swz(pos);
      int img, iy;
      if (p >= a.NP) {
        img = a.B;                                   // padding position of a rotated row
        iy = 0;
      } else if (a.LIN) {
        const int vr = vr0 + lr;
        img = vr / a.RIN;
        iy = vr - img * a.RIN - 1;
      } else {
        img = lr / a.RIN;
        iy = 2 * ty0 + (lr - img * a.RIN) - 1;
        img = img < imgs ? b0 + img : a.B;
      }
      if (img < a.B && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
        raw_off[j] = ((img * a.H + iy) * a.W + ix) * a.C + 4 * q;
    }
  }
  int u_off[U_PER_WAVE];
#pragma unroll
  for (int j = 0; j < U_PER_WAVE; ++j) {
    const int ins = wave + NW * j;
    const int row = ins * 16 + (lane >> 2);            // (e, n) row of 64 B
    const int e = row >> 5, n = row & 31;
    const int q = (lane & 3) ^ swz_r(n, 4);
    u_off[j] = (e * a.Cout + n0 + n) * a.C + 4 * q;
  }
  const int nk = a.C / 16;
  auto issue = [&](int k, int buf) {
    char* base = smem + buf * STG;
    const int c0 = k * 16;
#pragma unroll
    for (int j = 0; j < RAW_PER_WAVE; ++j) {
      const int ins = wave + NW * j;
      if (ins < n_ins) {
        const float* src = raw_off[j] >= 0 ? a.x + raw_off[j] + c0 : zero;
        __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + ins * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < U_PER_WAVE; ++j) {
      const int ins = wave + NW * j;
      __builtin_amdgcn_global_load_lds((glb_void_t*)(a.u + u_off[j] + c0),
                                       (lds_void_t*)(base + RAWB + ins * 1024), 16, 0, 0);
    }
  };

  // ---- this lane's tile and its patch addresses in the raw image --------------
  // (s_b, s_ty, s_tx): image, tile row, tile column; byte offset of patch element
  // (py, px): staged row (s_row + py), parity px&1, pixel tx + (px>>1), chunk g ^ swz(pixel)
  const int slot = wave * 16 + (lane & 15);
  int s_b, s_ty, s_tx, s_row;
  bool s_ok;
  if (a.LIN) {
    const int t = t0 + slot;
    s_ok = t < a.B * per;
    s_b = t / per;
    const int rem = t - s_b * per;
    s_ty = rem / a.TX;
    s_tx = rem - s_ty * a.TX;
    s_row = s_b * a.RIN + 2 * s_ty - vr0;
  } else {
    const int s_img = slot / per_img, s_rem = slot - s_img * per_img;
    const int s_tyl = s_rem / a.TX;
    s_tx = s_rem - s_tyl * a.TX;
    s_ok = slot < T && s_img < imgs && s_tyl < rows;
    s_b = b0 + s_img;
    s_ty = ty0 + s_tyl;
    s_row = s_img * a.RIN + 2 * s_tyl;
  }
  const int pbase = s_ok ? s_row * rowb : 0;
  // patch rows 0-1 and 2-3 sit in staged row pairs s_row/2 and s_row/2 + 1,
  // each rotated by its own f = (pair * RMUL) mod NPP: with RMUL = TX, the
  // lanes of one ds_read_b128 group (consecutive tiles, possibly across tile
  // rows) read pixels at consecutive positions mod 8 -> distinct bank slots
  int colb[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = (((s_row >> 1) + h) * a.RMUL) % a.NPP;
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const int pos = s_ok ? (s_tx + (px >> 1) + f) % a.NPP : 0;
      colb[h][px] = (px & 1) * a.NPP * 64 + pos * 64 + ((g ^ raw_swz(pos)) << 4);
    }
  }

  float4v acc[16][2];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    acc[e][0] = float4v{0.f, 0.f, 0.f, 0.f};
    acc[e][1] = float4v{0.f, 0.f, 0.f, 0.f};
  }

  const int abl = ABL ? a.ablate : 0;   // compiled out in production instances
  if (!(ABL && (abl & 1))) issue(0, 0);
  const int nk_run = (ABL && (abl & 16)) ? 0 : nk;            // 16: setup + epilogue only
  for (int k = 0; k < nk_run; ++k) {
    if constexpr (SINGLE) {
      if (k > 0) {
        __syncthreads();                                // every wave done reading chunk k-1
        if (!(ABL && (abl & 1))) issue(k, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of chunk k landed
    // everyone's landed; (double) buffer k+1 free.  Single stage: a full
    // __syncthreads (memory fence) -- its LDS reads are compiler-visible loads
    // that must not move above it; the ring keeps the raw s_barrier
    if constexpr (SINGLE) __syncthreads();
    else __builtin_amdgcn_s_barrier();
    if constexpr (!SINGLE) {
      if (k + 1 < nk && !(ABL && (abl & 1))) issue(k + 1, (k + 1) & 1);
    }
    const uint32_t sb = lds_addr(smem) + (SINGLE ? 0 : (k & 1)) * STG;

    // raw 4x4 patch of this lane's tile, its 4 channels -> V = B^T d B
    float4v d[4][4];
    if (ABL && (abl & 2)) {
#pragma unroll
      for (int py = 0; py < 4; ++py)
#pragma unroll
        for (int px = 0; px < 4; ++px) d[py][px] = float4v{1.f, 2.f, 3.f, (float)(py * 4 + px + k)};
    } else {
#pragma unroll
      for (int py = 0; py < 4; ++py)
#pragma unroll
        for (int px = 0; px < 4; ++px) d[py][px] = ldsr<ASMRD>(sb + pbase + py * rowb + colb[py >> 1][px]);
    }
    lds_wait<ASMRD, 0>();
#pragma unroll
    for (int py = 0; py < 4; ++py)
#pragma unroll
      for (int px = 0; px < 4; ++px) ldst<ASMRD>(d[py][px]);
    // V = B^T d B one row i at a time, just ahead of that row's 4 e-GEMMs: the
    // transform of row i+1 runs while row i's MFMAs are in flight, and only 4
    // V registers (not 16) are live next to the raw patch
    auto vrow = [&](int i, float4v (&v)[4]) {
      float4v t[4];
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        if (i == 0) t[px] = d[0][px] - d[2][px];
        else if (i == 1) t[px] = d[1][px] + d[2][px];
        else if (i == 2) t[px] = d[2][px] - d[1][px];
        else t[px] = d[1][px] - d[3][px];
      }
      v[0] = t[0] - t[2];
      v[1] = t[1] + t[2];
      v[2] = t[2] - t[1];
      v[3] = t[1] - t[3];
    };

    // 16 GEMM updates: M_e[32 couts][16 tiles] += U_e[32][16 ch] * V_e[16 ch][16 tiles]
    const uint32_t ub = sb + RAWB;
    auto uaddr = [&](int e, int i) {
      const int n = i * 16 + (lane & 15);
      return ub + (e * 32 + n) * 64 + ((g ^ swz_r(n, 4)) << 4);
    };
    if constexpr (PAIR) {
    // e is processed in PAIRS: the 4 MFMAs of one k-step t then cycle over 4
    // independent accumulators (e, e+1) x (cout half 0, 1), so a dependent
    // v_mfma_f32_16x16x4_f32 (40-cycle result latency, 32-cycle issue) never
    // waits on its predecessor (one e at a time alternated between only 2
    // accumulators: "MFMA-only" ablation ran at ~60 % of the issue rate).
    // U fragments of a pair: double-buffered (read pair p+1 while p multiplies)
    // at one wave per SIMD; single-buffered at two (the partner wave covers the
    // LDS latency, and the 8-wave kernel stays inside 256 registers).
    constexpr bool UDB = NW <= 4 && !SINGLE;
    float4v ua[UDB ? 2 : 1][2][2];                      // [buffer][e of pair][cout half]
    auto read_pair = [&](int p, int buf) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ua[buf][q][0] = ldsr<ASMRD>(uaddr(2 * p + q, 0));
        ua[buf][q][1] = ldsr<ASMRD>(uaddr(2 * p + q, 1));
      }
    };
    if constexpr (UDB) {
      if (!(ABL && (abl & 4))) read_pair(0, 0);
    }
    float4v vr[4];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int cb = UDB ? (p & 1) : 0;
      if ((p & 1) == 0) vrow(p >> 1, vr);
      if (ABL && (abl & 4)) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          ua[cb][q][0] = float4v{1.f, 2.f, (float)p, (float)k};
          ua[cb][q][1] = float4v{2.f, 1.f, (float)k, (float)q};
        }
      } else if constexpr (UDB) {
        if (p + 1 < 8) {
          read_pair(p + 1, cb ^ 1);
          lds_wait<ASMRD, 4>();
        } else {
          lds_wait<ASMRD, 0>();
        }
      } else {
        read_pair(p, 0);
        lds_wait<ASMRD, 0>();
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ldst<ASMRD>(ua[cb][q][0]);
        ldst<ASMRD>(ua[cb][q][1]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int e = 2 * p + q;
          acc[e][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][q][0][t], vr[e & 3][t], acc[e][0], 0, 0, 0);
          acc[e][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][q][1][t], vr[e & 3][t], acc[e][1], 0, 0, 0);
        }
    }
    } else {
    // read -> wait -> use (no register double buffer: a value an inline-asm
    // ds_read defines before its wait may be copied by the register allocator
    // ahead of the wait; with a read-ahead buffer variant 0 returned garbage)
    constexpr bool UDB = false;
    float4v ua[UDB ? 2 : 1][2];
    if constexpr (UDB) {
      if (!(ABL && (abl & 4))) {
        ua[0][0] = ldsr<ASMRD>(uaddr(0, 0));
        ua[0][1] = ldsr<ASMRD>(uaddr(0, 1));
      }
    }
    float4v vr[4];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int cb = UDB ? (e & 1) : 0, nbf = UDB ? (cb ^ 1) : 0;
      if ((e & 3) == 0) vrow(e >> 2, vr);
      if (ABL && (abl & 4)) {
        ua[cb][0] = float4v{1.f, 2.f, (float)e, (float)k};
        ua[cb][1] = float4v{2.f, 1.f, (float)k, (float)e};
      } else if constexpr (UDB) {
        if (e + 1 < 16) {
          ua[nbf][0] = ldsr<ASMRD>(uaddr(e + 1, 0));
          ua[nbf][1] = ldsr<ASMRD>(uaddr(e + 1, 1));
          lds_wait<ASMRD, 2>();
        } else {
          lds_wait<ASMRD, 0>();
        }
      } else {
        ua[0][0] = ldsr<ASMRD>(uaddr(e, 0));
        ua[0][1] = ldsr<ASMRD>(uaddr(e, 1));
        lds_wait<ASMRD, 0>();
      }
      ldst<ASMRD>(ua[cb][0]);
      ldst<ASMRD>(ua[cb][1]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        acc[e][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][0][t], vr[e & 3][t], acc[e][0], 0, 0, 0);
        acc[e][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][1][t], vr[e & 3][t], acc[e][1], 0, 0, 0);
      }
    }
    }
  }

  // ---- output transform Y = A^T M A, bias, residual, ReLU, NHWC store -----------
  if (!s_ok) return;
  const int b = s_b;
  const int oy0 = 2 * s_ty, ox0 = 2 * s_tx;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = n0 + i * 16 + 4 * g;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
    // per output channel r (vector lane of the float4 accumulators)
    float4v y00, y01, y10, y11;
    {
      float4v m[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) m[e] = acc[e][i];
      float4v t0[4], t1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        t0[j] = m[0 * 4 + j] + m[1 * 4 + j] + m[2 * 4 + j];
        t1[j] = m[1 * 4 + j] - m[2 * 4 + j] - m[3 * 4 + j];
      }
      y00 = t0[0] + t0[1] + t0[2];
      y01 = t0[1] - t0[2] - t0[3];
      y10 = t1[0] + t1[1] + t1[2];
      y11 = t1[1] - t1[2] - t1[3];
    }
    float4v yy[4] = {y00, y01, y10, y11};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oy = oy0 + (q >> 1), ox = ox0 + (q & 1);
      if (oy >= a.H || ox >= a.W) continue;
      const size_t off = (((size_t)b * a.H + oy) * a.W + ox) * a.Cout + n;
      float4v o = yy[q] + bv;
      if constexpr (HAS_RES) o += *reinterpret_cast<const float4v*>(a.res + off);
      if (a.relu) {
        o[0] = fmaxf(o[0], 0.f);
        o[1] = fmaxf(o[1], 0.f);
        o[2] = fmaxf(o[2], 0.f);
        o[3] = fmaxf(o[3], 0.f);
      }
      if (ABL && (a.ablate & 8)) {
        if (o[0] == 12345.f) a.y[0] = o[1];
        continue;
      }
      *reinterpret_cast<float4v*>(a.y + off) = o;
    }
  }
}


// ---------------------------------------------------------------------------
// v2: software-pipelined, 4 waves (one per SIMD, up to 512 registers each).
// v1's waves all hit the barrier together, so every SIMD idles its matrix pipe
// while the raw patch is read and transformed (and one wave per SIMD has no
// partner to cover it).  v2 keeps the raw input one chunk AHEAD of U in two
// separate rings: at chunk k the wave multiplies V(k) (registers) by U(k)
// while it reads raw(k+1) and transforms it into V(k+1) between the MFMAs.
//   LDS: raw ring 2 x 26 KiB + U ring 2 x 32 KiB = 116 KiB (one block per CU).
//   Before barrier k: raw(k+1) and U(k) landed (issued one chunk earlier);
//   after it: issue raw(k+2) into raw(k)'s slot and U(k+1) into U(k-1)'s slot.
// ---------------------------------------------------------------------------
constexpr int kRaw2 = 26 * 1024;

template <bool HAS_RES>
__global__ void __launch_bounds__(256, 1) conv_wino2_f32_kernel(const WinoArgs a) {
  constexpr int NW = 4, T = 64;
  constexpr int RAW_PER_WAVE = (kRaw2 / 1024 + NW - 1) / NW;
  constexpr int U_PER_WAVE = (kUBytes / 1024) / NW;
  constexpr int RAW0 = 0, U0 = 2 * kRaw2;                 // ring bases
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;

  const int nwg = a.nblk_t * a.nblk_n;
  const int lid = xcd_remap(blockIdx.x, nwg);
  const int tb = lid / a.nblk_n, nb = lid - tb * a.nblk_n;
  const int n0 = nb * 32;
  int b0, ty0, imgs, rows;
  if (a.IMG > 1) {
    b0 = tb * a.IMG;
    ty0 = 0;
    imgs = min(a.IMG, a.B - b0);
    rows = a.TY;
  } else {
    b0 = tb / a.bpi;
    ty0 = (tb - b0 * a.bpi) * a.R;
    imgs = 1;
    rows = min(a.R, a.TY - ty0);
  }
  const int per_img = a.R * a.TX;

  const float* zero = reinterpret_cast<const float*>(a.zero);
  int raw_off[RAW_PER_WAVE];
#pragma unroll
  for (int j = 0; j < RAW_PER_WAVE; ++j) {
    const int ins = wave + NW * j;
    const int L = ins * 64 + lane;
    raw_off[j] = -1;
    if (ins < a.raw_ins) {
      const int qs = L & 3;
      int rest = L >> 2;
      const int p = rest % a.NP;
      rest /= a.NP;
      const int half = rest & 1;
      const int lr = rest >> 1;
      const int img = lr / a.RIN, rin = lr - img * a.RIN;
      const int iy = 2 * ty0 + rin - 1, ix = 2 * p + half - 1;
      const int q = qs ^ raw_swz(p);
      if (img < imgs && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
        raw_off[j] = (((b0 + img) * a.H + iy) * a.W + ix) * a.C + 4 * q;
    }
  }
  int u_off[U_PER_WAVE];
#pragma unroll
  for (int j = 0; j < U_PER_WAVE; ++j) {
    const int ins = wave + NW * j;
    const int row = ins * 16 + (lane >> 2);
    const int e = row >> 5, n = row & 31;
    const int q = (lane & 3) ^ swz_r(n, 4);
    u_off[j] = (e * a.Cout + n0 + n) * a.C + 4 * q;
  }
  const int nk = a.C / 16;
  auto issue_raw = [&](int k) {
    char* base = smem + RAW0 + (k & 1) * kRaw2;
    const int c0 = k * 16;
#pragma unroll
    for (int j = 0; j < RAW_PER_WAVE; ++j) {
      const int ins = wave + NW * j;
      if (ins < a.raw_ins) {
        const float* src = raw_off[j] >= 0 ? a.x + raw_off[j] + c0 : zero;
        __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)(base + ins * 1024), 16, 0, 0);
      }
    }
  };
  auto issue_u = [&](int k) {
    char* base = smem + U0 + (k & 1) * kUBytes;
    const int c0 = k * 16;
#pragma unroll
    for (int j = 0; j < U_PER_WAVE; ++j) {
      const int ins = wave + NW * j;
      __builtin_amdgcn_global_load_lds((glb_void_t*)(a.u + u_off[j] + c0), (lds_void_t*)(base + ins * 1024), 16, 0,
                                       0);
    }
  };

  const int slot = wave * 16 + (lane & 15);
  const int s_img = slot / per_img, s_rem = slot - s_img * per_img;
  const int s_tyl = s_rem / a.TX, s_tx = s_rem - s_tyl * a.TX;
  const bool s_ok = slot < T && s_img < imgs && s_tyl < rows;
  const int rowb = 2 * a.NP * 64;
  const int pbase = s_ok ? ((s_img * a.RIN + 2 * s_tyl) * rowb) : 0;
  int colb[4];
#pragma unroll
  for (int px = 0; px < 4; ++px) {
    const int p = s_ok ? s_tx + (px >> 1) : 0;
    colb[px] = (px & 1) * a.NP * 64 + p * 64 + ((g ^ raw_swz(p)) << 4);
  }
  const uint32_t sbase = lds_addr(smem);
  auto read_raw = [&](int k, float4v (&d)[4][4]) {
    const uint32_t rb = sbase + RAW0 + (k & 1) * kRaw2 + pbase;
#pragma unroll
    for (int py = 0; py < 4; ++py)
#pragma unroll
      for (int px = 0; px < 4; ++px) d[py][px] = lds_read_f4(rb + py * rowb + colb[px]);
  };
  // V = B^T d B in two halves: rows (d -> B^T d, in place) then columns
  auto transform_rows = [&](float4v (&d)[4][4], int px) {
    const float4v t0 = d[0][px] - d[2][px], t1 = d[1][px] + d[2][px];
    const float4v t2 = d[2][px] - d[1][px], t3 = d[1][px] - d[3][px];
    d[0][px] = t0;
    d[1][px] = t1;
    d[2][px] = t2;
    d[3][px] = t3;
  };
  auto transform_cols = [&](float4v (&d)[4][4], float4v (&v)[16], int i) {
    v[i * 4 + 0] = d[i][0] - d[i][2];
    v[i * 4 + 1] = d[i][1] + d[i][2];
    v[i * 4 + 2] = d[i][2] - d[i][1];
    v[i * 4 + 3] = d[i][1] - d[i][3];
  };
  auto uaddr = [&](int k, int e, int i) {
    const int n = i * 16 + (lane & 15);
    return sbase + U0 + (k & 1) * kUBytes + (e * 32 + n) * 64 + ((g ^ swz_r(n, 4)) << 4);
  };

  float4v acc[16][2];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    acc[e][0] = float4v{0.f, 0.f, 0.f, 0.f};
    acc[e][1] = float4v{0.f, 0.f, 0.f, 0.f};
  }

  // prologue: raw(0), U(0), raw(1) in flight; V(0) transformed up front
  float4v va[16], vb[16];
  {
    issue_raw(0);
    issue_u(0);
    if (nk > 1) issue_raw(1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    float4v d[4][4];
    read_raw(0, d);
    lds_waitcnt<0>();
#pragma unroll
    for (int py = 0; py < 4; ++py)
#pragma unroll
      for (int px = 0; px < 4; ++px) lds_tie(d[py][px]);
#pragma unroll
    for (int px = 0; px < 4; ++px) transform_rows(d, px);
#pragma unroll
    for (int i = 0; i < 4; ++i) transform_cols(d, va, i);
  }

  // one chunk: MFMAs of V(k) x U(k); raw(k+1) -> V(k+1) between them
  auto chunk = [&](int k, float4v (&vc)[16], float4v (&vn)[16]) {
    __builtin_amdgcn_s_barrier();          // all waves done with chunk k-1 (raw(k) and U(k-1) slots free)
    if (k + 2 < nk) issue_raw(k + 2);
    if (k + 1 < nk) issue_u(k + 1);
    const bool more = k + 1 < nk;
    float4v d[4][4];
    if (more) read_raw(k + 1, d);
    // e in pairs: 4 independent accumulators per k-step (see the v1 kernel)
    float4v ua[2][2][2];                                // [buffer][e of pair][cout half]
    auto read_pair = [&](int p, int buf) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ua[buf][q][0] = lds_read_f4(uaddr(k, 2 * p + q, 0));
        ua[buf][q][1] = lds_read_f4(uaddr(k, 2 * p + q, 1));
      }
    };
    read_pair(0, 0);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int cb = p & 1;
      if (p + 1 < 8) {
        read_pair(p + 1, cb ^ 1);
        lds_waitcnt<4>();                  // in-order: raw(k+1) reads and pair p retired
      } else {
        lds_waitcnt<0>();
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        lds_tie(ua[cb][q][0]);
        lds_tie(ua[cb][q][1]);
      }
      if (p == 0 && more) {
#pragma unroll
        for (int py = 0; py < 4; ++py)
#pragma unroll
          for (int px = 0; px < 4; ++px) lds_tie(d[py][px]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int e = 2 * p + q;
          acc[e][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][q][0][t], vc[e][t], acc[e][0], 0, 0, 0);
          acc[e][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cb][q][1][t], vc[e][t], acc[e][1], 0, 0, 0);
        }
      // spread the next chunk's transform over the MFMA stream (16 MFMAs per pair)
      if (more) {
        if (p >= 1 && p <= 4) transform_rows(d, p - 1);
        if (p >= 4 && p <= 7) transform_cols(d, vn, p - 4);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // raw(k+2), U(k+1) of this wave landed
  };
  int k = 0;
  for (; k + 1 < nk; k += 2) {
    chunk(k, va, vb);
    chunk(k + 1, vb, va);
  }
  if (k < nk) chunk(k, va, vb);

  // ---- output transform Y = A^T M A, bias, residual, ReLU, NHWC store -----------
  if (!s_ok) return;
  const int b = b0 + s_img;
  const int oy0 = 2 * (ty0 + s_tyl), ox0 = 2 * s_tx;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = n0 + i * 16 + 4 * g;
    const float4v bv = *reinterpret_cast<const float4v*>(a.bias + n);
    float4v t0[4], t1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      t0[j] = acc[0 * 4 + j][i] + acc[1 * 4 + j][i] + acc[2 * 4 + j][i];
      t1[j] = acc[1 * 4 + j][i] - acc[2 * 4 + j][i] - acc[3 * 4 + j][i];
    }
    const float4v yy[4] = {t0[0] + t0[1] + t0[2], t0[1] - t0[2] - t0[3], t1[0] + t1[1] + t1[2],
                           t1[1] - t1[2] - t1[3]};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oy = oy0 + (q >> 1), ox = ox0 + (q & 1);
      if (oy >= a.H || ox >= a.W) continue;
      const size_t off = (((size_t)b * a.H + oy) * a.W + ox) * a.Cout + n;
      float4v o = yy[q] + bv;
      if constexpr (HAS_RES) o += *reinterpret_cast<const float4v*>(a.res + off);
      if (a.relu) {
        o[0] = fmaxf(o[0], 0.f);
        o[1] = fmaxf(o[1], 0.f);
        o[2] = fmaxf(o[2], 0.f);
        o[3] = fmaxf(o[3], 0.f);
      }
      *reinterpret_cast<float4v*>(a.y + off) = o;
    }
  }
}

// Host-side block geometry for T = 16*nw tiles per block; false if the shape
// does not fit (caller falls back to the direct conv).  ``lin``: use the
// consecutive-tile (LIN) blocking when the rectangular one leaves tile slots
// idle and every block's virtual-row range fits ``raw_max``.  ``rot``: rotate
// the staged rows (pixel positions padded to a multiple of 8 per half row) so
// the patch reads of lanes whose tiles lie in different tile rows hit distinct
// LDS banks; dropped when the padded rows do not fit.
static bool wino_geometry_np(WinoArgs& a, int nw, int raw_max, bool lin, int npp) {
  const int T = 16 * nw;
  a.TX = (a.W + 1) / 2;
  a.TY = (a.H + 1) / 2;
  a.LIN = 0;
  a.NP = a.TX + 1;
  a.NPP = npp;
  if (a.TX > T) return false;
  const int per = a.TX * a.TY;
  const int rowb = 2 * a.NPP * 64;
  auto raw_bytes = [&](int imgs, int R) { return imgs * (2 * R + 2) * rowb; };
  if (per <= T) {
    a.R = a.TY;
    a.IMG = T / per;
    while (a.IMG > 1 && raw_bytes(a.IMG, a.R) > raw_max) --a.IMG;
    if (a.IMG == 1) a.bpi = 1;
  } else {
    a.IMG = 1;
    a.R = T / a.TX;
    while (a.R > 1 && raw_bytes(1, a.R) > raw_max) --a.R;
    a.bpi = (a.TY + a.R - 1) / a.R;
  }
  if (raw_bytes(a.IMG, a.R) > raw_max) return false;
  a.RIN = 2 * a.R + 2;
  a.raw_ins = (raw_bytes(a.IMG, a.R) + 1023) / 1024;
  a.nblk_t = a.IMG > 1 ? (a.B + a.IMG - 1) / a.IMG : a.B * a.bpi;
  a.nblk_n = a.Cout / 32;
  const long used = (long)a.B * per;
  if (lin && used * 100 < (long)a.nblk_t * T * 95) {
    // every block's staged rows (the kernel's own formula); periodic in the
    // block index with period lcm(T, per) / T <= per blocks
    const int rin = 2 * a.TY + 2;
    const long nblk = (used + T - 1) / T;
    int worst = 0;
    for (long tb = 0; tb < nblk && tb <= per; ++tb) {
      const long t0 = tb * T, tl = std::min(t0 + T, used) - 1;
      const long bf = t0 / per, bl = tl / per;
      const long v0 = bf * rin + 2 * ((t0 - bf * per) / a.TX);
      const long v1 = bl * rin + 2 * ((tl - bl * per) / a.TX) + 4;
      worst = std::max(worst, (int)(v1 - v0) * rowb);
    }
    if (worst <= raw_max) {
      a.LIN = 1;
      a.RIN = rin;
      a.raw_ins = (worst + 1023) / 1024;
      a.nblk_t = (int)nblk;
    }
  }
  return true;
}

static bool wino_geometry(WinoArgs& a, int nw, int raw_max = kRawMax, bool lin = false, bool rot = false) {
  a.RMUL = 0;
  if (rot) {
    WinoArgs r = a;
    const int npp = (a.W + 1) / 2 + 1;
    if (wino_geometry_np(r, nw, raw_max, lin, (npp + 7) / 8 * 8)) {
      // keep the rotation only if it costs no tile slots
      WinoArgs p = a;
      wino_geometry_np(p, nw, raw_max, lin, npp);
      if (r.nblk_t <= p.nblk_t) {
        a = r;
        a.RMUL = a.TX;
        return true;
      }
    }
  }
  return wino_geometry_np(a, nw, raw_max, lin, (a.W + 1) / 2 + 1);
}

bool conv_wino_f32_supported(int H, int W, int C, int Cout) {
  WinoArgs a{};
  a.B = 1; a.H = H; a.W = W; a.C = C; a.Cout = Cout;
  return C % 16 == 0 && Cout % 32 == 0 && wino_geometry(a, 4, kRaw2);
}

// Variant 3 uses LIN blocking (consecutive tiles, virtual rows: 40.3k vs 39.4k img/s,
// profiles/r2_v8_wino_linear_40k.md) without rotated raw rows (the rotation removed the
// simulated 2-way raw-read bank conflicts but measured 0.99-1.02x, profiles/r2_v11_wino_rotation.md);
// e-GEMMs in pairs measured 4w -4 %, 8w +13 % time.  Those A/B switches were folded in round 5.
template <int NW, bool R>
static void wino_cfg(WinoArgs a, hipStream_t st) {
  const int lds = 2 * kStage;
  auto kern = conv_wino_f32_kernel<NW, R, false>;
  ensure_lds_attr(reinterpret_cast<const void*>(kern), lds);
  hipLaunchKernelGGL(kern, dim3(a.nblk_t * a.nblk_n), dim3(64 * NW), lds, st, a);
}

// variant: 0 = 4 waves (64 tiles per block), 1 = 8 waves (128 tiles per block),
//          2 = software-pipelined 4 waves (64 tiles per block),
//          3 = 4 waves, one 58-KiB stage, two blocks per CU
bool conv_wino_f32_launch(WinoArgs a, int variant, hipStream_t st) {
  if (variant == 3) {
    if (a.C % 16 || a.Cout % 32 || !wino_geometry(a, 4, kRaw3, true, false)) return false;
    const int lds = kRaw3 + kUBytes;
    const bool r = a.res != nullptr;
    auto kern = r ? conv_wino_f32_kernel<4, true, false, true> : conv_wino_f32_kernel<4, false, false, true>;
    ensure_lds_attr(reinterpret_cast<const void*>(kern), lds);
    hipLaunchKernelGGL(kern, dim3(a.nblk_t * a.nblk_n), dim3(256), lds, st, a);
    return true;
  }
  if (variant == 2) {
    if (a.C % 16 || a.Cout % 32 || !wino_geometry(a, 4, kRaw2)) return false;
    const int lds = 2 * kRaw2 + 2 * kUBytes;
    auto kern = a.res != nullptr ? conv_wino2_f32_kernel<true> : conv_wino2_f32_kernel<false>;
    ensure_lds_attr(reinterpret_cast<const void*>(kern), lds);
    hipLaunchKernelGGL(kern, dim3(a.nblk_t * a.nblk_n), dim3(256), lds, st, a);
    return true;
  }
  const int nw = variant == 1 ? 8 : 4;
  if (a.C % 16 || a.Cout % 32 || !wino_geometry(a, nw)) return false;
  const bool res = a.res != nullptr;
  if (nw == 8) {
    if (res) wino_cfg<8, true>(a, st);
    else wino_cfg<8, false>(a, st);
  } else {
    if (res) wino_cfg<4, true>(a, st);
    else wino_cfg<4, false>(a, st);
  }
  return true;
}

}  // namespace idunno
