// Host-visible launch entry points of the HIP kernels (one definition of the
// argument structs shared by the kernel TUs and the Python bindings).
#pragma once
#include "common.h"

namespace idunno {

struct ConvArgs {
  const half_t* x;     // NHWC [B][H][W][C]
  const half_t* w;     // [Cout][Kpad]
  const float* bias;   // [Cout]
  const half_t* res;   // NHWC [B][Ho][Wo][Cout] or nullptr
  void* y;             // NHWC [B][Ho][Wo][ldy]  (fp16 or fp32)
  int B, H, W, C;
  int Ho, Wo, Cout, ldy;
  int KH, KW, stride, pad;
  int M;        // B*Ho*Wo
  int nK;       // number of K stages
  int cblk;     // BIG: C / BK
  int nsub;     // SMALL: stages per kh row
  int Kpad;     // row length of w
  int relu;
  int tiles_n;  // ceil(Cout / BN)
  int tiles_m;  // ceil(M / BM)
  const void* zero;  // >= 16 zero bytes (DMA source for padding taps)
  int ldx;           // conv_glds: input pixel stride in halfs (0: C); a K-slice of a wider row
  int nc, wp, cpk;   // conv_glds pack3 (RGB stems on packed rows, preprocess_pack3_f16): row copies,
                     // halfs per copy row, 16-byte chunks per kernel row (ceil(3*KW/8)); cpk = 0: off
  int ksplit;        // conv_glds split-K in ONE launch (FC layers, fp32 partials): block s / tiles takes
  int kslice;        // K slice s: x and w advance by s*kslice halfs, y by s*ysplit floats; 0/1: off
  long ysplit;
  float acc_scale;   // conv_glds SPLIT: accumulator multiplier (2^-e of the pre-scaled split weights)
  int* ovf;          // conv_glds SPLIT: split range guard flag (common.h split_guard) or nullptr
  // conv_glds SPLIT dual conv (two convs of one input in one launch, outputs side
  // by side in y): output channels >= nsplit_n are the second conv -- its own
  // accumulator scale acc_scale2, no ReLU, and with center_only its K loop runs
  // over the centre tap only (a 1x1/s stride-s conv is the centre tap of the
  // 3x3/s pad-1 conv on the same input: ResNet downsample + first 3x3)
  int nsplit_n;
  int center_only;
  float acc_scale2;
  int ldr;           // residual pixel stride in halfs (0: the output width, 2*Cout split / Cout fp16)
  int kstage;        // conv split-K (small M): block s / tiles runs K stages [s*kstage, (s+1)*kstage) of the
                     // (kh, kw, cblk) loop into fp32 partials y + s*ysplit (kslice 0); 0: off
};

// fp32 (reference-precision) conv: same geometry fields as ConvArgs, f32 tensors.
struct ConvF32Args {
  const float* x;      // NHWC [B][H][W][C]  (C == 4: RGB+0 stem input)
  const float* w;      // [Cout][Kpad]: big (kh, kw, c); small (kh, tap(nsub*4), c4)
  const float* bias;   // [Cout]
  const float* res;    // NHWC [B][Ho][Wo][Cout] or nullptr
  float* y;            // NHWC [B][Ho][Wo][ldy]
  int B, H, W, C;
  int Ho, Wo, Cout, ldy;
  int KH, KW, stride, pad;
  int M;               // B*Ho*Wo
  int nK;              // K stages (set by the launcher)
  int cblk;            // big: C / BK; small: tap blocks per kh row (set by the launcher)
  int nsub;            // small: ceil(KW / 4)
  int Kpad;
  int relu;
  int tiles_n, tiles_m;
  const void* zero;    // >= 16 zero bytes
  int ldx;             // input pixel stride in floats (0: C)
  // packed-row stem input (mode 2, preprocess_pack3_f32): x = [B][H][nc][wp]
  int nc, wp, cpk;     // row copies, floats per copy row, 16-byte chunks per kh row (ceil(3*KW/4))
  // split-K in ONE launch (big-C 1x1 only, FC layers): block s / (tiles) takes
  // K slice s: x and w advance by s*kslice floats, y by s*ysplit (fp32 partials)
  int ksplit;          // 0/1: off
  int kslice;
  long ysplit;
};

// mode: 0 big-C (kh, kw, c), 1 small-C NHWC4 stems, 2 packed-row RGB stems
bool conv_f32_launch(ConvF32Args a, int mode, int tile, hipStream_t st);   // false: unknown tile id

// fp32 Winograd F(2x2,3x3) conv (3x3, stride 1, pad 1), conv_wino_f32.hip.
struct WinoArgs {
  const float* x;      // NHWC [B][H][W][C]
  const float* u;      // [16][Cout][C]: U = G g G^T per (e, cout, cin)
  const float* bias;   // [Cout]
  const float* res;    // NHWC [B][H][W][Cout] or nullptr
  float* y;            // NHWC [B][H][W][Cout]
  const void* zero;    // >= 16 zero bytes
  int B, H, W, C, Cout;
  int relu;
  // block geometry (set by the launcher)
  int TX, TY;          // 2x2 tiles per row / column
  int IMG, R, bpi;     // images per block, tile rows per block, blocks per image
  int RIN, NP;         // staged input rows per image, pixels per column-parity half row
  int NPP, RMUL;       // pixel positions per staged half row (>= NP) and the row rotation
                       // multiplier: row r holds pixel p at ((r/2)*RMUL + p) mod NPP
  int raw_ins;         // 1 KiB DMA instructions of the staged input region (max over blocks)
  int LIN;             // 1: a block takes 16*NW CONSECUTIVE tiles of the flattened (image,
                       // tile row, tile column) order, staging virtual rows (RIN = 2*TY+2 per
                       // image, pad rows included) -- no idle tile slots (variant 3 only)
  int nblk_t, nblk_n;  // tile blocks, 32-channel output blocks
  int ablate;          // profiling only (set_wino_ablation): 1 no DMA, 2 no raw read/transform,
                       // 4 no U reads, 8 no epilogue stores -- outputs are wrong
};
bool conv_wino_f32_launch(WinoArgs a, int variant, hipStream_t st);   // false: shape unsupported
bool conv_wino_f32_supported(int H, int W, int C, int Cout);
int conv_f32_pick(int M, int Cout, int K, bool small);
// uint8 HWC -> packed-row fp32 stem input [B][H][nc][wp] (conv mode 2): copy c of
// row y is the normalised row (3 floats per pixel, `pad` zero pixels first) shifted
// left by c * (4 / nc) floats
void preprocess_pack3_f32_launch(const uint8_t* img, float* out, int B, int H, int W, int pad, int nc, int wp,
                                 const long long* start_idx, long long start_off, long long max_start,
                                 long long sub, hipStream_t st);
void preprocess_pack3_f16_launch(const uint8_t* img, half_t* out, int B, int H, int W, int pad, int nc, int wp,
                                 const long long* start_idx, long long start_off, long long max_start,
                                 long long sub, hipStream_t st);
// split-fp16 packed rows [B][H][2][nc][wp] (plane 0 hi, plane 1 lo) for conv_glds P3+SPLIT
void preprocess_pack3_split_launch(const uint8_t* img, half_t* out, int B, int H, int W, int pad, int nc, int wp,
                                   const long long* start_idx, long long start_off, long long max_start,
                                   long long sub, hipStream_t st);
void preprocess_f32_launch(const uint8_t* img, float* out, long npix, const long long* start_idx,
                           long long start_off, long long max_start, long long sub, long pix_per_img,
                           hipStream_t st);
void maxpool_f32_launch(const float* x, float* y, int B, int H, int W, int C, int Ho, int Wo, int k, int s,
                        int pad, hipStream_t st);
void avgpool_f32_launch(const float* x, float* y, int B, int HW, int C, hipStream_t st);
// split-fp16 layout conversions and pooling (elementwise_split.hip)
void split_from_f32_launch(const float* x, half_t* y, long npix, int C, int* ovf, hipStream_t st);
void f32_from_split_launch(const half_t* x, float* y, long npix, int C, hipStream_t st);
void maxpool_split_launch(const void* x, bool in_split, half_t* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                          int s, int pad, int* ovf, hipStream_t st);

void conv_igemm_launch(ConvArgs a, bool small, bool out_f32, int tile, hipStream_t st);
int conv_pick_tile(int M, int Cout);
bool conv_glds_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st);
// split fp16 (fp32-accurate) implicit-GEMM conv: x/res/y are split-format halfs
// ([hi x32][lo x32] per 32 channels), y fp32 with out_f32
bool conv_glds_split_launch(ConvArgs a, bool out_f32, int tile, hipStream_t st);
int conv_glds_split_pick(int M, int Cout);
// K slices for a conv (1: none): force < 0 auto (the default tile), 0 / 1 off, k > 1 k slices (split-K tiles 27 / 36 / 42)
int conv_split_ksplit(int M, int Cout, int tile, int nk_total, int force, bool legacy = false);
bool conv1x1_small_m(long M);
// fmt: 0 split residual/output, 1 split residual + fp32 output, 2 fp16 residual/output, 3 fp16 residual + fp32 output
void splitk_reduce_res_launch(const float* part, int S, long MN, int N, const float* bias, const half_t* res,
                              int ldr, int relu, void* y, int ldy, int fmt, int* ovf, hipStream_t st);
int conv_f16_ksplit(int M, int Cout, int tile, int nk_total, int force);
// persistent streaming 1x1 fp16 conv, stride 1 or 2 (conv1x1_stream.hip): shapes in conv1x1_stream_supported
bool conv1x1_stream_supported(int C, int Cout, long M);
bool conv1x1_stream_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                           const void* zero, int M, int C, int Cout, int relu, int H, int W, int Wo, int HWo,
                           int stride, hipStream_t st);
bool conv1x1_stream_default(int C, int stride, long M);
bool conv1x1_stream_split_supported(int C, int Cout, long M);    // split fp16 (fp32-accurate) 1x1 convs
bool conv1x1_stream_split_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                                 const void* zero, int M, int C, int Cout, int relu, float acc_scale, int* ovf, int H,
                                 int W, int Wo, int HWo, int stride, hipStream_t st);
bool conv1x1_dual_supported(int K1, int K2, int Cout, long M);   // [x1 | x2] . [W1 | W2]: expansion + downsample
bool conv1x1_dual_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias, half_t* y,
                         const void* zero, int M, int K1, int K2, int Cout, int relu, int H, int W, int Wo, int HWo,
                         int stride, hipStream_t st);
bool conv1x1_dual_split_supported(int K1, int K2, int Cout, long M);
bool conv1x1_dual_split_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias, half_t* y,
                               const void* zero, int M, int K1, int K2, int Cout, int relu, float acc_scale, int* ovf,
                               int H, int W, int Wo, int HWo, int stride, hipStream_t st);
bool conv1x1_fused_next_supported(int K1, int K2, int N, int N2, long M);   // + next block's reduce 1x1
bool conv1x1_fused_next_launch(const half_t* x1, const half_t* x2, const half_t* w, const float* bias,
                               const half_t* res, half_t* y, const half_t* w2, const float* b2, half_t* z,
                               const void* zero, int M, int K1, int K2, int N, int N2, int relu, int H, int W, int Wo,
                               int HWo, int stride, hipStream_t st);
bool conv1x1_stream_split_default(int C, int stride);
// split 3x3/s1/p1 64 -> 64 conv, weights in registers, input rows streamed through an LDS ring
bool conv3x3_split_c64_supported(int H, int W, int C, int Cout);
bool conv3x3_split_c64_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                              const void* zero, int B, int H, int W, int relu, float acc_scale, int* ovf,
                              hipStream_t st, int per_cu = 0);
// band-staged 3x3/s1/p1 conv (conv3x3_band.hip): ResNet layers 2-4 (W 28 / 14 / 7,
// C % 64 == 0, Cout % 128 == 0); x / res read in place at pixel strides ldx / ldr (halfs).
// Split operands by default; f16: plain fp16 operands, weights [Cout][9*C], fp16 output.
bool conv3x3_band_supported(int H, int W, int C, int Cout);
int conv3x3_band_tiles(int B, int W, int Cout);
bool conv3x3_band_default(int B, int W, int Cout);       // auto-selection rule for conv2d_split
bool conv3x3_band_f16_default(int B, int W, int Cout, bool res);   // auto rule for conv2d_nhwc (fp16)
bool conv3x3_band_launch(const half_t* x, int ldx, const half_t* w, const float* bias, const half_t* res, int ldr,
                         void* y, int ldy, bool out_f32, int B, int H, int W, int C, int Cout, int relu,
                         float acc_scale, int* ovf, int max_grid, int flags, hipStream_t st, bool f16 = false);
// split-fp16 RGB stem on packed rows (a.cpk > 0, x from preprocess_pack3_split): fp32 output
bool conv_glds_split_p3_launch(ConvArgs a, int tile, hipStream_t st);   // a.cpk > 0: pack3 stem
bool conv3x3_c64_supported(int C, int Cout);
void conv3x3_c64_launch(const half_t* x, const half_t* w, const float* bias, const half_t* res, half_t* y,
                        const void* zero, int B, int H, int W, int relu, hipStream_t st);
int conv_glds_pick(int M, int Cout);
// split-fp16 (fp32-accurate) fused stem, exact-u8 form: w = [2][64][7*32] hi/lo of
// w * s_c (pre-scaled by 1/acc_scale), bias = folded bias + full sum of w * c_c,
// psum = [8][8][64] 2D prefix sums of w * c_c over (kh, kw); y = split [B][Hp][Wp][128]
// fused split AlexNet stem: uint8 -> conv 11x11/4 (exact-u8, split weights) -> ReLU -> max pool 3x3/2
// -> split [B][Hp][Wp][128]; w = [2][64][17*32] (models/packed.py pack_alex_stem_split)
bool alex_stem_u8_f16_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum,
                             float acc_scale, half_t* y, int B, int H, int W, const long long* start_idx,
                             long long start_off, long long max_start, long long sub, hipStream_t st);
void set_astem_f16_two_wg(bool on);
void set_astem_ahead(bool on);   // A/B switch: patch loads one tile ahead (1) or after the MFMA loop
void set_astem_phased(bool on);  // A/B switch: the phased two-half kernel (default) or the one-half form
void set_astem_variant(int v);   // tools/astem_ablate.py: 0 production, 16 loads after the loop, 1/2/4/6 ablations
bool alex_stem_split_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum,
                            float acc_scale, half_t* y, int B, int H, int W, const long long* start_idx,
                            long long start_off, long long max_start, long long sub, int* ovf, hipStream_t st);
void set_stem_prewait(bool on);  // A/B switch: vmcnt(0) ahead of the split stem's tile loop
void stem_split_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum, float acc_scale,
                       half_t* y, int B, int H, int W, const long long* start_idx, long long start_off,
                       long long max_start, long long sub, int* ovf, hipStream_t st);
// fp16 programs: the same exact-u8 stem with the hi MFMA only, y = fp16 [B][Hp][Wp][64]
void stem_u8_f16_launch(const uint8_t* img, const half_t* w, const float* bias, const float* psum, float acc_scale,
                        half_t* y, int B, int H, int W, const long long* start_idx, long long start_off,
                        long long max_start, long long sub, hipStream_t st);
void stem_fused_launch(const uint8_t* img, const half_t* w, const float* bias, half_t* y, int B, int H, int W,
                       const long long* start_idx, long long start_off, long long max_start, long long sub,
                       hipStream_t st);
void preprocess_launch(const uint8_t* img, half_t* out, long npix, const long long* start_idx,
                       long long start_off, long long max_start, long long sub, long pix_per_img, hipStream_t st);
void resize_crop_launch(const uint8_t* img, half_t* out, int B, int Hi, int Wi, int Hr, int Wr,
                        int crop, hipStream_t st);
void maxpool_launch(const half_t* x, half_t* y, int B, int H, int W, int C, int Ho, int Wo, int k,
                    int s, int pad, hipStream_t st);
void avgpool_launch(const half_t* x, half_t* y, int B, int HW, int C, hipStream_t st);
void synth_images_launch(uint8_t* out, uint64_t seed, long start, long n, long bytes_per_img,
                         hipStream_t st);
// split-K combine into the split-fp16 layout [M][2N] (N % 32 == 0)
void splitk_reduce_split_launch(const float* part, int S, long MN, int N, const float* bias, int relu, half_t* y,
                                int* ovf, hipStream_t st);
void splitk_reduce_launch(const float* part, int S, long MN, int N, const float* bias, int relu, void* y,
                          bool out_f32, hipStream_t st);
// ovf (or nullptr): a set split range guard marks every row class -2, prob 0 (rerun on the f32 path)
void softmax_top1_launch(const float* logits, int ld, int N, int rows, int* cls, float* prob, int* packed,
                         const int* ovf, hipStream_t st);

}  // namespace idunno
