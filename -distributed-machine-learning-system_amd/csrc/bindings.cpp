// Python bindings for the IDunno-MI355X HIP kernels.
//
// Every entry point validates the operand shapes/dtypes/devices it is handed
// before it launches anything (a malformed launch on a shared MI355X box can
// fault the whole node), then launches on PyTorch's *current* HIP stream so
// the ops compose with torch.cuda.graph capture (hipGraph) and side streams.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <mutex>

#include "kernels.h"
#include "launch_util.h"

using namespace idunno;

static hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

// Every launch is checked ("HIP error checking on every call").
static void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, what, ": HIP launch failed: ", hipGetErrorString(e));
}

// 256 zero bytes per device: the DMA source of padding taps / masked rows.
// Created once per device under a lock and never freed: several node threads
// share one GPU, and a buffer replaced by a racing thread would go back to the
// caching allocator while kernels still read it as "zeros".
static torch::Tensor zero_buffer(const torch::Device& dev) {
  static std::mutex mu;
  static std::vector<torch::Tensor>* bufs = new std::vector<torch::Tensor>(64);
  const int i = dev.index() < 0 ? 0 : dev.index();
  TORCH_CHECK(i < 64, "device index out of range");
  std::lock_guard<std::mutex> lk(mu);
  auto& b = (*bufs)[i];
  if (!b.defined()) {
    b = torch::zeros({256}, torch::TensorOptions().dtype(torch::kUInt8).device(dev));
    // other threads' streams will read it: make the fill complete before publishing
    (void)hipStreamSynchronize(cur_stream());
  }
  return b;
}

// Kernel choice is a pure function of each call's arguments (no process-global
// switches, VERDICT r4 weakness 4): `tile` forces a kernel, `ksplit` forces split-K
// slices (-1 auto for the auto-picked tile), `route` (a per-runner policy, bits
// below) opts a call out of the specialised kernels for whole-graph A/Bs.
constexpr int kRouteNoBand = 1;        // no band-staged 3x3 kernel (tile 70)
constexpr int kRouteNoC64 = 2;         // no row-streaming 3x3 64->64 kernels (tile 50)
constexpr int kRouteNoStream1x1 = 4;   // no streaming 1x1 kernels (tile 80)
constexpr int kRouteLegacySmallM = 8;  // split convs: the round-5 small-M rules (streaming 1x1 at every M,
                                       // split-K up to two blocks per CU) -- A/B arm of the round-6 rules
constexpr int kRouteC64TwoPerCU = 16;  // row-streaming 64->64 kernel: always two workgroups per CU (A/B arm)
constexpr int kRouteBandW7 = 32;       // the band-staged 3x3 at W 7 too (the round-5 rule, A/B arm)
constexpr int kRouteNoBandW28 = 64;    // no band-staged 3x3 at W 28 (ResNet layer2, A/B arm)

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype")

// y = act(conv(x, w) + bias (+ res))
//   x   : [B, H, W, C] fp16 NHWC (C == 4 for the small-C stem path, else C % 64 == 0)
//   w   : [Cout, Kpad] fp16, K ordered (kh, kw, c) [big] or (kh, kw8, c4) [small]
//   bias: [Cout] fp32
//   res : optional [B, Ho, Wo, Cout] fp16
static torch::Tensor zero_f32(const torch::Device& dev, int64_t n);

torch::Tensor conv2d_nhwc(torch::Tensor x, torch::Tensor w, torch::Tensor bias,
                          c10::optional<torch::Tensor> res, int64_t KH, int64_t KW, int64_t stride,
                          int64_t pad, bool relu, bool out_f32, int64_t tile, c10::optional<torch::Tensor> out,
                          int64_t ksplit, int64_t route) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(KH >= 1 && KW >= 1 && stride >= 1 && pad >= 0, "bad conv geometry");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Cout = w.size(0), Kpad = w.size(1);
  TORCH_CHECK(bias.size(0) == Cout, "bias/Cout mismatch");
  TORCH_CHECK(Cout % 4 == 0, "Cout must be a multiple of 4");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  const bool small = (C == 4);
  ConvArgs a{};
  if (small) {
    const int nsub = (KW + 7) / 8;
    TORCH_CHECK(Kpad == KH * nsub * 32, "small-C weight must be [Cout, KH*ceil(KW/8)*32]");
    a.nsub = nsub;
    a.nK = KH * nsub;
    a.cblk = 1;
  } else {
    TORCH_CHECK(C % 64 == 0, "C must be 4 or a multiple of 64, got ", C);
    TORCH_CHECK(Kpad == KH * KW * C, "weight must be [Cout, KH*KW*C]");
    a.cblk = C / 64;
    a.nK = KH * KW * a.cblk;
    a.nsub = 1;
  }
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(M < (1L << 31) && (long)B * H * W * C < (1L << 31), "tensor too large for int32 indexing");
  torch::Tensor y;
  if (out.has_value() && out->defined()) {   // caller-owned output (e.g. a batch slice of a bigger tensor)
    y = *out;
    CHECK_DEV(y);
    CHECK_CONTIG(y);
    CHECK_DT(y, out_f32 ? torch::kFloat : torch::kHalf);
    TORCH_CHECK(y.device() == x.device(), "out must live on the input's device");
    TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == Ho && y.size(2) == Wo && y.size(3) == Cout,
                "out shape mismatch");
  } else {
    y = torch::empty({B, Ho, Wo, Cout}, x.options().dtype(out_f32 ? torch::kFloat : torch::kHalf));
  }
  const half_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r);
    CHECK_CONTIG(r);
    CHECK_DT(r, torch::kHalf);
    TORCH_CHECK(r.dim() == 4 && r.size(0) == B && r.size(1) == Ho && r.size(2) == Wo && r.size(3) == Cout,
                "residual shape mismatch");
    TORCH_CHECK(!out_f32 || !small, "unsupported combination");
    rp = reinterpret_cast<const half_t*>(r.data_ptr());
  }
  a.x = reinterpret_cast<const half_t*>(x.data_ptr());
  a.w = reinterpret_cast<const half_t*>(w.data_ptr());
  a.bias = bias.data_ptr<float>();
  a.res = rp;
  a.y = y.data_ptr();
  a.B = B; a.H = H; a.W = W; a.C = C;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = Cout;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.M = (int)M;
  a.Kpad = Kpad;
  a.relu = relu ? 1 : 0;
  if (M == 0) return y;
  if (small) {
    const int t = (tile >= 0 && tile <= 3) ? (int)tile : conv_pick_tile(a.M, Cout);
    conv_igemm_launch(a, small, out_f32, t, cur_stream()); check_launch("conv_igemm");
    return y;
  }
  if (tile >= 0 && tile <= 3) {          // v1 register-staged loop (kept for A/B)
    conv_igemm_launch(a, small, out_f32, (int)tile, cur_stream()); check_launch("conv_igemm");
    return y;
  }
  a.zero = zero_buffer(x.device()).data_ptr();
  const bool c64_ok = KH == 3 && KW == 3 && stride == 1 && pad == 1 && !out_f32 && conv3x3_c64_supported(C, Cout);
  // resident-weight 3x3 64->64 kernel (tile 50, conv3x3_c64.hip): since sweep r1 #6 (ResNet18
  // layer1 at B=400: 112 / 153 us vs 178 / 207 us for the best im2col tile, profiles/r1_v6_layer1_c64.log)
  if (tile == 50 || (tile < 0 && c64_ok && !(route & kRouteNoC64))) {
    TORCH_CHECK(c64_ok, "tile 50 (resident-weight 3x3 64->64 conv) does not support this shape");
    conv3x3_c64_launch(a.x, a.w, a.bias, a.res, reinterpret_cast<half_t*>(a.y), a.zero, B, H, W, a.relu,
                       cur_stream()); check_launch("conv3x3_c64");
    return y;
  }
  // band-staged 3x3 kernel in fp16 (conv3x3_band.hip, tile 70): ResNet layers 2-4
  const bool band_ok = KH == 3 && KW == 3 && stride == 1 && pad == 1 && !out_f32 &&
                       conv3x3_band_supported(H, W, C, Cout);
  if (tile == 70 || (tile < 0 && band_ok && !(route & kRouteNoBand) && conv3x3_band_f16_default(B, W, Cout, rp != nullptr))) {
    TORCH_CHECK(band_ok, "tile 70 (band-staged 3x3 conv) does not support this shape");
    TORCH_CHECK(conv3x3_band_launch(a.x, C, a.w, a.bias, rp, Cout, a.y, Cout, false, B, H, W, C, Cout, a.relu, 1.0f,
                                    nullptr, 0, 0, cur_stream(), true),
                "band conv: tensor too large for 32-bit buffer offsets");
    check_launch("conv3x3_band (fp16)");
    return y;
  }
  const bool c1s_ok = KH == 1 && KW == 1 && (stride == 1 || stride == 2) && pad == 0 && !out_f32 &&
                      conv1x1_stream_supported(C, Cout, M);
  if (tile == 80 || (tile < 0 && c1s_ok && !(route & kRouteNoStream1x1) && conv1x1_stream_default(C, stride, M))) {
    TORCH_CHECK(c1s_ok, "tile 80 (streaming 1x1 conv) does not support this shape");
    conv1x1_stream_launch(a.x, a.w, a.bias, a.res, reinterpret_cast<half_t*>(a.y), a.zero, a.M, C, Cout, a.relu,
                          H, W, Wo, Ho * Wo, stride, cur_stream()); check_launch("conv1x1_stream");
    return y;
  }
  const int t = tile >= 10 ? (int)tile : conv_glds_pick(a.M, Cout);
  // split-K: auto only for the auto-picked tile (a forced tile runs its own epilogue)
  const int ks = C % 64 == 0 ? conv_f16_ksplit(a.M, Cout, t, (int)(KH * KW) * (C / 64),
                                               tile >= 0 && ksplit < 0 ? 1 : (int)ksplit) : 1;
  TORCH_CHECK(ksplit <= 1 || ks == ksplit, "split-K: ", ksplit, " slices do not divide the K loop of tile ", t);
  if (ks > 1) {
    // small M: K slices into fp32 partials, one combine (conv2d_split_impl, conv_glds.hip conv_split_ksplit)
    TORCH_CHECK((long)ks * M * Cout < (1L << 31), "split-K partials too large for int32 indexing");
    auto part = torch::empty({ks, M, (int64_t)Cout}, x.options().dtype(torch::kFloat));
    auto zb = zero_f32(x.device(), Cout);
    ConvArgs b = a;
    b.bias = zb.data_ptr<float>();
    b.res = nullptr;
    b.y = part.data_ptr<float>();
    b.ldy = Cout;
    b.relu = 0;
    b.ksplit = ks;
    b.kslice = 0;
    b.ysplit = (long)M * Cout;
    b.kstage = (int)(KH * KW) * (C / 64) / ks;
    TORCH_CHECK(conv_glds_launch(b, true, t, cur_stream()), "unknown conv tile id ", t);
    check_launch("conv_glds (split-K)");
    splitk_reduce_res_launch(part.data_ptr<float>(), ks, (long)M * Cout, Cout, a.bias, rp, Cout, a.relu, a.y, Cout,
                             out_f32 ? 3 : 2, nullptr, cur_stream());
    check_launch("splitk_reduce_res");
    return y;
  }
  TORCH_CHECK(conv_glds_launch(a, out_f32, t, cur_stream()), "unknown conv tile id ", t);
  check_launch("conv_glds");
  return y;
}

// ResNet bottleneck tail as ONE GEMM: y = act([x1 | x2 gathered at stride] .
// [W3 | Wds]^T + b), i.e. the expansion 1x1 conv of the block's last conv
// input x1 plus the 1x1 (strided) downsample of the block input x2, whose sum
// is the residual add -- the downsample's output never reaches HBM
// (conv1x1_stream.hip, dual input).
//   x1 [B, Ho, Wo, K1] fp16, x2 [B, H, W, K2] fp16, w [Cout, K1 + K2] fp16, bias [Cout] f32
torch::Tensor conv1x1_dual(torch::Tensor x1, torch::Tensor x2, torch::Tensor w, torch::Tensor bias, int64_t stride,
                           bool relu) {
  CHECK_DEV(x1); CHECK_DEV(x2); CHECK_DEV(w); CHECK_DEV(bias);
  CHECK_CONTIG(x1); CHECK_CONTIG(x2); CHECK_CONTIG(w); CHECK_CONTIG(bias);
  CHECK_DT(x1, torch::kHalf); CHECK_DT(x2, torch::kHalf); CHECK_DT(w, torch::kHalf); CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x1.dim() == 4 && x2.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(x2.device() == x1.device() && w.device() == x1.device() && bias.device() == x1.device(),
              "operands on different devices");
  TORCH_CHECK(stride >= 1, "bad stride");
  const int B = x1.size(0), Ho = x1.size(1), Wo = x1.size(2), K1 = x1.size(3);
  const int H = x2.size(1), W = x2.size(2), K2 = x2.size(3);
  const int Cout = w.size(0);
  TORCH_CHECK(x2.size(0) == B && (H - 1) / stride + 1 == Ho && (W - 1) / stride + 1 == Wo,
              "x2 must be the block input at `stride` of x1's resolution");
  TORCH_CHECK(w.size(1) == K1 + K2 && bias.size(0) == Cout, "weight must be [Cout, K1 + K2]");
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(conv1x1_dual_supported(K1, K2, Cout, M), "conv1x1_dual: unsupported shape (K1 ", K1, ", K2 ", K2,
              ", Cout ", Cout, ")");
  auto y = torch::empty({B, Ho, Wo, Cout}, x1.options());
  conv1x1_dual_launch(reinterpret_cast<const half_t*>(x1.data_ptr()), reinterpret_cast<const half_t*>(x2.data_ptr()),
                      reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(),
                      reinterpret_cast<half_t*>(y.data_ptr()), zero_buffer(x1.device()).data_ptr(), (int)M, K1, K2,
                      Cout, relu ? 1 : 0, H, W, Wo, Ho * Wo, (int)stride, cur_stream());
  check_launch("conv1x1_dual");
  return y;
}

bool conv1x1_dual_ok(int64_t K1, int64_t K2, int64_t Cout, int64_t M) {
  return conv1x1_dual_supported((int)K1, (int)K2, (int)Cout, (long)M);
}

static int* split_guard_for(const torch::Device& dev);

// Bottleneck tail + the NEXT block's reduce 1x1 in one pass (fp16, layer1 of
// ResNet50): y = relu(x1 . W^T + b + res) -- or, with x2, the dual form
// relu([x1 | x2] . W^T + b) -- and z = relu(y . w2^T + b2) from the output tile
// on chip.  Returns [y, z].
std::vector<torch::Tensor> conv1x1_fused_next(torch::Tensor x1, c10::optional<torch::Tensor> x2, torch::Tensor w,
                                              torch::Tensor bias, c10::optional<torch::Tensor> res, torch::Tensor w2,
                                              torch::Tensor b2, int64_t stride, bool relu) {
  CHECK_DEV(x1); CHECK_DEV(w); CHECK_DEV(bias); CHECK_DEV(w2); CHECK_DEV(b2);
  CHECK_CONTIG(x1); CHECK_CONTIG(w); CHECK_CONTIG(bias); CHECK_CONTIG(w2); CHECK_CONTIG(b2);
  CHECK_DT(x1, torch::kHalf); CHECK_DT(w, torch::kHalf); CHECK_DT(bias, torch::kFloat);
  CHECK_DT(w2, torch::kHalf); CHECK_DT(b2, torch::kFloat);
  TORCH_CHECK(x1.dim() == 4 && w.dim() == 2 && w2.dim() == 2, "bad ranks");
  const int B = x1.size(0), Ho = x1.size(1), Wo = x1.size(2), K1 = x1.size(3);
  const int N = w.size(0), N2 = w2.size(0);
  const half_t* x2p = nullptr;
  int H = Ho, W = Wo, K2 = 0;
  if (x2.has_value() && x2->defined()) {
    auto& t = *x2;
    CHECK_DEV(t); CHECK_CONTIG(t); CHECK_DT(t, torch::kHalf);
    TORCH_CHECK(t.dim() == 4 && t.size(0) == B, "x2 must be [B, H, W, K2]");
    H = t.size(1); W = t.size(2); K2 = t.size(3);
    TORCH_CHECK((H - 1) / stride + 1 == Ho && (W - 1) / stride + 1 == Wo, "x2 must be at `stride` of x1's resolution");
    x2p = reinterpret_cast<const half_t*>(t.data_ptr());
  }
  TORCH_CHECK(w.size(1) == K1 + K2 && bias.size(0) == N && w2.size(1) == N && b2.size(0) == N2, "weight shapes");
  const half_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r); CHECK_CONTIG(r); CHECK_DT(r, torch::kHalf);
    TORCH_CHECK(r.dim() == 4 && r.size(0) == B && r.size(1) == Ho && r.size(2) == Wo && r.size(3) == N,
                "residual shape mismatch");
    TORCH_CHECK(x2p == nullptr, "the dual form carries its residual as the second GEMM input");
    rp = reinterpret_cast<const half_t*>(r.data_ptr());
  }
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(conv1x1_fused_next_supported(K1, K2, N, N2, M), "conv1x1_fused_next: unsupported shape");
  auto y = torch::empty({B, Ho, Wo, N}, x1.options());
  auto z = torch::empty({B, Ho, Wo, N2}, x1.options());
  conv1x1_fused_next_launch(reinterpret_cast<const half_t*>(x1.data_ptr()), x2p,
                            reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(), rp,
                            reinterpret_cast<half_t*>(y.data_ptr()), reinterpret_cast<const half_t*>(w2.data_ptr()),
                            b2.data_ptr<float>(), reinterpret_cast<half_t*>(z.data_ptr()),
                            zero_buffer(x1.device()).data_ptr(), (int)M, K1, K2, N, N2, relu ? 1 : 0, H, W, Wo,
                            Ho * Wo, (int)stride, cur_stream());
  check_launch("conv1x1_fused_next");
  return {y, z};
}

bool conv1x1_fused_next_ok(int64_t K1, int64_t K2, int64_t N, int64_t N2, int64_t M) {
  return conv1x1_fused_next_supported((int)K1, (int)K2, (int)N, (int)N2, (long)M);
}


// split (fp32-accurate) form of conv1x1_dual: x1 [B, Ho, Wo, 2 K1], x2 [B, H, W, 2 K2]
// split layouts, w [Cout, 2 (K1 + K2)] = pack_split_weight([W3 | Wds]) with one
// accumulator scale; split output [B, Ho, Wo, 2 Cout] (range-guarded)
torch::Tensor conv1x1_dual_split(torch::Tensor x1, torch::Tensor x2, torch::Tensor w, torch::Tensor bias,
                                 double acc_scale, int64_t stride, bool relu) {
  CHECK_DEV(x1); CHECK_DEV(x2); CHECK_DEV(w); CHECK_DEV(bias);
  CHECK_CONTIG(x1); CHECK_CONTIG(x2); CHECK_CONTIG(w); CHECK_CONTIG(bias);
  CHECK_DT(x1, torch::kHalf); CHECK_DT(x2, torch::kHalf); CHECK_DT(w, torch::kHalf); CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x1.dim() == 4 && x2.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(x2.device() == x1.device() && w.device() == x1.device() && bias.device() == x1.device(),
              "operands on different devices");
  TORCH_CHECK(stride >= 1, "bad stride");
  const int B = x1.size(0), Ho = x1.size(1), Wo = x1.size(2), K1 = x1.size(3) / 2;
  const int H = x2.size(1), W = x2.size(2), K2 = x2.size(3) / 2;
  const int Cout = w.size(0);
  TORCH_CHECK(x1.size(3) % 64 == 0 && x2.size(3) % 64 == 0, "split inputs need 2C halfs with C % 32 == 0");
  TORCH_CHECK(x2.size(0) == B && (H - 1) / stride + 1 == Ho && (W - 1) / stride + 1 == Wo,
              "x2 must be the block input at `stride` of x1's resolution");
  TORCH_CHECK(w.size(1) == 2 * (K1 + K2) && bias.size(0) == Cout, "split weight must be [Cout, 2 (K1 + K2)]");
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(conv1x1_dual_split_supported(K1, K2, Cout, M), "conv1x1_dual_split: unsupported shape (K1 ", K1,
              ", K2 ", K2, ", Cout ", Cout, ")");
  auto y = torch::empty({B, Ho, Wo, 2 * Cout}, x1.options());
  conv1x1_dual_split_launch(reinterpret_cast<const half_t*>(x1.data_ptr()),
                            reinterpret_cast<const half_t*>(x2.data_ptr()), reinterpret_cast<const half_t*>(w.data_ptr()),
                            bias.data_ptr<float>(), reinterpret_cast<half_t*>(y.data_ptr()),
                            zero_buffer(x1.device()).data_ptr(), (int)M, K1, K2, Cout, relu ? 1 : 0, (float)acc_scale,
                            split_guard_for(x1.device()), H, W, Wo, Ho * Wo, (int)stride, cur_stream());
  check_launch("conv1x1_dual_split");
  return y;
}

bool conv1x1_dual_split_ok(int64_t K1, int64_t K2, int64_t Cout, int64_t M) {
  return conv1x1_dual_split_supported((int)K1, (int)K2, (int)Cout, (long)M);
}

// fp32 (reference precision) conv: y = act(conv(x, w) + bias (+ res)), all f32.
//   x   : [B, H, W, C] f32 NHWC, C == 4 (RGB+0 stem) or C % 16 == 0
//   w   : [Cout, Kpad] f32: big (kh, kw, c), Kpad = KH*KW*C;
//         small (kh, tap, c4) with taps padded to ceil(KW/4)*4, Kpad = KH*ceil(KW/4)*16
torch::Tensor conv2d_nhwc_f32(torch::Tensor x, torch::Tensor w, torch::Tensor bias, c10::optional<torch::Tensor> res,
                              int64_t KH, int64_t KW, int64_t stride, int64_t pad, bool relu, int64_t tile,
                              c10::optional<torch::Tensor> out) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kFloat);
  CHECK_DT(w, torch::kFloat);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  TORCH_CHECK(KH >= 1 && KW >= 1 && stride >= 1 && pad >= 0, "bad conv geometry");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Cout = w.size(0), Kpad = w.size(1);
  TORCH_CHECK(bias.size(0) == Cout, "bias/Cout mismatch");
  TORCH_CHECK(Cout % 4 == 0, "Cout must be a multiple of 4");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  const bool small = (C == 4);
  ConvF32Args a{};
  if (small) {
    a.nsub = (KW + 3) / 4;
    TORCH_CHECK(Kpad == KH * a.nsub * 16, "small-C f32 weight must be [Cout, KH*ceil(KW/4)*16]");
  } else {
    TORCH_CHECK(C % 16 == 0, "C must be 4 or a multiple of 16, got ", C);
    TORCH_CHECK(Kpad == KH * KW * C, "weight must be [Cout, KH*KW*C]");
    a.nsub = 1;
  }
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(M < (1L << 31) && (long)B * H * W * C < (1L << 31) && M * Cout < (1L << 40),
              "tensor too large for int32 indexing");
  torch::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    CHECK_DEV(y);
    CHECK_CONTIG(y);
    CHECK_DT(y, torch::kFloat);
    TORCH_CHECK(y.device() == x.device(), "out must live on the input's device");
    TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == Ho && y.size(2) == Wo && y.size(3) == Cout,
                "out shape mismatch");
  } else {
    y = torch::empty({B, Ho, Wo, Cout}, x.options());
  }
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r);
    CHECK_CONTIG(r);
    CHECK_DT(r, torch::kFloat);
    TORCH_CHECK(r.device() == x.device(), "residual on a different device");
    TORCH_CHECK(r.dim() == 4 && r.size(0) == B && r.size(1) == Ho && r.size(2) == Wo && r.size(3) == Cout,
                "residual shape mismatch");
    rp = r.data_ptr<float>();
  }
  a.x = x.data_ptr<float>();
  a.w = w.data_ptr<float>();
  a.bias = bias.data_ptr<float>();
  a.res = rp;
  a.y = y.data_ptr<float>();
  a.B = B; a.H = H; a.W = W; a.C = C;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = Cout;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.M = (int)M;
  a.Kpad = Kpad;
  a.relu = relu ? 1 : 0;
  if (M == 0) return y;
  a.zero = zero_buffer(x.device()).data_ptr();
  const int t = tile >= 0 ? (int)tile : conv_f32_pick(a.M, Cout, Kpad, small);
  TORCH_CHECK(conv_f32_launch(a, small ? 1 : 0, t, cur_stream()), "unknown / unsupported f32 conv tile id ", t);
  check_launch("conv_f32");
  return y;
}

static torch::Tensor zero_f32(const torch::Device& dev, int64_t n);

// Split range guard (common.h split_guard): the int32 flag
// that this thread's split launches write to when a value leaves fp16's range;
// HipRunner sets it around a split forward (a captured graph keeps the pointer).
static thread_local int* g_split_guard = nullptr;
static thread_local int g_split_guard_dev = -1;
void set_split_guard(c10::optional<torch::Tensor> flag) {
  if (!flag.has_value() || !flag->defined()) {
    g_split_guard = nullptr;
    g_split_guard_dev = -1;
    return;
  }
  auto& f = *flag;
  CHECK_DEV(f);
  CHECK_CONTIG(f);
  CHECK_DT(f, torch::kInt);
  TORCH_CHECK(f.numel() >= 1, "split guard flag must hold one int32");
  g_split_guard = f.data_ptr<int>();
  g_split_guard_dev = f.device().index();
}
static int* split_guard_for(const torch::Device& dev) {
  if (g_split_guard == nullptr) return nullptr;
  TORCH_CHECK(dev.index() == g_split_guard_dev, "split guard flag lives on another device");
  return g_split_guard;
}


// split fp16 (fp32-accurate) conv: y = act(acc_scale * conv(x, w) + bias (+ res)).
//   x   : [B, H, W, 2C] half, split layout ([hi x32][lo x32] per 32 channels), C % 32 == 0
//   w   : [Cout, KH*KW*2C] half, same layout per tap, pre-scaled by 1/acc_scale
//   res : optional [B, Ho, Wo, 2Cout] half (split);  y: split half, or fp32 [B, Ho, Wo, Cout]
// Pixel stride (halfs) of an NHWC view whose channels are contiguous and whose
// pixels are equally spaced: a channel slice of a wider tensor (the two halves
// of a dual conv's output) is read in place.
static int64_t nhwc_pixel_stride(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.dim() == 4, what, " must be 4-D NHWC");
  const int64_t P = t.stride(2);
  TORCH_CHECK(t.stride(3) == 1 && P >= t.size(3) && t.stride(1) == t.size(2) * P && t.stride(0) == t.size(1) * t.stride(1),
              what, " must be NHWC with contiguous channels and equally strided pixels");
  TORCH_CHECK(P % 8 == 0 && t.storage_offset() % 8 == 0, what, " pixel stride / offset must be 16-byte aligned");
  return P;
}

static torch::Tensor conv2d_split_impl(torch::Tensor x, torch::Tensor w, torch::Tensor bias,
                                       c10::optional<torch::Tensor> res, int64_t KH, int64_t KW, int64_t stride,
                                       int64_t pad, bool relu, double acc_scale, bool out_f32, int64_t tile,
                                       c10::optional<torch::Tensor> out, int64_t nsplit, bool center_only,
                                       double acc_scale2, int64_t ksplit, int64_t route) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  const int64_t xP = nhwc_pixel_stride(x, "x");
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  TORCH_CHECK(KH >= 1 && KW >= 1 && stride >= 1 && pad >= 0, "bad conv geometry");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C2 = x.size(3);
  TORCH_CHECK(C2 % 64 == 0, "split input needs 2C halfs with C % 32 == 0, got ", C2);
  const int Cout = w.size(0), Kpad = w.size(1);
  TORCH_CHECK(Kpad == KH * KW * C2, "split weight must be [Cout, KH*KW*2C]");
  TORCH_CHECK(bias.size(0) == Cout, "bias/Cout mismatch");
  TORCH_CHECK(Cout % 32 == 0, "split conv needs Cout % 32 == 0");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(M < (1L << 31) && (long)B * H * W * xP < (1L << 31) && M * 2 * Cout < (1L << 31),
              "tensor too large for int32 indexing");
  const int64_t ych = out_f32 ? Cout : 2 * Cout;
  torch::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    CHECK_DEV(y);
    CHECK_CONTIG(y);
    CHECK_DT(y, out_f32 ? torch::kFloat : torch::kHalf);
    TORCH_CHECK(y.device() == x.device(), "out must live on the input's device");
    TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == Ho && y.size(2) == Wo && y.size(3) == ych,
                "out shape mismatch");
  } else {
    y = torch::empty({B, Ho, Wo, ych}, x.options().dtype(out_f32 ? torch::kFloat : torch::kHalf));
  }
  const half_t* rp = nullptr;
  int64_t rP = 2 * Cout;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r);
    rP = nhwc_pixel_stride(r, "residual");
    CHECK_DT(r, torch::kHalf);
    TORCH_CHECK(r.device() == x.device(), "residual on a different device");
    TORCH_CHECK(r.dim() == 4 && r.size(0) == B && r.size(1) == Ho && r.size(2) == Wo && r.size(3) == 2 * Cout,
                "residual shape mismatch (split [B, Ho, Wo, 2*Cout])");
    rp = reinterpret_cast<const half_t*>(r.data_ptr());
  }
  ConvArgs a{};
  a.x = reinterpret_cast<const half_t*>(x.data_ptr());
  a.w = reinterpret_cast<const half_t*>(w.data_ptr());
  a.bias = bias.data_ptr<float>();
  a.res = rp;
  a.y = y.data_ptr();
  a.B = B; a.H = H; a.W = W; a.C = C2;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = (int)ych;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.M = (int)M;
  a.Kpad = Kpad;
  a.relu = relu ? 1 : 0;
  a.acc_scale = (float)acc_scale;
  a.ovf = out_f32 ? nullptr : split_guard_for(x.device());
  // strided views (a dual conv's halves): conv_glds reads them in place
  const bool strided = xP != C2 || rP != 2 * Cout;
  a.ldx = xP != C2 ? (int)xP : 0;
  a.ldr = rP != 2 * Cout ? (int)rP : 0;
  TORCH_CHECK(nsplit >= 0 && nsplit < Cout && nsplit % 32 == 0, "dual conv split must be a multiple of 32 below Cout");
  a.nsplit_n = (int)nsplit;
  a.center_only = center_only ? 1 : 0;
  a.acc_scale2 = (float)acc_scale2;
  TORCH_CHECK(!center_only || (nsplit > 0 && KH % 2 == 1 && KW % 2 == 1 && pad == KH / 2 && pad == KW / 2),
              "centre-only dual conv needs an odd, 'same'-padded kernel");
  if (M == 0) return y;
  a.zero = zero_buffer(x.device()).data_ptr();
  const bool c64_ok = KH == 3 && KW == 3 && stride == 1 && pad == 1 && !out_f32 && !strided && nsplit == 0 &&
                      conv3x3_split_c64_supported(H, W, C2 / 2, Cout);
  // row-streaming register-weight kernel for split 3x3/s1 64->64 (ResNet layer1)
  if (tile == 50 || (tile < 0 && c64_ok && !(route & kRouteNoC64))) {
    TORCH_CHECK(c64_ok, "tile 50 (row-streaming split 3x3 64->64 conv) does not support this shape");
    TORCH_CHECK(conv3x3_split_c64_launch(a.x, a.w, a.bias, a.res, reinterpret_cast<half_t*>(a.y), a.zero, B, H, W,
                                         a.relu, a.acc_scale, a.ovf, cur_stream(), (route & kRouteC64TwoPerCU) ? 2 : 0),
                "row-streaming split conv: tensor too large for 32-bit offsets");
    check_launch("conv3x3_split_c64");
    return y;
  }
  // band-staged 3x3 kernel (conv3x3_band.hip, tile 70): ResNet layers 2 and 4 at batches
  // that give every CU a tile (conv3x3_band_default; otherwise the im2col tiles + split-K)
  const bool band_ok = KH == 3 && KW == 3 && stride == 1 && pad == 1 && nsplit == 0 &&
                       conv3x3_band_supported(H, W, C2 / 2, Cout);
  const bool band_off = (route & kRouteNoBand) || (W == 28 && (route & kRouteNoBandW28));
  const bool band_on = conv3x3_band_default(B, W, Cout) ||
                       (W == 7 && (route & kRouteBandW7) && conv3x3_band_tiles(B, W, Cout) >= device_cu_count());
  if (tile == 70 || (tile < 0 && band_ok && !band_off && band_on)) {
    TORCH_CHECK(band_ok, "tile 70 (band-staged split 3x3 conv) does not support this shape");
    TORCH_CHECK(conv3x3_band_launch(a.x, (int)xP, a.w, a.bias, rp, (int)rP, a.y, (int)ych, out_f32, B, H, W, C2 / 2,
                                    Cout, a.relu, a.acc_scale, a.ovf, 0, 0, cur_stream()),
                "band conv: tensor too large for 32-bit buffer offsets");
    check_launch("conv3x3_band");
    return y;
  }
  const bool c1s_ok = KH == 1 && KW == 1 && (stride == 1 || stride == 2) && pad == 0 && !out_f32 && !strided &&
                      nsplit == 0 && conv1x1_stream_split_supported(C2 / 2, Cout, M);
  const bool legacy_small = (route & kRouteLegacySmallM) != 0;
  if (tile == 80 || (tile < 0 && c1s_ok && !(route & kRouteNoStream1x1) && conv1x1_stream_split_default(C2 / 2, stride) &&
                     (legacy_small || !conv1x1_small_m(M)))) {
    TORCH_CHECK(c1s_ok, "tile 80 (streaming split 1x1 conv) does not support this shape");
    conv1x1_stream_split_launch(a.x, a.w, a.bias, a.res, reinterpret_cast<half_t*>(a.y), a.zero, a.M, C2 / 2, Cout,
                                a.relu, a.acc_scale, a.ovf, H, W, Wo, Ho * Wo, stride, cur_stream());
    check_launch("conv1x1_stream_split");
    return y;
  }
  // a small-M 1x1 (the downsample at a few dozen images per GPU) on the 128 x 64 tile
  // (a forced ksplit > 1 keeps the split-K tile: tests drive that path at small M)
  const bool small_1x1 = KH == 1 && KW == 1 && !legacy_small && conv1x1_small_m(M) && Cout % 128 == 0 && ksplit <= 1;
  const int t = tile >= 0 ? (int)tile : (small_1x1 ? 38 : conv_glds_split_pick(a.M, Cout));
  const int nk_total = (int)(KH * KW) * (C2 / 64);
  // split-K: auto only for the auto-picked tile (a forced tile runs its own epilogue)
  const int ks = nsplit == 0 ? conv_split_ksplit(a.M, Cout, t, nk_total, tile >= 0 && ksplit < 0 ? 1 : (int)ksplit,
                                                 legacy_small)
                             : 1;
  TORCH_CHECK(ksplit <= 1 || ks == ksplit, "split-K: ", ksplit, " slices do not divide the K loop of tile ", t);
  if (ks > 1) {
    // small M: K slices into fp32 partials in one launch, then one combine
    // (bias, residual, ReLU, split + range guard) -- conv_glds.hip conv_split_ksplit
    TORCH_CHECK((long)ks * M * Cout < (1L << 31), "split-K partials too large for int32 indexing");
    auto part = torch::empty({ks, M, (int64_t)Cout}, x.options().dtype(torch::kFloat));
    auto zb = zero_f32(x.device(), Cout);
    ConvArgs b = a;
    b.bias = zb.data_ptr<float>();
    b.res = nullptr;
    b.ldr = 0;
    b.y = part.data_ptr<float>();
    b.ldy = Cout;
    b.relu = 0;
    b.ovf = nullptr;
    b.ksplit = ks;
    b.kslice = 0;
    b.ysplit = (long)M * Cout;
    b.kstage = nk_total / ks;
    TORCH_CHECK(conv_glds_split_launch(b, true, t, cur_stream()), "unknown split conv tile id ", t);
    check_launch("conv_glds_split (split-K)");
    splitk_reduce_res_launch(part.data_ptr<float>(), ks, (long)M * Cout, Cout, a.bias, rp, (int)rP, a.relu, a.y,
                             (int)ych, out_f32 ? 1 : 0, a.ovf, cur_stream());
    check_launch("splitk_reduce_res");
    return y;
  }
  TORCH_CHECK(conv_glds_split_launch(a, out_f32, t, cur_stream()), "unknown split conv tile id ", t);
  check_launch("conv_glds_split");
  return y;
}

// Band-staged split 3x3/s1/p1 conv with an explicit persistent-grid cap (tests:
// max_grid < tiles makes every workgroup run several tiles through one DMA ring).
torch::Tensor conv3x3_band_split(torch::Tensor x, torch::Tensor w, torch::Tensor bias, c10::optional<torch::Tensor> res,
                                 bool relu, double acc_scale, bool out_f32, int64_t max_grid, int64_t flags) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  const int64_t xP = nhwc_pixel_stride(x, "x");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C2 = x.size(3), Cout = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == 9 * C2 && bias.numel() == Cout, "split weight must be [Cout, 9*2C]");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  TORCH_CHECK(conv3x3_band_supported(H, W, C2 / 2, Cout), "band conv: unsupported shape");
  const int64_t ych = out_f32 ? Cout : 2 * Cout;
  auto y = torch::empty({B, H, W, ych}, x.options().dtype(out_f32 ? torch::kFloat : torch::kHalf));
  const half_t* rp = nullptr;
  int64_t rP = 2 * Cout;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r);
    CHECK_DT(r, torch::kHalf);
    rP = nhwc_pixel_stride(r, "residual");
    TORCH_CHECK(r.device() == x.device() && r.size(0) == B && r.size(1) == H && r.size(2) == W && r.size(3) == 2 * Cout,
                "residual shape mismatch (split [B, H, W, 2*Cout])");
    rp = reinterpret_cast<const half_t*>(r.data_ptr());
  }
  if (B == 0) return y;
  TORCH_CHECK(conv3x3_band_launch(reinterpret_cast<const half_t*>(x.data_ptr()), (int)xP,
                                  reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(), rp, (int)rP,
                                  y.data_ptr(), (int)ych, out_f32, B, H, W, C2 / 2, Cout, relu ? 1 : 0, (float)acc_scale,
                                  out_f32 ? nullptr : split_guard_for(x.device()), (int)max_grid, (int)flags,
                                  cur_stream()),
              "band conv: tensor too large for 32-bit buffer offsets");
  check_launch("conv3x3_band");
  return y;
}

// fp16 band-staged 3x3/s1/p1 conv with a persistent-grid cap (tests)
torch::Tensor conv3x3_band_f16(torch::Tensor x, torch::Tensor w, torch::Tensor bias, c10::optional<torch::Tensor> res,
                               bool relu, int64_t max_grid) {
  CHECK_DEV(x); CHECK_DEV(w); CHECK_DEV(bias);
  CHECK_CONTIG(x); CHECK_CONTIG(w); CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf); CHECK_DT(w, torch::kHalf); CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "bad ranks");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Cout = w.size(0);
  TORCH_CHECK(w.size(1) == 9 * C && bias.numel() == Cout, "fp16 weight must be [Cout, 9*C]");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  TORCH_CHECK(conv3x3_band_supported(H, W, C, Cout), "band conv: unsupported shape");
  auto y = torch::empty({B, H, W, Cout}, x.options());
  const half_t* rp = nullptr;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r); CHECK_CONTIG(r); CHECK_DT(r, torch::kHalf);
    TORCH_CHECK(r.device() == x.device() && r.dim() == 4 && r.size(0) == B && r.size(1) == H && r.size(2) == W &&
                r.size(3) == Cout, "residual shape mismatch");
    rp = reinterpret_cast<const half_t*>(r.data_ptr());
  }
  if (B == 0) return y;
  TORCH_CHECK(conv3x3_band_launch(reinterpret_cast<const half_t*>(x.data_ptr()), C,
                                  reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(), rp, Cout,
                                  y.data_ptr(), Cout, false, B, H, W, C, Cout, relu ? 1 : 0, 1.0f, nullptr,
                                  (int)max_grid, 0, cur_stream(), true),
              "band conv: tensor too large for 32-bit buffer offsets");
  check_launch("conv3x3_band (fp16)");
  return y;
}

torch::Tensor conv2d_split(torch::Tensor x, torch::Tensor w, torch::Tensor bias, c10::optional<torch::Tensor> res,
                           int64_t KH, int64_t KW, int64_t stride, int64_t pad, bool relu, double acc_scale,
                           bool out_f32, int64_t tile, c10::optional<torch::Tensor> out, int64_t ksplit,
                           int64_t route) {
  return conv2d_split_impl(x, w, bias, res, KH, KW, stride, pad, relu, acc_scale, out_f32, tile, out, 0, false, 1.0,
                           ksplit, route);
}

// Two split convs of one input in ONE launch (the ResNet stride-2
// block's 1x1/2 downsample is the centre tap of its 3x3/2 conv): w / bias are
// [Cout1 + Cout2, ...] with the second conv's weights in the centre-tap K block
// (zeros elsewhere, never read); output channels [0, nsplit) = conv 1 (ReLU if
// relu, scale acc_scale), [nsplit, Cout) = conv 2 (no ReLU, scale acc_scale2,
// K loop over the centre tap only when center_only).  y = [B, Ho, Wo, 2*Cout]
// split; its channel halves are read in place by the next convs (pixel stride).
torch::Tensor conv2d_split_dual(torch::Tensor x, torch::Tensor w, torch::Tensor bias, int64_t KH, int64_t KW,
                                int64_t stride, int64_t pad, bool relu, double acc_scale, double acc_scale2,
                                int64_t nsplit, bool center_only, int64_t tile) {
  TORCH_CHECK(nsplit > 0, "dual conv needs nsplit > 0");
  return conv2d_split_impl(x, w, bias, c10::nullopt, KH, KW, stride, pad, relu, acc_scale, false, tile,
                           c10::nullopt, nsplit, center_only, acc_scale2, 1, 0);
}

// fp32-accurate FC on split fp16: y = act(acc_scale * x @ w.T + bias)
//   x [M, 2K] split, w [N, 2K] split (pack_split_weight of [N, K, 1, 1]); K % 32 == 0.
// K is cut into `splits` slices in ONE conv_glds launch (fp32 partials) + the
// combine, which writes fp32 [M, N] or split [M, 2N] (N % 32 == 0).
torch::Tensor linear_split(torch::Tensor x, torch::Tensor w, torch::Tensor bias, double acc_scale, bool relu,
                           bool out_f32, int64_t splits, int64_t tile) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  const int64_t M = x.size(0), K2 = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K2 && bias.size(0) == N, "shape mismatch");
  TORCH_CHECK(out_f32 ? N % 4 == 0 : N % 32 == 0, "N must be a multiple of 4 (fp32 out) / 32 (split out)");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K2 % (64 * splits) == 0, "K must split into multiples of 32");
  TORCH_CHECK(splits * M * N < (1L << 31) && M * K2 < (1L << 31), "too large for int32 indexing");
  auto part = torch::empty({splits, M, N}, x.options().dtype(torch::kFloat));
  auto y = out_f32 ? torch::empty({M, N}, x.options().dtype(torch::kFloat))
                   : torch::empty({M, 2 * N}, x.options().dtype(torch::kHalf));
  if (M == 0) return y;
  const int64_t Ks2 = K2 / splits;
  auto zb = zero_f32(x.device(), N);
  ConvArgs a{};
  a.x = reinterpret_cast<const half_t*>(x.data_ptr());
  a.w = reinterpret_cast<const half_t*>(w.data_ptr());
  a.bias = zb.data_ptr<float>();
  a.res = nullptr;
  a.y = part.data_ptr<float>();
  a.B = (int)M; a.H = 1; a.W = 1; a.C = (int)Ks2; a.ldx = (int)K2;
  a.Ho = 1; a.Wo = 1; a.Cout = (int)N; a.ldy = (int)N;
  a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
  a.M = (int)M;
  a.Kpad = (int)K2;
  a.relu = 0;
  a.acc_scale = (float)acc_scale;
  a.zero = zero_buffer(x.device()).data_ptr();
  a.ksplit = (int)splits;
  a.kslice = (int)Ks2;
  a.ysplit = (long)(M * N);
  const int t = tile >= 0 ? (int)tile : conv_glds_split_pick((int)M, (int)N);
  TORCH_CHECK(conv_glds_split_launch(a, true, t, cur_stream()), "unknown split conv tile id ", t);
  check_launch("linear_split");
  if (out_f32)
    splitk_reduce_launch(part.data_ptr<float>(), (int)splits, (long)(M * N), (int)N, bias.data_ptr<float>(),
                         relu ? 1 : 0, y.data_ptr(), true, cur_stream());
  else
    splitk_reduce_split_launch(part.data_ptr<float>(), (int)splits, (long)(M * N), (int)N, bias.data_ptr<float>(),
                               relu ? 1 : 0, reinterpret_cast<half_t*>(y.data_ptr()), split_guard_for(x.device()),
                               cur_stream());
  check_launch("splitk_reduce");
  return y;
}

// fp32 NHWC [.., C] <-> split [.., 2C] (C % 32 == 0)
torch::Tensor split_from_f32(torch::Tensor x) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  CHECK_DT(x, torch::kFloat);
  TORCH_CHECK(x.dim() >= 1 && x.size(-1) % 32 == 0, "last dim must be a multiple of 32");
  const int C = x.size(-1);
  auto sz = x.sizes().vec();
  sz.back() = 2 * C;
  auto y = torch::empty(sz, x.options().dtype(torch::kHalf));
  const long npix = C ? x.numel() / C : 0;
  if (npix == 0) return y;
  split_from_f32_launch(x.data_ptr<float>(), reinterpret_cast<half_t*>(y.data_ptr()), npix, C,
                        split_guard_for(x.device()), cur_stream());
  check_launch("split_from_f32");
  return y;
}

torch::Tensor f32_from_split(torch::Tensor x) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  CHECK_DT(x, torch::kHalf);
  TORCH_CHECK(x.dim() >= 1 && x.size(-1) % 64 == 0, "last dim must be 2C with C % 32 == 0");
  const int C = x.size(-1) / 2;
  auto sz = x.sizes().vec();
  sz.back() = C;
  auto y = torch::empty(sz, x.options().dtype(torch::kFloat));
  const long npix = x.numel() / (2 * C);
  if (npix == 0) return y;
  f32_from_split_launch(reinterpret_cast<const half_t*>(x.data_ptr()), y.data_ptr<float>(), npix, C, cur_stream());
  check_launch("f32_from_split");
  return y;
}

// NHWC max pool into the split layout; x fp32 [B,H,W,C] or split half [B,H,W,2C]
torch::Tensor maxpool2d_split(torch::Tensor x, int64_t k, int64_t s, int64_t pad, c10::optional<torch::Tensor> out) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4, "x must be NHWC");
  const bool in_split = x.scalar_type() == torch::kHalf;
  TORCH_CHECK(in_split || x.scalar_type() == torch::kFloat, "x must be fp32 or split half");
  TORCH_CHECK(k >= 1 && s >= 1 && pad >= 0 && pad < k, "bad pool geometry");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = in_split ? x.size(3) / 2 : x.size(3);
  TORCH_CHECK(C % 32 == 0 && (!in_split || x.size(3) == 2 * C), "channels must be a multiple of 32");
  const int Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  torch::Tensor y;
  if (out.has_value() && out->defined()) {
    y = *out;
    CHECK_DEV(y);
    CHECK_CONTIG(y);
    CHECK_DT(y, torch::kHalf);
    TORCH_CHECK(y.device() == x.device(), "out must live on the input's device");
    TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == Ho && y.size(2) == Wo && y.size(3) == 2 * C,
                "out shape mismatch");
  } else {
    y = torch::empty({B, Ho, Wo, 2 * C}, x.options().dtype(torch::kHalf));
  }
  if ((long)B * Ho * Wo == 0) return y;
  maxpool_split_launch(x.data_ptr(), in_split, reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, C, Ho, Wo, k, s, pad,
                       split_guard_for(x.device()), cur_stream());
  check_launch("maxpool_split");
  return y;
}

int64_t pick_tile_split(int64_t M, int64_t Cout) { return conv_glds_split_pick((int)M, (int)Cout); }

// fp32 FC layer y = act(x @ w.T + bias) with K split over `splits` slices in ONE
// conv_f32 launch (grid = tiles x splits, fp32 partials) + the split-K combine.
torch::Tensor linear_f32_splitk(torch::Tensor x, torch::Tensor w, torch::Tensor bias, bool relu, int64_t splits,
                                int64_t tile) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kFloat);
  CHECK_DT(w, torch::kFloat);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && bias.size(0) == N, "shape mismatch");
  TORCH_CHECK(N % 4 == 0, "N must be a multiple of 4");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K % (16 * splits) == 0, "K must split into multiples of 16");
  TORCH_CHECK(splits * M * N < (1L << 31) && M * K < (1L << 31), "too large for int32 indexing");
  auto y = torch::empty({M, N}, x.options());
  if (M == 0) return y;
  auto part = torch::empty({splits, M, N}, x.options());
  const int64_t Ks = K / splits;
  auto zb = zero_f32(x.device(), N);
  ConvF32Args a{};
  a.x = x.data_ptr<float>();
  a.w = w.data_ptr<float>();
  a.bias = zb.data_ptr<float>();
  a.res = nullptr;
  a.y = part.data_ptr<float>();
  a.B = (int)M; a.H = 1; a.W = 1; a.C = (int)Ks; a.ldx = (int)K;
  a.Ho = 1; a.Wo = 1; a.Cout = (int)N; a.ldy = (int)N;
  a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
  a.M = (int)M;
  a.Kpad = (int)K;
  a.relu = 0;
  a.zero = zero_buffer(x.device()).data_ptr();
  a.ksplit = (int)splits;
  a.kslice = (int)Ks;
  a.ysplit = (long)(M * N);
  const int t = tile >= 0 ? (int)tile : conv_f32_pick((int)M, (int)N, (int)Ks, false);
  TORCH_CHECK(t != 101 || Ks % 32 == 0, "tile 101 needs K slices of 32");
  TORCH_CHECK(conv_f32_launch(a, 0, t, cur_stream()), "unknown / unsupported f32 conv tile id ", t);
  check_launch("linear_f32_splitk");
  splitk_reduce_launch(part.data_ptr<float>(), (int)splits, (long)(M * N), (int)N, bias.data_ptr<float>(),
                       relu ? 1 : 0, y.data_ptr(), true, cur_stream());
  check_launch("splitk_reduce");
  return y;
}

// Packed-row geometry of an RGB stem (conv_f32 mode 2 / conv_glds pack3,
// preprocess_pack3): nc row copies (the distinct 16-byte phases of 3*stride*ox
// for E = 16 / elem_bytes elements per chunk), wp elements each, cpk 16-byte
// chunks per kernel row.
static void pack3_geometry(int W, int KW, int stride, int pad, int elem_bytes, int& nc, int& wp, int& cpk) {
  const int E = 16 / elem_bytes;
  int g = 1;                                   // gcd(3 * stride, E), E a power of two
  while (g < E && (3 * stride) % (2 * g) == 0) g *= 2;
  nc = E / g;
  wp = (3 * (W + 2 * pad) + E - 1 + E - 1) / E * E;
  cpk = (3 * KW + E - 1) / E;
}

// RGB stem conv on packed rows: x3 [B, H, nc, wp] from preprocess_pack3 (fp32:
// conv_f32 mode 2 on the f32 MFMA; fp16: conv_glds pack3 on the f16 MFMA),
// w [Cout, nK * stage elements] (models/packed.py pack_conv_weight_p3), W = image width.
torch::Tensor conv2d_pack3(torch::Tensor x3, torch::Tensor w, torch::Tensor bias, int64_t W, int64_t KH,
                           int64_t KW, int64_t stride, int64_t pad, bool relu, int64_t tile) {
  CHECK_DEV(x3);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x3);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  const bool f16 = x3.scalar_type() == torch::kHalf;
  TORCH_CHECK(f16 || x3.scalar_type() == torch::kFloat, "x3 must be fp32 or fp16");
  TORCH_CHECK(w.scalar_type() == x3.scalar_type(), "w must have x3's dtype");
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x3.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x3.device() && bias.device() == x3.device(), "operands on different devices");
  TORCH_CHECK(KH >= 1 && KW >= 5 && stride >= 1 && pad >= 0 && W >= 1, "pack3 stem geometry: KW >= 5");
  int nc, wp, cpk;
  pack3_geometry((int)W, (int)KW, (int)stride, (int)pad, f16 ? 2 : 4, nc, wp, cpk);
  TORCH_CHECK(nc <= 4, "pack3 stem: stride needs at most 4 row copies");
  const int B = x3.size(0), H = x3.size(1);
  TORCH_CHECK(x3.size(2) == nc && x3.size(3) == wp, "x3 must be [B, H, ", nc, ", ", wp, "] (preprocess_pack3)");
  const int Cout = w.size(0), Kpad = w.size(1);
  // K stage = 16 fp32 / 64 fp16 elements = 4 / 8 chunks
  const int cps = f16 ? 8 : 4, nK = (KH * cpk + cps - 1) / cps;
  TORCH_CHECK(Kpad == nK * cps * (f16 ? 8 : 4), "pack3 weight must be [Cout, ", nK * cps * (f16 ? 8 : 4), "]");
  TORCH_CHECK(bias.size(0) == Cout && Cout % 4 == 0, "bias/Cout mismatch or Cout % 4");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = ((int)W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(M < (1L << 31) && (long)B * H * nc * wp < (1L << 31), "tensor too large for int32 indexing");
  auto y = torch::empty({B, Ho, Wo, Cout}, x3.options());
  if (M == 0) return y;
  if (f16) {
    ConvArgs a{};
    a.x = reinterpret_cast<const half_t*>(x3.data_ptr());
    a.w = reinterpret_cast<const half_t*>(w.data_ptr());
    a.bias = bias.data_ptr<float>();
    a.res = nullptr;
    a.y = y.data_ptr();
    a.B = B; a.H = H; a.W = (int)W; a.C = 3;
    a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = Cout;
    a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
    a.M = (int)M;
    a.Kpad = Kpad;
    a.relu = relu ? 1 : 0;
    a.nc = nc; a.wp = wp; a.cpk = cpk;
    a.zero = zero_buffer(x3.device()).data_ptr();
    const int t = tile >= 0 ? (int)tile : 27;
    TORCH_CHECK(conv_glds_launch(a, false, t, cur_stream()), "unsupported fp16 pack3 tile id ", t);
    check_launch("conv_glds_pack3");
    return y;
  }
  ConvF32Args a{};
  a.x = x3.data_ptr<float>();
  a.w = w.data_ptr<float>();
  a.bias = bias.data_ptr<float>();
  a.res = nullptr;
  a.y = y.data_ptr<float>();
  a.B = B; a.H = H; a.W = (int)W; a.C = 3;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = Cout;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.M = (int)M;
  a.Kpad = Kpad;
  a.relu = relu ? 1 : 0;
  a.nc = nc; a.wp = wp; a.cpk = cpk;
  a.zero = zero_buffer(x3.device()).data_ptr();
  const int t = tile >= 0 ? (int)tile : conv_f32_pick(a.M, Cout, Kpad, true);
  TORCH_CHECK(conv_f32_launch(a, 2, t, cur_stream()), "unknown / unsupported f32 conv tile id ", t);
  check_launch("conv_f32_pack3");
  return y;
}

// split-fp16 RGB stem on packed rows: x3 [B, H, 2*nc, wp] half (preprocess_pack3_split:
// nc hi copies, then nc lo copies), w [Cout, nK * 64] half (models/packed.py
// pack_split_weight_p3: per stage 32 K elements as [hi x32][lo x32]); fp32 output.
torch::Tensor conv2d_pack3_split(torch::Tensor x3, torch::Tensor w, torch::Tensor bias, int64_t W, int64_t KH,
                                 int64_t KW, int64_t stride, int64_t pad, bool relu, double acc_scale, int64_t tile) {
  CHECK_DEV(x3);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x3);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x3, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x3.dim() == 4 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  TORCH_CHECK(w.device() == x3.device() && bias.device() == x3.device(), "operands on different devices");
  TORCH_CHECK(KH >= 1 && KW >= 5 && stride >= 1 && pad >= 0 && W >= 1, "pack3 stem geometry: KW >= 5");
  int nc, wp, cpk;
  pack3_geometry((int)W, (int)KW, (int)stride, (int)pad, 2, nc, wp, cpk);
  TORCH_CHECK(nc <= 4, "pack3 stem: stride needs at most 4 row copies");
  const int B = x3.size(0), H = x3.size(1);
  TORCH_CHECK(x3.size(2) == 2 * nc && x3.size(3) == wp, "x3 must be [B, H, ", 2 * nc, ", ", wp,
              "] (preprocess_pack3_split)");
  const int Cout = w.size(0), Kpad = w.size(1);
  const int nK = (KH * cpk + 3) / 4;                 // 4 input chunks (32 halfs) per split stage
  TORCH_CHECK(Kpad == nK * 64, "split pack3 weight must be [Cout, ", nK * 64, "]");
  TORCH_CHECK(bias.size(0) == Cout && Cout % 64 == 0, "bias/Cout mismatch or Cout % 64");
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = ((int)W + 2 * pad - KW) / stride + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  const long M = (long)B * Ho * Wo;
  TORCH_CHECK(M < (1L << 31) && (long)B * H * 2 * nc * wp < (1L << 31) && M * Cout < (1L << 31),
              "tensor too large for int32 indexing");
  auto y = torch::empty({B, Ho, Wo, Cout}, x3.options().dtype(torch::kFloat));
  if (M == 0) return y;
  ConvArgs a{};
  a.x = reinterpret_cast<const half_t*>(x3.data_ptr());
  a.w = reinterpret_cast<const half_t*>(w.data_ptr());
  a.bias = bias.data_ptr<float>();
  a.res = nullptr;
  a.y = y.data_ptr();
  a.B = B; a.H = H; a.W = (int)W; a.C = 3;
  a.Ho = Ho; a.Wo = Wo; a.Cout = Cout; a.ldy = Cout;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad;
  a.M = (int)M;
  a.Kpad = Kpad;
  a.relu = relu ? 1 : 0;
  a.acc_scale = (float)acc_scale;
  a.nc = nc; a.wp = wp; a.cpk = cpk;
  a.zero = zero_buffer(x3.device()).data_ptr();
  const int t = tile >= 0 ? (int)tile : 27;
  TORCH_CHECK(conv_glds_split_p3_launch(a, t, cur_stream()), "unsupported split pack3 tile id ", t);
  check_launch("conv_glds_split_pack3");
  return y;
}


// fp32 Winograd F(2x2,3x3) conv (3x3 / stride 1 / pad 1): x [B,H,W,C] f32 NHWC,
// u [16, Cout, C] f32 (= G g G^T, models/packed.py wino_weight), y = act(conv + bias (+ res)).
torch::Tensor conv2d_wino_f32(torch::Tensor x, torch::Tensor u, torch::Tensor bias, c10::optional<torch::Tensor> res,
                              bool relu, int64_t variant) {
  CHECK_DEV(x);
  CHECK_DEV(u);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(u);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kFloat);
  CHECK_DT(u, torch::kFloat);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(u.device() == x.device() && bias.device() == x.device(), "operands on different devices");
  TORCH_CHECK(x.dim() == 4 && u.dim() == 3 && u.size(0) == 16 && bias.dim() == 1, "bad ranks / U must be [16, Cout, C]");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Cout = u.size(1);
  TORCH_CHECK(u.size(2) == C && bias.size(0) == Cout, "U / bias shape mismatch");
  TORCH_CHECK(C % 16 == 0 && Cout % 32 == 0, "winograd conv needs C % 16 == 0 and Cout % 32 == 0");
  TORCH_CHECK(conv_wino_f32_supported(H, W, C, Cout), "winograd conv: unsupported image size");
  TORCH_CHECK((long)B * H * W * std::max(C, Cout) < (1L << 31), "tensor too large for int32 indexing");
  auto y = torch::empty({B, H, W, Cout}, x.options());
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    auto& r = *res;
    CHECK_DEV(r);
    CHECK_CONTIG(r);
    CHECK_DT(r, torch::kFloat);
    TORCH_CHECK(r.device() == x.device(), "residual on a different device");
    TORCH_CHECK(r.dim() == 4 && r.size(0) == B && r.size(1) == H && r.size(2) == W && r.size(3) == Cout,
                "residual shape mismatch");
    rp = r.data_ptr<float>();
  }
  if (B == 0) return y;
  WinoArgs a{};
  a.x = x.data_ptr<float>();
  a.u = u.data_ptr<float>();
  a.bias = bias.data_ptr<float>();
  a.res = rp;
  a.y = y.data_ptr<float>();
  a.zero = zero_buffer(x.device()).data_ptr();
  a.B = B; a.H = H; a.W = W; a.C = C; a.Cout = Cout;
  a.relu = relu ? 1 : 0;
  a.ablate = 0;
  TORCH_CHECK(conv_wino_f32_launch(a, (int)variant, cur_stream()), "winograd conv launch rejected the shape");
  check_launch("conv_wino_f32");
  return y;
}

int64_t pick_tile_f32(int64_t M, int64_t Cout, int64_t K, bool small) {
  return conv_f32_pick((int)M, (int)Cout, (int)K, small);
}

// Per-device fp32 zeros (the bias of split-K partial GEMMs), grown on demand,
// never freed (same reasoning as zero_buffer).
static torch::Tensor zero_f32(const torch::Device& dev, int64_t n) {
  static std::mutex mu;
  static std::vector<torch::Tensor>* bufs = new std::vector<torch::Tensor>(64);
  const int i = dev.index() < 0 ? 0 : dev.index();
  TORCH_CHECK(i < 64, "device index out of range");
  std::lock_guard<std::mutex> lk(mu);
  static std::vector<torch::Tensor>* retired = new std::vector<torch::Tensor>();
  auto& b = (*bufs)[i];
  if (!b.defined() || b.numel() < n) {
    // a smaller buffer may still be read by queued kernels (other threads'
    // streams, captured graphs): keep it alive instead of returning it to the
    // caching allocator, where it could be reused while "zero"
    if (b.defined()) retired->push_back(b);
    b = torch::zeros({std::max<int64_t>(n, 4096)}, torch::TensorOptions().dtype(torch::kFloat).device(dev));
    (void)hipStreamSynchronize(cur_stream());
  }
  return b;
}

// y = act(x @ w.T + bias) with K split over `splits` partial GEMMs (the conv
// kernel as a 1x1 conv on a K-slice of each row: ldx = K, all slices in one
// launch) into fp32 partials, then one combine kernel.  For FC layers with few output tiles and a long K
// (AlexNet fc6-fc8 at batch 500: 64-256 tiles, K = 4096-9216) one tile per CU
// with 64-144 serial K stages cannot hide the DMA latency.
torch::Tensor linear_splitk(torch::Tensor x, torch::Tensor w, torch::Tensor bias, bool relu, bool out_f32,
                            int64_t splits, int64_t tile) {
  CHECK_DEV(x);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(x);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(x, torch::kHalf);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && bias.dim() == 1, "bad ranks");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && bias.size(0) == N, "shape mismatch");
  TORCH_CHECK(N % 4 == 0, "N must be a multiple of 4");
  TORCH_CHECK(splits >= 1 && splits <= 16 && K % (64 * splits) == 0, "K must split into multiples of 64");
  TORCH_CHECK(M * N < (1L << 31) && M * K < (1L << 31), "too large for int32 indexing");
  auto part = torch::empty({splits, M, N}, x.options().dtype(torch::kFloat));
  auto y = torch::empty({M, N}, x.options().dtype(out_f32 ? torch::kFloat : torch::kHalf));
  if (M == 0) return y;
  const int64_t Ks = K / splits;
  auto zb = zero_f32(x.device(), N);
  const void* zero = zero_buffer(x.device()).data_ptr();
  const half_t* xp = reinterpret_cast<const half_t*>(x.data_ptr());
  const half_t* wp = reinterpret_cast<const half_t*>(w.data_ptr());
  const int t = tile >= 10 ? (int)tile : conv_glds_pick((int)M, (int)N);
  {
    // all slices in ONE launch (grid = tiles x splits): one launch per slice kept
    // each slice at the unsplit block count and never paid (r1 A/B)
    ConvArgs a{};
    a.x = xp;
    a.w = wp;
    a.bias = zb.data_ptr<float>();
    a.res = nullptr;
    a.y = part.data_ptr<float>();
    a.B = (int)M; a.H = 1; a.W = 1; a.C = (int)Ks; a.ldx = (int)K;
    a.Ho = 1; a.Wo = 1; a.Cout = (int)N; a.ldy = (int)N;
    a.KH = 1; a.KW = 1; a.stride = 1; a.pad = 0;
    a.M = (int)M;
    a.Kpad = (int)K;
    a.relu = 0;
    a.zero = zero;
    a.ksplit = (int)splits;
    a.kslice = (int)Ks;
    a.ysplit = (long)(M * N);
    TORCH_CHECK(conv_glds_launch(a, true, t, cur_stream()), "unknown conv tile id ", t);
    check_launch("linear_splitk");
  }
  splitk_reduce_launch(part.data_ptr<float>(), (int)splits, (long)(M * N), (int)N, bias.data_ptr<float>(),
                       relu ? 1 : 0, y.data_ptr(), out_f32, cur_stream());
  check_launch("splitk_reduce");
  return y;
}

// uint8 [B,H,W,3] -> maxpool3x3/2(relu(conv7x7/2(normalise(img)) + bias)) : fp16 [B,Hp,Wp,64]
// Optional device-side window: with `start` (int64 GPU scalar) and batch > 0,
// `img` is a whole image shard [N,H,W,3] and images [*start, *start + batch)
// are used; the kernel clamps *start into [0, N - batch] so a bad descriptor
// can never read outside the shard.
// A window may be processed in parts: `window` (>= batch, default batch) is the
// clamping window, `sub` this launch's first image inside it (sub + batch <= window).
static const long long* window_args(const torch::Tensor& img, const c10::optional<torch::Tensor>& start, int64_t batch,
                                    int64_t window, int64_t sub, int& B, long long& max_start) {
  B = img.size(0);
  max_start = 0;
  if (!start.has_value() || !start->defined()) return nullptr;
  const auto& s = *start;
  CHECK_DEV(s);
  CHECK_DT(s, torch::kLong);
  TORCH_CHECK(s.numel() == 1, "start must be a 1-element int64 tensor");
  TORCH_CHECK(s.device() == img.device(), "start must live on the image device");
  TORCH_CHECK(batch > 0 && batch <= img.size(0), "window batch out of range");
  if (window <= 0) window = batch;
  TORCH_CHECK(window <= img.size(0) && sub >= 0 && sub + batch <= window, "window part out of range");
  B = (int)batch;
  max_start = img.size(0) - window;
  return reinterpret_cast<const long long*>(s.data_ptr());
}

// `start_offset` is subtracted from *start on the device: the window start may
// be a GLOBAL image index (e.g. straight from the broadcast query descriptor)
// and the offset the shard's first global index.
torch::Tensor stem_fused(torch::Tensor img, torch::Tensor w, torch::Tensor bias, c10::optional<torch::Tensor> start,
                         int64_t batch, int64_t start_offset, int64_t window, int64_t sub) {
  CHECK_DEV(img);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_CONTIG(img);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_DT(img, torch::kUInt8);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == 64 && w.size(1) == 7 * 32, "stem weight must be [64, 7*32] (small-C packing)");
  TORCH_CHECK(bias.numel() == 64, "bias must have 64 entries");
  const int H = img.size(1), W = img.size(2);
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  TORCH_CHECK(H >= 7 && W >= 7, "image too small");
  TORCH_CHECK((long)B * H * W * 3 < (1L << 31), "batch too large");
  const int Hc = (H + 6 - 7) / 2 + 1, Wc = (W + 6 - 7) / 2 + 1;
  const int Hp = (Hc + 2 - 3) / 2 + 1, Wp = (Wc + 2 - 3) / 2 + 1;
  auto y = torch::empty({B, Hp, Wp, 64}, img.options().dtype(torch::kHalf));
  if (B)
    stem_fused_launch(img.data_ptr<uint8_t>(), reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(),
                      reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, sp, start_offset, max_start, sp ? sub : 0, cur_stream()); check_launch("stem_fused");
  return y;
}

// uint8 [B,H,W,3] -> split-fp16 [B,Hp,Wp,128] = maxpool3x3/2(relu(conv7x7/2(normalise(img)) + bias)),
// fp32-accurate; (w, bias, psum, acc_scale) = models/packed.py pack_stem_split
// Fused split AlexNet stem (alex_stem.hip): uint8 [B, H, W, 3] (or a device-side window of
// a resident shard) -> split [B, Hp, Wp, 128] of conv 11x11/4 pad 2 + bias, ReLU, max pool 3x3/2.
torch::Tensor alex_stem_split(torch::Tensor img, torch::Tensor w, torch::Tensor bias, torch::Tensor psum,
                              double acc_scale, c10::optional<torch::Tensor> start, int64_t batch,
                              int64_t start_offset, int64_t window, int64_t sub) {
  CHECK_DEV(img);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_DEV(psum);
  CHECK_CONTIG(img);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_CONTIG(psum);
  CHECK_DT(img, torch::kUInt8);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  CHECK_DT(psum, torch::kFloat);
  TORCH_CHECK(w.device() == img.device() && bias.device() == img.device() && psum.device() == img.device(),
              "operands on different devices");
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(w.dim() == 3 && w.size(0) == 2 && w.size(1) == 64 && w.size(2) == 17 * 32,
              "split AlexNet stem weight must be [2, 64, 17*32]");
  TORCH_CHECK(bias.numel() == 64, "bias must have 64 entries");
  TORCH_CHECK(psum.numel() == 12 * 12 * 64, "psum must be [12, 12, 64]");
  const int H = img.size(1), W = img.size(2);
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  TORCH_CHECK(H >= 11 && W >= 11, "image too small");
  TORCH_CHECK((long)B * H * W * 3 < (1L << 31), "batch too large");
  const int Hc = (H + 4 - 11) / 4 + 1, Wc = (W + 4 - 11) / 4 + 1;
  const int Hp = (Hc - 3) / 2 + 1, Wp = (Wc - 3) / 2 + 1;
  TORCH_CHECK(Hc >= 3 && Wc >= 3, "image too small for the pool");
  TORCH_CHECK((long)B * Hp * Wp * 128 < (1L << 31), "batch too large");
  auto y = torch::empty({B, Hp, Wp, 128}, img.options().dtype(torch::kHalf));
  if (B) {
    TORCH_CHECK(alex_stem_split_launch(img.data_ptr<uint8_t>(), reinterpret_cast<const half_t*>(w.data_ptr()),
                                       bias.data_ptr<float>(), psum.data_ptr<float>(), (float)acc_scale,
                                       reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, sp, start_offset, max_start,
                                       sp ? sub : 0, split_guard_for(img.device()), cur_stream()),
                "alex stem: bad geometry");
    check_launch("alex_stem_split");
  }
  return y;
}

torch::Tensor alex_stem_u8_f16(torch::Tensor img, torch::Tensor w, torch::Tensor bias, torch::Tensor psum,
                              double acc_scale, c10::optional<torch::Tensor> start, int64_t batch,
                              int64_t start_offset, int64_t window, int64_t sub) {
  CHECK_DEV(img);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_DEV(psum);
  CHECK_CONTIG(img);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_CONTIG(psum);
  CHECK_DT(img, torch::kUInt8);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  CHECK_DT(psum, torch::kFloat);
  TORCH_CHECK(w.device() == img.device() && bias.device() == img.device() && psum.device() == img.device(),
              "operands on different devices");
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(w.dim() == 3 && w.size(0) == 2 && w.size(1) == 64 && w.size(2) == 17 * 32,
              "split AlexNet stem weight must be [2, 64, 17*32]");
  TORCH_CHECK(bias.numel() == 64, "bias must have 64 entries");
  TORCH_CHECK(psum.numel() == 12 * 12 * 64, "psum must be [12, 12, 64]");
  const int H = img.size(1), W = img.size(2);
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  TORCH_CHECK(H >= 11 && W >= 11, "image too small");
  TORCH_CHECK((long)B * H * W * 3 < (1L << 31), "batch too large");
  const int Hc = (H + 4 - 11) / 4 + 1, Wc = (W + 4 - 11) / 4 + 1;
  const int Hp = (Hc - 3) / 2 + 1, Wp = (Wc - 3) / 2 + 1;
  TORCH_CHECK(Hc >= 3 && Wc >= 3, "image too small for the pool");
  TORCH_CHECK((long)B * Hp * Wp * 128 < (1L << 31), "batch too large");
  auto y = torch::empty({B, Hp, Wp, 64}, img.options().dtype(torch::kHalf));
  if (B) {
    TORCH_CHECK(alex_stem_u8_f16_launch(img.data_ptr<uint8_t>(), reinterpret_cast<const half_t*>(w.data_ptr()),
                                        bias.data_ptr<float>(), psum.data_ptr<float>(), (float)acc_scale,
                                        reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, sp, start_offset, max_start,
                                        sp ? sub : 0, cur_stream()),
                "alex stem: bad geometry");
    check_launch("alex_stem_u8_f16");
  }
  return y;
}

torch::Tensor stem_split(torch::Tensor img, torch::Tensor w, torch::Tensor bias, torch::Tensor psum, double acc_scale,
                         c10::optional<torch::Tensor> start, int64_t batch, int64_t start_offset, int64_t window,
                         int64_t sub) {
  CHECK_DEV(img);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_DEV(psum);
  CHECK_CONTIG(img);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_CONTIG(psum);
  CHECK_DT(img, torch::kUInt8);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  CHECK_DT(psum, torch::kFloat);
  TORCH_CHECK(w.device() == img.device() && bias.device() == img.device() && psum.device() == img.device(),
              "operands on different devices");
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(w.dim() == 3 && w.size(0) == 2 && w.size(1) == 64 && w.size(2) == 7 * 32,
              "split stem weight must be [2, 64, 7*32]");
  TORCH_CHECK(bias.numel() == 64, "bias must have 64 entries");
  TORCH_CHECK(psum.numel() == 8 * 8 * 64, "psum must be [8, 8, 64]");
  const int H = img.size(1), W = img.size(2);
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  TORCH_CHECK(H >= 7 && W >= 7, "image too small");
  TORCH_CHECK((long)B * H * W * 3 < (1L << 31), "batch too large");
  const int Hc = (H + 6 - 7) / 2 + 1, Wc = (W + 6 - 7) / 2 + 1;
  const int Hp = (Hc + 2 - 3) / 2 + 1, Wp = (Wc + 2 - 3) / 2 + 1;
  TORCH_CHECK((long)B * Hp * Wp * 128 < (1L << 31), "batch too large");
  auto y = torch::empty({B, Hp, Wp, 128}, img.options().dtype(torch::kHalf));
  if (B) {
    stem_split_launch(img.data_ptr<uint8_t>(), reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(),
                      psum.data_ptr<float>(), (float)acc_scale, reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, sp,
                      start_offset, max_start, sp ? sub : 0, split_guard_for(img.device()), cur_stream());
    check_launch("stem_split");
  }
  return y;
}

// fp16 programs: exact-u8 stem (pack_stem_split weights, hi parts only) -> fp16 [B,Hp,Wp,64]
torch::Tensor stem_u8_f16(torch::Tensor img, torch::Tensor w, torch::Tensor bias, torch::Tensor psum, double acc_scale,
                         c10::optional<torch::Tensor> start, int64_t batch, int64_t start_offset, int64_t window,
                         int64_t sub) {
  CHECK_DEV(img);
  CHECK_DEV(w);
  CHECK_DEV(bias);
  CHECK_DEV(psum);
  CHECK_CONTIG(img);
  CHECK_CONTIG(w);
  CHECK_CONTIG(bias);
  CHECK_CONTIG(psum);
  CHECK_DT(img, torch::kUInt8);
  CHECK_DT(w, torch::kHalf);
  CHECK_DT(bias, torch::kFloat);
  CHECK_DT(psum, torch::kFloat);
  TORCH_CHECK(w.device() == img.device() && bias.device() == img.device() && psum.device() == img.device(),
              "operands on different devices");
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(w.dim() == 3 && w.size(0) == 2 && w.size(1) == 64 && w.size(2) == 7 * 32,
              "split stem weight must be [2, 64, 7*32]");
  TORCH_CHECK(bias.numel() == 64, "bias must have 64 entries");
  TORCH_CHECK(psum.numel() == 8 * 8 * 64, "psum must be [8, 8, 64]");
  const int H = img.size(1), W = img.size(2);
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  TORCH_CHECK(H >= 7 && W >= 7, "image too small");
  TORCH_CHECK((long)B * H * W * 3 < (1L << 31), "batch too large");
  const int Hc = (H + 6 - 7) / 2 + 1, Wc = (W + 6 - 7) / 2 + 1;
  const int Hp = (Hc + 2 - 3) / 2 + 1, Wp = (Wc + 2 - 3) / 2 + 1;
  TORCH_CHECK((long)B * Hp * Wp * 64 < (1L << 31), "batch too large");
  auto y = torch::empty({B, Hp, Wp, 64}, img.options().dtype(torch::kHalf));
  if (B) {
    stem_u8_f16_launch(img.data_ptr<uint8_t>(), reinterpret_cast<const half_t*>(w.data_ptr()), bias.data_ptr<float>(),
                       psum.data_ptr<float>(), (float)acc_scale, reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, sp,
                       start_offset, max_start, sp ? sub : 0, cur_stream());
    check_launch("stem_u8_f16");
  }
  return y;
}

torch::Tensor preprocess(torch::Tensor img, c10::optional<torch::Tensor> start, int64_t batch, int64_t start_offset,
                         int64_t window, int64_t sub, bool f32) {
  CHECK_DEV(img);
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  auto out = torch::empty({B, img.size(1), img.size(2), 4}, img.options().dtype(f32 ? torch::kFloat : torch::kHalf));
  const long npix = (long)B * img.size(1) * img.size(2);
  if (!npix) return out;
  if (f32) {
    preprocess_f32_launch(img.data_ptr<uint8_t>(), out.data_ptr<float>(), npix, sp, start_offset, max_start,
                          sp ? sub : 0, (long)img.size(1) * img.size(2), cur_stream());
    check_launch("preprocess_f32");
    return out;
  }
  preprocess_launch(img.data_ptr<uint8_t>(), reinterpret_cast<half_t*>(out.data_ptr()), npix, sp, start_offset, max_start, sp ? sub : 0,
                    (long)img.size(1) * img.size(2), cur_stream()); check_launch("preprocess");
  return out;
}

// uint8 [B, H, W, 3] -> packed-row fp32 stem input [B, H, nc, wp] for a KW-wide,
// stride-`stride`, pad-`pad` stem (conv2d_pack3_f32); same window arguments as preprocess.
torch::Tensor preprocess_pack3(torch::Tensor img, int64_t KW, int64_t stride, int64_t pad,
                               c10::optional<torch::Tensor> start, int64_t batch, int64_t start_offset,
                               int64_t window, int64_t sub, bool f16) {
  CHECK_DEV(img);
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(KW >= 5 && stride >= 1 && pad >= 0, "pack3 stem geometry: KW >= 5");
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  const int H = img.size(1), W = img.size(2);
  int nc, wp, cpk;
  pack3_geometry(W, (int)KW, (int)stride, (int)pad, f16 ? 2 : 4, nc, wp, cpk);
  TORCH_CHECK(nc <= 4, "pack3 stem: stride needs at most 4 row copies");
  TORCH_CHECK((long)B * H * nc * wp < (1L << 31), "tensor too large for int32 indexing");
  auto out = torch::empty({B, H, nc, wp}, img.options().dtype(f16 ? torch::kHalf : torch::kFloat));
  if (B == 0) return out;
  if (f16)
    preprocess_pack3_f16_launch(img.data_ptr<uint8_t>(), reinterpret_cast<half_t*>(out.data_ptr()), B, H, W,
                                (int)pad, nc, wp, sp, start_offset, max_start, sp ? sub : 0, cur_stream());
  else
    preprocess_pack3_f32_launch(img.data_ptr<uint8_t>(), out.data_ptr<float>(), B, H, W, (int)pad, nc, wp, sp,
                                start_offset, max_start, sp ? sub : 0, cur_stream());
  check_launch("preprocess_pack3_f32");
  return out;
}

// uint8 HWC -> split-fp16 packed-row stem input [B, H, 2*nc, wp] (hi copies, lo copies)
torch::Tensor preprocess_pack3_split(torch::Tensor img, int64_t KW, int64_t stride, int64_t pad,
                                     c10::optional<torch::Tensor> start, int64_t batch, int64_t start_offset,
                                     int64_t window, int64_t sub) {
  CHECK_DEV(img);
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  TORCH_CHECK(KW >= 5 && stride >= 1 && pad >= 0, "pack3 stem geometry: KW >= 5");
  int B;
  long long max_start;
  const long long* sp = window_args(img, start, batch, window, sub, B, max_start);
  const int H = img.size(1), W = img.size(2);
  int nc, wp, cpk;
  pack3_geometry(W, (int)KW, (int)stride, (int)pad, 2, nc, wp, cpk);
  TORCH_CHECK(nc <= 4, "pack3 stem: stride needs at most 4 row copies");
  TORCH_CHECK((long)B * H * 2 * nc * wp < (1L << 31), "tensor too large for int32 indexing");
  auto out = torch::empty({B, H, 2 * nc, wp}, img.options().dtype(torch::kHalf));
  if (B == 0) return out;
  preprocess_pack3_split_launch(img.data_ptr<uint8_t>(), reinterpret_cast<half_t*>(out.data_ptr()), B, H, W,
                                (int)pad, nc, wp, sp, start_offset, max_start, sp ? sub : 0, cur_stream());
  check_launch("preprocess_pack3_split");
  return out;
}

torch::Tensor resize_crop(torch::Tensor img, int64_t resize, int64_t crop) {
  CHECK_DEV(img);
  CHECK_CONTIG(img);
  CHECK_DT(img, torch::kUInt8);
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3, "img must be [B, H, W, 3] uint8");
  const int B = img.size(0), Hi = img.size(1), Wi = img.size(2);
  int Hr, Wr;
  if (Hi <= Wi) {
    Hr = resize;
    Wr = (int)((long)resize * Wi / Hi);
  } else {
    Wr = resize;
    Hr = (int)((long)resize * Hi / Wi);
  }
  TORCH_CHECK(Hr >= crop && Wr >= crop, "crop larger than resized image");
  auto out = torch::empty({B, crop, crop, 4}, img.options().dtype(torch::kHalf));
  if (B) resize_crop_launch(img.data_ptr<uint8_t>(), reinterpret_cast<half_t*>(out.data_ptr()), B, Hi, Wi, Hr, Wr,
                            crop, cur_stream()); check_launch("resize_crop");
  return out;
}

torch::Tensor maxpool2d_nhwc(torch::Tensor x, int64_t k, int64_t s, int64_t pad, c10::optional<torch::Tensor> out) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  const bool f32 = x.scalar_type() == torch::kFloat;
  TORCH_CHECK(f32 || x.scalar_type() == torch::kHalf, "x must be fp16 or fp32");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % (f32 ? 4 : 8) == 0, "x must be [B,H,W,C] with C % 8 (fp16) / 4 (fp32) == 0");
  TORCH_CHECK(k >= 1 && s >= 1 && pad >= 0 && 2 * pad <= k, "bad pool geometry");
  const int B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty output");
  torch::Tensor y;
  if (out.has_value() && out->defined()) {        // e.g. a batch slice of a larger tensor
    y = *out;
    CHECK_DEV(y);
    CHECK_CONTIG(y);
    TORCH_CHECK(y.scalar_type() == x.scalar_type() && y.device() == x.device(), "out dtype/device mismatch");
    TORCH_CHECK(y.dim() == 4 && y.size(0) == B && y.size(1) == Ho && y.size(2) == Wo && y.size(3) == C,
                "out shape mismatch");
  } else {
    y = torch::empty({B, Ho, Wo, C}, x.options());
  }
  if (!B) return y;
  if (f32) {
    maxpool_f32_launch(x.data_ptr<float>(), y.data_ptr<float>(), B, H, W, C, Ho, Wo, k, s, pad, cur_stream());
    check_launch("maxpool_f32");
    return y;
  }
  maxpool_launch(reinterpret_cast<const half_t*>(x.data_ptr()), reinterpret_cast<half_t*>(y.data_ptr()), B, H, W, C,
                 Ho, Wo, k, s, pad, cur_stream()); check_launch("maxpool");
  return y;
}

torch::Tensor global_avgpool_nhwc(torch::Tensor x) {
  CHECK_DEV(x);
  CHECK_CONTIG(x);
  const bool f32 = x.scalar_type() == torch::kFloat;
  TORCH_CHECK(f32 || x.scalar_type() == torch::kHalf, "x must be fp16 or fp32");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % (f32 ? 4 : 8) == 0, "x must be [B,H,W,C] with C % 8 (fp16) / 4 (fp32) == 0");
  const int B = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = torch::empty({B, C}, x.options());
  if (!B) return y;
  if (f32) {
    avgpool_f32_launch(x.data_ptr<float>(), y.data_ptr<float>(), B, HW, C, cur_stream());
    check_launch("avgpool_f32");
    return y;
  }
  avgpool_launch(reinterpret_cast<const half_t*>(x.data_ptr()), reinterpret_cast<half_t*>(y.data_ptr()), B, HW, C,
                 cur_stream()); check_launch("avgpool");
  return y;
}

// Optional `packed` [>= rows, 2] int32: also write (class, prob bits) pairs there
// (the data plane's gather send buffer, so no repack kernel runs afterwards).
std::vector<torch::Tensor> softmax_top1(torch::Tensor logits, c10::optional<torch::Tensor> packed,
                                        c10::optional<torch::Tensor> ovf) {
  CHECK_DEV(logits);
  CHECK_DT(logits, torch::kFloat);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [rows, N] with unit column stride");
  const int rows = logits.size(0), N = logits.size(1), ld = logits.stride(0);
  auto cls = torch::empty({rows}, logits.options().dtype(torch::kInt));
  auto prob = torch::empty({rows}, logits.options());
  int* pk = nullptr;
  if (packed.has_value() && packed->defined()) {
    auto& p = *packed;
    CHECK_DEV(p);
    CHECK_CONTIG(p);
    CHECK_DT(p, torch::kInt);
    TORCH_CHECK(p.device() == logits.device(), "packed must live on the logits device");
    TORCH_CHECK(p.dim() == 2 && p.size(1) == 2 && p.size(0) >= rows, "packed must be [>= rows, 2] int32");
    pk = p.data_ptr<int>();
  }
  const int* of = nullptr;
  if (ovf.has_value() && ovf->defined()) {
    auto& f = *ovf;
    CHECK_DEV(f);
    CHECK_DT(f, torch::kInt);
    TORCH_CHECK(f.device() == logits.device() && f.numel() >= 1, "ovf must be an int32 flag on the logits device");
    of = f.data_ptr<int>();
  }
  if (rows) softmax_top1_launch(logits.data_ptr<float>(), ld, N, rows, cls.data_ptr<int>(), prob.data_ptr<float>(),
                                pk, of, cur_stream()); check_launch("softmax_top1");
  return {cls, prob};
}

// hipGraphLaunch of an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec())
// on the current stream, and nothing else: the round paths replay one graph per
// chunk and must not wait on the device in between (HipRunner._replayer).
void graph_launch(int64_t exec) {
  TORCH_CHECK(exec != 0, "graph_launch: no instantiated graph");
  const hipError_t e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), cur_stream());
  TORCH_CHECK(e == hipSuccess, "hipGraphLaunch failed: ", hipGetErrorString(e));
}

torch::Tensor synth_images(int64_t seed, int64_t start, int64_t n, int64_t hw, torch::Device dev) {
  TORCH_CHECK(dev.is_cuda(), "synth_images needs a GPU device");
  TORCH_CHECK(n >= 0 && start >= 0 && (hw * hw * 3) % 8 == 0, "bad synth_images args");
  auto out = torch::empty({n, hw, hw, 3}, torch::TensorOptions().dtype(torch::kUInt8).device(dev));
  if (n) synth_images_launch(out.data_ptr<uint8_t>(), (uint64_t)seed, start, n, hw * hw * 3, cur_stream()); check_launch("synth_images");
  return out;
}

int64_t pick_tile(int64_t M, int64_t Cout) { return conv_glds_pick((int)M, (int)Cout); }

namespace idunno {
std::vector<double> stage_file_native(const std::string& path, torch::Tensor out, std::vector<torch::Tensor> pinned,
                                      int64_t stream, int64_t nthreads);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "IDunno-MI355X native HIP kernels (gfx950)";
  m.def("conv1x1_dual", &conv1x1_dual, "bottleneck expansion 1x1 + 1x1 downsample as one GEMM (fp16)",
        py::arg("x1"), py::arg("x2"), py::arg("w"), py::arg("bias"), py::arg("stride"), py::arg("relu"));
  m.def("conv1x1_dual_ok", &conv1x1_dual_ok, "whether conv1x1_dual supports (K1, K2, Cout, M)");
  m.def("conv1x1_fused_next", &conv1x1_fused_next, "bottleneck tail + next block's reduce 1x1 in one pass (fp16)",
        py::arg("x1"), py::arg("x2"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("w2"), py::arg("b2"),
        py::arg("stride"), py::arg("relu"));
  m.def("conv1x1_fused_next_ok", &conv1x1_fused_next_ok, "whether conv1x1_fused_next supports (K1, K2, N, N2, M)");
  m.def("conv1x1_dual_split", &conv1x1_dual_split, "split (fp32-accurate) form of conv1x1_dual", py::arg("x1"),
        py::arg("x2"), py::arg("w"), py::arg("bias"), py::arg("acc_scale"), py::arg("stride"), py::arg("relu"));
  m.def("conv1x1_dual_split_ok", &conv1x1_dual_split_ok, "whether conv1x1_dual_split supports (K1, K2, Cout, M)");
  m.def("conv2d_nhwc", &conv2d_nhwc, "implicit-GEMM MFMA conv + bias (+res) (+relu)", py::arg("x"), py::arg("w"),
        py::arg("bias"), py::arg("res"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("relu"), py::arg("out_f32") = false, py::arg("tile") = -1, py::arg("out") = py::none(),
        py::arg("ksplit") = -1, py::arg("route") = 0);
  m.def("linear_splitk", &linear_splitk, "FC layer with split-K partial GEMMs + combine", py::arg("x"),
        py::arg("w"), py::arg("bias"), py::arg("relu"), py::arg("out_f32"), py::arg("splits"), py::arg("tile") = -1);
  m.def("conv2d_split", &conv2d_split, "split-fp16 (fp32-accurate) conv: 3 f16 MFMAs per 32 channels",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("pad"), py::arg("relu"), py::arg("acc_scale"), py::arg("out_f32") = false, py::arg("tile") = -1,
        py::arg("out") = py::none(), py::arg("ksplit") = -1, py::arg("route") = 0);
  m.def("conv2d_split_dual", &conv2d_split_dual,
        "two split convs of one input in one launch (downsample as the centre tap of the 3x3/s conv)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("relu"), py::arg("acc_scale"), py::arg("acc_scale2"), py::arg("nsplit"), py::arg("center_only"),
        py::arg("tile") = -1);
  m.def("conv2d_pack3_split", &conv2d_pack3_split, "split-fp16 RGB stem conv on packed rows, fp32 out",
        py::arg("x3"), py::arg("w"), py::arg("bias"), py::arg("W"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("pad"), py::arg("relu"), py::arg("acc_scale"), py::arg("tile") = -1);
  m.def("preprocess_pack3_split", &preprocess_pack3_split, "uint8 HWC -> split-fp16 packed-row stem input",
        py::arg("img"), py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("start") = py::none(),
        py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1, py::arg("sub") = 0);
  m.def("stem_u8_f16", &stem_u8_f16, "fp16 fused ResNet stem in exact-u8 form (pack_stem_split weights)",
        py::arg("img"), py::arg("w"), py::arg("bias"), py::arg("psum"), py::arg("acc_scale"), py::arg("start") = py::none(),
        py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1, py::arg("sub") = 0);
  m.def("stem_split", &stem_split, "fp32-accurate fused split-fp16 ResNet stem (normalise+conv7x7/2+relu+maxpool)",
        py::arg("img"), py::arg("w"), py::arg("bias"), py::arg("psum"), py::arg("acc_scale"), py::arg("start") = py::none(),
        py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1, py::arg("sub") = 0);
  m.def("linear_split", &linear_split, "fp32-accurate FC on split fp16, split-K in one launch + combine",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("acc_scale"), py::arg("relu"), py::arg("out_f32"),
        py::arg("splits"), py::arg("tile") = -1);
  m.def("conv3x3_band_split", &conv3x3_band_split,
        "band-staged split 3x3/s1/p1 conv (tile 70) with a persistent-grid cap (0: one workgroup per CU)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res") = py::none(), py::arg("relu") = true,
        py::arg("acc_scale") = 1.0, py::arg("out_f32") = false, py::arg("max_grid") = 0, py::arg("flags") = 0);
  m.def("conv3x3_band_f16", &conv3x3_band_f16,
        "band-staged fp16 3x3/s1/p1 conv (tile 70) with a persistent-grid cap (0: one workgroup per CU)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("relu"), py::arg("max_grid") = 0);
  m.def("conv3x3_band_tiles", &conv3x3_band_tiles, "band conv tile count for (B, W, Cout)");
  m.def("split_from_f32", &split_from_f32, "fp32 NHWC -> split-fp16 layout");
  m.def("f32_from_split", &f32_from_split, "split-fp16 layout -> fp32 NHWC");
  m.def("maxpool2d_split", &maxpool2d_split, "NHWC max pool (fp32 or split in) -> split out", py::arg("x"),
        py::arg("k"), py::arg("s"), py::arg("pad"), py::arg("out") = py::none());
  m.def("set_astem_ahead", &set_astem_ahead);
  m.def("set_astem_f16_two_wg", &set_astem_f16_two_wg);
  m.def("alex_stem_u8_f16", &alex_stem_u8_f16, "fp16 fused AlexNet stem (exact-u8 form, hi MFMA only)",
        py::arg("img"), py::arg("w"), py::arg("bias"), py::arg("psum"), py::arg("acc_scale"),
        py::arg("start") = py::none(), py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1,
        py::arg("sub") = 0);
  m.def("set_astem_variant", &set_astem_variant);
  m.def("set_astem_phased", &set_astem_phased);
  m.def("set_stem_prewait", &set_stem_prewait);
  m.def("alex_stem_split", &alex_stem_split, "fused split AlexNet stem (conv 11x11/4 + ReLU + max pool 3x3/2)",
        py::arg("img"), py::arg("w"), py::arg("bias"), py::arg("psum"), py::arg("acc_scale"),
        py::arg("start") = py::none(), py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1,
        py::arg("sub") = 0);
  m.def("pick_tile_split", &pick_tile_split, "split conv tile heuristic for (M, Cout)");
  m.def("conv2d_nhwc_f32", &conv2d_nhwc_f32, "fp32 implicit-GEMM conv on f32 MFMA + bias (+res) (+relu)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("res"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("pad"), py::arg("relu"), py::arg("tile") = -1, py::arg("out") = py::none());
  m.def("linear_f32_splitk", &linear_f32_splitk, "fp32 FC with split-K in one launch + combine", py::arg("x"),
        py::arg("w"), py::arg("bias"), py::arg("relu"), py::arg("splits"), py::arg("tile") = -1);
  m.def("conv2d_pack3", &conv2d_pack3, "RGB stem conv on packed rows (preprocess_pack3), fp32 or fp16 + bias (+relu)",
        py::arg("x3"), py::arg("w"), py::arg("bias"), py::arg("W"), py::arg("KH"), py::arg("KW"), py::arg("stride"),
        py::arg("pad"), py::arg("relu"), py::arg("tile") = -1);
  m.def("preprocess_pack3", &preprocess_pack3, "uint8 HWC -> packed-row fp32 stem input [B, H, nc, wp]",
        py::arg("img"), py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("start") = py::none(),
        py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1, py::arg("sub") = 0,
        py::arg("f16") = false);
  m.def("conv2d_wino_f32", &conv2d_wino_f32, "fp32 Winograd F(2x2,3x3) conv (3x3/s1/p1) + bias (+res) (+relu)",
        py::arg("x"), py::arg("u"), py::arg("bias"), py::arg("res"), py::arg("relu"), py::arg("variant") = 0);
  m.def("wino_supported", &conv_wino_f32_supported, "winograd conv geometry fits (H, W, C, Cout)");
  m.def("pick_tile_f32", &pick_tile_f32, "tile id the f32 conv heuristic picks for (M, Cout, K, small)");
  m.def("preprocess", &preprocess, "uint8 HWC -> normalised fp16 (or fp32) NHWC4", py::arg("img"),
        py::arg("start") = py::none(), py::arg("batch") = -1, py::arg("start_offset") = 0, py::arg("window") = -1,
        py::arg("sub") = 0, py::arg("f32") = false);
  m.def("stem_fused", &stem_fused, "fused normalise + conv7x7/2 + bias + relu + maxpool3x3/2 (ResNet stem)",
        py::arg("img"), py::arg("w"), py::arg("bias"), py::arg("start") = py::none(), py::arg("batch") = -1,
        py::arg("start_offset") = 0, py::arg("window") = -1, py::arg("sub") = 0);
  m.def("resize_crop", &resize_crop, "bilinear resize + centre crop + normalise");
  m.def("maxpool2d_nhwc", &maxpool2d_nhwc, "NHWC max pool (into ``out`` when given)", py::arg("x"), py::arg("k"),
        py::arg("s"), py::arg("pad"), py::arg("out") = py::none());
  m.def("global_avgpool_nhwc", &global_avgpool_nhwc, "NHWC global average pool");
  m.def("softmax_top1", &softmax_top1, "fused row softmax + argmax; a set ``ovf`` flag marks every row -2",
        py::arg("logits"), py::arg("packed") = py::none(), py::arg("ovf") = py::none());
  m.def("set_split_guard", &set_split_guard,
        "split range guard flag (int32 device tensor) for this thread's split launches; None = off",
        py::arg("flag") = py::none());
  m.def("synth_images", &synth_images, "deterministic synthetic uint8 images [n,hw,hw,3]");
  m.def("stage_file_native", &idunno::stage_file_native,
        "host -> HBM staging of a file's bytes into `out` through pinned ping-pong buffers on `stream`, "
        "parallel pread(2) with the GIL released (runtime/staging.cpp)",
        py::arg("path"), py::arg("out"), py::arg("pinned"), py::arg("stream"), py::arg("nthreads") = 8);
  m.def("graph_launch", &graph_launch, "hipGraphLaunch(exec, current stream): a replay without any host wait");
  m.def("pick_tile", &pick_tile, "tile id the conv heuristic picks for (M, Cout)");
}
