// Inference path of the reference's inference.py:
//
//   preprocess_image (inference.py:28-46): cv2.resize(frame, (256,128)) with the
//     default INTER_LINEAR on the uint8 BGR frame, cv2.cvtColor(BGR2RGB),
//     transforms.ToTensor() (/255) and transforms.Normalize(ImageNet mean/std)
//     -> seg_preprocess_bgr writes the model's NHWC4 input rows directly;
//   model.eval() forward (inference.py:25,162-163) with every BatchNorm folded
//     into its conv (seg_bn_fold_batch; the convs then apply bias + activation in
//     their epilogues: seg_conv_igemm_act, seg_dw_fwd_bias_act);
//   overlay_predictions' torch.max(prediction, dim=1) + cv2.resize(...,
//     INTER_NEAREST) back to the frame size (inference.py:64-70) fused with the
//     model's final align_corners=True upsample (src/unet.py:30,49) ->
//     seg_argmax_nearest writes the uint8 class mask at frame resolution; the
//     full-resolution logits are never stored.
//
// cv2 is not installed in this image, so the resize arithmetic is a restatement
// of OpenCV's published INTER_LINEAR 8-bit path (imgproc/src/resize.cpp):
//   x: fx = float((dx+0.5)*scale_x - 0.5), sx = floor(fx), fx -= sx; sx < 0 ->
//      (sx, fx) = (0, 0); sx >= W-1 -> (W-1, 0); alpha = round((1-fx)*2048),
//      round(fx*2048) (cvRound: half to even)
//   y: same fy/sy without clamping; source rows clip(sy, 0, H-1), clip(sy+1, ...)
//   horizontal: D = S[sx]*a0 + S[sx+1]*a1                      (int32, exact)
//   vertical (VResizeLinearVec_32s8u, the SIMD path every full row takes):
//      out = sat_u8((((D0 >> 4) * b0 >> 16) + ((D1 >> 4) * b1 >> 16) + 2) >> 2)
// and INTER_NEAREST: sx = min(floor(x * (1 / (dst_w / src_w))), src_w - 1) in
// double.  Parity of these two against real cv2 is unpinned (oracle/cvresize.py
// restates the same arithmetic; tests pin kernel == restatement bit-exactly).
#include "common.h"

#ifndef SEG_ARGMAX_BAND
#define SEG_ARGMAX_BAND 1
#endif

namespace {

// ---------------------------------------------------------------- BN folding
struct SegFoldJob {
  const float* w;      // conv weight [Cout][kper]
  const float* bias;   // conv bias [Cout] or null
  const float* gamma;  // BN weight/bias/running stats [Cout] (gamma null: no BN -> copy)
  const float* beta;
  const float* rm;
  const float* rv;
  float* w_out;        // [Cout][kper]
  float* b_out;        // [Cout] (padded to a multiple of 4 by the caller; pad left untouched)
  int cout, kper;
  float eps;
  int pad_;
};
static_assert(sizeof(SegFoldJob) == 80, "seg_fold_job ABI");

// w' = w * g/sqrt(rv+eps); b' = b * g/sqrt(rv+eps) + (beta - rm*g/sqrt(rv+eps)): the
// eval BatchNorm y*scale + shift of seg_bn_eval_coef pushed through the conv.
__global__ __launch_bounds__(256) void fold_batch_kernel(const SegFoldJob* __restrict__ jobs) {
  const SegFoldJob j = jobs[blockIdx.y];
  const long total = (long)j.cout * j.kper;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total + j.cout; i += (long)gridDim.x * 256) {
    const int co = i < total ? (int)(i / j.kper) : (int)(i - total);
    float scale = 1.f, shift = 0.f;
    if (j.gamma) {
      const float inv = 1.f / sqrtf(j.rv[co] + j.eps);
      const float g = j.gamma[co];
      scale = g * inv;
      shift = j.beta[co] - j.rm[co] * g * inv;
    }
    if (i < total) {
      j.w_out[i] = j.gamma ? j.w[i] * scale : j.w[i];
    } else {
      const float b = j.bias ? j.bias[co] : 0.f;
      j.b_out[co] = j.gamma ? b * scale + shift : b;
    }
  }
}

// ---------------------------------------------------------------- preprocess
// Model pixel (dy, dx) of one frame: cv2.resize INTER_LINEAR (fixed-point weights, OpenCV's rounding),
// BGR -> RGB, ToTensor, Normalize (inference.py:28-46); channel 3 = 0.
__device__ __forceinline__ f32x4 pre_pixel(const uint8_t* __restrict__ fr, long row_bytes, int Hf, int Wf, int dy,
                                           int dx, double scale_x, double scale_y, float m0, float m1, float m2,
                                           float s0, float s1, float s2) {
#pragma clang fp contract(off)  // OpenCV computes (dx+0.5)*scale-0.5 as a separate multiply and subtract
  // x taps and fixed-point weights
  float fx = (float)((dx + 0.5) * scale_x - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { sx = 0; fx = 0.f; }
  if (sx >= Wf - 1) { sx = Wf - 1; fx = 0.f; }
  const int a0 = (int)rintf((1.f - fx) * 2048.f), a1 = (int)rintf(fx * 2048.f);
  const int sx1 = sx + 1 < Wf ? sx + 1 : Wf - 1;  // a1 == 0 whenever sx + 1 is outside
  // y taps (weights from the unclamped fy; rows clipped)
  float fy = (float)((dy + 0.5) * scale_y - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const int b0 = (int)rintf((1.f - fy) * 2048.f), b1 = (int)rintf(fy * 2048.f);
  const int y0 = sy < 0 ? 0 : (sy >= Hf ? Hf - 1 : sy);
  const int y1 = sy + 1 < 0 ? 0 : (sy + 1 >= Hf ? Hf - 1 : sy + 1);
  const uint8_t* r0 = fr + (long)y0 * row_bytes;
  const uint8_t* r1 = fr + (long)y1 * row_bytes;
  float v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int d0 = r0[sx * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
    const int d1 = r1[sx * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
    int t = (((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16);
    t = (t + 2) >> 2;
    const int u = t < 0 ? 0 : (t > 255 ? 255 : t);
    v[c] = (float)u / 255.f;  // transforms.ToTensor (float32 division)
  }
  // BGR -> RGB, then transforms.Normalize: (x - mean) / std
  f32x4 o;
  o[0] = (v[2] - m0) / s0;
  o[1] = (v[1] - m1) / s1;
  o[2] = (v[0] - m2) / s2;
  o[3] = 0.f;
  return o;
}

__global__ __launch_bounds__(256) void preprocess_bgr_kernel(const uint8_t* __restrict__ frame, long row_bytes,
                                                             long frame_bytes, int N, int Hf, int Wf,
                                                             float* __restrict__ out, int ld, int H, int W,
                                                             double scale_x, double scale_y, float m0, float m1,
                                                             float m2, float s0, float s1, float s2) {
  const long total = (long)N * H * W;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int dy = rem / W, dx = rem - dy * W;
    st4(out + p * ld, pre_pixel(frame + n * frame_bytes, row_bytes, Hf, Wf, dy, dx, scale_x, scale_y, m0, m1, m2, s0,
                                s1, s2));
  }
}

// The folded forward's stem (features[0]: 3x3 stride-2 conv, BN folded, ReLU6) on the preprocessed frame
// formed on load.  A block owns kStemTW output pixels of one output row: it preprocesses their 3 x (2 kStemTW
// + 1) input pixels from the frame bytes into LDS once (fp16-rounded, as seg_conv_igemm_f16 stages its
// operand), then each thread forms 8 of the 32 output channels of one pixel with fp32 accumulation (another
// sum order than the implicit GEMM's).  wk: the stem's packed weight [kStemCout][ldk], K = tap * 4 + channel.
constexpr int kStemCout = 32;
constexpr int kStemTW = 64;
__global__ __launch_bounds__(256) void stem_pre_f16_kernel(const uint8_t* __restrict__ frame, long row_bytes, int Hf,
                                                           int Wf, int H, int W, double scale_x, double scale_y,
                                                           float m0, float m1, float m2, float s0, float s1,
                                                           float s2, const float* __restrict__ wk, int ldk,
                                                           const float* __restrict__ bias, int act,
                                                           float* __restrict__ out, long ldo, int Ho, int Wo) {
  constexpr int PW = 2 * kStemTW + 1;
  __shared__ float Xs[3][PW][3];
  __shared__ float Wt[27][kStemCout];  // [tap * 3 + channel][co]
  __shared__ float Bs[kStemCout];
  const int tiles_w = (Wo + kStemTW - 1) / kStemTW;
  const int ho = blockIdx.x / tiles_w, w0 = (blockIdx.x - ho * tiles_w) * kStemTW;
  for (int i = threadIdx.x; i < 27 * kStemCout; i += 256) {
    const int co = i / 27, k = i - co * 27;
    Wt[k][co] = (float)(_Float16)wk[(long)co * ldk + (k / 3) * 4 + k % 3];
  }
  if (threadIdx.x < kStemCout) Bs[threadIdx.x] = bias ? bias[threadIdx.x] : 0.f;
  for (int i = threadIdx.x; i < 3 * PW; i += 256) {
    const int r = i / PW, c = i - r * PW;
    const int hi = 2 * ho - 1 + r, wi = 2 * w0 - 1 + c;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};  // zero padding
    if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
      x = pre_pixel(frame, row_bytes, Hf, Wf, hi, wi, scale_x, scale_y, m0, m1, m2, s0, s1, s2);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) Xs[r][c][ch] = (float)(_Float16)x[ch];
  }
  __syncthreads();
  const int px = threadIdx.x & (kStemTW - 1), cg = threadIdx.x / kStemTW;  // 4 groups of 8 channels
  const int wo = w0 + px;
  if (wo >= Wo) return;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float xv = Xs[t / 3][2 * px + t % 3][ch];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, Wt[t * 3 + ch][cg * 8 + j], acc[j]);
    }
  }
  float* o = out + ((long)ho * Wo + wo) * ldo + cg * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = seg_act(acc[4 * h + j] + Bs[cg * 8 + 4 * h + j], act);
    st4(o + 4 * h, v);
  }
}

// ---------------------------------------------------------------- argmax + nearest
// Class of model pixel (ym, xm): argmax_c of the align_corners=True bilinear of the low-res logits
// (aten max(dim) on CPU: the first maximum wins, a NaN wins and stops the scan).
__device__ __forceinline__ int model_class(const float* __restrict__ base, long ld, int H, int W, int C, int ym,
                                           int xm, float sh, float sw) {
  const Lin lh = lin_index(ym, H, sh, 1), lw = lin_index(xm, W, sw, 1);
  float best = 0.f;
  int arg = 0;
  bool done = false;
  for (int c = 0; c < C && !done; c += 4) {
    const f32x4 v00 = ld4(base + ((long)lh.i0 * W + lw.i0) * ld + c);
    const f32x4 v01 = ld4(base + ((long)lh.i0 * W + lw.i1) * ld + c);
    const f32x4 v10 = ld4(base + ((long)lh.i1 * W + lw.i0) * ld + c);
    const f32x4 v11 = ld4(base + ((long)lh.i1 * W + lw.i1) * ld + c);
    const f32x4 o = bilerp4(v00, v01, v10, v11, lh, lw);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = c + j;
      if (k >= C || done) continue;
      const float v = o[j];
      if (k == 0 || !(v <= best)) {
        best = v;
        arg = k;
        if (isnan(v)) done = true;
      }
    }
  }
  return arg;
}

__device__ __forceinline__ int nearest_src(int d, double inv, int m) {
  const int s = (int)floor((double)d * inv);
  return s < m - 1 ? s : m - 1;
}

// mask[n][yf][xf] = class of the nearest model pixel (ym, xm) of frame pixel (yf, xf), one thread per
// frame pixel (any shape).
__global__ __launch_bounds__(256) void argmax_nearest_kernel(const float* __restrict__ low, long ld, int N, int H,
                                                             int W, int C, int Hm, int Wm, float sh, float sw,
                                                             uint8_t* __restrict__ mask, int Hf, int Wf,
                                                             double ify, double ifx) {
  const long total = (long)N * Hf * Wf;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int n = (int)(p / ((long)Hf * Wf));
    const int rem = (int)(p - (long)n * Hf * Wf);
    const int yf = rem / Wf, xf = rem - yf * Wf;
    mask[p] = (uint8_t)model_class(low + (long)n * H * W * ld, ld, H, W, C, nearest_src(yf, ify, Hm),
                                   nearest_src(xf, ifx, Wm), sh, sw);
  }
}

// The same mask by bands of kBandRows frame rows per block: the block classifies the model rows its band
// maps to once (a frame 5.6x taller than the model repeats each model row ~6 times, and each model pixel
// ~28 times over a 720x1280 frame), keeps the classes in LDS and writes the band's frame rows from them,
// four pixels per 32-bit store.  Bitwise the per-pixel kernel (the same model_class per model pixel).
constexpr int kBandRows = 4;
constexpr int kBandMaxWm = 2048;
__global__ __launch_bounds__(256) void argmax_band_kernel(const float* __restrict__ low, long ld, int N, int H, int W,
                                                          int C, int Hm, int Wm, float sh, float sw,
                                                          uint8_t* __restrict__ mask, int Hf, int Wf, double ify,
                                                          double ifx) {
  __shared__ uint8_t lab[kBandRows][kBandMaxWm];
  __shared__ int slot_of[kBandRows], ym_of[kBandRows], nslots;
  const int bands = (Hf + kBandRows - 1) / kBandRows;
  const int n = blockIdx.x / bands, y0 = (blockIdx.x - n * bands) * kBandRows;
  const int rows = min(kBandRows, Hf - y0);
  if (threadIdx.x == 0) {  // distinct model rows of the band (nearest_src is monotone in yf)
    int ns = 0, prev = -1;
    for (int r = 0; r < rows; ++r) {
      const int ym = nearest_src(y0 + r, ify, Hm);
      if (ym != prev) {
        ym_of[ns++] = ym;
        prev = ym;
      }
      slot_of[r] = ns - 1;
    }
    nslots = ns;
  }
  __syncthreads();
  const float* base = low + (long)n * H * W * ld;
  for (int e = threadIdx.x; e < nslots * Wm; e += 256) {
    const int sl = e / Wm, xm = e - sl * Wm;
    lab[sl][xm] = (uint8_t)model_class(base, ld, H, W, C, ym_of[sl], xm, sh, sw);
  }
  __syncthreads();
  uint8_t* out = mask + ((long)n * Hf + y0) * Wf;
  const int q = Wf >> 2;  // Wf % 4 == 0 (host check): 32-bit stores
  for (int e = threadIdx.x; e < rows * q; e += 256) {
    const int r = e / q, x = (e - r * q) * 4;
    const uint8_t* lr = lab[slot_of[r]];
    const unsigned v = (unsigned)lr[nearest_src(x, ifx, Wm)] | ((unsigned)lr[nearest_src(x + 1, ifx, Wm)] << 8) |
                       ((unsigned)lr[nearest_src(x + 2, ifx, Wm)] << 16) |
                       ((unsigned)lr[nearest_src(x + 3, ifx, Wm)] << 24);
    *reinterpret_cast<unsigned*>(out + (long)r * Wf + x) = v;
  }
}

int grid_for(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 8192); }

}  // namespace

// Fold every eval BatchNorm of a model into its conv in ONE launch.  `jobs` is a
// DEVICE array of njobs seg_fold_job; max_elems = the largest Cout*kper + Cout.
SEG_API int seg_bn_fold_batch(const void* jobs, int njobs, long max_elems, hipStream_t stream) {
  if (njobs < 0 || max_elems < 0) return (int)hipErrorInvalidValue;
  if (njobs == 0) return 0;
  const int bx = (int)std::max<long>(1, std::min<long>(seg_cdiv(max_elems, 256), 64));
  hipLaunchKernelGGL(fold_batch_kernel, dim3(bx, njobs), dim3(256), 0, stream,
                     reinterpret_cast<const SegFoldJob*>(jobs));
  SEG_RET_LAST();
}

// N uint8 BGR frames [N][Hf][row_bytes] (3 bytes per pixel) -> normalised RGB NHWC
// rows out[N*H*W][ld] (channel 3 zeroed).  mean/std: transforms.Normalize's
// per-channel constants in RGB order (inference.py:35-36).
SEG_API int seg_preprocess_bgr(const uint8_t* frame, int N, int Hf, int Wf, long row_bytes, float* out, int ld, int H,
                               int W, float mean_r, float mean_g, float mean_b, float std_r, float std_g, float std_b,
                               hipStream_t stream) {
  if (ld < 4 || (ld & 3) || row_bytes < 3L * Wf || Hf <= 0 || Wf <= 0 || H <= 0 || W <= 0) return (int)hipErrorInvalidValue;
  const double scale_x = 1.0 / ((double)W / Wf), scale_y = 1.0 / ((double)H / Hf);
  hipLaunchKernelGGL(preprocess_bgr_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, stream, frame, row_bytes,
                     row_bytes * Hf, N, Hf, Wf, out, ld, H, W, scale_x, scale_y, mean_r, mean_g, mean_b, std_r, std_g,
                     std_b);
  SEG_RET_LAST();
}

// preprocess + the stem conv of the folded fp16 forward in one launch (stem_pre_f16_kernel): frame as
// seg_preprocess_bgr (N = 1), the stem's packed weight / folded bias / activation as seg_conv_igemm_f16
// (Cin 3 padded to 4, Cout 32, 3x3, stride 2, pad 1) into out [Ho*Wo][ldo].
SEG_API int seg_stem_pre_f16(const uint8_t* frame, int Hf, int Wf, long row_bytes, int H, int W, float mean_r,
                             float mean_g, float mean_b, float std_r, float std_g, float std_b, const float* wk,
                             int ldk, const float* bias, int act, int Cout, float* out, long ldo, hipStream_t stream) {
  if (!frame || !wk || !out || Cout != kStemCout || ldk < 36 || ldo < Cout || (ldo & 3) || ((uintptr_t)out & 15) ||
      Hf <= 0 || Wf <= 0 || H <= 0 || W <= 0 || row_bytes < 3L * Wf || act < SEG_ACT_NONE || act > SEG_ACT_RELU6)
    return (int)hipErrorInvalidValue;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const double scale_x = 1.0 / ((double)W / Wf), scale_y = 1.0 / ((double)H / Hf);
  hipLaunchKernelGGL(stem_pre_f16_kernel, dim3(Ho * seg_cdiv(Wo, kStemTW)), dim3(256), 0, stream, frame, row_bytes,
                     Hf, Wf, H, W, scale_x, scale_y, mean_r, mean_g, mean_b, std_r, std_g, std_b, wk, ldk, bias, act,
                     out, ldo, Ho, Wo);
  SEG_RET_LAST();
}

// Class mask at frame resolution from the low-res NHWC logits [N*H*W][ld]: the
// model output is their align_corners=True upsample to Hm x Wm (src/unet.py:49),
// torch.max(dim=1) picks the class (inference.py:64) and cv2 INTER_NEAREST maps
// it to Hf x Wf (inference.py:68-70).
SEG_API int seg_argmax_nearest(const float* low, long ld, int N, int H, int W, int C, int Hm, int Wm, uint8_t* mask,
                               int Hf, int Wf, hipStream_t stream) {
  if ((ld & 3) || ld < C || C <= 0 || C > 255 || Hm <= 0 || Wm <= 0 || Hf <= 0 || Wf <= 0) return (int)hipErrorInvalidValue;
  const float sh = Hm > 1 ? (float)(H - 1) / (float)(Hm - 1) : 0.f;
  const float sw = Wm > 1 ? (float)(W - 1) / (float)(Wm - 1) : 0.f;
  const double ify = 1.0 / ((double)Hf / Hm), ifx = 1.0 / ((double)Wf / Wm);
  if (SEG_ARGMAX_BAND && Wm <= kBandMaxWm && Wf % 4 == 0 && ((uintptr_t)mask & 3) == 0)
    hipLaunchKernelGGL(argmax_band_kernel, dim3(N * seg_cdiv(Hf, kBandRows)), dim3(256), 0, stream, low, ld, N, H, W,
                       C, Hm, Wm, sh, sw, mask, Hf, Wf, ify, ifx);
  else
    hipLaunchKernelGGL(argmax_nearest_kernel, dim3(grid_for((long)N * Hf * Wf)), dim3(256), 0, stream, low, ld, N, H,
                       W, C, Hm, Wm, sh, sw, mask, Hf, Wf, ify, ifx);
  SEG_RET_LAST();
}
