// GPU-side training augmentation: the albumentations
// pipeline of the reference's readers (src/BDD100KDataset.py:38-52,
// src/CarlaDataset.py:40-47, src/SEAMEDataset.py:55-62), applied to a batch of
// decoded uint8 images / class masks on the device so the host only decodes:
//
//   Resize(H, W)                      image INTER_LINEAR (cv2 8-bit restatement,
//                                     infer.hip), mask INTER_NEAREST; the BDD100K
//                                     class remap (src/BDD100KDataset.py:23-35,68-70)
//                                     as a 256-entry LUT on the mask
//   HorizontalFlip(p=0.5)
//   ShiftScaleRotate(0.05, 0.05, 10, p=0.5)   warpAffine with BORDER_REFLECT_101:
//                                     image bilinear, mask nearest
//   RandomBrightnessContrast(p=0.5)   uint8 LUT: trunc(clip(v*alpha + beta*255))
//   Normalize(ImageNet) + ToTensorV2  (v - 255*mean) * (1 / (255*std)), CHW float
//
// Per-sample random parameters are drawn on the host (seg_amd/augment.py) and
// passed as a table; the kernels are deterministic given the table.  albumentations
// and cv2 are not installed here: the warp's interpolation arithmetic is this
// file's own float32 bilinear (rounded to nearest-even into uint8), restated by
// oracle/augref.py -- parity with albumentations itself is unpinned.
#include "common.h"

namespace {

struct SegAugParam {   // one sample (host-filled, 48 bytes)
  float m[6];          // inverse affine: output (x, y) -> flipped-image (u, v)
  float alpha, beta;   // contrast, brightness (1, 0 = off)
  int flip, warp, bc, pad_;
};
static_assert(sizeof(SegAugParam) == 48, "seg_aug_param ABI");

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// Resize stage: image (3 ch, cv2 INTER_LINEAR 8-bit) or mask (1 ch, INTER_NEAREST
// + LUT) from [N][Hs][Ws][C] to [N][H][W][C] uint8.
__global__ __launch_bounds__(256) void resize_u8_kernel(const uint8_t* __restrict__ src, int N, int Hs, int Ws,
                                                         long src_row, long src_img, uint8_t* __restrict__ dst,
                                                         int H, int W, int C, const uint8_t* __restrict__ lut,
                                                         double scale_x, double scale_y) {
#pragma clang fp contract(off)  // OpenCV computes (dx+0.5)*scale-0.5 as a separate multiply and subtract
  const long total = (long)N * H * W;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int dy = rem / W, dx = rem - dy * W;
    const uint8_t* img = src + n * src_img;
    uint8_t* o = dst + p * C;
    if (C == 1) {  // INTER_NEAREST: sx = min(floor(dx * (1 / (W / Ws))), Ws - 1)
      int sx = (int)floor((double)dx * scale_x), sy = (int)floor((double)dy * scale_y);
      sx = sx < Ws - 1 ? sx : Ws - 1;
      sy = sy < Hs - 1 ? sy : Hs - 1;
      const uint8_t v = img[(long)sy * src_row + sx];
      o[0] = lut ? lut[v] : v;
      continue;
    }
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) { sx = 0; fx = 0.f; }
    if (sx >= Ws - 1) { sx = Ws - 1; fx = 0.f; }
    const int a0 = (int)rintf((1.f - fx) * 2048.f), a1 = (int)rintf(fx * 2048.f);
    const int sx1 = sx + 1 < Ws ? sx + 1 : Ws - 1;
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int b0 = (int)rintf((1.f - fy) * 2048.f), b1 = (int)rintf(fy * 2048.f);
    const int y0 = sy < 0 ? 0 : (sy >= Hs ? Hs - 1 : sy);
    const int y1 = sy + 1 < 0 ? 0 : (sy + 1 >= Hs ? Hs - 1 : sy + 1);
    const uint8_t* r0 = img + (long)y0 * src_row;
    const uint8_t* r1 = img + (long)y1 * src_row;
    for (int c = 0; c < 3; ++c) {
      const int d0 = r0[sx * 3 + c] * a0 + r0[sx1 * 3 + c] * a1;
      const int d1 = r1[sx * 3 + c] * a0 + r1[sx1 * 3 + c] * a1;
      const int t = ((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2;
      o[c] = (uint8_t)(t < 0 ? 0 : (t > 255 ? 255 : t));
    }
  }
}

// Flip + ShiftScaleRotate + brightness/contrast + Normalize + ToTensorV2.
// img [N][H][W][3] uint8 RGB, mask [N][H][W] uint8 -> x [N][3][H][W] float,
// y [N][H][W] int64.
__global__ __launch_bounds__(256) void augment_kernel(const uint8_t* __restrict__ img, const uint8_t* __restrict__ mask,
                                                      int N, int H, int W, const SegAugParam* __restrict__ prm,
                                                      float m0, float m1, float m2, float r0, float r1, float r2,
                                                      float* __restrict__ x, long long* __restrict__ y) {
#pragma clang fp contract(off)
  const long total = (long)N * H * W;
  for (long p = blockIdx.x * 256L + threadIdx.x; p < total; p += (long)gridDim.x * 256) {
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int oy = rem / W, ox = rem - oy * W;
    const SegAugParam q = prm[n];
    const uint8_t* im = img + (long)n * H * W * 3;
    const uint8_t* mk = mask + (long)n * H * W;
    float u = (float)ox, v = (float)oy;
    if (q.warp) {
      u = q.m[0] * (float)ox + q.m[1] * (float)oy + q.m[2];
      v = q.m[3] * (float)ox + q.m[4] * (float)oy + q.m[5];
    }
    // (u, v) lives in the flipped image: flipped(u, v) = image(W - 1 - u, v)
    if (q.flip) u = (float)(W - 1) - u;
    // image: bilinear with BORDER_REFLECT_101, rounded to uint8
    const int iu = (int)floorf(u), iv = (int)floorf(v);
    const float fu = u - (float)iu, fv = v - (float)iv;
    const int xa = reflect101(iu, W), xb = reflect101(iu + 1, W);
    const int ya = reflect101(iv, H), yb = reflect101(iv + 1, H);
    float pix[3];
    for (int c = 0; c < 3; ++c) {
      float val;
      if (q.warp) {
        const float p00 = im[((long)ya * W + xa) * 3 + c], p01 = im[((long)ya * W + xb) * 3 + c];
        const float p10 = im[((long)yb * W + xa) * 3 + c], p11 = im[((long)yb * W + xb) * 3 + c];
        const float top = p00 + (p01 - p00) * fu, bot = p10 + (p11 - p10) * fu;
        float s = rintf(top + (bot - top) * fv);
        s = s < 0.f ? 0.f : (s > 255.f ? 255.f : s);
        val = s;
      } else {
        val = (float)im[((long)ya * W + xa) * 3 + c];
      }
      if (q.bc) {  // albumentations uint8 LUT: trunc(clip(v * alpha + beta * 255, 0, 255))
        float t = val * q.alpha;
        t = t + q.beta * 255.f;
        t = t < 0.f ? 0.f : (t > 255.f ? 255.f : t);
        val = truncf(t);
      }
      pix[c] = val;
    }
    x[(((long)n * 3 + 0) * H + oy) * W + ox] = (pix[0] - m0) * r0;
    x[(((long)n * 3 + 1) * H + oy) * W + ox] = (pix[1] - m1) * r1;
    x[(((long)n * 3 + 2) * H + oy) * W + ox] = (pix[2] - m2) * r2;
    // mask: nearest neighbour (round half up) with BORDER_REFLECT_101
    const int nu = reflect101((int)floorf(u + 0.5f), W), nv = reflect101((int)floorf(v + 0.5f), H);
    y[p] = (long long)mk[(long)nv * W + nu];
  }
}

int grid_for(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 8192); }

}  // namespace

// Resize a batch of uint8 images (C = 3, cv2 INTER_LINEAR) or class masks (C = 1,
// INTER_NEAREST, then lut[v] when lut != NULL) [N][Hs][src_row] -> [N][H][W][C].
SEG_API int seg_resize_u8(const unsigned char* src, int N, int Hs, int Ws, long src_row, unsigned char* dst, int H,
                          int W, int C, const unsigned char* lut, hipStream_t stream) {
  if ((C != 1 && C != 3) || src_row < (long)Ws * C || N < 0 || H <= 0 || W <= 0 || Hs <= 0 || Ws <= 0)
    return (int)hipErrorInvalidValue;
  if (N == 0) return 0;
  const double sx = 1.0 / ((double)W / Ws), sy = 1.0 / ((double)H / Hs);
  hipLaunchKernelGGL(resize_u8_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, stream, src, N, Hs, Ws, src_row,
                     src_row * Hs, dst, H, W, C, lut, sx, sy);
  SEG_RET_LAST();
}

// params: DEVICE array of N seg_aug_param.  mean255 / rstd255: per channel
// 255*mean and 1/(255*std) in float32 (albumentations Normalize).
SEG_API int seg_augment(const unsigned char* img, const unsigned char* mask, int N, int H, int W, const void* params,
                        float mean_r, float mean_g, float mean_b, float rstd_r, float rstd_g, float rstd_b, float* x,
                        long long* y, hipStream_t stream) {
  if (N < 0 || H <= 0 || W <= 0 || !params) return (int)hipErrorInvalidValue;
  if (N == 0) return 0;
  hipLaunchKernelGGL(augment_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, stream, img, mask, N, H, W,
                     reinterpret_cast<const SegAugParam*>(params), mean_r, mean_g, mean_b, rstd_r, rstd_g, rstd_b, x,
                     y);
  SEG_RET_LAST();
}
