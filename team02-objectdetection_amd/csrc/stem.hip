// First convolution of each model: Cin = 3, 3x3, pad 1, read straight from the
// caller's NCHW float input (no layout pass over the image batch).
//   MobileNetV2UNet: torchvision features[0] conv 3->32, stride 2, no bias
//                    (reached through src/unet.py:15,34)
//   UNet/LightUNet:  inc double_conv first conv 3->64 (or 32), stride 1, bias
//                    (src/unet.py:58 via :71-77,127)
// Output is NHWC.  Cin = 3 is far too thin for MFMA (K = 27); this is an
// HBM-bound direct conv: thread = (pixel, 4 output channels), weights in LDS
// transposed to [27][Cout] so each thread reads float4 runs.
#include "common.h"

namespace {

template <int S>
__global__ __launch_bounds__(256) void stem_fwd_kernel(const float* __restrict__ x, int N, int H, int W,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       int Cout, float* __restrict__ out, long ldout, int Ho, int Wo) {
  __shared__ __attribute__((aligned(16))) float wl[27 * 64];
  for (int i = threadIdx.x; i < 27 * Cout; i += 256) {
    const int k = i / Cout, co = i - k * Cout;
    wl[i] = w[co * 27 + k];
  }
  __syncthreads();
  const int CG = Cout >> 2;
  const long total = (long)N * Ho * Wo * CG;
  const long plane = (long)H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / CG;
    const int cg = (int)(i - p * CG);
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    f32x4 acc = bias ? ld4(bias + cg * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      const float* xp = x + ((long)n * 3 + ci) * plane;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int hi = ho * S - 1 + ky;
        if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int wi = wo * S - 1 + kx;
          if ((unsigned)wi >= (unsigned)W) continue;
          acc += xp[(long)hi * W + wi] * ld4(&wl[(ci * 9 + ky * 3 + kx) * Cout + cg * 4]);
        }
      }
    }
    st4(out + p * ldout + cg * 4, acc);
  }
}

// Per-block partials part[blk][co*27 + ci*9 + ky*3 + kx] of
// dW[co][ci][ky][kx] = sum_p dY[p][co] * x[n][ci][src(p)].
// Thread = (4 output channels, pixel lane); 27 x float4 accumulate in
// registers, reduced over the pixel lanes by xor-shuffles and across the 4 waves
// through LDS.
template <int S, int COUT>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const float* __restrict__ dy, long lddy,
                                                         const float* __restrict__ x, int N, int H, int W, int Ho,
                                                         int Wo, float* __restrict__ part, int rows_per_block) {
  constexpr int CG = COUT / 4;
  constexpr int PL = 256 / CG;  // pixel lanes per block
  __shared__ float red[4][27 * COUT];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int cg = t % CG, pl = t / CG;
  const long M = (long)N * Ho * Wo;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = std::min<long>(M, r0 + rows_per_block);
  const long plane = (long)H * W;
  f32x4 acc[27];
#pragma unroll
  for (int k = 0; k < 27; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (long p = r0 + pl; p < r1; p += PL) {
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    const f32x4 g = ld4(dy + p * lddy + cg * 4);
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      const float* xp = x + ((long)n * 3 + ci) * plane;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int hi = ho * S - 1 + ky;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int wi = wo * S - 1 + kx;
          if ((unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W)
            acc[ci * 9 + ky * 3 + kx] += g * xp[(long)hi * W + wi];
        }
      }
    }
  }
  // reduce over lanes that share cg: lane bits >= log2(CG)
#pragma unroll
  for (int k = 0; k < 27; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[k][j];
#pragma unroll
      for (int o = CG; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[k][j] = v;
    }
  if (lane < CG) {
#pragma unroll
    for (int k = 0; k < 27; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave][(cg * 4 + j) * 27 + k] = acc[k][j];
  }
  __syncthreads();
  float* pb = part + (long)blockIdx.x * 27 * COUT;
  for (int i = t; i < 27 * COUT; i += 256) pb[i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
}

}  // namespace

SEG_API int seg_stem_fwd(const float* x, int N, int H, int W, const float* w, const float* bias, int Cout,
                         float* out, long ldout, int Ho, int Wo, int stride, hipStream_t stream) {
  if ((Cout != 32 && Cout != 64) || (ldout & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  const long total = (long)N * Ho * Wo * (Cout / 4);
  const int grid = (int)std::min<long>(seg_cdiv(total, 256), 8192);
  if (stride == 1)
    hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(grid), dim3(256), 0, stream, x, N, H, W, w, bias, Cout, out, ldout, Ho, Wo);
  else
    hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3(grid), dim3(256), 0, stream, x, N, H, W, w, bias, Cout, out, ldout, Ho, Wo);
  SEG_RET_LAST();
}

SEG_API long seg_stem_wgrad_blocks(long M) {
  long rpb = (M + 1023) / 1024;
  if (rpb < 128) rpb = 128;
  return (M + rpb - 1) / rpb;
}

// part holds seg_stem_wgrad_blocks(M) * 27 * Cout floats; reduce with
// seg_conv_wgrad_reduce(part, blocks, dw, Cout, 3, 3, /*mode*/2, ...).
SEG_API int seg_stem_wgrad(const float* dy, long lddy, const float* x, int N, int H, int W, int Ho, int Wo, int Cout,
                           int stride, float* part, hipStream_t stream) {
  if ((Cout != 32 && Cout != 64) || (lddy & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  const long M = (long)N * Ho * Wo;
  const long nblk = seg_stem_wgrad_blocks(M);
  const int rpb = (int)((M + nblk - 1) / nblk);
#define SEG_STEM_WG(S, CO) \
  hipLaunchKernelGGL((stem_wgrad_kernel<S, CO>), dim3(nblk), dim3(256), 0, stream, dy, lddy, x, N, H, W, Ho, Wo, part, rpb)
  if (stride == 1 && Cout == 32) SEG_STEM_WG(1, 32);
  else if (stride == 1) SEG_STEM_WG(1, 64);
  else if (Cout == 32) SEG_STEM_WG(2, 32);
  else SEG_STEM_WG(2, 64);
#undef SEG_STEM_WG
  SEG_RET_LAST();
}
