// Depthwise 3x3 convolution (stride 1 or 2, pad 1, no bias), NHWC.
//
// Replaces the groups=C Conv2d of every torchvision InvertedResidual block
// (features[1..17], reached through src/unet.py:15-19,34-38).
// HBM-bound: each thread owns one output pixel x 4 channels (one float4 lane of
// a channel run, so a wave reads whole 16-B segments of consecutive channels),
// the 9 taps' overlapping rows are served from L1/L2.
// Weights are packed tap-major wk[9][C] (seg_pack_dw_weight) so a thread's 9
// weight float4 are contiguous channel runs too.
#include "common.h"

namespace {

__global__ void pack_dw_kernel(const float* __restrict__ w, float* __restrict__ wk, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // i = tap*C + c
  if (i >= 9 * C) return;
  const int tap = i / C, c = i - tap * C;
  wk[i] = w[c * 9 + tap];
}

template <int S>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const float* __restrict__ in, long ldin, int N, int H, int W,
                                                     int C, const float* __restrict__ wk, float* __restrict__ out,
                                                     long ldout, int Ho, int Wo) {
  const int CG = C >> 2;
  const long total = (long)N * Ho * Wo * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / CG;
    const int c = (int)(i - p * CG) * 4;
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int hi = ho * S - 1 + ky;
      if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int wi = wo * S - 1 + kx;
        if ((unsigned)wi >= (unsigned)W) continue;
        acc += ld4(in + (((long)n * H + hi) * W + wi) * ldin + c) * ld4(wk + (ky * 3 + kx) * C + c);
      }
    }
    st4(out + p * ldout + c, acc);
  }
}

// dX[q][c] = sum_{ky,kx} W[c][ky][kx] * dY[(hq+1-ky)/S][(wq+1-kx)/S][c] (when integral and in range)
template <int S>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const float* __restrict__ dy, long lddy, int N, int Ho, int Wo,
                                                       int C, const float* __restrict__ wk, float* __restrict__ dx,
                                                       long lddx, int H, int W, int accumulate) {
  const int CG = C >> 2;
  const long total = (long)N * H * W * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long q = i / CG;
    const int c = (int)(i - q * CG) * 4;
    const int n = (int)(q / ((long)H * W));
    const int rem = (int)(q - (long)n * H * W);
    const int hq = rem / W, wq = rem - hq * W;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int th = hq + 1 - ky;
      if (th < 0 || (S == 2 && (th & 1))) continue;
      const int ho = th / S;
      if (ho >= Ho) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int tw = wq + 1 - kx;
        if (tw < 0 || (S == 2 && (tw & 1))) continue;
        const int wo = tw / S;
        if (wo >= Wo) continue;
        acc += ld4(dy + (((long)n * Ho + ho) * Wo + wo) * lddy + c) * ld4(wk + (ky * 3 + kx) * C + c);
      }
    }
    if (accumulate) acc += ld4(dx + q * lddx + c);
    st4(dx + q * lddx + c, acc);
  }
}

// Per-block partials of dW[c][tap] = sum_p dY[p][c] * X[src(p,tap)][c], laid out
// part[blk][tap][C]; the 9 taps x float4 accumulate in registers, then an LDS
// reduction over the block's row-lanes.
template <int S>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const float* __restrict__ dy, long lddy,
                                                       const float* __restrict__ x, long ldx, int N, int H, int W,
                                                       int C, int Ho, int Wo, float* __restrict__ part,
                                                       int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) f32x4 red[];  // [256][9]
  const int CG = C >> 2;
  const int TC = CG < 256 ? CG : 256;
  const int RG = 256 / TC;
  const int t = threadIdx.x, rg = t / TC, tc = t - rg * TC;
  const long M = (long)N * Ho * Wo;
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = std::min<long>(M, r0 + rows_per_block);
  float* pb = part + (long)blockIdx.x * 9 * C;
  for (int cgb = 0; cgb < CG; cgb += TC) {
    const int cg = cgb + tc;
    const bool active = rg < RG && cg < CG;
    f32x4 acc[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (active) {
      const int c = cg * 4;
      for (long p = r0 + rg; p < r1; p += RG) {
        const int n = (int)(p / ((long)Ho * Wo));
        const int rem = (int)(p - (long)n * Ho * Wo);
        const int ho = rem / Wo, wo = rem - ho * Wo;
        const f32x4 g = ld4(dy + p * lddy + c);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int hi = ho * S - 1 + ky;
          if ((unsigned)hi >= (unsigned)H) continue;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int wi = wo * S - 1 + kx;
            if ((unsigned)wi >= (unsigned)W) continue;
            acc[ky * 3 + kx] += g * ld4(x + (((long)n * H + hi) * W + wi) * ldx + c);
          }
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) red[t * 9 + k] = acc[k];
    __syncthreads();
    if (rg == 0 && active) {
      for (int j = 1; j < RG; ++j)
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] += red[(j * TC + tc) * 9 + k];
#pragma unroll
      for (int k = 0; k < 9; ++k) st4(pb + k * C + cg * 4, acc[k]);
    }
    __syncthreads();
  }
}

int ew_grid(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 8192); }

}  // namespace

SEG_API int seg_pack_dw_weight(const float* w, float* wk, int C, hipStream_t stream) {
  hipLaunchKernelGGL(pack_dw_kernel, dim3(seg_cdiv(9 * C, 256)), dim3(256), 0, stream, w, wk, C);
  SEG_RET_LAST();
}

SEG_API int seg_dw_fwd(const float* in, long ldin, int N, int H, int W, int C, const float* wk, float* out, long ldout,
                       int Ho, int Wo, int stride, hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (ldout & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  const int grid = ew_grid((long)N * Ho * Wo * (C / 4));
  if (stride == 1)
    hipLaunchKernelGGL(dw_fwd_kernel<1>, dim3(grid), dim3(256), 0, stream, in, ldin, N, H, W, C, wk, out, ldout, Ho, Wo);
  else
    hipLaunchKernelGGL(dw_fwd_kernel<2>, dim3(grid), dim3(256), 0, stream, in, ldin, N, H, W, C, wk, out, ldout, Ho, Wo);
  SEG_RET_LAST();
}

SEG_API int seg_dw_dgrad(const float* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk, float* dx,
                         long lddx, int H, int W, int stride, int accumulate, hipStream_t stream) {
  if ((C & 3) || (lddy & 3) || (lddx & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  const int grid = ew_grid((long)N * H * W * (C / 4));
  if (stride == 1)
    hipLaunchKernelGGL(dw_dgrad_kernel<1>, dim3(grid), dim3(256), 0, stream, dy, lddy, N, Ho, Wo, C, wk, dx, lddx, H, W, accumulate);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<2>, dim3(grid), dim3(256), 0, stream, dy, lddy, N, Ho, Wo, C, wk, dx, lddx, H, W, accumulate);
  SEG_RET_LAST();
}

SEG_API long seg_dw_wgrad_blocks(long M) {
  long rpb = (M + 2047) / 2048;  // ~2048 blocks: >= 8 blocks (32 waves) per CU
  if (rpb < 32) rpb = 32;
  return (M + rpb - 1) / rpb;
}

// part must hold seg_dw_wgrad_blocks(M) * 9 * C floats; reduce with
// seg_conv_wgrad_reduce(part, blocks, dw, C, 1, 3, /*mode*/1, ...).
SEG_API int seg_dw_wgrad(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int C, int Ho,
                         int Wo, int stride, float* part, hipStream_t stream) {
  if ((C & 3) || (lddy & 3) || (ldx & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  const long M = (long)N * Ho * Wo;
  const long nblk = seg_dw_wgrad_blocks(M);
  const int rpb = (int)((M + nblk - 1) / nblk);
  const size_t lds = 256 * 9 * sizeof(f32x4);
  if (stride == 1)
    hipLaunchKernelGGL(dw_wgrad_kernel<1>, dim3(nblk), dim3(256), lds, stream, dy, lddy, x, ldx, N, H, W, C, Ho, Wo,
                       part, rpb);
  else
    hipLaunchKernelGGL(dw_wgrad_kernel<2>, dim3(nblk), dim3(256), lds, stream, dy, lddy, x, ldx, N, H, W, C, Ho, Wo,
                       part, rpb);
  SEG_RET_LAST();
}
