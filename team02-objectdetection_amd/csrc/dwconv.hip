// Depthwise 3x3 convolution (stride 1 or 2, pad 1, no bias), NHWC.
//
// Replaces the groups=C Conv2d of every torchvision InvertedResidual block
// (features[1..17], reached through src/unet.py:15-19,34-38).
// HBM-bound.  A thread owns one float4 channel group and a strip of TW
// consecutive output pixels of one row; the 3 input rows slide through
// registers, so each output pixel costs 3 (stride 1) or 6 (stride 2) fresh
// 16-B loads instead of 9, and the 9 weight float4 are loaded once per strip.
// Lanes of a wave run over consecutive channel groups, so every load is a run
// of whole 16-B segments of one pixel row.
//
// Lazy BatchNorm: the forward and the weight gradient can apply the producing
// layer's BN affine + activation to their input on load (`isc`/`ish`/`iact`,
// the expand conv's scale/shift), so the expand conv's activated output is never
// written to HBM.  Padding taps stay exactly zero (the transform applies to
// in-image pixels only), as in the reference where padding follows the ReLU6.
//
// Weights are packed tap-major wk[9][C] (seg_pack_dw_weight).
#include "common.h"

namespace {

#ifndef SEG_DW_TW
#define SEG_DW_TW 4
#endif
#ifndef SEG_DW_TWW
#define SEG_DW_TWW 4
#endif
#ifndef SEG_DW_WG_BLOCKS
#define SEG_DW_WG_BLOCKS 2048
#endif
#ifndef SEG_DW_WG_MINSTRIPS
#define SEG_DW_WG_MINSTRIPS 4
#endif
constexpr int TW = SEG_DW_TW;    // output pixels per thread strip (forward, data gradient)
constexpr int TWW = SEG_DW_TWW;  // output pixels per strip of the weight gradient

__global__ void pack_dw_kernel(const float* __restrict__ w, float* __restrict__ wk, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // i = tap*C + c
  if (i >= 9 * C) return;
  const int tap = i / C, c = i - tap * C;
  wk[i] = w[c * 9 + tap];
}

// Input row reader: in-image pixels (optionally BN+act transformed), zero outside.
// Loads are unconditional (row and column clamped into the image, the value then
// masked) so the compiler can issue a whole strip's loads back to back instead of
// one branch-guarded, latency-exposed load at a time.
template <bool LAZY, typename T = float>
struct RowIn {
  const T* p;      // base of an in-image row (clamped) + channel offset
  long ld;
  int W;
  bool ok;         // the requested row is inside the image
  f32x4 sc, sh;
  int act;
  __device__ __forceinline__ void init(const T* base, int h, int H, int W_, long ld_) {
    ok = (unsigned)h < (unsigned)H;
    const int hc = h < 0 ? 0 : (h >= H ? H - 1 : h);
    p = base + (long)hc * W_ * ld_;
    ld = ld_;
    W = W_;
  }
  __device__ __forceinline__ f32x4 at(int wi) const {
    const int wc = wi < 0 ? 0 : (wi >= W ? W - 1 : wi);
    f32x4 v = ld4(p + (long)wc * ld);
    if (LAZY) v = seg_bn_act4(v, sc, sh, act);
    const bool in = ok && (unsigned)wi < (unsigned)W;
    return in ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
};

// Store a strip's TW results (after all of its loads were issued: no store sits
// between two loads, so the scheduler can batch the strip's loads).  CHECK: the
// strip crosses the row end (only the last strip of a row when TW does not divide it).
template <bool ACC, typename T>
__device__ __forceinline__ void store_strip(T* o, long ld, const f32x4 (&acc)[TW], int n_valid) {
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (t < n_valid) {
      f32x4 v = acc[t];
      if (ACC) v += ld4(o + t * ld);
      st4(o + t * ld, v);
    }
  }
}

// out[n][ho][wo][c] = sum_{ky,kx} w[ky][kx][c] * in[n][ho*S-1+ky][wo*S-1+kx][c]
// FLIP: taps read as w[8-tap] -- the stride-1 data gradient is this correlation
// of dY with the flipped kernel.  ACC: out += (the data gradient's accumulate).
// EPI (inference, BN folded into wk): out = act(acc + obias) -- the folded
// BatchNorm shift and the ReLU6 applied in the epilogue.
template <int S, bool LAZY, bool FLIP, bool ACC, bool EPI = false, typename T = float>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const T* __restrict__ in, long ldin, int N, int H, int W,
                                                     int C, const float* __restrict__ isc,
                                                     const float* __restrict__ ish, int iact,
                                                     const float* __restrict__ wk, T* __restrict__ out,
                                                     long ldout, int Ho, int Wo,
                                                     const float* __restrict__ obias, int oact) {
  const int CG = C >> 2;
  const int SPR = (Wo + TW - 1) / TW;
  const long total = (long)N * Ho * SPR * CG;
  // XCD-aware: consecutive items (neighbouring output rows, which share input
  // rows) run on one XCD, so each input row is fetched into one L2, not three
  const long i = (long)xcd_swizzle(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i < total) {
    const long st = i / CG;
    const int c = (int)(i - st * CG) * 4;
    const long row = st / SPR;  // n*Ho + ho
    const int ws = (int)(st - row * SPR) * TW;
    const int n = (int)(row / Ho), ho = (int)(row - (long)n * Ho);
    f32x4 w[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) w[t] = ld4(wk + (FLIP ? 8 - t : t) * C + c);
    RowIn<LAZY, T> r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      r[k].init(in + (long)n * H * W * ldin + c, ho * S - 1 + k, H, W, ldin);
      r[k].act = iact;
      if (LAZY) {
        r[k].sc = ld4(isc + c);
        r[k].sh = ld4(ish + c);
      }
    }
    f32x4 a[3], b[3];  // input columns wo*S-1 and wo*S (stride 1), or column wo*S-1 (stride 2)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      a[k] = r[k].at(ws * S - 1);
      if (S == 1) b[k] = r[k].at(ws);
    }
    f32x4 acc[TW];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int wo = ws + t;
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        f32x4 c1, c2;
        if (S == 1) {
          c1 = b[k];
          c2 = r[k].at(wo + 1);
        } else {
          c1 = r[k].at(2 * wo);
          c2 = r[k].at(2 * wo + 1);
        }
        acc[t] += a[k] * w[k * 3 + 0];
        acc[t] += c1 * w[k * 3 + 1];
        acc[t] += c2 * w[k * 3 + 2];
        if (S == 1) {
          a[k] = c1;
          b[k] = c2;
        } else {
          a[k] = c2;
        }
      }
    }
    if (EPI) {
      const f32x4 ob = ld4(obias + c), one = {1.f, 1.f, 1.f, 1.f};
#pragma unroll
      for (int t = 0; t < TW; ++t) acc[t] = seg_bn_act4(acc[t], one, ob, oact);
    }
    store_strip<ACC>(out + (row * Wo + ws) * ldout + c, ldout, acc, Wo - ws);
  }
}

// Stride-2 data gradient.  dX row hq receives dY row hq/2 through ky=1 (hq even)
// or rows (hq+1)/2 (ky=0) and (hq-1)/2 (ky=2) (hq odd); column pair (2j, 2j+1):
//   dX[2j]   = sum_rows w[ky][1] dY[.][j]
//   dX[2j+1] = sum_rows w[ky][0] dY[.][j+1] + w[ky][2] dY[.][j]
// A thread owns TW dX columns (TW/2 pairs); dY column j+1 slides to the next pair.
template <typename T>
__global__ __launch_bounds__(256) void dw_dgrad_s2_kernel(const T* __restrict__ dy, long lddy, int N, int Ho,
                                                          int Wo, int C, const float* __restrict__ wk,
                                                          T* __restrict__ dx, long lddx, int H, int W,
                                                          int accumulate) {
  const int CG = C >> 2;
  const int SPR = (W + TW - 1) / TW;
  const long total = (long)N * H * SPR * CG;
  const long i = (long)xcd_swizzle(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  if (i < total) {
    const long st = i / CG;
    const int c = (int)(i - st * CG) * 4;
    const long row = st / SPR;  // n*H + hq
    const int ws = (int)(st - row * SPR) * TW;
    const int n = (int)(row / H), hq = (int)(row - (long)n * H);
    const bool odd = hq & 1;
    // row slots: slot 0 = (even: ky 1, ho hq/2 | odd: ky 0, ho (hq+1)/2), slot 1 = (odd: ky 2, ho (hq-1)/2)
    const int ky0 = odd ? 0 : 1, ho0 = odd ? (hq + 1) >> 1 : hq >> 1, ho1 = (hq - 1) >> 1;
    RowIn<false, T> r[2];
    const T* img = dy + (long)n * Ho * Wo * lddy + c;
    r[0].init(img, ho0, Ho, Wo, lddy);
    r[1].init(img, odd ? ho1 : -1, Ho, Wo, lddy);
    f32x4 w[2][3];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ky = s == 0 ? ky0 : 2;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) w[s][kx] = ld4(wk + (ky * 3 + kx) * C + c);
    }
    const int j0 = ws >> 1;
    f32x4 dj[2] = {r[0].at(j0), r[1].at(j0)};
    f32x4 acc[TW];
#pragma unroll
    for (int t = 0; t < TW / 2; ++t) {
      const int j = j0 + t;
      f32x4 e = {0.f, 0.f, 0.f, 0.f}, f = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f32x4 dj1 = r[s].at(j + 1);
        e += dj[s] * w[s][1];
        f += dj1 * w[s][0];
        f += dj[s] * w[s][2];
        dj[s] = dj1;
      }
      acc[2 * t] = e;
      acc[2 * t + 1] = f;
    }
    T* o = dx + (row * W + ws) * lddx + c;
    if (accumulate)
      store_strip<true>(o, lddx, acc, W - ws);
    else
      store_strip<false>(o, lddx, acc, W - ws);
  }
}

// Weight-gradient partials: part[bx][tap][C] = sum over the block's strips of
// dY[p][c] * X[src(p, tap)][c].  Block = RG row groups x TC channel groups; a
// thread slides along its strips keeping 9 float4 accumulators, then a fixed-
// order LDS tree reduction over the row groups (deterministic).
template <int S, bool LAZY, typename T = float>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const T* __restrict__ dy, long lddy,
                                                       const T* __restrict__ x, long ldx, int N, int H, int W,
                                                       int C, const float* __restrict__ isc,
                                                       const float* __restrict__ ish, int iact, int Ho, int Wo,
                                                       int TC, int gy, int strips_per_block,
                                                       float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) f32x4 red[];  // [RG][TC][9]
  const int CG = C >> 2;
  const int RG = 256 / TC;
  const int t = threadIdx.x, rg = t / TC, tc = t - rg * TC;
  const int lin = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring strip chunks on one XCD
  const int gxs = gridDim.x / gy;
  const int bx = lin % gxs, byy = lin / gxs;
  const int cg = byy * TC + tc;
  const bool active = rg < RG && cg < CG;
  const int SPR = (Wo + TWW - 1) / TWW;
  const long nstrips = (long)N * Ho * SPR;
  const long s0 = (long)bx * strips_per_block;
  const long s1 = std::min<long>(nstrips, s0 + strips_per_block);
  f32x4 acc[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (active) {
    const int c = cg * 4;
    f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sh = sc;
    if (LAZY) {
      sc = ld4(isc + c);
      sh = ld4(ish + c);
    }
    for (long st = s0 + rg; st < s1; st += RG) {
      const long row = st / SPR;
      const int ws = (int)(st - row * SPR) * TWW;
      const int n = (int)(row / Ho), ho = (int)(row - (long)n * Ho);
      RowIn<LAZY, T> r[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        r[k].init(x + (long)n * H * W * ldx + c, ho * S - 1 + k, H, W, ldx);
        r[k].sc = sc;
        r[k].sh = sh;
        r[k].act = iact;
      }
      const T* g = dy + (row * Wo + ws) * lddy + c;
      f32x4 a[3], b[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a[k] = r[k].at(ws * S - 1);
        if (S == 1) b[k] = r[k].at(ws);
      }
#pragma unroll 2
      for (int u = 0; u < TWW; ++u) {
        const int wo = ws + u;
        const f32x4 g0 = ld4(g + (long)(wo < Wo ? u : Wo - 1 - ws) * lddy);
        const f32x4 gv = wo < Wo ? g0 : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          f32x4 c1, c2;
          if (S == 1) {
            c1 = b[k];
            c2 = r[k].at(wo + 1);
          } else {
            c1 = r[k].at(2 * wo);
            c2 = r[k].at(2 * wo + 1);
          }
          acc[k * 3 + 0] += gv * a[k];
          acc[k * 3 + 1] += gv * c1;
          acc[k * 3 + 2] += gv * c2;
          if (S == 1) {
            a[k] = c1;
            b[k] = c2;
          } else {
            a[k] = c2;
          }
        }
      }
    }
  }
  if (rg < RG) {
#pragma unroll
    for (int k = 0; k < 9; ++k) red[(rg * TC + tc) * 9 + k] = acc[k];
  }
  __syncthreads();
  int p2 = 1;
  while (p2 < RG) p2 <<= 1;
  for (int s = p2 >> 1; s > 0; s >>= 1) {
    if (rg < s && rg + s < RG) {
#pragma unroll
      for (int k = 0; k < 9; ++k) red[(rg * TC + tc) * 9 + k] += red[((rg + s) * TC + tc) * 9 + k];
    }
    __syncthreads();
  }
  if (rg == 0 && active) {
    float* pb = part + (long)bx * 9 * C + cg * 4;
#pragma unroll
    for (int k = 0; k < 9; ++k) st4(pb + k * C, red[tc * 9 + k]);
  }
}

int item_grid(long total) { return (int)seg_cdiv(total, 256); }

// Channel-group tiling of the weight-gradient block: TC lanes of channel
// groups (<= 64, balanced over the chunks), RG = 256 / TC row groups.
void wgrad_tiling(int C, int* TC, int* gy) {
  const int CG = C >> 2;
  const int chunks = (CG + 63) / 64;
  *TC = (CG + chunks - 1) / chunks;
  *gy = chunks;
}

void wgrad_grid(int N, int Ho, int Wo, int C, long* gx, int* spb) {
  int TC, gy;
  wgrad_tiling(C, &TC, &gy);
  const int RG = 256 / TC;
  const long nstrips = (long)N * Ho * ((Wo + TWW - 1) / TWW);
  long bx = std::max<long>(1, SEG_DW_WG_BLOCKS / gy);                              // blocks in all
  bx = std::min<long>(bx, std::max<long>(1, nstrips / ((long)SEG_DW_WG_MINSTRIPS * RG)));  // strips per thread
  long per = (nstrips + bx - 1) / bx;
  *spb = (int)per;
  *gx = (nstrips + per - 1) / per;
}

}  // namespace

SEG_API int seg_pack_dw_weight(const float* w, float* wk, int C, hipStream_t stream) {
  hipLaunchKernelGGL(pack_dw_kernel, dim3(seg_cdiv(9 * C, 256)), dim3(256), 0, stream, w, wk, C);
  SEG_RET_LAST();
}

template <typename T>
static int dw_fwd_impl(const T* in, long ldin, int N, int H, int W, int C, const float* in_scale,
                       const float* in_shift, int in_act, const float* wk, T* out, long ldout, int Ho, int Wo,
                       int stride, hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (ldout & 3) || (stride != 1 && stride != 2) || ((in_scale == nullptr) != (in_shift == nullptr)))
    return (int)hipErrorInvalidValue;
  const int grid = item_grid((long)N * Ho * ((Wo + TW - 1) / TW) * (C / 4));
  const bool lazy = in_scale != nullptr;
#define SEG_DW_FWD(S, L)                                                                                         \
  hipLaunchKernelGGL((dw_fwd_kernel<S, L, false, false, false, T>), dim3(grid), dim3(256), 0, stream, in, ldin, N, H, W, C, \
                     in_scale, in_shift, in_act, wk, out, ldout, Ho, Wo, nullptr, 0)
  if (stride == 1) {
    if (lazy) SEG_DW_FWD(1, true); else SEG_DW_FWD(1, false);
  } else {
    if (lazy) SEG_DW_FWD(2, true); else SEG_DW_FWD(2, false);
  }
#undef SEG_DW_FWD
  SEG_RET_LAST();
}
SEG_API int seg_dw_fwd(const float* in, long ldin, int N, int H, int W, int C, const float* in_scale,
                       const float* in_shift, int in_act, const float* wk, float* out, long ldout, int Ho, int Wo,
                       int stride, hipStream_t stream) {
  return dw_fwd_impl(in, ldin, N, H, W, C, in_scale, in_shift, in_act, wk, out, ldout, Ho, Wo, stride, stream);
}
SEG_API int seg_dw_fwd_bf16io(const __bf16* in, long ldin, int N, int H, int W, int C, const float* in_scale,
                              const float* in_shift, int in_act, const float* wk, __bf16* out, long ldout, int Ho,
                              int Wo, int stride, hipStream_t stream) {
  return dw_fwd_impl(in, ldin, N, H, W, C, in_scale, in_shift, in_act, wk, out, ldout, Ho, Wo, stride, stream);
}

// Inference depthwise conv with the BatchNorm folded into wk (seg_bn_fold):
// out = act(dwconv(in, wk) + bias).
SEG_API int seg_dw_fwd_bias_act(const float* in, long ldin, int N, int H, int W, int C, const float* wk,
                                const float* bias, int act, float* out, long ldout, int Ho, int Wo, int stride,
                                hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (ldout & 3) || (stride != 1 && stride != 2) || !bias || act < 0 || act > 2)
    return (int)hipErrorInvalidValue;
  const int grid = item_grid((long)N * Ho * ((Wo + TW - 1) / TW) * (C / 4));
  if (stride == 1)
    hipLaunchKernelGGL((dw_fwd_kernel<1, false, false, false, true>), dim3(grid), dim3(256), 0, stream, in, ldin, N, H,
                       W, C, nullptr, nullptr, 0, wk, out, ldout, Ho, Wo, bias, act);
  else
    hipLaunchKernelGGL((dw_fwd_kernel<2, false, false, false, true>), dim3(grid), dim3(256), 0, stream, in, ldin, N, H,
                       W, C, nullptr, nullptr, 0, wk, out, ldout, Ho, Wo, bias, act);
  SEG_RET_LAST();
}

template <typename T>
static int dw_dgrad_impl(const T* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk, T* dx,
                         long lddx, int H, int W, int stride, int accumulate, hipStream_t stream) {
  if ((C & 3) || (lddy & 3) || (lddx & 3) || (stride != 1 && stride != 2)) return (int)hipErrorInvalidValue;
  if (stride == 1) {
    if (H != Ho || W != Wo) return (int)hipErrorInvalidValue;
    const int grid = item_grid((long)N * H * ((W + TW - 1) / TW) * (C / 4));
    if (accumulate)
      hipLaunchKernelGGL((dw_fwd_kernel<1, false, true, true, false, T>), dim3(grid), dim3(256), 0, stream, dy, lddy, N, Ho, Wo,
                         C, nullptr, nullptr, 0, wk, dx, lddx, H, W, nullptr, 0);
    else
      hipLaunchKernelGGL((dw_fwd_kernel<1, false, true, false, false, T>), dim3(grid), dim3(256), 0, stream, dy, lddy, N, Ho,
                         Wo, C, nullptr, nullptr, 0, wk, dx, lddx, H, W, nullptr, 0);
  } else {
    const int grid = item_grid((long)N * H * ((W + TW - 1) / TW) * (C / 4));
    hipLaunchKernelGGL(dw_dgrad_s2_kernel<T>, dim3(grid), dim3(256), 0, stream, dy, lddy, N, Ho, Wo, C, wk, dx, lddx,
                       H, W, accumulate);
  }
  SEG_RET_LAST();
}
SEG_API int seg_dw_dgrad(const float* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk, float* dx,
                         long lddx, int H, int W, int stride, int accumulate, hipStream_t stream) {
  return dw_dgrad_impl(dy, lddy, N, Ho, Wo, C, wk, dx, lddx, H, W, stride, accumulate, stream);
}
SEG_API int seg_dw_dgrad_bf16io(const __bf16* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk, __bf16* dx,
                                long lddx, int H, int W, int stride, int accumulate, hipStream_t stream) {
  return dw_dgrad_impl(dy, lddy, N, Ho, Wo, C, wk, dx, lddx, H, W, stride, accumulate, stream);
}

SEG_API long seg_dw_wgrad_blocks(int N, int Ho, int Wo, int C) {
  long gx;
  int spb;
  wgrad_grid(N, Ho, Wo, C, &gx, &spb);
  return gx;
}

// part must hold seg_dw_wgrad_blocks(N, Ho, Wo, C) * 9 * C floats; reduce with
// seg_conv_wgrad_reduce(part, blocks, dw, C, 1, 3, /*mode*/1, ...).
template <typename T>
static int dw_wgrad_impl(const T* dy, long lddy, const T* x, long ldx, int N, int H, int W, int C,
                         const float* in_scale, const float* in_shift, int in_act, int Ho, int Wo, int stride,
                         float* part, hipStream_t stream) {
  if ((C & 3) || (lddy & 3) || (ldx & 3) || (stride != 1 && stride != 2) || ((in_scale == nullptr) != (in_shift == nullptr)))
    return (int)hipErrorInvalidValue;
  int TC, gy, spb;
  long gx;
  wgrad_tiling(C, &TC, &gy);
  wgrad_grid(N, Ho, Wo, C, &gx, &spb);
  const size_t lds = (size_t)(256 / TC) * TC * 9 * sizeof(f32x4);
  const bool lazy = in_scale != nullptr;
#define SEG_DW_WG(S, L)                                                                                         \
  hipLaunchKernelGGL((dw_wgrad_kernel<S, L, T>), dim3(gx * gy), dim3(256), lds, stream, dy, lddy, x, ldx, N, H, W, C, \
                     in_scale, in_shift, in_act, Ho, Wo, TC, gy, spb, part)
  if (stride == 1) {
    if (lazy) SEG_DW_WG(1, true); else SEG_DW_WG(1, false);
  } else {
    if (lazy) SEG_DW_WG(2, true); else SEG_DW_WG(2, false);
  }
#undef SEG_DW_WG
  SEG_RET_LAST();
}
SEG_API int seg_dw_wgrad(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int C,
                         const float* in_scale, const float* in_shift, int in_act, int Ho, int Wo, int stride,
                         float* part, hipStream_t stream) {
  return dw_wgrad_impl(dy, lddy, x, ldx, N, H, W, C, in_scale, in_shift, in_act, Ho, Wo, stride, part, stream);
}
SEG_API int seg_dw_wgrad_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W, int C,
                                const float* in_scale, const float* in_shift, int in_act, int Ho, int Wo, int stride,
                                float* part, hipStream_t stream) {
  return dw_wgrad_impl(dy, lddy, x, ldx, N, H, W, C, in_scale, in_shift, in_act, Ho, Wo, stride, part, stream);
}
