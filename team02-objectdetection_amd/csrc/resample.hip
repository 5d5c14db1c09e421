// Bilinear resampling and 2x2 max-pooling, NHWC.
//
//  * nn.Upsample(scale_factor=2, mode='bilinear') (align_corners=False) of every
//    decoder `up` block, src/unet.py:97,101 -- the result is written straight
//    into the channel slice [Cskip, Cskip+C) of the concat buffer that
//    torch.cat([x2, x1], dim=1) (src/unet.py:103, skip FIRST) would build.
//  * nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True), the final
//    upsample of MobileNetV2UNet (src/unet.py:30,49): NHWC low-res logits ->
//    NCHW full-res logits (the layout the reference returns).
//  * nn.MaxPool2d(2) of UNet's `down` (src/unet.py:85).
// Source-index arithmetic follows aten's CPU upsample_bilinear2d in float:
//   align_corners: src = scale*dst, scale = (in-1)/(out-1)
//   otherwise:     src = max(scale*(dst+0.5)-0.5, 0), scale = 1/scale_factor
//   i0 = min(floor(src), in-1), i1 = i0 + (i0 < in-1), l1 = src - i0, l0 = 1 - l1.
// Backward passes are gathers (every input pixel sums the few output pixels that
// sampled it, recomputing the forward's indices exactly): no atomics,
// bitwise reproducible.
#include "common.h"

namespace {

// Weight with which output index `dst` samples input index `i`.
__device__ __forceinline__ float lin_weight(int dst, int i, int in, float scale, int ac) {
  const Lin l = lin_index(dst, in, scale, ac);
  return (l.i0 == i ? l.l0 : 0.f) + (l.i1 == i ? l.l1 : 0.f);
}

// Output range [lo, hi] that can reference input index i.
__device__ __forceinline__ void dst_range(int i, int in, int out, float scale, int ac, int* lo, int* hi) {
  // src in [i-1, i+1) maps to dst in about [(i-1)/scale, (i+1)/scale); pad by 2.
  const float inv = 1.f / scale;
  float a = ac ? (float)(i - 1) * inv : ((float)(i - 1) + 0.5f) * inv - 0.5f;
  float b = ac ? (float)(i + 1) * inv : ((float)(i + 1) + 0.5f) * inv - 0.5f;
  int l = (int)floorf(a) - 2, h = (int)ceilf(b) + 2;
  *lo = l < 0 ? 0 : l;
  *hi = h > out - 1 ? out - 1 : h;
}

template <typename T>
__global__ void up_fwd_nhwc_kernel(const T* __restrict__ in, long ldin, int N, int H, int W, int C,
                                   T* __restrict__ out, long ldout, int Ho, int Wo, float sh, float sw, int ac) {
  const int CG = C >> 2;
  const long total = (long)N * Ho * Wo * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / CG;
    const int c = (int)(i - p * CG) * 4;
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    const Lin lh = lin_index(r, H, sh, ac), lw = lin_index(s, W, sw, ac);
    const T* base = in + (long)n * H * W * ldin;
    const f32x4 v00 = ld4(base + ((long)lh.i0 * W + lw.i0) * ldin + c);
    const f32x4 v01 = ld4(base + ((long)lh.i0 * W + lw.i1) * ldin + c);
    const f32x4 v10 = ld4(base + ((long)lh.i1 * W + lw.i0) * ldin + c);
    const f32x4 v11 = ld4(base + ((long)lh.i1 * W + lw.i1) * ldin + c);
    const f32x4 o = up_blend4(v00, v01, v10, v11, lh.l0, lh.l1, lw.l0, lw.l1);  // (the fold's blend, common.h)
    st4(out + p * ldout + c, o);
  }
}

// d_in[n][h][w][c] = sum_{r,s} w_h(r,h) w_w(s,w) d_out[n][r][s][c]
// LAYOUT 0: d_out NHWC [N*Ho*Wo][ldout];  LAYOUT 1: d_out NCHW [N][C][Ho][Wo].
// The column weights of the (at most SMAX) candidate output columns are computed
// once per thread into registers (for x2 resampling 4 of them are non-zero), so
// the inner loop is loads and FMAs only.
constexpr int SMAX = 12;

template <int LAYOUT, typename TI = float, typename TO = float>
__global__ void up_bwd_kernel(const TI* __restrict__ dout, long ldout, int N, int Ho, int Wo, int C,
                              TO* __restrict__ din, long ldin, int H, int W, float sh, float sw, int ac,
                              int accumulate) {
  const int CG = (C + 3) >> 2;
  const long total = (long)N * H * W * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long q = i / CG;
    const int c = (int)(i - q * CG) * 4;
    const int n = (int)(q / ((long)H * W));
    const int rem = (int)(q - (long)n * H * W);
    const int h = rem / W, w = rem - h * W;
    int rlo, rhi, slo, shi;
    dst_range(h, H, Ho, sh, ac, &rlo, &rhi);
    dst_range(w, W, Wo, sw, ac, &slo, &shi);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    auto add = [&](int r, int s, float wt) {
      if (LAYOUT == 0) {
        acc += wt * ld4(dout + (((long)n * Ho + r) * Wo + s) * ldout + c);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (c + j < C) acc[j] += wt * (float)dout[(((long)n * C + c + j) * Ho + r) * Wo + s];
      }
    };
    if (shi - slo + 1 <= SMAX) {
      float wsv[SMAX];
#pragma unroll
      for (int k = 0; k < SMAX; ++k) wsv[k] = slo + k <= shi ? lin_weight(slo + k, w, W, sw, ac) : 0.f;
      for (int r = rlo; r <= rhi; ++r) {
        const float wr = lin_weight(r, h, H, sh, ac);
        if (wr == 0.f) continue;
#pragma unroll
        for (int k = 0; k < SMAX; ++k)
          if (wsv[k] != 0.f) add(r, slo + k, wr * wsv[k]);
      }
    } else {
      for (int r = rlo; r <= rhi; ++r) {
        const float wr = lin_weight(r, h, H, sh, ac);
        if (wr == 0.f) continue;
        for (int s = slo; s <= shi; ++s) {
          const float ws = lin_weight(s, w, W, sw, ac);
          if (ws != 0.f) add(r, s, wr * ws);
        }
      }
    }
    TO* dst = din + q * ldin + c;
    if (accumulate) acc += ld4(dst);
    st4(dst, acc);
  }
}

// Exact x2, align_corners=False, NHWC (every decoder `up`): the output rows that
// sample input row h are 2h-1 .. 2h+2 with weights 0.25, 0.75, 0.75, 0.25 (the
// values lin_index produces; at the borders the clamped taps fold into 1.0), so
// the gather is 16 loads with constant weights and no index search.
template <typename T>
__global__ __launch_bounds__(256) void up2_bwd_kernel(const T* __restrict__ dout, long ldout, int N, int C,
                                                      T* __restrict__ din, long ldin, int H, int W,
                                                      int accumulate) {
  const int CG = C >> 2, Ho = 2 * H, Wo = 2 * W;
  const long total = (long)N * H * W * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long q = i / CG;
    const int c = (int)(i - q * CG) * 4;
    const int n = (int)(q / ((long)H * W));
    const int rem = (int)(q - (long)n * H * W);
    const int h = rem / W, w = rem - h * W;
    const float wr[4] = {h > 0 ? 0.25f : 0.f, h > 0 ? 0.75f : 1.f, h < H - 1 ? 0.75f : 1.f, h < H - 1 ? 0.25f : 0.f};
    const float wc[4] = {w > 0 ? 0.25f : 0.f, w > 0 ? 0.75f : 1.f, w < W - 1 ? 0.75f : 1.f, w < W - 1 ? 0.25f : 0.f};
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const T* base = dout + (long)n * Ho * Wo * ldout + c;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int r = 2 * h - 1 + a;
      const int rc = r < 0 ? 0 : (r > Ho - 1 ? Ho - 1 : r);  // weight 0 where clamped
      f32x4 row = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int s = 2 * w - 1 + b;
        const int sc = s < 0 ? 0 : (s > Wo - 1 ? Wo - 1 : s);
        row += wc[b] * ld4(base + ((long)rc * Wo + sc) * ldout);
      }
      acc += wr[a] * row;
    }
    T* dst = din + q * ldin + c;
    if (accumulate) acc += ld4(dst);
    st4(dst, acc);
  }
}

// up2_bwd_kernel for a 2x2 block of input pixels per thread (rows h, h+1; columns w,
// w+1; one float4 channel group): the four gathers share source rows 2h+1..2h+2 and
// columns 2w+1..2w+2, so the block loads a 6x6 window (9 loads per pixel instead of 16)
// and decodes its position once, from blockIdx.y = (n, h/2) and a 32-bit
// (column pair, channel group) index.  Each pixel's sum is formed in up2_bwd_kernel's
// order -- row sums over b, then rows over a, both ascending -- so the results are
// bitwise those of up2_bwd_kernel.
template <typename T>
__global__ __launch_bounds__(256) void up2_bwd_quad_kernel(const T* __restrict__ dout, long ldout, int N, int C,
                                                           T* __restrict__ din, long ldin, int H, int W,
                                                           int accumulate) {
  const int CG = C >> 2, Ho = 2 * H, Wo = 2 * W, HP = (H + 1) >> 1, WP = (W + 1) >> 1;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= WP * CG) return;
  const int n = blockIdx.y / HP, h = 2 * (blockIdx.y - n * HP);
  const int wp = idx / CG, c = (idx - wp * CG) * 4, w = 2 * wp;
  float wr[2][4], wc[2][4];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int hh = h + k, ww = w + k;
    wr[k][0] = hh > 0 ? 0.25f : 0.f;
    wr[k][1] = hh > 0 ? 0.75f : 1.f;
    wr[k][2] = hh < H - 1 ? 0.75f : 1.f;
    wr[k][3] = hh < H - 1 ? 0.25f : 0.f;
    wc[k][0] = ww > 0 ? 0.25f : 0.f;
    wc[k][1] = ww > 0 ? 0.75f : 1.f;
    wc[k][2] = ww < W - 1 ? 0.75f : 1.f;
    wc[k][3] = ww < W - 1 ? 0.25f : 0.f;
  }
  const T* base = dout + (long)n * Ho * Wo * ldout + c;
  long col[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int s = 2 * w - 1 + j;
    col[j] = (long)(s < 0 ? 0 : (s > Wo - 1 ? Wo - 1 : s)) * ldout;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int k = 0; k < 2; ++k) acc[k][0] = acc[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 6; ++j) {  // source row 2h-1+j; output row h uses j = 0..3, row h+1 j = 2..5
    const int r = 2 * h - 1 + j;
    const int rc = r < 0 ? 0 : (r > Ho - 1 ? Ho - 1 : r);
    const T* rowp = base + (long)rc * Wo * ldout;
    f32x4 v[6];
#pragma unroll
    for (int b = 0; b < 6; ++b) v[b] = ld4(rowp + col[b]);
    f32x4 rs0 = {0.f, 0.f, 0.f, 0.f}, rs1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      rs0 += wc[0][b] * v[b];
      rs1 += wc[1][b] * v[b + 2];
    }
    if (j < 4) {
      acc[0][0] += wr[0][j] * rs0;
      acc[0][1] += wr[0][j] * rs1;
    }
    if (j >= 2) {
      acc[1][0] += wr[1][j - 2] * rs0;
      acc[1][1] += wr[1][j - 2] * rs1;
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      if (h + k >= H || w + l >= W) continue;
      T* dst = din + ((long)(n * H + h + k) * W + w + l) * ldin + c;
      f32x4 o = acc[k][l];
      if (accumulate) o += ld4(dst);
      st4(dst, o);
    }
  }
}

// NHWC low-res -> NCHW full-res (the model's returned logits).
template <typename T>
__global__ void up_fwd_to_nchw_kernel(const T* __restrict__ in, long ldin, int N, int H, int W, int C,
                                      float* __restrict__ out, int Ho, int Wo, float sh, float sw, int ac) {
  const long total = (long)N * Ho * Wo;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    const Lin lh = lin_index(r, H, sh, ac), lw = lin_index(s, W, sw, ac);
    const T* base = in + (long)n * H * W * ldin;
    for (int c = 0; c < C; c += 4) {
      const f32x4 v00 = ld4(base + ((long)lh.i0 * W + lw.i0) * ldin + c);
      const f32x4 v01 = ld4(base + ((long)lh.i0 * W + lw.i1) * ldin + c);
      const f32x4 v10 = ld4(base + ((long)lh.i1 * W + lw.i0) * ldin + c);
      const f32x4 v11 = ld4(base + ((long)lh.i1 * W + lw.i1) * ldin + c);
      const f32x4 o = bilerp4(v00, v01, v10, v11, lh, lw);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < C) out[(((long)n * C + c + j) * Ho + r) * Wo + s] = o[j];
    }
  }
}

// MaxPool2d(2), floor mode: first maximum in (0,0),(0,1),(1,0),(1,1) order, NaN wins
// (aten CPU max_pool2d: `if (val > maxval || isnan(val))`).
__device__ __forceinline__ int pool_argmax(float v0, float v1, float v2, float v3, float* m) {
  float best = v0;
  int arg = 0;
  if (v1 > best || isnan(v1)) { best = v1; arg = 1; }
  if (v2 > best || isnan(v2)) { best = v2; arg = 2; }
  if (v3 > best || isnan(v3)) { best = v3; arg = 3; }
  *m = best;
  return arg;
}

template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ in, long ldin, int N, int H, int W, int C,
                                   T* __restrict__ out, long ldout) {
  const int Ho = H / 2, Wo = W / 2, CG = C >> 2;
  const long total = (long)N * Ho * Wo * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / CG;
    const int c = (int)(i - p * CG) * 4;
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    const T* b = in + (((long)n * H + 2 * r) * W + 2 * s) * ldin + c;
    const f32x4 a0 = ld4(b), a1 = ld4(b + ldin), a2 = ld4(b + (long)W * ldin), a3 = ld4(b + (long)W * ldin + ldin);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m;
      pool_argmax(a0[j], a1[j], a2[j], a3[j], &m);
      o[j] = m;
    }
    st4(out + p * ldout + c, o);
  }
}

template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ in, long ldin, const T* __restrict__ dout,
                                   long lddout, int N, int H, int W, int C, T* __restrict__ din, long lddin,
                                   int accumulate) {
  const int Ho = H / 2, Wo = W / 2, CG = C >> 2;
  const long total = (long)N * Ho * Wo * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / CG;
    const int c = (int)(i - p * CG) * 4;
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    const long q0 = ((long)n * H + 2 * r) * W + 2 * s;
    const long qs[4] = {q0, q0 + 1, q0 + W, q0 + W + 1};
    const f32x4 a0 = ld4(in + qs[0] * ldin + c), a1 = ld4(in + qs[1] * ldin + c);
    const f32x4 a2 = ld4(in + qs[2] * ldin + c), a3 = ld4(in + qs[3] * ldin + c);
    const f32x4 g = ld4(dout + p * lddout + c);
    f32x4 o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = accumulate ? ld4(din + qs[k] * lddin + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m;
      const int arg = pool_argmax(a0[j], a1[j], a2[j], a3[j], &m);
      o[arg][j] += g[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) st4(din + qs[k] * lddin + c, o[k]);
  }
}

// NCHW image batch -> NHWC rows of ld channels, channels [C, ld) zero-filled.
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int H, int W, T* __restrict__ out,
                                    int ld) {
  const long plane = (long)H * W;
  const long total = (long)N * plane;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const long n = p / plane, q = p - n * plane;
    const float* src = x + n * C * plane + q;
    for (int c = 0; c < ld; c += 4) {
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (c + j < C) ? src[(long)(c + j) * plane] : 0.f;
      st4(out + p * ld + c, v);
    }
  }
}

int ew_grid(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 8192); }

float up_scale(int in, int out, int ac) {
  if (ac) return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  return (float)in / (float)out;  // == 1/scale_factor for the exact 2x upsample
}

}  // namespace

// Bilinear resize NHWC -> NHWC (strided), ac = align_corners.
template <typename T>
static int upsample_fwd_impl(const T* in, long ldin, int N, int H, int W, int C, T* out, long ldout, int Ho, int Wo,
                             int ac, hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (ldout & 3)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(up_fwd_nhwc_kernel<T>, dim3(ew_grid((long)N * Ho * Wo * (C / 4))), dim3(256), 0, stream, in, ldin,
                     N, H, W, C, out, ldout, Ho, Wo, up_scale(H, Ho, ac), up_scale(W, Wo, ac), ac);
  SEG_RET_LAST();
}
SEG_API int seg_upsample_fwd(const float* in, long ldin, int N, int H, int W, int C, float* out, long ldout, int Ho,
                             int Wo, int ac, hipStream_t stream) {
  return upsample_fwd_impl(in, ldin, N, H, W, C, out, ldout, Ho, Wo, ac, stream);
}
SEG_API int seg_upsample_fwd_bf16io(const __bf16* in, long ldin, int N, int H, int W, int C, __bf16* out, long ldout,
                                    int Ho, int Wo, int ac, hipStream_t stream) {
  return upsample_fwd_impl(in, ldin, N, H, W, C, out, ldout, Ho, Wo, ac, stream);
}

// Gradient of seg_upsample_fwd / seg_upsample_to_nchw.  nchw_grad = 1 when d_out is
// the NCHW gradient of the model's returned logits (always fp32).  d_in is NHWC
// (ldin >= round4(C)).
template <typename T>
static int upsample_bwd_impl(const void* dout, long ldout, int nchw_grad, int N, int Ho, int Wo, int C, T* din,
                             long ldin, int H, int W, int ac, int accumulate, hipStream_t stream) {
  if ((ldin & 3) || (!nchw_grad && (ldout & 3))) return (int)hipErrorInvalidValue;
  const int grid = ew_grid((long)N * H * W * ((C + 3) / 4));
  const float sh = up_scale(H, Ho, ac), sw = up_scale(W, Wo, ac);
  const T* dn = static_cast<const T*>(dout);
  if (!nchw_grad && !ac && Ho == 2 * H && Wo == 2 * W && !(C & 3)) {
    const long rows = (long)N * ((H + 1) / 2), cols = (long)((W + 1) / 2) * (C / 4);
    if (rows <= 65535 && cols < (1L << 30))
      hipLaunchKernelGGL(up2_bwd_quad_kernel<T>, dim3((unsigned)seg_cdiv(cols, 256), (unsigned)rows), dim3(256), 0,
                         stream, dn, ldout, N, C, din, ldin, H, W, accumulate);
    else
      hipLaunchKernelGGL(up2_bwd_kernel<T>, dim3(grid), dim3(256), 0, stream, dn, ldout, N, C, din, ldin, H, W,
                         accumulate);
    SEG_RET_LAST();
  }
  if (nchw_grad)
    hipLaunchKernelGGL((up_bwd_kernel<1, float, T>), dim3(grid), dim3(256), 0, stream,
                       static_cast<const float*>(dout), ldout, N, Ho, Wo, C, din, ldin, H, W, sh, sw, ac, accumulate);
  else
    hipLaunchKernelGGL((up_bwd_kernel<0, T, T>), dim3(grid), dim3(256), 0, stream, dn, ldout, N, Ho, Wo, C, din, ldin,
                       H, W, sh, sw, ac, accumulate);
  SEG_RET_LAST();
}
SEG_API int seg_upsample_bwd(const float* dout, long ldout, int nchw_grad, int N, int Ho, int Wo, int C, float* din,
                             long ldin, int H, int W, int ac, int accumulate, hipStream_t stream) {
  return upsample_bwd_impl(dout, ldout, nchw_grad, N, Ho, Wo, C, din, ldin, H, W, ac, accumulate, stream);
}
// dout: bf16 NHWC, or fp32 NCHW when nchw_grad = 1.
SEG_API int seg_upsample_bwd_bf16io(const void* dout, long ldout, int nchw_grad, int N, int Ho, int Wo, int C,
                                    __bf16* din, long ldin, int H, int W, int ac, int accumulate, hipStream_t stream) {
  return upsample_bwd_impl(dout, ldout, nchw_grad, N, Ho, Wo, C, din, ldin, H, W, ac, accumulate, stream);
}

template <typename T>
static int upsample_to_nchw_impl(const T* in, long ldin, int N, int H, int W, int C, float* out, int Ho, int Wo, int ac,
                                 hipStream_t stream) {
  if (ldin & 3) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(up_fwd_to_nchw_kernel<T>, dim3(ew_grid((long)N * Ho * Wo)), dim3(256), 0, stream, in, ldin, N, H,
                     W, C, out, Ho, Wo, up_scale(H, Ho, ac), up_scale(W, Wo, ac), ac);
  SEG_RET_LAST();
}
SEG_API int seg_upsample_to_nchw(const float* in, long ldin, int N, int H, int W, int C, float* out, int Ho, int Wo,
                                 int ac, hipStream_t stream) {
  return upsample_to_nchw_impl(in, ldin, N, H, W, C, out, Ho, Wo, ac, stream);
}
SEG_API int seg_upsample_to_nchw_bf16io(const __bf16* in, long ldin, int N, int H, int W, int C, float* out, int Ho,
                                        int Wo, int ac, hipStream_t stream) {
  return upsample_to_nchw_impl(in, ldin, N, H, W, C, out, Ho, Wo, ac, stream);
}

// The model input (NCHW float, as the reference's DataLoader delivers it) as NHWC
// rows padded to `ld` channels -- lets the Cin = 3 first conv run on the MFMA
// implicit-GEMM path (K = 9 taps x 4 channels, the 4th weight channel packed 0).
template <typename T>
static int nchw_to_nhwc_impl(const float* x, int N, int C, int H, int W, T* out, int ld, hipStream_t stream) {
  if ((ld & 3) || ld < C) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(ew_grid((long)N * H * W)), dim3(256), 0, stream, x, N, C, H, W, out,
                     ld);
  SEG_RET_LAST();
}
SEG_API int seg_nchw_to_nhwc(const float* x, int N, int C, int H, int W, float* out, int ld, hipStream_t stream) {
  return nchw_to_nhwc_impl(x, N, C, H, W, out, ld, stream);
}
SEG_API int seg_nchw_to_nhwc_bf16io(const float* x, int N, int C, int H, int W, __bf16* out, int ld,
                                    hipStream_t stream) {
  return nchw_to_nhwc_impl(x, N, C, H, W, out, ld, stream);
}

template <typename T>
static int maxpool2_fwd_impl(const T* in, long ldin, int N, int H, int W, int C, T* out, long ldout,
                             hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (ldout & 3)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(ew_grid((long)N * (H / 2) * (W / 2) * (C / 4))), dim3(256), 0, stream,
                     in, ldin, N, H, W, C, out, ldout);
  SEG_RET_LAST();
}
SEG_API int seg_maxpool2_fwd(const float* in, long ldin, int N, int H, int W, int C, float* out, long ldout,
                             hipStream_t stream) {
  return maxpool2_fwd_impl(in, ldin, N, H, W, C, out, ldout, stream);
}
SEG_API int seg_maxpool2_fwd_bf16io(const __bf16* in, long ldin, int N, int H, int W, int C, __bf16* out, long ldout,
                                    hipStream_t stream) {
  return maxpool2_fwd_impl(in, ldin, N, H, W, C, out, ldout, stream);
}

template <typename T>
static int maxpool2_bwd_impl(const T* in, long ldin, const T* dout, long lddout, int N, int H, int W, int C, T* din,
                             long lddin, int accumulate, hipStream_t stream) {
  if ((C & 3) || (ldin & 3) || (lddout & 3) || (lddin & 3) || (H & 1) || (W & 1)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(ew_grid((long)N * (H / 2) * (W / 2) * (C / 4))), dim3(256), 0, stream,
                     in, ldin, dout, lddout, N, H, W, C, din, lddin, accumulate);
  SEG_RET_LAST();
}
SEG_API int seg_maxpool2_bwd(const float* in, long ldin, const float* dout, long lddout, int N, int H, int W, int C,
                             float* din, long lddin, int accumulate, hipStream_t stream) {
  return maxpool2_bwd_impl(in, ldin, dout, lddout, N, H, W, C, din, lddin, accumulate, stream);
}
SEG_API int seg_maxpool2_bwd_bf16io(const __bf16* in, long ldin, const __bf16* dout, long lddout, int N, int H, int W,
                                    int C, __bf16* din, long lddin, int accumulate, hipStream_t stream) {
  return maxpool2_bwd_impl(in, ldin, dout, lddout, N, H, W, C, din, lddin, accumulate, stream);
}
