// Per-pixel cross-entropy fused with the model's final align_corners=True
// bilinear x2 upsample.
//
// Reference: criterion = nn.CrossEntropyLoss() (main.py:99) applied to the model
// output (src/train.py:37), whose last op is final_upsample (src/unet.py:30,49).
// Semantics: loss = sum_{valid p} (logsumexp(z_p) - z_p[y_p]) / #valid,
// weight=None, ignore_index=-100, label_smoothing=0; labels are int64.
// d loss / d z_p = g * (softmax(z_p) - onehot(y_p)) / #valid  (g = upstream grad).
//
// The full-resolution logits z_p are never stored: each kernel recomputes them
// from the NHWC low-resolution logits (4 taps x C), which stay L2-resident.
// The loss reduction is deterministic: per-block partials, then one fp64 pass.
// A label outside [0, C) that is not ignore_index (aten raises "Target out of
// bounds") is counted in out2[2] and poisons the loss and the gradient with NaN --
// stream-ordered, no host sync; the host raises when it reads the loss
// (seg_amd.train / engine.check_targets).
#include "common.h"

namespace {

struct LinAC {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ LinAC lin_ac(int dst, int in, float scale) {
  const float src = scale * (float)dst;
  int i0 = (int)floorf(src);
  if (i0 > in - 1) i0 = in - 1;
  LinAC r;
  r.i0 = i0;
  r.i1 = i0 + (i0 < in - 1 ? 1 : 0);
  r.l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  r.l0 = 1.f - r.l1;
  return r;
}

constexpr int CMAX = 32;

// Recompute the CP (= round4(C)) full-res logits of pixel (n, r, s); the class
// loops are unrolled over CP so z stays in registers with constant indices.
template <int CP, typename T>
__device__ __forceinline__ void full_res_logits(const T* __restrict__ low, long ld, int H, int W, int n, int r,
                                                int s, float sh, float sw, float (&z)[CP]) {
  const LinAC lh = lin_ac(r, H, sh), lw = lin_ac(s, W, sw);
  const T* base = low + (long)n * H * W * ld;
  const T* p00 = base + ((long)lh.i0 * W + lw.i0) * ld;
  const T* p01 = base + ((long)lh.i0 * W + lw.i1) * ld;
  const T* p10 = base + ((long)lh.i1 * W + lw.i0) * ld;
  const T* p11 = base + ((long)lh.i1 * W + lw.i1) * ld;
#pragma unroll
  for (int c = 0; c < CP; c += 4) {
    const f32x4 o = lh.l0 * (lw.l0 * ld4(p00 + c) + lw.l1 * ld4(p01 + c)) +
                    lh.l1 * (lw.l0 * ld4(p10 + c) + lw.l1 * ld4(p11 + c));
#pragma unroll
    for (int j = 0; j < 4; ++j) z[c + j] = o[j];
  }
}

// max, sum of exp(z - max) and z[y] over the C valid classes
template <int CP>
__device__ __forceinline__ void softmax_stats(float (&z)[CP], int C, int y, float& m, float& se, float& zy,
                                              bool keep_exp) {
  m = z[0];
#pragma unroll
  for (int c = 1; c < CP; ++c)
    if (c < C) m = fmaxf(m, z[c]);
  se = 0.f;
  zy = 0.f;
#pragma unroll
  for (int c = 0; c < CP; ++c) {
    const float e = c < C ? expf(z[c] - m) : 0.f;
    zy = c == y ? z[c] : zy;
    se += e;
    if (keep_exp) z[c] = e;
  }
}

template <int CP, typename T>
__global__ __launch_bounds__(256) void ce_up_loss_kernel(const T* __restrict__ low, long ld, int N, int H, int W,
                                                         int C, const long long* __restrict__ labels, int Ho, int Wo,
                                                         float sh, float sw, int ignore_index,
                                                         float* __restrict__ part) {
  __shared__ float red_l[4], red_c[4], red_b[4];
  const long total = (long)N * Ho * Wo;
  float lsum = 0.f, cnt = 0.f, bad = 0.f;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const long long y = labels[p];
    if (y == ignore_index) continue;
    if (y < 0 || y >= C) {
      bad += 1.f;
      continue;
    }
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    float z[CP];
    full_res_logits<CP, T>(low, ld, H, W, n, r, s, sh, sw, z);
    float m, se, zy;
    softmax_stats<CP>(z, C, (int)y, m, se, zy, false);
    lsum += m + logf(se) - zy;
    cnt += 1.f;
  }
  lsum = wave_sum(lsum);
  cnt = wave_sum(cnt);
  bad = wave_sum(bad);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { red_l[wave] = lsum; red_c[wave] = cnt; red_b[wave] = bad; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = red_l[0] + red_l[1] + red_l[2] + red_l[3];
    part[3 * blockIdx.x + 1] = red_c[0] + red_c[1] + red_c[2] + red_c[3];
    part[3 * blockIdx.x + 2] = red_b[0] + red_b[1] + red_b[2] + red_b[3];
  }
}

// out[0] = mean loss, out[1] = #valid pixels, out[2] = #out-of-range labels (as floats)
__global__ void ce_finalize_kernel(const float* __restrict__ part, int nblk, float* out) {
  double l = 0.0, c = 0.0, b = 0.0;
  for (int k = threadIdx.x; k < nblk; k += 64) {
    l += part[3 * k];
    c += part[3 * k + 1];
    b += part[3 * k + 2];
  }
  for (int o = 32; o > 0; o >>= 1) {
    l += __shfl_xor(l, o, 64);
    c += __shfl_xor(c, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  if (threadIdx.x == 0) {
    out[0] = b > 0.0 ? __builtin_nanf("") : (float)(l / c);  // 0/0 = nan when every pixel is ignored, as aten
    out[1] = (float)c;
    out[2] = (float)b;
  }
}

// dhigh[p][c] = g * (softmax(z_p)[c] - [c == y_p]) / count, NHWC (ld >= round4(C)).
template <int CP, typename T>
__global__ __launch_bounds__(256) void ce_up_grad_kernel(const T* __restrict__ low, long ld, int N, int H, int W,
                                                         int C, const long long* __restrict__ labels, int Ho, int Wo,
                                                         float sh, float sw, int ignore_index,
                                                         const float* __restrict__ gout, const float* __restrict__ stats,
                                                         T* __restrict__ dhigh, long ldh) {
  const long total = (long)N * Ho * Wo;
  const float scale = stats[2] > 0.f ? __builtin_nanf("") : gout[0] / stats[1];
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const long long y = labels[p];
    T* d = dhigh + p * ldh;
    if (y == ignore_index || y < 0 || y >= C) {  // out of range: scale is NaN, the loss already is
#pragma unroll
      for (int c = 0; c < CP; c += 4) st4(d + c, f32x4{0.f, 0.f, 0.f, 0.f});
      continue;
    }
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int r = rem / Wo, s = rem - r * Wo;
    float z[CP];
    full_res_logits<CP, T>(low, ld, H, W, n, r, s, sh, sw, z);
    float m, se, zy;
    softmax_stats<CP>(z, C, (int)y, m, se, zy, true);
    const float inv = 1.f / se;
#pragma unroll
    for (int c = 0; c < CP; c += 4) {
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cc = c + j;
        o[j] = cc < C ? scale * (z[cc] * inv - (cc == (int)y ? 1.f : 0.f)) : 0.f;
      }
      st4(d + c, o);
    }
  }
}

int loss_blocks(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 2048); }

}  // namespace

SEG_API long seg_ce_workspace_floats(long pixels) { return 3L * loss_blocks(pixels); }

// Mean CE of bilinear_ac_true_x(Ho,Wo)(low) against labels.  out3[0] = loss,
// out3[1] = number of non-ignored pixels, out3[2] = number of out-of-range labels.  `work` >= seg_ce_workspace_floats(N*Ho*Wo).
template <typename T>
static int ce_loss_impl(const T* low, long ld, int N, int H, int W, int C, const long long* labels, int Ho, int Wo,
                        int ignore_index, float* work, float* out2, hipStream_t stream) {
  if ((ld & 3) || C > CMAX || C < 1) return (int)hipErrorInvalidValue;
  const long total = (long)N * Ho * Wo;
  const int nb = loss_blocks(total);
  const float sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
  const float sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
#define SEG_CE_L(CP)                                                                                          \
  case CP:                                                                                                    \
    hipLaunchKernelGGL((ce_up_loss_kernel<CP, T>), dim3(nb), dim3(256), 0, stream, low, ld, N, H, W, C, labels, Ho, \
                       Wo, sh, sw, ignore_index, work);                                                      \
    break
  switch ((C + 3) & ~3) {
    SEG_CE_L(4); SEG_CE_L(8); SEG_CE_L(12); SEG_CE_L(16); SEG_CE_L(20); SEG_CE_L(24); SEG_CE_L(28); SEG_CE_L(32);
  }
#undef SEG_CE_L
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(64), 0, stream, work, nb, out2);
  SEG_RET_LAST();
}
SEG_API int seg_ce_upsample_loss(const float* low, long ld, int N, int H, int W, int C, const long long* labels, int Ho,
                                 int Wo, int ignore_index, float* work, float* out2, hipStream_t stream) {
  return ce_loss_impl(low, ld, N, H, W, C, labels, Ho, Wo, ignore_index, work, out2, stream);
}
SEG_API int seg_ce_upsample_loss_bf16io(const __bf16* low, long ld, int N, int H, int W, int C,
                                        const long long* labels, int Ho, int Wo, int ignore_index, float* work,
                                        float* out2, hipStream_t stream) {
  return ce_loss_impl(low, ld, N, H, W, C, labels, Ho, Wo, ignore_index, work, out2, stream);
}

// Full-resolution logit gradient (NHWC, ldh >= round4(C)); follow with
// seg_upsample_bwd(nchw_grad = 0, ac = 1) to reach the low-res logits.
template <typename T>
static int ce_grad_impl(const T* low, long ld, int N, int H, int W, int C, const long long* labels, int Ho, int Wo,
                        int ignore_index, const float* grad_out, const float* stats, T* dhigh, long ldh,
                        hipStream_t stream) {
  if ((ld & 3) || (ldh & 3) || C > CMAX || C < 1) return (int)hipErrorInvalidValue;
  const long total = (long)N * Ho * Wo;
  const float sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
  const float sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  const int grid = (int)std::min<long>(seg_cdiv(total, 256), 8192);
#define SEG_CE_G(CP)                                                                                            \
  case CP:                                                                                                      \
    hipLaunchKernelGGL((ce_up_grad_kernel<CP, T>), dim3(grid), dim3(256), 0, stream, low, ld, N, H, W, C, labels, Ho, \
                       Wo, sh, sw, ignore_index, grad_out, stats, dhigh, ldh);                                 \
    break
  switch ((C + 3) & ~3) {
    SEG_CE_G(4); SEG_CE_G(8); SEG_CE_G(12); SEG_CE_G(16); SEG_CE_G(20); SEG_CE_G(24); SEG_CE_G(28); SEG_CE_G(32);
  }
#undef SEG_CE_G
  SEG_RET_LAST();
}
SEG_API int seg_ce_upsample_grad(const float* low, long ld, int N, int H, int W, int C, const long long* labels, int Ho,
                                 int Wo, int ignore_index, const float* grad_out, const float* stats, float* dhigh,
                                 long ldh, hipStream_t stream) {
  return ce_grad_impl(low, ld, N, H, W, C, labels, Ho, Wo, ignore_index, grad_out, stats, dhigh, ldh, stream);
}
SEG_API int seg_ce_upsample_grad_bf16io(const __bf16* low, long ld, int N, int H, int W, int C,
                                        const long long* labels, int Ho, int Wo, int ignore_index,
                                        const float* grad_out, const float* stats, __bf16* dhigh, long ldh,
                                        hipStream_t stream) {
  return ce_grad_impl(low, ld, N, H, W, C, labels, Ho, Wo, ignore_index, grad_out, stats, dhigh, ldh, stream);
}
