// seg_conv_igemm_act with bf16 math (the bf16 configurations, BASELINE configs[2]/[4]): the same fp32
// tensors, both operands rounded to bf16 (round-to-nearest-even) in the LDS staging,
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation, the fp32 epilogue (igemm_impl.h).
#include "igemm_impl.h"

SEG_API int seg_conv_igemm_bf16(const float* in, long ldin, int N, int H, int W, int Cin,
                                const float* wk, int ldk, const float* bias,
                                float* out, long ldout, int Ho, int Wo, int Cout,
                                int ks, int stride, int pad,
                                const float* add, long ldadd, float* stat, int act, float* work, int splits,
                                hipStream_t stream) {
  return conv_igemm_impl<__bf16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad,
                              add, ldadd, stat, act, work, splits, stream);
}

// seg_conv_igemm_xf (igemm.hip) with bf16 math: the transformed fp32 operand is rounded
// to bf16 in the LDS staging, as the materialized activation would have been.
SEG_API int seg_conv_igemm_bf16_xf(const float* in, long ldin, int N, int H, int W, int Cin,
                                   const float* wk, int ldk, const float* bias,
                                   float* out, long ldout, int Ho, int Wo, int Cout,
                                   int ks, int stride, int pad,
                                   const float* add, long ldadd, float* stat, const float* in_scale,
                                   const float* in_shift, int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_igemm_impl<__bf16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad,
                                 add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream, in_scale, in_shift, in_act);
}

// seg_conv_igemm_bf16 with the in-launch split-K combine (as seg_conv_igemm_f16_ic).
SEG_API int seg_conv_igemm_bf16_ic(const float* in, long ldin, int N, int H, int W, int Cin,
                                   const float* wk, int ldk, const float* bias, float* out, long ldout, int Ho, int Wo,
                                   int Cout, int ks, int stride, int pad, const float* add, long ldadd, int act,
                                   float* work, int splits, int tile, unsigned* cnt, hipStream_t stream) {
  return conv_igemm_impl<__bf16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad, add,
                              ldadd, nullptr, act, work, splits, stream, nullptr, nullptr, 0, (const float*)nullptr, 0, nullptr,
                              nullptr, nullptr, 0, nullptr, cnt, tile);
}
