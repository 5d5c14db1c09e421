// The bf16io implicit GEMM with bf16 packed weights (seg_pack_batch bf16 modes): the
// training path of the bf16io configuration.  Own translation unit: the WB
// instantiations compile in parallel with the fp32-weight ones (igemm_bf16io.hip).
#include "igemm_impl.h"

// seg_conv_igemm_bf16io with the weights packed as bf16 ([Cout][ldk], ldk % 8 == 0,
// 16-byte aligned; zero beyond K): the same result bit for bit (the fp32-weight
// kernel rounds the same values RNE on their way into LDS), half the weight traffic.
SEG_API int seg_conv_igemm_bf16io_w16(const __bf16* in, long ldin, int N, int H, int W, int Cin,
                                      const __bf16* wk, int ldk, const float* bias,
                                      __bf16* out, long ldout, int Ho, int Wo, int Cout,
                                      int ks, int stride, int pad,
                                      const __bf16* add, long ldadd, float* stat, hipStream_t stream) {
  return conv_igemm_impl<__bf16, __bf16, true>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks,
                                               stride, pad, add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream);
}

// seg_conv_igemm_bf16io_xf with bf16 packed weights.
SEG_API int seg_conv_igemm_bf16io_xf_w16(const __bf16* in, long ldin, int N, int H, int W, int Cin,
                                         const __bf16* wk, int ldk, const float* bias,
                                         __bf16* out, long ldout, int Ho, int Wo, int Cout,
                                         int ks, int stride, int pad,
                                         const __bf16* add, long ldadd, float* stat, const float* in_scale,
                                         const float* in_shift, int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_igemm_impl<__bf16, __bf16, true>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks,
                                               stride, pad, add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream,
                                               in_scale, in_shift, in_act);
}

// seg_conv_igemm_bf16io_w16 as a stride-1 data gradient that completes dA of a BatchNorm layer:
// plus the BN-backward partials of out (IgemmArgs::bpart; see seg_conv_igemm_bnout).
SEG_API int seg_conv_igemm_bnout_bf16io_w16(const __bf16* in, long ldin, int N, int H, int W, int Cin,
                                            const __bf16* wk, int ldk, __bf16* out, long ldout, int Cout, int ks,
                                            const __bf16* add, long ldadd, const __bf16* by, long ldby,
                                            const float* bscale, const float* bshift, const float* bmean, int bact,
                                            float* bpart, hipStream_t stream) {
  return conv_igemm_impl<__bf16, __bf16, true>(in, ldin, N, H, W, Cin, wk, ldk, nullptr, out, ldout, H, W, Cout, ks,
                                               1, ks / 2, add, ldadd, nullptr, SEG_ACT_NONE, nullptr, 1, stream,
                                               nullptr, nullptr, 0, by, ldby, bscale, bshift, bmean, bact, bpart);
}
