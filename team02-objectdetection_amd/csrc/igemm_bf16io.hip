// The bf16 implicit GEMM on bf16 activation storage (its own translation unit so the
// instantiation sets of igemm_impl.h compile in parallel).
#include "igemm_impl.h"

// seg_conv_igemm_bf16 on bf16 activation storage (in / add / out __bf16; the _bf16io
// training path): operands are already bf16, so the LDS staging is a plain copy.
// No split-K (training launches never split).
SEG_API int seg_conv_igemm_bf16io(const __bf16* in, long ldin, int N, int H, int W, int Cin,
                                  const float* wk, int ldk, const float* bias,
                                  __bf16* out, long ldout, int Ho, int Wo, int Cout,
                                  int ks, int stride, int pad,
                                  const __bf16* add, long ldadd, float* stat, hipStream_t stream) {
  return conv_igemm_impl<__bf16, __bf16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride,
                                         pad, add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream);
}

// seg_conv_igemm_xf on bf16 storage: the bf16 input is widened, transformed in fp32 and
// rounded back to bf16 (RNE) -- bit for bit the tensor the BN-apply pass would have stored.
SEG_API int seg_conv_igemm_bf16io_xf(const __bf16* in, long ldin, int N, int H, int W, int Cin,
                                     const float* wk, int ldk, const float* bias,
                                     __bf16* out, long ldout, int Ho, int Wo, int Cout,
                                     int ks, int stride, int pad,
                                     const __bf16* add, long ldadd, float* stat, const float* in_scale,
                                     const float* in_shift, int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_igemm_impl<__bf16, __bf16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride,
                                         pad, add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream, in_scale, in_shift,
                                         in_act);
}

// seg_conv_igemm_bnout on bf16 storage (fp32 packed weights).
SEG_API int seg_conv_igemm_bnout_bf16io(const __bf16* in, long ldin, int N, int H, int W, int Cin, const float* wk,
                                        int ldk, __bf16* out, long ldout, int Cout, int ks, const __bf16* add,
                                        long ldadd, const __bf16* by, long ldby, const float* bscale,
                                        const float* bshift, const float* bmean, int bact, float* bpart,
                                        hipStream_t stream) {
  return conv_igemm_impl<__bf16, __bf16>(in, ldin, N, H, W, Cin, wk, ldk, nullptr, out, ldout, H, W, Cout, ks, 1,
                                         ks / 2, add, ldadd, nullptr, SEG_ACT_NONE, nullptr, 1, stream, nullptr,
                                         nullptr, 0, by, ldby, bscale, bshift, bmean, bact, bpart);
}
