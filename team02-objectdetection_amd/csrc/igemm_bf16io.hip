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
