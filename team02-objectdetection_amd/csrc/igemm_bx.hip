// 1x1 data gradients with the layer's BatchNorm backward formed on load (BX): the
// training path's expand / project / head 1x1 convs (torchvision InvertedResidual,
// reached through src/unet.py:15-19; features[18]; src/unet.py:113-115).
//
// Unfused, the backward of conv -> BN (-> act) is seg_bn_backward (reduction, finalize,
// apply pass dA, y -> dY) followed by the conv's data gradient reading dY.  Here the apply
// pass is done by the GEMM's A loader instead: each K chunk loads dA and y at the same
// slots, forms dY with seg_bnbwd4 (the apply pass's fp32 arithmetic) and rounds it to the
// storage type exactly as the pass would have stored it, so the result is bitwise the
// unfused one (tests/test_gpu_bx.py).  Blocks of the first output-column tile also store
// the dY rows they formed, which the weight / bias gradients (side stream) read.  Saves
// one launch and two tensor passes (the apply's re-read of dA, y) per layer on the
// critical stream.  Own translation unit: the BX instantiations compile in parallel.
#include "igemm_impl.h"

template <typename OT, typename IT, bool WB>
static int bx_impl(const IT* da, long ldda, int N, int H, int W, int C, const void* wk, int ldk, IT* dx, long lddx,
                   int Cx, const IT* add, long ldadd, const IT* y, long ldy, const float* stats, const float* coef,
                   int act, IT* dy, long lddy, hipStream_t stream) {
  const BxArgs bx{y, ldy, stats, coef, act, dy, lddy};
  return conv_igemm_impl<OT, IT, WB, true>(da, ldda, N, H, W, C, wk, ldk, nullptr, dx, lddx, H, W, Cx, 1, 1, 0, add,
                                           ldadd, nullptr, SEG_ACT_NONE, nullptr, 1, stream, nullptr, nullptr, 0,
                                           &bx);
}

SEG_API int seg_conv_igemm_bx(const float* da, long ldda, int N, int H, int W, int C, const float* wk, int ldk,
                              float* dx, long lddx, int Cx, const float* add, long ldadd, const float* y, long ldy,
                              const float* stats, const float* coef, int act, float* dy, long lddy,
                              hipStream_t stream) {
  return bx_impl<float, float, false>(da, ldda, N, H, W, C, wk, ldk, dx, lddx, Cx, add, ldadd, y, ldy, stats, coef,
                                      act, dy, lddy, stream);
}

SEG_API int seg_conv_igemm_bf16io_bx_w16(const __bf16* da, long ldda, int N, int H, int W, int C, const __bf16* wk,
                                         int ldk, __bf16* dx, long lddx, int Cx, const __bf16* add, long ldadd,
                                         const __bf16* y, long ldy, const float* stats, const float* coef, int act,
                                         __bf16* dy, long lddy, hipStream_t stream) {
  if ((ldk & 7) || ((uintptr_t)wk & 15)) return (int)hipErrorInvalidValue;
  return bx_impl<__bf16, __bf16, true>(da, ldda, N, H, W, C, wk, ldk, dx, lddx, Cx, add, ldadd, y, ldy, stats, coef,
                                       act, dy, lddy, stream);
}
