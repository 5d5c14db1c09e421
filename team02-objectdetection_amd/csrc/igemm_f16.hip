// seg_conv_igemm_act with fp16 math (the fp16 inference configuration, BASELINE configs[3]): the same fp32
// tensors, both operands rounded to f16 (round-to-nearest-even) in the LDS staging,
// v_mfma_f32_32x32x16_f16 with fp32 accumulation, the fp32 epilogue (igemm_impl.h).
#include "igemm_impl.h"

SEG_API int seg_conv_igemm_f16(const float* in, long ldin, int N, int H, int W, int Cin,
                                const float* wk, int ldk, const float* bias,
                                float* out, long ldout, int Ho, int Wo, int Cout,
                                int ks, int stride, int pad,
                                const float* add, long ldadd, float* stat, int act, float* work, int splits,
                                hipStream_t stream) {
  return conv_igemm_impl<_Float16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad,
                              add, ldadd, stat, act, work, splits, stream);
}

// seg_conv_igemm_f16 with split-K combined inside the launch when the grid is co-resident (else the
// separate reduce, as seg_conv_igemm_f16): cnt = 2 * seg_conv_igemm_tiles(M, Cout) unsigned, zero before
// the first launch.  Bitwise the two-launch result.
SEG_API int seg_conv_igemm_f16_ic(const float* in, long ldin, int N, int H, int W, int Cin,
                                   const float* wk, int ldk, const float* bias, float* out, long ldout, int Ho, int Wo,
                                   int Cout, int ks, int stride, int pad, const float* add, long ldadd, int act,
                                   float* work, int splits, int tile, unsigned* cnt, hipStream_t stream) {
  return conv_igemm_impl<_Float16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad, add,
                              ldadd, nullptr, act, work, splits, stream, nullptr, nullptr, 0, (const float*)nullptr, 0, nullptr,
                              nullptr, nullptr, 0, nullptr, cnt, tile);
}

// seg_conv_igemm_f16_ic of a decoder conv whose input is cat([skip, Upsample(x2, bilinear)(low)]) (src/unet.py:97-104)
// with the upsample folded into the A-operand loads: `in` holds the skip in channels [0, ucs) of
// its Cin-wide rows, `up` the low-res tensor [N][H/2][W/2][ldup] whose x2 upsample is channels [ucs, Cin) -- formed
// per operand slot with seg_upsample_fwd's index arithmetic and blend, so the upsampled rows never exist and the
// upsample launch disappears.  3x3, stride 1, pad 1, H and W even, ucs % 4 == 0.
SEG_API int seg_conv_igemm_f16_ic_up(const float* in, long ldin, int N, int H, int W, int Cin, const float* up,
                                      long ldup, int ucs, const float* wk, int ldk, const float* bias, float* out,
                                      long ldout, int Cout, const float* add, long ldadd, int act, float* work,
                                      int splits, int tile, unsigned* cnt, hipStream_t stream) {
  if (!up) return (int)hipErrorInvalidValue;
  return conv_igemm_impl<_Float16>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, H, W, Cout, 3, 1, 1, add, ldadd,
                                   nullptr, act, work, splits, stream, nullptr, nullptr, 0, (const float*)nullptr, 0,
                                   nullptr, nullptr, nullptr, 0, nullptr, cnt, tile, up, ldup, ucs);
}
