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
