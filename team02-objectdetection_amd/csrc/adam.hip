// Adam step over every parameter tensor of a model in one launch.
//
// Reference: optim.Adam(model.parameters(), lr=1.5e-4) (main.py:100) stepped once
// per batch (src/train.py:39) -- defaults betas (0.9, 0.999), eps 1e-8, no weight
// decay, no amsgrad.  On the GPU torch runs it as the foreach
// implementation: ~8 multi-tensor launches per step, each streaming p / g / m / v
// again.  Here each element is read once and written once, with the arithmetic of the
// foreach ops in the same order, in fp32:
//   m = lerp(m, g, 1 - b1)                 _foreach_lerp_   (weight < 0.5 branch)
//   v = v * b2;  v = v + (1 - b2) * g * g  _foreach_mul_, _foreach_addcmul_
//   d = sqrt(v) / sqrt(bc2) + eps          _foreach_sqrt, _foreach_div_, _foreach_add_
//   p = p + (-lr / bc1) * (m / d)          _foreach_addcdiv_
// bc1 = 1 - b1^t and bc2 = 1 - b2^t are per tensor, computed on the host (as torch does
// from its CPU step counters) and passed in the tensor table.
//
// Work split: a host-built chunk map (tensor index, first element) of at most
// `chunk` elements each; one 256-thread block per chunk.  Parameters with no
// gradient (the unused classifier) are simply absent from the table.
#include "common.h"

struct SegAdamTensor {  // 48 bytes, the layout seg_amd/optim.py packs
  float* p;
  const float* g;
  float* m;
  float* v;
  long n;
  float step_size;  // -lr / bc1
  float bc2_sqrt;   // sqrt(1 - b2^t)
};

namespace {

__global__ __launch_bounds__(256) void adam_kernel(const SegAdamTensor* __restrict__ ts,
                                                   const long* __restrict__ chunks, int chunk, float w, float b2,
                                                   float cv, float eps, const float* __restrict__ skip) {
  if (skip && *skip != 0.f) return;  // the batch had an out-of-range label: no parameter or moment changes
  const long ti = chunks[2 * blockIdx.x], start = chunks[2 * blockIdx.x + 1];
  const SegAdamTensor t = ts[ti];
  const long end = std::min<long>(t.n, start + chunk);
  for (long i = start + threadIdx.x; i < end; i += 256) {
    const float g = t.g[i];
    float m = t.m[i], v = t.v[i];
    m = m + w * (g - m);
    v = v * b2;
    v = v + cv * g * g;
    const float d = sqrtf(v) / t.bc2_sqrt + eps;
    t.p[i] = t.p[i] + t.step_size * (m / d);
    t.m[i] = m;
    t.v[i] = v;
  }
}

}  // namespace

// tensors: device array of ntensors SegAdamTensor; chunks: device array of nchunks
// (tensor index, first element) int64 pairs, each chunk <= `chunk` elements.
// one_minus_beta1 / one_minus_beta2 are 1 - beta rounded once from double (torch
// passes the double 1 - beta as the lerp weight / addcmul value), not 1.f - (float)beta.
SEG_API int seg_adam_step_skip(const SegAdamTensor* tensors, const long* chunks, int nchunks, int chunk,
                               float one_minus_beta1, float beta2, float one_minus_beta2, float eps, const float* skip,
                               hipStream_t stream) {
  if (nchunks < 0 || chunk < 1) return (int)hipErrorInvalidValue;
  if (nchunks == 0) return (int)hipSuccess;
  hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, stream, tensors, chunks, chunk, one_minus_beta1, beta2,
                     one_minus_beta2, eps, skip);
  SEG_RET_LAST();
}
SEG_API int seg_adam_step(const SegAdamTensor* tensors, const long* chunks, int nchunks, int chunk,
                          float one_minus_beta1, float beta2, float one_minus_beta2, float eps, hipStream_t stream) {
  return seg_adam_step_skip(tensors, chunks, nchunks, chunk, one_minus_beta1, beta2, one_minus_beta2, eps, nullptr,
                            stream);
}
