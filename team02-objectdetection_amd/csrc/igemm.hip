// Implicit-GEMM convolution on the f32 matrix cores of gfx950.
//
// Replaces aten's conv2d for every non-depthwise conv of the hot path
// (reference: src/unet.py:58,61 dense 3x3 of double_conv; src/unet.py:113,116
// the 1x1 head; torchvision InvertedResidual expand/project 1x1 reached through
// src/unet.py:15-19).  One kernel serves
//   * forward:   out[p][co] = sum_{tap,ci} in[src(p,tap)][ci] * W[co][ci][tap] + bias[co]
//   * data-grad: the same GEMM run over dY with the weights packed transposed and
//                tap-flipped (seg_pack_conv_weight, mode 1) -- stride-1 convs only,
//                which is every dense/pointwise conv in MobileNetV2UNet and UNet.
//
// GEMM view: M = N*Ho*Wo pixels, N = Cout, K = ks*ks*Cin (k = tap*Cin + ci).
// Operands are staged through LDS m-major ([row][BK+4], 80-byte rows: the
// ds_read_b128 lane groups land on 16 distinct 16-B slots) and fed to
// v_mfma_f32_32x32x2_f32 (exact fp32, fmaf-chain numerics).  The K index of an
// MFMA step is remapped so each lane reads 4 consecutive k from LDS with one
// ds_read_b128: lane half h at step kk of sub-chunk ks carries k = 8ks + 4h + kk
// for BOTH operands, which is all the MFMA needs to sum the right products.
// Two LDS stages, register prefetch of the next K chunk, one barrier per chunk.
#include "igemm_impl.h"

int seg_igemm_forced_tile = -1;

// out = act(conv(in, W) + bias + add).  `wk` is the packed weight of seg_pack_conv_weight
// ([Cout][ldk], k = tap*Cin + ci).  ks in {1,3}; ks == 1 requires stride 1, pad 0.
// Cin, ldin, ldk must be multiples of 4 and `in`/`wk` 16-byte aligned.  splits > 1
// (from seg_conv_igemm_splits) runs split-K through `work` (>= splits*M*Cout floats)
// and a reduce pass; it excludes `stat`.
SEG_API int seg_conv_igemm_act(const float* in, long ldin, int N, int H, int W, int Cin,
                               const float* wk, int ldk, const float* bias,
                               float* out, long ldout, int Ho, int Wo, int Cout,
                               int ks, int stride, int pad,
                               const float* add, long ldadd, float* stat, int act, float* work, int splits,
                               hipStream_t stream) {
  return conv_igemm_impl<float>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad,
                                add, ldadd, stat, act, work, splits, stream);
}

// seg_conv_igemm of a 1x1 conv whose input is the raw output of a BatchNorm'd producer
// ("lazy BN": the depthwise conv of torchvision's InvertedResidual feeding the project
// conv, outconv's first conv feeding its second, src/unet.py:113-116): the A operand is
// act(in * in_scale[c] + in_shift[c]) formed on load, so the producer's BN-apply pass
// and its output tensor disappear.  ks 1, or ks 3 with Cin >= the K chunk (padding taps stay zero:
// the transform applies to real pixels only -- double_conv's first conv feeding its second).
SEG_API int seg_conv_igemm_xf(const float* in, long ldin, int N, int H, int W, int Cin,
                              const float* wk, int ldk, const float* bias,
                              float* out, long ldout, int Ho, int Wo, int Cout,
                              int ks, int stride, int pad,
                              const float* add, long ldadd, float* stat, const float* in_scale, const float* in_shift,
                              int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_igemm_impl<float>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad,
                                add, ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream, in_scale, in_shift, in_act);
}

// A stride-1 data gradient (out = the conv's input gradient, pad ks/2, no bias, optional fused
// addend) that completes dA of a BatchNorm layer whose pre-BN output is `by`: the epilogue also
// writes that layer's BN-backward partials per row tile -- bpart[seg_conv_igemm_row_tiles(M,
// Cout)][2][Cout] = (sum dz, sum dz (by - bmean)), dz = out act'(by bscale + bshift) on the stored
// values -- for seg_bn_bwd_finalize_tiles, in place of seg_bn_bwd_coef's reduction pass over dA.
// 1 when seg_conv_igemm_bnout (bf16 = 0) / _bnout_bf16io[_w16] (bf16 = 1) takes an M x Cout output.
SEG_API int seg_conv_igemm_bnout_ok(long M, int Cout, int bf16) { return igemm_bnout_tile_ok(M, Cout, bf16 ? 2 : 4); }

SEG_API int seg_conv_igemm_bnout(const float* in, long ldin, int N, int H, int W, int Cin, const float* wk, int ldk,
                                 float* out, long ldout, int Cout, int ks, const float* add, long ldadd,
                                 const float* by, long ldby, const float* bscale, const float* bshift,
                                 const float* bmean, int bact, float* bpart, hipStream_t stream) {
  return conv_igemm_impl<float>(in, ldin, N, H, W, Cin, wk, ldk, nullptr, out, ldout, H, W, Cout, ks, 1, ks / 2, add,
                                ldadd, nullptr, SEG_ACT_NONE, nullptr, 1, stream, nullptr, nullptr, 0, by, ldby,
                                bscale, bshift, bmean, bact, bpart);
}

SEG_API int seg_conv_igemm(const float* in, long ldin, int N, int H, int W, int Cin,
                           const float* wk, int ldk, const float* bias,
                           float* out, long ldout, int Ho, int Wo, int Cout,
                           int ks, int stride, int pad,
                           const float* add, long ldadd, float* stat, hipStream_t stream) {
  return seg_conv_igemm_act(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad, add,
                            ldadd, stat, SEG_ACT_NONE, nullptr, 1, stream);
}

// seg_conv_igemm_act with the in-launch split-K combine (as seg_conv_igemm_f16_ic).
SEG_API int seg_conv_igemm_act_ic(const float* in, long ldin, int N, int H, int W, int Cin,
                                   const float* wk, int ldk, const float* bias, float* out, long ldout, int Ho, int Wo,
                                   int Cout, int ks, int stride, int pad, const float* add, long ldadd, int act,
                                   float* work, int splits, int tile, unsigned* cnt, hipStream_t stream) {
  return conv_igemm_impl<float>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Ho, Wo, Cout, ks, stride, pad, add,
                              ldadd, nullptr, act, work, splits, stream, nullptr, nullptr, 0, (const float*)nullptr, 0, nullptr,
                              nullptr, nullptr, 0, nullptr, cnt, tile);
}

// Output tiles (M x Cout blocks) of the implicit GEMM: the split-K combine's counters are 2 per tile.
SEG_API int seg_conv_igemm_tiles(long M, int Cout) {
  const int t = pick_tile(M, Cout);
  return (int)(((M + kTiles[t].bm - 1) / kTiles[t].bm) * ((Cout + kTiles[t].bn - 1) / kTiles[t].bn));
}

// Plan of the folded inference forward's convs (seg_conv_igemm_*_ic), out[3] = (splits, tile, output tiles):
// where the cost model's tiles fill the chip, its own choice (1 split, tile -1).  Below that (batch-1 frames)
// per-launch timings of the decoder convs of a 128x256 frame (tools/icbench.py, profiles/r04ic_icbench.txt)
// set the rule: short K (<= 24 chunks) unsplit on the 64x64 tile (more blocks; a split's combine costs more
// than its chunks), longer K on the 8-wave 128x64 tile split to ~256 blocks with >= 4 chunks per split
// (at most 32 splits).
SEG_API int seg_conv_igemm_plan_b1(long M, int Cout, int Cin, int ks, int* out) {
  if (!out) return (int)hipErrorInvalidValue;
  int splits = 1, tile = -1;
  if (M > 0 && Cout > 0 && Cin > 0 && seg_igemm_forced_tile < 0) {
    const long K = (long)ks * ks * Cin;
    const int t = pick_tile(M, Cout);
    const long blocks = ((M + kTiles[t].bm - 1) / kTiles[t].bm) * ((Cout + kTiles[t].bn - 1) / kTiles[t].bn);
    const int nk = seg_cdiv(K, igemm_bk((int)K));
    if (blocks < 256) {
      if (nk <= 24) {
        tile = 3;
      } else {
        tile = 12;
        const long b12 = ((M + 127) / 128) * ((Cout + 63) / 64);
        long s = std::min<long>(std::min<long>(32, (256 + b12 - 1) / b12), nk / 4);
        s = std::max<long>(s, 1);
        splits = seg_cdiv(nk, seg_cdiv(nk, (int)s));  // no empty split
      }
    }
  }
  const int tt = tile >= 0 ? tile : pick_tile(std::max<long>(M, 1), std::max(Cout, 1));
  out[0] = splits;
  out[1] = tile;
  out[2] = (int)(((M + kTiles[tt].bm - 1) / kTiles[tt].bm) * ((Cout + kTiles[tt].bn - 1) / kTiles[tt].bn));
  return 0;
}

// Split-K factor seg_conv_igemm_act should be given for this conv (1 = none); the
// workspace is splits * N*Ho*Wo * Cout floats.
SEG_API int seg_conv_igemm_splits(long M, int Cout, int Cin, int ks) {
  if (M <= 0 || Cout <= 0 || Cin <= 0) return 1;
  return igemm_splits(M, Cout, ks * ks * Cin);
}

// Tuning hook: force tile configuration t (0..7, see kTiles) for every following
// seg_conv_igemm / seg_conv_igemm_row_tiles call of this process; -1 restores the
// cost model.  Tile choice never changes results (each output is the same
// k-ordered fmaf chain) except the BN-statistics tile partition.
SEG_API int seg_igemm_force_tile(int t) {
  if (t < -1 || t >= (int)(sizeof(kTiles) / sizeof(kTiles[0]))) return (int)hipErrorInvalidValue;
  seg_igemm_forced_tile = t;
  return 0;
}

// Row tiling seg_conv_igemm uses for an M x Cout output: returns the number of
// row tiles (= rows of its optional BN-statistics partials) and their height.
SEG_API int seg_conv_igemm_row_tiles(long M, int Cout, int* tile_rows) {
  const int bm = kTileBM[pick_tile(M, Cout)];
  if (tile_rows) *tile_rows = bm;
  return (int)((M + bm - 1) / bm);
}

// Pack a PyTorch conv weight w[Cout][Cin][ks][ks] for seg_conv_igemm.
//   mode 0 (forward):   wk[co][tap*Cin + ci]          = w[co][ci][tap]
//   mode 1 (data-grad): wk[ci][tap*Cout + co]          = w[co][ci][ks*ks-1-tap]
// The K run of each tap is padded with zeros to kin_pad channels (>= Cin in
// mode 0, >= Cout in mode 1), so a GEMM whose input has a padded channel count
// stays float4-aligned: the Cin = 3 image (stored NHWC4) and the dY of the
// C = 10 head.  Rows are zero-padded from taps*kin_pad to ldk.
__global__ void pack_conv_weight_kernel(const float* __restrict__ w, float* __restrict__ wk,
                                        int Cout, int Cin, int taps, int ldk, int mode, int kin_pad) {
  const int rows = mode == 0 ? Cout : Cin;
  const int kin = kin_pad;
  const long total = (long)rows * ldk;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / ldk), k = (int)(i - (long)r * ldk);
    float v = 0.f;
    if (k < taps * kin) {
      const int tap = k / kin, c = k - tap * kin;
      if (mode == 0) { if (c < Cin) v = w[((long)r * Cin + c) * taps + tap]; }
      else if (c < Cout) v = w[((long)c * Cin + r) * taps + (taps - 1 - tap)];
    }
    wk[i] = v;
  }
}

SEG_API int seg_pack_conv_weight(const float* w, float* wk, int Cout, int Cin, int ks, int ldk, int mode,
                                 int kin_pad, hipStream_t stream) {
  if (kin_pad < (mode == 0 ? Cin : Cout)) return (int)hipErrorInvalidValue;
  if (ldk < ks * ks * kin_pad) return (int)hipErrorInvalidValue;
  const long total = (long)(mode == 0 ? Cout : Cin) * ldk;
  const int grid = (int)std::min<long>(seg_cdiv(total, 256), 4096);
  hipLaunchKernelGGL(pack_conv_weight_kernel, dim3(grid), dim3(256), 0, stream, w, wk, Cout, Cin, ks * ks, ldk, mode, kin_pad);
  SEG_RET_LAST();
}

// ---------------------------------------------------------------- batched packing
// Every weight repack of a training step (forward mode 0, data-gradient mode 1,
// depthwise mode 2 = [9][C]) in ONE launch: blockIdx.y = job, blockIdx.x
// strides over the job's elements.  The job table lives in device memory and
// stays valid while the weight storage does (the engine builds it once per
// program and re-uploads only when a weight pointer changes).
struct SegPackJob {
  const float* w;
  float* wk;
  int cout, cin, ks, ldk, mode, kin_pad;
  int blk0, nblk;  // this job's block range of the launch
};
static_assert(sizeof(SegPackJob) == 48, "seg_pack_job ABI");

// One element per thread over a 1-D grid partitioned between the jobs by the host
// (job.blk0 / job.nblk: blocks proportional to each job's size -- the big decoder
// weights get thousands of blocks instead of the 64 a fixed per-job grid gave them).
__global__ __launch_bounds__(256) void pack_batch_kernel(const SegPackJob* __restrict__ jobs, int njobs) {
  int lo = 0, hi = njobs - 1;  // the job whose block range holds blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].blk0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const SegPackJob j = jobs[lo];
  const long i = ((long)blockIdx.x - j.blk0) * 256 + threadIdx.x;
  const int taps = j.ks * j.ks;
  if (j.mode == 2) {
    if (i >= 9L * j.cout) return;
    const int tap = (int)(i / j.cout), c = (int)(i - (long)tap * j.cout);
    j.wk[i] = j.w[c * 9 + tap];
    return;
  }
  if (j.mode == 3 || j.mode == 4) {
    // Winograd F(2x2,3x3) filter transform U = G g G^T (wino.hip): [16][rows][ldk];
    // mode 3 forward (rows = Cout, k = Cin), mode 4 data gradient (rows = Cin,
    // k = Cout, g = the transposed, flipped filter)
    const int rows = j.mode == 3 ? j.cout : j.cin;
    if (i >= (long)rows * j.ldk) return;
    const int r = (int)(i / j.ldk), k = (int)(i - (long)r * j.ldk);
    const bool in = k < (j.mode == 3 ? j.cin : j.cout);
    float g[3][3];
#pragma unroll
    for (int y = 0; y < 3; ++y)
#pragma unroll
      for (int x = 0; x < 3; ++x)
        g[y][x] = !in ? 0.f
                      : j.mode == 3 ? j.w[(((long)r * j.cin + k) * 3 + y) * 3 + x]
                                    : j.w[(((long)k * j.cin + r) * 3 + (2 - y)) * 3 + (2 - x)];
    float h[4][3];  // G g
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      h[0][x] = g[0][x];
      h[1][x] = 0.5f * (g[0][x] + g[1][x] + g[2][x]);
      h[2][x] = 0.5f * (g[0][x] - g[1][x] + g[2][x]);
      h[3][x] = g[2][x];
    }
    const long plane = (long)rows * j.ldk;
#pragma unroll
    for (int y = 0; y < 4; ++y) {  // (G g) G^T
      const float u[4] = {h[y][0], 0.5f * (h[y][0] + h[y][1] + h[y][2]), 0.5f * (h[y][0] - h[y][1] + h[y][2]),
                          h[y][2]};
#pragma unroll
      for (int x = 0; x < 4; ++x) j.wk[(y * 4 + x) * plane + i] = u[x];
    }
    return;
  }
  // modes 0 / 1; | 16: bf16 output (RNE; the _w16 GEMM entry points)
  const int mode = j.mode & 15;
  const int rows = mode == 0 ? j.cout : j.cin;
  if (i >= (long)rows * j.ldk) return;
  const int r = (int)(i / j.ldk), k = (int)(i - (long)r * j.ldk);
  float v = 0.f;
  if (k < taps * j.kin_pad) {
    const int tap = k / j.kin_pad, c = k - tap * j.kin_pad;
    if (mode == 0) { if (c < j.cin) v = j.w[((long)r * j.cin + c) * taps + tap]; }
    else if (c < j.cout) v = j.w[((long)c * j.cin + r) * taps + (taps - 1 - tap)];
  }
  if (j.mode & 16) reinterpret_cast<__bf16*>(j.wk)[i] = static_cast<__bf16>(v);
  else j.wk[i] = v;
}

// jobs: device array of njobs seg_pack_job, sorted by blk0, job k owning blocks
// [blk0, blk0 + nblk) with nblk = ceil(elements / 256); nblocks = the sum.
SEG_API int seg_pack_batch(const void* jobs, int njobs, long nblocks, hipStream_t stream) {
  if (njobs < 0 || nblocks < 0 || nblocks > INT32_MAX) return (int)hipErrorInvalidValue;
  if (njobs == 0 || nblocks == 0) return 0;
  hipLaunchKernelGGL(pack_batch_kernel, dim3((unsigned)nblocks), dim3(256), 0, stream,
                     reinterpret_cast<const SegPackJob*>(jobs), njobs);
  SEG_RET_LAST();
}

