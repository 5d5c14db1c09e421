// Depthwise 3x3 convolution (stride 1 or 2, pad 1, no bias) on bf16 rows for the bf16io
// configuration, tiled through LDS by LDS-DMA: forward (+ the BatchNorm tile statistics of
// its output), data gradient and weight gradient.
//
// Replaces the groups=C Conv2d of every torchvision InvertedResidual (features[1..17],
// reached through src/unet.py:15-19,34-38) and its convolution_backward.  The
// first-generation kernels (dwconv.hip: a thread slides a strip of 4 pixels x 4 channels
// through registers, 8-byte bf16 accesses) ran the large layers at 2.5-3.3 TB/s and the small
// ones far below.  Here a block owns an output tile (8 x 32 pixels at stride 1, 4 x 32 at
// stride 2) of a 64-channel slice:
//  * the input tile with its halo ((T-1) S + 3 rows x columns, 128 bytes = 64 channels per
//    pixel) is copied global -> LDS by LDS-DMA, 16-byte slots, out-of-image pixels and channels
//    beyond C from a zero page; several blocks per CU overlap one another's copies;
//  * lazy BatchNorm (the expand conv's BN + ReLU6 on the input, the forward and the weight
//    gradient): one in-place pass over the LDS tile, in-image pixels only (padding stays zero),
//    rounded to bf16 exactly as the BN-apply pass would store it;
//  * a thread owns 8 channels (one 16-byte LDS read per tap) of one output column and walks
//    the tile's rows; lanes of a wave cover 8 channel groups x 8 consecutive columns, so the
//    stride-1 reads are bank-conflict free and every store is a 1 KB row segment;
//  * fp32 arithmetic in the tap order of dwconv.hip (row-major taps, one fma each), so the
//    forward (without lazy BN: dwconv.hip keeps the transformed input in fp32, here it is
//    bf16 as the unfused BN-apply pass stores it) and the data gradient equal the
//    first-generation kernels bit for bit;
//  * forward epilogue: BatchNorm tile partials of the output (tile sum, M2 about the tile
//    mean; [tile][2][C], tile = one output tile of T_H x 32 pixels) for seg_bn_stats_tiles --
//    the statistics pass over the depthwise output disappears (tiles must divide the image);
//  * weight gradient: a block accumulates 9 taps x 8 channels per thread over several tiles,
//    then a fixed-order reduction (wave shuffles, LDS) writes one partial slab [block][9][C]
//    for seg_conv_wgrad_reduce (mode 1): deterministic, no atomics.
#include "common.h"

namespace {

constexpr int CB = 64;      // channels per slice (128 bytes per pixel)
constexpr int TWO = 32;     // output tile width
constexpr int kThreads = 256;

__device__ __attribute__((aligned(16))) unsigned g_dw2_zero[4];

template <int S> struct Geo {
  static constexpr int THO = S == 1 ? 8 : 4;          // output tile rows
  static constexpr int IH = (THO - 1) * S + 3;        // input tile rows (with halo)
  static constexpr int IW = (TWO - 1) * S + 3;        // input tile columns
  static constexpr int SLOTS = IH * IW * (CB / 8);    // 16-byte slots
  static constexpr int DMA = (SLOTS + 63) / 64;       // DMA instructions (1 KB each)
  static constexpr int BYTES = DMA * 1024;
};

struct Dw2Args {
  const __bf16* in; long ldin;   // [N*H*W][ldin]
  const float* isc; const float* ish; int iact;  // lazy BN of the input (forward / wgrad), or null
  const float* wk;               // [9][C] fp32 (seg_pack_dw_weight)
  __bf16* out; long ldout;       // [N*Ho*Wo][ldout]
  float* stat;                   // forward: BN tile partials [tiles][2][C] or null
  const __bf16* dy; long lddy;   // wgrad: [N*Ho*Wo][lddy]
  float* part;                   // wgrad: [blocks][9][C]
  int N, H, W, C, Ho, Wo;
  int tiles_w, tiles_h, ntiles, tiles_per_block, accumulate;
  // BIN (data / weight gradient): dY formed on load by the depthwise conv's own BatchNorm
  // backward, dY = seg_bnbwd4(dA, by; bsc, bsh, bmu, bk[3][C], bact) -- the tile holds dA
  const __bf16* by; long ldby;
  const float *bsc, *bsh, *bmu, *bk; int bact;
  // BOUT (data gradient): partials (sum dz, sum dz (oy - omu)), dz = dX act'(oy osc + osh), of the
  // BatchNorm backward of the layer that produced this conv's input, per dX tile into opart
  // [tiles][2][C]; the last tile of each 64-channel slice to finish finalizes them in-launch
  // (ocoef [3][C], odgamma, odbeta: bn_bwd_finalize's outputs; ocnt [C/64] arrival counters)
  const __bf16* oy; long ldoy;
  const float *osc, *osh, *omu, *ogamma, *oinvstd; int oact;
  float *opart, *odgamma, *odbeta, *ocoef; unsigned* ocnt; long oM;
};

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {  // vmcnt(N), 6-bit field split over bits 3:0 and 15:14
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ void unpack8(const bf16x8 v, float (&o)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
}

// Copy the input tile of output tile (n, oh0, ow0), channels c0 .. c0+63, into LDS (all waves
// issue; the caller waits).  Slot u: tile pixel u >> 3, channel group u & 7.
template <int S>
__device__ __forceinline__ void load_tile(const Dw2Args& a, const __bf16* src, long ld, int n, int ih0, int iw0, int c0,
                                          char* lds) {
  using G = Geo<S>;
  const int tid = threadIdx.x;
  for (int j = tid >> 6; j < G::DMA; j += kThreads / 64) {
    const int u = 64 * j + (tid & 63);
    const int hp = u >> 3, cg = u & 7;
    const int hy = hp / G::IW, hx = hp - hy * G::IW;
    const int ih = ih0 + hy, iw = iw0 + hx, ch = c0 + 8 * cg;
    const bool ok = hp < G::IH * G::IW && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W && ch < a.C;
    dma16(ok ? (const void*)(src + ((long)(n * a.H + ih) * a.W + iw) * ld + ch) : (const void*)g_dw2_zero,
          lds + j * 1024);
  }
}

// The lazy BatchNorm of the input, in place on the LDS tile: in-image pixels of real channels only.
template <int S, int IH = Geo<S>::IH, int IW = Geo<S>::IW>
__device__ __forceinline__ void xform_tile(const Dw2Args& a, int ih0, int iw0, int c0, char* lds) {
  const int tid = threadIdx.x, cg = tid & 7, ch = c0 + 8 * cg;  // kThreads % 8 == 0: a thread keeps its group
  if (ch >= a.C) return;
  const f32x4 s0 = ld4(a.isc + ch), s1 = ld4(a.isc + ch + 4), b0 = ld4(a.ish + ch), b1 = ld4(a.ish + ch + 4);
  for (int u = tid; u < IH * IW * 8; u += kThreads) {
    const int hp = u >> 3;
    const int hy = hp / IW, hx = hp - hy * IW;
    if ((unsigned)(ih0 + hy) >= (unsigned)a.H || (unsigned)(iw0 + hx) >= (unsigned)a.W) continue;
    bf16x8* p = reinterpret_cast<bf16x8*>(lds + 16 * u);
    const bf16x8 q = *p;
    const f32x4 lo = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 0, 1, 2, 3), f32x4), s0, b0,
                                 a.iact);
    const f32x4 hi = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 4, 5, 6, 7), f32x4), s1, b1,
                                 a.iact);
    *p = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
  }
}

// BIN: the pre-BN input y of a tile whose LDS copy holds dA (TH x TW pixels from (h0, w0) of an
// Hi x Wi image), staged in registers: issue() right after the tile's copy is issued, apply()
// after the copy landed -- dY = the BatchNorm backward of each in-image slot, rounded to bf16 as
// the apply pass stores it, in place.
template <int TH, int TW>
struct BinTile {
  static constexpr int SL = TH * TW * 8;
  static constexpr int K = (SL + kThreads - 1) / kThreads;
  bf16x8 yv[K];
  __device__ __forceinline__ bool slot(const Dw2Args& a, int k, int h0, int w0, int Hi, int Wi, int c0, int& ih,
                                       int& iw) const {
    const int u = threadIdx.x + k * kThreads, hp = u >> 3;
    const int hy = hp / TW, hx = hp - hy * TW;
    ih = h0 + hy;
    iw = w0 + hx;
    return u < SL && (unsigned)ih < (unsigned)Hi && (unsigned)iw < (unsigned)Wi && c0 + 8 * (threadIdx.x & 7) < a.C;
  }
  __device__ __forceinline__ void issue(const Dw2Args& a, int n, int h0, int w0, int Hi, int Wi, int c0) {
    const int ch = c0 + 8 * (threadIdx.x & 7);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int ih, iw;
      const bool ok = slot(a, k, h0, w0, Hi, Wi, c0, ih, iw);
      yv[k] = *reinterpret_cast<const bf16x8*>(ok ? (const void*)(a.by + ((long)(n * Hi + ih) * Wi + iw) * a.ldby + ch)
                                                  : (const void*)g_dw2_zero);
    }
  }
  __device__ __forceinline__ void apply(const Dw2Args& a, int h0, int w0, int Hi, int Wi, int c0, char* lds) const {
    const int ch = c0 + 8 * (threadIdx.x & 7);
    if (ch >= a.C) return;
    f32x4 sc[2], sh[2], mu[2], k1[2], k2[2], k3[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      sc[h] = ld4(a.bsc + ch + 4 * h);
      sh[h] = ld4(a.bsh + ch + 4 * h);
      mu[h] = ld4(a.bmu + ch + 4 * h);
      k1[h] = ld4(a.bk + ch + 4 * h);
      k2[h] = ld4(a.bk + a.C + ch + 4 * h);
      k3[h] = ld4(a.bk + 2 * a.C + ch + 4 * h);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int ih, iw;
      if (!slot(a, k, h0, w0, Hi, Wi, c0, ih, iw)) continue;
      bf16x8* p = reinterpret_cast<bf16x8*>(lds + 16 * (threadIdx.x + k * kThreads));
      const bf16x8 g = *p, v = yv[k];
      const f32x4 lo = seg_bnbwd4(__builtin_convertvector(__builtin_shufflevector(g, g, 0, 1, 2, 3), f32x4),
                                  __builtin_convertvector(__builtin_shufflevector(v, v, 0, 1, 2, 3), f32x4), sc[0],
                                  sh[0], mu[0], k1[0], k2[0], k3[0], a.bact);
      const f32x4 hi = seg_bnbwd4(__builtin_convertvector(__builtin_shufflevector(g, g, 4, 5, 6, 7), f32x4),
                                  __builtin_convertvector(__builtin_shufflevector(v, v, 4, 5, 6, 7), f32x4), sc[1],
                                  sh[1], mu[1], k1[1], k2[1], k3[1], a.bact);
      *p = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
    }
  }
};

// BOUT: a thread's running (sum dz, sum dz (y - mean)) over the dX values it stores.
struct BoutAcc {
  float s0[8], s1[8];
  f32x4 sc[2], sh[2], mu[2];
  __device__ __forceinline__ void init(const Dw2Args& a, int ch) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
    if (ch < a.C) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        sc[h] = ld4(a.osc + ch + 4 * h);
        sh[h] = ld4(a.osh + ch + 4 * h);
        mu[h] = ld4(a.omu + ch + 4 * h);
      }
    }
  }
  // dx: the stored (bf16-rounded) values, y: the producer's pre-BN output at the same pixel
  __device__ __forceinline__ void add(const bf16x8 dx, const bf16x8 y, int act) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = (float)dx[j], v = (float)y[j];
      const float dz = g * seg_act_mask(v * sc[j >> 2][j & 3] + sh[j >> 2][j & 3], act);
      s0[j] += dz;
      s1[j] += dz * (v - mu[j >> 2][j & 3]);
    }
  }
};

// BOUT epilogue: the block's partials (lanes with one channel group: xor 8, 16, 32; then the 4
// waves, fixed order) into opart[t] write-through, then the last block of the channel slice sums
// all tiles' partials in tile order (fp64) and finalizes the slice's channels as
// bn_bwd_finalize_kernel does.  Every thread of the block calls it.
__device__ __forceinline__ void bout_finish(const Dw2Args& a, BoutAcc& b, int t, int ntiles, int c0, float* red,
                                            int* word) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float u = b.s0[j], v = b.s1[j];
    u += __shfl_xor(u, 8, 64);
    v += __shfl_xor(v, 8, 64);
    u += __shfl_xor(u, 16, 64);
    v += __shfl_xor(v, 16, 64);
    u += __shfl_xor(u, 32, 64);
    v += __shfl_xor(v, 32, 64);
    b.s0[j] = u;
    b.s1[j] = v;
  }
  __syncthreads();  // red may alias LDS the block just read
  if (lane < 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * 2 + 0) * CB + 8 * lane + j] = b.s0[j];
      red[(wave * 2 + 1) * CB + 8 * lane + j] = b.s1[j];
    }
  }
  __syncthreads();
  if (tid < 2 * CB) {
    const int q = tid >> 6, c = tid & 63;
    const float v = red[(0 * 2 + q) * CB + c] + red[(1 * 2 + q) * CB + c] + red[(2 * 2 + q) * CB + c] +
                    red[(3 * 2 + q) * CB + c];
    if (c0 + c < a.C) seg_st_wt(a.opart + ((long)t * 2 + q) * a.C + c0 + c, v);
  }
  if (!seg_last_arrival(a.ocnt + blockIdx.y, (unsigned)ntiles, word)) return;
  // finalize: 4 tile groups x 64 channels, fp64 in tile order, then the groups in order
  double* dred = reinterpret_cast<double*>(red);  // [4][2][CB]
  {
    const int rg = tid >> 6, c = tid & 63;
    double u = 0.0, v = 0.0;
    if (c0 + c < a.C) {
      const float* p = a.opart + c0 + c;
      int k = rg;
      for (; k + 12 < ntiles; k += 16) {
        float x0[4], x1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x0[i] = seg_ld_wt(p + (long)(k + 4 * i) * 2 * a.C);
          x1[i] = seg_ld_wt(p + ((long)(k + 4 * i) * 2 + 1) * a.C);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          u += (double)x0[i];
          v += (double)x1[i];
        }
      }
      for (; k < ntiles; k += 4) {
        u += (double)seg_ld_wt(p + (long)k * 2 * a.C);
        v += (double)seg_ld_wt(p + ((long)k * 2 + 1) * a.C);
      }
    }
    __syncthreads();
    dred[(rg * 2 + 0) * CB + c] = u;
    dred[(rg * 2 + 1) * CB + c] = v;
  }
  __syncthreads();
  if (tid < CB && c0 + tid < a.C) {
    const int c = c0 + tid;
    const double sdz = dred[0 * CB + tid] + dred[2 * CB + tid] + dred[4 * CB + tid] + dred[6 * CB + tid];
    const double sdzx = dred[1 * CB + tid] + dred[3 * CB + tid] + dred[5 * CB + tid] + dred[7 * CB + tid];
    const double inv = a.oinvstd[c];
    const double g = a.ogamma ? a.ogamma[c] : 1.0;
    if (a.odbeta) a.odbeta[c] = (float)sdz;
    if (a.odgamma) a.odgamma[c] = (float)(sdzx * inv);
    a.ocoef[c] = (float)(g * inv);
    a.ocoef[a.C + c] = (float)(sdz / (double)a.oM);
    a.ocoef[2 * a.C + c] = (float)(sdzx * inv * inv / (double)a.oM);
  }
}

// Forward (FLIP = 0) or stride-1 data gradient (FLIP = 1: the correlation of dY with the
// flipped kernel; ACC: add into out).  STATS: BatchNorm tile partials of the output.
//
// Stride-1 data gradient only: BIN forms dY on load (the tile holds dA), BOUT accumulates the
// producer's BatchNorm-backward partials over the stored dX.
template <int S, bool LAZY, bool FLIP, bool STATS, bool BIN = false, bool BOUT = false>
__global__ __launch_bounds__(kThreads) void dw2_fwd_kernel(Dw2Args a) {
  using G = Geo<S>;
  static_assert(!(BIN || BOUT) || (FLIP && S == 1 && !LAZY && !STATS), "BN-backward fusions: the s1 data gradient");
  __shared__ __attribute__((aligned(1024))) char tile[G::BYTES];
  __shared__ float red[2][4][CB];
  __shared__ int word;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo rows) on one XCD
  const int c0 = blockIdx.y * CB;
  const int tw_i = t % a.tiles_w, rest = t / a.tiles_w;
  const int th_i = rest % a.tiles_h, n = rest / a.tiles_h;
  const int oh0 = th_i * G::THO, ow0 = tw_i * TWO;
  const int ih0 = oh0 * S - 1, iw0 = ow0 * S - 1;
  load_tile<S>(a, a.in, a.ldin, n, ih0, iw0, c0, tile);
  BinTile<G::IH, G::IW> bin;
  if constexpr (BIN) bin.issue(a, n, ih0, iw0, a.H, a.W, c0);
  const int cg = lane & 7, col = wave * 8 + (lane >> 3), ch = c0 + 8 * cg;
  float w[9][8] = {};
  if (ch < a.C) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const f32x4 lo = ld4(a.wk + (FLIP ? 8 - k : k) * a.C + ch), hi = ld4(a.wk + (FLIP ? 8 - k : k) * a.C + ch + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[k][j] = lo[j];
        w[k][4 + j] = hi[j];
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this thread's DMA (and weight loads) landed
  __syncthreads();
  if constexpr (LAZY) {
    xform_tile<S>(a, ih0, iw0, c0, tile);
    __syncthreads();
  }
  if constexpr (BIN) {
    bin.apply(a, ih0, iw0, a.H, a.W, c0, tile);
    __syncthreads();
  }
  const int ow = ow0 + col;
  const bool live = ch < a.C && ow < a.Wo;
  BoutAcc bo;
  bf16x8 oyv[G::THO];
  if constexpr (BOUT) {  // the producer's pre-BN output at this thread's dX pixels, in flight during the taps
    bo.init(a, ch);
#pragma unroll
    for (int r = 0; r < G::THO; ++r) {
      const bool ok = live && oh0 + r < a.Ho;
      oyv[r] = *reinterpret_cast<const bf16x8*>(
          ok ? (const void*)(a.oy + ((long)(n * a.Ho + oh0 + r) * a.Wo + ow) * a.ldoy + ch) : (const void*)g_dw2_zero);
    }
  }
  auto store_row = [&](int r, float (&v)[8]) {
    __bf16* dst = a.out + ((long)(n * a.Ho + oh0 + r) * a.Wo + ow) * a.ldout + ch;
    if (a.accumulate) {  // (data gradient) the value already there, widened exactly
      float old[8];
      unpack8(*reinterpret_cast<const bf16x8*>(dst), old);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += old[j];
    }
    const f32x4 lo = {v[0], v[1], v[2], v[3]}, hi = {v[4], v[5], v[6], v[7]};
    const bf16x8 q = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
    *reinterpret_cast<bf16x8*>(dst) = q;
    if constexpr (BOUT) bo.add(q, oyv[r], a.oact);
  };
  float o[STATS ? G::THO : 1][8];
#pragma unroll
  for (int r = 0; r < G::THO; ++r) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        float v[8];
        unpack8(*reinterpret_cast<const bf16x8*>(tile + 128 * ((r * S + ky) * G::IW + col * S + kx) + 16 * cg), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(v[j], w[ky * 3 + kx][j], acc[j]);
      }
    if constexpr (STATS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[r][j] = acc[j];
    } else if (live && oh0 + r < a.Ho) {
      store_row(r, acc);
    }
  }
  if constexpr (STATS) {
    // tile sum, then M2 about the tile mean, per channel (the tile divides the image: every
    // output pixel of it is real); lanes with the same channel group: xor 8, 16, 32
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      float part[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.f;
        const float mu = pass ? red[0][0][8 * cg + j] : 0.f;
#pragma unroll
        for (int r = 0; r < G::THO; ++r) {
          const float d = o[r][j] - mu;
          s += pass ? d * d : d;
        }
        s += __shfl_xor(s, 8, 64);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        part[j] = s;
      }
      if (lane < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[pass][wave][8 * lane + j] = part[j];
      }
      __syncthreads();
      if (tid < CB) {
        const float tot = red[pass][0][tid] + red[pass][1][tid] + red[pass][2][tid] + red[pass][3][tid];
        if (c0 + tid < a.C) a.stat[((long)t * 2 + pass) * a.C + c0 + tid] = tot;
        if (pass == 0) red[0][0][tid] = tot / (float)(G::THO * TWO);  // tile mean (read in pass 1)
      }
      if (pass == 0) __syncthreads();
    }
    if (live) {
#pragma unroll
      for (int r = 0; r < G::THO; ++r) store_row(r, o[r]);
    }
  }
  if constexpr (BOUT) bout_finish(a, bo, t, gridDim.x, c0, reinterpret_cast<float*>(tile), &word);
}

// Stride-2 data gradient: dX tile 8 x 32 of a 64-channel slice from the dY rows / columns
// that reach it (5 x 17), summed in the tap order of dwconv.hip's dw_dgrad_s2_kernel.  BIN / BOUT
// as dw2_fwd_kernel's.
template <bool BIN, bool BOUT>
__global__ __launch_bounds__(kThreads) void dw2_dgrad_s2_kernel(Dw2Args a) {
  constexpr int THX = 8, DH = 5, DW = 17;
  __shared__ __attribute__((aligned(1024))) char tile[((DH * DW * 8 + 63) / 64) * 1024];
  __shared__ int word;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int c0 = blockIdx.y * CB;
  const int tw_i = t % a.tiles_w, rest = t / a.tiles_w;
  const int th_i = rest % a.tiles_h, n = rest / a.tiles_h;
  const int h0 = th_i * THX, w0 = tw_i * TWO;  // dX tile origin (even)
  const int oh0 = h0 / 2, ow0 = w0 / 2;       // first dY row / column that reaches it
  for (int j = tid >> 6; j < (DH * DW * 8 + 63) / 64; j += kThreads / 64) {
    const int u = 64 * j + (tid & 63);
    const int hp = u >> 3, cg = u & 7;
    const int hy = hp / DW, hx = hp - hy * DW;
    const int oh = oh0 + hy, ow = ow0 + hx, ch = c0 + 8 * cg;
    const bool ok = hp < DH * DW && oh < a.Ho && ow < a.Wo && ch < a.C;
    dma16(ok ? (const void*)(a.in + ((long)(n * a.Ho + oh) * a.Wo + ow) * a.ldin + ch) : (const void*)g_dw2_zero,
          tile + j * 1024);
  }
  BinTile<DH, DW> bin;
  if constexpr (BIN) bin.issue(a, n, oh0, ow0, a.Ho, a.Wo, c0);
  const int cg = lane & 7, col = wave * 8 + (lane >> 3), ch = c0 + 8 * cg;
  const int wq = w0 + col;  // dX column
  const bool live = ch < a.C && wq < a.W;
  float w[9][8] = {};
  if (ch < a.C) {
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const f32x4 lo = ld4(a.wk + k * a.C + ch), hi = ld4(a.wk + k * a.C + ch + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w[k][j] = lo[j];
        w[k][4 + j] = hi[j];
      }
    }
  }
  BoutAcc bo;
  bf16x8 oyv[THX];
  if constexpr (BOUT) {
    bo.init(a, ch);
#pragma unroll
    for (int r = 0; r < THX; ++r) {
      const bool ok = live && h0 + r < a.H;
      oyv[r] = *reinterpret_cast<const bf16x8*>(
          ok ? (const void*)(a.oy + ((long)(n * a.H + h0 + r) * a.W + wq) * a.ldoy + ch) : (const void*)g_dw2_zero);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  if constexpr (BIN) {
    bin.apply(a, oh0, ow0, a.Ho, a.Wo, c0, tile);
    __syncthreads();
  }
  auto dyv = [&](int oh_l, int ow_l, float (&v)[8]) {  // dY at local (row, col); zero outside dY
    unpack8(*reinterpret_cast<const bf16x8*>(tile + 128 * (oh_l * DW + ow_l) + 16 * cg), v);
  };
  const int j0 = col >> 1;  // local dY column of this dX column pair
  const bool oddw = col & 1;
  if (live) {
#pragma unroll
    for (int r = 0; r < THX; ++r) {
      const int hq = h0 + r;
      if (hq >= a.H) break;
      const bool odd = hq & 1;
      // row slots: slot 0 = (even: ky 1, ho hq/2 | odd: ky 0, ho (hq+1)/2), slot 1 = (odd: ky 2, ho (hq-1)/2)
      const int ky0 = odd ? 0 : 1;
      const int l0 = (odd ? (hq + 1) >> 1 : hq >> 1) - oh0, l1 = ((hq - 1) >> 1) - oh0;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        if (sl == 1 && !odd) break;
        const int ky = sl == 0 ? ky0 : 2, lr = sl == 0 ? l0 : l1;
        float d[8], d1[8];
        dyv(lr, j0, d);
        if (!oddw) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(d[j], w[ky * 3 + 1][j], acc[j]);
        } else {
          dyv(lr, j0 + 1, d1);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc[j] = fmaf(d1[j], w[ky * 3 + 0][j], acc[j]);
            acc[j] = fmaf(d[j], w[ky * 3 + 2][j], acc[j]);
          }
        }
      }
      __bf16* dst = a.out + ((long)(n * a.H + hq) * a.W + wq) * a.ldout + ch;
      if (a.accumulate) {
        float old[8];
        unpack8(*reinterpret_cast<const bf16x8*>(dst), old);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += old[j];
      }
      const f32x4 lo = {acc[0], acc[1], acc[2], acc[3]}, hi = {acc[4], acc[5], acc[6], acc[7]};
      const bf16x8 q = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
      *reinterpret_cast<bf16x8*>(dst) = q;
      if constexpr (BOUT) bo.add(q, oyv[r], a.oact);
    }
  }
  if constexpr (BOUT) bout_finish(a, bo, t, gridDim.x, c0, reinterpret_cast<float*>(tile), &word);
}

// Weight gradient: part[block][tap][C] = sum over the block's tiles of dY[p][c] X[p S + tap - 1][c].
// A block walks a run of consecutive output tiles (THO = 8 rows at stride 1, 2 at stride 2, so
// that two stages fit in LDS): the next tile's X halo and dY rows are copied by LDS-DMA while
// the current one is accumulated (a thread: 9 taps x 8 channels of one column).
template <int S, bool BIN = false> struct WGeo {
  static constexpr int THO = S == 1 ? (BIN ? 4 : 8) : 2;
  static constexpr int IH = (THO - 1) * S + 3, IW = (TWO - 1) * S + 3;
  static constexpr int DMAX = (IH * IW * 8 + 63) / 64;
  static constexpr int DMAY = THO * TWO * 8 / 64;
  static constexpr int XB = DMAX * 1024, YB = DMAY * 1024;
  static constexpr int STAGE = XB + YB * (BIN ? 2 : 1);     // BIN: dA and the pre-BN y rows
  static constexpr int MINW = DMAX / 4 + (BIN ? 2 : 1) * (DMAY / 4);  // fewest copies one wave issues per stage
};

// BIN: dY = the depthwise conv's own BatchNorm backward of (dA, y), formed in the stage in place.
template <int S, bool LAZY, bool BIN>
__global__ __launch_bounds__(kThreads) void dw2_wgrad_kernel(Dw2Args a) {
  using G = WGeo<S, BIN>;
  static_assert(2 * G::STAGE <= 160 * 1024 && 4 * 9 * CB * 4 <= 2 * G::STAGE, "two stages (and the reduction) fit");
  __shared__ __attribute__((aligned(1024))) char buf[2 * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = xcd_swizzle(blockIdx.x, gridDim.x);
  const int c0 = blockIdx.y * CB;
  const int cg = lane & 7, col = wave * 8 + (lane >> 3);
  float acc[9][8];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
  const int tb = b * a.tiles_per_block, te = min(a.ntiles, tb + a.tiles_per_block);
  auto origin = [&](int t, int& n, int& oh0, int& ow0) {
    const int tw_i = t % a.tiles_w, rest = t / a.tiles_w;
    oh0 = (rest % a.tiles_h) * G::THO;
    n = rest / a.tiles_h;
    ow0 = tw_i * TWO;
  };
  auto rows_dma = [&](const __bf16* src, long ld, int n, int oh0, int ow0, char* dst) {  // pixel u >> 3, group u & 7
    for (int j = wave; j < G::DMAY; j += kThreads / 64) {
      const int u = 64 * j + lane;
      const int px = u >> 3, g8 = u & 7;
      const int r = px / TWO, cc = px - r * TWO;
      const int oh = oh0 + r, ow = ow0 + cc, c8 = c0 + 8 * g8;
      const bool ok = oh < a.Ho && ow < a.Wo && c8 < a.C;
      dma16(ok ? (const void*)(src + ((long)(n * a.Ho + oh) * a.Wo + ow) * ld + c8) : (const void*)g_dw2_zero,
            dst + j * 1024);
    }
  };
  auto issue = [&](int t, char* st) {
    int n, oh0, ow0;
    origin(t, n, oh0, ow0);
    const int ih0 = oh0 * S - 1, iw0 = ow0 * S - 1;
    for (int j = wave; j < G::DMAX; j += kThreads / 64) {
      const int u = 64 * j + lane;
      const int hp = u >> 3, g8 = u & 7;
      const int hy = hp / G::IW, hx = hp - hy * G::IW;
      const int ih = ih0 + hy, iw = iw0 + hx, c8 = c0 + 8 * g8;
      const bool ok = hp < G::IH * G::IW && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W && c8 < a.C;
      dma16(ok ? (const void*)(a.in + ((long)(n * a.H + ih) * a.W + iw) * a.ldin + c8) : (const void*)g_dw2_zero,
            st + j * 1024);
    }
    rows_dma(a.dy, a.lddy, n, oh0, ow0, st + G::XB);
    if constexpr (BIN) rows_dma(a.by, a.ldby, n, oh0, ow0, st + G::XB + G::YB);
  };
  if (tb < te) issue(tb, buf);
  for (int t = tb, i = 0; t < te; ++t, ++i) {
    char* st = buf + (i & 1) * G::STAGE;
    if (t + 1 < te) {
      issue(t + 1, buf + ((i + 1) & 1) * G::STAGE);  // that stage was released by the barrier ending tile t-1
      wait_vm<G::MINW>();
    } else {
      wait_vm<0>();
    }
    __syncthreads();
    if constexpr (LAZY || BIN) {
      int n, oh0, ow0;
      origin(t, n, oh0, ow0);
      if constexpr (LAZY) xform_tile<S, G::IH, G::IW>(a, oh0 * S - 1, ow0 * S - 1, c0, st);
      if constexpr (BIN) {  // dY rows: in-image pixels of real channels (the rest stays zero)
        const int ch = c0 + 8 * (tid & 7);
        if (ch < a.C) {
          f32x4 sc[2], sh[2], mu[2], k1[2], k2[2], k3[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            sc[h] = ld4(a.bsc + ch + 4 * h);
            sh[h] = ld4(a.bsh + ch + 4 * h);
            mu[h] = ld4(a.bmu + ch + 4 * h);
            k1[h] = ld4(a.bk + ch + 4 * h);
            k2[h] = ld4(a.bk + a.C + ch + 4 * h);
            k3[h] = ld4(a.bk + 2 * a.C + ch + 4 * h);
          }
          for (int u = tid; u < G::THO * TWO * 8; u += kThreads) {
            const int px = u >> 3, r = px / TWO, cc = px - r * TWO;
            if (oh0 + r >= a.Ho || ow0 + cc >= a.Wo) continue;
            bf16x8* p = reinterpret_cast<bf16x8*>(st + G::XB + 16 * u);
            const bf16x8 g = *p, v = *reinterpret_cast<const bf16x8*>(st + G::XB + G::YB + 16 * u);
            const f32x4 lo = seg_bnbwd4(__builtin_convertvector(__builtin_shufflevector(g, g, 0, 1, 2, 3), f32x4),
                                        __builtin_convertvector(__builtin_shufflevector(v, v, 0, 1, 2, 3), f32x4),
                                        sc[0], sh[0], mu[0], k1[0], k2[0], k3[0], a.bact);
            const f32x4 hi = seg_bnbwd4(__builtin_convertvector(__builtin_shufflevector(g, g, 4, 5, 6, 7), f32x4),
                                        __builtin_convertvector(__builtin_shufflevector(v, v, 4, 5, 6, 7), f32x4),
                                        sc[1], sh[1], mu[1], k1[1], k2[1], k3[1], a.bact);
            *p = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
          }
        }
      }
      __syncthreads();
    }
    const char* xt = st;
    const char* dyt = st + G::XB;
#pragma unroll 2
    for (int r = 0; r < G::THO; ++r) {
      float d[8];
      unpack8(*reinterpret_cast<const bf16x8*>(dyt + 128 * (r * TWO + col) + 16 * cg), d);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          float v[8];
          unpack8(*reinterpret_cast<const bf16x8*>(xt + 128 * ((r * S + ky) * G::IW + col * S + kx) + 16 * cg), v);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[ky * 3 + kx][j] = fmaf(d[j], v[j], acc[ky * 3 + kx][j]);
        }
    }
    __syncthreads();  // stage free for the copy issued next iteration
  }
  // fixed-order reduction over the 32 columns: lanes xor 8, 16, 32, then the 4 waves
  float* red = reinterpret_cast<float*>(buf);  // [4][9][CB], the stages are idle now
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = acc[k][j];
      s += __shfl_xor(s, 8, 64);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 8) red[(wave * 9 + k) * CB + 8 * lane + j] = s;
    }
  __syncthreads();
  for (int i = tid; i < 9 * CB; i += kThreads) {
    const int k = i / CB, c = i - k * CB;
    if (c0 + c < a.C)
      a.part[((long)blockIdx.x * 9 + k) * a.C + c0 + c] =
          red[(0 * 9 + k) * CB + c] + red[(1 * 9 + k) * CB + c] + red[(2 * 9 + k) * CB + c] + red[(3 * 9 + k) * CB + c];
  }
}

int dw2_tiles(int S, int N, int Ho, int Wo, int* tw, int* th) {
  const int tho = S == 1 ? 8 : 4;
  *tw = (Wo + TWO - 1) / TWO;
  *th = (Ho + tho - 1) / tho;
  return N * *tw * *th;
}

}  // namespace

// 1 when the seg_dw2_*_bf16io kernels apply: stride 1 or 2, C % 8 == 0, 16-byte rows.
SEG_API int seg_dw2_ok(int C, int stride) { return (C > 0 && C % 8 == 0 && (stride == 1 || stride == 2)) ? 1 : 0; }

// Output tiles of seg_dw2_fwd_bf16io (its BN partials' row tiles) and their rows; 0 when the
// tiles do not divide the Ho x Wo image (no statistics from the forward then).
SEG_API int seg_dw2_stat_tiles(int N, int Ho, int Wo, int stride, int* tile_rows) {
  const int tho = stride == 1 ? 8 : 4;
  if (tile_rows) *tile_rows = tho * TWO;
  if (Ho % tho || Wo % TWO) return 0;
  int tw, th;
  return dw2_tiles(stride, N, Ho, Wo, &tw, &th);
}

// Forward: out = dwconv3x3(act(in * in_scale + in_shift) if in_scale else in, wk), stride 1 or 2,
// pad 1; bf16 rows (ld % 8 == 0, 16-byte aligned); stat (optional, only when seg_dw2_stat_tiles > 0):
// BN tile partials [tiles][2][C].
SEG_API int seg_dw2_fwd_bf16io(const __bf16* in, long ldin, int N, int H, int W, int C, const float* in_scale,
                               const float* in_shift, int in_act, const float* wk, __bf16* out, long ldout, int Ho,
                               int Wo, int stride, float* stat, hipStream_t stream) {
  if (!seg_dw2_ok(C, stride) || (ldin & 7) || (ldout & 7) || ((uintptr_t)in & 15) || ((uintptr_t)out & 15) ||
      ((in_scale == nullptr) != (in_shift == nullptr)) || Ho != (H - 1) / stride + 1 || Wo != (W - 1) / stride + 1 ||
      (stat && !seg_dw2_stat_tiles(N, Ho, Wo, stride, nullptr)))
    return (int)hipErrorInvalidValue;
  Dw2Args a{};
  a.in = in; a.ldin = ldin; a.isc = in_scale; a.ish = in_shift; a.iact = in_act; a.wk = wk; a.out = out;
  a.ldout = ldout; a.stat = stat; a.N = N; a.H = H; a.W = W; a.C = C; a.Ho = Ho; a.Wo = Wo;
  a.ntiles = dw2_tiles(stride, N, Ho, Wo, &a.tiles_w, &a.tiles_h);
  const dim3 grid(a.ntiles, (C + CB - 1) / CB);
  const bool lazy = in_scale != nullptr, st = stat != nullptr;
#define SEG_DW2F(S, L, T) hipLaunchKernelGGL((dw2_fwd_kernel<S, L, false, T>), grid, dim3(kThreads), 0, stream, a)
  if (stride == 1) {
    if (lazy) { if (st) SEG_DW2F(1, true, true); else SEG_DW2F(1, true, false); }
    else { if (st) SEG_DW2F(1, false, true); else SEG_DW2F(1, false, false); }
  } else {
    if (lazy) { if (st) SEG_DW2F(2, true, true); else SEG_DW2F(2, true, false); }
    else { if (st) SEG_DW2F(2, false, true); else SEG_DW2F(2, false, false); }
  }
#undef SEG_DW2F
  SEG_RET_LAST();
}

static bool al16(const void* p, long ld) { return p == nullptr || (((uintptr_t)p & 15) == 0 && (ld & 7) == 0); }

// dX tiles of the data gradient (8 x 32 pixels of the H x W input image per 64-channel slice):
// the rows of seg_dw2_dgrad_bn_bf16io's opart.
SEG_API int seg_dw2_dgrad_tiles(int N, int H, int W) { return N * ((H + 7) / 8) * ((W + TWO - 1) / TWO); }

// Data gradient: dx (+)= the input gradient of the stride-1/2 depthwise conv, with two optional
// BatchNorm-backward fusions (either pointer group NULL to skip it):
//  * BIN (by != NULL): dy holds dA, the gradient of this conv's BN + act output; the conv's own
//    BatchNorm backward, dY = seg_bnbwd4(dA, by; bscale, bshift, bmean, bcoef, bact) with bcoef =
//    [3][C] from seg_bn_bwd_coef_*, is formed on load (bitwise the seg_bn_backward apply pass's
//    bf16 output) and never stored;
//  * BOUT (oy != NULL): dx is dA of the producer of this conv's input (pre-BN output oy, its BN
//    coefficients oscale / oshift / omean / ogamma / oinvstd, act oact over M = N*H*W rows): the
//    partials of its BatchNorm backward come out of this launch's epilogue (opart: [tiles][2][C],
//    tiles = seg_dw2_dgrad_tiles) and the last tile of each 64-channel slice finalizes them --
//    odgamma, odbeta (may be NULL) and ocoef [3][C] as seg_bn_bwd_coef_* would write them
//    (fixed-order fp64 sums: deterministic).  ocnt: C/64 (rounded up) counters, zero before the first
//    launch, re-armed by each launch.
SEG_API int seg_dw2_dgrad_bn_bf16io(const __bf16* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk,
                                    __bf16* dx, long lddx, int H, int W, int stride, int accumulate, const __bf16* by,
                                    long ldby, const float* bscale, const float* bshift, const float* bmean,
                                    const float* bcoef, int bact, const __bf16* oy, long ldoy, const float* oscale,
                                    const float* oshift, const float* omean, const float* ogamma,
                                    const float* oinvstd, int oact, float* opart, float* odgamma, float* odbeta,
                                    float* ocoef, unsigned* ocnt, hipStream_t stream) {
  if (!seg_dw2_ok(C, stride) || !dy || !dx || !al16(dy, lddy) || !al16(dx, lddx) || !al16(by, ldby) ||
      !al16(oy, ldoy) || Ho != (H - 1) / stride + 1 || Wo != (W - 1) / stride + 1 ||
      (by && (!bscale || !bshift || !bmean || !bcoef)) ||
      (oy && (!oscale || !oshift || !omean || !oinvstd || !opart || !ocoef || !ocnt)))
    return (int)hipErrorInvalidValue;
  Dw2Args a{};
  a.in = dy; a.ldin = lddy; a.wk = wk; a.out = dx; a.ldout = lddx; a.N = N; a.C = C; a.accumulate = accumulate;
  a.by = by; a.ldby = ldby; a.bsc = bscale; a.bsh = bshift; a.bmu = bmean; a.bk = bcoef; a.bact = bact;
  a.oy = oy; a.ldoy = ldoy; a.osc = oscale; a.osh = oshift; a.omu = omean; a.ogamma = ogamma; a.oinvstd = oinvstd;
  a.oact = oact; a.opart = opart; a.odgamma = odgamma; a.odbeta = odbeta; a.ocoef = ocoef; a.ocnt = ocnt;
  a.oM = (long)N * H * W;
  const bool bi = by != nullptr, bo = oy != nullptr;
  if (stride == 1) {  // the flipped-kernel correlation of dY, same geometry as the forward
    a.H = Ho; a.W = Wo; a.Ho = H; a.Wo = W;
    a.ntiles = dw2_tiles(1, N, H, W, &a.tiles_w, &a.tiles_h);
    const dim3 grid(a.ntiles, (C + CB - 1) / CB);
#define SEG_DW2D(B, O) hipLaunchKernelGGL((dw2_fwd_kernel<1, false, true, false, B, O>), grid, dim3(kThreads), 0, stream, a)
    if (bi) { if (bo) SEG_DW2D(true, true); else SEG_DW2D(true, false); }
    else { if (bo) SEG_DW2D(false, true); else SEG_DW2D(false, false); }
#undef SEG_DW2D
  } else {
    a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo;
    a.tiles_w = (W + TWO - 1) / TWO;
    a.tiles_h = (H + 7) / 8;
    a.ntiles = N * a.tiles_w * a.tiles_h;
    const dim3 grid(a.ntiles, (C + CB - 1) / CB);
#define SEG_DW2D(B, O) hipLaunchKernelGGL((dw2_dgrad_s2_kernel<B, O>), grid, dim3(kThreads), 0, stream, a)
    if (bi) { if (bo) SEG_DW2D(true, true); else SEG_DW2D(true, false); }
    else { if (bo) SEG_DW2D(false, true); else SEG_DW2D(false, false); }
#undef SEG_DW2D
  }
  SEG_RET_LAST();
}

// Data gradient: dx (+)= the input gradient of the stride-1/2 depthwise conv (arguments as seg_dw_dgrad).
SEG_API int seg_dw2_dgrad_bf16io(const __bf16* dy, long lddy, int N, int Ho, int Wo, int C, const float* wk,
                                 __bf16* dx, long lddx, int H, int W, int stride, int accumulate, hipStream_t stream) {
  return seg_dw2_dgrad_bn_bf16io(dy, lddy, N, Ho, Wo, C, wk, dx, lddx, H, W, stride, accumulate, nullptr, 0, nullptr,
                                 nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 0, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

static int dw2_wgrad_tho(int stride, int bin) {
  return stride == 1 ? (bin ? WGeo<1, true>::THO : WGeo<1>::THO) : WGeo<2>::THO;
}

// Weight-gradient blocks (partial slabs) of seg_dw2_wgrad_bf16io (bin = 0) / seg_dw2_wgrad_bn_bf16io
// (bin = 1): about one block per CU over all 64-channel slices (one block fills a CU's LDS), each a
// run of consecutive tiles.
SEG_API long seg_dw2_wgrad_blocks(int N, int Ho, int Wo, int C, int stride, int bin) {
  const int tho = dw2_wgrad_tho(stride, bin);
  const long nt = (long)N * ((Ho + tho - 1) / tho) * ((Wo + TWO - 1) / TWO);
  const int slices = (C + CB - 1) / CB;
  const long target = std::max(1, seg_num_cus() / slices);
  const long per = std::max<long>(1, (nt + target - 1) / target);
  return (nt + per - 1) / per;
}

// part[blocks][9][C] (blocks = seg_dw2_wgrad_blocks(..., by != NULL)) of the depthwise weight
// gradient; reduce with seg_conv_wgrad_reduce(part, blocks, dw, C, 1, 3, 1, acc).  Lazy BN of x as
// seg_dw_wgrad; BIN (by != NULL) as seg_dw2_dgrad_bn_bf16io's: dy holds dA and dY is formed on load.
SEG_API int seg_dw2_wgrad_bn_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W, int C,
                                    const float* in_scale, const float* in_shift, int in_act, int Ho, int Wo,
                                    int stride, float* part, const __bf16* by, long ldby, const float* bscale,
                                    const float* bshift, const float* bmean, const float* bcoef, int bact,
                                    hipStream_t stream) {
  if (!seg_dw2_ok(C, stride) || !dy || !x || !al16(dy, lddy) || !al16(x, ldx) || !al16(by, ldby) ||
      ((in_scale == nullptr) != (in_shift == nullptr)) || Ho != (H - 1) / stride + 1 || Wo != (W - 1) / stride + 1 ||
      (by && (!bscale || !bshift || !bmean || !bcoef)))
    return (int)hipErrorInvalidValue;
  Dw2Args a{};
  a.in = x; a.ldin = ldx; a.isc = in_scale; a.ish = in_shift; a.iact = in_act; a.dy = dy; a.lddy = lddy;
  a.part = part; a.N = N; a.H = H; a.W = W; a.C = C; a.Ho = Ho; a.Wo = Wo;
  a.by = by; a.ldby = ldby; a.bsc = bscale; a.bsh = bshift; a.bmu = bmean; a.bk = bcoef; a.bact = bact;
  const bool bi = by != nullptr;
  const int tho = dw2_wgrad_tho(stride, bi);
  a.tiles_w = (Wo + TWO - 1) / TWO;
  a.tiles_h = (Ho + tho - 1) / tho;
  a.ntiles = N * a.tiles_w * a.tiles_h;
  const long blocks = seg_dw2_wgrad_blocks(N, Ho, Wo, C, stride, bi);
  a.tiles_per_block = (int)((a.ntiles + blocks - 1) / blocks);
  const dim3 grid((unsigned)blocks, (C + CB - 1) / CB);
  const bool lazy = in_scale != nullptr;
#define SEG_DW2W(S, L, B) hipLaunchKernelGGL((dw2_wgrad_kernel<S, L, B>), grid, dim3(kThreads), 0, stream, a)
  if (stride == 1) {
    if (lazy) { if (bi) SEG_DW2W(1, true, true); else SEG_DW2W(1, true, false); }
    else { if (bi) SEG_DW2W(1, false, true); else SEG_DW2W(1, false, false); }
  } else {
    if (lazy) { if (bi) SEG_DW2W(2, true, true); else SEG_DW2W(2, true, false); }
    else { if (bi) SEG_DW2W(2, false, true); else SEG_DW2W(2, false, false); }
  }
#undef SEG_DW2W
  SEG_RET_LAST();
}

SEG_API int seg_dw2_wgrad_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W, int C,
                                 const float* in_scale, const float* in_shift, int in_act, int Ho, int Wo, int stride,
                                 float* part, hipStream_t stream) {
  return seg_dw2_wgrad_bn_bf16io(dy, lddy, x, ldx, N, H, W, C, in_scale, in_shift, in_act, Ho, Wo, stride, part,
                                 nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, stream);
}
