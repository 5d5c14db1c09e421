// BatchNorm2d (train + eval) with the fused activation / residual of the hot path.
//
// Reference semantics: nn.BatchNorm2d after every conv
// (src/unet.py:59,62,114 and the torchvision Conv2dNormActivation /
// InvertedResidual norms reached through src/unet.py:15-19); train mode uses the
// biased batch variance over (N,H,W), eps = 1e-5, and updates
// running_mean/var <- 0.9*old + 0.1*batch with the UNBIASED variance and
// num_batches_tracked += 1.  The activation that follows is ReLU6
// (torchvision), ReLU (src/unet.py:60,63,115) or nothing (the linear project
// conv, whose output takes the residual add of InvertedResidual).
//
// Layout: raw conv output y is NHWC [M][ldy]; channels C % 4 == 0.
// Statistics are computed in two steps: per-block shifted partial sums (fp32 over <= a
// few hundred rows, shift = first row so a large mean cannot cancel the variance away)
// and a per-channel finalize in fp64 (fixed order: deterministic).
#include "common.h"

namespace {

// Per-block partial sums over a row range, per channel.  512-thread blocks laid out as
// RG row lanes x TC channel-group lanes; a lane owns VW = 8 channels when C % 8 == 0
// (one 16-byte load per row and tensor on bf16 storage, two on fp32), else 4, and walks
// its rows four at a time, so 8-16 independent loads are in flight per lane.  The
// row / lane partition depends only on C, M and the row strides -- never on the storage
// type -- so the fp32 and bf16io twins sum in the same order (bitwise-equal on
// bf16-representable data, tests/test_gpu_bf16io.py).  Channel groups
// beyond 64 are split over blockIdx.y (the encoder's 384..1280-channel layers).  The
// row range is split into nblk = chan_blocks(M) blocks (<= 256: one or two waves of
// 512-thread blocks per CU, and few enough partial rows for the finalize kernels' one
// round trip).  Partials: part[blockIdx.x][2][C].
// kind 0: (sum(y-k), sum((y-k)^2)),  k = y[0][c]                   -> BN stats
// kind 1: (sum(dz),  sum(dz*(y-mean))), dz = dA * act'(y*scale+shift) -> BN backward
// kind 2: (sum(y), 0)                                               -> bias grad
#ifndef SEG_RED_THREADS
#define SEG_RED_THREADS 256  // measured (interleaved A/B, profiles/r05/ab_fused_bn_knobs.txt): bf16io +0.5 %, f32 flat vs 512
#endif
constexpr int kRedThreads = SEG_RED_THREADS;
#ifndef SEG_RQ
#define SEG_RQ 1  // rows per load group of the fp32 backward partials (4: the round-5 form, A/B)
#endif
constexpr int kRedSlice = 64;  // channel groups per block (blockIdx.y slices beyond)

#ifndef SEG_CHAN_MAXBLK
#define SEG_CHAN_MAXBLK 512  // row blocks of a channel reduction: 512 measured bf16io +0.8 %, f32 -0.25 % vs 256 (r05u)
#endif
#ifndef SEG_APPLY_ROWS4
#define SEG_APPLY_ROWS4 0
#endif
int chan_blocks(long M) { return (int)std::max<long>(1, std::min<long>(SEG_CHAN_MAXBLK, M / 64)); }

template <int VW, typename T>
__device__ __forceinline__ void ldw(const T* p, f32x4 (&o)[VW / 4]) {
  if constexpr (VW == 8 && sizeof(T) == 2) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
    o[0] = __builtin_convertvector(__builtin_shufflevector(v, v, 0, 1, 2, 3), f32x4);
    o[1] = __builtin_convertvector(__builtin_shufflevector(v, v, 4, 5, 6, 7), f32x4);
  } else {
#pragma unroll
    for (int j = 0; j < VW / 4; ++j) o[j] = ld4(p + 4 * j);
  }
}

template <int KIND, typename T, int VW>
__global__ __launch_bounds__(kRedThreads) void chan_partial_kernel(
    const T* __restrict__ y, long ldy, const T* __restrict__ da, long ldda, int M, int C,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ mean, int act,
    float* __restrict__ part, int rows_per_block) {
  constexpr int NV = VW / 4;
  __shared__ f32x4 red0[kRedThreads * NV], red1[kRedThreads * NV];
  const int CG = C / VW;
  const int cg0 = blockIdx.y * kRedSlice;
  const int TC = min(CG - cg0, kRedSlice);
  const int RG = kRedThreads / TC;
  const int t = threadIdx.x;
  const int rg = t / TC, tc = t - rg * TC;
  const bool active = rg < RG;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int c = (cg0 + tc) * VW;
  f32x4 s0[NV], s1[NV], k[NV], sc[NV], sh[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    s0[j] = s1[j] = k[j] = sc[j] = sh[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (active) {
    if (KIND == 0) ldw<VW>(y + c, k);
    if (KIND == 1) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        k[j] = ld4(mean + c + 4 * j);
        sc[j] = ld4(scale + c + 4 * j);
        sh[j] = ld4(shift + c + 4 * j);
      }
    }
    auto step = [&](const f32x4 (&v)[NV], const f32x4 (&g)[NV]) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        if (KIND == 0) {
          const f32x4 d = v[j] - k[j];
          s0[j] += d;
          s1[j] += d * d;
        } else if (KIND == 1) {
          f32x4 dz;
#pragma unroll
          for (int e = 0; e < 4; ++e) dz[e] = g[j][e] * seg_act_mask(v[j][e] * sc[j][e] + sh[j][e], act);
          s0[j] += dz;
          s1[j] += dz * (v[j] - k[j]);
        } else {
          s0[j] += v[j];
        }
      }
    };
    // RQ rows' loads issued together; one for the fp32 backward partials (4 x 16-byte loads per lane, 76 VGPRs):
    // that keeps the kernel within the 80 VGPRs per SIMD a side-stream weight gradient leaves
    // (wino_wgrad16_kernel: 2 waves x 216), so its waves fit beside one, where the four-row form (148 VGPRs)
    // waited for whole weight-gradient blocks to retire.  Same row order either way (the sums do not change).
    constexpr int RQ = (KIND == 1 && sizeof(T) == 4 && VW == 8) ? SEG_RQ : 4;
    int r = r0 + rg;
    for (; r + (RQ - 1) * RG < r1; r += RQ * RG) {
      f32x4 v[RQ][NV], g[RQ][NV];
#pragma unroll
      for (int q = 0; q < RQ; ++q) {
        ldw<VW>(y + (long)(r + q * RG) * ldy + c, v[q]);
        if (KIND == 1) ldw<VW>(da + (long)(r + q * RG) * ldda + c, g[q]);
      }
#pragma unroll
      for (int q = 0; q < RQ; ++q) step(v[q], g[q]);
    }
    for (; r < r1; r += RG) {
      f32x4 v[NV], g[NV];
      ldw<VW>(y + (long)r * ldy + c, v);
      if (KIND == 1) ldw<VW>(da + (long)r * ldda + c, g);
      step(v, g);
    }
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    red0[t * NV + j] = s0[j];
    red1[t * NV + j] = s1[j];
  }
  __syncthreads();
  // fixed-order tree over the RG row groups (deterministic)
  int p2 = 1;
  while (p2 < RG) p2 <<= 1;
  for (int h = p2 >> 1; h > 0; h >>= 1) {
    if (active && rg < h && rg + h < RG) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        red0[t * NV + j] += red0[(t + h * TC) * NV + j];
        red1[t * NV + j] += red1[(t + h * TC) * NV + j];
      }
    }
    __syncthreads();
  }
  if (rg == 0) {
    float* p0 = part + (long)blockIdx.x * 2 * C;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      st4(p0 + c + 4 * j, red0[tc * NV + j]);
      st4(p0 + C + c + 4 * j, red1[tc * NV + j]);
    }
  }
}

// Launch chan_partial_kernel<KIND> over [M][C] (C % 4 == 0): 8-channel lanes when C, the
// row strides and the tensors' element offsets are multiples of 8 (16-byte bf16 loads),
// else 4 -- a decision in elements, identical for fp32 and bf16 storage.
template <int KIND, typename T>
void launch_chan_partial(const T* y, long ldy, const T* da, long ldda, long M, int C, const float* scale,
                         const float* shift, const float* mean, int act, float* part, hipStream_t stream) {
  const int nblk = chan_blocks(M);
  const int rpb = seg_cdiv(M, nblk);
  auto eoff8 = [](const T* p) { return ((uintptr_t)p / sizeof(T)) % 8 == 0; };
  const bool v8 = C % 8 == 0 && ldy % 8 == 0 && (!da || ldda % 8 == 0) && eoff8(y) && (!da || eoff8(da));
  if (v8)
    hipLaunchKernelGGL((chan_partial_kernel<KIND, T, 8>), dim3(nblk, seg_cdiv(C / 8, kRedSlice)), dim3(kRedThreads),
                       0, stream, y, ldy, da, ldda, (int)M, C, scale, shift, mean, act, part, rpb);
  else
    hipLaunchKernelGGL((chan_partial_kernel<KIND, T, 4>), dim3(nblk, seg_cdiv(C / 4, kRedSlice)), dim3(kRedThreads),
                       0, stream, y, ldy, da, ldda, (int)M, C, scale, shift, mean, act, part, rpb);
}

// Finalize kernels.  Sum the per-block partials (<= SEG_CHAN_MAXBLK rows:
// chan_blocks) of one channel with one wave: lane l loads rows l, l+64, l+128, ... all at
// once (one memory round trip; clamped index, masked add), sums them in that order in
// fp64, then a fixed xor butterfly (fp64 adds are commutative, so every lane ends with the
// same bits; deterministic).  Four channels per 256-thread block: c = blockIdx.x * 4 + wave.
__device__ __forceinline__ bool sum_partials(const float* __restrict__ part, int nblk, int C, int ldp, int* cout,
                                             double* s0, double* s1) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  *cout = c;
  if (c >= C) return false;
  constexpr int Q = (SEG_CHAN_MAXBLK + 63) / 64;  // partial rows per lane (chan_blocks <= SEG_CHAN_MAXBLK)
  float va[Q], vb[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const long k = min(lane + 64 * q, nblk - 1);
    va[q] = part[k * 2 * ldp + c];
    vb[q] = part[k * 2 * ldp + ldp + c];
  }
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const bool ok = lane + 64 * q < nblk;
    a += ok ? (double)va[q] : 0.0;
    b += ok ? (double)vb[q] : 0.0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  *s0 = a;
  *s1 = b;
  return lane == 0;
}

template <typename T>
__global__ __launch_bounds__(256) void bn_finalize_kernel(
    const float* __restrict__ part, int nblk, const T* __restrict__ y, long M, int C,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
    float* running_mean, float* running_var, long long* nbt, float* mean_out, float* invstd_out, float* scale_out,
    float* shift_out) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  int c;
  double s, s2;
  if (!sum_partials(part, nblk, C, C, &c, &s, &s2)) return;
  const double k = (float)y[c];
  const double dm = s / (double)M;
  const double mean = k + dm;
  double var = s2 / (double)M - dm * dm;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale_out[c] = g * invstd;
  shift_out[c] = bt - (float)mean * g * invstd;
  if (running_mean) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, long M, int C,
                                       const float* __restrict__ gamma, const float* __restrict__ invstd,
                                       float* dgamma, float* dbeta, float* coef) {
  int c;
  double sdz, sdzx;
  if (!sum_partials(part, nblk, C, C, &c, &sdz, &sdzx)) return;
  const double inv = invstd[c];
  const double g = gamma ? gamma[c] : 1.0;
  if (dbeta) dbeta[c] = (float)sdz;
  if (dgamma) dgamma[c] = (float)(sdzx * inv);
  // dY = g*inv * (dz - mean(dz) - xhat*mean(dz*xhat)),  xhat = (y-mean)*inv
  coef[c] = (float)(g * inv);
  coef[C + c] = (float)(sdz / (double)M);
  coef[2 * C + c] = (float)(sdzx * inv * inv / (double)M);
}

__global__ void colsum_finalize_kernel(const float* __restrict__ part, int nblk, int C, int ldp, float* out,
                                       int accumulate) {
  int c;
  double s, unused;
  if (sum_partials(part, nblk, C, ldp, &c, &s, &unused)) out[c] = accumulate ? out[c] + (float)s : (float)s;
}

// BN statistics from the conv epilogue's per-row-tile partials part[t][2][C]
// (tile sum S_t and tile M2_t about the tile mean, tile t holding
// min(tile_rows, M - t*tile_rows) rows), merged in fp64 (deterministic).
// The merge in two passes against the global mean (the parallel-variance identity
// M2 = sum_t [M2_t + n_t (mean_t - mean)^2], as stable as pairwise Chan merges, with adds
// instead of a division per merge): pass 1 sums the tile sums -> mean, pass 2 sums the
// tile M2s and the between-tile terms.  fp64, fixed orders (deterministic).
__device__ __forceinline__ double tile_rows_of(int i, int tile_rows, long M) {
  return (double)std::min<long>(tile_rows, M - (long)i * tile_rows);
}

__device__ __forceinline__ void bn_stats_out(double mean, double m2, long M, int c, const float* gamma,
                                             const float* beta, float eps, float momentum, float* running_mean,
                                             float* running_var, float* mean_out, float* invstd_out,
                                             float* scale_out, float* shift_out) {
  double var = m2 / (double)M;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale_out[c] = g * invstd;
  shift_out[c] = bt - (float)mean * g * invstd;
  if (running_mean) {
    const double unbiased = M > 1 ? m2 / (double)(M - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unbiased);
  }
}

// Many tiles (the high-resolution layers: up to M / 128): one 256-thread block per
// channel, each lane summing every 256th tile, fixed-order LDS trees.
__global__ __launch_bounds__(256) void bn_finalize_tiles_kernel(
    const float* __restrict__ part, int ntiles, int tile_rows, long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* running_mean, float* running_var,
    long long* nbt, float* mean_out, float* invstd_out, float* scale_out, float* shift_out) {
  __shared__ double red[256];
  const int t = threadIdx.x;
  const int c = blockIdx.x;
  if (blockIdx.x == 0 && t == 0 && nbt) *nbt += 1;
  auto tree = [&](double v) -> double {  // every thread gets the fixed-order block sum
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
  };
  // 16 tiles' loads in flight per thread (clamped index, masked add), summed in tile order
  double s = 0.0;
  for (int i0 = t; i0 < ntiles; i0 += 16 * 256) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = part[(long)min(i0 + j * 256, ntiles - 1) * 2 * C + c];
#pragma unroll
    for (int j = 0; j < 16; ++j) s += i0 + j * 256 < ntiles ? (double)v[j] : 0.0;
  }
  const double mean = tree(s) / (double)M;
  double q = 0.0;
  for (int i0 = t; i0 < ntiles; i0 += 16 * 256) {
    float v[16], w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const long i = min(i0 + j * 256, ntiles - 1);
      v[j] = part[i * 2 * C + c];
      w[j] = part[i * 2 * C + C + c];
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int i = i0 + j * 256;
      const double nt = tile_rows_of(i, tile_rows, M);
      const double d = v[j] / nt - mean;
      q += i < ntiles ? w[j] + nt * d * d : 0.0;
    }
  }
  const double m2 = tree(q);
  if (t == 0)
    bn_stats_out(mean, m2, M, c, gamma, beta, eps, momentum, running_mean, running_var, mean_out, invstd_out,
                 scale_out, shift_out);
}

// Few tiles (<= 256: the small layers): one wave per channel, 4 channels per block, lanes
// over tiles, fixed xor butterflies (no LDS, no barriers).
__global__ __launch_bounds__(256) void bn_finalize_tiles_wave_kernel(
    const float* __restrict__ part, int ntiles, int tile_rows, long M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* running_mean, float* running_var,
    long long* nbt, float* mean_out, float* invstd_out, float* scale_out, float* shift_out) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  double sv[4], qv[4];
  float fs[4], fq[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // ntiles <= 256: at most 4 tiles per lane, loaded together
    const long i = min(lane + 64 * k, ntiles - 1);
    fs[k] = part[i * 2 * C + c];
    fq[k] = part[i * 2 * C + C + c];
  }
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool ok = lane + 64 * k < ntiles;
    sv[k] = fs[k];
    qv[k] = fq[k];
    s += ok ? sv[k] : 0.0;
  }
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o, 64);
  const double mean = s / (double)M;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double nt = tile_rows_of(lane + 64 * k, tile_rows, M);
    const double d = sv[k] / nt - mean;
    q += lane + 64 * k < ntiles ? qv[k] + nt * d * d : 0.0;
  }
  for (int o = 1; o < 64; o <<= 1) q += __shfl_xor(q, o, 64);
  if (lane == 0)
    bn_stats_out(mean, q, M, c, gamma, beta, eps, momentum, running_mean, running_var, mean_out, invstd_out,
                 scale_out, shift_out);
}

// Many tiles: R consecutive row tiles merged into one super-tile first (same format: sum and M2 about the
// super-tile's own mean, R * tile_rows rows, the last one short), so the per-channel finalize above reads
// ntiles / R rows instead of ntiles.  One thread per (super-tile, channel), consecutive threads on consecutive
// channels: a wave reads whole partial rows (coalesced), where the per-channel finalize's lanes each touch a
// different cache line.  fp64 inside, fixed order (deterministic).
constexpr int kTileMerge = 16;
#ifndef SEG_TILE_MERGE_MIN
#define SEG_TILE_MERGE_MIN 1024
#endif
constexpr int kTileMergeMin = SEG_TILE_MERGE_MIN;  // ntiles above which the merge stage runs

__global__ __launch_bounds__(256) void bn_tiles_merge_kernel(const float* __restrict__ part, int ntiles, int tile_rows,
                                                             long M, int C, float* __restrict__ out) {
  const long gid = blockIdx.x * 256L + threadIdx.x;
  const int ns = (ntiles + kTileMerge - 1) / kTileMerge;
  if (gid >= (long)ns * C) return;
  const int j = (int)(gid / C), c = (int)(gid - (long)j * C);
  const int t0 = j * kTileMerge;
  float fs[kTileMerge], fq[kTileMerge];
#pragma unroll
  for (int k = 0; k < kTileMerge; ++k) {
    const long i = min(t0 + k, ntiles - 1);
    fs[k] = part[i * 2 * C + c];
    fq[k] = part[i * 2 * C + C + c];
  }
  double S = 0.0;
#pragma unroll
  for (int k = 0; k < kTileMerge; ++k) S += t0 + k < ntiles ? (double)fs[k] : 0.0;
  const double n = (double)std::min<long>((long)kTileMerge * tile_rows, M - (long)t0 * tile_rows);
  const double mu = S / n;
  double Q = 0.0;
#pragma unroll
  for (int k = 0; k < kTileMerge; ++k) {
    const double nt = tile_rows_of(t0 + k, tile_rows, M);
    const double d = fs[k] / nt - mu;
    Q += t0 + k < ntiles ? (double)fq[k] + nt * d * d : 0.0;
  }
  out[(long)j * 2 * C + c] = (float)S;
  out[(long)j * 2 * C + C + c] = (float)Q;
}

__global__ void bn_eval_coef_kernel(const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                                    int C, float* scale_out, float* shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.f / sqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale_out[c] = g * inv;
  shift_out[c] = b - rm[c] * g * inv;
}

// out = act(y*scale + shift) (+ res)
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ y, long ldy, long M, int C, const float* __restrict__ scale,
                                const float* __restrict__ shift, int act, const T* __restrict__ res, long ldres,
                                T* __restrict__ out, long ldout) {
  const int CG = C >> 2;
  const long total = M * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / CG;
    const int c = (int)(i - r * CG) * 4;
    f32x4 o = seg_bn_act4(ld4(y + r * ldy + c), ld4(scale + c), ld4(shift + c), act);
    if (res) o += ld4(res + r * ldres + c);
    st4(out + r * ldout + c, o);
  }
}

template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ da, long ldda, const T* __restrict__ y, long ldy,
                                    long M, int C, const float* __restrict__ scale, const float* __restrict__ shift,
                                    const float* __restrict__ mean, int act, const float* __restrict__ coef,
                                    T* __restrict__ dy, long lddy) {
  const int CG = C >> 2;
  const long total = M * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / CG;
    const int c = (int)(i - r * CG) * 4;
    const f32x4 v = ld4(y + r * ldy + c), g = ld4(da + r * ldda + c);
    const f32x4 sc = ld4(scale + c), sh = ld4(shift + c), mu = ld4(mean + c);
    const f32x4 k1 = ld4(coef + c), k2 = ld4(coef + C + c), k3 = ld4(coef + 2 * C + c);
    st4(dy + r * lddy + c, seg_bnbwd4(g, v, sc, sh, mu, k1, k2, k3, act));
  }
}

// Eval-mode backward (BN uses running statistics, a pure affine map):
// dY = dA * act'(y*scale+shift) * scale.
__global__ void bn_eval_bwd_kernel(const float* __restrict__ da, long ldda, const float* __restrict__ y, long ldy,
                                   long M, int C, const float* __restrict__ scale, const float* __restrict__ shift,
                                   int act, float* __restrict__ dy, long lddy) {
  const int CG = C >> 2;
  const long total = M * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / CG;
    const int c = (int)(i - r * CG) * 4;
    const f32x4 v = ld4(y + r * ldy + c), g = ld4(da + r * ldda + c);
    const f32x4 sc = ld4(scale + c), sh = ld4(shift + c);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = g[j] * seg_act_mask(v[j] * sc[j] + sh[j], act) * sc[j];
    st4(dy + r * lddy + c, o);
  }
}

int ew_grid(long total) { return (int)std::min<long>(seg_cdiv(total, 256), 8192); }

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, long lda, const T* __restrict__ b, long ldb, long M, int C,
                           T* __restrict__ out, long ldout) {
  const int CG = C >> 2;
  const long total = M * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / CG;
    const int c = (int)(i - r * CG) * 4;
    f32x4 v = ld4(a + r * lda + c);
    if (b) v += ld4(b + r * ldb + c);
    st4(out + r * ldout + c, v);
  }
}

// Row-tiled elementwise passes (BN apply, BN backward apply, gradient add).  A
// 256-thread block is RG row lanes x TC channel-group lanes; each lane keeps its
// VW-channel group (one 16-byte access: 4 fp32 or 8 bf16 channels) and its
// per-channel coefficients in registers and strides over rows, two rows per trip so
// both rows' loads are in flight together.  No per-element index division and no
// per-element coefficient loads; the arithmetic per element is the flat kernels'
// (seg_bn_act4 / seg_bnbwd4), so results are bitwise those of the flat kernels.
// Launched for the 16-byte bf16 layout (8 channels per lane); the 4-channel layouts
// keep the flat kernels, which measured 2-7 % faster than these on fp32 (MI355X).
template <int VW, typename T>
__device__ __forceinline__ void ldv(const T* p, f32x4* o) {
  if constexpr (VW == 8) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
    o[0] = __builtin_convertvector(__builtin_shufflevector(v, v, 0, 1, 2, 3), f32x4);
    o[1] = __builtin_convertvector(__builtin_shufflevector(v, v, 4, 5, 6, 7), f32x4);
  } else {
    o[0] = ld4(p);
  }
}
template <int VW, typename T>
__device__ __forceinline__ void stv(T* p, const f32x4* o) {
  if constexpr (VW == 8) {
    const bf16x4 lo = __builtin_convertvector(o[0], bf16x4), hi = __builtin_convertvector(o[1], bf16x4);
    *reinterpret_cast<bf16x8*>(p) = seg_cat8(lo, hi);
  } else {
    st4(p, o[0]);
  }
}
template <int NV>
__device__ __forceinline__ void ldc(const float* p, f32x4* o) {
#pragma unroll
  for (int j = 0; j < NV; ++j) o[j] = ld4(p + 4 * j);
}

struct RowTile {
  int CG, TC, RG, rg, tc;
  __device__ RowTile(int C, int VW) {
    CG = C / VW;
    TC = CG < 256 ? CG : 256;
    RG = 256 / TC;
    rg = threadIdx.x / TC;
    tc = threadIdx.x - rg * TC;
  }
};

template <typename T, int VW>
__global__ __launch_bounds__(256) void bn_apply_rt_kernel(const T* __restrict__ y, long ldy, long M, int C,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int act,
                                                          const T* __restrict__ res, long ldres, T* out, long ldout) {
  constexpr int NV = VW / 4;
  const RowTile rt(C, VW);
  if (rt.rg >= rt.RG) return;
  const long step = (long)gridDim.x * rt.RG;
  for (int cg = rt.tc; cg < rt.CG; cg += rt.TC) {
    const int c = cg * VW;
    f32x4 sc[NV], sh[NV];
    ldc<NV>(scale + c, sc);
    ldc<NV>(shift + c, sh);
    long r = (long)blockIdx.x * rt.RG + rt.rg;
    for (; r + step < M; r += 2 * step) {
      f32x4 v0[NV], v1[NV], q0[NV], q1[NV];
      ldv<VW>(y + r * ldy + c, v0);
      ldv<VW>(y + (r + step) * ldy + c, v1);
      if (res) {
        ldv<VW>(res + r * ldres + c, q0);
        ldv<VW>(res + (r + step) * ldres + c, q1);
      }
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        v0[j] = seg_bn_act4(v0[j], sc[j], sh[j], act);
        v1[j] = seg_bn_act4(v1[j], sc[j], sh[j], act);
        if (res) {
          v0[j] += q0[j];
          v1[j] += q1[j];
        }
      }
      stv<VW>(out + r * ldout + c, v0);
      stv<VW>(out + (r + step) * ldout + c, v1);
    }
    if (r < M) {
      f32x4 v0[NV], q0[NV];
      ldv<VW>(y + r * ldy + c, v0);
      if (res) ldv<VW>(res + r * ldres + c, q0);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        v0[j] = seg_bn_act4(v0[j], sc[j], sh[j], act);
        if (res) v0[j] += q0[j];
      }
      stv<VW>(out + r * ldout + c, v0);
    }
  }
}

template <typename T, int VW>
__global__ __launch_bounds__(256) void bn_bwd_apply_rt_kernel(const T* __restrict__ da, long ldda,
                                                              const T* __restrict__ y, long ldy, long M, int C,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              const float* __restrict__ mean, int act,
                                                              const float* __restrict__ coef, T* dy, long lddy) {
  constexpr int NV = VW / 4;
  const RowTile rt(C, VW);
  if (rt.rg >= rt.RG) return;
  const long step = (long)gridDim.x * rt.RG;
  for (int cg = rt.tc; cg < rt.CG; cg += rt.TC) {
    const int c = cg * VW;
    f32x4 sc[NV], sh[NV], mu[NV], k1[NV], k2[NV], k3[NV];
    ldc<NV>(scale + c, sc);
    ldc<NV>(shift + c, sh);
    ldc<NV>(mean + c, mu);
    ldc<NV>(coef + c, k1);
    ldc<NV>(coef + C + c, k2);
    ldc<NV>(coef + 2 * C + c, k3);
    long r = (long)blockIdx.x * rt.RG + rt.rg;
    for (; SEG_APPLY_ROWS4 && r + 3 * step < M; r += 4 * step) {  // four rows' loads in flight together
      f32x4 v[4][NV], g[4][NV];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ldv<VW>(y + (r + q * step) * ldy + c, v[q]);
        ldv<VW>(da + (r + q * step) * ldda + c, g[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int j = 0; j < NV; ++j) v[q][j] = seg_bnbwd4(g[q][j], v[q][j], sc[j], sh[j], mu[j], k1[j], k2[j], k3[j], act);
        stv<VW>(dy + (r + q * step) * lddy + c, v[q]);
      }
    }
    for (; r + step < M; r += 2 * step) {
      f32x4 v0[NV], v1[NV], g0[NV], g1[NV];
      ldv<VW>(y + r * ldy + c, v0);
      ldv<VW>(da + r * ldda + c, g0);
      ldv<VW>(y + (r + step) * ldy + c, v1);
      ldv<VW>(da + (r + step) * ldda + c, g1);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        v0[j] = seg_bnbwd4(g0[j], v0[j], sc[j], sh[j], mu[j], k1[j], k2[j], k3[j], act);
        v1[j] = seg_bnbwd4(g1[j], v1[j], sc[j], sh[j], mu[j], k1[j], k2[j], k3[j], act);
      }
      stv<VW>(dy + r * lddy + c, v0);
      stv<VW>(dy + (r + step) * lddy + c, v1);
    }
    if (r < M) {
      f32x4 v0[NV], g0[NV];
      ldv<VW>(y + r * ldy + c, v0);
      ldv<VW>(da + r * ldda + c, g0);
#pragma unroll
      for (int j = 0; j < NV; ++j) v0[j] = seg_bnbwd4(g0[j], v0[j], sc[j], sh[j], mu[j], k1[j], k2[j], k3[j], act);
      stv<VW>(dy + r * lddy + c, v0);
    }
  }
}

template <typename T, int VW>
__global__ __launch_bounds__(256) void add_rt_kernel(const T* a, long lda, const T* b, long ldb, long M, int C,
                                                     T* out, long ldout) {
  constexpr int NV = VW / 4;
  const RowTile rt(C, VW);
  if (rt.rg >= rt.RG) return;
  const long step = (long)gridDim.x * rt.RG;
  for (int cg = rt.tc; cg < rt.CG; cg += rt.TC) {
    const int c = cg * VW;
    for (long r = (long)blockIdx.x * rt.RG + rt.rg; r < M; r += step) {
      f32x4 v[NV], q[NV];
      ldv<VW>(a + r * lda + c, v);
      if (b) {
        ldv<VW>(b + r * ldb + c, q);
#pragma unroll
        for (int j = 0; j < NV; ++j) v[j] += q[j];
      }
      stv<VW>(out + r * ldout + c, v);
    }
  }
}

// Channels per lane for the row-tiled passes: 8 for bf16 storage when every channel
// offset, row stride and pointer allows 16-byte accesses, else 4.
template <typename T>
int rt_vw(int C, std::initializer_list<long> lds, std::initializer_list<const void*> ptrs) {
  if (sizeof(T) != 2 || C % 8) return 4;
  for (long ld : lds) if (ld % 8) return 4;
  for (const void* p : ptrs) if (p && ((uintptr_t)p & 15)) return 4;
  return 8;
}
int rt_grid(long M, int C, int VW) {
  const int CG = C / VW, TC = CG < 256 ? CG : 256, RG = 256 / TC;
  return (int)std::max<long>(1, std::min<long>(seg_cdiv(M, RG), 4096));
}

template <typename T>
void launch_bn_bwd_apply(const T* da, long ldda, const T* y, long ldy, long M, int C, const float* scale,
                         const float* shift, const float* mean, int act, const float* coef, T* dy, long lddy,
                         hipStream_t stream) {
  if (M < 1) return;
  if (rt_vw<T>(C, {ldda, ldy, lddy}, {da, y, dy}) == 8)
    hipLaunchKernelGGL((bn_bwd_apply_rt_kernel<T, 8>), dim3(rt_grid(M, C, 8)), dim3(256), 0, stream, da, ldda, y, ldy,
                       M, C, scale, shift, mean, act, coef, dy, lddy);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(ew_grid(M * (C / 4))), dim3(256), 0, stream, da, ldda, y, ldy, M,
                       C, scale, shift, mean, act, coef, dy, lddy);
}

}  // namespace

// out = a (+ b), all [M][C] NHWC strided (out may alias a or b).  Gradient fan-in.
template <typename T>
static int add_impl(const T* a, long lda, const T* b, long ldb, long M, int C, T* out, long ldout, hipStream_t stream) {
  if ((C & 3) || (lda & 3) || (ldout & 3) || (b && (ldb & 3))) return (int)hipErrorInvalidValue;
  if (M < 1) return (int)hipSuccess;
  if (rt_vw<T>(C, {lda, b ? ldb : 0, ldout}, {a, b, out}) == 8)
    hipLaunchKernelGGL((add_rt_kernel<T, 8>), dim3(rt_grid(M, C, 8)), dim3(256), 0, stream, a, lda, b, ldb, M, C,
                       out, ldout);
  else
    hipLaunchKernelGGL(add_kernel<T>, dim3(ew_grid(M * (C / 4))), dim3(256), 0, stream, a, lda, b, ldb, M, C, out,
                       ldout);
  SEG_RET_LAST();
}
SEG_API int seg_add(const float* a, long lda, const float* b, long ldb, long M, int C, float* out, long ldout,
                    hipStream_t stream) {
  return add_impl(a, lda, b, ldb, M, C, out, ldout, stream);
}
// `_bf16io` entry points (this file and the others): the same operation on bf16
// activation / gradient tensors (arguments as the fp32 version, element strides);
// statistics, partial sums and coefficients stay fp32.
SEG_API int seg_add_bf16io(const __bf16* a, long lda, const __bf16* b, long ldb, long M, int C, __bf16* out,
                           long ldout, hipStream_t stream) {
  return add_impl(a, lda, b, ldb, M, C, out, ldout, stream);
}

// Size (floats) of the partial-sum workspace the channel reductions below need.
SEG_API long seg_chan_workspace_floats(long M, int C) { return (long)chan_blocks(M) * 2 * C; }

// Train-mode BN statistics: fills mean/invstd/scale/shift ([C] each) and updates
// the running buffers (skipped when running_mean is null) and num_batches_tracked.
template <typename T>
static int bn_stats_impl(const T* y, long ldy, long M, int C, const float* gamma, const float* beta, float eps,
                         float momentum, float* running_mean, float* running_var, long long* num_batches_tracked,
                         float* work, float* mean, float* invstd, float* scale, float* shift, hipStream_t stream) {
  if ((C & 3) || (ldy & 3) || M < 1) return (int)hipErrorInvalidValue;
  launch_chan_partial<0, T>(y, ldy, nullptr, 0L, M, C, nullptr, nullptr, nullptr, 0, work, stream);
  hipLaunchKernelGGL(bn_finalize_kernel<T>, dim3(seg_cdiv(C, 4)), dim3(256), 0, stream, work, chan_blocks(M), y, M, C,
                     gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, mean, invstd, scale,
                     shift);
  SEG_RET_LAST();
}
SEG_API int seg_bn_stats(const float* y, long ldy, long M, int C, const float* gamma, const float* beta, float eps,
                         float momentum, float* running_mean, float* running_var, long long* num_batches_tracked,
                         float* work, float* mean, float* invstd, float* scale, float* shift, hipStream_t stream) {
  return bn_stats_impl(y, ldy, M, C, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, work,
                       mean, invstd, scale, shift, stream);
}
SEG_API int seg_bn_stats_bf16io(const __bf16* y, long ldy, long M, int C, const float* gamma, const float* beta,
                                float eps, float momentum, float* running_mean, float* running_var,
                                long long* num_batches_tracked, float* work, float* mean, float* invstd, float* scale,
                                float* shift, hipStream_t stream) {
  return bn_stats_impl(y, ldy, M, C, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, work,
                       mean, invstd, scale, shift, stream);
}

// Train-mode BN statistics from seg_conv_igemm's epilogue partials (`stat`
// workspace of seg_conv_igemm_row_tiles(M, C) x 2 x C floats); same outputs and
// running-buffer update as seg_bn_stats, without re-reading the conv output.
SEG_API int seg_bn_stats_tiles(const float* part, int ntiles, int tile_rows, long M, int C, const float* gamma,
                               const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                               long long* num_batches_tracked, float* mean, float* invstd, float* scale, float* shift,
                               hipStream_t stream);

// Workspace floats of seg_bn_stats_tiles_ws (0: no merge stage at this tile count).
SEG_API long seg_bn_stats_tiles_work_floats(int ntiles, int C) {
  return ntiles > kTileMergeMin ? (long)seg_cdiv(ntiles, kTileMerge) * 2 * C : 0;
}

// seg_bn_stats_tiles with a workspace of seg_bn_stats_tiles_work_floats(ntiles, C) floats: many-tile
// layers merge kTileMerge tiles per row first (one more launch, coalesced) and finalize the merged rows.
SEG_API int seg_bn_stats_tiles_ws(const float* part, int ntiles, int tile_rows, long M, int C, const float* gamma,
                                  const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                                  long long* num_batches_tracked, float* mean, float* invstd, float* scale,
                                  float* shift, float* work, hipStream_t stream) {
  if (ntiles < 1 || tile_rows < 1 || M < 1) return (int)hipErrorInvalidValue;
  if (ntiles > kTileMergeMin) {
    if (!work) return (int)hipErrorInvalidValue;
    const long n = (long)seg_cdiv(ntiles, kTileMerge) * C;
    hipLaunchKernelGGL(bn_tiles_merge_kernel, dim3(seg_cdiv(n, 256)), dim3(256), 0, stream, part, ntiles, tile_rows, M,
                       C, work);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
    part = work;
    tile_rows *= kTileMerge;
    ntiles = seg_cdiv(ntiles, kTileMerge);
  }
  return seg_bn_stats_tiles(part, ntiles, tile_rows, M, C, gamma, beta, eps, momentum, running_mean, running_var,
                            num_batches_tracked, mean, invstd, scale, shift, stream);
}

SEG_API int seg_bn_stats_tiles(const float* part, int ntiles, int tile_rows, long M, int C, const float* gamma,
                               const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                               long long* num_batches_tracked, float* mean, float* invstd, float* scale, float* shift,
                               hipStream_t stream) {
  if (ntiles < 1 || tile_rows < 1 || M < 1) return (int)hipErrorInvalidValue;
  if (ntiles <= 256) {
    hipLaunchKernelGGL(bn_finalize_tiles_wave_kernel, dim3(seg_cdiv(C, 4)), dim3(256), 0, stream, part, ntiles,
                       tile_rows, M, C, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked,
                       mean, invstd, scale, shift);
    SEG_RET_LAST();
  }
  hipLaunchKernelGGL(bn_finalize_tiles_kernel, dim3(C), dim3(256), 0, stream, part, ntiles,
                     tile_rows, M, C, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked, mean,
                     invstd, scale, shift);
  SEG_RET_LAST();
}

SEG_API int seg_bn_eval_coef(const float* gamma, const float* beta, const float* running_mean,
                             const float* running_var, float eps, int C, float* scale, float* shift,
                             hipStream_t stream) {
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(seg_cdiv(C, 256)), dim3(256), 0, stream, gamma, beta, running_mean,
                     running_var, eps, C, scale, shift);
  SEG_RET_LAST();
}

template <typename T>
static int bn_apply_impl(const T* y, long ldy, long M, int C, const float* scale, const float* shift, int act,
                         const T* res, long ldres, T* out, long ldout, hipStream_t stream) {
  if ((C & 3) || (ldy & 3) || (ldout & 3) || (res && (ldres & 3))) return (int)hipErrorInvalidValue;
  if (M < 1) return (int)hipSuccess;
  if (rt_vw<T>(C, {ldy, res ? ldres : 0, ldout}, {y, res, out}) == 8)
    hipLaunchKernelGGL((bn_apply_rt_kernel<T, 8>), dim3(rt_grid(M, C, 8)), dim3(256), 0, stream, y, ldy, M, C, scale,
                       shift, act, res, ldres, out, ldout);
  else
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(ew_grid(M * (C / 4))), dim3(256), 0, stream, y, ldy, M, C, scale,
                       shift, act, res, ldres, out, ldout);
  SEG_RET_LAST();
}
SEG_API int seg_bn_apply(const float* y, long ldy, long M, int C, const float* scale, const float* shift, int act,
                         const float* res, long ldres, float* out, long ldout, hipStream_t stream) {
  return bn_apply_impl(y, ldy, M, C, scale, shift, act, res, ldres, out, ldout, stream);
}
SEG_API int seg_bn_apply_bf16io(const __bf16* y, long ldy, long M, int C, const float* scale, const float* shift,
                                int act, const __bf16* res, long ldres, __bf16* out, long ldout, hipStream_t stream) {
  return bn_apply_impl(y, ldy, M, C, scale, shift, act, res, ldres, out, ldout, stream);
}

// Train-mode BN backward through the activation: writes dgamma/dbeta ([C]) and
// dy = d(conv output).  `work` >= seg_chan_workspace_floats(M,C) + 3*C floats.
template <typename T>
static int bn_backward_impl(const T* da, long ldda, const T* y, long ldy, long M, int C, const float* gamma,
                            const float* mean, const float* invstd, const float* scale, const float* shift, int act,
                            float* dgamma, float* dbeta, float* work, T* dy, long lddy, hipStream_t stream) {
  if ((C & 3) || (ldy & 3) || (ldda & 3) || (lddy & 3)) return (int)hipErrorInvalidValue;
  if (M < 1) return (int)hipSuccess;
  float* coef = work + seg_chan_workspace_floats(M, C);
  launch_chan_partial<1, T>(y, ldy, da, ldda, M, C, scale, shift, mean, act, work, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(seg_cdiv(C, 4)), dim3(256), 0, stream, work, chan_blocks(M), M, C,
                     gamma, invstd, dgamma, dbeta, coef);
  launch_bn_bwd_apply<T>(da, ldda, y, ldy, M, C, scale, shift, mean, act, coef, dy, lddy, stream);
  SEG_RET_LAST();
}
SEG_API int seg_bn_backward(const float* da, long ldda, const float* y, long ldy, long M, int C, const float* gamma,
                            const float* mean, const float* invstd, const float* scale, const float* shift, int act,
                            float* dgamma, float* dbeta, float* work, float* dy, long lddy, hipStream_t stream) {
  return bn_backward_impl(da, ldda, y, ldy, M, C, gamma, mean, invstd, scale, shift, act, dgamma, dbeta, work, dy,
                          lddy, stream);
}
SEG_API int seg_bn_backward_bf16io(const __bf16* da, long ldda, const __bf16* y, long ldy, long M, int C,
                                   const float* gamma, const float* mean, const float* invstd, const float* scale,
                                   const float* shift, int act, float* dgamma, float* dbeta, float* work, __bf16* dy,
                                   long lddy, hipStream_t stream) {
  return bn_backward_impl(da, ldda, y, ldy, M, C, gamma, mean, invstd, scale, shift, act, dgamma, dbeta, work, dy,
                          lddy, stream);
}

// BN-backward finalize from per-row-tile partials part[t][2][C] = (sum dz, sum dz (y - mean)) of
// a producer's epilogue (seg_conv_igemm_bnout*): the outputs of bn_bwd_finalize_kernel.  A block
// owns 16 channels: 16 tile groups x 16 channels, each thread summing tiles g, g+16, ... in fp64,
// then the groups in order (fixed order: deterministic).
namespace {
__global__ __launch_bounds__(256) void bn_bwd_finalize_tiles_kernel(const float* __restrict__ part, int ntiles, long M,
                                                                    int C, const float* __restrict__ gamma,
                                                                    const float* __restrict__ invstd, float* dgamma,
                                                                    float* dbeta, float* coef) {
  __shared__ double red[2][16][16];
  const int g = threadIdx.x >> 4, cl = threadIdx.x & 15, c = blockIdx.x * 16 + cl;
  double u = 0.0, v = 0.0;
  if (c < C) {
    int t = g;
    for (; t + 48 < ntiles; t += 64) {
      float x0[4], x1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x0[i] = part[((long)(t + 16 * i) * 2) * C + c];
        x1[i] = part[((long)(t + 16 * i) * 2 + 1) * C + c];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u += (double)x0[i];
        v += (double)x1[i];
      }
    }
    for (; t < ntiles; t += 16) {
      u += (double)part[((long)t * 2) * C + c];
      v += (double)part[((long)t * 2 + 1) * C + c];
    }
  }
  red[0][g][cl] = u;
  red[1][g][cl] = v;
  __syncthreads();
  if (g == 0 && c < C) {
    double sdz = 0.0, sdzx = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      sdz += red[0][k][cl];
      sdzx += red[1][k][cl];
    }
    const double inv = invstd[c];
    const double gm = gamma ? gamma[c] : 1.0;
    if (dbeta) dbeta[c] = (float)sdz;
    if (dgamma) dgamma[c] = (float)(sdzx * inv);
    coef[c] = (float)(gm * inv);
    coef[C + c] = (float)(sdz / (double)M);
    coef[2 * C + c] = (float)(sdzx * inv * inv / (double)M);
  }
}
}  // namespace

// The two halves of seg_bn_backward, for a caller that fuses one of them into a neighbouring
// kernel:
//  * seg_bn_bwd_coef_*: the reduction -- dgamma, dbeta and coef[3][C] = (g*invstd, mean(dz),
//    mean(dz*xhat)*invstd) (`work` >= seg_chan_workspace_floats(M, C) floats);
//  * seg_bn_bwd_apply_*: dy = seg_bnbwd4(da, y; coef) -- what seg_bn_backward writes, bit for bit.
template <typename T>
static int bn_bwd_coef_impl(const T* da, long ldda, const T* y, long ldy, long M, int C, const float* gamma,
                            const float* mean, const float* invstd, const float* scale, const float* shift, int act,
                            float* dgamma, float* dbeta, float* work, float* coef, hipStream_t stream) {
  if ((C & 3) || (ldy & 3) || (ldda & 3) || M < 1 || !coef) return (int)hipErrorInvalidValue;
  launch_chan_partial<1, T>(y, ldy, da, ldda, M, C, scale, shift, mean, act, work, stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(seg_cdiv(C, 4)), dim3(256), 0, stream, work, chan_blocks(M), M, C,
                     gamma, invstd, dgamma, dbeta, coef);
  SEG_RET_LAST();
}
SEG_API int seg_bn_bwd_coef(const float* da, long ldda, const float* y, long ldy, long M, int C, const float* gamma,
                            const float* mean, const float* invstd, const float* scale, const float* shift, int act,
                            float* dgamma, float* dbeta, float* work, float* coef, hipStream_t stream) {
  return bn_bwd_coef_impl(da, ldda, y, ldy, M, C, gamma, mean, invstd, scale, shift, act, dgamma, dbeta, work, coef,
                          stream);
}
SEG_API int seg_bn_bwd_coef_bf16io(const __bf16* da, long ldda, const __bf16* y, long ldy, long M, int C,
                                   const float* gamma, const float* mean, const float* invstd, const float* scale,
                                   const float* shift, int act, float* dgamma, float* dbeta, float* work, float* coef,
                                   hipStream_t stream) {
  return bn_bwd_coef_impl(da, ldda, y, ldy, M, C, gamma, mean, invstd, scale, shift, act, dgamma, dbeta, work, coef,
                          stream);
}
template <typename T>
static int bn_bwd_apply_impl(const T* da, long ldda, const T* y, long ldy, long M, int C, const float* mean,
                             const float* scale, const float* shift, int act, const float* coef, T* dy, long lddy,
                             hipStream_t stream) {
  if ((C & 3) || (ldy & 3) || (ldda & 3) || (lddy & 3)) return (int)hipErrorInvalidValue;
  launch_bn_bwd_apply<T>(da, ldda, y, ldy, M, C, scale, shift, mean, act, coef, dy, lddy, stream);
  SEG_RET_LAST();
}
SEG_API int seg_bn_bwd_apply(const float* da, long ldda, const float* y, long ldy, long M, int C, const float* mean,
                             const float* scale, const float* shift, int act, const float* coef, float* dy, long lddy,
                             hipStream_t stream) {
  return bn_bwd_apply_impl(da, ldda, y, ldy, M, C, mean, scale, shift, act, coef, dy, lddy, stream);
}
SEG_API int seg_bn_bwd_apply_bf16io(const __bf16* da, long ldda, const __bf16* y, long ldy, long M, int C,
                                    const float* mean, const float* scale, const float* shift, int act,
                                    const float* coef, __bf16* dy, long lddy, hipStream_t stream) {
  return bn_bwd_apply_impl(da, ldda, y, ldy, M, C, mean, scale, shift, act, coef, dy, lddy, stream);
}

// dgamma, dbeta and coef[3][C] (as seg_bn_bwd_coef) from the BN-backward tile partials of a
// producer's epilogue (seg_conv_igemm_bnout*: part[ntiles][2][C]) over M rows.
SEG_API int seg_bn_bwd_finalize_tiles(const float* part, int ntiles, long M, int C, const float* gamma,
                                      const float* invstd, float* dgamma, float* dbeta, float* coef,
                                      hipStream_t stream) {
  if (!part || ntiles < 1 || M < 1 || C < 1 || !invstd || !coef) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_finalize_tiles_kernel, dim3(seg_cdiv(C, 16)), dim3(256), 0, stream, part, ntiles, M, C,
                     gamma, invstd, dgamma, dbeta, coef);
  SEG_RET_LAST();
}

SEG_API int seg_bn_eval_backward(const float* da, long ldda, const float* y, long ldy, long M, int C,
                                 const float* scale, const float* shift, int act, float* dy, long lddy,
                                 hipStream_t stream) {
  hipLaunchKernelGGL(bn_eval_bwd_kernel, dim3(ew_grid(M * (C / 4))), dim3(256), 0, stream, da, ldda, y, ldy, M, C,
                     scale, shift, act, dy, lddy);
  SEG_RET_LAST();
}

// out[c] (+)= sum_r y[r][c]  -- conv bias gradient.  `work` >= seg_chan_workspace_floats.
template <typename T>
static int colsum_impl(const T* y, long ldy, long M, int C, float* work, float* out, int accumulate,
                       hipStream_t stream) {
  if ((ldy & 3)) return (int)hipErrorInvalidValue;
  const int C4 = (C + 3) & ~3;  // ld >= C4 is guaranteed by the buffer contract
  launch_chan_partial<2, T>(y, ldy, nullptr, 0L, M, C4, nullptr, nullptr, nullptr, 0, work, stream);
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3(seg_cdiv(C, 4)), dim3(256), 0, stream, work, chan_blocks(M), C, C4,
                     out, accumulate);
  SEG_RET_LAST();
}
SEG_API int seg_colsum(const float* y, long ldy, long M, int C, float* work, float* out, int accumulate,
                       hipStream_t stream) {
  return colsum_impl(y, ldy, M, C, work, out, accumulate, stream);
}
SEG_API int seg_colsum_bf16io(const __bf16* y, long ldy, long M, int C, float* work, float* out, int accumulate,
                              hipStream_t stream) {
  return colsum_impl(y, ldy, M, C, work, out, accumulate, stream);
}
