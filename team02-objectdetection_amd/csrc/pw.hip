// Thin-K pointwise (1x1) convolutions: K <= 32 input channels, N <= 192 output channels.
//
// Replaces aten's conv2d / convolution_backward(input) of the output-heavy 1x1 convs of the
// training step: torchvision InvertedResidual expand convs with few input channels (16 -> 96,
// 24 -> 144, 32 -> 192, reached through src/unet.py:15-19), outconv's convs (src/unet.py:113,
// 116), and the data gradients of the project convs whose output side is thin (dY with 16..32
// channels -> dX with 32..192).
//
// The generic implicit GEMM (igemm_impl.h) spends these launches in its block-level
// choreography -- operand staging through LDS, a barrier per K chunk and two per epilogue band
// -- for one or two K chunks of work per tile, so they ran at 1.1-2.9 TB/s of a ~5 TB/s copy.
// Here the whole weight matrix ([N][K], <= 24 KB) is loaded into LDS once per block, each
// wave streams 32-row tiles of the input straight from HBM into MFMA fragment registers (the
// next tile's loads in flight under the current tile's MFMAs), and every wave writes its
// outputs through a wave-private LDS transpose as 16-byte row vectors: the only block-wide
// barriers left are the BatchNorm-statistics reductions (when `stat` is requested).
//
// Blocks are persistent: 4 waves own the 4 x 32 rows of a 128-row tile (the BN partial
// tile), tiles strided by the grid.  Numerics: f32 storage uses v_mfma_f32_32x32x2_f32 (exact
// fp32 products, the igemm k-order permutation), bf16 storage v_mfma_f32_32x32x16_bf16; the
// epilogue (bias, addend, BN tile sum / M2 about the tile mean) is igemm's.
#include "common.h"

namespace {

constexpr int kPwThreads = 256;
constexpr int kPwRows = 128;  // rows per tile (4 waves x 32): the BN partials' tile

struct PwArgs {
  const void* in; long ldin;       // [M][ldin] storage type T
  const void* wk; int ldk;         // [N][ldk] weights (fp32 for T = float, bf16 for T = __bf16), k < K
  const float* bias;               // [N] or null
  const void* add; long ldadd;     // addend [M][ldadd] (may alias out) or null
  void* out; long ldout;
  float* stat;                     // BN partials [tiles][2][N] (tile sum, M2 about the tile mean) or null
  const float* xs; const float* xb; int xact;  // lazy BN of the input (act(x * xs + xb)) or null
  int M, K, N, tiles;
};

template <typename T, int NT, int KP, bool XF>
__global__ __launch_bounds__(kPwThreads) void pw_kernel(PwArgs a) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int BP = BF ? KP + 8 : KP + 4;  // LDS weight row pitch (elements): 16-byte aligned rows
  constexpr int NA = BF ? KP / 16 : KP / 8;  // A fragments per lane per tile (16-byte loads)
  constexpr int TP = 36;                     // transpose tile pitch (floats)
  __shared__ __attribute__((aligned(16))) T Bs[NT * 32 * BP];
  __shared__ __attribute__((aligned(16))) float Ts[4][32 * TP];
  __shared__ float red[4][NT * 32];
  __shared__ float tmean[NT * 32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const T* in = static_cast<const T*>(a.in);
  const T* add = static_cast<const T*>(a.add);
  T* out = static_cast<T*>(a.out);

  // weights -> LDS once: row n, k < K (zero beyond K / N)
  const T* wk = static_cast<const T*>(a.wk);
  for (int i = tid; i < NT * 32 * KP; i += kPwThreads) {
    const int n = i / KP, k = i - n * KP;
    Bs[n * BP + k] = (n < a.N && k < a.K) ? wk[(long)n * a.ldk + k] : static_cast<T>(0.f);
  }
  // lazy-BN coefficients of this lane's A channels (k = 16s + 8h .. +7 / 8c + 4h .. +3)
  f32x4 xsc[XF ? (BF ? 2 * NA : NA) : 1], xsh[XF ? (BF ? 2 * NA : NA) : 1];
  if constexpr (XF) {
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int k = BF ? 16 * s + 8 * h : 8 * s + 4 * h;
      const bool ok = k < a.K;
#pragma unroll
      for (int j = 0; j < (BF ? 2 : 1); ++j) {
        xsc[(BF ? 2 : 1) * s + j] = ok ? ld4(a.xs + k + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
        xsh[(BF ? 2 : 1) * s + j] = ok ? ld4(a.xb + k + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  __syncthreads();

  auto load_a = [&](int tile, f32x4 (&ra)[NA]) {
    const int row = tile * kPwRows + wave * 32 + lr;
    const bool rok = row < a.M;
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      const int k = BF ? 16 * s + 8 * h : 8 * s + 4 * h;
      if (rok && k < a.K) ra[s] = *reinterpret_cast<const f32x4*>(in + (long)row * a.ldin + k);
      else ra[s] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  f32x4 ra[NA];
  int tile = blockIdx.x;
  if (tile < a.tiles) load_a(tile, ra);
  for (; tile < a.tiles; tile += gridDim.x) {
    // this tile's A operand (lazy BN applied and rounded as the apply pass would store it)
    f32x4 cur[NA];
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      f32x4 v = ra[s];
      if constexpr (XF) {
        const int k = BF ? 16 * s + 8 * h : 8 * s + 4 * h;
        if (k < a.K) {
          if constexpr (BF) {
            const bf16x8 q = __builtin_bit_cast(bf16x8, v);
            const f32x4 lo = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 0, 1, 2, 3), f32x4),
                                         xsc[2 * s], xsh[2 * s], a.xact);
            const f32x4 hi = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 4, 5, 6, 7), f32x4),
                                         xsc[2 * s + 1], xsh[2 * s + 1], a.xact);
            v = __builtin_bit_cast(f32x4, seg_cat8(__builtin_convertvector(lo, bf16x4),
                                                   __builtin_convertvector(hi, bf16x4)));
          } else {
            v = seg_bn_act4(v, xsc[s], xsh[s], a.xact);
          }
        }
      }
      cur[s] = v;
    }
    if (tile + (int)gridDim.x < a.tiles) load_a(tile + gridDim.x, ra);  // next tile's loads in flight

    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
      for (int s = 0; s < NA; ++s) {
        const int k = BF ? 16 * s + 8 * h : 8 * s + 4 * h;
        const f32x4 b = *reinterpret_cast<const f32x4*>(&Bs[(t * 32 + lr) * BP + k]);
        if constexpr (BF) {
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, cur[s]),
                                                          __builtin_bit_cast(bf16x8, b), acc[t], 0, 0, 0);
        } else {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(cur[s][kk], b[kk], acc[t], 0, 0, 0);
        }
      }
    }

    // epilogue.  C layout: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const int m0 = tile * kPwRows;
    if (a.bias) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int col = t * 32 + lr;
        const float b = col < a.N ? a.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += b;
      }
    }
    if (a.stat) {  // BN tile partials: column sums, then sums of squared deviations from the tile mean
      const int nrows = min(kPwRows, a.M - m0);
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int cl = t * 32 + lr;
          const float mu = pass ? tmean[cl] : 0.f;
          float s = 0.f;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float d = acc[t][r] - mu;
            s += row < a.M ? (pass ? d * d : d) : 0.f;
          }
          s += __shfl_xor(s, 32, 64);
          if (h == 0) red[wave][cl] = s;
        }
        __syncthreads();
        if (tid < NT * 32) {
          const float tot = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
          if (pass == 0) tmean[tid] = tot / (float)nrows;
          if (tid < a.N) a.stat[((long)tile * 2 + pass) * a.N + tid] = tot;
        }
        __syncthreads();
      }
    }
    // stores through this wave's LDS transpose tile: 16-byte row vectors (+ addend)
    float* ts = Ts[wave];
    const int wrow0 = m0 + wave * 32;
    constexpr int VO = 16 / (int)sizeof(T);  // elements per 16-byte store
    constexpr int VPR = 32 / VO;             // vectors per 32-column row
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 16; ++r) ts[((r & 3) + 8 * (r >> 2) + 4 * h) * TP + lr] = acc[t][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS writes land before its reads
#pragma unroll
      for (int i = 0; i < 32 * VPR / 64; ++i) {
        const int v = lane + 64 * i;
        const int rr = v / VPR, cv = (v - rr * VPR) * VO;
        const int row = wrow0 + rr, col = t * 32 + cv;
        float o[VO];
#pragma unroll
        for (int j = 0; j < VO; j += 4) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(&ts[rr * TP + cv + j]);
          o[j] = q[0]; o[j + 1] = q[1]; o[j + 2] = q[2]; o[j + 3] = q[3];
        }
        if (row >= a.M || col >= a.N) continue;
        T* dst = out + (long)row * a.ldout + col;
        const T* ad = add ? add + (long)row * a.ldadd + col : nullptr;
        if (col + VO <= a.N) {
          if (ad) {
            if constexpr (BF) {
              const bf16x8 q = *reinterpret_cast<const bf16x8*>(ad);
#pragma unroll
              for (int j = 0; j < 8; ++j) o[j] += (float)q[j];
            } else {
              const f32x4 q = ld4(reinterpret_cast<const float*>(ad));
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] += q[j];
            }
          }
          if constexpr (BF) {
            const f32x4 lo = {o[0], o[1], o[2], o[3]}, hi = {o[4], o[5], o[6], o[7]};
            *reinterpret_cast<bf16x8*>(dst) = seg_cat8(__builtin_convertvector(lo, bf16x4),
                                                       __builtin_convertvector(hi, bf16x4));
          } else {
            *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
          }
        } else {
#pragma unroll
          for (int j = 0; j < VO; ++j) {
            if (col + j >= a.N) break;
            float x = o[j];
            if (ad) x += (float)ad[j];
            dst[j] = static_cast<T>(x);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
    }
  }
}

template <typename T, int NT, int KP>
void launch_pw(const PwArgs& a, int grid, hipStream_t s) {
  if (a.xs) hipLaunchKernelGGL((pw_kernel<T, NT, KP, true>), dim3(grid), dim3(kPwThreads), 0, s, a);
  else hipLaunchKernelGGL((pw_kernel<T, NT, KP, false>), dim3(grid), dim3(kPwThreads), 0, s, a);
}

template <typename T, int KP>
void launch_pw_n(const PwArgs& a, int grid, hipStream_t s) {
  switch ((a.N + 31) / 32) {
    case 1: launch_pw<T, 1, KP>(a, grid, s); break;
    case 2: launch_pw<T, 2, KP>(a, grid, s); break;
    case 3: launch_pw<T, 3, KP>(a, grid, s); break;
    case 4: launch_pw<T, 4, KP>(a, grid, s); break;
    case 5: launch_pw<T, 5, KP>(a, grid, s); break;
    default: launch_pw<T, 6, KP>(a, grid, s); break;
  }
}

template <typename T>
int pw_impl(const T* in, long ldin, long M, int K, const T* wk, int ldk, const float* bias, T* out, long ldout, int N,
            const T* add, long ldadd, float* stat, const float* xs, const float* xb, int xact, hipStream_t stream) {
  constexpr int V = sizeof(T) == 2 ? 8 : 4;
  if (M < 1 || K < 8 || K > 32 || (K & 7) || N < 1 || N > 192 || ldk < K || M > 0x7fffffffL ||
      (ldin % V) || (ldout % V) || (add && (ldadd % V)) || ((uintptr_t)in & 15) || ((uintptr_t)out & 15) ||
      (add && ((uintptr_t)add & 15)) || (xs && (!xb || xact < SEG_ACT_NONE || xact > SEG_ACT_RELU6)))
    return (int)hipErrorInvalidValue;
  PwArgs a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias; a.add = add; a.ldadd = ldadd;
  a.out = out; a.ldout = ldout; a.stat = stat; a.xs = xs; a.xb = xb; a.xact = xact;
  a.M = (int)M; a.K = K; a.N = N; a.tiles = seg_cdiv(M, kPwRows);
  const int grid = std::min(a.tiles, 1024);  // persistent blocks, 4 per CU (fewer resident when registers are short)
  if (K <= 16) launch_pw_n<T, 16>(a, grid, stream);
  else launch_pw_n<T, 32>(a, grid, stream);
  SEG_RET_LAST();
}

}  // namespace

// Row tiles (BN partial tiles of kPwRows rows) of seg_conv_pw for M output rows.
SEG_API int seg_conv_pw_row_tiles(long M) { return seg_cdiv(M, kPwRows); }

// out = in[M][K] . W^T (+ bias) (+ add): a 1x1 conv (stride 1) as a thin-K GEMM, K <= 32 and
// K % 8 == 0, N <= 192; wk [N][ldk] row-major (the conv weight [N][K] as is, or its data-gradient
// pack).  stat (optional): BN partials [seg_conv_pw_row_tiles(M)][2][N] for seg_bn_stats_tiles
// (tile_rows 128).  xs/xb/xact (optional): the producer's lazy BatchNorm + activation applied
// to the input on load.  Rows 16-byte aligned (ld % 4 floats).
SEG_API int seg_conv_pw(const float* in, long ldin, long M, int K, const float* wk, int ldk, const float* bias,
                        float* out, long ldout, int N, const float* add, long ldadd, float* stat, const float* xs,
                        const float* xb, int xact, hipStream_t stream) {
  return pw_impl(in, ldin, M, K, wk, ldk, bias, out, ldout, N, add, ldadd, stat, xs, xb, xact, stream);
}

// seg_conv_pw on bf16 rows with bf16 weights (the bf16io configuration): bf16 MFMA operands,
// fp32 accumulation, one rounding on the store (ld % 8, 16-byte aligned rows).
SEG_API int seg_conv_pw_bf16io(const __bf16* in, long ldin, long M, int K, const __bf16* wk, int ldk,
                               const float* bias, __bf16* out, long ldout, int N, const __bf16* add, long ldadd,
                               float* stat, const float* xs, const float* xb, int xact, hipStream_t stream) {
  return pw_impl(in, ldin, M, K, wk, ldk, bias, out, ldout, N, add, ldadd, stat, xs, xb, xact, stream);
}
