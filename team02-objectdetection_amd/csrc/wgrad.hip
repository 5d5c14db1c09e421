// Weight gradient of the implicit-GEMM convolutions on f32 MFMA.
//
// Replaces aten's convolution_backward weight path for the dense 3x3
// (src/unet.py:58,61) and 1x1 convs (src/unet.py:113,116 and the torchvision
// InvertedResidual expand/project convs reached through src/unet.py:15-19) --
// 43 % of the reference CPU step together with the data gradient.
//
// GEMM view: C[co][n] = sum_p dY[p][co] * X[src(p, tap(n))][ci(n)],
//   rows co (Cout), columns n = tap*Cin + ci (Nw = ks*ks*Cin), K = output pixels.
// K is split over gridDim.y; each split writes its own fp32 partial slab and
// seg_conv_wgrad_reduce sums the slabs in fixed order (bitwise reproducible, no
// float atomics).  Both operands are staged k-major in LDS ([pixel][channel], the
// natural NHWC order, so global reads are whole channel runs); the MFMA operand
// read is one ds_read_b32 per lane, 32 consecutive floats per half-wave.
#include "common.h"

namespace {

#ifndef SEG_WGRAD_BLOCKS
// target blocks (tiles x splits) of an fp32 weight-gradient launch: 1024 measured beside the main stream with the
// Winograd weight gradient in place (profiles/r06/ab_wgrad_blocks*.txt): +0.3 / +0.7 % f32 on two boxes vs 2048,
// 512 -0.7 %, UNet f32 flat
#define SEG_WGRAD_BLOCKS 1024
#endif
#ifndef SEG_WGRAD_BLOCKS_BF16
#define SEG_WGRAD_BLOCKS_BF16 512
#endif
#ifndef SEG_WGRAD_BK
#define SEG_WGRAD_BK 16
#endif
#ifndef SEG_WGRAD_STAGES
#define SEG_WGRAD_STAGES 1  // measured: one LDS stage beats two by 2-12% (BK 16)
#endif
constexpr int BK = SEG_WGRAD_BK;
#ifndef SEG_WGRAD_BK_BF16
#define SEG_WGRAD_BK_BF16 32  // pixels per K step of the bf16 kernels (two 16-deep MFMA steps)
#endif

struct WgradArgs {
  const void* dy; long lddy;     // IT (float, or __bf16 for the _bf16io path)
  const void* x; long ldx;       // IT
  float* part;
  int N, H, W, Cin, Ho, Wo, Cout, stride, pad;
  int M, Nw, kchunk;
  // optional input transform of X (XF kernels; 3x3: real pixels only, padding stays zero): x = act(x * xs[c] + xb[c]) on
  // load -- the producer's lazy BatchNorm + activation (see seg_conv_igemm_xf)
  const float* xs; const float* xb; int xact;
};

// Row pitch (bf16 elements) of a k-major bf16 tile read with ds_read_b64_tr_b16: a
// 32-lane half reads 4 rows x 64 B, conflict-free when the pitch is 64 or 192 B mod 256.
constexpr int tr_pitch(int n) { return n % 128 == 32 || n % 128 == 96 ? n : tr_pitch(n + 32); }

// BF ("bf16 math", BASELINE configs[2]/[4]): operands rounded to bf16 (RNE) into LDS,
// still k-major ([pixel][channel], whole channel runs from HBM), 32 pixels per K chunk;
// the MFMA fragment (lane: row r, k = 8h .. 8h+7) is gathered with two
// ds_read_b64_tr_b16 (4 k-rows x 16 channels per 16-lane group, delivered
// column-major) and fed to v_mfma_f32_32x32x16_bf16; fp32 accumulation and slabs.
// VW: channels per load slot -- 8 (one 16-byte load, copied to LDS as is) on bf16
// storage when Cout, Cin and the row strides are multiples of 8, else 4.
template <int BM, int BN, int WM, int WN, int KS, bool BF = false, typename IT = float, int VW = 4, bool XF = false>
__global__ __launch_bounds__(256) void wgrad_kernel(WgradArgs a) {
  static_assert(VW == 4 || (BF && sizeof(IT) == 2), "16-byte slots carry bf16 operands");
  const IT* __restrict__ gdy = static_cast<const IT*>(a.dy);
  const IT* __restrict__ gx = static_cast<const IT*>(a.x);
  constexpr int BK = BF ? SEG_WGRAD_BK_BF16 : ::BK;  // pixels per K chunk
  constexpr int AR = BF ? tr_pitch(BM) : BM + 4, BR = BF ? tr_pitch(BN) : BN + 4;
  constexpr int A_VEC = BK * BM / VW, B_VEC = BK * BN / VW;
  constexpr int A_PER = (A_VEC + 255) / 256, B_PER = (B_VEC + 255) / 256;
  constexpr int MI = WM / 32, NI = WN / 32, WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");
  using lds_t = typename std::conditional<BF, __bf16, float>::type;

  __shared__ __attribute__((aligned(16))) lds_t As[SEG_WGRAD_STAGES][BK * AR];
  __shared__ __attribute__((aligned(16))) lds_t Bs[SEG_WGRAD_STAGES][BK * BR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  const int tiles_n = (a.Nw + BN - 1) / BN;
  const int tiles = tiles_n * ((a.Cout + BM - 1) / BM);
  // 1-D grid of tiles x splits; every XCD walks whole splits (all column tiles of
  // one pixel chunk share the L2 that holds that chunk of dY and X)
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int split = lid / tiles, tile = lid - split * tiles;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * a.kchunk;
  const int kend = min(a.M, kbeg + a.kchunk);

  // Fixed per-thread columns of the B (input) tile: decode tap / channel once.
  int b_prow[B_PER], b_ci[B_PER], b_ky[B_PER], b_kx[B_PER];
  bool b_ok[B_PER];
  // Pixel cursor of each B load row (advanced by BK per K step).
  int b_n[B_PER], b_ho[B_PER], b_wo[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int idx = tid + i * 256;
    b_prow[i] = idx / (BN / VW);
    const int ncol = n0 + (idx % (BN / VW)) * VW;
    b_ok[i] = idx < B_VEC && ncol < a.Nw;
    const int tap = b_ok[i] ? ncol / a.Cin : 0;
    b_ci[i] = b_ok[i] ? ncol - tap * a.Cin : 0;
    b_ky[i] = tap / KS;
    b_kx[i] = tap - b_ky[i] * KS;
    const int p = kbeg + b_prow[i];
    const int hw = a.Ho * a.Wo;
    b_n[i] = p / hw;
    const int rem = p - b_n[i] * hw;
    b_ho[i] = rem / a.Wo;
    b_wo[i] = rem - b_ho[i] * a.Wo;
  }

  // XF: each B slot's fixed channels' transform coefficients, and which slots of the
  // loaded chunk hold real pixels (padding / tail slots stay zero)
  f32x4 xbs[XF ? B_PER : 1][VW / 4], xbb[XF ? B_PER : 1][VW / 4];
  unsigned b_vm = 0;
  if constexpr (XF) {
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
#pragma unroll
      for (int j = 0; j < VW / 4; ++j) {
        xbs[i][j] = ld4(a.xs + (b_ok[i] ? b_ci[i] : 0) + 4 * j);
        xbb[i][j] = ld4(a.xb + (b_ok[i] ? b_ci[i] : 0) + 4 * j);
      }
  }
  f32x4 ra[A_PER], rb[B_PER];
  auto ldv = [](const IT* q) -> f32x4 {  // one load slot: 4 channels widened, or 8 bf16 raw
    if constexpr (VW == 8) return *reinterpret_cast<const f32x4*>(q);
    else return ld4(q);
  };
  auto load_tiles = [&](int k0) {  // k0 = first pixel of this chunk
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * 256;
      const int prow = idx / (BM / VW), c = co0 + (idx % (BM / VW)) * VW;
      const int p = k0 + prow;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const bool ok = idx < A_VEC && p < kend && c < a.Cout;
      if (ok) v = ldv(gdy + (long)p * a.lddy + c);
      ra[i] = v;
    }
    if (XF) b_vm = 0;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int p = k0 + b_prow[i];
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (b_ok[i] && p < kend) {
        if (KS == 1) {
          v = ldv(gx + (long)p * a.ldx + b_ci[i]);
          if (XF) b_vm |= 1u << i;
        } else {
          const int hi = b_ho[i] * a.stride - a.pad + b_ky[i];
          const int wi = b_wo[i] * a.stride - a.pad + b_kx[i];
          if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) {
            v = ldv(gx + (((long)b_n[i] * a.H + hi) * a.W + wi) * a.ldx + b_ci[i]);
            if (XF) b_vm |= 1u << i;
          }
        }
      }
      rb[i] = v;
      if (KS != 1) {  // advance this row's pixel cursor by BK
        int wo = b_wo[i] + BK, ho = b_ho[i], n = b_n[i];
        while (wo >= a.Wo) { wo -= a.Wo; if (++ho >= a.Ho) { ho = 0; ++n; } }
        b_wo[i] = wo; b_ho[i] = ho; b_n[i] = n;
      }
    }
  };
  auto st_op = [](lds_t* p, f32x4 v) {
    if constexpr (VW == 8) *reinterpret_cast<f32x4*>(p) = v;  // 8 bf16, already the operand type
    else if constexpr (BF) *reinterpret_cast<bf16x4*>(p) = __builtin_convertvector(v, bf16x4);
    else *reinterpret_cast<f32x4*>(p) = v;
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * 256;
      if (idx < A_VEC) {
        st_op(&As[buf][(idx / (BM / VW)) * AR + (idx % (BM / VW)) * VW], ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * 256;
      f32x4 v = rb[i];
      if constexpr (XF) {
        if ((b_vm >> i) & 1u) {
          if constexpr (VW == 8) {  // 8 bf16: widen, transform, round back as the BN-apply pass would
            const bf16x8 q = __builtin_bit_cast(bf16x8, v);
            const f32x4 lo = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 0, 1, 2, 3), f32x4),
                                         xbs[i][0], xbb[i][0], a.xact);
            const f32x4 hi = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 4, 5, 6, 7), f32x4),
                                         xbs[i][VW / 4 - 1], xbb[i][VW / 4 - 1], a.xact);
            v = __builtin_bit_cast(f32x4, seg_cat8(__builtin_convertvector(lo, bf16x4),
                                                   __builtin_convertvector(hi, bf16x4)));
          } else {
            v = seg_bn_act4(v, xbs[i][0], xbb[i][0], a.xact);
            if constexpr (sizeof(IT) == 2 && !BF)  // (not instantiated: bf16 storage implies bf16 math)
              v = __builtin_convertvector(__builtin_convertvector(v, bf16x4), f32x4);
          }
        }
      }
      if (idx < B_VEC) st_op(&Bs[buf][(idx / (BN / VW)) * BR + (idx % (BN / VW)) * VW], v);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int lrow = lane & 31, lh = lane >> 5;
  const int nk = (kend - kbeg + BK - 1) / BK;
  auto compute = [&](int cur) {
    if constexpr (BF) {
      // this lane's transposed-read address inside a 4 x 16 block: row q, columns 4p..4p+3,
      // block columns 16 * (lane >> 4 & 1) of the 32-wide fragment; k rows 8h + 4j + q
      const int q = (lane & 15) >> 2, c4 = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
        bf16x8 af[MI], bfr[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const lds_t* p = &As[cur][(16 * kk + 8 * lh + q) * AR + wm0 + mi * 32 + c4];
          af[mi] = seg_cat8(seg_lds_tr4(p), seg_lds_tr4(p + 4 * AR));
        }
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const lds_t* p = &Bs[cur][(16 * kk + 8 * lh + q) * BR + wn0 + ni * 32 + c4];
          bfr[ni] = seg_cat8(seg_lds_tr4(p), seg_lds_tr4(p + 4 * BR));
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
      return;
    }
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float af[MI], bf[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) af[mi] = As[cur][(2 * kk + lh) * AR + wm0 + mi * 32 + lrow];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bf[ni] = Bs[cur][(2 * kk + lh) * BR + wn0 + ni * 32 + lrow];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
      }
  };
  if (nk > 0) {
#if SEG_WGRAD_STAGES == 1
    load_tiles(kbeg);
    for (int kt = 0; kt < nk; ++kt) {
      store_tiles(0);
      __syncthreads();
      if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
      compute(0);
      __syncthreads();
    }
#else
    load_tiles(kbeg);
    store_tiles(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
      compute(cur);
      if (kt + 1 < nk) store_tiles(cur ^ 1);
      __syncthreads();
    }
#endif
  }

  float* slab = a.part + (long)split * a.Cout * a.Nw;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + lrow;
    if (col >= a.Nw) continue;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = co0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.Cout) slab[(long)row * a.Nw + col] = acc[mi][ni][r];
      }
  }
}

template <int BM, int BN, int WM, int WN, bool BF = false, typename IT = float>
int launch_wgrad(const WgradArgs& a, int ks, int splits, hipStream_t s) {
  dim3 grid(seg_cdiv(a.Cout, BM) * seg_cdiv(a.Nw, BN) * splits);
  if (a.xs) {  // input transform
    const bool v8 = sizeof(IT) == 2 && a.Cout % 8 == 0 && a.Cin % 8 == 0 && a.lddy % 8 == 0 && a.ldx % 8 == 0;
    if constexpr (sizeof(IT) == 2) {
      if (v8) {
        if (ks == 1) hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 1, true, IT, 8, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3, true, IT, 8, true>), grid, dim3(256), 0, s, a);
        SEG_RET_LAST();
      }
    }
    if (ks == 1) hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 1, BF, IT, 4, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3, BF, IT, 4, true>), grid, dim3(256), 0, s, a);
    SEG_RET_LAST();
  }
  if (BF) {
    const bool v8 = sizeof(IT) == 2 && a.Cout % 8 == 0 && a.Cin % 8 == 0 && a.lddy % 8 == 0 && a.ldx % 8 == 0;
    if constexpr (sizeof(IT) == 2) {
      if (v8) {
        if (ks == 1) hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 1, true, IT, 8>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3, true, IT, 8>), grid, dim3(256), 0, s, a);
        SEG_RET_LAST();
      }
    }
    if (ks == 1) {
      hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 1, true, IT>), grid, dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3, true, IT>), grid, dim3(256), 0, s, a);
    }
    SEG_RET_LAST();
  }
  if (ks == 1) hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 1>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, 3>), grid, dim3(256), 0, s, a);
  SEG_RET_LAST();
}

void wgrad_tiles(int Cout, int Nw, int* bm, int* bn) {
  if (Cout >= 128) { *bm = 128; *bn = Nw >= 128 ? 128 : 32; }
  else if (Cout >= 64) { *bm = 64; *bn = Nw >= 128 ? 128 : 64; }
  else { *bm = 32; *bn = 128; }
}

}  // namespace

// Number of K splits (partial slabs) seg_conv_wgrad will use; the caller provides
// a workspace of splits * Cout * ks*ks*Cin floats.
static int wgrad_splits(long M, int Cout, int Cin, int ks, long target_blocks) {
  const int Nw = ks * ks * Cin;
  int bm, bn;
  wgrad_tiles(Cout, Nw, &bm, &bn);
  const long tiles = (long)seg_cdiv(Cout, bm) * seg_cdiv(Nw, bn);
  long splits = (target_blocks + tiles - 1) / tiles;
  const long max_by_k = std::max<long>(1, M / 256);  // >= 256 pixels per split
  splits = std::min(splits, max_by_k);
  splits = std::min<long>(splits, 1024);  // small slabs (the stem: 32 x 36) need many splits to fill 256 CUs
  return (int)std::max<long>(1, splits);
}
#ifndef SEG_WGRAD_THIN
#define SEG_WGRAD_THIN 1024  // thin slabs (<= 2 tiles), same measurement
#endif
SEG_API int seg_conv_wgrad_splits(long M, int Cout, int Cin, int ks) {
  int bm, bn;
  wgrad_tiles(Cout, ks * ks * Cin, &bm, &bn);
  const long tiles = (long)seg_cdiv(Cout, bm) * seg_cdiv(ks * ks * Cin, bn);
  return wgrad_splits(M, Cout, Cin, ks, tiles <= 2 ? SEG_WGRAD_THIN : SEG_WGRAD_BLOCKS);
}
// Split count for the bf16-math weight gradients (seg_conv_wgrad_bf16 / _bf16io): a
// quarter of the blocks -- measured in the overlapped step (bf16io +1.7 %), where the
// side-stream weight gradients share the CUs with the data-gradient chain -- except for
// thin slabs (<= 2 output tiles), which take 1024 (+0.6 %).
#ifndef SEG_WGRAD_THIN_BF16
#define SEG_WGRAD_THIN_BF16 1024  // thin slabs (<= 2 tiles: the stem, OutConv, Cout-32 decoder convs): measured +0.6 % bf16io
#endif
#ifndef SEG_WGRAD_MAXPX_BF16
#define SEG_WGRAD_MAXPX_BF16 8192L  // measured: UNet 512x1024 bf16io +3.8 %, MobileNetV2UNet flat
#endif
SEG_API int seg_conv_wgrad_splits_bf16(long M, int Cout, int Cin, int ks) {
  int bm, bn;
  wgrad_tiles(Cout, ks * ks * Cin, &bm, &bn);
  const long tiles = (long)seg_cdiv(Cout, bm) * seg_cdiv(ks * ks * Cin, bn);
  long target = tiles <= 2 ? SEG_WGRAD_THIN_BF16 : SEG_WGRAD_BLOCKS_BF16;
  // bound the pixels per split (each block walks its split's 32-pixel chunks one after another)
  target = std::max<long>(target, tiles * seg_cdiv(M, SEG_WGRAD_MAXPX_BF16));
  return wgrad_splits(M, Cout, Cin, ks, target);
}

// part[s][co][tap*Cin+ci] = sum over split s's pixels of dY[p][co] * X[src(p,tap)][ci].
static int conv_wgrad(const void* dy, long lddy, const void* x, long ldx, int N, int H, int W, int Cin, int Ho,
                      int Wo, int Cout, int ks, int stride, int pad, float* part, int splits,
                      hipStream_t stream, bool bf = false, bool bf_io = false, const float* xs = nullptr,
                      const float* xb = nullptr, int xact = 0);

SEG_API int seg_conv_wgrad(const float* dy, long lddy, const float* x, long ldx,
                           int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                           int ks, int stride, int pad, float* part, int splits, hipStream_t stream) {
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream);
}

// seg_conv_wgrad with bf16 math (the bf16 configurations): operands rounded to bf16
// (RNE) in the LDS staging, fp32 accumulation, the same fp32 partial slabs.
SEG_API int seg_conv_wgrad_bf16(const float* dy, long lddy, const float* x, long ldx,
                                int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                                int ks, int stride, int pad, float* part, int splits, hipStream_t stream) {
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream,
                    true);
}

// seg_conv_wgrad_bf16 on bf16 activation storage (dy, x __bf16; the _bf16io training path).
SEG_API int seg_conv_wgrad_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx,
                                  int N, int H, int W, int Cin, int Ho, int Wo, int Cout,
                                  int ks, int stride, int pad, float* part, int splits, hipStream_t stream) {
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream,
                    true, true);
}

// seg_conv_wgrad(_bf16, _bf16io) of a 1x1 or 3x3 conv whose input X is the raw output of a
// BatchNorm'd producer: X = act(x * in_scale + in_shift) formed on load (the lazy BN of
// seg_conv_igemm_xf; the same value the BN-apply pass would have stored).
SEG_API int seg_conv_wgrad_xf(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int Cin,
                              int Ho, int Wo, int Cout, int ks, int stride, int pad, float* part, int splits,
                              const float* in_scale, const float* in_shift, int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream, false, false,
                    in_scale, in_shift, in_act);
}
SEG_API int seg_conv_wgrad_bf16_xf(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int Cin,
                                   int Ho, int Wo, int Cout, int ks, int stride, int pad, float* part, int splits,
                                   const float* in_scale, const float* in_shift, int in_act, hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream, true, false,
                    in_scale, in_shift, in_act);
}
SEG_API int seg_conv_wgrad_bf16io_xf(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W,
                                     int Cin, int Ho, int Wo, int Cout, int ks, int stride, int pad, float* part,
                                     int splits, const float* in_scale, const float* in_shift, int in_act,
                                     hipStream_t stream) {
  if (!in_scale) return (int)hipErrorInvalidValue;
  return conv_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Ho, Wo, Cout, ks, stride, pad, part, splits, stream, true, true,
                    in_scale, in_shift, in_act);
}

static int conv_wgrad(const void* dy, long lddy, const void* x, long ldx, int N, int H, int W, int Cin, int Ho,
                      int Wo, int Cout, int ks, int stride, int pad, float* part, int splits,
                      hipStream_t stream, bool bf, bool bf_io, const float* xs, const float* xb, int xact) {
  if ((Cin & 3) || (ldx & 3) || (lddy & 3) || (ks != 1 && ks != 3) || splits < 1) return (int)hipErrorInvalidValue;
  if (xs && (!xb || xact < SEG_ACT_NONE || xact > SEG_ACT_RELU6)) return (int)hipErrorInvalidValue;
  if (ks == 1 && (stride != 1 || pad != 0)) return (int)hipErrorInvalidValue;
  WgradArgs a;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.stride = stride; a.pad = pad; a.M = N * Ho * Wo; a.Nw = ks * ks * Cin;
  a.kchunk = seg_cdiv(seg_cdiv(a.M, splits), BK) * BK;
  a.xs = xs; a.xb = xb; a.xact = xact;
  int bm, bn;
  wgrad_tiles(Cout, a.Nw, &bm, &bn);
  if (bf_io) {
    a.kchunk = seg_cdiv(seg_cdiv(a.M, splits), 32) * 32;
    if (bm == 128 && bn == 128) return launch_wgrad<128, 128, 64, 64, true, __bf16>(a, ks, splits, stream);
    if (bm == 128) return launch_wgrad<128, 32, 32, 32, true, __bf16>(a, ks, splits, stream);
    if (bm == 64 && bn == 128) return launch_wgrad<64, 128, 32, 64, true, __bf16>(a, ks, splits, stream);
    if (bm == 64) return launch_wgrad<64, 64, 32, 32, true, __bf16>(a, ks, splits, stream);
    return launch_wgrad<32, 128, 32, 32, true, __bf16>(a, ks, splits, stream);
  }
  if (bf) {
    a.kchunk = seg_cdiv(seg_cdiv(a.M, splits), 32) * 32;
    if (bm == 128 && bn == 128) return launch_wgrad<128, 128, 64, 64, true>(a, ks, splits, stream);
    if (bm == 128) return launch_wgrad<128, 32, 32, 32, true>(a, ks, splits, stream);
    if (bm == 64 && bn == 128) return launch_wgrad<64, 128, 32, 64, true>(a, ks, splits, stream);
    if (bm == 64) return launch_wgrad<64, 64, 32, 32, true>(a, ks, splits, stream);
    return launch_wgrad<32, 128, 32, 32, true>(a, ks, splits, stream);
  }
  if (bm == 128 && bn == 128) return launch_wgrad<128, 128, 64, 64>(a, ks, splits, stream);
  if (bm == 128) return launch_wgrad<128, 32, 32, 32>(a, ks, splits, stream);
  if (bm == 64 && bn == 128) return launch_wgrad<64, 128, 32, 64>(a, ks, splits, stream);
  if (bm == 64) return launch_wgrad<64, 64, 32, 32>(a, ks, splits, stream);
  return launch_wgrad<32, 128, 32, 32>(a, ks, splits, stream);
}

// dW (PyTorch layout) = sum over the split-K partial slabs, fixed order.
//   mode 0: igemm partials part[s][co][tap][r4(Cin)] -> dW[co][ci][tap]
//           (channels >= Cin are the zero padding of a Cin % 4 != 0 input: dropped)
//   mode 1: depthwise partials part[s][tap][C]      -> dW[c][0][tap]
// Block = E slab elements x G = 256 / E split groups; each group sums every G-th slab
// with 4 independent accumulators, and the G group sums are added through LDS by a
// fixed pairwise tree, (g0 + g1) + (g2 + g3) ... (bitwise reproducible).  E = 64 / G = 4
// for large slabs; small slabs with many splits (the 1x1 head and the narrow decoder
// convs: 192..1344 elements, up to 1024 slabs) take E = 4..32 so more threads share
// the split dimension -- with 64 elements per block they ran 3-21 blocks whose
// threads each walked up to 256 slabs serially (50-110 us per launch).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, long slab,
                                                           float* __restrict__ dw, int Cout, int Cin, int taps,
                                                           int mode, int accumulate, int E) {
  __shared__ float red[256];
  const int G = 256 / E;
  const int lane = threadIdx.x % E, g = threadIdx.x / E;
  const long i = (long)blockIdx.x * E + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < slab) {
    int k = g;
    for (; k + 3 * G < splits; k += 4 * G) {
      s0 += part[(long)k * slab + i];
      s1 += part[(long)(k + G) * slab + i];
      s2 += part[(long)(k + 2 * G) * slab + i];
      s3 += part[(long)(k + 3 * G) * slab + i];
    }
    for (; k < splits; k += G) s0 += part[(long)k * slab + i];
  }
  red[threadIdx.x] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  for (int h = 1; h < G; h <<= 1) {  // red[g] += red[g + h] for g % 2h == 0
    if (g % (2 * h) == 0 && g + h < G) red[threadIdx.x] += red[threadIdx.x + h * E];
    __syncthreads();
  }
  if (g != 0 || i >= slab) return;
  const float s = red[lane];
  long o;
  if (mode == 0) {
    const int cp = (Cin + 3) & ~3;
    const long co = i / ((long)taps * cp);
    const int r = (int)(i - co * taps * cp);
    const int tap = r / cp, ci = r - tap * cp;
    if (ci >= Cin) return;
    o = (co * Cin + ci) * taps + tap;
  } else {
    const int tap = (int)(i / Cout), c = (int)(i - (long)tap * Cout);
    o = (long)c * taps + tap;
  }
  dw[o] = accumulate ? dw[o] + s : s;
}

SEG_API int seg_conv_wgrad_reduce(const float* part, int splits, float* dw, int Cout, int Cin, int ks,
                                  int mode, int accumulate, hipStream_t stream) {
  if (mode != 0 && mode != 1) return (int)hipErrorInvalidValue;
  const long slab = (long)Cout * (mode == 0 ? ((Cin + 3) & ~3) : Cin) * ks * ks;
  // elements per block: 64 when that still gives >= 256 blocks or few splits per group
  int E = 64;
  while (E > 4 && seg_cdiv(slab, E) < 256 && splits > 4 * (256 / E)) E >>= 1;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(seg_cdiv(slab, E)), dim3(256), 0, stream, part, splits, slab, dw,
                     Cout, Cin, ks * ks, mode, accumulate, E);
  SEG_RET_LAST();
}
