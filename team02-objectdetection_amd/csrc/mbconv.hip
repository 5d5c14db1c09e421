// Fused inverted residual for the BatchNorm-folded inference forward (fp16 conv operands,
// BASELINE configs[3]): expand 1x1 + bias + ReLU6 -> depthwise 3x3 (stride 1 / 2) + bias +
// ReLU6 -> project 1x1 + bias (+ residual) in ONE launch per torchvision InvertedResidual
// (features[1..17], reached through src/unet.py:15-19,34-38; inference.py:162-163 runs them
// per frame).  At bs=1 and 128x256 frames every one of these convs is a few microseconds of
// work behind a launch (round 3: ~89 launches / frame, launch-latency bound); here the
// expanded activations never leave LDS.
//
// A block owns an output tile (4 x 8 pixels at stride 1, 2 x 8 at stride 2) and a range of
// the hidden channels (split `hsplit` of `splits`):
//  * the input halo tile ((T-1) S + 3 rows and columns, Cin channels) is staged once in LDS as
//    fp16 (round to nearest even, as seg_conv_igemm_f16 rounds its operands);
//  * per 32-channel hidden chunk: the expand conv on v_mfma_f32_16x16x32_f16 over the halo pixels
//    (fp32 accumulation, + bias, ReLU6, zero outside the image = the depthwise conv's padding) into
//    LDS as fp32; the depthwise conv in fp32 in dwconv.hip's tap order; its ReLU6 output rounded
//    to fp16; the project conv's partial product accumulated in registers over the chunks;
//  * splits > 1: each block stores its fp32 partial tile write-through; when the whole grid fits on
//    the chip at once every block of a tile waits for the tile's other splits and then combines its
//    1/splits share of the tile (the splits summed in order: deterministic) -- one block combining
//    a whole 32 x 320 tile of 15 splits took ~30 us; otherwise the last block to arrive
//    (seg_last_arrival) combines the tile; + bias, + residual, stored.
// Without an expand conv (features[1], expand ratio 1) the input tile itself is the hidden tile.
#include "common.h"

#ifndef SEG_MBCONV_CAP
#define SEG_MBCONV_CAP 256
#endif

static int g_combine_spin = -1;
int seg_combine_spin(int automatic) { return g_combine_spin >= 0 ? g_combine_spin : automatic; }
// Override the poll bound of every in-launch split combine (seg_mbconv_f16, seg_conv_igemm_*_ic): -1 = automatic,
// 0 = no poll (every block but a tile's last hands its piece over).  Test hook: results are the same either way.
SEG_API int seg_set_combine_spin(int spin) {
  g_combine_spin = spin < 0 ? -1 : spin;
  return 0;
}

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kThreads = 256;
constexpr int HC = 32;        // hidden channels per chunk (one K step of the project MFMA)
constexpr int kMaxCin = 160;  // expand input channels staged in LDS
constexpr int kMaxCout = 320;

struct MbArgs {
  const float* x; long ldx;           // block input [N*H*W][ldx] fp32
  const float* we; const float* be;   // folded expand weight [Ch][Cin], bias [Ch] (we == null: no expand, Ch == Cin)
  const float* wd; const float* bd;   // folded depthwise weight [9][Ch] (seg_pack_dw_weight layout), bias [Ch]
  const float* wp; const float* bp;   // folded project weight [Cout][Ch], bias [Cout]
  const float* res; long ldres;       // residual (the block input) or null
  float* out; long ldo;               // [N*Ho*Wo][ldo]
  int N, H, W, Cin, Ch, Cout, Ho, Wo;
  int tiles_w, tiles_h, ntiles, splits, hper;  // hper: hidden channels per split (multiple of HC)
  float* work; unsigned* cnt;         // splits > 1: partials [ntiles][splits][TP][Cout], counters [2][ntiles]
  int spin;                           // seg_tile_combine's poll bound (0: the grid is not co-resident)
};

__device__ __attribute__((aligned(16))) float g_mb_zero[4];

__device__ __forceinline__ float relu6(float v) { return fminf(fmaxf(v, 0.f), 6.f); }

template <int S> struct MbGeo {
  static constexpr int TOH = S == 1 ? 4 : 2, TOW = 8, TP = TOH * TOW;  // output tile
  static constexpr int IH = (TOH - 1) * S + 3, IW = (TOW - 1) * S + 3, HP = IH * IW;
  static constexpr int HPP = (HP + 15) / 16 * 16;                        // halo pixels in 16-row MFMA tiles
};

template <int S, bool EXP>
__global__ __launch_bounds__(kThreads) void mbconv_f16_kernel(MbArgs a) {
  using G = MbGeo<S>;
  constexpr int XR = kMaxCin + 8;  // fp16 row pitch of the staged input (16-byte reads, staggered banks)
  __shared__ __attribute__((aligned(16))) _Float16 Xs[EXP ? G::HPP * XR : 8];
  __shared__ __attribute__((aligned(16))) _Float16 Ws[EXP ? HC * XR : 8];        // the chunk's expand rows
  __shared__ __attribute__((aligned(16))) _Float16 Wps[kMaxCout * (HC + 8)];      // the chunk's project columns
  __shared__ __attribute__((aligned(16))) float Es[G::HPP * (HC + 1)];
  __shared__ __attribute__((aligned(16))) _Float16 Ds[G::TP * (HC + 8)];
  __shared__ int word[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int t = blockIdx.x, split = blockIdx.y;
  const int tw_i = t % a.tiles_w, rest = t / a.tiles_w;
  const int n = rest / a.tiles_h, oh0 = (rest % a.tiles_h) * G::TOH, ow0 = tw_i * G::TOW;
  const int ih0 = oh0 * S - 1, iw0 = ow0 * S - 1;
  const float* xim = a.x + (long)n * a.H * a.W * a.ldx;
  auto halo_in = [&](int hp, int& ih, int& iw) {
    const int hy = hp / G::IW, hx = hp - hy * G::IW;
    ih = ih0 + hy;
    iw = iw0 + hx;
    return hp < G::HP && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
  };
  const int cinp = (a.Cin + 31) & ~31;
  const int h_beg = split * a.hper, h_end = min(a.Ch, h_beg + a.hper);
  // the chunk weights: expand rows c0 .. c0 + 31 ([32][cinp]) and project columns ([Cout][32]) as fp16 in LDS,
  // this thread's depthwise taps and bias in registers.  Loaded one chunk ahead: the next chunk's loads are in
  // flight while this chunk computes.
  constexpr int WI = (HC * kMaxCin / 4 + kThreads - 1) / kThreads;  // expand float4s per thread
  constexpr int PI = (kMaxCout * HC / 4 + kThreads - 1) / kThreads; // project float4s per thread
  const int q4 = cinp / 4, dj = tid % HC;
  f32x4 we4[EXP ? WI : 1], wp4[PI];
  float w9n[9], dbn;
  auto load_w = [&](int c0) {
    if constexpr (EXP) {
#pragma unroll
      for (int k = 0; k < WI; ++k) {
        const int i = tid + k * kThreads, r = i / q4, c = (i - r * q4) * 4;
        const bool ok = i < HC * q4 && c0 + r < h_end && c < a.Cin;
        we4[k] = ld4(ok ? a.we + (long)(c0 + r) * a.Cin + c : reinterpret_cast<const float*>(g_mb_zero));
      }
    }
#pragma unroll
    for (int k = 0; k < PI; ++k) {
      const int i = tid + k * kThreads, co = i >> 3, c = (i & 7) * 4;
      const bool ok = co < a.Cout && c0 + c < h_end;
      wp4[k] = ld4(ok ? a.wp + (long)co * a.Ch + c0 + c : reinterpret_cast<const float*>(g_mb_zero));
    }
    const int dc = min(c0 + dj, a.Ch - 1);
#pragma unroll
    for (int k = 0; k < 9; ++k) w9n[k] = a.wd[k * a.Ch + dc];
    dbn = a.bd[dc];
  };
  if (h_beg < h_end) load_w(h_beg);  // in flight with the input halo below
  if constexpr (EXP) {  // the input halo as fp16, zero outside the image and beyond Cin (all loads issued together)
    const int q4 = cinp / 4;
    constexpr int XI = (G::HPP * (kMaxCin + 31) / 32 * 8 + kThreads - 1) / kThreads;
    f32x4 v[XI];
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + k * kThreads, hp = i / q4, c = (i - hp * q4) * 4;
      int ih, iw;
      const bool ok = i < G::HPP * q4 && halo_in(hp, ih, iw) && c < a.Cin;
      v[k] = ld4(ok ? xim + ((long)ih * a.W + iw) * a.ldx + c : reinterpret_cast<const float*>(g_mb_zero));
    }
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + k * kThreads, hp = i / q4, c = (i - hp * q4) * 4;
      if (i < G::HPP * q4) {
        _Float16* d = Xs + hp * XR + c;
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = (_Float16)v[k][j];
      }
    }
  }
  // project accumulators: (m, n) 16x16 tiles p = wave, wave + 4, ... of (TP / 16) x ceil(Cout / 16)
  constexpr int MT = G::TP / 16;
  const int NT = (a.Cout + 15) / 16;
  constexpr int PMAX = (MT * (kMaxCout / 16) + 3) / 4;
  f32x4 pacc[PMAX];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) pacc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r16 = lane & 15, kq = lane >> 4;  // MFMA lane geometry: row / column, 8-deep K group
  for (int c0 = h_beg; c0 < h_end; c0 += HC) {
    __syncthreads();  // Xs staged / the previous chunk's reads of Ws, Wps, Es, Ds are done
    if constexpr (EXP) {
#pragma unroll
      for (int k = 0; k < WI; ++k) {
        const int i = tid + k * kThreads, r = i / q4, c = (i - r * q4) * 4;
        if (i < HC * q4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) Ws[r * XR + c + j] = (_Float16)we4[k][j];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < PI; ++k) {
      const int i = tid + k * kThreads, co = i >> 3, c = (i & 7) * 4;
      if (co < a.Cout) {
#pragma unroll
        for (int j = 0; j < 4; ++j) Wps[co * (HC + 8) + c + j] = (_Float16)wp4[k][j];
      }
    }
    float w9[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) w9[k] = w9n[k];
    const float dbias = dbn;
    const int dc = c0 + dj;
    __syncthreads();
    if (c0 + HC < h_end) load_w(c0 + HC);
    if constexpr (EXP) {
      // expand: Es[hp][j] = relu6(sum_k X[hp][k] We[c0 + j][k] + be), (HPP / 16) x 2 tiles over the waves
      constexpr int ET = G::HPP / 16 * 2;
      for (int p = wave; p < ET; p += 4) {
        const int mt = p >> 1, nt = p & 1;
        const int hc = c0 + nt * 16 + r16;  // this lane's B column (hidden channel)
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < cinp; k0 += 32) {
          const f16x8 av = *reinterpret_cast<const f16x8*>(Xs + (mt * 16 + r16) * XR + k0 + 8 * kq);
          const f16x8 bv = *reinterpret_cast<const f16x8*>(Ws + (nt * 16 + r16) * XR + k0 + 8 * kq);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
        }
        const float b = hc < h_end ? a.be[hc] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // C: row 4 kq + i, column r16
          const int hp = mt * 16 + 4 * kq + i;
          int ih, iw;
          Es[hp * (HC + 1) + nt * 16 + r16] = halo_in(hp, ih, iw) ? relu6(acc[i] + b) : 0.f;
        }
      }
    } else {  // no expand: the hidden tile is the input tile (channels c0 ..), loads issued together
      constexpr int EI = (G::HPP * HC + kThreads - 1) / kThreads;
      float ev[EI];
#pragma unroll
      for (int k = 0; k < EI; ++k) {
        const int i = tid + k * kThreads, hp = i / HC, j = i - hp * HC, c = c0 + j;
        int ih, iw;
        const bool ok = i < G::HPP * HC && halo_in(hp, ih, iw) && c < h_end;
        ev[k] = ok ? xim[((long)ih * a.W + iw) * a.ldx + c] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < EI; ++k) {
        const int i = tid + k * kThreads, hp = i / HC, j = i - hp * HC;
        if (i < G::HPP * HC) Es[hp * (HC + 1) + j] = ev[k];
      }
    }
    __syncthreads();
    // depthwise 3x3 + bias + ReLU6 in fp32 (tap order of dwconv.hip), rounded to fp16 for the project MFMA
    {
      const int j = dj, c = dc;
      const float b = dbias;
      for (int px = tid / HC; px < G::TP; px += kThreads / HC) {
        const int oy = px / G::TOW, ox = px - oy * G::TOW;
        float acc = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx)
            acc = fmaf(Es[((oy * S + ky) * G::IW + ox * S + kx) * (HC + 1) + j], w9[ky * 3 + kx], acc);
        Ds[px * (HC + 8) + j] = (_Float16)(c < h_end ? relu6(acc + b) : 0.f);
      }
    }
    __syncthreads();
    // project partial: pacc[(m, n)] += D[m rows][32] . Wp[n cols][c0 .. c0 + 31]^T
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {
      const int p = wave + 4 * q;
      if (p < MT * NT) {
        const int mt = p % MT, nt = p / MT;
        const f16x8 av = *reinterpret_cast<const f16x8*>(Ds + (mt * 16 + r16) * (HC + 8) + 8 * kq);
        const int co = min(nt * 16 + r16, kMaxCout - 1);  // columns >= Cout: unused accumulator lanes
        const f16x8 bv = *reinterpret_cast<const f16x8*>(Wps + co * (HC + 8) + 8 * kq);
        pacc[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, pacc[q], 0, 0, 0);
      }
    }
  }
  // epilogue: C of tile (mt, nt): row 16 mt + 4 kq + i, column 16 nt + r16
  auto out_px = [&](int px, long& orow) {  // output pixel of tile row px, or false
    const int oy = oh0 + px / G::TOW, ox = ow0 + px % G::TOW;
    orow = ((long)n * a.Ho + oy) * a.Wo + ox;
    return oy < a.Ho && ox < a.Wo;
  };
  if (a.splits == 1) {
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {
      const int p = wave + 4 * q;
      const int mt = p % MT, co = (p / MT) * 16 + r16;
      if (p < MT * NT && co < a.Cout) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          long orow;
          if (out_px(mt * 16 + 4 * kq + i, orow)) {
            float v = pacc[q][i] + a.bp[co];
            if (a.res) v += a.res[orow * a.ldres + co];
            a.out[orow * a.ldo + co] = v;
          }
        }
      }
    }
    return;
  }
  float* wt = a.work + ((long)t * a.splits + split) * G::TP * a.Cout;
#pragma unroll
  for (int q = 0; q < PMAX; ++q) {
    const int p = wave + 4 * q;
    const int mt = p % MT, co = (p / MT) * 16 + r16;
    if (p < MT * NT && co < a.Cout) {
#pragma unroll
      for (int i = 0; i < 4; ++i) seg_st_wt(wt + (mt * 16 + 4 * kq + i) * a.Cout + co, pacc[q][i]);
    }
  }
  const float* w0 = a.work + (long)t * a.splits * G::TP * a.Cout;
  const int ne = G::TP * a.Cout;
  auto split_sum = [&](int e) {  // the splits in order, 16 loads in flight at a time
    float v = 0.f;
    for (int s0 = 0; s0 < a.splits; s0 += 16) {
      float q[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) q[j] = s0 + j < a.splits ? seg_ld_wt(w0 + (long)(s0 + j) * ne + e) : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (s0 + j < a.splits) v += q[j];
    }
    return v;
  };
  auto emit = [&](int e, float v) {
    const int px = e / a.Cout, co = e - px * a.Cout;
    long orow;
    if (out_px(px, orow)) {
      v += a.bp[co];
      if (a.res) v += a.res[orow * a.ldres + co];
      a.out[orow * a.ldo + co] = v;
    }
  };
  // the tile's splits combine it together when the grid is co-resident (a.spin), each its 1/splits share of the
  // tile's elements (the splits summed in order: deterministic); a block that cannot wait -- or, when the grid is
  // larger than the chip, every block but the last -- leaves its share to the tile's last arrival
  auto piece = [&](int pz) {
    const int e0 = (int)((long)pz * ne / a.splits), e1 = (int)((long)(pz + 1) * ne / a.splits);
    for (int e = e0 + tid; e < e1; e += kThreads) emit(e, split_sum(e));
  };
  seg_tile_combine(a.cnt + 4 * t, a.splits, split, a.spin, word, piece);
}

int g_mb_cap = SEG_MBCONV_CAP;  // blocks per launch the hidden splits aim for (seg_mbconv_tune)

void mb_plan(int N, int H, int W, int Ch, int stride, int* tiles_w, int* tiles_h, int* splits, int* hper, int* tp) {
  const int toh = stride == 1 ? 4 : 2, tow = 8;
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  *tiles_w = (Wo + tow - 1) / tow;
  *tiles_h = (Ho + toh - 1) / toh;
  *tp = toh * tow;
  const int ntiles = N * *tiles_w * *tiles_h;
  const int chunks = (Ch + HC - 1) / HC;
  // hidden splits: up to g_mb_cap blocks in all (co-resident, so every block of a tile helps combine it)
  // (at most 32: the width of seg_tile_combine's hand-off mask -- ADVICE r5; MobileNetV2's Ch <= 960 needs <= 30)
  int s = std::max(1, std::min({chunks, 32, g_mb_cap / std::max(1, ntiles)}));
  const int per = (chunks + s - 1) / s;
  *splits = (chunks + per - 1) / per;
  *hper = per * HC;
}

}  // namespace

// Tuning hook: the blocks per launch the hidden splits aim for (> 0; returns the previous value).
SEG_API int seg_mbconv_tune(int max_blocks) {
  const int old = g_mb_cap;
  if (max_blocks > 0) g_mb_cap = max_blocks;
  return old;
}

// 1 when seg_mbconv_f16 takes the block: stride 1 or 2, Cin <= 160 (with an expand conv), Cout <= 320,
// channel counts multiples of 4.
SEG_API int seg_mbconv_ok(int Cin, int Ch, int Cout, int stride, int expand) {
  return (stride == 1 || stride == 2) && Cin > 0 && Ch > 0 && Cout > 0 && Cin % 4 == 0 && Ch % 4 == 0 &&
                 Cout % 4 == 0 && Cout <= kMaxCout && (expand ? Cin <= kMaxCin : Cin == Ch)
             ? 1
             : 0;
}

// Workspace of seg_mbconv_f16: partial floats (0 when the plan does not split) and tile counters.
SEG_API long seg_mbconv_work_floats(int N, int H, int W, int Ch, int Cout, int stride, int* counters) {
  int tw, th, sp, hp, tp;
  mb_plan(N, H, W, Ch, stride, &tw, &th, &sp, &hp, &tp);
  if (counters) *counters = 4 * N * tw * th;
  return sp > 1 ? (long)N * tw * th * sp * tp * Cout : 0;
}

// out = project(relu6(dw3x3_s(relu6(expand(x))))) + bp (+ res): one torchvision InvertedResidual with
// its BatchNorms folded (seg_bn_fold_batch), fp16 conv operands with fp32 accumulation, fp32 depthwise.
// we == NULL: no expand conv (expand ratio 1; Ch == Cin).  work / cnt: seg_mbconv_work_floats floats and
// *counters unsigned (zero before the first launch; every launch re-arms them).
SEG_API int seg_mbconv_f16(const float* x, long ldx, int N, int H, int W, int Cin, const float* we, const float* be,
                           int Ch, const float* wd, const float* bd, int stride, const float* wp, const float* bp,
                           int Cout, const float* res, long ldres, float* out, long ldo, float* work, unsigned* cnt,
                           hipStream_t stream) {
  if (!seg_mbconv_ok(Cin, Ch, Cout, stride, we != nullptr) || !x || !wd || !bd || !wp || !bp || !out ||
      (we && !be) || (ldx & 3) || (ldo & 3) || (res && (ldres & 3)) || ((uintptr_t)x & 15) || ((uintptr_t)wp & 15) ||
      (we && ((uintptr_t)we & 15)) || (res && stride != 1))
    return (int)hipErrorInvalidValue;
  MbArgs a{};
  a.x = x; a.ldx = ldx; a.we = we; a.be = be; a.wd = wd; a.bd = bd; a.wp = wp; a.bp = bp; a.res = res;
  a.ldres = ldres; a.out = out; a.ldo = ldo; a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Ch = Ch; a.Cout = Cout;
  a.Ho = (H - 1) / stride + 1; a.Wo = (W - 1) / stride + 1;
  int tp;
  mb_plan(N, H, W, Ch, stride, &a.tiles_w, &a.tiles_h, &a.splits, &a.hper, &tp);
  a.ntiles = N * a.tiles_w * a.tiles_h;
  a.work = work; a.cnt = cnt;
  if (a.splits > 1 && (!work || !cnt)) return (int)hipErrorInvalidValue;
  if (a.splits > 32) return (int)hipErrorInvalidValue;  // seg_tile_combine's report mask
  const dim3 grid(a.ntiles, a.splits);
  const bool e = we != nullptr;
  {  // the splits wait for each other (bounded) only when the whole grid is co-resident
    const void* fn = stride == 1 ? (e ? (const void*)mbconv_f16_kernel<1, true> : (const void*)mbconv_f16_kernel<1, false>)
                                 : (e ? (const void*)mbconv_f16_kernel<2, true> : (const void*)mbconv_f16_kernel<2, false>);
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kThreads, 0) != hipSuccess) {
      (void)hipGetLastError();
      occ = 1;
    }
    a.spin = seg_combine_spin((long)a.ntiles * a.splits <= (long)std::max(occ, 1) * seg_num_cus() ? kSegCombineSpin : 0);
  }
  if (stride == 1) {
    if (e) hipLaunchKernelGGL((mbconv_f16_kernel<1, true>), grid, dim3(kThreads), 0, stream, a);
    else hipLaunchKernelGGL((mbconv_f16_kernel<1, false>), grid, dim3(kThreads), 0, stream, a);
  } else {
    if (e) hipLaunchKernelGGL((mbconv_f16_kernel<2, true>), grid, dim3(kThreads), 0, stream, a);
    else hipLaunchKernelGGL((mbconv_f16_kernel<2, false>), grid, dim3(kThreads), 0, stream, a);
  }
  SEG_RET_LAST();
}

// ---------------------------------------------------------------- the segmentation head
// outconv of the folded fp16 forward (src/unet.py:108-121: 1x1 -> BN -> ReLU -> 1x1, the BN folded) in one
// launch: out = w2 . f16(act(w1 . f16(x) + b1)) + b2, one pixel per thread, fp16-rounded operands and fp32
// accumulation as seg_conv_igemm_f16 stages them (the sum order differs: within fp32 rounding of the two
// launches).  Weights rounded once into LDS, read as wave-uniform broadcasts.
namespace {
template <int CIN, int C1>
__global__ __launch_bounds__(256) void pw2_f16_kernel(const float* __restrict__ x, long ldx, long M,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      int act1, const float* __restrict__ w2,
                                                      const float* __restrict__ b2, int C2, float* __restrict__ out,
                                                      long ldo) {
  __shared__ __attribute__((aligned(16))) float W1s[C1 * CIN];
  __shared__ __attribute__((aligned(16))) float W2s[64 * C1];
  __shared__ float B1s[C1], B2s[64];
  for (int i = threadIdx.x; i < C1 * CIN; i += 256) W1s[i] = (float)(_Float16)w1[i];
  for (int i = threadIdx.x; i < C2 * C1; i += 256) W2s[i] = (float)(_Float16)w2[i];
  for (int i = threadIdx.x; i < C1; i += 256) B1s[i] = b1 ? b1[i] : 0.f;
  for (int i = threadIdx.x; i < C2; i += 256) B2s[i] = b2 ? b2[i] : 0.f;
  __syncthreads();
  const long p = blockIdx.x * 256L + threadIdx.x;
  if (p >= M) return;
  float xv[CIN];
#pragma unroll
  for (int k = 0; k < CIN; k += 4) {
    const f32x4 v = ld4(x + p * ldx + k);
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[k + j] = (float)(_Float16)v[j];
  }
  float h[C1];
#pragma unroll
  for (int c = 0; c < C1; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < CIN; ++k) acc = fmaf(xv[k], W1s[c * CIN + k], acc);
    h[c] = (float)(_Float16)seg_act(acc + B1s[c], act1);
  }
  for (int c2 = 0; c2 < C2; ++c2) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < C1; ++c) acc = fmaf(h[c], W2s[c2 * C1 + c], acc);
    out[p * ldo + c2] = acc + B2s[c2];
  }
}
}  // namespace

// 1 when seg_pw2_f16 takes the head: (Cin, C1) = (32, 16) (MobileNetV2UNet's outconv(32, n)), C2 <= 64.
SEG_API int seg_pw2_ok(int Cin, int C1, int C2) { return Cin == 32 && C1 == 16 && C2 > 0 && C2 <= 64 ? 1 : 0; }

// out[M][ldo] = w2 [C2][C1] . f16(act1(w1 [C1][Cin] . f16(x) + b1)) + b2 (b1 / b2 may be NULL); x rows in
// 16-byte vectors (ldx % 4 == 0, 16-byte aligned).
SEG_API int seg_pw2_f16(const float* x, long ldx, long M, int Cin, const float* w1, const float* b1, int C1,
                        int act1, const float* w2, const float* b2, int C2, float* out, long ldo,
                        hipStream_t stream) {
  if (!seg_pw2_ok(Cin, C1, C2) || !x || !w1 || !w2 || !out || (ldx & 3) || ((uintptr_t)x & 15) || ldo < C2 ||
      act1 < SEG_ACT_NONE || act1 > SEG_ACT_RELU6 || M < 0)
    return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  hipLaunchKernelGGL((pw2_f16_kernel<32, 16>), dim3(seg_cdiv(M, 256)), dim3(256), 0, stream, x, ldx, M, w1, b1, act1,
                     w2, b2, C2, out, ldo);
  SEG_RET_LAST();
}
