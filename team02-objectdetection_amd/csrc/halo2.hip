// Narrow 3x3 convolution (stride 1, pad 1) on bf16 rows for the bf16io configuration:
// a persistent LDS-halo kernel with the weights resident in LDS and the input halo
// streamed by LDS-DMA through a three-stage ring.
//
//   out[p][co] = sum_{tap, ci} in[p + tap][ci] * W[co][tap][ci] (+ bias) (+ add)
//
// Replaces aten's conv2d / convolution_backward(input) of the narrow decoder convs
// (src/unet.py:58,61 -- MobileNetV2UNet up3/up4: Cout 32-64, or their data gradients with
// 80 / 152 outputs; UNet's full-resolution 64-channel levels).  With so few output channels
// an implicit GEMM re-reads every input element once per tap from L2 (9 x the input per
// launch) and the first-generation halo kernel (halo.hip) stalls on every K chunk's loads
// (register staging, one chunk in flight: 104 us for up4.0's forward at bs=32, 2.7x its
// HBM time).  Here:
//  * one block per CU walks a contiguous run of 4 x 64-pixel output tiles (persistent), so
//    the weights are loaded into LDS ONCE per block, not once per tile;
//  * a dedicated loader wave streams the (4+2) x (64+2)-pixel input halo of each 32-channel
//    K chunk into a three-stage LDS ring by LDS-DMA (global_load_lds_dwordx4, no VGPR round
//    trip), two chunks in flight while the four compute waves work on the third; chunks of
//    the NEXT tile stream in while the current tile's epilogue runs;
//  * out-of-image halo pixels and channels beyond Cin read a 16-byte zero page (no branch);
//    halo pixels and weight rows are XOR-swizzled in 16-byte chunks (halo: chunk c of pixel
//    hp at c ^ ((hp >> 2) & 3); weights: wsw): conflict-free ds_read_b128 fragments;
//  * v_mfma_f32_32x32x16_bf16, fp32 accumulation; compute wave w owns output row w of the
//    tile (64 pixels = 2 MFMA row blocks) and all Cout columns (NI blocks of 32);
//  * epilogue as halo.hip's: bias, BatchNorm tile partials ([tile][2][Cout]: sum, then M2
//    about the tile mean; 256-row tiles, the same layout as seg_conv_halo_row_tiles), addend,
//    one rounding to bf16.  The compute waves never wait on their stores: only the loader
//    wave waits on vmcnt (for its own DMA), and the barriers are raw s_barriers.
// Numerics: every output element is the fp32 sum of exact bf16 x bf16 products in a fixed
// order (tap-major, then channel) -- deterministic, and the same rounding of operands as
// every other bf16io conv (tests/test_gpu_halo2.py compares against a float64 conv of the
// bf16 operands and against seg_conv_halo_bf16io_w16).
#include "common.h"

namespace {

constexpr int TH = 4, TW = 64;                  // output tile (pixels): one row per compute wave
constexpr int HH = TH + 2, HWP = TW + 2;        // halo tile
constexpr int BK = 32;                          // K chunk (input channels) = 64 B per pixel
constexpr int HALO_SLOTS = HH * HWP * (BK / 8); // 16-byte slots per ring stage (1584)
constexpr int HALO_DMA = (HALO_SLOTS + 63) / 64;  // DMA instructions per stage (25, 1 KB each)
constexpr int STAGE = HALO_DMA * 1024;          // bytes per ring stage
constexpr int kCompute = 4;                     // compute waves
constexpr int kThreads = (kCompute + 1) * 64;   // + one loader wave
constexpr int LDS_BYTES = 160 * 1024;
constexpr int RED_FLOATS = 2 * kCompute * 96 + 96;  // two reduction row sets + tile means (NI <= 3)
// ring stages NS (3 or 4: NS - 1 chunks in flight while one computes), chosen per launch by what
// the resident weights leave of the LDS
constexpr int w_off(int ns) { return ns * STAGE + RED_FLOATS * 4; }
constexpr int w_max(int ns) { return LDS_BYTES - w_off(ns); }  // bytes available for the resident weights

static_assert(2 * HALO_DMA <= 63, "vmcnt immediate");
#ifndef SEG_H2_NS4
#define SEG_H2_NS4 1  // four ring stages where the weights leave room (0: always three)
#endif

__device__ __attribute__((aligned(16))) unsigned g_h2_zero[4];

struct Halo2Args {
  const __bf16* in; long ldin;
  const __bf16* wk; int ldk;       // [Cout][ldk] bf16 (seg_pack_batch mode 16 / 17), k = tap * Cin + ci
  const float* bias;
  const __bf16* add; long ldadd;   // may alias out
  __bf16* out; long ldout;
  float* stat;                     // BN partials [tiles][2][Cout] (256-pixel tiles) or null
  int N, H, W, Cin, Cout;
  int tiles_w, tiles_h, ntiles, nk, wrow;  // wrow: LDS weight row stride (bytes) = nk * 64
};

// Weight-row chunk swizzle (row stride nk * 64 bytes, no padding): the 16 lanes of a
// ds_read_b128 group read 16 rows' chunk q on 16 distinct 16-byte bank quads for every nk
// (checked exhaustively for nk 1-8 against the gfx950 lane grouping).
__device__ __forceinline__ int wsw(int q, int row, int nk) {
  return (nk & 1) ? q ^ ((row >> 2) & 3) : (nk & 2) ? q ^ ((row >> 1) & 7) : q ^ (row & 15);
}

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Workgroup barrier that is also a compiler fence for memory but emits no wait: LDS-DMA
// transfers and global stores stay in flight across it.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);  // vmcnt N (6 bits split), others untouched
}

template <int NI, int NS>
__global__ __launch_bounds__(kThreads) void halo2_kernel(Halo2Args a) {
  constexpr int BNC = 32 * NI;
  constexpr int W_OFF = w_off(NS);
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* ring = smem;
  float* red0 = reinterpret_cast<float*>(smem + NS * STAGE);  // [kCompute][BNC]
  float* red1 = red0 + kCompute * BNC;                        // [kCompute][BNC]
  float* tmean = red1 + kCompute * BNC;                       // [BNC]
  char* Ws = smem + W_OFF;                                    // [9 * BNC rows][wrow bytes]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int t_beg = (int)((long)lid * a.ntiles / gridDim.x);
  const int t_end = (int)((long)(lid + 1) * a.ntiles / gridDim.x);
  const int nk = a.nk;
  const int S = (t_end - t_beg) * nk;  // (tile, K chunk) steps of this block

  // ---- resident weights: row (tap, co) = the Cin (padded to nk * 32) weights of one tap and
  // output channel in 16-byte chunks, chunk q stored at wsw(q, row) (conflict-free fragment reads)
  if (wave < kCompute) {  // (the loader wave starts its DMA meanwhile)
    const int qpr = nk * 4;  // 16-byte chunks per row
    for (int i = tid; i < 9 * BNC * qpr; i += kCompute * 64) {
      const int row = i / qpr, q = i - row * qpr;
      const int tap = row / BNC, co = row - tap * BNC, ci = q * 8;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (co < a.Cout && ci < a.Cin) v = *reinterpret_cast<const f32x4*>(a.wk + (long)co * a.ldk + tap * a.Cin + ci);
      *reinterpret_cast<f32x4*>(Ws + row * a.wrow + wsw(q, row, nk) * 16) = v;
    }
  }

  if (wave == kCompute) {
    // ======================= loader wave =======================
    // slot g = 64 j + lane of a stage: halo pixel hp = g >> 2, physical chunk g & 3, logical
    // chunk (g & 3) ^ ((hp >> 2) & 3) -- the channel offset of a lane is the same for every j
    const int cof = 8 * ((lane & 3) ^ ((lane >> 4) & 3));
    // tile-invariant slot geometry: element offset of the slot's pixel from the halo origin
    // (h0 - 1, w0 - 1), and its (hy, hx) for the edge tiles' bounds test (-1: beyond the halo)
    int rel[HALO_DMA], hyx[HALO_DMA];
#pragma unroll
    for (int j = 0; j < HALO_DMA; ++j) {
      const int hp = 16 * j + (lane >> 2);
      const int hy = hp / HWP, hx = hp - hy * HWP;
      rel[j] = (hy * a.W + hx) * (int)a.ldin;
      hyx[j] = hp < HH * HWP ? (hy << 8 | hx) : -1;
    }
    int cur_tile = -1, org = 0;
    unsigned okm = 0;  // slots of the current tile holding in-image pixels
    auto issue = [&](int step) {
      const int tl = t_beg + step / nk, kc = step - (step / nk) * nk;
      if (tl != cur_tile) {  // per tile: one scalar origin, and bounds tests only on the image edges
        cur_tile = tl;
        const int tw_i = tl % a.tiles_w, rest = tl / a.tiles_w;
        const int th_i = rest % a.tiles_h, n = rest / a.tiles_h;
        const int h0 = th_i * TH - 1, w0 = tw_i * TW - 1;
        org = ((n * a.H + h0) * a.W + w0) * (int)a.ldin;
        const bool interior = h0 >= 0 && h0 + HH <= a.H && w0 >= 0 && w0 + HWP <= a.W;
        okm = 0;
#pragma unroll
        for (int j = 0; j < HALO_DMA; ++j) {
          const int hy = hyx[j] >> 8, hx = hyx[j] & 255;
          const bool ok = hyx[j] >= 0 && (interior || ((unsigned)(h0 + hy) < (unsigned)a.H &&
                                                       (unsigned)(w0 + hx) < (unsigned)a.W));
          okm |= ok ? 1u << j : 0u;
        }
      }
      const int ch = kc * BK + cof;
      const unsigned m = ch < a.Cin ? okm : 0u;
      char* st = ring + (step % NS) * STAGE;
#pragma unroll
      for (int j = 0; j < HALO_DMA; ++j) {
        const bool ok = (m >> j) & 1u;
        dma16(ok ? (const void*)(a.in + (org + rel[j] + ch)) : (const void*)g_h2_zero, st + j * 1024);
      }
    };
    for (int s = 0; s < NS - 1 && s < S; ++s) issue(s);
    for (int s = 0; s < S; ++s) {
      // step s has landed; the steps issued after it (up to NS - 2) may still be in flight
      const int ahead = min(NS - 2, S - 1 - s);
      if (NS >= 4 && ahead >= 2) wait_vm<2 * HALO_DMA>();
      else if (ahead >= 1) wait_vm<HALO_DMA>();
      else wait_vm<0>();
      raw_barrier();                         // A: every compute wave is done with step s - 1's stage
      if (s + NS - 1 < S) issue(s + NS - 1); // ... which this refills
      if (s % nk == nk - 1) {                // the epilogue's three barriers
        raw_barrier();
        raw_barrier();
        raw_barrier();
      }
    }
    return;
  }

  // ======================= compute waves =======================
  const int fr = lane & 31, fh = lane >> 5;
  f32x16 acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  float bias[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) bias[ni] = (a.bias && ni * 32 + fr < a.Cout) ? a.bias[ni * 32 + fr] : 0.f;
  for (int s = 0; s < S; ++s) {
    const int tl = t_beg + s / nk, kc = s - (s / nk) * nk;
    wait_lgkm0();   // this wave's fragment reads of the previous stage (and its weight stores) are done
    raw_barrier();  // A
    const char* Hs = ring + (s % NS) * STAGE;
    const int rem = a.Cin - kc * BK;  // valid channels of this chunk (the last one may be half empty)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks == 1 && rem <= 16) break;
        const int c = 2 * ks + fh;
        bf16x8 af[2], bfr[NI];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          const int hp = (wave + ky) * HWP + mi * 32 + fr + kx;
          af[mi] = *reinterpret_cast<const bf16x8*>(Hs + hp * 64 + 16 * (c ^ ((hp >> 2) & 3)));
        }
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const int row = tap * BNC + ni * 32 + fr;
          bfr[ni] = *reinterpret_cast<const bf16x8*>(Ws + row * a.wrow + wsw(4 * kc + c, row, nk) * 16);
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    if (kc != nk - 1) continue;

    // ---- epilogue of tile tl (C layout of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4 fh)
    const int tw_i = tl % a.tiles_w, rest = tl / a.tiles_w;
    const int th_i = rest % a.tiles_h, n = rest / a.tiles_h;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] += bias[ni];
    // BatchNorm partials of the 256-pixel tile: column sums, then M2 about the tile mean
    // (three barriers, matched by the loader wave; red0 / red1 alternate so no barrier is
    // needed after the last read)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      float sum = 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += acc[mi][ni][r];
      sum += __shfl_xor(sum, 32, 64);
      if (lane < 32) red0[wave * BNC + ni * 32 + fr] = sum;
    }
    wait_lgkm0();
    raw_barrier();  // B
    if (tid < BNC) {
      const float t = red0[tid] + red0[BNC + tid] + red0[2 * BNC + tid] + red0[3 * BNC + tid];
      tmean[tid] = t / (float)(TH * TW);
      if (a.stat && tid < a.Cout) a.stat[(long)tl * 2 * a.Cout + tid] = t;
    }
    wait_lgkm0();
    raw_barrier();  // C
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const float mu = tmean[ni * 32 + fr];
      float sq = 0.f;
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[mi][ni][r] - mu;
          sq += d * d;
        }
      sq += __shfl_xor(sq, 32, 64);
      if (lane < 32) red1[wave * BNC + ni * 32 + fr] = sq;
    }
    wait_lgkm0();
    raw_barrier();  // D
    if (tid < BNC && a.stat && tid < a.Cout) {
      const float t = red1[tid] + red1[BNC + tid] + red1[2 * BNC + tid] + red1[3 * BNC + tid];
      a.stat[((long)tl * 2 + 1) * a.Cout + tid] = t;
    }
    const long pix0 = ((long)n * a.H + th_i * TH + wave) * a.W + tw_i * TW;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = ni * 32 + fr;
      if (col < a.Cout) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const long p = pix0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            float v = acc[mi][ni][r];
            if (a.add) v += (float)a.add[p * a.ldadd + col];
            a.out[p * a.ldout + col] = static_cast<__bf16>(v);
          }
      }
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    }
  }
}

int h2_nk(int Cin) { return (Cin + BK - 1) / BK; }
int h2_ni(int Cout) { return (Cout + 31) / 32; }
int h2_wbytes(int Cin, int Cout) { return 9 * 32 * h2_ni(Cout) * h2_nk(Cin) * 64; }

}  // namespace

// 1 when seg_conv_halo2_bf16io handles this stride-1 pad-1 3x3 conv: H % 4 == 0, W % 64 == 0,
// Cin % 8 == 0, Cout <= 96 and the weights (9 x Cout x Cin, padded) fit in LDS beside the ring.
SEG_API int seg_conv_halo2_ok(int N, int H, int W, int Cin, int Cout) {
  return (N > 0 && H > 0 && W > 0 && H % TH == 0 && W % TW == 0 && Cin >= 8 && Cin % 8 == 0 && Cout > 0 &&
          Cout <= 96 && h2_wbytes(Cin, Cout) <= w_max(3) && (long)N * H * W * 128 < 0x7fffffffL) ? 1 : 0;
}

// BN-partial row tiles of seg_conv_halo2_bf16io (256 pixels each; the layout of seg_conv_halo_row_tiles).
SEG_API int seg_conv_halo2_row_tiles(int N, int H, int W) { return N * (H / TH) * (W / TW); }

// out = conv3x3(in, W) (+bias) (+add), stride 1, pad 1, on bf16 rows with bf16-packed weights
// (seg_pack_batch mode 16 forward / 17 data gradient; ldk % 8 == 0, ldk >= 9 * Cin); fp32
// accumulation, one rounding on the store.  stat (optional): BN partials [row tiles][2][Cout].
// in / out / add rows: ld multiples of 8, 16-byte aligned bases for in.
SEG_API int seg_conv_halo2_bf16io(const __bf16* in, long ldin, int N, int H, int W, int Cin, const __bf16* wk,
                                  int ldk, const float* bias, __bf16* out, long ldout, int Cout, const __bf16* add,
                                  long ldadd, float* stat, hipStream_t stream) {
  if (!seg_conv_halo2_ok(N, H, W, Cin, Cout) || (ldin & 7) || ldin < Cin || (ldk & 7) || ldk < 9 * Cin ||
      ((uintptr_t)in & 15) || ((uintptr_t)wk & 15) || ldout < Cout || (add && ldadd < Cout) ||
      (long)N * H * W * ldin >= 0x7fffffffL)
    return (int)hipErrorInvalidValue;
  Halo2Args a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias; a.add = add; a.ldadd = ldadd;
  a.out = out; a.ldout = ldout; a.stat = stat; a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.tiles_w = W / TW; a.tiles_h = H / TH; a.ntiles = N * a.tiles_h * a.tiles_w;
  a.nk = h2_nk(Cin); a.wrow = a.nk * 64;
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
      int n = 0;
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) cus = n;
    }
  }
  const int grid = std::min(a.ntiles, cus);
  const int ni = h2_ni(Cout);
  const bool ns4 = h2_wbytes(Cin, Cout) <= w_max(4) && SEG_H2_NS4;
#define SEG_H2(NI)                                                                                  \
  do {                                                                                               \
    if (ns4) hipLaunchKernelGGL((halo2_kernel<NI, 4>), dim3(grid), dim3(kThreads), 0, stream, a);   \
    else hipLaunchKernelGGL((halo2_kernel<NI, 3>), dim3(grid), dim3(kThreads), 0, stream, a);       \
  } while (0)
  if (ni == 1) SEG_H2(1);
  else if (ni == 2) SEG_H2(2);
  else SEG_H2(3);
#undef SEG_H2
  SEG_RET_LAST();
}
