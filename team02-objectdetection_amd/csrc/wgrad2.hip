// Weight gradient of the narrow 3x3 convs on bf16 rows (bf16io configuration): a persistent
// LDS-halo kernel on the halo2.hip skeleton (VERDICT r3 item 3's convs, their weight path).
//
//   dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci]        (stride 1, pad 1)
//
// Replaces aten's convolution_backward weight path of src/unet.py:58,61 where Cout <= 64 and
// Cin is small enough for the accumulators (MobileNetV2UNet up3 / up4, UNet's 64-channel
// full-resolution levels).  The implicit-GEMM weight gradient (wgrad.hip) gathers the im2col
// columns of X once per (tap, channel) tile column -- 9 x the input through L2 per launch --
// and ran these layers at 0.3-1.2 TB/s; here each 4 x 64-pixel tile's input halo and dY tile
// are read once:
//  * one block per CU walks a contiguous run of output tiles; a loader wave streams, per step
//    (tile, 32-channel K chunk of X), the (4+2) x (64+2) halo chunk of X and the tile's dY rows
//    into an LDS ring by LDS-DMA (three stages for Cout <= 32, two for 64), one or two steps in
//    flight beside the one computing;
//  * the four compute waves own the (tap, 32-channel output block) accumulators round-robin,
//    all of them for every chunk of the current channel group (up to G chunks = G x 32 input
//    channels held in registers); more input channels than that walk the tiles again per group;
//  * operands are k-major in LDS ([pixel][channel], as DMA'd): both MFMA fragments (8 pixels of
//    one channel per lane) come from ds_read_b64_tr_b16 transposing reads;
//    v_mfma_f32_32x32x16_bf16, fp32 accumulation over the block's pixels in a fixed order;
//  * each block writes its fp32 partial dW as one slab [block][Cout][9][r4(Cin)] (the layout of
//    seg_conv_wgrad's split-K slabs), summed in fixed order by seg_conv_wgrad_reduce:
//    deterministic, no atomics.
#include "common.h"

namespace {

constexpr int TH = 4, TW = 64;
constexpr int HH = TH + 2, HWP = TW + 2;
constexpr int BK = 32;                              // input channels per X chunk
constexpr int HALO_SLOTS = HH * HWP * (BK / 8);     // 1584 16-byte slots
constexpr int HALO_DMA = (HALO_SLOTS + 63) / 64;    // 25
constexpr int X_BYTES = HALO_DMA * 1024;
constexpr int kCompute = 4;
constexpr int kThreads = (kCompute + 1) * 64;
constexpr int LDS_BYTES = 160 * 1024;

__device__ __attribute__((aligned(16))) unsigned g_w2_zero[4];

struct Wgrad2Args {
  const __bf16* dy; long lddy;   // [M][lddy] output gradient rows
  const __bf16* x; long ldx;     // [N*H*W][ldx] input rows
  float* part;                   // [gridDim.x][Cout][9][cinp]
  int N, H, W, Cin, Cout, cinp;
  int tiles_w, tiles_h, ntiles, nk, ngroups, gchunks;  // gchunks: K chunks per channel group
};

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}
// X stage layout: halo pixel hp's 32 channels at hp * 64 bytes, unswizzled -- a transposing read
// covers 4 consecutive pixel rows x 64 bytes, all 64 banks once (conflict-free as it stands)

// NM: 32-channel output blocks (Cout <= 32 NM); G: K chunks of X held per channel group.
template <int NM, int G>
__global__ __launch_bounds__(kThreads) void wgrad2_kernel(Wgrad2Args a) {
  constexpr int NP = 9 * NM;                     // (tap, output block) pairs per chunk
  constexpr int JPW = (NP + kCompute - 1) / kCompute;  // pairs per compute wave
  constexpr int COUT = 32 * NM;
  constexpr int DY_BYTES = TH * TW * COUT * 2;   // the tile's dY rows (bf16)
  constexpr int DY_DMA = DY_BYTES / 1024;
  constexpr int STEP_DMA = HALO_DMA + DY_DMA;
  constexpr int STAGE = X_BYTES + DY_BYTES;
  constexpr int NS = 3 * STAGE <= LDS_BYTES ? 3 : 2;  // ring stages (one step in flight beside the computing one)
  static_assert(NS * STAGE <= LDS_BYTES, "ring fits");
  static_assert(STEP_DMA <= 63, "vmcnt immediate");
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int t_beg = (int)((long)lid * a.ntiles / gridDim.x);
  const int t_end = (int)((long)(lid + 1) * a.ntiles / gridDim.x);
  const int nt = t_end - t_beg;
  // steps: (group g, tile, chunk c in group) in that nesting; gsize(g) chunks in group g
  auto gsize = [&](int g) { return min(a.gchunks, a.nk - g * a.gchunks); };

  if (wave == kCompute) {
    // ======================= loader wave =======================
    const int cof = 8 * (lane & 3);
    int rel[HALO_DMA], hyx[HALO_DMA];
#pragma unroll
    for (int j = 0; j < HALO_DMA; ++j) {
      const int hp = 16 * j + (lane >> 2);
      const int hy = hp / HWP, hx = hp - hy * HWP;
      rel[j] = (hy * a.W + hx) * (int)a.ldx;
      hyx[j] = hp < HH * HWP ? (hy << 8 | hx) : -1;
    }
    // dY slots: 16-byte chunk u = 64 j + lane of the tile's rows: pixel u / (COUT / 8), chunk u % (COUT / 8)
    int cur = -1, org = 0;
    long dyo = 0;
    unsigned okm = 0;
    int s_issue = 0;  // the loader's own walk over (group, tile, chunk)
    int ig = 0, it = 0, ic = 0;
    auto issue = [&]() {
      const int tl = t_beg + it;
      if (tl != cur) {
        cur = tl;
        const int tw_i = tl % a.tiles_w, rest = tl / a.tiles_w;
        const int th_i = rest % a.tiles_h, n = rest / a.tiles_h;
        const int h0 = th_i * TH - 1, w0 = tw_i * TW - 1;
        org = ((n * a.H + h0) * a.W + w0) * (int)a.ldx;
        dyo = ((long)(n * a.H + th_i * TH) * a.W + tw_i * TW);
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
      const int kc = ig * a.gchunks + ic;
      const int ch = kc * BK + cof;
      const unsigned m = ch < a.Cin ? okm : 0u;
      char* st = smem + (s_issue % NS) * STAGE;
#pragma unroll
      for (int j = 0; j < HALO_DMA; ++j) {
        const bool ok = (m >> j) & 1u;
        dma16(ok ? (const void*)(a.x + (org + rel[j] + ch)) : (const void*)g_w2_zero, st + j * 1024);
      }
      char* sd = st + X_BYTES;
#pragma unroll
      for (int j = 0; j < DY_DMA; ++j) {
        const int u = 64 * j + lane;
        const int px = u / (COUT / 8), q = u - px * (COUT / 8);
        const int r = px / TW, c = px - r * TW;
        const bool ok = q * 8 < a.Cout;
        dma16(ok ? (const void*)(a.dy + (dyo + (long)r * a.W + c) * a.lddy + q * 8) : (const void*)g_w2_zero,
              sd + j * 1024);
      }
      ++s_issue;
      if (++ic == gsize(ig)) {
        ic = 0;
        if (++it == nt) {
          it = 0;
          ++ig;
        }
      }
    };
    int S = 0;
    for (int g = 0; g < a.ngroups; ++g) S += nt * gsize(g);
    for (int s = 0; s < NS - 1 && s < S; ++s) issue();
    for (int s = 0; s < S; ++s) {
      if (NS >= 3 && s + 1 < S) wait_vm<STEP_DMA>();
      else wait_vm<0>();
      raw_barrier();                 // A: step s landed; step s - 1's stage is free
      if (s + NS - 1 < S) issue();
    }
    return;
  }

  // ======================= compute waves =======================
  // pair jj of this wave = tap t and output block mb: p = wave + kCompute * jj, t = p / NM, mb = p % NM
  f32x16 acc[G][JPW];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < JPW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[g][j][r] = 0.f;
  // transposing-read lane roles: 16-lane group Gq = lane >> 4 covers columns 16 (Gq & 1) .. +15
  // of rows (k) 8 (Gq >> 1) + 4 t + q, lane 4q + p of the group addressing row q, columns 4p .. 4p+3
  const int gq = lane >> 4, li = lane & 15, q4 = li >> 2, p4 = li & 3;
  const int colb = 16 * (gq & 1) + 4 * p4;   // column (channel) of this lane's 8-byte read
  const int krow = 8 * (gq >> 1) + q4;      // k row within a 16-deep slice (+ 4 t)
  int s = 0;
  for (int g = 0; g < a.ngroups; ++g) {
    const int gs = min(a.gchunks, a.nk - g * a.gchunks);
    for (int it = 0; it < nt; ++it) {
#pragma unroll
      for (int c = 0; c < G; ++c) {
        if (c >= gs) break;
        wait_lgkm0();
        raw_barrier();  // A
        const char* Xs = smem + (s % NS) * STAGE;
        const char* Ds = Xs + X_BYTES;
        ++s;
        // per-lane parts of the transposing reads (k row krow, column colb), then per k slice a
        // wave-uniform base: slice ks = output row ks / 4, columns 16 (ks % 4) .. +15
        const char* xl = Xs + krow * 64 + 2 * colb;
        const char* dl = Ds + (krow * COUT + colb) * 2;
#pragma unroll 1
        for (int ks = 0; ks < 16; ++ks) {
          const int orow = ks >> 2, ocol = 16 * (ks & 3);
          const char* xk = xl + (orow * HWP + ocol) * 64;
          const char* dk = dl + (orow * TW + ocol) * COUT * 2;
          bf16x8 af[NM];
#pragma unroll
          for (int mb = 0; mb < NM; ++mb)
            af[mb] = seg_cat8(seg_lds_tr4(reinterpret_cast<const __bf16*>(dk + mb * 64)),
                              seg_lds_tr4(reinterpret_cast<const __bf16*>(dk + mb * 64 + 4 * COUT * 2)));
#pragma unroll
          for (int jj = 0; jj < JPW; ++jj) {
            const int p = wave + kCompute * jj;  // wave-uniform
            if (p >= NP) break;
            const int tap = p / NM, mb = p - (p / NM) * NM;
            const int ky = tap / 3, kx = tap - 3 * (tap / 3);
            const char* xb = xk + (ky * HWP + kx) * 64;
            const bf16x8 bfr = seg_cat8(seg_lds_tr4(reinterpret_cast<const __bf16*>(xb)),
                                        seg_lds_tr4(reinterpret_cast<const __bf16*>(xb + 4 * 64)));
            bf16x8 am = af[0];
#pragma unroll
            for (int m = 1; m < NM; ++m)
              if (mb == m) am = af[m];
            acc[c][jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bfr, acc[c][jj], 0, 0, 0);
          }
        }
      }
    }
    // the group's partial dW: slab [block][co][tap][cinp]; C layout: col (ci) = lane & 31,
    // row (co) = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* slab = a.part + (long)blockIdx.x * a.Cout * 9 * a.cinp;
    const int rs = 9 * a.cinp;  // slab row stride (one output channel)
#pragma unroll
    for (int cc = 0; cc < G; ++cc) {
      const int ci = (g * a.gchunks + cc) * BK + (lane & 31);
      const bool cok = cc < gs && ci < a.Cin;
#pragma unroll
      for (int jj = 0; jj < JPW; ++jj) {
        const int p = wave + kCompute * jj;
        if (p >= NP) break;
        const int tap = p / NM, mb = p - (p / NM) * NM;
        const int co0 = mb * 32 + 4 * (lane >> 5);
        float* base = slab + (co0 * 9 + tap) * a.cinp + ci;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int dco = (r & 3) + 8 * (r >> 2);
          if (cok && co0 + dco < a.Cout) __builtin_nontemporal_store(acc[cc][jj][r], base + dco * rs);
          acc[cc][jj][r] = 0.f;
        }
      }
    }
  }
}

int w2_nm(int Cout) { return (Cout + 31) / 32; }

}  // namespace

// 1 when seg_conv_wgrad2_bf16io handles this stride-1 pad-1 3x3 weight gradient: H % 4 == 0,
// W % 64 == 0, Cout <= 64 (Cout % 8 == 0), Cin % 8 == 0.
SEG_API int seg_conv_wgrad2_ok(int N, int H, int W, int Cin, int Cout) {
  return (N > 0 && H % TH == 0 && W % TW == 0 && Cin >= 8 && Cin % 8 == 0 && Cout >= 8 && Cout % 8 == 0 &&
          Cout <= 64 && (long)N * H * W * 256 < 0x7fffffffL) ? 1 : 0;
}

// Blocks (= partial slabs) of seg_conv_wgrad2_bf16io: part holds blocks * Cout * 9 * r4(Cin) floats,
// reduced by seg_conv_wgrad_reduce(part, blocks, dw, Cout, Cin, 3, 0, accumulate).
SEG_API int seg_conv_wgrad2_blocks(int N, int H, int W) {
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) cus = n;
  }
  return std::max(1, std::min(N * (H / TH) * (W / TW), cus));
}

SEG_API int seg_conv_wgrad2_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W,
                                   int Cin, int Cout, float* part, hipStream_t stream) {
  if (!seg_conv_wgrad2_ok(N, H, W, Cin, Cout) || (lddy & 7) || (ldx & 7) || lddy < Cout || ldx < Cin ||
      ((uintptr_t)dy & 15) || ((uintptr_t)x & 15) || (long)N * H * W * ldx >= 0x7fffffffL)
    return (int)hipErrorInvalidValue;
  Wgrad2Args a;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.cinp = (Cin + 3) & ~3;
  a.tiles_w = W / TW; a.tiles_h = H / TH; a.ntiles = N * a.tiles_h * a.tiles_w;
  a.nk = (Cin + BK - 1) / BK;
  const int nm = w2_nm(Cout);
  const int gmax = nm == 1 ? 3 : 2;  // accumulator budget: JPW x G x 16 registers per lane
  a.gchunks = std::min(a.nk, gmax);
  a.ngroups = (a.nk + a.gchunks - 1) / a.gchunks;
  const int grid = seg_conv_wgrad2_blocks(N, H, W);
#define SEG_W2(NM, G) hipLaunchKernelGGL((wgrad2_kernel<NM, G>), dim3(grid), dim3(kThreads), 0, stream, a)
  if (nm == 1) {
    if (a.gchunks == 1) SEG_W2(1, 1); else if (a.gchunks == 2) SEG_W2(1, 2); else SEG_W2(1, 3);
  } else {
    if (a.gchunks == 1) SEG_W2(2, 1); else SEG_W2(2, 2);
  }
#undef SEG_W2
  SEG_RET_LAST();
}
