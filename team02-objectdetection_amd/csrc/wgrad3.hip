// Weight gradient of the wide 3x3 (and 1x1) convs on bf16 rows, built like igemm2 (round 6).
//
//   dW[co][tap][ci] = sum_p dY[p][co] * X[p + tap][ci]        (stride 1, pad ks/2)
//
// Replaces aten's convolution_backward weight path of src/unet.py:58,61 (the decoder's and UNet's
// double_conv), driven by loss.backward() at src/train.py:38.  The register-staged weight gradient
// (wgrad.hip) keeps one 32-pixel K chunk in flight per 4-wave block and ran these layers at 0.15-0.2 of
// the bf16 MFMA peak (PMC: MFMA busy 0.10, half its issue cycles VALU on the per-slot im2col cursors),
// and its weight gradients cost UNet 512x1024 bs 8 (BASELINE configs[4]) 5.5 ms of a 23.5 ms step
// (profiles/r06/ab_skip_wgrad.txt).  Here, as in igemm2's forward:
//  * GEMM view C[co][n] = sum_p A[co][p] B[n][p], n = tap * Cin + ci, K = output pixels; one 512-thread
//    block (8 waves, 64 x 64 or 64 x 32 wave tiles) owns a 128 x 256 or 64 x 256 (co, n) tile and a
//    contiguous run of 64-pixel K steps (a split-K slice); every K step is 64 consecutive pixels of one
//    image row (W % 64 == 0), so a step's im2col rows are contiguous runs of X and each lane's
//    16-byte chunk (8 input channels of one tap) is fixed for the whole launch -- no per-slot cursors;
//  * operands staged global -> LDS by LDS-DMA (global_load_lds_dwordx4), three LDS stages, two steps
//    in flight while one computes; padding taps and columns beyond 9 Cin read a zero page;
//  * both fragments (8 pixels of one row / column per lane) come from ds_read_b64_tr_b16 transposing
//    reads of the [pixel][channel] rows; the 16-byte chunks of row r are stored XOR-swizzled by
//    4 (r & 3) (the DMA loads each lane's source accordingly), so the 4 rows a 16-lane group reads sit
//    on disjoint banks;
//  * each block writes its fp32 partial as a slab [slice][Cout][9 Cin] -- seg_conv_wgrad's split-K
//    slab layout -- summed in fixed order by seg_conv_wgrad_reduce: deterministic, no atomics.
#include "common.h"

namespace {

constexpr int kKP = 64;     // pixels per K step
constexpr int kBN = 256;    // n (tap, ci) columns per block tile
constexpr int kNW = 8;      // waves per block
constexpr int kStages = 3;

__device__ __attribute__((aligned(16))) unsigned g_w3_zero[4];

struct Wgrad3Args {
  const __bf16* dy; long lddy;   // [M][lddy]
  const __bf16* x; long ldx;     // [N*H*W][ldx]
  float* part;                   // [splits][Cout][Nw]
  int N, H, W, Cin, Cout, Nw;    // Nw = ks * ks * Cin
  int tiles_m, tiles_n, splits, nsteps, sps;  // K steps in all / per slice
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

// XOR swizzle of the 16-byte chunks of row r in a tile with `row_bytes`-byte rows: the 4 consecutive rows a 16-lane
// group of ds_read_b64_tr_b16 reads land on disjoint banks (256 / 512-byte rows: 4 (r & 3); 128-byte rows, where
// rows r and r + 2 share banks: 4 ((r >> 1) & 1)).
__device__ __forceinline__ constexpr int w3_swz(int row_bytes, int r) {
  return row_bytes == 128 ? 4 * ((r >> 1) & 1) : 4 * (r & 3);
}

// BM: output channels per block (128: 64 x 64 wave tiles, 2 x 4 waves; 64: 64 x 32, 1 x 8).
template <int BM, int KS>
__global__ __launch_bounds__(kNW * 64) void wgrad3_kernel(Wgrad3Args a) {
  constexpr int WM = 64, WN = BM == 128 ? 64 : 32;
  constexpr int WAVES_N = kBN / WN;
  static_assert((BM / WM) * WAVES_N == kNW, "8 waves");
  constexpr int MI = WM / 32, NI = WN / 32;
  constexpr int A_ROW = BM * 2, B_ROW = kBN * 2;            // bytes per pixel row of each tile
  constexpr int A_BYTES = kKP * A_ROW, B_BYTES = kKP * B_ROW;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_RPI = 1024 / A_ROW, B_RPI = 1024 / B_ROW;  // rows per DMA instruction (1 KB)
  constexpr int NA = kKP / A_RPI / kNW, NB = kKP / B_RPI / kNW;  // DMA instructions per wave per step
  static_assert(NA * A_RPI * kNW == kKP && NB * B_RPI * kNW == kKP, "whole instructions per wave");
  __shared__ __attribute__((aligned(1024))) char smem[kStages * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  // every (co, n) tile of one pixel slice are adjacent logical ids: one XCD's L2 holds the slice's dY and X rows
  // for all of them
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int ntile = a.tiles_m * a.tiles_n;
  const int tile = lid % ntile, z = lid / ntile;
  const int tn = tile % a.tiles_n, tm = tile / a.tiles_n;
  const int co0 = tm * BM, n0 = tn * kBN;
  const int s_beg = z * a.sps;
  const int nst = min(a.nsteps - s_beg, a.sps);

  // ---- per-lane DMA sources.  A instruction j: rows A_RPI j .. (pixels), lane -> row A_RPI j + lane / (A_ROW / 16),
  // physical chunk lane % (A_ROW / 16) holding logical chunk phys ^ w3_swz(row) -- fixed per lane
  // (A_RPI is a multiple of 4).  B instruction j: rows B_RPI j + lane / 32 (B_RPI = 2), so row & 3 alternates with
  // j's parity: two logical chunks per lane, lcb[j & 1].
  constexpr int ACH = A_ROW / 16, BCH = B_ROW / 16;  // 16-byte chunks per row
  const int a_r = lane / ACH, a_pc = lane % ACH;
  const int a_lc = a_pc ^ w3_swz(A_ROW, a_r);  // A_RPI is a multiple of 4: row & 3 == a_r & 3
  const bool a_ok = co0 + 8 * a_lc < a.Cout;
  const long a_src = (long)(co0 + 8 * a_lc);
  const int b_r = lane / BCH, b_pc = lane % BCH;
  int b_ci[2], b_dy[2], b_dx[2];
  bool b_nok[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int row = 2 * v + b_r;  // (B_RPI j + b_r) & 3 for j even (v = 0) / odd (v = 1)
    const int lc = b_pc ^ w3_swz(B_ROW, row);
    const int n = n0 + 8 * lc;
    b_nok[v] = n < a.Nw;
    const int nn = b_nok[v] ? n : 0;
    const int tap = nn / a.Cin;
    b_ci[v] = nn - tap * a.Cin;
    b_dy[v] = KS == 3 ? tap / 3 - 1 : 0;
    b_dx[v] = KS == 3 ? tap % 3 - 1 : 0;
  }
  const long HW = (long)a.H * a.W;

  auto issue = [&](int s, int buf) {  // DMA of K step s (pixels 64 s .. 64 s + 63: one image row run) into `buf`
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
    const long p0 = (long)s * kKP;
    const int img = (int)(p0 / HW);
    const long rem = p0 - img * HW;
    const int h = (int)(rem / a.W), w0 = (int)(rem - (long)h * a.W);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int j = wave + kNW * i;
      const int px = A_RPI * j + a_r;
      dma16(a_ok ? (const void*)(a.dy + (p0 + px) * a.lddy + a_src) : (const void*)g_w3_zero, As + j * 1024);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int j = wave + kNW * i;
      const int v = j & 1;
      const int px = B_RPI * j + b_r;
      const int hs = h + b_dy[v], ws = w0 + px + b_dx[v];
      const bool ok = b_nok[v] && (unsigned)hs < (unsigned)a.H && (unsigned)ws < (unsigned)a.W;
      const __bf16* src = a.x + (((long)img * a.H + hs) * a.W + ws) * a.ldx + b_ci[v];
      dma16(ok ? (const void*)src : (const void*)g_w3_zero, Bs + j * 1024);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  // fragment reads: lane addresses row (pixel) 16 kk + 8 lh + q (+4 for the second half), columns c4 .. c4 + 3 of
  // its 32-wide block; the physical chunk of logical column c in row r is (c / 8) ^ w3_swz(row bytes, r)
  const int q = (lane & 15) >> 2, lh = lane >> 5;
  const int c4 = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  auto tr_addr = [&](int row_bytes, int row, int col) -> int {  // (row & 3 == q; bit 1 of row is bit 1 of q)
    return row * row_bytes + 16 * ((col >> 3) ^ w3_swz(row_bytes, q)) + 2 * (col & 7);
  };
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < kKP / 16; ++kk) {
      const int r0 = 16 * kk + 8 * lh + q;
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int col = wm0 + mi * 32 + c4;
        const __bf16* p0 = reinterpret_cast<const __bf16*>(As + tr_addr(A_ROW, r0, col));
        const __bf16* p1 = reinterpret_cast<const __bf16*>(As + tr_addr(A_ROW, r0 + 4, col));
        af[mi] = seg_cat8(seg_lds_tr4(p0), seg_lds_tr4(p1));
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int col = wn0 + ni * 32 + c4;
        const __bf16* p0 = reinterpret_cast<const __bf16*>(Bs + tr_addr(B_ROW, r0, col));
        const __bf16* p1 = reinterpret_cast<const __bf16*>(Bs + tr_addr(B_ROW, r0 + 4, col));
        bfr[ni] = seg_cat8(seg_lds_tr4(p0), seg_lds_tr4(p1));
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  // ---- K loop (igemm2's): buffer it % 3 holds step it; steps it + 1, it + 2 in flight meanwhile
  if (nst > 0) issue(s_beg, 0);
  if (nst > 1) issue(s_beg + 1, 1);
  if (nst > 2) issue(s_beg + 2, 2);
  for (int it = 0; it < nst; ++it) {
    const int ahead = min(nst - 1 - it, 2);
    if (ahead == 2) wait_vm<2 * (NA + NB)>();
    else if (ahead == 1) wait_vm<NA + NB>();
    else wait_vm<0>();
    raw_barrier();  // every wave's DMA of step `it` has landed
    const int buf = it % kStages;
    compute(buf);
    wait_lgkm0();
    raw_barrier();  // every wave is done reading `buf`
    if (it + kStages < nst) issue(s_beg + it + kStages, buf);
  }

  // ---- the slice's partial tile: C layout col = lane & 31 (n), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (co)
  float* slab = a.part + (long)z * a.Cout * a.Nw;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + (lane & 31);
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

#ifndef SEG_WG3_BLOCKS
#define SEG_WG3_BLOCKS 512  // target blocks (tiles x slices) of a launch
#endif
#ifndef SEG_WG3_MINSTEPS
#define SEG_WG3_MINSTEPS 8  // 64-pixel K steps per slice, at least
#endif

struct Plan3 {
  bool ok;
  int bm, tiles_m, tiles_n, splits, nsteps, sps;
};

Plan3 plan3(int N, int H, int W, int Cin, int Cout, int ks) {
  Plan3 p{};
  const long M = (long)N * H * W;
  if ((ks != 1 && ks != 3) || (Cin & 7) || (Cout & 7) || W % kKP || M < kKP || M / kKP > 0x7fffffffL || Cout < 32)
    return p;
  p.bm = Cout > 64 ? 128 : 64;
  p.tiles_m = seg_cdiv(Cout, p.bm);
  p.tiles_n = seg_cdiv((long)ks * ks * Cin, kBN);
  p.nsteps = (int)(M / kKP);
  const long tiles = (long)p.tiles_m * p.tiles_n;
  long s = std::max<long>(1, (SEG_WG3_BLOCKS + tiles - 1) / tiles);
  s = std::min<long>(s, std::max<long>(1, p.nsteps / SEG_WG3_MINSTEPS));
  s = std::min<long>(s, 1024);
  p.sps = seg_cdiv(p.nsteps, s);
  p.splits = seg_cdiv(p.nsteps, p.sps);  // no empty slice
  // padding columns of the 256-wide n tiles are wasted MFMA work: at most a quarter
  p.ok = (double)ks * ks * Cin / ((double)p.tiles_n * kBN) >= 0.75 && (double)Cout / (p.tiles_m * p.bm) >= 0.75;
  return p;
}

}  // namespace

// Slices (partial slabs) seg_conv_wgrad3_bf16io uses for this shape, or 0 when it does not apply (Cin, Cout
// multiples of 8, Cout >= 32, W a multiple of 64, little tile padding).  The workspace is splits * Cout * ks*ks*Cin
// floats; sum it with seg_conv_wgrad_reduce(part, splits, dW, Cout, Cin, ks, 0, accumulate).
SEG_API int seg_conv_wgrad3_splits(int N, int H, int W, int Cin, int Cout, int ks) {
  const Plan3 p = plan3(N, H, W, Cin, Cout, ks);
  return p.ok ? p.splits : 0;
}

// part[s][co][tap * Cin + ci] = sum over slice s's pixels of dY[p][co] * X[p + tap][ci] (stride 1, pad ks / 2),
// bf16 rows (ld % 8, 16-byte aligned), fp32 accumulation.
SEG_API int seg_conv_wgrad3_bf16io(const __bf16* dy, long lddy, const __bf16* x, long ldx, int N, int H, int W,
                                   int Cin, int Cout, int ks, float* part, hipStream_t stream) {
  const Plan3 p = plan3(N, H, W, Cin, Cout, ks);
  if (!p.ok || (lddy & 7) || (ldx & 7) || ((uintptr_t)dy & 15) || ((uintptr_t)x & 15) || !part)
    return (int)hipErrorInvalidValue;
  Wgrad3Args a;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.Nw = ks * ks * Cin;
  a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n; a.splits = p.splits; a.nsteps = p.nsteps; a.sps = p.sps;
  const dim3 grid(p.tiles_m * p.tiles_n * p.splits), block(kNW * 64);
  if (p.bm == 128) {
    if (ks == 3) hipLaunchKernelGGL((wgrad3_kernel<128, 3>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((wgrad3_kernel<128, 1>), grid, block, 0, stream, a);
  } else {
    if (ks == 3) hipLaunchKernelGGL((wgrad3_kernel<64, 3>), grid, block, 0, stream, a);
    else hipLaunchKernelGGL((wgrad3_kernel<64, 1>), grid, block, 0, stream, a);
  }
  SEG_RET_LAST();
}
