// Winograd F(2x2, 3x3) convolution on the f32 matrix cores (stride 1, pad 1).
//
// The fp32 configuration is compute-bound on the dense 3x3 convs of the decoder
// (src/unet.py:58,61: 86 % of the forward FLOPs), and f32 MFMA runs at
// the f32 vector rate.  Winograd's minimal filtering F(2x2,3x3) computes each 2x2
// output tile from a 4x4 input tile with 16 multiplies per (input, output)
// channel pair instead of 36 -- 2.25x fewer MFMA FLOPs -- at the cost of input /
// output transforms (additions only) and a 16-way batched GEMM.  This is the
// algorithm MIOpen and cuDNN pick for fp32 3x3 convolutions; its rounding stays
// within a few ulps of the direct sum (tests: <= 1e-5 relative to torch's conv).
//
//   V_xi[t][ci] = (B^T d_t B)[xi]   d_t = 4x4 input patch of tile t (pad 1)
//   U_xi[co][ci] = (G g G^T)[xi]    g = w[co][ci] (seg_pack_batch modes 3/4)
//   M_xi[t][co] = sum_ci V_xi[t][ci] U_xi[co][ci]       (16 GEMMs, blockIdx.z = xi)
//   Y_t = A^T M_t A (+ bias, + addend, BatchNorm partials)  (wino_out_kernel)
// with B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; .5 .5 .5;
// .5 -.5 .5; 0 0 1], A^T = [1 1 1 0; 0 1 -1 -1].  Each row of B^T has two
// nonzeros, so V_xi of one tile is a signed sum of 4 input pixels: the GEMM's A
// loader forms it from 4 float4 loads -- V is never written to HBM.  M goes
// through HBM (16 x tiles x Cout floats); the output kernel fuses the BN
// statistics epilogue of seg_conv_igemm (same [row tile][2][Cout] partials,
// seg_conv_wino_tile_rows()-pixel row tiles) so seg_bn_stats_tiles finalizes either.
//
// The data gradient of a stride-1 3x3 conv is the same convolution of dY with
// the transposed, flipped weights (pack mode 4), so it runs on the same kernels.
#include "common.h"

#ifndef SEG_WINO_OUT_CSPLIT
#define SEG_WINO_OUT_CSPLIT 1  // output transform: one block per (64 tiles, 64 channels); 0 = channels walked in-block
#endif

#ifndef SEG_WINO_OUT_QT
#define SEG_WINO_OUT_QT 4  // output transform: tiles per tile lane (16 * QT tiles = 64 * QT pixels per BN row tile)
#endif

namespace {

constexpr int kWinoQT = SEG_WINO_OUT_QT;
__device__ __attribute__((aligned(16))) float g_wzero4[4];

struct WinoArgs {
  const float* in; long ldin;   // NHWC conv input [N*H*W][ldin]
  const float* wk; int ldk;      // U [16][Cout][ldk]
  float* m;                      // M [16][T][Cout]
  int N, H, W, Cin, Cout;
  int T, th, tw;                 // tiles, tiles per column / row
};

// Nonzeros of row r of B^T: positions p0, p1 with signs s0, s1.
__device__ __forceinline__ void bt_row(int r, int& p0, int& p1, float& s0, float& s1) {
  p0 = r == 0 ? 0 : 1;
  p1 = r == 3 ? 3 : 2;
  s0 = r == 2 ? -1.f : 1.f;
  s1 = (r == 0 || r == 3) ? -1.f : 1.f;
}

// NT = 256 (4 waves) or 512 (8 waves: the 128 x 256 tile for Cout >= 256, which loads each
// tile's transformed input once for 256 output channels instead of twice for 2 x 128 --
// the A operand is most of this kernel's L2 traffic)
template <int BM, int BN, int WM, int WN, int BK, int NT = 256>
__global__ __launch_bounds__(NT) void wino_gemm_kernel(WinoArgs a) {
  constexpr int LDSR = BK + 4;
  constexpr int KQ = BK / 4;
  constexpr int A_VEC = BM * KQ, B_VEC = BN * KQ;
  constexpr int A_PER = (A_VEC + NT - 1) / NT;
  constexpr int B_PER = (B_VEC + NT - 1) / NT;
  constexpr int MI = WM / 32, NI = WN / 32;
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == NT / 64, "one wave per WM x WN sub-tile");
  static_assert(NT % KQ == 0, "uniform kq per thread");

  __shared__ __attribute__((aligned(16))) float As[BM * LDSR];
  __shared__ __attribute__((aligned(16))) float Bs[BN * LDSR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  const int tiles_n = (a.Cout + BN - 1) / BN;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tn = lid % tiles_n, tm = lid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int xi = blockIdx.z;
  int pa0, pa1, pb0, pb1;
  float sa0, sa1, sb0, sb1;
  bt_row(xi >> 2, pa0, pa1, sa0, sa1);
  bt_row(xi & 3, pb0, pb1, sb0, sb1);
  const float s00 = sa0 * sb0, s01 = sa0 * sb1, s10 = sa1 * sb0, s11 = sa1 * sb1;

  // A slots: tile fixed across the K loop; 4 pixel offsets (zero page when padded)
  const int kq4 = (tid % KQ) * 4;
  long off[A_PER][4];
  unsigned okm[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int idx = tid + i * NT;
    const int t = m0 + idx / KQ;
    const bool ok = idx < A_VEC && t < a.T;
    const int tt = ok ? t : 0;
    const int n = tt / (a.th * a.tw), r = tt - n * a.th * a.tw;
    const int ty = r / a.tw, tx = r - ty * a.tw;
    const int h0 = 2 * ty - 1, w0 = 2 * tx - 1;
    const int hh[2] = {h0 + pa0, h0 + pa1}, ww[2] = {w0 + pb0, w0 + pb1};
    unsigned m = 0;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const bool in = ok && (unsigned)hh[u] < (unsigned)a.H && (unsigned)ww[v] < (unsigned)a.W;
        off[i][u * 2 + v] = in ? (((long)n * a.H + hh[u]) * a.W + ww[v]) * a.ldin : 0;
        m |= (in ? 1u : 0u) << (u * 2 + v);
      }
    okm[i] = m;
  }
  const float* wk = a.wk + (long)xi * a.Cout * a.ldk;
  long boff[B_PER];
  bool bok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int idx = tid + i * NT;
    const int co = n0 + idx / KQ;
    bok[i] = idx < B_VEC && co < a.Cout;
    boff[i] = (long)(bok[i] ? co : 0) * a.ldk + kq4;
  }

  f32x4 ra[A_PER][4], rb[B_PER];
  auto load = [&](int k0) {
    const bool kin = k0 + kq4 < a.Cin;
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = kin && ((okm[i] >> q) & 1u);
        ra[i][q] = ld4(ok ? a.in + off[i][q] + k0 + kq4 : g_wzero4);
      }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) rb[i] = ld4(bok[i] && kin ? wk + boff[i] + k0 : g_wzero4);
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * NT;
      if (A_VEC % NT == 0 || idx < A_VEC) {
        const f32x4 v = (s00 * ra[i][0] + s01 * ra[i][1]) + (s10 * ra[i][2] + s11 * ra[i][3]);
        st4(&As[(idx / KQ) * LDSR + (idx % KQ) * 4], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      if (B_VEC % NT == 0 || idx < B_VEC) st4(&Bs[(idx / KQ) * LDSR + (idx % KQ) * 4], rb[i]);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int lrow = lane & 31, lk = (lane >> 5) * 4;
  const int nk = (a.Cin + BK - 1) / BK;
  load(0);
  for (int kt = 0; kt < nk; ++kt) {
    store();
    __syncthreads();
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 8; ++ks) {
      f32x4 af[MI], bf[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) af[mi] = ld4(&As[(wm0 + mi * 32 + lrow) * LDSR + ks * 8 + lk]);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) bf[ni] = ld4(&Bs[(wn0 + ni * 32 + lrow) * LDSR + ks * 8 + lk]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][kk], bf[ni][kk], acc[mi][ni], 0, 0, 0);
    }
    __syncthreads();
  }

  // raw M_xi rows (C layout of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
  float* M = a.m + (long)xi * a.T * a.Cout;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + lrow;
    if (col >= a.Cout) continue;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < a.T) M[(long)row * a.Cout + col] = acc[mi][ni][r];
      }
  }
}

// Y = A^T M A per tile and float4 channel group (+ bias, + addend), NHWC out; with
// `stat`, the BatchNorm partials of each 16*QT-tile (64*QT-pixel) block: per channel the
// block sum and the sum of squared deviations from the block mean, exactly the
// [row tile][2][Cout] layout of seg_conv_igemm's epilogue (tile_rows = seg_conv_wino_tile_rows()).
// Block = 256 threads = 16 tile lanes x 16 channel-group lanes (256 contiguous
// bytes of an M row per load); each tile lane owns QT tiles (tl + 16 q); blockIdx.y
// picks the block's 64 channels (the deep layers have only T / 64 = 16..256 tile blocks).
__global__ __launch_bounds__(256) void wino_out_kernel(const float* __restrict__ m, int T, int Cout, int N, int H,
                                                       int W, int th, int tw, const float* __restrict__ bias,
                                                       const float* __restrict__ add, long ldadd,
                                                       float* __restrict__ out, long ldout, float* __restrict__ stat) {
  __shared__ f32x4 red[4][16];  // [wave][cg lane]
  __shared__ f32x4 bmean[16];
  const int t = threadIdx.x, tl = t >> 4, cl = t & 15, wave = t >> 6;
  constexpr int QT = kWinoQT, TPB = 16 * QT;
  long pix[QT][4];
  bool tok[QT];
  int tile[QT];
#pragma unroll
  for (int q = 0; q < QT; ++q) {
    tile[q] = blockIdx.x * TPB + tl + 16 * q;
    tok[q] = tile[q] < T;
    const int tt = tok[q] ? tile[q] : 0;
    const int n = tt / (th * tw), r = tt - n * th * tw;
    const int ty = r / tw, tx = r - ty * tw;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v = 0; v < 2; ++v) pix[q][u * 2 + v] = ((long)n * H + 2 * ty + u) * W + 2 * tx + v;
  }
  const int ntile = min(TPB, T - (int)blockIdx.x * TPB);
  const float cnt = 4.f * (float)ntile;
  const long TC = (long)T * Cout;
#if SEG_WINO_OUT_CSPLIT
  {
    const int cgb = blockIdx.y * 64;
#else
  for (int cgb = 0; cgb < Cout; cgb += 64) {
#endif
    const int c = cgb + cl * 4;
    const bool cok = c < Cout;
    const f32x4 b = (bias && cok) ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 y[QT][4];
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      if (tok[q] && cok) {
        f32x4 qv[16];
#pragma unroll
        for (int x = 0; x < 16; ++x) qv[x] = ld4(m + x * TC + (long)tile[q] * Cout + c);
        // rows of A^T M: R0[j] = q0j + q1j + q2j, R1[j] = q1j - q2j - q3j
        f32x4 r0[4], r1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          r0[j] = qv[j] + qv[4 + j] + qv[8 + j];
          r1[j] = qv[4 + j] - qv[8 + j] - qv[12 + j];
        }
        y[q][0] = r0[0] + r0[1] + r0[2] + b;
        y[q][1] = r0[1] - r0[2] - r0[3] + b;
        y[q][2] = r1[0] + r1[1] + r1[2] + b;
        y[q][3] = r1[1] - r1[2] - r1[3] + b;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          if (add) y[q][p] += ld4(add + pix[q][p] * ldadd + c);
          st4(out + pix[q][p] * ldout + c, y[q][p]);
        }
      } else {
#pragma unroll
        for (int p = 0; p < 4; ++p) y[q][p] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#if SEG_WINO_OUT_CSPLIT
    if (!stat) return;
#else
    if (!stat) continue;
#endif
    // pass 1: block sum -> mean; pass 2: sum of squared deviations about it
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f};
      const f32x4 mu = pass ? bmean[cl] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < QT; ++q)
        if (tok[q] && cok) {
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x4 d = y[q][p] - mu;
            s += pass ? d * d : d;
          }
        }
#pragma unroll
      for (int o = 16; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[j] += __shfl_xor(s[j], o, 64);
      if ((t & 63) < 16) red[wave][cl] = s;
      __syncthreads();
      if (t < 16) {
        const f32x4 tot = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        const int cc = cgb + t * 4;
        if (pass == 0) bmean[t] = tot / cnt;
        if (cc < Cout) {
          float* dst = stat + ((long)blockIdx.x * 2 + pass) * Cout + cc;
#pragma unroll
          for (int j = 0; j < 4; ++j) dst[j] = tot[j];
        }
      }
      __syncthreads();
    }
  }
}

template <int BM, int BN, int WM, int WN, int NT = 256>
void launch_wino(const WinoArgs& a, hipStream_t s) {
  dim3 grid(seg_cdiv(a.T, BM) * seg_cdiv(a.Cout, BN), 1, 16);
  hipLaunchKernelGGL((wino_gemm_kernel<BM, BN, WM, WN, 32, NT>), grid, dim3(NT), 0, s, a);
}
#ifndef SEG_WINO_WIDE_MINBLK
#define SEG_WINO_WIDE_MINBLK 0  // ... and only when it still launches this many blocks
#endif
#ifndef SEG_WINO_WIDE
#define SEG_WINO_WIDE 256  // Cout from which the 8-wave 128 x 256 tile is used
#endif

// ---------------------------------------------------------------- fused forward / data gradient
// The 16 GEMMs and the output transform in one kernel, M never leaving the registers.  A wave owns 32 tiles x 32
// output channels for ALL 16 xi: 16 independent 32x32 accumulators (256 accumulator registers; gfx950's unified
// file holds them beside ~200 VGPRs at one wave per SIMD), so back-to-back MFMAs never wait on each other.  Per
// K chunk of 8 input channels a lane loads its tile's 4x4 input patch for 4 channels (16 float4; lane half h holds
// channels 4h..4h+3 and K step s uses channel 4h+s on both operands), forms V = B^T d B in place (adds only, all 16
// xi at once: 4 loads per input pixel instead of the per-xi loader's 16) and runs 4 x 16 MFMAs against U rows
// staged in LDS (shared by the block's 4 waves, double-buffered, one barrier per chunk), while the next chunk's
// patch and U rows are in flight.  Epilogue per accumulator element: Y = A^T M A from the 16 values of one lane
// (+ bias, + addend), and the same BatchNorm partials as wino_out_kernel (64-tile row tiles, two passes: sum, then
// squared deviations about the row tile's mean).  Block = 128 tiles x 32 channels (WT = 4 waves along the tiles).
struct WinoFusedArgs {
  const float* in; long ldin;   // NHWC conv input [N*H*W][ldin]
  const float* wk; int ldk;     // U [16][Cout][ldk] (seg_pack_batch modes 3 / 4)
  const float* bias;            // [Cout] or null
  const float* add; long ldadd; // optional addend (may alias out)
  float* out; long ldout;
  float* stat;                  // optional BN partials [row tiles of 64 tiles][2][Cout]
  int N, H, W, Cin, Cout;
  int T, th, tw;
  long in_elems;                // extent of `in` (elements)
  unsigned wk_bytes;            // extent of `wk` (buffer-load range check: < 2^31)
};

#ifndef SEG_WF_EXP
#define SEG_WF_EXP 0  // timing experiments: 1 = no loads in the K loop, 2 = no input transform, 4 = no MFMAs
#endif
constexpr int kFusedKC = 8;             // input channels per K chunk
constexpr int kFusedUR = kFusedKC + 4;  // LDS pitch (floats) of one (xi, co) row of U
constexpr unsigned kFusedOOB = 0x80000000u;  // a buffer offset past every range check: the load returns zeros

__device__ __forceinline__ __amdgpu_buffer_rsrc_t seg_rsrc(const void* p, unsigned bytes) {
  const unsigned long v = (unsigned long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ f32x4 seg_bld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <int WT>
__global__ __launch_bounds__(256) void wino_fused_kernel(WinoFusedArgs a) {
  constexpr int WN = 4 / WT, BT = 32 * WT, BC = 32 * WN;
  static_assert(WT == 2 || WT == 4, "a BN row tile (64 tiles) lies in one block");
  // the BN partials below use 64-tile row tiles; the engine sizes / finalizes them with seg_conv_wino_row_tiles /
  // seg_conv_wino_tile_rows, which derive from SEG_WINO_OUT_QT (16 * QT tiles) -- the two must agree
  static_assert(16 * kWinoQT == 64, "wino_fused_kernel's BN row tile is 64 Winograd tiles");
  constexpr int USZ = 16 * BC * kFusedUR;
  constexpr int UPT = 16 * BC * (kFusedKC / 4) / 256;  // U float4 slots per thread per chunk
  __shared__ __attribute__((aligned(16))) float Us[2 * USZ];
  __shared__ float red[4][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wt = wave / WN, wn = wave % WN;
  const int row = lane & 31, h = lane >> 5;
  const int tiles_n = (a.Cout + BC - 1) / BC;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tn = lid % tiles_n, tm = lid / tiles_n;
  const int m0 = tm * BT, n0 = tn * BC;
  // input descriptor based at the image of the block's first tile (32-bit offsets cover the images the block
  // touches: seg_conv_wino_fused checks their extent), U descriptor over the whole pack
  const int nfirst = m0 / (a.th * a.tw);
  const long boff = (long)nfirst * a.H * a.W * a.ldin;
  const __amdgpu_buffer_rsrc_t rin = seg_rsrc(a.in + boff, (unsigned)min((a.in_elems - boff) * 4, (long)kFusedOOB - 16));
  const __amdgpu_buffer_rsrc_t rwk = seg_rsrc(a.wk, a.wk_bytes);

  // this lane's tile (A row `row` of the wave's 32): byte offset of its 4x4 patch's corner (32-bit wrap arithmetic:
  // exact wherever a patch pixel is in the image) and the in-image mask
  const int t = m0 + wt * 32 + row;
  const bool tok = t < a.T;
  unsigned pm = 0, pbase = 0;
  int opix = 0;  // pixel index of the tile's top-left output (the epilogue fetches it from the owning lane)
  {
    const int tt = tok ? t : 0;
    const int n = tt / (a.th * a.tw), r = tt - n * a.th * a.tw;
    const int ty = r / a.tw, tx = r - ty * a.tw;
    const int h0 = 2 * ty - 1, w0 = 2 * tx - 1;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (tok && (unsigned)(h0 + p) < (unsigned)a.H && (unsigned)(w0 + q) < (unsigned)a.W) pm |= 1u << (p * 4 + q);
    pbase = (unsigned)((((long)(n - nfirst) * a.H + h0) * a.W + w0) * a.ldin * 4) + 16u * h;
    opix = (n * a.H + 2 * ty) * a.W + 2 * tx;
  }
  const unsigned rstep = (unsigned)(a.W * a.ldin * 4), cstep = (unsigned)(a.ldin * 4);

  auto load_patch = [&](int c0, f32x4 (&d)[16]) {
    const bool cok = c0 + 4 * h < a.Cin;
    const unsigned b = pbase + 4u * c0;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = cok && ((pm >> (p * 4 + q)) & 1u);
        d[p * 4 + q] = seg_bld4(rin, ok ? b + p * rstep + q * cstep : kFusedOOB);
      }
  };
  auto load_u = [&](int c0, f32x4 (&u)[UPT]) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int idx = tid + i * 256;
      const int xi = idx / (2 * BC), rem = idx - xi * (2 * BC);
      const int co = n0 + (rem >> 1), c = c0 + 4 * (rem & 1);
      const bool ok = co < a.Cout && c < a.Cin;
      u[i] = seg_bld4(rwk, ok ? (unsigned)((((long)xi * a.Cout + co) * a.ldk + c) * 4) : kFusedOOB);
    }
  };
  auto store_u = [&](float* dst, const f32x4 (&u)[UPT]) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int idx = tid + i * 256;
      const int xi = idx / (2 * BC), rem = idx - xi * (2 * BC);
      st4(dst + (xi * BC + (rem >> 1)) * kFusedUR + 4 * (rem & 1), u[i]);
    }
  };
  // V = B^T d B in place: d[4p + q] (patch row p, column q) -> V[4r + c] = V_xi, xi = 4r + c
  auto transform = [](f32x4 (&d)[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 d0 = d[q], d1 = d[4 + q], d2 = d[8 + q], d3 = d[12 + q];
      d[q] = d0 - d2;
      d[4 + q] = d1 + d2;
      d[8 + q] = d2 - d1;
      d[12 + q] = d1 - d3;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const f32x4 t0 = d[4 * r], t1 = d[4 * r + 1], t2 = d[4 * r + 2], t3 = d[4 * r + 3];
      d[4 * r] = t0 - t2;
      d[4 * r + 1] = t1 + t2;
      d[4 * r + 2] = t2 - t1;
      d[4 * r + 3] = t1 - t3;
    }
  };

  f32x16 acc[16];
#pragma unroll
  for (int x = 0; x < 16; ++x)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[x][r] = 0.f;

  const int nk = (a.Cin + kFusedKC - 1) / kFusedKC;
  const int urow = (wn * 32 + row) * kFusedUR + 4 * h;
  f32x4 d[16], ug[UPT];
  load_patch(0, d);
  load_u(0, ug);
  store_u(Us, ug);
  __syncthreads();
  // per K chunk: the next chunk's patch and U rows are issued first, then this chunk's transform and 64 MFMAs (U rows
  // read from LDS four xi ahead), then the U rows are staged and the patch moves over
  for (int kc = 0; kc < nk; ++kc) {
    const bool more = kc + 1 < nk;
    f32x4 dn[16];
    if (more && !(SEG_WF_EXP & 1)) {
      load_patch((kc + 1) * kFusedKC, dn);
      load_u((kc + 1) * kFusedKC, ug);
    }
    if (SEG_WF_EXP & 1) {
#pragma unroll
      for (int q = 0; q < 16; ++q) dn[q] = d[q] * 0.5f;
    }
    if (!(SEG_WF_EXP & 2)) transform(d);
    const float* ub = Us + (kc & 1) * USZ + urow;
    f32x4 u[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) u[0][j] = ld4(ub + j * BC * kFusedUR);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g < 3) {
#pragma unroll
        for (int j = 0; j < 4; ++j) u[(g + 1) & 1][j] = ld4(ub + (4 * (g + 1) + j) * BC * kFusedUR);
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (SEG_WF_EXP & 4)
            acc[4 * g + j][s2] += d[4 * g + j][s2] * u[g & 1][j][s2];
          else
            acc[4 * g + j] = __builtin_amdgcn_mfma_f32_32x32x2f32(d[4 * g + j][s2], u[g & 1][j][s2], acc[4 * g + j],
                                                                  0, 0, 0);
    }
    if (more) {
      store_u(Us + ((kc + 1) & 1) * USZ, ug);
#pragma unroll
      for (int q = 0; q < 16; ++q) d[q] = dn[q];
    }
    __syncthreads();
  }

  // epilogue: accumulator element r holds tile row (r&3) + 8(r>>2) + 4h of the wave, column lane&31
  const int col = n0 + wn * 32 + row;
  const bool cok = col < a.Cout;
  const float b = (a.bias && cok) ? a.bias[col] : 0.f;
  auto tile_y = [&](int r, float (&y)[4]) {
    float q[16];
#pragma unroll
    for (int x = 0; x < 16; ++x) q[x] = acc[x][r];
    float r0[4], r1[4];  // rows of A^T M
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r0[j] = q[j] + q[4 + j] + q[8 + j];
      r1[j] = q[4 + j] - q[8 + j] - q[12 + j];
    }
    y[0] = r0[0] + r0[1] + r0[2] + b;
    y[1] = r0[1] - r0[2] - r0[3] + b;
    y[2] = r1[0] + r1[1] + r1[2] + b;
    y[3] = r1[1] - r1[2] - r1[3] + b;
  };
  const int wbase = m0 + wt * 32 + 4 * h;
  float ssum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tt = wbase + (r & 3) + 8 * (r >> 2);
    const long p0 = __shfl(opix, (r & 3) + 8 * (r >> 2) + 4 * h, 64);  // all lanes active (bpermute)
    if (tt < a.T && cok) {
      float y[4];
      tile_y(r, y);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long pix = p0 + (u >> 1) * a.W + (u & 1);
        if (a.add) y[u] += a.add[pix * a.ldadd + col];
        a.out[pix * a.ldout + col] = y[u];
        ssum += y[u];
      }
    }
  }
  if (!a.stat) return;
  // BN partials of the wave pair (wt even, wt odd) that holds one 64-tile row tile
  const int rtile = (m0 + (wt & ~1) * 32) / 64;
  const int ntile = min(64, a.T - rtile * 64);
  const int we = (wt & ~1) * WN + wn, wo = we + WN;
  float mean = 0.f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    float sv = ssum;
    if (pass) {
      sv = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tt = wbase + (r & 3) + 8 * (r >> 2);
        if (tt < a.T && cok) {
          float y[4];
          tile_y(r, y);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float dv = y[u] - mean;
            sv += dv * dv;
          }
        }
      }
    }
    sv += __shfl_xor(sv, 32, 64);
    if (h == 0) red[wave][row] = sv;
    __syncthreads();
    const float tot = red[we][row] + red[wo][row];
    if (pass == 0) mean = ntile > 0 ? tot / (4.f * (float)ntile) : 0.f;
    if ((wt & 1) == 0 && h == 0 && cok && ntile > 0) a.stat[((long)rtile * 2 + pass) * a.Cout + col] = tot;
    __syncthreads();
  }
}

#ifdef SEG_WF2_TEST
// TEST-ONLY (never in the product library): round 5's two-waves-per-SIMD fused form, restored from commit 152956a to
// find the cause of its UNet-slice parity failure (tools/wf2diag.py).  Built into a variant by
// tools/variant.py wf2 -DSEG_WF2_TEST=1; seg_wf2_mask selects which seg_conv_wino_fused calls take it.
// Two waves per SIMD instead of one: a wave owns 16 tiles x 32 channels for all 16 xi on v_mfma_f32_16x16x4_f32
// (16 xi x 2 column halves x f32x4 = 128 accumulator registers; ~200 registers in all), so a second block shares
// every SIMD and covers the patch loads' latency that the one-wave form exposes (its timing experiments: loads =
// 37 % of the launch).  K chunk = 8 input channels: lane group g = lane >> 4 holds channels 2g, 2g + 1 (float2 per
// patch pixel) and K step s uses channel 2g + s on both operands.  Block = 64 tiles (one BN row tile) x 32 channels.
constexpr int kF2KC = 8, kF2UR = 10;  // channels per chunk; LDS pitch (floats) of a (xi, co) row of U
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 seg_bld2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

__global__ __launch_bounds__(256, 2) void wino_fused2_kernel(WinoFusedArgs a) {
  constexpr int BT = 64, BC = 32;
  constexpr int USZ = 16 * BC * kF2UR;
  constexpr int UPT = 16 * BC * (kF2KC / 4) / 256;  // U float4 slots per thread per chunk (4)
  __shared__ __attribute__((aligned(16))) float Us[2 * USZ];
  __shared__ float red[4][32];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int tiles_n = (a.Cout + BC - 1) / BC;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tn = lid % tiles_n, tm = lid / tiles_n;
  const int m0 = tm * BT, n0 = tn * BC;
  const int nfirst = m0 / (a.th * a.tw);
  const long boff = (long)nfirst * a.H * a.W * a.ldin;
  const __amdgpu_buffer_rsrc_t rin = seg_rsrc(a.in + boff, (unsigned)min((a.in_elems - boff) * 4, (long)kFusedOOB - 16));
  const __amdgpu_buffer_rsrc_t rwk = seg_rsrc(a.wk, a.wk_bytes);

  // this lane's tile (A row i16 of the wave's 16) and its patch
  const int t = m0 + wave * 16 + i16;
  const bool tok = t < a.T;
  unsigned pm = 0, pbase = 0;
  int opix = 0;
  {
    const int tt = tok ? t : 0;
    const int n = tt / (a.th * a.tw), r = tt - n * a.th * a.tw;
    const int ty = r / a.tw, tx = r - ty * a.tw;
    const int h0 = 2 * ty - 1, w0 = 2 * tx - 1;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (tok && (unsigned)(h0 + p) < (unsigned)a.H && (unsigned)(w0 + q) < (unsigned)a.W) pm |= 1u << (p * 4 + q);
    pbase = (unsigned)((((long)(n - nfirst) * a.H + h0) * a.W + w0) * a.ldin * 4) + 8u * g;
    opix = (n * a.H + 2 * ty) * a.W + 2 * tx;
  }
  const unsigned rstep = (unsigned)(a.W * a.ldin * 4), cstep = (unsigned)(a.ldin * 4);

  auto load_patch = [&](int c0, f32x2 (&d)[16]) {
    const bool cok = c0 + 2 * g < a.Cin;  // Cin % 4 == 0: both channels or neither
    const unsigned b = pbase + 4u * c0;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = cok && ((pm >> (p * 4 + q)) & 1u);
        d[p * 4 + q] = seg_bld2(rin, ok ? b + p * rstep + q * cstep : kFusedOOB);
      }
  };
  auto load_u = [&](int c0, f32x4 (&u)[UPT]) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int idx = tid + i * 256;
      const int xi = idx / (2 * BC), rem = idx - xi * (2 * BC);
      const int co = n0 + (rem >> 1), c = c0 + 4 * (rem & 1);
      const bool ok = co < a.Cout && c < a.Cin;
      u[i] = seg_bld4(rwk, ok ? (unsigned)((((long)xi * a.Cout + co) * a.ldk + c) * 4) : kFusedOOB);
    }
  };
  auto store_u = [&](float* dst, const f32x4 (&u)[UPT]) {
#pragma unroll
    for (int i = 0; i < UPT; ++i) {
      const int idx = tid + i * 256;
      const int xi = idx / (2 * BC), rem = idx - xi * (2 * BC);
      float* q = dst + (xi * BC + (rem >> 1)) * kF2UR + 4 * (rem & 1);
      *reinterpret_cast<f32x2*>(q) = f32x2{u[i][0], u[i][1]};
      *reinterpret_cast<f32x2*>(q + 2) = f32x2{u[i][2], u[i][3]};
    }
  };
  auto transform = [](f32x2 (&d)[16]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x2 d0 = d[q], d1 = d[4 + q], d2 = d[8 + q], d3 = d[12 + q];
      d[q] = d0 - d2;
      d[4 + q] = d1 + d2;
      d[8 + q] = d2 - d1;
      d[12 + q] = d1 - d3;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const f32x2 t0 = d[4 * r], t1 = d[4 * r + 1], t2 = d[4 * r + 2], t3 = d[4 * r + 3];
      d[4 * r] = t0 - t2;
      d[4 * r + 1] = t1 + t2;
      d[4 * r + 2] = t2 - t1;
      d[4 * r + 3] = t1 - t3;
    }
  };

  f32x4 acc[16][2];
#pragma unroll
  for (int x = 0; x < 16; ++x) acc[x][0] = acc[x][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (a.Cin + kF2KC - 1) / kF2KC;
  f32x4 ug[UPT];
  load_u(0, ug);
  store_u(Us, ug);
  __syncthreads();
  const int urow = i16 * kF2UR + 2 * g;
  for (int kc = 0; kc < nk; ++kc) {
    const bool more = kc + 1 < nk;
    f32x2 d[16];
    load_patch(kc * kF2KC, d);
    if (more) load_u((kc + 1) * kF2KC, ug);
    transform(d);
    const float* ub = Us + (kc & 1) * USZ + urow;
#pragma unroll
    for (int x = 0; x < 16; ++x) {
      const f32x2 u0 = *reinterpret_cast<const f32x2*>(ub + (x * BC) * kF2UR);
      const f32x2 u1 = *reinterpret_cast<const f32x2*>(ub + (x * BC + 16) * kF2UR);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        acc[x][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(d[x][s2], u0[s2], acc[x][0], 0, 0, 0);
        acc[x][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(d[x][s2], u1[s2], acc[x][1], 0, 0, 0);
      }
    }
    if (more) store_u(Us + ((kc + 1) & 1) * USZ, ug);
    __syncthreads();
  }

  // epilogue: acc[xi][half][r] = M_xi of tile (wave's row 4g + r), channel n0 + 16 half + (lane & 15)
  auto tile_y = [&](int hf, int r, float (&y)[4]) {
    float q[16];
#pragma unroll
    for (int x = 0; x < 16; ++x) q[x] = acc[x][hf][r];
    float r0[4], r1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r0[j] = q[j] + q[4 + j] + q[8 + j];
      r1[j] = q[4 + j] - q[8 + j] - q[12 + j];
    }
    y[0] = r0[0] + r0[1] + r0[2];
    y[1] = r0[1] - r0[2] - r0[3];
    y[2] = r1[0] + r1[1] + r1[2];
    y[3] = r1[1] - r1[2] - r1[3];
  };
  long p0s[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) p0s[r] = __shfl(opix, 4 * g + r, 64);  // all lanes active (bpermute)
  const int wbase = m0 + wave * 16 + 4 * g;
  float ssum[2] = {0.f, 0.f};
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const int col = n0 + 16 * hf + i16;
    if (col >= a.Cout) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (wbase + r >= a.T) continue;
      float y[4];
      tile_y(hf, r, y);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long pix = p0s[r] + (u >> 1) * a.W + (u & 1);
        float v = y[u] + b;
        if (a.add) v += a.add[pix * a.ldadd + col];
        a.out[pix * a.ldout + col] = v;
        ssum[hf] += v;
      }
    }
  }
  if (!a.stat) return;
  // BN partials of the block's 64-tile row tile: lanes of one column (4 lane groups), then the 4 waves
  const int rtile = m0 / 64, ntile = min(64, a.T - m0);
  float mean[2] = {0.f, 0.f};
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int col = n0 + 16 * hf + i16;
      float sv = ssum[hf];
      if (pass) {
        sv = 0.f;
        if (col < a.Cout) {
          const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (wbase + r >= a.T) continue;
            float y[4];
            tile_y(hf, r, y);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              float v = y[u] + b;
              if (a.add) v += a.add[(p0s[r] + (u >> 1) * a.W + (u & 1)) * a.ldadd + col];
              const float dv = v - mean[hf];
              sv += dv * dv;
            }
          }
        }
      }
      sv += __shfl_xor(sv, 16, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (g == 0) red[wave][16 * hf + i16] = sv;
    }
    __syncthreads();
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int c = 16 * hf + i16, col = n0 + c;
      const float tot = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
      if (pass == 0) mean[hf] = ntile > 0 ? tot / (4.f * (float)ntile) : 0.f;
      if (wave == 0 && g == 0 && col < a.Cout && ntile > 0) a.stat[((long)rtile * 2 + pass) * a.Cout + col] = tot;
    }
    __syncthreads();
  }
}

#endif  // SEG_WF2_TEST

// ---------------------------------------------------------------- weight gradient
// dW = G^T [ sum_t (A dY_t A^T) .* (B^T X_t B) ] G  per (co, ci): Winograd F(3x3, 2x2)
// (the transposition of F(2x2,3x3); A = [1 0; 1 1; 1 -1; 0 -1]).  Per xi a GEMM
//   P_xi[co][ci] = sum_t DY_xi[t][co] * XV_xi[t][ci]
// with K = 2x2 output tiles, split over gridDim.y into fixed-order partial slabs
// [split][16][Cout][Cin] (no float atomics); wino_wgrad_reduce_kernel sums the
// slabs and applies G^T . G.  Operands are staged k-major ([tile][channel], the
// natural NHWC order) like wgrad.hip's kernel; each loaded float4 is the signed
// sum of the tile's 4 dY pixels (A side) or 4 X pixels (B side, zero padding).
struct WinoWgradArgs {
  const float* dy; long lddy;
  const float* x; long ldx;
  float* part;
  int N, H, W, Cin, Cout;  // H, W: spatial size of dY and X (stride 1, pad 1)
  int T, th, tw, kchunk;
};

__device__ __forceinline__ float arow(int i, int a) {  // A = [1 0; 1 1; 1 -1; 0 -1]
  return a == 0 ? (i == 3 ? 0.f : 1.f) : (i == 0 ? 0.f : (i == 2 || i == 3 ? -1.f : 1.f));
}

constexpr int WBK = 16;

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void wino_wgrad_kernel(WinoWgradArgs a) {
  constexpr int AR = BM + 4, BR = BN + 4;
  constexpr int A_VEC = WBK * BM / 4, B_VEC = WBK * BN / 4;
  constexpr int A_PER = (A_VEC + 255) / 256, B_PER = (B_VEC + 255) / 256;
  constexpr int MI = WM / 32, NI = WN / 32, WAVES_N = BN / WN;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves per block");

  __shared__ __attribute__((aligned(16))) float As[WBK * AR];
  __shared__ __attribute__((aligned(16))) float Bs[WBK * BR];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  const int tiles_n = (a.Cin + BN - 1) / BN;
  const int tiles = tiles_n * ((a.Cout + BM - 1) / BM);
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int split = lid / tiles, tile = lid - split * tiles;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int xi = blockIdx.z, xr = xi >> 2, xc = xi & 3;
  const int kbeg = split * a.kchunk;
  const int kend = min(a.T, kbeg + a.kchunk);
  // A side coefficients (dY 2x2 -> 4x4), B side pixel subset and signs (X 4x4 -> 4x4)
  const float c00 = arow(xr, 0) * arow(xc, 0), c01 = arow(xr, 0) * arow(xc, 1);
  const float c10 = arow(xr, 1) * arow(xc, 0), c11 = arow(xr, 1) * arow(xc, 1);
  int pa0, pa1, pb0, pb1;
  float sa0, sa1, sb0, sb1;
  bt_row(xr, pa0, pa1, sa0, sa1);
  bt_row(xc, pb0, pb1, sb0, sb1);
  const float s00 = sa0 * sb0, s01 = sa0 * sb1, s10 = sa1 * sb0, s11 = sa1 * sb1;

  f32x4 ra[A_PER][4], rb[B_PER][4];
  auto tile_pos = [&](int t, int& n, int& ty, int& tx) {
    n = t / (a.th * a.tw);
    const int r = t - n * a.th * a.tw;
    ty = r / a.tw;
    tx = r - ty * a.tw;
  };
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * 256;
      const int trow = idx / (BM / 4), c = co0 + (idx % (BM / 4)) * 4;
      const int t = k0 + trow;
      const bool ok = idx < A_VEC && t < kend && c < a.Cout;
      int n, ty, tx;
      tile_pos(ok ? t : 0, n, ty, tx);
      const long p0 = ((long)n * a.H + 2 * ty) * a.W + 2 * tx;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const long p = p0 + (q >> 1) * a.W + (q & 1);
        ra[i][q] = ld4(ok ? a.dy + p * a.lddy + c : g_wzero4);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * 256;
      const int trow = idx / (BN / 4), c = n0 + (idx % (BN / 4)) * 4;
      const int t = k0 + trow;
      const bool ok = idx < B_VEC && t < kend && c < a.Cin;
      int n, ty, tx;
      tile_pos(ok ? t : 0, n, ty, tx);
      const int hh[2] = {2 * ty - 1 + pa0, 2 * ty - 1 + pa1}, ww[2] = {2 * tx - 1 + pb0, 2 * tx - 1 + pb1};
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const bool in = ok && (unsigned)hh[u] < (unsigned)a.H && (unsigned)ww[v] < (unsigned)a.W;
          rb[i][u * 2 + v] = ld4(in ? a.x + (((long)n * a.H + hh[u]) * a.W + ww[v]) * a.ldx + c : g_wzero4);
        }
    }
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * 256;
      if (idx < A_VEC) {
        const f32x4 v = (c00 * ra[i][0] + c01 * ra[i][1]) + (c10 * ra[i][2] + c11 * ra[i][3]);
        st4(&As[(idx / (BM / 4)) * AR + (idx % (BM / 4)) * 4], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * 256;
      if (idx < B_VEC) {
        const f32x4 v = (s00 * rb[i][0] + s01 * rb[i][1]) + (s10 * rb[i][2] + s11 * rb[i][3]);
        st4(&Bs[(idx / (BN / 4)) * BR + (idx % (BN / 4)) * 4], v);
      }
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
  const int nk = (kend - kbeg + WBK - 1) / WBK;
  if (nk > 0) {
    load_tiles(kbeg);
    for (int kt = 0; kt < nk; ++kt) {
      store_tiles();
      __syncthreads();
      if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * WBK);
#pragma unroll
      for (int kk = 0; kk < WBK / 2; ++kk) {
        float af[MI], bf[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) af[mi] = As[(2 * kk + lh) * AR + wm0 + mi * 32 + lrow];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bf[ni] = Bs[(2 * kk + lh) * BR + wn0 + ni * 32 + lrow];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  float* slab = a.part + ((long)split * 16 + xi) * a.Cout * a.Cin;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + lrow;
    if (col >= a.Cin) continue;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = co0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.Cout) slab[(long)row * a.Cin + col] = acc[mi][ni][r];
      }
  }
}

// The same slabs from blocks that own all 16 transform points of a (Cout, Cin) tile: each K step loads a
// KT-tile strip once -- the 2x2 dY pixels of BM output channels and the 4x4 X pixels of BN input channels, one
// job (tile, 4-channel group) per thread -- forms its 16 transformed values with two butterfly passes, and wave w
// runs the GEMMs of points 4w..4w+3.  The per-point kernel above loads 4 dY and 4 X pixels per point, i.e. 128
// pixel-channel reads per tile against 20 here, which bound it at ~0.36 of the fp32 MFMA peak (its L2->CU operand
// traffic, 128 B/clk/CU at 128 x 128).  The butterflies keep that kernel's association (columns first, then rows;
// the +-1 coefficients are exact), and the K order and split boundaries are the same, so the slabs match it.
template <int BM, int BN, int KT>
__global__ __launch_bounds__(256) void wino_wgrad16_kernel(WinoWgradArgs a) {
  constexpr int AJ = KT * BM / 4, BJ = KT * BN / 4;
  constexpr int MI = BM / 32, NI = BN / 32;
  static_assert(AJ + BJ == 256 && KT % 2 == 0, "one load job per thread");
  static_assert(AJ % 64 == 0, "dY and X jobs on whole waves");

  __shared__ __attribute__((aligned(16))) float As[16 * KT * BM];
  __shared__ __attribute__((aligned(16))) float Bs[16 * KT * BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (a.Cin + BN - 1) / BN;
  const int tiles = tiles_n * ((a.Cout + BM - 1) / BM);
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int split = lid / tiles, tile = lid - split * tiles;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * a.kchunk;
  const int kend = min(a.T, kbeg + a.kchunk);

  // this thread's job: dY (2x2 pixels, 4 output channels) or X (4x4 pixels, 4 input channels) of one tile
  const bool is_a = tid < AJ;
  const int j = is_a ? tid : tid - AJ;
  const int cw = is_a ? BM / 4 : BN / 4;
  const int jt = j / cw, c = (is_a ? co0 : n0) + (j % cw) * 4;
  const bool cok = c < (is_a ? a.Cout : a.Cin);
  // Branch-free buffer loads from per-block bases (the first pixel row the split can read): a padding pixel, a
  // tile past the split or a channel past C gets an offset past the range check and loads zeros.  The host
  // checks that a split's pixel span fits the 31-bit offsets (else it runs the per-point kernel).
  const int tpi = a.th * a.tw;
  const int tb = min(kbeg, a.T - 1), nb = tb / tpi, tyb = (tb - nb * tpi) / a.tw;
  const long pbase = ((long)nb * a.H + max(2 * tyb - 1, 0)) * a.W;
  const long npix = (long)a.N * a.H * a.W;
  const __amdgpu_buffer_rsrc_t rx =
      seg_rsrc(a.x + pbase * a.ldx, (unsigned)min((npix - pbase) * a.ldx * 4, (long)kFusedOOB - 16));
  const __amdgpu_buffer_rsrc_t rdy =
      seg_rsrc(a.dy + pbase * a.lddy, (unsigned)min((npix - pbase) * a.lddy * 4, (long)kFusedOOB - 16));
  // this thread's tile, advanced by KT tiles per step without divisions
  int tcur = kbeg + jt, pn, tty, ttx;
  {
    const int tt = min(tcur, a.T - 1);
    pn = tt / tpi;
    const int rem = tt - pn * tpi;
    tty = rem / a.tw;
    ttx = rem - tty * a.tw;
  }
  auto advance = [&]() {
    tcur += KT;
    ttx += KT;
    while (ttx >= a.tw) {
      ttx -= a.tw;
      if (++tty == a.th) tty = 0, ++pn;
    }
  };
  f32x4 r[16];
  auto load = [&]() {
    const bool ok = cok && tcur < kend;
    if (is_a) {
      const int p0 = (int)(((long)pn * a.H + 2 * tty) * a.W + 2 * ttx - pbase);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        r[q] = seg_bld4(rdy, ok ? (unsigned)(((long)(p0 + (q >> 1) * a.W + (q & 1)) * a.lddy + c) * 4) : kFusedOOB);
    } else {  // all 16 offsets first, then the 16 loads back to back
      const unsigned cs = (unsigned)(a.ldx * 4);
      unsigned off[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int hh = 2 * tty - 1 + u;
        const bool rok = ok && (unsigned)hh < (unsigned)a.H;
        const unsigned rb = (unsigned)(((((long)pn * a.H + hh) * a.W + 2 * ttx - 1 - pbase) * a.ldx + c) * 4);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int ww = 2 * ttx - 1 + v;
          off[u * 4 + v] = rok && (unsigned)ww < (unsigned)a.W ? rb + v * cs : kFusedOOB;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) r[i] = seg_bld4(rx, off[i]);
    }
  };
  auto store = [&]() {
    if (is_a) {  // A dY A^T, A = [1 0; 1 1; 1 -1; 0 -1]: columns (xc) first, then rows (xr)
      f32x4 q[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        q[u][0] = r[2 * u];
        q[u][1] = r[2 * u] + r[2 * u + 1];
        q[u][2] = r[2 * u] - r[2 * u + 1];
        q[u][3] = -r[2 * u + 1];
      }
      float* dst = As + jt * BM + (j % cw) * 4;
#pragma unroll
      for (int xc = 0; xc < 4; ++xc) {
        st4(dst + (0 * 4 + xc) * KT * BM, q[0][xc]);
        st4(dst + (1 * 4 + xc) * KT * BM, q[0][xc] + q[1][xc]);
        st4(dst + (2 * 4 + xc) * KT * BM, q[0][xc] - q[1][xc]);
        st4(dst + (3 * 4 + xc) * KT * BM, -q[1][xc]);
      }
    } else {  // B^T X B, B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]: columns first, then rows
      f32x4 z[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        z[u][0] = r[u * 4 + 0] - r[u * 4 + 2];
        z[u][1] = r[u * 4 + 1] + r[u * 4 + 2];
        z[u][2] = -r[u * 4 + 1] + r[u * 4 + 2];
        z[u][3] = r[u * 4 + 1] - r[u * 4 + 3];
      }
      float* dst = Bs + jt * BN + (j % cw) * 4;
#pragma unroll
      for (int xc = 0; xc < 4; ++xc) {
        st4(dst + (0 * 4 + xc) * KT * BN, z[0][xc] - z[2][xc]);
        st4(dst + (1 * 4 + xc) * KT * BN, z[1][xc] + z[2][xc]);
        st4(dst + (2 * 4 + xc) * KT * BN, -z[1][xc] + z[2][xc]);
        st4(dst + (3 * 4 + xc) * KT * BN, z[1][xc] - z[3][xc]);
      }
    }
  };

  f32x16 acc[4][MI][NI];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[p][mi][ni][e] = 0.f;

  const int lrow = lane & 31, lh = lane >> 5;
  const int nk = (kend - kbeg + KT - 1) / KT;
  if (nk > 0) {
    load();
    for (int kt = 0; kt < nk; ++kt) {
      store();
      __syncthreads();
      if (kt + 1 < nk) {
        advance();
        load();
      }
#pragma unroll
      for (int kk = 0; kk < KT / 2; ++kk)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int xi = 4 * wave + p;
          float af[MI], bf[NI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) af[mi] = As[(xi * KT + 2 * kk + lh) * BM + mi * 32 + lrow];
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) bf[ni] = Bs[(xi * KT + 2 * kk + lh) * BN + ni * 32 + lrow];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
              acc[p][mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi], bf[ni], acc[p][mi][ni], 0, 0, 0);
        }
      __syncthreads();
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float* slab = a.part + ((long)split * 16 + 4 * wave + p) * a.Cout * a.Cin;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + ni * 32 + lrow;
      if (col >= a.Cin) continue;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = co0 + mi * 32 + (e & 3) + 8 * (e >> 2) + 4 * lh;
          if (row < a.Cout) slab[(long)row * a.Cin + col] = acc[p][mi][ni][e];
        }
    }
  }
}

// Sums each run of L consecutive slabs into the run's first slab, in slab order (float4 per thread, grid.y =
// runs): with hundreds of splits the reduce below would otherwise be a chain of hundreds of dependent
// iterations over only Cout x Cin threads (measured 0.4 us per split on MI355X, tools/ww16sweep.py).
__global__ __launch_bounds__(256) void wino_wgrad_fold_kernel(float* __restrict__ part, int splits, int L, long E4) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= E4) return;
  const int s0 = blockIdx.y * L, s1 = min(splits, s0 + L);
  f32x4* p = reinterpret_cast<f32x4*>(part) + e;
  f32x4 acc = p[(long)s0 * E4];
#pragma unroll 8
  for (int s = s0 + 1; s < s1; ++s) acc += p[(long)s * E4];
  p[(long)s0 * E4] = acc;
}

// dW[co][ci][3][3] (+)= G^T (sum_s P_s) G, one thread per (co, ci < Cin_real); the
// split sums run in fixed order (bitwise reproducible).
__global__ __launch_bounds__(256) void wino_wgrad_reduce_kernel(const float* __restrict__ part, int splits, int stride,
                                                                int Cout, int Cin_pad, int Cin, float* __restrict__ dw,
                                                                int accumulate) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)Cout * Cin) return;
  const int co = (int)(i / Cin), ci = (int)(i - (long)co * Cin);
  const long plane = (long)Cout * Cin_pad, off = (long)co * Cin_pad + ci;
  float m[16];
#pragma unroll
  for (int x = 0; x < 16; ++x) m[x] = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float* p = part + (long)s * stride * 16 * plane + off;
#pragma unroll
    for (int x = 0; x < 16; ++x) m[x] += p[x * plane];
  }
  float t[3][4];  // G^T m
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t[0][j] = m[j] + 0.5f * (m[4 + j] + m[8 + j]);
    t[1][j] = 0.5f * (m[4 + j] - m[8 + j]);
    t[2][j] = 0.5f * (m[4 + j] + m[8 + j]) + m[12 + j];
  }
  float* o = dw + i * 9;
#pragma unroll
  for (int y = 0; y < 3; ++y) {
    const float v[3] = {t[y][0] + 0.5f * (t[y][1] + t[y][2]), 0.5f * (t[y][1] - t[y][2]),
                        0.5f * (t[y][1] + t[y][2]) + t[y][3]};
#pragma unroll
    for (int x = 0; x < 3; ++x) o[y * 3 + x] = accumulate ? o[y * 3 + x] + v[x] : v[x];
  }
}

}  // namespace

// Use Winograd for this stride-1 pad-1 3x3 conv?  (1 = yes.)  The transforms
// cost a round trip of M (16 x tiles x Cout floats) through HBM whose share of
// the work falls as 1/Cin, and the 4-pixel input transform in the GEMM loader
// needs enough output columns to amortise, so Winograd wins for deep convs.
// Boundary measured on MI355X with tools/winobench.py (speedup over the direct
// implicit GEMM; MobileNetV2UNet decoder and UNet 512x1024 shapes):
//   Cin x Cout  1344x256 2.02 | 256x1344 1.30 | 256x256 1.37-1.50 | 288x128 1.52
//   512x128 1.44 | 128x256 1.28 | 128x128 1.11-1.24 | 128x288 1.00 | 128x512 1.10
//   256x64 1.04 | 152x64 0.91 | 64x152 0.62 | 64x64 0.70-0.79 | Cin or Cout 32/80 0.36-0.54
// Deterministic: the choice depends on the shape only.
// 2 = the fused kernel (seg_conv_wino_fused) where it beats the direct / LDS-halo kernels and the two-launch form
// does not apply (tools/winobench.py per launch, profiles/r05/winobench_*.txt): MobileNetV2UNet bs 32 up3.0 152 -> 64
// forward 332 vs 372 us (LDS-halo), its data gradient 64 -> 152 398 vs 421 us (direct); UNet 512x1024 bs 8 64 -> 128
// forward 1314 vs 1516 us, 64 -> 256 data gradient 2591 vs 2673 us.  Not taken: 64 -> 64, 128 -> 64 and 256 -> 64
// (the LDS-halo kernel is 2-5 % faster) and the 32 / 80-channel convs (halo / direct 3-9 % faster).  Between the two
// Winograd forms for Cin, Cout >= 128: the two-launch one up to Cout = 2 Cin and from Cout 512 (128 -> 512 2086 vs
// 2411 us fused), the fused one in between (128 -> 288: 355 vs 361 us, and no 600 MB M round trip).
#ifndef SEG_WINO_FUSED
#define SEG_WINO_FUSED 1
#endif
// The images one 128-tile block of wino_fused_kernel reads (its first tile's image and the ones after it) fit its
// 32-bit buffer offsets.
static bool fused_fits(int N, int H, int W, long ldin) {
  const long tiles = (long)(H / 2) * (W / 2);
  const long imgs = std::min<long>(N, tiles > 0 ? 128 / tiles + 2 : N);
  return imgs * H * W * ldin * 4 < (long)kFusedOOB - 16;
}
SEG_API int seg_conv_wino_pick(int N, int H, int W, int Cin, int Cout) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (Cout & 3) || N <= 0) return 0;
  if (Cin >= 256 && Cout >= 128) return 1;
  if (Cin >= 128 && Cout >= 128 && (Cout <= 2 * Cin || Cout >= 512)) return 1;
  const bool fits = fused_fits(N, H, W, Cin + 64);  // buffer-load range (row stride slack)
  return (SEG_WINO_FUSED && fits && Cin >= 64 && (Cout >= 128 || (Cout >= 64 && Cin > 128 && Cin < 256))) ? 2 : 0;
}

SEG_API int seg_conv_wino_fused_ok(int N, int H, int W, long ldin) {
  return ((H & 1) || (W & 1) || N <= 0) ? 0 : (int)fused_fits(N, H, W, ldin);
}

// Number of row tiles of seg_conv_wino's BN partials.
SEG_API int seg_conv_wino_row_tiles(int N, int H, int W) {
  const long T = (long)N * (H / 2) * (W / 2);
  return (int)((T + 16 * kWinoQT - 1) / (16 * kWinoQT));
}

// Pixels per BN row tile of seg_conv_wino (the tile_rows of seg_bn_stats_tiles).
SEG_API int seg_conv_wino_tile_rows(void) { return 64 * kWinoQT; }

// out = conv3x3(in, w) (+bias) (+add), stride 1, pad 1, by Winograd F(2x2,3x3).
// wk: U from seg_pack_batch mode 3 (forward) / 4 (data gradient): [16][Cout][ldk],
// ldk >= Cin.  work >= 16 * N*(H/2)*(W/2) * Cout floats.  stat (optional): BN
// partials [seg_conv_wino_row_tiles][2][Cout] with tile_rows = seg_conv_wino_tile_rows().
SEG_API int seg_conv_wino(const float* in, long ldin, int N, int H, int W, int Cin, const float* wk, int ldk,
                          const float* bias, float* out, long ldout, int Cout, const float* add, long ldadd,
                          float* stat, float* work, hipStream_t stream) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (ldin & 3) || (ldk & 3) || ldk < Cin || (Cout & 3) || (ldout & 3) ||
      (add && (ldadd & 3)) || !work)
    return (int)hipErrorInvalidValue;
  WinoArgs a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.m = work;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.th = H / 2; a.tw = W / 2; a.T = N * a.th * a.tw;
  if (a.T == 0) return 0;
  // the wide tile where it pads no more columns than two narrow ones (measured: Cout 256 -5..-6 %,
  // Cout 1344 (6 x 256 = 1536 vs 11 x 128 = 1408 columns) +4 % per launch)
  if (Cout >= SEG_WINO_WIDE && seg_cdiv(Cout, 256) * 2 == seg_cdiv(Cout, 128) &&
      (long)seg_cdiv(a.T, 128) * seg_cdiv(Cout, 256) * 16 >= SEG_WINO_WIDE_MINBLK)
    launch_wino<128, 256, 64, 64, 512>(a, stream);
  else if (Cout >= 128) launch_wino<128, 128, 64, 64>(a, stream);
  else launch_wino<128, 64, 64, 32>(a, stream);
  hipLaunchKernelGGL(wino_out_kernel, dim3(seg_cdiv(a.T, 16 * kWinoQT), SEG_WINO_OUT_CSPLIT ? seg_cdiv(Cout, 64) : 1), dim3(256), 0, stream, work, a.T, Cout, N, H, W, a.th,
                     a.tw, bias, add, ldadd, out, ldout, stat);
  SEG_RET_LAST();
}

// seg_conv_wino's result (bitwise up to the association of the input transform's adds) from one launch with no M
// workspace: wino_fused_kernel.  Same arguments as seg_conv_wino without `work`.
#ifdef SEG_WF2_TEST
static int g_wf2_mask = 3;
#endif
SEG_API int seg_conv_wino_fused(const float* in, long ldin, int N, int H, int W, int Cin, const float* wk, int ldk,
                                const float* bias, float* out, long ldout, int Cout, const float* add, long ldadd,
                                float* stat, hipStream_t stream) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (ldin & 3) || (ldk & 3) || ldk < Cin || (Cout & 3) || (add && ldadd < Cout) ||
      ldout < Cout)
    return (int)hipErrorInvalidValue;
  WinoFusedArgs a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias; a.add = add; a.ldadd = ldadd;
  a.out = out; a.ldout = ldout; a.stat = stat;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.th = H / 2; a.tw = W / 2; a.T = N * a.th * a.tw;
  if (a.T == 0) return 0;
  const long wk_bytes = 16L * Cout * ldk * 4;
  if (!fused_fits(N, H, W, ldin) || wk_bytes >= (long)kFusedOOB) return (int)hipErrorInvalidValue;
  a.in_elems = ((long)N * H * W - 1) * ldin + Cin;
  a.wk_bytes = (unsigned)wk_bytes;
#ifdef SEG_WF2_TEST
  // bit 0: calls with a bias or BN partials (the forward), bit 1: the others (data gradients)
  if ((g_wf2_mask >> ((bias || stat) ? 0 : 1)) & 1) {
    hipLaunchKernelGGL(wino_fused2_kernel, dim3(seg_cdiv(a.T, 64) * seg_cdiv(Cout, 32)), dim3(256), 0, stream, a);
    SEG_RET_LAST();
  }
#endif
  hipLaunchKernelGGL(wino_fused_kernel<4>, dim3(seg_cdiv(a.T, 128) * seg_cdiv(Cout, 32)), dim3(256), 0, stream, a);
  SEG_RET_LAST();
}
#ifdef SEG_WF2_TEST
SEG_API int seg_wf2_mask(int m) {
  g_wf2_mask = m;
  return 0;
}
#endif

// Use the Winograd weight gradient?  Measured on MI355X (tools/winobench.py):
// 1.19-1.33x for Cin, Cout >= 128 at 65536+ tiles (UNet 512x1024) and for
// Cin, Cout >= 256 at 4096 tiles; 0.97-1.08x for 128-288 channels at 16384 tiles.
SEG_API int seg_conv_wino_wgrad_pick(int N, int H, int W, int Cin, int Cout) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (Cout & 3)) return 0;
  return (Cin >= 32 && Cout >= 32) ? 2 : 0;
}

// Tile (Cout x Cin, square) of wino_wgrad16_kernel.
#ifndef SEG_WW16_WIDE
#define SEG_WW16_WIDE 128
#endif
static int wgrad16_tile(int Cin, int Cout) { return (Cin >= SEG_WW16_WIDE && Cout >= SEG_WW16_WIDE) ? 64 : 32; }

// Split count of seg_conv_wino_wgrad16 from a cost model fitted to tools/ww16sweep.py on MI355X: a launch runs in
// rounds of `slots` resident blocks (256 CUs x 1 block of the 64 tile or 2 of the 32 tile); a block costs u ns per
// 2x2 tile of its K range (64 tile 490, 32 tile 300, with the CU full); the slabs cost their write + read at
// ~4 TB/s.  Picks the split count (<= 1024, >= 64 tiles per split) of least modelled time.
SEG_API int seg_conv_wino_wgrad16_splits(int N, int H, int W, int Cin, int Cout) {
  const long T = (long)N * (H / 2) * (W / 2);
  const int b = wgrad16_tile(Cin, Cout);
  const long tiles = (long)seg_cdiv(Cout, b) * seg_cdiv(Cin, b);
  const long slots = b == 64 ? 256 : 512;
  const double u = b == 64 ? 490.0 : 300.0, slab_ns = 16.0 * Cout * Cin * 4 * 2 / 4000.0;
  const long smax = std::max<long>(1, std::min<long>(1024, T / 64));
  long best = 1;
  double best_t = 0;
  for (long sp = 1; sp <= smax; ++sp) {
    const long chunk = seg_cdiv(seg_cdiv(T, sp), (long)WBK) * WBK;
    const long used = seg_cdiv(T, chunk);  // splits past the end write zero slabs
    const double t = (double)seg_cdiv(sp * tiles, slots) * chunk * u + sp * slab_ns;
    if (used == sp && (sp == 1 || t < best_t)) best = sp, best_t = t;
  }
  return (int)best;
}

// Split count of seg_conv_wino_wgrad (partial slabs of 16 * Cout * Cin_pad floats).
SEG_API int seg_conv_wino_wgrad_splits(int N, int H, int W, int Cin, int Cout) {
  const long T = (long)N * (H / 2) * (W / 2);
  const int bm = Cout >= 128 ? 128 : (Cout >= 64 ? 64 : 32);
  const int bn = bm == 32 ? 128 : (Cin >= 128 ? 128 : 64);
  const long tiles = 16L * seg_cdiv(Cout, bm) * seg_cdiv(Cin, bn);
  long splits = (2048 + tiles - 1) / tiles;
  splits = std::min(splits, std::max<long>(1, T / 128));  // >= 128 tiles (512 pixels) per split
  return (int)std::max<long>(1, std::min<long>(splits, 1024));
}

// Weight gradient of a stride-1 pad-1 3x3 conv by Winograd F(3x3,2x2):
// part[splits][16][Cout][Cin] (Cin % 4 == 0: the padded input channels).
SEG_API int seg_conv_wino_wgrad(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int Cin,
                                int Cout, float* part, int splits, hipStream_t stream) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (Cout & 3) || (lddy & 3) || (ldx & 3) || splits < 1)
    return (int)hipErrorInvalidValue;
  WinoWgradArgs a;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.th = H / 2; a.tw = W / 2; a.T = N * a.th * a.tw;
  a.kchunk = seg_cdiv(seg_cdiv(a.T, splits), WBK) * WBK;
  const int bm = Cout >= 128 ? 128 : (Cout >= 64 ? 64 : 32);
  const int bn = bm == 32 ? 128 : (Cin >= 128 ? 128 : 64);
  dim3 grid(seg_cdiv(Cout, bm) * seg_cdiv(Cin, bn) * splits, 1, 16);
  if (bm == 128 && bn == 128) hipLaunchKernelGGL((wino_wgrad_kernel<128, 128, 64, 64>), grid, dim3(256), 0, stream, a);
  else if (bm == 128) hipLaunchKernelGGL((wino_wgrad_kernel<128, 64, 64, 32>), grid, dim3(256), 0, stream, a);
  else if (bm == 64 && bn == 128) hipLaunchKernelGGL((wino_wgrad_kernel<64, 128, 32, 64>), grid, dim3(256), 0, stream, a);
  else if (bm == 64) hipLaunchKernelGGL((wino_wgrad_kernel<64, 64, 32, 32>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((wino_wgrad_kernel<32, 128, 32, 32>), grid, dim3(256), 0, stream, a);
  SEG_RET_LAST();
}

// seg_conv_wino_wgrad's slabs (the same arguments and split boundaries) from wino_wgrad16_kernel: one block per
// (Cout, Cin) tile and split for all 16 transform points.
SEG_API int seg_conv_wino_wgrad16(const float* dy, long lddy, const float* x, long ldx, int N, int H, int W, int Cin,
                                  int Cout, float* part, int splits, hipStream_t stream) {
  if ((H & 1) || (W & 1) || (Cin & 3) || (Cout & 3) || (lddy & 3) || (ldx & 3) || splits < 1)
    return (int)hipErrorInvalidValue;
  WinoWgradArgs a;
  a.dy = dy; a.lddy = lddy; a.x = x; a.ldx = ldx; a.part = part;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.th = H / 2; a.tw = W / 2; a.T = N * a.th * a.tw;
  a.kchunk = seg_cdiv(seg_cdiv(a.T, splits), WBK) * WBK;
  if (a.T == 0) return 0;
  // a split's pixel rows (its tile rows + the halo, across image boundaries) must fit the kernel's 31-bit buffer
  // offsets from its base; otherwise the per-point kernel writes the same slabs
  const long span = (2L * (seg_cdiv(a.kchunk, a.tw) + 1) + 2) * W * std::max(ldx, lddy) * 4;
  if (span >= (long)kFusedOOB - 16) return seg_conv_wino_wgrad(dy, lddy, x, ldx, N, H, W, Cin, Cout, part, splits, stream);
  const int b = wgrad16_tile(Cin, Cout);
  const dim3 grid(seg_cdiv(Cout, b) * seg_cdiv(Cin, b) * splits);
  if (b == 64) hipLaunchKernelGGL((wino_wgrad16_kernel<64, 64, 8>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((wino_wgrad16_kernel<32, 32, 16>), grid, dim3(256), 0, stream, a);
  SEG_RET_LAST();
}

// dW (PyTorch layout [Cout][Cin][3][3]) (+)= G^T (fixed-order sum of the slabs) G.
// Above 16 splits the slabs are first folded in place into <= 16 run sums (the slabs are consumed).
SEG_API int seg_conv_wino_wgrad_reduce(float* part, int splits, float* dw, int Cout, int Cin, int Cin_pad,
                                       int accumulate, hipStream_t stream) {
  if (Cin_pad < Cin || (Cin_pad & 3) || splits < 1) return (int)hipErrorInvalidValue;
  int runs = splits, L = 1;
  if (splits > 16) {
    L = seg_cdiv(splits, 16);
    runs = seg_cdiv(splits, L);
    const long E4 = 4L * Cout * Cin_pad;  // 16 * Cout * Cin_pad floats per slab
    hipLaunchKernelGGL(wino_wgrad_fold_kernel, dim3(seg_cdiv(E4, 256), runs), dim3(256), 0, stream, part, splits, L,
                       E4);
  }
  hipLaunchKernelGGL(wino_wgrad_reduce_kernel, dim3(seg_cdiv((long)Cout * Cin, 256)), dim3(256), 0, stream, part,
                     runs, L, Cout, Cin_pad, Cin, dw, accumulate);
  SEG_RET_LAST();
}
