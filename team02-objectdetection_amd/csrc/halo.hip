// Direct 3x3 convolution (stride 1, pad 1) with an LDS halo tile, on the f32
// matrix cores -- for the narrow, high-resolution decoder convs (src/unet.py:58,61:
// up3/up4 of MobileNetV2UNet, Cout 32-64 at 64x128 .. 128x256; UNet's full-size
// levels).  With so few output channels the implicit GEMM's A operand (im2col)
// feeds only Cout MACs per loaded element and the kernel runs at the L2 bandwidth
// (85-110 TF/s measured).  Here a block owns a 4 x 64 output-pixel tile and all
// output channels: each K chunk loads the (4+2) x (64+2) input halo once into
// LDS and the 9 taps read shifted windows of it, so global/L2 traffic per MAC
// drops ~6x and the MFMA pipe sets the pace.
//
//   out[p][co] = sum_{tap, ci} in[p + tap][ci] * W[co][tap][ci] (+ bias) (+ add)
//
// Operands are LDS rows of BK+4 floats (conflict-free ds_read_b128, as
// igemm.hip); v_mfma_f32_32x32x2_f32 (exact fp32).  Each of the 4 waves owns one
// output row of the tile (64 pixels = 2 MFMA row blocks) and all Cout columns.
// The epilogue is igemm.hip's: bias, BatchNorm partials of the 256-pixel tile
// ([tile][2][Cout], tile_rows 256), addend.  The data gradient of these convs is
// the same operation on dY with the transposed, flipped weights.
#include "common.h"

namespace {

constexpr int TH = 4, TW = 64;                // output tile (pixels)
constexpr int HH = TH + 2, HW = TW + 2;       // halo tile

__device__ __attribute__((aligned(16))) float g_hzero4[4];

struct HaloArgs {
  const void* in; long ldin;     // T (float, or __bf16 on the bf16io path)
  const void* wk; int ldk;       // packed [Cout][ldk], k = tap*Cin + ci (seg_pack_batch mode 0/1; fp32, or bf16: WB)
  const float* bias;
  const void* add; long ldadd;   // T
  void* out; long ldout;         // T
  float* stat;                   // BN partials [tiles][2][Cout]
  int N, H, W, Cin, Cout;
  int tiles_w, tiles_h;
};

// T: activation storage (in / add / out).  T = __bf16 (the bf16io configuration):
// bf16 operands in LDS (the halo copied as is, 8 channels per 16-byte slot; weights
// rounded on the way in), 32-deep K chunks and v_mfma_f32_32x32x16_bf16 with fp32
// accumulation; the fp32 epilogue rounds once on the store.
// WB: bf16-packed weights (mode | 16), 8 per 16-byte slot copied to LDS as is -- every
// 256-pixel tile re-reads all 9 x Cout x Cin weights, so this halves the kernel's L2
// weight traffic; bitwise the fp32-weight launch (the same RNE rounding, done at pack time).
template <int NI, typename T = float, bool WB = false>  // output-channel blocks of 32 (Cout padded to 32*NI)
__global__ __launch_bounds__(256) void halo3x3_kernel(HaloArgs a) {
  static_assert(!WB || sizeof(T) == 2, "bf16 weights: the bf16io kernel");
  const float* wk32 = static_cast<const float*>(a.wk);
  const __bf16* wk16 = static_cast<const __bf16*>(a.wk);
  constexpr bool LP = sizeof(T) == 2;
  constexpr int BK = LP ? 32 : 16;                 // K chunk (input channels)
  constexpr int LDSR = LP ? BK + 8 : BK + 4;       // LDS row stride (elements): conflict-free b128 reads
  constexpr int HV = LP ? 8 : 4;                   // halo channels per load slot
  constexpr int HALO_VEC = HH * HW * (BK / HV);    // slots of a halo chunk
  constexpr int HALO_PER = (HALO_VEC + 255) / 256;
  constexpr int BNC = 32 * NI;
  constexpr int WV = WB ? 8 : 4;                   // weights per load slot
  constexpr int W_VEC = 9 * BNC * (BK / WV);
  constexpr int W_PER = (W_VEC + 255) / 256;
  using lds_t = T;
  __shared__ __attribute__((aligned(16))) lds_t Hs[HH * HW * LDSR];
  __shared__ __attribute__((aligned(16))) lds_t Ws[9 * BNC * LDSR];
  static_assert(sizeof(lds_t) * HH * HW * LDSR >= 4 * 5 * BNC, "BN-statistics scratch fits in Hs");
  const T* in = static_cast<const T*>(a.in);
  const T* add = static_cast<const T*>(a.add);
  T* out = static_cast<T*>(a.out);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);  // neighbouring tiles share an XCD's L2
  const int tw_i = lid % a.tiles_w;
  const int th_i = (lid / a.tiles_w) % a.tiles_h;
  const int n = lid / (a.tiles_w * a.tiles_h);
  const int h0 = th_i * TH, w0 = tw_i * TW;
  const T* inb = in + (long)n * a.H * a.W * a.ldin;

  // halo slots: (halo pixel, float4 channel group) -> global offset or the zero page
  long hoff[HALO_PER];
  bool hok[HALO_PER];
#pragma unroll
  for (int i = 0; i < HALO_PER; ++i) {
    const int s = tid + i * 256;
    const int hp = s / (BK / HV), q = s % (BK / HV);
    const int hy = hp / HW, hx = hp % HW;
    const int gy = h0 - 1 + hy, gx = w0 - 1 + hx;
    hok[i] = s < HALO_VEC && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W;
    hoff[i] = hok[i] ? ((long)gy * a.W + gx) * a.ldin + q * HV : 0;
  }
  // weight slots: (tap, co, float4 group)
  long woff[W_PER];
  bool wok[W_PER];
#pragma unroll
  for (int i = 0; i < W_PER; ++i) {
    const int s = tid + i * 256;
    const int row = s / (BK / WV), q = s % (BK / WV);  // row = tap * BNC + co
    const int tap = row / BNC, co = row % BNC;
    wok[i] = s < W_VEC && co < a.Cout;
    woff[i] = wok[i] ? (long)co * a.ldk + tap * a.Cin + q * WV : 0;
  }

  f32x4 rh[HALO_PER], rw[W_PER];
  auto load = [&](int c0) {
#pragma unroll
    for (int i = 0; i < HALO_PER; ++i) {
      const int q4 = ((tid + i * 256) % (BK / HV)) * HV;
      if constexpr (LP)  // 8 bf16 as an opaque 16-byte payload (Cin % 8 == 0)
        rh[i] = *reinterpret_cast<const f32x4*>(hok[i] && c0 + q4 < a.Cin ? inb + hoff[i] + c0
                                                                          : reinterpret_cast<const T*>(g_hzero4));
      else
        rh[i] = ld4(hok[i] && c0 + q4 < a.Cin ? inb + hoff[i] + c0 : g_hzero4);
    }
#pragma unroll
    for (int i = 0; i < W_PER; ++i) {
      const int q4 = ((tid + i * 256) % (BK / WV)) * WV;
      if constexpr (WB)
        rw[i] = *reinterpret_cast<const f32x4*>(wok[i] && c0 + q4 < a.Cin ? (const void*)(wk16 + woff[i] + c0)
                                                                           : (const void*)g_hzero4);
      else
        rw[i] = ld4(wok[i] && c0 + q4 < a.Cin ? wk32 + woff[i] + c0 : g_hzero4);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < HALO_PER; ++i) {
      const int s = tid + i * 256;
      if (HALO_VEC % 256 == 0 || s < HALO_VEC) {
        const f32x4 v = rh[i];
        *reinterpret_cast<f32x4*>(&Hs[(s / (BK / HV)) * LDSR + (s % (BK / HV)) * HV]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < W_PER; ++i) {
      const int s = tid + i * 256;
      if (W_VEC % 256 == 0 || s < W_VEC) {
        lds_t* p = &Ws[(s / (BK / WV)) * LDSR + (s % (BK / WV)) * WV];
        if constexpr (WB) *reinterpret_cast<f32x4*>(p) = rw[i];  // 8 bf16 as packed
        else if constexpr (LP) *reinterpret_cast<bf16x4*>(p) = __builtin_convertvector(rw[i], bf16x4);
        else *reinterpret_cast<f32x4*>(p) = rw[i];
      }
    }
  };

  f32x16 acc[2][NI];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
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
    if constexpr (LP) {
      const int lk8 = (lane >> 5) * 8;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap % 3;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
          bf16x8 af[2], bf[NI];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
            af[mi] = *reinterpret_cast<const bf16x8*>(
                &Hs[((wave + ky) * HW + mi * 32 + lrow + kx) * LDSR + ks * 16 + lk8]);
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            bf[ni] = *reinterpret_cast<const bf16x8*>(&Ws[(tap * BNC + ni * 32 + lrow) * LDSR + ks * 16 + lk8]);
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
        }
      }
      __syncthreads();
      continue;
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap % 3;
#pragma unroll
      for (int ks = 0; ks < BK / 8; ++ks) {
        f32x4 af[2], bf[NI];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
          af[mi] = *reinterpret_cast<const f32x4*>(&Hs[((wave + ky) * HW + mi * 32 + lrow + kx) * LDSR + ks * 8 + lk]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          bf[ni] = *reinterpret_cast<const f32x4*>(&Ws[(tap * BNC + ni * 32 + lrow) * LDSR + ks * 8 + lk]);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][kk], bf[ni][kk], acc[mi][ni], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // epilogue (C layout of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5));
  // wave row `wave`, pixel column mi*32 + row
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = ni * 32 + lrow;
    const float b = (a.bias && col < a.Cout) ? a.bias[col] : 0.f;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] += b;
  }
  const long pix0 = ((long)n * a.H + h0 + wave) * a.W + w0;
  if (a.stat) {
    // BN partials of the 256-pixel tile: column sums, then M2 about the tile mean
    float* red = reinterpret_cast<float*>(Hs);  // [4 waves][BNC]
    float* tmean = red + 4 * BNC;               // [BNC]
    const long tile = lid;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int cl = ni * 32 + lrow;
        const float mu = pass ? tmean[cl] : 0.f;
        float sacc = 0.f;
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = acc[mi][ni][r] - mu;
            sacc += pass ? d * d : d;
          }
        sacc += __shfl_xor(sacc, 32, 64);
        if (lane < 32) red[wave * BNC + cl] = sacc;
      }
      __syncthreads();
      if (tid < BNC) {
        const float t = red[tid] + red[BNC + tid] + red[2 * BNC + tid] + red[3 * BNC + tid];
        if (pass == 0) tmean[tid] = t / (float)(TH * TW);
        if (tid < a.Cout) a.stat[(tile * 2 + pass) * a.Cout + tid] = t;
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = ni * 32 + lrow;
    if (col >= a.Cout) continue;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long p = pix0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        float v = acc[mi][ni][r];
        if (add) v += (float)add[p * a.ldadd + col];
        out[p * a.ldout + col] = static_cast<T>(v);
      }
  }
}


}  // namespace

// 1 when seg_conv_halo handles this stride-1 pad-1 3x3 conv: H % 4 == 0,
// W % 64 == 0, Cout <= 96, Cin % 4 == 0, Cin >= 16.
SEG_API int seg_conv_halo_ok(int N, int H, int W, int Cin, int Cout) {
  return (N > 0 && H % TH == 0 && W % TW == 0 && Cout > 0 && Cout <= 96 && (Cin & 3) == 0 && Cin >= 16) ? 1 : 0;
}

// 1 when the cost model prefers seg_conv_halo to seg_conv_igemm.  Measured on
// MI355X (tools/winobench.py): 1.06-1.27x for Cout 32 / 64 (MobileNetV2UNet up3/up4,
// UNet 512x1024 levels); 0.99x at Cout 80 (three 32-column blocks: one block per CU).
SEG_API int seg_conv_halo_pick(int N, int H, int W, int Cin, int Cout) {
  return seg_conv_halo_ok(N, H, W, Cin, Cout) && Cout <= 64 ? 1 : 0;
}

// BN-partial row tiles of seg_conv_halo (256 pixels each).
SEG_API int seg_conv_halo_row_tiles(int N, int H, int W) { return N * (H / TH) * (W / TW); }

// out = conv3x3(in, W) (+bias) (+add), stride 1, pad 1; wk packed by
// seg_pack_conv_weight (mode 0 forward / mode 1 data gradient), ldk >= 9*Cin.
template <typename T, bool WB = false>
static int conv_halo_impl(const T* in, long ldin, int N, int H, int W, int Cin, const void* wk, int ldk,
                          const float* bias, T* out, long ldout, int Cout, const T* add, long ldadd, float* stat,
                          hipStream_t stream) {
  if (!seg_conv_halo_ok(N, H, W, Cin, Cout) || (ldin & 3) || (ldk & 3) || ldk < 9 * Cin) return (int)hipErrorInvalidValue;
  if (sizeof(T) == 2 && ((Cin & 7) || (ldin & 7))) return (int)hipErrorInvalidValue;  // 16-byte bf16 halo slots
  if (WB && ((ldk & 7) || ((uintptr_t)wk & 15))) return (int)hipErrorInvalidValue;    // 16-byte bf16 weight slots
  HaloArgs a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias; a.add = add; a.ldadd = ldadd;
  a.out = out; a.ldout = ldout; a.stat = stat; a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
  a.tiles_w = W / TW; a.tiles_h = H / TH;
  const int grid = N * a.tiles_h * a.tiles_w;
  if (Cout <= 32) hipLaunchKernelGGL((halo3x3_kernel<1, T, WB>), dim3(grid), dim3(256), 0, stream, a);
  else if (Cout <= 64) hipLaunchKernelGGL((halo3x3_kernel<2, T, WB>), dim3(grid), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((halo3x3_kernel<3, T, WB>), dim3(grid), dim3(256), 0, stream, a);
  SEG_RET_LAST();
}

SEG_API int seg_conv_halo(const float* in, long ldin, int N, int H, int W, int Cin, const float* wk, int ldk,
                          const float* bias, float* out, long ldout, int Cout, const float* add, long ldadd,
                          float* stat, hipStream_t stream) {
  return conv_halo_impl(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Cout, add, ldadd, stat, stream);
}

// seg_conv_halo on bf16 activation storage with bf16 math (the bf16io configuration):
// bf16 operands, fp32 accumulation and epilogue, one rounding on the store.  Cin and
// ldin multiples of 8.
SEG_API int seg_conv_halo_bf16io(const __bf16* in, long ldin, int N, int H, int W, int Cin, const float* wk, int ldk,
                                 const float* bias, __bf16* out, long ldout, int Cout, const __bf16* add, long ldadd,
                                 float* stat, hipStream_t stream) {
  return conv_halo_impl(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Cout, add, ldadd, stat, stream);
}

// seg_conv_halo_bf16io with bf16-packed weights (seg_pack_batch mode | 16; ldk % 8 == 0,
// 16-byte aligned): bitwise the fp32-weight launch, half the weight traffic.
SEG_API int seg_conv_halo_bf16io_w16(const __bf16* in, long ldin, int N, int H, int W, int Cin, const __bf16* wk,
                                     int ldk, const float* bias, __bf16* out, long ldout, int Cout, const __bf16* add,
                                     long ldadd, float* stat, hipStream_t stream) {
  return conv_halo_impl<__bf16, true>(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Cout, add, ldadd, stat,
                                      stream);
}
