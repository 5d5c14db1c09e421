// Fused backward of a 1x1 conv followed by train-mode BatchNorm (+ ReLU6 / none):
// the torchvision InvertedResidual expand / project convs at high resolution
// (reached through src/unet.py:15-19).  The unfused path streams the
// Cout-channel tensors five times per layer -- BN reduction (dA, y), BN apply
// (dA, y -> dY), weight gradient (dY, x), data gradient (dY -> dx) -- and these
// layers carry the largest activations of the network (features.2's expand:
// 403 MB per tensor at bs=32, 256x512).  Here one kernel reads dA, y and x once:
//
//   per 32-pixel tile (blocks loop over tiles):
//     dY = g*inv * (dz - mean(dz) - xhat * mean(dz*xhat)),  dz = dA * act'(y)   -> LDS
//     x tile                                                                     -> LDS
//     dx[p][ci]  = sum_co dY[p][co] * W[co][ci]   (+ addend)   MFMA, written per tile
//     dW[co][ci] += sum_p dY[p][co] * x[p][ci]                 MFMA, kept in registers
//   per block: the dW partial slab (reduced by seg_conv_wgrad_reduce, fixed order).
//
// dY uses the exact expression of bn.hip's apply pass (bitwise the same values);
// the BN reduction (mean(dz), mean(dz*xhat), dgamma, dbeta) still comes first
// (seg_bn_backward_coef).  W^T and the six per-channel coefficient vectors are
// staged in LDS once per block.  Operands are fed to v_mfma_f32_32x32x2_f32 from
// LDS: the data gradient reads 4 consecutive k per lane (ds_read_b128), the
// weight gradient reads k-major columns (ds_read_b32), like igemm.hip / wgrad.hip.
#include "common.h"

namespace {

constexpr int PT = 32;        // pixels per tile
constexpr int MAXC = 192;     // channel limit of either side (padded to 32)

struct PwBwdArgs {
  const float* da; long ldda;
  const float* y; long ldy;
  const float* x; long ldx;
  const float* wkd; int ldkd;   // W^T [Cin][ldkd] (seg_pack_conv_weight mode 1, ks 1), zero past Cout
  const float* scale; const float* shift; const float* mean; const float* coef;  // coef [3][Cout]
  int act;
  const float* add; long ldadd;
  float* dx; long lddx;
  float* part;                  // [gridDim.x][Cout][Cin_pad]
  int M, Cin, Cin_pad, Cout, COP, CIP, ntiles;
};

// COP, CIP: channel counts padded to 32 (compile-time: exact register arrays)
template <int COP, int CIP>
__global__ __launch_bounds__(256) void pw_bwd_kernel(PwBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int DR = COP + 4, XR = CIP + 4;
  constexpr int ND = PT * COP / 4, NX = PT * CIP / 4;          // float4 slots per tile
  constexpr int SD = (ND + 255) / 256, SX = (NX + 255) / 256;  // per thread
  constexpr int NCIT = CIP / 32, NCOT = COP / 32;
  constexpr int NDG = NCIT, NWG = NCOT * NCIT;                 // dgrad / wgrad 32x32 tiles
  constexpr int DGW = (NDG + 3) / 4, WGW = (NWG + 3) / 4;      // per wave
  float* D = lds;                   // [PT][DR]   dY tile (pixel-major)
  float* X = D + PT * DR;           // [PT][XR]   x tile
  float* WT = X + PT * XR;          // [CIP][DR]  W^T
  float* CF = WT + CIP * DR;        // [6][COP]   scale, shift, mean, k1, k2, k3
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lrow = lane & 31, lh = lane >> 5, lk = lh * 4;

  // stage W^T and the BN coefficients (zero past the real channels)
  for (int i = tid; i < CIP * (COP / 4); i += 256) {
    const int ci = i / (COP / 4), c4 = (i - ci * (COP / 4)) * 4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (ci < a.Cin && c4 < a.ldkd) v = ld4(a.wkd + (long)ci * a.ldkd + c4);
    st4(WT + ci * DR + c4, v);
  }
  for (int i = tid; i < COP; i += 256) {
    const bool ok = i < a.Cout;
    CF[i] = ok ? a.scale[i] : 0.f;
    CF[COP + i] = ok ? a.shift[i] : 0.f;
    CF[2 * COP + i] = ok ? a.mean[i] : 0.f;
    CF[3 * COP + i] = ok ? a.coef[i] : 0.f;
    CF[4 * COP + i] = ok ? a.coef[a.Cout + i] : 0.f;
    CF[5 * COP + i] = ok ? a.coef[2 * a.Cout + i] : 0.f;
  }

  // fixed per-thread slots: (pixel row, float4 channel group) of the dA/y and x tiles
  int dro[SD], dco[SD], xro[SX], xco[SX];
#pragma unroll
  for (int i = 0; i < SD; ++i) {
    const int s = tid + i * 256;
    dro[i] = s / (COP / 4);
    dco[i] = (s % (COP / 4)) * 4;
  }
#pragma unroll
  for (int i = 0; i < SX; ++i) {
    const int s = tid + i * 256;
    xro[i] = s / (CIP / 4);
    xco[i] = (s % (CIP / 4)) * 4;
  }
  f32x4 rda[SD], ry[SD], rx[SX];
  auto load = [&](int tile) {
    const int p0 = tile * PT;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < SD; ++i) {
      const int p = p0 + dro[i];
      const bool ok = (ND % 256 == 0 || tid + i * 256 < ND) && p < a.M && dco[i] < a.Cout;
      rda[i] = ok ? ld4(a.da + (long)p * a.ldda + dco[i]) : z;
      ry[i] = ok ? ld4(a.y + (long)p * a.ldy + dco[i]) : z;
    }
#pragma unroll
    for (int i = 0; i < SX; ++i) {
      const int p = p0 + xro[i];
      const bool ok = (NX % 256 == 0 || tid + i * 256 < NX) && p < a.M && xco[i] < a.Cin;
      rx[i] = ok ? ld4(a.x + (long)p * a.ldx + xco[i]) : z;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < SD; ++i) {
      if (ND % 256 == 0 || tid + i * 256 < ND) {
        const int c = dco[i];
        const f32x4 v = ry[i], g = rda[i];
        const f32x4 sc = ld4(CF + c), sh = ld4(CF + COP + c), mu = ld4(CF + 2 * COP + c);
        const f32x4 k1 = ld4(CF + 3 * COP + c), k2 = ld4(CF + 4 * COP + c), k3 = ld4(CF + 5 * COP + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float dz = g[j] * seg_act_mask(v[j] * sc[j] + sh[j], a.act);
          o[j] = k1[j] * (dz - k2[j] - (v[j] - mu[j]) * k3[j]);
        }
        st4(D + dro[i] * DR + c, o);
      }
    }
#pragma unroll
    for (int i = 0; i < SX; ++i)
      if (NX % 256 == 0 || tid + i * 256 < NX) st4(X + xro[i] * XR + xco[i], rx[i]);
  };

  // tiles of the two GEMMs assigned round-robin to the 4 waves
  constexpr int ncit = NCIT, ndg = NDG, nwg = NWG;
  f32x16 adg[DGW], awg[WGW];
#pragma unroll
  for (int j = 0; j < WGW; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) awg[j][r] = 0.f;

  int tile = blockIdx.x;
  if (tile < a.ntiles) load(tile);
  __syncthreads();  // W^T / coefficients staged
  for (; tile < a.ntiles; tile += gridDim.x) {
    store();
    __syncthreads();
    if (tile + (int)gridDim.x < a.ntiles) load(tile + gridDim.x);
    // data gradient: dx[p][ci] = sum_co D[p][co] * WT[ci][co]
#pragma unroll
    for (int j = 0; j < DGW; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) adg[j][r] = 0.f;
      const int t = wave + 4 * j;
      if (t >= ndg) continue;
#pragma unroll
      for (int ks = 0; ks < COP / 8; ++ks) {
        const f32x4 af = ld4(D + lrow * DR + ks * 8 + lk);
        const f32x4 bf = ld4(WT + (t * 32 + lrow) * DR + ks * 8 + lk);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) adg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[kk], bf[kk], adg[j], 0, 0, 0);
      }
    }
    // weight gradient: dW[co][ci] += sum_p D[p][co] * X[p][ci]
#pragma unroll
    for (int j = 0; j < WGW; ++j) {
      const int t = wave + 4 * j;
      if (t >= nwg) continue;
      const int cot = t / ncit, cit = t - cot * ncit;
#pragma unroll
      for (int kk = 0; kk < PT / 2; ++kk) {
        const float af = D[(2 * kk + lh) * DR + cot * 32 + lrow];
        const float bf = X[(2 * kk + lh) * XR + cit * 32 + lrow];
        awg[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, awg[j], 0, 0, 0);
      }
    }
    // dx of this tile (C layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5))
    const int p0 = tile * PT;
#pragma unroll
    for (int j = 0; j < DGW; ++j) {
      const int t = wave + 4 * j;
      if (t >= ndg) continue;
      const int ci = t * 32 + lrow;
      if (ci >= a.Cin) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int p = p0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (p < a.M) {
          float v = adg[j][r];
          if (a.add) v += a.add[(long)p * a.ldadd + ci];
          a.dx[(long)p * a.lddx + ci] = v;
        }
      }
    }
    __syncthreads();
  }
  // this block's dW partial slab
  float* slab = a.part + (long)blockIdx.x * a.Cout * a.Cin_pad;
#pragma unroll
  for (int j = 0; j < WGW; ++j) {
    const int t = wave + 4 * j;
    if (t >= nwg) continue;
    const int cot = t / ncit, cit = t - cot * ncit;
    const int ci = cit * 32 + lrow;
    if (ci >= a.Cin_pad) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = cot * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      if (co < a.Cout) slab[(long)co * a.Cin_pad + ci] = awg[j][r];
    }
  }
}

int r32(int c) { return (c + 31) & ~31; }

}  // namespace

// 1 when seg_pw_bwd_fused handles this 1x1 conv: both channel counts <= 192, at
// most 16 weight-gradient tiles (4 per wave) and the LDS footprint <= 96 KiB.
SEG_API int seg_pw_bwd_fused_ok(int Cin, int Cout) {
  if (Cin <= 0 || Cout <= 0 || (Cin & 3) || Cin > MAXC || Cout > MAXC) return 0;
  const int COP = r32(Cout), CIP = r32(Cin);
  const bool inst = (CIP == 32 && (COP == 32 || COP == 64 || COP == 96 || COP == 160 || COP == 192)) ||
                    (COP == 32 && (CIP == 64 || CIP == 96 || CIP == 160 || CIP == 192)) || (COP == 64 && CIP == 64);
  if (!inst) return 0;
  const long bytes = 4L * (PT * (COP + 4) + PT * (CIP + 4) + CIP * (COP + 4) + 6 * COP);
  return bytes <= 96 * 1024 ? 1 : 0;
}

// Blocks (= dW partial slabs) seg_pw_bwd_fused uses for M pixels.
SEG_API int seg_pw_bwd_blocks(long M) {
  const long tiles = (M + PT - 1) / PT;
  return (int)std::max<long>(1, std::min<long>((tiles + 3) / 4, 2048));  // >= 4 tiles per block
}

// dx = (BN-backward of dA through y) * W (+ add), dW partials part[blocks][Cout][Cin_pad]
// (seg_conv_wgrad_reduce mode 0, ks 1).  wkd: seg_pack_conv_weight mode 1 of the 1x1
// weight (W^T [Cin][ldkd]).  coef: [3][Cout] from seg_bn_backward_coef.
SEG_API int seg_pw_bwd_fused(const float* da, long ldda, const float* y, long ldy, const float* x, long ldx,
                             const float* wkd, int ldkd, const float* scale, const float* shift, const float* mean,
                             const float* coef, int act, const float* add, long ldadd, float* dx, long lddx,
                             float* part, int blocks, long M, int Cin, int Cout, hipStream_t stream) {
  if (!seg_pw_bwd_fused_ok(Cin, Cout) || (ldda & 3) || (ldy & 3) || (ldx & 3) || (ldkd & 3) || ldkd < Cout ||
      (lddx & 3) || blocks < 1 || blocks != seg_pw_bwd_blocks(M))
    return (int)hipErrorInvalidValue;
  PwBwdArgs a;
  a.da = da; a.ldda = ldda; a.y = y; a.ldy = ldy; a.x = x; a.ldx = ldx; a.wkd = wkd; a.ldkd = ldkd;
  a.scale = scale; a.shift = shift; a.mean = mean; a.coef = coef; a.act = act;
  a.add = add; a.ldadd = ldadd; a.dx = dx; a.lddx = lddx; a.part = part;
  a.M = (int)M; a.Cin = Cin; a.Cin_pad = (Cin + 3) & ~3; a.Cout = Cout; a.COP = r32(Cout); a.CIP = r32(Cin);
  a.ntiles = seg_cdiv(M, PT);
  const size_t lds = 4 * (size_t)(PT * (a.COP + 4) + PT * (a.CIP + 4) + a.CIP * (a.COP + 4) + 6 * a.COP);
#define SEG_PW(CO, CI)                                                                                  \
  if (a.COP == CO && a.CIP == CI) {                                                                     \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(pw_bwd_kernel<CO, CI>),                     \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);                   \
    hipLaunchKernelGGL((pw_bwd_kernel<CO, CI>), dim3(blocks), dim3(256), lds, stream, a);               \
    SEG_RET_LAST();                                                                                     \
  }
  SEG_PW(32, 32) SEG_PW(64, 32) SEG_PW(96, 32) SEG_PW(160, 32) SEG_PW(192, 32)
  SEG_PW(32, 64) SEG_PW(32, 96) SEG_PW(32, 160) SEG_PW(32, 192) SEG_PW(64, 64)
#undef SEG_PW
  return (int)hipErrorInvalidValue;
}
