// Implicit-GEMM convolution kernel template (the kernel, its launchers, the tile cost
// model and the split-K reduce), shared by one translation unit per operand type so
// the three instantiation sets compile in parallel:
//   igemm.hip       float    (exact fp32, the default math; + pack kernels)
//   igemm_bf16.hip  __bf16   (seg_conv_igemm_bf16)
//   igemm_f16.hip   _Float16 (seg_conv_igemm_f16)
// See igemm.hip for the algorithm.
#pragma once
#include "common.h"

// tuning hook (seg_igemm_force_tile, defined in igemm.hip); -1 = cost model
extern int seg_igemm_forced_tile;

namespace {

// 16 zero bytes in device memory: operand slots that fall outside the image or
// the matrix load from here instead of being zeroed after the load, so no
// instruction touches a prefetched register before the K chunk that consumes it
// (a post-load select forces an early s_waitcnt and exposes the HBM latency).
__device__ __attribute__((aligned(16))) float g_zero4[4];

struct IgemmArgs {
  const void* in; long ldin;     // IT (activation storage type: float, or __bf16 for the _bf16io path)
  const void* wk; int ldk;       // packed weights [Cout][ldk], k contiguous: fp32, or bf16 (WB: ldk % 8 == 0)
  const float* bias;             // [Cout] or nullptr
  const void* add; long ldadd;   // optional addend [M][ldadd] (may alias out), IT
  void* out; long ldout;         // IT
  float* stat;                   // optional BN partials [tilesM][2][Cout]: tile sum and M2 of `out`
  int N, H, W, Cin;
  int Ho, Wo, Cout;
  int stride, pad;
  int K, M;
  int kchunk;                    // split-K: K range of blockIdx.y (a multiple of BK); == K when unsplit
  float* part;                   // split-K: raw partial sums [gridDim.y][M][Cout] (no epilogue), else null
  int act;                       // epilogue activation of act(acc + bias + add) (SegAct); 0 in training
  // optional input transform ("lazy BN", uniform-tap path, 1x1 or 3x3): the A operand is
  // act(in * xs[c] + xb[c]) per input channel c -- the producer's BatchNorm + activation
  // applied on load instead of by a separate pass (seg_bn_act4: the same fp32 value the
  // pass would have stored, rounded to the storage type only where the pass would have)
  const float* xs; const float* xb; int xact;
  // optional BatchNorm-backward partials of `out` (a data gradient that completes dA of a BN
  // layer whose pre-BN output is `by`, [M][ldby] IT): per BM-row tile and column, the sums of
  // dz and dz (by - bmu), dz = out act'(by bsc + bsh) on the values as stored, into bpart
  // [tilesM][2][Cout] for seg_bn_bwd_finalize_tiles -- the reduction pass over dA disappears
  const void* by; long ldby; const float* bsc; const float* bsh; const float* bmu; int bact; float* bpart;
  // split-K with the combine in the launch (part set, the whole grid co-resident, <= 32 splits): seg_tile_combine's
  // words, [tilesM * tilesN][4] (zero before the first launch; an epoch word, never re-armed)
  unsigned* kcnt;
  int kspin;                     // seg_tile_combine's poll bound
};

#ifndef SEG_IGEMM_DEPTH
#define SEG_IGEMM_DEPTH 1  // register prefetch depth of the K loop (chunks in flight)
#endif
#ifndef SEG_IGEMM_STAGES
#define SEG_IGEMM_STAGES 1  // LDS stages of the K loop
#endif
#ifndef SEG_IGEMM_UT
#define SEG_IGEMM_UT 1  // uniform-tap loader when Cin % BK == 0
#endif
#ifndef SEG_IGEMM_UT2
#define SEG_IGEMM_UT2 1  // uniform-tap loader also for Cin % BK != 0 (chunks spanning two taps)
#endif
#ifndef SEG_IGEMM_BK
#define SEG_IGEMM_BK 32  // measured (MI355X): single LDS stage + BK 32 beats 2 stages x BK 16 by 4-13% on the cfg2 shapes
#endif

// BM x BN output tile per 256-thread block, 4 waves laid out (BM/WM) x (BN/WN),
// each wave owning WM x WN = (WM/32) x (WN/32) accumulators of 32x32.
// UT ("uniform tap"): Cin >= BK, so every BK-deep K chunk spans at most two
// filter taps; the chunk's tap and channel offset are wave-uniform scalars and
// each operand slot is a fixed base offset plus one of two scalar tap offsets --
// a few VALU ops per slot instead of the general path's per-slot tap tracking
// and bounds arithmetic.  The general path remains for Cin < BK (the stem).
//
// OT = operand type.  float: exact fp32 products on v_mfma_f32_32x32x2_f32.  __bf16 /
// _Float16 ("bf16 / f16 math", the bf16 and fp16 configurations of BASELINE
// configs[2]-[4]): activations and weights stay fp32 in HBM; each operand is rounded
// (RNE) on its way into LDS and the K loop runs v_mfma_f32_32x32x16_{bf16,f16} (fp32
// accumulation, 8x the K per instruction).  The 16-bit LDS rows keep the same 80-byte
// pitch at BK 32, so the ds_read_b128 fragment reads (lane half h: k = 16ks + 8h .. +7)
// stay conflict-free; the epilogue (bias, BN statistics, addend) is the fp32 one.
// IT = activation storage type of in / add / out (float, or __bf16: the bf16io path).
// WB: the packed weights are already bf16 (seg_pack_batch bf16 modes): 8 k values per
// 16-byte B slot copied to LDS as is -- half the weight bytes of the fp32 pack, which every
// M tile re-reads from L2 (2 x 1.6 GB per launch of the deep decoder convs at bs=32), and
// no conversion on the way into LDS.  Bitwise the fp32-weight kernel: the RNE rounding
// is the same, done once at pack time.
template <int BM, int BN, int WM, int WN, int KS, int BK, bool UT, typename OT = float, typename IT = float,
          bool WB = false, bool BO = false>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void igemm_conv_kernel(IgemmArgs a) {
  static_assert(!WB || std::is_same<OT, __bf16>::value, "bf16 weights feed bf16 operands");
  const float* wk32 = static_cast<const float*>(a.wk);
  const __bf16* wk16 = static_cast<const __bf16*>(a.wk);
  const IT* __restrict__ in = static_cast<const IT*>(a.in);
  const IT* add = static_cast<const IT*>(a.add);
  IT* out = static_cast<IT*>(a.out);
  const IT* zero4 = reinterpret_cast<const IT*>(g_zero4);
  constexpr int NT = 64 * (BM / WM) * (BN / WN);  // threads: one wave per WM x WN sub-tile (4 or 8 waves)
  constexpr bool LP = sizeof(OT) == 2;       // 16-bit operands
  constexpr int LDSR = LP ? BK + 8 : BK + 4;  // LDS row stride (elements): conflict-free b128 reads
  using lds_t = OT;
  typedef OT ot4 __attribute__((ext_vector_type(4)));
  typedef OT ot8 __attribute__((ext_vector_type(8)));
  constexpr int VB = WB ? 8 : 4;      // k values per B slot (fp32 packed weights: 4, bf16: 8)
  constexpr int KQ = BK / VB;         // B slots per tile row
  // A operand on bf16 storage (uniform-tap loader): 8 channels = one 16-byte load per
  // slot, copied to LDS as is (it already is the operand type); otherwise 4 channels
  constexpr int VA = (sizeof(IT) == 2 && UT) ? 8 : 4;
  static_assert(VA == 4 || std::is_same<OT, IT>::value, "raw 16-byte A copies need OT == IT");
  constexpr int KQA = BK / VA;        // A slots per tile row
  constexpr int A_VEC = BM * KQA, B_VEC = BN * KQ;
  constexpr int A_PER = (A_VEC + NT - 1) / NT;
  constexpr int B_PER = (B_VEC + NT - 1) / NT;
  constexpr int MI = WM / 32, NI = WN / 32;
  constexpr int WAVES_N = BN / WN;
  static_assert(NT == 256 || NT == 512, "4 or 8 waves per block");
  static_assert(NT % KQ == 0 && NT % KQA == 0, "uniform kq per thread");
  static_assert(!LP || BK % 16 == 0, "16-bit MFMA steps are 16 deep");
  static_assert(sizeof(lds_t) * BM * LDSR >= 4 * (BM / WM + 1) * BN, "BN-statistics scratch fits in As");

  // One LDS arena: the K loop's operand tiles, then (reused) the BN-statistics scratch and
  // the staged epilogue's band of WM output rows [WM][CSR] fp32.
  constexpr int CSR = BN + 4;
  constexpr int AB_BYTES = SEG_IGEMM_STAGES * (BM + BN) * LDSR * (int)sizeof(lds_t);
  constexpr int C_BYTES = WM * CSR * 4;
  __shared__ __attribute__((aligned(16))) char smem[AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES];
  lds_t (*As)[BM * LDSR] = reinterpret_cast<lds_t (*)[BM * LDSR]>(smem);
  lds_t (*Bs)[BN * LDSR] = reinterpret_cast<lds_t (*)[BN * LDSR]>(smem + SEG_IGEMM_STAGES * BM * LDSR * sizeof(lds_t));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  const int tiles_n = (a.Cout + BN - 1) / BN;
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);  // adjacent image rows on one XCD's L2
  const int tn = lid % tiles_n, tm = lid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * a.kchunk;  // split-K: this block's K range [kbeg, kbeg + kchunk)

  // Per-thread A slots: the pixel is fixed across the K loop; the (tap, channel)
  // position advances by BK per chunk without integer division.
  long a_base[A_PER];
  int a_hi0[A_PER], a_wi0[A_PER], a_ci[A_PER], a_ky[A_PER], a_kx[A_PER], a_k[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int idx = tid + i * NT;
    const int row = idx / KQA, kq = idx % KQA;
    const int p = m0 + row;
    a_ok[i] = (idx < A_VEC) && (p < a.M);
    const int pp = a_ok[i] ? p : 0;
    a_k[i] = kq * VA + kbeg;
    const int tap = a_k[i] / a.Cin;
    a_ci[i] = a_k[i] - tap * a.Cin;
    a_ky[i] = tap / KS;
    a_kx[i] = tap - a_ky[i] * KS;
    if (KS == 1) {
      a_base[i] = (long)pp * a.ldin;
      a_hi0[i] = a_wi0[i] = 0;
    } else {
      const int hw = a.Ho * a.Wo;
      const int n = pp / hw, rem = pp - n * hw;
      const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
      a_base[i] = (long)n * a.H * a.W;
      a_hi0[i] = ho * a.stride - a.pad;
      a_wi0[i] = wo * a.stride - a.pad;
    }
  }

  // "UT" state (Cin >= BK: a K chunk spans at most two filter taps).  Per slot: the
  // pixel's base offset and its 9-bit tap-validity mask; the chunk's starting tap
  // and channel are wave-uniform scalars, and a slot whose k (= chunk start +
  // 4*kq) crosses Cin takes the next tap.  kq = tid % KQ for every slot (256 % KQ == 0).
  long u_aoff[A_PER], u_boff[B_PER];
  unsigned u_mask[A_PER];
  bool u_bok[B_PER];
  const int u_kq4 = (tid % KQ) * VB;
  const int u_kqa = (tid % KQA) * VA;  // this thread's A channel offset in a K chunk
  // input transform: the loaded chunk's channel for this thread's A slots (-1: beyond K)
  // and its coefficients, fetched with the chunk so store_tiles does not wait on them
  const bool XF = a.xs != nullptr;
  int xch = -1;
  unsigned xvm = 0;  // 3x3: the A slots of the loaded chunk that hold real pixels (padding taps stay zero)
  f32x4 xsc[VA / 4], xsh[VA / 4];
  int u_tap = 0, u_ci = 0;
  long u_toff0 = 0, u_toff1 = 0;
  auto tap_off = [&](int t) -> long { return ((long)(t / KS) * a.W + t % KS) * a.ldin; };
  if (UT) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / KQA;
      const int p = m0 + row;
      const bool ok = (idx < A_VEC) && (p < a.M);
      const int pp = ok ? p : 0;
      if (KS == 1) {
        u_aoff[i] = (long)pp * a.ldin;
        u_mask[i] = ok ? 1u : 0u;
      } else {
        const int hw = a.Ho * a.Wo;
        const int n = pp / hw, rem = pp - n * hw;
        const int ho = rem / a.Wo, wo = rem - ho * a.Wo;
        const int hi0 = ho * a.stride - a.pad, wi0 = wo * a.stride - a.pad;
        u_aoff[i] = (((long)n * a.H + hi0) * a.W + wi0) * a.ldin;
        unsigned m = 0;
#pragma unroll
        for (int t = 0; t < KS * KS; ++t) {
          const int hi = hi0 + t / KS, wi = wi0 + t % KS;
          if (ok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) m |= 1u << t;
        }
        u_mask[i] = m;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      const int co = n0 + idx / KQ;
      u_bok[i] = idx < B_VEC && co < a.Cout;
      u_boff[i] = (long)(u_bok[i] ? co : 0) * a.ldk + u_kq4;
    }
    u_tap = kbeg / a.Cin;
    u_ci = kbeg - u_tap * a.Cin;
    u_toff0 = tap_off(u_tap);
    u_toff1 = tap_off(u_tap + 1);
  }

  auto load_tiles = [&](int k0, f32x4 (&ra)[A_PER], f32x4 (&rb)[B_PER]) {
    if (UT) {
      // address selects only (out-of-image / out-of-matrix slots read g_zero4): no
      // branch splits the loader and no instruction touches the loaded registers
      // before the chunk that consumes them
      const int ci = u_ci + u_kqa;
      const bool wrap = ci >= a.Cin;
      const int tap = u_tap + (wrap ? 1 : 0);
      const long off = (wrap ? u_toff1 : u_toff0) + (wrap ? ci - a.Cin : ci);
      if (XF) {  // the chunk's channels for this thread: ci .. ci + VA - 1 of tap `tap` (1x1: no taps)
        xch = wrap ? -1 : ci;
        const int cc = KS == 1 ? (wrap ? 0 : ci) : (wrap ? ci - a.Cin : ci);
#pragma unroll
        for (int j = 0; j < VA / 4; ++j) {
          xsc[j] = ld4(a.xs + cc + 4 * j);
          xsh[j] = ld4(a.xb + cc + 4 * j);
        }
        xvm = 0;
      }
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const bool ok = (u_mask[i] >> tap) & 1u;
        if (KS != 1 && XF && ok) xvm |= 1u << i;
        if constexpr (VA == 8)  // 8 bf16 as an opaque 16-byte payload
          ra[i] = *reinterpret_cast<const f32x4*>(ok ? in + u_aoff[i] + off : zero4);
        else
          ra[i] = ld4(ok ? in + u_aoff[i] + off : zero4);
      }
      const bool kin = k0 + u_kq4 < a.K;
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        if constexpr (WB)
          rb[i] = *reinterpret_cast<const f32x4*>(u_bok[i] && kin ? (const void*)(wk16 + u_boff[i] + k0)
                                                                  : (const void*)g_zero4);
        else
          rb[i] = ld4(u_bok[i] && kin ? wk32 + u_boff[i] + k0 : g_zero4);
      }
      u_ci += BK;
      if (u_ci >= a.Cin) {
        u_ci -= a.Cin;
        ++u_tap;
        u_toff0 = u_toff1;
        u_toff1 = tap_off(u_tap + 1);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (a_ok[i] && a_k[i] < a.K) {
        if (KS == 1) {
          v = ld4(in + a_base[i] + a_k[i]);
        } else {
          const int hi = a_hi0[i] + a_ky[i], wi = a_wi0[i] + a_kx[i];
          if ((unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W)
            v = ld4(in + (a_base[i] + (long)hi * a.W + wi) * a.ldin + a_ci[i]);
        }
      }
      ra[i] = v;
      // advance this slot to the next chunk
      a_k[i] += BK;
      if (KS != 1) {
        int ci = a_ci[i] + BK;
        while (ci >= a.Cin) {
          ci -= a.Cin;
          if (++a_kx[i] == KS) { a_kx[i] = 0; ++a_ky[i]; }
        }
        a_ci[i] = ci;
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      const int row = idx / KQ, kq = idx % KQ;
      const int co = n0 + row, k = k0 + kq * VB;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx < B_VEC && co < a.Cout && k < a.K) {
        if constexpr (WB) v = *reinterpret_cast<const f32x4*>(wk16 + (long)co * a.ldk + k);
        else v = ld4(wk32 + (long)co * a.ldk + k);
      }
      rb[i] = v;
    }
  };
  auto st_op = [](lds_t* p, f32x4 v) {
    if constexpr (LP) *reinterpret_cast<ot4*>(p) = __builtin_convertvector(v, ot4);
    else *reinterpret_cast<f32x4*>(p) = v;
  };
  auto store_tiles = [&](int buf, const f32x4 (&ra)[A_PER], const f32x4 (&rb)[B_PER]) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int idx = tid + i * NT;
      if (A_VEC % NT == 0 || idx < A_VEC) {
        f32x4 v = ra[i];
        if (XF && (KS == 1 ? xch >= 0 : ((xvm >> i) & 1u) != 0)) {
          if constexpr (VA == 8) {  // 8 bf16: widen, transform, round back (RNE) as the pass would
            const bf16x8 q = __builtin_bit_cast(bf16x8, v);
            const f32x4 lo = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 0, 1, 2, 3), f32x4),
                                         xsc[0], xsh[0], a.xact);
            const f32x4 hi = seg_bn_act4(__builtin_convertvector(__builtin_shufflevector(q, q, 4, 5, 6, 7), f32x4),
                                         xsc[VA / 4 - 1], xsh[VA / 4 - 1], a.xact);
            v = __builtin_bit_cast(f32x4, seg_cat8(__builtin_convertvector(lo, bf16x4),
                                                   __builtin_convertvector(hi, bf16x4)));
          } else {
            v = seg_bn_act4(v, xsc[0], xsh[0], a.xact);
            if constexpr (sizeof(IT) == 2) {  // 4 bf16 channels widened by ld4: round as stored
              v = __builtin_convertvector(__builtin_convertvector(v, bf16x4), f32x4);
            }
          }
        }
        if constexpr (VA == 8)
          *reinterpret_cast<f32x4*>(&As[buf][(idx / KQA) * LDSR + (idx % KQA) * 8]) = v;
        else
          st_op(&As[buf][(idx / KQA) * LDSR + (idx % KQA) * 4], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int idx = tid + i * NT;
      if (B_VEC % NT == 0 || idx < B_VEC) {
        if constexpr (WB)  // 8 bf16 as stored by the pack
          *reinterpret_cast<f32x4*>(&Bs[buf][(idx / KQ) * LDSR + (idx % KQ) * 8]) = rb[i];
        else
          st_op(&Bs[buf][(idx / KQ) * LDSR + (idx % KQ) * 4], rb[i]);
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

  const int nk = (min(a.K - kbeg, a.kchunk) + BK - 1) / BK;
  const int lrow = lane & 31, lk = (lane >> 5) * 4;
  auto compute = [&](int cur) {
    if constexpr (LP) {
      const int lk8 = (lane >> 5) * 8;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        ot8 af[MI], bfr[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
          af[mi] = *reinterpret_cast<const ot8*>(&As[cur][(wm0 + mi * 32 + lrow) * LDSR + ks * 16 + lk8]);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          bfr[ni] = *reinterpret_cast<const ot8*>(&Bs[cur][(wn0 + ni * 32 + lrow) * LDSR + ks * 16 + lk8]);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            if constexpr (std::is_same<OT, _Float16>::value)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
            else
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
          }
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < BK / 8; ++ks) {
      f32x4 af[MI], bf[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
        af[mi] = *reinterpret_cast<const f32x4*>(&As[cur][(wm0 + mi * 32 + lrow) * LDSR + ks * 8 + lk]);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
        bf[ni] = *reinterpret_cast<const f32x4*>(&Bs[cur][(wn0 + ni * 32 + lrow) * LDSR + ks * 8 + lk]);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[mi][kk], bf[ni][kk], acc[mi][ni], 0, 0, 0);
    }
  };

#if SEG_IGEMM_STAGES == 1
  // one LDS stage: regs -> LDS, barrier, prefetch the next chunk, compute, barrier
  f32x4 ra[A_PER], rb[B_PER];
  load_tiles(kbeg, ra, rb);
  for (int kt = 0; kt < nk; ++kt) {
    store_tiles(0, ra, rb);
    __syncthreads();
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK, ra, rb);
    compute(0);
    __syncthreads();
  }
#elif SEG_IGEMM_DEPTH == 1
  f32x4 ra[A_PER], rb[B_PER];
  load_tiles(kbeg, ra, rb);
  store_tiles(0, ra, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK, ra, rb);
    compute(cur);
    if (kt + 1 < nk) store_tiles(cur ^ 1, ra, rb);
    __syncthreads();
  }
#else
  // Two register sets: the global loads of chunk kt+2 are issued before chunk kt's
  // MFMAs and written to LDS only after chunk kt+1's, so each load has two compute
  // phases (~2 x 2048 MFMA cycles at 64x64 per wave) to land -- one phase is shorter
  // than the HBM latency under load, which left one-block-per-CU grids stalled.
  f32x4 ra0[A_PER], rb0[B_PER], ra1[A_PER], rb1[B_PER];
  load_tiles(kbeg, ra0, rb0);
  store_tiles(0, ra0, rb0);
  if (nk > 1) load_tiles(kbeg + BK, ra1, rb1);
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    // LDS stage 0 holds chunk kt; set 1 holds chunk kt+1 (in flight)
    if (kt + 2 < nk) load_tiles(kbeg + (kt + 2) * BK, ra0, rb0);
    compute(0);
    if (kt + 1 < nk) store_tiles(1, ra1, rb1);
    __syncthreads();
    if (kt + 1 >= nk) break;
    // LDS stage 1 holds chunk kt+1; set 0 holds chunk kt+2
    if (kt + 3 < nk) load_tiles(kbeg + (kt + 3) * BK, ra1, rb1);
    compute(1);
    if (kt + 2 < nk) store_tiles(0, ra0, rb0);
    __syncthreads();
  }
#endif

  // Epilogue: C layout of 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5).
  if (a.part) {  // split-K: raw partial sums; seg_igemm_splitk_reduce (or the in-launch combine) applies the epilogue
    float* P = a.part + (long)blockIdx.y * a.M * a.Cout;
    const bool ic = a.kcnt != nullptr;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int col = n0 + wn0 + ni * 32 + lrow;
      if (col >= a.Cout) continue;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < a.M) {
            if (ic) seg_st_wt(P + (long)row * a.Cout + col, acc[mi][ni][r]);
            else P[(long)row * a.Cout + col] = acc[mi][ni][r];
          }
        }
    }
    if (!ic) return;
    // in-launch combine (the host launches this form only when the whole grid is co-resident): the tile's splits
    // combine it together, each block applying splitk_reduce_kernel's epilogue to a 1/splits share (piece) of the
    // tile -- the same fixed-order sum, so bitwise the two-launch result; seg_tile_combine hands the piece of a block
    // that could not wait to the tile's last arrival instead of letting it spin on a peer
    const int S = gridDim.y, z = blockIdx.y;
    auto piece = [&](int pz) {
      constexpr int E = BM * BN;
      const int e0 = (int)((long)pz * E / S), e1 = (int)((long)(pz + 1) * E / S);
      const long total = (long)a.M * a.Cout;
      for (int e = e0 + tid; e < e1; e += NT) {
        const int r = e / BN, c = e - r * BN, row = m0 + r, col = n0 + c;
        if (row >= a.M || col >= a.Cout) continue;
        const long i = (long)row * a.Cout + col;
        float v = 0.f;  // the splits in order, 16 loads in flight at a time
        for (int z0 = 0; z0 < S; z0 += 16) {
          float q[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) q[j] = z0 + j < S ? seg_ld_wt(a.part + (z0 + j) * total + i) : 0.f;
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (z0 + j < S) v += q[j];
        }
        if (a.bias) v += a.bias[col];
        if (add) v += (float)add[(long)row * a.ldadd + col];
        if (a.act) v = seg_act(v, a.act);
        out[(long)row * a.ldout + col] = static_cast<IT>(v);
      }
    };
    seg_tile_combine(a.kcnt + 4 * lid, S, z, a.kspin, reinterpret_cast<int*>(smem), piece);
    return;
  }
  float bcol[NI];
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + lrow;
    bcol[ni] = (a.bias && col < a.Cout) ? a.bias[col] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] += bcol[ni];
  }
  if (a.stat) {
    // BatchNorm batch statistics of this BM-row tile, per output channel: the tile
    // sum and the sum of squared deviations from the TILE mean (two passes over the
    // accumulators, so no E[y^2]-E[y]^2 cancellation); merged over tiles with
    // Chan's formula in fp64 by seg_bn_stats_tiles.  LDS of the K loop is reused.
    constexpr int WR = BM / WM;
    float* red = reinterpret_cast<float*>(&As[0][0]);  // [WR][BN]
    float* tmean = red + WR * BN;      // [BN]
    const int nrows = min(BM, a.M - m0);
    const int wr = wave / WAVES_N;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int cl = wn0 + ni * 32 + lrow;
        const float mu = pass ? tmean[cl] : 0.f;
        float s = 0.f;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const float d = acc[mi][ni][r] - mu;
            s += row < a.M ? (pass ? d * d : d) : 0.f;
          }
        s += __shfl_xor(s, 32, 64);
        if (lane < 32) red[wr * BN + cl] = s;
      }
      __syncthreads();
      if (tid < BN) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < WR; ++j) t += red[j * BN + tid];
        const int col = n0 + tid;
        if (pass == 0) tmean[tid] = t / (float)nrows;
        if (col < a.Cout) a.stat[((long)tm * 2 + pass) * a.Cout + col] = t;
      }
      __syncthreads();
    }
  }
  // Staged store: the C layout gives each lane one column of 16 rows, so direct stores
  // write 2 x 32 consecutive elements per instruction (64 B rows on bf16 storage --
  // the output-heavy 1x1 expand convs ran at 25-50 % of a copy).  Instead, per band of
  // WM rows, the waves owning it write their accumulators (+ bias) to LDS, then every
  // thread writes 16-byte row-contiguous vectors (4 fp32 / 8 bf16 channels) with the
  // addend and activation applied in fp32 -- the same value per element as before.
  {
    float* Cs = reinterpret_cast<float*>(smem);
    constexpr int VO = 16 / (int)sizeof(IT);  // output elements per 16-byte store
    constexpr int VPR = BN / VO;              // vectors per band row
    static_assert(BN % VO == 0, "whole vectors per tile row");
    // BN-backward partials (tiles with 64 % VPR == 0: a thread's stores all fall in one column
    // vector, lane % VPR; the host refuses bpart on the other tiles, seg_conv_igemm_bnout_ok)
    constexpr bool BOK = BO && 64 % VPR == 0;  // BO: the bpart instantiation (its registers only there)
    static_assert(!BOK || 2 * (NT / 64) * BN * 4 <= (int)sizeof(smem), "BN-backward scratch");
    const IT* by = static_cast<const IT*>(a.by);
    const int bcv = (tid % VPR) * VO;
    float bs0[VO], bs1[VO], bsc[VO], bsh[VO], bmu[VO];
    constexpr bool bon = BOK;
    (void)by;
    if (bon) {
#pragma unroll
      for (int j = 0; j < VO; ++j) {
        const int c = min(n0 + bcv + j, a.Cout - 1);
        bs0[j] = bs1[j] = 0.f;
        bsc[j] = a.bsc[c];
        bsh[j] = a.bsh[c];
        bmu[j] = a.bmu[c];
      }
    }
    auto bacc = [&](int j, float g, float v) {  // g: dA as stored, v: the pre-BN output
      const float dz = g * seg_act_mask(v * bsc[j] + bsh[j], a.bact);
      bs0[j] += dz;
      bs1[j] += dz * (v - bmu[j]);
    };
    // one 16-byte output vector v of band b (yq: the BN-backward y vector when BO, prefetched)
    auto store_vec = [&](int b, int v, f32x4 yq) {
        const int rr = v / VPR, cv = (v - rr * VPR) * VO;
        const int row = m0 + b * WM + rr, col = n0 + cv;
        if (row >= a.M || col >= a.Cout) return;
        float o[VO];
#pragma unroll
        for (int j = 0; j < VO; j += 4) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(&Cs[rr * CSR + cv + j]);
          o[j] = q[0]; o[j + 1] = q[1]; o[j + 2] = q[2]; o[j + 3] = q[3];
        }
        IT* dst = out + (long)row * a.ldout + col;
        const IT* ad = add ? add + (long)row * a.ldadd + col : nullptr;
        const bool vec = col + VO <= a.Cout && ((uintptr_t)dst & 15) == 0 && (!ad || ((uintptr_t)ad & 15) == 0);
        if (vec) {
          if (ad) {
            if constexpr (VO == 8) {
              f32x4 lo, hi;
              const bf16x8 q = *reinterpret_cast<const bf16x8*>(ad);
              lo = __builtin_convertvector(__builtin_shufflevector(q, q, 0, 1, 2, 3), f32x4);
              hi = __builtin_convertvector(__builtin_shufflevector(q, q, 4, 5, 6, 7), f32x4);
#pragma unroll
              for (int j = 0; j < 4; ++j) { o[j] += lo[j]; o[4 + j] += hi[j]; }
            } else {
              const f32x4 q = ld4(reinterpret_cast<const float*>(ad));
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] += q[j];
            }
          }
          if (a.act) {
#pragma unroll
            for (int j = 0; j < VO; ++j) o[j] = seg_act(o[j], a.act);
          }
          if constexpr (VO == 8) {
            const f32x4 lo = {o[0], o[1], o[2], o[3]}, hi = {o[4], o[5], o[6], o[7]};
            const bf16x8 q = seg_cat8(__builtin_convertvector(lo, bf16x4), __builtin_convertvector(hi, bf16x4));
            *reinterpret_cast<bf16x8*>(dst) = q;
            if constexpr (bon) {
              const bf16x8 yv = __builtin_bit_cast(bf16x8, yq);
#pragma unroll
              for (int j = 0; j < 8; ++j) bacc(j, (float)q[j], (float)yv[j]);
            }
          } else {
            *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
            if constexpr (bon) {
              const f32x4 yv = __builtin_bit_cast(f32x4, yq);
#pragma unroll
              for (int j = 0; j < VO; ++j) bacc(j, o[j], (float)yv[j]);
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < VO; ++j) {
            if (col + j >= a.Cout) break;
            float x = o[j];
            if (ad) x += (float)ad[j];
            if (a.act) x = seg_act(x, a.act);
            const IT q = static_cast<IT>(x);
            dst[j] = q;
            if constexpr (bon) bacc(j, (float)q, (float)by[(long)row * a.ldby + col + j]);
          }
        }
    };
    // BO: the pre-BN y vectors of every output vector this thread stores, loaded before the bands
    // (their latency overlaps the LDS staging instead of serialising each store)
    constexpr int NVB = (WM * VPR + NT - 1) / NT;
    f32x4 yreg[BOK ? BM / WM : 1][BOK ? NVB : 1];
    if constexpr (BOK) {
#pragma unroll
      for (int b = 0; b < BM / WM; ++b)
#pragma unroll
        for (int k = 0; k < NVB; ++k) {
          const int v = tid + k * NT, rr = v / VPR, cv = (v - rr * VPR) * VO;
          const int row = m0 + b * WM + rr, col = n0 + cv;
          const bool ok = v < WM * VPR && row < a.M && col + VO <= a.Cout;
          yreg[b][k] = *reinterpret_cast<const f32x4*>(ok ? (const void*)(by + (long)row * a.ldby + col)
                                                          : (const void*)g_zero4);
        }
    }
#pragma unroll
    for (int b = 0; b < BM / WM; ++b) {
      __syncthreads();  // the K loop / statistics / previous band are done with smem
      if (wm0 == b * WM) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              Cs[(mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * CSR + wn0 + ni * 32 + lrow] = acc[mi][ni][r];
      }
      __syncthreads();
      if constexpr (BOK) {
#pragma unroll
        for (int k = 0; k < NVB; ++k) {
          const int v = tid + k * NT;
          if (v < WM * VPR) store_vec(b, v, yreg[b][k]);
        }
      } else {
        for (int v = tid; v < WM * VPR; v += NT) store_vec(b, v, f32x4{});
      }
    }
    if constexpr (BOK) {
      {  // the tile's partials: lanes of one column vector (xor over lane bits >= VPR), then waves
        constexpr int NW = NT / 64;
        float* red = reinterpret_cast<float*>(smem);  // [2][NW][BN]
#pragma unroll
        for (int j = 0; j < VO; ++j) {
#pragma unroll
          for (int o = VPR; o < 64; o *= 2) {
            bs0[j] += __shfl_xor(bs0[j], o, 64);
            bs1[j] += __shfl_xor(bs1[j], o, 64);
          }
        }
        __syncthreads();
        if (lane < VPR) {
#pragma unroll
          for (int j = 0; j < VO; ++j) {
            red[(0 * NW + wave) * BN + bcv + j] = bs0[j];
            red[(1 * NW + wave) * BN + bcv + j] = bs1[j];
          }
        }
        __syncthreads();
        for (int q = tid; q < 2 * BN; q += NT) {
          const int h = q / BN, c = q - h * BN;
          float t = 0.f;
#pragma unroll
          for (int k = 0; k < NW; ++k) t += red[(h * NW + k) * BN + c];
          if (n0 + c < a.Cout) a.bpart[((long)tm * 2 + h) * a.Cout + n0 + c] = t;
        }
      }
    }
  }
}

// set by the last launch_igemm_bk: whether its split-K combine ran in the launch (no reduce kernel needed)
thread_local bool g_igemm_ic_used = false;

template <int BM, int BN, int WM, int WN, int BK, typename OT, typename IT, bool WB = false>
int launch_igemm_bk(IgemmArgs a, int ks, hipStream_t s) {
  const int grid = seg_cdiv(a.M, BM) * seg_cdiv(a.Cout, BN);
  const int splits = seg_cdiv(a.K, a.kchunk);
  const bool ut = SEG_IGEMM_UT && (SEG_IGEMM_UT2 ? a.Cin >= BK : a.Cin % BK == 0) &&
                  (sizeof(IT) == 4 || (a.Cin % 8 == 0 && a.ldin % 8 == 0));  // bf16 A: 16-byte slots
  constexpr int NT = 64 * (BM / WM) * (BN / WN);
  if (a.xs && !ut) return (int)hipErrorInvalidValue;  // input transform: the uniform-tap loader only (Cin >= BK)
  if (a.kcnt) {  // in-launch split-K combine: only when the whole grid is co-resident (its splits combine together)
    int occ = 0;
    const void* fn = ks == 1 ? (ut ? (const void*)igemm_conv_kernel<BM, BN, WM, WN, 1, BK, true, OT, IT, WB, false>
                                   : (const void*)igemm_conv_kernel<BM, BN, WM, WN, 1, BK, false, OT, IT, WB, false>)
                             : (ut ? (const void*)igemm_conv_kernel<BM, BN, WM, WN, 3, BK, true, OT, IT, WB, false>
                                   : (const void*)igemm_conv_kernel<BM, BN, WM, WN, 3, BK, false, OT, IT, WB, false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, NT, 0) != hipSuccess ||
        (long)grid * splits > (long)occ * seg_num_cus() || splits > 32) {
      (void)hipGetLastError();
      a.kcnt = nullptr;
    }
  }
  g_igemm_ic_used = a.kcnt != nullptr;
#define SEG_IG(KS, U, B) hipLaunchKernelGGL((igemm_conv_kernel<BM, BN, WM, WN, KS, BK, U, OT, IT, WB, B>), dim3(grid, splits), dim3(NT), 0, s, a)
  constexpr int VPR = BN / (16 / (int)sizeof(IT));
  // (instantiated for the training storage types only: f32 and bf16io, where operands are the storage type)
  if constexpr (std::is_same<OT, IT>::value && BN % (16 / (int)sizeof(IT)) == 0 && 64 % VPR == 0) {
    if (a.bpart) {  // the BN-backward-partials instantiation (seg_conv_igemm_bnout*)
      if (ks == 1) {
        if (ut) SEG_IG(1, true, true); else SEG_IG(1, false, true);
      } else {
        if (ut) SEG_IG(3, true, true); else SEG_IG(3, false, true);
      }
      SEG_RET_LAST();
    }
  }
  if (a.bpart) return (int)hipErrorInvalidValue;
  if (ks == 1) {
    if (ut) SEG_IG(1, true, false); else SEG_IG(1, false, false);
  } else {
    if (ut) SEG_IG(3, true, false); else SEG_IG(3, false, false);
  }
#undef SEG_IG
  SEG_RET_LAST();
}

// K chunk depth: SEG_IGEMM_BK (32) unless K is short and not a multiple of it
// (the stem's K = 36, 1x1 convs with Cin 16/24/144...), where padding K up to a
// 32 multiple would waste MFMA work: then 16.
inline int igemm_bk(int K) { return (SEG_IGEMM_BK != 16 && (K <= 64 || (K % SEG_IGEMM_BK != 0 && K < 512))) ? 16 : SEG_IGEMM_BK; }

// split-K: `splits` K ranges of whole BK chunks (a.part set by the caller when splits > 1)
template <int BM, int BN, int WM, int WN, typename OT = float, typename IT = float, bool WB = false>
int launch_igemm(IgemmArgs a, int ks, int splits, hipStream_t s) {
  int bk = igemm_bk(a.K);
  // 16-bit operands: 64-deep K chunks (4 MFMA k-steps per barrier) where the uniform-tap
  // loader still applies (Cin >= 64)
  // (unsplit launches only: with split-K, K ranges that are not a multiple of the
  // 64-deep chunk gave wrong partial sums -- tests/test_gpu_bf16.py::test_conv_16bit_splitk_act)
  if (sizeof(OT) == 2 && bk == SEG_IGEMM_BK && a.Cin >= 64 && a.K >= 256 && splits == 1) bk = 64;
  const int nk = seg_cdiv(a.K, bk);
  a.kchunk = seg_cdiv(nk, splits) * bk;
  if constexpr (sizeof(OT) == 2) {
    if (bk == 64) return launch_igemm_bk<BM, BN, WM, WN, 64, OT, IT, WB>(a, ks, s);
  }
  if (bk == 16) return launch_igemm_bk<BM, BN, WM, WN, 16, OT, IT, WB>(a, ks, s);
  return launch_igemm_bk<BM, BN, WM, WN, SEG_IGEMM_BK, OT, IT, WB>(a, ks, s);
}

struct TileCfg {
  int bm, bn, wm, wn;
  float eff;  // relative per-CU MFMA efficiency of the wave tile (LDS reads per MFMA)
};
// Relative efficiencies measured on MI355X (tools/tilesweep.py over the
// MobileNetV2UNet launch shapes); 64x64 wave tiles need 1 operand read per MFMA,
// 32x96 1.33, 32x32 2.
constexpr TileCfg kTiles[] = {
    {128, 128, 64, 64, 1.00f}, {64, 128, 32, 64, 0.95f}, {128, 64, 64, 32, 0.95f}, {64, 64, 32, 32, 0.85f},
    {128, 96, 32, 96, 0.97f},  {128, 160, 32, 160, 0.95f}, {256, 32, 64, 32, 0.90f}, {128, 32, 32, 32, 0.92f},
    // 8-wave (512-thread) blocks: two waves per SIMD at one block per CU
    {128, 128, 64, 32, 0.0f}, {128, 128, 32, 64, 0.0f}, {256, 128, 64, 64, 0.0f}, {128, 256, 64, 64, 0.0f},
    {128, 64, 32, 32, 0.0f}, {256, 64, 64, 32, 0.0f}, {64, 128, 32, 32, 0.0f},
};

constexpr int kTileBM[] = {128, 64, 128, 64, 128, 128, 256, 128, 128, 128, 256, 128, 128, 256, 64};

int pick_tile(long M, int N);
// seg_conv_igemm_bnout*: the picked tile's epilogue holds one column vector per lane (64 % (BN / VO) == 0)
inline bool igemm_bnout_tile_ok(long M, int N, int es) {
  const int bn = kTiles[pick_tile(M, N)].bn, vo = 16 / es;
  return bn % vo == 0 && 64 % (bn / vo) == 0;
}

int pick_tile(long M, int N) {
  if (seg_igemm_forced_tile >= 0) return seg_igemm_forced_tile;
  int best = 0;
  double best_score = -1.0;
  for (int i = 0; i < (int)(sizeof(kTiles) / sizeof(kTiles[0])); ++i) {
    const TileCfg& t = kTiles[i];
    const long bm_tiles = (M + t.bm - 1) / t.bm, bn_tiles = (N + t.bn - 1) / t.bn;
    const long blocks = bm_tiles * bn_tiles;
    const double util = (double)M * N / ((double)bm_tiles * t.bm * bn_tiles * t.bn);
    const double fill = std::min(1.0, (double)blocks / 512.0);  // >= 2 blocks per CU to hide latency
    const double score = util * t.eff * fill;
    if (score > best_score + 1e-9) {
      best_score = score;
      best = i;
    }
  }
  return best;
}



// Split-K factor for an M x Cout x K conv GEMM: > 1 only when the output tiles
// alone cannot fill the chip (small images / batch 1 inference), keeping >= 4 K
// chunks per split.
int igemm_splits(long M, int Cout, int K) {
  const int t = pick_tile(M, Cout);
  const long blocks = ((M + kTiles[t].bm - 1) / kTiles[t].bm) * ((Cout + kTiles[t].bn - 1) / kTiles[t].bn);
  const int nk = seg_cdiv(K, igemm_bk(K));
  if (blocks >= 256 || nk < 8) return 1;
  int s = (int)std::min<long>(seg_cdiv(512, blocks), nk / 4);
  s = std::min(s, 64);
  if (s < 2) return 1;
  return seg_cdiv(nk, seg_cdiv(nk, s));  // no empty split
}

// out = act(sum_z part[z] + bias + add): the split-K epilogue (fixed z order: deterministic).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, long M, int Cout,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ add, long ldadd,
                                                            float* __restrict__ out, long ldout, int act) {
  const long total = M * Cout;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long row = i / Cout;
    const int col = (int)(i - row * Cout);
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += part[z * total + i];
    if (bias) v += bias[col];
    if (add) v += add[row * ldadd + col];
    if (act) v = seg_act(v, act);
    out[row * ldout + col] = v;
  }
}

template <typename OT, typename IT = float, bool WB = false>
int conv_igemm_impl(const IT* in, long ldin, int N, int H, int W, int Cin, const void* wk, int ldk,
                    const float* bias, IT* out, long ldout, int Ho, int Wo, int Cout, int ks, int stride, int pad,
                    const IT* add, long ldadd, float* stat, int act, float* work, int splits, hipStream_t stream,
                    const float* xs = nullptr, const float* xb = nullptr, int xact = 0, const IT* by = nullptr,
                    long ldby = 0, const float* bsc = nullptr, const float* bsh = nullptr, const float* bmu = nullptr,
                    int bact = 0, float* bpart = nullptr, unsigned* kcnt = nullptr, int tile = -1) {
  if (!std::is_same<IT, float>::value && splits != 1) return (int)hipErrorInvalidValue;
  if ((Cin & 3) || (ldin & 3) || (ldk & 3) || (ks != 1 && ks != 3)) return (int)hipErrorInvalidValue;
  if (WB && ((ldk & 7) || ((uintptr_t)wk & 15) || splits != 1)) return (int)hipErrorInvalidValue;
  if (xs && (!xb || splits != 1 || SEG_IGEMM_STAGES != 1 || xact < SEG_ACT_NONE || xact > SEG_ACT_RELU6))
    return (int)hipErrorInvalidValue;
  if (ks == 1 && (stride != 1 || pad != 0 || Ho != H || Wo != W)) return (int)hipErrorInvalidValue;
  if (act < SEG_ACT_NONE || act > SEG_ACT_RELU6 || (act && stat)) return (int)hipErrorInvalidValue;
  if (splits < 1 || (splits > 1 && (!work || stat))) return (int)hipErrorInvalidValue;
  if (bpart && (!by || !bsc || !bsh || !bmu || splits != 1 || act || (ldby & 3))) return (int)hipErrorInvalidValue;
  if (splits > 1) {  // the K ranges actually launched: whole BK chunks, no empty range (launch_igemm)
    const int nk = seg_cdiv((long)ks * ks * Cin, igemm_bk(ks * ks * Cin));
    splits = seg_cdiv(nk, seg_cdiv(nk, splits));
  }
  IgemmArgs a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias;
  a.add = add; a.ldadd = ldadd; a.out = out; a.ldout = ldout; a.stat = stat;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.stride = stride; a.pad = pad; a.K = ks * ks * Cin; a.M = N * Ho * Wo; a.act = act;
  a.part = splits > 1 ? work : nullptr;
  a.xs = xs; a.xb = xb; a.xact = xact;
  a.by = by; a.ldby = ldby; a.bsc = bsc; a.bsh = bsh; a.bmu = bmu; a.bact = bact; a.bpart = bpart;
  a.kcnt = splits > 1 ? kcnt : nullptr;
  a.kspin = seg_combine_spin(kSegCombineSpin);
  g_igemm_ic_used = false;
  if (bpart && !igemm_bnout_tile_ok(a.M, Cout, (int)sizeof(IT))) return (int)hipErrorInvalidValue;
  if (tile < -1 || tile >= (int)(sizeof(kTiles) / sizeof(kTiles[0])) || (tile >= 0 && bpart))
    return (int)hipErrorInvalidValue;
  if (a.M == 0 || Cout == 0) return 0;
  int rc;
  switch (tile >= 0 ? tile : pick_tile(a.M, Cout)) {
    case 0: rc = launch_igemm<128, 128, 64, 64, OT, IT, WB>(a, ks, splits, stream); break;
    case 1: rc = launch_igemm<64, 128, 32, 64, OT, IT, WB>(a, ks, splits, stream); break;
    case 2: rc = launch_igemm<128, 64, 64, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 3: rc = launch_igemm<64, 64, 32, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 4: rc = launch_igemm<128, 96, 32, 96, OT, IT, WB>(a, ks, splits, stream); break;
    case 5: rc = launch_igemm<128, 160, 32, 160, OT, IT, WB>(a, ks, splits, stream); break;
    case 6: rc = launch_igemm<256, 32, 64, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 7: rc = launch_igemm<128, 32, 32, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 8: rc = launch_igemm<128, 128, 64, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 9: rc = launch_igemm<128, 128, 32, 64, OT, IT, WB>(a, ks, splits, stream); break;
    case 10: rc = launch_igemm<256, 128, 64, 64, OT, IT, WB>(a, ks, splits, stream); break;
    case 11: rc = launch_igemm<128, 256, 64, 64, OT, IT, WB>(a, ks, splits, stream); break;
    case 12: rc = launch_igemm<128, 64, 32, 32, OT, IT, WB>(a, ks, splits, stream); break;
    case 13: rc = launch_igemm<256, 64, 64, 32, OT, IT, WB>(a, ks, splits, stream); break;
    default: rc = launch_igemm<64, 128, 32, 32, OT, IT, WB>(a, ks, splits, stream); break;
  }
  if (rc || splits == 1 || g_igemm_ic_used) return rc;
  const long total = (long)a.M * Cout;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((int)std::min<long>(seg_cdiv(total, 256), 4096)), dim3(256), 0,
                     stream, work, splits, (long)a.M, Cout, bias, reinterpret_cast<const float*>(add), ldadd,
                     reinterpret_cast<float*>(out), ldout, act);
  SEG_RET_LAST();
}

}  // namespace
