// Implicit-GEMM convolution for the deep convs of the bf16io configuration, built for the
// bf16 MFMA's operand rate (the 16-bit igemm_conv_kernel ran the 3x3 family at
// 0.16 of the bf16 MFMA peak, bound by L2 -> LDS operand traffic).
//
//   out[p][co] = sum_{tap, ci} in[p + tap][ci] * W[co][tap][ci] (+ bias) (+ add)
//
// Replaces aten's conv2d / convolution_backward(input) of the decoder's double_conv
// (src/unet.py:58,61: up1/up2 of MobileNetV2UNet, the deep levels of UNet) and of 1x1
// convs, on bf16 activation rows with bf16-packed weights (seg_pack_batch mode | 16).
//
// Structure (one 512-thread block = 8 waves per CU):
//  * block tile 128 x 256 or 256 x 128 (pixels x output channels), wave tile 64 x 64
//    (2 x 2 v_mfma_f32_32x32x16_bf16 accumulators): one 16-byte LDS fragment read per MFMA
//    (4 per 4 MFMAs), half the re-reads of every operand tile in L2 of the 64 x 128 tile;
//  * K steps of 64 bf16 (128-byte operand rows) staged global -> LDS by LDS-DMA
//    (global_load_lds_dwordx4, no VGPR round trip), three LDS buffers, the next two steps'
//    DMA in flight while the current one computes; waits are counted vmcnt + raw
//    s_barrier, so no barrier drains a DMA that is still in flight;
//  * XOR-swizzled operand rows (16-byte chunk c of row r stored at c ^ ((r >> 1) & 7)):
//    the DMA writes LDS lane-linearly, so the permutation is applied to each lane's SOURCE
//    address and undone on the fragment read -- conflict-free ds_read_b128;
//  * the A operand is the implicit im2col of NHWC rows: a 64-deep K step covers at most two
//    filter taps (Cin >= 64), and a lane's 16-byte chunk is one pixel's 8 channels of one
//    tap -- out-of-image taps and rows beyond M read a zero page (no branch);
//  * split-K when the output tiles alone cannot fill the chip: each K slice writes its fp32
//    tile write-through, the slice whose ticket arrives last sums the slices in slice order
//    (deterministic, whatever the arrival order) and runs the epilogue -- no reduce launch;
//  * epilogue as igemm_conv_kernel's: bias, BatchNorm tile partials (sum, M2 about the tile
//    mean) for seg_bn_stats_tiles, addend, one rounding to bf16, 16-byte row stores staged
//    through LDS.
// Round 4: the same pipeline on 4-wave blocks with 128 x 128 / 128 x 64 / 64 x 128 / 64 x 64
// tiles (wave tiles 64x64 / 64x32 / 32x64 / 32x32) for the small-image 1x1 convs of the
// MobileNetV2 encoder (M = 4k-65k rows at bs=32: the generic register-staged kernel keeps one
// K chunk in flight and ran them at 0.4-1.5 TB/s).  (Round 4's lazy-BN fragment transform for
// 1x1 consumers measured slower than the generic kernels and was removed in round 5.)
#include "common.h"

namespace {

constexpr int kBK = 64;             // K step (bf16 elements) = one 128-byte operand row

__device__ __attribute__((aligned(16))) unsigned g_zero_row[4];  // 16 zero bytes

struct Igemm2Args {
  const __bf16* in; long ldin;
  const __bf16* wk; int ldk;        // [Cout][ldk] bf16, k = tap * Cin + ci
  const float* bias;
  const __bf16* add; long ldadd;    // may alias out
  __bf16* out; long ldout;
  float* stat;                      // BN tile partials [tiles_m][2][Cout] or null
  float* slab;                      // split-K: [tiles][splits][BM * BN] fp32
  unsigned* cnt;                    // split-K: [tiles] tickets (zero before the first launch; left zero)
  int N, H, W, Cin, Cout, ks, pad;
  int K, M, nsteps, steps_per_split, splits, tiles_m, tiles_n;
};

#ifndef SEG_IG2_NODMA
#define SEG_IG2_NODMA 0   // diagnostics only (wrong results): skip the operand DMA
#endif
#ifndef SEG_IG2_NOMFMA
#define SEG_IG2_NOMFMA 0  // diagnostics only (wrong results): skip the MFMAs
#endif

__device__ __forceinline__ void dma16(const void* src, char* lds) {
  if (SEG_IG2_NODMA) return;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Workgroup barrier that is also a compiler fence for memory accesses but emits no wait:
// LDS-DMA transfers stay in flight across it (a __syncthreads() would drain them).
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }  // lgkmcnt(0) only

template <int N>
__device__ __forceinline__ void wait_vm() {  // s_waitcnt vmcnt(N), other counters untouched
  static_assert(N >= 0 && N < 64, "vmcnt immediate");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);  // vmcnt is 6 bits, split 3:0 / 15:14
}

template <int BM, int BN, int WM, int WN, int KS>
__global__ __launch_bounds__(64 * (BM / WM) * (BN / WN)) void igemm2_kernel(Igemm2Args a) {
  constexpr int NW = (BM / WM) * (BN / WN), kThreads = 64 * NW, WAVES_N = BN / WN;
  constexpr int MI = WM / 32, NI = WN / 32;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "whole DMA instructions per wave");
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int NA = BM / (8 * NW), NB = BN / (8 * NW);  // DMA instructions per wave per K step
  constexpr int CSR = BN + 4;                // epilogue band row stride (floats)
  constexpr int NSTAGE = 3;                  // LDS buffers: two K steps in flight while one computes
  constexpr int SMEM = NSTAGE * STAGE > WM * CSR * 4 ? NSTAGE * STAGE : WM * CSR * 4;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WAVES_N) * WM, wn0 = (wave % WAVES_N) * WN;
  // a tile's K slices are adjacent logical ids: the same XCD (and L2) combines them
  const int lid = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tile = lid / a.splits, z = lid - tile * a.splits;
  const int tn = tile % a.tiles_n, tm = tile / a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int s_beg = z * a.steps_per_split;
  const int nst = min(a.nsteps - s_beg, a.steps_per_split);

  // ---- per-lane DMA sources.  Instruction j of a tile covers rows 8j .. 8j+7 (1 KB of LDS);
  // wave w issues j = w, w + NW, ...; lane l fills row 8j + (l >> 3), physical chunk l & 7,
  // i.e. logical chunk cl = (l & 7) ^ swz(row).
  const int lrow = lane >> 3, lchk = lane & 7;
  long a_off[NA];
  unsigned a_mask[NA];
  int a_cl[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = 8 * (wave + NW * i) + lrow;
    a_cl[i] = lchk ^ ((row >> 1) & 7);
    const int p = m0 + row;
    const bool ok = p < a.M;
    const int pp = ok ? p : 0;
    const int hw = a.H * a.W;
    const int n = pp / hw, rem = pp - n * hw;
    const int ho = rem / a.W, wo = rem - ho * a.W;
    const int hi0 = ho - KS / 2, wi0 = wo - KS / 2;
    a_off[i] = (((long)n * a.H + hi0) * a.W + wi0) * a.ldin;
    unsigned m = 0;
#pragma unroll
    for (int t = 0; t < KS * KS; ++t) {
      const int hi = hi0 + t / KS, wi = wi0 + t % KS;
      if (ok && (unsigned)hi < (unsigned)a.H && (unsigned)wi < (unsigned)a.W) m |= 1u << t;
    }
    a_mask[i] = m;
  }
  long b_off[NB];
  int b_k[NB];  // this lane's k offset within a step (8 * logical chunk); 2^30: row beyond Cout
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = 8 * (wave + NW * i) + lrow;
    const int cl = lchk ^ ((row >> 1) & 7);
    const int co = n0 + row;
    b_k[i] = co < a.Cout ? 8 * cl : 1 << 30;
    b_off[i] = (long)(co < a.Cout ? co : 0) * a.ldk + 8 * cl;
  }
  // wave-uniform K-step position: tap u_tap, channel u_ci of the step's first k
  const int k_beg = s_beg * kBK;
  int u_tap = k_beg / a.Cin, u_ci = k_beg - u_tap * a.Cin;
  auto tap_off = [&](int t) -> long { return ((long)(t / KS) * a.W + t % KS) * a.ldin; };
  long u_toff0 = tap_off(u_tap), u_toff1 = tap_off(u_tap + 1);
  int k0 = k_beg;

  auto issue = [&](int buf) {  // DMA of the K step at (u_tap, u_ci, k0) into LDS buffer `buf`
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int ci = u_ci + 8 * a_cl[i];
      const bool wrap = ci >= a.Cin;
      const int tap = u_tap + (wrap ? 1 : 0);
      const bool ok = (a_mask[i] >> tap) & 1u;
      const __bf16* src = a.in + a_off[i] + (wrap ? u_toff1 : u_toff0) + (wrap ? ci - a.Cin : ci);
      dma16(ok ? (const void*)src : (const void*)g_zero_row, As + (wave + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const bool ok = k0 + b_k[i] < a.K;
      dma16(ok ? (const void*)(a.wk + b_off[i] + k0) : (const void*)g_zero_row, Bs + (wave + NW * i) * 1024);
    }
    // advance one K step
    k0 += kBK;
    u_ci += kBK;
    while (u_ci >= a.Cin) {
      u_ci -= a.Cin;
      ++u_tap;
      u_toff0 = u_toff1;
      u_toff1 = tap_off(u_tap + 1);
    }
  };

  f32x16 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
    // fragments of the next 16-deep k slice are read while the current slice's MFMAs run
    bf16x8 af[2][MI], bfr[2][NI];
    auto frag = [&](int ks, int st) {
      const int chunk = 2 * ks + fh;  // logical 16-byte chunk of this lane's 8 k values
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int r = wm0 + mi * 32 + fr;
        af[st][mi] = *reinterpret_cast<const bf16x8*>(As + r * 128 + 16 * (chunk ^ ((r >> 1) & 7)));
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int r = wn0 + ni * 32 + fr;
        bfr[st][ni] = *reinterpret_cast<const bf16x8*>(Bs + r * 128 + 16 * (chunk ^ ((r >> 1) & 7)));
      }
    };
    frag(0, 0);
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      if (ks + 1 < kBK / 16) frag(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          if (SEG_IG2_NOMFMA) {
            asm volatile("" ::"v"(af[ks & 1][mi]), "v"(bfr[ks & 1][ni]));
            continue;
          }
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][mi], bfr[ks & 1][ni], acc[mi][ni], 0, 0, 0);
        }
    }
  };

  // ---- K loop: buffer it % 3 holds step it; steps it + 1 and it + 2 stay in flight meanwhile
  // (each step is NA + NB DMA instructions per wave, so "k steps still in flight" is
  // vmcnt(k * (NA + NB)))
  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  if (nst > 2) issue(2);
  for (int it = 0; it < nst; ++it) {
    const int ahead = min(nst - 1 - it, 2);  // steps issued beyond this one
    if (ahead == 2) wait_vm<2 * (NA + NB)>();
    else if (ahead == 1) wait_vm<NA + NB>();
    else wait_vm<0>();
    raw_barrier();                         // every wave's DMA of step `it` has landed
    const int buf = it % NSTAGE;
    compute(buf);
    wait_lgkm0();                          // this wave's fragment reads of `buf` are done
    raw_barrier();                         // ... every wave's: the buffer may be refilled
    if (it + NSTAGE < nst) issue(buf);
  }

  // ---- split-K: publish this slice, the last-arriving slice of the tile combines
  if (a.splits > 1) {
    float* mine = a.slab + ((long)tile * a.splits + z) * (BM * BN);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          seg_st_wt(mine + (((wave * MI + mi) * NI + ni) * 16 + r) * 64 + lane, acc[mi][ni][r]);
    int* word = reinterpret_cast<int*>(smem);
    if (!seg_last_arrival(a.cnt + tile, a.splits, word)) return;
    // sum the slices in slice order (every slice read back, this one included: no
    // data-dependent select between a register and a load)
    f32x16 tot[MI][NI];
    for (int zz = 0; zz < a.splits; ++zz) {
      const float* sl = a.slab + ((long)tile * a.splits + zz) * (BM * BN);
      f32x16 v[MI][NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int r = 0; r < 16; ++r) v[mi][ni][r] = seg_ld_wt(sl + (((wave * MI + mi) * NI + ni) * 16 + r) * 64 + lane);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) tot[mi][ni] = zz == 0 ? v[mi][ni] : tot[mi][ni] + v[mi][ni];
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = tot[mi][ni];
  }

  // ---- epilogue.  C layout of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5).
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    const int col = n0 + wn0 + ni * 32 + fr;
    const float b = (a.bias && col < a.Cout) ? a.bias[col] : 0.f;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] += b;
  }
  __syncthreads();  // the K loop / combine is done with smem
  if (a.stat) {
    // BatchNorm partials of this BM-row tile per output channel: tile sum, then the sum of
    // squared deviations from the tile mean (two passes over the accumulators)
    constexpr int WR = BM / WM;
    float* red = reinterpret_cast<float*>(smem);  // [WR][BN]
    float* tmean = red + WR * BN;                 // [BN]
    const int nrows = min(BM, a.M - m0);
    const int wr = wave / WAVES_N;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int cl = wn0 + ni * 32 + fr;
        const float mu = pass ? tmean[cl] : 0.f;
        float sum = 0.f;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = m0 + wm0 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
            const float d = acc[mi][ni][r] - mu;
            sum += row < a.M ? (pass ? d * d : d) : 0.f;
          }
        sum += __shfl_xor(sum, 32, 64);
        if (lane < 32) red[wr * BN + cl] = sum;
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
  // staged store: per band of WM rows, the owning waves park their accumulators in LDS,
  // then every thread writes 16-byte row vectors (8 bf16 channels) with the addend
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int VPR = BN / 8;
#pragma unroll
  for (int band = 0; band < BM / WM; ++band) {
    __syncthreads();
    if (wm0 == band * WM) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            Cs[(mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh) * CSR + wn0 + ni * 32 + fr] = acc[mi][ni][r];
    }
    __syncthreads();
    for (int v = tid; v < WM * VPR; v += kThreads) {
      const int rr = v / VPR, cv = (v - rr * VPR) * 8;
      const int row = m0 + band * WM + rr, col = n0 + cv;
      if (row >= a.M || col >= a.Cout) continue;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(&Cs[rr * CSR + cv + j]);
        o[j] = q[0]; o[j + 1] = q[1]; o[j + 2] = q[2]; o[j + 3] = q[3];
      }
      __bf16* dst = a.out + (long)row * a.ldout + col;
      const __bf16* ad = a.add ? a.add + (long)row * a.ldadd + col : nullptr;
      if (col + 8 <= a.Cout) {  // 16-byte aligned: ldout, ldadd and col are multiples of 8
        if (ad) {
          const bf16x8 q = *reinterpret_cast<const bf16x8*>(ad);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += (float)q[j];
        }
        const f32x4 lo = {o[0], o[1], o[2], o[3]}, hi = {o[4], o[5], o[6], o[7]};
        *reinterpret_cast<bf16x8*>(dst) = seg_cat8(__builtin_convertvector(lo, bf16x4),
                                                   __builtin_convertvector(hi, bf16x4));
      } else {
        for (int j = 0; j < 8 && col + j < a.Cout; ++j) {
          float x = o[j];
          if (ad) x += (float)ad[j];
          dst[j] = static_cast<__bf16>(x);
        }
      }
    }
  }
}

struct Tile2 {
  int bm, bn, wm, wn;
  float eff;  // relative per-step efficiency (LDS fragment reads per MFMA, barrier share)
};
// 0, 1: the 8-wave tiles of round 3 (deep 3x3 convs); 2-5: 4-wave tiles (round 4)
constexpr Tile2 kT2[] = {{128, 256, 64, 64, 1.00f}, {256, 128, 64, 64, 1.00f}, {128, 128, 64, 64, 0.95f},
                         {128, 64, 64, 32, 0.90f},  {64, 128, 32, 64, 0.90f},  {64, 64, 32, 32, 0.80f}};
constexpr int kNT2 = sizeof(kT2) / sizeof(kT2[0]);

int g_ig2_force = -1;      // tuning hooks (seg_igemm2_force_tile, seg_igemm2_tune)
int g_ig2_target = 512;    // 4-wave tiles: split-K up to this many blocks ...
int g_ig2_minsteps = 3;    // ... keeping at least this many 64-deep K steps per slice

struct Plan2 {
  int tile;       // index into kT2, -1: not applicable
  int bm, bn, tiles_m, tiles_n, splits, nsteps, steps_per_split;
  long work_floats;
};

#ifndef SEG_IG2_SMALL
#define SEG_IG2_SMALL 1  // the 4-wave tiles (0: round-3 plan, 8-wave tiles only)
#endif

// Tile choice.  Round-3 rule first (8-wave tiles at >= 85 % utilisation, split-K to ~256
// blocks) -- it keeps the deep 3x3 convs' launches as they were.  Otherwise (or when the
// 8-wave tiles would leave the chip mostly idle) the 4-wave tiles are scored by utilisation
// x efficiency x fill (fill: >= 2 blocks per CU counting split-K slices, which pay a slab
// round trip each), for the small-image 1x1 / 3x3 convs.
Plan2 plan2(long M, int Cout, int Cin, int ks, int force = -1) {
  Plan2 p{};
  p.tile = -1;
  const long K = (long)ks * ks * Cin;
  if (M < 1 || Cout < 1 || (Cin & 7) || (ks != 1 && ks != 3) || (ks == 3 && Cin < 64)) return p;
  const int nsteps = (int)((K + kBK - 1) / kBK);
  auto util = [&](int c) {
    const long tm = (M + kT2[c].bm - 1) / kT2[c].bm, tn = (Cout + kT2[c].bn - 1) / kT2[c].bn;
    return (double)M * Cout / ((double)tm * kT2[c].bm * tn * kT2[c].bn);
  };
  auto splits_for = [&](int c) {
    // the 8-wave tiles: split-K to ~256 blocks with >= 8 K steps per slice (round 3); the 4-wave
    // tiles of the small images: to ~g_ig2_target blocks with >= g_ig2_minsteps steps per slice
    const long tiles = ((M + kT2[c].bm - 1) / kT2[c].bm) * ((Cout + kT2[c].bn - 1) / kT2[c].bn);
    const long target = c < 2 ? 256 : g_ig2_target;
    const long minst = c < 2 ? 8 : g_ig2_minsteps;
    int s = 1;
    if (tiles < target) s = (int)std::min<long>(std::min<long>((target + tiles - 1) / tiles, nsteps / minst), 8);
    return std::max(s, 1);
  };
  int best = -1;
  if (force >= 0 && force < kNT2) {
    best = force;
  } else {
    double bu = 0.0;
    for (int c = 0; c < 2; ++c)
      if (Cin >= 64 && util(c) > bu + 1e-9) { bu = util(c); best = c; }
    const bool big_ok = best >= 0 && bu >= 0.85;
    if (!big_ok) best = -1;
    if (SEG_IG2_SMALL) {
      const long tiles_big = big_ok ? ((M + kT2[best].bm - 1) / kT2[best].bm) * ((Cout + kT2[best].bn - 1) / kT2[best].bn)
                                    : 0;
      if (!big_ok || tiles_big < 128) {
        double bs = 0.0;
        int bsmall = -1;
        for (int c = 2; c < kNT2; ++c) {
          const long tiles = ((M + kT2[c].bm - 1) / kT2[c].bm) * ((Cout + kT2[c].bn - 1) / kT2[c].bn);
          const int sp = splits_for(c);
          const double fill = std::min(1.0, (double)(tiles * sp) / 512.0) / (sp > 1 ? 1.0 + 0.05 * sp : 1.0);
          const double score = util(c) * kT2[c].eff * fill;
          if (score > bs + 1e-9) { bs = score; bsmall = c; }
        }
        if (bsmall >= 0 && util(bsmall) >= 0.6) best = bsmall;
      }
    }
  }
  if (best < 0) return p;
  p.tile = best;
  p.bm = kT2[best].bm;
  p.bn = kT2[best].bn;
  p.tiles_m = (int)((M + p.bm - 1) / p.bm);
  p.tiles_n = (Cout + p.bn - 1) / p.bn;
  p.nsteps = nsteps;
  const long tiles = (long)p.tiles_m * p.tiles_n;
  const int s = splits_for(best);
  p.steps_per_split = (p.nsteps + s - 1) / s;
  p.splits = (p.nsteps + p.steps_per_split - 1) / p.steps_per_split;  // no empty slice
  p.work_floats = p.splits > 1 ? tiles + tiles * p.splits * (long)p.bm * p.bn : 0;
  return p;
}

}  // namespace

// Tuning hook: the 4-wave tiles' split-K targets (blocks, minimum K steps per slice); <= 0 keeps a value.
SEG_API int seg_igemm2_tune(int target_blocks, int min_steps) {
  if (target_blocks > 0) g_ig2_target = target_blocks;
  if (min_steps > 0) g_ig2_minsteps = min_steps;
  return 0;
}

// Tuning hook: force seg_conv_igemm2_bf16io's tile (index into its table; -1 = the plan).
SEG_API int seg_igemm2_force_tile(int t) {
  g_ig2_force = t;
  return 0;
}

// Plan of seg_conv_igemm2_bf16io for an M x Cout GEMM over K = ks*ks*Cin: out[0] = tile
// rows (the BN partials' row tiles), out[1] = row tiles, out[2] = split-K slices,
// out[3] = workspace floats (tickets + slice tiles; 0 when unsplit).  Returns 1 when the
// kernel applies (Cin % 8 == 0; 3x3: Cin >= 64; little tile padding), else 0.
SEG_API int seg_conv_igemm2_plan(long M, int Cout, int Cin, int ks, long* out) {
  const Plan2 p = plan2(M, Cout, Cin, ks, g_ig2_force);
  if (p.tile < 0) return 0;
  if (out) {
    out[0] = p.bm;
    out[1] = p.tiles_m;
    out[2] = p.splits;
    out[3] = p.work_floats;
  }
  return 1;
}

static int igemm2_impl(const __bf16* in, long ldin, int N, int H, int W, int Cin, const __bf16* wk, int ldk,
                       const float* bias, __bf16* out, long ldout, int Cout, int ks, const __bf16* add, long ldadd,
                       float* stat, float* work, hipStream_t stream) {
  const long M = (long)N * H * W;
  const Plan2 p = plan2(M, Cout, Cin, ks, g_ig2_force);
  if (p.tile < 0 || (ldin & 7) || (ldk & 7) || (ldout & 7) || (add && (ldadd & 7)) || ldk < ks * ks * Cin ||
      ((uintptr_t)in & 15) || ((uintptr_t)wk & 15) || ((uintptr_t)out & 15) || (add && ((uintptr_t)add & 15)) ||
      (p.splits > 1 && !work) || M > 0x7fffffffL)
    return (int)hipErrorInvalidValue;
  Igemm2Args a;
  a.in = in; a.ldin = ldin; a.wk = wk; a.ldk = ldk; a.bias = bias; a.add = add; a.ldadd = ldadd;
  a.out = out; a.ldout = ldout; a.stat = stat;
  a.cnt = p.splits > 1 ? reinterpret_cast<unsigned*>(work) : nullptr;
  a.slab = p.splits > 1 ? work + (long)p.tiles_m * p.tiles_n : nullptr;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ks = ks; a.pad = (ks - 1) / 2;
  a.K = ks * ks * Cin; a.M = (int)M; a.nsteps = p.nsteps; a.steps_per_split = p.steps_per_split;
  a.splits = p.splits; a.tiles_m = p.tiles_m; a.tiles_n = p.tiles_n;
  const int grid = p.tiles_m * p.tiles_n * p.splits;
#define SEG_I2(BM, BN, WM, WN)                                                                                   \
  do {                                                                                                          \
    constexpr int nt = 64 * (BM / WM) * (BN / WN);                                                              \
    if (ks == 3) hipLaunchKernelGGL((igemm2_kernel<BM, BN, WM, WN, 3>), dim3(grid), dim3(nt), 0, stream, a); \
    else hipLaunchKernelGGL((igemm2_kernel<BM, BN, WM, WN, 1>), dim3(grid), dim3(nt), 0, stream, a);            \
  } while (0)
  switch (p.tile) {
    case 0: SEG_I2(128, 256, 64, 64); break;
    case 1: SEG_I2(256, 128, 64, 64); break;
    case 2: SEG_I2(128, 128, 64, 64); break;
    case 3: SEG_I2(128, 64, 64, 32); break;
    case 4: SEG_I2(64, 128, 32, 64); break;
    default: SEG_I2(64, 64, 32, 32); break;
  }
#undef SEG_I2
  SEG_RET_LAST();
}

// out = conv(in, W) (+bias) (+add), stride 1, pad (ks-1)/2, bf16 rows in / add / out,
// bf16 packed weights (ldk % 8 == 0); fp32 accumulation, one rounding on the store.
// stat (optional): BN partials [row tiles][2][Cout] of the plan's tile rows.  work: the
// plan's workspace (zero it once before its first use; every call leaves its tickets zero).
SEG_API int seg_conv_igemm2_bf16io(const __bf16* in, long ldin, int N, int H, int W, int Cin, const __bf16* wk,
                                   int ldk, const float* bias, __bf16* out, long ldout, int Cout, int ks,
                                   const __bf16* add, long ldadd, float* stat, float* work, hipStream_t stream) {
  return igemm2_impl(in, ldin, N, H, W, Cin, wk, ldk, bias, out, ldout, Cout, ks, add, ldadd, stat, work, stream);
}
