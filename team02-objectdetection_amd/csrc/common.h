// Shared helpers for the segamd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC fp32; a "row" is one pixel, `ld` is the row stride in
//     floats (>= channels, lets a producer write straight into a channel slice of a
//     concat buffer -- the reference's torch.cat, src/unet.py:103, becomes free);
//   * every entry point is `extern "C"`, takes plain pointers/ints and the caller's
//     hipStream_t, never allocates, and returns the hipError_t of its launch(es);
//   * wave = 64 lanes; block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>

#define SEG_API extern "C" __attribute__((visibility("default")))

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// ds_read_b64_tr_b16: per 16-lane group, the 4 x 16 bf16 block whose row q / columns
// 4p..4p+3 lane 4q+p addresses, delivered column-major (lane i gets column i, row q
// in element q).  `p` must point into LDS, 8-byte aligned; all 64 lanes active.
__device__ __forceinline__ bf16x4 seg_lds_tr4(const __bf16* p) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 seg_cat8(bf16x4 lo, bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

enum SegAct { SEG_ACT_NONE = 0, SEG_ACT_RELU = 1, SEG_ACT_RELU6 = 2 };

__device__ __forceinline__ float seg_act(float z, int act) {
  if (act == SEG_ACT_RELU) return z > 0.f ? z : 0.f;
  if (act == SEG_ACT_RELU6) return fminf(fmaxf(z, 0.f), 6.f);
  return z;
}

// Derivative mask of the activation at pre-activation value z.  Matches aten's
// threshold_backward (ReLU, inplace => uses the result, y > 0) and
// hardtanh_backward (ReLU6, 0 < y < 6, strict on both sides).
__device__ __forceinline__ float seg_act_mask(float z, int act) {
  if (act == SEG_ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == SEG_ACT_RELU6) return (z > 0.f && z < 6.f) ? 1.f : 0.f;
  return 1.f;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
// bf16 activation storage (the `_bf16io` entry points): 4 channels = one 8-byte access,
// widened to / rounded (RNE) from fp32 -- every kernel computes in fp32 either way.
__device__ __forceinline__ f32x4 ld4(const __bf16* p) {
  return __builtin_convertvector(*reinterpret_cast<const bf16x4*>(p), f32x4);
}
__device__ __forceinline__ void st4(__bf16* p, f32x4 v) {
  *reinterpret_cast<bf16x4*>(p) = __builtin_convertvector(v, bf16x4);
}

// BatchNorm affine + activation of 4 channels: act(y * scale + shift).  The one
// definition used by the BN apply pass and by every consumer that applies it
// lazily on load, so a materialised and a lazily transformed activation are
// bitwise identical.  Branch-free in `act` (a clamp), so it never splits the
// caller's basic block -- a branch between loads stops the scheduler from
// batching them.
__device__ __forceinline__ f32x4 seg_bn_act4(f32x4 v, f32x4 sc, f32x4 sh, int act) {
  const float hi = act == SEG_ACT_RELU6 ? 6.f : __builtin_inff();
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float z = fmaf(v[j], sc[j], sh[j]);
    o[j] = act == SEG_ACT_NONE ? z : fminf(fmaxf(z, 0.f), hi);
  }
  return o;
}

// BatchNorm backward of 4 channels (train mode, through the activation):
//   dY = k1 * (dz - k2 - (y - mean) * k3),  dz = dA * act'(y * scale + shift)
// with k1 = g*invstd, k2 = mean(dz), k3 = mean(dz * xhat) * invstd.  The one
// definition used by the apply pass (bn.hip).
__device__ __forceinline__ f32x4 seg_bnbwd4(f32x4 g, f32x4 v, f32x4 sc, f32x4 sh, f32x4 mu, f32x4 k1, f32x4 k2,
                                            f32x4 k3, int act) {
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float dz = g[j] * seg_act_mask(v[j] * sc[j] + sh[j], act);
    o[j] = k1[j] * (dz - k2[j] - (v[j] - mu[j]) * k3[j]);
  }
  return o;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static inline int seg_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// In-launch hand-off to the block that arrives last (a reduction's finalize folded into
// the reduction's own launch).  The 8 XCDs' L2s are not coherent with each other, so the
// payload (a few partial-sum words per block) is stored and loaded write-through at agent
// scope -- relaxed atomic accesses, which bypass the non-coherent caches (no release or
// acquire fence needed) -- and every storing wave drains its stores before the block's
// one ticket add.  The block whose add returns the last ticket therefore reads every
// other block's payload, whatever the dispatch order or XCD placement; it re-arms the
// counter (zero) for the next launch, so a caller zeroes it once, before the first use.
// Ordering: this is the gfx950 hand-off form "every payload store sc1 (agent
// relaxed atomic store = global_store sc1), every storing wave drained by s_waitcnt vmcnt(0)
// behind a workgroup barrier, one agent-scope atomic add per workgroup, the last adder told
// by the returned ticket, every payload load sc1" -- the measured-valid row of the hand-off
// table in the MI355X microarchitecture guide, which needs no release / acquire fence (an
// acq_rel ticket would add a buffer_wbl2 + buffer_inv, ~3.5 us, to every block's tail).  It
// relies on the sc1 forms staying write-through / L1-bypassing; tests/test_gpu_igemm2.py
// checks the split-K combine (repeated launches bitwise equal, values against float64).
__device__ __forceinline__ void seg_st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float seg_ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Called by every thread of the block after its payload stores; block-uniform result.
// `word`: one int of LDS the block does not otherwise use at this point.
__device__ __forceinline__ bool seg_last_arrival(unsigned* cnt, unsigned nblocks, int* word) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's payload has landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == nblocks - 1;
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    *word = last;
  }
  __syncthreads();
  return *word != 0;
}

// In-launch combine of a split tile (split-K / split hidden range) by its own S <= 32 blocks, with no block
// ever waiting on a block that may not be resident (a plain "wait until all S splits arrived" spin
// hangs when another kernel holds the CUs a peer needs, e.g. two such kernels on two streams).  The tile's
// combine is cut into S pieces, piece z belonging to split block z.  One 64-bit word per tile: bits 0-5 the
// arrivals of the current epoch, 6-37 the pieces given up, 38-63 the epoch.
//   * every block publishes its partial (write-through, drained: the seg_last_arrival form above) and arrives
//     (one atomic add); the arrival that completes the count is the tile's last: it combines its own piece and
//     the pieces given up before it (the mask its add returned), after starting the next epoch (one store: no
//     block can change the word in between -- see below), and never waits for anyone;
//   * a non-last block polls for at most `spin` rounds (0: not at all -- the grid is known not to be co-resident)
//     until the tile is complete (the count reached S, or the epoch moved on); then it combines its own piece;
//   * a block whose poll ran out hands its piece over with a compare-and-swap that sets its mask bit only while the
//     epoch is its own and the count is below S -- so the last arrival's add, which comes later in the word's
//     order, returns the bit; if the tile completed meanwhile it combines its piece itself.
// Every piece is combined exactly once, by a block that saw the tile complete; results do not depend on who.
// No counter needs re-arming (the epoch advances), so a poller can never mistake a later launch for its own.
// cnt: 4 words per tile (the first two used), zero before the first launch.  piece(p): the block's combine of
// piece p (called by all threads, block-uniform p).  word: 2 ints of LDS.
#ifndef SEG_COMBINE_LEGACY
#define SEG_COMBINE_LEGACY 0  // timing experiments only: round 4's unbounded all-arrived spin (hangs when a peer
#endif                        // cannot become resident -- never a default)
template <typename F>
__device__ __forceinline__ void seg_tile_combine(unsigned* cnt, int S, int z, int spin, int* word, F&& piece) {
#if SEG_COMBINE_LEGACY
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)S) __builtin_amdgcn_s_sleep(1);
  }
  __syncthreads();
  piece(z);
  __syncthreads();
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)S - 1) {
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return;
#endif
  typedef unsigned long long u64;
  constexpr u64 kArr = 0x3full;
  constexpr int kMaskShift = 6, kEpochShift = 38;
  u64* w = reinterpret_cast<u64*>(cnt);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial has landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const u64 old = __hip_atomic_fetch_add(w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 ep = old >> kEpochShift;
    bool own = true;
    unsigned extra = 0;
    if ((old & kArr) == (u64)(S - 1)) {  // last arrival: the next epoch, then the pieces given up before us
      extra = (unsigned)(old >> kMaskShift);
      __hip_atomic_store(w, (ep + 1) << kEpochShift, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      auto complete = [&](u64 v) { return (v >> kEpochShift) != ep || (v & kArr) >= (u64)S; };
      bool done = false;
      for (int i = 0; !done && i < spin; ++i) {
        done = complete(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (!done) __builtin_amdgcn_s_sleep(1);
      }
      if (!done) {  // hand the piece to the last arrival, unless it has arrived meanwhile
        u64 cur = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (!complete(cur)) {
          if (__hip_atomic_compare_exchange_strong(w, &cur, cur | (1ull << (kMaskShift + z)), __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            own = false;
            break;
          }
        }
      }
    }
    word[0] = own;
    word[1] = (int)extra;
  }
  __syncthreads();
  const int own = word[0];
  const unsigned extra = (unsigned)word[1];
  if (own) piece(z);
  for (int p = 0; p < S; ++p)
    if ((extra >> p) & 1u) piece(p);
}
// Bound of seg_tile_combine's poll when the grid is co-resident (~1 us per round: a few ms before a block gives
// its piece to the last arrival -- only ever reached when another kernel holds the CUs a peer needs).
constexpr int kSegCombineSpin = 4096;
// The poll bound a launch passes to seg_tile_combine: `automatic`, unless seg_set_combine_spin (csrc/mbconv.hip) set
// an override (tests force 0 / 1: every non-last block hands its piece over).
int seg_combine_spin(int automatic);

// XCD-aware block swizzle (bijective for any nblk): the dispatcher deals blocks
// round-robin over the 8 XCDs (block b and b+8 share an XCD and its 4 MiB L2), so
// remap hardware block b to a logical id such that each XCD walks a CONTIGUOUS
// range of logical ids in dispatch order.  Neighbouring tiles (adjacent image rows
// of an implicit GEMM, all column tiles of one split-K chunk) then share an L2.
// Placement only changes speed, never results.
__device__ __forceinline__ int xcd_swizzle(int b, int nblk) {
  const int xcd = b & 7, pos = b >> 3;
  const int q = nblk >> 3, r = nblk & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// Bilinear source index/weights of output index `dst` along one axis, in aten's
// CPU upsample_bilinear2d float arithmetic (see resample.hip).  Shared by the
// resampling kernels and the fused inference argmax (infer.hip) so both compute
// bitwise the same interpolated logits.
struct Lin {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ Lin lin_index(int dst, int in, float scale, int ac) {
  float src = ac ? scale * (float)dst : fmaxf(scale * ((float)dst + 0.5f) - 0.5f, 0.f);
  int i0 = (int)floorf(src);
  if (i0 > in - 1) i0 = in - 1;
  Lin r;
  r.i0 = i0;
  r.i1 = i0 + (i0 < in - 1 ? 1 : 0);
  r.l1 = fminf(fmaxf(src - (float)i0, 0.f), 1.f);
  r.l0 = 1.f - r.l1;
  return r;
}

// The 2-D bilinear blend of four float4 taps -- one definition for every kernel
// that interpolates logits, so they round identically.
__device__ __forceinline__ f32x4 bilerp4(f32x4 v00, f32x4 v01, f32x4 v10, f32x4 v11, const Lin& lh, const Lin& lw) {
  return lh.l0 * (lw.l0 * v00 + lw.l1 * v01) + lh.l1 * (lw.l0 * v10 + lw.l1 * v11);
}

// The x2 upsample's blend (nn.Upsample bilinear, align_corners=False: seg_upsample_fwd) with one fixed fma
// association -- no contraction left to the compiler -- so any kernel that forms the upsample on load rounds bit for
// bit as the upsample kernel does (round 6's folded decoder conv did; it measured slower and was removed).
__device__ __forceinline__ f32x4 up_blend4(f32x4 v00, f32x4 v01, f32x4 v10, f32x4 v11, float h0, float h1, float w0,
                                           float w1) {
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = __builtin_fmaf(w1, v01[j], w0 * v00[j]);
    const float b = __builtin_fmaf(w1, v11[j], w0 * v10[j]);
    o[j] = __builtin_fmaf(h1, b, h0 * t);
  }
  return o;
}

#define SEG_RET_LAST() return (int)hipGetLastError()

// Compute units of the current device (256 on MI355X; also the answer without a device, so
// host-side slab sizing queried on a CPU-only machine matches the GPU's).
static inline int seg_num_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
    return n;
  (void)hipGetLastError();
  return 256;
}
