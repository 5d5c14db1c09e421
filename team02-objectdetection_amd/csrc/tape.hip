// Launch tape: a recorded sequence of C-ABI launches replayed by one host call.
//
// The segamd engine compiles a model into a program and walks it in Python; a training
// step is ~600 kernel launches over two streams, and issuing them one ctypes call at a
// time costs ~10 ms of host time per step -- more than the bf16io step's GPU time.  The
// engine therefore walks the program ONCE per (shape, mode) in recording mode: every
// launch becomes a tape entry (entry-point index + its arguments as 64-bit slots; all
// buffers are persistent, so every pointer is fixed), and later steps replay the tape
// with one seg_tape_run per segment.  Unlike a hipGraph replay, the tape issues the
// same launches on the same two streams (main + weight-gradient side stream), so the
// side-stream overlap of the eager engine is kept.
//
// Entry kinds:
//   CALL     fn = index into kFns (generated from include/segamd.h), args at `arg`,
//            stream 0 = main / 1 = side (passed as the entry point's trailing
//            hipStream_t);
//   RECORD   hipEventRecord(events[fn], stream);
//   WAIT     hipStreamWaitEvent(stream, events[fn]);
//   MEMSET2D hipMemset2DAsync(args[arg] pointer, pitch, value, width, height);
//   STOP     return to the caller (a host callback -- e.g. a DDP bucket all-reduce --
//            runs between segments); fn = callback id.
// Argument slots hold pointers / integers as int64 and floats as their fp32 bit pattern
// in the low 32 bits.  Slots may be patched between replays (seg_tape_set_arg: the
// caller's input / output tensors).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "common.h"
#include "segamd.h"

namespace {

inline float f32_of(uint64_t v) {
  const uint32_t b = (uint32_t)v;
  float f;
  memcpy(&f, &b, 4);
  return f;
}

typedef int (*TrampolineFn)(const uint64_t*, hipStream_t);
struct FnInfo {
  const char* name;
  TrampolineFn fn;
  int nargs;
};

#include "tape_gen.inc"  // kFns[]: one trampoline per launcher of include/segamd.h

constexpr int kNumFns = (int)(sizeof(kFns) / sizeof(kFns[0]));

enum Kind : int32_t { CALL = 0, RECORD = 1, WAIT = 2, MEMSET2D = 3, STOP = 4 };

struct Entry {
  int32_t kind, fn, stream, pad;
  int64_t arg;
};
static_assert(sizeof(Entry) == 24, "host layout of seg_tape entries");

struct Tape {
  std::vector<Entry> e;
  std::vector<uint64_t> a;
  std::vector<hipEvent_t> ev;
  // optional per-entry timing: timed[i] = slot of entry i (-1: untimed); events
  // [replay][slot][begin/end] for up to max_replays replays
  std::vector<int> timed;
  std::vector<hipEvent_t> tev;
  int nslots = 0, max_replays = 0, replay = -1;
};

}  // namespace

SEG_API int seg_tape_fn_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kNumFns; ++i)
    if (strcmp(kFns[i].name, name) == 0) return i;
  return -1;
}

SEG_API int seg_tape_fn_nargs(int fn) { return fn >= 0 && fn < kNumFns ? kFns[fn].nargs : -1; }

SEG_API int seg_tape_create(const void* entries, int n, const void* args, long nargs, int nevents, void** out) {
  if (!out || n < 0 || nargs < 0 || nevents < 0 || (n && !entries) || (nargs && !args)) return (int)hipErrorInvalidValue;
  const Entry* e = static_cast<const Entry*>(entries);
  for (int i = 0; i < n; ++i) {
    const Entry& x = e[i];
    const bool st_ok = x.stream == 0 || x.stream == 1;
    switch (x.kind) {
      case CALL:
        if (x.fn < 0 || x.fn >= kNumFns || !st_ok || x.arg < 0 || x.arg + kFns[x.fn].nargs > nargs)
          return (int)hipErrorInvalidValue;
        break;
      case RECORD:
      case WAIT:
        if (x.fn < 0 || x.fn >= nevents || !st_ok) return (int)hipErrorInvalidValue;
        break;
      case MEMSET2D:
        if (!st_ok || x.arg < 0 || x.arg + 5 > nargs) return (int)hipErrorInvalidValue;
        break;
      case STOP:
        break;
      default:
        return (int)hipErrorInvalidValue;
    }
  }
  Tape* t = new Tape;
  t->e.assign(e, e + n);
  t->a.assign(static_cast<const uint64_t*>(args), static_cast<const uint64_t*>(args) + nargs);
  t->ev.resize(nevents, nullptr);
  for (int i = 0; i < nevents; ++i) {
    const hipError_t rc = hipEventCreateWithFlags(&t->ev[i], hipEventDisableTiming);
    if (rc != hipSuccess) {
      for (int j = 0; j < i; ++j) (void)hipEventDestroy(t->ev[j]);
      delete t;
      return (int)rc;
    }
  }
  t->timed.assign(n, -1);
  *out = t;
  return 0;
}

static void drop_timing(Tape* t) {
  for (hipEvent_t v : t->tev) (void)hipEventDestroy(v);
  t->tev.clear();
  t->timed.assign(t->e.size(), -1);
  t->nslots = t->max_replays = 0;
  t->replay = -1;
}

SEG_API int seg_tape_destroy(void* tape) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t) return 0;
  drop_timing(t);
  for (hipEvent_t v : t->ev) (void)hipEventDestroy(v);
  delete t;
  return 0;
}

// Patch argument slot i (an input / output pointer that changes between replays).
SEG_API int seg_tape_set_arg(void* tape, long i, long value) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t || i < 0 || i >= (long)t->a.size()) return (int)hipErrorInvalidValue;
  t->a[i] = (uint64_t)value;
  return 0;
}

// Time the CALL entries listed in `idx` (n of them) over the next max_replays replays
// (each replay = a run from entry 0); n = 0 switches timing off.
SEG_API int seg_tape_timing(void* tape, const int* idx, int n, int max_replays) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t || n < 0 || max_replays < 0 || (n && !idx)) return (int)hipErrorInvalidValue;
  drop_timing(t);
  if (n == 0 || max_replays == 0) return 0;
  for (int k = 0; k < n; ++k) {
    if (idx[k] < 0 || idx[k] >= (int)t->e.size() || t->e[idx[k]].kind != CALL) return (int)hipErrorInvalidValue;
    t->timed[idx[k]] = k;
  }
  t->tev.resize((size_t)2 * n * max_replays, nullptr);
  for (size_t i = 0; i < t->tev.size(); ++i) {
    const hipError_t rc = hipEventCreate(&t->tev[i]);
    if (rc != hipSuccess) {
      t->tev.resize(i);
      drop_timing(t);
      return (int)rc;
    }
  }
  t->nslots = n;
  t->max_replays = max_replays;
  return 0;
}

// Elapsed milliseconds of the timed entries, out[replay][slot] for the replays done
// (<= max_replays); returns that count, or -hipError.  Call after the work completed.
// The timed launches of replay r as a timeline: out[2k], out[2k + 1] = start and end of timed launch k in ms after
// the start of timed launch 0 (the replay's first timed launch).  Returns 0, or minus a hipError_t.
SEG_API int seg_tape_timeline(void* tape, int r, float* out) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t || !out || r < 0 || r >= std::min(t->replay + 1, t->max_replays) || t->nslots < 1)
    return -(int)hipErrorInvalidValue;
  const size_t b0 = (size_t)r * t->nslots * 2;
  for (int k = 0; k < t->nslots; ++k)
    for (int e = 0; e < 2; ++e) {
      const hipError_t rc = hipEventElapsedTime(&out[2 * k + e], t->tev[b0], t->tev[b0 + 2 * k + e]);
      if (rc != hipSuccess) return -(int)rc;
    }
  return 0;
}

SEG_API int seg_tape_elapsed(void* tape, float* out) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t || !out) return -(int)hipErrorInvalidValue;
  const int done = std::min(t->replay + 1, t->max_replays);
  for (int r = 0; r < done; ++r)
    for (int k = 0; k < t->nslots; ++k) {
      const size_t b = ((size_t)r * t->nslots + k) * 2;
      const hipError_t rc = hipEventElapsedTime(&out[(size_t)r * t->nslots + k], t->tev[b], t->tev[b + 1]);
      if (rc != hipSuccess) return -(int)rc;
    }
  return done;
}

// Run entries [begin, ...) until a STOP or the end.  *stop = index of the STOP entry
// (its callback runs on the host; resume at *stop + 1), or the entry count at the end,
// or the failing entry's index when a launch returns an error (the return value).
SEG_API int seg_tape_run(void* tape, int begin, hipStream_t main, hipStream_t side, int* stop) {
  Tape* t = static_cast<Tape*>(tape);
  if (!t || !stop || begin < 0 || begin > (int)t->e.size()) return (int)hipErrorInvalidValue;
  if (begin == 0) ++t->replay;
  const hipStream_t st[2] = {main, side};
  const int n = (int)t->e.size();
  for (int i = begin; i < n; ++i) {
    const Entry& x = t->e[i];
    hipError_t rc = hipSuccess;
    switch (x.kind) {
      case CALL: {
        const int slot = t->timed[i];
        const bool tm = slot >= 0 && t->replay < t->max_replays;
        const size_t b = ((size_t)t->replay * t->nslots + slot) * 2;
        if (tm) rc = hipEventRecord(t->tev[b], st[x.stream]);
        if (rc == hipSuccess) rc = (hipError_t)kFns[x.fn].fn(&t->a[x.arg], st[x.stream]);
        if (tm && rc == hipSuccess) rc = hipEventRecord(t->tev[b + 1], st[x.stream]);
        break;
      }
      case RECORD:
        rc = hipEventRecord(t->ev[x.fn], st[x.stream]);
        break;
      case WAIT:
        rc = hipStreamWaitEvent(st[x.stream], t->ev[x.fn], 0);
        break;
      case MEMSET2D: {
        const uint64_t* a = &t->a[x.arg];
        rc = hipMemset2DAsync(reinterpret_cast<void*>(a[0]), (size_t)a[1], (int)a[2], (size_t)a[3], (size_t)a[4],
                              st[x.stream]);
        break;
      }
      case STOP:
        *stop = i;
        return 0;
    }
    if (rc != hipSuccess) {
      *stop = i;
      return (int)rc;
    }
  }
  *stop = n;
  return 0;
}
