"""Recording and replay of launch tapes (csrc/tape.hip, include/segamd.h "launch tape").

A `Recorder` collects the C-ABI launches the engine's program walk issues -- entry
point, arguments, stream (main / side), plus event record / stream wait pairs, 2-D
memsets and host-callback stops -- instead of calling them; `Recorder.build()` hands
them to libsegamd as one tape.  `Tape.run()` replays it: one ctypes call per segment
(segments end at host callbacks, e.g. a DataParallel bucket all-reduce).

Argument encoding (64-bit slots): pointers and integers as int64, floats as their
fp32 bit pattern.  Pointer arguments equal to a registered external pointer (the
caller's input / output tensors, which change from step to step) are remembered and
re-patched before every replay (`Tape.bind`).
"""
from __future__ import annotations

import ctypes
import struct
import time

import numpy as np

from . import _lib

CALL, RECORD, WAIT, MEMSET2D, STOP = 0, 1, 2, 3, 4
_ENTRY = np.dtype([("kind", "<i4"), ("fn", "<i4"), ("stream", "<i4"), ("pad", "<i4"), ("arg", "<i8")])
assert _ENTRY.itemsize == 24

_U64 = (1 << 64) - 1
# host-callback stops replayed (DataParallel bucket launches) and the host time spent in them: bench.py's
# world-1 RCCL block reads the per-step figures
STOP_STATS = {"stops": 0, "host_s": 0.0}
_SIG = {}  # entry point -> (fn index, per-argument kind "p" / "i" / "f")


def _signature(name):
    sig = _SIG.get(name)
    if sig is None:
        res, argtypes = _lib.PROTOTYPES[name]
        if not argtypes or argtypes[-1] is not ctypes.c_void_p:
            raise ValueError(f"{name} is not a stream-ordered launcher")
        kinds = []
        for t in argtypes[:-1]:
            kinds.append("f" if t is ctypes.c_float else "p" if t is ctypes.c_void_p else "i")
        idx = _lib.lib().seg_tape_fn_index(name.encode())
        if idx < 0 or _lib.lib().seg_tape_fn_nargs(idx) != len(kinds):
            raise RuntimeError(f"{name}: no launch-tape trampoline (rebuild libsegamd)")
        sig = _SIG[name] = (idx, kinds)
    return sig


def _f32_bits(v) -> int:
    return struct.unpack("<I", struct.pack("<f", float(v)))[0]


class Recorder:
    def __init__(self, streams):
        """streams: {raw hipStream_t handle: 0 (main) or 1 (side)} of the recording walk."""
        self.streams = dict(streams)
        self.entries = []      # (kind, fn, stream, arg offset)
        self.args = []
        self.timers = []       # (entry index, kind tag, flops, op label, entry point) of every launch
        self.label = ""        # the program op being recorded (diagnostics)
        self.callbacks = []
        self.externals = {}    # pointer value -> name
        self.ext_slots = {}    # name -> [arg slot]
        self.n_events = 0

    def external(self, name, ptr):
        """Pointer arguments equal to `ptr` are the caller's tensor `name` (patched per replay)."""
        if ptr:
            self.externals[int(ptr)] = name

    def _stream(self, s):
        try:
            return self.streams[int(s or 0)]
        except KeyError:
            raise RuntimeError("launch on a stream the tape does not know") from None

    def call(self, name, args, timer=None):
        fn, kinds = _signature(name)
        if len(args) != len(kinds) + 1:
            raise TypeError(f"{name}: {len(args)} arguments, expected {len(kinds) + 1}")
        off = len(self.args)
        for i, (k, v) in enumerate(zip(kinds, args)):
            if k == "f":
                self.args.append(_f32_bits(v))
            elif k == "p":
                v = int(v or 0)
                ext = self.externals.get(v)
                if ext is not None:
                    self.ext_slots.setdefault(ext, []).append(off + i)
                self.args.append(v)
            else:
                self.args.append(int(v) & _U64)  # two's complement slot; the trampoline casts back
        self.entries.append((CALL, fn, self._stream(args[-1]), off))
        kind, flops = timer if timer is not None else (name, 0)
        self.timers.append((len(self.entries) - 1, kind, flops, self.label, name))

    def event(self):
        self.n_events += 1
        return self.n_events - 1

    def record(self, ev, stream):
        self.entries.append((RECORD, ev, self._stream(stream), 0))

    def wait(self, stream, ev):
        self.entries.append((WAIT, ev, self._stream(stream), 0))

    def memset2d(self, ptr, pitch, value, width, height, stream):
        off = len(self.args)
        self.args += [int(ptr), int(pitch), int(value), int(width), int(height)]
        self.entries.append((MEMSET2D, 0, self._stream(stream), off))

    def stop(self, callback):
        self.callbacks.append(callback)
        self.entries.append((STOP, len(self.callbacks) - 1, 0, 0))

    def build(self):
        return Tape(self)


class Tape:
    def __init__(self, rec: Recorder):
        ent = np.zeros(len(rec.entries), dtype=_ENTRY)
        for i, (k, f, s, a) in enumerate(rec.entries):
            ent[i] = (k, f, s, 0, a)
        args = np.array(rec.args, dtype=np.uint64) if rec.args else np.zeros(1, np.uint64)
        h = ctypes.c_void_p()
        _lib.call("seg_tape_create", ent.ctypes.data, len(ent), args.ctypes.data, len(rec.args), rec.n_events,
                  ctypes.byref(h))
        self.handle = h
        self.n = len(ent)
        self.callbacks = rec.callbacks
        self.ext_slots = {k: list(v) for k, v in rec.ext_slots.items()}
        self.timers = rec.timers
        self.streams = [s for (_, _, s, _) in rec.entries]  # 0 = main, 1 = side (tools/timeline.py)
        self._stop_ids = {i: f for i, (k, f, _, _) in enumerate(rec.entries) if k == STOP}
        self._timed = None
        self._replays = 0
        self._bound = {}

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            try:
                _lib.lib().seg_tape_destroy(h)
            except Exception:  # interpreter teardown
                pass

    def bind(self, **ptrs):
        """Patch the external pointers (input / output tensors) for the next replay."""
        lib = _lib.lib()
        for name, ptr in ptrs.items():
            ptr = int(ptr or 0)
            if self._bound.get(name) == ptr:
                continue
            for slot in self.ext_slots.get(name, ()):
                rc = lib.seg_tape_set_arg(self.handle, slot, ptr)
                if rc:
                    raise _lib.SegLibError(f"seg_tape_set_arg failed: {rc}")
            self._bound[name] = ptr

    def run(self, main, side):
        lib = _lib.lib()
        stop = ctypes.c_int(0)
        i = 0
        while True:
            rc = lib.seg_tape_run(self.handle, i, main, side, ctypes.byref(stop))
            if rc:
                raise _lib.SegLibError(f"launch tape entry {stop.value} failed: hipError_t {rc}")
            if stop.value >= self.n:
                return
            t0 = time.perf_counter()
            self.callbacks[self._stop_ids[stop.value]]()
            STOP_STATS["stops"] += 1
            STOP_STATS["host_s"] += time.perf_counter() - t0
            i = stop.value + 1

    # timing (bench.py's roofline): HIP events around the selected launches
    def time(self, kinds, replays):
        sel = [t for t in self.timers if kinds is None or t[1] in kinds]
        idx = np.array([t[0] for t in sel], dtype=np.int32)
        _lib.call("seg_tape_timing", self.handle, idx.ctypes.data if len(idx) else None, len(idx), replays)
        self._timed = sel if len(idx) else None
        self._replays = replays

    def timeline(self, r):
        """Replay r's timed launches as [(entry index, start ms, end ms)] after its first timed launch."""
        n = len(self._timed or ())
        out = np.zeros(2 * max(n, 1), dtype=np.float32)
        rc = _lib.lib().seg_tape_timeline(self.handle, r, out.ctypes.data)
        if rc:
            raise _lib.SegLibError(f"seg_tape_timeline failed: {-rc}")
        return [(t[0], float(out[2 * k]), float(out[2 * k + 1])) for k, t in enumerate(self._timed)]

    def elapsed(self, detail=False):
        """[(kind, flops, seconds)] of every timed launch of the replays so far (after a
        sync); detail: [(replay, op label, entry point, kind, flops, seconds)]."""
        if not self._timed:
            return []
        n = len(self._timed)
        out = np.zeros(n * max(self._replays, 1), dtype=np.float32)
        done = _lib.lib().seg_tape_elapsed(self.handle, out.ctypes.data)
        if done < 0:
            raise _lib.SegLibError(f"seg_tape_elapsed failed: {-done}")
        res = []
        for r in range(done):
            for k, (_, kind, flops, label, name) in enumerate(self._timed):
                sec = float(out[r * n + k]) * 1e-3
                res.append((r, label, name, kind, flops, sec) if detail else (kind, flops, sec))
        return res
