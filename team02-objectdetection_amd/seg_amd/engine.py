"""The HIP execution engine for MobileNetV2UNet / UNet / LightUNet.

A model (seg_amd/unet.py) is compiled once per input shape into a *program*:
a flat list of ops over named NHWC fp32 buffers.  The forward walks the list;
the backward walks it in reverse with mirrored gradient buffers.  The whole
network is one torch.autograd.Function, so `loss.backward()` works exactly as
in the reference loop (src/train.py:36-39) while every FLOP runs in
libsegamd.so (include/segamd.h).

Buffers / layout (DESIGN.md "Data layout in HBM"):
  * every activation is a [pixels][ld] row tensor, ld = round_up(C, 4);
  * the decoder concat `torch.cat([skip, up(x)], 1)` (src/unet.py:103) is a
    single buffer: the encoder writes its skip output into channels [0, Cs),
    the bilinear upsample writes [Cs, Cs+Cu) -- no copy;
  * each conv keeps its raw (pre-BN) output `y` for the BN backward; the
    normalised/activated output is the next op's input.
Gradients of a buffer region are written by the first consumer in reverse
order and accumulated by later ones; a residual (InvertedResidual
`x + conv(x)`) hands its upstream gradient to the first writer of dx as a
fused addend.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch
from torch import nn

from ._lib import call, query as _query

# Host-only size / plan queries of the C ABI are pure functions of their integer
# arguments: memoised, so a training step does not pay a ctypes call for each of them.
# (Not the implicit GEMM's tile-dependent queries -- seg_conv_igemm_tiles / _row_tiles / _bnout_ok, igemm2's
# plan: a forced tile (force_igemm_tile) changes them)
_PURE_QUERIES = {"seg_chan_workspace_floats", "seg_conv_wgrad_splits", "seg_conv_wgrad_splits_bf16", "seg_dw_wgrad_blocks",
                 "seg_conv_igemm_splits", "seg_ce_workspace_floats", "seg_conv_wino_row_tiles", "seg_conv_wino_tile_rows",
                 "seg_conv_halo_row_tiles", "seg_conv_wino_wgrad_splits", "seg_conv_wino_wgrad16_splits",
                 "seg_mbconv_ok"}
_QCACHE = {}


def query(name, *args):
    if name not in _PURE_QUERIES:
        return _query(name, *args)
    key = (name, args)
    r = _QCACHE.get(key)
    if r is None:
        r = _QCACHE[key] = _query(name, *args)
    return r
from .mobilenet import ConvBNReLU6, InvertedResidual

ACT_NONE, ACT_RELU, ACT_RELU6 = 0, 1, 2
IGNORE_INDEX = -100
_ROW_TILES = {}  # (M, Cout) -> (row tiles, tile height) of seg_conv_igemm


_IG2 = {}  # (M, Cout, Cin, ks) -> (tile rows, row tiles, splits, workspace floats) or None


def _pw_pick(op, v: int):
    """(forward, data gradient) of a 1x1 conv on the thin-K kernel (seg_conv_pw): K <= 32 with
    K % 8 == 0, N <= 192, rows in 16-byte vectors of v elements."""
    if not PW or op.kind != "igemm" or op.ks != 1 or op.stride != 1:
        return False, False
    i, y = op.inp, op.y
    # measured per launch (bf16io, tools/tapeprof.py): 1.2-1.8x faster than the implicit GEMM on the
    # full- and half-resolution layers, 5-20 % slower on the 65k-row ones (one tile per block)
    if y.M < PW_MIN_ROWS:
        return False, False
    rows = lambda *ts: all(t.ld % v == 0 and t.off % v == 0 for t in ts)  # noqa: E731
    fwd = 8 <= op.cin_pad <= 32 and op.cin_pad % 8 == 0 and op.cout <= 192 and rows(i, y)
    kin = r4(op.cout)
    bwd = not op.first and 8 <= kin <= 32 and kin % 8 == 0 and op.cin <= 192 and rows(i) and kin % v == 0
    return fwd, bwd


def igemm2_plan(M: int, cout: int, cin: int, ks: int):
    """seg_conv_igemm2_plan (memoised): None when the deep-conv kernel does not apply."""
    key = (M, cout, cin, ks)
    if key not in _IG2:
        out = (ctypes.c_long * 4)()
        ok = query("seg_conv_igemm2_plan", M, cout, cin, ks, ctypes.addressof(out))
        _IG2[key] = tuple(out) if ok else None
    return _IG2[key]


def force_tiles(igemm: int | None = None, igemm2: int | None = None) -> None:
    """Tuning hook: force the implicit GEMM's (seg_igemm_force_tile) and / or igemm2's (seg_igemm2_force_tile) tile
    table entry (-1 = the cost model again), and drop every memoised tile-dependent plan (row tiles, igemm2 plans) so
    the next program walk sizes its workspaces for the tile actually launched.  Plans recorded before the
    change keep their tapes: release_plans() / a fresh Predictor re-record them."""
    if igemm is not None:
        _query("seg_igemm_force_tile", int(igemm))
    if igemm2 is not None:
        _query("seg_igemm2_force_tile", int(igemm2))
    _ROW_TILES.clear()
    _IG2.clear()
    _QCACHE.clear()


def r8(c: int) -> int:
    return (c + 7) & ~7


def r4(c: int) -> int:
    return (c + 3) & ~3


class KernelTimer:
    """Opt-in HIP-event timing of the dense MFMA convolution launches (used by
    bench.py for the roofline figure).  Each timed launch is bracketed by two
    events on the stream it runs on (torch's current stream)."""

    def __init__(self, kinds=None, max_replays=64):
        self.records = []  # (kind, flops, start_event, end_event) of immediate launches
        # only these launch kinds are bracketed (None: all): every event pair is a marker
        # packet on the queue, ~3 % of the step when all ~130 conv launches are timed
        self.kinds = kinds
        # launch tapes armed for this timer (Plan._arm_timer): each times its selected
        # entries over up to max_replays replays with events inside libsegamd
        self.tapes = []
        self.max_replays = max_replays

        self.collected = []

    def collect(self, tape):
        """Move a tape's timings into this timer (the tape is being re-armed)."""
        if tape in self.tapes:
            torch.cuda.synchronize()
            self.collected += tape.elapsed()
            self.tapes.remove(tape)

    def elapsed(self):
        """[(kind, flops, seconds)] -- call after synchronising."""
        out = [(k, f, a.elapsed_time(b) * 1e-3) for k, f, a, b in self.records] + self.collected
        for t in self.tapes:
            out += t.elapsed()
        return out


TIMER: KernelTimer | None = None

def _stat_ptrs(st, C):
    """Device pointers of the mean / invstd / scale / shift rows of a saved [4][C] BN
    statistics tensor (no per-call view tensors on the host path)."""
    b = st.data_ptr()
    return b, b + 4 * C, b + 8 * C, b + 12 * C


def _timed_call(kind, flops, name, *args):
    if TIMER is None or (TIMER.kinds is not None and kind not in TIMER.kinds):
        return call(name, *args)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    call(name, *args)
    b.record()
    TIMER.records.append((kind, flops, a, b))


class Act:
    """NHWC view: channels [off, off+C) of buffer `buf` ([N*H*W][ld])."""
    __slots__ = ("buf", "off", "ld", "C", "N", "H", "W")

    def __init__(self, buf, off, ld, C, N, H, W):
        self.buf, self.off, self.ld, self.C, self.N, self.H, self.W = buf, off, ld, C, N, H, W

    @property
    def M(self):
        return self.N * self.H * self.W

    def key(self):
        return (self.buf, self.off, self.C)

    def slice(self, off, C):
        return Act(self.buf, self.off + off, self.ld, C, self.N, self.H, self.W)


# ----------------------------------------------------------------------------- ops

IMAGE = "image"   # buffer holding the NHWC4 copy of the NCHW model input


class ConvOp:
    """conv (igemm | dw) -> [BN -> act (+residual)]."""

    def __init__(self, kind, conv: nn.Conv2d, bn, act, inp, out, y, res, xform=None):
        self.kind, self.conv, self.bn, self.act = kind, conv, bn, act
        self.inp, self.out, self.y, self.res = inp, out, y, res
        # lazy BN: this op's BN + act is applied by its (only) consumer on load, out is y;
        # xform: the producer op whose BN + act this op applies to its input on load
        self.lazy = False
        self.xform = xform
        # packed weights (Program.pack): forward [Cout][ldk_f] (None: a 1x1 conv uses the
        # weight as is), data gradient [Cin][ldk_d]; depthwise: wk_f = [9][C]
        self.wk_f = self.wk_d = None
        self.ldk_f = self.ldk_d = 0
        # BN-folded inference weights (Program.fold): fk [Cout][Cin/g][ks][ks], fb [r4(Cout)], fk_pack
        self.fk = self.fb = self.fk_pack = None
        # Winograd F(2x2,3x3) (seg_conv_wino) for the forward / data gradient, chosen by
        # seg_conv_wino_pick at pack time; U_f [16][Cout][cin_pad], U_d [16][Cin][r4(Cout)]
        self.wino_f = self.wino_d = self.wino_w = False
        self.wino_ff = self.wino_fd = False  # ... on the fused kernel (seg_conv_wino_fused: no M workspace)
        # LDS-halo direct 3x3 (seg_conv_halo) for the forward / data gradient of narrow convs
        self.halo_f = self.halo_d = False
        self.w2 = False  # weight gradient on seg_conv_wgrad2_bf16io (narrow bf16io 3x3)
        # bf16 math (Program.math == "bf16"): seg_conv_igemm_bf16 / seg_conv_wgrad_bf16
        self.bf = False
        # bf16io: wk_f / wk_d packed as bf16 for seg_conv_igemm_bf16io_w16 (Program._build_pack)
        self.w16_f = self.w16_d = False
        # bf16io deep convs on seg_conv_igemm2_bf16io (igemm2_plan tuples, chosen at pack time)
        self.ig2_f = self.ig2_d = None
        # thin-K 1x1 forward / data gradient on seg_conv_pw (K <= 32, N <= 192; chosen at pack time)
        self.pw_f = self.pw_d = False
        self.ks = conv.kernel_size[0]
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.cin = conv.in_channels
        self.cin_pad = r4(self.cin)  # GEMM K runs are float4 channel groups (the image: 3 -> 4)
        self.cout = conv.out_channels
        self.first = inp.buf == IMAGE  # no data gradient for the model input

    def flops(self) -> int:
        """Algorithmic FLOPs of this conv's forward (2 * MACs; dgrad and wgrad each equal it)."""
        groups = self.conv.groups
        return 2 * self.y.M * self.cout * (self.cin // groups) * self.ks * self.ks

    def params(self):
        ps = [self.conv.weight]
        if self.conv.bias is not None:
            ps.append(self.conv.bias)
        if self.bn is not None:
            ps += [self.bn.weight, self.bn.bias]
        return ps

    # -- forward
    def forward(self, rt):
        s, y = rt.stream, self.y
        w = self.conv.weight
        bias = self.conv.bias.data_ptr() if self.conv.bias is not None else None
        if self.kind == "dw":
            i = self.inp
            stat = None
            rt.call(rt.k("seg_dw_fwd"), rt.ptr(i), i.ld, i.N, i.H, i.W, i.C, *self._in_xform(rt),
                    self.wk_f.data_ptr(), rt.ptr(y), y.ld, y.H, y.W, self.stride, s)
        else:
            i = self.inp
            if self.wk_f is None:
                ldk, wk_ptr = self.cin, w.data_ptr()  # [Cout][Cin][1][1] already is the packed layout
            else:
                ldk, wk_ptr = self.ldk_f, self.wk_f.data_ptr()  # packed by Program.pack at the step start
            stat = None
            if self.bn is not None and rt.training:  # BN statistics fused into the conv epilogue
                if self.pw_f:
                    tile_rows, ntiles = 128, query("seg_conv_pw_row_tiles", y.M)
                elif self.ig2_f is not None:
                    tile_rows, ntiles = self.ig2_f[0], self.ig2_f[1]
                elif self.wino_f:
                    ntiles = query("seg_conv_wino_row_tiles", y.N, y.H, y.W)
                    tile_rows = query("seg_conv_wino_tile_rows")
                elif self.halo_f:
                    ntiles, tile_rows = query("seg_conv_halo_row_tiles", y.N, y.H, y.W), 256
                else:
                    ntiles, tile_rows = rt.row_tiles(y.M, self.cout)
                stat = rt.tmp(ntiles * 2 * self.cout)
            statp = stat.data_ptr() if stat is not None else None
            if self.pw_f:  # thin-K 1x1 (its producer's lazy BN, if any, on load)
                rt.tcall("igemm1_fwd", self.flops(), rt.k("seg_conv_pw"), rt.ptr(i), i.ld, y.M, self.cin_pad, wk_ptr,
                         ldk, bias, rt.ptr(y), y.ld, self.cout, None, 0, statp, *self._in_xform(rt), s)
            elif self.halo_f:
                name = rt.k("seg_conv_halo") + ("_w16" if self.w16_f else "")
                rt.tcall("igemm3_fwd", self.flops(), name, rt.ptr(i), i.ld, i.N, i.H, i.W, self.cin_pad,
                         wk_ptr, ldk, bias, rt.ptr(y), y.ld, self.cout, None, 0, statp, s)
            elif self.wino_ff and query("seg_conv_wino_fused_ok", i.N, i.H, i.W, i.ld):
                rt.tcall("wino3_fwd", self.flops(), "seg_conv_wino_fused", rt.ptr(i), i.ld, i.N, i.H, i.W,
                         self.cin_pad, self.wk_wf.data_ptr(), self.cin_pad, bias, rt.ptr(y), y.ld, self.cout, None, 0,
                         statp, s)
            elif self.wino_f:
                work = rt.tmp(16 * (y.M // 4) * self.cout)
                rt.tcall("wino3_fwd", self.flops(), "seg_conv_wino", rt.ptr(i), i.ld, i.N, i.H, i.W, self.cin_pad,
                            self.wk_wf.data_ptr(), self.cin_pad, bias, rt.ptr(y), y.ld, self.cout, None, 0, statp,
                            work.data_ptr(), s)
            elif self.ig2_f is not None:  # bf16io LDS-DMA implicit GEMM (deep 3x3 convs)
                work = rt.tmp(self.ig2_f[3], zero=True)
                rt.tcall(f"igemm{self.ks}_fwd", self.flops(), "seg_conv_igemm2_bf16io", rt.ptr(i),
                         i.ld, i.N, i.H, i.W, self.cin_pad, wk_ptr, ldk, bias, rt.ptr(y), y.ld, self.cout, self.ks, None, 0,
                         statp, work.data_ptr(), s)
            elif self.xform is not None:  # a conv applying its producer's lazy BN on load
                name = "seg_conv_igemm_bf16io_xf" if rt.io else "seg_conv_igemm_bf16_xf" if self.bf else "seg_conv_igemm_xf"
                if rt.io and self.w16_f:
                    name += "_w16"
                rt.tcall(f"igemm{self.ks}_fwd", self.flops(), name, rt.ptr(i), i.ld, i.N, i.H, i.W, self.cin_pad, wk_ptr, ldk,
                         bias, rt.ptr(y), y.ld, y.H, y.W, self.cout, self.ks, self.stride, self.pad, None, 0, statp,
                         *self._in_xform(rt), s)
            elif rt.io:
                rt.tcall(f"igemm{self.ks}_fwd", self.flops(),
                         "seg_conv_igemm_bf16io_w16" if self.w16_f else "seg_conv_igemm_bf16io", rt.ptr(i), i.ld, i.N, i.H,
                            i.W, self.cin_pad, wk_ptr, ldk, bias, rt.ptr(y), y.ld, y.H, y.W, self.cout, self.ks,
                            self.stride, self.pad, None, 0, statp, s)
            elif self.bf:
                rt.tcall(f"igemm{self.ks}_fwd", self.flops(), "seg_conv_igemm_bf16", rt.ptr(i), i.ld, i.N, i.H,
                            i.W, self.cin_pad, wk_ptr, ldk, bias, rt.ptr(y), y.ld, y.H, y.W, self.cout, self.ks,
                            self.stride, self.pad, None, 0, statp, ACT_NONE, None, 1, s)
            else:
                rt.tcall(f"igemm{self.ks}_fwd", self.flops(), "seg_conv_igemm", rt.ptr(i), i.ld, i.N, i.H, i.W,
                            self.cin_pad, wk_ptr, ldk, bias, rt.ptr(y), y.ld, y.H, y.W, self.cout, self.ks,
                            self.stride, self.pad, None, 0, statp, s)
        if self.bn is None:
            return
        bn, C, M = self.bn, self.cout, y.M
        st = torch.empty(4 * C, device=rt.device, dtype=torch.float32)
        mean, invstd, scale, shift = _stat_ptrs(st, C)
        if rt.training:
            if bn.momentum is None:
                raise NotImplementedError("BatchNorm2d(momentum=None) (cumulative average) is not supported")
            rm = bn.running_mean.data_ptr() if bn.track_running_stats else None
            rv = bn.running_var.data_ptr() if bn.track_running_stats else None
            nbt = bn.num_batches_tracked.data_ptr() if bn.track_running_stats else None
            if self.kind == "dw" and stat is None:
                work = rt.tmp(query("seg_chan_workspace_floats", M, C))
                rt.call(rt.k("seg_bn_stats"), rt.ptr(y), y.ld, M, C, bn.weight.data_ptr(), bn.bias.data_ptr(), bn.eps,
                     bn.momentum, rm, rv, nbt, work.data_ptr(), mean, invstd,
                     scale, shift, s)
            else:
                # many-tile layers: 16 tiles merged per row before the per-channel finalize (SEG_BN_MERGE=0: direct)
                nw = query("seg_bn_stats_tiles_work_floats", ntiles, C) if BN_MERGE else 0
                ws = (rt.tmp(nw).data_ptr(),) if nw else ()
                rt.call("seg_bn_stats_tiles_ws" if nw else "seg_bn_stats_tiles", stat.data_ptr(), ntiles, tile_rows, M,
                        C, bn.weight.data_ptr(), bn.bias.data_ptr(), bn.eps, bn.momentum, rm, rv, nbt, mean, invstd,
                        scale, shift, *ws, s)
        else:
            rt.call("seg_bn_eval_coef", bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                 bn.running_var.data_ptr(), bn.eps, C, scale, shift, s)
        rt.saved[id(self)] = st
        if self.lazy:
            return
        o, r = self.out, self.res
        rt.call(rt.k("seg_bn_apply"), rt.ptr(y), y.ld, M, C, scale, shift, self.act,
             rt.ptr(r) if r is not None else None, r.ld if r is not None else 0, rt.ptr(o), o.ld, s)

    # -- inference (BatchNorm folded into the conv: Program.fold)
    def forward_folded(self, rt):
        """act(conv(x, W') + b') (+ residual) in one launch; W', b' from seg_bn_fold_batch.
        A lazy producer writes its activated output into its `y` buffer (= `out`), so its
        depthwise consumer reads it without the on-load BN transform."""
        s, i, o = rt.stream, self.inp, self.out
        act = self.act if self.bn is not None else ACT_NONE
        if self.kind == "dw":
            rt.call("seg_dw_fwd_bias_act", rt.ptr(i), i.ld, i.N, i.H, i.W, i.C, self.fk_pack.data_ptr(),
                 self.fb.data_ptr(), act, rt.ptr(o), o.ld, o.H, o.W, self.stride, s)
            return
        if self.fk_pack is None:
            ldk, wk = self.cin, self.fk.data_ptr()
        else:
            ldk, wk = self.ldk_f, self.fk_pack.data_ptr()
        r = self.res
        bias = self.fb.data_ptr() if self.fb is not None else None
        M = o.N * o.H * o.W
        # (splits, tile, output tiles) of seg_conv_igemm_plan_b1; split-K combined inside the launch
        # (seg_conv_igemm_*_ic); workspace and tile counters persistent across graph replays (allocated by the
        # warm-up launch, before any capture)
        bufs = rt._mb.get(("ic", id(self)))
        if bufs is None:
            plan = (ctypes.c_int * 3)()
            query("seg_conv_igemm_plan_b1", M, self.cout, self.cin_pad, self.ks, ctypes.addressof(plan))
            splits, tile, ntl = plan
            if not PLAN_B1:  # the cost model's tile and split count
                splits, tile = query("seg_conv_igemm_splits", M, self.cout, self.cin_pad, self.ks), -1
                ntl = query("seg_conv_igemm_tiles", M, self.cout)
            bufs = rt._mb[("ic", id(self))] = (
                torch.empty(splits * M * self.cout if splits > 1 else 1, device=rt.device, dtype=torch.float32),
                torch.zeros(4 * ntl, device=rt.device, dtype=torch.int32), splits, tile)
        work, cnt, splits, tile = bufs
        rt.call(_FOLDED_CONV[rt.prog.math] + "_ic", rt.ptr(i), i.ld, i.N, i.H, i.W, self.cin_pad, wk, ldk, bias,
                rt.ptr(o), o.ld, o.H, o.W, self.cout, self.ks, self.stride, self.pad,
                rt.ptr(r) if r is not None else None, r.ld if r is not None else 0, act, work.data_ptr(), splits, tile,
                cnt.data_ptr(), s)

    def _in_xform(self, rt):
        """(scale, shift, act) of the producer's lazy BN for this op's input loads, or (None, None, 0)."""
        xf = self.xform
        if xf is None:
            return None, None, 0
        st, C = rt.saved[id(xf)], xf.cout
        return st[2 * C:3 * C].data_ptr(), st[3 * C:4 * C].data_ptr(), xf.act

    # -- backward
    def _bnout(self, rt, i):
        """BN-backward partials from this data gradient's epilogue (seg_conv_igemm_bnout*), when its output
        region is exactly the output of a train-mode BatchNorm layer P: the extra arguments, or None.  P's
        backward uses them if no other write reached the buffer afterwards (Run.wgen)."""
        if not BNOUT or not rt.training:
            return None
        p = rt.prog.bn_owner().get(i.key())
        if p is None or id(p) not in rt.saved:
            return None
        v = 16 // rt.es
        py = p.y
        if py.ld % v or py.off % v or rt.ptr(py) % 16:
            return None
        if not query("seg_conv_igemm_bnout_ok", i.M, self.cin, int(rt.io)):
            return None
        tiles, _ = rt.row_tiles(i.M, self.cin)
        if tiles > BNOUT_MAX_TILES:
            return None
        C = p.cout
        mean, invstd, scale, shift = _stat_ptrs(rt.saved[id(p)], C)
        part = rt.tmp(tiles * 2 * C)
        rt.bn_parts[id(p)] = [part, tiles, None]
        return (rt.ptr(py), py.ld, scale, shift, mean, p.act, part.data_ptr()), p

    def backward(self, rt):
        s, y = rt.stream, self.y
        dA = rt.grad_of(self.out)
        if self.bn is not None:
            if not rt.training:
                raise NotImplementedError("backward through eval-mode BatchNorm is not supported")
            C, M = self.cout, y.M
            st = rt.saved[id(self)]
            mean, invstd, scale, shift = _stat_ptrs(st, C)
            g_w, g_b = rt.grad_param(self.bn.weight), rt.grad_param(self.bn.bias)
            # bench.py's "bn_bwd" family: algorithmic bytes of a BatchNorm backward = dA and y read once, dY written
            # once (3 |Y|), credited to the launch that writes dY
            abytes = 3 * M * C * rt.es
            bp = rt.bn_parts.pop(id(self), None)
            dY = Act(rt.tmp_buf(M * r4(C)), 0, r4(C), C, y.N, y.H, y.W)
            if bp is not None and bp[2] == rt.wgen.get(self.out.buf):
                # the reduction's partials came out of the epilogue of the data gradient that completed dA (nothing
                # wrote the buffer since): finalize them, then the apply
                coef = rt.tmp(3 * C)
                rt.tcall("bn_bwd", 0, "seg_bn_bwd_finalize_tiles", bp[0].data_ptr(), bp[1], M, C,
                         self.bn.weight.data_ptr(), invstd, g_w, g_b, coef.data_ptr(), s)
                rt.tcall("bn_bwd", abytes, rt.k("seg_bn_bwd_apply"), rt.gptr(dA), dA.ld, rt.ptr(y), y.ld, M, C, mean,
                         scale, shift, self.act, coef.data_ptr(), rt.ptr(dY), dY.ld, s)
            else:
                work = rt.tmp(query("seg_chan_workspace_floats", M, C) + 3 * C)
                rt.tcall("bn_bwd", abytes, rt.k("seg_bn_backward"), rt.gptr(dA), dA.ld, rt.ptr(y), y.ld, M, C,
                         self.bn.weight.data_ptr(), mean, invstd, scale, shift, self.act,
                         g_w, g_b, work.data_ptr(), rt.ptr(dY), dY.ld, s)
            if self.res is not None:
                rt.add_pending(self.res, dA)
        else:
            dY = dA
        dYp = rt.ptr(dY) if dY.buf.startswith("#") else rt.gptr(dY)
        M = y.M
        # parameter gradients: on the side stream when overlapping (they only read dY and x,
        # and nothing on the main stream's data-gradient chain waits for them)
        # gradient tensors handed back to autograd are allocated on the main stream
        # (they outlive the backward; the side stream only writes into them)
        for p in (self.conv.weight, self.conv.bias):
            if p is not None and p.requires_grad:
                rt.grad_param(p)
        late = FORK_LATE and not self.first
        if late:  # the data gradient first: the side stream's weight gradient then runs beside
            self._dgrad(rt, dY, dYp, s)  # the next layer's memory-bound BN backward, not this dgrad
        k = getattr(rt, "cur_op", -1)
        if WGRAD_TAIL and rt.side is not None and rt.sync is None and 0 <= k < WGRAD_TAIL:
            # the backward's last layers: their parameter gradients go on the MAIN stream after its last data
            # gradient (Run.flush_tail), sharing the end-of-step backlog with the side stream
            for p in (self.conv.weight, self.conv.bias):
                if p is not None and p.requires_grad:
                    rt.grad_param(p)
            rt.tail.append((self, dY, dYp))
        elif rt.defer is not None and rt.side is not None and k >= rt.defer[0]:
            # issued later, beside the memory-bound part of the backward (Run.flush_deferred); dY stays valid
            # (persistent within the run)
            for p in (self.conv.weight, self.conv.bias):
                if p is not None and p.requires_grad:
                    rt.grad_param(p)
            rt.deferred.append((self, dY, dYp))
        else:
            ctx, sw = rt.fork()
            with ctx:
                self._param_grads(rt, dY, dYp, sw)
        if not self.first and not late:
            self._dgrad(rt, dY, dYp, s)

    def _param_grads(self, rt, dY, dYp, s):
        """Bias gradient (column sum of dY), weight gradient (split-K slabs + fixed-order
        reduce) and the DDP readiness hook, all on stream `s`."""
        y, M = self.y, self.y.M
        if DIAG_SKIP_WGRAD is not None and DIAG_SKIP_WGRAD[0] <= getattr(rt, "cur_op", -1) < DIAG_SKIP_WGRAD[1]:
            rt.params_done(self.params(), s)  # diagnostics only: no conv weight / bias gradients (wrong training)
            return
        if self.conv.bias is not None and self.conv.bias.requires_grad:
            if self.bn is not None and ZERO_BN_BIAS:
                # conv -> train-mode BatchNorm (src/unet.py:58-59,61-62): the bias shifts its whole channel by
                # a constant that the batch mean removes again, so d loss / d bias = sum_p dY[p][c] = 0
                # exactly (the reference computes that sum and gets fp32 rounding noise, ~1e-9 relative)
                rt.zero_param_grad(self.conv.bias, s)
            else:
                work = rt.tmp(query("seg_chan_workspace_floats", M, r4(self.cout)))
                rt.call(rt.k("seg_colsum"), dYp, dY.ld, M, self.cout, work.data_ptr(), rt.grad_param(self.conv.bias),
                        0, s)
        if self.conv.weight.requires_grad:
            gw = rt.grad_param(self.conv.weight)
            i = self.inp
            if self.kind == "dw":
                nblk = query("seg_dw_wgrad_blocks", y.N, y.H, y.W, self.cout)
                part = rt.tmp(nblk * 9 * self.cout)
                rt.call(rt.k("seg_dw_wgrad"), dYp, dY.ld, rt.ptr(i), i.ld, i.N, i.H, i.W, i.C, *self._in_xform(rt), y.H, y.W,
                     self.stride, part.data_ptr(), s)
                rt.call("seg_conv_wgrad_reduce", part.data_ptr(), nblk, gw, self.cout, 1, 3, 1, 0, s)
            elif self.wino_w:
                form = "seg_conv_wino_wgrad16" if self.wino_w == 2 else "seg_conv_wino_wgrad"
                splits = query(form + "_splits", y.N, y.H, y.W, self.cin_pad, self.cout)
                part = rt.tmp(splits * 16 * self.cout * self.cin_pad)
                rt.tcall("wino3_wgrad", self.flops(), form, dYp, dY.ld, rt.ptr(i), i.ld, y.N, y.H,
                         y.W, self.cin_pad, self.cout, part.data_ptr(), splits, s)
                rt.call("seg_conv_wino_wgrad_reduce", part.data_ptr(), splits, gw, self.cout, self.cin, self.cin_pad, 0, s)
            elif self.w2:  # narrow bf16io 3x3: persistent LDS-halo weight gradient, one slab per block
                blocks = query("seg_conv_wgrad2_blocks", y.N, y.H, y.W)
                part = rt.tmp(blocks * self.cout * 9 * self.cin_pad)
                rt.tcall("igemm3_wgrad", self.flops(), "seg_conv_wgrad2_bf16io", dYp, dY.ld, rt.ptr(i), i.ld, y.N, y.H,
                         y.W, self.cin_pad, self.cout, part.data_ptr(), s)
                rt.call("seg_conv_wgrad_reduce", part.data_ptr(), blocks, gw, self.cout, self.cin, 3, 0, 0, s)
            else:
                splits = query("seg_conv_wgrad_splits_bf16" if self.bf else "seg_conv_wgrad_splits", M, self.cout,
                               self.cin_pad, self.ks)
                part = rt.tmp(splits * self.cout * self.ks * self.ks * self.cin_pad)
                name = ("seg_conv_wgrad_bf16io" if rt.io else "seg_conv_wgrad_bf16") if self.bf else "seg_conv_wgrad"
                xf = ()
                if self.xform is not None:  # X = the producer's lazy BN + act, formed on load
                    name, xf = name + "_xf", self._in_xform(rt)
                rt.tcall(f"igemm{self.ks}_wgrad", self.flops(), name, dYp, dY.ld, rt.ptr(i), i.ld,
                            i.N, i.H, i.W, self.cin_pad, y.H, y.W, self.cout, self.ks, self.stride, self.pad,
                            part.data_ptr(), splits, *xf, s)
                rt.call("seg_conv_wgrad_reduce", part.data_ptr(), splits, gw, self.cout, self.cin, self.ks, 0, 0, s)
        rt.params_done(self.params(), s)

    def _dgrad(self, rt, dY, dYp, s):
        """Data gradient into the input's gradient region (first writer / fused addend)."""
        y, i = self.y, self.inp
        if self.kind == "dw":
            acc = rt.begin_write_accumulate(i)
            rt.call(rt.k("seg_dw_dgrad"), dYp, dY.ld, y.N, y.H, y.W, self.cout, self.wk_f.data_ptr(), rt.gptr(i),
                    i.ld, i.H, i.W, self.stride, acc, s)
        else:
            if self.stride != 1:
                raise NotImplementedError("data gradient of a strided dense conv")
            kin = r4(self.cout)  # dY channels padded to 4 (the C=10 head)
            bo = None
            add_ptr, add_ld = rt.begin_write_add(i)
            # seg_conv_pw / seg_conv_igemm2 read the addend as 16-byte row vectors
            add16 = add_ptr is None or (add_ld % (16 // rt.es) == 0 and add_ptr % 16 == 0)
            if self.pw_d and add16:  # thin-K 1x1 data gradient
                rt.tcall("igemm1_dgrad", self.flops(), rt.k("seg_conv_pw"), dYp, dY.ld, y.M, kin, self.wk_d.data_ptr(),
                         self.ldk_d, None, rt.gptr(i), i.ld, self.cin, add_ptr, add_ld, None, None, None, 0, s)
            elif self.halo_d:
                rt.tcall("igemm3_dgrad", self.flops(), rt.k("seg_conv_halo") + ("_w16" if self.w16_d else ""), dYp,
                         dY.ld, y.N, y.H, y.W, kin,
                            self.wk_d.data_ptr(), self.ldk_d, None, rt.gptr(i), i.ld, self.cin, add_ptr, add_ld, None, s)
            elif self.wino_fd and query("seg_conv_wino_fused_ok", y.N, y.H, y.W, dY.ld):
                rt.tcall("wino3_dgrad", self.flops(), "seg_conv_wino_fused", dYp, dY.ld, y.N, y.H, y.W, kin,
                         self.wk_wd.data_ptr(), kin, None, rt.gptr(i), i.ld, self.cin, add_ptr, add_ld, None, s)
            elif self.wino_d:
                work = rt.tmp(16 * (y.M // 4) * self.cin)
                rt.tcall("wino3_dgrad", self.flops(), "seg_conv_wino", dYp, dY.ld, y.N, y.H, y.W, kin,
                            self.wk_wd.data_ptr(), kin, None, rt.gptr(i), i.ld, self.cin, add_ptr, add_ld, None,
                            work.data_ptr(), s)
            elif self.ig2_d is not None and add16:
                work = rt.tmp(self.ig2_d[3], zero=True)
                rt.tcall(f"igemm{self.ks}_dgrad", self.flops(), "seg_conv_igemm2_bf16io", dYp, dY.ld, y.N, y.H, y.W, kin,
                         self.wk_d.data_ptr(), self.ldk_d, None, rt.gptr(i), i.ld, self.cin, self.ks, add_ptr, add_ld,
                         None, work.data_ptr(), s)
            elif rt.io:
                bo = self._bnout(rt, i)
                if bo is not None:  # + the BN-backward partials of the layer whose dA this completes
                    rt.tcall(f"igemm{self.ks}_dgrad", self.flops(),
                             "seg_conv_igemm_bnout_bf16io_w16" if self.w16_d else "seg_conv_igemm_bnout_bf16io", dYp,
                             dY.ld, y.N, y.H, y.W, kin, self.wk_d.data_ptr(), self.ldk_d, rt.gptr(i), i.ld, self.cin,
                             self.ks, add_ptr, add_ld, *bo[0], s)
                else:
                    rt.tcall(f"igemm{self.ks}_dgrad", self.flops(),
                             "seg_conv_igemm_bf16io_w16" if self.w16_d else "seg_conv_igemm_bf16io", dYp, dY.ld, y.N, y.H,
                             y.W, kin, self.wk_d.data_ptr(), self.ldk_d, None, rt.gptr(i), i.ld, i.H, i.W, self.cin,
                             self.ks, 1, self.pad, add_ptr, add_ld, None, s)
            elif self.bf:
                rt.tcall(f"igemm{self.ks}_dgrad", self.flops(), "seg_conv_igemm_bf16", dYp, dY.ld, y.N, y.H, y.W,
                            kin, self.wk_d.data_ptr(), self.ldk_d, None, rt.gptr(i), i.ld, i.H, i.W, self.cin,
                            self.ks, 1, self.pad, add_ptr, add_ld, None, ACT_NONE, None, 1, s)
            else:
                bo = self._bnout(rt, i)
                if bo is not None:
                    rt.tcall(f"igemm{self.ks}_dgrad", self.flops(), "seg_conv_igemm_bnout", dYp, dY.ld, y.N, y.H, y.W,
                             kin, self.wk_d.data_ptr(), self.ldk_d, rt.gptr(i), i.ld, self.cin, self.ks, add_ptr, add_ld,
                             *bo[0], s)
                else:
                    rt.tcall(f"igemm{self.ks}_dgrad", self.flops(), "seg_conv_igemm", dYp, dY.ld, y.N, y.H, y.W, kin,
                             self.wk_d.data_ptr(), self.ldk_d, None, rt.gptr(i), i.ld, i.H, i.W, self.cin, self.ks, 1,
                             self.pad, add_ptr, add_ld, None, s)
            if bo is not None:  # the partials are valid while this write is the buffer's last
                rt.mark_written(i)
                rt.bn_parts[id(bo[1])][2] = rt.wgen[i.buf]
                return
        rt.mark_written(i)


class UpsampleOp:
    """nn.Upsample(x2, bilinear, align_corners=False) into a concat slice (src/unet.py:97-103)."""

    def __init__(self, low, out):
        self.low, self.out = low, out

    def params(self):
        return []

    def forward(self, rt):
        l, o = self.low, self.out
        rt.call(rt.k("seg_upsample_fwd"), rt.ptr(l), l.ld, l.N, l.H, l.W, l.C, rt.ptr(o), o.ld, o.H, o.W, 0, rt.stream)

    def backward(self, rt):
        l, o = self.low, self.out
        d = rt.grad_of(o)
        acc = rt.begin_write_accumulate(l)
        rt.call(rt.k("seg_upsample_bwd"), rt.gptr(d), d.ld, 0, o.N, o.H, o.W, o.C, rt.gptr(l), l.ld, l.H, l.W, 0, acc,
             rt.stream)
        rt.mark_written(l)


class PoolOp:
    """nn.MaxPool2d(2) (src/unet.py:85)."""

    def __init__(self, inp, out):
        self.inp, self.out = inp, out

    def params(self):
        return []

    def forward(self, rt):
        i, o = self.inp, self.out
        rt.call(rt.k("seg_maxpool2_fwd"), rt.ptr(i), i.ld, i.N, i.H, i.W, i.C, rt.ptr(o), o.ld, rt.stream)

    def backward(self, rt):
        i, o = self.inp, self.out
        d = rt.grad_of(o)
        acc = rt.begin_write_accumulate(i)
        rt.call(rt.k("seg_maxpool2_bwd"), rt.ptr(i), i.ld, rt.gptr(d), d.ld, i.N, i.H, i.W, i.C, rt.gptr(i), i.ld, acc,
             rt.stream)
        rt.mark_written(i)


# ------------------------------------------------------------------------ program

class Program:
    def __init__(self, N, H, W, math="f32"):
        if math not in MATHS:
            raise ValueError(f"conv math must be one of {MATHS}, got {math!r}")
        self.N, self.H, self.W = N, H, W
        self.math = math     # "f32" | "bf16" (set_conv_math)
        self.bufs = {}       # name -> (rows, ld)
        self.ops = []
        self.logits = None   # Act of the (low-res for MobileNetV2UNet) logits
        self.out_hw = (H, W)
        self._n = 0
        self.image = self.new(3, H, W, name=IMAGE)  # NHWC4 copy of the input batch

    def wgrad_defer(self):
        """(from, at): the parameter gradients of ops >= from wait until the backward reaches op `at`, or None.
        bf16io default (DEFER_DECODER): the decoder's (from its first upsample on) until the encoder's last op --
        issued beside the encoder's memory-bound backward instead of the decoder's data-gradient convs
        (interleaved A/B, profiles/r06/ab_wgrad_defer.txt: bf16io +1.3 %, f32 -0.8 %)."""
        if WGRAD_DEFER is not None:
            return WGRAD_DEFER
        if not DEFER_DECODER or self.math != "bf16io":
            return None
        first_up = next((k for k, op in enumerate(self.ops) if isinstance(op, UpsampleOp)), None)
        return (first_up, first_up - 1) if first_up else None

    def mbconv_groups(self):
        """Folded forward: op index -> the (expand, depthwise, project) or (depthwise, project) ConvOps of a
        torchvision InvertedResidual that seg_mbconv_f16 runs as one launch (each intermediate activation
        consumed only inside the block: the lazy BN chain Program.make_lazy built)."""
        m = getattr(self, "_mb_groups", None)
        if m is not None:
            return m
        m, ops = {}, self.ops
        ok1 = (lambda op: isinstance(op, ConvOp) and op.kind == "igemm" and op.ks == 1 and op.stride == 1
               and op.bn is not None and op.conv.bias is None and op.cin_pad == op.cin)
        for k in range(len(ops) - 1):
            d, p = ops[k], ops[k + 1]
            if not (isinstance(d, ConvOp) and d.kind == "dw" and d.bn is not None and d.act == ACT_RELU6 and d.lazy
                    and ok1(p) and p.xform is d and p.act == ACT_NONE and p.inp is d.out):
                continue
            e = ops[k - 1] if k > 0 else None
            exp = (ok1(e) and e.act == ACT_RELU6 and e.lazy and e.res is None and d.xform is e and d.inp is e.out)
            cin = e.cin if exp else d.cout
            if p.res is not None and d.stride != 1:
                continue
            if not query("seg_mbconv_ok", cin, d.cout, p.cout, d.stride, int(exp)):
                continue
            if exp:
                m[k - 1] = (e, d, p)
            elif d.xform is None or d.xform.kind != "dw":
                m[k] = (d, p)
        self._mb_groups = m
        return m

    def stem_pre(self):
        """Folded fp16 forward: the stem ConvOp (features[0]: 3x3 stride-2 conv 3 -> 32, BN folded, ReLU6, the
        image its only input) when seg_stem_pre_f16 can run it on the frame directly, else None."""
        ops = self.ops
        if not ops:
            return None
        op = ops[0]
        if not (isinstance(op, ConvOp) and op.kind == "igemm" and op.ks == 3 and op.stride == 2 and op.pad == 1
                and op.cin == 3 and op.cin_pad == 4 and op.cout == 32 and op.bn is not None and op.res is None
                and op.inp is self.image and op.fk_pack is not None and op.ldk_f == 36 and op.out.ld % 4 == 0
                and 0 not in self.mbconv_groups()):
            return None
        if any(getattr(o, "inp", None) is self.image or getattr(o, "res", None) is self.image for o in ops[1:]):
            return None
        return op

    def pw2_head(self):
        """Folded forward: index of outconv's first 1x1 conv when seg_pw2_f16 runs the head (1x1 -> folded BN ->
        ReLU -> 1x1, the program's last two ops, the hidden activation consumed only by the last conv), else
        None."""
        ops = self.ops
        if len(ops) < 2:
            return None
        c1, c2 = ops[-2], ops[-1]
        pw = (lambda op: isinstance(op, ConvOp) and op.kind == "igemm" and op.ks == 1 and op.stride == 1
              and op.fk_pack is None and op.res is None and op.cin_pad == op.cin)
        if not (pw(c1) and pw(c2) and c2.inp is c1.out and c1.bn is not None and c2.bn is None
                and c1.act in (ACT_RELU, ACT_RELU6) and c1.inp.ld % 4 == 0
                and query("seg_pw2_ok", c1.cin, c1.cout, c2.cout)):
            return None
        return len(ops) - 2

    def bn_owner(self):
        """Activation key -> the ConvOp with a BatchNorm whose output it is (the BN-backward reduction target of a
        data gradient writing exactly that region; ConvOp._bnout)."""
        m = getattr(self, "_bn_owner", None)
        if m is None:
            m = self._bn_owner = {op.out.key(): op for op in self.ops if isinstance(op, ConvOp) and op.bn is not None}
        return m
    def new(self, C, H, W, name=None):
        name = name or f"t{self._n}"
        self._n += 1
        ld = r4(C)
        self.bufs[name] = (self.N * H * W, ld)
        return Act(name, 0, ld, C, self.N, H, W)

    def conv(self, kind, conv, bn, act, inp, out=None, res=None, xform=None):
        ks, st, pd = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        Hi, Wi = inp.H, inp.W
        Ho, Wo = (Hi + 2 * pd - ks) // st + 1, (Wi + 2 * pd - ks) // st + 1
        if out is None:
            out = self.new(conv.out_channels, Ho, Wo)
        y = self.new(conv.out_channels, Ho, Wo) if bn is not None else out
        self.ops.append(ConvOp(kind, conv, bn, act, inp, out, y, res, xform))
        return out

    def make_lazy(self, a: Act, pointwise=False):
        """If `a` is the private BN+act output of the last op, drop its buffer and let
        the consumer apply the BN on load; returns the producer op (or None).
        pointwise: the consumer is a 1x1 conv (seg_conv_igemm_xf / seg_conv_wgrad_xf:
        the uniform-tap loader, 8-channel groups) -- any conv producer; otherwise a
        depthwise consumer (seg_dw_fwd / seg_dw_wgrad) of a dense producer.  (3x3
        consumers re-read every input element once per tap: measured slower, round 3.)"""
        op = self.ops[-1] if self.ops else None
        kinds = ("igemm", "dw") if pointwise else ("igemm",)
        if pointwise and not (LAZY_PW and a.C % 8 == 0 and a.C >= 16):
            return None
        if not (isinstance(op, ConvOp) and op.kind in kinds and op.bn is not None and op.res is None
                and op.out is a and op.y is not a and a.off == 0 and a.ld == r4(a.C)
                and self.bufs.get(a.buf) == (a.M, a.ld) and not a.buf.startswith("cat")):
            return None
        del self.bufs[a.buf]
        op.out, op.lazy = op.y, True
        return op

    def pack(self, rt):
        """Repack every conv weight for this step (one seg_pack_batch launch on the run's
        stream).  The packed buffers and the device job table are built once and rebuilt
        only when a weight's storage moves (e.g. model.to())."""
        convs = [op for op in self.ops if isinstance(op, ConvOp)]
        key = tuple(op.conv.weight.data_ptr() for op in convs)
        if getattr(self, "_pack_key", None) != key:
            self._build_pack(convs, key)
        if self._njobs:
            rt.call("seg_pack_batch", self._jobs.data_ptr(), self._njobs, self._pack_blocks, rt.stream)

    def _build_pack(self, convs, key):
        import numpy as np
        if self.math == "f16":
            raise NotImplementedError("f16 conv math is the inference configuration (Predictor(model, math='f16')); "
                                      "train with 'f32' or 'bf16'")
        jobs, max_elems = [], 0
        for op in convs:
            w = op.conv.weight
            dev = w.device
            if op.kind == "dw":
                op.wk_f = torch.empty(9 * op.cout, device=dev, dtype=torch.float32)
                jobs.append((w.data_ptr(), op.wk_f.data_ptr(), op.cout, 1, 3, 9, 2, 1))
                max_elems = max(max_elems, 9 * op.cout)
                continue
            y = op.y
            op.bf = self.math in ("bf16", "bf16io")
            if op.bf:
                # bf16 math: every dense / pointwise conv (fwd, dgrad, wgrad) on the bf16 implicit GEMM
                op.wino_f = op.wino_d = op.wino_w = op.halo_f = op.halo_d = False
                op.wino_ff = op.wino_fd = False
                # narrow bf16io 3x3 weight gradients on seg_conv_wgrad2_bf16io (SEG_WGRAD2=0: the implicit GEMM)
                op.w2 = (self.math == "bf16io" and WGRAD2 and op.ks == 3 and op.stride == 1 and op.pad == 1
                         and op.xform is None and op.cin_pad == op.cin and y.ld % 8 == 0 and op.inp.ld % 8 == 0
                         and op.inp.off % 8 == 0
                         and bool(query("seg_conv_wgrad2_ok", y.N, y.H, y.W, op.cin_pad, op.cout)))
                if self.math == "bf16io" and op.ks == 3 and op.stride == 1 and op.pad == 1:
                    # narrow convs: the LDS-halo direct conv (seg_conv_halo_bf16io): 8-channel slots
                    op.halo_f = (op.cin_pad % 8 == 0 and HALO_BF16
                                 and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, op.cin_pad, op.cout)))
                    op.halo_d = (not op.first and r4(op.cout) % 8 == 0 and HALO_BF16
                                 and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, r4(op.cout), op.cin)))
                # bf16io implicit-GEMM and LDS-halo launches take bf16 packed weights (seg_conv_*_bf16io_w16:
                # half the weight bytes every M tile / pixel tile re-reads)
                w16f = w16d = self.math == "bf16io" and W16
                op.w16_f, op.w16_d = w16f, w16d
                # the deep 3x3 convs on seg_conv_igemm2_bf16io
                op.ig2_f = op.ig2_d = None
                # beyond IGEMM2_MAX_ROWS only GEMMs whose N fills the 8-wave tiles (N % 128 == 0: UNet's deep levels)
                wide = y.M > IGEMM2_MAX_ROWS and IGEMM2_WIDE
                if (w16f and IGEMM2 and op.ks == 3 and op.stride == 1 and op.pad == 1
                        and (y.M <= IGEMM2_MAX_ROWS or wide)):
                    i = op.inp  # 16-byte rows: ld and channel offset multiples of 8 elements
                    rows16 = i.ld % 8 == 0 and i.off % 8 == 0 and y.ld % 8 == 0 and y.off % 8 == 0
                    if (rows16 and not op.halo_f and op.xform is None and op.cin_pad == op.cin
                            and (not wide or op.cout % 128 == 0)):
                        op.ig2_f = igemm2_plan(y.M, op.cout, op.cin_pad, op.ks)
                    if (rows16 and not op.first and not op.halo_d and op.cout % 8 == 0
                            and (not wide or op.cin % 128 == 0)):
                        op.ig2_d = igemm2_plan(y.M, op.cin, op.cout, op.ks)
                if w16f:
                    op.pw_f, op.pw_d = _pw_pick(op, 8)
                if w16f or not (op.ks == 1 and op.cin_pad == op.cin):
                    op.ldk_f = r8(op.ks * op.ks * op.cin_pad) if w16f else r4(op.ks * op.ks * op.cin_pad)
                    op.wk_f = torch.empty(op.cout * op.ldk_f, device=dev,
                                          dtype=torch.bfloat16 if w16f else torch.float32)
                    jobs.append((w.data_ptr(), op.wk_f.data_ptr(), op.cout, op.cin, op.ks, op.ldk_f, 16 if w16f else 0,
                                 op.cin_pad))
                    max_elems = max(max_elems, op.cout * op.ldk_f)
                if not op.first:
                    kin = r4(op.cout)
                    op.ldk_d = r8(op.ks * op.ks * kin) if w16d else r4(op.ks * op.ks * kin)
                    op.wk_d = torch.empty(op.cin * op.ldk_d, device=dev, dtype=torch.bfloat16 if w16d else torch.float32)
                    jobs.append((w.data_ptr(), op.wk_d.data_ptr(), op.cout, op.cin, op.ks, op.ldk_d, 17 if w16d else 1,
                                 kin))
                    max_elems = max(max_elems, op.cin * op.ldk_d)
                continue
            op.pw_f, op.pw_d = _pw_pick(op, 4)
            dense3 = op.ks == 3 and op.stride == 1 and op.pad == 1
            wino_ok = dense3 and WINOGRAD
            # seg_conv_wino_pick: 1 = the two-launch form, 2 = the fused kernel
            pf = query("seg_conv_wino_pick", y.N, y.H, y.W, op.cin_pad, op.cout) if wino_ok and WINOGRAD_FWD else 0
            pd = (query("seg_conv_wino_pick", y.N, y.H, y.W, r4(op.cout), op.cin)
                  if wino_ok and WINOGRAD_DGRAD and not op.first else 0)
            op.wino_f, op.wino_ff = pf != 0, pf == 2
            op.wino_d, op.wino_fd = pd != 0, pd == 2
            # seg_conv_wino_wgrad_pick: 2 = the all-points kernel (seg_conv_wino_wgrad16), 1 = the per-point one
            op.wino_w = (query("seg_conv_wino_wgrad_pick", y.N, y.H, y.W, op.cin_pad, op.cout)
                         if wino_ok and WINOGRAD_WGRAD and op.xform is None else 0)
            if op.wino_w == 2 and not WINO_WGRAD16:  # A/B switch: the round-5 rule (per-point kernel, deep convs)
                T = y.N * (y.H // 2) * (y.W // 2)
                deep = op.cin_pad >= 128 and op.cout >= 128 and (T >= 65536 or min(op.cin_pad, op.cout) >= 256)
                op.wino_w = 1 if deep else 0
            op.halo_f = (dense3 and not op.wino_f
                         and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, op.cin_pad, op.cout)))
            op.halo_d = (dense3 and not op.first and not op.wino_d
                         and bool(query("seg_conv_halo_pick", y.N, y.H, y.W, r4(op.cout), op.cin)))
            if op.wino_f:
                op.wk_wf = torch.empty(16 * op.cout * op.cin_pad, device=dev, dtype=torch.float32)
                jobs.append((w.data_ptr(), op.wk_wf.data_ptr(), op.cout, op.cin, 3, op.cin_pad, 3, op.cin_pad))
                max_elems = max(max_elems, op.cout * op.cin_pad)
            elif not (op.ks == 1 and op.cin_pad == op.cin):
                op.ldk_f = r4(op.ks * op.ks * op.cin_pad)
                op.wk_f = torch.empty(op.cout * op.ldk_f, device=dev, dtype=torch.float32)
                jobs.append((w.data_ptr(), op.wk_f.data_ptr(), op.cout, op.cin, op.ks, op.ldk_f, 0, op.cin_pad))
                max_elems = max(max_elems, op.cout * op.ldk_f)
            if op.wino_d:
                kin = r4(op.cout)
                op.wk_wd = torch.empty(16 * op.cin * kin, device=dev, dtype=torch.float32)
                jobs.append((w.data_ptr(), op.wk_wd.data_ptr(), op.cout, op.cin, 3, kin, 4, kin))
                max_elems = max(max_elems, op.cin * kin)
            elif not op.first:
                kin = r4(op.cout)
                op.ldk_d = r4(op.ks * op.ks * kin)
                op.wk_d = torch.empty(op.cin * op.ldk_d, device=dev, dtype=torch.float32)
                jobs.append((w.data_ptr(), op.wk_d.data_ptr(), op.cout, op.cin, op.ks, op.ldk_d, 1, kin))
                max_elems = max(max_elems, op.cin * op.ldk_d)
        self._jobs, self._njobs, self._pack_blocks = pack_table(jobs, convs[0].conv.weight.device)
        self._pack_key = key

    def fold(self, stream):
        """Eval: fold every BatchNorm into its conv (one seg_bn_fold_batch launch) and
        pack the folded weights (one seg_pack_batch launch).  Buffers and job tables
        are built once per weight storage; re-run after the weights or running
        statistics change (Predictor.refresh)."""
        convs = [op for op in self.ops if isinstance(op, ConvOp)]
        key = tuple(op.conv.weight.data_ptr() for op in convs)
        if getattr(self, "_fold_key", None) != key:
            self._build_fold(convs, key)
        call("seg_bn_fold_batch", self._fjobs.data_ptr(), len(convs), self._fmax, stream)
        if self._fpjobs is not None:
            call("seg_pack_batch", self._fpjobs.data_ptr(), self._fpn, self._fpmax, stream)

    def _build_fold(self, convs, key):
        import numpy as np
        ft = np.dtype([("w", "<u8"), ("bias", "<u8"), ("gamma", "<u8"), ("beta", "<u8"), ("rm", "<u8"),
                       ("rv", "<u8"), ("w_out", "<u8"), ("b_out", "<u8"), ("cout", "<i4"), ("kper", "<i4"),
                       ("eps", "<f4"), ("pad", "<i4")])
        assert ft.itemsize == 80
        fjobs, pjobs, fmax, pmax = [], [], 0, 0
        for op in convs:
            w, b, bn = op.conv.weight, op.conv.bias, op.bn
            dev = w.device
            kper = w[0].numel()
            op.fk = torch.empty_like(w, memory_format=torch.contiguous_format)
            op.fb = torch.zeros(r4(op.cout), device=dev, dtype=torch.float32)
            if bn is not None and not (bn.track_running_stats and bn.running_mean is not None):
                raise NotImplementedError("eval BatchNorm2d without running statistics")
            ptr = (lambda t: t.data_ptr() if t is not None else 0)
            fjobs.append((w.data_ptr(), ptr(b), ptr(bn.weight) if bn is not None else 0,
                          ptr(bn.bias) if bn is not None else 0, ptr(bn.running_mean) if bn is not None else 0,
                          ptr(bn.running_var) if bn is not None else 0, op.fk.data_ptr(), op.fb.data_ptr(),
                          op.cout, kper, bn.eps if bn is not None else 0.0, 0))
            if bn is not None and (bn.weight is None or bn.bias is None):
                raise NotImplementedError("BatchNorm2d(affine=False) folding")
            fmax = max(fmax, op.cout * kper + op.cout)
            if op.kind == "dw":
                op.fk_pack = torch.empty(9 * op.cout, device=dev, dtype=torch.float32)
                pjobs.append((op.fk.data_ptr(), op.fk_pack.data_ptr(), op.cout, 1, 3, 9, 2, 1))
                pmax = max(pmax, 9 * op.cout)
            elif op.ks == 1 and op.cin_pad == op.cin:
                op.fk_pack = None
            else:
                op.ldk_f = r4(op.ks * op.ks * op.cin_pad)
                op.fk_pack = torch.empty(op.cout * op.ldk_f, device=dev, dtype=torch.float32)
                pjobs.append((op.fk.data_ptr(), op.fk_pack.data_ptr(), op.cout, op.cin, op.ks, op.ldk_f, 0,
                              op.cin_pad))
                pmax = max(pmax, op.cout * op.ldk_f)
        dev = convs[0].conv.weight.device
        self._fjobs = torch.from_numpy(np.array(fjobs, dtype=ft).view(np.uint8).copy()).to(dev)
        self._fmax = fmax
        if pjobs:
            self._fpjobs, self._fpn, self._fpmax = pack_table(pjobs, dev)
        else:
            self._fpjobs, self._fpn, self._fpmax = None, 0, 0
        self._fold_key = key

    def params(self):
        seen, ps = set(), []
        for op in self.ops:
            for p in op.params():
                if id(p) not in seen:
                    seen.add(id(p))
                    ps.append(p)
        return ps


_PACK_JOB = [("w", "<u8"), ("wk", "<u8"), ("cout", "<i4"), ("cin", "<i4"), ("ks", "<i4"), ("ldk", "<i4"),
             ("mode", "<i4"), ("kin", "<i4"), ("blk0", "<i4"), ("nblk", "<i4")]


def pack_table(jobs, device):
    """Device table of seg_pack_job for seg_pack_batch from (w, wk, cout, cin, ks, ldk, mode,
    kin_pad) tuples: each job gets ceil(elements / 256) blocks of the launch.
    Returns (table, njobs, total blocks)."""
    import numpy as np
    rows, blk = [], 0
    for (w, wk, cout, cin, ks, ldk, mode, kin) in jobs:
        elems = 9 * cout if mode == 2 else (cout if (mode & 15) in (0, 3) else cin) * ldk
        nblk = max(1, (elems + 255) // 256)
        rows.append((w, wk, cout, cin, ks, ldk, mode, kin, blk, nblk))
        blk += nblk
    t = np.array(rows, dtype=np.dtype(_PACK_JOB))
    assert t.dtype.itemsize == 48
    return torch.from_numpy(t.view(np.uint8).copy()).to(device), len(rows), blk


def _cna(prog, m: ConvBNReLU6, inp, out=None, kind=None, xform=None):
    conv, bn = m[0], m[1]
    if kind is None:
        kind = "dw" if conv.groups > 1 else "igemm"
    return prog.conv(kind, conv, bn, ACT_RELU6, inp, out=out, xform=xform)


def _inverted_residual(prog, blk: InvertedResidual, inp, out=None):
    layers = list(blk.conv)
    x = inp
    if len(layers) == 4:  # expand ratio != 1
        x = _cna(prog, layers[0], x)
        layers = layers[1:]
    # the depthwise conv applies its producer's BN + ReLU6 on load (the expand conv,
    # or the stem for features[1]) unless that activation is also the residual
    xf = None if (blk.use_res_connect and x is inp) else prog.make_lazy(x)
    if xf is not None:
        x = xf.out
    x = _cna(prog, layers[0], x, kind="dw", xform=xf)
    # ... and the 1x1 project conv applies the depthwise conv's BN + ReLU6 the same way
    xf = prog.make_lazy(x, pointwise=True)
    if xf is not None:
        x = xf.out
    return prog.conv("igemm", layers[1], layers[2], ACT_NONE, x, out=out,
                     res=inp if blk.use_res_connect else None, xform=xf)


def _double_conv(prog, dc, inp, out=None):
    c = dc.conv
    x = prog.conv("igemm", c[0], c[1], ACT_RELU, inp)
    return prog.conv("igemm", c[3], c[4], ACT_RELU, x, out=out)


def _up(prog, u, low, cat):
    """cat = [skip (already written) | upsample(low)]; returns double_conv output."""
    cs = cat.C - low.C
    if u.conv.conv[0].in_channels != cat.C:
        raise ValueError("up block channel mismatch")
    prog.ops.append(UpsampleOp(low, cat.slice(cs, low.C)))
    return _double_conv(prog, u.conv, cat)


def _outconv(prog, oc, inp):
    c = oc.conv
    x = prog.conv("igemm", c[0], c[1], ACT_RELU, inp)
    xf = prog.make_lazy(x, pointwise=True) if c[3].kernel_size[0] == 1 else None
    if xf is not None:
        x = xf.out
    return prog.conv("igemm", c[3], None, ACT_NONE, x, xform=xf)


def build_mobilenet_unet(model, N, H, W, math="f32") -> Program:
    """Program for MobileNetV2UNet.forward (src/unet.py:32-51)."""
    if H % 32 or W % 32:
        raise ValueError(f"MobileNetV2UNet needs H, W divisible by 32 (got {H}x{W}); the reference fails "
                         "with a torch.cat size mismatch on such inputs")
    p = Program(N, H, W, math)
    ups = [model.up1, model.up2, model.up3, model.up4]
    skip_c = [u.conv.conv[0].in_channels for u in ups]  # concat widths
    # concat buffers, finest first: cat4 @ H/2 (up4), cat3 @ H/4, cat2 @ H/8, cat1 @ H/16
    cats = {}
    for k, (u, div) in enumerate(zip(ups, (16, 8, 4, 2))):
        cats[k] = p.new(skip_c[k], H // div, W // div, name=f"cat{4 - k}")
    stages = [model.down1, model.down2, model.down3, model.down4, model.down5]
    skip_target = {0: cats[3], 1: cats[2], 2: cats[1], 3: cats[0]}
    x = p.image
    for si, stage in enumerate(stages):
        blocks = list(stage)
        for bi, blk in enumerate(blocks):
            last = bi == len(blocks) - 1
            out = None
            if last and si in skip_target:
                oc = blk.out_channels
                out = skip_target[si].slice(0, oc)
            if isinstance(blk, InvertedResidual):
                x = _inverted_residual(p, blk, x, out=out)
            elif isinstance(blk, ConvBNReLU6):
                x = _cna(p, blk, x, out=out)
            else:
                raise TypeError(f"unexpected encoder block {type(blk).__name__}")
    for k, u in enumerate(ups):
        x = _up(p, u, x, cats[k])
    p.logits = _outconv(p, model.outc, x)
    fu = model.final_upsample
    if fu.scale_factor not in (2, 2.0) or not fu.align_corners:
        raise ValueError("final_upsample must be x2 bilinear align_corners=True")
    p.out_hw = (H, W)
    return p


def build_unet(model, N, H, W, math="f32") -> Program:
    """Program for UNet / LightUNet.forward (src/unet.py:137-147, :160-171)."""
    if H % 8 or W % 8:
        raise ValueError(f"UNet needs H, W divisible by 8 (got {H}x{W})")
    p = Program(N, H, W, math)
    b = model.inc.conv.conv[0].out_channels
    cat3 = p.new(model.up3.conv.conv[0].in_channels, H, W, name="cat3")          # [x1 | up(u2)]
    cat2 = p.new(model.up2.conv.conv[0].in_channels, H // 2, W // 2, name="cat2")  # [x2 | up(u1)]
    cat1 = p.new(model.up1.conv.conv[0].in_channels, H // 4, W // 4, name="cat1")  # [x3 | up(x4)]
    x1 = _double_conv(p, model.inc.conv, p.image, out=cat3.slice(0, b))
    d1 = model.down1.mpconv[1]
    pooled = p.new(x1.C, H // 2, W // 2)
    p.ops.append(PoolOp(x1, pooled))
    x2 = _double_conv(p, d1, pooled, out=cat2.slice(0, d1.conv[3].out_channels))
    d2 = model.down2.mpconv[1]
    pooled = p.new(x2.C, H // 4, W // 4)
    p.ops.append(PoolOp(x2, pooled))
    x3 = _double_conv(p, d2, pooled, out=cat1.slice(0, d2.conv[3].out_channels))
    d3 = model.down3.mpconv[1]
    pooled = p.new(x3.C, H // 8, W // 8)
    p.ops.append(PoolOp(x3, pooled))
    x4 = _double_conv(p, d3, pooled)
    x = _up(p, model.up1, x4, cat1)
    x = _up(p, model.up2, x, cat2)
    x = _up(p, model.up3, x, cat3)
    p.logits = _outconv(p, model.sem_out, x)
    p.out_hw = (H, W)
    return p


def build_program(model, N, H, W, math="f32") -> Program:
    from .unet import MobileNetV2UNet, UNet, LightUNet
    if isinstance(model, MobileNetV2UNet):
        prog = build_mobilenet_unet(model, N, H, W, math)
    elif isinstance(model, (UNet, LightUNet)):
        prog = build_unet(model, N, H, W, math)
    else:
        raise TypeError(f"no HIP program for {type(model).__name__}")
    return prog


# Conv arithmetic of a model's programs.  "f32" (default): exact fp32 products on the
# f32 MFMA (plus Winograd / LDS-halo kernels where they measured faster), the
# reference's own arithmetic.  "bf16": the bf16 configurations (BASELINE configs[2],
# [4]; the reference's equivalent is torch.autocast(dtype=torch.bfloat16) around the
# forward) -- every dense / pointwise conv, forward and both gradients, multiplies
# bf16-rounded operands on the bf16 MFMA with fp32 accumulation; activations, BN,
# depthwise convs, the loss and the optimizer stay fp32.
MATHS = ("f32", "bf16", "bf16io", "f16")
# "bf16io": bf16 conv math AND bf16 activation / gradient storage (every tensor between
# kernels is bf16 in HBM, halving the memory-bound passes; BN statistics, partial sums,
# parameter gradients, the loss and Adam stay fp32) -- the _bf16io entry points.
# "f16" is the fp16 inference configuration (BASELINE configs[3]): the BN-folded eval
# forward (Predictor) with fp16 conv operands; training programs refuse it.
_FOLDED_CONV = {"f32": "seg_conv_igemm_act", "bf16": "seg_conv_igemm_bf16", "f16": "seg_conv_igemm_f16"}


def set_conv_math(model, math: str):
    """Select the conv arithmetic ("f32" | "bf16") of `model` (or a DataParallel wrapper's module)."""
    if math not in MATHS:
        raise ValueError(f"conv math must be one of {MATHS}, got {math!r}")
    model = getattr(model, "module", model)
    model.__dict__["_segamd_math"] = math
    return model


# ------------------------------------------------------------------------ runtime

class Run:
    """State of one forward (and its backward): buffers, saved BN statistics,
    gradient buffers and which gradient regions have been written.

    Two ways to execute the walk: immediately (every launch is a ctypes call on the
    current stream -- the Predictor's folded eval forward, captured in a hipGraph), or
    recorded (`rec` set: every launch, event pair and memset becomes an entry of a
    launch tape, seg_amd/tape.py; all buffers are then persistent so the tape can be
    replayed step after step)."""

    def __init__(self, prog: Program, image: torch.Tensor, training: bool, rec=None, side=None):
        self.prog, self.image, self.training = prog, image, training
        self.device = image.device
        self.stream = torch.cuda.current_stream(self.device).cuda_stream
        self.rec = rec
        # activation / gradient storage: fp32, or bf16 for math "bf16io" (the _bf16io kernels)
        self.io = prog.math == "bf16io"
        self.store = torch.bfloat16 if self.io else torch.float32
        self.es = 2 if self.io else 4
        self.bufs = {n: torch.empty(rows * ld, device=self.device, dtype=self.store)
                     for n, (rows, ld) in prog.bufs.items()}
        self.saved = {}
        self.bn_parts = {}    # id(op) -> [tile partials, tiles, write generation]: its BN-backward reduction from
                              # the epilogue of the data gradient that completed its dA (seg_conv_igemm_bnout*)
        self.wgen = {}        # gradient buffer name -> write generation (every write to the buffer bumps it)
        self._mb = {}         # folded forward: op index -> (partials, tile counters) of a fused inverted residual
        self.gbufs = {}
        self.keep = []        # workspaces of a recorded run (persistent: the tape points at them)
        self.written = {}     # grad buffer name -> list of (lo, hi) channel ranges
        self.pending = {}     # Act.key() -> addend Act (residual upstream gradient)
        self.grads = {}       # id(param) -> grad tensor
        self.flat = None      # recorded run: one flat fp32 buffer holding every parameter gradient
        self.sync = None
        self._tmp_n = 0
        self.side = side      # side stream of the parameter gradients (recorded backward)
        self._n_fork = 0      # side-stream forks so far (index into the program's event pool)
        self.deferred = []    # (op, dY, dY ptr) whose parameter gradients wait for flush_deferred (WGRAD_DEFER)
        self.tail = []        # ... for flush_tail (WGRAD_TAIL)
        self.defer = prog.wgrad_defer()  # (from, at) of the deferred parameter gradients, or None

    def k(self, name: str) -> str:
        """C-ABI entry point of an activation kernel for this run's storage type."""
        return name + "_bf16io" if self.io else name

    # launches
    def call(self, name, *args):
        if self.rec is not None:
            self.rec.call(name, args)
        else:
            call(name, *args)

    def tcall(self, kind, flops, name, *args):
        """A launch of the roofline kernel families (bench.py times them)."""
        if self.rec is not None:
            self.rec.call(name, args, timer=(kind, flops))
        else:
            _timed_call(kind, flops, name, *args)

    def zero_param_grad(self, p: torch.Tensor, stream) -> None:
        """An all-zero gradient for parameter `p`.  A recorded run's gradient slot is persistent and
        nothing else writes it, so it is zeroed once, now (on the current stream, ahead of every
        replay), and the tape gets no entry; an immediate run zeroes its fresh tensor on the current stream
        (`stream`: inside the fork context).  Under DataParallel the slot is a view into an
        all-reduced gradient bucket into which a synchronised backward folds any `.grad` a rank
        still holds, so a recorded run re-zeroes it every step (a tape memset on `stream`) -- a
        once-only zero would keep that fold and double it on every later step."""
        self.grad_param(p)
        g = self.grads[id(p)]
        g.zero_()
        if self.rec is not None and self.sync is not None:
            self.rec.memset2d(g.data_ptr(), g.numel() * 4, 0, g.numel() * 4, 1, stream)

    def zero(self, a: Act):
        """Zero-fill the gradient region of `a` (a channel slice of a row buffer)."""
        self.wgen[a.buf] = self.wgen.get(a.buf, 0) + 1
        if self.rec is not None:
            self.rec.memset2d(self.gptr(a), a.ld * self.es, 0, a.C * self.es, a.M, self.stream)
        else:
            self.gbuf(a.buf).view(-1, a.ld)[:, a.off:a.off + a.C].zero_()

    # pointers
    def ptr(self, a: Act) -> int:
        if a.buf.startswith("#"):
            return self.gbufs[a.buf].data_ptr() + self.es * a.off
        return self.bufs[a.buf].data_ptr() + self.es * a.off

    def gptr(self, a: Act) -> int:
        if a.buf.startswith("#"):
            return self.gbufs[a.buf].data_ptr() + self.es * a.off
        return self.gbuf(a.buf).data_ptr() + self.es * a.off

    def gbuf(self, name):
        g = self.gbufs.get(name)
        if g is None:
            g = self.gbufs[name] = torch.empty_like(self.bufs[name])
        return g

    def tmp(self, n: int, zero: bool = False) -> torch.Tensor:
        """A float32 workspace; zero=True for the channel reductions' workspaces, whose ticket
        words (the in-launch finalize, csrc/bn.hip) must be zero before their first use."""
        t = (torch.zeros if zero else torch.empty)(max(int(n), 1), device=self.device, dtype=torch.float32)
        if self.rec is not None:
            self.keep.append(t)
        return t

    @staticmethod
    def row_tiles(M: int, C: int):
        key = (M, C)
        r = _ROW_TILES.get(key)
        if r is None:
            rows = ctypes.c_int(0)
            n = query("seg_conv_igemm_row_tiles", M, C, ctypes.addressof(rows))
            r = _ROW_TILES[key] = (n, rows.value)
        return r

    def tmp_buf(self, n: int) -> str:
        name = f"#tmp{self._tmp_n}"
        self._tmp_n += 1
        self.gbufs[name] = torch.empty(max(int(n), 1), device=self.device, dtype=self.store)
        return name

    # streams
    def fork(self):
        """(context, stream handle) for work that may run beside the main stream: with
        overlap on, the side stream first waits for everything issued so far on the main
        stream; temporaries allocated inside the context belong to the side stream."""
        if self.side is None:
            return contextlib.nullcontext(), self.stream
        if self.rec is not None:
            ev = self.rec.event()
            self.rec.record(ev, self.stream)
            self.rec.wait(self.side.cuda_stream, ev)
            return contextlib.nullcontext(), self.side.cuda_stream
        # events are reused step after step (a wait binds to the record before it)
        pool = self.prog.__dict__.setdefault("_fork_events", [])
        if self._n_fork == len(pool):
            pool.append(torch.cuda.Event())
        ev = pool[self._n_fork]
        self._n_fork += 1
        ev.record(self.main)
        self.side.wait_event(ev)
        return self._side_ctx, self.side.cuda_stream

    def flush_deferred(self):
        """Issue the deferred parameter gradients on the side stream, in backward order, behind one fork."""
        if not self.deferred:
            return
        ctx, sw = self.fork()
        with ctx:
            for op, dY, dYp in self.deferred:
                op._param_grads(self, dY, dYp, sw)
        self.deferred = []

    def flush_tail(self):
        """The WGRAD_TAIL parameter gradients on the main stream, after every data gradient of the backward."""
        for op, dY, dYp in self.tail:
            op._param_grads(self, dY, dYp, self.stream)
        self.tail = []

    def join(self):
        if self.side is None:
            return
        if self.rec is not None:
            ev = self.rec.event()
            self.rec.record(ev, self.side.cuda_stream)
            self.rec.wait(self.stream, ev)
        else:
            self.main.wait_stream(self.side)

    # gradient-region bookkeeping
    def _covered(self, a: Act) -> bool:
        lo, hi = a.off, a.off + a.C
        for (l, h) in self.written.get(a.buf, ()):
            if l <= lo and hi <= h:
                return True
        return False

    def mark_written(self, a: Act):
        self.written.setdefault(a.buf, []).append((a.off, a.off + a.C))
        self.wgen[a.buf] = self.wgen.get(a.buf, 0) + 1

    def grad_of(self, a: Act) -> Act:
        """Gradient region of activation `a` (zero-filled if nobody wrote it)."""
        if not self._covered(a):
            add = self.pending.pop(a.key(), None)
            if add is not None:
                self.call(self.k("seg_add"), self.gptr(add), add.ld, None, 0, a.M, a.C, self.gptr(a), a.ld, self.stream)
            else:
                self.zero(a)
            self.mark_written(a)
        return a

    def add_pending(self, target: Act, addend: Act):
        if self._covered(target):
            self.call(self.k("seg_add"), self.gptr(target), target.ld, self.gptr(addend), addend.ld, target.M, target.C,
                      self.gptr(target), target.ld, self.stream)
            self.wgen[target.buf] = self.wgen.get(target.buf, 0) + 1
        else:
            self.pending[target.key()] = addend

    def begin_write_add(self, a: Act):
        """For writers with a fused addend: returns (add_ptr, add_ld)."""
        if self._covered(a):
            return self.gptr(a), a.ld
        add = self.pending.pop(a.key(), None)
        if add is not None:
            return self.gptr(add), add.ld
        return None, 0

    def begin_write_accumulate(self, a: Act) -> int:
        """For writers with only an accumulate flag: materialise a pending addend first."""
        if self._covered(a):
            return 1
        add = self.pending.pop(a.key(), None)
        if add is not None:
            self.call(self.k("seg_add"), self.gptr(add), add.ld, None, 0, a.M, a.C, self.gptr(a), a.ld, self.stream)
            self.mark_written(a)
            return 1
        return 0

    def grad_param(self, p: torch.Tensor) -> int:
        g = self.grads.get(id(p))
        if g is None:
            g = self.sync.grad_storage(p) if self.sync is not None else None
            if g is None and self.flat is not None:
                o, n = self.flat_slots[id(p)]
                g = self.flat[o:o + n].view_as(p)
            if g is None:
                g = torch.empty_like(p)
            self.grads[id(p)] = g
        return g.data_ptr()

    def params_done(self, ps, stream=None):
        """The gradients of `ps` are complete on `stream` (DataParallel bucket readiness)."""
        if self.sync is None:
            return
        ready = [p for p in ps if id(p) in self.grads]
        if self.rec is None:
            self.sync.on_ready(ready)
            return
        sync = self.sync
        st = self.side if (self.side is not None and stream == self.side.cuda_stream) else None
        done = sync.plan_ready(ready)  # the buckets this point completes; a host stop only then
        if not done:
            return

        def on_ready():  # host callback between tape segments
            if st is None:
                sync.launch_ready(done)
            else:
                with torch.cuda.stream(st):
                    sync.launch_ready(done)
        self.rec.stop(on_ready)

    # drivers
    def forward(self):
        global LAST_RUN
        x, img = self.image, self.prog.image
        self.prog.pack(self)
        self.call(self.k("seg_nchw_to_nhwc"), x.data_ptr(), img.N, 3, img.H, img.W, self.ptr(img), img.ld, self.stream)
        for k, op in enumerate(self.prog.ops):
            if self.rec is not None:
                self.rec.label = f"{k}:fwd"
            op.forward(self)
        if DEBUG_KEEP_RUN:
            LAST_RUN = self

    def forward_folded(self, start=0):
        """Eval forward with every BatchNorm folded (Program.fold must have run): one
        launch per conv, or per inverted residual with fp16 conv math (seg_mbconv_f16).  The
        NHWC4 input rows must already be in the image buffer (start = 0), or ops[:start] have
        run (the stem fused with the preprocess, Program.stem_pre)."""
        ops = self.prog.ops
        f16 = self.prog.math == "f16"
        groups = self.prog.mbconv_groups() if MBCONV and f16 else {}
        head = self.prog.pw2_head() if PW2 and f16 else None
        k = start
        while k < len(ops):
            g = groups.get(k)
            if g is not None:
                self._mbconv(k, g)
                k += len(g)
                continue
            if k == head:
                c1, c2 = ops[k], ops[k + 1]
                x, o = c1.inp, c2.out
                call("seg_pw2_f16", self.ptr(x), x.ld, x.N * x.H * x.W, c1.cin, c1.fk.data_ptr(),
                     c1.fb.data_ptr() if c1.fb is not None else None, c1.cout, c1.act, c2.fk.data_ptr(),
                     c2.fb.data_ptr() if c2.fb is not None else None, c2.cout, self.ptr(o), o.ld, self.stream)
                k += 2
                continue
            op = ops[k]
            if isinstance(op, ConvOp):
                op.forward_folded(self)
            else:
                op.forward(self)
            k += 1

    def _mbconv(self, k, g):
        """One fused inverted residual (expand?, depthwise, project) of the folded forward."""
        e, d, p = (g[0], g[1], g[2]) if len(g) == 3 else (None, g[0], g[1])
        x = e.inp if e is not None else d.inp
        o, r = p.out, p.res
        bufs = self._mb.get(k)
        if bufs is None:  # persistent across graph replays: allocated by the warm-up launch, before any capture
            ncnt = ctypes.c_int(0)
            nw = query("seg_mbconv_work_floats", x.N, x.H, x.W, d.cout, p.cout, d.stride, ctypes.addressof(ncnt))
            bufs = self._mb[k] = (torch.empty(max(nw, 1), device=self.device, dtype=torch.float32),
                                  torch.zeros(max(ncnt.value, 1), device=self.device, dtype=torch.int32))
        call("seg_mbconv_f16", self.ptr(x), x.ld, x.N, x.H, x.W, x.C, e.fk.data_ptr() if e is not None else None,
             e.fb.data_ptr() if e is not None else None, d.cout, d.fk_pack.data_ptr(), d.fb.data_ptr(), d.stride,
             p.fk.data_ptr(), p.fb.data_ptr(), p.cout, self.ptr(r) if r is not None else None,
             r.ld if r is not None else 0, self.ptr(o), o.ld, bufs[0].data_ptr(), bufs[1].data_ptr(), self.stream)

    def backward_from_logits(self):
        global LAST_RUN
        if self.rec is None and OVERLAP:
            self.main = torch.cuda.current_stream(self.device)
            self.side = _side_stream(self.device)
            self._side_ctx = torch.cuda.StreamContext(self.side)  # re-entered by every fork
        try:
            for k in range(len(self.prog.ops) - 1, -1, -1):
                self.cur_op = k
                if self.defer is not None and k == self.defer[1]:
                    self.flush_deferred()
                if self.rec is not None:
                    self.rec.label = f"{k}:bwd"
                self.prog.ops[k].backward(self)
            self.flush_deferred()
            self.flush_tail()
        finally:
            self.join()
        if DEBUG_KEEP_RUN:
            LAST_RUN = self


# Engine switches.  Environment switches (SEG_*) are the A/B knobs of measured design choices, read at import;
# the module constants below them are diagnostics the tests flip directly (monkeypatch), not user settings.
#
# Parameter gradients (weight / bias / BN-affine readiness) run on a second HIP stream
# beside the data-gradient chain: the compute-bound 3x3 weight gradients overlap the
# memory-bound BatchNorm / depthwise / 1x1 kernels of the main stream.  Results are the
# same either way (the kernels and their reduction orders do not change).
OVERLAP = os.environ.get("SEG_OVERLAP", "1") == "1"
# fork the weight-gradient side stream after the layer's data gradient (measured: f32 +1.5 %, bf16io +-0)
FORK_LATE = os.environ.get("SEG_FORK_LATE", "1") == "1"
# Winograd F(2x2,3x3) for the deep f32 3x3 convs (read when a program's weights are first
# packed); SEG_WINO=0 routes them to the LDS-halo / implicit-GEMM kernels instead.
WINOGRAD = os.environ.get("SEG_WINO", "1") == "1"
# LDS-halo direct 3x3 conv for the narrow convs in the bf16io configuration; SEG_HALO_BF16=0 turns it off.
HALO_BF16 = os.environ.get("SEG_HALO_BF16", "1") == "1"
# ... and their weight gradients on the persistent LDS-halo kernel (seg_conv_wgrad2_bf16io); SEG_WGRAD2=0 = off
WGRAD2 = os.environ.get("SEG_WGRAD2", "1") == "1"
# BatchNorm-backward reduction from the epilogue of the implicit-GEMM data gradient that completes a BN layer's dA
# (seg_conv_igemm_bnout*: no reduction pass over dA; the finalize reads the tile partials); SEG_BNOUT=0 = off.  Up to
# BNOUT_MAX_TILES row tiles (the finalize's serial tile loop), i.e. the small-image layers where the three-launch
# BN backward is latency-bound
BNOUT = os.environ.get("SEG_BNOUT", "1") == "1"
BNOUT_MAX_TILES = int(os.environ.get("SEG_BNOUT_MAX_TILES", "1024"))
# lazy BatchNorm for 1x1 consumers (the inverted residuals' project convs, OutConv's last
# conv): SEG_LAZY_PW=0 keeps the separate BN-apply pass (read at program build)
LAZY_PW = os.environ.get("SEG_LAZY_PW", "1") == "1"
# the bias gradient of a conv followed by train-mode BatchNorm is exactly zero: write zeros instead of
# reducing dY (SEG_ZERO_BN_BIAS=0 keeps the reduction, whose result is rounding noise)
ZERO_BN_BIAS = os.environ.get("SEG_ZERO_BN_BIAS", "1") == "1"
# thin-K 1x1 convs (K <= 32) on seg_conv_pw instead of the generic implicit GEMM; SEG_PW=0 = off
PW = os.environ.get("SEG_PW", "1") == "1"
PW_MIN_ROWS = int(os.environ.get("SEG_PW_MIN_ROWS", "262144"))
# bf16io deep 3x3 convs on the 8-wave LDS-DMA implicit GEMM (seg_conv_igemm2_bf16io, csrc/igemm2.hip); SEG_IGEMM2=0
# = off
IGEMM2 = os.environ.get("SEG_IGEMM2", "1") == "1"
# ... on images of at most this many output rows: measured per launch on UNet 512x1024 bf16io, igemm2 is 5-25 %
# slower than the 4-wave implicit GEMM at 262k-4M rows and 1-6 % faster at 65k (profiles/r03k)
IGEMM2_MAX_ROWS = int(os.environ.get("SEG_IGEMM2_MAX_ROWS", "65536"))
# ... and beyond that on the convs whose GEMM N is a multiple of 128 (the 8-wave tiles without padding): measured per
# launch at HEAD of round 4 on UNet 512x1024 bf16io, side stream off, 1-10 % faster than the 4-wave implicit GEMM on
# every such launch (profiles/r04ig/); SEG_IGEMM2_WIDE=0 = off
IGEMM2_WIDE = os.environ.get("SEG_IGEMM2_WIDE", "1") == "1"
# bf16io implicit GEMMs on bf16-packed weights (seg_conv_igemm_bf16io_w16); SEG_W16=0 keeps the fp32 packs
W16 = os.environ.get("SEG_W16", "1") == "1"
# SEG_WGRAD_DEFER=from:at (A/B): the parameter gradients of program ops >= `from` are issued on the side stream only
# when the backward reaches op `at` (all of them behind one fork), instead of right after each layer's data gradient
_wd = os.environ.get("SEG_WGRAD_DEFER", "")
WGRAD_DEFER = tuple(int(v) for v in _wd.split(":")) if _wd else None
# bf16io: the decoder's parameter gradients deferred until the backward reaches the encoder (Program.wgrad_defer);
# SEG_DEFER_DECODER=0 = off
DEFER_DECODER = os.environ.get("SEG_DEFER_DECODER", "1") == "1"
# SEG_WGRAD_TAIL=K (A/B): the parameter gradients of program ops < K go on the main stream after the backward's last
# data gradient instead of on the side stream
WGRAD_TAIL = int(os.environ.get("SEG_WGRAD_TAIL", "0"))
# many-tile BN statistics merged 16 tiles per row before the per-channel finalize; SEG_BN_MERGE=0 = direct
BN_MERGE = os.environ.get("SEG_BN_MERGE", "1") == "1"

# Diagnostics only (wrong training): SEG_DIAG_SKIP_WGRAD=1 issues no conv weight / bias gradient at all -- the step
# time of the main stream's work alone, with no side-stream contention (the weight gradients' share of the step,
# DESIGN round 6); SEG_DIAG_SKIP_WGRAD=lo:hi skips only those of the program ops lo <= k < hi
_dsw = os.environ.get("SEG_DIAG_SKIP_WGRAD", "0")
DIAG_SKIP_WGRAD = None if _dsw == "0" else (0, 1 << 30) if _dsw == "1" else tuple(int(v) for v in _dsw.split(":"))
# Diagnostics (tests flip these): the Winograd transforms one at a time (parity attribution,
# tests/test_gpu_unet_cfg5.py) ...
WINOGRAD_WGRAD = True  # the F(3x3,2x2) weight gradients
# ... on the all-points kernel (seg_conv_wino_wgrad16; SEG_WINO_WGRAD16=0: the round-5 choice, A/B only)
WINO_WGRAD16 = os.environ.get("SEG_WINO_WGRAD16", "1") != "0"
WINOGRAD_FWD = True    # the F(2x2,3x3) forward
WINOGRAD_DGRAD = True  # ... and data-gradient transforms
# ... and the fp16 inference (Predictor, BASELINE configs[3]) fusions against their unfused launches: each inverted
# residual of the folded forward as one launch (seg_mbconv_f16), the stem forming the preprocessed frame on load
# (seg_stem_pre_f16), outconv's 1x1 -> BN -> ReLU -> 1x1 head in one launch (seg_pw2_f16), and the folded convs on
# seg_conv_igemm_plan_b1's tile / split count (the batch-1 decoder convs) instead of the training cost model's
MBCONV = True
STEM_PRE = True
PW2 = True
PLAN_B1 = True
_SIDE = {}


def _side_stream(device):
    st = _SIDE.get(device)
    if st is None:
        st = _SIDE[device] = torch.cuda.Stream(device, priority=0)
    return st


DEBUG_KEEP_RUN = False  # diagnostics: keep the last Run (buffers + gradient buffers)
LAST_RUN = None


def debug_preactivations(model) -> dict:
    """Diagnostics (needs DEBUG_KEEP_RUN = True before the forward): every activation
    layer's post-BatchNorm pre-activation z = y * scale + shift of the last run, as fp64
    NCHW CPU tensors keyed by the conv's module path + "." (the parity tests compare them
    with the oracle and take the ReLU/ReLU6 masks from them)."""
    run = LAST_RUN
    if run is None:
        raise RuntimeError("set engine.DEBUG_KEEP_RUN = True before the forward")
    model = getattr(model, "module", model)
    names = {}
    for n, m in model.named_modules():
        names.setdefault(id(m), n)
    out = {}
    for op in run.prog.ops:
        if isinstance(op, ConvOp) and op.bn is not None and op.act != ACT_NONE:
            y, C = op.y, op.cout
            t = run.bufs[y.buf].view(-1, y.ld)[:, y.off:y.off + C].double()
            st = run.saved[id(op)].double()
            z = t * st[2 * C:3 * C] + st[3 * C:4 * C]
            out[names[id(op.conv)] + "."] = z.view(y.N, y.H, y.W, C).permute(0, 3, 1, 2).cpu()
    return out


_PROGRAM_CACHE_ATTR = "_segamd_programs"


def debug_pool_positions(model) -> dict:
    """Diagnostics (DEBUG_KEEP_RUN, like debug_preactivations): the 2x2-window position (0..3, row-major; first
    maximum, the kernel's and aten's tie rule) every max-pool of the last run chose, from the values the kernel read,
    keyed "down1.", "down2.", ... in forward order (UNet's `down` blocks, src/unet.py:85) -- the parity checker routes
    the fp64 oracle's max-pool gradients through them (oracle/budget.py)."""
    run = LAST_RUN
    if run is None:
        raise RuntimeError("set engine.DEBUG_KEEP_RUN = True before the forward")
    out, k = {}, 0
    for op in run.prog.ops:
        if isinstance(op, PoolOp):
            i = op.inp
            a = run.bufs[i.buf].view(-1, i.ld)[:, i.off:i.off + i.C].float().cpu()
            a = a.view(i.N, i.H // 2, 2, i.W // 2, 2, i.C).permute(0, 5, 1, 3, 2, 4).reshape(i.N, i.C, i.H // 2,
                                                                                           i.W // 2, 4)
            k += 1
            out[f"down{k}."] = a.argmax(-1)
    return out


def get_program(model, N, H, W, math=None) -> Program:
    cache = model.__dict__.setdefault(_PROGRAM_CACHE_ATTR, {})
    math = math or model.__dict__.get("_segamd_math", "f32")
    key = (N, H, W, math)
    prog = cache.get(key)
    if prog is None:
        prog = cache[key] = build_program(model, N, H, W, math)
    return prog


def _check_input(x: torch.Tensor):
    if not x.is_cuda:
        raise RuntimeError("segamd models run on the MI355X HIP path only; move the model and input to 'cuda' "
                           "(there is no CPU execution path)")
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"expected float32 input [N,3,H,W], got {tuple(x.shape)} {x.dtype}")
    if x.requires_grad:
        raise NotImplementedError("gradient w.r.t. the input image is not supported")


def _loss_forward(run, t, ignore_index):
    """Fused final upsample + CrossEntropy over the run's low-res logits: stats = [loss, count, #bad labels]."""
    prog, lo, s = run.prog, run.prog.logits, run.stream
    N = prog.N
    Ho, Wo = prog.out_hw
    stats = run.tmp(3)  # loss, #valid, #out-of-range labels
    work = run.tmp(query("seg_ce_workspace_floats", N * Ho * Wo))
    run.call(run.k("seg_ce_upsample_loss"), run.ptr(lo), lo.ld, N, lo.H, lo.W, lo.C, t.data_ptr(), Ho, Wo,
             ignore_index, work.data_ptr(), stats.data_ptr(), s)
    run.target, run.stats = t, stats
    return stats


def _loss_backward(run, g, ignore_index):
    """Gradient of the fused loss (g: [1] fp32 upstream gradient) through the whole program."""
    prog, lo, s = run.prog, run.prog.logits, run.stream
    N = prog.N
    Ho, Wo = prog.out_hw
    dhigh = torch.empty(max(N * Ho * Wo * lo.ld, 1), device=run.device, dtype=run.store)
    run.keep.append(dhigh)
    run.call(run.k("seg_ce_upsample_grad"), run.ptr(lo), lo.ld, N, lo.H, lo.W, lo.C, run.target.data_ptr(), Ho, Wo,
             ignore_index, g.data_ptr(), run.stats.data_ptr(), dhigh.data_ptr(), lo.ld, s)
    run.call(run.k("seg_upsample_bwd"), dhigh.data_ptr(), lo.ld, 0, N, Ho, Wo, lo.C, run.gptr(lo), lo.ld, lo.H, lo.W,
             1, 0, s)
    run.mark_written(lo)
    run.backward_from_logits()


class Plan:
    """One (input shape, mode) of a model compiled to two launch tapes (seg_amd/tape.py):
    the forward (weight repack, NCHW -> NHWC, every op, the fused loss or the NCHW logits)
    and the backward (loss / logits gradient, every op in reverse, parameter gradients on
    the side stream, DataParallel bucket all-reduces at host-callback stops).  Recorded
    by the first step -- a normal program walk with every launch captured instead of
    issued -- and replayed by the following ones with the caller's input / target /
    output / upstream-gradient pointers patched in.  Buffers, workspaces, saved BN
    statistics and the flat parameter-gradient buffer are persistent (allocated while
    recording, ~13 GB at bs=32 256x512 fp32 -- nothing is recomputed).

    The replay issues the same launches on the same two streams as an eager walk, so
    results are bitwise those of the eager engine (tests/test_gpu_tape.py)."""

    def __init__(self, prog, training, mode, ignore_index, sync, needs_grad, device):
        self.prog, self.training, self.mode, self.ignore_index = prog, training, mode, ignore_index
        self.sync, self.needs_grad, self.device = sync, needs_grad, device
        self.side = _side_stream(device) if (OVERLAP and needs_grad) else None
        self.run = self.fwd = self.bwd = None
        self.t = None            # the last forward's labels (loss mode)
        self.busy = False        # a forward whose backward has not run yet
        self.timer = None        # the KernelTimer the tapes' timing is armed for
        self.fp = None           # _fingerprint(prog) the tapes were recorded against

    def _streams(self):
        main = torch.cuda.current_stream(self.device).cuda_stream
        return main, (self.side.cuda_stream if self.side is not None else main)

    def _arm_timer(self, tape):
        if TIMER is not self.timer:
            for t in (self.fwd, self.bwd):
                if t is not None:
                    if self.timer is not None:
                        self.timer.collect(t)
                    t.time([], 0)
            self.timer = TIMER
        if TIMER is not None and tape not in TIMER.tapes:
            tape.time(TIMER.kinds, TIMER.max_replays)
            TIMER.tapes.append(tape)

    def forward(self, x, t):
        from .tape import Recorder
        main, side = self._streams()
        N, _, H, W = x.shape
        Ho, Wo = self.prog.out_hw
        out = None
        if self.mode == "logits":
            out = torch.empty((N, self.prog.logits.C, Ho, Wo), device=x.device, dtype=torch.float32)
        if self.fwd is None:
            rec = Recorder({side: 1, main: 0})
            rec.external("x", x.data_ptr())
            if t is not None:
                rec.external("t", t.data_ptr())
            if out is not None:
                rec.external("out", out.data_ptr())
            run = Run(self.prog, x, self.training, rec=rec, side=self.side)
            run.sync = self.sync
            if self.needs_grad:
                ps = [p for p in self.prog.params() if p.requires_grad]
                run.flat_slots, off = {}, 0
                for p in ps:
                    run.flat_slots[id(p)] = (off, p.numel())
                    off += p.numel()
                run.flat = torch.empty(max(off, 1), device=x.device, dtype=torch.float32)
            run.forward()
            lo = self.prog.logits
            if self.mode == "logits":
                run.call(run.k("seg_upsample_to_nchw"), run.ptr(lo), lo.ld, N, lo.H, lo.W, lo.C, out.data_ptr(), Ho,
                         Wo, 1, run.stream)
            else:
                _loss_forward(run, t, self.ignore_index)
            run.rec = None
            self.run, self.fwd = run, rec.build()
        self._arm_timer(self.fwd)
        self.t = t  # the backward tape reads the labels: keep them alive until then
        self.fwd.bind(x=x.data_ptr(), t=t.data_ptr() if t is not None else 0,
                      out=out.data_ptr() if out is not None else 0)
        self.fwd.run(main, side)
        if DEBUG_KEEP_RUN:
            global LAST_RUN
            LAST_RUN = self.run
        return out

    def backward(self, gout):
        from .tape import Recorder
        run = self.run
        main, side = self._streams()
        if self.mode == "logits":
            g = gout.contiguous()
        else:
            g = gout.reshape(1).to(torch.float32).contiguous()
        if self.bwd is None:
            rec = Recorder({side: 1, main: 0})
            if self.sync is not None:
                self.sync.begin_record()
            rec.external("gout", g.data_ptr())
            if self.t is not None:
                rec.external("t", self.t.data_ptr())
            run.rec = rec
            if self.mode == "logits":
                prog, lo = self.prog, self.prog.logits
                Ho, Wo = prog.out_hw
                run.call(run.k("seg_upsample_bwd"), g.data_ptr(), 0, 1, prog.N, Ho, Wo, lo.C, run.gptr(lo), lo.ld,
                         lo.H, lo.W, 1, 0, run.stream)
                run.mark_written(lo)
                run.backward_from_logits()
            else:
                _loss_backward(run, g, self.ignore_index)
            run.rec = None
            self.bwd = rec.build()
        self._arm_timer(self.bwd)
        self.bwd.bind(gout=g.data_ptr(), t=self.t.data_ptr() if self.t is not None else 0)
        self.bwd.run(main, side)
        if DEBUG_KEEP_RUN:
            global LAST_RUN
            LAST_RUN = run
        if self.sync is not None:
            self.sync.finish_gradient_sync()  # stream-ordered wait on the last all-reduces


def _fingerprint(prog):
    """Storage pointers of every tensor a plan's tapes point into: conv / BN parameters and
    BN running statistics.  A change (load_state_dict(assign=True), p.data = ..., .half(),
    DataParallel's flat BN buffers) invalidates the recorded tapes."""
    out = []  # read from the modules each time: a rebinding replaces the tensor object
    for op in prog.ops:
        if isinstance(op, ConvOp):
            c, b = op.conv, op.bn
            out += [c.weight.data_ptr(), c.bias.data_ptr() if c.bias is not None else 0]
            if b is not None:
                out += [t.data_ptr() if t is not None else 0
                        for t in (b.weight, b.bias, b.running_mean, b.running_var, b.num_batches_tracked)]
    return tuple(out)


# Launch plans kept per model (each holds its buffers: ~13 GB at bs=32 256x512 fp32, half in
# bf16io).  Least recently used plans beyond this are dropped; release_plans() drops all.
MAX_PLANS = int(os.environ.get("SEG_MAX_PLANS", "4"))


def release_plans(model):
    """Drop every recorded plan (tapes + persistent buffers) of `model`; the next step
    re-records.  Frees the plan memory, e.g. after evaluating at another resolution."""
    model = getattr(model, "module", model)
    model.__dict__.pop("_segamd_plans", None)


def _plan(model, prog, mode, ignore_index, sync, needs_grad, device):
    cache = model.__dict__.setdefault("_segamd_plans", {})
    key = (id(prog), mode, model.training, ignore_index, id(sync) if sync is not None else None, needs_grad, OVERLAP)
    fp = _fingerprint(prog)
    plan = cache.pop(key, None)  # re-inserted below: dict order = least recently used first
    if plan is None or plan.sync is not sync or plan.fp != fp:
        if plan is not None and plan.busy:
            raise RuntimeError("segamd: parameters or buffers were rebound between a forward and its backward")
        plan = Plan(prog, model.training, mode, ignore_index, sync, needs_grad, device)
        plan.fp = fp
    cache[key] = plan
    while len(cache) > max(MAX_PLANS, 1):
        old = next(k for k in cache)
        if cache[old].busy:  # its backward is still to come: keep it (and stop evicting)
            break
        del cache[old]
    if plan.busy:
        # a second forward before this plan's backward ran: a one-off plan keeps the first
        # forward's activations intact (recorded and run once, then dropped)
        plan = Plan(prog, model.training, mode, ignore_index, sync, needs_grad, device)
        plan.fp = fp
    return plan


class _SegFunction(torch.autograd.Function):
    """Whole-network forward/backward as one autograd node (replaying the plan's tapes)."""

    @staticmethod
    def forward(ctx, model, mode, x, target, ignore_index, sync, *params):
        x = x.contiguous()
        N, _, H, W = x.shape
        prog = get_program(model, N, H, W)
        Ho, Wo = prog.out_hw
        t = None
        if mode == "loss":
            t = target.contiguous()
            if t.dtype != torch.int64 or tuple(t.shape) != (N, Ho, Wo):
                raise ValueError(f"target must be int64 [{N},{Ho},{Wo}], got {tuple(t.shape)} {t.dtype}")
        needs_grad = any(ctx.needs_input_grad[6:])
        plan = _plan(model, prog, mode, ignore_index, sync, needs_grad, x.device)
        out = plan.forward(x, t)
        if mode == "loss":
            model.__dict__["_segamd_last_stats"] = plan.run.stats
            out = plan.run.stats[0].clone()  # the stats buffer is rewritten by the next step
            # the out-of-range label count, copied to the host as soon as the loss kernel has run:
            # train_one_epoch reads it before optimizer.step() without waiting for the backward
            # (on the stats tensor's device and stream: the model need not be on the current device)
            dev = plan.run.stats.device
            host = model.__dict__.get("_segamd_bad_host")
            if host is None or host[2] != dev:
                host = (torch.zeros(1, dtype=torch.float32).pin_memory(), torch.cuda.Event(), dev)
                model.__dict__["_segamd_bad_host"] = host
            with torch.cuda.device(dev):
                host[0].copy_(plan.run.stats[2:3], non_blocking=True)
                host[1].record(torch.cuda.current_stream(dev))
        else:  # an unfused criterion checks its own labels: no stale flag from an earlier fused loss
            model.__dict__.pop("_segamd_last_stats", None)
            model.__dict__.pop("_segamd_bad_host", None)
        if needs_grad:
            plan.busy = True
            ctx.plan, ctx.params = plan, params
        else:
            ctx.plan = None
        return out

    @staticmethod
    def backward(ctx, gout):
        plan = ctx.plan
        if plan is None:
            raise RuntimeError("segamd: backward called on a forward that saved nothing")
        try:
            plan.backward(gout)
        finally:
            plan.busy = False
        run = plan.run
        if run.sync is not None:  # DataParallel: copies of the averaged buckets, never the buckets
            grads = run.sync.autograd_grads(ctx.params)
        else:
            # one copy of the flat gradient buffer (the next backward rewrites it): a .grad
            # never aliases engine memory, and AccumulateGrad adopts the views as they are
            flat = run.flat.clone()
            grads = []
            for p in ctx.params:
                slot = run.flat_slots.get(id(p)) if id(p) in run.grads else None
                grads.append(flat[slot[0]:slot[0] + slot[1]].view_as(p) if slot else None)
        grads = [g if ctx.needs_input_grad[6 + k] else None for k, g in enumerate(grads)]
        ctx.plan = ctx.params = None
        return (None, None, None, None, None, None, *grads)


def bad_label_count(model):
    """Device tensor [1] (fp32): the number of labels outside [0, C) other than
    ignore_index seen by `model`'s last fused loss, or None (no fused loss yet).  Reading it
    is one host sync; train_one_epoch reads it (summed over ranks) before optimizer.step()."""
    model = getattr(model, "module", model)
    st = model.__dict__.get("_segamd_last_stats")
    return None if st is None else st[2:3].clone()


def label_flag(model):
    """Device tensor [1] (fp32) that is non-zero iff the last fused loss saw a label outside [0, C) other than
    ignore_index -- on ANY rank under seg_amd.ddp.DataParallel (the count rides in the last gradient bucket's
    all-reduce: valid in stream order after finish_gradient_sync, no extra collective); None when there is no fused
    loss to check (or, under DataParallel, when this step's buckets did not go out)."""
    sync = getattr(model, "label_flag", None)
    if sync is not None:  # DataParallel
        return sync()
    model = getattr(model, "module", model)
    st = model.__dict__.get("_segamd_last_stats")
    return None if st is None else st[2:3]


def bad_label_count_host(model):
    """The out-of-range label count of `model`'s last fused loss as a host int, or None: waits
    only for that forward's loss kernel (an event recorded behind its device-to-host copy), not
    for the backward queued after it, so the host keeps running ahead of the GPU."""
    model = getattr(model, "module", model)
    host = model.__dict__.get("_segamd_bad_host")
    if host is None or model.__dict__.get("_segamd_last_stats") is None:
        return None
    host[1].synchronize()
    return int(host[0].item())


def check_targets(model, bad=None):
    """Raise like nn.CrossEntropyLoss ("Target out of bounds") if the last fused loss of
    `model` saw a label outside [0, C) other than ignore_index.  The kernels flag it
    stream-ordered (the loss and every gradient become NaN); this reads the flag (one
    host sync).  bad: an already-gathered count (e.g. summed over ranks)."""
    if bad is None:
        bad = bad_label_count(model)
    n = 0 if bad is None else int(bad.item())
    if n:
        raise IndexError(f"Target out of bounds: {n} label(s) outside [0, num_classes) that are not "
                         "ignore_index (nn.CrossEntropyLoss raises on these)")


def _params_for(model, x):
    N, _, H, W = x.shape
    return get_program(model, N, H, W).params()


def run_logits(model, x: torch.Tensor) -> torch.Tensor:
    _check_input(x)
    sync = model.__dict__.get("_segamd_sync")
    return _SegFunction.apply(model, "logits", x, None, IGNORE_INDEX, sync, *_params_for(model, x))


def run_loss(model, x: torch.Tensor, target: torch.Tensor, ignore_index: int = IGNORE_INDEX) -> torch.Tensor:
    _check_input(x)
    sync = model.__dict__.get("_segamd_sync")
    return _SegFunction.apply(model, "loss", x, target, ignore_index, sync, *_params_for(model, x))
